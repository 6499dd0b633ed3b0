#!/bin/bash
# GPU tests → interleaved bench A/B of the given specs (3 rounds) → kernel-trace timeline of the default build.
#   bash tools/gpu_check.sh TAG [spec ...]     (specs as tools/gpu_ab_bench.sh; none: base only)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=$1; shift
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf \
  > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 "$OUT/pytest_gpu_$TAG.log"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
[ $# -gt 0 ] || set -- base
bash tools/gpu_ab_bench.sh "$TAG" 3 "$@" || exit $?
bash tools/gpu_ab_trace.sh "$TAG" base || exit $?
