#!/bin/bash
# Round-3 var-late GPU check: GPU tests → interleaved bench A/B (CDX_VAR_LATE 1/0) → kernel-trace timeline.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
TAG=${1:-r03y}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf \
  > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 "$OUT/pytest_gpu_$TAG.log"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/gpu_ab_bench.sh "$TAG" 3 base+CDX_VAR_LATE=1 base+CDX_VAR_LATE=0 || exit $?
bash tools/gpu_ab_trace.sh "$TAG" base+CDX_VAR_LATE=1 || exit $?
