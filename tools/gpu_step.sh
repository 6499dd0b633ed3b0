#!/bin/bash
# One GPU call of the session: full GPU tests, then an interleaved bench A/B and kernel-trace timelines.
#   bash tools/gpu_step.sh TAG "ab specs" "trace specs"      (specs space-separated; "" skips a part)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
TAG=$1; AB=${2:-}; TR=${3:-}
stop_if_fault() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "GPU step failed hard (rc=$1): stopping"; exit "$1"; fi; }
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -rf \
    > "gpurun_out/pytest_gpu_$TAG.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 "gpurun_out/pytest_gpu_$TAG.log"; stop_if_fault $rc
  [ $rc -ne 0 ] && exit 1
fi
if [ -n "$AB" ]; then bash tools/gpu_ab_bench.sh "$TAG" "${ROUNDS:-2}" $AB; rc=$?; stop_if_fault $rc; fi
if [ -n "$TR" ]; then bash tools/gpu_ab_trace.sh "$TAG" $TR; rc=$?; stop_if_fault $rc; fi
exit 0
