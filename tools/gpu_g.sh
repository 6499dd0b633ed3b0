#!/bin/bash
# Session GPU call: pack parity tests, exchange timing, then kernel-trace A/B of the given libs.
#   bash tools/gpu_g.sh TAG lib...
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/exchange_bench.py > gpurun_out/${TAG}_exchange.json 2>&1 || exit 3
cat gpurun_out/${TAG}_exchange.json
bash tools/gpu_ab_trace.sh $TAG "$@"
