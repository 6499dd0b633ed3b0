#!/bin/bash
# screen epilogue A/B: tests (product lib), standalone screen variants, closure bench A/B, screen tests on the variant
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
SKIP_TESTS= ROUNDS=3 bash tools/gpu_step.sh g4 "base epireg" "" || exit $?
CDX_VARIANTS=epilds,epireg,diag_noepi CDX_VARIANT_ROUNDS=2 timeout -k 10 400 python tools/screen_variants.py run 4096 > gpurun_out/g4_screen_variants.jsonl 2>gpurun_out/g4_sv.err
rc=$?; cat gpurun_out/g4_screen_variants.jsonl; [ $rc -ne 0 ] && exit $rc
CDX_LIB=$(pwd)/compliancedex_amd/lib/libcdx_epireg.so timeout -k 10 400 python -u -m pytest tests/test_screen.py tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/g4_pytest_epireg.log 2>&1
rc=$?; tail -3 gpurun_out/g4_pytest_epireg.log; exit $rc
