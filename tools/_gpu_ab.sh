set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout=240 --timeout-method thread > gpurun_out/pytest_gpu_r01zg.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_r01zg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r01zg_diag.log 2>&1 || exit $?
CDX_LIB=$PWD/compliancedex_amd/lib/libcdx_nodiag.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r01zg_nodiag.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_r01zg_diag2.log 2>&1 || exit $?
CDX_VARIANTS=wn4,nodiag timeout -k 10 300 python tools/std_variants.py run > gpurun_out/stdvar_r01zg.log 2>&1 || exit $?
for f in gpurun_out/bench_r01zg_*.log; do echo $f; python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], d['stage_ms'])"; done
tail -5 gpurun_out/stdvar_r01zg.log
