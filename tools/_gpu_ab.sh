# A/B helper: GPU parity tests, then bench of the default build against a variant library, twice.
#   bash tools/_gpu_ab.sh TAG VARIANT
set -o pipefail
TAG=${1:-ab}; VAR=${2:-vargen}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout=240 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_default.log 2>&1 || exit $?
CDX_LIB=$PWD/compliancedex_amd/lib/libcdx_$VAR.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_$VAR.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_default2.log 2>&1 || exit $?
CDX_VARIANTS=wn4,$VAR timeout -k 10 300 python tools/std_variants.py run > gpurun_out/stdvar_$TAG.log 2>&1 || exit $?
for f in gpurun_out/bench_${TAG}_*.log; do echo $f; python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], d['stage_ms'])"; done
grep '^{' gpurun_out/stdvar_$TAG.log
