# A/B: screened closure with the mean on the side stream (default) vs on the caller's stream
# (CDX_NO_FORK), alternating, plus the screen tests first.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_screen.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout=240 --timeout-method thread > gpurun_out/pytest_fork.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_fork.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_fork_$i.log 2>&1 || exit $?
  CDX_NO_FORK=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_nofork_$i.log 2>&1 || exit $?
done
for f in gpurun_out/bench_fork_*.log gpurun_out/bench_nofork_*.log; do echo $f; python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(round(d['value']), round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['stage_ms'].items() if v})"; done
