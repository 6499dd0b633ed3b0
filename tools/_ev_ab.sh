# A/B of the profiling-event flags (CDX_PROF_EVENT_FLAGS, hex) on bench throughput, one box.
#   bash tools/_ev_ab.sh [FLAGS ...]   (default: 0 20000000 40000000)
set -o pipefail
for F in ${@:-0 20000000 40000000}; do
  CDX_PROF_EVENT_FLAGS=$F timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_evflags_$F.log 2>&1 || exit $?
  echo "$F $(tail -1 gpurun_out/bench_evflags_$F.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_ms"]["gpis_std_var"], d["stage_ms"]["gpis_std_grad"])')"
done
