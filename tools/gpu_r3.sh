#!/bin/bash
# One GPU call (round 3): parity tests → smoke → bench [→ rocprofv3 kernel trace → PMC passes].
#   bash tools/gpu_r3.sh TAG [full]
# Each GPU step has its own time limit; a crash/timeout (rc not 0/1) ends the call.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
TAG=${1:-r03}
MODE=${2:-quick}
STEPS=${STEPS:-50}
stop_if_fault() { if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "GPU step failed hard (rc=$1): stopping"; exit "$1"; fi; }

echo "== pytest -m gpu"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread -rf \
  > "$OUT/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" "$OUT/pytest_gpu_$TAG.log" | tail -12; stop_if_fault $rc

echo "== smoke"; date
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke_$TAG.log"; stop_if_fault $rc

echo "== bench"; date
timeout -k 10 300 python bench.py --steps "$STEPS" --warmup 20 > "$OUT/bench_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 "$OUT/bench_$TAG.log"; stop_if_fault $rc
[ "$MODE" = "full" ] || exit 0

echo "== rocprofv3 kernel trace"; date
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run -- python3 "$ROOT/bench.py" --steps 30 --warmup 20 --no-cpu-baseline > "$OUT/rocprof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 "$OUT/rocprof_$TAG.log"; stop_if_fault $rc

echo "== rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs)"; date
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc_${C}_$TAG" -o run -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pmc_${C}_$TAG.log" 2>&1
  rc=$?; echo "pmc $C rc=$rc"; stop_if_fault $rc
done
date
