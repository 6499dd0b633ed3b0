#!/bin/bash
# GPU round helper: runs steps in order, stops at the first step that did not end with 0 or 1
# (a pytest failure is 1; a fault / abort / time limit ends the call).
mkdir -p gpurun_out
run() {
  local name=$1; shift
  echo "== $name: $*"
  "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -5 gpurun_out/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
for step in "$@"; do
  case $step in
    screen) run screen timeout -k 10 400 python -u -m pytest tests/test_screen.py -x -v --timeout 300 --timeout-method thread ;;
    gpu) run pytest_gpu timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    bench) run bench timeout -k 10 300 python -u bench.py --steps 50 --warmup 20 ;;
    benchq) run bench timeout -k 10 300 python -u bench.py --steps 50 --warmup 20 --no-cpu-baseline ;;
    smoke) run smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
  esac
done
