#!/bin/bash
# Survivor pack: GPU tests of the distributed path → exchange pieces at E = 4096 / 65 536 → a bench's exchange block.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > "$OUT/pack_tests.log" 2>&1
rc=$?; tail -3 "$OUT/pack_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/exchange_bench.py | tee "$OUT/exchange_4096.json" || exit $?
timeout -k 10 120 python tools/exchange_bench.py --E 65536 | tee "$OUT/exchange_65536.json" || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 20 --no-cpu-baseline > "$OUT/bench_pack.log" 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"exchange": {[^}]*}' "$OUT/bench_pack.log"
