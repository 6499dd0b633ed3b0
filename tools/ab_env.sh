#!/bin/bash
# A/B of an environment switch on bench.py (GPU box): alternates VAR=a / VAR=b runs, one JSON line each.
#   bash tools/ab_env.sh VAR a b [rounds] [tag]
set -u
VAR=$1; A=$2; B=$3; N=${4:-3}; TAG=${5:-ab}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
for i in $(seq 1 "$N"); do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 200 python bench.py --steps 50 --warmup 20 --no-cpu-baseline > "$OUT/ab_tmp.json" 2>/dev/null
    rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; exit $rc; }
    python -c "
import json,sys
d=json.loads(open('$OUT/ab_tmp.json').read().strip().splitlines()[-1])
print(json.dumps({'$VAR': '$v', 'ms_per_step': d['ms_per_step'], 'value': d['value'], 'exact_rows': d.get('screen',{}).get('exact_rows')}))
" | tee -a "$OUT/ab_$TAG.jsonl"
  done
done
