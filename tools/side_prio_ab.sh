#!/bin/bash
# A/B of where the closure forks the GPIS mean onto its side stream (CDX_FORK_MEAN) and at which
# priority that stream runs (CDX_SIDE_PRIO), ROUNDS interleaved rounds of bench.py per variant
# (VARIANTS = "fork,prio,lean ..."; lean = CDX_MEAN_LEAN).
# Each bench run has its own time limit; a crash or timeout ends the call.
set -u
OUT=gpurun_out/side_prio_ab
mkdir -p "$OUT"
ROUNDS=${ROUNDS:-2}
VARIANTS=${VARIANTS:-"2,0,0 2,-1,0 2,1,0 4,0,0 4,-1,0"}
for round in $(seq 1 $ROUNDS); do
  for v in $VARIANTS; do
    v=${v//,/ }
    set -- $v
    tag="fork$1_prio$2_lean$3_r$round"
    CDX_FORK_MEAN=$1 CDX_SIDE_PRIO=$2 CDX_MEAN_LEAN=$3 timeout -k 10 120 python -u bench.py --steps 50 --warmup 20 --no-cpu-baseline > "$OUT/$tag.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; tail -5 "$OUT/$tag.log"; exit $rc; fi
    python - "$OUT/$tag.log" "$tag" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith('{')][-1]
d = json.loads(line)
print(f"{sys.argv[2]:20s} {d['ms_per_step']:.4f} ms  {d['value']/1e6:.3f} M evals/s  bound_misses {d['screen']['bound_misses']}")
EOF
  done
done
