#!/bin/bash
# Interleaved bench A/B of library builds / env settings on one box (ms_per_step of an unprofiled
# bench, R rounds): bash tools/gpu_ab_bench.sh TAG R spec1 spec2 ...
# spec = lib name ("base" = libcdx.so) optionally followed by +VAR=VAL settings.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=$1; R=$2; shift 2
OUT=$ROOT/gpurun_out/abb_$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for SPEC in "$@"; do
    IFS=+ read -r L ENVS <<< "$SPEC"
    for v in $(compgen -e | grep '^CDX_'); do unset "$v"; done  # each spec starts from the defaults
    if [ -n "$ENVS" ]; then for kv in ${ENVS//+/ }; do export "$kv"; done; fi
    if [ "$L" = base ]; then export CDX_LIB=$ROOT/compliancedex_amd/lib/libcdx.so; else export CDX_LIB=$ROOT/compliancedex_amd/lib/libcdx_$L.so; fi
    timeout -k 10 200 python3 "$ROOT/bench.py" --steps 50 --warmup 20 --no-cpu-baseline > "$OUT/run.log" 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$SPEC rc=$rc"; tail -5 "$OUT/run.log"; exit $rc; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/run.log') if l.startswith('{')][-1]); print(json.dumps({'spec': '$SPEC', 'round': $r, 'ms_per_step': d['ms_per_step'], 'stage_ms': d['stage_ms'], 'exact_rows': d.get('screen', {}).get('exact_rows')}))" | tee -a "$OUT/ab.jsonl"
  done
done
exit 0
