#!/bin/bash
# Kernel-trace A/B of library builds on one box: bash tools/gpu_ab_trace.sh TAG lib1 lib2 ...
# (lib = compliancedex_amd/lib/libcdx_<name>.so, "base" = libcdx.so); per lib a rocprofv3 kernel trace of
# a short bench and the per-closure timeline (tools/closure_timeline.py).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=$1; shift
OUT=$ROOT/gpurun_out/ab_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
# a spec may carry environment settings: name+VAR=VAL+VAR2=VAL2 (e.g. base+CDX_MEAN_SPLIT=1)
for SPEC in "$@"; do
  IFS=+ read -r L ENVS <<< "$SPEC"
  for v in $(compgen -e | grep '^CDX_'); do unset "$v"; done  # each spec starts from the defaults
  if [ -n "$ENVS" ]; then for kv in ${ENVS//+/ }; do export "$kv"; done; fi
  if [ "$L" = base ]; then export CDX_LIB=$ROOT/compliancedex_amd/lib/libcdx.so; else export CDX_LIB=$ROOT/compliancedex_amd/lib/libcdx_$L.so; fi
  L=${SPEC//=/-}
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$L" -o run -- python3 "$ROOT/bench.py" --steps 30 --warmup 20 --no-cpu-baseline > "$OUT/$L.log" 2>&1
  rc=$?; echo "$L rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 tools/closure_timeline.py "$OUT/$L/run_kernel_trace.csv" > "$OUT/$L.timeline.txt" 2>&1
  cat "$OUT/$L.timeline.txt"
done
exit 0
