#!/bin/bash
# Builds lib/libcdx_mean_<name>.so per VARIANTS entry (name:-Dflag,-Dflag; direct = the per-pair TPS mean)
# beside libcdx.so (moment form); on the GPU ("run") times cdx_gpis_mean alone (tools/time_mean.py, M = 53 248 =
# config 2's 13 queries per candidate) and bench.py unforked (CDX_FORK_MEAN=0) for each library.
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
VARIANTS=${VARIANTS:-"direct:-DCDX_MEAN_DIRECT fullsqrt:-DCDX_MEAN_FULLSQRT unroll8:-DCDX_MEAN_UNROLL=8"}
if [ "${1:-}" = build ]; then
  T=$(mktemp -d)
  F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-pass-failed -I $ROOT/include -DCDX_FAST_SQRT -DCDX_STD_SCHED"
  for s in cdx_screen cdx_fit cdx_optim; do /opt/rocm/bin/hipcc $F -c $ROOT/compliancedex_amd/csrc/$s.hip -o $T/$s.o; done
  for s in cdx_closure cdx_sdf; do /opt/rocm/bin/hipcc $F -ffp-contract=off -c $ROOT/compliancedex_amd/csrc/$s.hip -o $T/$s.o; done
  for v in $VARIANTS; do
    /opt/rocm/bin/hipcc $F $(echo ${v#*:} | tr ',' ' ') -c $ROOT/compliancedex_amd/csrc/cdx_gpis.hip -o $T/gpis.o
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $T/cdx_*.o $T/gpis.o -o $ROOT/compliancedex_amd/lib/libcdx_mean_${v%%:*}.so
  done
  rm -rf $T
  exit 0
fi
mkdir -p gpurun_out
for r in 1 2; do
  for lib in libcdx.so $(for v in $VARIANTS; do echo libcdx_mean_${v%%:*}.so; done); do
    echo "== $lib round $r"
    CDX_LIB=$ROOT/compliancedex_amd/lib/$lib timeout -k 10 120 python -u tools/time_mean.py 53248 2000 50
    CDX_LIB=$ROOT/compliancedex_amd/lib/$lib CDX_FORK_MEAN=0 timeout -k 10 120 python -u bench.py --steps 50 --warmup 20 --no-cpu-baseline | python -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print('unforked bench', round(d['ms_per_step'],4), 'ms', d['stage_ms'])"
  done
done
