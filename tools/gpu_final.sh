#!/bin/bash
# Round-end GPU call: tests → smoke → bench → rocprof kernel trace → HBM PMC passes → closure timeline →
# the screen's MFMA-busy PMC pass.   bash tools/gpu_final.sh TAG
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=${1:-r03}
bash tools/gpu_r3.sh "$TAG" full || exit $?
export TMPDIR=/tmp
python3 tools/closure_timeline.py "gpurun_out/prof_$TAG/run_kernel_trace.csv" > "gpurun_out/closure_timeline_$TAG.txt" 2>&1
OUT=gpurun_out/pmc_screen_$TAG; mkdir -p "$OUT"
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
  --output-format csv -d "$OUT/p1" -o run -- python3 tools/screen_variants.py child "$ROOT/compliancedex_amd/lib/libcdx.so" 4096 \
  > "$OUT/p1.log" 2>&1
echo "screen pmc rc=$?"
exit 0
