#!/bin/bash
# MFMA-utilisation / LDS / stall counters of the closure's kernels (screen, refine, ∇std), one
# counter group per rocprofv3 run over a short bench.  bash tools/pmc_closure.sh <tag>   (GPU box)
set -u
TAG=${1:-r02}
OUT=gpurun_out/pmc_closure_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for G in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_F64" \
         "SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_INST_ANY" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"; do
  i=$((i + 1))
  timeout -k 10 200 rocprofv3 --pmc $G --output-format csv -d "$OUT/p$i" -o run -- \
    python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
