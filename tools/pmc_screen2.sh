#!/bin/bash
# Stall-breakdown PMC passes (one counter group per run) of the screen kernel over the timing child of
# tools/screen_variants.py.   bash tools/pmc_screen2.sh <lib path> <tag>      (on the GPU box)
set -u
LIB=${1:-compliancedex_amd/lib/libcdx.so}; TAG=${2:-r03}
OUT=gpurun_out/pmc_screen_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for G in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAIT_INST_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_VMEM_RD" \
         "SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT"; do
  i=$((i + 1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "$OUT/p$i" -o run -- \
    python3 tools/screen_variants.py child "$PWD/$LIB" 4096 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
done
exit 0
