#!/bin/bash
# PMC passes (one counter group per run) over tools/c4_kin.py: config 4's fused Kin loop, kin_cost4_kernel.
#   bash tools/pmc_kin.sh <tag>      (on the GPU box; CDX_LIB selects the library)
set -u
TAG=${1:-r06}
OUT=gpurun_out/pmc_kin_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for G in "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CU_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_WAIT_INST_LDS" \
         "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "$OUT/p$i" -o run -- python3 tools/c4_kin.py 5 1 \
    > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -3 "$OUT/p$i.log"; }
done
python3 tools/pmc_kernel_summary.py "$OUT" kin_cost4 > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
exit 0
