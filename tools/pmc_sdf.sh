#!/bin/bash
# PMC passes (one counter group per run) over tools/sdf_child.py: the config-4 TorchSDF forward.
#   bash tools/pmc_sdf.sh <tag>      (on the GPU box; CDX_LIB selects the library; SDF_BATCH=1: the loop's batched
#                                    launch, sdf_tree_batch_kernel, with its schedule)
set -u
TAG=${1:-r05}
OUT=gpurun_out/pmc_sdf_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for G in "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CU_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
         "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d "$OUT/p$i" -o run -- python3 tools/sdf_child.py 3 around ${SDF_BATCH:+batch} \
    > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
KNAME=sdf_tree_kernel; [ -n "${SDF_BATCH:-}" ] && KNAME=sdf_tree_batch
python3 tools/pmc_kernel_summary.py "$OUT" $KNAME > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
exit 0
