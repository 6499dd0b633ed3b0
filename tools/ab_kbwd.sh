# kin_cost4's FK backward: one walk with the joints' axes / origins in LDS (base) vs two walks (kbwd2)
set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "one_launch or kin or fused or config4 or mode_" > gpurun_out/pytest_kbwd.log 2>&1
for r in 1 2 3; do
  for v in kbwd2 base; do
    lib=compliancedex_amd/lib/libcdx.so; [ $v != base ] && lib=compliancedex_amd/lib/libcdx_$v.so
    CDX_LIB=$lib timeout -k 10 200 python -u tools/c4_kin.py 100 3 > gpurun_out/c4kbwd_${v}_$r.json
  done
done
