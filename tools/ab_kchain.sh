# kin_cost4's FK walks on the chain / joint rows staged in LDS vs read from the kernel-argument segment / memory
set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "one_launch or kin or fused or config4" > gpurun_out/pytest_kchain.log 2>&1
for r in 1 2; do
  for v in karg base; do
    lib=compliancedex_amd/lib/libcdx.so; [ $v != base ] && lib=compliancedex_amd/lib/libcdx_$v.so
    CDX_LIB=$lib timeout -k 10 200 python -u tools/c4_kin.py 40 5 > gpurun_out/c4kchain_${v}_$r.json
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kchain_prof -o run -- python3 tools/c4_kin.py 10 2 > gpurun_out/kchain_prof.log 2>&1
