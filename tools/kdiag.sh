# kin_cost4 time split: the kernel in diagnostic builds without the force-equilibrium reward / the FK backward /
# the SVD (outputs wrong; timing only), under rocprofv3 kernel stats over tools/c4_kin.py
set -e
for v in base knofe knofk knosvd; do
  lib=compliancedex_amd/lib/libcdx.so; [ $v != base ] && lib=compliancedex_amd/lib/libcdx_$v.so
  CDX_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kdiag_$v -o run -- python3 tools/c4_kin.py 10 2 > gpurun_out/kdiag_$v.log 2>&1
done
