set -e
for r in 1 2; do
  for v in 0 1; do
    CDX_SDF_SCHED=$v timeout -k 10 200 python -u tools/c4_kin.py 40 5 > gpurun_out/c4sched_${v}_$r.json
  done
done
CDX_SDF_SCHED=1 timeout -k 10 200 python -u tools/sdf_child.py 10 around batch > gpurun_out/sdfb_sched_around.json
CDX_SDF_SCHED=1 CDX_LIB=compliancedex_amd/lib/libcdx_sdfdiag.so timeout -k 10 200 python -u tools/sdf_child.py 10 around batch > gpurun_out/sdfb_sched_diag_around.json
