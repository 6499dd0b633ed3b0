# bad (non-finite / out-of-range) points in the tree kernel: the point's faces split over a wave (base) vs the whole
# group by the tile rule (exgrp, CDX_SDF_EXACT_GROUP); the SDF GPU tests, then the Kin loop at 20 and 100 iterations
set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sdf or fused or config4 or one_launch" > gpurun_out/pytest_exact.log 2>&1
for r in 1 2; do
  for v in exgrp base; do
    lib=compliancedex_amd/lib/libcdx.so; [ $v != base ] && lib=compliancedex_amd/lib/libcdx_$v.so
    CDX_LIB=$lib timeout -k 10 200 python -u tools/c4_kin.py 20 3 > gpurun_out/c4exact20_${v}_$r.json
    CDX_LIB=$lib timeout -k 10 200 python -u tools/c4_kin.py 100 2 > gpurun_out/c4exact100_${v}_$r.json
  done
done
