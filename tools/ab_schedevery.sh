# the batch schedule's order recomputed every launch (1) or every 4th (CDX_SDF_SCHED_EVERY)
set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sdf or fused or config4 or one_launch" > gpurun_out/pytest_schedevery.log 2>&1
for r in 1 2 3; do
  for v in 1 4; do
    CDX_SDF_SCHED_EVERY=$v timeout -k 10 200 python -u tools/c4_kin.py 100 3 > gpurun_out/c4every_${v}_$r.json
  done
done
