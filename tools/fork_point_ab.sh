#!/bin/bash
# A/B of the closure's mean fork point (GPU box): bash tools/fork_point_ab.sh
for v in 0 2 3 0 2 3; do
  if [ $v = 0 ]; then unset CDX_FORK_MEAN; else export CDX_FORK_MEAN=$v; fi
  timeout -k 10 200 python -u bench.py --steps 50 --warmup 20 --no-cpu-baseline > gpurun_out/fork_$v.log 2>&1 || exit $?
  echo "fork=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fork_$v.log)"
done
