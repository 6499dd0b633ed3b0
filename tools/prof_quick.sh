#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench (GPU box): bash tools/prof_quick.sh <tag>
set -u
export TMPDIR=/tmp
TAG=${1:-q}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profq_$TAG -o run -- \
  python3 bench.py --steps 30 --warmup 20 --no-cpu-baseline > gpurun_out/profq_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"
[ $rc -eq 0 ] && head -16 gpurun_out/profq_$TAG/run_kernel_stats.csv | cut -c1-60,180-260
exit $rc
