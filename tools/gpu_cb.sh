#!/bin/bash
# Combine-block A/B (64 default vs 256) and the mean forked beside the screen (with var-late).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=${1:-r03z}
bash tools/gpu_ab_bench.sh "$TAG" 3 base cb256 base+CDX_KABSCH_AHEAD=0+CDX_FORK_MEAN=1 || exit $?
bash tools/gpu_ab_trace.sh "$TAG" base || exit $?
