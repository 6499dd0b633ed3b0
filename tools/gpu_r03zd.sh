#!/bin/bash
# ∇std finalize: folded into the combine (default) vs its own kernel, interleaved; refine per-piece timeline.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_ab_bench.sh r03zd 3 base base+CDX_GRAD_FOLD=0 || exit $?
CDX_LIB=$ROOT/compliancedex_amd/lib/libcdx_wgtime.so timeout -k 10 120 python tools/refine_pieces.py \
  | tee gpurun_out/refine_pieces_r03zd.json || exit $?
