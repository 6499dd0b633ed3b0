# closure_combine_kernel time split: diagnostic builds without the FK backward / without the ∇std fold (outputs
# wrong; timing only), per-closure timeline of each
set -e
for v in base cnofk cnofold; do
  lib=compliancedex_amd/lib/libcdx.so; [ $v != base ] && lib=compliancedex_amd/lib/libcdx_$v.so
  CDX_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cdiag_$v -o run -- python3 bench.py --steps 30 --warmup 20 --no-cpu-baseline --no-config4 > gpurun_out/cdiag_$v.log 2>&1
  python3 tools/closure_timeline.py gpurun_out/cdiag_$v/run_kernel_trace.csv > gpurun_out/cdiag_timeline_$v.txt 2>&1
done
