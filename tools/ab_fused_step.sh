# one-launch Kin iteration (cdx_kin_iteration) vs cost + step: tests, then an interleaved c4 loop A/B
set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "one_launch or kin or fused or config4" > gpurun_out/pytest_fused_step.log 2>&1
for r in 1 2; do
  for v in 0 1; do
    CDX_KIN_FUSED_STEP=$v timeout -k 10 200 python -u tools/c4_kin.py 40 5 > gpurun_out/c4fstep2_${v}_$r.json
  done
done
