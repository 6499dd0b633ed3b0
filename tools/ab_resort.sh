# re-sort interval of the fused loop's query points (CDX_SDF_RESORT), with the batched launch's schedule
set -e
for r in 1 2; do
  for v in 4 8 16 1000; do
    CDX_SDF_RESORT=$v timeout -k 10 200 python -u tools/c4_kin.py 40 5 > gpurun_out/c4resort_${v}_$r.json
  done
done
