# the config-4 loop at the reference's 1000 iterations per call, with the SDF tests first
set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "sdf or fused or config4 or one_launch" > gpurun_out/pytest_c4long.log 2>&1
timeout -k 10 300 python -u tools/c4_kin.py 1000 2 > gpurun_out/c4_1000_nan.json
