# GPU call: the -m gpu suite with measured-error logging, then the 1-GPU bench and a 2-rank gloo rehearsal.
set -u
mkdir -p gpurun_out
TAG=${1:-r02}
rm -f gpurun_out/parity_$TAG.jsonl
CDX_PARITY_LOG=$PWD/gpurun_out/parity_$TAG.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu_$TAG.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
python tools/parity_report.py gpurun_out/parity_$TAG.jsonl > gpurun_out/parity_errors_$TAG.txt
timeout -k 10 300 python bench.py --steps 50 --warmup 20 > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --backend gloo > gpurun_out/bench2_gloo_$TAG.log 2>&1
rc=$?; echo "bench2 rc=$rc"; tail -1 gpurun_out/bench2_gloo_$TAG.log
