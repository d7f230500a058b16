set -u
cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu_aggregation.py tests/test_gpu_train.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/gpu_tests3.log 2>&1
echo rc=$? >> gpurun_out/gpu_tests3.log
timeout -k 10 300 python -u bench.py --config C4 --steps 2 --warmup 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
echo rc=$? >> gpurun_out/bench_c4.err
