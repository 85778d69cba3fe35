set -o pipefail
mkdir -p gpurun_out/r2b
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "lane3" > gpurun_out/r2b/tests.log 2>&1; echo "tests rc=$?"
tail -3 gpurun_out/r2b/tests.log
timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl > gpurun_out/r2b/bench_c2.log 2>&1; echo "bench rc=$?"
tail -c 1500 gpurun_out/r2b/bench_c2.log
