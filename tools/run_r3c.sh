set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 200 python -u -m pytest tests/test_crc.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/gpu_tests_crc.log 2>&1 && \
ENET_RC_DEC=5 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lane3 and not only and (digest or fixtures or fuzz or c4 or long)" > gpurun_out/r3c/gpu_tests_dec5.log 2>&1 && \
bash tools/abenv.sh r3c "ENET_RC_DEC=4" "ENET_RC_DEC=5" "c2 c4" 2 > gpurun_out/r3c/ab_summary.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-dgram --no-configs --no-multi --steps 5 > gpurun_out/r3c/bench_crc.log 2>&1
