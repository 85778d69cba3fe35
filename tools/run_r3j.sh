set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread -k "digest or c4 or long or fuzz or fixtures or wide" > gpurun_out/r3j_tests.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 5 --workload c3 > gpurun_out/r3j_c3.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 10 > gpurun_out/r3j_c2.log 2>&1
timeout -k 10 200 python tools/enc2_prof.py 65536 c3 > gpurun_out/e2prof_c3_w8.log 2>&1
