set -o pipefail
mkdir -p gpurun_out/r3f
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3f/gpu_tests_wide.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "digest or c4 or fixtures" > gpurun_out/r3f/gpu_tests_parity.log 2>&1 && \
bash tools/abenv.sh r3f "ENET_RC_ENC2_WIDE=0" "ENET_RC_ENC2_WIDE=1" "c3 c2" 1 > gpurun_out/r3f/ab_summary.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3f/kt -o kt -- python bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 5 --workload c3 > gpurun_out/r3f/bench_kt_c3.log 2>&1
