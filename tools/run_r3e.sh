set -o pipefail
mkdir -p gpurun_out/r3e
ENET_RC_DEC=5 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lane3 and not only and (digest or fixtures or fuzz or c4 or long)" > gpurun_out/r3e/gpu_tests_dec5.log 2>&1 && \
bash tools/abenv.sh r3e "ENET_RC_DEC=4" "ENET_RC_DEC=5" "c2" 3 > gpurun_out/r3e/ab_summary.log 2>&1
