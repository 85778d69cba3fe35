set -e
timeout -k 10 300 python -m pytest tests/test_crc.py tests/test_integration.py -m gpu -x -q > gpurun_out/pytest_crc.log 2>&1 || { echo crc_fail; }
B="python bench.py --no-cpu --no-pcie --steps 3 --warmup 1"
for L in 64 32; do ENET_RC_LANES=$L timeout -k 10 200 $B > gpurun_out/exp_c2_L$L.log 2>&1; done
ENET_RC_SLOTS=131072 timeout -k 10 200 $B --no-crc --workload c4 --packets 1048576 --steps 2 > gpurun_out/exp_c4_s131k.log 2>&1
ENET_RC_LANES=32 ENET_RC_SLOTS=131072 timeout -k 10 200 $B --no-crc --workload c4 --packets 1048576 --steps 2 > gpurun_out/exp_c4_L32_s131k.log 2>&1
echo fin
