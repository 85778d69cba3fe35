set -e
B="python bench.py --no-cpu --no-pcie --no-crc --steps 3 --warmup 1"
for L in 64 32 16; do ENET_RC_LANES=$L timeout -k 10 200 $B > gpurun_out/exp_c2_L$L.log 2>&1; done
timeout -k 10 200 $B --workload c4 --packets 1048576 --steps 2 > gpurun_out/exp_c4_s64k.log 2>&1
ENET_RC_SLOTS=131072 timeout -k 10 200 $B --workload c4 --packets 1048576 --steps 2 > gpurun_out/exp_c4_s131k.log 2>&1
ENET_RC_SLOTS=262144 timeout -k 10 200 $B --workload c4 --packets 1048576 --steps 2 > gpurun_out/exp_c4_s262k.log 2>&1
echo fin
