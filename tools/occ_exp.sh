cd /root/repo
B="python bench.py --no-cpu --no-pcie --no-crc --steps 5"
for cfg in "A 64" "W 64" "W 32" "A 32"; do set -- $cfg
  ENET_RC_LIB=$PWD/enet_amd/lib/libenet_rc_amd_$1.so ENET_RC_LANES=$2 timeout -k 10 200 $B > gpurun_out/occ_$1_$2.log 2>&1 || exit 1
done
ENET_RC_LIB=$PWD/enet_amd/lib/libenet_rc_amd_W.so ENET_RC_SLOTS=131072 timeout -k 10 200 $B --workload c4 --packets 1048576 --steps 2 > gpurun_out/occ_W_c4s131k.log 2>&1
ENET_RC_LIB=$PWD/enet_amd/lib/libenet_rc_amd_A.so timeout -k 10 200 $B --workload c4 --packets 1048576 --steps 2 > gpurun_out/occ_A_c4.log 2>&1
for f in gpurun_out/occ_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["compress_GiBps"], d["decompress_GiBps"], d["bit_exact_roundtrip"])')"; done
