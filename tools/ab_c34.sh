#!/bin/bash
# A/B of library builds on C2, C3 and C4 (1 Mi packets): tools/ab_c34.sh "A B" [rounds]
cd "$(dirname "$0")/.."
for r in $(seq 1 ${2:-1}); do
  for x in $1; do
    L=$PWD/enet_amd/lib/libenet_rc_amd_$x.so
    ENET_RC_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-crc --no-dgram --steps 8 > gpurun_out/ab_${x}_c2_$r.log 2>&1 || exit 1
    ENET_RC_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-pcie --no-crc --no-dgram --steps 4 --workload c3 > gpurun_out/ab_${x}_c3_$r.log 2>&1 || exit 1
    ENET_RC_LIB=$L timeout -k 10 300 python bench.py --no-cpu --no-pcie --no-crc --no-dgram --steps 2 --workload c4 --packets 1048576 > gpurun_out/ab_${x}_c4_$r.log 2>&1 || exit 1
  done
done
for f in gpurun_out/ab_*_c*_*.log; do echo "$f $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["compress_GiBps"], d["decompress_GiBps"], d["bit_exact_roundtrip"])')"; done
