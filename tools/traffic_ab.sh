#!/bin/bash
# Fabric traffic per launch of one kernel for library builds (TCC_EA0 request counters, two --pmc passes each).
# usage: tools/traffic_ab.sh TAG WORKLOAD "KERNEL_REGEX" name...   (names as tools/ab_kt.sh; "cur" = the product build)
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; W=$2; K=$3; shift 3
cd /tmp && export TMPDIR=/tmp
for n in "$@"; do
  L=$R/enet_amd/lib/libenet_rc_amd_$n.so; [ $n = cur ] && L=$R/enet_amd/lib/libenet_rc_amd.so
  O=$R/gpurun_out/$T/tr_$n; rm -rf $O; mkdir -p $O
  i=0
  for grp in "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B"; do
    i=$((i+1))
    ENET_RC_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$K" --output-format csv -d $O/pmc$i -o run -- \
      python3 $R/bench.py --workload $W --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 1 --warmup 0 > $O/p$i.log 2>&1 || exit 1
  done
  python3 $R/tools/traffic.py $O $W 65536 $O/traffic.json > /dev/null
  echo "$n: $(python3 -c "import json; t=json.load(open('$O/traffic.json')); print({k: (round((v['hbm_read_bytes_per_launch'] or 0)/1e9, 3), round((v['hbm_write_bytes_per_launch'] or 0)/1e9, 3)) for k, v in t['kernels'].items()})")"
done
