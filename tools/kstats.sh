#!/bin/bash
# rocprofv3 kernel stats of bench.py per workload (run under gpurun)
# usage: tools/kstats.sh TAG "c3 c4"
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
for w in $2; do
  O=$R/gpurun_out/ks_$1_$w
  mkdir -p $O
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --steps 3 --warmup 1 --workload $w $([ $w = c4 ] && echo --packets 1048576) > $O/bench.log 2>&1)
done
echo done
