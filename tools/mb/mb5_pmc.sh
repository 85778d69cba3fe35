#!/bin/bash
# membench5 timing + TCC request counters per dispatch (run under gpurun)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/mb5
mkdir -p $O
timeout -k 10 120 $R/tools/mb/membench5 > $O/membench5.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_128B TCC_EA0_WRREQ TCC_EA0_WRREQ_64B --output-format csv -d $O/pmc -o run -- $R/tools/mb/membench5 > $O/pmc.log 2>&1
echo done
