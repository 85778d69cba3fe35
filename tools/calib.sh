#!/bin/bash
# Counter calibration (round-5 review item 9): tools/mb/calib's kernels under
# separate rocprofv3 --pmc passes; tools/calib.py turns them into requests and
# bytes per access.  usage (GPU box): tools/calib.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=$1; O=$R/gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $R/tools/mb/calib > $O/calib.log 2>&1 || exit 1
i=0
for grp in "TCC_EA0_WRREQ TCC_EA0_WRREQ_64B" "TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $O/pmc$i -o run -- $R/tools/mb/calib > $O/pmc$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 $R/tools/calib.py $O > $O/calib_summary.txt && cat $O/calib_summary.txt
