#!/bin/bash
# Final checks of a round on one GPU box: the GPU suite, smoke(), the default
# bench line (what the driver runs) and a rocprofv3 kernel-trace summary of
# that same command.  usage: bash tools/final_round.sh TAG  -> gpurun_out/TAG/
set -o pipefail
R=$(pwd); O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo SUITE_FAIL; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py > $O/bench_kt.log 2>&1 || { echo KT_FAIL; exit 1; }
echo done
