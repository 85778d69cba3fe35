#!/bin/bash
# One GPU call: the -m gpu suite, then optional A/B / bench steps; stops at the
# first step that fails (a test failure included: nothing else runs after it).
# usage: tools/gpu_round.sh TAG [tests|notests] [cmd ...]   (each cmd a quoted shell string)
cd "$(dirname "$0")/.."
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
if [ "$1" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
fi
shift
for c in "$@"; do
  echo "== $c"
  bash -c "$c" || exit $?
done
