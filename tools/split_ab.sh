#!/bin/bash
# Interleaved A/B of host-batch settings (ENET_RC_HOST_SPLIT pieces and the
# like), one process per run, so that each run's streams have the hardware
# queues to themselves.
# usage: tools/split_ab.sh TAG rounds workload "ENV=.. ENV=.." "ENV=.." ...
cd "$(dirname "$0")/.."
T=$1; R=$2; W=$3; shift 3
mkdir -p gpurun_out/$T
for r in $(seq 1 $R); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    env $e timeout -k 10 200 python -u tools/split_ab.py 0 ${ITERS:-3} $W > gpurun_out/$T/split_${W}_${i}_$r.log 2>&1 || exit 1
  done
done
i=0
for e in "$@"; do
  i=$((i + 1))
  for f in gpurun_out/$T/split_${W}_${i}_*.log; do echo "[$e] $(tail -2 $f | tr "\n" " ")"; done
done
