# Live-host comparison (32 peers, 200 packets each, two hosts in one process):
# per-datagram GPU coder vs deferred-batch GPU mode vs reference compress.c.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/fan_cmp.log
: > $out
timeout -k 10 90 oracle/_ref/loopback_ref fan 47201 200 32 >> $out 2>&1 && \
timeout -k 10 90 oracle/_ref/loopback_deferred fan 47202 200 32 >> $out 2>&1 && \
timeout -k 10 120 oracle/_ref/loopback_amd fan 47203 200 32 >> $out 2>&1
