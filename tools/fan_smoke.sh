set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 90 oracle/_ref/loopback_deferred fan 47101 200 32 > gpurun_out/fan1.log 2>&1 && \
ENET_LOOPBACK_CHECKSUM=1 timeout -k 10 90 oracle/_ref/loopback_deferred fan 47102 200 32 >> gpurun_out/fan1.log 2>&1 && \
timeout -k 10 90 oracle/_ref/loopback_deferred fan 47103 100 1 >> gpurun_out/fan1.log 2>&1
