set -o pipefail
mkdir -p gpurun_out/r3g
bash tools/abenv.sh r3g "ENET_RC_ENC2_WIDE=0" "ENET_RC_ENC2_WIDE=1" "c3 c2" 2 > gpurun_out/r3g/ab_summary.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3g/kt -o kt -- python bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-configs --no-multi --steps 5 --workload c3 > gpurun_out/r3g/bench_kt_c3.log 2>&1
