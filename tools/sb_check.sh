# Small-batch routing check: GPU parity, batch latency vs size, live hosts, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests2.log 2>&1 && \
timeout -k 10 240 python -u tools/smallbatch.py > gpurun_out/smallbatch3.log 2>&1 && \
timeout -k 10 120 bash tools/fan_cmp.sh && \
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/bench_sb.log 2>&1
