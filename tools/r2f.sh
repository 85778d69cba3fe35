set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2f
cd /tmp && export TMPDIR=/tmp
for L in 64 32; do
ENET_RC_ENC2_LANES=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2f/kt$L -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --steps 3 --warmup 1 > $R/gpurun_out/r2f/bench$L.log 2>&1; echo "rc=$?"
find $R/gpurun_out/r2f/kt$L -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-4 | head -4
grep -o '"bit_exact_roundtrip": [a-z]*' $R/gpurun_out/r2f/bench$L.log
done
