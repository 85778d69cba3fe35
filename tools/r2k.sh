set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/r2k
cd /tmp && export TMPDIR=/tmp
for V in "" e2b; do
L=""; [ -n "$V" ] && L="$R/enet_amd/lib/libenet_rc_amd_$V.so"
ENET_RC_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2k/kt$V -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-crc --no-dgram --no-rccl --steps 3 --warmup 1 > $R/gpurun_out/r2k/bench$V.log 2>&1; echo "rc=$? $V"
find $R/gpurun_out/r2k/kt$V -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-4 | grep enc2
grep -o '"bit_exact_roundtrip": [a-z]*' $R/gpurun_out/r2k/bench$V.log
done
