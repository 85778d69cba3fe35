set -o pipefail
PMC_TAG=r3d_pmc_dec4 PMC_KERNEL=rc_decompress_dec4 ENET_RC_DEC=4 bash tools/pmc_dec4.sh > gpurun_out/r3d_dec4.txt 2>&1
PMC_TAG=r3d_pmc_dec5 PMC_KERNEL=rc_decompress_dec5 ENET_RC_DEC=5 bash tools/pmc_dec4.sh > gpurun_out/r3d_dec5.txt 2>&1
