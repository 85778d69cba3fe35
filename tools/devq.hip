// Prints the device attributes launch() in rc_kernels.hip sizes small batches by.
#include <hip/hip_runtime.h>
#include <stdio.h>
int main()
{
    int cus = 0, lds_cu = 0, lds_blk = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, 0);
    hipDeviceGetAttribute(&lds_blk, hipDeviceAttributeMaxSharedMemoryPerBlock, 0);
    printf("{\"cus\": %d, \"lds_per_cu\": %d, \"lds_per_block\": %d}\n", cus, lds_cu, lds_blk);
    return 0;
}
