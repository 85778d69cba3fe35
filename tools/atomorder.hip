#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* out, int mode) {
    __shared__ unsigned c[64];
    if (threadIdx.x < 64) c[threadIdx.x] = 0;
    __syncthreads();
    unsigned l = threadIdx.x;
    unsigned key = mode == 0 ? 0 : (mode == 1 ? (l * 7) % 5 : ((l * 2654435761u) >> 28) & 3);
    unsigned r = atomicAdd(&c[key], 1u);
    out[blockIdx.x * 256 + threadIdx.x] = (key << 16) | r;
}
int main() {
    unsigned* d; hipMalloc(&d, 1024 * 256 * 4);
    unsigned* h = (unsigned*) malloc(1024 * 256 * 4);
    for (int mode = 0; mode < 3; ++mode) {
        hipLaunchKernelGGL(k, dim3(1024), dim3(256), 0, 0, d, mode);
        hipMemcpy(h, d, 1024 * 256 * 4, hipMemcpyDeviceToHost);
        long bad = 0, badwave = 0;
        for (int b = 0; b < 1024; ++b) for (int w = 0; w < 4; ++w) {
            // within a wave: for equal keys, returns must increase with lane
            for (int i = 0; i < 64; ++i) for (int j = i + 1; j < 64; ++j) {
                unsigned a = h[b * 256 + w * 64 + i], c2 = h[b * 256 + w * 64 + j];
                if ((a >> 16) == (c2 >> 16) && (a & 0xFFFF) > (c2 & 0xFFFF)) bad++;
            }
        }
        printf("mode %d: lane-order violations within a wave: %ld\n", mode, bad);
    }
    return 0;
}
