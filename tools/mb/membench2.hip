// Microbenchmark (diagnostic, not product): the bucket-history decoder's
// access pattern with its dependent compute, for candidate record layouts.
// Per lane and step: one random record read-modify-write in a primary table
// (REC bytes per record, 256 records per lane), with probability P/256 a
// second read-modify-write of OVF bytes in an overflow table (issued with the
// first), then `sleep` x 64 cycles of dependent "compute" before the next
// address is known.  Reports ns per step.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

template <int REC, int OVF>
__global__ __launch_bounds__(256) void chain(uint8_t* pool, uint8_t* ovf, uint32_t steps, uint32_t p, uint32_t* out,
                                             int sleep)
{
    const uint32_t lane = blockIdx.x * 256 + threadIdx.x;
    uint8_t* reg = pool + static_cast<size_t>(lane) * 256 * REC;
    uint8_t* oreg = ovf + static_cast<size_t>(lane) * 256 * 64;
    uint32_t x = lane * 2654435761u + 12345u, acc = 0;
    for (uint32_t i = 0; i < steps; ++i) {
        x = x * 1664525u + 1013904223u;
        const uint32_t r = (x >> 8) & 255;
        const bool o = ((x >> 20) & 255) < p;
        uint4* q = reinterpret_cast<uint4*>(reg + static_cast<size_t>(r) * REC);
        uint4 v[REC / 16], w[OVF / 16 + 1];
#pragma unroll
        for (int k = 0; k < REC / 16; ++k) v[k] = q[k];
        uint4* qo = reinterpret_cast<uint4*>(oreg + static_cast<size_t>(r) * 64);
        if (OVF && o) {
#pragma unroll
            for (int k = 0; k < OVF / 16; ++k) w[k] = qo[k];
        }
#pragma unroll
        for (int k = 0; k < REC / 16; ++k) acc += v[k].x ^ v[k].w;
        if (OVF && o) {
#pragma unroll
            for (int k = 0; k < OVF / 16; ++k) acc += w[k].y;
        }
        if (sleep > 0) __builtin_amdgcn_s_sleep(30);
        if (sleep > 1) __builtin_amdgcn_s_sleep(30);
        x ^= acc & 1;   // the next address depends on the data
#pragma unroll
        for (int k = 0; k < REC / 16; ++k) { v[k].x += 1; q[k] = v[k]; }
        if (OVF && o) {
#pragma unroll
            for (int k = 0; k < OVF / 16; ++k) { w[k].x += 1; qo[k] = w[k]; }
        }
    }
    out[lane] = acc;
}

template <int REC, int OVF>
void run(uint8_t* pool, uint8_t* ovf, uint32_t lanes, uint32_t p, int sleep, uint32_t* out)
{
    const uint32_t steps = 300;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    chain<REC, OVF><<<lanes / 256, 256>>>(pool, ovf, 40, p, out, sleep);
    hipEventRecord(a);
    chain<REC, OVF><<<lanes / 256, 256>>>(pool, ovf, steps, p, out, sleep);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("rec=%3d ovf=%2d p=%3u/256 sleep=%d lanes=%6u table=%7.1f MB : %7.1f ns/step\n", REC, OVF, p, sleep, lanes,
           (double) lanes * 256 * REC / 1e6, ms * 1e6 / steps);
}

int main()
{
    uint8_t *pool, *ovf; uint32_t* out;
    const uint32_t lanes = 65536;
    if (hipMalloc(&pool, (size_t) lanes * 256 * 64) != hipSuccess) return 1;
    if (hipMalloc(&ovf, (size_t) lanes * 256 * 64) != hipSuccess) return 1;
    hipMemset(pool, 0, (size_t) lanes * 256 * 64);
    hipMemset(ovf, 0, (size_t) lanes * 256 * 64);
    hipMalloc(&out, 4 * lanes);
    for (int sleep : {0, 1, 2}) {
        run<64, 0>(pool, ovf, lanes, 0, sleep, out);
        run<32, 0>(pool, ovf, lanes, 0, sleep, out);
        run<16, 0>(pool, ovf, lanes, 0, sleep, out);
        run<16, 48>(pool, ovf, lanes, 31, sleep, out);
        run<16, 48>(pool, ovf, lanes, 64, sleep, out);
        run<32, 32>(pool, ovf, lanes, 31, sleep, out);
    }
    return 0;
}
