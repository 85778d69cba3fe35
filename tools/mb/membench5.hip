// Microbenchmark (diagnostic, not product): smaller decoder records written as
// whole 64-B units.  Per lane 256 records of REC bytes (table = 65536 x 256 x
// REC); a step reads record v (the L2 fetches its 128-B line) and writes back
// the 64-B unit holding the previous step's record p (its neighbours in the
// unit unchanged: the writer holds them from its read).  Question: does a
// table that (mostly) fits the 256-MB Infinity Cache make the random
// read-modify-write step cheaper, when no write is partial?  ns per step.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

template <int REC>
__global__ __launch_bounds__(256) void chain(uint8_t* pool, uint32_t steps, uint32_t* out)
{
    const uint32_t lane = blockIdx.x * 256 + threadIdx.x;
    uint8_t* reg = pool + static_cast<size_t>(lane) * 256 * REC;
    uint32_t x = lane * 2654435761u + 12345u, acc = 0, p = 0;
    uint4 u[4] = {};
    for (uint32_t i = 0; i < steps; ++i) {
        acc += u[0].x ^ u[3].w;
        x = (x ^ (acc & 1)) * 1664525u + 1013904223u;
        const uint32_t v = (x >> 8) & 255;
        const uint4* q = reinterpret_cast<const uint4*>(reg + ((v * REC) & ~63u));   // v's 64-B unit
        uint4 n[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) n[k] = q[k];
        u[0].x += 1;
        uint4* w = reinterpret_cast<uint4*>(reg + ((p * REC) & ~63u));
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = u[k];
        p = v;
#pragma unroll
        for (int k = 0; k < 4; ++k) u[k] = n[k];
    }
    out[lane] = acc;
}

template <int REC>
void run(uint8_t* pool, uint32_t lanes, uint32_t steps, uint32_t* out)
{
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    chain<REC><<<lanes / 256, 256>>>(pool, 40, out);
    hipEventRecord(a);
    chain<REC><<<lanes / 256, 256>>>(pool, steps, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("rec=%3d (64-B units) lanes=%6u table=%7.1f MB : %7.1f ns/step\n", REC, lanes,
           static_cast<double>(lanes) * 256 * REC / 1e6, ms * 1e6 / steps);
}

int main()
{
    const uint32_t lanes = 65536, steps = 600;
    uint8_t* pool; uint32_t* out;
    if (hipMalloc(&pool, static_cast<size_t>(lanes) * 256 * 64) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(pool, 0, static_cast<size_t>(lanes) * 256 * 64);
    hipMalloc(&out, 4 * lanes);
    for (int r = 0; r < 2; ++r) {
        run<64>(pool, lanes, steps, out);
        run<48>(pool, lanes, steps, out);
        run<32>(pool, lanes, steps, out);
        run<24>(pool, lanes, steps, out);
        run<16>(pool, lanes, steps, out);
    }
    return 0;
}
