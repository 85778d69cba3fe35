// Microbenchmark (diagnostic, not product): the decoder's per-step record
// traffic with the bucket records kept in place (read bucket v, write bucket
// p back where it was: a random read-modify-write, today's layout) against a
// per-lane append log (read bucket v at log[ptr[v]], write the new version of
// bucket p to the lane's next log slot: the writes become sequential per lane
// and two consecutive steps fill one 128-B line).  ptr[] per lane: LDS (u16)
// or a small global table.  Reports ns per step; `sleep` adds dependent
// compute before the next address is known.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

// mode 0: in place; 1: log, ptr in LDS; 2: log, ptr in a global table; 3: log, no
// ptr (read a random earlier slot of the log: the traffic without the lookup)
template <int MODE>
__global__ __launch_bounds__(256) void chain(uint8_t* pool, size_t region, uint16_t* gptr, uint32_t steps,
                                             uint32_t* out, int sleep)
{
    __shared__ uint16_t sptr[256 * 256];
    const uint32_t lane = blockIdx.x * 256 + threadIdx.x;
    uint8_t* reg = pool + static_cast<size_t>(lane) * region;
    uint16_t* lp = MODE == 1 ? sptr + threadIdx.x : gptr + static_cast<size_t>(lane) * 256;
    const uint32_t ps = MODE == 1 ? 256 : 1;   // LDS: interleaved by lane (no bank conflicts)
    if (MODE == 1 || MODE == 2)
        for (uint32_t r = 0; r < 256; ++r) lp[r * ps] = static_cast<uint16_t>(r);
    uint32_t x = lane * 2654435761u + 12345u, acc = 0, p = 0, slot = 256;
    uint4 cur[4];
    const uint4* q0 = reinterpret_cast<const uint4*>(reg);
    for (int k = 0; k < 4; ++k) cur[k] = q0[k];
    for (uint32_t i = 0; i < steps; ++i) {
        for (int k = 0; k < 4; ++k) acc += cur[k].x ^ cur[k].w;
        if (sleep > 0) __builtin_amdgcn_s_sleep(30);
        if (sleep > 1) __builtin_amdgcn_s_sleep(30);
        x = (x ^ (acc & 1)) * 1664525u + 1013904223u;
        const uint32_t v = (x >> 8) & 255;
        uint32_t src;
        if (MODE == 0) src = v;
        else if (MODE == 3) src = (x >> 16) % slot;
        else src = lp[v * ps];
        const uint4* q = reinterpret_cast<const uint4*>(reg + static_cast<size_t>(src) * 64);
        uint4 nx[4];
        for (int k = 0; k < 4; ++k) nx[k] = q[k];
        for (int k = 0; k < 4; ++k) cur[k].x += 1;
        const uint32_t dst = MODE == 0 ? p : slot;
        uint4* w = reinterpret_cast<uint4*>(reg + static_cast<size_t>(dst) * 64);
        for (int k = 0; k < 4; ++k) w[k] = cur[k];
        if (MODE == 1 || MODE == 2) lp[p * ps] = static_cast<uint16_t>(slot);
        ++slot;
        p = v;
        for (int k = 0; k < 4; ++k) cur[k] = nx[k];
    }
    out[lane] = acc;
}

template <int MODE>
void run(uint8_t* pool, size_t region, uint16_t* gptr, uint32_t lanes, uint32_t steps, int sleep, uint32_t* out)
{
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    chain<MODE><<<lanes / 256, 256>>>(pool, region, gptr, 40, out, sleep);
    hipEventRecord(a);
    chain<MODE><<<lanes / 256, 256>>>(pool, region, gptr, steps, out, sleep);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const char* names[] = {"in place     ", "log, ptr LDS ", "log, ptr HBM ", "log, no ptr  "};
    printf("%s sleep=%d lanes=%6u steps=%u : %7.1f ns/step\n", names[MODE], sleep, lanes, steps,
           ms * 1e6 / steps);
}

int main()
{
    const uint32_t lanes = 65536, steps = 1000;
    const size_t region = static_cast<size_t>(256 + steps + 64) * 64;   // 84 KB per lane, 5.5 GB
    uint8_t* pool; uint16_t* gptr; uint32_t* out;
    if (hipMalloc(&pool, region * lanes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(pool, 0, region * lanes);
    hipMalloc(&gptr, static_cast<size_t>(lanes) * 512);
    hipMalloc(&out, 4 * lanes);
    for (int sleep : {0, 2}) {
        run<0>(pool, region, gptr, lanes, steps, sleep, out);
        run<1>(pool, region, gptr, lanes, steps, sleep, out);
        run<2>(pool, region, gptr, lanes, steps, sleep, out);
        run<3>(pool, region, gptr, lanes, steps, sleep, out);
    }
    return 0;
}
