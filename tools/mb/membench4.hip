// Microbenchmark (diagnostic, not product): the decoder's per-step record
// read-modify-write (64-B record, 256 per lane, one dependent chain per lane,
// 65536 lanes) with the cache-policy bits of the record load and store varied
// (gfx950 sc0 / sc1 / nt on global_load_dwordx4 / global_store_dwordx4).
// Question: does any policy make the L2 fetch 64 B instead of a 128-B line,
// or make the write-back cheaper?  Reports ns per step.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

#define LD4(pol)                                                                                              \
    asm volatile("global_load_dwordx4 %0, %4, off " pol "\n"                                                  \
                 "global_load_dwordx4 %1, %4, off offset:16 " pol "\n"                                        \
                 "global_load_dwordx4 %2, %4, off offset:32 " pol "\n"                                        \
                 "global_load_dwordx4 %3, %4, off offset:48 " pol "\n"                                        \
                 "s_waitcnt vmcnt(0)"                                                                         \
                 : "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)                                                 \
                 : "v"(q)                                                                                     \
                 : "memory")
#define ST4(pol)                                                                                              \
    asm volatile("global_store_dwordx4 %4, %0, off " pol "\n"                                                 \
                 "global_store_dwordx4 %4, %1, off offset:16 " pol "\n"                                       \
                 "global_store_dwordx4 %4, %2, off offset:32 " pol "\n"                                       \
                 "global_store_dwordx4 %4, %3, off offset:48 " pol "\n"                                       \
                 :                                                                                            \
                 : "v"(c0), "v"(c1), "v"(c2), "v"(c3), "v"(w)                                                 \
                 : "memory")

template <int LP, int SP>
__global__ __launch_bounds__(256) void chain(uint8_t* pool, uint32_t steps, uint32_t* out)
{
    const uint32_t lane = blockIdx.x * 256 + threadIdx.x;
    uint8_t* reg = pool + static_cast<size_t>(lane) * 16384;
    uint32_t x = lane * 2654435761u + 12345u, acc = 0, p = 0;
    v4u c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (uint32_t i = 0; i < steps; ++i) {
        acc += c0.x ^ c1.y ^ c2.z ^ c3.w;
        x = (x ^ (acc & 1)) * 1664525u + 1013904223u;
        const uint32_t v = (x >> 8) & 255;
        const uint8_t* q = reg + v * 64;
        v4u v0, v1, v2, v3;
        if (LP == 0) LD4("");
        else if (LP == 1) LD4("nt");
        else if (LP == 2) LD4("sc0 sc1");
        else if (LP == 3) LD4("sc1");
        else LD4("sc0");
        c0.x += 1;
        uint8_t* w = reg + p * 64;
        if (SP == 0) ST4("");
        else if (SP == 1) ST4("nt");
        else if (SP == 2) ST4("sc0 sc1");
        else ST4("sc1");
        p = v;
        c0 = v0; c1 = v1; c2 = v2; c3 = v3;
    }
    out[lane] = acc;
}

template <int LP, int SP>
void run(uint8_t* pool, uint32_t lanes, uint32_t steps, uint32_t* out, const char* name)
{
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    chain<LP, SP><<<lanes / 256, 256>>>(pool, 40, out);
    hipEventRecord(a);
    chain<LP, SP><<<lanes / 256, 256>>>(pool, steps, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-28s lanes=%6u steps=%u : %7.1f ns/step\n", name, lanes, steps, ms * 1e6 / steps);
}

int main()
{
    const uint32_t lanes = 65536, steps = 600;
    uint8_t* pool; uint32_t* out;
    if (hipMalloc(&pool, static_cast<size_t>(lanes) * 16384) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(pool, 0, static_cast<size_t>(lanes) * 16384);
    hipMalloc(&out, 4 * lanes);
    run<0, 0>(pool, lanes, steps, out, "load -, store -");
    run<1, 0>(pool, lanes, steps, out, "load nt, store -");
    run<2, 0>(pool, lanes, steps, out, "load sc0 sc1, store -");
    run<3, 0>(pool, lanes, steps, out, "load sc1, store -");
    run<4, 0>(pool, lanes, steps, out, "load sc0, store -");
    run<0, 1>(pool, lanes, steps, out, "load -, store nt");
    run<1, 1>(pool, lanes, steps, out, "load nt, store nt");
    run<0, 2>(pool, lanes, steps, out, "load -, store sc0 sc1");
    run<2, 2>(pool, lanes, steps, out, "load sc0 sc1, store sc0 sc1");
    run<0, 3>(pool, lanes, steps, out, "load -, store sc1");
    run<0, 0>(pool, lanes, steps, out, "load -, store - (again)");
    return 0;
}
