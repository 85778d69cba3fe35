// Microbenchmark (diagnostic, not product): blind stores for a record-light
// decoder.  65536 lanes; per step each lane writes one small element into a
// random record of its own region (no read of that record), optionally loads
// a random 64-B record on a fraction of steps (the rare path; the loaded
// value feeds the lane's chain, so the wavefront waits for it).  Question:
// what does a random partial write cost when nothing reads the line first?
// ns per step.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

// MODE 0: 2-B store at a random record (slot = per-record counter in regs)
// MODE 1: 4-B store at a random record
// MODE 2: 4-B store appended sequentially (per-lane log)
// MODE 3: 64-B read + 64-B write back (the current decoder's pattern)
template <int MODE, int REC, int RARE>
__global__ __launch_bounds__(256) void chain(uint8_t* pool, uint32_t steps, uint32_t* out)
{
    const uint32_t lane = blockIdx.x * 256 + threadIdx.x;
    uint8_t* reg = pool + static_cast<size_t>(lane) * 256 * REC;
    uint32_t x = lane * 2654435761u + 12345u, acc = 0;
    for (uint32_t i = 0; i < steps; ++i) {
        x = (x ^ (acc & 1)) * 1664525u + 1013904223u;
        const uint32_t v = (x >> 8) & 255;
        if (MODE == 0) {
            *reinterpret_cast<uint16_t*>(reg + v * REC + ((i * 2) & (REC - 2))) = static_cast<uint16_t>(x);
        } else if (MODE == 1) {
            *reinterpret_cast<uint32_t*>(reg + v * REC + ((i * 4) & (REC - 4))) = x;
        } else if (MODE == 2) {
            *reinterpret_cast<uint32_t*>(reg + ((i * 4) & (256 * REC - 4))) = x;
        } else {
            uint4* q = reinterpret_cast<uint4*>(reg + v * REC);
            uint4 n[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) n[k] = q[k];
            n[0].x += x;
            acc += n[1].y;
#pragma unroll
            for (int k = 0; k < 4; ++k) q[k] = n[k];
        }
        if (RARE > 0 && ((x >> 20) % RARE) == 0) {
            const uint4* q = reinterpret_cast<const uint4*>(reg + ((x >> 3) & 255) * REC);
            uint4 n = q[0];
            acc += n.x ^ n.w;
        }
    }
    out[lane] = acc;
}

template <int MODE, int REC, int RARE>
void run(const char* name, uint8_t* pool, uint32_t lanes, uint32_t steps, uint32_t* out)
{
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    chain<MODE, REC, RARE><<<lanes / 256, 256>>>(pool, 40, out);
    hipEventRecord(a);
    chain<MODE, REC, RARE><<<lanes / 256, 256>>>(pool, steps, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    printf("%-28s rec=%3d rare=1/%-3d table=%7.1f MB : %7.1f ns/step\n", name, REC, RARE,
           static_cast<double>(lanes) * 256 * REC / 1e6, ms * 1e6 / steps);
}

int main()
{
    const uint32_t lanes = 65536, steps = 1200;
    uint8_t* pool; uint32_t* out;
    if (hipMalloc(&pool, static_cast<size_t>(lanes) * 256 * 64) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(pool, 0, static_cast<size_t>(lanes) * 256 * 64);
    hipMalloc(&out, 4 * lanes);
    for (int r = 0; r < 2; ++r) {
        run<3, 64, 0>("rmw64 (current)", pool, lanes, steps, out);
        run<0, 64, 0>("blind 2B", pool, lanes, steps, out);
        run<1, 64, 0>("blind 4B", pool, lanes, steps, out);
        run<1, 32, 0>("blind 4B", pool, lanes, steps, out);
        run<1, 16, 0>("blind 4B", pool, lanes, steps, out);
        run<2, 64, 0>("seq 4B log", pool, lanes, steps, out);
        run<0, 64, 32>("blind 2B + rare load", pool, lanes, steps, out);
        run<0, 64, 16>("blind 2B + rare load", pool, lanes, steps, out);
        run<0, 64, 8>("blind 2B + rare load", pool, lanes, steps, out);
        run<2, 64, 32>("seq log + rare load", pool, lanes, steps, out);
        run<2, 64, 1>("seq log + load every step", pool, lanes, steps, out);
    }
    return 0;
}
