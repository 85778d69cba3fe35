// Microbenchmark (diagnostic, not product): dependent random record
// read-modify-write chains, one per lane, the access pattern of the lane
// kernels' order-1 table.  Reports ns per step per lane and achieved rates.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

template <int REC, bool WRITE>
__global__ __launch_bounds__(256) void chain(uint8_t* pool, uint32_t region, uint32_t nrec, uint32_t steps, uint32_t* out)
{
    const uint32_t lane = blockIdx.x * 256 + threadIdx.x;
    uint8_t* reg = pool + (size_t) lane * region;
    uint32_t x = lane * 2654435761u + 12345u, acc = 0;
    for (uint32_t i = 0; i < steps; ++i) {
        x = x * 1664525u + 1013904223u;
        const uint32_t r = (x >> 8) % nrec;
        uint4* p = reinterpret_cast<uint4*>(reg + (size_t) r * REC);
        uint4 v[REC / 16];
#pragma unroll
        for (int k = 0; k < REC / 16; ++k) v[k] = p[k];
#pragma unroll
        for (int k = 0; k < REC / 16; ++k) acc += v[k].x ^ v[k].w;
        x ^= acc & 1;   // make the chain dependent on the data
        if (WRITE) {
#pragma unroll
            for (int k = 0; k < REC / 16; ++k) { v[k].x += 1; p[k] = v[k]; }
        }
    }
    out[lane] = acc;
}

// The encoder's pattern: addresses known ahead (not data-dependent), the
// record of step i+D loaded at step i, modified and written back when used.
template <int D>
__global__ __launch_bounds__(256) void ahead(uint8_t* pool, uint32_t region, uint32_t nrec, uint32_t steps, uint32_t* out)
{
    const uint32_t lane = blockIdx.x * 256 + threadIdx.x;
    uint8_t* reg = pool + (size_t) lane * region;
    uint32_t x = lane * 2654435761u + 12345u, acc = 0;
    uint32_t addr[D + 1];
    uint4 v[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        x = x * 1664525u + 1013904223u;
        addr[d] = (x >> 8) % nrec;
        const uint4* p = reinterpret_cast<const uint4*>(reg + (size_t) addr[d] * 64);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[d][k] = p[k];
    }
    for (uint32_t i = 0; i < steps; ++i) {
        x = x * 1664525u + 1013904223u;
        addr[D] = (x >> 8) % nrec;
        uint4 nv[4];
        const uint4* pn = reinterpret_cast<const uint4*>(reg + (size_t) addr[D] * 64);
#pragma unroll
        for (int k = 0; k < 4; ++k) nv[k] = pn[k];
        uint4* p = reinterpret_cast<uint4*>(reg + (size_t) addr[0] * 64);
#pragma unroll
        for (int k = 0; k < 4; ++k) { acc += v[0][k].x ^ v[0][k].w; v[0][k].x += 1; p[k] = v[0][k]; }
#pragma unroll
        for (int d = 0; d < D - 1; ++d) {
            addr[d] = addr[d + 1];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[d][k] = v[d + 1][k];
        }
        addr[D - 1] = addr[D];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[D - 1][k] = nv[k];
    }
    out[lane] = acc;
}

template <int D>
void run_ahead(uint8_t* pool, uint32_t lanes, uint32_t nrec, uint32_t* out)
{
    const uint32_t region = nrec * 64, steps = 400;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    ahead<D><<<lanes / 256, 256>>>(pool, region, nrec, 50, out);
    hipEventRecord(a);
    ahead<D><<<lanes / 256, 256>>>(pool, region, nrec, steps, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const double per = ms * 1e6 / steps;
    const double acc = (double) lanes * steps / (ms * 1e-3);
    printf("ahead D=%d lanes=%6u table/lane=%6u B total=%7.1f MB : %7.1f ns/step  %6.2f G rec/s  %7.1f GB/s line traffic (128 B read + 64 B write)\n",
           D, lanes, region, (double) lanes * region / 1e6, per, acc / 1e9, acc * 192 / 1e9);
}

template <int REC, bool WRITE>
void run(uint8_t* pool, uint32_t lanes, uint32_t nrec, uint32_t* out)
{
    const uint32_t region = nrec * REC, steps = 400;
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    chain<REC, WRITE><<<lanes / 256, 256>>>(pool, region, nrec, 50, out);
    hipEventRecord(a);
    chain<REC, WRITE><<<lanes / 256, 256>>>(pool, region, nrec, steps, out);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const double per = ms * 1e6 / steps;
    const double acc = (double) lanes * steps / (ms * 1e-3);
    printf("rec=%3d write=%d lanes=%6u table/lane=%6u B total=%7.1f MB : %7.1f ns/step  %6.2f G rec/s  %7.1f GB/s (rec bytes%s)\n",
           REC, WRITE, lanes, region, (double) lanes * region / 1e6, per, acc / 1e9, acc * REC * (WRITE ? 2 : 1) / 1e9,
           WRITE ? " r+w" : "");
}

int main()
{
    uint8_t* pool; uint32_t* out;
    const size_t bytes = (size_t) 65536 * 16384 * 2;
    if (hipMalloc(&pool, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(pool, 0, bytes);
    hipMalloc(&out, 4 * 262144);
    if (getenv("MB_AHEAD")) {
        for (uint32_t lanes : {65536u, 131072u}) {
            run<64, true>(pool, lanes, 256, out);
            run_ahead<1>(pool, lanes, 256, out);
            run_ahead<2>(pool, lanes, 256, out);
            run_ahead<3>(pool, lanes, 256, out);
        }
        return 0;
    }
    for (uint32_t lanes : {65536u, 131072u}) {
        run<64, true>(pool, lanes, 256, out);
        run<64, false>(pool, lanes, 256, out);
        run<32, true>(pool, lanes, 256, out);
        run<32, false>(pool, lanes, 256, out);
        run<16, true>(pool, lanes, 256, out);
        run<16, false>(pool, lanes, 256, out);
        run<128, true>(pool, lanes, 256, out);
        run<64, true>(pool, lanes, 64, out);    // 4 KB table per lane (256 MB total)
        run<16, true>(pool, lanes, 128, out);   // 2 KB per lane
        run<64, true>(pool, lanes, 8, out);     // 512 B per lane (L2-sized)
    }
    return 0;
}
