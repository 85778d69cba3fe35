// Microbenchmark (diagnostic, not product): dependent-chain latency of the
// coder's arithmetic on gfx950, one wavefront per SIMD (1024 wavefronts).
// Each chain feeds its result back as the next operand; cycles per link from
// s_memtime around the loop.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#include "../../enet_amd/csrc/rc_udiv.h"

template <int K>
__global__ __launch_bounds__(64) void chain(uint32_t* out, unsigned long long* cyc, uint32_t n, uint32_t seed)
{
    uint32_t x = seed + threadIdx.x * 7919u + blockIdx.x, y = x * 3u + 1u;
    const uint32_t b = 100u + (threadIdx.x & 31) * 997u;
    const float rb = rcp16(b);
    const double rbd = rcp64(b);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (uint32_t i = 0; i < n; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (K == 0) x = x + y;                                   // v_add_u32
            if (K == 1) x = x * y;                                   // v_mul_lo_u32
            if (K == 2) x = static_cast<uint32_t>(static_cast<uint64_t>(x) * y + y);  // mad_u64
            if (K == 3) x = (udiv16r(x | 0x80000000u, b, rb)) ^ y;   // the coder's division now
            if (K == 4) x = (udiv16d(x | 0x80000000u, b, rbd)) ^ y;     // f64 quotient
            if (K == 5) x = __float_as_uint(__builtin_amdgcn_rcpf(__uint_as_float(x)));
            if (K == 6) x = static_cast<uint32_t>(static_cast<double>(x) * 0.75);   // cvt + mul f64 + cvt
            if (K == 7) { const uint32_t l = x + y; x = (x ^ l) == 0 ? x : (x << (8 * (__builtin_clz(x ^ l) >> 3))); }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
void run(const char* name, uint32_t* out, unsigned long long* cyc, unsigned long long* h)
{
    const uint32_t n = 2000, blocks = 1024;
    chain<K><<<blocks, 64>>>(out, cyc, 10, 1);
    chain<K><<<blocks, 64>>>(out, cyc, n, 2);
    (void) hipMemcpy(h, cyc, 8 * blocks, hipMemcpyDeviceToHost);
    double s = 0;
    for (uint32_t i = 0; i < blocks; ++i) s += h[i];
    printf("%-34s %7.1f cycles per link\n", name, s / blocks / (8.0 * n));
}

// exactness of udiv16d against integer division: per divisor b, spread
// dividends, the nearest multiples of b and their neighbours, and a = 2^32-1
__global__ void check(uint32_t* bad, uint32_t b0)
{
    const uint32_t b = b0 + blockIdx.y;
    if (b == 0 || b > 65535) return;
    const double rbd = rcp64(b);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t nb = 0;
    for (uint32_t j = 0; j < 16; ++j) {
        const uint32_t a = t * 262139u + j * 16777259u;
        const uint32_t m = (a / b) * b;
        const uint32_t c[5] = {a, m, m - 1, m + b - 1, 0xFFFFFFFFu - t};
        for (int k = 0; k < 5; ++k) nb += udiv16d(c[k], b, rbd) != c[k] / b;
    }
    if (nb) atomicAdd(bad, nb);
}

int main()
{
    uint32_t* out; unsigned long long *cyc, h[1024];
    (void) hipMalloc(&out, 4 * 65536); (void) hipMalloc(&cyc, 8 * 1024);
    run<0>("v_add_u32", out, cyc, h);
    run<1>("v_mul_lo_u32", out, cyc, h);
    run<2>("mad_u64 low word", out, cyc, h);
    run<3>("udiv16r (f32, two steps) + xor", out, cyc, h);
    run<4>("udiv16d (f64 fma) + xor", out, cyc, h);
    run<5>("v_rcp_f32", out, cyc, h);
    run<6>("cvt f64, mul f64, cvt u32", out, cyc, h);
    run<7>("settle shift (add,xor,clz,shl)", out, cyc, h);
    uint32_t* bad; (void) hipMalloc(&bad, 4); (void) hipMemset(bad, 0, 4);
    for (uint32_t b0 = 1; b0 <= 65535; b0 += 4096) check<<<dim3(64, 4096), 256>>>(bad, b0);   // 16384 threads x 80 checks per b
    uint32_t hb = 0; (void) hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("udiv16d mismatches: %u\n", hb);
    return 0;
}
