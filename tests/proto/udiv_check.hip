// TEST ONLY: checks enet_amd/csrc/rc_udiv.h against integer division on the GPU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "rc_udiv.h"

__device__ uint64_t mix(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// per thread `iters` cases: random a, b of random bit widths, plus exact
// multiples q*b and q*b - 1 and a = 2^32 - 1; counts mismatches
extern "C" __global__ void udiv_check(uint64_t seed, uint32_t iters, unsigned long long* bad)
{
    const uint64_t t = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x;
    unsigned long long nbad = 0;
    for (uint32_t i = 0; i < iters; ++i) {
        const uint64_t x = mix(seed ^ (t * 0x100000001b3ull + i));
        const uint32_t bw = 1 + (uint32_t) (x & 31), aw = 1 + (uint32_t) ((x >> 5) & 31);
        uint32_t b = (uint32_t) (x >> 16) & (uint32_t) ((1ull << bw) - 1);
        if (b == 0) b = 1;
        const uint32_t a0 = (uint32_t) (x >> 32) & (uint32_t) ((1ull << aw) - 1);
        const uint32_t q = a0 / b;
        const uint32_t cases[4] = {a0, q * b, q * b ? q * b - 1 : 0u, 0xFFFFFFFFu};
        for (int c = 0; c < 4; ++c) nbad += udiv(cases[c], b) != cases[c] / b;
        // udiv16: divisors below 2^16 (context totals)
        const uint32_t b16 = (b & 0xFFFF) ? (b & 0xFFFF) : 1u;
        const uint32_t q16 = a0 / b16;
        const uint32_t c16[4] = {a0, q16 * b16, q16 * b16 ? q16 * b16 - 1 : 0u, 0xFFFFFFFFu};
        for (int c = 0; c < 4; ++c) nbad += udiv16(c16[c], b16) != c16[c] / b16;
        // udiv16d: the same divisors, the double-precision quotient
        const double r16 = rcp64(b16);
        for (int c = 0; c < 4; ++c) nbad += udiv16d(c16[c], b16, r16) != c16[c] / b16;
        nbad += udiv16d(q16 * b16 + b16 - 1 >= q16 * b16 ? q16 * b16 + b16 - 1 : 0xFFFFFFFFu, b16, r16) !=
                (q16 * b16 + b16 - 1 >= q16 * b16 ? q16 * b16 + b16 - 1 : 0xFFFFFFFFu) / b16;
        // udiv_lo16: any divisor, low 16 bits of the quotient
        for (int c = 0; c < 4; ++c) nbad += udiv_lo16(cases[c], b) != ((cases[c] / b) & 0xFFFF);
        // quotients just below 2^16 (a READ at the top of a context's range)
        const uint32_t bq = b > 65536 ? b >> 16 : (b ? b : 1u), qq = 65535u - (uint32_t) (x & 1023);
        const uint64_t aq = (uint64_t) qq * bq + (x >> 53) % bq;
        if (aq <= 0xFFFFFFFFull) nbad += udiv_lo16((uint32_t) aq, bq) != (((uint32_t) aq / bq) & 0xFFFF);
    }
    if (nbad) atomicAdd(bad, nbad);
}

extern "C" int udiv_run(uint64_t seed, uint32_t blocks, uint32_t iters, unsigned long long* out)
{
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 8) != hipSuccess) return -1;
    if (hipMemset(d, 0, 8) != hipSuccess) return -1;
    hipLaunchKernelGGL(udiv_check, dim3(blocks), dim3(256), 0, 0, seed, iters, d);
    if (hipMemcpy(out, d, 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    (void) hipFree(d);
    return 0;
}
