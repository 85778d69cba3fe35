// Microbenchmark (diagnostic, not product): what a second wavefront on the
// same SIMD costs or gives a wavefront running a serial chain (gfx950).
//
// One 256- or 512-thread workgroup per CU (forced by a 96 KB LDS request).
// Waves 0-3 ("main") run a dependent chain of mixed VALU work per lane, the
// way the decoder's step does; waves 4-7 ("helper", 512-thread case) run
//   mode 0: nothing (exit at once)
//   mode 1: an independent VALU stream (8 chains interleaved)
//   mode 2: the same chain as the main waves
//   mode 3: a polling loop over an LDS word with s_sleep 1
// Cycles per chain link of the main waves from s_memtime; also the SIMD id
// of every wave (HW_REG_HW_ID bits 5:4) to confirm waves w and w+4 share one.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t link(uint32_t x, uint32_t y)
{
    // a mix like the coder step: add, mul, shift by clz, compare-select, f32 convert
    x = x * y + 0x9E3779B9u;
    x ^= x >> (__builtin_clz(x | 1u) & 15);
    const float f = static_cast<float>(x) * 1.0000001f;
    x += static_cast<uint32_t>(f) >> 7;
    x = x > y ? x - y : x + 3u;
    return x;
}

__global__ __launch_bounds__(512) void kern(uint32_t* out, unsigned long long* cyc, uint32_t* simd, uint32_t n,
                                            uint32_t mode, uint32_t act)
{
    extern __shared__ uint32_t lds[];
    const uint32_t wave = threadIdx.x >> 6, l = threadIdx.x & 63;
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if (l == 0) simd[blockIdx.x * 8 + wave] = (hw >> 4) & 3;
    if (wave == 0 && l == 0) lds[0] = 0;
    __syncthreads();
    uint32_t x = threadIdx.x * 7919u + blockIdx.x, y = x * 3u + 1u;
    if (wave < 4) {
        if (l >= act) return;
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
        for (uint32_t i = 0; i < n; ++i) {
#pragma unroll
            for (int u = 0; u < 8; ++u) x = link(x, y);
        }
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        out[blockIdx.x * 512 + threadIdx.x] = x;
        if (l == 0) cyc[blockIdx.x * 4 + wave] = t1 - t0;
        if (l == 0) __hip_atomic_fetch_add(&lds[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return;
    }
    if (mode == 0) return;
    if (mode == 1) {
        uint32_t v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = x + k;
#pragma unroll 1
        for (uint32_t i = 0; i < n; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = link(v[k], y);
        }
        uint32_t s = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) s += v[k];
        out[blockIdx.x * 512 + threadIdx.x] = s;
        return;
    }
    if (mode == 2) {
#pragma unroll 1
        for (uint32_t i = 0; i < n; ++i) {
#pragma unroll
            for (int u = 0; u < 8; ++u) x = link(x, y);
        }
        out[blockIdx.x * 512 + threadIdx.x] = x;
        return;
    }
    // mode 3: poll until the 4 main waves are done
    uint32_t polls = 0;
    while (__hip_atomic_load(&lds[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 4) {
        __builtin_amdgcn_s_sleep(1);
        ++polls;
    }
    out[blockIdx.x * 512 + threadIdx.x] = polls;
}

int main()
{
    const uint32_t blocks = 256, n = 4000;
    uint32_t *out, *simd;
    unsigned long long *cyc, h[blocks * 4];
    uint32_t hs[blocks * 8];
    (void) hipMalloc(&out, blocks * 512 * 4);
    (void) hipMalloc(&simd, blocks * 8 * 4);
    (void) hipMalloc(&cyc, blocks * 4 * 8);
    const size_t lds = 96 * 1024;
    (void) hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    struct { const char* name; uint32_t threads, mode, act; } cases[] = {
        {"1 wave/SIMD, 64 lanes", 256, 0, 64},
        {"main + idle helper (exits)", 512, 0, 64},
        {"main + independent-VALU helper", 512, 1, 64},
        {"main + same-chain helper", 512, 2, 64},
        {"main + polling helper (s_sleep 1)", 512, 3, 64},
        {"1 wave/SIMD, 32 lanes", 256, 0, 32},
        {"main 32 lanes + same-chain helper", 512, 2, 32},
    };
    for (auto& c : cases) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(c.threads), lds, 0, out, cyc, simd, 10u, c.mode, c.act);
        hipEvent_t e0, e1;
        (void) hipEventCreate(&e0); (void) hipEventCreate(&e1);
        (void) hipEventRecord(e0, 0);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(c.threads), lds, 0, out, cyc, simd, n, c.mode, c.act);
        (void) hipEventRecord(e1, 0);
        (void) hipDeviceSynchronize();
        float ms = 0;
        (void) hipEventElapsedTime(&ms, e0, e1);
        (void) hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
        (void) hipMemcpy(hs, simd, sizeof hs, hipMemcpyDeviceToHost);
        double s = 0;
        for (uint32_t i = 0; i < blocks * 4; ++i) s += h[i];
        uint32_t same = 0;
        for (uint32_t b = 0; b < blocks; ++b)
            for (uint32_t w = 0; w < 4; ++w) same += hs[b * 8 + w] == hs[b * 8 + w + 4];
        printf("%-36s %7.2f cycles/link  %8.3f ms  (waves w, w+4 on one SIMD: %u/%u)\n", c.name,
               s / (blocks * 4) / (8.0 * n), ms, c.threads == 512 ? same : 0, blocks * 4);
    }
    return 0;
}
