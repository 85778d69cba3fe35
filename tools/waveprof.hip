// waveprof.hip -- phase timing of the wave compress kernel (rc_kernels.hip
// built with RC_WAVE_PROF): shader-clock cycles per input byte spent in the
// order-2 step, the order-1 step, the root + coding, and the advance, for
// one-packet launches (the per-datagram call shape).  Diagnostics only.
#define RC_WAVE_PROF 1
#include "../enet_amd/csrc/rc_kernels.hip"
#include <vector>
#include <cstdio>

extern "C" int rc_hip_lane_launch(int, const rc_batch_dev*, const rc_workspace_dev*, void*) { return -1; }

static uint64_t mix(uint64_t& s)
{
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main()
{
    const uint32_t n = 1200;
    for (int gen = 0; gen < 2; ++gen) {
        std::vector<uint8_t> h(n);
        uint64_t st = 0x454E4554ull + gen;
        for (uint32_t i = 0; i < n; ++i)
            h[i] = gen == 0 ? (uint8_t) mix(st) : (uint8_t) ((i % 24) < 8 ? mix(st) % 4 : (i % 24 == 11 ? 100 : 0));
        uint8_t *din, *dout; uint64_t *off; uint32_t *len, *cap, *olen, *fl, *cnt;
        hipMalloc(&din, n); hipMalloc(&dout, 2 * n + 64);
        hipMalloc(&off, 8); hipMalloc(&len, 4); hipMalloc(&cap, 4); hipMalloc(&olen, 4);
        hipMalloc(&fl, 64); hipMalloc(&cnt, 16);
        hipMemcpy(din, h.data(), n, hipMemcpyHostToDevice);
        hipMemset(off, 0, 8); hipMemset(cnt, 0, 16);
        const uint32_t c = 2 * n + 64;
        hipMemcpy(len, &n, 4, hipMemcpyHostToDevice);
        hipMemcpy(cap, &c, 4, hipMemcpyHostToDevice);
        rc_batch_dev b = { din, off, len, dout, off, cap, olen, 1, n };
        rc_workspace_dev ws = {};
        ws.flag_list = fl; ws.counters = cnt; ws.n_cap = 1;
        const uint32_t stage = stage_bytes_for(n), lds = lds_bytes_for(n);
        for (int rep = 0; rep < 2; ++rep) {
            unsigned long long z[8] = {};
            hipMemcpyToSymbol(HIP_SYMBOL(g_wave_prof), z, sizeof z);
            hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(rc_compress_wave, dim3(1), dim3(64), lds, 0, b, ws, stage, lds);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms = 0; hipEventElapsedTime(&ms, e0, e1);
            hipMemcpyFromSymbol(z, HIP_SYMBOL(g_wave_prof), sizeof z);
            uint32_t ol = 0; hipMemcpy(&ol, olen, 4, hipMemcpyDeviceToHost);
            const double per = 1.0 / (double) (z[4] ? z[4] : 1);
            if (rep == 1)
                printf("{\"gen\": \"%s\", \"bytes\": %u, \"out\": %u, \"kernel_us\": %.1f, \"cycles_per_byte\": "
                       "{\"order2\": %.0f, \"order1\": %.0f, \"root_code\": %.0f, \"advance\": %.0f}}\n",
                       gen ? "game" : "random", n, ol, ms * 1e3, z[0] * per, z[1] * per, z[2] * per, z[3] * per);
        }
    }
    return 0;
}
