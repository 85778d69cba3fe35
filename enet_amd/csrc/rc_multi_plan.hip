// rc_multi_plan.hip -- the split of a device-pointer batch over several GPUs
// (rc_multi.c), computed on the device that holds the batch, so that the host
// reads back 5 * parts + 1 words instead of every packet's offsets and lengths.
//
// plan[0 .. parts]: first[k], the smallest packet index whose prefix sum of
//   in_len reaches k / parts of the total (enet_rc_multi_split's rule; first[0]
//   = 0, first[parts] = n);
// plan[parts + 1 + 4k ..]: part k's lowest in_off, highest in_off + in_len,
//   lowest out_off, highest out_off + out_cap (UINT64_MAX, 0, UINT64_MAX, 0
//   for an empty part) -- the byte ranges copied to the part's device.
// enet_rc_multi_plan (rc_multi.c) is the host restatement the tests hold it to.
//
// Four launches: segment sums (1024 packets per segment), one block scanning
// them, one block per split point (the segment that crosses k / parts of the
// total, then the packet inside it), the extents (each segment's packets
// min / max-reduced per part in LDS, one global atomic per part touched).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rc_abi_internal.h"

namespace {
constexpr uint32_t kSeg = 1024;       // packets per segment
constexpr uint32_t kT = 256;

__device__ uint64_t block_sum64(uint64_t* s, uint64_t v)
{
    const uint32_t t = threadIdx.x;
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    if ((t & 63) == 0) s[t >> 6] = v;
    __syncthreads();
    const uint64_t r = s[0] + s[1] + s[2] + s[3];
    __syncthreads();
    return r;
}

// exclusive scan of v over the block (Hillis-Steele in LDS)
__device__ uint64_t block_excl64(uint64_t* s, uint64_t v, uint64_t& total)
{
    const uint32_t t = threadIdx.x;
    s[t] = v;
    __syncthreads();
    for (uint32_t d = 1; d < kT; d <<= 1) {
        const uint64_t x = t >= d ? s[t - d] : 0u;
        __syncthreads();
        s[t] += x;
        __syncthreads();
    }
    total = s[kT - 1];
    const uint64_t incl = s[t];
    __syncthreads();
    return incl - v;
}
}  // namespace

extern "C" __global__ __launch_bounds__(kT) void rc_plan_sums(const uint32_t* len, uint64_t n, uint64_t* bsum)
{
    __shared__ uint64_t s[4];
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kSeg;
    uint64_t v = 0;
    for (uint32_t k = 0; k < kSeg / kT; ++k) {
        const uint64_t i = base + k * kT + threadIdx.x;
        v += i < n ? len[i] : 0u;
    }
    v = block_sum64(s, v);
    if (threadIdx.x == 0) bsum[blockIdx.x] = v;
}

// bsum[0 .. nb) -> exclusive prefix sums in place, bsum[nb] = the total
extern "C" __global__ __launch_bounds__(kT) void rc_plan_scan(uint64_t* bsum, uint32_t nb)
{
    __shared__ uint64_t s[kT];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nb; b0 += kT) {
        const uint32_t b = b0 + threadIdx.x;
        uint64_t total;
        const uint64_t ex = block_excl64(s, b < nb ? bsum[b] : 0u, total);
        const uint64_t c = carry;
        __syncthreads();
        if (b < nb) bsum[b] = c + ex;
        if (threadIdx.x == 0) carry = c + total;
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[nb] = carry;
}

// block k: first[k]; also part k's extents set to empty
extern "C" __global__ __launch_bounds__(kT)
void rc_plan_first(const uint32_t* len, uint64_t n, const uint64_t* bsum, uint32_t nb, uint32_t parts, uint64_t* plan)
{
    __shared__ uint64_t s[kT];
    __shared__ uint32_t seg;
    const uint32_t k = blockIdx.x, t = threadIdx.x;
    uint64_t* ext = plan + parts + 1;
    if (t < 4) ext[4 * k + t] = (t & 1) ? 0u : ~0ull;
    if (k == 0) {
        if (t == 0) { plan[0] = 0; plan[parts] = n; }
        return;
    }
    const uint64_t total = bsum[nb];
    if (total == 0) {                 // (no packet has a byte: every split point is 0)
        if (t == 0) plan[k] = 0;
        return;
    }
    const uint64_t goal = total * k;  // first[k]: smallest i with prefix(i) * parts >= goal
    // the segment whose packets carry the prefix across goal / parts
    for (uint32_t b = t; b < nb; b += kT)
        if (bsum[b] * parts < goal && bsum[b + 1] * parts >= goal) seg = b;
    __syncthreads();
    const uint64_t base = static_cast<uint64_t>(seg) * kSeg + 4 * t;
    uint32_t l[4];
    uint64_t v = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        l[j] = base + j < n ? len[base + j] : 0u;
        v += l[j];
    }
    uint64_t tot;
    uint64_t e = bsum[seg] + block_excl64(s, v, tot);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        if (l[j] && e * parts < goal && (e + l[j]) * parts >= goal) plan[k] = base + j + 1;
        e += l[j];
    }
}

// block s: the extents of segment s's packets, per part
extern "C" __global__ __launch_bounds__(kT)
void rc_plan_extents(const uint32_t* in_len, const uint64_t* in_off, const uint64_t* out_off,
                     const uint32_t* out_cap, uint64_t n, uint32_t parts, uint64_t* plan)
{
    __shared__ uint64_t first[65];
    __shared__ unsigned long long ext[64 * 4];
    const uint32_t t = threadIdx.x;
    if (t <= parts) first[t] = plan[t];
    for (uint32_t j = t; j < 4 * parts; j += kT) ext[j] = (j & 1) ? 0ull : ~0ull;
    __syncthreads();
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kSeg;
    for (uint32_t r = 0; r < kSeg / kT; ++r) {
        const uint64_t i = base + r * kT + t;
        const bool ok = i < n;
        // the part holding packet i: the last k with first[k] <= i (parts may be empty)
        uint32_t lo = 0, hi = parts - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (first[mid] <= i) lo = mid; else hi = mid - 1;
        }
        uint64_t a = ok ? in_off[i] : ~0ull, b = ok ? in_off[i] + in_len[i] : 0u;
        uint64_t c = ok ? out_off[i] : ~0ull, d = ok ? out_off[i] + out_cap[i] : 0u;
        const uint32_t p0 = __shfl(lo, 0);
        if (__all(!ok || lo == p0)) {          // the wavefront's packets in one part: reduce, one lane adds
            for (int w = 32; w >= 1; w >>= 1) {
                a = min(a, static_cast<uint64_t>(__shfl_xor(a, w)));
                b = max(b, static_cast<uint64_t>(__shfl_xor(b, w)));
                c = min(c, static_cast<uint64_t>(__shfl_xor(c, w)));
                d = max(d, static_cast<uint64_t>(__shfl_xor(d, w)));
            }
            if ((t & 63) == 0) {
                atomicMin(&ext[4 * p0], a); atomicMax(&ext[4 * p0 + 1], b);
                atomicMin(&ext[4 * p0 + 2], c); atomicMax(&ext[4 * p0 + 3], d);
            }
        } else if (ok) {
            atomicMin(&ext[4 * lo], a); atomicMax(&ext[4 * lo + 1], b);
            atomicMin(&ext[4 * lo + 2], c); atomicMax(&ext[4 * lo + 3], d);
        }
    }
    __syncthreads();
    unsigned long long* g = reinterpret_cast<unsigned long long*>(plan + parts + 1);
    for (uint32_t j = t; j < 4 * parts; j += kT) {
        const unsigned long long x = ext[j];
        if (j & 1) { if (x != 0ull) atomicMax(&g[j], x); }
        else if (x != ~0ull) atomicMin(&g[j], x);
    }
}

// rebased offsets of a part on its device: off[i] -= lo
extern "C" __global__ __launch_bounds__(kT) void rc_plan_rebase(uint64_t* a, uint64_t la, uint64_t* b, uint64_t lb,
                                                                 uint64_t cnt)
{
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * kT + threadIdx.x; i < cnt;
         i += static_cast<uint64_t>(gridDim.x) * kT) {
        a[i] -= la;
        b[i] -= lb;
    }
}

// ws: at least rc_hip_multi_plan_ws(n) words of device memory; plan: 5 parts + 1 words
extern "C" size_t rc_hip_multi_plan_ws(size_t n) { return (n + kSeg - 1) / kSeg + 1; }

extern "C" int rc_hip_multi_plan(const uint32_t* in_len, const uint64_t* in_off, const uint64_t* out_off,
                                 const uint32_t* out_cap, uint64_t n, uint32_t parts, uint64_t* ws, uint64_t* plan,
                                 void* stream)
{
    if (parts == 0 || parts > 64 || n == 0) return static_cast<int>(hipErrorInvalidValue);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint64_t nb = (n + kSeg - 1) / kSeg;
    if (nb > 0xFFFFFFFFull) return static_cast<int>(hipErrorInvalidValue);
    hipLaunchKernelGGL(rc_plan_sums, dim3(static_cast<uint32_t>(nb)), dim3(kT), 0, st, in_len, n, ws);
    hipLaunchKernelGGL(rc_plan_scan, dim3(1), dim3(kT), 0, st, ws, static_cast<uint32_t>(nb));
    hipLaunchKernelGGL(rc_plan_first, dim3(parts), dim3(kT), 0, st, in_len, n, ws, static_cast<uint32_t>(nb), parts,
                       plan);
    hipLaunchKernelGGL(rc_plan_extents, dim3(static_cast<uint32_t>(nb)), dim3(kT), 0, st, in_len, in_off, out_off,
                       out_cap, n, parts, plan);
    return static_cast<int>(hipGetLastError());
}

extern "C" int rc_hip_multi_rebase(uint64_t* a, uint64_t la, uint64_t* b, uint64_t lb, uint64_t cnt, void* stream)
{
    if (cnt == 0) return 0;
    const uint64_t g = (cnt + kT - 1) / kT;
    hipLaunchKernelGGL(rc_plan_rebase, dim3(static_cast<uint32_t>(g < 1024 ? g : 1024)), dim3(kT), 0,
                       static_cast<hipStream_t>(stream), a, la, b, lb, cnt);
    return static_cast<int>(hipGetLastError());
}
