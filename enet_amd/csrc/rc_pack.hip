// rc_pack.hip -- pack a batch's outputs back to back before the D2H copy of
// the host-pointer calls: out_len[i] bytes of packet i (at out_off[i] in a
// slot of out_cap[i] bytes, e.g. 2N + 64) go to packed[sum of out_len[<i]].
// PCIe then carries the compressed bytes, not the slot capacities.
//
// Three launches: per-block sums of out_len (1024 packets per block), one
// block scanning those sums (also writing the total), and per block a local
// scan plus the copies (one wavefront per packet, 4-B words where both ends
// are aligned, bytes otherwise).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rc_abi_internal.h"

namespace {
constexpr uint32_t kPer = 1024;     // packets per block
constexpr uint32_t kThreads = 256;

__device__ uint32_t block_excl_scan(uint32_t* s, uint32_t v, uint32_t& total)
{
    // 256 threads, Hillis-Steele in LDS
    const uint32_t t = threadIdx.x;
    s[t] = v;
    __syncthreads();
    for (uint32_t d = 1; d < kThreads; d <<= 1) {
        const uint32_t x = t >= d ? s[t - d] : 0u;
        __syncthreads();
        s[t] += x;
        __syncthreads();
    }
    total = s[kThreads - 1];
    const uint32_t incl = s[t];
    __syncthreads();
    return incl - v;
}
}  // namespace

extern "C" __global__ __launch_bounds__(kThreads) void rc_pack_sums(const uint32_t* len, uint32_t n, uint64_t* bsum)
{
    __shared__ uint32_t s[kThreads];
    const uint32_t base = blockIdx.x * kPer;
    uint32_t v = 0;
    for (uint32_t k = 0; k < kPer / kThreads; ++k) {
        const uint32_t i = base + k * kThreads + threadIdx.x;
        v += i < n ? len[i] : 0u;
    }
    uint32_t total;
    block_excl_scan(s, v, total);
    if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// one block: exclusive scan of the block sums in place; bsum[nb] = total
extern "C" __global__ __launch_bounds__(kThreads) void rc_pack_scan(uint64_t* bsum, uint32_t nb)
{
    __shared__ uint64_t carry;
    __shared__ uint32_t s[kThreads];
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nb; b0 += kThreads) {
        const uint32_t b = b0 + threadIdx.x;
        const uint64_t v = b < nb ? bsum[b] : 0u;
        uint32_t total;
        const uint32_t ex = block_excl_scan(s, static_cast<uint32_t>(v), total);   // block sums < 2^32
        const uint64_t c = carry;
        __syncthreads();
        if (b < nb) bsum[b] = c + ex;
        if (threadIdx.x == 0) carry = c + total;
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[nb] = carry;
}

// UNPACK: the reverse, packed[sum of len[<i]] -> out[out_off[i]] (rc_multi.c:
// results of another device, gathered back to back, into the root's slots)
template <bool UNPACK>
__device__ void pack_copy(uint8_t* out, const uint64_t* out_off, const uint32_t* len, uint32_t n,
                          const uint64_t* bsum, uint8_t* packed)
{
    __shared__ uint32_t s[kThreads];
    __shared__ uint32_t off[kPer];
    const uint32_t base = blockIdx.x * kPer;
    // local exclusive offsets: each thread owns 4 consecutive packets
    uint32_t l4[4], v = 0;
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t i = base + 4 * threadIdx.x + k;
        l4[k] = i < n ? len[i] : 0u;
        v += l4[k];
    }
    uint32_t total;
    uint32_t ex = block_excl_scan(s, v, total);
    for (uint32_t k = 0; k < 4; ++k) { off[4 * threadIdx.x + k] = ex; ex += l4[k]; }
    __syncthreads();
    const uint64_t b0 = bsum[blockIdx.x];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t k = wave; k < kPer; k += kThreads / 64) {
        const uint32_t i = base + k;
        if (i >= n) break;
        const uint32_t m = len[i];
        const uint8_t* src = UNPACK ? packed + b0 + off[k] : out + out_off[i];
        uint8_t* dst = UNPACK ? out + out_off[i] : packed + b0 + off[k];
        if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 3) == 0) {
            const uint32_t w = m >> 2;
            for (uint32_t j = lane; j < w; j += 64)
                reinterpret_cast<uint32_t*>(dst)[j] = reinterpret_cast<const uint32_t*>(src)[j];
            for (uint32_t j = 4 * w + lane; j < m; j += 64) dst[j] = src[j];
        } else {
            for (uint32_t j = lane; j < m; j += 64) dst[j] = src[j];
        }
    }
}

extern "C" __global__ __launch_bounds__(kThreads)
void rc_pack_copy(const uint8_t* out, const uint64_t* out_off, const uint32_t* len, uint32_t n,
                  const uint64_t* bsum, uint8_t* packed)
{
    pack_copy<false>(const_cast<uint8_t*>(out), out_off, len, n, bsum, packed);
}

extern "C" __global__ __launch_bounds__(kThreads)
void rc_unpack_copy(uint8_t* out, const uint64_t* out_off, const uint32_t* len, uint32_t n,
                    const uint64_t* bsum, const uint8_t* packed)
{
    pack_copy<true>(out, out_off, len, n, bsum, const_cast<uint8_t*>(packed));
}

extern "C" int rc_hip_unpack(const uint8_t* packed, uint8_t* out, const uint64_t* out_off, const uint32_t* out_len,
                             uint32_t n, uint64_t* bsum, void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (n == 0) return 0;
    const uint32_t nb = (n + kPer - 1) / kPer;
    hipLaunchKernelGGL(rc_pack_sums, dim3(nb), dim3(kThreads), 0, st, out_len, n, bsum);
    hipLaunchKernelGGL(rc_pack_scan, dim3(1), dim3(kThreads), 0, st, bsum, nb);
    hipLaunchKernelGGL(rc_unpack_copy, dim3(nb), dim3(kThreads), 0, st, out, out_off, out_len, n, bsum, packed);
    return static_cast<int>(hipGetLastError());
}

extern "C" int rc_hip_pack(const uint8_t* out, const uint64_t* out_off, const uint32_t* out_len, uint32_t n,
                           uint64_t* bsum, uint8_t* packed, void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (n == 0) return 0;
    const uint32_t nb = (n + kPer - 1) / kPer;
    hipLaunchKernelGGL(rc_pack_sums, dim3(nb), dim3(kThreads), 0, st, out_len, n, bsum);
    hipLaunchKernelGGL(rc_pack_scan, dim3(1), dim3(kThreads), 0, st, bsum, nb);
    hipLaunchKernelGGL(rc_pack_copy, dim3(nb), dim3(kThreads), 0, st, out, out_off, out_len, n, bsum, packed);
    return static_cast<int>(hipGetLastError());
}
