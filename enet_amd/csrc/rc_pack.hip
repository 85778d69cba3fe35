// rc_pack.hip -- pack a batch's outputs back to back before the D2H copy of
// the host-pointer calls: out_len[i] bytes of packet i (at out_off[i] in a
// slot of out_cap[i] bytes, e.g. 2N + 64) go to packed[sum of out_len[<i]].
// PCIe then carries the compressed bytes, not the slot capacities.
//
// Three launches: per-segment sums of out_len (1024 packets per segment), one
// block scanning those sums (also writing the total), and the copies: 16
// workgroups per segment, one wavefront per packet, aligned dword stores
// assembled from the source with alignbyte (copy_bytes).

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

// One packet's bytes [src, src + m) -> [dst, dst + m) by one wavefront, any
// alignment on either side: every destination dword inside the range is one
// aligned store assembled from two aligned source dwords (alignbyte); the
// bytes of the range's first and last partial dwords are stored singly (a
// neighbouring packet owns the rest of those dwords).
__device__ __forceinline__ void copy_bytes(const uint8_t* src, uint8_t* dst, uint32_t m, uint32_t lane)
{
    if (m == 0) return;
    const uintptr_t d0 = reinterpret_cast<uintptr_t>(dst), d1 = d0 + m;
    const uintptr_t b0 = (d0 + 3) & ~static_cast<uintptr_t>(3), b1 = d1 & ~static_cast<uintptr_t>(3);
    if (b0 >= b1) {                                      // no whole dword inside
        if (lane < m) dst[lane] = src[lane];
        return;
    }
    const uint32_t head = static_cast<uint32_t>(b0 - d0), tail = static_cast<uint32_t>(d1 - b1);
    if (lane < head) dst[lane] = src[lane];
    if (lane < tail) dst[m - tail + lane] = src[m - tail + lane];
    const uintptr_t s0 = reinterpret_cast<uintptr_t>(src) + head;   // source of the first whole dword
    const uint32_t sh = static_cast<uint32_t>(s0 & 3);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(s0 & ~static_cast<uintptr_t>(3));
    uint32_t* dw = reinterpret_cast<uint32_t*>(b0);
    const uint32_t nw = static_cast<uint32_t>((b1 - b0) >> 2);
    for (uint32_t k = lane; k < nw; k += 64) {
        const uint32_t lo = sw[k];
        const uint32_t hi = sh ? sw[k + 1] : 0u;          // (only read when the source is misaligned)
        dw[k] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
    }
}

constexpr uint32_t kPerBlock = 64;          // packets per copy workgroup (16 per wavefront)

// UNPACK: the reverse, packed[sum of len[<i]] -> out[out_off[i]] (rc_multi.c:
// results of another device, gathered back to back, into the root's slots).
// Workgroup (segment s, part q) copies packets [1024 s + 64 q, +64): their
// offsets are the segment's base (bsum) plus the lengths before them.
template <bool UNPACK>
__device__ void pack_copy(uint8_t* out, const uint64_t* out_off, const uint32_t* len, uint32_t n,
                          const uint64_t* bsum, uint8_t* packed)
{
    __shared__ uint32_t s[kThreads];
    __shared__ uint32_t off[kPerBlock];
    const uint32_t seg = blockIdx.x / (kPer / kPerBlock), part = blockIdx.x % (kPer / kPerBlock);
    const uint32_t base = seg * kPer, first = base + part * kPerBlock;
    // lengths of the segment's packets before this part
    uint32_t v = 0;
    for (uint32_t i = base + threadIdx.x; i < first; i += kThreads) v += i < n ? len[i] : 0u;
    uint32_t before;
    block_excl_scan(s, v, before);
    // exclusive offsets of this part's packets
    const uint32_t t = threadIdx.x;
    const uint32_t mine = (t < kPerBlock && first + t < n) ? len[first + t] : 0u;
    uint32_t total;
    const uint32_t ex = block_excl_scan(s, mine, total);
    if (t < kPerBlock) off[t] = ex;
    __syncthreads();
    const uint64_t b0 = bsum[seg] + before;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t k = wave; k < kPerBlock; k += kThreads / 64) {
        const uint32_t i = first + k;
        if (i >= n) break;
        uint8_t* pk = packed + b0 + off[k];
        uint8_t* sl = out + out_off[i];
        if (UNPACK) copy_bytes(pk, sl, len[i], lane);
        else copy_bytes(sl, pk, len[i], lane);
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
    hipLaunchKernelGGL(rc_unpack_copy, dim3(nb * (kPer / kPerBlock)), dim3(kThreads), 0, st, out, out_off, out_len, n,
                       bsum, packed);
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
    hipLaunchKernelGGL(rc_pack_copy, dim3(nb * (kPer / kPerBlock)), dim3(kThreads), 0, st, out, out_off, out_len, n,
                       bsum, packed);
    return static_cast<int>(hipGetLastError());
}

// Gather of a host batch's packets by the GPU over PCIe (rc_host.c: an input
// in gapped slots of a mapped, page-locked caller buffer): packet i's bytes
// [src + soff[i], +len[i]) -> dst + doff[i], where doff[i] has the source's
// alignment mod 16 and the 16-B granules around [doff[i], +len[i]) belong to
// packet i alone, so whole aligned 16-B chunks are copied (the bytes around
// the packet in its first and last granule come along; they are never read).
// Sixteen lanes per packet, four packets per wavefront.
extern "C" __global__ __launch_bounds__(kThreads)
void rc_gather16(const uint8_t* src, const uint64_t* soff, uint8_t* dst, const uint64_t* doff, const uint32_t* len,
                 uint32_t n)
{
    const uint32_t lane = threadIdx.x & 15;
    const uint32_t groups = gridDim.x * (kThreads / 16);
    for (uint32_t i = (blockIdx.x * kThreads + threadIdx.x) >> 4; i < n; i += groups) {
        const uint32_t m = len[i];
        if (m == 0) continue;
        const uintptr_t s0 = reinterpret_cast<uintptr_t>(src) + soff[i];
        const uintptr_t sa = s0 & ~static_cast<uintptr_t>(15), se = (s0 + m + 15) & ~static_cast<uintptr_t>(15);
        const uintptr_t da = (reinterpret_cast<uintptr_t>(dst) + doff[i]) & ~static_cast<uintptr_t>(15);
        const uint32_t nch = static_cast<uint32_t>((se - sa) >> 4);
        for (uint32_t c = lane; c < nch; c += 16)
            reinterpret_cast<uint4*>(da)[c] = reinterpret_cast<const uint4*>(sa)[c];
    }
}

extern "C" int rc_hip_gather16(const uint8_t* src, const uint64_t* soff, uint8_t* dst, const uint64_t* doff,
                               const uint32_t* len, uint32_t n, void* stream)
{
    if (n == 0) return 0;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    uint32_t blocks = (n + kThreads / 16 - 1) / (kThreads / 16);
    const uint32_t cap = static_cast<uint32_t>(cus) * 8;
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL(rc_gather16, dim3(blocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream), src, soff, dst,
                       doff, len, n);
    return static_cast<int>(hipGetLastError());
}

// Each packet's produced bytes from its device slot into the same offset of
// another buffer (rc_host.c: the results of a host batch written by the GPU
// straight into the caller's mapped, page-locked slots over PCIe), one
// wavefront per packet: no packing pass, no prefix sums.
extern "C" __global__ __launch_bounds__(kThreads)
void rc_slot_copy(const uint8_t* src, const uint64_t* off, const uint32_t* len, uint32_t n, uint8_t* dst)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t waves = gridDim.x * (kThreads / 64);
    for (uint32_t i = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6); i < n; i += waves)
        copy_bytes(src + off[i], dst + off[i], len[i], lane);
}

extern "C" int rc_hip_slot_copy(const uint8_t* src, const uint64_t* off, const uint32_t* len, uint32_t n,
                                uint8_t* dst, uint32_t max_wgs, void* stream)
{
    if (n == 0) return 0;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    uint32_t blocks = (n + kThreads / 64 - 1) / (kThreads / 64);
    // max_wgs: at most that many workgroups (0: 8 per CU) -- a copy beside
    // other kernels (a piece of a split host batch, run_host_split) leaves
    // their CUs' issue slots to them; PCIe, not the waves, bounds the copy
    const uint32_t cap = max_wgs ? max_wgs : static_cast<uint32_t>(cus) * 8;
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL(rc_slot_copy, dim3(blocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream), src, off, len,
                       n, dst);
    return static_cast<int>(hipGetLastError());
}
