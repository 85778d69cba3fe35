// rc_route.hip -- the lane-path launcher: length binning of ragged batches,
// then the fast kernels (two-pass encoder rc_enc2.hip, record-light decoder
// rc_dec6.hip) and the v3 lane kernels (rc_lane3.hip) for what they leave.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rc_abi_internal.h"

// ---------------------------------------------------------- ragged batches
// The 64 packets of a wavefront advance in lock-step, so a wavefront lasts
// as long as its longest packet.  For batches of mixed lengths (config C4)
// the packets are first binned by length (16-B bins, longest first) and the
// lane kernels walk that order.  Order inside a bin is arbitrary; it only
// affects scheduling, never results.
__device__ __forceinline__ uint32_t len_bin(uint32_t len)
{
    const uint32_t b = len >> 4;
    return RC_LEN_BINS - 1 - (b < RC_LEN_BINS - 1 ? b : RC_LEN_BINS - 1);
}

constexpr uint32_t kBinChunk = 1024;     // packets per binning workgroup (4 per thread: 64 workgroups for 64 Ki packets)

// Wave-aggregated LDS histogram of one element per lane: lanes that share a
// bin are served by one LDS atomic (uniform batches take a single pass).
// Returns the element's rank among the workgroup's elements of its bin.
__device__ __forceinline__ uint32_t bin_rank(uint32_t* hist, uint32_t bin, bool valid)
{
    uint64_t rem = __ballot(valid);
    const uint64_t below = (1ull << (threadIdx.x & 63)) - 1;
    uint32_t rank = 0;
    while (rem) {
        const int leader = __ffsll(static_cast<unsigned long long>(rem)) - 1;
        const uint32_t lb = __shfl(bin, leader);
        const bool mine = valid && bin == lb;
        const uint64_t peers = __ballot(mine);
        uint32_t base = 0;
        if ((threadIdx.x & 63) == static_cast<uint32_t>(leader))
            base = atomicAdd(&hist[lb], static_cast<uint32_t>(__popcll(peers)));
        base = __shfl(base, leader);
        if (mine) rank = base + static_cast<uint32_t>(__popcll(peers & below));
        rem &= ~peers;
    }
    return rank;
}

// The histogram, then -- in the workgroup that finishes last (its ticket in
// bins[RC_LEN_TICKET], cleared with the counters by launch()) -- the exclusive
// prefix over the bins; bins[RC_LEN_BINS] = 1 when every packet falls in one
// bin (uniform lengths: the lane kernels then keep batch order).
extern "C" __global__ __launch_bounds__(RC_LEN_BINS) void rc_len_hist(const uint32_t* len, uint32_t n, uint32_t* bins)
{
    __shared__ uint32_t h[RC_LEN_BINS];
    __shared__ uint32_t last;
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kBinChunk;
    for (uint32_t k = 0; k < kBinChunk / 256; ++k) {
        const uint32_t i = base + k * 256 + threadIdx.x;
        (void) bin_rank(h, i < n ? len_bin(len[i]) : 0u, i < n);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&bins[threadIdx.x], h[threadIdx.x]);
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(&bins[RC_LEN_TICKET], 1u) == gridDim.x - 1 ? 1u : 0u;
    __syncthreads();
    if (!last) return;
    // every workgroup's counts are in: the scan (atomic reads: device-coherent)
    const uint32_t t = threadIdx.x;
    const uint32_t mine = atomicAdd(&bins[t], 0u);
    h[t] = mine;
    const int used = __syncthreads_count(mine != 0);
    for (uint32_t d = 1; d < RC_LEN_BINS; d <<= 1) {
        const uint32_t x = t >= d ? h[t - d] : 0u;
        __syncthreads();
        h[t] += x;
        __syncthreads();
    }
    bins[t] = h[t] - mine;               // exclusive prefix = first slot of the bin
    if (t == 0) bins[RC_LEN_BINS] = used <= 1 ? 1u : 0u;
}

extern "C" __global__ __launch_bounds__(256)
void rc_len_scatter(const uint32_t* len, uint32_t n, uint32_t* bins, uint32_t* order)
{
    if (bins[RC_LEN_BINS]) return;       // uniform: identity order
    __shared__ uint32_t h[RC_LEN_BINS];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kBinChunk;
    uint32_t rank[kBinChunk / 256], bin[kBinChunk / 256];
#pragma unroll
    for (uint32_t k = 0; k < kBinChunk / 256; ++k) {
        const uint32_t i = base + k * 256 + threadIdx.x;
        bin[k] = i < n ? len_bin(len[i]) : 0u;
        rank[k] = bin_rank(h, bin[k], i < n);
    }
    __syncthreads();
    const uint32_t c = h[threadIdx.x];
    if (c) h[threadIdx.x] = atomicAdd(&bins[threadIdx.x], c);   // this workgroup's slots in the bin
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kBinChunk / 256; ++k) {
        const uint32_t i = base + k * 256 + threadIdx.x;
        if (i < n) order[h[bin[k]] + rank[k]] = i;
    }
}

extern "C" int rc_hip_lane3_launch(int decompress, const rc_batch_dev* b, const rc_workspace_dev* ws,
                                   uint32_t blocks, void* stream);   // rc_lane3.hip
extern "C" int rc_hip_wave_tail_launch(int decompress, const rc_batch_dev* b, const rc_workspace_dev* ws,
                                       void* stream);                // rc_kernels.hip

extern "C" int rc_hip_lane_launch(int decompress, const rc_batch_dev* b, const rc_workspace_dev* ws,
                                  void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint32_t act = ws->lane_active;
    if (act != 64 && act != 32 && act != 16) return static_cast<int>(hipErrorInvalidValue);
    const uint32_t per_block = 4 * act;
    uint32_t blocks = (b->n + per_block - 1) / per_block;
    const uint32_t maxb = ws->lane_slots / per_block;
    if (blocks > maxb) blocks = maxb;
    if (blocks == 0) return static_cast<int>(hipErrorInvalidValue);
    rc_workspace_dev w = *ws;
    w.order = nullptr;
    if (b->n >= 1024 && ws->order && ws->bins) {        // bin packets by length (ragged batches)
        // (the bins were cleared with the counters by launch(), rc_kernels.hip)
        const uint32_t g = (b->n + kBinChunk - 1) / kBinChunk;
        hipLaunchKernelGGL(rc_len_hist, dim3(g), dim3(RC_LEN_BINS), 0, st, b->in_len, b->n, ws->bins);
        hipLaunchKernelGGL(rc_len_scatter, dim3(g), dim3(256), 0, st, b->in_len, b->n, ws->bins, ws->order);
        w.order = ws->order;
    }
    if (!decompress && ws->enc2_stream) {
        // the two-pass encoder takes what it can (rc_enc2.hip); the lanes run
        // only the packets it lists
        const int rc = rc_hip_enc2_launch(b, &w, stream);
        if (rc != 0) return rc;
        w.sub_list = ws->enc2_list;
        w.sub_count = ws->counters + 3;
    }
    if (decompress && ws->fast_dec && act == 64) {
        // the fast decoder takes what it can (rc_dec6.hip); the lanes decode
        // only the packets it lists
        const int rc = rc_hip_dec6_launch(b, &w, blocks, stream);
        if (rc != 0) return rc;
        w.sub_list = ws->enc2_list;
        w.sub_count = ws->counters + 3;
        // a small batch: what the decoder leaves goes to the wave kernel
        // (its model in LDS: faster than a lane's for a few packets)
        if (ws->wave_tail) return rc_hip_wave_tail_launch(1, b, &w, stream);
    }
    return rc_hip_lane3_launch(decompress, b, &w, blocks, stream);
}
