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

// LDS histogram of one element per lane; returns the element's rank among
// the workgroup's elements of its bin (any order inside a bin).  A
// wavefront whose elements share one bin (uniform batches) takes a single
// LDS atomic; a ragged one takes one per lane (the LDS serialises the lanes
// of one address in hardware: a loop over the wavefront's distinct bins --
// ~50 for C4's lengths -- cost 81 + 57 us per binning of 1 Mi packets).
__device__ __forceinline__ uint32_t bin_rank(uint32_t* hist, uint32_t bin, bool valid)
{
    const uint64_t vm = __ballot(valid);
    if (vm == 0) return 0;
    const int leader = __ffsll(static_cast<unsigned long long>(vm)) - 1;
    const uint32_t lb = __shfl(bin, leader);
    if (__ballot(valid && bin != lb) == 0) {
        const uint64_t below = (1ull << (threadIdx.x & 63)) - 1;
        uint32_t base = 0;
        if ((threadIdx.x & 63) == static_cast<uint32_t>(leader))
            base = atomicAdd(&hist[lb], static_cast<uint32_t>(__popcll(vm)));
        base = __shfl(base, leader);
        return valid ? base + static_cast<uint32_t>(__popcll(vm & below)) : 0u;
    }
    return valid ? atomicAdd(&hist[bin], 1u) : 0u;
}

// The histogram: each workgroup's counts added into bins[0, RC_LEN_BINS)
// (cleared with the counters by launch()).  (Until round 5 the workgroup that
// finished last also turned the counts into bin starts: a ticket, a fence
// and a 256-entry scan behind every other workgroup, 9.6 us of a 14-us
// binning per call; rc_len_scatter now scans the counts itself.)
extern "C" __global__ __launch_bounds__(RC_LEN_BINS) void rc_len_hist(const uint32_t* len, uint32_t n, uint32_t* bins)
{
    __shared__ uint32_t h[RC_LEN_BINS];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kBinChunk;
    for (uint32_t k = 0; k < kBinChunk / 256; ++k) {
        const uint32_t i = base + k * 256 + threadIdx.x;
        (void) bin_rank(h, i < n ? len_bin(len[i]) : 0u, i < n);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&bins[threadIdx.x], h[threadIdx.x]);
}

// The packets in bin order: each workgroup scans the bin counts (exclusive
// prefix = the first slot of each bin), claims its slots in each bin from
// the fill counters bins[RC_LEN_FILL ..] and writes its packets there.  When
// every packet falls in one bin, workgroup 0 sets bins[RC_LEN_BINS] (uniform
// lengths: the lane kernels keep batch order) and nothing is written.
extern "C" __global__ __launch_bounds__(256)
void rc_len_scatter(const uint32_t* len, uint32_t n, uint32_t* bins, uint32_t* order)
{
    __shared__ uint32_t h[RC_LEN_BINS], pre[RC_LEN_BINS];
    const uint32_t t = threadIdx.x;
    const uint32_t cnt = bins[t];
    const int used = __syncthreads_count(cnt != 0);
    if (used <= 1) {
        if (blockIdx.x == 0 && t == 0) bins[RC_LEN_BINS] = 1u;
        return;
    }
    pre[t] = cnt;
    h[t] = 0;
    __syncthreads();
    for (uint32_t d = 1; d < RC_LEN_BINS; d <<= 1) {
        const uint32_t x = t >= d ? pre[t - d] : 0u;
        __syncthreads();
        pre[t] += x;
        __syncthreads();
    }
    const uint32_t first = pre[t] - cnt;             // exclusive prefix: the bin's first slot
    __syncthreads();
    const uint32_t base = blockIdx.x * kBinChunk;
    uint32_t rank[kBinChunk / 256], bin[kBinChunk / 256];
#pragma unroll
    for (uint32_t k = 0; k < kBinChunk / 256; ++k) {
        const uint32_t i = base + k * 256 + t;
        bin[k] = i < n ? len_bin(len[i]) : 0u;
        rank[k] = bin_rank(h, bin[k], i < n);
    }
    __syncthreads();
    const uint32_t c = h[t];
    if (c) h[t] = first + atomicAdd(&bins[RC_LEN_FILL + t], c);   // this workgroup's slots in the bin
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kBinChunk / 256; ++k) {
        const uint32_t i = base + k * 256 + t;
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
