// rc_dgram.hip -- ENet datagram framing around the batched range coder
// (SURVEY.md §8f rows 3-4): whole wire datagrams in, whole datagrams out.
//
// Wire layout (protocol.h:48-53, protocol.c:1026-1033 / :1676-1718):
//   u16 big-endian peerID word: bits 0-11 peer, 12-13 session,
//       14 COMPRESSED, 15 SENT_TIME
//   u16 big-endian sentTime         (only with SENT_TIME)
//   u32 checksum                    (only when the host has a checksum callback)
//   commands                        (range-coded when COMPRESSED)
// headerSize = 2 or 4, + 4 with a checksum.
//
// Send (protocol.c:1686-1718): the commands (L bytes) are coded with
// outLimit = L; the compressed form is used iff 0 < C < L, which sets
// COMPRESSED.  The checksum is enet_crc32 over the UNCOMPRESSED datagram
// (final header, checksum field = the peer's connectID or 0) and is written
// into the checksum field.
// Receive (protocol.c:1022-1091): a COMPRESSED datagram's commands are
// decoded into 4096 - headerSize bytes (0 or more fails); the header is copied
// in front.  With a checksum the field is replaced by connectID (or 0) and
// enet_crc32 over the whole datagram must equal the received field.
//
// The coding itself is the lane kernels' batch (rc_hip_compress /
// rc_hip_decompress on the command ranges); the CRC is rc_crc32_batch.  These
// kernels only frame: one thread per datagram for the headers, one wavefront
// per datagram for the byte copies (16-B stores).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rc_abi_internal.h"

namespace {

constexpr uint32_t kMtu = 4096;                   // ENET_PROTOCOL_MAXIMUM_MTU = sizeof packetData[1]
constexpr uint8_t kFlagCompressed = 0x40;         // bit 14 of the big-endian word, in byte 0
constexpr uint8_t kFlagSentTime = 0x80;           // bit 15

__device__ __forceinline__ uint32_t header_size(uint8_t b0, uint32_t checksum)
{
    return ((b0 & kFlagSentTime) ? 4u : 2u) + (checksum ? 4u : 0u);
}

__device__ __forceinline__ uint32_t load_u32_unaligned(const uint8_t* p)
{
    return static_cast<uint32_t>(p[0]) | (static_cast<uint32_t>(p[1]) << 8) |
           (static_cast<uint32_t>(p[2]) << 16) | (static_cast<uint32_t>(p[3]) << 24);
}

__device__ __forceinline__ void store_u32_unaligned(uint8_t* p, uint32_t v)
{
    p[0] = static_cast<uint8_t>(v); p[1] = static_cast<uint8_t>(v >> 8);
    p[2] = static_cast<uint8_t>(v >> 16); p[3] = static_cast<uint8_t>(v >> 24);
}

// one wavefront copies n bytes; 16-B vector stores where both sides allow
__device__ void wave_copy(uint8_t* dst, const uint8_t* src, uint32_t n, uint32_t lane)
{
    const uintptr_t d = reinterpret_cast<uintptr_t>(dst), s = reinterpret_cast<uintptr_t>(src);
    if (((d | s) & 15) == 0) {
        const uint32_t nv = n >> 4;
        for (uint32_t i = lane; i < nv; i += 64)
            reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
        for (uint32_t i = (nv << 4) + lane; i < n; i += 64) dst[i] = src[i];
    } else {
        for (uint32_t i = lane; i < n; i += 64) dst[i] = src[i];
    }
}

}  // namespace

// ---------------------------------------------------------------- send side

// per datagram: the command range and its output slot (after the header)
extern "C" __global__ void rc_dgram_enc_prep(rc_dgram_dev g)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.n) return;
    const uint32_t len = g.in_len[i];
    const uint32_t hs = len ? header_size(g.in[g.in_off[i]], g.checksum) : 0u;
    const bool ok = len >= hs && len >= 2 && len <= kMtu;
    g.p_off[i] = g.in_off[i] + hs;
    g.p_len[i] = ok ? len - hs : 0u;
    g.q_off[i] = g.out_off[i] + hs;
    g.q_cap[i] = ok ? len - hs : 0u;                     // outLimit = originalSize (protocol.c:1688-1694)
    g.s_off[i] = static_cast<uint64_t>(i) * kMtu;        // checksum scratch slot
}

// per datagram (one wavefront): choose the form, write the checksum input
// (the uncompressed datagram with the final header and the seed) into the
// scratch, and copy the uncompressed datagram to its slot when it is sent as is
extern "C" __global__ __launch_bounds__(256) void rc_dgram_enc_stage(rc_dgram_dev g)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (i >= g.n) return;
    const uint32_t len = g.in_len[i];
    const uint8_t* src = g.in + g.in_off[i];
    const uint32_t hs = len ? header_size(src[0], g.checksum) : 0u;
    if (len < 2 || len < hs || len > kMtu) {
        if (lane == 0) { g.out_len[i] = 0; g.s_len[i] = 0; }
        return;
    }
    const uint32_t L = len - hs, c = g.c_len[i];
    const bool comp = c > 0 && c < L;                   // protocol.c:1696
    uint8_t* dst = g.out + g.out_off[i];
    if (!comp) wave_copy(dst, src, len, lane);
    if (g.checksum) wave_copy(g.scratch + static_cast<uint64_t>(i) * kMtu, src, len, lane);
    __builtin_amdgcn_s_waitcnt(0);   // the copies land before lane 0 patches header bytes
    if (lane == 0) {
        const uint8_t b0 = static_cast<uint8_t>((src[0] & ~kFlagCompressed) | (comp ? kFlagCompressed : 0));
        dst[0] = b0;
        for (uint32_t k = 1; k < hs - (g.checksum ? 4u : 0u); ++k) dst[k] = src[k];
        if (g.checksum) {
            uint8_t* s = g.scratch + static_cast<uint64_t>(i) * kMtu;
            s[0] = b0;
            store_u32_unaligned(s + hs - 4, g.seed[i]);
        }
        g.s_len[i] = g.checksum ? len : 0u;
        g.out_len[i] = comp ? hs + c : len;
    }
}

// the checksum into its field (protocol.c:1709-1718)
extern "C" __global__ void rc_dgram_enc_finish(rc_dgram_dev g)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.n || !g.checksum || g.out_len[i] == 0) return;
    const uint8_t* src = g.in + g.in_off[i];
    const uint32_t hs = header_size(src[0], g.checksum);
    store_u32_unaligned(g.out + g.out_off[i] + hs - 4, g.crc[i]);
}

// ------------------------------------------------------------- receive side

extern "C" __global__ void rc_dgram_dec_prep(rc_dgram_dev g)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.n) return;
    const uint32_t len = g.in_len[i];
    const uint8_t b0 = len ? g.in[g.in_off[i]] : 0;
    const uint32_t hs = header_size(b0, g.checksum);
    const bool comp = len >= 2 && len >= hs && (b0 & kFlagCompressed);
    g.p_off[i] = g.in_off[i] + hs;
    g.p_len[i] = comp ? len - hs : 0u;                  // (0: nothing to decode)
    g.q_off[i] = g.out_off[i] + hs;
    g.q_cap[i] = kMtu - hs;                             // protocol.c:1062-1066
}

// per datagram (one wavefront): assemble header + commands in the slot and
// put the seed into the checksum field (protocol.c:1070-1085)
extern "C" __global__ __launch_bounds__(256) void rc_dgram_dec_stage(rc_dgram_dev g)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    if (i >= g.n) return;
    const uint32_t len = g.in_len[i];
    const uint8_t* src = g.in + g.in_off[i];
    const uint8_t b0 = len ? src[0] : 0;
    const uint32_t hs = header_size(b0, g.checksum);
    uint8_t* dst = g.out + g.out_off[i];
    uint32_t total = 0;
    if (len >= 2 && len >= hs) {                        // protocol.c:1022-1023
        if (b0 & kFlagCompressed) {
            const uint32_t d = g.c_len[i];
            if (d > 0 && d <= kMtu - hs) total = hs + d;   // protocol.c:1067-1068
            if (total) wave_copy(dst, src, hs, lane);
        } else {
            if (len <= kMtu) total = len;
            if (total) wave_copy(dst, src, len, lane);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);   // the copies land before lane 0 patches the checksum field
    if (lane == 0) {
        if (total && g.checksum) {
            g.want[i] = load_u32_unaligned(src + hs - 4);
            store_u32_unaligned(dst + hs - 4, g.seed[i]);
        }
        g.s_len[i] = g.checksum ? total : 0u;
        g.out_len[i] = total;
    }
}

// drop datagrams whose checksum does not match (protocol.c:1088-1089)
extern "C" __global__ void rc_dgram_dec_finish(rc_dgram_dev g)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.n || !g.checksum || g.out_len[i] == 0) return;
    if (g.crc[i] != g.want[i]) g.out_len[i] = 0;
}

extern "C" int rc_hip_dgram_launch(int stage, const rc_dgram_dev* g, void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint32_t n = g->n;
    if (n == 0) return 0;
    const dim3 thr(256), thr_blocks((n + 255) / 256), wave_blocks((n + 3) / 4);
    switch (stage) {
    case RC_DGRAM_ENC_PREP: hipLaunchKernelGGL(rc_dgram_enc_prep, thr_blocks, thr, 0, st, *g); break;
    case RC_DGRAM_ENC_STAGE: hipLaunchKernelGGL(rc_dgram_enc_stage, wave_blocks, thr, 0, st, *g); break;
    case RC_DGRAM_ENC_FINISH: hipLaunchKernelGGL(rc_dgram_enc_finish, thr_blocks, thr, 0, st, *g); break;
    case RC_DGRAM_DEC_PREP: hipLaunchKernelGGL(rc_dgram_dec_prep, thr_blocks, thr, 0, st, *g); break;
    case RC_DGRAM_DEC_STAGE: hipLaunchKernelGGL(rc_dgram_dec_stage, wave_blocks, thr, 0, st, *g); break;
    case RC_DGRAM_DEC_FINISH: hipLaunchKernelGGL(rc_dgram_dec_finish, thr_blocks, thr, 0, st, *g); break;
    default: return static_cast<int>(hipErrorInvalidValue);
    }
    return static_cast<int>(hipGetLastError());
}
