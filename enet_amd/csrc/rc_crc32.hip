// rc_crc32.hip -- batched ENet datagram checksums on MI355X (gfx950).
//
// Same result as enet_crc32 (packet.c:143-163) over one buffer per packet:
// reflected CRC-32, polynomial 0xEDB88320, register preset 0xFFFFFFFF, final
// complement, returned in network byte order (ENET_HOST_TO_NET_32).
// protocol.c:1709-1718 (send) and :1075-1091 (receive) are the call sites.
//
// Four lanes per packet (sixteen packets per wavefront), LDS-bound:
//   * The packet is cut into 256-B rounds aligned to its END (a raw CRC with
//     a zero register ignores leading zero bytes, so the first round is
//     padded at the front for free).  Lane s of the packet's 4 owns bytes
//     [64 s, 64 s + 64) of every round: four aligned 16-B loads per lane and
//     round, a funnel shift (with the next lane's first granule) for the
//     packet's alignment.
//   * A lane's raw CRC of its 64 contiguous bytes is four slice-by-16 lookups
//     chained through the register (the CRC so far xor-ed into the next 16
//     bytes' first four), folded into the lane's running value across
//     rounds: acc = shift(acc, 256) ^ crc64 -- the lane's interleaved stream,
//     256 B apart.
//   * The 4 running values are combined once per packet in a 2-level xor
//     tree: crc(A||B) = shift(crc(A), |B|) ^ crc(B), where shift(v, n) -- n
//     zero bytes through the register -- is linear in v, i.e. four 256-entry
//     lookups (n = 64 << level).
//   * The 0xFFFFFFFF preset is folded in by complementing the first four
//     message bytes (identical for packets of >= 4 bytes); shorter packets add
//     shift(0xFFFFFFFF, L) directly.
// Per byte: 1 + 1/16 table lookups in the rounds (16 lanes per packet with
// 16-B chunks took 1 + 1/4: the fold after every 16 bytes) and a quarter of
// the tree's; the LDS array's cycles (random bytes: 3-4-way bank conflicts
// per 32-lane group) are the bound.
// Tables (28 KiB) are built on the host once per context and staged into LDS
// by each workgroup of a persistent grid.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rc_abi_internal.h"

namespace {

constexpr uint32_t kSlice = 16;                 // slice-by-16 tables
constexpr uint32_t kLevels = 3;                 // shift tables for 64 << 0..2 bytes (tree levels 0..1, rounds)
constexpr uint32_t kTableWords = (kSlice + 4 * kLevels) * 256;
constexpr uint32_t kLanesPer = 4;               // lanes per packet
constexpr uint32_t kGran = 4;                   // 16-B granules per lane and round
constexpr uint32_t kLaneBytes = 16 * kGran;     // 64
constexpr uint32_t kRound = kLaneBytes * kLanesPer;     // bytes per round (256)
constexpr uint32_t kPer = 64 / kLanesPer;       // packets per wavefront
constexpr uint32_t kWavesPerGroup = 16;             // 1024-thread workgroups: the 36-KiB table staging per workgroup is read once per 16 wavefronts

__device__ __forceinline__ uint32_t byte_of(uint32_t w, uint32_t k) { return (w >> (8 * k)) & 0xFFu; }

// 0xFF in every byte whose index (0..3 within dword d of a 16-B chunk) is >= k
// (branch-free: this runs on every round that holds some packet's start)
__device__ __forceinline__ uint32_t bytes_from(int k, int d)
{
    const int kd = min(max(k - 4 * d, 0), 4);
    return static_cast<uint32_t>(0xFFFFFFFFull << (8 * kd));
}

__device__ __forceinline__ uint32_t shift_by(const uint32_t* s, uint32_t v)
{
    return s[byte_of(v, 0)] ^ s[256 + byte_of(v, 1)] ^ s[512 + byte_of(v, 2)] ^ s[768 + byte_of(v, 3)];
}

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
// 16-B load through a global-address-space pointer (an integer address would
// otherwise become a flat load)
__device__ __forceinline__ uint4 gload16(uint64_t a)
{
    const v4u32 v = *((const __attribute__((address_space(1))) v4u32*) a);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// the value of lane + 1 within the lane's row of 16 (DPP row_shl:1; 0 for
// the row's last lane; a packet's last lane loads its own)
__device__ __forceinline__ uint32_t row_next(uint32_t x)
{
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x101, 0xF, 0xF, true));
}

__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t sh)
{
    // bytes sh.. of the 8-byte little-endian pair (lo, hi), sh in 0..3
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

}  // namespace

extern "C" __global__ __launch_bounds__(64 * kWavesPerGroup)
void rc_crc32_batch(const uint8_t* __restrict__ in, const uint64_t* __restrict__ in_off,
                    const uint32_t* __restrict__ in_len, uint32_t n, uint32_t* __restrict__ crc_out,
                    const uint32_t* __restrict__ tables)
{
    __shared__ uint32_t tab[kTableWords];
    for (uint32_t i = threadIdx.x; i < kTableWords / 4; i += blockDim.x)
        reinterpret_cast<uint4*>(tab)[i] = reinterpret_cast<const uint4*>(tables)[i];
    __syncthreads();
    const uint32_t* sh = tab + kSlice * 256;    // shift tables, level-major: 64, 128, 256 bytes
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t s = lane & (kLanesPer - 1);  // lane within the packet's 4
    const uint32_t q = lane / kLanesPer;        // the wavefront's packet slot
    const uint32_t wave = blockIdx.x * kWavesPerGroup + (threadIdx.x >> 6);
    const uint32_t stride = gridDim.x * kWavesPerGroup * kPer;
    const uint64_t base = reinterpret_cast<uint64_t>(in);
    // Each group of 4 lanes walks its own packets (p, p + stride, ...) one
    // round per iteration, so that a ragged batch does not leave lanes idle
    // until the wavefront's longest packet ends; the xor tree runs when any
    // group of the wavefront has finished its packet.
    uint32_t p = wave * kPer + q;
    bool live = p < n;
    uint64_t start = 0, end = 0;
    uint32_t len = 0, rounds = 0, mis = 0, rr = 0, acc = 0;
    if (live) {
        start = base + in_off[p];
        len = in_len[p];
        end = start + len;
        rounds = (len + kRound - 1) / kRound;
        mis = static_cast<uint32_t>(end & 15);
    }
    while (__builtin_amdgcn_ballot_w64(live) != 0) {
        const bool on = live && rr < rounds;
        const uint32_t dq = mis >> 2, bs = mis & 3;
        // this lane's 64 bytes: [c, c + 64) (may start before the packet in the first round)
        const uint64_t c = end - static_cast<uint64_t>(kRound) * (rounds - rr) + kLaneBytes * s;
        const uint64_t a = c - mis;                             // aligned granule holding byte c
        uint32_t w[4 * kGran + 4];
#pragma unroll
        for (uint32_t g = 0; g < kGran; ++g) {
            uint4 x = make_uint4(0, 0, 0, 0);
            if (on && a + 16 * (g + 1) > start) x = gload16(a + 16 * g);   // granule overlaps the packet
            w[4 * g] = x.x; w[4 * g + 1] = x.y; w[4 * g + 2] = x.z; w[4 * g + 3] = x.w;
        }
        uint32_t d[4 * kGran];
#pragma unroll
        for (uint32_t k = 0; k < 4 * kGran; ++k) d[k] = w[k];
        if (__builtin_amdgcn_ballot_w64(on && mis != 0) != 0) {
            // the granule after the lane's four: the neighbour's first (a DPP
            // row shift; the group's lanes share packet and round); the
            // packet's last lane loads its own
            uint4 x;
            x.x = row_next(w[0]); x.y = row_next(w[1]); x.z = row_next(w[2]); x.w = row_next(w[3]);
            if (on && s == kLanesPer - 1 && mis) x = gload16(a + kLaneBytes);
            w[4 * kGran] = x.x; w[4 * kGran + 1] = x.y; w[4 * kGran + 2] = x.z; w[4 * kGran + 3] = x.w;
            // funnel-shift the 80 bytes right by mis -> 64 bytes d[0..15]: a
            // two-stage dword shifter (two-way selects; a four-way select on
            // dq became a branch per dword), then the byte shift
            // (as bit selects: the compiler turns two-way selects over the
            // array into a scratch-memory indexed copy)
            const uint32_t m2 = 0u - ((dq >> 1) & 1u), m1 = 0u - (dq & 1u);
#pragma unroll
            for (uint32_t k = 0; k < 4 * kGran + 2; ++k) w[k] = (w[k + 2] & m2) | (w[k] & ~m2);
#pragma unroll
            for (uint32_t k = 0; k < 4 * kGran + 1; ++k) w[k] = (w[k + 1] & m1) | (w[k] & ~m1);
#pragma unroll
            for (uint32_t k = 0; k < 4 * kGran; ++k) d[k] = funnel(w[k], w[k + 1], bs);
        }
        // zero the bytes before the packet; complement its first four
        // (register preset): only the chunks at a packet's start
        const int lead = static_cast<int>(static_cast<int64_t>(start - c));   // packet byte 0 in chunk
        if (__builtin_amdgcn_ballot_w64(on && lead > -4) != 0) {
            // (bytes_from(lead + 4, k) == bytes_from(lead, k - 1))
            const uint32_t cm = len >= 4 ? ~0u : 0u;
            uint32_t prev = bytes_from(lead, -1);
#pragma unroll
            for (int k = 0; k < static_cast<int>(4 * kGran); ++k) {
                const uint32_t keep = bytes_from(lead, k);
                d[k] = (d[k] & keep) ^ (keep & ~prev & cm);
                prev = keep;
            }
        }
        // raw CRC of the 64 bytes (slice-by-16 per granule, the register
        // carried into the next granule's first four bytes), folded into the
        // lane's stream
        uint32_t v = 0;
#pragma unroll
        for (uint32_t g = 0; g < kGran; ++g) {
            d[4 * g] ^= v;
            v = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int j = 0; j < 4; ++j) v ^= tab[(15 - (4 * k + j)) * 256 + byte_of(d[4 * g + k], j)];
        }
        const uint32_t nacc = shift_by(sh + 2 * 1024, acc) ^ v;
        acc = on ? nacc : acc;
        rr += 1;
        const bool fin = live && rr >= rounds;                  // (an empty packet: at once)
        if (__builtin_amdgcn_ballot_w64(fin) != 0) {
            // xor tree over the packet's 4 lanes (lane order = message order)
            uint32_t t2 = acc;
#pragma unroll
            for (uint32_t lv = 0; lv < 2; ++lv) {
                const uint32_t m = 1u << lv;
                const uint32_t t = shift_by(sh + lv * 1024, t2);
                const uint32_t ot = __shfl_xor(t, m), oa = __shfl_xor(t2, m);
                t2 = (s & m) ? (ot ^ t2) : (t ^ oa);
            }
            if (fin) {
                if (s == 0) {
                    uint32_t crc = t2;
                    if (len < 4) {                   // preset through len bytes, zero data
                        uint32_t rg = 0xFFFFFFFFu;
                        for (uint32_t k = 0; k < len; ++k) rg = (rg >> 8) ^ tab[rg & 0xFF];
                        crc ^= rg;
                    }
                    crc_out[p] = __builtin_bswap32(~crc);
                }
                p += stride;
                live = p < n;
                rr = 0;
                acc = 0;
                start = 0; end = 0; len = 0; rounds = 0; mis = 0;
                if (live) {
                    start = base + in_off[p];
                    len = in_len[p];
                    end = start + len;
                    rounds = (len + kRound - 1) / kRound;
                    mis = static_cast<uint32_t>(end & 15);
                }
            }
        }
    }
}

extern "C" uint32_t rc_hip_crc32_table_words(void) { return kTableWords; }

// Host-side table build (called once per context by rc_host.c).
extern "C" void rc_hip_crc32_build_tables(uint32_t* t)
{
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t c = b;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
        t[b] = c;
    }
    for (uint32_t s = 1; s < kSlice; ++s)
        for (uint32_t b = 0; b < 256; ++b) {
            const uint32_t prev = t[(s - 1) * 256 + b];
            t[s * 256 + b] = (prev >> 8) ^ t[prev & 0xFF];
        }
    // shift(x, n): n zero bytes through a raw register holding x
    auto shift = [&](uint32_t x, uint32_t nbytes) {
        for (uint32_t k = 0; k < nbytes; ++k) x = (x >> 8) ^ t[x & 0xFF];
        return x;
    };
    uint32_t* sh = t + kSlice * 256;
    for (uint32_t lv = 0; lv < kLevels; ++lv)
        for (uint32_t j = 0; j < 4; ++j)
            for (uint32_t b = 0; b < 256; ++b)
                sh[lv * 1024 + j * 256 + b] = shift(b << (8 * j), 64u << lv);
}

extern "C" int rc_hip_crc32(const uint8_t* in, const uint64_t* in_off, const uint32_t* in_len, uint32_t n,
                            uint32_t* crc_out, const uint32_t* tables, void* stream)
{
    if (n == 0) return 0;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    uint32_t groups = (n + kPer * kWavesPerGroup - 1) / (kPer * kWavesPerGroup);
    const uint32_t cap = static_cast<uint32_t>(cus) * 2;        // 2 x 16 wavefronts per CU (the wave limit), 56 KiB LDS
    if (groups > cap) groups = cap;
    hipLaunchKernelGGL(rc_crc32_batch, dim3(groups), dim3(64 * kWavesPerGroup), 0,
                       static_cast<hipStream_t>(stream), in, in_off, in_len, n, crc_out, tables);
    return static_cast<int>(hipGetLastError());
}
