// rc_lane_common.h -- per-lane building blocks shared by the lane kernels
// (rc_lane3.hip) and the fast decoders (rc_dec4.hip, rc_dec6.hip, rc_dec7.hip)
// and encoder (rc_enc2.hip): the order-0 model in LDS,
// byte-parallel (SWAR) helpers, dense 256-symbol context blocks, the byte
// streams and the range coder.  Semantics follow compress.c (cited per item).
#pragma once

#ifndef RC_LANE_HOST_TEST
#include <hip/hip_runtime.h>
#else
#include "lane_host_shim.h"   // tests/proto: host build of the per-lane logic (test only)
#endif
#include <stdint.h>

#include "rc_abi_internal.h"
#include "rc_udiv.h"

#define DEV __device__ __forceinline__

// Diagnostic build only (-DRC_PROFILE, tools/lane_prof.py): per-phase cycle
// stamps accumulated per wave and summed into g_prof.  The product build
// compiles every PROF_* to nothing.
#ifdef RC_PROFILE
__device__ unsigned long long g_prof[64];
__device__ __forceinline__ unsigned long long prof_now()
{
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define PROF_DECL unsigned long long prof_t = prof_now(), prof_acc[12] = {0};
#define PROF(k) { const unsigned long long t_ = prof_now(); prof_acc[k] += t_ - prof_t; prof_t = t_; }
#define PROF_FLUSH(base) { if ((threadIdx.x & 63) == 0) for (int k_ = 0; k_ < 12; ++k_) atomicAdd(&g_prof[(base) + k_], prof_acc[k_]); }
#else
#define PROF_DECL
#define PROF(k)
#define PROF_FLUSH(base)
#endif

namespace {

constexpr uint32_t kTop = 1u << 24;          // compress.c:27
constexpr uint32_t kBot = 1u << 16;          // compress.c:28
constexpr uint32_t kRootDelta = 3;           // compress.c:30
constexpr uint32_t kSubDelta = 2;            // compress.c:35
constexpr uint32_t kSubEscDelta = 5;         // compress.c:36
constexpr uint32_t kMaxNodes = 4096 - 2;     // compress.c:150
constexpr uint32_t kTotalLimit = kBot - 0x100;

constexpr uint32_t kRootStride = 304;        // LDS bytes per lane; 76 dwords (76/4 odd: b128 conflict-free)

DEV uint32_t val_of(uint32_t e) { return e & 0xFF; }
DEV uint32_t cnt_of(uint32_t e) { return (e >> 8) & 0xFF; }
DEV uint32_t sad(uint32_t x, uint32_t acc) { return __builtin_amdgcn_sad_u8(x, 0u, acc); }
// component i of q as a masked OR: a select chain on a lane-varying index
// compiles to branches, or to a dynamically indexed scratch load
DEV uint32_t pick4(uint32_t i, const uint4& q)
{
    return (q.x & (0u - static_cast<uint32_t>(i == 0))) | (q.y & (0u - static_cast<uint32_t>(i == 1))) |
           (q.z & (0u - static_cast<uint32_t>(i == 2))) | (q.w & (0u - static_cast<uint32_t>(i == 3)));
}
DEV bool any_lane(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }
// the same for paths that are rare per wave: their blocks are laid out away
// from the hot loop (instruction-cache locality, fall-through hot path)
#ifndef RC_HOTPATH_ONLY
DEV bool rare_lane(bool p) { return __builtin_expect(__builtin_amdgcn_ballot_w64(p) != 0, 0); }
#else   // static analysis only (tools/phase_asm.sh): the rare paths compiled out
DEV bool rare_lane(bool) { return false; }
#endif

// ---- packed u16 pairs (the 16 cumulative group sums of a 256-symbol context)
#ifndef RC_LANE_HOST_TEST
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
DEV u16x2 as2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
DEV uint32_t as1(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
// (inline asm: the compiler rewrites min(subsat(x, d), 1) into per-half
// compares and selects, four times the instructions)
DEV uint32_t pk_subsat(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_pk_sub_u16 %0, %1, %2 clamp" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
DEV uint32_t pk_min(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
DEV uint32_t pk_mad(uint32_t a, uint32_t b, uint32_t c)     // a * b + c per u16 half
{
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
DEV uint32_t pk_max(uint32_t a, uint32_t b) { return as1(__builtin_elementwise_max(as2(a), as2(b))); }
DEV uint32_t pk_add(uint32_t a, uint32_t b) { return as1(as2(a) + as2(b)); }
DEV uint32_t pk_mul(uint32_t a, uint32_t b) { return as1(as2(a) * as2(b)); }
#else
template <class F> uint32_t pk2(uint32_t a, uint32_t b, F f)
{
    return (f(a & 0xFFFF, b & 0xFFFF) & 0xFFFF) | ((f(a >> 16, b >> 16) & 0xFFFF) << 16);
}
inline uint32_t pk_subsat(uint32_t a, uint32_t b) { return pk2(a, b, [](uint32_t x, uint32_t y) { return x > y ? x - y : 0u; }); }
inline uint32_t pk_min(uint32_t a, uint32_t b) { return pk2(a, b, [](uint32_t x, uint32_t y) { return x < y ? x : y; }); }
inline uint32_t pk_max(uint32_t a, uint32_t b) { return pk2(a, b, [](uint32_t x, uint32_t y) { return x > y ? x : y; }); }
inline uint32_t pk_add(uint32_t a, uint32_t b) { return pk2(a, b, [](uint32_t x, uint32_t y) { return x + y; }); }
inline uint32_t pk_mul(uint32_t a, uint32_t b) { return pk2(a, b, [](uint32_t x, uint32_t y) { return x * y; }); }
inline uint32_t pk_mad(uint32_t a, uint32_t b, uint32_t c) { return pk_add(pk_mul(a, b), c); }
#endif

// C[t] += d for every t >= g, C as 8 packed pairs (C[2i] | C[2i+1] << 16):
// per pair, (t + 1) -sat g is nonzero exactly where t >= g
DEV void cum_add(uint32_t* c, uint32_t g, uint32_t d)
{
    const uint32_t gg = g * 0x00010001u, dd = d * 0x00010001u;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i)
        c[i] = pk_mad(pk_min(pk_subsat((2 * i + 1) | ((2 * i + 2) << 16), gg), 0x00010001u), dd, c[i]);
}

// ------------------------------------------------------------ order 0 (LDS)

DEV void root_clear(uint8_t* r)
{
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int i = 0; i < 18; ++i) reinterpret_cast<uint4*>(r)[i] = z;
}

DEV uint32_t root_c(const uint8_t* r, uint32_t g) { return reinterpret_cast<const uint16_t*>(r + 256)[g]; }

// under = v * 1 + sum of counts below v; cnt = count[v] (compress.c:159-199, minimum 1)
DEV void root_lookup(const uint8_t* r, uint32_t v, uint32_t& under, uint32_t& cnt)
{
    const uint32_t g = v >> 4, j = v & 15;
    const uint4 q = *reinterpret_cast<const uint4*>(r + 16 * g);
    const uint32_t below = g ? root_c(r, g - 1) : 0u;
    uint32_t within = 0;
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d) {
        const uint32_t nb = j > 4 * d ? min(j - 4 * d, 4u) : 0u;
        const uint32_t mask = nb >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
        within = sad(pick4(d, q) & mask, within);
    }
    cnt = (pick4(j >> 2, q) >> (8 * (j & 3))) & 0xFF;
    under = v + below + within;
}

DEV void root_add(uint8_t* r, uint32_t v, uint32_t cnt)
{
    r[v] = static_cast<uint8_t>(cnt + kRootDelta);
    const uint32_t g = v >> 4;
    uint4* cp = reinterpret_cast<uint4*>(r + 256);
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
        uint4 c = cp[h];
        uint32_t* w = reinterpret_cast<uint32_t*>(&c);
#pragma unroll
        for (uint32_t d = 0; d < 4; ++d) {
            const uint32_t g0 = 8 * h + 2 * d;
            w[d] += (g0 >= g ? kRootDelta : 0u) | (g0 + 1 >= g ? (kRootDelta << 16) : 0u);
        }
        cp[h] = c;
    }
}

// first symbol whose interval [v + C(<v), v + 1 + C(<=v)) holds code
// (code < 256 + sum); also returns that interval's start (under) and count[v]
DEV uint32_t root_search(const uint8_t* r, uint32_t code, uint32_t& under, uint32_t& cnt)
{
    const uint4 c0 = reinterpret_cast<const uint4*>(r + 256)[0];
    const uint4 c1 = reinterpret_cast<const uint4*>(r + 256)[1];
    uint32_t g = 0, prev = 0;
#pragma unroll
    for (uint32_t t = 0; t < 16; ++t) {
        const uint32_t w = pick4((t >> 1) & 3, t < 8 ? c0 : c1);
        const uint32_t ct = (t & 1) ? (w >> 16) : (w & 0xFFFF);
        const bool below = 16 * (t + 1) + ct <= code;
        g += below ? 1u : 0u;
        prev = below ? ct : prev;
    }
    // binary search inside the group: 8, 4, 2, 1 symbols, byte sums by SAD
    // (each symbol also owns the root's minimum count of 1)
    const uint4 q = *reinterpret_cast<const uint4*>(r + 16 * g);
    uint32_t base = 16 * g + prev, j = 0;
    uint32_t s = sad(q.x, sad(q.y, 8u));
    bool hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 8u : 0u;
    const uint32_t d0 = hi ? q.z : q.x, d1 = hi ? q.w : q.y;
    s = sad(d0, 4u);
    hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 4u : 0u;
    uint32_t w = hi ? d1 : d0;
    s = sad(w & 0xFFFFu, 2u);
    hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 2u : 0u;
    w = hi ? (w >> 16) : w;
    s = (w & 0xFFu) + 1u;
    hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 1u : 0u;
    w = hi ? (w >> 8) : w;
    under = base;
    cnt = w & 0xFFu;
    return 16 * g + j;
}

// compress.c:90-112 for the root: halve, rebuild C, return the new total
DEV uint32_t root_rescale(uint8_t* r)
{
    uint32_t sum = 0;
    uint32_t cw[8];
#pragma unroll
    for (uint32_t g = 0; g < 16; ++g) {
        uint4 q = reinterpret_cast<uint4*>(r)[g];
        q.x -= (q.x >> 1) & 0x7F7F7F7Fu;
        q.y -= (q.y >> 1) & 0x7F7F7F7Fu;
        q.z -= (q.z >> 1) & 0x7F7F7F7Fu;
        q.w -= (q.w >> 1) & 0x7F7F7F7Fu;
        reinterpret_cast<uint4*>(r)[g] = q;
        sum = sad(q.w, sad(q.z, sad(q.y, sad(q.x, sum))));
        if (g & 1) cw[g >> 1] |= sum << 16; else cw[g >> 1] = sum;
    }
    reinterpret_cast<uint4*>(r + 256)[0] = make_uint4(cw[0], cw[1], cw[2], cw[3]);
    reinterpret_cast<uint4*>(r + 256)[1] = make_uint4(cw[4], cw[5], cw[6], cw[7]);
    return (sum + 1 + 256) & 0xFFFF;
}

DEV uint32_t dot4(uint32_t a, uint32_t b, uint32_t acc) { return __builtin_amdgcn_udot4(a, b, acc, false); }
DEV uint32_t bperm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }
DEV uint32_t align8(uint32_t hi, uint32_t lo, uint32_t n) { return __builtin_amdgcn_alignbyte(hi, lo, n); }

// 0x01 in each byte of w that is >= the value behind ny (= 0x01000100 - v * 0x00010001)
DEV uint32_t swar_ge(uint32_t w, uint32_t ny)
{
    const uint32_t te = bperm(0u, w, 0x0C020C00u) + ny;   // bytes 0, 2 in 16-bit halves, + 256 - v
    const uint32_t to = bperm(0u, w, 0x0C030C01u) + ny;   // bytes 1, 3
    return bperm(to, te, 0x07030501u);                     // the carry bytes: 1 iff byte >= v
}

// bytes [0, k) of dword d (k relative to the array start) as a mask
DEV uint32_t below_mask(int k, int d)
{
    const int kk = k - 4 * d;
    return kk <= 0 ? 0u : (kk >= 4 ? 0xFFFFFFFFu : ((1u << (8 * kk)) - 1u));
}

DEV uint32_t byte_mask(int k, int d)
{
    const int kk = k - 4 * d;
    return (kk >= 0 && kk < 4) ? (0xFFu << (8 * kk)) : 0u;
}

// lane region: [0, 64) header (epoch), [64, 128) a scratch record for
// stores and loads whose result is not used (rc_lane3.hip keeps its memory
// operations unconditional), then the order-1 table: 256 records of 64 B
constexpr uint32_t kDummyRec = 64, kO1Base = 128, kO1Rec = 64;
// dense block sizes: C[16] u16 + counts[256] (+ a u16 per symbol for order-1 contexts)
constexpr uint32_t kDenseO1 = 32 + 256 + 512, kDenseO2 = 32 + 256;

// ---------------------------------------------------------------- dense
// block: C[16] (u16, C[g] = counts of groups 0..g) | counts[256] | links[256] (o1)

struct Dense { uint4 c0, c1, grp; uint32_t link; };

DEV uint32_t dense_c(const Dense& z, uint32_t g)       // C[g]
{
    const uint32_t i = (g >> 1) & 3;
    const uint32_t w = g < 8 ? pick4(i, z.c0) : pick4(i, z.c1);   // (not a select of references)
    return (g & 1) ? (w >> 16) : (w & 0xFFFF);
}

// counts below v (minimum 0) and count[v] in a dense context; loads C, v's group and link
DEV void dense_find(const uint8_t* blk, uint32_t v, bool links, Dense& z, uint32_t& under, uint32_t& cnt)
{
    const uint32_t g = v >> 4, j = v & 15;
    const uint4* p = reinterpret_cast<const uint4*>(blk);
    z.c0 = p[0]; z.c1 = p[1]; z.grp = p[2 + g];
    z.link = links ? reinterpret_cast<const uint16_t*>(blk + 288)[v] : 0u;
    uint32_t within = 0;
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d) {
        const uint32_t nb = j > 4 * d ? min(j - 4 * d, 4u) : 0u;
        const uint32_t mask = nb >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
        within = sad(pick4(d, z.grp) & mask, within);
    }
    under = (g ? dense_c(z, g - 1) : 0u) + within;
    cnt = (pick4(j >> 2, z.grp) >> (8 * (j & 3))) & 0xFF;
}

// count[v] += d and C[g..15] += d, given z from dense_find / dense_search for v
DEV void dense_add(uint8_t* blk, uint32_t v, uint32_t d, Dense& z)
{
    const uint32_t g = v >> 4, j = v & 15, bd = d << (8 * (j & 3)), q = j >> 2;
    z.grp.x += q == 0 ? bd : 0u; z.grp.y += q == 1 ? bd : 0u;
    z.grp.z += q == 2 ? bd : 0u; z.grp.w += q == 3 ? bd : 0u;
    // C[t] += d for t >= g: word i holds C[2i] | C[2i + 1] << 16
    uint32_t cw[8] = {z.c0.x, z.c0.y, z.c0.z, z.c0.w, z.c1.x, z.c1.y, z.c1.z, z.c1.w};
    cum_add(cw, g, d);
    z.c0 = make_uint4(cw[0], cw[1], cw[2], cw[3]);
    z.c1 = make_uint4(cw[4], cw[5], cw[6], cw[7]);
    uint4* p = reinterpret_cast<uint4*>(blk);
    p[0] = z.c0; p[1] = z.c1; p[2 + g] = z.grp;
}

// decoder: symbol whose interval [C(<v), C(<=v)) holds code (minimum 0)
// (have_c: z.c0 / z.c1 already hold the block's C -- rc_lane3.hip keeps an
// order-1 context's C in its record)
DEV bool dense_search(const uint8_t* blk, uint32_t code, bool links, Dense& z, uint32_t& v, uint32_t& under,
                      uint32_t& cnt, bool have_c = false)
{
    const uint4* p = reinterpret_cast<const uint4*>(blk);
    if (!have_c) { z.c0 = p[0]; z.c1 = p[1]; }
    uint32_t g = 0, prev = 0;
#pragma unroll
    for (uint32_t t = 0; t < 16; ++t) {
        const uint32_t ct = dense_c(z, t);
        const bool below = ct <= code;
        g += below ? 1u : 0u;
        prev = below ? ct : prev;
    }
    const bool inside = g < 16;
    g = inside ? g : 15u;
    z.grp = p[2 + g];
    uint32_t base = prev, j = 0;
    uint32_t s = sad(z.grp.x, sad(z.grp.y, 0u));
    bool hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 8u : 0u;
    const uint32_t d0 = hi ? z.grp.z : z.grp.x, d1 = hi ? z.grp.w : z.grp.y;
    s = sad(d0, 0u);
    hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 4u : 0u;
    uint32_t w = hi ? d1 : d0;
    s = sad(w & 0xFFFFu, 0u);
    hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 2u : 0u;
    w = hi ? (w >> 16) : w;
    s = w & 0xFFu;
    hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 1u : 0u;
    w = hi ? (w >> 8) : w;
    v = 16 * g + j;
    under = base;
    cnt = w & 0xFFu;
    z.link = links ? reinterpret_cast<const uint16_t*>(blk + 288)[v] : 0u;
    return inside && cnt != 0 && code < base + cnt;
}

// compress.c:90-112 on a dense context; returns sum of the halved counts.
// All 16 group loads are issued before any of them is used: one memory round
// trip (the compiler otherwise interleaves them with the stores four at a
// time, each batch behind a vmcnt(0): four round trips, taken on ~1/3 of the
// wavefront-steps of a game-state batch, where some lane rescales).
DEV uint32_t dense_rescale(uint8_t* blk)
{
    uint4* p = reinterpret_cast<uint4*>(blk);
    uint32_t sum = 0, cw[8];
    uint4 qs[16];
#pragma unroll
    for (uint32_t g = 0; g < 16; ++g) qs[g] = p[2 + g];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (uint32_t g = 0; g < 16; ++g) {
        uint4 q = qs[g];
        q.x -= (q.x >> 1) & 0x7F7F7F7Fu;
        q.y -= (q.y >> 1) & 0x7F7F7F7Fu;
        q.z -= (q.z >> 1) & 0x7F7F7F7Fu;
        q.w -= (q.w >> 1) & 0x7F7F7F7Fu;
        p[2 + g] = q;
        sum = sad(q.w, sad(q.z, sad(q.y, sad(q.x, sum))));
        if (g & 1) cw[g >> 1] |= sum << 16; else cw[g >> 1] = sum;
    }
    p[0] = make_uint4(cw[0], cw[1], cw[2], cw[3]);
    p[1] = make_uint4(cw[4], cw[5], cw[6], cw[7]);
    return sum;
}

// ------------------------------------------------------- byte streams (HBM)
// Each lane walks its own packet.  Bytes never move through per-byte memory
// accesses or per-byte branches:
//   input  (ByteSrc): a 64-bit lookahead register holds the next `na` bytes
//          (first byte in bits 63..56); taking k bytes is two shifts.  Once
//          per step it is topped up by one aligned dword from a 16-B chunk
//          register; the chunk after that one is loaded a chunk ahead, so the
//          only wait on input data is for a load issued ~16 bytes earlier.
//   output (ByteSink): bytes collect in a 64-bit register, then in a 16-B
//          window; a full window is stored at the top of the next step
//          (sink_flush), before that step's loads.
// Packet edges (unaligned starts, the last partial chunk) take byte-wise
// paths behind wave-uniform guards, so nothing outside [p, p+len) is read or
// written.  Bytes past the end of the input read as 0 (compress.c:366-367).

// Byte-stream addresses are integers (alignment arithmetic); accesses through
// them must name the global address space, otherwise they become flat_*
// operations, which complete out of order and force vmcnt(0) waits -- a full
// drain of every outstanding load and store, including the prefetches.
#ifndef RC_LANE_HOST_TEST
#define GPTR(T, a) ((__attribute__((address_space(1))) T*) (a))
#define GPTRC(T, a) ((const __attribute__((address_space(1))) T*) (a))
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
DEV uint4 gload16(uintptr_t a) { const v4u32 v = *GPTRC(v4u32, a); return make_uint4(v.x, v.y, v.z, v.w); }
#else
#define GPTR(T, a) ((T*) (a))
#define GPTRC(T, a) ((const T*) (a))
DEV uint4 gload16(uintptr_t a) { return *GPTRC(uint4, a); }
#endif

DEV uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

DEV uint32_t sel4(uint32_t q, const uint4& c) { return pick4(q, c); }

// the aligned 16-B chunk at c, zero outside [lo, hi)
DEV uint4 chunk_load(uintptr_t lo, uintptr_t hi, uintptr_t c, bool en)
{
    const bool full = c >= lo && c + 16 <= hi;
    uint4 w = make_uint4(0u, 0u, 0u, 0u);
    if (en && full) w = gload16(c);
    if (rare_lane(en && !full && c < hi && c + 16 > lo)) {
        if (en && !full) {
            uint64_t d0 = 0, d1 = 0;          // (shifts, not an indexed array: that would live in scratch)
#pragma unroll 1
            for (uint32_t t = 0; t < 16; ++t) {
                const uintptr_t a = c + t;
                const uint64_t b = (a >= lo && a < hi) ? *GPTRC(uint8_t, a) : 0u;
                d0 |= t < 8 ? b << (8 * t) : 0ull;
                d1 |= t < 8 ? 0ull : b << (8 * (t - 8));
            }
            w = make_uint4(static_cast<uint32_t>(d0), static_cast<uint32_t>(d0 >> 32),
                           static_cast<uint32_t>(d1), static_cast<uint32_t>(d1 >> 32));
        }
    }
    return w;
}

struct ByteSrc {
    uint64_t la;            // lookahead, next byte in bits 63..56
    uint32_t na, q;         // bytes in la; next dword of c
    uint4 c, n;             // current chunk; the chunk after it (in flight, unmasked)
    uintptr_t next, lo, hi; // address of the chunk after n; packet bounds
    uintptr_t last;         // the aligned chunk holding byte hi - 1
};

// bytes of the chunk at a that lie below hi (the rest reads as 0)
DEV uint4 chunk_mask_hi(uint4 w, uintptr_t a, uintptr_t hi)
{
    const uint32_t v = hi <= a ? 0u : (hi - a >= 16 ? 16u : static_cast<uint32_t>(hi - a));
    uint32_t m[4];
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d) {
        const uint32_t k = v > 4 * d ? min(v - 4 * d, 4u) : 0u;
        m[d] = k >= 4 ? 0xFFFFFFFFu : ((1u << (8 * k)) - 1u);
    }
    return make_uint4(w.x & m[0], w.y & m[1], w.z & m[2], w.w & m[3]);
}

// one more dword into the lookahead where it has room for it (na <= 4).
// Leaves q == 4 when c is used up; src_adv then moves to the next chunk.
DEV void src_fill(ByteSrc& s, bool en)
{
    const bool need = en && s.na <= 4;
    const uint32_t d = bswap(sel4(s.q, s.c));
    const uint32_t sh = need ? 32 - 8 * s.na : 0u;
    s.la |= need ? (static_cast<uint64_t>(d) << sh) : 0ull;
    s.na += need ? 4u : 0u;
    s.q += need ? 1u : 0u;
}

// c := n where c is used up, and load the chunk after it into n.  The load is
// issued for every lane of the wave (lanes that keep n reload it): a load
// predicated per lane makes the compiler copy its result into n right away,
// i.e. wait for it, behind every store in flight.  Chunks past the packet read
// the last one in bounds; bytes past the packet are masked when n is used.
// The decoder calls this at the end of a step: a loop exit between this load
// and the next use of n would make that use wait for vmcnt(0).
DEV void src_adv(ByteSrc& s)
{
    const bool adv = s.q == 4;
    if (any_lane(adv)) {
        // (only a packet's last chunk needs its bytes past the end masked)
        uint4 m = s.n;
        if (rare_lane(adv && s.next > s.hi)) m = chunk_mask_hi(s.n, s.next - 16, s.hi);
        s.c.x = adv ? m.x : s.c.x; s.c.y = adv ? m.y : s.c.y;
        s.c.z = adv ? m.z : s.c.z; s.c.w = adv ? m.w : s.c.w;
        s.q = adv ? 0u : s.q;
        s.next += adv ? 16 : 0;
        const uintptr_t a = s.next - 16;
        s.n = gload16(a <= s.last ? a : s.last);
    }
}

DEV void src_refill(ByteSrc& s, bool en)
{
    src_fill(s, en);
    src_adv(s);
}

DEV void src_init(ByteSrc& s, const uint8_t* p, uint32_t len, bool settle = true)
{
    s.lo = reinterpret_cast<uintptr_t>(p);
    s.hi = s.lo + len;
    s.last = (s.hi - 1) & ~static_cast<uintptr_t>(15);
    const uintptr_t a = s.lo & ~static_cast<uintptr_t>(15);
    s.c = chunk_load(s.lo, s.hi, a, true);
    s.n = chunk_load(s.lo, s.hi, a + 16, true);
    s.next = a + 32;
    const uint32_t sk = static_cast<uint32_t>(s.lo & 3);   // bytes of the first dword before p
    s.q = static_cast<uint32_t>(s.lo & 15) >> 2;
    s.la = static_cast<uint64_t>(bswap(sel4(s.q, s.c)) << (8 * sk)) << 32;
    s.na = 4 - sk;
    s.q += 1;
    if (rare_lane(s.q == 4)) {
        const bool adv = s.q == 4;
        s.c.x = adv ? s.n.x : s.c.x; s.c.y = adv ? s.n.y : s.c.y;
        s.c.z = adv ? s.n.z : s.c.z; s.c.w = adv ? s.n.w : s.c.w;
        s.q = adv ? 0u : s.q;
        if (adv) s.n = chunk_load(s.lo, s.hi, s.next, true);
        s.next += adv ? 16 : 0;
    }
    src_refill(s, true);
    // settle the chunk loads before the step loop: a load still pending at
    // the loop header makes the compiler wait for vmcnt(0) at every step
    if (settle) __builtin_amdgcn_s_waitcnt(0);
}

// next byte (encoder input; the caller refills once per step)
DEV uint32_t src_byte(ByteSrc& s)
{
    const uint32_t b = static_cast<uint32_t>(s.la >> 56);
    s.la <<= 8;
    s.na -= 1;
    return b;
}

// code = code << 8k | next k bytes, k <= min(3, na)
DEV uint32_t src_shift_in(ByteSrc& s, uint32_t code, uint32_t k)
{
    const uint32_t t = static_cast<uint32_t>(s.la >> 32);
    const uint32_t in = static_cast<uint32_t>((static_cast<uint64_t>(t) << (8 * k)) >> 32);
    s.la <<= 8 * k;
    s.na -= k;
    return (code << (8 * k)) | in;
}

struct ByteSink {
    uint64_t acc;           // bytes not yet in the window; byte 0 belongs at waddr + 4 * ws
    uint32_t nb, ws;        // bytes in acc; dwords filled in w
    uint4 w, wp;            // the 16-B window being filled; a full one awaiting its store
    bool pend;              // wp holds a full window (sink_flush stores it)
    uintptr_t waddr, wpaddr, lo;   // 16-aligned addresses of w and wp; packet output start
    uint32_t n, cap;        // bytes produced; capacity
};

DEV void sink_init(ByteSink& o, uint8_t* p, uint32_t cap)
{
    o.lo = reinterpret_cast<uintptr_t>(p);
    o.waddr = o.lo & ~static_cast<uintptr_t>(15);
    o.wpaddr = o.waddr;
    o.ws = static_cast<uint32_t>(o.lo & 15) >> 2;     // (the lead before an unaligned start is never stored)
    o.nb = static_cast<uint32_t>(o.lo & 3);
    o.acc = 0;
    o.w = make_uint4(0u, 0u, 0u, 0u);
    o.wp = o.w;
    o.pend = false;
    o.n = 0;
    o.cap = cap;
}

// bytes [0, k) of (w, tail) at a + i, skipping those before the packet start
DEV void sink_bytes(uintptr_t a, const uint4& w, uint64_t tail, uint32_t k, uintptr_t lo)
{
    const uint64_t w0 = w.x | (static_cast<uint64_t>(w.y) << 32), w1 = w.z | (static_cast<uint64_t>(w.w) << 32);
#pragma unroll 1
    for (uint32_t t = 0; t < k; ++t) {
        const uint64_t src = t < 8 ? w0 : (t < 16 ? w1 : tail);
        if (a + t >= lo) *GPTR(uint8_t, a + t) = static_cast<uint8_t>(src >> (8 * (t & 7)));
    }
}

DEV void sink_store(uintptr_t a, const uint4& w, uintptr_t lo, bool en)
{
    const bool edge = en && a < lo;
#ifndef RC_LANE_HOST_TEST
    if (en && !edge) { v4u32 v = {w.x, w.y, w.z, w.w}; *GPTR(v4u32, a) = v; }
#else
    if (en && !edge) *GPTR(uint4, a) = w;
#endif
    if (rare_lane(edge)) {
        if (edge) sink_bytes(a, w, 0, 16, lo);
    }
}

// Stores the window completed by the previous step.  Called at the top of a
// step, before that step issues its loads: a store issued after a load makes
// the next wait for that load wait for the store as well (vmcnt is in order).
DEV void sink_flush(ByteSink& o)
{
    sink_store(o.wpaddr, o.wp, o.lo, o.pend);
    o.pend = false;
}

// append k <= 3 bytes m (first byte in bits 7..0) where `en`; the caller has
// checked the capacity
DEV void sink_put(ByteSink& o, uint32_t m, uint32_t k, bool en)
{
    o.acc |= en ? (static_cast<uint64_t>(m) << (8 * o.nb)) : 0ull;
    o.nb += en ? k : 0u;
    o.n += en ? k : 0u;
    const bool mv = o.nb >= 4;
    const uint32_t d = static_cast<uint32_t>(o.acc);
    o.w.x = (mv && o.ws == 0) ? d : o.w.x; o.w.y = (mv && o.ws == 1) ? d : o.w.y;
    o.w.z = (mv && o.ws == 2) ? d : o.w.z; o.w.w = (mv && o.ws == 3) ? d : o.w.w;
    o.acc = mv ? (o.acc >> 32) : o.acc;
    o.nb -= mv ? 4u : 0u;
    o.ws += mv ? 1u : 0u;
    const bool full = o.ws == 4;
    if (rare_lane(full && o.pend)) sink_flush(o);      // a second window in one step
    o.wp.x = full ? o.w.x : o.wp.x; o.wp.y = full ? o.w.y : o.wp.y;
    o.wp.z = full ? o.w.z : o.wp.z; o.wp.w = full ? o.w.w : o.wp.w;
    o.wpaddr = full ? o.waddr : o.wpaddr;
    o.pend = o.pend || full;
    o.w.x = full ? 0u : o.w.x; o.w.y = full ? 0u : o.w.y; o.w.z = full ? 0u : o.w.z; o.w.w = full ? 0u : o.w.w;
    o.ws = full ? 0u : o.ws;
    o.waddr += full ? 16 : 0;
}

// the pending window, then what is left in w and acc
DEV void sink_finish(ByteSink& o, bool en)
{
    if (rare_lane(en)) {
        if (en) {
            sink_flush(o);
            const uint32_t d = static_cast<uint32_t>(o.acc);     // nb <= 3: the partial dword at slot ws
            uint4 w = o.w;
            w.x = o.ws == 0 ? d : w.x; w.y = o.ws == 1 ? d : w.y; w.z = o.ws == 2 ? d : w.z; w.w = o.ws == 3 ? d : w.w;
            sink_bytes(o.waddr, w, 0, 4 * o.ws + o.nb, o.lo);
        }
    }
}

// ------------------------------------------------------------- range coder
// Normalisation (compress.c:125-136, :359-370) in closed form: the loop
// shifts while the top byte of low and low + range agree; with
// x = low ^ (low + range) those are the leading zero bytes of x, since every
// shift shifts x too.  The loop only differs from that when the top byte is
// unsettled and range < BOTTOM (range := -low & 0xFFFF); those lanes finish
// in the byte-wise loop behind a wave-uniform guard.

DEV uint32_t settled_bytes(uint32_t low, uint32_t range)
{
    return static_cast<uint32_t>(__builtin_clz((low ^ (low + range)) | 1u)) >> 3;   // 0..3
}

// compress.c:121-137 where `en`; clears `ok` when the output is full (the
// whole compress call then returns 0, compress.c:116-117)
DEV void enc_code(uint32_t& low, uint32_t& range, uint32_t under, uint32_t count, uint32_t total,
                  ByteSink& o, bool en, bool& ok)
{
    en = en && ok;
    if (!any_lane(en)) return;
    const uint32_t r = udiv16(range, en ? total : 1u);
    low = en ? low + under * r : low;
    range = en ? r * count : range;
    const uint32_t k = en ? settled_bytes(low, range) : 0u;
    const bool full = o.n + k > o.cap;
    ok = ok && !full;
    const bool put = en && !full;
    sink_put(o, bswap(low) & ((1u << (8 * k)) - 1u), k, put);
    low = put ? low << (8 * k) : low;
    range = put ? range << (8 * k) : range;
    bool more = put && range < kBot;
    while (rare_lane(more)) {
        const bool carry = (low ^ (low + range)) >= kTop;
        const bool stop = carry && range >= kBot;
        more = more && !stop;
        if (!any_lane(more)) break;
        range = (more && carry) ? ((0u - low) & (kBot - 1)) : range;
        const bool f = more && o.n >= o.cap;
        ok = ok && !f;
        more = more && !f;
        sink_put(o, low >> 24, 1, more);
        range = more ? range << 8 : range;
        low = more ? low << 8 : low;
    }
}

// compress.c:352 (truncated to u16 at :545/:575); divides range by total where `en`
DEV uint32_t dec_read(uint32_t& range, uint32_t low, uint32_t code, uint32_t total, bool en)
{
    const uint32_t r = udiv16(range, en ? total : 1u);
    range = en ? r : range;
    return udiv_lo16(code - low, en ? r : 1u);
}

// dec_read with the reciprocal of total at hand (rc_udiv.h udiv16r)
DEV uint32_t dec_read_r(uint32_t& range, uint32_t low, uint32_t code, uint32_t total, float rtotal)
{
    range = udiv16r(range, total, rtotal);
    return udiv_lo16(code - low, range);
}

// dec_read with the double reciprocal of total at hand (rc_udiv.h udiv16d)
DEV uint32_t dec_read_d(uint32_t& range, uint32_t low, uint32_t code, uint32_t total, double rtotal)
{
    range = udiv16d(range, total, rtotal);
    return udiv_lo16(code - low, range);
}

// compress.c:354-371 where `en`
DEV void dec_code(uint32_t& low, uint32_t& code, uint32_t& range, uint32_t under, uint32_t count,
                  ByteSrc& in, bool en)
{
    low = en ? low + under * range : low;
    range = en ? range * count : range;
    const uint32_t k = en ? settled_bytes(low, range) : 0u;
    const bool fast = k <= in.na;
    const uint32_t kk = fast ? k : 0u;
    code = src_shift_in(in, code, kk);
    low <<= 8 * kk;
    range <<= 8 * kk;
    bool more = en && (!fast || range < kBot);
    if (rare_lane(more)) {
        do {
            const bool carry = (low ^ (low + range)) >= kTop;
            const bool stop = carry && range >= kBot;
            more = more && !stop;
            if (!any_lane(more)) break;
            range = (more && carry) ? ((0u - low) & (kBot - 1)) : range;
            src_adv(in);                   // (the decoder's top src_fill may have used c up)
            src_fill(in, more && in.na == 0);
            code = src_shift_in(in, code, more ? 1u : 0u);
            range = more ? range << 8 : range;
            low = more ? low << 8 : low;
        } while (rare_lane(more));
        // settle this path's input load here: left in flight, it makes the
        // compiler wait for vmcnt(0) -- behind every store -- wherever its
        // registers are next touched on the common path, i.e. on every step
        __builtin_amdgcn_s_waitcnt(0);
    }
}

// dec_code (rc_lane_common.h) for a code applied after the step's record load
// is issued: its rare path shifts in bytes from the lookahead and the current
// chunk (registers) and advances to the next chunk -- a load, then a wait for
// all loads, the record's included -- only where both are used up.
DEV void dec_code_late(uint32_t& low, uint32_t& code, uint32_t& range, uint32_t under, uint32_t count,
                       ByteSrc& in, bool en)
{
    low = en ? low + under * range : low;
    range = en ? range * count : range;
    const uint32_t k = en ? settled_bytes(low, range) : 0u;
    const bool fast = k <= in.na;
    const uint32_t kk = fast ? k : 0u;
    code = src_shift_in(in, code, kk);
    low <<= 8 * kk;
    range <<= 8 * kk;
    bool more = en && (!fast || range < kBot);
    if (rare_lane(more)) {
        bool loaded = false;
        do {
            const bool carry = (low ^ (low + range)) >= kTop;
            const bool stop = carry && range >= kBot;
            more = more && !stop;
            if (!any_lane(more)) break;
            range = (more && carry) ? ((0u - low) & (kBot - 1)) : range;
            if (rare_lane(more && in.na == 0 && in.q == 4)) { src_adv(in); loaded = true; }
            src_fill(in, more && in.na == 0);
            code = src_shift_in(in, code, more ? 1u : 0u);
            range = more ? range << 8 : range;
            low = more ? low << 8 : low;
        } while (rare_lane(more));
        if (loaded) __builtin_amdgcn_s_waitcnt(0);        // (see dec_code)
    }
}

DEV void flag_exact(const rc_workspace_dev& ws, uint32_t pkt)
{
    const uint32_t slot = atomicAdd(&ws.counters[0], 1u);
    ws.flag_list[slot] = pkt;
}

// ------------------------------------------------------------ one packet

// next epoch of the lane's region (a packet start or a model reset); on wrap
// the o1 tags are cleared so that no stale record can match again
DEV uint32_t next_epoch(uint8_t* reg, uint32_t e)
{
    e += 1;
    if (rare_lane((e & 0xFFFF) == 0)) {
        if ((e & 0xFFFF) == 0) {
            for (uint32_t x = 0; x < 256; ++x) *reinterpret_cast<uint32_t*>(reg + kO1Base + x * kO1Rec) = 0u;
            e += 1;
        }
    }
    *reinterpret_cast<uint32_t*>(reg) = e;
    return e;
}

}  // namespace

#if defined(RC_PROFILE) && !defined(RC_LANE_HOST_TEST)
// diagnostic build: copy out (and optionally clear) the phase counters
extern "C" int rc_lane_prof_read(unsigned long long* out, int reset)
{
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * 64);
    if (e == hipSuccess && reset) {
        static const unsigned long long z[64] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof z);
    }
    return static_cast<int>(e);
}
#endif
