// rc_lane.hip -- lane-per-packet range-coder kernels for MI355X (gfx950).
//
// Same semantics as compress.c (enet_range_coder_compress :246-342,
// enet_range_coder_decompress :498-627), bit-exact.
//
// Why one packet per LANE: the coder is a byte-serial dependency chain.  With
// one packet per wavefront (rc_kernels.hip "wave" kernels) that chain is
// wave-uniform work, i.e. it runs on the CU's scalar unit, which every
// resident wave shares; rocprof showed those kernels issuing ~500 SALU
// instructions per byte (profiles/r1_v1wave_pmc_sq.json).  Here 64 packets
// advance in lock-step in one wave, so the same arithmetic is one VALU
// instruction for 64 packets.
//
// Model (only {count[v], escapes, total} per context and the node count are
// observable):
//   order 0 (root): per lane in LDS, counts[256] (u8) + C[16] (u16 cumulative
//       count at the end of each 16-symbol group) -> lookups are 1-2 LDS
//       reads + byte-SAD sums, no tree walk.
//   orders 1 and 2: records in a per-lane HBM region holding each context's
//       symbols as sorted byte arrays (values, counts) that are searched and
//       updated four symbols per instruction (byte permutes, v_dot4, v_sad);
//       large contexts switch to a dense 256-symbol table.  See "order 1/2
//       contexts" below for the layout.
//   Each byte costs one HBM round trip, and that load is issued a step ahead.
//
// Code shape: 64 lanes run 64 different packets, so every `if` on per-lane
// data is divergent.  Common paths are written as straight-line predicated
// register code; rare paths (dense contexts, rescale, packet edges, model
// reset) sit behind wave-uniform ballot guards so a wave that does not need
// them pays one scalar branch.
//
// Packets this model cannot reproduce -- corrupt streams whose root code
// points past symbol 255 (compress.c:427-438 then depends on tree shape) --
// and packets that exhaust their region are appended to the exact-path list
// (rc_kernels.hip), which re-runs compress.c's binary-tree model.

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
DEV uint32_t pick4(uint32_t i, const uint4& q) { return i == 0 ? q.x : i == 1 ? q.y : i == 2 ? q.z : q.w; }
DEV bool any_lane(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

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

// ------------------------------------------------ order 1/2 contexts (HBM)
// Per lane region (rc_hip_lane_region_bytes):
//   [0, 64)        lane header: epoch counter (u32)
//   [64, +16 KiB)  order-1 table: 256 records of 64 B, direct-mapped by the
//                  context byte
//   arena          bump-allocated: order-2 records (32 B) and dense blocks
//
// A record holds a context's symbols as parallel byte arrays, sorted by value:
//   w0 = tag | len << 16 | dense << 24   (o1: tag = epoch, the record is
//                                          empty unless it matches; o2: 0)
//   w1 = esc | total << 16               (total = esc + sum(counts) mod 2^16,
//                                          maintained as compress.c:309-314)
//   w2 = dense block offset (when dense)
//   o1 (64 B): w4..w6 vals[12], w7..w9 counts[12], w10..w15 links[12] (u16:
//       the o2 record of context (prev, val), compress.c's `parent` chain)
//   o2 (32 B): w4..w5 vals[8], w6..w7 counts[8]
// Unused slots hold value 0xFF and count 0, so the byte-parallel (SWAR)
// scans need no length mask: a present symbol's count is never 0 (rescale
// keeps c - c/2 >= 1).  A context that outgrows its inline slots becomes
// dense: C[16] (u16 cumulative group sums) + counts[256] (+ links[256] for
// o1), found through w2 -- lookups are O(1) like the root's.
//
// Every packet and every model reset (compress.c:148-157) starts a new epoch:
// o1 records from older epochs read as empty, the arena restarts, and o2
// records are only reachable through current o1 links -- nothing is cleared.
// o2 entries carry no links: the next o2 context (prev, v) is found through
// o1[prev], which the step has loaded anyway.

constexpr uint32_t kO1Base = 64, kO1Rec = 64, kO1NV = 3, kO2Rec = 32, kO2NV = 2;
constexpr uint32_t kArenaBase = kO1Base + 256 * kO1Rec;
constexpr uint32_t kDenseO1 = 32 + 256 + 512, kDenseO2 = 32 + 256;
constexpr uint32_t kDenseBudget = 0xFFFFFFFFu;   // dense blocks are bounded by the region size

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

template <uint32_t NV>
struct Ctx {
    uint32_t off, tag, len, dense, esc, tot, ext;
    uint32_t val[NV], cnt[NV];
    uint32_t lnk[2 * NV];            // o1 only (u16 pairs); unused for o2
};
using Ctx1 = Ctx<kO1NV>;
using Ctx2 = Ctx<kO2NV>;

template <uint32_t NV>
DEV void ctx_empty(Ctx<NV>& c, uint32_t off, uint32_t tag)
{
    c.off = off; c.tag = tag; c.len = 0; c.dense = 0; c.esc = 0; c.tot = 0; c.ext = 0;
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) { c.val[d] = 0xFFFFFFFFu; c.cnt[d] = 0u; }
#pragma unroll
    for (uint32_t d = 0; d < 2 * NV; ++d) c.lnk[d] = 0u;
}

// o1 records are loaded a step ahead as raw words and decoded only when the
// step that needs them starts: a select on loaded data placed right after the
// load would make the wave wait for HBM there.
struct Raw1 { uint4 q0, q1, q2, q3; uint32_t x; };

DEV void o1_fetch(const uint8_t* reg, uint32_t x, Raw1& w)
{
    const uint4* p = reinterpret_cast<const uint4*>(reg + kO1Base + x * kO1Rec);
    w.q0 = p[0]; w.q1 = p[1]; w.q2 = p[2]; w.q3 = p[3]; w.x = x;
}

DEV void o1_decode(const Raw1& w, uint32_t epoch, Ctx1& c)
{
    const bool live = (w.q0.x & 0xFFFF) == epoch;
    c.off = kO1Base + w.x * kO1Rec; c.tag = epoch;
    c.len = live ? (w.q0.x >> 16) & 0xFF : 0u;
    c.dense = live ? w.q0.x >> 24 : 0u;
    c.esc = live ? w.q0.y & 0xFFFF : 0u;
    c.tot = live ? w.q0.y >> 16 : 0u;
    c.ext = w.q0.z;
    c.val[0] = live ? w.q1.x : 0xFFFFFFFFu; c.val[1] = live ? w.q1.y : 0xFFFFFFFFu;
    c.val[2] = live ? w.q1.z : 0xFFFFFFFFu;
    c.cnt[0] = live ? w.q1.w : 0u; c.cnt[1] = live ? w.q2.x : 0u; c.cnt[2] = live ? w.q2.y : 0u;
    c.lnk[0] = w.q2.z; c.lnk[1] = w.q2.w; c.lnk[2] = w.q3.x; c.lnk[3] = w.q3.y; c.lnk[4] = w.q3.z; c.lnk[5] = w.q3.w;
}

DEV void o1_store(uint8_t* reg, const Ctx1& c)
{
    uint4* p = reinterpret_cast<uint4*>(reg + c.off);
    p[0] = make_uint4(c.tag | (c.len << 16) | (c.dense << 24), c.esc | (c.tot << 16), c.ext, 0u);
    p[1] = make_uint4(c.val[0], c.val[1], c.val[2], c.cnt[0]);
    p[2] = make_uint4(c.cnt[1], c.cnt[2], c.lnk[0], c.lnk[1]);
    p[3] = make_uint4(c.lnk[2], c.lnk[3], c.lnk[4], c.lnk[5]);
}

struct Raw2 { uint4 q0, q1; };

DEV void o2_fetch(const uint8_t* reg, uint32_t idx, Raw2& w)
{
    const uint4* p = reinterpret_cast<const uint4*>(reg + idx * kO2Rec);
    w.q0 = p[0]; w.q1 = p[1];
}

DEV void o2_decode(const Raw2& w, uint32_t idx, Ctx2& c)
{
    c.off = idx * kO2Rec; c.tag = 0;
    c.len = (w.q0.x >> 16) & 0xFF; c.dense = w.q0.x >> 24;
    c.esc = w.q0.y & 0xFFFF; c.tot = w.q0.y >> 16; c.ext = w.q0.z;
    c.val[0] = w.q1.x; c.val[1] = w.q1.y; c.cnt[0] = w.q1.z; c.cnt[1] = w.q1.w;
    c.lnk[0] = c.lnk[1] = c.lnk[2] = c.lnk[3] = 0u;
}

DEV void o2_store(uint8_t* reg, const Ctx2& c)
{
    uint4* p = reinterpret_cast<uint4*>(reg + c.off);
    p[0] = make_uint4((c.len << 16) | (c.dense << 24), c.esc | (c.tot << 16), c.ext, 0u);
    p[1] = make_uint4(c.val[0], c.val[1], c.cnt[0], c.cnt[1]);
}

// link of slot k (o1 inline)
template <uint32_t NV>
DEV uint32_t lnk_get(const Ctx<NV>& c, uint32_t k)
{
    // masked OR, not a select chain: the compiler turns selects between
    // fields into a dynamically indexed load, which forces the record into
    // scratch memory
    const uint32_t d = k >> 1;
    uint32_t w = 0;
#pragma unroll
    for (uint32_t i = 0; i < 2 * NV; ++i) w |= c.lnk[i] & (0u - static_cast<uint32_t>(d == i));
    return (w >> (16 * (k & 1))) & 0xFFFF;
}

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
#define RC_CADD(w, t) w += ((t) >= g ? d : 0u) | ((t) + 1 >= g ? (d << 16) : 0u)
    RC_CADD(z.c0.x, 0u); RC_CADD(z.c0.y, 2u); RC_CADD(z.c0.z, 4u); RC_CADD(z.c0.w, 6u);
    RC_CADD(z.c1.x, 8u); RC_CADD(z.c1.y, 10u); RC_CADD(z.c1.z, 12u); RC_CADD(z.c1.w, 14u);
#undef RC_CADD
    uint4* p = reinterpret_cast<uint4*>(blk);
    p[0] = z.c0; p[1] = z.c1; p[2 + g] = z.grp;
}

// decoder: symbol whose interval [C(<v), C(<=v)) holds code (minimum 0)
DEV bool dense_search(const uint8_t* blk, uint32_t code, bool links, Dense& z, uint32_t& v, uint32_t& under,
                      uint32_t& cnt)
{
    const uint4* p = reinterpret_cast<const uint4*>(blk);
    z.c0 = p[0]; z.c1 = p[1];
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

// compress.c:90-112 on a dense context; returns sum of the halved counts
DEV uint32_t dense_rescale(uint8_t* blk)
{
    uint4* p = reinterpret_cast<uint4*>(blk);
    uint32_t sum = 0, cw[8];
#pragma unroll
    for (uint32_t g = 0; g < 16; ++g) {
        uint4 q = p[2 + g];
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

// move an inline context to a fresh dense block (where `en`); false = arena full
template <uint32_t NV>
DEV bool densify(uint8_t* reg, Ctx<NV>& c, uint32_t& bump, uint32_t end, bool links, bool en)
{
    const uint32_t size = links ? kDenseO1 : kDenseO2;
    const uint32_t at = (bump + 15) & ~15u;
    const bool ok = at + size <= end;
    if (!(en && ok)) return !en;
    bump = at + size;
    uint8_t* blk = reg + at;
    uint4* p = reinterpret_cast<uint4*>(blk);
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    for (uint32_t i = 2; i < 18; ++i) p[i] = z;
    uint32_t cw[8];
#pragma unroll
    for (uint32_t g = 0; g < 16; ++g) {                 // C[g] = counts of values < 16 (g + 1)
        const uint32_t ny = 0x01000100u - (16 * (g + 1)) * 0x00010001u;
        uint32_t s = 0;
#pragma unroll
        for (uint32_t d = 0; d < NV; ++d) s = dot4(c.cnt[d], swar_ge(c.val[d], ny) ^ 0x01010101u, s);
        if (g & 1) cw[g >> 1] |= s << 16; else cw[g >> 1] = s;
    }
    p[0] = make_uint4(cw[0], cw[1], cw[2], cw[3]);
    p[1] = make_uint4(cw[4], cw[5], cw[6], cw[7]);
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) {
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) {
            if (4 * d + t < c.len) {
                const uint32_t vv = (c.val[d] >> (8 * t)) & 0xFF;
                blk[32 + vv] = static_cast<uint8_t>((c.cnt[d] >> (8 * t)) & 0xFF);
                if (links) reinterpret_cast<uint16_t*>(blk + 288)[vv] =
                    static_cast<uint16_t>((c.lnk[2 * d + (t >> 1)] >> (16 * (t & 1))) & 0xFFFF);
            }
        }
    }
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) { c.val[d] = 0xFFFFFFFFu; c.cnt[d] = 0u; }
    c.dense = 1;
    c.ext = at;
    return true;
}

// ------------------------------------------------ lookup and update (SWAR)

template <uint32_t NV>
struct Look {
    uint32_t k, under, cnt, link;
    bool found;
    uint32_t eq[NV];
    Dense z;
};

// compress.c:159-199 lookup of v (minimum 0): insertion slot k, counts below
// v, count[v]; plus the link (o1) when present
template <uint32_t NV>
DEV Look<NV> ctx_find(const uint8_t* reg, const Ctx<NV>& c, uint32_t v, bool links)
{
    Look<NV> h;
    h.k = 0; h.under = 0; h.cnt = 0; h.link = 0;
    const uint32_t ny = 0x01000100u - v * 0x00010001u;
    const uint32_t ny1 = ny - 0x00010001u;
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) {
        const uint32_t ge = swar_ge(c.val[d], ny);
        const uint32_t lt = ge ^ 0x01010101u;
        // equal = >= v and not >= v + 1, among the live slots (v = 255 matches padding)
        h.eq[d] = (ge ^ swar_ge(c.val[d], ny1)) & below_mask(static_cast<int>(c.len), d) & 0x01010101u;
        h.k = sad(lt, h.k);
        h.under = dot4(c.cnt[d], lt, h.under);
        h.cnt = dot4(c.cnt[d], h.eq[d], h.cnt);
    }
    if (links) h.link = lnk_get<NV>(c, h.k);
    if (any_lane(c.dense != 0)) {
        if (c.dense != 0) {
            uint32_t u, n;
            dense_find(reg + c.ext, v, links, h.z, u, n);
            h.under = u; h.cnt = n; h.link = h.z.link;
        }
    }
    h.found = h.cnt != 0;
    return h;
}

// insert (v, count 2[, link]) at slot k of an inline context with a free slot
template <uint32_t NV>
DEV void inline_insert(Ctx<NV>& c, uint32_t k, uint32_t v, uint32_t link, bool links, bool en)
{
    const int kk = static_cast<int>(k);
    uint32_t pv = 0xFFFFFFFFu, pc = 0u;
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) {
        const uint32_t bm = below_mask(kk, d), im = byte_mask(kk, d);
        const uint32_t sv = align8(c.val[d], pv, 3), sc = align8(c.cnt[d], pc, 3);
        pv = c.val[d]; pc = c.cnt[d];
        const uint32_t nv = (c.val[d] & bm) | (sv & ~bm & ~im) | ((v * 0x01010101u) & im);
        const uint32_t nc = (c.cnt[d] & bm) | (sc & ~bm & ~im) | ((kSubDelta * 0x01010101u) & im);
        c.val[d] = en ? nv : c.val[d];
        c.cnt[d] = en ? nc : c.cnt[d];
    }
    if (links) {
        uint32_t pl = 0u;
#pragma unroll
        for (uint32_t d = 0; d < 2 * NV; ++d) {
            const int kk2 = kk - 2 * static_cast<int>(d);
            const uint32_t bm = kk2 <= 0 ? 0u : (kk2 >= 2 ? 0xFFFFFFFFu : 0xFFFFu);
            const uint32_t im = kk2 == 0 ? 0xFFFFu : (kk2 == 1 ? 0xFFFF0000u : 0u);
            const uint32_t sl = align8(c.lnk[d], pl, 2);
            pl = c.lnk[d];
            const uint32_t nl = (c.lnk[d] & bm) | (sl & ~bm & ~im) | ((link * 0x00010001u) & im);
            c.lnk[d] = en ? nl : c.lnk[d];
        }
    }
}

// compress.c:90-112 where `en`
template <uint32_t NV>
DEV void ctx_rescale(uint8_t* reg, Ctx<NV>& c, bool en)
{
    if (!any_lane(en)) return;
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) {
        const uint32_t h = c.cnt[d] - ((c.cnt[d] >> 1) & 0x7F7F7F7Fu);
        c.cnt[d] = en ? h : c.cnt[d];
        sum = sad(h, sum);
    }
    if (any_lane(en && c.dense != 0)) {
        if (en && c.dense != 0) sum = dense_rescale(reg + c.ext);
    }
    c.esc -= en ? (c.esc >> 1) : 0u;
    c.tot = en ? ((c.esc + sum) & 0xFFFF) : c.tot;
}

// compress.c:293-314 (and the decoder's patch, :598-615) where `en`: bump
// v or insert it.  ALLOC (order-1 contexts): a new symbol gets a fresh o2
// record, whose index becomes its link.  Returns the lookup (old count).
template <uint32_t NV, bool ALLOC>
DEV Look<NV> ctx_update(uint8_t* reg, Ctx<NV>& c, uint32_t v, uint32_t& bump, uint32_t end,
                        uint32_t& nodes, uint32_t& dense_left, bool& ovf, bool en)
{
    Look<NV> h = ctx_find<NV>(reg, c, v, ALLOC);
    const bool ins = en && !h.found;
    uint32_t newlink = h.link;
    if (ALLOC) {
        const uint32_t at = bump;
        newlink = ins ? at / kO2Rec : h.link;
        bump += ins ? kO2Rec : 0u;
        ovf = ovf || (ins && bump > end);
    }
    const bool inl = c.dense == 0;
    // inline bump
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) c.cnt[d] += (en && h.found && inl) ? (h.eq[d] << 1) : 0u;
    // inline insert with room
    const uint32_t cap = 4u * NV;
    inline_insert<NV>(c, h.k, v, newlink, ALLOC, ins && inl && c.len < cap);
    // full inline context -> dense; dense bump / insert
    const bool grow = ins && inl && c.len >= cap;
    if (any_lane(grow || (en && !inl))) {
        if (grow) {
            const bool ok = dense_left > 0 && densify<NV>(reg, c, bump, end, ALLOC, true);
            dense_left -= ok ? 1u : 0u;
            ovf = ovf || !ok;
            if (ok) {
                uint32_t u, n;
                dense_find(reg + c.ext, v, ALLOC, h.z, u, n);
            }
        }
        if (en && c.dense != 0 && !ovf) {
            dense_add(reg + c.ext, v, kSubDelta, h.z);
            if (ALLOC && ins) reinterpret_cast<uint16_t*>(reg + c.ext + 288)[v] = static_cast<uint16_t>(newlink);
        }
    }
    h.link = newlink;
    c.len += ins ? 1u : 0u;
    nodes += ins ? 1u : 0u;
    c.esc += ins ? kSubEscDelta : 0u;
    const uint32_t tot = (c.tot + (ins ? kSubEscDelta : 0u) + kSubDelta) & 0xFFFF;
    c.tot = en ? tot : c.tot;
    ctx_rescale<NV>(reg, c, en && (h.cnt > 0xFF - 2 * kSubDelta || tot > kTotalLimit));
    return h;
}

// Decoder: the symbol whose interval [under, under + count) holds code
// (minimum 0), by halving on byte sums of the sorted counts
template <uint32_t NV>
DEV bool ctx_search(const uint8_t* reg, const Ctx<NV>& c, uint32_t code, bool links, Look<NV>& h, uint32_t& v)
{
    const uint32_t c0 = c.cnt[0], c1 = c.cnt[1], c2 = NV > 2 ? c.cnt[NV > 2 ? 2 : 0] : 0u, c3 = 0u;
    const uint32_t v0 = c.val[0], v1 = c.val[1], v2 = NV > 2 ? c.val[NV > 2 ? 2 : 0] : 0xFFFFFFFFu;
    uint32_t base = 0, j = 0, wa, wb, va, vb;
    if (NV > 2) {
        const uint32_t s = sad(c0, sad(c1, 0u));
        const bool hi = code >= s;
        base = hi ? s : 0u; j = hi ? 8u : 0u;
        wa = hi ? c2 : c0; wb = hi ? c3 : c1;
        va = hi ? v2 : v0; vb = hi ? 0xFFFFFFFFu : v1;
    } else {
        wa = c0; wb = c1; va = v0; vb = v1;
    }
    uint32_t s = sad(wa, 0u);
    bool hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 4u : 0u;
    uint32_t w = hi ? wb : wa, vw = hi ? vb : va;
    s = sad(w & 0xFFFFu, 0u);
    hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 2u : 0u;
    w = hi ? (w >> 16) : w; vw = hi ? (vw >> 16) : vw;
    s = w & 0xFFu;
    hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 1u : 0u;
    w = hi ? (w >> 8) : w; vw = hi ? (vw >> 8) : vw;
    h.k = j; h.under = base; h.cnt = w & 0xFFu; v = vw & 0xFFu;
    bool ok = h.cnt != 0 && code < base + h.cnt;
    h.link = links ? lnk_get<NV>(c, j) : 0u;
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) h.eq[d] = byte_mask(static_cast<int>(j), d) & 0x01010101u;
    if (any_lane(c.dense != 0)) {
        if (c.dense != 0) {
            uint32_t u, n, vv;
            ok = dense_search(reg + c.ext, code, links, h.z, vv, u, n);
            h.under = u; h.cnt = n; v = vv; h.link = h.z.link;
        }
    }
    h.found = ok;
    return ok;
}

// decoder hit at a sub-context: count[v] += 2, total += 2, rescale (compress.c:559-568)
template <uint32_t NV>
DEV void ctx_hit(uint8_t* reg, Ctx<NV>& c, Look<NV>& h, uint32_t v)
{
    if (c.dense == 0) {
#pragma unroll
        for (uint32_t d = 0; d < NV; ++d) c.cnt[d] += h.eq[d] << 1;
    }
    if (any_lane(c.dense != 0)) {
        if (c.dense != 0) dense_add(reg + c.ext, v, kSubDelta, h.z);
    }
    const uint32_t tot = (c.tot + kSubDelta) & 0xFFFF;
    c.tot = tot;
    ctx_rescale<NV>(reg, c, h.cnt > 0xFF - 2 * kSubDelta || tot > kTotalLimit);
}

// ------------------------------------------------------- byte streams (HBM)
// Each lane walks its own packet.  Byte-wide loads/stores would cost a 64-B
// sector transfer per byte (a lane's line is evicted between steps under
// 65536-way interleaving), so bytes move through 16-B register windows:
// one aligned dwordx4 load / store per 16 bytes; packet edges fall back to
// byte accesses so nothing outside [p, p+len) is read or written.

// Byte-stream addresses are integers (alignment arithmetic); accesses through
// them must name the global address space, otherwise they become flat_*
// operations, which complete out of order and force vmcnt(0) waits -- a full
// drain of every outstanding load and store, including the prefetches.
#ifndef RC_LANE_HOST_TEST
#define GPTR(T, a) ((__attribute__((address_space(1))) T*) (a))
#define GPTRC(T, a) ((const __attribute__((address_space(1))) T*) (a))
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
DEV uint4 gload16(uintptr_t a) { const v4u32 v = *GPTRC(v4u32, a); return make_uint4(v.x, v.y, v.z, v.w); }
DEV void gstore16(uintptr_t a, const uint4& w) { v4u32 v = {w.x, w.y, w.z, w.w}; *GPTR(v4u32, a) = v; }
#else
#define GPTR(T, a) ((T*) (a))
#define GPTRC(T, a) ((const T*) (a))
DEV uint4 gload16(uintptr_t a) { return *GPTRC(uint4, a); }
DEV void gstore16(uintptr_t a, const uint4& w) { *GPTR(uint4, a) = w; }
#endif

DEV uint32_t win_get(const uint4& w, uint32_t i) { return (pick4(i >> 2, w) >> (8 * (i & 3))) & 0xFF; }

DEV void win_set(uint4& w, uint32_t i, uint32_t b)
{
    const uint32_t sh = 8 * (i & 3), d = i >> 2, m = ~(0xFFu << sh), x = b << sh;
    w.x = d == 0 ? ((w.x & m) | x) : w.x;
    w.y = d == 1 ? ((w.y & m) | x) : w.y;
    w.z = d == 2 ? ((w.z & m) | x) : w.z;
    w.w = d == 3 ? ((w.w & m) | x) : w.w;
}

DEV uint4 chunk_load(const uint8_t* lo, const uint8_t* hi, uintptr_t c, bool en)
{
    const bool full = c >= reinterpret_cast<uintptr_t>(lo) && c + 16 <= reinterpret_cast<uintptr_t>(hi);
    uint4 w = make_uint4(0u, 0u, 0u, 0u);
    if (en && full) w = gload16(c);
    if (any_lane(en && !full)) {
        if (en && !full) {
            for (uint32_t t = 0; t < 16; ++t) {
                const uintptr_t a = c + t;
                if (a >= reinterpret_cast<uintptr_t>(lo) && a < reinterpret_cast<uintptr_t>(hi))
                    win_set(w, t, *GPTRC(uint8_t, a));
            }
        }
    }
    return w;
}

// sequential reader of [p, p+len); bytes past the end read as 0 (compress.c:366-367).
// Three 16-B chunks in flight: the chunk loaded when the reader advances is
// first read 16 bytes later, so no step waits on it.
struct InWin { const uint8_t* p; uint32_t len, pos; uint4 cur, nxt, fut; };

DEV void inwin_init(InWin& s, const uint8_t* p, uint32_t len)
{
    s.p = p; s.len = len; s.pos = 0;
    const uintptr_t c = reinterpret_cast<uintptr_t>(p) & ~static_cast<uintptr_t>(15);
    s.cur = chunk_load(p, p + len, c, true);
    s.nxt = chunk_load(p, p + len, c + 16, true);
    s.fut = chunk_load(p, p + len, c + 32, true);
    // settle these before the step loop: a load still pending at the loop
    // header makes the compiler wait for vmcnt(0) at the top of every step
    __builtin_amdgcn_s_waitcnt(0);   // (the builtin, which the waitcnt pass understands)
}

// next byte where `en` (0 past the end)
DEV uint32_t inwin_take(InWin& s, bool en)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(s.p) + s.pos;
    const bool live = en && s.pos < s.len;
    const uint32_t b = live ? win_get(s.cur, a & 15) : 0u;
    s.pos += live ? 1u : 0u;
    const bool adv = live && (a & 15) == 15;
    if (any_lane(adv)) {                  // advance; fetch the chunk three ahead
        // component-wise: a select of whole vectors is lowered through scratch
        s.cur.x = adv ? s.nxt.x : s.cur.x; s.cur.y = adv ? s.nxt.y : s.cur.y;
        s.cur.z = adv ? s.nxt.z : s.cur.z; s.cur.w = adv ? s.nxt.w : s.cur.w;
        s.nxt.x = adv ? s.fut.x : s.nxt.x; s.nxt.y = adv ? s.fut.y : s.nxt.y;
        s.nxt.z = adv ? s.fut.z : s.nxt.z; s.nxt.w = adv ? s.fut.w : s.nxt.w;
        // the load lands in `fut` directly; the rest of the step does not
        // read it, so only this (one-in-16) step waits for it
        const uintptr_t c = (a & ~static_cast<uintptr_t>(15)) + 48;
        const uintptr_t lo = reinterpret_cast<uintptr_t>(s.p), hi = lo + s.len;
        const bool full = c >= lo && c + 16 <= hi;
        if (adv && full) s.fut = gload16(c);
        if (any_lane(adv && !full)) {
            if (adv && !full) s.fut = chunk_load(s.p, s.p + s.len, c, true);
        }
    }
    return b;
}

struct OutWin { uint8_t* p; uint32_t cap, n; uint4 w; };

DEV void outwin_edge(uint8_t* p, uint32_t n, uintptr_t c, const uint4& w)
{
    for (uint32_t t = 0; t < 16; ++t) {
        const uintptr_t a = c + t;
        if (a >= reinterpret_cast<uintptr_t>(p) && a < reinterpret_cast<uintptr_t>(p) + n)
            *GPTR(uint8_t, a) = static_cast<uint8_t>(win_get(w, t));
    }
}

// append a byte where `en` (caller guarantees n < cap)
DEV void outwin_put(OutWin& o, uint32_t byte, bool en)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(o.p) + o.n;
    uint4 w = o.w;
    win_set(w, a & 15, byte);
    o.w.x = en ? w.x : o.w.x; o.w.y = en ? w.y : o.w.y;
    o.w.z = en ? w.z : o.w.z; o.w.w = en ? w.w : o.w.w;
    o.n += en ? 1u : 0u;
    const bool flush = en && (a & 15) == 15;
    if (any_lane(flush)) {
        const uintptr_t c = a & ~static_cast<uintptr_t>(15);
        const bool whole = c >= reinterpret_cast<uintptr_t>(o.p);
        if (flush && whole) gstore16(c, o.w);
        if (any_lane(flush && !whole)) {
            if (flush && !whole) outwin_edge(o.p, o.n, c, o.w);
        }
    }
}

DEV void outwin_finish(OutWin& o, bool en)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(o.p) + o.n - 1;
    if (en && o.n > 0 && (a & 15) != 15) outwin_edge(o.p, o.n, a & ~static_cast<uintptr_t>(15), o.w);
}

// ------------------------------------------------------------- range coder


// compress.c:121-137 where `en`; clears `ok` when the output is full (the
// whole compress call then returns 0, compress.c:116-117)
DEV void enc_code(uint32_t& low, uint32_t& range, uint32_t under, uint32_t count, uint32_t total,
                  OutWin& o, bool en, bool& ok)
{
    en = en && ok;
    const uint32_t r = udiv(range, en ? total : 1u);
    low = en ? low + under * r : low;
    range = en ? r * count : range;
    bool more = en;
    while (any_lane(more)) {
        const bool carry = (low ^ (low + range)) >= kTop;
        const bool stop = carry && range >= kBot;
        more = more && !stop;
        if (!any_lane(more)) break;
        range = (more && carry) ? ((0u - low) & (kBot - 1)) : range;
        const bool full = more && o.n >= o.cap;
        ok = ok && !full;
        more = more && !full;
        outwin_put(o, low >> 24, more);
        range = more ? range << 8 : range;
        low = more ? low << 8 : low;
    }
}

// compress.c:352 (truncated to u16 at :545/:575); divides range by total where `en`
DEV uint32_t dec_read(uint32_t& range, uint32_t low, uint32_t code, uint32_t total, bool en)
{
    const uint32_t r = udiv(range, en ? total : 1u);
    range = en ? r : range;
    return udiv(code - low, en ? r : 1u) & 0xFFFF;
}

// compress.c:354-371 where `en`
DEV void dec_code(uint32_t& low, uint32_t& code, uint32_t& range, uint32_t under, uint32_t count,
                  InWin& in, bool en)
{
    low = en ? low + under * range : low;
    range = en ? range * count : range;
    bool more = en;
    while (any_lane(more)) {
        const bool carry = (low ^ (low + range)) >= kTop;
        const bool stop = carry && range >= kBot;
        more = more && !stop;
        if (!any_lane(more)) break;
        range = (more && carry) ? ((0u - low) & (kBot - 1)) : range;
        const uint32_t b = inwin_take(in, more);
        code = more ? ((code << 8) | b) : code;
        range = more ? range << 8 : range;
        low = more ? low << 8 : low;
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
    if (any_lane((e & 0xFFFF) == 0)) {
        if ((e & 0xFFFF) == 0) {
            for (uint32_t x = 0; x < 256; ++x) *reinterpret_cast<uint32_t*>(reg + kO1Base + x * kO1Rec) = 0u;
            e += 1;
        }
    }
    *reinterpret_cast<uint32_t*>(reg) = e;
    return e;
}

DEV void compress_one(const rc_batch_dev& b, const rc_workspace_dev& ws, uint32_t pkt,
                      uint8_t* reg, uint8_t* root)
{
    const uint32_t len = b.in_len[pkt];
    const uint32_t cap = b.out_cap[pkt];
    if (len == 0) { b.out_len[pkt] = 0; return; }                   // compress.c:257
    InWin in;
    inwin_init(in, b.in + b.in_off[pkt], len);
    OutWin o = { b.out + b.out_off[pkt], cap, 0u, make_uint4(0u, 0u, 0u, 0u) };
    const uint32_t end = ws.lane_region;

    uint32_t epoch = next_epoch(reg, *reinterpret_cast<const uint32_t*>(reg));
    root_clear(root);
    uint32_t rtot = 1 + 256, bump = kArenaBase, nodes = 1, dense_left = kDenseBudget;
    uint32_t order = 0, b1 = 0;
    uint32_t low = 0, range = ~0u;
    bool ok = true, ovf = false;
    // software pipeline: the records of step i+1 are loaded during step i
    // (the next order-1 context is the current byte, known at the top of the
    // step; the next order-2 record once the order-1 lookup is done).
    Ctx1 r1;
    Ctx2 r2;
    ctx_empty(r1, kO1Base, epoch & 0xFFFF);
    ctx_empty(r2, 0u, 0u);

    PROF_DECL
    for (uint32_t i = 0; i < len; ++i) {
#ifdef RC_PROFILE_DRAIN
        __builtin_amdgcn_s_waitcnt(0);
        PROF(9)
#endif
        const uint32_t v = inwin_take(in, true);
        Raw1 n1;
        o1_fetch(reg, v, n1);                                       // next step's order-1 record
        const bool en2 = order >= 2;
        PROF(0)

        // order 2, compress.c:286-316
        const uint32_t esc2 = r2.esc, tot2 = r2.tot;
        const Look<kO2NV> h2 = ctx_update<kO2NV, false>(reg, r2, v, bump, end, nodes, dense_left, ovf, en2);
        const bool done2 = en2 && h2.found;
        PROF(1)
        enc_code(low, range, done2 ? esc2 + h2.under : 0u, done2 ? h2.cnt : esc2, tot2, o,
                 done2 || (en2 && esc2 > 0 && esc2 < tot2), ok);
        PROF(2)

        // order 1 (its lookup also yields the next order-2 record: the link of v)
        const bool en1 = !done2 && order >= 1;
        const uint32_t esc1 = r1.esc, tot1 = r1.tot;
        const Look<kO1NV> h1 = ctx_update<kO1NV, true>(reg, r1, v, bump, end, nodes, dense_left, ovf, en1);
        const bool done1 = en1 && h1.found;
        const uint32_t nxt = h1.link;
        const bool nfresh = en1 && !h1.found;
        PROF(3)
        enc_code(low, range, done1 ? esc1 + h1.under : 0u, done1 ? h1.cnt : esc1, tot1, o,
                 done1 || (en1 && esc1 > 0 && esc1 < tot1), ok);
        PROF(4)

        // next order-2 record: fresh, the one just updated, or a load
        const bool same2 = en2 && nxt * kO2Rec == r2.off;
        const bool ld2 = order >= 1 && !nfresh && !same2;
        Raw2 n2;
        if (ld2) o2_fetch(reg, nxt, n2);
        if (en1) o1_store(reg, r1);
        if (en2) o2_store(reg, r2);
        PROF(5)

        // root, compress.c:318-329
        const bool en0 = !done2 && !done1;
        uint32_t under0, cnt0;
        root_lookup(root, v, under0, cnt0);
        if (en0) root_add(root, v, cnt0);
        nodes += (en0 && cnt0 == 0) ? 1u : 0u;
        PROF(6)
        enc_code(low, range, 1 + under0, 1 + cnt0, rtot, o, en0, ok);
        rtot = en0 ? ((rtot + kRootDelta) & 0xFFFF) : rtot;
        const bool rs0 = en0 && (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit);
        if (any_lane(rs0)) { if (rs0) rtot = root_rescale(root); }
        PROF(7)

        if (any_lane(!ok || ovf)) { if (!ok || ovf) break; }

        // advance, compress.c:331-336
        if (order >= 1 && !same2) {
            if (ld2) o2_decode(n2, nxt, r2);
            else ctx_empty(r2, nxt * kO2Rec, 0u);
        }
        // the prefetched order-1 record is stale when it is the one this step updated
        if (!(en1 && v == b1)) o1_decode(n1, epoch & 0xFFFF, r1);
        order += order < 2 ? 1u : 0u;
        b1 = v;
        if (any_lane(nodes >= kMaxNodes)) {                          // compress.c:148-157
            if (nodes >= kMaxNodes) {
                epoch = next_epoch(reg, epoch);
                root_clear(root);
                rtot = 1 + 256; bump = kArenaBase; nodes = 1; order = 0; dense_left = kDenseBudget;
            }
        }
        PROF(8)
    }
    PROF_FLUSH(0)
    if (ovf) { flag_exact(ws, pkt); return; }
    // flush, compress.c:139-146
    while (any_lane(ok && low != 0)) {
        const bool more = ok && low != 0;
        const bool full = more && o.n >= o.cap;
        ok = ok && !full;
        outwin_put(o, low >> 24, more && !full);
        low = (more && !full) ? low << 8 : low;
    }
    outwin_finish(o, ok);
    b.out_len[pkt] = ok ? o.n : 0u;
}

// The decoder keeps data-dependent branches: unlike the encoder, each level's
// work (two divisions, a search) is only needed by the lanes that reach it.
DEV void decompress_one(const rc_batch_dev& b, const rc_workspace_dev& ws, uint32_t pkt,
                        uint8_t* reg, uint8_t* root)
{
    const uint32_t len = b.in_len[pkt];
    const uint32_t cap = b.out_cap[pkt];
    if (len == 0) { b.out_len[pkt] = 0; return; }                   // compress.c:513
    OutWin o = { b.out + b.out_off[pkt], cap, 0u, make_uint4(0u, 0u, 0u, 0u) };
    const uint32_t end = ws.lane_region;
    InWin in;
    inwin_init(in, b.in + b.in_off[pkt], len);

    uint32_t epoch = next_epoch(reg, *reinterpret_cast<const uint32_t*>(reg));
    root_clear(root);
    uint32_t rtot = 1 + 256, bump = kArenaBase, nodes = 1, dense_left = kDenseBudget;
    uint32_t order = 0, b1 = 0;
    uint32_t low = 0, code = 0, range = ~0u;
    for (int k = 0; k < 4; ++k) code = (code << 8) | inwin_take(in, true);   // compress.c:344-350
    bool fail = false, anomaly = false, ovf = false;
    // the next step's records are loaded as soon as the symbol is decoded
    Ctx1 r1;
    Ctx2 r2;
    ctx_empty(r1, kO1Base, epoch & 0xFFFF);
    ctx_empty(r2, 0u, 0u);

    PROF_DECL
    for (;;) {
        PROF(11)
#ifdef RC_PROFILE_DRAIN
        __builtin_amdgcn_s_waitcnt(0);
        PROF(8)
#endif
        int at = -1;                         // context that produced the symbol (2, 1, 0)
        uint32_t v = 0, nxt = 0;
        bool nfresh = false;

        if (order >= 2 && r2.esc > 0) {                              // compress.c:529-568
            const uint32_t tot = r2.tot;
            if (r2.esc < tot) {
                range = udiv(range, tot);
                uint32_t cd = udiv(code - low, range) & 0xFFFF;
                if (cd < r2.esc) {
                    dec_code(low, code, range, 0, r2.esc, in, true);
                } else {
                    Look<kO2NV> h;
                    if (!ctx_search<kO2NV>(reg, r2, cd - r2.esc, false, h, v)) { fail = true; break; }
                    dec_code(low, code, range, r2.esc + h.under, h.cnt, in, true);
                    ctx_hit<kO2NV>(reg, r2, h, v);
                    at = 2;
                }
            }
        }
        PROF(0)
        if (at < 0 && order >= 1 && r1.esc > 0) {
            const uint32_t tot = r1.tot;
            if (r1.esc < tot) {
                range = udiv(range, tot);
                uint32_t cd = udiv(code - low, range) & 0xFFFF;
                if (cd < r1.esc) {
                    dec_code(low, code, range, 0, r1.esc, in, true);
                } else {
                    Look<kO1NV> h;
                    if (!ctx_search<kO1NV>(reg, r1, cd - r1.esc, true, h, v)) { fail = true; break; }
                    dec_code(low, code, range, r1.esc + h.under, h.cnt, in, true);
                    ctx_hit<kO1NV>(reg, r1, h, v);
                    nxt = h.link;
                    at = 1;
                }
            }
        }
        PROF(1)
        if (at < 0) {                                                // root, compress.c:570-596
            range = udiv(range, rtot);
            uint32_t cd = udiv(code - low, range) & 0xFFFF;
            if (cd < 1) { dec_code(low, code, range, 0, 1, in, true); break; }   // end of stream
            cd -= 1;
            if (cd >= rtot - 1) { anomaly = true; break; }          // past symbol 255
            uint32_t under, cnt;
            v = root_search(root, cd, under, cnt);
            if (cnt == 0) ++nodes;
            root_add(root, v, cnt);
            dec_code(low, code, range, 1 + under, 1 + cnt, in, true);
            rtot = (rtot + kRootDelta) & 0xFFFF;
            if (1 + cnt > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit) rtot = root_rescale(root);
            at = 0;
        }
        PROF(2)
        Raw1 n1;
        o1_fetch(reg, v, n1);                                       // next step's order-1 record
        PROF(3)
        // patch the contexts above, compress.c:598-615
        if (order >= 2 && at < 2) {
            ctx_update<kO2NV, false>(reg, r2, v, bump, end, nodes, dense_left, ovf, true);
            if (ovf) break;
        }
        PROF(4)
        if (order >= 1 && at < 1) {
            const Look<kO1NV> h = ctx_update<kO1NV, true>(reg, r1, v, bump, end, nodes, dense_left, ovf, true);
            if (ovf) break;
            nxt = h.link;
            nfresh = !h.found;
        }
        if (order >= 1 && at == 2) nxt = ctx_find<kO1NV>(reg, r1, v, true).link;   // (prev, v) via o1[prev]
        PROF(5)
        const bool same2 = order >= 2 && nxt * kO2Rec == r2.off;
        const bool ld2 = order >= 1 && !nfresh && !same2;
        Raw2 n2;
        if (ld2) o2_fetch(reg, nxt, n2);
        if (order >= 2) o2_store(reg, r2);
        if (order >= 1 && at <= 1) o1_store(reg, r1);
        PROF(6)
        if (o.n >= o.cap) { fail = true; break; }                    // compress.c:617
        outwin_put(o, v, true);
        PROF(7)
        if (order >= 1 && !same2) {
            if (ld2) o2_decode(n2, nxt, r2);
            else ctx_empty(r2, nxt * kO2Rec, 0u);
        }
        if (!(order >= 1 && v == b1)) o1_decode(n1, epoch & 0xFFFF, r1);
        if (order < 2) ++order;
        b1 = v;
        if (any_lane(nodes >= kMaxNodes)) {
            if (nodes >= kMaxNodes) {
                epoch = next_epoch(reg, epoch);
                root_clear(root);
                rtot = 1 + 256; bump = kArenaBase; nodes = 1; order = 0; dense_left = kDenseBudget;
            }
        }
    }
    PROF_FLUSH(16)
    if (ovf || anomaly) { flag_exact(ws, pkt); return; }
    outwin_finish(o, !fail);
    b.out_len[pkt] = fail ? 0u : o.n;
}

}  // namespace

#ifdef RC_PROFILE
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

extern "C" uint32_t rc_hip_lane_region_bytes(uint32_t max_len)
{
    // header + order-1 table + one 32-B order-2 record per o1 symbol (<= one
    // per byte between resets) + dense blocks: a dense context holds > 8
    // symbols, i.e. > 8 of the <= 2L + 256 (<= 4094) nodes between resets,
    // and takes <= 800 B, so <= 89 B per node covers any input.
    const uint64_t L = max_len < 4096 ? max_len : 4096;
    const uint64_t nodes = 2 * L + 256 < 4094 ? 2 * L + 256 : 4094;
    uint64_t bytes = kArenaBase + kO2Rec * (L + 1) + 89 * nodes + 1024;
    bytes = (bytes + 255) & ~255ull;
    return static_cast<uint32_t>(bytes);
}

#ifndef RC_LANE_HOST_TEST
// Lane mapping: a workgroup is 4 wavefronts; the first `act` lanes of each
// wavefront own one packet each (act = 64 by default; 32/16 trade VALU
// efficiency for more resident waves per SIMD to overlap HBM latency).
template <bool DECOMP>
DEV void lane_main(const rc_batch_dev& b, const rc_workspace_dev& ws)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t act = ws.lane_active;
    const uint32_t wave = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l >= act) return;
    const uint32_t local = wave * act + l;
    uint8_t* root = smem + local * kRootStride;
    const uint32_t per_block = 4 * act;
    const uint32_t slot = blockIdx.x * per_block + local;
    uint8_t* reg = static_cast<uint8_t*>(ws.lane_pool) + static_cast<size_t>(slot) * ws.lane_region;
    const uint32_t* order = ws.order && !ws.bins[RC_LEN_BINS] ? ws.order : nullptr;
    for (uint32_t i = slot; i < b.n; i += gridDim.x * per_block) {
        const uint32_t pkt = order ? order[i] : i;
        if (DECOMP) decompress_one(b, ws, pkt, reg, root);
        else compress_one(b, ws, pkt, reg, root);
    }
}

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

constexpr uint32_t kBinChunk = 4096;     // packets per binning workgroup (16 per thread)

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

extern "C" __global__ __launch_bounds__(256) void rc_len_hist(const uint32_t* len, uint32_t n, uint32_t* bins)
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

// Exclusive prefix over the bins; bins[RC_LEN_BINS] = 1 when every packet
// falls in one bin (uniform lengths: the lane kernels then keep batch order).
extern "C" __global__ __launch_bounds__(RC_LEN_BINS) void rc_len_scan(uint32_t* bins)
{
    __shared__ uint32_t s[RC_LEN_BINS];
    const uint32_t t = threadIdx.x;
    const uint32_t mine = bins[t];
    s[t] = mine;
    const int used = __syncthreads_count(mine != 0);
    for (uint32_t d = 1; d < RC_LEN_BINS; d <<= 1) {
        const uint32_t x = t >= d ? s[t - d] : 0u;
        __syncthreads();
        s[t] += x;
        __syncthreads();
    }
    bins[t] = s[t] - mine;               // exclusive prefix = first slot of the bin
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

extern "C" __global__ __launch_bounds__(256)
void rc_compress_lane(rc_batch_dev b, rc_workspace_dev ws) { lane_main<false>(b, ws); }

extern "C" __global__ __launch_bounds__(256)
void rc_decompress_lane(rc_batch_dev b, rc_workspace_dev ws) { lane_main<true>(b, ws); }

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
    const size_t lds = static_cast<size_t>(per_block) * kRootStride;
    rc_workspace_dev w = *ws;
    w.order = nullptr;
    if (b->n >= 1024 && ws->order && ws->bins) {        // bin packets by length (ragged batches)
        hipError_t e = hipMemsetAsync(ws->bins, 0, (RC_LEN_BINS + 1) * sizeof(uint32_t), st);
        if (e != hipSuccess) return static_cast<int>(e);
        const uint32_t g = (b->n + kBinChunk - 1) / kBinChunk;
        hipLaunchKernelGGL(rc_len_hist, dim3(g), dim3(256), 0, st, b->in_len, b->n, ws->bins);
        hipLaunchKernelGGL(rc_len_scan, dim3(1), dim3(RC_LEN_BINS), 0, st, ws->bins);
        hipLaunchKernelGGL(rc_len_scatter, dim3(g), dim3(256), 0, st, b->in_len, b->n, ws->bins, ws->order);
        w.order = ws->order;
    }
    if (decompress)
        hipLaunchKernelGGL(rc_decompress_lane, dim3(blocks), dim3(256), lds, st, *b, w);
    else
        hipLaunchKernelGGL(rc_compress_lane, dim3(blocks), dim3(256), lds, st, *b, w);
    return static_cast<int>(hipGetLastError());
}
#endif  // RC_LANE_HOST_TEST
