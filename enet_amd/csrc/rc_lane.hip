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
// Model layout (only {count[v], escapes, total} per context and the node
// count are observable):
//   order 0 (root): per lane in LDS, counts[256] (u8) + C[16] (u16 cumulative
//       count at the end of each 16-symbol group) -> lookups are 1-2 LDS
//       reads + byte-SAD sums, no tree walk.
//   order 1: 256 records of 64 B, direct-mapped by the previous byte, in a
//       per-lane HBM region; order 2: 8-B records bump-allocated in the same
//       region, reached through links stored in the entries (compress.c's
//       suffix links, `parent`).  Entries are sorted {value | count | link};
//       contexts that outgrow their inline slots use an extension block.
//   Each byte costs one HBM round trip, and that load is issued a step ahead.
//
// Code shape: 64 lanes run 64 different packets, so every `if` on per-lane
// data is divergent.  Common paths are written as straight-line predicated
// register code; rare paths (extension blocks, growth, rescale, packet edges,
// model reset) sit behind wave-uniform ballot guards so a wave that does not
// need them pays one scalar branch.
//
// Packets this model cannot reproduce -- corrupt streams whose root code
// points past symbol 255 (compress.c:427-438 then depends on tree shape) --
// and packets whose region overflows are appended to the exact-path list
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
    const uint4 q = *reinterpret_cast<const uint4*>(r + 16 * g);
    uint32_t run = 16 * g + prev, j = 15, at = run, c = 0;
    bool found = false;
#pragma unroll
    for (uint32_t t = 0; t < 16; ++t) {
        const uint32_t ct = (pick4(t >> 2, q) >> (8 * (t & 3))) & 0xFF;
        const uint32_t nrun = run + 1 + ct;
        const bool hit = !found && code < nrun;
        j = hit ? t : j;
        at = hit ? run : at;
        c = hit ? ct : c;
        found = found || hit;
        run = nrun;
    }
    under = at;
    cnt = c;
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

// ---------------------------------------------------- order 1/2 records (HBM)
// Both record kinds start with the same two words:
//     w0 = esc | len << 16,  w1 = ext / 16 | total << 16
// (ext = extension block offset, 0 while the entries are inline; total =
// esc + sum(counts) mod 2^16, maintained like compress.c's (:309-312, rescale
// :107-112), so no lookup has to sum the counts).
// o1 record, 64 B, direct-mapped by the context byte: header + 14 inline entries.
// o2 record, 16 B, bump-allocated so that the records touched by consecutive
//     steps share HBM sectors: header + 2 inline entries.
// entry = value | count << 8 | link << 16, link = o2 record index (offset / 16):
//     in an o1 entry the context (prev, value); in an o2 entry the suffix
//     context (compress.c's `parent`, :294-295, :615).
// A freshly allocated o2 record is never zero-filled or loaded: its first
// visit is the very next step, which knows it is empty.

constexpr uint32_t kO1Rec = 64, kO1Inl = 14, kO1MinCap = 32;
constexpr uint32_t kO2Rec = 16, kO2Inl = 2, kO2MinCap = 4;
constexpr uint32_t kArenaBase = 256 * kO1Rec;

template <uint32_t INL>
struct Rec { uint32_t off, esc, len, ext, tot; uint32_t e[INL]; };

DEV uint32_t hdr_w1(uint32_t ext, uint32_t tot) { return (ext >> 4) | (tot << 16); }

struct Hit { uint32_t k, under, cnt, link, val, tot; bool found; };

DEV uint32_t cap_for(uint32_t len, uint32_t mincap)
{
    return len <= mincap ? mincap : (1u << (32 - __builtin_clz(len - 1)));
}

DEV void o1_load(const uint8_t* reg, uint32_t x, Rec<kO1Inl>& r)
{
    const uint4* p = reinterpret_cast<const uint4*>(reg + x * kO1Rec);
    const uint4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
    r.off = x * kO1Rec; r.esc = q0.x & 0xFFFF; r.len = q0.x >> 16;
    r.ext = (q0.y & 0xFFFF) << 4; r.tot = q0.y >> 16;
    r.e[0] = q0.z; r.e[1] = q0.w;
    r.e[2] = q1.x; r.e[3] = q1.y; r.e[4] = q1.z; r.e[5] = q1.w;
    r.e[6] = q2.x; r.e[7] = q2.y; r.e[8] = q2.z; r.e[9] = q2.w;
    r.e[10] = q3.x; r.e[11] = q3.y; r.e[12] = q3.z; r.e[13] = q3.w;
}

// in ext mode the inline slots are dead, so they are written unconditionally
DEV void o1_store(uint8_t* reg, const Rec<kO1Inl>& r)
{
    uint4* p = reinterpret_cast<uint4*>(reg + r.off);
    p[0] = make_uint4(r.esc | (r.len << 16), hdr_w1(r.ext, r.tot), r.e[0], r.e[1]);
    p[1] = make_uint4(r.e[2], r.e[3], r.e[4], r.e[5]);
    p[2] = make_uint4(r.e[6], r.e[7], r.e[8], r.e[9]);
    p[3] = make_uint4(r.e[10], r.e[11], r.e[12], r.e[13]);
}

DEV void o2_load(const uint8_t* reg, uint32_t idx, Rec<kO2Inl>& r)
{
    const uint4 q = *reinterpret_cast<const uint4*>(reg + idx * kO2Rec);
    r.off = idx * kO2Rec; r.esc = q.x & 0xFFFF; r.len = q.x >> 16;
    r.ext = (q.y & 0xFFFF) << 4; r.tot = q.y >> 16;
    r.e[0] = q.z; r.e[1] = q.w;
}

DEV void o2_fresh(uint32_t idx, Rec<kO2Inl>& r)
{
    r.off = idx * kO2Rec; r.esc = 0; r.len = 0; r.ext = 0; r.tot = 0; r.e[0] = 0; r.e[1] = 0;
}

DEV void o2_store(uint8_t* reg, const Rec<kO2Inl>& r)
{
    *reinterpret_cast<uint4*>(reg + r.off) = make_uint4(r.esc | (r.len << 16), hdr_w1(r.ext, r.tot), r.e[0], r.e[1]);
}

// Extension blocks are read and written 16 entries (four 16-B chunks) at a
// time: the four loads are in flight together, so a context of n entries costs
// ceil(n / 16) memory round trips instead of one per chunk or per entry.
constexpr uint32_t kGrp = 16;

DEV void grp_load(const uint32_t* ep, uint32_t g0, uint32_t n, uint4 (&q)[4])
{
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
        q[j] = g0 + 4 * j < n ? *reinterpret_cast<const uint4*>(ep + g0 + 4 * j) : make_uint4(0u, 0u, 0u, 0u);
}

DEV uint32_t grp_get(const uint4 (&q)[4], uint32_t i) { return pick4(i & 3, q[i >> 2]); }

// Encoder-side lookup of v (compress.c:159-199, minimum 0): k = first entry >= v,
// under = counts below, found/cnt/link, tot = esc + all counts (before update).
template <uint32_t INL>
DEV Hit rec_find(const uint8_t* reg, const Rec<INL>& r, uint32_t v)
{
    Hit h = { 0u, 0u, 0u, 0u, v, 0u, false };
    uint32_t sum = 0;
    const uint32_t ilen = r.ext == 0 ? r.len : 0u;
#pragma unroll
    for (uint32_t t = 0; t < INL; ++t) {
        const uint32_t e = r.e[t];
        const bool in = t < ilen;
        const uint32_t c = in ? cnt_of(e) : 0u;
        const bool lt = in && val_of(e) < v;
        const bool eq = in && val_of(e) == v;
        sum += c;
        h.under += lt ? c : 0u;
        h.k += lt ? 1u : 0u;
        h.found = h.found || eq;
        h.cnt = eq ? c : h.cnt;
        h.link = eq ? (e >> 16) : h.link;
    }
    if (any_lane(r.ext != 0)) {
        if (r.ext != 0) {
            const uint32_t* ep = reinterpret_cast<const uint32_t*>(reg + r.ext);
            for (uint32_t g0 = 0; g0 < r.len; g0 += kGrp) {
                uint4 q[4];
                grp_load(ep, g0, r.len, q);
#pragma unroll
                for (uint32_t t = 0; t < kGrp; ++t) {
                    const uint32_t e = grp_get(q, t);
                    const bool in = g0 + t < r.len;
                    const uint32_t c = in ? cnt_of(e) : 0u;
                    const bool lt = in && val_of(e) < v;
                    const bool eq = in && val_of(e) == v;
                    sum += c;
                    h.under += lt ? c : 0u;
                    h.k += lt ? 1u : 0u;
                    h.found = h.found || eq;
                    h.cnt = eq ? c : h.cnt;
                    h.link = eq ? (e >> 16) : h.link;
                }
            }
        }
    }
    (void) sum;
    h.tot = r.tot;
    return h;
}

template <uint32_t INL>
DEV uint32_t rec_total(const uint8_t*, const Rec<INL>& r) { return r.tot; }

// Decoder search (compress.c:373-416, minimum 0) where `en`: entry whose
// interval holds code.  Returns false (corrupt stream) when none does.
template <uint32_t INL>
DEV Hit rec_search(const uint8_t* reg, const Rec<INL>& r, uint32_t code, bool en)
{
    Hit h = { 0u, 0u, 0u, 0u, 0u, 0u, false };
    uint32_t cum = 0;
    bool found = false;
    const uint32_t ilen = (en && r.ext == 0) ? r.len : 0u;
#pragma unroll
    for (uint32_t t = 0; t < INL; ++t) {
        const uint32_t e = r.e[t];
        const bool in = t < ilen;
        const uint32_t c = in ? cnt_of(e) : 0u;
        const bool hit = in && !found && code < cum + c;
        h.k = hit ? t : h.k; h.under = hit ? cum : h.under; h.cnt = hit ? c : h.cnt;
        h.link = hit ? (e >> 16) : h.link; h.val = hit ? val_of(e) : h.val;
        found = found || hit;
        cum += c;
    }
    if (any_lane(en && r.ext != 0)) {
        if (en && r.ext != 0) {
            const uint32_t* ep = reinterpret_cast<const uint32_t*>(reg + r.ext);
            for (uint32_t g0 = 0; g0 < r.len && !found; g0 += kGrp) {
                uint4 q[4];
                grp_load(ep, g0, r.len, q);
#pragma unroll
                for (uint32_t t = 0; t < kGrp; ++t) {
                    const uint32_t e = grp_get(q, t);
                    const bool in = g0 + t < r.len;
                    const uint32_t c = in ? cnt_of(e) : 0u;
                    const bool hit = in && !found && code < cum + c;
                    h.k = hit ? g0 + t : h.k; h.under = hit ? cum : h.under; h.cnt = hit ? c : h.cnt;
                    h.link = hit ? (e >> 16) : h.link; h.val = hit ? val_of(e) : h.val;
                    found = found || hit;
                    cum += c;
                }
            }
        }
    }
    h.found = found;
    return h;
}

// count[k] = cnt + d where `en`
template <uint32_t INL>
DEV void rec_bump(uint8_t* reg, Rec<INL>& r, uint32_t k, uint32_t cnt, uint32_t d, bool en)
{
    const bool inl = en && r.ext == 0;
#pragma unroll
    for (uint32_t t = 0; t < INL; ++t) r.e[t] += (inl && t == k) ? (d << 8) : 0u;
    if (any_lane(en && r.ext != 0)) {
        if (en && r.ext != 0) reg[r.ext + 4 * k + 1] = static_cast<uint8_t>(cnt + d);
    }
}

DEV void grp_put(uint4 (&o)[4], uint32_t i, uint32_t x)
{
    uint4& c = o[i >> 2];
    switch (i & 3) { case 0: c.x = x; break; case 1: c.y = x; break; case 2: c.z = x; break; default: c.w = x; }
}

// dst[j], j in [0, n]: src[j] below k, ne at k, src[j-1] above k (src holds n
// entries; the block holding dst has room for n + 1, rounded up to 4).  In
// place (dst == src) the groups below k are not touched.  A group's stores
// never reach the next group's entries, so they can precede its loads.
DEV void ext_shift_insert(uint32_t* dst, const uint32_t* src, uint32_t n, uint32_t k, uint32_t ne, bool inplace)
{
    uint32_t carry = 0;
    for (uint32_t g0 = inplace ? (k & ~(kGrp - 1)) : 0u; g0 <= n; g0 += kGrp) {
        uint4 q[4], o[4];
        grp_load(src, g0, n, q);
#pragma unroll
        for (uint32_t t = 0; t < kGrp; ++t) {
            const uint32_t j = g0 + t;
            const uint32_t prev = t == 0 ? carry : grp_get(q, t - 1);
            grp_put(o, t, j < k ? grp_get(q, t) : (j == k ? ne : prev));
        }
        carry = grp_get(q, kGrp - 1);
#pragma unroll
        for (uint32_t c = 0; c < 4; ++c)
            if (g0 + 4 * c <= n) *reinterpret_cast<uint4*>(dst + g0 + 4 * c) = o[c];
    }
}

// Insert entry `ne` at position k where `en`; moves to / grows an extension
// block when the inline slots or the block are full.  false = region full.
template <uint32_t INL, uint32_t MINCAP>
DEV bool rec_insert(uint8_t* reg, Rec<INL>& r, uint32_t k, uint32_t ne, uint32_t& bump, uint32_t end, bool en)
{
    const bool fast = en && r.ext == 0 && r.len < INL;
#pragma unroll
    for (int t = INL - 1; t >= 0; --t) {
        const uint32_t prev = t > 0 ? r.e[t > 0 ? t - 1 : 0] : 0u;
        const uint32_t shifted = (static_cast<uint32_t>(t) > k) ? prev
                               : (static_cast<uint32_t>(t) == k ? ne : r.e[t]);
        r.e[t] = fast ? shifted : r.e[t];
    }
    bool ok = true;
    if (any_lane(en && !fast)) {
        if (en && !fast) {
            const uint32_t cap = r.ext ? cap_for(r.len, MINCAP) : INL;
            if (r.ext != 0 && r.len < cap) {
                uint32_t* ep = reinterpret_cast<uint32_t*>(reg + r.ext);
                ext_shift_insert(ep, ep, r.len, k, ne, true);
            } else {
                const uint32_t ncap = r.ext ? 2 * cap : MINCAP;
                const uint32_t at = (bump + 15) & ~15u;
                if (at + 4 * ncap > end) {
                    ok = false;
                } else {
                    uint32_t* np = reinterpret_cast<uint32_t*>(reg + at);
                    if (r.ext == 0) {
#pragma unroll
                        for (uint32_t t = 0; t < INL; ++t) np[t + (t >= k ? 1u : 0u)] = r.e[t];
                        np[k] = ne;
                    } else {
                        const uint32_t* ep = reinterpret_cast<const uint32_t*>(reg + r.ext);
                        ext_shift_insert(np, ep, r.len, k, ne, false);
                    }
                    r.ext = at;
                    bump = at + 4 * ncap;
                }
            }
        }
    }
    r.len += (en && ok) ? 1u : 0u;
    return ok;
}

// Link of entry k where `en` (an o2 entry created before its suffix context was known).
template <uint32_t INL>
DEV void rec_set_link(uint8_t* reg, Rec<INL>& r, uint32_t k, uint32_t link, bool en)
{
    const bool inl = en && r.ext == 0;
#pragma unroll
    for (uint32_t t = 0; t < INL; ++t)
        r.e[t] = (inl && t == k) ? ((r.e[t] & 0xFFFFu) | (link << 16)) : r.e[t];
    if (any_lane(en && r.ext != 0)) {
        if (en && r.ext != 0) *reinterpret_cast<uint16_t*>(reg + r.ext + 4 * k + 2) = static_cast<uint16_t>(link);
    }
}

// compress.c:90-112 on a record, where `en`
template <uint32_t INL>
DEV void rec_rescale(uint8_t* reg, Rec<INL>& r, bool en)
{
    if (!any_lane(en)) return;
    const bool inl = en && r.ext == 0;
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t t = 0; t < INL; ++t) {
        const uint32_t e = r.e[t];
        uint32_t c = cnt_of(e);
        c -= c >> 1;
        const bool live = inl && t < r.len;
        r.e[t] = live ? ((e & 0xFFFF00FFu) | (c << 8)) : e;
        sum += live ? c : 0u;
    }
    if (en && r.ext != 0) {
        uint32_t* ep = reinterpret_cast<uint32_t*>(reg + r.ext);
        for (uint32_t g0 = 0; g0 < r.len; g0 += kGrp) {
            uint4 q[4];
            grp_load(ep, g0, r.len, q);
#pragma unroll
            for (uint32_t t = 0; t < kGrp; ++t) {
                const uint32_t e = grp_get(q, t);
                const uint32_t c = cnt_of(e) - (cnt_of(e) >> 1);
                grp_put(q, t, (e & 0xFFFF00FFu) | (c << 8));
                sum += g0 + t < r.len ? c : 0u;
            }
#pragma unroll
            for (uint32_t c = 0; c < 4; ++c)
                if (g0 + 4 * c < r.len) *reinterpret_cast<uint4*>(ep + g0 + 4 * c) = q[c];
        }
    }
    r.esc -= en ? (r.esc >> 1) : 0u;
    r.tot = en ? ((r.esc + sum) & 0xFFFF) : r.tot;                  // compress.c:107-112
}

// Encoder-side update of a sub-context where `en` (compress.c:293-314, patch
// :603-613): find or insert v.  Returns the hit: old count (0 if new), cum
// below, total before the update, and the entry's link.  ALLOC: an inserted
// entry gets a fresh o2 record (order-1 contexts); otherwise its link is set
// later with rec_set_link (order-2 contexts).
template <uint32_t INL, uint32_t MINCAP, bool ALLOC>
DEV Hit sub_update(uint8_t* reg, Rec<INL>& r, uint32_t v, uint32_t& bump,
                   uint32_t end, uint32_t& nodes, bool& ovf, bool en)
{
    Hit h = rec_find(reg, r, v);
    const bool ins = en && !h.found;
    rec_bump(reg, r, h.k, h.cnt, kSubDelta, en && h.found);
    uint32_t newlink = 0;
    if (ALLOC) {
        newlink = bump / kO2Rec;
        bump += ins ? kO2Rec : 0u;
        if (ins && bump > end) ovf = true;
    }
    const bool ok = rec_insert<INL, MINCAP>(reg, r, h.k, v | (kSubDelta << 8) | (newlink << 16),
                                            bump, end, ins);
    ovf = ovf || !ok;
    h.link = ins ? newlink : h.link;
    nodes += ins ? 1u : 0u;
    r.esc += ins ? kSubEscDelta : 0u;
    const uint32_t tot = (h.tot + (ins ? kSubEscDelta : 0u) + kSubDelta) & 0xFFFF;
    r.tot = en ? tot : r.tot;
    rec_rescale(reg, r, en && (h.cnt > 0xFF - 2 * kSubDelta || tot > kTotalLimit));
    return h;
}

DEV void region_reset(uint8_t* reg, uint8_t* root)
{
    root_clear(root);
    for (uint32_t x = 0; x < 256; ++x) *reinterpret_cast<uint2*>(reg + x * kO1Rec) = make_uint2(0u, 0u);
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

DEV void rec_clear(Rec<kO1Inl>& r1)
{
    r1.off = 0; r1.esc = 0; r1.len = 0; r1.ext = 0; r1.tot = 0;
#pragma unroll
    for (uint32_t t = 0; t < kO1Inl; ++t) r1.e[t] = 0;
}

// ------------------------------------------------------------ one packet

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

    region_reset(reg, root);
    uint32_t rtot = 1 + 256, bump = kArenaBase, nodes = 1;
    uint32_t order = 0, b1 = 0;
    uint32_t low = 0, range = ~0u;
    bool ok = true, ovf = false;
    // software pipeline: the records of step i+1 are loaded during step i
    // (the next order-1 context is the current byte, known at the top of the
    // step; the next order-2 context once the current contexts are resolved).
    Rec<kO1Inl> r1;
    Rec<kO2Inl> r2;
    o2_fresh(0, r2);
    rec_clear(r1);

    PROF_DECL
    for (uint32_t i = 0; i < len; ++i) {
#ifdef RC_PROFILE_DRAIN
        __builtin_amdgcn_s_waitcnt(0);       // diagnostic: charge outstanding memory to slot 9
        PROF(9)
#endif
        const uint32_t v = inwin_take(in, true);
        Rec<kO1Inl> n1;
        o1_load(reg, v, n1);                                         // next step's order-1 record
        Rec<kO2Inl> n2;
        const bool en2 = order >= 2;
        PROF(0)

        // order 2, compress.c:286-316
        const uint32_t esc2 = r2.esc;
        const Hit h2 = sub_update<kO2Inl, kO2MinCap, false>(reg, r2, v, bump, end, nodes, ovf, en2);
        const bool done2 = en2 && h2.found;
        PROF(1)
        enc_code(low, range, done2 ? esc2 + h2.under : 0u, done2 ? h2.cnt : esc2, h2.tot, o,
                 done2 || (en2 && esc2 > 0 && esc2 < h2.tot), ok);
        PROF(2)
        const bool pend = en2 && !h2.found;
        uint32_t nxt = h2.link;

        // order 1
        const bool en1 = !done2 && order >= 1;
        const uint32_t esc1 = r1.esc;
        const Hit h1 = sub_update<kO1Inl, kO1MinCap, true>(reg, r1, v, bump, end, nodes, ovf, en1);
        const bool done1 = en1 && h1.found;
        nxt = en1 ? h1.link : nxt;
        const bool nfresh = en1 && !h1.found;
        rec_set_link(reg, r2, h2.k, nxt, pend);
        PROF(3)
        enc_code(low, range, done1 ? esc1 + h1.under : 0u, done1 ? h1.cnt : esc1, h1.tot, o,
                 done1 || (en1 && esc1 > 0 && esc1 < h1.tot), ok);
        PROF(4)

        // next order-2 record: fresh, the one just updated, or a load
        const bool same2 = en2 && nxt * kO2Rec == r2.off;
        o2_fresh(0, n2);
        if (order >= 1 && !nfresh && !same2) o2_load(reg, nxt, n2);
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
        if (order >= 1) {
            if (nfresh) o2_fresh(nxt, n2);
            else if (same2) n2 = r2;
            r2 = n2;
        }
        // the prefetched order-1 record is stale when it is the one this step updated
        if (!(en1 && v == b1)) r1 = n1;
        order += order < 2 ? 1u : 0u;
        b1 = v;
        if (any_lane(nodes >= kMaxNodes)) {                          // compress.c:148-157
            if (nodes >= kMaxNodes) {
                region_reset(reg, root);
                rtot = 1 + 256; bump = kArenaBase; nodes = 1; order = 0;
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

DEV void rec2_copy(Rec<kO2Inl>& d, const Rec<kO2Inl>& r)
{
    d.off = r.off; d.esc = r.esc; d.len = r.len; d.ext = r.ext; d.tot = r.tot; d.e[0] = r.e[0]; d.e[1] = r.e[1];
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

    region_reset(reg, root);
    uint32_t rtot = 1 + 256, bump = kArenaBase, nodes = 1;
    uint32_t order = 0, b1 = 0;
    uint32_t low = 0, code = 0, range = ~0u;
    for (int k = 0; k < 4; ++k) code = (code << 8) | inwin_take(in, true);   // compress.c:344-350
    bool fail = false, anomaly = false, ovf = false;
    // the next step's records are loaded as soon as the symbol is decoded
    Rec<kO1Inl> r1;
    Rec<kO2Inl> r2;
    o2_fresh(0, r2);
    rec_clear(r1);

    PROF_DECL
    for (;;) {
        PROF(11)
#ifdef RC_PROFILE_DRAIN
        __builtin_amdgcn_s_waitcnt(0);       // diagnostic: charge outstanding memory to slot 8
        PROF(8)
#endif
        int at = -1;                         // context that produced the symbol (2, 1, 0)
        uint32_t v = 0, nxt = 0;
        bool nfresh = false;

        if (order >= 2 && r2.esc > 0) {                              // compress.c:529-568
            const uint32_t tot = rec_total(reg, r2);
            if (r2.esc < tot) {
                range = udiv(range, tot);
                uint32_t cd = udiv(code - low, range) & 0xFFFF;
                if (cd < r2.esc) {
                    dec_code(low, code, range, 0, r2.esc, in, true);
                } else {
                    const Hit h = rec_search(reg, r2, cd - r2.esc, true);
                    if (!h.found) { fail = true; break; }
                    v = h.val;
                    rec_bump(reg, r2, h.k, h.cnt, kSubDelta, true);
                    dec_code(low, code, range, r2.esc + h.under, h.cnt, in, true);
                    r2.tot = (tot + kSubDelta) & 0xFFFF;
                    rec_rescale(reg, r2, h.cnt > 0xFF - 2 * kSubDelta || tot + kSubDelta > kTotalLimit);
                    nxt = h.link;
                    at = 2;
                }
            }
        }
        PROF(0)
        if (at < 0 && order >= 1 && r1.esc > 0) {
            const uint32_t tot = rec_total(reg, r1);
            if (r1.esc < tot) {
                range = udiv(range, tot);
                uint32_t cd = udiv(code - low, range) & 0xFFFF;
                if (cd < r1.esc) {
                    dec_code(low, code, range, 0, r1.esc, in, true);
                } else {
                    const Hit h = rec_search(reg, r1, cd - r1.esc, true);
                    if (!h.found) { fail = true; break; }
                    v = h.val;
                    rec_bump(reg, r1, h.k, h.cnt, kSubDelta, true);
                    dec_code(low, code, range, r1.esc + h.under, h.cnt, in, true);
                    r1.tot = (tot + kSubDelta) & 0xFFFF;
                    rec_rescale(reg, r1, h.cnt > 0xFF - 2 * kSubDelta || tot + kSubDelta > kTotalLimit);
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
        Rec<kO1Inl> n1;
        o1_load(reg, v, n1);                                         // next step's order-1 record
        // patch the contexts above, compress.c:598-615
        bool pend = false;
        uint32_t kpend = 0;
        PROF(3)
        if (order >= 2 && at < 2) {
            const Hit h = sub_update<kO2Inl, kO2MinCap, false>(reg, r2, v, bump, end, nodes, ovf, true);
            if (ovf) break;
            if (!h.found) { pend = true; kpend = h.k; }
        }
        PROF(4)
        if (order >= 1 && at < 1) {
            const Hit h = sub_update<kO1Inl, kO1MinCap, true>(reg, r1, v, bump, end, nodes, ovf, true);
            if (ovf) break;
            nxt = h.link;
            nfresh = !h.found;
        }
        rec_set_link(reg, r2, kpend, nxt, pend);
        PROF(5)
        Rec<kO2Inl> n2;
        o2_fresh(nxt, n2);
        const bool same2 = order >= 2 && nxt * kO2Rec == r2.off;
        if (order >= 1 && !nfresh && !same2) o2_load(reg, nxt, n2);
        if (order >= 2) o2_store(reg, r2);
        if (order >= 1 && at <= 1) o1_store(reg, r1);
        PROF(6)
        if (o.n >= o.cap) { fail = true; break; }                    // compress.c:617
        outwin_put(o, v, true);
        PROF(7)
        if (order >= 1 && !same2) rec2_copy(r2, n2);
        if (!(order >= 1 && v == b1)) r1 = n1;
        if (order < 2) ++order;
        b1 = v;
        if (any_lane(nodes >= kMaxNodes)) {
            if (nodes >= kMaxNodes) {
                region_reset(reg, root);
                rtot = 1 + 256; bump = kArenaBase; nodes = 1; order = 0;
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
    // order-1 table + one 8-B order-2 record per byte + extension blocks
    // (< 16 B per model node over their lifetime; <= 4094 nodes between resets)
    const uint64_t L = max_len < 4096 ? max_len : 4096;
    const uint64_t nodes = 2 * L + 256 < 4094 ? 2 * L + 256 : 4094;
    uint64_t bytes = kArenaBase + kO2Rec * L + 16 * nodes + 1024;
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
