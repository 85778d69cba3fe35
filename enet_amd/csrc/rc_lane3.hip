// rc_lane3.hip -- lane-per-packet range-coder kernels, model v3 (default).
//
// Same semantics as compress.c (enet_range_coder_compress :246-342,
// enet_range_coder_decompress :498-627), bit-exact.  One packet per lane; the
// lane logic is shared by the encoder and the decoder.
//
// Why this layout: the per-lane model of an order-2 PPM does not fit on chip
// (256 order-1 contexts per packet, 65536 packets in flight), so every byte
// touches at least one order-1 record in HBM at a random address.  At this
// concurrency HBM3E serves about 50-60 G random accesses per second
// (tools/mb/membench.hip: a dependent 64-B read-modify-write chain per lane
// runs at 2.9 us per step over a 1 GB table, a read-only one at 1.1 us), so the
// cost per byte is the number of random accesses it makes.  Model v2
// (rc_lane.hip) made about 3.5: the order-1 record read and write plus a
// 32-B order-2 record write and extra partial-line writes.  v3 makes 2 on the
// common path: one 64-B record read and one 64-B record write.
//
//   order 0 (root): LDS, as v2 (rc_lane_common.h).
//   order 1: a 64-B record per context byte, direct-mapped in the lane's
//       region, holding up to 12 symbols as sorted byte arrays (values,
//       counts) plus, per symbol, the state of the order-2 context that
//       symbol heads ("o2 info", below).  Larger contexts become dense
//       256-symbol blocks in the arena.
//   order 2: the context (a, b) is symbol b of order-1 context a.  While it
//       holds at most one symbol its whole state fits the o2 info of that
//       entry (escapes 5, total 5 + count); beyond that it gets a 64-B
//       record (24 symbols) in the arena, or a dense block.
//
// A record is therefore modified in two consecutive steps -- as the order-1
// context (context b at step i) and as the holder of the order-2 context
// (b, v) at step i+1 -- and is written once, when it leaves the registers.
// The next step's order-1 record R[v] is the only load on the common path; it
// is forwarded from registers when v is one of the two contexts in flight.
//
// Packets longer than 1919 bytes can reach compress.c's model reset
// (:148-157): the lanes count compress.c's nodes and reset at the same byte
// (lane_reset).  Corrupt streams whose root code points past symbol 255 and
// region overflows go to the exact path (rc_kernels.hip).

#ifndef RC_LANE_HOST_TEST
#include <hip/hip_runtime.h>
#else
#include "lane_host_shim.h"   // tests/proto: host build of the per-lane logic (test only)
#endif
#include <stdint.h>

#include "rc_abi_internal.h"
#include "rc_udiv.h"
#include "rc_lane_common.h"
#include "rc_root3.h"

namespace {

constexpr uint32_t kRec = 64;                       // order-1 record, big order-2 record
// decoder: links (o2 info) of symbols 0..kLinkCache-1 of the packet's first
// dense order-1 context, cached in LDS (64 B per lane).  A step decoded at
// order 2 needs only the link of (b, v) from its order-1 context b, and on
// game state b is mostly 0, whose dense block is in HBM: the cache takes that
// dependent load off the step for small v.  A link of a symbol b lacks is 0
// (blocks start zeroed, links are written only for present symbols), so the
// link alone gives the next step's order-2 info.
constexpr uint32_t kLinkCache = 32;
constexpr uint32_t kArena3 = kO1Base + 256 * kRec;  // arena start (after header and order-1 table)
constexpr uint32_t kMaxLen3 = 1919;                 // <= 2*1919 + 256 nodes < 4094: no reset (compress.c:150)
constexpr uint32_t kNodeLimit = 4096 - 2;           // compress.c:148-157: sizeof symbols / sizeof ENetSymbol - order
constexpr uint32_t kInlineMax = 127;                // inline order-2 counts stay below 0x80

// o2 info (u16) of an order-1 symbol: the state of the order-2 context it heads
//   0                        empty: escapes = total = 0 (compress.c:68-79)
//   a | c << 8, 1 <= c <= 127 one symbol a, count c; escapes 5, total 5 + c
//   i | (0x80 | i >> 8) << 8   a record at arena offset 64 * i
DEV bool info_big(uint32_t info) { return info >= 0x8000u; }
DEV uint32_t info_rec(uint32_t info) { return (info & 0x7FFFu) * kRec; }

// ------------------------------------------------------------ contexts
// O2 = true: order-1 record (12 symbols + o2 info bytes); false: big order-2
// record (24 symbols).  Unused slots hold value 0xFF and count 0, so the SWAR
// scans need no length mask except for equality with 255.
template <uint32_t NV, bool O2>
struct Ctx {
    uint32_t len, dense, esc, tot, ext;   // ext: dense block offset
    uint32_t val[NV], cnt[NV];
    uint32_t oa[O2 ? NV : 1], ob[O2 ? NV : 1];   // o2 info low / high bytes
};
using Rec1 = Ctx<3, true>;
using Rec2 = Ctx<6, false>;

struct Raw { uint4 q0, q1, q2, q3; };

DEV void raw_load(const uint8_t* reg, uint32_t off, Raw& w)
{
    const uint4* p = reinterpret_cast<const uint4*>(reg + off);
    w.q0 = p[0]; w.q1 = p[1]; w.q2 = p[2]; w.q3 = p[3];
}

// A dense order-1 context keeps its block's C (16 cumulative group counts,
// 32 B) in its record, where an inline one keeps its symbols (w4..w11: val,
// cnt, oa[0..1]).  The record load a step issues ahead then brings C along,
// and the decoder's dense search waits for one dependent load (the symbol's
// group) instead of two.  The copy follows every change of the block's C:
// densify, dense_add, dense_rescale.
template <uint32_t NV, bool O2>
DEV void rec_c_get(const Ctx<NV, O2>& c, uint4& c0, uint4& c1)
{
    if constexpr (O2 && NV == 3) {
        c0 = make_uint4(c.val[0], c.val[1], c.val[2], c.cnt[0]);
        c1 = make_uint4(c.cnt[1], c.cnt[2], c.oa[0], c.oa[1]);
    }
}

template <uint32_t NV, bool O2>
DEV void rec_c_set(Ctx<NV, O2>& c, const uint4& c0, const uint4& c1, bool en)
{
    if constexpr (O2 && NV == 3) {
        c.val[0] = en ? c0.x : c.val[0]; c.val[1] = en ? c0.y : c.val[1]; c.val[2] = en ? c0.z : c.val[2];
        c.cnt[0] = en ? c0.w : c.cnt[0]; c.cnt[1] = en ? c1.x : c.cnt[1]; c.cnt[2] = en ? c1.y : c.cnt[2];
        c.oa[0] = en ? c1.z : c.oa[0]; c.oa[1] = en ? c1.w : c.oa[1];
    }
}

template <uint32_t NV, bool O2>
DEV void ctx_clear(Ctx<NV, O2>& c)
{
    c.len = 0; c.dense = 0; c.esc = 0; c.tot = 0; c.ext = 0;
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) { c.val[d] = 0xFFFFFFFFu; c.cnt[d] = 0u; }
#pragma unroll
    for (uint32_t d = 0; d < (O2 ? NV : 1); ++d) { c.oa[d] = 0u; c.ob[d] = 0u; }
}

// ------------------------------------------------------- the hot block
// The decoder keeps the counts of the packet's first dense order-1 context
// (the one whose first links the LDS cache holds, L.cext) in registers: its
// 16 groups, 64 VGPRs.  On game state that context (byte 0) takes ~86 % of
// the dense order-1 steps; its lookups (a search's group, a find's group),
// updates and rescales then touch no memory, where each was a dependent
// random read.  C rides in the record as for any dense
// order-1 context; the links stay in the arena behind the LDS link cache.
// The block's counts in the arena are left as they were when it became hot:
// nothing reads them afterwards.
// Measured, and off: the block lives in AGPRs (the kernel's 256 VGPRs are
// taken), so each lookup is 64 AGPR reads and 60 selects, each update as
// many again, for any lane of the wavefront in the hot context (most steps);
// C3 rc_decompress_lane3 5.70 -> 6.13 ms although its fabric traffic fell
// 16.3 -> 15.2 GB (profiles/r6/r6m_lane3_hot_block_c3.txt).  -DLANE3_HOT: on.
#ifdef LANE3_HOT
constexpr bool kHot = true;
#else
constexpr bool kHot = false;
#endif
struct Hot { uint4 g[16]; };

DEV uint4 sel_u4(bool p, const uint4& a, const uint4& b)
{
    return make_uint4(p ? a.x : b.x, p ? a.y : b.y, p ? a.z : b.z, p ? a.w : b.w);
}

// p ? a : b where the compiler cannot see a select: a select between two
// elements of the block becomes a load from a lane-varying address, which
// would put the block in scratch memory
#ifndef RC_LANE_HOST_TEST
DEV uint32_t vsel(bool p, uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(__builtin_amdgcn_ballot_w64(p)));
    return r;
}
#else
DEV uint32_t vsel(bool p, uint32_t a, uint32_t b) { return p ? a : b; }
#endif
DEV uint4 vsel_u4(bool p, const uint4& a, const uint4& b)
{
    return make_uint4(vsel(p, a.x, b.x), vsel(p, a.y, b.y), vsel(p, a.z, b.z), vsel(p, a.w, b.w));
}

// group g of the hot block (a select tree on the bits of g: registers only)
DEV uint4 hot_get(const Hot& H, uint32_t g)
{
    uint4 t8[8], t4[4], t2[2];
    const bool b0 = (g & 1u) != 0, b1 = (g & 2u) != 0, b2 = (g & 4u) != 0, b3 = (g & 8u) != 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) t8[k] = vsel_u4(b0, H.g[2 * k + 1], H.g[2 * k]);
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) t4[k] = vsel_u4(b1, t8[2 * k + 1], t8[2 * k]);
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) t2[k] = vsel_u4(b2, t4[2 * k + 1], t4[2 * k]);
    return vsel_u4(b3, t2[1], t2[0]);
}

// group g := q where en
DEV void hot_put(Hot& H, uint32_t g, const uint4& q, bool en)
{
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) H.g[k] = sel_u4(en && g == k, q, H.g[k]);
}

// compress.c:90-112 on the hot block where en: halve, the new C; returns the sum
DEV uint32_t hot_rescale(Hot& H, uint4& c0, uint4& c1, bool en)
{
    uint32_t sum = 0, cw[8];
#pragma unroll
    for (uint32_t g = 0; g < 16; ++g) {
        uint4 q = H.g[g];
        q.x -= (q.x >> 1) & 0x7F7F7F7Fu;
        q.y -= (q.y >> 1) & 0x7F7F7F7Fu;
        q.z -= (q.z >> 1) & 0x7F7F7F7Fu;
        q.w -= (q.w >> 1) & 0x7F7F7F7Fu;
        H.g[g] = sel_u4(en, q, H.g[g]);
        sum = sad(q.w, sad(q.z, sad(q.y, sad(q.x, sum))));
        if (g & 1) cw[g >> 1] |= sum << 16; else cw[g >> 1] = sum;
    }
    c0 = make_uint4(cw[0], cw[1], cw[2], cw[3]);
    c1 = make_uint4(cw[4], cw[5], cw[6], cw[7]);
    return sum;
}

// dense_add (rc_lane_common.h) on z alone where en: count[v] += d, C[g..15] += d
DEV void dense_bump(Dense& z, uint32_t v, uint32_t d, bool en)
{
    const uint32_t g = v >> 4, j = v & 15, bd = en ? d << (8 * (j & 3)) : 0u, q = j >> 2;
    z.grp.x += q == 0 ? bd : 0u; z.grp.y += q == 1 ? bd : 0u;
    z.grp.z += q == 2 ? bd : 0u; z.grp.w += q == 3 ? bd : 0u;
    uint32_t cw[8] = {z.c0.x, z.c0.y, z.c0.z, z.c0.w, z.c1.x, z.c1.y, z.c1.z, z.c1.w};
    cum_add(cw, g, en ? d : 0u);
    z.c0 = make_uint4(cw[0], cw[1], cw[2], cw[3]);
    z.c1 = make_uint4(cw[4], cw[5], cw[6], cw[7]);
}

// is c (an order-1 context) the hot block
// (on: the caller keeps a hot block -- a template flag, never a test of the
// block's address, which would keep the block out of registers)
DEV bool is_hot(bool on, uint32_t cext, uint32_t dense, uint32_t ext)
{
    return kHot && on && cext != 0 && dense != 0 && ext == cext;
}

// order-1 record: w0 tag | len << 16 | dense << 24, w1 esc | tot << 16, w2 ext,
// w4..6 val, w7..9 cnt, w10..12 oa, w13..15 ob.  A tag other than the epoch
// reads as an empty context.
DEV void rec1_from(const Raw& w, uint32_t epoch, Rec1& c)
{
    const bool live = (w.q0.x & 0xFFFFu) == epoch;
    const uint32_t f = live ? 0xFFFFFFFFu : 0u;
    c.len = (w.q0.x >> 16) & 0xFF & f; c.dense = (w.q0.x >> 24) & f;
    c.esc = w.q0.y & 0xFFFF & f; c.tot = (w.q0.y >> 16) & f; c.ext = w.q0.z;
    c.val[0] = w.q1.x | ~f; c.val[1] = w.q1.y | ~f; c.val[2] = w.q1.z | ~f;
    c.cnt[0] = w.q1.w & f; c.cnt[1] = w.q2.x & f; c.cnt[2] = w.q2.y & f;
    c.oa[0] = w.q2.z & f; c.oa[1] = w.q2.w & f; c.oa[2] = w.q3.x & f;
    c.ob[0] = w.q3.y & f; c.ob[1] = w.q3.z & f; c.ob[2] = w.q3.w & f;
}

DEV void rec1_store_at(uint8_t* reg, uint32_t off, uint32_t epoch, const Rec1& c)
{
    uint4* p = reinterpret_cast<uint4*>(reg + off);
    p[0] = make_uint4(epoch | (c.len << 16) | (c.dense << 24), c.esc | (c.tot << 16), c.ext, 0u);
    p[1] = make_uint4(c.val[0], c.val[1], c.val[2], c.cnt[0]);
    p[2] = make_uint4(c.cnt[1], c.cnt[2], c.oa[0], c.oa[1]);
    p[3] = make_uint4(c.oa[2], c.ob[0], c.ob[1], c.ob[2]);
}

// big order-2 record: w0 len << 16 | dense << 24, w1 esc | tot << 16, w2 ext,
// w4..9 val, w10..15 cnt
DEV void rec2_from(const Raw& w, Rec2& c)
{
    c.len = (w.q0.x >> 16) & 0xFF; c.dense = w.q0.x >> 24;
    c.esc = w.q0.y & 0xFFFF; c.tot = w.q0.y >> 16; c.ext = w.q0.z;
    c.val[0] = w.q1.x; c.val[1] = w.q1.y; c.val[2] = w.q1.z; c.val[3] = w.q1.w; c.val[4] = w.q2.x; c.val[5] = w.q2.y;
    c.cnt[0] = w.q2.z; c.cnt[1] = w.q2.w; c.cnt[2] = w.q3.x; c.cnt[3] = w.q3.y; c.cnt[4] = w.q3.z; c.cnt[5] = w.q3.w;
    c.oa[0] = 0u; c.ob[0] = 0u;
}

DEV void rec2_store(uint8_t* reg, uint32_t off, const Rec2& c)
{
    uint4* p = reinterpret_cast<uint4*>(reg + off);
    p[0] = make_uint4((c.len << 16) | (c.dense << 24), c.esc | (c.tot << 16), c.ext, 0u);
    p[1] = make_uint4(c.val[0], c.val[1], c.val[2], c.val[3]);
    p[2] = make_uint4(c.val[4], c.val[5], c.cnt[0], c.cnt[1]);
    p[3] = make_uint4(c.cnt[2], c.cnt[3], c.cnt[4], c.cnt[5]);
}

// ------------------------------------------------ lookup and update (SWAR)

template <uint32_t NV>
struct Look {
    uint32_t k, under, cnt, info;   // slot (insertion slot if absent), counts below, count, o2 info
    uint32_t found;                 // 0 / 1 (a word: a bool would be an SGPR lane mask)
    uint32_t eq[NV];                // 0x01 in the byte of the found slot
    Dense z;                        // dense contexts: C, the symbol's group, its o2 info
};

// o2 info of slot k (one-hot eq) of an order-1 record
template <uint32_t NV, bool O2>
DEV uint32_t slot_info(const Ctx<NV, O2>& c, const uint32_t* eq)
{
    uint32_t a = 0, b = 0;
    if (O2) {
#pragma unroll
        for (uint32_t d = 0; d < NV; ++d) { a = dot4(c.oa[d], eq[d], a); b = dot4(c.ob[d], eq[d], b); }
    }
    return a | (b << 8);
}

// Dense blocks of big order-2 contexts (Ctx<6, false>) live in the arena
// (dense 1) or, for the first one of a packet, in the lane's 288-B LDS block
// ldsb (dense 2): game-state packets have exactly one such context, (0, 0),
// visited by about half of their bytes, whose lookups, updates and rescales
// then stay on chip.  (Two call sites, one per address space: a pointer
// select would become flat memory operations.)
template <uint32_t NV, bool O2>
DEV void ctx_dense_find(const uint8_t* reg, const uint8_t* ldsb, const Ctx<NV, O2>& c, uint32_t v, Dense& z,
                        uint32_t& u, uint32_t& n)
{
    if constexpr (!O2) {
        // The arena path in a branch of its own that waits for its loads:
        // LDS reads into registers of an arena load the compiler must assume
        // pending would wait vmcnt(0) for it -- and, in the decoder, for the
        // record load issued before it -- even in wavefronts where no lane
        // read the arena (game state: the dense order-2 block is the LDS one).
        const uint4 zz = make_uint4(0u, 0u, 0u, 0u);
        z.c0 = zz; z.c1 = zz; z.grp = zz; z.link = 0;
        u = 0; n = 0;
        if (any_lane(c.dense == 1)) {
            if (c.dense == 1) dense_find(reg + c.ext, v, O2, z, u, n);
            __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0)
        }
        if (c.dense == 2) dense_find(ldsb, v, O2, z, u, n);
        return;
    }
    if (!O2 && c.dense == 2) dense_find(ldsb, v, O2, z, u, n);
    else dense_find(reg + c.ext, v, O2, z, u, n);
}

template <uint32_t NV, bool O2>
DEV bool ctx_dense_search(const uint8_t* reg, const uint8_t* ldsb, const Ctx<NV, O2>& c, uint32_t code, Dense& z,
                          uint32_t& v, uint32_t& u, uint32_t& n)
{
    if (!O2 && c.dense == 2) return dense_search(ldsb, code, O2, z, v, u, n);
    if (O2) {                                   // (C from the record)
        rec_c_get(c, z.c0, z.c1);
        return dense_search(reg + c.ext, code, O2, z, v, u, n, true);
    }
    return dense_search(reg + c.ext, code, O2, z, v, u, n);
}

// compress.c:159-199 lookup of v (minimum 0): slot, counts below v, count[v], o2 info
template <uint32_t NV, bool O2>
DEV Look<NV> ctx_find(const uint8_t* reg, const uint8_t* ldsb, const Ctx<NV, O2>& c, uint32_t v)
{
    Look<NV> h;
    h.k = 0; h.under = 0; h.cnt = 0;
    const uint32_t ny = 0x01000100u - v * 0x00010001u;
    const uint32_t ny1 = ny - 0x00010001u;
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) {
        const uint32_t ge = swar_ge(c.val[d], ny);
        const uint32_t lt = ge ^ 0x01010101u;
        h.eq[d] = (ge ^ swar_ge(c.val[d], ny1)) & below_mask(static_cast<int>(c.len), d) & 0x01010101u;
        h.k = sad(lt, h.k);
        h.under = dot4(c.cnt[d], lt, h.under);
        h.cnt = dot4(c.cnt[d], h.eq[d], h.cnt);
    }
    h.info = slot_info<NV, O2>(c, h.eq);
    if (any_lane(c.dense != 0)) {
        if (c.dense != 0) {
            uint32_t u, n;
            ctx_dense_find(reg, ldsb, c, v, h.z, u, n);
            h.under = u; h.cnt = n; h.info = h.z.link;
        }
    }
    h.found = h.cnt != 0 ? 1u : 0u;
    return h;
}

// ctx_find for the decoder's order-1 lookups, with a dense context's group and
// link already loaded (zp, issued before the next record's load: loads return
// in order, so waiting for them no longer waits for that record) and its C
// from the record
DEV Look<3> ctx_find_pre(const Rec1& c, uint32_t v, const Dense& zp)
{
    Look<3> h;
    h.k = 0; h.under = 0; h.cnt = 0;
    const uint32_t ny = 0x01000100u - v * 0x00010001u;
    const uint32_t ny1 = ny - 0x00010001u;
#pragma unroll
    for (uint32_t d = 0; d < 3; ++d) {
        const uint32_t ge = swar_ge(c.val[d], ny);
        const uint32_t lt = ge ^ 0x01010101u;
        h.eq[d] = (ge ^ swar_ge(c.val[d], ny1)) & below_mask(static_cast<int>(c.len), d) & 0x01010101u;
        h.k = sad(lt, h.k);
        h.under = dot4(c.cnt[d], lt, h.under);
        h.cnt = dot4(c.cnt[d], h.eq[d], h.cnt);
    }
    h.info = slot_info<3, true>(c, h.eq);
    // (selects, not a branch: the preloaded registers are read, never
    // overwritten in place, so no later write to them waits for the load --
    // and for the record load behind it)
    {
        Dense z;
        rec_c_get(c, z.c0, z.c1);
        z.grp = zp.grp;
        z.link = zp.link;
        const uint32_t g = v >> 4, j = v & 15;
        uint32_t within = 0;
#pragma unroll
        for (uint32_t d = 0; d < 4; ++d) {
            const uint32_t nb = j > 4 * d ? min(j - 4 * d, 4u) : 0u;
            const uint32_t mask = nb >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
            within = sad(pick4(d, z.grp) & mask, within);
        }
        const bool dn = c.dense != 0;
        h.under = dn ? (g ? dense_c(z, g - 1) : 0u) + within : h.under;
        h.cnt = dn ? (pick4(j >> 2, z.grp) >> (8 * (j & 3))) & 0xFF : h.cnt;
        h.info = dn ? z.link : h.info;
        h.z = z;
    }
    h.found = h.cnt != 0 ? 1u : 0u;
    return h;
}

// Decoder: the symbol whose interval [under, under + count) holds code
// (minimum 0): the dword whose running byte sum passes code, then halving
// on byte sums inside it.  False = no such symbol (corrupt, compress.c:416).
template <uint32_t NV, bool O2>
DEV bool ctx_search(const uint8_t* reg, const uint8_t* ldsb, const Ctx<NV, O2>& c, uint32_t code, Look<NV>& h,
                    uint32_t& v)
{
    uint32_t acc = 0, base = 0, wc = 0, wv = 0xFFFFFFFFu, j = 0;
    bool hit = false;
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) {
        const uint32_t s = sad(c.cnt[d], 0u);
        const bool here = !hit && code < acc + s;
        base = here ? acc : base; wc = here ? c.cnt[d] : wc; wv = here ? c.val[d] : wv; j = here ? 4 * d : j;
        hit = hit || here;
        acc += s;
    }
    uint32_t s = sad(wc & 0xFFFFu, 0u);
    bool hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 2u : 0u;
    wc = hi ? (wc >> 16) : wc; wv = hi ? (wv >> 16) : wv;
    s = wc & 0xFFu;
    hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 1u : 0u;
    wc = hi ? (wc >> 8) : wc; wv = hi ? (wv >> 8) : wv;
    h.k = j; h.under = base; h.cnt = wc & 0xFFu; v = wv & 0xFFu;
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) h.eq[d] = byte_mask(static_cast<int>(j), d) & 0x01010101u;
    h.info = slot_info<NV, O2>(c, h.eq);
    bool ok = hit && h.cnt != 0;
    if (any_lane(c.dense != 0)) {
        if (c.dense != 0) {
            uint32_t u, n, vv;
            ok = ctx_dense_search(reg, ldsb, c, code, h.z, vv, u, n);
            h.under = u; h.cnt = n; v = vv; h.info = h.z.link;
        }
    }
    h.found = ok ? 1u : 0u;
    return ok;
}

// ctx_search of the decoder's order-1 context c: a dense one's group from the
// hot block's registers where c is the hot block (else its load), and its
// link from the LDS link cache where that holds it (else its load); either
// load is issued only when some lane of the wavefront needs it
DEV bool o1_search(const uint8_t* reg, const Rec1& c, const Hot& H, uint32_t cext, const uint16_t* lc,
                   uint32_t code, Look<3>& h, uint32_t& v)
{
    uint32_t acc = 0, base = 0, wc = 0, wv = 0xFFFFFFFFu, j = 0;
    bool hit = false;
#pragma unroll
    for (uint32_t d = 0; d < 3; ++d) {
        const uint32_t s = sad(c.cnt[d], 0u);
        const bool here = !hit && code < acc + s;
        base = here ? acc : base; wc = here ? c.cnt[d] : wc; wv = here ? c.val[d] : wv; j = here ? 4 * d : j;
        hit = hit || here;
        acc += s;
    }
    uint32_t s = sad(wc & 0xFFFFu, 0u);
    bool hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 2u : 0u;
    wc = hi ? (wc >> 16) : wc; wv = hi ? (wv >> 16) : wv;
    s = wc & 0xFFu;
    hi = code >= base + s;
    base += hi ? s : 0u; j += hi ? 1u : 0u;
    wc = hi ? (wc >> 8) : wc; wv = hi ? (wv >> 8) : wv;
    h.k = j; h.under = base; h.cnt = wc & 0xFFu; v = wv & 0xFFu;
#pragma unroll
    for (uint32_t d = 0; d < 3; ++d) h.eq[d] = byte_mask(static_cast<int>(j), d) & 0x01010101u;
    h.info = slot_info<3, true>(c, h.eq);
    bool ok = hit && h.cnt != 0;
    if (any_lane(c.dense != 0)) {
        if (c.dense != 0) {
            const bool hot = is_hot(true, cext, c.dense, c.ext);
            Dense z;
            rec_c_get(c, z.c0, z.c1);
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
            uint4 grp = make_uint4(0u, 0u, 0u, 0u);
            if (any_lane(!hot)) {
                if (!hot) grp = *reinterpret_cast<const uint4*>(reg + c.ext + 32 + 16 * g);
            }
            if (any_lane(hot)) grp = sel_u4(hot, hot_get(H, g), grp);
            z.grp = grp;
            uint32_t bs = prev, jj = 0;
            uint32_t t = sad(grp.x, sad(grp.y, 0u));
            bool up = code >= bs + t;
            bs += up ? t : 0u; jj += up ? 8u : 0u;
            const uint32_t d0 = up ? grp.z : grp.x, d1 = up ? grp.w : grp.y;
            t = sad(d0, 0u);
            up = code >= bs + t;
            bs += up ? t : 0u; jj += up ? 4u : 0u;
            uint32_t w = up ? d1 : d0;
            t = sad(w & 0xFFFFu, 0u);
            up = code >= bs + t;
            bs += up ? t : 0u; jj += up ? 2u : 0u;
            w = up ? (w >> 16) : w;
            t = w & 0xFFu;
            up = code >= bs + t;
            bs += up ? t : 0u; jj += up ? 1u : 0u;
            w = up ? (w >> 8) : w;
            const uint32_t vv = 16 * g + jj, cnt = w & 0xFFu;
            const bool lch = hot && vv < kLinkCache;
            uint32_t link = lc[vv & (kLinkCache - 1)];
            if (any_lane(!lch)) {
                if (!lch) link = *reinterpret_cast<const uint16_t*>(reg + c.ext + 288 + 2 * vv);
            }
            z.link = link;
            ok = inside && cnt != 0 && code < bs + cnt;
            h.under = bs; h.cnt = cnt; v = vv; h.info = link; h.z = z;
        }
    }
    h.found = ok ? 1u : 0u;
    return ok;
}

// insert (v, count 2, o2 info 0) at slot k of an inline context with a free slot
template <uint32_t NV, bool O2>
DEV void inline_insert(Ctx<NV, O2>& c, uint32_t k, uint32_t v, bool en)
{
    const int kk = static_cast<int>(k);
    uint32_t pv = 0xFFFFFFFFu, pc = 0u, pa = 0u, pb = 0u;
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) {
        const uint32_t bm = below_mask(kk, d), im = byte_mask(kk, d), keep = en ? bm : 0xFFFFFFFFu;
        // bytes below k stay, byte k is new, bytes above move up one slot
        const uint32_t sv = align8(c.val[d], pv, 3), sc = align8(c.cnt[d], pc, 3);
        pv = c.val[d]; pc = c.cnt[d];
        c.val[d] = (c.val[d] & keep) | (((sv & ~im) | ((v * 0x01010101u) & im)) & ~keep);
        c.cnt[d] = (c.cnt[d] & keep) | (((sc & ~im) | ((kSubDelta * 0x01010101u) & im)) & ~keep);
        if (O2) {
            const uint32_t sa = align8(c.oa[d], pa, 3), sb = align8(c.ob[d], pb, 3);
            pa = c.oa[d]; pb = c.ob[d];
            c.oa[d] = (c.oa[d] & keep) | (sa & ~im & ~keep);
            c.ob[d] = (c.ob[d] & keep) | (sb & ~im & ~keep);
        }
    }
}

// o2 info of slot k (one-hot eq) := info where `en`
template <uint32_t NV, bool O2>
DEV void slot_set_info(Ctx<NV, O2>& c, const uint32_t* eq, uint32_t info, bool en)
{
    if (O2) {
#pragma unroll
        for (uint32_t d = 0; d < NV; ++d) {
            const uint32_t m = en ? eq[d] * 0xFFu : 0u;
            c.oa[d] = (c.oa[d] & ~m) | ((info & 0xFFu) * 0x01010101u & m);
            c.ob[d] = (c.ob[d] & ~m) | ((info >> 8) * 0x01010101u & m);
        }
    }
}

// a dense block's contents from an inline context (C[16], counts, o2 info)
template <uint32_t NV, bool O2>
DEV void dense_fill(uint8_t* blk, const Ctx<NV, O2>& c)
{
    const uint32_t size = O2 ? kDenseO1 : kDenseO2;
    uint4* p = reinterpret_cast<uint4*>(blk);
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    for (uint32_t i = 2; i < size / 16; ++i) p[i] = z;
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
#pragma unroll 1
    for (uint32_t t = 0; t < c.len; ++t) {
        uint32_t vv = 0, cc = 0, ia = 0, ib = 0;
#pragma unroll
        for (uint32_t d = 0; d < NV; ++d) {
            const uint32_t m = byte_mask(static_cast<int>(t), d);
            const uint32_t sh = 8 * (t & 3);
            vv |= (c.val[d] & m) >> sh; cc |= (c.cnt[d] & m) >> sh;
            if (O2) { ia |= (c.oa[d] & m) >> sh; ib |= (c.ob[d] & m) >> sh; }
        }
        blk[32 + vv] = static_cast<uint8_t>(cc);
        if (O2) reinterpret_cast<uint16_t*>(blk + 288)[vv] = static_cast<uint16_t>(ia | (ib << 8));
    }
}

// move an inline context to a fresh dense block -- the lane's LDS block for
// the packet's first big order-2 context (ldsu: taken), else the arena;
// false = arena full
template <uint32_t NV, bool O2>
DEV bool densify(uint8_t* reg, uint8_t* ldsb, uint32_t& ldsu, Ctx<NV, O2>& c, uint32_t& bump, uint32_t end)
{
    const bool lds = !O2 && ldsu == 0;
    if (lds) {
        dense_fill<NV, O2>(ldsb, c);
        ldsu = 1;
        c.ext = 0;
    } else {
        const uint32_t size = O2 ? kDenseO1 : kDenseO2;
        const uint32_t at = (bump + 15) & ~15u;
        if (at + size > end) return false;
        bump = at + size;
        dense_fill<NV, O2>(reg + at, c);
        c.ext = at;
    }
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) { c.val[d] = 0xFFFFFFFFu; c.cnt[d] = 0u; }
#pragma unroll
    for (uint32_t d = 0; d < (O2 ? NV : 1); ++d) { c.oa[d] = 0u; c.ob[d] = 0u; }
    c.dense = lds ? 2u : 1u;
    if (O2) {                                   // the block's C into the record (as dense_fill wrote it)
        const uint4* q = reinterpret_cast<const uint4*>(reg + c.ext);
        rec_c_set(c, q[0], q[1], true);
    }
    return true;
}

// compress.c:90-112 where `en`
template <uint32_t NV, bool O2, bool HOT = false>
DEV void ctx_rescale(uint8_t* reg, uint8_t* ldsb, Ctx<NV, O2>& c, bool en, Hot* H = nullptr, uint32_t cext = 0)
{
    if (!rare_lane(en)) return;
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) {
        const uint32_t h = c.cnt[d] - ((c.cnt[d] >> 1) & 0x7F7F7F7Fu);
        c.cnt[d] = en ? h : c.cnt[d];
        sum = sad(h, sum);
    }
    const bool hot = O2 && is_hot(HOT, cext, c.dense, c.ext);
    if (O2 && HOT && rare_lane(en && hot)) {     // (registers only)
        uint4 c0, c1;
        const uint32_t hs = hot_rescale(*H, c0, c1, en && hot);
        sum = (en && hot) ? hs : sum;
        rec_c_set(c, c0, c1, en && hot);
    }
    if (rare_lane(en && c.dense != 0 && !hot)) {
        if (en && c.dense != 0 && !hot) {
            if (!O2 && c.dense == 2) sum = dense_rescale(ldsb);
            else sum = dense_rescale(reg + c.ext);
            if (O2) {                           // (the halving above hit the record's copy of C: the new C)
                const uint4* q = reinterpret_cast<const uint4*>(reg + c.ext);
                rec_c_set(c, q[0], q[1], true);
            }
        }
    }
    c.esc -= en ? (c.esc >> 1) : 0u;
    c.tot = en ? ((c.esc + sum) & 0xFFFF) : c.tot;
}

// compress.c:293-314 (and the decoder's patch, :598-615) where `en`, given
// the lookup h of v: bump v or insert it, then total and rescale.  h.k stays
// the slot of v.
template <uint32_t NV, bool O2, bool HOT = false>
DEV void ctx_update(uint8_t* reg, uint8_t* ldsb, uint32_t& ldsu, Ctx<NV, O2>& c, Look<NV>& h, uint32_t v,
                    uint32_t& bump, uint32_t end, bool& ovf, bool en, Hot* H = nullptr, uint32_t cext = 0)
{
    const bool ins = en && !h.found;
    const bool inl = c.dense == 0;
    constexpr uint32_t cap = 4u * NV;
#pragma unroll
    for (uint32_t d = 0; d < NV; ++d) c.cnt[d] += (en && h.found && inl) ? (h.eq[d] << 1) : 0u;
    inline_insert<NV, O2>(c, h.k, v, ins && inl && c.len < cap);
    const bool grow = ins && inl && c.len >= cap;
    if (rare_lane(grow || (en && !inl))) {
        if (grow) {
            const bool ok = densify<NV, O2>(reg, ldsb, ldsu, c, bump, end);
            ovf = ovf || !ok;
            if (ok) { uint32_t u, n; ctx_dense_find(reg, ldsb, c, v, h.z, u, n); }
        }
        if (en && c.dense != 0 && !ovf) {                                   // (new: o2 info is 0)
            if (!O2 && c.dense == 2) dense_add(ldsb, v, kSubDelta, h.z);
            else if (!(O2 && is_hot(HOT, cext, c.dense, c.ext))) dense_add(reg + c.ext, v, kSubDelta, h.z);
            rec_c_set(c, h.z.c0, h.z.c1, true);
        }
    }
    // the hot block (registers): a bump or an insert, its group and C
    if (O2 && HOT) {
        const bool hot = en && !ovf && is_hot(HOT, cext, c.dense, c.ext);
        if (any_lane(hot)) {
            Dense z = h.z;
            dense_bump(z, v, kSubDelta, hot);
            hot_put(*H, v >> 4, z.grp, hot);
            h.z.grp = sel_u4(hot, z.grp, h.z.grp);
            h.z.c0 = sel_u4(hot, z.c0, h.z.c0);
            h.z.c1 = sel_u4(hot, z.c1, h.z.c1);
            rec_c_set(c, z.c0, z.c1, hot);
        }
    }
    if (ins && c.dense == 0) {
#pragma unroll
        for (uint32_t d = 0; d < NV; ++d) h.eq[d] = byte_mask(static_cast<int>(h.k), d) & 0x01010101u;
    }
    c.len += ins ? 1u : 0u;
    c.esc += ins ? kSubEscDelta : 0u;
    const uint32_t tot = (c.tot + (ins ? kSubEscDelta : 0u) + kSubDelta) & 0xFFFF;
    c.tot = en ? tot : c.tot;
    ctx_rescale<NV, O2, HOT>(reg, ldsb, c, en && (h.cnt > 0xFF - 2 * kSubDelta || tot > kTotalLimit), H, cext);
}

// ------------------------------------------------------------ lane state

// Everything a lane carries from one step to the next.  Contexts of step i:
// a = byte i-2, b = byte i-1.  `cur` is R[b]; `prv` is R[a], which holds the
// o2 info of (a, b) in slot `kp` (or `cur` does, when a == b: `same`).  A dense
// holder keeps it at `ipos` instead.  `q` is the big record of (a, b).
struct Lane {
    Rec1 cur, prv;
    Rec2 q;
    Raw rc, rq;                 // loads in flight for the next step (cur, q)
    uint32_t eqp[3];            // one-hot slot of b in its holder
    uint32_t info;              // o2 info of (a, b)
    uint32_t ipos;              // dense holder: region offset of that info (0 = inline holder)
    uint32_t a, b, order, epoch, bump, qoff;
    // (flags as 0/1 words: the compiler keeps a bool as a 64-bit lane mask in
    // SGPRs, and a dozen loop-carried ones spill into VGPR lanes)
    uint32_t same, fwd, prv_dirty, q_dirty, q_fwd, ovf;
    uint32_t nsame, fromprv;    // where the next step's R[v] comes from (lane_prefetch)
    uint32_t nodes;             // compress.c's nextSymbol: 1 (root) + the (context, value) pairs created
    uint32_t ldsu;              // the lane's LDS dense block holds a big order-2 context
    uint32_t cext;              // decoder: the dense order-1 block whose first links are in the LDS cache (0: none)
    uint8_t* dm;                // the scratch record (see lane_dummy)
};

// The scratch record that the step's unconditional loads and stores use
// when a lane needs none (lane_prefetch): one per wavefront, in the region
// of its first lane, so that the lanes without a real access touch one line
// between them -- one request that stays in the L1/L2 -- instead of 64
// separate lines (rc_lane3's C3 fabric traffic).
// LANE3_LANE_DUMMY (A/B): each lane's own scratch record.
DEV uint8_t* lane_dummy(uint8_t* reg, uint8_t* wave_reg)
{
#ifdef LANE3_LANE_DUMMY
    (void) wave_reg;
    return reg + kDummyRec;
#else
    return (wave_reg ? wave_reg : reg) + kDummyRec;
#endif
}

DEV void lane_init(Lane& L, uint8_t* reg, uint8_t* dm)
{
    L.dm = dm;
    L.epoch = next_epoch(reg, *reinterpret_cast<const uint32_t*>(reg)) & 0xFFFF;
    ctx_clear(L.cur); ctx_clear(L.prv); ctx_clear(L.q);
    L.info = 0; L.ipos = 0; L.a = 0; L.b = 0; L.order = 0; L.bump = kArena3; L.qoff = 0;
    L.eqp[0] = L.eqp[1] = L.eqp[2] = 0u;
    L.same = false; L.fwd = true; L.prv_dirty = false; L.q_dirty = false; L.q_fwd = true; L.ovf = false;
    L.nsame = false; L.fromprv = false;
    L.nodes = 1;
    L.ldsu = 0;
    L.cext = 0;
}

// compress.c:148-157: the model starts over (new epoch: every order-1 record
// reads as empty; arena from the start; order 0), as at a packet start.  The
// caller clears the root.  Loads in flight read as empty under the new epoch.
DEV void lane_reset(Lane& L, uint8_t* reg)
{
    L.epoch = next_epoch(reg, L.epoch) & 0xFFFF;
    ctx_clear(L.cur); ctx_clear(L.prv); ctx_clear(L.q);
    L.info = 0; L.ipos = 0; L.a = 0; L.b = 0; L.order = 0; L.bump = kArena3; L.qoff = 0;
    L.eqp[0] = L.eqp[1] = L.eqp[2] = 0u;
    L.same = false; L.fwd = true; L.prv_dirty = false; L.q_dirty = false; L.q_fwd = true;
    L.nsame = false; L.fromprv = false;
    L.nodes = 1;
    L.ldsu = 0;
    L.cext = 0;
}

// top of a step: the records loaded by the previous step become registers
// (a select on loaded data placed right after the load would wait for HBM there)
DEV void lane_top(Lane& L)
{
    if (!L.fwd) rec1_from(L.rc, L.epoch, L.cur);
    if (!L.q_fwd) rec2_from(L.rq, L.q);
}

// The next step's order-1 record R[v], issued as soon as v is known (the
// encoder: at the top of the step; the decoder: once v is decoded), so that
// its latency overlaps the rest of the step.  It is cur (v == b) or prv
// (v == a) when those are in flight -- the only records this step writes.
//
// Memory operations and waits: vmcnt counts loads and stores together, in
// issue order, and the compiler can only wait for a load with vmcnt(n) when n
// ops follow it on every path.  So the step's loads and stores are
// unconditional (a lane that needs none uses the scratch record), the
// order-1 record store is the step's last memory operation, and the next
// step waits for R[v] with vmcnt(4), not for the stores.  A conditional load
// would also make the compiler copy its result into the loop-carried
// registers right after issuing it, i.e. wait for it on the spot.
DEV void lane_prefetch(Lane& L, const uint8_t* reg, uint32_t v)
{
    L.nsame = L.order >= 1 && v == L.b;
    L.fromprv = !L.nsame && L.order >= 2 && !L.same && v == L.a;
    const bool ld = !L.nsame && !L.fromprv;
    raw_load(ld ? reg + kO1Base + v * kRec : L.dm, 0, L.rc);
    L.fwd = !ld;
}

// o2 context (a, b): escapes, total, and whether it takes part (compress.c:307, :536-544)
DEV void o2_stats(const Lane& L, uint32_t& esc, uint32_t& tot)
{
    const bool big = info_big(L.info);
    esc = big ? L.q.esc : (L.info ? kSubEscDelta : 0u);
    tot = big ? L.q.tot : (L.info ? kSubEscDelta + (L.info >> 8) : 0u);
}

// End of a step that produced v, found at level `at` (2, 1, 0: the context
// whose statistics coded it).  h1 = lookup of v in cur (valid for at <= 1 and,
// in the encoder, always), h2 = lookup of v in q (big o2 contexts).
//   1. update the o2 context (a, b): bump v (at == 2) or insert it
//   2. update the o1 context b (at <= 1): bump or insert
//   3. the o2 info of (b, v) and where it lives, the loads for step i+1
template <bool HAVE_H1, bool HOT = false>
DEV void lane_advance(Lane& L, uint8_t* reg, uint8_t* ldsb, uint32_t end, uint32_t v, int at, Look<3>& h1,
                      Look<6>& h2, bool new0, bool track, uint16_t* lc = nullptr, Hot* H = nullptr)
{
    // nodes compress.c creates this step: v in each visited context that lacks
    // it (the order-2 context is always visited, order 1 when order 2 did not
    // code v, the root when neither did -- new0, from the caller)
    uint32_t created = new0 ? 1u : 0u;
    // ---- 1. o2 context (a, b), compress.c:286-316
    uint32_t o2_new = 0;
    if (L.order >= 2) {
        const bool big = info_big(L.info);
        if (track) created += (big ? !h2.found : !(L.info != 0 && (L.info & 0xFF) == v)) ? 1u : 0u;
        uint32_t ni = L.info;
        // inline: empty -> (v, 2); (v, c) -> (v, c + 2) while c + 2 <= 127.
        // (A hit is v == the symbol, whatever level decoded v: a corrupt
        // stream can escape past a symbol it then patches, compress.c:598-615.)
        const uint32_t c0 = L.info >> 8;
        const bool ihit = !big && L.info != 0 && (L.info & 0xFF) == v;
        const bool iins = !big && L.info == 0;
        ni = ihit ? (L.info + (kSubDelta << 8)) : ni;
        ni = iins ? (v | (kSubDelta << 8)) : ni;
        // inline contexts that outgrow the encoding become a big record:
        // a second symbol, or a count past 127
        const bool conv = !big && L.info != 0 && (!ihit || c0 + kSubDelta > kInlineMax);
        if (any_lane(conv)) {
            // a fresh record holding the context after this update: the old
            // symbol bumped (count past 127), or the old symbol and v sorted
            // (escapes 5 + 5, total 5 + c0 + 5 + 2); no rescale is possible
            if (conv) {
                const uint32_t at64 = (L.bump + kRec - 1) & ~(kRec - 1);
                L.ovf = L.ovf || at64 + kRec > end;
                L.bump = at64 + kRec;
                const uint32_t s0 = L.info & 0xFF, lo = min(s0, v), hi = max(s0, v);
                const uint32_t clo = s0 < v ? c0 : kSubDelta, chi = s0 < v ? kSubDelta : c0;
                ctx_clear(L.q);
                L.q.len = ihit ? 1u : 2u;
                L.q.esc = ihit ? kSubEscDelta : 2 * kSubEscDelta;
                L.q.tot = ihit ? kSubEscDelta + c0 + kSubDelta : 2 * kSubEscDelta + c0 + kSubDelta;
                L.q.val[0] = ihit ? (0xFFFFFF00u | s0) : (0xFFFF0000u | (hi << 8) | lo);
                L.q.cnt[0] = ihit ? c0 + kSubDelta : ((chi << 8) | clo);
                L.qoff = at64;
                ni = 0x8000u | (at64 / kRec);
                L.q_dirty = true;
            }
        }
        if (any_lane(big)) {
            if (big && !L.ovf) {
                bool ovf = L.ovf != 0;
                ctx_update<6, false>(reg, ldsb, L.ldsu, L.q, h2, v, L.bump, end, ovf, true);
                L.ovf = ovf;
                L.q_dirty = true;
            }
        }
        o2_new = ni;
        // write the info back into its holder
        if (L.ipos == 0) {
            // (both, predicated: a select between the two records would put them in scratch)
            slot_set_info<3, true>(L.cur, L.eqp, ni, L.same && ni != L.info);
            slot_set_info<3, true>(L.prv, L.eqp, ni, !L.same && ni != L.info);
            L.prv_dirty = L.prv_dirty || (!L.same && ni != L.info);
        } else if (ni != L.info) {
            *reinterpret_cast<uint16_t*>(reg + L.ipos) = static_cast<uint16_t>(ni);
            // (the link cache: a copy of the cached block's first links)
            const uint32_t li = (L.ipos - L.cext - 288) >> 1;
            if (lc && L.cext != 0 && L.ipos >= L.cext + 288 && li < kLinkCache) lc[li] = static_cast<uint16_t>(ni);
        }
    }
    // ---- 2. o1 context b, compress.c:286-316 (its lookup, when the decoder did not need it)
    if (!HAVE_H1 && L.order >= 1 && at == 2) h1 = ctx_find<3, true>(reg, ldsb, L.cur, v);
    if (L.order >= 1 && at <= 1) {
        if (track) created += h1.found ? 0u : 1u;
        bool ovf = L.ovf != 0;
        const bool was = L.cur.dense != 0;
        ctx_update<3, true, HOT>(reg, ldsb, L.ldsu, L.cur, h1, v, L.bump, end, ovf, true, H, L.cext);
        L.ovf = ovf;
        // the decoder's first dense order-1 block: its links for symbols below
        // kLinkCache copied to the lane's LDS cache (once per packet)
        if (lc && any_lane(!was && L.cur.dense != 0 && L.cext == 0 && !L.ovf)) {
            if (!was && L.cur.dense != 0 && L.cext == 0 && !L.ovf) {
                L.cext = L.cur.ext;
                const uint4* src = reinterpret_cast<const uint4*>(reg + L.cext + 288);
                uint4* dst = reinterpret_cast<uint4*>(lc);
#pragma unroll
                for (uint32_t k = 0; k < 2 * kLinkCache / 16; ++k) dst[k] = src[k];
            }
            // (and its counts into the registers: it is the hot block from here on)
            if (HOT) {
                const bool nh = !was && L.cur.dense != 0 && L.cext == L.cur.ext && !L.ovf;
                const uint4* gp = reinterpret_cast<const uint4*>(reg + (nh ? L.cext + 32 : kDummyRec));
                uint4 q[16];
#pragma unroll
                for (uint32_t k = 0; k < 16; ++k) q[k] = gp[nh ? k : 0];
#pragma unroll
                for (uint32_t k = 0; k < 16; ++k) H->g[k] = sel_u4(nh, q[k], H->g[k]);
            }
        }
    }
    if (track) L.nodes += created;
    // ---- 3. next step: contexts (b, v)
    uint32_t ninfo = 0, nipos = 0;
    if (L.order >= 1) {
        ninfo = h1.found ? h1.info : 0u;                // a new symbol heads an empty context
        nipos = L.cur.dense ? L.cur.ext + 288 + 2 * v : 0u;
        // (b, v) == (a, b): the info was just rewritten above
        if (L.order >= 2 && L.same && v == L.b) ninfo = o2_new;
    }
    // big record of (b, v): keep q when it is the same record, else write q back and load
    const bool nbig = L.order >= 1 && info_big(ninfo);
    const uint32_t nqoff = nbig ? info_rec(ninfo) : 0u;
    // (q holds record qoff when (a, b) is big after this step's update, conversions included)
    const bool keepq = nbig && L.order >= 2 && info_big(o2_new) && nqoff == L.qoff;
    if (L.q_dirty && !keepq && L.order >= 2 && !L.ovf) { rec2_store(reg, L.qoff, L.q); L.q_dirty = false; }
    if (nbig && !keepq) raw_load(reg, nqoff, L.rq);
    L.q_fwd = !nbig || keepq;
    L.qoff = nbig ? nqoff : L.qoff;
    // order-1 record of v: cur (v == b), prv (v == a), or the load lane_prefetch issued
    const bool nsame = L.nsame, fromprv = L.fromprv;
    // (the step's last memory operation; see lane_prefetch)
    const bool st = L.order >= 2 && !L.same && !fromprv && L.prv_dirty;
    rec1_store_at(st ? reg + kO1Base + L.a * kRec : L.dm, 0, L.epoch, L.prv);
    // rotate: prv := cur, cur := R[v]
    Rec1 old = L.prv;
    if (L.order >= 1) {
        L.prv = L.cur;
        L.prv_dirty = true;              // cur was read-modify-written or now holds new o2 info
    }
    if (fromprv) L.cur = old;
    // slot of v in its holder (prv' = cur): one-hot from the lookup / insert
    L.eqp[0] = h1.eq[0]; L.eqp[1] = h1.eq[1]; L.eqp[2] = h1.eq[2];
    L.info = ninfo;
    L.ipos = nipos;
    L.same = nsame;
    L.a = L.b;
    L.b = v;
    L.order += L.order < 2 ? 1u : 0u;
}

// the records still in registers when the packet ends (nothing to do: the
// next packet starts a new epoch, so unwritten state is simply dropped)

// ------------------------------------------------------------ one packet

DEV void compress_one3(const rc_batch_dev& bt, const rc_workspace_dev& ws, uint32_t pkt, uint8_t* reg, uint8_t* root,
                       uint8_t* ldsb, const uint8_t* mtab, uint8_t* wave_reg = nullptr)
{
    const uint32_t len = bt.in_len[pkt];
    const uint32_t cap = bt.out_cap[pkt];
    if (len == 0) { bt.out_len[pkt] = 0; return; }                   // compress.c:257
    ByteSrc in;
    src_init(in, bt.in + bt.in_off[pkt], len);
    ByteSink o;
    sink_init(o, bt.out + bt.out_off[pkt], cap);
    const uint32_t end = ws.lane_region;
    Lane L;
    lane_init(L, reg, lane_dummy(reg, wave_reg));
    Root R;
    root3_clear<true>(root, R);
    uint32_t rtot = 1 + 256;
    uint32_t low = 0, range = ~0u;
    bool ok = true;

    // compress.c's node count only matters for packets that can reach the
    // model reset (> 1919 bytes); a wave counts when any of its lanes has one
    const bool track = any_lane(len > kMaxLen3);
    PROF_DECL
    for (uint32_t i = 0; i < len; ++i) {
#ifdef RC_PROFILE_DRAIN
        __builtin_amdgcn_s_waitcnt(0);
        PROF(9)
#endif
        const uint32_t v = src_byte(in);
        // the root lookup only needs v: its LDS latency overlaps the steps below
        uint32_t under0, cnt0;
        root3_lookup(root, mtab, v, under0, cnt0);
        lane_top(L);
        sink_flush(o);
        src_refill(in, true);
        PROF(0)
        lane_prefetch(L, reg, v);
        // order 2, compress.c:286-316
        uint32_t esc2, tot2;
        o2_stats(L, esc2, tot2);
        const bool en2 = L.order >= 2 && esc2 != 0;
        const bool big = info_big(L.info);
        Look<6> h2;
        h2.found = (L.info & 0xFF) == v ? 1u : 0u; h2.under = 0; h2.cnt = L.info >> 8;
        if (any_lane(en2 && big)) {
            if (en2 && big) h2 = ctx_find<6, false>(reg, ldsb, L.q, v);
        }
        const bool done2 = en2 && h2.found;
        PROF(1)
        enc_code(low, range, done2 ? esc2 + h2.under : 0u, done2 ? h2.cnt : esc2, tot2, o,
                 done2 || (en2 && esc2 < tot2), ok);
        PROF(2)
        // order 1
        const bool en1 = !done2 && L.order >= 1;
        Look<3> h1 = ctx_find<3, true>(reg, ldsb, L.cur, v);
        PROF(3)
        const bool done1 = en1 && h1.found;
        const uint32_t esc1 = L.cur.esc, tot1 = L.cur.tot;
        enc_code(low, range, done1 ? esc1 + h1.under : 0u, done1 ? h1.cnt : esc1, tot1, o,
                 done1 || (en1 && esc1 > 0 && esc1 < tot1), ok);
        PROF(4)
        // root, compress.c:318-329
        const bool en0 = !done2 && !done1;
        if (en0) root3_add<true>(root, R, v, cnt0);
        enc_code(low, range, 1 + under0, 1 + cnt0, rtot, o, en0, ok);
        rtot = en0 ? ((rtot + kRootDelta) & 0xFFFF) : rtot;
        const bool rs0 = en0 && (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit);
        if (any_lane(rs0)) { if (rs0) rtot = root3_rescale<true>(root, R); }
        PROF(5)
        // no loop exit between the record load (lane_prefetch) and the record
        // store (lane_advance): an exit path there makes the compiler's vmcnt
        // bookkeeping wait for the store at the top of every step
        lane_advance<true>(L, reg, ldsb, end, v, done2 ? 2 : done1 ? 1 : 0, h1, h2, en0 && cnt0 == 0, track);
        PROF(6)
        if (rare_lane(!ok || L.ovf)) { if (!ok || L.ovf) break; }
        if (track) {                                                  // compress.c:332 -> :148-157
            if (rare_lane(L.nodes >= kNodeLimit)) {
                if (L.nodes >= kNodeLimit) { lane_reset(L, reg); root3_clear<true>(root, R); rtot = 1 + 256; }
            }
        }
        PROF(7)
    }
    PROF_FLUSH(0)
    if (ok && L.ovf) { flag_exact(ws, pkt); return; }
    // flush, compress.c:139-146
    while (any_lane(ok && low != 0)) {
        const bool more = ok && low != 0;
        const bool full = more && o.n >= o.cap;
        ok = ok && !full;
        sink_put(o, low >> 24, 1, more && !full);
        low = (more && !full) ? low << 8 : low;
    }
    sink_finish(o, ok);
    bt.out_len[pkt] = ok ? o.n : 0u;
}

DEV void decompress_one3(const rc_batch_dev& bt, const rc_workspace_dev& ws, uint32_t pkt, uint8_t* reg,
                         uint8_t* root, uint8_t* ldsb, uint16_t* lc, uint8_t* wave_reg = nullptr)
{
    const uint32_t len = bt.in_len[pkt];
    const uint32_t cap = bt.out_cap[pkt];
    if (len == 0) { bt.out_len[pkt] = 0; return; }                   // compress.c:513
    ByteSink o;
    sink_init(o, bt.out + bt.out_off[pkt], cap);
    const uint32_t end = ws.lane_region;
    ByteSrc in;
    src_init(in, bt.in + bt.in_off[pkt], len);
    Lane L;
    lane_init(L, reg, lane_dummy(reg, wave_reg));
    Root R;
    root3_clear<false>(root, R);
    uint32_t rtot = 1 + 256;
    uint32_t low = 0, range = ~0u;
    uint32_t code = static_cast<uint32_t>(in.la >> 32);            // compress.c:344-350 (0 past the end)
    in.la <<= 32;
    in.na -= 4;
    src_refill(in, true);
    bool fail = false, anomaly = false;
    Hot H;                                   // (meaningful once L.cext is set)
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k) H.g[k] = make_uint4(0u, 0u, 0u, 0u);

    PROF_DECL
    for (;;) {
#ifdef RC_PROFILE_DRAIN
        __builtin_amdgcn_s_waitcnt(0);
        PROF(9)
#endif
        lane_top(L);
        sink_flush(o);
        src_fill(in, true);
        PROF(0)
        int at = -1;
        uint32_t v = 0;
        Look<3> h1;
        Look<6> h2;
        h1.found = 0u;
        bool new0 = false;
        uint32_t fu = 0, fc = 1, cnt0 = 0;       // the step's last code: applied after the prefetch below
        // order 2, compress.c:529-568
        uint32_t esc2, tot2;
        o2_stats(L, esc2, tot2);
        if (L.order >= 2 && esc2 > 0 && esc2 < tot2) {
            const uint32_t cd = dec_read(range, low, code, tot2, true);
            if (cd < esc2) {
                dec_code(low, code, range, 0, esc2, in, true);
            } else if (!info_big(L.info)) {
                if (cd - esc2 >= (L.info >> 8)) { fail = true; break; }
                v = L.info & 0xFF;
                h2.under = 0; h2.cnt = L.info >> 8;
                fu = esc2; fc = h2.cnt;
                at = 2;
            } else {
                if (!ctx_search<6, false>(reg, ldsb, L.q, cd - esc2, h2, v)) { fail = true; break; }
                fu = esc2 + h2.under; fc = h2.cnt;
                at = 2;
            }
        }
        PROF(1)
        // order 1
        if (at < 0 && L.order >= 1 && L.cur.esc > 0 && L.cur.esc < L.cur.tot) {
            const uint32_t cd = dec_read(range, low, code, L.cur.tot, true);
            if (cd < L.cur.esc) {
                dec_code(low, code, range, 0, L.cur.esc, in, true);
            } else {
                if (!o1_search(reg, L.cur, H, L.cext, lc, cd - L.cur.esc, h1, v)) { fail = true; break; }
                fu = L.cur.esc + h1.under; fc = h1.cnt;
                at = 1;
            }
        }
        PROF(2)
        // root, compress.c:570-596
        if (at < 0) {
            const uint32_t cd = dec_read(range, low, code, rtot, true);
            if (cd < 1) { dec_code(low, code, range, 0, 1, in, true); break; }   // end of stream
            if (cd - 1 >= rtot - 1) { anomaly = true; break; }           // past symbol 255
            uint32_t under, cnt;
            v = root3_search(root, R, cd - 1, under, cnt);
            new0 = cnt == 0;
            cnt0 = cnt;
            fu = 1 + under; fc = 1 + cnt;
            at = 0;
        }
        PROF(3)
#ifdef RC_PROFILE
        // event counts (lanes, summed per wave): steps in a dense order-1
        // context, its lookups (search or the root step's find), order-2 hits
        // whose next link misses the LDS cache, root steps
        {
            const bool dn = L.order >= 1 && L.cur.dense != 0;
            const bool lcv0 = dn && L.cext != 0 && L.cur.ext == L.cext && v < kLinkCache;
            prof_acc[7] += __builtin_popcountll(__builtin_amdgcn_ballot_w64(dn));
            prof_acc[8] += __builtin_popcountll(__builtin_amdgcn_ballot_w64(dn && at <= 1));
            prof_acc[10] += __builtin_popcountll(__builtin_amdgcn_ballot_w64(dn && at == 2 && !lcv0));
            prof_acc[11] += __builtin_popcountll(__builtin_amdgcn_ballot_w64(at == 0));
        }
#endif
        // the dense order-1 lookup of this step (a root step, or an order-2
        // hit whose link the LDS cache lacks): its group and link loaded
        // before the next record (the scratch record for lanes without one)
        const bool lcv = L.cur.dense != 0 && L.cext != 0 && L.cur.ext == L.cext && v < kLinkCache;
        const bool lk = L.order >= 1 && L.cur.dense != 0 && (at == 0 || (at == 2 && !lcv));
        // (the hot block's group from registers and, below symbol kLinkCache, its
        // link from the LDS cache: those lanes load the scratch record)
        const bool hotc = L.order >= 1 && is_hot(true, L.cext, L.cur.dense, L.cur.ext);
        Dense zp;
        zp.grp = *reinterpret_cast<const uint4*>(lk && !hotc ? reg + L.cur.ext + 32 + 16 * (v >> 4) : L.dm);
        zp.link = *reinterpret_cast<const uint16_t*>(lk && !lcv ? reg + L.cur.ext + 288 + 2 * v : L.dm);
        lane_prefetch(L, reg, v);
        // the step's last code and the root's update: only the next step
        // needs them, so they run after the record load is issued (as in
        // rc_dec4.hip)
        dec_code_late(low, code, range, fu, fc, in, true);
        if (at == 0) {
            root3_add<false>(root, R, v, cnt0);
            rtot = (rtot + kRootDelta) & 0xFFFF;
            if (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit) rtot = root3_rescale<false>(root, R);
        }
        // the patched o1 context needs v's lookup (compress.c:598-615); an
        // order-2 step needs the link of (b, v), from the LDS cache where it
        // holds v
        {
            const uint32_t lcl = lc[v & (kLinkCache - 1)];     // (read by every lane: its own register)
            if (any_lane(lk && hotc)) zp.grp = sel_u4(lk && hotc, hot_get(H, v >> 4), zp.grp);
            zp.link = lcv ? lcl : zp.link;
            if (L.order >= 1 && (at == 0 || (at == 2 && !lcv))) h1 = ctx_find_pre(L.cur, v, zp);
            const bool ul = at == 2 && L.order >= 1 && lcv;
            h1.info = ul ? lcl : h1.info;
            h1.found = ul ? 1u : h1.found;
        }
        if (at != 2 && L.order >= 2 && info_big(L.info)) h2 = ctx_find<6, false>(reg, ldsb, L.q, v);
        fail = o.n >= o.cap;                                         // compress.c:617
        PROF(4)
        lane_advance<true, kHot>(L, reg, ldsb, end, v, at, h1, h2, new0, true, lc, &H); // (see compress_one3)
        PROF(5)
        if (fail || L.ovf) break;
        if (rare_lane(L.nodes >= kNodeLimit)) {                      // compress.c:617-621 -> :148-157
            if (L.nodes >= kNodeLimit) { lane_reset(L, reg); root3_clear<false>(root, R); rtot = 1 + 256; }
        }
        sink_put(o, v, 1, true);
        src_adv(in);
        PROF(6)
    }
    PROF_FLUSH(16)
    if ((L.ovf && !fail) || anomaly) { flag_exact(ws, pkt); return; }
    sink_finish(o, !fail);
    bt.out_len[pkt] = fail ? 0u : o.n;
}

}  // namespace

extern "C" uint32_t rc_hip_lane3_region_bytes(uint32_t max_len)
{
    // header + order-1 table + arena.  Arena bound for <= kMaxLen3 bytes:
    // each byte adds at most one order-2 symbol; a big order-2 record needs
    // >= 2 symbols (64 B per 2 bytes), a dense order-2 block > 24 (288 B per
    // 24 bytes), a dense order-1 block > 12 symbols of its own (800 B per 12
    // bytes): <= 32 + 12 + 67 B per byte, plus alignment slack.
    // Longer packets reset the model at 4094 nodes (compress.c:148-157); one
    // model's arena is then bounded by its nodes: <= 67 B per order-1 symbol,
    // <= 44 B + 64-B alignment slack per two order-2 symbols; 80 B per node.
    // (An overflow is still caught: the packet takes the exact path.)
    const uint64_t L = max_len < kMaxLen3 ? max_len : kMaxLen3;
    uint64_t bytes = max_len <= kMaxLen3 ? kArena3 + 112 * L + 4096 : kArena3 + 80ull * kNodeLimit + 4096;
    bytes = (bytes + 255) & ~255ull;
    return static_cast<uint32_t>(bytes);
}

#ifndef RC_LANE_HOST_TEST
template <bool DECOMP>
DEV void lane3_main(const rc_batch_dev& b, const rc_workspace_dev& ws)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t act = ws.lane_active;
    const uint32_t wave = threadIdx.x >> 6, l = threadIdx.x & 63;
    uint8_t* mtab = smem + 4 * act * kRootStride3;
    if (!DECOMP) {
        if (threadIdx.x < 16) root3_mask_init(mtab, threadIdx.x);
        __syncthreads();
    }
    if (l >= act) return;
    const uint32_t local = wave * act + l;
    uint8_t* root = smem + local * (DECOMP ? kRootStrideDec : kRootStride3);
    uint8_t* ldsb = smem + (DECOMP ? 4 * act * kRootStrideDec : 4 * act * kRootStride3 + 256) + local * kDenseO2;
    uint16_t* lc = reinterpret_cast<uint16_t*>(smem + 4 * act * (kRootStrideDec + kDenseO2) + local * 2 * kLinkCache);
    const uint32_t per_block = 4 * act;
    const uint32_t slot = blockIdx.x * per_block + local;
    uint8_t* reg = static_cast<uint8_t*>(ws.lane_pool) + static_cast<size_t>(slot) * ws.lane_region;
    uint8_t* wave_reg = static_cast<uint8_t*>(ws.lane_pool) + static_cast<size_t>(slot - l) * ws.lane_region;
    const uint32_t* order = ws.order && !ws.bins[RC_LEN_BINS] ? ws.order : nullptr;
    const uint32_t count = ws.sub_count ? *ws.sub_count : b.n;   // a sub-list: the two-pass encoder's leftovers
    for (uint32_t i = slot; i < count; i += gridDim.x * per_block) {
        const uint32_t pkt = ws.sub_list ? ws.sub_list[i] : (order ? order[i] : i);
        if (DECOMP) decompress_one3(b, ws, pkt, reg, root, ldsb, lc, wave_reg);
        else compress_one3(b, ws, pkt, reg, root, ldsb, mtab, wave_reg);
    }
}

// one wave per SIMD by design (a packet per lane, 65536 lanes fill the chip),
// so the kernels may use the whole register file
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void rc_compress_lane3(rc_batch_dev b, rc_workspace_dev ws) { lane3_main<false>(b, ws); }

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void rc_decompress_lane3(rc_batch_dev b, rc_workspace_dev ws) { lane3_main<true>(b, ws); }

extern "C" int rc_hip_lane3_launch(int decompress, const rc_batch_dev* b, const rc_workspace_dev* ws,
                                   uint32_t blocks, void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    // the encoder: roots with their D copy + the mask table; the decoder: roots;
    // then a dense order-2 block per lane
    // (+ the decoder's link cache)
    const size_t lds = (decompress ? static_cast<size_t>(4 * ws->lane_active) * (kRootStrideDec + 2 * kLinkCache)
                                   : static_cast<size_t>(4 * ws->lane_active) * kRootStride3 + 256) +
                       static_cast<size_t>(4 * ws->lane_active) * kDenseO2;
    if (decompress)
        hipLaunchKernelGGL(rc_decompress_lane3, dim3(blocks), dim3(256), lds, st, *b, *ws);
    else
        hipLaunchKernelGGL(rc_compress_lane3, dim3(blocks), dim3(256), lds, st, *b, *ws);
    return static_cast<int>(hipGetLastError());
}
#endif  // RC_LANE_HOST_TEST
