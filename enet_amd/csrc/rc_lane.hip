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

#include "rc_lane_common.h"

namespace {

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

constexpr uint32_t kO1NV = 3, kO2Rec = 32, kO2NV = 2;
constexpr uint32_t kArenaBase = kO1Base + 256 * kO1Rec;
constexpr uint32_t kDenseBudget = 0xFFFFFFFFu;   // dense blocks are bounded by the region size

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


DEV void compress_one(const rc_batch_dev& b, const rc_workspace_dev& ws, uint32_t pkt,
                      uint8_t* reg, uint8_t* root)
{
    const uint32_t len = b.in_len[pkt];
    const uint32_t cap = b.out_cap[pkt];
    if (len == 0) { b.out_len[pkt] = 0; return; }                   // compress.c:257
    ByteSrc in;
    src_init(in, b.in + b.in_off[pkt], len);
    ByteSink o;
    sink_init(o, b.out + b.out_off[pkt], cap);
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
        sink_flush(o);
        const uint32_t v = src_byte(in);
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
        src_refill(in, true);
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
        sink_put(o, low >> 24, 1, more && !full);
        low = (more && !full) ? low << 8 : low;
    }
    sink_finish(o, ok);
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
    ByteSink o;
    sink_init(o, b.out + b.out_off[pkt], cap);
    const uint32_t end = ws.lane_region;
    ByteSrc in;
    src_init(in, b.in + b.in_off[pkt], len);

    uint32_t epoch = next_epoch(reg, *reinterpret_cast<const uint32_t*>(reg));
    root_clear(root);
    uint32_t rtot = 1 + 256, bump = kArenaBase, nodes = 1, dense_left = kDenseBudget;
    uint32_t order = 0, b1 = 0;
    uint32_t low = 0, code = 0, range = ~0u;
    code = static_cast<uint32_t>(in.la >> 32);                   // compress.c:344-350 (0 past the end)
    in.la <<= 32;
    in.na -= 4;
    src_refill(in, true);
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
        sink_flush(o);
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
        sink_put(o, v, 1, true);
        PROF(7)
        if (order >= 1 && !same2) {
            if (ld2) o2_decode(n2, nxt, r2);
            else ctx_empty(r2, nxt * kO2Rec, 0u);
        }
        if (!(order >= 1 && v == b1)) o1_decode(n1, epoch & 0xFFFF, r1);
        if (order < 2) ++order;
        b1 = v;
        src_refill(in, true);
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
    sink_finish(o, !fail);
    b.out_len[pkt] = fail ? 0u : o.n;
}

}  // namespace


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

extern "C" int rc_hip_lane3_launch(int decompress, const rc_batch_dev* b, const rc_workspace_dev* ws,
                                   uint32_t blocks, void* stream);   // rc_lane3.hip

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
    if (ws->kernel == RC_KERNEL_LANE3 && !decompress && ws->enc2_stream) {
        // the two-pass encoder takes what it can (rc_enc2.hip); the lanes run
        // only the packets it lists
        const int rc = rc_hip_enc2_launch(b, &w, stream);
        if (rc != 0) return rc;
        w.sub_list = ws->enc2_list;
        w.sub_count = ws->counters + 3;
    }
    if (ws->kernel == RC_KERNEL_LANE3 && decompress && ws->dec4) {
        // the bucket-history decoder takes what it can (rc_dec4.hip); the
        // lanes decode only the packets it lists
        const int rc = rc_hip_dec4_launch(b, &w, blocks, stream);
        if (rc != 0) return rc;
        w.sub_list = ws->enc2_list;
        w.sub_count = ws->counters + 3;
    }
    if (ws->kernel == RC_KERNEL_LANE3) return rc_hip_lane3_launch(decompress, b, &w, blocks, stream);
    if (decompress)
        hipLaunchKernelGGL(rc_decompress_lane, dim3(blocks), dim3(256), lds, st, *b, w);
    else
        hipLaunchKernelGGL(rc_compress_lane, dim3(blocks), dim3(256), lds, st, *b, w);
    return static_cast<int>(hipGetLastError());
}
#endif  // RC_LANE_HOST_TEST
