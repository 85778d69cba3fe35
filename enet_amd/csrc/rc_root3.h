// rc_root3.h -- the order-0 (root) context of one lane: counts in LDS, the
// cumulative group boundaries in registers (compress.c:159-199, :318-329,
// :570-596, :90-112).  Shared by the lane kernels (rc_lane3.hip) and the
// bucket-history decoder (rc_dec4.hip).  Include after rc_lane_common.h.
#pragma once

namespace {

// ------------------------------------------------------------ order 0
// Per lane: counts[256] (u8) in LDS; the 16 group boundaries in registers,
// D[t] = 16 (t + 1) + the counts of symbols < 16 (t + 1) -- the cumulative
// frequency including every symbol's minimum 1 (compress.c:159-199) -- as
// packed u16 pairs d[i] = D[2i] | D[2i + 1] << 16.  The root total is
// 1 + D[15].  The encoder also keeps a copy of D in LDS after the counts, so
// that a lookup is three independent LDS reads (the symbol's 16-B group, D of
// the groups below, the prefix mask of its position in the group from a
// block-wide table) and no register selects; an update writes one byte (and
// the encoder's copy of D).  The decoder finds the group with packed compares
// on the registers (no LDS reads).
constexpr uint32_t kRootStride3 = 304;   // counts[256], D[16] (u16), pad
constexpr uint32_t kRootStrideDec = 272; // decoders (no D copy): counts[256], pad (68 dwords: b128 conflict-free)
constexpr uint32_t kRootD = 256;

struct Root { uint32_t d[8]; };

// Layout of one lane's root: ROW is the distance between its 16-B rows (the
// 16 count groups, then the two rows of the D copy).  ROW = 16: the rows back
// to back (the lane kernels, the decoders, the one-wavefront code pass).
// The two-wavefront code pass's helpers keep their roots transposed, row g
// of every lane side by side (ROW = 16 x the block's lanes): a lane's random
// group read then hits banks of its own, where 256 roots at one stride put
// the lanes of a wavefront on random banks (rc_enc2.hip kC2Row).
template <uint32_t ROW> DEV uint32_t rofs(uint32_t v) { return ROW * (v >> 4) + (v & 15); }   // count of v
template <uint32_t ROW> DEV uint32_t rdofs(uint32_t h) { return ROW * (16 + h); }             // D row h

// the block-wide table of prefix masks: entry j has bytes 0..j-1 set
DEV void root3_mask_init(uint8_t* tab, uint32_t j)
{
    uint32_t w[4];
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d) {
        const uint32_t nb = j > 4 * d ? min(j - 4 * d, 4u) : 0u;
        w[d] = nb >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
    }
    reinterpret_cast<uint4*>(tab)[j] = make_uint4(w[0], w[1], w[2], w[3]);
}

template <bool COPY, uint32_t ROW = 16>
DEV void root3_store_d(uint8_t* r, const Root& R)
{
    if (COPY) {
        *reinterpret_cast<uint4*>(r + rdofs<ROW>(0)) = make_uint4(R.d[0], R.d[1], R.d[2], R.d[3]);
        *reinterpret_cast<uint4*>(r + rdofs<ROW>(1)) = make_uint4(R.d[4], R.d[5], R.d[6], R.d[7]);
    }
}

template <bool COPY, uint32_t ROW = 16>
DEV void root3_clear(uint8_t* r, Root& R)
{
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) *reinterpret_cast<uint4*>(r + ROW * i) = z;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) R.d[i] = (32 * i + 16) | ((32 * i + 32) << 16);
    root3_store_d<COPY, ROW>(r, R);
}

// Encoder: the block-wide table of D increments, entry g = +3 in every D[t]
// with t >= g (packed like R.d), so that an update of the LDS copy of D is
// two table reads and eight adds (no carry can cross a half: D <= 64256).
DEV void root3_inc_init(uint8_t* tab, uint32_t g)
{
    uint32_t w[8];
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i)
        w[i] = (2 * i >= g ? kRootDelta : 0u) | ((2 * i + 1 >= g ? kRootDelta : 0u) << 16);
    reinterpret_cast<uint4*>(tab)[2 * g] = make_uint4(w[0], w[1], w[2], w[3]);
    reinterpret_cast<uint4*>(tab)[2 * g + 1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// encoder update: count[v] and the LDS copy of D (the registers R.d are not kept)
DEV void root3_add_tab(uint8_t* r, const uint8_t* itab, uint32_t v, uint32_t cnt)
{
    r[v] = static_cast<uint8_t>(cnt + kRootDelta);
    const uint4* ip = reinterpret_cast<const uint4*>(itab + 32 * (v >> 4));
    uint4* dp = reinterpret_cast<uint4*>(r + kRootD);
    uint4 d0 = dp[0], d1 = dp[1];
    const uint4 i0 = ip[0], i1 = ip[1];
    d0.x += i0.x; d0.y += i0.y; d0.z += i0.z; d0.w += i0.w;
    d1.x += i1.x; d1.y += i1.y; d1.z += i1.z; d1.w += i1.w;
    dp[0] = d0;
    dp[1] = d1;
}

// root3_add_tab in two halves: the reads, issued early in a step, and the
// writes, after the step's codes (no wait for the reads on the coder's chain)
struct RootAddPre { uint4 d0, d1, i0, i1; };
template <uint32_t ROW = 16>
DEV RootAddPre root3_add_read(const uint8_t* r, const uint8_t* itab, uint32_t v)
{
    const uint4* ip = reinterpret_cast<const uint4*>(itab + 32 * (v >> 4));
    return RootAddPre{*reinterpret_cast<const uint4*>(r + rdofs<ROW>(0)), *reinterpret_cast<const uint4*>(r + rdofs<ROW>(1)),
                      ip[0], ip[1]};
}
template <uint32_t ROW = 16>
DEV void root3_add_write(uint8_t* r, uint32_t v, uint32_t cnt, RootAddPre a)
{
    r[rofs<ROW>(v)] = static_cast<uint8_t>(cnt + kRootDelta);
    a.d0.x += a.i0.x; a.d0.y += a.i0.y; a.d0.z += a.i0.z; a.d0.w += a.i0.w;
    a.d1.x += a.i1.x; a.d1.y += a.i1.y; a.d1.z += a.i1.z; a.d1.w += a.i1.w;
    *reinterpret_cast<uint4*>(r + rdofs<ROW>(0)) = a.d0;
    *reinterpret_cast<uint4*>(r + rdofs<ROW>(1)) = a.d1;
}

// D[g - 1] from the lane's D copy (g >= 1; g = 0 reads D[15], unused)
template <uint32_t ROW>
DEV uint32_t root3_dprev(const uint8_t* r, uint32_t g)
{
    if (ROW == 16) return reinterpret_cast<const uint16_t*>(r + kRootD)[static_cast<int>(g) - 1];
    const uint32_t t = (g - 1) & 15;
    return *reinterpret_cast<const uint16_t*>(r + rdofs<ROW>(t >> 3) + 2 * (t & 7));
}

// under = cumulative frequency below v, cnt = count[v] (compress.c:159-199, minimum 1)
template <uint32_t ROW = 16>
DEV void root3_lookup(const uint8_t* r, const uint8_t* mtab, uint32_t v, uint32_t& under, uint32_t& cnt)
{
    const uint32_t g = v >> 4, j = v & 15;
    const uint4 q = *reinterpret_cast<const uint4*>(r + ROW * g);
    const uint4 m = *reinterpret_cast<const uint4*>(mtab + 16 * j);
    const uint32_t dprev = root3_dprev<ROW>(r, g);
    cnt = r[rofs<ROW>(v)];
    const uint32_t within = sad(q.w & m.w, sad(q.z & m.z, sad(q.y & m.y, sad(q.x & m.x, 0u))));
    under = (g ? dprev : 0u) + j + within;
}

// root3_lookup in two halves: the LDS reads (several issued together by the
// encoder's helper) and the sums
struct RootLk { uint4 q, m; uint32_t dprev, cnt; };
template <uint32_t ROW = 16>
DEV RootLk root3_lookup_read(const uint8_t* r, const uint8_t* mtab, uint32_t v)
{
    const uint32_t g = v >> 4, j = v & 15;
    RootLk l;
    l.q = *reinterpret_cast<const uint4*>(r + ROW * g);
    l.m = *reinterpret_cast<const uint4*>(mtab + 16 * j);
    l.dprev = root3_dprev<ROW>(r, g);
    l.cnt = r[rofs<ROW>(v)];
    return l;
}
DEV void root3_lookup_sum(const RootLk& l, uint32_t v, uint32_t& under, uint32_t& cnt)
{
    const uint32_t within = sad(l.q.w & l.m.w, sad(l.q.z & l.m.z, sad(l.q.y & l.m.y, sad(l.q.x & l.m.x, 0u))));
    under = ((v >> 4) ? l.dprev : 0u) + (v & 15) + within;
    cnt = l.cnt;
}

template <bool COPY>
DEV void root3_add(uint8_t* r, Root& R, uint32_t v, uint32_t cnt)
{
    r[v] = static_cast<uint8_t>(cnt + kRootDelta);
    cum_add(R.d, v >> 4, kRootDelta);
    root3_store_d<COPY>(r, R);
}

// decoder update with the block-wide increment table (root3_inc_init): count[v]
// and the registers D by two LDS reads and eight adds (no carry can cross a
// half: D <= 64256) instead of cum_add's compares
DEV void root3_add_inc(uint8_t* r, Root& R, const uint8_t* itab, uint32_t v, uint32_t cnt)
{
    r[v] = static_cast<uint8_t>(cnt + kRootDelta);
    const uint4* ip = reinterpret_cast<const uint4*>(itab + 32 * (v >> 4));
    const uint4 i0 = ip[0], i1 = ip[1];
    R.d[0] += i0.x; R.d[1] += i0.y; R.d[2] += i0.z; R.d[3] += i0.w;
    R.d[4] += i1.x; R.d[5] += i1.y; R.d[6] += i1.z; R.d[7] += i1.w;
}

// Decoder: the symbol whose interval holds code (code < root total - 1):
// g = #{t : D[t] <= code} by packed saturating compares, then halving on byte
// sums inside group g.  Returns v; under = its cumulative frequency, cnt = count[v].
DEV uint32_t root3_search(const uint8_t* r, const Root& R, uint32_t code, uint32_t& under, uint32_t& cnt)
{
    const uint32_t x1 = (code + 1) * 0x00010001u;
    // (sums and maxima as trees, not chains: this is on the decoder's critical path)
    uint32_t b[8], m[8];
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
        b[i] = pk_min(pk_subsat(x1, R.d[i]), 0x00010001u);             // 1 where D <= code
        m[i] = pk_mul(R.d[i], b[i]);
    }
    const uint32_t acc = pk_add(pk_add(pk_add(b[0], b[1]), pk_add(b[2], b[3])),
                                pk_add(pk_add(b[4], b[5]), pk_add(b[6], b[7])));
    const uint32_t pm = pk_max(pk_max(pk_max(m[0], m[1]), pk_max(m[2], m[3])),
                               pk_max(pk_max(m[4], m[5]), pk_max(m[6], m[7])));
    const uint32_t g = (acc & 0xFFFF) + (acc >> 16);
    const uint32_t prev = max(pm & 0xFFFF, pm >> 16);                 // D[g - 1], 0 for g = 0
    const uint4 q = *reinterpret_cast<const uint4*>(r + 16 * g);
    uint32_t base = prev, j = 0;
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

// root3_search that also reads the increment table's entry of the symbol's
// group (root3_inc_init) right behind the group itself, so that the update
// after it (root3_add_pre) waits for no LDS round trip of its own
DEV uint32_t root3_search_inc(const uint8_t* r, const Root& R, const uint8_t* itab, uint32_t code, uint32_t& under,
                              uint32_t& cnt, uint4& i0, uint4& i1)
{
    const uint32_t x1 = (code + 1) * 0x00010001u;
    uint32_t b[8], m[8];
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) {
        b[i] = pk_min(pk_subsat(x1, R.d[i]), 0x00010001u);             // 1 where D <= code
        m[i] = pk_mul(R.d[i], b[i]);
    }
    const uint32_t acc = pk_add(pk_add(pk_add(b[0], b[1]), pk_add(b[2], b[3])),
                                pk_add(pk_add(b[4], b[5]), pk_add(b[6], b[7])));
    const uint32_t pm = pk_max(pk_max(pk_max(m[0], m[1]), pk_max(m[2], m[3])),
                               pk_max(pk_max(m[4], m[5]), pk_max(m[6], m[7])));
    const uint32_t g = (acc & 0xFFFF) + (acc >> 16);
    const uint32_t prev = max(pm & 0xFFFF, pm >> 16);                 // D[g - 1], 0 for g = 0
    const uint4 q = *reinterpret_cast<const uint4*>(r + 16 * g);
    const uint4* ip = reinterpret_cast<const uint4*>(itab + 32 * (g & 15));
    i0 = ip[0];
    i1 = ip[1];
    uint32_t base = prev, j = 0;
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

// root3_add_inc with the table entry of v's group already read (root3_search_inc)
DEV void root3_add_pre(uint8_t* r, Root& R, uint32_t v, uint32_t cnt, const uint4& i0, const uint4& i1)
{
    r[v] = static_cast<uint8_t>(cnt + kRootDelta);
    R.d[0] += i0.x; R.d[1] += i0.y; R.d[2] += i0.z; R.d[3] += i0.w;
    R.d[4] += i1.x; R.d[5] += i1.y; R.d[6] += i1.z; R.d[7] += i1.w;
}

// compress.c:90-112 for the root: halve the counts, rebuild D; returns the new total
template <bool COPY, uint32_t ROW = 16>
DEV uint32_t root3_rescale(uint8_t* r, Root& R)
{
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t g = 0; g < 16; ++g) {
        uint4 q = *reinterpret_cast<uint4*>(r + ROW * g);
        q.x -= (q.x >> 1) & 0x7F7F7F7Fu;
        q.y -= (q.y >> 1) & 0x7F7F7F7Fu;
        q.z -= (q.z >> 1) & 0x7F7F7F7Fu;
        q.w -= (q.w >> 1) & 0x7F7F7F7Fu;
        *reinterpret_cast<uint4*>(r + ROW * g) = q;
        sum = sad(q.w, sad(q.z, sad(q.y, sad(q.x, sum))));
        const uint32_t dg = sum + 16 * (g + 1);
        if (g & 1) R.d[g >> 1] |= dg << 16; else R.d[g >> 1] = dg;
    }
    root3_store_d<COPY, ROW>(r, R);
    return (sum + 1 + 256) & 0xFFFF;
}

}  // namespace
