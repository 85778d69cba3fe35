// rc_bucket4.h -- the bucket-history model of the decoder (rc_dec4.hip):
// one 64-B record per previous byte p listing the positions
// decoded so far with x[j-1] = p (compress.c:159-199, :536-615; see
// rc_dec4.hip for the algebra).  Include after rc_lane_common.h / rc_root3.h.
#pragma once

namespace {

constexpr uint32_t kCap4 = 24;              // elements per bucket record
constexpr uint32_t kRec4 = 64;
constexpr uint32_t kNodeLimit4 = 4096 - 2;  // compress.c:148-157

// bucket record (16 dwords):
//   w0  tag | k << 16 | nh2 << 21 | nn1 << 26  (k elements; nh2 of them decoded
//       at order 2; nn1 new to order 1 when added)
//   w1  hit mask: element decoded at order 2           (bit i = element i)
//   w2  new mask: element new to its order-2 context
//   w3  run mask: element's value differs from its predecessor's
//   w4..9   a[24] (the byte before the bucket byte)
//   w10..15 v[24] (ascending, stable; 0xFF past k)
// Position 1 has no order-2 context: its element carries hit and new, a
// combination no other element has (a hit is never new), which keeps it out
// of every order-2 group and in its order-1 group.  A tag other than the
// lane's epoch reads as an empty bucket.
struct Bucket { uint32_t h, hit, nw, run; uint32_t a[6], v[6]; };
struct Raw4 { uint4 q0, q1, q2, q3; };

DEV uint32_t bk_k(uint32_t h) { return (h >> 16) & 31; }

DEV void raw4_load(const uint8_t* reg, uint32_t off, Raw4& w)
{
    const uint4* p = reinterpret_cast<const uint4*>(reg + off);
    w.q0 = p[0]; w.q1 = p[1]; w.q2 = p[2]; w.q3 = p[3];
}

DEV void bk_empty(Bucket& B, uint32_t epoch)
{
    B.h = epoch; B.hit = 0; B.nw = 0; B.run = 0;
#pragma unroll
    for (uint32_t d = 0; d < 6; ++d) { B.a[d] = 0u; B.v[d] = 0xFFFFFFFFu; }
}

DEV void bk_from(const Raw4& w, uint32_t epoch, Bucket& B)
{
    const bool live = (w.q0.x & 0xFFFFu) == epoch;
    const uint32_t f = live ? 0xFFFFFFFFu : 0u;
    B.h = live ? w.q0.x : epoch;
    B.hit = w.q0.y & f; B.nw = w.q0.z & f; B.run = w.q0.w & f;
    B.a[0] = w.q1.x; B.a[1] = w.q1.y; B.a[2] = w.q1.z; B.a[3] = w.q1.w; B.a[4] = w.q2.x; B.a[5] = w.q2.y;
    B.v[0] = w.q2.z | ~f; B.v[1] = w.q2.w | ~f; B.v[2] = w.q3.x | ~f;
    B.v[3] = w.q3.y | ~f; B.v[4] = w.q3.z | ~f; B.v[5] = w.q3.w | ~f;
}

DEV void bk_store(uint8_t* reg, uint32_t off, const Bucket& B)
{
    uint4* p = reinterpret_cast<uint4*>(reg + off);
    p[0] = make_uint4(B.h, B.hit, B.nw, B.run);
    p[1] = make_uint4(B.a[0], B.a[1], B.a[2], B.a[3]);
    p[2] = make_uint4(B.a[4], B.a[5], B.v[0], B.v[1]);
    p[3] = make_uint4(B.v[2], B.v[3], B.v[4], B.v[5]);
}

// 0x01 in each byte where x and y agree
DEV uint32_t eq01(uint32_t x, uint32_t y)
{
    const uint32_t z = x ^ y;
    const uint32_t t = ((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z;
    return (~t >> 7) & 0x01010101u;
}

// the 0x01 bytes of e as four bits
DEV uint32_t gather4(uint32_t e) { return (e | (e >> 7) | (e >> 14) | (e >> 21)) & 0xFu; }

// ny for swar_ge: 0x01 in each byte >= u (u <= 256)
DEV uint32_t ny_of(uint32_t u) { return 0x01000100u - u * 0x00010001u; }

DEV uint32_t popc(uint32_t x) { return static_cast<uint32_t>(__builtin_popcount(x)); }
DEV uint32_t low_bits(uint32_t n) { return n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u); }

// the two sub-contexts of a position, as bit masks over the bucket's elements
struct Groups {
    uint32_t g2, g1;            // members: order 2 (a, p), order 1 (p)
    uint32_t t2, d2, t1, d1;    // members, members added as new symbols
};

// Dwords of the byte arrays that hold an element, or the insertion point, in
// any lane of the wave (a wave-uniform count: the rest is skipped).
DEV uint32_t live_dwords(uint32_t k)
{
    uint32_t nd = 1;
#pragma unroll
    for (uint32_t d = 1; d < 6; ++d) nd += any_lane(k >= 4 * d) ? 1u : 0u;
    return nd;
}

DEV void bk_groups(const Bucket& B, uint32_t nd, uint32_t acur, bool o2, Groups& s)
{
    const uint32_t k = bk_k(B.h), km = low_bits(k);
    const uint32_t ap = acur * 0x01010101u;
    uint32_t am = 0;
#pragma unroll
    for (uint32_t d = 0; d < 6; ++d)
        if (d < nd) am |= gather4(eq01(B.a[d], ap)) << (4 * d);
    s.g2 = o2 ? (am & km & ~(B.hit & B.nw)) : 0u;
    s.g1 = (~B.hit | B.nw) & km;
    s.t2 = popc(s.g2);
    s.d2 = popc(s.g2 & B.nw);
    s.t1 = k - ((B.h >> 21) & 31);
    s.d1 = (B.h >> 26) & 31;
}

// index of the member of rank r (0-based) of the bit set g: the largest j
// with fewer than r + 1 members below j
DEV uint32_t select_bit(uint32_t g, uint32_t r)
{
    uint32_t j = 0;
#pragma unroll
    for (uint32_t step = 16; step >= 1; step >>= 1) {
        const uint32_t jj = j + step;
        j = popc(g & low_bits(jj)) <= r ? jj : j;
    }
    return j;
}

// byte j of a 24-byte array (a masked OR: a select chain on a lane-varying
// index compiles to a dynamically indexed scratch load)
DEV uint32_t byte_at(const uint32_t* x, uint32_t j)
{
    const uint32_t d = j >> 2;
    uint32_t w = 0;
#pragma unroll
    for (uint32_t e = 0; e < 6; ++e) w |= x[e] & (0u - static_cast<uint32_t>(d == e));
    return (w >> (8 * (j & 3))) & 0xFFu;
}

// elements with a value below u, and at most u (the bucket is sorted: the
// elements equal to u are [lt, le))
DEV void bk_rank(const Bucket& B, uint32_t nd, uint32_t u, uint32_t& lt, uint32_t& le)
{
    const uint32_t n0 = ny_of(u), n1 = ny_of(u + 1);
    uint32_t ge0 = 0, ge1 = 0;
#pragma unroll
    for (uint32_t d = 0; d < 6; ++d) {
        if (d < nd) {
            ge0 = sad(swar_ge(B.v[d], n0), ge0);
            ge1 = sad(swar_ge(B.v[d], n1), ge1);
        }
    }
    const uint32_t k = bk_k(B.h);
    lt = 4 * nd - ge0;                        // (slots past k hold 0xFF: never below u)
    le = min(4 * nd - ge1, k);                // (... but at most 0xFF: u = 255 counts them)
}

// compress.c:536-568 in one sub-context: READ, then an escape (false) or the
// member the code selects (true; v and its member index j: the caller codes
// its interval, hit_interval, after issuing the next record load).  fail: the
// code is past the context's symbols (compress.c:416).
DEV bool sub_decode(const Bucket& B, uint32_t g, uint32_t t, uint32_t dd, double rtot, uint32_t& low,
                    uint32_t& code, uint32_t& range, ByteSrc& in, uint32_t& v, uint32_t& j, bool& fail)
{
    const uint32_t esc = kSubEscDelta * dd, tot = esc + kSubDelta * t;
    const uint32_t cd = dec_read_d(range, low, code, tot, rtot);
    if (cd < esc) {
        dec_code(low, code, range, 0, esc, in, true);
        return false;
    }
    const uint32_t r = cd - esc;
    if (r >= kSubDelta * t) { fail = true; return false; }
    j = select_bit(g, r >> 1);
    v = byte_at(B.v, j);
    return true;
}

// the interval of member j's value in the sub-context of members g with
// escapes esc: the members with that value form the run of the run mask
// that holds j
DEV void hit_interval(const Bucket& B, uint32_t g, uint32_t esc, uint32_t j, uint32_t& under, uint32_t& count)
{
    const uint32_t upto = low_bits(j + 1);
    const uint32_t lo = 31u - static_cast<uint32_t>(__builtin_clz(B.run & upto));   // (bit 0 is a run start)
    const uint32_t above = B.run & ~upto & low_bits(bk_k(B.h));
    const uint32_t hi = above ? static_cast<uint32_t>(__builtin_ctz(above)) : bk_k(B.h);
    const uint32_t less = popc(g & low_bits(lo)), same = popc(g & low_bits(hi)) - less;
    under = esc + kSubDelta * less;
    count = kSubDelta * same;
}

// bit pos of m gets b, bits above move up one
DEV uint32_t bit_insert(uint32_t m, uint32_t pos, uint32_t b)
{
    const uint32_t lo = low_bits(pos);
    return (m & lo) | ((m & ~lo) << 1) | (b << pos);
}

// the element (a, v) joins the bucket at pos (after the values <= v)
DEV void bk_insert(Bucket& B, uint32_t nd, uint32_t pos, uint32_t a, uint32_t v, uint32_t hit, uint32_t nw,
                   uint32_t run, uint32_t hadd, bool en)
{
    const int pp = static_cast<int>(pos);
    const uint32_t ar = a * 0x01010101u, vr = v * 0x01010101u;
    uint32_t pa = 0, pv = 0;
#pragma unroll
    for (uint32_t d = 0; d < 6; ++d) {
        if (d < nd) {
            // bytes below pos stay, byte pos is new, bytes above move up one
            const uint32_t keep = en ? below_mask(pp, static_cast<int>(d)) : 0xFFFFFFFFu;
            const uint32_t im = en ? byte_mask(pp, static_cast<int>(d)) : 0u;
            const uint32_t ca = B.a[d], cv = B.v[d];
            B.a[d] = (ca & keep) | (align8(ca, pa, 3) & ~keep & ~im) | (ar & im);
            B.v[d] = (cv & keep) | (align8(cv, pv, 3) & ~keep & ~im) | (vr & im);
            pa = ca; pv = cv;
        }
    }
    B.hit = en ? bit_insert(B.hit, pos, hit) : B.hit;
    B.nw = en ? bit_insert(B.nw, pos, nw) : B.nw;
    B.run = en ? bit_insert(B.run, pos, run) : B.run;
    B.h += en ? hadd : 0u;
}

DEV void bail(const rc_workspace_dev& ws, uint32_t pkt)
{
    const uint32_t slot = atomicAdd(&ws.counters[3], 1u);
    ws.enc2_list[slot] = pkt;
}

}  // namespace
