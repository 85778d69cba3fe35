// rc_dec6_rare.h -- the record-light decoder's exact step over a bucket's
// elements (rc_dec6.hip's rare phase): compress.c:536-568 in the order-2 and
// order-1 contexts of position j, both rebuilt from the elements of bucket
// x[j-1] (the bucket algebra of rc_dec6.hip's header; tests/proto/histdec.py
// restates it).  Include after rc_lane_common.h.
#pragma once

namespace {

// 0x01 in each byte where x and y agree
DEV uint32_t eq01(uint32_t x, uint32_t y)
{
    const uint32_t z = x ^ y;
    const uint32_t t = ((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z;
    return (~t >> 7) & 0x01010101u;
}

// the 0x01 bytes of e as four bits
DEV uint32_t gather4(uint32_t e) { return (e | (e >> 7) | (e >> 14) | (e >> 21)) & 0xFu; }

DEV uint32_t popc(uint32_t x) { return static_cast<uint32_t>(__builtin_popcount(x)); }
DEV uint32_t low_bits(uint32_t n) { return n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u); }

// a packet left for the lane kernels (their sub-list, counters[3])
DEV void bail(const rc_workspace_dev& ws, uint32_t pkt)
{
    const uint32_t slot = atomicAdd(&ws.counters[3], 1u);
    ws.enc2_list[slot] = pkt;
}

// A lane's records: its first table (16-B records, 4 KB) in a dense array of
// first tables, its second table (48-B records) and dummy slots apart, so
// that the first tables every bucket touches stay one contiguous 268 MB
// (65536 lanes) and the second tables only buckets past 8 elements touch.
constexpr uint32_t kTab1 = 256 * 16;
constexpr uint32_t kTab2Rec = 48;
constexpr uint32_t kTab2 = 256 * kTab2Rec + 128;  // per lane: the second table and 128 B of dummy slots
constexpr uint32_t kTabCap = 28;                 // order-1 elements a bucket's records hold (+ 4 order-2 hits: 32)

// a bucket rebuilt from the history: elements in position order
struct Hist6 { uint32_t A[8], V[8]; uint32_t p1, hit, k; };

// A 16-B record, read past the vector L1 (agent-scope loads: sc1): the lane
// appends to its records with stores, and a copy of the line an earlier load
// left in the L1 would be stale.
DEV uint4 hload16(uintptr_t a)
{
#ifndef RC_LANE_HOST_TEST
    const uint64_t lo = __hip_atomic_load(GPTRC(uint64_t, a), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t hi = __hip_atomic_load(GPTRC(uint64_t, a + 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_uint4(static_cast<uint32_t>(lo), static_cast<uint32_t>(lo >> 32), static_cast<uint32_t>(hi),
                      static_cast<uint32_t>(hi >> 32));
#else
    return gload16(a);
#endif
}

// elements whose byte in X equals u (nd wave-uniform live dwords)
DEV uint32_t eqmask6(const uint32_t* X, uint32_t u, uint32_t nd)
{
    const uint32_t ur = u * 0x01010101u;
    uint32_t m = 0;
#pragma unroll
    for (uint32_t d = 0; d < 8; ++d)
        if (d < nd) m |= gather4(eq01(X[d], ur)) << (4 * d);
    return m;
}

// the record slot of a bucket's element t (t < kTabCap)
DEV uintptr_t rec_addr(const uint8_t* tab, const uint8_t* tab2, uint32_t p, uint32_t t)
{
    return t < 8 ? reinterpret_cast<uintptr_t>(tab) + 16 * p + 2 * t
                 : reinterpret_cast<uintptr_t>(tab2) + kTab2Rec * p + 2 * (t - 8);
}

DEV void rec_load(const uint8_t* tab, const uint8_t* tab2, uint32_t p, uint32_t t1, bool en, uint4& r1, uint4& r2,
                  uint4& r3, uint4& r4)
{
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    r1 = z; r2 = z; r3 = z; r4 = z;
    const uintptr_t b2 = reinterpret_cast<uintptr_t>(tab2) + kTab2Rec * p;
    if (en) r1 = hload16(reinterpret_cast<uintptr_t>(tab) + 16 * p);
    if (en && t1 > 8) {
        r2 = hload16(b2);
        r3 = hload16(b2 + 16);
    }
    if (rare_lane(en && t1 > 24)) {
        if (en && t1 > 24) r4 = hload16(b2 + 32);
    }
}

DEV void rec_fill(const uint4& r1, const uint4& r2, const uint4& r3, const uint4& r4, uint32_t p, uint32_t t1,
                  const uint32_t* hl, uint32_t nh, uint32_t x0, uint32_t n, Hist6& H)
{
    H.A[0] = bperm(r1.y, r1.x, 0x06040200u); H.V[0] = bperm(r1.y, r1.x, 0x07050301u);
    H.A[1] = bperm(r1.w, r1.z, 0x06040200u); H.V[1] = bperm(r1.w, r1.z, 0x07050301u);
    H.A[2] = bperm(r2.y, r2.x, 0x06040200u); H.V[2] = bperm(r2.y, r2.x, 0x07050301u);
    H.A[3] = bperm(r2.w, r2.z, 0x06040200u); H.V[3] = bperm(r2.w, r2.z, 0x07050301u);
    H.A[4] = bperm(r3.y, r3.x, 0x06040200u); H.V[4] = bperm(r3.y, r3.x, 0x07050301u);
    H.A[5] = bperm(r3.w, r3.z, 0x06040200u); H.V[5] = bperm(r3.w, r3.z, 0x07050301u);
    H.A[6] = bperm(r4.y, r4.x, 0x06040200u); H.V[6] = bperm(r4.y, r4.x, 0x07050301u);
    H.A[7] = 0u; H.V[7] = 0u;
    H.p1 = (p == x0 && t1 > 0 && n >= 2) ? 1u : 0u;
    H.hit = 0u;
    uint32_t k = t1;
    if (any_lane(nh > 0))
#pragma unroll
    for (uint32_t h = 0; h < 4; ++h) {
        const bool mine = h < nh && (hl[h] & 0xFFu) == p;
        const uint32_t ks = 8 * (k & 3);
#pragma unroll
        for (uint32_t d = 0; d < 8; ++d) {
            const bool here = mine && (k >> 2) == d;
            H.A[d] = here ? ((H.A[d] & ~(0xFFu << ks)) | (((hl[h] >> 8) & 0xFFu) << ks)) : H.A[d];
            H.V[d] = here ? ((H.V[d] & ~(0xFFu << ks)) | (((hl[h] >> 16) & 0xFFu) << ks)) : H.V[d];
        }
        H.hit |= mine ? (1u << k) : 0u;
        k += mine ? 1u : 0u;
    }
    H.k = k;
}

// The elements of bucket p from the lane's two tables of records (the
// bucket's first 8 order-1 elements in a 16-B record, the next 20 in a 48-B
// one, appended blind, a | v << 8)
// and its order-2 hits from the hit list hl[nh] (p | a << 8 | v << 16).
// Record bytes past t1 are stale (earlier packets): only t1 are taken.
// Position 1 (no order-2 context) is element 0 of bucket x0.
DEV void rec_build(const uint8_t* tab, const uint8_t* tab2, uint32_t p, uint32_t t1, const uint32_t* hl, uint32_t nh,
                   uint32_t x0, uint32_t n, bool en, Hist6& H)
{
    uint4 r1, r2, r3, r4;
    rec_load(tab, tab2, p, t1, en, r1, r2, r3, r4);
    rec_fill(r1, r2, r3, r4, p, t1, hl, nh, x0, n, H);
}

// The values of a bucket's elements as bit planes: bit j of pl[b] is bit b of
// element j's value (nd live dwords).  A select, an equality mask or a count
// below a value is then 8 steps on 32-bit masks.
DEV void planes6(const uint32_t* V, uint32_t nd, uint32_t* pl)
{
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b) {
        uint32_t m = 0;
#pragma unroll
        for (uint32_t d = 0; d < 8; ++d)
            if (d < nd) m |= dot4((V[d] >> b) & 0x01010101u, 0x08040201u, 0u) << (4 * d);
        pl[b] = m;
    }
}

// elements of the 32 whose value is u
DEV uint32_t peq6(const uint32_t* pl, uint32_t u)
{
    uint32_t m = 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b) m &= ((u >> b) & 1u) ? pl[b] : ~pl[b];
    return m;
}

// the value of rank q (0-based, by value) among the elements g, bit by bit
// from the top; lt / eq: the members below it / equal to it
DEV uint32_t pselect6(const uint32_t* pl, uint32_t g, uint32_t q, uint32_t& lt, uint32_t& eq)
{
    uint32_t cand = g, below = 0, u = 0;
#pragma unroll
    for (int b = 7; b >= 0; --b) {
        const uint32_t zeros = cand & ~pl[b];
        const uint32_t nz = popc(zeros);
        const bool one = q >= below + nz;
        below += one ? nz : 0u;
        cand = one ? (cand & pl[b]) : zeros;
        u |= one ? (1u << b) : 0u;
    }
    lt = below;
    eq = popc(cand);
    return u;
}

// the value of element j
DEV uint32_t pval6(const uint32_t* pl, uint32_t j)
{
    uint32_t u = 0;
#pragma unroll
    for (uint32_t b = 0; b < 8; ++b) u |= ((pl[b] >> j) & 1u) << b;
    return u;
}

// compress.c:536-568 in a sub-context holding the elements g of H with d
// distinct values: READ, then an escape (false) or the symbol the code selects
// (true: v, its interval under/count -- coded by the caller).  fail: the
// code is past the context's symbols (compress.c:416).
template <class Src>
DEV bool sub_decode6(const uint32_t* pl, uint32_t g, uint32_t t, uint32_t d, bool en, uint32_t& low,
                     uint32_t& code, uint32_t& range, Src& in, uint32_t& v, uint32_t& under, uint32_t& count,
                     bool& fail)
{
    const uint32_t esc = kSubEscDelta * d, tot = en ? esc + kSubDelta * t : 1u;
    const uint32_t r1 = udiv16d(range, tot, rcp64(tot));
    const uint32_t cd = udiv_lo16(code - low, r1);
    range = en ? r1 : range;
    const bool e = en && cd < esc;
    dec_code(low, code, range, 0u, esc, in, e);
    const bool hit = en && !e;
    fail = fail || (hit && cd - esc >= kSubDelta * t);
    const bool sel = hit && cd - esc < kSubDelta * t;
    // the member of rank q in value order: its value, and the members below it / equal to it
    if (any_lane(sel)) {
        uint32_t lt, eq;
        const uint32_t u = pselect6(pl, g, sel ? (cd - esc) >> 1 : 0u, lt, eq);
        under = sel ? esc + kSubDelta * lt : under;
        count = sel ? kSubDelta * eq : count;
        v = sel ? u : v;
    }
    return sel;
}

}  // namespace
