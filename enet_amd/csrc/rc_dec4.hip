// rc_dec4.hip -- bucket-history range decoder (compress.c:498-627), bit-exact.
//
// One packet per lane, like the lane kernels (rc_lane3.hip), with a leaner
// model.  compress.c's order-1 context of position i is (x[i-1]) and its
// order-2 context is (x[i-2], x[i-1]); both hold only positions j with
// x[j-1] = x[i-1].  So the decoder keeps, per packet, one 64-B record per
// previous byte p ("bucket p") listing the positions decoded so far with
// x[j-1] = p, each as an element (a = x[j-2], v = x[j], flags), and derives
// every sub-context statistic from it (compress.c:159-199, :536-615):
//
//   order 2 (a, p): the elements with that a; t2 of them, dist2 of them new
//       to the context when added:  escapes 5 * dist2, total escapes + 2 * t2
//   order 1 (p): the elements not decoded at order 2 (the ones that visited
//       order 1, compress.c:598-615); t1 of them, dist1 new to it:
//       escapes 5 * dist1, total escapes + 2 * t1
//   a symbol u of a context counts 2 per element with v = u, its cumulative
//   count is 2 per element with v < u: the code r = READ - escapes selects
//   the element of rank floor(r / 2) in value order.
//
// Elements are kept sorted by value (stable), with bit masks of their flags
// and of where each run of equal values starts, so the selection is a rank
// in a bit mask and a symbol's interval two bit scans.  Appending the decoded position to its bucket is
// every update the reference makes; nothing else is stored.  The root (order
// 0) is the lane kernels' LDS table (rc_root3.h).
//
// Per byte: one record read (the bucket of the byte just decoded, issued as
// soon as it is known) and one record write.  The flags record whether a
// symbol was new (compress.c:306-310 / :606-610) -- a property of the history,
// not of the decode path: a corrupt stream can escape from a context that
// holds the symbol, and the reference's patch then finds it there.
// tests/proto/histdec.py restates the algebra (CPU test against the oracle).
//
// Fast path: no bucket over kCap4 elements (no sub-context count or total
// can then reach compress.c's rescale thresholds), no model reset (fewer
// than 4094 nodes, compress.c:148-157), root codes within symbol 255.  A lane
// that leaves it lists its packet (ws.enc2_list, count ws.counters[3]) and
// the lane kernels decode that packet from the start.

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

// wbail: this wavefront's count of packets left to the lanes (LDS).  Once a
// quarter of the wavefront has left its packet, the rest follow at once:
// a batch of low-entropy packets (large buckets) then costs this decoder a
// few steps instead of the steps until its last lane fills a bucket.
constexpr uint32_t kWaveBail = 16;

DEV void decompress_one4(const rc_batch_dev& bt, const rc_workspace_dev& ws, uint32_t pkt, uint8_t* reg,
                         uint8_t* root, uint32_t* wbail)
{
    const uint32_t len = bt.in_len[pkt];
    const uint32_t cap = bt.out_cap[pkt];
    if (len == 0) { bt.out_len[pkt] = 0; return; }                   // compress.c:513
    ByteSink o;
    sink_init(o, bt.out + bt.out_off[pkt], cap);
    ByteSrc in;
    src_init(in, bt.in + bt.in_off[pkt], len);
    const uint32_t epoch = next_epoch(reg, *reinterpret_cast<const uint32_t*>(reg)) & 0xFFFF;
    Root R;
    root3_clear<false>(root, R);
    uint32_t rtot = 1 + 256;
    double rrt = rcp64(rtot);
    uint32_t low = 0, range = ~0u;
    uint32_t code = static_cast<uint32_t>(in.la >> 32);            // compress.c:344-350 (0 past the end)
    in.la <<= 32;
    in.na -= 4;
    src_refill(in, true);

    Bucket B;                       // bucket p of this step
    bk_empty(B, epoch);
    Raw4 rw;                        // the next step's bucket, in flight
    uint32_t fwd = 1;               // (a word: a bool would be an SGPR lane mask)
    uint32_t order = 0, a = 0, p = 0, nodes = 1;
    bool fail = false, off = false;

    PROF_DECL
    for (;;) {
#ifdef RC_PROFILE_DRAIN
        __builtin_amdgcn_s_waitcnt(0);
        PROF(9)
#endif
        // (the lookahead refill and the output store need no record: issued
        // before the wait for it)
        src_fill(in, true);
#ifdef DEC4_NO_OUT
        o.pend = false;                               // (timing experiment: output not stored)
#else
        sink_flush(o);
#endif
        if (!fwd) bk_from(rw, epoch, B);
        PROF(0)
        const uint32_t nd = live_dwords(bk_k(B.h));
        Groups s;
        bk_groups(B, nd, a, order >= 2, s);
        // the totals' reciprocals, ahead of the READs that divide by them
        const double rt2 = rcp64(max(kSubEscDelta * s.d2 + kSubDelta * s.t2, 1u));
        const double rt1 = rcp64(max(kSubEscDelta * s.d1 + kSubDelta * s.t1, 1u));
        PROF(1)
        int at = -1;
        uint32_t hj = 0;                                             // (a hit: the member index)
        uint32_t v = 0;
        bool new0 = false;
        // order 2, then order 1: visited when the context holds elements
        // (escapes 0 < 5 * dist < total, compress.c:536-544)
        if (order >= 2 && s.t2 > 0) {
            if (sub_decode(B, s.g2, s.t2, s.d2, rt2, low, code, range, in, v, hj, fail)) at = 2;
            if (fail) break;
        }
        if (at < 0 && order >= 1 && s.t1 > 0) {
            if (sub_decode(B, s.g1, s.t1, s.d1, rt1, low, code, range, in, v, hj, fail)) at = 1;
            if (fail) break;
        }
        PROF(2)
        // root, compress.c:570-596
        uint32_t cnt0 = 0, under0 = 0;
        if (at < 0) {
            const uint32_t cd = dec_read_d(range, low, code, rtot, rrt);
            if (cd < 1) { dec_code(low, code, range, 0, 1, in, true); break; }   // end of stream
            if (cd - 1 >= rtot - 1) { off = true; break; }                 // past symbol 255
            uint32_t under, cnt;
            v = root3_search(root, R, cd - 1, under, cnt);
            new0 = cnt == 0;
            cnt0 = cnt;
            under0 = under;
            at = 0;                                  // (the root's update: after the load below)
        }
        // the next step's bucket: this one when v == p (updated below), else a
        // load issued now so that its latency overlaps the rest of the step.
        // The step's memory operations are unconditional (the scratch record
        // for lanes that need none; see rc_lane3.hip lane_prefetch).
        PROF(3)
        const bool nfwd = order >= 1 && v == p;
#ifdef DEC4_PAD
        __builtin_amdgcn_s_sleep(DEC4_PAD);           // (timing experiment: compute added before the load)
#endif
        raw4_load(reg, nfwd ? kDummyRec : kO1Base + v * kRec4, rw);
        // the root's code and update (compress.c:583-595): only the next
        // step's READs need them, so they run in the shadow of the load
        // (+2.9 % and +1.9 % decompress, same-box A/B)
        uint32_t fu = 1 + under0, fc = 1 + cnt0;             // the step's last code: root, or a hit
        if (any_lane(at != 0)) {
            uint32_t hu, hc;
            hit_interval(B, at == 2 ? s.g2 : s.g1, kSubEscDelta * (at == 2 ? s.d2 : s.d1), hj, hu, hc);
            fu = at != 0 ? hu : fu;
            fc = at != 0 ? hc : fc;
        }
        dec_code_late(low, code, range, fu, fc, in, true);
        if (at == 0) {
            root3_add<false>(root, R, v, cnt0);
            rtot = (rtot + kRootDelta) & 0xFFFF;
            if (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit) rtot = root3_rescale<false>(root, R);
            rrt = rcp64(rtot);                       // (for the next root READ)
        }
        fail = o.n >= o.cap;                                         // compress.c:617
        // the element joins bucket p (compress.c:598-615: every visited
        // context gains v); nodes as compress.c creates them
        uint32_t lt, le;
        bk_rank(B, nd, v, lt, le);
        const uint32_t eqr = low_bits(le) & ~low_bits(lt);
        const bool n2 = order >= 2 && (s.g2 & eqr) == 0;
        const bool n1 = order >= 1 && at != 2 && (s.g1 & eqr) == 0;
        nodes += (new0 ? 1u : 0u) + (n2 ? 1u : 0u) + (n1 ? 1u : 0u);
        PROF(4)
        const bool full = order >= 1 && bk_k(B.h) >= kCap4;
        const uint32_t first = order == 1 ? 1u : 0u;                 // position 1: hit and new
        bk_insert(B, nd, le, a, v, (at == 2 ? 1u : 0u) | first, (n2 ? 1u : 0u) | first, lt == le ? 1u : 0u,
                  (1u << 16) + (at == 2 ? (1u << 21) : 0u) + (n1 ? (1u << 26) : 0u), order >= 1 && !full);
        // (the step's last memory operation)
        bk_store(reg, order >= 1 ? kO1Base + p * kRec4 : kDummyRec, B);
        PROF(5)
        off = full || nodes >= kNodeLimit4 || *wbail >= kWaveBail;
        if (fail || off) break;
        sink_put(o, v, 1, true);
        src_adv(in);
        PROF(6)
        fwd = nfwd ? 1u : 0u;
        a = p;
        p = v;
        order += order < 2 ? 1u : 0u;
    }
    PROF_FLUSH(16)
    if (off && !fail) { atomicAdd(wbail, 1u); bail(ws, pkt); return; }
    sink_finish(o, !fail);
    bt.out_len[pkt] = fail ? 0u : o.n;
}

}  // namespace

#ifndef RC_LANE_HOST_TEST
// per lane in LDS: the root counts, pad (68 dwords: b128 conflict-free)
constexpr uint32_t kDec4Lds = kRootStrideDec;

// one wave per SIMD by design (a packet per lane, 65536 lanes fill the chip)
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void rc_decompress_dec4(rc_batch_dev b, rc_workspace_dev ws)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t act = ws.lane_active;
    const uint32_t wave = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l >= act) return;
    const uint32_t local = wave * act + l;
    uint8_t* root = smem + local * kDec4Lds;
    uint32_t* wbail = reinterpret_cast<uint32_t*>(smem + 4 * act * kDec4Lds) + wave;
    if (l == 0) *wbail = 0u;
    const uint32_t per_block = 4 * act;
    const uint32_t slot = blockIdx.x * per_block + local;
    uint8_t* reg = static_cast<uint8_t*>(ws.lane_pool) + static_cast<size_t>(slot) * ws.lane_region;
    const uint32_t* order = ws.order && !ws.bins[RC_LEN_BINS] ? ws.order : nullptr;
    for (uint32_t i = slot; i < b.n; i += gridDim.x * per_block) {
        const uint32_t pkt = order ? order[i] : i;
        decompress_one4(b, ws, pkt, reg, root, wbail);
    }
}

// The decoder over the batch; packets off its fast path are listed in
// ws->enc2_list, count in ws->counters[3], for the lane kernels.
extern "C" int rc_hip_dec4_launch(const rc_batch_dev* b, const rc_workspace_dev* ws, uint32_t blocks, void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    const size_t lds = static_cast<size_t>(4 * ws->lane_active) * kDec4Lds + 16;   // + wbail[4]
    hipLaunchKernelGGL(rc_decompress_dec4, dim3(blocks), dim3(256), lds, st, *b, *ws);
    return static_cast<int>(hipGetLastError());
}
#endif  // RC_LANE_HOST_TEST
