// rc_dec7.hip -- record-light range decoder with a helper wavefront per SIMD
// (compress.c:498-627), bit-exact.  The default fast decoder.
//
// The model and the common step are rc_dec6.hip's (read its header first):
// per bucket one LDS byte (t1, r1) gives the order-1 context's escapes and
// total; a byte decoded at the root after escaping order 1 is new to that
// context, so the next position's order-2 context has never been visited.
// A step that needs a context's symbols -- order 1 holds the coded symbol, or
// the order-2 context exists -- stalls its lane.
//
// What differs is who does what.  rc_dec6 runs one wavefront per SIMD: its
// lanes stall until every 16th step, when the whole wavefront runs the rare
// phase for ~9 of them (30 % of its cycles), and its per-step input reload
// waits for a load issued one step earlier (14 %).  A lone wavefront leaves
// about half of its SIMD's issue cycles unused (it waits on its own chain),
// and a second wavefront on the SIMD takes those cycles without slowing it
// (tools/mb/issue2.hip: a main wavefront's chain runs at the same cycles per
// link beside an idle, a polling or a busy partner).  So each workgroup has
// 4 main wavefronts (waves 0-3, one packet per lane, the common steps) and 4
// helper wavefronts (waves 4-7: wave w + 4 shares wave w's SIMD; lane l of
// the helper serves lane l of its main wavefront).  They talk through LDS
// only, each word written by one side:
//
//   * the element ring (main -> helper, 8 x 4 B per lane): every element the
//     common step adds to an order-1 context, (p, t1, a, v).  The helper
//     appends it to the lane's bucket records in HBM (rc_dec6's tables, 2-B
//     stores), so the main wavefront stores nothing but its output windows;
//   * the input slot (helper -> main, 16 B per lane): the next aligned chunk
//     of the lane's compressed stream.  The main lane takes it when its
//     current chunk is used up and asks for the one after; it never waits on
//     a global load (it issues none after the packet's first two chunks);
//   * the mailbox (both ways, 24 B per lane): a stalled lane posts its coder
//     state; the helper drains the ring, loads the bucket's records and the
//     stream bytes at the lane's position, decodes the step exactly over the
//     elements (rc_dec6_rare.h) and, while the next step again has a visited
//     order-2 context, the steps after it (up to kChain7 symbols), and posts
//     the new coder state, the bytes consumed and the symbols decoded.  A
//     step whose sub-contexts all escaped comes back "root pending": the main
//     lane's next step decodes at the root (the common step without its
//     order-1 part), so the root model stays in the main lane's registers;
//   * the control words: m_ctl (ring head, request count, wanted chunk, packet
//     generation) and m_pkt (the packet) from main, h_ctl (ring tail, answer
//     count, the slot's chunk and generation) from the helper.
//
// The main step reads h_ctl and the slot at its top and acts on them at its
// end (resumes, input advance), so the LDS round trips overlap the step.
// Nothing the main wavefront waits for depends on anything but the helper,
// and the helper waits only on its own memory operations: no deadlock.  A
// main lane that needs a slot or an answer that is not there yet keeps
// stepping nothing; the wavefront sleeps when none of its lanes can step.
//
// The check (rc_dec6_verify) and the routing of packets off the fast path are
// rc_dec6's.  tests/proto/lane_host.cpp (variant v7) compiles both sides for
// the host with the helper run synchronously after each main step.

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
#include "rc_bucket4.h"
#include "rc_dec6_rare.h"

namespace {

constexpr uint32_t kLane7 = 528;      // per lane: root counts[256] | input slot (16 B) | bucket bytes[256]
constexpr uint32_t kSlot7 = 256;
constexpr uint32_t kStats7 = 272;
constexpr uint32_t kRing7 = 16;       // element ring entries per lane
constexpr uint32_t kMbox7 = 6;        // mailbox dwords per lane
#ifndef DEC7_CHAIN
#define DEC7_CHAIN 3
#endif
constexpr uint32_t kChain7 = DEC7_CHAIN;   // symbols per answer at most
constexpr uint32_t kFin7 = 0xFFFFFFFFu;
constexpr uint32_t kNoPkt7 = 0xFFFFFFFEu;
constexpr uint32_t kWaveBail7 = 16;
constexpr uint32_t kLanes7 = 256;     // main lanes per workgroup

__host__ __device__ constexpr uint32_t lds7_bytes(uint32_t lanes) { return lanes * (kLane7 + 4 * kRing7 + 4 * kMbox7 + 8 + 8); }

struct Lds7 {
    uint8_t* lane;     // root | slot | bucket bytes
    uint32_t* ring;
    uint32_t* mbox;
    uint32_t* mctl;    // [0] ctl, [1] packet (one 8-B word)
    uint32_t* hctl;    // [0] the serving helper's word, [1] the storing helper's (one 8-B word)
};

DEV Lds7 lds7(uint8_t* smem, uint32_t L, uint32_t lanes)
{
    Lds7 s;
    s.lane = smem + L * kLane7;
    uint8_t* q = smem + lanes * kLane7;
    s.ring = reinterpret_cast<uint32_t*>(q) + L * kRing7;
    q += lanes * kRing7 * 4;
    s.mbox = reinterpret_cast<uint32_t*>(q) + L * kMbox7;
    q += lanes * kMbox7 * 4;
    s.mctl = reinterpret_cast<uint32_t*>(q) + L * 2;
    q += lanes * 8;
    s.hctl = reinterpret_cast<uint32_t*>(q) + L * 2;
    return s;
}

DEV uint32_t mctl_word(uint32_t head, uint32_t req, uint32_t want, uint32_t gen)
{
    return (head & 0xFFu) | ((req & 0xFFu) << 8) | ((want & 0xFFFu) << 16) | (gen << 28);
}

// ------------------------------------------------------------------ helper
// The helper's per-lane state (registers of the helper wavefront).
constexpr uint32_t kCache7 = 8;   // the lane's last record stores, newest first
struct Help7 {
    uint32_t tail, resp, have, hgen, cgen, pub;
    uint32_t pkt, cap, len;
    uintptr_t lo;
    uint32_t hl[4], nh;           // elements decoded at order 2: p | a << 8 | v << 16
    uint32_t ec[kCache7];         // elements stored last (p | t1 << 8 | a << 16 | v << 24)
#ifdef RC_PROFILE
    unsigned long long ps, pt, pr, pw;   // (diagnostic) lanes served, cycles serving, ring passes, load waits
#endif
};

DEV void help7_init(Help7& h)
{
    h.tail = 0; h.resp = 0; h.have = 0; h.hgen = 0; h.cgen = 0; h.pub = 0;
    h.pkt = 0; h.cap = 0; h.len = 0; h.lo = 0;
    h.hl[0] = h.hl[1] = h.hl[2] = h.hl[3] = 0; h.nh = 0;
#pragma unroll
    for (uint32_t k = 0; k < kCache7; ++k) h.ec[k] = 0xFFFFFFFFu;   // (t1 255: matches no slot)
#ifdef RC_PROFILE
    h.ps = h.pt = h.pr = h.pw = 0;
#endif
}

// element e into its bucket's records (a blind 2-B store), remembered in the cache
DEV void help7_store(uint8_t* tab, Help7& h, uint32_t e, bool en)
{
    const uint32_t p = e & 0xFFu, t1 = (e >> 8) & 0xFFu;
    if (en)
        *GPTR(uint16_t, reinterpret_cast<uintptr_t>(tab) + (t1 < 8 ? 16 * p + 2 * t1 : kTab2 + 32 * p + 2 * (t1 - 8))) =
            static_cast<uint16_t>(e >> 16);
#pragma unroll
    for (uint32_t k = kCache7 - 1; k > 0; --k) h.ec[k] = en ? h.ec[k - 1] : h.ec[k];
    h.ec[0] = en ? e : h.ec[0];
}

// A record load may be issued before the lane's last stores have completed:
// the loads are issued behind `s_waitcnt vmcnt(kCache7)` (every vector memory
// operation of this wavefront but the last kCache7 done), so every store the
// load might miss is among the lane's last kCache7 stores, which are written
// over the loaded words here, oldest first (a store the load did see is
// written again with the same value).
DEV void patch1(uint32_t* w, uint32_t e, uint32_t p)
{
    const uint32_t t1 = (e >> 8) & 0xFFu, val = e >> 16;
    const bool mine = (e & 0xFFu) == p && t1 < kTabCap;
#pragma unroll
    for (uint32_t i = 0; i < 12; ++i) {
        const bool here = mine && (t1 >> 1) == i;
        const uint32_t nw = (t1 & 1) ? ((w[i] & 0xFFFFu) | (val << 16)) : ((w[i] & 0xFFFF0000u) | val);
        w[i] = here ? nw : w[i];
    }
}

// ring: the lane's element ring (kRing7 entries), its entries [from, to) (mod
// 256) not yet confirmed stored by the storing helper: written over the
// loaded words first (main's elements are older than the serving helper's own)
DEV void help7_patch(const Help7& h, uint32_t p, const uint32_t* ring, uint32_t from, uint32_t to, uint4& r1,
                     uint4& r2, uint4& r3)
{
    uint32_t w[12] = {r1.x, r1.y, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w, r3.x, r3.y, r3.z, r3.w};
    const uint32_t nr = (to - from) & 0xFFu;
    // (a ring entry rarely holds bucket p: one LDS read and a ballot per entry)
    for (uint32_t k = 0; any_lane(k < nr); ++k) {
        const uint32_t e = k < nr ? ring[(from + k) & (kRing7 - 1)] : 0xFFFFFFFFu;
        const bool mine = (e & 0xFFu) == p && ((e >> 8) & 0xFFu) < kTabCap;
        if (any_lane(mine)) patch1(w, mine ? e : 0xFFFFFFFFu, p);
    }
#pragma unroll
    for (int k = kCache7 - 1; k >= 0; --k) {
        const uint32_t e = h.ec[k];
        const uint32_t t1 = (e >> 8) & 0xFFu, val = e >> 16;
        const bool mine = (e & 0xFFu) == p && t1 < kTabCap;
#pragma unroll
        for (uint32_t i = 0; i < 12; ++i) {
            const bool here = mine && (t1 >> 1) == i;
            const uint32_t nw = (t1 & 1) ? ((w[i] & 0xFFFFu) | (val << 16)) : ((w[i] & 0xFFFF0000u) | val);
            w[i] = here ? nw : w[i];
        }
    }
    r1 = make_uint4(w[0], w[1], w[2], w[3]);
    r2 = make_uint4(w[4], w[5], w[6], w[7]);
    r3 = make_uint4(w[8], w[9], w[10], w[11]);
}

DEV void vm_window()
{
#ifndef RC_LANE_HOST_TEST
    static_assert(kCache7 == 8, "the wait below names the cache size");
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
#endif
}

// One pass over the requests (rq) and the wanted input chunks (inq) of the
// helper's lanes, with one memory round trip for all of them: the requests'
// first records and stream bytes and the chunks are loaded together.  A
// request is the exact step(s) of a stalled lane (rc_dec6.hip's rare phase
// without the root: a step that escapes every sub-context is handed back).
// Reads the requests from the mailboxes and writes the answers there.
DEV void help7_serve(const Lds7& x, uint8_t* tab, Help7& h, bool en, bool inq, uint32_t want, uint32_t head)
{
    // the elements of main's ring not yet confirmed in the records (read before the records)
    const uint32_t stored = x.hctl[1] & 0xFFu;
    const uint4 q0 = *reinterpret_cast<const uint4*>(x.mbox);
    const uint2 q1 = *reinterpret_cast<const uint2*>(x.mbox + 4);
    uint32_t low = q0.x, code = q0.y, range = q0.z;
    uint32_t p = q0.w & 0xFFu, a = (q0.w >> 8) & 0xFFu, x0 = (q0.w >> 16) & 0xFFu, order = (q0.w >> 24) & 3u;
    bool repeat = ((q0.w >> 26) & 1u) != 0;
    const uint32_t pos = q1.x & 0xFFFFu;
    uint32_t on = q1.x >> 16;
    uint32_t nodes = q1.y & 0xFFFFu, claims = q1.y >> 16;
    uint8_t* stats = x.lane + kStats7;
    // the stream from the lane's position (bytes past the packet read as 0)
    const uint32_t start = pos < h.len ? pos : h.len;
    // (lanes without a request read nothing: an empty stream inside their own table)
    const uint8_t* sp = en ? reinterpret_cast<const uint8_t*>(h.lo) + start : tab + 32;
    const uint32_t sn = en ? h.len - start : 0u;
    ByteSrc in;
    uint32_t outb = 0, nout = 0;
    bool lv = false, fl = false, rootonly = false;
    bool act = en;
    for (uint32_t it = 0; it < kChain7 && any_lane(act); ++it) {
        const bool rs = act;
        const uint32_t st = rs && order >= 1 ? stats[p] : 0u;
        const uint32_t t1 = st & 31u, d1 = t1 - (st >> 5);
        uint4 r1, r2, r3;
#ifdef RC_PROFILE
        const unsigned long long tw = prof_now();
#endif
        vm_window();
        rec_load(tab, p, rs ? t1 : 0u, rs, r1, r2, r3);
        if (it == 0) {
            // the wanted input chunks, then the stream (src_init waits for everything)
            const uintptr_t lo = h.lo, base = lo & ~static_cast<uintptr_t>(15);
            const uint4 c = chunk_load(lo, lo + h.len, base + 16 * static_cast<uintptr_t>(want), inq);
            src_init(in, sp, sn, false);
            if (inq) *reinterpret_cast<uint4*>(x.lane + kSlot7) = c;
        }
        help7_patch(h, p, x.ring, stored, head, r1, r2, r3);
#ifdef RC_PROFILE
        {
            uint32_t sink = r1.x ^ r2.y ^ r3.z;
            asm volatile("" :: "v"(sink));
            h.pw += prof_now() - tw;
        }
#endif
        Hist6 H;
        rec_fill(r1, r2, r3, p, rs ? t1 : 0u, h.hl, h.nh, x0, on, H);
        uint32_t nd = 1;
#pragma unroll
        for (uint32_t j = 1; j < 8; ++j) nd += any_lane(H.k > 4 * j) ? 1u : 0u;
        uint32_t pl[8];
        planes6(H.V, nd, pl);
        const uint32_t km = low_bits(H.k);
        const uint32_t g2 = (rs && order >= 2) ? (eqmask6(H.A, a, nd) & km & ~H.p1) : 0u;
        const uint32_t g1 = km & ~H.hit;
        const uint32_t t2 = popc(g2);
        uint32_t d2 = 0;
        {
            uint32_t rem = g2;
            while (any_lane(rem != 0)) {
                const uint32_t j = rem ? static_cast<uint32_t>(__builtin_ctz(rem)) : 0u;
                const uint32_t same = peq6(pl, pval6(pl, j)) & g2 & low_bits(j);
                d2 += (rem != 0 && same == 0) ? 1u : 0u;
                rem &= rem ? rem - 1u : 0u;
            }
        }
        int at = -1;
        uint32_t v = 0, hu = 0, hc = 0;
        bool sf = false;
        const bool c2 = rs && order >= 2 && t2 > 0;
        if (any_lane(c2)) {
            if (sub_decode6(pl, g2, t2, d2, c2, low, code, range, in, v, hu, hc, sf)) at = 2;
        }
        const bool c1 = rs && !sf && at < 0 && order >= 1 && t1 > 0;
        if (any_lane(c1)) {
            if (sub_decode6(pl, g1, t1, d1, c1, low, code, range, in, v, hu, hc, sf)) at = 1;
        }
        const bool sym = rs && !sf && at > 0;
        dec_code(low, code, range, hu, hc, in, sym);
        // every sub-context escaped: the root's code is the main lane's (its next step)
        rootonly = rootonly || (rs && !sf && at < 0);
        // the element joins its contexts (compress.c:598-615)
        const uint32_t eqv = peq6(pl, v) & km;
        const bool n2 = order >= 2 && (eqv & g2) == 0;
        const bool n1 = order >= 1 && at != 2 && (eqv & g1) == 0;
        const bool nb = eqv == 0;
        nodes += sym ? (n2 ? 1u : 0u) + (n1 ? 1u : 0u) : 0u;
        const bool o1v = sym && order >= 1 && at != 2;
        if (o1v) stats[p] = static_cast<uint8_t>(st + 1 + (n1 ? 0u : 32u));
        const bool tfull = o1v && t1 >= kTabCap;
        help7_store(tab, h, p | (t1 << 8) | (a << 16) | (v << 24), o1v && !tfull);
        claims += (sym && order >= 1 && nb && on < h.cap) ? 1u : 0u;
        const bool h2 = sym && at == 2;
        const uint32_t he = p | (a << 8) | (v << 16);
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) h.hl[k] = (h2 && h.nh == k) ? he : h.hl[k];
        const bool hfull = h2 && h.nh >= 4;
        h.nh += h2 ? 1u : 0u;
        const bool f = sym && on >= h.cap;
        const bool l = sf || hfull || tfull || (o1v && !n1 && (st >> 5) >= 7) || (sym && nodes >= kMaxNodes);
        lv = lv || (rs && l);
        fl = fl || (rs && f);
        const bool put = sym && !l && !f;
        outb |= put ? v << (8 * nout) : 0u;
        nout += put ? 1u : 0u;
        on += put ? 1u : 0u;
        a = sym ? p : a;
        p = sym ? v : p;
        order += (sym && order < 2) ? 1u : 0u;
        repeat = sym ? !nb : repeat;
        // the step after a hit with a visited order-2 context is rare again
        act = put && order >= 2 && repeat;
    }
    // the answer: coder state, bytes consumed, symbols, model state
    const uint32_t used = static_cast<uint32_t>((in.next - 32 + 4 * in.q - in.na) - reinterpret_cast<uintptr_t>(sp));
    if (en) {
        *reinterpret_cast<uint4*>(x.mbox) =
            make_uint4(low, code, range, outb | (nout << 24) | (min(used, 63u) << 26));
        *reinterpret_cast<uint2*>(x.mbox + 4) =
            make_uint2(p | (a << 8) | (order << 16) | ((repeat ? 1u : 0u) << 18) | ((rootonly ? 1u : 0u) << 19) |
                           ((lv ? 1u : 0u) << 20) | ((fl ? 1u : 0u) << 21),
                       (nodes & 0xFFFFu) | (claims << 16));
    }
}

// the wanted input chunks alone (no request in the wavefront)
DEV void help7_chunks(const Lds7& x, Help7& h, bool inq, uint32_t want)
{
    const uintptr_t lo = h.lo, base = lo & ~static_cast<uintptr_t>(15);
    const uint4 c = chunk_load(lo, lo + h.len, base + 16 * static_cast<uintptr_t>(want), inq);
    if (inq) *reinterpret_cast<uint4*>(x.lane + kSlot7) = c;
}

// One pass of the serving helper over its 64 lanes: new packets, input
// chunks and requests; publishes its h_ctl word.  Returns whether it did
// anything; fin_all: every lane's main side has finished.
DEV bool help7_iter(const rc_batch_dev& bt, const Lds7& x, uint8_t* tab, Help7& h, bool& fin_all)
{
    const uint2 m = *reinterpret_cast<const uint2*>(x.mctl);
    const uint32_t mc = m.x, mp = m.y;
    const bool fin = mp == kFin7;
    const uint32_t head = mc & 0xFFu, req = (mc >> 8) & 0xFFu, want = (mc >> 16) & 0xFFFu, mgen = mc >> 28;
    bool busy = false;
    // a new packet: its input range and output capacity, no order-2 hits yet
    const bool np = !fin && mp != kNoPkt7 && mgen != h.cgen;
    if (any_lane(np)) {
        if (np) {
            h.pkt = mp;
            h.len = bt.in_len[mp];
            h.lo = reinterpret_cast<uintptr_t>(bt.in + bt.in_off[mp]);
            h.cap = bt.out_cap[mp];
            h.nh = 0;
            h.cgen = mgen;
#pragma unroll
            for (uint32_t k = 0; k < kCache7; ++k) h.ec[k] = 0xFFFFFFFFu;   // (another packet's stores)
        }
    }
    // the next input chunk the main lane wants, and requests
    const bool inq = !fin && h.cgen != 0 && mgen == h.cgen && (want != h.have || h.hgen != h.cgen);
    const bool rq = !fin && req != h.resp;
    if (any_lane(rq)) {
        busy = true;
#ifdef RC_PROFILE
        const unsigned long long t0 = prof_now();
        h.ps += static_cast<unsigned long long>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(rq)));
#endif
        help7_serve(x, tab, h, rq, inq, want, head);
        h.resp = rq ? req : h.resp;
#ifdef RC_PROFILE
        h.pt += prof_now() - t0;
#endif
    } else if (any_lane(inq)) {
        busy = true;
        help7_chunks(x, h, inq, want);
    }
    h.have = inq ? want : h.have;
    h.hgen = inq ? h.cgen : h.hgen;
    const uint32_t hc = (h.resp << 8) | (h.have << 16) | (h.hgen << 28);
    if (hc != h.pub) {
        __builtin_amdgcn_s_waitcnt(0xC07F);      // lgkmcnt(0): slots and answers written before the word that announces them
        *x.hctl = hc;
        h.pub = hc;
    }
    fin_all = !any_lane(!fin);
    return busy;
}

// One pass of the storing helper: main's ring entries into the bucket records
// (2-B stores), then a wait for them, then the confirmed tail in its h_ctl
// word -- the serving helper takes the entries past it from the ring itself,
// and main reuses a ring slot only once its entry is confirmed.  It never
// loads, so no load waits behind its stores.
struct Store7 { uint32_t tail; };
DEV bool store7_iter(const Lds7& x, uint8_t* tab, Store7& t, bool& fin_all)
{
    const uint2 m = *reinterpret_cast<const uint2*>(x.mctl);
    const uint32_t head = m.x & 0xFFu;
    const bool fin = m.y == kFin7;
    bool busy = false;
    if (any_lane(t.tail != head)) {
        busy = true;
        while (any_lane(t.tail != head)) {
            const bool en = t.tail != head;
            const uint32_t e = x.ring[t.tail & (kRing7 - 1)];
            const uint32_t p = e & 0xFFu, t1 = (e >> 8) & 0xFFu;
            if (en)
                *GPTR(uint16_t, reinterpret_cast<uintptr_t>(tab) + (t1 < 8 ? 16 * p + 2 * t1 : kTab2 + 32 * p + 2 * (t1 - 8))) =
                    static_cast<uint16_t>(e >> 16);
            t.tail = en ? (t.tail + 1) & 0xFFu : t.tail;
        }
        __builtin_amdgcn_s_waitcnt(0);            // (the stores done: visible to the serving helper's loads)
        x.hctl[1] = t.tail;
    }
    fin_all = !any_lane(!fin);
    return busy;
}

#ifndef RC_LANE_HOST_TEST
#define DEC7_IDLE() __builtin_amdgcn_s_sleep(1)
#else
static void dec7_host_kick();
#define DEC7_IDLE() dec7_host_kick()
#endif

// -------------------------------------------------------------------- main
// The main lane's input: a 64-bit lookahead (next byte in bits 63..56) topped
// up from the 16-B chunk c (chunk j of the packet's aligned stream), which is
// refilled from the LDS slot.  Bytes past the packet read as 0.
struct MSrc {
    uint64_t la;
    uint32_t na, q, j, lo15;
    uint4 c;
};

struct Main7 {
    uint32_t head, req, want, gen;
};

DEV uint64_t shl8(uint64_t x, uint32_t k) { return k >= 8 ? 0ull : x << (8 * k); }

DEV void mpublish(const Lds7& x, const Main7& m)
{
    x.mctl[0] = mctl_word(m.head, m.req, m.want, m.gen);
}

DEV void mfill(MSrc& s, bool en)
{
    const bool need = en && s.na <= 4 && s.q < 4;
    const uint32_t d = bswap(sel4(s.q, s.c));
    const uint32_t sh = need ? 32 - 8 * s.na : 0u;
    s.la |= need ? (static_cast<uint64_t>(d) << sh) : 0ull;
    s.na += need ? 4u : 0u;
    s.q += need ? 1u : 0u;
}

// c used up: the slot if it holds chunk j + 1 (hc: the h_ctl word read)
DEV void mtake(MSrc& s, const uint4& sl, uint32_t hc, Main7& m, bool en)
{
    const bool ready = ((hc >> 16) & 0xFFFu) == ((s.j + 1) & 0xFFFu) && (hc >> 28) == m.gen;
    const bool t = en && s.q == 4 && ready;
    s.c.x = t ? sl.x : s.c.x; s.c.y = t ? sl.y : s.c.y; s.c.z = t ? sl.z : s.c.z; s.c.w = t ? sl.w : s.c.w;
    s.q = t ? 0u : s.q;
    s.j += t ? 1u : 0u;
    m.want = t ? s.j + 1 : m.want;
}

// at least one byte in the lookahead where `en` (the rare paths): from c, or
// from the slot once the helper has put the next chunk there
DEV void mneed1(MSrc& s, const Lds7& x, Main7& m, bool en)
{
    bool w = en && s.na == 0 && s.q == 4;
    while (rare_lane(w)) {
        const uint32_t hc = *x.hctl;
        const uint4 sl = *reinterpret_cast<const uint4*>(x.lane + kSlot7);
        mtake(s, sl, hc, m, w);
        mpublish(x, m);
        w = w && s.q == 4;
        if (any_lane(w)) DEC7_IDLE();
    }
    mfill(s, en && s.na == 0);
}

DEV uint32_t mshift_in(MSrc& s, uint32_t code, uint32_t k)
{
    const uint32_t t = static_cast<uint32_t>(s.la >> 32);
    const uint32_t in = static_cast<uint32_t>((static_cast<uint64_t>(t) << (8 * k)) >> 32);
    s.la = shl8(s.la, k);
    s.na -= k;
    return (code << (8 * k)) | in;
}

// compress.c:354-371 where `en` (rc_lane_common.h dec_code over MSrc)
DEV void mdec_code(uint32_t& low, uint32_t& code, uint32_t& range, uint32_t under, uint32_t count, MSrc& in,
                   const Lds7& x, Main7& m, bool en)
{
    low = en ? low + under * range : low;
    range = en ? range * count : range;
    const uint32_t k = en ? settled_bytes(low, range) : 0u;
    const bool fast = k <= in.na;
    const uint32_t kk = fast ? k : 0u;
    code = mshift_in(in, code, kk);
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
            mneed1(in, x, m, more);
            code = mshift_in(in, code, more ? 1u : 0u);
            range = more ? range << 8 : range;
            low = more ? low << 8 : low;
        } while (rare_lane(more));
    }
}

// skip k bytes the helper consumed
DEV void mskip(MSrc& s, uint32_t k, const Lds7& x, Main7& m, bool en)
{
    const bool fast = en && k <= s.na;
    s.la = fast ? shl8(s.la, k) : s.la;
    s.na -= fast ? k : 0u;
    bool more = en && !fast;
    if (rare_lane(more)) {
        uint32_t r = more ? k - s.na : 0u;
        s.la = more ? 0ull : s.la;
        s.na = more ? 0u : s.na;
        while (rare_lane(more && r > 0)) {
            const bool e = more && r > 0;
            mneed1(s, x, m, e);
            const uint32_t t = e ? min(r, s.na) : 0u;
            s.la = shl8(s.la, t);
            s.na -= t;
            r -= t;
        }
    }
}

// the packet's first chunks (the main lane's only global loads besides the
// packet's lengths and offsets) and the seed (compress.c:344-350).  Three
// dwords from the one holding the first byte: chunks 0 and 1 hold them.
DEV void madv0(MSrc& s, const uint4& c1)
{
    const bool adv = s.q == 4 && s.j == 0;
    s.c.x = adv ? c1.x : s.c.x; s.c.y = adv ? c1.y : s.c.y; s.c.z = adv ? c1.z : s.c.z; s.c.w = adv ? c1.w : s.c.w;
    s.j += adv ? 1u : 0u;
    s.q = adv ? 0u : s.q;
}

DEV uint32_t msrc_init(MSrc& s, const uint8_t* p, uint32_t len)
{
    const uintptr_t lo = reinterpret_cast<uintptr_t>(p), hi = lo + len;
    const uintptr_t base = lo & ~static_cast<uintptr_t>(15);
    const uint4 c0 = chunk_load(lo, hi, base, true);
    const uint4 c1 = chunk_load(lo, hi, base + 16, true);
    s.lo15 = static_cast<uint32_t>(lo & 15);
    const uint32_t sk = static_cast<uint32_t>(lo & 3);
    s.q = s.lo15 >> 2;
    s.c = c0;
    s.j = 0;
    s.la = static_cast<uint64_t>(bswap(sel4(s.q, s.c)) << (8 * sk)) << 32;
    s.na = 4 - sk;
    s.q += 1;
    madv0(s, c1);
    mfill(s, true);
    const uint32_t code = static_cast<uint32_t>(s.la >> 32);
    s.la <<= 32;
    s.na -= 4;
    madv0(s, c1);
    mfill(s, true);
    madv0(s, c1);
    return code;
}

DEV uint32_t mpos(const MSrc& s) { return 16 * s.j + 4 * s.q - s.na - s.lo15; }

DEV void main7_packet(const rc_batch_dev& bt, const rc_workspace_dev& ws, uint32_t pkt, const Lds7& x, Main7& m)
{
    const uint32_t len = bt.in_len[pkt];
    const uint32_t cap = bt.out_cap[pkt];
    if (len == 0) { bt.out_len[pkt] = 0; ws.claims[pkt] = 0; return; }     // compress.c:513
    uint8_t* root = x.lane;
    uint8_t* stats = x.lane + kStats7;
    // a new packet: generation, first wanted chunk (published once the stream is set up)
    m.gen = m.gen % 15u + 1u;
    ByteSink o;
    sink_init(o, bt.out + bt.out_off[pkt], cap);
    MSrc in;
    uint32_t code = msrc_init(in, bt.in + bt.in_off[pkt], len);
    m.want = in.j + 1;
    *reinterpret_cast<uint2*>(x.mctl) = make_uint2(mctl_word(m.head, m.req, m.want, m.gen), pkt);
    Root R;
    root3_clear<false>(root, R);
    {
        const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (int i = 0; i < 16; ++i) reinterpret_cast<uint4*>(stats)[i] = z;
    }
    uint32_t rtot = 1 + 256;
    double rrt = rcp64(rtot);
    uint32_t low = 0, range = ~0u;
    uint32_t order = 0, a = 0, p = 0, nodes = 1, claims = 0, x0 = 0;
    bool repeat = false, rootonly = false;
    bool stall = false, done = false, off = false, fail = false;
    bool ring_ok = true;      // room in the ring for this step's element (from the last step's h_ctl)

    PROF_DECL
    for (;;) {
        // ------------------------------------------------------------ top
        // (the control words and the slot are used at the end of the step, the
        // ring's confirmed tail at the top of the next one: their LDS round
        // trip stays off the step's chain)
        const uint2 hw = *reinterpret_cast<const uint2*>(x.hctl);
        const uint32_t hc = hw.x;
        const uint4 sl = *reinterpret_cast<const uint4*>(x.lane + kSlot7);
        const uint32_t stp = stats[p];
        sink_flush(o);
        const bool go = !done && !stall && ring_ok;
        const uint32_t st = (go && order >= 1) ? stp : 0u;
        const uint32_t t1 = st & 31u, d1 = t1 - (st >> 5);
        bool need = go && !rootonly && order >= 2 && repeat;
        // order 1 (compress.c:536-568): an escape is coded here, a hit goes to the helper
        const bool o1 = go && !rootonly && !need && order >= 1 && t1 > 0;
        const uint32_t esc1 = kSubEscDelta * d1, tot1 = o1 ? esc1 + kSubDelta * t1 : 1u;
        const uint32_t r1 = udiv16d(range, tot1, rcp64(tot1));
        const bool e1 = o1 && code - low < esc1 * r1;
        need = need || (o1 && !e1);
        if (any_lane(need)) {
            // the request: the coder state at the top of this step
            if (need) {
                *reinterpret_cast<uint4*>(x.mbox) =
                    make_uint4(low, code, range, p | (a << 8) | (x0 << 16) | (order << 24) | ((repeat ? 1u : 0u) << 26));
                *reinterpret_cast<uint2*>(x.mbox + 4) =
                    make_uint2((mpos(in) & 0xFFFFu) | (o.n << 16), (nodes & 0xFFFFu) | (claims << 16));
            }
            m.req = need ? (m.req + 1) & 0xFFu : m.req;
        }
        stall = stall || need;
        range = e1 ? r1 : range;
        mdec_code(low, code, range, 0u, esc1, in, x, m, e1);
        // the root (compress.c:570-596)
        const bool rg = go && !need;
        const uint32_t r0 = udiv16d(range, rtot, rrt);
        const uint32_t cd0 = udiv_lo16(code - low, r0);
        const bool eos = rg && cd0 < 1;
        const bool past = rg && !eos && cd0 - 1 >= rtot - 1;
        const bool sym = rg && !eos && !past;
        range = sym ? r0 : range;
        uint32_t under0 = 0, cnt0 = 0;
        const uint32_t v = root3_search(root, R, sym ? cd0 - 1 : 0u, under0, cnt0);
        mdec_code(low, code, range, 1 + under0, 1 + cnt0, in, x, m, sym);
        if (sym) {
            root3_add<false>(root, R, v, cnt0);
            rtot = (rtot + kRootDelta) & 0xFFFF;
        }
        if (rare_lane(sym && (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit))) {
            if (sym && (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit))
                rtot = root3_rescale<false>(root, R);
        }
        rrt = sym ? rcp64(rtot) : rrt;
        rootonly = rg ? false : rootonly;
        // the element joins bucket p: new to its order-2 context and (the
        // assumption rc_dec6_verify checks) to order 1; nodes as compress.c creates them
        nodes += sym ? (cnt0 == 0 ? 1u : 0u) + (order >= 1 ? 1u : 0u) + (order >= 2 ? 1u : 0u) : 0u;
        const bool o1v = sym && order >= 1;
        if (o1v) stats[p] = static_cast<uint8_t>(st + 1);
        const bool full = o1v && t1 >= kTabCap;
        if (o1v && !full) x.ring[m.head & (kRing7 - 1)] = p | (t1 << 8) | (a << 16) | (v << 24);
        m.head = (o1v && !full) ? (m.head + 1) & 0xFFu : m.head;
        x0 = (sym && order == 0) ? v : x0;
        const bool fl = sym && o.n >= o.cap;                           // compress.c:617
        claims += (o1v && !fl) ? 1u : 0u;
        const bool lv = past || full || (sym && nodes >= kMaxNodes);
        off = off || lv;
        fail = fail || fl;
        done = done || eos || lv || fl;
        sink_put(o, v, 1, sym && !lv && !fl);
        a = sym ? p : a;
        p = sym ? v : p;
        order += (sym && order < 2) ? 1u : 0u;
        repeat = sym ? false : repeat;
        PROF(0)
        // ------------------------------------------------------------ end
        // answers: the helper's coder state, bytes and symbols
        const bool rdy = stall && ((hc >> 8) & 0xFFu) == m.req;
        if (any_lane(rdy)) {
            const uint4 w0 = *reinterpret_cast<const uint4*>(x.mbox);
            const uint2 w1 = *reinterpret_cast<const uint2*>(x.mbox + 4);
            low = rdy ? w0.x : low;
            code = rdy ? w0.y : code;
            range = rdy ? w0.z : range;
            mskip(in, w0.w >> 26, x, m, rdy);
            const uint32_t nout = (w0.w >> 24) & 3u;
            sink_put(o, w0.w & 0xFFFFFFu, nout, rdy);
            p = rdy ? (w1.x & 0xFFu) : p;
            a = rdy ? ((w1.x >> 8) & 0xFFu) : a;
            order = rdy ? ((w1.x >> 16) & 3u) : order;
            repeat = rdy ? ((w1.x >> 18) & 1u) != 0 : repeat;
            rootonly = rdy ? ((w1.x >> 19) & 1u) != 0 : rootonly;
            const bool hlv = rdy && ((w1.x >> 20) & 1u) != 0;
            const bool hfl = rdy && ((w1.x >> 21) & 1u) != 0;
            nodes = rdy ? (w1.y & 0xFFFFu) : nodes;
            claims = rdy ? (w1.y >> 16) : claims;
            off = off || hlv;
            fail = fail || hfl;
            done = done || hlv || hfl;
            stall = stall && !rdy;
        }
        PROF(1)
        // input: the next chunk from the slot, the lookahead topped up
        mtake(in, sl, hc, m, in.q == 4);
        mfill(in, true);
        mfill(in, true);
        mpublish(x, m);
        ring_ok = ((m.head - (hw.y & 0xFFu)) & 0xFFu) < kRing7 - 1;
#ifdef RC_LANE_HOST_TEST
        dec7_host_kick();
#endif
        PROF(2)
        // once a quarter of the wavefront has left, the rest follow
        const uint32_t left = static_cast<uint32_t>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(off)));
        if (left >= kWaveBail7) { off = off || !done; done = true; }
        if (!any_lane(!done)) break;
#ifdef RC_PROFILE
        prof_acc[8] += 1;                                                       // steps
        prof_acc[9] += static_cast<unsigned long long>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(stall)));
        prof_acc[10] += static_cast<unsigned long long>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(go)));
        prof_acc[11] += any_lane(go) ? 0ull : 1ull;                             // idle steps
        prof_acc[6] += static_cast<unsigned long long>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(!done && !stall && !ring_ok)));
        prof_acc[7] += static_cast<unsigned long long>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(done)));
        prof_acc[5] += static_cast<unsigned long long>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(!done && in.q == 4)));
#endif
        if (!any_lane(go)) DEC7_IDLE();
        PROF(3)
    }
    // no request of this packet may still be open when the next one starts
    // (the mailbox is reused): lanes that left while stalled wait for their answer
    while (any_lane(((*x.hctl >> 8) & 0xFFu) != m.req)) DEC7_IDLE();
    PROF_FLUSH(16)
    if (off) { bail(ws, pkt); ws.claims[pkt] = 0xFFFFFFFFu; return; }
    // an output that does not fit returns 0 (compress.c:617) once the check has
    // passed: until then out_len holds the bytes decoded (bit 31 of the claims)
    sink_finish(o, true);
    bt.out_len[pkt] = o.n;
    ws.claims[pkt] = claims | (fail ? 0x80000000u : 0u);
}

}  // namespace

#ifndef RC_LANE_HOST_TEST
// 4 main, 4 storing and 4 serving wavefronts per workgroup (waves w, w + 4
// and w + 8 share a SIMD), one workgroup per CU (its LDS)
extern "C" __global__ __launch_bounds__(768) void rc_decompress_dec7(rc_batch_dev b, rc_workspace_dev ws)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t wave = threadIdx.x >> 6, l = threadIdx.x & 63;
    const uint32_t role = wave >> 2;          // 0 main, 1 storing helper, 2 serving helper
    const uint32_t L = (wave & 3) * 64 + l;
    const Lds7 x = lds7(smem, L, kLanes7);
    const uint32_t slot = blockIdx.x * kLanes7 + L;
    if (role == 0) *reinterpret_cast<uint2*>(x.mctl) = make_uint2(0u, slot < b.n ? kNoPkt7 : kFin7);
    else x.hctl[role - 1] = 0u;
    __syncthreads();
    uint8_t* tab = static_cast<uint8_t*>(ws.dec6_pool) + static_cast<size_t>(slot) * RC_DEC6_TAB_BYTES;
    if (role == 1) {
        Store7 t = {0u};
        for (;;) {
            bool fin = false;
            const bool busy = store7_iter(x, tab, t, fin);
            if (fin) break;
#ifdef DEC7_SSLEEP
            __builtin_amdgcn_s_sleep(DEC7_SSLEEP);
#else
            if (!busy) __builtin_amdgcn_s_sleep(1);
#endif
        }
        return;
    }
    if (role == 2) {
        Help7 h;
        help7_init(h);
#ifdef RC_PROFILE
        unsigned long long it = 0, idle = 0, t0 = prof_now();
#endif
        for (;;) {
            bool fin = false;
            const bool busy = help7_iter(b, x, tab, h, fin);
            if (fin) break;
#ifdef RC_PROFILE
            ++it; idle += busy ? 0ull : 1ull;
#endif
            if (!busy) __builtin_amdgcn_s_sleep(1);
        }
#ifdef RC_PROFILE
        if (l == 0) {
            atomicAdd(&g_prof[32], it);
            atomicAdd(&g_prof[33], idle);
            atomicAdd(&g_prof[34], prof_now() - t0);
            atomicAdd(&g_prof[35], h.ps);
            atomicAdd(&g_prof[36], h.pt);
            atomicAdd(&g_prof[37], h.pr);
            atomicAdd(&g_prof[38], h.pw);
        }
#endif
        return;
    }
#ifdef DEC7_PRIO
    __builtin_amdgcn_s_setprio(DEC7_PRIO);
#endif
    const uint32_t* order = ws.order && !ws.bins[RC_LEN_BINS] ? ws.order : nullptr;
    Main7 m = {0u, 0u, 0u, 0u};
    for (uint32_t i = slot; i < b.n; i += gridDim.x * kLanes7) {
        const uint32_t pkt = order ? order[i] : i;
        main7_packet(b, ws, pkt, x, m);
    }
    x.mctl[1] = kFin7;
}


// The decoder over the batch, then rc_dec6's check; packets off its fast path
// or failing the check are listed in ws->enc2_list, count ws->counters[3].
extern "C" int rc_hip_dec7_launch(const rc_batch_dev* b, const rc_workspace_dev* ws, uint32_t blocks, void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (ws->lane_active != 64) return static_cast<int>(hipErrorInvalidValue);
    hipLaunchKernelGGL(rc_decompress_dec7, dim3(blocks), dim3(768), lds7_bytes(kLanes7), st, *b, *ws);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
    return rc_hip_dec6_verify_launch(b, ws, stream);
}
#endif  // RC_LANE_HOST_TEST
