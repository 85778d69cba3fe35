// rc_dec6.hip -- record-light range decoder (compress.c:498-627), bit-exact.
//
// One packet per lane.  The bucket algebra: position j's order-1 context is
// x[j-1], its order-2 context (x[j-2], x[j-1]); both hold only the positions
// of bucket x[j-1], and every sub-context statistic is a function of those
// elements (a = x[j-2], v = x[j], decoded at order 2 or not).  A decoder that
// keeps each bucket as a 64-B record in HBM reads and writes one for every
// byte -- one random read-modify-write per byte over a 1-GB table, which bound
// the round-2 decoder (rc_dec4.hip, retired in round 5).  Here the
// common step touches no model in memory at all:
//
//   * per bucket, one LDS byte: t1 (positions that visited order 1) and
//     r1 = t1 - d1 (those that found their symbol there): the order-1
//     context's escapes 5 d1 and total 5 d1 + 2 t1 (compress.c:536-568);
//   * a symbol decoded at the root after escaping order 1 is new to the
//     order-1 context -- compress.c escapes only past symbols a context
//     lacks -- so (x[j-1], x[j]) is a new bigram, and position j+1's order-2
//     context (x[j-1], x[j]) has never been visited: its escapes are 0 and
//     compress.c skips it (:536-538).  The step after a root-decoded byte
//     therefore needs nothing but the LDS byte, the root and the coder.
//
// Every element also goes, with a blind 2-B store (no read), into the lane's
// bucket records: a 16-B record per bucket for its first 8 order-1 elements
// (4 KB per lane, 268 MB for 65536 lanes), a 48-B one for the next 20, touched
// only by buckets that grow that big.  A random partial write costs about
// what its footprint costs in the 256-MB Infinity Cache
// (tools/mb/membench6.hip: 0.77 us per step over 268 MB, 2.2 us over 1 GB).  A step that
// needs a context's symbols -- order 1 holds the coded symbol (a hit), or the
// order-2 context exists (the step after a hit) -- stalls its lane.  Every
// kBlock6 steps the wavefront runs the rare phase for its stalled lanes
// together: each loads its bucket's records and decodes its step exactly, with
// the bucket algebra over the unsorted elements (order-2 hits, which leave order
// 1 alone, are kept in registers).  An earlier version rebuilt the bucket by
// scanning the packet's decoded output instead: ~40 dependent 16-B loads per
// rare phase, 7.3 ms for C2 against 1.06 ms for the common steps alone.

// The common step's one assumption -- a root-decoded byte is new to its
// order-1 context -- holds for every stream compress.c produces, but a
// corrupt stream can escape past a symbol the context holds.  Each lane
// therefore counts the positions it took to start a new bigram (the common
// step's assumptions, and the rare phase's exact findings); the bigrams that
// really are new are at most as many, with equality iff every assumption
// held, i.e. iff the decode followed compress.c's model exactly (every
// context's statistics are functions of which elements it holds).
// rc_dec6_verify counts the distinct bigrams of every decoded packet and
// lists those that differ for the lane kernels, which decode them again.
//
// Off the fast path (listed for the lane kernels from the start): a bucket
// with more than 28 order-1 visits or more than 7 order-1 hits (no rescale is
// possible below that, compress.c:313), more than 4 order-2 hits, the model
// reset (4094 nodes, compress.c:148-157), root codes past symbol 255 (the
// exact path), an output that does not fit, or -- once a quarter of the
// wavefront has left -- the rest of the wavefront (low-entropy batches).
// tests/proto/lane_host.cpp compiles the per-lane code for the host
// (tests/test_lane_host.py, variant v6).

#ifndef RC_LANE_HOST_TEST
#include <hip/hip_runtime.h>
#else
#include "lane_host_shim.h"   // tests/proto: host build of the per-lane logic (test only)
#endif
#include <stdint.h>
#include <type_traits>

#include "rc_abi_internal.h"
#include "rc_udiv.h"
#include "rc_lane_common.h"
#include "rc_root3.h"
#include "rc_dec6_rare.h"
#include "rc_slot.h"

namespace {

#ifndef DEC6_BLOCK
#define DEC6_BLOCK 16
#endif
#ifndef DEC6_PRIO
#define DEC6_PRIO 3
#endif
#ifndef DEC6_HELP_SLEEP
#define DEC6_HELP_SLEEP 4          // the helper wavefront's pause when no lane wants a chunk (x 64 clocks; 2-16 within 0.5 %)
#endif
#ifndef DEC6_RARE_ITERS
#define DEC6_RARE_ITERS 2
#endif
constexpr uint32_t kBlock6 = DEC6_BLOCK;        // common steps between rare phases
constexpr uint32_t kRareIters6 = DEC6_RARE_ITERS;   // rare steps per phase and lane
constexpr uint32_t kWaveBail6 = 16;
constexpr uint32_t kStats6 = kRootStrideDec;     // the LDS bucket bytes follow the root
constexpr uint32_t kLds6 = kRootStrideDec + 256; // 528 B per lane (33 x 16 B: b128 conflict-free)
constexpr uint32_t kDummy6 = 256 * kTab2Rec;    // in the second table's block: the slot of the stores that record nothing

DEV void bail6(const rc_workspace_dev& ws, uint32_t pkt) { bail(ws, pkt); }

// compress.c:148-157 (FREE_SYMBOLS) after the byte at output position n - 1:
// a fresh model -- the root, every bucket byte (the records past a bucket's
// count are never read), order 0 -- while the coder runs on.  The check
// (rc_dec6_verify) counts bigrams per model segment: rst records where each
// segment after the first starts (12 bits each, the count in bits 24-25).
DEV void reset6(uint8_t* root, uint8_t* stats, Root& R, uint32_t& rtot, double& rrt, uint32_t& order, uint32_t& a,
                uint32_t& p, uint32_t& nodes, uint32_t& nh, bool& repeat, bool& o2s, bool& e2d, uint32_t& seg0,
                uint32_t& rst, uint32_t n)
{
    root3_clear<false>(root, R);
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int i = 0; i < 16; ++i) reinterpret_cast<uint4*>(stats)[i] = z;
    rtot = 1 + 256;
    rrt = rcp64(rtot);
    order = 0; a = 0; p = 0; nodes = 1; nh = 0;
    repeat = false; o2s = false; e2d = false;
    rst = (rst | (n << (12 * (rst >> 24)))) + (1u << 24);
    seg0 = n;
}

// another segment fits the record: at most two resets, starts below 4096
DEV bool can_reset6(uint32_t rst, uint32_t n) { return (rst >> 24) < 2 && n < 4096; }

// ---- output: one byte per step (rc_lane_common.h's ByteSink, specialised).
// Bytes gather in a dword (acc, nb of them); a full dword shifts into the
// 16-B window w (a shift register: its dwords in output order, the window's
// lead dwords before an unaligned start counted in ws from the start); a
// full window waits in wp for its store at the top of the next step.  At
// most one window completes per step, and every step (common or rare)
// flushes the previous one first.
struct ByteSink1 {
    uint32_t acc, nb, ws;
    uint4 w, wp;
    bool pend;
    uintptr_t waddr, wpaddr, lo;
    uint32_t n, cap;
};

DEV void sink1_init(ByteSink1& o, uint8_t* p, uint32_t cap)
{
    o.lo = reinterpret_cast<uintptr_t>(p);
    o.waddr = o.lo & ~static_cast<uintptr_t>(15);
    o.wpaddr = o.waddr;
    o.ws = static_cast<uint32_t>(o.lo & 15) >> 2;     // (lead bytes before an unaligned start are never stored)
    o.nb = static_cast<uint32_t>(o.lo & 3);
    o.acc = 0;
    o.w = make_uint4(0u, 0u, 0u, 0u);
    o.wp = o.w;
    o.pend = false;
    o.n = 0;
    o.cap = cap;
}

DEV void sink1_flush(ByteSink1& o)
{
    sink_store(o.wpaddr, o.wp, o.lo, o.pend);
    o.pend = false;
}

DEV void sink1_put(ByteSink1& o, uint32_t v, bool en)
{
    o.acc |= en ? (v << (8 * o.nb)) : 0u;
    o.nb += en ? 1u : 0u;
    o.n += en ? 1u : 0u;
    const bool mv = o.nb == 4;
    o.w.x = mv ? o.w.y : o.w.x; o.w.y = mv ? o.w.z : o.w.y; o.w.z = mv ? o.w.w : o.w.z; o.w.w = mv ? o.acc : o.w.w;
    o.acc = mv ? 0u : o.acc;
    o.nb = mv ? 0u : o.nb;
    o.ws += mv ? 1u : 0u;
    const bool full = o.ws == 4;
    o.wp.x = full ? o.w.x : o.wp.x; o.wp.y = full ? o.w.y : o.wp.y;
    o.wp.z = full ? o.w.z : o.wp.z; o.wp.w = full ? o.w.w : o.wp.w;
    o.wpaddr = full ? o.waddr : o.wpaddr;
    o.pend = o.pend || full;
    o.ws = full ? 0u : o.ws;
    o.waddr += full ? 16 : 0;
}

// the pending window, then the partial one: its ws dwords (the last ws of the
// shift register) and the nb bytes of acc
DEV void sink1_finish(ByteSink1& o)
{
    sink1_flush(o);
    const uint32_t ws = o.ws;
    const uint32_t d[4] = {o.w.x, o.w.y, o.w.z, o.w.w};
    uint32_t q[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t k = 4 - ws + j;                // (j < ws: dword k of the shift register)
        q[j] = j < ws ? (k == 0 ? d[0] : k == 1 ? d[1] : k == 2 ? d[2] : d[3]) : (j == ws ? o.acc : 0u);
    }
    sink_bytes(o.waddr, make_uint4(q[0], q[1], q[2], q[3]), 0ull, 4 * ws + o.nb, o.lo);
}

// Src: SlotSrc (through the LDS slot a helper wavefront refills, rc_slot.h,
// rc_decompress_dec6s) or ByteSrc (the stream's chunks loaded by the lane
// itself: the host build of tests/proto/lane_host.cpp, variant v6).
template <class Src>
DEV void decompress_one6(const rc_batch_dev& bt, const rc_workspace_dev& ws, uint32_t pkt, uint8_t* root,
                         uint8_t* stats, uint8_t* tab, uint8_t* tab2, const uint8_t* itab, Src& in,
                         const double* rtab = nullptr)
{
    constexpr bool kSlot = std::is_same<Src, SlotSrc>::value;
    const uint32_t len = bt.in_len[pkt];
    const uint32_t cap = bt.out_cap[pkt];
    if (len == 0) { bt.out_len[pkt] = 0; ws.claims[pkt] = 0; ws.dec6_resets[pkt] = 0; return; }     // compress.c:513
    ByteSink1 o;
    sink1_init(o, bt.out + bt.out_off[pkt], cap);
    uint32_t code;
    if constexpr (kSlot) {
        code = slot_init(in, bt.in + bt.in_off[pkt], len, pkt);
    } else {
        src_init(in, bt.in + bt.in_off[pkt], len);
        code = static_cast<uint32_t>(in.la >> 32);            // compress.c:344-350 (0 past the end)
        in.la <<= 32;
        in.na -= 4;
        src_refill(in, true);
    }
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
    uint32_t hl[4] = {0u, 0u, 0u, 0u}, nh = 0;   // elements decoded at order 2: p | a << 8 | v << 16
    bool repeat = false;                      // this step's order-2 context has been visited
    // ... once, with one symbol (escapes 5, total 7): the common step codes its escape itself
    bool o2s = false;
    bool e2d = false;                         // that escape coded, the order-1 READ left to the rare step
    bool stall = false, done = false, off = false, fail = false;
    uint32_t seg0 = 0, rst = 0;               // the model segment's first output position; resets (reset6)

    PROF_DECL
    // One loop of common steps; every kBlock6 steps (or once no lane can take
    // one) the rare phase.  The step's memory operations are unconditional --
    // a lane that stores no element stores to its dummy slot -- so that the
    // compiler can wait for an input chunk with vmcnt(n) rather than behind
    // every store in flight (see rc_lane3.hip lane_prefetch).
    uint32_t s = 0;
#ifdef DEC6_STATS_PREFETCH
    uint32_t stn = 0;
    double rtn = 1.0;                         // 1 / the order-1 total of the next step's bucket
#endif
    for (;;) {
        {
            // ------------------------------------------------------ a common step
            uint32_t shc = 0;                                  // (SlotSrc: h_ctl and the slot, used at the end)
            uint4 ssl = make_uint4(0u, 0u, 0u, 0u);
            if constexpr (kSlot) {
                slot_read(in, shc, ssl);
            } else {
                src_fill(in, true);
            }
            sink1_flush(o);
            const bool go = !done && !stall;
#ifdef DEC6_STATS_PREFETCH
            const uint32_t st = (go && order >= 1) ? stn : 0u;
#else
            const uint32_t sraw = stats[p];                    // (read on every path: no exec mask)
            const uint32_t st = (go && order >= 1) ? sraw : 0u;
#endif
            const uint32_t t1 = st & 31u, d1 = t1 - (st >> 5);
            bool need = go && order >= 2 && repeat && !o2s;
            // order 2 when its context holds one visit: an escape is coded here, the
            // context's one symbol stalls the lane (compress.c:536-568 over total 7)
            bool e2 = false;
            const bool c2s = go && order >= 2 && repeat && o2s;
            if (any_lane(c2s)) {
                const uint32_t r2 = udiv16d(range, 7u, 1.0 / 7.0);
                e2 = c2s && code - low < 5u * r2;
                need = need || (c2s && !e2);
                range = e2 ? r2 : range;
                dec_code(low, code, range, 0u, 5u, in, e2);
            }
            // order 1 (compress.c:536-568): READ; an escape is coded here, a hit stalls the lane
            const bool o1 = go && !need && order >= 1 && t1 > 0;
            const uint32_t esc1 = kSubEscDelta * d1, tot1 = o1 ? esc1 + kSubDelta * t1 : 1u;
#ifdef DEC6_STATS_PREFETCH
            const uint32_t r1 = udiv16d(range, tot1, o1 ? rtn : 1.0);
#elif defined(DEC6_RCP_TAB) && !defined(RC_LANE_HOST_TEST)
            // (1 / the order-1 total from the block's table by the bucket byte: a
            // lane without an order-1 code reads an entry it does not use; -0.3 %,
            // within noise: profiles/r6/r6e_dec6_prefetch_rcptab_ab_c2.txt)
            const uint32_t r1 = udiv16d(range, tot1, rtab[st]);
#else
            const uint32_t r1 = udiv16d(range, tot1, rcp64(tot1));
#endif
#ifndef DEC6_READ1
            // READ < escapes without the READ's division: (code - low) / r1 < esc1
            // iff code - low < esc1 r1 (the quotient is then below 2^16: no
            // truncation, compress.c:352); otherwise a hit -- or, on a corrupt
            // stream, a quotient truncated to 16 bits -- both for the rare step,
            // which READs in full
            const bool e1 = o1 && code - low < esc1 * r1;
            need = need || (o1 && !e1);
#else
            const uint32_t cd1 = udiv_lo16(code - low, r1);
            need = need || (o1 && cd1 >= esc1);
            const bool e1 = o1 && cd1 < esc1;
#endif
            need = need && !(ws.dec6_debug & 2);      // (timing experiment: no rare steps, output lost)
            range = e1 ? r1 : range;
            dec_code(low, code, range, 0u, esc1, in, e1);
            // the root (compress.c:570-596)
            const bool rg = go && !need;
            const uint32_t r0 = udiv16d(range, rtot, rrt);
            const uint32_t cd0 = udiv_lo16(code - low, r0);
            const bool eos = rg && cd0 < 1;                                // end of stream
            const bool past = rg && !eos && cd0 - 1 >= rtot - 1;           // past symbol 255: exact path
            const bool sym = rg && !eos && !past;
            range = sym ? r0 : range;
            uint32_t under0 = 0, cnt0 = 0;
#ifndef DEC6_ITAB_LATE
            uint4 i0, i1;
            const uint32_t v = root3_search_inc(root, R, itab, sym ? cd0 - 1 : 0u, under0, cnt0, i0, i1);
#else
            const uint32_t v = root3_search(root, R, sym ? cd0 - 1 : 0u, under0, cnt0);
#endif
            dec_code_late(low, code, range, 1 + under0, 1 + cnt0, in, sym);
            if (sym) {
#ifndef DEC6_ITAB_LATE
                root3_add_pre(root, R, v, cnt0, i0, i1);
#else
                root3_add_inc(root, R, itab, v, cnt0);
#endif
                rtot = (rtot + kRootDelta) & 0xFFFF;
            }
            if (rare_lane(sym && (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit))) {
                if (sym && (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit))
                    rtot = root3_rescale<false>(root, R);
            }
            rrt = sym ? rcp64(rtot) : rrt;
            // the element joins bucket p: new to its order-2 context (never visited) and,
            // by the assumption above, to order 1; nodes as compress.c creates them
            nodes += sym ? (cnt0 == 0 ? 1u : 0u) + (order >= 1 ? 1u : 0u) + (order >= 2 ? 1u : 0u) : 0u;
            const bool o1v = sym && order >= 1;
#ifndef DEC6_STATS_PREFETCH
            stats[p] = static_cast<uint8_t>(o1v ? st + 1 : sraw);   // (written on every path: no exec mask)
#else
            if (o1v) stats[p] = static_cast<uint8_t>(st + 1);
#endif
            const bool full = o1v && t1 >= kTabCap;
            // the element into the bucket's records (a blind 2-B store; no read)
            *GPTR(uint16_t, !(o1v && !full) ? reinterpret_cast<uintptr_t>(tab2) + kDummy6 : rec_addr(tab, tab2, p, t1)) =
                static_cast<uint16_t>(a | (v << 8));
            x0 = (sym && order == 0) ? v : x0;
            const bool fl = sym && o.n >= o.cap;                           // compress.c:617
            claims += (o1v && !fl) ? 1u : 0u;
            const bool rs0 = sym && nodes >= kMaxNodes;                    // compress.c:148-157
            const bool lv = past || full || (rs0 && !can_reset6(rst, o.n + 1));
            off = off || lv;
            fail = fail || fl;
            done = done || eos || lv || fl;
            sink1_put(o, v, sym && !lv && !fl);
            a = sym ? p : a;
            p = sym ? v : p;
            order += (sym && order < 2) ? 1u : 0u;
            repeat = sym ? false : repeat;
            o2s = sym ? false : o2s;
            e2d = go ? (e2 && need) : e2d;
            stall = stall || need;
            if (rare_lane(rs0 && !done)) {
                if (rs0 && !done) reset6(root, stats, R, rtot, rrt, order, a, p, nodes, nh, repeat, o2s, e2d, seg0, rst, o.n);
            }
#ifdef DEC6_STATS_PREFETCH
            stn = stats[p];                           // (the next step's bucket byte, read ahead)
            {
                const uint32_t nt = stn & 31u, nd1 = nt - (stn >> 5);
                rtn = rcp64(max(kSubEscDelta * nd1 + kSubDelta * nt, 1u));
            }
#endif
            PROF(0)
            if constexpr (kSlot) slot_step_end(in, ssl, shc);
            else src_adv(in);
            PROF(5)
        }
        ++s;
        if (s < kBlock6 && any_lane(!done && !stall)) continue;
        s = 0;
        // ------------------------------------------------------------ rare phase
        for (uint32_t it = 0; it < kRareIters6 && any_lane(stall && !done); ++it) {
            const bool rs = stall && !done;
            uint32_t shc = 0;
            uint4 ssl = make_uint4(0u, 0u, 0u, 0u);
            if constexpr (kSlot) {
                slot_read(in, shc, ssl);
            } else {
                src_fill(in, true);
            }
            sink1_flush(o);
            // (no drain before the record loads: a lane's loads of its records come
            // after its stores to them in program order, which the memory pipeline
            // keeps -- as for any store and later load of one address by one thread,
            // between which the compiler puts no wait either; vmcnt retires the
            // loads behind those stores in any case.  -DDEC6_DRAIN: s_waitcnt(0) here)
#ifdef DEC6_DRAIN
            __builtin_amdgcn_s_waitcnt(0);
#endif
            const uint32_t st = rs && order >= 1 ? stats[p] : 0u;
            const uint32_t t1 = st & 31u, d1 = t1 - (st >> 5);
            Hist6 H;
            rec_build(tab, tab2, p, rs ? t1 : 0u, hl, nh, x0, o.n - seg0, rs, H);
            const bool over = false;
            PROF(1)
#ifdef RC_PROFILE
            prof_acc[8] += 1;
            prof_acc[9] += static_cast<unsigned long long>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(rs)));
#endif
            uint32_t nd = 1;                          // live dwords of the element arrays, wave-wide
#pragma unroll
            for (uint32_t j = 1; j < 8; ++j) nd += any_lane(H.k > 4 * j) ? 1u : 0u;
            uint32_t pl[8];
            planes6(H.V, nd, pl);
            const uint32_t km = low_bits(H.k);
            const uint32_t g2 = (rs && order >= 2) ? (eqmask6(H.A, a, nd) & km & ~H.p1) : 0u;
            const uint32_t g1 = km & ~H.hit;
            const uint32_t t2 = popc(g2);
            // distinct values of the order-2 context (members first of their value)
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
            const bool c2 = rs && !over && !e2d && order >= 2 && t2 > 0;
            if (any_lane(c2)) {
                if (sub_decode6(pl, g2, t2, d2, c2, low, code, range, in, v, hu, hc, sf)) at = 2;
            }
            const bool c1 = rs && !over && !sf && at < 0 && order >= 1 && t1 > 0;
            if (any_lane(c1)) {
                if (sub_decode6(pl, g1, t1, d1, c1, low, code, range, in, v, hu, hc, sf)) at = 1;
            }
            // the root, or the hit's interval
            const bool rg = rs && !over && !sf && at < 0;
            const uint32_t r0 = udiv16d(range, rtot, rrt);
            const uint32_t cd0 = udiv_lo16(code - low, r0);
            const bool eos = rg && cd0 < 1;
            const bool past = rg && !eos && cd0 - 1 >= rtot - 1;
            const bool sym0 = rg && !eos && !past;
            range = sym0 ? r0 : range;
            uint32_t under0 = 0, cnt0 = 0;
            const uint32_t v0 = root3_search(root, R, sym0 ? cd0 - 1 : 0u, under0, cnt0);
            const bool sym = sym0 || at > 0;
            v = sym0 ? v0 : v;
            dec_code(low, code, range, sym0 ? 1 + under0 : hu, sym0 ? 1 + cnt0 : hc, in, sym);
            if (sym0) {
                root3_add_inc(root, R, itab, v, cnt0);
                rtot = (rtot + kRootDelta) & 0xFFFF;
            }
            if (rare_lane(sym0 && (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit))) {
                if (sym0 && (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit))
                    rtot = root3_rescale<false>(root, R);
            }
            rrt = sym0 ? rcp64(rtot) : rrt;
            PROF(2)
            // the element joins its contexts (compress.c:598-615)
            const uint32_t eqv = peq6(pl, v) & km;
            const bool n2 = order >= 2 && (eqv & g2) == 0;
            const bool n1 = order >= 1 && at != 2 && (eqv & g1) == 0;
            const bool nb = eqv == 0;                                       // a new bigram (p, v)
            nodes += sym ? (sym0 && cnt0 == 0 ? 1u : 0u) + (n2 ? 1u : 0u) + (n1 ? 1u : 0u) : 0u;
            const bool o1v = sym && order >= 1 && at != 2;
            const uint32_t nst = st + 1 + (n1 ? 0u : 32u);
            if (o1v) stats[p] = static_cast<uint8_t>(nst);
            const bool tfull = o1v && t1 >= kTabCap;
            if (o1v && !tfull)
                *GPTR(uint16_t, rec_addr(tab, tab2, p, t1)) =
                    static_cast<uint16_t>(a | (v << 8));
            claims += (sym && order >= 1 && nb && o.n < o.cap) ? 1u : 0u;
            const bool h2 = sym && at == 2;
            const uint32_t he = p | (a << 8) | (v << 16);
#pragma unroll
            for (uint32_t h = 0; h < 4; ++h) hl[h] = (h2 && nh == h) ? he : hl[h];
            const bool hfull = h2 && nh >= 4;
            nh += h2 ? 1u : 0u;
            const bool fl = sym && o.n >= o.cap;
            const bool rs0 = rs && sym && nodes >= kMaxNodes;               // compress.c:148-157
            const bool lv = over || sf || past || hfull || tfull || (o1v && !n1 && (st >> 5) >= 7) ||
                            (rs0 && !can_reset6(rst, o.n + 1));
            off = off || (rs && lv);
            fail = fail || (rs && fl);
            done = done || (rs && (eos || lv || fl));
            sink1_put(o, v, sym && !lv && !fl);
            a = sym ? p : a;
            p = sym ? v : p;
            order += (sym && order < 2) ? 1u : 0u;
            repeat = sym ? !nb : repeat;
            // the step after a hit has a visited order-2 context (p, v): its visits are
            // the elements of bucket p with value v.  One visit: one symbol, the
            // common step's; more: another rare step.
            const bool one = sym && popc(eqv) == 1;
            o2s = rs ? one : o2s;
            e2d = rs ? false : e2d;
            stall = rs ? (sym && !lv && !fl && order >= 2 && repeat && !one) : stall;
            if (rare_lane(rs0 && !done)) {
                if (rs0 && !done) {
                    reset6(root, stats, R, rtot, rrt, order, a, p, nodes, nh, repeat, o2s, e2d, seg0, rst, o.n);
                    stall = false;
                }
            }
            if constexpr (kSlot) slot_step_end(in, ssl, shc);
            else src_adv(in);
            PROF(3)
        }
        // (no wait for the phase's stores here: the rare steps consume their record
        // loads themselves, so the common steps hold no load the compiler would
        // wait for, and the next phase's record loads wait behind the stores in
        // any case (vmcnt retires in order).  -DDEC6_END_WAIT: s_waitcnt(0) here,
        // 0.3-0.8 % slower, profiles/r4e_dec6_end_wait.txt)
#ifdef DEC6_END_WAIT
        __builtin_amdgcn_s_waitcnt(0);
#endif
#ifdef DEC6_STATS_PREFETCH
        stn = stats[p];
        {
            const uint32_t nt = stn & 31u, nd1 = nt - (stn >> 5);
            rtn = rcp64(max(kSubEscDelta * nd1 + kSubDelta * nt, 1u));
        }
#endif
        // once a quarter of the wavefront has left, the rest follow
        const uint32_t left = static_cast<uint32_t>(__builtin_popcountll(__builtin_amdgcn_ballot_w64(off)));
        if (left >= kWaveBail6) { off = off || !done; done = true; }
        PROF(4)
        if (!any_lane(!done)) break;
    }
    PROF_FLUSH(16)
#ifndef DEC6_NO_USED_CHECK            // (tests/test_lane_host.py: the build without it, for comparison)
    if constexpr (kSlot) {
        // Every stream compress.c writes is read to its end: the seed takes 4
        // bytes and each settled byte of the coder one more, as the encoder
        // emitted them, and the flush wrote 0-4 bytes past those
        // (compress.c:114-146, :344-371), so a decode that reaches its end of
        // stream has taken between C and C + 4 bytes (zeros past the end).  A
        // decode that took otherwise saw other bytes than the packet's -- or
        // is a corrupt stream's, which the lane kernels decode as well -- and
        // goes to them (tests/test_lane_host.py stale-chunk injections).
        const uint32_t used = 16 * in.j + 4 * in.q - in.lo15 - in.na;
        off = off || (!fail && (used < len || used > len + 4));
    }
#endif
    if (off) { bail6(ws, pkt); ws.claims[pkt] = 0xFFFFFFFFu; return; }
    ws.dec6_resets[pkt] = rst;
    if constexpr (kSlot) ws.dec6_icks[pkt] = in.cks;       // (rc_slot.h slot_mix; the helper's in dec6_hcks)
    // an output that does not fit returns 0 (compress.c:617) once the check has
    // passed: until then out_len holds the bytes decoded (bit 31 of the claims)
    sink1_finish(o);
    bt.out_len[pkt] = o.n;
    ws.claims[pkt] = claims | (fail ? 0x80000000u : 0u);
}

}  // namespace

#ifndef RC_LANE_HOST_TEST
// The decoder, with the lanes' input through LDS (rc_slot.h): waves 0-3 decode,
// wave w + 4 (on wave w's SIMD) keeps their slots filled.  LDS per lane:
// root | slot (the root's pad) | bucket bytes, then m_ctl / m_pkt, h_ctl;
// then root3_inc_init's table (16 x 32 B).
constexpr uint32_t kLanes6s = 256;
extern "C" __global__ __launch_bounds__(512) void rc_decompress_dec6s(rc_batch_dev b, rc_workspace_dev ws)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t wave = threadIdx.x >> 6;
    const bool helper = wave >= 4;
    const uint32_t L = (wave & 3) * 64 + (threadIdx.x & 63);
    uint8_t* root = smem + L * kLds6;
    uint8_t* stats = root + kStats6;
    uint8_t* slotp = root + 256;
    uint32_t* mctl = reinterpret_cast<uint32_t*>(smem + kLanes6s * kLds6) + 2 * L;
    uint32_t* hctl = reinterpret_cast<uint32_t*>(smem + kLanes6s * kLds6 + 8 * kLanes6s) + L;
    uint8_t* itab = smem + kLanes6s * (kLds6 + 12);
    const uint32_t slot = blockIdx.x * kLanes6s + L;
    if (!helper) *reinterpret_cast<uint2*>(mctl) = make_uint2(0u, slot < b.n ? kNoPktS : kFinS);
    else *hctl = 0u;
    if (threadIdx.x < 16) root3_inc_init(itab, threadIdx.x);
    double* rtab = reinterpret_cast<double*>(itab + 512);
#ifdef DEC6_RCP_TAB
    // 1 / the order-1 total of every bucket byte (t1 | (t1 - d1) << 5: total
    // 5 d1 + 2 t1, compress.c:536-568; 1 where t1 = 0)
    if (threadIdx.x < 256) {
        const uint32_t t1 = threadIdx.x & 31u, r1 = threadIdx.x >> 5;
        const uint32_t tot = (t1 > 0 && r1 <= t1) ? kSubEscDelta * (t1 - r1) + kSubDelta * t1 : 1u;
        rtab[threadIdx.x] = rcp64(tot);
    }
#endif
    __syncthreads();
    if (helper) {
        SlotHelp h;
        slot_help_init(h);
#ifdef DEC6_HELP_COUNT
        uint32_t nb = 0, ni = 0;     // (diagnostic: the helper's busy and idle passes, ws.counters[5..6])
#endif
        for (;;) {
            bool fin = false;
            const bool busy = slot_help_iter(b, mctl, hctl, slotp, h, ws.dec6_hcks, ws.n_cap, fin);
#ifdef DEC6_HELP_COUNT
            nb += busy ? 1u : 0u;
            ni += busy ? 0u : 1u;
#endif
            if (fin) break;
            if (!busy) __builtin_amdgcn_s_sleep(DEC6_HELP_SLEEP);
        }
#ifdef DEC6_HELP_COUNT
        if ((threadIdx.x & 63) == 0) { atomicAdd(&ws.counters[5], nb); atomicAdd(&ws.counters[6], ni); }
#endif
        return;
    }
    uint8_t* tab = static_cast<uint8_t*>(ws.dec6_pool) + static_cast<size_t>(slot) * kTab1;
    uint8_t* tab2 = static_cast<uint8_t*>(ws.dec6_pool) + static_cast<size_t>(ws.lane_slots) * kTab1 +
                    static_cast<size_t>(slot) * kTab2;
    const uint32_t* order = ws.order && !ws.bins[RC_LEN_BINS] ? ws.order : nullptr;
    // the decoding wavefront ahead of its helper when both can issue (-0.5 %,
    // profiles/r4e_dec6_prio.txt; -DDEC6_PRIO=0: equal)
    __builtin_amdgcn_s_setprio(DEC6_PRIO);
    SlotSrc in;
    in.gen = 0; in.mctl = mctl; in.hctl = hctl; in.slot = slotp;
    for (uint32_t i = slot; i < b.n; i += gridDim.x * kLanes6s) {
        const uint32_t pkt = order ? order[i] : i;
        decompress_one6(b, ws, pkt, root, stats, tab, tab2, itab, in, rtab);
    }
    mctl[1] = kFinS;
}

// Counts the distinct bigrams of each packet rc_decompress_dec6s decoded and
// lists the packets whose count differs from the decoder's (see the header).
// A wavefront per packet: a 65536-bit set in LDS, cleared per packet; a lane
// sets the bits of its positions' bigrams with LDS atomics and counts the
// bits it found clear.  The common packet (one model segment, at most
// 64 x kVerDw dwords) is software-pipelined two deep: its output dwords were
// loaded -- lane l round r: dword 64 r + l -- while the wave counted the
// packet before, and the header of the one after is in flight (vector loads
// only, so that waiting for an atomic's return never waits for them).  Other
// packets take verify_slow.
constexpr uint32_t kVerifyWaves = 4;
constexpr uint32_t kVerifyBlocksPerCu = 10;     // 32 KB of LDS per workgroup: 5 resident per CU, two rounds
constexpr uint32_t kVerDw = 8;                  // dwords per lane: packets to 2 KB - 4

// the header words of packet k, lane l < 8: claims, out_len, out_off (2),
// resets, and the hand-off's check sums (the decoder's, the helper's and its
// last chunk's term: rc_slot.h)
DEV uint32_t vhead_load(const rc_batch_dev& b, const rc_workspace_dev& ws, uint32_t k, uint32_t l)
{
    const uint32_t* src = l == 0 ? ws.claims + k
                        : l == 1 ? b.out_len + k
                        : l < 4 ? reinterpret_cast<const uint32_t*>(b.out_off + k) + (l - 2)
                        : l == 4 ? ws.dec6_resets + k
                        : l == 5 ? ws.dec6_icks + k
                        : l == 6 ? ws.dec6_hcks + k
                                 : ws.dec6_hcks + ws.n_cap + k;
    return (k < b.n && l < 8) ? *src : 0u;
}


struct VHead {
    uint32_t cl, n, rst, off, nd;   // off: lo - sb; nd: dwords from sb
    uintptr_t lo, sb;
    bool skip, fast, cks;           // cks: the hand-off's sums agree
};

DEV VHead vhead_get(const rc_batch_dev& b, uint32_t k, uint32_t hv)
{
    VHead h;
    h.cl = __shfl(hv, 0);
    h.n = __shfl(hv, 1);
    const uint64_t oo = static_cast<uint64_t>(static_cast<uint32_t>(__shfl(hv, 2))) |
                        static_cast<uint64_t>(static_cast<uint32_t>(__shfl(hv, 3))) << 32;
    h.rst = __shfl(hv, 4);
    h.cks = cks_agree(__shfl(hv, 5), __shfl(hv, 6), __shfl(hv, 7));
    h.skip = k >= b.n || h.cl == 0xFFFFFFFFu;                    // none, or left to the lanes already
    h.lo = reinterpret_cast<uintptr_t>(b.out) + oo;
    h.sb = h.lo & ~static_cast<uintptr_t>(3);
    h.off = static_cast<uint32_t>(h.lo - h.sb);
    h.nd = (h.off + h.n + 3) >> 2;
    h.fast = !h.skip && (h.rst >> 24) == 0 && h.nd <= 64 * kVerDw;
    return h;
}

DEV void vdata_load(const VHead& h, uint32_t l, uint32_t (&w)[kVerDw])
{
    const uint32_t* p = reinterpret_cast<const uint32_t*>(h.sb);
#pragma unroll
    for (uint32_t r = 0; r < kVerDw; ++r) {
        const uint32_t c = 64 * r + l;
        w[r] = (h.fast && c < h.nd) ? p[c] : 0u;
    }
}

// ck: the slot hand-off's check sums agree (rc_slot.h slot_mix)
DEV void vresult(const rc_batch_dev& b, const rc_workspace_dev& ws, uint32_t k, uint32_t cl, uint32_t cnt, bool ck,
                 uint32_t l)
{
    for (int sft = 32; sft >= 1; sft >>= 1) cnt += static_cast<uint32_t>(__shfl_xor(static_cast<int>(cnt), sft));
    const uint32_t want = cl & 0x7FFFFFFFu;
    const bool ok = cnt == want && ck && !(ws.dec6_debug & 1);
    if (l == 0 && !ok) {
        const uint32_t i = atomicAdd(&ws.counters[3], 1u);
        ws.enc2_list[i] = k;
        if (!ck) atomicAdd(&ws.counters[7], 1u);      // (the hand-off sums disagreed: enet_rc_debug_counter 7)
    }
    if (l == 0 && ok && (cl >> 31)) b.out_len[k] = 0;     // compress.c:617
}

DEV void vclear(uint4* set4, uint32_t l)
{
#pragma unroll
    for (uint32_t i = 0; i < 512 / 64; ++i) set4[i * 64 + l] = make_uint4(0u, 0u, 0u, 0u);
}

// the common packet: its dwords in w
DEV void verify_fast(const rc_batch_dev& b, const rc_workspace_dev& ws, uint32_t k, const VHead& h,
                     const uint32_t (&w)[kVerDw], uint4* set4, uint32_t l)
{
    uint32_t* set = reinterpret_cast<uint32_t*>(set4);
    vclear(set4, l);
    uint32_t cnt = 0, last = 0;                  // last: lane 63's dword of the round before
#pragma unroll
    for (uint32_t r = 0; r < kVerDw; ++r) {
        if (64 * r >= h.nd) break;
        const uint32_t up = static_cast<uint32_t>(__shfl_up(static_cast<int>(w[r]), 1));
        const uint32_t pw = l ? up : last;       // the dword before this lane's
        last = static_cast<uint32_t>(__shfl(static_cast<int>(w[r]), 63));
        const uint32_t c = 64 * r + l;
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t) {
            const uint32_t x = (w[r] >> (8 * t)) & 0xFFu;
            const uint32_t pv = t ? (w[r] >> (8 * t - 8)) & 0xFFu : pw >> 24;
            const uint32_t pos = 4 * c + t - h.off;          // position in the packet (wraps below 0)
            const bool in = pos >= 1 && pos < h.n;
            // (no branch: a position outside ORs nothing into a word of the lane's own,
            // so the four atomics issue back to back and their returns are awaited once)
            const uint32_t bg = (pv << 8) | x, bit = 1u << (bg & 31);
#ifdef VERIFY_RETURNS
            const uint32_t old = atomicOr(&set[in ? bg >> 5 : l], in ? bit : 0u);
            cnt += (in && !(old & bit)) ? 1u : 0u;
#else
            atomicOr(&set[in ? bg >> 5 : l], in ? bit : 0u);
#endif
        }
    }
#ifndef VERIFY_RETURNS
    // the distinct bigrams are the set's bits: the ORs go without returns (no
    // wait per round), and one pass counts them.  (A wavefront's LDS
    // operations complete in order, so the reads see every lane's ORs.)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (uint32_t i = 0; i < 512 / 64; ++i) {
        const uint4 q = set4[i * 64 + l];
        cnt += static_cast<uint32_t>(__builtin_popcount(q.x) + __builtin_popcount(q.y) + __builtin_popcount(q.z) +
                                     __builtin_popcount(q.w));
    }
#endif
    vresult(b, ws, k, h.cl, cnt, h.cks, l);
}

// any other packet: per model segment (compress.c:148-157: bigrams are counted
// within each, the pair across a reset belongs to neither), loads as it goes
DEV void verify_slow(const rc_batch_dev& b, const rc_workspace_dev& ws, uint32_t pkt, uint4* set4, uint32_t l)
{
    uint32_t* set = reinterpret_cast<uint32_t*>(set4);
    {
        const uint32_t cl = ws.claims[pkt];
        const uint32_t n = b.out_len[pkt];
        const uintptr_t lo = reinterpret_cast<uintptr_t>(b.out + b.out_off[pkt]);
        const uint32_t rst = ws.dec6_resets[pkt], nseg = (rst >> 24) + 1;
        uint32_t cnt = 0;
        for (uint32_t sg = 0; sg < nseg; ++sg) {
            const uint32_t s0 = sg ? (rst >> (12 * (sg - 1))) & 0xFFFu : 0u;
            const uint32_t s1 = sg + 1 < nseg ? (rst >> (12 * sg)) & 0xFFFu : n;
#pragma unroll
            for (uint32_t i = 0; i < 512 / 64; ++i) set4[i * 64 + l] = make_uint4(0u, 0u, 0u, 0u);
            __builtin_amdgcn_wave_barrier();
            const uintptr_t slo = lo + s0;
            const uintptr_t sb = slo & ~static_cast<uintptr_t>(15);
            const uint32_t m = s1 > s0 ? s1 - s0 : 0u;
            const uint32_t chunks = m > 1 ? static_cast<uint32_t>((slo + m - sb + 15) >> 4) : 0u;
            for (uint32_t c = l; c < chunks; c += 64) {
                const uintptr_t a = sb + 16 * c;
                const uint4 w = *reinterpret_cast<const uint4*>(a);
                uint32_t prev = a > slo ? *reinterpret_cast<const uint8_t*>(a - 1) : 0u;
                const uint32_t d[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (uint32_t t = 0; t < 16; ++t) {
                    const uint32_t x = (d[t >> 2] >> (8 * (t & 3))) & 0xFFu;
                    const uintptr_t at = a + t;                   // position at - lo
                    if (at > slo && at < slo + m) {
                        const uint32_t bg = (prev << 8) | x;
                        atomicOr(&set[bg >> 5], 1u << (bg & 31));
                    }
                    prev = x;
                }
            }
            __builtin_amdgcn_wave_barrier();
            uint32_t sc = 0;
#pragma unroll
            for (uint32_t i = 0; i < 512 / 64; ++i) {
                const uint4 q = set4[i * 64 + l];
                sc += static_cast<uint32_t>(__builtin_popcount(q.x) + __builtin_popcount(q.y) +
                                            __builtin_popcount(q.z) + __builtin_popcount(q.w));
            }
            cnt += sc;
            __builtin_amdgcn_wave_barrier();
        }
        vresult(b, ws, pkt, cl, cnt, cks_agree(ws.dec6_icks[pkt], ws.dec6_hcks[pkt], ws.dec6_hcks[ws.n_cap + pkt]), l);
    }
}

DEV void verify_one(const rc_batch_dev& b, const rc_workspace_dev& ws, uint32_t k, const VHead& h,
                    const uint32_t (&w)[kVerDw], uint4* set4, uint32_t l)
{
    if (h.skip) return;
    if (h.fast) verify_fast(b, ws, k, h, w, set4, l);
    else verify_slow(b, ws, k, set4, l);
    __builtin_amdgcn_wave_barrier();
}

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5)))
void rc_dec6_verify(rc_batch_dev b, rc_workspace_dev ws)
{
    __shared__ uint4 bits[kVerifyWaves][512];
    const uint32_t wave = threadIdx.x >> 6, l = threadIdx.x & 63;
    uint4* set4 = bits[wave];
    const uint32_t stride = gridDim.x * kVerifyWaves;
    uint32_t k = blockIdx.x * kVerifyWaves + wave;
    if (k >= b.n) return;
    // two register sets, A and B: a packet's dwords load while the other's count
    uint32_t wa[kVerDw], wb[kVerDw];
    uint32_t hva = vhead_load(b, ws, k, l);
    VHead ha = vhead_get(b, k, hva), hb;
    vdata_load(ha, l, wa);
    uint32_t hvb = vhead_load(b, ws, k + stride, l);
    for (;;) {
        // A holds packet k; B's header (packet k + stride) is in flight
        hb = vhead_get(b, k + stride, hvb);
        vdata_load(hb, l, wb);
        hva = vhead_load(b, ws, k + 2 * stride, l);
        verify_one(b, ws, k, ha, wa, set4, l);
        k += stride;
        if (k >= b.n) break;
        ha = vhead_get(b, k + stride, hva);
        vdata_load(ha, l, wa);
        hvb = vhead_load(b, ws, k + 2 * stride, l);
        verify_one(b, ws, k, hb, wb, set4, l);
        k += stride;
        if (k >= b.n) break;
    }
}

// The decoder over the batch, then the check; packets off its fast path or
// failing the check are listed in ws->enc2_list, count in ws->counters[3],
// for the lane kernels.
extern "C" int rc_hip_dec6_verify_launch(const rc_batch_dev* b, const rc_workspace_dev* ws, void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint32_t vb = (b->n + kVerifyWaves - 1) / kVerifyWaves;
    // twice the resident workgroups: each wave walks several packets, the next
    // one's loads in flight, and the second round starts as first-round
    // workgroups finish (C2: 66 -> 60 us against the resident count, 72 at 64
    // per CU; profiles/r5_scan_grid/vbpc_c2.txt)
    static const char* vb_env = getenv("ENET_RC_VERIFY_BPC");     // (experiments: workgroups per CU)
    const uint32_t bpc = vb_env && atoi(vb_env) > 0 ? static_cast<uint32_t>(atoi(vb_env)) : kVerifyBlocksPerCu;
    const uint32_t cap = (ws->cus ? ws->cus : 256u) * bpc;
    hipLaunchKernelGGL(rc_dec6_verify, dim3(vb < cap ? vb : cap), dim3(256), 0, st, *b, *ws);
    return static_cast<int>(hipGetLastError());
}

extern "C" int rc_hip_dec6_launch(const rc_batch_dev* b, const rc_workspace_dev* ws, uint32_t blocks, void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (ws->lane_active != 64) return static_cast<int>(hipErrorInvalidValue);
    // (12 B more per lane than the model for the slot control words)
    // (+ root3_inc_init's table, 512 B; -DDEC6_RCP_TAB: the order-1 reciprocals, 2 KB)
#ifdef DEC6_RCP_TAB
    const size_t lds = static_cast<size_t>(kLanes6s) * (kLds6 + 12) + 512 + 2048;
#else
    const size_t lds = static_cast<size_t>(kLanes6s) * (kLds6 + 12) + 512;
#endif
    hipLaunchKernelGGL(rc_decompress_dec6s, dim3(blocks), dim3(512), lds, st, *b, *ws);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
    return rc_hip_dec6_verify_launch(b, ws, stream);
}
#endif  // RC_LANE_HOST_TEST
