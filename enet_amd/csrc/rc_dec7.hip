// rc_dec7.hip -- record-light range decoder with a serving wavefront per
// SIMD (compress.c:498-627), bit-exact.
//
// The model and the common step are rc_dec6.hip's (read its header first):
// per bucket one LDS byte (t1, r1) gives the order-1 context's escapes and
// total; a byte decoded at the root after escaping order 1 is new to that
// context, so the next position's order-2 context has never been visited.
// A step that needs a context's symbols -- order 1 holds the coded symbol, or
// the order-2 context exists -- stalls its lane.
//
// What differs is who serves a stalled lane, and from what.
//   * rc_dec6 runs one wavefront per SIMD.  Every byte it decodes is also
//     appended to its bucket's record in HBM (a blind 2-B store at a random
//     address: 78.6 M per C2 batch, at the memory system's random-access
//     rate), every 16th step the whole wavefront serves its ~9 stalled lanes
//     from those records (30 % of its cycles), and each record load waits
//     behind the stores (~5 us per round trip under that traffic).
//   * Here each workgroup has 4 main wavefronts (waves 0-3, one packet per
//     lane, the common steps) and 4 serving wavefronts (waves 4-7; wave w + 4
//     shares wave w's SIMD, and lane l serves lane l of its main wavefront:
//     its requests and its input).  A lone wavefront leaves about half of its
//     SIMD's issue cycles unused, and a partner takes them without slowing its
//     chain (tools/mb/issue2.hip).  Nothing is stored per byte: bucket p's
//     elements are the positions k of the decoded output with x[k-1] = p (a
//     = x[k-2], v = x[k]), and the serving wavefront rebuilds the bucket from
//     the output itself, all 64 lanes loading 16-B windows of the stalled
//     lane's output (one round trip, served by the L2: main wrote them
//     recently), each lane matching its windows against p, the matches
//     compacted one element per lane, and the context statistics then taken
//     as ballots (dec4's algebra, rc_dec4.hip, over the elements: order-1
//     members are the elements not decoded at order 2, order-2 members those
//     with a = x[j-2]).
//
// The wavefronts talk through LDS only, each word written by one side:
//   * the input slot (16 B per lane): the next aligned chunk of the lane's
//     compressed stream, loaded by the serving lane.  The main lane takes it
//     when its chunk is used up and asks for the one after; after the
//     packet's first two chunks it issues no global load at all;
//   * the mailbox (64 B per lane): a stalled lane posts its coder state and
//     its output tail -- the last window it stored and the one it is filling
//     (main waits for vmcnt(0) before each window store, so every window
//     before the last one stored is complete in memory, and the serving
//     wavefront reads those with L1-bypassing loads).  The answer: the coder
//     state after the step(s) (up to kChain7 symbols, while the next step
//     again has a visited order-2 context), the bytes consumed, the symbols.
//     A step whose sub-contexts all escaped comes back "root pending": the
//     main lane's next step decodes at the root, so the root model stays in
//     the main lane's registers and LDS;
//   * the control words: m_ctl (request count, wanted chunk, packet
//     generation) and m_pkt (the packet) from main, h_ctl (answer count, the
//     slot's chunk and generation) from the serving lane.
// The main step reads h_ctl and the slot at its top and acts on them at its
// end (answers, input), so the LDS round trip stays off the step's chain.
// The main wavefront waits only for the serving wavefront, which waits only
// for its own loads: no deadlock.
//
// The check (rc_dec6_verify) and the routing of packets off the fast path are
// rc_dec6's.  tests/proto/lane_host.cpp (variant v7) compiles the main side
// for the host with a scalar restatement of the serve (serve7_host), run
// after every main step and, at random, late.

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
#include "rc_dec6_rare.h"   // (hload16)

namespace {

constexpr uint32_t kLane7 = 528;      // per lane: root counts[256] | input slot (16 B) | bucket bytes[256]
constexpr uint32_t kSlot7 = 256;
constexpr uint32_t kStats7 = 272;
constexpr uint32_t kMbox7 = 22;       // mailbox dwords per lane
#ifndef DEC7_CHAIN
#define DEC7_CHAIN 3
#endif
constexpr uint32_t kChain7 = DEC7_CHAIN;   // symbols per answer at most (3: 24 bits of the answer)
constexpr uint32_t kRounds7 = 3;      // output windows per serving lane: 3 x 64 x 16 B (longer outputs leave)
constexpr uint32_t kCap7 = 24;        // order-1 elements per bucket on the fast path (as rc_dec6)
constexpr uint32_t kFin7 = 0xFFFFFFFFu;
constexpr uint32_t kNoPkt7 = 0xFFFFFFFEu;
constexpr uint32_t kWaveBail7 = 16;
constexpr uint32_t kLanes7 = 256;     // main lanes per workgroup
constexpr uint32_t kScr7 = 64;        // compaction slots per serving wavefront
#ifndef DEC7_SERVE
#define DEC7_SERVE 2
#endif
constexpr uint32_t kServe7 = DEC7_SERVE;   // requests per serving pass at most

__host__ __device__ constexpr uint32_t lds7_bytes(uint32_t lanes)
{
    return lanes * (kLane7 + 4 * kMbox7 + 8 + 4) + (lanes / 64) * 4 * kScr7;
}

struct Lds7 {
    uint8_t* lane;     // root | slot | bucket bytes
    uint32_t* mbox;
    uint32_t* mctl;    // [0] ctl, [1] packet (one 8-B word)
    uint32_t* hctl;
    uint32_t* scr;     // the serving wavefront's compaction slots
};

DEV Lds7 lds7(uint8_t* smem, uint32_t L, uint32_t lanes)
{
    Lds7 s;
    s.lane = smem + L * kLane7;
    uint8_t* q = smem + lanes * kLane7;
    s.mbox = reinterpret_cast<uint32_t*>(q) + L * kMbox7;
    q += lanes * kMbox7 * 4;
    s.mctl = reinterpret_cast<uint32_t*>(q) + L * 2;
    q += lanes * 8;
    s.hctl = reinterpret_cast<uint32_t*>(q) + L;
    q += lanes * 4;
    s.scr = reinterpret_cast<uint32_t*>(q) + (L / 64) * kScr7;
    return s;
}

// the same areas of another lane of the wavefront (lane r of the 64)
DEV Lds7 lds7_of(const Lds7& x, uint32_t mine, uint32_t r)
{
    Lds7 s = x;
    s.lane = x.lane + (static_cast<int>(r) - static_cast<int>(mine)) * static_cast<int>(kLane7);
    s.mbox = x.mbox + (static_cast<int>(r) - static_cast<int>(mine)) * static_cast<int>(kMbox7);
    s.mctl = x.mctl + (static_cast<int>(r) - static_cast<int>(mine)) * 2;
    s.hctl = x.hctl + (static_cast<int>(r) - static_cast<int>(mine));
    return s;
}

DEV uint32_t mctl_word(uint32_t req, uint32_t want, uint32_t gen)
{
    return ((req & 0xFFu) << 8) | ((want & 0xFFFu) << 16) | (gen << 28);
}

// ----------------------------------------------------------------- serving
// The serving lane's registers: its main lane's packet and hit list.
struct Help7 {
    uint32_t resp, have, hgen, cgen, pub;
    uint32_t len, cap;
    uintptr_t ib, ob;             // the packet's input and output
    uint32_t hl[4], nh;           // positions decoded at order 2 (they leave order 1 alone)
#ifdef RC_PROFILE
    unsigned long long ps, pt, pw, pc, pdd, pit;   // (diagnostic) requests, cycles serving, load waits, compaction, decode, chain iterations
#endif
};

DEV void help7_init(Help7& h)
{
    h.resp = 0; h.have = 0; h.hgen = 0; h.cgen = 0; h.pub = 0;
    h.len = 0; h.cap = 0; h.ib = 0; h.ob = 0;
    h.hl[0] = h.hl[1] = h.hl[2] = h.hl[3] = 0xFFFFu; h.nh = 0;
#ifdef RC_PROFILE
    h.ps = h.pt = h.pw = h.pc = h.pdd = h.pit = 0;
#endif
}

// A request as posted: coder state, model state, output tail.
struct Req7 {
    uint32_t low, code, range, p, a, x0, order, pos, on, nodes, claims;
    bool repeat;
    uint4 wpp, wp, w;             // the two output windows stored last; the one being filled
    uint32_t acc, ws, nb;         // its next dword (nb bytes), its filled dwords
    uint64_t la;                  // the stream's next na bytes
    uint32_t na;
};

// mailbox: [0-3] low, code, range, p | a | x0 | order | repeat; [4] pos | on;
// [5] nodes | claims; [6] acc; [7] ws | nb | na; [8-11] wpp; [12-15] wp;
// [16-19] w; [20-21] the stream lookahead (na bytes, the next in bits 63..56)
DEV Req7 req7_read(const uint32_t* mb)
{
    const uint4 q0 = *reinterpret_cast<const uint4*>(mb);
    const uint4 q1 = *reinterpret_cast<const uint4*>(mb + 4);
    Req7 r;
    r.low = q0.x; r.code = q0.y; r.range = q0.z;
    r.p = q0.w & 0xFFu; r.a = (q0.w >> 8) & 0xFFu; r.x0 = (q0.w >> 16) & 0xFFu; r.order = (q0.w >> 24) & 3u;
    r.repeat = ((q0.w >> 26) & 1u) != 0;
    r.pos = q1.x & 0xFFFFu; r.on = q1.x >> 16;
    r.nodes = q1.y & 0xFFFFu; r.claims = q1.y >> 16;
    r.acc = q1.z; r.ws = q1.w & 0xFFu; r.nb = (q1.w >> 8) & 0xFFu;
    r.wpp = *reinterpret_cast<const uint4*>(mb + 8);
    r.wp = *reinterpret_cast<const uint4*>(mb + 12);
    r.w = *reinterpret_cast<const uint4*>(mb + 16);
    const uint2 l2 = *reinterpret_cast<const uint2*>(mb + 20);
    r.la = static_cast<uint64_t>(l2.x) | (static_cast<uint64_t>(l2.y) << 32);
    r.na = (q1.w >> 16) & 0xFFu;
    return r;
}

// The answer: coder state, bytes consumed, symbols, model state.
DEV void ans7_write(uint32_t* mb, uint32_t low, uint32_t code, uint32_t range, uint32_t outb, uint32_t nout,
                    uint32_t used, uint32_t p, uint32_t a, uint32_t order, bool repeat, bool rootonly, bool lv,
                    bool fl, uint32_t nodes, uint32_t claims)
{
    *reinterpret_cast<uint4*>(mb) = make_uint4(low, code, range, outb | (nout << 24) | (min(used, 63u) << 26));
    *reinterpret_cast<uint2*>(mb + 4) =
        make_uint2(p | (a << 8) | (order << 16) | ((repeat ? 1u : 0u) << 18) | ((rootonly ? 1u : 0u) << 19) |
                       ((lv ? 1u : 0u) << 20) | ((fl ? 1u : 0u) << 21),
                   (nodes & 0xFFFFu) | (claims << 16));
}

// The serving side's stream: main's lookahead (the next na bytes), then --
// rarely, a chain reading past it -- single bytes from the packet (bytes past
// its end read as 0, compress.c:366-367).
struct SSrc {
    uint64_t la;
    uint32_t na, next, used, len;   // next: offset of the byte after la's; bytes taken
    uintptr_t ib;
};

DEV uint32_t ss_shift_in(SSrc& s, uint32_t code, uint32_t k)
{
    const uint32_t t = static_cast<uint32_t>(s.la >> 32);
    const uint32_t in = static_cast<uint32_t>((static_cast<uint64_t>(t) << (8 * k)) >> 32);
    s.la = k >= 8 ? 0ull : s.la << (8 * k);
    s.na -= k;
    s.used += k;
    return (code << (8 * k)) | in;
}

// (the lookahead empty: one more byte from the packet)
DEV void ss_need1(SSrc& s, bool en)
{
    if (rare_lane(en && s.na == 0)) {
        const bool e = en && s.na == 0;
        const uint32_t b = (e && s.next < s.len) ? *GPTRC(uint8_t, s.ib + s.next) : 0u;
        s.la = e ? static_cast<uint64_t>(b) << 56 : s.la;
        s.na += e ? 1u : 0u;
        s.next += e ? 1u : 0u;
    }
}

// compress.c:354-371 where `en` (rc_lane_common.h dec_code over SSrc)
DEV void sdec_code(uint32_t& low, uint32_t& code, uint32_t& range, uint32_t under, uint32_t count, SSrc& in, bool en)
{
    low = en ? low + under * range : low;
    range = en ? range * count : range;
    const uint32_t k = en ? settled_bytes(low, range) : 0u;
    const bool fast = k <= in.na;
    const uint32_t kk = fast ? k : 0u;
    code = ss_shift_in(in, code, kk);
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
            ss_need1(in, more);
            code = ss_shift_in(in, code, more ? 1u : 0u);
            range = more ? range << 8 : range;
            low = more ? low << 8 : low;
        } while (rare_lane(more));
    }
}

#ifndef RC_LANE_HOST_TEST
// ---- wavefront primitives for the serve (one request, all 64 lanes)
DEV uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
DEV uint32_t below64(uint64_t m)      // set bits of m below this lane
{
    return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
}
DEV uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
DEV uint32_t popc64(uint64_t m) { return static_cast<uint32_t>(__builtin_popcountll(m)); }
DEV uint32_t rdlane(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
DEV uint32_t prev_lane(uint32_t v) { return static_cast<uint32_t>(__shfl_up(static_cast<int>(v), 1)); }

// the lanes of `set` whose key is below mine (lt) and equal to mine (the mask)
DEV uint64_t rank8(uint32_t key, uint64_t set, uint32_t& lt)
{
    uint64_t e = set;
    lt = 0;
#pragma unroll
    for (int b = 7; b >= 0; --b) {
        const uint64_t bb = ballot(((key >> b) & 1u) != 0);
        const bool one = ((key >> b) & 1u) != 0;
        const uint64_t zeros = e & ~bb;
        lt += one ? popc64(zeros) : 0u;
        e = one ? (e & bb) : zeros;
    }
    return e;
}

// distinct keys among the lanes of `set`
DEV uint32_t distinct8(uint32_t key, uint64_t set)
{
    uint32_t lt;
    const uint64_t eq = rank8(key, set, lt);
    const uint64_t below = (1ull << lane_id()) - 1ull;
    return popc64(ballot(((set >> lane_id()) & 1ull) != 0 && (eq & below) == 0));
}

// bytes of dword-pair (hi, lo) shifted up by k bytes: the k bytes before each byte
DEV uint32_t shift_in(uint32_t cur, uint32_t prev, uint32_t k) { return align8(cur, prev, 4 - k); }

// one 16-B window: 0x01 in every byte equal to u, as a 16-bit mask
DEV uint32_t eqmask16(const uint4& w, uint32_t u)
{
    const uint32_t ur = u * 0x01010101u;
    return gather4(eq01(w.x, ur)) | (gather4(eq01(w.y, ur)) << 4) | (gather4(eq01(w.z, ur)) << 8) |
           (gather4(eq01(w.w, ur)) << 12);
}

DEV uint32_t byte_of(const uint4& w, uint32_t b) { return (pick4(b >> 2, w) >> (8 * (b & 3))) & 0xFFu; }

// A request being served: its lane's packet and the output windows (window
// m of the packet's aligned output in W[m >> 6] of lane m & 63).  Loaded by
// serve7_prep, used by serve7_run: the next request's loads are issued before
// the current one is computed.
struct Srv7 {
    uint32_t r, len, cap, lead, iw, nr;
    uintptr_t ib;
    uint4 W[kRounds7];
};

DEV void serve7_prep(const Lds7& x, uint32_t me, uint32_t r, const Help7& h, Srv7& s)
{
    const Lds7 xr = lds7_of(x, me, r);
    s.r = r;
    const uint32_t on = *(xr.mbox + 4) >> 16;
    const uint32_t wsnb = *(xr.mbox + 7);
    const uint32_t ws = wsnb & 0xFFu, nb = (wsnb >> 8) & 0xFFu;
    s.len = rdlane(h.len, r);
    s.cap = rdlane(h.cap, r);
    const uintptr_t ob = (static_cast<uintptr_t>(rdlane(static_cast<uint32_t>(h.ob >> 32), r)) << 32) |
                         rdlane(static_cast<uint32_t>(h.ob), r);
    s.ib = (static_cast<uintptr_t>(rdlane(static_cast<uint32_t>(h.ib >> 32), r)) << 32) |
           rdlane(static_cast<uint32_t>(h.ib), r);
    // the output so far: windows of 16 B from the aligned base; window iw is
    // being filled (w, then acc), windows iw - 1 and iw - 2 are the two stored
    // last (wp, wpp), the ones before them are complete in memory
    s.lead = static_cast<uint32_t>(ob & 15);
    const uintptr_t a0 = ob & ~static_cast<uintptr_t>(15);
    s.iw = (s.lead + on - 4 * ws - nb) >> 4;
    s.nr = min((s.iw >> 6) + 1, kRounds7);
    const uint32_t me64 = lane_id();
#pragma unroll
    for (uint32_t rr = 0; rr < kRounds7; ++rr) {
        const uint32_t m = 64 * rr + me64;
        uint4 t = make_uint4(0u, 0u, 0u, 0u);
        if (rr < s.nr && m + 2 < s.iw) t = hload16(a0 + 16 * static_cast<uintptr_t>(m));
        s.W[rr] = t;
    }
}

// (x[k-2], x[k-1]) of each byte k of a window: its dwords shifted up by 2 and 1
// bytes, the bytes before it from pd (dword 3 of the window before)
DEV void win_shift(const uint4& w, uint32_t pd, uint4& s1, uint4& s2)
{
    s1 = make_uint4(shift_in(w.x, pd, 1), shift_in(w.y, w.x, 1), shift_in(w.z, w.y, 1), shift_in(w.w, w.z, 1));
    s2 = make_uint4(shift_in(w.x, pd, 2), shift_in(w.y, w.x, 2), shift_in(w.z, w.y, 2), shift_in(w.w, w.z, 2));
}

// the positions 1 <= k < on among the 16 bytes of a window (byte 0 at position base)
DEV uint32_t win_valid(int base, uint32_t on)
{
    const int lo_b = 1 - base, hi_b = static_cast<int>(on) - base;
    const uint32_t vlo = lo_b <= 0 ? 0xFFFFu : (lo_b >= 16 ? 0u : (0xFFFFu << lo_b) & 0xFFFFu);
    const uint32_t vhi = hi_b >= 16 ? 0xFFFFu : (hi_b <= 0 ? 0u : (1u << hi_b) - 1u);
    return vlo & vhi;
}

// sum over the wavefront of a per-lane count c <= 16
DEV uint32_t wave_sum16(uint32_t c)
{
    if (!any_lane(c > 1)) return popc64(ballot(c != 0));
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t b = 0; b < 5; ++b) sum += popc64(ballot(((c >> b) & 1u) != 0)) << b;
    return sum;
}

// t2: the visits of order-2 context (a, p), i.e. the positions 2 <= k < on with
// (x[k-2], x[k-1]) = (a, p) -- a pair match, no element list needed
DEV uint32_t pair_count7(const uint4* W, uint32_t nr, uint32_t lead, uint32_t on, uint32_t a, uint32_t p)
{
    const uint32_t me64 = lane_id();
    uint32_t c = 0;
#pragma unroll
    for (uint32_t rr = 0; rr < kRounds7; ++rr) {
        if (rr >= nr) break;
        const uint4 w = W[rr];
        uint32_t pd = prev_lane(w.w);
        const uint32_t carry = rr > 0 ? rdlane(W[rr - 1].w, 63) : 0u;
        pd = me64 == 0 ? carry : pd;
        uint4 s1, s2;
        win_shift(w, pd, s1, s2);
        const int base = static_cast<int>(16 * (64 * rr + me64)) - static_cast<int>(lead);
        const int k2 = 2 - base;                                 // byte of position 2
        const uint32_t M = eqmask16(s1, p) & eqmask16(s2, a) & win_valid(base, on) &
                           (k2 <= 0 ? 0xFFFFu : (k2 >= 16 ? 0u : (0xFFFFu << k2) & 0xFFFFu));
        c += static_cast<uint32_t>(__builtin_popcount(M));
    }
    return wave_sum16(c);
}

// bucket p's elements, one per lane (lanes < the count): v | a << 8 | (k >= 2)
// << 16 | (decoded at order 2) << 17.  Returns the count (> kScr7: too many).
DEV uint32_t compact7(const Lds7& x, const uint4* W, uint32_t nr, uint32_t lead, uint32_t on, uint32_t p,
                      const uint32_t* hp, uint32_t& e)
{
    const uint32_t me64 = lane_id();
    uint32_t total = 0;
#pragma unroll
    for (uint32_t rr = 0; rr < kRounds7; ++rr) {
        if (rr >= nr) break;
        const uint4 w = W[rr];
        uint32_t pd = prev_lane(w.w);
        const uint32_t carry = rr > 0 ? rdlane(W[rr - 1].w, 63) : 0u;
        pd = me64 == 0 ? carry : pd;
        uint4 s1, s2;
        win_shift(w, pd, s1, s2);
        const int base = static_cast<int>(16 * (64 * rr + me64)) - static_cast<int>(lead);
        const uint32_t M = eqmask16(s1, p) & win_valid(base, on);
        const uint32_t c = static_cast<uint32_t>(__builtin_popcount(M));
        uint32_t pre, sum;
        if (!any_lane(c > 1)) {
            const uint64_t bb = ballot(c != 0);
            pre = below64(bb);
            sum = popc64(bb);
        } else {
            pre = 0; sum = 0;
#pragma unroll
            for (uint32_t b = 0; b < 5; ++b) {
                const uint64_t bb = ballot(((c >> b) & 1u) != 0);
                pre += below64(bb) << b;
                sum += popc64(bb) << b;
            }
        }
        if (sum) {
            uint32_t rem = M, sl = total + pre;
            while (any_lane(rem != 0)) {
                const uint32_t b = rem ? static_cast<uint32_t>(__builtin_ctz(rem)) : 0u;
                const uint32_t k = static_cast<uint32_t>(base + static_cast<int>(b));
                const bool hit = k == hp[0] || k == hp[1] || k == hp[2] || k == hp[3];
                const uint32_t el = byte_of(w, b) | (byte_of(s2, b) << 8) | ((k >= 2 ? 1u : 0u) << 16) |
                                    ((hit ? 1u : 0u) << 17);
                if (rem && sl < kScr7) x.scr[sl] = el;
                sl += rem ? 1u : 0u;
                rem &= rem ? rem - 1u : 0u;
            }
        }
        total += sum;
    }
    e = me64 < total && total <= kScr7 ? x.scr[me64] : 0u;
    return total;
}

// READ in a sub-context of t visits and d symbols (compress.c:536-568): an
// escape is coded here; otherwise the code's offset c into the symbols
DEV bool wread7(uint32_t t, uint32_t d, uint32_t& low, uint32_t& code, uint32_t& range, SSrc& in, uint32_t& c,
                bool& fail)
{
    const uint32_t esc = kSubEscDelta * d, tot = esc + kSubDelta * t;
    const uint32_t r1 = udiv16d(range, tot, rcp64(tot));
    const uint32_t cd = udiv_lo16(code - low, r1);
    range = r1;
    const bool e = cd < esc;
    sdec_code(low, code, range, 0u, esc, in, e);
    c = cd - esc;
    fail = fail || (!e && c >= kSubDelta * t);
    return !e && c < kSubDelta * t;
}

// the symbol whose interval holds offset c among the lanes g (values V), in value order
DEV void wselect7(uint64_t g, uint32_t t, uint32_t d, uint32_t V, uint32_t c, uint32_t esc, uint32_t& v,
                  uint32_t& under, uint32_t& count)
{
    if (d == 1) {
        const uint32_t f = static_cast<uint32_t>(__builtin_ctzll(g | (1ull << 63)));
        v = rdlane(V, f);
        under = esc;
        count = kSubDelta * t;
        return;
    }
    uint32_t lt;
    const uint64_t eq = rank8(V, g, lt);
    const uint32_t ne = popc64(eq);
    const uint64_t pick = ballot(((g >> lane_id()) & 1ull) != 0 && kSubDelta * lt <= c && c < kSubDelta * (lt + ne));
    const uint32_t f = static_cast<uint32_t>(__builtin_ctzll(pick | (1ull << 63)));
    v = rdlane(V, f);
    under = esc + kSubDelta * rdlane(lt, f);
    count = kSubDelta * rdlane(ne, f);
}

DEV void serve7_run(const Lds7& x, uint32_t me, Help7& h, Srv7& s)
{
    const uint32_t r = s.r;
    const Lds7 xr = lds7_of(x, me, r);
    const Req7 q = req7_read(xr.mbox);
    uint8_t* stats = xr.lane + kStats7;
    const uint32_t lead = s.lead, iw = s.iw, nr = s.nr, cap = s.cap;
    uint32_t hp[4];
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) hp[k] = rdlane(h.hl[k], r);
    uint32_t nh = rdlane(h.nh, r);
    const uint32_t me64 = lane_id();
    uint4 W[kRounds7];
    {
        uint4 wm = q.w;
        wm.x = q.ws == 0 ? q.acc : wm.x; wm.y = q.ws == 1 ? q.acc : wm.y;
        wm.z = q.ws == 2 ? q.acc : wm.z; wm.w = q.ws == 3 ? q.acc : wm.w;
#pragma unroll
        for (uint32_t rr = 0; rr < kRounds7; ++rr) {
            const uint32_t m = 64 * rr + me64;
            const bool p2 = m + 2 == iw, p1 = m + 1 == iw, p0 = m == iw;
            W[rr].x = p2 ? q.wpp.x : (p1 ? q.wp.x : (p0 ? wm.x : s.W[rr].x));
            W[rr].y = p2 ? q.wpp.y : (p1 ? q.wp.y : (p0 ? wm.y : s.W[rr].y));
            W[rr].z = p2 ? q.wpp.z : (p1 ? q.wp.z : (p0 ? wm.z : s.W[rr].z));
            W[rr].w = p2 ? q.wpp.w : (p1 ? q.wp.w : (p0 ? wm.w : s.W[rr].w));
        }
    }
    SSrc in;
    in.la = q.la; in.na = q.na; in.used = 0; in.len = s.len; in.ib = s.ib;
    in.next = q.pos + q.na;
    uint32_t low = q.low, code = q.code, range = q.range;
    uint32_t p = q.p, a = q.a, order = q.order, on = q.on, nodes = q.nodes, claims = q.claims;
    bool repeat = q.repeat;
    uint32_t outb = 0, nout = 0;
    bool lv = iw + 1 >= 64 * kRounds7, fl = false, rootonly = false;
    bool act = !lv;
    for (uint32_t it = 0; it < kChain7 && act; ++it) {
        const uint32_t st = order >= 1 ? stats[p] : 0u;
        const uint32_t t1 = st & 31u, d1 = t1 - (st >> 5);
        // bucket p's elements, compacted only when a symbol must be found or counted
        bool have = false, sf = false;
        uint32_t e = 0, V = 0;
        uint64_t g1 = 0, g2 = 0;
        uint32_t ne = 0;
        auto elements = [&]() {
            if (have) return;
            have = true;
            ne = compact7(x, W, nr, lead, on, p, hp, e);
            const bool el = me64 < ne;
            V = e & 0xFFu;
            const uint32_t A = (e >> 8) & 0xFFu;
            const bool o2 = ((e >> 16) & 1u) != 0, hit = ((e >> 17) & 1u) != 0;
            g1 = ballot(el && !hit);
            g2 = order >= 2 ? ballot(el && o2 && A == a) : 0ull;
            sf = sf || ne > kScr7 || popc64(g1) != t1;   // (the history disagrees with the counts: leave)
        };
        const uint32_t t2 = order >= 2 ? pair_count7(W, nr, lead, on, a, p) : 0u;
        uint32_t d2 = t2;
        if (t2 > 1) { elements(); d2 = distinct8(V, g2); }
        int at = -1;
        uint32_t v = 0, hu = 0, hc = 0, c = 0;
        if (!sf && t2 > 0 && wread7(t2, d2, low, code, range, in, c, sf)) {
            elements();
            if (!sf) { wselect7(g2, t2, d2, V, c, kSubEscDelta * d2, v, hu, hc); at = 2; }
        }
        if (!sf && at < 0 && order >= 1 && t1 > 0 && wread7(t1, d1, low, code, range, in, c, sf)) {
            elements();
            if (!sf) { wselect7(g1, t1, d1, V, c, kSubEscDelta * d1, v, hu, hc); at = 1; }
        }
        const bool sym = !sf && at > 0;
        sdec_code(low, code, range, hu, hc, in, sym);
        // every sub-context escaped: the root's code is the main lane's (its next step)
        rootonly = !sf && at < 0;
        // the element joins its contexts (compress.c:598-615; a hit has its element list)
        const uint64_t eqv = sym ? ballot(me64 < ne && V == v) : 0ull;
        const bool n2 = order >= 2 && (eqv & g2) == 0;
        const bool n1 = order >= 1 && at != 2 && (eqv & g1) == 0;
        const bool nb = eqv == 0;
        nodes += sym ? (n2 ? 1u : 0u) + (n1 ? 1u : 0u) : 0u;
        const bool o1v = sym && order >= 1 && at != 2;
        if (o1v && me64 == 0) stats[p] = static_cast<uint8_t>(st + 1 + (n1 ? 0u : 32u));
        const bool tfull = o1v && t1 >= kCap7;
        claims += (sym && order >= 1 && nb && on < cap) ? 1u : 0u;
        const bool h2 = sym && at == 2;
        const bool hfull = h2 && nh >= 4;
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            hp[k] = (h2 && nh == k) ? on : hp[k];
            h.hl[k] = (h2 && nh == k && me64 == r) ? on : h.hl[k];
        }
        nh += h2 ? 1u : 0u;
        const bool f = sym && on >= cap;
        const bool l = sf || hfull || tfull || (o1v && !n1 && (st >> 5) >= 7) || (sym && nodes >= kMaxNodes);
        lv = lv || l;
        fl = fl || f;
        const bool put = sym && !l && !f;
        if (put) {
            // the symbol joins the output held here: byte `on` of the windows
            const uint32_t bpos = lead + on, mo = bpos >> 4, bo = bpos & 15;
            const uint32_t sh = 8 * (bo & 3), mk = ~(0xFFu << sh), vv = v << sh;
#pragma unroll
            for (uint32_t rr = 0; rr < kRounds7; ++rr) {
                if (rr != (mo >> 6)) continue;
                const bool here = (mo & 63) == me64;
                W[rr].x = here && (bo >> 2) == 0 ? (W[rr].x & mk) | vv : W[rr].x;
                W[rr].y = here && (bo >> 2) == 1 ? (W[rr].y & mk) | vv : W[rr].y;
                W[rr].z = here && (bo >> 2) == 2 ? (W[rr].z & mk) | vv : W[rr].z;
                W[rr].w = here && (bo >> 2) == 3 ? (W[rr].w & mk) | vv : W[rr].w;
            }
            outb |= v << (8 * nout);
            nout += 1;
            on += 1;
        }
        a = sym ? p : a;
        p = sym ? v : p;
        order += (sym && order < 2) ? 1u : 0u;
        repeat = sym ? !nb : repeat;
        // the step after a hit with a visited order-2 context is rare again
        act = put && order >= 2 && repeat && on + lead + 1 < 16 * 64 * nr;
    }
    h.nh = me64 == r ? nh : h.nh;
    if (me64 == 0) ans7_write(xr.mbox, low, code, range, outb, nout, in.used, p, a, order, repeat, rootonly, lv, fl, nodes, claims);
}
#endif  // !RC_LANE_HOST_TEST

#ifdef RC_LANE_HOST_TEST
// The serve restated for one lane on the host (test only): the same request
// and answer, the bucket rebuilt from the output bytes by plain loops.
DEV bool hsub7(const uint32_t* Vs, const bool* in_g, uint32_t n, uint32_t t, uint32_t d, bool en, uint32_t& low,
               uint32_t& code, uint32_t& range, SSrc& in, uint32_t& v, uint32_t& under, uint32_t& count,
               bool& fail)
{
    const uint32_t esc = kSubEscDelta * d, tot = en ? esc + kSubDelta * t : 1u;
    const uint32_t r1 = range / tot;
    const uint32_t cd = ((code - low) / r1) & 0xFFFF;
    range = en ? r1 : range;
    const bool e = en && cd < esc;
    sdec_code(low, code, range, 0u, esc, in, e);
    const bool hit = en && !e;
    fail = fail || (hit && cd - esc >= kSubDelta * t);
    const bool sel = hit && cd - esc < kSubDelta * t;
    if (sel) {
        // the symbol whose cumulative interval holds cd - esc, in value order
        uint32_t cnt[256] = {0};
        for (uint32_t i = 0; i < n; ++i) if (in_g[i]) cnt[Vs[i]]++;
        uint32_t acc = 0;
        for (uint32_t u = 0; u < 256; ++u) {
            if (cnt[u] && cd - esc < kSubDelta * (acc + cnt[u])) { v = u; under = esc + kSubDelta * acc; count = kSubDelta * cnt[u]; break; }
            acc += cnt[u];
        }
    }
    return sel;
}

DEV void serve7_host(const Lds7& x, Help7& h)
{
    const Req7 q = req7_read(x.mbox);
    uint8_t* stats = x.lane + kStats7;
    const uint32_t lead = static_cast<uint32_t>(h.ob & 15);
    const uintptr_t a0 = h.ob & ~static_cast<uintptr_t>(15);
    const uint32_t iw = (lead + q.on - 4 * q.ws - q.nb) >> 4;
    // the output bytes as the serving wavefront sees them
    static uint8_t X[16 * 64 * kRounds7 + 16];
    memset(X, 0, sizeof X);
    for (uint32_t m = 0; m <= iw && m < 64 * kRounds7; ++m) {
        uint4 w = make_uint4(0u, 0u, 0u, 0u);
        if (m + 2 < iw) {
            // (the caller's bytes: only the packet's own positions)
            for (uint32_t b = 0; b < 16; ++b) {
                const uintptr_t ad = a0 + 16 * m + b;
                if (ad >= h.ob) X[16 * m + b] = *reinterpret_cast<const uint8_t*>(ad);
            }
            continue;
        }
        if (m + 2 == iw) w = q.wpp;
        else if (m + 1 == iw) w = q.wp;
        else {
            w = q.w;
            w.x = q.ws == 0 ? q.acc : w.x; w.y = q.ws == 1 ? q.acc : w.y; w.z = q.ws == 2 ? q.acc : w.z; w.w = q.ws == 3 ? q.acc : w.w;
        }
        memcpy(X + 16 * m, &w, 16);
    }
    SSrc in;
    in.la = q.la; in.na = q.na; in.used = 0; in.len = h.len; in.ib = h.ib;
    in.next = q.pos + q.na;
    uint32_t low = q.low, code = q.code, range = q.range;
    uint32_t p = q.p, a = q.a, order = q.order, on = q.on, nodes = q.nodes, claims = q.claims;
    bool repeat = q.repeat;
    uint32_t outb = 0, nout = 0;
    bool lv = iw + 1 >= 64 * kRounds7, fl = false, rootonly = false;
    bool act = !lv;
    for (uint32_t it = 0; it < kChain7 && act; ++it) {
        uint32_t Vs[64], n = 0;
        bool g1[64], g2[64], ok = true;
        for (uint32_t k = 1; k < on; ++k) {
            if (X[lead + k - 1] != p) continue;
            if (n == 64) { ok = false; break; }
            const bool hit = k == h.hl[0] || k == h.hl[1] || k == h.hl[2] || k == h.hl[3];
            Vs[n] = X[lead + k];
            g1[n] = !hit;
            g2[n] = order >= 2 && k >= 2 && X[lead + k - 2] == a;
            ++n;
        }
        const uint32_t st = order >= 1 ? stats[p] : 0u;
        const uint32_t t1 = st & 31u, d1 = t1 - (st >> 5);
        uint32_t c1n = 0, t2 = 0, d2 = 0;
        bool seen[256] = {false};
        for (uint32_t i = 0; i < n; ++i) {
            c1n += g1[i] ? 1u : 0u;
            if (g2[i]) { ++t2; if (!seen[Vs[i]]) { seen[Vs[i]] = true; ++d2; } }
        }
        int at = -1;
        uint32_t v = 0, hu = 0, hc = 0;
        bool sf = !ok || c1n != t1;
        const bool c2 = !sf && order >= 2 && t2 > 0;
        if (c2 && hsub7(Vs, g2, n, t2, d2, c2, low, code, range, in, v, hu, hc, sf)) at = 2;
        const bool c1 = !sf && at < 0 && order >= 1 && t1 > 0;
        if (c1 && hsub7(Vs, g1, n, t1, d1, c1, low, code, range, in, v, hu, hc, sf)) at = 1;
        const bool sym = !sf && at > 0;
        sdec_code(low, code, range, hu, hc, in, sym);
        rootonly = !sf && at < 0;
        bool inall = false, in1 = false, in2 = false;
        for (uint32_t i = 0; i < n; ++i)
            if (Vs[i] == v) { inall = true; in1 = in1 || g1[i]; in2 = in2 || g2[i]; }
        const bool n2 = order >= 2 && !in2;
        const bool n1 = order >= 1 && at != 2 && !in1;
        const bool nb = !inall;
        nodes += sym ? (n2 ? 1u : 0u) + (n1 ? 1u : 0u) : 0u;
        const bool o1v = sym && order >= 1 && at != 2;
        if (o1v) stats[p] = static_cast<uint8_t>(st + 1 + (n1 ? 0u : 32u));
        const bool tfull = o1v && t1 >= kCap7;
        claims += (sym && order >= 1 && nb && on < h.cap) ? 1u : 0u;
        const bool h2 = sym && at == 2;
        const bool hfull = h2 && h.nh >= 4;
        if (h2 && h.nh < 4) h.hl[h.nh] = on;
        h.nh += h2 ? 1u : 0u;
        const bool f = sym && on >= h.cap;
        const bool l = sf || hfull || tfull || (o1v && !n1 && (st >> 5) >= 7) || (sym && nodes >= kMaxNodes);
        lv = lv || l;
        fl = fl || f;
        const bool put = sym && !l && !f;
        if (put) { X[lead + on] = static_cast<uint8_t>(v); outb |= v << (8 * nout); nout += 1; on += 1; }
        a = sym ? p : a;
        p = sym ? v : p;
        order += (sym && order < 2) ? 1u : 0u;
        repeat = sym ? !nb : repeat;
        act = put && order >= 2 && repeat && on + lead + 1 < 16 * 64 * kRounds7;
    }
    ans7_write(x.mbox, low, code, range, outb, nout, in.used, p, a, order, repeat, rootonly, lv, fl, nodes, claims);
}
#endif

// h_ctl: answer count, the slot's chunk and generation
DEV void help7_publish(const Lds7& x, Help7& h)
{
    const uint32_t hc = (h.resp << 8) | (h.have << 16) | (h.hgen << 28);
    if (hc != h.pub) {
        __builtin_amdgcn_s_waitcnt(0xC07F);      // lgkmcnt(0): slots and answers written before the word that announces them
        *x.hctl = hc;
        h.pub = hc;
    }
}

// One pass of the serving wavefront over its 64 lanes: new packets, input
// chunks, requests (one at a time, each with the whole wavefront); publishes
// h_ctl.  Returns whether it did anything; fin_all: every main lane is done.
DEV bool help7_iter(const rc_batch_dev& bt, const Lds7& x, Help7& h, bool& fin_all)
{
    const uint2 m = *reinterpret_cast<const uint2*>(x.mctl);
    const uint32_t mc = m.x, mp = m.y;
    const bool fin = mp == kFin7;
    const uint32_t req = (mc >> 8) & 0xFFu, want = (mc >> 16) & 0xFFFu, mgen = mc >> 28;
    bool busy = false;
    // a new packet: its input, output and capacity, no order-2 hits yet
    const bool np = !fin && mp != kNoPkt7 && mgen != h.cgen;
    if (any_lane(np)) {
        if (np) {
            h.len = bt.in_len[mp];
            h.ib = reinterpret_cast<uintptr_t>(bt.in + bt.in_off[mp]);
            h.ob = reinterpret_cast<uintptr_t>(bt.out + bt.out_off[mp]);
            h.cap = bt.out_cap[mp];
            h.hl[0] = h.hl[1] = h.hl[2] = h.hl[3] = 0xFFFFu;
            h.nh = 0;
            h.cgen = mgen;
        }
    }
    // the next input chunk the main lane wants (issued first: its round trip
    // overlaps the requests')
    const bool inq = !fin && h.cgen != 0 && mgen == h.cgen && (want != h.have || h.hgen != h.cgen);
    uint4 c = make_uint4(0u, 0u, 0u, 0u);
    if (any_lane(inq)) {
        busy = true;
        const uintptr_t base = h.ib & ~static_cast<uintptr_t>(15);
        c = chunk_load(h.ib, h.ib + h.len, base + 16 * static_cast<uintptr_t>(want), inq);
    }
    // the chunk into the slot and announced before any request is served: a
    // main lane whose lookahead runs dry stops its whole wavefront
    if (inq) *reinterpret_cast<uint4*>(x.lane + kSlot7) = c;
    h.have = inq ? want : h.have;
    h.hgen = inq ? h.cgen : h.hgen;
    help7_publish(x, h);
    const bool rq = !fin && req != h.resp;
#ifndef RC_LANE_HOST_TEST
    uint64_t todo = ballot(rq);
    // (at most kServe7 requests per pass: the next pass refills slots first)
    {
        uint64_t cap = todo;
        for (uint32_t k = 0; k < kServe7 && cap; ++k) cap &= cap - 1;
        todo &= ~cap;
    }
    if (todo) {
        busy = true;
        const uint32_t me = lane_id();
#ifdef RC_PROFILE
        const unsigned long long t0 = prof_now();
        h.ps += popc64(todo);
#endif
        const uint64_t served = todo;
        Srv7 cur, nxt;
        serve7_prep(x, me, static_cast<uint32_t>(__builtin_ctzll(todo)), h, nxt);
        todo &= todo - 1;
        for (;;) {
            cur = nxt;
            // the next request's loads in flight while this one is computed
            if (todo) {
                serve7_prep(x, me, static_cast<uint32_t>(__builtin_ctzll(todo)), h, nxt);
                todo &= todo - 1;
                serve7_run(x, me, h, cur);
                continue;
            }
            serve7_run(x, me, h, cur);
            break;
        }
        h.resp = ((served >> me) & 1ull) ? req : h.resp;
#ifdef RC_PROFILE
        h.pt += prof_now() - t0;
#endif
    }
#else
    if (rq) { busy = true; serve7_host(x, h); }
    h.resp = rq ? req : h.resp;
#endif
    help7_publish(x, h);
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
    uint32_t req, want, gen;
};

DEV uint64_t shl8(uint64_t x, uint32_t k) { return k >= 8 ? 0ull : x << (8 * k); }

DEV void mpublish(const Lds7& x, const Main7& m)
{
    x.mctl[0] = mctl_word(m.req, m.want, m.gen);
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
// from the slot once the serving lane has put the next chunk there
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

// skip k bytes the serving lane consumed
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

// The window completed by the last step, stored once every store of the
// wavefront but the latest is complete (vmcnt(1): main issues no loads in its
// loop, so this waits only for window stores issued at least a step ago).  A
// lane's windows are stored one store instruction apart at least, so every
// window before the two it stored last (kept in wl2, wl for its requests) is
// in memory for the serving lanes.
DEV void mflush(ByteSink& o, uint4& wl, uint4& wl2)
{
    if (any_lane(o.pend)) {
#if !defined(RC_LANE_HOST_TEST) && !defined(DEC7_NOWAIT)
        __builtin_amdgcn_s_waitcnt(0x0F71);     // vmcnt(1)
#endif
        // (component selects: a select of uint4 references becomes a select of
        // addresses, and the sink then lives in scratch memory)
        const bool pd = o.pend;
        wl2.x = pd ? wl.x : wl2.x; wl2.y = pd ? wl.y : wl2.y; wl2.z = pd ? wl.z : wl2.z; wl2.w = pd ? wl.w : wl2.w;
        wl.x = pd ? o.wp.x : wl.x; wl.y = pd ? o.wp.y : wl.y; wl.z = pd ? o.wp.z : wl.z; wl.w = pd ? o.wp.w : wl.w;
        sink_flush(o);
    }
}

DEV void main7_packet(const rc_batch_dev& bt, const rc_workspace_dev& ws, uint32_t pkt, const Lds7& x, Main7& m)
{
    const uint32_t len = bt.in_len[pkt];
    const uint32_t cap = bt.out_cap[pkt];
    if (len == 0) { bt.out_len[pkt] = 0; ws.claims[pkt] = 0; ws.dec6_resets[pkt] = 0; return; }     // compress.c:513
    uint8_t* root = x.lane;
    uint8_t* stats = x.lane + kStats7;
    // a new packet: generation, first wanted chunk (published once the stream is set up)
    m.gen = m.gen % 15u + 1u;
    ByteSink o;
    sink_init(o, bt.out + bt.out_off[pkt], cap);
    MSrc in;
    uint32_t code = msrc_init(in, bt.in + bt.in_off[pkt], len);
    m.want = in.j + 1;
    *reinterpret_cast<uint2*>(x.mctl) = make_uint2(mctl_word(m.req, m.want, m.gen), pkt);
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
    uint4 wl = make_uint4(0u, 0u, 0u, 0u), wl2 = wl;   // the two windows stored last

    PROF_DECL
    for (;;) {
        // ------------------------------------------------------------ top
        // (the control word and the slot are used at the end of the step:
        // their LDS round trip stays off the step's chain)
        const uint32_t hc = *x.hctl;
        const uint4 sl = *reinterpret_cast<const uint4*>(x.lane + kSlot7);
        const uint32_t stp = stats[p];
        mflush(o, wl, wl2);
        const bool go = !done && !stall;
        const uint32_t st = (go && order >= 1) ? stp : 0u;
        const uint32_t t1 = st & 31u, d1 = t1 - (st >> 5);
        bool need = go && !rootonly && order >= 2 && repeat;
        // order 1 (compress.c:536-568): an escape is coded here, a hit goes to the serving lane
        const bool o1 = go && !rootonly && !need && order >= 1 && t1 > 0;
        const uint32_t esc1 = kSubEscDelta * d1, tot1 = o1 ? esc1 + kSubDelta * t1 : 1u;
        const uint32_t r1 = udiv16d(range, tot1, rcp64(tot1));
        const bool e1 = o1 && code - low < esc1 * r1;
        need = need || (o1 && !e1);
        if (any_lane(need)) {
            // the request: the coder state at the top of this step, the output tail
            if (need) {
                uint32_t* mb = x.mbox;
                *reinterpret_cast<uint4*>(mb) =
                    make_uint4(low, code, range, p | (a << 8) | (x0 << 16) | (order << 24) | ((repeat ? 1u : 0u) << 26));
                *reinterpret_cast<uint4*>(mb + 4) =
                    make_uint4((mpos(in) & 0xFFFFu) | (o.n << 16), (nodes & 0xFFFFu) | (claims << 16),
                               static_cast<uint32_t>(o.acc), o.ws | (o.nb << 8) | (in.na << 16));
                *reinterpret_cast<uint2*>(mb + 20) =
                    make_uint2(static_cast<uint32_t>(in.la), static_cast<uint32_t>(in.la >> 32));
                *reinterpret_cast<uint4*>(mb + 8) = wl2;
                *reinterpret_cast<uint4*>(mb + 12) = wl;
                *reinterpret_cast<uint4*>(mb + 16) = o.w;
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
        const bool full = o1v && t1 >= kCap7;
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
        // answers: the serving lane's coder state, bytes and symbols
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
    ws.dec6_resets[pkt] = 0;                          // (one model segment: rc_dec6_verify's layout)
}

}  // namespace

#ifndef RC_LANE_HOST_TEST
// 4 main and 4 serving wavefronts per workgroup (waves w and w + 4 share a
// SIMD), one workgroup per CU (its LDS)
extern "C" __global__ __launch_bounds__(512) void rc_decompress_dec7(rc_batch_dev b, rc_workspace_dev ws)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t wave = threadIdx.x >> 6, l = threadIdx.x & 63;
    const bool serving = wave >= 4;
    const uint32_t L = (wave & 3) * 64 + l;
    const Lds7 x = lds7(smem, L, kLanes7);
    const uint32_t slot = blockIdx.x * kLanes7 + L;
    if (!serving) *reinterpret_cast<uint2*>(x.mctl) = make_uint2(0u, slot < b.n ? kNoPkt7 : kFin7);
    else *x.hctl = 0u;
    __syncthreads();
    if (serving) {
        Help7 h;
        help7_init(h);
#ifdef RC_PROFILE
        unsigned long long it = 0, idle = 0, t0 = prof_now();
#endif
        for (;;) {
            bool fin = false;
            const bool busy = help7_iter(b, x, h, fin);
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
            atomicAdd(&g_prof[38], h.pw);
            atomicAdd(&g_prof[39], h.pc);
            atomicAdd(&g_prof[40], h.pdd);
            atomicAdd(&g_prof[41], h.pit);
        }
#endif
        return;
    }
#ifdef DEC7_PRIO
    __builtin_amdgcn_s_setprio(DEC7_PRIO);
#endif
    const uint32_t* order = ws.order && !ws.bins[RC_LEN_BINS] ? ws.order : nullptr;
    Main7 m = {0u, 0u, 0u};
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
    hipLaunchKernelGGL(rc_decompress_dec7, dim3(blocks), dim3(512), lds7_bytes(kLanes7), st, *b, *ws);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return static_cast<int>(e);
    return rc_hip_dec6_verify_launch(b, ws, stream);
}
#endif  // RC_LANE_HOST_TEST
