// rc_slot.h -- a decoder lane's compressed stream through LDS, refilled by a
// helper wavefront on the same SIMD (rc_dec6.hip's rc_decompress_dec6s).
//
// rc_lane_common.h's ByteSrc reloads the next 16-B chunk of the stream with a
// global load every step, and the step after waits for it: vmcnt retires
// loads and stores in order, so the reload waits behind the step's record and
// output stores (rc_dec6: 0.78 k of 5.5 k cycles per packet-step).  Here the
// lane's next chunk sits in a 16-B LDS slot, put there by lane l of a helper
// wavefront (wave w + 4 of the workgroup, which shares wave w's SIMD and
// otherwise sleeps): the decoding lane takes it when its current chunk is used
// up and asks for the one after.  Past the packet's first two chunks the
// decoding wavefront issues no global load for its input at all.
//
// Words (each written by one side only):
//   m_ctl = wanted chunk (12 bits) << 16 | packet generation (16 bits),
//   m_pkt = the packet (kNoPktS before the first, kFinS when the lane is done),
//   h_ctl = the slot's chunk << 16 | its generation.
// The decoding side waits only for the helper, the helper only for its own
// loads: no deadlock.
//
// Ordering.  The helper stores the slot, then h_ctl with a workgroup-scope
// release (the slot's LDS write has completed before h_ctl is written).  The
// decoder reads h_ctl, then the slot, with a compiler barrier between the two
// reads (slot_read), so they issue in that order; a wavefront's LDS operations
// are performed in issue order, so a slot read that follows an h_ctl read
// which saw chunk j sees chunk j (or a later one, which the chunk index in
// h_ctl then does not announce yet: the decoder only takes a slot whose
// announced chunk is the one it wants).  No wait is put on the decoder's step
// (an acquire load would add an LDS round trip to every step).
// A 16-bit generation per lane -- wrapping only after 65535 packets on one lane
// -- and the packet index (m_pkt) both mark a new packet for the helper, which
// then forgets the chunk it holds.
#pragma once

namespace {

constexpr uint32_t kFinS = 0xFFFFFFFFu;
constexpr uint32_t kNoPktS = 0xFFFFFFFEu;

#ifndef RC_LANE_HOST_TEST
#define SLOT_IDLE() __builtin_amdgcn_s_sleep(1)
#define SLOT_POINT() ((void) 0)
#define SLOT_TAKEN(s, sl) ((void) 0)
#else
// tests/proto/lane_host.cpp: one helper pass; tests/proto/slot_sched.cpp: the
// decoding side hands the turn to the helper (it waits for it)
static void slot_host_kick();
static void slot_host_step();    // the end of a decoding step: lane_host.cpp runs a helper pass
// tests/proto/slot_sched.cpp: a point between two of the protocol's LDS word
// accesses where its seeded scheduler may switch sides; and the check of a
// chunk the decoding side took against the packet's bytes (no-ops elsewhere)
static void slot_host_point(int site);
static void slot_host_taken(uint32_t j, uint4& sl);
#ifndef SLOT_MUTANT
#define SLOT_MUTANT 0
#endif
#define SLOT_IDLE() slot_host_kick()
#define SLOT_POINT() slot_host_point(__LINE__)
#define SLOT_TAKEN(s, sl) slot_host_taken((s).j, sl)
#endif

struct SlotSrc {
    uint64_t la;                  // lookahead: the next na bytes, first in bits 63..56
    uint32_t na, q, j, lo15;      // bytes in la; dwords of c taken; c is chunk j; packet start & 15
    uint4 c;                      // (shifted as taken: c.x is dword q of chunk j)
    uint32_t want, gen;
    uint32_t cks;                 // the chunks taken from the slot, summed (slot_mix)
    uint32_t* mctl;               // [0] m_ctl, [1] m_pkt
    const uint32_t* hctl;
    const uint8_t* slot;
};

// Chunk k of a packet's stream as a term of the hand-off's check sum: both
// sides sum the chunks that pass through the slot -- the helper what it
// loads, the decoder what it takes -- and rc_dec6_verify sends a packet
// whose sums differ (but for the helper's last chunk, which a decoder that
// stopped early never takes) to the lane kernels, which read the stream
// themselves.  A chunk of zeros (past the stream's end) adds nothing.
DEV uint32_t slot_mix(const uint4& c, uint32_t k)
{
    return ((c.x ^ (c.y * 0x9E3779B1u)) + (c.z ^ (c.w * 0x85EBCA77u))) * (2u * k + 1u);
}

// the decoder took what its helper loaded, but perhaps the last chunk
DEV bool cks_agree(uint32_t icks, uint32_t hcks, uint32_t hlast)
{
#ifdef SLOT_NO_CKS
    return true;                      // (tests/test_lane_host.py: the check without the sums, for comparison)
#else
    return icks == hcks || icks == hcks - hlast;
#endif
}

DEV void slot_publish(const SlotSrc& s)
{
    s.mctl[0] = ((s.want & 0xFFFu) << 16) | s.gen;
    SLOT_POINT();
}

// h_ctl, then the slot, in that order (see the header)
DEV void slot_read(const SlotSrc& s, uint32_t& hc, uint4& sl)
{
#ifndef RC_LANE_HOST_TEST
    hc = __hip_atomic_load(s.hctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
    sl = *reinterpret_cast<const uint4*>(s.slot);
#else
    // (the host scheduler's model: every dword access on its own, either side
    // may run between any two of them)
    SLOT_POINT();
    hc = *s.hctl;
    SLOT_POINT();
    const uint32_t* w = reinterpret_cast<const uint32_t*>(s.slot);
    sl.x = w[0]; SLOT_POINT();
    sl.y = w[1]; SLOT_POINT();
    sl.z = w[2]; SLOT_POINT();
    sl.w = w[3]; SLOT_POINT();
#endif
}

DEV void slot_shift(SlotSrc& s, bool en)
{
    s.c.x = en ? s.c.y : s.c.x; s.c.y = en ? s.c.z : s.c.y; s.c.z = en ? s.c.w : s.c.z;
}

// one dword into the lookahead where it has room for it and c has one
DEV void slot_fill(SlotSrc& s, bool en)
{
    const bool need = en && s.na <= 4 && s.q < 4;
    const uint32_t d = bswap(s.c.x);
    const uint32_t sh = need ? 32 - 8 * s.na : 0u;
    s.la |= need ? (static_cast<uint64_t>(d) << sh) : 0ull;
    s.na += need ? 4u : 0u;
    s.q += need ? 1u : 0u;
    slot_shift(s, need);
}

// c used up: the slot's chunk if it is chunk j + 1 (hc: h_ctl as read, sl: the slot)
DEV void slot_take(SlotSrc& s, const uint4& sl_in, uint32_t hc, bool en)
{
    const bool ready = ((hc >> 16) & 0xFFFu) == ((s.j + 1) & 0xFFFu) && (hc & 0xFFFFu) == s.gen;
    const bool t = en && s.q == 4 && ready;
#ifdef RC_LANE_HOST_TEST
    uint4 sl = sl_in;                 // (the host tests check it, or replace it: a stale chunk)
    if (t) SLOT_TAKEN(s, sl);
#else
    const uint4& sl = sl_in;
#endif
    s.c.x = t ? sl.x : s.c.x; s.c.y = t ? sl.y : s.c.y; s.c.z = t ? sl.z : s.c.z; s.c.w = t ? sl.w : s.c.w;
#ifndef SLOT_NO_CKS
    s.cks += t ? slot_mix(sl, s.j + 1) : 0u;
#endif
    s.q = t ? 0u : s.q;
    s.j += t ? 1u : 0u;
    s.want = t ? s.j + 1 : s.want;
}

// the end of a step: the next chunk if the slot holds it, the lookahead topped
// up by a dword (a step takes about one byte; one that takes more than the
// lookahead holds waits in dec_code's slow path)
DEV void slot_step_end(SlotSrc& s, const uint4& sl, uint32_t hc)
{
    slot_take(s, sl, hc, s.q == 4);
    slot_fill(s, true);
    slot_publish(s);
#ifdef RC_LANE_HOST_TEST
    slot_host_step();
#endif
}


// at least one byte in the lookahead where `en` (the rare paths): from c, or
// from the slot once the helper has put the next chunk there
DEV void slot_need1(SlotSrc& s, bool en)
{
    bool w = en && s.na == 0 && s.q == 4;
    while (rare_lane(w)) {
        uint32_t hc;
        uint4 sl;
        slot_read(s, hc, sl);
        slot_take(s, sl, hc, w);
        slot_publish(s);
        w = w && s.q == 4;
        if (any_lane(w)) SLOT_IDLE();
    }
    slot_fill(s, en && s.na == 0);
}

DEV uint32_t slot_shift_in(SlotSrc& s, uint32_t code, uint32_t k)
{
    const uint32_t t = static_cast<uint32_t>(s.la >> 32);
    const uint32_t in = static_cast<uint32_t>((static_cast<uint64_t>(t) << (8 * k)) >> 32);
    s.la = k >= 8 ? 0ull : s.la << (8 * k);
    s.na -= k;
    return (code << (8 * k)) | in;
}

// compress.c:354-371 where `en` (rc_lane_common.h dec_code over the slot source)
DEV void dec_code(uint32_t& low, uint32_t& code, uint32_t& range, uint32_t under, uint32_t count, SlotSrc& in,
                  bool en)
{
    low = en ? low + under * range : low;
    range = en ? range * count : range;
    const uint32_t k = en ? settled_bytes(low, range) : 0u;
    const bool fast = k <= in.na;
    const uint32_t kk = fast ? k : 0u;
    code = slot_shift_in(in, code, kk);
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
            slot_need1(in, more);
            code = slot_shift_in(in, code, more ? 1u : 0u);
            range = more ? range << 8 : range;
            low = more ? low << 8 : low;
        } while (rare_lane(more));
    }
}

DEV void dec_code_late(uint32_t& low, uint32_t& code, uint32_t& range, uint32_t under, uint32_t count, SlotSrc& in,
                       bool en)
{
    dec_code(low, code, range, under, count, in, en);
}

// The packet's first chunks (the decoding lane's only global loads for its
// input) and the seed (compress.c:344-350): three dwords from the one holding
// the first byte, so chunks 0 and 1 hold them.  Publishes the packet and the
// first wanted chunk.
DEV void slot_adv0(SlotSrc& s, const uint4& c1)
{
    const bool adv = s.q == 4 && s.j == 0;
    s.c.x = adv ? c1.x : s.c.x; s.c.y = adv ? c1.y : s.c.y; s.c.z = adv ? c1.z : s.c.z; s.c.w = adv ? c1.w : s.c.w;
    s.j += adv ? 1u : 0u;
    s.q = adv ? 0u : s.q;
}

DEV uint32_t slot_init(SlotSrc& s, const uint8_t* p, uint32_t len, uint32_t pkt)
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
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) slot_shift(s, k < s.q);
    s.la = static_cast<uint64_t>(bswap(s.c.x) << (8 * sk)) << 32;
    s.na = 4 - sk;
    s.q += 1;
    slot_shift(s, true);
    slot_adv0(s, c1);
    slot_fill(s, true);
    const uint32_t code = static_cast<uint32_t>(s.la >> 32);
    s.la <<= 32;
    s.na -= 4;
    slot_adv0(s, c1);
    slot_fill(s, true);
    slot_adv0(s, c1);
    s.gen = s.gen % 0xFFFFu + 1u;
    s.want = s.j + 1;
    s.cks = 0;
    // m_pkt, then m_ctl with the new generation (two word stores in that
    // order; the helper reads m_ctl, then m_pkt): a helper that sees the new
    // generation sees this packet, or a later one, whose chunk it would then
    // announce under this generation after the decoder has left it -- never
    // taken.  (One 64-bit store would do on gfx950, whose LDS performs an
    // instruction whole; this order needs only word-sized accesses, which the
    // host scheduler test, tests/proto/slot_sched.cpp, models.)
#if defined(RC_LANE_HOST_TEST) && SLOT_MUTANT == 1
    s.mctl[0] = ((s.want & 0xFFFu) << 16) | s.gen;      // (test mutant: the generation first)
    SLOT_POINT();
    s.mctl[1] = pkt;
#else
    s.mctl[1] = pkt;
#ifndef RC_LANE_HOST_TEST
    asm volatile("" ::: "memory");
#endif
    SLOT_POINT();
    s.mctl[0] = ((s.want & 0xFFFu) << 16) | s.gen;
#endif
    SLOT_POINT();
    // (settled here: a load pending at the step loop's header makes the compiler
    // wait for vmcnt(0) at every step)
    __builtin_amdgcn_s_waitcnt(0);
    return code;
}

// ------------------------------------------------------------------ helper
struct SlotHelp {
    uint32_t have, hgen, cgen, pub, len, pkt, cks, last;   // last: the last loaded chunk's term
    uintptr_t ib;
};

DEV void slot_help_init(SlotHelp& h)
{
    h.have = 0; h.hgen = 0; h.cgen = 0; h.pub = 0; h.len = 0; h.ib = 0; h.pkt = kNoPktS; h.cks = 0; h.last = 0;
}

// One pass over the helper's lanes: a new packet's input range, the wanted
// chunk into the slot, h_ctl.  Returns whether it loaded anything; fin_all:
// every decoding lane of the wavefront is done.  hcks[p]: the sum of the
// chunks loaded for packet p (slot_mix), and hcks[p + stride] the last one's
// term (a decoder that stops before the end of its stream -- an output that
// does not fit -- never takes the chunk it asked for last), stored when the
// lane moves on (a packet seen under a generation not its own -- the reads of
// m_ctl and m_pkt straddling the decoder's start of the next packet -- is
// stored again, with its full sum, when the lane leaves it: the last store is
// the whole packet's).
DEV bool slot_help_iter(const rc_batch_dev& bt, const uint32_t* mctl, uint32_t* hctl, uint8_t* slot, SlotHelp& h,
                        uint32_t* hcks, uint32_t stride, bool& fin_all)
{
    // m_ctl, then m_pkt (see slot_init)
    SLOT_POINT();
    uint2 m;
    m.x = mctl[0];
#ifndef RC_LANE_HOST_TEST
    asm volatile("" ::: "memory");
#endif
    SLOT_POINT();
    m.y = mctl[1];
    SLOT_POINT();
    const bool fin = m.y == kFinS;
    const uint32_t want = (m.x >> 16) & 0xFFFu, mgen = m.x & 0xFFFFu;
    // a new packet: a new generation, or (should the generation have wrapped
    // round unseen) a new packet index; the chunk held is then forgotten
    const bool np = !fin && m.y != kNoPktS && (mgen != h.cgen || m.y != h.pkt);
    const bool leave = (np || fin) && h.pkt != kNoPktS && h.pkt != kFinS;
    if (any_lane(np || leave)) {
        if (leave) {
            hcks[h.pkt] = h.cks;
            hcks[h.pkt + stride] = h.last;
        }
        h.pkt = leave && !np ? kFinS : h.pkt;         // (fin: stored once)
        if (np) {
            h.cks = 0;
            h.last = 0;
            h.len = bt.in_len[m.y];
            h.ib = reinterpret_cast<uintptr_t>(bt.in + bt.in_off[m.y]);
            h.cgen = mgen;
            h.pkt = m.y;
            h.hgen = 0;             // (generation 0: no decoder's, slot_init counts from 1)
        }
    }
    const bool inq = !fin && h.cgen != 0 && mgen == h.cgen && (want != h.have || h.hgen != h.cgen);
    bool busy = false;
    if (any_lane(inq)) {
        busy = true;
        const uintptr_t base = h.ib & ~static_cast<uintptr_t>(15);
        const uint4 c = chunk_load(h.ib, h.ib + h.len, base + 16 * static_cast<uintptr_t>(want), inq);
#ifndef RC_LANE_HOST_TEST
        if (inq) *reinterpret_cast<uint4*>(slot) = c;
#else
        if (inq) {
#if SLOT_MUTANT == 2
            // (test mutant: the announcement before the slot)
            *hctl = (want << 16) | h.cgen;
            h.pub = *hctl;
            SLOT_POINT();
#endif
            uint32_t* w = reinterpret_cast<uint32_t*>(slot);
            w[0] = c.x; SLOT_POINT();
            w[1] = c.y; SLOT_POINT();
            w[2] = c.z; SLOT_POINT();
            w[3] = c.w; SLOT_POINT();
        }
#endif
#ifndef SLOT_NO_CKS
        const uint32_t term = slot_mix(c, want);
        h.cks += inq ? term : 0u;
        h.last = inq ? term : h.last;
#endif
        h.have = inq ? want : h.have;
        h.hgen = inq ? h.cgen : h.hgen;
    }
    const uint32_t hc = (h.have << 16) | h.hgen;
    if (hc != h.pub) {
        // the slot written before the word that announces it (release: the
        // slot's LDS write completes first, and no store moves past this one)
#ifndef RC_LANE_HOST_TEST
        __hip_atomic_store(hctl, hc, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
        *hctl = hc;
        SLOT_POINT();
#endif
        h.pub = hc;
    }
    fin_all = !any_lane(!fin);
    return busy;
}

}  // namespace
