// rc_enc2.hip -- two-pass range-coder encoder (compress.c:246-342), bit-exact.
//
// compress.c's order-1 and order-2 statistics are functions of the packet's
// own bytes, never of the coder's output.  The lane kernels (rc_lane3.hip)
// still rebuild that model byte by byte in HBM, one random record access per
// byte; this encoder derives it from the packet instead, and keeps only the
// root context (order 0) and the range coder serial:
//
//   pass 1, rc_enc2_scan: one wavefront per packet, in LDS.
//     Positions 1..N-1 are bucketed by their previous byte x[i-1].  Both
//     sub-contexts of position i -- order 1 = (x[i-1]), order 2 =
//     (x[i-2], x[i-1]) -- hold only positions of i's bucket, so thread b
//     walks bucket b in position order and derives every order-1/order-2
//     coding interval from counts over the position's bucket predecessors
//     (compress.c:159-199, :286-316):
//        escapes = 5 * dist, total = escapes + 2 * t,
//        count = 2 * same, under = 2 * less
//     (t earlier visits of the context, dist of them with a new symbol,
//     same of them with this symbol, less with a smaller one).  A position
//     visits order 1 only if order 2 lacked its byte, and the root only if
//     order 1 lacked it too.  Output: one 8-B record per position, written
//     straight to the packet's slot of the record stream (no LDS staging).
//   pass 2, rc_enc2_code: one lane per packet.  The root context in LDS
//     (rc_lane_common.h) and the range coder, over the records.  The records
//     also carry the packet's bytes, so a lane reads one uniform stream:
//     every lane consumes one record per step, its loads are the same for all
//     lanes (issued three chunks ahead), and the output window is stored
//     every step (to a dummy slot when nothing is pending).  With the same
//     memory operations on every path, the compiler never has to wait for
//     all outstanding stores before using a record (vmcnt is in order).
//
// tests/proto/twopass.py restates both passes and the record format in
// Python (checked against the oracle on the CPU, tests/test_twopass_model.py).
//
// Fast path: 1 <= N <= 4096 and no bucket over 64 positions (every
// statistic <= 63, so no count reaches the rescale threshold,
// compress.c:313).  A packet over 1919 B can reach the model reset
// (compress.c:148-157): the scan takes it in windows, one per model segment
// (reset_after), and the code pass resets the root where a record carries
// kRst.  Packets with a bigger bucket go to the wide mode (rc_enc2_wscan /
// rc_enc2_wcode, below: explicit intervals, dense walks with rescales) when
// they are at most 1919 B; the rest are listed for the lane kernels, which
// run after the passes on that list only.
//
// Record of position i: two words (w0, w1)
//   w0 bits 0-2 type, 3-8 tA, 9-14 dA, 16-27 ext
//   w1 bits 0-23 second (type 5), 24-31 the byte x[i]
//   type 0  no sub-context codes (root)
//        1  order 1 escape, (tA, dA) = (t1, dist1)                  (root)
//        2  order 1 hit (t1, dist1), ext = same1 | less1 << 6
//        3  order 2 escape (t2, dist2)                              (root)
//        4  order 2 escape (t2, dist2), ext = t1 | dist1 << 6       (root)
//        5  order 2 escape (t2, dist2), second = t1 | dist1 << 6 |
//           same1 << 12 | less1 << 18 (order 1 hit)
//        6  order 2 hit (t2, dist2), ext = same2 | less2 << 6

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "rc_abi_internal.h"
#include "rc_udiv.h"
#include "rc_lane_common.h"
#include "rc_root3.h"

// The file is compiled twice for the library (Makefile): RC_ENC2_PART=1, the
// plain kernels and the launcher (rc_enc2.o), and RC_ENC2_PART=2, the wide
// kernels and their launches (rc_enc2_wide.o, built with the iterative ILP
// scheduler: C3 rc_enc2_wcode2 -9 %, where the plain kernels gain nothing;
// the scheduling strategy is per object file).  Unset (0): the whole file in
// one object (the diagnostic builds).
#ifndef RC_ENC2_PART
#define RC_ENC2_PART 0
#endif
#define E2_PLAIN (RC_ENC2_PART != 2)
#define E2_WIDE (RC_ENC2_PART != 1)

// Diagnostic build only (-DE2_PROF, tools/enc2_prof.py): per-phase cycles of
// the scan pass, summed over wavefronts.  The product build has no stamps.
#ifdef E2_PROF
__device__ unsigned long long g_e2prof[32];
#define E2P_DECL unsigned long long e2p_t = __builtin_amdgcn_s_memtime(), e2p_acc[8] = {0};
#define E2P(k) { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
                 e2p_acc[k] += t_ - e2p_t; e2p_t = t_; __builtin_amdgcn_sched_barrier(0); }
#define E2P_FLUSH { if (threadIdx.x == 0) for (int k_ = 0; k_ < 8; ++k_) atomicAdd(&g_e2prof[k_], e2p_acc[k_]); }
// the code pass: per-phase stamps of code_step, into g_e2prof[8..15]
struct E2Prof { unsigned long long t, acc[8]; };
#define E2Q(k) { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
                 pf.acc[k] += t_ - pf.t; pf.t = t_; __builtin_amdgcn_sched_barrier(0); }
#define E2Q_FLUSH { if ((threadIdx.x & 63) == 0) for (int k_ = 0; k_ < 8; ++k_) atomicAdd(&g_e2prof[8 + k_], pf.acc[k_]); }
// the wide scan: per-phase stamps into g_e2prof[16..27]
struct W2Prof { unsigned long long t, acc[12]; };
#define W2P(k) { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
                 wp.acc[k] += t_ - wp.t; wp.t = t_; __builtin_amdgcn_sched_barrier(0); }
#define W2P_INIT { wp.t = __builtin_amdgcn_s_memtime(); for (int k_ = 0; k_ < 12; ++k_) wp.acc[k_] = 0; }
#define W2P_FLUSH { if ((threadIdx.x & 63) == 0) for (int k_ = 0; k_ < 12; ++k_) atomicAdd(&g_e2prof[16 + k_], wp.acc[k_]); }
#else
struct W2Prof {};
#define W2P(k)
#define W2P_INIT
#define W2P_FLUSH
struct E2Prof {};
#define E2Q(k)
#define E2Q_FLUSH
#define E2P_DECL
#define E2P(k)
#define E2P_FLUSH
#endif

namespace {

constexpr uint32_t kE2MaxLen = 1919;          // compress.c:148-157: no reset below 1920 B
[[maybe_unused]] constexpr uint32_t kE2SlotMax = 4096;        // longest packet of the narrow scan (windows past a reset)
constexpr uint32_t kE2Bucket = 64;            // statistics <= 63
constexpr uint32_t kScanThreads = 64;         // one wavefront per packet, four buckets per lane
constexpr uint32_t kSkipFallback = 0xFFFFFFFFu;   // first word of a slot: lane kernels
constexpr uint32_t kSkipDone = 0xFFFFFFFEu;       // empty packet, out_len already 0
constexpr uint32_t kSkipWide = 0xFFFFFFFDu;       // the wide kernels (the smallest marker)

struct E2Params {
    uint8_t*        stream;     // record stream, one slot per packet of the chunk
    uint64_t        slot_bytes;
    uint32_t        slot_len;   // longest packet a slot holds: min(max_len or 4096, kE2SlotMax)
    uint32_t        lo, hi;     // chunk: batch indices [lo, hi)
    const uint32_t* order;      // batch index -> packet (length-binned), or null
    const uint32_t* bins;       // bins[RC_LEN_BINS] != 0: order not built (uniform batch)
    uint32_t*       list;       // packets for the lane kernels
    uint32_t*       count;
    uint32_t        act;        // pass 2: packets per wavefront (64 or 32)
    uint8_t*        dummy;      // pass 2: 1 MB, 16 B per lane, the target of stores with nothing to store
    uint32_t        slow;       // test switch (ENET_RC_ENC2_SLOW=1): every position exceptional, every bucket re-walked
    // wide mode (below): packets with a bucket over kE2Bucket positions
    uint8_t*        wide;       // wide record stream, one slot per listed packet, or null (off)
    uint64_t        wslot_bytes;
    uint32_t*       wlist;      // listed packets (batch indices): RC_WSHARDS regions of wcap / RC_WSHARDS
    uint32_t*       wcount;     // the regions' counts, RC_WSHARD_STRIDE words apart
    uint32_t        wcap;
    uint32_t        wreg;       // entries per region: min(wcap, the chunk rounded up to RC_WSHARDS) / RC_WSHARDS
};

// the last element slot: buckets of 1918 positions, each padded to 4, end
// below it (1918 + 3 * 255 < 2815); lanes past a packet's end write there

// The wide list in RC_WSHARDS regions, each with its own counter (a
// workgroup appends to region blockIdx.x % RC_WSHARDS): one counter for the
// batch took one atomic per scan workgroup on one address, C3
// rc_enc2_scan_s 0.125 -> 0.207 ms at 64 workgroups per CU.  List position q
// (region q / C, C = e.wreg) is live when its region holds it; the wide
// stream's slot of a listed packet is its list position.  A scan grid that
// is a multiple of RC_WSHARDS (or one packet per workgroup) sends region r
// only packets whose chunk index is r modulo RC_WSHARDS, so a chunk's wide
// packets always fit when the stream has a slot per packet; past a region's
// capacity a packet goes to the lane kernels.
DEV uint32_t wreg_cap(const E2Params& e) { return e.wreg; }
DEV uint32_t wreg_count(const E2Params& e, uint32_t r) { return min(e.wcount[r * RC_WSHARD_STRIDE], wreg_cap(e)); }
DEV bool wq_live(const E2Params& e, uint32_t q)
{
    const uint32_t C = wreg_cap(e);
    if (C == 0) return false;
    const uint32_t r = q / C;
    return r < RC_WSHARDS && q - r * C < wreg_count(e, r);
}
// the live list positions in order: d -> its position (d < the live count)
struct WRegs { uint32_t pre[RC_WSHARDS + 1]; };
DEV WRegs wregs(const E2Params& e)
{
    WRegs w;
    w.pre[0] = 0;
    for (uint32_t r = 0; r < RC_WSHARDS; ++r) w.pre[r + 1] = w.pre[r] + wreg_count(e, r);
    return w;
}
DEV uint32_t wq_of(const E2Params& e, const WRegs& w, uint32_t d)
{
    uint32_t r = 0;
    for (uint32_t k = 1; k < RC_WSHARDS; ++k) r += d >= w.pre[k] ? 1u : 0u;
    return r * wreg_cap(e) + (d - w.pre[r]);
}

// list positions [q0, q0 + m): any live (wave-uniform arguments)
DEV bool wq_any(const E2Params& e, uint32_t q0, uint32_t m)
{
    const uint32_t C = wreg_cap(e);
    bool any = false;
    for (uint32_t r = 0; r < RC_WSHARDS; ++r) {
        const uint32_t lo = r * C, hi = lo + wreg_count(e, r);
        any = any || (q0 < hi && q0 + m > lo);
    }
    return any;
}

DEV uint32_t packet_of(const E2Params& e, uint32_t idx)
{
    return (e.order && !e.bins[RC_LEN_BINS]) ? e.order[idx] : idx;
}

// ------------------------------------------------------------------ pass 1

// L: the longest packet of the launch (as WScanLdsT below): with 1216 the
// element array fits the bigram set's space (14 KB instead of 17 KB per
// wavefront)
constexpr uint32_t kWideSmallL = 1216;     // the smaller LDS layouts: packets up to this many bytes
[[maybe_unused]] constexpr uint32_t kScanMidL = 1408;       // the narrow scan's middle layout (ENet's default MTU: <= 1392 B)
template <uint32_t L>
struct ScanLdsT {
    static constexpr uint32_t kDummyE = L;             // element slot of lanes past the packet
    // packet bytes at x[16 + mis + i] (128 chunks of 16 B; the 1216 layout: the 77
    // chunks a packet of <= L bytes at any alignment needs -- 14.2 -> 13.4 KB, 12
    // scan wavefronts per CU instead of 11, as many as its 149 VGPRs allow)
    uint8_t  x[L + 32 < 16 + 2048 ? 16 + L + 16 : 16 + 2048];
    uint32_t cnt[256];                // bucket sizes, then fill pointers
    uint32_t start[256];              // bucket starts
    union {
        uint32_t seen[2048];          // bigrams (x[i-1], x[i]) seen, 64 Ki bits
        uint32_t e[L + 1];            // elements in bucket order (below), buckets back to back; the dummy slot
    };
    uint32_t excm[64];                // exceptional positions: i or i - 1 repeats an earlier bigram (2048 bits)
    uint32_t probe[16];               // lane-order probe (rc_enc2_scan)
    uint32_t dummy[4];                // target of the atomics of lanes past the packet's end
    uint32_t xmask[256];              // ranks of the bucket's exceptional positions (bit min(rank, 31))
    uint8_t  xlist[256];              // buckets with one
    uint32_t fb[32];                  // packets for the lane kernels, not yet listed
    uint32_t nfb;
    uint32_t wb[32];                  // packets for the wide kernels (batch indices), not yet listed
    uint32_t nwb;
};

// element word: pos (0-10) | v (11-18) | a | 256 (19-27, 0 for position 1) |
//               found2 (28) | does not visit order 1 (29) | found1 (30) |
//               exceptional (31).  A plain position has flags 0.
constexpr uint32_t kF2 = 1u << 28, kNV1 = 1u << 29, kF1 = 1u << 30, kExc = 1u << 31;

// inclusive prefix sum over the wavefront's lanes: DPP row shifts within
// rows of 16, then the row broadcasts (no LDS round trips)
DEV uint32_t wave_incl_scan(uint32_t x)
{
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);   // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return x;
}

// the maximum over the wavefront's lanes (the same network, max for +)
DEV uint32_t wave_max(uint32_t x)
{
    x = max(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false)));
    x = max(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false)));
    x = max(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false)));
    x = max(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false)));
    x = max(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false)));
    x = max(x, static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false)));
    return __builtin_amdgcn_readlane(x, 63);
}

DEV uint32_t lane_id() { return threadIdx.x & 63; }
DEV uint64_t below_mask() { return (1ull << lane_id()) - 1ull; }
DEV uint32_t popc64(uint64_t m) { return static_cast<uint32_t>(__builtin_popcountll(m)); }

// The lanes of `act` whose 8-bit key equals this lane's, from eight ballots
// (one per key bit: at each bit, keep the lanes that agree with this lane);
// lt: how many lanes below this one (of `act`) hold a smaller key (counted at
// the highest bit where they differ).  No LDS, no atomics, any number of
// distinct keys.
DEV uint64_t match8(uint32_t key, uint64_t act, uint32_t& lt)
{
    const uint64_t below = below_mask();
    uint64_t e = act;
    lt = 0;
#pragma unroll
    for (int b = 7; b >= 0; --b) {
        const bool one = (key >> b) & 1u;
        const uint64_t B = __builtin_amdgcn_ballot_w64(one);
        lt += one ? popc64(e & ~B & below) : 0u;
        e &= one ? B : ~B;
    }
    return e;
}

// match8 against ballots taken once (B[b] = lanes with key bit b set):
// several matches on the same key share them
struct KeyBits { uint64_t b[8]; };
DEV KeyBits key_bits(uint32_t key)
{
    KeyBits k;
#pragma unroll
    for (int b = 0; b < 8; ++b) k.b[b] = __builtin_amdgcn_ballot_w64((key >> b) & 1u);
    return k;
}
DEV uint64_t match_bits(uint32_t key, const KeyBits& kb, uint64_t e, uint32_t& lt)
{
    const uint64_t below = below_mask();
    lt = 0;
#pragma unroll
    for (int b = 7; b >= 0; --b) {
        const bool one = (key >> b) & 1u;
        lt += one ? popc64(e & ~kb.b[b] & below) : 0u;
        e &= one ? kb.b[b] : ~kb.b[b];
    }
    return e;
}

// match_bits as masks: the lanes of e with this lane's key (returned) and,
// in ltm, the lanes of e with a smaller key -- counts over any subset of e
// are then popcounts
DEV uint64_t match_bits_lt(uint32_t key, const KeyBits& kb, uint64_t e, uint64_t& ltm)
{
    ltm = 0;
#pragma unroll
    for (int b = 7; b >= 0; --b) {
        const bool one = (key >> b) & 1u;
        ltm |= one ? (e & ~kb.b[b]) : 0ull;
        e &= one ? kb.b[b] : ~kb.b[b];
    }
    return e;
}

DEV bool bit_at(const uint32_t* m, uint32_t i) { return (m[i >> 5] >> (i & 31)) & 1; }

// bytes q-2, q-1, q of the LDS byte array xb (q >= 4) in bits 0-23: two
// dword reads and a funnel shift instead of three byte reads
DEV uint32_t bytes3(const uint8_t* xb, uint32_t q)
{
    const uint32_t* d = reinterpret_cast<const uint32_t*>(xb) + (q >> 2) - 1;
    const uint64_t w = static_cast<uint64_t>(d[1]) << 32 | d[0];
    return static_cast<uint32_t>(w >> (8 * ((q & 3) + 2)));
}

// The scan's workgroup is one wavefront, and LDS operations of a wavefront
// complete in order: lanes see each other's LDS writes without a workgroup
// barrier.  This only keeps the compiler from moving memory operations
// across the point.
DEV void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// The wavefront's packets for the lane kernels are listed 32 at a time: one
// global atomic per 32 packets instead of one per packet (a batch of low-
// entropy packets sends every packet there, and atomics on one address
// serialise).
template <class S>
DEV void fb_flush(S& s, const E2Params& e, uint32_t t)
{
    wave_sync();
    const uint32_t k = s.nfb;
    if (k == 0) return;
    uint32_t base = 0;
    if (t == 0) base = atomicAdd(e.count, k);
    base = __shfl(base, 0, 64);
    if (t < k) e.list[base + t] = s.fb[t];
    wave_sync();
    if (t == 0) s.nfb = 0;
    wave_sync();
}

template <class S>
DEV void fb_add(S& s, const E2Params& e, uint32_t* slot, uint32_t pkt, uint32_t t)
{
    if (t == 0) {
        slot[0] = kSkipFallback;
        s.fb[s.nfb] = pkt;
        s.nfb = s.nfb + 1;
    }
    wave_sync();
    if (s.nfb == 32) fb_flush(s, e, t);
}

// The wavefront's packets for the wide kernels, 32 per global atomic as
// above; a packet past the wide stream's capacity goes to the lane kernels.
template <class S>
DEV void wb_flush(S& s, const E2Params& e, uint32_t t)
{
    wave_sync();
    const uint32_t k = s.nwb;
    if (k == 0) return;
    uint32_t base = 0;
    const uint32_t r = blockIdx.x % RC_WSHARDS, C = wreg_cap(e);
    if (t == 0) base = atomicAdd(e.wcount + r * RC_WSHARD_STRIDE, k);
    base = __shfl(base, 0, 64);
    if (t < k) {
        const uint32_t idx = s.wb[t];
        uint32_t* slot = reinterpret_cast<uint32_t*>(e.stream + static_cast<size_t>(idx - e.lo) * e.slot_bytes);
        if (base + t < C) {
            slot[0] = kSkipWide;
            e.wlist[r * C + base + t] = idx;
        } else {
            slot[0] = kSkipFallback;
            e.list[atomicAdd(e.count, 1u)] = packet_of(e, idx);
        }
    }
    wave_sync();
    if (t == 0) s.nwb = 0;
    wave_sync();
}

// a packet with a bucket over kE2Bucket positions: the wide kernels, or the
// lane kernels when wide mode is off
template <class S>
DEV void big_add(S& s, const E2Params& e, uint32_t* slot, uint32_t pkt, uint32_t idx, uint32_t t)
{
    if (!e.wide) {
        fb_add(s, e, slot, pkt, t);
        return;
    }
    if (t == 0) {
        s.wb[s.nwb] = idx;
        s.nwb = s.nwb + 1;
    }
    wave_sync();
    if (s.nwb == 32) wb_flush(s, e, t);
}

// one predecessor u of an element (v, akey): SWAR accumulators
// t | same << 8 | less << 16 | dist << 24 of order 2 and order 1
DEV void pair(uint32_t u, uint32_t v, uint32_t akey, bool in, uint32_t& acc2, uint32_t& acc1)
{
    const uint32_t uv = (u >> 11) & 255;
    const uint32_t base = 1u | (uv == v ? 0x100u : 0u) | (uv < v ? 0x10000u : 0u);
    const bool m2 = in && ((u >> 19) & 511) == akey;
    const bool m1 = in && (u & kNV1) == 0;
    acc2 += m2 ? (base | ((u & kF2) ? 0u : 0x1000000u)) : 0u;
    acc1 += m1 ? (base | ((u & kF1) ? 0u : 0x1000000u)) : 0u;
}

// record of position pos from its statistics (see the format above)
DEV uint2 make_record(uint32_t acc2, uint32_t acc1, bool f2, bool f1, uint32_t v)
{
    const uint32_t t2 = acc2 & 255, same2 = (acc2 >> 8) & 255, less2 = (acc2 >> 16) & 255, d2 = acc2 >> 24;
    const uint32_t t1 = acc1 & 255, same1 = (acc1 >> 8) & 255, less1 = (acc1 >> 16) & 255, d1 = acc1 >> 24;
    uint32_t r, r2 = 0;
    if (f2) {
        r = 6u | t2 << 3 | d2 << 9 | (same2 | less2 << 6) << 16;
    } else if (t2 != 0) {
        if (t1 == 0) r = 3u | t2 << 3 | d2 << 9;
        else if (f1) { r = 5u | t2 << 3 | d2 << 9; r2 = t1 | d1 << 6 | same1 << 12 | less1 << 18; }
        else r = 4u | t2 << 3 | d2 << 9 | (t1 | d1 << 6) << 16;
    } else if (t1 == 0) {
        r = 0u;
    } else if (f1) {
        r = 2u | t1 << 3 | d1 << 9 | (same1 | less1 << 6) << 16;
    } else {
        r = 1u | t1 << 3 | d1 << 9;
    }
    return make_uint2(r, r2 | v << 24);
}

// exceptional position j of bucket [bs, ...): statistics over all its
// predecessors [bs, j) (their flags are final), its flags, its record
template <class S>
DEV uint32_t scan_exceptional(S& s, uint32_t bs, uint32_t j, uint32_t w,
                                                               uint2* rec)
{
    const uint32_t pos = w & 2047, v = (w >> 11) & 255;
    const uint32_t akey = (w & (256u << 19)) ? (w >> 19) & 511 : 1024u;   // never matches at position 1
    uint32_t acc2 = 0, acc1 = 0;
    for (uint32_t q = bs; q < j; q += 4) {            // bucket starts are 4-aligned
        const uint4 u = *reinterpret_cast<const uint4*>(&s.e[q]);
        pair(u.x, v, akey, true, acc2, acc1);
        pair(u.y, v, akey, q + 1 < j, acc2, acc1);
        pair(u.z, v, akey, q + 2 < j, acc2, acc1);
        pair(u.w, v, akey, q + 3 < j, acc2, acc1);
    }
    const bool f2 = ((acc2 >> 8) & 255) != 0;
    if (f2) acc1 = 0;                                 // compress.c:315: order 1 only after an escape
    const bool f1 = !f2 && ((acc1 >> 8) & 255) != 0;
    rec[pos] = make_record(acc2, acc1, f2, f1, v);
    const uint32_t fl = (f2 ? kF2 | kNV1 : 0u) | (f1 ? kF1 : 0u);
    s.e[j] = w | fl;
    return fl;
}

// insertion sort of a bucket by position (diagnostic safety net: the scatter
// keeps position order when LDS atomics apply in lane order, as on gfx950)
template <class S>
DEV void sort_bucket(S& s, uint32_t bs, uint32_t be)
{
    for (uint32_t j = bs + 1; j < be; ++j) {
        const uint32_t w = s.e[j];
        uint32_t q = j;
        while (q > bs && (s.e[q - 1] & 2047) > (w & 2047)) { s.e[q] = s.e[q - 1]; --q; }
        s.e[q] = w;
    }
}

// Bucket b in position order.  A plain position (neither of its bigrams
// (x[i-2], x[i-1]) and (x[i-1], x[i]) occurs twice in the packet) has no
// order-2 context seen before (t2 = 0) and a new order-1 symbol, so its
// record needs only how many predecessors visited order 1 (t1) and how many
// of those were order-1 hits (dist1 = t1 - hits): counters kept along the
// walk.  Exceptional positions get the full count over their predecessors.
// A bucket holding exceptional positions, in position order: each
// exceptional position needs the flags of the earlier ones; a plain one
// codes t1 = j - (earlier order-2 hits), dist1 = t1 - (earlier order-1 hits),
// hits that occur only at exceptional positions.  xm marks the exceptional
// ranks (bit min(rank, 31)): until the first hit the walk visits only those
// (the plain positions between keep the scatter's records), after it every
// position (their t1, dist1 change).  xm = ~0: every position, every record
// rewritten (after a sort).
template <class S>
DEV void walk_from(S& s, uint32_t bs, uint32_t k, uint32_t xm, uint2* rec)
{
    const bool all = xm == ~0u;
    uint32_t nf2 = 0, nh1 = 0;
    uint32_t j = static_cast<uint32_t>(__builtin_ctz(xm));
#pragma unroll 1
    while (j < k) {
        const uint32_t w = s.e[bs + j];
        if (w & kExc) {
            const uint32_t fl = scan_exceptional(s, bs, bs + j, w, rec);
            nf2 += (fl & kF2) ? 1u : 0u;
            nh1 += (fl & kF1) ? 1u : 0u;
        } else if (all || (nf2 | nh1) != 0) {
            const uint32_t t1 = j - nf2, d1 = t1 - nh1;
            rec[w & 2047] = make_uint2(t1 ? (1u | t1 << 3 | d1 << 9) : 0u, ((w >> 11) & 255) << 24);
        }
        // the next position: the next exceptional one while there was no hit
        const uint32_t rest = (j >= 31 || all || (nf2 | nh1) != 0) ? 0u : (xm & ~((2u << j) - 1u));
        j = (j >= 31 || all || (nf2 | nh1) != 0) ? j + 1 : (rest ? static_cast<uint32_t>(__builtin_ctz(rest)) : k);
    }
}

// The next packet of a scan wavefront, fetched while the current one is
// walked: its length, where its bytes start, and its 16-B chunks in
// registers (two per lane cover 1919 B at any alignment).
struct ScanPf {
    uint32_t pkt, n, mis;
    uint4 r0, r1;
};

// A read-only input array read through the constant address space: wave-
// uniform reads of it become scalar loads (counted in lgkmcnt, so using them
// never waits for the vector stores in flight).  The batch's lengths, offsets
// and the length order are not written while the scan runs.
template <typename T>
DEV T const_load(const T* p, uint32_t i)
{
    typedef const __attribute__((address_space(4))) T* cptr;
    return ((cptr) reinterpret_cast<uintptr_t>(p))[i];
}

DEV ScanPf scan_prefetch(const rc_batch_dev& b, const E2Params& e, uint32_t idx)
{
    ScanPf f;
    f.pkt = 0; f.n = 0; f.mis = 0;
    // (the loads are issued on every path -- a register written on one path
    // only would make the compiler wait for them at the merge; with nothing to
    // fetch they read the batch's first 16 B)
    uintptr_t a0 = reinterpret_cast<uintptr_t>(b.in) & ~static_cast<uintptr_t>(15), a1 = a0;
    if (idx < e.hi) {
        f.pkt = (e.order && !const_load(e.bins, RC_LEN_BINS)) ? const_load(e.order, idx) : idx;
        f.n = const_load(b.in_len, f.pkt);
        if (f.n != 0 && f.n <= e.slot_len) {
            const uintptr_t src = reinterpret_cast<uintptr_t>(b.in + const_load(b.in_off, f.pkt));
            const uintptr_t a16 = src & ~static_cast<uintptr_t>(15);
            f.mis = static_cast<uint32_t>(src & 15);
            // (clamped to the packet's last chunk: chunks past it land in LDS
            // past the packet, where nothing reads them)
            const uint32_t last = (f.mis + f.n - 1) >> 4;
            a0 = a16 + 16 * min(threadIdx.x, last);
            a1 = a16 + 16 * min(threadIdx.x + kScanThreads, last);
        }
    }
    f.r0 = gload16(a0);
    f.r1 = gload16(a1);
    return f;
}

// first word of a model segment's position-0 record after a reset (w0 bit 15: unused by the types)
constexpr uint32_t kRst = 1u << 15;
constexpr uint32_t kMaxNodesE2 = 4096 - 2;       // compress.c:150

// bucket ends from the scatter's fill counters (start << 16 | elements)
DEV uint4 bucket_ends(const uint4 c)
{
    return make_uint4((c.x >> 16) + (c.x & 0xFFFFu), (c.y >> 16) + (c.y & 0xFFFFu), (c.z >> 16) + (c.z & 0xFFFFu),
                      (c.w >> 16) + (c.w & 0xFFFFu));
}

// The nodes compress.c creates at each position of a window scanned as a
// packet (compress.c:68-88 via :286-337): position 0 the root's; a position
// found nowhere (its record visits the root) creates the root's node at the
// byte's first root visit, its order-1 node (position >= 1) and its order-2
// node (>= 2); an order-1 hit its order-2 node (>= 2); an order-2 hit none.
// Returns the window position after whose byte the node count reaches 4094
// (compress.c:148-157), or n.  After the scan's walks (every element's
// found flags final); the window's bytes in s.x and the bucket ends in s.cnt
// are reused.
template <class S>
DEV uint32_t reset_after(S& s, uint32_t n, uint32_t x0, uint32_t t)
{
    uint8_t* inc = s.x;                                   // per position: nodes | 0x80 = root visit
    const uint4 b4 = *reinterpret_cast<const uint4*>(&s.start[4 * t]);
    const uint4 e4 = bucket_ends(*reinterpret_cast<const uint4*>(&s.cnt[4 * t]));
    wave_sync();
    *reinterpret_cast<uint4*>(&s.cnt[4 * t]) = make_uint4(~0u, ~0u, ~0u, ~0u);   // the first root visit per byte
    wave_sync();
    if (t == 0) { s.cnt[x0] = 0u; inc[0] = 1; }
#pragma unroll 1
    for (uint32_t r = 0; r < 4; ++r) {
        const uint32_t be = pick4(r, e4);
        for (uint32_t k = pick4(r, b4); k < be; ++k) {
            const uint32_t w = s.e[k], pos = w & 2047;
            const bool rv = (w & (kF2 | kF1)) == 0;
            const uint32_t c = rv ? (pos >= 1 ? 1u : 0u) + (pos >= 2 ? 1u : 0u) : ((w & kF2) ? 0u : (pos >= 2 ? 1u : 0u));
            inc[pos] = static_cast<uint8_t>(c | (rv ? 0x80u : 0u));
            if (rv) atomicMin(&s.cnt[(w >> 11) & 255], pos);
        }
    }
    wave_sync();
#pragma unroll 1
    for (uint32_t r = 0; r < 4; ++r) {
        const uint32_t be = pick4(r, e4);
        for (uint32_t k = pick4(r, b4); k < be; ++k) {
            const uint32_t w = s.e[k], pos = w & 2047;
            if ((w & (kF2 | kF1)) == 0 && s.cnt[(w >> 11) & 255] == pos) inc[pos] = static_cast<uint8_t>(inc[pos] + 1);
        }
    }
    wave_sync();
    // positions 32 t .. 32 t + 31: their sum, the prefix over the lanes, the first crossing
    uint32_t sum = 0;
#pragma unroll 8
    for (uint32_t q = 0; q < 32; ++q) {
        const uint32_t pos = 32 * t + q;
        sum += pos < n ? (inc[pos] & 0x7Fu) : 0u;
    }
    uint32_t acc = 1 + wave_incl_scan(sum) - sum;        // nodes before position 32 t (the root: 1)
    uint32_t hit = n;
    if (acc + sum >= kMaxNodesE2) {
#pragma unroll 1
        for (uint32_t q = 0; q < 32; ++q) {
            const uint32_t pos = 32 * t + q;
            if (pos >= n) break;
            acc += inc[pos] & 0x7Fu;
            if (acc >= kMaxNodesE2) { hit = pos; break; }
        }
    }
    // the lowest lane's crossing
    const uint64_t m = __builtin_amdgcn_ballot_w64(hit < n);
    const uint32_t r = m ? __builtin_amdgcn_readlane(hit, static_cast<uint32_t>(__builtin_ctzll(m))) : n;
    wave_sync();
    return r;
}

// Same-address LDS atomics in lane order within an instruction and in
// program order across instructions, for a full conflict (twice) and for
// partial ones (4 words, lanes interleaved, blocked and hashed onto them).
// Checked once per wavefront; the scan's shortcuts are taken only if it holds.
DEV bool lane_order_probe(uint32_t* pr, uint32_t t)
{
    if (t < 16) pr[t] = 0;
    wave_sync();
    const uint64_t below = (1ull << t) - 1ull;
    const uint32_t k3 = (t * 2654435761u >> 28) & 3;
    uint64_t same3 = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        const uint64_t m = __builtin_amdgcn_ballot_w64(k3 == q);
        same3 = k3 == q ? m : same3;
    }
    bool ok = atomicAdd(&pr[0], 1u) == t;
    ok = (atomicAdd(&pr[0], 1u) == 64 + t) && ok;
    ok = (atomicAdd(&pr[1 + (t & 3)], 1u) == (t >> 2)) && ok;
    ok = (atomicAdd(&pr[5 + (t >> 4)], 1u) == (t & 15)) && ok;
    ok = (atomicAdd(&pr[9 + k3], 1u) == static_cast<uint32_t>(__builtin_popcountll(same3 & below))) && ok;
    return !any_lane(!ok);
}

template <class S>
DEV void scan_main(const rc_batch_dev& b, const E2Params& e, S& s)
{
    const uint32_t t = threadIdx.x;
    E2P_DECL
    // The repeat bits and bucket ranks below rely on same-address LDS atomics
    // applying in lane order within an instruction and in program order
    // across instructions (gfx950 does, tools/atomorder.hip); without it
    // every position takes the full statistics and every bucket is sorted.
    // The shortcut is taken only on the architecture it was verified on
    // (gfx950: tools/atomorder.hip, every conflict pattern of the scatter), and
    // only where the per-wavefront probe confirms it; a per-packet check of
    // every bucket's order cost 23 % of this kernel (0.43 -> 0.53 ms, C2).
#if defined(__gfx950__)
    const bool ordered = lane_order_probe(s.probe, t) && !e.slow;
#else
    const bool ordered = false;
#endif
    if (t == 0) { s.nfb = 0; s.nwb = 0; }
    ScanPf pf = scan_prefetch(b, e, e.lo + blockIdx.x);
    for (uint32_t idx = e.lo + blockIdx.x; idx < e.hi; idx += gridDim.x) {
        const ScanPf cur = pf;
        const uint32_t pkt = cur.pkt, len = cur.n;
        uint32_t* slot = reinterpret_cast<uint32_t*>(e.stream + static_cast<size_t>(idx - e.lo) * e.slot_bytes);
        // compress.c:257, or longer than the caller's max_len (its slot holds
        // 8 B per position up to slot_len only)
        if (len == 0 || len > e.slot_len) {
            if (len == 0) {
                if (t == 0) { slot[0] = kSkipDone; b.out_len[pkt] = 0; }
            } else {
                fb_add(s, e, slot, pkt, t);
            }
            pf = scan_prefetch(b, e, idx + gridDim.x);
            continue;
        }
        // A packet longer than kE2MaxLen can reach compress.c's model reset
        // (:148-157): it is scanned in windows, each starting a model segment
        // (the window a packet of its own) and as long as the LDS holds; the
        // nodes the window's positions create give the byte after which the
        // model resets, the next window starts after it (its position 0
        // record carries kRst), and the records this window wrote past that
        // byte are rewritten by the next.
        uint32_t s0 = 0, mis = cur.mis;
        uint4 c0 = cur.r0, c1 = cur.r1;
        bool fetched = false;
        const uintptr_t src0 = reinterpret_cast<uintptr_t>(b.in + const_load(b.in_off, pkt));
#pragma unroll 1
        for (;;) {
        const uint32_t n = min(len - s0, 2048u - mis);
        // the window into LDS: aligned 16-B chunks, x = s.x + 16 + misalignment
        *reinterpret_cast<uint4*>(s.x + 16 + 16 * t) = c0;
        if (16 + 16 * (t + kScanThreads) + 16 <= sizeof(s.x))   // (chunks past the layout's repeat the last)
            *reinterpret_cast<uint4*>(s.x + 16 + 16 * (t + kScanThreads)) = c1;
        const uint4 z = make_uint4(0u, 0u, 0u, 0u);
        *reinterpret_cast<uint4*>(&s.cnt[4 * t]) = z;
        if (t < 16) *reinterpret_cast<uint4*>(&s.excm[4 * t]) = z;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) *reinterpret_cast<uint4*>(&s.seen[4 * (t + 64 * k)]) = z;
        wave_sync();
        E2P(0)
        const uint8_t* x = s.x + 16 + mis;
        const uint32_t q0 = 16 + mis;                  // s.x index of position 0
        // bucket sizes, and the positions whose bigram occurred before (the
        // old bit of the seen set: position order, when same-address
        // atomics of one instruction apply in lane order -- `ordered`)
        // (branch-free: a lane past the packet's end reads the last position
        // and sends its atomics to a dummy word, so no wait sits inside a
        // per-position branch)
        for (uint32_t i = 1 + t; i < n; i += 4 * kScanThreads) {
            uint32_t key[4], old[4];
            bool ok[4];
#pragma unroll
            for (uint32_t m = 0; m < 4; ++m) {
                const uint32_t ii = i + m * kScanThreads;
                ok[m] = ii < n;
                key[m] = (__builtin_bswap32(bytes3(s.x, q0 + min(ii, n - 1))) >> 8) & 0xFFFFu;
            }
#pragma unroll
            for (uint32_t m = 0; m < 4; ++m) {
                atomicAdd(ok[m] ? &s.cnt[key[m] >> 8] : &s.dummy[0], 1u);
                old[m] = atomicOr(ok[m] ? &s.seen[key[m] >> 5] : &s.dummy[1], 1u << (key[m] & 31));
            }
            if (i == 1 + t) {
                // after the first 256 positions: a bucket already past kE2Bucket
                // sends the packet to the lane kernels now (the check below);
                // low-entropy packets would otherwise count on through
                // same-address atomics that serialise (C3: 7x this loop's time)
                wave_sync();
                const uint4 c4 = *reinterpret_cast<const uint4*>(&s.cnt[4 * t]);
                if (any_lane(max(max(c4.x, c4.y), max(c4.z, c4.w)) > kE2Bucket)) break;
            }
#pragma unroll
            for (uint32_t m = 0; m < 4; ++m)
                if (ok[m] && (old[m] & (1u << (key[m] & 31)))) {
                    // position ii's bigram repeats: ii and ii + 1 are exceptional
                    const uint32_t ii = i + m * kScanThreads;
                    atomicOr(&s.excm[ii >> 5], 1u << (ii & 31));
                    atomicOr(&s.excm[(ii + 1) >> 5], 1u << ((ii + 1) & 31));
                }
        }
        wave_sync();
        E2P(1)
        // lane t owns buckets 4t .. 4t+3: sizes, 4-aligned starts
        const uint4 c4 = *reinterpret_cast<const uint4*>(&s.cnt[4 * t]);
        const uint32_t mx = max(max(c4.x, c4.y), max(c4.z, c4.w));
        if (any_lane(mx > kE2Bucket)) {
            big_add(s, e, slot, pkt, idx, t);            // (the wide kernels reset as this scan does)
            if (!fetched) pf = scan_prefetch(b, e, idx + gridDim.x);
            break;
        }
        // (buckets back to back: with the old padding to 4 the elements of an
        // MTU-bounded packet outgrew the bigram set they share LDS with)
        const uint32_t a0 = c4.x, a1 = c4.y, a2 = c4.z, a3 = c4.w;
        const uint32_t mine = a0 + a1 + a2 + a3;
        const uint32_t st = wave_incl_scan(mine) - mine;
        const uint4 s4 = make_uint4(st, st + a0, st + a0 + a1, st + a0 + a1 + a2);
        *reinterpret_cast<uint4*>(&s.start[4 * t]) = s4;
        *reinterpret_cast<uint4*>(&s.cnt[4 * t]) = make_uint4(s4.x << 16, s4.y << 16, s4.z << 16, s4.w << 16);
        wave_sync();
        E2P(2)
        *reinterpret_cast<uint4*>(&s.xmask[4 * t]) = z;
        wave_sync();
        // Scatter into buckets, and each position's record as in a bucket with
        // no exceptional position: t1 = dist1 = its rank j in the bucket (the
        // walk below rewrites the buckets that have one).  The rank is the
        // slot from the LDS atomic, i.e. position order when same-address
        // atomics apply in lane and program order (lane_order_probe; gfx950
        // does, tools/atomorder.hip); otherwise every bucket is sorted and
        // walked in full below.  (A per-position check of the predecessor
        // slot cost 4 % of the encoder and could not see a later position
        // taking an earlier slot, whose write comes after the check.)
        uint2* rec = reinterpret_cast<uint2*>(slot) + s0;
        for (uint32_t i = 1 + t; i < n; i += 4 * kScanThreads) {
            // (branch-free as above: reads, then atomics and starts, then writes)
            uint32_t b3[4], ew[4], w[4], k[4], bb[4], jr[4];
            bool ok[4];
#pragma unroll
            for (uint32_t m = 0; m < 4; ++m) {
                const uint32_t ii = min(i + m * kScanThreads, n - 1);
                b3[m] = bytes3(s.x, q0 + ii);
                ew[m] = s.excm[ii >> 5];
            }
#pragma unroll
            for (uint32_t m = 0; m < 4; ++m) {
                const uint32_t ii = i + m * kScanThreads;
                ok[m] = ii < n;
                const uint32_t p = (b3[m] >> 8) & 255, v = (b3[m] >> 16) & 255, a = ii >= 2 ? b3[m] & 255 : 0u;
                // full statistics where v may already be in the order-1
                // context (its bigram occurred before) or the order-2
                // context exists (the bigram before it occurred before);
                // every other position is plain (see walk_from)
                const bool exc = ((ew[m] >> (ii & 31)) & 1u) != 0 || !ordered;
                w[m] = ii | v << 11 | (ii >= 2 ? (a | 256u) << 19 : 0u) | (exc ? kExc : 0u);
                bb[m] = p;
            }
#pragma unroll
            for (uint32_t m = 0; m < 4; ++m) {
                // (start << 16 | rank: one atomic gives the slot and the rank)
                const uint32_t r = atomicAdd(ok[m] ? &s.cnt[bb[m]] : &s.dummy[0], 1u);
                jr[m] = r & 0xFFFFu;
                k[m] = (r >> 16) + jr[m];
            }
#pragma unroll
            for (uint32_t m = 0; m < 4; ++m) {
                s.e[ok[m] ? k[m] : S::kDummyE] = w[m];
                const uint32_t j = jr[m];
                if (ok[m]) {
                    rec[w[m] & 2047] = make_uint2(j ? (1u | j << 3 | j << 9) : 0u, ((w[m] >> 11) & 255) << 24);
                    if (w[m] & kExc) atomicOr(&s.xmask[bb[m]], 1u << min(j, 31u));
                }
            }
        }
        E2P(3)
        const uint32_t x0 = x[0];
        wave_sync();
        const bool disorder = !ordered;                // (wave-uniform)
        if (!fetched) pf = scan_prefetch(b, e, idx + gridDim.x);     // (the bytes in LDS are not read past here)
        fetched = true;
        E2P(6)
        // buckets with exceptional positions: compacted over the lanes, one
        // per lane, each walked in full
        {
            const uint4 f = *reinterpret_cast<const uint4*>(&s.xmask[4 * t]);
            const uint32_t m0 = f.x != 0, m1 = f.y != 0, m2 = f.z != 0, m3 = f.w != 0;
            const uint32_t cntx = m0 + m1 + m2 + m3;
            const uint32_t incl = wave_incl_scan(cntx);
            uint32_t o = incl - cntx;
            if (m0) s.xlist[o++] = static_cast<uint8_t>(4 * t);
            if (m1) s.xlist[o++] = static_cast<uint8_t>(4 * t + 1);
            if (m2) s.xlist[o++] = static_cast<uint8_t>(4 * t + 2);
            if (m3) s.xlist[o++] = static_cast<uint8_t>(4 * t + 3);
            const uint32_t nx = __builtin_amdgcn_readlane(incl, 63);
            wave_sync();
#pragma unroll 1
            for (uint32_t q = t; q < nx; q += kScanThreads) {
                const uint32_t bk = s.xlist[q];
                const uint32_t bs = s.start[bk], kk = s.cnt[bk] & 0xFFFFu;
                walk_from(s, bs, kk, s.xmask[bk], rec);
            }
        }
        E2P(4)
        if (rare_lane(disorder)) {
            // (not seen on gfx950) the scatter's ranks were not position
            // order somewhere: every bucket sorted, its flags cleared, every
            // position exceptional (the repeat bits came from the same
            // atomics), walked from its start with every record rewritten
            wave_sync();
#pragma unroll 1
            for (uint32_t r = 0; r < 4; ++r) {
                const uint32_t bs = pick4(r, s4), kk = pick4(r, c4);
                for (uint32_t j = 0; j < kk; ++j) s.e[bs + j] = (s.e[bs + j] & ~(kF2 | kNV1 | kF1)) | kExc;
                sort_bucket(s, bs, bs + kk);
                walk_from(s, bs, kk, ~0u, rec);
            }
        }
        if (t == 0) rec[0] = make_uint2(s0 ? kRst : 0u, x0 << 24);  // position 0: root only (after a reset)
        wave_sync();                              // LDS reuse by the next packet
        E2P(5)
        if (len <= kE2MaxLen) break;              // (no reset: <= 2 * 1918 + 256 nodes, compress.c:150)
        const uint32_t r = reset_after(s, n, x0, t);
        if (r >= n) {                             // no reset in the window
            if (s0 + n < len) fb_add(s, e, slot, pkt, t);   // a segment longer than the window: lane kernels
            break;
        }
        s0 += r + 1;
        if (s0 >= len) break;                     // (the reset after the last byte changes nothing)
        // the next window's bytes (not prefetched: only long packets get here)
        const uintptr_t src = src0 + s0, a16 = src & ~static_cast<uintptr_t>(15);
        mis = static_cast<uint32_t>(src & 15);
        const uint32_t last = (mis + (len - s0) - 1) >> 4;
        c0 = gload16(a16 + 16 * min(t, last));
        c1 = gload16(a16 + 16 * min(t + kScanThreads, last));
        }
    }
    fb_flush(s, e, t);
    wb_flush(s, e, t);
    E2P_FLUSH
}

#if E2_PLAIN
extern "C" __global__ __launch_bounds__(kScanThreads)
void rc_enc2_scan(rc_batch_dev b, E2Params e)
{
    __shared__ __attribute__((aligned(16))) ScanLdsT<2048> s;
    scan_main(b, e, s);
}
#endif

// the same for launches whose packets are at most kWideSmallL bytes
#if E2_PLAIN
extern "C" __global__ __launch_bounds__(kScanThreads)
void rc_enc2_scan_s(rc_batch_dev b, E2Params e)
{
    __shared__ __attribute__((aligned(16))) ScanLdsT<kWideSmallL> s;
    scan_main(b, e, s);
}

// ... and for launches of MTU-bounded packets (C4: 64-1392 B): 13.6 KB of LDS,
// 12 wavefronts per CU where the 2048 layout (17.3 KB) fits 9
extern "C" __global__ __launch_bounds__(kScanThreads)
void rc_enc2_scan_m(rc_batch_dev b, E2Params e)
{
    __shared__ __attribute__((aligned(16))) ScanLdsT<kScanMidL> s;
    scan_main(b, e, s);
}
#endif

// ------------------------------------------------------------------ pass 2

// ---- output: a 32-B ring per lane in LDS.  Byte A of the packet's output
// (A an absolute address) lives at ring[A & 31], so every aligned 16-B chunk
// of the output is an aligned 16-B slot of the ring.  A code appends its
// settled bytes with three byte writes (bytes past the count are rewritten by
// the next code before their chunk completes); a chunk that completes during
// a step is read back then and stored at the end of the next step, by a
// store issued on every path (to a dummy slot when no chunk is due).
struct Ring {
    uint8_t* r;
    uintptr_t lo;               // output start
    uint32_t n, cap;            // bytes produced, capacity (compress.c:114-119)
    uint4 ch;                   // completed chunk awaiting its store
    uintptr_t ca;               // its address, or the dummy slot
};

DEV void ring_put(Ring& o, uint32_t low, uint32_t k, bool put)
{
    if (put) {
        const uint32_t p = static_cast<uint32_t>(o.lo) + o.n;
        o.r[p & 31] = static_cast<uint8_t>(low >> 24);
        o.r[(p + 1) & 31] = static_cast<uint8_t>(low >> 16);
        o.r[(p + 2) & 31] = static_cast<uint8_t>(low >> 8);
        o.n += k;
    }
}

// the chunk store of the previous step (always issued; the dummy slot is the
// lane's first record chunk, consumed before the loop)
DEV void ring_store(Ring& o)
{
    const v4u32 d = {o.ch.x, o.ch.y, o.ch.z, o.ch.w};
    *GPTR(v4u32, o.ca) = d;
}

// after a step's codes: a chunk completed since n0 is read back for storing
// (positions as the address's low 32 bits; one 64-bit add for the store)
DEV void ring_chunk(Ring& o, uint32_t n0, uintptr_t dummy)
{
    const uint32_t lo32 = static_cast<uint32_t>(o.lo);
    const uint32_t e0 = lo32 + n0, e1 = lo32 + o.n;
    const bool done = (e0 >> 4) != (e1 >> 4);         // codes add <= 12 bytes: at most one chunk
    const uint32_t c = (e1 & ~15u) - 16u;
    o.ch = *reinterpret_cast<const uint4*>(o.r + (c & 31));
    const int32_t rel = static_cast<int32_t>(c - lo32);   // the chunk's start, from the output start
    const bool fits = rel + 16 <= static_cast<int32_t>(o.cap);   // (only a failing packet has one that does not)
    const bool edge = done && fits && rel < 0;        // the first chunk starts before the output
    o.ca = (done && fits && rel >= 0) ? o.lo + static_cast<intptr_t>(rel) : dummy;
    if (rare_lane(edge)) {
        if (edge) sink_bytes(o.lo + static_cast<intptr_t>(rel), o.ch, 0, 16, o.lo);
    }
}

// the last, partial chunk
DEV void ring_finish(Ring& o, bool en)
{
    if (rare_lane(en)) {
        if (en) {
            const uintptr_t e1 = o.lo + o.n, c = e1 & ~static_cast<uintptr_t>(15);
            if (e1 > c) {
                const uint4 w = *reinterpret_cast<const uint4*>(o.r + (c & 31));
                sink_bytes(c, w, 0, static_cast<uint32_t>(e1 - c), o.lo);
            }
        }
    }
}

// the rest of compress.c:125-136 after the settled bytes: range < BOTTOM
// (rare: one ballot on the common path)
DEV void code_slow(uint32_t& low, uint32_t& range, Ring& o)
{
    bool more = range < kBot;
    while (any_lane(more)) {
        const bool carry = (low ^ (low + range)) >= kTop;
        const bool stop = carry && range >= kBot;
        more = more && !stop;
        if (!any_lane(more)) break;
        range = (more && carry) ? ((0u - low) & (kBot - 1)) : range;
        ring_put(o, low, 1, more);
        range = more ? range << 8 : range;
        low = more ? low << 8 : low;
    }
}

// compress.c:121-137, branch-free: rt = rcp64(total), prepared a step ahead.
// A lane without this code passes (under, count, rt) = (0, 1, 1.0), which
// leaves low and range as they are and settles no byte (a normalised coder
// has no settled byte), so no lane needs a mask.  The output capacity is not
// checked per code: compress.c returns 0 as soon as a byte does not fit
// (compress.c:116-117), i.e. iff the whole output exceeds it, which the
// caller checks at the end; chunks past the capacity are never stored.
DEV void code(uint32_t& low, uint32_t& range, uint32_t under, uint32_t count, double rt, Ring& o)
{
    const uint32_t r = udiv16d(range, 0u, rt);
    low = low + under * r;
    range = r * count;
    const uint32_t k = settled_bytes(low, range);
    // (three byte writes: bytes past the count are rewritten by the next code
    // before their chunk completes)
    const uint32_t p = static_cast<uint32_t>(o.lo) + o.n;
    o.r[p & 31] = static_cast<uint8_t>(low >> 24);
    o.r[(p + 1) & 31] = static_cast<uint8_t>(low >> 16);
    o.r[(p + 2) & 31] = static_cast<uint8_t>(low >> 8);
    o.n += k;
    low <<= 8 * k;
    range <<= 8 * k;
    if (rare_lane(range < kBot)) code_slow(low, range, o);
}

// keeps a value's computation ahead of this point: the compiler otherwise
// sinks it next to its use, where it stalls the in-order issue
DEV void pin(double& x) { asm volatile("" : "+v"(x)); }

// interval of a sub-context code from (t, dist[, same, less]): compress.c:301-308
DEV void sub_interval(uint32_t t, uint32_t d, uint32_t same, uint32_t less, bool hit, uint32_t& under,
                      uint32_t& count, uint32_t& total)
{
    const uint32_t esc = 5 * d;
    total = esc + 2 * t;
    under = hit ? esc + 2 * less : 0u;
    count = hit ? 2 * same : esc;
}

// A position's sub-context codes, prepared from its record a step ahead (off
// the chain through low and range): order 2 (types 3-6) or order 1 (types 1,
// 2) first, then order 1 after an order-2 escape (types 4, 5); e0: the root
// codes it (types 0, 1, 3, 4).
struct Pre {
    uint32_t u1, c1, u2, c2, v;
    double r1, r2;
    bool e2, e0, rst;           // rst: the model resets before this position (kRst)
};

DEV Pre prep(uint32_t w0, uint32_t w1, bool en)
{
    Pre p;
    const uint32_t typ = w0 & 7, ext = w0 >> 16;
    uint32_t un, ct, tt, un2, ct2, tt2;
    sub_interval((w0 >> 3) & 63, (w0 >> 9) & 63, ext & 63, (ext >> 6) & 63, typ == 2 || typ == 6, un, ct, tt);
    const uint32_t fb = typ == 5 ? w1 : ext;
    sub_interval(fb & 63, (fb >> 6) & 63, (fb >> 12) & 63, (fb >> 18) & 63, typ == 5, un2, ct2, tt2);
    const bool e1 = en && typ != 0;
    p.e2 = en && (typ == 4 || typ == 5);
    p.e0 = en && (typ <= 1 || typ == 3 || typ == 4);
    p.u1 = e1 ? un : 0u;
    p.c1 = e1 ? ct : 1u;
    p.r1 = rcp64(e1 ? tt : 1u);
    p.u2 = p.e2 ? un2 : 0u;
    p.c2 = p.e2 ? ct2 : 1u;
    p.r2 = rcp64(p.e2 ? tt2 : 1u);
    p.v = w1 >> 24;
    p.rst = en && (w0 & kRst) != 0;
    return p;
}

// prep with the reciprocals of the sub-context totals (<= 5 * 63 + 2 * 63)
// from an LDS table instead of computed
constexpr uint32_t kRcpTab = 5 * 63 + 2 * 63 + 1;
DEV Pre prep_tab(uint32_t w0, uint32_t w1, bool en, const double* rtab)
{
    Pre p;
    const uint32_t typ = w0 & 7, ext = w0 >> 16;
    uint32_t un, ct, tt, un2, ct2, tt2;
    sub_interval((w0 >> 3) & 63, (w0 >> 9) & 63, ext & 63, (ext >> 6) & 63, typ == 2 || typ == 6, un, ct, tt);
    const uint32_t fb = typ == 5 ? w1 : ext;
    sub_interval(fb & 63, (fb >> 6) & 63, (fb >> 12) & 63, (fb >> 18) & 63, typ == 5, un2, ct2, tt2);
    const bool e1 = en && typ != 0;
    p.e2 = en && (typ == 4 || typ == 5);
    p.e0 = en && (typ <= 1 || typ == 3 || typ == 4);
    p.u1 = e1 ? un : 0u;
    p.c1 = e1 ? ct : 1u;
    p.r1 = rtab[e1 ? tt : 1u];
    p.u2 = p.e2 ? un2 : 0u;
    p.c2 = p.e2 ? ct2 : 1u;
    p.r2 = rtab[p.e2 ? tt2 : 1u];
    p.v = w1 >> 24;
    p.rst = en && (w0 & kRst) != 0;
    return p;
}

struct CodeState {
    uint32_t low, range, rtot;
    double rrt;                 // rcp64(rtot)
};

// one position: its sub-context codes, then the root (compress.c:286-337);
// p = this position's prepared codes, replaced by the next position's
// (record words w0n, w1n)
DEV void code_step(CodeState& k, Ring& o, uint8_t* root, const uint8_t* mtab, const uint8_t* itab, Pre& p,
                   uint32_t w0n, uint32_t w1n, bool enn, uintptr_t dummy, E2Prof& pf)
{
    E2Q(0)
    const uint32_t n0 = o.n;
    if (rare_lane(p.rst)) {                           // compress.c:148-157, after the previous byte
        if (p.rst) {
            Root R;
            root3_clear<true>(root, R);
            k.rtot = 1 + 256;
            k.rrt = rcp64(k.rtot);
        }
    }
    // the root lookup needs only v: LDS reads whose latency overlaps the
    // sub-context codes
    uint32_t under0, cnt0;
    root3_lookup(root, mtab, p.v, under0, cnt0);
    const RootAddPre ra = root3_add_read(root, itab, p.v);   // (the update's reads, early)
    E2Q(1)
    const Pre q = prep(w0n, w1n, enn);
    const uint32_t rtot1 = p.e0 ? ((k.rtot + kRootDelta) & 0xFFFF) : k.rtot;
    double rrt1 = rcp64(rtot1);                       // (the next root code's, unless a rescale)
    code(k.low, k.range, p.u1, p.c1, p.r1, o);
    E2Q(2)
    if (any_lane(p.e2)) code(k.low, k.range, p.u2, p.c2, p.r2, o);
    E2Q(3)
    E2Q(4)
    // root, compress.c:318-329
    code(k.low, k.range, p.e0 ? 1 + under0 : 0u, p.e0 ? 1 + cnt0 : 1u, p.e0 ? k.rrt : 1.0, o);
    if (p.e0) root3_add_write(root, p.v, cnt0, ra);
    E2Q(5)
    k.rtot = rtot1;
    const bool rs0 = p.e0 && (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || k.rtot > kTotalLimit);
    if (any_lane(rs0)) {
        if (rs0) { Root R; k.rtot = root3_rescale<true>(root, R); }
        rrt1 = rcp64(k.rtot);
    }
    k.rrt = rrt1;
    ring_store(o);                                    // the chunk read back a step ago
    ring_chunk(o, n0, dummy);
    p = q;
    E2Q(6)
}

// Per lane: the root (counts, D copy) at 0, the ring at 288, pad to 336 B
// (84 dwords: b128 accesses conflict-free).  Two chunks suffice: a step adds
// at most 12 bytes, so at most one chunk completes per step, and it is read
// back at the end of that step, before its slot can be written again.
constexpr uint32_t kRingAt = 288;
constexpr uint32_t kCodeLds = 336;
constexpr uint32_t kCodeMtab = 256 * kCodeLds;         // the block's prefix-mask table (rc_root3.h)
constexpr uint32_t kCodeItab = kCodeMtab + 256;        // the block's D increment table

#if E2_PLAIN
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2)))
void rc_enc2_code(rc_batch_dev b, E2Params e)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint8_t* mtab = smem + kCodeMtab;
    const uint8_t* itab = smem + kCodeItab;
    if (threadIdx.x < 16) root3_mask_init(smem + kCodeMtab, threadIdx.x);
    if (threadIdx.x < 16) root3_inc_init(smem + kCodeItab, threadIdx.x);
    __syncthreads();
    const uint32_t l = threadIdx.x & 63;
    if (l >= e.act) return;
    const uint32_t idx = e.lo + blockIdx.x * 4 * e.act + (threadIdx.x >> 6) * e.act + l;
    if (idx >= e.hi) return;
    const uintptr_t base = reinterpret_cast<uintptr_t>(e.stream) + static_cast<size_t>(idx - e.lo) * e.slot_bytes;
    uint4 c0 = gload16(base);
    if (c0.x >= kSkipWide) return;                    // lane kernels / wide kernels / empty
    uint4 c1 = gload16(base + 16), c2 = gload16(base + 32);
    // (a wavefront's dummies are 1 KB contiguous: every store is one coalesced
    // 1-KB write to lines that stay in L2; a dummy per lane in its own line
    // was written back to HBM every ~7 steps, 0.7 GB per C2 launch)
    const uintptr_t dummy = reinterpret_cast<uintptr_t>(e.dummy) + ((blockIdx.x * 256u + threadIdx.x) & 65535u) * 16u;
    const uint32_t pkt = packet_of(e, idx);
    const uint32_t len = b.in_len[pkt];
    uint8_t* root = smem + threadIdx.x * kCodeLds;
    Ring o;
    o.r = root + kRingAt;
    o.lo = reinterpret_cast<uintptr_t>(b.out + b.out_off[pkt]);
    o.n = 0;
    o.cap = b.out_cap[pkt];
    o.ch = make_uint4(0u, 0u, 0u, 0u);
    o.ca = dummy;
    CodeState k;
    {
        Root R;
        root3_clear<true>(root, R);
    }
    k.rtot = 1 + 256; k.low = 0; k.range = ~0u;
    k.rrt = rcp64(k.rtot);
    __builtin_amdgcn_s_waitcnt(0);                    // settle the first chunks before the loop
    E2Prof pf;
#ifdef E2_PROF
    pf.t = __builtin_amdgcn_s_memtime();
    for (int k_ = 0; k_ < 8; ++k_) pf.acc[k_] = 0;
#endif
    // Six positions per iteration from three chunk registers; each register
    // is reloaded right after its two positions are prepared, with the chunk
    // three ahead, and is next read two register-steps later.  (Rotating one
    // set of registers instead would copy a load's result within the
    // iteration that issued it, i.e. wait for it.)  Each step prepares the
    // next position's codes.
    Pre p = prep(c0.x, c0.y, 0 < len);
    uintptr_t a = base + 48;
    for (uint32_t i = 0; any_lane(i < len && o.n <= o.cap); i += 6, a += 48) {
        code_step(k, o, root, mtab, itab, p, c0.z, c0.w, i + 1 < len, dummy, pf);
        code_step(k, o, root, mtab, itab, p, c1.x, c1.y, i + 2 < len, dummy, pf);
        c0 = gload16(a);
        code_step(k, o, root, mtab, itab, p, c1.z, c1.w, i + 3 < len, dummy, pf);
        code_step(k, o, root, mtab, itab, p, c2.x, c2.y, i + 4 < len, dummy, pf);
        c1 = gload16(a + 16);
        code_step(k, o, root, mtab, itab, p, c2.z, c2.w, i + 5 < len, dummy, pf);
        code_step(k, o, root, mtab, itab, p, c0.x, c0.y, i + 6 < len, dummy, pf);
        c2 = gload16(a + 32);
    }
    E2Q(7)
    E2Q_FLUSH
    ring_store(o);
    ring_chunk(o, o.n, dummy);                        // (nothing new: the next store goes to the dummy)
    // flush, compress.c:139-146
    bool ok = o.n <= o.cap;
    uint32_t low = k.low;
    while (any_lane(ok && low != 0)) {
        const bool more = ok && low != 0;
        const bool full = more && o.n >= o.cap;
        ok = ok && !full;
        const uint32_t n0 = o.n;
        ring_put(o, low, 1, more && !full);
        low = (more && !full) ? low << 8 : low;
        ring_chunk(o, n0, dummy);
        ring_store(o);
    }
    ring_finish(o, ok);
    b.out_len[pkt] = ok ? o.n : 0u;
}
#endif

// ---- pass 2, two wavefronts per SIMD: a helper and a coder per packet.
// The root model (order 0) evolves with the packet's symbols only, never with
// the coder's state, so it can run ahead of the coder.  A block holds 256
// packets in 8 wavefronts: wavefronts 4-7 (helpers) read the records, keep
// the root in LDS and queue per position its record words with the root's
// interval and total at that position (a 16-B entry); wavefronts 0-3
// (coders) prepare the sub-context intervals from the record words and run
// the range coder and the output ring.  The queue holds four parts of four
// positions per packet: the helpers fill two while the coders drain the
// other two, a block barrier between pairs.  With two wavefronts per SIMD the
// SIMD issues a vector instruction every 2 cycles instead of every 4 for one
// wavefront alone.
#ifdef E2_PROF
#define C2P_DECL unsigned long long c2t = __builtin_amdgcn_s_memtime(), c2w = 0, c2b = 0;
#define C2P_WORK { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); c2w += t_ - c2t; c2t = t_; __builtin_amdgcn_sched_barrier(0); }
#define C2P_WAIT { __builtin_amdgcn_sched_barrier(0); const unsigned long long t_ = __builtin_amdgcn_s_memtime(); c2b += t_ - c2t; c2t = t_; __builtin_amdgcn_sched_barrier(0); }
#define C2P_FLUSH(k) { if ((threadIdx.x & 63) == 0) { atomicAdd(&g_e2prof[k], c2w); atomicAdd(&g_e2prof[(k) + 1], c2b); } }
#else
#define C2P_DECL
#define C2P_WORK
#define C2P_WAIT
#define C2P_FLUSH(k)
#endif
constexpr uint32_t kQPart = 4;                                   // positions per part
constexpr uint32_t kQEntry = 16;                                 // bytes per queued position
constexpr uint32_t kQSlots = 4;                                  // parts in the queue: two filled while two drain
// The helpers' roots, transposed (rc_root3.h rofs): row g of lane l's root at
// kC2Row g + 16 l -- a lane's group read, count read and update and its D copy
// hit banks of its own.  (Before: 256 roots at a 304-B stride, where random
// groups put a wavefront's b128 reads on random banks: SQ_LDS_BANK_CONFLICT
// 140 M cycles per C2 launch.)
constexpr uint32_t kC2Row = 256 * 16;
constexpr uint32_t kC2Mtab = 18 * kC2Row;                        // helper roots, then tables
constexpr uint32_t kC2Itab = kC2Mtab + 256;
constexpr uint32_t kC2Ring = kC2Itab + 544;                      // (row 16 of the increment table: zeros); coder rings, 32 B per packet
// (rings at a 48-B stride: 16 lanes' 16-B ring chunks then cover the 64 banks
// once; at 32 B lanes l and l + 8 read the same four banks)
constexpr uint32_t kC2RingStride = 48;
constexpr uint32_t kC2Queue = kC2Ring + 256 * kC2RingStride;     // [kQSlots parts][kQPart][256 packets] entries
constexpr uint32_t kC2Max = kC2Queue + kQSlots * kQPart * 256 * kQEntry;   // the block's longest packet
constexpr uint32_t kC2Rcp = kC2Max + 16;                         // rcp64 of the sub-context totals
constexpr uint32_t kC2Lds = kC2Rcp + 8 * kRcpTab;
static_assert(kC2Lds <= 160 * 1024, "rc_enc2_code2's LDS");

// barrier for the block's LDS traffic only (a workgroup fence would also wait
// for the helpers' record loads and the coders' output stores)
DEV void lds_barrier()
{
    __builtin_amdgcn_s_waitcnt(0xC07F);                          // lgkmcnt(0), vmcnt/expcnt untouched
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_wave_barrier();
}

DEV uint8_t* q_entry(uint8_t* smem, uint32_t part, uint32_t j, uint32_t lane)
{
    return smem + kC2Queue + (((part & (kQSlots - 1)) * kQPart + j) * 256 + lane) * kQEntry;
}

DEV bool root_codes(uint32_t w0) { const uint32_t typ = w0 & 7; return typ <= 1 || typ == 3 || typ == 4; }

// helper: one position (the rare path: a part where some lane rescales)
DEV void help_pos(uint8_t* root, const uint8_t* mtab, const uint8_t* itab, uint32_t w0, uint32_t w1, bool en,
                  uint32_t& rtot, uint8_t* qe)
{
    if (en && (w0 & kRst)) {                          // compress.c:148-157, after the previous byte
        Root R;
        root3_clear<true, kC2Row>(root, R);
        rtot = 1 + 256;
    }
    const uint32_t v = w1 >> 24;
    uint32_t under0, cnt0;
    root3_lookup<kC2Row>(root, mtab, v, under0, cnt0);
    const RootAddPre ra = root3_add_read<kC2Row>(root, itab, v);
    const bool e0 = en && root_codes(w0);
    if (e0) root3_add_write<kC2Row>(root, v, cnt0, ra);
    uint32_t rt = e0 ? ((rtot + kRootDelta) & 0xFFFF) : rtot;
    const bool rs = e0 && (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || rt > kTotalLimit);
    if (any_lane(rs)) {
        if (rs) { Root R; rt = root3_rescale<true, kC2Row>(root, R); }
    }
    *reinterpret_cast<uint4*>(qe) = make_uint4(w0, w1, under0 | cnt0 << 16, rtot);
    rtot = rt;
}

// helper: a part of four positions with one round of LDS reads.  The four
// root lookups and the root's D copy are read before any of the part's
// updates; position j's interval is corrected for the updates of positions
// before it in the part (kRootDelta to under where their symbol is below,
// to the count where it is the same), and the updates are written after.
// A part where some lane would rescale the root is done position by position.
DEV void help_part(uint8_t* root, const uint8_t* mtab, const uint8_t* itab, const uint4& ca, const uint4& cb,
                   uint32_t i, uint32_t len, uint32_t& rtot, uint8_t* smem, uint32_t part, uint32_t lane)
{
    const uint32_t w0[4] = {ca.x, ca.z, cb.x, cb.z}, w1[4] = {ca.y, ca.w, cb.y, cb.w};
    uint32_t v[4], under[4], cnt[4], rt[4];
    bool e0[4];
    RootLk lk[4];
    uint4 inc[4][2];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        v[j] = w1[j] >> 24;
        e0[j] = i + j < len && root_codes(w0[j]);
        lk[j] = root3_lookup_read<kC2Row>(root, mtab, v[j]);
        const uint4* ip = reinterpret_cast<const uint4*>(itab + 32 * (e0[j] ? v[j] >> 4 : 16u));   // (row 16: no update)
        inc[j][0] = ip[0];
        inc[j][1] = ip[1];
    }
    uint4 d0 = *reinterpret_cast<const uint4*>(root + rdofs<kC2Row>(0));
    uint4 d1 = *reinterpret_cast<const uint4*>(root + rdofs<kC2Row>(1));
    bool rs = false;
    uint32_t t = rtot;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        rs = rs || (i + j < len && (w0[j] & kRst));     // a model reset in the part: position by position
        root3_lookup_sum(lk[j], v[j], under[j], cnt[j]);
#pragma unroll
        for (uint32_t q = 0; q < j; ++q) {
            under[j] += (e0[q] && v[q] < v[j]) ? kRootDelta : 0u;
            cnt[j] += (e0[q] && v[q] == v[j]) ? kRootDelta : 0u;
        }
        rt[j] = t;
        t = e0[j] ? ((t + kRootDelta) & 0xFFFF) : t;
        rs = rs || (e0[j] && (1 + cnt[j] > 0xFF - 2 * kRootDelta + 1 || t > kTotalLimit));
    }
    if (any_lane(rs)) {                               // (rare) position by position, rescales and resets included
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            help_pos(root, mtab, itab, w0[j], w1[j], i + j < len, rtot, q_entry(smem, part, j, lane));
        return;
    }
    // the part's updates: counts (in position order: a repeated symbol's
    // last write holds its final count) and the D copy
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        if (e0[j]) root[rofs<kC2Row>(v[j])] = static_cast<uint8_t>(cnt[j] + kRootDelta);
        d0.x += inc[j][0].x; d0.y += inc[j][0].y; d0.z += inc[j][0].z; d0.w += inc[j][0].w;
        d1.x += inc[j][1].x; d1.y += inc[j][1].y; d1.z += inc[j][1].z; d1.w += inc[j][1].w;
    }
    *reinterpret_cast<uint4*>(root + rdofs<kC2Row>(0)) = d0;
    *reinterpret_cast<uint4*>(root + rdofs<kC2Row>(1)) = d1;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
        *reinterpret_cast<uint4*>(q_entry(smem, part, j, lane)) = make_uint4(w0[j], w1[j], under[j] | cnt[j] << 16, rt[j]);
    rtot = t;
}

// coder: one position from its entry (record words; the root's under,
// count and total at the position) and its prepared sub-context codes p (the
// part's four prepared before its first code: their LDS reads and reciprocals
// are off the chain through low and range)
DEV void code_pos(CodeState& k, Ring& o, const uint4& qe, const Pre& p, double r0, uintptr_t dummy)
{
    const uint32_t n0 = o.n;
    code(k.low, k.range, p.u1, p.c1, p.r1, o);
    if (any_lane(p.e2)) code(k.low, k.range, p.u2, p.c2, p.r2, o);
    code(k.low, k.range, p.e0 ? 1 + (qe.z & 0xFFFF) : 0u, p.e0 ? 1 + (qe.z >> 16) : 1u, r0, o);
    ring_store(o);                                    // the chunk read back a step ago
    ring_chunk(o, n0, dummy);
}

#if E2_PLAIN
extern "C" __global__ __launch_bounds__(512)
void rc_enc2_code2(rc_batch_dev b, E2Params e)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint8_t* mtab = smem + kC2Mtab;
    const uint8_t* itab = smem + kC2Itab;
    uint32_t* bmax = reinterpret_cast<uint32_t*>(smem + kC2Max);
    double* rtab = reinterpret_cast<double*>(smem + kC2Rcp);
    if (threadIdx.x < kRcpTab) rtab[threadIdx.x] = rcp64(max(threadIdx.x, 1u));
    const bool helper = threadIdx.x >= 256;
    const uint32_t lane = threadIdx.x & 255;               // the block's packet
    if (threadIdx.x < 16) root3_mask_init(smem + kC2Mtab, threadIdx.x);
    if (threadIdx.x < 16) root3_inc_init(smem + kC2Itab, threadIdx.x);
    if (threadIdx.x == 16)
        reinterpret_cast<uint4*>(smem + kC2Itab)[32] = reinterpret_cast<uint4*>(smem + kC2Itab)[33] = make_uint4(0u, 0u, 0u, 0u);
    if (threadIdx.x == 0) *bmax = 0;
    const uint32_t idx = e.lo + blockIdx.x * 256 + lane;
    const uintptr_t base = reinterpret_cast<uintptr_t>(e.stream) + static_cast<size_t>(min(idx, e.hi - 1) - e.lo) * e.slot_bytes;
    const uintptr_t slot_last = base + e.slot_bytes - 16;
    const bool live = idx < e.hi && gload16(base).x < kSkipWide;   // (else: lane / wide kernels, empty, past the chunk)
    const uint32_t pkt = packet_of(e, min(idx, e.hi - 1));
    const uint32_t len = live ? b.in_len[pkt] : 0u;
    __syncthreads();
    if (helper) atomicMax(bmax, len);
    __syncthreads();
    const uint32_t parts = (*bmax + kQPart - 1) / kQPart;
    // The queue holds four parts: the helpers fill two while the coders drain
    // the other two, one block barrier per pair (one per part before round 5:
    // the coders then waited ~0.5 k cycles a part at the barrier)
    if (helper) {
        uint8_t* root = smem + lane * 16;
        {
            Root R;
            root3_clear<true, kC2Row>(root, R);
        }
        uint32_t rtot = 1 + 256;
        // records: a part is two 16-B chunks; two register sets (even and odd
        // parts), each reloaded right after its part is queued with the part
        // two ahead
        uint4 x0 = gload16(base), x1 = gload16(min(base + 16, slot_last));
        uint4 y0 = gload16(min(base + 32, slot_last)), y1 = gload16(min(base + 48, slot_last));
        __builtin_amdgcn_s_waitcnt(0);
        // parts 0 and 1 before the loop
        help_part(root, mtab, itab, x0, x1, 0, len, rtot, smem, 0, lane);
        x0 = gload16(min(base + 64, slot_last));
        x1 = gload16(min(base + 80, slot_last));
        help_part(root, mtab, itab, y0, y1, 4, len, rtot, smem, 1, lane);
        y0 = gload16(min(base + 96, slot_last));
        y1 = gload16(min(base + 112, slot_last));
        lds_barrier();
        C2P_DECL
        for (uint32_t s = 0; s < parts; s += 2) {
            // parts s + 2 (set x) and s + 3 (set y) while the coders drain s, s + 1
            help_part(root, mtab, itab, x0, x1, 4 * (s + 2), len, rtot, smem, s + 2, lane);
            x0 = gload16(min(base + 32 * (s + 4), slot_last));
            x1 = gload16(min(base + 32 * (s + 4) + 16, slot_last));
            help_part(root, mtab, itab, y0, y1, 4 * (s + 3), len, rtot, smem, s + 3, lane);
            y0 = gload16(min(base + 32 * (s + 5), slot_last));
            y1 = gload16(min(base + 32 * (s + 5) + 16, slot_last));
            C2P_WORK
            lds_barrier();
            C2P_WAIT
        }
        C2P_FLUSH(8)
        return;
    }
    // coder
    const uintptr_t dummy = reinterpret_cast<uintptr_t>(e.dummy) + ((blockIdx.x * 256u + lane) & 65535u) * 16u;
    Ring o;
    o.r = smem + kC2Ring + kC2RingStride * lane;
    o.lo = reinterpret_cast<uintptr_t>(b.out + (live ? b.out_off[pkt] : 0));
    o.n = 0;
    o.cap = live ? b.out_cap[pkt] : 0u;
    o.ch = make_uint4(0u, 0u, 0u, 0u);
    o.ca = dummy;
    CodeState k;
    k.rtot = 0; k.rrt = 0.0; k.low = 0; k.range = ~0u;
    lds_barrier();                                    // parts 0 and 1 queued
    C2P_DECL
    for (uint32_t s = 0; s < parts; ++s) {
        const uint4 q0 = *reinterpret_cast<const uint4*>(q_entry(smem, s, 0, lane));
        const uint4 q1 = *reinterpret_cast<const uint4*>(q_entry(smem, s, 1, lane));
        const uint4 q2 = *reinterpret_cast<const uint4*>(q_entry(smem, s, 2, lane));
        const uint4 q3 = *reinterpret_cast<const uint4*>(q_entry(smem, s, 3, lane));
        const uint32_t i = 4 * s;
        const Pre p0 = prep_tab(q0.x, q0.y, i < len, rtab), p1 = prep_tab(q1.x, q1.y, i + 1 < len, rtab);
        const Pre p2 = prep_tab(q2.x, q2.y, i + 2 < len, rtab), p3 = prep_tab(q3.x, q3.y, i + 3 < len, rtab);
        const double r00 = rcp64(p0.e0 ? q0.w : 1u), r01 = rcp64(p1.e0 ? q1.w : 1u);
        const double r02 = rcp64(p2.e0 ? q2.w : 1u), r03 = rcp64(p3.e0 ? q3.w : 1u);
        code_pos(k, o, q0, p0, r00, dummy);
        code_pos(k, o, q1, p1, r01, dummy);
        code_pos(k, o, q2, p2, r02, dummy);
        code_pos(k, o, q3, p3, r03, dummy);
        C2P_WORK
        if (s & 1) {
            lds_barrier();                            // (the helpers may overwrite parts s - 1, s now)
            C2P_WAIT
        }
    }
    if (parts & 1) lds_barrier();                     // (the helpers' last barrier)
    C2P_FLUSH(10)
    ring_store(o);
    ring_chunk(o, o.n, dummy);                        // (nothing new: the next store goes to the dummy)
    // flush, compress.c:139-146
    bool ok = live && o.n <= o.cap;
    uint32_t low = k.low;
    while (any_lane(ok && low != 0)) {
        const bool more = ok && low != 0;
        const bool full = more && o.n >= o.cap;
        ok = ok && !full;
        const uint32_t n0 = o.n;
        ring_put(o, low, 1, more && !full);
        low = (more && !full) ? low << 8 : low;
        ring_chunk(o, n0, dummy);
        ring_store(o);
    }
    ring_finish(o, ok);
    if (live) b.out_len[pkt] = ok ? o.n : 0u;
}
#endif

// ------------------------------------------------------------------ wide mode
//
// Packets with a bucket over kE2Bucket positions (low-entropy data: game
// state) can rescale their sub-contexts (compress.c:90-112, :313-314), which
// the closed form of pass 1 does not model.  rc_enc2_scan lists them (up to
// slot_len bytes) for these two kernels instead of the lane kernels:
//
//   rc_enc2_wscan (wavefront per listed packet, LDS): every position's
//     order-2 and order-1 codes as explicit (under, count, total) intervals.
//     Buckets of <= kE2Bucket positions: the closed form, one lane per bucket.
//     Bigger buckets, one at a time with the whole wavefront: the elements
//     sorted (stably) by a = x[i-2] into runs, one per order-2 context; runs of
//     <= kWideDense visits by the closed form (no rescale before a symbol's
//     127th visit), longer ones by a dense walk; then the bucket's order-1
//     visits (the elements order 2 did not find, in position order) the same
//     way.  A dense walk keeps the context's counts in an LDS table and takes
//     its visits 64 at a time, one per lane: a visit's count and under are the
//     table's plus twice the earlier lanes' visits of the same / smaller
//     symbols, its escapes and total the running ones plus the earlier lanes'
//     new symbols; the first lane whose visit rescales ends the round, and the
//     lanes after it are redone in the next round on the rescaled table.
//   rc_enc2_wcode (lane per listed packet): the root and the range coder over
//     the explicit records, as rc_enc2_code.
//
// Wide record of position i (16 B, in the wide stream, slot = list position):
//   x = underA | countA << 16    the order-2 code, (0, 1, 1) when none
//   y = totalA | v << 16
//   z = underB | countB << 16    the order-1 code
//   w = totalB | B coded << 16 | root codes << 17
// (an absent code is the identity interval, which the coder passes through).
// tests/proto/twopass.py (scan_wide, code_wide) restates both kernels.

constexpr uint32_t kWideDense = 32;             // runs longer than this take a dense walk

// Wide element word: pos (0-11) | v (12-19) | a | 256 (20-28, 0 for position 1).
// (12 bits of position: model segments of up to 4096 positions, rc_enc2_wscan_l.)
constexpr uint32_t kWPos = 4095u, kWV = 12, kWA = 20, kWHas = 256u << kWA;
DEV uint32_t wv_of(uint32_t w) { return (w >> kWV) & 255; }
DEV uint32_t wa_of(uint32_t w) { return (w >> kWA) & 255; }
// wide record, w word (half B): totalB | B coded << 16 | root codes << 17 |
// model reset before this position << 18 (compress.c:148-157, the first position
// of a segment after the first) | packet left to the lane kernels << 19 (position 0)
constexpr uint32_t kWRst = 1u << 18, kWLeft = 1u << 19;
[[maybe_unused]] constexpr uint32_t kWideLong = 4096;          // rc_enc2_wscan_l: segments of up to this many positions

// L: the longest packet of the launch (its positions); three sizes are built,
// 4096, 2048 and 1216.  The scan is latency-bound (LDS round trips and
// ballots on each wavefront's own path), so its speed is the number of
// resident wavefronts, which LDS sets: the 1216 layout is 8.7 KB, 18 per CU
// (17.7 KB and 9 per CU with 32-bit element words and buckets padded to 4).
// The element lists hold positions (u16); a word is rebuilt from the
// window's bytes where it is read (wword: one LDS read of x, which the
// window keeps for the whole packet).
//
// A big bucket's long runs: a run is the elements j of bucket p with one a =
// x[j-2]; an element j with a != p has x[j-2] != p, so j - 1 is no element of
// the bucket -- at most L / 2 elements have a != p, so at most L / 66 runs
// with a != p exceed kWideDense (32) visits, plus the run a = p.
template <uint32_t L>
constexpr uint32_t wide_runs_max() { return L / 64 + 2; }

template <uint32_t L>
struct WScanLdsT {
    uint8_t  x[16 + L + 16];          // the window's bytes at x[16 + mis + i]
    uint32_t cnt[256];                // bucket sizes, then fill pointers; a big bucket's run sizes by a
    uint32_t start[256];              // bucket starts; a big bucket's run starts, then run ends
    uint32_t tab[64];                 // dense walk: a round's updated counts (256 bytes); the lane-order probe
    uint16_t sw[L];                   // a big bucket's positions by a, then its order-1 visits (the small
                                      // buckets' 2-KB order-2 lane-mask table before)
    uint16_t e[L];                    // positions in bucket order, buckets back to back
    uint32_t f2bits[L / 32];          // positions found at order 2 (big buckets; every bucket in a
                                      // packet that can reach the model reset)
    uint32_t rootbits[L > kE2MaxLen ? L / 32 : 1];   // ... positions coded at the root (a packet that can reset)
    uint32_t runs[wide_runs_max<L>()];   // a big bucket's long runs (a keys)
    uint32_t nruns;
};
static_assert(sizeof(WScanLdsT<kWideSmallL>) <= 163840 / 18, "18 wide-scan wavefronts per CU");
static_assert(2 * kWideSmallL >= 256 * 8, "the order-2 lane-mask table inside sw");

// the element word of position pos (>= 1) from the window's bytes: pos |
// v = x[pos] | a = x[pos - 2] with its flag (position 1 has no a); p, the
// bucket key x[pos - 1], in bits 8-15 of b3
DEV uint32_t wword_b3(uint32_t pos, uint32_t b3)
{
    return pos | ((b3 >> 16) & 255) << kWV | (pos >= 2 ? ((b3 & 255) | 256u) << kWA : 0u);
}
DEV uint32_t wword(const uint8_t* x, uint32_t q0, uint32_t pos) { return wword_b3(pos, bytes3(x, q0 + pos)); }


// cnt[key] += 1 for every lane with ok: one LDS atomic per distinct key (its
// lowest lane adds the group's size).  RET: returns the lane's slot, the old
// value plus its rank among the lanes with its key (lane order).
template <bool RET>
DEV uint32_t group_add(uint32_t* cnt, uint32_t key, bool ok)
{
    const uint32_t t = lane_id();
    uint32_t lt;
    const uint64_t e = match8(key, __builtin_amdgcn_ballot_w64(ok), lt);
    const uint32_t ld = e ? static_cast<uint32_t>(__builtin_ctzll(e)) : t;
    uint32_t old = 0;
    if (ok && t == ld) {
        if (RET) old = atomicAdd(&cnt[key], popc64(e));
        else atomicAdd(&cnt[key], popc64(e));
    }
    if (!RET) return 0;
    return __shfl(old, static_cast<int>(ld), 64) + popc64(e & below_mask());
}

// the identity interval: a code that changes nothing
constexpr uint32_t kNoCodeLo = 1u << 16;        // under 0, count 1
constexpr uint32_t kNoCodeTot = 1u;
constexpr uint32_t kPadWord = 0xFFFFFFFFu;      // no element (a lane past WScanLds::e's elements)

// explicit interval of a sub-context visit from its statistics (t earlier
// visits, dist of them new, same / less earlier visits of this / a smaller
// symbol; no rescale): (lo = under | count << 16, total), or the identity
DEV uint2 closed_code(uint32_t t, uint32_t dist, uint32_t same, uint32_t less)
{
    const uint32_t esc = kSubEscDelta * dist, tot = esc + kSubDelta * t;
    if (same) return make_uint2((esc + kSubDelta * less) | (kSubDelta * same) << 16, tot);
    if (esc) return make_uint2(esc << 16, tot);
    return make_uint2(kNoCodeLo, kNoCodeTot);
}

DEV uint32_t akey_of(uint32_t w) { return (w & kWHas) ? (w >> kWA) & 511 : 1024u; }   // 1024: none (position 1)

// Buckets of <= kE2Bucket elements, whole buckets per round: a window of 64
// element slots starting at a bucket start takes every bucket that ends inside
// it (the next window starts at the first one that does not; big buckets are
// skipped).  With a bucket's elements side by side in the lanes, every
// statistic is a count of lanes (compress.c:159-199, :286-316): with
// match(key) = the lanes of a set whose key equals this lane's,
//   order 2: C = match(a) in my bucket, t2 = |C below me|, same2 / less2 from
//            match(v) in C, found2 = same2 > 0, dist2 = |C below me, not found2|;
//   order 1 (not found2): the bucket's lanes not found2, likewise.
// found2 of every lane is known at once (an earlier lane with the same a and
// v), so nothing runs lane after lane.
template <class S>
DEV void wide_small_buckets(S& s, uint32_t q0, uint32_t total, uint2* wrec, bool track)
{
    const uint32_t t = lane_id();
    const uint64_t below = below_mask();
    // lanes by order-2 key a: a 256-entry table of lane masks (in sw, free
    // until the big buckets), or-ed into and read back per window, then
    // cleared by the lanes that set it
    uint64_t* amask = reinterpret_cast<uint64_t*>(s.sw);
    *reinterpret_cast<uint4*>(&amask[4 * t]) = make_uint4(0u, 0u, 0u, 0u);
    *reinterpret_cast<uint4*>(&amask[4 * t + 2]) = make_uint4(0u, 0u, 0u, 0u);
    wave_sync();
#pragma unroll 1
    for (uint32_t W = 0; W < total;) {
        const uint32_t ei = W + t;
        const bool pad = ei >= total;
        uint32_t w = kPadWord, bs = 0, be = 0, p = 0;
        if (!pad) {
            const uint32_t pos = s.e[ei];
            const uint32_t b3 = bytes3(s.x, q0 + pos);
            w = wword_b3(pos, b3);
            p = (b3 >> 8) & 255;
            bs = s.start[p];
            be = s.cnt[p];
        }
        const bool small = !pad && be - bs <= kE2Bucket;
        const bool act = small && be <= W + 64;
        // the next window: the first lane not taken (a big bucket: past its end)
        const uint64_t nt = __builtin_amdgcn_ballot_w64(!pad && !act);
        uint32_t nextW = W + 64;
        if (nt) {
            const uint32_t ld = static_cast<uint32_t>(__builtin_ctzll(nt));
            const uint32_t lbs = __builtin_amdgcn_readlane(bs, ld), lbe = __builtin_amdgcn_readlane(be, ld);
            const uint32_t lsm = __builtin_amdgcn_readlane(small ? 1u : 0u, ld);
            nextW = lsm ? lbs : lbe;
            nextW = max(nextW, W + (ld ? 0u : 1u));  // (progress: a first lane never taken is a big bucket's)
        }
        const uint64_t am = __builtin_amdgcn_ballot_w64(act);
        if (am) {
            const uint32_t v = wv_of(w), a = wa_of(w);
            const bool has = (w & kWHas) != 0;
            const KeyBits kv = key_bits(v);
            // my bucket: its elements are lanes [bs - W, be - W) of the window
            // (buckets are contiguous in e[], and an active one lies inside it)
            const uint32_t blo = bs - W, bhi = be - W;
            const uint64_t mine = act ? ((bhi >= 64 ? ~0ull : (1ull << bhi) - 1ull) & ~((1ull << blo) - 1ull)) : 0ull;
            // my order-2 context: the lanes of my bucket with my a
            const bool ah = act && has;
            if (ah) atomicOr(reinterpret_cast<unsigned long long*>(&amask[a]), 1ull << t);
            wave_sync();
            const uint64_t am2 = ah ? amask[a] : 0ull;
            wave_sync();
            if (ah) amask[a] = 0ull;
            const uint64_t ctx2 = am2 & mine;
            // my bucket's lanes with my v, and with a smaller v: both contexts' counts
            uint64_t ltv;
            const uint64_t eqv = match_bits_lt(v, kv, mine, ltv);
            const uint64_t same2m = eqv & ctx2;
            const uint32_t less2 = popc64(ltv & ctx2 & below);
            const bool f2 = act && (same2m & below) != 0;
            const uint64_t F2 = __builtin_amdgcn_ballot_w64(f2);
            const uint32_t t2 = popc64(ctx2 & below), same2 = popc64(same2m & below);
            const uint32_t dist2 = popc64(ctx2 & below & ~F2);
            const uint64_t vis1 = mine & ~F2;                                      // the bucket's order-1 visitors
            const uint64_t same1m = eqv & vis1;
            const uint32_t less1 = popc64(ltv & vis1 & below);
            const bool f1 = act && !f2 && (same1m & below) != 0;
            const uint64_t F1 = __builtin_amdgcn_ballot_w64(f1);
            if (track && act) {                       // (the model reset's node count: wreset_after)
                const uint32_t pos = w & kWPos;
                if (f2) atomicOr(&s.f2bits[pos >> 5], 1u << (pos & 31));
                if (!f2 && !f1) atomicOr(&s.rootbits[pos >> 5], 1u << (pos & 31));
            }
            if (act) {
                const uint32_t pos = w & kWPos;
                const uint2 ca = closed_code(t2, dist2, same2, less2);
                wrec[2 * pos] = make_uint2(ca.x, ca.y | v << 16);
                if (f2) {
                    wrec[2 * pos + 1] = make_uint2(kNoCodeLo, kNoCodeTot);
                } else {
                    const uint2 cb = closed_code(popc64(vis1 & below), popc64(vis1 & below & ~F1),
                                                 popc64(same1m & below), less1);
                    const bool coded = cb.y != kNoCodeTot || cb.x != kNoCodeLo;
                    wrec[2 * pos + 1] = make_uint2(cb.x, cb.y | (coded ? 1u << 16 : 0u) | (f1 ? 0u : 1u << 17));
                }
            }
        }
        W = nextW;
    }
}

// A big bucket's short order-2 runs (<= kWideDense visits: no rescale) in
// windows of whole runs over their sorted words sw[0, ks) (short runs first),
// counted over lanes as in wide_small_buckets: record half A, and the
// position's order-2 hit bit.
template <class S>
DEV void wide_short_runs(S& s, uint32_t q0, uint32_t ks, const uint32_t* hist, const uint32_t* rend, uint2* wrec)
{
    const uint32_t t = lane_id();
    const uint64_t below = below_mask();
#pragma unroll 1
    for (uint32_t W = 0; W < ks;) {
        const uint32_t j = W + t;
        const bool in = j < ks;
        const uint32_t w = wword(s.x, q0, s.sw[in ? j : ks - 1]);
        const uint32_t a = wa_of(w), v = wv_of(w);
        const uint32_t re = rend[a], rs = re - hist[a];
        const bool act = in && re <= W + 64;
        const uint64_t nt = __builtin_amdgcn_ballot_w64(in && !act);
        const uint32_t nextW = nt ? __builtin_amdgcn_readlane(rs, static_cast<uint32_t>(__builtin_ctzll(nt))) : W + 64;
        uint32_t less;
        const KeyBits kv = key_bits(v);
        // my run (order-2 context): lanes [rs - W, re - W) of the window
        const uint32_t rlo = rs - W, rhi = re - W;
        const uint64_t ctx = act ? ((rhi >= 64 ? ~0ull : (1ull << rhi) - 1ull) & ~((1ull << rlo) - 1ull)) : 0ull;
        const uint64_t samem = match_bits(v, kv, ctx, less);
        const bool f2 = act && (samem & below) != 0;
        const uint64_t F2 = __builtin_amdgcn_ballot_w64(f2);
        if (act) {
            const uint32_t pos = w & kWPos;
            const uint2 c = closed_code(popc64(ctx & below), popc64(ctx & below & ~F2), popc64(samem & below), less);
            wrec[2 * pos] = make_uint2(c.x, c.y | v << 16);
            if (f2) {
                wrec[2 * pos + 1] = make_uint2(kNoCodeLo, kNoCodeTot);
                atomicOr(&s.f2bits[pos >> 5], 1u << (pos & 31));
            }
        }
        W = nextW;
    }
}

// bytes of x that are not zero, as 0xFF bytes
DEV uint32_t nonzero_bytes(uint32_t x)
{
    const uint32_t y = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;
    return ((y >> 7) & 0x01010101u) * 0xFFu;
}

// The dense walk of one context's visits (element words list[0..m), visit
// order), the whole wavefront, compress.c:286-316 with rescales (see the
// section header).  The context's 256 counts live in registers, four per
// lane (lane l: symbols 4l .. 4l+3), with the counts below each lane's four
// (a wave prefix sum); a visit reads its symbol's dword and prefix from the
// owning lane (ds_bpermute).  order2: record half A, a hit sets the
// position's order-2 hit bit and closes half B; else half B with the root
// flag.
template <class S>
DEV void wide_dense_walk(S& s, uint32_t q0, const uint16_t* list, uint32_t m, bool order2, uint2* wrec,
                         bool track = false)
{
    const uint32_t t = lane_id();
    uint32_t* tab = s.tab;
    uint8_t* sc = reinterpret_cast<uint8_t*>(tab);     // a round's final counts of its symbols (0: untouched)
    uint32_t tabr = 0, pre = 0;
    uint32_t esc = 0, tot = 0;                        // (wave-uniform)
    tab[t] = 0;
    wave_sync();
#pragma unroll 1
    for (uint32_t base = 0; base < m;) {
        const uint32_t j = base + t;
        const bool act = j < m;
        const uint32_t pos = list[act ? j : m - 1];
        const uint32_t v = s.x[q0 + pos];
        const uint32_t dw = __shfl(tabr, static_cast<int>(v >> 2), 64);
        const uint32_t pd = __shfl(pre, static_cast<int>(v >> 2), 64);
        const uint32_t sh = 8 * (v & 3);
        const uint32_t c0 = (dw >> sh) & 255;
        // lanes of this round with the same symbol; earlier ones with a smaller one
        uint32_t lt;
        const uint64_t m_mine = match8(v, __builtin_amdgcn_ballot_w64(act), lt);
        const uint32_t eq = popc64(m_mine & below_mask());
        const uint32_t c = c0 + kSubDelta * eq;
        const uint32_t under = pd + sad(dw & ((1u << sh) - 1u), 0u) + kSubDelta * lt;
        const bool isnew = act && c == 0;
        const uint64_t nm = __builtin_amdgcn_ballot_w64(isnew);
        const uint32_t nb = popc64(nm & below_mask());
        const uint32_t esc_l = esc + kSubEscDelta * nb;
        const uint32_t tot_l = tot + kSubDelta * t + kSubEscDelta * nb;
        const bool resc = act && (c > 0xFF - 2 * kSubDelta ||
                                  tot_l + kSubDelta + (isnew ? kSubEscDelta : 0u) > kTotalLimit);
        const uint64_t rm = __builtin_amdgcn_ballot_w64(resc);
        const uint32_t jstar = rm ? static_cast<uint32_t>(__builtin_ctzll(rm)) : 64u;
        const bool commit = act && t <= jstar;
        const bool hit = c != 0;
        uint2 code;
        if (hit) code = make_uint2((esc_l + under) | c << 16, tot_l);
        else if (esc_l) code = make_uint2(esc_l << 16, tot_l);
        else code = make_uint2(kNoCodeLo, kNoCodeTot);
        if (commit) {
            if (order2) {
                wrec[2 * pos] = make_uint2(code.x, code.y | v << 16);
                if (hit) {
                    wrec[2 * pos + 1] = make_uint2(kNoCodeLo, kNoCodeTot);
                    atomicOr(&s.f2bits[pos >> 5], 1u << (pos & 31));
                }
            } else {
                const bool coded = hit || esc_l != 0;
                wrec[2 * pos + 1] = make_uint2(code.x, code.y | (coded ? 1u << 16 : 0u) | (hit ? 0u : 1u << 17));
                if (track && !hit) atomicOr(&s.rootbits[pos >> 5], 1u << (pos & 31));
            }
        }
        // the table: the last committed visit of each symbol posts its count,
        // the owning lanes merge them
        const uint64_t cm = __builtin_amdgcn_ballot_w64(commit);
        const uint64_t later = t == 63 ? 0ull : (m_mine & cm) >> (t + 1);
        if (commit && later == 0) sc[v] = static_cast<uint8_t>(c + kSubDelta);
        wave_sync();
        const uint32_t nw = tab[t];
        tab[t] = 0;
        tabr = (tabr & ~nonzero_bytes(nw)) | nw;
        const uint32_t ncm = popc64(cm), nnew = popc64(nm & cm);
        esc += kSubEscDelta * nnew;
        tot += kSubDelta * ncm + kSubEscDelta * nnew;
        if (jstar < 64) {
            // rescale after visit jstar (compress.c:90-112): halve every count
            // (rounding up), escapes likewise, total = counts + escapes
            tabr = tabr - ((tabr >> 1) & 0x7F7F7F7Fu);
            esc -= esc >> 1;
        }
        const uint32_t bsum = sad(tabr, 0u);
        const uint32_t incl = wave_incl_scan(bsum);
        pre = incl - bsum;
        if (jstar < 64) {
            tot = __builtin_amdgcn_readlane(incl, 63) + esc;
            base += jstar + 1;
        } else {
            base += 64;
        }
    }
    wave_sync();
}

// a big bucket of a wide packet (> kE2Bucket elements, [bs, bs + k) in
// position order), the whole wavefront
template <uint32_t L>
DEV void wide_big_bucket(WScanLdsT<L>& s, uint32_t q0, uint32_t bs, uint32_t k, uint2* wrec, W2Prof& wp,
                         bool ordered, bool track)
{
    const uint32_t t = lane_id();
    uint32_t* hist = s.cnt;                                      // [256] run sizes by a
    uint32_t* rst = s.start;                                     // [256] run starts, then run ends
    uint32_t* runs = s.runs;
    uint32_t* nruns = &s.nruns;
    *reinterpret_cast<uint4*>(&hist[4 * t]) = make_uint4(0u, 0u, 0u, 0u);
    if (t == 0) *nruns = 0;
    wave_sync();
    // order 2: the elements' a (position 1 has none: its record half A is the identity)
#pragma unroll 1
    for (uint32_t q = 0; q < k; q += 64) {
        const bool ok0 = q + t < k;
        const uint32_t w = wword(s.x, q0, s.e[bs + (ok0 ? q + t : k - 1)]);
        const bool has = (w & kWHas) != 0;
        if (ok0 && has) atomicAdd(&hist[wa_of(w)], 1u);
        if (ok0 && !has) wrec[2 * (w & kWPos)] = make_uint2(kNoCodeLo, kNoCodeTot | (wv_of(w)) << 16);
    }
    wave_sync();
    uint32_t ks;
    {
        // run starts: the short runs first (sw[0, ks)), then the long ones
        const uint4 h = *reinterpret_cast<const uint4*>(&hist[4 * t]);
        const uint4 hs = make_uint4(h.x <= kWideDense ? h.x : 0u, h.y <= kWideDense ? h.y : 0u,
                                    h.z <= kWideDense ? h.z : 0u, h.w <= kWideDense ? h.w : 0u);
        const uint4 hl = make_uint4(h.x - hs.x, h.y - hs.y, h.z - hs.z, h.w - hs.w);
        const uint32_t ms = hs.x + hs.y + hs.z + hs.w, ml = hl.x + hl.y + hl.z + hl.w;
        const uint32_t is = wave_incl_scan(ms), il = wave_incl_scan(ml);
        ks = __builtin_amdgcn_readlane(is, 63);
        const uint32_t ss = is - ms, sl = ks + il - ml;
        *reinterpret_cast<uint4*>(&rst[4 * t]) =
            make_uint4(h.x <= kWideDense ? ss : sl,
                       h.y <= kWideDense ? ss + hs.x : sl + hl.x,
                       h.z <= kWideDense ? ss + hs.x + hs.y : sl + hl.x + hl.y,
                       h.w <= kWideDense ? ss + hs.x + hs.y + hs.z : sl + hl.x + hl.y + hl.z);
    }
    wave_sync();
    // stable scatter of the element words by a into sw (run starts become run ends)
#pragma unroll 1
    for (uint32_t q = 0; q < k; q += 64) {
        const bool ok0 = q + t < k;
        const uint32_t w = wword(s.x, q0, s.e[bs + (ok0 ? q + t : k - 1)]);
        const bool has = ok0 && (w & kWHas) != 0;
        uint32_t rk = 0;
        if (ordered) {
            if (has) rk = atomicAdd(&rst[wa_of(w)], 1u);     // (lane order: see wscan_main)
        } else {
            rk = group_add<true>(rst, wa_of(w), has);
        }
        if (has) s.sw[rk] = static_cast<uint16_t>(w & kWPos);
    }
    wave_sync();
    W2P(5)
    // short runs: the closed form, element-parallel; long runs: dense walks
    wide_short_runs(s, q0, ks, hist, rst, wrec);
#pragma unroll 1
    for (uint32_t r = 0; r < 4; ++r) {
        const uint32_t a = 4 * t + r;
        if (hist[a] > kWideDense) runs[min(atomicAdd(nruns, 1u), wide_runs_max<L>() - 1)] = a;   // (bound: WScanLdsT)
    }
    wave_sync();
    W2P(6)
    const uint32_t nr = *nruns;
#pragma unroll 1
    for (uint32_t r = 0; r < nr; ++r) {
        const uint32_t a = runs[r];
        const uint32_t len = hist[a], st = rst[a] - len;
        wide_dense_walk(s, q0, s.sw + st, len, true, wrec);
    }
    wave_sync();
    W2P(7)
    // order 1: the elements order 2 did not find, in position order (a dense walk)
    uint32_t m1 = 0;
#pragma unroll 1
    for (uint32_t q = 0; q < k; q += 64) {
        const bool ok0 = q + t < k;
        const uint32_t pos = s.e[bs + (ok0 ? q + t : k - 1)];
        const bool vis = ok0 && !bit_at(s.f2bits, pos);
        const uint64_t vm = __builtin_amdgcn_ballot_w64(vis);
        if (vis) s.sw[m1 + popc64(vm & below_mask())] = static_cast<uint16_t>(pos);
        m1 += popc64(vm);
    }
    wave_sync();
    W2P(8)
    wide_dense_walk(s, q0, s.sw, m1, false, wrec, track);
    wave_sync();
    W2P(9)
}

// The wide scan's next packet, fetched while the current one is walked: its
// length, alignment and 16-B chunks (list, order, lengths and offsets through
// scalar loads; the loads are issued on every path, as in scan_prefetch).
struct WPf {
    uint32_t n, mis;
    uint4 r0, r1;
};

DEV WPf wide_prefetch(const rc_batch_dev& b, const E2Params& e, const WRegs& w, uint32_t d)
{
    WPf f;
    f.n = 0; f.mis = 0;
    uintptr_t a0 = reinterpret_cast<uintptr_t>(b.in) & ~static_cast<uintptr_t>(15), a1 = a0;
    if (d < w.pre[RC_WSHARDS]) {
        const uint32_t q = wq_of(e, w, d);
        const uint32_t idx = const_load(e.wlist, q);
        const uint32_t pkt = (e.order && !const_load(e.bins, RC_LEN_BINS)) ? const_load(e.order, idx) : idx;
        f.n = const_load(b.in_len, pkt);
        const uintptr_t src = reinterpret_cast<uintptr_t>(b.in + const_load(b.in_off, pkt));
        const uintptr_t a16 = src & ~static_cast<uintptr_t>(15);
        f.mis = static_cast<uint32_t>(src & 15);
        const uint32_t last = (f.mis + f.n - 1) >> 4;
        a0 = a16 + 16 * min(threadIdx.x, last);
        a1 = a16 + 16 * min(threadIdx.x + kScanThreads, last);
    }
    f.r0 = gload16(a0);
    f.r1 = gload16(a1);
    return f;
}

// The nodes compress.c creates at each position of a wide window scanned as
// a model segment (as reset_after for the narrow scan, compress.c:68-88 via
// :286-337): position 0 the root's; a position coded at the root creates the
// root's node at its byte's first root visit, its order-1 node (position >= 1)
// and its order-2 node (>= 2); an order-1 hit its order-2 node (>= 2); an
// order-2 hit none.  The walks' f2bits / rootbits say which.  Returns the
// window position after whose byte the count reaches 4094 (compress.c:148-157),
// or n.  After the walks; s.sw and s.cnt are reused.
template <uint32_t L, class S>
DEV uint32_t wreset_after(S& s, uint32_t q0, uint32_t n, uint32_t total, uint32_t x0, uint32_t t)
{
    uint8_t* inc = reinterpret_cast<uint8_t*>(s.sw);     // per position: nodes | 0x80 = root visit
    uint32_t* first = s.cnt;                             // the first root visit per byte value
    *reinterpret_cast<uint4*>(&first[4 * t]) = make_uint4(~0u, ~0u, ~0u, ~0u);
    wave_sync();
    if (t == 0) { first[x0] = 0u; inc[0] = 1; }
#pragma unroll 1
    for (uint32_t k = t; k < total; k += kScanThreads) {
        const uint32_t pos = s.e[k];
        const uint32_t v = s.x[q0 + pos];
        const bool rv = bit_at(s.rootbits, pos), f2 = bit_at(s.f2bits, pos);
        const uint32_t c = rv ? (pos >= 1 ? 1u : 0u) + (pos >= 2 ? 1u : 0u) : (f2 ? 0u : (pos >= 2 ? 1u : 0u));
        inc[pos] = static_cast<uint8_t>(c | (rv ? 0x80u : 0u));
        if (rv) atomicMin(&first[v], pos);
    }
    wave_sync();
#pragma unroll 1
    for (uint32_t k = t; k < total; k += kScanThreads) {
        const uint32_t pos = s.e[k];
        if (bit_at(s.rootbits, pos) && first[s.x[q0 + pos]] == pos) inc[pos] = static_cast<uint8_t>(inc[pos] + 1);
    }
    wave_sync();
    // positions C t .. C t + C - 1: their sum, the prefix over the lanes, the first crossing
    constexpr uint32_t C = (L + kScanThreads - 1) / kScanThreads;
    uint32_t sum = 0;
#pragma unroll 8
    for (uint32_t q = 0; q < C; ++q) {
        const uint32_t pos = C * t + q;
        sum += pos < n ? (inc[pos] & 0x7Fu) : 0u;
    }
    uint32_t acc = 1 + wave_incl_scan(sum) - sum;        // nodes before position C t (the root: 1)
    uint32_t hit = n;
    if (acc + sum >= kMaxNodesE2) {
#pragma unroll 1
        for (uint32_t q = 0; q < C; ++q) {
            const uint32_t pos = C * t + q;
            if (pos >= n) break;
            acc += inc[pos] & 0x7Fu;
            if (acc >= kMaxNodesE2) { hit = pos; break; }
        }
    }
    const uint64_t m = __builtin_amdgcn_ballot_w64(hit < n);
    const uint32_t r = m ? __builtin_amdgcn_readlane(hit, static_cast<uint32_t>(__builtin_ctzll(m))) : n;
    wave_sync();
    return r;
}

// A listed packet is taken in windows (as scan_main's): each window is a
// model segment scanned as a packet of its own, up to L positions; when the
// packet can reach compress.c's reset (> 1919 bytes) the nodes its positions
// create give the byte after which the model resets, and the next window
// starts after it, its position-0 record flagged kWRst (the code pass clears
// its root there).  A segment longer than the LDS layout holds (L positions)
// leaves the packet to the lane kernels (kWLeft in its first record).
template <uint32_t L>
DEV void wscan_main(const rc_batch_dev& b, const E2Params& e, WScanLdsT<L>& s)
{
    const uint32_t t = threadIdx.x;
    const WRegs wr = wregs(e);                        // the live list positions: d < nw
    const uint32_t nw = wr.pre[RC_WSHARDS];
    if (blockIdx.x >= nw) return;                     // (no packet for this workgroup: no probe, no prefetch --
                                                      // a batch with no wide packet, C2, launches the grid for nothing)
    // The stable scatters (elements into buckets in position order, a big
    // bucket's elements into runs) take one LDS atomic per lane where
    // same-address atomics apply in lane order (as in scan_main: gfx950,
    // checked by the probe once per wavefront), else the key-match ranks.
#if defined(__gfx950__)
    const bool ordered = lane_order_probe(s.tab, t);
#else
    const bool ordered = false;
#endif
    W2Prof wp;
    W2P_INIT
    WPf pf = wide_prefetch(b, e, wr, blockIdx.x);
    for (uint32_t d = blockIdx.x; d < nw; d += gridDim.x) {
        const WPf cur = pf;
        const uint32_t q = wq_of(e, wr, d);           // the list position
        const uint32_t len = cur.n;                   // (1 <= len <= slot_len: rc_enc2_scan)
        uint2* wrec0 = reinterpret_cast<uint2*>(e.wide + static_cast<size_t>(q) * e.wslot_bytes);
        const bool track = L > kE2MaxLen && len > kE2MaxLen;   // (wave-uniform) the model can reset
        uint32_t s0 = 0, mis = cur.mis;
        uintptr_t src0 = 0;
        if (len + mis > 2048 || track) {
            const uint32_t idx = const_load(e.wlist, q);
            src0 = reinterpret_cast<uintptr_t>(b.in + const_load(b.in_off, packet_of(e, idx)));
        }
        bool fetched = false;
#pragma unroll 1
        for (;;) {
        const uint32_t n = min(len - s0, L);         // the window: positions s0 .. s0 + n - 1
        uint2* wrec = wrec0 + 2 * s0;
        *reinterpret_cast<uint4*>(&s.cnt[4 * t]) = make_uint4(0u, 0u, 0u, 0u);
        for (uint32_t k = t; k < L / 32; k += kScanThreads) {
            s.f2bits[k] = 0u;
            if (L > kE2MaxLen) s.rootbits[k] = 0u;
        }
        if (s0 == 0) {
            *reinterpret_cast<uint4*>(s.x + 16 + 16 * t) = cur.r0;
            // (x holds L + 16 bytes past its first 16: chunks up to L / 16, the last a
            // packet of <= L bytes at any alignment needs; later ones repeat it)
            if (L >= 2048 || 16 * (t + kScanThreads) <= L)
                *reinterpret_cast<uint4*>(s.x + 16 + 16 * (t + kScanThreads)) = cur.r1;
        }
        if (s0 > 0 || n + mis > 2048) {
            // the window's bytes past the prefetched 2 KB (or a later window's): aligned 16-B chunks
            const uintptr_t a16 = (src0 + s0) & ~static_cast<uintptr_t>(15);
            const uint32_t last = (mis + n - 1) >> 4;
#pragma unroll 1
            for (uint32_t c = (s0 > 0 ? 0u : 2u * kScanThreads) + t; c <= last; c += kScanThreads)
                *reinterpret_cast<uint4*>(s.x + 16 + 16 * c) = gload16(a16 + 16 * c);
        }
        wave_sync();
        W2P(0)
        const uint32_t q0 = 16 + mis;
        // bucket sizes
#pragma unroll 1
        for (uint32_t i = 1 + t; i < n + t; i += kScanThreads) {
            const bool ok = i < n;
            const uint32_t p = s.x[q0 + (ok ? i : 1) - 1];
            if (ok) atomicAdd(&s.cnt[p], 1u);          // (a count: the order of same-address adds does not matter)
        }
        wave_sync();
        W2P(1)
        // bucket starts, buckets back to back (total = n - 1 elements)
        const uint4 c4 = *reinterpret_cast<const uint4*>(&s.cnt[4 * t]);
        const uint32_t mine = c4.x + c4.y + c4.z + c4.w;
        const uint32_t incl = wave_incl_scan(mine);
        const uint32_t st = incl - mine;
        const uint32_t total = __builtin_amdgcn_readlane(incl, 63);
        const uint4 s4 = make_uint4(st, st + c4.x, st + c4.x + c4.y, st + c4.x + c4.y + c4.z);
        *reinterpret_cast<uint4*>(&s.start[4 * t]) = s4;
        *reinterpret_cast<uint4*>(&s.cnt[4 * t]) = s4;
        wave_sync();
        W2P(2)
        // scatter into buckets, position order (two positions per lane and iteration)
#pragma unroll 1
        for (uint32_t i = 1 + t; i < n + t; i += 2 * kScanThreads) {
            uint32_t w[2], p[2];
            bool ok[2];
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                const uint32_t i2 = i + h * kScanThreads;
                ok[h] = i2 < n;
                w[h] = ok[h] ? i2 : 1u;                    // (the position)
                p[h] = s.x[q0 + w[h] - 1];
            }
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                uint32_t slot = 0;
                if (ordered) {
                    if (ok[h]) slot = atomicAdd(&s.cnt[p[h]], 1u);
                } else {
                    slot = group_add<true>(s.cnt, p[h], ok[h]);
                }
                if (ok[h]) s.e[slot] = static_cast<uint16_t>(w[h]);
            }
        }
        const uint32_t x0 = s.x[q0];
        wave_sync();
        if (!fetched) pf = wide_prefetch(b, e, wr, d + gridDim.x);  // (the next packet, while this one is walked)
        fetched = true;
        W2P(3)
        // buckets of <= kE2Bucket elements, whole buckets per round
        wide_small_buckets(s, q0, total, wrec, track);
        wave_sync();
        W2P(4)
        // big ones: the wavefront, one at a time (their extents from registers:
        // a big bucket's walk reuses cnt and start)
        uint32_t bigm = 0;
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) bigm |= pick4(r, c4) > kE2Bucket ? 1u << r : 0u;
        uint64_t bl = __builtin_amdgcn_ballot_w64(bigm != 0);
        while (bl != 0) {
            const uint32_t ld = static_cast<uint32_t>(__builtin_ctzll(bl));
            const uint32_t bm = __builtin_amdgcn_readlane(bigm, ld);
#pragma unroll 1
            for (uint32_t r = 0; r < 4; ++r) {
                if (!((bm >> r) & 1u)) continue;
                const uint32_t bs = __builtin_amdgcn_readlane(pick4(r, s4), ld);
                const uint32_t bn = __builtin_amdgcn_readlane(pick4(r, c4), ld);
                wide_big_bucket(s, q0, bs, bn, wrec, wp, ordered, track);
            }
            bl &= bl - 1;
        }
        if (t == 0) {                                 // position 0: root only (after a reset: the root cleared)
            wrec[0] = make_uint2(kNoCodeLo, kNoCodeTot | x0 << 16);
            wrec[1] = make_uint2(kNoCodeLo, kNoCodeTot | 1u << 17 | (s0 ? kWRst : 0u));
        }
        wave_sync();
        W2P(10)
        if (!track) break;                            // (no reset: <= 2 * 1918 + 256 nodes, compress.c:150)
        const uint32_t r = wreset_after<L>(s, q0, n, total, x0, t);
        if (r >= n) {                                 // no reset in the window
            if (s0 + n < len) {
                // a model segment longer than the window: the lane kernels take the packet
                if (t == 0) {
                    wrec0[1] = make_uint2(kNoCodeLo, kNoCodeTot | 1u << 17 | kWLeft);
                    e.list[atomicAdd(e.count, 1u)] = packet_of(e, const_load(e.wlist, q));
                }
            }
            break;
        }
        s0 += r + 1;
        if (s0 >= len) break;                         // (the reset after the last byte changes nothing)
        mis = static_cast<uint32_t>((src0 + s0) & 15);
        wave_sync();
        }
    }
    W2P_FLUSH
}

#if E2_WIDE
extern "C" __global__ __launch_bounds__(kScanThreads)
void rc_enc2_wscan(rc_batch_dev b, E2Params e)
{
    __shared__ __attribute__((aligned(16))) WScanLdsT<2048> s;
    wscan_main<2048>(b, e, s);
}

// the same for launches whose packets are at most kWideSmallL bytes
// (five wavefronts per SIMD: 96 VGPRs, a few spilled; with 8.7 KB of LDS 18
// fit per CU instead of the 16 that 105 VGPRs allowed -- 1.166 -> 1.147 ms on
// C3, profiles/r6/s7f_wscan_w5_c3.txt)
#ifndef WSCAN_S_ATTR
#define WSCAN_S_ATTR __attribute__((amdgpu_waves_per_eu(5)))
#endif
extern "C" __global__ __launch_bounds__(kScanThreads) WSCAN_S_ATTR
void rc_enc2_wscan_s(rc_batch_dev b, E2Params e)
{
    __shared__ __attribute__((aligned(16))) WScanLdsT<kWideSmallL> s;
    wscan_main<kWideSmallL>(b, e, s);
}

// ... and for launches with packets over 2048 bytes: model segments of up to
// kWideLong positions (43 KB of LDS: 3 wavefronts per CU)
extern "C" __global__ __launch_bounds__(kScanThreads)
void rc_enc2_wscan_l(rc_batch_dev b, E2Params e)
{
    __shared__ __attribute__((aligned(16))) WScanLdsT<kWideLong> s;
    wscan_main<kWideLong>(b, e, s);
}

// ---- wide code pass: rc_enc2_code over explicit records
DEV Pre prep_wide(const uint4& r, bool en)
{
    Pre p;
    p.u1 = en ? r.x & 0xFFFF : 0u;
    p.c1 = en ? r.x >> 16 : 1u;
    p.r1 = rcp64(en ? r.y & 0xFFFF : 1u);
    p.v = (r.y >> 16) & 255;
    p.e2 = en && ((r.w >> 16) & 1u);
    p.e0 = en && ((r.w >> 17) & 1u);
    p.u2 = p.e2 ? r.z & 0xFFFF : 0u;
    p.c2 = p.e2 ? r.z >> 16 : 1u;
    p.r2 = rcp64(p.e2 ? r.w & 0xFFFF : 1u);
    p.rst = en && (r.w & kWRst) != 0;
    return p;
}

// code_step with the next position's wide record.  RST: the batch has packets
// that can reach the model reset (compress.c:148-157): a position flagged
// kWRst starts a new segment, its root cleared first.
template <bool RST>
DEV void wcode_step(CodeState& k, Ring& o, uint8_t* root, const uint8_t* mtab, const uint8_t* itab, Pre& p,
                    const uint4& nx, bool enn, uintptr_t dummy)
{
    if (RST && any_lane(p.rst)) {
        if (p.rst) {
            Root R;
            root3_clear<true>(root, R);
            k.rtot = 1 + 256;
            k.rrt = rcp64(k.rtot);
        }
    }
    const uint32_t n0 = o.n;
    uint32_t under0, cnt0;
    root3_lookup(root, mtab, p.v, under0, cnt0);
    const RootAddPre ra = root3_add_read(root, itab, p.v);
    const Pre q = prep_wide(nx, enn);
    const uint32_t rtot1 = p.e0 ? ((k.rtot + kRootDelta) & 0xFFFF) : k.rtot;
    double rrt1 = rcp64(rtot1);
    code(k.low, k.range, p.u1, p.c1, p.r1, o);
    if (any_lane(p.e2)) code(k.low, k.range, p.u2, p.c2, p.r2, o);
    // (the root's code is the identity for the lanes without e0: skipped when
    // no lane of the wavefront has one)
    if (any_lane(p.e0)) code(k.low, k.range, p.e0 ? 1 + under0 : 0u, p.e0 ? 1 + cnt0 : 1u, p.e0 ? k.rrt : 1.0, o);
    if (p.e0) root3_add_write(root, p.v, cnt0, ra);
    k.rtot = rtot1;
    const bool rs0 = p.e0 && (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || k.rtot > kTotalLimit);
    if (any_lane(rs0)) {
        if (rs0) { Root R; k.rtot = root3_rescale<true>(root, R); }
        rrt1 = rcp64(k.rtot);
    }
    k.rrt = rrt1;
    ring_store(o);
    ring_chunk(o, n0, dummy);
    p = q;
}

template <bool RST>
DEV void wcode_main(const rc_batch_dev& b, const E2Params& e)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint8_t* mtab = smem + kCodeMtab;
    const uint8_t* itab = smem + kCodeItab;
    if (threadIdx.x < 16) root3_mask_init(smem + kCodeMtab, threadIdx.x);
    if (threadIdx.x < 16) root3_inc_init(smem + kCodeItab, threadIdx.x);
    __syncthreads();
    const uint32_t q = blockIdx.x * 256 + threadIdx.x;
    if (!wq_any(e, blockIdx.x * 256, 256)) return;    // (the whole block)
    const bool live = wq_live(e, q);
    const uint32_t pkt = live ? packet_of(e, e.wlist[q]) : 0u;
    const uint32_t len0 = live ? b.in_len[pkt] : 0u;
    const uintptr_t base = reinterpret_cast<uintptr_t>(e.wide) + static_cast<size_t>(live ? q : 0u) * e.wslot_bytes;
    const uintptr_t dummy = reinterpret_cast<uintptr_t>(e.dummy) + ((blockIdx.x * 256u + threadIdx.x) & 65535u) * 16u;
    uint8_t* root = smem + threadIdx.x * kCodeLds;
    Ring o;
    o.r = root + kRingAt;
    o.lo = reinterpret_cast<uintptr_t>(b.out + (live ? b.out_off[pkt] : 0));
    o.n = 0;
    o.cap = live ? b.out_cap[pkt] : 0u;
    o.ch = make_uint4(0u, 0u, 0u, 0u);
    o.ca = dummy;
    CodeState k;
    {
        Root R;
        root3_clear<true>(root, R);
    }
    k.rtot = 1 + 256; k.low = 0; k.range = ~0u;
    k.rrt = rcp64(k.rtot);
    // one 16-B record per position; four registers, each reloaded (four
    // positions ahead) right after its position is prepared
    uint4 c0 = gload16(base), c1 = gload16(base + 16), c2 = gload16(base + 32), c3 = gload16(base + 48);
    __builtin_amdgcn_s_waitcnt(0);
    // a packet the wide scan left to the lane kernels (a model segment past its LDS): nothing here
    const bool left = RST && live && (c0.w & kWLeft) != 0;
    const uint32_t len = left ? 0u : len0;
    Pre p = prep_wide(c0, 0 < len);
    c0 = gload16(base + 64);
    uintptr_t a = base + 80;
    for (uint32_t i = 0; any_lane(i < len && o.n <= o.cap); i += 4, a += 64) {
        wcode_step<RST>(k, o, root, mtab, itab, p, c1, i + 1 < len, dummy);
        c1 = gload16(a);
        wcode_step<RST>(k, o, root, mtab, itab, p, c2, i + 2 < len, dummy);
        c2 = gload16(a + 16);
        wcode_step<RST>(k, o, root, mtab, itab, p, c3, i + 3 < len, dummy);
        c3 = gload16(a + 32);
        wcode_step<RST>(k, o, root, mtab, itab, p, c0, i + 4 < len, dummy);
        c0 = gload16(a + 48);
    }
    ring_store(o);
    ring_chunk(o, o.n, dummy);
    bool ok = live && !left && o.n <= o.cap;
    uint32_t low = k.low;
    while (any_lane(ok && low != 0)) {
        const bool more = ok && low != 0;
        const bool full = more && o.n >= o.cap;
        ok = ok && !full;
        const uint32_t n0 = o.n;
        ring_put(o, low, 1, more && !full);
        low = (more && !full) ? low << 8 : low;
        ring_chunk(o, n0, dummy);
        ring_store(o);
    }
    ring_finish(o, ok);
    if (live && !left) b.out_len[pkt] = ok ? o.n : 0u;
}

extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2)))
void rc_enc2_wcode(rc_batch_dev b, E2Params e) { wcode_main<false>(b, e); }

// The wide code pass on a helper and a coder wavefront per packet, as
// rc_enc2_code2 (one wavefront per packet: rc_enc2_wcode, 28 % slower on the
// narrow records, 0.853 against 0.614 ms on C2): the helpers keep the root and
// queue each position's root interval and total, the coders read the explicit
// records themselves (two parts ahead; the helpers read them first, so they
// come from the L2) and run the range coder.  Packets without model resets
// (slot_len <= kE2MaxLen); rc_enc2_wcode_r takes the others.
//
// help_part's record words for two wide records: type 1 where the root codes
// the byte, 2 where it does not (root_codes), no reset; the byte in w1
DEV uint4 wide_as_plain(const uint4& ra, const uint4& rb)
{
    return make_uint4(((ra.w >> 17) & 1u) ? 1u : 2u, ((ra.y >> 16) & 255u) << 24,
                      ((rb.w >> 17) & 1u) ? 1u : 2u, ((rb.y >> 16) & 255u) << 24);
}

// a part's four wide records (clamped to the slot: parts past the packet read its end)
DEV void wload4(uintptr_t a, uintptr_t last, uint4* r)
{
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) r[j] = gload16(min(a + 16 * j, last));
}

extern "C" __global__ __launch_bounds__(512)
void rc_enc2_wcode2(rc_batch_dev b, E2Params e)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint8_t* mtab = smem + kC2Mtab;
    const uint8_t* itab = smem + kC2Itab;
    uint32_t* bmax = reinterpret_cast<uint32_t*>(smem + kC2Max);
    if (!wq_any(e, blockIdx.x * 256, 256)) return;    // (the whole block)
    const bool helper = threadIdx.x >= 256;
    const uint32_t lane = threadIdx.x & 255;
    if (threadIdx.x < 16) root3_mask_init(smem + kC2Mtab, threadIdx.x);
    if (threadIdx.x < 16) root3_inc_init(smem + kC2Itab, threadIdx.x);
    if (threadIdx.x == 16)
        reinterpret_cast<uint4*>(smem + kC2Itab)[32] = reinterpret_cast<uint4*>(smem + kC2Itab)[33] = make_uint4(0u, 0u, 0u, 0u);
    if (threadIdx.x == 0) *bmax = 0;
    const uint32_t q = blockIdx.x * 256 + lane;
    const bool live = wq_live(e, q);
    const uint32_t pkt = live ? packet_of(e, e.wlist[q]) : 0u;
    const uint32_t len = live ? b.in_len[pkt] : 0u;
    const uintptr_t base = reinterpret_cast<uintptr_t>(e.wide) + static_cast<size_t>(live ? q : 0u) * e.wslot_bytes;
    const uintptr_t last = base + e.wslot_bytes - 16;
    __syncthreads();
    if (helper) atomicMax(bmax, len);
    __syncthreads();
    const uint32_t parts = (*bmax + kQPart - 1) / kQPart;
    if (helper) {
        uint8_t* root = smem + lane * 16;
        {
            Root R;
            root3_clear<true, kC2Row>(root, R);
        }
        uint32_t rtot = 1 + 256;
        uint4 x[4], y[4];                             // even and odd parts' records
        wload4(base, last, x);
        wload4(base + 64, last, y);
        __builtin_amdgcn_s_waitcnt(0);
        help_part(root, mtab, itab, wide_as_plain(x[0], x[1]), wide_as_plain(x[2], x[3]), 0, len, rtot, smem, 0, lane);
        wload4(base + 128, last, x);
        help_part(root, mtab, itab, wide_as_plain(y[0], y[1]), wide_as_plain(y[2], y[3]), 4, len, rtot, smem, 1, lane);
        wload4(base + 192, last, y);
        lds_barrier();
        C2P_DECL
        for (uint32_t s = 0; s < parts; s += 2) {
            help_part(root, mtab, itab, wide_as_plain(x[0], x[1]), wide_as_plain(x[2], x[3]), 4 * (s + 2), len, rtot,
                      smem, s + 2, lane);
            wload4(base + 64 * (s + 4), last, x);
            help_part(root, mtab, itab, wide_as_plain(y[0], y[1]), wide_as_plain(y[2], y[3]), 4 * (s + 3), len, rtot,
                      smem, s + 3, lane);
            wload4(base + 64 * (s + 5), last, y);
            C2P_WORK
            lds_barrier();
            C2P_WAIT
        }
        C2P_FLUSH(8)
        return;
    }
    // coder
    const uintptr_t dummy = reinterpret_cast<uintptr_t>(e.dummy) + ((blockIdx.x * 256u + lane) & 65535u) * 16u;
    Ring o;
    o.r = smem + kC2Ring + kC2RingStride * lane;
    o.lo = reinterpret_cast<uintptr_t>(b.out + (live ? b.out_off[pkt] : 0));
    o.n = 0;
    o.cap = live ? b.out_cap[pkt] : 0u;
    o.ch = make_uint4(0u, 0u, 0u, 0u);
    o.ca = dummy;
    CodeState k;
    k.rtot = 0; k.rrt = 0.0; k.low = 0; k.range = ~0u;
    uint4 x[4], y[4];                                 // this pair of parts' records
    wload4(base, last, x);
    wload4(base + 64, last, y);
    lds_barrier();                                    // parts 0 and 1 queued
    C2P_DECL
    for (uint32_t s = 0; s < parts; s += 2) {
#pragma unroll
        for (uint32_t h = 0; h < 2; ++h) {
            uint4* r = h ? y : x;
            const uint32_t i = 4 * (s + h);
            Pre p[4];
            double r0[4];
            uint4 qe[4];
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) {
                qe[j] = *reinterpret_cast<const uint4*>(q_entry(smem, s + h, j, lane));
                p[j] = prep_wide(r[j], i + j < len);
                r0[j] = rcp64(p[j].e0 ? qe[j].w : 1u);
            }
            wload4(base + 64 * (s + h + 2), last, r);     // (the pair after this one)
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j) code_pos(k, o, qe[j], p[j], r0[j], dummy);
        }
        C2P_WORK
        lds_barrier();                                // (the helpers may overwrite parts s, s + 1 now)
        C2P_WAIT
    }
    C2P_FLUSH(10)
    ring_store(o);
    ring_chunk(o, o.n, dummy);
    bool ok = live && o.n <= o.cap;
    uint32_t low = k.low;
    while (any_lane(ok && low != 0)) {
        const bool more = ok && low != 0;
        const bool full = more && o.n >= o.cap;
        ok = ok && !full;
        const uint32_t n0 = o.n;
        ring_put(o, low, 1, more && !full);
        low = (more && !full) ? low << 8 : low;
        ring_chunk(o, n0, dummy);
        ring_store(o);
    }
    ring_finish(o, ok);
    if (live) b.out_len[pkt] = ok ? o.n : 0u;
}

// launches with packets over 1919 bytes: model resets (kWRst) and left packets (kWLeft)
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2)))
void rc_enc2_wcode_r(rc_batch_dev b, E2Params e) { wcode_main<true>(b, e); }
#endif  // E2_WIDE

}  // namespace

#if E2_WIDE
// The wide kernels over the packets the scan listed (its chunk of cnt
// packets, scan-sized grid g); e: the chunk's E2Params (rc_hip_enc2_launch).
extern "C" int rc_hip_enc2_wide_launch(const rc_batch_dev* b, const void* ep, uint32_t g, uint32_t cnt, void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    const E2Params& e = *static_cast<const E2Params*>(ep);
    if (e.slot_len <= kWideSmallL)
        hipLaunchKernelGGL(rc_enc2_wscan_s, dim3(g), dim3(kScanThreads), 0, st, *b, e);
    else if (e.slot_len <= 2048)
        hipLaunchKernelGGL(rc_enc2_wscan, dim3(g), dim3(kScanThreads), 0, st, *b, e);
    else
        hipLaunchKernelGGL(rc_enc2_wscan_l, dim3(g), dim3(kScanThreads), 0, st, *b, e);
    static const char* w1 = getenv("ENET_RC_WCODE1");            // the one-wavefront wide code pass (A/B)
    if (e.slot_len <= kE2MaxLen && !(w1 && atoi(w1) == 1))
        hipLaunchKernelGGL(rc_enc2_wcode2, dim3((cnt + 255) / 256), dim3(512), kC2Lds, st, *b, e);
    else if (e.slot_len <= kE2MaxLen)
        hipLaunchKernelGGL(rc_enc2_wcode, dim3((cnt + 255) / 256), dim3(256), kCodeItab + 512, st, *b, e);
    else
        hipLaunchKernelGGL(rc_enc2_wcode_r, dim3((cnt + 255) / 256), dim3(256), kCodeItab + 512, st, *b, e);
    return static_cast<int>(hipGetLastError());
}
#endif

#if E2_PLAIN
#if RC_ENC2_PART == 1
extern "C" int rc_hip_enc2_wide_launch(const rc_batch_dev* b, const void* ep, uint32_t g, uint32_t cnt,
                                       void* stream);   // rc_enc2_wide.o
#endif

#ifdef E2_PROF
extern "C" int rc_enc2_prof_read(unsigned long long* out, int reset)
{
    hipError_t err = hipDeviceSynchronize();
    if (err == hipSuccess) err = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_e2prof), sizeof(unsigned long long) * 32);
    if (err == hipSuccess && reset) {
        static const unsigned long long zero[32] = {0};
        err = hipMemcpyToSymbol(HIP_SYMBOL(g_e2prof), zero, sizeof zero);
    }
    return static_cast<int>(err);
}
#endif

// bytes of one packet's record slot for packets of up to max_len bytes
extern "C" uint64_t rc_hip_enc2_slot_bytes(uint32_t max_len)
{
    const uint64_t l = max_len < kE2SlotMax ? max_len : kE2SlotMax;
    return ((8 * l + 15) & ~15ull) + 96;              // 8 B per position, + the chunks read ahead
}

// bytes of one wide-mode slot (16-B records, rc_enc2_wcode reads 4 ahead)
extern "C" uint64_t rc_hip_enc2_wide_slot_bytes(uint32_t max_len)
{
    const uint64_t l = max_len < kE2SlotMax ? max_len : kE2SlotMax;
    return 16 * l + 256;
}

// Both passes over the batch, in chunks that fit the record stream; packets
// off the fast path end up in ws->enc2_list / counters[3] for the lane kernels.
// Per chunk: rc_enc2_scan, rc_enc2_code2 (narrow packets), then the wide
// kernels over the packets the scan listed for them (the wide list's regions).
extern "C" int rc_hip_enc2_launch(const rc_batch_dev* b, const rc_workspace_dev* ws, void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint32_t ml = b->max_len ? b->max_len : 4096;
    const uint64_t slot = rc_hip_enc2_slot_bytes(ml);
    uint64_t per = ws->enc2_cap / slot;
    if (per == 0) return static_cast<int>(hipErrorInvalidValue);
    // chunks of whole code-pass rounds (one 256-packet block per CU): a chunk
    // of 1.5 rounds costs the code pass two rounds of its longest packets
    const uint64_t round = static_cast<uint64_t>(ws->cus ? ws->cus : 256) * 256;
    if (per < b->n && per > round) per -= per % round;
    E2Params e;
    e.stream = static_cast<uint8_t*>(ws->enc2_stream);
    e.slot_bytes = slot;
    e.slot_len = ml < kE2SlotMax ? ml : kE2SlotMax;
    e.dummy = static_cast<uint8_t*>(ws->enc2_stream) + ws->enc2_cap;   // (allocated past the stream)
    e.order = ws->order;
    e.bins = ws->bins;
    e.list = ws->enc2_list;
    e.count = ws->counters + 3;
    e.wslot_bytes = rc_hip_enc2_wide_slot_bytes(ml);
    e.wide = ws->enc2_wide && ws->enc2_wide_cap >= e.wslot_bytes ? static_cast<uint8_t*>(ws->enc2_wide) : nullptr;
    e.wlist = ws->enc2_wlist;
    e.wcount = ws->counters + RC_WSHARD_AT;
    const uint64_t wcap = e.wide ? ws->enc2_wide_cap / e.wslot_bytes : 0;
    e.wcap = static_cast<uint32_t>(wcap < 0xFFFFFFFFull ? wcap : 0xFFFFFFFFull);
    // The scans' grids: 64 workgroups per CU, each wavefront looping over a few
    // packets (4 on C2), although only 9-11 are resident per CU (LDS).
    // Workgroups that start as others finish keep the resident wavefronts in
    // different phases of their packets (counting atomics, scatter, walks),
    // where wavefronts started together and looping over many packets stay in
    // step and contend for the same unit: rocprof, C2 rc_enc2_scan_s 0.438 ms
    // at 16 per CU, 0.510 at 11 (the resident count), 0.367 at 64, 0.361 at
    // 128; C3 rc_enc2_wscan_s 1.767 -> 1.558 at 64 (1.505 at 256, but an empty
    // wide launch then costs 20 us on C2).  Fewer pays where the scan lists
    // most packets for the wide kernels (C3 rc_enc2_scan_s 0.125 -> 0.207 ms
    // at 64: one list append per workgroup on one counter).  ENET_RC_SCAN_BPC:
    // workgroups per CU instead (experiments)
    static const char* bpc_env = getenv("ENET_RC_SCAN_BPC");
    const int bpc = bpc_env ? atoi(bpc_env) : 0;
    const uint32_t scan_blocks_max = ws->cus * (bpc > 0 ? static_cast<uint32_t>(bpc) : 64u);
    // The wide scan's grid: 128 workgroups per CU since it fits 18 per CU
    // (C3 rc_enc2_wscan_s 1.142 -> 1.094 ms against 64; 1.238 at 32;
    // profiles/r6/s7i_scan_grid.txt).  ENET_RC_WSCAN_BPC: per CU instead.
    static const char* wbpc_env = getenv("ENET_RC_WSCAN_BPC");
    const int wbpc = wbpc_env ? atoi(wbpc_env) : 0;
    const uint32_t wscan_blocks_max = ws->cus * (wbpc > 0 ? static_cast<uint32_t>(wbpc) : 128u);
    static const char* lanes = getenv("ENET_RC_ENC2_LANES");      // experiment: 32 packets per wavefront
    e.act = (lanes && atoi(lanes) == 32) ? 32u : 64u;
    e.slow = ws->enc2_slow;
    for (uint64_t lo = 0; lo < b->n; lo += per) {
        const uint64_t hi = lo + per < b->n ? lo + per : b->n;
        e.lo = static_cast<uint32_t>(lo);
        e.hi = static_cast<uint32_t>(hi);
        const uint32_t cnt = static_cast<uint32_t>(hi - lo);
        {
            const uint32_t per = (cnt + RC_WSHARDS - 1) / RC_WSHARDS, cap = e.wcap / RC_WSHARDS;
            e.wreg = per < cap ? per : cap;
        }
        if (lo > 0 && e.wide) {                        // (the batch's memset cleared it for the first chunk)
            const hipError_t err = hipMemsetAsync(e.wcount, 0, RC_WSHARDS * RC_WSHARD_STRIDE * sizeof(uint32_t), st);
            if (err != hipSuccess) return static_cast<int>(err);
        }
        if (e.slot_len <= kWideSmallL)
            hipLaunchKernelGGL(rc_enc2_scan_s, dim3(cnt < scan_blocks_max ? cnt : scan_blocks_max), dim3(kScanThreads),
                               0, st, *b, e);
        else if (e.slot_len <= kScanMidL)
            hipLaunchKernelGGL(rc_enc2_scan_m, dim3(cnt < scan_blocks_max ? cnt : scan_blocks_max), dim3(kScanThreads),
                               0, st, *b, e);
        else
            hipLaunchKernelGGL(rc_enc2_scan, dim3(cnt < scan_blocks_max ? cnt : scan_blocks_max), dim3(kScanThreads),
                               0, st, *b, e);
        static const char* one = getenv("ENET_RC_ENC2_CODE1");        // the one-wavefront code pass (A/B)
        if ((one && atoi(one) == 1) || e.act != 64)
            hipLaunchKernelGGL(rc_enc2_code, dim3((cnt + 4 * e.act - 1) / (4 * e.act)), dim3(256), kCodeItab + 512, st,
                               *b, e);
        else
            hipLaunchKernelGGL(rc_enc2_code2, dim3((cnt + 255) / 256), dim3(512), kC2Lds, st, *b, e);
        if (e.wide) {
            const int rc = rc_hip_enc2_wide_launch(b, &e, cnt < wscan_blocks_max ? cnt : wscan_blocks_max, cnt, stream);
            if (rc != 0) return rc;
        }
    }
    return static_cast<int>(hipGetLastError());
}
#endif  // E2_PLAIN
