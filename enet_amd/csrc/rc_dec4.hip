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

#include "rc_bucket4.h"

namespace {

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
    const uint32_t per_block = 4 * act;
    const uint32_t slot = blockIdx.x * per_block + local;
    uint8_t* reg = static_cast<uint8_t*>(ws.lane_pool) + static_cast<size_t>(slot) * ws.lane_region;
    const uint32_t* order = ws.order && !ws.bins[RC_LEN_BINS] ? ws.order : nullptr;
    for (uint32_t i = slot; i < b.n; i += gridDim.x * per_block) {
        // the bail count is per round of packets: the lanes of a wavefront
        // start their next packets together (a batch of many packets per lane
        // would otherwise send every later packet on after the first 16 bails)
        if (l == 0) *wbail = 0u;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
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
