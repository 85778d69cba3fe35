// rc_dec5.hip -- bucket-history range decoder with speculative steps
// (compress.c:498-627), bit-exact.
//
// The model and its algebra are rc_dec4.hip's (rc_bucket4.h): per packet one
// 64-B record per previous byte p (bucket p), every sub-context statistic
// derived from it.  What changes is when a step waits for its record.
//
// rc_dec4 reads bucket p = x[i-1] at the top of step i: the load is issued as
// soon as x[i-1] is decoded, and everything step i decodes depends on it, so
// about half a step of its latency is exposed (PMC: ~45 % of a wavefront's
// cycles are memory waits).  But on most steps the record does not change
// what is decoded -- only two of its properties matter before the symbol is
// known:
//   - whether the order-2 context (x[i-2], x[i-1]) holds symbols (then it is
//     coded first, compress.c:536-568): ~1 % of random-byte steps;
//   - order 1's escape count and total (5 dist1, 5 dist1 + 2 t1), which a
//     one-byte table per packet in LDS keeps (T[p] = t1 | dist1 << 4, 0xFF
//     when t1 > 14); the record's element values matter only for an order-1
//     hit (~1 %).
// So step i decodes speculatively with T[p] and "no order-2 symbols", issues
// the load of the next bucket, and only then waits for bucket p (issued a
// whole step earlier), which verifies the guess: the order-2 group is empty
// and T[p] agrees with the record.  A step that guessed wrong -- or needed the
// record's values (a hit), or more input than the lookahead holds -- is rolled
// back (coder registers only: nothing is stored, no chunk is loaded, the root
// is updated only after the check) and redone in the next iteration with its
// record in registers, exactly as rc_dec4 decodes.  T is a hint: every
// speculative step is checked against the record, so a stale or wrong T entry
// costs a redo, never a wrong byte.
//
// A step's record load is issued once the step is committed, after its
// record store, and waited for after the next step's decode: the next step's
// speculative decode runs in its shadow.
//
// Fast path and hand-off as rc_dec4: buckets of at most kCap4 elements, fewer
// than 4094 nodes, root codes within symbol 255; a lane leaving it lists its
// packet for the lane kernels (ws.enc2_list, count ws.counters[3]).

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

constexpr uint32_t kWaveBail5 = 16;          // as rc_dec4's kWaveBail

#if defined(RC_LANE_HOST_TEST) && defined(DEC5_STATS)
}  // namespace
extern "C" { unsigned long long g_dec5_stats[4]; }   // iterations, commits, redos, redos from a stall
namespace {
#define DEC5_STAT(i, c) do { if (c) ++g_dec5_stats[i]; } while (0)
#else
#define DEC5_STAT(i, c) do { } while (0)
#endif
constexpr uint32_t kTUnknown = 0xFF;

// T entry of a bucket from its order-1 statistics
DEV uint32_t t_code(uint32_t t1, uint32_t d1) { return t1 > 14 ? kTUnknown : (t1 | d1 << 4); }

// dec_code (rc_lane_common.h) for a speculative step: a lane that would need
// its byte-wise rare path (a settle past the lookahead, or range < BOTTOM)
// does not take it but stalls (the step is rolled back and redone).  Lanes
// that are not speculative take the rare path as dec_code does.
DEV void dec_code5(uint32_t& low, uint32_t& code, uint32_t& range, uint32_t under, uint32_t count,
                   ByteSrc& in, bool en, bool spec, bool& stall)
{
    low = en ? low + under * range : low;
    range = en ? range * count : range;
    const uint32_t k = en ? settled_bytes(low, range) : 0u;
    const bool fast = k <= in.na;
    const uint32_t kk = fast ? k : 0u;
    code = src_shift_in(in, code, kk);
    low <<= 8 * kk;
    range <<= 8 * kk;
    bool more = en && (!fast || range < kBot);
    stall = stall || (more && spec);
    more = more && !spec;
    if (rare_lane(more)) {
        bool loaded = false;
        do {
            const bool carry = (low ^ (low + range)) >= kTop;
            const bool stop = carry && range >= kBot;
            more = more && !stop;
            if (!any_lane(more)) break;
            range = (more && carry) ? ((0u - low) & (kBot - 1)) : range;
            if (rare_lane(more && in.na == 0 && in.q == 4)) { src_adv(in); loaded = true; }
            src_fill(in, more && in.na == 0);
            code = src_shift_in(in, code, more ? 1u : 0u);
            range = more ? range << 8 : range;
            low = more ? low << 8 : low;
        } while (rare_lane(more));
        // (a pending rare input load would make every later use of the chunk
        // registers wait for vmcnt(0): settled here, on the rare path)
        if (loaded) __builtin_amdgcn_s_waitcnt(0);
    }
}

// compress.c:536-568 in one sub-context (rc_dec4 sub_decode); a speculative
// lane whose code selects a symbol (a hit: the record's values are needed)
// stalls instead
DEV bool sub_decode5(const Bucket& B, uint32_t g, uint32_t t, uint32_t dd, double rtot, uint32_t& low,
                     uint32_t& code, uint32_t& range, ByteSrc& in, uint32_t& v, uint32_t& j, bool& fail,
                     bool spec, bool& stall)
{
    const uint32_t esc = kSubEscDelta * dd, tot = esc + kSubDelta * t;
    const uint32_t cd = dec_read_d(range, low, code, tot, rtot);
    if (cd < esc) {
        dec_code5(low, code, range, 0, esc, in, true, spec, stall);
        return false;
    }
    if (spec) { stall = true; return false; }
    const uint32_t r = cd - esc;
    if (r >= kSubDelta * t) { fail = true; return false; }
    j = select_bit(g, r >> 1);
    v = byte_at(B.v, j);
    return true;
}

DEV void bail5(const rc_workspace_dev& ws, uint32_t pkt)
{
    const uint32_t slot = atomicAdd(&ws.counters[3], 1u);
    ws.enc2_list[slot] = pkt;
}

DEV void t_clear(uint8_t* tt)
{
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int i = 0; i < 16; ++i) reinterpret_cast<uint4*>(tt)[i] = z;
}

DEV void decompress_one5(const rc_batch_dev& bt, const rc_workspace_dev& ws, uint32_t pkt, uint8_t* reg,
                         uint8_t* root, uint8_t* tt, uint32_t* wbail)
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
    t_clear(tt);
    uint32_t rtot = 1 + 256;
    double rrt = rcp64(rtot);
    uint32_t low = 0, range = ~0u;
    uint32_t code = static_cast<uint32_t>(in.la >> 32);            // compress.c:344-350 (0 past the end)
    in.la <<= 32;
    in.na -= 4;
    src_refill(in, true);

    Bucket B;                       // the step's context record when held (redo, or the last step's bucket)
    bk_empty(B, epoch);
    Raw4 rw;                        // bucket p in flight (issued by the previous step)
    rw.q0 = rw.q1 = rw.q2 = rw.q3 = make_uint4(0u, 0u, 0u, 0u);
    Groups S;                       // redo: the groups of B for the step being redone
    S.g2 = S.g1 = S.t2 = S.d2 = S.t1 = S.d1 = 0;
    // (words, not bools: a bool would be an SGPR lane mask)
    uint32_t redo = 0;              // this step is redone with B and S
    uint32_t pfwd = 1;              // this step's context record is B (the previous step's bucket)
    uint32_t tcur = 0;              // T[p]
    uint32_t order = 0, a = 0, p = 0, nodes = 1;
    bool fail = false, off = false;

    // One step per iteration: (A) decode the symbol speculatively (unless
    // redone) -- every code but the step's last; (C) wait for bucket p
    // (issued by the previous step, a whole decode ago) and check the guess;
    // then either roll back, or commit: the element into bucket p and its
    // store, (B) the load of the next step's bucket, the step's last code,
    // the root's update and the output -- in the shadow of that load.
    for (;;) {
        src_fill(in, true);
        const bool spec = redo == 0;
        const uint32_t s_low = low, s_range = range, s_code = code, s_na = in.na;
        const uint64_t s_la = in.la;
        bool stall = spec && order >= 1 && tcur == kTUnknown;
        Groups s;
        s.t2 = spec ? 0u : S.t2; s.d2 = spec ? 0u : S.d2; s.g2 = spec ? 0u : S.g2;
        s.t1 = spec ? (tcur & 15) : S.t1; s.d1 = spec ? (tcur >> 4) : S.d1; s.g1 = spec ? 0u : S.g1;
        const double rt2 = rcp64(max(kSubEscDelta * s.d2 + kSubDelta * s.t2, 1u));
        const double rt1 = rcp64(max(kSubEscDelta * s.d1 + kSubDelta * s.t1, 1u));
        int at = -1;
        uint32_t hj = 0, v = 0;
        bool new0 = false, lfail = false, leof = false, loff = false;
        // (A) order 2 (only a redone step can have its symbols), then order 1
        if (order >= 2 && !stall && s.t2 > 0) {
            if (sub_decode5(B, s.g2, s.t2, s.d2, rt2, low, code, range, in, v, hj, lfail, spec, stall)) at = 2;
        }
        if (at < 0 && !lfail && !stall && order >= 1 && s.t1 > 0) {
            if (sub_decode5(B, s.g1, s.t1, s.d1, rt1, low, code, range, in, v, hj, lfail, spec, stall)) at = 1;
        }
        // root, compress.c:570-596
        uint32_t cnt0 = 0, under0 = 0;
        if (at < 0 && !lfail && !stall) {
            const uint32_t cd = dec_read_d(range, low, code, rtot, rrt);
            if (cd < 1) {
                leof = true;                                         // end of stream
            } else if (cd - 1 >= rtot - 1) {
                loff = true;                                         // past symbol 255
            } else {
                uint32_t under, cnt;
                v = root3_search(root, R, cd - 1, under, cnt);
                new0 = cnt == 0;
                cnt0 = cnt;
                under0 = under;
                at = 0;
            }
        }
        const bool have = at >= 0 && !stall && !lfail;
        // the interval of the step's last code: the root's, or a hit's (redo only)
        uint32_t fu = 1 + under0, fc = 1 + cnt0;
        if (any_lane(have && at != 0)) {
            uint32_t hu, hc;
            hit_interval(B, at == 2 ? s.g2 : s.g1, kSubEscDelta * (at == 2 ? s.d2 : s.d1), hj, hu, hc);
            fu = at != 0 ? hu : fu;
            fc = at != 0 ? hc : fc;
        }
        // (C) bucket p: the record issued by the previous step, or B.  Unpacked
        // on every path: a load consumed on some paths only stays pending for
        // the compiler at the merge, and the next write to its registers would
        // wait for vmcnt(0).
        {
            Bucket Bn;
            bk_from(rw, epoch, Bn);
            const bool take = spec && !pfwd;
            B.h = take ? Bn.h : B.h; B.hit = take ? Bn.hit : B.hit;
            B.nw = take ? Bn.nw : B.nw; B.run = take ? Bn.run : B.run;
#pragma unroll
            for (int d = 0; d < 6; ++d) { B.a[d] = take ? Bn.a[d] : B.a[d]; B.v[d] = take ? Bn.v[d] : B.v[d]; }
        }
        const uint32_t nd = live_dwords(bk_k(B.h));
        Groups g;
        bk_groups(B, nd, a, order >= 2, g);
        // the guess: no order-2 symbols, T[p] = the record's order-1 statistics
        const bool ok = !spec || (!stall && g.t2 == 0 && (order < 1 || (g.t1 == s.t1 && g.d1 == s.d1)));
        DEC5_STAT(0, true);
        DEC5_STAT(1, ok && have);
        DEC5_STAT(2, !ok);
        DEC5_STAT(3, !ok && stall);
        if (!ok) {
            // roll back and redo the step with its record
            low = s_low; range = s_range; code = s_code; in.na = s_na; in.la = s_la;
            S = g;
            redo = 1;
        }
        if (ok && lfail) { fail = true; break; }
        if (ok && leof) { dec_code5(low, code, range, 0, 1, in, true, false, stall); break; }   // (EOF)
        if (ok && loff) { off = true; break; }
        const bool commit = ok && have;
        fail = commit && o.n >= o.cap;                               // compress.c:617
        // the element joins bucket p (compress.c:598-615); nodes as compress.c creates them
        uint32_t lt, le;
        bk_rank(B, nd, v, lt, le);
        const uint32_t eqr = low_bits(le) & ~low_bits(lt);
        const bool n2 = order >= 2 && (g.g2 & eqr) == 0;
        const bool n1 = order >= 1 && at != 2 && (g.g1 & eqr) == 0;
        nodes += commit ? (new0 ? 1u : 0u) + (n2 ? 1u : 0u) + (n1 ? 1u : 0u) : 0u;
        const bool full = commit && order >= 1 && bk_k(B.h) >= kCap4;
        const uint32_t first = order == 1 ? 1u : 0u;                 // position 1: hit and new
        const bool ins = commit && order >= 1;
        bk_insert(B, nd, le, a, v, (at == 2 ? 1u : 0u) | first, (n2 ? 1u : 0u) | first, lt == le ? 1u : 0u,
                  (1u << 16) + (at == 2 ? (1u << 21) : 0u) + (n1 ? (1u << 26) : 0u), ins && !full);
        // (stored before the next load is issued: a later wait for the store
        // then never waits for that load; lanes with nothing to store write
        // the scratch record)
        bk_store(reg, ins ? kO1Base + p * kRec4 : kDummyRec, B);
        // the output window the previous step completed: also before the load
        // (what is issued after it -- the input chunk only -- is then what the
        // next step's wait for it waits for as well)
        sink_flush(o);
        // (B) the next step's bucket: this one when v == p, else a load whose
        // latency the rest of this step and the next step's decode overlap
        const bool nfwd = commit && order >= 1 && v == p;
        raw4_load(reg, (commit && !nfwd) ? kO1Base + v * kRec4 : kDummyRec, rw);
        if (ins) tt[p] = static_cast<uint8_t>(t_code(g.t1 + (at != 2 ? 1u : 0u), g.d1 + (n1 ? 1u : 0u)));
        // the step's last code, the root's update (compress.c:583-595)
        dec_code5(low, code, range, fu, fc, in, commit, false, stall);
        if (commit && at == 0) {
            root3_add<false>(root, R, v, cnt0);
            rtot = (rtot + kRootDelta) & 0xFFFF;
            if (1 + cnt0 > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit) rtot = root3_rescale<false>(root, R);
            rrt = rcp64(rtot);
        }
        off = full || (commit && nodes >= kNodeLimit4) || *wbail >= kWaveBail5;
        if (fail || off) break;
        if (!commit) continue;                                       // redo next iteration
        sink_put(o, v, 1, true);
        src_adv(in);
        tcur = tt[v];
        redo = 0;
        pfwd = nfwd ? 1u : 0u;
        a = p;
        p = v;
        order += order < 2 ? 1u : 0u;
    }
    if (off && !fail) { atomicAdd(wbail, 1u); bail5(ws, pkt); return; }
    sink_finish(o, !fail);
    bt.out_len[pkt] = fail ? 0u : o.n;
}

}  // namespace

#ifndef RC_LANE_HOST_TEST
// per lane in LDS: the root counts + pad (272 B), then T (256 B): 132 dwords, b128 conflict-free
constexpr uint32_t kDec5T = kRootStrideDec;
constexpr uint32_t kDec5Lds = kRootStrideDec + 256;

// one wave per SIMD by design (a packet per lane, 65536 lanes fill the chip)
extern "C" __global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void rc_decompress_dec5(rc_batch_dev b, rc_workspace_dev ws)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t act = ws.lane_active;
    const uint32_t wave = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (l >= act) return;
    const uint32_t local = wave * act + l;
    uint8_t* root = smem + local * kDec5Lds;
    uint8_t* tt = root + kDec5T;
    uint32_t* wbail = reinterpret_cast<uint32_t*>(smem + 4 * act * kDec5Lds) + wave;
    const uint32_t per_block = 4 * act;
    const uint32_t slot = blockIdx.x * per_block + local;
    uint8_t* reg = static_cast<uint8_t*>(ws.lane_pool) + static_cast<size_t>(slot) * ws.lane_region;
    const uint32_t* order = ws.order && !ws.bins[RC_LEN_BINS] ? ws.order : nullptr;
    for (uint32_t i = slot; i < b.n; i += gridDim.x * per_block) {
        // the bail count is per round of packets (rc_dec4)
        if (l == 0) *wbail = 0u;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t pkt = order ? order[i] : i;
        decompress_one5(b, ws, pkt, reg, root, tt, wbail);
    }
}

extern "C" int rc_hip_dec5_launch(const rc_batch_dev* b, const rc_workspace_dev* ws, uint32_t blocks, void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    const size_t lds = static_cast<size_t>(4 * ws->lane_active) * kDec5Lds + 16;   // + wbail[4]
    hipLaunchKernelGGL(rc_decompress_dec5, dim3(blocks), dim3(256), lds, st, *b, *ws);
    return static_cast<int>(hipGetLastError());
}
#endif  // RC_LANE_HOST_TEST
