// rc_kernels.hip -- MI355X (gfx950) kernels for ENet's order-2 PPM range coder.
//
// Reference behaviour: lsalzman/enet compress.c (enet_range_coder_compress
// :246-342, enet_range_coder_decompress :498-627).  Output must be bit-exact.
//
// Fast path ("wave" kernels): one 64-lane wavefront per packet, the adaptive
// model resident in LDS + VGPRs.  compress.c keeps every context as a binary
// tree of nodes; only {count[v], escapes, total} of each context and the node
// count are observable, so the model here is laid out for
// wave-parallel search instead:
//   root (order 0)  : 256 counts + 256 inclusive prefix sums in 3 VGPRs
//                     (lane l owns symbols 4l..4l+3) -> search = 1 ballot
//   order-1 headers : 256 x {esc, tot, off, len} in 8 VGPRs (lane = ctx & 63)
//   order-1 / order-2 symbol lists: LDS blocks of sorted entries
//                     {value:8 | count:8 | cum:16}, lane i holds entry i, so a
//                     lookup is one ds_read + ballot + readlane (no BST walk)
//   order-2 headers : LDS pool {esc, tot, off, len}, stable ids
// The range-coder arithmetic is wave-uniform (SGPR) work.
//
// Exact path ("exact" kernels): one lane per packet running compress.c's own
// binary-tree model in a 64 KiB global scratch pool.  It handles the only
// cases the flat model cannot reproduce -- a corrupt stream whose root code
// points past symbol 255 (compress.c:427-438 then inserts a truncated duplicate
// value and later behaviour depends on tree shape) -- and packets whose model
// outgrows the LDS arena.  The fast kernel appends such packets to a device
// list; the exact kernel drains it in the same stream (no host round trip).

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "rc_abi_internal.h"

#define DEV __device__ __forceinline__

namespace {

constexpr uint32_t kTop = 1u << 24;           // compress.c:27
constexpr uint32_t kBot = 1u << 16;           // compress.c:28
constexpr uint32_t kRootDelta = 3;            // compress.c:30
constexpr uint32_t kSubDelta = 2;             // compress.c:35
constexpr uint32_t kSubEscDelta = 5;          // compress.c:36
constexpr uint32_t kMaxNodes = 4096 - 2;      // compress.c:150
constexpr uint32_t kTotalLimit = kBot - 0x100;

// LDS layout per workgroup (one wave):
constexpr uint32_t kFreeHeads = 0;            // u16[2][9] free-list heads (kind, log2 cap)
constexpr uint32_t kOutStage = 64;            // 64-byte output staging
constexpr uint32_t kInStage = 128;            // input staging, stage_bytes long
constexpr uint32_t kNoBlock = 0xFFFFu;

// Phase timing of the wave compress kernel (tools/waveprof.hip only): shader
// clock cycles per phase, summed over packets.
#ifdef RC_WAVE_PROF
__device__ unsigned long long g_wave_prof[8];
#define PROF_T(t) const uint64_t t = __builtin_amdgcn_s_memtime()
#define PROF_ADD(acc, a, b) acc += (b) - (a)
#else
#define PROF_T(t)
#define PROF_ADD(acc, a, b)
#endif

// ------------------------------------------------------------- wave helpers

DEV uint32_t lane() { return __lane_id(); }
DEV uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
DEV uint32_t lane_val(uint32_t x, uint32_t l) { return __builtin_amdgcn_readlane(x, l); }
DEV uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// Inclusive wave-wide prefix sum (DPP row shifts + row broadcasts, gfx9 DPP).
DEV uint32_t wave_scan(uint32_t x)
{
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);   // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return x;
}

DEV uint32_t cap_of(uint32_t len, uint32_t mincap)
{
    return len <= mincap ? mincap : (1u << (32 - __builtin_clz(len - 1)));
}
DEV uint32_t log2u(uint32_t p) { return 31 - __builtin_clz(p); }

DEV uint32_t* ent(uint8_t* s, uint32_t off) { return reinterpret_cast<uint32_t*>(s + off); }
DEV uint16_t* ids(uint8_t* s, uint32_t off, uint32_t cap) { return reinterpret_cast<uint16_t*>(s + off + 4 * cap); }

// ------------------------------------------------------------------ model

// Context header; all fields wave-uniform.
struct Ctx { uint32_t esc, tot, off, len; };

struct Model {
    // root: lane l owns symbols 4l..4l+3
    uint32_t rcnt;            // 4 x u8 counts
    uint32_t rcum01, rcum23;  // inclusive prefix sums, u16 pairs
    // order-1 headers: context x lives in lane x&63 of register x>>6
    uint32_t ha0, ha1, ha2, ha3;   // esc | tot << 16
    uint32_t hb0, hb1, hb2, hb3;   // off | len << 16
    // uniform
    uint32_t rtot, lo, hi, nodes;
    uint32_t arena_lo, arena_hi;
    bool overflow;
};

DEV void model_reset(uint8_t* s, Model& m)
{
    m.rcnt = 0; m.rcum01 = 0; m.rcum23 = 0;
    m.ha0 = m.ha1 = m.ha2 = m.ha3 = 0;
    m.hb0 = m.hb1 = m.hb2 = m.hb3 = 0;
    m.rtot = 1 + 256;          // ENET_CONTEXT_CREATE(root, 1, 1), compress.c:82-88
    m.lo = m.arena_lo; m.hi = m.arena_hi;
    m.nodes = 1;
    if (lane() < 18) reinterpret_cast<uint16_t*>(s + kFreeHeads)[lane()] = kNoBlock;
}

DEV void o1_get(const Model& m, uint32_t x, Ctx& c)
{
    // read all four candidates and select in the scalar domain: a select of
    // register *addresses* would force Model into scratch memory
    const uint32_t q = x >> 6, l = x & 63;
    const uint32_t a0 = lane_val(m.ha0, l), a1 = lane_val(m.ha1, l);
    const uint32_t a2 = lane_val(m.ha2, l), a3 = lane_val(m.ha3, l);
    const uint32_t b0 = lane_val(m.hb0, l), b1 = lane_val(m.hb1, l);
    const uint32_t b2 = lane_val(m.hb2, l), b3 = lane_val(m.hb3, l);
    const uint32_t a = q == 0 ? a0 : q == 1 ? a1 : q == 2 ? a2 : a3;
    const uint32_t b = q == 0 ? b0 : q == 1 ? b1 : q == 2 ? b2 : b3;
    c.esc = a & 0xFFFF; c.tot = a >> 16; c.off = b & 0xFFFF; c.len = b >> 16;
}

DEV void o1_put(Model& m, uint32_t x, const Ctx& c)
{
    const uint32_t q = x >> 6;
    const bool me = lane() == (x & 63);
    const uint32_t a = c.esc | (c.tot << 16), b = c.off | (c.len << 16);
    const bool w0 = me && q == 0, w1 = me && q == 1, w2 = me && q == 2, w3 = me && q == 3;
    m.ha0 = w0 ? a : m.ha0; m.hb0 = w0 ? b : m.hb0;
    m.ha1 = w1 ? a : m.ha1; m.hb1 = w1 ? b : m.hb1;
    m.ha2 = w2 ? a : m.ha2; m.hb2 = w2 ? b : m.hb2;
    m.ha3 = w3 ? a : m.ha3; m.hb3 = w3 ? b : m.hb3;
}

DEV void o2_get(uint8_t* s, uint32_t id, Ctx& c)
{
    const uint2 w = *reinterpret_cast<const uint2*>(s + id);
    const uint32_t a = uni(w.x), b = uni(w.y);
    c.esc = a & 0xFFFF; c.tot = a >> 16; c.off = b & 0xFFFF; c.len = b >> 16;
}

DEV void o2_put(uint8_t* s, uint32_t id, const Ctx& c)
{
    if (lane() == 0)
        *reinterpret_cast<uint2*>(s + id) = make_uint2(c.esc | (c.tot << 16), c.off | (c.len << 16));
}

DEV uint32_t o2_new(uint8_t* s, Model& m)
{
    if (m.hi < m.lo + 8) { m.overflow = true; return 0; }
    m.hi -= 8;
    if (lane() == 0) *reinterpret_cast<uint2*>(s + m.hi) = make_uint2(0u, 0u);
    return m.hi;
}

// kind 0: order-2 block (4 B/entry); kind 1: order-1 block (4 B entry + 2 B o2 id)
DEV uint32_t blk_alloc(uint8_t* s, Model& m, uint32_t kind, uint32_t cap)
{
    uint16_t* head = reinterpret_cast<uint16_t*>(s + kFreeHeads) + kind * 9 + log2u(cap);
    const uint32_t h = uni(*head);
    if (h != kNoBlock) {
        const uint32_t nx = uni(*reinterpret_cast<const uint16_t*>(s + h));
        if (lane() == 0) *head = static_cast<uint16_t>(nx);
        return h;
    }
    const uint32_t bytes = cap * (kind ? 6u : 4u);
    const uint32_t off = (m.lo + 3u) & ~3u;
    if (off + bytes > m.hi) { m.overflow = true; return 0; }
    m.lo = off + bytes;
    return off;
}

DEV void blk_free(uint8_t* s, uint32_t kind, uint32_t off, uint32_t cap)
{
    uint16_t* head = reinterpret_cast<uint16_t*>(s + kFreeHeads) + kind * 9 + log2u(cap);
    const uint32_t h = uni(*head);
    if (lane() == 0) {
        *reinterpret_cast<uint16_t*>(s + off) = static_cast<uint16_t>(h);
        *head = static_cast<uint16_t>(off);
    }
}

// First entry with value >= v: k, whether it is v, the cumulative count below
// k and (if found) the entry's count.
struct Find { uint32_t k, under, cnt; bool found; };

DEV Find blk_find(uint8_t* s, const Ctx& c, uint32_t v)
{
    Find f;
    uint32_t carry = 0;
    for (uint32_t base = 0;; base += 64) {
        const uint32_t idx = base + lane();
        const bool in = idx < c.len;
        const uint32_t e = in ? ent(s, c.off)[idx] : 0u;
        const uint32_t nlt = __builtin_popcountll(ballot(in && (e & 0xFF) < v));
        const uint32_t nin = c.len > base ? min(64u, c.len - base) : 0u;
        if (nlt < nin || base + 64 >= c.len) {
            f.k = base + nlt;
            f.under = nlt ? (lane_val(e, nlt - 1) >> 16) : carry;
            if (nlt < nin) {
                const uint32_t ek = lane_val(e, nlt);
                f.found = (ek & 0xFF) == v;
                f.cnt = f.found ? ((ek >> 8) & 0xFF) : 0u;
            } else {
                f.found = false; f.cnt = 0;
            }
            return f;
        }
        carry = lane_val(e, 63) >> 16;
    }
}

// Decoder search: first entry whose inclusive cum exceeds code.  Returns
// false when code lies beyond the last symbol (compress.c:415-416: corrupt).
DEV bool blk_search(uint8_t* s, const Ctx& c, uint32_t code, uint32_t& k, uint32_t& v,
                    uint32_t& under, uint32_t& cnt)
{
    for (uint32_t base = 0; base < c.len; base += 64) {
        const uint32_t idx = base + lane();
        const bool in = idx < c.len;
        const uint32_t e = in ? ent(s, c.off)[idx] : 0u;
        const uint64_t hit = ballot(in && code < (e >> 16));
        if (hit) {
            const uint32_t j = static_cast<uint32_t>(__builtin_ctzll(hit));
            const uint32_t ek = lane_val(e, j);
            k = base + j; v = ek & 0xFF; cnt = (ek >> 8) & 0xFF; under = (ek >> 16) - cnt;
            return true;
        }
    }
    return false;
}

// count[k] += d; cum[j] += d for j >= k
DEV void blk_bump(uint8_t* s, const Ctx& c, uint32_t k, uint32_t d)
{
    for (uint32_t base = k & ~63u; base < c.len; base += 64) {
        const uint32_t idx = base + lane();
        if (idx >= k && idx < c.len) {
            uint32_t* p = ent(s, c.off) + idx;
            *p = *p + (d << 16) + (idx == k ? (d << 8) : 0u);
        }
    }
}

// Insert a new entry at k with count d (c.len/c.off updated).  kind 1 blocks
// carry an o2 id per entry.
DEV void blk_insert(uint8_t* s, Model& m, Ctx& c, uint32_t kind, uint32_t k, uint32_t v,
                    uint32_t under, uint32_t d, uint32_t newid)
{
    const uint32_t mincap = kind ? 2u : 1u;
    const uint32_t len = c.len;
    const uint32_t cap = cap_of(len, mincap);
    const uint32_t newe = v | (d << 8) | (((under + d) & 0xFFFFu) << 16);
    if (len == 0 || len == cap) {
        const uint32_t ncap = len == 0 ? mincap : cap * 2;
        const uint32_t noff = blk_alloc(s, m, kind, ncap);
        if (m.overflow) return;
        for (uint32_t base = 0; base < len; base += 64) {
            const uint32_t idx = base + lane();
            if (idx < len) {
                const uint32_t e = ent(s, c.off)[idx];
                const uint32_t ni = idx + (idx >= k ? 1u : 0u);
                ent(s, noff)[ni] = e + (idx >= k ? (d << 16) : 0u);
                if (kind) ids(s, noff, ncap)[ni] = ids(s, c.off, cap)[idx];
            }
        }
        if (lane() == 0) {
            ent(s, noff)[k] = newe;
            if (kind) ids(s, noff, ncap)[k] = static_cast<uint16_t>(newid);
        }
        if (len) blk_free(s, kind, c.off, cap);
        c.off = noff;
    } else {
        if (len > k) {
            for (int32_t base = static_cast<int32_t>((len - 1) & ~63u);
                 base >= static_cast<int32_t>(k & ~63u); base -= 64) {
                const uint32_t idx = static_cast<uint32_t>(base) + lane();
                if (idx >= k && idx < len) {
                    const uint32_t e = ent(s, c.off)[idx];
                    uint16_t id = 0;
                    if (kind) id = ids(s, c.off, cap)[idx];
                    ent(s, c.off)[idx + 1] = e + (d << 16);
                    if (kind) ids(s, c.off, cap)[idx + 1] = id;
                }
            }
        }
        if (lane() == 0) {
            ent(s, c.off)[k] = newe;
            if (kind) ids(s, c.off, cap)[k] = static_cast<uint16_t>(newid);
        }
    }
    c.len = len + 1;
    m.nodes++;
}

// compress.c:90-112 on a flat block: halve counts, rebuild cums, halve escapes.
DEV void blk_rescale(uint8_t* s, Ctx& c)
{
    uint32_t carry = 0;
    for (uint32_t base = 0; base < c.len; base += 64) {
        const uint32_t idx = base + lane();
        const bool in = idx < c.len;
        const uint32_t e = in ? ent(s, c.off)[idx] : 0u;
        uint32_t n = (e >> 8) & 0xFF;
        n -= n >> 1;
        const uint32_t inc = wave_scan(n);
        if (in) ent(s, c.off)[idx] = (e & 0xFF) | (n << 8) | (((carry + inc) & 0xFFFF) << 16);
        carry += lane_val(inc, 63);
    }
    c.esc -= c.esc >> 1;
    c.tot = (carry + c.esc) & 0xFFFF;
}

// Encoder-side visit of an order-1/2 context (compress.c:293-316 and the
// decoder's patch :603-613).  Returns the symbol's old count (0 if new) and
// the cum below it; esc/tot are updated, rescale applied.  For kind 1 the
// o2 id of the symbol's entry is returned in *o2id.
DEV uint32_t sub_update(uint8_t* s, Model& m, Ctx& c, uint32_t kind, uint32_t v,
                        uint32_t& under, uint32_t* o2id)
{
    const Find f = blk_find(s, c, v);
    under = f.under;
    if (f.found) {
        blk_bump(s, c, f.k, kSubDelta);
        if (o2id) *o2id = uni(ids(s, c.off, cap_of(c.len, 2))[f.k]);
    } else {
        uint32_t nid = 0;
        if (kind) { nid = o2_new(s, m); if (m.overflow) return 0; }
        blk_insert(s, m, c, kind, f.k, v, f.under, kSubDelta, nid);
        if (m.overflow) return 0;
        c.esc += kSubEscDelta;
        c.tot += kSubEscDelta;
        if (o2id) *o2id = nid;
    }
    c.tot = (c.tot + kSubDelta) & 0xFFFF;
    if (f.cnt > 0xFF - 2 * kSubDelta || c.tot > kTotalLimit) blk_rescale(s, c);
    return f.cnt;
}

// --------------------------------------------------------------- root (VGPRs)

DEV void root_lookup(const Model& m, uint32_t v, uint32_t& under, uint32_t& cnt)
{
    const uint32_t q = v >> 2, j = v & 3;
    cnt = (lane_val(m.rcnt, q) >> (8 * j)) & 0xFF;
    const uint32_t w = lane_val(j < 2 ? m.rcum01 : m.rcum23, q);
    const uint32_t cum = (j & 1) ? (w >> 16) : (w & 0xFFFF);
    under = v + cum - cnt;                   // v * minimum + sum of smaller counts
}

DEV void root_add(Model& m, uint32_t v)
{
    const uint32_t q = v >> 2, j = v & 3, l = lane();
    const uint32_t all = kRootDelta | (kRootDelta << 16);
    const uint32_t a01 = l > q ? all : l == q ? ((j == 0 ? kRootDelta : 0u) | (j <= 1 ? kRootDelta << 16 : 0u)) : 0u;
    const uint32_t a23 = l > q ? all : l == q ? ((j <= 2 ? kRootDelta : 0u) | (kRootDelta << 16)) : 0u;
    m.rcum01 += a01;
    m.rcum23 += a23;
    m.rcnt += l == q ? (kRootDelta << (8 * j)) : 0u;
}

DEV void root_rescale(Model& m)
{
    uint32_t c = m.rcnt;
    c -= (c >> 1) & 0x7F7F7F7Fu;
    m.rcnt = c;
    const uint32_t c0 = c & 0xFF, c1 = (c >> 8) & 0xFF, c2 = (c >> 16) & 0xFF, c3 = c >> 24;
    const uint32_t sum = c0 + c1 + c2 + c3;
    const uint32_t inc = wave_scan(sum);
    const uint32_t x0 = inc - sum + c0, x1 = x0 + c1, x2 = x1 + c2, x3 = x2 + c3;
    m.rcum01 = x0 | (x1 << 16);
    m.rcum23 = x2 | (x3 << 16);
    m.rtot = (lane_val(inc, 63) + 1 + 256) & 0xFFFF;
}

// ------------------------------------------------------------------ output

struct Out { uint8_t* g; uint32_t cap, n; };

DEV void out_flush_full(uint8_t* s, Out& o)   // called when n % 64 == 0
{
    o.g[o.n - 64 + lane()] = s[kOutStage + lane()];
}

DEV bool out_put(uint8_t* s, Out& o, uint32_t byte)
{
    if (o.n >= o.cap) return false;
    if (lane() == 0) s[kOutStage + (o.n & 63)] = static_cast<uint8_t>(byte);
    o.n++;
    if ((o.n & 63) == 0) out_flush_full(s, o);
    return true;
}

DEV void out_finish(uint8_t* s, const Out& o)
{
    const uint32_t rem = o.n & 63;
    if (lane() < rem) o.g[(o.n & ~63u) + lane()] = s[kOutStage + lane()];
}

// ------------------------------------------------------------- range coder

struct Enc { uint32_t low, range; };

// compress.c:121-137; false = output full (whole call returns 0)
DEV bool enc_code(uint8_t* s, Enc& e, Out& o, uint32_t under, uint32_t count, uint32_t total)
{
    e.range = uni(e.range / total);
    e.low += under * e.range;
    e.range *= count;
    for (;;) {
        if ((e.low ^ (e.low + e.range)) >= kTop) {
            if (e.range >= kBot) return true;
            e.range = (0u - e.low) & (kBot - 1);
        }
        if (!out_put(s, o, e.low >> 24)) return false;
        e.range <<= 8;
        e.low <<= 8;
    }
}

struct Dec { uint32_t low, code, range, ipos, ilen; };

DEV uint32_t dec_byte(uint8_t* s, Dec& d)
{
    if (d.ipos < d.ilen) return s[kInStage + d.ipos++];
    return 0;
}

// compress.c:352 (truncated to u16 at :545/:575)
DEV uint32_t dec_read(Dec& d, uint32_t total)
{
    d.range = uni(d.range / total);
    return uni((d.code - d.low) / d.range) & 0xFFFF;
}

// compress.c:354-371
DEV void dec_code(uint8_t* s, Dec& d, uint32_t under, uint32_t count)
{
    d.low += under * d.range;
    d.range *= count;
    for (;;) {
        if ((d.low ^ (d.low + d.range)) >= kTop) {
            if (d.range >= kBot) break;
            d.range = (0u - d.low) & (kBot - 1);
        }
        d.code = (d.code << 8) | dec_byte(s, d);
        d.range <<= 8;
        d.low <<= 8;
    }
}

DEV void flag_exact(const rc_workspace_dev& ws, uint32_t pkt)
{
    if (lane() == 0) {
        const uint32_t slot = atomicAdd(&ws.counters[0], 1u);
        ws.flag_list[slot] = pkt;
    }
}

DEV void stage_in(uint8_t* s, const uint8_t* g, uint32_t len)
{
    for (uint32_t i = lane(); i < len; i += 64) s[kInStage + i] = g[i];
}

}  // namespace

// ======================================================== fast wave kernels

extern "C" __global__ __launch_bounds__(64)
void rc_compress_wave(rc_batch_dev b, rc_workspace_dev ws, uint32_t stage_bytes, uint32_t lds_bytes)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t s[];
    if (ws.sub_list && blockIdx.x >= *ws.sub_count) return;        // (a sub-list: its first sub_count packets)
    const uint32_t pkt = ws.sub_list ? ws.sub_list[blockIdx.x] : blockIdx.x;
    const uint32_t len = b.in_len[pkt];
    Out o;
    o.g = b.out + b.out_off[pkt];
    o.cap = b.out_cap[pkt];
    o.n = 0;
    if (len == 0) { if (lane() == 0) b.out_len[pkt] = 0; return; }   // compress.c:257
    if (len > stage_bytes - 8) { flag_exact(ws, pkt); return; }
    stage_in(s, b.in + b.in_off[pkt], len);

    Model m;
    m.arena_lo = kInStage + stage_bytes;
    m.arena_hi = lds_bytes & ~7u;
    m.overflow = false;
    model_reset(s, m);

    Enc e = { 0u, ~0u };
    uint32_t order = 0, b1 = 0, c2 = 0;
    bool ok = true;

#ifdef RC_WAVE_PROF
    uint64_t p2 = 0, p1 = 0, p0 = 0, pa = 0;
#endif
    uint32_t inw = 0;                                      // input bytes i & ~63 .. +63, one per lane
    for (uint32_t i = 0; i < len; ++i) {
        PROF_T(ta);
        // (a readlane instead of an LDS round trip per byte; the read past
        // len stays inside the arena that follows the staging buffer)
        if ((i & 63) == 0) inw = s[kInStage + i + lane()];
        const uint32_t v = lane_val(inw, i & 63);
        uint32_t under, cnt, nxt = 0;
        bool have_nxt = false, done = false;

        if (order >= 2) {                                  // order-2 context
            Ctx c; o2_get(s, c2, c);
            const uint32_t esc0 = c.esc, tot0 = c.tot;
            cnt = sub_update(s, m, c, 0, v, under, nullptr);
            if (m.overflow) break;
            o2_put(s, c2, c);
            if (cnt) { ok = enc_code(s, e, o, esc0 + under, cnt, tot0); done = true; }
            else if (esc0 > 0 && esc0 < tot0) ok = enc_code(s, e, o, 0, esc0, tot0);
            if (!ok) break;
        }
        PROF_T(tb);
        PROF_ADD(p2, ta, tb);
        if (!done && order >= 1) {                         // order-1 context
            Ctx c; o1_get(m, b1, c);
            const uint32_t esc0 = c.esc, tot0 = c.tot;
            cnt = sub_update(s, m, c, 1, v, under, &nxt);
            if (m.overflow) break;
            have_nxt = true;
            o1_put(m, b1, c);
            if (cnt) { ok = enc_code(s, e, o, esc0 + under, cnt, tot0); done = true; }
            else if (esc0 > 0 && esc0 < tot0) ok = enc_code(s, e, o, 0, esc0, tot0);
            if (!ok) break;
        }
        PROF_T(tc);
        PROF_ADD(p1, tb, tc);
        if (!done) {                                       // root, compress.c:318-329
            root_lookup(m, v, under, cnt);
            const uint32_t tot0 = m.rtot;
            if (cnt == 0) m.nodes++;
            root_add(m, v);
            ok = enc_code(s, e, o, 1 + under, 1 + cnt, tot0);
            if (!ok) break;
            m.rtot = (m.rtot + kRootDelta) & 0xFFFF;
            if (1 + cnt > 0xFF - 2 * kRootDelta + 1 || m.rtot > kTotalLimit) root_rescale(m);
        }
        PROF_T(td);
        PROF_ADD(p0, tc, td);
        // advance, compress.c:331-336
        if (order >= 1) {
            if (!have_nxt) {
                Ctx c; o1_get(m, b1, c);
                const Find f = blk_find(s, c, v);
                nxt = uni(ids(s, c.off, cap_of(c.len, 2))[f.k]);
            }
            c2 = nxt;
        }
        if (order < 2) ++order;
        b1 = v;
        if (m.nodes >= kMaxNodes) { model_reset(s, m); order = 0; }
        PROF_T(te);
        PROF_ADD(pa, td, te);
    }
#ifdef RC_WAVE_PROF
    if (lane() == 0) {
        atomicAdd(&g_wave_prof[0], (unsigned long long) p2);
        atomicAdd(&g_wave_prof[1], (unsigned long long) p1);
        atomicAdd(&g_wave_prof[2], (unsigned long long) p0);
        atomicAdd(&g_wave_prof[3], (unsigned long long) pa);
        atomicAdd(&g_wave_prof[4], (unsigned long long) len);
    }
#endif

    if (m.overflow) { flag_exact(ws, pkt); return; }
    if (ok) {                                              // flush, compress.c:139-146
        while (e.low) {
            if (!out_put(s, o, e.low >> 24)) { ok = false; break; }
            e.low <<= 8;
        }
    }
    if (ok) out_finish(s, o);
    if (lane() == 0) b.out_len[pkt] = ok ? o.n : 0u;
}

extern "C" __global__ __launch_bounds__(64)
void rc_decompress_wave(rc_batch_dev b, rc_workspace_dev ws, uint32_t stage_bytes, uint32_t lds_bytes)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t s[];
    if (ws.sub_list && blockIdx.x >= *ws.sub_count) return;        // (a sub-list: its first sub_count packets)
    const uint32_t pkt = ws.sub_list ? ws.sub_list[blockIdx.x] : blockIdx.x;
    const uint32_t len = b.in_len[pkt];
    Out o;
    o.g = b.out + b.out_off[pkt];
    o.cap = b.out_cap[pkt];
    o.n = 0;
    if (len == 0) { if (lane() == 0) b.out_len[pkt] = 0; return; }   // compress.c:513
    if (len > stage_bytes - 8) { flag_exact(ws, pkt); return; }
    stage_in(s, b.in + b.in_off[pkt], len);

    Model m;
    m.arena_lo = kInStage + stage_bytes;
    m.arena_hi = lds_bytes & ~7u;
    m.overflow = false;
    model_reset(s, m);

    Dec d = { 0u, 0u, ~0u, 0u, len };
    for (int k = 0; k < 4; ++k) d.code = (d.code << 8) | dec_byte(s, d);   // seed, compress.c:344-350

    uint32_t order = 0, b1 = 0, c2 = 0;
    bool fail = false, anomaly = false;

    for (;;) {
        uint32_t v = 0, under = 0, cnt = 0, nxt = 0;
        int at = -1;                    // context level that produced the symbol
        bool have_nxt = false;

        if (order >= 2) {
            Ctx c; o2_get(s, c2, c);
            if (c.esc > 0 && c.esc < c.tot) {
                uint32_t code = dec_read(d, c.tot);
                if (code < c.esc) {
                    dec_code(s, d, 0, c.esc);
                } else {
                    code -= c.esc;
                    uint32_t k;
                    if (!blk_search(s, c, code, k, v, under, cnt)) { fail = true; break; }
                    blk_bump(s, c, k, kSubDelta);
                    dec_code(s, d, c.esc + under, cnt);
                    c.tot = (c.tot + kSubDelta) & 0xFFFF;
                    if (cnt > 0xFF - 2 * kSubDelta || c.tot > kTotalLimit) blk_rescale(s, c);
                    o2_put(s, c2, c);
                    at = 2;
                }
            }
        }
        if (at < 0 && order >= 1) {
            Ctx c; o1_get(m, b1, c);
            if (c.esc > 0 && c.esc < c.tot) {
                uint32_t code = dec_read(d, c.tot);
                if (code < c.esc) {
                    dec_code(s, d, 0, c.esc);
                } else {
                    code -= c.esc;
                    uint32_t k;
                    if (!blk_search(s, c, code, k, v, under, cnt)) { fail = true; break; }
                    blk_bump(s, c, k, kSubDelta);
                    nxt = uni(ids(s, c.off, cap_of(c.len, 2))[k]);
                    have_nxt = true;
                    dec_code(s, d, c.esc + under, cnt);
                    c.tot = (c.tot + kSubDelta) & 0xFFFF;
                    if (cnt > 0xFF - 2 * kSubDelta || c.tot > kTotalLimit) blk_rescale(s, c);
                    o1_put(m, b1, c);
                    at = 1;
                }
            }
        }
        if (at < 0) {                                      // root, compress.c:570-596
            const uint32_t tot0 = m.rtot;
            uint32_t code = dec_read(d, tot0);
            if (code < 1) { dec_code(s, d, 0, 1); break; }          // escape at root = end
            code -= 1;
            if (code >= tot0 - 1) { anomaly = true; break; }       // past symbol 255: exact path
            const uint32_t l = lane();
            const uint64_t hit = ballot(code < 4 * l + 4 + (m.rcum23 >> 16));
            const uint32_t L = static_cast<uint32_t>(__builtin_ctzll(hit));
            const uint32_t a = lane_val(m.rcum01, L), bb = lane_val(m.rcum23, L);
            const uint32_t base = 4 * L;
            uint32_t j;
            if (code < base + 1 + (a & 0xFFFF)) j = 0;
            else if (code < base + 2 + (a >> 16)) j = 1;
            else if (code < base + 3 + (bb & 0xFFFF)) j = 2;
            else j = 3;
            v = base + j;
            root_lookup(m, v, under, cnt);
            if (cnt == 0) m.nodes++;
            root_add(m, v);
            dec_code(s, d, 1 + under, 1 + cnt);
            m.rtot = (m.rtot + kRootDelta) & 0xFFFF;
            if (1 + cnt > 0xFF - 2 * kRootDelta + 1 || m.rtot > kTotalLimit) root_rescale(m);
            at = 0;
        }
        // patch the higher contexts, compress.c:598-615
        if (order >= 2 && at < 2) {
            Ctx c; o2_get(s, c2, c);
            sub_update(s, m, c, 0, v, under, nullptr);
            if (m.overflow) break;
            o2_put(s, c2, c);
        }
        if (order >= 1 && at < 1) {
            Ctx c; o1_get(m, b1, c);
            sub_update(s, m, c, 1, v, under, &nxt);
            if (m.overflow) break;
            have_nxt = true;
            o1_put(m, b1, c);
        }
        if (!out_put(s, o, v)) { fail = true; break; }     // compress.c:617
        if (order >= 1) {
            if (!have_nxt) {
                Ctx c; o1_get(m, b1, c);
                const Find f = blk_find(s, c, v);
                nxt = uni(ids(s, c.off, cap_of(c.len, 2))[f.k]);
            }
            c2 = nxt;
        }
        if (order < 2) ++order;
        b1 = v;
        if (m.nodes >= kMaxNodes) { model_reset(s, m); order = 0; }
    }

    if (m.overflow || anomaly) { flag_exact(ws, pkt); return; }
    if (!fail) out_finish(s, o);
    if (lane() == 0) b.out_len[pkt] = fail ? 0u : o.n;
}

// ====================================================== exact lane kernels
// compress.c's own binary-tree model, one packet per lane, pool in global.

namespace {

struct XNode {               // compress.c:9-22 (absolute child indices)
    uint8_t value, count;
    uint16_t under, left, right, child, escapes, total, parent;
};

struct XPool { XNode* n; uint32_t next; };

DEV uint16_t x_new(XPool& p, uint32_t value, uint32_t count)
{
    const uint16_t id = static_cast<uint16_t>(p.next++);
    XNode z;
    z.value = static_cast<uint8_t>(value); z.count = static_cast<uint8_t>(count);
    z.under = static_cast<uint16_t>(count);
    z.left = z.right = z.child = z.escapes = z.total = z.parent = 0;
    p.n[id] = z;
    return id;
}

DEV void x_root(XPool& p)
{
    const uint16_t id = x_new(p, 0, 0);
    p.n[id].escapes = 1;
    p.n[id].total = 1 + 256;
}

// compress.c:90-112.  The reference recurses down left links; here the
// recursion frames live in the packet's global scratch (after the 4096 nodes)
// because a corrupt stream can grow a context tree up to 4094 nodes deep.
struct XFrame { uint16_t node, sum; uint32_t state; };

DEV void x_rescale(XNode* n, uint16_t ctx, uint32_t minimum)
{
    uint32_t total = 0;
    if (n[ctx].child) {
        XFrame* fr = reinterpret_cast<XFrame*>(n + 4096);
        int fp = 0;
        fr[0].node = n[ctx].child; fr[0].sum = 0; fr[0].state = 0;
        uint16_t ret = 0;
        for (;;) {
            XFrame& f = fr[fp];
            XNode& s = n[f.node];
            if (f.state == 0) {                      // enter node: halve, descend left
                s.count = static_cast<uint8_t>(s.count - (s.count >> 1));
                s.under = s.count;
                if (s.left) {
                    f.state = 1; ++fp;
                    fr[fp].node = s.left; fr[fp].sum = 0; fr[fp].state = 0;
                    continue;
                }
            } else {                                 // back from the left subtree
                s.under = static_cast<uint16_t>(s.under + ret);
            }
            f.sum = static_cast<uint16_t>(f.sum + s.under);
            if (s.right) { f.node = s.right; f.state = 0; continue; }
            ret = f.sum;
            if (fp == 0) break;
            --fp;
        }
        total = ret;
    }
    n[ctx].total = static_cast<uint16_t>(total);
    n[ctx].escapes = static_cast<uint16_t>(n[ctx].escapes - (n[ctx].escapes >> 1));
    n[ctx].total = static_cast<uint16_t>(n[ctx].total + n[ctx].escapes + 256 * minimum);
}

DEV uint16_t x_encode(XPool& p, uint16_t ctx, uint32_t value, uint16_t& under_, uint16_t& count_,
                      uint32_t update, uint32_t minimum)
{
    XNode* n = p.n;
    uint16_t under = static_cast<uint16_t>(value * minimum), count = static_cast<uint16_t>(minimum), id;
    if (!n[ctx].child) {
        id = x_new(p, value, update);
        n[ctx].child = id;
    } else {
        uint16_t cur = n[ctx].child;
        for (;;) {
            XNode& s = n[cur];
            if (value < s.value) {
                s.under = static_cast<uint16_t>(s.under + update);
                if (s.left) { cur = s.left; continue; }
                id = x_new(p, value, update);
                n[cur].left = id;
            } else if (value > s.value) {
                under = static_cast<uint16_t>(under + s.under);
                if (s.right) { cur = s.right; continue; }
                id = x_new(p, value, update);
                n[cur].right = id;
            } else {
                count = static_cast<uint16_t>(count + s.count);
                under = static_cast<uint16_t>(under + s.under - s.count);
                s.under = static_cast<uint16_t>(s.under + update);
                s.count = static_cast<uint8_t>(s.count + update);
                id = cur;
            }
            break;
        }
    }
    under_ = under; count_ = count;
    return id;
}

struct XEnc { uint32_t low, range; uint8_t* out; uint32_t n, cap; };

DEV bool x_enc(XEnc& e, uint32_t under, uint32_t count, uint32_t total)
{
    e.range /= total; e.low += under * e.range; e.range *= count;
    for (;;) {
        if ((e.low ^ (e.low + e.range)) >= kTop) {
            if (e.range >= kBot) return true;
            e.range = (0u - e.low) & (kBot - 1);
        }
        if (e.n >= e.cap) return false;
        e.out[e.n++] = static_cast<uint8_t>(e.low >> 24);
        e.range <<= 8; e.low <<= 8;
    }
}

DEV uint32_t x_compress(XNode* pool, const uint8_t* in, uint32_t len, uint8_t* out, uint32_t cap)
{
    if (len == 0) return 0;
    XPool p = { pool, 0 };
    XEnc e = { 0u, ~0u, out, 0u, cap };
    uint16_t predicted = 0;
    uint32_t order = 0;
    x_root(p);
    for (uint32_t i = 0; i < len; ++i) {
        XNode* n = p.n;
        const uint32_t value = in[i];
        uint16_t* link = &predicted;
        uint16_t under, count, total, ctx, sym;
        bool stop = false;
        for (ctx = predicted; ctx != 0; ctx = n[ctx].parent) {
            sym = x_encode(p, ctx, value, under, count, kSubDelta, 0);
            *link = sym; link = &n[sym].parent;
            total = n[ctx].total;
            if (count > 0) {
                if (!x_enc(e, n[ctx].escapes + (uint32_t) under, count, total)) return 0;
            } else {
                if (n[ctx].escapes > 0 && n[ctx].escapes < total)
                    if (!x_enc(e, 0, n[ctx].escapes, total)) return 0;
                n[ctx].escapes = static_cast<uint16_t>(n[ctx].escapes + kSubEscDelta);
                n[ctx].total = static_cast<uint16_t>(n[ctx].total + kSubEscDelta);
            }
            n[ctx].total = static_cast<uint16_t>(n[ctx].total + kSubDelta);
            if (count > 0xFF - 2 * kSubDelta || n[ctx].total > kTotalLimit) x_rescale(n, ctx, 0);
            if (count > 0) { stop = true; break; }
        }
        if (!stop) {
            sym = x_encode(p, 0, value, under, count, kRootDelta, 1);
            *link = sym;
            total = n[0].total;
            if (!x_enc(e, n[0].escapes + (uint32_t) under, count, total)) return 0;
            n[0].total = static_cast<uint16_t>(n[0].total + kRootDelta);
            if (count > 0xFF - 2 * kRootDelta + 1 || n[0].total > kTotalLimit) x_rescale(n, 0, 1);
        }
        if (order >= 2) predicted = n[predicted].parent; else ++order;
        if (p.next >= kMaxNodes) { p.next = 0; x_root(p); predicted = 0; order = 0; }
    }
    while (e.low) {
        if (e.n >= e.cap) return 0;
        e.out[e.n++] = static_cast<uint8_t>(e.low >> 24);
        e.low <<= 8;
    }
    return e.n;
}

struct XDec { uint32_t low, code, range; const uint8_t* ip; const uint8_t* ie; };

DEV void x_dec(XDec& d, uint32_t under, uint32_t count)
{
    d.low += under * d.range; d.range *= count;
    for (;;) {
        if ((d.low ^ (d.low + d.range)) >= kTop) {
            if (d.range >= kBot) break;
            d.range = (0u - d.low) & (kBot - 1);
        }
        d.code <<= 8;
        if (d.ip < d.ie) d.code |= *d.ip++;
        d.range <<= 8; d.low <<= 8;
    }
}

DEV uint32_t x_decompress(XNode* pool, const uint8_t* in, uint32_t len, uint8_t* out, uint32_t cap)
{
    if (len == 0) return 0;
    XPool p = { pool, 0 };
    x_root(p);
    XDec d = { 0u, 0u, ~0u, in, in + len };
    for (int k = 0; k < 4; ++k) { d.code <<= 8; if (d.ip < d.ie) d.code |= *d.ip++; }
    uint16_t predicted = 0;
    uint32_t order = 0, on = 0;
    for (;;) {
        XNode* n = p.n;
        uint16_t* link = &predicted;
        uint16_t under = 0, count = 0, total, code, bottom = 0, ctx, sym = 0;
        uint32_t value = 0;
        bool decoded = false;
        for (ctx = predicted; ctx != 0; ctx = n[ctx].parent) {
            if (n[ctx].escapes <= 0) continue;
            total = n[ctx].total;
            if (n[ctx].escapes >= total) continue;
            d.range /= total;
            code = static_cast<uint16_t>((d.code - d.low) / d.range);
            if (code < n[ctx].escapes) { x_dec(d, 0, n[ctx].escapes); continue; }
            code = static_cast<uint16_t>(code - n[ctx].escapes);
            // TRY_DECODE, compress.c:373-416 (minimum 0)
            if (!n[ctx].child) return 0;
            uint16_t cur = n[ctx].child, u = 0;
            for (;;) {
                XNode& s = n[cur];
                const uint16_t after = static_cast<uint16_t>(u + s.under), before = s.count;
                if (code >= after) {
                    u = static_cast<uint16_t>(u + s.under);
                    if (s.right) { cur = s.right; continue; }
                    return 0;
                } else if ((int) code < (int) after - (int) before) {
                    s.under = static_cast<uint16_t>(s.under + kSubDelta);
                    if (s.left) { cur = s.left; continue; }
                    return 0;
                }
                value = s.value;
                count = s.count;
                under = static_cast<uint16_t>(after - before);
                s.under = static_cast<uint16_t>(s.under + kSubDelta);
                s.count = static_cast<uint8_t>(s.count + kSubDelta);
                sym = cur;
                break;
            }
            bottom = sym;
            x_dec(d, n[ctx].escapes + (uint32_t) under, count);
            n[ctx].total = static_cast<uint16_t>(n[ctx].total + kSubDelta);
            if (count > 0xFF - 2 * kSubDelta || n[ctx].total > kTotalLimit) x_rescale(n, ctx, 0);
            decoded = true;
            break;
        }
        if (!decoded) {
            ctx = 0;
            total = n[0].total;
            d.range /= total;
            code = static_cast<uint16_t>((d.code - d.low) / d.range);
            if (code < n[0].escapes) { x_dec(d, 0, n[0].escapes); break; }
            code = static_cast<uint16_t>(code - n[0].escapes);
            // ROOT_DECODE, compress.c:418-438 (minimum 1)
            uint16_t u = 0;
            count = 1;
            if (!n[0].child) {
                value = code & 0xFF;
                under = code;
                sym = x_new(p, value, kRootDelta);
                n[0].child = sym;
            } else {
                uint16_t cur = n[0].child;
                for (;;) {
                    XNode& s = n[cur];
                    const uint16_t after = static_cast<uint16_t>(u + s.under + (s.value + 1));
                    const uint16_t before = static_cast<uint16_t>(s.count + 1);
                    if (code >= after) {
                        u = static_cast<uint16_t>(u + s.under);
                        if (s.right) { cur = s.right; continue; }
                        value = (s.value + 1 + (code - after)) & 0xFF;
                        under = code;
                        sym = x_new(p, value, kRootDelta);
                        n[cur].right = sym;
                    } else if ((int) code < (int) after - (int) before) {
                        s.under = static_cast<uint16_t>(s.under + kRootDelta);
                        if (s.left) { cur = s.left; continue; }
                        value = (s.value - 1 - ((int) after - (int) before - (int) code - 1)) & 0xFF;
                        under = code;
                        sym = x_new(p, value, kRootDelta);
                        n[cur].left = sym;
                    } else {
                        value = s.value;
                        count = static_cast<uint16_t>(1 + s.count);
                        under = static_cast<uint16_t>(after - before);
                        s.under = static_cast<uint16_t>(s.under + kRootDelta);
                        s.count = static_cast<uint8_t>(s.count + kRootDelta);
                        sym = cur;
                    }
                    break;
                }
            }
            bottom = sym;
            x_dec(d, n[0].escapes + (uint32_t) under, count);
            n[0].total = static_cast<uint16_t>(n[0].total + kRootDelta);
            if (count > 0xFF - 2 * kRootDelta + 1 || n[0].total > kTotalLimit) x_rescale(n, 0, 1);
        }
        // patch, compress.c:598-615
        for (uint16_t pc = predicted; pc != ctx; pc = n[pc].parent) {
            uint16_t pu, pcnt;
            const uint16_t ps = x_encode(p, pc, value, pu, pcnt, kSubDelta, 0);
            *link = ps; link = &n[ps].parent;
            if (pcnt <= 0) {
                n[pc].escapes = static_cast<uint16_t>(n[pc].escapes + kSubEscDelta);
                n[pc].total = static_cast<uint16_t>(n[pc].total + kSubEscDelta);
            }
            n[pc].total = static_cast<uint16_t>(n[pc].total + kSubDelta);
            if (pcnt > 0xFF - 2 * kSubDelta || n[pc].total > kTotalLimit) x_rescale(n, pc, 0);
        }
        *link = bottom;
        if (on >= cap) return 0;
        out[on++] = static_cast<uint8_t>(value);
        if (order >= 2) predicted = n[predicted].parent; else ++order;
        if (p.next >= kMaxNodes) { p.next = 0; x_root(p); predicted = 0; order = 0; }
    }
    return on;
}

}  // namespace

extern "C" __global__ __launch_bounds__(64)
void rc_compress_exact(rc_batch_dev b, rc_workspace_dev ws)
{
    const uint32_t cnt = ws.counters[0];
    const uint32_t tid = blockIdx.x * 64 + threadIdx.x;
    XNode* pool = reinterpret_cast<XNode*>(static_cast<uint8_t*>(ws.exact_pool) + (size_t) tid * RC_EXACT_POOL_BYTES);
    for (uint32_t i = tid; i < cnt; i += gridDim.x * 64) {
        const uint32_t pkt = ws.flag_list[i];
        b.out_len[pkt] = x_compress(pool, b.in + b.in_off[pkt], b.in_len[pkt],
                                    b.out + b.out_off[pkt], b.out_cap[pkt]);
    }
}

extern "C" __global__ __launch_bounds__(64)
void rc_decompress_exact(rc_batch_dev b, rc_workspace_dev ws)
{
    const uint32_t cnt = ws.counters[0];
    const uint32_t tid = blockIdx.x * 64 + threadIdx.x;
    XNode* pool = reinterpret_cast<XNode*>(static_cast<uint8_t*>(ws.exact_pool) + (size_t) tid * RC_EXACT_POOL_BYTES);
    for (uint32_t i = tid; i < cnt; i += gridDim.x * 64) {
        const uint32_t pkt = ws.flag_list[i];
        b.out_len[pkt] = x_decompress(pool, b.in + b.in_off[pkt], b.in_len[pkt],
                                      b.out + b.out_off[pkt], b.out_cap[pkt]);
    }
}

// ================================================================ launchers

namespace {

constexpr uint32_t kMaxLds = 65536;

uint32_t stage_bytes_for(uint32_t max_len) { return ((max_len + 8 + 15) / 16) * 16; }

constexpr uint32_t kMinArena = 4096;

uint64_t arena_bytes_for(uint32_t model_bytes_bound)
{
    const uint64_t a = 22ull * model_bytes_bound + 2048;
    return a < kMinArena ? kMinArena : a;
}

uint32_t lds_bytes_for(uint32_t max_len)
{
    // arena: <= 18 B of model per input byte in the worst case (o2 header 8 +
    // o2 entry 4 + o1 entry 6) plus power-of-two slack; never below the 4 KB
    // the launcher requires of a usable arena.
    uint64_t arena = arena_bytes_for(max_len);
    uint64_t total = kInStage + stage_bytes_for(max_len) + arena;
    if (total > kMaxLds) total = kMaxLds;
    return static_cast<uint32_t>(total & ~15ull);
}

}  // namespace

extern "C" uint32_t rc_hip_lds_bytes(uint32_t max_len) { return lds_bytes_for(max_len); }

extern "C" int rc_hip_lane_launch(int decompress, const rc_batch_dev* b, const rc_workspace_dev* ws,
                                  void* stream);   // rc_route.hip

extern "C" const char* rc_hip_fast_kernel_name(int decompress, uint32_t kernel)
{
    if (kernel == RC_KERNEL_WAVE) return decompress ? "rc_decompress_wave" : "rc_compress_wave";
    return decompress ? "rc_decompress_lane3" : "rc_compress_lane3";
}

constexpr uint32_t kLdsPerCu = 160 * 1024;   // gfx950

// LDS per wavefront of the wave kernels.  The decoder's model grows with the
// bytes it produces, not the bytes it reads (max_len bounds the input): its
// arena is sized by the output bound when the caller knows one (max_out, the
// host-pointer batches), else it takes the largest arena.
uint32_t wave_lds(bool decompress, uint32_t max_len, uint32_t max_out)
{
    if (!decompress) return lds_bytes_for(max_len);
    if (max_out == 0) return kMaxLds;
    uint64_t total = kInStage + stage_bytes_for(max_len) + arena_bytes_for(max_out);
    if (total > kMaxLds) total = kMaxLds;
    return static_cast<uint32_t>(total & ~15ull);
}

// Batches that fit on the chip in one wave per packet (the per-datagram
// drop-in calls and a live host's send / receive passes among them) ran on
// the wavefront-per-packet kernel: a packet's byte chain runs there with its
// model in LDS, 1.4-2.9x sooner than on one lane of the v3 lane kernels
// (tools/smallbatch.py).  The fast kernels in front of those are faster
// still for such batches (small_route): compress takes the two-pass encoder
// (one 1200-B datagram: 0.53 ms against 2.4 random, 0.62 against 1.5 game
// state), decompress the record-light decoder, with the wave kernel (not the
// lane kernels) taking what it leaves (1.5 ms against 2.9 random; game state
// leaves it early).  Larger batches are throughput work: lanes.
static bool small_batch(bool decompress, const rc_batch_dev* b, const rc_workspace_dev* ws, uint32_t& lds_w)
{
    const uint32_t max_len = b->max_len ? b->max_len : 4096;
    lds_w = wave_lds(decompress, max_len, b->max_out);
    // The decoder caps at 4 wavefronts per CU: with a right-sized model 5 fit,
    // but 1280 random packets then decode slower than on the lanes (5.9 vs
    // 3.9 ms, profiles/r1h_smallbatch.log).
    uint32_t per_cu = kLdsPerCu / lds_w ? kLdsPerCu / lds_w : 1u;
    if (decompress && per_cu > 4u) per_cu = 4u;
    const uint32_t resident = ws->cus * per_cu;
    // (not min(): on the host it resolves to the int overload, and small_max
    // RC_SMALL_AUTO would read as -1)
    return ws->kernel == RC_KERNEL_LANE3 && b->n <= resident && b->n <= ws->small_max;
}

// a small batch: 0 = the wave kernel, 1 = the lane path (two-pass encoder),
// 2 = the record-light decoder, then the wave kernel on what it leaves
static int small_route(bool decompress, const rc_workspace_dev* ws)
{
    if (ws->kernel == RC_KERNEL_WAVE || ws->small_max != RC_SMALL_AUTO) return 0;   // (ENET_RC_SMALL_BATCH=n: as set)
    if (!decompress) return ws->enc2_on ? 1 : 0;
    return ws->fast_dec && ws->lane_active == 64 ? 2 : 0;
}

extern "C" int rc_hip_uses_lanes(int decompress, const rc_batch_dev* b, const rc_workspace_dev* ws)
{
    uint32_t lds_w;
    return ws->kernel != RC_KERNEL_WAVE &&
           (!small_batch(decompress != 0, b, ws, lds_w) || small_route(decompress != 0, ws) != 0);
}

// The wave kernel over the sub-list ws->sub_list (count ws->sub_count[0],
// at most b->n): a grid of b->n blocks, the ones past the count leave at once.
extern "C" int rc_hip_wave_tail_launch(int decompress, const rc_batch_dev* b, const rc_workspace_dev* ws,
                                       void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    const uint32_t max_len = b->max_len ? b->max_len : 4096;
    uint32_t lds = wave_lds(decompress != 0, max_len, b->max_out);
    uint32_t stage = stage_bytes_for(max_len);
    if (stage + kInStage + kMinArena > lds) { stage = 16; lds = 16384; }
    if (decompress)
        hipLaunchKernelGGL(rc_decompress_wave, dim3(b->n), dim3(64), lds, st, *b, *ws, stage, lds);
    else
        hipLaunchKernelGGL(rc_compress_wave, dim3(b->n), dim3(64), lds, st, *b, *ws, stage, lds);
    return static_cast<int>(hipGetLastError());
}

// The control block (counters, length bins, wide-list counters; rc_host.c)
// cleared by one workgroup: 4.6 us, as the runtime's fill (hipMemsetAsync,
// ENET_RC_CTL_FILL=1) of the same 3 KB (profiles/r6/r6g_ctl_clear_c2.txt).
static_assert(RC_CTL_WORDS <= 4 * 256, "rc_ctl_clear: one uint4 per thread");
extern "C" __global__ __launch_bounds__(256) void rc_ctl_clear(uint32_t* ctl)
{
    if (4 * threadIdx.x < RC_CTL_WORDS) reinterpret_cast<uint4*>(ctl)[threadIdx.x] = make_uint4(0u, 0u, 0u, 0u);
}

static int launch(bool decompress, const rc_batch_dev* b, const rc_workspace_dev* ws, void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (b->n == 0) return 0;
    if (b->n > ws->n_cap) return static_cast<int>(hipErrorInvalidValue);
    // the counters and the length bins (one block, rc_host.c)
    static const bool fill = getenv("ENET_RC_CTL_FILL") != nullptr;     // (A/B: the runtime's fill)
    hipError_t err = hipSuccess;
    if (fill) {
        err = hipMemsetAsync(ws->counters, 0, RC_CTL_WORDS * sizeof(uint32_t), st);
    } else {
        hipLaunchKernelGGL(rc_ctl_clear, dim3(1), dim3(256), 0, st, ws->counters);
        err = hipGetLastError();
    }
    if (err != hipSuccess) return static_cast<int>(err);
    const uint32_t max_len = b->max_len ? b->max_len : 4096;
    uint32_t lds_w;
    const bool small = small_batch(decompress, b, ws, lds_w);
    static const bool debug = getenv("ENET_RC_DEBUG") != nullptr;
    if (debug)
        fprintf(stderr, "enet_rc: %s n=%u max_len=%u cus=%u lds=%u small_max=%u -> %s\n",
                decompress ? "decompress" : "compress", b->n, max_len, ws->cus, lds_w,
                ws->small_max, small || ws->kernel == RC_KERNEL_WAVE ? "wave" : "lanes");
    // (the decoder's tail on the wave kernel up to twice what fits at once: a
    // second round of wave blocks still beats the lane kernels' full packet
    // time for up to ~3000 low-entropy packets, profiles/r5_smallbatch.log)
    uint32_t lds2;
    rc_batch_dev half = *b;
    half.n = (b->n + 1) / 2;
    const bool tail2 = decompress && small_batch(decompress, &half, ws, lds2) && small_route(decompress, ws) == 2;
    const int route = small ? small_route(decompress, ws) : tail2 ? 2 : 1;
    if (ws->kernel != RC_KERNEL_WAVE && route != 0) {
        rc_workspace_dev w = *ws;
        w.wave_tail = route == 2 ? 1u : 0u;
        const int rc = rc_hip_lane_launch(decompress ? 1 : 0, b, &w, stream);
        if (rc != 0) return rc;
    } else {
        uint32_t stage = stage_bytes_for(max_len);
        uint32_t lds = lds_w;
        if (stage + kInStage + kMinArena > lds) {   // absurd max_len: everything goes exact
            stage = 16; lds = 16384;
        }
        if (decompress)
            hipLaunchKernelGGL(rc_decompress_wave, dim3(b->n), dim3(64), lds, st, *b, *ws, stage, lds);
        else
            hipLaunchKernelGGL(rc_compress_wave, dim3(b->n), dim3(64), lds, st, *b, *ws, stage, lds);
        err = hipGetLastError();
        if (err != hipSuccess) return static_cast<int>(err);
    }
    const uint32_t blocks = ws->exact_slots / 64 ? ws->exact_slots / 64 : 1;
    if (decompress)
        hipLaunchKernelGGL(rc_decompress_exact, dim3(blocks), dim3(64), 0, st, *b, *ws);
    else
        hipLaunchKernelGGL(rc_compress_exact, dim3(blocks), dim3(64), 0, st, *b, *ws);
    return static_cast<int>(hipGetLastError());
}

extern "C" int rc_hip_compress(const rc_batch_dev* b, const rc_workspace_dev* ws, void* stream)
{
    return launch(false, b, ws, stream);
}

extern "C" int rc_hip_decompress(const rc_batch_dev* b, const rc_workspace_dev* ws, void* stream)
{
    return launch(true, b, ws, stream);
}
