// rc_lane.hip -- lane-per-packet range-coder kernels for MI355X (gfx950).
//
// Same semantics as compress.c (enet_range_coder_compress :246-342,
// enet_range_coder_decompress :498-627), bit-exact.
//
// Why one packet per LANE: the coder is a byte-serial dependency chain.  With
// one packet per wavefront (rc_kernels.hip "wave" kernels) that chain is
// wave-uniform work, i.e. it runs on the CU's scalar unit, which every
// resident wave shares; rocprof showed those kernels issuing ~500 SALU
// instructions per byte (profiles/r1_v1wave_pmc_sq.json).  Here 64 packets
// advance in lock-step in one wave, so the same arithmetic is one VALU
// instruction for 64 packets.
//
// Model layout (only {count[v], escapes, total} per context and the node
// count are observable):
//   order 0 (root): per lane in LDS, counts[256] (u8) + C[16] (u16 cumulative
//       count at the end of each 16-symbol group) -> lookups are 1-2 LDS
//       reads + byte-SAD sums, no tree walk.
//   order 1: 256 records of 64 B, direct-mapped by the previous byte, in a
//       per-lane HBM region; order 2: 32-B records bump-allocated in the same
//       region and reached through links stored in the entries (compress.c's
//       suffix links, `parent`).  A record = 16-B header {esc, tot, len, ext}
//       + inline sorted entries {value:8 | count:8 | link:16}; contexts that
//       outgrow the inline slots move their entries to an extension block.
//   Every byte therefore costs one dependent HBM round trip (the order-1 and
//   order-2 records are loaded together), not a BST walk.
//
// Packets this model cannot reproduce -- corrupt streams whose root code
// points past symbol 255 (compress.c:427-438 then depends on tree shape) --
// and packets whose region overflows are appended to the exact-path list
// (rc_kernels.hip), which re-runs compress.c's binary-tree model.

#ifndef RC_LANE_HOST_TEST
#include <hip/hip_runtime.h>
#else
#include "lane_host_shim.h"   // tests/proto: host build of the per-lane logic (test only)
#endif
#include <stdint.h>

#include "rc_abi_internal.h"

#define DEV __device__ __forceinline__

namespace {

constexpr uint32_t kTop = 1u << 24;          // compress.c:27
constexpr uint32_t kBot = 1u << 16;          // compress.c:28
constexpr uint32_t kRootDelta = 3;           // compress.c:30
constexpr uint32_t kSubDelta = 2;            // compress.c:35
constexpr uint32_t kSubEscDelta = 5;         // compress.c:36
constexpr uint32_t kMaxNodes = 4096 - 2;     // compress.c:150
constexpr uint32_t kTotalLimit = kBot - 0x100;

constexpr uint32_t kBlock = 256;             // lanes (packets) per workgroup
constexpr uint32_t kRootStride = 304;        // LDS bytes per lane; 76 dwords (76/4 odd: b128 conflict-free)
constexpr uint32_t kO1Rec = 64, kO1Inl = 12, kO1MinLog = 5;   // ext blocks start at 32 entries
constexpr uint32_t kO2Rec = 32, kO2Inl = 4, kO2MinLog = 3;    // ext blocks start at 8 entries
constexpr uint32_t kArenaBase = 256 * kO1Rec;                 // order-2 records + ext blocks follow

DEV uint32_t val_of(uint32_t e) { return e & 0xFF; }
DEV uint32_t cnt_of(uint32_t e) { return (e >> 8) & 0xFF; }
DEV uint32_t sad(uint32_t x, uint32_t acc) { return __builtin_amdgcn_sad_u8(x, 0u, acc); }
DEV uint32_t pick4(uint32_t i, const uint4& q) { return i == 0 ? q.x : i == 1 ? q.y : i == 2 ? q.z : q.w; }

// ------------------------------------------------------------ order 0 (LDS)

DEV void root_clear(uint8_t* r)
{
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int i = 0; i < 18; ++i) reinterpret_cast<uint4*>(r)[i] = z;
}

DEV uint32_t root_c(const uint8_t* r, uint32_t g) { return reinterpret_cast<const uint16_t*>(r + 256)[g]; }

// under = v * 1 + sum of counts below v; cnt = count[v] (compress.c:159-199, minimum 1)
DEV void root_lookup(const uint8_t* r, uint32_t v, uint32_t& under, uint32_t& cnt)
{
    const uint32_t g = v >> 4, j = v & 15;
    const uint4 q = *reinterpret_cast<const uint4*>(r + 16 * g);
    const uint32_t below = g ? root_c(r, g - 1) : 0u;
    uint32_t within = 0;
#pragma unroll
    for (uint32_t d = 0; d < 4; ++d) {
        const uint32_t nb = j > 4 * d ? min(j - 4 * d, 4u) : 0u;
        const uint32_t mask = nb >= 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1u);
        within = sad(pick4(d, q) & mask, within);
    }
    cnt = (pick4(j >> 2, q) >> (8 * (j & 3))) & 0xFF;
    under = v + below + within;
}

DEV void root_add(uint8_t* r, uint32_t v, uint32_t cnt)
{
    r[v] = static_cast<uint8_t>(cnt + kRootDelta);
    const uint32_t g = v >> 4;
    uint4* cp = reinterpret_cast<uint4*>(r + 256);
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
        uint4 c = cp[h];
        uint32_t* w = reinterpret_cast<uint32_t*>(&c);
#pragma unroll
        for (uint32_t d = 0; d < 4; ++d) {
            const uint32_t g0 = 8 * h + 2 * d;
            w[d] += (g0 >= g ? kRootDelta : 0u) | (g0 + 1 >= g ? (kRootDelta << 16) : 0u);
        }
        cp[h] = c;
    }
}

// first symbol whose interval [v + C(<v), v + 1 + C(<=v)) holds code; code < 256 + sum
DEV uint32_t root_search(const uint8_t* r, uint32_t code)
{
    const uint4 c0 = reinterpret_cast<const uint4*>(r + 256)[0];
    const uint4 c1 = reinterpret_cast<const uint4*>(r + 256)[1];
    uint32_t g = 0, prev = 0;
#pragma unroll
    for (uint32_t t = 0; t < 16; ++t) {
        const uint32_t w = pick4((t >> 1) & 3, t < 8 ? c0 : c1);
        const uint32_t ct = (t & 1) ? (w >> 16) : (w & 0xFFFF);
        const bool below = 16 * (t + 1) + ct <= code;
        g += below ? 1u : 0u;
        prev = below ? ct : prev;
    }
    const uint4 q = *reinterpret_cast<const uint4*>(r + 16 * g);
    uint32_t run = 16 * g + prev, j = 15;
    bool found = false;
#pragma unroll
    for (uint32_t t = 0; t < 16; ++t) {
        run += 1 + ((pick4(t >> 2, q) >> (8 * (t & 3))) & 0xFF);
        const bool hit = !found && code < run;
        j = hit ? t : j;
        found = found || hit;
    }
    return 16 * g + j;
}

// compress.c:90-112 for the root: halve, rebuild C, return the new total
DEV uint32_t root_rescale(uint8_t* r)
{
    uint32_t sum = 0;
    uint32_t cw[8];
#pragma unroll
    for (uint32_t g = 0; g < 16; ++g) {
        uint4 q = reinterpret_cast<uint4*>(r)[g];
        q.x -= (q.x >> 1) & 0x7F7F7F7Fu;
        q.y -= (q.y >> 1) & 0x7F7F7F7Fu;
        q.z -= (q.z >> 1) & 0x7F7F7F7Fu;
        q.w -= (q.w >> 1) & 0x7F7F7F7Fu;
        reinterpret_cast<uint4*>(r)[g] = q;
        sum = sad(q.w, sad(q.z, sad(q.y, sad(q.x, sum))));
        if (g & 1) cw[g >> 1] |= sum << 16; else cw[g >> 1] = sum;
    }
    reinterpret_cast<uint4*>(r + 256)[0] = make_uint4(cw[0], cw[1], cw[2], cw[3]);
    reinterpret_cast<uint4*>(r + 256)[1] = make_uint4(cw[4], cw[5], cw[6], cw[7]);
    return (sum + 1 + 256) & 0xFFFF;
}

// ---------------------------------------------------- order 1/2 records (HBM)

template <uint32_t INL>
struct Rec {
    uint32_t off, esc, tot, len, extlog, ext;
    uint32_t e[INL];
};

struct Hit { uint32_t k, under, cnt, link, val; bool found; };

template <uint32_t INL>
DEV void rec_load(const uint8_t* reg, uint32_t off, Rec<INL>& r)
{
    const uint4* p = reinterpret_cast<const uint4*>(reg + off);
    const uint4 h = p[0];
    r.off = off;
    r.esc = h.x & 0xFFFF; r.tot = h.x >> 16;
    r.len = h.y & 0xFFFF; r.extlog = h.y >> 16;
    r.ext = h.z;
#pragma unroll
    for (uint32_t c = 0; c < INL / 4; ++c) {
        const uint4 q = p[1 + c];
        r.e[4 * c] = q.x; r.e[4 * c + 1] = q.y; r.e[4 * c + 2] = q.z; r.e[4 * c + 3] = q.w;
    }
}

template <uint32_t INL>
DEV void rec_store(uint8_t* reg, const Rec<INL>& r)
{
    uint4* p = reinterpret_cast<uint4*>(reg + r.off);
    p[0] = make_uint4(r.esc | (r.tot << 16), r.len | (r.extlog << 16), r.ext, 0u);
    if (r.ext == 0) {
#pragma unroll
        for (uint32_t c = 0; c < INL / 4; ++c)
            p[1 + c] = make_uint4(r.e[4 * c], r.e[4 * c + 1], r.e[4 * c + 2], r.e[4 * c + 3]);
    }
}

// Encoder-side lookup of v: k = first entry >= v, under = counts below, found/cnt/link.
template <uint32_t INL>
DEV Hit rec_find(const uint8_t* reg, const Rec<INL>& r, uint32_t v)
{
    Hit h = { 0u, 0u, 0u, 0u, v, false };
    if (r.ext == 0) {
#pragma unroll
        for (uint32_t t = 0; t < INL; ++t) {
            const uint32_t e = r.e[t];
            const bool in = t < r.len;
            const bool lt = in && val_of(e) < v;
            const bool eq = in && val_of(e) == v;
            h.under += lt ? cnt_of(e) : 0u;
            h.k += lt ? 1u : 0u;
            h.found = h.found || eq;
            h.cnt = eq ? cnt_of(e) : h.cnt;
            h.link = eq ? (e >> 16) : h.link;
        }
    } else {
        const uint32_t* ep = reinterpret_cast<const uint32_t*>(reg + r.ext);
        for (uint32_t c = 0; c < r.len; c += 4) {
            const uint4 q = *reinterpret_cast<const uint4*>(ep + c);
            bool stop = false;
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t) {
                const uint32_t e = pick4(t, q);
                const bool in = c + t < r.len && !stop;
                const bool lt = in && val_of(e) < v;
                const bool eq = in && val_of(e) == v;
                h.under += lt ? cnt_of(e) : 0u;
                h.k += lt ? 1u : 0u;
                h.found = h.found || eq;
                h.cnt = eq ? cnt_of(e) : h.cnt;
                h.link = eq ? (e >> 16) : h.link;
                stop = stop || (in && !lt);
            }
            if (stop) break;
        }
    }
    return h;
}

// Decoder search (compress.c:373-416, minimum 0): entry whose interval holds code.
template <uint32_t INL>
DEV bool rec_search(const uint8_t* reg, const Rec<INL>& r, uint32_t code, Hit& h)
{
    uint32_t cum = 0;
    bool found = false;
    h.k = 0; h.under = 0; h.cnt = 0; h.link = 0; h.val = 0;
    if (r.ext == 0) {
#pragma unroll
        for (uint32_t t = 0; t < INL; ++t) {
            const uint32_t e = r.e[t];
            const bool in = t < r.len;
            const uint32_t c = in ? cnt_of(e) : 0u;
            const bool hit = in && !found && code < cum + c;
            h.k = hit ? t : h.k; h.under = hit ? cum : h.under; h.cnt = hit ? c : h.cnt;
            h.link = hit ? (e >> 16) : h.link; h.val = hit ? val_of(e) : h.val;
            found = found || hit;
            cum += c;
        }
    } else {
        const uint32_t* ep = reinterpret_cast<const uint32_t*>(reg + r.ext);
        for (uint32_t c0 = 0; c0 < r.len && !found; c0 += 4) {
            const uint4 q = *reinterpret_cast<const uint4*>(ep + c0);
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t) {
                const uint32_t e = pick4(t, q);
                const bool in = c0 + t < r.len;
                const uint32_t c = in ? cnt_of(e) : 0u;
                const bool hit = in && !found && code < cum + c;
                h.k = hit ? c0 + t : h.k; h.under = hit ? cum : h.under; h.cnt = hit ? c : h.cnt;
                h.link = hit ? (e >> 16) : h.link; h.val = hit ? val_of(e) : h.val;
                found = found || hit;
                cum += c;
            }
        }
    }
    h.found = found;
    return found;
}

// count[k] += d (old count `cnt`)
template <uint32_t INL>
DEV void rec_bump(uint8_t* reg, Rec<INL>& r, uint32_t k, uint32_t cnt, uint32_t d)
{
    if (r.ext == 0) {
#pragma unroll
        for (uint32_t t = 0; t < INL; ++t) r.e[t] += (t == k) ? (d << 8) : 0u;
    } else {
        reg[r.ext + 4 * k + 1] = static_cast<uint8_t>(cnt + d);
    }
}

// Insert entry `ne` at position k; grows into a (bigger) extension block when full.
template <uint32_t INL, uint32_t MINLOG>
DEV bool rec_insert(uint8_t* reg, Rec<INL>& r, uint32_t k, uint32_t ne, uint32_t& bump, uint32_t end)
{
    if (r.ext == 0 && r.len < INL) {
#pragma unroll
        for (int t = INL - 1; t >= 0; --t) {
            const uint32_t prev = t > 0 ? r.e[t > 0 ? t - 1 : 0] : 0u;
            r.e[t] = (static_cast<uint32_t>(t) > k) ? prev : (static_cast<uint32_t>(t) == k ? ne : r.e[t]);
        }
    } else {
        const uint32_t cap = r.ext ? (1u << r.extlog) : INL;
        if (r.len < cap) {
            uint32_t* ep = reinterpret_cast<uint32_t*>(reg + r.ext);
            for (uint32_t j = r.len; j > k; --j) ep[j] = ep[j - 1];
            ep[k] = ne;
        } else {
            const uint32_t nlog = r.ext ? r.extlog + 1 : MINLOG;
            const uint32_t bytes = 4u << nlog;
            if (bump + bytes > end) return false;
            uint32_t* np = reinterpret_cast<uint32_t*>(reg + bump);
            if (r.ext == 0) {
#pragma unroll
                for (uint32_t t = 0; t < INL; ++t) np[t + (t >= k ? 1u : 0u)] = r.e[t];
            } else {
                const uint32_t* ep = reinterpret_cast<const uint32_t*>(reg + r.ext);
                for (uint32_t j = 0; j < r.len; ++j) np[j + (j >= k ? 1u : 0u)] = ep[j];
            }
            np[k] = ne;
            r.ext = bump;
            r.extlog = nlog;
            bump += bytes;
        }
    }
    r.len += 1;
    return true;
}

// Set the link of entry k (an order-2 entry created before its suffix was known).
template <uint32_t INL>
DEV void rec_set_link(uint8_t* reg, Rec<INL>& r, uint32_t k, uint32_t link)
{
    if (r.ext == 0) {
#pragma unroll
        for (uint32_t t = 0; t < INL; ++t) r.e[t] = (t == k) ? ((r.e[t] & 0xFFFFu) | (link << 16)) : r.e[t];
    } else {
        *reinterpret_cast<uint16_t*>(reg + r.ext + 4 * k + 2) = static_cast<uint16_t>(link);
    }
}

// compress.c:90-112 on a record
template <uint32_t INL>
DEV void rec_rescale(uint8_t* reg, Rec<INL>& r)
{
    uint32_t sum = 0;
    if (r.ext == 0) {
#pragma unroll
        for (uint32_t t = 0; t < INL; ++t) {
            const uint32_t e = r.e[t];
            uint32_t c = cnt_of(e);
            c -= c >> 1;
            const bool in = t < r.len;
            sum += in ? c : 0u;
            r.e[t] = in ? ((e & 0xFFFF00FFu) | (c << 8)) : e;
        }
    } else {
        uint8_t* ep = reg + r.ext;
        for (uint32_t j = 0; j < r.len; ++j) {
            uint32_t c = ep[4 * j + 1];
            c -= c >> 1;
            ep[4 * j + 1] = static_cast<uint8_t>(c);
            sum += c;
        }
    }
    r.esc -= r.esc >> 1;
    r.tot = (sum + r.esc) & 0xFFFF;
}

// Encoder-side update of a sub-context (compress.c:293-314, patch :603-613):
// find or insert v; returns the hit (old count, cum below, link).  `newlink`
// is the link of an inserted entry.
DEV uint32_t new_o2(uint8_t* reg, uint32_t& bump, uint32_t end, bool& ovf);

// ALLOC: an inserted entry gets a fresh order-2 record as its link (order-1
// contexts); otherwise its link is filled in later (order-2 contexts).
template <uint32_t INL, uint32_t MINLOG, bool ALLOC>
DEV Hit sub_update(uint8_t* reg, Rec<INL>& r, uint32_t v, uint32_t& bump,
                   uint32_t end, uint32_t& nodes, bool& ovf)
{
    Hit h = rec_find(reg, r, v);
    if (h.found) {
        rec_bump(reg, r, h.k, h.cnt, kSubDelta);
    } else {
        uint32_t newlink = 0;
        if (ALLOC) { newlink = new_o2(reg, bump, end, ovf); if (ovf) return h; }
        if (!rec_insert<INL, MINLOG>(reg, r, h.k, v | (kSubDelta << 8) | (newlink << 16), bump, end)) {
            ovf = true;
            return h;
        }
        h.link = newlink;
        ++nodes;
        r.esc += kSubEscDelta;
        r.tot += kSubEscDelta;
    }
    r.tot = (r.tot + kSubDelta) & 0xFFFF;
    if (h.cnt > 0xFF - 2 * kSubDelta || r.tot > kTotalLimit) rec_rescale(reg, r);
    return h;
}

DEV void region_reset(uint8_t* reg, uint8_t* root)
{
    root_clear(root);
    const uint4 z = make_uint4(0u, 0u, 0u, 0u);
    for (uint32_t x = 0; x < 256; ++x) *reinterpret_cast<uint4*>(reg + x * kO1Rec) = z;
}

DEV uint32_t new_o2(uint8_t* reg, uint32_t& bump, uint32_t end, bool& ovf)
{
    if (bump + kO2Rec > end) { ovf = true; return 0; }
    const uint32_t off = bump;
    *reinterpret_cast<uint4*>(reg + off) = make_uint4(0u, 0u, 0u, 0u);
    bump += kO2Rec;
    return off / 32;
}

// ------------------------------------------------------------- range coder

// compress.c:121-137; false = output full
DEV bool enc_code(uint32_t& low, uint32_t& range, uint32_t under, uint32_t count, uint32_t total,
                  uint8_t* op, uint32_t& n, uint32_t cap)
{
    range /= total;
    low += under * range;
    range *= count;
    for (;;) {
        if ((low ^ (low + range)) >= kTop) {
            if (range >= kBot) return true;
            range = (0u - low) & (kBot - 1);
        }
        if (n >= cap) return false;
        op[n++] = static_cast<uint8_t>(low >> 24);
        range <<= 8;
        low <<= 8;
    }
}

struct DecIn { const uint8_t* p; uint32_t pos, len, nb; };

DEV uint32_t din_take(DecIn& d)
{
    const uint32_t b = d.nb;
    if (d.pos < d.len) ++d.pos;
    d.nb = d.pos < d.len ? d.p[d.pos] : 0u;
    return b;
}

// compress.c:354-371
DEV void dec_code(uint32_t& low, uint32_t& code, uint32_t& range, uint32_t under, uint32_t count, DecIn& in)
{
    low += under * range;
    range *= count;
    for (;;) {
        if ((low ^ (low + range)) >= kTop) {
            if (range >= kBot) break;
            range = (0u - low) & (kBot - 1);
        }
        code = (code << 8) | din_take(in);
        range <<= 8;
        low <<= 8;
    }
}

DEV void flag_exact(const rc_workspace_dev& ws, uint32_t pkt)
{
    const uint32_t slot = atomicAdd(&ws.counters[0], 1u);
    ws.flag_list[slot] = pkt;
}

// ------------------------------------------------------------ one packet

DEV void compress_one(const rc_batch_dev& b, const rc_workspace_dev& ws, uint32_t pkt,
                      uint8_t* reg, uint8_t* root)
{
    const uint32_t len = b.in_len[pkt];
    const uint32_t cap = b.out_cap[pkt];
    if (len == 0) { b.out_len[pkt] = 0; return; }                   // compress.c:257
    const uint8_t* ip = b.in + b.in_off[pkt];
    uint8_t* op = b.out + b.out_off[pkt];
    const uint32_t end = ws.lane_region;

    region_reset(reg, root);
    uint32_t rtot = 1 + 256, bump = kArenaBase, nodes = 1;
    uint32_t order = 0, b1 = 0, c2 = 0;
    uint32_t low = 0, range = ~0u, n = 0;
    bool ok = true, ovf = false;
    uint32_t nv = ip[0];

    for (uint32_t i = 0; i < len; ++i) {
        const uint32_t v = nv;
        if (i + 1 < len) nv = ip[i + 1];
        bool done = false, pend = false;
        uint32_t nxt = 0, kpend = 0;
        Rec<kO2Inl> r2;
        Rec<kO1Inl> r1;
        if (order >= 2) rec_load(reg, c2 * 32, r2);
        if (order >= 1) rec_load(reg, b1 * kO1Rec, r1);

        if (order >= 2) {                                            // order 2, compress.c:286-316
            const uint32_t esc0 = r2.esc, tot0 = r2.tot;
            const Hit h = sub_update<kO2Inl, kO2MinLog, false>(reg, r2, v, bump, end, nodes, ovf);
            if (ovf) break;
            if (h.found) {
                rec_store(reg, r2);
                ok = enc_code(low, range, esc0 + h.under, h.cnt, tot0, op, n, cap);
                nxt = h.link;
                done = true;
            } else {
                pend = true;
                kpend = h.k;
                if (esc0 > 0 && esc0 < tot0) ok = enc_code(low, range, 0, esc0, tot0, op, n, cap);
            }
            if (!ok) break;
        }
        if (!done && order >= 1) {                                   // order 1
            const uint32_t esc0 = r1.esc, tot0 = r1.tot;
            const Hit h = sub_update<kO1Inl, kO1MinLog, true>(reg, r1, v, bump, end, nodes, ovf);
            if (ovf) break;
            rec_store(reg, r1);
            nxt = h.link;
            if (pend) { rec_set_link(reg, r2, kpend, nxt); rec_store(reg, r2); }
            if (h.found) { ok = enc_code(low, range, esc0 + h.under, h.cnt, tot0, op, n, cap); done = true; }
            else if (esc0 > 0 && esc0 < tot0) ok = enc_code(low, range, 0, esc0, tot0, op, n, cap);
            if (!ok) break;
        }
        if (!done) {                                                 // root, compress.c:318-329
            uint32_t under, cnt;
            root_lookup(root, v, under, cnt);
            const uint32_t tot0 = rtot;
            if (cnt == 0) ++nodes;
            root_add(root, v, cnt);
            ok = enc_code(low, range, 1 + under, 1 + cnt, tot0, op, n, cap);
            if (!ok) break;
            rtot = (rtot + kRootDelta) & 0xFFFF;
            if (1 + cnt > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit) rtot = root_rescale(root);
        }
        if (order >= 1) c2 = nxt;                                    // compress.c:331-335
        if (order < 2) ++order;
        b1 = v;
        if (nodes >= kMaxNodes) {                                    // compress.c:148-157
            region_reset(reg, root);
            rtot = 1 + 256; bump = kArenaBase; nodes = 1; order = 0;
        }
    }
    if (ovf) { flag_exact(ws, pkt); return; }
    if (ok) {                                                        // compress.c:139-146
        while (low) {
            if (n >= cap) { ok = false; break; }
            op[n++] = static_cast<uint8_t>(low >> 24);
            low <<= 8;
        }
    }
    b.out_len[pkt] = ok ? n : 0u;
}

DEV void decompress_one(const rc_batch_dev& b, const rc_workspace_dev& ws, uint32_t pkt,
                        uint8_t* reg, uint8_t* root)
{
    const uint32_t len = b.in_len[pkt];
    const uint32_t cap = b.out_cap[pkt];
    if (len == 0) { b.out_len[pkt] = 0; return; }                   // compress.c:513
    uint8_t* op = b.out + b.out_off[pkt];
    const uint32_t end = ws.lane_region;
    DecIn in = { b.in + b.in_off[pkt], 0u, len, 0u };
    in.nb = in.p[0];

    region_reset(reg, root);
    uint32_t rtot = 1 + 256, bump = kArenaBase, nodes = 1;
    uint32_t order = 0, b1 = 0, c2 = 0;
    uint32_t low = 0, code = 0, range = ~0u, n = 0;
    for (int k = 0; k < 4; ++k) code = (code << 8) | din_take(in);   // compress.c:344-350
    bool fail = false, anomaly = false, ovf = false;

    for (;;) {
        int at = -1;                         // context that produced the symbol (2, 1, 0)
        uint32_t v = 0, nxt = 0;
        Rec<kO2Inl> r2;
        Rec<kO1Inl> r1;
        if (order >= 2) rec_load(reg, c2 * 32, r2);
        if (order >= 1) rec_load(reg, b1 * kO1Rec, r1);

        if (order >= 2 && r2.esc > 0 && r2.esc < r2.tot) {          // compress.c:529-568
            range /= r2.tot;
            uint32_t cd = ((code - low) / range) & 0xFFFF;
            if (cd < r2.esc) {
                dec_code(low, code, range, 0, r2.esc, in);
            } else {
                cd -= r2.esc;
                Hit h;
                if (!rec_search(reg, r2, cd, h)) { fail = true; break; }
                v = h.val;
                rec_bump(reg, r2, h.k, h.cnt, kSubDelta);
                dec_code(low, code, range, r2.esc + h.under, h.cnt, in);
                r2.tot = (r2.tot + kSubDelta) & 0xFFFF;
                if (h.cnt > 0xFF - 2 * kSubDelta || r2.tot > kTotalLimit) rec_rescale(reg, r2);
                rec_store(reg, r2);
                nxt = h.link;
                at = 2;
            }
        }
        if (at < 0 && order >= 1 && r1.esc > 0 && r1.esc < r1.tot) {
            range /= r1.tot;
            uint32_t cd = ((code - low) / range) & 0xFFFF;
            if (cd < r1.esc) {
                dec_code(low, code, range, 0, r1.esc, in);
            } else {
                cd -= r1.esc;
                Hit h;
                if (!rec_search(reg, r1, cd, h)) { fail = true; break; }
                v = h.val;
                rec_bump(reg, r1, h.k, h.cnt, kSubDelta);
                dec_code(low, code, range, r1.esc + h.under, h.cnt, in);
                r1.tot = (r1.tot + kSubDelta) & 0xFFFF;
                if (h.cnt > 0xFF - 2 * kSubDelta || r1.tot > kTotalLimit) rec_rescale(reg, r1);
                rec_store(reg, r1);
                nxt = h.link;
                at = 1;
            }
        }
        if (at < 0) {                                                // root, compress.c:570-596
            range /= rtot;
            uint32_t cd = ((code - low) / range) & 0xFFFF;
            if (cd < 1) { dec_code(low, code, range, 0, 1, in); break; }   // end of stream
            cd -= 1;
            if (cd >= rtot - 1) { anomaly = true; break; }          // past symbol 255
            v = root_search(root, cd);
            uint32_t under, cnt;
            root_lookup(root, v, under, cnt);
            if (cnt == 0) ++nodes;
            root_add(root, v, cnt);
            dec_code(low, code, range, 1 + under, 1 + cnt, in);
            rtot = (rtot + kRootDelta) & 0xFFFF;
            if (1 + cnt > 0xFF - 2 * kRootDelta + 1 || rtot > kTotalLimit) rtot = root_rescale(root);
            at = 0;
        }
        // patch the contexts above, compress.c:598-615
        bool pend = false;
        uint32_t kpend = 0;
        if (order >= 2 && at < 2) {
            const Hit h = sub_update<kO2Inl, kO2MinLog, false>(reg, r2, v, bump, end, nodes, ovf);
            if (ovf) break;
            if (h.found) rec_store(reg, r2);
            else { pend = true; kpend = h.k; }
        }
        if (order >= 1 && at < 1) {
            const Hit h = sub_update<kO1Inl, kO1MinLog, true>(reg, r1, v, bump, end, nodes, ovf);
            if (ovf) break;
            rec_store(reg, r1);
            nxt = h.link;
        }
        if (pend) { rec_set_link(reg, r2, kpend, nxt); rec_store(reg, r2); }
        if (n >= cap) { fail = true; break; }                        // compress.c:617
        op[n++] = static_cast<uint8_t>(v);
        if (order >= 1) c2 = nxt;
        if (order < 2) ++order;
        b1 = v;
        if (nodes >= kMaxNodes) {
            region_reset(reg, root);
            rtot = 1 + 256; bump = kArenaBase; nodes = 1; order = 0;
        }
    }
    if (ovf || anomaly) { flag_exact(ws, pkt); return; }
    b.out_len[pkt] = fail ? 0u : n;
}

}  // namespace

extern "C" uint32_t rc_hip_lane_region_bytes(uint32_t max_len)
{
    // order-1 table + order-2 records (<= one per byte) + extension blocks
    // (<= 16 B per model node); at most 4094 nodes between resets.
    const uint64_t L = max_len < 4096 ? max_len : 4096;
    const uint64_t nodes = 2 * L + 256 < 4094 ? 2 * L + 256 : 4094;
    uint64_t bytes = kArenaBase + 32 * L + 16 * nodes + 4096;
    bytes = (bytes + 255) & ~255ull;
    return static_cast<uint32_t>(bytes);
}

#ifndef RC_LANE_HOST_TEST
extern "C" __global__ __launch_bounds__(256)
void rc_compress_lane(rc_batch_dev b, rc_workspace_dev ws)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* root = smem + threadIdx.x * kRootStride;
    const uint32_t slot = blockIdx.x * kBlock + threadIdx.x;
    uint8_t* reg = static_cast<uint8_t*>(ws.lane_pool) + static_cast<size_t>(slot) * ws.lane_region;
    for (uint32_t pkt = slot; pkt < b.n; pkt += gridDim.x * kBlock)
        compress_one(b, ws, pkt, reg, root);
}

extern "C" __global__ __launch_bounds__(256)
void rc_decompress_lane(rc_batch_dev b, rc_workspace_dev ws)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* root = smem + threadIdx.x * kRootStride;
    const uint32_t slot = blockIdx.x * kBlock + threadIdx.x;
    uint8_t* reg = static_cast<uint8_t*>(ws.lane_pool) + static_cast<size_t>(slot) * ws.lane_region;
    for (uint32_t pkt = slot; pkt < b.n; pkt += gridDim.x * kBlock)
        decompress_one(b, ws, pkt, reg, root);
}

extern "C" int rc_hip_lane_launch(int decompress, const rc_batch_dev* b, const rc_workspace_dev* ws,
                                  void* stream)
{
    hipStream_t st = static_cast<hipStream_t>(stream);
    uint32_t blocks = (b->n + kBlock - 1) / kBlock;
    const uint32_t maxb = ws->lane_slots / kBlock;
    if (blocks > maxb) blocks = maxb;
    if (blocks == 0) return static_cast<int>(hipErrorInvalidValue);
    const size_t lds = static_cast<size_t>(kBlock) * kRootStride;
    if (decompress)
        hipLaunchKernelGGL(rc_decompress_lane, dim3(blocks), dim3(kBlock), lds, st, *b, *ws);
    else
        hipLaunchKernelGGL(rc_compress_lane, dim3(blocks), dim3(kBlock), lds, st, *b, *ws);
    return static_cast<int>(hipGetLastError());
}
#endif  // RC_LANE_HOST_TEST
