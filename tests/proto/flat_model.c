/*
 * flat_model.c -- DESIGN PROTOTYPE, TEST INFRASTRUCTURE ONLY.
 *
 * Sequential C model of the data structure the HIP kernels use
 * (enet_amd/csrc/rc_kernels.hip), written to validate its semantics against
 * the golden fixtures on the CPU and to measure its LDS footprint.  It is not
 * part of the product and nothing in enet_amd/ links it.
 *
 * Model (SURVEY.md §8a "semantic restatement"): per context only
 * {count[v], escapes, total} are observable, so instead of compress.c's
 * per-context binary trees:
 *   root  : flat cum[256] / cnt[256]                (wave registers on the GPU)
 *   o1    : 256 headers {esc, off, len} (total = esc + cum[len-1])
 *           + sorted blocks of {value, count, cum16} + o2 id
 *   o2    : header pool {esc, off, len} + sorted blocks of {value, count, cum16}
 * Blocks have power-of-two capacity and are re-allocated on growth.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ARENA_BYTES 65536

typedef struct {
    /* root */
    uint16_t rcum[256];   /* cum of counts <= v */
    uint8_t  rcnt[256];
    uint16_t rtot;
    /* o1 headers */
    uint16_t o1esc[256], o1off[256], o1len[256];
    /* arena: blocks grow up from 0, o2 headers grow down from the top */
    uint8_t  arena[ARENA_BYTES];
    uint32_t lo, hi;
    uint32_t nodes;
    uint32_t hiwater;
    int overflow;
    uint16_t freehead[2][10];
} model_t;

/* entry word: value | count<<8 | cum<<16 */
#define E_VAL(e) ((e) & 0xFF)
#define E_CNT(e) (((e) >> 8) & 0xFF)
#define E_CUM(e) ((e) >> 16)

static unsigned cap_of(unsigned len, unsigned mincap)
{ unsigned c = mincap; while (c < len) c <<= 1; return c; }

static unsigned lg2(unsigned c) { unsigned l = 0; while ((1u << l) < c) ++l; return l; }

/* kind 0 = o2 block (4 B/entry), kind 1 = o1 block (6 B/entry) */
static unsigned blk_bytes(int kind, unsigned cap) { return cap * (kind ? 6u : 4u); }

static uint32_t blk_alloc(model_t *m, int kind, unsigned cap)
{
    unsigned l = lg2(cap);
    uint16_t h = m->freehead[kind][l];
    if (h != 0xFFFF) {
        uint16_t next; memcpy(&next, &m->arena[h], 2);
        m->freehead[kind][l] = next;
        return h;
    }
    unsigned b = blk_bytes(kind, cap);
    uint32_t off = (m->lo + 3u) & ~3u;
    if (off + b > m->hi) { m->overflow = 1; return 0; }
    m->lo = off + b;
    if (m->lo + (ARENA_BYTES - m->hi) > m->hiwater) m->hiwater = m->lo + (ARENA_BYTES - m->hi);
    return off;
}

static void blk_free(model_t *m, int kind, uint32_t off, unsigned cap)
{
    unsigned l = lg2(cap);
    uint16_t next = m->freehead[kind][l];
    memcpy(&m->arena[off], &next, 2);
    m->freehead[kind][l] = (uint16_t) off;
}

static uint32_t o2_new(model_t *m)
{
    if (m->hi < m->lo + 8) { m->overflow = 1; return 0; }
    m->hi -= 8;
    memset(&m->arena[m->hi], 0, 8);
    if (m->lo + (ARENA_BYTES - m->hi) > m->hiwater) m->hiwater = m->lo + (ARENA_BYTES - m->hi);
    return m->hi;
}

static void model_reset(model_t *m)
{
    memset(m->rcum, 0, sizeof m->rcum); memset(m->rcnt, 0, sizeof m->rcnt);
    m->rtot = 257;
    memset(m->o1esc, 0, sizeof m->o1esc); memset(m->o1off, 0, sizeof m->o1off);
    memset(m->o1len, 0, sizeof m->o1len);
    m->lo = 0; m->hi = ARENA_BYTES; m->nodes = 1;
    memset(m->freehead, 0xFF, sizeof m->freehead);
}

/* ---------------------------------------------------------------- contexts */

typedef struct { uint16_t *esc, *len; uint16_t *off; int kind; } ctx_ref;

static uint32_t *ent(model_t *m, uint32_t off, unsigned i) { return (uint32_t *) &m->arena[off + 4 * i]; }
static uint16_t *o2id_of(model_t *m, uint32_t off, unsigned cap, unsigned i)
{ return (uint16_t *) &m->arena[off + 4 * cap + 2 * i]; }

static unsigned ctx_total(model_t *m, ctx_ref c)
{ return *c.len ? (unsigned) (*c.esc + E_CUM(*ent(m, *c.off, *c.len - 1))) : *c.esc; }

/* halve every count, rebuild cum, halve escapes (compress.c:90-112) */
static void ctx_rescale(model_t *m, ctx_ref c)
{
    unsigned cum = 0;
    for (unsigned i = 0; i < *c.len; ++i) {
        uint32_t e = *ent(m, *c.off, i);
        unsigned cnt = E_CNT(e); cnt -= cnt >> 1; cum += cnt;
        *ent(m, *c.off, i) = E_VAL(e) | (cnt << 8) | ((cum & 0xFFFF) << 16);
    }
    *c.esc = (uint16_t) (*c.esc - (*c.esc >> 1));
}

/* position of first entry with value >= v */
static unsigned ctx_lower(model_t *m, ctx_ref c, uint8_t v)
{
    unsigned k = 0;
    while (k < *c.len && E_VAL(*ent(m, *c.off, k)) < v) ++k;
    return k;
}

/* increment entry k by d (count and every cum from k on) */
static void ctx_bump(model_t *m, ctx_ref c, unsigned k, unsigned d)
{
    for (unsigned i = k; i < *c.len; ++i) {
        uint32_t e = *ent(m, *c.off, i);
        if (i == k) e += d << 8;
        e += d << 16;
        *ent(m, *c.off, i) = e;
    }
}

/* insert v at k with count d; returns new position k (o1: fills o2id) */
static void ctx_insert(model_t *m, ctx_ref c, unsigned k, uint8_t v, unsigned d, uint16_t o2id)
{
    unsigned mincap = c.kind ? 2 : 1;
    unsigned len = *c.len, cap = len ? cap_of(len, mincap) : 0;
    if (len + 1 > cap) {
        unsigned ncap = cap_of(len + 1, mincap);
        uint32_t noff = blk_alloc(m, c.kind, ncap);
        if (m->overflow) return;
        for (unsigned i = 0; i < len; ++i) {
            *ent(m, noff, i) = *ent(m, *c.off, i);
            if (c.kind) *o2id_of(m, noff, ncap, i) = *o2id_of(m, *c.off, cap, i);
        }
        if (len) blk_free(m, c.kind, *c.off, cap);
        *c.off = (uint16_t) noff;
        cap = ncap;
    }
    for (unsigned i = len; i > k; --i) {
        *ent(m, *c.off, i) = *ent(m, *c.off, i - 1);
        if (c.kind) *o2id_of(m, *c.off, cap, i) = *o2id_of(m, *c.off, cap, i - 1);
    }
    unsigned below = k ? E_CUM(*ent(m, *c.off, k - 1)) : 0;
    *ent(m, *c.off, k) = v | (d << 8) | (((below + d) & 0xFFFF) << 16);
    if (c.kind) *o2id_of(m, *c.off, cap, k) = o2id;
    *c.len = (uint16_t) (len + 1);
    for (unsigned i = k + 1; i <= len; ++i) *ent(m, *c.off, i) += d << 16;
    m->nodes++;
}

/* encoder-side visit of a sub-context (compress.c:293-316 / patch :603-613).
 * Returns old count (0 if new); *under_ = cum below v; *total_ = total
 * before the update; *k_ = final position of v. */
static unsigned sub_encode(model_t *m, ctx_ref c, uint8_t v, unsigned *under_, unsigned *total_,
                           unsigned *k_, uint16_t *o2id_out)
{
    unsigned k = ctx_lower(m, c, v);
    unsigned total = ctx_total(m, c);
    unsigned under = k ? E_CUM(*ent(m, *c.off, k - 1)) : 0;
    unsigned count = 0;
    *total_ = total; *under_ = under;
    if (k < *c.len && E_VAL(*ent(m, *c.off, k)) == v) {
        count = E_CNT(*ent(m, *c.off, k));
        ctx_bump(m, c, k, 2);
    } else {
        uint16_t id = 0;
        if (c.kind) id = (uint16_t) o2_new(m);
        if (m->overflow) return 0;
        ctx_insert(m, c, k, v, 2, id);
        if (m->overflow) return 0;
        *c.esc = (uint16_t) (*c.esc + 5);
    }
    if (c.kind && o2id_out) {
        unsigned cap = cap_of(*c.len, 2);
        *o2id_out = *o2id_of(m, *c.off, cap, k);
    }
    *k_ = k;
    unsigned ntot = *c.esc + E_CUM(*ent(m, *c.off, *c.len - 1));
    if (count > 251 || ntot > 65280) ctx_rescale(m, c);
    return count;
}

static ctx_ref o1_ref(model_t *m, uint8_t x)
{ ctx_ref c = { &m->o1esc[x], &m->o1len[x], &m->o1off[x], 1 }; return c; }

static ctx_ref o2_ref(model_t *m, uint16_t id)
{
    ctx_ref c = { (uint16_t *) &m->arena[id], (uint16_t *) &m->arena[id + 4],
                  (uint16_t *) &m->arena[id + 2], 0 };
    return c;
}

/* root (minimum 1, delta 3) */
static void root_encode(model_t *m, uint8_t v, unsigned *under, unsigned *count)
{
    unsigned below = v ? m->rcum[v - 1] : 0;
    *under = v + below;
    *count = 1u + m->rcnt[v];
    if (!m->rcnt[v]) m->nodes++;
    m->rcnt[v] = (uint8_t) (m->rcnt[v] + 3);
    for (unsigned u = v; u < 256; ++u) m->rcum[u] = (uint16_t) (m->rcum[u] + 3);
}

static void root_rescale(model_t *m)
{
    unsigned cum = 0;
    for (unsigned u = 0; u < 256; ++u) {
        m->rcnt[u] = (uint8_t) (m->rcnt[u] - (m->rcnt[u] >> 1));
        cum += m->rcnt[u]; m->rcum[u] = (uint16_t) cum;
    }
    m->rtot = (uint16_t) (cum + 1 + 256);
}

/* ------------------------------------------------------------ range coder */

typedef struct { uint32_t low, range; uint8_t *out; size_t n, cap; int fail; } enc_t;

static void enc(enc_t *e, uint32_t under, uint32_t count, uint32_t total)
{
    e->range /= total; e->low += under * e->range; e->range *= count;
    for (;;) {
        if ((e->low ^ (e->low + e->range)) >= (1u << 24)) {
            if (e->range >= (1u << 16)) return;
            e->range = (0u - e->low) & 0xFFFF;
        }
        if (e->n >= e->cap) { e->fail = 1; return; }
        e->out[e->n++] = (uint8_t) (e->low >> 24);
        e->range <<= 8; e->low <<= 8;
    }
}

static model_t M;

size_t flat_compress(const uint8_t *in, size_t n, uint8_t *out, size_t cap, unsigned *hiwater, int *ovf)
{
    model_t *m = &M;
    enc_t e = { 0, ~0u, out, 0, cap, 0 };
    unsigned order = 0; uint8_t b1 = 0; uint16_t c2 = 0;
    if (n == 0) return 0;
    model_reset(m); m->hiwater = 0; m->overflow = 0;
    for (size_t i = 0; i < n; ++i) {
        uint8_t v = in[i];
        unsigned under, total, k, count;
        uint16_t next_c2 = 0;
        int have_next = 0;
        if (order >= 2) {
            ctx_ref c = o2_ref(m, c2);
            unsigned esc0 = *c.esc;
            count = sub_encode(m, c, v, &under, &total, &k, NULL);
            if (m->overflow) break;
            if (count) { enc(&e, esc0 + under, count, total); goto advance; }
            if (esc0 > 0 && esc0 < total) enc(&e, 0, esc0, total);
        }
        if (order >= 1) {
            ctx_ref c = o1_ref(m, b1);
            unsigned esc0 = *c.esc;
            count = sub_encode(m, c, v, &under, &total, &k, &next_c2);
            if (m->overflow) break;
            have_next = 1;
            if (count) { enc(&e, esc0 + under, count, total); goto advance; }
            if (esc0 > 0 && esc0 < total) enc(&e, 0, esc0, total);
        }
        {
            unsigned tot = m->rtot;
            root_encode(m, v, &under, &count);
            enc(&e, 1 + under, count, tot);
            m->rtot = (uint16_t) (m->rtot + 3);
            if (count > 250 || m->rtot > 65280) root_rescale(m);
        }
    advance:
        if (e.fail) return 0;
        if (order >= 1) {
            if (!have_next) {
                ctx_ref c = o1_ref(m, b1);
                unsigned kk = ctx_lower(m, c, v);
                next_c2 = *o2id_of(m, *c.off, cap_of(*c.len, 2), kk);
            }
            c2 = next_c2;
        }
        if (order < 2) ++order;
        b1 = v;
        if (m->nodes >= 4094) { model_reset(m); order = 0; }
    }
    *hiwater = m->hiwater; *ovf = m->overflow;
    if (m->overflow) return (size_t) -1;
    if (e.fail) return 0;
    while (e.low) {
        if (e.n >= e.cap) return 0;
        e.out[e.n++] = (uint8_t) (e.low >> 24); e.low <<= 8;
    }
    return e.n;
}

/* ------------------------------------------------------------- decoder */

typedef struct { uint32_t low, code, range; const uint8_t *ip, *ie; } dec_t;

static uint16_t dread(dec_t *d, unsigned total)
{ d->range /= total; return (uint16_t) ((d->code - d->low) / d->range); }

static void ddec(dec_t *d, uint32_t under, uint32_t count)
{
    d->low += under * d->range; d->range *= count;
    for (;;) {
        if ((d->low ^ (d->low + d->range)) >= (1u << 24)) {
            if (d->range >= (1u << 16)) break;
            d->range = (0u - d->low) & 0xFFFF;
        }
        d->code <<= 8; if (d->ip < d->ie) d->code |= *d->ip++;
        d->range <<= 8; d->low <<= 8;
    }
}

/* returns -2 on anomaly (needs the exact path), -1 overflow, else length */
long flat_decompress(const uint8_t *in, size_t n, uint8_t *out, size_t cap, unsigned *hiwater)
{
    model_t *m = &M;
    dec_t d = { 0, 0, ~0u, in, in + n };
    unsigned order = 0; uint8_t b1 = 0; uint16_t c2 = 0; size_t on = 0;
    if (n == 0) return 0;
    model_reset(m); m->hiwater = 0; m->overflow = 0;
    for (int s = 0; s < 4; ++s) { d.code <<= 8; if (d.ip < d.ie) d.code |= *d.ip++; }
    for (;;) {
        int at = -1;    /* context level that produced the symbol: 2, 1, 0 */
        uint8_t v = 0;
        unsigned under, count, total, k;
        int skipped2 = 0, skipped1 = 0;
        if (order >= 2) {
            ctx_ref c = o2_ref(m, c2);
            unsigned esc = *c.esc; total = ctx_total(m, c);
            if (esc == 0 || esc >= total) skipped2 = 1;
            else {
                uint16_t code = dread(&d, total);
                if (code < esc) { ddec(&d, 0, esc); skipped2 = 1; }
                else {
                    code = (uint16_t) (code - esc);
                    unsigned j = 0;
                    while (j < *c.len && code >= E_CUM(*ent(m, *c.off, j))) ++j;
                    if (j == *c.len) return 0;
                    uint32_t e = *ent(m, *c.off, j);
                    v = (uint8_t) E_VAL(e); count = E_CNT(e); under = E_CUM(e) - count;
                    ctx_bump(m, c, j, 2);
                    ddec(&d, esc + under, count);
                    if (count > 251 || ctx_total(m, c) > 65280) ctx_rescale(m, c);
                    at = 2;
                }
            }
        }
        if (at < 0 && order >= 1) {
            ctx_ref c = o1_ref(m, b1);
            unsigned esc = *c.esc; total = ctx_total(m, c);
            if (esc == 0 || esc >= total) skipped1 = 1;
            else {
                uint16_t code = dread(&d, total);
                if (code < esc) { ddec(&d, 0, esc); skipped1 = 1; }
                else {
                    code = (uint16_t) (code - esc);
                    unsigned j = 0;
                    while (j < *c.len && code >= E_CUM(*ent(m, *c.off, j))) ++j;
                    if (j == *c.len) return 0;
                    uint32_t e = *ent(m, *c.off, j);
                    v = (uint8_t) E_VAL(e); count = E_CNT(e); under = E_CUM(e) - count;
                    ctx_bump(m, c, j, 2);
                    ddec(&d, esc + under, count);
                    if (count > 251 || ctx_total(m, c) > 65280) ctx_rescale(m, c);
                    at = 1;
                }
            }
        }
        (void) skipped1; (void) skipped2;
        if (at < 0) {
            unsigned tot = m->rtot;
            uint16_t code = dread(&d, tot);
            if (code < 1) { ddec(&d, 0, 1); break; }
            code = (uint16_t) (code - 1);
            if (code >= tot - 1) return -2;   /* implicit symbol beyond 255: BST-shape dependent */
            unsigned u = 0;
            while (code >= u + 1 + m->rcum[u]) ++u;
            v = (uint8_t) u;
            root_encode(m, v, &under, &count);
            ddec(&d, 1 + under, count);
            m->rtot = (uint16_t) (m->rtot + 3);
            if (count > 250 || m->rtot > 65280) root_rescale(m);
            at = 0;
        }
        /* patch higher contexts (compress.c:598-615) */
        uint16_t next_c2 = 0; int have_next = 0;
        if (order >= 2 && at < 2) {
            ctx_ref c = o2_ref(m, c2);
            sub_encode(m, c, v, &under, &total, &k, NULL);
            if (m->overflow) return -1;
        }
        if (order >= 1 && at < 1) {
            ctx_ref c = o1_ref(m, b1);
            sub_encode(m, c, v, &under, &total, &k, &next_c2);
            if (m->overflow) return -1;
            have_next = 1;
        }
        if (on >= cap) return 0;
        out[on++] = v;
        if (order >= 1) {
            if (!have_next) {
                ctx_ref c = o1_ref(m, b1);
                unsigned kk = ctx_lower(m, c, v);
                next_c2 = *o2id_of(m, *c.off, cap_of(*c.len, 2), kk);
            }
            c2 = next_c2;
        }
        if (order < 2) ++order;
        b1 = v;
        if (m->nodes >= 4094) { model_reset(m); order = 0; }
    }
    *hiwater = m->hiwater;
    return (long) on;
}
