/*
 * rc_oracle.c -- TEST INFRASTRUCTURE ONLY (see rc_oracle.h).
 *
 * A from-scratch CPU restatement of the order-2 PPM range coder of
 * lsalzman/enet compress.c.  Data structure and integer semantics follow the
 * reference exactly (including its behaviour on corrupt input), because the
 * decoder's reaction to garbage depends on the binary-tree shape.  Every
 * function names the reference lines it restates.
 *
 * Differences in *representation* only (no observable effect):
 *   - child links are absolute pool indices instead of relative offsets
 *     (a child is always created after its parent, so index 0 = "none");
 *   - the macros are functions.
 */
#include "rc_oracle.h"

#include <stdlib.h>
#include <string.h>

/* compress.c:25-37 (adaptation constants); context exclusion is compiled out
 * at compress.c:39-40 and is therefore not restated. */
#define POOL_NODES     4096u
#define RC_TOP         (1u << 24)
#define RC_BOTTOM      (1u << 16)
#define ROOT_DELTA     3
#define ROOT_MIN       1
#define ROOT_ESC_MIN   1
#define SUB_ORDER      2
#define SUB_DELTA      2
#define SUB_ESC_DELTA  5

/* compress.c:9-22: one pool node; both a symbol of its parent context's
 * binary tree and (for orders 1-2) a context of its own. */
typedef struct {
    uint8_t  value;
    uint8_t  count;
    uint16_t under;    /* own count + left-subtree counts */
    uint16_t left, right;
    uint16_t child;    /* root of this context's tree ("symbols") */
    uint16_t escapes;
    uint16_t total;
    uint16_t parent;   /* suffix link: next lower-order context */
} or_node;

struct or_coder { or_node n[POOL_NODES]; };

/* ------------------------------------------------------------------ pool */

typedef struct { or_node *n; size_t next; } pool_t;

/* compress.c:68-80 */
static uint16_t node_new(pool_t *p, uint8_t value, uint8_t count)
{
    uint16_t id = (uint16_t) p->next++;
    or_node *s = &p->n[id];
    s->value = value; s->count = count; s->under = count;
    s->left = s->right = s->child = 0;
    s->escapes = s->total = 0; s->parent = 0;
    return id;
}

/* compress.c:82-88 */
static uint16_t context_new(pool_t *p, uint16_t escapes, uint16_t minimum)
{
    uint16_t id = node_new(p, 0, 0);
    p->n[id].escapes = escapes;
    p->n[id].total = (uint16_t) (escapes + 256 * minimum);
    p->n[id].child = 0;
    return id;
}

/* compress.c:90-105: halve every count of a tree, rebuild `under`,
 * return the sum of counts along the right spine (= whole tree). */
static uint16_t tree_halve(or_node *n, uint16_t id)
{
    uint16_t sum = 0;
    for (;;) {
        or_node *s = &n[id];
        s->count = (uint8_t) (s->count - (s->count >> 1));
        s->under = s->count;
        if (s->left) s->under = (uint16_t) (s->under + tree_halve(n, s->left));
        sum = (uint16_t) (sum + s->under);
        if (!s->right) break;
        id = s->right;
    }
    return sum;
}

/* compress.c:107-112 */
static void context_rescale(or_node *n, uint16_t ctx, uint16_t minimum)
{
    or_node *c = &n[ctx];
    c->total = c->child ? tree_halve(n, c->child) : 0;
    c->escapes = (uint16_t) (c->escapes - (c->escapes >> 1));
    c->total = (uint16_t) (c->total + c->escapes + 256 * minimum);
}

/* compress.c:159-199: find or insert `value` in context `ctx`.  Returns the
 * node id; *under_ = cumulative count below value (with `minimum` per
 * smaller symbol value), *count_ = minimum + old count (minimum if new). */
static uint16_t context_encode(pool_t *p, uint16_t ctx, uint8_t value,
                               uint16_t *under_, uint16_t *count_,
                               int update, int minimum)
{
    or_node *n = p->n;
    uint16_t under = (uint16_t) (value * minimum), count = (uint16_t) minimum;
    uint16_t id;
    if (!n[ctx].child) {
        id = node_new(p, value, (uint8_t) update);
        n[ctx].child = id;
    } else {
        uint16_t cur = n[ctx].child;
        for (;;) {
            or_node *s = &n[cur];
            if (value < s->value) {
                s->under = (uint16_t) (s->under + update);
                if (s->left) { cur = s->left; continue; }
                id = node_new(p, value, (uint8_t) update);
                n[cur].left = id;
            } else if (value > s->value) {
                under = (uint16_t) (under + s->under);
                if (s->right) { cur = s->right; continue; }
                id = node_new(p, value, (uint8_t) update);
                n[cur].right = id;
            } else {
                count = (uint16_t) (count + s->count);
                under = (uint16_t) (under + s->under - s->count);
                s->under = (uint16_t) (s->under + update);
                s->count = (uint8_t) (s->count + update);
                id = cur;
            }
            break;
        }
    }
    *under_ = under; *count_ = count;
    return id;
}

/* --------------------------------------------------------------- encoder */

typedef struct { uint32_t low, range; uint8_t *out, *end; } enc_t;

/* compress.c:114-137.  Returns 0 when the output is full (the whole
 * compress call then returns 0, compress.c:116-117). */
static int enc_code(enc_t *e, uint32_t under, uint32_t count, uint32_t total)
{
    e->range /= total;
    e->low += under * e->range;
    e->range *= count;
    for (;;) {
        if ((e->low ^ (e->low + e->range)) >= RC_TOP) {
            if (e->range >= RC_BOTTOM) return 1;
            e->range = (0u - e->low) & (RC_BOTTOM - 1);
        }
        if (e->out >= e->end) return 0;
        *e->out++ = (uint8_t) (e->low >> 24);
        e->range <<= 8;
        e->low <<= 8;
    }
}

/* compress.c:139-146 */
static int enc_flush(enc_t *e)
{
    while (e->low) {
        if (e->out >= e->end) return 0;
        *e->out++ = (uint8_t) (e->low >> 24);
        e->low <<= 8;
    }
    return 1;
}

or_coder *or_create(void) { return (or_coder *) malloc(sizeof(or_coder)); }
void or_destroy(or_coder *c) { free(c); }

/* compress.c:246-342 */
size_t or_compress(or_coder *coder, const OrBuffer *bufs, size_t nbufs,
                   size_t in_limit, uint8_t *out, size_t out_limit)
{
    pool_t pool;
    enc_t e;
    const uint8_t *ip, *ie;
    uint16_t predicted = 0;
    size_t order = 0;

    if (coder == NULL || nbufs == 0 || in_limit == 0) return 0;   /* :257-258 */

    pool.n = coder->n; pool.next = 0;
    e.low = 0; e.range = ~0u; e.out = out; e.end = out + out_limit;
    ip = (const uint8_t *) bufs->data; ie = ip + bufs->dataLength;
    ++bufs; --nbufs;
    context_new(&pool, ROOT_ESC_MIN, ROOT_MIN);                    /* root = node 0 */

    for (;;) {
        or_node *n = pool.n;
        uint16_t *link = &predicted, under, count, total, ctx, sym;
        uint8_t value;

        /* gather-list walk, compress.c:275-284 (an empty non-first buffer
         * still yields one byte: its data[0]). */
        if (ip >= ie) {
            if (nbufs == 0) break;
            ip = (const uint8_t *) bufs->data; ie = ip + bufs->dataLength;
            ++bufs; --nbufs;
        }
        value = *ip++;

        /* order-2 / order-1 contexts, compress.c:286-316 */
        for (ctx = predicted; ctx != 0; ctx = n[ctx].parent) {
            sym = context_encode(&pool, ctx, value, &under, &count, SUB_DELTA, 0);
            *link = sym;
            link = &n[sym].parent;
            total = n[ctx].total;
            if (count > 0) {
                if (!enc_code(&e, (uint32_t) n[ctx].escapes + under, count, total)) return 0;
            } else {
                if (n[ctx].escapes > 0 && n[ctx].escapes < total)
                    if (!enc_code(&e, 0, n[ctx].escapes, total)) return 0;
                n[ctx].escapes = (uint16_t) (n[ctx].escapes + SUB_ESC_DELTA);
                n[ctx].total = (uint16_t) (n[ctx].total + SUB_ESC_DELTA);
            }
            n[ctx].total = (uint16_t) (n[ctx].total + SUB_DELTA);
            if (count > 0xFF - 2 * SUB_DELTA || n[ctx].total > RC_BOTTOM - 0x100)
                context_rescale(n, ctx, 0);
            if (count > 0) goto advance;
        }

        /* order-0 root, compress.c:318-329 */
        sym = context_encode(&pool, 0, value, &under, &count, ROOT_DELTA, ROOT_MIN);
        *link = sym;
        total = n[0].total;
        if (!enc_code(&e, (uint32_t) n[0].escapes + under, count, total)) return 0;
        n[0].total = (uint16_t) (n[0].total + ROOT_DELTA);
        if (count > 0xFF - 2 * ROOT_DELTA + ROOT_MIN || n[0].total > RC_BOTTOM - 0x100)
            context_rescale(n, 0, ROOT_MIN);

    advance:                                                        /* :331-336 */
        if (order >= SUB_ORDER) predicted = n[predicted].parent;
        else ++order;
        if (pool.next >= POOL_NODES - SUB_ORDER) {                  /* :148-157 */
            pool.next = 0;
            context_new(&pool, ROOT_ESC_MIN, ROOT_MIN);
            predicted = 0;
            order = 0;
        }
    }

    if (!enc_flush(&e)) return 0;
    return (size_t) (e.out - out);
}

/* --------------------------------------------------------------- decoder */

typedef struct { uint32_t low, code, range; const uint8_t *ip, *ie; } dec_t;

/* compress.c:352: READ, truncated to 16 bits by its callers (:545, :575) */
static uint16_t dec_read(dec_t *d, uint16_t total)
{
    d->range /= total;
    return (uint16_t) ((d->code - d->low) / d->range);
}

/* compress.c:354-371 */
static void dec_code(dec_t *d, uint32_t under, uint32_t count)
{
    d->low += under * d->range;
    d->range *= count;
    for (;;) {
        if ((d->low ^ (d->low + d->range)) >= RC_TOP) {
            if (d->range >= RC_BOTTOM) break;
            d->range = (0u - d->low) & (RC_BOTTOM - 1);
        }
        d->code <<= 8;
        if (d->ip < d->ie) d->code |= *d->ip++;
        d->range <<= 8;
        d->low <<= 8;
    }
}

/* compress.c:373-416 with minimum 0: locate the symbol whose interval holds
 * `code` in an order-1/2 context.  Returns 0 (corrupt) on a miss. */
static int sub_decode(pool_t *p, uint16_t ctx, uint16_t code, uint8_t *value,
                      uint16_t *under_, uint16_t *count_, uint16_t *sym)
{
    or_node *n = p->n;
    uint16_t under = 0, count = 0, cur;
    if (!n[ctx].child) return 0;
    cur = n[ctx].child;
    for (;;) {
        or_node *s = &n[cur];
        uint16_t after = (uint16_t) (under + s->under), before = s->count;
        if (code >= after) {
            under = (uint16_t) (under + s->under);
            if (s->right) { cur = s->right; continue; }
            return 0;
        } else if (code < after - before) {
            s->under = (uint16_t) (s->under + SUB_DELTA);
            if (s->left) { cur = s->left; continue; }
            return 0;
        }
        *value = s->value;
        count = (uint16_t) (count + s->count);
        under = (uint16_t) (after - before);
        s->under = (uint16_t) (s->under + SUB_DELTA);
        s->count = (uint8_t) (s->count + SUB_DELTA);
        *sym = cur;
        break;
    }
    *under_ = under; *count_ = count;
    return 1;
}

/* compress.c:373-413 + 418-438 with minimum 1: the root context, where a
 * miss creates the implicit symbol the code points at (value truncated to
 * 8 bits, compress.c:428/:434). */
static void root_decode(pool_t *p, uint16_t code, uint8_t *value,
                        uint16_t *under_, uint16_t *count_, uint16_t *sym)
{
    or_node *n = p->n;
    uint16_t under = 0, count = ROOT_MIN, cur;
    if (!n[0].child) {
        *value = (uint8_t) (code / ROOT_MIN);
        under = (uint16_t) (code - code % ROOT_MIN);
        *sym = node_new(p, *value, ROOT_DELTA);
        n[0].child = *sym;
        *under_ = under; *count_ = count;
        return;
    }
    cur = n[0].child;
    for (;;) {
        or_node *s = &n[cur];
        uint16_t after = (uint16_t) (under + s->under + (s->value + 1) * ROOT_MIN);
        uint16_t before = (uint16_t) (s->count + ROOT_MIN);
        if (code >= after) {
            under = (uint16_t) (under + s->under);
            if (s->right) { cur = s->right; continue; }
            *value = (uint8_t) (s->value + 1 + (code - after) / ROOT_MIN);
            under = (uint16_t) (code - (code - after) % ROOT_MIN);
            *sym = node_new(p, *value, ROOT_DELTA);
            n[cur].right = *sym;
        } else if (code < after - before) {
            s->under = (uint16_t) (s->under + ROOT_DELTA);
            if (s->left) { cur = s->left; continue; }
            *value = (uint8_t) (s->value - 1 - (after - before - code - 1) / ROOT_MIN);
            under = (uint16_t) (code - (after - before - code - 1) % ROOT_MIN);
            *sym = node_new(p, *value, ROOT_DELTA);
            n[cur].left = *sym;
        } else {
            *value = s->value;
            count = (uint16_t) (count + s->count);
            under = (uint16_t) (after - before);
            s->under = (uint16_t) (s->under + ROOT_DELTA);
            s->count = (uint8_t) (s->count + ROOT_DELTA);
            *sym = cur;
        }
        break;
    }
    *under_ = under; *count_ = count;
}

/* compress.c:498-627 */
size_t or_decompress(or_coder *coder, const uint8_t *in, size_t in_limit,
                     uint8_t *out, size_t out_limit)
{
    pool_t pool;
    dec_t d;
    uint8_t *op = out, *oe = out + out_limit;
    uint16_t predicted = 0;
    size_t order = 0;

    if (coder == NULL || in_limit == 0) return 0;                 /* :513-514 */

    pool.n = coder->n; pool.next = 0;
    context_new(&pool, ROOT_ESC_MIN, ROOT_MIN);
    d.low = 0; d.code = 0; d.range = ~0u; d.ip = in; d.ie = in + in_limit;
    /* seed, compress.c:344-350 */
    if (d.ip < d.ie) d.code |= (uint32_t) *d.ip++ << 24;
    if (d.ip < d.ie) d.code |= (uint32_t) *d.ip++ << 16;
    if (d.ip < d.ie) d.code |= (uint32_t) *d.ip++ << 8;
    if (d.ip < d.ie) d.code |= *d.ip++;

    for (;;) {
        or_node *n = pool.n;
        uint16_t *link = &predicted, under = 0, count = 0, total, code, bottom = 0;
        uint16_t ctx, sym = 0, patch;
        uint8_t value = 0;

        /* order-2 / order-1 contexts, compress.c:529-568 */
        for (ctx = predicted; ctx != 0; ctx = n[ctx].parent) {
            if (n[ctx].escapes <= 0) continue;
            total = n[ctx].total;
            if (n[ctx].escapes >= total) continue;
            code = dec_read(&d, total);
            if (code < n[ctx].escapes) {
                dec_code(&d, 0, n[ctx].escapes);
                continue;
            }
            code = (uint16_t) (code - n[ctx].escapes);
            if (!sub_decode(&pool, ctx, code, &value, &under, &count, &sym)) return 0;
            bottom = sym;
            dec_code(&d, (uint32_t) n[ctx].escapes + under, count);
            n[ctx].total = (uint16_t) (n[ctx].total + SUB_DELTA);
            if (count > 0xFF - 2 * SUB_DELTA || n[ctx].total > RC_BOTTOM - 0x100)
                context_rescale(n, ctx, 0);
            goto patch_contexts;
        }

        /* root, compress.c:570-596; a root escape is end of stream */
        total = n[0].total;
        code = dec_read(&d, total);
        if (code < n[0].escapes) {
            dec_code(&d, 0, n[0].escapes);
            break;
        }
        code = (uint16_t) (code - n[0].escapes);
        root_decode(&pool, code, &value, &under, &count, &sym);
        bottom = sym;
        dec_code(&d, (uint32_t) n[0].escapes + under, count);
        n[0].total = (uint16_t) (n[0].total + ROOT_DELTA);
        if (count > 0xFF - 2 * ROOT_DELTA + ROOT_MIN || n[0].total > RC_BOTTOM - 0x100)
            context_rescale(n, 0, ROOT_MIN);

    patch_contexts:
        /* compress.c:598-615: replay the encoder's updates on every context
         * above the one that produced the symbol. */
        for (patch = predicted; patch != ctx; patch = n[patch].parent) {
            sym = context_encode(&pool, patch, value, &under, &count, SUB_DELTA, 0);
            *link = sym;
            link = &n[sym].parent;
            if (count <= 0) {
                n[patch].escapes = (uint16_t) (n[patch].escapes + SUB_ESC_DELTA);
                n[patch].total = (uint16_t) (n[patch].total + SUB_ESC_DELTA);
            }
            n[patch].total = (uint16_t) (n[patch].total + SUB_DELTA);
            if (count > 0xFF - 2 * SUB_DELTA || n[patch].total > RC_BOTTOM - 0x100)
                context_rescale(n, patch, 0);
        }
        *link = bottom;

        if (op >= oe) return 0;                                     /* :617 */
        *op++ = value;

        if (order >= SUB_ORDER) predicted = n[predicted].parent;   /* :619-623 */
        else ++order;
        if (pool.next >= POOL_NODES - SUB_ORDER) {
            pool.next = 0;
            context_new(&pool, ROOT_ESC_MIN, ROOT_MIN);
            predicted = 0;
            order = 0;
        }
    }
    return (size_t) (op - out);
}

/* ------------------------------------------------------------ batch glue */

void or_compress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                       size_t n, uint8_t *out, const uint64_t *out_off,
                       const uint32_t *out_cap, uint32_t *out_len)
{
    or_coder *c = or_create();
    for (size_t i = 0; i < n; ++i) {
        OrBuffer b = { (void *) (in + in_off[i]), in_len[i] };
        out_len[i] = (uint32_t) or_compress(c, &b, 1, in_len[i], out + out_off[i], out_cap[i]);
    }
    or_destroy(c);
}

void or_decompress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                         size_t n, uint8_t *out, const uint64_t *out_off,
                         const uint32_t *out_cap, uint32_t *out_len)
{
    or_coder *c = or_create();
    for (size_t i = 0; i < n; ++i)
        out_len[i] = (uint32_t) or_decompress(c, in + in_off[i], in_len[i],
                                              out + out_off[i], out_cap[i]);
    or_destroy(c);
}

/* FNV-1a-64 over the concatenation, per packet, of (u16le length || bytes):
 * the batch digest of SURVEY.md §8c. */
uint64_t or_fnv1a64_packets(const uint8_t *buf, const uint64_t *off, const uint32_t *len, size_t n)
{
    uint64_t h = 0xcbf29ce484222325ull;
    const uint64_t prime = 0x100000001b3ull;
    for (size_t i = 0; i < n; ++i) {
        uint8_t hdr[2] = { (uint8_t) (len[i] & 0xFF), (uint8_t) ((len[i] >> 8) & 0xFF) };
        h = (h ^ hdr[0]) * prime;
        h = (h ^ hdr[1]) * prime;
        const uint8_t *p = buf + off[i];
        for (uint32_t k = 0; k < len[i]; ++k) h = (h ^ p[k]) * prime;
    }
    return h;
}

/* enet_crc32 (packet.c:143-163): reflected CRC-32, polynomial 0xEDB88320,
 * preset 0xFFFFFFFF, one table lookup per byte across the buffer list, result
 * complemented and put in network byte order (ENET_HOST_TO_NET_32). The table
 * is generated here from the polynomial rather than spelled out. */
static uint32_t crc_table[256];
static int crc_table_ready;

static void crc_init(void)
{
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t c = b;
        for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
        crc_table[b] = c;
    }
    crc_table_ready = 1;
}

uint32_t or_crc32(const OrBuffer *bufs, size_t nbufs)
{
    if (!crc_table_ready) crc_init();
    uint32_t crc = 0xFFFFFFFFu;
    for (size_t i = 0; i < nbufs; ++i) {
        const uint8_t *p = (const uint8_t *) bufs[i].data;
        for (size_t k = 0; k < bufs[i].dataLength; ++k) crc = (crc >> 8) ^ crc_table[(crc ^ p[k]) & 0xFFu];
    }
    crc = ~crc;
    return ((crc & 0xFFu) << 24) | ((crc & 0xFF00u) << 8) | ((crc >> 8) & 0xFF00u) | (crc >> 24);
}

void or_crc32_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len, size_t n,
                    uint32_t *crc_out)
{
    for (size_t i = 0; i < n; ++i) {
        OrBuffer b = { (void *) (in + in_off[i]), in_len[i] };
        crc_out[i] = or_crc32(&b, 1);
    }
}
