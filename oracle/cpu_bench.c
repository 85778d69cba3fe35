/*
 * cpu_bench.c -- TEST / BASELINE INFRASTRUCTURE ONLY.
 *
 * Times a range-coder round trip on host cores, one coder context per
 * pthread, packets striped across threads (the survey's CPU-baseline plan,
 * SURVEY.md §8d).  The coder is either
 *   - the real reference compress.c, loaded with dlopen() from
 *     oracle/_ref/libenet_ref.so (kind "reference"), or
 *   - this directory's restatement rc_oracle.c (kind "port").
 * Used only by bench.py's cpu_baseline leg and by tests.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rc_oracle.h"

typedef void *(*create_fn)(void);
typedef void (*destroy_fn)(void *);
typedef size_t (*compress_fn)(void *, const OrBuffer *, size_t, size_t, uint8_t *, size_t);
typedef size_t (*decompress_fn)(void *, const uint8_t *, size_t, uint8_t *, size_t);

typedef struct {
    create_fn create; destroy_fn destroy;
    compress_fn compress; decompress_fn decompress;
} coder_vt;

typedef struct {
    const coder_vt *vt;
    const uint8_t *in; const uint64_t *off; const uint32_t *len;
    size_t n; int tid, nthreads;
    uint8_t *cbuf; const uint64_t *coff;   /* compressed scratch, 2N+64 per packet */
    uint32_t *clen;
    uint8_t *dbuf;                          /* decompressed scratch (per thread, 4096 B) */
    int phase;                              /* 0 = compress, 1 = decompress */
    uint64_t mismatches;
} job_t;

static void *worker(void *arg)
{
    job_t *j = (job_t *) arg;
    void *ctx = j->vt->create();
    for (size_t i = (size_t) j->tid; i < j->n; i += (size_t) j->nthreads) {
        if (j->phase == 0) {
            OrBuffer b = { (void *) (j->in + j->off[i]), j->len[i] };
            j->clen[i] = (uint32_t) j->vt->compress(ctx, &b, 1, j->len[i],
                                                    j->cbuf + j->coff[i], 2u * j->len[i] + 64u);
        } else {
            size_t got = j->vt->decompress(ctx, j->cbuf + j->coff[i], j->clen[i],
                                           j->dbuf, 4096);
            if (got != j->len[i] || memcmp(j->dbuf, j->in + j->off[i], got) != 0)
                j->mismatches++;
        }
    }
    j->vt->destroy(ctx);
    return NULL;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

static void *port_create(void) { return or_create(); }
static void port_destroy(void *c) { or_destroy((or_coder *) c); }
static size_t port_compress(void *c, const OrBuffer *b, size_t nb, size_t il, uint8_t *o, size_t ol)
{ return or_compress((or_coder *) c, b, nb, il, o, ol); }
static size_t port_decompress(void *c, const uint8_t *i, size_t il, uint8_t *o, size_t ol)
{ return or_decompress((or_coder *) c, i, il, o, ol); }

/*
 * Round trip over a packed batch.  ref_path == NULL or "" selects the port.
 * Returns 0 on success; fills t_compress/t_decompress (seconds), the total
 * compressed byte count and the number of packets that failed to round-trip.
 * Packets longer than 4096 B are not supported by the decompress scratch.
 */
int cpubench_roundtrip(const char *ref_path, const uint8_t *in, const uint64_t *off,
                       const uint32_t *len, size_t n, int nthreads,
                       double *t_compress, double *t_decompress,
                       uint64_t *compressed_bytes, uint64_t *mismatches)
{
    coder_vt vt;
    void *h = NULL;
    if (ref_path && ref_path[0]) {
        h = dlopen(ref_path, RTLD_NOW | RTLD_LOCAL);
        if (!h) return -1;
        vt.create = (create_fn) dlsym(h, "enet_range_coder_create");
        vt.destroy = (destroy_fn) dlsym(h, "enet_range_coder_destroy");
        vt.compress = (compress_fn) dlsym(h, "enet_range_coder_compress");
        vt.decompress = (decompress_fn) dlsym(h, "enet_range_coder_decompress");
        if (!vt.create || !vt.destroy || !vt.compress || !vt.decompress) { dlclose(h); return -2; }
    } else {
        vt.create = port_create; vt.destroy = port_destroy;
        vt.compress = port_compress; vt.decompress = port_decompress;
    }
    if (nthreads < 1) nthreads = 1;

    uint64_t *coff = (uint64_t *) malloc(n * sizeof(uint64_t));
    uint32_t *clen = (uint32_t *) calloc(n, sizeof(uint32_t));
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) { coff[i] = total; total += 2u * len[i] + 64u; }
    uint8_t *cbuf = (uint8_t *) malloc(total ? total : 1);
    job_t *jobs = (job_t *) calloc((size_t) nthreads, sizeof(job_t));
    pthread_t *th = (pthread_t *) calloc((size_t) nthreads, sizeof(pthread_t));
    uint8_t *dbufs = (uint8_t *) malloc((size_t) nthreads * 4096u);

    for (int phase = 0; phase < 2; ++phase) {
        double t0 = now_s();
        for (int t = 0; t < nthreads; ++t) {
            job_t *j = &jobs[t];
            j->vt = &vt; j->in = in; j->off = off; j->len = len; j->n = n;
            j->tid = t; j->nthreads = nthreads; j->cbuf = cbuf; j->coff = coff;
            j->clen = clen; j->dbuf = dbufs + (size_t) t * 4096u; j->phase = phase;
            pthread_create(&th[t], NULL, worker, j);
        }
        for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
        double dt = now_s() - t0;
        if (phase == 0) *t_compress = dt; else *t_decompress = dt;
    }
    uint64_t cb = 0, mm = 0;
    for (size_t i = 0; i < n; ++i) cb += clen[i];
    for (int t = 0; t < nthreads; ++t) mm += jobs[t].mismatches;
    *compressed_bytes = cb;
    *mismatches = mm;

    free(coff); free(clen); free(cbuf); free(jobs); free(th); free(dbufs);
    if (h) dlclose(h);
    return 0;
}
