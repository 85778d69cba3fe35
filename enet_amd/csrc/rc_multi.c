/*
 * rc_multi.c -- one process, several GPUs.
 *
 * Packets are independent (compress.c keeps no state across calls,
 * compress.c:252-265), so a batch splits into contiguous packet ranges of
 * about equal payload bytes, one per device, and each device codes its range
 * with its own coder context (rc_host.c), concurrently.  This is the C-side
 * counterpart of enet_amd/shard.py (one process per GPU over RCCL): an ENet C
 * host linked against libenet_rc_amd.so can shard with it.
 *
 *   host pointers:   one host thread per device runs that context's
 *                    host-pointer batch (pinned staging, H2D, kernels, D2H)
 *                    on its own range;
 *   device pointers: the batch lives on the first listed device (the root);
 *                    every other device's range is copied to it over the
 *                    peer link (hipMemcpyPeerAsync: xGMI between MI355X),
 *                    coded there, packed back to back (rc_pack.hip) and
 *                    copied back, then unpacked into the root's output slots
 *                    -- only the produced bytes cross the link, and nothing
 *                    outside [out_off[i], out_off[i] + out_len[i]) is written.
 * The split is enet_rc_multi_split (also exported, for tests and callers
 * that place packets themselves).
 */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "enet_rc_amd.h"
#include "rc_abi_internal.h"
#include "rc_host_internal.h"

#define RC_MULTI_MAX 64

typedef struct {
    void *ctx;                      /* coder context bound to the device */
    int device;
    uint8_t *buf;                   /* device version, non-root: this device's copy of its range */
    size_t buf_cap;
    hipEvent_t done;                /* its packed results are on the root */
} rc_dev;

typedef struct {
    size_t n;
    rc_dev d[RC_MULTI_MAX];
    uint8_t *stage;                 /* root: the other devices' packed results */
    size_t stage_cap;
} rc_multi;

int enet_rc_multi_split(const uint32_t *in_len, size_t n, size_t parts, uint64_t *first)
{
    if (!first || parts == 0 || parts > RC_MULTI_MAX || (n && !in_len)) return -1;
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) total += in_len[i];
    /* first[k]: the smallest i whose prefix sum of lengths reaches k / parts of the total */
    size_t i = 0;
    uint64_t acc = 0;
    first[0] = 0;
    for (size_t k = 1; k < parts; ++k) {
        while (i < n && acc * parts < total * k) acc += in_len[i++];
        first[k] = i;
    }
    first[parts] = n;
    return 0;
}

void enet_rc_multi_destroy(void *multi)
{
    rc_multi *m = (rc_multi *) multi;
    if (!m) return;
    int prev = 0;
    hipGetDevice(&prev);
    for (size_t k = 0; k < m->n; ++k) {
        hipSetDevice(m->d[k].device);
        hipDeviceSynchronize();
        if (m->d[k].buf) hipFree(m->d[k].buf);
        if (m->d[k].done) hipEventDestroy(m->d[k].done);
        enet_range_coder_destroy(m->d[k].ctx);
    }
    if (m->stage && m->n) {
        hipSetDevice(m->d[0].device);
        hipFree(m->stage);
    }
    hipSetDevice(prev);
    free(m);
}

void *enet_rc_multi_create(const int *devices, size_t n_devices)
{
    if (!devices || n_devices == 0 || n_devices > RC_MULTI_MAX) return NULL;
    int prev = 0, count = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipGetDeviceCount(&count) != hipSuccess) return NULL;
    rc_multi *m = (rc_multi *) calloc(1, sizeof *m);
    if (!m) return NULL;
    for (size_t k = 0; k < n_devices; ++k) {
        if (devices[k] < 0 || devices[k] >= count || hipSetDevice(devices[k]) != hipSuccess) goto fail;
        m->d[k].device = devices[k];
        m->d[k].ctx = enet_range_coder_create();
        if (!m->d[k].ctx) goto fail;
        m->n = k + 1;
        if (hipEventCreateWithFlags(&m->d[k].done, hipEventDisableTiming) != hipSuccess) goto fail;
    }
    /* direct peer access between the root and every other device (xGMI);
     * where it is unavailable (same device, no link) copies are staged by the
     * runtime, which is slower but correct */
    for (size_t k = 1; k < n_devices; ++k) {
        if (devices[k] == devices[0]) continue;
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, devices[0], devices[k]) == hipSuccess && can) {
            hipSetDevice(devices[0]);
            hipDeviceEnablePeerAccess(devices[k], 0);
            hipSetDevice(devices[k]);
            hipDeviceEnablePeerAccess(devices[0], 0);
        }
    }
    (void) hipGetLastError();       /* "already enabled" is not an error here */
    hipSetDevice(prev);
    return m;
fail:
    hipSetDevice(prev);
    enet_rc_multi_destroy(m);
    return NULL;
}

/* ---------------------------------------------------------- host pointers */

typedef struct {
    void *ctx;
    int decompress;
    const uint8_t *in;
    const uint64_t *in_off;
    const uint32_t *in_len;
    size_t n;
    uint8_t *out;
    const uint64_t *out_off;
    const uint32_t *out_cap;
    uint32_t *out_len;
    int rc;
} host_job;

/* one device's range, its offsets rebased to the range's lowest byte (the
 * host-pointer batch copies [0, max end) of its input) */
static void *host_worker(void *p)
{
    host_job *j = (host_job *) p;
    j->rc = 0;
    if (j->n == 0) return NULL;
    uint64_t lo_in = UINT64_MAX, lo_out = UINT64_MAX;
    for (size_t i = 0; i < j->n; ++i) {
        if (j->in_off[i] < lo_in) lo_in = j->in_off[i];
        if (j->out_off[i] < lo_out) lo_out = j->out_off[i];
    }
    uint64_t *ro = (uint64_t *) malloc(2 * j->n * sizeof(uint64_t));
    if (!ro) { j->rc = (int) hipErrorOutOfMemory; return NULL; }
    for (size_t i = 0; i < j->n; ++i) {
        ro[i] = j->in_off[i] - lo_in;
        ro[j->n + i] = j->out_off[i] - lo_out;
    }
    if (hipSetDevice(rc_ctx_device(j->ctx)) != hipSuccess) j->rc = (int) hipErrorInvalidDevice;
    else j->rc = rc_ctx_run_host(j->ctx, j->decompress, j->in + lo_in, ro, j->in_len, j->n, j->out + lo_out,
                                 ro + j->n, j->out_cap, j->out_len);
    free(ro);
    return NULL;
}

static int multi_host(rc_multi *m, int decompress, const uint8_t *in, const uint64_t *in_off,
                      const uint32_t *in_len, size_t n, uint8_t *out, const uint64_t *out_off,
                      const uint32_t *out_cap, uint32_t *out_len)
{
    if (!m) return (int) hipErrorInvalidValue;
    if (n == 0) return 0;
    uint64_t first[RC_MULTI_MAX + 1];
    if (enet_rc_multi_split(in_len, n, m->n, first) != 0) return (int) hipErrorInvalidValue;
    int prev = 0;
    hipGetDevice(&prev);
    host_job jobs[RC_MULTI_MAX];
    pthread_t th[RC_MULTI_MAX];
    int started[RC_MULTI_MAX] = {0};
    for (size_t k = 0; k < m->n; ++k) {
        const size_t lo = first[k];
        jobs[k] = (host_job){m->d[k].ctx, decompress, in, in_off + lo, in_len + lo, first[k + 1] - lo,
                             out, out_off + lo, out_cap + lo, out_len + lo, 0};
    }
    for (size_t k = 1; k < m->n; ++k) started[k] = pthread_create(&th[k], NULL, host_worker, &jobs[k]) == 0;
    host_worker(&jobs[0]);
    int rc = jobs[0].rc;
    for (size_t k = 1; k < m->n; ++k) {
        if (started[k]) pthread_join(th[k], NULL);
        else host_worker(&jobs[k]);
        if (rc == 0) rc = jobs[k].rc;
    }
    hipSetDevice(prev);
    return rc;
}

int enet_rc_multi_compress_batch_host(void *multi, const uint8_t *in, const uint64_t *in_off,
                                      const uint32_t *in_len, size_t n, uint8_t *out,
                                      const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len)
{
    return multi_host((rc_multi *) multi, 0, in, in_off, in_len, n, out, out_off, out_cap, out_len);
}

int enet_rc_multi_decompress_batch_host(void *multi, const uint8_t *in, const uint64_t *in_off,
                                        const uint32_t *in_len, size_t n, uint8_t *out,
                                        const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len)
{
    return multi_host((rc_multi *) multi, 1, in, in_off, in_len, n, out, out_off, out_cap, out_len);
}

/* -------------------------------------------------------- device pointers */

static size_t al16(size_t x) { return (x + 15) & ~(size_t) 15; }

/* one non-root device's share: layout of its buffer */
typedef struct {
    size_t lo, cnt;                 /* packet range */
    uint64_t lo_in, pay;            /* input bytes [lo_in, lo_in + pay) of the root's in */
    uint64_t slots;                 /* output slot bytes (rebased extent) */
    size_t a_ioff, a_ilen, a_out, a_ooff, a_ocap, a_olen, a_pack, total;
    uint64_t packed;                /* bytes produced (read back after the kernels) */
    uint64_t *h_off;                /* rebased in_off | out_off (host) */
} share;

static int multi_device(rc_multi *m, int decompress, const uint8_t *in, const uint64_t *in_off,
                        const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                        const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len)
{
    if (!m) return (int) hipErrorInvalidValue;
    if (n == 0) return 0;
    if (n > 0xFFFFFFFFu) return (int) hipErrorInvalidValue;
    int prev = 0;
    hipGetDevice(&prev);
    const int root = m->d[0].device;
    hipError_t err = hipSetDevice(root);
    /* the caller's inputs are ready on any stream of the root */
    if (err == hipSuccess) err = hipDeviceSynchronize();
    uint64_t *h_ioff = (uint64_t *) malloc(n * 8), *h_ooff = (uint64_t *) malloc(n * 8);
    uint32_t *h_ilen = (uint32_t *) malloc(n * 4), *h_ocap = (uint32_t *) malloc(n * 4);
    share sh[RC_MULTI_MAX];
    memset(sh, 0, sizeof sh);
    int rc = 0;
    if (!h_ioff || !h_ooff || !h_ilen || !h_ocap) rc = (int) hipErrorOutOfMemory;
    if (!rc && err == hipSuccess) err = hipMemcpy(h_ioff, in_off, n * 8, hipMemcpyDeviceToHost);
    if (!rc && err == hipSuccess) err = hipMemcpy(h_ooff, out_off, n * 8, hipMemcpyDeviceToHost);
    if (!rc && err == hipSuccess) err = hipMemcpy(h_ilen, in_len, n * 4, hipMemcpyDeviceToHost);
    if (!rc && err == hipSuccess) err = hipMemcpy(h_ocap, out_cap, n * 4, hipMemcpyDeviceToHost);
    if (!rc && err != hipSuccess) rc = (int) err;
    uint64_t first[RC_MULTI_MAX + 1];
    if (!rc && enet_rc_multi_split(h_ilen, n, m->n, first) != 0) rc = (int) hipErrorInvalidValue;
    /* phase 1: scatter, code, pack -- every device enqueued before any wait */
    for (size_t k = 0; k < m->n && !rc; ++k) {
        rc_dev *d = &m->d[k];
        share *s = &sh[k];
        s->lo = first[k];
        s->cnt = first[k + 1] - first[k];
        if (s->cnt == 0) continue;
        void *st = rc_ctx_stream(d->ctx);
        if (k == 0) {               /* the root codes its range in place */
            rc = rc_ctx_run_device(d->ctx, decompress, in, in_off + s->lo, in_len + s->lo, s->cnt, max_len, out,
                                   out_off + s->lo, out_cap + s->lo, out_len + s->lo, st);
            continue;
        }
        uint64_t lo_in = UINT64_MAX, hi_in = 0, lo_out = UINT64_MAX, hi_out = 0;
        for (size_t i = s->lo; i < s->lo + s->cnt; ++i) {
            if (h_ioff[i] < lo_in) lo_in = h_ioff[i];
            if (h_ioff[i] + h_ilen[i] > hi_in) hi_in = h_ioff[i] + h_ilen[i];
            if (h_ooff[i] < lo_out) lo_out = h_ooff[i];
            if (h_ooff[i] + h_ocap[i] > hi_out) hi_out = h_ooff[i] + h_ocap[i];
        }
        s->lo_in = lo_in;
        s->pay = hi_in - lo_in;
        s->slots = hi_out - lo_out;
        s->a_ioff = al16(s->pay);
        s->a_ilen = s->a_ioff + s->cnt * 8;
        s->a_out = al16(s->a_ilen + s->cnt * 4);
        s->a_ooff = al16(s->a_out + s->slots);
        s->a_ocap = s->a_ooff + s->cnt * 8;
        s->a_olen = al16(s->a_ocap + s->cnt * 4);
        s->a_pack = al16(s->a_olen + s->cnt * 4);
        s->total = s->a_pack + s->slots + 16;
        s->h_off = (uint64_t *) malloc(2 * s->cnt * 8);
        if (!s->h_off) { rc = (int) hipErrorOutOfMemory; break; }
        for (size_t i = 0; i < s->cnt; ++i) {
            s->h_off[i] = h_ioff[s->lo + i] - lo_in;
            s->h_off[s->cnt + i] = h_ooff[s->lo + i] - lo_out;
        }
        if ((err = hipSetDevice(d->device)) != hipSuccess) { rc = (int) err; break; }
        if (s->total > d->buf_cap) {
            hipDeviceSynchronize();
            if (d->buf) hipFree(d->buf);
            d->buf = NULL; d->buf_cap = 0;
            if (hipMalloc((void **) &d->buf, s->total) != hipSuccess) { rc = (int) hipErrorOutOfMemory; break; }
            d->buf_cap = s->total;
        }
        uint8_t *b = d->buf;
        uint64_t *bsum = rc_ctx_bsum(d->ctx, s->cnt);
        if (!bsum) { rc = (int) hipErrorOutOfMemory; break; }
        err = hipMemcpyPeerAsync(b, d->device, in + lo_in, root, s->pay, (hipStream_t) st);
        if (err == hipSuccess) err = hipMemcpyPeerAsync(b + s->a_ilen, d->device, in_len + s->lo, root, s->cnt * 4,
                                                        (hipStream_t) st);
        if (err == hipSuccess) err = hipMemcpyPeerAsync(b + s->a_ocap, d->device, out_cap + s->lo, root, s->cnt * 4,
                                                        (hipStream_t) st);
        if (err == hipSuccess) err = hipMemcpyAsync(b + s->a_ioff, s->h_off, s->cnt * 8, hipMemcpyHostToDevice,
                                                    (hipStream_t) st);
        if (err == hipSuccess) err = hipMemcpyAsync(b + s->a_ooff, s->h_off + s->cnt, s->cnt * 8,
                                                    hipMemcpyHostToDevice, (hipStream_t) st);
        if (err != hipSuccess) { rc = (int) err; break; }
        rc = rc_ctx_run_device(d->ctx, decompress, b, (const uint64_t *) (b + s->a_ioff),
                               (const uint32_t *) (b + s->a_ilen), s->cnt, max_len, b + s->a_out,
                               (const uint64_t *) (b + s->a_ooff), (const uint32_t *) (b + s->a_ocap),
                               (uint32_t *) (b + s->a_olen), st);
        if (rc) break;
        rc = rc_hip_pack(b + s->a_out, (const uint64_t *) (b + s->a_ooff), (const uint32_t *) (b + s->a_olen),
                         (uint32_t) s->cnt, bsum, b + s->a_pack, st);
        if (rc) break;
        /* the lengths to the root now; the packed bytes once their total is known */
        err = hipMemcpyPeerAsync(out_len + s->lo, root, b + s->a_olen, d->device, s->cnt * 4, (hipStream_t) st);
        if (err == hipSuccess)
            err = hipMemcpyAsync(&s->packed, bsum + (s->cnt + 1023) / 1024, 8, hipMemcpyDeviceToHost, (hipStream_t) st);
        if (err != hipSuccess) { rc = (int) err; break; }
    }
    /* phase 2: gather -- each device's packed bytes to the root's staging,
     * unpacked into the output slots on the root's stream */
    uint64_t stage_need = 0, stage_at[RC_MULTI_MAX];
    for (size_t k = 1; k < m->n && !rc; ++k) {
        if (sh[k].cnt == 0) continue;
        if ((err = hipSetDevice(m->d[k].device)) != hipSuccess ||
            (err = hipStreamSynchronize((hipStream_t) rc_ctx_stream(m->d[k].ctx))) != hipSuccess) { rc = (int) err; break; }
        if (sh[k].packed > sh[k].slots) { rc = (int) hipErrorUnknown; break; }
        stage_at[k] = stage_need;
        stage_need += al16(sh[k].packed);
    }
    void *rst = rc_ctx_stream(m->d[0].ctx);
    if (!rc && stage_need) {
        hipSetDevice(root);
        if (stage_need > m->stage_cap) {
            hipDeviceSynchronize();
            if (m->stage) hipFree(m->stage);
            m->stage = NULL; m->stage_cap = 0;
            if (hipMalloc((void **) &m->stage, stage_need) != hipSuccess) rc = (int) hipErrorOutOfMemory;
            else m->stage_cap = stage_need;
        }
        uint64_t *rbsum = rc ? NULL : rc_ctx_bsum(m->d[0].ctx, n);
        if (!rc && !rbsum) rc = (int) hipErrorOutOfMemory;
        for (size_t k = 1; k < m->n && !rc; ++k) {
            share *s = &sh[k];
            if (s->cnt == 0) continue;
            hipSetDevice(m->d[k].device);
            void *st = rc_ctx_stream(m->d[k].ctx);
            err = s->packed ? hipMemcpyPeerAsync(m->stage + stage_at[k], root, m->d[k].buf + s->a_pack, m->d[k].device,
                                                 s->packed, (hipStream_t) st) : hipSuccess;
            if (err == hipSuccess) err = hipEventRecord(m->d[k].done, (hipStream_t) st);
            if (err == hipSuccess) { hipSetDevice(root); err = hipStreamWaitEvent((hipStream_t) rst, m->d[k].done, 0); }
            if (err != hipSuccess) { rc = (int) err; break; }
            rc = rc_hip_unpack(m->stage + stage_at[k], out, out_off + s->lo, out_len + s->lo, (uint32_t) s->cnt,
                               rbsum, rst);
        }
    }
    /* everything done before returning (the device batch calls of one
     * context return with work enqueued; this one returns with results) */
    for (size_t k = 0; k < m->n; ++k) {
        hipSetDevice(m->d[k].device);
        err = hipStreamSynchronize((hipStream_t) rc_ctx_stream(m->d[k].ctx));
        if (!rc && err != hipSuccess) rc = (int) err;
        free(sh[k].h_off);
    }
    free(h_ioff); free(h_ooff); free(h_ilen); free(h_ocap);
    hipSetDevice(prev);
    return rc;
}

int enet_rc_multi_compress_batch_device(void *multi, const uint8_t *in, const uint64_t *in_off,
                                        const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                                        const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len)
{
    return multi_device((rc_multi *) multi, 0, in, in_off, in_len, n, max_len, out, out_off, out_cap, out_len);
}

int enet_rc_multi_decompress_batch_device(void *multi, const uint8_t *in, const uint64_t *in_off,
                                          const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                                          const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len)
{
    return multi_device((rc_multi *) multi, 1, in, in_off, in_len, n, max_len, out, out_off, out_cap, out_len);
}

size_t enet_rc_multi_devices(void *multi) { return multi ? ((rc_multi *) multi)->n : 0; }
