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
 *   device pointers: the batch lives on the first listed device (the root),
 *                    which computes the split and each range's byte extents
 *                    (rc_multi_plan.hip; the host reads back 5 words per
 *                    device, nothing per packet); every other device's range
 *                    is copied to it over the peer link (hipMemcpyPeerAsync:
 *                    xGMI between MI355X), its offsets rebased there and
 *                    coded there; its slot range comes back over the link in
 *                    one copy into a root stage buffer sized from the plan,
 *                    the root's stream waits for that device's event, and a
 *                    copy kernel on the root moves each packet's produced
 *                    bytes into the root's slots -- nothing outside
 *                    [out_off[i], out_off[i] + out_len[i]) is written, and the
 *                    host waits for nothing between the plan's read-back and
 *                    the end.  (ENET_RC_MULTI_PEER_READ=1: the copy kernel
 *                    reads the device's slots over the link directly, no
 *                    stage; cross-device visibility of that read after the
 *                    event wait is unmeasured without a multi-GPU box.)
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
    int peer;                       /* the root reads this device's memory directly (same device, or peer access) */
    uint8_t *buf;                   /* device version, non-root: this device's copy of its range */
    size_t buf_cap;
    hipEvent_t done;                /* its results are ready for the root to read */
} rc_dev;

typedef struct {
    size_t n;
    rc_dev d[RC_MULTI_MAX];
    uint8_t *stage;                 /* root: slot ranges of devices without peer access */
    size_t stage_cap;
    uint64_t *d_plan;               /* root: the split's plan and scan words (rc_multi_plan.hip) */
    size_t plan_cap;
    uint64_t *h_plan;               /* pinned: the plan as read back */
    hipEvent_t ready;               /* root: the caller's inputs */
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
    if (m->n) {
        hipSetDevice(m->d[0].device);
        if (m->stage) hipFree(m->stage);
        if (m->d_plan) hipFree(m->d_plan);
        if (m->ready) hipEventDestroy(m->ready);
    }
    if (m->h_plan) hipHostFree(m->h_plan);
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
    hipSetDevice(devices[0]);
    if (hipEventCreateWithFlags(&m->ready, hipEventDisableTiming) != hipSuccess) goto fail;
    if (hipHostMalloc((void **) &m->h_plan, (5 * RC_MULTI_MAX + 1) * 8, 0) != hipSuccess) {
        m->h_plan = NULL;
        goto fail;
    }
    /* peer access between the root and every other device (xGMI) for the
     * copies.  The results of another device come back as a DMA of its slot
     * range into the root's stage buffer (hipMemcpyPeerAsync), which the
     * root's copy kernel then reads: that the root's kernel sees a peer's
     * writes when it reads them across the link after only an event wait is
     * unmeasured here (one GPU per test box), so the direct read of a peer's
     * slots is opt-in, ENET_RC_MULTI_PEER_READ=1.  A range on the root's own
     * device is read in place (ENET_RC_MULTI_NO_PEER=1: through the stage
     * too -- the test switch that runs the stage path on one GPU). */
    const char *pr = getenv("ENET_RC_MULTI_PEER_READ"), *np = getenv("ENET_RC_MULTI_NO_PEER");
    const int peer_read = pr && atoi(pr) != 0, no_peer = np && atoi(np) != 0;
    m->d[0].peer = 1;
    for (size_t k = 1; k < n_devices; ++k) {
        if (devices[k] == devices[0]) { m->d[k].peer = !no_peer; continue; }
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, devices[0], devices[k]) == hipSuccess && can) {
            hipSetDevice(devices[0]);
            const hipError_t e = hipDeviceEnablePeerAccess(devices[k], 0);
            m->d[k].peer = peer_read && !no_peer && (e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled);
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

/* The split with the byte ranges each part covers: first[0 .. parts] as
 * enet_rc_multi_split, then per part k at plan[parts + 1 + 4k]: the lowest
 * in_off, highest in_off + in_len, lowest out_off, highest out_off + out_cap
 * (UINT64_MAX, 0, UINT64_MAX, 0 when the part is empty).  Host restatement
 * of rc_multi_plan.hip, which computes it on the root device. */
int enet_rc_multi_plan(const uint32_t *in_len, const uint64_t *in_off, const uint64_t *out_off,
                       const uint32_t *out_cap, size_t n, size_t parts, uint64_t *plan)
{
    if (!plan || (n && (!in_off || !out_off || !out_cap))) return -1;
    if (enet_rc_multi_split(in_len, n, parts, plan) != 0) return -1;
    uint64_t *ext = plan + parts + 1;
    for (size_t k = 0; k < parts; ++k) {
        uint64_t *e = ext + 4 * k;
        e[0] = UINT64_MAX; e[1] = 0; e[2] = UINT64_MAX; e[3] = 0;
        for (uint64_t i = plan[k]; i < plan[k + 1]; ++i) {
            if (in_off[i] < e[0]) e[0] = in_off[i];
            if (in_off[i] + in_len[i] > e[1]) e[1] = in_off[i] + in_len[i];
            if (out_off[i] < e[2]) e[2] = out_off[i];
            if (out_off[i] + out_cap[i] > e[3]) e[3] = out_off[i] + out_cap[i];
        }
    }
    return 0;
}

/* root-side buffers of the plan: the device's scan words and plan, the pinned
 * copy the host reads */
static int plan_reserve(rc_multi *m, size_t n)
{
    const size_t need = rc_hip_multi_plan_ws(n) + 5 * RC_MULTI_MAX + 1;
    if (need <= m->plan_cap) return 0;
    if (m->d_plan) { hipStreamSynchronize((hipStream_t) rc_ctx_stream(m->d[0].ctx)); hipFree(m->d_plan); }
    m->d_plan = NULL; m->plan_cap = 0;
    if (hipMalloc((void **) &m->d_plan, need * 8) != hipSuccess) return -1;
    m->plan_cap = need;
    return 0;
}

/* The plan on the root's stream (behind the caller's inputs) and its one
 * small read-back: the only host wait before the ranges go out. */
static int device_plan(rc_multi *m, const uint64_t *in_off, const uint32_t *in_len, size_t n,
                       const uint64_t *out_off, const uint32_t *out_cap, void *rst)
{
    if (plan_reserve(m, n) != 0) return (int) hipErrorOutOfMemory;
    uint64_t *dplan = m->d_plan, *ws = m->d_plan + 5 * RC_MULTI_MAX + 1;
    int rc = rc_hip_multi_plan(in_len, in_off, out_off, out_cap, n, (uint32_t) m->n, ws, dplan, rst);
    if (rc) return rc;
    hipError_t err = hipMemcpyAsync(m->h_plan, dplan, (5 * m->n + 1) * 8, hipMemcpyDeviceToHost, (hipStream_t) rst);
    if (err == hipSuccess) err = hipStreamSynchronize((hipStream_t) rst);
    return (int) err;
}

/* one non-root device's share: layout of its buffer */
typedef struct {
    size_t lo, cnt;                 /* packet range */
    uint64_t lo_in, pay;            /* input bytes [lo_in, lo_in + pay) of the root's in */
    uint64_t lo_out, slots;         /* output slot bytes [lo_out, lo_out + slots) */
    size_t a_ioff, a_ilen, a_out, a_ooff, a_ocap, a_olen, total;
} share;

/* root stage bytes for the devices the root cannot read directly: each one's
 * whole slot range, sized from the plan (no read-back of produced sizes) */
static int stage_reserve_multi(rc_multi *m, uint64_t need, void *rst)
{
    if (need <= m->stage_cap) return 0;
    hipStreamSynchronize((hipStream_t) rst);
    if (m->stage) hipFree(m->stage);
    m->stage = NULL; m->stage_cap = 0;
    if (hipMalloc((void **) &m->stage, need) != hipSuccess) return (int) hipErrorOutOfMemory;
    m->stage_cap = need;
    return 0;
}

static int multi_device(rc_multi *m, int decompress, const uint8_t *in, const uint64_t *in_off,
                        const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                        const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len, void *stream,
                        int have_stream)
{
    if (!m) return (int) hipErrorInvalidValue;
    if (n == 0) return 0;
    if (n > 0xFFFFFFFFu) return (int) hipErrorInvalidValue;
    int prev = 0;
    hipGetDevice(&prev);
    const int root = m->d[0].device;
    void *rst = rc_ctx_stream(m->d[0].ctx);
    hipError_t err = hipSetDevice(root);
    /* the caller's inputs: complete on the caller's stream (the root's stream
     * waits for an event recorded there; the host does not), or -- no stream
     * given -- on the whole root device (a device-wide wait: streams created
     * non-blocking, as PyTorch's are, do not order with the null stream) */
    if (err == hipSuccess) {
        if (have_stream) {
            err = hipEventRecord(m->ready, (hipStream_t) stream);
            if (err == hipSuccess) err = hipStreamWaitEvent((hipStream_t) rst, m->ready, 0);
        } else {
            err = hipDeviceSynchronize();
        }
    }
    if (err != hipSuccess) { hipSetDevice(prev); return (int) err; }
    int rc = 0;
    if (m->n == 1) {                /* one device: the plain batch */
        rc = rc_ctx_run_device(m->d[0].ctx, decompress, in, in_off, in_len, n, max_len, out, out_off, out_cap,
                               out_len, rst);
        err = hipStreamSynchronize((hipStream_t) rst);
        hipSetDevice(prev);
        return rc ? rc : (int) err;
    }
    rc = device_plan(m, in_off, in_len, n, out_off, out_cap, rst);
    const uint64_t *first = m->h_plan, *ext = m->h_plan + m->n + 1;
    share sh[RC_MULTI_MAX];
    memset(sh, 0, sizeof sh);
    /* the stage for devices without peer access, sized from the plan */
    uint64_t stage_need = 0, stage_at[RC_MULTI_MAX];
    for (size_t k = 1; k < m->n && !rc; ++k) {
        const uint64_t *e = ext + 4 * k;
        stage_at[k] = stage_need;
        if (!m->d[k].peer && first[k + 1] > first[k]) stage_need += al16(e[3] - e[2]);
    }
    if (!rc && stage_need) rc = stage_reserve_multi(m, stage_need, rst);
    /* phase 1: scatter and code -- every device enqueued, nothing waited for */
    for (size_t k = 0; k < m->n && !rc; ++k) {
        rc_dev *d = &m->d[k];
        share *s = &sh[k];
        s->lo = first[k];
        s->cnt = first[k + 1] - first[k];
        if (s->cnt == 0) continue;
        void *st = rc_ctx_stream(d->ctx);
        if (k == 0) {               /* the root codes its range in place */
            if ((err = hipSetDevice(root)) != hipSuccess) { rc = (int) err; break; }
            rc = rc_ctx_run_device(d->ctx, decompress, in, in_off + s->lo, in_len + s->lo, s->cnt, max_len, out,
                                   out_off + s->lo, out_cap + s->lo, out_len + s->lo, st);
            continue;
        }
        const uint64_t *e = ext + 4 * k;
        s->lo_in = e[0];
        s->pay = e[1] - e[0];
        s->lo_out = e[2];
        s->slots = e[3] - e[2];
        s->a_ioff = al16(s->pay);
        s->a_ilen = s->a_ioff + s->cnt * 8;
        s->a_out = al16(s->a_ilen + s->cnt * 4);
        s->a_ooff = al16(s->a_out + s->slots);
        s->a_ocap = s->a_ooff + s->cnt * 8;
        s->a_olen = al16(s->a_ocap + s->cnt * 4);
        s->total = s->a_olen + s->cnt * 4 + 16;
        if ((err = hipSetDevice(d->device)) != hipSuccess) { rc = (int) err; break; }
        if (s->total > d->buf_cap) {
            hipStreamSynchronize((hipStream_t) st);
            if (d->buf) hipFree(d->buf);
            d->buf = NULL; d->buf_cap = 0;
            if (hipMalloc((void **) &d->buf, s->total) != hipSuccess) { rc = (int) hipErrorOutOfMemory; break; }
            d->buf_cap = s->total;
        }
        uint8_t *b = d->buf;
        /* the range's bytes and metadata over the peer link; offsets rebased there */
        hipStream_t hs = (hipStream_t) st;
        err = hipMemcpyPeerAsync(b, d->device, in + s->lo_in, root, s->pay, hs);
        if (err == hipSuccess) err = hipMemcpyPeerAsync(b + s->a_ioff, d->device, in_off + s->lo, root, s->cnt * 8, hs);
        if (err == hipSuccess) err = hipMemcpyPeerAsync(b + s->a_ilen, d->device, in_len + s->lo, root, s->cnt * 4, hs);
        if (err == hipSuccess) err = hipMemcpyPeerAsync(b + s->a_ooff, d->device, out_off + s->lo, root, s->cnt * 8, hs);
        if (err == hipSuccess) err = hipMemcpyPeerAsync(b + s->a_ocap, d->device, out_cap + s->lo, root, s->cnt * 4, hs);
        if (err != hipSuccess) { rc = (int) err; break; }
        rc = rc_hip_multi_rebase((uint64_t *) (b + s->a_ioff), s->lo_in, (uint64_t *) (b + s->a_ooff), s->lo_out,
                                 s->cnt, st);
        if (rc) break;
        rc = rc_ctx_run_device(d->ctx, decompress, b, (const uint64_t *) (b + s->a_ioff),
                               (const uint32_t *) (b + s->a_ilen), s->cnt, max_len, b + s->a_out,
                               (const uint64_t *) (b + s->a_ooff), (const uint32_t *) (b + s->a_ocap),
                               (uint32_t *) (b + s->a_olen), st);
        if (rc) break;
        /* the lengths to the root; without peer access the whole slot range too */
        err = hipMemcpyPeerAsync(out_len + s->lo, root, b + s->a_olen, d->device, s->cnt * 4, hs);
        if (err == hipSuccess && !d->peer)
            err = hipMemcpyPeerAsync(m->stage + stage_at[k], root, b + s->a_out, d->device, s->slots, hs);
        if (err == hipSuccess) err = hipEventRecord(d->done, hs);
        if (err != hipSuccess) { rc = (int) err; break; }
    }
    /* phase 2: gather -- the root's stream waits for each device's event, then
     * one copy kernel per device moves each packet's produced bytes into the
     * root's slots, reading the device's slots over the link (or the stage) */
    if (!rc) hipSetDevice(root);
    for (size_t k = 1; k < m->n && !rc; ++k) {
        share *s = &sh[k];
        if (s->cnt == 0) continue;
        err = hipStreamWaitEvent((hipStream_t) rst, m->d[k].done, 0);
        if (err != hipSuccess) { rc = (int) err; break; }
        /* src + out_off[i] is packet i's slot on the device: its slots sit at
         * a_out + (out_off[i] - lo_out) */
        const uint8_t *src = (m->d[k].peer ? m->d[k].buf + s->a_out : m->stage + stage_at[k]) - s->lo_out;
        rc = rc_hip_slot_copy(src, out_off + s->lo, out_len + s->lo, (uint32_t) s->cnt, out, 0, rst);
    }
    /* everything done before returning (the device batch calls of one
     * context return with work enqueued; this one returns with results) */
    for (size_t k = 0; k < m->n; ++k) {
        hipSetDevice(m->d[k].device);
        err = hipStreamSynchronize((hipStream_t) rc_ctx_stream(m->d[k].ctx));
        if (!rc && err != hipSuccess) rc = (int) err;
    }
    hipSetDevice(prev);
    return rc;
}

/* The device plan alone (tests: against enet_rc_multi_plan): device pointers
 * on the current device, plan (5 parts + 1 words) to host memory. */
int enet_rc_multi_plan_device(const uint32_t *in_len, const uint64_t *in_off, const uint64_t *out_off,
                              const uint32_t *out_cap, size_t n, size_t parts, uint64_t *plan)
{
    if (!plan || n == 0 || parts == 0 || parts > RC_MULTI_MAX) return (int) hipErrorInvalidValue;
    const size_t words = rc_hip_multi_plan_ws(n) + 5 * parts + 1;
    uint64_t *d = NULL;
    if (hipMalloc((void **) &d, words * 8) != hipSuccess) return (int) hipErrorOutOfMemory;
    int rc = rc_hip_multi_plan(in_len, in_off, out_off, out_cap, n, (uint32_t) parts, d + 5 * parts + 1, d, NULL);
    hipError_t err = rc ? hipSuccess : hipMemcpy(plan, d, (5 * parts + 1) * 8, hipMemcpyDeviceToHost);
    hipFree(d);
    return rc ? rc : (int) err;
}

int enet_rc_multi_compress_batch_device(void *multi, const uint8_t *in, const uint64_t *in_off,
                                        const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                                        const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len)
{
    return multi_device((rc_multi *) multi, 0, in, in_off, in_len, n, max_len, out, out_off, out_cap, out_len, NULL, 0);
}

int enet_rc_multi_decompress_batch_device(void *multi, const uint8_t *in, const uint64_t *in_off,
                                          const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                                          const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len)
{
    return multi_device((rc_multi *) multi, 1, in, in_off, in_len, n, max_len, out, out_off, out_cap, out_len, NULL, 0);
}

int enet_rc_multi_compress_batch_device_stream(void *multi, const uint8_t *in, const uint64_t *in_off,
                                               const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                                               const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len,
                                               void *stream)
{
    return multi_device((rc_multi *) multi, 0, in, in_off, in_len, n, max_len, out, out_off, out_cap, out_len, stream, 1);
}

int enet_rc_multi_decompress_batch_device_stream(void *multi, const uint8_t *in, const uint64_t *in_off,
                                                 const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                                                 const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len,
                                                 void *stream)
{
    return multi_device((rc_multi *) multi, 1, in, in_off, in_len, n, max_len, out, out_off, out_cap, out_len, stream, 1);
}

size_t enet_rc_multi_devices(void *multi) { return multi ? ((rc_multi *) multi)->n : 0; }
