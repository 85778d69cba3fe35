/*
 * rc_host.c -- C host side of the MI355X range coder.
 *
 * Implements the reference's compressor plugin surface (enet.h:323-335,
 * :574, :603-606) on top of the HIP kernels in rc_kernels.hip:
 *   - a coder context owns a HIP stream, a device workspace and pinned
 *     staging;
 *   - the per-datagram entry points run a one-packet batch on the GPU (the
 *     gather list is flattened on the host exactly as compress.c:275-284
 *     consumes it);
 *   - the batch entry points hand whole packet batches to the kernels.
 * There is no CPU coder in this library: if no HIP device is usable,
 * enet_range_coder_create() returns NULL and the batch calls fail.
 */
#define _POSIX_C_SOURCE 200809L
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <time.h>

#include "enet_rc_amd.h"
#include "rc_abi_internal.h"
#include "rc_host_internal.h"

/* ENet's allocator and host hook, resolved from libenet when it is linked
 * (callbacks.c:37-52, host.c:294-304). */
extern void *enet_malloc(size_t) __attribute__((weak));
extern void enet_free(void *) __attribute__((weak));
extern void enet_host_compress(ENetHost *, const ENetCompressor *) __attribute__((weak));

#define SPLIT_MAX 4                 /* pieces of a large host batch (run_host_split) */
#define SPLIT_DEFAULT 3
#define EXACT_SLOTS 256u            /* concurrent exact-path packets (64 KiB pool each) */

typedef struct {
    int device;
    hipStream_t stream;
    rc_workspace_dev ws;            /* flag list sized n_cap */
    /* device staging for host-pointer calls */
    uint8_t *d_stage;
    size_t d_stage_cap;
    uint8_t *h_stage;               /* pinned */
    size_t h_stage_cap;
    uint32_t last_exact;
    uint32_t max_slots;             /* lanes with a model region (ENET_RC_SLOTS) */
    int enc2_on;                    /* compress batches on the two-pass encoder (ENET_RC_ENC2=0: off) */
    int enc2_wide_on;               /* ... and its wide mode (ENET_RC_ENC2_WIDE=0: off) */
    uint64_t enc2_stream_max;       /* record-stream caps, read when the context is created */
    uint64_t enc2_wide_max;
    uint64_t enc2_failed;     /* the smallest record-stream size an allocation failed for (0: none) */
    uint32_t *crc_tables;           /* device: slice-by-16 + shift tables (rc_crc32.hip) */
    /* datagram framing workspace (rc_dgram.hip): per-datagram arrays + checksum scratch */
    uint8_t *dg_arrays;
    size_t dg_cap;
    uint8_t *dg_scratch;
    size_t dg_scratch_cap;
    /* host-pointer calls: outputs packed back to back before D2H (rc_pack.hip) */
    uint8_t *d_pack;
    size_t d_pack_cap;
    uint64_t *d_bsum;
    size_t d_bsum_cap;
    /* host batches in pieces (run_host_split): the further contexts on the
       device, and the hand-off of each piece's input DMA to the next piece */
    void *twin[SPLIT_MAX - 1];
    struct h2d_sync *sync_sig, *sync_wait;
    int last_split;                 /* pieces of the last host batch (0: one piece) */
    uint32_t last_paths;            /* enet_rc_last_host_paths */
    int split_k;                    /* pieces of a large host batch (ENET_RC_HOST_SPLIT) */
} rc_ctx;

/* A piece records ev on its stream once its input DMA is enqueued (ready 1;
 * -1: it ended before that), the next piece's stream waits for it before its
 * own. */
struct h2d_sync {
    pthread_mutex_t m;
    pthread_cond_t cv;
    int ready;
    hipEvent_t ev;
};

static void h2d_sync_set(struct h2d_sync *y, int v)
{
    pthread_mutex_lock(&y->m);
    if (!y->ready) y->ready = v;
    pthread_cond_broadcast(&y->cv);
    pthread_mutex_unlock(&y->m);
}

static void *ctx_alloc(size_t n) { return enet_malloc ? enet_malloc(n) : malloc(n); }
static void ctx_release(void *p) { if (enet_free) enet_free(p); else free(p); }

static int ws_reserve(rc_ctx *c, size_t n)
{
    if (n <= c->ws.n_cap) return 0;
    size_t cap = c->ws.n_cap ? c->ws.n_cap : 1024;
    while (cap < n) cap *= 2;
    uint32_t *fl = NULL, *ord = NULL, *el = NULL, *wl = NULL, *cl = NULL;
    /* claims, the decoder's reset positions and its two hand-off sums side by side */
    if (hipMalloc((void **) &cl, 5 * cap * sizeof(uint32_t)) != hipSuccess) return -1;
    if (hipMalloc((void **) &fl, cap * sizeof(uint32_t)) != hipSuccess) { hipFree(cl); return -1; }
    if (hipMalloc((void **) &ord, cap * sizeof(uint32_t)) != hipSuccess) { hipFree(cl); hipFree(fl); return -1; }
    if (hipMalloc((void **) &el, cap * sizeof(uint32_t)) != hipSuccess) {
        hipFree(cl); hipFree(fl); hipFree(ord); return -1;
    }
    if (hipMalloc((void **) &wl, cap * sizeof(uint32_t)) != hipSuccess) {
        hipFree(cl); hipFree(fl); hipFree(ord); hipFree(el); return -1;
    }
    if (c->ws.flag_list) {
        hipDeviceSynchronize();
        hipFree(c->ws.flag_list);
        hipFree(c->ws.order);
        hipFree(c->ws.enc2_list);
        hipFree(c->ws.enc2_wlist);
        hipFree(c->ws.claims);
    }
    c->ws.claims = cl;
    c->ws.dec6_resets = cl + cap;
    c->ws.dec6_icks = cl + 2 * cap;
    c->ws.dec6_hcks = cl + 3 * cap;
    c->ws.flag_list = fl;
    c->ws.order = ord;
    c->ws.enc2_list = el;
    c->ws.enc2_wlist = wl;
    c->ws.n_cap = (uint32_t) cap;
    return 0;
}

/* Per-lane model regions for the lane kernels: one per packet in flight
 * (at most one per lane of a full chip wave set; larger batches loop). */
#define MAX_LANE_SLOTS 65536u

static int lanes_reserve(rc_ctx *c, size_t n, uint32_t max_len)
{
    uint32_t region = rc_hip_lane3_region_bytes(max_len ? max_len : 4096);
    const char *ov = getenv("ENET_RC_REGION");      /* diagnostic: smaller regions (overflows take the exact path) */
    if (ov && atoi(ov) > 0 && (uint32_t) atoi(ov) < region) region = ((uint32_t) atoi(ov) + 255) & ~255u;
    /* (whole 8192-slot groups: the pieces of a split host batch differ by a
       few thousand packets between calls, and a pool that grew by each would
       be reallocated -- a device-wide wait -- on the calls after the first) */
    size_t slots = n >= 8192 ? (n + 8191) & ~(size_t) 8191 : n;
    if (slots > c->max_slots) slots = c->max_slots;
    slots = (slots + 255) & ~(size_t) 255;
    if (slots <= c->ws.lane_slots && region <= c->ws.lane_region) return 0;
    if (slots < c->ws.lane_slots) slots = c->ws.lane_slots;
    if (region < c->ws.lane_region) region = c->ws.lane_region;
    hipDeviceSynchronize();
    if (c->ws.lane_pool) hipFree(c->ws.lane_pool);
    if (c->ws.dec6_pool) hipFree(c->ws.dec6_pool);
    c->ws.lane_pool = NULL; c->ws.dec6_pool = NULL; c->ws.lane_slots = 0; c->ws.lane_region = 0;
    if (hipMalloc(&c->ws.lane_pool, slots * (size_t) region) != hipSuccess) return -1;
    /* rc_dec6.hip's bucket records: never cleared (a record's stale bytes past
       the bucket's element count are never read) */
    if (hipMalloc(&c->ws.dec6_pool, slots * (size_t) RC_DEC6_TAB_BYTES) != hipSuccess) return -1;
    /* lane regions start at epoch 0: no order-1 record is live (rc_lane3.hip) */
    if (hipMemset(c->ws.lane_pool, 0, slots * (size_t) region) != hipSuccess) return -1;
    /* hipMemset runs on the null stream, which the context's non-blocking
     * stream (and a caller's) does not wait for: finish it before any kernel */
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    c->ws.lane_slots = (uint32_t) slots;
    c->ws.lane_region = region;
    if (getenv("ENET_RC_DEBUG"))
        fprintf(stderr, "enet_rc: lane pool %p, %zu slots x %u B\n", c->ws.lane_pool, slots, region);
    return 0;
}

/* Record stream of the two-pass encoder (rc_enc2.hip): one slot per packet,
 * at most ENC2_STREAM_MAX bytes (larger batches run in whole code-pass rounds
 * of chunks; ENET_RC_ENC2_STREAM_MB=m caps it lower).  Its wide mode has a
 * stream of 16-B records for as many packets as a chunk holds (at most
 * ENC2_WIDE_MAX bytes, ENET_RC_ENC2_WIDE_MB=m caps it lower: packets past it
 * take the lane kernels; ENET_RC_ENC2_WIDE=0 turns the mode off).  Reserved
 * only for batches that take the lane path (run_device). */
/* (3 GB: a chip's worth of 4096-B packets, 65536 x 32.9 KB, in one chunk --
 * a chunk smaller than that leaves the code pass's lanes partly idle for a
 * whole packet's time) */
#define ENC2_STREAM_MAX (3ull << 30)
#define ENC2_WIDE_MAX (5ull << 30)      /* (65536 wide 4096-B packets: 4.3 GB, one chunk) */

static uint64_t env_mb_cap(const char *name, uint64_t cap)
{
    const char *mb = getenv(name);
    if (mb && atol(mb) > 0 && (uint64_t) atol(mb) << 20 < cap) cap = (uint64_t) atol(mb) << 20;
    return cap;
}

static int enc2_reserve(rc_ctx *c, size_t n, uint32_t max_len)
{
    if (!c->enc2_on || c->ws.kernel != RC_KERNEL_LANE3) return 0;
    const uint32_t ml = max_len ? max_len : 4096;
    const uint64_t slot = rc_hip_enc2_slot_bytes(ml);
    const uint64_t cap = c->enc2_stream_max;
    uint64_t want = (uint64_t) (n >= 8192 ? (n + 8191) & ~(size_t) 8191 : n) * slot;   /* (as lanes_reserve) */
    if (want > cap) want = cap > slot ? cap : slot;
    /* (a size that failed once is not retried: the stream the device could
     * give then serves, in more chunks, without a device-wide sync per call) */
    if (c->enc2_failed && want >= c->enc2_failed && c->ws.enc2_cap) want = c->ws.enc2_cap;
    if (want > c->ws.enc2_cap) {
        hipDeviceSynchronize();
        if (c->ws.enc2_stream) hipFree(c->ws.enc2_stream);
        c->ws.enc2_stream = NULL; c->ws.enc2_cap = 0;
        /* + 1 MB past the stream: the code pass's dummy store targets (rc_enc2.hip).
         * A device short of memory gets a smaller stream (the batch then runs in
         * more chunks), down to one packet's slot. */
        while (hipMalloc(&c->ws.enc2_stream, want + (1u << 20)) != hipSuccess) {
            c->ws.enc2_stream = NULL;
            (void) hipGetLastError();
            if (!c->enc2_failed || want < c->enc2_failed) c->enc2_failed = want;
            if (want <= slot) return -1;
            want = want / 2 > slot ? (want / 2) / slot * slot : slot;
        }
        c->ws.enc2_cap = want;
    }
    if (c->enc2_wide_on) {
        /* a slot per packet of a chunk, and the rounding of its RC_WSHARDS
           list regions (rc_enc2.hip wreg_cap) */
        const uint64_t wslot = rc_hip_enc2_wide_slot_bytes(ml);
        uint64_t wwant = (want / slot + RC_WSHARDS) * wslot;
        const uint64_t wcap = c->enc2_wide_max;
        if (wwant > wcap) wwant = wcap > wslot ? wcap : wslot;
        if (wwant > c->ws.enc2_wide_cap) {
            hipDeviceSynchronize();
            if (c->ws.enc2_wide) hipFree(c->ws.enc2_wide);
            c->ws.enc2_wide = NULL; c->ws.enc2_wide_cap = 0;
            /* the wide mode is optional: without its stream (an allocation that
               failed) low-entropy packets take the lane kernels */
            if (hipMalloc(&c->ws.enc2_wide, wwant) != hipSuccess) {
                c->ws.enc2_wide = NULL;
                (void) hipGetLastError();
                return 0;
            }
            c->ws.enc2_wide_cap = wwant;
        }
    }
    return 0;
}

static int stage_reserve(rc_ctx *c, size_t bytes)
{
    if (bytes <= c->d_stage_cap && bytes <= c->h_stage_cap) return 0;
    size_t cap = 1u << 16;
    while (cap < bytes) cap *= 2;
    hipStreamSynchronize(c->stream);
    if (c->d_stage) hipFree(c->d_stage);
    if (c->h_stage) hipHostFree(c->h_stage);
    c->d_stage = NULL; c->h_stage = NULL; c->d_stage_cap = c->h_stage_cap = 0;
    if (hipMalloc((void **) &c->d_stage, cap) != hipSuccess) return -1;
    if (hipHostMalloc((void **) &c->h_stage, cap, 0) != hipSuccess) return -1;
    c->d_stage_cap = c->h_stage_cap = cap;
    return 0;
}

void *enet_range_coder_create(void)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return NULL;
    rc_ctx *c = (rc_ctx *) ctx_alloc(sizeof(rc_ctx));
    if (!c) return NULL;
    memset(c, 0, sizeof *c);
    c->device = dev;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) goto fail;
    /* counters[8] and the length bins in one block: one fill clears both per call */
    if (hipMalloc((void **) &c->ws.counters, RC_CTL_WORDS * sizeof(uint32_t)) != hipSuccess) goto fail;
    c->ws.bins = c->ws.counters + 8;
    c->ws.exact_slots = EXACT_SLOTS;
    if (hipMalloc(&c->ws.exact_pool, (size_t) EXACT_SLOTS * RC_EXACT_POOL_BYTES) != hipSuccess) goto fail;
    if (ws_reserve(c, 1024) != 0) goto fail;
    {
        const uint32_t words = rc_hip_crc32_table_words();
        uint32_t *t = (uint32_t *) malloc(words * sizeof(uint32_t));
        if (!t) goto fail;
        rc_hip_crc32_build_tables(t);
        hipError_t e = hipMalloc((void **) &c->crc_tables, words * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMemcpy(c->crc_tables, t, words * sizeof(uint32_t), hipMemcpyHostToDevice);
        free(t);
        if (e != hipSuccess) goto fail;
    }
    {
        const char *k = getenv("ENET_RC_KERNEL");
        c->ws.kernel = RC_KERNEL_LANE3;
        if (k && strcmp(k, "wave") == 0) c->ws.kernel = RC_KERNEL_WAVE;
        const char *a = getenv("ENET_RC_LANES");
        c->ws.lane_active = 64;
        if (a && (atoi(a) == 32 || atoi(a) == 16)) c->ws.lane_active = (uint32_t) atoi(a);
        /* ENET_RC_SMALL_BATCH=n caps the batches routed to the wave kernel
         * (0: never); unset = every batch that fits on the chip at once */
        const char *sb = getenv("ENET_RC_SMALL_BATCH");
        c->ws.small_max = sb ? (uint32_t) strtoul(sb, NULL, 10) : RC_SMALL_AUTO;
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || cus <= 0)
            cus = 256;
        c->ws.cus = (uint32_t) cus;
        const char *e2 = getenv("ENET_RC_ENC2");
        c->enc2_on = !(e2 && strcmp(e2, "0") == 0);
        c->ws.enc2_on = (uint32_t) c->enc2_on;
        const char *ew = getenv("ENET_RC_ENC2_WIDE");
        c->enc2_wide_on = !(ew && strcmp(ew, "0") == 0);
        c->enc2_stream_max = env_mb_cap("ENET_RC_ENC2_STREAM_MB", ENC2_STREAM_MAX);
        c->enc2_wide_max = env_mb_cap("ENET_RC_ENC2_WIDE_MB", ENC2_WIDE_MAX);
        /* large host batches in pieces (run_host_split): ENET_RC_HOST_SPLIT=k
           pieces, 2..SPLIT_MAX (0 or 1: off) */
        const char *hs = getenv("ENET_RC_HOST_SPLIT");
        c->split_k = hs ? atoi(hs) : SPLIT_DEFAULT;
        if (c->split_k < 1) c->split_k = 1;
        if (c->split_k > SPLIT_MAX) c->split_k = SPLIT_MAX;
        /* each piece's stream needs a hardware queue of its own (streams
           sharing one run one after the other), and the process's default
           stream holds one of the runtime's GPU_MAX_HW_QUEUES (default 4) */
        const char *hq = getenv("GPU_MAX_HW_QUEUES");
        const int queues = hq && atoi(hq) > 0 ? atoi(hq) : 4;
        if (c->split_k > queues - 1) c->split_k = queues > 2 ? queues - 1 : 1;
        /* the fast decoder: rc_dec6.hip's rc_decompress_dec6s (64 packets per
           wavefront); none with ENET_RC_DEC=0 (ENET_RC_DEC4=0, the older name,
           too) or with 32 / 16 packets per wavefront */
        const char *d4 = getenv("ENET_RC_DEC4");
        const char *dk = getenv("ENET_RC_DEC");
        c->ws.fast_dec = c->ws.lane_active == 64;
        if ((dk && strcmp(dk, "0") == 0) || (d4 && strcmp(d4, "0") == 0)) c->ws.fast_dec = 0;
        const char *dd = getenv("ENET_RC_DEC6_DEBUG");
        c->ws.dec6_debug = dd ? (uint32_t) atoi(dd) : 0u;
        const char *es = getenv("ENET_RC_ENC2_SLOW");
        c->ws.enc2_slow = (es && strcmp(es, "1") == 0) ? 1u : 0u;
        const char *sl = getenv("ENET_RC_SLOTS");
        c->max_slots = MAX_LANE_SLOTS;
        if (sl && atol(sl) >= 256 && atol(sl) <= (1l << 22)) c->max_slots = (uint32_t) atol(sl);
    }
    if (stage_reserve(c, 1u << 16) != 0) goto fail;
    return c;
fail:
    enet_range_coder_destroy(c);
    return NULL;
}

/* The settings enet_range_coder_create reads from the environment, copied
 * from a context to another on the same device (run_host_split's second
 * half runs with its parent's configuration, whatever the environment says
 * by then). */
static void ctx_copy_config(rc_ctx *dst, const rc_ctx *src)
{
    dst->ws.kernel = src->ws.kernel;
    dst->ws.lane_active = src->ws.lane_active;
    dst->ws.small_max = src->ws.small_max;
    dst->ws.cus = src->ws.cus;
    dst->ws.fast_dec = src->ws.fast_dec;
    dst->ws.dec6_debug = src->ws.dec6_debug;
    dst->ws.enc2_slow = src->ws.enc2_slow;
    dst->enc2_on = src->enc2_on;
    dst->ws.enc2_on = src->ws.enc2_on;
    dst->enc2_wide_on = src->enc2_wide_on;
    dst->enc2_stream_max = src->enc2_stream_max;
    dst->enc2_wide_max = src->enc2_wide_max;
    dst->max_slots = src->max_slots;
    dst->split_k = 1;
}

void enet_range_coder_destroy(void *context)
{
    rc_ctx *c = (rc_ctx *) context;
    if (!c) return;
    if (c->stream) hipStreamSynchronize(c->stream);
    if (c->ws.flag_list) hipFree(c->ws.flag_list);
    if (c->ws.counters) hipFree(c->ws.counters);
    if (c->ws.order) hipFree(c->ws.order);
    if (c->ws.enc2_list) hipFree(c->ws.enc2_list);
    if (c->ws.claims) hipFree(c->ws.claims);
    if (c->ws.dec6_pool) hipFree(c->ws.dec6_pool);
    if (c->ws.enc2_stream) hipFree(c->ws.enc2_stream);
    if (c->ws.enc2_wlist) hipFree(c->ws.enc2_wlist);
    if (c->ws.enc2_wide) hipFree(c->ws.enc2_wide);
    if (c->ws.exact_pool) hipFree(c->ws.exact_pool);
    if (c->ws.lane_pool) hipFree(c->ws.lane_pool);
    if (c->crc_tables) hipFree(c->crc_tables);
    if (c->dg_arrays) hipFree(c->dg_arrays);
    if (c->dg_scratch) hipFree(c->dg_scratch);
    if (c->d_pack) hipFree(c->d_pack);
    if (c->d_bsum) hipFree(c->d_bsum);
    if (c->d_stage) hipFree(c->d_stage);
    if (c->h_stage) hipHostFree(c->h_stage);
    if (c->stream) hipStreamDestroy(c->stream);
    for (int i = 0; i < SPLIT_MAX - 1; ++i)
        if (c->twin[i]) enet_range_coder_destroy(c->twin[i]);
    ctx_release(c);
}

/* (as rc_fail, for the device-pointer path) */
static int rc_fail_dev(int err, int line)
{
    if (err && getenv("ENET_RC_DEBUG"))
        fprintf(stderr, "enet_rc: batch failed at rc_host.c:%d: %d (%s)\n", line, err, hipGetErrorString((hipError_t) err));
    return err;
}

static int run_device(rc_ctx *c, int decompress, const uint8_t *in, const uint64_t *in_off,
                      const uint32_t *in_len, size_t n, uint32_t max_len, uint32_t max_out, uint8_t *out,
                      const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len,
                      void *stream)
{
    if (!c) return (int) hipErrorInvalidValue;
    c->last_split = 0;
    if (n == 0) return 0;
    if (n > 0xFFFFFFFFu) return (int) hipErrorInvalidValue;
    if (hipSetDevice(c->device) != hipSuccess) return (int) hipErrorInvalidDevice;
    if (ws_reserve(c, n) != 0) return rc_fail_dev((int) hipErrorOutOfMemory, __LINE__);
    rc_batch_dev b;
    b.in = in; b.in_off = in_off; b.in_len = in_len;
    b.out = out; b.out_off = out_off; b.out_cap = out_cap; b.out_len = out_len;
    b.n = (uint32_t) n;
    b.max_len = max_len;
    b.max_out = max_out;
    /* the lane pool and the encoder's record stream only for batches that run
     * on the lane path (small batches run on the wave kernel without them) */
    if (rc_hip_uses_lanes(decompress, &b, &c->ws)) {
        if (lanes_reserve(c, n, max_len) != 0) return rc_fail_dev((int) hipErrorOutOfMemory, __LINE__);
        if (!decompress && enc2_reserve(c, n, max_len) != 0) return rc_fail_dev((int) hipErrorOutOfMemory, __LINE__);
    }
    /* stream is a hipStream_t; NULL is HIP's default (null) stream */
    return decompress ? rc_hip_decompress(&b, &c->ws, stream) : rc_hip_compress(&b, &c->ws, stream);
}

int enet_rc_compress_batch_device(void *context, const uint8_t *in, const uint64_t *in_off,
                                  const uint32_t *in_len, size_t n, uint32_t max_len,
                                  uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                                  uint32_t *out_len, void *stream)
{
    return run_device((rc_ctx *) context, 0, in, in_off, in_len, n, max_len, 0, out, out_off,
                      out_cap, out_len, stream);
}

int enet_rc_decompress_batch_device(void *context, const uint8_t *in, const uint64_t *in_off,
                                    const uint32_t *in_len, size_t n, uint32_t max_len,
                                    uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                                    uint32_t *out_len, void *stream)
{
    return run_device((rc_ctx *) context, 1, in, in_off, in_len, n, max_len, 0, out, out_off,
                      out_cap, out_len, stream);
}

int enet_rc_decompress_batch_device_bounded(void *context, const uint8_t *in, const uint64_t *in_off,
                                            const uint32_t *in_len, size_t n, uint32_t max_len,
                                            uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                                            uint32_t *out_len, uint32_t max_out, void *stream)
{
    return run_device((rc_ctx *) context, 1, in, in_off, in_len, n, max_len, max_out, out, out_off,
                      out_cap, out_len, stream);
}

/* Host-memory batch: [in | in_off | in_len | out_off | out_cap | out_len | out]
 * packed into one pinned buffer, one H2D, kernels, one D2H of out_len+out. */
/* ---- host-side copies on several threads (the staging memcpy in and the
 * scatter of the packed results out are the largest host costs) */
typedef struct {
    int kind;                       /* 0: memcpy range, 1: scatter packets, 2: flatten gather lists */
    uint8_t *dst;
    const uint8_t *src;
    size_t bytes;
    const uint64_t *out_off, *poff;
    const uint32_t *len;
    size_t lo, hi;
    const ENetBuffer *gbuf;         /* kind 2: packet i = gbuf[gfirst[i] .. gfirst[i + 1]) */
    const size_t *gfirst;
} copy_job;

/* packet i's gather list flattened the way compress.c:260-285 walks it: the
 * first buffer as it is (empty: nothing), every later buffer at least its
 * data[0] (an empty one still yields that byte, the phantom byte) */
static size_t gather_len(const ENetBuffer *b, size_t k)
{
    if (k == 0) return 0;
    size_t total = b[0].dataLength;
    for (size_t j = 1; j < k; ++j) total += b[j].dataLength ? b[j].dataLength : 1;
    return total;
}

static void gather_copy(uint8_t *dst, const ENetBuffer *b, size_t k)
{
    if (k == 0) return;
    size_t pos = b[0].dataLength;
    if (pos) memcpy(dst, b[0].data, pos);
    for (size_t j = 1; j < k; ++j) {
        const size_t l = b[j].dataLength;
        if (l) { memcpy(dst + pos, b[j].data, l); pos += l; }
        else dst[pos++] = *(const uint8_t *) b[j].data;
    }
}

static void *copy_worker(void *p)
{
    copy_job *j = (copy_job *) p;
    if (j->kind == 0) {
        memcpy(j->dst, j->src, j->bytes);
    } else if (j->kind == 2) {
        for (size_t i = j->lo; i < j->hi; ++i)
            gather_copy(j->dst + j->poff[i], j->gbuf + j->gfirst[i], j->gfirst[i + 1] - j->gfirst[i]);
    } else {
        for (size_t i = j->lo; i < j->hi; ++i)
            if (j->len[i]) memcpy(j->dst + j->out_off[i], j->src + j->poff[i], j->len[i]);
    }
    return NULL;
}

#define COPY_THREADS_MAX 16
#define COPY_MIN_BYTES (4u << 20)

/* Threads of the host copies (ENET_RC_COPY_THREADS, 1..16; default 8) */
static int copy_threads(void)
{
    static int k = 0;
    if (k == 0) {
        const char *e = getenv("ENET_RC_COPY_THREADS");
        int v = e ? atoi(e) : 8;
        k = v < 1 ? 1 : (v > COPY_THREADS_MAX ? COPY_THREADS_MAX : v);
    }
    return k;
}
#define COPY_THREADS (copy_threads())

/* A persistent pool of COPY_THREADS - 1 workers (created on first use):
 * creating threads per copy group cost ~1-3 ms per host batch.  One caller
 * at a time uses it; a concurrent caller (several contexts driven from
 * several threads, rc_multi.c) runs its jobs on its own thread. */
static struct {
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    copy_job *jobs;
    int k, next, pending;
} pool = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, PTHREAD_COND_INITIALIZER, NULL, 0, 0, 0};
static pthread_mutex_t pool_user = PTHREAD_MUTEX_INITIALIZER;
static pthread_once_t pool_once = PTHREAD_ONCE_INIT;
static int pool_workers;

static void *pool_worker(void *unused)
{
    (void) unused;
    pthread_mutex_lock(&pool.mu);
    for (;;) {
        while (pool.next >= pool.k) pthread_cond_wait(&pool.go, &pool.mu);
        copy_job *j = &pool.jobs[pool.next++];
        pthread_mutex_unlock(&pool.mu);
        copy_worker(j);
        pthread_mutex_lock(&pool.mu);
        if (--pool.pending == 0) pthread_cond_signal(&pool.done);
    }
    return NULL;
}

static void pool_start(void)
{
    for (int i = 1; i < COPY_THREADS; ++i) {
        pthread_t t;
        if (pthread_create(&t, NULL, pool_worker, NULL) != 0) break;
        pthread_detach(t);
        ++pool_workers;
    }
}

static void par_run(copy_job *jobs, int k)
{
    pthread_once(&pool_once, pool_start);
    if (k <= 1 || pool_workers == 0 || pthread_mutex_trylock(&pool_user) != 0) {
        for (int i = 0; i < k; ++i) copy_worker(&jobs[i]);
        return;
    }
    pthread_mutex_lock(&pool.mu);
    pool.jobs = jobs;
    pool.next = 1;                  /* job 0 runs here */
    pool.pending = k - 1;
    pool.k = k;
    pthread_cond_broadcast(&pool.go);
    pthread_mutex_unlock(&pool.mu);
    copy_worker(&jobs[0]);
    pthread_mutex_lock(&pool.mu);
    while (pool.pending > 0) {
        if (pool.next < pool.k) {   /* help with what is left */
            copy_job *j = &pool.jobs[pool.next++];
            pthread_mutex_unlock(&pool.mu);
            copy_worker(j);
            pthread_mutex_lock(&pool.mu);
            --pool.pending;
            continue;
        }
        pthread_cond_wait(&pool.done, &pool.mu);
    }
    pool.k = pool.next = 0;
    pthread_mutex_unlock(&pool.mu);
    pthread_mutex_unlock(&pool_user);
}

static void par_memcpy(uint8_t *dst, const uint8_t *src, size_t bytes)
{
    int k = bytes >= COPY_MIN_BYTES ? COPY_THREADS : 1;
    copy_job jobs[COPY_THREADS_MAX];
    size_t per = (bytes + k - 1) / k;
    for (int i = 0; i < k; ++i) {
        size_t lo = (size_t) i * per, hi = lo + per < bytes ? lo + per : bytes;
        jobs[i].kind = 0;
        jobs[i].dst = dst + lo; jobs[i].src = src + lo; jobs[i].bytes = hi > lo ? hi - lo : 0;
    }
    par_run(jobs, k);
}

/* packets [lo, hi): out + out_off[i] <- packed + poff[i], len[i] bytes */
static void par_scatter(uint8_t *out, const uint64_t *out_off, const uint8_t *packed, const uint64_t *poff,
                        const uint32_t *len, size_t lo, size_t hi, uint64_t bytes)
{
    int k = bytes >= COPY_MIN_BYTES ? COPY_THREADS : 1;
    copy_job jobs[COPY_THREADS_MAX];
    const size_t n = hi - lo, per = (n + k - 1) / k;
    for (int i = 0; i < k; ++i) {
        jobs[i].kind = 1;
        jobs[i].dst = out; jobs[i].src = packed; jobs[i].out_off = out_off; jobs[i].poff = poff; jobs[i].len = len;
        jobs[i].lo = lo + ((size_t) i * per < n ? (size_t) i * per : n);
        jobs[i].hi = lo + ((size_t) (i + 1) * per < n ? (size_t) (i + 1) * per : n);
    }
    par_run(jobs, k);
}

/* packets [lo, hi) of gather lists flattened into dst + poff[i] */
static void par_gather(uint8_t *dst, const uint64_t *poff, const ENetBuffer *gbuf, const size_t *gfirst,
                       size_t lo, size_t hi, uint64_t bytes)
{
    int k = bytes >= COPY_MIN_BYTES ? COPY_THREADS : 1;
    copy_job jobs[COPY_THREADS_MAX];
    const size_t n = hi - lo, per = (n + k - 1) / k;
    for (int i = 0; i < k; ++i) {
        jobs[i].kind = 2;
        jobs[i].dst = dst; jobs[i].poff = poff; jobs[i].gbuf = gbuf; jobs[i].gfirst = gfirst;
        jobs[i].lo = lo + ((size_t) i * per < n ? (size_t) i * per : n);
        jobs[i].hi = lo + ((size_t) (i + 1) * per < n ? (size_t) (i + 1) * per : n);
    }
    par_run(jobs, k);
}

static int pack_reserve(rc_ctx *c, size_t bytes, size_t blocks)
{
    if (bytes > c->d_pack_cap) {
        hipStreamSynchronize(c->stream);
        if (c->d_pack) hipFree(c->d_pack);
        c->d_pack = NULL; c->d_pack_cap = 0;
        if (hipMalloc((void **) &c->d_pack, bytes) != hipSuccess) return -1;
        c->d_pack_cap = bytes;
    }
    if (blocks + 1 > c->d_bsum_cap) {
        hipStreamSynchronize(c->stream);
        if (c->d_bsum) hipFree(c->d_bsum);
        c->d_bsum = NULL; c->d_bsum_cap = 0;
        if (hipMalloc((void **) &c->d_bsum, (blocks + 1) * 8) != hipSuccess) return -1;
        c->d_bsum_cap = blocks + 1;
    }
    return 0;
}

/* Host pointers: inputs copied (on several threads) into pinned staging, one
 * H2D, the device path, then the results packed back to back on the device
 * (rc_pack.hip) so that only the produced bytes cross PCIe, and scattered to
 * out_off on the host. */
/* Page-locks [p, p + bytes) for direct DMA (hipHostRegister: ~0.35 ms for
 * 80 MB the first time, microseconds after), so that a host batch skips the
 * copy through pinned staging.  1: registered here (host_unpin after the
 * transfers), 2: the caller's memory is page-locked already (its own
 * hipHostMalloc / hipHostRegister, e.g. a long-lived receive buffer) and the
 * whole range lies inside that one allocation or registration: DMA'd
 * directly, left registered; 0: not usable (the call failed, or the range
 * only touches memory some other caller registered, whose registration may
 * end during our transfer) -- the staging path then.  Pageable caller memory
 * is page-locked for the call only with ENET_RC_HOST_REGISTER=1 (below). */
static int host_pin(const void *p, size_t bytes)
{
    static int off = -1;
    if (off < 0) off = getenv("ENET_RC_NO_HOST_PIN") != NULL;
    if (off || bytes < (1u << 20)) return 0;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) == hipSuccess && at.type == hipMemoryTypeHost) {
        /* page-locked by the caller: usable only if one allocation holds the range */
        void *start = NULL;
        size_t size = 0;
        if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t) p) == hipSuccess &&
            hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t) p) == hipSuccess &&
            (uintptr_t) p >= (uintptr_t) start && (uintptr_t) p + bytes <= (uintptr_t) start + size)
            return 2;
        (void) hipGetLastError();
        return 0;
    }
    (void) hipGetLastError();
    /* Pageable caller memory is page-locked for the call only on request
     * (ENET_RC_HOST_REGISTER=1): soak runs interleaving host and device calls
     * met a GPU memory fault in the one-DMA result copy into such a range
     * (about one call in 6000), and none in 24308 calls with it off
     * (profiles/r6/r6z*); the pinned staging serves instead. */
    static int reg = -1;
    if (reg < 0) {
        const char *e = getenv("ENET_RC_HOST_REGISTER");
        reg = e && atoi(e) == 1;
    }
    if (!reg) return 0;
    const uintptr_t a = (uintptr_t) p & ~(uintptr_t) 4095, e = ((uintptr_t) p + bytes + 4095) & ~(uintptr_t) 4095;
    if (hipHostRegister((void *) a, e - a, hipHostRegisterDefault) == hipSuccess) return 1;
    (void) hipGetLastError();
    return 0;
}

static void host_unpin(const void *p, int pinned)
{
    if (pinned == 1) hipHostUnregister((void *) ((uintptr_t) p & ~(uintptr_t) 4095));
}

/* ENET_RC_GPU_COPY=0: host batches move gapped inputs and outputs through
 * pinned staging on the host instead of the GPU's gather / scatter kernels
 * over mapped caller memory */
static int gpu_copy(void)
{
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("ENET_RC_GPU_COPY");
        on = e ? atoi(e) != 0 : 1;
    }
    return on;
}

/* ENET_RC_HOST_PROFILE=1: phase times of run_host on stderr (diagnostic) */
static double now_ms(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

/* A host-to-device copy from page-locked memory as 2D copies (rows of 1 MiB,
 * or 64 KiB below 4 MiB; the tail as two overlapping rows): the runtime runs
 * 2D copies on a DMA engine, a plain one of this size as a copy kernel, which
 * takes CUs from the kernels of the pieces already running (run_host_split).
 * ENET_RC_H2D_DMA=0: plain copies. */
static hipError_t h2d_copy(void *dst, const void *src, size_t bytes, hipStream_t s)
{
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("ENET_RC_H2D_DMA");
        on = e ? atoi(e) != 0 : 1;
    }
    const size_t w = bytes >= (4u << 20) ? (1u << 20) : (1u << 16), rows = bytes / w;
    /* (past 48 MB the runtime ran some 2D copies as a row-by-row copy kernel
     * at a tenth of the link's rate: C4's pieces, profiles/r5s_split) */
    if (!on || rows < 2 || bytes > (48u << 20)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s);
    hipError_t err = hipMemcpy2DAsync(dst, w, src, w, w, rows, hipMemcpyHostToDevice, s);
    const size_t t = bytes - rows * w;
    if (err == hipSuccess && t) {
        /* the last 2 * ceil(t / 2) bytes (re-copying at most one byte of the rows) */
        const size_t h = (t + 1) / 2, at = bytes - 2 * h;
        err = hipMemcpy2DAsync((uint8_t *) dst + at, h, (const uint8_t *) src + at, h, h, 2, hipMemcpyHostToDevice, s);
    }
    return err;
}

static int host_results(rc_ctx *c, int decompress, size_t n, uint8_t *out, const uint64_t *out_off,
                        const uint32_t *out_cap, uint32_t *out_len, int allow_pin, uint64_t out_bytes, size_t total,
                        size_t a_olen, size_t a_out, size_t a_ooff, uint64_t in_bytes, int prof, double *tp);

/* Workgroups of the slot copy of a piece of a split host batch
 * (ENET_RC_PIECE_COPY_WGS, default 64; 0: 8 per CU) */
static uint32_t piece_copy_wgs(void)
{
    static long w = -1;
    if (w < 0) {
        const char *e = getenv("ENET_RC_PIECE_COPY_WGS");
        w = e ? atol(e) : 64;
        if (w < 0) w = 0;
    }
    return (uint32_t) w;
}

/* A large device-to-host copy into page-locked memory; ENET_RC_D2H_DMA=1: as
 * 2D copies (a DMA engine, not a copy kernel on the CUs), like h2d_copy.  Off
 * by default: for the results of a split batch's pieces the DMA engine ran at
 * half the copy kernel's rate and one piece after the other
 * (profiles/r5_split/ab_c2_d2h_dma.txt) */
static hipError_t d2h_copy(void *dst, const void *src, size_t bytes, hipStream_t s)
{
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("ENET_RC_D2H_DMA");
        on = e ? atoi(e) != 0 : 0;
    }
    const size_t w = bytes >= (4u << 20) ? (1u << 20) : (1u << 16), rows = bytes / w;
    if (!on || rows < 2 || bytes > (48u << 20)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s);
    hipError_t err = hipMemcpy2DAsync(dst, w, src, w, w, rows, hipMemcpyDeviceToHost, s);
    const size_t t = bytes - rows * w;
    if (err == hipSuccess && t) {
        const size_t h = (t + 1) / 2, at = bytes - 2 * h;
        err = hipMemcpy2DAsync((uint8_t *) dst + at, h, (const uint8_t *) src + at, h, h, 2, hipMemcpyDeviceToHost, s);
    }
    return err;
}

/* A host batch's failure, with the line that saw it, on stderr when
 * ENET_RC_DEBUG is set (a failed call returns the HIP error either way) */
static int rc_fail(int err, int line)
{
    static int dbg = -1;
    if (dbg < 0) dbg = getenv("ENET_RC_DEBUG") != NULL;
    if (dbg && err) fprintf(stderr, "enet_rc: host batch failed at rc_host.c:%d: %d (%s)\n", line, err,
                            hipGetErrorString((hipError_t) err));
    return err;
}

static int run_host(rc_ctx *c, int decompress, const uint8_t *in, const uint64_t *in_off,
                    const uint32_t *in_len, size_t n, uint8_t *out, const uint64_t *out_off,
                    const uint32_t *out_cap, uint32_t *out_len, int allow_pin,
                    const ENetBuffer *gbuf, const size_t *gfirst)
{
    static int prof = -1;
    if (prof < 0) prof = getenv("ENET_RC_HOST_PROFILE") != NULL;
    double tp[8] = {0};
    if (prof) tp[0] = now_ms();
    if (!c) return (int) hipErrorInvalidValue;
    if (n == 0) return 0;
    /* the input as it goes to the device: packed back to back (a batch whose
     * packets sit in gapped slots -- the compressed side of a round trip --
     * moves only its bytes); a batch that already is back to back is one range */
    /* (gbuf: the input is packet i's gather list gbuf[gfirst[i] .. gfirst[i + 1]),
     * flattened into the staging; in_len = the flattened lengths) */
    uint64_t in_bytes = 0, out_bytes = 0, in_lo = gbuf ? 0 : in_off[0];
    uint32_t max_len = 0, max_cap = 0;
    int packed_in = gbuf == NULL;
    for (size_t i = 0; i < n; ++i) {
        if (!gbuf && in_off[i] != in_lo + in_bytes) packed_in = 0;
        in_bytes += in_len[i];
        uint64_t f = out_off[i] + out_cap[i];
        if (f > out_bytes) out_bytes = f;
        if (in_len[i] > max_len) max_len = in_len[i];
        if (out_cap[i] > max_cap) max_cap = out_cap[i];
    }
    /* An input in gapped slots (the compressed side of a round trip), from a
     * caller buffer page-locked for the call (ENET_RC_GPU_COPY=0: through
     * pinned staging on the host instead):
     *  - slots at a uniform pitch (a caller's array of fixed-size buffers):
     *    one strided DMA (hipMemcpy2DAsync: max_len bytes of each slot, rows
     *    round_up(max_len, 16) apart on the device);
     *  - other gaps: the buffer is mapped and rc_gather16 (rc_pack.hip) reads
     *    the packets over PCIe in whole 16-B granules into the device input
     *    (each packet in granules of its own, at its source alignment), so
     *    the gaps between slots never cross PCIe. */
    if (hipSetDevice(c->device) != hipSuccess) return (int) hipErrorInvalidDevice;
    int zc_pin = 0;
    const uint8_t *zc_dev = NULL;
    uint64_t zc_lo = 0;
    uint64_t pitch = 0, row = 0;
    if (!packed_in && !gbuf && allow_pin && gpu_copy() && in_bytes >= (16u << 20) && n >= 2 &&
        in_off[1] > in_off[0] && in_off[1] - in_off[0] >= max_len) {
        pitch = in_off[1] - in_off[0];
        for (size_t i = 2; i < n && pitch; ++i)
            if (in_off[i] != in_off[0] + i * pitch) pitch = 0;
        if (pitch) {
            zc_lo = in_off[0];
            zc_pin = host_pin(in + zc_lo, in_off[n - 1] + in_len[n - 1] - zc_lo);
            if (zc_pin) row = (max_len + 15) & ~(uint64_t) 15;
            else pitch = 0;
        }
    }
    if (!pitch && !packed_in && !gbuf && allow_pin && gpu_copy() && in_bytes >= (16u << 20)) {
        uint64_t lo = UINT64_MAX, hi = 0;
        for (size_t i = 0; i < n; ++i)
            if (in_len[i]) {
                if (in_off[i] < lo) lo = in_off[i];
                if (in_off[i] + in_len[i] > hi) hi = in_off[i] + in_len[i];
            }
        if (hi > lo) zc_pin = host_pin(in + lo, hi - lo);
        if (zc_pin) {
            void *dp = NULL;
            /* (the mapping keeps the page offset: granule phases match) */
            if (hipHostGetDevicePointer(&dp, (void *) (in + lo), 0) == hipSuccess && dp &&
                (((uintptr_t) dp ^ (uintptr_t) (in + lo)) & 4095) == 0) {
                zc_dev = (const uint8_t *) dp;
                zc_lo = lo;
            } else {
                (void) hipGetLastError();
                host_unpin(in + lo, zc_pin);
                zc_pin = 0;
            }
        }
    }
    /* device input bytes: back to back, or (GPU gather) granule-padded */
    uint64_t dev_in = pitch ? n * row : in_bytes;
    if (zc_dev) {
        dev_in = 0;
        for (size_t i = 0; i < n; ++i)
            if (in_len[i]) dev_in += (((uintptr_t) (in + in_off[i]) & 15) + in_len[i] + 15) & ~(uint64_t) 15;
    }
    size_t a_in = 0;
    size_t a_ioff = (a_in + dev_in + 15) & ~(size_t) 15;
    size_t a_ilen = a_ioff + n * 8;
    size_t a_ooff = (a_ilen + n * 4 + 15) & ~(size_t) 15;
    size_t a_ocap = a_ooff + n * 8;
    size_t a_olen = (a_ocap + n * 4 + 15) & ~(size_t) 15;
    size_t a_out = (a_olen + n * 4 + 15) & ~(size_t) 15;
    size_t total = a_out + out_bytes + 16;
    size_t a_soff = (total + 15) & ~(size_t) 15;        /* source offsets of a device-side gather */
    const size_t blocks = (n + 1023) / 1024;
    if (stage_reserve(c, a_soff + n * 8) != 0 || pack_reserve(c, out_bytes + 16, blocks) != 0) {
        host_unpin(in + zc_lo, zc_pin);
        return rc_fail((int) hipErrorOutOfMemory, __LINE__);
    }
    uint8_t *h = c->h_stage, *d = c->d_stage;
    uint64_t *hio = (uint64_t *) (h + a_ioff);
    if (pitch) {
        for (size_t i = 0; i < n; ++i) hio[i] = i * row;
    } else if (zc_dev) {
        uint64_t acc = 0;
        for (size_t i = 0; i < n; ++i) {
            const uint64_t ph = (uintptr_t) (in + in_off[i]) & 15;
            hio[i] = in_len[i] ? acc + ph : acc;
            if (in_len[i]) acc += (ph + in_len[i] + 15) & ~(uint64_t) 15;
        }
    } else {
        uint64_t acc = 0;
        for (size_t i = 0; i < n; ++i) { hio[i] = acc; acc += in_len[i]; }
    }
    memcpy(h + a_ilen, in_len, n * 4);
    memcpy(h + a_ooff, out_off, n * 8);
    memcpy(h + a_ocap, out_cap, n * 4);
    if (c->sync_wait) {             /* a later piece: its DMA after the previous piece's */
        struct h2d_sync *y = c->sync_wait;
        pthread_mutex_lock(&y->m);
        while (!y->ready) pthread_cond_wait(&y->cv, &y->m);
        const int r = y->ready;
        pthread_mutex_unlock(&y->m);
        if (r > 0) (void) hipStreamWaitEvent(c->stream, y->ev, 0);
    }
    hipError_t err = h2d_copy(d + a_ioff, h + a_ioff, a_olen - a_ioff, c->stream);
    if (err != hipSuccess) { host_unpin(in + zc_lo, zc_pin); return rc_fail((int) err, __LINE__); }
    /* the payload: straight from the caller's memory when it is one range and
     * can be page-locked; else in four packet groups through pinned staging,
     * the staging copy of group k+1 overlapping the DMA of group k */
    const int pin_in = packed_in && allow_pin ? host_pin(in + in_lo, in_bytes) : 0;
    if (pin_in) err = h2d_copy(d + a_in, in + in_lo, in_bytes, c->stream);
    if (pitch) {
        err = hipMemcpy2DAsync(d + a_in, row, in + zc_lo, pitch, max_len, n - 1, hipMemcpyHostToDevice, c->stream);
        if (err == hipSuccess && in_len[n - 1])
            err = hipMemcpyAsync(d + a_in + (n - 1) * row, in + in_off[n - 1], in_len[n - 1], hipMemcpyHostToDevice,
                                 c->stream);
    }
    if (zc_dev) {
        uint64_t *hso = (uint64_t *) (h + a_soff);
        for (size_t i = 0; i < n; ++i) hso[i] = in_len[i] ? in_off[i] - zc_lo : 0;
        err = hipMemcpyAsync(d + a_soff, h + a_soff, n * 8, hipMemcpyHostToDevice, c->stream);
        if (err == hipSuccess)
            err = (hipError_t) rc_hip_gather16(zc_dev, (const uint64_t *) (d + a_soff), d + a_in,
                                               (const uint64_t *) (d + a_ioff), (const uint32_t *) (d + a_ilen),
                                               (uint32_t) n, (void *) c->stream);
    }
    if (err != hipSuccess) {
        if (pin_in || zc_pin) hipStreamSynchronize(c->stream);
        host_unpin(in + in_lo, pin_in);
        host_unpin(in + zc_lo, zc_pin);
        return rc_fail((int) err, __LINE__);
    }
    c->last_paths = zc_dev ? 4u : pitch ? 3u : pin_in ? 2u : 1u;
    const int ig = pin_in || zc_pin ? 0 : in_bytes >= (16u << 20) ? 4 : 1;
    for (int g = 0; g < ig; ++g) {
        const size_t lo = n * (size_t) g / (size_t) ig, hi = n * (size_t) (g + 1) / (size_t) ig;
        if (hi <= lo) continue;
        const uint64_t b0 = hio[lo], b1 = hio[hi - 1] + in_len[hi - 1];
        if (gbuf) par_gather(h + a_in, hio, gbuf, gfirst, lo, hi, b1 - b0);
        else if (packed_in) par_memcpy(h + a_in + b0, in + in_lo + b0, b1 - b0);
        else par_scatter(h + a_in, hio, in, in_off, in_len, lo, hi, b1 - b0);
        if (b1 > b0) err = hipMemcpyAsync(d + a_in + b0, h + a_in + b0, b1 - b0, hipMemcpyHostToDevice, c->stream);
        if (err != hipSuccess) return rc_fail((int) err, __LINE__);
    }
    if (c->sync_sig) {              /* its input DMA is enqueued: the next piece's may follow */
        h2d_sync_set(c->sync_sig, hipEventRecord(c->sync_sig->ev, c->stream) == hipSuccess ? 1 : -1);
    }
    if (prof) { tp[1] = now_ms(); hipStreamSynchronize(c->stream); tp[2] = now_ms(); }
    int rc = run_device(c, decompress, d + a_in, (const uint64_t *) (d + a_ioff),
                        (const uint32_t *) (d + a_ilen), n, max_len, max_cap, d + a_out,
                        (const uint64_t *) (d + a_ooff), (const uint32_t *) (d + a_ocap),
                        (uint32_t *) (d + a_olen), (void *) c->stream);
    if (rc == 0) rc = host_results(c, decompress, n, out, out_off, out_cap, out_len, allow_pin, out_bytes, total,
                                   a_olen, a_out, a_ooff, in_bytes, prof, tp);
    if (pin_in == 1 || zc_pin == 1) {   /* (registered for this call: the input DMA / gather is done by now) */
        hipStreamSynchronize(c->stream);
        host_unpin(in + in_lo, pin_in);
        host_unpin(in + zc_lo, zc_pin);
    }
    return rc ? rc_fail(rc, __LINE__) : 0;
}

/* The results of run_host's kernels into the caller's slots; returns after
 * the stream has drained (on success). */
static int host_results(rc_ctx *c, int decompress, size_t n, uint8_t *out, const uint64_t *out_off,
                        const uint32_t *out_cap, uint32_t *out_len, int allow_pin, uint64_t out_bytes, size_t total,
                        size_t a_olen, size_t a_out, size_t a_ooff, uint64_t in_bytes, int prof, double *tp)
{
    uint8_t *h = c->h_stage, *d = c->d_stage;
    const size_t blocks = (n + 1023) / 1024;
    hipError_t err = hipSuccess;
    int rc = 0;
    if (prof) { hipStreamSynchronize(c->stream); tp[3] = now_ms(); }
    if (out_bytes <= (1u << 20)) {
        /* small batches (the per-datagram drop-in calls): one D2H of the slots,
         * fewer launches and syncs than packing */
        err = hipMemcpyAsync(h + a_olen, d + a_olen, total - 16 - a_olen, hipMemcpyDeviceToHost, c->stream);
        if (err == hipSuccess) err = hipMemcpyAsync(&c->last_exact, c->ws.counters, 4, hipMemcpyDeviceToHost, c->stream);
        if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
        if (err != hipSuccess) return rc_fail((int) err, __LINE__);
        memcpy(out_len, h + a_olen, n * 4);
        for (size_t i = 0; i < n; ++i)
            if (out_len[i]) memcpy(out + out_off[i], h + a_out + out_off[i], out_len[i]);
        c->last_paths |= 1u << 4;
        return 0;
    }
    /* a decompress batch whose slots are back to back (out_cap = the packet
     * lengths) and every one of them filled: the whole span in one DMA
     * straight behind the kernels.  The lengths are read first: a slot a
     * packet did not fill (a corrupt stream, an output that does not fit)
     * keeps the caller's bytes past its out_len, as compress.c writes only
     * what it decodes -- the span's DMA would put the staging memory's old
     * contents there (an earlier batch's payload) -- so such a batch takes
     * the slot copy below. */
    /* (a piece of a split batch of packets of >= 512 B on average: its slot
     * copy below with few workgroups, leaving the other pieces' kernels
     * their CUs' issue slots; the copy's wavefronts each move a packet, so
     * smaller packets need them all to keep PCIe busy) */
    const uint32_t wgs = (c->sync_sig || c->sync_wait) && in_bytes >= 512 * (uint64_t) n ? piece_copy_wgs() : 0u;
    static int contig_dma = -1;       /* ENET_RC_CONTIG_DMA=0: back-to-back slots take the slot copy too */
    if (contig_dma < 0) {
        const char *e = getenv("ENET_RC_CONTIG_DMA");
        contig_dma = e ? atoi(e) != 0 : 1;
    }
    int contig_out = decompress && contig_dma;
    for (size_t i = 1; i < n && contig_out; ++i) contig_out = out_off[i] == out_off[i - 1] + out_cap[i - 1];
    if (contig_out) {
        /* (the lengths, and the kernels done: registering the caller's range
         * while they run made the copy 1.2 ms slower; a piece of a split
         * batch finds its range registered already) */
        err = hipMemcpyAsync(h + a_olen, d + a_olen, n * 4, hipMemcpyDeviceToHost, c->stream);
        if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
        if (err != hipSuccess) return rc_fail((int) err, __LINE__);
        const uint32_t *ol = (const uint32_t *) (h + a_olen);
        for (size_t i = 0; i < n && contig_out; ++i) contig_out = ol[i] == out_cap[i];
    }
    if (contig_out) {
        const uint64_t span = out_off[n - 1] + out_cap[n - 1] - out_off[0];
        const int pin_out = allow_pin ? host_pin(out + out_off[0], span) : 0;
        if (pin_out) {
            err = d2h_copy(out + out_off[0], d + a_out + out_off[0], span, c->stream);
            if (err == hipSuccess)
                err = hipMemcpyAsync(&c->last_exact, c->ws.counters, 4, hipMemcpyDeviceToHost, c->stream);
            const hipError_t e2 = hipStreamSynchronize(c->stream);
            host_unpin(out + out_off[0], pin_out);
            if (err == hipSuccess) err = e2;
            if (err != hipSuccess) return rc_fail((int) err, __LINE__);
            memcpy(out_len, h + a_olen, n * 4);
            if (prof) {
                tp[5] = now_ms();
                fprintf(stderr, "enet_rc host %s n=%zu in=%.1f MB out=%.1f MB (direct): stage+H2D enqueue %.3f, "
                        "H2D drain %.3f, kernels %.3f, D2H %.3f, total %.3f ms\n", decompress ? "dec" : "enc", n,
                        in_bytes / 1e6, span / 1e6, tp[1] - tp[0], tp[2] - tp[1], tp[3] - tp[2], tp[5] - tp[3],
                        tp[5] - tp[0]);
            }
            c->last_paths |= 2u << 4;
            return 0;
        }
    }
    /* the results straight from their device slots into the caller's slots
     * by the GPU (rc_slot_copy writing the mapped, page-locked caller buffer
     * over PCIe): no packing pass and no host scatter.  ENET_RC_GPU_COPY=0:
     * packed on the device, D2H and scattered on the host. */
    if (allow_pin && gpu_copy() && out_bytes >= (16u << 20)) {
        uint64_t lo = UINT64_MAX, hi = 0;
        for (size_t i = 0; i < n; ++i) {
            if (out_off[i] < lo) lo = out_off[i];
            if (out_off[i] + out_cap[i] > hi) hi = out_off[i] + out_cap[i];
        }
        const int op = hi > lo ? host_pin(out + lo, hi - lo) : 0;
        void *dp = NULL;
        if (op && hipHostGetDevicePointer(&dp, (void *) (out + lo), 0) == hipSuccess && dp) {
            err = (hipError_t) rc_hip_slot_copy(d + a_out, (const uint64_t *) (d + a_ooff),
                                                (const uint32_t *) (d + a_olen), (uint32_t) n, (uint8_t *) dp - lo,
                                                wgs, (void *) c->stream);
            if (err == hipSuccess) err = hipMemcpyAsync(h + a_olen, d + a_olen, n * 4, hipMemcpyDeviceToHost, c->stream);
            if (err == hipSuccess)
                err = hipMemcpyAsync(&c->last_exact, c->ws.counters, 4, hipMemcpyDeviceToHost, c->stream);
            const hipError_t e2 = hipStreamSynchronize(c->stream);
            host_unpin(out + lo, op);
            if (err == hipSuccess) err = e2;
            if (err != hipSuccess) return rc_fail((int) err, __LINE__);
            memcpy(out_len, h + a_olen, n * 4);
            if (prof) {
                tp[5] = now_ms();
                fprintf(stderr, "enet_rc host %s n=%zu in=%.1f MB (GPU slot copy): stage+H2D enqueue %.3f, "
                        "H2D drain %.3f, kernels %.3f, slot copy %.3f, total %.3f ms\n", decompress ? "dec" : "enc",
                        n, in_bytes / 1e6, tp[1] - tp[0], tp[2] - tp[1], tp[3] - tp[2], tp[5] - tp[3], tp[5] - tp[0]);
            }
            c->last_paths |= 3u << 4;
            return 0;
        }
        (void) hipGetLastError();
        host_unpin(out + lo, op);
    }
    rc = rc_hip_pack(d + a_out, (const uint64_t *) (d + a_ooff), (const uint32_t *) (d + a_olen), (uint32_t) n,
                     c->d_bsum, c->d_pack, (void *) c->stream);
    if (rc != 0) return rc_fail(rc, __LINE__);
    uint64_t packed = 0;
    err = hipMemcpyAsync(h + a_olen, d + a_olen, n * 4, hipMemcpyDeviceToHost, c->stream);
    if (err == hipSuccess) err = hipMemcpyAsync(&c->last_exact, c->ws.counters, 4, hipMemcpyDeviceToHost, c->stream);
    if (err == hipSuccess) err = hipMemcpyAsync(&packed, c->d_bsum + blocks, 8, hipMemcpyDeviceToHost, c->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
    if (err != hipSuccess) return rc_fail((int) err, __LINE__);
    if (prof) tp[4] = now_ms();
    if (packed > out_bytes) return rc_fail((int) hipErrorUnknown, __LINE__);
    memcpy(out_len, h + a_olen, n * 4);
    uint64_t *poff = (uint64_t *) malloc((n + 1) * sizeof(uint64_t));
    if (!poff) return rc_fail((int) hipErrorOutOfMemory, __LINE__);
    uint64_t acc = 0;
    for (size_t i = 0; i < n; ++i) { poff[i] = acc; acc += out_len[i]; }
    poff[n] = acc;
    /* D2H in packet groups; the scatter of group g overlaps the DMA of g+1 */
    const int groups = packed >= (16u << 20) ? 4 : 1;
    hipEvent_t ev[4];
    int nev = 0;
    size_t first[5];
    for (int g = 0; g <= groups; ++g) first[g] = n * (size_t) g / (size_t) groups;
    for (int g = 0; g < groups && err == hipSuccess; ++g) {
        const uint64_t lo = poff[first[g]], hi = poff[first[g + 1]];
        if (hi > lo) err = hipMemcpyAsync(h + a_out + lo, c->d_pack + lo, hi - lo, hipMemcpyDeviceToHost, c->stream);
        if (err == hipSuccess) err = hipEventCreateWithFlags(&ev[g], hipEventDisableTiming);
        if (err == hipSuccess) { nev = g + 1; err = hipEventRecord(ev[g], c->stream); }
    }
    for (int g = 0; g < nev && err == hipSuccess; ++g) {
        err = hipEventSynchronize(ev[g]);
        if (err == hipSuccess)
            par_scatter(out, out_off, h + a_out, poff, out_len, first[g], first[g + 1],
                        poff[first[g + 1]] - poff[first[g]]);
    }
    for (int g = 0; g < nev; ++g) hipEventDestroy(ev[g]);
    free(poff);
    if (prof) {
        tp[5] = now_ms();
        fprintf(stderr, "enet_rc host %s n=%zu in=%.1f MB out=%.1f MB: stage+H2D enqueue %.3f, H2D drain %.3f, "
                "kernels %.3f, pack+lens %.3f, D2H+scatter %.3f, total %.3f ms\n", decompress ? "dec" : "enc", n,
                in_bytes / 1e6, packed / 1e6, tp[1] - tp[0], tp[2] - tp[1], tp[3] - tp[2], tp[4] - tp[3],
                tp[5] - tp[4], tp[5] - tp[0]);
    }
    c->last_paths |= 4u << 4;
    return err == hipSuccess ? 0 : rc_fail((int) err, __LINE__);
}

/* ---- a large host batch in pieces, on this context and further contexts
 * on the same device (each with its own stream and workspace): each piece's
 * input DMA follows the previous piece's, so its kernels start while the
 * later pieces' inputs still cross PCIe and run beside the earlier pieces'
 * on the other CUs, and the earlier pieces' results cross PCIe while the later
 * ones compute.  The lane kernels take as long for part of a batch as for the
 * whole (a packet per lane), so the pieces run side by side,
 * never one after the other.  Pieces hold equal input bytes.  The caller's
 * input and output ranges are page-locked once here for all pieces (adjacent
 * pieces share boundary pages: see host_pin).  ENET_RC_HOST_SPLIT=k: k pieces
 * (2..SPLIT_MAX; 0 or 1: off). */
typedef struct {
    rc_ctx *c;
    int decompress;
    const uint8_t *in; const uint64_t *in_off; const uint32_t *in_len; size_t n;
    uint8_t *out; const uint64_t *out_off; const uint32_t *out_cap; uint32_t *out_len;
    int rc;
} piece_job;

static void *piece_worker(void *p)
{
    piece_job *j = (piece_job *) p;
    j->rc = run_host(j->c, j->decompress, j->in, j->in_off, j->in_len, j->n, j->out, j->out_off, j->out_cap,
                     j->out_len, 1, NULL, NULL);
    /* (a failed piece may have left DMAs of the caller's page-locked ranges in
     * flight: drained before run_host_split unregisters them) */
    if (j->rc != 0) hipStreamSynchronize(j->c->stream);
    /* (a piece that ended before its input DMA: the next one waits for nothing) */
    if (j->c->sync_sig) h2d_sync_set(j->c->sync_sig, -1);
    return NULL;
}

#define SPLIT_MIN_PACKETS 8192u         /* per piece */
#define SPLIT_MIN_BYTES (8ull << 20)    /* per piece */
static int run_host_split(rc_ctx *c, int decompress, const uint8_t *in, const uint64_t *in_off,
                          const uint32_t *in_len, size_t n, uint8_t *out, const uint64_t *out_off,
                          const uint32_t *out_cap, uint32_t *out_len)
{
    if (!c) return (int) hipErrorInvalidValue;
    c->last_split = 0;
    int k = c->split_k;
    uint64_t bytes = 0, ilo = UINT64_MAX, ihi = 0, olo = UINT64_MAX, ohi = 0;
    if (k > 1 && n >= 32768 && c->ws.kernel != RC_KERNEL_WAVE) {
        for (size_t i = 0; i < n; ++i) {
            bytes += in_len[i];
            if (in_len[i]) {
                if (in_off[i] < ilo) ilo = in_off[i];
                if (in_off[i] + in_len[i] > ihi) ihi = in_off[i] + in_len[i];
            }
            if (out_off[i] < olo) olo = out_off[i];
            if (out_off[i] + out_cap[i] > ohi) ohi = out_off[i] + out_cap[i];
        }
    }
    if (n < 32768 || bytes < (32ull << 20)) k = 1;   /* (smaller batches: one piece) */
    while (k > 1 && (n < (size_t) k * SPLIT_MIN_PACKETS || bytes < (uint64_t) k * SPLIT_MIN_BYTES)) --k;
    if (k < 2 || ihi <= ilo || ohi <= olo)
        return run_host(c, decompress, in, in_off, in_len, n, out, out_off, out_cap, out_len, 1, NULL, NULL);
    if (hipSetDevice(c->device) != hipSuccess) return (int) hipErrorInvalidDevice;
    for (int i = 0; i < k - 1; ++i)
        if (!c->twin[i]) {
            c->twin[i] = enet_range_coder_create();
            if (c->twin[i]) ctx_copy_config((rc_ctx *) c->twin[i], c);
            else { k = i + 1; break; }
        }
    const int pi = k > 1 ? host_pin(in + ilo, ihi - ilo) : 0;
    const int po = host_pin(out + olo, ohi - olo);
    struct h2d_sync y[SPLIT_MAX - 1];
    int ny = 0;
    /* (pieces of pageable caller memory, pi = po = 0, take each piece's pinned
     * staging: their host copies then run on the pieces' threads side by side) */
    for (; ny < k - 1; ++ny) {
        if (hipEventCreateWithFlags(&y[ny].ev, hipEventDisableTiming) != hipSuccess) break;
        pthread_mutex_init(&y[ny].m, NULL);
        pthread_cond_init(&y[ny].cv, NULL);
        y[ny].ready = 0;
    }
    if (ny < k - 1) {               /* (no further context or event: one piece) */
        for (int i = 0; i < ny; ++i) {
            hipEventDestroy(y[i].ev);
            pthread_cond_destroy(&y[i].cv);
            pthread_mutex_destroy(&y[i].m);
        }
        host_unpin(out + olo, po);
        host_unpin(in + ilo, pi);
        return run_host(c, decompress, in, in_off, in_len, n, out, out_off, out_cap, out_len, 1, NULL, NULL);
    }
    /* piece boundaries at equal shares of the input bytes */
    size_t first[SPLIT_MAX + 1];
    first[0] = 0;
    first[k] = n;
    {
        uint64_t acc = 0;
        size_t i = 0;
        for (int p = 1; p < k; ++p) {
            const uint64_t goal = bytes * (uint64_t) p / (uint64_t) k;
            while (i < n && acc + in_len[i] <= goal) acc += in_len[i++];
            /* whole 2048-packet groups: a piece's decoder and code-pass
               workgroups (256 packets each) then spread evenly over the 8
               XCDs, and the pieces' workgroups together fill each XCD's CUs
               once (a piece one workgroup over lands it on a busy CU and
               doubles that piece's time) */
            size_t f = (i + 1024) & ~(size_t) 2047;
            if (f <= first[p - 1]) f = first[p - 1] + 2048;
            first[p] = f < n ? f : n;
        }
    }
    piece_job job[SPLIT_MAX];
    pthread_t th[SPLIT_MAX];
    int threaded[SPLIT_MAX] = {0};
    uint64_t *rebased[SPLIT_MAX] = {NULL};
    for (int p = 0; p < k; ++p) {
        rc_ctx *x = p ? (rc_ctx *) c->twin[p - 1] : c;
        const size_t a = first[p], m = first[p + 1] - a;
        /* the piece's output offsets from its own first slot, so that its
         * staging (sized from the largest out_off + out_cap) covers its slots
         * only, not the output from byte 0 */
        uint64_t lo = UINT64_MAX;
        for (size_t i = a; i < a + m; ++i) if (out_off[i] < lo) lo = out_off[i];
        rebased[p] = m ? (uint64_t *) malloc(m * sizeof(uint64_t)) : NULL;
        if (rebased[p]) for (size_t i = 0; i < m; ++i) rebased[p][i] = out_off[a + i] - lo;
        piece_job j = {x, decompress, in, in_off + a, in_len + a, m, rebased[p] ? out + lo : out,
                       rebased[p] ? rebased[p] : out_off + a, out_cap + a, out_len + a, 0};
        job[p] = j;
        x->sync_wait = p ? &y[p - 1] : NULL;
        x->sync_sig = p < k - 1 ? &y[p] : NULL;
    }
    for (int p = 1; p < k; ++p) threaded[p] = pthread_create(&th[p], NULL, piece_worker, &job[p]) == 0;
    piece_worker(&job[0]);
    for (int p = 1; p < k; ++p) {
        if (threaded[p]) pthread_join(th[p], NULL);
        else piece_worker(&job[p]);     /* (its predecessors have all signalled by now) */
    }
    int rc = 0;
    uint32_t exact = 0;
    for (int p = 0; p < k; ++p) {
        rc_ctx *x = job[p].c;
        x->sync_wait = x->sync_sig = NULL;
        if (!rc) rc = job[p].rc;
        exact += x->last_exact;
    }
    c->last_exact = exact;
    for (int p = 0; p < k; ++p) free(rebased[p]);
    for (int i = 0; i < k - 1; ++i) {
        hipEventDestroy(y[i].ev);
        pthread_cond_destroy(&y[i].cv);
        pthread_mutex_destroy(&y[i].m);
    }
    host_unpin(out + olo, po);
    host_unpin(in + ilo, pi);
    c->last_split = k;
    return rc;
}

int enet_rc_compress_batch_host(void *context, const uint8_t *in, const uint64_t *in_off,
                                const uint32_t *in_len, size_t n, uint8_t *out,
                                const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len)
{
    return run_host_split((rc_ctx *) context, 0, in, in_off, in_len, n, out, out_off, out_cap, out_len);
}

int enet_rc_decompress_batch_host(void *context, const uint8_t *in, const uint64_t *in_off,
                                  const uint32_t *in_len, size_t n, uint8_t *out,
                                  const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len)
{
    return run_host_split((rc_ctx *) context, 1, in, in_off, in_len, n, out, out_off, out_cap, out_len);
}

/* compress.c:246-342 over a batch of gather lists: packet i is
 * buffers[first[i] .. first[i + 1]), consumed as enet_range_coder_compress
 * consumes its inBuffers (protocol.c:1688-1695 passes &buffers[1],
 * bufferCount - 1); the lists are flattened straight into the pinned
 * staging on the copy threads. */
int enet_rc_compress_gather_batch_host(void *context, const ENetBuffer *buffers, const size_t *first, size_t n,
                                       uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                                       uint32_t *out_len)
{
    rc_ctx *c = (rc_ctx *) context;
    if (!c || (n && (!buffers || !first))) return (int) hipErrorInvalidValue;
    if (n == 0) return 0;
    uint32_t *len = (uint32_t *) malloc(n * sizeof(uint32_t));
    if (!len) return (int) hipErrorOutOfMemory;
    for (size_t i = 0; i < n; ++i) {
        /* the lists must not run backwards: the copy threads flatten
           first[i + 1] - first[i] buffers of packet i */
        if (first[i + 1] < first[i]) { free(len); return (int) hipErrorInvalidValue; }
        const size_t l = gather_len(buffers + first[i], first[i + 1] - first[i]);
        if (l > 0xFFFFFFFFu) { free(len); return (int) hipErrorInvalidValue; }
        len[i] = (uint32_t) l;
    }
    const int rc = run_host(c, 0, NULL, NULL, len, n, out, out_off, out_cap, out_len, 0, buffers, first);
    free(len);
    return rc;
}

/* --------------------------------------------------- datagram framing (§8f) */

#define DG_MTU 4096u                /* ENET_PROTOCOL_MAXIMUM_MTU (protocol.h:13) */

static int dgram_reserve(rc_ctx *c, size_t n, int scratch)
{
    if (n > c->dg_cap) {
        size_t cap = c->dg_cap ? c->dg_cap : 1024;
        while (cap < n) cap *= 2;
        hipDeviceSynchronize();             /* (the device calls run on the caller's stream) */
        if (c->dg_arrays) hipFree(c->dg_arrays);
        c->dg_arrays = NULL; c->dg_cap = 0;
        if (hipMalloc((void **) &c->dg_arrays, cap * (3 * 8 + 6 * 4)) != hipSuccess) return -1;
        c->dg_cap = cap;
    }
    if (scratch && n * DG_MTU > c->dg_scratch_cap) {
        hipDeviceSynchronize();
        if (c->dg_scratch) hipFree(c->dg_scratch);
        c->dg_scratch = NULL; c->dg_scratch_cap = 0;
        if (hipMalloc((void **) &c->dg_scratch, n * DG_MTU) != hipSuccess) return -1;
        c->dg_scratch_cap = n * DG_MTU;
    }
    return 0;
}

/* protocol.c:1686-1718 (send) or :1022-1091 (receive) for a batch of whole
 * datagrams: frame, code the command ranges with the lane kernels, checksum. */
static int run_dgram(rc_ctx *c, int decode, const uint8_t *in, const uint64_t *in_off,
                     const uint32_t *in_len, size_t n, int checksum, const uint32_t *seed,
                     uint8_t *out, const uint64_t *out_off, uint32_t *out_len, void *stream)
{
    if (!c || n > 0xFFFFFFFFu || (checksum && !seed)) return (int) hipErrorInvalidValue;
    if (n == 0) return 0;
    if (hipSetDevice(c->device) != hipSuccess) return (int) hipErrorInvalidDevice;
    if (dgram_reserve(c, n, checksum && !decode) != 0) return (int) hipErrorOutOfMemory;
    uint8_t *a = c->dg_arrays;
    const size_t cap = c->dg_cap;
    rc_dgram_dev g;
    g.in = in; g.in_off = in_off; g.in_len = in_len;
    g.out = out; g.out_off = out_off; g.out_len = out_len;
    g.seed = seed;
    g.p_off = (uint64_t *) a;
    g.q_off = (uint64_t *) (a + cap * 8);
    g.s_off = (uint64_t *) (a + cap * 16);
    g.p_len = (uint32_t *) (a + cap * 24);
    g.q_cap = (uint32_t *) (a + cap * 28);
    g.c_len = (uint32_t *) (a + cap * 32);
    g.s_len = (uint32_t *) (a + cap * 36);
    g.crc = (uint32_t *) (a + cap * 40);
    g.want = (uint32_t *) (a + cap * 44);
    g.scratch = c->dg_scratch;
    g.n = (uint32_t) n;
    g.checksum = checksum ? 1u : 0u;
    int rc = rc_hip_dgram_launch(decode ? RC_DGRAM_DEC_PREP : RC_DGRAM_ENC_PREP, &g, stream);
    if (rc) return rc;
    rc = run_device(c, decode, in, g.p_off, g.p_len, n, DG_MTU, 0, out, g.q_off, g.q_cap, g.c_len, stream);
    if (rc) return rc;
    rc = rc_hip_dgram_launch(decode ? RC_DGRAM_DEC_STAGE : RC_DGRAM_ENC_STAGE, &g, stream);
    if (rc) return rc;
    if (checksum) {
        rc = decode ? rc_hip_crc32(out, out_off, g.s_len, (uint32_t) n, g.crc, c->crc_tables, stream)
                    : rc_hip_crc32(g.scratch, g.s_off, g.s_len, (uint32_t) n, g.crc, c->crc_tables, stream);
        if (rc) return rc;
        rc = rc_hip_dgram_launch(decode ? RC_DGRAM_DEC_FINISH : RC_DGRAM_ENC_FINISH, &g, stream);
    }
    return rc;
}

int enet_rc_datagram_encode_batch_device(void *context, const uint8_t *in, const uint64_t *in_off,
                                         const uint32_t *in_len, size_t n, int checksum,
                                         const uint32_t *seed, uint8_t *out, const uint64_t *out_off,
                                         uint32_t *out_len, void *stream)
{
    return run_dgram((rc_ctx *) context, 0, in, in_off, in_len, n, checksum, seed, out, out_off,
                     out_len, stream);
}

int enet_rc_datagram_decode_batch_device(void *context, const uint8_t *in, const uint64_t *in_off,
                                         const uint32_t *in_len, size_t n, int checksum,
                                         const uint32_t *seed, uint8_t *out, const uint64_t *out_off,
                                         uint32_t *out_len, void *stream)
{
    return run_dgram((rc_ctx *) context, 1, in, in_off, in_len, n, checksum, seed, out, out_off,
                     out_len, stream);
}

/* Host-pointer variants: one pinned staging area, H2D, the device path, D2H
 * of the lengths and of each slot's used bytes only. */
static int run_dgram_host(rc_ctx *c, int decode, const uint8_t *in, const uint64_t *in_off,
                          const uint32_t *in_len, size_t n, int checksum, const uint32_t *seed,
                          uint8_t *out, const uint64_t *out_off, uint32_t *out_len)
{
    if (!c || n > 0xFFFFFFFFu || (checksum && !seed)) return (int) hipErrorInvalidValue;
    if (n == 0) return 0;
    uint64_t in_bytes = 0, out_bytes = 0;
    for (size_t i = 0; i < n; ++i) {
        uint64_t e = in_off[i] + in_len[i];
        if (e > in_bytes) in_bytes = e;
        uint64_t f = out_off[i] + (decode ? DG_MTU : in_len[i]);
        if (f > out_bytes) out_bytes = f;
    }
    size_t a_ioff = (in_bytes + 15) & ~(size_t) 15;
    size_t a_ilen = a_ioff + n * 8;
    size_t a_seed = (a_ilen + n * 4 + 15) & ~(size_t) 15;
    size_t a_ooff = (a_seed + n * 4 + 15) & ~(size_t) 15;
    size_t a_olen = (a_ooff + n * 8 + 15) & ~(size_t) 15;
    size_t a_out = (a_olen + n * 4 + 15) & ~(size_t) 15;
    size_t total = a_out + out_bytes + 16;
    size_t a_soff = (total + 15) & ~(size_t) 15;        /* source offsets of a device-side gather */
    if (hipSetDevice(c->device) != hipSuccess) return (int) hipErrorInvalidDevice;
    if (stage_reserve(c, a_soff + n * 8) != 0) return (int) hipErrorOutOfMemory;
    uint8_t *h = c->h_stage, *d = c->d_stage;
    memcpy(h, in, in_bytes);
    memcpy(h + a_ioff, in_off, n * 8);
    memcpy(h + a_ilen, in_len, n * 4);
    if (checksum) memcpy(h + a_seed, seed, n * 4);
    memcpy(h + a_ooff, out_off, n * 8);
    hipError_t err = hipMemcpyAsync(d, h, a_olen, hipMemcpyHostToDevice, c->stream);
    if (err != hipSuccess) return (int) err;
    int rc = run_dgram(c, decode, d, (const uint64_t *) (d + a_ioff), (const uint32_t *) (d + a_ilen), n,
                       checksum, (const uint32_t *) (d + a_seed), d + a_out, (const uint64_t *) (d + a_ooff),
                       (uint32_t *) (d + a_olen), (void *) c->stream);
    if (rc) return rc;
    err = hipMemcpyAsync(h + a_olen, d + a_olen, total - 16 - a_olen, hipMemcpyDeviceToHost, c->stream);
    if (err != hipSuccess) return (int) err;
    err = hipStreamSynchronize(c->stream);
    if (err != hipSuccess) return (int) err;
    memcpy(out_len, h + a_olen, n * 4);
    for (size_t i = 0; i < n; ++i)
        if (out_len[i]) memcpy(out + out_off[i], h + a_out + out_off[i], out_len[i]);
    return 0;
}

int enet_rc_datagram_encode_batch_host(void *context, const uint8_t *in, const uint64_t *in_off,
                                       const uint32_t *in_len, size_t n, int checksum, const uint32_t *seed,
                                       uint8_t *out, const uint64_t *out_off, uint32_t *out_len)
{
    return run_dgram_host((rc_ctx *) context, 0, in, in_off, in_len, n, checksum, seed, out, out_off, out_len);
}

int enet_rc_datagram_decode_batch_host(void *context, const uint8_t *in, const uint64_t *in_off,
                                       const uint32_t *in_len, size_t n, int checksum, const uint32_t *seed,
                                       uint8_t *out, const uint64_t *out_off, uint32_t *out_len)
{
    return run_dgram_host((rc_ctx *) context, 1, in, in_off, in_len, n, checksum, seed, out, out_off, out_len);
}

/* ------------------------------------------------------------------ CRC-32 */

int enet_rc_crc32_batch_device(void *context, const uint8_t *in, const uint64_t *in_off,
                               const uint32_t *in_len, size_t n, uint32_t *crc_out, void *stream)
{
    rc_ctx *c = (rc_ctx *) context;
    if (!c || n > 0xFFFFFFFFu) return (int) hipErrorInvalidValue;
    if (n == 0) return 0;
    if (hipSetDevice(c->device) != hipSuccess) return (int) hipErrorInvalidDevice;
    return rc_hip_crc32(in, in_off, in_len, (uint32_t) n, crc_out, c->crc_tables, stream);
}

int enet_rc_crc32_batch_host(void *context, const uint8_t *in, const uint64_t *in_off,
                             const uint32_t *in_len, size_t n, uint32_t *crc_out)
{
    rc_ctx *c = (rc_ctx *) context;
    if (!c || n > 0xFFFFFFFFu) return (int) hipErrorInvalidValue;
    if (n == 0) return 0;
    uint64_t in_bytes = 0;
    for (size_t i = 0; i < n; ++i) {
        uint64_t e = in_off[i] + in_len[i];
        if (e > in_bytes) in_bytes = e;
    }
    size_t a_ioff = (in_bytes + 15) & ~(size_t) 15;
    size_t a_ilen = a_ioff + n * 8;
    size_t a_crc = (a_ilen + n * 4 + 15) & ~(size_t) 15;
    size_t total = a_crc + n * 4;
    if (hipSetDevice(c->device) != hipSuccess) return (int) hipErrorInvalidDevice;
    if (stage_reserve(c, total) != 0) return (int) hipErrorOutOfMemory;
    uint8_t *h = c->h_stage, *d = c->d_stage;
    memcpy(h, in, in_bytes);
    memcpy(h + a_ioff, in_off, n * 8);
    memcpy(h + a_ilen, in_len, n * 4);
    hipError_t err = hipMemcpyAsync(d, h, a_crc, hipMemcpyHostToDevice, c->stream);
    if (err != hipSuccess) return (int) err;
    int rc = rc_hip_crc32(d, (const uint64_t *) (d + a_ioff), (const uint32_t *) (d + a_ilen), (uint32_t) n,
                          (uint32_t *) (d + a_crc), c->crc_tables, (void *) c->stream);
    if (rc != 0) return rc;
    err = hipMemcpyAsync(h + a_crc, d + a_crc, n * 4, hipMemcpyDeviceToHost, c->stream);
    if (err != hipSuccess) return (int) err;
    err = hipStreamSynchronize(c->stream);
    if (err != hipSuccess) return (int) err;
    memcpy(crc_out, h + a_crc, n * 4);
    return 0;
}

/* ENetChecksumCallback (enet.h:338) with no context argument: a process-wide
 * context, created on first use.  Gather lists are checksummed as one stream,
 * like enet_crc32's loop over buffers (packet.c:148-160). */
static pthread_once_t crc_once = PTHREAD_ONCE_INIT;
static void *crc_ctx;
static pthread_mutex_t crc_lock = PTHREAD_MUTEX_INITIALIZER;
static void crc_ctx_init(void) { crc_ctx = enet_range_coder_create(); }

enet_uint32 enet_rc_crc32(const ENetBuffer *buffers, size_t bufferCount)
{
    pthread_once(&crc_once, crc_ctx_init);
    size_t total = 0;
    for (size_t i = 0; i < bufferCount; ++i) total += buffers[i].dataLength;
    if (!crc_ctx || total > 0xFFFFFFFFu) abort();          /* no silent CPU fallback */
    uint8_t *flat = (uint8_t *) malloc(total ? total : 1);
    if (!flat) abort();
    size_t pos = 0;
    for (size_t i = 0; i < bufferCount; ++i) {
        if (buffers[i].dataLength) memcpy(flat + pos, buffers[i].data, buffers[i].dataLength);
        pos += buffers[i].dataLength;
    }
    uint64_t off = 0;
    uint32_t len = (uint32_t) total, crc = 0;
    pthread_mutex_lock(&crc_lock);
    int rc = enet_rc_crc32_batch_host(crc_ctx, flat, &off, &len, 1, &crc);
    pthread_mutex_unlock(&crc_lock);
    free(flat);
    if (rc != 0) abort();
    return crc;
}

/* --------------------------------------------------------- per-datagram ABI */

size_t enet_range_coder_compress(void *context, const ENetBuffer *inBuffers, size_t inBufferCount,
                                 size_t inLimit, enet_uint8 *outData, size_t outLimit)
{
    rc_ctx *c = (rc_ctx *) context;
    if (c == NULL || inBufferCount <= 0 || inLimit <= 0) return 0;      /* compress.c:257-258 */
    /* the gather list is flattened into the staging the way compress.c:275-284
     * walks it (gather_len / gather_copy) */
    const size_t total = gather_len(inBuffers, inBufferCount);
    if (total > 0xFFFFFFFFu || outLimit > 0xFFFFFFFFu) return 0;
    if (total == 0) return 0;   /* only an empty first buffer: compress.c flushes nothing */
    const size_t first[2] = {0, inBufferCount};
    uint64_t ooff = 0;
    uint32_t ocap = (uint32_t) outLimit, olen = 0;
    const int rc = enet_rc_compress_gather_batch_host(c, inBuffers, first, 1, outData, &ooff, &ocap, &olen);
    return rc == 0 ? (size_t) olen : 0;
}

size_t enet_range_coder_decompress(void *context, const enet_uint8 *inData, size_t inLimit,
                                   enet_uint8 *outData, size_t outLimit)
{
    rc_ctx *c = (rc_ctx *) context;
    if (c == NULL || inLimit <= 0) return 0;                             /* compress.c:513-514 */
    if (inLimit > 0xFFFFFFFFu) return 0;
    uint64_t ioff = 0, ooff = 0;
    uint32_t ilen = (uint32_t) inLimit, ocap = (uint32_t) (outLimit > 0xFFFFFFFFu ? 0xFFFFFFFFu : outLimit);
    uint32_t olen = 0;
    int rc = enet_rc_decompress_batch_host(c, inData, &ioff, &ilen, 1, outData, &ooff, &ocap, &olen);
    return rc == 0 ? (size_t) olen : 0;
}

int enet_host_compress_with_range_coder(ENetHost *host)
{
    ENetCompressor compressor;
    if (!enet_host_compress) return -1;
    memset(&compressor, 0, sizeof compressor);
    compressor.context = enet_range_coder_create();
    if (compressor.context == NULL) return -1;
    compressor.compress = enet_range_coder_compress;
    compressor.decompress = enet_range_coder_decompress;
    compressor.destroy = enet_range_coder_destroy;
    enet_host_compress(host, &compressor);
    return 0;
}

uint32_t enet_rc_last_lane_count(void *context)
{
    rc_ctx *c = (rc_ctx *) context;
    if (!c) return 0;
    uint32_t v = 0, w = 0;
    hipDeviceSynchronize();
    if (hipMemcpy(&v, c->ws.counters + 3, 4, hipMemcpyDeviceToHost) != hipSuccess) return 0;
    for (int i = 0; i + 1 < c->last_split; ++i) {
        if (!c->twin[i] ||
            hipMemcpy(&w, ((rc_ctx *) c->twin[i])->ws.counters + 3, 4, hipMemcpyDeviceToHost) != hipSuccess) return 0;
        v += w;
    }
    return v;
}

uint32_t enet_rc_last_exact_count(void *context)
{
    rc_ctx *c = (rc_ctx *) context;
    if (!c) return 0;
    uint32_t v = 0, w = 0;
    hipDeviceSynchronize();
    if (hipMemcpy(&v, c->ws.counters, 4, hipMemcpyDeviceToHost) != hipSuccess) return 0;
    for (int i = 0; i + 1 < c->last_split; ++i) {
        if (!c->twin[i] || hipMemcpy(&w, ((rc_ctx *) c->twin[i])->ws.counters, 4, hipMemcpyDeviceToHost) != hipSuccess)
            return 0;
        v += w;
    }
    return v;
}

/* The context's kernel configuration as flag bits (the settings
 * enet_range_coder_create read from the environment); bit 31: the context
 * that runs the second half of its split host batches (run_host_split) has a
 * different one. */
static uint32_t config_flags(const rc_ctx *c)
{
    return (c->ws.kernel == RC_KERNEL_WAVE ? 1u : 0u) | (c->enc2_on ? 2u : 0u) | (c->enc2_wide_on ? 4u : 0u) |
           (c->ws.fast_dec ? 8u : 0u) | (c->ws.enc2_slow ? 16u : 0u) | ((c->ws.lane_active & 0x7Fu) << 8);
}

uint32_t enet_rc_config_flags(void *context)
{
    const rc_ctx *c = (const rc_ctx *) context;
    if (!c) return 0;
    const uint32_t f = config_flags(c);
    int differ = 0;
    for (int i = 0; i < SPLIT_MAX - 1; ++i) {
        const rc_ctx *t = (const rc_ctx *) c->twin[i];
        differ |= t && (config_flags(t) != f || t->enc2_stream_max != c->enc2_stream_max ||
                        t->enc2_wide_max != c->enc2_wide_max || t->max_slots != c->max_slots ||
                        t->ws.small_max != c->ws.small_max || t->ws.dec6_debug != c->ws.dec6_debug);
    }
    return f | (differ ? 0x80000000u : 0u);
}

uint32_t enet_rc_last_split(void *context) { return context ? (uint32_t) ((rc_ctx *) context)->last_split : 0u; }

uint32_t enet_rc_debug_counter(void *context, uint32_t i)
{
    rc_ctx *c = (rc_ctx *) context;
    uint32_t v = 0;
    if (!c || i >= 8 || !c->ws.counters || hipSetDevice(c->device) != hipSuccess) return 0;
    if (hipStreamSynchronize(c->stream) != hipSuccess ||
        hipMemcpy(&v, c->ws.counters + i, 4, hipMemcpyDeviceToHost) != hipSuccess) {
        (void) hipGetLastError();
        return 0;
    }
    return v;
}

uint32_t enet_rc_last_host_paths(void *context)
{
    const rc_ctx *c = (const rc_ctx *) context;
    if (!c) return 0;
    /* a split batch: its last piece's */
    for (int i = c->last_split - 2; i >= 0; --i)
        if (c->twin[i]) return ((const rc_ctx *) c->twin[i])->last_paths;
    return c->last_paths;
}

/* ------------------------------------------------------ for rc_multi.c */

int rc_ctx_device(void *context) { return context ? ((rc_ctx *) context)->device : -1; }
void *rc_ctx_stream(void *context) { return context ? (void *) ((rc_ctx *) context)->stream : NULL; }

int rc_ctx_run_device(void *context, int decompress, const uint8_t *in, const uint64_t *in_off,
                      const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                      const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len, void *stream)
{
    return run_device((rc_ctx *) context, decompress, in, in_off, in_len, n, max_len, 0, out, out_off, out_cap,
                      out_len, stream);
}

int rc_ctx_run_host(void *context, int decompress, const uint8_t *in, const uint64_t *in_off,
                    const uint32_t *in_len, size_t n, uint8_t *out, const uint64_t *out_off,
                    const uint32_t *out_cap, uint32_t *out_len)
{
    /* (no page-locking of the caller's memory: the devices' ranges share
     * boundary pages, and one range's unregister would unpin another's) */
    return run_host((rc_ctx *) context, decompress, in, in_off, in_len, n, out, out_off, out_cap, out_len, 0, NULL, NULL);
}

/* The context's block-sum workspace of rc_pack.hip for n packets (device
 * pointer, ceil(n / 1024) + 1 words; the last holds the packed total). */
uint64_t *rc_ctx_bsum(void *context, size_t n)
{
    rc_ctx *c = (rc_ctx *) context;
    if (!c || hipSetDevice(c->device) != hipSuccess) return NULL;
    const size_t blocks = (n + 1023) / 1024;
    if (blocks + 1 > c->d_bsum_cap) {
        hipDeviceSynchronize();
        if (c->d_bsum) hipFree(c->d_bsum);
        c->d_bsum = NULL; c->d_bsum_cap = 0;
        if (hipMalloc((void **) &c->d_bsum, (blocks + 1) * 8) != hipSuccess) return NULL;
        c->d_bsum_cap = blocks + 1;
    }
    return c->d_bsum;
}

/* Packs out_len[i] bytes of each packet back to back (rc_pack.hip). */
int enet_rc_pack_batch_device(void *context, const uint8_t *out, const uint64_t *out_off, const uint32_t *out_len,
                              size_t n, uint8_t *packed, void *stream)
{
    rc_ctx *c = (rc_ctx *) context;
    if (!c || n > 0xFFFFFFFFu) return (int) hipErrorInvalidValue;
    if (n == 0) return 0;
    uint64_t *bsum = rc_ctx_bsum(c, n);
    if (!bsum) return (int) hipErrorOutOfMemory;
    return rc_hip_pack(out, out_off, out_len, (uint32_t) n, bsum, packed, stream);
}

const char *enet_rc_version(void) { return "enet_rc_amd 0.3 (gfx950)"; }
