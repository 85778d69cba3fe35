/*
 * rc_abi_internal.h -- descriptors shared by the C host shim (rc_host.c) and
 * the HIP launch code (rc_kernels.hip, rc_route.hip).  Plain C, plain pointers.
 */
#ifndef ENET_RC_ABI_INTERNAL_H
#define ENET_RC_ABI_INTERNAL_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One batch of independent packets, all pointers in device memory.
 * packet i: in[in_off[i] .. in_off[i]+in_len[i]) -> out[out_off[i] .. +out_cap[i]);
 * out_len[i] receives what enet_range_coder_{compress,decompress} would return. */
typedef struct {
    const uint8_t  *in;
    const uint64_t *in_off;
    const uint32_t *in_len;
    uint8_t        *out;
    const uint64_t *out_off;
    const uint32_t *out_cap;
    uint32_t       *out_len;
    uint32_t        n;
    uint32_t        max_len;   /* upper bound of in_len[] used to size LDS; longer packets take the exact path */
    uint32_t        max_out;   /* upper bound of out_cap[] when the caller knows it, else 0; sizes the
                                  wave decoder's LDS arena (a model that outgrows it takes the exact path) */
} rc_batch_dev;

/* Device workspace owned by a coder context. */
typedef struct {
    uint32_t *flag_list;    /* [n_cap] packets routed to the exact path */
    uint32_t *counters;     /* [8]: 0 = flagged count, 1 = work queue head (fast), 2 = exact queue head,
                               3 = packets the two-pass encoder (compress) or the bucket-history
                               decoder (decompress) leaves to the lane kernels, 4 = packets the
                               encoder's scan lists for its wide mode (per chunk) */
    void     *exact_pool;   /* exact_slots * RC_EXACT_POOL_BYTES */
    uint32_t  exact_slots;
    uint32_t  n_cap;
    void     *lane_pool;    /* lane_slots * lane_region bytes: per-lane order-1/2 model regions */
    uint32_t  lane_slots;   /* lanes with a region (multiple of 256) */
    uint32_t  lane_region;  /* bytes per region */
    uint32_t  kernel;       /* RC_KERNEL_* */
    uint32_t  lane_active;  /* lane kernels: packets per wavefront (64, 32 or 16) */
    uint32_t *order;        /* [n_cap] processing order (packets binned by length), lane kernels */
    uint32_t *bins;         /* length-bin counts [RC_LEN_BINS], uniform flag, fill counters at
                               RC_LEN_FILL; = counters + 8 (one control block, RC_CTL_WORDS, cleared
                               by one fill per call) */
    uint32_t  cus;          /* compute units of the device */
    uint32_t  small_max;    /* lane3 contexts: batches of up to this many packets (and no more than
                               fit on the chip at once) run on the wave kernel; RC_SMALL_AUTO = no cap */
    /* two-pass encoder (rc_enc2.hip): record stream and the packets it leaves to the lane kernels */
    void     *enc2_stream;  /* NULL: the encoder is off (ENET_RC_ENC2=0) or not allocated yet */
    uint64_t  enc2_cap;     /* bytes */
    uint32_t *enc2_list;    /* [n_cap] */
    /* its wide mode (packets with a bucket over 64 positions): 16-B records per position,
       one slot per packet listed in enc2_wlist (RC_WSHARDS regions, counts at counters +
       RC_WSHARD_AT); NULL: off (ENET_RC_ENC2_WIDE=0) */
    void     *enc2_wide;
    uint64_t  enc2_wide_cap;  /* bytes */
    uint32_t *enc2_wlist;     /* [n_cap] */
    /* the fast decoder in front of the v3 lane decoder: 1 = the record-light decoder with its
       input through LDS slots a helper wavefront refills (rc_dec6.hip rc_decompress_dec6s; the
       default, lane_active == 64), 0 = none (ENET_RC_DEC=0, or lane_active != 64);
       the packets it leaves go to enc2_list / counters[3] */
    uint32_t  fast_dec;
    /* rc_dec6.hip: per packet, the positions the decoder took to start a new bigram (its
       check, rc_dec6_verify), 0xFFFFFFFF for a packet left to the lane kernels */
    uint32_t *claims;       /* [n_cap] */
    /* rc_dec6.hip: per packet, where its model segments after the first start (the resets of
       compress.c:148-157): 12 bits each, their count in bits 24-25 */
    uint32_t *dec6_resets;  /* [n_cap] */
    /* rc_dec6.hip: per packet, the sums of the input chunks that passed through the decoder's
       LDS slot (rc_slot.h slot_mix) as the decoder took them and as its helper loaded them;
       rc_dec6_verify sends a packet whose sums differ to the lane kernels */
    uint32_t *dec6_icks;    /* [n_cap] */
    uint32_t *dec6_hcks;    /* [2 n_cap]: the helper's sums, then its last chunk's terms */
    uint32_t  dec6_debug;   /* diagnostic (ENET_RC_DEC6_DEBUG): 1 = the check lists every packet */
    void     *dec6_pool;    /* lane_slots * RC_DEC6_TAB_BYTES: rc_dec6.hip's bucket records */
    /* test switch (ENET_RC_ENC2_SLOW=1): the scan takes its slow paths (every position
       exceptional, every bucket sorted and re-walked) */
    uint32_t  enc2_slow;
    /* lane kernels: when set, run only the sub_count[0] packets of sub_list
       (the wave kernels too: their block i takes sub_list[i]) */
    const uint32_t *sub_list;
    const uint32_t *sub_count;
    /* the context compresses on the two-pass encoder (ENET_RC_ENC2): small
       batches take it too (rc_kernels.hip small_route) */
    uint32_t  enc2_on;
    /* rc_route.hip: the packets the record-light decoder leaves go to the
       wave kernel instead of the lane kernels (small batches) */
    uint32_t  wave_tail;
} rc_workspace_dev;

#define RC_SMALL_AUTO 0xFFFFFFFFu
#define RC_DEC6_TAB_BYTES 16512u  /* per lane: 256 buckets x (a 16-B and a 48-B record), 128 B of dummy slots
                                     (the 16-B records of all lanes first, then the rest: rc_dec6_rare.h) */

#define RC_LEN_BINS 256u     /* 16-byte length bins, longest first; 4096 B / 16 */
#define RC_LEN_FILL (RC_LEN_BINS + 4u)     /* bins[]: rc_len_scatter's fill counters, one per bin */
#define RC_CTL_BINS_END (8u + RC_LEN_FILL + RC_LEN_BINS)   /* counters[8], bins (counts, uniform flag, fills) */
/* the wide list's counters (rc_enc2.hip): RC_WSHARDS of them, 128 B apart, after the bins */
#define RC_WSHARDS 8u
#define RC_WSHARD_STRIDE 32u
#define RC_WSHARD_AT ((RC_CTL_BINS_END + 31u) & ~31u)
#define RC_CTL_WORDS (RC_WSHARD_AT + RC_WSHARDS * RC_WSHARD_STRIDE)
#define RC_KERNEL_WAVE 1u   /* one packet per wavefront */
#define RC_KERNEL_LANE3 2u  /* one packet per lane, model v3 (rc_lane3.hip, default) */

#define RC_EXACT_POOL_BYTES 98304u   /* 4096 nodes x 16 B (compress.c:42-46) + 4096 x 8 B rescale frames */

/* Launchers (rc_kernels.hip).  Return 0 or a hipError_t value. Stream-ordered, no host sync. */
int rc_hip_compress(const rc_batch_dev *b, const rc_workspace_dev *ws, void *stream);
int rc_hip_decompress(const rc_batch_dev *b, const rc_workspace_dev *ws, void *stream);

/* Two-pass encoder (rc_enc2.hip): record-stream bytes per packet of up to
 * max_len bytes, and the launcher (both passes, chunked by ws->enc2_cap;
 * packets off its fast path are listed in ws->enc2_list, count in
 * ws->counters[3]). */
uint64_t rc_hip_enc2_slot_bytes(uint32_t max_len);
uint64_t rc_hip_enc2_wide_slot_bytes(uint32_t max_len);
int rc_hip_enc2_launch(const rc_batch_dev *b, const rc_workspace_dev *ws, void *stream);

/* Record-light decoder (rc_dec6.hip) and its check: one packet per lane, model in LDS;
 * packets off its fast path or failing the check are listed in ws->enc2_list, count in
 * ws->counters[3]. */
int rc_hip_dec6_launch(const rc_batch_dev *b, const rc_workspace_dev *ws, uint32_t blocks, void *stream);
/* rc_dec6.hip's check alone (after rc_decompress_dec6s). */
int rc_hip_dec6_verify_launch(const rc_batch_dev *b, const rc_workspace_dev *ws, void *stream);

/* Per-lane region size the lane kernels need for packets up to max_len bytes. */
uint32_t rc_hip_lane3_region_bytes(uint32_t max_len);

/* Whether a batch runs on the lane path (rc_route.hip: fast kernels + lane
 * kernels, which need the lane pool and the encoder's record stream) rather
 * than on the wavefront-per-packet kernels (rc_kernels.hip launch). */
int rc_hip_uses_lanes(int decompress, const rc_batch_dev *b, const rc_workspace_dev *ws);

/* CRC-32 of each packet (rc_crc32.hip): crc_out[i] = enet_crc32 (packet.c:143-163)
 * of in[in_off[i] .. +in_len[i]).  tables: rc_hip_crc32_table_words() words
 * built by rc_hip_crc32_build_tables, in device memory. */
int rc_hip_crc32(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len, uint32_t n,
                 uint32_t *crc_out, const uint32_t *tables, void *stream);
uint32_t rc_hip_crc32_table_words(void);
void rc_hip_crc32_build_tables(uint32_t *t);

/* Datagram framing (rc_dgram.hip).  All pointers in
 * device memory; p_*, q_*, c_len, s_*, crc, want are workspace arrays of n. */
typedef struct {
    const uint8_t  *in;
    const uint64_t *in_off;
    const uint32_t *in_len;
    uint8_t        *out;
    const uint64_t *out_off;
    uint32_t       *out_len;
    const uint32_t *seed;       /* checksum field value while summing: connectID or 0 */
    uint64_t       *p_off;      /* command range of each datagram (coder input) */
    uint32_t       *p_len;
    uint64_t       *q_off;      /* its slot in out (coder output) */
    uint32_t       *q_cap;
    uint32_t       *c_len;      /* coder result */
    uint8_t        *scratch;    /* encode: n x 4096 B, the datagrams the checksum covers */
    uint64_t       *s_off;
    uint32_t       *s_len;
    uint32_t       *crc;
    uint32_t       *want;       /* decode: received checksum field */
    uint32_t        n;
    uint32_t        checksum;   /* the host has a checksum callback (4-B field in the header) */
} rc_dgram_dev;

enum { RC_DGRAM_ENC_PREP = 0, RC_DGRAM_ENC_STAGE, RC_DGRAM_ENC_FINISH,
       RC_DGRAM_DEC_PREP, RC_DGRAM_DEC_STAGE, RC_DGRAM_DEC_FINISH };
int rc_hip_dgram_launch(int stage, const rc_dgram_dev *g, void *stream);

/* Pack out_len[i] bytes of each packet (at out_off[i]) back to back into
 * packed (rc_pack.hip); bsum: ceil(n / 1024) + 1 words, bsum[last] = total. */
int rc_hip_pack(const uint8_t *out, const uint64_t *out_off, const uint32_t *out_len, uint32_t n,
                uint64_t *bsum, uint8_t *packed, void *stream);
/* packets [src + soff[i], +len[i]) -> dst + doff[i] in whole 16-B granules
 * (doff[i] has the source address's alignment mod 16, its granules belong
 * to packet i alone); src may
 * be mapped host memory (rc_pack.hip) */
int rc_hip_gather16(const uint8_t *src, const uint64_t *soff, uint8_t *dst, const uint64_t *doff,
                    const uint32_t *len, uint32_t n, void *stream);
/* out_len bytes of each packet from src + off[i] to dst + off[i], one
 * wavefront per packet; dst may be mapped host memory (rc_pack.hip) */
int rc_hip_slot_copy(const uint8_t *src, const uint64_t *off, const uint32_t *len, uint32_t n, uint8_t *dst,
                     uint32_t max_wgs, void *stream);
/* The reverse of rc_hip_pack: packed (back to back) -> out[out_off[i] .. +out_len[i]). */
int rc_hip_unpack(const uint8_t *packed, uint8_t *out, const uint64_t *out_off, const uint32_t *out_len,
                  uint32_t n, uint64_t *bsum, void *stream);

/* rc_multi.c's split on the device holding the batch (rc_multi_plan.hip):
 * plan (5 parts + 1 words, device) = first[0 .. parts], then per part the
 * lowest in_off, highest in_off + in_len, lowest out_off, highest out_off +
 * out_cap; ws: rc_hip_multi_plan_ws(n) words.  1 <= parts <= 64, n >= 1. */
size_t rc_hip_multi_plan_ws(size_t n);
int rc_hip_multi_plan(const uint32_t *in_len, const uint64_t *in_off, const uint64_t *out_off,
                      const uint32_t *out_cap, uint64_t n, uint32_t parts, uint64_t *ws, uint64_t *plan,
                      void *stream);
/* a[i] -= la, b[i] -= lb for i < cnt (a part's offsets rebased on its device) */
int rc_hip_multi_rebase(uint64_t *a, uint64_t la, uint64_t *b, uint64_t lb, uint64_t cnt, void *stream);

/* Kernel introspection for bench/profiling. */
const char *rc_hip_fast_kernel_name(int decompress, uint32_t kernel);
uint32_t    rc_hip_lds_bytes(uint32_t max_len);

#ifdef __cplusplus
}
#endif
#endif
