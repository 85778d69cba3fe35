/*
 * enet_rc_amd.h -- C ABI of the MI355X range-coder packet compressor.
 *
 * Drop-in for ENet's range coder (lsalzman/enet compress.c).  Link
 * libenet_rc_amd.so ahead of libenet (or drop compress.o from libenet): the
 * four enet_range_coder_* symbols and enet_host_compress_with_range_coder
 * below have exactly the reference signatures and return conventions, so
 * host.c / protocol.c call them unchanged.  The batch entry points are new:
 * they are how the GPU is meant to be used: large batches run one packet
 * per lane (the two-pass encoder and the record-light decoder with its
 * check, then the lane kernels for what they leave), batches that fit on the
 * chip at one wavefront per packet run on the wavefront-per-packet kernels.
 *
 * Plain C, plain pointers and sizes; no HIP or torch types appear here
 * (streams are passed as void*).
 */
#ifndef ENET_RC_AMD_H
#define ENET_RC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- reference types (include/enet/types.h:8-10, unix.h:30-34, enet.h:325-335).
 * If enet/enet.h was included first these are already defined. */
#ifndef __ENET_TYPES_H__
typedef unsigned char enet_uint8;
typedef unsigned short enet_uint16;
typedef unsigned int enet_uint32;
#endif
#ifndef __ENET_ENET_H__
typedef struct { void *data; size_t dataLength; } ENetBuffer;
typedef struct _ENetCompressor {
    void *context;
    size_t (*compress)(void *context, const ENetBuffer *inBuffers, size_t inBufferCount,
                       size_t inLimit, enet_uint8 *outData, size_t outLimit);
    size_t (*decompress)(void *context, const enet_uint8 *inData, size_t inLimit,
                         enet_uint8 *outData, size_t outLimit);
    void (*destroy)(void *context);
} ENetCompressor;
typedef struct _ENetHost ENetHost;
typedef struct _ENetAddress { enet_uint32 host; enet_uint16 port; } ENetAddress;   /* enet.h:85-89 */
#endif

/* =================================================================== drop-in
 * Replaces compress.c:48-56.  Creates a coder context bound to the current HIP
 * device (its own stream + device workspace).  NULL on failure (no device,
 * out of memory).  Like the reference, one context is not thread-safe;
 * distinct contexts are independent.
 *
 * Read once here from the environment (all optional):
 *   ENET_RC_KERNEL=wave         force the wavefront-per-packet kernels
 *                               (default: the lane path above)
 *   ENET_RC_SMALL_BATCH=n       batches of up to n packets (and no more than
 *                               fit on the chip at one wavefront each) run on
 *                               the wavefront-per-packet kernels; 0 = never;
 *                               unset = every batch that fits
 *   ENET_RC_DEBUG=1             log pool sizes and kernel routing to stderr */
void *enet_range_coder_create(void);

/* Replaces compress.c:58-66.  NULL is ignored. */
void enet_range_coder_destroy(void *context);

/* Replaces compress.c:246-342.  Compresses the gather list (consumed exactly as
 * compress.c:275-284 does, including its one-byte read of an empty non-first
 * buffer) into outData.  Returns the compressed size, or 0 when context is
 * NULL, inBufferCount or inLimit is 0, or the output would exceed outLimit. */
size_t enet_range_coder_compress(void *context, const ENetBuffer *inBuffers, size_t inBufferCount,
                                 size_t inLimit, enet_uint8 *outData, size_t outLimit);

/* Replaces compress.c:498-627.  Returns the decompressed size, or 0 on a
 * corrupt stream, NULL context, empty input, or output beyond outLimit. */
size_t enet_range_coder_decompress(void *context, const enet_uint8 *inData, size_t inLimit,
                                   enet_uint8 *outData, size_t outLimit);

/* Replaces compress.c:637-650: registers the GPU coder with an ENet host
 * through the host library's enet_host_compress (host.c:294-304).  0 on
 * success, -1 if the context cannot be created or libenet is not linked. */
int enet_host_compress_with_range_coder(ENetHost *host);

/* ===================================================================== batch
 * A batch is n independent packets: packet i is in[in_off[i] .. +in_len[i])
 * and its result goes to out[out_off[i] .. +out_cap[i]); out_len[i] receives
 * exactly what enet_range_coder_compress (single buffer, inLimit = in_len[i],
 * outLimit = out_cap[i]) or enet_range_coder_decompress would return.
 * max_len bounds in_len[] (it sizes each lane's model region in HBM; longer
 * packets are still handled, on the slower exact path); 0 means 4096.
 * Return value: 0 on success, otherwise a HIP error code. */

/* All pointers are DEVICE pointers; work is enqueued on `stream` (a
 * hipStream_t; NULL = the default null stream) and not waited for.  The
 * calls of one context share its device workspace: issue them on one stream,
 * or order the streams, as for any buffer reused across streams. */
int enet_rc_compress_batch_device(void *context, const uint8_t *in, const uint64_t *in_off,
                                  const uint32_t *in_len, size_t n, uint32_t max_len,
                                  uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                                  uint32_t *out_len, void *stream);
int enet_rc_decompress_batch_device(void *context, const uint8_t *in, const uint64_t *in_off,
                                    const uint32_t *in_len, size_t n, uint32_t max_len,
                                    uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                                    uint32_t *out_len, void *stream);
/* As enet_rc_decompress_batch_device, plus max_out >= every out_cap[i] (0 =
 * unknown).  The bound sizes the model of the wavefront-per-packet decoder
 * that small batches run on, so twice as many packets decode at one wavefront
 * per packet (1024 instead of 512 at max_out 1200).  A smaller max_out than some
 * out_cap[i] is not an error: a packet whose model outgrows it takes the exact
 * path.  No reference counterpart (the reference decompresses one datagram
 * per call, compress.c:506). */
int enet_rc_decompress_batch_device_bounded(void *context, const uint8_t *in, const uint64_t *in_off,
                                            const uint32_t *in_len, size_t n, uint32_t max_len,
                                            uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                                            uint32_t *out_len, uint32_t max_out, void *stream);

/* Same with HOST pointers: copies in through pinned staging, runs, copies
 * out, and returns when the results are in host memory. */
int enet_rc_compress_batch_host(void *context, const uint8_t *in, const uint64_t *in_off,
                                const uint32_t *in_len, size_t n, uint8_t *out,
                                const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len);
int enet_rc_decompress_batch_host(void *context, const uint8_t *in, const uint64_t *in_off,
                                  const uint32_t *in_len, size_t n, uint8_t *out,
                                  const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len);

/* Compress a batch of gather lists (host pointers): packet i is the list
 * buffers[first[i] .. first[i + 1]) (first has n + 1 entries), consumed
 * exactly as enet_range_coder_compress consumes its inBuffers
 * (compress.c:260-285: an empty first buffer contributes nothing, an empty
 * later buffer its data[0]); protocol.c:1688-1695 hands the compressor
 * &buffers[1], bufferCount - 1 per datagram.  A list of one empty buffer
 * (or none) yields out_len 0.  Outputs as enet_rc_compress_batch_host.  The
 * lists are flattened straight into the context's pinned staging. */
int enet_rc_compress_gather_batch_host(void *context, const ENetBuffer *buffers, const size_t *first, size_t n,
                                       uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                                       uint32_t *out_len);

/* ==================================================================== CRC-32
 * crc_out[i] = enet_crc32 (packet.c:143-163) of the single buffer
 * in[in_off[i] .. +in_len[i]): CRC-32/IEEE, returned in network byte order
 * exactly like the reference (ENET_HOST_TO_NET_32 of the complement), i.e.
 * the value protocol.c:1709-1718 writes into the datagram header and
 * protocol.c:1075-1091 compares.  Device / host pointer variants as above. */
int enet_rc_crc32_batch_device(void *context, const uint8_t *in, const uint64_t *in_off,
                               const uint32_t *in_len, size_t n, uint32_t *crc_out, void *stream);
int enet_rc_crc32_batch_host(void *context, const uint8_t *in, const uint64_t *in_off,
                             const uint32_t *in_len, size_t n, uint32_t *crc_out);
/* Same signature as enet_crc32 / ENetChecksumCallback (enet.h:338, enet.h:564):
 * host->checksum = enet_rc_crc32.  Uses a process-wide GPU context; aborts if
 * no GPU is usable (there is no CPU fallback). */
enet_uint32 enet_rc_crc32(const ENetBuffer *buffers, size_t bufferCount);

/* ========================================================= datagram framing
 * Whole ENet wire datagrams in and out: the framing
 * of protocol.c around the compressor and checksum callbacks, for n datagrams
 * in one pass.  Layout (protocol.h:48-53): big-endian peerID word (bit 14
 * COMPRESSED, bit 15 SENT_TIME), big-endian sentTime if SENT_TIME, a 4-byte
 * checksum field if `checksum` (the host has a checksum callback), then the
 * commands.  seed[i] is the value the checksum field holds while summing: the
 * peer's connectID, or 0 for peerID 0xFFF (protocol.c:1079, :1711); it may be
 * NULL when checksum == 0.  Datagrams are at most 4096 bytes
 * (ENET_PROTOCOL_MAXIMUM_MTU).
 *
 * Encode replaces protocol.c:1686-1718 for each datagram: in[i] is the
 * datagram as assembled (header, checksum field, uncompressed commands; the
 * COMPRESSED bit is ignored); out[out_off[i] ..] receives the wire datagram --
 * commands range-coded with outLimit = their length and used only if smaller
 * (COMPRESSED set), checksum (enet_crc32 of the uncompressed datagram with
 * the final header and the seed in the field) filled in; out_len[i] is its
 * length (<= in_len[i]), 0 if the datagram is shorter than its header.
 *
 * Decode replaces protocol.c:1022-1091: in[i] is a received datagram;
 * out[out_off[i] ..] (4096 bytes per slot) receives what protocol.c goes on
 * parsing -- header + decompressed commands, checksum field holding the seed
 * -- and out_len[i] its length, or 0 where protocol.c drops the datagram
 * (shorter than 2 bytes or its header, decompression failing or longer than
 * 4096 - headerSize, checksum mismatch).  Peer-state checks (:1035-1050) stay
 * with the caller.  Return value as for the batch calls. */
int enet_rc_datagram_encode_batch_device(void *context, const uint8_t *in, const uint64_t *in_off,
                                         const uint32_t *in_len, size_t n, int checksum,
                                         const uint32_t *seed, uint8_t *out, const uint64_t *out_off,
                                         uint32_t *out_len, void *stream);
int enet_rc_datagram_decode_batch_device(void *context, const uint8_t *in, const uint64_t *in_off,
                                         const uint32_t *in_len, size_t n, int checksum,
                                         const uint32_t *seed, uint8_t *out, const uint64_t *out_off,
                                         uint32_t *out_len, void *stream);
int enet_rc_datagram_encode_batch_host(void *context, const uint8_t *in, const uint64_t *in_off,
                                       const uint32_t *in_len, size_t n, int checksum, const uint32_t *seed,
                                       uint8_t *out, const uint64_t *out_off, uint32_t *out_len);
int enet_rc_datagram_decode_batch_host(void *context, const uint8_t *in, const uint64_t *in_off,
                                       const uint32_t *in_len, size_t n, int checksum, const uint32_t *seed,
                                       uint8_t *out, const uint64_t *out_off, uint32_t *out_len);

/* ============================================================ batched I/O
 * enet_socket_receive / enet_socket_send (unix.c:440-528) for many datagrams
 * per system call (recvmmsg / sendmmsg), non-blocking.  Receive: up to max
 * datagrams into buf + i * slot_bytes, lengths[i] (0 for a truncated one,
 * which the reference skips, unix.c:509-512), addresses[i] (may be NULL);
 * returns the count (0 if none is queued) or -1.  Send: datagram i is
 * buf[off[i] .. +len[i]) to addresses[i] (NULL: a connected socket); returns
 * how many went out, or -1.  Host memory only; no GPU needed. */
int enet_rc_socket_receive_batch(int socket, uint8_t *buf, size_t slot_bytes, size_t max,
                                 uint32_t *lengths, ENetAddress *addresses);
int enet_rc_socket_send_batch(int socket, const uint8_t *buf, const uint64_t *off, const uint32_t *len,
                              const ENetAddress *addresses, size_t n);

/* ================================================================ multi-GPU
 * One process, several GPUs (no reference counterpart).  Packets
 * are independent (compress.c:252-265): a batch is split into contiguous
 * packet ranges of about equal payload bytes, one per device, and every
 * device codes its range with its own context, concurrently.  Results are
 * exactly those of the single-device calls.
 *
 * enet_rc_multi_create binds one context per listed device (devices[0] is
 * the root of the device-pointer calls; a device may be listed twice, which
 * only makes sense for testing).  NULL on failure. */
void *enet_rc_multi_create(const int *devices, size_t n_devices);
void enet_rc_multi_destroy(void *multi);
size_t enet_rc_multi_devices(void *multi);
/* The split: device k gets packets [first[k], first[k + 1]) (first has
 * parts + 1 entries); the smallest index whose prefix sum of in_len reaches
 * k / parts of the total.  0, or -1 on bad arguments.  Host-only. */
int enet_rc_multi_split(const uint32_t *in_len, size_t n, size_t parts, uint64_t *first);
/* The split with each part's byte ranges: first[0 .. parts] as above, then
 * per part k at plan[parts + 1 + 4k]: lowest in_off, highest in_off + in_len,
 * lowest out_off, highest out_off + out_cap (UINT64_MAX, 0, UINT64_MAX, 0
 * when empty); plan holds 5 parts + 1 words.  Host pointers, host-only; 0 or
 * -1.  enet_rc_multi_plan_device computes the same on the current device
 * from device pointers (as the device-pointer calls below do; n >= 1) and
 * copies the plan to host memory; 0 or a hipError_t. */
int enet_rc_multi_plan(const uint32_t *in_len, const uint64_t *in_off, const uint64_t *out_off,
                       const uint32_t *out_cap, size_t n, size_t parts, uint64_t *plan);
int enet_rc_multi_plan_device(const uint32_t *in_len, const uint64_t *in_off, const uint64_t *out_off,
                              const uint32_t *out_cap, size_t n, size_t parts, uint64_t *plan);
/* HOST pointers, as enet_rc_*_batch_host: one host thread per device copies
 * its range in, codes it and copies it out; returns with the results. */
int enet_rc_multi_compress_batch_host(void *multi, const uint8_t *in, const uint64_t *in_off,
                                      const uint32_t *in_len, size_t n, uint8_t *out,
                                      const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len);
int enet_rc_multi_decompress_batch_host(void *multi, const uint8_t *in, const uint64_t *in_off,
                                        const uint32_t *in_len, size_t n, uint8_t *out,
                                        const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len);
/* DEVICE pointers on devices[0]: the split is computed there; every other
 * device's range is copied to it over the peer link (hipMemcpyPeerAsync,
 * xGMI) and coded there, and a copy kernel on the root reads each packet's
 * produced bytes back into the root's slots over the link (only bytes
 * [out_off[i], +out_len[i]) are written).  The _stream calls take the
 * caller's stream on the root (hipStream_t, NULL = the null stream): the
 * inputs must be complete in its order, and the root's work waits for it
 * there, not on the host.  The calls without a stream wait for the whole root
 * device first (any stream's work on the inputs).  Both return with the
 * results in place. */
int enet_rc_multi_compress_batch_device(void *multi, const uint8_t *in, const uint64_t *in_off,
                                        const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                                        const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len);
int enet_rc_multi_decompress_batch_device(void *multi, const uint8_t *in, const uint64_t *in_off,
                                          const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                                          const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len);
int enet_rc_multi_compress_batch_device_stream(void *multi, const uint8_t *in, const uint64_t *in_off,
                                               const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                                               const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len,
                                               void *stream);
int enet_rc_multi_decompress_batch_device_stream(void *multi, const uint8_t *in, const uint64_t *in_off,
                                                 const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                                                 const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len,
                                                 void *stream);

/* Packs out_len[i] bytes of each packet (at out_off[i]) back to back into
 * packed, on the device (the gather of a batch's results before a copy);
 * packed holds at least the sum of out_len.  Device pointers, on `stream`. */
int enet_rc_pack_batch_device(void *context, const uint8_t *out, const uint64_t *out_off, const uint32_t *out_len,
                              size_t n, uint8_t *packed, void *stream);

/* ============================================================ introspection */
/* Number of packets of the last batch that took the exact (binary-tree) path. */
uint32_t enet_rc_last_exact_count(void *context);
/* Number of packets of the last batch that the first pass (the two-pass
 * encoder, or the record-light decoder and its check) left to the lane kernels. */
uint32_t enet_rc_last_lane_count(void *context);
/* The context's kernel configuration, fixed when it was created (bits: 1 wave
 * kernel, 2 two-pass encoder, 4 its wide mode, 8 fast decoder, 16 the
 * encoder's slow paths forced, 8-14 packets per lane-kernel wavefront); bit 31
 * set if a context that runs a piece of its split host batches was
 * configured differently (never, by construction). */
uint32_t enet_rc_config_flags(void *context);
/* The number of pieces the last host-pointer batch ran in, each on its own
 * context of the device (large batches: a piece's input copy under the
 * earlier pieces' kernels; ENET_RC_HOST_SPLIT), or 0 if it ran in one. */
uint32_t enet_rc_last_split(void *context);
/* How the last host-pointer batch (its last piece, if split) moved its data:
 * bits 0-3 the input (1 pinned staging, 2 the caller's page-locked range by
 * DMA, 3 strided DMA of uniform slots, 4 GPU gather over the caller's mapped
 * range), bits 4-7 the results (1 one D2H of all slots (small batches), 2 one
 * DMA of back-to-back slots every packet filled, 3 GPU copy into the caller's
 * mapped slots, 4 packed on the device, D2H, scattered on the host); 0 before
 * any host batch. */
uint32_t enet_rc_last_host_paths(void *context);
/* Diagnostic: word i (< 8) of the context's device counter block after the
 * last batch (synchronous read; 0 on error).  Used by tools/, not by ENet. */
uint32_t enet_rc_debug_counter(void *context, uint32_t i);
/* Library version string. */
const char *enet_rc_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ENET_RC_AMD_H */
