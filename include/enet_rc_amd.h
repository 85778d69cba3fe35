/*
 * enet_rc_amd.h -- C ABI of the MI355X range-coder packet compressor.
 *
 * Drop-in for ENet's range coder (lsalzman/enet compress.c).  Link
 * libenet_rc_amd.so ahead of libenet (or drop compress.o from libenet): the
 * four enet_range_coder_* symbols and enet_host_compress_with_range_coder
 * below have exactly the reference signatures and return conventions, so
 * host.c / protocol.c call them unchanged.  The batch entry points are new:
 * they are how the GPU is meant to be used (one wavefront per packet).
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
#endif

/* =================================================================== drop-in
 * Replaces compress.c:48-56.  Creates a coder context bound to the current HIP
 * device (its own stream + device workspace).  NULL on failure (no device,
 * out of memory).  Like the reference, one context is not thread-safe;
 * distinct contexts are independent. */
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
 * hipStream_t; NULL = the default null stream) and not waited for. */
int enet_rc_compress_batch_device(void *context, const uint8_t *in, const uint64_t *in_off,
                                  const uint32_t *in_len, size_t n, uint32_t max_len,
                                  uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                                  uint32_t *out_len, void *stream);
int enet_rc_decompress_batch_device(void *context, const uint8_t *in, const uint64_t *in_off,
                                    const uint32_t *in_len, size_t n, uint32_t max_len,
                                    uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                                    uint32_t *out_len, void *stream);

/* Same with HOST pointers: copies in through pinned staging, runs, copies
 * out, and returns when the results are in host memory. */
int enet_rc_compress_batch_host(void *context, const uint8_t *in, const uint64_t *in_off,
                                const uint32_t *in_len, size_t n, uint8_t *out,
                                const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len);
int enet_rc_decompress_batch_host(void *context, const uint8_t *in, const uint64_t *in_off,
                                  const uint32_t *in_len, size_t n, uint8_t *out,
                                  const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len);

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

/* ============================================================ introspection */
/* Number of packets of the last batch that took the exact (binary-tree) path. */
uint32_t enet_rc_last_exact_count(void *context);
/* Library version string. */
const char *enet_rc_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ENET_RC_AMD_H */
