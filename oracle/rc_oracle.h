/*
 * rc_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of ENet's adaptive order-2 PPM range coder
 * (reference: compress.c in lsalzman/enet 1.3.18).  It exists to check the
 * MI355X product path; nothing in enet_amd/ links, loads or calls it.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 *
 * Parity pin: tests/test_oracle.py checks this restatement byte-for-byte
 * against fixtures produced by the real compress.c (built from the reference
 * sources into oracle/_ref/ by oracle/Makefile; see tests/golden/README.md).
 */
#ifndef RC_ORACLE_H
#define RC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same layout as ENetBuffer on Unix (include/enet/unix.h:30-34). */
typedef struct { void *data; size_t dataLength; } OrBuffer;

typedef struct or_coder or_coder;

or_coder *or_create(void);                          /* compress.c:48-56 */
void      or_destroy(or_coder *c);                  /* compress.c:58-66 */
size_t    or_compress(or_coder *c, const OrBuffer *bufs, size_t nbufs,
                      size_t in_limit, uint8_t *out, size_t out_limit);   /* compress.c:246-342 */
size_t    or_decompress(or_coder *c, const uint8_t *in, size_t in_limit,
                        uint8_t *out, size_t out_limit);                 /* compress.c:498-627 */

/* Batch helpers over a packed batch (packet i = in[in_off[i] .. +in_len[i]]).
 * out_len[i] receives the call's return value. Single thread, one context. */
void or_compress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                       size_t n, uint8_t *out, const uint64_t *out_off,
                       const uint32_t *out_cap, uint32_t *out_len);
void or_decompress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                         size_t n, uint8_t *out, const uint64_t *out_off,
                         const uint32_t *out_cap, uint32_t *out_len);

/* Batch digest, SURVEY.md §8c. */
uint32_t or_crc32(const OrBuffer *bufs, size_t nbufs);      /* packet.c:143-163 */
void or_crc32_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len, size_t n,
                    uint32_t *crc_out);
uint64_t or_fnv1a64_packets(const uint8_t *buf, const uint64_t *off, const uint32_t *len, size_t n);

#ifdef __cplusplus
}
#endif
#endif
