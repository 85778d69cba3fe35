/*
 * rc_host_internal.h -- what rc_multi.c uses of a coder context (rc_host.c).
 * Plain C, plain pointers.
 */
#ifndef ENET_RC_HOST_INTERNAL_H
#define ENET_RC_HOST_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

int rc_ctx_device(void *context);
void *rc_ctx_stream(void *context);
/* enet_rc_{compress,decompress}_batch_device / _host of one context */
int rc_ctx_run_device(void *context, int decompress, const uint8_t *in, const uint64_t *in_off,
                      const uint32_t *in_len, size_t n, uint32_t max_len, uint8_t *out,
                      const uint64_t *out_off, const uint32_t *out_cap, uint32_t *out_len, void *stream);
int rc_ctx_run_host(void *context, int decompress, const uint8_t *in, const uint64_t *in_off,
                    const uint32_t *in_len, size_t n, uint8_t *out, const uint64_t *out_off,
                    const uint32_t *out_cap, uint32_t *out_len);

/* rc_pack.hip's block-sum workspace of the context, for n packets (NULL: out of memory) */
uint64_t *rc_ctx_bsum(void *context, size_t n);

#endif
