/* deferred_double.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A CPU test double for the four libenet_rc_amd entry points that
 * enet_amd/csrc/rc_deferred.c calls (enet_range_coder_create / _destroy and
 * enet_rc_datagram_{encode,decode}_batch_host), built on the oracle's
 * restatement of compress.c (oracle/rc_oracle.c) and the datagram framing of
 * oracle/pyoracle.py (datagram_encode / datagram_decode, protocol.c:1686-1718
 * and :1022-1091).  oracle/Makefile links it into _ref/loopback_deferred_cpu so
 * that the deferred-batch plumbing (queues, --wrap hooks, seeds, flag and
 * byte accounting) runs in live hosts on a machine without a GPU; the GPU
 * build (_ref/loopback_deferred) links the real library instead.
 */
#include <stdint.h>
#include <string.h>

#include "../../oracle/rc_oracle.h"

enum { MTU = 4096 };

const char *enet_rc_version(void) { return "cpu test double (oracle)"; }

void *enet_range_coder_create(void) { return or_create(); }
void enet_range_coder_destroy(void *c) { if (c) or_destroy((or_coder *) c); }

static size_t header_size(uint8_t b0, int checksum)
{
    return (size_t) ((b0 & 0x80) ? 4 : 2) + (checksum ? 4 : 0);
}

static uint32_t crc_of(const uint8_t *p, size_t n)
{
    OrBuffer b = { (void *) p, n };
    return or_crc32(&b, 1);
}

int enet_rc_datagram_encode_batch_host(void *ctx, const uint8_t *in, const uint64_t *in_off,
                                       const uint32_t *in_len, size_t n, int checksum, const uint32_t *seed,
                                       uint8_t *out, const uint64_t *out_off, uint32_t *out_len)
{
    static uint8_t tmp[MTU], packed[MTU];
    for (size_t i = 0; i < n; ++i) {
        const uint8_t *d = in + in_off[i];
        const size_t len = in_len[i];
        out_len[i] = 0;
        if (len < 2 || len > MTU || len < header_size(d[0], checksum)) continue;
        const size_t hs = header_size(d[0], checksum), L = len - hs;
        OrBuffer cmds = { (void *) (d + hs), L };
        const size_t c = L ? or_compress((or_coder *) ctx, &cmds, 1, L, packed, L) : 0;
        const int comp = c > 0 && c < L;
        memcpy(tmp, d, len);
        tmp[0] = (uint8_t) ((d[0] & ~0x40) | (comp ? 0x40 : 0));
        if (checksum) {
            const uint32_t s = seed ? seed[i] : 0;
            memcpy(tmp + hs - 4, &s, 4);
            const uint32_t crc = crc_of(tmp, len);
            memcpy(tmp + hs - 4, &crc, 4);
        }
        uint8_t *o = out + out_off[i];
        memcpy(o, tmp, hs);
        memcpy(o + hs, comp ? packed : d + hs, comp ? c : L);
        out_len[i] = (uint32_t) (hs + (comp ? c : L));
    }
    return 0;
}

int enet_rc_datagram_decode_batch_host(void *ctx, const uint8_t *in, const uint64_t *in_off,
                                       const uint32_t *in_len, size_t n, int checksum, const uint32_t *seed,
                                       uint8_t *out, const uint64_t *out_off, uint32_t *out_len)
{
    for (size_t i = 0; i < n; ++i) {
        const uint8_t *w = in + in_off[i];
        const size_t len = in_len[i];
        uint8_t *o = out + out_off[i];
        out_len[i] = 0;
        if (len < 2 || len < header_size(w[0], checksum)) continue;
        const size_t hs = header_size(w[0], checksum);
        size_t total;
        if (w[0] & 0x40) {
            const size_t r = or_decompress((or_coder *) ctx, w + hs, len - hs, o + hs, MTU - hs);
            if (r == 0 || r > MTU - hs) continue;
            memcpy(o, w, hs);
            total = hs + r;
        } else {
            if (len > MTU) continue;
            memcpy(o, w, len);
            total = len;
        }
        if (checksum) {
            uint32_t want, s = seed ? seed[i] : 0;
            memcpy(&want, o + hs - 4, 4);
            memcpy(o + hs - 4, &s, 4);
            if (crc_of(o, total) != want) continue;
        }
        out_len[i] = (uint32_t) total;
    }
    return 0;
}
