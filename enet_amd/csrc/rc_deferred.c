/*
 * rc_deferred.c -- deferred-batch mode for a live ENet host (SURVEY.md §8f
 * row 1); the contract and the link recipe are in include/enet_rc_deferred.h.
 *
 * Compiled against the application's enet/enet.h and linked next to the ENet
 * objects with -Wl,--wrap for the six functions below (it is not part of
 * libenet_rc_amd.so, which does not depend on enet.h).  Every GPU step goes
 * through the library's batch entry points; there is no CPU coding path here.
 *
 * Per attached host: a send queue of uncompressed datagrams in fixed
 * 4096-byte slots (ENET_PROTOCOL_MAXIMUM_MTU, protocol.h:13), and a receive
 * queue of decoded datagrams handed to protocol.c one per
 * enet_socket_receive call.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <enet/enet.h>

#include "enet_rc_amd.h"
#include "enet_rc_deferred.h"

int __real_enet_socket_send(ENetSocket, const ENetAddress *, const ENetBuffer *, size_t);
int __real_enet_socket_receive(ENetSocket, ENetAddress *, ENetBuffer *, size_t);
int __real_enet_socket_wait(ENetSocket, enet_uint32 *, enet_uint32);
int __real_enet_host_service(ENetHost *, ENetEvent *, enet_uint32);
void __real_enet_host_flush(ENetHost *);
void __real_enet_host_destroy(ENetHost *);

enum {
    SLOT = ENET_PROTOCOL_MAXIMUM_MTU,
    QCAP = 256,             /* datagrams per batch: protocol.c's receive-pass limit (:1238) */
    MAX_HOSTS = 64,
    FLAG_COMPRESSED = ENET_PROTOCOL_HEADER_FLAG_COMPRESSED >> 8,   /* bits of the first header byte */
    FLAG_SENT_TIME = ENET_PROTOCOL_HEADER_FLAG_SENT_TIME >> 8,
};

typedef struct {
    ENetHost *host;
    void *coder;
    int checksum;
    /* send queue */
    uint8_t *s_in, *s_out;
    uint64_t s_off[QCAP];
    uint32_t s_len[QCAP], s_seed[QCAP], s_out_len[QCAP];
    ENetAddress s_addr[QCAP];
    size_t s_n;
    /* receive queue */
    uint8_t *r_in, *r_out;
    uint64_t r_off[QCAP];
    uint32_t r_len[QCAP], r_seed[QCAP], r_out_len[QCAP];
    ENetAddress r_addr[QCAP];
    size_t r_n, r_next;
    enet_rc_deferred_stats st;
} Deferred;

static Deferred *g_hosts[MAX_HOSTS];

static Deferred *find_host(const ENetHost *h)
{
    for (int i = 0; i < MAX_HOSTS; ++i)
        if (g_hosts[i] && g_hosts[i]->host == h) return g_hosts[i];
    return NULL;
}

static Deferred *find_socket(ENetSocket s)
{
    for (int i = 0; i < MAX_HOSTS; ++i)
        if (g_hosts[i] && g_hosts[i]->host->socket == s) return g_hosts[i];
    return NULL;
}

/* offset of the checksum field: after the peerID word and, if SENT_TIME is
 * set, the sentTime word (protocol.c:1033, :1710) */
static size_t checksum_offset(const uint8_t *d)
{
    return (d[0] & FLAG_SENT_TIME) ? 4 : 2;
}

enet_uint32 enet_rc_deferred_checksum(const ENetBuffer *buffers, size_t bufferCount)
{
    if (bufferCount == 0 || buffers[0].dataLength < 2) return 0;
    const uint8_t *d = (const uint8_t *) buffers[0].data;
    const size_t at = checksum_offset(d);
    enet_uint32 v = 0;
    if (buffers[0].dataLength >= at + 4) memcpy(&v, d + at, 4);
    return v;
}

int enet_rc_deferred_attach(ENetHost *host, int checksum)
{
    if (!host || find_host(host)) return host ? 0 : -1;
    int slot = -1;
    for (int i = 0; i < MAX_HOSTS && slot < 0; ++i)
        if (!g_hosts[i]) slot = i;
    if (slot < 0) return -1;
    Deferred *d = (Deferred *) calloc(1, sizeof *d);
    if (!d) return -1;
    d->s_in = (uint8_t *) malloc((size_t) 4 * QCAP * SLOT);
    d->coder = enet_range_coder_create();
    if (!d->s_in || !d->coder) {
        free(d->s_in);
        enet_range_coder_destroy(d->coder);
        free(d);
        return -1;
    }
    d->s_out = d->s_in + (size_t) QCAP * SLOT;
    d->r_in = d->s_out + (size_t) QCAP * SLOT;
    d->r_out = d->r_in + (size_t) QCAP * SLOT;
    for (size_t i = 0; i < QCAP; ++i) d->s_off[i] = d->r_off[i] = i * SLOT;
    d->host = host;
    d->checksum = checksum != 0;
    enet_host_compress(host, NULL);                      /* host.c:294-304: no per-datagram coder */
    host->checksum = d->checksum ? enet_rc_deferred_checksum : NULL;
    g_hosts[slot] = d;
    return 0;
}

int enet_rc_deferred_flush(ENetHost *host)
{
    Deferred *d = find_host(host);
    if (!d || d->s_n == 0) return 0;
    const size_t n = d->s_n;
    d->s_n = 0;
    if (enet_rc_datagram_encode_batch_host(d->coder, d->s_in, d->s_off, d->s_len, n, d->checksum,
                                           d->s_seed, d->s_out, d->s_off, d->s_out_len) != 0)
        return -1;
    /* protocol.c counted the uncompressed lengths (:1737); count the wire bytes */
    for (size_t i = 0; i < n; ++i) {
        host->totalSentData -= d->s_len[i] - d->s_out_len[i];
        d->st.send_compressed += d->s_out_len[i] < d->s_len[i];
    }
    d->st.send_batches += 1;
    d->st.send_datagrams += n;
    return enet_rc_socket_send_batch(host->socket, d->s_out, d->s_off, d->s_out_len, d->s_addr, n);
}

void enet_rc_deferred_detach(ENetHost *host)
{
    for (int i = 0; i < MAX_HOSTS; ++i) {
        Deferred *d = g_hosts[i];
        if (!d || d->host != host) continue;
        enet_rc_deferred_flush(host);
        g_hosts[i] = NULL;
        host->checksum = NULL;
        enet_range_coder_destroy(d->coder);
        free(d->s_in);
        free(d);
    }
}

void enet_rc_deferred_get_stats(const ENetHost *host, enet_rc_deferred_stats *stats)
{
    const Deferred *d = find_host(host);
    if (d) *stats = d->st;
    else memset(stats, 0, sizeof *stats);
}

/* ------------------------------------------------------------- wrapped calls */

int __wrap_enet_socket_send(ENetSocket s, const ENetAddress *address, const ENetBuffer *buffers,
                            size_t bufferCount)
{
    Deferred *d = find_socket(s);
    if (!d) return __real_enet_socket_send(s, address, buffers, bufferCount);
    if (d->s_n == QCAP && enet_rc_deferred_flush(d->host) < 0) return -1;
    uint8_t *p = d->s_in + d->s_n * SLOT;
    size_t len = 0;
    for (size_t b = 0; b < bufferCount; ++b) {
        if (len + buffers[b].dataLength > SLOT) return -1;    /* protocol.c never exceeds the MTU */
        memcpy(p + len, buffers[b].data, buffers[b].dataLength);
        len += buffers[b].dataLength;
    }
    /* the seed protocol.c put in the checksum field (:1711-1716) is still
     * there: enet_rc_deferred_checksum returned it unchanged */
    uint32_t seed = 0;
    if (d->checksum && len >= 2 && len >= checksum_offset(p) + 4) memcpy(&seed, p + checksum_offset(p), 4);
    d->s_len[d->s_n] = (uint32_t) len;
    d->s_seed[d->s_n] = seed;
    d->s_addr[d->s_n] = address ? *address : (ENetAddress) { 0, 0 };
    ++d->s_n;
    return (int) len;
}

/* one recvmmsg + one decode batch; returns the number received or -1 */
static int refill(Deferred *d)
{
    ENetHost *h = d->host;
    const int got = enet_rc_socket_receive_batch(h->socket, d->r_in, SLOT, QCAP, d->r_len, d->r_addr);
    if (got <= 0) return got;
    for (int i = 0; i < got; ++i) {
        /* seed of protocol.c:1079: the addressed peer's connectID, 0 for
         * peerID 0xFFF (or an index protocol.c rejects at :1040) */
        const uint8_t *p = d->r_in + (size_t) i * SLOT;
        uint32_t seed = 0;
        if (d->r_len[i] >= 2) {
            const unsigned pid = (((unsigned) p[0] << 8) | p[1]) & ENET_PROTOCOL_MAXIMUM_PEER_ID;
            if (pid != ENET_PROTOCOL_MAXIMUM_PEER_ID && pid < h->peerCount) seed = h->peers[pid].connectID;
        }
        d->r_seed[i] = seed;
    }
    if (enet_rc_datagram_decode_batch_host(d->coder, d->r_in, d->r_off, d->r_len, (size_t) got, d->checksum,
                                           d->r_seed, d->r_out, d->r_off, d->r_out_len) != 0)
        return -1;
    d->r_n = (size_t) got;
    d->r_next = 0;
    d->st.recv_batches += 1;
    d->st.recv_datagrams += (uint64_t) got;
    return got;
}

int __wrap_enet_socket_receive(ENetSocket s, ENetAddress *address, ENetBuffer *buffers, size_t bufferCount)
{
    Deferred *d = find_socket(s);
    if (!d) return __real_enet_socket_receive(s, address, buffers, bufferCount);
    if (bufferCount != 1) return -1;                     /* protocol.c passes one buffer (:1240-1247) */
    for (;;) {
        if (d->r_next == d->r_n) {
            const int got = refill(d);
            if (got <= 0) return got;                    /* 0: nothing queued, as unix.c:500-501 */
        }
        const size_t i = d->r_next++;
        const uint32_t n = d->r_out_len[i];
        if (n == 0 || n > buffers[0].dataLength) {       /* a datagram protocol.c would drop */
            d->st.recv_dropped += 1;
            continue;
        }
        uint8_t *out = (uint8_t *) buffers[0].data;
        memcpy(out, d->r_out + i * SLOT, n);
        out[0] &= (uint8_t) ~FLAG_COMPRESSED;            /* already decompressed (:1052-1070) */
        if (address) *address = d->r_addr[i];
        /* protocol.c adds the returned length (:1256); count the wire bytes */
        d->host->totalReceivedData += d->r_len[i] - n;
        return (int) n;
    }
}

int __wrap_enet_socket_wait(ENetSocket s, enet_uint32 *condition, enet_uint32 timeout)
{
    Deferred *d = find_socket(s);
    if (d) {
        if (enet_rc_deferred_flush(d->host) < 0) return -1;
        /* datagrams already pulled off the socket are pending receives */
        if (d->r_next < d->r_n && (*condition & ENET_SOCKET_WAIT_RECEIVE)) {
            *condition = ENET_SOCKET_WAIT_RECEIVE;
            return 0;
        }
    }
    return __real_enet_socket_wait(s, condition, timeout);
}

int __wrap_enet_host_service(ENetHost *host, ENetEvent *event, enet_uint32 timeout)
{
    const int r = __real_enet_host_service(host, event, timeout);
    if (enet_rc_deferred_flush(host) < 0) return -1;
    return r;
}

void __wrap_enet_host_flush(ENetHost *host)
{
    __real_enet_host_flush(host);
    enet_rc_deferred_flush(host);
}

void __wrap_enet_host_destroy(ENetHost *host)
{
    enet_rc_deferred_detach(host);
    __real_enet_host_destroy(host);
}
