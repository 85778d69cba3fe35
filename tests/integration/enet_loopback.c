/* enet_loopback.c -- live ENet hosts over 127.0.0.1 with the range coder
 * enabled (enet_host_compress_with_range_coder, enet.h:574), used to show the
 * drop-in: the same source is linked once against the reference library
 * (compress.c inside) and once against the reference library WITHOUT
 * compress.c plus libenet_rc_amd.so (oracle/Makefile, targets loopback_ref /
 * loopback_amd).  Peers of either build talk to each other, so the GPU coder's
 * datagrams are decoded by compress.c and vice versa (tests/test_integration.py).
 *
 *   enet_loopback both   PORT COUNT   two hosts in this process
 *   enet_loopback server PORT COUNT   echo COUNT packets back, then exit
 *   enet_loopback client PORT COUNT   send COUNT packets, check the echoes
 *   enet_loopback fan PORT COUNT K    K peers between two hosts in this process
 *
 * Payloads are low-entropy "game state" records so that datagrams compress
 * (protocol.c:1696 only sends the compressed form when it is smaller).
 * Prints one JSON line; exit status 0 iff every echo matched. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <enet/enet.h>

extern const char *enet_rc_version(void) __attribute__((weak));

#ifdef ENET_LOOPBACK_DEFERRED
/* loopback_deferred: the hosts run in deferred-batch mode (rc_deferred.c,
 * include/enet_rc_deferred.h): one GPU batch per send / receive pass */
#include "enet_rc_deferred.h"
#endif

static uint64_t mix(uint64_t *s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* packet k: 40..1300 bytes of 24-B entity records with small deltas */
static size_t make_payload(uint32_t k, uint8_t *p)
{
    uint64_t s = 0x454E4554ull + k;
    size_t n = 40 + (size_t) (mix(&s) % 1261);
    uint16_t pos[3] = { (uint16_t) mix(&s), (uint16_t) mix(&s), (uint16_t) mix(&s) };
    for (size_t i = 0; i < n; ++i) {
        size_t f = i % 24;
        if (f == 0) {
            for (int a = 0; a < 3; ++a) pos[a] = (uint16_t) (pos[a] + (int) (mix(&s) % 7) - 3);
            p[i] = (uint8_t) (i / 24 + k);
        } else if (f == 1) p[i] = 1;
        else if (f >= 2 && f < 8) p[i] = (uint8_t) (pos[(f - 2) / 2] >> (8 * (f & 1)));
        else if (f == 8) p[i] = (uint8_t) (mix(&s) % 4);
        else if (f == 11) p[i] = 100;
        else p[i] = 0;
    }
    return n;
}

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

/* ENET_LOOPBACK_DUMP=path: every received datagram (as on the wire) and the
 * checksum seed protocol.c would use for it (:1079) are appended to path as
 * JSON lines, through the host's intercept hook (protocol.c:1259-1274); used
 * by tests/golden/make_dgram_golden.py to pin the datagram framing to real
 * ENet traffic.  ENET_LOOPBACK_CHECKSUM=1 enables enet_crc32 (enet.h:564). */
static FILE *g_dump;

static int ENET_CALLBACK dump_datagram(ENetHost *host, ENetEvent *event)
{
    (void) event;
    const enet_uint8 *d = host->receivedData;
    size_t n = host->receivedDataLength;
    enet_uint32 seed = 0;
    if (n >= 2) {
        unsigned pid = (((unsigned) d[0] << 8) | d[1]) & 0x0FFFu;
        if (pid != 0x0FFFu && pid < host->peerCount) seed = host->peers[pid].connectID;
    }
    fprintf(g_dump, "{\"checksum\": %d, \"seed\": %u, \"wire\": \"", host->checksum != NULL, seed);
    for (size_t i = 0; i < n; ++i) fprintf(g_dump, "%02x", d[i]);
    fprintf(g_dump, "\"}\n");
    return 0;   /* protocol.c goes on handling it */
}

static ENetHost *mk_host(const ENetAddress *a, size_t peers, int *rc)
{
    ENetHost *h = enet_host_create(a, peers, 2, 0, 0);
    if (!h) { fprintf(stderr, "enet_host_create failed\n"); exit(2); }
    const char *ck = getenv("ENET_LOOPBACK_CHECKSUM");
    const int checksum = ck && atoi(ck);
#ifdef ENET_LOOPBACK_DEFERRED
    *rc = enet_rc_deferred_attach(h, checksum);
    if (*rc != 0) { fprintf(stderr, "enet_rc_deferred_attach = %d\n", *rc); exit(3); }
#else
    *rc = enet_host_compress_with_range_coder(h);
    if (*rc != 0) { fprintf(stderr, "enet_host_compress_with_range_coder = %d\n", *rc); exit(3); }
    if (checksum) h->checksum = enet_crc32;
#endif
    const char *dp = getenv("ENET_LOOPBACK_DUMP");
    if (dp) {
        if (!g_dump) g_dump = fopen(dp, "w");
        if (!g_dump) { fprintf(stderr, "cannot open %s\n", dp); exit(2); }
        h->intercept = dump_datagram;
    }
    return h;
}

typedef struct {
    ENetHost *host;
    ENetPeer *peer;
    int is_client, connected, done;
    uint32_t count, sent, got, bad;
    uint64_t raw_bytes;
} Side;

static void pump(Side *s)
{
    ENetEvent ev;
    while (enet_host_service(s->host, &ev, 0) > 0) {
        switch (ev.type) {
        case ENET_EVENT_TYPE_CONNECT:
            s->connected = 1;
            s->peer = ev.peer;
            break;
        case ENET_EVENT_TYPE_RECEIVE: {
            if (s->is_client) {
                uint8_t want[1400];
                size_t n = make_payload(s->got, want);
                if (ev.packet->dataLength != n || memcmp(ev.packet->data, want, n) != 0) ++s->bad;
                ++s->got;
                if (s->got == s->count) s->done = 1;
            } else {                       /* echo */
                ENetPacket *e = enet_packet_create(ev.packet->data, ev.packet->dataLength,
                                                   ENET_PACKET_FLAG_RELIABLE);
                enet_peer_send(ev.peer, 0, e);
                s->raw_bytes += ev.packet->dataLength;
                if (++s->got == s->count) s->done = 1;
            }
            enet_packet_destroy(ev.packet);
            break;
        }
        case ENET_EVENT_TYPE_DISCONNECT:
            s->connected = 0;
            break;
        default:
            break;
        }
    }
    if (s->is_client && s->connected) {
        /* keep a window of packets in flight */
        while (s->sent < s->count && s->sent < s->got + 64) {
            uint8_t buf[1400];
            size_t n = make_payload(s->sent, buf);
            enet_peer_send(s->peer, 0, enet_packet_create(buf, n, ENET_PACKET_FLAG_RELIABLE));
            s->raw_bytes += n;
            ++s->sent;
        }
        enet_host_flush(s->host);
    }
}

static void print_stats(const char *name, ENetHost *h)
{
#ifdef ENET_LOOPBACK_DEFERRED
    enet_rc_deferred_stats st;
    enet_rc_deferred_get_stats(h, &st);
    printf("\"%s\": {\"send_batches\": %llu, \"send_datagrams\": %llu, \"send_compressed\": %llu, "
           "\"recv_batches\": %llu, \"recv_datagrams\": %llu, \"recv_dropped\": %llu}", name,
           (unsigned long long) st.send_batches, (unsigned long long) st.send_datagrams,
           (unsigned long long) st.send_compressed, (unsigned long long) st.recv_batches,
           (unsigned long long) st.recv_datagrams, (unsigned long long) st.recv_dropped);
#else
    (void) h;
    printf("\"%s\": null", name);
#endif
}

/* fan PORT COUNT K: a server host and a client host in this process, K peers
 * between them; every client peer keeps a window of packets in flight and
 * checks the echoes.  With K peers, one send pass of either host assembles up
 * to K datagrams -- what a deferred host turns into one GPU batch. */
typedef struct { uint32_t sent, got, bad; int connected; } Lane;

static int run_fan(const ENetAddress *addr, uint32_t count, uint32_t k)
{
    int rc = 0;
    ENetHost *sv = mk_host(addr, k, &rc), *cl = mk_host(NULL, k, &rc);
    Lane *ln = (Lane *) calloc(k, sizeof *ln);
    for (uint32_t i = 0; i < k; ++i) {
        ENetPeer *p = enet_host_connect(cl, addr, 2, i);
        if (!p) return 4;
        p->data = &ln[i];
    }
    uint32_t done = 0, echoed = 0;
    uint64_t raw = 0;
    double t0 = now(), deadline = t0 + 60.0;
    while (now() < deadline && done < k) {
        ENetEvent ev;
        while (enet_host_service(sv, &ev, 0) > 0) {
            if (ev.type != ENET_EVENT_TYPE_RECEIVE) continue;
            enet_peer_send(ev.peer, 0, enet_packet_create(ev.packet->data, ev.packet->dataLength,
                                                          ENET_PACKET_FLAG_RELIABLE));
            ++echoed;
            enet_packet_destroy(ev.packet);
        }
        while (enet_host_service(cl, &ev, 0) > 0) {
            Lane *l = (Lane *) ev.peer->data;
            if (ev.type == ENET_EVENT_TYPE_CONNECT) l->connected = 1;
            if (ev.type != ENET_EVENT_TYPE_RECEIVE) continue;
            uint8_t want[1400];
            size_t n = make_payload((uint32_t) (l - ln) * count + l->got, want);
            if (ev.packet->dataLength != n || memcmp(ev.packet->data, want, n) != 0) ++l->bad;
            if (++l->got == count) ++done;
            enet_packet_destroy(ev.packet);
        }
        for (uint32_t i = 0; i < k; ++i) {
            Lane *l = &ln[i];
            while (l->connected && l->sent < count && l->sent < l->got + 8) {
                uint8_t buf[1400];
                size_t n = make_payload(i * count + l->sent, buf);
                enet_peer_send(&cl->peers[i], 0, enet_packet_create(buf, n, ENET_PACKET_FLAG_RELIABLE));
                raw += n;
                ++l->sent;
            }
        }
        enet_host_flush(cl);
        enet_host_flush(sv);
    }
    uint32_t got = 0, bad = 0;
    for (uint32_t i = 0; i < k; ++i) { got += ln[i].got; bad += ln[i].bad; }
    const int ok = done == k && bad == 0;
    printf("{\"role\": \"fan\", \"coder\": \"%s\", \"peers\": %u, \"packets\": %u, \"received\": %u, "
           "\"echoed\": %u, \"mismatches\": %u, \"payload_bytes\": %llu, \"seconds\": %.3f, ",
           enet_rc_version ? enet_rc_version() : "reference compress.c", k, k * count, got, echoed, bad,
           (unsigned long long) raw, now() - t0);
    print_stats("server", sv);
    printf(", ");
    print_stats("client", cl);
    printf(", \"ok\": %s}\n", ok ? "true" : "false");
    fflush(stdout);
    enet_host_destroy(cl);
    enet_host_destroy(sv);
    free(ln);
    return ok ? 0 : 1;
}

int main(int argc, char **argv)
{
    if (argc < 4) { fprintf(stderr, "usage: %s both|server|client|fan PORT COUNT [PEERS]\n", argv[0]); return 2; }
    const char *role = argv[1];
    const int both = !strcmp(role, "both"), server = both || !strcmp(role, "server"),
              client = both || !strcmp(role, "client");
    uint32_t count = (uint32_t) strtoul(argv[3], NULL, 10);
    if (enet_initialize() != 0) return 2;
    ENetAddress addr;
    enet_address_set_host(&addr, "127.0.0.1");
    addr.port = (enet_uint16) atoi(argv[2]);
    if (!strcmp(role, "fan")) {
        const int r = run_fan(&addr, count, argc > 4 ? (uint32_t) strtoul(argv[4], NULL, 10) : 16);
        enet_deinitialize();
        return r;
    }

    Side sv, cl;
    memset(&sv, 0, sizeof sv);
    memset(&cl, 0, sizeof cl);
    int rc = 0;
    if (server) { sv.host = mk_host(&addr, 4, &rc); sv.count = count; }
    if (client) {
        cl.host = mk_host(NULL, 4, &rc);
        cl.is_client = 1;
        cl.count = count;
        cl.peer = enet_host_connect(cl.host, &addr, 2, 0);
        if (!cl.peer) return 4;
    }
    double t0 = now(), deadline = t0 + 60.0;
    while (now() < deadline) {
        if (server) pump(&sv);
        if (client) pump(&cl);
        if ((!server || sv.done) && (!client || cl.done)) break;
        if (!both) {                     /* block briefly in the single-role modes */
            ENetHost *h = server ? sv.host : cl.host;
            enet_host_flush(h);
            struct timespec ts = { 0, 200000 };
            nanosleep(&ts, NULL);
        }
    }
    /* let the last echoes / acks leave */
    for (int i = 0; i < 50; ++i) {
        if (server) { pump(&sv); enet_host_flush(sv.host); }
        if (client) { pump(&cl); enet_host_flush(cl.host); }
        struct timespec ts = { 0, 2000000 };
        nanosleep(&ts, NULL);
    }
    Side *s = client ? &cl : &sv;
    int ok = s->done && s->bad == 0;
    printf("{\"role\": \"%s\", \"coder\": \"%s\", \"packets\": %u, \"received\": %u, \"mismatches\": %u, "
           "\"payload_bytes\": %llu, \"wire_bytes_sent\": %u, \"seconds\": %.3f, \"ok\": %s}\n",
           role, enet_rc_version ? enet_rc_version() : "reference compress.c", count, s->got, s->bad,
           (unsigned long long) s->raw_bytes, s->host->totalSentData, now() - t0, ok ? "true" : "false");
    fflush(stdout);
    if (server) enet_host_destroy(sv.host);
    if (client) enet_host_destroy(cl.host);
    enet_deinitialize();
    if (g_dump) fclose(g_dump);
    return ok ? 0 : 1;
}
