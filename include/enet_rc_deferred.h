/*
 * enet_rc_deferred.h -- deferred-batch mode for a live ENet host
 * (SURVEY.md §8f row 1).
 *
 * protocol.c calls the compressor and checksum callbacks once per datagram,
 * synchronously (protocol.c:1686-1718 on send, :1052-1091 on receive), so a
 * GPU behind them pays a launch and two copies per ~1 KB.  The deferred mode
 * moves both callbacks out of protocol.c and into one GPU batch per pass:
 *
 *  - send: every datagram protocol.c hands to enet_socket_send (:1729) is
 *    queued uncompressed; at the end of the pass (enet_host_service /
 *    enet_host_flush returning, or enet_socket_wait about to block) the queue
 *    is compressed + checksummed by one enet_rc_datagram_encode_batch_host and
 *    sent by one enet_rc_socket_send_batch (sendmmsg);
 *  - receive: the first enet_socket_receive of a receive pass (:1244) drains
 *    the socket with one recvmmsg (up to 256 datagrams, the pass limit of
 *    :1238), decodes them with one enet_rc_datagram_decode_batch_host and then
 *    hands protocol.c one decoded datagram per call.
 *
 * The wire is byte-identical to a host running compress.c per datagram, so
 * deferred hosts talk to unmodified ENet peers (tests/test_integration.py).
 *
 * Hooking.  Nothing in the reference sources changes: the application links
 * the ENet objects statically (libenet.a without compress.o) together with
 * rc_deferred.c and libenet_rc_amd.so, and asks the linker to route six calls
 * through this module:
 *
 *   -Wl,--wrap=enet_socket_send,--wrap=enet_socket_receive,--wrap=enet_socket_wait
 *   -Wl,--wrap=enet_host_service,--wrap=enet_host_flush,--wrap=enet_host_destroy
 *
 * Sockets of hosts that are not attached pass straight through to unix.c.
 *
 * Threading follows ENet's: one host is serviced by one thread.  Attach and
 * detach hosts from one thread (the host table is not locked).  A batch that
 * fails on the GPU is lost like a dropped UDP datagram (the call returns -1).
 *
 * Requires enet/enet.h to be included first (ENetHost, ENetBuffer).
 */
#ifndef ENET_RC_DEFERRED_H
#define ENET_RC_DEFERRED_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Put `host` into deferred mode.  Replaces enet_host_compress_with_range_coder
 * (compress.c:637-650) plus, if `checksum`, `host->checksum = enet_crc32`
 * (enet.h:564): the host's compressor is removed (protocol.c then assembles
 * datagrams uncompressed) and host->checksum becomes
 * enet_rc_deferred_checksum, a placeholder that leaves the checksum field as
 * protocol.c seeded it; the batches compute the real enet_crc32.  Creates the
 * host's GPU coder context.  0 on success, -1 on failure (no GPU, too many
 * hosts, out of memory). */
int enet_rc_deferred_attach(ENetHost *host, int checksum);

/* Send what is queued for `host` now (one encode batch + one sendmmsg).
 * Called automatically by the wrapped enet_host_service / enet_host_flush /
 * enet_socket_wait.  Returns the number of datagrams sent, or -1. */
int enet_rc_deferred_flush(ENetHost *host);

/* Flush and leave deferred mode (the wrapped enet_host_destroy calls it).  The
 * host is left without compressor and checksum callbacks. */
void enet_rc_deferred_detach(ENetHost *host);

/* The placeholder checksum callback (ENetChecksumCallback, enet.h:338): it
 * returns the value already in the datagram's checksum field.  On send that is
 * the seed protocol.c put there (:1711-1716); on receive the decode batch has
 * already verified the CRC and left the seed there (:1079-1086). */
enet_uint32 enet_rc_deferred_checksum(const ENetBuffer *buffers, size_t bufferCount);

typedef struct {
    uint64_t send_batches, send_datagrams, send_compressed;
    uint64_t recv_batches, recv_datagrams, recv_dropped;
} enet_rc_deferred_stats;

/* Counters since attach; zeros for a host that is not attached. */
void enet_rc_deferred_get_stats(const ENetHost *host, enet_rc_deferred_stats *stats);

#ifdef __cplusplus
}
#endif

#endif
