/*
 * rc_io.c -- batched UDP datagram I/O for the GPU coder.
 *
 * enet_socket_receive / enet_socket_send (unix.c:440-528) move one datagram
 * per system call.  These move up to `max` per call with recvmmsg / sendmmsg,
 * straight into / out of caller memory -- typically the pinned staging that
 * the datagram batch calls copy to the GPU from, so a receive pass (up to 256
 * datagrams, protocol.c:1238) costs one system call and one H2D copy.
 *
 * Same address convention as the reference: ENetAddress.host is the IPv4
 * address in network byte order, .port in host byte order (unix.c:455-459,
 * :513-516).  Plain host code; no HIP.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <netinet/in.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/uio.h>

#include "enet_rc_amd.h"

#define IO_CHUNK 256u   /* datagrams per system call */

int enet_rc_socket_receive_batch(int socket, uint8_t *buf, size_t slot_bytes, size_t max,
                                 uint32_t *lengths, ENetAddress *addresses)
{
    if (socket < 0 || !buf || !lengths || slot_bytes == 0) return -1;
    struct mmsghdr msgs[IO_CHUNK];
    struct iovec iov[IO_CHUNK];
    struct sockaddr_in sin[IO_CHUNK];
    size_t got = 0;
    while (got < max) {
        const unsigned k = (unsigned) (max - got < IO_CHUNK ? max - got : IO_CHUNK);
        memset(msgs, 0, k * sizeof msgs[0]);
        for (unsigned j = 0; j < k; ++j) {
            iov[j].iov_base = buf + (got + j) * slot_bytes;
            iov[j].iov_len = slot_bytes;
            msgs[j].msg_hdr.msg_iov = &iov[j];
            msgs[j].msg_hdr.msg_iovlen = 1;
            msgs[j].msg_hdr.msg_name = &sin[j];
            msgs[j].msg_hdr.msg_namelen = sizeof sin[j];
        }
        int r = recvmmsg(socket, msgs, k, MSG_DONTWAIT, NULL);
        if (r < 0) {
            if (errno == EWOULDBLOCK || errno == EAGAIN) break;      /* unix.c:500-501 */
            if (errno == EINTR) continue;                            /* unix.c:502-504: retry */
            return got ? (int) got : -1;
        }
        for (int j = 0; j < r; ++j) {
            /* a truncated datagram is skipped by the reference (unix.c:509-512):
             * keep its slot with length 0 so that indices stay aligned */
            lengths[got + j] = (msgs[j].msg_hdr.msg_flags & MSG_TRUNC) ? 0u : msgs[j].msg_len;
            if (addresses) {
                addresses[got + j].host = (enet_uint32) sin[j].sin_addr.s_addr;
                addresses[got + j].port = ntohs(sin[j].sin_port);
            }
        }
        got += (size_t) r;
        if ((unsigned) r < k) break;   /* the queue is drained */
    }
    return (int) got;
}

int enet_rc_socket_send_batch(int socket, const uint8_t *buf, const uint64_t *off, const uint32_t *len,
                              const ENetAddress *addresses, size_t n)
{
    if (socket < 0 || !buf || !off || !len) return -1;
    struct mmsghdr msgs[IO_CHUNK];
    struct iovec iov[IO_CHUNK];
    struct sockaddr_in sin[IO_CHUNK];
    size_t sent = 0;
    while (sent < n) {
        const unsigned k = (unsigned) (n - sent < IO_CHUNK ? n - sent : IO_CHUNK);
        memset(msgs, 0, k * sizeof msgs[0]);
        for (unsigned j = 0; j < k; ++j) {
            iov[j].iov_base = (void *) (buf + off[sent + j]);
            iov[j].iov_len = len[sent + j];
            msgs[j].msg_hdr.msg_iov = &iov[j];
            msgs[j].msg_hdr.msg_iovlen = 1;
            if (addresses) {                                         /* unix.c:449-460 */
                memset(&sin[j], 0, sizeof sin[j]);
                sin[j].sin_family = AF_INET;
                sin[j].sin_port = htons(addresses[sent + j].port);
                sin[j].sin_addr.s_addr = addresses[sent + j].host;
                msgs[j].msg_hdr.msg_name = &sin[j];
                msgs[j].msg_hdr.msg_namelen = sizeof sin[j];
            }
        }
        int r = sendmmsg(socket, msgs, k, MSG_NOSIGNAL);
        if (r < 0) {
            if (errno == EWOULDBLOCK || errno == EAGAIN) break;      /* unix.c:467-469 */
            if (errno == EINTR) continue;
            return sent ? (int) sent : -1;
        }
        sent += (size_t) r;
        if ((unsigned) r < k) break;
    }
    return (int) sent;
}
