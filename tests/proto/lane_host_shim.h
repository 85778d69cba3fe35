/* TEST ONLY: lets tests/proto/lane_host.cpp compile the per-lane logic of
 * enet_amd/csrc/rc_lane3.hip and rc_dec6.hip for the
 * host, to check it against the golden fixtures without a GPU.  Never part of
 * the product library. */
#pragma once
#include <stdint.h>
#include <algorithm>
#define __device__
#define __host__
#define __forceinline__ inline
struct uint4 { uint32_t x, y, z, w; };
struct uint2 { uint32_t x, y; };
inline uint2 make_uint2(uint32_t a, uint32_t b) { return uint2{a, b}; }
inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return uint4{a, b, c, d}; }
inline uint32_t host_sad_u8(uint32_t a, uint32_t b, uint32_t acc)
{
    for (int i = 0; i < 4; ++i) {
        int x = (a >> (8 * i)) & 0xFF, y = (b >> (8 * i)) & 0xFF;
        acc += (uint32_t) (x > y ? x - y : y - x);
    }
    return acc;
}
#define __builtin_amdgcn_sad_u8 host_sad_u8
#define __builtin_amdgcn_s_waitcnt(x) ((void) 0)
#define __builtin_amdgcn_sched_barrier(x) ((void) 0)
#define __builtin_amdgcn_ballot_w64(p) ((unsigned long long) ((p) ? 1 : 0))
using std::min;
using std::max;
inline uint32_t atomicAdd(uint32_t* p, uint32_t v) { uint32_t o = *p; *p += v; return o; }
inline uint32_t atomicOr(uint32_t* p, uint32_t v) { uint32_t o = *p; *p |= v; return o; }

inline uint32_t host_udot4(uint32_t a, uint32_t b, uint32_t c, bool)
{
    for (int i = 0; i < 4; ++i) c += ((a >> (8 * i)) & 0xFF) * ((b >> (8 * i)) & 0xFF);
    return c;
}
inline uint32_t host_perm(uint32_t s0, uint32_t s1, uint32_t sel)
{
    const uint64_t v = ((uint64_t) s0 << 32) | s1;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t b = (sel >> (8 * i)) & 0xFF;
        const uint32_t x = b < 8 ? (uint32_t) ((v >> (8 * b)) & 0xFF) : (b == 0x0C ? 0u : 0xFFu);
        r |= x << (8 * i);
    }
    return r;
}
inline uint32_t host_alignbyte(uint32_t s0, uint32_t s1, uint32_t s2)
{
    return (uint32_t) ((((uint64_t) s0 << 32) | s1) >> (8 * (s2 & 3)));
}
#define __builtin_amdgcn_udot4 host_udot4
#define __builtin_amdgcn_perm host_perm
#define __builtin_amdgcn_alignbyte host_alignbyte
