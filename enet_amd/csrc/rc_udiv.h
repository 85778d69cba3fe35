// rc_udiv.h -- exact 32-bit unsigned division for the coder kernels.
//
// The compiler's u32 division is ~20 dependent instructions with five
// quarter-rate multiplies.  Here a double-precision reciprocal refined by two
// Newton steps (relative error < 2^-52) gives a * (1/b) within (a/b) * 2^-51
// of a/b, which is below 1/b for every a < 2^51: truncation is therefore
// exact, except when a/b is an integer approached from below, which one
// multiply-back corrects.  Valid for all a and all b >= 1.
// (tests/test_udiv.py checks it on the GPU against integer division.)
#pragma once
#include <stdint.h>

#ifndef RC_LANE_HOST_TEST
__device__ __forceinline__ uint32_t udiv(uint32_t a, uint32_t b)
{
    const double db = static_cast<double>(b);
    double r = __builtin_amdgcn_rcp(db);
    double e = __builtin_fma(-db, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-db, r, 1.0);
    r = __builtin_fma(r, e, r);
    uint32_t q = static_cast<uint32_t>(static_cast<double>(a) * r);
    q += (a - q * b >= b) ? 1u : 0u;
    return q;
}

// The coder's divisions by a context total (b < 2^16) in single precision:
// a first quotient from a float reciprocal (within 2^10 / b + 1 of a / b), a
// second one from the remainder (|r| < 2^17, exact in float), then one
// remainder check.  Exact for all a and 1 <= b <= 65535 (tests/test_udiv.py).
__device__ __forceinline__ uint32_t udiv16(uint32_t a, uint32_t b)
{
    const float rb = __builtin_amdgcn_rcpf(static_cast<float>(b));
    uint32_t q = static_cast<uint32_t>(static_cast<float>(a) * rb);
    const int32_t r = static_cast<int32_t>(a - q * b);
    q += static_cast<int32_t>(static_cast<float>(r) * rb);
    const int32_t r2 = static_cast<int32_t>(a - q * b);
    q += r2 < 0 ? 0xFFFFFFFFu : (r2 >= static_cast<int32_t>(b) ? 1u : 0u);
    return q;
}

// udiv16 with the reciprocal of b already at hand (rb = rcp(float(b)),
// computed off the dependency chain): the same two-step quotient.
__device__ __forceinline__ uint32_t udiv16r(uint32_t a, uint32_t b, float rb)
{
    uint32_t q = static_cast<uint32_t>(static_cast<float>(a) * rb);
    const int32_t r = static_cast<int32_t>(a - q * b);
    q += static_cast<int32_t>(static_cast<float>(r) * rb);
    const int32_t r2 = static_cast<int32_t>(a - q * b);
    q += r2 < 0 ? 0xFFFFFFFFu : (r2 >= static_cast<int32_t>(b) ? 1u : 0u);
    return q;
}
__device__ __forceinline__ float rcp16(uint32_t b) { return __builtin_amdgcn_rcpf(static_cast<float>(b)); }

// 1/b in double precision for 1 <= b <= 65535: v_rcp_f64 (relative error up
// to 2^-24.4) and one Newton step, relative error < 2^-48.7 for every such b
// (measured exhaustively, tools/mb/rcpacc.hip) -- at least 89x inside what
// udiv16d needs (below b * 2^-49 * 0.9375 and below 2^-33).
__device__ __forceinline__ double rcp64(uint32_t b)
{
    const double db = static_cast<double>(b);
    const double r = __builtin_amdgcn_rcp(db);
    return __builtin_fma(r, __builtin_fma(-db, r, 1.0), r);
}

// floor(a / b) for 1 <= b <= 65535 with rb = rcp64(b): three dependent
// instructions (convert, fma, convert; ~20 cycles against ~90 for udiv16r,
// tools/mb/chainlat.hip).  With rb = (1/b)(1 + d), a * rb is within
// (2^32 / b) d of a/b and the fma's rounding adds < 2^-21, so a/b + 2^-17 is
// computed at least at the integer a/b when it is one (needs (2^32/b) d +
// 2^-21 < 2^-17: d < b * 2^-49 * 0.9375), and below the next integer
// otherwise, the fraction of a/b being at most 1 - 1/b (needs 2^-17 + 2^-21 +
// (2^32/b) d < 1/b: d < 2^-33 for b <= 65535).  GPU-checked over random and
// boundary pairs (tests/test_udiv.py, chainlat's sweep).
__device__ __forceinline__ uint32_t udiv16d(uint32_t a, uint32_t, double rb)
{
    return static_cast<uint32_t>(__builtin_fma(static_cast<double>(a), rb, 0x1p-17));
}

// floor(a / b) & 0xFFFF for any b >= 1 (the decoder's READ, compress.c:352):
// single precision while the quotient is below 2^16 (every valid stream:
// code - low < range), udiv otherwise.
__device__ __forceinline__ uint32_t udiv_lo16(uint32_t a, uint32_t b)
{
    const float qf = static_cast<float>(a) * __builtin_amdgcn_rcpf(static_cast<float>(b));
    uint32_t q = static_cast<uint32_t>(qf);
    const uint64_t m = static_cast<uint64_t>(q) * b;
    q += m > a ? 0xFFFFFFFFu : (a - static_cast<uint32_t>(m) >= b ? 1u : 0u);
    const bool wide = qf >= 65000.0f;
    if (__builtin_amdgcn_ballot_w64(wide) != 0) q = wide ? udiv(a, b) : q;
    return q & 0xFFFF;
}
#else
// (host test build: a quotient by 0 -- computed and discarded by lanes a
// step does not concern, as on the GPU, where it does not trap -- reads 0)
inline uint32_t udiv(uint32_t a, uint32_t b) { return b ? a / b : 0u; }
inline uint32_t udiv16(uint32_t a, uint32_t b) { return b ? a / b : 0u; }
inline uint32_t udiv16r(uint32_t a, uint32_t b, float) { return b ? a / b : 0u; }
inline float rcp16(uint32_t b) { return 1.0f / static_cast<float>(b); }
inline double rcp64(uint32_t b) { return 1.0 / static_cast<double>(b); }
inline uint32_t udiv16d(uint32_t a, uint32_t b, double) { return b ? a / b : 0u; }
inline uint32_t udiv_lo16(uint32_t a, uint32_t b) { return b ? (a / b) & 0xFFFF : 0u; }
#endif
