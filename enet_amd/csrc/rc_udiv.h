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
#else
inline uint32_t udiv(uint32_t a, uint32_t b) { return a / b; }
#endif
