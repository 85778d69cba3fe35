// Diagnostic: accuracy of v_rcp_f64 (raw, and after one Newton step) for
// every divisor b in [1, 65535]: the largest relative error |1 - b*r| and the
// smallest margin against what udiv16d needs (delta < 2^-49.1 * b and
// delta < 2^-33.1, rc_udiv.h).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>

__global__ void acc(double* out)
{
    const unsigned b = blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (b > 65535) return;
    const double db = b;
    const double r0 = __builtin_amdgcn_rcp(db);
    const double e0 = __builtin_fma(-db, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-db, r1, 1.0);
    out[2 * (b - 1)] = fabs(e0);
    out[2 * (b - 1) + 1] = fabs(e1);
}

int main()
{
    double* d; (void) hipMalloc(&d, 16 * 65535);
    acc<<<256, 256>>>(d);
    static double h[2 * 65535];
    (void) hipMemcpy(h, d, 16 * 65535, hipMemcpyDeviceToHost);
    for (int k = 0; k < 2; ++k) {
        double worst = 0, margin = 1e300; int wb = 0, mb = 0;
        for (int b = 1; b <= 65535; ++b) {
            const double e = h[2 * (b - 1) + k];
            if (e > worst) { worst = e; wb = b; }
            const double need = fmin(ldexp(1.0, -49) * 0.93 * b, ldexp(1.0, -34));
            const double m = e > 0 ? need / e : 1e300;
            if (m < margin) { margin = m; mb = b; }
        }
        printf("%s: max rel err %.3g (log2 %.2f) at b=%d; smallest margin need/err %.3g at b=%d\n",
               k ? "rcp+1 Newton" : "raw v_rcp_f64", worst, worst > 0 ? log2(worst) : -999.0, wb, margin, mb);
    }
    return 0;
}
