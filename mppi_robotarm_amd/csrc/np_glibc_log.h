// np_glibc_log.h — the natural logarithm exactly as NumPy's legacy Gaussian gets it.
//
// NumPy's legacy_gauss (the reference's draw, control.py:163, np.random.multivariate_normal on the legacy
// global RandomState) computes f = sqrt(-2 log(r2) / r2) with the C library's log.  On this image that is
// glibc 2.35's log, whose x86-64 build dispatches (ifunc) to a variant compiled with FMA on CPUs that have it
// (every host this runs on): the table-driven algorithm of glibc >= 2.28 (ARM optimized-routines, 128
// subintervals, degree-5 correction polynomial; a separate degree-11 polynomial near 1).  Its result is not
// always the correctly rounded one (ULP error up to ~0.52), so an exact device draw must evaluate the SAME
// operations on the SAME constants: this function is that sequence — every fused multiply-add where the
// FMA variant fuses, every other operation rounded on its own — and takes glibc's constants (ln2 hi/lo, the
// two polynomials, the 128 (1/c, log c) pairs) as data, read from the loaded libm at run time and accepted
// only after this function matched libm's log() on a sample of inputs (np_legacy_gauss.c,
// mppi_np_log_params).  Domain here: normal x in (0, 1] (r2 of an accepted polar attempt is >= 2^-104); the
// special-value branch of glibc (zero, subnormal, negative, inf, nan) is not reproduced.
//
// Included by the host C library (gcc, -ffp-contract=off) and by the HIP device code.
#pragma once
#include <stdint.h>
#include <string.h>

#ifdef __HIPCC__
#define NPLOG_FN __host__ __device__ static __forceinline__
#else
#define NPLOG_FN static inline
#endif

// data layout (doubles): [0] ln2hi, [1] ln2lo, [2..6] A[0..4], [7..17] B[0..10], [18 + 2i] 1/c_i,
// [19 + 2i] log c_i for i < 128 — glibc's struct log_data up to and including its tab[]
#define NPLOG_NDATA (18 + 256)

NPLOG_FN double nplog_asdouble(uint64_t u) {
    double d;
    memcpy(&d, &u, 8);
    return d;
}
NPLOG_FN uint64_t nplog_asuint64(double d) {
    uint64_t u;
    memcpy(&u, &d, 8);
    return u;
}

NPLOG_FN double np_glibc_log(const double* D, double x) {
#pragma STDC FP_CONTRACT OFF
    const double* A = D + 2;
    const double* B = D + 7;
    const uint64_t ix = nplog_asuint64(x);
    if (ix - 0x3fee000000000000ull < 0x3090000000000ull) {   // x in [1 - 2^-4, 1 + 0x1.09p-4)
        if (ix == 0x3ff0000000000000ull) return 0.0;
        const double r = x - 1.0;
        double p2 = __builtin_fma(r, B[2], B[1]);
        double p5 = __builtin_fma(r, B[5], B[4]);
        const double p8 = __builtin_fma(r, B[8], B[7]);
        const double r2 = r * r;
        p2 = __builtin_fma(r2, B[3], p2);
        p5 = __builtin_fma(r2, B[6], p5);
        const double r3 = r * r2;
        double q = __builtin_fma(r2, B[9], p8);
        q = __builtin_fma(r3, B[10], q);
        q = __builtin_fma(q, r3, p5);
        q = __builtin_fma(q, r3, p2);
        // rhi = r + w - w with w = r * 2^27, the first sum fused
        const double t = __builtin_fma(r, 0x1p27, r);
        const double rhi = __builtin_fma(-0x1p27, r, t);
        const double rhi2 = rhi * rhi;
        const double rlo = r - rhi;
        const double hi = __builtin_fma(rhi2, B[0], r);   // B[0] = -0.5
        const double d = r - hi;
        const double s = r + rhi;
        double lo = __builtin_fma(rhi2, B[0], d);
        const double bl = B[0] * rlo;
        lo = __builtin_fma(bl, s, lo);
        const double y = __builtin_fma(q, r3, lo);
        return hi + y;
    }
    // x = 2^k z with z in [0x1.6p-1, 0x1.6p0) (OFF = 0x3fe6000000000000), subinterval i of z
    const uint64_t tmp = ix - 0x3fe6000000000000ull;
    const int i = (int)((tmp >> 45) & 127u);
    const int k = (int)((int64_t)tmp >> 52);
    const uint64_t iz = ix - (tmp & 0xfff0000000000000ull);
    const double invc = D[18 + 2 * i], logc = D[19 + 2 * i];
    const double z = nplog_asdouble(iz);
    const double kd = (double)k;
    const double r = __builtin_fma(z, invc, -1.0);
    const double w = __builtin_fma(kd, D[0], logc);
    const double p12 = __builtin_fma(r, A[2], A[1]);
    const double hi = r + w;
    const double r2 = r * r;
    double lo = w - hi;
    lo = lo + r;
    lo = __builtin_fma(kd, D[1], lo);
    const double r3 = r * r2;
    double p34 = __builtin_fma(r, A[4], A[3]);
    lo = __builtin_fma(r2, A[0], lo);
    p34 = __builtin_fma(p34, r2, p12);
    const double y = __builtin_fma(r3, p34, lo);
    return y + hi;
}
