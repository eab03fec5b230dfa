// orbx_sincos.h -- (float)cos((double)r) and (float)sin((double)r) for r in [0, 2*pi],
// the rotation of steered BRIEF (ORBextractor.cc:123-125, hazard H3 in DESIGN.md).
//
// The library's double cos/sin carry large-argument reduction paths (~200 vector
// instructions per pair).  The angle here is fastAtan2's [0, 360] degrees scaled to
// radians, so one Cody-Waite step by pi/2 reduces it, and the fdlibm kernels
// (__kernel_sin / __kernel_cos, < 1 ulp) finish it in ~30 double operations.  Rounded
// to float, the result equals glibc's (float)cos / (float)sin for EVERY float in
// [0, 6.2832] (1,086,918,650 inputs, checked exhaustively; tests/test_sincos.py keeps a
// strided sample of that check).  Compiled -ffp-contract=off, operation by operation.
#pragma once

#ifdef __HIPCC__
#define ORBX_HD __host__ __device__
#else
#define ORBX_HD
#endif

namespace orbx {

ORBX_HD inline void sincos_0_2pi(double x, double& c, double& s) {
    const double invpio2 = 6.36619772367581382433e-01;
    const double pio2_1 = 1.57079632673412561417e+00;   // first 33 bits of pi/2
    const double pio2_1t = 6.07710050650619224932e-11;  // pi/2 - pio2_1
    const double fn = __builtin_rint(x * invpio2);
    const int n = (int)fn;
    const double r = (x - fn * pio2_1) - fn * pio2_1t;  // |r| <= pi/4
    const double z = r * r;
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double v = z * r;
    const double ps = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    const double sn = r + v * (S1 + z * ps);
    const double pc = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double cs = w + (((1.0 - w) - hz) + z * pc);
    switch (n & 3) {
        case 0: c = cs; s = sn; break;
        case 1: c = -sn; s = cs; break;
        case 2: c = -cs; s = -sn; break;
        default: c = sn; s = -cs; break;
    }
}

}  // namespace orbx
