/* Exhaustive check of bdpt_sincos_dp (the product's fp64 sin/cos, bdpt_math.h) against the
 * oracle's semantics (float)sin((double)x) / (float)cos((double)x) of glibc, over every x the
 * render path can pass: x = (2.f*FLOAT_PI) * u with u = f / 2^32 for every float f in [1, 2^32]
 * (a superset of ((float)y + 1.0f) / 4294967296.0f, MersenneTwister_kernel.cu:108).
 * Optional argv[1] = stride over the float bit patterns (1 = exhaustive). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../../gpu_bidirectional_raytracer_amd/csrc/bdpt_math.h"
/* built twice by tests/test_math.py: -DBDPT_SC_COARSE=0 (512-entry table) and =1 (256) */

int main(int argc, char **argv)
{
    unsigned stride = argc > 1 ? (unsigned)atoi(argv[1]) : 1u;
    float lo = 1.0f, hi = 4294967296.0f;
    uint32_t b0, b1;
    memcpy(&b0, &lo, 4);
    memcpy(&b1, &hi, 4);
    static const double tab[BDPT_SC_N][2] = BDPT_SINCOS_TABLE_INIT;
    double sintab[BDPT_SC_N];               /* the device's LDS copy: sin(2pi k/N) only */
    for (int k = 0; k < (BDPT_SC_N >> BDPT_SC_COARSE); k++) sintab[k] = tab[k << BDPT_SC_COARSE][0];
    long n = 0, bad = 0, bad_tab = 0;
    for (uint64_t b = b0; b <= b1; b += stride) {
        uint32_t bb = (uint32_t)b;
        float f;
        memcpy(&f, &bb, 4);
        const float u = f / 4294967296.0f;
        const float x = 2.f * 3.14159265358979323846f * u;
        double s, c;
        bdpt_sincos_dp((double)x, &s, &c);
        const float gs = (float)sin((double)x), gc = (float)cos((double)x);
        if ((float)s != gs || (float)c != gc) {
            if (bad < 5) printf("mismatch u=%a x=%a\n", u, x);
            bad++;
        }
        bdpt_sincos_tab((double)x, sintab, &s, &c);
        if ((float)s != gs || (float)c != gc) {
            if (bad_tab < 5) printf("table mismatch u=%a x=%a\n", u, x);
            bad_tab++;
        }
        n++;
    }
    printf("checked %ld inputs, %ld mismatches, %ld table-version mismatches\n", n, bad, bad_tab);
    return bad != 0 || bad_tab != 0;
}
