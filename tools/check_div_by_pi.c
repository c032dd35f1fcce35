/* Exhaustive check of pt_device.h's div_by_pi (x * RN(1/PI), one Markstein correction) against
 * IEEE single-precision x / PI: 0 and every float in [2^-30, 1] (the cosine sample's z is 0 or at
 * least 2^-24); --all: every float from 2^-100 up (near 2^-124 the residual x - PI q is subnormal
 * and the correction loses bits; no caller comes near).
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math check_div_by_pi.c -lm.  Exit 0 = identical bits. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
int main(int argc, char** argv) {
    const float PI = 3.1415926535897932384626422832795028841971f;
    const float INV_PI_RN = 0.318309873342514038085938f;
    volatile float one = 1.0f;
    if (one / PI != INV_PI_RN) { printf("RN(1/PI) mismatch\n"); return 2; }
    const int all = argc > 1 && strcmp(argv[1], "--all") == 0;
    const uint32_t lo = all ? 0x0d800000u : 0x30800000u, hi = all ? 0x7f7fffffu : 0x3f800000u;
    uint64_t bad = 0, n = 0;
    {   /* x = 0 */
        const float q = 0.0f * INV_PI_RN, got = fmaf(fmaf(-PI, q, 0.0f), INV_PI_RN, q), ref = 0.0f / PI;
        if (memcmp(&got, &ref, 4) != 0) ++bad;
        ++n;
    }
    for (uint32_t b = lo;; ++b) {
        float x;
        memcpy(&x, &b, 4);
        const float ref = x / PI;
        const float q = x * INV_PI_RN;
        const float got = fmaf(fmaf(-PI, q, x), INV_PI_RN, q);
        uint32_t a1, a2;
        memcpy(&a1, &ref, 4);
        memcpy(&a2, &got, 4);
        if (a1 != a2) {
            if (bad < 5) printf("mismatch x=%a ref=%a got=%a\n", x, ref, got);
            ++bad;
        }
        ++n;
        if (b == hi) break;
    }
    printf("checked %llu floats, %llu mismatches\n", (unsigned long long)n, (unsigned long long)bad);
    return bad ? 1 : 0;
}
