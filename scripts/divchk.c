// Exhaustive check of div_const (computer-graphics_amd/csrc/cg_math.h): for every
// float x, IEEE fl(x / b) == div_const(x) where
//   r = fl(1/b), q0 = fl(x * r), e = fma(-q0, b, x),
//   div_const = (e == 0 || x not finite) ? q0 : fma(e, r, q0).
// Usage: divchk B [STRIDE]   (exit 0 = no mismatch).  Run for B = 3, 5, 9 with
// stride 1 (all 2^32 inputs, ~40 s each): no mismatch.
//   gcc -O2 -ffp-contract=off -mfma -o divchk scripts/divchk.c -lm
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
int main(int argc, char **argv)
{
    float b = strtof(argv[1], 0);
    volatile float bv = b;
    float r = 1.0f / bv;
    unsigned long long bad = 0;
    const uint64_t stride = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
    for (uint64_t u = 0; u <= 0xffffffffull; u += stride) {
        uint32_t w = (uint32_t)u;
        float x;
        memcpy(&x, &w, 4);
        volatile float xv = x;
        float ref = xv / bv;
        float q0 = x * r;
        float e = fmaf(-q0, b, x);
        float q1 = (e == 0.0f || !isfinite(x)) ? q0 : fmaf(e, r, q0);
        if (isnan(ref) && isnan(q1)) continue;
        uint32_t a, c;
        memcpy(&a, &ref, 4);
        memcpy(&c, &q1, 4);
        if (a != c) {
            if (bad < 5) printf("x=%a ref=%a got=%a\n", x, ref, q1);
            ++bad;
        }
    }
    printf("b=%g r=%a mismatches=%llu\n", b, r, bad);
    return bad != 0;
}
