/* Host check of rt_kernels.hip div_ia: x / a from ia = RN(1/a) with two
 * residual (fma) steps must equal the IEEE quotient x / a.  Same operations
 * as the device function (fma = fused, everything else rounded per op:
 * compiled with -ffp-contract=off).  usage: div_ia_check N seed
 * prints "mismatches K of N"; exit status 1 if K > 0. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t st;
static uint64_t next(void) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; return st; }
static double with_exp(int e) {                 /* random significand, exponent e */
    const uint64_t bits = ((uint64_t)(e + 1023) << 52) | (next() & ((1ull << 52) - 1));
    double d;
    memcpy(&d, &bits, sizeof d);
    return d;
}
static double div_ia(const double x, const double a, const double ia) {
    const double q0 = x * ia;
    const double q1 = fma(fma(-q0, a, x), ia, q0);
    return fma(fma(-q1, a, x), ia, q1);
}
int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    st = argc > 2 ? strtoull(argv[2], 0, 0) : 0x9E3779B97F4A7C15ull;
    long bad = 0;
    for (long i = 0; i < n; ++i) {
        double a;
        switch (i & 3) {
        case 0: a = 1.0 + (double)(next() & 0xFFFFF) * 0x1p-52; break;     /* |unit d|^2 ~ 1 */
        case 1: a = with_exp(-30 + (int)(next() % 61)); break;              /* any ray length */
        case 2: a = with_exp(0) * (next() & 1 ? 1.0 : 0.5); break;
        default: a = 2.0 - (double)(next() & 0xFF) * 0x1p-52; break;        /* all-ones significands */
        }
        double x = with_exp(-60 + (int)(next() % 121));
        if (next() & 1) x = -x;
        const double ia = 1.0 / a;
        const double q = div_ia(x, a, ia), want = x / a;
        if (memcmp(&q, &want, sizeof q) != 0) {
            if (bad < 5) printf("x=%a a=%a got %a want %a\n", x, a, q, want);
            ++bad;
        }
    }
    printf("mismatches %ld of %ld\n", bad, n);
    return bad != 0;
}
