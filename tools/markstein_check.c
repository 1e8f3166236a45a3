// Markstein division by a fixed divisor (amp_fused.hip sm_arg_st): q = v RN(1/tau),
// q + fma(-q, tau, v) RN(1/tau) against v / tau.
//  1. random pairs over the decoder's range (10^8);
//  2. corners where q = RN(v RN(1/tau)) may be more than one ulp off, so that
//     Markstein's theorem does not apply: divisor significands near 2 (and
//     near 1), quotients just below and just above powers of two, and an
//     exhaustive sweep of the low 16 significand bits of tau against
//     dividends whose quotient sits at the top of its binade.
// build: gcc -O2 -mfma tools/markstein_check.c -o /tmp/markstein_check -lm
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static uint64_t s = 88172645463325252ULL;
static double rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (double)(s >> 11) * (1.0 / 9007199254740992.0); }
static long bad = 0, n = 0;
static void check(double v, double tau) {
    double r = 1.0 / tau;
    double q = v * r;
    double rem = fma(-q, tau, v);
    double q2 = fma(rem, r, q);
    double ex = v / tau;
    if (memcmp(&q2, &ex, 8) && !(q2 == 0.0 && ex == 0.0)) {
        if (bad < 8) printf("mismatch v=%a tau=%a got %a want %a\n", v, tau, q2, ex);
        ++bad;
    }
    ++n;
}
static double bits(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
int main(void) {
    // 1. random pairs of the decoder's range
    for (int k = 0; k < 2000; ++k) {
        double tau = ldexp(0.5 + rnd(), -12 + (int)(rnd() * 20));  // 2^-12 .. 2^8
        for (int i = 0; i < 50000; ++i) {
            double v = (rnd() - 0.5) * ldexp(1.0, (int)(rnd() * 16) - 4);
            if (i % 97 == 0) v = -v * 1e3;
            check(v, tau);
        }
    }
    long n1 = n, b1 = bad;
    printf("random pairs: %ld of %ld differ\n", b1, n1);
    // 2a. divisor significands within 2^16 ulp of 2 (and of 1), quotients within
    //     2^10 ulp below / above a power of two: v = RN(target * tau) and its neighbours
    for (int e = -12; e <= 8; e += 4)
        for (uint64_t k = 1; k <= 65536; k += (k < 256 ? 1 : 97)) {
            double taus[2] = {ldexp(bits(0x3ff0000000000000ULL + (0x000fffffffffffffULL - k + 1)), e),  // 2 - k ulp
                              ldexp(bits(0x3ff0000000000000ULL + k), e)};                             // 1 + k ulp
            for (int t = 0; t < 2; ++t)
                for (int j = -6; j <= 10; j += 2)
                    for (int m = -1024; m <= 1024; m += 7) {
                        double target = ldexp(1.0, j) * (1.0 + m * 0x1p-53);
                        double v = target * taus[t];
                        check(v, taus[t]);
                        check(nextafter(v, 0.0), taus[t]);
                        check(nextafter(v, 1e300), taus[t]);
                        check(-v, taus[t]);
                    }
        }
    long n2 = n - n1, b2 = bad - b1;
    printf("corner pairs (divisor near 1 or 2, quotient near a power of two): %ld of %ld differ\n", b2, n2);
    // 2b. every value of tau's low 16 significand bits (top bits random), with
    //     dividends whose quotient is at the top of its binade
    for (int hi = 0; hi < 64; ++hi) {
        uint64_t top = ((uint64_t)(rnd() * 68719476736.0)) << 16;  // 36 random high bits
        for (uint64_t lo = 0; lo < 65536; ++lo) {
            double tau = bits(0x3ff0000000000000ULL | ((top | lo) & 0x000fffffffffffffULL));
            double v = nextafter(2.0, 0.0) * tau;
            check(v, tau);
            check(nextafter(v, 0.0), tau);
        }
    }
    long n3 = n - n1 - n2, b3 = bad - b1 - b2;
    printf("exhaustive low significand bits: %ld of %ld differ\n", b3, n3);
    printf("total: %ld of %ld differ\n", bad, n);
    return bad ? 1 : 0;
}
