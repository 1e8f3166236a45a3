// Markstein division by a fixed divisor (amp_fused.hip sm_arg_st): q = v RN(1/tau),
// q + fma(-q, tau, v) RN(1/tau) against v / tau over random pairs of the decoder's range.
// build: gcc -O2 -mfma tools/markstein_check.c -o /tmp/markstein_check -lm
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
static uint64_t s = 88172645463325252ULL;
static double rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (double)(s >> 11) * (1.0 / 9007199254740992.0); }
int main(void) {
    long bad = 0, n = 0;
    for (int k = 0; k < 2000; ++k) {
        double tau = ldexp(0.5 + rnd(), -12 + (int)(rnd() * 20));  // 2^-12 .. 2^8
        double r = 1.0 / tau;
        for (int i = 0; i < 50000; ++i) {
            double v = (rnd() - 0.5) * ldexp(1.0, (int)(rnd() * 16) - 4);
            if (i % 97 == 0) v = -v * 1e3;
            double q = v * r;
            double rem = fma(-q, tau, v);
            double q2 = fma(rem, r, q);
            double ex = v / tau;
            if (memcmp(&q2, &ex, 8)) { if (bad < 5) printf("mismatch v=%a tau=%a got %a want %a\n", v, tau, q2, ex); ++bad; }
            ++n;
        }
    }
    printf("%ld of %ld differ\n", bad, n);
    return 0;
}
