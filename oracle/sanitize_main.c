/* TEST INFRASTRUCTURE ONLY -- driver that runs the CPU restatement
 * (oracle/bp_oracle.c) under AddressSanitizer and UndefinedBehaviorSanitizer
 * (sanitizers on the CPU restatement; `make -C oracle san`).
 *
 * usage: bp_oracle_san IN OUT
 *   IN : int32 nv, nc, nmsg, B, max_it; double factor; int64 vdeg[nv],
 *        cdeg[nc], intrlv[nmsg]; double ch[B][nv]
 *   OUT: for kind in sumprod, sumprod2, minsum, minsum_refbug:
 *        double app[B][nv], int32 it[B]; then double Lxfb aggregates of the
 *        first check's ports at corr 0 and 1.
 * Exit status 0 on success; a sanitizer report aborts with a nonzero status. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int or_decode_batch(int kind, const double *ch, int B, const int64_t *vdeg, const int64_t *cdeg,
                    const int64_t *intrlv, int nv, int nc, int nmsg, double factor, int max_it,
                    double *app, int32_t *its);
double or_lxfb(double *llr, int64_t dc, int corr);

static void *rd(FILE *f, size_t n)
{
    void *p = malloc(n ? n : 1);
    if (!p || fread(p, 1, n, f) != n) {
        fprintf(stderr, "short input\n");
        exit(2);
    }
    return p;
}

int main(int argc, char **argv)
{
    if (argc != 3)
        return 2;
    FILE *f = fopen(argv[1], "rb");
    if (!f)
        return 2;
    int32_t *hdr = rd(f, 5 * sizeof(int32_t));
    const int nv = hdr[0], nc = hdr[1], nmsg = hdr[2], B = hdr[3], max_it = hdr[4];
    double *factor = rd(f, sizeof(double));
    int64_t *vdeg = rd(f, (size_t)nv * 8), *cdeg = rd(f, (size_t)nc * 8), *intrlv = rd(f, (size_t)nmsg * 8);
    double *ch = rd(f, (size_t)B * nv * 8);
    fclose(f);
    FILE *o = fopen(argv[2], "wb");
    if (!o)
        return 2;
    double *app = malloc((size_t)B * nv * 8);
    int32_t *its = malloc((size_t)B * 4);
    for (int kind = 0; kind < 4; kind++) {
        if (or_decode_batch(kind, ch, B, vdeg, cdeg, intrlv, nv, nc, nmsg, *factor, max_it, app, its) != 0)
            return 3;
        fwrite(app, 8, (size_t)B * nv, o);
        fwrite(its, 4, (size_t)B, o);
    }
    double *L = malloc((size_t)cdeg[0] * 8);
    for (int corr = 0; corr < 2; corr++) {
        for (int64_t k = 0; k < cdeg[0]; k++)
            L[k] = ch[k % nv];
        const double agg = or_lxfb(L, cdeg[0], corr);
        fwrite(&agg, 8, 1, o);
    }
    fclose(o);
    free(L);
    free(app);
    free(its);
    free(ch);
    free(intrlv);
    free(cdeg);
    free(vdeg);
    free(factor);
    free(hdr);
    return 0;
}
