/*
 * oracle/bp_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the flooding belief-propagation decoders of the
 * reference (ldpc_jossy/src/c_ldpc.c).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library, and only as the
 * checker / the timed CPU baseline -- never as part of the product path.
 *
 * Arithmetic order follows the reference exactly so that, compiled with the
 * same flags (gcc -O2, no fast-math), results are bit-identical:
 *   - variable pass   c_ldpc.c:171-178  (aggr = ch + sum over ports in port
 *                                        order; extrinsic = aggr - msg)
 *   - check pass      c_ldpc.c:183-194  via the forward/backward trellis
 *                                        Lxfb c_ldpc.c:294-314
 *   - pairwise op     Lxor c_ldpc.c:234-251 (plain log(1+exp()), no log1p)
 *   - sumprod         c_ldpc.c:32-113  (tanh product / atanh of quotient)
 *   - minsum          c_ldpc.c:339-381 (Lxfb without correction, every
 *                                        outgoing message times the factor)
 * Stopping rule: every check aggregate > 0 after the check pass
 * (c_ldpc.c:191,196); the return value is the 0-based index of the iteration
 * that stopped, or max_it.
 *
 * minsum: the reference advances its message offset by the degree of the
 * *next* check (c_ldpc.c:364, "j++, imsg += cdeg[j]"), which regroups
 * messages into the wrong checks whenever check degrees are not uniform.
 * `or_minsum` implements the corrected indexing; `or_minsum_refbug`
 * reproduces the shipped behaviour so the restatement can be pinned against
 * the reference library bit-for-bit (tests/test_oracle_pin.py).
 *
 * Graph arrays are int64 (Linux LP64 `long`, see SURVEY finding 0.4).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#define OR_MAX_DEGREE 64

/* LLR of the XOR of two bits (reference Lxor, c_ldpc.c:234-251). */
double or_lxor(double a, double b, int corr)
{
    int same = ((signbit(a) != 0) == (signbit(b) != 0));
    double out = (same ? 1.0 : -1.0) * fmin(fabs(a), fabs(b));
    if (corr) {
        out += log(1 + exp(-fabs(a + b)));
        out -= log(1 + exp(-fabs(a - b)));
    }
    return out;
}

/* Extrinsic LLRs of dc bits whose XOR is zero, in place; returns the full
 * (non-extrinsic) aggregate.  Reference Lxfb, c_ldpc.c:294-314. */
double or_lxfb(double *llr, int64_t dc, int corr)
{
    double fwd[OR_MAX_DEGREE], bwd[OR_MAX_DEGREE];
    int64_t i;
    if (dc < 2 || dc > OR_MAX_DEGREE)
        return NAN;
    fwd[0] = llr[0];
    bwd[dc - 1] = llr[dc - 1];
    for (i = 1; i < dc; i++) {
        fwd[i] = or_lxor(fwd[i - 1], llr[i], corr);
        bwd[dc - 1 - i] = or_lxor(bwd[dc - i], llr[dc - 1 - i], corr);
    }
    llr[0] = bwd[1];
    llr[dc - 1] = fwd[dc - 2];
    for (i = 1; i < dc - 1; i++)
        llr[i] = or_lxor(fwd[i - 1], bwd[i + 1], corr);
    return bwd[0];
}

/* Variable-node pass shared by every decoder (c_ldpc.c:171-178). */
static void var_pass(const double *ch, const int64_t *vdeg, const int64_t *port2msg,
                     int nv, double *msg, double *app)
{
    int64_t port = 0;
    for (int v = 0; v < nv; v++) {
        double acc = ch[v];
        int64_t d = vdeg[v];
        for (int64_t k = 0; k < d; k++)
            acc += msg[port2msg[port + k]];
        for (int64_t k = 0; k < d; k++)
            msg[port2msg[port + k]] = acc - msg[port2msg[port + k]];
        app[v] = acc;
        port += d;
    }
}

enum { OR_SUMPROD = 0, OR_SUMPROD2 = 1, OR_MINSUM = 2, OR_MINSUM_REFBUG = 3 };

static int decode_generic(int kind, const double *ch, const int64_t *vdeg, const int64_t *cdeg,
                          const int64_t *port2msg, int nv, int nc, int nmsg, double *app,
                          double factor, int max_it)
{
    double *msg = (double *)calloc((size_t)nmsg, sizeof(double));
    int it;
    if (!msg)
        return -1;
    for (it = 0; it < max_it; it++) {
        int unsatisfied = 0;
        var_pass(ch, vdeg, port2msg, nv, msg, app);
        if (kind == OR_SUMPROD) {
            int64_t base = 0;
            for (int c = 0; c < nc; c++) {
                int64_t d = cdeg[c];
                double prod = 1.0;
                for (int64_t k = 0; k < d; k++) {
                    msg[base + k] = tanh(msg[base + k] / 2.0);
                    prod *= msg[base + k];
                }
                if (!unsatisfied && 2.0 * atanh(prod) <= 0.0)
                    unsatisfied = 1;
                for (int64_t k = 0; k < d; k++)
                    msg[base + k] = 2.0 * atanh(prod / msg[base + k]);
                base += d;
            }
        } else if (kind == OR_SUMPROD2 || kind == OR_MINSUM) {
            int corr = (kind == OR_SUMPROD2);
            int64_t base = 0;
            for (int c = 0; c < nc; c++) {
                int64_t d = cdeg[c];
                double agg = or_lxfb(&msg[base], d, corr);
                if (!unsatisfied && agg <= 0.0)
                    unsatisfied = 1;
                if (!corr)
                    for (int64_t k = 0; k < d; k++)
                        msg[base + k] *= factor;
                base += d;
            }
        } else { /* OR_MINSUM_REFBUG: offset advanced by the next check's degree */
            int64_t base = 0;
            for (int c = 0; c < nc; c++) {
                int64_t d = cdeg[c];
                double agg = or_lxfb(&msg[base], d, 0);
                if (!unsatisfied && agg <= 0.0)
                    unsatisfied = 1;
                for (int64_t k = 0; k < d; k++)
                    msg[base + k] *= factor;
                if (c + 1 < nc)
                    base += cdeg[c + 1];
            }
        }
        if (!unsatisfied)
            break;
    }
    free(msg);
    return it;
}

int or_sumprod(const double *ch, const int64_t *vdeg, const int64_t *cdeg, const int64_t *intrlv,
               int nv, int nc, int nmsg, double *app, int max_it)
{
    return decode_generic(OR_SUMPROD, ch, vdeg, cdeg, intrlv, nv, nc, nmsg, app, 0.0, max_it);
}

int or_sumprod2(const double *ch, const int64_t *vdeg, const int64_t *cdeg, const int64_t *intrlv,
                int nv, int nc, int nmsg, double *app, int max_it)
{
    return decode_generic(OR_SUMPROD2, ch, vdeg, cdeg, intrlv, nv, nc, nmsg, app, 0.0, max_it);
}

int or_minsum(const double *ch, const int64_t *vdeg, const int64_t *cdeg, const int64_t *intrlv,
              int nv, int nc, int nmsg, double *app, double factor, int max_it)
{
    return decode_generic(OR_MINSUM, ch, vdeg, cdeg, intrlv, nv, nc, nmsg, app, factor, max_it);
}

int or_minsum_refbug(const double *ch, const int64_t *vdeg, const int64_t *cdeg,
                     const int64_t *intrlv, int nv, int nc, int nmsg, double *app, double factor,
                     int max_it)
{
    return decode_generic(OR_MINSUM_REFBUG, ch, vdeg, cdeg, intrlv, nv, nc, nmsg, app, factor,
                          max_it);
}

/* Batched convenience entry used by the CPU baseline: B codewords, row-major
 * [B][nv] LLRs, decoded one after the other on the calling thread. */
int or_decode_batch(int kind, const double *ch, int B, const int64_t *vdeg, const int64_t *cdeg,
                    const int64_t *intrlv, int nv, int nc, int nmsg, double factor, int max_it,
                    double *app, int32_t *its)
{
    for (int b = 0; b < B; b++) {
        int r = decode_generic(kind, ch + (size_t)b * nv, vdeg, cdeg, intrlv, nv, nc, nmsg,
                               app + (size_t)b * nv, factor, max_it);
        if (r < 0)
            return r;
        its[b] = r;
    }
    return 0;
}
