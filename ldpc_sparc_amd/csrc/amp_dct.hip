// AMP decoder for SPARCs with sub-sampled DCT designs on gfx950.
//
// Reference: sparc_public/sparc.py sparc_amp :883-999 (loop), sparc_transforms
// :703-880 with sub_dct :648-701 (design operator), msg_vector_mmse_estimator
// :402-465 (softmax denoiser), msg_vector_map_estimator :467-512 (final MAP).
//
// Operator (DESIGN.md "DCT operator"): for each transform (nonzero block of W)
//   Ab:  r = sqrt(2 W_rc/L) * DCT-II_w(scatter(beta_c, order1))[order0]
//   Az:  u = sqrt(2 W_rc/L) * DCT-III_w(scatter(z_r/phi_r, order0))[order1]
// A length-w DCT is a length-N2 = w/2 complex FFT of the Makhoul-packed
// sequence; positions p of the length-w vector map one-to-one onto "w-space
// slots" n(p) = p/2 (p even) or w-1-(p-1)/2 (p odd), slot n = complex index
// n>>1, component n&1.  The N2-point FFT runs four-step, N2 = P*Q:
//   ab_passA  (per tile of CT columns m2): gather beta into h[Q m1 + m2], P-point
//             FFT over m1, twiddle w_N2^{m2 k1}, store T[k1][m2]
//   ab_passB  (per row pair {k1, P-k1}): Q-point FFTs, then only the needed
//             outputs X[order0[i]] = Re(c1 H[a] + c2 conj H[b]) -> rbuf
//   az_passA  (per row pair): sparse G rows from z/phi (<=4 terms per slot),
//             Q-point inverse FFTs, twiddle, store U[k1][m2]
//   az_passB  (per column tile): P-point inverse FFTs -> g[m] (w-space)
//   eta       (one wavefront per section): gather u from g, s = beta + tau u,
//             per-section softmax (max-shifted, mathematically identical to
//             the reference's global-max float128 form), section statistics
//   control   (one workgroup per codeword): Onsager residual, phi, tau, psi,
//             NMSE, early stop (sparc.py:931-988) in double precision.
#include "amp.hpp"

namespace sg {

template <typename T>
__device__ __forceinline__ T dexp(T x);
template <>
__device__ __forceinline__ float dexp<float>(float x) { return __expf(x); }
template <>
__device__ __forceinline__ double dexp<double>(double x) { return exp(x); }

template <typename T>
__device__ __forceinline__ cx<T> big_twiddle(const AmpTables<T> &tb, int e) {
    return cmul(tb.twHi[e >> 10], tb.twLo[e & 1023]);
}

// ------------------------------------------------------------------ Ab pass A
template <typename T, int EPT>
__global__ __launch_bounds__(256) void ab_passA(AmpTables<T> tb, AmpBufs<T> bf, int CT) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cx<T> *d = reinterpret_cast<cx<T> *>(smem_raw);
    const int cw = blockIdx.z, t = blockIdx.y;
    if (!bf.active[cw]) return;
    const int nthr = blockDim.x, tid = threadIdx.x;
    const int m2_0 = blockIdx.x * CT;
    const int total = tb.P * CT;
    const int32_t *inmap = tb.inmap + (size_t)t * tb.w;
    const T *beta = bf.beta + (size_t)cw * tb.LM + (size_t)tb.t_col[t] * tb.Mc;
    for (int idx = tid; idx < total; idx += nthr) {
        const int m1 = idx / CT, c = idx - m1 * CT;
        const int m = tb.Q * m1 + m2_0 + c;
        const int j0 = inmap[2 * m], j1 = inmap[2 * m + 1];
        d[idx] = cx<T>{j0 >= 0 ? beta[j0] : T(0), j1 >= 0 ? beta[j1] : T(0)};
    }
    __syncthreads();
    lds_fft<T, false, EPT, true>(d, tb.log2P, CT, CT, 1, tb.twP, tid, nthr);
    cx<T> *out = bf.buf0 + ((size_t)cw * tb.nT + t) * tb.N2;
    for (int idx = tid; idx < total; idx += nthr) {
        const int k1 = idx / CT, c = idx - k1 * CT;
        const int m2 = m2_0 + c;
        out[(size_t)k1 * tb.Q + m2] = cmul(d[idx], big_twiddle(tb, m2 * k1));
    }
}

// ------------------------------------------------------------------ Ab pass B
template <typename T, int EPT>
__global__ __launch_bounds__(256) void ab_passB(AmpTables<T> tb, AmpBufs<T> bf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cx<T> *d = reinterpret_cast<cx<T> *>(smem_raw);
    const int cw = blockIdx.z, t = blockIdx.y, p = blockIdx.x;
    if (!bf.active[cw]) return;
    const int nthr = blockDim.x, tid = threadIdx.x;
    const int rowA = p, rowB = (tb.P - p) % tb.P;
    const cx<T> *src = bf.buf0 + ((size_t)cw * tb.nT + t) * tb.N2;
    for (int e = tid; e < tb.Q; e += nthr) {
        d[e] = src[(size_t)rowA * tb.Q + e];
        d[tb.Q + e] = src[(size_t)rowB * tb.Q + e];
    }
    __syncthreads();
    lds_fft<T, false, EPT, false>(d, tb.log2Q, 2, 1, tb.Q, tb.twQ, tid, nthr);
    const int o0 = tb.rp_ptr[t * (tb.npairs + 1) + p], o1 = tb.rp_ptr[t * (tb.npairs + 1) + p + 1];
    T *r = bf.rbuf + ((size_t)cw * tb.nT + t) * tb.Mr;
    for (int o = o0 + tid; o < o1; o += nthr) {
        const uint32_t ab = tb.rp_ab[o];
        const cx<T> ha = d[ab & 0xffffu], hb = d[ab >> 16];
        const cx<T> c1 = tb.rp_c[2 * o], c2 = tb.rp_c[2 * o + 1];
        // Re(c1*ha + c2*conj(hb))
        r[tb.rp_i[o]] = (c1.x * ha.x - c1.y * ha.y) + (c2.x * hb.x + c2.y * hb.y);
    }
}

// ------------------------------------------------------------------ Az pass A
template <typename T, int EPT>
__global__ __launch_bounds__(256) void az_passA(AmpTables<T> tb, AmpBufs<T> bf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cx<T> *d = reinterpret_cast<cx<T> *>(smem_raw);
    const int cw = blockIdx.z, t = blockIdx.y, p = blockIdx.x;
    if (!bf.active[cw]) return;
    const int nthr = blockDim.x, tid = threadIdx.x;
    const int rowA = p, rowB = (tb.P - p) % tb.P;
    for (int e = tid; e < 2 * tb.Q; e += nthr) d[e] = cx<T>{T(0), T(0)};
    __syncthreads();
    const int row = tb.t_row[t];
    const T *z = bf.z + (size_t)cw * tb.n + (size_t)row * tb.Mr;
    const T phi = (T)bf.phi[(size_t)cw * tb.Lr + row];
    const int s0 = tb.gs_ptr[t * (tb.npairs + 1) + p], s1 = tb.gs_ptr[t * (tb.npairs + 1) + p + 1];
    for (int s = s0 + tid; s < s1; s += nthr) {
        cx<T> acc{T(0), T(0)};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = tb.gs_i[4 * s + q];
            if (i >= 0) {
                const T v = z[i] / phi;
                const cx<T> c = tb.gs_c[4 * s + q];
                acc.x += c.x * v;
                acc.y += c.y * v;
            }
        }
        d[tb.gs_loc[s]] = acc;
    }
    __syncthreads();
    lds_fft<T, true, EPT, false>(d, tb.log2Q, 2, 1, tb.Q, tb.twQ, tid, nthr);
    cx<T> *out = bf.buf0 + ((size_t)cw * tb.nT + t) * tb.N2;
    const int halves = (rowA == rowB) ? 1 : 2;
    for (int e = tid; e < halves * tb.Q; e += nthr) {
        const int h = e >= tb.Q, m2 = e - h * tb.Q;
        const int k1 = h ? rowB : rowA;
        out[(size_t)k1 * tb.Q + m2] = cmul(d[e], cconj(big_twiddle(tb, m2 * k1)));
    }
}

// ------------------------------------------------------------------ Az pass B
template <typename T, int EPT>
__global__ __launch_bounds__(256) void az_passB(AmpTables<T> tb, AmpBufs<T> bf, int CT) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    cx<T> *d = reinterpret_cast<cx<T> *>(smem_raw);
    const int cw = blockIdx.z, t = blockIdx.y;
    if (!bf.active[cw]) return;
    const int nthr = blockDim.x, tid = threadIdx.x;
    const int m2_0 = blockIdx.x * CT;
    const int total = tb.P * CT;
    const cx<T> *src = bf.buf0 + ((size_t)cw * tb.nT + t) * tb.N2;
    for (int idx = tid; idx < total; idx += nthr) {
        const int k1 = idx / CT, c = idx - k1 * CT;
        d[idx] = src[(size_t)k1 * tb.Q + m2_0 + c];
    }
    __syncthreads();
    lds_fft<T, true, EPT, true>(d, tb.log2P, CT, CT, 1, tb.twP, tid, nthr);
    cx<T> *g = bf.buf1 + ((size_t)cw * tb.nT + t) * tb.N2;
    for (int idx = tid; idx < total; idx += nthr) {
        const int m1 = idx / CT, c = idx - m1 * CT;
        g[(size_t)tb.Q * m1 + m2_0 + c] = d[idx];
    }
}

// ------------------------------------------------------------------ eta
// One wavefront per section; EPL = ceil(M/64) elements per lane.
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <typename T>
__device__ __forceinline__ T gather_u(const AmpTables<T> &tb, const AmpBufs<T> &bf, int cw, int c, int jl) {
    T u = T(0);
    for (int q = tb.col_ptr[c]; q < tb.col_ptr[c + 1]; ++q) {
        const int t = tb.col_t[q];
        const int slot = tb.outslot[(size_t)t * tb.Mc + jl];
        const cx<T> g = bf.buf1[((size_t)cw * tb.nT + t) * tb.N2 + (slot >> 1)];
        u += (slot & 1) ? g.y : g.x;
    }
    return u;
}

template <typename T, int EPL>
__global__ __launch_bounds__(256) void eta_kernel(AmpTables<T> tb, AmpBufs<T> bf) {
    const int cw = blockIdx.y;
    if (!bf.active[cw]) return;
    const int lane = threadIdx.x & 63;
    const int l = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (l >= tb.L) return;
    const int secs_per_col = tb.L / tb.Lc;
    const int c = l / secs_per_col;
    const T tau = (T)bf.tau[(size_t)cw * tb.Lc + c];
    T *beta = bf.beta + (size_t)cw * tb.LM + (size_t)l * tb.M;
    const int jl0 = l * tb.M - c * tb.Mc;
    T s[EPL], x[EPL];
    T smax = -INFINITY, xmax = -INFINITY;
    int arg = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        const int e = lane + 64 * k;
        if (e < tb.M) {
            const T u = gather_u(tb, bf, cw, c, jl0 + e);
            s[k] = beta[e] + tau * u;           // sparc.py:972
            x[k] = s[k] / tau;                  // sparc.py:430
            xmax = fmax(xmax, x[k]);
            if (s[k] > smax) { smax = s[k]; arg = e; }
        } else {
            s[k] = -INFINITY;
            x[k] = -INFINITY;
        }
    }
    xmax = wave_max(xmax);
    // MAP index: first (lowest) index attaining the maximum of s (numpy argmax)
    const T gmax = wave_max(smax);
    int cand = (smax == gmax) ? arg : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
    T den = T(0);
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        const int e = lane + 64 * k;
        if (e < tb.M) { x[k] = dexp<T>(x[k] - xmax); den += x[k]; }
    }
    den = wave_sum(den);
    const int truth = bf.true_idx ? bf.true_idx[(size_t)cw * tb.L + l] : -1;
    T ss = T(0), se = T(0);
#pragma unroll
    for (int k = 0; k < EPL; ++k) {
        const int e = lane + 64 * k;
        if (e < tb.M) {
            const T b = x[k] / den;
            beta[e] = b;
            ss += b * b;
            const T dlt = b - (e == truth ? T(1) : T(0));
            se += dlt * dlt;
        }
    }
    ss = wave_sum(ss);
    se = wave_sum(se);
    if (lane == 0) {
        bf.sec_sumsq[(size_t)cw * tb.L + l] = (double)ss;
        bf.sec_err[(size_t)cw * tb.L + l] = (double)se;
        bf.sec_argmax[(size_t)cw * tb.L + l] = cand;
    }
}

// ------------------------------------------------------------------ control
// phase 0 (before Az, iteration t): Onsager residual and phi/tau
// (sparc.py:932-969); phase 1 (after eta): psi, NMSE, stopping
// (sparc.py:976-988); phase 2: initialisation.
__device__ __forceinline__ double block_sum(double v, double *red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double t = 0.0;
    for (int w = 0; w < nw; ++w) t += red[w];
    return t;
}

template <typename T>
__global__ __launch_bounds__(1024) void control_kernel(AmpTables<T> tb, AmpBufs<T> bf, AmpScalars sc, AmpParams pr,
                                                       int phase, int t) {
    __shared__ double red[16];
    const int cw = blockIdx.x, tid = threadIdx.x;
    const int Lr = tb.Lr, Lc = tb.Lc;
    double *psi = sc.psi + (size_t)cw * Lc, *psi_prev = sc.psi_prev + (size_t)cw * Lc;
    double *phi = bf.phi + (size_t)cw * Lr, *phi_prev = sc.phi_prev + (size_t)cw * Lr;
    double *gamma = sc.gamma + (size_t)cw * Lr, *bco = sc.bcoef + (size_t)cw * Lr;
    double *tau = bf.tau + (size_t)cw * Lc;
    double *nmse = sc.nmse + (size_t)cw * pr.t_max * Lc;
    if (phase == 2) {  // init: beta = 0 (memset on host), nmse[0] = 1
        for (int i = tid; i < pr.t_max * Lc; i += blockDim.x) nmse[i] = 1.0;
        if (tid == 0) { bf.active[cw] = 1; sc.t_final[cw] = 0; }
        return;
    }
    if (!bf.active[cw]) return;
    if (phase == 0) {
        T *z = bf.z + (size_t)cw * tb.n;
        const T *y = bf.y + (size_t)cw * tb.n;
        if (t > 0) {
            __syncthreads();
            // per row block in parallel (same per-entry arithmetic as the serial form)
            for (int r = tid; r < Lr; r += blockDim.x) {
                phi_prev[r] = phi[r];
                double g;
                if (tb.ndim == 0) g = pr.W[0] * psi[0];
                else {
                    double acc = 0.0;
                    for (int c = 0; c < Lc; ++c) acc += pr.W[r * Lc + c] * psi[c];
                    g = acc / Lc;
                }
                gamma[r] = g;
                bco[r] = g / phi[r];
            }
            __syncthreads();
            for (int c = tid; c < Lc; c += blockDim.x) psi_prev[c] = psi[c];
            // z = y - Ab(beta) + b*z, Ab summed over the transforms of each row block in table order.
            // ZU entries per thread at a time with the first QM transforms of each row requested
            // together, unconditionally (indices clamped into the tables, values masked): as a plain loop
            // every entry's table -> transform index -> rbuf chain, and each transform's load, was its
            // own round trip
            constexpr int ZU = 2, QM = 8;  // (ZU = 4 spilled at the 1024-thread kernel's 128 VGPRs)
            const int qlast = tb.row_ptr[Lr] - 1;  // -1: a plan with no transforms, nothing to load (uniform)
            for (int b0 = tid; b0 < tb.n; b0 += ZU * (int)blockDim.x) {
                int rr[ZU], qa[ZU], qb[ZU], il[ZU];
                T yv[ZU], zv[ZU];
                double bv[ZU];
#pragma unroll
                for (int u = 0; u < ZU; ++u) {
                    const int i = min(b0 + u * (int)blockDim.x, tb.n - 1);
                    const int r = i / tb.Mr;
                    rr[u] = r;
                    il[u] = i - r * tb.Mr;
                    qa[u] = tb.row_ptr[r];
                    qb[u] = tb.row_ptr[r + 1];
                    yv[u] = y[i];
                    zv[u] = z[i];
                    bv[u] = bco[r];
                }
                T rv[ZU][QM];
#pragma unroll
                for (int u = 0; u < ZU; ++u) {
                    if (qlast < 0) {
#pragma unroll
                        for (int k = 0; k < QM; ++k) rv[u][k] = T(0);
                        continue;
                    }
                    int tq[QM];
#pragma unroll
                    for (int k = 0; k < QM; ++k) tq[k] = tb.row_t[min(qa[u] + k, qlast)];
#pragma unroll
                    for (int k = 0; k < QM; ++k) rv[u][k] = bf.rbuf[((size_t)cw * tb.nT + tq[k]) * tb.Mr + il[u]];
                }
#pragma unroll
                for (int u = 0; u < ZU; ++u) {
                    const int i = b0 + u * (int)blockDim.x;
                    if (i >= tb.n) continue;
                    T ab = T(0);
#pragma unroll
                    for (int k = 0; k < QM; ++k)
                        if (qa[u] + k < qb[u]) ab += rv[u][k];
                    for (int q = qa[u] + QM; q < qb[u]; ++q)  // (rows of more than QM transforms)
                        ab += bf.rbuf[((size_t)cw * tb.nT + tb.row_t[q]) * tb.Mr + il[u]];
                    z[i] = (yv[u] - ab) + (T)bv[u] * zv[u];
                }
            }
        } else {
            for (int i = tid; i < tb.n; i += blockDim.x) z[i] = y[i];
            if (tid == 0) {
                if (tb.ndim == 0) gamma[0] = pr.W[0];
                else
                    for (int r = 0; r < Lr; ++r) {
                        double acc = 0.0;
                        for (int c = 0; c < Lc; ++c) acc += pr.W[r * Lc + c];
                        gamma[r] = acc / Lc;
                    }
            }
        }
        __syncthreads();
        if (pr.phi_method == 1) {
            if (tid == 0)
                for (int r = 0; r < Lr; ++r) phi[r] = pr.awgn_var + gamma[r];
        } else if (tb.ndim == 2) {  // one wavefront per row block, no workgroup barriers
            const int lane = tid & 63, nw = blockDim.x >> 6;
            for (int r = tid >> 6; r < Lr; r += nw) {
                double acc = 0.0;
                for (int i = r * tb.Mr + lane; i < (r + 1) * tb.Mr; i += 64) { const double v = (double)z[i]; acc += v * v; }
                acc = wave_sum(acc);
                if (lane == 0) phi[r] = acc / (double)tb.Mr;
            }
        } else {
            double acc = 0.0;
            for (int i = tid; i < tb.n; i += blockDim.x) { const double v = (double)z[i]; acc += v * v; }
            acc = block_sum(acc, red);
            if (tid == 0) phi[0] = acc / (double)tb.n;
        }
        __syncthreads();
        for (int c = tid; c < (tb.ndim == 0 ? 1 : Lc); c += blockDim.x) {  // per column block in parallel
            if (tb.ndim == 0) tau[0] = (tb.L * phi[0] / tb.n) / pr.W[0];
            else if (tb.ndim == 1) tau[c] = (tb.L * phi[0] / tb.n) / pr.W[c];
            else {
                double acc = 0.0;
                for (int r = 0; r < Lr; ++r) acc += pr.W[r * Lc + c] * (1.0 / phi[r]);
                tau[c] = ((double)tb.L / tb.Mr) / acc;
            }
        }
        return;
    }
    // phase 1: psi / NMSE / stop
    const int spc = tb.L / Lc;
    const double denom = (tb.ndim == 0) ? (double)tb.L : ((double)tb.L / Lc);
    if (Lc > 1) {  // one wavefront per column block, no workgroup barriers
        const int lane = tid & 63, nw = blockDim.x >> 6;
        for (int c = tid >> 6; c < Lc; c += nw) {
            double a = 0.0, e = 0.0;
            for (int l = c * spc + lane; l < (c + 1) * spc; l += 64) {
                a += bf.sec_sumsq[(size_t)cw * tb.L + l];
                e += bf.sec_err[(size_t)cw * tb.L + l];
            }
            a = wave_sum(a);
            e = wave_sum(e);
            if (lane == 0) {
                psi[c] = 1.0 - a / denom;
                nmse[(size_t)(t + 1) * Lc + c] = e / denom;
            }
        }
    } else {
        double a = 0.0, e = 0.0;
        for (int l = tid; l < spc; l += blockDim.x) {
            a += bf.sec_sumsq[(size_t)cw * tb.L + l];
            e += bf.sec_err[(size_t)cw * tb.L + l];
        }
        a = block_sum(a, red);
        e = block_sum(e, red);
        if (tid == 0) {
            psi[0] = 1.0 - a / denom;
            nmse[(size_t)(t + 1) * Lc] = e / denom;
        }
    }
    __syncthreads();
    if (tid == 0) {
        bool stop = false;
        if (t > 0) {
            stop = true;
            for (int c = 0; c < Lc; ++c)
                if (!(fabs(psi[c] - psi_prev[c]) <= pr.atol + pr.rtol * fabs(psi_prev[c]))) stop = false;
        }
        if (stop) {  // nmse[t:] = nmse[t]
            for (int tt = t + 1; tt < pr.t_max; ++tt)
                for (int c = 0; c < Lc; ++c) nmse[(size_t)tt * Lc + c] = nmse[(size_t)t * Lc + c];
            sc.t_final[cw] = t + 1;
            bf.active[cw] = 0;
        } else if (t == pr.t_max - 2) {
            sc.t_final[cw] = t + 1;
            bf.active[cw] = 0;
        }
    }
}

// ------------------------------------------------------------------ helpers
template <typename T>
__global__ void rowsum_kernel(AmpTables<T> tb, AmpBufs<T> bf, T *out) {
    const int cw = blockIdx.y;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < tb.n; i += gridDim.x * blockDim.x) {
        const int r = i / tb.Mr, il = i - r * tb.Mr;
        T acc = T(0);
        for (int q = tb.row_ptr[r]; q < tb.row_ptr[r + 1]; ++q)
            acc += bf.rbuf[((size_t)cw * tb.nT + tb.row_t[q]) * tb.Mr + il];
        out[(size_t)cw * tb.n + i] = acc;
    }
}

template <typename T>
__global__ void colgather_kernel(AmpTables<T> tb, AmpBufs<T> bf, T *out) {
    const int cw = blockIdx.y;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < tb.LM; j += gridDim.x * blockDim.x) {
        const int c = j / tb.Mc;
        out[(size_t)cw * tb.LM + j] = gather_u(tb, bf, cw, c, j - c * tb.Mc);
    }
}

template <typename T>
__global__ void cast_kernel(const void *in, int in_is_double, T *out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = in_is_double ? (T)((const double *)in)[i] : (T)((const float *)in)[i];
}
template <typename T>
__global__ void uncast_kernel(const T *in, double *out, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        out[i] = (double)in[i];
}

// Section / bit / codeword error counts and iteration sums (sparc_sim.py:27-37,
// calc_ber :62-70, calc_ser :72-98): bits of a section are the MSB-first binary
// digits of its index (sparc.py:182-197), so bit errors = popcount(idx ^ true).
__global__ void count_kernel(const int32_t *map_idx, const int32_t *true_idx, const int32_t *t_final, int L,
                             int logM, unsigned long long *counts) {
    __shared__ int red[2][4];
    const int cw = blockIdx.x;
    int sec = 0, bits = 0;
    for (int l = threadIdx.x; l < L; l += blockDim.x) {
        const int a = map_idx[(size_t)cw * L + l], b = true_idx[(size_t)cw * L + l];
        const int d = (a ^ b) & ((1 << logM) - 1);
        sec += (a != b);
        bits += __popc((unsigned)d);
    }
    for (int o = 32; o > 0; o >>= 1) {
        sec += __shfl_xor(sec, o, 64);
        bits += __shfl_xor(bits, o, 64);
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) { red[0][wid] = sec; red[1][wid] = bits; }
    __syncthreads();
    if (threadIdx.x == 0) {
        int s = 0, b = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { s += red[0][w]; b += red[1][w]; }
        atomicAdd(&counts[0], (unsigned long long)s);
        atomicAdd(&counts[1], (unsigned long long)b);
        atomicAdd(&counts[2], (unsigned long long)(s > 0));
        atomicAdd(&counts[3], (unsigned long long)t_final[cw]);
    }
}

// ------------------------------------------------------------------ launchers
static void col_geometry(int P, int Q, bool dbl, int *CT, int *nthr, int *ept) {
    int ct = dbl ? 8 : 16;
    const int cap = dbl ? 4096 : 8192;
    while (ct > 1 && ct * P > cap) ct >>= 1;
    if (ct > Q) ct = Q;
    const int total = ct * P;
    int nt = total / 8;
    if (nt > 256) nt = 256;
    if (nt < 1) nt = 1;
    *CT = ct;
    *nthr = nt;
    *ept = total / nt;
}

static void row_geometry(int Q, int *nthr, int *ept) {
    const int total = 2 * Q;
    int nt = total / 8;
    if (nt > 256) nt = 256;
    if (nt < 1) nt = 1;
    *nthr = nt;
    *ept = total / nt;
}

#define SG_EPT_DISPATCH(EPT_VAR, FN, TT, ...)                                                                 \
    do {                                                                                                      \
        switch (EPT_VAR) {                                                                                    \
            case 8: FN<TT, 8>(__VA_ARGS__); break;                                                             \
            case 16: FN<TT, 16>(__VA_ARGS__); break;                                                           \
            case 32: FN<TT, 32>(__VA_ARGS__); break;                                                           \
            default: return fail(SG_ERR_UNSUPPORTED, "FFT geometry EPT=%d unsupported", EPT_VAR);              \
        }                                                                                                     \
    } while (0)

template <typename T, int EPT>
static void launch_abA(const AmpTables<T> &tb, const AmpBufs<T> &bf, int CT, int nthr, hipStream_t s) {
    const size_t lds = sizeof(cx<T>) * (size_t)CT * tb.P;
    hipLaunchKernelGGL((ab_passA<T, EPT>), dim3(tb.Q / CT, tb.nT, bf.B), dim3(nthr), lds, s, tb, bf, CT);
}
template <typename T, int EPT>
static void launch_abB(const AmpTables<T> &tb, const AmpBufs<T> &bf, int nthr, hipStream_t s) {
    const size_t lds = sizeof(cx<T>) * 2 * (size_t)tb.Q;
    hipLaunchKernelGGL((ab_passB<T, EPT>), dim3(tb.npairs, tb.nT, bf.B), dim3(nthr), lds, s, tb, bf);
}
template <typename T, int EPT>
static void launch_azA(const AmpTables<T> &tb, const AmpBufs<T> &bf, int nthr, hipStream_t s) {
    const size_t lds = sizeof(cx<T>) * 2 * (size_t)tb.Q;
    hipLaunchKernelGGL((az_passA<T, EPT>), dim3(tb.npairs, tb.nT, bf.B), dim3(nthr), lds, s, tb, bf);
}
template <typename T, int EPT>
static void launch_azB(const AmpTables<T> &tb, const AmpBufs<T> &bf, int CT, int nthr, hipStream_t s) {
    const size_t lds = sizeof(cx<T>) * (size_t)CT * tb.P;
    hipLaunchKernelGGL((az_passB<T, EPT>), dim3(tb.Q / CT, tb.nT, bf.B), dim3(nthr), lds, s, tb, bf, CT);
}

template <typename T>
static int set_lds_limits() {
    static bool done = false;
    if (done) return SG_OK;
#define SG_LDS_ATTR(K) SG_HIP(hipFuncSetAttribute((const void *)(K), hipFuncAttributeMaxDynamicSharedMemorySize, 65536))
    SG_LDS_ATTR((ab_passA<T, 8>)); SG_LDS_ATTR((ab_passA<T, 16>)); SG_LDS_ATTR((ab_passA<T, 32>));
    SG_LDS_ATTR((ab_passB<T, 8>)); SG_LDS_ATTR((ab_passB<T, 16>)); SG_LDS_ATTR((ab_passB<T, 32>));
    SG_LDS_ATTR((az_passA<T, 8>)); SG_LDS_ATTR((az_passA<T, 16>)); SG_LDS_ATTR((az_passA<T, 32>));
    SG_LDS_ATTR((az_passB<T, 8>)); SG_LDS_ATTR((az_passB<T, 16>)); SG_LDS_ATTR((az_passB<T, 32>));
#undef SG_LDS_ATTR
    done = true;
    return SG_OK;
}

template <typename T>
int amp_launch_ab(const AmpTables<T> &tb, const AmpBufs<T> &bf, hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    SG_TRY(set_lds_limits<T>());
    int CT, nthr, ept;
    col_geometry(tb.P, tb.Q, sizeof(T) == 8, &CT, &nthr, &ept);
    {
        ProfScope ps(SG_PH_AB_A, s);
        SG_EPT_DISPATCH(ept, launch_abA, T, tb, bf, CT, nthr, s);
    }
    SG_HIP(hipGetLastError());
    row_geometry(tb.Q, &nthr, &ept);
    {
        ProfScope ps(SG_PH_AB_B, s);
        SG_EPT_DISPATCH(ept, launch_abB, T, tb, bf, nthr, s);
    }
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
int amp_launch_az(const AmpTables<T> &tb, const AmpBufs<T> &bf, hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    SG_TRY(set_lds_limits<T>());
    int CT, nthr, ept;
    row_geometry(tb.Q, &nthr, &ept);
    {
        ProfScope ps(SG_PH_AZ_A, s);
        SG_EPT_DISPATCH(ept, launch_azA, T, tb, bf, nthr, s);
    }
    SG_HIP(hipGetLastError());
    col_geometry(tb.P, tb.Q, sizeof(T) == 8, &CT, &nthr, &ept);
    {
        ProfScope ps(SG_PH_AZ_B, s);
        SG_EPT_DISPATCH(ept, launch_azB, T, tb, bf, CT, nthr, s);
    }
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
int amp_launch_eta(const AmpTables<T> &tb, const AmpBufs<T> &bf, hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    const int waves = 4;
    dim3 grid((tb.L + waves - 1) / waves, bf.B);
    const int epl = (tb.M + 63) / 64;
    ProfScope ps(SG_PH_ETA, s);
    if (epl <= 1) hipLaunchKernelGGL((eta_kernel<T, 1>), grid, dim3(64 * waves), 0, s, tb, bf);
    else if (epl <= 2) hipLaunchKernelGGL((eta_kernel<T, 2>), grid, dim3(64 * waves), 0, s, tb, bf);
    else if (epl <= 4) hipLaunchKernelGGL((eta_kernel<T, 4>), grid, dim3(64 * waves), 0, s, tb, bf);
    else if (epl <= 8) hipLaunchKernelGGL((eta_kernel<T, 8>), grid, dim3(64 * waves), 0, s, tb, bf);
    else if (epl <= 16) hipLaunchKernelGGL((eta_kernel<T, 16>), grid, dim3(64 * waves), 0, s, tb, bf);
    else if (epl <= 32) hipLaunchKernelGGL((eta_kernel<T, 32>), grid, dim3(64 * waves), 0, s, tb, bf);
    else return fail(SG_ERR_UNSUPPORTED, "section size M=%d > 2048 unsupported", tb.M);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
int amp_launch_control(const AmpTables<T> &tb, const AmpBufs<T> &bf, const AmpScalars &sc, const AmpParams &pr,
                       int phase, int t, hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    ProfScope ps(SG_PH_CONTROL, s);
    hipLaunchKernelGGL((control_kernel<T>), dim3(bf.B), dim3(1024), 0, s, tb, bf, sc, pr, phase, t);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
int amp_launch_rowsum(const AmpTables<T> &tb, const AmpBufs<T> &bf, T *out, hipStream_t s) {
    hipLaunchKernelGGL((rowsum_kernel<T>), dim3((tb.n + 255) / 256, bf.B), dim3(256), 0, s, tb, bf, out);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
int amp_launch_colgather(const AmpTables<T> &tb, const AmpBufs<T> &bf, T *out, hipStream_t s) {
    int gx = (tb.LM + 255) / 256;
    if (gx > 4096) gx = 4096;
    hipLaunchKernelGGL((colgather_kernel<T>), dim3(gx, bf.B), dim3(256), 0, s, tb, bf, out);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
int amp_launch_cast(const void *in, int in_is_double, T *out, size_t n, hipStream_t s) {
    if (!n) return SG_OK;
    size_t g = (n + 255) / 256;
    if (g > 65535) g = 65535;
    hipLaunchKernelGGL((cast_kernel<T>), dim3((unsigned)g), dim3(256), 0, s, in, in_is_double, out, n);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
int amp_launch_uncast(const T *in, double *out, size_t n, hipStream_t s) {
    if (!n) return SG_OK;
    size_t g = (n + 255) / 256;
    if (g > 65535) g = 65535;
    hipLaunchKernelGGL((uncast_kernel<T>), dim3((unsigned)g), dim3(256), 0, s, in, out, n);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

int amp_launch_count(const int32_t *map_idx, const int32_t *true_idx, const int32_t *t_final, int B, int L, int logM,
                     int64_t *counts, hipStream_t s) {
    if (B <= 0) return SG_OK;
    hipLaunchKernelGGL(count_kernel, dim3(B), dim3(256), 0, s, map_idx, true_idx, t_final, L, logM,
                       reinterpret_cast<unsigned long long *>(counts));
    SG_HIP(hipGetLastError());
    return SG_OK;
}

#define SG_INST(T)                                                                                            \
    template int amp_launch_ab<T>(const AmpTables<T> &, const AmpBufs<T> &, hipStream_t);                    \
    template int amp_launch_az<T>(const AmpTables<T> &, const AmpBufs<T> &, hipStream_t);                    \
    template int amp_launch_eta<T>(const AmpTables<T> &, const AmpBufs<T> &, hipStream_t);                   \
    template int amp_launch_control<T>(const AmpTables<T> &, const AmpBufs<T> &, const AmpScalars &,         \
                                       const AmpParams &, int, int, hipStream_t);                            \
    template int amp_launch_rowsum<T>(const AmpTables<T> &, const AmpBufs<T> &, T *, hipStream_t);           \
    template int amp_launch_colgather<T>(const AmpTables<T> &, const AmpBufs<T> &, T *, hipStream_t);        \
    template int amp_launch_cast<T>(const void *, int, T *, size_t, hipStream_t);                            \
    template int amp_launch_uncast<T>(const T *, double *, size_t, hipStream_t);
SG_INST(float)
SG_INST(double)

}  // namespace sg
