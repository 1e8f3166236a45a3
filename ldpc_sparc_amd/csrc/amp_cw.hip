// Per-codeword AMP engine on gfx950: one 512-thread workgroup per codeword
// runs a whole AMP iteration of the regular design (sparc.py:883-999 with the
// sub-sampled DCT operators of sub_dct :648-701) at the benchmark sizes.
//
// The staged engine (amp_fused.hip) spreads each transform over Q class
// workgroups and passes the needed rows T[m2][rho] / U[m2][rho] between its
// two FFT stages through HBM: ~9 MB per codeword-iteration at C2 on top of
// the 6 MB of s.  Here the Q-point stage is folded into the class loop
// instead:
//   Ab   for each class m2: beta of the class (from s, section max, 1/sum) ->
//        LDS scatter -> P-point FFT -> every needed index k = k1 + P k2
//        accumulates X[k] += w_N2^(m2 k1) w_Q^(m2 k2) Y[k1] in the registers
//        of the thread that owns k's row
//   ctrl X -> LDS; z = y - Re(c1 X[a] + c2 conj X[b]) + b z; phi, tau
//        (sparc.py:931-969); G[k] from z/phi (<= 4 terms) into the owners'
//        registers
//   Az   for each class m2: the owners write conj(w_N2^(m2 k1)) sum_k2
//        G[k] conj(w_Q^(m2 k2)) at row k1 of the zeroed LDS image ->
//        inverse P-point FFT -> s = beta_prev + tau u (sparc.py:972) in class
//        order -> per-section running max / rest sums merged class by class
//   merge section max and 1/sum, psi, NMSE, early stop (sparc.py:973-988)
// HBM traffic per codeword-iteration is s read twice and written once
// (3 * 4 LM bytes) plus z, y and the shared design tables.
#include "amp.hpp"

namespace sg {
namespace {

// hides the thread index from loop-invariant code motion, so the FFT's LDS
// addresses are recomputed per class instead of held across the class loop
__device__ __forceinline__ int cw_opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

__device__ __forceinline__ double cw_block_sum(double v, double *red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double t = 0.0;
    for (int w = 0; w < CW_THREADS / 64; ++w) t += red[w];
    return t;
}

constexpr int CW_CH = 8;   // global loads a thread issues before using them
constexpr int CW_CO = 16;  // output rows per thread (host: n <= CW_CO * CW_THREADS)
constexpr int CW_SPT = 2;  // sections per thread (host: Lblk <= CW_SPT * CW_THREADS)

}  // namespace

size_t cw_lds_bytes(int img, int KT, int Lblk, int nB, int Q) {
    return (size_t)img * 4 + (size_t)KT * CW_THREADS * 4 + (size_t)2 * Lblk * 4 + (size_t)(64 + nB + Q) * 8;
}

// class entries a thread holds: host checks largest class <= cw_sn(LOG2P) * CW_THREADS
constexpr int cw_sn(int log2p) { return 2 * ((1 << log2p) / CW_THREADS) + 4; }

// the class twiddle factors w_N2^(m2 k1) = twa[m2][k1 & 63] twb[m2][k1 >> 6]
// as one value per thread (64 + nB <= CW_THREADS, host-checked)
__device__ __forceinline__ cx<float> cw_tw_load(const CwTables &tb, int m2, int tl) {
    cx<float> v{0.f, 0.f};
    if (m2 < tb.Q && tl < 64 + tb.nB) v = tl < 64 ? tb.twa[m2 * 64 + tl] : tb.twb[m2 * tb.nB + tl - 64];
    return v;
}

#ifndef CW_FFT
#define CW_FFT lds_fft1_ct_lean
#endif

// diagnostics (SG_AMP_TPROF): thread 0 stamps the shader clock at point k
#define CW_TP(k)                                                                                                \
    do {                                                                                                        \
        if (tb.tprof && threadIdx.x == 0) tb.tprof[(size_t)blockIdx.x * 32 + (k)] = __builtin_readcyclecounter(); \
    } while (0)

template <int KT, int LOG2P>
__global__ __launch_bounds__(CW_THREADS) void cw_iter(CwTables tb, RegBufs<float> bf, AmpScalars sc, AmpParams pr,
                                                      int t) {
    constexpr int CW_P = 1 << LOG2P, CW_EPT = CW_P / CW_THREADS, CW_SN = cw_sn(LOG2P);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ double red[CW_THREADS / 64];
    // LDS: FFT / class image (also z / phi) | owned-index table | section
    // statistics of the previous beta | class twiddles
    cx<float> *d = reinterpret_cast<cx<float> *>(smem);
    float *dr = reinterpret_cast<float *>(smem);
    uint32_t *ktl = reinterpret_cast<uint32_t *>(dr + tb.img);
    float *sM = reinterpret_cast<float *>(ktl + KT * CW_THREADS);
    float *sI = sM + tb.Lblk;
    cx<float> *ta = reinterpret_cast<cx<float> *>(sI + tb.Lblk);
    cx<float> *tbb = ta + 64;
    cx<float> *twq = tbb + tb.nB;
    const int cw = blockIdx.x, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    const int qm = tb.Q - 1, Lb = tb.Lblk;
    const size_t lb = (size_t)cw * tb.L;
    const bool have_beta = t > 0;
    float inv_tp = 1.f;
    for (int i = tid; i < tb.Q; i += CW_THREADS) twq[i] = tb.twQ[i];
    for (int i = tid; i < KT * CW_THREADS; i += CW_THREADS) ktl[i] = tb.kt[i];
    if (have_beta) {
        for (int l = tid; l < Lb; l += CW_THREADS) {
            sM[l] = bf.stM[lb + l];
            sI[l] = bf.stI[lb + l];
        }
        const double tv = bf.tau[cw];
        inv_tp = (float)(1.0 / tv);
    }
    float *s = bf.s + (size_t)cw * tb.LM;
    cx<float> X[KT];
#pragma unroll
    for (int j = 0; j < KT; ++j) X[j] = {0.f, 0.f};
    CW_TP(0);
    __syncthreads();

    // ---------------------------------------------------------------- Ab
    if (have_beta) {
        for (int m2 = 0; m2 < tb.Q; ++m2) {
            const int tl = cw_opaque(tid);
            if (m2 == 2) CW_TP(8);
            // one round trip: the class twiddles, the class slice of s and its
            // table entries (clamped indices, every load issued together)
            const cx<float> tav = cw_tw_load(tb, m2, tl);
            const int q0 = tb.cls_ptr[m2], q1 = tb.cls_ptr[m2 + 1];
            float v[CW_SN];
            uint32_t e[CW_SN];
#pragma unroll
            for (int i = 0; i < CW_SN; ++i) {
                const int q = min(q0 + tl + i * CW_THREADS, q1 - 1);
                v[i] = s[q];
                e[i] = tb.cls_ls[q];
            }
            for (int i = tl; i < CW_P * 8 / 16; i += CW_THREADS) reinterpret_cast<uint4 *>(smem)[i] = uint4{0, 0, 0, 0};
            if (tl < 64 + tb.nB) ta[tl] = tav;
            __syncthreads();
            if (m2 == 2) CW_TP(9);
#pragma unroll
            for (int i = 0; i < CW_SN; ++i)
                if (q0 + tl + i * CW_THREADS < q1) {
                    const int l = e[i] >> 16;
                    dr[e[i] & 0xffffu] = __expf((v[i] - sM[l]) * inv_tp) * sI[l];  // beta = eta(s), sparc.py:429-432
                }
            __syncthreads();
            if (m2 == 2) CW_TP(10);
            CW_FFT<float, false, CW_EPT, LOG2P>(d, tb.stw, tl);
            if (m2 == 2) CW_TP(11);
#pragma unroll
            for (int j = 0; j < KT; ++j) {  // invalid entries accumulate into unused slots
                const uint32_t kv = ktl[j * CW_THREADS + tl];
                const int k1 = kv & 0x3fff, k2 = (kv >> 14) & 63;
                const cx<float> Tv = cmul(d[fsw(k1)], cmul(ta[k1 & 63], tbb[k1 >> 6]));
                const cx<float> w = twq[(m2 * k2) & qm];
                X[j].x += Tv.x * w.x - Tv.y * w.y;
                X[j].y += Tv.x * w.y + Tv.y * w.x;
            }
            __syncthreads();
            if (m2 == 2) CW_TP(12);
        }
    }
    CW_TP(1);

    // ---------------------------------------------------------------- control
    double *psi = sc.psi + cw, *psi_prev = sc.psi_prev + cw;
    float *z = bf.z + (size_t)cw * tb.n;
    const float *y = bf.y + (size_t)cw * tb.n;
    const bool sum_z = pr.phi_method != 1;
    double g;
    float bco = 0.f;
    if (have_beta) {
        const double ps = *psi, ph = bf.phi[cw];
        g = pr.W[0] * ps;  // ndim 0: gamma = W psi (sparc.py:938-940)
        if (tid == 0) {
            *psi_prev = ps;
            bf.tau_prev[cw] = bf.tau[cw];
            sc.phi_prev[cw] = ph;
            sc.gamma[cw] = g;
            sc.bcoef[cw] = g / ph;
        }
        bco = (float)(g / ph);
        // compact X to the codeword's scratch (one CU: the workgroup's own
        // stores are visible to its loads after the barrier)
        cx<float> *xg = bf.xn + (size_t)cw * KT * CW_THREADS;
#pragma unroll
        for (int j = 0; j < KT; ++j) xg[j * CW_THREADS + tid] = X[j];
        __syncthreads();
    } else {
        g = pr.W[0];
        if (tid == 0) sc.gamma[cw] = g;
    }
    float zr[CW_CO];
    double acc = 0.0;
    {
        float yv[CW_CO], zv[CW_CO];
        int ia[CW_CO], ib[CW_CO];
        cx<float> c1[CW_CO], c2[CW_CO];
#pragma unroll
        for (int k = 0; k < CW_CO; ++k) {  // clamped indices: every load of the round issued together
            const int i = min(tid + k * CW_THREADS, tb.n - 1);
            yv[k] = y[i];
            if (have_beta) {
                zv[k] = z[i];
                ia[k] = tb.oa[i];
                ib[k] = tb.ob[i];
                c1[k] = tb.oc[2 * i];
                c2[k] = tb.oc[2 * i + 1];
            }
        }
        cx<float> ha[CW_CO], hb[CW_CO];
        if (have_beta) {
            const cx<float> *xg = bf.xn + (size_t)cw * KT * CW_THREADS;
#pragma unroll
            for (int k = 0; k < CW_CO; ++k) {
                ha[k] = xg[ia[k]];
                hb[k] = xg[ib[k]];
            }
        }
#pragma unroll
        for (int k = 0; k < CW_CO; ++k) {
            float zn = yv[k];
            if (have_beta) {  // Onsager residual, sparc.py:943-946
                float r = 0.f;
                r += (c1[k].x * ha[k].x - c1[k].y * ha[k].y) + (c2[k].x * hb[k].x + c2[k].y * hb[k].y);
                zn = (yv[k] - r) + bco * zv[k];
            }
            zr[k] = zn;
        }
    }
#pragma unroll
    for (int k = 0; k < CW_CO; ++k) {
        const int i = tid + k * CW_THREADS;
        if (i < tb.n) {
            z[i] = zr[k];
            if (sum_z) acc += (double)zr[k] * (double)zr[k];
        }
    }
    double phi;
    if (sum_z) {
        phi = cw_block_sum(acc, red) / (double)tb.n;  // sparc.py:949-955
    } else {
        __syncthreads();
        phi = pr.awgn_var + g;
    }
    const double tv_new = (tb.L * phi / tb.n) / pr.W[0];  // sparc.py:958-969
    if (tid == 0) {
        bf.phi[cw] = phi;
        bf.tau[cw] = tv_new;
    }
    const float tau = (float)tv_new, inv_tau = (float)(1.0 / tv_new);
    const float phf = (float)phi;
    float *zl = dr;  // z / phi, sparc.py:972
#pragma unroll
    for (int k = 0; k < CW_CO; ++k) {
        const int i = tid + k * CW_THREADS;
        if (i < tb.n) zl[i] = zr[k] / phf;
    }
    __syncthreads();
    {
        // G[k] of the owned indices (unused terms: index 0, coefficient 0), four
        // indices per round: each round's table loads wait for the previous
        // round's results, which bounds the registers in flight
        int tc = tid;
#pragma unroll
        for (int j0 = 0; j0 < KT; j0 += 4) {
            int4 gi[4];
            float4 ga[4], gb[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = (j0 + j) * CW_THREADS + tc;
                gi[j] = reinterpret_cast<const int4 *>(tb.gi)[c];
                ga[j] = reinterpret_cast<const float4 *>(tb.gc)[2 * c];
                gb[j] = reinterpret_cast<const float4 *>(tb.gc)[2 * c + 1];
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                cx<float> a{0.f, 0.f};
                float v = zl[gi[j].x];
                a.x += ga[j].x * v;
                a.y += ga[j].y * v;
                v = zl[gi[j].y];
                a.x += ga[j].z * v;
                a.y += ga[j].w * v;
                v = zl[gi[j].z];
                a.x += gb[j].x * v;
                a.y += gb[j].y * v;
                v = zl[gi[j].w];
                a.x += gb[j].z * v;
                a.y += gb[j].w * v;
                X[j0 + j] = a;
                asm volatile("" : "+v"(tc) : "v"(a.x), "v"(a.y));
            }
        }
    }
    __syncthreads();
    CW_TP(2);

    // ---------------------------------------------------------------- Az
    // running statistics of s_new for the thread's sections l = tid + r * CW_THREADS
    float Mr[CW_SPT], R1[CW_SPT], R2[CW_SPT], s_true[CW_SPT];
    int jt[CW_SPT];
#pragma unroll
    for (int r = 0; r < CW_SPT; ++r) {
        const int l = tid + r * CW_THREADS;
        Mr[r] = -INFINITY;
        R1[r] = R2[r] = s_true[r] = 0.f;
        jt[r] = -1;
        if (bf.true_idx && l < Lb) jt[r] = tb.qpos[l * tb.M + bf.true_idx[lb + l]];
    }
    for (int m2 = 0; m2 < tb.Q; ++m2) {
        const int tl = cw_opaque(tid);
        if (m2 == 2) CW_TP(16);
        const cx<float> tav = cw_tw_load(tb, m2, tl);
        for (int i = tl; i < CW_P * 8 / 16; i += CW_THREADS) reinterpret_cast<uint4 *>(smem)[i] = uint4{0, 0, 0, 0};
        if (tl < 64 + tb.nB) ta[tl] = tav;
        __syncthreads();
        if (m2 == 2) CW_TP(17);
        {
            cx<float> u{0.f, 0.f};
#pragma unroll
            for (int j = 0; j < KT; ++j) {
                const uint32_t e = ktl[j * CW_THREADS + tl];
                const int k1 = e & 0x3fff, k2 = (e >> 14) & 63;
                if (e & CW_NEWROW) u = {0.f, 0.f};
                const cx<float> w = twq[(m2 * k2) & qm];  // G conj(w)
                u.x += X[j].x * w.x + X[j].y * w.y;
                u.y += X[j].y * w.x - X[j].x * w.y;
                if (e & CW_ENDROW) d[fsw(k1)] = cmul(u, cconj(cmul(ta[k1 & 63], tbb[k1 >> 6])));
            }
        }
        __syncthreads();
        if (m2 == 2) CW_TP(18);
        CW_FFT<float, true, CW_EPT, LOG2P>(d, tb.stw, tl);
        if (m2 == 2) CW_TP(19);
        // one round trip: the class slice of s_prev and its table entries
        const int tg = cw_opaque(tl);
        const int q0 = tb.cls_ptr[m2], q1 = tb.cls_ptr[m2 + 1];
        float v[CW_SN];
        uint32_t e[CW_SN];
#pragma unroll
        for (int i = 0; i < CW_SN; ++i) {
            const int q = min(q0 + tg + i * CW_THREADS, q1 - 1);
            e[i] = tb.cls_ls[q];
            v[i] = s[q];  // (t = 0: unused)
        }
        float snv[CW_SN];
#pragma unroll
        for (int i = 0; i < CW_SN; ++i) {
            const int l = e[i] >> 16;
            const float b = have_beta ? __expf((v[i] - sM[l]) * inv_tp) * sI[l] : 0.f;
            snv[i] = b + tau * dr[e[i] & 0xffffu];
        }
        if (m2 == 2) CW_TP(20);
        __syncthreads();
#pragma unroll
        for (int c = 0; c < CW_SN; ++c) {  // s of the class in class order, skewed by fpad
            const int q = q0 + tl + c * CW_THREADS;
            if (q < q1) dr[fpad(q - q0)] = snv[c];
        }
        __syncthreads();
        if (m2 == 2) CW_TP(21);
        const uint16_t *sg = tb.seg + (size_t)m2 * (Lb + 1);
#pragma unroll
        for (int r = 0; r < CW_SPT; ++r) {
            const int l = tl + r * CW_THREADS;
            if (l >= Lb) continue;
            // partial of section l over its segment of the class: running
            // maximum, sums without the (first) maximum (amp_fused.hip az_stage2)
            const int a = sg[l], b = sg[l + 1];
            constexpr int RC = 16;
            float m = -INFINITY, S1 = 0.f, S2 = 0.f;
            for (int c = a; c < b; c += RC) {
                float v[RC];
#pragma unroll
                for (int i = 0; i < RC; ++i) v[i] = dr[fpad(c + i)];  // inside the LDS image; masked below
#pragma unroll
                for (int i = 0; i < RC; ++i)
                    if (c + i < b) {
                        const bool up = v[i] > m;
                        const float dlt = up ? (m - v[i]) : (v[i] - m);
                        const float e = __expf(dlt * inv_tau);
                        S1 = up ? (S1 + 1.f) * e : S1 + e;
                        S2 = up ? (S2 + 1.f) * (e * e) : S2 + e * e;
                        m = up ? v[i] : m;
                    }
            }
            if (m > -INFINITY) {  // merge into the section's running statistics
                if (m > Mr[r]) {
                    const float f = __expf((Mr[r] - m) * inv_tau);
                    R1[r] = (R1[r] + 1.f) * f + S1;
                    R2[r] = (R2[r] + 1.f) * (f * f) + S2;
                    Mr[r] = m;
                } else {
                    const float f = __expf((m - Mr[r]) * inv_tau);
                    R1[r] += (1.f + S1) * f;
                    R2[r] += (1.f + S2) * (f * f);
                }
            }
            if (jt[r] >= q0 && jt[r] < q1) s_true[r] = dr[fpad(jt[r] - q0)];
        }
        if (m2 == 2) CW_TP(22);
        for (int q = q0 + tl; q < q1; q += CW_THREADS) s[q] = dr[fpad(q - q0)];
        __syncthreads();
        if (m2 == 2) CW_TP(23);
    }
    CW_TP(3);

    // ---------------------------------------------------------------- merge
    double a = 0.0, e = 0.0;
#pragma unroll
    for (int r = 0; r < CW_SPT; ++r) {
        const int l = tid + r * CW_THREADS;
        if (l >= Lb) continue;
        const float inv = 1.f / (1.f + R1[r]);
        bf.stM[lb + l] = Mr[r];
        bf.stI[lb + l] = inv;
        // 1 - sum beta^2 = (2 R1 + R1^2 - R2) / (1 + R1)^2, no cancellation
        const double i2 = (double)inv * (double)inv, r1 = R1[r], r2 = R2[r];
        a += (2.0 * r1 + r1 * r1 - r2) * i2;
        if (jt[r] >= 0) {
            if (s_true[r] == Mr[r]) {
                e += (r1 * r1 + r2) * i2;
            } else {
                const double bt = (double)(__expf((s_true[r] - Mr[r]) * inv_tau) * inv);
                e += (1.0 + r2) * i2 - 2.0 * bt + 1.0;
            }
        }
    }
    a = cw_block_sum(a, red);
    e = cw_block_sum(e, red);
    if (tid == 0) {
        double *nmse = sc.nmse + (size_t)cw * pr.t_max;
        const double denom = (double)tb.L;
        const double pnew = a / denom;
        *psi = pnew;
        nmse[t + 1] = e / denom;
        bool stop = false;
        if (t > 0) {
            const double pp = *psi_prev;
            stop = fabs(pnew - pp) <= pr.atol + pr.rtol * fabs(pp);  // sparc.py:984-986
        }
        if (stop) {  // nmse[t:] = nmse[t] (sparc.py:985)
            for (int tt = t + 1; tt < pr.t_max; ++tt) nmse[tt] = nmse[t];
            sc.t_final[cw] = t + 1;
            bf.active[cw] = 0;
        } else if (t == pr.t_max - 2) {
            sc.t_final[cw] = t + 1;
            bf.active[cw] = 0;
        }
    }
    CW_TP(4);
}

template <int KT, int LOG2P>
static int cw_launch(const CwTables &tb, const RegBufs<float> &bf, const AmpScalars &sc, const AmpParams &pr, int t,
                     hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        // (the block-sum scratch is static LDS on top of the dynamic part)
        SG_HIP(hipFuncSetAttribute((const void *)cw_iter<KT, LOG2P>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024 - 1024));
        attr = true;
    }
    const size_t lds = cw_lds_bytes(tb.img, KT, tb.Lblk, tb.nB, tb.Q);
    if (lds > 160 * 1024 - 1024) return fail(SG_ERR_UNSUPPORTED, "per-codeword engine: %zu bytes of LDS", lds);
    hipLaunchKernelGGL((cw_iter<KT, LOG2P>), dim3(bf.B), dim3(CW_THREADS), lds, s, tb, bf, sc, pr, t);
    return SG_OK;
}

template <int LOG2P>
static int cw_dispatch(const CwTables &tb, const RegBufs<float> &bf, const AmpScalars &sc, const AmpParams &pr, int t,
                       hipStream_t s) {
    if (tb.maxcls > cw_sn(LOG2P) * CW_THREADS)
        return fail(SG_ERR_UNSUPPORTED, "per-codeword engine: a class of %d entries", tb.maxcls);
    switch (tb.KT) {
    case 24: return cw_launch<24, LOG2P>(tb, bf, sc, pr, t, s);
    case 28: return cw_launch<28, LOG2P>(tb, bf, sc, pr, t, s);
    case 32: return cw_launch<32, LOG2P>(tb, bf, sc, pr, t, s);
    default: return fail(SG_ERR_UNSUPPORTED, "per-codeword engine: %d indices per thread", tb.KT);
    }
}

int cw_launch_iter(const CwTables &tb, const RegBufs<float> &bf, const AmpScalars &sc, const AmpParams &pr, int t,
                   hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    if (tb.n > CW_CO * CW_THREADS || tb.Lblk > CW_SPT * CW_THREADS || tb.Q > 64 || 64 + tb.nB > CW_THREADS)
        return fail(SG_ERR_UNSUPPORTED, "per-codeword engine: sizes outside its compile-time bounds");
    ProfScope ps(SG_PH_AMP_CW, s);
    if (tb.log2P == 13) SG_TRY(cw_dispatch<13>(tb, bf, sc, pr, t, s));
    else return fail(SG_ERR_UNSUPPORTED, "per-codeword engine: P = 2^%d", tb.log2P);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

}  // namespace sg
