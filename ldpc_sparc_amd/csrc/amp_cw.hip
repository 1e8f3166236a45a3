// Per-codeword AMP engine on gfx950: one 1024-thread workgroup per codeword
// runs a whole AMP iteration of the regular design (sparc.py:883-999 with the
// sub-sampled DCT operators of sub_dct :648-701).
//
// The staged engine (amp_fused.hip) spreads each transform over Q class
// workgroups and passes the needed rows T[m2][rho] / U[m2][rho] between its
// two FFT stages through HBM: ~9 MB per codeword-iteration at C2 on top of
// the 6 MB of s.  Here the Q-point stage is folded into the class loop, and
// the needed spectrum X (then G) stays in LDS for the whole iteration:
//   Ab   for each class m2: beta of the class (from s, section max, 1/sum) ->
//        LDS scatter -> P-point FFT -> every needed index k = k1 + P k2
//        accumulates X[k] += w_N2^(m2 k1) w_Q^(m2 k2) Y[k1]
//   ctrl z = y - Re(c1 X[a] + c2 conj X[b]) + b z; phi, tau
//        (sparc.py:931-969); G[k] from z/phi (<= 4 terms) replaces X
//   Az   for each class m2: the thread owning a row writes conj(w_N2^(m2 k1))
//        sum_k2 G[k] conj(w_Q^(m2 k2)) at row k1 of the zeroed LDS image ->
//        inverse P-point FFT -> s = beta_prev + tau u (sparc.py:972) in class
//        order -> per-section running max / rest sums merged class by class
//   merge section max and 1/sum, psi, NMSE, early stop (sparc.py:973-988)
// LDS: the P-point image (64 KB) and X/G (12 x 1024 slots, 96 KB) -- all of it.
// The class slice of s and its table entries for class m2 + 1 are in flight
// in registers under class m2's accumulation (Ab) or store and statistics
// (Az); every twiddle comes from the hardware sine / cosine.  HBM traffic per
// codeword-iteration is s read twice and written once (3 * 4 LM bytes) plus
// z, y and the tables shared by every codeword (L2-resident).
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

constexpr int CW_LOG2P = 13, CW_P = 1 << CW_LOG2P, CW_EPT = CW_P / CW_THREADS;
constexpr int CW_SN = 9;   // class entries per thread (host: largest class <= CW_SN * 1024)
constexpr int CW_CO = 8;   // output rows per thread (host: n <= CW_CO * 1024)
constexpr int CW_KL = 12;  // X / G slots per thread in LDS (96 KB); any further ones in registers

// w_N2^j = exp(-2 pi i j / N2) from the hardware sine / cosine, whose
// argument is in revolutions: j mod N2 scaled by 1/N2 is exact in f32
// (N2 <= 2^19).  For needed index k = k1 + P k2 and class m2,
// w_N2^(m2 k) = w_N2^(m2 k1) w_Q^(m2 k2) is the whole factor of the folded
// Q-point stage.
__device__ __forceinline__ cx<float> cw_w(const CwTables &tb, uint32_t j) {
    const float x = (float)(j & (uint32_t)(tb.N2 - 1)) * tb.inv_n2;
    return {__builtin_amdgcn_cosf(x), -__builtin_amdgcn_sinf(x)};
}

// Radix plan of the P-point FFT at 8 values per thread (CW_RADIX_PLAN 0:
// fft.hpp's 4, 4, 8, 8, 8; 1: 8, 8, 8, 8, 2; 2: 2, 8, 8, 8, 8; 3: 16, 8, 8, 8
// with the radix-16 first stage split over lanes l and l ^ 32, cw_stage0_r16)
#ifndef CW_RADIX_PLAN
#define CW_RADIX_PLAN 3
#endif
constexpr int cw_nstages() { return CW_RADIX_PLAN == 3 ? 4 : 5; }
constexpr int cw_radix(int st) {
    return CW_RADIX_PLAN == 0   ? fft1_radix_ct(CW_LOG2P, CW_EPT, st)
           : CW_RADIX_PLAN == 1 ? (st < 4 ? 8 : 2)
           : CW_RADIX_PLAN == 2 ? (st == 0 ? 2 : 8)
                                : (st == 0 ? 16 : 8);
}
constexpr int cw_log2ns(int st) {
    int l = 0;
    for (int i = 0; i < st; ++i) l += cw_radix(i) == 2 ? 1 : cw_radix(i) == 4 ? 2 : cw_radix(i) == 8 ? 3 : 4;
    return l;
}

// lanes 32..63 of a <-> lanes 0..31 of b (v_permlane32_swap, no LDS)
__device__ __forceinline__ void cw_swap32(cx<float> &a, cx<float> &b) {
    const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
    const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
    a = {__uint_as_float(rx[0]), __uint_as_float(ry[0])};
    b = {__uint_as_float(rx[1]), __uint_as_float(ry[1])};
}

// First Stockham stage at radix 16 (Ns = 1, no twiddles) with 8 values per
// thread: butterfly j = 32 w + (l & 31) of wavefront w is shared by lanes l
// and l ^ 32, lane half H holding inputs m = 8 H + jj (x[j + 512 m]).  A
// radix-2 step across the halves (two rounds of permlane32 swaps) and a
// radix-8 DFT in registers give lane half H the outputs 2 q + H, stored at
// j 16 + 2 q + H like stockham1_stage_ct's.  With CW_MASKIN the image is not
// zeroed before the class scatter / row writes: bit 2 jj + c of msk says
// whether component c of value jj was written for this transform (host
// table, capi_amp.cpp build_cw), and the stale ones read as zero.
#ifndef CW_MASKIN
#define CW_MASKIN 1
#endif
template <bool INV>
__device__ __forceinline__ void cw_stage0_r16(cx<float> *d, int tid, uint32_t msk) {
    const int l = tid & 63, H = l >> 5, j = ((tid >> 6) << 5) | (l & 31);
    cx<float> v[8];
    const int jp = fsw(j);  // adding multiples of 256 commutes with the swizzle
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) v[jj] = d[jp + ((8 * H + jj) << 9)];
    if constexpr (CW_MASKIN) {
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {  // all-ones / zero from the sign-extended bit
            const uint32_t mx = (uint32_t)((int)(msk << (31 - 2 * jj)) >> 31);
            const uint32_t my = (uint32_t)((int)(msk << (30 - 2 * jj)) >> 31);
            v[jj] = {__uint_as_float(__float_as_uint(v[jj].x) & mx), __uint_as_float(__float_as_uint(v[jj].y) & my)};
        }
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) cw_swap32(v[jj], v[jj + 4]);  // lane half H: x[J], x[8 + J], J = jj + 4 H
    {
        constexpr float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f, r2 = 0.70710678118654752440f;
        const cx<float> w16[4] = {{1.f, 0.f}, {c1, INV ? s1 : -s1}, {r2, INV ? r2 : -r2}, {s1, INV ? c1 : -c1}};
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const cx<float> u = v[jj], x8 = v[jj + 4];
            v[jj] = cadd(u, x8);
            const cx<float> t = jj == 0 ? csub(u, x8) : cmul(csub(u, x8), w16[jj]);  // (u - x8) w16^jj
            v[jj + 4] = H ? mul_mi<float, INV>(t) : t;                                 // * w16^(4 H)
        }
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) cw_swap32(v[jj], v[jj + 4]);  // lane half p: y_p[0..7]
    dft8<float, INV>(v);                                         // v[q] = X_j[2 q + H]
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) d[fsw((j << 4) | (q << 1) | H)] = v[q];
    __syncthreads();
}

// The P-point LDS FFT (fft.hpp stages) with its stage twiddles
// w_{Ns R}^(e k) from the hardware sine / cosine instead of a table: no
// global loads between its barriers.
template <bool INV, int ST>
__device__ __forceinline__ void cw_fft_from(cx<float> *d, int tid, uint32_t msk = 0xffffu) {
    static_assert(!CW_MASKIN || cw_radix(0) == 16, "the masked first stage is the radix-16 one");
    if constexpr (ST == 0 && cw_radix(0) == 16) {
        cw_stage0_r16<INV>(d, tid, msk);
        cw_fft_from<INV, 1>(d, tid);
    } else if constexpr (ST < cw_nstages()) {
        constexpr int R = cw_radix(ST), LNS = cw_log2ns(ST);
        constexpr int NB = CW_EPT / R, TWN = tw_per_k(R);
        cx<float> wl[LNS > 0 ? NB * TWN : 1];
        if constexpr (LNS > 0) {
            constexpr int LR = R == 2 ? 1 : R == 4 ? 2 : R == 8 ? 3 : 4;
            constexpr float inv = 1.0f / (float)(1 << (LNS + LR));
#pragma unroll
            for (int i = 0; i < NB; ++i) {
                const int k = (tid + i * CW_THREADS) & ((1 << LNS) - 1);
#pragma unroll
                for (int q = 0; q < TWN; ++q) {
                    const float x = (float)((tw_exp(R, q) * k) & ((1 << (LNS + LR)) - 1)) * inv;
                    wl[i * TWN + q] = {__builtin_amdgcn_cosf(x), -__builtin_amdgcn_sinf(x)};
                }
            }
        }
        stockham1_stage_ct<float, INV, R, CW_EPT, CW_LOG2P, LNS>(d, wl, tid);
        cw_fft_from<INV, ST + 1>(d, tid);
    }
}

}  // namespace

size_t cw_lds_bytes(int img, int nslots) { return (size_t)img * 4 + (size_t)nslots * 8; }

// diagnostics (SG_AMP_TPROF): thread 0 stamps the shader clock at point k
#define CW_TP(k)                                                                                                \
    do {                                                                                                        \
        if (tb.tprof && threadIdx.x == 0) tb.tprof[(size_t)blockIdx.x * 32 + (k)] = __builtin_readcyclecounter(); \
    } while (0)

// Ab accumulation of one class: X[slot] += w_N2^(m2 k) Y[k1] for the thread's
// slots.  The image and the X slots are disjoint LDS regions; saying so
// (restrict) lets the compiler issue the slots' reads together instead of one
// read-modify-write round trip after the other.
template <int KT>
__device__ __forceinline__ void cw_accumulate(const cx<float> *__restrict__ img, cx<float> *__restrict__ xs,
                                              cx<float> *xr, const uint32_t *kt, const cx<float> *w, int tl) {
    // slot j + 1's reads are issued before slot j's write (a two-deep pipeline:
    // the compiler keeps LDS reads and writes in program order here)
    auto ld = [&](int j, cx<float> &T, cx<float> &x) {
        T = img[fsw(kt[j] & (CW_P - 1))];
        x = j < CW_KL ? xs[j * CW_THREADS + tl] : xr[j < CW_KL ? 0 : j - CW_KL];
    };
    cx<float> Tn, xn;
    ld(0, Tn, xn);
#pragma unroll
    for (int j = 0; j < KT; ++j) {  // invalid slots accumulate into themselves, unused
        const cx<float> Tv = Tn;
        cx<float> x = xn;
        if (j + 1 < KT) ld(j + 1 < KT ? j + 1 : j, Tn, xn);
        x = cmac_pk(x, Tv, w[j]);
        if (j < CW_KL) xs[j * CW_THREADS + tl] = x;
        else xr[j < CW_KL ? 0 : j - CW_KL] = x;
    }
}

// Az rows of one class: the thread's rows of sum_k G[k] conj(w_N2^(m2 k)) into
// the image (disjoint from the G slots: restrict, as above)
template <int KT>
__device__ __forceinline__ void cw_rows(const cx<float> *__restrict__ gs, cx<float> *__restrict__ img,
                                        const cx<float> *xr, const uint32_t *kt, const cx<float> *w, int tl) {
    cx<float> u{0.f, 0.f};
#pragma unroll
    for (int j = 0; j < KT; ++j) {
        if (!(kt[j] & CW_VALID)) continue;
        const cx<float> gv = j < CW_KL ? gs[j * CW_THREADS + tl] : xr[j < CW_KL ? 0 : j - CW_KL];
        if (kt[j] & CW_NEWROW) u = {0.f, 0.f};
        u = cmacc_pk(u, gv, w[j]);  // G conj(w_N2^(m2 k))
        if (kt[j] & CW_ENDROW) img[fsw(kt[j] & (CW_P - 1))] = u;
    }
}

template <int KT>
__global__ __launch_bounds__(CW_THREADS) void cw_iter(CwTables tb, RegBufs<float> bf, AmpScalars sc, AmpParams pr,
                                                      int t) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cx<float> *d = reinterpret_cast<cx<float> *>(smem);
    float *dr = reinterpret_cast<float *>(smem);
    cx<float> *Xl = reinterpret_cast<cx<float> *>(dr + tb.img);   // X, then G, by slot
    double *red = reinterpret_cast<double *>(smem) + (CW_P - 16);  // block sums: the image's last 128 B
    const int cw = blockIdx.x, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    const size_t lb = (size_t)cw * tb.L;
    const bool have_beta = t > 0;
    const float *stM = bf.stM + lb, *stI = bf.stI + lb;  // previous beta's section max, 1/sum (L1)
    const float inv_tp = have_beta ? (float)(1.0 / bf.tau[cw]) : 1.f;
    float *s = bf.s + (size_t)cw * tb.LM;
    // owned needed indices k | flags, slot j * 1024 + tid of X / G
    constexpr int KR = KT > CW_KL ? KT - CW_KL : 1;  // register-held slots (j >= CW_KL)
    uint32_t kt[KT];
    cx<float> Xr[KR];
#pragma unroll
    for (int j = 0; j < KT; ++j) {
        kt[j] = tb.kt[j * CW_THREADS + tid];
        if (j < CW_KL) Xl[j * CW_THREADS + tid] = {0.f, 0.f};
        else Xr[j - CW_KL] = {0.f, 0.f};
    }
    CW_TP(0);

    // ---------------------------------------------------------------- Ab
    if (have_beta) {
        float v[CW_SN];
        uint32_t e[CW_SN];
        int q0 = tb.cls_ptr[0], q1 = tb.cls_ptr[1];
#pragma unroll
        for (int i = 0; i < CW_SN; ++i) {
            const int q = min(q0 + tid + i * CW_THREADS, q1 - 1);
            v[i] = s[q];
            e[i] = tb.cls_ls[q];
        }
        // section max and 1/sum of the class's entries; with CW_MASKIN those of
        // class m2 + 1 are gathered before class m2's closing barrier (not with
        // register-held slots: <14> then spills 12 VGPRs)
        constexpr bool early = CW_MASKIN && KT <= CW_KL;
        float bm[CW_SN], bi[CW_SN];
        auto gather_stats = [&]() {
#pragma unroll
            for (int i = 0; i < CW_SN; ++i) {
                const int l = e[i] >> 16;
                bm[i] = stM[l];
                bi[i] = stI[l];
            }
        };
        if constexpr (early) gather_stats();
        for (int m2 = 0; m2 < tb.Q; ++m2) {
            const int tl = cw_opaque(tid);
            if (m2 == 2) CW_TP(8);
            if constexpr (!CW_MASKIN)
                for (int i = tl; i < CW_P * 8 / 16; i += CW_THREADS) reinterpret_cast<uint4 *>(smem)[i] = uint4{0, 0, 0, 0};
            if constexpr (!early) gather_stats();
            if constexpr (!CW_MASKIN) __syncthreads();  // (masked: the previous class's closing barrier)
            if (m2 == 2) CW_TP(9);
#pragma unroll
            for (int i = 0; i < CW_SN; ++i)
                if (q0 + tl + i * CW_THREADS < q1)  // beta = eta(s), sparc.py:429-432
                    dr[e[i] & 0xffffu] = __expf((v[i] - bm[i]) * inv_tp) * bi[i];
            const uint32_t cmk = CW_MASKIN ? tb.cmask[m2 * CW_THREADS + tl] : 0xffffu;  // under the barrier
            __syncthreads();
            if (m2 == 2) CW_TP(10);
            cw_fft_from<false, 0>(d, tl, cmk);
            if (m2 == 2) CW_TP(11);
            if (m2 + 1 < tb.Q) {  // the next class in flight under the accumulation
                const int tn = cw_opaque(tl);
                q0 = tb.cls_ptr[m2 + 1];
                q1 = tb.cls_ptr[m2 + 2];
#pragma unroll
                for (int i = 0; i < CW_SN; ++i) {
                    const int q = min(q0 + tn + i * CW_THREADS, q1 - 1);
                    v[i] = s[q];
                    e[i] = tb.cls_ls[q];
                }
            }
            {
                cx<float> w[KT];
#pragma unroll
                for (int j = 0; j < KT; ++j) w[j] = cw_w(tb, (uint32_t)m2 * (kt[j] & CW_KMASK));
                cw_accumulate<KT>(d, Xl, Xr, kt, w, tl);
            }
            if (early && m2 + 1 < tb.Q) gather_stats();
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
        if constexpr (KT > CW_KL) {  // the register-held slots into the (free) image for the residual
            __syncthreads();
#pragma unroll
            for (int j = CW_KL; j < KT; ++j) d[(j - CW_KL) * CW_THREADS + tid] = Xr[j - CW_KL];
            __syncthreads();
        }
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
#pragma unroll
        for (int k = 0; k < CW_CO; ++k) {
            float zn = yv[k];
            if (have_beta) {  // Onsager residual, sparc.py:943-946
                cx<float> ha, hb;
                if constexpr (KT > CW_KL) {
                    ha = ia[k] < CW_KL * CW_THREADS ? Xl[ia[k]] : d[ia[k] - CW_KL * CW_THREADS];
                    hb = ib[k] < CW_KL * CW_THREADS ? Xl[ib[k]] : d[ib[k] - CW_KL * CW_THREADS];
                } else {
                    ha = Xl[ia[k]];
                    hb = Xl[ib[k]];
                }
                float r = 0.f;
                r += (c1[k].x * ha.x - c1[k].y * ha.y) + (c2[k].x * hb.x + c2[k].y * hb.y);
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
    float *zl = dr + (KT > CW_KL ? 2 * (KT - CW_KL) * CW_THREADS : 0);  // z / phi (sparc.py:972), after those slots
#pragma unroll
    for (int k = 0; k < CW_CO; ++k) {
        const int i = tid + k * CW_THREADS;
        if (i < tb.n) zl[i] = zr[k] / phf;
    }
    __syncthreads();
    // G by slot (unused terms: index 0, coefficient 0)
    for (int c = tid; c < CW_KL * CW_THREADS; c += CW_THREADS) {
        const int4 gi = reinterpret_cast<const int4 *>(tb.gi)[c];
        const float4 ga = reinterpret_cast<const float4 *>(tb.gc)[2 * c];
        const float4 gb = reinterpret_cast<const float4 *>(tb.gc)[2 * c + 1];
        cx<float> a{0.f, 0.f};
        float v = zl[gi.x];
        a.x += ga.x * v;
        a.y += ga.y * v;
        v = zl[gi.y];
        a.x += ga.z * v;
        a.y += ga.w * v;
        v = zl[gi.z];
        a.x += gb.x * v;
        a.y += gb.y * v;
        v = zl[gi.w];
        a.x += gb.z * v;
        a.y += gb.w * v;
        Xl[c] = a;
    }
    if constexpr (KT > CW_KL) {
#pragma unroll
        for (int j = CW_KL; j < KT; ++j) {
            const int c = j * CW_THREADS + tid;
            const int4 gi = reinterpret_cast<const int4 *>(tb.gi)[c];
            const float4 ga = reinterpret_cast<const float4 *>(tb.gc)[2 * c];
            const float4 gb = reinterpret_cast<const float4 *>(tb.gc)[2 * c + 1];
            cx<float> a{0.f, 0.f};
            float v = zl[gi.x];
            a.x += ga.x * v;
            a.y += ga.y * v;
            v = zl[gi.y];
            a.x += ga.z * v;
            a.y += ga.w * v;
            v = zl[gi.z];
            a.x += gb.x * v;
            a.y += gb.y * v;
            v = zl[gi.w];
            a.x += gb.z * v;
            a.y += gb.w * v;
            Xr[j - CW_KL] = a;
        }
    }
    __syncthreads();
    CW_TP(2);

    // ---------------------------------------------------------------- Az
    // running statistics of s_new for section l = tid (L <= 1024)
    const int Lb = tb.Lblk;
    float Mr = -INFINITY, R1 = 0.f, R2 = 0.f, s_true = 0.f;
    int jt = -1;
    if (bf.true_idx && tid < Lb) jt = tb.qpos[tid * tb.M + bf.true_idx[lb + tid]];
    float v[CW_SN];
    uint32_t e[CW_SN];
    {
        const int q0 = tb.cls_ptr[0], q1 = tb.cls_ptr[1];
#pragma unroll
        for (int i = 0; i < CW_SN; ++i) {
            const int q = min(q0 + tid + i * CW_THREADS, q1 - 1);
            e[i] = tb.cls_ls[q];
            v[i] = s[q];  // (t = 0: unused)
        }
    }
    for (int m2 = 0; m2 < tb.Q; ++m2) {
        const int tl = cw_opaque(tid);
        if (m2 == 2) CW_TP(16);
        // the rows' image values (the same every class; reloaded, not held across the loop)
        const uint32_t rmk = CW_MASKIN ? tb.cmask[tb.Q * CW_THREADS + tl] : 0xffffu;
        if constexpr (!CW_MASKIN)
            for (int i = tl; i < CW_P * 8 / 16; i += CW_THREADS) reinterpret_cast<uint4 *>(smem)[i] = uint4{0, 0, 0, 0};
        cx<float> w[KT];
#pragma unroll
        for (int j = 0; j < KT; ++j) w[j] = cw_w(tb, (uint32_t)m2 * (kt[j] & CW_KMASK));
        if constexpr (!CW_MASKIN) __syncthreads();  // (masked: the previous class's closing barrier)
        if (m2 == 2) CW_TP(17);
        cw_rows<KT>(Xl, d, Xr, kt, w, tl);
        __syncthreads();
        if (m2 == 2) CW_TP(18);
        const int q0 = tb.cls_ptr[m2], q1 = tb.cls_ptr[m2 + 1];
        cw_fft_from<true, 0>(d, tl, rmk);
        if (m2 == 2) CW_TP(19);
        float bm[CW_SN], bi[CW_SN];
#pragma unroll
        for (int i = 0; i < CW_SN; ++i) {
            const int l = e[i] >> 16;
            bm[i] = have_beta ? stM[l] : 0.f;
            bi[i] = have_beta ? stI[l] : 0.f;
        }
        int sa = 0, sb = 0;  // the section's segment of the class, read under the s update
        if (tl < Lb) {
            const uint16_t *sg = tb.seg + (size_t)m2 * (Lb + 1);
            sa = sg[tl];
            sb = sg[tl + 1];
        }
        float snv[CW_SN];
#pragma unroll
        for (int i = 0; i < CW_SN; ++i) {
            const float b = have_beta ? __expf((v[i] - bm[i]) * inv_tp) * bi[i] : 0.f;
            snv[i] = b + tau * dr[e[i] & 0xffffu];
        }
        if (m2 + 1 < tb.Q) {  // the next class's slice in flight under the statistics
            const int n0 = tb.cls_ptr[m2 + 1], n1 = tb.cls_ptr[m2 + 2];
#pragma unroll
            for (int i = 0; i < CW_SN; ++i) {
                const int q = min(n0 + tl + i * CW_THREADS, n1 - 1);
                e[i] = tb.cls_ls[q];
                v[i] = s[q];
            }
        }
#pragma unroll
        for (int c = 0; c < CW_SN; ++c) {  // s to HBM straight from the registers (class order)
            const int q = q0 + tl + c * CW_THREADS;
            if (q < q1) s[q] = snv[c];
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
        // wavefronts with a segment longer than one round run at raised issue
        // priority: they set the time of the closing barrier
        const bool long_wave = __ballot(tl < Lb && sb - sa > 16) != 0;
        if (long_wave) __builtin_amdgcn_s_setprio(2);
        if (tl < Lb) {
            // partial of section tl over its segment of the class: running
            // maximum, sums without the (first) maximum (amp_fused.hip az_stage2)
            const int a = sa, b = sb;
            // two independent online chains (even / odd entries), merged at the
            // end: half the serial exp latency per round
            constexpr int RC = 16;
            float m = -INFINITY, S1 = 0.f, S2 = 0.f, mo = -INFINITY, S1o = 0.f, S2o = 0.f;
            auto step = [&](float &mm, float &T1, float &T2, float xi) {
                const bool up = xi > mm;
                const float dlt = up ? (mm - xi) : (xi - mm);
                const float ex = __expf(dlt * inv_tau);
                T1 = up ? (T1 + 1.f) * ex : T1 + ex;
                T2 = up ? (T2 + 1.f) * (ex * ex) : T2 + ex * ex;
                mm = up ? xi : mm;
            };
            for (int c = a; c < b; c += RC) {
                float x[RC];
#pragma unroll
                for (int i = 0; i < RC; ++i) x[i] = dr[fpad(c + i)];  // inside the LDS image; masked below
#pragma unroll
                for (int i = 0; i < RC; i += 2) {
                    if (c + i < b) step(m, S1, S2, x[i]);
                    if (c + i + 1 < b) step(mo, S1o, S2o, x[i + 1]);
                }
            }
            if (mo > -INFINITY) {  // the odd chain into the even one (same merge as below)
                if (mo > m) {
                    const float f = __expf((m - mo) * inv_tau);
                    S1 = (S1 + 1.f) * f + S1o;
                    S2 = (S2 + 1.f) * (f * f) + S2o;
                    m = mo;
                } else {
                    const float f = __expf((mo - m) * inv_tau);
                    S1 += (1.f + S1o) * f;
                    S2 += (1.f + S2o) * (f * f);
                }
            }
            if (m > -INFINITY) {  // merge into the section's running statistics
                if (m > Mr) {
                    const float f = __expf((Mr - m) * inv_tau);
                    R1 = (R1 + 1.f) * f + S1;
                    R2 = (R2 + 1.f) * (f * f) + S2;
                    Mr = m;
                } else {
                    const float f = __expf((m - Mr) * inv_tau);
                    R1 += (1.f + S1) * f;
                    R2 += (1.f + S2) * (f * f);
                }
            }
            if (jt >= q0 && jt < q1) s_true = dr[fpad(jt - q0)];
        }
        if (long_wave) __builtin_amdgcn_s_setprio(0);
        if (m2 == 2) CW_TP(22);
        __syncthreads();  // the next class overwrites the image
        if (m2 == 2) CW_TP(23);
    }
    CW_TP(3);

    // ---------------------------------------------------------------- merge
    double a = 0.0, er = 0.0;
    if (tid < Lb) {
        const float inv = 1.f / (1.f + R1);
        bf.stM[lb + tid] = Mr;
        bf.stI[lb + tid] = inv;
        // 1 - sum beta^2 = (2 R1 + R1^2 - R2) / (1 + R1)^2, no cancellation
        const double i2 = (double)inv * (double)inv, r1 = R1, r2 = R2;
        a = (2.0 * r1 + r1 * r1 - r2) * i2;
        if (jt >= 0) {
            if (s_true == Mr) {
                er = (r1 * r1 + r2) * i2;
            } else {
                const double bt = (double)(__expf((s_true - Mr) * inv_tau) * inv);
                er = (1.0 + r2) * i2 - 2.0 * bt + 1.0;
            }
        }
    }
    a = cw_block_sum(a, red);
    er = cw_block_sum(er, red);
    if (tid == 0) {
        double *nmse = sc.nmse + (size_t)cw * pr.t_max;
        const double denom = (double)tb.L;
        const double pnew = a / denom;
        *psi = pnew;
        nmse[t + 1] = er / denom;
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

template <int KT>
static int cw_launch(const CwTables &tb, const RegBufs<float> &bf, const AmpScalars &sc, const AmpParams &pr, int t,
                     hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        SG_HIP(hipFuncSetAttribute((const void *)cw_iter<KT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr = true;
    }
    const size_t lds = cw_lds_bytes(tb.img, CW_KL * CW_THREADS);
    if (lds > 160 * 1024) return fail(SG_ERR_UNSUPPORTED, "per-codeword engine: %zu bytes of LDS", lds);
    hipLaunchKernelGGL((cw_iter<KT>), dim3(bf.B), dim3(CW_THREADS), lds, s, tb, bf, sc, pr, t);
    return SG_OK;
}

int cw_launch_iter(const CwTables &tb, const RegBufs<float> &bf, const AmpScalars &sc, const AmpParams &pr, int t,
                   hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    if (tb.log2P != CW_LOG2P || tb.n > CW_CO * CW_THREADS || tb.Lblk > CW_THREADS || tb.Q > 64 ||
        tb.maxcls > CW_SN * CW_THREADS || tb.img < 2 * CW_P || fpad(tb.maxcls + 16) >= tb.img)
        return fail(SG_ERR_UNSUPPORTED, "per-codeword engine: sizes outside its compile-time bounds");
    ProfScope ps(SG_PH_AMP_CW, s);
    if (tb.KT == 12) SG_TRY(cw_launch<12>(tb, bf, sc, pr, t, s));
    else if (tb.KT == 14) SG_TRY(cw_launch<14>(tb, bf, sc, pr, t, s));
    else return fail(SG_ERR_UNSUPPORTED, "per-codeword engine: %d indices per thread", tb.KT);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

}  // namespace sg
