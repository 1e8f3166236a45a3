// Block engine, two-class form: AMP for spatially coupled sub-sampled DCT
// designs whose transforms have w = 2^16 (N2 = 2^15 complex points) -- the
// geometry of the reference's notebook (sparc_demo_sc_decode_wave.ipynb
// cell 1: omega = 6, Lambda = 32, L = 2048, M = 512; sparc.py:535-568
// sc_basic, :851-875 the per-block operators).  A 2^15-point image does not
// fit one workgroup's LDS, so every transform runs as two classes of 2^14
// points (the per-codeword engine's class decomposition, amp_cw.hip):
//   packed input v[m], m = 2 m1 + m2:  H[k] = sum_m2 w_N2^(m2 k) Y_m2[k mod P],
//   Y_m2 = the P-point FFT of class m2 (P = 2^14, in LDS);
//   inverse: x[2 m1 + m2] = P-point inverse FFT over k1 of
//            U_m2[k1] = sum_{k = k1 mod P} G[k] conj(w_N2^(m2 k)).
// Reference: sparc_public/sparc.py sparc_amp :883-999, sub_dct :648-701,
// msg_vector_mmse_estimator :402-465, msg_vector_map_estimator :467-512.
//
// One 1024-thread workgroup owns one column block c (Mc = 32768 entries, 32
// a thread) of one codeword and runs its omega transforms, each class in turn:
//   blk2_ab  for each transform and class: beta of the class's column entries
//            -> scatter -> three radix-16 stages -> the Mr needed outputs with
//            the last radix-4 stage and the class factor folded into their
//            coefficients, summed over the classes in registers -> rbuf[t]
//   blk2_az  for each transform and class: the class's rows of G (at most two
//            slots per row, k1 and k1 + P) -> inverse FFT -> the class's column
//            entries gathered into u (registers); then the column's sections:
//            s = beta + tau_c u, softmax, MAP, section statistics (amp_block.hip)
#include "amp.hpp"

namespace sg {

// Two geometries (template parameter LP = log2 P, 16 image values per thread):
//   LP = 14: the notebook's w = 2^16, Mc = 2^15, 1024 threads, one workgroup per CU;
//   LP = 13: C4's w = 2^15, Mc = 2^14 as two classes of 2^13 points, 512 threads
//            and a 66 KB image, so two workgroups share a CU and one's barriers
//            and LDS latency run beside the other's transform (the single-class
//            engine, amp_block.hip, holds 132 KB and runs alone on its CU).
template <int LP>
struct B2G {
    static constexpr int P = 1 << LP;
    static constexpr int THREADS = P / 16;
    // The class image in the padded layout of fft.hpp ppos (element i at i + i/32:
    // every FFT stage access is a per-thread base plus a constant, no swizzle
    // arithmetic)
    static constexpr int IMG = ppos(P);  // complex slots of the padded image
    static constexpr int RF = P / 4096;  // radix of the last stage, folded into the output coefficients
    static_assert(RF == 2 || RF == 4, "P = 2^13 or 2^14");
};
constexpr int B2_J = 32;  // column entries per thread (Mc = 2 P = 32 threads), all held in registers
// a padding slot -- never written by the rows or the FFT stages, so zero after
// b2_clear -- is the trash slot of the position tables
constexpr int B2_TRASH = 2 * 32;  // real index of the padding slot at complex position 32
static_assert(ppos(B2_TRASH / 2) == B2_TRASH / 2 + 1, "the trash slot is a padding slot (capi_amp.cpp build_block2)");

namespace {

template <typename T>
__device__ __forceinline__ T b2_wave_max(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
template <typename T>
__device__ __forceinline__ T b2_wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ int b2_wave_min(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ int b2_opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

template <int LP>
__device__ __forceinline__ void b2_clear(unsigned char *smem, int tid) {
    constexpr int T = B2G<LP>::THREADS, N16 = B2G<LP>::IMG * (int)sizeof(cx<float>) / 16;  // (8 per thread and a quarter)
#pragma unroll
    for (int i = 0; i < (N16 + T - 1) / T; ++i)
        if (tid + i * T < N16) reinterpret_cast<uint4 *>(smem)[tid + i * T] = uint4{0, 0, 0, 0};
}

// Column entry i (< 32) of thread tid: wavefront w owns sections
// w spw .. w spw + spw - 1 of the column block (spw = 2048 / M), lane l holds
// entries l eps .. l eps + eps - 1 of each (eps = M / 64).  Host mirror in
// capi_amp.cpp build_block2.
template <int EPS>
__device__ __forceinline__ int b2_j(int tid, int i) {
    constexpr int M = 64 * EPS, SPW = 2048 / M;
    const int sq = i / EPS, e = i - sq * EPS;
    return ((tid >> 6) * SPW + sq) * M + (tid & 63) * EPS + e;
}

// real LDS index in the image of class m2 (2 ppos(m1) + component; B2_TRASH
// for the entries of the other class) of the thread's column entries of
// transform t, packed in pairs
template <int LP>
__device__ __forceinline__ void b2_pos_load(const BlkTables &tb, int t, int m2, int tid, uint32_t *pv) {
    constexpr int T = B2G<LP>::THREADS;
    const uint32_t *p2 = tb.pos2 + ((size_t)t * 2 + m2) * (B2_J / 2) * T;
#pragma unroll
    for (int i = 0; i < B2_J / 2; ++i) pv[i] = p2[i * T + tid];
}
__device__ __forceinline__ uint32_t b2_pos(const uint32_t *pv, int i) { return (pv[i >> 1] >> (16 * (i & 1))) & 0xffffu; }
// One-table form (A/B: -DB2_ONETABLE=1): one 16-bit entry per column entry and
// transform for both classes, m1 << 2 | component << 1 | class, the padded index rebuilt per class pass --
// half the position-table bytes, four vector instructions more per entry and pass
// Wave issue priority of the transforms and of the rest (A/B; flat by default: the split C2 engine's
// scheme -- transforms 0, the rest 1 -- measured 1000 -> 945 codewords/s here, profiles/r05_prio_ab.txt)
#ifndef B2_PRIO_FFT
#define B2_PRIO_FFT 0
#endif
#ifndef B2_PRIO_REST
#define B2_PRIO_REST 0
#endif
#define B2_SETPRIO(p)                                                       \
    do {                                                                    \
        if (B2_PRIO_FFT != B2_PRIO_REST) __builtin_amdgcn_s_setprio(p);     \
    } while (0)
#ifndef B2_ONETABLE
#define B2_ONETABLE 0
#endif
template <int LP>
__device__ __forceinline__ void b2_pos_load1(const BlkTables &tb, int t, int tid, uint32_t *pv) {
    constexpr int T = B2G<LP>::THREADS;
    const uint32_t *p1 = tb.pos1 + (size_t)t * (B2_J / 2) * T;
#pragma unroll
    for (int i = 0; i < B2_J / 2; ++i) pv[i] = p1[i * T + tid];
}
__device__ __forceinline__ uint32_t b2_pos1(const uint32_t *pv, int i, int m2) {
    const uint32_t e = (pv[i >> 1] >> (16 * (i & 1))) & 0xffffu;
    return (e & 1u) == (uint32_t)m2 ? 2u * (uint32_t)ppos((int)(e >> 2)) + ((e >> 1) & 1u) : (uint32_t)B2_TRASH;
}

// the first three stages (radix 16) of the P-point FFT over the padded image,
// twiddles from the hardware sine / cosine (no table entries in flight: blk2_ab
// holds beta_c in registers; with the table prefetch it spills)
template <int LP>
__device__ __forceinline__ void b2_fwd_stages(cx<float> *d, int tid) {
    lds_fft1_sincos<false, 16, LP, 0, 3, true>(d, tid);
}

}  // namespace

size_t blk2_lds_bytes(int log2p) {
    return log2p == 13 ? (size_t)B2G<13>::IMG * sizeof(cx<float>) : (size_t)B2G<14>::IMG * sizeof(cx<float>);
}

// ------------------------------------------------------------------ Ab
// The column's forward transforms from beta_c in registers (bv[i] = beta_c at
// b2_j(tid, i)): for each transform and class, scatter -> three radix-16
// stages -> the needed outputs (last radix-RF stage and class factor folded into
// the coefficients), summed over the classes in registers -> rbuf[t]
template <int LP>
__device__ __forceinline__ void b2_ab_column(const BlkTables &tb, const AmpBufs<float> &bf, int c, int cw, int tid,
                                             const float *bv, unsigned char *smem) {
    cx<float> *d = reinterpret_cast<cx<float> *>(smem);
    float *dr = reinterpret_cast<float *>(smem);
    for (int q = tb.col_ptr[c]; q < tb.col_ptr[c + 1]; ++q) {
        const int t = tb.col_t[q];
        float acc = 0.f;  // output tid (Mr <= THREADS), summed over the two classes
        for (int m2 = 0; m2 < 2; ++m2) {
            const int tl = b2_opaque(tid);
            // the positions, in flight while the image clears
            uint32_t pv[B2_J / 2];
            if (B2_ONETABLE) b2_pos_load1<LP>(tb, t, tl, pv);
            else b2_pos_load<LP>(tb, t, m2, tl, pv);
            b2_clear<LP>(smem, tl);
            __syncthreads();
#pragma unroll
            for (int i = 0; i < B2_J; ++i)  // (the other class's entries: trash slot)
                dr[B2_ONETABLE ? b2_pos1(pv, i, m2) : b2_pos(pv, i)] = bv[i];
            // the output's bins and coefficients, requested before the transform (their L2 round trip
            // hides behind it; requested after it, one workgroup per CU waited for it every class)
            constexpr int RF = B2G<LP>::RF;
            const bool own = tl < tb.Mr;
            const int io = own ? tl : 0;
            const uint32_t ab = tb.oab[(size_t)t * tb.Mr + io];
            const cx<float> *oc = tb.oc + (((size_t)t * 2 + m2) * tb.Mr + io) * 8;
            cx<float> al[RF], be[RF];
#pragma unroll
            for (int r = 0; r < RF; ++r) {
                al[r] = oc[r];
                be[r] = oc[4 + r];
            }
            __syncthreads();
            B2_SETPRIO(B2_PRIO_FFT);
            b2_fwd_stages<LP>(d, tl);
            B2_SETPRIO(B2_PRIO_REST);
            // X_i += Re(sum_r al_r Y[a mod 4096 + 4096 r] + be_r conj Y[b mod ...]), r < RF:
            // the last stage and w_N2^(m2 k) are in the coefficients
            if (own) {
                const int ja = ab & 0xffffu, jb = ab >> 16;
#pragma unroll
                for (int r = 0; r < RF; ++r) {  // ppos(j + 4096 r) = ppos(j) + 4224 r for j < 4096
                    const cx<float> ya = d[ppos(ja) + 4224 * r], yb = d[ppos(jb) + 4224 * r];
                    acc += (al[r].x * ya.x - al[r].y * ya.y) + (be[r].x * yb.x + be[r].y * yb.y);
                }
            }
            __syncthreads();
        }
        if (tid < tb.Mr) bf.rbuf[((size_t)cw * tb.nT + t) * tb.Mr + tid] = acc;
    }
}

// Standalone Ab (beta_c read once for all the column's transforms and
// classes); iterations after the first run it inside the previous blk2_az
template <int LP, int EPS>
__global__ __launch_bounds__(B2G<LP>::THREADS, 4) void blk2_ab(BlkTables tb, AmpBufs<float> bf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int c = blockIdx.x, cw = blockIdx.y, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    B2_SETPRIO(B2_PRIO_REST);
    const float *beta = bf.beta + (size_t)cw * tb.LM + (size_t)c * tb.Mc;
    float bv[B2_J];
#pragma unroll
    for (int i = 0; i < B2_J; ++i) bv[i] = beta[b2_j<EPS>(tid, i)];
    b2_ab_column<LP>(tb, bf, c, cw, tid, bv, smem);
}

// ------------------------------------------------------------------ Az + eta
// (__launch_bounds__ with 4 waves per SIMD: 128 VGPRs, so two 512-thread
// workgroups share a CU at LP = 13)
template <int LP, int EPS>
__global__ __launch_bounds__(B2G<LP>::THREADS, 4) void blk2_az(BlkTables tb, AmpBufs<float> bf, const cx<float> *gbuf,
                                                      int do_ab) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cx<float> *d = reinterpret_cast<cx<float> *>(smem);
    float *dr = reinterpret_cast<float *>(smem);
    const int c = blockIdx.x, cw = blockIdx.y, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    B2_SETPRIO(B2_PRIO_REST);
    float u[B2_J];
#pragma unroll
    for (int i = 0; i < B2_J; ++i) u[i] = 0.f;
    const cx<float> *gcw = gbuf + (size_t)cw * tb.ngs;
    constexpr int T = B2G<LP>::THREADS, P = B2G<LP>::P;
    const float inv_n2 = 1.0f / (float)(2 * P);
    for (int q = tb.col_ptr[c]; q < tb.col_ptr[c + 1]; ++q) {
        const int t = tb.col_t[q];
        const int g0 = tb.gptr[t], ng = tb.gptr[t + 1] - g0;
        for (int m2 = 0; m2 < 2; ++m2) {
            const int tl = b2_opaque(tid);
            // rows of class m2: U[k1] = sum over k = k1 mod P of G[k] conj(w_N2^(m2 k));
            // at most two slots (k1, k1 + P) share a row, and two float additions
            // onto a zero commute, so the atomic sum is deterministic.  The thread's
            // first two slots are requested before the clear (in flight during it).
            int kp[2];
            cx<float> vp[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int g = tl + e * T < ng ? tl + e * T : 0;
                kp[e] = tb.gk[g0 + g];
                vp[e] = gcw[g0 + g];
            }
            b2_clear<LP>(smem, tl);
            __syncthreads();
            auto row = [&](int k, cx<float> v) {
                if (m2) {
                    const float x = (float)k * inv_n2;  // conj(w_N2^k) = exp(+2 pi i k / N2)
                    const float cs = __builtin_amdgcn_cosf(x), sn = __builtin_amdgcn_sinf(x);
                    v = {v.x * cs - v.y * sn, v.x * sn + v.y * cs};
                }
                cx<float> *dst = &d[ppos(k & (P - 1))];
                atomicAdd(&dst->x, v.x);
                atomicAdd(&dst->y, v.y);
            };
#pragma unroll
            for (int e = 0; e < 2; ++e)
                if (tl + e * T < ng) row(kp[e], vp[e]);
            for (int g = tl + 2 * T; g < ng; g += T) row(tb.gk[g0 + g], gcw[g0 + g]);
            __syncthreads();
            // (stage twiddles from the hardware sine / cosine: no table entries in flight, u[] stays in registers)
            B2_SETPRIO(B2_PRIO_FFT);
            lds_fft1_sincos<true, 16, LP, 0, 4, true>(d, tl);
            B2_SETPRIO(B2_PRIO_REST);
            uint32_t pv[B2_J / 2];
            if (B2_ONETABLE) b2_pos_load1<LP>(tb, t, tl, pv);
            else b2_pos_load<LP>(tb, t, m2, tl, pv);
#pragma unroll
            for (int i = 0; i < B2_J; ++i)  // (the other class's entries read the zero trash slot)
                u[i] += dr[B2_ONETABLE ? b2_pos1(pv, i, m2) : b2_pos(pv, i)];
            __syncthreads();
        }
    }
    // ---- sections of the column block (sparc.py:972, :429-432, :485-487), one
    // at a time: s = beta + tau u, x = s / tau, beta = exp(x - max) / sum, MAP =
    // first index of max s.  A wavefront owns whole sections (b2_j).
    const int lane = tid & 63, wv = tid >> 6;
    constexpr int eps = EPS, spw = 2048 / (64 * EPS);
    const int nsec = tb.Mc / tb.M;
    // x = s log2(e) / tau (sparc.py:430 in base 2: exp(s / tau - max) = exp2(x - max x), one v_exp_f32;
    // __expf is a multiply by log2 e and v_exp_f32), the reciprocal once (IEEE division is ~10 VALU)
    const float tau = (float)bf.tau[(size_t)cw * tb.Lc + c], itau = (float)(1.4426950408889634074 / (double)tau);
    float *beta = bf.beta + (size_t)cw * tb.LM + (size_t)c * tb.Mc;
    const int l0 = c * nsec;  // first section of the column block
    float bv[B2_J];  // the new beta_c, kept for the next iteration's Ab (do_ab)
#pragma unroll
    for (int sq = 0; sq < spw; ++sq) {
        const int ls = wv * spw + sq;  // section within the column block
        const int i0 = sq * eps;
        float s[eps], x[eps];
#pragma unroll
        for (int e = 0; e < eps; ++e) {
            s[e] = beta[ls * tb.M + lane * eps + e] + tau * u[i0 + e];  // sparc.py:972
            x[e] = s[e] * itau;                                         // sparc.py:430, scaled by log2 e
        }
        float xm = -INFINITY, sm = -INFINITY;
        int arg = 0x7fffffff;
#pragma unroll
        for (int e = 0; e < eps; ++e) {
            xm = fmax(xm, x[e]);
            if (s[e] > sm) {
                sm = s[e];
                arg = lane * eps + e;
            }
        }
        xm = b2_wave_max(xm);
        const float gm = b2_wave_max(sm);
        arg = b2_wave_min(sm == gm ? arg : 0x7fffffff);
        float dn = 0.f;
#pragma unroll
        for (int e = 0; e < eps; ++e) {
            x[e] = __builtin_amdgcn_exp2f(x[e] - xm);
            dn += x[e];
        }
        dn = b2_wave_sum(dn);
        const float idn = 1.0f / dn;
        const int truth = bf.true_idx ? bf.true_idx[(size_t)cw * tb.L + l0 + ls] : -1;
        float ss = 0.f, se = 0.f;
#pragma unroll
        for (int e = 0; e < eps; ++e) {
            const float b = x[e] * idn;
            beta[ls * tb.M + lane * eps + e] = b;
            bv[i0 + e] = b;
            const float dl = b - ((lane * eps + e) == truth ? 1.f : 0.f);
            ss += b * b;
            se += dl * dl;
        }
        ss = b2_wave_sum(ss);
        se = b2_wave_sum(se);
        if (lane == 0) {
            const size_t o = (size_t)cw * tb.L + l0 + ls;
            bf.sec_sumsq[o] = (double)ss;
            bf.sec_err[o] = (double)se;
            bf.sec_argmax[o] = arg;
        }
    }
    // the next iteration's forward transforms of the column from the new beta_c
    // in registers (not read back; a codeword that stops in this iteration
    // computes one Ab nobody reads)
    if (do_ab) {
        __syncthreads();  // the image is free
        b2_ab_column<LP>(tb, bf, c, cw, tid, bv, smem);
    }
}

template <int LP, int EPS>
static int blk2_set_attrs(size_t lds) {
    static size_t done = 0;
    if (done >= lds) return SG_OK;
    SG_HIP(hipFuncSetAttribute((const void *)blk2_ab<LP, EPS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    SG_HIP(hipFuncSetAttribute((const void *)blk2_az<LP, EPS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    done = lds;
    return SG_OK;
}

// section size M = 64 EPS, 64 <= M <= 2048
#define B2_EPS_DISPATCH(LP, M, F, ...)                                                          \
    switch (M) {                                                                                \
    case 64: F<LP, 1>(__VA_ARGS__); break;                                                      \
    case 128: F<LP, 2>(__VA_ARGS__); break;                                                     \
    case 256: F<LP, 4>(__VA_ARGS__); break;                                                     \
    case 512: F<LP, 8>(__VA_ARGS__); break;                                                     \
    case 1024: F<LP, 16>(__VA_ARGS__); break;                                                   \
    case 2048: F<LP, 32>(__VA_ARGS__); break;                                                   \
    default: return fail(SG_ERR_UNSUPPORTED, "block engine (two classes): section size M=%d", M); \
    }

template <int LP, int EPS>
static void b2_launch_ab(const BlkTables &tb, const AmpBufs<float> &bf, size_t lds, hipStream_t s, int *rc) {
    *rc = blk2_set_attrs<LP, EPS>(lds);
    if (*rc == SG_OK)
        hipLaunchKernelGGL((blk2_ab<LP, EPS>), dim3(tb.Lc, bf.B), dim3(B2G<LP>::THREADS), lds, s, tb, bf);
}
template <int LP, int EPS>
static void b2_launch_az(const BlkTables &tb, const AmpBufs<float> &bf, const cx<float> *gbuf, int do_ab, size_t lds,
                         hipStream_t s, int *rc) {
    *rc = blk2_set_attrs<LP, EPS>(lds);
    if (*rc == SG_OK)
        hipLaunchKernelGGL((blk2_az<LP, EPS>), dim3(tb.Lc, bf.B), dim3(B2G<LP>::THREADS), lds, s, tb, bf, gbuf, do_ab);
}

static int b2_check(const BlkTables &tb) {
    if ((tb.log2p != 13 && tb.log2p != 14) || tb.Mc != 2 << tb.log2p || tb.Mr > (1 << tb.log2p) / 16)
        return fail(SG_ERR_UNSUPPORTED, "block engine (two classes): P=2^%d, Mc=%d, Mr=%d", tb.log2p, tb.Mc, tb.Mr);
    return SG_OK;
}

int blk2_launch_ab(const BlkTables &tb, const AmpBufs<float> &bf, hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    SG_TRY(b2_check(tb));
    const size_t lds = blk2_lds_bytes(tb.log2p);
    int rc = SG_OK;
    ProfScope ps(SG_PH_AB_A, s);
    if (tb.log2p == 13) {
        B2_EPS_DISPATCH(13, tb.M, b2_launch_ab, tb, bf, lds, s, &rc);
    } else {
        B2_EPS_DISPATCH(14, tb.M, b2_launch_ab, tb, bf, lds, s, &rc);
    }
    SG_TRY(rc);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

int blk2_launch_az(const BlkTables &tb, const AmpBufs<float> &bf, cx<float> *gbuf, bool then_ab, hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    SG_TRY(b2_check(tb));
    SG_TRY(blk_launch_g(tb, bf, gbuf, s));
    const size_t lds = blk2_lds_bytes(tb.log2p);
    int rc = SG_OK;
    ProfScope ps(SG_PH_AZ_B, s);
    if (tb.log2p == 13) {
        B2_EPS_DISPATCH(13, tb.M, b2_launch_az, tb, bf, (const cx<float> *)gbuf, then_ab ? 1 : 0, lds, s, &rc);
    } else {
        B2_EPS_DISPATCH(14, tb.M, b2_launch_az, tb, bf, (const cx<float> *)gbuf, then_ab ? 1 : 0, lds, s, &rc);
    }
    SG_TRY(rc);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

}  // namespace sg
