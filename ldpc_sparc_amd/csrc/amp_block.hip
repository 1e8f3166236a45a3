// Block engine: AMP for sub-sampled DCT designs whose transforms fit one
// workgroup's LDS (single precision, w = 2^15, N2 = 2^14 complex points) and
// whose base matrix has several transforms per column block -- the spatially
// coupled designs of sparc_demo_sc_decode_wave (sparc.py:535-568 sc_basic,
// :851-875 the per-block operators).
//
// Reference: sparc_public/sparc.py sparc_amp :883-999, sub_dct :648-701,
// msg_vector_mmse_estimator :402-465, msg_vector_map_estimator :467-512.
//
// One workgroup owns one column block c of one codeword and runs the omega
// transforms of that column back to back, each entirely in LDS (Makhoul-packed
// N2-point FFT, natural order in the padded layout of fft.hpp ppos):
//   Ab       beta_c (registers) -> for each transform (r, c): scatter by
//            order1, forward FFT, the Mr needed outputs Re(c1 H[a] + c2 conj
//            H[b]) -> rbuf[t] (summed per row block in a fixed order by the
//            control kernel); run at the end of the previous iteration's blk_az
//   blk_az   for each transform (r, c): G from z_r / phi_r (<= 4 terms per
//            slot), inverse FFT, gather by order1 into u (registers); then the
//            column's sections: s = beta + tau_c u, softmax, MAP index and the
//            section statistics of eta_kernel (amp_dct.hip), beta written back;
//            then (all but the last iteration) the next iteration's Ab
//            work for the column from the new beta_c in registers, so HBM
//            reads beta once per iteration.
// Versus the general four-step path (amp_dct.hip) no transform intermediate
// reaches HBM and the random-order gather of u happens in LDS.
#include "amp.hpp"

namespace sg {

constexpr int BK_THREADS = 1024;
constexpr int BK_LOG2N = 14;
constexpr int BK_J = 16;  // column entries per thread (Mc = 16384)

template <typename T>
__device__ __forceinline__ T bk_wave_max(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
template <typename T>
__device__ __forceinline__ T bk_wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ int bk_wave_min(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}

// LDS: the FFT image in the padded layout (element i at ppos(i) = i + i/32:
// every FFT stage access a per-thread base plus a constant, no swizzle
// arithmetic)
constexpr int BK_IMG = ppos(1 << BK_LOG2N);  // complex slots
size_t blk_lds_bytes(int Mc) { return (size_t)BK_IMG * sizeof(cx<float>); }

__device__ __forceinline__ void bk_clear(unsigned char *smem, int tid) {
    constexpr int N16 = BK_IMG * (int)sizeof(cx<float>) / 16;  // (8448: 8 per thread and a quarter)
#pragma unroll
    for (int i = 0; i < (N16 + BK_THREADS - 1) / BK_THREADS; ++i)
        if (tid + i * BK_THREADS < N16) reinterpret_cast<uint4 *>(smem)[tid + i * BK_THREADS] = uint4{0, 0, 0, 0};
}

// The thread index as a value the compiler cannot see through: the FFT's LDS
// addresses are then recomputed inside the loop over a column's transforms
// instead of being hoisted out of it and held (and spilled) across the loop.
__device__ __forceinline__ int bk_opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// Column entry i (< 16) of thread tid: wavefront w owns sections
// w spw .. w spw + spw - 1 of the column block (spw = 1024 / M), lane l holds
// entries l eps .. l eps + eps - 1 of each (eps = M / 64).  Needs Mc = 16384
// and 64 <= M <= 1024 (host mirror in capi_amp.cpp build_block).
template <int EPS>
__device__ __forceinline__ int bk_j(int tid, int i) {
    constexpr int M = 64 * EPS, SPW = 1024 / M;
    const int sq = i / EPS, e = i - sq * EPS;
    return ((tid >> 6) * SPW + sq) * M + (tid & 63) * EPS + e;
}

// LDS positions of the thread's column entries bk_j(tid, i) of transform t,
// packed in pairs (i = 2 i2, 2 i2 + 1) in thread order
__device__ __forceinline__ void bk_pos_load(const BlkTables &tb, int t, int tid, uint32_t *pv) {
    const uint32_t *p2 = tb.pos2 + (size_t)t * (BK_J / 2) * BK_THREADS;
#pragma unroll
    for (int i = 0; i < BK_J / 2; ++i) pv[i] = p2[i * BK_THREADS + tid];
}
__device__ __forceinline__ uint32_t bk_pos(const uint32_t *pv, int i) { return (pv[i >> 1] >> (16 * (i & 1))) & 0xffffu; }

// The first three stages of the 2^14-point FFT of fft.hpp (radix 16, 16, 16,
// then 4): the forward transform stops before the radix-4 stage, which Ab
// folds into the needed outputs.  Stages 0-1 and stage 2 separately, so that
// the outputs' table entries can be requested in between (in flight during
// the last stage; across all three stages they would spill).
__device__ __forceinline__ void bk_fwd_stages01(cx<float> *d, const cx<float> *__restrict__ stw, int tid,
                                                cx<float> *w2) {
    if constexpr (SG_BLK_SINCOS & 1) {
        lds_fft1_sincos<false, 16, BK_LOG2N, 0, 2, true>(d, tid);
    } else {
        cx<float> w0[1], w1[6];
        fft1_tw_load_ct<float, 16, BK_LOG2N, 1>(stw, tid, w1);
        stockham1_stage_ct<float, false, 16, 16, BK_LOG2N, 0, true>(d, w0, tid);
        fft1_tw_load_ct<float, 16, BK_LOG2N, 2>(stw, tid, w2);
        stockham1_stage_ct<float, false, 16, 16, BK_LOG2N, 4, true>(d, w1, tid);
    }
}
__device__ __forceinline__ void bk_fwd_stage2(cx<float> *d, int tid, const cx<float> *w2) {
    if constexpr (SG_BLK_SINCOS & 1) lds_fft1_sincos<false, 16, BK_LOG2N, 2, 3, true>(d, tid);
    else stockham1_stage_ct<float, false, 16, 16, BK_LOG2N, 8, true>(d, w2, tid);
}

// ------------------------------------------------------------------ Ab
// The omega forward transforms of column block c from beta_c in registers
// (bv[i] = beta_c[bk_j(tid, i)])
__device__ __forceinline__ void bk_ab_column(const BlkTables &tb, const AmpBufs<float> &bf, int c, int cw, int tid,
                                             const float *bv, unsigned char *smem) {
    cx<float> *d = reinterpret_cast<cx<float> *>(smem);
    float *dr = reinterpret_cast<float *>(smem);
    for (int q = tb.col_ptr[c]; q < tb.col_ptr[c + 1]; ++q) {
        const int t = tb.col_t[q];
        const int tl = bk_opaque(tid);
        // the positions of this transform, in flight while the image clears
        uint32_t pv[BK_J / 2];
        bk_pos_load(tb, t, tl, pv);
        bk_clear(smem, tl);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < BK_J; ++i)
            dr[bk_pos(pv, i)] = bv[i];
        __syncthreads();
        cx<float> w2[6];
        bk_fwd_stages01(d, tb.stw, tl, w2);
        // the last (radix-4, Ns = 4096) stage only for the needed bins, folded
        // into the outputs: H[a] = sum_r Y[a mod 4096 + 4096 r] w_N2^(r a), so
        // X_i = Re(c1 H[a] + c2 conj H[b]) = Re(sum_r al_r Y_a,r + be_r conj Y_b,r)
        float *r = bf.rbuf + ((size_t)cw * tb.nT + t) * tb.Mr;
        const uint32_t *oab = tb.oab + (size_t)t * tb.Mr;
        const cx<float> *oc = tb.oc + (size_t)t * tb.Mr * 8;
        {  // the thread's first output: its entries requested before the last stage
            const bool own = tl < tb.Mr;
            const int io = own ? tl : 0;
            const uint32_t ab = oab[io];
            cx<float> al[4], be[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                al[q] = oc[8 * io + q];
                be[q] = oc[8 * io + 4 + q];
            }
            bk_fwd_stage2(d, tl, w2);
            if (own) {
                const int ja = ab & 0xffffu, jb = ab >> 16;
                float acc = 0.f;
#pragma unroll
                for (int q = 0; q < 4; ++q) {  // ppos(j + 4096 q) = ppos(j) + 4224 q for j < 4096
                    const cx<float> ya = d[ppos(ja) + 4224 * q], yb = d[ppos(jb) + 4224 * q];
                    acc += (al[q].x * ya.x - al[q].y * ya.y) + (be[q].x * yb.x + be[q].y * yb.y);
                }
                r[tl] = acc;
            }
        }
        for (int i = tl + BK_THREADS; i < tb.Mr; i += BK_THREADS) {  // (Mr > 1024 only)
            const uint32_t ab = oab[i];
            const int ja = ab & 0xffffu, jb = ab >> 16;
            float acc = 0.f;
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // ppos(j + 4096 q) = ppos(j) + 4224 q for j < 4096
                const cx<float> ya = d[ppos(ja) + 4224 * q], yb = d[ppos(jb) + 4224 * q];
                const cx<float> al = oc[8 * i + q], be = oc[8 * i + 4 + q];
                acc += (al.x * ya.x - al.y * ya.y) + (be.x * yb.x + be.y * yb.y);
            }
            r[i] = acc;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ G slots
// Packed spectrum of Az's input for every transform (sparc.py:694-699 via the
// Makhoul packing): G[k] = sum of <= 4 terms c * z_i / phi_r, one thread per
// slot, written to gbuf so that blk_az loads each transform's slots in one
// coalesced round trip.
// (two dependent rounds of loads: the slot's table entries, then phi and the four z values,
// unconditionally at clamped indices -- with a branch per term each term's z load waited on its own)
__device__ __forceinline__ cx<float> bk_gslot(const BlkTables &tb, const AmpBufs<float> &bf, int cw, int g) {
    const int row = tb.grow[g];
    int gi[4];
    cx<float> gc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        gi[k] = tb.gi[4 * g + k];
        gc[k] = tb.gc[4 * g + k];
    }
    const float *z = bf.z + (size_t)cw * tb.n + (size_t)row * tb.Mr;
    const float ph = (float)bf.phi[(size_t)cw * tb.Lr + row];
    float zv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) zv[k] = z[max(gi[k], 0)];
    const float iphi = 1.0f / ph;
    cx<float> acc{0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (gi[k] >= 0) {
            const float v = zv[k] * iphi;  // Az(z / phi), sparc.py:972 (one division per slot)
            acc.x += gc[k].x * v;
            acc.y += gc[k].y * v;
        }
    }
    return acc;
}
// One thread per G slot and BK_GCW codewords: the slot's table entries (row,
// up to four output indices and coefficients: 52 B) are read once for the
// group instead of once per codeword (with one codeword per thread they were
// re-read from beyond L2 for every codeword, ~6 MB per codeword at the
// notebook geometry).
constexpr int BK_GCW = 16;
__global__ __launch_bounds__(256) void blk_g(BlkTables tb, AmpBufs<float> bf, cx<float> *gbuf) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= tb.ngs) return;
    const int row = tb.grow[g];
    int gi[4];
    cx<float> gc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        gi[k] = tb.gi[4 * g + k];
        gc[k] = tb.gc[4 * g + k];
    }
    const int c0 = blockIdx.y * BK_GCW, c1 = min(c0 + BK_GCW, bf.B);
    for (int cw = c0; cw < c1; ++cw) {
        if (!bf.active[cw]) continue;
        const float *z = bf.z + (size_t)cw * tb.n + (size_t)row * tb.Mr;
        const float iphi = 1.0f / (float)bf.phi[(size_t)cw * tb.Lr + row];
        cx<float> acc{0.f, 0.f};  // same terms, same order as bk_gslot
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (gi[k] >= 0) {
                const float v = z[gi[k]] * iphi;  // Az(z / phi), sparc.py:972
                acc.x += gc[k].x * v;
                acc.y += gc[k].y * v;
            }
        }
        gbuf[(size_t)cw * tb.ngs + g] = acc;
    }
}

// ------------------------------------------------------------------ Az + eta
// with do_ab: then the next iteration's forward transforms of the column from
// the new beta_c still in registers (bk_ab_column; beta_c is not read back)
template <int EPS>
__global__ __launch_bounds__(BK_THREADS) void blk_az(BlkTables tb, AmpBufs<float> bf, int do_ab) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cx<float> *d = reinterpret_cast<cx<float> *>(smem);
    float *dr = reinterpret_cast<float *>(smem);
    const int c = blockIdx.x, cw = blockIdx.y, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    float u[BK_J];
#pragma unroll
    for (int i = 0; i < BK_J; ++i) u[i] = 0.f;
    // Az(z / phi) restricted to column block c, summed over its transforms in
    // the order of gather_u (amp_dct.hip)
    for (int q = tb.col_ptr[c]; q < tb.col_ptr[c + 1]; ++q) {
        const int t = tb.col_t[q];
        const int tl = bk_opaque(tid);
        // G slots (from z / phi, <= 4 terms), in flight while the image clears
        const int g0 = tb.gptr[t], ng = tb.gptr[t + 1] - g0;
        cx<float> gv[2];
        uint32_t gl[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int g = tl + k * BK_THREADS;
            if (g < ng) {
                gv[k] = bk_gslot(tb, bf, cw, g0 + g);
                gl[k] = tb.gloc[g0 + g];
            }
        }
        bk_clear(smem, tl);
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (tl + k * BK_THREADS < ng) d[gl[k]] = gv[k];
        for (int g = tl + 2 * BK_THREADS; g < ng; g += BK_THREADS) d[tb.gloc[g0 + g]] = bk_gslot(tb, bf, cw, g0 + g);
        __syncthreads();
        // the positions of this transform's column entries are requested before the last stage (in flight
        // during it; the padded image leaves no LDS to stage them in, and held across the whole FFT they
        // would spill)
        uint32_t pv[BK_J / 2];
        if (!(tb.skip & 2)) lds_fft1_sincos<true, 16, BK_LOG2N, 0, 3, true>(d, tl);
        bk_pos_load(tb, t, tl, pv);
        if (!(tb.skip & 2)) lds_fft1_sincos<true, 16, BK_LOG2N, 3, 4, true>(d, tl);
#pragma unroll
        for (int i = 0; i < BK_J; ++i) u[i] += dr[bk_pos(pv, i)];
        __syncthreads();
    }
    if (tb.skip & 1) return;  // timing ablation only
    // ---- sections of the column block (sparc.py:972, :429-432, :485-487):
    // s = beta + tau u, x = s / tau, beta = exp(x - max) / sum, MAP = first
    // index of max s.  A wavefront owns whole sections (bk_j): each lane
    // reduces its EPS entries, then one butterfly over the lanes -- no LDS, no
    // workgroup barrier.
    const int lane = tid & 63, wv = tid >> 6;
    constexpr int eps = EPS, spw = 1024 / (64 * EPS);
    const int nsec = tb.Mc / tb.M;
    // x = s log2(e) / tau (sparc.py:430 in base 2: exp(s / tau - max) = exp2(x - max x), one v_exp_f32;
    // __expf is a multiply by log2 e and v_exp_f32), the reciprocal once (IEEE division is ~10 VALU)
    const float tau = (float)bf.tau[(size_t)cw * tb.Lc + c], itau = (float)(1.4426950408889634074 / (double)tau);
    float *beta = bf.beta + (size_t)cw * tb.LM + (size_t)c * tb.Mc;
    float s[BK_J], x[BK_J], bv[BK_J];
#pragma unroll
    for (int i = 0; i < BK_J; ++i) {
        const int j = bk_j<EPS>(tid, i);
        s[i] = beta[j] + tau * u[i];  // sparc.py:972
        x[i] = s[i] * itau;           // sparc.py:430, scaled by log2 e
    }
    const int l0 = c * nsec;  // first section of the column block
#pragma unroll
    for (int sq = 0; sq < spw; ++sq) {
        const int ls = wv * spw + sq;  // section within the column block
        const int i0 = sq * eps;
        // maxima and the MAP index (entries of a lane are in increasing j)
        float xm = -INFINITY, sm = -INFINITY;
        int arg = 0x7fffffff;
#pragma unroll
        for (int e = 0; e < eps; ++e) {
            xm = fmax(xm, x[i0 + e]);
            if (s[i0 + e] > sm) {
                sm = s[i0 + e];
                arg = lane * eps + e;
            }
        }
        xm = bk_wave_max(xm);
        const float gm = bk_wave_max(sm);
        arg = bk_wave_min(sm == gm ? arg : 0x7fffffff);
        float dn = 0.f;
#pragma unroll
        for (int e = 0; e < eps; ++e) {
            x[i0 + e] = __builtin_amdgcn_exp2f(x[i0 + e] - xm);
            dn += x[i0 + e];
        }
        dn = bk_wave_sum(dn);
        const float idn = 1.0f / dn;
        const int truth = bf.true_idx ? bf.true_idx[(size_t)cw * tb.L + l0 + ls] : -1;
        float ss = 0.f, se = 0.f;
#pragma unroll
        for (int e = 0; e < eps; ++e) {
            const float b = x[i0 + e] * idn;
            beta[ls * tb.M + lane * eps + e] = b;
            bv[i0 + e] = b;
            const float dl = b - ((lane * eps + e) == truth ? 1.f : 0.f);
            ss += b * b;
            se += dl * dl;
        }
        ss = bk_wave_sum(ss);
        se = bk_wave_sum(se);
        if (lane == 0) {
            const size_t o = (size_t)cw * tb.L + l0 + ls;
            bf.sec_sumsq[o] = (double)ss;
            bf.sec_err[o] = (double)se;
            bf.sec_argmax[o] = arg;
        }
    }
    if (do_ab) {
        __syncthreads();
        bk_ab_column(tb, bf, c, cw, tid, bv, smem);
    }
}

template <int EPS>
static int blk_set_attrs(size_t lds) {
    static size_t done = 0;
    if (done >= lds) return SG_OK;
    SG_HIP(hipFuncSetAttribute((const void *)blk_az<EPS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    done = lds;
    return SG_OK;
}

// section size M = 64 EPS, 64 <= M <= 1024 (compile-time, so the per-lane
// entry arrays stay in registers)
#define BK_EPS_DISPATCH(M, F, ...)                                                   \
    switch (M) {                                                                     \
    case 64: F<1>(__VA_ARGS__); break;                                               \
    case 128: F<2>(__VA_ARGS__); break;                                              \
    case 256: F<4>(__VA_ARGS__); break;                                              \
    case 512: F<8>(__VA_ARGS__); break;                                              \
    case 1024: F<16>(__VA_ARGS__); break;                                            \
    default: return fail(SG_ERR_UNSUPPORTED, "block engine: section size M=%d", M); \
    }

template <int EPS>
static void bk_launch_az(const BlkTables &tb, const AmpBufs<float> &bf, int do_ab, size_t lds, hipStream_t s,
                         int *rc) {
    *rc = blk_set_attrs<EPS>(lds);
    if (*rc == SG_OK) hipLaunchKernelGGL(blk_az<EPS>, dim3(tb.Lc, bf.B), dim3(BK_THREADS), lds, s, tb, bf, do_ab);
}

int blk_launch_g(const BlkTables &tb, const AmpBufs<float> &bf, cx<float> *gbuf, hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    ProfScope ps(SG_PH_AZ_A, s);
    hipLaunchKernelGGL(blk_g, dim3((tb.ngs + 255) / 256, (bf.B + BK_GCW - 1) / BK_GCW), dim3(256), 0, s, tb, bf, gbuf);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

int blk_launch_az(const BlkTables &tb, const AmpBufs<float> &bf, bool then_ab, hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    const size_t lds = blk_lds_bytes(tb.Mc);
    int rc = SG_OK;
    ProfScope ps(SG_PH_AZ_B, s);
    BK_EPS_DISPATCH(tb.M, bk_launch_az, tb, bf, then_ab ? 1 : 0, lds, s, &rc);
    SG_TRY(rc);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

}  // namespace sg
