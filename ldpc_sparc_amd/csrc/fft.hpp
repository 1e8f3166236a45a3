// Workgroup-cooperative complex FFTs in LDS for gfx950 (device code).
//
// Used by the sub-sampled DCT design operator (amp_dct.hip): the length-w
// DCT-II/III of the reference (sparc.py:687-699, scipy.fftpack dct/idct,
// norm='ortho') is evaluated as a length-w/2 complex FFT (Makhoul packing),
// itself split four-step into P-point column FFTs and Q-point row FFTs.  Each
// of those short FFTs runs here: a Stockham autosort radix-8/4/2 schedule in
// which every thread keeps EPT complex values in registers; one stage = load
// R inputs per butterfly from LDS, twiddle, R-point DFT in registers, barrier,
// store R outputs, barrier.  Twiddles come from a per-size table
// tw[i] = exp(-2*pi*i*i/n), i < n, computed in double on the host.
#pragma once
#include <hip/hip_runtime.h>

namespace sg {

template <typename T>
struct cx {
    T x, y;
};

template <typename T>
__device__ __forceinline__ cx<T> cadd(cx<T> a, cx<T> b) { return {a.x + b.x, a.y + b.y}; }
template <typename T>
__device__ __forceinline__ cx<T> csub(cx<T> a, cx<T> b) { return {a.x - b.x, a.y - b.y}; }
template <typename T>
__device__ __forceinline__ cx<T> cmul(cx<T> a, cx<T> b) {
    return {a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
}
// Single precision: the product in two packed instructions, t = a.x (b.x, b.y)
// by v_pk_mul_f32, then t + (-a.y b.y, a.y b.x) by one v_pk_fma_f32 whose
// operand swizzles and lane negation the compiler folds into op_sel / neg_lo.
// The scalar form lowers to three to six instructions; in the 8192-point LDS
// FFT of the per-codeword engine this takes the stage-twiddle cost from 4.5 k
// to 2.0 k cycles per transform (tools/fftbench variant 5).  Written as vector
// arithmetic, not inline assembly: the compiler's hazard recognizer must see
// the operands (a v_pk op reading a v_sin_f32 result in the next instruction
// needs a wait state that it does not insert for an asm block -- measured
// wrong in tools/fftbench's accuracy check).
typedef float sg_f2 __attribute__((ext_vector_type(2)));
// The packed instructions' modifiers negate whole operands and the compiler
// does not fold a one-lane negation into them (a {-y, y} operand costs a xor
// and a move), so the sign patterns are constant pairs (amp_cw2.hip c2_mul).
__device__ __forceinline__ sg_f2 sg_pm() { return sg_f2{1.f, -1.f}; }
__device__ __forceinline__ sg_f2 sg_mp() { return sg_f2{-1.f, 1.f}; }
template <>
__device__ __forceinline__ cx<float> cmul<float>(cx<float> a, cx<float> b) {
    const sg_f2 A = {a.x, a.y}, B = {b.x, b.y};
    const sg_f2 r = __builtin_elementwise_fma(A.yy * B.yx, sg_mp(), A.xx * B);
    return {r.x, r.y};
}
// a conj(b) in three packed instructions
__device__ __forceinline__ cx<float> cmulc_f(cx<float> a, cx<float> b) {
    const sg_f2 A = {a.x, a.y}, B = {b.x, b.y};
    const sg_f2 r = __builtin_elementwise_fma(A.yy, B.yx, (A.xx * B) * sg_pm());
    return {r.x, r.y};
}
// x + a b and x + a conj(b) in two packed FMAs (single precision)
__device__ __forceinline__ cx<float> cmac_pk(cx<float> x, cx<float> a, cx<float> b) {
    const sg_f2 X = {x.x, x.y}, A = {a.x, a.y}, B = {b.x, b.y};
    const sg_f2 an = {-a.y, a.y};
    const sg_f2 r = __builtin_elementwise_fma(an, B.yx, __builtin_elementwise_fma(A.xx, B, X));
    return {r.x, r.y};
}
__device__ __forceinline__ cx<float> cmacc_pk(cx<float> x, cx<float> a, cx<float> b) {
    const sg_f2 X = {x.x, x.y}, A = {a.x, a.y}, B = {b.x, b.y};
    const sg_f2 an = {a.y, -a.x};
    const sg_f2 r = __builtin_elementwise_fma(an, B.yy, __builtin_elementwise_fma(A, B.xx, X));
    return {r.x, r.y};
}
template <typename T>
__device__ __forceinline__ cx<T> cconj(cx<T> a) { return {a.x, -a.y}; }
// multiply by -i (forward) or +i (inverse)
template <typename T, bool INV>
__device__ __forceinline__ cx<T> mul_mi(cx<T> a) {
    if constexpr (sizeof(T) == 4) {
        const sg_f2 r = sg_f2{a.y, a.x} * (INV ? sg_mp() : sg_pm());
        return {r.x, r.y};
    } else {
        return INV ? cx<T>{-a.y, a.x} : cx<T>{a.y, -a.x};
    }
}

template <typename T, bool INV>
__device__ __forceinline__ void dft2(cx<T> *a) {
    const cx<T> t = a[0];
    a[0] = cadd(t, a[1]);
    a[1] = csub(t, a[1]);
}

template <typename T, bool INV>
__device__ __forceinline__ void dft4(cx<T> *a) {
    if constexpr (sizeof(T) == 4) {  // x -+ i d as one packed FMA with a constant sign pair
        const sg_f2 a0 = {a[0].x, a[0].y}, a1 = {a[1].x, a[1].y}, a2 = {a[2].x, a[2].y}, a3 = {a[3].x, a[3].y};
        const sg_f2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, d = a1 - a3;
        const sg_f2 r0 = t0 + t2, r2 = t0 - t2;
        const sg_f2 r1 = __builtin_elementwise_fma(d.yx, INV ? sg_mp() : sg_pm(), t1);
        const sg_f2 r3 = __builtin_elementwise_fma(d.yx, INV ? sg_pm() : sg_mp(), t1);
        a[0] = {r0.x, r0.y};
        a[1] = {r1.x, r1.y};
        a[2] = {r2.x, r2.y};
        a[3] = {r3.x, r3.y};
    } else {
        const cx<T> t0 = cadd(a[0], a[2]), t1 = csub(a[0], a[2]);
        const cx<T> t2 = cadd(a[1], a[3]), t3 = mul_mi<T, INV>(csub(a[1], a[3]));
        a[0] = cadd(t0, t2);
        a[2] = csub(t0, t2);
        a[1] = cadd(t1, t3);
        a[3] = csub(t1, t3);
    }
}

template <typename T, bool INV>
__device__ __forceinline__ void dft8(cx<T> *a) {
    const T r = T(0.70710678118654752440084436210484903928);
    cx<T> b[4], c[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        b[k] = cadd(a[k], a[k + 4]);
        c[k] = csub(a[k], a[k + 4]);
    }
    // c[k] *= w8^k (forward w8 = e^{-i pi/4}; inverse conjugated)
    c[1] = INV ? cx<T>{(c[1].x - c[1].y) * r, (c[1].x + c[1].y) * r}
               : cx<T>{(c[1].x + c[1].y) * r, (c[1].y - c[1].x) * r};
    c[2] = mul_mi<T, INV>(c[2]);
    c[3] = INV ? cx<T>{-(c[3].x + c[3].y) * r, (c[3].x - c[3].y) * r}
               : cx<T>{(c[3].y - c[3].x) * r, -(c[3].x + c[3].y) * r};
    dft4<T, INV>(b);
    dft4<T, INV>(c);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        a[2 * m] = b[m];
        a[2 * m + 1] = c[m];
    }
}

// 16-point DFT as 4 x 4: inputs n = 4 n1 + n2, outputs k = k1 + 4 k2.
template <typename T, bool INV>
__device__ __forceinline__ void dft16(cx<T> *a) {
    const T c1 = T(0.92387953251128675612818318939678828682);  // cos(pi/8)
    const T s1 = T(0.38268343236508977172845998403039886676);  // sin(pi/8)
    const T r2 = T(0.70710678118654752440084436210484903928);
    cx<T> y[4][4];
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
        cx<T> v[4] = {a[n2], a[n2 + 4], a[n2 + 8], a[n2 + 12]};
        dft4<T, INV>(v);
#pragma unroll
        for (int k1 = 0; k1 < 4; ++k1) y[n2][k1] = v[k1];
    }
    // y[n2][k1] *= w16^(n2 k1) (forward w16 = e^{-i pi/8}; inverse conjugated)
    auto tw16 = [&](cx<T> x, T c, T s) -> cx<T> {  // x * (c - i s) forward, (c + i s) inverse
        if constexpr (sizeof(T) == 4) {
            const sg_f2 X = {x.x, x.y};
            const sg_f2 r = __builtin_elementwise_fma(X.yx, INV ? sg_f2{-s, s} : sg_f2{s, -s}, X * sg_f2{c, c});
            return {r.x, r.y};
        } else {
            return INV ? cx<T>{x.x * c - x.y * s, x.x * s + x.y * c} : cx<T>{x.x * c + x.y * s, x.y * c - x.x * s};
        }
    };
    y[1][1] = tw16(y[1][1], c1, s1);
    y[1][2] = tw16(y[1][2], r2, r2);
    y[1][3] = tw16(y[1][3], s1, c1);
    y[2][1] = tw16(y[2][1], r2, r2);
    y[2][2] = mul_mi<T, INV>(y[2][2]);
    y[2][3] = tw16(y[2][3], -r2, r2);
    y[3][1] = tw16(y[3][1], s1, c1);
    y[3][2] = tw16(y[3][2], -r2, r2);
    y[3][3] = tw16(y[3][3], -c1, -s1);
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
        cx<T> v[4] = {y[0][k1], y[1][k1], y[2][k1], y[3][k1]};
        dft4<T, INV>(v);
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) a[k1 + 4 * k2] = v[k2];
    }
}

template <typename T, bool INV, int R>
__device__ __forceinline__ void dftR(cx<T> *a) {
    if (R == 2) dft2<T, INV>(a);
    else if (R == 4) dft4<T, INV>(a);
    else if (R == 8) dft8<T, INV>(a);
    else dft16<T, INV>(a);
}

// Sequence layout in LDS: element e of sequence s lives at d[s*ss + e*es].
// SEQ_FAST: consecutive butterflies walk sequences first (use when sequences
// are the unit-stride dimension, e.g. column tiles); otherwise they walk the
// elements of one sequence first.
template <typename T, bool INV, int R, int EPT, bool SEQ_FAST>
__device__ __forceinline__ void stockham_stage(cx<T> *d, int n, int nseq, int es, int ss, int Ns,
                                               const cx<T> *__restrict__ tw, int tid, int nthr) {
    constexpr int NB = EPT / R;  // butterflies per thread
    const int nbf = n / R;       // butterflies per sequence
    cx<T> v[EPT];
    int base_out[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int b = tid + i * nthr;
        const int s = SEQ_FAST ? (b % nseq) : (b / nbf);
        const int j = SEQ_FAST ? (b / nseq) : (b % nbf);
        const int k = j % Ns;
        cx<T> *ds = d + s * ss;
#pragma unroll
        for (int r = 0; r < R; ++r) v[i * R + r] = ds[(j + r * nbf) * es];
        if (Ns > 1) {
            const int step = n / (Ns * R);  // tw index of w_{Ns R}^{r k}
#pragma unroll
            for (int r = 1; r < R; ++r) {
                cx<T> w = tw[r * k * step];
                if (INV) w.y = -w.y;
                v[i * R + r] = cmul(v[i * R + r], w);
            }
        }
        dftR<T, INV, R>(&v[i * R]);
        base_out[i] = s * ss + ((j - k) * R + k) * es;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NB; ++i) {
#pragma unroll
        for (int r = 0; r < R; ++r) d[base_out[i] + r * Ns * es] = v[i * R + r];
    }
    __syncthreads();
}

// Full FFT of nseq sequences of length n = 2^log2n in LDS, nthr*EPT == n*nseq.
// Radix plan: as many radix-8 stages as possible, the remainder as one radix-4
// or two radix-4 (never a radix-2 unless n == 2).
template <typename T, bool INV, int EPT, bool SEQ_FAST>
__device__ void lds_fft(cx<T> *d, int log2n, int nseq, int es, int ss, const cx<T> *__restrict__ tw, int tid,
                        int nthr) {
    const int n = 1 << log2n;
    int a8 = log2n / 3, rem = log2n % 3, n4 = 0, n2 = 0;
    if (rem == 2) n4 = 1;
    else if (rem == 1) {
        if (a8 >= 1) { a8 -= 1; n4 = 2; }
        else n2 = 1;
    }
    int Ns = 1;
    for (int s = 0; s < n2; ++s) {
        stockham_stage<T, INV, 2, EPT, SEQ_FAST>(d, n, nseq, es, ss, Ns, tw, tid, nthr);
        Ns *= 2;
    }
    for (int s = 0; s < n4; ++s) {
        stockham_stage<T, INV, 4, EPT, SEQ_FAST>(d, n, nseq, es, ss, Ns, tw, tid, nthr);
        Ns *= 4;
    }
    for (int s = 0; s < a8; ++s) {
        stockham_stage<T, INV, 8, EPT, SEQ_FAST>(d, n, nseq, es, ss, Ns, tw, tid, nthr);
        Ns *= 8;
    }
}

// ---------------------------------------------------------------------------
// Single-sequence variant for the LDS-resident stage-1 transforms of the
// regular AMP engine: one sequence of n = 2^log2n points in d[0..n), every
// index computed with shifts and masks (no integer division), the twiddles of
// a butterfly loaded before its first use.
// Twiddles come from a per-stage table laid out in thread order:
// stw[k * (R - 1) + r - 1] = w_{Ns R}^{r k} (forward), so the R - 1 twiddles of
// a butterfly are contiguous and a wavefront reads a contiguous range.
// LDS layout of the single-sequence FFT: element i at fsw(i), the low four
// index bits XOR-swizzled by the next four.  Runs of 32 consecutive elements
// (every stage's loads, and the stores of the later stages) stay inside one
// aligned 32-element block, so a ds_read_b64 lane group touches 64 distinct
// banks; the stride-16 stores of the first radix-16 stage land on 16 distinct
// bank pairs.  Adding a multiple of 256 commutes with the swizzle.
__host__ __device__ __forceinline__ int fsw(int i) { return i ^ ((i >> 4) & 15); }
// Skewed layout of the class-ordered s image (reduction of section segments):
// element i at fpad(i) = i + i/16, so one-thread-per-segment reads spread
// over the banks.
__host__ __device__ __forceinline__ int fpad(int i) { return i + (i >> 4); }
// Padded layout (PAD = true in the compile-time stages below; the split
// engine's image layout, amp.hpp c2pos): element i at ppos(i) = i + i/32.
// Every load and store of a stage is then a per-thread base plus a constant
// (ppos(b + c) = ppos(b) + ppos_off(...)), so no swizzle arithmetic per
// element; the price is one padding slot per 32 elements.
__host__ __device__ constexpr int ppos(int i) { return i + (i >> 5); }
// ppos(b + NS r) - ppos(b) for the bases b of stockham1_stage_ct: NS = 1 with
// b a multiple of R (R | 32), NS = 16 with b mod 32 < 16, NS a multiple of 32
__host__ __device__ constexpr int ppos_off(int NS, int r) {
    return NS == 1 ? r : NS == 16 ? 16 * r + (r >> 1) : r * (NS + NS / 32);
}

// Stage twiddles w^(r k), r < R, of butterfly k are rebuilt from TWN(R) table
// entries per k (a twentieth of the table traffic of R - 1 entries, and few
// enough registers to be loaded a stage ahead):
//   R = 16: w, w^2, w^3, w^4, w^8, w^12 -> w^(4a+b) = w^(4a) w^b (one product)
//   R = 8:  w, w^2, w^3, w^4             -> w^(4+b) = w^4 w^b
//   R = 4:  w -> w^2 = w w, w^3 = w w^2;  R = 2: w
__host__ __device__ constexpr int tw_per_k(int R) { return R == 16 ? 6 : R == 8 ? 4 : 1; }
// table exponents of the TWN(R) entries
__host__ __device__ inline int tw_exp(int R, int t) {
    if (R == 16) return t < 4 ? t + 1 : 4 * (t - 2);  // 1 2 3 4 8 12
    return t + 1;                                     // R = 8: 1 2 3 4; R <= 4: 1
}

template <typename T, bool INV, int R>
__device__ __forceinline__ void tw_expand(const cx<T> *wl, cx<T> *w /* [R], w[0] unused */) {
    cx<T> a[tw_per_k(R)];
#pragma unroll
    for (int t = 0; t < tw_per_k(R); ++t) a[t] = INV ? cconj(wl[t]) : wl[t];
    if constexpr (R == 2) {
        w[1] = a[0];
    } else if constexpr (R == 4) {
        w[1] = a[0];
        w[2] = cmul(a[0], a[0]);
        w[3] = cmul(a[0], w[2]);
    } else if constexpr (R == 8) {
#pragma unroll
        for (int b = 1; b < 4; ++b) {
            w[b] = a[b - 1];
            w[4 + b] = cmul(a[3], a[b - 1]);
        }
        w[4] = a[3];
    } else {
#pragma unroll
        for (int b = 1; b < 4; ++b) w[b] = a[b - 1];
        w[4] = a[3];
        w[8] = a[4];
        w[12] = a[5];
#pragma unroll
        for (int q = 1; q < 4; ++q)
#pragma unroll
            for (int b = 1; b < 4; ++b) w[4 * q + b] = cmul(w[4 * q], a[b - 1]);
    }
}

// v[r] *= w^r with the products of tw_expand, each formed right before its
// use (fewer live registers than the expanded w[R]; identical arithmetic)
template <typename T, bool INV, int R>
__device__ __forceinline__ void tw_apply(const cx<T> *wl, cx<T> *v) {
    if constexpr (R == 16 && sizeof(T) == 4) {  // the products of the forward twiddles; the inverse
                                                // applies their conjugates (three packed instructions)
        auto ap = [&](cx<float> x, cx<float> w) { return INV ? cmulc_f(x, w) : cmul(x, w); };
#pragma unroll
        for (int b = 1; b < 4; ++b) v[b] = ap(v[b], wl[b - 1]);
#pragma unroll
        for (int q = 1; q < 4; ++q) {
            const cx<T> wq = wl[q + 2];  // w^4, w^8, w^12
            v[4 * q] = ap(v[4 * q], wq);
#pragma unroll
            for (int b = 1; b < 4; ++b) v[4 * q + b] = ap(v[4 * q + b], cmul(wq, wl[b - 1]));
        }
    } else if constexpr (R == 16) {
        cx<T> a[6];
#pragma unroll
        for (int t = 0; t < 6; ++t) a[t] = INV ? cconj(wl[t]) : wl[t];
#pragma unroll
        for (int b = 1; b < 4; ++b) v[b] = cmul(v[b], a[b - 1]);
#pragma unroll
        for (int q = 1; q < 4; ++q) {
            const cx<T> wq = a[q + 2];  // w^4, w^8, w^12
            v[4 * q] = cmul(v[4 * q], wq);
#pragma unroll
            for (int b = 1; b < 4; ++b) v[4 * q + b] = cmul(v[4 * q + b], cmul(wq, a[b - 1]));
        }
    } else {
        cx<T> w[R];
        tw_expand<T, INV, R>(wl, w);
#pragma unroll
        for (int r = 1; r < R; ++r) v[r] = cmul(v[r], w[r]);
    }
}

template <typename T, bool INV, int R, int EPT>
__device__ __forceinline__ void stockham1_stage(cx<T> *d, int log2n, int log2Ns, const cx<T> *__restrict__ stw,
                                                int tid, int nthr) {
    constexpr int NB = EPT / R;
    constexpr int LR = (R == 2) ? 1 : (R == 4) ? 2 : (R == 8) ? 3 : 4;
    const int nbf = 1 << (log2n - LR);
    const int Ns = 1 << log2Ns;
    cx<T> v[EPT];
    int base_out[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int j = tid + i * nthr;
        const int k = j & (Ns - 1);
#pragma unroll
        for (int r = 0; r < R; ++r) v[i * R + r] = d[fsw(j + r * nbf)];
        if (log2Ns > 0) {
            constexpr int TWN = tw_per_k(R);
            cx<T> wl[TWN], w[R];
#pragma unroll
            for (int t = 0; t < TWN; ++t) wl[t] = stw[k * TWN + t];
            tw_expand<T, INV, R>(wl, w);
#pragma unroll
            for (int r = 1; r < R; ++r) v[i * R + r] = cmul(v[i * R + r], w[r]);
        }
        dftR<T, INV, R>(&v[i * R]);
        base_out[i] = ((j - k) << LR) + k;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NB; ++i) {
#pragma unroll
        for (int r = 0; r < R; ++r) d[fsw(base_out[i] + r * Ns)] = v[i * R + r];
    }
    __syncthreads();
}

// n = 2^log2n, nthr * EPT == n; radix-8 stages with one radix-4 or two
// radix-4 (or one radix-2) for the remainder, smallest radices first.
// Radix plan shared with the host table builder: EPT 16 -> radix-16 stages
// after one smaller first stage for the remainder; EPT 8 -> radix-8 stages
// with radix-4 (or one radix-2) first.  Returns the number of stages.
__host__ __device__ inline int fft1_plan(int log2n, int ept, int *radix /* [8] */) {
    int ns = 0;
    if (ept >= 16) {  // radix-16 stages first: with stride-1 inputs a small first radix writes bank-conflicted
        const int rem = log2n % 4;
        for (int i = 0; i < log2n / 4; ++i) radix[ns++] = 16;
        if (rem) radix[ns++] = 1 << rem;
    } else {
        int a8 = log2n / 3, rem = log2n % 3;
        if (rem == 2) radix[ns++] = 4;
        else if (rem == 1) {
            if (a8 >= 1) { a8 -= 1; radix[ns++] = 4; radix[ns++] = 4; }
            else radix[ns++] = 2;
        }
        for (int i = 0; i < a8; ++i) radix[ns++] = 8;
    }
    return ns;
}

// In-place FFT of d[fpad(0..n)), n = 2^log2n = nthr * EPT.  stw: per-stage
// twiddle tables concatenated in stage order (see stockham1_stage).
template <typename T, bool INV, int EPT>
__device__ void lds_fft1(cx<T> *d, int log2n, const cx<T> *__restrict__ stw, int tid, int nthr) {
    int radix[8];
    const int ns = fft1_plan(log2n, EPT, radix);
    int lns = 0;
    size_t off = 0;
    for (int st = 0; st < ns; ++st) {
        const int R = radix[st];
        if (R == 2) stockham1_stage<T, INV, 2, EPT>(d, log2n, lns, stw + off, tid, nthr);
        else if (R == 4) stockham1_stage<T, INV, 4, EPT>(d, log2n, lns, stw + off, tid, nthr);
        else if (R == 8) stockham1_stage<T, INV, 8, EPT>(d, log2n, lns, stw + off, tid, nthr);
        else if (EPT >= 16) stockham1_stage<T, INV, (EPT >= 16 ? 16 : 8), EPT>(d, log2n, lns, stw + off, tid, nthr);
        off += (size_t)(1 << lns) * (R == 16 ? 6 : R == 8 ? 4 : 1);
        lns += (R == 2) ? 1 : (R == 4) ? 2 : (R == 8) ? 3 : 4;
    }
}

// ---------------------------------------------------------------------------
// Compile-time specialisation of lds_fft1 for the hot sizes: every stride and
// stage offset is a constant, so LDS addresses fold into instruction offsets.
constexpr int fft1_nstages_ct(int log2n, int ept) {
    return ept >= 16 ? (log2n / 4 + (log2n % 4 ? 1 : 0))
                     : (log2n % 3 == 1 && log2n / 3 >= 1 ? log2n / 3 + 1 : log2n / 3 + (log2n % 3 ? 1 : 0));
}
constexpr int fft1_radix_ct(int log2n, int ept, int st) {
    if (ept >= 16) {
        const int rem = log2n % 4;
        return (rem && st == log2n / 4) ? (1 << rem) : 16;
    }
    const int rem = log2n % 3;
    if (rem == 2) return st == 0 ? 4 : 8;
    if (rem == 1) return (log2n / 3 >= 1) ? (st < 2 ? 4 : 8) : 2;
    return 8;
}
constexpr int fft1_log2ns_ct(int log2n, int ept, int st) {
    int l = 0;
    for (int i = 0; i < st; ++i) {
        const int R = fft1_radix_ct(log2n, ept, i);
        l += R == 2 ? 1 : R == 4 ? 2 : R == 8 ? 3 : 4;
    }
    return l;
}
constexpr int fft1_off_ct(int log2n, int ept, int st) {
    int off = 0;
    for (int i = 0; i < st; ++i) off += (1 << fft1_log2ns_ct(log2n, ept, i)) * tw_per_k(fft1_radix_ct(log2n, ept, i));
    return off;
}

// number of table entries a thread loads for stage ST (NB butterflies)
constexpr int fft1_twl_ct(int log2n, int ept, int st) {
    return (st < fft1_nstages_ct(log2n, ept) && fft1_log2ns_ct(log2n, ept, st) > 0)
               ? (ept / fft1_radix_ct(log2n, ept, st)) * tw_per_k(fft1_radix_ct(log2n, ept, st))
               : 0;
}

template <typename T, int EPT, int LOG2N, int ST>
__device__ __forceinline__ void fft1_tw_load_ct(const cx<T> *__restrict__ stw, int tid, cx<T> *wl) {
    if constexpr (fft1_twl_ct(LOG2N, EPT, ST) > 0) {
        constexpr int R = fft1_radix_ct(LOG2N, EPT, ST), NB = EPT / R, TWN = tw_per_k(R);
        constexpr int NS = 1 << fft1_log2ns_ct(LOG2N, EPT, ST), NTHR = (1 << LOG2N) / EPT;
        const cx<T> *t = stw + fft1_off_ct(LOG2N, EPT, ST);
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int k = (tid + i * NTHR) & (NS - 1);
#pragma unroll
            for (int q = 0; q < TWN; ++q) wl[i * TWN + q] = t[k * TWN + q];
        }
    }
}

template <typename T, bool INV, int R, int EPT, int LOG2N, int LOG2NS, bool PAD = false>
__device__ __forceinline__ void stockham1_stage_ct(cx<T> *d, const cx<T> *wl, int tid) {
    constexpr int NB = EPT / R;
    constexpr int LR = (R == 2) ? 1 : (R == 4) ? 2 : (R == 8) ? 3 : 4;
    constexpr int NBF = 1 << (LOG2N - LR);
    constexpr int NS = 1 << LOG2NS;
    constexpr int NTHR = (1 << LOG2N) / EPT;
    static_assert(!PAD || ((NS == 1 || NS == 16 || NS % 32 == 0) && NBF % 32 == 0 && 32 % R == 0),
                  "padded layout: stage offsets are constants only for these strides");
    cx<T> v[EPT];
    int base_out[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int j = tid + i * NTHR;
        const int k = j & (NS - 1);
        const int jp = PAD ? ppos(j) : fsw(j);
#pragma unroll
        for (int r = 0; r < R; ++r)
            v[i * R + r] = d[PAD ? jp + r * (NBF + NBF / 32) : (NBF % 256 == 0) ? jp + r * NBF : fsw(j + r * NBF)];
        if constexpr (LOG2NS > 0) tw_apply<T, INV, R>(wl + i * tw_per_k(R), &v[i * R]);
        dftR<T, INV, R>(&v[i * R]);
        base_out[i] = ((j - k) << LR) + k;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int bp = PAD ? ppos(base_out[i]) : fsw(base_out[i]);
#pragma unroll
        for (int r = 0; r < R; ++r)
            d[PAD ? bp + ppos_off(NS, r) : (NS % 256 == 0) ? bp + r * NS : fsw(base_out[i] + r * NS)] = v[i * R + r];
    }
    __syncthreads();
}

// Stage ST runs with its table entries already in registers (wl) while the
// next stage's entries are in flight.
template <typename T, bool INV, int EPT, int LOG2N, int ST>
__device__ __forceinline__ void lds_fft1_ct_from(cx<T> *d, const cx<T> *__restrict__ stw, int tid, const cx<T> *wl) {
    if constexpr (ST < fft1_nstages_ct(LOG2N, EPT)) {
        constexpr int R = fft1_radix_ct(LOG2N, EPT, ST);
        constexpr int NXT = fft1_twl_ct(LOG2N, EPT, ST + 1);
        cx<T> wn[NXT > 0 ? NXT : 1];
        fft1_tw_load_ct<T, EPT, LOG2N, ST + 1>(stw, tid, wn);
        stockham1_stage_ct<T, INV, R, EPT, LOG2N, fft1_log2ns_ct(LOG2N, EPT, ST)>(d, wl, tid);
        lds_fft1_ct_from<T, INV, EPT, LOG2N, ST + 1>(d, stw, tid, wn);
    }
}

template <typename T, bool INV, int EPT, int LOG2N>
__device__ __forceinline__ void lds_fft1_ct(cx<T> *d, const cx<T> *__restrict__ stw, int tid) {
    constexpr int N0 = fft1_twl_ct(LOG2N, EPT, 0);
    cx<T> w0[N0 > 0 ? N0 : 1];
    fft1_tw_load_ct<T, EPT, LOG2N, 0>(stw, tid, w0);
    lds_fft1_ct_from<T, INV, EPT, LOG2N, 0>(d, stw, tid, w0);
}

// Stage ST of the same plan with its stage twiddles w_(Ns R)^(e k) from the
// hardware sine / cosine instead of the table (single precision): the
// argument is in revolutions and (e k mod Ns R) / (Ns R) is exact, and no
// global load sits between the transform's barriers.
template <bool INV, int EPT, int LOG2N, int ST, bool PAD = false>
__device__ __forceinline__ void fft1_stage_sincos(cx<float> *d, int tid) {
    constexpr int R = fft1_radix_ct(LOG2N, EPT, ST), LNS = fft1_log2ns_ct(LOG2N, EPT, ST);
    constexpr int NB = EPT / R, TWN = tw_per_k(R), NTHR = (1 << LOG2N) / EPT;
    constexpr int LR = R == 2 ? 1 : R == 4 ? 2 : R == 8 ? 3 : 4;
    cx<float> wl[LNS > 0 ? NB * TWN : 1];
    if constexpr (LNS > 0) {
        constexpr float inv = 1.0f / (float)(1 << (LNS + LR));
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int k = (tid + i * NTHR) & ((1 << LNS) - 1);
#pragma unroll
            for (int q = 0; q < TWN; ++q) {
                const float x = (float)((tw_exp(R, q) * k) & ((1 << (LNS + LR)) - 1)) * inv;
                wl[i * TWN + q] = {__builtin_amdgcn_cosf(x), -__builtin_amdgcn_sinf(x)};
            }
        }
    }
    stockham1_stage_ct<float, INV, R, EPT, LOG2N, LNS, PAD>(d, wl, tid);
}
// stages ST0 .. ST1 - 1 (PAD: element i at ppos(i))
template <bool INV, int EPT, int LOG2N, int ST0, int ST1, bool PAD = false>
__device__ __forceinline__ void lds_fft1_sincos(cx<float> *d, int tid) {
    if constexpr (ST0 < ST1) {
        fft1_stage_sincos<INV, EPT, LOG2N, ST0, PAD>(d, tid);
        lds_fft1_sincos<INV, EPT, LOG2N, ST0 + 1, ST1, PAD>(d, tid);
    }
}

// Variant without the next stage's twiddles in flight (fewer live registers
// for kernels that hold other state across the FFT)
template <typename T, bool INV, int EPT, int LOG2N, int ST>
__device__ __forceinline__ void lds_fft1_ct_lean_from(cx<T> *d, const cx<T> *__restrict__ stw, int tid) {
    if constexpr (ST < fft1_nstages_ct(LOG2N, EPT)) {
        constexpr int R = fft1_radix_ct(LOG2N, EPT, ST);
        constexpr int NW = fft1_twl_ct(LOG2N, EPT, ST);
        cx<T> wl[NW > 0 ? NW : 1];
        fft1_tw_load_ct<T, EPT, LOG2N, ST>(stw, tid, wl);
        stockham1_stage_ct<T, INV, R, EPT, LOG2N, fft1_log2ns_ct(LOG2N, EPT, ST)>(d, wl, tid);
        lds_fft1_ct_lean_from<T, INV, EPT, LOG2N, ST + 1>(d, stw, tid);
    }
}
template <typename T, bool INV, int EPT, int LOG2N>
__device__ __forceinline__ void lds_fft1_ct_lean(cx<T> *d, const cx<T> *__restrict__ stw, int tid) {
    lds_fft1_ct_lean_from<T, INV, EPT, LOG2N, 0>(d, stw, tid);
}

}  // namespace sg
