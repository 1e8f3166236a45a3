// Split per-codeword AMP engine in double precision (the f64 C2 path, what an
// unmodified sparc_sim caller runs).  Same iteration as amp_cw2.hip --
// sparc.py:883-999 with the sub-sampled DCT operators of sub_dct :648-701 --
// over the split engine's host tables (build_cw2: output slots grouped by
// conjugate row pair, class slices, first-stage masks), five launches:
//
//   cw2d_ab    (2 B)  half h of the Q classes, in DESCENDING class order: beta
//              of the class (cw2d_stats' output, class order) -> LDS scatter
//              -> P-point FFT -> for every owned output, Horner steps
//                  H[a]      <- H[a] S + Y_m[r],
//                  conj H[b] <- conj H[b] S + conj Y_m[P - r],  S = w_N2^a,
//              so the sum over the half's classes of w_N2^(m a) Y_m needs one
//              complex multiply-add per output and class and no per-class
//              twiddle; times S^(first class) at the end.
//   cw2d_ctrl  (B)  z = y - (the halves' parts) + b z, phi, tau (sparc.py:931-969).
//   cw2d_az    (2 B)  half h of the classes, ascending: rows r and P - r of each
//              owned pair from al z/phi conj(W) and be z/phi W (W = w_N2^(m a)
//              rotated by S per class) -> inverse FFT -> s = beta_prev + tau u
//              (sparc.py:972) in class order.
//   cw2d_stats (B L / 4)  one wavefront per section: the softmax of s over the
//              section (sparc.py:429-432) -> beta (class order), section max and
//              1/sum, sum beta^2 and squared error (sparc.py:973-981).
//   cw2d_final (B)  psi, NMSE, early stop (sparc.py:973-988).
//
// Why a separate engine: the staged f64 engine (amp_fused.hip) passes the
// needed rows of both FFT stages through HBM (four passes of ~6.5 MB per
// codeword-iteration at C2, beside 12 MB of s) and runs each class at one
// workgroup per CU with nothing overlapping its memory phases.  Here the
// per-iteration HBM traffic is s and beta (Ab reads beta, Az reads beta and
// writes s, the statistics read s and write beta: 20 MB per codeword-iteration)
// and the per-codeword slot vectors.  A complex double image of P = 8192 points
// is 132 KB, so one 512-thread workgroup per CU (8 wavefronts): the softmax and
// its statistics, whose section reductions need barriers and LDS round trips,
// run in their own launch at full occupancy instead (inside Az they took half
// of its time, profiles/r05_f64_ablation.txt), and the exponentials are one per
// entry and iteration.
//
// Twiddles are double precision: the radix-32 stage's and the DFT-16's
// constants as literals, the first radix-16 stage's (w_512^(r k)) from an LDS
// table filled per launch from the plan's w_8192^k table, the second's from
// w_8192^k and w_8192^(4k) of the thread (two L1 loads per transform) and
// their products.  Parity bar: the f64 bars of DESIGN.md "Oracle and parity"
// (same decisions and stopping iterations as the staged engine and the CPU
// restatement, NMSE within 1e-9; tests/test_amp_cw2d_gpu.py).
#include "amp.hpp"

namespace sg {
namespace {

constexpr int D_T = CW2_THREADS;  // 512
// Phase ablation for timing studies only (tools/mk_variant.sh ... -DD_ABL=<mask>; results are garbage, the
// shipped build has 0): Ab 1 FFT, 2 accumulation, 4 slice loads, 8 beta exponentials, 16 beta stores,
// 32 scatter; Az 64 FFT, 128 rows, 256 slice loads, 512 statistics, 1024 s stores, 2048 statistics'
// exponentials
#ifndef D_ABL
#define D_ABL 0
#endif
#define D_SKIP(bit) ((D_ABL & (bit)) != 0)
// Az: the rows' class-invariant tables requested at the end of the previous class (1: 84 loop-carried
// VGPRs, 68 spilled, Az 1.05 -> 1.93 ms per launch) or at the rows (0)
#ifndef D_AZPF
#define D_AZPF 0
#endif
constexpr int D_P = 8192;
constexpr int D_SC = 9, D_NC = 2, D_SN = D_SC * D_NC;  // 18 class entries per thread (CW2_SLICE / 512)
static_assert(D_SN * D_T == CW2_SLICE, "class slices of 18 entries per thread");

typedef double d2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) d2 d2lds;
typedef __attribute__((address_space(3))) double dlds;
// complex element pos of the LDS (16 bytes each); the kernels have no static LDS
__device__ __forceinline__ d2lds *d_at(int pos) { return (d2lds *)(size_t)(16u * (uint32_t)pos); }
// real element idx (8 bytes each): the class tables' image indices 2 c2pos(i) + component
__device__ __forceinline__ dlds *d_re(uint32_t idx) { return (dlds *)(size_t)(8u * idx); }

// LDS layout, complex (16-byte) positions
constexpr int D_IMG = c2pos(D_P);           // 8448: the padded image, element i at c2pos(i)
constexpr int D_TRASH = D_IMG + 1024;       // one complex slot: writes of padded entries and unused rows (where
                                            // the class tables' trash index puts it: after the image and the
                                            // f32 engine's section statistics, amp_cw2.hip)
static_assert(16 * D_TRASH == 8 * (int)CW2_TRASH, "the class tables' trash index lands on the trash slot");
constexpr int D_TW1 = D_TRASH + 1;          // [15][32] w_512^(r k) of the first radix-16 stage
constexpr int D_CP_BYTES = 16 * (D_TW1 + 15 * 32);
constexpr int D_LDS_BYTES = D_CP_BYTES + 4 * 72;  // + the class pointers (Q + 1 <= 72)
static_assert(D_LDS_BYTES <= 160 * 1024, "LDS budget");

__device__ __forceinline__ int d_opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

__device__ __forceinline__ d2 dmul(d2 a, d2 w) {
    return d2{__builtin_fma(a.x, w.x, -(a.y * w.y)), __builtin_fma(a.x, w.y, a.y * w.x)};
}
__device__ __forceinline__ d2 dconj(d2 a) { return d2{a.x, -a.y}; }
// a w + c
__device__ __forceinline__ d2 dmad(d2 a, d2 w, d2 c) {
    return d2{__builtin_fma(a.x, w.x, __builtin_fma(-a.y, w.y, c.x)), __builtin_fma(a.x, w.y, __builtin_fma(a.y, w.x, c.y))};
}
template <bool INV>
__device__ __forceinline__ d2 dmi(d2 a) {  // * -i (forward), * +i (inverse)
    return INV ? d2{-a.y, a.x} : d2{a.y, -a.x};
}

template <bool INV>
__device__ __forceinline__ void d_dft4(d2 &a0, d2 &a1, d2 &a2, d2 &a3) {
    const d2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, d = dmi<INV>(a1 - a3);
    a0 = t0 + t2;
    a2 = t0 - t2;
    a1 = t1 + d;
    a3 = t1 - d;
}

// 16-point DFT as 4 x 4 (inputs n = 4 n1 + n2, outputs k = k1 + 4 k2), as amp_cw2.hip c2_dft16
template <bool INV>
__device__ __forceinline__ void d_dft16(d2 *a) {
    const double c1 = 0.92387953251128675613, s1 = 0.38268343236508977173, r2 = 0.70710678118654752440;
    d2 y[4][4];
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
        d2 v0 = a[n2], v1 = a[n2 + 4], v2 = a[n2 + 8], v3 = a[n2 + 12];
        d_dft4<INV>(v0, v1, v2, v3);
        y[n2][0] = v0;
        y[n2][1] = v1;
        y[n2][2] = v2;
        y[n2][3] = v3;
    }
    // y[n2][k1] *= w16^(n2 k1): x (c - i s) forward, x (c + i s) inverse
    auto tw = [&](d2 x, double c, double s) -> d2 {
        return INV ? d2{__builtin_fma(x.x, c, -(x.y * s)), __builtin_fma(x.y, c, x.x * s)}
                   : d2{__builtin_fma(x.x, c, x.y * s), __builtin_fma(x.y, c, -(x.x * s))};
    };
    y[1][1] = tw(y[1][1], c1, s1);
    y[1][2] = tw(y[1][2], r2, r2);
    y[1][3] = tw(y[1][3], s1, c1);
    y[2][1] = tw(y[2][1], r2, r2);
    y[2][2] = dmi<INV>(y[2][2]);
    y[2][3] = tw(y[2][3], -r2, r2);
    y[3][1] = tw(y[3][1], s1, c1);
    y[3][2] = tw(y[3][2], -r2, r2);
    y[3][3] = tw(y[3][3], -c1, -s1);
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
        d2 v0 = y[0][k1], v1 = y[1][k1], v2 = y[2][k1], v3 = y[3][k1];
        d_dft4<INV>(v0, v1, v2, v3);
        a[k1] = v0;
        a[k1 + 4] = v1;
        a[k1 + 8] = v2;
        a[k1 + 12] = v3;
    }
}

// lanes 32..63 of a <-> lanes 0..31 of b, every dword of the two doubles (v_permlane32_swap)
__device__ __forceinline__ void d_swap32(d2 &a, d2 &b) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    u4 ua = __builtin_bit_cast(u4, a), ub = __builtin_bit_cast(u4, b);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const auto r = __builtin_amdgcn_permlane32_swap(ua[c], ub[c], false, false);
        ua[c] = r[0];
        ub[c] = r[1];
    }
    a = __builtin_bit_cast(d2, ua);
    b = __builtin_bit_cast(d2, ub);
}

// First Stockham stage at radix 32, the read pattern of amp_cw2.hip c2_stage0_r32 (its masks, host
// table cmask, say which image values this transform wrote; the stale ones read as zero)
template <bool INV>
__device__ __forceinline__ void d_stage0_r32(int tid, uint32_t msk) {
    const int l = tid & 63, H = l >> 5, w = tid >> 6, j = (w << 5) | (l & 31);
    d2 v[16];
    const d2lds *src = d_at(j + w + 264 * 16 * H);  // c2pos(j + 256 m) = j + w + 264 m
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) v[jj] = src[264 * jj];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {  // all-ones / zero from the sign-extended bit, on both dwords
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        const uint32_t mx = (uint32_t)((int)(msk << (31 - 2 * jj)) >> 31);
        const uint32_t my = (uint32_t)((int)(msk << (30 - 2 * jj)) >> 31);
        u4 u = __builtin_bit_cast(u4, v[jj]);
        u[0] &= mx;
        u[1] &= mx;
        u[2] &= my;
        u[3] &= my;
        v[jj] = __builtin_bit_cast(d2, u);
    }
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) d_swap32(v[jj], v[jj + 8]);  // lane half H: x[J], x[16 + J], J = jj + 8 H
    {
        constexpr double co[8] = {1.0, 0.98078528040323044913, 0.92387953251128675613, 0.83146961230254523708,
                                  0.70710678118654752440, 0.55557023301960222474, 0.38268343236508977173,
                                  0.19509032201612826785};
        constexpr double si[8] = {0.0, 0.19509032201612826785, 0.38268343236508977173, 0.55557023301960222474,
                                  0.70710678118654752440, 0.83146961230254523708, 0.92387953251128675613,
                                  0.98078528040323044913};
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            const d2 u = v[jj], x16 = v[jj + 8];
            v[jj] = u + x16;
            const d2 wf = d2{co[jj], INV ? si[jj] : -si[jj]};
            const d2 wv = H ? dmi<INV>(wf) : wf;  // w32^(jj + 8) = -+i w32^jj
            v[jj + 8] = dmul(u - x16, wv);
        }
    }
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) d_swap32(v[jj], v[jj + 8]);  // lane half p: sub-sequence p
    d_dft16<INV>(v);                                             // v[q] = X_j[2 q + H]
    __syncthreads();
    d2lds *dst = d_at(33 * j + H);  // c2pos(32 j + 2 q + H) = 33 j + 2 q + H
#pragma unroll
    for (int q = 0; q < 16; ++q) dst[2 * q] = v[q];
    __syncthreads();
}

// Radix-16 Stockham stage with Ns = 2^LNS, one butterfly j = tid per thread (amp_cw2.hip
// c2_stage_r16); Ns = 32: twiddles from the LDS table, Ns = 512: from w1 = w_8192^k, w4 = w_8192^(4 k)
template <bool INV, int LNS>
__device__ __forceinline__ void d_stage_r16(int tid, d2 w1, d2 w4) {
    constexpr int NS = 1 << LNS;
    const int j = tid, k = j & (NS - 1);
    d2 v[16];
    const d2lds *src = d_at(j + (j >> 5));  // c2pos(j + 512 r) = c2pos(j) + 528 r
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = src[528 * r];
    if constexpr (NS == 32) {
        const d2lds *tw = d_at(D_TW1 + k);
#pragma unroll
        for (int r = 1; r < 16; ++r) v[r] = dmul(v[r], tw[32 * (r - 1)]);
    } else {
        static_assert(NS == 512, "second radix-16 stage");
        // w^(4 q + b) applied as w^b then w^(4 q): as many complex multiplies as forming the 15 powers,
        // with 6 of them live instead of 15
        const d2 w2 = dmul(w1, w1), w3 = dmul(w2, w1), w8 = dmul(w4, w4), w12 = dmul(w8, w4);
        const d2 wb[3] = {w1, w2, w3}, wq[3] = {w4, w8, w12};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int b = 1; b < 4; ++b) v[4 * q + b] = dmul(v[4 * q + b], wb[b - 1]);
#pragma unroll
        for (int q = 1; q < 4; ++q)
#pragma unroll
            for (int b = 0; b < 4; ++b) v[4 * q + b] = dmul(v[4 * q + b], wq[q - 1]);
    }
    d_dft16<INV>(v);
    const int bo = ((j - k) << 4) + k;
    __syncthreads();
    d2lds *dst = d_at(bo + (bo >> 5));
#pragma unroll
    for (int r = 0; r < 16; ++r) dst[(NS + NS / 32) * r] = v[r];
    __syncthreads();
}

// Natural-order P-point DFT of the image (element i at c2pos(i)), in place
template <bool INV>
__device__ __forceinline__ void d_fft(int tid, uint32_t msk, const double *twp) {
    // the second radix-16 stage's w_8192^k, w_8192^(4 k), k = tid (512 threads): requested first
    const d2 *tp = reinterpret_cast<const d2 *>(twp);
    d2 w1 = tp[tid], w4 = tp[4 * tid];
    d_stage0_r32<INV>(tid, msk);
    d_stage_r16<INV, 5>(d_opaque(tid), w1, w4);
    if (INV) {
        w1 = dconj(w1);
        w4 = dconj(w4);
    }
    d_stage_r16<INV, 9>(d_opaque(tid), w1, w4);
}

// the first radix-16 stage's table w_512^(r k) = w_8192^(16 (r k mod 512)), r = 1..15, k < 32
template <bool INV>
__device__ __forceinline__ void d_tw1_init(int tid, const double *twp) {
    const d2 *tp = reinterpret_cast<const d2 *>(twp);
    for (int i = tid; i < 15 * 32; i += D_T) {
        const int r = i / 32 + 1, k = i & 31;
        const d2 w = tp[16 * ((r * k) & 511)];
        *d_at(D_TW1 + i) = INV ? dconj(w) : w;
    }
}

__device__ __forceinline__ const int *d_stage_cp(unsigned char *smem, const Cw2dTables &tb, int tid) {
    int *cp = reinterpret_cast<int *>(smem + D_CP_BYTES);
    for (int i = tid; i <= tb.Q; i += D_T) cp[i] = tb.cls_ptr[i];
    return cp;
}

// raw buffer resources (amp_cw2.hip c2_rsrc): out-of-range loads read 0, stores are dropped
__device__ __forceinline__ __amdgpu_buffer_rsrc_t d_rsrc(const void *p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, bytes > 0 ? bytes : 0, 0x00020000);
}
__device__ __forceinline__ double d_ldd(__amdgpu_buffer_rsrc_t r, int vo, int so) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, vo, so, 0));
}
__device__ __forceinline__ d2 d_ld2(__amdgpu_buffer_rsrc_t r, int vo, int so) {
    return __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(r, vo, so, 0));
}
__device__ __forceinline__ void d_std(__amdgpu_buffer_rsrc_t r, double v, int vo, int so) {
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, vo, so, 0);
}
__device__ __forceinline__ int d_uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

// a thread's OT slot words of a thread-major [512][OTP] table, 16 bytes per load
template <int OT>
__device__ __forceinline__ void d_ld_slots(__amdgpu_buffer_rsrc_t r, int tl, uint32_t *out) {
    constexpr int OTP = cw2_otp(OT);
#pragma unroll
    for (int q = 0; q < OTP / 4; ++q) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, 4 * OTP * tl, 16 * q, 0);
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (4 * q + c < OT) out[4 * q + c] = v[c];
    }
}

// x when i < n, else the double whose high word is fill (low word 0), by bit masks: written as a compare
// and a select, the 16 entries' lane masks stayed live in SGPR pairs across the exponentials, were
// spilled to VGPR lanes, and the results moved in the ninth digit (tools/f64_diff.py)
__device__ __forceinline__ double d_keep(double x, int i, int n, uint32_t fill) {
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    const uint32_t mk = (uint32_t)((i - n) >> 31);  // all ones inside
    u2 u = __builtin_bit_cast(u2, x);
    u[0] &= mk;
    u[1] = (u[1] & mk) | (fill & ~mk);
    return __builtin_bit_cast(double, u);
}

// S^e for a uniform exponent e (square and multiply)
__device__ __forceinline__ d2 d_pow(d2 s, int e) {
    d2 w = d2{1.0, 0.0};
    for (; e; e >>= 1) {
        if (e & 1) w = dmul(w, s);
        s = dmul(s, s);
    }
    return w;
}

// x / tau - ms with x / tau as the staged engine's Markstein division (amp_fused.hip sm_arg_st)
__device__ __forceinline__ double d_arg(double v, double ms, double tau, double inv_tau) {
    const double q = v * inv_tau;
    return __builtin_fma(__builtin_fma(-q, tau, v), inv_tau, q) - ms;
}

}  // namespace

// ---------------------------------------------------------------------------- Ab
// beta of the class in class order comes from cw2d_stats (tb.beta): no exponentials and no section
// statistics here
template <int OT>
__global__ __launch_bounds__(D_T, 1) void cw2d_ab(Cw2dTables tb, RegBufs<double> bf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int h = blockIdx.x & 1, cw = blockIdx.x >> 1, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    const double *beta = tb.beta + (size_t)cw * tb.LM;
    const int Qh = tb.Q >> 1, mlo = h * Qh, mhi = mlo + Qh;
    d2 Ha[OT], Hb[OT];
#pragma unroll
    for (int j = 0; j < OT; ++j) Ha[j] = Hb[j] = d2{0.0, 0.0};
    d_tw1_init<false>(tid, tb.twp);
    const int *cpl = d_stage_cp(smem, tb, tid);
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rk = d_rsrc(tb.ka, 4 * OT * D_T), rS = d_rsrc(tb.sa, 16 * OT * D_T);
    // the thread's slot words and S = w_N2^a, slot-major: every load a contiguous run of the wavefront's
    // lanes (thread-major rows of 12 complex doubles put each lane on its own cache lines:
    // profiles/r05_f64_ablation.txt); class-invariant, so requested after each transform and in flight
    // during the loop edge and the next slice's requests
    uint32_t ka[OT];
    d2 S[OT];
    auto acc_tables = [&](int tl) {
#pragma unroll
        for (int j = 0; j < OT; ++j) {
            ka[j] = __builtin_amdgcn_raw_buffer_load_b32(rk, 4 * tl, 4 * j * D_T, 0);
            S[j] = d_ld2(rS, 16 * tl, 16 * j * D_T);
        }
    };
    // Horner step of class m's transform (still in the image) for every owned output
    // (four slots' image reads at a time: all of them in flight beside H, S and the next class's slice
    // spill)
    auto accumulate = [&]() {
#pragma unroll
        for (int j0 = 0; j0 < OT; j0 += 4) {
#pragma unroll
            for (int j = j0; j < j0 + 4 && j < OT; ++j) {
                const int r = (int)(ka[j] & CW_KMASK) & (D_P - 1);
                const d2 ya = *d_at(c2pos(r)), yb = *d_at(c2pos((D_P - r) & (D_P - 1)));
                Ha[j] = dmad(Ha[j], S[j], ya);
                Hb[j] = dmad(Hb[j], S[j], dconj(yb));
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    for (int m2 = mhi - 1; m2 >= mlo; --m2) {
        const int tl = d_opaque(tid);
        const int q0 = d_uni(cpl[m2]), q1 = d_uni(cpl[m2 + 1]);
        const bool prev = m2 < mhi - 1;
        double v[D_SN];
        uint32_t e[D_SN];
        {
            const __amdgpu_buffer_rsrc_t rb = d_rsrc(beta + q0, 8 * (q1 - q0));  // past the class's end: 0
            const __amdgpu_buffer_rsrc_t re = d_rsrc(tb.cls2 + (size_t)m2 * CW2_SLICE, 4 * CW2_SLICE);
#pragma unroll
            for (int i = 0; i < D_SN; ++i) {
                if (D_SKIP(4)) {  // (synthetic entries inside the image, section 0)
                    v[i] = (double)(tl + i);
                    e[i] = (uint32_t)(((tl * 37 + i * 4099) & 8191) * 2);
                    continue;
                }
                v[i] = d_ldd(rb, 8 * tl + 8 * i * D_T, 0);
                e[i] = __builtin_amdgcn_raw_buffer_load_b32(re, 4 * tl, 4 * i * D_T, 0);
            }
        }
        const uint32_t cmk = tb.cmask[m2 * D_T + tl];
        if (prev && !D_SKIP(2)) {
            if (prev) accumulate();
            __syncthreads();  // the image is read before the scatter overwrites it
        }
#pragma unroll
        for (int i = 0; i < D_SN; ++i)  // beta scattered into the image (padded entries: the trash slot)
            if (!D_SKIP(32)) *d_re(e[i] & 0xffffu) = v[i];
        __syncthreads();
        if (!D_SKIP(1)) d_fft<false>(tl, cmk, tb.twp);
        acc_tables(d_opaque(tid));
    }
    accumulate();
    // this half's part of the forward output Re(c1 H[a] + c2 conj H[b]), H = S^mlo (Horner sums)
    const __amdgpu_buffer_rsrc_t rc = d_rsrc(tb.cf, 32 * OT * D_T);
    double *xr = tb.xr + ((size_t)cw * 2 + h) * OT * D_T;
#pragma unroll
    for (int j = 0; j < OT; ++j) {
        d2 ha = Ha[j], hb = Hb[j];
        if (mlo > 0) {
            const d2 w0 = d_pow(S[j], mlo);
            ha = dmul(ha, w0);
            hb = dmul(hb, w0);
        }
        const d2 c1 = d_ld2(rc, 32 * tid, 32 * j * D_T), c2 = d_ld2(rc, 32 * tid, 32 * j * D_T + 16);
        xr[j * D_T + tid] = (c1.x * ha.x - c1.y * ha.y) + (c2.x * hb.x - c2.y * hb.y);
    }
}

// ---------------------------------------------------------------------------- control
__device__ __forceinline__ double d_block_sum(double v, double *red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    return t;
}

// Before Az (sparc.py:931-969), in slot order; the staged engine's reg_ctrl0 at Lc = 1
template <int OT>
__global__ __launch_bounds__(D_T) void cw2d_ctrl(Cw2dTables tb, RegBufs<double> bf, AmpScalars sc, AmpParams pr,
                                                 int t) {
    __shared__ double red[D_T / 64];
    const int cw = blockIdx.x, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    const bool have_beta = t > 0;
    double *psi = sc.psi + cw, *psi_prev = sc.psi_prev + cw;
    double *z = bf.z + (size_t)cw * tb.n;
    const double *y = bf.y + (size_t)cw * tb.n;
    const bool sum_z = pr.phi_method != 1;
    double g, bco = 0.0;
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
        bco = g / ph;
    } else {
        g = pr.W[0];
        if (tid == 0) sc.gamma[cw] = g;
    }
    const double *xr0 = tb.xr + (size_t)cw * 2 * OT * D_T, *xr1 = xr0 + (size_t)OT * D_T;
    double zr[OT];
    double acc = 0.0;
    {
        int oi[OT];
        uint32_t kv[OT];
        double yv[OT], zv[OT], r0[OT], r1[OT];
        double *ys = tb.ys + (size_t)cw * OT * D_T, *zs = tb.zs + (size_t)cw * OT * D_T;
#pragma unroll
        for (int j = 0; j < OT; ++j) {
            oi[j] = tb.oi[j * D_T + tid];
            kv[j] = tb.ka[j * D_T + tid];
        }
        if (have_beta) {
#pragma unroll
            for (int j = 0; j < OT; ++j) {
                yv[j] = ys[j * D_T + tid];
                zv[j] = zs[j * D_T + tid];
                r0[j] = xr0[j * D_T + tid];
                r1[j] = xr1[j * D_T + tid];
            }
#pragma unroll
            for (int j = 0; j < OT; ++j)  // Onsager residual, sparc.py:943-946
                zr[j] = (yv[j] - (r0[j] + r1[j])) + bco * zv[j];
        } else {
#pragma unroll
            for (int j = 0; j < OT; ++j) yv[j] = y[oi[j]];
#pragma unroll
            for (int j = 0; j < OT; ++j) {
                ys[j * D_T + tid] = yv[j];
                zr[j] = yv[j];
            }
        }
#pragma unroll
        for (int j = 0; j < OT; ++j) {
            zs[j * D_T + tid] = zr[j];
            if (kv[j] & CW_VALID) {
                z[oi[j]] = zr[j];  // natural order: the staged engine's after a hand-over
                if (sum_z) acc += zr[j] * zr[j];
            }
        }
    }
    double phi;
    if (sum_z) {
        phi = d_block_sum(acc, red) / (double)tb.n;  // sparc.py:949-955
    } else {
        phi = pr.awgn_var + g;
    }
    const double tv_new = (tb.L * phi / tb.n) / pr.W[0];  // sparc.py:958-969
    if (tid == 0) {
        bf.phi[cw] = phi;
        bf.tau[cw] = tv_new;
    }
    double *vz = tb.vz + (size_t)cw * OT * D_T;  // slot-major
#pragma unroll
    for (int j = 0; j < OT; ++j) vz[j * D_T + tid] = zr[j] / phi;  // z / phi (sparc.py:972)
}

// ---------------------------------------------------------------------------- Az
// rows -> inverse transform -> s = beta_prev + tau u, stored in class order; the section statistics are
// cw2d_stats' (a separate launch at full occupancy: inside this one-workgroup-per-CU kernel they took
// half its time, profiles/r05_f64_ablation.txt)
template <int OT>
__global__ __launch_bounds__(D_T, 1) void cw2d_az(Cw2dTables tb, RegBufs<double> bf, int t) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int h = blockIdx.x & 1, cw = blockIdx.x >> 1, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    const bool have_beta = t > 0;
    const double tau = bf.tau[cw];
    double *s = bf.s + (size_t)cw * tb.LM;
    const double *beta = tb.beta + (size_t)cw * tb.LM;
    const double *vz = tb.vz + (size_t)cw * OT * D_T;
    const int Qh = tb.Q >> 1, mlo = h * Qh, mhi = mlo + Qh;
    const __amdgpu_buffer_rsrc_t rS = d_rsrc(tb.sa, 16 * OT * D_T);
    d2 W[OT];  // w_N2^(m a) of the class, rotated by S = w_N2^a per class
#pragma unroll
    for (int j = 0; j < OT; ++j) W[j] = d_pow(d_ld2(rS, 16 * tid, 16 * j * D_T), mlo);
    d_tw1_init<true>(tid, tb.twp);
    const int *cpl = d_stage_cp(smem, tb, tid);
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rv = d_rsrc(vz, 8 * OT * D_T), rk = d_rsrc(tb.ka, 4 * OT * D_T),
                                 rg = d_rsrc(tb.gf, 32 * OT * D_T);
    // the rows' slot words, z / phi and S are class-invariant: requested at the end of the previous class
    uint32_t kall[OT];
    double vall[OT];
    d2 S[OT];
    auto rows_tables = [&](int tl) {
#pragma unroll
        for (int j = 0; j < OT; ++j) {
            kall[j] = __builtin_amdgcn_raw_buffer_load_b32(rk, 4 * tl, 4 * j * D_T, 0);
            vall[j] = d_ldd(rv, 8 * tl, 8 * j * D_T);
            S[j] = d_ld2(rS, 16 * tl, 16 * j * D_T);
        }
    };
    if (D_AZPF) rows_tables(tid);
    for (int m2 = mlo; m2 < mhi; ++m2) {
        const int tl = d_opaque(tid);
        const uint32_t rmk = tb.cmask[tb.Q * D_T + tl];
        const int q0 = d_uni(cpl[m2]), q1 = d_uni(cpl[m2 + 1]);
        if (!D_SKIP(128)) {
            if (!D_AZPF) rows_tables(tl);
            // rows r and P - r of each owned pair: sums of al v conj(W) / be v W over its outputs (v = z / phi),
            // branch-free as amp_cw2.hip's rows (NEWROW restarts the sums; both rows written on the pair's last
            // slot, the trash slot otherwise; r = 0, P / 2: the sum at row r)
            constexpr int CH = 4;  // slots per round of coefficient loads
            d2 u0{0.0, 0.0}, u1{0.0, 0.0};
#pragma unroll
            for (int j0 = 0; j0 < OT; j0 += CH) {
                d2 al[CH], be[CH];
#pragma unroll
                for (int i = 0; i < CH; ++i) {
                    if (j0 + i >= OT) break;
                    al[i] = d_ld2(rg, 32 * tl, 32 * (j0 + i) * D_T);
                    be[i] = d_ld2(rg, 32 * tl, 32 * (j0 + i) * D_T + 16);
                }
#pragma unroll
                for (int i = 0; i < CH; ++i) {
                    const int j = j0 + i;
                    if (j >= OT) break;
                    const uint32_t k = kall[j];
                    const double keep = (k & CW_NEWROW) ? 0.0 : 1.0, vv = vall[j];
                    u0 = dmad(d2{al[i].x * vv, al[i].y * vv}, dconj(W[j]), u0 * keep);
                    u1 = dmad(d2{be[i].x * vv, be[i].y * vv}, W[j], u1 * keep);
                    const int r = (int)(k & (uint32_t)(D_P - 1)), rb = D_P - r;
                    const bool end = (k & CW_ENDROW) != 0, self = (k & CW_SELF) != 0;
                    d2lds *pa = d_at(end ? c2pos(r) : D_TRASH), *pb = d_at((end && !self) ? c2pos(rb) : D_TRASH);
                    *pa = u0;
                    *pb = u1;
                    if (self) *pa = u0 + u1;
                    W[j] = dmul(W[j], S[j]);  // the next class
                }
            }
        }
        // the class slice (image positions, beta_prev), in flight during the transform
        double v[D_SN];
        uint32_t e[D_SN];
        {
            const __amdgpu_buffer_rsrc_t rb = d_rsrc(beta + q0, 8 * (q1 - q0));
            const __amdgpu_buffer_rsrc_t re = d_rsrc(tb.cls2 + (size_t)m2 * CW2_SLICE, 4 * CW2_SLICE);
#pragma unroll
            for (int i = 0; i < D_SN; ++i) {
                if (D_SKIP(256)) {
                    v[i] = (double)(tl + i);
                    e[i] = (uint32_t)(((tl * 37 + i * 4099) & 8191) * 2);
                    continue;
                }
                e[i] = __builtin_amdgcn_raw_buffer_load_b32(re, 4 * tl, 4 * i * D_T, 0);
                v[i] = have_beta ? d_ldd(rb, 8 * tl + 8 * i * D_T, 0) : 0.0;
            }
        }
        __syncthreads();
        if (!D_SKIP(64)) d_fft<true>(tl, rmk, tb.twp);
        {
            const __amdgpu_buffer_rsrc_t rs = d_rsrc(s + q0, 8 * (q1 - q0));  // past the class's end: dropped
#pragma unroll
            for (int i = 0; i < D_SN; ++i) {  // s = beta_prev + tau u (sparc.py:972), class order
                const double sv = v[i] + tau * *d_re(e[i] & 0xffffu);
                if (!D_SKIP(1024)) d_std(rs, sv, 8 * tl + 8 * i * D_T, 0);
            }
        }
        if (D_AZPF && m2 + 1 < mhi) rows_tables(tl);
        __syncthreads();  // the next class overwrites the image
    }
}

// ---------------------------------------------------------------------------- statistics
// After Az: per section, the softmax of s over its M entries (sparc.py:429-432, the staged engine's
// argument x / tau - max / tau), its statistics and beta itself (class order, tb.beta: the next Ab's
// input and the next Az's beta_prev), the previous beta's section max and 1 / sum for a hand-over
// (stM, stI) and the section's sum beta^2 and squared error (sparc.py:973-981) for cw2d_final.
// One wavefront per section (a segment of it per class: a contiguous run of s in class order, about
// LM / (Q L) = 8 entries; Q <= 64, M <= 512): every entry read once from HBM, one exponential per
// entry, sums in a fixed order (per lane, then a xor-shuffle tree).
// the class of each entry from a per-section owner table each class's lane fills (1), or a binary search
// over the classes' prefix sums per entry (0) (A/B)
#ifndef D_ST_OWNER
#define D_ST_OWNER 1
#endif
// sections per workgroup (one wavefront each): the widest of 16, 8, 4 that divides L, at most D_ST_MAXW.  A
// workgroup's sections are consecutive, so its wavefronts read and write neighbouring segments of every
// class -- neighbouring cache lines -- together.  Same box, f64 iteration (ms): 4 sections 2.392, 8 2.310,
// 16 2.198 (2: 2.493), decisions bit-identical (profiles/r05_f64_ablation.txt)
#ifndef D_ST_MAXW
#define D_ST_MAXW 16
#endif
constexpr int ST_WAVES_MIN = 4;
constexpr int ST_K = 8;      // entries per lane: sections of M <= 512 entries
__device__ __forceinline__ double d_wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ double d_wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
template <int ST_WAVES>
__global__ __launch_bounds__(64 * ST_WAVES) void cw2d_stats(Cw2dTables tb, RegBufs<double> bf) {
    // per wavefront: exclusive prefix of the segment lengths over the classes, and each segment's base
    // (class-order position minus that prefix): entry k of the section lives at base[m] + k, m the last
    // class with prefix[m] <= k
    __shared__ int pre[ST_WAVES][64], bas[ST_WAVES][64];
#if D_ST_OWNER
    __shared__ uint8_t own[ST_WAVES][64 * ST_K];  // the class of each entry of the section
#endif
    const int wpc = tb.L / ST_WAVES;  // workgroups per codeword
    const int w = (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int cw = blockIdx.x / wpc, l = (blockIdx.x % wpc) * ST_WAVES + w;
    if (!bf.active[cw]) return;
    const size_t lb = (size_t)cw * tb.L;
    const double tau = bf.tau[cw], inv_tau = 1.0 / tau;
    const double *s = bf.s + (size_t)cw * tb.LM;
    double *beta = tb.beta + (size_t)cw * tb.LM;
    int p0 = 0, n = 0;
    if (lane < tb.Q) {
        const uint16_t *sg = tb.seg + (size_t)lane * (tb.Lblk + 1);
        p0 = tb.cls_ptr[lane] + sg[l];
        n = sg[l + 1] - sg[l];
    }
    int inc = n;  // inclusive scan over the lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
    }
    const int total = __shfl(inc, 63, 64);  // the section's entries (M)
    pre[w][lane] = inc - n;
    bas[w][lane] = p0 - (inc - n);
#if D_ST_OWNER
    for (int k = inc - n; k < inc; ++k) own[w][k] = (uint8_t)lane;  // each class marks its segment's entries
#endif
    __syncthreads();
    // the section's entries k = lane + 64 j in concatenated class order: consecutive lanes read consecutive
    // positions of a segment (coalesced runs), no padding, one exponential per entry
#if !D_ST_OWNER
    const int nq = tb.Q;
#endif
    int ad[ST_K];
    double x[ST_K];
#pragma unroll
    for (int j = 0; j < ST_K; ++j) {
        const int k = lane + 64 * j;
        const bool in = k < total;
#if D_ST_OWNER
        const int lo = in ? (int)own[w][k] : 0;  // (one LDS read instead of a six-step search)
#else
        int lo = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1)  // last class with pre <= k (empty classes: same pre)
            if (lo + step < nq && pre[w][lo + step] <= k) lo += step;
#endif
        ad[j] = in ? bas[w][lo] + k : 0;
        x[j] = d_keep(s[ad[j]], k, total, 0xfff00000u);  // past the section: -inf
    }
    double m = x[0];
#pragma unroll
    for (int j = 1; j < ST_K; ++j) m = fmax(m, x[j]);
    const double M = d_wave_max(m);
    const double ms = M / tau;  // (amp_fused.hip sm_stage)
    double S1 = 0.0, S2 = 0.0;
#pragma unroll
    for (int j = 0; j < ST_K; ++j) {  // past the section: 0 (the Markstein quotient of -inf is NaN)
        x[j] = d_keep(exp(d_arg(x[j], ms, tau, inv_tau)), lane + 64 * j, total, 0u);
        S1 += x[j];
        S2 = __builtin_fma(x[j], x[j], S2);
    }
    S1 = d_wave_sum(S1);
    S2 = d_wave_sum(S2);
    const double inv = 1.0 / S1;
#pragma unroll
    for (int j = 0; j < ST_K; ++j)
        if (lane + 64 * j < total) beta[ad[j]] = x[j] * inv;
    if (lane == 0) {
        bf.stM[lb + l] = M;
        bf.stI[lb + l] = inv;
        const double ss = S2 * inv * inv;
        double err = ss;
        if (bf.true_idx) {
            const double st = s[tb.qpos[l * tb.M + bf.true_idx[lb + l]]];
            err = ss - 2.0 * (exp(d_arg(st, ms, tau, inv_tau)) * inv) + 1.0;  // as the entries (and sm_arg)
        }
        tb.sec[(lb + l) * 2] = ss;
        tb.sec[(lb + l) * 2 + 1] = err;
    }
}

// psi, NMSE and the stopping rule from the sections' sums (sparc.py:973-988), fixed summation order
__global__ __launch_bounds__(1024) void cw2d_final(Cw2dTables tb, RegBufs<double> bf, AmpScalars sc, AmpParams pr,
                                                   int t) {
    __shared__ double red[16];
    const int cw = blockIdx.x, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    const size_t lb = (size_t)cw * tb.L;
    double a = 0.0, er = 0.0;
    for (int l = tid; l < tb.L; l += 1024) {
        a += tb.sec[(lb + l) * 2];
        er += tb.sec[(lb + l) * 2 + 1];
    }
    a = d_block_sum(a, red);
    er = d_block_sum(er, red);
    if (tid == 0) {
        double *psi = sc.psi + cw, *psi_prev = sc.psi_prev + cw;
        double *nmse = sc.nmse + (size_t)cw * pr.t_max;
        const double denom = (double)tb.L;
        const double pnew = 1.0 - a / denom;
        *psi = pnew;
        nmse[t + 1] = er / denom;
        bool stop = false;
        if (t > 0 && D_ABL == 0) {  // (ablation builds never stop early: every launch does the same work)
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
}

template <int OT>
static int cw2d_launch(const Cw2dTables &tb, const RegBufs<double> &bf, const AmpScalars &sc, const AmpParams &pr,
                       int t, hipStream_t s) {
    static const int ready = []() -> int {  // the LDS addresses assume no static LDS (d_at)
        hipFuncAttributes fa, fz;
        if (hipFuncGetAttributes(&fa, (const void *)cw2d_ab<OT>) != hipSuccess ||
            hipFuncGetAttributes(&fz, (const void *)cw2d_az<OT>) != hipSuccess || fa.sharedSizeBytes ||
            fz.sharedSizeBytes)
            return 0;
        return hipFuncSetAttribute((const void *)cw2d_ab<OT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   D_LDS_BYTES) == hipSuccess &&
               hipFuncSetAttribute((const void *)cw2d_az<OT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   D_LDS_BYTES) == hipSuccess;
    }();
    if (!ready) return fail(SG_ERR_HIP, "f64 split engine: kernel attributes (static LDS / LDS size)");
    const dim3 g2(2 * bf.B), gB(bf.B);
    if (t > 0) {
        ProfScope ps(SG_PH_CW2_AB, s);
        hipLaunchKernelGGL((cw2d_ab<OT>), g2, dim3(D_T), D_LDS_BYTES, s, tb, bf);
    }
    {
        ProfScope ps(SG_PH_CW2_CTRL, s);
        hipLaunchKernelGGL((cw2d_ctrl<OT>), gB, dim3(D_T), 0, s, tb, bf, sc, pr, t);
    }
    {
        ProfScope ps(SG_PH_CW2_AZ, s);
        hipLaunchKernelGGL((cw2d_az<OT>), g2, dim3(D_T), D_LDS_BYTES, s, tb, bf, t);
    }
    {
        ProfScope ps(SG_PH_CW2_CTRL, s);
        if (D_ST_MAXW >= 16 && tb.L % 16 == 0)
            hipLaunchKernelGGL((cw2d_stats<16>), dim3(bf.B * (tb.L / 16)), dim3(64 * 16), 0, s, tb, bf);
        else if (D_ST_MAXW >= 8 && tb.L % 8 == 0)
            hipLaunchKernelGGL((cw2d_stats<8>), dim3(bf.B * (tb.L / 8)), dim3(64 * 8), 0, s, tb, bf);
        else
            hipLaunchKernelGGL((cw2d_stats<4>), dim3(bf.B * (tb.L / 4)), dim3(64 * 4), 0, s, tb, bf);
        hipLaunchKernelGGL((cw2d_final), gB, dim3(1024), 0, s, tb, bf, sc, pr, t);
    }
    return SG_OK;
}

int cw2d_launch_iter(const Cw2dTables &tb, const RegBufs<double> &bf, const AmpScalars &sc, const AmpParams &pr,
                     int t, hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    static_assert(D_P == 8192 && ST_WAVES_MIN == 4 && 64 * ST_K == 512, "cw2d_supported (amp.hpp) states these");
    if (!cw2d_supported(tb)) return fail(SG_ERR_UNSUPPORTED, "f64 split engine: sizes outside its compile-time bounds");
    ProfScope ps(SG_PH_AMP_CW, s);
    switch (tb.OT) {
    case 12: SG_TRY(cw2d_launch<12>(tb, bf, sc, pr, t, s)); break;
    case 13: SG_TRY(cw2d_launch<13>(tb, bf, sc, pr, t, s)); break;
    case 14: SG_TRY(cw2d_launch<14>(tb, bf, sc, pr, t, s)); break;
    case 16: SG_TRY(cw2d_launch<16>(tb, bf, sc, pr, t, s)); break;
    default: return fail(SG_ERR_UNSUPPORTED, "f64 split engine: %d outputs per thread", tb.OT);
    }
    SG_HIP(hipGetLastError());
    return SG_OK;
}

}  // namespace sg
