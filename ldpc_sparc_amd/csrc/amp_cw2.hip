// Split per-codeword AMP engine on gfx950 (the C2 headline path).  One AMP
// iteration of the regular design (sparc.py:883-999 with the sub-sampled DCT
// operators of sub_dct, sparc.py:648-701) per codeword as four launches:
//
//   cw2_ab    (2 B workgroups)  half h of the Q classes: beta of the class
//             (from s and the section statistics) -> LDS scatter -> P-point
//             FFT -> for every output i owned by the thread:
//                 H[a]      += W Y_m2[r],
//                 conj H[b] += W conj Y_m2[P - r],   W = w_N2^(m2 a), r = a mod P
//             in registers; each half's part of Re(c1 H[a] + c2 conj H[b])
//             goes to xr.
//   cw2_ctrl  (B)  z = y - (sum of the halves' parts) + b z, phi, tau
//             (sparc.py:931-969); z / phi in slot order (vz).
//   cw2_az    (2 B)  half h of the classes: rows r and P - r of each owned
//             conjugate pair from the outputs' al z/phi conj(W) and be z/phi W
//             -> inverse P-point FFT -> s = beta_prev + tau u (sparc.py:972) in
//             class order -> per-section partial (max, sums without the max).
//   cw2_merge (B)  the two halves' section statistics -> max, 1/sum, psi,
//             NMSE, early stop (sparc.py:973-988).
//
// Why split: with one 1024-thread workgroup per CU (amp_cw.hip) every phase of
// a class is separated by workgroup barriers and nothing overlaps them (SQ:
// ~42 % of wave cycles waiting).  Here each codeword's classes are shared by
// two 512-thread workgroups with 64 KB of LDS each, two per CU, so one
// workgroup's barriers, LDS latency and global loads run beside the other's
// transform.  The needed spectrum no longer lives in LDS: the forward output
// Re(c1 H[a] + c2 conj H[N2 - a]) and the inverse input of output i touch
// only the conjugate row pair {a mod P, P - a mod P} of the P-point stage, so
// a thread that owns whole pairs accumulates H[a] and conj H[b] of its
// outputs in registers (one twiddle per output and class, no X slots in LDS,
// no read-modify-write), and writes the pair's rows without conflicts.
//
// The P-point transform (P = 8192) runs at 16 values per thread in three
// LDS passes: radix 32 (each butterfly shared by lanes l and l ^ 32 through
// v_permlane32_swap, no twiddles), then radix 16 twice with twiddles from the
// hardware sine / cosine.
#include "amp.hpp"

namespace sg {
namespace {

constexpr int C2_T = CW2_THREADS;
constexpr int C2_LOG2P = 13, C2_P = 1 << C2_LOG2P, C2_EPT = C2_P / C2_T;  // 16 values per thread
constexpr int C2_SC = 9;   // class entries per thread and chunk
constexpr int C2_NC = 2;   // chunks: a class holds at most C2_SC * C2_NC * 512 = 9216 entries
static_assert(C2_EPT == 16, "the transform is written for 16 values per thread");

// Phase ablation for timing studies only (tools/c2_ablate.py on variants built by
// tools/mk_variant.sh with -DC2_ABL=<mask>; results are garbage, the shipped build has 0):
// 1 Ab FFT, 2 Ab accumulation, 4 Ab slice loads, 8 Az FFT, 16 Az rows, 32 Az rows' table
// loads (values from the thread index), 64 Az statistics + class copy, 128 Az slice loads, 256 Ab scatter,
// 512 Ab beta stores, 1024 Az gathers from the image
#ifndef C2_ABL
#define C2_ABL 0
#endif
#define C2_SKIP(bit) ((C2_ABL & (bit)) != 0)

// Az rows: the row addresses from the slot's flags instead of the host table wab (A/B)
#ifndef C2_ROWS_DERIVE
#define C2_ROWS_DERIVE 1
#endif
// Az rows in the polar form (build_cw2): one phase per slot and class from the slot word, z/phi scaled by
// (|al|, |be|) -- no per-slot complex coefficient table (gf) re-read every class (1), or that table (0) (A/B)
#ifndef C2_POLAR
#define C2_POLAR 1
#endif
// Az: the gathers' image positions from the packed 16-bit table clsp (1) or the full class words cls2 (0) (A/B)
#ifndef C2_AZPOS
#define C2_AZPOS 1
#endif
// Wave issue priority during the transforms and outside them.  Two workgroups share a CU and alternate
// between the transform (VALU and LDS throughput) and phases that are chains of memory round trips and
// barriers (class loads, rows, gathers, statistics).  At equal priority the older wave wins each issue
// slot, so a workgroup's chain waited behind the other's transform; with the chains at 1 over the
// transforms at 0 the transform fills the chains' gaps instead: cw2_az 0.531 -> 0.501, cw2_ab 0.382 ->
// 0.378 ms per launch, C2 probe 11.77 k -> 12.29 k codewords/s same box, identical results (priority 2 or
// 3 for the chains, 2 for the statistics alone, or Az alone measured the same or less, and the gain is the
// class-start phase's: with it at 0 and the rest at 1 the iteration is slower than flat;
// profiles/r05_prio_ab.txt).  Both 0: flat, for the A/B.
#ifndef C2_PRIO_FFT
#define C2_PRIO_FFT 0
#endif
#ifndef C2_PRIO_REST
#define C2_PRIO_REST 1
#endif
#define C2_SETPRIO(p)                                                       \
    do {                                                                    \
        if (C2_PRIO_FFT != 0 || C2_PRIO_REST != 0) __builtin_amdgcn_s_setprio(p); \
    } while (0)
// Ab: the accumulation's slot words requested after each transform (1) or at the class start (0) (A/B)
#ifndef C2_AB_PF
#define C2_AB_PF 1
#endif

// Section statistics: in cw2_az (class copy and two-pass scan per class, merged over the classes, then
// cw2_merge: 0), or in their own full-occupancy launch after cw2_az (cw2_stats: one wavefront per section
// reading its class segments of s from HBM, then cw2_final: 1), the f64 engine's form (amp_cw2d.hip) (A/B)
#ifndef C2_STATS_LAUNCH
#define C2_STATS_LAUNCH 0
#endif
// Az rows: every slot writes its pair's running sums at the pair's rows, addresses and factors from the slot
// word without compares (1), or the last slot of a pair writes them, other slots write the trash slot (0) (A/B)
#ifndef C2_ROWS_ALWAYS
#define C2_ROWS_ALWAYS 1
#endif
// Polar rows' per-codeword input: z / phi alone, 4 bytes per slot, scaled in cw2_az by (|al|, |be|) from the
// plan's thread-major table (shared by every codeword: L2-resident) (1), or the scaled pair stored by cw2_ctrl,
// 8 bytes per slot re-read from the MALL in every class (0) (A/B; at most 12 slots per thread).  With the two
// switches below, same box: fabric bytes 11.35 -> 9.69 MB per codeword-iteration (cw2_az 6.97 -> 5.34), C2
// +0.4 % (profiles/r06_c2_vz_half_ab.txt)
#ifndef C2_VZ_HALF
#define C2_VZ_HALF 1
#endif
// Az statistics: the segment mask from a per-section bit mask, v_bfe + v_bfi per entry (1), or the sign-mask form
// (0), which the compiler turns into v_cmp + v_cndmask through an SGPR pair with a hazard s_nop per entry (A/B);
// bit-identical results.  (Pairing (x - max) / tau into v_pk_add / v_pk_mul halves their count but not their
// issue cycles: a packed f32 instruction issues in 4 cycles, a plain one in 2 -- MI355X_MICROARCH.md.)
#ifndef C2_ST_BITS
#define C2_ST_BITS 1
#endif
// Az statistics: segment entries read per lane in the first round, the rest in rounds of as many until the
// wavefront's longest segment is done (segments average LM / (Q L) = 8 entries).  The entries are summed in
// segment order whatever the round size, so every choice gives bit-identical statistics.  Three calls of three
// interleaved rounds (profiles/r06_c2_stats_rounds_ab.txt): 12 is 2 % slower than 16 (the round-5 form, one
// round covering nearly every segment), 2 to 8 are faster; 4: 0.840 -> 0.830 ms per iteration, C2 +1.2 % (default)
#ifndef C2_RC
#define C2_RC 4
#endif
// Az statistics: every round of reads in the two loops, none held in registers across the maximum (1), or a
// first round read once for both passes (0) (A/B; bit-identical).  Two same-box calls of three rounds: +0.4 %,
// +0.2 % (profiles/r06_c2_stats_rounds_ab.txt); the two sections' rounds interleaved in one pair of loops
// measured 2 % slower
#ifndef C2_NOFIRST
#define C2_NOFIRST 1
#endif
// workgroups per codeword: tb.np (amp.hpp CW2_NP: at most 8, the largest of 8, 4, 2 dividing Q)
// Az rows' per-codeword class-invariant input (a thread's scaled z / phi, 24 VGPRs at 12 slots) loaded once per
// launch and held in registers across the class loop (1; with the statistics launch cw2_az has the registers),
// or re-read from L2 / MALL every class (0) (A/B); the slot words are the plan's, shared by every codeword
#ifndef C2_AZ_HOLD
#define C2_AZ_HOLD 0
#endif

// exp(x / tau) as exp2(x * (log2 e / tau)): __expf lowers to a multiply by log2 e and v_exp_f32, so
// with log2 e folded into the per-codeword scale every exponential is one instruction
constexpr double C2_LOG2E = 1.4426950408889634074;
__device__ __forceinline__ float c2_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ int c2_opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// the first transform stage's stale-value masks as v_bfe_i32 + v_and (1), or as the compiler's own
// compare + select (0) (A/B)
#ifndef C2_MASK_BFE
#define C2_MASK_BFE 1
#endif

// w_N2^j = exp(-2 pi i j / N2) from the hardware sine / cosine (revolutions;
// (j mod N2) / N2 is exact in f32 for N2 <= 2^19)
__device__ __forceinline__ cx<float> c2_w(const Cw2Tables &tb, uint32_t j) {
    const float x = (float)(j & (uint32_t)(tb.N2 - 1)) * tb.inv_n2;
    return {__builtin_amdgcn_cosf(x), -__builtin_amdgcn_sinf(x)};
}

// ---- the P-point transform -------------------------------------------------
// Complex values as two-float vectors, so the packed f32 instructions
// (v_pk_add / v_pk_mul / v_pk_fma, with their operand swizzles and negations
// as op_sel / neg modifiers) work on register pairs that stay paired: written
// with a {x, y} struct, the compiler spent ~150 moves per transform re-pairing
// them.  The image is addressed through LDS pointers built from complex
// indices (the kernels have no static LDS, so the dynamic image starts at
// address 0): every access of a stage is a per-thread base plus a constant,
// folded into the instruction's offset.
typedef float c2f __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) c2f c2lds;
__device__ __forceinline__ c2lds *c2_at(int pos) { return (c2lds *)(size_t)(8u * (uint32_t)pos); }
// complex index of the first radix-16 stage's twiddle table (after the image,
// the staged statistics and the trash slot): w_512^(r k) at (r - 1) 32 + k,
// r = 1..15, k < 32, forward or (cw2_az) inverse
constexpr int C2_TW1 = ((8192 + 256) * 8 + 2 * 1024 * 4 + 16) / 8;
template <bool INV>
__device__ __forceinline__ void c2_tw1_init(int tid) {
    for (int i = tid; i < 15 * 32; i += C2_T) {
        const int r = i / 32 + 1, k = i & 31;
        const float x = (float)((r * k) & 511) * (1.0f / 512.0f);
        const float sn = __builtin_amdgcn_sinf(x);
        *c2_at(C2_TW1 + i) = c2f{__builtin_amdgcn_cosf(x), INV ? sn : -sn};
    }
}

// The packed instructions' modifiers negate whole operands, and the compiler
// does not fold a one-lane negation into them (it spends a xor and a move on
// each {-y, x} pair), so every sign pattern is a constant pair: one packed
// multiply or FMA by (1, -1) / (-1, 1).
__device__ __forceinline__ c2f c2_pm() { return c2f{1.f, -1.f}; }
__device__ __forceinline__ c2f c2_mp() { return c2f{-1.f, 1.f}; }
template <bool INV>
__device__ __forceinline__ c2f c2_mi(c2f a) {  // * -i (forward), * +i (inverse)
    return a.yx * (INV ? c2_mp() : c2_pm());
}
// x + (* -i or * +i)(d) in one packed FMA
template <bool INV>
__device__ __forceinline__ c2f c2_addmi(c2f x, c2f d) {
    return __builtin_elementwise_fma(d.yx, INV ? c2_mp() : c2_pm(), x);
}
template <bool INV>
__device__ __forceinline__ c2f c2_submi(c2f x, c2f d) {
    return __builtin_elementwise_fma(d.yx, INV ? c2_pm() : c2_mp(), x);
}
__device__ __forceinline__ c2f c2_mul(c2f a, c2f w) {  // three packed instructions
    return __builtin_elementwise_fma(a.yy * w.yx, c2_mp(), a.xx * w);
}

template <bool INV>
__device__ __forceinline__ void c2_dft4(c2f &a0, c2f &a1, c2f &a2, c2f &a3) {
    const c2f t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, d = a1 - a3;
    a0 = t0 + t2;
    a2 = t0 - t2;
    a1 = c2_addmi<INV>(t1, d);
    a3 = c2_submi<INV>(t1, d);
}

// 16-point DFT as 4 x 4 (fft.hpp dft16: inputs n = 4 n1 + n2, outputs k = k1 + 4 k2)
template <bool INV>
__device__ __forceinline__ void c2_dft16(c2f *a) {
    const float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f, r2 = 0.70710678118654752440f;
    c2f y[4][4];
#pragma unroll
    for (int n2 = 0; n2 < 4; ++n2) {
        c2f v0 = a[n2], v1 = a[n2 + 4], v2 = a[n2 + 8], v3 = a[n2 + 12];
        c2_dft4<INV>(v0, v1, v2, v3);
        y[n2][0] = v0;
        y[n2][1] = v1;
        y[n2][2] = v2;
        y[n2][3] = v3;
    }
    // y[n2][k1] *= w16^(n2 k1): x (c - i s) forward, x (c + i s) inverse
    auto tw = [&](c2f x, float c, float s) -> c2f {
        return __builtin_elementwise_fma(x.yx, INV ? c2f{-s, s} : c2f{s, -s}, x * c2f{c, c});
    };
    y[1][1] = tw(y[1][1], c1, s1);
    y[1][2] = tw(y[1][2], r2, r2);
    y[1][3] = tw(y[1][3], s1, c1);
    y[2][1] = tw(y[2][1], r2, r2);
    y[2][2] = c2_mi<INV>(y[2][2]);
    y[2][3] = tw(y[2][3], -r2, r2);
    y[3][1] = tw(y[3][1], s1, c1);
    y[3][2] = tw(y[3][2], -r2, r2);
    y[3][3] = tw(y[3][3], -c1, -s1);
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
        c2f v0 = y[0][k1], v1 = y[1][k1], v2 = y[2][k1], v3 = y[3][k1];
        c2_dft4<INV>(v0, v1, v2, v3);
        a[k1] = v0;
        a[k1 + 4] = v1;
        a[k1 + 8] = v2;
        a[k1 + 12] = v3;
    }
}

// lanes 32..63 of a <-> lanes 0..31 of b (v_permlane32_swap, no LDS)
__device__ __forceinline__ void c2_swap32(c2f &a, c2f &b) {
    const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
    const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
    a = c2f{__uint_as_float(rx[0]), __uint_as_float(ry[0])};
    b = c2f{__uint_as_float(rx[1]), __uint_as_float(ry[1])};
}

// First Stockham stage at radix 32 (Ns = 1, no twiddles), 16 values per
// thread: butterfly j = 32 w + (l & 31) of wavefront w is shared by lanes l
// and l ^ 32, lane half H holding inputs m = 16 H + jj (x[j + 256 m]).  Two
// rounds of permlane32 swaps around a radix-2 decimation-in-frequency step
// (half H then holds x[J], x[J + 16] for J = jj + 8 H; a_J = x_J + x_(J+16),
// b_J = (x_J - x_(J+16)) w32^J) give half p the 16 values of sub-sequence p,
// whose 16-point DFT in registers is X[2 q + p]; stored at j 32 + 2 q + H.
// The image is not zeroed before a scatter / the row writes: bit 2 jj + c of
// msk says whether component c of value jj was written for this transform
// (host table, build_cw2), the stale ones read as zero.
template <bool INV>
__device__ __forceinline__ void c2_stage0_r32(int tid, uint32_t msk) {
    const int l = tid & 63, H = l >> 5, w = tid >> 6, j = (w << 5) | (l & 31);
    c2f v[16];
    const c2lds *src = c2_at(j + w + 264 * 16 * H);  // c2pos(j + 256 m) = j + w + 264 m
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) v[jj] = src[264 * jj];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {  // all-ones / zero from the sign-extended bit (v_bfe_i32)
        int mx = __builtin_amdgcn_sbfe((int)msk, 2 * jj, 1), my = __builtin_amdgcn_sbfe((int)msk, 2 * jj + 1, 1);
#if C2_MASK_BFE
        // (opaque: otherwise the compiler turns bit-extract-and-AND back into a compare and a select per
        // component, serialised on VCC with hazard nops -- 3 VALU and a nop instead of 2 VALU)
        asm volatile("" : "+v"(mx), "+v"(my));
#endif
        v[jj] = c2f{__uint_as_float(__float_as_uint(v[jj].x) & (uint32_t)mx),
                    __uint_as_float(__float_as_uint(v[jj].y) & (uint32_t)my)};
    }
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) c2_swap32(v[jj], v[jj + 8]);  // lane half H: x[J], x[16 + J], J = jj + 8 H
    {
        // w32^J = cos(2 pi J / 32) -+ i sin(2 pi J / 32) for J = jj + 8 H (forward -, inverse +);
        // w32^(jj + 8) = -i w32^jj
        constexpr float co[8] = {1.f, 0.98078528040323044913f, 0.92387953251128675613f, 0.83146961230254523708f,
                                 0.70710678118654752440f, 0.55557023301960222474f, 0.38268343236508977173f,
                                 0.19509032201612826785f};
        constexpr float si[8] = {0.f, 0.19509032201612826785f, 0.38268343236508977173f, 0.55557023301960222474f,
                                 0.70710678118654752440f, 0.83146961230254523708f, 0.92387953251128675613f,
                                 0.98078528040323044913f};
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            const c2f u = v[jj], x16 = v[jj + 8];
            v[jj] = u + x16;
            const c2f wf = c2f{co[jj], INV ? si[jj] : -si[jj]};
            const c2f w = H ? c2_mi<INV>(wf) : wf;
            v[jj + 8] = c2_mul(u - x16, w);  // (jj = 0: w = 1 or -+i, exact)
        }
    }
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) c2_swap32(v[jj], v[jj + 8]);  // lane half p: sub-sequence p, J = 0..15
    c2_dft16<INV>(v);                                            // v[q] = X_j[2 q + H]
    __syncthreads();
    c2lds *dst = c2_at(33 * j + H);  // c2pos(32 j + 2 q + H) = 33 j + 2 q + H
#pragma unroll
    for (int q = 0; q < 16; ++q) dst[2 * q] = v[q];
    __syncthreads();
}

// Radix-16 Stockham stage with Ns = 2^LNS (>= 32), one butterfly j = tid per
// thread: inputs x[j + 512 r], twiddles w_(16 Ns)^(r k) (k = j mod Ns) from
// two hardware sine / cosine pairs (w, w^4) and packed products (w^2, w^3,
// w^8, w^12, then the 15 powers as in fft.hpp tw_apply), 16-point DFT,
// outputs at b + Ns r, b = 16 (j - k) + k.
template <bool INV, int LNS>
__device__ __forceinline__ void c2_stage_r16(int tid) {
    constexpr int NS = 1 << LNS;
    static_assert(NS >= 32, "c2pos offsets assume Ns a multiple of 32");
    const int j = tid, k = j & (NS - 1);
    c2f v[16];
    const c2lds *src = c2_at(j + (j >> 5));  // c2pos(j + 512 r) = c2pos(j) + 528 r
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = src[528 * r];
    if constexpr (NS == 32) {  // the 15 x 32 twiddles of this stage from the workgroup's LDS table
        const c2lds *tw = c2_at(C2_TW1 + k);
#pragma unroll
        for (int r = 1; r < 16; ++r) v[r] = c2_mul(v[r], tw[32 * (r - 1)]);
    } else {
        constexpr float inv = 1.0f / (float)(16 * NS);
        const float x1 = (float)k * inv, x4 = (float)((4 * k) & (16 * NS - 1)) * inv;
        const c2f w1 = c2f{__builtin_amdgcn_cosf(x1), INV ? __builtin_amdgcn_sinf(x1) : -__builtin_amdgcn_sinf(x1)};
        const c2f w4 = c2f{__builtin_amdgcn_cosf(x4), INV ? __builtin_amdgcn_sinf(x4) : -__builtin_amdgcn_sinf(x4)};
        const c2f w2 = c2_mul(w1, w1), w3 = c2_mul(w2, w1), w8 = c2_mul(w4, w4), w12 = c2_mul(w8, w4);
        const c2f wb[3] = {w1, w2, w3}, wq[3] = {w4, w8, w12};
#pragma unroll
        for (int b = 1; b < 4; ++b) v[b] = c2_mul(v[b], wb[b - 1]);
#pragma unroll
        for (int q = 1; q < 4; ++q) {
            v[4 * q] = c2_mul(v[4 * q], wq[q - 1]);
#pragma unroll
            for (int b = 1; b < 4; ++b) v[4 * q + b] = c2_mul(v[4 * q + b], c2_mul(wq[q - 1], wb[b - 1]));
        }
    }
    c2_dft16<INV>(v);
    const int bo = ((j - k) << 4) + k;
    __syncthreads();
    c2lds *dst = c2_at(bo + (bo >> 5));  // c2pos(bo + Ns r) = c2pos(bo) + (Ns + Ns / 32) r
#pragma unroll
    for (int r = 0; r < 16; ++r) dst[(NS + NS / 32) * r] = v[r];
    __syncthreads();
}

// Natural-order P-point DFT of the image (element i at c2pos(i)), in place
template <bool INV>
__device__ __forceinline__ void c2_fft(int tid, uint32_t msk) {
    c2_stage0_r32<INV>(tid, msk);
    c2_stage_r16<INV, 5>(c2_opaque(tid));
    c2_stage_r16<INV, 9>(c2_opaque(tid));
}

}  // namespace

// diagnostics (SG_AMP_TPROF): thread 0 stamps the shader clock at point k of
// the half's third class (cw2_ab: 0-15, cw2_az: 32-47) and at kernel entry / exit
// (compiled in only with the stamps: -DC2_STAMPS=1, or a diagnostic build `make DIAG=1`; in the shipped
// build each point's runtime test cost about five scalar instructions per class and stamp point)
#if !defined(C2_STAMPS) && defined(SG_DIAG)
#define C2_STAMPS 1
#endif
#ifndef C2_STAMPS
#define C2_STAMPS 0
#endif
#define C2_TP(k)                                                                                                \
    do {                                                                                                        \
        if (C2_STAMPS && tb.tprof && threadIdx.x == 0)                                                          \
            tb.tprof[(size_t)blockIdx.x * 64 + (k)] = __builtin_readcyclecounter();                             \
    } while (0)
#define C2_TPC(k)                          \
    do {                                   \
        if (m2 == h * Qh + 2) C2_TP(k);   \
    } while (0)

// ---------------------------------------------------------------------------- Ab
// LDS: the P-point image (64 KB), then the previous beta's section max and
// 1/sum (stM, stI: 8 KB), staged once per launch.
constexpr size_t C2_IMG_BYTES = (size_t)c2pos(C2_P) * 8;  // padded: element i at c2pos(i)
constexpr size_t C2_CP_BYTES = C2_IMG_BYTES + 2 * 1024 * 4 + 16 + 15 * 32 * 8;  // class pointers (c2_stage_cp)
constexpr size_t C2_LDS_BYTES = C2_CP_BYTES + 4 * 72;  // + the trash slot (CW2_TRASH), the stage twiddles
                                                       // (C2_TW1), the class pointers (Q + 1 <= 72)
// The class bounds from LDS: read through vector memory they made every class start wait for all
// outstanding vector-memory operations (vmcnt(0)), the previous class's stores included.
__device__ __forceinline__ const int *c2_stage_cp(unsigned char *smem, const Cw2Tables &tb, int tid) {
    int *cp = reinterpret_cast<int *>(smem + C2_CP_BYTES);
    for (int i = tid; i <= tb.Q; i += C2_T) cp[i] = tb.cls_ptr[i];
    return cp;
}
static_assert(C2_TW1 * 8 == C2_IMG_BYTES + 2 * 1024 * 4 + 16, "twiddle table after the trash slot");
static_assert(CW2_TRASH == (C2_IMG_BYTES + 2 * 1024 * 4) / 4, "trash slot after the staged statistics");

// Raw buffer resources: loads and stores address by a per-lane byte offset
// plus a scalar one (no 64-bit address arithmetic on the vector ALUs), and
// the hardware range check (offset >= bytes) returns 0 for loads and drops
// stores -- the class slices' ragged ends need no clamps or branches.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t c2_rsrc(const void *p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, bytes > 0 ? bytes : 0, 0x00020000);
}
__device__ __forceinline__ float c2_ldf(__amdgpu_buffer_rsrc_t r, int vo, int so) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0));
}
__device__ __forceinline__ uint32_t c2_ldu(__amdgpu_buffer_rsrc_t r, int vo, int so) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, vo, so, 0);
}
// workgroup-uniform values (class bounds) in scalar registers: a buffer
// resource built from them stays scalar (no waterfall loop)
__device__ __forceinline__ int c2_uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
// a thread's OT slot words of a thread-major [512][OTP] table, 16 bytes per load
template <int OT>
__device__ __forceinline__ void c2_ld_slots(__amdgpu_buffer_rsrc_t r, int tl, uint32_t *out) {
    constexpr int OTP = cw2_otp(OT);
#pragma unroll
    for (int q = 0; q < OTP / 4; ++q) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, 4 * OTP * tl, 16 * q, 0);
#pragma unroll
        for (int c = 0; c < 4; ++c)
            if (4 * q + c < OT) out[4 * q + c] = v[c];
    }
}
constexpr int C2_SN = C2_NC * C2_SC;  // class entries per thread


template <int OT>
__global__ __launch_bounds__(C2_T, 4) void cw2_ab(Cw2Tables tb, RegBufs<float> bf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float *dr = reinterpret_cast<float *>(smem);
    c2f *sMI = reinterpret_cast<c2f *>(smem + C2_IMG_BYTES);  // previous beta's (section max, 1 / sum)
    const int h = blockIdx.x % tb.np, cw = blockIdx.x / tb.np, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    C2_SETPRIO(C2_PRIO_REST);
    const size_t lb = (size_t)cw * tb.L;
    for (int l = tid; l < tb.L; l += C2_T) {  // previous beta's section max, 1/sum
        sMI[l] = c2f{bf.stM[lb + l], bf.stI[lb + l]};
    }
    const float inv_tp = (float)(C2_LOG2E / bf.tau[cw]);  // log2 e / tau (c2_exp2)
    float *s = bf.s + (size_t)cw * tb.LM;  // s in; beta out (read by cw2_az, which writes the new s)
    cx<float> Ha[OT], Hb[OT];  // H[a], conj H[b] of the thread's outputs over this half's classes
#pragma unroll
    for (int j = 0; j < OT; ++j) Ha[j] = Hb[j] = {0.f, 0.f};
    const int Qh = tb.Q / tb.np;
    c2_tw1_init<false>(tid);
    const int *cpl = c2_stage_cp(smem, tb, tid);
    __syncthreads();  // the staged statistics
    C2_TP(10);
    // H[a] += W Y[r], conj H[b] += W conj Y[P - r] from the image's transform of class m (invalid slots:
    // a = 0, unused); the owned indices a and the rows' LDS byte addresses (host table rab) reloaded per
    // class from L1 (held across the transform they spill), in two rounds
    constexpr int OTP = cw2_otp(OT);
    const __amdgpu_buffer_rsrc_t rk = c2_rsrc(tb.kat, 4 * OTP * C2_T);  // thread-major: OTP / 4 loads of 16 B
    auto acc_tables = [&](int tl, uint32_t *ka) {
        c2_ld_slots<OT>(rk, tl, ka);
    };
    auto accumulate = [&](int m, const uint32_t *ka) {
        if (C2_SKIP(2)) return;
#pragma unroll
        for (int j = 0; j < OT; ++j) {
            const uint32_t a = ka[j] & CW_KMASK;
            const int r = (int)a & (C2_P - 1);
            const c2f ya2 = *c2_at(c2pos(r)), yb2 = *c2_at(c2pos((C2_P - r) & (C2_P - 1)));
            const cx<float> ya = {ya2.x, ya2.y}, yb = {yb2.x, yb2.y};
            const cx<float> w = c2_w(tb, __umul24((uint32_t)m, a));  // (a < 2^19, m < 2^6: full-rate multiply)
            Ha[j] = cmac_pk(Ha[j], w, ya);
            Hb[j] = cmacc_pk(Hb[j], w, yb);
        }
    };
    // Software-pipelined over the classes: class m2's slice is requested, then the previous class's
    // transform (still in the image) is accumulated while the loads are in flight, then m2 is scattered
    // and transformed
    // (at most 12 outputs per thread: the accumulation's slot words are class-invariant, so they are
    // requested after each transform and arrive across the loop edge -- cw2_ab 0.397 -> 0.391 ms per launch,
    // profiles/r05_c2_r13_fix.txt)
    constexpr bool PF = C2_AB_PF && OT <= 12;
    uint32_t kapf[PF ? OT : 1];
    for (int m2 = h * Qh; m2 < (h + 1) * Qh; ++m2) {
        const int tl = c2_opaque(tid);
        C2_TPC(0);
        const int q0 = c2_uni(cpl[m2]), q1 = c2_uni(cpl[m2 + 1]);
        // (at more than 12 outputs per thread the slice is requested after the accumulation: in flight
        // during it, it spills)
        constexpr bool PL = OT <= 12;
        if (!PL && m2 > h * Qh) {
            uint32_t ka[OT];
            acc_tables(tl, ka);
            accumulate(m2 - 1, ka);
            __syncthreads();
        }
        // (the accumulation's table loads first: vector-memory loads complete in order)
        uint32_t kl[PL && !PF ? OT : 1];
        if constexpr (PL && !PF)
            if (m2 > h * Qh) acc_tables(tl, kl);
        const uint32_t *ka = PF ? kapf : kl;
        float v[C2_SN];
        uint32_t e[C2_SN];
        {  // every load of the class slice in one round trip; past the class's end s reads 0 and the
           // padded table points at the trash slot (sparc.py:429-432 below writes there harmlessly)
            const __amdgpu_buffer_rsrc_t rs0 = c2_rsrc(s + q0, 4 * (q1 - q0));
            const __amdgpu_buffer_rsrc_t re = c2_rsrc(tb.cls2 + (size_t)m2 * CW2_SLICE, 4 * CW2_SLICE);
#pragma unroll
            for (int i = 0; i < C2_SN; ++i) {
                if (C2_SKIP(4)) {  // (synthetic entries inside the image, section 0)
                    v[i] = (float)(tl + i);
                    e[i] = (uint32_t)(((tl * 37 + i * 4099) & 8191) * 2);
                    continue;
                }
                v[i] = c2_ldf(rs0, 4 * tl + 4 * i * C2_T, 0);
                e[i] = c2_ldu(re, 4 * tl, 4 * i * C2_T);
            }
        }
        // (requested before the scatter's stores: a later load would wait for them, vmcnt is in order)
        const uint32_t cmk = tb.cmask[m2 * C2_T + tl];
        if (PL && m2 > h * Qh) {
            accumulate(m2 - 1, ka);
            __syncthreads();  // the image is read before the scatter overwrites it
        }
        C2_TPC(8);
        const __amdgpu_buffer_rsrc_t rs = c2_rsrc(s + q0, 4 * (q1 - q0));
#pragma unroll
        for (int c = 0; c < C2_NC; ++c) {  // beta = eta(s), sparc.py:429-432, scattered into the image and
                                           // stored over s for cw2_az (its beta_prev; past the end: dropped)
#pragma unroll
            for (int i = c * C2_SC; i < (c + 1) * C2_SC; ++i) {
                const int sec = e[i] >> 16;
                const c2f mi = sMI[sec];
                v[i] = c2_exp2((v[i] - mi.x) * inv_tp) * mi.y;
                if (!C2_SKIP(256)) dr[e[i] & 0xffffu] = v[i];
                if (!C2_SKIP(512))
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[i]), rs, 4 * tl + 4 * i * C2_T,
                                                      0, 0);
            }
            C2_TPC(1 + c);
        }
        __syncthreads();
        C2_TPC(3);
        C2_SETPRIO(C2_PRIO_FFT);
        if (!C2_SKIP(1)) c2_fft<false>(tl, cmk);
        C2_SETPRIO(C2_PRIO_REST);
        C2_TPC(6);
        if constexpr (PF) acc_tables(c2_opaque(tid), kapf);  // class-invariant: in flight across the loop edge
    }
    {
        uint32_t ka[OT];
        acc_tables(c2_opaque(tid), ka);
        accumulate((h + 1) * Qh - 1, ka);
    }
    C2_TP(11);
    // this half's part of the forward output Re(c1 H[a] + c2 conj H[b]) (linear in H: cw2_ctrl adds the
    // two halves' parts; a quarter of the bytes of the partial H pair)
    float *xr = tb.xr + ((size_t)cw * tb.np + h) * OT * C2_T;
#pragma unroll
    for (int j = 0; j < OT; ++j) {
        const float4 c = tb.cf[j * C2_T + tid];
        xr[j * C2_T + tid] = (c.x * Ha[j].x - c.y * Ha[j].y) + (c.z * Hb[j].x - c.w * Hb[j].y);
    }
}

// ---------------------------------------------------------------------------- control
__device__ __forceinline__ double c2_block_sum(double v, double *red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    return t;
}

// two sums at once (one pair of barriers), each in c2_block_sum's order
__device__ __forceinline__ void c2_block_sum2(double &a, double &b, double *red) {
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (int)(blockDim.x >> 6);
    __syncthreads();
    if (lane == 0) {
        red[wid] = a;
        red[nw + wid] = b;
    }
    __syncthreads();
    double ta = 0.0, tb = 0.0;
    for (int w = 0; w < nw; ++w) {
        ta += red[w];
        tb += red[nw + w];
    }
    a = ta;
    b = tb;
}

template <int OT>
__global__ __launch_bounds__(C2_T) void cw2_ctrl(Cw2Tables tb, RegBufs<float> bf, AmpScalars sc, AmpParams pr,
                                                 int t) {
    __shared__ double red[C2_T / 64];
    const int cw = blockIdx.x, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    const bool have_beta = t > 0;
    double *psi = sc.psi + cw, *psi_prev = sc.psi_prev + cw;
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
    } else {
        g = pr.W[0];
        if (tid == 0) sc.gamma[cw] = g;
    }
    const float *xr0 = tb.xr + (size_t)cw * tb.np * OT * C2_T, *xr1 = xr0 + (size_t)OT * C2_T;
    float zr[OT];
    float2 gmv[C2_POLAR ? OT : 1];
    double acc = 0.0;
    {
        // every load first, in one round trip (the uniform branch outside the slot loops: written per slot,
        // with the stores between, the compiler waited for each slot's loads in turn -- 36 dependent round
        // trips per launch); invalid slots: output 0, unused
        float yv[OT], zv[OT], r0[OT], r1[OT];
        float *ys = tb.ys + (size_t)cw * OT * C2_T, *zs = tb.zs + (size_t)cw * OT * C2_T;
#pragma unroll
        for (int j = 0; j < OT; ++j)
            if constexpr (C2_POLAR != 0) gmv[j] = tb.gm[j * C2_T + tid];
        if (have_beta) {  // y, the previous z and the two halves' parts in slot order: coalesced
#pragma unroll
            for (int j = 0; j < OT; ++j) {
                yv[j] = ys[j * C2_T + tid];
                zv[j] = zs[j * C2_T + tid];
                r0[j] = xr0[j * C2_T + tid];
                r1[j] = xr1[j * C2_T + tid];
                for (int pp = 2; pp < tb.np; ++pp) r1[j] += xr0[(size_t)pp * OT * C2_T + j * C2_T + tid];
            }
#pragma unroll
            for (int j = 0; j < OT; ++j)  // Onsager residual, sparc.py:943-946; r = Re(c1 H[a] + c2 conj H[b])
                zr[j] = (yv[j] - (r0[j] + r1[j])) + bco * zv[j];
        } else {  // first iteration: gather y and keep it in slot order, 0 in the invalid slots -- so their
                  // z stays 0 in every iteration (their forward part is 0: zero coefficients) and they add
                  // exact zeros to the sum below, which then needs no validity test
#pragma unroll
            for (int j = 0; j < OT; ++j)
                yv[j] = (tb.ka[j * C2_T + tid] & CW_VALID) ? y[tb.oi[j * C2_T + tid]] : 0.f;
#pragma unroll
            for (int j = 0; j < OT; ++j) {
                ys[j * C2_T + tid] = yv[j];
                zr[j] = yv[j];
            }
        }
        // z in slot order only: a hand-over to the staged engine rebuilds its natural order once
        // (cw2_z_natural); scattered here every iteration it cost 12 index loads and 12 scattered stores
        // per thread
#pragma unroll
        for (int j = 0; j < OT; ++j) {
            zs[j * C2_T + tid] = zr[j];
            if (sum_z) acc += (double)zr[j] * (double)zr[j];
        }
    }
    double phi;
    if (sum_z) {
        phi = c2_block_sum(acc, red) / (double)tb.n;  // sparc.py:949-955
    } else {
        phi = pr.awgn_var + g;
    }
    const double tv_new = (tb.L * phi / tb.n) / pr.W[0];  // sparc.py:958-969
    if (tid == 0) {
        bf.phi[cw] = phi;
        bf.tau[cw] = tv_new;
    }
    const float iph = (float)(1.0 / phi);
    constexpr int OTP = cw2_otp(OT);
#if C2_POLAR
    // z / phi times the slot's (|al|, |be|) (build_cw2 polar form), two floats per slot; padding slots 0
    if constexpr (cw2_vz_tm(OT) && C2_VZ_HALF) {  // z / phi alone (cw2_az scales it)
        float4 *vz4 = reinterpret_cast<float4 *>(tb.vz + ((size_t)cw * C2_T + tid) * OTP);  // thread-major
#pragma unroll
        for (int q = 0; q < OTP / 4; ++q) {
            float w[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) w[c] = 4 * q + c < OT ? zr[4 * q + c] * iph : 0.f;
            vz4[q] = make_float4(w[0], w[1], w[2], w[3]);
        }
    } else if constexpr (cw2_vz_tm(OT)) {
        float4 *vz4 = reinterpret_cast<float4 *>(tb.vz + ((size_t)cw * C2_T + tid) * OTP * 2);  // thread-major
#pragma unroll
        for (int q = 0; q < OTP / 2; ++q) {
            float w[4];
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int j = 2 * q + c;
                const float2 g = j < OT ? gmv[j] : make_float2(0.f, 0.f);
                const float v = j < OT ? zr[j] * iph : 0.f;
                w[2 * c] = v * g.x;
                w[2 * c + 1] = v * g.y;
            }
            vz4[q] = make_float4(w[0], w[1], w[2], w[3]);
        }
    } else {
        float2 *vzs = reinterpret_cast<float2 *>(tb.vz) + (size_t)cw * OT * C2_T;  // slot-major
#pragma unroll
        for (int j = 0; j < OT; ++j) {
            const float v = zr[j] * iph;
            vzs[j * C2_T + tid] = make_float2(v * gmv[j].x, v * gmv[j].y);
        }
    }
#else
    if constexpr (cw2_vz_tm(OT)) {
        float4 *vz4 = reinterpret_cast<float4 *>(tb.vz + ((size_t)cw * C2_T + tid) * OTP);  // thread-major
#pragma unroll
        for (int q = 0; q < OTP / 4; ++q) {  // z / phi (sparc.py:972); padding slots 0
            float w[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) w[c] = 4 * q + c < OT ? zr[4 * q + c] * iph : 0.f;
            vz4[q] = make_float4(w[0], w[1], w[2], w[3]);
        }
    } else {
        float *vzs = tb.vz + (size_t)cw * OT * C2_T;  // slot-major
#pragma unroll
        for (int j = 0; j < OT; ++j) vzs[j * C2_T + tid] = zr[j] * iph;
    }
#endif
}

// ---------------------------------------------------------------------------- Az
template <int OT>
__global__ __launch_bounds__(C2_T, 4) void cw2_az(Cw2Tables tb, RegBufs<float> bf, int t) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float *dr = reinterpret_cast<float *>(smem);
    const int h = blockIdx.x % tb.np, cw = blockIdx.x / tb.np, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    C2_SETPRIO(C2_PRIO_REST);
    const size_t lb = (size_t)cw * tb.L;
    const bool have_beta = t > 0;
    const double tv = bf.tau[cw];
    const float tau = (float)tv, inv_tau = (float)(C2_LOG2E / tv);  // log2 e / tau (c2_exp2)
    float *s = bf.s + (size_t)cw * tb.LM;
    constexpr int OTP = cw2_otp(OT);
    // [512][OTP][2] / [OT][512][2] (polar form: (|al|, |be|) z / phi); [512][OTP] / [OT][512] (C2_POLAR 0)
    constexpr bool VZH = C2_VZ_HALF && C2_POLAR && cw2_vz_tm(OT);
    const float *vz = tb.vz + (size_t)cw * (cw2_vz_tm(OT) ? OTP : OT) * C2_T * (C2_POLAR && !VZH ? 2 : 1);
    // running statistics of sections tid and tid + 512 over this half's classes
    const int Lb = tb.Lblk;
#if !C2_STATS_LAUNCH
    float Mr[2] = {-INFINITY, -INFINITY}, R1[2] = {0.f, 0.f}, R2[2] = {0.f, 0.f}, st[2] = {NAN, NAN};
    int jt[2] = {-1, -1};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int sec = tid + k * C2_T;
        if (bf.true_idx && sec < Lb) jt[k] = tb.qpos[sec * tb.M + bf.true_idx[lb + sec]];
    }
#else
    (void)lb;
    (void)Lb;
    (void)inv_tau;
#endif
    const int Qh = tb.Q / tb.np;
    c2_tw1_init<true>(tid);
    const int *cpl = c2_stage_cp(smem, tb, tid);
    constexpr bool HOLD = C2_AZ_HOLD && C2_POLAR && OT <= 12;
    c2f vhold[HOLD ? OT : 1];
    if constexpr (HOLD) {
        const __amdgpu_buffer_rsrc_t rv = c2_rsrc(vz, 8 * OTP * C2_T);
#pragma unroll
        for (int q = 0; q < OTP / 2; ++q) {
            const auto w = __builtin_amdgcn_raw_buffer_load_b128(rv, 8 * OTP * tid, 16 * q, 0);
            if (2 * q < OT) vhold[2 * q] = c2f{__uint_as_float(w[0]), __uint_as_float(w[1])};
            if (2 * q + 1 < OT) vhold[2 * q + 1] = c2f{__uint_as_float(w[2]), __uint_as_float(w[3])};
        }
    }
    __syncthreads();  // the staged statistics
    C2_TP(42);
    for (int m2 = h * Qh; m2 < (h + 1) * Qh; ++m2) {
        const int tl = c2_opaque(tid);
        C2_TPC(32);
        const uint32_t rmk = tb.cmask[tb.Q * C2_T + tl];
        // the class slice (entries' image positions, beta_prev), requested before the transform and
        // consumed after it, so its HBM latency hides behind the transform
        const int q0 = c2_uni(cpl[m2]), q1 = c2_uni(cpl[m2 + 1]);
        const __amdgpu_buffer_rsrc_t rs = c2_rsrc(s + q0, 4 * (q1 - q0));  // past the class's end: reads 0,
                                                                           // stores dropped
        // (at more than 12 outputs per thread the slice stays out of flight during the rows and the
        // transform: it would spill)
        constexpr bool EARLY = OT <= 12;
        float v[C2_SN];
        uint32_t e[C2_SN];
        auto load_v = [&]() {  // beta_prev of the class slice
#pragma unroll
            for (int i = 0; i < C2_SN; ++i) {
                if (C2_SKIP(128)) {  // (synthetic entries inside the image, section 0)
                    v[i] = (float)(tl + i);
                    e[i] = (uint32_t)(((tl * 37 + i * 4099) & 8191) * 2);
                    continue;
                }
                v[i] = c2_ldf(rs, 4 * tl + 4 * i * C2_T, 0);  // (t = 0: unused)
            }
        };
        // the entries' positions and (HOLD 0) beta_prev; with the scaled z / phi held in registers (HOLD) beta_prev
        // is requested after the transform (in flight across it beside the held values, it spills)
        auto load_slice = [&]() {
#if C2_AZPOS
            // the entries' image positions two per word (clsp: entries i and i + 9 of the thread), half the
            // table loads and bytes of the full words (the sections are not needed here)
            const __amdgpu_buffer_rsrc_t re = c2_rsrc(tb.clsp + (size_t)m2 * (CW2_SLICE / 2), 2 * CW2_SLICE);
#pragma unroll
            for (int i = 0; i < C2_SN / 2; ++i) {
                const uint32_t w = c2_ldu(re, 4 * tl, 4 * i * C2_T);
                e[i] = w;  // (packed: entries i and i + 9, unpacked at the gather -- 9 VGPRs across the transform)
            }
#else
            const __amdgpu_buffer_rsrc_t re = c2_rsrc(tb.cls2 + (size_t)m2 * CW2_SLICE, 4 * CW2_SLICE);
#pragma unroll
            for (int i = 0; i < C2_SN; ++i) e[i] = c2_ldu(re, 4 * tl, 4 * i * C2_T);
#endif
            if constexpr (!HOLD) load_v();
        };
#if C2_POLAR
        if (!C2_SKIP(16)) {  // rows r and P - r of each owned pair: sum of al v conj(W) / be v W over its outputs
            // (v = z / phi).  Polar form (build_cw2): al conj(W) = |al| (cos x, sin x) and be W = |be| (sin x,
            // cos x) with x = ((3 + 8 m2) a + o N/2) / 4N revolutions from the slot word alone, and cw2_ctrl
            // stores (|al| v, |be| v): per slot and class one phase, two packed FMAs per row, and 12 bytes of
            // tables instead of 24 (the complex al, be were 16 of them).  Branch-free: every slot accumulates
            // (NEWROW restarts the sums) and writes both rows -- the pair's rows on its last slot (ENDROW), the
            // trash slot otherwise (invalid slots: zero scale) -- so the two pairs whose rows coincide (r = 0,
            // P / 2) write their sum.  (Slot words and v reloaded per class from L1 / L2: held across the
            // transform, or loaded one class ahead, they spill.)
            constexpr int CH = OT > 12 ? (OT + 1) / 2 : OT;  // slots per load round (one round at 12 per thread)
            const __amdgpu_buffer_rsrc_t rv = c2_rsrc(vz, 8 * OTP * C2_T),
                                         rk = c2_rsrc(cw2_vz_tm(OT) ? tb.kat : tb.ka, 4 * OTP * C2_T);
            uint32_t kall[CH == OT ? OT : 1];
            c2f vall[CH == OT ? OT : 1];
            if constexpr (HOLD) {  // the slot words (shared by every codeword: L2 hits) reloaded per class
                if (!C2_SKIP(32)) c2_ld_slots<OT>(rk, tl, kall);
#pragma unroll
                for (int j = 0; j < OT; ++j) vall[j] = vhold[j];
            } else if constexpr (VZH) {  // slot words, z / phi (4 B per slot) and the plan's (|al|, |be|)
                if (!C2_SKIP(32)) {
                    c2_ld_slots<OT>(rk, tl, kall);
                    const __amdgpu_buffer_rsrc_t rv1 = c2_rsrc(vz, 4 * OTP * C2_T),
                                                 rg = c2_rsrc(tb.gmt, 8 * OTP * C2_T);
                    float v1[OTP];
#pragma unroll
                    for (int q = 0; q < OTP / 4; ++q) {
                        const auto w = __builtin_amdgcn_raw_buffer_load_b128(rv1, 4 * OTP * tl, 16 * q, 0);
#pragma unroll
                        for (int c = 0; c < 4; ++c) v1[4 * q + c] = __uint_as_float(w[c]);
                    }
#pragma unroll
                    for (int q = 0; q < OTP / 2; ++q) {
                        const auto w = __builtin_amdgcn_raw_buffer_load_b128(rg, 8 * OTP * tl, 16 * q, 0);
                        if (2 * q < OT)
                            vall[2 * q] = c2f{__uint_as_float(w[0]), __uint_as_float(w[1])} * v1[2 * q];
                        if (2 * q + 1 < OT)
                            vall[2 * q + 1] = c2f{__uint_as_float(w[2]), __uint_as_float(w[3])} * v1[2 * q + 1];
                    }
                }
            } else if constexpr (CH == OT) {  // one load round: a thread's slot words and scaled z / phi, 16-byte loads
                if (!C2_SKIP(32)) {
                    c2_ld_slots<OT>(rk, tl, kall);
#pragma unroll
                    for (int q = 0; q < OTP / 2; ++q) {
                        const auto w = __builtin_amdgcn_raw_buffer_load_b128(rv, 8 * OTP * tl, 16 * q, 0);
                        if (2 * q < OT) vall[2 * q] = c2f{__uint_as_float(w[0]), __uint_as_float(w[1])};
                        if (2 * q + 1 < OT) vall[2 * q + 1] = c2f{__uint_as_float(w[2]), __uint_as_float(w[3])};
                    }
                }
            }
            const uint32_t cm = 3u + 8u * (uint32_t)m2;
            c2f u0{0.f, 0.f}, u1{0.f, 0.f};
#pragma unroll
            for (int j0 = 0; j0 < OT; j0 += CH) {
                uint32_t ka[CH];
                c2f vv[CH];
#pragma unroll
                for (int i = 0; i < CH; ++i) {
                    const int j = j0 + i < OT ? j0 + i : OT - 1;
                    if (C2_SKIP(32)) {
                        const uint32_t r = (uint32_t)(tl * 8 + j) & 4095u;
                        ka[i] = r | CW_VALID | ((j & 1) ? CW_ENDROW : CW_NEWROW);
                        vv[i] = c2f{0.5f, (float)j};
                        continue;
                    }
                    if constexpr (CH == OT) {
                        ka[i] = kall[j];
                        vv[i] = vall[j];
                    } else {  // (two load rounds: slot-major, each load a contiguous run of the wavefront)
                        ka[i] = c2_ldu(rk, 4 * tl, 4 * j * C2_T);
                        const auto w = __builtin_amdgcn_raw_buffer_load_b64(rv, 8 * tl, 8 * j * C2_T, 0);
                        vv[i] = c2f{__uint_as_float(w[0]), __uint_as_float(w[1])};
                    }
                }
#pragma unroll
                for (int j = 0; j < CH; ++j) {
                    if (j0 + j >= OT) break;
                    const uint32_t k = ka[j];
                    const uint32_t xu =
                        (__umul24(cm, k & CW_KMASK) + (((k >> CW_OFFSHIFT) & 7u) << tb.sh_off)) & tb.m4n;
                    const float x = (float)xu * tb.inv_4n;  // (exact: 4N <= 2^24)
                    const c2f cs = c2f{__builtin_amdgcn_cosf(x), __builtin_amdgcn_sinf(x)};
#if C2_ROWS_ALWAYS
                    // every slot writes its pair's running sums at the pair's rows (one thread owns a pair, so
                    // the pair's last slot writes last: the complete sums), padding slots continue the thread's
                    // last pair with a zero term (build_cw2); row P - r of the r = 0 pair is P, just past the
                    // image (the Ab-only statistics area), and a pair whose rows coincide (CW_SELF) writes
                    // u0 + u1 at row r after u1.  Keep / self factors by v_bfe + v_bfi, no compare: no SGPR
                    // masks, no hazard nops, no exec-masked store
                    uint32_t keepb, selfb;
                    {
                        const int nr = __builtin_amdgcn_sbfe((int)k, 20, 1), sf = __builtin_amdgcn_sbfe((int)k, 23, 1);
                        asm("v_bfi_b32 %0, %1, 0, %2" : "=v"(keepb) : "v"(nr), "v"(0x3f800000u));  // NEWROW: 0, else 1
                        asm("v_bfi_b32 %0, %1, %2, 0" : "=v"(selfb) : "v"(sf), "v"(0x3f800000u));  // SELF: 1, else 0
                    }
                    const float keep = __uint_as_float(keepb), selff = __uint_as_float(selfb);
                    u0 = __builtin_elementwise_fma(cs, vv[j].xx, u0 * keep);
                    u1 = __builtin_elementwise_fma(cs.yx, vv[j].yy, u1 * keep);
                    const uint32_t r = k & (uint32_t)(C2_P - 1), rb = (uint32_t)C2_P - r;
                    c2lds *pa = (c2lds *)(size_t)(8u * (r + (r >> 5))), *pb = (c2lds *)(size_t)(8u * (rb + (rb >> 5)));
                    *pb = u1;
                    *pa = __builtin_elementwise_fma(u1, c2f{selff, selff}, u0);
#else
                    const float keep = (k & CW_NEWROW) ? 0.f : 1.f;
                    u0 = __builtin_elementwise_fma(cs, vv[j].xx, u0 * keep);
                    u1 = __builtin_elementwise_fma(cs.yx, vv[j].yy, u1 * keep);
                    const int r = (int)(k & (uint32_t)(C2_P - 1)), rb = C2_P - r;
                    const bool end = (k & CW_ENDROW) != 0;
                    c2lds *pa = (c2lds *)(size_t)(end ? 8u * (uint32_t)c2pos(r) : 4u * CW2_TRASH);
                    c2lds *pb = (c2lds *)(size_t)((end && !(k & CW_SELF)) ? 8u * (uint32_t)c2pos(rb) : 4u * CW2_TRASH);
                    *pa = u0;
                    *pb = u1;
                    if (k & CW_SELF) *pa = u0 + u1;
#endif
                }
            }
        }
#else
        if (!C2_SKIP(16)) {  // rows r and P - r of each owned pair: sum of al v conj(W) / be v W over its outputs (v = z / phi),
           // branch-free: every slot accumulates (NEWROW restarts the sums) and writes both rows -- the
           // pair's rows on its last slot (ENDROW), the trash slot otherwise (invalid slots: al = be = 0),
           // addresses derived from the slot word (C2_ROWS_DERIVE; the host table wab is the A/B form) --
           // the two pairs whose rows coincide (r = 0, P / 2) then write their sum.  (a, al, be, v and the addresses reloaded per class from L1 / L2: held across the transform,
           // or loaded one class ahead, they spill; al v and be v precomputed per codeword were slower -- four
           // times the per-codeword bytes re-read from L2 every class.)
            constexpr int CH = OT > 12 ? (OT + 1) / 2 : OT;  // slots per load round (one round at 12 per thread)
            const __amdgpu_buffer_rsrc_t rg = c2_rsrc(tb.gf, 16 * OT * C2_T), rv = c2_rsrc(vz, 4 * OTP * C2_T),
                                         rk = c2_rsrc(cw2_vz_tm(OT) ? tb.kat : tb.ka, 4 * OTP * C2_T),
                                         rw = c2_rsrc(tb.wab, 8 * OT * C2_T);
            // one load round (CH == OT): a thread's slot words and z / phi in 16-byte loads (thread-major)
            uint32_t kall[CH == OT ? OT : 1], vall[CH == OT ? OT : 1];
            if constexpr (CH == OT) {
                if (!C2_SKIP(32)) {
                    c2_ld_slots<OT>(rk, tl, kall);
                    c2_ld_slots<OT>(rv, tl, vall);
                }
            }
            cx<float> u0{0.f, 0.f}, u1{0.f, 0.f};
#pragma unroll
            for (int j0 = 0; j0 < OT; j0 += CH) {
                uint32_t ka[CH];
                float4 gc[CH];
                float vv[CH];
                uint2 wa[CH];
#pragma unroll
                for (int i = 0; i < CH; ++i) {
                    const int j = j0 + i < OT ? j0 + i : OT - 1;
                    if (C2_SKIP(32)) {
                        const uint32_t r = (uint32_t)(tl * 8 + j) & 4095u;
                        ka[i] = r | CW_VALID | ((j & 1) ? CW_ENDROW : CW_NEWROW);
                        gc[i] = make_float4(0.5f, 0.25f, 0.125f, 0.75f);
                        vv[i] = (float)j;
                        wa[i] = make_uint2(8u * (uint32_t)c2pos((int)r), 8u * (uint32_t)c2pos(8192 - (int)r));
                        continue;
                    }
                    if constexpr (CH == OT) {
                        ka[i] = kall[j];
                        vv[i] = __uint_as_float(vall[j]);
                    } else {  // (two load rounds: slot-major, each load a contiguous run of the wavefront --
                              // thread-major, every lane of every per-slot load was a cache line of its own)
                        ka[i] = c2_ldu(rk, 4 * tl, 4 * j * C2_T);
                        vv[i] = c2_ldf(rv, 4 * tl, 4 * j * C2_T);
                    }
                    gc[i] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rg, 16 * tl, 16 * j * C2_T, 0));
                    if (!C2_ROWS_DERIVE)
                        wa[i] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rw, 8 * tl, 8 * j * C2_T, 0));
                }
#pragma unroll
                for (int j = 0; j < CH; ++j) {
                    if (j0 + j >= OT) break;
                    const uint32_t k = ka[j];
                    const cx<float> w = c2_w(tb, __umul24((uint32_t)m2, k & CW_KMASK));  // (a < 2^19, m2 < 2^6)
                    const float keep = (k & CW_NEWROW) ? 0.f : 1.f;
                    u0 = cmacc_pk({u0.x * keep, u0.y * keep}, {gc[j].x * vv[j], gc[j].y * vv[j]}, w);
                    u1 = cmac_pk({u1.x * keep, u1.y * keep}, {gc[j].z * vv[j], gc[j].w * vv[j]}, w);
                    if (C2_ROWS_DERIVE) {  // the host table wab from the slot's flags: rows on the pair's last slot
                        const int r = (int)(k & (uint32_t)(C2_P - 1)), rb = C2_P - r;
                        const bool end = (k & CW_ENDROW) != 0;
                        wa[j].x = end ? 8u * (uint32_t)c2pos(r) : 4u * CW2_TRASH;
                        wa[j].y = (end && !(k & CW_SELF)) ? 8u * (uint32_t)c2pos(rb) : 4u * CW2_TRASH;
                    }
                    c2lds *pa = (c2lds *)(size_t)wa[j].x, *pb = (c2lds *)(size_t)wa[j].y;
                    *pa = c2f{u0.x, u0.y};
                    *pb = c2f{u1.x, u1.y};
                    if (k & CW_SELF) *pa = c2f{u0.x + u1.x, u0.y + u1.y};
                }
            }
        }
#endif
        // (requested after the rows' table loads: vector-memory loads complete in order, so a slice
        // requested before them would hold the rows up for its whole HBM latency)
        if constexpr (EARLY) load_slice();
#if !C2_STATS_LAUNCH
        int sa[2], sb[2];  // the sections' segments of the class (in flight during the transform; sections
                           // past Lb read 0 as their end: empty)
        {
            const __amdgpu_buffer_rsrc_t rg = c2_rsrc(tb.seg + (size_t)m2 * (Lb + 1), 2 * (Lb + 1));
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int sec = tl + k * C2_T;
                sa[k] = __builtin_amdgcn_raw_buffer_load_b16(rg, 2 * sec, 0, 0);
                sb[k] = __builtin_amdgcn_raw_buffer_load_b16(rg, 2 * sec + 2, 0, 0);
            }
        }
#endif
        C2_TPC(33);
        __syncthreads();
        C2_TPC(34);
        C2_SETPRIO(C2_PRIO_FFT);
        if (!C2_SKIP(8)) c2_fft<true>(tl, rmk);
        C2_SETPRIO(C2_PRIO_REST);
        C2_TPC(35);
        float snv[C2_SN];
        if constexpr (!EARLY) load_slice();
        if constexpr (HOLD) load_v();
        {
#pragma unroll
            for (int i = 0; i < C2_SN; ++i) {  // s = beta_prev + tau u (sparc.py:972); beta_prev stored by cw2_ab
                const float b = have_beta ? v[i] : 0.f;
                const uint32_t pos = C2_AZPOS ? (i < C2_SN / 2 ? e[i] & 0xffffu : e[i - C2_SN / 2] >> 16)
                                              : e[i] & 0xffffu;
                snv[i] = b + tau * (C2_SKIP(1024) ? (float)i : dr[pos]);
            }
        }
        C2_TPC(36);
#ifndef C2_DIAG_NO_SSTORE  // (diagnostic builds only: timing without the s stores)
#pragma unroll
        for (int c = 0; c < C2_SN; ++c)  // s to HBM straight from the registers (class order)
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, snv[c]), rs, 4 * tl + 4 * c * C2_T, 0, 0);
#endif
        C2_TPC(37);
        __syncthreads();
        C2_TPC(38);
#if !C2_STATS_LAUNCH
        if (!C2_SKIP(64)) {
#pragma unroll
        for (int c = 0; c < C2_SN; ++c) dr[tl + c * C2_T] = snv[c];  // s of the class in class order (past the
                                                                     // end: unread)
        __syncthreads();
        C2_TPC(39);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            // partial of the section over its segment: the maximum, then the
            // sums of e and e^2 over every entry but one maximum
            // (e = exp((x - max) / tau)); two passes instead of the online
            // rescaling (fewer vector instructions).  The first C2_RC entries are
            // read once for both passes (segments average LM / (Q L) = 8
            // entries; the rest take the loops below), the reads are
            // unskewed (every read a base plus a constant; the segment starts
            // are irregular either way) and entries past the segment are -inf
            // (exp -> 0).  Same box, every codeword active (tools/c2_ablate.py,
            // profiles/r05_c2_variants.txt): the statistics were 28 % of
            // cw2_az; unconditional reads, the fract form below and the rows'
            // derived addresses took cw2_az 0.588 -> 0.570 ms per launch.
            const int a = sa[k], n = sb[k] - sa[k];
            constexpr int RC = C2_RC;
#if C2_NOFIRST
            // every round in the loops (no first round held in registers across the maximum)
            float m = -INFINITY;
            for (int c = 0; c < n; c += RC) {
                float y[RC];
#pragma unroll
                for (int i = 0; i < RC; ++i) y[i] = dr[a + c + i];
#pragma unroll
                for (int i = 0; i < RC; ++i) m = fmaxf(m, c + i < n ? y[i] : -INFINITY);
            }
            float S1 = 0.f, S2 = 0.f, Se = 0.f;
            for (int c = 0; c < n; c += RC) {
                float y[RC];
#pragma unroll
                for (int i = 0; i < RC; ++i) y[i] = dr[a + c + i];
#pragma unroll
                for (int i = 0; i < RC; ++i) {
                    const float ex = c2_exp2(((c + i < n ? y[i] : -INFINITY) - m) * inv_tau);
                    const float f = __builtin_amdgcn_fractf(ex);
                    S1 += f;
                    S2 += f * f;
                    Se += ex;
                }
            }
#else
            const float *sgp = dr + a;  // inside the LDS image past the segment's end too
            float x[RC];
            // every read unconditional, the entries past the segment masked afterwards: written as
            // `i < n ? sgp[i] : -inf` the compiler put each read in its own exec-masked block (two SALU
            // mask operations per read, no paired reads)
#pragma unroll
            for (int i = 0; i < RC; ++i) x[i] = sgp[i];
#if C2_ST_BITS
            {  // -inf past the segment: a lane mask of the segment's first RC entries, then per entry v_bfe_i32
               // (all ones / zero) and v_bfi -- written as a sign mask the compiler turned it into v_cmp + v_cndmask
               // through an SGPR pair, with a hazard s_nop per entry
                uint32_t bits = n >= RC ? 0xffffffffu : ((1u << (n > 0 ? n : 0)) - 1u);
                const uint32_t ninf = 0xff800000u;
#pragma unroll
                for (int i = 0; i < RC; ++i) {
                    const int mk = __builtin_amdgcn_sbfe((int)bits, i, 1);
                    uint32_t r;  // (mk & x) | (~mk & -inf) in one v_bfi_b32 (plain VALU, no hazard with its inputs)
                    asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(mk), "v"(__float_as_uint(x[i])), "v"(ninf));
                    x[i] = __uint_as_float(r);
                }
            }
#else
#pragma unroll
            for (int i = 0; i < RC; ++i) {  // -inf past the segment by a sign mask and v_bfi
                const uint32_t mk = (uint32_t)((i - n) >> 31);  // all ones inside the segment
                x[i] = __uint_as_float((__float_as_uint(x[i]) & mk) | (0xff800000u & ~mk));
            }
#endif
            // no argmax: the maximum by a max3 tree; in the sums, v_fract_f32 drops the entries equal to the
            // maximum (e = exp2(0) = 1 exactly, fract 0; below it e < 1, fract(e) = e) and the entries that
            // tie with it are added back afterwards from Se - S1 = their count (exact small integers), so
            // S1 = sum over every entry but one maximum, as before -- two mask operations fewer per entry
            float m = x[0];
#pragma unroll
            for (int i = 1; i + 1 < RC; i += 2) m = fmaxf(fmaxf(m, x[i]), x[i + 1]);
            if constexpr (RC % 2 == 0) m = fmaxf(m, x[RC - 1]);
            for (int c = RC; c < n; c += RC) {
                float y[RC];
#pragma unroll
                for (int i = 0; i < RC; ++i) y[i] = dr[a + c + i];
#pragma unroll
                for (int i = 0; i < RC; ++i) m = fmaxf(m, c + i < n ? y[i] : -INFINITY);
            }
            float S1 = 0.f, S2 = 0.f, Se = 0.f;
#pragma unroll
            for (int i = 0; i < RC; ++i) {
                const float ex = c2_exp2((x[i] - m) * inv_tau);
                const float f = __builtin_amdgcn_fractf(ex);
                S1 += f;
                S2 += f * f;
                Se += ex;
            }
            for (int c = RC; c < n; c += RC) {
                float y[RC];
#pragma unroll
                for (int i = 0; i < RC; ++i) y[i] = dr[a + c + i];
#pragma unroll
                for (int i = 0; i < RC; ++i) {
                    const float ex = c2_exp2(((c + i < n ? y[i] : -INFINITY) - m) * inv_tau);
                    const float f = __builtin_amdgcn_fractf(ex);
                    S1 += f;
                    S2 += f * f;
                    Se += ex;
                }
            }
#endif
            {
                const float ties = rintf(Se - S1) - 1.f;  // entries equal to the maximum, but one (NaN: empty)
                if (ties > 0.f) {
                    S1 += ties;
                    S2 += ties;
                }
            }
            if (m > -INFINITY) {  // merge into the section's running statistics
                if (m > Mr[k]) {
                    const float f = c2_exp2((Mr[k] - m) * inv_tau);
                    R1[k] = (R1[k] + 1.f) * f + S1;
                    R2[k] = (R2[k] + 1.f) * (f * f) + S2;
                    Mr[k] = m;
                } else {
                    const float f = c2_exp2((m - Mr[k]) * inv_tau);
                    R1[k] += (1.f + S1) * f;
                    R2[k] += (1.f + S2) * (f * f);
                }
            }
            if (jt[k] >= q0 && jt[k] < q1) st[k] = dr[jt[k] - q0];
        }
        }  // (C2_SKIP(64))
        C2_TPC(40);
        __syncthreads();  // the next class overwrites the image
#endif
        C2_TPC(41);
    }
    C2_TP(43);
#if !C2_STATS_LAUNCH
    float4 *part = tb.part + ((size_t)cw * tb.np + h) * Lb;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int sec = tid + k * C2_T;
        if (sec < Lb) part[sec] = make_float4(Mr[k], R1[k], R2[k], st[k]);
    }
#endif
}

// ---------------------------------------------------------------------------- statistics launch
// (C2_STATS_LAUNCH) After cw2_az: one wavefront per section, lane m its class-m segment of s (class order),
// the section's entries k = lane + 64 j read in concatenated class order (each entry's class from an owner
// table the classes' lanes fill); the maximum, then the sums of e = exp((x - max) / tau) and e^2 over every
// entry but one maximum (the fract form of cw2_az's scan), the section's max and 1 / sum (the next Ab's
// softmax, sparc.py:429-432, and a hand-over's state), and 1 - sum beta^2 and the squared error per section
// (sparc.py:973-981) for cw2_final.  Per-lane sums, then a xor tree: a fixed order.
constexpr int C2_ST_K = 8;  // entries per lane: sections of M <= 512 entries
__device__ __forceinline__ float c2_wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ float c2_wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
template <int ST_W>
__global__ __launch_bounds__(64 * ST_W) void cw2_stats(Cw2Tables tb, RegBufs<float> bf) {
    __shared__ int bas[ST_W][64];
    __shared__ uint8_t own[ST_W][64 * C2_ST_K];  // the class of each entry of the section
    const int wpc = tb.Lblk / ST_W;  // workgroups per codeword
    const int w = (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int cw = blockIdx.x / wpc, l = (blockIdx.x % wpc) * ST_W + w;
    if (!bf.active[cw]) return;
    const size_t lb = (size_t)cw * tb.L;
    const float inv_tau = (float)(C2_LOG2E / bf.tau[cw]);  // log2 e / tau (c2_exp2)
    const float *s = bf.s + (size_t)cw * tb.LM;
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
    bas[w][lane] = p0 - (inc - n);
    for (int k = inc - n; k < inc; ++k) own[w][k] = (uint8_t)lane;
    float st = 0.f;
    if (bf.true_idx && lane == 0) st = s[tb.qpos[l * tb.M + bf.true_idx[lb + l]]];  // (in flight meanwhile)
    __syncthreads();
    float x[C2_ST_K];
#pragma unroll
    for (int j = 0; j < C2_ST_K; ++j) {
        const int k = lane + 64 * j;
        const bool in = k < total;
        const int ad = in ? bas[w][own[w][k]] + k : 0;
        const float v = s[ad];
        x[j] = in ? v : -INFINITY;
    }
    float m = x[0];
#pragma unroll
    for (int j = 1; j < C2_ST_K; ++j) m = fmaxf(m, x[j]);
    m = c2_wave_max(m);
    float S1 = 0.f, S2 = 0.f, Se = 0.f;
#pragma unroll
    for (int j = 0; j < C2_ST_K; ++j) {  // (past the section: exp2(-inf) = 0)
        const float ex = c2_exp2((x[j] - m) * inv_tau);
        const float f = __builtin_amdgcn_fractf(ex);
        S1 += f;
        S2 += f * f;
        Se += ex;
    }
    S1 = c2_wave_sum(S1);
    S2 = c2_wave_sum(S2);
    Se = c2_wave_sum(Se);
    if (lane == 0) {
        const float ties = rintf(Se - S1) - 1.f;  // entries equal to the maximum, but one
        if (ties > 0.f) {
            S1 += ties;
            S2 += ties;
        }
        const float inv = 1.f / (1.f + S1);
        bf.stM[lb + l] = m;
        bf.stI[lb + l] = inv;
        // 1 - sum beta^2 = (2 R1 + R1^2 - R2) / (1 + R1)^2, no cancellation (as cw2_merge)
        const double i2 = (double)inv * (double)inv, r1 = S1, r2 = S2;
        double er = 0.0;
        if (bf.true_idx) {
            if (st == m) {
                er = (r1 * r1 + r2) * i2;
            } else {
                const double bt = (double)(c2_exp2((st - m) * inv_tau) * inv);
                er = (1.0 + r2) * i2 - 2.0 * bt + 1.0;
            }
        }
        reinterpret_cast<double2 *>(tb.part)[lb + l] = make_double2((2.0 * r1 + r1 * r1 - r2) * i2, er);
    }
}

// psi, NMSE and the stopping rule from the summed sections (sparc.py:973-988); thread 0
__device__ __forceinline__ void c2_psi_stop(const RegBufs<float> &bf, const AmpScalars &sc, const AmpParams &pr, int cw, int t,
                                            double denom, double a, double er) {
    if (threadIdx.x == 0) {
        double *psi = sc.psi + cw, *psi_prev = sc.psi_prev + cw;
        double *nmse = sc.nmse + (size_t)cw * pr.t_max;
        const double pnew = a / denom;
        *psi = pnew;
        nmse[t + 1] = er / denom;
        bool stop = false;
        if (t > 0 && C2_ABL == 0) {  // (ablation builds never stop early: every launch does the same work)
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

// ---------------------------------------------------------------------------- merge
__global__ __launch_bounds__(1024) void cw2_merge(Cw2Tables tb, RegBufs<float> bf, AmpScalars sc, AmpParams pr,
                                                  int t) {
    __shared__ double red[32];
    const int cw = blockIdx.x, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    const size_t lb = (size_t)cw * tb.L;
    const int Lb = tb.Lblk;
    const float inv_tau = (float)(C2_LOG2E / bf.tau[cw]);  // log2 e / tau (c2_exp2)
    double a = 0.0, er = 0.0;
    if (tid < Lb) {
        const float4 *part = tb.part + (size_t)cw * tb.np * Lb;
        float Mr = -INFINITY, R1 = 0.f, R2 = 0.f, s_true = NAN;
        float4 ph[CW2_NP];
#pragma unroll
        for (int h = 0; h < CW2_NP; ++h)  // (all requested together)
            ph[h] = h < tb.np ? part[h * Lb + tid] : make_float4(-INFINITY, 0.f, 0.f, NAN);
#pragma unroll
        for (int h = 0; h < CW2_NP; ++h) {  // the parts in order: same merge as the class merge of cw2_az
            const float4 p = ph[h];
            const float m = p.x;
            if (!(p.w != p.w)) s_true = p.w;
            if (m > -INFINITY) {
                if (m > Mr) {
                    const float f = c2_exp2((Mr - m) * inv_tau);
                    R1 = (R1 + 1.f) * f + p.y;
                    R2 = (R2 + 1.f) * (f * f) + p.z;
                    Mr = m;
                } else {
                    const float f = c2_exp2((m - Mr) * inv_tau);
                    R1 += (1.f + p.y) * f;
                    R2 += (1.f + p.z) * (f * f);
                }
            }
        }
        const float inv = 1.f / (1.f + R1);
        bf.stM[lb + tid] = Mr;
        bf.stI[lb + tid] = inv;
        // 1 - sum beta^2 = (2 R1 + R1^2 - R2) / (1 + R1)^2, no cancellation
        const double i2 = (double)inv * (double)inv, r1 = R1, r2 = R2;
        a = (2.0 * r1 + r1 * r1 - r2) * i2;
        if (bf.true_idx) {
            if (s_true == Mr) {
                er = (r1 * r1 + r2) * i2;
            } else {
                const double bt = (double)(c2_exp2((s_true - Mr) * inv_tau) * inv);
                er = (1.0 + r2) * i2 - 2.0 * bt + 1.0;
            }
        }
    }
    c2_block_sum2(a, er, red);
    c2_psi_stop(bf, sc, pr, cw, t, (double)tb.L, a, er);
}

// (C2_STATS_LAUNCH) the sections' sums of cw2_stats -> psi, NMSE, stop, in cw2_merge's summation order
__global__ __launch_bounds__(1024) void cw2_final(Cw2Tables tb, RegBufs<float> bf, AmpScalars sc, AmpParams pr,
                                                  int t) {
    __shared__ double red[32];
    const int cw = blockIdx.x, tid = threadIdx.x;
    if (!bf.active[cw]) return;
    const size_t lb = (size_t)cw * tb.L;
    double a = 0.0, er = 0.0;
    if (tid < tb.Lblk) {  // (one section per thread, the merge's summation order)
        const double2 v = reinterpret_cast<const double2 *>(tb.part)[lb + tid];
        a = v.x;
        er = v.y;
    }
    c2_block_sum2(a, er, red);
    c2_psi_stop(bf, sc, pr, cw, t, (double)tb.L, a, er);
}

// z of every codeword in natural order from its slot-order copy (cw2_ctrl keeps z in slot order only): run
// once, at a hand-over to the staged engine, whose control kernel reads z in natural order
__global__ __launch_bounds__(C2_T) void cw2_z_natural(Cw2Tables tb, RegBufs<float> bf) {
    const int cw = blockIdx.x, tid = threadIdx.x;
    const float *zs = tb.zs + (size_t)cw * tb.OT * C2_T;
    float *z = bf.z + (size_t)cw * tb.n;
    for (int j = 0; j < tb.OT; ++j)
        if (tb.ka[j * C2_T + tid] & CW_VALID) z[tb.oi[j * C2_T + tid]] = zs[j * C2_T + tid];
}

int cw2_launch_z_natural(const Cw2Tables &tb, const RegBufs<float> &bf, hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    hipLaunchKernelGGL(cw2_z_natural, dim3(bf.B), dim3(C2_T), 0, s, tb, bf);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <int OT>
static int cw2_launch(const Cw2Tables &tb, const RegBufs<float> &bf, const AmpScalars &sc, const AmpParams &pr,
                      int t, hipStream_t s) {
    const size_t lds = C2_LDS_BYTES;  // the P-point image (also the class copy: fpad(maxcls + 16) < 2 P), stM, stI
    static const int ready = []() -> int {  // the image addresses assume no static LDS (c2_at)
        hipFuncAttributes fa, fz;
        if (hipFuncGetAttributes(&fa, (const void *)cw2_ab<OT>) != hipSuccess ||
            hipFuncGetAttributes(&fz, (const void *)cw2_az<OT>) != hipSuccess || fa.sharedSizeBytes ||
            fz.sharedSizeBytes)
            return 0;
        return hipFuncSetAttribute((const void *)cw2_ab<OT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)C2_LDS_BYTES) == hipSuccess &&
               hipFuncSetAttribute((const void *)cw2_az<OT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)C2_LDS_BYTES) == hipSuccess;
    }();
    if (!ready) return fail(SG_ERR_HIP, "split per-codeword engine: kernel attributes (static LDS / LDS size)");
    const dim3 g2(tb.np * bf.B), gB(bf.B);
    if (t > 0) {
        ProfScope ps(SG_PH_CW2_AB, s);
        hipLaunchKernelGGL((cw2_ab<OT>), g2, dim3(C2_T), lds, s, tb, bf);
    }
    {
        ProfScope ps(SG_PH_CW2_CTRL, s);
        hipLaunchKernelGGL((cw2_ctrl<OT>), gB, dim3(C2_T), 0, s, tb, bf, sc, pr, t);
    }
    {
        ProfScope ps(SG_PH_CW2_AZ, s);
        hipLaunchKernelGGL((cw2_az<OT>), g2, dim3(C2_T), lds, s, tb, bf, t);
    }
    {
        ProfScope ps(SG_PH_CW2_CTRL, s);
        if (C2_STATS_LAUNCH) {
            if (tb.Lblk % 16 == 0)
                hipLaunchKernelGGL((cw2_stats<16>), dim3(bf.B * (tb.Lblk / 16)), dim3(64 * 16), 0, s, tb, bf);
            else
                hipLaunchKernelGGL((cw2_stats<4>), dim3(bf.B * (tb.Lblk / 4)), dim3(64 * 4), 0, s, tb, bf);
            hipLaunchKernelGGL((cw2_final), gB, dim3(1024), 0, s, tb, bf, sc, pr, t);
        } else {
            hipLaunchKernelGGL((cw2_merge), gB, dim3(1024), 0, s, tb, bf, sc, pr, t);
        }
    }
    return SG_OK;
}

int cw2_launch_iter(const Cw2Tables &tb, const RegBufs<float> &bf, const AmpScalars &sc, const AmpParams &pr, int t,
                    hipStream_t s) {
    if (bf.B <= 0) return SG_OK;
    if (tb.Q % 2 || tb.L > 1024 || tb.Lblk > 2 * C2_T || tb.maxcls > C2_NC * C2_SC * C2_T ||
        fpad(tb.maxcls + 16) >= 2 * C2_P || tb.N2 != C2_P * tb.Q ||
        (C2_STATS_LAUNCH && (tb.Lblk != tb.L || tb.L % 4 || tb.M > 64 * C2_ST_K || tb.Q > 64)))
        return fail(SG_ERR_UNSUPPORTED, "split per-codeword engine: sizes outside its compile-time bounds");
    ProfScope ps(SG_PH_AMP_CW, s);
    switch (tb.OT) {
    case 12: SG_TRY(cw2_launch<12>(tb, bf, sc, pr, t, s)); break;
    case 13: SG_TRY(cw2_launch<13>(tb, bf, sc, pr, t, s)); break;
    case 14: SG_TRY(cw2_launch<14>(tb, bf, sc, pr, t, s)); break;
    case 16: SG_TRY(cw2_launch<16>(tb, bf, sc, pr, t, s)); break;
    default: return fail(SG_ERR_UNSUPPORTED, "split per-codeword engine: %d outputs per thread", tb.OT);
    }
    SG_HIP(hipGetLastError());
    return SG_OK;
}

}  // namespace sg
