// Degree-grouped single-precision min-sum BP for gfx950 (the C3 path).
//
// Same decoder as bp.hip's table kernel for dectype SG_MINSUM / SG_F32
// (c_ldpc.c:339-381 with the index fix of SURVEY.md 8(c); variable sums in the
// reference's port order, c_ldpc.c:171-178), over the degree-grouped layout
// of bp.hpp BpGrpArgs built by capi_ldpc.cpp build_groups.
//
// Why a second kernel: the table kernel is bound by vector-ALU issue (SQ: ~490
// VALU and ~280 SALU instructions per wave per iteration on the C3 code, VALU
// ~86 % busy): per-lane degrees make every port loop divergent, and its check
// update carries the argmin index and per-port sign bits.  Here
//   * every group has one degree, so each wave runs straight-line code
//     unrolled for that degree (the per-wave degree is a scalar, dispatched
//     by a scalar switch);
//   * the check update is branch-free:
//       m1 = min |L|, m2 = second min  (m2 = med3(|L|, m1, m2), m1 = min(m1, |L|)),
//       S  = XOR of the raw words (its sign bit is the reference's `sall`),
//       out_k = (|L_k| == m1 ? |m2 f| : |m1 f|) with sign bit of L_k ^ S ^ f,
//     identical values to the reference: it gives m2 to its first argmin
//     only, and a tie |L_k| == m1 elsewhere means m2 == m1; and
//     (neg ? -mag : mag) * f == +-(mag * f) exactly;
//   * the stopping test is a ballot per wave and one flag word per wave in
//     LDS (double-buffered by iteration parity, so one barrier suffices), in
//     place of __syncthreads_or (whose static LDS also offset every dynamic
//     LDS address by 256 B, one add per port).
// Per group and pass one table load (vector L1) and two LDS round trips;
// 2 VALU per variable port, ~7 per check port.  Built with -fno-honor-nans: no NaN reaches the min/max (the
// channel LLRs are saturated to finite values on load, GRP_CH_MAX, and the
// messages are sums and products of them), so the compiler drops the
// canonicalisation of their operands.  A NaN channel LLR is outside the
// kernel's contract: the host entry point sends such a batch to the table
// kernel (capi_ldpc.cpp), the device entry point documents it.
#include "bp.hpp"

// one workgroup per codeword (1: the hardware dispatcher hands each finished workgroup's CU slot to the next
// codeword; a workgroup's LDS image starts uninitialised, which the first iteration's read-free variable pass
// and the per-iteration flag words allow), or a persistent grid of (workgroups per CU) x CUs looping over the
// batch (0) (A/B).  Same box, two calls (profiles/r06_bp_grid_ab.txt): C3 5.91 M -> 6.24 M and 5.94 M -> 6.34 M
// codewords/s, 0.62-0.63 -> 0.66-0.67 of the LDS bound, bit-identical
#ifndef BPG_GRID_B
#define BPG_GRID_B 1
#endif

namespace sg {

// Channel LLRs are saturated at this magnitude on load (far beyond any LLR a
// channel produces: 2y / sigma^2 ~ 1e30 needs |y| / sigma^2 ~ 5e29).  Up to 17
// terms of it still sum to a finite float, so no inf - inf reaches the
// variable pass from the input.
constexpr float GRP_CH_MAX = 1e30f;
// two check groups of one degree in a wave run together (A/B: -DBPG_CHECK_PAIRS=1; same box within noise,
// profiles/r05_bp_ab.txt, and it spills a VGPR in the codeword loop: off)
#ifndef BPG_CHECK_PAIRS
#define BPG_CHECK_PAIRS 0
#endif
// Wave issue priority of the variable and the check pass.  Four workgroups share a CU, each pass a chain
// of table / LDS round trips between two barriers; the check pass at 1 over the variable pass at 0:
// 0.694 / 0.701 / 0.685 -> 0.659 / 0.661 / 0.654 ms per launch at 1.0 / 1.5 / 2.0 dB, same box, bit-identical
// (check pass at 2 or 3, or variable pass at 1 under a check pass at 2, within noise of it:
// profiles/r05_prio_ab.txt).  Both equal: flat, for the A/B.
#ifndef BPG_PRIO_V
#define BPG_PRIO_V 0
#endif
#ifndef BPG_PRIO_C
#define BPG_PRIO_C 1
#endif
#ifndef BPG_SETUP_BATCH
#define BPG_SETUP_BATCH 0
#endif

// LDS words addressed by their byte address.  The kernel has no static LDS
// (grouped_one checks), so its dynamic image starts at address 0 and the
// table's slot addresses are used as they are: through the dynamic-LDS symbol
// the compiler adds its (relocated, zero) base to every slot address, one VALU
// per port.
typedef __attribute__((address_space(3))) float lds_f32;
__device__ __forceinline__ lds_f32 *ldsf(uint32_t byte) { return (lds_f32 *)(size_t)byte; }

// Variable group of degree D: the lane's slot addresses straight from the
// global port table (gtab = the lane's entry; the table is L1-resident and
// shared by the CU's workgroups, so the LDS holds only the messages), then the
// reference's sum in port order and the extrinsic write-backs.
// F2: first2 holds the slot addresses of the first two ports (low, high half)
// in a register for the whole decode, so a degree-2 group reads no table at
// all (the <4, 2> kernel; at <8, 4> the eight registers would spill)
// init: the first iteration, whose incoming messages are all zero (the
// reference starts from zero messages): nothing is read and the same sums of
// zeros are formed (acc = ch + 0 + ... turns a -0 channel value into +0, as
// the reference's does), so the image needs no zeroing before a codeword.
template <int D, bool F2>
__device__ __forceinline__ float grp_var(const uint16_t *gtab, float acc, uint32_t first2, bool init) {
    if constexpr (D == 0) {
        return acc;
    } else {
        uint32_t sl[D];
        float m[D];
#pragma unroll
        for (int k = 0; k < D; ++k)
            sl[k] = (F2 && k == 0) ? (first2 & 0xffffu) : (F2 && k == 1) ? (first2 >> 16) : (uint32_t)gtab[64 * k];
        if (init) {  // (uniform)
#pragma unroll
            for (int k = 0; k < D; ++k) m[k] = 0.0f;
        } else {
#pragma unroll
            for (int k = 0; k < D; ++k) m[k] = *ldsf(sl[k]);
        }
#pragma unroll
        for (int k = 0; k < D; ++k) acc += m[k];
#pragma unroll
        for (int k = 0; k < D; ++k) *ldsf(sl[k]) = acc - m[k];
        return acc;
    }
}

// Two variable groups of one degree D run together: both groups' table
// loads, then both groups' LDS reads, are in flight at once (one chain of
// round trips for the pair instead of two).  Each variable still sums its
// ports in the reference's order.
template <int D, bool F2>
__device__ __forceinline__ void grp_var2(const uint16_t *gt0, const uint16_t *gt1, float &acc0, float &acc1,
                                         uint32_t f0, uint32_t f1, bool init) {
    uint32_t s0[D], s1[D];
    float m0[D], m1[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        s0[k] = (F2 && k == 0) ? (f0 & 0xffffu) : (F2 && k == 1) ? (f0 >> 16) : (uint32_t)gt0[64 * k];
        s1[k] = (F2 && k == 0) ? (f1 & 0xffffu) : (F2 && k == 1) ? (f1 >> 16) : (uint32_t)gt1[64 * k];
    }
    if (init) {  // (uniform)
#pragma unroll
        for (int k = 0; k < D; ++k) m0[k] = m1[k] = 0.0f;
    } else {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            m0[k] = *ldsf(s0[k]);
            m1[k] = *ldsf(s1[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < D; ++k) {
        acc0 += m0[k];
        acc1 += m1[k];
    }
#pragma unroll
    for (int k = 0; k < D; ++k) {
        *ldsf(s0[k]) = acc0 - m0[k];
        *ldsf(s1[k]) = acc1 - m1[k];
    }
}

template <bool F2>
__device__ __forceinline__ void grp_var2_d(int d, const uint16_t *gt0, const uint16_t *gt1, float &acc0,
                                           float &acc1, uint32_t f0, uint32_t f1, bool init) {
    static_assert(GRP_PAIR_MAXD == 3, "pair degrees");
    switch (d) {
        case 1: grp_var2<1, F2>(gt0, gt1, acc0, acc1, f0, f1, init); break;
        case 2: grp_var2<2, F2>(gt0, gt1, acc0, acc1, f0, f1, init); break;
        case 3: grp_var2<3, F2>(gt0, gt1, acc0, acc1, f0, f1, init); break;
        default: break;  // (the host pairs degrees 1..GRP_PAIR_MAXD only)
    }
}

template <int DC>
__device__ __forceinline__ uint32_t grp_check(uint32_t addr, float factor, uint32_t fsign) {
    float L[DC];
    lds_f32 *c = ldsf(addr);
#pragma unroll
    for (int k = 0; k < DC; ++k) L[k] = c[64 * k];
    float m1 = INFINITY, m2 = INFINITY;
    uint32_t S = 0u;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const float a = fabsf(L[k]);
        m2 = __builtin_amdgcn_fmed3f(a, m1, m2);  // second smallest of {m1 <= m2, a}
        m1 = fminf(m1, a);
        S ^= __float_as_uint(L[k]);
    }
    const uint32_t unsat = (S >> 31) | (m1 > 0.0f ? 0u : 1u);
    // magnitudes of the two outputs, materialised once per check (kept out of
    // the per-port select)
    uint32_t b1 = __float_as_uint(m1 * factor) & 0x7fffffffu, b2 = __float_as_uint(m2 * factor) & 0x7fffffffu;
    asm volatile("" : "+v"(b1), "+v"(b2));
    const uint32_t Sf = S ^ fsign;
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        const uint32_t mag = fabsf(L[k]) == m1 ? b2 : b1;
        c[64 * k] = __uint_as_float(((__float_as_uint(L[k]) ^ Sf) & 0x80000000u) | mag);
    }
    return unsat;
}

// Two check groups of one degree DC together: both groups' LDS reads in flight
// at once, then both updates (one chain of round trips for the pair).  Each
// check's update is grp_check's, operation for operation.
template <int DC>
__device__ __forceinline__ uint32_t grp_check2(uint32_t addr0, uint32_t addr1, float factor, uint32_t fsign,
                                               bool valid0, bool valid1) {
    float L0[DC], L1[DC];
    lds_f32 *c0 = ldsf(addr0), *c1 = ldsf(addr1);
#pragma unroll
    for (int k = 0; k < DC; ++k) {
        L0[k] = c0[64 * k];
        L1[k] = c1[64 * k];
    }
    uint32_t u = 0u;
    auto upd = [&](float *L, lds_f32 *c, bool valid) {
        float m1 = INFINITY, m2 = INFINITY;
        uint32_t S = 0u;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            const float a = fabsf(L[k]);
            m2 = __builtin_amdgcn_fmed3f(a, m1, m2);
            m1 = fminf(m1, a);
            S ^= __float_as_uint(L[k]);
        }
        const uint32_t unsat = (S >> 31) | (m1 > 0.0f ? 0u : 1u);
        uint32_t b1 = __float_as_uint(m1 * factor) & 0x7fffffffu, b2 = __float_as_uint(m2 * factor) & 0x7fffffffu;
        asm volatile("" : "+v"(b1), "+v"(b2));
        const uint32_t Sf = S ^ fsign;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
            const uint32_t mag = fabsf(L[k]) == m1 ? b2 : b1;
            c[64 * k] = __uint_as_float(((__float_as_uint(L[k]) ^ Sf) & 0x80000000u) | mag);
        }
        u |= valid ? unsat : 0u;
    };
    upd(L0, c0, valid0);
    upd(L1, c1, valid1);
    return u;
}

__device__ __forceinline__ uint32_t grp_check2_d(int d, uint32_t a0, uint32_t a1, float f, uint32_t fs, bool v0,
                                                 bool v1) {
    switch (d) {
#define SG_GC2(N) case N: return grp_check2<N>(a0, a1, f, fs, v0, v1);
        SG_GC2(2) SG_GC2(3) SG_GC2(4) SG_GC2(5) SG_GC2(6) SG_GC2(7)
#undef SG_GC2
        default: return 0u;
    }
}

// uniform (per-wave) degree dispatch
template <bool F2>
__device__ __forceinline__ float grp_var_d(int d, const uint16_t *gtab, float acc, uint32_t first2, bool init) {
    switch (d) {
#define SG_GV(N) case N: return grp_var<N, F2>(gtab, acc, first2, init);
        SG_GV(0) SG_GV(1) SG_GV(2) SG_GV(3) SG_GV(4) SG_GV(5) SG_GV(6) SG_GV(7) SG_GV(8)
        SG_GV(9) SG_GV(10) SG_GV(11) SG_GV(12) SG_GV(13) SG_GV(14) SG_GV(15) SG_GV(16)
#undef SG_GV
        default: return acc;  // (the host admits degrees <= GRP_MAXDV only)
    }
}
__device__ __forceinline__ uint32_t grp_check_d(int d, uint32_t addr, float f, uint32_t fs) {
    switch (d) {
#define SG_GC(N) case N: return grp_check<N>(addr, f, fs);
        SG_GC(2) SG_GC(3) SG_GC(4) SG_GC(5) SG_GC(6) SG_GC(7) SG_GC(8)
#undef SG_GC
        default: return 0u;
    }
}

// LDS image: [msg_bytes) messages + trash slot, then [2][GRP_WAVES] u32 stop
// flags (GRP_FLAG_BYTES).

// meta layout: [0] vdeg[W][VJ], [1] vtab (byte address)[W][VJ],
// [2] cdeg[W][CJ], [3] caddr (byte address)[W][CJ], [4] cvalid lanes[W][CJ]
// The LDS image is the messages and flags only (the port table is read from
// global memory through L1; staging it in LDS measured 7 % slower: three
// workgroups per CU instead of four), so four workgroups share a CU at
// <4, 2> (8 waves per SIMD, <= 64 VGPRs); <8, 4> needs more registers.
template <int VJ, int CJ>
__global__ __launch_bounds__(BP_THREADS, VJ <= 4 ? 8 : 6) void bp_grouped_minsum_kernel(BpGrpArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint32_t *flags = reinterpret_cast<uint32_t *>(smem + a.msg_bytes);
    // per-wave group parameters are uniform (scalar registers); the lanes'
    // offsets are added at the use
    const int32_t *mv = a.meta + wave * VJ;
    const int32_t *mc = a.meta + 2 * GRP_WAVES * VJ + wave * CJ;
    int vd[VJ];
    uint32_t vt[VJ];
    bool vpair[VJ];  // groups j and j + 1 (j even) run as a pair (GRP_PAIR)
#pragma unroll
    for (int j = 0; j < VJ; ++j) {
        const int w = __builtin_amdgcn_readfirstlane(mv[j]);
        vd[j] = w & (GRP_PAIR - 1);
        vpair[j] = (j & 1) == 0 && (w & GRP_PAIR) != 0;
        vt[j] = (uint32_t)__builtin_amdgcn_readfirstlane(mv[GRP_WAVES * VJ + j]) >> 1;  // table entry
    }
    int cdg[CJ], cn[CJ];
    uint32_t ca[CJ];
#pragma unroll
    for (int q = 0; q < CJ; ++q) {
        cdg[q] = __builtin_amdgcn_readfirstlane(mc[q]);
        ca[q] = (uint32_t)__builtin_amdgcn_readfirstlane(mc[GRP_WAVES * CJ + q]);
        cn[q] = __builtin_amdgcn_readfirstlane(mc[2 * GRP_WAVES * CJ + q]);
    }
    const int32_t *vmap = a.vmap + wave * VJ * 64 + lane;
    constexpr bool F2 = VJ <= 4;
    uint32_t first2[VJ];  // slot addresses of each variable group's first two ports (grp_var)
#pragma unroll
    for (int j = 0; j < VJ; ++j) {
        const uint16_t *gt = a.vtab + vt[j] + lane;
        first2[j] = !F2 ? 0u
                        : (j < a.vj && vd[j] >= 1 ? (uint32_t)gt[0] : 0u) |
                              (j < a.vj && vd[j] >= 2 ? (uint32_t)gt[64] << 16 : 0u);
    }
    const float factor = a.factor;
    const uint32_t fsign = __float_as_uint(factor) & 0x80000000u;
    for (int cw = blockIdx.x; cw < a.B; cw += gridDim.x) {
        const float *ch = a.ch + (size_t)cw * a.nv;
        float chv[VJ], apv[VJ];
        {
            // the lanes' variables, then their channel values, each in one round of loads (padding lanes read
            // variable 0 and drop it); the zero offset is opaque so the codeword-invariant index loads are not
            // hoisted out of the codeword loop (live across the decode they would not fit the 64 VGPRs)
            int zo = 0;
            asm volatile("" : "+v"(zo));
#if BPG_SETUP_BATCH
            // raw buffer loads, no branch: a padding lane (variable -1) reads past the buffer's end, which the
            // hardware range check returns as 0
            const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<int32_t *>(a.vmap + wave * VJ * 64), 0, 4 * 64 * VJ, 0x00020000);
            const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(ch), 0,
                                                                                4 * a.nv, 0x00020000);
            int v[VJ];
#pragma unroll
            for (int j = 0; j < VJ; ++j)
                v[j] = j < a.vj ? (int)__builtin_amdgcn_raw_buffer_load_b32(rm, 4 * (lane + zo), 4 * 64 * j, 0) : -1;
#pragma unroll
            for (int j = 0; j < VJ; ++j) {
                // saturated at +-GRP_CH_MAX (and inf with it): the kernel is built
                // without NaN semantics, and a sum of saturated inputs stays finite
                const float x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rc, 4 * v[j], 0, 0));
                chv[j] = __builtin_amdgcn_fmed3f(x, -GRP_CH_MAX, GRP_CH_MAX);
                apv[j] = 0.0f;
            }
#else
#pragma unroll
            for (int j = 0; j < VJ; ++j) {
                const int v = j < a.vj ? vmap[64 * j + zo] : -1;
                chv[j] = v >= 0 ? __builtin_amdgcn_fmed3f(ch[v], -GRP_CH_MAX, GRP_CH_MAX) : 0.0f;
                apv[j] = 0.0f;
            }
#endif
        }
        // ---- variable pass (c_ldpc.c:171-178): groups 2i and 2i + 1 as a pair
        // when the host flagged one (pairs sit at even positions)
        auto var_pass = [&](bool init) {
#pragma unroll
            for (int j = 0; j < VJ; j += 2) {
                if (j >= a.vj) continue;
                if (vpair[j]) {
                    float a0 = chv[j], a1 = chv[j + 1];
                    grp_var2_d<F2>(vd[j], a.vtab + vt[j] + lane, a.vtab + vt[j + 1] + lane, a0, a1, first2[j],
                                   first2[j + 1], init);
                    apv[j] = a0;
                    apv[j + 1] = a1;
                } else {
                    apv[j] = grp_var_d<F2>(vd[j], a.vtab + vt[j] + lane, chv[j], first2[j], init);
                    if (j + 1 < a.vj)
                        apv[j + 1] = grp_var_d<F2>(vd[j + 1], a.vtab + vt[j + 1] + lane, chv[j + 1], first2[j + 1],
                                                   init);
                }
            }
        };
        // (the previous codeword's last reads of the image and of the flags are behind the barrier that
        // ended it)
        int it = 0;
        for (; it < a.max_it; ++it) {
            if (BPG_PRIO_V != BPG_PRIO_C) __builtin_amdgcn_s_setprio(BPG_PRIO_V);
            var_pass(it == 0);  // (the first: zero incoming messages, no reads, no zeroed image)
            if (BPG_PRIO_V != BPG_PRIO_C) __builtin_amdgcn_s_setprio(BPG_PRIO_C);
            __syncthreads();
            // ---- check pass (c_ldpc.c:183-194 with the min-sum update)
            uint32_t unsat = 0u;
#pragma unroll
            for (int q = 0; q < CJ; q += 2) {
                if (q >= a.cj) continue;
                if (BPG_CHECK_PAIRS && q + 1 < a.cj && cdg[q + 1] == cdg[q] && cdg[q] <= 7) {  // (uniform; degree 8 pairs spill)
                    unsat |= grp_check2_d(cdg[q], ca[q] + 4 * lane, ca[q + 1] + 4 * lane, factor, fsign,
                                          lane < cn[q], lane < cn[q + 1]);
                } else {
                    const uint32_t u = grp_check_d(cdg[q], ca[q] + 4 * lane, factor, fsign);
                    unsat |= lane < cn[q] ? u : 0u;
                    if (q + 1 < a.cj) {
                        const uint32_t u1 = grp_check_d(cdg[q + 1], ca[q + 1] + 4 * lane, factor, fsign);
                        unsat |= lane < cn[q + 1] ? u1 : 0u;
                    }
                }
            }
            // ---- stop when every check is satisfied (c_ldpc.c:196-197): one
            // flag per wave, parity-buffered (this iteration's words were last
            // read before the previous iteration's variable-pass barrier)
            const uint32_t any = __ballot(unsat != 0u) != 0ull ? 1u : 0u;
            uint32_t *fl = flags + (it & 1) * GRP_WAVES;
            fl[wave] = any;
            __syncthreads();
            const uint4 f0 = *reinterpret_cast<const uint4 *>(fl);
            const uint4 f1 = *reinterpret_cast<const uint4 *>(fl + 4);
            if (((f0.x | f0.y | f0.z | f0.w) | (f1.x | f1.y | f1.z | f1.w)) == 0u) break;
        }
        float *out = a.app + (size_t)cw * a.nv;
#pragma unroll
        for (int j = 0; j < VJ; ++j) {
            const int v = j < a.vj ? vmap[64 * j] : -1;
            if (v >= 0) out[v] = apv[j];
        }
        if (tid == 0) a.it[cw] = it;
        __syncthreads();
    }
}

static size_t grouped_lds(const BpGrpArgs &a) { return (size_t)a.msg_bytes + GRP_FLAG_BYTES; }

template <int VJ, int CJ>
static int grouped_one(const BpGrpArgs &a, hipStream_t s) {
    auto kern = bp_grouped_minsum_kernel<VJ, CJ>;
    const size_t lds = grouped_lds(a);
    static const size_t static_lds = [&] {
        hipFuncAttributes fa;
        return hipFuncGetAttributes(&fa, (const void *)kern) == hipSuccess ? (size_t)fa.sharedSizeBytes : (size_t)-1;
    }();
    if (static_lds != 0)  // the slot addresses assume the dynamic image at LDS address 0
        return fail(SG_ERR_UNSUPPORTED, "grouped BP kernel has static LDS (%zu B)", static_lds);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, BP_THREADS, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    int grid = per_cu * device_cu_count();
    if (BPG_GRID_B || grid > a.B) grid = a.B;
    if (lds > 64 * 1024)
        SG_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    ProfScope ps(SG_PH_BP, s);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BP_THREADS), lds, s, a);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

int bp_grouped_launch(const BpGrpArgs &a, hipStream_t s) {
    if (a.msg_bytes > 65536 || a.msg_bytes % 16 || grouped_lds(a) > BP_MAX_LDS || a.vj < 1 || a.cj < 1 ||
        a.vj > 8 || a.cj > 4)
        return fail(SG_ERR_INVALID, "grouped BP layout out of range (msg %d B, table %d, %d/%d groups per wave)",
                    a.msg_bytes, a.ntab, a.vj, a.cj);
    if (a.B <= 0) return SG_OK;
    if (grp_kvj(a.vj, a.cj) == 4) return grouped_one<4, 2>(a, s);
    return grouped_one<8, 4>(a, s);
}

}  // namespace sg
