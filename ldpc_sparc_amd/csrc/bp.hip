// Batched flooding belief propagation for QC-LDPC Tanner graphs on gfx950.
//
// Replaces the reference's per-codeword C loop (ldpc_jossy/src/c_ldpc.c:
// sumprod :32-113, sumprod2 :138-206 with Lxfb :294-314 / Lxor :234-251,
// minsum :339-381) that ldpc.py:463-490 and sparc_new.py:1176-1179 call once
// per 1944-bit block.
//
// Design (DESIGN.md "BP kernel"):
//   * one workgroup decodes one codeword at a time: one workgroup per codeword
//     for single-precision min-sum, persistent over the batch otherwise
//     (grid = occupancy x CUs, codewords pulled by blockIdx stride; BPF_GRID_B);
//   * the whole message state of the codeword lives in LDS for all
//     iterations: HBM sees only the channel LLRs (read once per iteration
//     through L2) and the final a-posteriori LLRs;
//   * messages are stored check-port-major, slot(c, k) = k * nc + c, so the
//     check pass (thread = check) reads and writes contiguous LDS words across
//     the wavefront (conflict-free); the variable pass reaches its ports
//     through the port->slot table (the reference's intrlv composed with
//     this layout, built on the host in capi.cpp);
//   * per-codeword early stop exactly as the reference (every check aggregate
//     > 0 after the check pass); the iteration index that stopped is returned.
//
// Arithmetic order follows the reference so that the double-precision min-sum
// decoder is bit-identical to the corrected reference (exact min/sign
// algebra, one multiply by the factor), and sum-product variants differ only
// by the last-ulp behaviour of the device exp/log/tanh.  This file is built
// with -ffp-contract=off.
#include <algorithm>

#include "bp.hpp"

// table kernels, single-precision min-sum: one workgroup per codeword (1), or a persistent grid of (workgroups
// per CU) x CUs looping over the batch with the graph tables staged once per workgroup (0) (A/B).  Same box
// (profiles/r06_bp_grid_ab.txt): 802.11n r5/6 z = 81 (the lean kernel) 6.54 M -> 7.07 M codewords/s; the
// double-precision sum-product kernels lose 6 % with it (their table staging per codeword), so they stay
// persistent
#ifndef BPF_GRID_B
#define BPF_GRID_B 1
#endif

namespace sg {

// ports per round of the variable pass, and the padding of the LDS port
// table that lets a round read past the last variable's ports
#ifndef BP_VU
#define BP_VU 2
#endif
constexpr int BP_PS_PAD = 2;

// Single-precision min-sum: the check pass at issue priority 1 over the variable pass at 0 (the grouped
// kernel's scheme; three workgroups share a CU): 1.456 -> 1.392 ms per launch on the C3 code (table kernel
// forced), bit-identical.  Double-precision sumprod2 measured 1 % slower with it, so the other kinds stay
// flat (profiles/r05_prio_ab.txt).  0: flat for every kind (A/B).
#ifndef BPF_PRIO
#define BPF_PRIO 1
#endif
template <typename T>
__device__ __forceinline__ T dev_log(T x);
template <>
__device__ __forceinline__ double dev_log<double>(double x) { return log(x); }
template <>
__device__ __forceinline__ float dev_log<float>(float x) { return __logf(x); }
template <typename T>
__device__ __forceinline__ T dev_exp(T x);
template <>
__device__ __forceinline__ double dev_exp<double>(double x) { return exp(x); }
template <>
__device__ __forceinline__ float dev_exp<float>(float x) { return __expf(x); }

// Pairwise XOR-LLR (reference Lxor, c_ldpc.c:234-251).
template <typename T, bool CORR>
__device__ __forceinline__ T lxor(T a, T b) {
    const bool same = (signbit(a) != 0) == (signbit(b) != 0);
    T out = (same ? T(1) : T(-1)) * fmin(fabs(a), fabs(b));
    if (CORR) {
        out += dev_log<T>(T(1) + dev_exp<T>(-fabs(a + b)));
        out -= dev_log<T>(T(1) + dev_exp<T>(-fabs(a - b)));
    }
    return out;
}

template <typename T, int MAXDC>
__device__ __forceinline__ void check_load(const T *__restrict__ msg, int c, int nc, int d, T *L) {
#pragma unroll
    for (int k = 0; k < MAXDC; ++k)
        if (k < d) L[k] = msg[k * nc + c];
}

// check node update from the check's incoming messages L (check_load)
template <typename T, int KIND, int MAXDC>
__device__ __forceinline__ bool check_update_from(T *__restrict__ msg, int c, int nc, int d, T factor, T *L) {
    bool unsat = false;
    if (KIND == SG_MINSUM) {
        // Compressed form of Lxfb(.., corr=0): |out_k| = min over the others,
        // sign(out_k) = XOR of the others' sign bits; both exact, so this is
        // bit-identical to the forward/backward trellis.
        T m1 = T(INFINITY), m2 = T(INFINITY);
        int i1 = -1;
        unsigned sgn = 0u, sall = 0u;
#pragma unroll
        for (int k = 0; k < MAXDC; ++k) {
            if (k < d) {
                const T a = fabs(L[k]);
                const unsigned s = signbit(L[k]) ? 1u : 0u;
                sgn |= s << k;
                sall ^= s;
                if (a < m1) { m2 = m1; m1 = a; i1 = k; }
                else if (a < m2) { m2 = a; }
            }
        }
        // aggregate b[0] = (+/-) m1; "aggr <= 0" <=> negative or zero
        unsat = (sall != 0u) || !(m1 > T(0));
#pragma unroll
        for (int k = 0; k < MAXDC; ++k) {
            if (k < d) {
                const T mag = (k == i1) ? m2 : m1;
                const bool neg = (sall ^ ((sgn >> k) & 1u)) != 0u;
                msg[k * nc + c] = (neg ? -mag : mag) * factor;
            }
        }
    } else if (KIND == SG_SUMPROD2) {
        T f[MAXDC], b[MAXDC];
        f[0] = L[0];
#pragma unroll
        for (int k = 1; k < MAXDC; ++k)
            if (k < d) f[k] = lxor<T, true>(f[k - 1], L[k]);
#pragma unroll
        for (int p = MAXDC - 1; p >= 0; --p) {
            if (p == d - 1) b[p] = L[p];
            else if (p < d - 1) b[p] = lxor<T, true>(b[p + 1 < MAXDC ? p + 1 : p], L[p]);
        }
        unsat = !(b[0] > T(0));
#pragma unroll
        for (int k = 0; k < MAXDC; ++k) {
            if (k < d) {
                T out;
                if (k == 0) out = b[MAXDC > 1 ? 1 : 0];
                else if (k == d - 1) out = f[k > 0 ? k - 1 : 0];
                else out = lxor<T, true>(f[k > 0 ? k - 1 : 0], b[k + 1 < MAXDC ? k + 1 : k]);
                msg[k * nc + c] = out;
            }
        }
    } else {  // SG_SUMPROD: tanh product, quotient, atanh (c_ldpc.c:76-102)
        T prod = T(1);
#pragma unroll
        for (int k = 0; k < MAXDC; ++k)
            if (k < d) { L[k] = tanh(L[k] / T(2)); prod *= L[k]; }
        unsat = (T(2) * atanh(prod)) <= T(0);
#pragma unroll
        for (int k = 0; k < MAXDC; ++k)
            if (k < d) msg[k * nc + c] = T(2) * atanh(prod / L[k]);
    }
    return unsat;
}

template <typename T, int KIND, int MAXDC>
__device__ __forceinline__ bool check_update(T *__restrict__ msg, int c, int nc, int d, T factor) {
    T L[MAXDC];
    check_load<T, MAXDC>(msg, c, nc, d, L);
    return check_update_from<T, KIND, MAXDC>(msg, c, nc, d, factor, L);
}

// Register-lean check update for high check degrees and double precision:
// no per-port register arrays (they spilled: T L[MAXDC], f[MAXDC], b[MAXDC]).
// The message slots themselves hold what a second pass needs; sum-product
// (Lxfb) keeps its backward values b[k+1] in an LDS scratch image laid out
// like the messages (scr[k * nc + c]), so every access stays conflict-free.
// Same arithmetic, in the same order, as check_update.
template <typename T, int KIND>
__device__ __forceinline__ bool check_update_lean(T *__restrict__ msg, T *__restrict__ scr, int c, int nc, int d,
                                                  T factor) {
    bool unsat = false;
    if (KIND == SG_MINSUM) {
        T m1 = T(INFINITY), m2 = T(INFINITY);
        int i1 = -1;
        unsigned sgn = 0u, sall = 0u;
        for (int k = 0; k < d; ++k) {
            const T x = msg[k * nc + c];
            const T a = fabs(x);
            const unsigned sb = signbit(x) ? 1u : 0u;
            sgn |= sb << k;
            sall ^= sb;
            if (a < m1) { m2 = m1; m1 = a; i1 = k; }
            else if (a < m2) { m2 = a; }
        }
        unsat = (sall != 0u) || !(m1 > T(0));
        for (int k = 0; k < d; ++k) {
            const T mag = (k == i1) ? m2 : m1;
            const bool neg = (sall ^ ((sgn >> k) & 1u)) != 0u;
            msg[k * nc + c] = (neg ? -mag : mag) * factor;
        }
    } else if (KIND == SG_SUMPROD2) {
        // backward values b[k] = Lxor(b[k+1], L[k]); b[k+1] kept for port k
        T b = msg[(d - 1) * nc + c];
        for (int k = d - 2; k >= 0; --k) {
            scr[(k + 1) * nc + c] = b;
            b = lxor<T, true>(b, msg[k * nc + c]);
        }
        unsat = !(b > T(0));  // b[0], the aggregate
        // forward values f[k] = Lxor(f[k-1], L[k]); port k gets Lxor(f[k-1], b[k+1])
        T f = msg[c];
        msg[c] = scr[nc + c];  // L[0] = b[1]
        for (int k = 1; k < d - 1; ++k) {
            const T Lk = msg[k * nc + c];
            msg[k * nc + c] = lxor<T, true>(f, scr[(k + 1) * nc + c]);
            f = lxor<T, true>(f, Lk);
        }
        msg[(d - 1) * nc + c] = f;  // L[d-1] = f[d-2]
    } else {  // SG_SUMPROD: the slots hold tanh(L/2) between the passes
        T prod = T(1);
        for (int k = 0; k < d; ++k) {
            const T t = tanh(msg[k * nc + c] / T(2));
            msg[k * nc + c] = t;
            prod *= t;
        }
        unsat = (T(2) * atanh(prod)) <= T(0);
        for (int k = 0; k < d; ++k) msg[k * nc + c] = T(2) * atanh(prod / msg[k * nc + c]);
    }
    return unsat;
}

// Kernels that take the lean path: double precision, and check degrees above 8
template <typename T, int MAXDC>
constexpr bool bp_lean() { return sizeof(T) == 8 || MAXDC > 8; }

// LDS image of one workgroup: the messages of its current codeword and --
// loaded once per workgroup -- the port -> slot table (16-bit) and the check
// degrees, so the per-iteration passes never leave LDS.  The channel LLRs,
// the app and the port range of the thread's variables (v = tid +
// BP_THREADS j) stay in registers.
template <typename T>
size_t bp_lds_bytes(int slots, int nv, int nports, int nc, bool scratch = false) {
    size_t b = sizeof(T) * (size_t)slots * (scratch ? 2 : 1);
    b += sizeof(uint16_t) * ((size_t)nports + BP_PS_PAD) + nc;
    return (b + 15) / 16 * 16;
}

// waves per SIMD the register allocation must allow: three 512-thread
// workgroups per CU (80 VGPRs) for single-precision min-sum, whose LDS image
// of an 802.11n z=81 graph is 50 KB; two (128 VGPRs) for the rest, whose
// transcendental check nodes would spill at 80
template <typename T, int KIND>
constexpr int bp_waves_per_simd() { return (sizeof(T) == 4 && KIND == SG_MINSUM) ? 6 : 4; }

template <typename T, int KIND, int MAXDC, int VJ>
__global__ __launch_bounds__(BP_THREADS, (bp_waves_per_simd<T, KIND>())) void bp_flood_kernel(BpArgs<T> a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr bool LEAN = bp_lean<T, MAXDC>();
    constexpr bool SCR = LEAN && KIND == SG_SUMPROD2;
    T *msg = reinterpret_cast<T *>(smem);
    T *scr = msg + (SCR ? a.slots : 0);                         // Lxfb backward values (lean sumprod2)
    uint16_t *ps = reinterpret_cast<uint16_t *>(msg + (SCR ? 2 : 1) * a.slots);  // variable port -> message slot
    uint8_t *cd = reinterpret_cast<uint8_t *>(ps + a.nports + BP_PS_PAD);  // check degrees
    const int tid = threadIdx.x;
    for (int i = tid; i < a.nports + BP_PS_PAD; i += BP_THREADS) ps[i] = i < a.nports ? (uint16_t)a.port_slot[i] : 0;
    for (int i = tid; i < a.nc; i += BP_THREADS) cd[i] = a.cdeg[i];
    // the port range of the thread's variables, constant over iterations and
    // codewords: held in registers (no offset-table round trip per iteration)
    // (first port | degree << 16; nports <= 65535 and degrees < 2^16 by bp_launch)
    constexpr bool R0 = !LEAN && VJ <= 4;  // first two ports' slots in registers too
    uint32_t vpd[VJ];
    uint32_t vs01[R0 ? VJ : 1];  // message slots of the first two ports, packed
#pragma unroll
    for (int j = 0; j < VJ; ++j) {
        const int v = tid + j * BP_THREADS;
        const int p0 = v < a.nv ? (int)a.voff[v] : 0;
        const int d = v < a.nv ? (int)a.voff[v + 1] - p0 : 0;
        vpd[j] = (uint32_t)p0 | ((uint32_t)d << 16);
        if constexpr (R0) {
            const uint32_t s0 = d > 0 ? (uint32_t)a.port_slot[p0] : 0u;
            const uint32_t s1 = d > 1 ? (uint32_t)a.port_slot[p0 + 1] : 0u;
            vs01[j] = s0 | (s1 << 16);
        }
    }
    for (int cw = blockIdx.x; cw < a.B; cw += gridDim.x) {
        const T *ch = a.ch + (size_t)cw * a.nv;
        T chv[VJ], apv[VJ];
#pragma unroll
        for (int j = 0; j < VJ; ++j) {
            const int v = tid + j * BP_THREADS;
            chv[j] = v < a.nv ? ch[v] : T(0);
            apv[j] = T(0);
        }
        for (int i = tid; i < a.slots; i += BP_THREADS) msg[i] = T(0);
        __syncthreads();
        int it = 0;
        for (; it < a.max_it; ++it) {
            // ---- variable pass (c_ldpc.c:171-178): two loops over the ports, the
            // second re-reading the slots (holding them in per-port register
            // arrays unrolled to the maximum degree measured 5 % slower: divergent
            // branches and their exec-mask bookkeeping)
#pragma unroll
            for (int j = 0; j < VJ; ++j) {
                const int v = tid + j * BP_THREADS;
                if (v >= a.nv) continue;
                const int p0 = (int)(vpd[j] & 0xffffu), d = (int)(vpd[j] >> 16);
                T acc = chv[j];
                if constexpr (BP_VU == 2) {
                    // two ports per round: their table and message reads issued
                    // together (one LDS round trip per round instead of per port);
                    // a round may read one padded table entry past d, which is not
                    // used; acc takes the ports in order (c_ldpc.c:171-178).  The
                    // check-degree <= 8 kernels at 4 variables a thread take the
                    // first round's slots from registers (vs01): C3 +10 %, but the
                    // high-degree (lean) kernels measured slower with it
                    const int s0 = R0 ? (int)(vs01[R0 ? j : 0] & 0xffffu) : 0;
                    const int s1 = R0 ? (int)(vs01[R0 ? j : 0] >> 16) : 0;
                    T m0 = T(0), m1 = T(0);  // (only this thread touches its ports' slots in this pass)
                    if constexpr (R0) {
                        m0 = msg[s0];
                        m1 = msg[s1];
                        acc = d > 0 ? acc + m0 : acc;
                        acc = d > 1 ? acc + m1 : acc;
                    }
                    for (int k = R0 ? 2 : 0; k < d; k += 2) {
                        const int sa = ps[p0 + k], sb = ps[p0 + k + 1];
                        const T ma = msg[sa], mb = msg[sb];
                        acc += ma;
                        acc = k + 1 < d ? acc + mb : acc;
                    }
                    if constexpr (R0) {
                        if (d > 0) msg[s0] = acc - m0;
                        if (d > 1) msg[s1] = acc - m1;
                    }
                    for (int k = R0 ? 2 : 0; k < d; k += 2) {
                        const int sa = ps[p0 + k], sb = ps[p0 + k + 1];
                        const T ma = msg[sa], mb = msg[sb];
                        msg[sa] = acc - ma;
                        if (k + 1 < d) msg[sb] = acc - mb;
                    }
                } else {
                    for (int k = 0; k < d; ++k) acc += msg[ps[p0 + k]];
                    for (int k = 0; k < d; ++k) {
                        const int sl = ps[p0 + k];
                        msg[sl] = acc - msg[sl];
                    }
                }
                apv[j] = acc;
            }
            if (BPF_PRIO && sizeof(T) == 4 && KIND == SG_MINSUM) __builtin_amdgcn_s_setprio(1);
            __syncthreads();
            // ---- check pass (c_ldpc.c:183-194)
            int unsat = 0;
            if constexpr (LEAN) {
                for (int c = tid; c < a.nc; c += BP_THREADS)
                    unsat |= check_update_lean<T, KIND>(msg, scr, c, a.nc, cd[c], a.factor) ? 1 : 0;
            } else if constexpr (KIND != SG_MINSUM || VJ > 4) {  // (two checks' arrays would spill)
                for (int c = tid; c < a.nc; c += BP_THREADS)
                    unsat |= check_update<T, KIND, MAXDC>(msg, c, a.nc, cd[c], a.factor) ? 1 : 0;
            } else {
                // min-sum: two checks per round, both checks' messages read before
                // either update (their LDS round trips overlap)
                for (int c = tid; c < a.nc; c += 2 * BP_THREADS) {
                    const int c1 = c + BP_THREADS;
                    const int d0 = cd[c], d1 = c1 < a.nc ? cd[c1] : 0;
                    T L0[MAXDC], L1[MAXDC];
                    check_load<T, MAXDC>(msg, c, a.nc, d0, L0);
                    check_load<T, MAXDC>(msg, c1, a.nc, d1, L1);
                    unsat |= check_update_from<T, KIND, MAXDC>(msg, c, a.nc, d0, a.factor, L0) ? 1 : 0;
                    if (d1 > 0) unsat |= check_update_from<T, KIND, MAXDC>(msg, c1, a.nc, d1, a.factor, L1) ? 1 : 0;
                }
            }
            if (BPF_PRIO && sizeof(T) == 4 && KIND == SG_MINSUM) __builtin_amdgcn_s_setprio(0);
            if (!__syncthreads_or(unsat)) break;  // c_ldpc.c:196-197
        }
        T *out = a.app + (size_t)cw * a.nv;
#pragma unroll
        for (int j = 0; j < VJ; ++j) {
            const int v = tid + j * BP_THREADS;
            if (v < a.nv) out[v] = apv[j];
        }
        if (tid == 0) a.it[cw] = it;
        __syncthreads();
    }
}

template <typename T, int KIND, int MAXDC, int VJ>
static int launch_one(const BpArgs<T> &a, size_t lds, hipStream_t s) {
    auto kern = bp_flood_kernel<T, KIND, MAXDC, VJ>;
    if (bp_lean<T, MAXDC>() && KIND == SG_SUMPROD2) {  // + the LDS scratch of the backward values
        lds = bp_lds_bytes<T>(a.slots, a.nv, a.nports, a.nc, true);
        if (lds > BP_MAX_LDS)
            return fail(SG_ERR_UNSUPPORTED, "graph needs %zu B of LDS per codeword for sum-product (> %d B)", lds,
                        BP_MAX_LDS);
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, BP_THREADS, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    int grid = per_cu * device_cu_count();
    if ((BPF_GRID_B && sizeof(T) == 4 && KIND == SG_MINSUM) || grid > a.B) grid = a.B;
    if (lds > 64 * 1024)
        SG_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    ProfScope ps(SG_PH_BP, s);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(BP_THREADS), lds, s, a);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

// variables per thread: 4 (nv <= 2048, every 802.11n code) or BP_VJ
template <typename T, int KIND, int MAXDC>
static int dispatch_vj(const BpArgs<T> &a, size_t lds, hipStream_t s) {
    if (a.nv <= 4 * BP_THREADS) return launch_one<T, KIND, MAXDC, 4>(a, lds, s);
    return launch_one<T, KIND, MAXDC, BP_VJ>(a, lds, s);
}

template <typename T, int KIND>
static int dispatch_dc(const BpArgs<T> &a, int max_cdeg, size_t lds, hipStream_t s) {
    if (max_cdeg <= 8) return dispatch_vj<T, KIND, 8>(a, lds, s);
    if (max_cdeg <= 16) return dispatch_vj<T, KIND, 16>(a, lds, s);
    if (max_cdeg <= 24) return dispatch_vj<T, KIND, 24>(a, lds, s);
    if (max_cdeg <= 32) return dispatch_vj<T, KIND, 32>(a, lds, s);
    return fail(SG_ERR_UNSUPPORTED, "check degree %d exceeds the supported maximum of 32", max_cdeg);
}

template <typename T>
int bp_launch(const BpArgs<T> &a, int dectype, int max_cdeg, hipStream_t s) {
    const size_t lds = bp_lds_bytes<T>(a.slots, a.nv, a.nports, a.nc);
    if (a.slots > 65536 || a.nports > 65535 || a.nv > BP_VJ * BP_THREADS)
        return fail(SG_ERR_UNSUPPORTED, "graph with %d variables / %d message slots / %d ports exceeds the decoder's "
                    "16-bit LDS tables or %d variables", a.nv, a.slots, a.nports, BP_VJ * BP_THREADS);
    if (lds > BP_MAX_LDS)
        return fail(SG_ERR_UNSUPPORTED,
                    "graph needs %zu B of LDS per codeword (> %d B): too large for the LDS-resident decoder",
                    lds, BP_MAX_LDS);
    if (a.B <= 0) return SG_OK;
    switch (dectype) {
        case SG_SUMPROD: return dispatch_dc<T, SG_SUMPROD>(a, max_cdeg, lds, s);
        case SG_SUMPROD2: return dispatch_dc<T, SG_SUMPROD2>(a, max_cdeg, lds, s);
        case SG_MINSUM: return dispatch_dc<T, SG_MINSUM>(a, max_cdeg, lds, s);
        default: return fail(SG_ERR_INVALID, "Decoder type unknonwn (dectype=%d)", dectype);
    }
}

template int bp_launch<float>(const BpArgs<float> &, int, int, hipStream_t);
template int bp_launch<double>(const BpArgs<double> &, int, int, hipStream_t);

// ---------------------------------------------------------------- error counts
// One wavefront per codeword: hard decision app < 0 (ldpc_awgn.py:97) against
// the transmitted bits; counts over all nv bits (ldpc_awgn.py:99) and over the
// first k systematic bits (ldpc_sparc hard decisions, sparc_new.py:1185-1187).
// At most 256 workgroups of four wavefronts loop over the batch and add their
// sums with four atomics each: with a workgroup per codeword, the 4 B
// device-scope atomics on one cache line (about 12 ns apiece, serialised)
// took 0.2 ms at B = 4096, 30 % of a C3 decode.
constexpr int BP_COUNT_WGS = 256;
template <typename T>
__global__ __launch_bounds__(256) void bp_count_kernel(const T *__restrict__ app, const uint8_t *__restrict__ x,
                                                       const int32_t *__restrict__ its, int B, int nv, int k,
                                                       unsigned long long *__restrict__ counts,
                                                       int32_t *__restrict__ per_cw) {
    __shared__ unsigned long long red[4][4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long c_all = 0, c_fe = 0, c_k = 0, c_it = 0;  // (lane 0)
    // rows of 4-element vectors when nv % 4 == 0 (16-byte app rows, 4-byte bit rows), eight vectors in flight per
    // lane: rocprofv3 27.6 -> 18.9 us per C3 step at B = 4096 (profiles/r06_bp_count_ab.txt), the counts identical
    const bool vec = sizeof(T) == 4 && (nv & 3) == 0 && ((uintptr_t)app & 15) == 0 && ((uintptr_t)x & 3) == 0;
    for (int cw = blockIdx.x * 4 + wid; cw < B; cw += gridDim.x * 4) {
        int e_all = 0, e_k = 0;
        if (vec) {
            const float4 *a4 = reinterpret_cast<const float4 *>(app + (size_t)cw * nv);
            const uchar4 *x4 = reinterpret_cast<const uchar4 *>(x + (size_t)cw * nv);
            const int n4 = nv >> 2;
            for (int b = 0; b < n4; b += 64 * 8) {
                float4 av[8];
                uchar4 xv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int q = b + u * 64 + lane;
                    av[u] = q < n4 ? a4[q] : make_float4(0.f, 0.f, 0.f, 0.f);
                    xv[u] = q < n4 ? x4[q] : make_uchar4(0, 0, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int q = b + u * 64 + lane;
                    if (q >= n4) continue;
                    const int e0 = (int)(av[u].x < 0.f) != (int)xv[u].x, e1 = (int)(av[u].y < 0.f) != (int)xv[u].y;
                    const int e2 = (int)(av[u].z < 0.f) != (int)xv[u].z, e3 = (int)(av[u].w < 0.f) != (int)xv[u].w;
                    e_all += e0 + e1 + e2 + e3;
                    const int v = 4 * q;
                    e_k += (v < k ? e0 : 0) + (v + 1 < k ? e1 : 0) + (v + 2 < k ? e2 : 0) + (v + 3 < k ? e3 : 0);
                }
            }
        } else {
            for (int v = lane; v < nv; v += 64) {
                const int hard = app[(size_t)cw * nv + v] < T(0) ? 1 : 0;
                const int err = hard != (int)x[(size_t)cw * nv + v];
                e_all += err;
                if (v < k) e_k += err;
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            e_all += __shfl_down(e_all, off, 64);
            e_k += __shfl_down(e_k, off, 64);
        }
        if (lane == 0) {
            if (per_cw) per_cw[cw] = e_all;  // bit errors of this codeword over all nv bits
            c_all += (unsigned long long)e_all;
            c_fe += e_all > 0 ? 1ull : 0ull;
            c_k += (unsigned long long)e_k;
            if (its) c_it += (unsigned long long)its[cw];
        }
    }
    if (!counts) return;
    if (lane == 0) {
        red[0][wid] = c_all;
        red[1][wid] = c_fe;
        red[2][wid] = c_k;
        red[3][wid] = c_it;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        unsigned long long t = 0;
        for (int w = 0; w < 4; ++w) t += red[threadIdx.x][w];
        atomicAdd(&counts[threadIdx.x], t);
    }
}

template <typename T>
int bp_count_launch(const T *app, const uint8_t *x, const int32_t *its, int B, int nv, int k,
                    int64_t *counts, hipStream_t s, int32_t *per_cw) {
    if (B <= 0) return SG_OK;
    const int wgs = std::min((B + 3) / 4, BP_COUNT_WGS);
    hipLaunchKernelGGL(bp_count_kernel<T>, dim3(wgs), dim3(256), 0, s, app, x, its, B, nv, k,
                       reinterpret_cast<unsigned long long *>(counts), per_cw);
    SG_HIP(hipGetLastError());
    return SG_OK;
}
template int bp_count_launch<float>(const float *, const uint8_t *, const int32_t *, int, int, int, int64_t *, hipStream_t,
                                    int32_t *);
template int bp_count_launch<double>(const double *, const uint8_t *, const int32_t *, int, int, int, int64_t *,
                                     hipStream_t, int32_t *);

// ---------------------------------------------------------------- scalar helpers
// Device evaluation of the reference's exported Lxor / Lxfb utilities.
__global__ void lxfb_kernel(double *L, int dc, int corr, double *agg) {
    double f[64], b[64];
    f[0] = L[0];
    b[dc - 1] = L[dc - 1];
    for (int k = 1; k < dc; ++k) {
        f[k] = corr ? lxor<double, true>(f[k - 1], L[k]) : lxor<double, false>(f[k - 1], L[k]);
        b[dc - 1 - k] = corr ? lxor<double, true>(b[dc - k], L[dc - 1 - k]) : lxor<double, false>(b[dc - k], L[dc - 1 - k]);
    }
    L[0] = b[1];
    L[dc - 1] = f[dc - 2];
    for (int k = 1; k < dc - 1; ++k)
        L[k] = corr ? lxor<double, true>(f[k - 1], b[k + 1]) : lxor<double, false>(f[k - 1], b[k + 1]);
    *agg = b[0];
}

int lxfb_launch(double *dL, int dc, int corr, double *dagg, hipStream_t s) {
    hipLaunchKernelGGL(lxfb_kernel, dim3(1), dim3(1), 0, s, dL, dc, corr, dagg);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

}  // namespace sg
