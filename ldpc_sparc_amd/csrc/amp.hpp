// Declarations shared by the AMP decoder kernels (amp_dct.hip) and the host
// plan / C ABI (capi_amp.cpp).
#pragma once
#include "common.hpp"
#include "fft.hpp"

namespace sg {

constexpr int AMP_MAX_EPT = 32;

// Stage twiddles of the block engines' 2^14-point transforms: bit 0 forward,
// bit 1 inverse from the hardware sine / cosine, otherwise from the plan's
// table (tb.stw)
#ifndef SG_BLK_SINCOS
#define SG_BLK_SINCOS 2
#endif

// Design operator tables of one design (all transforms), device pointers.
// A "transform" is one nonzero block (r, c) of the base matrix W
// (sparc.py:777-875): a sub-sampled DCT of size w with its own orders.
template <typename T>
struct AmpTables {
    int nT, w, N2, P, Q, log2P, log2Q, npairs;
    int L, M, LM, n, Lr, Lc, Mr, Mc, ndim;
    const int32_t *t_row, *t_col;     // [nT]
    const int32_t *col_ptr, *col_t;   // CSR: transforms of each column block, row-major order
    const int32_t *inmap;             // [nT][w]  w-space slot -> local column index, or -1
    const int32_t *outslot;           // [nT][Mc] local column index -> w-space slot
    const int32_t *rp_ptr;            // [nT*(npairs+1)] absolute offsets into rp_*
    const int32_t *rp_i;              // output row index (local to the row block)
    const uint32_t *rp_ab;            // LDS indices (la | lb << 16) of H[a], H[b]
    const cx<T> *rp_c;                // [2] per output: X = Re(c1 H[a] + c2 conj(H[b]))
    const int32_t *gs_ptr;            // [nT*(npairs+1)] absolute offsets into gs_*
    const int32_t *gs_loc;            // LDS index of the G slot
    const int32_t *gs_i;              // [4] per slot: contributing row index or -1
    const cx<T> *gs_c;                // [4] per slot: coefficient
    const cx<T> *twP, *twQ, *twHi, *twLo;
    const int32_t *row_ptr, *row_t;   // CSR: transforms of each row block, row-major order
};

// Block engine (amp_block.hip): single precision, N2 = 2^14, one workgroup per
// (column block, codeword) running that column's transforms in LDS.
struct BlkTables {
    int nT, L, M, LM, n, Lr, Lc, Mr, Mc;
    const int32_t *col_ptr, *col_t, *t_row;
    const uint32_t *pos2;     // [nT][8][1024] real LDS index (2 fsw(m) + component) of column entry
                              // j = tid + 1024 i, pairs (i = 2 i2, 2 i2 + 1) at [t][i2][tid]; the two-class
                              // engine: [nT][2][16][1024], 2 ppos(m1) + component per class (amp_block2.hip)
    const uint32_t *pos1;     // two-class engine, one-table form (A/B, -DB2_ONETABLE=1): [nT][16][1024] per column
                              // entry m1 << 2 | component << 1 | class (16 bits, pairs), both classes' passes
    const uint32_t *oab;      // [nT][Mr] (a mod 4096) | (b mod 4096) << 16 of output i
    const cx<float> *oc;      // [nT][Mr][8] X_i = Re(sum_r al_r Y[a mod 4096 + 4096 r] + be_r conj Y[b mod ...]),
                              // al_r = c1 w_N2^(r a), be_r = c2 conj w_N2^(r b) (the last FFT stage folded in)
    int ngs;                  // G slots of all transforms (= gptr[nT])
    const int32_t *gptr;      // [nT + 1] G slots of each transform (CSR)
    const int32_t *grow;      // row block of each slot's transform
    const uint16_t *gloc;     // fsw(k) of the slot
    const int32_t *gk;        // k of the slot (two-class form, amp_block2.hip)
    const int32_t *gi;        // [4] per slot: contributing output row index (local to the row block) or -1
    const cx<float> *gc;      // [4] per slot: coefficient
    const cx<float> *stw;     // per-stage twiddles of the N2-point FFT (fft.hpp lds_fft1_ct, EPT 16)
    int skip;                 // timing ablation only (SG_AMP_SKIP): 1 sections, 2 inverse FFT
    int log2p;                // two-class engine: class size P = 2^log2p (13: C4's w = 2^15, 14: w = 2^16)
};
size_t blk_lds_bytes(int Mc);
size_t blk2_lds_bytes(int log2p);

// Per-batch device buffers.
template <typename T>
struct AmpBufs {
    int B;
    T *beta;        // [B][LM]
    const T *y;     // [B][n]
    T *z;           // [B][n]
    T *rbuf;        // [B][nT][Mr]
    cx<T> *buf0;    // [B][nT][N2]  four-step intermediates (T, then U)
    cx<T> *buf1;    // [B][nT][N2]  inverse-transform output g (w-space)
    double *phi;    // [B][Lr]
    double *tau;    // [B][Lc]
    int32_t *active;     // [B]
    double *sec_sumsq;   // [B][L]   sum of beta^2 per section
    double *sec_err;     // [B][L]   sum of (beta - beta0)^2 per section
    int32_t *sec_argmax; // [B][L]   MAP index per section (argmax of s)
    const int32_t *true_idx; // [B][L] or null
};

// Per-codeword scalar state of the AMP recursion (double), see amp_control.
struct AmpScalars {
    double *psi, *psi_prev, *phi_prev, *gamma, *bcoef;  // [B][Lc] / [B][Lr]
    double *nmse;       // [B][t_max][Lc]
    int32_t *t_final;   // [B]
};

struct AmpParams {
    const double *W;    // [Lr*Lc] base matrix (ndim 0: one value, ndim 1: Lc values)
    double awgn_var, rtol, atol;
    int phi_method, t_max;
};

// ------------------------------------------------------------------------
// Regular engine (amp_fused.hip): designs with one transform per column block
// (W.ndim 0 or 1, every W entry nonzero).  See DESIGN.md "AMP engine".
//
// Complex w-space index m = Q*m1 + m2.  A "class" is the residue m2: the P
// complex slots {Q*m1 + m2}.  The decoder keeps s (sparc.py:972) per codeword
// in CLASS ORDER: entries of a column block sorted by (class, section, j), so
// the P-point FFT stage of each class reads and writes its slice of s
// contiguously and the reference's random orders (generate_ordering,
// sparc.py:735-775) become LDS scatters.  Only the rows k1 that hold needed
// outputs of the forward transform (= nonzero inputs of the inverse) cross
// HBM between the two FFT stages ("needed rows", compact index rho).
template <typename T>
struct RegTables {
    int nT, L, M, LM, n, Lc, Mc, Lblk;  // Lblk = sections per column block
    int N2, P, Q, log2P;
    int nRmax, nKmax, RB, nrb;          // needed rows / indices (max over t), row-block size, #row blocks
    int maxKb;                          // most needed indices in one row block
    const int32_t *nR;       // [nT]
    const int32_t *row_k1;   // [nT][nRmax]
    const uint32_t *row_k1p; // [nT][EPT/2][P/EPT] rows (tid + 2j nthr, + nthr) as 16-bit pairs (stage-1 order)
    const int32_t *kptr;     // [nT][nRmax+1] needed indices of each row (CSR, within t)
    const int32_t *kk2;      // [nT][nKmax]
    const int32_t *krho;     // [nT][nKmax]
    const int32_t *oa, *ob;  // [nT][n] forward outputs: X = Re(c1 X[oa] + c2 conj X[ob])
    const cx<T> *oc;         // [nT][n][2]
    const int32_t *gi;       // [nT][nKmax][4] inverse inputs: G[k] = sum c * z[i]/phi
    const cx<T> *gc;         // [nT][nKmax][4]
    const int32_t *cls_ptr;  // [nT][Q+1]
    const uint32_t *cls_ls;  // [nT][Mc] padded real LDS index | section within the block << 16
    const int32_t *cls_j;    // [nT][Mc] column index within the block
    const int32_t *qpos;     // [nT][Mc] column index -> class-order position
    const uint16_t *seg;     // [nT][Q][Lblk+1] section segments within a class
    const cx<T> *twP, *twQ, *twHi, *twLo;
    const cx<T> *stw;         // per-stage P-point FFT twiddles (lds_fft1)
    const cx<T> *twa, *twb;   // w_N2^(m2 k1) = twa[m2][k1 & 63] * twb[m2][k1 >> 6]
    int nB;                   // ceil(P / 64)
    int ept;                  // stage-1 FFT elements per thread (block = P / ept)
    int maxcls;               // largest class (entries of one m2 within a column block)
    int stagger;              // first-wave start offset of odd workgroups, cycles (SG_AMP_STAGGER)
    int img;                  // reals of the stage-1 LDS image: max(2P, fpad(maxcls + 16))
    int skip;                 // timing ablation only (SG_AMP_SKIP): 1 FFT, 2 gather/scatter, 4 row I/O
};

template <typename T>
struct RegBufs {
    int B;
    int mode;               // 0: decode; 1: operator application (ext_in / ext_out)
    T *s;                   // [B][LM] class order
    cx<T> *tu;              // [B][nT][Q][nRmax]
    cx<T> *xn;              // [B][nT][nKmax]
    T *part;                // [B][nT][Q][3][Lblk] per-class section max, sum e, sum e^2
    T *stM, *stI;           // [B][L] section max of s, 1/sum
    const T *y;             // [B][n]
    T *z;                   // [B][n]
    double *phi, *tau, *tau_prev;  // [B], [B][Lc], [B][Lc]
    int32_t *active;        // [B]
    const int32_t *true_idx;  // [B][L] or null
    int32_t *map;           // [B][L]
    const T *ext_in;        // mode 1: [B][LM] (Ab) or [B][n] (Az)
    T *ext_out;             // mode 1: [B][n] (Ab) or [B][LM] (Az)
    uint64_t *tprof_ab, *tprof_az;  // diagnostics (SG_AMP_TPROF): [B][nT][Q][8] phase timestamps, or null
    uint64_t *trt_ab, *trt_az;      // diagnostics: [B][nT][Q][2] realtime start / end
};

// Per-codeword engine (amp_cw.hip): the regular design at the benchmark sizes
// (single precision, one transform, P = 2^13), one 1024-thread workgroup per
// codeword running a whole AMP iteration -- every class of both transforms,
// the residual and the section statistics -- with the needed spectrum in LDS
// and no HBM intermediates.  The needed indices k = k1 + P k2 are owned by
// threads (all of a row's indices by one thread, at most KT per thread).
constexpr int CW_THREADS = 1024;
constexpr uint32_t CW_KMASK = (1u << 19) - 1;  // needed index k < N2 <= 2^19
constexpr uint32_t CW_NEWROW = 1u << 20, CW_ENDROW = 1u << 21, CW_VALID = 1u << 22;
struct CwTables {
    int L, M, LM, n, N2, Q, Lblk, KT, log2P, maxcls;
    int maxseg;               // longest section segment of a class
    float inv_n2;             // 1 / N2
    int img;                  // LDS reals of the FFT / class image (>= z / phi)
    const uint32_t *kt;       // [KT][1024] owned needed index k | flags; X / G slot j * 1024 + tid
    const uint16_t *cmask;    // [Q + 1][1024] image values written per thread (class m2; rows: Q)
    const int32_t *oa, *ob;   // [n] slots of the forward outputs' X[a], X[b]
    const cx<float> *oc;      // [n][2]
    const int32_t *gi;        // [KT * 1024][4] inverse inputs by slot (output row index; unused: 0)
    const cx<float> *gc;      // [KT * 1024][4] (unused: 0)
    const int32_t *cls_ptr;   // [Q+1]
    const uint32_t *cls_ls;   // [Mc] padded real LDS index | section << 16
    const int32_t *qpos;      // [Mc]
    const uint16_t *seg;      // [Q][Lblk+1]
    const cx<float> *stw;     // the P-point FFT's stage twiddles at 8 elements per thread
    uint64_t *tprof;          // diagnostics (SG_AMP_TPROF): [B][32] shader-clock stamps, or null
};
size_t cw_lds_bytes(int img, int nslots);

// Split per-codeword engine (amp_cw2.hip): each codeword's AMP iteration as
// two 512-thread workgroups (the two halves of the Q classes), two
// workgroups per CU, so one workgroup's barrier waits and memory latency
// overlap the other's work.  Four launches per iteration: Ab halves (partial
// H of every output, in registers), control (residual, phi, tau, z/phi),
// Az halves (rows, inverse transform, s update, partial section statistics),
// merge.  Output-owned: thread tid owns the outputs of slots j * 512 + tid,
// j < OT, grouped by conjugate row pair {r, P - r} of the P-point stage (host
// build_cw2).  See DESIGN.md "Split per-codeword engine".
constexpr int CW2_THREADS = 512;
// f32 split engine: workgroups per codeword at most (Cw2Tables.np: 2, or 4 once codewords have stopped), each
// taking Q / np of the classes; the partial buffers are sized for CW2_NP
#ifndef CW2_NP
#define CW2_NP 4
#endif
constexpr int CW2_SLICE = 9216;     // class entries per workgroup pass (18 per thread)
// P-point image layout of the split engine: complex element i at c2pos(i) =
// i + i / 32 (one pad value per 32), so every LDS access of the transform's
// stages is a per-thread base plus a constant (amp_cw2.hip c2_fft)
__host__ __device__ constexpr int c2pos(int i) { return i + (i >> 5); }
constexpr uint32_t CW2_TRASH = 2 * (8192 + 256) + 2048;  // LDS float index of the trash slot (after the
                                                         // padded image and the statistics)
constexpr uint32_t CW_SELF = 1u << 23;  // the pair's two rows coincide (r = 0 or P / 2)
// bits 24-26 of a split-engine slot word (f32): the output's phase offset o in units of N / 2 (build_cw2
// polar form: al = |al| e^(2 pi i (3a + o N/2) / 4N), be = |be| e^(2 pi i (N - 3a - o N/2) / 4N))
constexpr int CW_OFFSHIFT = 24;
// a thread's slots padded to a multiple of four (thread-major tables: 16-byte loads)
__host__ __device__ constexpr int cw2_otp(int ot) { return (ot + 3) & ~3; }
// z / phi thread-major (one load round of 16-byte loads in cw2_az) up to 12 slots per thread; above, cw2_az
// loads the slots in two rounds of single words, slot-major
__host__ __device__ constexpr bool cw2_vz_tm(int ot) { return ot <= 12; }
struct Cw2Tables {
    int L, M, LM, n, N2, Q, Lblk, OT, maxcls;
    int np;                   // workgroups per codeword (f32 split engine): 2, or 4 once codewords have stopped
    float inv_n2;             // 1 / N2
    const uint32_t *cmask;    // [Q + 1][512] image values each thread's first FFT stage reads (class m2; rows: Q)
    const uint32_t *ka;       // [OT][512] a | CW_VALID | CW_NEWROW (first of its pair) | CW_ENDROW | CW_SELF
    const uint32_t *kat;      // [512][OTP] the same, thread-major (a thread's slots in 16-byte loads)
    const int32_t *oi;        // [OT][512] output index (invalid slots: 0)
    const float4 *cf;         // [OT][512] (c1, c2): output = Re(c1 H[a] + c2 conj H[N2 - a])
    const float4 *gf;         // [OT][512] (al, be): G[a] += al z/phi, G[N2 - a] += be z/phi
    const float2 *gm;         // [OT][512] (|al|, |be|) of the polar form (CW_OFFSHIFT; cw2_ctrl scales z/phi)
    const float4 *gmt;        // [512][OTP / 2] the same thread-major, two slots per 16 bytes (C2_VZ_HALF rows)
    int sh_off;               // log2(N / 2): the slot's phase offset o N/2 = o << sh_off
    uint32_t m4n;             // 4N - 1 (phases in units of 1 / 4N revolutions, N = 2 N2 a power of two)
    float inv_4n;             // 1 / 4N
    const int32_t *cls_ptr;   // [Q+1]
    const uint32_t *cls_ls;   // [Mc] padded real LDS index | section << 16
    const uint32_t *cls2;     // [Q][9216] cls_ls of each class padded to 9216 entries with CW2_TRASH
    const uint32_t *clsp;     // [Q][4608] image positions of entries q and q + 4608 of cls2 (low, high half)
    const int32_t *qpos;      // [Mc]
    const uint16_t *seg;      // [Q][Lblk+1]
    float *xr;                // [B][2][OT][512] each half's part of Re(c1 H[a] + c2 conj H[b]) per output
    const uint2 *rab;         // [OT][512] LDS byte addresses of rows r, P - r of the slot's output (cw2_ab reads)
    const uint2 *wab;         // [OT][512] LDS byte addresses of the slot's row writes (rows r, P - r on the
                              // pair's last slot, else the trash slot; r = 0, P / 2: row r and trash)
    float *vz;                // z / phi in slot order, times (|al|, |be|) (two floats per slot): [B][512][OTP][2]
                              // thread-major (OTP = OT rounded up to 4) if cw2_vz_tm(OT), else [B][OT][512][2]
    float *ys, *zs;           // [B][OT][512] y (copied at t = 0) and z in slot order (cw2_ctrl reads them
                              // coalesced; z in natural order is still written for a hand-over)
    float4 *part;             // [B][2][Lblk] partial section statistics (max, R1, R2, s of the true entry or NaN)
    uint64_t *tprof;          // diagnostics (SG_AMP_TPROF): [2 B][64] shader-clock stamps (Ab 0-31, Az 32-63), or null
};
int cw2_launch_iter(const Cw2Tables &tb, const RegBufs<float> &bf, const AmpScalars &sc, const AmpParams &pr, int t,
                    hipStream_t s);
// z in natural order from the split engine's slot-order copy (before a hand-over to the staged engine)
int cw2_launch_z_natural(const Cw2Tables &tb, const RegBufs<float> &bf, hipStream_t s);
// The same engine in double precision (amp_cw2d.hip): the split engine's slot and class tables, double
// coefficients, the slots' w_N2^a (Horner / rotation steps over the classes) and the P-point stage twiddles.
// One 512-thread workgroup per CU (the complex double image is 132 KB).
struct Cw2dTables {
    int L, M, LM, n, N2, Q, Lblk, OT, maxcls;
    const uint32_t *cmask, *ka, *kat;  // as Cw2Tables
    const int32_t *oi;
    const double *cf;         // [OT][512][4] (c1, c2): output = Re(c1 H[a] + c2 conj H[N2 - a])
    const double *gf;         // [OT][512][4] (al, be): G[a] += al z/phi, G[N2 - a] += be z/phi
    const double *sa;         // [OT][512][2] w_N2^a of the slot (invalid slots: 1)
    const double *twp;        // [8192][2] w_8192^k
    const int32_t *cls_ptr;
    const uint32_t *cls2;
    const int32_t *qpos;
    const uint16_t *seg;
    double *xr;               // [B][2][OT][512] each half's part of the forward output
    double *vz;               // [B][OT][512] z / phi
    double *ys, *zs;          // [B][OT][512]
    double *beta;             // [B][LM] beta in class order (cw2d_stats -> the next Ab, Az's beta_prev)
    double *sec;              // [B][L][2] per section: sum beta^2, squared error (cw2d_stats -> cw2d_final)
};
int cw2d_launch_iter(const Cw2dTables &tb, const RegBufs<double> &bf, const AmpScalars &sc, const AmpParams &pr,
                     int t, hipStream_t s);
// The compile-time bounds of amp_cw2d.hip, checked by the plan builder (build_regular: a plan outside them keeps
// the staged engine) and again by cw2d_launch_iter: P = 8192 (N2 = 8192 Q), an even Q <= 64, one column block,
// L <= 1024 and a multiple of 4 (statistics workgroups), M <= 512 (one wavefront of 8 entries per lane per
// section), class slices of at most CW2_SLICE entries, 12, 13, 14 or 16 outputs per thread.
inline bool cw2d_supported(const Cw2dTables &tb) {
    return tb.Q % 2 == 0 && tb.Q > 0 && tb.Q <= 64 && tb.L > 0 && tb.L <= 1024 && tb.L % 4 == 0 &&
           tb.Lblk == tb.L && tb.maxcls <= CW2_SLICE && tb.M > 0 && tb.M <= 512 && tb.N2 == 8192 * tb.Q &&
           (tb.OT == 12 || tb.OT == 13 || tb.OT == 14 || tb.OT == 16);
}
int cw_launch_iter(const CwTables &tb, const RegBufs<float> &bf, const AmpScalars &sc, const AmpParams &pr, int t,
                   hipStream_t s);

template <typename T>
int reg_launch_ab(const RegTables<T> &tb, const RegBufs<T> &bf, hipStream_t s);
template <typename T>
int reg_launch_az(const RegTables<T> &tb, const RegBufs<T> &bf, int t_iter, hipStream_t s);
template <typename T>
int reg_launch_ctrl0(const RegTables<T> &tb, const RegBufs<T> &bf, const AmpScalars &sc, const AmpParams &pr,
                     int t, hipStream_t s);
template <typename T>
int reg_launch_merge(const RegTables<T> &tb, const RegBufs<T> &bf, const AmpScalars &sc, const AmpParams &pr,
                     int t, hipStream_t s);
template <typename T>
int reg_launch_map(const RegTables<T> &tb, const RegBufs<T> &bf, hipStream_t s);
template <typename T>
int reg_launch_ab_finish(const RegTables<T> &tb, const RegBufs<T> &bf, hipStream_t s);
size_t reg_stage1_lds(int img, int P, int Lblk, size_t real_bytes);
// stage-1 elements per thread: f32 at P >= 8192 uses 16 (P = 8192 -> 512-thread
// workgroups, two per CU); otherwise P/1024 threads' worth, at least 8
inline int reg_ept(int P, size_t real_bytes) {
    if (real_bytes == 4 && P >= 8192) return 16;
    return P / 1024 > 8 ? P / 1024 : 8;
}
int reg_launch_init(int B, int Lc, int t_max, double *nmse, int32_t *active, int32_t *t_final, hipStream_t s);

template <typename T>
int amp_launch_ab(const AmpTables<T> &tb, const AmpBufs<T> &bf, hipStream_t s);   // beta -> rbuf
template <typename T>
int amp_launch_az(const AmpTables<T> &tb, const AmpBufs<T> &bf, hipStream_t s);   // z/phi -> buf1
template <typename T>
int amp_launch_eta(const AmpTables<T> &tb, const AmpBufs<T> &bf, hipStream_t s);
template <typename T>
int amp_launch_control(const AmpTables<T> &tb, const AmpBufs<T> &bf, const AmpScalars &sc,
                       const AmpParams &pr, int phase, int t, hipStream_t s);
template <typename T>
int amp_launch_rowsum(const AmpTables<T> &tb, const AmpBufs<T> &bf, T *out, hipStream_t s);
template <typename T>
int amp_launch_colgather(const AmpTables<T> &tb, const AmpBufs<T> &bf, T *out, hipStream_t s);
template <typename T>
int amp_launch_cast(const void *in, int in_is_double, T *out, size_t n, hipStream_t s);
template <typename T>
int amp_launch_uncast(const T *in, double *out, size_t n, hipStream_t s);
int blk_launch_az(const BlkTables &tb, const AmpBufs<float> &bf, bool then_ab,
                  hipStream_t s);  // z/phi -> G -> beta, section statistics (then the next Ab)
int blk_launch_g(const BlkTables &tb, const AmpBufs<float> &bf, cx<float> *gbuf, hipStream_t s);  // G slots
// two-class form for w = 2^16 (amp_block2.hip)
int blk2_launch_ab(const BlkTables &tb, const AmpBufs<float> &bf, hipStream_t s);
int blk2_launch_az(const BlkTables &tb, const AmpBufs<float> &bf, cx<float> *gbuf, bool then_ab, hipStream_t s);  // z/phi -> G slots (gbuf [B][ngs]) -> beta, section statistics
int amp_launch_count(const int32_t *map_idx, const int32_t *true_idx, const int32_t *t_final, int B, int L,
                     int logM, int64_t *counts, hipStream_t s);

}  // namespace sg
