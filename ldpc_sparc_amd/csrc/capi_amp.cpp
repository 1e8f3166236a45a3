// C ABI of the AMP decoder: design plans (sub-sampled DCT operator tables),
// batched decode, the design operators Ab / Az, error counting.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <complex>
#include <memory>
#include <random>
#include <type_traits>
#include <vector>

#include "amp.hpp"

using cd = std::complex<double>;

struct sg_amp_plan {
    int precision = SG_F32;
    // what the last decode through this handle ran (sg_amp_last_decode): the
    // sub-plan (itself or the companion), its first engine, and the iteration
    // at which the per-codeword engine handed over to the staged one (-1: none)
    sg_amp_plan *last_ran = nullptr;
    int last_engine = -1, last_handover = -1;
    int device = 0;
    int ndim = 0, L = 0, M = 0, LM = 0, n = 0, Lr = 1, Lc = 1, Mr = 0, Mc = 0, nT = 0;
    int w = 0, N2 = 0, P = 0, Q = 0, log2P = 0, log2Q = 0, npairs = 0;
    std::vector<double> W;
    std::vector<void *> allocs;  // every device allocation owned by the plan
    // device tables
    int32_t *t_row = nullptr, *t_col = nullptr, *col_ptr = nullptr, *col_t = nullptr, *row_ptr = nullptr,
            *row_t = nullptr;
    int32_t *inmap = nullptr, *outslot = nullptr, *rp_ptr = nullptr, *rp_i = nullptr;
    uint32_t *rp_ab = nullptr;
    int32_t *gs_ptr = nullptr, *gs_loc = nullptr, *gs_i = nullptr;
    void *rp_c = nullptr, *gs_c = nullptr, *twP = nullptr, *twQ = nullptr, *twHi = nullptr, *twLo = nullptr;
    double *dW = nullptr;
    // batch workspace (grow-only)
    int cap_B = 0, cap_tmax = 0;
    void *ws_beta = nullptr, *ws_y = nullptr, *ws_z = nullptr, *ws_rbuf = nullptr, *ws_buf0 = nullptr, *ws_buf1 = nullptr;
    void *ws_io = nullptr;  // staging for host entry points
    size_t ws_io_bytes = 0;
    double *ws_phi = nullptr, *ws_tau = nullptr, *ws_sumsq = nullptr, *ws_err = nullptr;
    double *ws_psi = nullptr, *ws_psi_prev = nullptr, *ws_phi_prev = nullptr, *ws_gamma = nullptr, *ws_bco = nullptr;
    double *ws_nmse = nullptr;
    int32_t *ws_active = nullptr, *ws_argmax = nullptr, *ws_true = nullptr, *ws_tfinal = nullptr;
    // regular engine (one transform per column block, amp_fused.hip)
    bool regular = false;
    int rP = 0, rQ = 0, rlog2P = 0, rept = 0, rmaxcls = 0, rmaxseg = 0, rimg = 0, nRmax = 0, nKmax = 0, RB = 0, nrb = 0, maxKb = 0, Lblk = 0, nB = 0;
    uint32_t *r_row_k1p = nullptr;
    int32_t *r_nR = nullptr, *r_row_k1 = nullptr, *r_kptr = nullptr, *r_kk2 = nullptr, *r_krho = nullptr;
    int32_t *r_oa = nullptr, *r_ob = nullptr, *r_gi = nullptr, *r_cls_ptr = nullptr, *r_cls_j = nullptr,
            *r_qpos = nullptr;
    uint32_t *r_cls_ls = nullptr;
    uint16_t *r_seg = nullptr;
    void *r_oc = nullptr, *r_gc = nullptr, *r_twP = nullptr, *r_twQ = nullptr, *r_stw = nullptr, *r_twa = nullptr,
         *r_twb = nullptr;
    uint64_t *tprof = nullptr;  // diagnostics: stage-1 phase timestamps (SG_AMP_TPROF)
    size_t tprof_items = 0;
    // active-flag poll (ActivePoll): pinned host copy and its completion event
    int32_t *h_active = nullptr;
    int h_active_cap = 0;
    hipEvent_t poll_ev = nullptr;
    void *ws_s = nullptr, *ws_tu = nullptr, *ws_xn = nullptr, *ws_part = nullptr, *ws_stM = nullptr,
         *ws_stI = nullptr;
    double *ws_tau_prev = nullptr;
    // per-codeword engine (amp_cw.hip), built beside the regular tables when eligible
    bool cw = false;
    int cwKT = 0;
    // A per-codeword plan uses P = 8192 for both engines; batches below one
    // wave of the CUs decode on this companion plan instead: the staged
    // engine at P = 16384 (17-21 % faster there, profiles/README.md)
    bool no_cw = false;
    sg_amp_plan *alt = nullptr;
    uint32_t *c_kt = nullptr;
    // split per-codeword engine (amp_cw2.hip): outputs per thread (0 = not built) and its tables
    int cw2OT = 0;
    int c2_np = 2;                // f32 split engine: workgroups per codeword for the next launches (decode_regular)
    uint32_t *c2_ka = nullptr, *c2_kat = nullptr, *c2_cmask = nullptr, *c2_cls = nullptr, *c2_clsp = nullptr;
    int32_t *c2_oi = nullptr;
    uint32_t *c2_wab = nullptr, *c2_rab = nullptr;
    void *c2_cf = nullptr, *c2_gf = nullptr;
    float *c2_gm = nullptr;  // [OT][512][2] (|al|, |be|) of the polar row form (build_cw2)
    float *c2_gmt = nullptr; // [512][OTP][2] the same, thread-major
    int c2_shoff = 0;        // log2(N / 2): unit of the slot's phase offset
    // its double-precision form (amp_cw2d.hip): coefficients, the slots' w_N2^a, the P-point twiddles
    double *c2d_cf = nullptr, *c2d_gf = nullptr, *c2d_sa = nullptr, *c2d_twp = nullptr;
    void *ws_c2xp = nullptr, *ws_c2vz = nullptr, *ws_c2part = nullptr, *ws_c2ys = nullptr, *ws_c2zs = nullptr;
    void *ws_c2beta = nullptr, *ws_c2sec = nullptr;  // f64 form: beta in class order, per-section sums
    uint16_t *c_cmask = nullptr;  // [Q + 1][1024] per-codeword engine: written image values per thread
    int32_t *c_oa = nullptr, *c_ob = nullptr, *c_gi = nullptr;
    void *c_gc = nullptr, *c_stw = nullptr;
    // block engine (several transforms per column block, amp_block.hip)
    bool block = false;
    bool block2 = false;         // two-class block engine (amp_block2.hip): w = 2^16, or w = 2^15 in two
    int b2_log2p = 0;            // classes of 2^13 points (two workgroups per CU); class size P = 2^b2_log2p
    int32_t *b_gk = nullptr;
    uint16_t *b_gloc = nullptr;
    uint32_t *b_pos2 = nullptr, *b_pos1 = nullptr, *b_oab = nullptr;
    int32_t *b_gptr = nullptr, *b_gi = nullptr, *b_grow = nullptr;
    int b_ngs = 0;
    void *ws_gbuf = nullptr;  // [B][b_ngs] G slots (block engine)
    void *b_oc = nullptr, *b_gc = nullptr, *b_stw = nullptr;
};

extern "C" int sg_amp_plan_destroy(sg_amp_plan *p);

namespace sg {

static int ilog2(int v) {
    int l = 0;
    while ((1 << l) < v) ++l;
    return l;
}

template <typename X>
static int upload(sg_amp_plan *p, X **dst, const std::vector<X> &src) {
    void *d = nullptr;
    SG_HIP(hipMalloc(&d, std::max<size_t>(1, src.size() * sizeof(X))));
    p->allocs.push_back(d);
    if (!src.empty()) SG_HIP(hipMemcpy(d, src.data(), src.size() * sizeof(X), hipMemcpyHostToDevice));
    *dst = (X *)d;
    return SG_OK;
}

static int upload_cx(sg_amp_plan *p, void **dst, const std::vector<cd> &src) {
    if (p->precision == SG_F64) {
        std::vector<double> v(2 * src.size());
        for (size_t i = 0; i < src.size(); ++i) { v[2 * i] = src[i].real(); v[2 * i + 1] = src[i].imag(); }
        double *d = nullptr;
        SG_TRY(upload(p, &d, v));
        *dst = d;
    } else {
        std::vector<float> v(2 * src.size());
        for (size_t i = 0; i < src.size(); ++i) { v[2 * i] = (float)src[i].real(); v[2 * i + 1] = (float)src[i].imag(); }
        float *d = nullptr;
        SG_TRY(upload(p, &d, v));
        *dst = d;
    }
    return SG_OK;
}

static cd expi(double a) { return cd(std::cos(a), std::sin(a)); }

// Twiddle exp(-2 pi i k / m) with exact integer reduction of k mod m.
static cd tw(long long k, long long m) {
    k %= m;
    if (k < 0) k += m;
    return expi(-2.0 * M_PI * (double)k / (double)m);
}

// Forward output at DCT position k (sparc.py:687-692 via the Makhoul packed
// FFT): X_dct[k] = Re(c1 H[a] + c2 conj(H[b])), H = FFT_{N/2} of the packed
// sequence; sc = sqrt(W/L) of the block (sparc.py:786-794).
static void fwd_coef(long long k, long long N, long long N2, double sc, long long *a, long long *b, cd *c1, cd *c2) {
    const long long kk = (k <= N2) ? k : N - k;
    *a = kk % N2;
    *b = (N2 - kk) % N2;
    const cd e = (k <= N2) ? expi(-M_PI * (double)k / (2.0 * N)) : expi(M_PI * (double)k / (2.0 * N));
    const cd wk = tw(kk, N);
    const cd I(0, 1);
    const double sqrt2 = std::sqrt(2.0);
    *c1 = e * (0.5 - 0.5 * I * wk) * (sqrt2 * sc);
    *c2 = e * (0.5 + 0.5 * I * wk) * (sqrt2 * sc);
}

// Inverse input: a value v at DCT position q (sparc.py:694-699) contributes
// coef * v to the packed spectrum G at one or two N/2-indices:
// G[k] = A_k y[k] - i A_k y[N-k] + C_k y[N2+k] - i C_k y[N2-k].
template <typename F>
static void inv_contrib(long long q, long long N, long long N2, double sc, F &&add) {
    const cd I(0, 1);
    auto Ak = [&](long long k) { return expi(M_PI * (double)k / (2.0 * N)) * (1.0 + I * tw(-k, N)); };
    auto Ck = [&](long long k) { return expi(M_PI * (double)(k + N2) / (2.0 * N)) * (1.0 - I * tw(-k, N)); };
    const double gsc = sc / std::sqrt(2.0);  // sqrt(2 W/L) * (1/2)
    if (q < N2) {
        add(q, Ak(q) * gsc);
        add(N2 - q, -I * Ck(N2 - q) * gsc);
    } else if (q > N2) {
        add(N - q, -I * Ak(N - q) * gsc);
        add(q - N2, Ck(q - N2) * gsc);
    } else {
        add(0, Ck(0) * (1.0 - I) * gsc);
    }
}

static long long slot_of_pos(long long pos, long long N) {  // w-space slot of DCT position pos
    return (pos % 2 == 0) ? pos / 2 : N - 1 - (pos - 1) / 2;
}

static int plan_free_ws(sg_amp_plan *p) {
    void **ws[] = {&p->ws_beta, &p->ws_y, &p->ws_z, &p->ws_rbuf, &p->ws_buf0, &p->ws_buf1, &p->ws_io,
                   (void **)&p->ws_phi, (void **)&p->ws_tau, (void **)&p->ws_sumsq, (void **)&p->ws_err,
                   (void **)&p->ws_psi, (void **)&p->ws_psi_prev, (void **)&p->ws_phi_prev, (void **)&p->ws_gamma,
                   (void **)&p->ws_bco, (void **)&p->ws_nmse, (void **)&p->ws_active, (void **)&p->ws_argmax,
                   (void **)&p->ws_true, (void **)&p->ws_tfinal, &p->ws_s, &p->ws_tu, &p->ws_xn, &p->ws_part,
                   &p->ws_stM, &p->ws_stI, (void **)&p->ws_tau_prev, &p->ws_gbuf, &p->ws_c2xp, &p->ws_c2vz, &p->ws_c2ys, &p->ws_c2zs,
                   &p->ws_c2part, &p->ws_c2beta, &p->ws_c2sec};
    for (void **x : ws) {
        if (*x) hipFree(*x);
        *x = nullptr;
    }
    p->cap_B = 0;
    p->cap_tmax = 0;
    p->ws_io_bytes = 0;
    return SG_OK;
}

static int ensure_ws(sg_amp_plan *p, int B, int t_max) {
    if (B <= p->cap_B && t_max <= p->cap_tmax) return SG_OK;
    plan_free_ws(p);
    const size_t rs = p->precision == SG_F64 ? 8 : 4;
    const size_t Bz = (size_t)B;
#define SG_ALLOC(ptr, bytes) SG_HIP(hipMalloc((void **)&(ptr), std::max<size_t>(16, (bytes))))
    SG_ALLOC(p->ws_y, Bz * p->n * rs);
    SG_ALLOC(p->ws_z, Bz * p->n * rs);
    if (p->regular) {
        SG_ALLOC(p->ws_s, Bz * p->LM * rs);
        SG_ALLOC(p->ws_tu, Bz * p->nT * p->rQ * p->nRmax * 2 * rs);
        SG_ALLOC(p->ws_xn, Bz * p->nT * p->nKmax * 2 * rs);
        SG_ALLOC(p->ws_part, Bz * p->nT * p->rQ * 3 * p->Lblk * rs);
        if (std::getenv("SG_AMP_TPROF")) {  // diagnostics only
            if (p->tprof) hipFree(p->tprof);
            p->tprof_items = Bz * p->nT * p->rQ;
            // [2 kernels][items][8] shader-clock stamps, then [2 kernels][items][2] realtime start / end
            SG_ALLOC(p->tprof, p->tprof_items * 20 * sizeof(uint64_t));
            SG_HIP(hipMemset(p->tprof, 0, p->tprof_items * 20 * sizeof(uint64_t)));
        }
        if (p->cw2OT) {  // (reals of the plan's precision; partial statistics: four per section)
            SG_ALLOC(p->ws_c2xp, Bz * std::max(CW2_NP, 2) * p->cw2OT * CW2_THREADS * rs);
            SG_ALLOC(p->ws_c2vz, Bz * cw2_otp(p->cw2OT) * CW2_THREADS * 8);  // (f32: two reals per slot)
            SG_ALLOC(p->ws_c2ys, Bz * p->cw2OT * CW2_THREADS * rs);
            SG_ALLOC(p->ws_c2zs, Bz * p->cw2OT * CW2_THREADS * rs);
            SG_ALLOC(p->ws_c2part, Bz * std::max(CW2_NP, 2) * p->Lblk * 4 * rs);
            if (p->precision == SG_F64) {
                SG_ALLOC(p->ws_c2beta, Bz * p->LM * rs);
                SG_ALLOC(p->ws_c2sec, Bz * p->L * 2 * rs);
            }
        }
        SG_ALLOC(p->ws_stM, Bz * p->L * rs);
        SG_ALLOC(p->ws_stI, Bz * p->L * rs);
        SG_ALLOC(p->ws_tau_prev, Bz * p->Lc * 8);
    } else {
        SG_ALLOC(p->ws_beta, Bz * p->LM * rs);
        SG_ALLOC(p->ws_rbuf, Bz * p->nT * p->Mr * rs);
        SG_ALLOC(p->ws_buf0, Bz * p->nT * p->N2 * 2 * rs);
        SG_ALLOC(p->ws_buf1, Bz * p->nT * p->N2 * 2 * rs);
        SG_ALLOC(p->ws_sumsq, Bz * p->L * 8);
        SG_ALLOC(p->ws_err, Bz * p->L * 8);
    }
    if (p->block || p->block2) SG_ALLOC(p->ws_gbuf, Bz * (size_t)p->b_ngs * 8);
    SG_ALLOC(p->ws_phi, Bz * p->Lr * 8);
    SG_ALLOC(p->ws_tau, Bz * p->Lc * 8);
    SG_ALLOC(p->ws_psi, Bz * p->Lc * 8);
    SG_ALLOC(p->ws_psi_prev, Bz * p->Lc * 8);
    SG_ALLOC(p->ws_phi_prev, Bz * p->Lr * 8);
    SG_ALLOC(p->ws_gamma, Bz * p->Lr * 8);
    SG_ALLOC(p->ws_bco, Bz * p->Lr * 8);
    SG_ALLOC(p->ws_nmse, Bz * std::max(t_max, 2) * p->Lc * 8);
    SG_ALLOC(p->ws_active, Bz * 4);
    SG_ALLOC(p->ws_argmax, Bz * p->L * 4);
    SG_ALLOC(p->ws_true, Bz * p->L * 4);
    SG_ALLOC(p->ws_tfinal, Bz * 4);
#undef SG_ALLOC
    p->cap_B = B;
    p->cap_tmax = std::max(t_max, 2);
    return SG_OK;
}

template <typename T>
static AmpTables<T> tables(const sg_amp_plan *p) {
    AmpTables<T> tb;
    tb.nT = p->nT; tb.w = p->w; tb.N2 = p->N2; tb.P = p->P; tb.Q = p->Q; tb.log2P = p->log2P; tb.log2Q = p->log2Q;
    tb.npairs = p->npairs; tb.L = p->L; tb.M = p->M; tb.LM = p->LM; tb.n = p->n; tb.Lr = p->Lr; tb.Lc = p->Lc;
    tb.Mr = p->Mr; tb.Mc = p->Mc; tb.ndim = p->ndim;
    tb.t_row = p->t_row; tb.t_col = p->t_col; tb.col_ptr = p->col_ptr; tb.col_t = p->col_t;
    tb.inmap = p->inmap; tb.outslot = p->outslot; tb.rp_ptr = p->rp_ptr; tb.rp_i = p->rp_i; tb.rp_ab = p->rp_ab;
    tb.rp_c = (const cx<T> *)p->rp_c; tb.gs_ptr = p->gs_ptr; tb.gs_loc = p->gs_loc; tb.gs_i = p->gs_i;
    tb.gs_c = (const cx<T> *)p->gs_c; tb.twP = (const cx<T> *)p->twP; tb.twQ = (const cx<T> *)p->twQ;
    tb.twHi = (const cx<T> *)p->twHi; tb.twLo = (const cx<T> *)p->twLo;
    tb.row_ptr = p->row_ptr; tb.row_t = p->row_t;
    return tb;
}

// Phase ablation for timing studies (tools/ablate3.sh): compiled only into a
// diagnostic build (make DIAG=1), because the results are wrong when a phase
// is skipped.  The product library ignores SG_AMP_SKIP.
static int diag_skip() {
#ifdef SG_DIAG
    const char *sk = std::getenv("SG_AMP_SKIP");
    return sk ? std::atoi(sk) : 0;
#else
    return 0;
#endif
}

static BlkTables btables(const sg_amp_plan *p) {
    BlkTables tb;
    tb.nT = p->nT; tb.L = p->L; tb.M = p->M; tb.LM = p->LM; tb.n = p->n; tb.Lr = p->Lr; tb.Lc = p->Lc;
    tb.Mr = p->Mr; tb.Mc = p->Mc;
    tb.col_ptr = p->col_ptr; tb.col_t = p->col_t; tb.t_row = p->t_row;
    tb.pos2 = p->b_pos2; tb.pos1 = p->b_pos1; tb.oab = p->b_oab; tb.oc = (const cx<float> *)p->b_oc;
    tb.ngs = p->b_ngs; tb.gptr = p->b_gptr; tb.grow = p->b_grow; tb.gloc = p->b_gloc; tb.gi = p->b_gi; tb.gc = (const cx<float> *)p->b_gc;
    tb.gk = p->b_gk;
    tb.stw = (const cx<float> *)p->b_stw;
    tb.skip = diag_skip();
    tb.log2p = p->b2_log2p;
    return tb;
}

template <typename T>
static AmpBufs<T> bufs(const sg_amp_plan *p, int B, const void *y) {
    AmpBufs<T> bf;
    bf.B = B;
    bf.beta = (T *)p->ws_beta; bf.y = (const T *)(y ? y : p->ws_y); bf.z = (T *)p->ws_z; bf.rbuf = (T *)p->ws_rbuf;
    bf.buf0 = (cx<T> *)p->ws_buf0; bf.buf1 = (cx<T> *)p->ws_buf1; bf.phi = p->ws_phi; bf.tau = p->ws_tau;
    bf.active = p->ws_active; bf.sec_sumsq = p->ws_sumsq; bf.sec_err = p->ws_err; bf.sec_argmax = p->ws_argmax;
    bf.true_idx = nullptr;
    return bf;
}

// Bank-aware placement of the rows on the threads (amp_cw.hip cw_accumulate:
// at slot j, lanes 0-31 and 32-63 of a wavefront each read one image value
// at fsw(k1) with ds_read_b64, whose bank pair is fsw(k1) mod 32; distinct
// rows on one bank pair serialise).  Local search from the load-balanced
// placement: swap two rows of the same length that start at the same slot of
// threads in different lane groups when the summed worst bank multiplicity
// of the cells they touch does not grow.  Deterministic (fixed seed); the
// slot structure of every thread is unchanged.
#ifndef CW_BANKBAL
#define CW_BANKBAL 1
#endif
static void cw_bank_balance(std::vector<std::vector<int>> &own, const std::vector<int32_t> &row_k1,
                            const std::vector<int32_t> &kptr, int KT) {
    const int T = CW_THREADS;
    std::vector<int> at((size_t)T * KT, -1), pos((size_t)T * KT, -1), start((size_t)T * KT, 0);
    for (int t = 0; t < T; ++t) {  // row / list position at each slot; rows start where flagged
        int j = 0;
        for (int i = 0; i < (int)own[t].size(); ++i) {
            const int r = own[t][i], len = kptr[r + 1] - kptr[r];
            start[(size_t)t * KT + j] = len;
            for (int q = 0; q < len; ++q, ++j) {
                at[(size_t)t * KT + j] = r;
                pos[(size_t)t * KT + j] = i;
            }
        }
    }
    auto addr = [&](int t, int j) { const int r = at[(size_t)t * KT + j]; return r < 0 ? 0 : fsw(row_k1[r]); };
    auto cell = [&](int g, int j) {  // LDS cycles of the 32 lanes' reads at slot j (distinct addresses per bank pair)
        int a[32], cnt[32] = {0}, worst = 0;
        for (int l = 0; l < 32; ++l) {
            a[l] = addr(g * 32 + l, j);
            bool dup = false;
            for (int m = 0; m < l && !dup; ++m) dup = a[m] == a[l];
            if (!dup) worst = std::max(worst, ++cnt[a[l] & 31]);
        }
        return worst;
    };
    // candidates by (start slot, length)
    std::vector<std::vector<int>> by((size_t)KT * (KT + 1));
    for (int t = 0; t < T; ++t)
        for (int j = 0; j < KT; ++j)
            if (const int len = start[(size_t)t * KT + j]) by[(size_t)j * (KT + 1) + len].push_back(t);
    std::mt19937 rng(12345);
    const int iters = 8 * T * KT;
    for (int it = 0; it < iters; ++it) {
        const int A = (int)(rng() % T), j = (int)(rng() % KT), len = start[(size_t)A * KT + j];
        if (!len) continue;
        const auto &cand = by[(size_t)j * (KT + 1) + len];
        const int B = cand[rng() % cand.size()];
        const int gA = A / 32, gB = B / 32;
        if (gA == gB) continue;
        int before = 0, after = 0;
        for (int q = j; q < j + len; ++q) before += cell(gA, q) + cell(gB, q);
        for (int q = j; q < j + len; ++q) std::swap(at[(size_t)A * KT + q], at[(size_t)B * KT + q]);
        for (int q = j; q < j + len; ++q) after += cell(gA, q) + cell(gB, q);
        if (after > before) {
            for (int q = j; q < j + len; ++q) std::swap(at[(size_t)A * KT + q], at[(size_t)B * KT + q]);
            continue;
        }
        std::swap(own[A][pos[(size_t)A * KT + j]], own[B][pos[(size_t)B * KT + j]]);
    }
}

// Per-codeword engine tables (amp_cw.hip): the needed indices of each row go
// to one thread (longest rows first, to the least loaded thread), so a thread
// owns at most KT indices; slot (j, tid) at j * 1024 + tid; then
// cw_bank_balance.
static int build_cw(sg_amp_plan *p, const std::vector<int32_t> &row_k1, const std::vector<int32_t> &kptr,
                    const std::vector<int32_t> &kk2, const std::vector<int32_t> &oa, const std::vector<int32_t> &ob,
                    const std::vector<int32_t> &gi, const std::vector<cd> &gc, const std::vector<int32_t> &cls_ptr,
                    const std::vector<uint32_t> &cls_ls) {
    const int nr = (int)row_k1.size(), nk = kptr[nr];
    if (nk > 14 * CW_THREADS) return SG_OK;  // 12 slots per thread in LDS beside the image, 2 in registers
    std::vector<int> rows(nr);
    for (int r = 0; r < nr; ++r) rows[r] = r;
    std::stable_sort(rows.begin(), rows.end(),
                     [&](int a, int b) { return kptr[a + 1] - kptr[a] > kptr[b + 1] - kptr[b]; });
    std::vector<std::pair<int, int>> heap;  // (load, thread), min-heap
    for (int i = 0; i < CW_THREADS; ++i) heap.push_back({0, i});
    auto cmp = [](const std::pair<int, int> &a, const std::pair<int, int> &b) { return a > b; };
    std::make_heap(heap.begin(), heap.end(), cmp);
    std::vector<std::vector<int>> own(CW_THREADS);
    int KT = 0;
    for (int r : rows) {
        std::pop_heap(heap.begin(), heap.end(), cmp);
        auto &h = heap.back();
        own[h.second].push_back(r);
        h.first += kptr[r + 1] - kptr[r];
        KT = std::max(KT, h.first);
        std::push_heap(heap.begin(), heap.end(), cmp);
    }
    if (KT > 14) return SG_OK;  // the staged engine only
    KT = KT <= 12 ? 12 : 14;   // kernel instances (cw_iter<12>: all slots in LDS; <14>: two in registers)
#if CW_BANKBAL
    cw_bank_balance(own, row_k1, kptr, KT);
#endif
    const int P = p->rP, n = p->n;
    std::vector<uint32_t> kt((size_t)KT * CW_THREADS, 0u);
    std::vector<int32_t> cmap(nk, 0);
    for (int tid = 0; tid < CW_THREADS; ++tid) {
        int j = 0;
        for (int r : own[tid])
            for (int k = kptr[r]; k < kptr[r + 1]; ++k, ++j) {
                uint32_t e = ((uint32_t)row_k1[r] + (uint32_t)P * (uint32_t)kk2[k]) | CW_VALID;
                if (k == kptr[r]) e |= CW_NEWROW;
                if (k == kptr[r + 1] - 1) e |= CW_ENDROW;
                kt[(size_t)j * CW_THREADS + tid] = e;
                cmap[k] = j * CW_THREADS + tid;
            }
    }
    // forward outputs and inverse terms by slot; unused inverse terms: row 0
    // with coefficient 0 (the kernel reads all four)
    std::vector<int32_t> c_oa(n), c_ob(n), c_gi((size_t)KT * CW_THREADS * 4, 0);
    std::vector<cd> c_gc((size_t)KT * CW_THREADS * 4, cd(0, 0));
    for (int i = 0; i < n; ++i) {
        c_oa[i] = cmap[oa[i]];
        c_ob[i] = cmap[ob[i]];
    }
    for (int k = 0; k < nk; ++k)
        for (int q = 0; q < 4; ++q) {
            const int32_t i = gi[(size_t)k * 4 + q];
            if (i >= 0) {
                c_gi[(size_t)cmap[k] * 4 + q] = i;
                c_gc[(size_t)cmap[k] * 4 + q] = gc[(size_t)k * 4 + q];
            }
        }
    // stage twiddles of the P-point FFT at 8 elements per thread (fft.hpp layout)
    std::vector<cd> stw;
    {
        int radix[8];
        const int ns = fft1_plan(p->rlog2P, 8, radix);
        int lns = 0;
        for (int st = 0; st < ns; ++st) {
            const int R = radix[st];
            const long long Ns = 1LL << lns;
            for (long long k = 0; k < Ns; ++k)
                for (int q = 0; q < tw_per_k(R); ++q) stw.push_back(tw(tw_exp(R, q) * k, Ns * R));
            lns += ilog2(R);
        }
    }
    // Which image values the class scatter (Ab, class m2 < Q) and the row
    // writes (Az, entry Q) leave behind, as bits of the thread that reads them
    // in the first FFT stage (amp_cw.hip cw_stage0_r16: thread of complex
    // index m1 = j + 512 g reads it as value g & 7, bit 2 (g & 7) + component),
    // so that stage masks stale values instead of the image being zeroed.
    const int Q = p->rQ;
    std::vector<uint16_t> cmask((size_t)(Q + 1) * CW_THREADS, 0);
    auto mbit = [&](int m2, int m1, int c) {
        const int j = m1 & 511, g = m1 >> 9;
        const int tid = ((j >> 5) << 6) | ((g >> 3) << 5) | (j & 31);
        cmask[(size_t)m2 * CW_THREADS + tid] |= (uint16_t)(1u << (2 * (g & 7) + c));
    };
    for (int m2 = 0; m2 < Q; ++m2)
        for (int q = cls_ptr[m2]; q < cls_ptr[m2 + 1]; ++q) {
            const int loc = (int)(cls_ls[q] & 0xffffu);
            mbit(m2, fsw(loc >> 1), loc & 1);  // fsw is its own inverse
        }
    for (int r = 0; r < nr; ++r) {
        mbit(Q, row_k1[r], 0);
        mbit(Q, row_k1[r], 1);
    }
    SG_TRY(upload(p, &p->c_cmask, cmask));
    SG_TRY(upload(p, &p->c_kt, kt));
    SG_TRY(upload(p, &p->c_oa, c_oa));
    SG_TRY(upload(p, &p->c_ob, c_ob));
    SG_TRY(upload(p, &p->c_gi, c_gi));
    SG_TRY(upload_cx(p, &p->c_gc, c_gc));
    SG_TRY(upload_cx(p, &p->c_stw, stw));
    p->cwKT = KT;
    p->cw = true;
    return SG_OK;
}

// Bank-aware placement of the conjugate row pairs on the split engine's threads (amp_cw2.hip: at slot j
// the lanes of each 32-lane half of a wavefront read rows r and P - r of their slot's pair with
// ds_read_b64, bank pair c2pos(row) mod 32, in cw2_ab's accumulation, and write them in cw2_az's rows).
// Local search from the load-balanced placement, as cw_bank_balance: swap two pairs of the same length
// that start at the same slot of threads in different lane groups when the summed worst bank multiplicity
// of the cells they touch does not grow.  Every output keeps its arithmetic (same slot structure per
// thread, same class order); only the order of cw2_ctrl's sum of z^2 (phi) follows the placement.
// Deterministic (fixed seed).
// f32 split engine: four workgroups per codeword once codewords have stopped (1), always two (0) (A/B)
#ifndef C2_PARTS_ADAPT
#define C2_PARTS_ADAPT 1
#endif
#ifndef CW2_BANKBAL
#define CW2_BANKBAL 1
#endif
#ifndef CW2_BANKW
#define CW2_BANKW 0
#endif
static void cw2_bank_balance(std::vector<std::vector<int>> &own, const std::vector<std::vector<int>> &pair_of,
                             int OT, int P) {
    const int T = CW2_THREADS;
    std::vector<int> at((size_t)T * OT, -1), pos((size_t)T * OT, -1), start((size_t)T * OT, 0);
    for (int t = 0; t < T; ++t) {
        int j = 0;
        for (int i = 0; i < (int)own[t].size(); ++i) {
            const int r = own[t][i], len = (int)pair_of[r].size();
            start[(size_t)t * OT + j] = len;
            for (int q = 0; q < len; ++q, ++j) {
                at[(size_t)t * OT + j] = r;
                pos[(size_t)t * OT + j] = i;
            }
        }
    }
    // the lanes of a group hold distinct pairs at a slot, so distinct rows; empty slots all read row 0.
    // CW2_BANKW: cw2_az's row writes counted too -- ds_write_b64 serves 16-lane groups on 32 banks, so two
    // lanes of one 16-lane half collide when their rows' slots agree mod 16 (padding slots write the
    // thread's last pair again: C2_ROWS_ALWAYS)
    auto last_row = [&](int t, int j) {
        for (int q = j; q >= 0; --q)
            if (at[(size_t)t * OT + q] >= 0) return at[(size_t)t * OT + q];
        return 0;
    };
    auto cell = [&](int g, int j) {
        int ca[32] = {0}, cb[32] = {0}, wa = 0, wb = 0;
        bool empty = false;
        for (int l = 0; l < 32; ++l) {
            const int r = at[(size_t)(g * 32 + l) * OT + j];
            if (r < 0) {
                if (empty) continue;
                empty = true;
            }
            const int ra = r < 0 ? 0 : r, rb = r < 0 ? 0 : (P - r) % P;
            wa = std::max(wa, ++ca[c2pos(ra) & 31]);
            if (rb != ra) wb = std::max(wb, ++cb[c2pos(rb) & 31]);
        }
        int w = wa + wb;
        if (CW2_BANKW) {
            for (int hf = 0; hf < 2; ++hf) {
                int sa[16] = {0}, sb[16] = {0}, xa = 0, xb = 0;
                for (int l = 16 * hf; l < 16 * hf + 16; ++l) {
                    const int ra = last_row(g * 32 + l, j), rb = (P - ra) % P;
                    xa = std::max(xa, ++sa[c2pos(ra) & 15]);
                    xb = std::max(xb, ++sb[c2pos(rb) & 15]);
                }
                w += xa + xb;
            }
        }
        return w;
    };
    std::vector<std::vector<int>> by((size_t)OT * (OT + 1));
    for (int t = 0; t < T; ++t)
        for (int j = 0; j < OT; ++j)
            if (const int len = start[(size_t)t * OT + j]) by[(size_t)j * (OT + 1) + len].push_back(t);
    std::mt19937 rng(12345);
    const int iters = 8 * T * OT;
    for (int it = 0; it < iters; ++it) {
        const int A = (int)(rng() % T), j = (int)(rng() % OT), len = start[(size_t)A * OT + j];
        if (!len) continue;
        const auto &cand = by[(size_t)j * (OT + 1) + len];
        const int B = cand[rng() % cand.size()];
        const int gA = A / 32, gB = B / 32;
        if (gA == gB) continue;
        int before = 0, after = 0;
        for (int q = j; q < j + len; ++q) before += cell(gA, q) + cell(gB, q);
        for (int q = j; q < j + len; ++q) std::swap(at[(size_t)A * OT + q], at[(size_t)B * OT + q]);
        for (int q = j; q < j + len; ++q) after += cell(gA, q) + cell(gB, q);
        if (after > before) {
            for (int q = j; q < j + len; ++q) std::swap(at[(size_t)A * OT + q], at[(size_t)B * OT + q]);
            continue;
        }
        std::swap(own[A][pos[(size_t)A * OT + j]], own[B][pos[(size_t)B * OT + j]]);
    }
}

// Split per-codeword engine tables (amp_cw2.hip).  Output i at DCT position
// K reads H[a] and H[b], b = N2 - a (fwd_coef), and its inverse input adds to
// G[a] and G[b] (inv_contrib: first call a, second b): both touch only the
// conjugate row pair {a mod P, P - a mod P} of the P-point stage.  Each output
// is normalised so that a mod P is the smaller row of its pair (swapping a and
// b takes (c1, c2) to (conj c2, conj c1) and (al, be) to (be, al):
// Re(x) = Re(conj x)); the outputs of a pair go to one thread (the largest
// pairs first, each to the least loaded thread), at most OT per thread; a
// thread's slots list its pairs one after the other (CW_NEWROW on the first
// output of a pair, CW_ENDROW on the last, CW_SELF when the pair's rows
// coincide: r = 0 or P / 2).  Plus the first-FFT-stage masks of the
// 16-values-per-thread transform (amp_cw2.hip c2_stage0_r32).
static int build_cw2(sg_amp_plan *p, const uint32_t *o0, double sc, const std::vector<int32_t> &row_k1,
                     const std::vector<int32_t> &cls_ptr, const std::vector<uint32_t> &cls_ls) {
    const long long N = p->w, N2 = p->N2;
    const int P = p->rP, n = p->n, T = CW2_THREADS, Q = p->rQ;
    if (P != 8192 || Q % 2 || p->Lblk > 2 * T || p->rmaxcls > CW2_SLICE) return SG_OK;
    struct Out { long long a; cd c1, c2, al, be; };
    std::vector<Out> out(n);
    std::vector<std::vector<int>> pair_of(P / 2 + 1);
    for (int i = 0; i < n; ++i) {
        Out &o = out[i];
        long long b;
        fwd_coef(o0[i], N, N2, sc, &o.a, &b, &o.c1, &o.c2);
        int nc = 0;
        bool ok = true;
        o.al = o.be = cd(0, 0);
        inv_contrib(o0[i], N, N2, sc, [&](long long k, cd c) {
            if (nc++ == 0) {
                ok = ok && k % N2 == o.a;
                o.al = c;
            } else {
                ok = ok && k % N2 == b;
                o.be = c;
            }
        });
        SG_CHECK_ARG(ok && nc <= 2, "internal: inverse input of output %d outside its pair", i);
        const int r = (int)(o.a % P), r2 = (P - r) % P;
        if (r > r2) {  // normalise: a mod P is the smaller row of the pair
            o.a = b;
            const cd c1 = o.c1, al = o.al;
            o.c1 = std::conj(o.c2);
            o.c2 = std::conj(c1);
            o.al = o.be;
            o.be = al;
        }
        pair_of[(int)(o.a % P)].push_back(i);
    }
    std::vector<int> pairs;
    for (int r = 0; r <= P / 2; ++r)
        if (!pair_of[r].empty()) pairs.push_back(r);
    std::stable_sort(pairs.begin(), pairs.end(),
                     [&](int x, int y) { return pair_of[x].size() > pair_of[y].size(); });
    std::vector<std::pair<int, int>> heap;  // (load, thread), min-heap
    for (int i = 0; i < T; ++i) heap.push_back({0, i});
    auto cmp = [](const std::pair<int, int> &x, const std::pair<int, int> &y) { return x > y; };
    std::make_heap(heap.begin(), heap.end(), cmp);
    std::vector<std::vector<int>> own(T);
    int OT = 0;
    for (int r : pairs) {
        std::pop_heap(heap.begin(), heap.end(), cmp);
        auto &h = heap.back();
        own[h.second].push_back(r);
        h.first += (int)pair_of[r].size();
        OT = std::max(OT, h.first);
        std::push_heap(heap.begin(), heap.end(), cmp);
    }
    if (OT > 16) return SG_OK;  // kernel instances for 12, 13, 14 and 16 outputs per thread
    OT = OT <= 12 ? 12 : OT <= 14 ? OT : 16;
    if (CW2_BANKBAL) cw2_bank_balance(own, pair_of, OT, P);
    std::vector<uint32_t> ka((size_t)OT * T, 0u);
    std::vector<int32_t> oi((size_t)OT * T, 0);
    std::vector<float> cf((size_t)OT * T * 4, 0.f), gf((size_t)OT * T * 4, 0.f);
    const bool f64 = p->precision == SG_F64;
    std::vector<double> cfd(f64 ? (size_t)OT * T * 4 : 0, 0.0), gfd(f64 ? (size_t)OT * T * 4 : 0, 0.0),
        sad(f64 ? (size_t)OT * T * 2 : 0, 0.0);
    for (size_t i = 0; i < sad.size(); i += 2) sad[i] = 1.0;  // invalid slots: S = 1
    std::vector<uint32_t> wab((size_t)OT * T * 2, 4u * CW2_TRASH), rab((size_t)OT * T * 2, 0u);
    // Polar form of the inverse coefficients (amp_cw2.hip Az rows): with U = 1 / (4N) revolutions,
    // inv_contrib's al and be are real multiples of unit phasors, al = |al| e^(2 pi i A U) and
    // be = |be| e^(2 pi i (N - A) U), A = 3a + o N/2 (o in {0, 1, 6, 7} by the output's case: q below or
    // above N2, normalised by a swap or not).  Then the rows' al conj(W) and be W (W = w_N2^(m2 a)) are
    // |al| (cos x, sin x) and |be| (sin x, cos x) of ONE angle x = ((3 + 8 m2) a + o N/2) U: the rows
    // need the slot word and z/phi scaled by |al|, |be| (cw2_ctrl), not the complex (al, be) per class.
    // Fitted and checked per output here (any mismatch: no split engine for the plan).
    std::vector<float> gm((size_t)OT * T * 2, 0.f);
    const bool pow2 = N >= 4 && (N & (N - 1)) == 0 && 4 * N <= (1ll << 24);
    auto polar = [&](const Out &o, uint32_t *code, double *ma, double *mb) -> bool {
        if (!pow2) return false;
        const long long N4 = 4 * N;
        double best = 1e300;
        for (uint32_t c : {0u, 1u, 6u, 7u}) {
            const long long A = ((3 * o.a + (long long)c * (N / 2)) % N4 + N4) % N4;
            const cd ra = o.al * expi(-2.0 * M_PI * (double)A / (double)N4);
            const cd rb = o.be * expi(-2.0 * M_PI * (double)(N - A) / (double)N4);
            const double err = std::abs(ra.imag()) + std::abs(rb.imag());
            if (err < best) {
                best = err;
                *code = c;
                *ma = ra.real();
                *mb = rb.real();
            }
        }
        return best <= 1e-12 * (std::abs(o.al) + std::abs(o.be) + 1e-300);
    };
    if (p->precision != SG_F64 && !pow2) return SG_OK;
    std::vector<uint32_t> last_word(T, 0u);
    for (int tid = 0; tid < T; ++tid) {
        int j = 0;
        if (own[tid].empty()) return SG_OK;  // (amp_cw2.hip's rows write where the thread's last pair is)
        for (int r : own[tid]) {
            const auto &lst = pair_of[r];
            for (size_t q = 0; q < lst.size(); ++q, ++j) {
                const int i = lst[q];
                const Out &o = out[i];
                uint32_t e = (uint32_t)o.a | CW_VALID;
                if (q == 0) e |= CW_NEWROW;
                if (q + 1 == lst.size()) e |= CW_ENDROW;
                if (r == 0 || 2 * r == P) e |= CW_SELF;
                const size_t c = (size_t)j * T + tid;
                if (p->precision != SG_F64) {
                    uint32_t code = 0;
                    double ma = 0.0, mb = 0.0;
                    if (!polar(o, &code, &ma, &mb)) return SG_OK;  // (not the DCT's coefficients: no split engine)
                    e |= code << CW_OFFSHIFT;
                    gm[2 * c] = (float)ma;
                    gm[2 * c + 1] = (float)mb;
                }
                ka[c] = e;
                rab[2 * c] = 8u * (uint32_t)c2pos(r);
                rab[2 * c + 1] = 8u * (uint32_t)c2pos((P - r) % P);
                if (q + 1 == lst.size()) {  // the pair's row writes (amp_cw2.hip Az rows)
                    wab[2 * c] = 8u * (uint32_t)c2pos(r);
                    wab[2 * c + 1] = (e & CW_SELF) ? 4u * CW2_TRASH : 8u * (uint32_t)c2pos(P - r);
                }
                oi[c] = i;
                last_word[tid] = e & ~(CW_VALID | CW_NEWROW);  // (the padding slots below)
                const float v[8] = {(float)o.c1.real(), (float)o.c1.imag(), (float)o.c2.real(), (float)o.c2.imag(),
                                    (float)o.al.real(), (float)o.al.imag(), (float)o.be.real(), (float)o.be.imag()};
                std::copy(v, v + 4, cf.begin() + 4 * c);
                std::copy(v + 4, v + 8, gf.begin() + 4 * c);
                if (f64) {
                    const double d[8] = {o.c1.real(), o.c1.imag(), o.c2.real(), o.c2.imag(),
                                         o.al.real(), o.al.imag(), o.be.real(), o.be.imag()};
                    std::copy(d, d + 4, cfd.begin() + 4 * c);
                    std::copy(d + 4, d + 8, gfd.begin() + 4 * c);
                    const cd w = tw(o.a, N2);  // S = w_N2^a (amp_cw2d.hip: Horner / rotation step per class)
                    sad[2 * c] = w.real();
                    sad[2 * c + 1] = w.imag();
                }
            }
        }
    }
    // Padding slots (after a thread's pairs; zero coefficients, zero z/phi scale, not VALID) carry the word of
    // the thread's last output without CW_NEWROW: the f32 rows (amp_cw2.hip, C2_ROWS_ALWAYS) write every
    // slot's running sum at its pair's rows, so a padding slot adds 0 to the last pair's sums and writes them
    // again -- never a row of another thread's pair
    if (p->precision != SG_F64)
        for (int tid = 0; tid < T; ++tid)
            for (int j = 0; j < OT; ++j) {
                uint32_t &e = ka[(size_t)j * T + tid];
                if (!(e & CW_VALID)) e = last_word[tid];
            }
    // Which image values the class scatter (Ab, class m2 < Q) and the row
    // writes (Az, entry Q) leave behind, as bits of the thread that reads
    // them in the first FFT stage (c2_stage0_r32: complex index m1 = j + 256 g
    // is value g & 15 of lane half g >> 4 of butterfly j; bit 2 (g & 15) + c)
    std::vector<uint32_t> cmask((size_t)(Q + 1) * T, 0u);
    auto mbit = [&](int m2, int m1, int c) {
        const int j = m1 & 255, g = m1 >> 8;
        const int tid = ((j >> 5) << 6) | ((g >> 4) << 5) | (j & 31);
        cmask[(size_t)m2 * T + tid] |= 1u << (2 * (g & 15) + c);
    };
    for (int m2 = 0; m2 < Q; ++m2)
        for (int q = cls_ptr[m2]; q < cls_ptr[m2 + 1]; ++q) {
            const int loc = (int)(cls_ls[q] & 0xffffu);
            mbit(m2, fsw(loc >> 1), loc & 1);  // fsw is its own inverse
        }
    for (int r : row_k1) {
        mbit(Q, r, 0);
        mbit(Q, r, 1);
    }
    // class tables padded to CW2_SLICE entries per class, the padding pointing
    // at the trash slot (section 0), so the kernels need no range checks
    // (entries re-addressed from the one-workgroup engine's fsw image to the
    // split engine's padded one, c2pos)
    std::vector<uint32_t> cls2((size_t)Q * CW2_SLICE, CW2_TRASH);
    for (int m2 = 0; m2 < Q; ++m2)
        for (int q = cls_ptr[m2]; q < cls_ptr[m2 + 1]; ++q) {
            const uint32_t loc = cls_ls[q] & 0xffffu;
            const uint32_t pl = 2u * (uint32_t)c2pos(fsw((int)(loc >> 1))) + (loc & 1u);
            cls2[(size_t)m2 * CW2_SLICE + (q - cls_ptr[m2])] = (cls_ls[q] & ~0xffffu) | pl;
        }
    SG_TRY(upload(p, &p->c2_cls, cls2));
    {  // image positions alone, two per word (cw2_az's gathers: entries tl + 512 i and tl + 512 (i + 9))
        constexpr int H = CW2_SLICE / 2;
        std::vector<uint32_t> clsp((size_t)Q * H);
        for (int m2 = 0; m2 < Q; ++m2)
            for (int q = 0; q < H; ++q) {
                const uint32_t *c = &cls2[(size_t)m2 * CW2_SLICE];
                clsp[(size_t)m2 * H + q] = (c[q] & 0xffffu) | (c[q + H] << 16);
            }
        SG_TRY(upload(p, &p->c2_clsp, clsp));
    }
    SG_TRY(upload(p, &p->c2_cmask, cmask));
    SG_TRY(upload(p, &p->c2_ka, ka));
    {  // thread-major copy: thread tid's slots at [tid][OTP] (amp_cw2.hip loads them 16 bytes at a time)
        const int OTP = cw2_otp(OT);
        std::vector<uint32_t> kat((size_t)OTP * T, 0u);
        for (int tid = 0; tid < T; ++tid)
            for (int j = 0; j < OT; ++j) kat[(size_t)tid * OTP + j] = ka[(size_t)j * T + tid];
        SG_TRY(upload(p, &p->c2_kat, kat));
    }
    SG_TRY(upload(p, &p->c2_oi, oi));
    SG_TRY(upload(p, &p->c2_wab, wab));
    SG_TRY(upload(p, &p->c2_rab, rab));
    float *dcf = nullptr, *dgf = nullptr;
    SG_TRY(upload(p, &dcf, cf));
    SG_TRY(upload(p, &dgf, gf));
    p->c2_cf = dcf;
    p->c2_gf = dgf;
    SG_TRY(upload(p, &p->c2_gm, gm));
    {  // thread-major copy of (|al|, |be|): thread tid's slots at [tid][OTP][2] (16-byte loads of two slots)
        const int OTP = cw2_otp(OT);
        std::vector<float> gmt((size_t)OTP * T * 2, 0.f);
        for (int tid = 0; tid < T; ++tid)
            for (int j = 0; j < OT; ++j)
                for (int c = 0; c < 2; ++c) gmt[((size_t)tid * OTP + j) * 2 + c] = gm[((size_t)j * T + tid) * 2 + c];
        SG_TRY(upload(p, &p->c2_gmt, gmt));
    }
    p->c2_shoff = pow2 ? ilog2((int)(N / 2)) : 0;
    if (f64) {
        std::vector<double> twp((size_t)P * 2);
        for (int k = 0; k < P; ++k) {
            const cd w = tw(k, P);
            twp[2 * k] = w.real();
            twp[2 * k + 1] = w.imag();
        }
        SG_TRY(upload(p, &p->c2d_cf, cfd));
        SG_TRY(upload(p, &p->c2d_gf, gfd));
        SG_TRY(upload(p, &p->c2d_sa, sad));
        SG_TRY(upload(p, &p->c2d_twp, twp));
    }
    p->cw2OT = OT;
    return SG_OK;
}

// Tables of the regular engine (amp_fused.hip), one transform per column
// block: class order of each block's entries and the needed-row structure of
// the two FFT stages.  Sizes: P = stage-1 FFT length (LDS resident), Q = N2/P.
static Cw2dTables c2dtables(const sg_amp_plan *p);

static int build_regular(sg_amp_plan *p, const uint32_t *order0, const uint32_t *order1,
                         const std::vector<double> &t_scale) {
    const long long N = p->w, N2 = p->N2;
    const int nT = p->nT, Mc = p->Mc, n = p->n, M = p->M;
    const int Lblk = p->L / p->Lc;
    SG_CHECK_ARG(Lblk < 65536, "too many sections per column block (%d)", Lblk);
    const size_t rb = p->precision == SG_F64 ? 8 : 4;
    long long Pmax = p->precision == SG_F64 ? 8192 : 16384;
    // Single-precision single-transform designs whose needed spectrum fits the
    // per-codeword engine's LDS (2 n <= 12288 indices, L <= 1024): P = 8192 and
    // its tables; SG_AMP_ENGINE=staged at plan creation keeps P = 16384
    const char *eng = getenv("SG_AMP_ENGINE");
    if (p->precision == SG_F32 && nT == 1 && 2 * n <= 14 * CW_THREADS && Lblk <= CW_THREADS && N2 >= (1 << 14) &&
        !p->no_cw && !(eng && std::strcmp(eng, "staged") == 0))
        Pmax = 8192;
    if (const char *e = getenv("SG_AMP_PMAX")) Pmax = std::max(8LL, std::min(16384LL, atoll(e)));  // tuning knob
    int P = (int)std::min<long long>(N2, Pmax);
    auto img_bound = [](int P) { return 2 * (P + (P >> 4)); };  // before the classes are known
    while (P > 8 && reg_stage1_lds(img_bound(P), P, Lblk, rb) > 160 * 1024) P >>= 1;
    SG_CHECK_ARG(reg_stage1_lds(img_bound(P), P, Lblk, rb) <= 160 * 1024, "section statistics exceed the LDS budget");
    const int Q = (int)(N2 / P);
    p->rP = P; p->rQ = Q; p->rlog2P = ilog2(P); p->Lblk = Lblk;
    p->rept = reg_ept(P, rb);
    const size_t cxb = 2 * rb;
    p->RB = (int)std::min<size_t>(128, std::max<size_t>(1, 32768 / ((size_t)Q * cxb)));
    SG_CHECK_ARG(256 % p->RB == 0, "row block %d must divide 256", p->RB);

    std::vector<std::vector<int32_t>> row_k1(nT), kptr(nT), kk2(nT), krho(nT), oa(nT), ob(nT), gi(nT);
    std::vector<std::vector<cd>> oc(nT), gc(nT);
    std::vector<int32_t> cls_ptr((size_t)nT * (Q + 1)), cls_j((size_t)nT * Mc), qpos((size_t)nT * Mc);
    std::vector<uint16_t> cls_sec((size_t)nT * Mc), seg((size_t)nT * Q * (Lblk + 1));
    std::vector<uint32_t> cls_ls((size_t)nT * Mc);
    std::vector<int32_t> kidx(N2, -1);
    std::vector<uint8_t> used(N), need(N2);
    for (int t = 0; t < nT; ++t) {
        const uint32_t *o0 = order0 + (size_t)t * n, *o1 = order1 + (size_t)t * Mc;
        // ---- class order of the column block: (class m2, section, j)
        std::fill(used.begin(), used.end(), 0);
        std::vector<int32_t> cnt(Q + 1, 0), m2of(Mc), locof(Mc);
        for (int j = 0; j < Mc; ++j) {
            const long long pos = o1[j];
            SG_CHECK_ARG(pos >= 1 && pos < N, "order1 entry %lld outside [1, w)", pos);
            const long long sl = slot_of_pos(pos, N);
            SG_CHECK_ARG(!used[sl], "order1 has a repeated position");
            used[sl] = 1;
            const long long m = sl >> 1;
            m2of[j] = (int)(m % Q);
            locof[j] = (int)(2 * fsw((int)(m / Q)) + (sl & 1));  // swizzled LDS layout of lds_fft1
            cnt[m2of[j] + 1]++;
        }
        int32_t *cpt = cls_ptr.data() + (size_t)t * (Q + 1);
        cpt[0] = 0;
        for (int c = 0; c < Q; ++c) cpt[c + 1] = cpt[c] + cnt[c + 1];
        std::vector<int32_t> fill(cpt, cpt + Q);
        for (int j = 0; j < Mc; ++j) {  // ascending j: each class sorted by (section, j)
            const int q = fill[m2of[j]]++;
            const size_t o = (size_t)t * Mc + q;
            cls_sec[o] = (uint16_t)(j / M);
            cls_ls[o] = (uint32_t)locof[j] | ((uint32_t)(j / M) << 16);
            cls_j[o] = j;
            qpos[(size_t)t * Mc + j] = q;
        }
        for (int c = 0; c < Q; ++c) {
            uint16_t *sg = seg.data() + ((size_t)t * Q + c) * (Lblk + 1);
            const int q0 = cpt[c], q1 = cpt[c + 1];
            int q = q0;
            for (int l = 0; l <= Lblk; ++l) {
                while (q < q1 && cls_sec[(size_t)t * Mc + q] < l) ++q;
                sg[l] = (uint16_t)(q - q0);
                if (l > 0) p->rmaxseg = std::max(p->rmaxseg, (int)sg[l] - (int)sg[l - 1]);
            }
        }
        // ---- needed N/2-indices: forward outputs = inverse inputs
        std::fill(need.begin(), need.end(), 0);
        std::fill(used.begin(), used.end(), 0);
        for (int i = 0; i < n; ++i) {
            const long long k = o0[i];
            SG_CHECK_ARG(k >= 1 && k < N, "order0 entry %lld outside [1, w)", k);
            SG_CHECK_ARG(!used[k], "order0 has a repeated position");
            used[k] = 1;
            const long long kk = (k <= N2) ? k : N - k;
            need[kk % N2] = 1;
            need[(N2 - kk) % N2] = 1;
        }
        int nk = 0;
        for (int k1 = 0; k1 < P; ++k1) {
            bool any = false;
            for (int k2 = 0; k2 < Q; ++k2) {
                const long long idx = k1 + (long long)P * k2;
                if (!need[idx]) continue;
                if (!any) {
                    row_k1[t].push_back(k1);
                    kptr[t].push_back(nk);
                    any = true;
                }
                kk2[t].push_back(k2);
                krho[t].push_back((int)row_k1[t].size() - 1);
                kidx[idx] = nk++;
            }
        }
        kptr[t].push_back(nk);
        oa[t].resize(n);
        ob[t].resize(n);
        oc[t].resize(2 * (size_t)n);
        for (int i = 0; i < n; ++i) {
            long long a, b;
            cd c1, c2;
            fwd_coef(o0[i], N, N2, t_scale[t], &a, &b, &c1, &c2);
            oa[t][i] = kidx[a];
            ob[t][i] = kidx[b];
            oc[t][2 * i] = c1;
            oc[t][2 * i + 1] = c2;
        }
        gi[t].assign(4 * (size_t)nk, -1);
        gc[t].assign(4 * (size_t)nk, cd(0, 0));
        std::vector<int> ng(nk, 0);
        bool ok = true;
        for (int i = 0; i < n; ++i)
            inv_contrib(o0[i], N, N2, t_scale[t], [&](long long k, cd c) {
                const int kx = kidx[k];
                if (kx < 0 || ng[kx] >= 4) { ok = false; return; }
                gi[t][4 * (size_t)kx + ng[kx]] = i;
                gc[t][4 * (size_t)kx + ng[kx]] = c;
                ng[kx]++;
            });
        SG_CHECK_ARG(ok, "internal: inverse contribution outside the needed set");
        for (int i = 0; i < n; ++i) {  // reset the index map for the next transform
            const long long k = o0[i], kk = (k <= N2) ? k : N - k;
            kidx[kk % N2] = -1;
            kidx[(N2 - kk) % N2] = -1;
        }
    }
    int nRmax = 1, nKmax = 1;
    for (int t = 0; t < nT; ++t) {
        nRmax = std::max(nRmax, (int)row_k1[t].size());
        nKmax = std::max(nKmax, (int)kk2[t].size());
    }
    p->nRmax = nRmax; p->nKmax = nKmax;
    p->nrb = (nRmax + p->RB - 1) / p->RB;
    std::vector<int32_t> nR(nT), f_rk((size_t)nT * nRmax, 0), f_kp((size_t)nT * (nRmax + 1), 0);
    std::vector<int32_t> f_k2((size_t)nT * nKmax, 0), f_kr((size_t)nT * nKmax, 0), f_oa((size_t)nT * n),
        f_ob((size_t)nT * n), f_gi((size_t)nT * nKmax * 4, -1);
    std::vector<cd> f_oc((size_t)nT * n * 2), f_gc((size_t)nT * nKmax * 4, cd(0, 0));
    int maxKb = 0;
    for (int t = 0; t < nT; ++t) {
        const int r = (int)row_k1[t].size(), k = (int)kk2[t].size();
        nR[t] = r;
        std::copy(row_k1[t].begin(), row_k1[t].end(), f_rk.begin() + (size_t)t * nRmax);
        for (int i = 0; i <= nRmax; ++i) f_kp[(size_t)t * (nRmax + 1) + i] = kptr[t][std::min(i, r)];
        std::copy(kk2[t].begin(), kk2[t].end(), f_k2.begin() + (size_t)t * nKmax);
        std::copy(krho[t].begin(), krho[t].end(), f_kr.begin() + (size_t)t * nKmax);
        std::copy(oa[t].begin(), oa[t].end(), f_oa.begin() + (size_t)t * n);
        std::copy(ob[t].begin(), ob[t].end(), f_ob.begin() + (size_t)t * n);
        std::copy(oc[t].begin(), oc[t].end(), f_oc.begin() + (size_t)t * n * 2);
        std::copy(gi[t].begin(), gi[t].end(), f_gi.begin() + (size_t)t * nKmax * 4);
        std::copy(gc[t].begin(), gc[t].end(), f_gc.begin() + (size_t)t * nKmax * 4);
        for (int b = 0; b * p->RB < r; ++b)
            maxKb = std::max(maxKb, kptr[t][std::min(r, (b + 1) * p->RB)] - kptr[t][b * p->RB]);
        (void)k;
    }
    p->maxKb = maxKb;
    std::vector<cd> twP(P), twQ(Q);
    for (int i = 0; i < P; ++i) twP[i] = tw(i, P);
    for (int i = 0; i < Q; ++i) twQ[i] = tw(i, Q);
    // per-stage twiddles of the P-point FFT in thread order (fft.hpp lds_fft1)
    std::vector<cd> stw;
    {
        int radix[8];
        const int ns = fft1_plan(p->rlog2P, p->rept, radix);
        int lns = 0;
        for (int st = 0; st < ns; ++st) {
            const int R = radix[st];
            const long long Ns = 1LL << lns;
            for (long long k = 0; k < Ns; ++k)  // fft.hpp tw_per_k / tw_exp layout
                for (int q = 0; q < tw_per_k(R); ++q) stw.push_back(tw(tw_exp(R, q) * k, Ns * R));
            lns += ilog2(R);
        }
        if (stw.empty()) stw.push_back(cd(1, 0));
    }
    const int nB = (P + 63) / 64;
    p->nB = nB;
    std::vector<cd> twa((size_t)Q * 64), twb((size_t)Q * nB);
    for (int m2 = 0; m2 < Q; ++m2) {
        for (int a = 0; a < 64; ++a) twa[(size_t)m2 * 64 + a] = tw((long long)m2 * a, N2);
        for (int b = 0; b < nB; ++b) twb[(size_t)m2 * nB + b] = tw((long long)m2 * 64 * b, N2);
    }
    SG_TRY(upload(p, &p->r_nR, nR));
    SG_TRY(upload(p, &p->r_row_k1, f_rk));
    {  // stage-1 order: thread tid holds rows tid + i nthr, i < ept, packed in pairs
        const int ept = p->rept, nthr = P / ept;
        SG_CHECK_ARG(P <= 65536 && ept % 2 == 0, "stage-1 FFT length %d exceeds the 16-bit row index", P);
        std::vector<uint32_t> pk((size_t)nT * (P / 2), 0u);
        for (int t = 0; t < nT; ++t) {
            const int nr = (int)row_k1[t].size();
            for (int j = 0; j < ept / 2; ++j)
                for (int tid = 0; tid < nthr; ++tid) {
                    const int r0 = tid + 2 * j * nthr, r1 = r0 + nthr;
                    const uint32_t a = r0 < nr ? (uint32_t)row_k1[t][r0] : 0u, b = r1 < nr ? (uint32_t)row_k1[t][r1] : 0u;
                    pk[(size_t)t * (P / 2) + (size_t)j * nthr + tid] = a | (b << 16);
                }
        }
        SG_TRY(upload(p, &p->r_row_k1p, pk));
    }
    SG_TRY(upload(p, &p->r_kptr, f_kp));
    SG_TRY(upload(p, &p->r_kk2, f_k2));
    SG_TRY(upload(p, &p->r_krho, f_kr));
    SG_TRY(upload(p, &p->r_oa, f_oa));
    SG_TRY(upload(p, &p->r_ob, f_ob));
    SG_TRY(upload_cx(p, &p->r_oc, f_oc));
    SG_TRY(upload(p, &p->r_gi, f_gi));
    SG_TRY(upload_cx(p, &p->r_gc, f_gc));
    for (int t = 0; t < nT; ++t)
        for (int m2 = 0; m2 < Q; ++m2)
            p->rmaxcls = std::max(p->rmaxcls, cls_ptr[(size_t)t * (Q + 1) + m2 + 1] - cls_ptr[(size_t)t * (Q + 1) + m2]);
    p->rimg = (std::max(2 * P, fpad(p->rmaxcls + 16) + 1) + 3) / 4 * 4;
    SG_CHECK_ARG(reg_stage1_lds(p->rimg, P, Lblk, rb) <= 160 * 1024, "a class exceeds the LDS budget");
    SG_TRY(upload(p, &p->r_cls_ptr, cls_ptr));
    SG_TRY(upload(p, &p->r_cls_ls, cls_ls));
    SG_TRY(upload(p, &p->r_cls_j, cls_j));
    SG_TRY(upload(p, &p->r_qpos, qpos));
    SG_TRY(upload(p, &p->r_seg, seg));
    SG_TRY(upload_cx(p, &p->r_twP, twP));
    SG_TRY(upload_cx(p, &p->r_twQ, twQ));
    SG_TRY(upload_cx(p, &p->r_stw, stw));
    SG_TRY(upload_cx(p, &p->r_twa, twa));
    SG_TRY(upload_cx(p, &p->r_twb, twb));
    if (p->precision == SG_F32 && nT == 1 && P == (1 << 13) && Lblk <= CW_THREADS && n <= 8 * CW_THREADS &&
        Q <= 64 && p->rmaxcls <= 9 * CW_THREADS && p->rimg == 2 * P && fpad(p->rmaxcls + 16) < p->rimg)
    {
        SG_TRY(build_cw(p, row_k1[0], kptr[0], kk2[0], f_oa, f_ob, f_gi, f_gc, cls_ptr, cls_ls));
        if (p->cw) SG_TRY(build_cw2(p, order0, t_scale[0], row_k1[0], cls_ptr, cls_ls));
    }
    // double precision: the split engine only (amp_cw2d.hip), its tables built directly; the plan then
    // counts as a per-codeword plan (use_cw), without the companion (f64 keeps P = 8192 either way)
    // (the bounds of amp_cw2d.hip cw2d_launch_iter: its statistics launch takes a section's M <= 512 entries
    // over Q <= 64 class segments in one wavefront, four sections per workgroup)
    if (p->precision == SG_F64 && nT == 1 && P == (1 << 13) && Lblk <= 2 * CW2_THREADS && p->L <= 1024 &&
        p->L % 4 == 0 && M <= 512 && Q % 2 == 0 && Q <= 64 && p->rmaxcls <= CW2_SLICE && !p->no_cw) {
        SG_TRY(build_cw2(p, order0, t_scale[0], row_k1[0], cls_ptr, cls_ls));
        p->cw = p->cw2OT != 0 && cw2d_supported(c2dtables(p));  // else the staged engine, never a decode-time error
    }
    return SG_OK;
}

template <typename T>
static RegTables<T> rtables(const sg_amp_plan *p) {
    RegTables<T> tb;
    tb.nT = p->nT; tb.L = p->L; tb.M = p->M; tb.LM = p->LM; tb.n = p->n; tb.Lc = p->Lc; tb.Mc = p->Mc;
    tb.Lblk = p->Lblk; tb.N2 = p->N2; tb.P = p->rP; tb.Q = p->rQ; tb.log2P = p->rlog2P; tb.ept = p->rept; tb.maxcls = p->rmaxcls; tb.img = p->rimg;
    {
        // measured best at C2: 20000 (f32 staged engine +1.4 %, f64 +0.9 %: profiles/r04_f64_env_sweep.txt)
        const char *st = std::getenv("SG_AMP_STAGGER");
        tb.stagger = st ? std::atoi(st) : 20000;
    }
    tb.nRmax = p->nRmax; tb.nKmax = p->nKmax; tb.RB = p->RB; tb.nrb = p->nrb; tb.maxKb = p->maxKb;
    tb.nR = p->r_nR; tb.row_k1 = p->r_row_k1; tb.row_k1p = p->r_row_k1p; tb.kptr = p->r_kptr; tb.kk2 = p->r_kk2; tb.krho = p->r_krho;
    tb.oa = p->r_oa; tb.ob = p->r_ob; tb.oc = (const cx<T> *)p->r_oc; tb.gi = p->r_gi; tb.gc = (const cx<T> *)p->r_gc;
    tb.cls_ptr = p->r_cls_ptr; tb.cls_ls = p->r_cls_ls; tb.cls_j = p->r_cls_j;
    tb.qpos = p->r_qpos; tb.seg = p->r_seg;
    tb.twP = (const cx<T> *)p->r_twP; tb.twQ = (const cx<T> *)p->r_twQ;
    tb.twHi = (const cx<T> *)p->twHi; tb.twLo = (const cx<T> *)p->twLo;
    tb.stw = (const cx<T> *)p->r_stw; tb.twa = (const cx<T> *)p->r_twa; tb.twb = (const cx<T> *)p->r_twb;
    tb.nB = p->nB;
    tb.skip = diag_skip();
    return tb;
}

static CwTables ctables(const sg_amp_plan *p, int B) {
    CwTables tb;
    tb.L = p->L; tb.M = p->M; tb.LM = p->LM; tb.n = p->n; tb.N2 = p->N2; tb.Q = p->rQ; tb.Lblk = p->Lblk;
    tb.KT = p->cwKT; tb.log2P = p->rlog2P; tb.maxcls = p->rmaxcls; tb.maxseg = p->rmaxseg;
    tb.img = p->rimg;
    tb.cmask = p->c_cmask;
    tb.kt = p->c_kt; tb.oa = p->c_oa; tb.ob = p->c_ob; tb.oc = (const cx<float> *)p->r_oc;
    tb.gi = p->c_gi; tb.gc = (const cx<float> *)p->c_gc;
    tb.cls_ptr = p->r_cls_ptr; tb.cls_ls = p->r_cls_ls; tb.qpos = p->r_qpos; tb.seg = p->r_seg;
    tb.stw = (const cx<float> *)p->c_stw;
    tb.inv_n2 = 1.0f / (float)p->N2;
    // [B][32] stamps, only when the diagnostics buffer holds them
    tb.tprof = (p->tprof && p->tprof_items * 20 >= (size_t)64 * CW2_NP * B) ? p->tprof : nullptr;  // (64 per workgroup)
    return tb;
}

static Cw2Tables c2tables(const sg_amp_plan *p, int B) {
    Cw2Tables tb;
    tb.L = p->L; tb.M = p->M; tb.LM = p->LM; tb.n = p->n; tb.N2 = p->N2; tb.Q = p->rQ; tb.Lblk = p->Lblk;
    tb.OT = p->cw2OT; tb.maxcls = p->rmaxcls;
    // (build_cw2: Q even; the decode loop asks for more than two once codewords have stopped)
    tb.np = p->c2_np >= 4 && CW2_NP >= 4 && p->rQ % 4 == 0 ? 4 : 2;
    tb.inv_n2 = 1.0f / (float)p->N2;
    tb.cmask = p->c2_cmask; tb.ka = p->c2_ka; tb.kat = p->c2_kat; tb.oi = p->c2_oi;
    tb.cf = (const float4 *)p->c2_cf; tb.gf = (const float4 *)p->c2_gf; tb.gm = (const float2 *)p->c2_gm;
    tb.gmt = (const float4 *)p->c2_gmt;
    tb.sh_off = p->c2_shoff; tb.m4n = (uint32_t)(4 * p->w - 1); tb.inv_4n = (float)(1.0 / (4.0 * (double)p->w));
    tb.cls_ptr = p->r_cls_ptr; tb.cls_ls = p->r_cls_ls; tb.cls2 = p->c2_cls; tb.clsp = p->c2_clsp; tb.qpos = p->r_qpos; tb.seg = p->r_seg;
    tb.xr = (float *)p->ws_c2xp; tb.vz = (float *)p->ws_c2vz; tb.ys = (float *)p->ws_c2ys; tb.zs = (float *)p->ws_c2zs; tb.wab = (const uint2 *)p->c2_wab; tb.rab = (const uint2 *)p->c2_rab; tb.part = (float4 *)p->ws_c2part;
    // [2 B][64] stamps, only when the diagnostics buffer holds them (build_cw2
    // accepts any even Q, and B * Q * 20 < 128 B for Q < 7)
    tb.tprof = (p->tprof && p->tprof_items * 20 >= (size_t)128 * B) ? p->tprof : nullptr;
    return tb;
}

// The split engine (amp_cw2.hip) runs the per-codeword engine's iterations
// when its tables were built; SG_AMP_CW2=0 keeps the one-workgroup form
// (A/B tests).
static Cw2dTables c2dtables(const sg_amp_plan *p) {
    Cw2dTables tb;
    tb.L = p->L; tb.M = p->M; tb.LM = p->LM; tb.n = p->n; tb.N2 = p->N2; tb.Q = p->rQ; tb.Lblk = p->Lblk;
    tb.OT = p->cw2OT; tb.maxcls = p->rmaxcls;
    tb.cmask = p->c2_cmask; tb.ka = p->c2_ka; tb.kat = p->c2_kat; tb.oi = p->c2_oi;
    tb.cf = p->c2d_cf; tb.gf = p->c2d_gf; tb.sa = p->c2d_sa; tb.twp = p->c2d_twp;
    tb.cls_ptr = p->r_cls_ptr; tb.cls2 = p->c2_cls; tb.qpos = p->r_qpos; tb.seg = p->r_seg;
    tb.xr = (double *)p->ws_c2xp; tb.vz = (double *)p->ws_c2vz; tb.ys = (double *)p->ws_c2ys;
    tb.zs = (double *)p->ws_c2zs; tb.beta = (double *)p->ws_c2beta; tb.sec = (double *)p->ws_c2sec;
    return tb;
}

static bool use_cw2(const sg_amp_plan *p) {
    if (!p->cw2OT) return false;
    const char *e = std::getenv("SG_AMP_CW2");
    return !(e && std::strcmp(e, "0") == 0);
}

// Engine choice for a decode of B codewords: the per-codeword engine keeps
// one workgroup per codeword, so it wants a batch that fills the CUs.
// SG_AMP_ENGINE=cw / staged forces either at decode time (tests, A/B).
static bool use_cw(const sg_amp_plan *p, int B) {
    if (!p->cw) return false;
    const char *e = std::getenv("SG_AMP_ENGINE");
    if (e && std::strcmp(e, "cw") == 0) return true;
    if (e && std::strcmp(e, "staged") == 0) return false;
    // one workgroup per codeword and CU: worth it when the batch fills whole
    // waves of the CUs (at B = CUs it is ~11 % ahead of the staged engine,
    // which keeps every CU busy at any B)
    const int cu = std::max(device_cu_count(), 1);
    const int waves = (B + cu - 1) / cu;
    return B >= cu && (double)B / ((double)waves * cu) >= 0.9;
}

// The plan a decode of B codewords runs on: the companion P = 16384 plan when
// the automatic choice is the staged engine from the first iteration (the
// SG_AMP_ENGINE overrides keep the plan itself, for same-table A/B tests).
static sg_amp_plan *decode_plan(sg_amp_plan *p, int B) {
    if (!p->alt) return p;
    const char *e = std::getenv("SG_AMP_ENGINE");
    if (e && (std::strcmp(e, "cw") == 0 || std::strcmp(e, "staged") == 0)) return p;
    return use_cw(p, B) ? p : p->alt;
}

template <typename T>
static RegBufs<T> rbufs(const sg_amp_plan *p, int B, const void *y) {
    RegBufs<T> bf;
    bf.B = B; bf.mode = 0;
    bf.s = (T *)p->ws_s; bf.tu = (cx<T> *)p->ws_tu; bf.xn = (cx<T> *)p->ws_xn; bf.part = (T *)p->ws_part;
    bf.stM = (T *)p->ws_stM; bf.stI = (T *)p->ws_stI;
    bf.y = (const T *)(y ? y : p->ws_y); bf.z = (T *)p->ws_z;
    bf.phi = p->ws_phi; bf.tau = p->ws_tau; bf.tau_prev = p->ws_tau_prev; bf.active = p->ws_active;
    bf.true_idx = nullptr; bf.map = p->ws_argmax; bf.ext_in = nullptr; bf.ext_out = nullptr;
    bf.tprof_ab = bf.tprof_az = bf.trt_ab = bf.trt_az = nullptr;
    if (p->tprof && (size_t)B * p->nT * p->rQ <= p->tprof_items) {
        bf.tprof_ab = p->tprof;
        bf.tprof_az = p->tprof + p->tprof_items * 8;
        bf.trt_ab = p->tprof + p->tprof_items * 16;
        bf.trt_az = p->tprof + p->tprof_items * 18;
    }
    return bf;
}

// Tables of the block engine (amp_block.hip): per transform, the LDS position
// of every column entry, the output gathers and the G slots, all in the
// natural-order FFT image in the padded layout (fft.hpp ppos).
static int build_block(sg_amp_plan *p, const uint32_t *order0, const uint32_t *order1,
                       const std::vector<double> &t_scale, const std::vector<int32_t> &row_of) {
    const long long N = p->w, N2 = p->N2;
    const int nT = p->nT, Mc = p->Mc, Mr = p->Mr;
    std::vector<uint16_t> gloc;
    std::vector<uint32_t> pos2((size_t)nT * 8 * 1024, 0u);
    std::vector<uint32_t> oab((size_t)nT * Mr);
    std::vector<cd> oc((size_t)nT * Mr * 8), gc;
    std::vector<int32_t> gptr(nT + 1, 0), gi, grow;
    for (int t = 0; t < nT; ++t) {
        const uint32_t *o0 = order0 + (size_t)t * Mr, *o1 = order1 + (size_t)t * Mc;
        for (int j = 0; j < Mc; ++j) {
            const long long sl = slot_of_pos(o1[j], N);
            const uint32_t lds = (uint32_t)(2 * ppos((int)(sl >> 1)) + (int)(sl & 1));
            SG_CHECK_ARG(lds < 65536u, "internal: padded LDS index beyond 16 bits");
            // owner (thread, entry) of column entry j: amp_block.hip bk_j
            const int M = p->M, eps = M / 64, spw = 1024 / M;
            const int l = j / M, rr = j % M;
            const int tid = (l / spw) * 64 + rr / eps, i = (l % spw) * eps + rr % eps;
            pos2[((size_t)t * 8 + i / 2) * 1024 + tid] |= lds << (16 * (i & 1));
        }
        std::vector<std::vector<std::pair<int, cd>>> gcon(N2);
        for (int i = 0; i < Mr; ++i) {
            long long a, b;
            cd c1, c2;
            fwd_coef(o0[i], N, N2, t_scale[t], &a, &b, &c1, &c2);
            // amp_block.hip blk_ab: the radix-4 stage of bins a, b folded into the output
            oab[(size_t)t * Mr + i] = (uint32_t)(a % 4096) | ((uint32_t)(b % 4096) << 16);
            for (int q = 0; q < 4; ++q) {
                oc[((size_t)t * Mr + i) * 8 + q] = c1 * tw((long long)q * a, N2);
                oc[((size_t)t * Mr + i) * 8 + 4 + q] = c2 * std::conj(tw((long long)q * b, N2));
            }
            inv_contrib(o0[i], N, N2, t_scale[t], [&](long long k, cd c) { gcon[k].push_back({i, c}); });
        }
        for (int k = 0; k < N2; ++k) {
            if (gcon[k].empty()) continue;
            SG_CHECK_ARG(gcon[k].size() <= 4, "internal: >4 contributions to one G slot");
            gloc.push_back((uint16_t)ppos(k));
            grow.push_back(row_of[t]);
            for (int q = 0; q < 4; ++q) {
                if (q < (int)gcon[k].size()) { gi.push_back(gcon[k][q].first); gc.push_back(gcon[k][q].second); }
                else { gi.push_back(-1); gc.push_back(cd(0, 0)); }
            }
        }
        gptr[t + 1] = (int32_t)gloc.size();
    }
    std::vector<cd> stw;  // per-stage twiddles of the N2-point FFT (fft.hpp lds_fft1_ct, EPT 16)
    {
        int radix[8];
        const int ns = fft1_plan(ilog2((int)N2), 16, radix);
        int lns = 0;
        for (int st = 0; st < ns; ++st) {
            const int R = radix[st];
            const long long Ns = 1LL << lns;
            for (long long k = 0; k < Ns; ++k)
                for (int q = 0; q < tw_per_k(R); ++q) stw.push_back(tw(tw_exp(R, q) * k, Ns * R));
            lns += ilog2(R);
        }
    }
    SG_TRY(upload(p, &p->b_pos2, pos2));
    SG_TRY(upload(p, &p->b_oab, oab));
    SG_TRY(upload_cx(p, &p->b_oc, oc));
    SG_TRY(upload(p, &p->b_gptr, gptr));
    SG_TRY(upload(p, &p->b_grow, grow));
    p->b_ngs = gptr[nT];
    SG_TRY(upload(p, &p->b_gloc, gloc));
    SG_TRY(upload(p, &p->b_gi, gi));
    SG_TRY(upload_cx(p, &p->b_gc, gc));
    SG_TRY(upload_cx(p, &p->b_stw, stw));
    SG_CHECK_ARG(blk_lds_bytes(Mc) <= 160 * 1024, "block engine LDS budget");
    return SG_OK;
}

// Tables of the two-class block engine (amp_block2.hip): N2 = 2 P with P = 2^14
// (w = 2^16) or 2^13 (w = 2^15).  Column entry j sits at packed slot
// m = 2 m1 + m2 of its transform: class m2, real LDS index 2 ppos(m1) +
// component in the class image; owned by (thread, entry) as b2_j.  Output
// coefficients per class fold the class factor w_N2^(m2 k) and the last
// radix-RF stage (RF = P / 4096): al = c1 w_N2^((m2 + 2 r) a).
static int build_block2(sg_amp_plan *p, const uint32_t *order0, const uint32_t *order1,
                        const std::vector<double> &t_scale, const std::vector<int32_t> &row_of) {
    const long long N = p->w, N2 = p->N2;
    const int nT = p->nT, Mc = p->Mc, Mr = p->Mr, M = p->M;
    const int LP = p->b2_log2p, T = (1 << LP) / 16, RF = (1 << LP) / 4096;  // amp_block2.hip B2G
    constexpr int J = 32;
    SG_CHECK_ARG((LP == 13 || LP == 14) && N2 == 2LL << LP && Mc == 2 << LP, "internal: two-class geometry");
    // per (transform, class): the real LDS index 2 ppos(m1) + component of each column entry of the class in
    // the padded image, the trash slot (a padding slot, amp_block2.hip B2_TRASH) for the other class's entries
    constexpr uint32_t TRASH = 2 * 32;
    static_assert(ppos(32) == 33, "complex position 32 is a padding slot");
    std::vector<uint32_t> pos2((size_t)nT * 2 * (J / 2) * T, TRASH | (TRASH << 16));
    std::vector<uint32_t> pos1((size_t)nT * (J / 2) * T, 0u);  // one-table form (amp_block2.hip B2_ONETABLE)
    std::vector<uint32_t> oab((size_t)nT * Mr);
    std::vector<cd> oc((size_t)nT * 2 * Mr * 8), gc;
    std::vector<int32_t> gptr(nT + 1, 0), gi, grow, gk;
    std::vector<uint16_t> gloc;
    const int eps = M / 64, spw = 2048 / M;
    for (int t = 0; t < nT; ++t) {
        const uint32_t *o0 = order0 + (size_t)t * Mr, *o1 = order1 + (size_t)t * Mc;
        for (int j = 0; j < Mc; ++j) {
            const long long sl = slot_of_pos(o1[j], N);
            const long long m = sl >> 1;
            const uint32_t lds = (uint32_t)(2 * ppos((int)(m >> 1)) + (int)(sl & 1));
            SG_CHECK_ARG(lds < 65536u, "internal: padded LDS index beyond 16 bits");
            const int l = j / M, rr = j % M;
            const int tid = (l / spw) * 64 + rr / eps, i = (l % spw) * eps + rr % eps;
            uint32_t &w = pos2[(((size_t)t * 2 + (m & 1)) * (J / 2) + i / 2) * T + tid];
            w = (w & ~(0xffffu << (16 * (i & 1)))) | (lds << (16 * (i & 1)));
            const uint32_t e1 = (uint32_t)((m >> 1) << 2) | (uint32_t)((sl & 1) << 1) | (uint32_t)(m & 1);
            SG_CHECK_ARG((m >> 1) < (1LL << 14), "internal: one-table entry beyond 16 bits");
            pos1[((size_t)t * (J / 2) + i / 2) * T + tid] |= e1 << (16 * (i & 1));
        }
        std::vector<std::vector<std::pair<int, cd>>> gcon(N2);
        for (int i = 0; i < Mr; ++i) {
            long long a, b;
            cd c1, c2;
            fwd_coef(o0[i], N, N2, t_scale[t], &a, &b, &c1, &c2);
            oab[(size_t)t * Mr + i] = (uint32_t)(a % 4096) | ((uint32_t)(b % 4096) << 16);
            for (int m2 = 0; m2 < 2; ++m2)
                for (int r = 0; r < RF; ++r) {  // (the last radix-RF stage folded in; RF = 2 leaves 4 zeros)
                    cd *o = &oc[(((size_t)t * 2 + m2) * Mr + i) * 8];
                    o[r] = c1 * tw((long long)(m2 + 2 * r) * a, N2);
                    o[4 + r] = c2 * std::conj(tw((long long)(m2 + 2 * r) * b, N2));
                }
            inv_contrib(o0[i], N, N2, t_scale[t], [&](long long k, cd c) { gcon[k].push_back({i, c}); });
        }
        for (int k = 0; k < N2; ++k) {
            if (gcon[k].empty()) continue;
            SG_CHECK_ARG(gcon[k].size() <= 4, "internal: >4 contributions to one G slot");
            gk.push_back(k);
            gloc.push_back((uint16_t)ppos(k & (int)(N2 / 2 - 1)));  // (blk2_az computes it from gk)
            grow.push_back(row_of[t]);
            for (int q = 0; q < 4; ++q) {
                if (q < (int)gcon[k].size()) { gi.push_back(gcon[k][q].first); gc.push_back(gcon[k][q].second); }
                else { gi.push_back(-1); gc.push_back(cd(0, 0)); }
            }
        }
        gptr[t + 1] = (int32_t)gk.size();
    }
    std::vector<cd> stw;  // stage twiddles of the P-point FFT (fft.hpp lds_fft1_ct, EPT 16; unused by the
                          // sine / cosine stages of amp_block2.hip)
    {
        int radix[8];
        const int ns = fft1_plan(LP, 16, radix);
        int lns = 0;
        for (int st = 0; st < ns; ++st) {
            const int R = radix[st];
            const long long Ns = 1LL << lns;
            for (long long k = 0; k < Ns; ++k)
                for (int q = 0; q < tw_per_k(R); ++q) stw.push_back(tw(tw_exp(R, q) * k, Ns * R));
            lns += ilog2(R);
        }
    }
    SG_TRY(upload(p, &p->b_pos2, pos2));
    SG_TRY(upload(p, &p->b_pos1, pos1));
    SG_TRY(upload(p, &p->b_oab, oab));
    SG_TRY(upload_cx(p, &p->b_oc, oc));
    SG_TRY(upload(p, &p->b_gptr, gptr));
    SG_TRY(upload(p, &p->b_grow, grow));
    p->b_ngs = gptr[nT];
    SG_TRY(upload(p, &p->b_gloc, gloc));
    SG_TRY(upload(p, &p->b_gk, gk));
    SG_TRY(upload(p, &p->b_gi, gi));
    SG_TRY(upload_cx(p, &p->b_gc, gc));
    SG_TRY(upload_cx(p, &p->b_stw, stw));
    SG_CHECK_ARG(blk2_lds_bytes(LP) <= 160 * 1024, "block engine LDS budget");
    return SG_OK;
}

static int build_plan(int ndim, const double *W, int Lr_in, int Lc_in, int L, int M, int n, const uint32_t *order0,
                      const uint32_t *order1, int precision, bool no_cw, sg_amp_plan **out) {
    SG_CHECK_ARG(out && W && order0 && order1, "null argument");
    SG_CHECK_ARG(ndim >= 0 && ndim <= 2, "W.ndim must be 0, 1 or 2");
    SG_CHECK_ARG(precision == SG_F32 || precision == SG_F64, "precision must be SG_F32 or SG_F64");
    SG_CHECK_ARG(L > 0 && M > 0 && n > 0 && (M & (M - 1)) == 0, "bad (L, M, n)");
    SG_TRY(ensure_device());
    int Lr = 1, Lc = 1;
    if (ndim == 1) Lc = Lc_in;
    if (ndim == 2) { Lr = Lr_in; Lc = Lc_in; }
    SG_CHECK_ARG(Lr >= 1 && Lc >= 1, "bad base-matrix shape");
    const long long LM = (long long)L * M;
    SG_CHECK_ARG(LM < (1LL << 30), "L*M too large");
    SG_CHECK_ARG(L % Lc == 0, "Lc must divide L");
    SG_CHECK_ARG(ndim != 2 || n % Lr == 0, "Lr must divide n");
    const int Mr = (ndim == 2) ? n / Lr : n;
    const int Mc = (int)(LM / Lc);
    int w = 1;
    while (w < std::max(Mr + 1, Mc + 1)) w <<= 1;  // sparc.py:744
    SG_CHECK_ARG(w >= 16 && w <= (1 << 23), "transform size w=%d outside [16, 2^23]", w);
    std::unique_ptr<sg_amp_plan> p(new sg_amp_plan());
    hipGetDevice(&p->device);
    p->no_cw = no_cw;
    p->precision = precision; p->ndim = ndim; p->L = L; p->M = M; p->LM = (int)LM; p->n = n;
    p->Lr = Lr; p->Lc = Lc; p->Mr = Mr; p->Mc = Mc; p->w = w; p->N2 = w / 2;
    const int lg = ilog2(p->N2);
    p->log2P = lg / 2; p->log2Q = lg - p->log2P;
    p->P = 1 << p->log2P; p->Q = 1 << p->log2Q;
    p->npairs = p->P / 2 + 1;
    p->W.assign(W, W + (ndim == 0 ? 1 : (size_t)Lr * Lc));
    // transforms = nonzero blocks in row-major order (sparc.py:758-771)
    std::vector<int32_t> t_row, t_col;
    std::vector<double> t_scale;
    for (int r = 0; r < Lr; ++r)
        for (int c = 0; c < Lc; ++c) {
            const double wv = (ndim == 0) ? p->W[0] : p->W[(size_t)r * Lc + c];
            if (wv != 0.0) {
                t_row.push_back(r); t_col.push_back(c);
                t_scale.push_back(std::sqrt(wv / L));  // np.sqrt(W/L)
            }
        }
    p->nT = (int)t_row.size();
    SG_CHECK_ARG(p->nT > 0, "base matrix is all zero");
    std::vector<int32_t> col_ptr(Lc + 1, 0), col_t, row_ptr(Lr + 1, 0), row_t;
    for (int c = 0; c < Lc; ++c) {
        for (int t = 0; t < p->nT; ++t)
            if (t_col[t] == c) col_t.push_back(t);
        col_ptr[c + 1] = (int32_t)col_t.size();
    }
    for (int r = 0; r < Lr; ++r) {
        for (int t = 0; t < p->nT; ++t)
            if (t_row[t] == r) row_t.push_back(t);
        row_ptr[r + 1] = (int32_t)row_t.size();
    }
    // one transform per column block: the regular engine (amp_fused.hip);
    // SG_AMP_ENGINE=legacy keeps the general four-step path for comparison
    const char *eng = std::getenv("SG_AMP_ENGINE");
    // (the per-section softmax statistics of a column block must fit in LDS
    // beside the stage-1 FFT: at most 2048 (f64) / 4096 (f32) sections)
    const size_t sec_bytes = (size_t)2 * (L / Lc) * (precision == SG_F64 ? 8 : 4);
    p->regular = ndim <= 1 && p->nT == Lc && sec_bytes <= 32 * 1024 && !(eng && std::strcmp(eng, "legacy") == 0);
    // several transforms per column block, each small enough for one
    // workgroup's LDS: the block engine (single precision, w = 2^15)
    const bool no_blk = eng && (std::strcmp(eng, "legacy") == 0 || std::strcmp(eng, "general") == 0);
    // w = 2^15 with Mc = 2^14 (C4): the single-class engine (one 1024-thread workgroup per CU, 132 KB of LDS);
    // SG_AMP_BLOCK=two-class selects the two-class form at P = 2^13 (two 512-thread workgroups per CU), which
    // measured no faster (block engine)
    const char *bk = std::getenv("SG_AMP_BLOCK");
    const bool single = !(bk && std::strcmp(bk, "two-class") == 0);
    const bool c4 = !p->regular && precision == SG_F32 && p->N2 == (1 << 14) && Mc == (1 << 14) && M >= 64 && !no_blk;
    p->block = c4 && single && M <= 1024 && Mr < 65536;
    // w = 2^16 with Mc = 2^15 (the notebook geometry): the two-class form at P = 2^14
    const bool nb = !p->regular && precision == SG_F32 && p->N2 == (1 << 15) && Mc == (1 << 15) && M >= 64 &&
                    M <= 2048 && Mr <= 1024 && !no_blk;
    p->block2 = (c4 && !single && M <= 2048 && Mr <= 512) || nb;
    p->b2_log2p = p->block2 ? (nb ? 14 : 13) : 0;
    const int N = w, N2 = p->N2, P = p->P, Q = p->Q, np1 = p->npairs + 1;
    auto slot_of = [&](long long pos) -> long long {  // w-space slot of position pos
        return (pos % 2 == 0) ? pos / 2 : (long long)N - 1 - (pos - 1) / 2;
    };
    auto pair_of = [&](long long k) -> int {  // row pair of an N2-index
        const int row = (int)(k % P);
        return row <= P / 2 ? row : P - row;
    };
    auto local_of = [&](long long k) -> uint32_t {  // LDS index of N2-index k inside its pair's two rows
        const int row = (int)(k % P);
        const int pr = row <= P / 2 ? row : P - row;
        const int half = (row == pr) ? 0 : 1;
        return (uint32_t)(half * Q + (int)(k / P));
    };
    std::vector<int32_t> inmap((size_t)p->nT * N, -1), outslot((size_t)p->nT * Mc);
    std::vector<int32_t> rp_ptr((size_t)p->nT * np1), rp_i;
    std::vector<uint32_t> rp_ab;
    std::vector<cd> rp_c;
    std::vector<int32_t> gs_ptr((size_t)p->nT * np1), gs_loc, gs_i;
    std::vector<cd> gs_c;
    for (int t = 0; t < p->nT && !p->regular; ++t) {
        const uint32_t *o0 = order0 + (size_t)t * Mr, *o1 = order1 + (size_t)t * Mc;
        int32_t *im = inmap.data() + (size_t)t * N;
        for (int j = 0; j < Mc; ++j) {
            const long long pos = o1[j];
            SG_CHECK_ARG(pos >= 1 && pos < N, "order1 entry %lld outside [1, w)", pos);
            const long long sl = slot_of(pos);
            SG_CHECK_ARG(im[sl] < 0, "order1 has a repeated position");
            im[sl] = j;
            outslot[(size_t)t * Mc + j] = (int32_t)sl;
        }
        const double sc = t_scale[t];
        // ---- forward outputs X[k], k = order0[i], grouped by row pair
        std::vector<std::vector<int>> by_pair(p->npairs);
        std::vector<int> seen0(N, 0);
        for (int i = 0; i < Mr; ++i) {
            const long long k = o0[i];
            SG_CHECK_ARG(k >= 1 && k < N, "order0 entry %lld outside [1, w)", k);
            SG_CHECK_ARG(!seen0[k], "order0 has a repeated position");
            seen0[k] = 1;
            const long long kk = (k <= N2) ? k : N - k;
            by_pair[pair_of(kk % N2)].push_back(i);
        }
        for (int pr = 0; pr < p->npairs; ++pr) {
            rp_ptr[(size_t)t * np1 + pr] = (int32_t)rp_i.size();
            for (int i : by_pair[pr]) {
                long long a, b;
                cd c1, c2;
                fwd_coef(o0[i], N, N2, sc, &a, &b, &c1, &c2);
                rp_i.push_back(i);
                rp_ab.push_back(local_of(a) | (local_of(b) << 16));
                rp_c.push_back(c1);
                rp_c.push_back(c2);
            }
        }
        rp_ptr[(size_t)t * np1 + p->npairs] = (int32_t)rp_i.size();
        // ---- inverse inputs: G[k] = A_k y[k] - i A_k y[N-k] + C_k y[N2+k] - i C_k y[N2-k]
        std::vector<std::vector<std::pair<int, cd>>> gcon(N2);
        for (int i = 0; i < Mr; ++i)
            inv_contrib(o0[i], N, N2, sc, [&](long long k, cd c) { gcon[k].push_back({i, c}); });
        std::vector<std::vector<int>> slots_by_pair(p->npairs);
        for (int k = 0; k < N2; ++k)
            if (!gcon[k].empty()) slots_by_pair[pair_of(k)].push_back(k);
        for (int pr = 0; pr < p->npairs; ++pr) {
            gs_ptr[(size_t)t * np1 + pr] = (int32_t)gs_loc.size();
            for (int k : slots_by_pair[pr]) {
                SG_CHECK_ARG(gcon[k].size() <= 4, "internal: >4 contributions to one G slot");
                gs_loc.push_back((int32_t)local_of(k));
                for (int q = 0; q < 4; ++q) {
                    if (q < (int)gcon[k].size()) { gs_i.push_back(gcon[k][q].first); gs_c.push_back(gcon[k][q].second); }
                    else { gs_i.push_back(-1); gs_c.push_back(cd(0, 0)); }
                }
            }
        }
        gs_ptr[(size_t)t * np1 + p->npairs] = (int32_t)gs_loc.size();
    }
    std::vector<cd> twP(P), twQ(Q), twHi((N2 + 1023) / 1024), twLo(std::min(N2, 1024));
    for (int i = 0; i < P; ++i) twP[i] = tw(i, P);
    for (int i = 0; i < Q; ++i) twQ[i] = tw(i, Q);
    for (size_t i = 0; i < twHi.size(); ++i) twHi[i] = tw((long long)i * 1024, N2);
    for (size_t i = 0; i < twLo.size(); ++i) twLo[i] = tw((long long)i, N2);
    std::vector<double> Wd = p->W;
    sg_amp_plan *pp = p.release();
    int rc = [&]() -> int {
    SG_TRY(upload(pp, &pp->t_row, t_row));
    SG_TRY(upload(pp, &pp->t_col, t_col));
    SG_TRY(upload(pp, &pp->col_ptr, col_ptr));
    SG_TRY(upload(pp, &pp->col_t, col_t));
    SG_TRY(upload(pp, &pp->row_ptr, row_ptr));
    SG_TRY(upload(pp, &pp->row_t, row_t));
    SG_TRY(upload(pp, &pp->inmap, inmap));
    SG_TRY(upload(pp, &pp->outslot, outslot));
    SG_TRY(upload(pp, &pp->rp_ptr, rp_ptr));
    SG_TRY(upload(pp, &pp->rp_i, rp_i));
    SG_TRY(upload(pp, &pp->rp_ab, rp_ab));
    SG_TRY(upload_cx(pp, &pp->rp_c, rp_c));
    SG_TRY(upload(pp, &pp->gs_ptr, gs_ptr));
    SG_TRY(upload(pp, &pp->gs_loc, gs_loc));
    SG_TRY(upload(pp, &pp->gs_i, gs_i));
    SG_TRY(upload_cx(pp, &pp->gs_c, gs_c));
    SG_TRY(upload_cx(pp, &pp->twP, twP));
    SG_TRY(upload_cx(pp, &pp->twQ, twQ));
    SG_TRY(upload_cx(pp, &pp->twHi, twHi));
    SG_TRY(upload_cx(pp, &pp->twLo, twLo));
    SG_TRY(upload(pp, &pp->dW, Wd));
    if (pp->regular) SG_TRY(build_regular(pp, order0, order1, t_scale));
    if (pp->block) SG_TRY(build_block(pp, order0, order1, t_scale, t_row));
    if (pp->block2) SG_TRY(build_block2(pp, order0, order1, t_scale, t_row));
    return SG_OK;
    }();
    if (rc != SG_OK) {
        sg_amp_plan_destroy(pp);
        return rc;
    }
    *out = pp;
    return SG_OK;
}

// Active-flag poll, one iteration behind the launches: the copy of the flags
// after iteration t is requested behind t's launches, iteration t + 1 is
// launched, and only then does the host wait for the copy -- the GPU works on
// t + 1 meanwhile, so the poll leaves no idle gap on the stream (a synchronous
// poll cost ~40 us of idle GPU each time, profiles/README.md).  Decisions
// taken from the flags after t apply from iteration t + 2 on, at every run and
// rank count alike (the decode stays deterministic).
struct ActivePoll {
    sg_amp_plan *p;
    int B;
    hipStream_t s;
    bool pending = false;
    int request() {  // behind the launches already on the stream
        if (!p->poll_ev) SG_HIP(hipEventCreateWithFlags(&p->poll_ev, hipEventDisableTiming));
        if (p->h_active_cap < B) {
            if (p->h_active) {
                SG_HIP(hipEventSynchronize(p->poll_ev));
                SG_HIP(hipHostFree(p->h_active));
                p->h_active = nullptr;
            }
            SG_HIP(hipHostMalloc((void **)&p->h_active, sizeof(int32_t) * B, hipHostMallocDefault));
            p->h_active_cap = B;
        }
        SG_HIP(hipMemcpyAsync(p->h_active, p->ws_active, sizeof(int32_t) * B, hipMemcpyDeviceToHost, s));
        SG_HIP(hipEventRecord(p->poll_ev, s));
        pending = true;
        return SG_OK;
    }
    // the number of active codewords at the last request (-1: none pending)
    int collect(int *n_active) {
        *n_active = -1;
        if (!pending) return SG_OK;
        SG_HIP(hipEventSynchronize(p->poll_ev));
        pending = false;
        int na = 0;
        for (int b = 0; b < B; ++b) na += p->h_active[b] != 0;
        *n_active = na;
        return SG_OK;
    }
};

template <typename T>
static int decode_regular(sg_amp_plan *p, const void *d_y, int B, const int32_t *d_true, double awgn_var, int t_max,
                          double rtol, int phi_method, int32_t *d_map, int32_t *d_tfinal, double *d_nmse,
                          double *d_psi, hipStream_t s) {
    SG_TRY(ensure_ws(p, B, t_max));
    RegTables<T> tb = rtables<T>(p);
    RegBufs<T> bf = rbufs<T>(p, B, d_y);
    bf.true_idx = d_true;
    AmpScalars sc;
    sc.psi = p->ws_psi; sc.psi_prev = p->ws_psi_prev; sc.phi_prev = p->ws_phi_prev; sc.gamma = p->ws_gamma;
    sc.bcoef = p->ws_bco; sc.nmse = p->ws_nmse; sc.t_final = p->ws_tfinal;
    AmpParams pr;
    pr.W = p->dW; pr.awgn_var = awgn_var; pr.rtol = rtol;
    pr.atol = 2e-15;  // 2*np.finfo(float).resolution, sparc.py:916
    pr.phi_method = phi_method; pr.t_max = t_max;
    SG_TRY(reg_launch_init(B, p->Lc, t_max, p->ws_nmse, p->ws_active, p->ws_tfinal, s));
    ActivePoll poll{p, B, s};
    // f32 split engine: two workgroups per codeword (each half of the classes) while every codeword is active;
    // once the active-flag poll shows stopped codewords, four, so the dispatcher refills the CU slots of the
    // stopped ones (same box: R = 1.3 +4 %, profiles/r06_c2_parts_ab.txt; four from the start cost the
    // all-active R = 1.5 line 0.2-0.8 %: the control kernel sums twice the parts)
    p->c2_np = 2;
    // (double precision has the split engine only: SG_AMP_CW2=0 leaves it the staged engine)
    bool cw = use_cw(p, B) && (std::is_same<T, float>::value || use_cw2(p));
    p->last_engine = cw ? 2 : 1;
    p->last_handover = -1;
    const char *eng = std::getenv("SG_AMP_ENGINE");
    const bool cw_forced = eng && std::strcmp(eng, "cw") == 0;
    double handover = 0.5;  // active fraction below which the staged engine takes over
    if (const char *h = std::getenv("SG_AMP_HANDOVER"))  // tuning knob, clamped to [0, 1]
        handover = std::min(1.0, std::max(0.0, atof(h)));
    for (int t = 0; t < t_max - 1; ++t) {
        if constexpr (std::is_same<T, float>::value) {
            if (cw) {
                if (use_cw2(p)) SG_TRY(cw2_launch_iter(c2tables(p, B), bf, sc, pr, t, s));
                else SG_TRY(cw_launch_iter(ctables(p, B), bf, sc, pr, t, s));
            }
        } else {
            if (cw) SG_TRY(cw2d_launch_iter(c2dtables(p), bf, sc, pr, t, s));
        }
        if (!cw) {
            if (t > 0) SG_TRY(reg_launch_ab<T>(tb, bf, s));
            SG_TRY(reg_launch_ctrl0<T>(tb, bf, sc, pr, t, s));
            SG_TRY(reg_launch_az<T>(tb, bf, t, s));
            SG_TRY(reg_launch_merge<T>(tb, bf, sc, pr, t, s));
        }
        // Poll the active flags (after iterations 3, 7, 11, ..., read one
        // iteration later, ActivePoll): stop once every codeword has stopped,
        // and hand the remaining iterations to the staged engine once half of
        // the batch has stopped -- the per-codeword engine keeps one CU per
        // codeword, so stopped codewords leave CUs idle, while the staged
        // engine spreads the active ones over every CU.  Both keep the same
        // state (s in class order, section statistics, scalars), so the
        // switch is seamless.
        int na = -1;
        SG_TRY(poll.collect(&na));  // the flags after iteration t - 1
        if (na == 0) break;
        if (na > 0 && na < B && C2_PARTS_ADAPT) p->c2_np = 4;
        if (na > 0 && cw && !cw_forced && na < handover * B) {
            cw = false;
            p->last_handover = t + 1;  // first iteration on the staged engine
            if constexpr (std::is_same<T, float>::value)  // (the split engine keeps z in slot order only)
                if (use_cw2(p)) SG_TRY(cw2_launch_z_natural(c2tables(p, B), bf, s));
        }
        if (t % 4 == 3 && t + 2 < t_max - 1 && !tb.skip) SG_TRY(poll.request());
    }
    if (poll.pending) SG_HIP(hipEventSynchronize(p->poll_ev));
    SG_HIP(hipMemsetAsync(p->ws_argmax, 0x7f, sizeof(int32_t) * B * p->L, s));
    SG_TRY(reg_launch_map<T>(tb, bf, s));
    if (d_map) SG_HIP(hipMemcpyAsync(d_map, p->ws_argmax, sizeof(int32_t) * B * p->L, hipMemcpyDeviceToDevice, s));
    if (d_tfinal) SG_HIP(hipMemcpyAsync(d_tfinal, p->ws_tfinal, sizeof(int32_t) * B, hipMemcpyDeviceToDevice, s));
    if (d_nmse) SG_HIP(hipMemcpyAsync(d_nmse, p->ws_nmse, sizeof(double) * B * t_max * p->Lc, hipMemcpyDeviceToDevice, s));
    if (d_psi) SG_HIP(hipMemcpyAsync(d_psi, p->ws_psi, sizeof(double) * B * p->Lc, hipMemcpyDeviceToDevice, s));
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
static int decode_impl(sg_amp_plan *p, const void *d_y, int B, const int32_t *d_true, double awgn_var, int t_max,
                       double rtol, int phi_method, int32_t *d_map, int32_t *d_tfinal, double *d_nmse, double *d_psi,
                       hipStream_t s) {
    if (p->regular)
        return decode_regular<T>(p, d_y, B, d_true, awgn_var, t_max, rtol, phi_method, d_map, d_tfinal, d_nmse,
                                 d_psi, s);
    SG_TRY(ensure_ws(p, B, t_max));
    AmpTables<T> tb = tables<T>(p);
    AmpBufs<T> bf = bufs<T>(p, B, d_y);
    bf.true_idx = d_true;
    AmpScalars sc;
    sc.psi = p->ws_psi; sc.psi_prev = p->ws_psi_prev; sc.phi_prev = p->ws_phi_prev; sc.gamma = p->ws_gamma;
    sc.bcoef = p->ws_bco; sc.nmse = p->ws_nmse; sc.t_final = p->ws_tfinal;
    AmpParams pr;
    pr.W = p->dW; pr.awgn_var = awgn_var; pr.rtol = rtol;
    pr.atol = 2e-15;  // 2*np.finfo(float).resolution, sparc.py:916
    pr.phi_method = phi_method; pr.t_max = t_max;
    const size_t rs = sizeof(T);
    SG_HIP(hipMemsetAsync(p->ws_beta, 0, (size_t)B * p->LM * rs, s));
    SG_TRY(amp_launch_control<T>(tb, bf, sc, pr, 2, 0, s));
    ActivePoll poll{p, B, s};
    const bool blk =(p->block || p->block2) && sizeof(T) == 4;
    const BlkTables bt = blk ? btables(p) : BlkTables{};
    p->last_engine = blk ? 3 : 0;
    p->last_handover = -1;
    for (int t = 0; t < t_max - 1; ++t) {
        if constexpr (sizeof(T) == 4) {
            if (blk) {
                // (both block engines run iteration t's Ab inside iteration t - 1's Az)
                SG_TRY(amp_launch_control<T>(tb, bf, sc, pr, 0, t, s));
                SG_TRY(p->block2 ? blk2_launch_az(bt, bf, (cx<float> *)p->ws_gbuf, t + 1 < t_max - 1, s)
                                 : blk_launch_az(bt, bf, t + 1 < t_max - 1, s));
                SG_TRY(amp_launch_control<T>(tb, bf, sc, pr, 1, t, s));
            }
        }
        if (!blk) {
            if (t > 0) SG_TRY(amp_launch_ab<T>(tb, bf, s));
            SG_TRY(amp_launch_control<T>(tb, bf, sc, pr, 0, t, s));
            SG_TRY(amp_launch_az<T>(tb, bf, s));
            SG_TRY(amp_launch_eta<T>(tb, bf, s));
            SG_TRY(amp_launch_control<T>(tb, bf, sc, pr, 1, t, s));
        }
        // skip the remaining launches once every codeword stopped (ActivePoll: the flags after
        // iterations 3, 7, 11, ..., read one iteration later)
        int na = -1;
        SG_TRY(poll.collect(&na));
        if (na == 0) break;
        if (t % 4 == 3 && t + 2 < t_max - 1) SG_TRY(poll.request());
    }
    if (poll.pending) SG_HIP(hipEventSynchronize(p->poll_ev));
    if (d_map) SG_HIP(hipMemcpyAsync(d_map, p->ws_argmax, sizeof(int32_t) * B * p->L, hipMemcpyDeviceToDevice, s));
    if (d_tfinal) SG_HIP(hipMemcpyAsync(d_tfinal, p->ws_tfinal, sizeof(int32_t) * B, hipMemcpyDeviceToDevice, s));
    if (d_nmse) SG_HIP(hipMemcpyAsync(d_nmse, p->ws_nmse, sizeof(double) * B * t_max * p->Lc, hipMemcpyDeviceToDevice, s));
    if (d_psi) SG_HIP(hipMemcpyAsync(d_psi, p->ws_psi, sizeof(double) * B * p->Lc, hipMemcpyDeviceToDevice, s));
    SG_HIP(hipGetLastError());
    return SG_OK;
}

template <typename T>
static int apply_impl(sg_amp_plan *p, int transpose, const void *d_in, int in_is_double, int B, void *d_out,
                      int out_double, hipStream_t s) {
    SG_TRY(ensure_ws(p, B, 2));
    if (p->regular) {
        RegTables<T> rt = rtables<T>(p);
        RegBufs<T> rf = rbufs<T>(p, B, nullptr);
        rf.mode = 1;
        if (!transpose) {
            SG_TRY(amp_launch_cast<T>(d_in, in_is_double, (T *)p->ws_s, (size_t)B * p->LM, s));
            rf.ext_in = (const T *)p->ws_s;
            rf.ext_out = out_double ? (T *)p->ws_z : (T *)d_out;
            SG_TRY(reg_launch_ab<T>(rt, rf, s));
            SG_TRY(reg_launch_ab_finish<T>(rt, rf, s));
            if (out_double) SG_TRY(amp_launch_uncast<T>((T *)p->ws_z, (double *)d_out, (size_t)B * p->n, s));
        } else {
            SG_TRY(amp_launch_cast<T>(d_in, in_is_double, (T *)p->ws_y, (size_t)B * p->n, s));
            rf.ext_in = (const T *)p->ws_y;
            rf.ext_out = out_double ? (T *)p->ws_s : (T *)d_out;
            SG_TRY(reg_launch_az<T>(rt, rf, 0, s));
            if (out_double) SG_TRY(amp_launch_uncast<T>((T *)p->ws_s, (double *)d_out, (size_t)B * p->LM, s));
        }
        SG_HIP(hipStreamSynchronize(s));
        return SG_OK;
    }
    AmpTables<T> tb = tables<T>(p);
    AmpBufs<T> bf = bufs<T>(p, B, nullptr);
    // all codewords active
    std::vector<int32_t> ones(B, 1);
    SG_HIP(hipMemcpyAsync(p->ws_active, ones.data(), sizeof(int32_t) * B, hipMemcpyHostToDevice, s));
    if (!transpose) {
        SG_TRY(amp_launch_cast<T>(d_in, in_is_double, (T *)p->ws_beta, (size_t)B * p->LM, s));
        SG_TRY(amp_launch_ab<T>(tb, bf, s));
        T *out = out_double ? (T *)p->ws_z : (T *)d_out;
        SG_TRY(amp_launch_rowsum<T>(tb, bf, out, s));
        if (out_double) SG_TRY(amp_launch_uncast<T>(out, (double *)d_out, (size_t)B * p->n, s));
    } else {
        SG_TRY(amp_launch_cast<T>(d_in, in_is_double, (T *)p->ws_z, (size_t)B * p->n, s));
        std::vector<double> ph((size_t)B * p->Lr, 1.0);
        SG_HIP(hipMemcpyAsync(p->ws_phi, ph.data(), sizeof(double) * ph.size(), hipMemcpyHostToDevice, s));
        SG_TRY(amp_launch_az<T>(tb, bf, s));
        T *out = out_double ? (T *)p->ws_beta : (T *)d_out;
        SG_TRY(amp_launch_colgather<T>(tb, bf, out, s));
        if (out_double) SG_TRY(amp_launch_uncast<T>(out, (double *)d_out, (size_t)B * p->LM, s));
    }
    SG_HIP(hipStreamSynchronize(s));
    return SG_OK;
}

static int ensure_io(sg_amp_plan *p, size_t bytes) {
    if (bytes <= p->ws_io_bytes) return SG_OK;
    if (p->ws_io) hipFree(p->ws_io);
    p->ws_io = nullptr;
    p->ws_io_bytes = 0;
    SG_HIP(hipMalloc(&p->ws_io, bytes));
    p->ws_io_bytes = bytes;
    return SG_OK;
}

}  // namespace sg

using namespace sg;

// One-hot message vectors (value 1, the public SPARC's beta0 before the
// sqrt(W / L) scaling that the design applies, sparc.py:17-53) -> x = A beta0.
template <typename T>
__global__ void onehot_one_kernel(const int32_t *idx, int L, int M, T *beta) {
    const int b = blockIdx.y;
    for (int l = blockIdx.x * blockDim.x + threadIdx.x; l < L; l += gridDim.x * blockDim.x)
        beta[(size_t)b * L * M + (size_t)l * M + idx[(size_t)b * L + l]] = T(1);
}

template <typename T>
static int encode_impl(sg_amp_plan *p, const int32_t *d_idx, int B, T *d_x, hipStream_t s) {
    SG_TRY(ensure_ws(p, B, 2));
    T *beta0 = p->regular ? (T *)p->ws_s : (T *)p->ws_beta;
    SG_HIP(hipMemsetAsync(beta0, 0, (size_t)B * p->LM * sizeof(T), s));
    hipLaunchKernelGGL(onehot_one_kernel<T>, dim3((p->L + 255) / 256, B), dim3(256), 0, s, d_idx, p->L, p->M, beta0);
    if (p->regular) {
        RegTables<T> rt = rtables<T>(p);
        RegBufs<T> rf = rbufs<T>(p, B, nullptr);
        rf.mode = 1;
        rf.ext_in = beta0;
        rf.ext_out = d_x;
        SG_TRY(reg_launch_ab<T>(rt, rf, s));
        SG_TRY(reg_launch_ab_finish<T>(rt, rf, s));
        return SG_OK;
    }
    AmpTables<T> tb = tables<T>(p);
    AmpBufs<T> bf = bufs<T>(p, B, nullptr);
    std::vector<int32_t> ones(B, 1);
    SG_HIP(hipMemcpyAsync(p->ws_active, ones.data(), sizeof(int32_t) * B, hipMemcpyHostToDevice, s));
    SG_TRY(amp_launch_ab<T>(tb, bf, s));
    SG_TRY(amp_launch_rowsum<T>(tb, bf, d_x, s));
    SG_HIP(hipStreamSynchronize(s));  // the host vector above
    return SG_OK;
}

extern "C" {

int sg_amp_plan_create(int ndim, const double *W, int Lr, int Lc, int L, int M, int n, const uint32_t *order0,
                       const uint32_t *order1, int precision, sg_amp_plan **out) {
    sg_amp_plan *p = nullptr;
    SG_TRY(build_plan(ndim, W, Lr, Lc, L, M, n, order0, order1, precision, false, &p));
    if (p->cw && precision == SG_F32) {
        const int rc = build_plan(ndim, W, Lr, Lc, L, M, n, order0, order1, precision, true, &p->alt);
        if (rc != SG_OK) {
            sg_amp_plan_destroy(p);
            return rc;
        }
    }
    *out = p;
    return SG_OK;
}

int sg_amp_plan_destroy(sg_amp_plan *p) {
    if (!p) return SG_OK;
    sg_amp_plan_destroy(p->alt);
    plan_free_ws(p);
    for (void *a : p->allocs) hipFree(a);
    if (p->tprof) hipFree(p->tprof);
    if (p->poll_ev) {
        hipEventSynchronize(p->poll_ev);  // (a copy into h_active may still be in flight)
        hipEventDestroy(p->poll_ev);
    }
    if (p->h_active) hipHostFree(p->h_active);
    delete p;
    return SG_OK;
}

int sg_amp_plan_engine(const sg_amp_plan *p, int B) {
    SG_CHECK_ARG(p, "plan is NULL");
    if (p->regular) return (sg::use_cw(p, B) && (p->precision == SG_F32 || sg::use_cw2(p))) ? 2 : 1;
    return (p->block || p->block2) ? 3 : 0;
}

int sg_amp_last_decode(const sg_amp_plan *p, int *engine, int *handover_iter, int *on_companion) {
    SG_CHECK_ARG(p && engine && handover_iter, "null argument");
    const sg_amp_plan *r = p->last_ran ? p->last_ran : p;
    *engine = r->last_engine;
    *handover_iter = r->last_handover;
    if (on_companion) *on_companion = (p->last_ran && p->last_ran != p) ? 1 : 0;
    return SG_OK;
}

int sg_amp_plan_info(const sg_amp_plan *p, int *w, int *nT, int *Mr, int *Mc, int *P, int *Q) {
    SG_CHECK_ARG(p, "plan is NULL");
    if (w) *w = p->w;
    if (nT) *nT = p->nT;
    if (Mr) *Mr = p->Mr;
    if (Mc) *Mc = p->Mc;
    if (P) *P = p->regular ? p->rP : p->P;
    if (Q) *Q = p->regular ? p->rQ : p->Q;
    return SG_OK;
}

// sg_amp_last_decode reports what the latest decode call ran: reset at the
// entry of every decode, so a call that returns early (B == 0) or fails
// partway reports engine -1 instead of a previous call's engine and hand-over
static void reset_last(sg_amp_plan *p) {
    for (sg_amp_plan *q : {p, p->alt}) {
        if (!q) continue;
        q->last_ran = nullptr;
        q->last_engine = -1;
        q->last_handover = -1;
    }
}

int sg_amp_decode_device(sg_amp_plan *p, const void *d_y, int B, const int32_t *d_true_idx, double awgn_var,
                         int t_max, double rtol, int phi_method, int32_t *d_map_idx, int32_t *d_t_final,
                         double *d_nmse, double *d_psi, void *stream) {
    SG_CHECK_ARG(p, "plan is NULL");
    reset_last(p);
    SG_CHECK_ARG(t_max > 1, "t_max must be > 1 (sparc.py:168)");
    SG_CHECK_ARG(rtol > 0 && rtol < 1, "rtol must be in (0, 1)");
    SG_CHECK_ARG(phi_method == 1 || phi_method == 2, "phi_est_method must be 1 or 2");
    SG_CHECK_ARG(awgn_var >= 0, "awgn_var must be >= 0");
    SG_CHECK_ARG(B >= 0, "negative batch");
    if (B == 0) return SG_OK;
    SG_CHECK_ARG(d_y, "d_y is NULL");
    p = p->last_ran = sg::decode_plan(p, B);
    SG_TRY(ensure_device());
    SG_HIP(hipSetDevice(p->device));
    hipStream_t s = pick_stream(stream);
    if (p->precision == SG_F64)
        return decode_impl<double>(p, d_y, B, d_true_idx, awgn_var, t_max, rtol, phi_method, d_map_idx, d_t_final,
                                   d_nmse, d_psi, s);
    return decode_impl<float>(p, d_y, B, d_true_idx, awgn_var, t_max, rtol, phi_method, d_map_idx, d_t_final, d_nmse,
                              d_psi, s);
}

int sg_amp_decode(sg_amp_plan *p, const double *y, int B, const int32_t *true_idx, double awgn_var, int t_max,
                  double rtol, int phi_method, int32_t *map_idx, int32_t *t_final, double *nmse, double *psi) {
    SG_CHECK_ARG(p, "plan is NULL");
    reset_last(p);
    SG_CHECK_ARG(B >= 0, "negative batch");
    if (B == 0) return SG_OK;
    SG_CHECK_ARG(y && map_idx && t_final && nmse && psi, "null host buffer");
    SG_CHECK_ARG(t_max > 1, "t_max must be > 1 (sparc.py:168)");
    p = p->last_ran = sg::decode_plan(p, B);
    SG_TRY(ensure_device());
    SG_HIP(hipSetDevice(p->device));
    hipStream_t s = lib_stream();
    SG_TRY(ensure_ws(p, B, t_max));
    const size_t ny = (size_t)B * p->n;
    SG_TRY(ensure_io(p, ny * sizeof(double)));
    SG_HIP(hipMemcpyAsync(p->ws_io, y, ny * sizeof(double), hipMemcpyHostToDevice, s));
    int r;
    if (p->precision == SG_F64) {
        r = amp_launch_cast<double>(p->ws_io, 1, (double *)p->ws_y, ny, s);
    } else {
        r = amp_launch_cast<float>(p->ws_io, 1, (float *)p->ws_y, ny, s);
    }
    SG_TRY(r);
    const int32_t *d_true = nullptr;
    if (true_idx) {
        SG_HIP(hipMemcpyAsync(p->ws_true, true_idx, sizeof(int32_t) * B * p->L, hipMemcpyHostToDevice, s));
        d_true = p->ws_true;
    }
    if (p->precision == SG_F64)
        r = decode_impl<double>(p, p->ws_y, B, d_true, awgn_var, t_max, rtol, phi_method, nullptr, nullptr, nullptr,
                                nullptr, s);
    else
        r = decode_impl<float>(p, p->ws_y, B, d_true, awgn_var, t_max, rtol, phi_method, nullptr, nullptr, nullptr,
                               nullptr, s);
    SG_TRY(r);
    SG_HIP(hipMemcpyAsync(map_idx, p->ws_argmax, sizeof(int32_t) * B * p->L, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(t_final, p->ws_tfinal, sizeof(int32_t) * B, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(nmse, p->ws_nmse, sizeof(double) * B * t_max * p->Lc, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(psi, p->ws_psi, sizeof(double) * B * p->Lc, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    return SG_OK;
}

int sg_amp_apply(sg_amp_plan *p, int transpose, const double *in, int B, double *out) {
    SG_CHECK_ARG(p && in && out, "null argument");
    SG_CHECK_ARG(B >= 0, "negative batch");
    if (B == 0) return SG_OK;
    SG_TRY(ensure_device());
    SG_HIP(hipSetDevice(p->device));
    hipStream_t s = lib_stream();
    const size_t nin = (size_t)B * (transpose ? p->n : p->LM), nout = (size_t)B * (transpose ? p->LM : p->n);
    SG_TRY(ensure_ws(p, B, 2));
    SG_TRY(ensure_io(p, (nin + nout) * sizeof(double)));
    double *din = (double *)p->ws_io, *dout = din + nin;
    SG_HIP(hipMemcpyAsync(din, in, nin * sizeof(double), hipMemcpyHostToDevice, s));
    int r = (p->precision == SG_F64) ? apply_impl<double>(p, transpose, din, 1, B, dout, 1, s)
                                     : apply_impl<float>(p, transpose, din, 1, B, dout, 1, s);
    SG_TRY(r);
    SG_HIP(hipMemcpyAsync(out, dout, nout * sizeof(double), hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    return SG_OK;
}

int sg_amp_encode_device(sg_amp_plan *p, const int32_t *d_idx, int B, void *d_x, void *stream) {
    SG_CHECK_ARG(p && d_idx && d_x, "null argument");
    if (B <= 0) return SG_OK;
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    return p->precision == SG_F64 ? encode_impl<double>(p, d_idx, B, (double *)d_x, s)
                                  : encode_impl<float>(p, d_idx, B, (float *)d_x, s);
}

// Diagnostics: mean shader-clock cycles between the phase timestamps of the
// last stage-1 launches (kernel 0 = reg_ab_stage1, 1 = reg_az_stage2), over
// every workgroup that recorded them; needs SG_AMP_TPROF set at plan use.
int sg_amp_stage_profile(sg_amp_plan *p, int kernel, double *mean_cycles, int *nphases) {
    SG_CHECK_ARG(p && mean_cycles && nphases && (kernel == 0 || kernel == 1), "bad argument");
    *nphases = 0;
    if (p->last_ran) p = p->last_ran;  // the sub-plan the last decode ran on (maybe the companion)
    if (!p->tprof) return SG_OK;
    std::vector<uint64_t> h(p->tprof_items * 8);
    SG_HIP(hipDeviceSynchronize());
    SG_HIP(hipMemcpy(h.data(), p->tprof + (size_t)kernel * p->tprof_items * 8, h.size() * 8, hipMemcpyDeviceToHost));
    double sum[8] = {0};
    size_t n = 0;
    for (size_t i = 0; i < p->tprof_items; ++i) {
        const uint64_t *r = &h[i * 8];
        if (!r[0] || !r[7]) continue;
        ++n;
        for (int k = 1; k < 8; ++k) sum[k] += (double)(r[k] - r[k - 1]);
    }
    for (int k = 0; k < 8; ++k) mean_cycles[k] = n ? sum[k] / n : 0.0;
    *nphases = 8;
    return SG_OK;
}

int sg_amp_stage_raw(sg_amp_plan *p, int kernel, uint64_t *out, size_t *items) {
    SG_CHECK_ARG(p && items && (kernel == 0 || kernel == 1), "bad argument");
    if (p->last_ran) p = p->last_ran;
    *items = p->tprof ? p->tprof_items : 0;
    if (!p->tprof || !out) return SG_OK;
    const size_t ni = p->tprof_items;
    std::vector<uint64_t> cyc(ni * 8), rt(ni * 2);
    SG_HIP(hipDeviceSynchronize());
    SG_HIP(hipMemcpy(cyc.data(), p->tprof + (size_t)kernel * ni * 8, ni * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    SG_HIP(hipMemcpy(rt.data(), p->tprof + ni * 16 + (size_t)kernel * ni * 2, ni * 2 * sizeof(uint64_t),
                     hipMemcpyDeviceToHost));
    for (size_t i = 0; i < ni; ++i) {
        std::copy(&cyc[i * 8], &cyc[i * 8] + 8, out + i * 10);
        out[i * 10 + 8] = rt[i * 2];
        out[i * 10 + 9] = rt[i * 2 + 1];
    }
    return SG_OK;
}

int sg_amp_apply_device(sg_amp_plan *p, int transpose, const void *d_in, int B, void *d_out, void *stream) {
    SG_CHECK_ARG(p && d_in && d_out, "null argument");
    if (B <= 0) return SG_OK;
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    if (p->precision == SG_F64) return apply_impl<double>(p, transpose, d_in, 1, B, d_out, 0, s);
    return apply_impl<float>(p, transpose, d_in, 0, B, d_out, 0, s);
}

int sg_amp_count_errors_device(const int32_t *d_map_idx, const int32_t *d_true_idx, const int32_t *d_t_final, int B,
                               int L, int logM, int64_t *d_counts, void *stream) {
    SG_CHECK_ARG(d_map_idx && d_true_idx && d_t_final && d_counts, "null device buffer");
    SG_TRY(ensure_device());
    return amp_launch_count(d_map_idx, d_true_idx, d_t_final, B, L, logM, d_counts, pick_stream(stream));
}

}  // extern "C"
