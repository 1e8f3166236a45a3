// Declarations shared by the AMP decoder kernels (amp_dct.hip) and the host
// plan / C ABI (capi_amp.cpp).
#pragma once
#include "common.hpp"
#include "fft.hpp"

namespace sg {

constexpr int AMP_MAX_EPT = 32;

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
};

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
int amp_launch_count(const int32_t *map_idx, const int32_t *true_idx, const int32_t *t_final, int B, int L,
                     int logM, int64_t *counts, hipStream_t s);

}  // namespace sg
