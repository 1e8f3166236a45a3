// Dense Gaussian-design AMP (sparc_sophie/sparc_new.py:885-912) and the
// AMP -> BP glue (sparc_new.py:1118-1193): declarations shared by dense.hip
// and capi_dense.cpp.
#pragma once
#include "common.hpp"

namespace sg {

// Batched dense AMP state.  The design matrix A [n][LM] (row-major, as
// create_design_matrix draws it, sparc_new.py:1284-1294) is shared by the
// batch; z is padded to npad = roundup(n, 32) columns (zeros beyond n).
template <typename T>
struct DenseBufs {
    const T *A;        // [n][LM]
    int n, npad, L, M, LM, B;
    double P;          // total power; P_l = P / L, sqrt(n P_l) is the nonzero value
    const T *y;        // [B][n]
    T *z;              // [B][npad]
    T *beta;           // [B][LM]
    T *s;              // [B][LM]
    T *part;           // [nsplit][B][n] split-K partial sums of A beta
    int nsplit;
    double *tau2;      // [B]   ||z||^2 / n
    double *bsq;       // [B]   ||beta||^2
    double *sec_bsq;   // [B][L] per-section sum beta^2 (deterministic reduction)
    // Onsager term of the residual: 0 = (z / tau^2)(P - ||beta||^2 / n)
    // (sparc_new.py:903-905); 1 = (z / n) * ons[b] (integrated_decoder :490);
    // 2 = z * (ons[b] / n) (integrated_decoder_posteriors :693)
    int ons_mode;
    const double *ons;  // [B] sum of the differentiated eta
};

template <typename T>
int dense_launch_ab(const DenseBufs<T> &b, hipStream_t s);            // part = A beta (split K)
template <typename T>
int dense_launch_residual(const DenseBufs<T> &b, int t, hipStream_t s);  // z, tau^2 (sparc_new.py:902-908)
template <typename T>
int dense_launch_az(const DenseBufs<T> &b, hipStream_t s);            // s = beta + A^T z
template <typename T>
int dense_launch_bsq(const DenseBufs<T> &b, hipStream_t s);           // sec_bsq from a given beta
template <typename T>
int dense_launch_eta(const DenseBufs<T> &b, hipStream_t s);           // beta = eta(s), ||beta||^2
template <typename T>
int dense_launch_gen_A(T *A, int n, int LM, uint64_t seed, hipStream_t s);  // A ~ N(0, 1/n), Philox
template <typename T>
int dense_launch_map(const T *s, int B, int L, int M, int32_t *idx, hipStream_t st);
template <typename T>
int glue_launch_llr(const T *beta, int B, int L, int M, int l0, int nl, double inv_sqrt_nPl, int llr_ld, T *llr,
                    int probs_only, hipStream_t s);

// integrated decoders (integrated.hip)
template <typename T>
int integ_launch_llr(const T *p, size_t nn, T *llr, hipStream_t s);
template <typename T>
int integ_launch_probs(const T *app, size_t nn, T *p, hipStream_t s);
template <typename T>
int integ_launch_bp_to_beta(const T *probs, int B, int L, int M, double snp, int as_gamma, T *out, hipStream_t s);
template <typename T>
int integ_launch_update(const T *gamma, const T *alpha_w, double ascale, int B, int L, int M, double snp, T *beta,
                        hipStream_t s);
template <typename T>
int integ_launch_deta(int post, const T *beta, const T *gamma, const T *alpha_w, double ascale, const T *vk,
                      const T *vk0, const double *tau2, int B, int L, int M, double snp, double *part, double *ons,
                      T *out, hipStream_t s);
template <typename T>
int integ_launch_hard_bits(const T *app, int nblocks, int N, int K, uint8_t *bits, hipStream_t s);

template <typename T>
int concat_launch_count(const int32_t *map_idx, const int32_t *true_idx, int B, int L, int L_unp, int logM,
                        const T *app, const uint8_t *info, int mults, int N, int K, int64_t *counts, hipStream_t s);

}  // namespace sg
