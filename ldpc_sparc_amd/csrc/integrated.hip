// AMP <-> BP integrated decoders on gfx950: the soft glue between the dense
// AMP state and the LDPC decoder (sparc_sophie/sparc_new.py).
//
//   bp_to_beta       bp_output_to_beta_estimate :1260-1279 -- per (section,
//                    index) product over the section's bit probabilities
//   update_post      update_using_bp_probs :1030-1038 -- per-section
//                    renormalised alpha * gamma
//   deta             differentiated_eta_calc :824-841 (+ sub_term :871-883)
//                    and differentiated_eta_calc_posteriors :843-869, in
//                    closed form (DESIGN.md "integrated decoders"): the
//                    reference's O(L M^2 log M) loops become, per section,
//                    log M sums A_k over the indices whose bit k is 0 and one
//                    log M term per index
//   llr / probs      ldpc_bp's clip + log-ratio and exp(app) / (1 + exp(app))
//                    :1162-1193
//   hard_bits        app[:K] < 0 of every block :1185-1187
// Every section is one 256-thread workgroup (M <= 4096); sums go through a
// fixed-order block reduction, so results are deterministic.
#include <algorithm>

#include "dense.hpp"

namespace sg {

namespace {

constexpr int IB = 256;  // block size of the section kernels

__device__ __forceinline__ double block_sum(double v, double *red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double t = 0.0;
    for (int w = 0; w < IB / 64; ++w) t += red[w];
    return t;
}

__device__ __forceinline__ int log2i(int M) {
    int k = 0;
    while ((1 << k) < M) ++k;
    return k;
}

template <typename T>
__device__ __forceinline__ T iexp(T x);
template <>
__device__ __forceinline__ float iexp<float>(float x) { return __expf(x); }
template <>
__device__ __forceinline__ double iexp<double>(double x) { return exp(x); }

template <typename T>
__device__ __forceinline__ T ilog(T x);
template <>
__device__ __forceinline__ float ilog<float>(float x) { return __logf(x); }
template <>
__device__ __forceinline__ double ilog<double>(double x) { return log(x); }

}  // namespace

// probabilities of bit 0 -> LLRs: clip to [1e-15, 1 - 1e-15], log p - log(1 - p)
template <typename T>
__global__ __launch_bounds__(256) void llr_from_probs_kernel(const T *p, size_t nn, T *llr) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nn; i += (size_t)gridDim.x * blockDim.x) {
        const T eps = T(1e-15);
        const T v = fmin(fmax(p[i], eps), T(1) - eps);
        llr[i] = ilog<T>(v) - ilog<T>(T(1) - v);
    }
}

// app LLRs -> P(bit = 0) = exp(app) / (1 + exp(app))
template <typename T>
__global__ __launch_bounds__(256) void probs_from_app_kernel(const T *app, size_t nn, T *p) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nn; i += (size_t)gridDim.x * blockDim.x) {
        const T e = iexp<T>(app[i]);
        p[i] = e / (T(1) + e);
    }
}

// beta[l][i] = (prod_j (p_lj if bit j of i (MSB first) is 0 else 1 - p_lj)) * snp,
// the product taken left to right like the reference; gamma = that / snp.
template <typename T>
__global__ __launch_bounds__(256) void bp_to_beta_kernel(const T *probs, int L, int M, double snp, int as_gamma,
                                                         T *out) {
    const int l = blockIdx.x, b = blockIdx.y;
    const int logM = log2i(M);
    __shared__ T p[32];
    if (threadIdx.x < logM) p[threadIdx.x] = probs[((size_t)b * L + l) * logM + threadIdx.x];
    __syncthreads();
    T *o = out + ((size_t)b * L + l) * M;
    for (int i = threadIdx.x; i < M; i += blockDim.x) {
        T a = T(1);
        for (int j = 0; j < logM; ++j) {
            const int bit = (i >> (logM - 1 - j)) & 1;
            a = a * (bit == 0 ? p[j] : T(1) - p[j]);
        }
        const T v = a * (T)snp;
        o[i] = as_gamma ? v / (T)snp : v;
    }
}

// beta = snp * (alpha gamma) / sum_section(alpha gamma), alpha = alpha_w / ascale
// (the decoders pass the weighted estimate and ascale = snp)
template <typename T>
__global__ __launch_bounds__(IB) void update_post_kernel(const T *gamma, const T *alpha_w, double ascale, int L,
                                                         int M, double snp, T *beta) {
    __shared__ double red[IB / 64];
    const int l = blockIdx.x, b = blockIdx.y;
    const size_t o = ((size_t)b * L + l) * M;
    double bot = 0.0;
    for (int i = threadIdx.x; i < M; i += IB) bot += (double)((alpha_w[o + i] / (T)ascale) * gamma[o + i]);
    const T bt = (T)block_sum(bot, red);
    for (int i = threadIdx.x; i < M; i += IB) {
        const T top = (alpha_w[o + i] / (T)ascale) * gamma[o + i];
        beta[o + i] = (T)snp * (top / bt);
    }
}

// Differentiated eta of one section (integrated decoders).  post = 0:
// beta * main_term (sparc_new.py:824-841); post = 1: eta_dash of :843-869.
// alpha = alpha_w / ascale; c = snp / tau^2.  Writes the section's sum of the
// vector to part[b][l] and, when out != null, the vector itself.
template <typename T>
__global__ __launch_bounds__(IB) void deta_kernel(int post, const T *beta, const T *gamma, const T *alpha_w,
                                                  double ascale, const T *vk, const T *vk0, const double *tau2,
                                                  int L, int M, double snp, double *part, T *out) {
    __shared__ double red[IB / 64];
    __shared__ double sA[32], sW[32], sV[32];
    const int l = blockIdx.x, b = blockIdx.y;
    const int logM = log2i(M);
    const size_t o = ((size_t)b * L + l) * M;
    const double c = snp / tau2[b];
    // A_k = sum over the indices with bit k = 0 of alpha
    for (int k = 0; k < logM; ++k) {
        double a = 0.0;
        for (int i = threadIdx.x; i < M; i += IB)
            if (((i >> (logM - 1 - k)) & 1) == 0) a += (double)(alpha_w[o + i] / (T)ascale);
        a = block_sum(a, red);
        if (threadIdx.x == 0) {
            const double v = fmin(fmax((double)vk0[((size_t)b * L + l) * logM + k], 1e-10), 1.0 - 1e-10);
            sA[k] = a;
            sW[k] = 1.0 / (v * (1.0 - v));
            sV[k] = (double)vk[((size_t)b * L + l) * logM + k];
        }
    }
    __syncthreads();
    double bot = 0.0, botd = 0.0;
    if (post) {  // section sums of top = alpha gamma and top' = alpha' gamma + alpha gamma'
        for (int i = threadIdx.x; i < M; i += IB) {
            const double al = (double)(alpha_w[o + i] / (T)ascale), g = (double)gamma[o + i];
            double mt = 0.0;
            for (int k = 0; k < logM; ++k) {
                const bool zero = ((i >> (logM - 1 - k)) & 1) == 0;
                const double sub = sW[k] * (c * al * ((zero ? 1.0 : 0.0) - sA[k]));
                mt += zero ? (1.0 - sV[k]) * sub : -sV[k] * sub;
            }
            const double ad = al * (snp / tau2[b]) * (1.0 - al);
            bot += al * g;
            botd += ad * g + al * (g * mt);
        }
        bot = block_sum(bot, red);
        botd = block_sum(botd, red);
    }
    double sum = 0.0;
    for (int i = threadIdx.x; i < M; i += IB) {
        const double al = (double)(alpha_w[o + i] / (T)ascale);
        double mt = 0.0;
        for (int k = 0; k < logM; ++k) {
            const bool zero = ((i >> (logM - 1 - k)) & 1) == 0;
            const double sub = sW[k] * (c * al * ((zero ? 1.0 : 0.0) - sA[k]));
            mt += zero ? (1.0 - sV[k]) * sub : -sV[k] * sub;
        }
        double de;
        if (!post) {
            de = (double)beta[o + i] * mt;
        } else {
            const double g = (double)gamma[o + i];
            const double ad = al * (snp / tau2[b]) * (1.0 - al);
            const double top = al * g, topd = ad * g + al * (g * mt);
            de = (snp * ((topd * bot) - (top * botd))) / (bot * bot);
        }
        if (out) out[o + i] = (T)de;
        sum += de;
    }
    sum = block_sum(sum, red);
    if (threadIdx.x == 0) part[(size_t)b * L + l] = sum;
}

// ons[b] = sum over the sections of part[b][.], fixed order
__global__ void deta_finish_kernel(const double *part, int L, double *ons) {
    __shared__ double red[IB / 64];
    const int b = blockIdx.x;
    double v = 0.0;
    for (int l = threadIdx.x; l < L; l += IB) v += part[(size_t)b * L + l];
    v = block_sum(v, red);
    if (threadIdx.x == 0) ons[b] = v;
}

// information bits of every block: app[:K] < 0 (sparc_new.py:1185-1187)
template <typename T>
__global__ __launch_bounds__(256) void hard_bits_kernel(const T *app, int nblocks, int N, int K, uint8_t *bits) {
    const int blk = blockIdx.y;
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < K; j += gridDim.x * blockDim.x)
        bits[(size_t)blk * K + j] = app[(size_t)blk * N + j] < T(0) ? 1 : 0;
}

static unsigned gridn(size_t nn) { return (unsigned)std::min<size_t>(65535, (nn + 255) / 256); }
static int log2_exact(int M) {  // -1 unless M is a power of two
    if (M <= 0 || (M & (M - 1))) return -1;
    int k = 0;
    while ((1 << k) < M) ++k;
    return k;
}

template <typename T>
int integ_launch_llr(const T *p, size_t nn, T *llr, hipStream_t s) {
    hipLaunchKernelGGL((llr_from_probs_kernel<T>), dim3(gridn(nn)), dim3(256), 0, s, p, nn, llr);
    SG_HIP(hipGetLastError());
    return SG_OK;
}
template <typename T>
int integ_launch_probs(const T *app, size_t nn, T *p, hipStream_t s) {
    hipLaunchKernelGGL((probs_from_app_kernel<T>), dim3(gridn(nn)), dim3(256), 0, s, app, nn, p);
    SG_HIP(hipGetLastError());
    return SG_OK;
}
template <typename T>
int integ_launch_bp_to_beta(const T *probs, int B, int L, int M, double snp, int as_gamma, T *out, hipStream_t s) {
    SG_CHECK_ARG(log2_exact(M) >= 1 && log2_exact(M) <= 30, "bad section size %d", M);
    hipLaunchKernelGGL((bp_to_beta_kernel<T>), dim3(L, B), dim3(256), 0, s, probs, L, M, snp, as_gamma, out);
    SG_HIP(hipGetLastError());
    return SG_OK;
}
template <typename T>
int integ_launch_update(const T *gamma, const T *alpha_w, double ascale, int B, int L, int M, double snp, T *beta,
                        hipStream_t s) {
    hipLaunchKernelGGL((update_post_kernel<T>), dim3(L, B), dim3(IB), 0, s, gamma, alpha_w, ascale, L, M, snp, beta);
    SG_HIP(hipGetLastError());
    return SG_OK;
}
template <typename T>
int integ_launch_deta(int post, const T *beta, const T *gamma, const T *alpha_w, double ascale, const T *vk,
                      const T *vk0, const double *tau2, int B, int L, int M, double snp, double *part, double *ons,
                      T *out, hipStream_t s) {
    SG_CHECK_ARG(log2_exact(M) >= 1 && log2_exact(M) <= 30, "bad section size %d", M);
    hipLaunchKernelGGL((deta_kernel<T>), dim3(L, B), dim3(IB), 0, s, post, beta, gamma, alpha_w, ascale, vk, vk0,
                       tau2, L, M, snp, part, out);
    if (ons) hipLaunchKernelGGL(deta_finish_kernel, dim3(B), dim3(IB), 0, s, part, L, ons);
    SG_HIP(hipGetLastError());
    return SG_OK;
}
template <typename T>
int integ_launch_hard_bits(const T *app, int nblocks, int N, int K, uint8_t *bits, hipStream_t s) {
    hipLaunchKernelGGL((hard_bits_kernel<T>), dim3((K + 255) / 256, nblocks), dim3(256), 0, s, app, nblocks, N, K,
                       bits);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

#define SG_INTEG_INST(T)                                                                                        \
    template int integ_launch_llr<T>(const T *, size_t, T *, hipStream_t);                                      \
    template int integ_launch_probs<T>(const T *, size_t, T *, hipStream_t);                                   \
    template int integ_launch_bp_to_beta<T>(const T *, int, int, int, double, int, T *, hipStream_t);           \
    template int integ_launch_update<T>(const T *, const T *, double, int, int, int, double, T *, hipStream_t); \
    template int integ_launch_deta<T>(int, const T *, const T *, const T *, double, const T *, const T *,          \
                                      const double *, int, int, int, double, double *, double *, T *,           \
                                      hipStream_t);                                                             \
    template int integ_launch_hard_bits<T>(const T *, int, int, int, uint8_t *, hipStream_t);
SG_INTEG_INST(float)
SG_INTEG_INST(double)
#undef SG_INTEG_INST

}  // namespace sg
