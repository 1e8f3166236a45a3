// Stand-alone section estimators (the public msg_vector_mmse_estimator /
// msg_vector_map_estimator API of sparc.py:402-512 and sparc_new.py:1040-1116),
// double precision, one wavefront per section.  The fused decoder (eta_kernel
// in amp_dct.hip) does not use these.
#include "common.hpp"

namespace sg {

__global__ void section_softmax_kernel(const double *__restrict__ x, int L, int M, double scale,
                                       double *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int l = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (l >= L) return;
    const double *xs = x + (size_t)l * M;
    double m = -INFINITY;
    for (int e = lane; e < M; e += 64) m = fmax(m, xs[e]);
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    double den = 0.0;
    for (int e = lane; e < M; e += 64) den += exp(xs[e] - m);
    for (int o = 32; o > 0; o >>= 1) den += __shfl_xor(den, o, 64);
    for (int e = lane; e < M; e += 64) out[(size_t)l * M + e] = scale * (exp(xs[e] - m) / den);
}

__global__ void section_argmax_kernel(const double *__restrict__ s, int L, int M, int32_t *__restrict__ idx) {
    const int lane = threadIdx.x & 63;
    const int l = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (l >= L) return;
    const double *ss = s + (size_t)l * M;
    double best = -INFINITY;
    int arg = 0x7fffffff;
    for (int e = lane; e < M; e += 64)
        if (arg == 0x7fffffff || ss[e] > best) { best = ss[e]; arg = e; }
    double g = best;
    for (int o = 32; o > 0; o >>= 1) g = fmax(g, __shfl_xor(g, o, 64));
    int cand = (best == g) ? arg : 0x7fffffff;
    for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
    if (lane == 0) idx[l] = cand == 0x7fffffff ? 0 : cand;
}

}  // namespace sg

using namespace sg;

extern "C" {

// out[l*M + j] = scale * exp(x_j - max_l) / sum_l exp(x - max_l)
int sg_section_softmax(const double *x, int L, int M, double scale, double *out) {
    SG_CHECK_ARG(x && out && L >= 0 && M > 0, "bad arguments");
    if (L == 0) return SG_OK;
    SG_TRY(ensure_device());
    hipStream_t s = lib_stream();
    const size_t bytes = (size_t)L * M * sizeof(double);
    double *d = nullptr;
    SG_HIP(hipMalloc(&d, 2 * bytes));
    SG_HIP(hipMemcpyAsync(d, x, bytes, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(section_softmax_kernel, dim3((L + 3) / 4), dim3(256), 0, s, d, L, M, scale, d + (size_t)L * M);
    SG_HIP(hipGetLastError());
    SG_HIP(hipMemcpyAsync(out, d + (size_t)L * M, bytes, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    SG_HIP(hipFree(d));
    return SG_OK;
}

// idx[l] = first index of the maximum of section l (numpy argmax semantics)
int sg_section_argmax(const double *x, int L, int M, int32_t *idx) {
    SG_CHECK_ARG(x && idx && L >= 0 && M > 0, "bad arguments");
    if (L == 0) return SG_OK;
    SG_TRY(ensure_device());
    hipStream_t s = lib_stream();
    const size_t bytes = (size_t)L * M * sizeof(double);
    void *d = nullptr;
    SG_HIP(hipMalloc(&d, bytes + (size_t)L * 4));
    SG_HIP(hipMemcpyAsync(d, x, bytes, hipMemcpyHostToDevice, s));
    int32_t *di = (int32_t *)((char *)d + bytes);
    hipLaunchKernelGGL(section_argmax_kernel, dim3((L + 3) / 4), dim3(256), 0, s, (const double *)d, L, M, di);
    SG_HIP(hipGetLastError());
    SG_HIP(hipMemcpyAsync(idx, di, (size_t)L * 4, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    SG_HIP(hipFree(d));
    return SG_OK;
}

}  // extern "C"
