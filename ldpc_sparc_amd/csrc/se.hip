// State evolution of SPARC AMP (sparc_public/sparc_se.py:82-183) on gfx950:
// the Monte-Carlo expectation sparc_se_E (:82-115) over resident Gaussian
// samples u [mc][M], for many tau values at once (one per column block of
// the base matrix).  The tau / psi recursion itself is scalar host work.
//
//   K = 1:  E = mean_s  e^(1/tau + u_s0/sqrt(tau)) / (e^(1/tau + u_s0/sqrt(tau)) + sum_{j>0} e^(u_sj/sqrt(tau)))
//   K = 2:  sinh / cosh in place of exp (real modulated SPARCs, :91-94)
//
// One wavefront per sample (lanes stride the M entries); per-block partial
// sums, then a fixed-order sum, so E is deterministic.
#include <algorithm>

#include "common.hpp"

struct sg_se_samples {
    int mc = 0, M = 0;
    double *u = nullptr;     // [mc][M]
    double *part = nullptr;  // [nt_cap][nblk]
    int nt_cap = 0;
    double *taus = nullptr, *E = nullptr;
};

namespace sg {

namespace {

constexpr int SE_WAVES = 4;  // samples per 256-thread block

__global__ __launch_bounds__(256) void se_E_kernel(const double *__restrict__ u, int mc, int M, int K,
                                                   const double *taus, double *part, int nblk) {
    __shared__ double red[SE_WAVES];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int s = blockIdx.x * SE_WAVES + wid, t = blockIdx.y;
    const double itau = 1.0 / taus[t], rtau = sqrt(itau);
    double e = 0.0;
    if (s < mc) {
        const double *row = u + (size_t)s * M;
        double c = 0.0;
        for (int j = 1 + lane; j < M; j += 64) c += K == 1 ? exp(rtau * row[j]) : cosh(rtau * row[j]);
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        const double a = K == 1 ? exp(itau + rtau * row[0]) : sinh(itau + rtau * row[0]);
        e = a / (a + c);  // expsB = expsA for K = 1, 2 (:88-94)
    }
    if (lane == 0) red[wid] = e;
    __syncthreads();
    if (threadIdx.x == 0) {
        double v = 0.0;
        for (int w = 0; w < SE_WAVES; ++w) v += red[w];
        part[(size_t)t * nblk + blockIdx.x] = v;
    }
}

__global__ void se_finish_kernel(const double *part, int nblk, int mc, double *E) {
    __shared__ double red[4];
    const int t = blockIdx.x;
    double v = 0.0;
    for (int b = threadIdx.x; b < nblk; b += blockDim.x) v += part[(size_t)t * nblk + b];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) E[t] = (red[0] + red[1] + red[2] + red[3]) / mc;
}

}  // namespace

}  // namespace sg

using namespace sg;

extern "C" {

int sg_se_samples_create(const double *u, int mc, int M, sg_se_samples **out) {
    SG_CHECK_ARG(u && out && mc > 0 && M > 1, "bad argument");
    SG_TRY(ensure_device());
    sg_se_samples *h = new sg_se_samples();
    h->mc = mc;
    h->M = M;
    const size_t bytes = (size_t)mc * M * 8;
    if (hipMalloc(&h->u, bytes) != hipSuccess) {
        delete h;
        return fail(SG_ERR_NOMEM, "cannot allocate %zu bytes of samples", bytes);
    }
    if (hipMemcpy(h->u, u, bytes, hipMemcpyHostToDevice) != hipSuccess) {
        hipFree(h->u);
        delete h;
        return fail(SG_ERR_HIP, "sample upload failed");
    }
    *out = h;
    return SG_OK;
}

int sg_se_samples_destroy(sg_se_samples *h) {
    if (!h) return SG_OK;
    for (void *p : {(void *)h->u, (void *)h->part, (void *)h->taus, (void *)h->E})
        if (p) hipFree(p);
    delete h;
    return SG_OK;
}

int sg_se_expectation(sg_se_samples *h, int K, const double *taus, int nt, double *E) {
    SG_CHECK_ARG(h && taus && E && nt >= 0, "bad argument");
    SG_CHECK_ARG(K == 1 || K == 2, "state evolution supports K = 1 and K = 2 (real SPARCs)");
    if (!nt) return SG_OK;
    SG_TRY(ensure_device());
    const int nblk = (h->mc + SE_WAVES - 1) / SE_WAVES;
    if (nt > h->nt_cap) {
        for (void *p : {(void *)h->part, (void *)h->taus, (void *)h->E})
            if (p) hipFree(p);
        h->part = h->taus = h->E = nullptr;
        h->nt_cap = 0;
        SG_HIP(hipMalloc(&h->part, (size_t)nt * nblk * 8));
        SG_HIP(hipMalloc(&h->taus, (size_t)nt * 8));
        SG_HIP(hipMalloc(&h->E, (size_t)nt * 8));
        h->nt_cap = nt;
    }
    hipStream_t s = lib_stream();
    SG_HIP(hipMemcpyAsync(h->taus, taus, (size_t)nt * 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(se_E_kernel, dim3(nblk, nt), dim3(256), 0, s, h->u, h->mc, h->M, K, h->taus, h->part, nblk);
    hipLaunchKernelGGL(se_finish_kernel, dim3(nt), dim3(256), 0, s, h->part, nblk, h->mc, h->E);
    SG_HIP(hipGetLastError());
    SG_HIP(hipMemcpyAsync(E, h->E, (size_t)nt * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    return SG_OK;
}

}  // extern "C"
