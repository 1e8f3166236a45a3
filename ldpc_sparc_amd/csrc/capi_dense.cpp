// C ABI of the dense Gaussian-design AMP decoder (sparc_new.py:885-912) and
// of the AMP -> BP glue (sparc_new.py:1118-1193).
#include <algorithm>
#include <cmath>
#include <initializer_list>
#include <utility>
#include <vector>

#include "dense.hpp"

struct sg_dense_plan {
    int precision = SG_F32;
    int device = 0;
    int n = 0, npad = 0, L = 0, M = 0, LM = 0, nsplit = 1;
    double P = 0;
    void *A = nullptr;
    int cap_B = 0;
    void *ws_y = nullptr, *ws_z = nullptr, *ws_beta = nullptr, *ws_s = nullptr, *ws_part = nullptr;
    double *ws_tau2 = nullptr, *ws_sec_bsq = nullptr;
    int32_t *ws_idx = nullptr;
    void *ws_io = nullptr;
    size_t ws_io_bytes = 0;
    // integrated decoders (integrated.hip): weighted alpha, gamma [B][LM];
    // bit probabilities vk0, vk, LLRs and app [B][L log M]; BP iteration counts;
    // per-section / per-codeword sums of the differentiated eta
    int cap_Bi = 0;
    void *wi_alpha = nullptr, *wi_gamma = nullptr, *wi_vk0 = nullptr, *wi_vk = nullptr, *wi_llr = nullptr,
         *wi_app = nullptr;
    int32_t *wi_it = nullptr;
    double *wi_part = nullptr, *wi_ons = nullptr;
};

namespace sg {

static size_t rsize(const sg_dense_plan *p) { return p->precision == SG_F64 ? 8 : 4; }

static void dense_free_ws(sg_dense_plan *p) {
    void *bufs[] = {p->ws_y, p->ws_z, p->ws_beta, p->ws_s, p->ws_part, p->ws_tau2, p->ws_sec_bsq, p->ws_idx, p->ws_io};
    for (void *b : bufs)
        if (b) hipFree(b);
    p->ws_y = p->ws_z = p->ws_beta = p->ws_s = p->ws_part = p->ws_io = nullptr;
    p->ws_tau2 = p->ws_sec_bsq = nullptr;
    p->ws_idx = nullptr;
    p->cap_B = 0;
    p->ws_io_bytes = 0;
}

static int dense_ensure_ws(sg_dense_plan *p, int B) {
    if (B <= p->cap_B) return SG_OK;
    dense_free_ws(p);
    const size_t rs = rsize(p), Bz = (size_t)B;
    const int nblk = (p->npad + 255) / 256;
    SG_HIP(hipMalloc(&p->ws_y, Bz * p->n * rs));
    SG_HIP(hipMalloc(&p->ws_z, Bz * p->npad * rs));
    SG_HIP(hipMalloc(&p->ws_beta, Bz * p->LM * rs));
    SG_HIP(hipMalloc(&p->ws_s, Bz * p->LM * rs));
    SG_HIP(hipMalloc(&p->ws_part, (size_t)p->nsplit * Bz * p->n * rs));
    SG_HIP(hipMalloc(&p->ws_tau2, Bz * (1 + nblk) * sizeof(double)));
    SG_HIP(hipMalloc(&p->ws_sec_bsq, Bz * p->L * sizeof(double)));
    SG_HIP(hipMalloc(&p->ws_idx, Bz * p->L * sizeof(int32_t)));
    p->cap_B = B;
    return SG_OK;
}

static void integ_free_ws(sg_dense_plan *p) {
    void *bufs[] = {p->wi_alpha, p->wi_gamma, p->wi_vk0, p->wi_vk, p->wi_llr, p->wi_app, p->wi_it, p->wi_part,
                    p->wi_ons};
    for (void *b : bufs)
        if (b) hipFree(b);
    p->wi_alpha = p->wi_gamma = p->wi_vk0 = p->wi_vk = p->wi_llr = p->wi_app = nullptr;
    p->wi_it = nullptr;
    p->wi_part = p->wi_ons = nullptr;
    p->cap_Bi = 0;
}

static int integ_ensure_ws(sg_dense_plan *p, int B, int nbits) {
    if (B <= p->cap_Bi) return SG_OK;
    integ_free_ws(p);
    const size_t rs = rsize(p), Bz = (size_t)B;
    SG_HIP(hipMalloc(&p->wi_alpha, Bz * p->LM * rs));
    SG_HIP(hipMalloc(&p->wi_gamma, Bz * p->LM * rs));
    SG_HIP(hipMalloc(&p->wi_vk0, Bz * nbits * rs));
    SG_HIP(hipMalloc(&p->wi_vk, Bz * nbits * rs));
    SG_HIP(hipMalloc(&p->wi_llr, Bz * nbits * rs));
    SG_HIP(hipMalloc(&p->wi_app, Bz * nbits * rs));
    SG_HIP(hipMalloc(&p->wi_it, Bz * nbits * sizeof(int32_t)));
    SG_HIP(hipMalloc(&p->wi_part, Bz * p->L * sizeof(double)));
    SG_HIP(hipMalloc(&p->wi_ons, Bz * sizeof(double)));
    p->cap_Bi = B;
    return SG_OK;
}

static int dense_ensure_io(sg_dense_plan *p, size_t bytes) {
    if (bytes <= p->ws_io_bytes) return SG_OK;
    if (p->ws_io) hipFree(p->ws_io);
    p->ws_io = nullptr;
    p->ws_io_bytes = 0;
    SG_HIP(hipMalloc(&p->ws_io, bytes));
    p->ws_io_bytes = bytes;
    return SG_OK;
}

template <typename T>
static DenseBufs<T> dbufs(const sg_dense_plan *p, int B, const void *y) {
    DenseBufs<T> d;
    d.A = (const T *)p->A; d.n = p->n; d.npad = p->npad; d.L = p->L; d.M = p->M; d.LM = p->LM; d.B = B; d.P = p->P;
    d.y = (const T *)(y ? y : p->ws_y); d.z = (T *)p->ws_z; d.beta = (T *)p->ws_beta; d.s = (T *)p->ws_s;
    d.part = (T *)p->ws_part; d.nsplit = p->nsplit; d.tau2 = p->ws_tau2; d.bsq = nullptr;
    d.sec_bsq = p->ws_sec_bsq;
    d.ons_mode = 0;
    d.ons = nullptr;
    return d;
}

static int plan_common(int n, int L, int M, double P, int precision, sg_dense_plan **out, sg_dense_plan **pp) {
    SG_CHECK_ARG(out, "null argument");
    SG_CHECK_ARG(n > 0 && L > 0 && M > 0 && (M & (M - 1)) == 0, "bad (n, L, M)");
    SG_CHECK_ARG(precision == SG_F32 || precision == SG_F64, "precision must be SG_F32 or SG_F64");
    SG_CHECK_ARG(P > 0, "P must be positive");
    const long long LM = (long long)L * M;
    SG_CHECK_ARG(LM < (1LL << 31), "L*M too large");
    SG_CHECK_ARG(precision == SG_F64 || LM % 32 == 0, "the f32 matrix-core path needs L*M to be a multiple of 32");
    SG_TRY(ensure_device());
    sg_dense_plan *p = new sg_dense_plan();
    hipGetDevice(&p->device);
    p->precision = precision; p->n = n; p->npad = (n + 31) / 32 * 32; p->L = L; p->M = M; p->LM = (int)LM; p->P = P;
    // split K = LM of the A beta product so that the grid covers the chip
    if (precision == SG_F32) {
        const long long tiles = (long long)((n + 127) / 128);
        long long ns = std::max<long long>(1, 2048 / std::max<long long>(1, tiles));
        ns = std::min<long long>(ns, std::max<long long>(1, LM / 1024));
        p->nsplit = (int)ns;
    }
    const size_t bytes = (size_t)n * LM * (precision == SG_F64 ? 8 : 4);
    if (hipMalloc(&p->A, bytes) != hipSuccess) {
        delete p;
        return fail(SG_ERR_NOMEM, "cannot allocate the %zu-byte design matrix", bytes);
    }
    *pp = p;
    *out = p;
    return SG_OK;
}

template <typename T>
static int amp_impl(sg_dense_plan *p, const void *d_y, int B, int t_max, hipStream_t s) {
    SG_TRY(dense_ensure_ws(p, B));
    DenseBufs<T> d = dbufs<T>(p, B, d_y);
    SG_HIP(hipMemsetAsync(p->ws_beta, 0, (size_t)B * p->LM * sizeof(T), s));
    for (int t = 0; t < t_max; ++t) {  // sparc_new.py:901-910, fixed t_max iterations
        if (t > 0) SG_TRY(dense_launch_ab<T>(d, s));
        SG_TRY(dense_launch_residual<T>(d, t, s));
        SG_TRY(dense_launch_az<T>(d, s));
        SG_TRY(dense_launch_eta<T>(d, s));
    }
    return SG_OK;
}

template <typename T>
__global__ void cast_to(const double *in, T *out, size_t nn) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nn; i += (size_t)gridDim.x * blockDim.x)
        out[i] = (T)in[i];
}
template <typename T>
__global__ void cast_from(const T *in, double *out, size_t nn) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nn; i += (size_t)gridDim.x * blockDim.x)
        out[i] = (double)in[i];
}
template <typename T>
__global__ void onehot_kernel(const int32_t *idx, int L, int M, double val, T *beta) {
    const int b = blockIdx.y;
    for (int l = blockIdx.x * blockDim.x + threadIdx.x; l < L; l += gridDim.x * blockDim.x)
        beta[(long)b * L * M + (long)l * M + idx[(long)b * L + l]] = (T)val;
}
template <typename T>
__global__ void sum_split(const T *part, int nsplit, int B, int n, T *x) {
    const int b = blockIdx.y;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        T r = T(0);
        for (int sp = 0; sp < nsplit; ++sp) r += part[((long)sp * B + b) * n + i];
        x[(long)b * n + i] = r;
    }
}

static unsigned grid_for(size_t nn) { return (unsigned)std::min<size_t>(65535, (nn + 255) / 256); }

// One AMP iteration from a caller-supplied state (sparc_amp_single_it,
// sparc_new.py:975-990): beta, z, tau^2 -> beta', z', tau^2'.
template <typename T>
static int iteration_impl(sg_dense_plan *p, const double *y, const double *beta, const double *z, double tau_sqr,
                          double *beta_out, double *z_out, double *tau_out, hipStream_t s) {
    SG_TRY(dense_ensure_ws(p, 1));
    const size_t n = p->n, LM = p->LM;
    SG_TRY(dense_ensure_io(p, (LM + 2 * p->npad) * 8));
    double *io = (double *)p->ws_io;
    std::vector<double> zp(p->npad, 0.0);
    std::copy(z, z + n, zp.begin());
    SG_HIP(hipMemcpyAsync(io, beta, LM * 8, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(io + LM, zp.data(), p->npad * 8, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(io + LM + p->npad, y, n * 8, hipMemcpyHostToDevice, s));
    SG_HIP(hipMemcpyAsync(p->ws_tau2, &tau_sqr, 8, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(cast_to<T>, dim3(grid_for(LM)), dim3(256), 0, s, (const double *)io, (T *)p->ws_beta, LM);
    hipLaunchKernelGGL(cast_to<T>, dim3(grid_for(p->npad)), dim3(256), 0, s, (const double *)(io + LM),
                       (T *)p->ws_z, (size_t)p->npad);
    hipLaunchKernelGGL(cast_to<T>, dim3(grid_for(n)), dim3(256), 0, s, (const double *)(io + LM + p->npad),
                       (T *)p->ws_y, n);
    DenseBufs<T> d = dbufs<T>(p, 1, nullptr);
    SG_TRY(dense_launch_bsq<T>(d, s));
    SG_TRY(dense_launch_ab<T>(d, s));
    SG_TRY(dense_launch_residual<T>(d, 1, s));
    SG_TRY(dense_launch_az<T>(d, s));
    SG_TRY(dense_launch_eta<T>(d, s));
    hipLaunchKernelGGL(cast_from<T>, dim3(grid_for(LM)), dim3(256), 0, s, (const T *)p->ws_beta, io, LM);
    hipLaunchKernelGGL(cast_from<T>, dim3(grid_for(n)), dim3(256), 0, s, (const T *)p->ws_z, io + LM, n);
    SG_HIP(hipMemcpyAsync(beta_out, io, LM * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(z_out, io + LM, n * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipMemcpyAsync(tau_out, p->ws_tau2, 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    return SG_OK;
}


// The AMP <-> BP integrated decoders (sparc_new.py:257-282 naive, :411-439
// naive posteriors, :472-502 integrated, :675-705 integrated posteriors) for a
// batch sharing the design: every LDPC block of every codeword goes through
// one batched BP launch per iteration.  bits [B][nblk K] = app[:K] < 0 of the
// final 200-iteration (bp_its_final) decode; tau_hist [B][t_max] optional.
template <typename T>
static int integ_impl(sg_dense_plan *p, sg_graph *g, int mode, int N, int K, const void *d_y, int B, int t_max,
                      int its, int its_final, uint8_t *d_bits, double *d_tau_hist, hipStream_t s) {
    const int logM = [&] { int k = 0; while ((1 << k) < p->M) ++k; return k; }();
    const int nbits = p->L * logM, nblk = nbits / N;
    SG_TRY(dense_ensure_ws(p, B));
    SG_TRY(integ_ensure_ws(p, B, nbits));
    DenseBufs<T> d = dbufs<T>(p, B, d_y);
    const double snp = std::sqrt((double)p->n * (p->P / p->L));
    const bool naive = mode == SG_INT_NAIVE || mode == SG_INT_NAIVE_POST;
    const bool post = mode == SG_INT_NAIVE_POST || mode == SG_INT_DIFF_POST;
    T *alpha_w = (T *)p->wi_alpha, *gamma = (T *)p->wi_gamma, *vk0 = (T *)p->wi_vk0, *vk = (T *)p->wi_vk;
    T *llr = (T *)p->wi_llr, *app = (T *)p->wi_app;
    const size_t nb = (size_t)B * nbits;
    const int prec = sizeof(T) == 8 ? SG_F64 : SG_F32;
    SG_HIP(hipMemsetAsync(p->ws_beta, 0, (size_t)B * p->LM * sizeof(T), s));
    SG_HIP(hipMemsetAsync(p->ws_sec_bsq, 0, (size_t)B * p->L * sizeof(double), s));
    DenseBufs<T> da = d;  // eta writes the weighted alpha (the MMSE estimate) here
    da.beta = alpha_w;
    if (!naive) {
        d.ons_mode = mode == SG_INT_DIFF ? 1 : 2;
        d.ons = p->wi_ons;
    }
    for (int t = 0; t < t_max; ++t) {
        if (!naive && t > 0)  // sum of the differentiated eta with the previous tau^2
            SG_TRY(integ_launch_deta<T>(post ? 1 : 0, d.beta, gamma, alpha_w, snp, vk, vk0, p->ws_tau2, B, p->L, p->M,
                                        snp, p->wi_part, p->wi_ons, (T *)nullptr, s));
        if (t > 0) SG_TRY(dense_launch_ab<T>(d, s));
        SG_TRY(dense_launch_residual<T>(d, t, s));  // z; tau^2 = ||z||^2 / n
        SG_TRY(dense_launch_az<T>(d, s));            // s = beta + A^T z
        if (d_tau_hist)
            SG_HIP(hipMemcpy2DAsync(d_tau_hist + t, (size_t)t_max * 8, p->ws_tau2, 8, 8, B, hipMemcpyDeviceToDevice, s));
        SG_TRY(dense_launch_eta<T>(da, s));
        SG_TRY(glue_launch_llr<T>(alpha_w, B, p->L, p->M, 0, p->L, 1.0 / snp, nbits, vk0, 1, s));  // P(bit = 0)
        SG_TRY(integ_launch_llr<T>(vk0, nb, llr, s));
        if (t == t_max - 1) {
            SG_TRY(sg_ldpc_decode_device(g, SG_SUMPROD2, prec, llr, B * nblk, its_final, 0.7, app, p->wi_it, s));
            SG_TRY(integ_launch_hard_bits<T>(app, B * nblk, N, K, d_bits, s));
            break;
        }
        SG_TRY(sg_ldpc_decode_device(g, SG_SUMPROD2, prec, llr, B * nblk, its, 0.7, app, p->wi_it, s));
        SG_TRY(integ_launch_probs<T>(app, nb, vk, s));
        if (!post) {
            SG_TRY(integ_launch_bp_to_beta<T>(vk, B, p->L, p->M, snp, 0, d.beta, s));
        } else {
            SG_TRY(integ_launch_bp_to_beta<T>(vk, B, p->L, p->M, snp, 1, gamma, s));
            SG_TRY(integ_launch_update<T>(gamma, alpha_w, snp, B, p->L, p->M, snp, d.beta, s));
        }
        if (naive) SG_TRY(dense_launch_bsq<T>(d, s));  // ||beta||^2 of the BP-derived beta for the Onsager term
    }
    return SG_OK;
}

// The soft-glue pieces on host arrays (the reference's functions, batched over B).
template <typename F>
static int integ_host_call(int precision, std::initializer_list<std::pair<const double *, size_t>> ins,
                           std::initializer_list<std::pair<double *, size_t>> outs, F &&launch) {
    SG_CHECK_ARG(precision == SG_F32 || precision == SG_F64, "bad precision");
    SG_TRY(ensure_device());
    hipStream_t s = lib_stream();
    const size_t rs = precision == SG_F64 ? 8 : 4;
    std::vector<void *> dev;
    auto cleanup = [&] {
        for (void *v : dev) hipFree(v);
    };
    int rc = SG_OK;
    std::vector<void *> din, dout;
    for (auto &in : ins) {
        void *a = nullptr, *st = nullptr;
        if (hipMalloc(&a, std::max<size_t>(1, in.second * rs)) != hipSuccess ||
            hipMalloc(&st, std::max<size_t>(1, in.second * 8)) != hipSuccess) {
            if (a) hipFree(a);
            if (st) hipFree(st);
            cleanup();
            return fail(SG_ERR_NOMEM, "device buffers");
        }
        dev.push_back(a);
        dev.push_back(st);
        if (in.first) {
            if (hipMemcpyAsync(st, in.first, in.second * 8, hipMemcpyHostToDevice, s) != hipSuccess) rc = SG_ERR_HIP;
            if (precision == SG_F64)
                hipMemcpyAsync(a, st, in.second * 8, hipMemcpyDeviceToDevice, s);
            else
                hipLaunchKernelGGL(cast_to<float>, dim3(grid_for(in.second)), dim3(256), 0, s, (const double *)st,
                                   (float *)a, in.second);
        }
        din.push_back(in.first ? a : nullptr);
    }
    for (auto &o : outs) {
        void *a = nullptr, *st = nullptr;
        if (hipMalloc(&a, std::max<size_t>(1, o.second * rs)) != hipSuccess ||
            hipMalloc(&st, std::max<size_t>(1, o.second * 8)) != hipSuccess) {
            if (a) hipFree(a);
            if (st) hipFree(st);
            cleanup();
            return fail(SG_ERR_NOMEM, "device buffers");
        }
        dev.push_back(a);
        dev.push_back(st);
        dout.push_back(a);
        dout.push_back(st);
    }
    if (rc == SG_OK) rc = launch(din, dout, s);
    size_t k = 0;
    for (auto &o : outs) {
        void *a = dout[2 * k], *st = dout[2 * k + 1];
        ++k;
        if (rc != SG_OK) break;
        if (precision == SG_F64)
            hipMemcpyAsync(st, a, o.second * 8, hipMemcpyDeviceToDevice, s);
        else
            hipLaunchKernelGGL(cast_from<float>, dim3(grid_for(o.second)), dim3(256), 0, s, (const float *)a,
                               (double *)st, o.second);
        if (hipMemcpyAsync(o.first, st, o.second * 8, hipMemcpyDeviceToHost, s) != hipSuccess) rc = SG_ERR_HIP;
    }
    if (hipStreamSynchronize(s) != hipSuccess && rc == SG_OK) rc = SG_ERR_HIP;
    cleanup();
    return rc == SG_OK ? SG_OK : fail(rc, "integrated glue call failed");
}

}  // namespace sg

using namespace sg;

extern "C" {

int sg_dense_plan_create(const double *A, int n, int L, int M, double P, int precision, sg_dense_plan **out) {
    SG_CHECK_ARG(A, "A is NULL");
    sg_dense_plan *p = nullptr;
    SG_TRY(plan_common(n, L, M, P, precision, out, &p));
    const size_t nn = (size_t)n * p->LM;
    hipStream_t s = lib_stream();
    int rc = SG_OK;
    if (precision == SG_F64) {
        if (hipMemcpy(p->A, A, nn * 8, hipMemcpyHostToDevice) != hipSuccess) rc = SG_ERR_HIP;
    } else {
        // stream the double matrix through a staging buffer, cast on the device
        const size_t chunk = std::min<size_t>(nn, (size_t)1 << 26);
        double *stage = nullptr;
        if (hipMalloc(&stage, chunk * 8) != hipSuccess) rc = SG_ERR_NOMEM;
        for (size_t o = 0; rc == SG_OK && o < nn; o += chunk) {
            const size_t c = std::min(chunk, nn - o);
            if (hipMemcpyAsync(stage, A + o, c * 8, hipMemcpyHostToDevice, s) != hipSuccess) rc = SG_ERR_HIP;
            hipLaunchKernelGGL(cast_to<float>, dim3(grid_for(c)), dim3(256), 0, s, stage, (float *)p->A + o, c);
            if (hipStreamSynchronize(s) != hipSuccess) rc = SG_ERR_HIP;
        }
        if (stage) hipFree(stage);
    }
    if (rc != SG_OK) {
        sg_dense_plan_destroy(p);
        *out = nullptr;
        return fail(rc, "uploading the design matrix failed");
    }
    return SG_OK;
}

int sg_dense_plan_create_random(int n, int L, int M, double P, uint64_t seed, int precision, sg_dense_plan **out) {
    sg_dense_plan *p = nullptr;
    SG_TRY(plan_common(n, L, M, P, precision, out, &p));
    hipStream_t s = lib_stream();
    int rc = precision == SG_F64 ? dense_launch_gen_A<double>((double *)p->A, n, p->LM, seed, s)
                                 : dense_launch_gen_A<float>((float *)p->A, n, p->LM, seed, s);
    if (rc == SG_OK && hipStreamSynchronize(s) != hipSuccess) rc = SG_ERR_HIP;
    if (rc != SG_OK) {
        sg_dense_plan_destroy(p);
        *out = nullptr;
        return rc;
    }
    return SG_OK;
}

int sg_dense_plan_destroy(sg_dense_plan *p) {
    if (!p) return SG_OK;
    dense_free_ws(p);
    integ_free_ws(p);
    if (p->A) hipFree(p->A);
    delete p;
    return SG_OK;
}

int sg_dense_plan_info(const sg_dense_plan *p, int *n, int *L, int *M, int *nsplit) {
    SG_CHECK_ARG(p, "plan is NULL");
    if (n) *n = p->n;
    if (L) *L = p->L;
    if (M) *M = p->M;
    if (nsplit) *nsplit = p->nsplit;
    return SG_OK;
}

int sg_dense_amp_device(sg_dense_plan *p, const void *d_y, int B, int t_max, void *d_beta, void *d_s, void *stream) {
    SG_CHECK_ARG(p && d_y, "null argument");
    SG_CHECK_ARG(t_max >= 1, "t_max must be >= 1");
    if (B <= 0) return SG_OK;
    SG_TRY(ensure_device());
    SG_HIP(hipSetDevice(p->device));
    hipStream_t s = pick_stream(stream);
    const size_t rs = rsize(p), nb = (size_t)B * p->LM * rs;
    SG_TRY(p->precision == SG_F64 ? amp_impl<double>(p, d_y, B, t_max, s) : amp_impl<float>(p, d_y, B, t_max, s));
    if (d_beta) SG_HIP(hipMemcpyAsync(d_beta, p->ws_beta, nb, hipMemcpyDeviceToDevice, s));
    if (d_s) SG_HIP(hipMemcpyAsync(d_s, p->ws_s, nb, hipMemcpyDeviceToDevice, s));
    return SG_OK;
}

int sg_dense_amp(sg_dense_plan *p, const double *y, int B, int t_max, double *beta, double *s_out) {
    SG_CHECK_ARG(p && y && beta && s_out, "null argument");
    if (B <= 0) return SG_OK;
    SG_TRY(ensure_device());
    SG_HIP(hipSetDevice(p->device));
    hipStream_t s = lib_stream();
    SG_TRY(dense_ensure_ws(p, B));
    const size_t ny = (size_t)B * p->n, nb = (size_t)B * p->LM;
    SG_TRY(dense_ensure_io(p, std::max(ny, nb) * 8));
    SG_HIP(hipMemcpyAsync(p->ws_io, y, ny * 8, hipMemcpyHostToDevice, s));
    if (p->precision == SG_F64) {
        SG_HIP(hipMemcpyAsync(p->ws_y, p->ws_io, ny * 8, hipMemcpyDeviceToDevice, s));
        SG_TRY(amp_impl<double>(p, p->ws_y, B, t_max, s));
        SG_HIP(hipMemcpyAsync(beta, p->ws_beta, nb * 8, hipMemcpyDeviceToHost, s));
        SG_HIP(hipMemcpyAsync(s_out, p->ws_s, nb * 8, hipMemcpyDeviceToHost, s));
    } else {
        hipLaunchKernelGGL(cast_to<float>, dim3(grid_for(ny)), dim3(256), 0, s, (const double *)p->ws_io,
                           (float *)p->ws_y, ny);
        SG_TRY(amp_impl<float>(p, p->ws_y, B, t_max, s));
        hipLaunchKernelGGL(cast_from<float>, dim3(grid_for(nb)), dim3(256), 0, s, (const float *)p->ws_beta,
                           (double *)p->ws_io, nb);
        SG_HIP(hipMemcpyAsync(beta, p->ws_io, nb * 8, hipMemcpyDeviceToHost, s));
        SG_HIP(hipStreamSynchronize(s));
        hipLaunchKernelGGL(cast_from<float>, dim3(grid_for(nb)), dim3(256), 0, s, (const float *)p->ws_s,
                           (double *)p->ws_io, nb);
        SG_HIP(hipMemcpyAsync(s_out, p->ws_io, nb * 8, hipMemcpyDeviceToHost, s));
    }
    SG_HIP(hipStreamSynchronize(s));
    return SG_OK;
}

int sg_dense_amp_iteration(sg_dense_plan *p, const double *y, const double *beta, const double *z, double tau_sqr,
                           double *beta_out, double *z_out, double *tau_sqr_out) {
    SG_CHECK_ARG(p && y && beta && z && beta_out && z_out && tau_sqr_out, "null argument");
    SG_CHECK_ARG(tau_sqr > 0, "tau_sqr must be positive");
    SG_TRY(ensure_device());
    SG_HIP(hipSetDevice(p->device));
    hipStream_t s = lib_stream();
    return p->precision == SG_F64 ? iteration_impl<double>(p, y, beta, z, tau_sqr, beta_out, z_out, tau_sqr_out, s)
                                  : iteration_impl<float>(p, y, beta, z, tau_sqr, beta_out, z_out, tau_sqr_out, s);
}

// x[b] = A beta0[b], beta0 one-hot per section with value sqrt(n P / L) at
// idx[b][l] (sparc_new.py:46-49), on the device.
int sg_dense_encode_device(sg_dense_plan *p, const int32_t *d_idx, int B, void *d_x, void *stream) {
    SG_CHECK_ARG(p && d_idx && d_x, "null argument");
    if (B <= 0) return SG_OK;
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    SG_TRY(dense_ensure_ws(p, B));
    const double val = std::sqrt((double)p->n * (p->P / p->L));
    const size_t rs = rsize(p);
    SG_HIP(hipMemsetAsync(p->ws_beta, 0, (size_t)B * p->LM * rs, s));
    if (p->precision == SG_F64) {
        hipLaunchKernelGGL(onehot_kernel<double>, dim3((p->L + 255) / 256, B), dim3(256), 0, s, d_idx, p->L, p->M, val,
                           (double *)p->ws_beta);
        DenseBufs<double> d = dbufs<double>(p, B, nullptr);
        d.nsplit = 1;
        SG_TRY(dense_launch_ab<double>(d, s));
        hipLaunchKernelGGL(sum_split<double>, dim3((p->n + 255) / 256, B), dim3(256), 0, s,
                           (const double *)p->ws_part, 1, B, p->n, (double *)d_x);
    } else {
        hipLaunchKernelGGL(onehot_kernel<float>, dim3((p->L + 255) / 256, B), dim3(256), 0, s, d_idx, p->L, p->M, val,
                           (float *)p->ws_beta);
        DenseBufs<float> d = dbufs<float>(p, B, nullptr);
        SG_TRY(dense_launch_ab<float>(d, s));
        hipLaunchKernelGGL(sum_split<float>, dim3((p->n + 255) / 256, B), dim3(256), 0, s, (const float *)p->ws_part,
                           p->nsplit, B, p->n, (float *)d_x);
    }
    SG_HIP(hipGetLastError());
    return SG_OK;
}

int sg_dense_state_device(sg_dense_plan *p, void **d_beta, void **d_s) {
    SG_CHECK_ARG(p, "plan is NULL");
    if (d_beta) *d_beta = p->ws_beta;
    if (d_s) *d_s = p->ws_s;
    return SG_OK;
}

int sg_dense_plan_matrix_device(const sg_dense_plan *p, const void **d_A) {
    SG_CHECK_ARG(p && d_A, "null argument");
    *d_A = p->A;
    return SG_OK;
}

int sg_dense_map_device(sg_dense_plan *p, const void *d_s, int B, int32_t *d_idx, void *stream) {
    SG_CHECK_ARG(p && d_s && d_idx, "null argument");
    if (B <= 0) return SG_OK;
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    return p->precision == SG_F64 ? dense_launch_map<double>((const double *)d_s, B, p->L, p->M, d_idx, s)
                                  : dense_launch_map<float>((const float *)d_s, B, p->L, p->M, d_idx, s);
}

// Bit LLRs of sections [l0, l0 + nl) from soft section estimates beta
// [B][L*M] (beta_estimate_to_bp_probs + the clip/log of ldpc_bp,
// sparc_new.py:1118-1138, 1167-1169).  llr row b starts at b * llr_ld.
// probs_only: write the bit-0 probabilities themselves (no clip, no log).
int sg_beta_to_llr_device(int precision, const void *d_beta, int B, int L, int M, double sqrt_nPl, int l0, int nl,
                          int llr_ld, int probs_only, void *d_llr, void *stream) {
    SG_CHECK_ARG(d_beta && d_llr, "null argument");
    SG_CHECK_ARG(M > 1 && (M & (M - 1)) == 0 && l0 >= 0 && nl >= 0 && l0 + nl <= L, "bad section range");
    SG_CHECK_ARG(sqrt_nPl > 0, "sqrt(n P_l) must be positive");
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    const double inv = 1.0 / sqrt_nPl;
    return precision == SG_F64
               ? glue_launch_llr<double>((const double *)d_beta, B, L, M, l0, nl, inv, llr_ld, (double *)d_llr,
                                         probs_only, s)
               : glue_launch_llr<float>((const float *)d_beta, B, L, M, l0, nl, inv, llr_ld, (float *)d_llr,
                                        probs_only, s);
}

int sg_concat_count_errors_device(int precision, const int32_t *d_map_idx, const int32_t *d_true_idx, int B, int L,
                                  int L_unprotected, int logM, const void *d_app, const uint8_t *d_info, int mults,
                                  int N, int K, int64_t *d_counts, void *stream) {
    SG_CHECK_ARG(d_map_idx && d_true_idx && d_app && d_info && d_counts, "null device buffer");
    SG_CHECK_ARG(L_unprotected >= 0 && L_unprotected <= L && mults >= 0 && K <= N, "bad lengths");
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    return precision == SG_F64
               ? concat_launch_count<double>(d_map_idx, d_true_idx, B, L, L_unprotected, logM, (const double *)d_app,
                                             d_info, mults, N, K, d_counts, s)
               : concat_launch_count<float>(d_map_idx, d_true_idx, B, L, L_unprotected, logM, (const float *)d_app,
                                            d_info, mults, N, K, d_counts, s);
}

int sg_integrated_decode_device(sg_dense_plan *p, sg_graph *g, int mode, int K, const void *d_y, int B, int t_max,
                                int bp_its, int bp_its_final, uint8_t *d_bits, double *d_tau2, void *stream) {
    SG_CHECK_ARG(p && g && d_y && d_bits, "null argument");
    SG_CHECK_ARG(mode >= SG_INT_NAIVE && mode <= SG_INT_DIFF_POST, "unknown integrated decoder %d", mode);
    SG_CHECK_ARG(t_max >= 1 && bp_its >= 0 && bp_its_final >= 0, "bad iteration counts");
    int N = 0, nc = 0;
    SG_TRY(sg_ldpc_graph_info(g, &N, &nc, nullptr, nullptr, nullptr));
    int logM = 0;
    while ((1 << logM) < p->M) ++logM;
    SG_CHECK_ARG(N > 0 && (p->L * logM) % N == 0, "L log2 M = %d bits must be a multiple of the block length %d",
                 p->L * logM, N);  // ldpc_bp's assert (sparc_new.py:1171)
    SG_CHECK_ARG(K > 0 && K <= N, "bad information length %d", K);
    if (B <= 0) return SG_OK;
    SG_TRY(ensure_device());
    SG_HIP(hipSetDevice(p->device));
    hipStream_t s = pick_stream(stream);
    return p->precision == SG_F64
               ? integ_impl<double>(p, g, mode, N, K, d_y, B, t_max, bp_its, bp_its_final, d_bits, d_tau2, s)
               : integ_impl<float>(p, g, mode, N, K, d_y, B, t_max, bp_its, bp_its_final, d_bits, d_tau2, s);
}

int sg_integrated_decode(sg_dense_plan *p, sg_graph *g, int mode, int K, const double *y, int B, int t_max,
                         int bp_its, int bp_its_final, uint8_t *bits, double *tau2) {
    SG_CHECK_ARG(p && g && y && bits, "null argument");
    if (B <= 0) return SG_OK;
    SG_TRY(ensure_device());
    SG_HIP(hipSetDevice(p->device));
    int N = 0;
    SG_TRY(sg_ldpc_graph_info(g, &N, nullptr, nullptr, nullptr, nullptr));
    int logM = 0;
    while ((1 << logM) < p->M) ++logM;
    SG_CHECK_ARG(N > 0 && (p->L * logM) % N == 0, "L log2 M must be a multiple of the block length");
    const size_t nbits = (size_t)B * (p->L * logM / N) * K;
    hipStream_t s = lib_stream();
    SG_TRY(dense_ensure_ws(p, B));
    const size_t rs = rsize(p), ny = (size_t)B * p->n;
    SG_TRY(dense_ensure_io(p, ny * 8 + nbits + (size_t)B * t_max * 8 + 64));
    double *io = (double *)p->ws_io;
    uint8_t *dbits = (uint8_t *)(io + ny);
    double *dtau = (double *)((char *)p->ws_io + ((ny * 8 + nbits + 63) / 64) * 64);
    SG_HIP(hipMemcpyAsync(io, y, ny * 8, hipMemcpyHostToDevice, s));
    if (p->precision == SG_F32)  // cast into the plan's own y buffer
        hipLaunchKernelGGL(cast_to<float>, dim3(grid_for(ny)), dim3(256), 0, s, (const double *)io, (float *)p->ws_y,
                           ny);
    const void *dy = p->precision == SG_F32 ? p->ws_y : (const void *)io;
    (void)rs;
    SG_TRY(sg_integrated_decode_device(p, g, mode, K, dy, B, t_max, bp_its, bp_its_final, dbits,
                                       tau2 ? dtau : nullptr, s));
    SG_HIP(hipMemcpyAsync(bits, dbits, nbits, hipMemcpyDeviceToHost, s));
    if (tau2) SG_HIP(hipMemcpyAsync(tau2, dtau, (size_t)B * t_max * 8, hipMemcpyDeviceToHost, s));
    SG_HIP(hipStreamSynchronize(s));
    return SG_OK;
}

int sg_bp_output_to_beta(int precision, const double *probs, int B, int L, int M, double sqrt_nPl, double *beta) {
    SG_CHECK_ARG(probs && beta && B >= 0 && L > 0 && M > 1 && (M & (M - 1)) == 0, "bad argument");
    int logM = 0;
    while ((1 << logM) < M) ++logM;
    const size_t np = (size_t)B * L * logM, nbeta = (size_t)B * L * M;
    return integ_host_call(precision, {{probs, np}}, {{beta, nbeta}}, [&](auto &in, auto &out, hipStream_t s) {
        return precision == SG_F64
                   ? integ_launch_bp_to_beta<double>((const double *)in[0], B, L, M, sqrt_nPl, 0, (double *)out[0], s)
                   : integ_launch_bp_to_beta<float>((const float *)in[0], B, L, M, sqrt_nPl, 0, (float *)out[0], s);
    });
}

int sg_update_using_bp_probs(int precision, const double *gamma, const double *alpha, int B, int L, int M,
                             double sqrt_nPl, double *beta) {
    SG_CHECK_ARG(gamma && alpha && beta && B >= 0 && L > 0 && M > 0, "bad argument");
    const size_t nn = (size_t)B * L * M;
    return integ_host_call(precision, {{gamma, nn}, {alpha, nn}}, {{beta, nn}}, [&](auto &in, auto &out, hipStream_t s) {
        return precision == SG_F64
                   ? integ_launch_update<double>((const double *)in[0], (const double *)in[1], 1.0, B, L, M, sqrt_nPl,
                                                 (double *)out[0], s)
                   : integ_launch_update<float>((const float *)in[0], (const float *)in[1], 1.0, B, L, M, sqrt_nPl,
                                                (float *)out[0], s);
    });
}

int sg_differentiated_eta(int precision, int posteriors, const double *beta, const double *gamma,
                          const double *alpha, const double *vk, const double *vk0, const double *tau2, int B, int L,
                          int M, double sqrt_nPl, double *out) {
    SG_CHECK_ARG(beta && alpha && vk && vk0 && tau2 && out && (!posteriors || gamma), "null argument");
    SG_CHECK_ARG(B >= 0 && L > 0 && M > 1 && (M & (M - 1)) == 0, "bad shape");
    int logM = 0;
    while ((1 << logM) < M) ++logM;
    const size_t nn = (size_t)B * L * M, nv = (size_t)B * L * logM;
    SG_TRY(ensure_device());
    double *dtau = nullptr, *dpart = nullptr;
    SG_HIP(hipMalloc(&dtau, std::max<size_t>(1, B) * 8));
    SG_HIP(hipMalloc(&dpart, std::max<size_t>(1, (size_t)B * L) * 8));
    hipMemcpy(dtau, tau2, (size_t)B * 8, hipMemcpyHostToDevice);
    const int rc = integ_host_call(
        precision, {{beta, nn}, {gamma, gamma ? nn : 0}, {alpha, nn}, {vk, nv}, {vk0, nv}}, {{out, nn}},
        [&](auto &in, auto &o, hipStream_t s) {
            return precision == SG_F64
                       ? integ_launch_deta<double>(posteriors ? 1 : 0, (const double *)in[0], (const double *)in[1],
                                                   (const double *)in[2], 1.0, (const double *)in[3],
                                                   (const double *)in[4], dtau, B, L, M, sqrt_nPl, dpart, nullptr,
                                                   (double *)o[0], s)
                       : integ_launch_deta<float>(posteriors ? 1 : 0, (const float *)in[0], (const float *)in[1],
                                                  (const float *)in[2], 1.0, (const float *)in[3],
                                                  (const float *)in[4], dtau, B, L, M, sqrt_nPl, dpart, nullptr,
                                                  (float *)o[0], s);
        });
    hipFree(dtau);
    hipFree(dpart);
    return rc;
}

}  // extern "C"
