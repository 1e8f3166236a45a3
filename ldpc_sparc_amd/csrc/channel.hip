// Device-side encoder and channel for the throughput mode:
// random message bits, the systematic LDPC encoder (ldpc.py:400-460) as a
// GF(2) product with the code's parity generator, bits -> section indices
// (sparc.py:330-364, MSB first), AWGN (sparc_sim.py:179-204) and BPSK LLRs
// (ldpc_awgn.py:39-56), all keyed by Philox4x32-10 counters so that a
// Monte-Carlo block is the same on any rank or GPU count.  Parity mode (seed
// for seed with the reference's numpy generators) stays on the host.
#include <algorithm>
#include <vector>

#include "common.hpp"
#include "philox.hpp"

struct sg_ldpc_encoder {
    int K = 0, N = 0, Kw = 0;  // information bits, codeword bits, 64-bit words per info word
    uint64_t *pt = nullptr;    // [N-K][Kw] parity bit j = parity of popcount(pt[j] & info)
};

namespace sg {

namespace {

// Philox key domains: independent streams for bits and noise
constexpr uint32_t kBitsDomain = 0xB175u, kNoiseDomain = 0x0A1Eu;

// bit j of row b: bit (j mod 128) of Philox((j / 128, b, stream), seed ^ domain)
__global__ __launch_bounds__(256) void rng_bits_kernel(uint64_t seed, uint64_t stream_id, int nbits, uint8_t *bits) {
    const int b = blockIdx.y;
    const int nblk = (nbits + 127) / 128;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < nblk; q += gridDim.x * blockDim.x) {
        uint32_t c[4] = {(uint32_t)q, (uint32_t)b, (uint32_t)stream_id, (uint32_t)(stream_id >> 32)};
        philox4x32_10(c, (uint32_t)seed ^ kBitsDomain, (uint32_t)(seed >> 32));
        uint8_t *o = bits + (size_t)b * nbits + (size_t)q * 128;
        const int m = min(128, nbits - q * 128);
        for (int j = 0; j < m; ++j) o[j] = (uint8_t)((c[j >> 5] >> (j & 31)) & 1u);
    }
}

// section index of every logM-bit group, MSB first (bin_arr_2_msg_vector)
__global__ __launch_bounds__(256) void bits_to_sections_kernel(const uint8_t *bits, size_t bit_stride, int L, int logM,
                                                               int32_t *idx, size_t idx_stride) {
    const int b = blockIdx.y;
    for (int l = blockIdx.x * blockDim.x + threadIdx.x; l < L; l += gridDim.x * blockDim.x) {
        const uint8_t *x = bits + (size_t)b * bit_stride + (size_t)l * logM;
        int v = 0;
        for (int j = 0; j < logM; ++j) v = (v << 1) | (x[j] & 1);
        idx[(size_t)b * idx_stride + l] = v;
    }
}

// y = x + sigma g, g ~ N(0, 1) from Philox((i / 2, b, stream), seed ^ domain)
template <typename T>
__global__ __launch_bounds__(256) void awgn_kernel(uint64_t seed, uint64_t stream_id, const T *x, int n, double sigma,
                                                   T *y) {
    const int b = blockIdx.y;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; 2 * q < n; q += gridDim.x * blockDim.x) {
        uint32_t c[4] = {(uint32_t)q, (uint32_t)b, (uint32_t)stream_id, (uint32_t)(stream_id >> 32)};
        philox4x32_10(c, (uint32_t)seed ^ kNoiseDomain, (uint32_t)(seed >> 32));
        double g0, g1;
        philox_normal2(c, &g0, &g1);
        const size_t o = (size_t)b * n + 2 * (size_t)q;
        y[o] = (T)((double)x[o] + sigma * g0);
        if (2 * q + 1 < n) y[o + 1] = (T)((double)x[o + 1] + sigma * g1);
    }
}

// BPSK 1 - 2 c over AWGN, channel LLR 2 y / sigma^2 (ldpc_awgn.py:49-56)
template <typename T>
__global__ __launch_bounds__(256) void bpsk_llr_kernel(uint64_t seed, uint64_t stream_id, const uint8_t *cw, int N,
                                                       double sigma2, T *llr) {
    const int b = blockIdx.y;
    const double sigma = sqrt(sigma2), g = 2.0 / sigma2;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; 2 * q < N; q += gridDim.x * blockDim.x) {
        uint32_t c[4] = {(uint32_t)q, (uint32_t)b, (uint32_t)stream_id, (uint32_t)(stream_id >> 32)};
        philox4x32_10(c, (uint32_t)seed ^ kNoiseDomain, (uint32_t)(seed >> 32));
        double g0, g1;
        philox_normal2(c, &g0, &g1);
        const size_t o = (size_t)b * N + 2 * (size_t)q;
        llr[o] = (T)(g * ((1.0 - 2.0 * cw[o]) + sigma * g0));
        if (2 * q + 1 < N) llr[o + 1] = (T)(g * ((1.0 - 2.0 * cw[o + 1]) + sigma * g1));
    }
}

// Systematic GF(2) encoder, one workgroup per codeword: the information word
// is packed into 64-bit words with wave ballots (LDS), parity bit j is the
// parity of popcount(pt[j] & info).  cw[:K] = info, cw[K:] = parity.
__global__ __launch_bounds__(256) void ldpc_encode_kernel(const uint64_t *__restrict__ pt, int K, int N, int Kw,
                                                          const uint8_t *info, uint8_t *cw) {
    extern __shared__ uint64_t words[];
    const int b = blockIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const uint8_t *u = info + (size_t)b * K;
    uint8_t *x = cw + (size_t)b * N;
    for (int w = wid; w < Kw; w += nw) {
        const int j = w * 64 + lane;
        const bool bit = j < K && (u[j] & 1);
        const uint64_t m = __ballot(bit);
        if (lane == 0) words[w] = m;
    }
    for (int j = threadIdx.x; j < K; j += blockDim.x) x[j] = u[j] & 1;
    __syncthreads();
    for (int j = threadIdx.x; j < N - K; j += blockDim.x) {
        const uint64_t *r = pt + (size_t)j * Kw;
        int pc = 0;
        for (int w = 0; w < Kw; ++w) pc += __popcll(r[w] & words[w]);
        x[K + j] = (uint8_t)(pc & 1);
    }
}

unsigned grid1(size_t nn, unsigned cap = 1024) { return (unsigned)std::max<size_t>(1, std::min<size_t>(cap, (nn + 255) / 256)); }

}  // namespace

}  // namespace sg

using namespace sg;

extern "C" {

int sg_rng_bits_device(uint64_t seed, uint64_t stream_id, int B, int nbits, uint8_t *d_bits, void *stream) {
    SG_CHECK_ARG(d_bits && nbits >= 0 && B >= 0, "bad argument");
    if (!B || !nbits) return SG_OK;
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    hipLaunchKernelGGL(rng_bits_kernel, dim3(grid1((nbits + 127) / 128), B), dim3(256), 0, s, seed, stream_id, nbits,
                       d_bits);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

int sg_bits_to_sections_strided_device(const uint8_t *d_bits, size_t bit_stride, int B, int L, int logM,
                                       int32_t *d_idx, size_t idx_stride, void *stream) {
    SG_CHECK_ARG(d_bits && d_idx && L >= 0 && logM >= 1 && logM <= 30, "bad argument");
    SG_CHECK_ARG(bit_stride >= (size_t)L * logM && idx_stride >= (size_t)L, "strides shorter than a row");
    if (!B || !L) return SG_OK;
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    hipLaunchKernelGGL(bits_to_sections_kernel, dim3(grid1(L), B), dim3(256), 0, s, d_bits, bit_stride, L, logM, d_idx,
                       idx_stride);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

int sg_bits_to_sections_device(const uint8_t *d_bits, int B, int L, int logM, int32_t *d_idx, void *stream) {
    return sg_bits_to_sections_strided_device(d_bits, (size_t)L * logM, B, L, logM, d_idx, (size_t)L, stream);
}

int sg_awgn_device(int precision, uint64_t seed, uint64_t stream_id, const void *d_x, int B, int n, double sigma,
                   void *d_y, void *stream) {
    SG_CHECK_ARG(d_x && d_y && n >= 0 && sigma >= 0, "bad argument");
    if (!B || !n) return SG_OK;
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    const dim3 grid(grid1((n + 1) / 2), B);
    if (precision == SG_F64)
        hipLaunchKernelGGL((awgn_kernel<double>), grid, dim3(256), 0, s, seed, stream_id, (const double *)d_x, n, sigma,
                           (double *)d_y);
    else
        hipLaunchKernelGGL((awgn_kernel<float>), grid, dim3(256), 0, s, seed, stream_id, (const float *)d_x, n, sigma,
                           (float *)d_y);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

int sg_bpsk_awgn_llr_device(int precision, uint64_t seed, uint64_t stream_id, const uint8_t *d_cw, int B, int N,
                            double sigma2, void *d_llr, void *stream) {
    SG_CHECK_ARG(d_cw && d_llr && N >= 0 && sigma2 > 0, "bad argument");
    if (!B || !N) return SG_OK;
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    const dim3 grid(grid1((N + 1) / 2), B);
    if (precision == SG_F64)
        hipLaunchKernelGGL((bpsk_llr_kernel<double>), grid, dim3(256), 0, s, seed, stream_id, d_cw, N, sigma2,
                           (double *)d_llr);
    else
        hipLaunchKernelGGL((bpsk_llr_kernel<float>), grid, dim3(256), 0, s, seed, stream_id, d_cw, N, sigma2,
                           (float *)d_llr);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

int sg_ldpc_encoder_create(const uint8_t *parity, int K, int N, sg_ldpc_encoder **out) {
    SG_CHECK_ARG(parity && out && K > 0 && N > K, "bad argument");
    SG_TRY(ensure_device());
    const int Kw = (K + 63) / 64, R = N - K;
    std::vector<uint64_t> pt((size_t)R * Kw, 0);
    for (int k = 0; k < K; ++k)
        for (int j = 0; j < R; ++j)
            if (parity[(size_t)k * R + j] & 1) pt[(size_t)j * Kw + k / 64] |= (uint64_t)1 << (k % 64);
    sg_ldpc_encoder *e = new sg_ldpc_encoder();
    e->K = K; e->N = N; e->Kw = Kw;
    if (hipMalloc(&e->pt, pt.size() * 8) != hipSuccess) {
        delete e;
        return fail(SG_ERR_NOMEM, "encoder table");
    }
    if (hipMemcpy(e->pt, pt.data(), pt.size() * 8, hipMemcpyHostToDevice) != hipSuccess) {
        hipFree(e->pt);
        delete e;
        return fail(SG_ERR_HIP, "encoder upload");
    }
    *out = e;
    return SG_OK;
}

int sg_ldpc_encoder_destroy(sg_ldpc_encoder *e) {
    if (!e) return SG_OK;
    if (e->pt) hipFree(e->pt);
    delete e;
    return SG_OK;
}

int sg_ldpc_encode_device(sg_ldpc_encoder *e, const uint8_t *d_info, int B, uint8_t *d_cw, void *stream) {
    SG_CHECK_ARG(e && d_info && d_cw, "bad argument");
    if (B <= 0) return SG_OK;
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    hipLaunchKernelGGL(ldpc_encode_kernel, dim3(B), dim3(256), (size_t)e->Kw * 8, s, e->pt, e->K, e->N, e->Kw, d_info,
                       d_cw);
    SG_HIP(hipGetLastError());
    return SG_OK;
}

}  // extern "C"
