// Microbenchmark of the 8192-point LDS FFT of the per-codeword AMP engine
// (amp_cw.hip): 256 workgroups of 1024 threads (one per CU: 160 KB of LDS
// requested), each running NF forward transforms back to back; prints the
// mean shader-clock cycles per transform.  Variants:
//   0  amp_cw.hip's stage schedule: radix 8,8,8,8,2, twiddles from the
//      hardware sine/cosine, one image, two barriers per stage
//   1  ping-pong between two images: one barrier per stage
//   2  no twiddles; 3  no twiddles and no butterflies (LDS traffic and barriers)
//   4  two transforms through the same barriers; 5  packed complex products
//   6, 7  as 5 with 1 or 2 sine/cosine pairs per radix-8 butterfly (the other
//         powers of w as packed products) instead of 4
//   8  wfft.hpp: 16 x 512 four-step, one workgroup exchange, the 512-point
//      sub-transforms inside each wavefront (two workgroup barriers)
// and an accuracy check of variants 5-8 against a double-precision DFT
// Build: hipcc -O3 --offload-arch=gfx950 -I../../ldpc_sparc_amd/csrc -I. fftbench.hip -o fftbench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "fft.hpp"
#include "wfft.hpp"

using namespace sg;

constexpr int T = 1024, LOG2P = 13, P = 1 << LOG2P, EPT = P / T;

__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// complex product in two packed instructions (fft.hpp's cmul<float>)
__device__ __forceinline__ cx<float> cmul_pk(cx<float> a, cx<float> b) { return cmul(a, b); }
__device__ __forceinline__ cx<float> csq(cx<float> a) {
    return {a.x * a.x - a.y * a.y, 2.f * a.x * a.y};
}
template <bool INV>
__device__ __forceinline__ void tw_apply8_pk(const cx<float> *wl, cx<float> *v) {
    cx<float> a[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) a[t] = INV ? cconj(wl[t]) : wl[t];
#pragma unroll
    for (int b = 1; b < 4; ++b) v[b] = cmul_pk(v[b], a[b - 1]);
    v[4] = cmul_pk(v[4], a[3]);
#pragma unroll
    for (int b = 1; b < 4; ++b) v[4 + b] = cmul_pk(v[4 + b], cmul_pk(a[3], a[b - 1]));
}
template <bool INV>
__device__ __forceinline__ void tw_apply2_pk(const cx<float> *wl, cx<float> *v) {
    v[1] = cmul_pk(v[1], INV ? cconj(wl[0]) : wl[0]);
}

constexpr int radix(int st) { return st < 4 ? 8 : 2; }
constexpr int log2ns(int st) {
    int l = 0;
    for (int i = 0; i < st; ++i) l += radix(i) == 2 ? 1 : 3;
    return l;
}

// one Stockham stage from src to dst (src == dst: two barriers)
template <bool INV, int ST, bool PP, bool TW = true, bool DFT = true, bool PK = false, int NTR = 4>
__device__ __forceinline__ void stage(const cx<float> *src, cx<float> *dst, int tid) {
    constexpr int R = radix(ST), LNS = log2ns(ST), NB = EPT / R, TWN = tw_per_k(R);
    constexpr int LR = R == 2 ? 1 : 3;
    constexpr int NBF = P / R, NS = 1 << LNS;
    cx<float> wl[LNS > 0 ? NB * TWN : 1];
    if constexpr (LNS > 0 && TW) {
        constexpr float inv = 1.0f / (float)(1 << (LNS + LR));
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int k = (tid + i * T) & (NS - 1);
#pragma unroll
            for (int q = 0; q < TWN; ++q) {
                if (R == 8 && q >= NTR) continue;
                const float x = (float)((tw_exp(R, q) * k) & ((1 << (LNS + LR)) - 1)) * inv;
                wl[i * TWN + q] = {__builtin_amdgcn_cosf(x), -__builtin_amdgcn_sinf(x)};
            }
            if constexpr (R == 8 && NTR == 1) {  // w^2, w^3, w^4 as products of w
                wl[i * TWN + 1] = csq(wl[i * TWN]);
                wl[i * TWN + 2] = cmul_pk(wl[i * TWN], wl[i * TWN + 1]);
                wl[i * TWN + 3] = csq(wl[i * TWN + 1]);
            } else if constexpr (R == 8 && NTR == 2) {  // w^3 = w w^2, w^4 = w^2 w^2
                wl[i * TWN + 2] = cmul_pk(wl[i * TWN], wl[i * TWN + 1]);
                wl[i * TWN + 3] = csq(wl[i * TWN + 1]);
            }
        }
    }
    cx<float> v[EPT];
    int base_out[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int j = tid + i * T;
        const int k = j & (NS - 1);
        const int jp = fsw(j);
#pragma unroll
        for (int r = 0; r < R; ++r) v[i * R + r] = src[(NBF % 256 == 0) ? jp + r * NBF : fsw(j + r * NBF)];
        if constexpr (LNS > 0 && TW) {
            if constexpr (PK && R == 8) tw_apply8_pk<INV>(wl + i * TWN, &v[i * R]);
            else if constexpr (PK && R == 2) tw_apply2_pk<INV>(wl + i * TWN, &v[i * R]);
            else tw_apply<float, INV, R>(wl + i * TWN, &v[i * R]);
        }
        if constexpr (DFT) dftR<float, INV, R>(&v[i * R]);
        base_out[i] = ((j - k) << LR) + k;
    }
    if (!PP) __syncthreads();
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int bp = fsw(base_out[i]);
#pragma unroll
        for (int r = 0; r < R; ++r) dst[(NS % 256 == 0) ? bp + r * NS : fsw(base_out[i] + r * NS)] = v[i * R + r];
    }
    __syncthreads();
}

// two independent transforms (images A and B) through the same barriers
template <bool INV, int ST>
__device__ __forceinline__ void stage2(cx<float> *A, cx<float> *Bm, int tid) {
    constexpr int R = radix(ST), LNS = log2ns(ST), NB = EPT / R, TWN = tw_per_k(R);
    constexpr int LR = R == 2 ? 1 : 3;
    constexpr int NBF = P / R, NS = 1 << LNS;
    cx<float> wl[LNS > 0 ? NB * TWN : 1];
    if constexpr (LNS > 0) {
        constexpr float inv = 1.0f / (float)(1 << (LNS + LR));
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int k = (tid + i * T) & (NS - 1);
#pragma unroll
            for (int q = 0; q < TWN; ++q) {
                const float x = (float)((tw_exp(R, q) * k) & ((1 << (LNS + LR)) - 1)) * inv;
                wl[i * TWN + q] = {__builtin_amdgcn_cosf(x), -__builtin_amdgcn_sinf(x)};
            }
        }
    }
    cx<float> v[EPT], u[EPT];
    int base_out[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int j = tid + i * T;
        const int k = j & (NS - 1);
        const int jp = fsw(j);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int ix = (NBF % 256 == 0) ? jp + r * NBF : fsw(j + r * NBF);
            v[i * R + r] = A[ix];
            u[i * R + r] = Bm[ix];
        }
        if constexpr (LNS > 0) {
            tw_apply<float, INV, R>(wl + i * TWN, &v[i * R]);
            tw_apply<float, INV, R>(wl + i * TWN, &u[i * R]);
        }
        dftR<float, INV, R>(&v[i * R]);
        dftR<float, INV, R>(&u[i * R]);
        base_out[i] = ((j - k) << LR) + k;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int bp = fsw(base_out[i]);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int ox = (NS % 256 == 0) ? bp + r * NS : fsw(base_out[i] + r * NS);
            A[ox] = v[i * R + r];
            Bm[ox] = u[i * R + r];
        }
    }
    __syncthreads();
}

// generic stage: NT threads, E values per thread, radix plan RP (0: 8,8,8,8,2; 1: 16,16,16,2)
template <int RP>
constexpr int gradix(int st) { return RP == 0 ? (st < 4 ? 8 : 2) : (st < 3 ? 16 : 2); }
template <int RP>
constexpr int gnst() { return RP == 0 ? 5 : 4; }
template <int RP>
constexpr int glog2ns(int st) {
    int l = 0;
    for (int i = 0; i < st; ++i) l += gradix<RP>(i) == 2 ? 1 : gradix<RP>(i) == 8 ? 3 : 4;
    return l;
}
template <bool INV, int ST, int NT, int E, int RP, bool PP>
__device__ __forceinline__ void gstage(const cx<float> *src, cx<float> *dst, int tid) {
    constexpr int R = gradix<RP>(ST), LNS = glog2ns<RP>(ST), NB = E / R, TWN = tw_per_k(R);
    constexpr int LR = R == 2 ? 1 : R == 8 ? 3 : 4;
    constexpr int NBF = P / R, NS = 1 << LNS;
    cx<float> wl[LNS > 0 ? NB * TWN : 1];
    if constexpr (LNS > 0) {
        constexpr float inv = 1.0f / (float)(1 << (LNS + LR));
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            const int k = (tid + i * NT) & (NS - 1);
#pragma unroll
            for (int q = 0; q < TWN; ++q) {
                const float x = (float)((tw_exp(R, q) * k) & ((1 << (LNS + LR)) - 1)) * inv;
                wl[i * TWN + q] = {__builtin_amdgcn_cosf(x), -__builtin_amdgcn_sinf(x)};
            }
        }
    }
    cx<float> v[E];
    int base_out[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int j = tid + i * NT;
        const int k = j & (NS - 1);
        const int jp = fsw(j);
#pragma unroll
        for (int r = 0; r < R; ++r) v[i * R + r] = src[(NBF % 256 == 0) ? jp + r * NBF : fsw(j + r * NBF)];
        if constexpr (LNS > 0) tw_apply<float, INV, R>(wl + i * TWN, &v[i * R]);
        dftR<float, INV, R>(&v[i * R]);
        base_out[i] = ((j - k) << LR) + k;
    }
    if (!PP) __syncthreads();
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const int bp = fsw(base_out[i]);
#pragma unroll
        for (int r = 0; r < R; ++r) dst[(NS % 256 == 0) ? bp + r * NS : fsw(base_out[i] + r * NS)] = v[i * R + r];
    }
    __syncthreads();
}
template <int NT, int E, int RP, bool PP, int ST = 0>
__device__ __forceinline__ void gfft(cx<float> *A, cx<float> *Bb, int tid) {
    if constexpr (ST < gnst<RP>()) {
        if constexpr (PP) {
            if constexpr (ST % 2 == 0) gstage<false, ST, NT, E, RP, true>(A, Bb, tid);
            else gstage<false, ST, NT, E, RP, true>(Bb, A, tid);
        } else {
            gstage<false, ST, NT, E, RP, false>(A, A, tid);
        }
        gfft<NT, E, RP, PP, ST + 1>(A, Bb, tid);
    }
}

template <int NT, int E, int RP, bool PP>
__global__ __launch_bounds__(NT) void gbench(float *out, long long *cyc, int nf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cx<float> *A = reinterpret_cast<cx<float> *>(smem), *Bf = A + P;
    const int tid = threadIdx.x;
    for (int i = tid; i < 2 * P; i += NT) A[i] = {(float)(i & 7), (float)(blockIdx.x & 3)};
    __syncthreads();
    const long long t0 = clock64();
    for (int f = 0; f < nf; ++f) gfft<NT, E, RP, PP>(A, Bf, opaque(tid));
    const long long t1 = clock64();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * NT + tid] = A[tid].x + Bf[tid].y;
}

template <int NT, int E, int RP, bool PP>
static void grun(const char *name, int nb, int nf) {
    float *out;
    long long *cyc;
    hipMalloc(&out, sizeof(float) * nb * NT);
    hipMalloc(&cyc, sizeof(long long) * nb);
    hipFuncSetAttribute((const void *)gbench<NT, E, RP, PP>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL((gbench<NT, E, RP, PP>), dim3(nb), dim3(NT), 160 * 1024, 0, out, cyc, nf);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((gbench<NT, E, RP, PP>), dim3(nb), dim3(NT), 160 * 1024, 0, out, cyc, nf);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(nb);
    hipMemcpy(h.data(), cyc, sizeof(long long) * nb, hipMemcpyDeviceToHost);
    double sm = 0;
    for (auto v : h) sm += v;
    printf("%s: %.0f cycles per FFT, %.2f us per FFT\n", name, sm / nb / nf, ms * 1e3 / nf);
    hipFree(out);
    hipFree(cyc);
}

template <int VAR>
__global__ __launch_bounds__(T) void bench(float *out, long long *cyc, int nf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cx<float> *A = reinterpret_cast<cx<float> *>(smem), *Bf = A + P;
    const int tid = threadIdx.x;
    for (int i = tid; i < P; i += T) A[i] = {(float)(i & 7), (float)(blockIdx.x & 3)};
    __syncthreads();
    const long long t0 = clock64();
    for (int f = 0; f < nf; ++f) {
        const int tl = opaque(tid);
        if constexpr (VAR == 0) {
            stage<false, 0, false>(A, A, tl);
            stage<false, 1, false>(A, A, tl);
            stage<false, 2, false>(A, A, tl);
            stage<false, 3, false>(A, A, tl);
            stage<false, 4, false>(A, A, tl);
        } else if constexpr (VAR == 2) {  // no twiddles
            stage<false, 0, false, false>(A, A, tl);
            stage<false, 1, false, false>(A, A, tl);
            stage<false, 2, false, false>(A, A, tl);
            stage<false, 3, false, false>(A, A, tl);
            stage<false, 4, false, false>(A, A, tl);
        } else if constexpr (VAR == 3) {  // no twiddles, no butterflies: LDS traffic and barriers only
            stage<false, 0, false, false, false>(A, A, tl);
            stage<false, 1, false, false, false>(A, A, tl);
            stage<false, 2, false, false, false>(A, A, tl);
            stage<false, 3, false, false, false>(A, A, tl);
            stage<false, 4, false, false, false>(A, A, tl);
        } else if constexpr (VAR == 5) {  // packed complex products (inline asm)
            stage<false, 0, false, true, true, true>(A, A, tl);
            stage<false, 1, false, true, true, true>(A, A, tl);
            stage<false, 2, false, true, true, true>(A, A, tl);
            stage<false, 3, false, true, true, true>(A, A, tl);
            stage<false, 4, false, true, true, true>(A, A, tl);
        } else if constexpr (VAR == 6 || VAR == 7) {  // packed, 1 (6) or 2 (7) sine/cosine pairs per radix-8 butterfly
            constexpr int NT = VAR == 6 ? 1 : 2;
            stage<false, 0, false, true, true, true, NT>(A, A, tl);
            stage<false, 1, false, true, true, true, NT>(A, A, tl);
            stage<false, 2, false, true, true, true, NT>(A, A, tl);
            stage<false, 3, false, true, true, true, NT>(A, A, tl);
            stage<false, 4, false, true, true, true, NT>(A, A, tl);
        } else if constexpr (VAR == 8) {  // wfft.hpp: 16 x 512 with one workgroup exchange
            wfft8192<false>(A, tl);
        } else if constexpr (VAR == 4) {  // two transforms per pass (counted as two)
            if (f & 1) continue;
            stage2<false, 0>(A, Bf, tl);
            stage2<false, 1>(A, Bf, tl);
            stage2<false, 2>(A, Bf, tl);
            stage2<false, 3>(A, Bf, tl);
            stage2<false, 4>(A, Bf, tl);
        } else {
            stage<false, 0, true>(A, Bf, tl);
            stage<false, 1, true>(Bf, A, tl);
            stage<false, 2, true>(A, Bf, tl);
            stage<false, 3, true>(Bf, A, tl);
            stage<false, 4, true>(A, Bf, tl);
            // (the result in Bf; the next transform reads A, which is fine for timing)
        }
    }
    const long long t1 = clock64();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * T + tid] = A[tid].x + Bf[tid].y;
}

template <int VAR>
static double run(int nb, int nf) {
    float *out;
    long long *cyc;
    hipMalloc(&out, sizeof(float) * nb * T);
    hipMalloc(&cyc, sizeof(long long) * nb);
    hipFuncSetAttribute((const void *)bench<VAR>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(bench<VAR>, dim3(nb), dim3(T), 160 * 1024, 0, out, cyc, nf);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(bench<VAR>, dim3(nb), dim3(T), 160 * 1024, 0, out, cyc, nf);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(nb);
    hipMemcpy(h.data(), cyc, sizeof(long long) * nb, hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : h) s += v;
    printf("variant %d: %.0f cycles per FFT (clock64), %.2f us per FFT (wall / transforms per CU)\n", VAR,
           s / nb / nf, ms * 1e3 / nf);
    hipFree(out);
    hipFree(cyc);
    return s / nb / nf;
}

// one forward transform of a fixed input per NTR setting, written out (accuracy check of variants 5-7)
template <int NT>
__global__ __launch_bounds__(T) void check_fft(float2 *out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cx<float> *A = reinterpret_cast<cx<float> *>(smem);
    const int tid = threadIdx.x;
    for (int i = tid; i < P; i += T) A[fsw(i)] = {(float)((i * 37) % 101) / 101.f - 0.5f, (float)((i * i) % 97) / 97.f - 0.5f};
    __syncthreads();
    stage<false, 0, false, true, true, true, NT>(A, A, tid);
    stage<false, 1, false, true, true, true, NT>(A, A, tid);
    stage<false, 2, false, true, true, true, NT>(A, A, tid);
    stage<false, 3, false, true, true, true, NT>(A, A, tid);
    stage<false, 4, false, true, true, true, NT>(A, A, tid);
    for (int i = tid; i < P; i += T) out[i] = make_float2(A[fsw(i)].x, A[fsw(i)].y);
}
template <int NT>
static std::vector<float2> check(void) {
    float2 *o;
    hipMalloc(&o, sizeof(float2) * P);
    hipFuncSetAttribute((const void *)check_fft<NT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(check_fft<NT>, dim3(1), dim3(T), 160 * 1024, 0, o);
    std::vector<float2> h(P);
    hipMemcpy(h.data(), o, sizeof(float2) * P, hipMemcpyDeviceToHost);
    hipFree(o);
    return h;
}

// occupancy study: NT threads run nf transforms of 2^LOG2N points (EPT 8,
// sine/cosine stage twiddles, fft.hpp lds_fft1_sincos); LDS requested per
// workgroup sets how many workgroups share a CU
template <int LOG2N, int NT>
__global__ __launch_bounds__(NT) void occ_bench(float *out, long long *cyc, int nf) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cx<float> *A = reinterpret_cast<cx<float> *>(smem);
    const int tid = threadIdx.x;
    for (int i = tid; i < (1 << LOG2N); i += NT) A[i] = {(float)(i & 7), (float)(blockIdx.x & 3)};
    __syncthreads();
    const long long t0 = clock64();
    for (int f = 0; f < nf; ++f) lds_fft1_sincos<false, 8, LOG2N, 0, fft1_nstages_ct(LOG2N, 8)>(A, opaque(tid));
    const long long t1 = clock64();
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * NT + tid] = A[tid].x;
}
template <int LOG2N, int NT>
static void occ_run(const char *name, int nb, int nf, int lds) {
    float *out;
    long long *cyc;
    hipMalloc(&out, sizeof(float) * nb * NT);
    hipMalloc(&cyc, sizeof(long long) * nb);
    hipFuncSetAttribute((const void *)occ_bench<LOG2N, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL((occ_bench<LOG2N, NT>), dim3(nb), dim3(NT), lds, 0, out, cyc, nf);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((occ_bench<LOG2N, NT>), dim3(nb), dim3(NT), lds, 0, out, cyc, nf);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%s: %.1f us wall for %d workgroups x %d transforms of 2^%d\n", name, ms * 1e3, nb, nf, LOG2N);
    hipFree(out);
    hipFree(cyc);
}

template <bool INV>
__global__ __launch_bounds__(T) void check_wfft(float2 *out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    cx<float> *A = reinterpret_cast<cx<float> *>(smem);
    const int tid = threadIdx.x;
    for (int i = tid; i < P; i += T) A[i] = {(float)((i * 37) % 101) / 101.f - 0.5f, (float)((i * i) % 97) / 97.f - 0.5f};
    __syncthreads();
    wfft8192<INV>(A, tid);
    for (int k = tid; k < P; k += T) out[k] = make_float2(A[wf_pos_out(k)].x, A[wf_pos_out(k)].y);
}
template <bool INV>
static std::vector<float2> checkw(void) {
    float2 *o;
    hipMalloc(&o, sizeof(float2) * P);
    hipFuncSetAttribute((const void *)check_wfft<INV>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(check_wfft<INV>, dim3(1), dim3(T), 160 * 1024, 0, o);
    std::vector<float2> h(P);
    hipMemcpy(h.data(), o, sizeof(float2) * P, hipMemcpyDeviceToHost);
    hipFree(o);
    return h;
}

int main() {
    const int nb = 256, nf = 256;
    {
        std::vector<double> xr(P), xi(P);
        for (int i = 0; i < P; ++i) {
            xr[i] = (float)((i * 37) % 101) / 101.f - 0.5f;
            xi[i] = (float)(((long long)i * i) % 97) / 97.f - 0.5f;
        }
        auto f = checkw<false>(), g = checkw<true>();
        double ef = 0, eg = 0, nrm = 0;
        for (int k = 0; k < P; k += 13) {
            double sr = 0, si = 0, tr = 0, ti = 0;
            for (int m = 0; m < P; ++m) {
                const double ang = -2 * M_PI * (double)((long long)m * k % P) / P;
                sr += xr[m] * cos(ang) - xi[m] * sin(ang);
                si += xr[m] * sin(ang) + xi[m] * cos(ang);
                tr += xr[m] * cos(ang) + xi[m] * sin(ang);
                ti += -xr[m] * sin(ang) + xi[m] * cos(ang);
            }
            nrm = fmax(nrm, hypot(sr, si));
            ef = fmax(ef, hypot(f[k].x - sr, f[k].y - si));
            eg = fmax(eg, hypot(g[k].x - tr, g[k].y - ti));
        }
        printf("wfft accuracy (max abs error / max |X|): forward %.3g, inverse %.3g\n", ef / nrm, eg / nrm);
    }
    {
        // reference: direct DFT in double of the same input
        std::vector<double> xr(P), xi(P);
        for (int i = 0; i < P; ++i) {
            xr[i] = (float)((i * 37) % 101) / 101.f - 0.5f;
            xi[i] = (float)(((long long)i * i) % 97) / 97.f - 0.5f;
        }
        auto a4 = check<4>(), a2 = check<2>(), a1 = check<1>();
        double e4 = 0, e2 = 0, e1 = 0, nrm = 0;
        for (int k = 0; k < P; k += 61) {
            double sr = 0, si = 0;
            for (int m = 0; m < P; ++m) {
                const double ang = -2 * M_PI * (double)((long long)m * k % P) / P;
                sr += xr[m] * cos(ang) - xi[m] * sin(ang);
                si += xr[m] * sin(ang) + xi[m] * cos(ang);
            }
            nrm = fmax(nrm, hypot(sr, si));
            e4 = fmax(e4, hypot(a4[k].x - sr, a4[k].y - si));
            e2 = fmax(e2, hypot(a2[k].x - sr, a2[k].y - si));
            e1 = fmax(e1, hypot(a1[k].x - sr, a1[k].y - si));
        }
        printf("accuracy (max abs error / max |X|): 4 sincos %.3g, 2 sincos %.3g, 1 sincos %.3g\n", e4 / nrm, e2 / nrm,
               e1 / nrm);
    }
    run<0>(nb, nf);
    run<1>(nb, nf);
    run<2>(nb, nf);
    run<3>(nb, nf);
    run<4>(nb, nf);
    run<5>(nb, nf);
    run<6>(nb, nf);
    run<7>(nb, nf);
    run<8>(nb, nf);
    // one codeword-iteration's forward transforms per CU: 64 x 2^13 in one
    // workgroup against 128 x 2^12 in two workgroups sharing the CU
    occ_run<13, 1024>("occupancy: 1 workgroup/CU, 1024 threads, 64 x 8192", 256, 64, 160 * 1024);
    occ_run<12, 512>("occupancy: 2 workgroups/CU, 512 threads, 64 x 4096 each", 512, 64, 80 * 1024);
    occ_run<12, 512>("occupancy: 1 workgroup/CU, 512 threads, 128 x 4096", 256, 128, 160 * 1024);
    grun<1024, 8, 0, false>("g1024x8 r8 2bar", nb, nf);
    grun<512, 16, 0, false>("g512x16 r8 2bar", nb, nf);
    grun<512, 16, 0, true>("g512x16 r8 pingpong", nb, nf);
    grun<512, 16, 1, false>("g512x16 r16 2bar", nb, nf);
    grun<512, 16, 1, true>("g512x16 r16 pingpong", nb, nf);
    grun<256, 32, 0, false>("g256x32 r8 2bar", nb, nf);
    grun<256, 32, 1, true>("g256x32 r16 pingpong", nb, nf);
    return 0;
}
