// Microbenchmark of the 8192-point LDS FFT of the per-codeword AMP engine
// (amp_cw.hip): 256 workgroups of 1024 threads (one per CU: 160 KB of LDS
// requested), each running NF forward transforms back to back; prints the
// mean shader-clock cycles per transform.  Variants:
//   0  amp_cw.hip's stage schedule: radix 8,8,8,8,2, twiddles from the
//      hardware sine/cosine, one image, two barriers per stage
//   1  ping-pong between two images: one barrier per stage
// Build: hipcc -O3 --offload-arch=gfx950 -I../../ldpc_sparc_amd/csrc fftbench.hip -o fftbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "fft.hpp"

using namespace sg;

constexpr int T = 1024, LOG2P = 13, P = 1 << LOG2P, EPT = P / T;

__device__ __forceinline__ int opaque(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

typedef float f2v __attribute__((ext_vector_type(2)));
// complex product in two packed instructions (v_pk_mul_f32 + v_pk_fma_f32)
__device__ __forceinline__ cx<float> cmul_pk(cx<float> a, cx<float> b) {
    f2v A = {a.x, a.y}, Bv = {b.x, b.y}, t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(t) : "v"(A), "v"(Bv));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_lo:[0,0,1]" : "=v"(r) : "v"(A), "v"(Bv), "v"(t));
    return {r.x, r.y};
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
template <bool INV, int ST, bool PP, bool TW = true, bool DFT = true, bool PK = false>
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
                const float x = (float)((tw_exp(R, q) * k) & ((1 << (LNS + LR)) - 1)) * inv;
                wl[i * TWN + q] = {__builtin_amdgcn_cosf(x), -__builtin_amdgcn_sinf(x)};
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

int main() {
    const int nb = 256, nf = 256;
    run<0>(nb, nf);
    run<1>(nb, nf);
    run<2>(nb, nf);
    run<3>(nb, nf);
    run<4>(nb, nf);
    run<5>(nb, nf);
    grun<1024, 8, 0, false>("g1024x8 r8 2bar", nb, nf);
    grun<512, 16, 0, false>("g512x16 r8 2bar", nb, nf);
    grun<512, 16, 0, true>("g512x16 r8 pingpong", nb, nf);
    grun<512, 16, 1, false>("g512x16 r16 2bar", nb, nf);
    grun<512, 16, 1, true>("g512x16 r16 pingpong", nb, nf);
    grun<256, 32, 0, false>("g256x32 r8 2bar", nb, nf);
    grun<256, 32, 1, true>("g256x32 r16 pingpong", nb, nf);
    return 0;
}
