// Vector FMA peak on the box: independent chains of v_fma_f64 (and, for
// comparison, v_pk_fma_f32) per lane, enough waves to fill every SIMD.  Prints
// TFLOP/s for each (2 flops per f64 FMA, 4 per packed f32 FMA).  Used for the
// f64 C2 line's peak (bench.py VALU_F64_PEAK_TFS; profiles/r04_fp64peak.txt).
//
// build: hipcc -O3 --offload-arch=gfx950 tools/fp64peak.hip -o tools/fp64peak
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int CHAINS = 8, ITERS = 4096;

__global__ __launch_bounds__(256) void fma64(double *out, double a, double b) {
    double x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-9 + c;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_fma(x[c], a, b);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    if (s == 12345.678) out[0] = s;  // keep the chains alive
}

typedef float f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void pkfma32(float *out, float a, float b) {
    f2 x[CHAINS];
    const f2 av = {a, a}, bv = {b, b};
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = f2{threadIdx.x * 1e-9f + c, (float)c};
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_elementwise_fma(x[c], av, bv);
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c].x + x[c].y;
    if (s == 12345.678f) out[0] = s;
}

int main() {
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    void *buf;
    hipMalloc(&buf, 64);
    const int blocks = ncu * 8;  // 8 workgroups of 4 waves per CU: 8 waves per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int kind = 0; kind < 2; ++kind) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(e0);
            if (kind == 0)
                hipLaunchKernelGGL(fma64, dim3(blocks), dim3(256), 0, 0, (double *)buf, 0.999999, 1e-7);
            else
                hipLaunchKernelGGL(pkfma32, dim3(blocks), dim3(256), 0, 0, (float *)buf, 0.999999f, 1e-7f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep && ms < best) best = ms;
        }
        const double flops = (double)blocks * 256 * CHAINS * ITERS * (kind == 0 ? 2.0 : 4.0);
        printf("%s: %.1f TFLOP/s (%d CUs, %.3f ms)\n", kind == 0 ? "v_fma_f64" : "v_pk_fma_f32",
               flops / (best * 1e-3) / 1e12, ncu, best);
    }
    return 0;
}
