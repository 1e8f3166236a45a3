// 8192-point complex FFT in LDS for one 1024-thread workgroup with two
// workgroup barriers (device code, gfx950).
//
// The Stockham schedule of fft.hpp moves every value through LDS once per
// radix-8 stage with two barriers per stage (five stages, ten barriers for
// 8192 points).  Here the transform is split four-step as 16 x 512 so that
// only the first split crosses wavefronts:
//   n = 512 a + b, k = kA + 16 kB
//   X[kA + 16 kB] = sum_b w_512^(b kB) w_8192^(b kA) sum_a x[512 a + b] w_16^(a kA)
//   pass A   thread (w, lane l) holds a = 8 (l >> 5) + j, j < 8 (registers),
//            b = 32 w + (l & 31): a 16-point DFT over a as a radix-2 step
//            across the wave halves (v_permlane32_swap, no LDS) and a
//            radix-8 DFT in registers, then the twiddle w_8192^(b kA)
//   exchange the only workgroup-wide one: wavefront kA receives the 512
//            values of its sub-transform (barrier, write, barrier, read)
//   pass B/C/D  the 512-point DFT inside the wavefront as 8 x 8 x 8 with
//            two wavefront-local LDS transposes in its own 4 KB region
//            (no workgroup barrier)
// Every LDS access pattern is conflict-free for ds_read_b64 (2 x 32 lanes,
// 64 banks) and ds_write_b64 (4 x 16 lanes, 32 banks): see the XOR swizzles
// of the wavefront-local transposes.
//
// Layouts: input element n at d[n] (natural order); output element k at
// d[wf_pos_out(k)] (wavefront kA's region, swizzled by kA).  The callers' position tables use these two maps.
// INV = true computes the unnormalised inverse DFT (conjugate twiddles).
#pragma once
#include "fft.hpp"

namespace sg {

constexpr int WF_N = 8192, WF_THREADS = 1024;

// (kA = k mod 16 is the wavefront of the last passes; XOR-ing it into the low
// bits keeps consecutive k on distinct banks for the callers' gathers)
__host__ __device__ __forceinline__ int wf_pos_out(int k) {
    return ((k & 15) << 9) | ((((k >> 10) << 6) | (((k >> 4) & 7) << 3) | ((k >> 7) & 7)) ^ (k & 15));
}

namespace wfd {

// exp(-2 pi i m / n) (forward) or its conjugate, m taken mod n; the argument
// of the hardware sine / cosine is in revolutions and (m mod n) / n is exact
template <bool INV, int LOG2N>
__device__ __forceinline__ cx<float> cis(int m) {
    const float x = (float)(m & ((1 << LOG2N) - 1)) * (1.0f / (float)(1 << LOG2N));
    const float c = __builtin_amdgcn_cosf(x), s = __builtin_amdgcn_sinf(x);
    return INV ? cx<float>{c, s} : cx<float>{c, -s};
}

// lanes 32..63 of a <-> lanes 0..31 of b
__device__ __forceinline__ void swap32(cx<float> &a, cx<float> &b) {
    const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
    const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
    a = {__uint_as_float(rx[0]), __uint_as_float(ry[0])};
    b = {__uint_as_float(rx[1]), __uint_as_float(ry[1])};
}

// LDS writes of this wavefront complete before its later reads (the lanes
// exchange values), and no compiler motion of memory accesses across.  Only
// lgkmcnt is waited for: a memory fence would also wait for the caller's
// global loads in flight (vmcnt(0)).
__device__ __forceinline__ void wave_sync() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0), vmcnt / expcnt unconstrained (gfx9 encoding)
    __builtin_amdgcn_wave_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// v[q] *= w_(2^LOG2N)^(m q), q = 1..7: four sine / cosine pairs, the rest as products
template <bool INV, int LOG2N>
__device__ __forceinline__ void twiddle8(cx<float> *v, int m) {
    cx<float> t[5];
#pragma unroll
    for (int q = 1; q <= 4; ++q) t[q] = cis<INV, LOG2N>(m * q);
#pragma unroll
    for (int q = 1; q <= 3; ++q) v[4 + q] = cmul(v[4 + q], cmul(t[4], t[q]));
#pragma unroll
    for (int q = 1; q <= 4; ++q) v[q] = cmul(v[q], t[q]);
}

}  // namespace wfd

template <bool INV>
__device__ __forceinline__ void wfft8192(cx<float> *d, int tid) {
    const int w = tid >> 6, l = tid & 63, H = l >> 5;
    const int b = (w << 5) | (l & 31);
    cx<float> v[8];
    // ---- pass A: 16-point DFTs over a = 8 H + j
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = d[(H << 12) | (j << 9) | b];
    // lane half H now takes u = x[J], x[8 + J] for J = jj + 4 H
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) wfd::swap32(v[jj], v[jj + 4]);
    {
        constexpr float c1 = 0.92387953251128675613f, s1 = 0.38268343236508977173f, r2 = 0.70710678118654752440f;
        const cx<float> w16[4] = {{1.f, 0.f}, {c1, INV ? s1 : -s1}, {r2, INV ? r2 : -r2}, {s1, INV ? c1 : -c1}};
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const cx<float> u = v[jj], x8 = v[jj + 4];
            v[jj] = cadd(u, x8);                                        // y_0[J]
            cx<float> t = jj == 0 ? csub(u, x8) : cmul(csub(u, x8), w16[jj]);  // (u - x8) w16^jj
            const cx<float> tm = mul_mi<float, INV>(t);                 // * w16^4
            v[jj + 4] = H ? tm : t;                                     // y_1[J] = (u - x8) w16^J
        }
    }
    // lane half p takes y_p[0..7]
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) wfd::swap32(v[jj], v[jj + 4]);
    dft8<float, INV>(v);  // v[q] = X_A[kA = 2 q + H][b]
    {
        // v[q] *= w_8192^(b (2 q + H))
        const cx<float> z0 = wfd::cis<INV, 13>(b * H), s1 = wfd::cis<INV, 13>(2 * b), s2 = wfd::cis<INV, 13>(4 * b),
                        s4 = wfd::cis<INV, 13>(8 * b);
        const cx<float> z1 = cmul(z0, s1), z2 = cmul(z0, s2), z3 = cmul(z1, s2);
        v[7] = cmul(v[7], cmul(z3, s4));
        v[6] = cmul(v[6], cmul(z2, s4));
        v[5] = cmul(v[5], cmul(z1, s4));
        v[4] = cmul(v[4], cmul(z0, s4));
        v[3] = cmul(v[3], z3);
        v[2] = cmul(v[2], z2);
        v[1] = cmul(v[1], z1);
        v[0] = cmul(v[0], z0);
    }
    // ---- exchange: wavefront kA receives sub-transform kA
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) d[(((q << 1) | H) << 9) | b] = v[q];
    __syncthreads();
    const int R = w << 9;
    // ---- pass B: 512 = 8 (registers, b = 64 r + l) x 64 (lanes)
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] = d[R | (r << 6) | l];
    dft8<float, INV>(v);  // v[q]: kB1 = q
    wfd::twiddle8<INV, 9>(v, l);  // w_512^(l kB1)
    // transpose: lane (kB1 = l >> 3, llo = l & 7) takes l' = 8 hi + llo, hi < 8
#pragma unroll
    for (int q = 0; q < 8; ++q) d[R | (q << 6) | (l ^ (q << 3))] = v[q];
    wfd::wave_sync();
    const int kB1 = l >> 3, llo = l & 7;
#pragma unroll
    for (int hi = 0; hi < 8; ++hi) v[hi] = d[R | (kB1 << 6) | ((hi ^ kB1) << 3) | llo];
    // ---- pass C: over hi
    dft8<float, INV>(v);  // v[c]: kC = c
    wfd::twiddle8<INV, 6>(v, llo);  // w_64^(llo kC)
    // transpose: lane (kB1 = l >> 3, kC = l & 7) takes llo = r, r < 8
#pragma unroll
    for (int c = 0; c < 8; ++c) d[R | (kB1 << 6) | ((c ^ (kB1 & 1)) << 3) | (llo ^ ((kB1 & 3) | (c & 4)))] = v[c];
    wfd::wave_sync();
    {
        const int kC = l & 7, tau = (kB1 & 3) | (kC & 4);
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = d[R | (kB1 << 6) | ((kC ^ (kB1 & 1)) << 3) | (r ^ tau)];
    }
    // ---- pass D: over llo
    dft8<float, INV>(v);  // v[dd]: kD = dd
    wfd::wave_sync();
#pragma unroll
    for (int dd = 0; dd < 8; ++dd) d[R | (((dd << 6) | l) ^ w)] = v[dd];
    __syncthreads();
}

}  // namespace sg
