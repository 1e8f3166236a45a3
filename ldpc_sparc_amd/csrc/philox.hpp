// Philox4x32-10 counter-based generator (Salmon et al., SC'11): the device
// random numbers of the throughput mode (random designs, random bits, AWGN).
// Counter = (element block, codeword, stream low, stream high), key = seed.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace sg {

__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0, h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
        c[0] = h1 ^ c[1] ^ k0;
        c[1] = l1;
        c[2] = h0 ^ c[3] ^ k1;
        c[3] = l0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// Two standard normals from one Philox output (Box-Muller on 53-bit uniforms).
__device__ __forceinline__ void philox_normal2(const uint32_t c[4], double *g0, double *g1) {
    const double u1 = ((double)(((uint64_t)c[0] << 21) ^ (c[1] >> 11)) + 1.0) * (1.0 / 9007199254740993.0);  // (0,1]
    const double u2 = (double)(((uint64_t)c[2] << 21) ^ (c[3] >> 11)) * (1.0 / 9007199254740992.0);           // [0,1)
    const double r = sqrt(-2.0 * log(u1));
    double sn, cs;
    sincospi(2.0 * u2, &sn, &cs);
    *g0 = r * cs;
    *g1 = r * sn;
}

}  // namespace sg
