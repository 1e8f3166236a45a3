// Kernel-side declarations of the batched BP decoder (bp.hip).
#pragma once
#include "common.hpp"

namespace sg {

constexpr int BP_THREADS = 512;
constexpr int BP_VJ = 8;                // variables per thread held in registers (nv <= BP_VJ * BP_THREADS)
constexpr int BP_MAX_LDS = 160 * 1024;  // one workgroup's LDS limit on gfx950

template <typename T>
struct BpArgs {
    const int32_t *voff;       // [nv+1] variable-port offsets
    const int32_t *port_slot;  // [nmsg] variable port -> LDS message slot (k*nc + c)
    const uint8_t *cdeg;       // [nc]
    int nv, nc, slots;         // slots = max_cdeg * nc
    int nports;                // variable ports = edges (voff[nv])
    const T *ch;               // [B][nv]
    T *app;                    // [B][nv]
    int32_t *it;               // [B]
    int B, max_it;
    T factor;
};

template <typename T>
int bp_launch(const BpArgs<T> &a, int dectype, int max_cdeg, hipStream_t s);
template <typename T>
int bp_count_launch(const T *app, const uint8_t *x, const int32_t *its, int B, int nv, int k,
                    int64_t *counts, hipStream_t s, int32_t *per_cw = nullptr);
int lxfb_launch(double *dL, int dc, int corr, double *dagg, hipStream_t s);

}  // namespace sg
