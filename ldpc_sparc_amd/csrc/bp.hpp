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

// Degree-grouped layout of a Tanner graph (bp.hip "grouped min-sum kernel"):
// variables and checks sorted by degree into groups of 64 (one wavefront
// lane each) of equal degree, so every wave loop is uniform.  Check group g
// of degree dc owns the dc x 64 message block at LDS byte address addr_g
// (slot = addr_g + 256 k + 4 lane); variable group g reads its ports' slot
// byte addresses from the global table at entry tab_g / 2 + 64 k + lane.
// Groups are assigned to the workgroup's 8 waves (at most 8 variable and 4
// check groups per wave).
constexpr int GRP_WAVES = BP_THREADS / 64;
constexpr int GRP_MAXDV = 16;  // variable degrees the unrolled variable groups take
constexpr int GRP_MAXDC = 8;   // check degrees the unrolled check groups take
constexpr int GRP_FLAG_BYTES = 2 * GRP_WAVES * 4;  // LDS stop flags after the messages (the whole image)
constexpr int GRP_PAIR = 1 << 8;  // degree-word flag: this variable group and the next one run as a pair
constexpr int GRP_PAIR_MAXD = 3;  // variable degrees whose groups pair up (the pair's slots and messages stay
                                  // within the <4, 2> kernel's 64 VGPRs)
struct BpGrpArgs {
    const int32_t *meta;      // [5][GRP_WAVES][VJ or CJ]: vdeg, vtab, cdeg, caddr, cvalid (see bp.hip)
    const int32_t *vmap;      // [GRP_WAVES][VJ][64] variable of each lane (-1: dummy)
    const uint16_t *vtab;     // [ntab] LDS slot byte addresses of the variable groups' ports (global)
    int ntab;                 // table entries
    int msg_bytes;            // message image incl. the trash slot (16-byte multiple)
    int vj, cj;               // groups per wave of the layout (<= the kernel's VJ, CJ)
    int nv;
    const float *ch;          // [B][nv]
    float *app;               // [B][nv]
    int32_t *it;              // [B]
    int B, max_it;
    float factor;
};
int bp_grouped_launch(const BpGrpArgs &a, hipStream_t s);
// groups per wave of the kernel instance that takes a layout of vj / cj groups
// per wave (the host lays meta / vmap out with these strides)
inline int grp_kvj(int vj, int cj) { return (vj <= 4 && cj <= 2) ? 4 : 8; }
inline int grp_kcj(int vj, int cj) { return (vj <= 4 && cj <= 2) ? 2 : 4; }
template <typename T>
int bp_count_launch(const T *app, const uint8_t *x, const int32_t *its, int B, int nv, int k,
                    int64_t *counts, hipStream_t s, int32_t *per_cw = nullptr);
int lxfb_launch(double *dL, int dc, int corr, double *dagg, hipStream_t s);

}  // namespace sg
