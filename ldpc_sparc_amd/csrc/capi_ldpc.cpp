// C ABI of the LDPC decoder: graph upload, batched decode, reference-compatible
// scalar shims (ldpc.py:463-503 ctypes targets).
#include <cstring>
#include <mutex>
#include <vector>

#include "bp.hpp"

struct sg_graph {
    int device = 0;
    int nv = 0, nc = 0, nmsg = 0, max_cdeg = 0, max_vdeg = 0, slots = 0;
    int32_t *d_voff = nullptr;
    int32_t *d_port_slot = nullptr;
    uint8_t *d_cdeg = nullptr;
    // grow-only staging for the host entry points
    void *d_ch = nullptr, *d_app = nullptr;
    int32_t *d_it = nullptr;
    size_t cap_bytes = 0;
    int cap_b = 0;
    std::vector<int64_t> h_vdeg, h_cdeg, h_intrlv;  // kept for the shim cache
};

namespace sg {

static int build_graph(const int64_t *vdeg, const int64_t *cdeg, const int64_t *intrlv, int nv, int nc,
                       int nmsg, sg_graph **out) {
    SG_CHECK_ARG(vdeg && cdeg && intrlv && out, "null graph array");
    SG_CHECK_ARG(nv > 0 && nc > 0 && nmsg > 0, "empty graph (Nv=%d Nc=%d Nmsg=%d)", nv, nc, nmsg);
    SG_TRY(ensure_device());
    std::vector<int32_t> voff(nv + 1), coff(nc + 1);
    int max_v = 0, max_c = 0;
    voff[0] = 0;
    for (int v = 0; v < nv; ++v) {
        SG_CHECK_ARG(vdeg[v] >= 0 && vdeg[v] < 256, "variable degree %lld out of range", (long long)vdeg[v]);
        voff[v + 1] = voff[v] + (int32_t)vdeg[v];
        if (vdeg[v] > max_v) max_v = (int)vdeg[v];
    }
    coff[0] = 0;
    for (int c = 0; c < nc; ++c) {
        SG_CHECK_ARG(cdeg[c] >= 2 && cdeg[c] < 256, "check degree %lld out of range (need 2..255)", (long long)cdeg[c]);
        coff[c + 1] = coff[c] + (int32_t)cdeg[c];
        if (cdeg[c] > max_c) max_c = (int)cdeg[c];
    }
    SG_CHECK_ARG(voff[nv] == nmsg && coff[nc] == nmsg,
                 "degree sums (%d, %d) do not match Nmsg=%d", voff[nv], coff[nc], nmsg);
    // message index -> (check, port) -> LDS slot k*nc + c
    std::vector<int32_t> msg_slot(nmsg);
    for (int c = 0; c < nc; ++c)
        for (int k = 0; k < coff[c + 1] - coff[c]; ++k) msg_slot[coff[c] + k] = k * nc + c;
    std::vector<int32_t> port_slot(nmsg);
    std::vector<uint8_t> seen(nmsg, 0);
    for (int p = 0; p < nmsg; ++p) {
        const int64_t m = intrlv[p];
        SG_CHECK_ARG(m >= 0 && m < nmsg && !seen[m], "intrlv is not a permutation of [0, Nmsg)");
        seen[m] = 1;
        port_slot[p] = msg_slot[m];
    }
    std::vector<uint8_t> cd(nc);
    for (int c = 0; c < nc; ++c) cd[c] = (uint8_t)cdeg[c];

    sg_graph *g = new sg_graph();
    hipGetDevice(&g->device);
    g->nv = nv; g->nc = nc; g->nmsg = nmsg; g->max_cdeg = max_c; g->max_vdeg = max_v;
    g->slots = max_c * nc;
    g->h_vdeg.assign(vdeg, vdeg + nv);
    g->h_cdeg.assign(cdeg, cdeg + nc);
    g->h_intrlv.assign(intrlv, intrlv + nmsg);
    hipStream_t s = lib_stream();
    bool ok = hipMalloc(&g->d_voff, sizeof(int32_t) * (nv + 1)) == hipSuccess &&
              hipMalloc(&g->d_port_slot, sizeof(int32_t) * nmsg) == hipSuccess &&
              hipMalloc(&g->d_cdeg, nc) == hipSuccess;
    ok = ok && hipMemcpyAsync(g->d_voff, voff.data(), sizeof(int32_t) * (nv + 1), hipMemcpyHostToDevice, s) == hipSuccess &&
         hipMemcpyAsync(g->d_port_slot, port_slot.data(), sizeof(int32_t) * nmsg, hipMemcpyHostToDevice, s) == hipSuccess &&
         hipMemcpyAsync(g->d_cdeg, cd.data(), nc, hipMemcpyHostToDevice, s) == hipSuccess &&
         hipStreamSynchronize(s) == hipSuccess;
    if (!ok) {
        sg_ldpc_graph_destroy(g);
        return fail(SG_ERR_NOMEM, "device allocation/upload of the Tanner graph failed");
    }
    *out = g;
    return SG_OK;
}

template <typename T>
static BpArgs<T> make_args(sg_graph *g, const void *ch, int B, int max_it, double corr, void *app, int32_t *it) {
    BpArgs<T> a;
    a.voff = g->d_voff;
    a.port_slot = g->d_port_slot;
    a.cdeg = g->d_cdeg;
    a.nv = g->nv; a.nc = g->nc; a.slots = g->slots; a.nports = g->nmsg;
    a.ch = (const T *)ch;
    a.app = (T *)app;
    a.it = it;
    a.B = B; a.max_it = max_it;
    a.factor = (T)corr;
    return a;
}

static int decode_device(sg_graph *g, int dectype, int precision, const void *d_ch, int B, int max_it,
                         double corr, void *d_app, int32_t *d_it, hipStream_t s) {
    SG_CHECK_ARG(g, "graph is NULL");
    SG_CHECK_ARG(B >= 0, "negative batch");
    SG_CHECK_ARG(dectype == SG_SUMPROD || dectype == SG_SUMPROD2 || dectype == SG_MINSUM,
                 "Decoder type unknonwn (dectype=%d)", dectype);
    SG_CHECK_ARG(precision == SG_F64 || precision == SG_F32, "precision must be SG_F64 or SG_F32");
    if (B == 0) return SG_OK;
    SG_CHECK_ARG(d_ch && d_app && d_it, "null device buffer");
    if (max_it <= 0) {  // reference: loop never runs, app untouched (zeros), returns max_it
        SG_HIP(hipMemsetAsync(d_app, 0, (size_t)B * g->nv * (precision == SG_F64 ? 8 : 4), s));
        std::vector<int32_t> v(B, max_it);
        SG_HIP(hipMemcpyAsync(d_it, v.data(), sizeof(int32_t) * B, hipMemcpyHostToDevice, s));
        SG_HIP(hipStreamSynchronize(s));
        return SG_OK;
    }
    if (precision == SG_F64)
        return bp_launch<double>(make_args<double>(g, d_ch, B, max_it, corr, d_app, d_it), dectype, g->max_cdeg, s);
    return bp_launch<float>(make_args<float>(g, d_ch, B, max_it, corr, d_app, d_it), dectype, g->max_cdeg, s);
}

static int ensure_staging(sg_graph *g, int B) {
    const size_t need = (size_t)B * g->nv * sizeof(double);
    if (need <= g->cap_bytes && B <= g->cap_b) return SG_OK;
    if (g->d_ch) hipFree(g->d_ch);
    if (g->d_app) hipFree(g->d_app);
    if (g->d_it) hipFree(g->d_it);
    g->d_ch = g->d_app = nullptr;
    g->d_it = nullptr;
    g->cap_bytes = 0;
    g->cap_b = 0;
    SG_HIP(hipMalloc(&g->d_ch, need));
    SG_HIP(hipMalloc(&g->d_app, need));
    SG_HIP(hipMalloc(&g->d_it, sizeof(int32_t) * B));
    g->cap_bytes = need;
    g->cap_b = B;
    return SG_OK;
}

static int decode_host(sg_graph *g, int dectype, int precision, const double *ch, int B, int max_it, double corr,
                       double *app, int32_t *it) {
    SG_CHECK_ARG(g, "graph is NULL");
    SG_CHECK_ARG(B >= 0, "negative batch");
    if (B == 0) return SG_OK;
    SG_CHECK_ARG(ch && app && it, "null host buffer");
    SG_TRY(ensure_device());
    SG_HIP(hipSetDevice(g->device));
    SG_TRY(ensure_staging(g, B));
    hipStream_t s = lib_stream();
    const size_t n = (size_t)B * g->nv;
    if (precision == SG_F64) {
        SG_HIP(hipMemcpyAsync(g->d_ch, ch, n * sizeof(double), hipMemcpyHostToDevice, s));
    } else {
        std::vector<float> tmp(n);
        for (size_t i = 0; i < n; ++i) tmp[i] = (float)ch[i];
        SG_HIP(hipMemcpyAsync(g->d_ch, tmp.data(), n * sizeof(float), hipMemcpyHostToDevice, s));
        SG_HIP(hipStreamSynchronize(s));
    }
    SG_TRY(decode_device(g, dectype, precision, g->d_ch, B, max_it, corr, g->d_app, g->d_it, s));
    SG_HIP(hipMemcpyAsync(it, g->d_it, sizeof(int32_t) * B, hipMemcpyDeviceToHost, s));
    if (precision == SG_F64) {
        SG_HIP(hipMemcpyAsync(app, g->d_app, n * sizeof(double), hipMemcpyDeviceToHost, s));
        SG_HIP(hipStreamSynchronize(s));
    } else {
        std::vector<float> tmp(n);
        SG_HIP(hipMemcpyAsync(tmp.data(), g->d_app, n * sizeof(float), hipMemcpyDeviceToHost, s));
        SG_HIP(hipStreamSynchronize(s));
        for (size_t i = 0; i < n; ++i) app[i] = tmp[i];
    }
    return SG_OK;
}

// Graph cache for the scalar shims: the reference calls decode once per block
// with the same (vdeg, cdeg, intrlv) arrays, so rebuilding every call would
// dominate.  Keyed by content.
static std::mutex g_shim_mu;
static sg_graph *g_shim_graph = nullptr;

static int shim_graph(const long *vdeg, const long *cdeg, const long *intrlv, int nv, int nc, int nmsg,
                      sg_graph **out) {
    SG_CHECK_ARG(vdeg && cdeg && intrlv, "null graph array");
    SG_CHECK_ARG(nv > 0 && nc > 0 && nmsg > 0, "empty graph");
    sg_graph *g = g_shim_graph;
    int dev = 0;
    hipGetDevice(&dev);
    if (g && g->nv == nv && g->nc == nc && g->nmsg == nmsg && g->device == dev &&
        std::memcmp(g->h_vdeg.data(), vdeg, sizeof(int64_t) * nv) == 0 &&
        std::memcmp(g->h_cdeg.data(), cdeg, sizeof(int64_t) * nc) == 0 &&
        std::memcmp(g->h_intrlv.data(), intrlv, sizeof(int64_t) * nmsg) == 0) {
        *out = g;
        return SG_OK;
    }
    static_assert(sizeof(long) == sizeof(int64_t), "LP64 expected");
    sg_graph *ng = nullptr;
    SG_TRY(build_graph((const int64_t *)vdeg, (const int64_t *)cdeg, (const int64_t *)intrlv, nv, nc, nmsg, &ng));
    if (g) sg_ldpc_graph_destroy(g);
    g_shim_graph = ng;
    *out = ng;
    return SG_OK;
}

static int shim_decode(int dectype, double *ch, long *vdeg, long *cdeg, long *intrlv, int nv, int nc, int nmsg,
                       double *app, double corr, int max_it) {
    std::lock_guard<std::mutex> lk(g_shim_mu);
    sg_graph *g = nullptr;
    int r = shim_graph(vdeg, cdeg, intrlv, nv, nc, nmsg, &g);
    if (r != SG_OK) return r;
    int32_t it = 0;
    r = decode_host(g, dectype, SG_F64, ch, 1, max_it, corr, app, &it);
    return r == SG_OK ? it : r;
}

}  // namespace sg

using namespace sg;

extern "C" {

int sg_ldpc_graph_create(const int64_t *vdeg, const int64_t *cdeg, const int64_t *intrlv, int nv, int nc,
                         int nmsg, sg_graph **out) {
    return build_graph(vdeg, cdeg, intrlv, nv, nc, nmsg, out);
}

int sg_ldpc_graph_destroy(sg_graph *g) {
    if (!g) return SG_OK;
    if (g->d_voff) hipFree(g->d_voff);
    if (g->d_port_slot) hipFree(g->d_port_slot);
    if (g->d_cdeg) hipFree(g->d_cdeg);
    if (g->d_ch) hipFree(g->d_ch);
    if (g->d_app) hipFree(g->d_app);
    if (g->d_it) hipFree(g->d_it);
    delete g;
    return SG_OK;
}

int sg_ldpc_graph_info(const sg_graph *g, int *nv, int *nc, int *nmsg, int *max_cdeg, int *max_vdeg) {
    SG_CHECK_ARG(g, "graph is NULL");
    if (nv) *nv = g->nv;
    if (nc) *nc = g->nc;
    if (nmsg) *nmsg = g->nmsg;
    if (max_cdeg) *max_cdeg = g->max_cdeg;
    if (max_vdeg) *max_vdeg = g->max_vdeg;
    return SG_OK;
}

int sg_ldpc_decode(sg_graph *g, int dectype, int precision, const double *ch, int B, int max_it, double corr,
                   double *app, int32_t *it) {
    return decode_host(g, dectype, precision, ch, B, max_it, corr, app, it);
}

int sg_ldpc_decode_device(sg_graph *g, int dectype, int precision, const void *d_ch, int B, int max_it,
                          double corr, void *d_app, int32_t *d_it, void *stream) {
    SG_TRY(ensure_device());
    return decode_device(g, dectype, precision, d_ch, B, max_it, corr, d_app, d_it, pick_stream(stream));
}

int sg_ldpc_count_errors_device(sg_graph *g, int precision, const void *d_app, const uint8_t *d_x,
                                const int32_t *d_it, int B, int k, int64_t *d_counts, void *stream) {
    SG_CHECK_ARG(g, "graph is NULL");
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    if (precision == SG_F64)
        return bp_count_launch<double>((const double *)d_app, d_x, d_it, B, g->nv, k, d_counts, s);
    return bp_count_launch<float>((const float *)d_app, d_x, d_it, B, g->nv, k, d_counts, s);
}

int sg_ldpc_codeword_errors_device(sg_graph *g, int precision, const void *d_app, const uint8_t *d_x, int B,
                                   int32_t *d_bit_errors, void *stream) {
    SG_CHECK_ARG(g && d_app && d_x && d_bit_errors, "null argument");
    SG_TRY(ensure_device());
    hipStream_t s = pick_stream(stream);
    if (precision == SG_F64)
        return bp_count_launch<double>((const double *)d_app, d_x, nullptr, B, g->nv, g->nv, nullptr, s, d_bit_errors);
    return bp_count_launch<float>((const float *)d_app, d_x, nullptr, B, g->nv, g->nv, nullptr, s, d_bit_errors);
}

int sumprod(double *ch, long *vdeg, long *cdeg, long *intrlv, int Nv, int Nc, int Nmsg, double *app,
            int max_itcount) {
    return shim_decode(SG_SUMPROD, ch, vdeg, cdeg, intrlv, Nv, Nc, Nmsg, app, 0.0, max_itcount);
}

int sumprod2(double *ch, long *vdeg, long *cdeg, long *intrlv, int Nv, int Nc, int Nmsg, double *app,
             int max_itcount) {
    return shim_decode(SG_SUMPROD2, ch, vdeg, cdeg, intrlv, Nv, Nc, Nmsg, app, 0.0, max_itcount);
}

int minsum(double *ch, long *vdeg, long *cdeg, long *intrlv, int Nv, int Nc, int Nmsg, double *app,
           double correction_factor, int max_itcount) {
    return shim_decode(SG_MINSUM, ch, vdeg, cdeg, intrlv, Nv, Nc, Nmsg, app, correction_factor, max_itcount);
}

double Lxfb(double *L, long dc, int corr_flag) {
    if (!L || dc < 2 || dc > 64 || ensure_device() != SG_OK) return NAN;
    hipStream_t s = lib_stream();
    double *d = nullptr;
    if (hipMalloc(&d, sizeof(double) * (dc + 1)) != hipSuccess) return NAN;
    double agg = NAN;
    bool ok = hipMemcpyAsync(d, L, sizeof(double) * dc, hipMemcpyHostToDevice, s) == hipSuccess &&
              lxfb_launch(d, (int)dc, corr_flag ? 1 : 0, d + dc, s) == SG_OK &&
              hipMemcpyAsync(L, d, sizeof(double) * dc, hipMemcpyDeviceToHost, s) == hipSuccess &&
              hipMemcpyAsync(&agg, d + dc, sizeof(double), hipMemcpyDeviceToHost, s) == hipSuccess &&
              hipStreamSynchronize(s) == hipSuccess;
    hipFree(d);
    return ok ? agg : NAN;
}

double Lxor(double L1, double L2, int corr_flag) {
    // Lxfb on two inputs returns their pairwise XOR-LLR as the aggregate.
    double L[2] = {L1, L2};
    return Lxfb(L, 2, corr_flag);
}

}  // extern "C"
