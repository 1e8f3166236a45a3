// C ABI of the LDPC decoder: graph upload, batched decode, reference-compatible
// scalar shims (ldpc.py:463-503 ctypes targets).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
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
    // degree-grouped layout for the single-precision min-sum kernel (bp.hpp)
    bool grp_ok = false;
    int grp_ntab = 0, grp_msg_bytes = 0, grp_vj = 0, grp_cj = 0;
    int32_t *d_grp_meta = nullptr, *d_grp_vmap = nullptr;
    uint16_t *d_grp_vtab = nullptr;
};

namespace sg {

// Longest-processing-time assignment of groups (weights w) to GRP_WAVES waves
// of at most `cap` groups each; returns the wave and position of every group.
static void lpt_waves(const std::vector<int> &w, int cap, std::vector<int> &wave, std::vector<int> &pos) {
    std::vector<int> order(w.size());
    for (size_t i = 0; i < w.size(); ++i) order[i] = (int)i;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return w[x] > w[y]; });
    std::vector<long> load(GRP_WAVES, 0);
    std::vector<int> cnt(GRP_WAVES, 0);
    wave.assign(w.size(), -1);
    pos.assign(w.size(), -1);
    for (int g : order) {
        int best = -1;
        for (int q = 0; q < GRP_WAVES; ++q)
            if (cnt[q] < cap && (best < 0 || load[q] < load[best])) best = q;
        wave[g] = best;
        pos[g] = cnt[best]++;
        load[best] += w[g];
    }
}

// Pairs of equal-degree variable groups run together (SG_BP_PAIR=0: one group at a time; A/B knob)
static bool grp_pairs() {
    const char *e = std::getenv("SG_BP_PAIR");
    return !(e && std::strcmp(e, "0") == 0);
}

// The degree-grouped layout of a graph (host arrays; bp.hpp BpGrpArgs)
struct GrpLayout {
    std::vector<int32_t> meta, vmap;
    std::vector<uint16_t> vtab;
    int msg_bytes = 0, vj = 0, cj = 0, npairs = 0;
};

// Degree-grouped layout (bp.hpp BpGrpArgs) of the graph, or false when the
// graph does not fit the grouped kernel (degrees, group counts, 16-bit LDS
// byte addresses).  voff/coff are the port offsets, intrlv the reference's
// variable-port -> check-port map.  Host only (sg_ldpc_grouped_layout exposes
// it for CPU tests).
static bool grp_layout(int nv, int nc, int nmsg, int max_vdeg, int max_cdeg, const int64_t *vdeg,
                       const int64_t *cdeg, const int64_t *intrlv, const std::vector<int32_t> &voff,
                       const std::vector<int32_t> &coff, bool pairs, GrpLayout &out) {
    if (max_cdeg > GRP_MAXDC || max_vdeg > GRP_MAXDV) return false;
    // the per-degree check code covers degrees 2..8 only (grp_check_d): a
    // check of degree 0 or 1 takes the table kernel
    for (int c = 0; c < nc; ++c)
        if (cdeg[c] < 2) return false;
    // checks by degree (descending, stable), groups of 64 of one degree
    std::vector<int> corder(nc);
    for (int c = 0; c < nc; ++c) corder[c] = c;
    std::stable_sort(corder.begin(), corder.end(), [&](int x, int y) { return cdeg[x] > cdeg[y]; });
    std::vector<int> cg_deg, cg_first, cg_n;
    for (int i = 0; i < nc;) {
        const int d = (int)cdeg[corder[i]];
        int n = 0;
        while (i + n < nc && n < 64 && cdeg[corder[i + n]] == d) ++n;
        cg_deg.push_back(d); cg_first.push_back(i); cg_n.push_back(n);
        i += n;
    }
    std::vector<int> vorder(nv);
    for (int v = 0; v < nv; ++v) vorder[v] = v;
    std::stable_sort(vorder.begin(), vorder.end(), [&](int x, int y) { return vdeg[x] > vdeg[y]; });
    std::vector<int> vg_deg, vg_first, vg_n;
    for (int i = 0; i < nv;) {
        const int d = (int)vdeg[vorder[i]];
        int n = 0;
        while (i + n < nv && n < 64 && vdeg[vorder[i + n]] == d) ++n;
        vg_deg.push_back(d); vg_first.push_back(i); vg_n.push_back(n);
        i += n;
    }
    const int ncg = (int)cg_deg.size(), nvg = (int)vg_deg.size();
    const int cj = (ncg + GRP_WAVES - 1) / GRP_WAVES, vj = (nvg + GRP_WAVES - 1) / GRP_WAVES;
    if (vj > 8 || cj > 4) return false;
    const int KVJ = grp_kvj(vj, cj), KCJ = grp_kcj(vj, cj);
    // check groups: weights = degree; message blocks laid out wave by wave
    std::vector<int> cw, cp, vw, vp;
    lpt_waves(cg_deg, cj, cw, cp);
    std::vector<int> vweight(nvg);
    for (int i = 0; i < nvg; ++i) vweight[i] = vg_deg[i] + 1;  // + the group's fixed cost
    lpt_waves(vweight, vj, vw, vp);
    // within each wave, groups of one pairable degree (GRP_PAIR_MAXD) side by side: the kernel runs such a
    // pair's chains together (grp_var2), the first of the pair flagged with GRP_PAIR in its degree word
    std::vector<char> pair_first(nvg, 0);
    for (int w = 0; w < GRP_WAVES; ++w) {
        std::vector<int> mine;
        for (int i = 0; i < nvg; ++i)
            if (vw[i] == w) mine.push_back(i);
        std::stable_sort(mine.begin(), mine.end(), [&](int x, int y) { return vp[x] < vp[y]; });
        // pairs first (so every pair starts at an even position), then the single groups
        std::vector<int> ord, singles;
        std::vector<char> used(mine.size(), 0);
        for (size_t a = 0; a < mine.size(); ++a) {
            if (used[a]) continue;
            used[a] = 1;
            size_t b = a + 1;
            if (vg_deg[mine[a]] >= 1 && vg_deg[mine[a]] <= GRP_PAIR_MAXD)
                for (; b < mine.size(); ++b)
                    if (!used[b] && vg_deg[mine[b]] == vg_deg[mine[a]]) break;
            if (b < mine.size() && vg_deg[mine[a]] >= 1 && vg_deg[mine[a]] <= GRP_PAIR_MAXD) {
                used[b] = 1;
                pair_first[mine[a]] = 1;
                ord.push_back(mine[a]);
                ord.push_back(mine[b]);
            } else {
                singles.push_back(mine[a]);
            }
        }
        ord.insert(ord.end(), singles.begin(), singles.end());
        for (size_t q = 0; q < ord.size(); ++q) vp[ord[q]] = (int)q;
    }
    std::vector<int32_t> meta(2 * GRP_WAVES * KVJ + 3 * GRP_WAVES * KCJ, 0);
    int32_t *m_vdeg = meta.data(), *m_vtab = m_vdeg + GRP_WAVES * KVJ;
    int32_t *m_cdeg = m_vtab + GRP_WAVES * KVJ, *m_caddr = m_cdeg + GRP_WAVES * KCJ, *m_cval = m_caddr + GRP_WAVES * KCJ;
    std::vector<int32_t> caddr(ncg, 0);
    long bytes = 0;
    for (int w = 0; w < GRP_WAVES; ++w)
        for (int q = 0; q < KCJ; ++q)
            for (int i = 0; i < ncg; ++i)
                if (cw[i] == w && cp[i] == q) {
                    caddr[i] = (int32_t)bytes;
                    bytes += 256L * cg_deg[i];
                    m_cdeg[w * KCJ + q] = cg_deg[i];
                    m_caddr[w * KCJ + q] = caddr[i];
                    m_cval[w * KCJ + q] = cg_n[i];
                }
    const long trash = bytes;
    const long msg_bytes = (bytes + 4 + 15) / 16 * 16;
    if (msg_bytes > 65536) return false;
    // check-port byte address of every message index (check c, port k)
    std::vector<int32_t> cslot_base(nc);
    for (int i = 0; i < ncg; ++i)
        for (int l = 0; l < cg_n[i]; ++l) cslot_base[corder[cg_first[i] + l]] = caddr[i] + 4 * l;
    std::vector<int32_t> msg_addr(nmsg);
    for (int c = 0; c < nc; ++c)
        for (int k = 0; k < coff[c + 1] - coff[c]; ++k) msg_addr[coff[c] + k] = cslot_base[c] + 256 * k;
    // variable groups: table blocks [degree][64] wave by wave, lanes' variables
    std::vector<int32_t> vmap((size_t)GRP_WAVES * KVJ * 64, -1);
    std::vector<uint16_t> vtab;
    for (int w = 0; w < GRP_WAVES; ++w)
        for (int j = 0; j < KVJ; ++j)
            for (int i = 0; i < nvg; ++i)
                if (vw[i] == w && vp[i] == j) {
                    const int d = vg_deg[i];
                    m_vdeg[w * KVJ + j] = d | (pair_first[i] && pairs ? GRP_PAIR : 0);
                    out.npairs += pair_first[i] && pairs ? 1 : 0;
                    m_vtab[w * KVJ + j] = (int32_t)(2 * vtab.size());
                    const size_t off = vtab.size();
                    vtab.resize(off + 64 * (size_t)d, (uint16_t)trash);
                    for (int l = 0; l < vg_n[i]; ++l) {
                        const int v = vorder[vg_first[i] + l];
                        vmap[(size_t)(w * KVJ + j) * 64 + l] = v;
                        for (int k = 0; k < d; ++k) vtab[off + 64 * k + l] = (uint16_t)msg_addr[intrlv[voff[v] + k]];
                    }
                }
    if ((size_t)msg_bytes + GRP_FLAG_BYTES > (size_t)BP_MAX_LDS || vtab.empty()) return false;
    // every real port addresses a distinct 4-byte slot inside the message image
    // and every check-group slot of a real check is reached exactly once
    std::vector<uint8_t> hit(msg_bytes / 4, 0);
    long real = 0;
    for (uint16_t e : vtab) {
        if (e == (uint16_t)trash) continue;
        if (e % 4 || e >= trash || hit[e / 4]++) return false;
        ++real;
    }
    if (real != nmsg) return false;
    out.meta = std::move(meta);
    out.vmap = std::move(vmap);
    out.vtab = std::move(vtab);
    out.msg_bytes = (int)msg_bytes;
    out.vj = vj;
    out.cj = cj;
    return true;
}

// The grouped layout of a graph uploaded for the kernel (false: the graph takes the table kernel)
static bool build_groups(sg_graph *g, const int64_t *vdeg, const int64_t *cdeg, const int64_t *intrlv,
                         const std::vector<int32_t> &voff, const std::vector<int32_t> &coff, hipStream_t s) {
    GrpLayout lay;
    if (!grp_layout(g->nv, g->nc, g->nmsg, g->max_vdeg, g->max_cdeg, vdeg, cdeg, intrlv, voff, coff, grp_pairs(),
                    lay))
        return false;
    const std::vector<int32_t> &meta = lay.meta, &vmap = lay.vmap;
    const std::vector<uint16_t> &vtab = lay.vtab;
    bool ok = hipMalloc(&g->d_grp_meta, sizeof(int32_t) * meta.size()) == hipSuccess &&
              hipMalloc(&g->d_grp_vmap, sizeof(int32_t) * vmap.size()) == hipSuccess &&
              hipMalloc(&g->d_grp_vtab, sizeof(uint16_t) * vtab.size()) == hipSuccess;
    ok = ok && hipMemcpyAsync(g->d_grp_meta, meta.data(), sizeof(int32_t) * meta.size(), hipMemcpyHostToDevice, s) == hipSuccess &&
         hipMemcpyAsync(g->d_grp_vmap, vmap.data(), sizeof(int32_t) * vmap.size(), hipMemcpyHostToDevice, s) == hipSuccess &&
         hipMemcpyAsync(g->d_grp_vtab, vtab.data(), sizeof(uint16_t) * vtab.size(), hipMemcpyHostToDevice, s) == hipSuccess &&
         hipStreamSynchronize(s) == hipSuccess;
    if (!ok) return false;
    g->grp_ntab = (int)vtab.size();
    g->grp_msg_bytes = lay.msg_bytes;
    g->grp_vj = lay.vj;
    g->grp_cj = lay.cj;
    g->grp_ok = true;
    return true;
}

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
    build_groups(g, vdeg, cdeg, intrlv, voff, coff, s);  // (optional: the table kernel takes every graph)
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

// SG_BP_GROUPED=0 routes single-precision min-sum to the table kernel (A/B)
static bool use_grouped() {
    const char *e = std::getenv("SG_BP_GROUPED");
    return !(e && e[0] == '0');
}

static int decode_device(sg_graph *g, int dectype, int precision, const void *d_ch, int B, int max_it,
                         double corr, void *d_app, int32_t *d_it, hipStream_t s, bool ch_has_nan = false) {
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
    if (precision == SG_F32 && dectype == SG_MINSUM && g->grp_ok && use_grouped() && !ch_has_nan) {
        BpGrpArgs a;
        a.meta = g->d_grp_meta; a.vmap = g->d_grp_vmap; a.vtab = g->d_grp_vtab;
        a.ntab = g->grp_ntab; a.msg_bytes = g->grp_msg_bytes; a.vj = g->grp_vj; a.cj = g->grp_cj;
        a.nv = g->nv;
        a.ch = (const float *)d_ch; a.app = (float *)d_app; a.it = d_it;
        a.B = B; a.max_it = max_it; a.factor = (float)corr;
        return bp_grouped_launch(a, s);
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
    bool ch_has_nan = false;
    if (precision == SG_F64) {
        SG_HIP(hipMemcpyAsync(g->d_ch, ch, n * sizeof(double), hipMemcpyHostToDevice, s));
    } else {
        std::vector<float> tmp(n);
        bool nonfinite = false;
        for (size_t i = 0; i < n; ++i) {
            const double v = ch[i];
            if (std::isfinite(v)) {  // a finite double past float's range stays finite: +-FLT_MAX
                tmp[i] = (float)std::min(std::max(v, -(double)FLT_MAX), (double)FLT_MAX);
            } else {
                tmp[i] = (float)v;
                nonfinite = true;
            }
        }
        // a NaN or infinite input goes to the table kernel: NaN and inf semantics of the reference; finite
        // inputs (clamped to +-FLT_MAX above) take the grouped kernel, which saturates channel LLRs at +-1e30
        ch_has_nan = nonfinite;
        SG_HIP(hipMemcpyAsync(g->d_ch, tmp.data(), n * sizeof(float), hipMemcpyHostToDevice, s));
        SG_HIP(hipStreamSynchronize(s));
    }
    SG_TRY(decode_device(g, dectype, precision, g->d_ch, B, max_it, corr, g->d_app, g->d_it, s, ch_has_nan));
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
    if (g->d_grp_meta) hipFree(g->d_grp_meta);
    if (g->d_grp_vmap) hipFree(g->d_grp_vmap);
    if (g->d_grp_vtab) hipFree(g->d_grp_vtab);
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

int sg_ldpc_grouped_layout(const int64_t *vdeg, const int64_t *cdeg, const int64_t *intrlv, int nv, int nc, int nmsg,
                           int pairs, int32_t *info, int32_t *meta, int meta_cap, int32_t *vmap, int vmap_cap,
                           uint16_t *vtab, int vtab_cap) {
    using namespace sg;
    SG_CHECK_ARG(vdeg && cdeg && intrlv && info, "null argument");
    SG_CHECK_ARG(nv > 0 && nc > 0 && nmsg > 0, "empty graph (Nv=%d Nc=%d Nmsg=%d)", nv, nc, nmsg);
    std::vector<int32_t> voff(nv + 1, 0), coff(nc + 1, 0);
    int max_v = 0, max_c = 0;
    for (int v = 0; v < nv; ++v) {
        SG_CHECK_ARG(vdeg[v] >= 0 && vdeg[v] < 256, "variable degree %lld out of range", (long long)vdeg[v]);
        voff[v + 1] = voff[v] + (int32_t)vdeg[v];
        max_v = std::max(max_v, (int)vdeg[v]);
    }
    for (int c = 0; c < nc; ++c) {
        SG_CHECK_ARG(cdeg[c] >= 2 && cdeg[c] < 256, "check degree %lld out of range (need 2..255)", (long long)cdeg[c]);
        coff[c + 1] = coff[c] + (int32_t)cdeg[c];
        max_c = std::max(max_c, (int)cdeg[c]);
    }
    SG_CHECK_ARG(voff[nv] == nmsg && coff[nc] == nmsg, "degree sums (%d, %d) do not match Nmsg=%d", voff[nv],
                 coff[nc], nmsg);
    {  // the same permutation check as graph creation: grp_layout indexes msg_addr[intrlv[p]]
        std::vector<uint8_t> seen(nmsg, 0);
        for (int p = 0; p < nmsg; ++p) {
            const int64_t m = intrlv[p];
            SG_CHECK_ARG(m >= 0 && m < nmsg && !seen[m], "intrlv is not a permutation of [0, Nmsg)");
            seen[m] = 1;
        }
    }
    GrpLayout lay;
    const bool ok = grp_layout(nv, nc, nmsg, max_v, max_c, vdeg, cdeg, intrlv, voff, coff, pairs != 0, lay);
    const int32_t v[10] = {ok ? 1 : 0, lay.vj, lay.cj, ok ? grp_kvj(lay.vj, lay.cj) : 0,
                           ok ? grp_kcj(lay.vj, lay.cj) : 0, lay.msg_bytes, (int32_t)lay.vtab.size(), lay.npairs,
                           (int32_t)lay.meta.size(), (int32_t)lay.vmap.size()};
    std::copy(v, v + 10, info);
    if (!ok) return SG_OK;
    if (meta) {
        SG_CHECK_ARG(meta_cap >= (int)lay.meta.size(), "meta buffer too small");
        std::copy(lay.meta.begin(), lay.meta.end(), meta);
    }
    if (vmap) {
        SG_CHECK_ARG(vmap_cap >= (int)lay.vmap.size(), "vmap buffer too small");
        std::copy(lay.vmap.begin(), lay.vmap.end(), vmap);
    }
    if (vtab) {
        SG_CHECK_ARG(vtab_cap >= (int)lay.vtab.size(), "vtab buffer too small");
        std::copy(lay.vtab.begin(), lay.vtab.end(), vtab);
    }
    return SG_OK;
}

int sg_ldpc_decode_kernel(const sg_graph *g, int dectype, int precision, char *name, size_t len) {
    using namespace sg;
    SG_CHECK_ARG(g && name && len > 0, "null graph or name buffer");
    SG_CHECK_ARG(dectype == SG_SUMPROD || dectype == SG_SUMPROD2 || dectype == SG_MINSUM,
                 "Decoder type unknonwn (dectype=%d)", dectype);
    SG_CHECK_ARG(precision == SG_F64 || precision == SG_F32, "precision must be SG_F64 or SG_F32");
    char buf[96];
    if (precision == SG_F32 && dectype == SG_MINSUM && g->grp_ok && use_grouped()) {
        snprintf(buf, sizeof buf, "bp_grouped_minsum_kernel<%d, %d>", grp_kvj(g->grp_vj, g->grp_cj),
                 grp_kcj(g->grp_vj, g->grp_cj));
    } else {  // bp.hip dispatch_dc / dispatch_vj
        const int dc = g->max_cdeg <= 8 ? 8 : g->max_cdeg <= 16 ? 16 : g->max_cdeg <= 24 ? 24 : 32;
        const int vj = g->nv <= 4 * BP_THREADS ? 4 : BP_VJ;
        snprintf(buf, sizeof buf, "bp_flood_kernel<%s, %d, %d, %d>", precision == SG_F64 ? "double" : "float",
                 dectype, dc, vj);
    }
    snprintf(name, len, "%s", buf);
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
