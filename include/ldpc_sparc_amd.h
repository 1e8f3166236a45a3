/*
 * ldpc_sparc_amd.h -- C ABI of libldpc_sparc_amd.so, the MI355X (gfx950)
 * AMP/BP decoding engine behind the reference's Python call surface.
 *
 * Conventions
 *   - every entry point returns 0 on success and a negative code on failure
 *     (no C++ exceptions cross the ABI); sg_last_error() describes the last
 *     failure on the calling thread;
 *   - "host" entry points take caller-owned host buffers and block until the
 *     result is back in them; "_device" entry points take device pointers and
 *     a hipStream_t (NULL = the library's stream for the current device) and
 *     return without synchronising;
 *   - handles (sg_graph, sg_amp_plan, sg_comm) own device memory and belong to
 *     the device that was current when they were created; one process per GPU.
 *   - the library has no CPU decode path: without a visible gfx950 device every
 *     decode entry point fails with SG_ERR_NO_DEVICE.
 *
 * Reference interfaces replaced are cited per entry point (path:line under the
 * reference repository SophieLangdon27/LDPC_SPARC).
 */
#ifndef LDPC_SPARC_AMD_H
#define LDPC_SPARC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum sg_status {
    SG_OK = 0,
    SG_ERR_INVALID = -2,   /* bad argument (shape, degree, enum) */
    SG_ERR_NO_DEVICE = -3, /* no usable GPU */
    SG_ERR_HIP = -4,       /* HIP runtime failure */
    SG_ERR_NOMEM = -5,     /* allocation failure (the reference returns -1 here, c_ldpc.c:41) */
    SG_ERR_UNSUPPORTED = -6,
    SG_ERR_COMM = -7       /* RCCL failure */
};

enum sg_dectype { SG_SUMPROD = 0, SG_SUMPROD2 = 1, SG_MINSUM = 2 };
enum sg_precision { SG_F64 = 0, SG_F32 = 1 };

/* ---------------------------------------------------------------- runtime */
const char *sg_last_error(void);
const char *sg_version(void);
int sg_device_count(int *count);
int sg_device_cu_count(int *cus); /* compute units of the current device */
int sg_set_device(int device);
int sg_get_stream(void **stream);           /* library stream of the current device */
int sg_malloc(void **dptr, size_t bytes);
int sg_free(void *dptr);
int sg_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream);
int sg_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream);
int sg_memset(void *dptr, int value, size_t bytes, void *stream);
int sg_stream_synchronize(void *stream);
/* An extra non-blocking stream (concurrent batches on one GPU). */
int sg_stream_create(void **stream);
int sg_stream_destroy(void *stream);

/* HIP events on a given stream (bench.py times the kernels on the stream they
 * run on, not on torch's current stream). */
int sg_event_create(void **ev);
int sg_event_destroy(void *ev);
int sg_event_record(void *ev, void *stream);
int sg_event_elapsed_ms(void *start, void *stop, float *ms);
int sg_device_synchronize(void);

/* Per-phase kernel timing.  When enabled, every kernel launch of the decoders
 * is bracketed by HIP events on the stream it is launched on; collect
 * synchronises the pending events, returns the summed milliseconds and the
 * launch count per phase (arrays of SG_PH_COUNT) and resets the counters.
 * on = 2 records only the per-iteration scope of the split per-codeword
 * engine, not its per-kernel scopes inside it: every timed event record on a
 * stream holds the next kernel back by several microseconds, so bench.py's
 * timed region brackets each iteration (two events) rather than each of its
 * four kernels. */
enum sg_phase {
    SG_PH_AB_A = 0, SG_PH_AB_B = 1, SG_PH_AZ_A = 2, SG_PH_AZ_B = 3, SG_PH_ETA = 4,
    SG_PH_CONTROL = 5, SG_PH_BP = 6, SG_PH_DENSE = 7, SG_PH_AMP_CW = 8, SG_PH_CW2_AB = 9, SG_PH_CW2_AZ = 10,
    SG_PH_CW2_CTRL = 11, SG_PH_COUNT = 12
};
int sg_profile_enable(int on);
int sg_profile_collect(double *total_ms, int64_t *launches);
const char *sg_phase_name(int phase);

/* ------------------------------------------------------- dense design AMP */
typedef struct sg_dense_plan sg_dense_plan;

/* Dense Gaussian design A [n][L*M] row-major (create_design_matrix,
 * sparc_new.py:1284-1294: default_rng(seed).normal(0, 1/sqrt(n))), uploaded
 * once and shared by every codeword of a batch.  P is the total power
 * (nonzero entries sqrt(n P / L), sparc_new.py:45-46).  SG_F32 runs the two
 * products as matrix-core GEMMs (v_mfma_f32_32x32x2_f32); SG_F64 is the
 * parity path.  _random draws A on the device (Philox4x32-10 + Box-Muller,
 * statistically equal to the reference's draw, not bitwise) for throughput runs. */
int sg_dense_plan_create(const double *A, int n, int L, int M, double P, int precision, sg_dense_plan **out);
int sg_dense_plan_create_random(int n, int L, int M, double P, uint64_t seed, int precision,
                                sg_dense_plan **out);
int sg_dense_plan_destroy(sg_dense_plan *p);
int sg_dense_plan_info(const sg_dense_plan *p, int *n, int *L, int *M, int *nsplit);
/* Batched AMP with fixed t_max iterations (sparc_new.py:885-912, one call per
 * codeword in the reference): y [B][n] -> soft estimate beta [B][L*M] and
 * effective observation s [B][L*M] (the reference's return values). */
int sg_dense_amp(sg_dense_plan *p, const double *y, int B, int t_max, double *beta, double *s);
int sg_dense_amp_device(sg_dense_plan *p, const void *d_y, int B, int t_max, void *d_beta, void *d_s,
                        void *stream);
/* One iteration from a given state (sparc_amp_single_it, sparc_new.py:975-990):
 * y [n], beta [L*M], z [n], tau_sqr -> beta', z', tau_sqr'. */
int sg_dense_amp_iteration(sg_dense_plan *p, const double *y, const double *beta, const double *z,
                           double tau_sqr, double *beta_out, double *z_out, double *tau_sqr_out);
/* Device pointers of the plan's own beta and s [B][L*M] after the last
 * sg_dense_amp_device call (valid until the next call; lets a pipeline feed
 * the glue without copies). */
int sg_dense_state_device(sg_dense_plan *p, void **d_beta, void **d_s);
/* Device pointer of the plan's design matrix A [n][L*M] (row-major, the
 * plan's precision, no padding) -- lets a checker read A back in row blocks
 * (tests/test_c5_full_gpu.py) without a second copy. */
int sg_dense_plan_matrix_device(const sg_dense_plan *p, const void **d_A);
/* x = A beta0 for one-hot beta0 (section index d_idx [B][L], value sqrt(n P / L)). */
int sg_dense_encode_device(sg_dense_plan *p, const int32_t *d_idx, int B, void *d_x, void *stream);
/* MAP section indices of s [B][L*M] (msg_vector_map_estimator, sparc_new.py:1099-1116). */
int sg_dense_map_device(sg_dense_plan *p, const void *d_s, int B, int32_t *d_idx, void *stream);
/* AMP -> BP glue (beta_estimate_to_bp_probs, sparc_new.py:1118-1138, then the
 * clip and log of ldpc_bp :1167-1169): for sections [l0, l0+nl) of beta
 * [B][L*M], bit LLRs (MSB first, positive => 0) at d_llr[b*llr_ld + (l-l0)*log2 M + i],
 * or the bit-0 probabilities themselves when probs_only. */
int sg_beta_to_llr_device(int precision, const void *d_beta, int B, int L, int M, double sqrt_nPl, int l0,
                          int nl, int llr_ld, int probs_only, void *d_llr, void *stream);

/* Error counts of the concatenated scheme (sparc_sim_new.py:12-23):
 * unprotected bits from MAP indices d_map_idx [B][L] (first L_unprotected
 * sections) against d_true_idx, protected bits app[:K] < 0 of each of the
 * `mults` BP blocks (d_app [B*mults][N]) against d_info [B][mults*K].  Adds
 * {codewords, bit errors, codeword errors, unprotected bit errors, protected
 * bit errors} into d_counts[5]. */
int sg_concat_count_errors_device(int precision, const int32_t *d_map_idx, const int32_t *d_true_idx, int B,
                                  int L, int L_unprotected, int logM, const void *d_app, const uint8_t *d_info,
                                  int mults, int N, int K, int64_t *d_counts, void *stream);

/* ------------------------------------------------------------- multi-GPU */
/* One RCCL communicator per process (one process per GPU).  Rank 0 creates
 * the 128-byte unique id, the launcher distributes it, every rank calls init.
 * New capability: the reference parallelises only by independent processes
 * (ldpc_jossy/py/ldpc_awgn.py:125-131). */
typedef struct sg_comm sg_comm;
int sg_comm_unique_id(void *id_out /* 128 bytes */);
int sg_comm_init(int nranks, int rank, const void *id, sg_comm **out);
int sg_comm_allreduce_sum_i64(sg_comm *c, int64_t *d_buf, size_t count, void *stream);
int sg_comm_info(sg_comm *c, int *nranks, int *device); /* ranks and device as RCCL sees them */
int sg_comm_destroy(sg_comm *c);

/* ------------------------------------------------------------------- LDPC */
typedef struct sg_graph sg_graph;

/* Upload a Tanner graph in the reference layout (ldpc.py:303-396): vdeg[nv],
 * cdeg[nc], intrlv[nmsg] mapping variable ports to check-ordered message
 * indices.  Validates that intrlv is a permutation and the degree sums match. */
int sg_ldpc_graph_create(const int64_t *vdeg, const int64_t *cdeg, const int64_t *intrlv, int nv,
                         int nc, int nmsg, sg_graph **out);
int sg_ldpc_graph_destroy(sg_graph *g);
int sg_ldpc_graph_info(const sg_graph *g, int *nv, int *nc, int *nmsg, int *max_cdeg,
                       int *max_vdeg);
/* Name of the kernel sg_ldpc_decode(_device) launches for this graph, decoder
 * type and precision, as rocprofv3 lists it (e.g. "bp_grouped_minsum_kernel<4, 2>"
 * for the degree-grouped single-precision min-sum kernel, "bp_flood_kernel<float,
 * 1, 8, 4>" for the table kernel); NUL-terminated, truncated to len bytes. */
int sg_ldpc_decode_kernel(const sg_graph *g, int dectype, int precision, char *name, size_t len);
/* The degree-grouped layout the single-precision min-sum kernel would use for
 * a graph (bp.hpp BpGrpArgs), computed on the host with no device: info[10] =
 * {grouped (1) or table kernel (0), variable / check groups per wave, the
 * kernel instance's groups per wave (2), message image bytes, port-table
 * entries, variable-group pairs, meta and vmap lengths}; meta / vmap / vtab are
 * copied out when non-null (call once with nulls for the sizes).  pairs: run
 * equal-degree variable groups in pairs (the decode default; SG_BP_PAIR=0
 * turns it off there).  For tests that emulate the kernel on the CPU. */
int sg_ldpc_grouped_layout(const int64_t *vdeg, const int64_t *cdeg, const int64_t *intrlv, int nv, int nc,
                           int nmsg, int pairs, int32_t *info, int32_t *meta, int meta_cap, int32_t *vmap,
                           int vmap_cap, uint16_t *vtab, int vtab_cap);

/* Batched flooding BP (replaces one c_ldpc.c sumprod/sumprod2/minsum call per
 * codeword, c_ldpc.c:32,138,339; driven serially by ldpc.py:463-490 and
 * sparc_new.py:1176-1179).  ch/app are row-major [B][nv] LLRs, it[B] receives
 * the reference's return value per codeword (0-based index of the stopping
 * iteration, or max_it).  minsum uses the corrected check indexing
 * (DESIGN.md "minsum") and `corr` as the normalisation factor (reference
 * default 0.7, ldpc.py:463).  precision SG_F64 reproduces the reference's
 * double arithmetic; SG_F32 is the throughput path. */
int sg_ldpc_decode(sg_graph *g, int dectype, int precision, const double *ch, int B, int max_it,
                   double corr, double *app, int32_t *it);
/* Device variant: d_ch/d_app are float or double per `precision`.  SG_F32
 * min-sum on a graph of the degree-grouped layout (bp_grouped.hip) expects
 * NaN-free channel LLRs and saturates them at +-1e30 (so +-inf decodes as
 * +-1e30); the host entry point above sends a batch holding a NaN, an
 * infinity or a value that overflows float to the table kernel instead. */
int sg_ldpc_decode_device(sg_graph *g, int dectype, int precision, const void *d_ch, int B,
                          int max_it, double corr, void *d_app, int32_t *d_it, void *stream);
/* Device-side error counting against known codewords (ldpc_awgn.py:97-104):
 * d_x[B][nv] uint8 transmitted bits, app from sg_ldpc_decode_device.  Adds to
 * d_counts[4] = {bit errors over nv, frame errors, bit errors over the first
 * k (systematic) bits, sum of it}. */
int sg_ldpc_count_errors_device(sg_graph *g, int precision, const void *d_app, const uint8_t *d_x,
                                const int32_t *d_it, int B, int k, int64_t *d_counts,
                                void *stream);
/* Bit errors (hard decision app < 0 against d_x, over all Nv bits) of each
 * codeword: d_bit_errors[B].  The per-codeword form lets a campaign stop at
 * the codeword where the frame-error count is reached (ldpc_awgn.py:86-105). */
int sg_ldpc_codeword_errors_device(sg_graph *g, int precision, const void *d_app, const uint8_t *d_x, int B,
                                   int32_t *d_bit_errors, void *stream);

/* ------------------------------------------- device encoder and channel */
/* Throughput-mode generation, keyed by Philox4x32-10
 * counters (seed, stream_id, codeword index, element): results depend only on
 * the key, not on B, the grid or the rank.  Parity mode (the reference's
 * numpy generators, seed for seed) stays on the host. */
/* nbits random bits per row, d_bits [B][nbits] uint8 (ldpc_awgn.py:44 / sparc.py:174-180) */
int sg_rng_bits_device(uint64_t seed, uint64_t stream_id, int B, int nbits, uint8_t *d_bits, void *stream);
/* section indices from MSB-first bit groups (sparc.py:330-364): d_bits [B][L*logM] -> d_idx [B][L] */
int sg_bits_to_sections_device(const uint8_t *d_bits, int B, int L, int logM, int32_t *d_idx, void *stream);
/* The same with row strides: codeword b's bits at d_bits + b * bit_stride,
 * its L indices at d_idx + b * idx_stride (a part of a longer message, e.g.
 * the protected sections of a concatenated codeword, sparc_new.py:15-51). */
int sg_bits_to_sections_strided_device(const uint8_t *d_bits, size_t bit_stride, int B, int L, int logM,
                                       int32_t *d_idx, size_t idx_stride, void *stream);
/* y = x + sigma N(0, 1) [B][n] (sparc_sim.py:179-204) */
int sg_awgn_device(int precision, uint64_t seed, uint64_t stream_id, const void *d_x, int B, int n, double sigma,
                   void *d_y, void *stream);
/* BPSK 1 - 2c over AWGN with variance sigma2, channel LLRs 2y/sigma2 [B][N] (ldpc_awgn.py:39-56) */
int sg_bpsk_awgn_llr_device(int precision, uint64_t seed, uint64_t stream_id, const uint8_t *d_cw, int B, int N,
                            double sigma2, void *d_llr, void *stream);
/* Systematic LDPC encoder (ldpc.py:400-460) as a GF(2) product: parity
 * [K][N-K] uint8 is the parity part of the code's generator (the encoder's
 * image of the unit vectors); cw = [info, info P]. */
typedef struct sg_ldpc_encoder sg_ldpc_encoder;
int sg_ldpc_encoder_create(const uint8_t *parity, int K, int N, sg_ldpc_encoder **out);
int sg_ldpc_encoder_destroy(sg_ldpc_encoder *e);
int sg_ldpc_encode_device(sg_ldpc_encoder *e, const uint8_t *d_info, int B, uint8_t *d_cw, void *stream);

/* ------------------------------------------------------ state evolution */
/* SPARC state evolution (sparc_public/sparc_se.py:82-183): Monte-Carlo samples
 * u [mc][M] (the reference's np.random.randn draw) stay on the device;
 * sg_se_expectation evaluates sparc_se_E (:82-115) for nt values of tau at
 * once (K = 1, or K = 2 for real modulated SPARCs). */
typedef struct sg_se_samples sg_se_samples;
int sg_se_samples_create(const double *u, int mc, int M, sg_se_samples **out);
int sg_se_samples_destroy(sg_se_samples *h);
int sg_se_expectation(sg_se_samples *h, int K, const double *taus, int nt, double *E);

/* ------------------------------------------------- integrated AMP <-> BP */
/* The integrated decoders of sparc_sophie/sparc_new.py on a dense design
 * plan and an LDPC graph; every L log2 M bits of a codeword are LDPC
 * protected (ldpc_bp asserts it, sparc_new.py:1171).  mode:
 *   SG_INT_NAIVE       naively_integrated_decoder :257-282
 *   SG_INT_NAIVE_POST  naively_integrated_decoder_posteriors :411-439
 *   SG_INT_DIFF        integrated_decoder :472-502 (differentiated eta :824-841)
 *   SG_INT_DIFF_POST   integrated_decoder_posteriors :675-705 (:843-869)
 * y [B][n] -> bits [B][(L log2 M / N) K] (app[:K] < 0 of the final decode,
 * bp_its_final iterations; bp_its per intermediate decode; the reference uses
 * 6 and 200, sumprod2).  tau2 [B][t_max] (optional) receives tau^2 of every
 * iteration. */
enum sg_integrated_mode { SG_INT_NAIVE = 0, SG_INT_NAIVE_POST = 1, SG_INT_DIFF = 2, SG_INT_DIFF_POST = 3 };
int sg_integrated_decode(sg_dense_plan *p, sg_graph *g, int mode, int K, const double *y, int B, int t_max,
                         int bp_its, int bp_its_final, uint8_t *bits, double *tau2);
int sg_integrated_decode_device(sg_dense_plan *p, sg_graph *g, int mode, int K, const void *d_y, int B,
                                int t_max, int bp_its, int bp_its_final, uint8_t *d_bits, double *d_tau2,
                                void *stream);
/* The soft-glue functions on host arrays, batched over B codewords:
 * bp_output_to_beta_estimate :1260-1279 (probs [B][L log2 M] -> beta [B][L M]),
 * update_using_bp_probs :1030-1038, differentiated_eta_calc(_posteriors)
 * :824-869 (tau2 [B]; gamma ignored unless posteriors). */
int sg_bp_output_to_beta(int precision, const double *probs, int B, int L, int M, double sqrt_nPl,
                         double *beta);
int sg_update_using_bp_probs(int precision, const double *gamma, const double *alpha, int B, int L, int M,
                             double sqrt_nPl, double *beta);
int sg_differentiated_eta(int precision, int posteriors, const double *beta, const double *gamma,
                          const double *alpha, const double *vk, const double *vk0, const double *tau2, int B,
                          int L, int M, double sqrt_nPl, double *out);

/* Reference-compatible scalar entry points: exact signatures of the ctypes
 * targets in ldpc.py:481-503 (c_ldpc.c:32,138,234,294,339) with Linux LP64
 * `long`.  Each call decodes one codeword on the GPU in double precision. */
int sumprod(double *ch, long *vdeg, long *cdeg, long *intrlv, int Nv, int Nc, int Nmsg,
            double *app, int max_itcount);
int sumprod2(double *ch, long *vdeg, long *cdeg, long *intrlv, int Nv, int Nc, int Nmsg,
             double *app, int max_itcount);
int minsum(double *ch, long *vdeg, long *cdeg, long *intrlv, int Nv, int Nc, int Nmsg,
           double *app, double correction_factor, int max_itcount);
double Lxor(double L1, double L2, int corr_flag);
double Lxfb(double *L, long dc, int corr_flag);


/* -------------------------------------------------------------------- AMP */
typedef struct sg_amp_plan sg_amp_plan;

/* Design of a real SPARC with sub-sampled DCT operator (sparc.py:703-880):
 * base matrix W (ndim 0: scalar P; 1: power allocation vector of Lc blocks;
 * 2: spatially coupled Lr x Lc matrix), one transform per nonzero entry of W
 * in row-major order, whose row/column orders are order0[t][Mr] and
 * order1[t][Mc] exactly as generate_ordering (sparc.py:735-775) draws them
 * (Mr = n or n/Lr, Mc = L*M/Lc).  precision SG_F64 follows the reference's
 * double arithmetic; SG_F32 is the throughput path.  A plan eligible for the
 * per-codeword engine also holds a staged-engine plan at P = 16384, which
 * decodes batches too small for the per-codeword engine (sg_amp_plan_info
 * reports the per-codeword plan's P). */
int sg_amp_plan_create(int ndim, const double *W, int Lr, int Lc, int L, int M, int n,
                       const uint32_t *order0, const uint32_t *order1, int precision,
                       sg_amp_plan **out);
int sg_amp_plan_destroy(sg_amp_plan *p);
int sg_amp_plan_info(const sg_amp_plan *p, int *w, int *nT, int *Mr, int *Mc, int *P, int *Q);
/* Engine a decode of B codewords with this plan runs on: 0 general four-step
 * (amp_dct.hip), 1 staged regular (amp_fused.hip), 2 per-codeword
 * (amp_cw.hip), 3 block (amp_block.hip).  Reads SG_AMP_ENGINE like the
 * decoder; returns the engine or a negative error code. */
int sg_amp_plan_engine(const sg_amp_plan *p, int B);
/* What the last decode through this plan ran: *engine as sg_amp_plan_engine
 * (-1 before any decode and after a decode call with B = 0 or one that failed
 * before choosing an engine: every decode call resets it), *handover_iter the first iteration the per-codeword
 * engine left to the staged engine (-1: no hand-over), *on_companion 1 when
 * the decode ran on the P = 16384 companion plan (may be NULL). */
int sg_amp_last_decode(const sg_amp_plan *p, int *engine, int *handover_iter, int *on_companion);

/* Batched AMP decode (sparc.py:883-999, one call per codeword in the
 * reference): y[B][n] received words sharing the plan's design; true_idx
 * [B][L] (optional) the transmitted section indices, used for NMSE.
 * Outputs: map_idx[B][L] final MAP section indices (argmax of s, sparc.py:997),
 * t_final[B], nmse[B][t_max][Lc], psi[B][Lc] (sparc.py:999 return values). */
int sg_amp_decode(sg_amp_plan *p, const double *y, int B, const int32_t *true_idx, double awgn_var,
                  int t_max, double rtol, int phi_method, int32_t *map_idx, int32_t *t_final,
                  double *nmse, double *psi);
/* Device variant: d_y in the plan precision (float or double), all outputs
 * device-resident (any output may be NULL). */
int sg_amp_decode_device(sg_amp_plan *p, const void *d_y, int B, const int32_t *d_true_idx,
                         double awgn_var, int t_max, double rtol, int phi_method,
                         int32_t *d_map_idx, int32_t *d_t_final, double *d_nmse, double *d_psi,
                         void *stream);
/* Design operators (the Ab / Az closures of sparc_transforms, sparc.py:786-875):
 * transpose 0: in[B][L*M] -> out[B][n];  transpose 1: in[B][n] -> out[B][L*M]. */
int sg_amp_apply(sg_amp_plan *p, int transpose, const double *in, int B, double *out);
/* x = A beta0 [B][n] on the device for section indices d_idx [B][L]
 * (one-hot beta0 with value 1, sparc.py:17-53 sparc_encode). */
int sg_amp_encode_device(sg_amp_plan *p, const int32_t *d_idx, int B, void *d_x, void *stream);
/* Diagnostics: mean shader-clock cycles of the phases of the last stage-1
 * launches (kernel 0 = Ab stage 1, 1 = Az stage 2; mean_cycles[8], entry k =
 * timestamp k minus timestamp k-1).  Only with SG_AMP_TPROF set in the
 * environment; otherwise *nphases = 0. */
int sg_amp_stage_profile(sg_amp_plan *p, int kernel, double *mean_cycles, int *nphases);
/* Diagnostics: the raw phase timestamps behind sg_amp_stage_profile, [items][10]:
 * 8 shader-clock values (per-XCD clocks) then the start and end on the 100 MHz
 * device-wide realtime clock, of the last iteration (items = B * column blocks * classes);
 * *items = 0 when SG_AMP_TPROF was not set.  out may be null to query *items. */
int sg_amp_stage_raw(sg_amp_plan *p, int kernel, uint64_t *out, size_t *items);
int sg_amp_apply_device(sg_amp_plan *p, int transpose, const void *d_in, int B, void *d_out,
                        void *stream);
/* Adds {section errors, bit errors (popcount of index XOR, MSB-first bits as
 * sparc.py:182-197), codeword errors, sum of t_final} into d_counts[4]. */
int sg_amp_count_errors_device(const int32_t *d_map_idx, const int32_t *d_true_idx,
                               const int32_t *d_t_final, int B, int L, int logM, int64_t *d_counts,
                               void *stream);

/* Stand-alone section estimators, double precision on the GPU:
 * out[l*M+j] = scale * softmax_j(x[l*M : (l+1)*M])  (msg_vector_mmse_estimator,
 * sparc.py:429-432 / sparc_new.py:1058-1066 with x = s/tau);
 * idx[l] = argmax_j s[l*M+j], first maximum (msg_vector_map_estimator, sparc.py:485-487). */
int sg_section_softmax(const double *x, int L, int M, double scale, double *out);
int sg_section_argmax(const double *x, int L, int M, int32_t *idx);

#ifdef __cplusplus
}
#endif
#endif /* LDPC_SPARC_AMD_H */
