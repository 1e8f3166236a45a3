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
int sg_set_device(int device);
int sg_get_stream(void **stream);           /* library stream of the current device */
int sg_malloc(void **dptr, size_t bytes);
int sg_free(void *dptr);
int sg_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream);
int sg_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream);
int sg_memset(void *dptr, int value, size_t bytes, void *stream);
int sg_stream_synchronize(void *stream);

/* HIP events on a given stream (bench.py times the kernels on the stream they
 * run on, not on torch's current stream). */
int sg_event_create(void **ev);
int sg_event_destroy(void *ev);
int sg_event_record(void *ev, void *stream);
int sg_event_elapsed_ms(void *start, void *stop, float *ms);

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
/* Device variant: d_ch/d_app are float or double per `precision`. */
int sg_ldpc_decode_device(sg_graph *g, int dectype, int precision, const void *d_ch, int B,
                          int max_it, double corr, void *d_app, int32_t *d_it, void *stream);
/* Device-side error counting against known codewords (ldpc_awgn.py:97-104):
 * d_x[B][nv] uint8 transmitted bits, app from sg_ldpc_decode_device.  Adds to
 * d_counts[4] = {bit errors over nv, frame errors, bit errors over the first
 * k (systematic) bits, sum of it}. */
int sg_ldpc_count_errors_device(sg_graph *g, int precision, const void *d_app, const uint8_t *d_x,
                                const int32_t *d_it, int B, int k, int64_t *d_counts,
                                void *stream);

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

#ifdef __cplusplus
}
#endif
#endif /* LDPC_SPARC_AMD_H */
