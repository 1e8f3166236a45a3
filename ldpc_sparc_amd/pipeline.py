"""Batched, device-resident concatenated SPARC + LDPC decoding (the hot loop of
sparc_sim_new.sparc_ldpc_sim with many codewords sharing one design).

Per batch: dense AMP (sparc_new.py:885-912) -> MAP bits of the
unprotected sections (:70-71) -> bit LLRs of the protected sections
(beta_estimate_to_bp_probs :1118-1138 and ldpc_bp's clip/log :1167-1169) ->
batched BP over every LDPC block (ldpc_bp :1176-1187, sumprod2, 200 iterations
by default) -> device-side error counts.  Nothing returns to the host but the
five counters.
"""
import ctypes as ct

import numpy as np

from . import _native
from .ldpc import code
from .sparc_new import DenseDesign


class ConcatPipeline:
    def __init__(self, L, M, n, P, L_unprotected, mults, ldpc=("802.11n", "1/2", 81), design_seed=0,
                 precision="f32", t_max=25, bp_dectype="sumprod2", bp_its=200, A=None):
        self.L, self.M, self.n, self.P = int(L), int(M), int(n), float(P)
        self.logM = int(np.log2(M))
        self.L_unp, self.mults = int(L_unprotected), int(mults)
        self.c = code(*ldpc)
        assert (self.L - self.L_unp) * self.logM == self.mults * self.c.N, "protected sections must hold the blocks"
        self.prec = {"f64": _native.SG_F64, "f32": _native.SG_F32}[precision]
        self.dt = np.float64 if self.prec == _native.SG_F64 else np.float32
        self.t_max, self.bp_dectype, self.bp_its = int(t_max), bp_dectype, int(bp_its)
        self.design = DenseDesign(A, P, L, M, n=n, seed=design_seed)
        self.plan = self.design.plan(self.prec)
        self.graph = self.c._device_graph()
        self.snp = float(np.sqrt(n * P / L))
        self._cap = 0

    def _ensure(self, B):
        if B <= self._cap:
            return
        c, sz = self.c, np.dtype(self.dt).itemsize
        self.d_y = _native.DeviceBuffer(B * self.n * sz)
        self.d_x = _native.DeviceBuffer(B * self.n * sz)
        self.d_idx = _native.DeviceBuffer(B * self.L * 4)
        self.d_true = _native.DeviceBuffer(B * self.L * 4)
        self.d_llr = _native.DeviceBuffer(B * self.mults * c.N * sz)
        self.d_app = _native.DeviceBuffer(B * self.mults * c.N * sz)
        self.d_it = _native.DeviceBuffer(B * self.mults * 4)
        self.d_info = _native.DeviceBuffer(B * self.mults * c.K)
        self.d_unp = _native.DeviceBuffer(max(1, B * self.L_unp * self.logM))
        self.d_cw = _native.DeviceBuffer(B * self.mults * c.N)
        self.d_cnt = _native.DeviceBuffer(5 * 8)
        self._cap = B

    def make_batch(self, B, awgn_var, rng):
        """Random user bits -> LDPC blocks -> section indices; x = A beta0 on
        the GPU; y = x + AWGN (host RNG).  Leaves y, the true indices and the
        information bits resident on the device."""
        self._ensure(B)
        c, logM = self.c, self.logM
        unp = rng.integers(0, 2, (B, self.L_unp * logM))
        info = rng.integers(0, 2, (B * self.mults, c.K))
        cw = c.encode_batch(info).reshape(B, self.mults * c.N)
        bits = np.concatenate([unp, cw], axis=1).reshape(B, self.L, logM)
        idx = (bits.astype(np.int64) @ (1 << np.arange(logM)[::-1])).astype(np.int32)
        self.d_true.upload(idx)
        self.d_info.upload(info.reshape(B, -1).astype(np.uint8))
        lib = _native.lib()
        _native.check(lib.sg_dense_encode_device(self.plan, self.d_true.ptr, B, self.d_x.ptr, None))
        x = self.d_x.download(np.empty((B, self.n), self.dt))
        y = (x + np.sqrt(awgn_var) * rng.standard_normal(x.shape)).astype(self.dt)
        self.d_y.upload(y)
        self.B = B
        return idx, info

    # distinct Philox keys of the parts of a device batch
    _SEED_INFO = 0x5DEECE66D

    def make_batch_device(self, B, awgn_var, seed, stream_id):
        """The same batch generated on the GPU (throughput mode, nothing from
        the host): Philox user bits of the unprotected sections and of the
        LDPC information words (sparc_new.py:15-51), the systematic LDPC
        encoder (ldpc.py:400-460) on the device, MSB-first bits -> section
        indices, x = A beta0, y = x + AWGN.  The draw of codeword b depends only
        on (seed, stream_id, b): a Monte-Carlo block keyed by (point, block) is
        the same whatever the rank count."""
        self._ensure(B)
        c, logM, lib = self.c, self.logM, _native.lib()
        off = _native.offset
        nu = self.L_unp * logM
        if nu:
            _native.check(lib.sg_rng_bits_device(seed, stream_id, B, nu, self.d_unp.ptr, None))
            _native.check(lib.sg_bits_to_sections_strided_device(self.d_unp.ptr, nu, B, self.L_unp, logM,
                                                                 self.d_true.ptr, self.L, None))
        _native.check(lib.sg_rng_bits_device(seed ^ self._SEED_INFO, stream_id, B * self.mults, c.K, self.d_info.ptr,
                                             None))
        c.encode_device(self.d_info.ptr, B * self.mults, self.d_cw.ptr)
        _native.check(lib.sg_bits_to_sections_strided_device(self.d_cw.ptr, self.mults * c.N, B, self.L - self.L_unp,
                                                             logM, off(self.d_true.ptr, 4 * self.L_unp), self.L, None))
        _native.check(lib.sg_dense_encode_device(self.plan, self.d_true.ptr, B, self.d_x.ptr, None))
        _native.check(lib.sg_awgn_device(self.prec, seed, stream_id, self.d_x.ptr, B, self.n,
                                         float(np.sqrt(awgn_var)), self.d_y.ptr, None))
        self.B = B

    def decode(self):
        """One batch: returns nothing; counters accumulate in d_cnt."""
        lib, c, B = _native.lib(), self.c, self.B
        _native.check(lib.sg_dense_amp_device(self.plan, self.d_y.ptr, B, self.t_max, None, None, None))
        d_beta, d_s = ct.c_void_p(), ct.c_void_p()
        _native.check(lib.sg_dense_state_device(self.plan, ct.byref(d_beta), ct.byref(d_s)))
        _native.check(lib.sg_dense_map_device(self.plan, d_s, B, self.d_idx.ptr, None))
        ld = self.mults * c.N
        _native.check(lib.sg_beta_to_llr_device(self.prec, d_beta, B, self.L, self.M, self.snp, self.L_unp,
                                                self.L - self.L_unp, ld, 0, self.d_llr.ptr, None))
        _native.check(lib.sg_ldpc_decode_device(self.graph, _native.DECTYPES[self.bp_dectype], self.prec,
                                                self.d_llr.ptr, B * self.mults, self.bp_its, 0.7, self.d_app.ptr,
                                                self.d_it.ptr, None))
        _native.check(lib.sg_concat_count_errors_device(self.prec, self.d_idx.ptr, self.d_true.ptr, B, self.L,
                                                        self.L_unp, self.logM, self.d_app.ptr, self.d_info.ptr,
                                                        self.mults, c.N, c.K, self.d_cnt.ptr, None))

    def reset_counts(self):
        self.d_cnt.zero()

    def counts(self):
        _native.synchronize()
        return self.d_cnt.download(np.zeros(5, np.int64))
