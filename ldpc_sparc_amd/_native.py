"""ctypes binding of libldpc_sparc_amd.so (the C ABI in include/ldpc_sparc_amd.h).

This is the only way the Python host layer reaches the GPU.  There is no CPU
fallback: if the library is missing or no GPU is visible, every decode raises.
"""
import ctypes as ct
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LDPC_SPARC_AMD_LIB", os.path.join(_HERE, "_lib", "libldpc_sparc_amd.so"))

SG_SUMPROD, SG_SUMPROD2, SG_MINSUM = 0, 1, 2
SG_F64, SG_F32 = 0, 1
DECTYPES = {"sumprod": SG_SUMPROD, "sumprod2": SG_SUMPROD2, "minsum": SG_MINSUM}

_lib = None

dp = ct.POINTER(ct.c_double)
lp = ct.POINTER(ct.c_long)
vp = ct.c_void_p


class NativeError(RuntimeError):
    pass


def _sig(lib, name, restype, argtypes):
    f = getattr(lib, name)
    f.restype = restype
    f.argtypes = argtypes
    return f


# (name, restype, argtypes) of every symbol include/ldpc_sparc_amd.h declares.
SIGNATURES = [
    ("sg_last_error", ct.c_char_p, []),
    ("sg_version", ct.c_char_p, []),
    ("sg_device_count", ct.c_int, [ct.POINTER(ct.c_int)]),
    ("sg_device_cu_count", ct.c_int, [ct.POINTER(ct.c_int)]),
    ("sg_set_device", ct.c_int, [ct.c_int]),
    ("sg_get_stream", ct.c_int, [ct.POINTER(vp)]),
    ("sg_malloc", ct.c_int, [ct.POINTER(vp), ct.c_size_t]),
    ("sg_free", ct.c_int, [vp]),
    ("sg_memcpy_h2d", ct.c_int, [vp, vp, ct.c_size_t, vp]),
    ("sg_memcpy_d2h", ct.c_int, [vp, vp, ct.c_size_t, vp]),
    ("sg_memset", ct.c_int, [vp, ct.c_int, ct.c_size_t, vp]),
    ("sg_stream_create", ct.c_int, [vp]),
    ("sg_stream_destroy", ct.c_int, [vp]),
    ("sg_stream_synchronize", ct.c_int, [vp]),
    ("sg_event_create", ct.c_int, [ct.POINTER(vp)]),
    ("sg_event_destroy", ct.c_int, [vp]),
    ("sg_event_record", ct.c_int, [vp, vp]),
    ("sg_event_elapsed_ms", ct.c_int, [vp, vp, ct.POINTER(ct.c_float)]),
    ("sg_ldpc_graph_create", ct.c_int, [vp, vp, vp, ct.c_int, ct.c_int, ct.c_int, ct.POINTER(vp)]),
    ("sg_ldpc_graph_destroy", ct.c_int, [vp]),
    ("sg_ldpc_graph_info", ct.c_int, [vp] + [ct.POINTER(ct.c_int)] * 5),
    ("sg_ldpc_decode_kernel", ct.c_int, [vp, ct.c_int, ct.c_int, ct.c_char_p, ct.c_size_t]),
    ("sg_ldpc_grouped_layout", ct.c_int, [vp, vp, vp, ct.c_int, ct.c_int, ct.c_int, ct.c_int, vp, vp, ct.c_int, vp,
                                          ct.c_int, vp, ct.c_int]),
    ("sg_ldpc_decode", ct.c_int, [vp, ct.c_int, ct.c_int, vp, ct.c_int, ct.c_int, ct.c_double, vp, vp]),
    ("sg_ldpc_decode_device", ct.c_int,
     [vp, ct.c_int, ct.c_int, vp, ct.c_int, ct.c_int, ct.c_double, vp, vp, vp]),
    ("sg_ldpc_codeword_errors_device", ct.c_int, [vp, ct.c_int, vp, vp, ct.c_int, vp, vp]),
    ("sg_ldpc_count_errors_device", ct.c_int,
     [vp, ct.c_int, vp, vp, vp, ct.c_int, ct.c_int, vp, vp]),
    ("sumprod", ct.c_int, [dp, lp, lp, lp, ct.c_int, ct.c_int, ct.c_int, dp, ct.c_int]),
    ("sumprod2", ct.c_int, [dp, lp, lp, lp, ct.c_int, ct.c_int, ct.c_int, dp, ct.c_int]),
    ("minsum", ct.c_int, [dp, lp, lp, lp, ct.c_int, ct.c_int, ct.c_int, dp, ct.c_double, ct.c_int]),
    ("Lxor", ct.c_double, [ct.c_double, ct.c_double, ct.c_int]),
    ("sg_amp_plan_create", ct.c_int, [ct.c_int, vp, ct.c_int, ct.c_int, ct.c_int, ct.c_int, ct.c_int,
                                      vp, vp, ct.c_int, ct.POINTER(vp)]),
    ("sg_amp_plan_destroy", ct.c_int, [vp]),
    ("sg_amp_plan_info", ct.c_int, [vp] + [ct.POINTER(ct.c_int)] * 6),
    ("sg_amp_plan_engine", ct.c_int, [vp, ct.c_int]),
    ("sg_amp_last_decode", ct.c_int, [vp, ct.POINTER(ct.c_int), ct.POINTER(ct.c_int), ct.POINTER(ct.c_int)]),
    ("sg_amp_decode", ct.c_int, [vp, vp, ct.c_int, vp, ct.c_double, ct.c_int, ct.c_double, ct.c_int,
                                 vp, vp, vp, vp]),
    ("sg_amp_decode_device", ct.c_int, [vp, vp, ct.c_int, vp, ct.c_double, ct.c_int, ct.c_double,
                                        ct.c_int, vp, vp, vp, vp, vp]),
    ("sg_amp_apply", ct.c_int, [vp, ct.c_int, vp, ct.c_int, vp]),
    ("sg_amp_apply_device", ct.c_int, [vp, ct.c_int, vp, ct.c_int, vp, vp]),
    ("sg_amp_count_errors_device", ct.c_int, [vp, vp, vp, ct.c_int, ct.c_int, ct.c_int, vp, vp]),
    ("sg_section_softmax", ct.c_int, [vp, ct.c_int, ct.c_int, ct.c_double, vp]),
    ("sg_section_argmax", ct.c_int, [vp, ct.c_int, ct.c_int, vp]),
    ("Lxfb", ct.c_double, [dp, ct.c_long, ct.c_int]),
    ("sg_device_synchronize", ct.c_int, []),
    ("sg_profile_enable", ct.c_int, [ct.c_int]),
    ("sg_profile_collect", ct.c_int, [vp, vp]),
    ("sg_phase_name", ct.c_char_p, [ct.c_int]),
    ("sg_comm_unique_id", ct.c_int, [vp]),
    ("sg_comm_init", ct.c_int, [ct.c_int, ct.c_int, vp, ct.POINTER(vp)]),
    ("sg_comm_allreduce_sum_i64", ct.c_int, [vp, vp, ct.c_size_t, vp]),
    ("sg_comm_info", ct.c_int, [vp, ct.POINTER(ct.c_int), ct.POINTER(ct.c_int)]),
    ("sg_comm_destroy", ct.c_int, [vp]),
    ("sg_dense_plan_create", ct.c_int, [vp, ct.c_int, ct.c_int, ct.c_int, ct.c_double, ct.c_int,
                                        ct.POINTER(vp)]),
    ("sg_dense_plan_create_random", ct.c_int, [ct.c_int, ct.c_int, ct.c_int, ct.c_double, ct.c_uint64,
                                               ct.c_int, ct.POINTER(vp)]),
    ("sg_dense_plan_destroy", ct.c_int, [vp]),
    ("sg_dense_plan_info", ct.c_int, [vp] + [ct.POINTER(ct.c_int)] * 4),
    ("sg_dense_amp", ct.c_int, [vp, vp, ct.c_int, ct.c_int, vp, vp]),
    ("sg_dense_amp_device", ct.c_int, [vp, vp, ct.c_int, ct.c_int, vp, vp, vp]),
    ("sg_dense_amp_iteration", ct.c_int, [vp, vp, vp, vp, ct.c_double, vp, vp, vp]),
    ("sg_dense_encode_device", ct.c_int, [vp, vp, ct.c_int, vp, vp]),
    ("sg_dense_map_device", ct.c_int, [vp, vp, ct.c_int, vp, vp]),
    ("sg_dense_state_device", ct.c_int, [vp, ct.POINTER(vp), ct.POINTER(vp)]),
    ("sg_dense_plan_matrix_device", ct.c_int, [vp, ct.POINTER(vp)]),
    ("sg_concat_count_errors_device", ct.c_int, [ct.c_int, vp, vp, ct.c_int, ct.c_int, ct.c_int, ct.c_int, vp, vp,
                                                 ct.c_int, ct.c_int, ct.c_int, vp, vp]),
    ("sg_beta_to_llr_device", ct.c_int, [ct.c_int, vp, ct.c_int, ct.c_int, ct.c_int, ct.c_double, ct.c_int,
                                         ct.c_int, ct.c_int, ct.c_int, vp, vp]),
    ("sg_amp_encode_device", ct.c_int, [vp, vp, ct.c_int, vp, vp]),
    ("sg_amp_stage_profile", ct.c_int, [vp, ct.c_int, vp, vp]),
    ("sg_amp_stage_raw", ct.c_int, [vp, ct.c_int, vp, vp]),
    # device encoder and channel
    ("sg_rng_bits_device", ct.c_int, [ct.c_uint64, ct.c_uint64, ct.c_int, ct.c_int, vp, vp]),
    ("sg_bits_to_sections_strided_device", ct.c_int,
     [vp, ct.c_size_t, ct.c_int, ct.c_int, ct.c_int, vp, ct.c_size_t, vp]),
    ("sg_bits_to_sections_device", ct.c_int, [vp, ct.c_int, ct.c_int, ct.c_int, vp, vp]),
    ("sg_awgn_device", ct.c_int, [ct.c_int, ct.c_uint64, ct.c_uint64, vp, ct.c_int, ct.c_int, ct.c_double, vp, vp]),
    ("sg_bpsk_awgn_llr_device", ct.c_int, [ct.c_int, ct.c_uint64, ct.c_uint64, vp, ct.c_int, ct.c_int, ct.c_double,
                                           vp, vp]),
    ("sg_ldpc_encoder_create", ct.c_int, [vp, ct.c_int, ct.c_int, vp]),
    ("sg_ldpc_encoder_destroy", ct.c_int, [vp]),
    ("sg_ldpc_encode_device", ct.c_int, [vp, vp, ct.c_int, vp, vp]),
    # state evolution
    ("sg_se_samples_create", ct.c_int, [vp, ct.c_int, ct.c_int, vp]),
    ("sg_se_samples_destroy", ct.c_int, [vp]),
    ("sg_se_expectation", ct.c_int, [vp, ct.c_int, vp, ct.c_int, vp]),
    # integrated AMP <-> BP decoders
    ("sg_integrated_decode", ct.c_int, [vp, vp, ct.c_int, ct.c_int, vp, ct.c_int, ct.c_int, ct.c_int, ct.c_int,
                                        vp, vp]),
    ("sg_integrated_decode_device", ct.c_int, [vp, vp, ct.c_int, ct.c_int, vp, ct.c_int, ct.c_int, ct.c_int,
                                               ct.c_int, vp, vp, vp]),
    ("sg_bp_output_to_beta", ct.c_int, [ct.c_int, vp, ct.c_int, ct.c_int, ct.c_int, ct.c_double, vp]),
    ("sg_update_using_bp_probs", ct.c_int, [ct.c_int, vp, vp, ct.c_int, ct.c_int, ct.c_int, ct.c_double, vp]),
    ("sg_differentiated_eta", ct.c_int, [ct.c_int, ct.c_int, vp, vp, vp, vp, vp, vp, ct.c_int, ct.c_int, ct.c_int,
                                         ct.c_double, vp]),
]

SG_INT_NAIVE, SG_INT_NAIVE_POST, SG_INT_DIFF, SG_INT_DIFF_POST = 0, 1, 2, 3
INTEGRATED_MODES = {"naive": SG_INT_NAIVE, "naive_posteriors": SG_INT_NAIVE_POST, "integrated": SG_INT_DIFF,
                    "integrated_posteriors": SG_INT_DIFF_POST}

SG_PH_COUNT = 12


def lib():
    """Load the shared library (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"{LIB_PATH} not found: build it with `make -C ldpc_sparc_amd/csrc` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        L = ct.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            _sig(L, name, res, args)
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        msg = lib().sg_last_error().decode(errors="replace")
        raise NativeError(f"libldpc_sparc_amd error {rc}: {msg}")
    return rc


def device_count():
    n = ct.c_int(0)
    check(lib().sg_device_count(ct.byref(n)))
    return n.value


def cu_count():
    n = ct.c_int(0)
    check(lib().sg_device_cu_count(ct.byref(n)))
    return n.value


def require_gpu():
    if device_count() <= 0:
        raise NativeError("no GPU visible: ldpc_sparc_amd decodes only on MI355X (gfx950); "
                          "there is no CPU fallback")


def ptr(a):
    return ct.c_void_p(a.ctypes.data) if a is not None else ct.c_void_p(0)


def offset(p, nbytes):
    """Device pointer p (c_void_p) advanced by nbytes."""
    return ct.c_void_p((p.value or 0) + int(nbytes))


class DeviceBuffer:
    """A device allocation owned by Python (freed on GC)."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = ct.c_void_p()
        check(lib().sg_malloc(ct.byref(p), self.nbytes))
        self.ptr = p

    @classmethod
    def from_array(cls, arr, stream=None):
        arr = np.ascontiguousarray(arr)
        buf = cls(arr.nbytes)
        buf.upload(arr, stream)
        return buf

    def upload(self, arr, stream=None):
        arr = np.ascontiguousarray(arr)
        if arr.nbytes > self.nbytes:  # (a real check, not an assert: python -O must not drop it)
            raise ValueError(f"upload of {arr.nbytes} bytes into a {self.nbytes}-byte device buffer")
        check(lib().sg_memcpy_h2d(self.ptr, ptr(arr), arr.nbytes, stream))

    def download(self, out, stream=None):
        if not out.flags.c_contiguous or out.nbytes > self.nbytes:
            raise ValueError(f"download into a {'non-contiguous ' if not out.flags.c_contiguous else ''}"
                             f"{out.nbytes}-byte array from a {self.nbytes}-byte device buffer")
        check(lib().sg_memcpy_d2h(ptr(out), self.ptr, out.nbytes, stream))
        return out

    def zero(self, stream=None):
        check(lib().sg_memset(self.ptr, 0, self.nbytes, stream))

    def free(self):
        if self.ptr is not None and self.ptr.value:
            try:
                lib().sg_free(self.ptr)
            except Exception:
                pass
        self.ptr = None

    def __del__(self):
        self.free()


def synchronize(stream=None):
    check(lib().sg_stream_synchronize(stream))


def library_stream():
    s = ct.c_void_p()
    check(lib().sg_get_stream(ct.byref(s)))
    return s


class Event:
    def __init__(self):
        e = ct.c_void_p()
        check(lib().sg_event_create(ct.byref(e)))
        self.ev = e

    def record(self, stream=None):
        check(lib().sg_event_record(self.ev, stream))

    def elapsed_ms(self, later):
        ms = ct.c_float()
        check(lib().sg_event_elapsed_ms(self.ev, later.ev, ct.byref(ms)))
        return ms.value

    def __del__(self):
        try:
            lib().sg_event_destroy(self.ev)
        except Exception:
            pass


def device_synchronize():
    check(lib().sg_device_synchronize())


class Profiler:
    """Per-phase kernel timing through HIP events on the launch streams
    (sg_profile_enable / sg_profile_collect).  level 2: the split engine's
    per-iteration scope only, without events between its kernels."""

    def __init__(self, level=1):
        check(lib().sg_profile_enable(level))
        self.collect()  # drop anything recorded before

    def collect(self):
        ms = np.zeros(SG_PH_COUNT)
        n = np.zeros(SG_PH_COUNT, dtype=np.int64)
        check(lib().sg_profile_collect(ptr(ms), ptr(n)))
        return {lib().sg_phase_name(i).decode(): (float(ms[i]), int(n[i]))
                for i in range(SG_PH_COUNT) if n[i]}

    def stop(self):
        check(lib().sg_profile_enable(0))
        return self.collect()


class Comm:
    """RCCL communicator of this process (one process per GPU)."""

    ID_BYTES = 128

    @staticmethod
    def unique_id():
        buf = (ct.c_char * Comm.ID_BYTES)()
        check(lib().sg_comm_unique_id(ct.cast(buf, ct.c_void_p)))
        return bytes(buf)

    def __init__(self, nranks, rank, uid):
        if len(uid) != Comm.ID_BYTES:
            raise ValueError(f"RCCL unique id of {len(uid)} bytes, expected {Comm.ID_BYTES}")
        self._id = (ct.c_char * Comm.ID_BYTES).from_buffer_copy(uid)
        h = ct.c_void_p()
        check(lib().sg_comm_init(int(nranks), int(rank), ct.cast(self._id, ct.c_void_p), ct.byref(h)))
        self.h = h

    def allreduce_sum_i64(self, dbuf, count, stream=None):
        check(lib().sg_comm_allreduce_sum_i64(self.h, dbuf.ptr, int(count), stream))

    def info(self):
        """(ranks, device) of this communicator as RCCL reports them."""
        n, dev = ct.c_int(0), ct.c_int(-1)
        check(lib().sg_comm_info(self.h, ct.byref(n), ct.byref(dev)))
        return n.value, dev.value

    def destroy(self):
        if self.h is not None:
            lib().sg_comm_destroy(self.h)
            self.h = None


def amp_last_decode(plan):
    """What the last decode through `plan` ran: {"engine": 0 general / 1 staged /
    2 per-codeword / 3 block, "handover_iter": first staged iteration after the
    per-codeword engine (-1: none), "companion": ran on the P = 16384 plan}."""
    e, h, c = ct.c_int(-1), ct.c_int(-1), ct.c_int(0)
    check(lib().sg_amp_last_decode(plan, ct.byref(e), ct.byref(h), ct.byref(c)))
    return {"engine": e.value, "handover_iter": h.value, "companion": bool(c.value)}
