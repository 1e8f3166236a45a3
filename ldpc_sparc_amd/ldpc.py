"""IEEE 802.11n / 802.16 QC-LDPC codes with a GPU belief-propagation decoder.

Drop-in for ldpc_jossy/py/ldpc.py: same class name `code`, constructor
arguments, attributes (N, K, Nv, Nc, Nmsg, vdeg, cdeg, intrlv, proto,
standard, rate, z, ptype), methods (assign_proto, pcmat, prepare_decoder,
encode, decode, Lxor, Lxfb), return types and NameError messages
(ldpc.py:4-503).  Decoding runs on the MI355X through libldpc_sparc_amd
(include/ldpc_sparc_amd.h); `decode_batch` / `encode_batch` are the batched
entry points the throughput paths use.
"""
import ctypes as ct
import json
import os

import numpy as np

from . import _native

_PROTO_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "protographs.json")
_PROTOS = None


def _protographs():
    global _PROTOS
    if _PROTOS is None:
        with open(_PROTO_FILE) as f:
            _PROTOS = json.load(f)
    return _PROTOS


def _shift(blocks, s):
    """Cyclic shift of z-blocks along the last axis: out[..., i] = blocks[..., (i + s) % z]
    (the permutation of a protograph entry with offset s, ldpc.py:298,426)."""
    return np.roll(blocks, -int(s), axis=-1)


class code:
    def __init__(self, standard='802.11n', rate='1/2', z=27, ptype='A'):
        self.standard = standard
        self.rate = rate
        self.z = z
        self.ptype = ptype
        self.proto = self.assign_proto()
        vdeg, cdeg, intrlv = self.prepare_decoder()
        self.vdeg = vdeg
        self.cdeg = cdeg
        self.intrlv = intrlv
        self.Nv = len(vdeg)
        self.Nc = len(cdeg)
        self.Nmsg = len(intrlv)
        self.N = self.Nv
        self.K = self.Nv - self.Nc
        self._graph = None
        self._graph_dev = None
        self._encoder = None

    # ------------------------------------------------------------ structure
    def assign_proto(self):
        """Protograph of the requested code (tables of ldpc.py:24-272)."""
        tables = _protographs()
        if self.standard == "802.16":
            by_rate = tables["802.16"]
            if self.rate not in by_rate:
                raise NameError('802.16 invalid rate')
            variants = by_rate[self.rate]
            if len(variants) > 1:
                if self.ptype not in variants:
                    raise NameError('802.16 type must be either A or B')
                proto = variants[self.ptype]
            else:
                proto = variants["A"]
        elif self.standard == "802.11n":
            key = str(self.z)
            if key not in tables["802.11n"] or not isinstance(self.z, (int, np.integer)):
                raise NameError('802.11n invalid z (must be 27,54 or 81)')
            by_rate = tables["802.11n"][key]
            if self.rate not in by_rate:
                raise NameError('802.11n invalid rate')
            proto = by_rate[self.rate]
        else:
            raise NameError('IEEE standard unknown')
        return np.array(proto)

    def pcmat(self):
        """Binary parity-check matrix expanded from the protograph (ldpc.py:275-300)."""
        z = self.z
        mp, np_ = self.proto.shape
        H = np.zeros((z * mp, z * np_), dtype=int)
        eye = np.eye(z, dtype=int)
        for r, c in zip(*np.nonzero(self.proto != -1)):
            H[r * z:(r + 1) * z, c * z:(c + 1) * z] = np.roll(eye, self.proto[r, c] % z, 1)
        return H

    def prepare_decoder(self):
        """Tanner graph in the reference decoder layout (ldpc.py:303-396).

        Every nonzero protograph entry (r, c) with offset s contributes, for
        k in [0, z), the edge check r*z+k <-> variable c*z+(k+s)%z.  Messages
        are check-ordered; the reference assigns ports in row-major order of
        the protograph, so the edge's port on the check is the rank of c
        among the nonzero columns of row r, and its port on the variable is
        the rank of r among the nonzero rows of column c.  `intrlv` maps
        variable-port index -> check-ordered message index (int32).
        """
        proto = self.proto
        z = self.z
        mask = proto != -1
        cdeg = np.repeat(np.sum(mask, 1), z)
        vdeg = np.repeat(np.sum(mask, 0), z)
        coff = np.concatenate(([0], np.cumsum(cdeg)))
        voff = np.concatenate(([0], np.cumsum(vdeg)))
        col_rank = np.cumsum(mask, axis=1) - 1   # rank of column within its row
        row_rank = np.cumsum(mask, axis=0) - 1   # rank of row within its column
        intrlv = np.empty(int(coff[-1]), dtype=np.int64)
        k = np.arange(z)
        for r, c in zip(*np.nonzero(mask)):
            chk = r * z + k
            var = c * z + (k + proto[r, c]) % z
            intrlv[voff[var] + row_rank[r, c]] = coff[chk] + col_rank[r, c]
        return vdeg, cdeg, intrlv.astype(np.int32)

    # ------------------------------------------------------------ encoder
    def encode(self, info):
        """Systematic QC encoder (ldpc.py:400-460): x[0:K] = info, parity by
        back-substitution through the dual-diagonal parity part."""
        z = self.z
        mp, np_ = self.proto.shape
        if len(info) != (np_ - mp) * z:
            raise NameError('information word length not compatible with proto and z')
        return self.encode_batch(np.asarray(info)[None, :])[0]

    def encode_batch(self, info):
        """Encode a [B, K] batch of information words -> [B, N] int codewords."""
        proto = self.proto
        z = self.z
        mp, np_ = proto.shape
        kp = np_ - mp
        info = np.asarray(info)
        if info.ndim != 2 or info.shape[1] != kp * z:
            raise NameError('information word length not compatible with proto and z')
        B = info.shape[0]
        u = (info.astype(np.int64) & 1).reshape(B, kp, z)
        # systematic contribution of every block row
        syn = np.zeros((B, mp, z), dtype=np.int64)
        for r in range(mp):
            for c in np.nonzero(proto[r, :kp] != -1)[0]:
                syn[:, r] ^= _shift(u[:, c], proto[r, c])
        # first parity block: the column-kp circulants add up to one shift t
        tcount = np.zeros(z, dtype=np.int64)
        for r in np.nonzero(proto[:, kp] != -1)[0]:
            tcount[proto[r, kp] % z] += 1
        tnz = np.nonzero(tcount % 2)[0]
        if len(tnz) != 1:
            raise NameError('The offsets in colum Kp+1 of proto do not add to a single offset')
        par = np.zeros((B, mp, z), dtype=np.int64)
        total = np.bitwise_xor.reduce(syn, axis=1)
        par[:, 0] = _shift(total, -int(tnz[0]))
        # remaining parity blocks, one block row at a time
        for r in range(mp - 1):
            acc = syn[:, r].copy()
            for c in np.nonzero(proto[r, kp:kp + r + 1] != -1)[0]:
                acc ^= _shift(par[:, c], proto[r, kp + c])
            par[:, r + 1] = acc
        x = np.concatenate([u, par], axis=1).reshape(B, np_ * z)
        return x.astype(int)

    # ------------------------------------------------------------ decoder
    def _device_graph(self):
        _native.require_gpu()
        if self._graph is None:
            L = _native.lib()
            v = np.ascontiguousarray(self.vdeg, dtype=np.int64)
            c = np.ascontiguousarray(self.cdeg, dtype=np.int64)
            i = np.ascontiguousarray(self.intrlv, dtype=np.int64)
            g = ct.c_void_p()
            _native.check(L.sg_ldpc_graph_create(_native.ptr(v), _native.ptr(c), _native.ptr(i),
                                                 self.Nv, self.Nc, self.Nmsg, ct.byref(g)))
            self._graph = g
        return self._graph

    def decode_kernel(self, dectype="minsum", precision=None):
        """Name of the GPU kernel decode_batch launches for this code (as
        rocprofv3 lists it): the degree-grouped min-sum kernel for
        single-precision min-sum on graphs it takes, else the table kernel."""
        prec = _native.SG_F32 if precision is None else precision
        buf = ct.create_string_buffer(128)
        _native.check(_native.lib().sg_ldpc_decode_kernel(self._device_graph(), _native.DECTYPES[dectype], prec, buf, 128))
        return buf.value.decode()

    def __del__(self):
        g = getattr(self, "_graph", None)
        if g is not None and g.value:
            try:
                _native.lib().sg_ldpc_graph_destroy(g)
            except Exception:
                pass
        e = getattr(self, "_encoder", None)
        if e is not None and e.value:
            try:
                _native.lib().sg_ldpc_encoder_destroy(e)
            except Exception:
                pass

    # ------------------------------------------------------------ device encoder
    def parity_generator(self):
        """[K, N-K] uint8: the encoder's parity bits of every unit information
        word (the encoder is GF(2)-linear and systematic, so cw = [u, u P])."""
        cw = self.encode_batch(np.eye(self.K, dtype=np.int64))
        assert np.array_equal(cw[:, :self.K], np.eye(self.K, dtype=int)), "encoder is not systematic"
        return np.ascontiguousarray(cw[:, self.K:], dtype=np.uint8)

    def _device_encoder(self):
        _native.require_gpu()
        if self._encoder is None:
            P = self.parity_generator()
            e = ct.c_void_p()
            _native.check(_native.lib().sg_ldpc_encoder_create(_native.ptr(P), self.K, self.N, ct.byref(e)))
            self._encoder = e
        return self._encoder

    def encode_device(self, d_info, B, d_cw, stream=None):
        """Encode B information words already on the GPU (uint8 [B, K]) into
        codewords (uint8 [B, N]) -- the throughput-mode encoder."""
        _native.check(_native.lib().sg_ldpc_encode_device(self._device_encoder(), d_info, int(B), d_cw, stream))

    def decode(self, ch, max_itcount=200, dectype='sumprod2', corr_factor=0.7):
        """Decode one codeword of channel LLRs (ldpc.py:463-490) on the GPU in
        double precision.  Returns (app float64[N], iterations)."""
        ch = np.asarray(ch, dtype=np.float64)
        if len(ch) != len(self.vdeg):
            raise NameError('Channel inputs not consistent with variable degrees')
        if dectype not in _native.DECTYPES:
            raise NameError('Decoder type unknonwn')
        app, it = self.decode_batch(ch[None, :], max_itcount, dectype, corr_factor)
        return app[0], int(it[0])

    def decode_batch(self, ch, max_itcount=200, dectype='sumprod2', corr_factor=0.7,
                     precision='f64'):
        """Decode a [B, N] batch of LLR vectors in one GPU launch.
        Returns (app float64[B, N], it int32[B])."""
        ch = np.ascontiguousarray(ch, dtype=np.float64)
        if ch.ndim != 2 or ch.shape[1] != self.Nv:
            raise NameError('Channel inputs not consistent with variable degrees')
        if dectype not in _native.DECTYPES:
            raise NameError('Decoder type unknonwn')
        prec = {'f64': _native.SG_F64, 'f32': _native.SG_F32}[precision]
        g = self._device_graph()
        B = ch.shape[0]
        app = np.zeros_like(ch)
        it = np.zeros(B, dtype=np.int32)
        _native.check(_native.lib().sg_ldpc_decode(
            g, _native.DECTYPES[dectype], prec, _native.ptr(ch), B, int(max_itcount),
            float(corr_factor), _native.ptr(app), _native.ptr(it)))
        return app, it

    def Lxor(self, L1, L2, corrflag=1):
        """LLR of the XOR of two bits (ldpc.py:492-495), evaluated on the GPU."""
        _native.require_gpu()
        return _native.lib().Lxor(float(L1), float(L2), int(corrflag))

    def Lxfb(self, L, corrflag=1):
        """Extrinsic LLRs of a parity constraint (ldpc.py:497-503): returns
        (aggregate, extrinsic array)."""
        _native.require_gpu()
        L = np.array(L, dtype=float)
        agg = _native.lib().Lxfb(L.ctypes.data_as(_native.dp), len(L), int(corrflag))
        return agg, L
