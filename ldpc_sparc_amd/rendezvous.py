"""Host-side rendezvous of the ranks of one node, standard library only.

The reference's parallelism is independent processes, one per `sim_id`
(ldpc_jossy/py/ldpc_awgn.py:125-131); here the processes of one campaign (one
per GPU) meet once to exchange the RCCL unique id, to barrier around timed
regions and -- in CPU rehearsals, where several ranks share a GPU or there is
none -- to sum their int64 error counters.  The data-path collective itself is
RCCL (`_native.Comm`); this module carries only those few small host messages,
over TCP on the node, without PyTorch.

Every operation is an all-gather of one byte string per rank: rank 0 runs a
relay thread that reads one frame from each rank in rank order and answers
every rank with all of them, so results are identical on every rank and sums
are taken in rank order (deterministic).

Where the relay listens:
  * SG_RDZV_PORT set (bench.py's own launcher, the tests): that port on
    MASTER_ADDR;
  * else (ranks started by torch.distributed.run, whose agent already holds
    MASTER_PORT): rank 0 listens on a free port and publishes it in a file in
    the temp directory keyed by MASTER_ADDR, MASTER_PORT, the launcher's run id
    and the world size (one node: the ranks share the file system); the others
    read it and connect, and a handshake on the same key rejects a stale file's
    port.
"""
import hashlib
import json
import os
import socket
import struct
import tempfile
import threading
import time

import numpy as np

_HDR = struct.Struct("<Q")


def _send(so, b):
    so.sendall(_HDR.pack(len(b)) + b)


def _recv_exact(so, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = so.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(so):
    (n,) = _HDR.unpack(_recv_exact(so, _HDR.size))
    return _recv_exact(so, n)


class HostGroup:
    """The ranks of one node, for rendezvous, barriers and small host collectives."""

    def __init__(self, rank=None, world=None, addr=None, port=None, timeout=120.0):
        env = os.environ
        self.rank = int(env.get("RANK", "0")) if rank is None else int(rank)
        self.world = int(env.get("WORLD_SIZE", "1")) if world is None else int(world)
        self.addr = addr or env.get("MASTER_ADDR", "127.0.0.1")
        self.timeout = float(timeout)
        self._so = None
        self._relay = None
        if self.world <= 1:
            return
        if port is None and env.get("SG_RDZV_PORT"):
            port = int(env["SG_RDZV_PORT"])
        key_src = f"{self.addr}:{env.get('MASTER_PORT', '')}:{env.get('TORCHELASTIC_RUN_ID', '')}:{self.world}"
        self._key = hashlib.sha256(key_src.encode()).hexdigest()[:32].encode()
        self._file = None if port is not None else os.path.join(
            tempfile.gettempdir(), f"ldpc_sparc_amd_rdzv_{self._key.decode()}.port")
        if self.rank == 0:
            self._start_relay(port)
        self._connect(port)

    # ---------------------------------------------------------------- relay (rank 0)
    def _start_relay(self, port):
        if self._file and os.path.exists(self._file):
            os.unlink(self._file)
        srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        srv.bind((self.addr, port or 0))
        srv.listen(self.world + 8)
        self._port = srv.getsockname()[1]
        if self._file:
            tmp = f"{self._file}.{os.getpid()}"
            with open(tmp, "w") as f:
                f.write(str(self._port))
            os.replace(tmp, self._file)
        self._relay = threading.Thread(target=self._serve, args=(srv,), daemon=True)
        self._relay.start()

    def _serve(self, srv):
        conns = {}
        srv.settimeout(self.timeout)
        try:
            while len(conns) < self.world:
                c, _ = srv.accept()
                c.settimeout(1.0)  # a peer that connects and never says hello must not stall the relay
                try:
                    hello = json.loads(_recv(c))
                    ok = (isinstance(hello, dict) and hello.get("key") == self._key.decode()
                          and isinstance(hello.get("rank"), int) and 0 <= hello["rank"] < self.world)
                    _send(c, b"OK" if ok else b"NO")
                except (OSError, ConnectionError, ValueError):
                    c.close()
                    continue
                if ok:
                    c.settimeout(None)
                    old = conns.pop(int(hello["rank"]), None)  # a rank that retried: its newer connection
                    if old is not None:
                        old.close()
                    conns[int(hello["rank"])] = c
                else:
                    c.close()
        except OSError:  # the world never assembled: release the ranks that did connect
            for c in conns.values():
                c.close()
            return
        finally:
            srv.close()
        try:
            while True:
                frames = [_recv(conns[r]) for r in range(self.world)]
                reply = b"".join(_HDR.pack(len(f)) + f for f in frames)
                for r in range(self.world):
                    _send(conns[r], reply)
        except (ConnectionError, OSError):
            pass
        finally:
            for c in conns.values():
                c.close()

    # ---------------------------------------------------------------- every rank
    def _connect(self, port):
        deadline = time.monotonic() + self.timeout
        while True:
            p = port
            if p is None:
                try:
                    with open(self._file) as f:
                        p = int(f.read().strip() or "0")
                except (OSError, ValueError):
                    p = None
            if p:
                try:
                    # (the handshake keeps a timeout: a stale port file may name a port that some other server
                    # now holds, which would never answer; it is longer than the relay's 1 s per silent peer, so a
                    # rank does not give up -- and leave a half-registered connection behind -- while the relay
                    # is busy with another peer)
                    so = socket.create_connection((self.addr, p), timeout=5.0)
                    so.settimeout(15.0)
                    try:
                        _send(so, json.dumps({"key": self._key.decode(), "rank": self.rank}).encode())
                        ok = _recv(so) == b"OK"
                    except (OSError, ConnectionError):
                        ok = False
                    if ok:
                        so.settimeout(None)
                        so.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                        self._so = so
                        return
                    so.close()
                except (OSError, ConnectionError):
                    pass
            if time.monotonic() > deadline:
                raise TimeoutError(f"rank {self.rank}: no rendezvous with rank 0 at {self.addr} within "
                                   f"{self.timeout:.0f} s")
            time.sleep(0.05)

    def allgather_bytes(self, b):
        """One byte string from every rank, in rank order, on every rank."""
        if self.world <= 1:
            return [bytes(b)]
        _send(self._so, bytes(b))
        reply = _recv(self._so)
        out, o = [], 0
        for _ in range(self.world):
            (n,) = _HDR.unpack_from(reply, o)
            o += _HDR.size
            out.append(reply[o:o + n])
            o += n
        return out

    def barrier(self):
        self.allgather_bytes(b"")

    def bcast_bytes(self, b, src=0):
        return self.allgather_bytes(b if self.rank == src else b"")[src]

    def allgather_obj(self, obj):
        return [json.loads(x) for x in self.allgather_bytes(json.dumps(obj).encode())]

    def allreduce_sum_i64(self, counts):
        """Sum of int64 vectors over the ranks (in rank order)."""
        a = np.ascontiguousarray(counts, dtype=np.int64)
        parts = self.allgather_bytes(a.tobytes())
        out = np.zeros_like(a)
        for p in parts:
            out += np.frombuffer(p, dtype=np.int64).reshape(a.shape)
        return out

    def max(self, x):
        return max(struct.unpack("<d", p)[0] for p in self.allgather_bytes(struct.pack("<d", float(x))))

    def close(self):
        if self._so is not None:
            self._so.close()
            self._so = None
        if self._relay is not None:
            self._relay.join(5.0)
            self._relay = None
        if self._file and self.rank == 0:
            try:
                os.unlink(self._file)
            except OSError:
                pass


def free_port(addr="127.0.0.1"):
    with socket.socket() as so:
        so.bind((addr, 0))
        return so.getsockname()[1]
