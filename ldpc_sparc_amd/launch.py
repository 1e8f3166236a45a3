"""One process per GPU of one node, without PyTorch: starts `nproc` copies of
a Python script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR and the
rendezvous port (SG_RDZV_PORT, rendezvous.HostGroup) in their environment, and
exits with the first non-zero exit code (the other ranks are then stopped:
their exact PIDs, nothing matched by name).  The reference fans out the same
way, one process per sim_id (ldpc_jossy/py/ldpc_awgn.py:125-131).

  python -m ldpc_sparc_amd.launch --nproc 8 tools/c5_sweep.py --codewords 10000000

Nothing here touches the GPU: the parent holds no GPU state while the ranks
run.  torch.distributed.run remains usable as the launcher too (HostGroup then
finds rank 0 through a file in the temp directory)."""
import argparse
import os
import signal
import subprocess
import sys
import time

from .rendezvous import free_port


GRACE_S = 30.0


def spawn(nproc, cmd, env=None, addr="127.0.0.1"):
    """Run cmd (an argv list) as nproc ranks; returns the job's exit code."""
    base = dict(os.environ if env is None else env)
    port = free_port(addr)
    procs = []
    for r in range(nproc):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                 MASTER_ADDR=addr, MASTER_PORT=str(port), SG_RDZV_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=e))
    code = 0
    kill_at = None  # after a failure: SIGTERM to the others, SIGKILL to any still running GRACE_S later
    try:
        live = list(procs)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0 and code == 0:
                    code = rc if rc > 0 else 128 - rc  # killed by signal s: 128 + s, as a shell reports it
                    for q in live:  # a failed rank: the others would wait for it at the next rendezvous
                        q.send_signal(signal.SIGTERM)
                    kill_at = time.monotonic() + GRACE_S
            if kill_at is not None and time.monotonic() > kill_at:
                for q in live:
                    q.kill()
                kill_at = None
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return code


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, required=True)
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    sys.exit(spawn(a.nproc, [sys.executable, a.script] + a.args, addr=a.master_addr))


if __name__ == "__main__":
    main()
