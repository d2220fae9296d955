"""One process per GPU from a plain command line.

``python bench.py --gpus N`` (the driver's command) must run N ranks even without torchrun.  The
parent process therefore never touches HIP: it only starts ``python -m torch.distributed.run
--nproc-per-node N ... <script> <argv>`` as a CHILD process (never an exec of itself: a process
that has initialised the GPU must not be replaced), waits, and returns the child's exit code.
Each rank then reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the environment torchrun sets
and joins the process group over RCCL ("nccl"), or gloo in the CPU tests.

The reference has no multi-process path (its only parallelism is a dead ``nn.DataParallel``,
/root/reference/inference.py:209-210); this is the launcher for SURVEY §8(e)'s chunk sharding.
"""
import os
import socket
import subprocess
import sys


def free_port(addr="127.0.0.1"):
    with socket.socket() as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def needs_spawn(n_procs, env=None):
    """True when ``n_procs`` ranks are asked for and this process is not already one of them."""
    env = os.environ if env is None else env
    return int(n_procs) > 1 and "WORLD_SIZE" not in env


def spawn_world(n_procs, script, argv, extra_env=None, master_addr="127.0.0.1", port=None):
    """Run ``script argv`` as ``n_procs`` ranks under torch.distributed.run (127.0.0.1 rendezvous);
    returns the launcher's exit code (non-zero if any rank failed).  Rank output streams through."""
    env = dict(os.environ)
    env.update(extra_env or {})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this host driver
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(n_procs)}",
           f"--master-addr={master_addr}", f"--master-port={int(port or free_port(master_addr))}",
           script, *[str(a) for a in argv]]
    return subprocess.call(cmd, env=env)


def world_from_env():
    """(rank, local_rank, world) as torchrun exports them; (0, 0, 1) for a single process."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))
