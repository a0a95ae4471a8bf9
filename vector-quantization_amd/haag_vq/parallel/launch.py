"""One process per GPU for the command-line callers (`vq-benchmark sweep / streaming-sweep
--gpus N`), SURVEY.md §8e.

``launch_ranks`` starts ``python -m torch.distributed.run --nproc-per-node N -m haag_vq ...``
as a CHILD process of the calling command (never an exec, and before anything in the caller
touches the GPU) and returns its exit code.  Inside the ranks, ``init_rank`` joins the process
group and picks the rank's device: backend "nccl" (RCCL over xGMI) when a GPU is present,
"gloo" otherwise or when ``$VQ_DIST_BACKEND`` says so (the one-GPU tests run two ranks on one
card with gloo); rank r takes ``cuda:(LOCAL_RANK % device_count)``.
"""

from __future__ import annotations

import os
import socket
import subprocess
import sys
from dataclasses import dataclass
from datetime import timedelta
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class RankInfo:
    rank: int
    world: int
    local_rank: int
    backend: Optional[str]
    device: Optional[torch.device]


def launched_world() -> int:
    """WORLD_SIZE of torch.distributed.run (1 outside it)."""
    return int(os.environ.get("WORLD_SIZE", "1"))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_command(gpus: int, module_args: List[str], port: Optional[int] = None) -> List[str]:
    """The child command line: torch.distributed.run over 127.0.0.1 running ``python -m haag_vq``."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(gpus)}",
            "--master-addr=127.0.0.1", f"--master-port={port or free_port()}",
            # "--" ends torchrun's options: flags of ours that abbreviate one of its options
            # (e.g. --n, --d) would otherwise be rejected as ambiguous
            "-m", "--", "haag_vq"] + list(module_args)


def launch_ranks(gpus: int, module_args: List[str], extra_env: Optional[dict] = None) -> int:
    """Runs ``haag_vq <module_args>`` on ``gpus`` ranks as a child process; returns its exit code."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this platform
    env.setdefault("OMP_NUM_THREADS", "1")
    pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env.update(extra_env or {})
    cmd = rank_command(gpus, module_args)
    print(f"[launcher] {' '.join(cmd)}", flush=True)
    return subprocess.call(cmd, env=env)


# Ranks of the CLI callers wait in collectives while another rank trains or runs a longer
# configuration (streaming-sweep: ranks 1..N-1 wait in the quantizer broadcast while rank 0 fits
# on 1M rows): the default 10-minute watchdog would abort them
RANK_TIMEOUT = timedelta(hours=12)


def init_rank(device_index: Optional[int] = None, collectives: bool = True) -> RankInfo:
    """Joins the process group of torch.distributed.run (no-op at world size 1).  A single
    process runs on ``device_index`` (default: the current device).  ``collectives=False``
    (``sweep --gpus N``, which only deals configurations by RANK / WORLD_SIZE) picks the rank's
    device and opens no process group at all."""
    world = launched_world()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    has_gpu = torch.cuda.is_available()
    device = None
    if has_gpu:
        if world > 1:
            idx = local % max(1, torch.cuda.device_count())
        else:
            idx = torch.cuda.current_device() if device_index is None else int(device_index)
        device = torch.device("cuda", idx)
        torch.cuda.set_device(device)
    backend = None
    if world > 1 and collectives:
        backend = os.environ.get("VQ_DIST_BACKEND") or ("nccl" if has_gpu else "gloo")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device, timeout=RANK_TIMEOUT)
        else:
            dist.init_process_group(backend, timeout=RANK_TIMEOUT)
    return RankInfo(rank, world, local, backend, device)


def finish_rank(info: RankInfo) -> None:
    if info.world > 1 and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def comm_device(info: RankInfo) -> torch.device:
    """Where collective buffers live: the GPU under nccl, the host under gloo."""
    return info.device if info.backend == "nccl" else torch.device("cpu")
