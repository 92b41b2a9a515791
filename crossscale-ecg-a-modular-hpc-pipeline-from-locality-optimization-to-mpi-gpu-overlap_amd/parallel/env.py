"""Process-group bring-up: torchrun env, MPI/Slurm launcher shim, one GPU per local rank.

Reference: ``comm = MPI.COMM_WORLD`` + ``setup_device() -> cuda:0`` (Module_3/part3_mpi_gpu_train.py:82-86,
433-437; TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py:60-65), one rank per node via ``srun``
(run_part3_sweep.sh:38-42).  MI355X design: one process per GPU on an 8-GPU node, ``torch.distributed``
backend ``"nccl"`` (== RCCL on ROCm, xGMI peer links), ``gloo`` on CPU.  ``mpiexec``/``srun`` keep
working: OMPI_COMM_WORLD_* / PMI_* / SLURM_* variables are mapped onto RANK/WORLD_SIZE/LOCAL_RANK, so
mpi4py is never needed.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

_MPI_MAP = [
    # (rank, world, local_rank)
    ("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK"),
    ("PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID"),
    ("PMIX_RANK", "PMIX_SIZE", "PMIX_LOCAL_RANK"),
    ("SLURM_PROCID", "SLURM_NTASKS", "SLURM_LOCALID"),
]


def apply_launcher_env_shim(env: Optional[dict] = None) -> Optional[str]:
    """If RANK/WORLD_SIZE are absent but an MPI/Slurm launcher set its own, translate them.

    Returns the name of the launcher family that was mapped (or None)."""
    env = os.environ if env is None else env
    if "RANK" in env and "WORLD_SIZE" in env:
        return None
    for rk, ws, lr in _MPI_MAP:
        if rk in env and ws in env:
            env["RANK"] = env[rk]
            env["WORLD_SIZE"] = env[ws]
            env["LOCAL_RANK"] = env.get(lr, "0")
            env.setdefault("MASTER_ADDR", env.get("SLURM_LAUNCH_NODE_IPADDR", "127.0.0.1"))
            env.setdefault("MASTER_PORT", "29511")
            return rk.split("_")[0]
    return None


@dataclass
class DistContext:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")
    initialized_here: bool = False

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1 and dist.is_available() and dist.is_initialized()


_CTX: Optional[DistContext] = None


def setup_device(local_rank: int = 0, prefer_gpu: bool = True, exclusive: bool = False) -> torch.device:
    """``cuda:{local_rank}`` when a GPU is present (reference always used cuda:0, one GPU per node).

    ``exclusive`` (RCCL ranks): every local rank needs a GPU of its own - more local ranks than GPUs is an
    error rather than two ranks silently sharing a device (RCCL would fail or hang).  Without it (gloo
    rehearsals) ranks wrap around the visible GPUs."""
    if prefer_gpu and torch.cuda.is_available():
        n = torch.cuda.device_count()
        if exclusive and local_rank >= n:
            raise RuntimeError(f"local rank {local_rank} has no GPU of its own ({n} visible); the nccl (RCCL) "
                               f"backend needs one GPU per rank - launch at most {n} ranks per node, or set "
                               f"ECG_DIST_BACKEND=gloo to rehearse several ranks on a shared GPU")
        dev = torch.device("cuda", local_rank % max(1, n))
        torch.cuda.set_device(dev)
        return dev
    return torch.device("cpu")


def init_distributed(backend: Optional[str] = None, timeout_s: float = 600.0, prefer_gpu: bool = True) -> DistContext:
    """Initialise (idempotently) the default process group from env; single process works without env."""
    global _CTX
    if _CTX is not None:
        return _CTX
    apply_launcher_env_shim()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:  # ECG_DIST_BACKEND=gloo rehearses several ranks on one shared GPU (RCCL needs 1 GPU/rank)
        backend = os.environ.get("ECG_DIST_BACKEND")
    gpu = prefer_gpu and torch.cuda.is_available()
    device = setup_device(local_rank, prefer_gpu, exclusive=world > 1 and gpu and backend in (None, "nccl"))
    if backend is None:
        backend = "nccl" if device.type == "cuda" else "gloo"
    ctx = DistContext(rank, world, local_rank, backend if world > 1 else "none", device)
    if world > 1 and dist.is_available() and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = device
            opts = nccl_pg_options()
            if opts is not None:
                kw["pg_options"] = opts
        dist.init_process_group(**kw)
        ctx.initialized_here = True
    elif world > 1 and dist.is_initialized():
        ctx.backend = dist.get_backend()
    _CTX = ctx
    return ctx


def nccl_pg_options():
    """RCCL process-group options: RCCL's internal stream from torch's HIGH-priority pool (``ECG_RCCL_HIGH_PRIORITY``,
    default 1).  Measured on MI355X (profiles/r6/stream_queues.txt): with the default normal-priority pool stream,
    RCCL's kernels landed on the SAME hardware queue as the compute (null) stream - HIP maps streams onto at most
    GPU_MAX_HW_QUEUES=4 queues per priority - so a collective ran only after every compute kernel enqueued before it
    (a 40 us all-reduce issued under a 1.7 ms compute kernel finished at 1.72 ms) and the comm stream behind it
    stalled too.  The high-priority pool maps onto separate queues (the comm stream's class), so the collective runs
    beside the compute kernels."""
    if os.environ.get("ECG_RCCL_HIGH_PRIORITY", "1") == "0":
        return None
    try:
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        return opts
    except (AttributeError, RuntimeError):  # a build without the NCCL process group
        return None


def get_context() -> DistContext:
    return _CTX if _CTX is not None else init_distributed()


def shutdown_distributed() -> None:
    global _CTX
    if _CTX is not None and _CTX.initialized_here and dist.is_initialized():
        dist.destroy_process_group()
    _CTX = None


def barrier(ctx: Optional[DistContext] = None) -> None:
    ctx = ctx or get_context()
    if ctx.distributed:
        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier()


# ----------------------------------------------------------------------------------- RCCL transport record
def rccl_init_log(directory: Optional[str] = None) -> Optional[str]:
    """Route RCCL's INIT-subsystem log to a per-process file, so the transport RCCL chose for every ring / tree
    channel (``via P2P/IPC`` over xGMI, ``via SHM``, ``via NET``) can be read back after the run
    (``rccl_transports``).  Must run before the first communicator is created; leaves a user's own NCCL_DEBUG
    setting alone (returns None then)."""
    if "NCCL_DEBUG" in os.environ:
        return None
    directory = directory or os.environ.get("TMPDIR", "/tmp")
    path = os.path.join(directory, f"ecg_rccl_init.{os.getpid()}.log")
    for k in _RCCL_LOG_VARS:
        _RCCL_ENV_PREV[k] = os.environ.get(k)
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ["NCCL_DEBUG_SUBSYS"] = "INIT"
    os.environ["NCCL_DEBUG_FILE"] = path
    return path


_RCCL_LOG_VARS = ("NCCL_DEBUG", "NCCL_DEBUG_SUBSYS", "NCCL_DEBUG_FILE")
_RCCL_ENV_PREV: dict = {}


def rccl_log_env_restore() -> None:
    """Put the NCCL_DEBUG* variables back as they were before ``rccl_init_log`` (call once the communicator exists:
    the eager ``device_id`` init creates it inside ``init_process_group``), so child processes do not inherit them."""
    for k, v in _RCCL_ENV_PREV.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    _RCCL_ENV_PREV.clear()


def rccl_log_remove(path: Optional[str]) -> None:
    """Delete the per-process INIT log once ``rccl_transports`` has read it."""
    if path:
        try:
            os.remove(path)
        except OSError:
            pass


def rccl_transports(path: Optional[str]) -> dict:
    """Count the channel connections per transport in an RCCL INIT log (``rccl_init_log``): e.g.
    ``{"P2P/IPC": 24}`` when every ring/tree neighbour is reached over xGMI peer-to-peer."""
    out: dict = {}
    if not path or not os.path.exists(path):
        return out
    import re
    pat = re.compile(r"\bvia (P2P/[\w ]+?|SHM(?:/\w+)?|NET/[\w/]+|NVLS|CollNet\w*)(?:\s|$|/read|/direct)")
    with open(path, errors="replace") as f:
        for line in f:
            m = pat.search(line)
            if m:
                key = m.group(1).strip()
                out[key] = out.get(key, 0) + 1
    return out


def peer_access(device: torch.device) -> list:
    """Per visible GPU j != this rank's: whether HIP reports direct peer access (xGMI) from ``device`` to j."""
    if device.type != "cuda":
        return []
    n = torch.cuda.device_count()
    return [bool(torch.cuda.can_device_access_peer(device.index, j)) for j in range(n) if j != device.index]
