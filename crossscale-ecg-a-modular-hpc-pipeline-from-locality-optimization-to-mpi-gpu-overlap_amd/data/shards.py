"""Binary ECG shard format and shard assignment.

On-disk layout (little-endian, row-major), identical to the reference so shards are interchangeable:

    [int64 N][int64 L][float32 x N*L]

Reference parity:
  * ``write_shard``            <- Module_1/shard_prep.py:10-19
  * ``make_mitbih_windows``    <- Module_1/shard_prep.py:21-33
  * ``make_synth_windows``     <- Module_1/shard_prep.py:35-37
  * ``assign_shards_evenly``   <- Module_3/shard_dataset.py:9-27
  * ``load_shard``             <- Module_3/shard_dataset.py:30-47
  * ``get_shards_for_rank``    <- Module_3/part3_mpi_gpu_train.py:89-95

Differences (deliberate): ``load_shard`` can memory-map (zero-copy) instead of reading; a header/size
mismatch raises with the offending numbers; ``shard_header`` reads N, L without touching the payload.
"""
from __future__ import annotations

import os
from glob import glob
from typing import Iterable, List, Sequence, Tuple

import numpy as np

HEADER_BYTES = 16
SHARD_PATTERN = "ecg_*.bin"


def shard_name(shard_id: int) -> str:
    return f"ecg_{shard_id:05d}.bin"


def write_shard(path: str, windows_np: np.ndarray) -> int:
    """Write ``windows_np`` [N, L] as one shard. Returns the number of bytes written."""
    w = np.ascontiguousarray(windows_np, dtype=np.float32)
    if w.ndim != 2:
        raise ValueError(f"write_shard expects [N, L], got shape {w.shape}")
    n, l = w.shape
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "wb") as f:
        f.write(np.asarray([n, l], dtype="<i8").tobytes())
        w.astype("<f4", copy=False).tofile(f)
    return HEADER_BYTES + 4 * n * l


def shard_header(path: str) -> Tuple[int, int]:
    """Return (N, L) of a shard after validating the file size."""
    with open(path, "rb") as f:
        hdr = np.frombuffer(f.read(HEADER_BYTES), dtype="<i8")
    if hdr.size != 2:
        raise RuntimeError(f"Bad shard header in {path}")
    n, l = int(hdr[0]), int(hdr[1])
    expect = HEADER_BYTES + 4 * n * l
    size = os.path.getsize(path)
    if n < 0 or l <= 0 or size != expect:
        raise RuntimeError(f"Unexpected size in {path}: header N={n} L={l} wants {expect} B, file has {size} B")
    return n, l


def load_shard(path: str, mmap: bool = False) -> np.ndarray:
    """Read one shard as float32 [N, L]. ``mmap=True`` returns a read-only memory-mapped view."""
    n, l = shard_header(path)
    if mmap:
        return np.memmap(path, dtype="<f4", mode="r", offset=HEADER_BYTES, shape=(n, l))
    with open(path, "rb") as f:
        f.seek(HEADER_BYTES)
        data = np.fromfile(f, dtype="<f4", count=n * l)
    if data.size != n * l:
        raise RuntimeError(f"Unexpected size in {path}")
    return data.reshape(n, l)


def list_shards(root: str) -> List[str]:
    return sorted(glob(os.path.join(root, SHARD_PATTERN)))


def assign_shards_evenly(shard_paths: Sequence[str], world_size: int, rank: int) -> List[str]:
    """Round-robin shards over ranks (sorted order); a rank that gets none takes ``shards[rank % n]``."""
    if len(shard_paths) == 0:
        raise RuntimeError("No shards exist on disk.")
    if world_size <= 0 or not (0 <= rank < world_size):
        raise ValueError(f"bad rank/world_size: {rank}/{world_size}")
    shards = sorted(shard_paths)
    assigned = [s for i, s in enumerate(shards) if i % world_size == rank]
    if not assigned:
        assigned = [shards[rank % len(shards)]]
    return assigned


def get_shards_for_rank(rank: int, world_size: int, base_dir: str) -> List[str]:
    """Strided assignment ``paths[rank::world_size]`` (reference alt helper)."""
    paths = list_shards(base_dir)
    if not paths:
        raise RuntimeError(f"No shards found in {base_dir}")
    return paths[rank::world_size]


def make_synth_windows(N: int = 20000, L: int = 500, seed: int = 1337) -> np.ndarray:
    """Gaussian N(0,1) windows, same generator/seed semantics as the reference."""
    rng = np.random.default_rng(seed)
    return rng.normal(0, 1, size=(N, L)).astype(np.float32)


def make_mitbih_windows(records: Iterable[str] = ("100", "101", "103", "105", "106"),
                        win_len: int = 500, stride: int = 250, channel: int = 0) -> np.ndarray:
    """MIT-BIH windows via ``wfdb`` (needs the package and network; not available on the GPU pool)."""
    try:
        import wfdb  # type: ignore
    except Exception as e:  # pragma: no cover - wfdb is not installed in this image
        raise RuntimeError("wfdb not installed; use --dataset synthetic") from e
    xs = []
    for rid in records:  # pragma: no cover - needs network
        sig, _info = wfdb.rdsamp(f"mitdb/{rid}", pn_dir="mitdb")
        x = sig[:, channel].astype(np.float32)
        for start in range(0, len(x) - win_len, stride):
            xs.append(x[start:start + win_len])
    return np.stack(xs, axis=0).astype(np.float32)  # pragma: no cover


def write_shards(windows: np.ndarray, out_dir: str, shard_size: int = 32768) -> List[str]:
    """Split [N, L] windows into ``ecg_%05d.bin`` shards of ``shard_size`` windows."""
    if shard_size <= 0:
        raise ValueError("shard_size must be positive")
    paths = []
    n = windows.shape[0]
    i, sid = 0, 0
    while i < n:
        j = min(i + shard_size, n)
        p = os.path.join(out_dir, shard_name(sid))
        write_shard(p, windows[i:j])
        paths.append(p)
        i, sid = j, sid + 1
    return paths


def ensure_synthetic_shards(out_dir: str, n_windows: int, win_len: int = 500, shard_size: int = 32768,
                            seed: int = 1337) -> List[str]:
    """Create synthetic shards in ``out_dir`` unless matching ones already exist."""
    existing = list_shards(out_dir)
    if existing:
        total = 0
        ok = True
        for p in existing:
            try:
                n, l = shard_header(p)
            except RuntimeError:
                ok = False
                break
            ok &= (l == win_len)
            total += n
        if ok and total >= n_windows:
            return existing
        for p in existing:
            os.remove(p)
    return write_shards(make_synth_windows(n_windows, win_len, seed), out_dir, shard_size)
