"""Utilities: CSV schemas, timing (hipEvent), logging, profiling ranges, checkpointing, config."""

import os as _os


def usable_cpus() -> int:
    """CPUs this process may actually use: OMP_NUM_THREADS if set, else the scheduler affinity mask
    (``os.cpu_count()`` reports the whole host, e.g. 256 cores on a GPU box limited to a 16-core share)."""
    env = _os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return max(1, len(_os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        return _os.cpu_count() or 1
