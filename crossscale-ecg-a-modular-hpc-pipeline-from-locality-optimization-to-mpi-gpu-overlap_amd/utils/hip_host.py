"""Host-side HIP runtime settings applied through the runtime torch itself mapped (never a second copy).

``spin_sync_flag`` sets ``hipDeviceScheduleSpin`` (host waits spin instead of yielding) on the HIP runtime this process
has mapped - torch's ``torch/lib/libamdhip64.so`` - opened with RTLD_NOLOAD, and reads the flags back with
``hipGetDeviceFlags``; call it before the device is initialised.  Used by the Module-2 single-call timings
(bench/module2.py, ``ECG_M2_SPIN``).  Measured for bench.py's K=20 region too (a spin-waiting closing synchronize):
11.43-11.56 vs 11.42-11.48 us/step, no gain (profiles/r6/tiny_step_pmc.txt) - bench.py keeps the runtime default.
"""
from __future__ import annotations

import os
from typing import Dict


def _loaded_hip_runtime() -> str | None:
    """Path of the HIP runtime this process has mapped (torch's, torch/lib/libamdhip64.so.*), from /proc/self/maps."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                i = line.find("/")
                if i >= 0 and "libamdhip64.so" in line[i:]:
                    return line[i:].strip()
    except OSError:
        pass
    return None


def spin_sync_flag() -> Dict[str, object]:
    """``hipSetDeviceFlags(hipDeviceScheduleSpin)`` through the HIP runtime torch already loaded (RTLD_NOLOAD on
    the mapped path: never a second runtime whose flags torch would not see), read back with ``hipGetDeviceFlags``.
    ``torch.cuda.synchronize()`` then spins instead of yielding the CPU, as the HIP op's own completion wait already
    does (host-flag spin), so both sides of a single-call timing pay the same wake-up cost."""
    import ctypes
    rec: Dict[str, object] = {"spin_sync": False, "hip_runtime": None, "device_flags": None}
    path = _loaded_hip_runtime()
    rec["hip_runtime"] = path
    if path is None:
        return rec
    try:
        hip = ctypes.CDLL(path, mode=os.RTLD_NOLOAD | ctypes.RTLD_GLOBAL)
    except OSError as e:
        rec["error"] = repr(e)[:120]
        return rec
    st = hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
    flags = ctypes.c_uint(0)
    if hip.hipGetDeviceFlags(ctypes.byref(flags)) == 0:
        rec["device_flags"] = int(flags.value)
    rec["set_status"] = int(st)
    rec["spin_sync"] = rec["device_flags"] is not None and (rec["device_flags"] & 0x7) == 1
    return rec
