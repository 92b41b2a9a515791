"""Per-rank CPU placement: bind each rank to CPUs of its own GPU's NUMA node.

Reference: every FedAvg client gets ``--cpus-per-task=4`` from Slurm (Module_3/TRUE_FL_M3/run_part3_sweep.sh:38-42).
On one 8-GPU MI355X node the eight ranks are launch-latency bound (a TinyECG step is ~11 µs of GPU work behind a
host-side graph launch), so a rank whose launch thread lands on a far socket, or shares a core with another rank,
turns into a straggler that the MAX-over-ranks timing exposes.  Each rank therefore pins itself, after it selected
its GPU, to a disjoint slice of the CPUs of that GPU's NUMA node:

    GPU PCI address (torch device properties) -> /sys/bus/pci/devices/<bdf>/numa_node
    -> /sys/devices/system/node/node<n>/cpulist  (intersected with the CPUs this process may use)
    -> the node's PHYSICAL cores (logical CPUs grouped by ``cpu<n>/topology/thread_siblings_list``)
    -> the GPUs on the same NUMA node split those cores into contiguous, equal slices (in PCI-address order);
       each rank gets every allowed hyper-thread of its own cores, so no two ranks share a core (on the usual
       EPYC numbering CPU n+128 is the SMT sibling of n: a split of the logical list ``0-63,128-191`` into four
       would have put rank 2 on the siblings of rank 0's cores).

The GPUs that share a node are taken from the KFD topology (``/sys/class/kfd/kfd/topology/nodes``: every GPU of
the machine, whatever ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` or ``srun --gpus-per-task=1`` let this
process see), so ranks that each see only their own GPU still get disjoint slices; only when the topology is
unreadable does the split fall back to the visible devices.  The basis used is part of the returned record.

Everything reads a ``sysfs`` root argument so the mapping is unit-tested on a fake tree.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional, Sequence, Tuple


def parse_cpulist(text: str) -> List[int]:
    """``"0-3,8,10-11"`` -> [0, 1, 2, 3, 8, 10, 11] (the sysfs cpulist format)."""
    cpus: List[int] = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            lo, hi = part.split("-", 1)
            cpus.extend(range(int(lo), int(hi) + 1))
        else:
            cpus.append(int(part))
    return sorted(set(cpus))


def format_cpulist(cpus: Iterable[int]) -> str:
    """Inverse of ``parse_cpulist`` (compact ranges)."""
    s = sorted(set(cpus))
    out, i = [], 0
    while i < len(s):
        j = i
        while j + 1 < len(s) and s[j + 1] == s[j] + 1:
            j += 1
        out.append(str(s[i]) if i == j else f"{s[i]}-{s[j]}")
        i = j + 1
    return ",".join(out)


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def numa_node_of(bdf: str, sysfs: str = "/sys") -> int:
    """NUMA node of a PCI device (-1 when unknown / single-node systems report -1)."""
    v = _read(os.path.join(sysfs, "bus", "pci", "devices", bdf, "numa_node"))
    try:
        return int(v.strip()) if v is not None else -1
    except ValueError:
        return -1


def node_cpus(node: int, sysfs: str = "/sys") -> List[int]:
    v = _read(os.path.join(sysfs, "devices", "system", "node", f"node{node}", "cpulist"))
    return parse_cpulist(v) if v else []


def core_groups(cpus: Sequence[int], sysfs: str = "/sys") -> List[List[int]]:
    """``cpus`` grouped by physical core (``thread_siblings_list``; a CPU without the file is its own core), each
    group sorted, groups ordered by their lowest CPU.  Siblings outside ``cpus`` are dropped."""
    want = set(cpus)
    seen, groups = set(), []
    for c in sorted(want):
        if c in seen:
            continue
        sib = _read(os.path.join(sysfs, "devices", "system", "cpu", f"cpu{c}", "topology", "thread_siblings_list"))
        g = sorted((set(parse_cpulist(sib)) & want) | {c}) if sib else [c]
        seen.update(g)
        groups.append(g)
    return sorted(groups, key=lambda g: g[0])


def plan_affinity(bdfs: Sequence[str], index: int, allowed: Iterable[int],
                  sysfs: str = "/sys") -> Tuple[int, List[int]]:
    """CPUs for the rank driving GPU ``bdfs[index]``: its NUMA node's CPUs (within ``allowed``) grouped into physical
    cores, the cores split into equal contiguous slices among the GPUs of ``bdfs`` on the same node, in list order;
    the rank gets both hyper-threads of each of its cores.  Returns (node, cpus); cpus is empty when nothing can be
    decided (unknown node, no allowed CPU on it)."""
    allowed = set(allowed)
    nodes = [numa_node_of(b, sysfs) for b in bdfs]
    node = nodes[index]
    if node < 0:
        return node, []
    cpus = [c for c in node_cpus(node, sysfs) if c in allowed]
    if not cpus:
        return node, []
    peers = [i for i, n in enumerate(nodes) if n == node]
    k, n_peers = peers.index(index), len(peers)
    cores = core_groups(cpus, sysfs)
    if len(cores) >= n_peers:  # whole cores per rank
        per = len(cores) // n_peers
        return node, sorted(c for g in cores[k * per:(k + 1) * per] for c in g)
    if len(cpus) < n_peers:  # fewer CPUs than ranks on this node: share the node's CPUs
        return node, cpus
    per = len(cpus) // n_peers  # fewer cores than ranks: ranks must share cores, split the threads
    return node, cpus[k * per:(k + 1) * per]


def kfd_gpu_bdfs(kfd_root: str = "/sys/class/kfd/kfd/topology/nodes") -> List[str]:
    """PCI addresses of EVERY GPU of the machine from the KFD topology (``gpu_id`` != 0; ``location_id`` =
    bus << 8 | device << 3 | function, ``domain``), sorted - independent of the *_VISIBLE_DEVICES masks."""
    out = []
    try:
        nodes = os.listdir(kfd_root)
    except OSError:
        return out
    for n in nodes:
        gid = _read(os.path.join(kfd_root, n, "gpu_id"))
        try:
            if gid is None or int(gid.strip() or 0) == 0:
                continue
        except ValueError:
            continue
        props = {}
        for line in (_read(os.path.join(kfd_root, n, "properties")) or "").splitlines():
            parts = line.split()
            if len(parts) == 2:
                props[parts[0]] = parts[1]
        try:
            loc, dom = int(props["location_id"]), int(props.get("domain", "0"))
        except (KeyError, ValueError):
            continue
        out.append(f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}")
    return sorted(set(out))


def device_bdfs() -> List[str]:
    """PCI addresses (``dddd:bb:dd.0``) of the visible GPUs, in device order (initialises the HIP runtime)."""
    import torch
    out = []
    for i in range(torch.cuda.device_count()):
        p = torch.cuda.get_device_properties(i)
        out.append(f"{int(getattr(p, 'pci_domain_id', 0)):04x}:{int(p.pci_bus_id):02x}:{int(p.pci_device_id):02x}.0")
    return out


def _set_process_affinity(cpus: Sequence[int]) -> None:
    """Apply the mask to every thread of the process (``sched_setaffinity(0)`` moves only the calling thread; the
    HIP runtime's own threads, started when the device was selected, would keep the old mask)."""
    os.sched_setaffinity(0, cpus)
    try:
        tids = [int(t) for t in os.listdir("/proc/self/task")]
    except OSError:
        return
    for t in tids:
        try:
            os.sched_setaffinity(t, cpus)
        except OSError:
            pass


def bind_to_gpu_numa(device_index: int, sysfs: str = "/sys", bdfs: Optional[Sequence[str]] = None,
                     kfd_root: str = "/sys/class/kfd/kfd/topology/nodes") -> Dict:
    """Pin this process to its slice of the CPUs of GPU ``device_index``'s NUMA node (``device_index`` indexes the
    VISIBLE devices, ``bdfs``).  The slice is planned over every GPU of the machine (KFD topology) so that ranks
    with narrowed visibility still split disjointly.  Returns a record {"numa_node", "cpus", "bound", "basis"} for
    the bench JSON; never raises (placement is a performance measure)."""
    rec: Dict = {"numa_node": -1, "cpus": "", "bound": False, "basis": "none"}
    try:
        allowed = os.sched_getaffinity(0)
        if bdfs is None:
            bdfs = device_bdfs()
        if not 0 <= device_index < len(bdfs):
            return rec
        mine = bdfs[device_index]
        every = kfd_gpu_bdfs(kfd_root)
        if mine in every:
            plan_bdfs, idx, rec["basis"] = every, every.index(mine), "kfd"
        else:  # topology unreadable (or a device it does not list): split among the visible GPUs
            plan_bdfs, idx, rec["basis"] = list(bdfs), device_index, "visible"
        node, cpus = plan_affinity(plan_bdfs, idx, allowed, sysfs)
        rec["numa_node"] = node
        if cpus:
            _set_process_affinity(cpus)
            rec["cpus"], rec["bound"] = format_cpulist(cpus), True
        else:
            rec["cpus"] = format_cpulist(allowed)
    except Exception as e:  # pragma: no cover - sysfs / affinity quirks must not break a run
        rec["error"] = repr(e)[:120]
    return rec
