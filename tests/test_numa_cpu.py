"""Per-rank NUMA placement (parallel/numa.py) on a fake sysfs tree: GPU PCI address -> numa_node -> the node's
cpulist, intersected with the allowed CPUs and split among the ranks whose GPUs share the node."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.parallel import numa  # noqa: E402


def _fake_sysfs(tmp_path, gpu_nodes, node_cpus):
    for bdf, node in gpu_nodes.items():
        d = tmp_path / "bus" / "pci" / "devices" / bdf
        d.mkdir(parents=True)
        (d / "numa_node").write_text(f"{node}\n")
    for node, cl in node_cpus.items():
        d = tmp_path / "devices" / "system" / "node" / f"node{node}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cl + "\n")
    return str(tmp_path)


def test_cpulist_roundtrip():
    assert numa.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert numa.format_cpulist([11, 10, 8, 3, 2, 1, 0]) == "0-3,8,10-11"
    assert numa.parse_cpulist("") == []


def test_eight_gpus_two_sockets(tmp_path):
    bdfs = [f"0000:{b:02x}:00.0" for b in (0x05, 0x15, 0x25, 0x35, 0x85, 0x95, 0xa5, 0xb5)]
    root = _fake_sysfs(tmp_path, {b: (0 if i < 4 else 1) for i, b in enumerate(bdfs)},
                       {0: "0-31,64-95", 1: "32-63,96-127"})
    allowed = range(128)
    plans = [numa.plan_affinity(bdfs, i, allowed, root) for i in range(8)]
    assert [p[0] for p in plans] == [0, 0, 0, 0, 1, 1, 1, 1]
    assert plans[0][1] == list(range(0, 16)) and plans[3][1] == list(range(80, 96))
    assert plans[4][1] == list(range(32, 48)) and plans[7][1] == list(range(112, 128))
    seen = [c for _, cpus in plans for c in cpus]
    assert len(seen) == len(set(seen)) == 128  # disjoint, complete


def test_allowed_set_and_unknown_node(tmp_path):
    bdfs = ["0000:05:00.0", "0000:15:00.0", "0000:25:00.0"]
    root = _fake_sysfs(tmp_path, {bdfs[0]: 0, bdfs[1]: 0, bdfs[2]: -1}, {0: "0-7"})
    node, cpus = numa.plan_affinity(bdfs, 1, [2, 3, 4, 5], root)  # container cpuset 2-5
    assert node == 0 and cpus == [4, 5]
    assert numa.plan_affinity(bdfs, 2, range(8), root) == (-1, [])  # single-node systems report -1
    assert numa.plan_affinity(bdfs, 0, [100], root) == (0, [])  # nothing allowed on the node


def test_bind_record_never_raises(tmp_path):
    rec = numa.bind_to_gpu_numa(5, sysfs=str(tmp_path), bdfs=["0000:05:00.0"])
    assert rec["bound"] is False and rec["numa_node"] == -1


def _fake_kfd(tmp_path, bdfs):
    root = tmp_path / "kfd"
    (root / "0").mkdir(parents=True)  # CPU node: gpu_id 0
    (root / "0" / "gpu_id").write_text("0\n")
    (root / "0" / "properties").write_text("cpu_cores_count 64\n")
    for i, b in enumerate(bdfs, start=1):
        dom, bus, rest = b.split(":")
        dev, fn = rest.split(".")
        loc = int(bus, 16) << 8 | int(dev, 16) << 3 | int(fn)
        d = root / str(i)
        d.mkdir()
        (d / "gpu_id").write_text(f"{1000 + i}\n")
        (d / "properties").write_text(f"simd_count 1024\nlocation_id {loc}\ndomain {int(dom, 16)}\n")
    return str(root)


def test_kfd_topology_lists_every_gpu(tmp_path):
    bdfs = [f"0000:{b:02x}:00.0" for b in (0xb5, 0x05, 0x85, 0x15)]
    assert numa.kfd_gpu_bdfs(_fake_kfd(tmp_path, bdfs)) == sorted(bdfs)
    assert numa.kfd_gpu_bdfs(str(tmp_path / "missing")) == []


def test_one_visible_gpu_per_rank_gets_disjoint_slices(tmp_path, monkeypatch):
    """4 ranks on one socket, each launched with one visible GPU (srun --gpus-per-task=1 / per-rank
    HIP_VISIBLE_DEVICES): the split is planned over the KFD topology, so the slices stay disjoint
    (advisor r4)."""
    bdfs = [f"0000:{b:02x}:00.0" for b in (0x05, 0x15, 0x25, 0x35, 0x85, 0x95, 0xa5, 0xb5)]
    root = _fake_sysfs(tmp_path, {b: (0 if i < 4 else 1) for i, b in enumerate(bdfs)},
                       {0: "0-31,64-95", 1: "32-63,96-127"})
    kfd = _fake_kfd(tmp_path, bdfs)
    applied = []
    monkeypatch.setattr(numa.os, "sched_getaffinity", lambda pid: set(range(128)))
    monkeypatch.setattr(numa, "_set_process_affinity", lambda cpus: applied.append(list(cpus)))
    recs = [numa.bind_to_gpu_numa(0, sysfs=root, bdfs=[bdfs[r]], kfd_root=kfd) for r in range(4)]
    assert all(r["bound"] and r["basis"] == "kfd" and r["numa_node"] == 0 for r in recs)
    assert [len(c) for c in applied] == [16] * 4
    seen = [c for cpus in applied for c in cpus]
    assert len(seen) == len(set(seen)) == 64  # disjoint quarters of socket 0
    # without a topology the same launch falls back to the visible device: every rank would take the whole node
    rec = numa.bind_to_gpu_numa(0, sysfs=root, bdfs=[bdfs[1]], kfd_root=str(tmp_path / "missing"))
    assert rec["basis"] == "visible" and len(applied[-1]) == 64


def _fake_siblings(tmp_path, n_phys, offset):
    """SMT pairs (c, c + offset) for c < n_phys, in the sysfs ``thread_siblings_list`` format."""
    for c in range(n_phys):
        for t in (c, c + offset):
            d = tmp_path / "devices" / "system" / "cpu" / f"cpu{t}" / "topology"
            d.mkdir(parents=True)
            (d / "thread_siblings_list").write_text(f"{c},{c + offset}\n")


def test_smt_siblings_never_split_across_ranks(tmp_path):
    """Node 0 = ``0-63,128-191`` with CPU n+128 the SMT sibling of n (the driver box's node-0 list, BENCH_r05
    rank_cpus) and 4 GPUs on it: every rank gets 16 whole cores (both threads), no core is shared."""
    bdfs = [f"0000:{b:02x}:00.0" for b in (0x05, 0x15, 0x25, 0x35)]
    root = _fake_sysfs(tmp_path, {b: 0 for b in bdfs}, {0: "0-63,128-191"})
    _fake_siblings(tmp_path, 64, 128)
    plans = [numa.plan_affinity(bdfs, i, range(256), root)[1] for i in range(4)]
    assert plans[0] == list(range(0, 16)) + list(range(128, 144))
    assert plans[2] == list(range(32, 48)) + list(range(160, 176))
    cores = [{c % 128 for c in p} for p in plans]
    for i in range(4):
        assert len(plans[i]) == 32 and len(cores[i]) == 16
        for j in range(i + 1, 4):
            assert not cores[i] & cores[j], (i, j)
    # a cpuset holding one thread of some cores: those cores still belong to exactly one rank
    plans = [numa.plan_affinity(bdfs, i, list(range(0, 64)) + list(range(128, 160)), root)[1] for i in range(4)]
    cores = [{c % 128 for c in p} for p in plans]
    assert all(not cores[i] & cores[j] for i in range(4) for j in range(i + 1, 4))


def test_fewer_cores_than_ranks_splits_threads(tmp_path):
    bdfs = [f"0000:{b:02x}:00.0" for b in (0x05, 0x15, 0x25, 0x35)]
    root = _fake_sysfs(tmp_path, {b: 0 for b in bdfs}, {0: "0-1,128-129"})
    _fake_siblings(tmp_path, 2, 128)
    plans = [numa.plan_affinity(bdfs, i, range(256), root)[1] for i in range(4)]
    assert plans == [[0], [1], [128], [129]]
