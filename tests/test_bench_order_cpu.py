"""bench.py's FedAvgRunner enqueue order: launch -> all-reduce issue -> stage(next) -> wait -> next launch.

Issuing the collective before the next round's staging is what lets ``--overlap tail`` overlap anything: RCCL's
stream waits on the compute stream at issue time, so staging enqueued first would serialise the collective
behind it.  Also: the GPU-free device count used by the self-launcher."""
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402


class _Work:
    def __init__(self, log, k):
        self.log, self.k = log, k

    def wait(self):
        self.log.append(("wait", self.k))


class _Recorder:
    def __init__(self):
        self.log = []
        self.staged = None
        self.n_ar = 0

    # trainer API
    def prepare_round(self, n, reset_loss=True):
        if self.staged != n:
            self.log.append(("prepare", n))
        self.staged = None

    def launch_round(self, n, next_n=None):
        assert next_n is None, "the runner stages the next round itself, after issuing the all-reduce"
        self.log.append(("launch", n))

    def stage(self, n):
        self.staged = n
        self.log.append(("stage", n))

    # collective
    def allreduce(self, flat, ctx, async_op=False):
        k = self.n_ar
        self.n_ar += 1
        self.log.append(("issue", k, async_op))
        return _Work(self.log, k) if async_op else None


def _run(overlap, plan, then=None):
    rec = _Recorder()
    ctx = SimpleNamespace(distributed=True)
    r = bench.FedAvgRunner(rec, None, ctx, overlap, allreduce=rec.allreduce)
    r.run(plan, then=then)
    return rec.log, r


def test_tail_issue_before_stage_before_wait():
    log, r = _run("tail", [5, 5, 2], then=5)
    assert r.syncs == 3
    assert log == [
        ("prepare", 5), ("launch", 5), ("issue", 0, True), ("stage", 5),
        ("wait", 0), ("launch", 5), ("issue", 1, True), ("stage", 2),
        ("wait", 1), ("launch", 2), ("issue", 2, True), ("stage", 5),
        ("wait", 2),  # drain at the end of the plan
    ]


def test_none_waits_then_stages():
    log, r = _run("none", [3, 3])
    assert log == [("prepare", 3), ("launch", 3), ("issue", 0, True), ("wait", 0), ("stage", 3),
                   ("launch", 3), ("issue", 1, True), ("wait", 1)]


def test_compute_only_pass_issues_nothing():
    rec = _Recorder()
    r = bench.FedAvgRunner(rec, None, SimpleNamespace(distributed=True), "tail", allreduce=rec.allreduce)
    r.collectives = False
    r.run([3, 3], then=3)
    assert r.syncs == 0 and r.recs == []
    assert rec.log == [("prepare", 3), ("launch", 3), ("stage", 3), ("launch", 3), ("stage", 3)]


def test_single_process_is_never_async():
    rec = _Recorder()
    r = bench.FedAvgRunner(rec, None, SimpleNamespace(distributed=False), "tail", allreduce=rec.allreduce)
    assert r.overlap == "none"


def test_count_gpus_kfd(tmp_path, monkeypatch):
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    for i, gid in enumerate([0, 1234, 5678, 91011]):  # node 0 is the CPU
        d = tmp_path / str(i)
        d.mkdir()
        (d / "gpu_id").write_text(f"{gid}\n")
    assert bench.count_gpus_kfd(str(tmp_path)) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1")
    assert bench.count_gpus_kfd(str(tmp_path)) == 2
    assert bench.count_gpus_kfd(str(tmp_path / "missing")) == -1


def test_self_launch_parent_never_imports_torch_cuda(monkeypatch):
    """The parent counts GPUs from sysfs; with too few it refuses before starting anything."""
    monkeypatch.setattr(bench, "count_gpus_kfd", lambda: 1)
    monkeypatch.setenv("ECG_DIST_BACKEND", "nccl")
    a = bench.parse(["--gpus", "2"])
    assert bench.self_launch(a, ["--gpus", "2"]) == 2
