"""bench.py launch/sync/JSON contract rehearsed on CPU: ``--gpus 2`` self-launches two gloo ranks (the parent
never initialises a GPU), every round - including the trailing partial one - ends with the FedAvg all-reduce."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env_extra=None):
    env = dict(os.environ, ECG_DIST_BACKEND="gloo", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               OMP_NUM_THREADS="1", **(env_extra or {}))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--max-windows", "600",
                        "--batch-size", "16", *args], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def test_bench_self_launch_world2_partial_round_syncs():
    rec = _bench("--gpus", "2", "--steps", "7", "--warmup", "3", "--local-steps", "5")
    assert rec["n_gpus"] == 2 and rec["rccl_world_size"] == 2 and rec["dist_backend"] == "gloo"
    assert rec["timed_round_plan"] == [5, 2] and rec["fedavg_syncs_timed"] == 2
    assert rec["timing_barrier"] == "shm"  # both ranks on this node: shared-memory timing barrier
    assert rec["config"]["global_batch"] == 32 and rec["config"]["parallelism"] == "dp2"
    assert rec["value"] == rec["n_gpus"] * 16 * 7 / (rec["ms_per_step"] * 7 / 1e3) or \
        abs(rec["value"] - 32 / (rec["ms_per_step"] / 1e3)) < 1e-3 * rec["value"]


def test_bench_overlap_none_world2():
    rec = _bench("--gpus", "2", "--steps", "4", "--warmup", "0", "--local-steps", "2", "--overlap", "none")
    assert rec["fedavg_syncs_timed"] == 2 and "overlap=none" in rec["config"]["sync"]


def test_bench_single_rank():
    rec = _bench("--steps", "3", "--warmup", "1", "--local-steps", "2")
    assert rec["n_gpus"] == 1 and rec["rccl_world_size"] == 1 and rec["fedavg_syncs_timed"] == 2
    assert rec["timing_barrier"] == "none"


def test_bench_world2_reports_per_rank_comm_and_placement():
    """The N>1 JSON line diagnoses its own MAX: per-rank wall / GPU ms, the timed all-reduces' span and the stall
    on them, and each rank's CPU placement."""
    rec = _bench("--gpus", "2", "--steps", "6", "--warmup", "2", "--local-steps", "3")
    assert len(rec["per_rank_ms_per_step"]) == 2 and max(rec["per_rank_ms_per_step"]) == rec["ms_per_step"]
    assert len(rec["per_rank_gpu_ms_per_step"]) == 2
    assert len(rec["comm_ms"]) == 2 and all(c > 0 for c in rec["comm_ms"])  # two timed all-reduces per rank
    assert len(rec["comm_exposed_ms"]) == 2 and all(0 <= e for e in rec["comm_exposed_ms"])
    # one comm-timing path (parallel/overlap.FedAvgComm): CPU tensors -> host clocks + work-completion callbacks;
    # the wall-clock exposure (elapsed - the same steps without collectives) is reported next to the stall
    assert rec["comm_timing"] == "host"
    assert len(rec["comm_exposed_wall_ms"]) == 2 and all(0 <= e for e in rec["comm_exposed_wall_ms"])
    assert len(rec["rank_cpus"]) == 2 and all(s.startswith("node") for s in rec["rank_cpus"])
    assert rec["gc_paused_in_timed_region"] is True and rec["first_round_staged_in_warmup"] is True


def test_bench_world2_fedavg_weights_identical_and_tail_equals_none():
    """After the timed region every rank holds bit-identical weights (the final FedAvg all-reduce ran), and the
    ``tail`` overlap (all-reduce under the next round's batch staging) lands on exactly the weights of ``none``
    (VERDICT r4 next #3)."""
    recs = {ov: _bench("--gpus", "2", "--steps", "6", "--warmup", "2", "--local-steps", "3", "--overlap", ov)
            for ov in ("none", "tail")}
    for ov, rec in recs.items():
        assert rec["fedavg_weights_identical"] is True, ov
        assert "overlap=" + ov in rec["config"]["sync"]
    assert recs["none"]["fedavg_weights_checksum"] == recs["tail"]["fedavg_weights_checksum"]
    assert recs["none"]["final_avg_loss"] == recs["tail"]["final_avg_loss"]
