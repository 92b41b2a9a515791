"""Round-6 trace tools on synthetic rocprofv3 kernel-trace CSVs: the stream -> hardware-queue audit
(scripts/probe_stream_queues.py parse) and the blit-kernel attribution (scripts/attribute_copies.py)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COLS = ["Kind", "Agent_Id", "Queue_Id", "Stream_Id", "Thread_Id", "Dispatch_Id", "Kernel_Id", "Kernel_Name",
        "Correlation_Id", "Start_Timestamp", "End_Timestamp", "Grid_Size_X"]


def _write(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(COLS)
        for i, (q, s, name, t0, t1, grid) in enumerate(rows):
            w.writerow(["KERNEL_DISPATCH", "Agent 2", q, s, 1, i, 1, name, i, t0, t1, grid])


def test_queue_audit_reads_roles_and_overlap(tmp_path):
    us = 1000
    rows = []
    for it in range(2):  # synthetic part: compute spin on q4, side spin q5, comm add q6, RCCL q7 inside the spin
        t = it * 5000 * us
        rows += [(4, 0, "spin_kernel(long)", t, t + 1700 * us, 1),
                 (5, 7, "spin_kernel(long)", t + 20 * us, t + 450 * us, 1),
                 (6, 8, "void at::native::vectorized_elementwise_kernel<4, add>", t + 40 * us, t + 42 * us, 1),
                 (7, 9, "void (anonymous namespace)::oneRankReduce<FuncPreMulSum<float> >(void*)", t + 60 * us,
                  t + 62 * us, 1)]
    t = 20000 * us  # resnet part: a compute kernel with an SGD (comm stream) and an RCCL kernel inside it
    rows += [(4, 0, "conv1d_nlc_fwd_tap_kernel", t, t + 100 * us, 256),
             (6, 8, "(anonymous namespace)::sgd_flat_kernel(float*)", t + 10 * us, t + 12 * us, 64),
             (7, 9, "void (anonymous namespace)::oneRankReduce<FuncPreMulSum<float> >(void*)", t + 20 * us,
              t + 22 * us, 1)]
    d = tmp_path / "q"
    d.mkdir()
    _write(d / "q_kernel_trace.csv", rows)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "probe_stream_queues.py"), "parse", str(d)],
                         capture_output=True, text=True, check=True).stdout
    assert "compute spins: 2" in out
    assert "'rccl': [(7, 9)]" in out and "'compute_spin': [(4, 0)]" in out and "'side_spin': [(5, 7)]" in out
    assert "SGD kernels that overlap a kernel on another hardware queue: 1 / 1" in out
    assert "running beside a compute-stream kernel: 1 / 1" in out


def test_copy_attribution_phases(tmp_path):
    us = 1000
    rows = [(1, 0, "__amd_rocclr_copyBuffer", 0, us, 512)]  # setup
    t = 10 * us
    for step in range(4):  # steps end with the optimizer kernel
        rows += [(1, 0, "fwd_kernel", t, t + 5 * us, 256), (1, 0, "sgd_flat_kernel", t + 6 * us, t + 7 * us, 64)]
        t += 10 * us
        if step == 1:  # the timed round's staging, behind the last warm-up step
            rows += [(1, 0, "__amd_rocclr_copyBuffer", t - 2 * us, t - us, 12800)]
    rows += [(1, 0, "__amd_rocclr_copyBuffer", t + us, t + 2 * us, 512)]  # teardown
    path = tmp_path / "trace.csv"
    _write(path, rows)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "attribute_copies.py"), str(path), "2"],
                         capture_output=True, text=True, check=True).stdout
    lines = {ln.split()[0]: ln for ln in out.splitlines() if ln.startswith("  ") and ln.split()[0].isidentifier()}
    assert lines["setup"].split()[1] == "1"
    assert lines["between_warmup_and_timed"].split()[1] == "1"
    assert lines["timed_steps"].split()[1] == "0"
    assert lines["teardown"].split()[1] == "1"
