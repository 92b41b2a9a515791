#!/usr/bin/env python3
"""Stream / hardware-queue audit of an N>1 rank's stream layout on ONE GPU.

An N>1 rank uses four streams: torch's current (compute) stream, the ResNet engine's low-priority side lane
(csrc/kernels/resnet_nlc.hip ``side_lane``), the device's high-priority comm stream (parallel/overlap.comm_stream)
and RCCL's internal stream.  HIP maps streams onto at most GPU_MAX_HW_QUEUES (4 on the box) hardware queues per
priority; two streams that share a queue execute in order, so a collective could wait behind compute kernels.
This probe replays the layout in one process with a world-1 RCCL group (the box has one GPU) and is run under
``rocprofv3 --kernel-trace``; ``parse`` reads the trace and reports, per stream role, the hardware queue
(``Queue_Id``) its kernels ran on and whether the comm-lane kernels ran INSIDE the compute kernels' spans.

  run        synthetic: compute spin (~2 ms) | side-lane spin (~0.5 ms) | comm-stream add + RCCL all-reduce, x5;
             resnet:    ResNet1D-18 B=256 tail-FedAvg steps - per-bucket SGD on the comm stream + all-reduce while
                        the backward continues on the compute stream and the side lane
  parse DIR  the kernel_trace.csv under DIR -> the report (profiles/r6/stream_queues.txt)
"""
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SPIN_COMPUTE, SPIN_SIDE = 4_000_000, 1_000_000


def run():
    import torch
    import torch.distributed as dist
    import crossscale_ecg  # noqa: F401
    from crossscale_ecg.parallel.env import DistContext, nccl_pg_options
    from crossscale_ecg.parallel.overlap import comm_stream, CommRecord, FedAvgComm
    from crossscale_ecg.models.resnet1d import resnet1d18
    from crossscale_ecg.train.resnet_trainer import ResNetEngineTrainer
    from crossscale_ecg.ops import _lib
    import ctypes

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29555"), RANK="0",
                      WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    opts = nccl_pg_options()  # exactly what init_distributed passes (ECG_RCCL_HIGH_PRIORITY=0: torch's default)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev,
                            **({"pg_options": opts} if opts is not None else {}))
    print(f"RCCL stream high priority: {opts is not None}")
    # a context that issues collectives like an N>1 rank (the real group has one rank: AVG is the identity)
    ctx = DistContext(0, 2, 0, "nccl", dev)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (None, None)
    print(f"stream priority range (torch): {lo}, {hi}; GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')}")

    torch.manual_seed(0)
    m = resnet1d18().to(dev)
    x = torch.randn(2048, 500, device=dev)
    y = (x.mean(1) > 0).long()
    tr = ResNetEngineTrainer(m, x, y, 256, 4, seed=0, ctx=ctx, bucket_mb=1.0)
    lib = tr.engine.lib
    sp = ctypes.c_void_p()
    _lib.check(lib.ecg_plan_side_stream(ctypes.byref(sp)), "ecg_plan_side_stream")
    side = torch.cuda.ExternalStream(sp.value, device=dev)
    comm = comm_stream(dev)
    compute = torch.cuda.current_stream(dev)
    print(f"streams: compute={compute.cuda_stream:#x} side={side.cuda_stream:#x} comm={comm.cuda_stream:#x} "
          f"(comm priority {comm.priority})")

    # ---- synthetic: which kernel runs where, and does the comm lane overlap the compute lane
    buf = torch.zeros(1458, device=dev)
    torch.cuda.synchronize()
    for it in range(5):
        ev = {k: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for k in ("compute", "side", "comm")}
        ev["compute"][0].record(compute)
        torch.cuda._sleep(SPIN_COMPUTE)
        ev["compute"][1].record(compute)
        with torch.cuda.stream(side):
            ev["side"][0].record(side)
            torch.cuda._sleep(SPIN_SIDE)
            ev["side"][1].record(side)
        with torch.cuda.stream(comm):
            ev["comm"][0].record(comm)
            buf.add_(1.0)
            dist.all_reduce(buf, op=dist.ReduceOp.AVG, async_op=True).wait()
            buf.add_(1.0)
            ev["comm"][1].record(comm)
        torch.cuda.synchronize()
        t0 = ev["compute"][0]
        spans = {k: (t0.elapsed_time(a), t0.elapsed_time(b)) for k, (a, b) in ev.items()}
        inside = spans["comm"][1] < spans["compute"][1] and spans["side"][1] < spans["compute"][1]
        print(f"synthetic it{it}: " + " ".join(f"{k}=[{a:.3f},{b:.3f}]ms" for k, (a, b) in spans.items())
              + f" -> comm+side finished inside the compute spin: {inside}")

    # ---- the real ResNet tail-FedAvg layout (per-bucket SGD on the comm stream + all-reduce under the backward)
    fc = FedAvgComm(ctx)
    for it in range(3):
        tr.run_round(2)
        rec = CommRecord()
        tr.tail_fedavg(fc, rec)
        torch.cuda.synchronize()
        print(f"resnet tail step {it}: buckets={len(tr.issue_log)} comm_ms={rec.comm_ms():.3f} "
              f"exposed_ms={rec.exposed_ms():.3f}")
        tr.issue_log.clear()
    tr.close()
    dist.destroy_process_group()


def _role(name, dur_us):
    if "spin_kernel" in name or "sleep" in name.lower():
        return "compute_spin" if dur_us > 1200 else "side_spin"
    low = name.lower()
    if "nccl" in low or "rccl" in low or "onerank" in low:
        return "rccl"
    return None


def parse(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows = sorted(csv.DictReader(open(files[0])), key=lambda r: int(r["Start_Timestamp"]))
    ks = [dict(name=r["Kernel_Name"], q=int(r["Queue_Id"]), s=int(r["Stream_Id"]), t0=int(r["Start_Timestamp"]),
               t1=int(r["End_Timestamp"])) for r in rows]
    # synthetic section: the compute spins, the side spins, and the comm-stream kernels between them
    spins = [k for k in ks if _role(k["name"], (k["t1"] - k["t0"]) / 1e3) == "compute_spin"]
    print(f"kernels in trace: {len(ks)}; compute spins: {len(spins)}")
    queue_of = {}
    for sp in spins:
        window = [k for k in ks if sp["t0"] - 50_000 <= k["t0"] <= sp["t1"] + 50_000 and k is not sp]
        for k in window:
            role = _role(k["name"], (k["t1"] - k["t0"]) / 1e3)
            if role is None and "elementwise" in k["name"]:
                role = "comm_add"
            if role:
                queue_of.setdefault(role, set()).add((k["q"], k["s"]))
        queue_of.setdefault("compute_spin", set()).add((sp["q"], sp["s"]))
        inside = [k for k in window if sp["t0"] <= k["t0"] and k["t1"] <= sp["t1"]]
        desc = ", ".join(f"{(_role(k['name'], (k['t1'] - k['t0']) / 1e3) or k['name'][:40])}"
                         f"@q{k['q']}/s{k['s']} [{(k['t0'] - sp['t0']) / 1e3:.1f},{(k['t1'] - sp['t0']) / 1e3:.1f}]us"
                         for k in inside)
        print(f"compute spin q{sp['q']}/s{sp['s']} {(sp['t1'] - sp['t0']) / 1e3:.1f} us; inside it: {desc or 'nothing'}")
    print("queue/stream per role (synthetic):", {k: sorted(v) for k, v in queue_of.items()})
    # resnet section: after the last spin
    last = spins[-1]["t1"] if spins else 0
    rk = [k for k in ks if k["t0"] > last]
    sgd = [k for k in rk if "sgd" in k["name"].lower()]
    by_q = {}
    for k in rk:
        by_q.setdefault((k["q"], k["s"]), []).append(k)
    print("resnet section kernels per (queue, stream):",
          {f"q{q}/s{s}": len(v) for (q, s), v in sorted(by_q.items())})
    sgd_q = {(k["q"], k["s"]) for k in sgd}
    print(f"SGD kernels: {len(sgd)} on {sorted(sgd_q)}")
    # a per-bucket SGD (comm stream) overlapping any kernel of another queue = concurrency across queues
    over = 0
    for k in sgd:
        if any(o["q"] != k["q"] and o["t0"] < k["t1"] and k["t0"] < o["t1"] for o in rk):
            over += 1
    print(f"SGD kernels that overlap a kernel on another hardware queue: {over} / {len(sgd)}")
    rc = [k for k in rk if _role(k["name"], 0) == "rccl"]
    main_q = {(k["q"], k["s"]) for k in rk if k["s"] == 0}
    rc_over = sum(1 for k in rc if any((o["q"], o["s"]) in main_q and o["t0"] < k["t1"] and k["t0"] < o["t1"]
                                       for o in rk))
    print(f"RCCL kernels: {len(rc)} on {sorted({(k['q'], k['s']) for k in rc})}; running beside a compute-stream "
          f"kernel: {rc_over} / {len(rc)}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "parse":
        parse(sys.argv[2])
    else:
        run()
