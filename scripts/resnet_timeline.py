#!/usr/bin/env python3
"""ResNet1D-34 B=1024 side-lane steps for a kernel-trace timeline: ``resnet_timeline.py run`` runs 8 eager
steps (profile it with rocprofv3 --kernel-trace); ``resnet_timeline.py parse <kernel_trace.csv>`` summarises
the last 4 steps per queue: busy time, overlap of the two queues, top kernels per queue."""
import collections
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(B=1024, steps=8):
    import torch
    import crossscale_ecg  # noqa: F401
    from crossscale_ecg.models.resnet1d import resnet1d34
    from crossscale_ecg.ops.resnet_engine import ResNetStepEngine
    torch.manual_seed(0)
    eng = ResNetStepEngine(resnet1d34().cuda(), B, 500)
    eng.set_batch(torch.randn(B, 1, 500, device="cuda"), torch.randint(0, 2, (B,), device="cuda"))
    for _ in range(steps):
        eng.step()
    torch.cuda.synchronize()


def parse(path, last=4):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], r["Kernel_Name"]) for r in rows))
    # step boundaries: the weight-prep kernel starts every step
    starts = [k[0] for k in ks if "weight_prep" in k[3]]
    t0, t1 = starts[-last - 1], starts[-1]
    sel = [k for k in ks if t0 <= k[0] < t1]
    wall = (t1 - t0) / 1e3
    print(f"{last} steps: {wall / last:.1f} us/step wall")
    by_q = collections.defaultdict(list)
    for k in sel:
        by_q[k[2]].append(k)

    def union(iv):
        tot, cur_s, cur_e = 0, None, None
        for s, e in sorted(iv):
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        return tot + ((cur_e - cur_s) if cur_e is not None else 0)

    allbusy = union([(k[0], k[1]) for k in sel]) / 1e3
    print(f"any-queue busy {allbusy / last:.1f} us/step ({100 * allbusy / wall:.1f} % of wall)")
    for q, kk in by_q.items():
        busy = union([(k[0], k[1]) for k in kk]) / 1e3
        agg = collections.Counter()
        for k in kk:
            agg[k[3][:100]] += (k[1] - k[0]) / 1e3
        print(f"queue {q}: {len(kk) // last} kernels/step, busy {busy / last:.1f} us/step")
        for name, us in agg.most_common(8):
            print(f"    {us / last:8.1f} us/step  {name}")
    # the main (critical) queue: the one that runs the weight prep; idle gaps between its consecutive kernels
    mq = next(k[2] for k in sel if "weight_prep" in k[3])
    mk = sorted(by_q[mq])
    gaps = []
    for a, b in zip(mk, mk[1:]):
        gaps.append(((b[0] - a[1]) / 1e3, a[3][:60], b[3][:60]))
    idle = sum(max(0.0, g[0]) for g in gaps)
    print(f"main queue {mq}: idle between kernels {idle / last:.1f} us/step "
          f"({len(gaps) // last} boundaries, {idle / max(1, len(gaps)):.2f} us each on average)")
    agg_g = collections.Counter()
    for g, a, b in gaps:
        agg_g[(a, b)] += max(0.0, g)
    print("largest idle gaps (summed over the steps, per step):")
    for (a, b), us in agg_g.most_common(10):
        print(f"    {us / last:8.1f} us  after {a}  ->  {b}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(sys.argv[2])
