#!/usr/bin/env python3
"""Append every default-configuration bench line of a GPU session to profiles/rN/bench_runs.jsonl, with the box it ran
on (GPU serial number from the session's host.txt) and the commit the session ran, so the README headline can be
rendered from ALL measured lines - not the best box.  Driver records (BENCH_rNN.json at the repo
root) are added with ``--driver``.

    python scripts/collect_bench_runs.py --commit <sha> gpurun_out/r5_<tag> [...]
    python scripts/collect_bench_runs.py --driver BENCH_r03.json
Only the default configurations are collected: ``bench20_<i>.log`` (the driver's command), ``bench500.log``
(K=500) and ``resnet_<i>.log`` (ResNet1D-34 B=1024, K=20); A/B logs with knobs set carry other names.
"""
import argparse
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_OUT = os.path.join(ROOT, "profiles", "r6", "bench_runs.jsonl")
KEEP = ("value", "ms_per_step", "gpu_ms_per_step", "steps", "warmup", "n_gpus")


def _box(session: str) -> str:
    try:
        txt = open(os.path.join(session, "host.txt")).read()
    except OSError:
        return "?"
    m = re.search(r"Serial Number:\s*(\S+)", txt)
    return m.group(1) if m else "?"


def _model(rec: dict) -> str:
    return "resnet1d34" if "ResNet1D-34" in rec.get("metric", "") else "tiny_ecg"


def session_records(session: str, commit: str):
    box, tag = _box(session), os.path.basename(session.rstrip("/"))
    for name in sorted(os.listdir(session)):
        if not re.fullmatch(r"(bench20_\d+|bench500|resnet_\d+)\.log", name):
            continue
        for line in open(os.path.join(session, name)):
            if line.startswith("{"):
                rec = json.loads(line)
                out = {"source": "builder", "session": tag, "log": name, "box": box, "commit": commit,
                       "model": _model(rec)}
                out.update({k: rec.get(k) for k in KEEP})
                yield out


def driver_record(path: str):
    d = json.load(open(path))
    rec = d.get("parsed") or {}
    m = re.search(r"r(\d+)", os.path.basename(path))
    out = {"source": "driver", "session": os.path.basename(path), "log": "", "box": d.get("where", "?"),
           "commit": str(d.get("head", ""))[:12], "model": _model(rec), "round": int(m.group(1)) if m else None}
    out.update({k: rec.get(k) for k in KEEP})
    tail = d.get("tail", "")
    g = re.search(r'"gpu_ms_per_step": ([0-9.]+)', tail)
    out["gpu_ms_per_step"] = float(g.group(1)) if g else None
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("sessions", nargs="*")
    ap.add_argument("--commit", default="")
    ap.add_argument("--driver", action="append", default=[])
    ap.add_argument("--out", default=DEFAULT_OUT)
    a = ap.parse_args(argv)
    seen = set()
    if os.path.exists(a.out):
        for line in open(a.out):
            r = json.loads(line)
            seen.add((r["session"], r["log"], r["source"]))
    new = []
    for s in a.sessions:
        new += [r for r in session_records(s, a.commit) if (r["session"], r["log"], r["source"]) not in seen]
    for p in a.driver:
        r = driver_record(p)
        if (r["session"], r["log"], r["source"]) not in seen:
            new.append(r)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "a") as f:
        for r in new:
            f.write(json.dumps(r) + "\n")
    print(f"{len(new)} new records -> {a.out}")


if __name__ == "__main__":
    main()
