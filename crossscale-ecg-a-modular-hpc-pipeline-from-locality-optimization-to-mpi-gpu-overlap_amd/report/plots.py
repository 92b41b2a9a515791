"""Reporting layer: the reference's figures from the CSVs (matplotlib, Agg backend).

Reference scripts and formulas reproduced:
  * plot_locality       <- Module_1/plot_locality.py:7-76 (throughput vs batch, stacked data/h2d/compute)
  * plot_all_results    <- Module_1/plot_all_results.py:1-130 (A0-A4 merge; effective A4 throughput
                           ``sps / (1 + shard_time / (EPOCHS * N / sps))`` with EPOCHS=10 (:53-58);
                           per-step shard ms ``(shard_time/EPOCHS)/(N/bs)*1e3`` (:84-90)); its two figures:
                           plot_all_results_figures
  * plot_part2          <- Module_2/benchmark_part_2.py:149-173 and Module_2/plot_part2.py
  * plot_pseudo_fl      <- Module_3/plot_part3.py (mean per (world, config), throughput-vs-world + stacked bars)
  * plot_fedavg         <- Module_3/TRUE_FL_M3/plot_part3.py (``step_ms = local_train_ms + comm_ms`` (:48));
                           additionally the node-aggregate samples/s scaling curve.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict, List, Optional

import numpy as np

EPOCHS = 10


def _plt():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt


def _read(path: str):
    import pandas as pd
    return pd.read_csv(path)


def effective_a4_throughput(sps: float, shard_time_s: float, n_windows: int, epochs: int = EPOCHS) -> float:
    """A4 throughput with the one-time shard preparation amortised over ``epochs`` epochs."""
    train_s = epochs * n_windows / sps
    return sps / (1.0 + shard_time_s / train_s)


def shard_ms_per_step(shard_time_s: float, n_windows: int, batch: int, epochs: int = EPOCHS) -> float:
    return (shard_time_s / epochs) / (n_windows / batch) * 1e3


def plot_locality(csv_path: str, out_dir: str, batch: Optional[int] = None) -> List[str]:
    plt = _plt()
    df = _read(csv_path)
    outs = []
    fig = plt.figure(figsize=(6.8, 4.2))
    for cfg in df["config"].unique():
        sub = df[df["config"] == cfg].sort_values("batch_size")
        plt.plot(sub["batch_size"], sub["samples_per_s"], marker="o", label=cfg)
    plt.xlabel("Batch size"); plt.ylabel("Samples / second"); plt.title("Throughput vs Batch Size (MI355X)")
    plt.grid(True); plt.legend(); plt.tight_layout()
    p = os.path.join(out_dir, "throughput_vs_batch.png"); plt.savefig(p, dpi=150); plt.close(fig); outs.append(p)
    bs = batch or int(df["batch_size"].max())
    sub = df[df["batch_size"] == bs][["config", "data_ms", "h2d_ms", "compute_ms"]].set_index("config")
    ax = sub.plot(kind="bar", stacked=True, figsize=(6.8, 4.2))
    ax.set_ylabel("Milliseconds per step"); ax.set_title(f"Time Breakdown per Step (batch={bs})")
    plt.tight_layout()
    p = os.path.join(out_dir, "time_breakdown_stacked.png"); plt.savefig(p, dpi=150); plt.close(); outs.append(p)
    return outs


def plot_all_results(results_dir: str) -> Optional[str]:
    """Merge A0-A3 + A4 CSVs into part1_all_results.csv with the amortised-shard-cost A4 column."""
    import pandas as pd
    loc = os.path.join(results_dir, "part1_locality_results.csv")
    if not os.path.exists(loc):
        return None
    df = pd.read_csv(loc)
    labl = os.path.join(results_dir, "part1_labl_results.csv")
    if os.path.exists(labl):
        d4 = pd.read_csv(labl)
        d4 = d4[~d4["batch_size"].isin(df[df["config"] == "A4_LABL"]["batch_size"])]
        df = pd.concat([df, d4], ignore_index=True)
    meta = os.path.join(results_dir, "shard_prep_metrics.json")
    if os.path.exists(meta):
        m = json.load(open(meta))
        t, n = m["total_time_s"], m["total_windows"]
        mask = df["config"] == "A4_LABL"
        df.loc[mask, "effective_samples_per_s"] = [effective_a4_throughput(s, t, n)
                                                   for s in df.loc[mask, "samples_per_s"]]
        df.loc[mask, "shard_ms_per_step"] = [shard_ms_per_step(t, n, b) for b in df.loc[mask, "batch_size"]]
    out = os.path.join(results_dir, "part1_all_results.csv")
    df.to_csv(out, index=False)
    return out


def plot_all_results_figures(results_dir: str, batch: int = 512) -> List[str]:
    """The two figures of Module_1/plot_all_results.py from ``part1_all_results.csv`` (written first): throughput
    vs batch for every configuration plus the A4 curve with the shard preparation amortised (when the shard-prep
    JSON exists), and the per-step time breakdown at ``batch`` with A4's amortised shard ms stacked on top."""
    csv_path = plot_all_results(results_dir)
    if csv_path is None:
        return []
    plt = _plt()
    df = _read(csv_path)
    outs = []
    fig = plt.figure(figsize=(6.8, 4.2))
    for cfg in df["config"].unique():
        sub = df[df["config"] == cfg].sort_values("batch_size")
        plt.plot(sub["batch_size"], sub["samples_per_s"], marker="o", label=cfg)
    if "effective_samples_per_s" in df:
        a4 = df[df["effective_samples_per_s"].notna()].sort_values("batch_size")
        if len(a4):
            plt.plot(a4["batch_size"], a4["effective_samples_per_s"], marker="x", linestyle="--",
                     label="A4_LABL (shard prep amortised)")
    plt.xlabel("Batch size"); plt.ylabel("Samples / second"); plt.title("Throughput Comparison (A0-A4, MI355X)")
    plt.grid(True); plt.legend(fontsize=7); plt.tight_layout()
    p = os.path.join(results_dir, "throughput_comparison_A0_A4.png"); plt.savefig(p, dpi=150); plt.close(fig)
    outs.append(p)
    d = df[df["batch_size"] == batch]
    if len(d):
        x = np.arange(len(d))
        fig = plt.figure(figsize=(7.2, 4.2))
        bottom = np.zeros(len(d))
        for col in ("data_ms", "h2d_ms", "compute_ms"):
            v = d[col].fillna(0.0).values
            plt.bar(x, v, width=0.6, bottom=bottom, label=col)
            bottom = bottom + v
        if "shard_ms_per_step" in d and d["shard_ms_per_step"].notna().any():
            plt.bar(x, d["shard_ms_per_step"].fillna(0.0).values, width=0.6, bottom=bottom, hatch="//",
                    label="shard_ms (amortised)")
        plt.xticks(x, d["config"], rotation=20, fontsize=7); plt.ylabel("Milliseconds per step")
        plt.title(f"Time Breakdown per Step (batch={batch})"); plt.legend(fontsize=7); plt.tight_layout()
        p = os.path.join(results_dir, f"time_breakdown_batch{batch}_A0_A4.png"); plt.savefig(p, dpi=150)
        plt.close(fig)
        outs.append(p)
    return outs


def plot_part2(results_dir: str) -> List[str]:
    plt = _plt()
    outs = []
    for name, col_a, col_b, label in (("part2_hip_results.csv", "torch_ms_median", "hip_ms_median", "HIP"),
                                      ("part2_openmp_results.csv", "torch_ms_median", "omp_ms_median", "OpenMP")):
        p = os.path.join(results_dir, name)
        if not os.path.exists(p):
            continue
        df = _read(p)
        tag = "hip" if label == "HIP" else "openmp"
        fig = plt.figure(figsize=(6.8, 4.2))
        sps_col = "hip_sps" if label == "HIP" else "omp_sps"
        std_col = col_b.replace("median", "std")
        for K in sorted(df["kernel_size"].unique()):
            d = df[df["kernel_size"] == K].sort_values("batch_size")
            ms, bs = d[col_b].values, d["batch_size"].values
            err = np.abs(bs * 1000.0 / (ms ** 2)) * d[std_col].values
            plt.errorbar(bs, d[sps_col], yerr=err, marker="o", capsize=3, label=f"K={K}")
        plt.xlabel("Batch size"); plt.ylabel("Samples / second"); plt.title(f"{label} conv1d throughput (median ± std)")
        plt.grid(True); plt.legend(); plt.tight_layout()
        q = os.path.join(results_dir, f"part2_{tag}_throughput.png"); plt.savefig(q, dpi=150); plt.close(fig)
        outs.append(q)
        fig = plt.figure(figsize=(6.8, 4.2))
        for K in sorted(df["kernel_size"].unique()):
            d = df[df["kernel_size"] == K].sort_values("batch_size")
            plt.plot(d["batch_size"], d["speedup_med"], marker="o", label=f"K={K}")
        plt.xlabel("Batch size"); plt.ylabel(f"Speedup ({label} / Torch, median)")
        plt.title(f"Part 2: {label} conv1d speedup over PyTorch"); plt.grid(True); plt.legend(); plt.tight_layout()
        q = os.path.join(results_dir, f"part2_{tag}_speedup.png"); plt.savefig(q, dpi=150); plt.close(fig)
        outs.append(q)
    p = os.path.join(results_dir, "part2_openmp_simd_results.csv")
    if os.path.exists(p):
        df = _read(p)
        fig = plt.figure(figsize=(6.8, 4.2))
        for bs in sorted(df["batch"].unique()):
            d = df[df["batch"] == bs].sort_values("threads")
            plt.plot(d["threads"], d["samples_per_s"], marker="o", label=f"B={bs}")
        plt.xlabel("Threads"); plt.ylabel("Samples / second"); plt.title("CPU conv1d thread scaling (K=32)")
        plt.grid(True); plt.legend(); plt.tight_layout()
        q = os.path.join(results_dir, "part2_scaling.png"); plt.savefig(q, dpi=150); plt.close(fig)
        outs.append(q)
    return outs


def plot_pseudo_fl(csv_path: str, out_dir: str) -> List[str]:
    plt = _plt()
    df = _read(csv_path)
    g = df.groupby(["world_size", "config"]).mean(numeric_only=True).reset_index()
    outs = []
    fig = plt.figure(figsize=(6.8, 4.2))
    for cfg in g["config"].unique():
        d = g[g["config"] == cfg].sort_values("world_size")
        plt.plot(d["world_size"], d["samples_per_s"], marker="o", label=cfg)
    plt.xlabel("World size"); plt.ylabel("Samples / second (per rank, mean)"); plt.title("Pseudo-FL throughput")
    plt.grid(True); plt.legend(); plt.tight_layout()
    p = os.path.join(out_dir, "part3_throughput_vs_world.png"); plt.savefig(p, dpi=150); plt.close(fig); outs.append(p)
    # grouped stacked bars (Module_3/plot_part3.py plot 2): per world size one bar per configuration, each stacked
    # h2d_ms + compute_ms (the reference leaves data_ms out of this figure)
    worlds = sorted(g["world_size"].unique())
    cfgs = list(g["config"].unique())
    width = 0.8 / max(1, len(cfgs))
    x = np.arange(len(worlds))
    fig = plt.figure(figsize=(7.2, 4.2))
    for i, cfg in enumerate(cfgs):
        d = g[g["config"] == cfg].set_index("world_size").reindex(worlds)
        pos = x + (i - (len(cfgs) - 1) / 2) * width
        h2d, comp = d["h2d_ms"].fillna(0.0).values, d["compute_ms"].fillna(0.0).values
        plt.bar(pos, h2d, width=width, label=f"{cfg} h2d_ms")
        plt.bar(pos, comp, width=width, bottom=h2d, label=f"{cfg} compute_ms")
    plt.xticks(x, [str(w) for w in worlds]); plt.xlabel("World size (ranks)"); plt.ylabel("Milliseconds per step (mean)")
    plt.title("Pseudo-FL time breakdown (h2d + compute)"); plt.legend(fontsize=6); plt.tight_layout()
    p = os.path.join(out_dir, "part3_step_breakdown_grouped.png"); plt.savefig(p, dpi=150); plt.close(fig)
    outs.append(p)
    return outs


def load_fedavg(results_glob: str):
    import pandas as pd
    paths = sorted(glob.glob(results_glob))
    if not paths:
        raise FileNotFoundError(results_glob)
    df = pd.concat([pd.read_csv(p) for p in paths], ignore_index=True)
    df["config"] = df["config"].astype(str).str.extract(r"(G[01])", expand=False).fillna(df["config"])
    df["step_ms"] = df["local_train_ms"] + df["comm_ms"]
    return df


def fedavg_summary(df) -> "object":
    """Mean per (world, config) + node-aggregate samples/s (sum over ranks / max wall per round)."""
    import pandas as pd
    rows = []
    for (w, c), d in df.groupby(["world_size", "config"]):
        per_rank = d["samples_per_s"].mean()
        node = []
        for _, dr in d.groupby("round_idx"):
            wall = (dr["round_wall_ms"] if "round_wall_ms" in dr else dr["step_ms"]).max() / 1e3
            node.append((dr["batch_size"] * dr["local_steps"]).sum() / wall)
        rows.append({"world_size": w, "config": c, "samples_per_s": per_rank, "node_samples_per_s": np.mean(node),
                     "local_train_ms": d["local_train_ms"].mean(), "comm_ms": d["comm_ms"].mean(),
                     "comm_share": d["comm_ms"].mean() / d["step_ms"].mean()})
    return pd.DataFrame(rows)


def plot_fedavg(results_glob: str, out_dir: str) -> List[str]:
    plt = _plt()
    df = load_fedavg(results_glob)
    s = fedavg_summary(df)
    os.makedirs(out_dir, exist_ok=True)
    s.to_csv(os.path.join(out_dir, "fedavg_summary.csv"), index=False)
    outs = []
    for col, ylabel, name in (("samples_per_s", "Samples/s per rank (excl. comm)", "fedavg_throughput_per_rank.png"),
                              ("node_samples_per_s", "Node samples/s (incl. comm)", "fedavg_node_scaling.png")):
        fig = plt.figure(figsize=(6.8, 4.2))
        for cfg in sorted(s["config"].unique()):
            d = s[s["config"] == cfg].sort_values("world_size")
            plt.plot(d["world_size"], d[col], marker="o", label=cfg)
        if col == "node_samples_per_s" and len(s):
            d = s[s["config"] == sorted(s["config"].unique())[-1]].sort_values("world_size")
            base = d[col].values[0] / d["world_size"].values[0]
            plt.plot(d["world_size"], base * d["world_size"], "k--", lw=0.8, label="linear")
        plt.xlabel("World size (GPUs)"); plt.ylabel(ylabel); plt.title("FedAvg TinyECG on MI355X")
        plt.grid(True); plt.legend(); plt.tight_layout()
        p = os.path.join(out_dir, name); plt.savefig(p, dpi=150); plt.close(fig); outs.append(p)
    fig, ax = plt.subplots(figsize=(7.2, 4.2))
    labels, tr, cm = [], [], []
    for _, r in s.sort_values(["world_size", "config"]).iterrows():
        labels.append(f"W{int(r['world_size'])}-{r['config']}")
        tr.append(r["local_train_ms"]); cm.append(r["comm_ms"])
    ax.bar(labels, tr, label="local_train_ms")
    ax.bar(labels, cm, bottom=tr, label="comm_ms")
    ax.set_ylabel("ms per round"); ax.set_title("Round time breakdown"); ax.legend()
    plt.xticks(rotation=45); plt.tight_layout()
    p = os.path.join(out_dir, "fedavg_time_breakdown.png"); plt.savefig(p, dpi=150); plt.close(fig); outs.append(p)
    return outs
