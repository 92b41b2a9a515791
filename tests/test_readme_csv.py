"""README <-> CSV consistency: the module-result rows of README.md are exactly what
crossscale_ecg.report.readme renders from the CSV directory the block names, and that directory is the newest
committed profiles/rN/modules."""
import os

import pytest

from crossscale_ecg.report import readme

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_readme_module_rows_match_csvs():
    ok, expected, found = readme.check(os.path.join(ROOT, "README.md"), root=ROOT)
    assert ok, "README module block is stale; run `python -m crossscale_ecg.report.readme --write`\n" + expected


def test_readme_block_cites_newest_modules_dir():
    with open(os.path.join(ROOT, "README.md")) as f:
        block = readme._split(f.read())[1]
    assert f"<!-- source: {readme.latest_modules_dir(ROOT)} -->" in block


def test_render_marks_bar_and_spread(tmp_path):
    """A synthetic CSV pair: the A3 bar is judged per batch size and the IQR columns are quoted when present."""
    d = tmp_path / "modules"
    d.mkdir()
    hdr = "config,batch_size,pin_memory,contiguous,non_blocking,data_ms,h2d_ms,compute_ms,step_ms,samples_per_s," \
          "samples_per_s_q1,samples_per_s_q3,reps\n"
    rows = []
    for b, a0, a3 in ((64, 100e3, 120e3), (128, 200e3, 210e3)):
        for cfg, v in (("A0_baseline", a0), ("A1_contiguous", a0), ("A2_contig_pinned", a0),
                       ("A3_contig_pinned_nb", a3)):
            rows.append(f"{cfg},{b},0,0,0,0,0,0,0,{v},{v * 0.9},{v * 1.1},5\n")
    (d / "part1_locality_results.csv").write_text(hdr + "".join(rows))
    (d / "part2_hip_results.csv").write_text(
        "batch_size,kernel_size,torch_ms_median,hip_ms_median,speedup_med\n64,3,0.04,0.01,4.0\n64,5,0.045,0.01,4.5\n")
    row = readme.module1_row(str(d))
    assert "+20 % (B=64)" in row and "+5 % (B=128)" in row and "bar at B=64." in row
    assert "Medians of 5 interleaved repetitions" in row and "B=64 90–110 / 90–110 / 108–132" in row
    assert "**4.00–4.50×**" in readme.module2_row(str(d))


def test_readme_headline_matches_bench_runs():
    """The headline rows are rendered from every recorded bench line (profiles/rN/bench_runs.jsonl) of HEAD's code,
    and the runs file holds the newest driver record (BENCH_rNN.json)."""
    import json
    runs_file = readme.latest_runs_file(ROOT)
    commits = {json.loads(ln)["commit"] for ln in open(os.path.join(ROOT, runs_file)) if ln.strip()}
    if not readme.git_ready(c for c in commits if c):
        pytest.skip("git history (HEAD and the recorded commits) not available: code identity cannot be decided")
    ok, expected, found = readme.check_headline(os.path.join(ROOT, "README.md"), root=ROOT)
    assert ok, "README headline is stale; run `python -m crossscale_ecg.report.readme --write`\n" + expected
    assert f"<!-- runs: {readme.latest_runs_file(ROOT)} -->" in found


def test_render_headline_median_over_boxes(tmp_path, monkeypatch):
    """Builder rows: median and range over all runs of HEAD's code (other commits ignored), box count; the driver
    column quotes the newest driver record."""
    import json
    recs = [
        {"source": "builder", "session": "s0", "log": "bench20_1.log", "box": "A", "commit": "old", "model": "tiny_ecg",
         "value": 30e6, "ms_per_step": 0.0085, "gpu_ms_per_step": 0.008, "steps": 20, "warmup": 5, "n_gpus": 1},
        {"source": "driver", "session": "BENCH_r07.json", "log": "", "box": "x", "commit": "c7", "model": "tiny_ecg",
         "round": 7, "value": 20e6, "ms_per_step": 0.0128, "gpu_ms_per_step": 0.0118, "steps": 20, "warmup": 5,
         "n_gpus": 1},
    ]
    for i, (v, box) in enumerate(((18e6, "A"), (20e6, "B"), (19e6, "B"))):
        recs.append({"source": "builder", "session": "s1", "log": f"bench20_{i}.log", "box": box, "commit": "new",
                     "model": "tiny_ecg", "value": v, "ms_per_step": 256 / v * 1e3, "gpu_ms_per_step": None,
                     "steps": 20, "warmup": 5, "n_gpus": 1})
    p = tmp_path / "bench_runs.jsonl"
    p.write_text("".join(json.dumps(r) + "\n" for r in recs))
    # code identity: "new" carries HEAD's code, "old" does not
    monkeypatch.setattr(readme, "_same_code", lambda a, b: a == "new" and b == "HEAD")
    text = readme.render_headline(str(p))
    row = [ln for ln in text.splitlines() if "driver's command" in ln][0]
    assert "round 7: **20.0 M/s**" in row
    assert "median **19.0 M/s** (18.0 M/s–20.0 M/s) over 3 runs on 2 boxes, commit `new`" in row
    assert "no run of the current code" in [ln for ln in text.splitlines() if "ResNet1D-34" in ln][0]
    # a code change without new runs: every builder row says so instead of quoting the old numbers
    monkeypatch.setattr(readme, "_same_code", lambda a, b: False)
    stale = readme.render_headline(str(p))
    assert "median" not in [ln for ln in stale.splitlines() if "driver's command" in ln][0]


def test_headline_check_tolerates_only_the_round_end_driver_record(tmp_path):
    """BENCH_rNN.json of the current round is written after the builder's session ends: the check accepts its
    absence from the runs file, but not the absence of an older driver record (advisor r5)."""
    import json
    (tmp_path / "profiles" / "r9").mkdir(parents=True)
    runs = tmp_path / "profiles" / "r9" / "bench_runs.jsonl"
    for n in (4, 5):
        (tmp_path / f"BENCH_r{n:02d}.json").write_text("{}")
    (tmp_path / "README.md").write_text(f"x\n{readme.HBEGIN}\n<!-- runs: profiles/r9/bench_runs.jsonl -->\n{readme.HEND}\n")

    def drv(rnd):
        return json.dumps({"source": "driver", "session": f"BENCH_r{rnd:02d}.json", "log": "", "box": "x",
                           "commit": "c", "model": "tiny_ecg", "round": rnd, "value": 1e6, "ms_per_step": 0.2,
                           "gpu_ms_per_step": 0.2, "steps": 20, "warmup": 5, "n_gpus": 1}) + "\n"
    runs.write_text(drv(3))
    ok, msg, _ = readme.check_headline(str(tmp_path / "README.md"), root=str(tmp_path))
    assert not ok and "BENCH_r04.json is newer" in msg
    runs.write_text(drv(3) + drv(4))
    ok, msg, _ = readme.check_headline(str(tmp_path / "README.md"), root=str(tmp_path))
    assert "is newer" not in msg  # round 5's record may still be missing
