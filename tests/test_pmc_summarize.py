"""scripts/pmc_summarize.py on a synthetic rocprofv3 counter CSV: FLOP = MOPS_BF16 x 512, TF/s from durations."""
import csv
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    spec = importlib.util.spec_from_file_location("pmc_summarize", os.path.join(ROOT, "scripts", "pmc_summarize.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_pmc_summarize(tmp_path, capsys):
    m = _load()
    name = "void (anonymous namespace)::conv_k<128, 64>((anonymous namespace)::Args, int)"
    assert m.short(name) == "conv_k<128, 64>"
    cc = tmp_path / "cc.csv"
    fields = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]
    with open(cc, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields)
        w.writeheader()
        for d in (1, 2):  # two dispatches of 10 us, 1e7 MOPS each -> 5.12 GFLOP, 512 TF/s
            for cn, v in (("SQ_INSTS_VALU_MFMA_MOPS_BF16", 1e7), ("SQ_BUSY_CYCLES", 1000), ("SQ_WAIT_INST_LDS", 250),
                          ("SQ_LDS_BANK_CONFLICT", 10), ("SQ_LDS_IDX_ACTIVE", 100)):
                w.writerow(dict(Dispatch_Id=d, Kernel_Name=name, Counter_Name=cn, Counter_Value=v,
                                Start_Timestamp=0, End_Timestamp=10000))
    st = tmp_path / "st.csv"
    with open(st, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Name", "AverageNs"])
        w.writeheader()
        w.writerow(dict(Name=name, AverageNs=20000))
    m.main(str(cc), str(st))
    line = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("conv_k")][0].split()
    # kernel name has a space: "conv_k<128," "64>"
    assert line[2] == "2" and line[3] == "5.12"
    assert line[4] == "512" and line[5] == "256"
    assert line[7] == "0.100" and line[8] == "0.250"
