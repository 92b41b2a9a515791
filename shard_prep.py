#!/usr/bin/env python3
"""Shard preparation CLI (reference Module_1/shard_prep.py): ``python shard_prep.py --dataset synthetic``
writes data/shards/ecg_%05d.bin and results/shard_prep_metrics.json.  Functions write_shard,
make_mitbih_windows and make_synth_windows are re-exported with the reference signatures."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from crossscale_ecg.data.shards import write_shard, make_mitbih_windows, make_synth_windows  # noqa: E402,F401
from crossscale_ecg.data.prep import main, run_prep  # noqa: E402,F401

if __name__ == "__main__":
    main()
