#!/usr/bin/env python3
"""Run bench.py's C5 leg at a chosen scale and print its parity block (development)."""
import json
import os
import sys
from argparse import Namespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from veneur_amd.dist import Group  # noqa: E402

for spec in sys.argv[1:]:
    hosts, hk, sk, batch = (int(x) for x in spec.split(",")[:4])
    r = bench.c5_leg(Namespace(seed=1, c5_histo_keys=hk, c5_set_keys=sk, c5_hosts=hosts, c5_windows=1,
                               c5_parity_keys=16, c5_batch=batch, c5_group=50), 0, 1, Group(), 0)
    print(spec, json.dumps(r["parity"]), round(r["ms_per_window"], 1), json.dumps(r["phases_ms_synchronised"]), json.dumps(r["kernel_ms_timing_mode_rank0"]), flush=True)
