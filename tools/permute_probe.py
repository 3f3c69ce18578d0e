"""The bench's permutation shapes (bench.py bench_permute: dispatch timestamps, rotated buffers), one line each.
    python tools/permute_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from xerus_amd import capi  # noqa: E402

h = capi.Handle(0)
for r in bench.bench_permute(h):
    print(json.dumps({k: r[k] for k in ("shape", "mbytes", "us", "gbs", "frac_hbm_peak")}), flush=True)
