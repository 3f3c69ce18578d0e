"""Stub rank for tests/test_bench_launcher_cpu.py: records the rank environment bench.launch_ranks gives it
(no GPU, no torch), prints one JSON line like a bench rank, and fails on request."""
import json
import os
import sys
import time

rank = int(os.environ["RANK"])
rec = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                                      "HSA_ENABLE_IPC_MODE_LEGACY")}
rec["argv"] = sys.argv[1:]
with open(os.path.join(os.environ["STUB_DIR"], f"rank{rank}.json"), "w") as f:
    json.dump(rec, f)
if os.environ.get("STUB_FAIL_RANK") == str(rank):
    sys.exit(3)
if os.environ.get("STUB_FAIL_RANK") is not None:
    time.sleep(60)          # a healthy rank blocked in a collective: the launcher must end it
print("noise line")
print(json.dumps({"metric": "stub", "n_gpus": int(rec["WORLD_SIZE"]), "rank": rank}))
