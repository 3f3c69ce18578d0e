"""bench.py --gpus N without an outer launcher: the parent starts N rank processes before
anything touches the GPU and relays rank 0's JSON line. CPU only: the ranks are a stub worker."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "bench_stub_rank.py")

_DRIVER = r"""
import json, sys
sys.path.insert(0, %r)
import bench
rc = bench.launch_ranks(%d, ["--steps", "3", "--warmup", "1"], worker=%r, timeout=%r)
loaded = sorted(m for m in sys.modules if m.split(".")[0] in ("torch", "xerus_amd"))
print("LAUNCHER " + json.dumps({"rc": rc, "loaded": loaded}))
"""


def _run(tmp_path, n, fail_rank=None, timeout=60):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["STUB_DIR"] = str(tmp_path)
    if fail_rank is not None:
        env["STUB_FAIL_RANK"] = str(fail_rank)
    p = subprocess.run([sys.executable, "-c", _DRIVER % (ROOT, n, STUB, timeout)], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    lines = p.stdout.strip().splitlines()
    meta = json.loads(lines[-1][len("LAUNCHER "):])
    return meta, lines[:-1], p.stderr


@pytest.mark.parametrize("n", [2, 4])
def test_launcher_starts_n_ranks(tmp_path, n):
    meta, relayed, _ = _run(tmp_path, n)
    assert meta["rc"] == 0
    assert meta["loaded"] == [], "the launcher process must not import torch / the HIP library"
    recs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(n)]
    assert [int(r["RANK"]) for r in recs] == list(range(n))
    assert [int(r["LOCAL_RANK"]) for r in recs] == list(range(n))
    assert {r["WORLD_SIZE"] for r in recs} == {str(n)}
    assert {r["MASTER_ADDR"] for r in recs} == {"127.0.0.1"}
    assert len({r["MASTER_PORT"] for r in recs}) == 1
    assert {r["HSA_ENABLE_IPC_MODE_LEGACY"] for r in recs} == {"0"}
    assert recs[0]["argv"] == ["--steps", "3", "--warmup", "1"]
    # exactly rank 0's last line is relayed
    assert len(relayed) == 1
    line = json.loads(relayed[0])
    assert line == {"metric": "stub", "n_gpus": n, "rank": 0}


def test_launcher_failed_rank_ends_job(tmp_path):
    t0 = time.time()
    meta, relayed, err = _run(tmp_path, 3, fail_rank=1)
    assert meta["rc"] != 0
    assert "rank(s) failed" in err
    assert time.time() - t0 < 45, "the blocked ranks must be ended, not waited for"


def test_main_routes_to_launcher(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench

    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "launch_ranks", lambda n, argv, **kw: calls.append((n, list(argv))) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--steps", "4"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0
    assert calls == [(8, ["--gpus", "8", "--steps", "4"])]
