"""Every XRS_* environment switch the library reads, each run in a subprocess
(tests/switch_probe.py: the switches are read once per process): results stay within the parity bars and
each switch has its documented effect (path taken, diagnostics printed)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _probe(env):
    e = dict(os.environ)
    for k in list(e):
        if k.startswith("XRS_"):
            del e[k]
    e.update(env)
    p = subprocess.run([sys.executable, os.path.join(HERE, "switch_probe.py")], env=e, capture_output=True, text=True,
                       timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line), p.stderr


def _bars(r):
    assert r["gemm_err"] <= 1e-13
    assert r["sgemm_err"] <= 1e-6
    assert r["dot_err"] <= 1e-12 and r["dot_async_err"] <= 1e-12
    assert r["dot32_err"] <= 1e-6
    assert r["chain_path"] == "chain" and r["chain_err"] <= 1e-10
    assert r["trunc_ranks_ok"] and r["trunc_err_diff"] <= 1e-6
    assert r["graded_ranks_ok"] and r["graded_err_diff"] <= 1e-6
    assert r["flat_ranks_ok"] and r["flat_err_ok"]
    assert r["svd_err"] <= 1e-12 and r["eig_err"] <= 1e-12
    assert r["api_svd_res"] <= 1e-14 and r["api_svd_orth"] <= 1e-14


@pytest.mark.parametrize("env,check", [
    ({}, lambda r, err: r["trunc_path"] == "truncate" and r["graded_path"] == "general" and r["flat_path"] in ("general", "reference")),
    ({"XRS_DOT_GATE": "0"}, lambda r, err: True),                                      # ungated async product
    ({"XRS_GEMM_GLDS": "0"}, lambda r, err: True),                                     # general GEMM kernel only
    ({"XRS_GEMM_CFG": "2,256,512"}, lambda r, err: True),                              # forced 64x64 tiles
    ({"XRS_NO_GENERAL_ROUND": "1"}, lambda r, err: r["graded_path"] == "reference"),   # reference sweep
    ({"XRS_TRUNC_JACOBI": "1"}, lambda r, err: r["trunc_path"] == "truncate"),         # Jacobi kept subspace
    ({"XRS_SYEV_MAX": "16"}, lambda r, err: r["trunc_path"] == "truncate"),            # eigensolver order cap
    ({"XRS_DEBUG_ROUND": "1"}, lambda r, err: "round_truncate:" in err and "round_general:" in err),
    ({"XRS_STAMPS": "all"}, lambda r, err: "[round host us]" in err and "jacobi_vt p=" in err and "k_sytrd n=" in err),
    ({"XRS_SYNC_DEBUG": "1"}, lambda r, err: "[xrs] launched k_gemm" in err),
    ({"XRS_JACOBI_NO_EARLY": "1"}, lambda r, err: r["graded_path"] == "general" and r["flat_path"] in ("general", "reference")),
    ({"XRS_GLDS_ST2": "0"}, lambda r, err: True),                                      # 3-stage LDS-DMA tiles
    ({"XRS_SG_TARGET": "96"}, lambda r, err: True),                                    # fp32 split-K target
    ({"XRS_SGEMM": "1,8"}, lambda r, err: True),                                       # forced fp32 tile / split
    ({"XRS_GLDS_XCD_SPLIT": "0"}, lambda r, err: True),                                # plain split-K order
    ({"XRS_SG_XCD_SPLIT": "1"}, lambda r, err: True),                                  # fp32 split-K per XCD
    ({"XRS_REDUCE_SYM": "0"}, lambda r, err: True),                                    # elementwise sym reduce
    ({"XRS_SVD_BIDIAG": "0"}, lambda r, err: True),                                    # Jacobi-only dense SVD
    ({"XRS_ZIP32": "1"}, lambda r, err: True),                                         # fused zipper front end
    ({"XRS_ZIP32": "2", "XRS_ZIP_STAMPS": "1"}, lambda r, err: "[zip stamps]" in err),  # fused zipper + stamps
], ids=["default", "dot_gate", "gemm_glds", "gemm_cfg", "no_general", "trunc_jacobi", "syev_max", "debug_round",
        "stamps", "sync_debug", "jacobi_no_early", "glds_st2", "sg_target", "sgemm", "glds_xcd_split", "sg_xcd_split",
        "reduce_sym", "svd_bidiag", "zip32_front", "zip32_stamps"])
def test_switch(env, check):
    r, err = _probe(env)
    _bars(r)
    assert check(r, err), (r, err[-2000:])
