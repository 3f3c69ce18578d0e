"""The indexed-expression oracle (oracle/indexed.py) against the reference's hand-computed answers."""
import json
import os

import numpy as np
import pytest

from oracle import indexed

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_products.json")))


def _inputs(case):
    return {k: np.array(v["values"], dtype=np.float64).reshape(v["dims"]) for k, v in case["inputs"].items()}


@pytest.mark.parametrize("case", GOLDEN["cases"], ids=[c["name"] for c in GOLDEN["cases"]])
def test_oracle_known_answers(case):
    arrs = _inputs(case)
    out = indexed.evaluate(case["lhs"], [(arrs[n], toks) for n, toks in case["rhs"]], case["scale"])
    np.testing.assert_array_equal(out.reshape(-1), np.array(case["expected"], dtype=np.float64))


@pytest.mark.parametrize("case", GOLDEN["errors"], ids=[c["name"] for c in GOLDEN["errors"]])
def test_oracle_rejects(case):
    A = np.zeros(case["dims"])
    B = np.zeros(case.get("dims_b", [1]))
    arrs = {"A": A, "B": B}
    with pytest.raises(indexed.ExpressionError):
        indexed.evaluate(case["lhs"], [(arrs[n], toks) for n, toks in case["rhs"]])


def test_oracle_three_occurrences_rejected():
    a = np.ones((2, 2))
    with pytest.raises(indexed.ExpressionError):
        indexed.evaluate([], [(a, ["i", "j"]), (a, ["j", "k"]), (a, ["j", "k"])])


def test_oracle_scale_and_chain():
    rng = np.random.default_rng(1)
    A, B, C = rng.standard_normal((3, 4)), rng.standard_normal((4, 5)), rng.standard_normal((5, 3))
    out = indexed.evaluate(["i", "l"], [(A, ["i", "j"]), (B, ["j", "k"]), (C, ["k", "l"])], scale=2.0)
    np.testing.assert_allclose(out, 2.0 * A @ B @ C, rtol=1e-13)
