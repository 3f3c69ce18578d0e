"""Which certificate of the truncating round fails for the test_round_truncating cfg3 input (diagnostics)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import xerus_ref as ref  # noqa: E402
from xerus_amd import capi  # noqa: E402

h = capi.Handle(0)
x = ref.TT.random([20] * 10, [128] * 9, ref.Rng(13))
g = capi.TTDevice.from_cores(h, x.cores, canonicalized=True, core_position=0)
g.round(64)
print("path", h.last_round_path(), g.ranks)
