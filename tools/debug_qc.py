import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from xerus_amd import capi
from oracle import xerus_ref as ref
h = capi.Handle(0)
rng = np.random.default_rng(600 + 200 + 50)
A = rng.standard_normal((600, 50)) @ rng.standard_normal((50, 200))
print("calling qc", flush=True)
Q, C, r = h.qc(h.array(A))
print("qc returned rank", r, "ref", ref.qc(A)[2], flush=True)
h.synchronize()
print("synced", flush=True)
Qh = Q.numpy(); Ch = C.numpy()
print("err", np.linalg.norm(Qh @ Ch - A) / np.linalg.norm(A), flush=True)
