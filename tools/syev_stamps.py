import numpy as np, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from xerus_amd import capi
h = capi.Handle(0)
for n in (20, 64, 128, 256):
    B = np.random.default_rng(0).standard_normal((n, 20 * n)); A = B @ B.T
    lam, Ut, st = h.sym_eig_top(h.array(A), n // 2)
    print(n, st, flush=True)
