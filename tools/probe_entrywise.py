import sys, numpy as np
sys.path.insert(0, '/root/repo')
import xerus_amd.xerus as xe
rng = np.random.default_rng(755)
extra = [int(v) for v in rng.integers(1, 4, size=6)]
dims1 = extra[:4]
xe.seed(755)
dimsA = dims1 + dims1
A = xe.Tensor.random(dimsA)
ttA = xe.TTOperator(A, 0.33)
print("ranks", ttA.ranks(), "dims", dimsA)
a = xe.Tensor(ttA).to_ndarray()
C = xe.entrywise_product(ttA, ttA)
c = xe.Tensor(C).to_ndarray()
print("ep op ranks", C.ranks(), "rel err", np.linalg.norm(c - a * a) / np.linalg.norm(a * a))
# merged TT view without canonicalisation
d = len(dims1)
mdims = [dims1[k] * dims1[k] for k in range(d)]
T = xe.TTTensor(mdims)
for k in range(d):
    comp = ttA.get_component(k).to_ndarray()
    T.set_component(k, xe.Tensor.from_ndarray(comp.reshape(comp.shape[0], -1, comp.shape[-1])))
print("T canonical?", T.canonicalized)
E = xe.entrywise_product(T, T)
e = xe.Tensor(E).to_ndarray().reshape(a.shape[:0] + tuple(mdims))
tt_full = xe.Tensor(T).to_ndarray()
print("noncanon ep rel err", np.linalg.norm(xe.Tensor(E).to_ndarray() - tt_full * tt_full) / np.linalg.norm(tt_full ** 2), E.ranks())
E.move_core(0)
print("after move_core(0)", E.ranks(), np.linalg.norm(xe.Tensor(E).to_ndarray() - tt_full * tt_full) / np.linalg.norm(tt_full ** 2))
E2 = xe.entrywise_product(T, T)
E2.move_core(d - 1)
print("after move_core(d-1)", E2.ranks(), np.linalg.norm(xe.Tensor(E2).to_ndarray() - tt_full * tt_full) / np.linalg.norm(tt_full ** 2))
for k in range(d):
    M = E.get_component(k).to_ndarray()
    print(k, M.shape)
