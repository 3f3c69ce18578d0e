"""Test helpers: TT difference norms without cancellation (test infrastructure, numpy only)."""
import numpy as np


def tt_diff_norm(a_cores, b_cores):
    """(||A - B||, ||B||) of two TTs of equal dims (block-diagonal difference, QR sweep)."""
    d = len(a_cores)

    def orth_norm(cores):
        carry = None
        for k, c in enumerate(cores):
            if carry is not None:
                c = np.tensordot(carry, c, axes=(1, 0))
            if k == d - 1:
                return float(np.linalg.norm(c))
            a, n, b = c.shape
            q, rr = np.linalg.qr(c.reshape(a * n, b))
            carry = rr
        return 0.0

    diff = []
    for k, (A, B) in enumerate(zip(a_cores, b_cores)):
        B = -B if k == 0 else B
        a1, n, b1 = A.shape
        a2, _, b2 = B.shape
        if k == 0:
            diff.append(np.concatenate([A, B], axis=2))
        elif k == d - 1:
            diff.append(np.concatenate([A, B], axis=0))
        else:
            Z = np.zeros((a1 + a2, n, b1 + b2))
            Z[:a1, :, :b1] = A
            Z[a1:, :, b1:] = B
            diff.append(Z)
    return orth_norm(diff), orth_norm([c.copy() for c in b_cores])


def read_xerus_file(path):
    """Parse a BINARY xerus datafile (misc/fileIO.h:103-118) with numpy: (type name, payload dict).
    Tensor (tensor.cpp:1781-1804), TensorNetwork (tensorNetwork.cpp:1429-1466), TTNetwork<false>
    (ttNetwork.cpp:1455-1468). Dense tensors only."""
    import struct

    raw = open(path, "rb").read()
    l1 = raw.index(b"\n")
    l2 = raw.index(b"\n", l1 + 1)
    head = raw[:l1].decode()
    assert head.startswith("Xerus ") and head.endswith(" datafile."), head
    assert raw[l1 + 1:l2] == b"Format: Binary"
    kind = head[len("Xerus "):-len(" datafile.")]
    pos = [l2 + 1]

    def u64():
        v = struct.unpack_from("<Q", raw, pos[0])[0]
        pos[0] += 8
        return v

    def boolean():
        v = raw[pos[0]] != 0
        pos[0] += 1
        return v

    def tensor():
        assert u64() == 1
        dims = [u64() for _ in range(u64())]
        assert u64() == 1
        n = int(np.prod(dims)) if dims else 1
        data = np.frombuffer(raw, dtype="<f8", count=n, offset=pos[0]).copy()
        pos[0] += 8 * n
        return {"dims": dims, "data": data}

    def network():
        assert u64() == 1
        dims = [u64() for _ in range(u64())]
        ext = [(u64(), u64(), u64()) for _ in dims]
        nodes = []
        for _ in range(u64()):
            nodes.append({"links": [(boolean(), u64(), u64(), u64()) for _ in range(u64())]})
        for nd in nodes:
            nd["tensor"] = tensor()
        return {"dims": dims, "external": ext, "nodes": nodes}

    if kind == "xerus::Tensor":
        out = tensor()
    elif kind == "xerus::TensorNetwork":
        out = network()
    else:
        assert u64() == 1
        out = {"canonicalized": boolean(), "corePosition": u64()}
        out["network"] = network()
    assert pos[0] == len(raw), "trailing bytes"
    return kind, out
