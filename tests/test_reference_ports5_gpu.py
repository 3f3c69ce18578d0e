"""Ports of the reference's last unit tests on the path: src/unitTests/fileIO.cxx:28-100 (read_write_file for
Tensor, TensorNetwork and TT, TSV and binary) and src/unitTests/tensorNetwork_element_access.cxx:27-100
(element_access, many_element_access), with the reference's tolerances.

Differences: the build is dense-only, so the reference's sparse tensors are dense tensors with
the same entries (`TEST(Ab.is_sparse())` does not apply); files of sparse tensors written in the reference's
stream layout (tensor.cpp:1781-1845, representation 2) are read into dense tensors, checked below with files
assembled byte by byte in that layout.
"""
import os
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _approx_equal(a, b, eps=4 * np.finfo(float).eps):
    """misc::approx_equal of two tensors (tensor.cpp approx_equal: ||a-b|| <= eps (||a|| + ||b||) / 2)."""
    return np.linalg.norm(a - b) <= eps * (np.linalg.norm(a) + np.linalg.norm(b)) / 2


def _sparse_entries():
    return {(5, 7, 99): 1.0, (80, 123, 5): 6.0, (1, 2, 3): 4.0, (99, 233, 566): 5.0, (12, 12, 12): 8.0, (15, 15, 15): 7.0,
            (99, 99, 99): 3.0, (65, 65, 65): 2.0}


def test_tensor_read_write_file(xe, tmp_path):
    """Tensor:read_write_file (fileIO.cxx:28-52)."""
    f = str(tmp_path / "test.dat")
    A = xe.Tensor.random([12, 13, 14])
    a = A.to_ndarray()
    for tsv in (True, False):
        xe.save_to_file(A, f, tsv)
        Ab = xe.load_from_file(f)
        assert _approx_equal(a, Ab.to_ndarray()), ("tsv" if tsv else "bin", np.linalg.norm(a - Ab.to_ndarray()))
    # the reference's sparse S (100 x 234 x 567, 8 entries), dense here
    dims = (100, 234, 567)
    s = np.zeros(dims)
    for p, v in _sparse_entries().items():
        s[p] = v
    S = xe.Tensor.from_ndarray(s)
    for tsv in (False, True):
        xe.save_to_file(S, f, tsv)
        Sb = xe.load_from_file(f)
        assert np.linalg.norm(s - Sb.to_ndarray()) < 1e-16


@pytest.mark.parametrize("tsv", [False, True])
def test_tensor_read_sparse_stream(xe, tmp_path, tsv):
    """A file of a SPARSE tensor in the reference's layout (tensor.cpp:1781-1803: version 1, dims, representation 2,
    entry count, (flat position, value) pairs) reads back into the dense tensor with those entries."""
    f = str(tmp_path / "sparse.dat")
    dims = (100, 234, 567)
    entries = _sparse_entries()
    flat = {int(np.ravel_multi_index(p, dims)): v for p, v in entries.items()}
    head = b"Xerus xerus::Tensor datafile.\nFormat: " + (b"TSV" if tsv else b"Binary") + b"\n"
    with open(f, "wb") as fh:
        fh.write(head)
        if tsv:
            vals = [1, len(dims), *dims, 2, len(flat)]
            for pos, v in flat.items():
                vals += [pos, repr(v)]
            fh.write(("\t".join(str(x) for x in vals) + "\t").encode())
        else:
            fh.write(struct.pack("<QQ", 1, len(dims)) + struct.pack("<3Q", *dims) + struct.pack("<QQ", 2, len(flat)))
            for pos, v in flat.items():
                fh.write(struct.pack("<Qd", pos, v))
    got = xe.load_from_file(f).to_ndarray()
    assert got.shape == dims
    expect = np.zeros(dims)
    for p, v in entries.items():
        expect[p] = v
    assert np.array_equal(got, expect)


def test_tensor_network_read_write_file(xe, tmp_path):
    """TensorNetwork:read_write_file (fileIO.cxx:54-75): T(k,l,n) = A(i,j,k) * B(i,l,m) * C(n,j,m) kept as a
    network (no contraction), saved, loaded as a network, < 6e-16 relative."""
    f = str(tmp_path / "test.dat")
    A = xe.Tensor.random([12, 13, 14])
    b = np.zeros((12, 13, 14))
    for p, v in {(1, 1, 1): 1, (2, 3, 4): 2, (7, 10, 3): 3, (5, 12, 13): 4, (8, 7, 6): 5}.items():
        b[p] = v
    B = xe.Tensor.from_ndarray(b)
    C = xe.Tensor.random([12, 13, 14])
    i, j, k, l, m, n = xe.indices(6)
    T = xe.TensorNetwork()
    T(k, l, n) << A(i, j, k) * B(i, l, m) * C(n, j, m)
    assert T.num_nodes() == 3
    t = T.to_tensor().to_ndarray()
    expect = np.einsum("ijk,ilm,njm->kln", A.to_ndarray(), b, C.to_ndarray())
    assert np.linalg.norm(t - expect) <= 1e-12 * np.linalg.norm(expect)
    for tsv in (True, False):
        xe.save_to_file(T, f, tsv)
        Tb = xe.load_network_from_file(f)
        assert list(T.dimensions) == list(Tb.dimensions)
        Tb.require_valid_network()
        assert np.linalg.norm(t - Tb.to_tensor().to_ndarray()) / np.linalg.norm(t) < 6e-16


def test_tt_read_write_file(xe, tmp_path):
    """TT:read_write_file (fileIO.cxx:78-92)."""
    f = str(tmp_path / "test.dat")
    A = xe.TTTensor.random([7, 8, 9, 10], [2, 2, 2])
    xe.save_to_file(A, f)
    with pytest.raises(Exception):
        xe.load_network_from_file(f)          # FAILTEST: a TT file is not a TensorNetwork file
    Ab = xe.load_tt_from_file(f)
    Ab.require_correct_format()
    assert Ab.canonicalized and Ab.corePosition == 0
    assert list(A.dimensions) == list(Ab.dimensions)
    a, ab = xe.Tensor(A).to_ndarray(), xe.Tensor(Ab).to_ndarray()
    assert np.linalg.norm(a - ab) / np.linalg.norm(a) < 6e-16


def _ab(xe):
    A = xe.Tensor([1, 2])
    B = xe.Tensor([2, 3])
    A[[0, 0]] = 1
    A[[0, 1]] = 2
    for (p, v) in {(0, 0): 3, (0, 1): 4, (0, 2): 5, (1, 0): 6, (1, 1): 7, (1, 2): 8}.items():
        B[list(p)] = v
    return A, B


def test_tensor_network_element_access(xe):
    """TensorNetwork:element_access (tensorNetwork_element_access.cxx:26-63)."""
    A, B = _ab(xe)
    i, j, k, l = xe.indices(4)
    res = xe.TensorNetwork()
    res(i, j, k, l) << A(i, j) * B(k, l)        # no index contracted
    assert res.num_nodes() == 2
    resX = [3, 4, 5, 6, 7, 8, 6, 8, 10, 12, 14, 16]
    for t in range(int(np.prod(res.dimensions))):
        assert np.isclose(res[t], resX[t], rtol=4 * np.finfo(float).eps, atol=0)
    assert np.isclose(res[[0, 1, 1, 1]], 14.0, rtol=4 * np.finfo(float).eps, atol=0)
    res(k, i) << B(j, k) * A(i, j)              # one index contracted
    for t, v in enumerate([15.0, 18.0, 21.0]):
        assert np.isclose(res[t], v, rtol=4 * np.finfo(float).eps, atol=0)
    for p, v in (([0, 0], 15.0), ([1, 0], 18.0), ([2, 0], 21.0)):
        assert np.isclose(res[p], v, rtol=4 * np.finfo(float).eps, atol=0)


def test_tensor_network_many_element_access(xe):
    """TensorNetwork:many_element_access (tensorNetwork_element_access.cxx:66-100)."""
    A, B = _ab(xe)
    i, j, k, l = xe.indices(4)
    res = xe.TensorNetwork()
    res(i, j, k, l) << A(i, j) * B(k, l)
    ms = xe.SinglePointMeasurementSet()
    for p in [[0, 0, 0, 0], [0, 0, 0, 1], [0, 0, 0, 2], [0, 0, 1, 0], [0, 0, 1, 1], [0, 0, 1, 2],
              [0, 1, 0, 0], [0, 1, 0, 1], [0, 1, 0, 2], [0, 1, 1, 0], [0, 1, 1, 1], [0, 1, 1, 2]]:
        ms.add(p, 0.0)
    ms.measure(res)
    for m in range(ms.size()):
        assert np.isclose(ms.measuredValues[m], res[ms.positions[m]], rtol=4 * np.finfo(float).eps, atol=0)
    assert ms.test(res) < 1e-15
