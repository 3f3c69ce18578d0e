"""Contraction-order parity of the expression engine ("must stay identical").

value_t(x(i&0) * y(i&0)) builds a 2d+4-node TensorNetwork (x: ghost 0, cores 1..d, ghost d+1; y: the
same from d+2; ttNetwork.cpp:57-108, tensorNetwork.cpp:553-675) and contracts it in the order chosen by
the reference's heuristics (5 greedy scores + exchange, contractionHeuristic.cpp:35-381, picked in
tensorNetwork.cpp:1316-1329). SURVEY §3.4 traced the reference at order 12, n = 20, rank 256: the ghost
nodes and the two boundary core pairs are merged first, then a strict left-to-right zipper E*X_k over
one mode, (E*X_k)*Y_k over two modes. Host-only planning: runs without a GPU.
"""
import pytest

import bench


def _expected_zipper(d):
    gx, gy = 0, d + 2                       # first ghost of x / of y
    xc = lambda k: gx + 1 + k               # noqa: E731  (core k of x, k = 0..d-1)
    yc = lambda k: gy + 1 + k               # noqa: E731
    order = [(0, d + 1), (0, gy), (0, gy + d + 1),          # the four ghosts
             (xc(0), yc(0)), (xc(d - 1), yc(d - 1)),          # the two boundary core pairs
             (0, xc(0))]                                      # ghosts * left boundary pair
    for k in range(1, d - 1):
        order += [(0, xc(k)), (0, yc(k))]                     # E * X_k, then (E X_k) * Y_k
    order.append((0, xc(d - 1)))                              # close with the right boundary pair
    return order


@pytest.mark.parametrize("d,n,r", [(12, 20, 256), (10, 20, 256), (10, 20, 128), (8, 20, 64)])
def test_tt_dot_order_is_the_traced_zipper(d, n, r):
    import xerus_amd.xerus as xe

    ranks = bench.tt_ranks(d, n, r)
    order = [tuple(p) for p in xe.tt_dot_contraction_order([n] * d, ranks, ranks)]
    assert len(order) == 2 * d + 3
    assert order == _expected_zipper(d)
