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
