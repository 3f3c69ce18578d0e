"""CPU restatement of the reference's indexed-expression semantics (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module; the product
path (libxerus_amd) never calls it.

An expression is written with string tokens: "i" (span 1), "i^2" (span 2), "i&1" (all but 1 mode),
"i/2" (half of the modes), or an integer (fixed index / slice). Semantics follow
  - span resolution per tensor: index.cpp:64-92 (set_span), indexedTensorReadOnly.cpp:81-115;
  - an index twice within one factor = trace, twice across factors = contraction, once = open
    (indexedTensorReadOnly.cpp:92-105, tensorNetwork.cpp:598-653), three times = error (:571);
  - the LHS spans are resolved against the number of open modes of the RHS and every LHS index must be
    open on the RHS exactly once (indexedTensorWritable.cpp:97-118, indexedTensor_tensor_evaluate.cpp:286-290);
  - fixed indices slice their mode (tensorNetwork.cpp:655-672, evaluate.cpp:330-331).
The arithmetic is numpy.einsum in float64.
"""
from __future__ import annotations

import re
import string

import numpy as np

_TOKEN = re.compile(r"^([A-Za-z_]\w*)(?:([\^&/])(\d+))?$")


class ExpressionError(ValueError):
    """Raised where the reference throws misc::generic_error."""


def parse(token):
    """token -> (name or None, op, n, fixed position or None)."""
    if isinstance(token, int):
        return (None, "^", 1, token)
    m = _TOKEN.match(token)
    if not m:
        raise ValueError(f"bad index token {token!r}")
    name, op, n = m.group(1), m.group(2) or "^", int(m.group(3) or 1)
    return (name, op, n, None)


def actual_span(op, n, degree):
    """Index::actual_span (index.cpp:80-93)."""
    if op == "&":
        if n > degree:
            raise ExpressionError("Index with inverse span would have negative actual span")
        return degree - n
    if op == "/":
        if n == 0 or degree % n:
            raise ExpressionError("Fractional span must divide the tensor degree")
        return degree // n
    return n


def resolve(tokens, degree):
    """[(name, span, fixed)] with span-0 indices removed; total span must equal degree."""
    out, total = [], 0
    for t in tokens:
        name, op, n, fixed = parse(t)
        span = actual_span(op, n, degree)
        total += span
        if span:
            out.append((name, span, fixed))
    if total != degree:
        raise ExpressionError(f"Order determined by Indices ({total}) differs from the tensor order ({degree})")
    return out


def evaluate(lhs, terms, scale=1.0):
    """lhs: list of tokens; terms: list of (ndarray, tokens). Returns the LHS ndarray."""
    letters = iter(string.ascii_letters)
    label_letter = {}
    subs, operands, order = [], [], []   # order: open labels in appearance order
    counts = {}
    for arr, tokens in terms:
        arr = np.asarray(arr, dtype=np.float64)
        res = resolve(tokens, arr.ndim)
        sl, labels, mode = [], [], 0
        seen_here = {}
        for name, span, fixed in res:
            if fixed is not None:
                if fixed >= arr.shape[mode]:
                    raise ExpressionError("fixed index out of range")
                sl.append(fixed)
                mode += 1
                continue
            seen_here[name] = seen_here.get(name, 0) + 1
            if seen_here[name] > 2:
                raise ExpressionError("An index must not appere more than twice!")
            for s in range(span):
                sl.append(slice(None))
                labels.append((name, s))
            mode += span
        arr = arr[tuple(sl)] if sl else arr
        for lab in labels:
            if lab not in label_letter:
                label_letter[lab] = next(letters)
        for name in {lab[0] for lab in labels}:
            counts[name] = counts.get(name, 0) + seen_here.get(name, 0)
        subs.append("".join(label_letter[lab] for lab in labels))
        operands.append(arr)
        for lab in labels:
            if lab not in order:
                order.append(lab)
    for name, c in counts.items():
        if c > 2:
            raise ExpressionError("Index must not appear three (or more) times.")
    # open labels: the index name occurs once over all factors
    open_labels = [lab for lab in order if counts[lab[0]] == 1]
    E = len(open_labels)
    out_labels = []
    used = set()
    for name, span, fixed in resolve(lhs, E):
        if fixed is not None:
            raise ExpressionError("Traces and fixed indices are not allowed in the target of evaluation.")
        labs = [lab for lab in open_labels if lab[0] == name]
        if not labs or name in used:
            raise ExpressionError("Every index on the LHS must appear somewhere on the RHS")
        if len(labs) != span:
            raise ExpressionError("The indexSpans in the target and base of evaluation must coincide.")
        used.add(name)
        out_labels += labs
    if len(out_labels) != E:
        raise ExpressionError("All indices of evaluation base must appear in the target")
    spec = ",".join(subs) + "->" + "".join(label_letter[lab] for lab in out_labels)
    return scale * np.einsum(spec, *operands, optimize=False)
