"""ORACLE - test infrastructure only.  numpy reduction order, restated (SURVEY.md §8 a-R).

The HIP reduction kernels reproduce exactly this order so that channel / time-bin
masks are bit-exact.  tests/test_numpy_order.py checks these emulations against
numpy itself on ragged shapes, so a numpy upgrade that changed the order would be
caught on CPU before any GPU parity test.

* ``add.reduce`` of a contiguous vector (``mean(1)``, ``sum(1)``, ``std`` pieces):
  the accumulator starts at 0 and adds, block by block, the numpy ``pairwise_sum``
  of consecutive 8192-element buffers.
* ``pairwise_sum(a, n)``: n < 8 sequential; n <= 128: 8 strided accumulators
  combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the n%8 tail sequentially;
  otherwise split at n2 = n/2 - (n/2)%8 and add the two halves.
* ``mean(0)`` of a C-contiguous 2-D array: sequential over rows.
"""
import numpy as np


def pairwise_sum(a):
    a = np.asarray(a)
    dt = a.dtype.type
    n = a.size
    if n < 8:
        r = dt(0)
        for i in range(n):
            r = dt(r + a[i])
        return r
    if n <= 128:
        r = [a[j] for j in range(8)]
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] = dt(r[j] + a[i + j])
            i += 8
        res = dt(dt(dt(r[0] + r[1]) + dt(r[2] + r[3])) + dt(dt(r[4] + r[5]) + dt(r[6] + r[7])))
        while i < n:
            res = dt(res + a[i])
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return dt(pairwise_sum(a[:n2]) + pairwise_sum(a[n2:]))


def reduce_sum(a, block=8192):
    a = np.asarray(a)
    dt = a.dtype.type
    r = dt(0)
    for s in range(0, a.size, block):
        r = dt(r + pairwise_sum(a[s:s + block]))
    return r


def row_sums(x):
    return np.array([reduce_sum(r) for r in np.asarray(x)], dtype=np.asarray(x).dtype)


def col_sums(x):
    x = np.asarray(x)
    acc = np.zeros(x.shape[1], x.dtype)
    for r in x:
        acc = (acc + r).astype(x.dtype)
    return acc
