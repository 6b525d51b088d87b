"""The zamboni heap (mt_core.h heapAdd / heapGet: the wave-parallel sift for up to 63 entries and
the scalar one above) pops in exactly the order of the reference's Heap (MT/collections.ts:214-267),
ties included: which block a zamboni pass scours first depends on it.  Runs the engine's code in
the host emulation (tests/emu) against a restatement of that class."""
import ctypes

import numpy as np
import pytest

from emu_lib import emu_engine


class RefHeap:
    """collections.ts Heap with the zamboni comparer (maxSeq): add = push + fixup, get = last
    to the root + fixdown (left child on ties; stop when the moving entry is <= the child)."""

    def __init__(self):
        self.L = [None]

    def add(self, x):
        self.L.append(x)
        k = len(self.L) - 1
        while k > 1 and self.L[k >> 1][1] > self.L[k][1]:
            self.L[k >> 1], self.L[k] = self.L[k], self.L[k >> 1]
            k >>= 1

    def get(self):
        x = self.L[1]
        self.L[1] = self.L[-1]
        self.L.pop()
        n, k = len(self.L) - 1, 1
        while 2 * k <= n:
            j = 2 * k
            if j < n and self.L[j][1] > self.L[j + 1][1]:
                j += 1
            if self.L[k][1] <= self.L[j][1]:
                break
            self.L[k], self.L[j] = self.L[j], self.L[k]
            k = j
        return x


def _ops(rng, n, key_range, max_size):
    ops, size = [], 0
    for _ in range(n):
        if size and (size >= max_size or rng.random() < 0.45):
            ops.append(-1); size -= 1
        else:
            ops.append(int(rng.integers(0, key_range))); size += 1
    return ops


@pytest.mark.parametrize("key_range,max_size", [(4, 20), (16, 63), (1000, 63), (8, 64), (32, 200)])
def test_heap_pop_order_matches_reference(key_range, max_size):
    eng = emu_engine(1, heap_per_doc=256)
    eng.open_docs(0, 1)
    f = eng.lib.emu_test_heap
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    f.restype = ctypes.c_int
    rng = np.random.default_rng(key_range * 1000 + max_size)
    for _ in range(20):
        ops = _ops(rng, 600, key_range, max_size)
        ref, want = RefHeap(), []
        for i, o in enumerate(ops):
            if o >= 0:
                ref.add((i, o))
            else:
                want.append(ref.get())
        while len(ref.L) > 1:                        # drain: every entry leaves in order
            ops.append(-1); want.append(ref.get())
        a = np.asarray(ops, np.int32)
        out = np.zeros(2 * len(want), np.int32)
        np_ = f(eng.h, 0, a.ctypes.data, len(a), out.ctypes.data)
        assert np_ == len(want)
        assert [tuple(p) for p in out.reshape(-1, 2).tolist()] == want
    eng.close()
