"""Caches keyed by tensor addresses (host-side checks and derived index
tensors computed once per batch tensor).

A captured HIP graph holds raw pointers to whatever cached tensors its
kernels read (CSR arrays, int32 index copies, topologies).  The caches drop
entries (a full cache is cleared), so a capture runs under `pinning()`:
every cached value looked up or stored while it is active is appended to a
list the graph wrapper keeps alive for as long as the graph can be replayed.
"""
from __future__ import annotations

import weakref
from contextlib import contextmanager
from typing import Dict, List, Tuple

_PIN_STACK: List[list] = []


def pin(val):
    """Keep `val` alive for the innermost active pinning() scope."""
    if _PIN_STACK and val is not None:
        _PIN_STACK[-1].append(val)
    return val


@contextmanager
def pinning():
    """Collect every cache value used inside the scope (yields the list)."""
    pins: list = []
    _PIN_STACK.append(pins)
    try:
        yield pins
    finally:
        _PIN_STACK.pop()


class TensorKeyed:
    """Cache keyed by tensors' (address, version, ...).  An entry is valid only
    while the tensors it was computed from are alive: a new tensor allocated
    at a dead one's address with the same version counter must not see the
    dead tensor's entry (it may hold other data)."""

    def __init__(self, cap: int = 64):
        self.d: Dict[Tuple, Tuple] = {}
        self.cap = cap

    def get(self, key, default=None):
        hit = self.d.get(key)
        if hit is None or any(r() is None for r in hit[0]):
            return default
        return pin(hit[1])

    def __contains__(self, key):
        hit = self.d.get(key)
        return hit is not None and all(r() is not None for r in hit[0])

    def __getitem__(self, key):
        return pin(self.d[key][1])

    def put(self, key, tensors, val):
        if len(self.d) > self.cap:
            # dead entries first; clear everything only when all are live
            dead = [k for k, (refs, _) in self.d.items() if any(r() is None for r in refs)]
            for k in dead:
                del self.d[k]
            if len(self.d) > self.cap:
                self.d.clear()
        self.d[key] = (tuple(weakref.ref(t) for t in tensors), pin(val))

    def clear(self):
        self.d.clear()
