"""Caches keyed by tensor addresses (host-side checks and derived index
tensors computed once per batch tensor)."""
from __future__ import annotations

import weakref
from typing import Dict, Tuple


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
        return hit[1]

    def __contains__(self, key):
        hit = self.d.get(key)
        return hit is not None and all(r() is not None for r in hit[0])

    def __getitem__(self, key):
        return self.d[key][1]

    def put(self, key, tensors, val):
        if len(self.d) > self.cap:
            self.d.clear()
        self.d[key] = (tuple(weakref.ref(t) for t in tensors), val)

    def clear(self):
        self.d.clear()
