"""CPU restatement of the reference's prioritized-replay sum tree -- TEST
INFRASTRUCTURE ONLY (the checker for trx_per32_*; never imported by the
product).  Pinned against tests/golden/per_tree_ref.npz, which the reference's
own ReplayBuffer class produced (tools/gen_golden_r2.py).

src/train.py:27-91 under numpy >= 2 (NEP 50) scalar rules, spelled out:
  _set_priority (train.py:43-48): delta = fl32(p) - leaf   (Python float p is
      "weak", so the subtraction runs in float32), then leaf and every ancestor
      += delta in float32, leaf first, root last;
  add (train.py:50-59): priority = max_p + eps (float64), max_p = priority,
      p = priority ** alpha (float64 pow);
  sample (train.py:61-84): total = float(tree[1]); r = u * total is a Python
      float, rounded to float32 at its first comparison with a float32 node and
      float32 from the first subtraction on, so r = fl32(u * total) throughout;
      probs = pri / fl32(total), weights = (fl32(size) * probs) ** fl32(-beta),
      weights /= max -- all float32;
  update_priorities (train.py:86-91): in order, priority = |err| + eps
      (float64), max_p = max(max_p, priority), _set_priority(i, priority ** alpha).
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


class RefTree:
    def __init__(self, capacity: int, alpha: float = 0.6, beta: float = 0.4, eps: float = 1e-6):
        self.capacity, self.alpha, self.beta, self.eps = int(capacity), float(alpha), float(beta), float(eps)
        self.tree = np.zeros(2 * self.capacity, dtype=np.float32)
        self.max_p = 1.0
        self.ptr = 0
        self.size = 0

    def set_priority(self, i: int, p: float):
        t = i + self.capacity
        delta = f32(f32(p) - self.tree[t])
        while t >= 1:
            self.tree[t] = f32(self.tree[t] + delta)
            t //= 2

    def add(self):
        pr = abs(self.max_p) + self.eps
        self.max_p = max(self.max_p, pr)
        self.set_priority(self.ptr, pr ** self.alpha)
        self.ptr = (self.ptr + 1) % self.capacity
        self.size = min(self.size + 1, self.capacity)

    def sample(self, u: np.ndarray):
        total = float(self.tree[1])
        idx = np.zeros(len(u), dtype=np.int64)
        pri = np.zeros(len(u), dtype=np.float32)
        for k, uk in enumerate(u):
            r = f32(float(uk) * total)
            node = 1
            while node < self.capacity:
                left = 2 * node
                if r <= self.tree[left]:
                    node = left
                else:
                    r = f32(r - self.tree[left])
                    node = left + 1
            idx[k], pri[k] = node - self.capacity, self.tree[node]
        probs = (pri / f32(total)).astype(np.float32)
        w = ((f32(self.size) * probs).astype(np.float32) ** f32(-self.beta)).astype(np.float32)
        w = (w / (w.max() if w.max() > 0 else f32(1.0))).astype(np.float32)
        return idx, pri, w

    def update_priorities(self, idx, err):
        for i, e in zip(idx, err):
            pr = abs(float(e)) + self.eps
            self.max_p = max(self.max_p, pr)
            self.set_priority(int(i), pr ** self.alpha)
