"""Scenario-tree index arithmetic (BFS order of ``MPC_branch.inittree``, :1678-1747).

Mirrors what the C++ plan builder computes, for host-side unpacking (BT2array, BranchTree
views)."""
from __future__ import annotations


class TreeIndex:
    def __init__(self, N, NB, m):
        self.N, self.NB, self.m = N, NB, m
        self.depth, self.length, self.parent, self.children = [0], [1], [-1], [[]]
        self.ndx, self.ndu = [0], [0]
        cx = cu = 1
        queue = [0]
        while queue:
            b = queue.pop(0)
            if self.depth[b] >= NB:
                continue
            for _ in range(m):
                c = len(self.depth)
                self.depth.append(self.depth[b] + 1)
                self.length.append(N)
                self.parent.append(b)
                self.children.append([])
                self.children[b].append(c)
                self.ndx.append(cx)
                self.ndu.append(cu)
                cx += N + 1 if self.depth[c] == NB else N
                cu += N
                queue.append(c)
        self.T, self.U = cx, cu
        self.bdim = sum(1 for d in self.depth if d < NB)

    @property
    def nbranch(self):
        return len(self.depth)

    def is_leaf(self, b):
        return self.depth[b] == self.NB
