"""Literal pure-Python restatement of ORBextractor::DistributeOctTree
(ORBextractor.cc:667-1013) for small inputs: the std::list is a Python list with
push_front = insert(0, ...), nodes carry an allocation counter standing in for their
heap address (hazard H1: ties in the final-phase sort go to the later allocation).
Used only to cross-check the C oracle and the GPU kernel.
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32


class Node:
    __slots__ = ("ul", "ur", "bl", "br", "keys", "no_more", "seq")

    def __init__(self):
        self.keys = []
        self.no_more = False
        self.seq = -1


def divide(n: Node, pts):
    hx = math.ceil(F32(n.ur[0] - n.ul[0]) / F32(2))
    hy = math.ceil(F32(n.br[1] - n.ul[1]) / F32(2))
    c = [Node() for _ in range(4)]
    c[0].ul = n.ul
    c[0].ur = (n.ul[0] + hx, n.ul[1])
    c[0].bl = (n.ul[0], n.ul[1] + hy)
    c[0].br = (n.ul[0] + hx, n.ul[1] + hy)
    c[1].ul, c[1].ur, c[1].bl, c[1].br = c[0].ur, n.ur, c[0].br, (n.ur[0], n.ul[1] + hy)
    c[2].ul, c[2].ur, c[2].bl, c[2].br = c[0].bl, c[0].br, n.bl, (c[0].br[0], n.bl[1])
    c[3].ul, c[3].ur, c[3].bl, c[3].br = c[2].ur, c[1].br, c[2].br, n.br
    for k in n.keys:
        x, y = pts[k][0], pts[k][1]
        if x < c[0].ur[0]:
            c[0 if y < c[0].br[1] else 2].keys.append(k)
        else:
            c[1 if y < c[0].br[1] else 3].keys.append(k)
    for ch in c:
        if len(ch.keys) == 1:
            ch.no_more = True
    return c


def distribute_octree(pts, minX, maxX, minY, maxY, N):
    """pts: list of (x, y, response) relative to (minX, minY).  Returns kept indices in list order."""
    seq = [0]

    def alloc(node):
        node.seq = seq[0]
        seq[0] += 1
        return node

    nIni = int(math.floor(float(F32(maxX - minX) / F32(maxY - minY)) + 0.5))  # std::round (half away)
    hX = F32(maxX - minX) / F32(nIni)
    lst = []
    ini = []
    for i in range(nIni):
        n = Node()
        n.ul = (int(hX * F32(i)), 0)
        n.ur = (int(hX * F32(i + 1)), 0)
        n.bl = (n.ul[0], maxY - minY)
        n.br = (n.ur[0], maxY - minY)
        lst.append(alloc(n))
        ini.append(n)
    for k, p in enumerate(pts):
        ini[int(F32(p[0]) / hX)].keys.append(k)
    lst = [n for n in lst if len(n.keys) > 0]
    for n in lst:
        if len(n.keys) == 1:
            n.no_more = True

    finish = False
    vsize = []
    while not finish:
        prev = len(lst)
        nexp = 0
        vsize = []
        i = 0
        while i < len(lst):
            n = lst[i]
            if n.no_more:
                i += 1
                continue
            for ch in divide(n, pts):
                if ch.keys:
                    lst.insert(0, alloc(ch))
                    i += 1
                    if len(ch.keys) > 1:
                        nexp += 1
                        vsize.append((len(ch.keys), ch))
            lst.pop(i)
        if len(lst) >= N or len(lst) == prev:
            finish = True
        elif len(lst) + nexp * 3 > N:
            while not finish:
                prev = len(lst)
                vprev = sorted(vsize, key=lambda t: (t[0], t[1].seq))
                vsize = []
                for j in range(len(vprev) - 1, -1, -1):
                    parent = vprev[j][1]
                    for ch in divide(parent, pts):
                        if ch.keys:
                            lst.insert(0, alloc(ch))
                            if len(ch.keys) > 1:
                                vsize.append((len(ch.keys), ch))
                    lst.remove(parent)
                    if len(lst) >= N:
                        break
                if len(lst) >= N or len(lst) == prev:
                    finish = True
    out = []
    for n in lst:
        best = n.keys[0]
        for k in n.keys[1:]:
            if pts[k][2] > pts[best][2]:
                best = k
        out.append(best)
    return out
