"""Quadric-error edge-collapse decimation (Garland & Heckbert, SIGGRAPH 1997) for the offline render
model compiler (tools/compile_render.py).  Build-time only: its outputs are committed data.

Many meshes are decimated under ONE budget: all their edges share one priority queue, so the
triangles go where the geometric error is (a flat decal keeps 2, a curved casting hundreds).
Per mesh:
  * vertices welded by position (the OBJ files split them at UV seams);
  * every face adds its plane's quadric, weighted by its area, to its three vertices; every boundary
    edge adds a plane through it perpendicular to its face (weight BOUNDARY_W x area) so open
    edges keep their outline;
  * the cost of collapsing edge (a, b) is the summed quadric's error at the position that minimises
    it (the 3 x 3 solve; the best of a, b and the midpoint when that solve is ill-conditioned or
    lands farther than one edge length from the midpoint), times the mesh's weight;
  * a collapse is skipped when it breaks the link condition (the two vertices share more
    neighbours than the edge's opposite vertices: it would pinch the surface) or turns a surviving
    face by more than ~80 degrees (a fold-over).
The surviving faces keep the input winding."""
from __future__ import annotations

import heapq
import math

import numpy as np

BOUNDARY_W = 10.0
FLIP_COS = 0.2


def weld(v, t, tol=1e-7):
    q = np.round(v / tol).astype(np.int64)
    _, first, inv = np.unique(q, axis=0, return_index=True, return_inverse=True)
    inv = inv.ravel()
    tt = inv[t]
    tt = tt[(tt[:, 0] != tt[:, 1]) & (tt[:, 1] != tt[:, 2]) & (tt[:, 0] != tt[:, 2])]
    # one copy of each face (a face and its reverse are both kept: two-sided sheets)
    _, keep = np.unique(tt, axis=0, return_index=True)
    return v[first], tt[np.sort(keep)]


def _plane_q(n, d, w):
    p = np.array([n[0], n[1], n[2], d])
    return w * np.outer(p, p)


class _Mesh:
    def __init__(self, v, t, weight):
        self.v = [np.asarray(x, float) for x in v]
        self.t = [list(map(int, f)) for f in t]
        self.alive_t = [True] * len(self.t)
        self.alive_v = [True] * len(self.v)
        self.vt = [set() for _ in self.v]  # faces per vertex
        for fi, f in enumerate(self.t):
            for a in f:
                self.vt[a].add(fi)
        self.Q = [np.zeros((4, 4)) for _ in self.v]
        self.weight = weight
        self.stamp = [0] * len(self.v)
        edge_faces = {}
        for fi, (a, b, c) in enumerate(self.t):
            pa, pb, pc = self.v[a], self.v[b], self.v[c]
            n = np.cross(pb - pa, pc - pa)
            ln = np.linalg.norm(n)
            if ln <= 0:
                continue
            area = 0.5 * ln
            n = n / ln
            K = _plane_q(n, -float(n @ pa), area)
            for x in (a, b, c):
                self.Q[x] += K
            for x, y in ((a, b), (b, c), (c, a)):
                edge_faces.setdefault((min(x, y), max(x, y)), []).append((fi, n))
        for (x, y), fl in edge_faces.items():
            if len(fl) == 1:  # boundary edge: a plane through it, perpendicular to its face
                n = fl[0][1]
                e = self.v[y] - self.v[x]
                le = float(np.linalg.norm(e))
                if le <= 0:
                    continue
                m = np.cross(e / le, n)
                K = _plane_q(m, -float(m @ self.v[x]), BOUNDARY_W * le * le)
                self.Q[x] += K
                self.Q[y] += K

    def neighbours(self, a):
        s = set()
        for fi in self.vt[a]:
            s.update(self.t[fi])
        s.discard(a)
        return s

    def n_faces(self):
        return sum(self.alive_t)

    def cost(self, a, b):
        Q = self.Q[a] + self.Q[b]
        pa, pb = self.v[a], self.v[b]
        mid = 0.5 * (pa + pb)
        cands = [pa, pb, mid]
        A = Q[:3, :3]
        if abs(np.linalg.det(A)) > 1e-18:
            x = np.linalg.solve(A, -Q[:3, 3])
            if np.linalg.norm(x - mid) <= np.linalg.norm(pb - pa):
                cands.insert(0, x)
        best, bp = math.inf, None
        for p in cands:
            h = np.append(p, 1.0)
            e = float(h @ Q @ h)
            if e < best:
                best, bp = e, p
        return max(best, 0.0) * self.weight, bp

    def can_collapse(self, a, b, p):
        shared = self.neighbours(a) & self.neighbours(b)
        opp = set()
        for fi in self.vt[a] & self.vt[b]:
            opp.update(x for x in self.t[fi] if x != a and x != b)
        if shared != opp:
            return False
        for x in (a, b):
            for fi in self.vt[x]:
                f = self.t[fi]
                if a in f and b in f:
                    continue
                P = [self.v[y] for y in f]
                n0 = np.cross(P[1] - P[0], P[2] - P[0])
                P = [p if y == x else self.v[y] for y in f]
                n1 = np.cross(P[1] - P[0], P[2] - P[0])
                l0, l1 = np.linalg.norm(n0), np.linalg.norm(n1)
                if l1 <= 1e-14 or (l0 > 0 and float(n0 @ n1) < FLIP_COS * l0 * l1):
                    return False
        return True

    def collapse(self, a, b, p):
        """b merges into a at p; returns the faces removed."""
        removed = 0
        for fi in list(self.vt[b]):
            f = self.t[fi]
            if a in f:
                self.alive_t[fi] = False
                removed += 1
                for x in f:
                    self.vt[x].discard(fi)
            else:
                self.t[fi] = [a if x == b else x for x in f]
                self.vt[a].add(fi)
        self.vt[b] = set()
        self.alive_v[b] = False
        self.v[a] = np.asarray(p, float)
        self.Q[a] = self.Q[a] + self.Q[b]
        self.stamp[a] += 1
        self.stamp[b] += 1
        return removed

    def result(self):
        used = sorted({x for fi, f in enumerate(self.t) if self.alive_t[fi] for x in f})
        remap = {x: i for i, x in enumerate(used)}
        V = np.array([self.v[x] for x in used])
        T = np.array([[remap[x] for x in f] for fi, f in enumerate(self.t) if self.alive_t[fi]], np.int64).reshape(-1, 3)
        return V, T


def decimate_many(meshes, target_faces, weights=None, min_faces=4):
    """meshes: [(V [n, 3], T [m, 3])]; decimates them together to about target_faces faces in total
    (each keeps at least min_faces).  Returns [(V, T)] in the input order."""
    weights = weights or [1.0] * len(meshes)
    M = [_Mesh(*weld(np.asarray(v, float), np.asarray(t, np.int64)), w) for (v, t), w in zip(meshes, weights)]
    nf = [m.n_faces() for m in M]
    total = sum(nf)
    heap = []

    def push(k, a, b):
        m = M[k]
        c, p = m.cost(a, b)
        heapq.heappush(heap, (c, k, a, b, m.stamp[a], m.stamp[b]))

    for k, m in enumerate(M):
        seen = set()
        for f in m.t:
            for x, y in ((f[0], f[1]), (f[1], f[2]), (f[2], f[0])):
                e = (min(x, y), max(x, y))
                if e not in seen:
                    seen.add(e)
                    push(k, *e)
    while total > target_faces and heap:
        c, k, a, b, sa, sb = heapq.heappop(heap)
        m = M[k]
        if not (m.alive_v[a] and m.alive_v[b]) or m.stamp[a] != sa or m.stamp[b] != sb:
            continue
        if nf[k] <= min_faces:
            continue
        _, p = m.cost(a, b)
        if not m.can_collapse(a, b, p):
            continue
        r = m.collapse(a, b, p)
        nf[k] -= r
        total -= r
        for x in m.neighbours(a):
            push(k, min(a, x), max(a, x))
    return [m.result() for m in M]
