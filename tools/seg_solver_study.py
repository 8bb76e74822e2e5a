"""Design study (not product code): the segment-aligned ("seg") solver of the per-sample
97-unknown system, lane by lane, checked against a dense solve.

The seg kernel gives every lane of an utterance's 16 the same currents in
every phase -- network, rows, elimination, update -- so the matrix never goes through LDS:

* Static condensation.  Rows of currents whose two sections are static (trachea 0..22, nose
  70..83 with the sinus leaves 89..92 and the nostril pair 95/96, fossa 85..88) have constant
  coefficients: the three static subtrees T, N, Fo hang from the dynamic currents 23, 69 and
  84 by one constant edge each.  Their LDL^T is computed once on the host; per sample only
  z = K^-1 y_T is needed (a forward and a backward linear recurrence with constant
  coefficients: a lane-local sweep plus a 4-step lane scan each way), the attach node d gets
  a constant pivot term -e^2 (K^-1)_rr and the right-hand side -e z_r, and after the dynamic
  solve x_T = z - g x_d with the constant vector g = e K^-1 delta_r.
* The 50 dynamic currents: 11 arm lanes of exactly four positions in walk order (arm A
  23..38 with the fossa entry 84 folded on 28/29, arm B 93, 64..42 with 94 folded on 93/64,
  arm C 69..66) and a junction lane with {39, 40, 41, 65}; every lane walks its four
  positions in registers, the boundaries are reduced lane to lane (arm B: 5 steps), the
  junction lane solves its four nodes, the solutions flow back.

python tools/seg_solver_study.py [--trials 20]
"""
from __future__ import annotations

import argparse
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from sched_search import NC, topology  # noqa: E402

# ---- dynamic lanes: four positions in walk order (far end first) -------------------------
DYN = [
    [23, 24, 25, 26], [27, 28, 29, 30], [31, 32, 33, 34], [35, 36, 37, 38],          # arm A
    [93, 64, 63, 62], [61, 60, 59, 58], [57, 56, 55, 54], [53, 52, 51, 50],
    [49, 48, 47, 46], [45, 44, 43, 42],                                              # arm B
    [69, 68, 67, 66],                                                                # arm C
    [39, 40, 41, 65],                                                                # junction
]
ARM = [0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 2, -1]
JUNCTION_LANE = 11
ARM_END = {0: (3, 39), 1: (9, 41), 2: (10, 65)}  # arm -> (last lane, junction node its boundary joins)
FOLD = {1: (84, 1), 4: (94, 0)}                  # lane -> (leaf, attach position q: joins q, q+1)
# ---- static lanes: three chain positions (far end first) + leaf slots on (0,1) and (1,2) ---
STAT = [
    [0, 1, 2], [3, 4, 5], [6, 7, 8], [9, 10, 11], [12, 13, 14], [15, 16, 17], [18, 19, 20], [21, 22],
    [95, 83, 82], [81, 80, 79], [78, 77, 76], [75, 74, 73], [72, 71, 70],
    [88, 87, 86], [85],
]
SLEAF = {8: (96, None), 10: (92, 91), 11: (90, 89)}  # lane -> (leaf on (0,1), leaf on (1,2))
SUBTREE = [0] * 8 + [1] * 5 + [2] * 2               # static lane -> subtree (T, N, Fo)
ROOT = {0: (22, 23), 1: (70, 69), 2: (85, 84)}      # subtree -> (root, dynamic attach node)


def random_system(adj, rng):
    A = np.zeros((NC, NC))
    for i in range(NC):
        for j in adj[i]:
            if j > i:
                A[i, j] = A[j, i] = -rng.uniform(0.1, 1.0)
    for i in range(NC):
        A[i, i] = -A[i].sum() + rng.uniform(0.5, 2.0)
    return A, rng.standard_normal(NC)


class StaticPlan:
    """Host side: the LDL^T of the static block in the lanes' order and the scan constants."""

    def __init__(self, A):
        order = []
        for k, seg in enumerate(STAT):
            lv = SLEAF.get(k, (None, None))
            order += [c for c in lv if c is not None] + seg
        self.order = order
        n = len(order)
        pos = {c: i for i, c in enumerate(order)}
        K = A[np.ix_(order, order)].copy()
        # LDL^T in this order (no fill outside the chains' pattern: checked)
        L = np.eye(n)
        D = np.zeros(n)
        W = K.copy()
        for i in range(n):
            D[i] = W[i, i]
            for j in range(i + 1, n):
                if W[j, i] != 0.0:
                    L[j, i] = W[j, i] / D[i]
            for j in range(i + 1, n):
                if L[j, i] == 0.0:
                    continue
                for m in range(i + 1, n):
                    if W[i, m] != 0.0:
                        if W[j, m] == 0.0 and j != m:
                            raise SystemExit(f"fill at {order[j]},{order[m]}")
                        W[j, m] -= L[j, i] * W[i, m]
        self.L, self.D, self.pos = L, D, pos
        Kinv = np.linalg.inv(K)
        self.delta, self.g = {}, {}
        for t, (r, d) in ROOT.items():
            e = A[r, d]
            self.delta[d] = -e * e * Kinv[pos[r], pos[r]]
            self.g[t] = e * Kinv[:, pos[r]]
        self.Kinv = Kinv

    def l(self, a, b):  # multiplier of predecessor b into a
        return self.L[self.pos[a], self.pos[b]]


def static_z(sp: StaticPlan, y):
    """z = K^-1 y_T the way the lanes compute it: per lane a local sweep with carry in 0, a
    4-step Hillis-Steele scan of the lane maps (constant products, segmented by subtree), a
    local sweep with the true carry; the same backwards."""
    nl = 16
    # ---- forward: carry = y' of the lane's last chain node
    def fwd(k, cin):
        seg = STAT[k] if k < len(STAT) else []
        lv = SLEAF.get(k, (None, None))
        yp = {}
        for c in lv:
            if c is not None:
                yp[c] = y[c]
        prev = None
        for p, c in enumerate(seg):
            v = y[c]
            for q, leaf in ((0, lv[0]), (1, lv[1])):  # leaf q joins positions q, q+1
                if leaf is not None and p in (q, q + 1):
                    v -= sp.l(c, leaf) * yp[leaf]
            if p == 0:
                if 0 < k < len(STAT) and SUBTREE[k - 1] == SUBTREE[k]:
                    v -= sp.l(c, STAT[k - 1][-1]) * cin
            else:
                v -= sp.l(c, prev) * yp[prev]
            yp[c] = v
            prev = c
        return yp

    def lane_map(k):  # carry_out = A + P carry_in
        if k >= len(STAT):
            return 0.0, 0.0
        a = fwd(k, 0.0)[STAT[k][-1]]
        P = 1.0
        seg = STAT[k]
        first = k > 0 and SUBTREE[k - 1] == SUBTREE[k]
        if not first:
            P = 0.0
        else:
            P = -sp.l(seg[0], STAT[k - 1][-1])
            for p in range(1, len(seg)):
                P *= -sp.l(seg[p], seg[p - 1])
        return a, P

    maps = [lane_map(k) for k in range(nl)]
    v = np.array([m[0] for m in maps])
    Q = np.array([m[1] for m in maps])
    for s in (1, 2, 4, 8):  # inclusive scan: v_k = A_k + P_k A_{k-1} + ...
        sh = np.concatenate([np.zeros(s), v[:-s]])
        qs = np.concatenate([np.zeros(s), Q[:-s]])
        v = v + Q * sh
        Q = Q * qs
    carry_in = np.concatenate([[0.0], v[:-1]])
    yp = {}
    for k in range(len(STAT)):
        yp.update(fwd(k, carry_in[k]))
    # ---- backward: z = D^-1 y' - L^T z, carry = z of the lane's first chain node
    def bwd(k, cnext):
        seg = STAT[k]
        lv = SLEAF.get(k, (None, None))
        z = {}
        last = k + 1 < len(STAT) and SUBTREE[k + 1] == SUBTREE[k]
        for p in range(len(seg) - 1, -1, -1):
            c = seg[p]
            v = yp[c] / sp.D[sp.pos[c]]
            if p == len(seg) - 1:
                if last:
                    v -= sp.l(STAT[k + 1][0], c) * cnext
            else:
                v -= sp.l(seg[p + 1], c) * z[seg[p + 1]]
            z[c] = v
        for q, leaf in ((0, lv[0]), (1, lv[1])):
            if leaf is None:
                continue
            v = yp[leaf] / sp.D[sp.pos[leaf]]
            for p in (q, q + 1):
                v -= sp.l(seg[p], leaf) * z[seg[p]]
            z[leaf] = v
        return z

    def back_map(k):  # z_first = B + Q z_next_first
        if k >= len(STAT):
            return 0.0, 0.0
        b = bwd(k, 0.0)[STAT[k][0]]
        seg = STAT[k]
        last = k + 1 < len(STAT) and SUBTREE[k + 1] == SUBTREE[k]
        if not last:
            return b, 0.0
        P = -sp.l(STAT[k + 1][0], seg[-1])
        for p in range(len(seg) - 2, -1, -1):
            P *= -sp.l(seg[p + 1], seg[p])
        return b, P

    maps = [back_map(k) for k in range(nl)]
    v = np.array([m[0] for m in maps])
    Q = np.array([m[1] for m in maps])
    for s in (1, 2, 4, 8):  # scan toward lower lanes
        sh = np.concatenate([v[s:], np.zeros(s)])
        qs = np.concatenate([Q[s:], np.zeros(s)])
        v = v + Q * sh
        Q = Q * qs
    cnext = np.concatenate([v[1:], [0.0]])
    z = {}
    for k in range(len(STAT)):
        z.update(bwd(k, cnext[k]))
    return z


def dyn_solve(A, y):
    """The dynamic currents' system (with the static terms already condensed into A, y),
    lane by lane: folds, walks, arm reductions, junction lane, back substitution."""
    nl = len(DYN)
    D = np.array([[A[c, c] for c in DYN[k]] for k in range(nl)])
    Y = np.array([[y[c] for c in DYN[k]] for k in range(nl)])
    E = np.array([[A[DYN[k][p], DYN[k][p + 1]] if k != JUNCTION_LANE else 0.0 for p in range(3)] for k in range(nl)])
    ea = np.zeros(nl)
    for k in range(nl):
        if k != JUNCTION_LANE and k > 0 and ARM[k - 1] == ARM[k]:
            ea[k] = A[DYN[k - 1][3], DYN[k][0]]
    # folds
    fold = {}
    for k, (leaf, q) in FOLD.items():
        a0, a1 = DYN[k][q], DYN[k][q + 1]
        dl, yl = A[leaf, leaf], y[leaf]
        l0, l1 = A[leaf, a0], A[leaf, a1]
        il = 1.0 / dl
        D[k, q] -= l0 * l0 * il
        D[k, q + 1] -= l1 * l1 * il
        Y[k, q] -= l0 * il * yl
        Y[k, q + 1] -= l1 * il * yl
        E[k, q] -= l0 * l1 * il
        fold[k] = (leaf, q, il, yl, l0, l1)
    # walks (positions 0..2 eliminated, 3 is the boundary; the anchor is lane k-1's boundary)
    inv = np.zeros((nl, 3))
    Fw = np.zeros((nl, 3))
    dA = np.zeros(nl)
    yA = np.zeros(nl)
    Ffin = np.zeros(nl)
    for k in range(nl):
        if k == JUNCTION_LANE:
            continue
        F = ea[k]
        for p in range(3):
            iv = 1.0 / D[k, p]
            g, h = F * iv, E[k, p] * iv
            dA[k] -= g * F
            yA[k] -= g * Y[k, p]
            D[k, p + 1] -= E[k, p] ** 2 * iv
            Y[k, p + 1] -= h * Y[k, p]
            inv[k, p] = iv
            Fw[k, p] = F
            F = -g * E[k, p]
        Ffin[k] = F
    Db, Yb = D[:, 3].copy(), Y[:, 3].copy()
    for k in range(1, nl):  # the anchors' updates go back one lane
        if k != JUNCTION_LANE and ARM[k - 1] == ARM[k]:
            Db[k - 1] += dA[k]
            Yb[k - 1] += yA[k]
    # arm reductions toward the junction
    binv = np.zeros(nl)
    for k in range(nl):
        if k == JUNCTION_LANE:
            continue
        if k > 0 and ARM[k - 1] == ARM[k]:
            iv = binv[k - 1]
            Db[k] -= Ffin[k] ** 2 * iv
            Yb[k] -= Ffin[k] * iv * Yb[k - 1]
        binv[k] = 1.0 / Db[k]
    # junction lane: nodes 39, 40, 41, 65 (its four positions), arms' last boundaries folded in
    J = DYN[JUNCTION_LANE]
    jd = {c: D[JUNCTION_LANE, i] for i, c in enumerate(J)}
    jy = {c: Y[JUNCTION_LANE, i] for i, c in enumerate(J)}
    ej = {}
    for arm, (lane, node) in ARM_END.items():
        b = DYN[lane][3]
        e = A[b, node]
        ej[arm] = e
        jd[node] -= e * e * binv[lane]
        jy[node] -= e * binv[lane] * Yb[lane]
    e39_40, e40_41, e40_65, e41_65 = A[39, 40], A[40, 41], A[40, 65], A[41, 65]
    i39 = 1.0 / jd[39]
    jd[40] -= e39_40 ** 2 * i39
    jy[40] -= e39_40 * i39 * jy[39]
    i65 = 1.0 / jd[65]
    jd[40] -= e40_65 ** 2 * i65
    jy[40] -= e40_65 * i65 * jy[65]
    jd[41] -= e41_65 ** 2 * i65
    jy[41] -= e41_65 * i65 * jy[65]
    e4041 = e40_41 - e40_65 * e41_65 * i65
    i41 = 1.0 / jd[41]
    jd[40] -= e4041 ** 2 * i41
    jy[40] -= e4041 * i41 * jy[41]
    x = {}
    x[40] = jy[40] / jd[40]
    x[41] = (jy[41] - e4041 * x[40]) * i41
    x[65] = (jy[65] - e40_65 * x[40] - e41_65 * x[41]) * i65
    x[39] = (jy[39] - e39_40 * x[40]) * i39
    # back along the arms
    xb = np.zeros(nl)
    for arm, (lane, node) in ARM_END.items():
        xb[lane] = (Yb[lane] - ej[arm] * x[node]) * binv[lane]
    for k in range(nl - 1, -1, -1):
        if k == JUNCTION_LANE or ARM_END[ARM[k]][0] == k:
            continue
        xb[k] = (Yb[k] - Ffin[k + 1] * xb[k + 1]) * binv[k]
    for k in range(nl):
        if k == JUNCTION_LANE:
            continue
        xA = xb[k - 1] if (k > 0 and ARM[k - 1] == ARM[k]) else 0.0
        xs = [0.0] * 4
        xs[3] = xb[k]
        for p in range(2, -1, -1):
            xs[p] = (Y[k, p] - E[k, p] * xs[p + 1] - Fw[k, p] * xA) * inv[k, p]
        for p, c in enumerate(DYN[k]):
            x[c] = xs[p]
        if k in fold:
            leaf, q, il, yl, l0, l1 = fold[k]
            x[leaf] = (yl - l0 * xs[q] - l1 * xs[q + 1]) * il
    return x


def seg_solve(A, y):
    sp = StaticPlan(A)
    z = static_z(sp, y)
    A2, y2 = A.copy(), y.copy()
    for t, (r, d) in ROOT.items():
        A2[d, d] += sp.delta[d]
        y2[d] -= A[r, d] * z[r]
    xd = dyn_solve(A2, y2)
    x = np.zeros(NC)
    for c, v in xd.items():
        x[c] = v
    for k, seg in enumerate(STAT):
        t = SUBTREE[k]
        d = ROOT[t][1]
        lv = [c for c in SLEAF.get(k, (None, None)) if c is not None]
        for c in seg + lv:
            x[c] = z[c] - sp.g[t][sp.pos[c]] * xd[d]
    return x


def check_partition():
    dyn = sorted(c for lane in DYN for c in lane) + sorted(l for l, _ in FOLD.values())
    stat = sorted(c for lane in STAT for c in lane) + sorted(c for lv in SLEAF.values() for c in lv if c is not None)
    allc = sorted(dyn + stat)
    assert allc == list(range(NC)), "every current exactly once"
    assert len(dyn) == 50 and len(stat) == 47


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=20)
    a = ap.parse_args()
    check_partition()
    adj = topology()
    rng = np.random.default_rng(7)
    worst = 0.0
    for _ in range(a.trials):
        A, b = random_system(adj, rng)
        x = seg_solve(A, b)
        ref = np.linalg.solve(A, b)
        worst = max(worst, float(np.abs(x - ref).max() / np.abs(ref).max()))
    print(f"max relative error vs dense solve over {a.trials} systems: {worst:.2e}")
    return worst


if __name__ == "__main__":
    main()
