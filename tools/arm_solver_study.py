"""Design study (not product code): an arm-wise segment solver for the per-sample 97-unknown
system, to replace the 12+12-round LDS elimination of the tree kernel.

The round-2 solver it replaced (afs_tables.cpp tree_schedule, removed) eliminated at most one
unknown per lane and round with every operand in LDS; a round costs the LDS round trip plus the pivot reciprocal
(~370 cycles forward, ~180 backward; 6.6 k of 29.9 k cycles per sample).  Here the graph is
cut into arms that meet at the junction triangle {40, 41, 65}:

  arm A  currents 0..39 (trachea, glottis, pharynx), far end 0, with the fossa (84..88) hanging
         from the triangle {28, 29, 84}
  arm B  currents 64..42 (mouth), far end 64 with the radiation pair {93, 94}
  arm C  currents 83..66 (nose), far end 83 with the radiation pair {95, 96}, the four sinus
         leaves 89..92 on the nose nodes 73..78

Every lane owns one contiguous segment of an arm (its last node is the lane's boundary) and, in
registers, (1) folds the leaves attached to its segment, (2) walks its segment from the far end
eliminating every node but the boundary (each step: one reciprocal, the fill edge to the
previous lane's boundary carried along); the boundaries then form one short chain per arm,
reduced lane to lane by DPP shifts toward the junction, the junction triangle is solved, and
the solution flows back the same way.  No LDS round trip inside the elimination.

This script (1) builds the partition, (2) runs the algorithm in numpy on random diagonally
dominant SPD matrices with the real sparsity pattern and checks it against a dense solve, and
(3) prints the step counts the cost model uses.

python tools/arm_solver_study.py [--trials 20]
"""
from __future__ import annotations

import argparse
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from sched_search import NC, topology  # noqa: E402

# lanes: arm A 7 (segments end at the boundaries), arm B 4, arm C 3, the junction lane, the fossa lane
ARM_A = [(0, 6), (7, 13), (14, 20), (21, 28), (29, 29), (30, 34), (35, 39)]  # walk ascending
ARM_B = [(64, 59), (58, 53), (52, 47), (46, 42)]                              # walk descending
ARM_C = [(83, 79), (78, 73), (72, 66)]
JUNCTION = (40, 41, 65)
FOSSA = (88, 87, 86, 85)  # walked toward 84, which stays with the triangle {28, 29, 84}
# leaves folded first, in this order: the radiation triangles {64, 93, 94} and {83, 95, 96} (93 then
# 94 into 64), the sinus leaves, each on two consecutive nose nodes (89: 73-74, 90: 74-75, 91: 76-77,
# 92: 77-78); the deepest fold chain is two steps (94 after 93, 90 after 89 on 74, 92 after 91 on 77)
LEAVES = (93, 94, 95, 96, 89, 90, 91, 92)


def segment_nodes(a, b):
    return list(range(a, b + 1)) if a <= b else list(range(a, b - 1, -1))


def random_system(adj, rng):
    A = np.zeros((NC, NC))
    for i in range(NC):
        for j in adj[i]:
            if j > i:
                v = -rng.uniform(0.1, 1.0)
                A[i, j] = A[j, i] = v
    for i in range(NC):
        A[i, i] = -A[i].sum() + rng.uniform(0.5, 2.0)  # diagonally dominant: SPD
    return A, rng.standard_normal(NC)


def solve_arms(A0, b0):
    """The arm solver's elimination order, executed on a dense copy (the numerics of the
    device version are the same steps on registers); returns x and the step counts."""
    A, b = A0.copy(), b0.copy()
    order = []
    steps = {"leaf_folds": 0, "walk_max": 0, "arm_reduce": {}, "junction": 3}
    # (1) leaves, (2) fossa walk, (3) segment walks (all lanes at once on the GPU)
    lane_steps = []
    order.extend(LEAVES)
    steps["leaf_folds"] = 2
    for c in FOSSA:
        order.append(c)
    lane_steps.append(len(FOSSA))
    for arm in (ARM_A, ARM_B, ARM_C):
        for (a, z) in arm:
            seg = segment_nodes(a, z)
            order.extend(seg[:-1])           # every node but the boundary
            lane_steps.append(len(seg) - 1)
    steps["walk_max"] = max(lane_steps)
    # (4) the triangle {28, 29, 84}: 84 first, (5) arm reductions lane to lane toward the
    # junction, (6) the junction triangle
    order.append(84)
    for name, arm in (("A", ARM_A), ("B", ARM_B), ("C", ARM_C)):
        bounds = [segment_nodes(a, z)[-1] for a, z in arm]
        order.extend(bounds)
        steps["arm_reduce"][name] = len(bounds) - 1
    order.extend(JUNCTION[::-1])
    assert sorted(order) == list(range(NC)), "every unknown exactly once"
    recs = []
    for c in order:
        nb = [j for j in np.nonzero(A[c])[0] if j != c]
        assert len(nb) <= 2 or c in JUNCTION or c == 84, (c, nb)  # at most two neighbours (fill-free chains)
        inv = 1.0 / A[c, c]
        row = A[c].copy()
        bc = b[c]
        for i in nb:
            f = A[i, c] * inv
            b[i] -= f * bc
            for j in nb:
                A[i, j] -= f * row[j]
        for i in nb:
            A[i, c] = A[c, i] = 0.0
        recs.append((c, nb, inv, row, bc))
    x = np.zeros(NC)
    for c, nb, inv, row, bc in reversed(recs):
        x[c] = (bc - sum(row[j] * x[j] for j in nb)) * inv
    return x, steps, order


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=20)
    a = ap.parse_args()
    adj = topology()
    rng = np.random.default_rng(7)
    worst = 0.0
    for _ in range(a.trials):
        A, b = random_system(adj, rng)
        x, steps, order = solve_arms(A, b)
        ref = np.linalg.solve(A, b)
        worst = max(worst, float(np.abs(x - ref).max() / np.abs(ref).max()))
    print(f"max relative error vs dense solve over {a.trials} systems: {worst:.2e}")
    print("steps:", steps)
    # cost model (cycles, one wave per SIMD; MI355X: fp64 dependent op ~7, v_rcp_f64 18,
    # pivot reciprocal with two Newton steps ~46, DPP exchange of a double ~16, LDS round trip ~150)
    step = 46 + 3 * 7          # one register elimination step
    red = step + 2 * 16        # one lane-to-lane reduction step (DPP in)
    back = 3 * 7 + 16          # one back-substitution step across lanes
    walk = steps["walk_max"]
    arm = max(steps["arm_reduce"].values())
    est = 150 + steps["leaf_folds"] * step + walk * step + 50 + arm * red + 3 * step + arm * back + walk * 20 + 100
    print(f"critical path estimate: ~{est} cycles per sample (current solver: 6.6 k measured: "
          f"4.4 k forward + 2.2 k backward)")
    # VALU issue: every lane executes every step slot (sink steps on lanes with less work)
    slots = 6 + walk + arm * 2 + 3
    print(f"step slots per sample: {slots} (~25 VALU instructions each, ~{slots * 25 * 4} cycles of issue)")


if __name__ == "__main__":
    main()
