"""The arm solver's elimination order (tree_core.h solve_arms, partition in afs_tables.cpp
arm_records) on random SPD matrices with the current graph's sparsity, in numpy
(tools/arm_solver_study.py): every elimination has at most two remaining neighbours outside
the junction / fossa folds, and the solution matches a dense solve to rounding level."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import arm_solver_study as st  # noqa: E402
from sched_search import topology  # noqa: E402


def test_arm_order_is_exact_on_random_spd():
    adj = topology()
    rng = np.random.default_rng(11)
    for _ in range(10):
        A, b = st.random_system(adj, rng)
        x, steps, order = st.solve_arms(A, b)
        ref = np.linalg.solve(A, b)
        assert np.abs(x - ref).max() <= 1e-12 * np.abs(ref).max()
    assert sorted(order) == list(range(97))
    assert steps["walk_max"] == 7 and max(steps["arm_reduce"].values()) == 6
