"""Search for a shorter elimination schedule of the tree solver (development tool).

The per-sample system is SPD on the graph of the 97 currents (afs_tables.cpp topology()).
One solver round eliminates, on each of up to K lanes, one unknown c with at most two
remaining neighbours n0, n1; the lanes of a round must touch disjoint unknowns {c, n0, n1}
and edges; eliminating c with two neighbours that are not adjacent creates the fill edge
(n0, n1), stored in a free slot of the first-eliminated of n0, n1 (NSLOT slots per unknown).

python tools/sched_search.py [--lanes 16] [--slots 1] [--trials 2000]

Randomised greedy list scheduling: each round takes eligible unknowns in priority order
(distance from a root, with random tie-breaking) until the lanes are used up; lanes are then
assigned to keep each lane on its own chain (an unknown's step goes to the lane that
eliminated its neighbour last round) so that the kernel's carried-pivot rounds apply.  Prints
the best round count found and the per-round eliminations.
"""
import argparse
import random
from collections import deque

NS, NC = 93, 97
SINUS_COUPLING = (8, 9, 11, 12)


def topology():
    src = [i - 1 for i in range(NC)]
    src[0] = -1
    src[65] = 40
    src[84] = 28
    for i, k in enumerate(SINUS_COUPLING):
        src[89 + i] = 65 + k
    src[93] = src[94] = 64
    src[95] = src[96] = 83
    outs = [[] for _ in range(NS)]
    for c in range(1, NC):
        if src[c] >= 0:
            outs[src[c]].append(c)
    adj = [set() for _ in range(NC)]
    for s in range(NS):
        m = [s] + outs[s]
        for a in m:
            for b in m:
                if a != b:
                    adj[a].add(b)
    return adj


def simulate(adj0, lanes, nslot, prio, rng):
    adj = [set(a) for a in adj0]
    gone = [False] * NC
    host = [0] * NC          # fill edges hosted per unknown (slot use)
    fill_edges = []          # (x, y, round)
    order = [None] * NC
    rounds = []
    while not all(gone):
        r = len(rounds)
        cand = [c for c in range(NC) if not gone[c] and len(adj[c]) <= 2]
        rng.shuffle(cand)
        cand.sort(key=lambda c: -prio[c])
        touched, edges_t, step = set(), set(), []
        for c in cand:
            if len(step) == lanes:
                break
            nb = sorted(adj[c])
            t = {c, *nb}
            if t & touched:
                continue
            es = {frozenset((c, n)) for n in nb}
            if len(nb) == 2:
                es.add(frozenset(nb))
            if es & edges_t:
                continue
            step.append((c, nb))
            touched |= t
            edges_t |= es
        if not step:
            return None
        for c, nb in step:
            if len(nb) == 2 and nb[1] not in adj[nb[0]]:
                adj[nb[0]].add(nb[1])
                adj[nb[1]].add(nb[0])
                fill_edges.append((nb[0], nb[1]))
            for n in nb:
                adj[n].discard(c)
            adj[c] = set()
            gone[c] = True
            order[c] = r
        rounds.append(step)
    # fill-edge slots: stored at the first-eliminated end
    for x, y in fill_edges:
        h = x if order[x] < order[y] else y
        host[h] += 1
        if host[h] > nslot:
            return None
    return rounds, order


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=16)
    ap.add_argument("--slots", type=int, default=1)
    ap.add_argument("--trials", type=int, default=2000)
    ap.add_argument("--root", type=int, default=40)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    adj0 = topology()
    # priority: graph distance from the root (far first)
    dist = [None] * NC
    dist[a.root] = 0
    q = deque([a.root])
    while q:
        u = q.popleft()
        for v in adj0[u]:
            if dist[v] is None:
                dist[v] = dist[u] + 1
                q.append(v)
    rng = random.Random(a.seed)
    best = None
    for t in range(a.trials):
        w = rng.random() * 0.5
        prio = [dist[c] + w * rng.random() * 10 for c in range(NC)]
        res = simulate(adj0, a.lanes, a.slots, prio, rng)
        if res and (best is None or len(res[0]) < len(best[0])):
            best = res
    if best is None:
        print("no valid schedule")
        return
    rounds, order = best
    print(f"best: {len(rounds)} rounds with {a.lanes} lanes, {a.slots} fill slot(s) per unknown")
    for r, st in enumerate(rounds):
        print(f"  round {r:2d}: " + " ".join(f"{c}" for c, _ in st))


if __name__ == "__main__":
    main()


def check_programs(lanes, nslot=1, verbose=True):
    """The C++ builder's check (afs_tables.cpp tree_schedule, the LDS-rounds solver that the arm
    solver replaced; this tool is kept for its topology() and as the record of that search) for lane programs
    [[(start_round, [nodes...]), ...], ...]: returns (rounds, fwd_carry_count, bwd_carry_count)
    or raises ValueError."""
    adj = [set(a) for a in topology()]
    K = len(lanes)
    prog = {}
    order = [None] * NC
    for k, progs in enumerate(lanes):
        for start, nodes in progs:
            for i, c in enumerate(nodes):
                r = start + i
                if (r, k) in prog or order[c] is not None:
                    raise ValueError(f"lane {k} round {r} node {c}: slot or node used twice")
                prog[(r, k)] = c
                order[c] = r
    if any(o is None for o in order):
        raise ValueError("unscheduled: " + str([c for c in range(NC) if order[c] is None]))
    R = max(r for r, _ in prog) + 1
    gone = [False] * NC
    host = [0] * NC
    steps = {}
    for r in range(R):
        wr, rd = {}, {}
        for k in range(K):
            c = prog.get((r, k))
            if c is None:
                continue
            nb = sorted(x for x in adj[c] if not gone[x])
            if len(nb) > 2:
                raise ValueError(f"round {r} lane {k}: {c} has neighbours {nb}")
            nxt = prog.get((r + 1, k))
            if len(nb) == 2 and nb[1] == nxt:
                nb = [nb[1], nb[0]]
            steps[(r, k)] = (c, nb)
            t = {c, *nb}
            es = {frozenset((c, n)) for n in nb}
            wes = {frozenset(nb)} if len(nb) == 2 else set()
            wr[k] = t | wes
            rd[k] = t | es | wes
        for a in wr:
            for b in rd:
                if a != b and wr[a] & rd[b]:
                    raise ValueError(f"round {r}: lanes {a} and {b} conflict on {wr[a] & rd[b]}")
        for k in range(K):
            if (r, k) not in steps:
                continue
            c, nb = steps[(r, k)]
            if len(nb) == 2 and nb[1] not in adj[nb[0]]:
                x = nb[0] if order[nb[0]] < order[nb[1]] else nb[1]
                host[x] += 1
                if host[x] > nslot:
                    raise ValueError(f"round {r}: fill slot of {x} used twice")
                adj[nb[0]].add(nb[1])
                adj[nb[1]].add(nb[0])
        for k in range(K):
            if (r, k) in steps:
                gone[steps[(r, k)][0]] = True
    # carries (as tree_schedule)
    fwd = 0
    carry = [None] * K
    for r in range(R):
        if all(steps[(r, k)][0] == carry[k] for k in range(K) if (r, k) in steps):
            fwd += 1
        for k in range(K):
            st = steps.get((r, k))
            carry[k] = st[1][0] if st and st[1] else None
            if st:
                for q in [st[0], *st[1]]:
                    for j in range(K):
                        if j != k and carry[j] == q:
                            carry[j] = None
    bwd = 0
    carry = [None] * K
    for r in range(R - 1, -1, -1):
        if all(steps[(r, k)][1] and steps[(r, k)][1][0] == carry[k] for k in range(K) if (r, k) in steps):
            bwd += 1
        for k in range(K):
            carry[k] = steps[(r, k)][0] if (r, k) in steps else None
    if verbose:
        print(f"{R} rounds, {fwd} carried forward, {bwd} carried backward")
    return R, fwd, bwd


def span(a, b):
    return list(range(a, b + 1)) if a <= b else list(range(a, b - 1, -1))


CURRENT = [
    [(0, span(0, 9))], [(0, span(11, 19))], [(0, span(21, 27))], [(0, span(88, 84))],
    [(0, span(39, 30))], [(0, span(42, 52))], [(0, [94, 93] + span(64, 54)), (13, [53, 41, 40])],
    [(0, [96, 95] + span(83, 77))], [(0, span(66, 76) + [65])], [(0, [89, 90])], [(0, [91, 92])],
    [(10, [10, 20, 28, 29])],
]


def assign_lanes(rounds, K):
    """Lane programs for a round list [[(c, nb), ...], ...]: a step goes to the lane whose
    previous step had c as a neighbour when possible (so the pivot can stay in registers).
    Returns prog[r][k] (node or -1)."""
    prog = []
    prev = [None] * K  # neighbours of each lane's previous step
    for st in rounds:
        row = [-1] * K
        free = set(range(K))
        rest = []
        for c, nb in st:
            k = next((k for k in sorted(free) if prev[k] and c in prev[k]), None)
            if k is None:
                rest.append((c, nb))
            else:
                row[k] = c
                free.discard(k)
                prev[k] = nb
        for c, nb in rest:
            k = min(free)
            row[k] = c
            free.discard(k)
            prev[k] = nb
        for k in free:
            prev[k] = None
        prog.append(row)
    return prog


def search_best(K=16, trials=4000, seed=1, root=40):
    adj0 = topology()
    dist = [None] * NC
    dist[root] = 0
    q = deque([root])
    while q:
        u = q.popleft()
        for v in adj0[u]:
            if dist[v] is None:
                dist[v] = dist[u] + 1
                q.append(v)
    rng = random.Random(seed)
    best = None
    for t in range(trials):
        w = rng.random() * 0.5
        prio = [dist[c] + w * rng.random() * 10 for c in range(NC)]
        res = simulate(adj0, K, 1000, prio, rng)
        if not res:
            continue
        rounds, _ = res
        prog = assign_lanes(rounds, K)
        lanes = [[(r, [prog[r][k]]) for r in range(len(prog)) if prog[r][k] >= 0] for k in range(K)]
        try:
            R, fwd, bwd = check_programs(lanes, nslot=1000, verbose=False)
        except ValueError:
            continue
        key = (R, -(fwd + bwd))
        if best is None or key < best[0]:
            best = (key, prog, fwd, bwd)
    return best
