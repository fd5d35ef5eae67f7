"""Steps settled per speculative round, simulated on accept decisions that are
iid (rate p) or bursty (a two-state Markov chain switching between a low and
a high rate, as a chain that leaves a local minimum accepts in runs).

  python tools/probes/spec_tree_sim.py [rounds]

Compares, for slot counts S: round 3's two paths (the reject chain or the
accept chain, accept while 2a >= n, memory 3/4 per round), speculation trees
on a uniform p = b/16 grid, and the kernels' trees (ipmc_spec_tree.hpp:
sixteenths plus 1/32, 1/64, 1/128 from either end) with the estimate's memory
3/4 (the kernels') or 0.95.  The trees are rebuilt here best-first exactly as
the header builds them (tests/test_spec_tree_cpu.py checks the header's).
One JSON line per (S, process).
"""
import heapq
import json
import sys

import numpy as np

GRID_UNIFORM = [b / 16 for b in range(17)]
GRID_KERNEL = [0, 1 / 128, 1 / 64, 1 / 32] + [b / 16 for b in range(1, 16)] + [1 - 1 / 32, 1 - 1 / 64, 1 - 1 / 128, 1]


def tree(p, nodes=256):
    """children[i] = (after a reject, after an accept) of node i, -1: none."""
    heap, seq, kids = [(-1.0, 0, -1, 0)], 1, []
    for i in range(nodes):
        pr, _, par, edge = heapq.heappop(heap)
        kids.append([-1, -1])
        if par >= 0:
            kids[par][edge] = i
        heapq.heappush(heap, (pr * (1 - p), seq, i, 0))
        heapq.heappush(heap, (pr * p, seq + 1, i, 1))
        seq += 2
    return kids


_TREES = {}


def simulate(p, S, grid, memory, two_paths=False, rounds=20000, seed=0):
    """p: an acceptance rate, or (low, high, switch probability per step)."""
    trees = _TREES.setdefault(tuple(grid), [tree(g) for g in grid])
    mids = [(grid[i] + grid[i + 1]) / 2 for i in range(len(grid) - 1)]
    rng = np.random.default_rng(seed)
    a, n, total = 1.0, 1.0, 0
    plo, phi, sw = p if isinstance(p, tuple) else (p, p, 0.0)
    state = 0
    for _ in range(rounds):
        if two_paths:
            b = len(grid) - 1 if 2 * a >= n else 0
        else:
            b = sum(a / n > m for m in mids)
        kids, node, used, nar = trees[b], 0, 0, 0
        while True:
            if sw and rng.random() < sw:
                state ^= 1
            acc = rng.random() < (phi if state else plo)
            used += 1
            nar += acc
            c = kids[node][1 if acc else 0]
            if c < 0 or c >= S:
                break
            node = c
        a, n = memory * a + nar, memory * n + used
        total += used
    return total / rounds


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    procs = [0.01, 0.05, 0.12, 0.25, 0.5, 0.75, 0.88, 0.97, 0.99,
             (0.0, 0.5, 0.02), (0.02, 0.6, 0.05), (0.05, 0.9, 0.02), (0.1, 0.3, 0.01)]
    for S in (4, 16, 64, 256):
        for p in procs:
            print(json.dumps({
                "S": S, "p": p,
                "two_paths": simulate(p, S, GRID_UNIFORM, 0.75, two_paths=True, rounds=rounds),
                "tree_uniform_grid_m075": simulate(p, S, GRID_UNIFORM, 0.75, rounds=rounds),
                "tree_kernel_grid_m075": simulate(p, S, GRID_KERNEL, 0.75, rounds=rounds),
                "tree_kernel_grid_m095": simulate(p, S, GRID_KERNEL, 0.95, rounds=rounds),
            }), flush=True)


if __name__ == "__main__":
    main()
