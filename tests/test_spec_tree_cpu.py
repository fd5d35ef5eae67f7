"""The speculation trees of the speculative sweeps (csrc/ipmc_spec_tree.hpp),
built at compile time, checked on the CPU: the header is compiled with g++
into a tiny program that prints the tables, and every bucket's tree is
verified against its definition -- prefix-closed, best-first (every prefix of
S nodes holds the S most probable decision paths, so it is the best S-node
tree), origins and levels consistent with the paths, the reject / accept
chains at p = 0 / 1 -- and the walk the kernels do (spec_walk) is replayed on
random decision streams: every visited node proposes from the state the
sequential chain holds there, and a round settles exactly the steps up to the
first node outside the slots."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "ip_mcmc_amd", "csrc", "ipmc_spec_tree.hpp")

PROG = r"""
#include <cstdio>
#include "%s"
using namespace ipmc;
static const SpecTrees T = make_spec_trees();
int main() {
  std::printf("{\"nodes\": %%d, \"p\": [", kSpecNodes);
  for (int b = 0; b < kSpecBuckets; ++b) std::printf("%%s%%.17g", b ? "," : "", kSpecGridP[b]);
  std::printf("], \"bucket_of\": [");
  for (int i = 0; i <= 1000; ++i) std::printf("%%s%%d", i ? "," : "", spec_bucket_of(i / 1000.0));
  std::printf("], \"anc\": [");
  for (int b = 0; b < kSpecBuckets; ++b) {
    std::printf("%%s[", b ? "," : "");
    for (int i = 0; i < kSpecWaveNodes; ++i)
      std::printf("%%s[\"%%llu\",\"%%llu\"]", i ? "," : "", (unsigned long long)T.anc[b][i],
                  (unsigned long long)T.edge[b][i]);
    std::printf("]");
  }
  std::printf("], \"trees\": [");
  for (int b = 0; b < kSpecBuckets; ++b) {
    std::printf("%%s[", b ? "," : "");
    for (int i = 0; i < kSpecNodes; ++i) {
      const SpecNode& x = T.nd[b][i];
      std::printf("%%s[%%d,%%d,%%d,%%d,%%d,%%d]", i ? "," : "", x.orig, x.child[0], x.child[1], x.depth, x.lvl,
                  T.maxlvl[b][i + 1]);
    }
    std::printf("]");
  }
  std::printf("]}\n");
}
"""


@pytest.fixture(scope="module")
def tables(tmp_path_factory):
    d = tmp_path_factory.mktemp("spec_tree")
    src, exe = d / "t.cpp", d / "t"
    src.write_text(PROG % HDR)
    subprocess.run(["g++", "-std=c++17", "-O1", str(src), "-o", str(exe)], check=True)
    out = json.loads(subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout)
    return out


def _paths(tree):
    """Each node's decision path from the root (0 reject, 1 accept) and parent."""
    path, parent = {0: ()}, {0: -1}
    for i, (_, c0, c1, *_rest) in enumerate(tree):
        for e, c in ((0, c0), (1, c1)):
            if c >= 0:
                assert c > i  # best-first: a child comes after its parent
                path[c] = path[i] + (e,)
                parent[c] = i
    return path, parent


def test_trees_are_consistent_best_first_prefixes(tables):
    N, grid = tables["nodes"], tables["p"]
    assert len(tables["trees"]) == len(grid) and grid[0] == 0 and grid[-1] == 1
    for b, tree in enumerate(tables["trees"]):
        p = grid[b]
        assert len(tree) == N
        path, parent = _paths(tree)
        assert sorted(path) == list(range(N))  # every node reachable from the root
        prob = []
        ml = 0
        for i, (orig, c0, c1, depth, lvl, maxlvl) in enumerate(tree):
            pa = path[i]
            assert depth == len(pa)
            assert lvl == sum(pa)
            # origin: the last node on the path reached through an accept edge
            o, n = -1, 0
            for e in pa:
                nxt = tree[n][1 + e]
                if e == 1:
                    o = n
                n = nxt
            assert orig == o, (b, i)
            ml = max(ml, lvl)
            assert maxlvl == ml
            prob.append(np.prod([p if e else 1 - p for e in pa]) if pa else 1.0)
        # best-first: path probabilities never increase along the node order
        assert all(prob[i] >= prob[i + 1] - 1e-15 for i in range(N - 1)), b
        if b == 0:
            assert all(t[2] == -1 and t[0] == -1 and t[3] == i for i, t in enumerate(tree))  # the reject chain
        if b == len(grid) - 1:
            assert all(t[1] == -1 and t[0] == i - 1 and t[3] == i for i, t in enumerate(tree))  # the accept chain


def _expected_steps(tree, S, p):
    path, _ = _paths(tree)
    tot = 0.0
    for i in range(S):
        pa = path[i]
        tot += np.prod([p if e else 1 - p for e in pa]) if pa else 1.0
    return tot


def test_trees_are_optimal(tables):
    """No tree of S nodes settles more steps in expectation: the optimum by
    dynamic programming over the sizes of the reject and accept subtrees,
    V(S) = 1 + max_a [(1-p) V(a) + p V(S-1-a)]."""
    grid = tables["p"]
    for b in (1, 3, 5, 8, 11, 15, 18, 21):
        p = grid[b]
        V = [0.0]
        for S in range(1, 65):
            V.append(1 + max((1 - p) * V[a] + p * V[S - 1 - a] for a in range(S)))
        for S in (1, 2, 3, 5, 8, 16, 33, 64):
            assert _expected_steps(tables["trees"][b], S, p) == pytest.approx(V[S], rel=1e-12), (b, S)


def test_speculation_gain_over_the_chains(tables):
    """The numbers DESIGN quotes: a mixing chain (p = 0.25) settles 7.25 steps
    per 64-slot round with the tree against 4.0 along the reject chain; at p =
    0.875 and 16 slots the tree is the accept chain."""
    grid = tables["p"]
    t4 = tables["trees"][grid.index(0.25)]
    assert _expected_steps(t4, 64, 0.25) == pytest.approx(7.25, abs=0.01)
    assert sum(0.75**i for i in range(64)) == pytest.approx(4.0, abs=0.01)
    t14 = tables["trees"][grid.index(0.875)]
    assert [t[3] for t in t14[:16]] == list(range(16))


def test_bucket_is_the_nearest_grid_rate(tables):
    grid = np.array(tables["p"])
    for i, b in enumerate(tables["bucket_of"]):
        p = i / 1000
        d = np.abs(grid - p)
        assert d[b] == d.min(), (p, b)


def test_walk_replays_the_sequential_chain(tables):
    """spec_walk on random decision streams: the visited nodes are consecutive
    steps, each proposing from the sequential chain's state at that step (its
    origin = the last accepted visited node), and the walk stops at the first
    node whose next node is outside the S slots (or after `left` steps)."""
    rng = np.random.default_rng(5)
    for _ in range(400):
        b = int(rng.integers(0, len(tables["p"])))
        S = int(rng.choice([1, 2, 4, 8, 16, 32, 64, 256]))
        left = int(rng.integers(1, 80))
        tree = tables["trees"][b]
        dec = rng.random(300) < rng.random()  # the sequential chain's decisions from step st on
        n, used, win, visited = 0, 0, -1, []
        while True:
            orig, c0, c1, depth = tree[n][:4]
            assert depth == used and orig == win
            a = bool(dec[used])
            visited.append(n)
            if a:
                win = n
            used += 1
            c = c1 if a else c0
            if used >= left or c < 0 or c >= S:
                break
            n = c
        assert all(v < S for v in visited)
        assert used == left or len(visited) == used


def test_parallel_path_equals_the_walk(tables):
    """The in-wave resolution (spec_on_path / spec_path_round): node n is on the
    realized path iff every ancestor decided the way n's path goes; the path's
    nodes, in index order, are exactly the walk's visited nodes, and the last
    accepted one is the walk's new state."""
    rng = np.random.default_rng(7)
    for _ in range(600):
        b = int(rng.integers(0, len(tables["p"])))
        S = int(rng.choice([1, 2, 4, 8, 16, 32, 64]))
        left = int(rng.integers(1, 80))
        tree = tables["trees"][b]
        anc = [(int(a), int(e)) for a, e in tables["anc"][b]]
        acc = 0
        for n in range(S):
            if tree[n][3] < left and rng.random() < rng.random():
                acc |= 1 << n
        # the walk
        n, used, visited, win = 0, 0, [], -1
        while True:
            a = (acc >> n) & 1
            visited.append(n)
            if a:
                win = n
            used += 1
            c = tree[n][2] if a else tree[n][1]
            if used >= left or c < 0 or c >= S:
                break
            n = c
        # the parallel form
        path = [m for m in range(S) if tree[m][3] < left and ((acc ^ anc[m][1]) & anc[m][0]) == 0]
        assert path == visited, (b, S, left)
        pa = [m for m in path if (acc >> m) & 1]
        assert (pa[-1] if pa else -1) == win
