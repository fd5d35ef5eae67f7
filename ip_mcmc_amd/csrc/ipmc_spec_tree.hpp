// Speculation trees for the speculative sweeps (ipmc_sweep_common.hpp).
//
// A speculative round evaluates several future steps of one chain at once.
// Step st+d's proposal depends on the decisions of steps st .. st+d-1 only
// through the state it proposes from: the last proposal accepted before it
// (or the round's starting state).  A node of the tree is one such proposal:
// the decision path leading to it fixes its depth d (its step), its origin
// (the node whose proposal it starts from, -1: the round's state) and its
// level (the accepted edges on its path: the proposals that must be formed
// before it).  A round gives its S slots the first S nodes of a tree; the
// chain then walks the tree along the real decisions, each node's decision
// being the one the sequential chain makes there (same proposal, same
// uniform), so results are bit-identical to the sequential chain whatever
// the tree -- the tree only sets how many steps a round settles.
//
// For an acceptance rate p the best tree of S nodes (most settled steps in
// expectation) holds the S most probable paths: a node reached along a
// accepted and r rejected edges has probability p^a (1-p)^r, and a child is
// never more probable than its parent, so taking nodes best-first gives every
// prefix of S nodes as the best S-node tree.  p = 0 gives the reject chain
// (every slot from the current state: the first acceptance ends the round),
// p = 1 the accept chain (slot s from slot s-1's proposal); in between the
// tree branches: at p = 0.24 and S = 64 it settles 7.4 steps per round in
// expectation against the better chain's 4.2; at p = 0.88, S = 16 it is the
// accept chain (7.3).
//
// The tables are built at compile time: kSpecBuckets acceptance rates
// (kSpecGridP: sixteenths, and finer towards 0 and 1, where wide rounds tell
// 1/32 from 1/16), kSpecNodes nodes each, ties broken by creation order (the
// reject child first).
#pragma once

#include <stdint.h>

namespace ipmc {

constexpr int kSpecBuckets = 23;
constexpr int kSpecNodes = 256;
// SpecNode.depth / .lvl and maxlvl are uint8_t: a node index, depth or level
// must fit in 8 bits
static_assert(kSpecNodes <= 256, "spec-tree node fields are uint8_t");
constexpr double kSpecGridP[kSpecBuckets] = {
    0.0,         1.0 / 128,   1.0 / 64,    1.0 / 32,    1.0 / 16,     2.0 / 16,   3.0 / 16,   4.0 / 16,
    5.0 / 16,    6.0 / 16,    7.0 / 16,    8.0 / 16,    9.0 / 16,     10.0 / 16,  11.0 / 16,  12.0 / 16,
    13.0 / 16,   14.0 / 16,   15.0 / 16,   31.0 / 32,   63.0 / 64,    127.0 / 128, 1.0};

// The bucket nearest an estimated acceptance rate (the midpoints between
// grid points as thresholds).
inline constexpr int spec_bucket_of(double p) {
  int b = 0;
  for (int i = 0; i + 1 < kSpecBuckets; ++i) b += p > 0.5 * (kSpecGridP[i] + kSpecGridP[i + 1]) ? 1 : 0;
  return b;
}

struct SpecNode {
  int16_t orig;  // the node whose proposal this one starts from (-1: the round's state)
  int16_t child[2];  // the next node after a reject / an accept here (-1: none)
  uint8_t depth;  // the step offset in the round
  uint8_t lvl;    // accepted edges on the path: proposals formed before this one
};

// In-wave rounds (at most 64 slots) resolve the walk in parallel: node n is
// on the realized path iff every ancestor a decided the way n's path goes
// there -- ((acc ^ edge[n]) & anc[n]) == 0 over the slots' decision bits.
constexpr int kSpecWaveNodes = 64;

struct SpecTrees {
  SpecNode nd[kSpecBuckets][kSpecNodes];
  uint8_t maxlvl[kSpecBuckets][kSpecNodes + 1];  // max lvl over the first n nodes
  uint64_t anc[kSpecBuckets][kSpecWaveNodes];    // node n's ancestors (bit a)
  uint64_t edge[kSpecBuckets][kSpecWaveNodes];   // ... and the decision its path takes at each (1: accept)
};

namespace spec_tree_detail {
struct Cand {
  double pr;
  int seq, parent, edge;
};
constexpr bool before(const Cand& a, const Cand& b) { return a.pr > b.pr || (a.pr == b.pr && a.seq < b.seq); }
struct Heap {
  Cand h[2 * kSpecNodes + 2]{};
  int n = 0;
  constexpr void push(const Cand& c) {
    int i = n++;
    h[i] = c;
    while (i > 0) {
      const int p = (i - 1) / 2;
      if (!before(h[i], h[p])) break;
      const Cand t = h[i];
      h[i] = h[p];
      h[p] = t;
      i = p;
    }
  }
  constexpr Cand pop() {
    const Cand top = h[0];
    h[0] = h[--n];
    int i = 0;
    while (true) {
      const int l = 2 * i + 1, r = l + 1;
      int b = i;
      if (l < n && before(h[l], h[b])) b = l;
      if (r < n && before(h[r], h[b])) b = r;
      if (b == i) break;
      const Cand t = h[i];
      h[i] = h[b];
      h[b] = t;
      i = b;
    }
    return top;
  }
};
}  // namespace spec_tree_detail

constexpr SpecTrees make_spec_trees() {
  SpecTrees t{};
  for (int b = 0; b < kSpecBuckets; ++b) {
    const double p = kSpecGridP[b];
    spec_tree_detail::Heap heap{};
    int seq = 0;
    heap.push({1.0, seq++, -1, 0});
    int ml = 0;
    t.maxlvl[b][0] = 0;
    for (int i = 0; i < kSpecNodes; ++i) {
      const spec_tree_detail::Cand c = heap.pop();
      SpecNode& x = t.nd[b][i];
      x.child[0] = x.child[1] = -1;
      if (c.parent < 0) {
        x.orig = -1;
        x.depth = 0;
        x.lvl = 0;
      } else {
        SpecNode& par = t.nd[b][c.parent];
        par.child[c.edge] = (int16_t)i;
        x.depth = (uint8_t)(par.depth + 1);
        x.orig = c.edge ? (int16_t)c.parent : par.orig;
        x.lvl = (uint8_t)(par.lvl + (c.edge ? 1 : 0));
      }
      ml = x.lvl > ml ? x.lvl : ml;
      t.maxlvl[b][i + 1] = (uint8_t)ml;
      if (i < kSpecWaveNodes) {
        t.anc[b][i] = 0;
        t.edge[b][i] = 0;
        if (c.parent >= 0) {  // the parent's ancestors plus the parent itself
          t.anc[b][i] = t.anc[b][c.parent] | (uint64_t(1) << c.parent);
          t.edge[b][i] = t.edge[b][c.parent] | (uint64_t(c.edge) << c.parent);
        }
      }
      heap.push({c.pr * (1.0 - p), seq++, i, 0});
      heap.push({c.pr * p, seq++, i, 1});
    }
  }
  return t;
}

}  // namespace ipmc
