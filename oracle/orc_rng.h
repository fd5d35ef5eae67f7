/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  CPU restatement used as the parity checker
 * for libipmc.so.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product path never does.
 *
 * Counter-based randomness + deterministic transcendentals (host C).
 *
 * The reference draws its proposal from numpy's PCG64 Generator
 * (distribution.py:114-118, rng.multivariate_normal) and its accept uniform
 * from Generator.random() (accepter.py:62).  A shared sequential stream cannot
 * be reproduced by 65 536 concurrent chains, so the build replaces it by a
 * counter-based stream (Philox4x32-10, Salmon et al. SC'11 / Random123):
 *   ctr = (slot, chain_global, step_lo32, step_hi32), key = (seed_lo32, seed_hi32)
 *   slot = j  -> normal pair (2j, 2j+1) of the proposal
 *   slot = 0xFFFFFFFF -> the accept uniform
 * The reference's own RNG-injection seam (test_utilities.py:11-26, MockRNG)
 * feeds exactly these draws into the reference sampler when the golden
 * fixtures are made (tests/golden/make_golden.py).
 *
 * log / sincos are evaluated with + - * / only, in a fixed order, so that the
 * HIP device code and this file produce bit-identical doubles (the contract
 * is spelled out in DESIGN.md §4).
 */
#ifndef ORC_RNG_H
#define ORC_RNG_H
#include <stdint.h>

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double orc_log(double x);
void orc_sincos_2pi(double t, double* s, double* c);
/* standard normal z[0], z[1] for components 2*slot, 2*slot+1 */
void orc_normal_pair(uint64_t seed, uint64_t chain, uint64_t step, uint32_t slot, double z[2]);
double orc_normal(uint64_t seed, uint64_t chain, uint64_t step, uint32_t comp);
double orc_accept_uniform(uint64_t seed, uint64_t chain, uint64_t step);

#endif
