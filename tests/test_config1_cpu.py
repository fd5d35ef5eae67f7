"""BASELINE config 1 without a GPU: "1 chain on NumPy CPU path (plumbing, no GPU)".

The reference's own composition (report/scripts/stuart_examples.py:50-55,
58-109: a closure G(u) = np.dot(g, u), pCNProposer, CountedAccepter(pCNAccepter(
EvolutionPotential(G, data, noise))), one chain) runs in a child process that
sees no GPU (CUDA_VISIBLE_DEVICES="" and HIP_VISIBLE_DEVICES=""): MCMCSampler's
host step takes its draws from libipmc_host.so, and the chains equal the
reference sampler's (tests/golden lin_*: the reference MCMCSampler with the
same Philox draws injected) bit for bit.  Nothing under oracle/ is loaded by
the child (asserted from sys.modules).
"""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent(r"""
    import json, sys
    import numpy as np
    sys.path.insert(0, REPO)
    import torch
    from ip_mcmc_amd import (CountedAccepter, EvolutionPotential, GaussianDistribution, MCMCSampler, PhiloxRNG,
                             pCNAccepter, pCNProposer)
    from ip_mcmc_amd import hostloop

    z = np.load(GOLDEN)
    gamma, beta, seed, n_samples, burn_in, interval = z["lin_meta"]
    g, y = z["lin_g"], z["lin_y"]

    def build_evolution_pCN_sampler(observation_operator, data, noise, prior, rng, chain):
        # stuart_examples.py:50-55 (its beta, the fixture's)
        potential = EvolutionPotential(observation_operator, data, noise)
        proposer = pCNProposer(beta=beta, prior=prior)
        accepter = CountedAccepter(pCNAccepter(potential=potential))
        return MCMCSampler(proposer, accepter, rng, chain_offset=chain), accepter

    out = {"cuda": torch.cuda.is_available(), "draws": hostloop.draw_source(), "chains": []}
    for chain in range(4):
        s, acc = build_evolution_pCN_sampler(lambda u: np.dot(g, u), y, GaussianDistribution(0, gamma**2),
                                             GaussianDistribution(np.zeros(4), np.identity(4)),
                                             PhiloxRNG(int(seed)), chain)
        smp = s.run(np.zeros(4), n_samples=int(n_samples), burn_in=int(burn_in), sample_interval=int(interval))
        out["chains"].append({"equal": bool(np.array_equal(smp, z["lin_samples"][chain])),
                              "accepts": int(acc.accepts), "calls": int(acc.calls), "path": s.last_path})
    out["oracle_loaded"] = sorted(m for m in sys.modules if m == "oracle" or m.startswith("oracle."))
    out["libs"] = sorted({l.split()[-1] for l in open("/proc/self/maps") if "libipmc" in l})
    print(json.dumps(out))
""")


def test_config1_reference_composition_runs_without_a_gpu_and_matches_the_fixture(golden):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    code = f"REPO = {REPO!r}\nGOLDEN = {os.path.join(REPO, 'tests', 'golden', 'reference_golden.npz')!r}\n" + CHILD
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["cuda"] is False and res["draws"] == "host"
    assert res["oracle_loaded"] == []
    assert any(x.endswith("libipmc_host.so") for x in res["libs"])
    for c, r in enumerate(res["chains"]):
        assert r["path"] == "host" and r["equal"], (c, r)
        assert r["accepts"] == int(golden["lin_counts"][c, 1]) and r["calls"] == int(golden["lin_counts"][c, 0])


def test_stuart_reference_example_runs_without_a_gpu():
    """examples/stuart_reference.py (the reference script's two examples, 5 000
    samples each by default; 300 here) end to end on the CPU: the sample means
    approach the exact posterior (results.org:59-62)."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    p = subprocess.run([sys.executable, os.path.join(REPO, "examples", "stuart_reference.py"), "300"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    recs = [json.loads(line) for line in p.stdout.splitlines() if line.startswith("{")]
    assert [r["example"] for r in recs] == ["2.1", "2.2"]
    for r in recs:
        assert r["path"] == "host" and 0 < r["accept_ratio"] < 1
        assert np.allclose(r["sample_mean"], r["exact_mean"], atol=0.1), r
