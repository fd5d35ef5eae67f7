"""The examples/ scripts (the reference's own studies on the GPU) at reduced
sizes: each must run through the public API and land on the answer the
reference's problem has (an exact posterior where one exists)."""
import importlib.util
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REPO, "examples", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need the MI355X"
    return torch.device("cuda", 0)


@pytest.mark.parametrize("example", ["2.1", "2.2"])
def test_stuart_examples_reach_the_exact_posterior(dev, example):
    """stuart_examples.py:58-163 (Stuart 2010 examples 2.1 and 2.2): the pooled
    posterior mean of 512 chains is within 4 Monte-Carlo standard errors of the
    exact Gaussian posterior mean, the variance within 10 %."""
    ex = _load("stuart_examples")
    gamma = 0.5
    if example == "2.1":
        A, u, noise = (ex.digits(np.pi, 1).astype(float).reshape(1, 1), np.array([2.0]),
                       ex.GaussianDistribution(mean=0, covariance=gamma**2))
    else:
        A, u, noise = (ex.digits(np.pi, 2).astype(float).reshape(2, 1), np.array([0.5]),
                       ex.GaussianDistribution(mean=np.zeros(2), covariance=np.identity(2) * gamma**2))
    r = ex.run_example(example, A, u, gamma, noise, chains=512, n_samples=200)
    assert np.all(np.abs(r["mean_error_in_mcse"]) < 4), r
    assert np.allclose(r["posterior_var"], r["exact_var"], rtol=0.1), r
    assert 0.05 < r["accept_rate"] < 0.95, r


def test_sharded_config5_example_one_gpu(dev):
    """examples/sharded_config5.py (config 5 through shard.run_sharded) on one
    GPU with a reduced ensemble: both precisions run and report a finite
    posterior-mean difference."""
    import json
    import subprocess
    import sys

    p = subprocess.run([sys.executable, os.path.join(REPO, "examples", "sharded_config5.py"), "2048", "2"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    recs = [json.loads(line) for line in p.stdout.splitlines() if line.startswith("{")]
    assert [r.get("dtype") for r in recs[:2]] == ["float64", "float32"]
    assert all(r["pcn_steps_per_s"] > 0 and r["chains"] == 2048 for r in recs[:2])
    assert np.isfinite(recs[2]["posterior_mean_max_abs_diff_f32_f64"])
