"""bench.py argument handling that needs no GPU."""
import json
import subprocess
import sys

import pytest

from conftest import REPO


def _bench(*args):
    return subprocess.run([sys.executable, "bench.py", *args], cwd=REPO, capture_output=True, text=True, timeout=300)


def test_share_device_needs_gloo():
    r = _bench("--share-device")
    assert r.returncode != 0 and "--share-device needs --dist-backend gloo" in r.stderr


def test_help_lists_the_options():
    r = _bench("--help")
    assert r.returncode == 0 and "--scaling" in r.stdout and "--dist-backend" in r.stdout
    assert "--steps-per-launch" in r.stdout
    for opt in ("--workload", "--kernel-only", "--pmc-file", "--no-configs"):
        assert opt in r.stdout, opt


def test_unknown_workload_is_refused():
    r = _bench("--workload", "cfg9")
    assert r.returncode != 0 and "invalid choice" in r.stderr


def test_world_size_must_equal_gpus():
    """Under an external launcher WORLD_SIZE has to match --gpus (refused before any GPU call)."""
    import os

    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4"], cwd=REPO, capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_auto_steps_per_launch():
    sys.path.insert(0, REPO)
    import bench

    assert bench.auto_per_launch(65536) == 1  # the full ensemble fills the GPU: one step per launch
    assert bench.auto_per_launch(16384) == 1
    assert bench.auto_per_launch(8192) == 512  # strong scaling over 8 GPUs: long speculative launches
    assert bench.auto_per_launch(1) == 512


@pytest.mark.parametrize("gpus", [1, 2, 3, 4, 8])
def test_default_line_is_the_metrics_ensemble_for_any_gpu_count(gpus):
    """BASELINE's metric is 65 536 chains over the whole node: by default
    `bench.py --gpus N` splits them over the N GPUs (strong scaling), and the
    line's metric string names exactly the chains it timed."""
    sys.path.insert(0, REPO)
    import bench
    from ip_mcmc_amd.shard import chain_range

    metric = json.load(open(f"{REPO}/BASELINE.json"))["metric"]
    scaling, total = bench.ensemble("cfg3", gpus)
    assert scaling == "strong" and total == 65536
    assert bench.metric_name("cfg3", "lorenz96_d40_rk4_2000_pcn", total) == metric
    assert sum(b - a for a, b in (chain_range(total, r, gpus) for r in range(gpus))) == 65536
    if gpus == 8:
        assert chain_range(total, 7, 8) == (7 * 8192, 8 * 8192)  # 8 192 chains per GPU
    # weak: 65 536 on every GPU -- a different ensemble, so a different metric string
    scaling, total = bench.ensemble("cfg3", gpus, None, "weak")
    assert total == 65536 * gpus
    name = bench.metric_name("cfg3", "lorenz96_d40_rk4_2000_pcn", total)
    assert (name == metric) == (gpus == 1)
    assert f"{65536 * gpus:,} chains".replace(",", " ") in name
    # configs 4 and 5: their node ensembles, split
    assert bench.ensemble("cfg4", gpus) == ("strong", 16384)
    assert bench.ensemble("cfg5", gpus) == ("strong", 1 << 20)


def test_metric_names_the_chains_run():
    sys.path.insert(0, REPO)
    import bench

    assert bench.metric_name("cfg3", "x", 8192) == "pCN steps/sec (whole node), Lorenz-96 d=40 T=2000, 8 192 chains"
    assert bench.ensemble("cfg3", 1, 8192) == ("strong", 8192)


def _committed_lines():
    import glob

    return sorted(glob.glob(f"{REPO}/profiles/r*/bench_line.json"))


def test_committed_bench_line_keeps_the_contract():
    """profiles/r*/bench_line.json (one per round) has every key the driver's
    contract names."""
    assert _committed_lines()
    for path in _committed_lines():
        _check_line(json.load(open(path)))


def _check_line(line):
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in line, key
    assert line["config"]["workload"] and "model" not in line["config"]
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in line["roofline"], key
    for key in ("value", "unit", "cores", "kind", "sample"):
        assert key in line["cpu_baseline"], key
    assert abs(line["roofline"]["frac"] - line["roofline"]["achieved"] / line["roofline"]["peak"]) < 1e-9


def test_pmc_record_matches_the_layout():
    """roofline.traffic comes from the PMC passes of the kernel the bench runs:
    same dtype, chains, shape and lanes-per-chain layout, newest round first."""
    sys.path.insert(0, REPO)
    import bench

    rec, src = bench.pmc_record("f64", 65536, 4)
    assert rec is not None and src.startswith("profiles/r") and "40, 4, true" in " ".join(rec["kernel"])
    assert rec["hbm_bytes_per_launch"] > 0
    assert bench.pmc_record("f64", 65536, 8) == (None, None)  # no PMC pass of that layout
    assert bench.pmc_record("f64", 1000, 4) == (None, None)
