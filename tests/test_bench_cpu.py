"""bench.py argument handling that needs no GPU."""
import json
import subprocess
import sys

from conftest import REPO


def _bench(*args):
    return subprocess.run([sys.executable, "bench.py", *args], cwd=REPO, capture_output=True, text=True, timeout=300)


def test_share_device_needs_gloo():
    r = _bench("--share-device")
    assert r.returncode != 0 and "--share-device needs --dist-backend gloo" in r.stderr


def test_help_lists_the_options():
    r = _bench("--help")
    assert r.returncode == 0 and "--scaling" in r.stdout and "--dist-backend" in r.stdout


def test_committed_bench_line_keeps_the_contract():
    """profiles/r1/bench_line.json has every key the driver's contract names."""
    line = json.load(open(f"{REPO}/profiles/r1/bench_line.json"))
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in line, key
    assert line["config"]["workload"] and "model" not in line["config"]
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in line["roofline"], key
    for key in ("value", "unit", "cores", "kind", "sample"):
        assert key in line["cpu_baseline"], key
    assert abs(line["roofline"]["frac"] - line["roofline"]["achieved"] / line["roofline"]["peak"]) < 1e-9
