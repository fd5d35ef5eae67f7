"""bench.py's N-rank path (torch.distributed.run, barriers, max-over-ranks time,
the final gather, rank-0 JSON line) rehearsed with 2 ranks on the one-GPU box:
both ranks on cuda:0 and gloo for the collectives (RCCL needs one GPU per rank;
the driver's 8-GPU runs use it).  Started both ways: under an external
torch.distributed.run (the driver's form) and as plain `python bench.py --gpus 2`,
which launches the ranks itself (strong scaling by default: the metric's 65 536
chains split over the ranks, the weak figure -- 65 536 on every rank -- beside it),
and the config-5 workload (2^20 chains over the ranks, f64, through
shard.run_sharded with the rank-sequential posterior mean)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_rehearsal():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--chains", "4096", "--scaling", "weak", "--no-cpu", "--no-extra",
           "--no-configs", "--dist-backend", "gloo", "--share-device"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints one line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["total_chains"] == 8192 and "8 192 chains" in line["metric"]
    assert line["final_gather"]["rows"] == 8192 and "gloo" in line["final_gather"]["collective"]
    assert line["final_gather"]["mode"] == "mean"
    assert line["value"] > 0 and 0 < line["accept_rate"] < 1


def test_bench_gpus_2_launches_its_own_ranks():
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-cpu", "--dist-backend", "gloo", "--share-device"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    # BASELINE's metric is 65 536 chains over the whole node: split over the ranks
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["metric"] == json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
    assert line["config"]["total_chains"] == 65536 and line["config"]["chains_per_gpu"] == 32768
    assert line["final_gather"]["rows"] == 65536 and line["final_gather"]["inside_timed_region"]
    ex = line["extra"]
    assert ex["weak_scaling"]["total_chains"] == 131072 and ex["weak_scaling"]["chains_per_gpu"] == 65536
    assert ex["weak_scaling"]["pcn_steps_per_s"] > 0 and "131 072 chains" in ex["weak_scaling"]["metric"]
    assert ex["run_e2e_moments"]["u0_rows_per_rank"] == 32768  # rank-local u_0
    assert ex["reference_arith_kernel_pcn_steps_per_s"] > 0 and ex["run_e2e_samples"]["pcn_steps_per_s"] > 0
    # value is the end-to-end run; the kernel leg is beside it
    assert line["value"] == ex["run_e2e_moments"]["pcn_steps_per_s"] and ex["kernel_pcn_steps_per_s"] > 0
    assert abs(line["ms_per_step"] * line["steps"] / 1e3 - ex["run_e2e_moments"]["wall_s"]) < 1e-9
    # value's data in HBM; the host-buffer run (PCIe included) beside it
    assert ex["run_e2e_moments"]["data_in_hbm"] and not ex["run_e2e_pcie"]["data_in_hbm"]
    assert ex["run_e2e_pcie"]["pcn_steps_per_s"] > 0
    assert ex["mixing_posterior"]["total_chains"] == 65536 and ex["mixing_posterior"]["pcn_steps_per_s"] > 0
    # REFERENCE arith end to end beside value; the paired streams run at N = 1 only
    assert line["parity"]["reference_arith_value"] > 0 and "paired_identical_accept_frac" not in line["parity"]
    assert ex["configs"]["cfg4"]["f64"]["total_chains"] == 16384
    assert ex["configs"]["cfg5"]["f64"]["total_chains"] == 1 << 20 and ex["configs"]["cfg5"]["f32"]["pcn_steps_per_s"] > 0
    ap = ex["configs"]["cfg5"]["arith_parity"]  # config 5's bit-exact carrier and its rate
    assert ap["bit_exact_arith"] == "reference" and ap["bit_exact_pcn_steps_per_s"] > 0
    assert 0 < ap["reference_frac_of_peak"] < ap["reference_op_ceiling_frac"] < 0.5


def test_bench_cfg5_workload_two_ranks():
    """`bench.py --gpus 2 --workload cfg5`: one line for BASELINE config 5 at its
    full ensemble (2^20 chains, 524 288 per rank)."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--workload", "cfg5", "--steps", "2",
           "--warmup", "1", "--no-cpu", "--dist-backend", "gloo", "--share-device"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["config"]["workload"] == "lorenz96_d256_rk4_10000_pcn"
    assert line["config"]["total_chains"] == 1 << 20 and line["config"]["chains_per_gpu"] == 1 << 19
    assert line["final_gather"]["mode"] == "mean" and line["final_gather"]["rows"] == 1 << 20
    assert line["value"] > 0


def test_bench_one_rank_over_rccl():
    """`torch.distributed.run --nproc-per-node 1 bench.py` (the driver's launch
    form with N = 1): the line's barriers, gathers and max over ranks go
    through a one-rank RCCL group on the MI355X -- the collectives the
    8-GPU line issues, on hardware (RCCL refuses two ranks on one GPU)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "1", "--chains", "8192", "--no-cpu", "--no-extra",
           "--no-configs", "--no-parity"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and "RCCL" in line["final_gather"]["collective"]
    assert line["config"]["total_chains"] == 8192 and "8 192 chains" in line["metric"]
    assert line["value"] > 0 and line["final_gather"]["rows"] == 8192
