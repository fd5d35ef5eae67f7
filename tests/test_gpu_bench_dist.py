"""bench.py's N-rank path (torch.distributed.run, barriers, max-over-ranks time,
the final gather, rank-0 JSON line) rehearsed with 2 ranks on the one-GPU box:
both ranks on cuda:0 and gloo for the collectives (RCCL needs one GPU per rank;
the driver's 8-GPU runs use it).  Started both ways: under an external
torch.distributed.run (the driver's form) and as plain `python bench.py --gpus 2`,
which launches the ranks itself (strong scaling on the metric's 65 536 chains)."""
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
           "--dist-backend", "gloo", "--share-device"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints one line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["total_chains"] == 8192
    assert line["final_gather"]["rows"] == 8192 and "gloo" in line["final_gather"]["collective"]
    assert line["value"] > 0 and 0 < line["accept_rate"] < 1


def test_bench_gpus_2_launches_its_own_ranks():
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-cpu", "--dist-backend", "gloo", "--share-device"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["total_chains"] == 65536 and line["config"]["chains_per_gpu"] == 32768
    assert line["final_gather"]["rows"] == 65536
    ex = line["extra"]
    assert ex["weak_scaling"]["total_chains"] == 131072 and ex["weak_scaling"]["pcn_steps_per_s"] > 0
    assert ex["reference_arith_pcn_steps_per_s"] > 0 and ex["run_e2e_pcn_steps_per_s"] > 0
