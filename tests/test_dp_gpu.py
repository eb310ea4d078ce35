"""Data-parallel training on the GPU box (SURVEY.md §8e, configs/jhu_fog2snow.yml): two ranks
sharing the one GPU over gloo (the driver's 8-GPU runs use RCCL; the collective call sites
are the same).  (1) one final-mode DGTrainer step, data-parallel, equals the single-process
emulation (per-half gradients averaged, per-rank BN); (2) `bench.py --gpus 2` launches its
own ranks and reports n_gpus 2 with parameters in sync."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_dp_final_train_step_matches_emulation(dev):
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", f"--master-port={_port()}",
                        os.path.join(HERE, "dp_final_worker.py")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.count("OK") == 2, (r.stdout[-2000:], r.stderr[-3000:])


def test_dp_syncbn_strong_scaling(dev):
    """Strong-scaled DP with SyncBatchNorm (tests/dp_syncbn_worker.py): rank-averaged gradients,
    loss and BN running statistics equal the single-process full-batch step."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", f"--master-port={_port()}",
                        os.path.join(HERE, "dp_syncbn_worker.py")],
                       capture_output=True, text=True, timeout=300)
    print(r.stdout[-1500:])
    assert r.returncode == 0 and r.stdout.count("OK") == 2, (r.stdout[-2000:], r.stderr[-3000:])


def test_bench_gpus_flag_launches_ranks(dev):
    env = dict(os.environ, DGVCC_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup",
                        "1", "--batch", "2", "--height", "256", "--width", "256", "--no-cpu-baseline", "--no-bf16"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(line) == 1, r.stdout
    out = json.loads(line[0])
    assert out["n_gpus"] == 2 and out["config"]["rccl_world_size"] == 2, out
    assert out["params_in_sync"] is True, out


def test_rccl_backend_executes(dev):
    """The DP path's collectives through RCCL (backend "nccl") on one rank (tests/rccl_worker.py)."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
                        "--master-addr", "127.0.0.1", f"--master-port={_port()}",
                        os.path.join(HERE, "rccl_worker.py")],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0 and "OK rccl" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
