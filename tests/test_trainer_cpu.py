"""End-to-end trainer (reference resnet/main.py behaviour) on CPU: single process
and 2-rank gloo through our launcher; evaluation + checkpoint + resume."""
import os
import random
import subprocess
import sys

import pytest
from conftest import free_port
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "2"
    return env


def test_trainer_single_process(tmp_path):
    from pytorch_distributed_tutorials_amd.train import main
    args = ["--arch", "resnet18", "--data", "synthetic-cifar", "--synthetic-samples", "64",
            "--batch-size", "16", "--num_epochs", "2", "--eval-every", "1",
            "--max-steps-per-epoch", "2", "--model_dir", str(tmp_path), "--num-classes", "10",
            "--backend", "gloo"]
    assert main(args) == 0
    path = tmp_path / "resnet_distributed.pth"
    sd = torch.load(path, weights_only=True)
    assert len(sd) == 122 and all(k.startswith("module.") for k in sd)
    assert os.path.exists(str(path) + ".train_state.pt")
    # resume continues from the saved epoch (sidecar) and trains one more epoch
    resume = [a for a in args]
    resume[resume.index("--num_epochs") + 1] = "3"
    assert main(resume + ["--resume"]) == 0


@pytest.mark.slow
def test_trainer_two_ranks_via_launcher(tmp_path):
    port = free_port()
    cmd = [sys.executable, "-m", "pytorch_distributed_tutorials_amd.launch", "--nproc_per_node=2",
           "--master_port", str(port), "--use-local-rank-arg",
           "--arch", "resnet18", "--data", "synthetic-cifar", "--synthetic-samples", "64",
           "--batch-size", "8", "--num_epochs", "2", "--eval-every", "1",
           "--max-steps-per-epoch", "2", "--model_dir", str(tmp_path), "--num-classes", "10",
           "--backend", "gloo"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), timeout=400, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = r.stdout
    assert "Local Rank: 0, Epoch: 0, Training ..." in out
    assert "Local Rank: 1, Epoch: 1, Training ..." in out
    assert "Epoch: 0, Accuracy:" in out and "Epoch: 1, Accuracy:" in out
    assert os.path.exists(tmp_path / "resnet_distributed.pth")
