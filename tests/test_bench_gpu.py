"""bench.py's multi-rank entry point on the GPU: `--gpus 2` without a launcher starts two ranks
itself (env launch, as the reference's comm_torch.py:146-168 expects RANK / WORLD_SIZE /
MASTER_ADDR), here both on cuda:0 over gloo (RCCL needs one GPU per rank).  The JSON line must
report n_gpus 2 and the reduced amplitudes must equal the 1-rank run's."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--config", "C4", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-c5", "--no-alt", "--no-other"]


def _run(args, out):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args + COMMON + ["--save-out", out],
                       capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(600)
def test_bench_two_ranks_self_launch(tmp_path):
    one = _run(["--gpus", "1"], str(tmp_path / "one.npy"))
    two = _run(["--gpus", "2", "--devices", "0,0", "--dist-backend", "gloo"], str(tmp_path / "two.npy"))
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["slices"] == 8 and two["config"]["slices_per_rank"] == 4
    assert two["value"] > 0 and two["roofline"]["launches_timed"] > 0
    a, b = np.load(tmp_path / "one.npy"), np.load(tmp_path / "two.npy")
    assert a.shape == b.shape == (2,) * 20
    err = np.abs(a - b).max() / np.abs(a).max()
    assert err < 2e-5, err


@pytest.mark.timeout(900)
def test_bench_eight_ranks_one_slice_each(tmp_path):
    """The N = 8 layout of the driver's scaling run rehearsed on one GPU: eight self-launched
    ranks (gloo), one slice each (no slice lanes: the batch-1 split-K GEMM path), one all-reduce
    of eight partial amplitude buffers -- equal to the 1-rank amplitudes."""
    one = _run(["--gpus", "1"], str(tmp_path / "one.npy"))
    eight = _run(["--gpus", "8", "--devices", "0,0,0,0,0,0,0,0", "--dist-backend", "gloo"],
                 str(tmp_path / "eight.npy"))
    assert eight["n_gpus"] == 8 and eight["config"]["slices_per_rank"] == 1
    a, b = np.load(tmp_path / "one.npy"), np.load(tmp_path / "eight.npy")
    err = np.abs(a - b).max() / np.abs(a).max()
    assert err < 2e-5, err
