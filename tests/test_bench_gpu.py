"""bench.py's multi-rank entry point on the GPU: `--gpus N` without a launcher starts the ranks
itself (env launch, as the reference's comm_torch.py:146-168 expects RANK / WORLD_SIZE /
MASTER_ADDR), here all on cuda:0 over gloo (RCCL needs one GPU per rank).

* bitstring sharding (the default): rank r's block equals a 1-rank run of block r (`--batch r`),
  and the strong-scaling pass on block 0 (slices sharded + all-reduce) equals the 1-rank block 0;
* `--shard slices`: the reduced amplitudes equal the 1-rank run's.
"""
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
    """bench.py's stdout is ONE compact headline line; the full result comes from --details."""
    details = out + ".details.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args + COMMON
                       + ["--save-out", out, "--details", details],
                       capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    head = json.loads(lines[0])
    assert len(lines[0]) <= 2048 and r.stdout.rstrip().splitlines()[-1] == lines[0]
    with open(details) as f:
        full = json.load(f)
    assert head["value"] == full["value"]
    return full


def _close(a, b):
    assert a.shape == b.shape == (2,) * 20
    err = np.abs(a - b).max() / np.abs(a).max()
    assert err < 1e-5, err


@pytest.mark.timeout(600)
def test_bench_two_ranks_self_launch(tmp_path):
    one = _run(["--gpus", "1"], str(tmp_path / "one.npy"))
    one_b1 = _run(["--gpus", "1", "--batch", "1"], str(tmp_path / "one_b1.npy"))
    two = _run(["--gpus", "2", "--devices", "0,0", "--dist-backend", "gloo"], str(tmp_path / "two.npy"))
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2 and two["scaling"] == "weak"
    assert two["config"]["parallelism"] == "bitstrings2" and two["config"]["slices_per_rank"] == 8
    assert two["config"]["amplitudes_per_step"] == 2 * one["config"]["amplitudes_per_step"]
    assert two["value"] > 0 and two["roofline"]["launches_timed"] > 0
    assert two["slices_strong"]["slices_per_rank"] == 4 and two["slices_strong"]["value"] > 0
    a, a1 = np.load(tmp_path / "one.npy"), np.load(tmp_path / "one_b1.npy")
    assert np.abs(a - a1).max() > 1e-3 * np.abs(a).max()   # another block of amplitudes
    _close(a, np.load(tmp_path / "two.npy"))
    _close(a1, np.load(tmp_path / "two.rank1.npy"))
    _close(a, np.load(tmp_path / "two.slices.npy"))
    sl = _run(["--gpus", "2", "--devices", "0,0", "--dist-backend", "gloo", "--shard", "slices"],
              str(tmp_path / "sl.npy"))
    assert sl["scaling"] == "strong" and sl["config"]["slices_per_rank"] == 4 and "slices_strong" not in sl
    _close(a, np.load(tmp_path / "sl.npy"))


@pytest.mark.timeout(900)
def test_bench_eight_ranks_one_slice_each(tmp_path):
    """The N = 8 layout of the driver's scaling run rehearsed on one GPU: eight self-launched
    ranks (gloo), each its own block, then one block with one slice per rank and one all-reduce
    of eight partial amplitude buffers -- equal to the 1-rank amplitudes."""
    one = _run(["--gpus", "1"], str(tmp_path / "one.npy"))
    one_b7 = _run(["--gpus", "1", "--batch", "7"], str(tmp_path / "one_b7.npy"))
    eight = _run(["--gpus", "8", "--devices", "0,0,0,0,0,0,0,0", "--dist-backend", "gloo"],
                 str(tmp_path / "eight.npy"))
    assert eight["n_gpus"] == 8 and eight["slices_strong"]["slices_per_rank"] == 1
    a = np.load(tmp_path / "one.npy")
    _close(a, np.load(tmp_path / "eight.npy"))
    _close(a, np.load(tmp_path / "eight.slices.npy"))
    _close(np.load(tmp_path / "one_b7.npy"), np.load(tmp_path / "eight.rank7.npy"))
