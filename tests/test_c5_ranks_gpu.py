"""C5 across ranks (BASELINE.json configs[4]): scripts/c5_bench.py with WORLD_SIZE = 2 (both ranks
on cuda:0, a gloo timing group) deals the 8 pruning candidates round-robin over the ranks (the
reference's independent candidate fits, symmetry_breaking_quantum.py:196-238) and runs every
forward on the split/merge path (QCTN.split halves + boundary contraction).  Each candidate
keeps its own SGDG draw stream, so after the same steps every candidate's loss equals the
one-rank run's (the data path has no collective)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world):
    port = _port()
    cmd = [sys.executable, os.path.join(ROOT, "scripts", "c5_bench.py"), "--steps", "3", "--warmup", "2",
           "--cpu-steps", "0", "--port", str(port)]
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1")
        procs.append(subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=280) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-2000:] for o in outs]
    line = [x for x in outs[0][0].splitlines() if x.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.timeout(600)
def test_c5_candidates_split_over_two_ranks():
    one = _run(1)
    two = _run(2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["candidates_per_rank"] == [4, 4]
    assert "split" in two["forward"]
    assert len(one["loss_after"]) == len(two["loss_after"]) == 8
    for a, b in zip(one["loss_after"], two["loss_after"]):
        assert abs(a - b) < 1e-12, (a, b)
    assert len(two["host_issue_ms_per_step"]) == 2
