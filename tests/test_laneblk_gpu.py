"""Lane blocks (TQ_S2_LANEBLK=1, tq_plan.cpp lane_span / tq_sweep2.hip blk_swap): register blocks of
6 positions, 4 in a thread's registers and 2 on its lane bits 4 / 5, with v_permlane16 / 32_swap
trading positions between them.  Off by default (the same speed); this checks the
opt-in path end to end on the headline network: a C4 block with lane blocks active against the
default plan (child processes: the flag is read once per process).  The gates' arithmetic is the
same, only the canonical leg order of some 4x4 gates differs (the summation order), so the two
complex64 results agree to the two-result bound 2e-5 of max|amp|."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL = 1e-5

_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from tneq_qc_amd.circuits import config_task, with_batch
from tneq_qc_amd.expression import HipContractExpression
t = with_batch(config_task("C4"), 3)
e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
ops = [torch.from_numpy(o).to("cuda:0", torch.complex64) for o in t.operands]
amp = e(*ops).cpu().numpy()
d = e.plan(torch.complex64).describe().splitlines()
lanes = sum(int(l.split("lanes=")[1].split()[0]) for l in d if "lanes=" in l)
np.savez(sys.argv[2], amp=amp, lanes=np.array(lanes))
"""


def _run(tmp_path, on):
    path = str(tmp_path / f"lane{on}.npz")
    env = dict(os.environ, TQ_S2_LANEBLK=str(on))
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, path], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return np.load(path)


@pytest.mark.timeout(600)
def test_lane_blocks_match_the_default_plan(tmp_path):
    on, off = _run(tmp_path, 1), _run(tmp_path, 0)
    assert int(on["lanes"]) > 0 and int(off["lanes"]) == 0
    ref = np.abs(off["amp"]).max()
    assert ref > 0
    assert np.abs(on["amp"] - off["amp"]).max() <= 2 * TOL * ref
