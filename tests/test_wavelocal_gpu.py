"""The sweep2 pass-barrier elision (kS2PmSync, tq_plan.cpp s2_layout: no workgroup barrier between
two passes whose elements stay with the same waves) must not change a single bit: the same plans
compiled with TQ_S2_WAVELOCAL=0 (a barrier before every pass) in a child process give bitwise the
same amplitudes on multi-pass layouts (C2: 33 dependent levels; a C4-form network with deferred
tails and slices).  ADVICE r5: the elision assumes gi == threadIdx.x (mod 512) and 64-lane waves,
asserted in tq_sweep2.hip; this is the end-to-end check of it."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from tneq_qc_amd.circuits import BrickWall, amplitude_task, config_task
from tneq_qc_amd.expression import HipContractExpression
out = {}
tasks = {"C2": config_task("C2"),
         "cut": amplitude_task(BrickWall(16, 8, 4), list(range(5, 11)), cut=8, n_slice=2, defer=(3, 3))}
for name, t in tasks.items():
    e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
    ops = [torch.from_numpy(o).to("cuda:0", torch.complex64) for o in t.operands]
    out[name] = e(*ops).cpu().numpy()
    out[name + "_syncs"] = np.array([int(l.split("syncs=")[1].split("/")[0]) for l in e.plan(torch.complex64).describe().splitlines() if "syncs=" in l])
    out[name + "_passes"] = np.array([int(l.split("syncs=")[1].split("/")[1].split()[0]) for l in e.plan(torch.complex64).describe().splitlines() if "syncs=" in l])
np.savez(sys.argv[2], **out)
"""


def _run(tmp_path, wavelocal):
    path = str(tmp_path / f"wl{wavelocal}.npz")
    env = dict(os.environ, TQ_S2_WAVELOCAL=str(wavelocal))
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, path], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return np.load(path)


@pytest.mark.timeout(600)
def test_barrier_elision_is_bitwise_neutral(tmp_path):
    on, off = _run(tmp_path, 1), _run(tmp_path, 0)
    for name in ("C2", "cut"):
        # the elision is active (fewer barriers than passes) on these layouts, and absent with 0
        assert on[name + "_syncs"].sum() < on[name + "_passes"].sum(), name
        assert np.array_equal(off[name + "_syncs"], off[name + "_passes"]), name
        assert np.array_equal(on[name], off[name]), name
