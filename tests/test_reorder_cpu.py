"""The sweep2 compiler's gate re-listing (tq_plan.cpp s2_reorder_squares, TQ_S2_REORDER): commuting
square gates are re-listed into fuller register blocks only when that saves passes, so every op
keeps or lowers its pass count, and the plan's other ops stay as they were.  Compile-only (no GPU):
the flag is read once per process, so each setting compiles in a child process.  Parity of the
re-listed chains on the GPU: the C2 / C3 / C4 oracle tests (test_contract_gpu.py,
test_fullsize_gpu.py), which run with the default (on)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import json, sys, torch
sys.path.insert(0, sys.argv[1])
from tneq_qc_amd.circuits import config_task
from tneq_qc_amd.expression import HipContractExpression
out = {}
for cfg in sys.argv[2:]:
    t = config_task(cfg)
    e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
    d = e.plan(torch.complex64).describe().splitlines()
    ops = [l for l in d if l.startswith("[once]") or l.startswith("[slice]")]
    out[cfg] = [(l.split(" step ")[0], int(l.split("passes=")[1].split()[0]) if "passes=" in l else -1,
                 l.split("gates=")[1].split()[0] if "gates=" in l else "") for l in ops]
print(json.dumps(out))
"""


def _passes(reorder, cfgs):
    import json
    env = dict(os.environ, TQ_S2_REORDER=str(reorder))
    r = subprocess.run([sys.executable, "-c", _CHILD, ROOT, *cfgs], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.timeout(900)
def test_relisting_never_adds_passes():
    cfgs = ["C2", "C4"]
    on, off = _passes(1, cfgs), _passes(0, cfgs)
    for cfg in cfgs:
        assert len(on[cfg]) == len(off[cfg]), cfg   # the same ops, in the same order
        for (b1, p1, g1), (b0, p0, g0) in zip(on[cfg], off[cfg]):
            assert (b1, g1) == (b0, g0), cfg
            assert p1 <= p0, (cfg, p1, p0)
    # C2's chains leave room: strictly fewer passes overall (r06: 216 -> 209)
    assert sum(p for _, p, _ in on["C2"] if p > 0) < sum(p for _, p, _ in off["C2"] if p > 0)


_LANES = r"""
import json, sys, torch
sys.path.insert(0, sys.argv[1])
from tneq_qc_amd.circuits import config_task, with_batch
from tneq_qc_amd.expression import HipContractExpression
t = with_batch(config_task("C4"), 0)
e = HipContractExpression(t.eq, *t.shapes, optimize=t.path, slices=t.sliced)
d = e.plan(torch.complex64).describe().splitlines()
s2 = [l for l in d if " SWEEP2 " in l and "passes=" in l]
print(json.dumps({"passes": sum(int(l.split("passes=")[1].split()[0]) for l in s2),
                  "lanes": sum(int(l.split("lanes=")[1].split()[0]) for l in s2 if "lanes=" in l),
                  "ops": len(s2)}))
"""


@pytest.mark.timeout(600)
def test_lane_blocks_are_opt_in_and_cut_passes():
    """TQ_S2_LANEBLK=1 (lane blocks: 6-position register blocks over 4 lanes, tq_plan.cpp
    lane_span) compiles C4 with lane passes and fewer passes than the default, which has none
    (r06: C4's big sweep ops 174 -> 125 passes).  Parity of the opt-in path: test_laneblk_gpu.py."""
    import json
    res = {}
    for on in (0, 1):
        env = dict(os.environ, TQ_S2_LANEBLK=str(on))
        r = subprocess.run([sys.executable, "-c", _LANES, ROOT], env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        res[on] = json.loads(r.stdout.strip().splitlines()[-1])
    assert res[0]["lanes"] == 0 and res[1]["lanes"] > 0
    assert res[1]["ops"] == res[0]["ops"]
    assert res[1]["passes"] < res[0]["passes"]
