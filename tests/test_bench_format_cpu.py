"""bench.py's output contract: the driver parses the LAST stdout line from a
tail of a few KB, so that line is the compact headline (<= 4 KB) and every secondary section goes
to stderr / the --details file.  Fed with a full r05 result (profiles/bench_r05j.json, a 22-KB
line that the r05 driver could not parse)."""
import io
import json
import os
import sys
from contextlib import redirect_stderr, redirect_stdout

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")


def _full():
    with open(os.path.join(ROOT, "profiles", "bench_r05j.json")) as f:
        return json.load(f)


def test_headline_is_compact_and_complete():
    res = _full()
    assert len(json.dumps(res)) > 3 * bench.HEADLINE_MAX_BYTES   # the r05 failure mode
    line = bench.headline_line(res)
    assert len(line.encode()) <= bench.HEADLINE_MAX_BYTES
    h = json.loads(line)
    for k in REQUIRED:
        assert k in h, k
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in h["roofline"], k
    for k in ("value", "unit", "cores", "kind", "cpu_model"):
        assert k in h["cpu_baseline"], k
    assert h["value"] == res["value"] and h["ms_per_step"] == res["ms_per_step"]
    assert h["roofline"]["frac"] == pytest.approx(res["roofline"]["frac"], rel=1e-4)
    assert h["secondary"]["C3"][0] == pytest.approx(res["config_C3"]["value"], rel=1e-4)
    assert h["secondary"]["permute"][2] is True


def test_headline_fits_even_with_huge_strings():
    res = _full()
    res["data"] = "x" * 10000
    res["roofline"]["kernel"] = "k" * 10000
    res["cpu_baseline"]["sample"] = "s" * 10000
    for i in range(200):
        res[f"config_C{i}"] = {"value": 1.0, "unit": "u" * 50}
    line = bench.headline_line(res)
    assert len(line.encode()) <= bench.HEADLINE_MAX_BYTES
    assert json.loads(line)["value"] == res["value"]


def test_emit_last_stdout_line_is_the_headline(tmp_path):
    res = _full()
    out, err = io.StringIO(), io.StringIO()
    path = tmp_path / "details.json"
    with redirect_stdout(out), redirect_stderr(err):
        bench.emit(res, str(path))
    lines = out.getvalue().splitlines()
    assert len(lines) == 1
    h = json.loads(lines[-1])
    assert h["metric"] == res["metric"]
    assert "[bench-detail] config_C4g " in err.getvalue()
    assert json.loads(path.read_text())["config_C4x4"] == res["config_C4x4"]


@pytest.mark.parametrize("key", ["roofline", "cpu_baseline"])
def test_headline_survives_missing_sections(key):
    res = _full()
    res.pop(key)
    h = json.loads(bench.headline_line(res))
    assert h["value"] == res["value"]
