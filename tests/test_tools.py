"""CPU tests of the measurement tooling: tools/prof.py's rocprofv3 CSV readers (the PMC
traffic bench.py's roofline.traffic is read from, the launch-form split, the timeline) on
small synthetic CSVs in rocprofv3's column layout, and the committed traffic files bench.py
loads."""
from __future__ import annotations

import csv
import glob
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "tools", "prof.py")
K = "void bgcn::(anonymous namespace)::k_prep_b<float>(bgcn::(anonymous namespace)::PrepArgs)"
A = "void bgcn::(anonymous namespace)::k_adam(bgcn_adam_args, bgcn::WeightImages)"


def _pmc(d, counter, rows):
    os.makedirs(os.path.join(d, "host"), exist_ok=True)
    with open(os.path.join(d, "host", "run_counter_collection.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for i, (name, grid, kib) in enumerate(rows):
            w.writerow([i, grid, name, counter, kib])


def _run(*args):
    return subprocess.run([sys.executable, PROF, *args], capture_output=True, text=True, check=True).stdout


def test_traffic_corrections_and_dominant_form(tmp_path):
    f, w = str(tmp_path / "fetch"), str(tmp_path / "write")
    # the in-step pass (grid 98560) dispatched 3x, the standalone pass (grid 1966336) once and
    # reading a little more, the DropEdge form (grid 65536) reading little
    _pmc(f, "FETCH_SIZE", [(K, 98560, 1000.0)] * 3 + [(K, 1966336, 1100.0), (K, 65536, 10.0)])
    _pmc(w, "WRITE_SIZE", [(K, 98560, 5.0)] * 3 + [(K, 1966336, 5.0), (K, 65536, 1.0)])
    out = str(tmp_path / "t.json")
    _run("traffic", f, w, "--out", out)
    d = json.load(open(out))["kernels"]["bgcn::k_prep_b<float>"]
    assert d["read_bytes"] == 2 * 1000.0 * 1024      # FETCH_SIZE x2 (gfx950), KiB -> B
    assert d["write_bytes"] == 5.0 * 1024
    assert d["dispatches"] == 3                       # the most dispatched of the heavy forms
    assert set(d["forms"]) == {"98560", "1966336", "65536"}


def test_forms_and_timeline(tmp_path):
    trace = tmp_path / "run_kernel_trace.csv"
    cols = ["Kernel_Name", "Stream_Id", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Grid_Size_Y",
            "Grid_Size_Z"]
    rows = [(A, 1, 0, 1000), (K, 2, 1500, 3500), (K, 2, 1600, 5600), (A, 1, 6000, 7000)]
    with open(trace, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(cols)
        for name, st, t0, t1 in rows:
            w.writerow([name, st, t0, t1, 98560 if t1 - t0 == 2000 else 65536, 1, 1])
    forms = _run("forms", str(trace), "--match", "k_prep_b")
    assert "98560" in forms and "65536" in forms
    tl = _run("timeline", str(trace), "--step", "0").splitlines()
    assert tl[-1].startswith("step 6.0 us")              # previous Adam's end -> next Adam's end
    assert any("k_prep_b<float>" in l and "s2" in l for l in tl)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(ROOT, "profiles", "r04_pmc_traffic_*.json"))))
def test_committed_traffic_files(path):
    """bench.py reads roofline.traffic from these: the pass over X carries a dominant form with
    read bytes at least its algorithmic X bytes' order (hundreds of MB)."""
    d = json.load(open(path))
    k = d["kernels"]
    name = next(n for n in k if n.startswith("bgcn::k_prep_b"))
    assert k[name]["read_bytes"] > 1e8 and k[name]["dispatches"] >= 1


def test_ab_variant_env(monkeypatch):
    """tools/ab.py's variant parsing: base drops BGCN_LIB, a .so path sets it, NAME=VALUE
    pairs set the overrides."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import ab
    finally:
        sys.path.pop(0)
    monkeypatch.setenv("BGCN_LIB", "/elsewhere/libbgcn.so")
    assert "BGCN_LIB" not in ab.variant_env("base")
    assert ab.variant_env("build/variants/libbgcn_x.so")["BGCN_LIB"].endswith("build/variants/libbgcn_x.so")
    e = ab.variant_env("BGCN_PREP_LANES=1,BGCN_X6_PIPE=0")
    assert e["BGCN_PREP_LANES"] == "1" and e["BGCN_X6_PIPE"] == "0" and "BGCN_LIB" not in e
    e = ab.variant_env("build/variants/libbgcn_x.so,BGCN_PREP_BLOCKS=256")
    assert e["BGCN_LIB"].endswith("libbgcn_x.so") and e["BGCN_PREP_BLOCKS"] == "256"
    with pytest.raises(SystemExit):
        ab.variant_env("nonsense")
