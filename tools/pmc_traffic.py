"""Per-dispatch HBM traffic of libbgcn kernels from rocprofv3 PMC passes.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> [--out profiles/<name>.json]

<fetch_dir> / <write_dir>: output directories of separate passes
``rocprofv3 --pmc FETCH_SIZE --output-format csv`` and ``--pmc WRITE_SIZE`` (the two
counters do not fit one pass on gfx950).  Applies the MI355X_MICROARCH.md corrections:
FETCH_SIZE (KiB) reports half the bytes of a wide streaming read on gfx950 -> x2;
WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.  Prints and writes, per kernel,
the mean corrected bytes per dispatch of its dominant launch form (the most dispatched of
the forms reading at least half the most: a kernel launched in several forms - k_prep_b's
in-step X pass, its second-lane launch of DropEdge / K1 roles, the bench's standalone
unpaced pass - is told apart by grid size), and every form under "forms"."""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def _short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return re.sub(r"\(.*", "", name)


def _load(d: str, counter: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(lambda: defaultdict(list))   # kernel -> grid size -> values
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter:
                    per[_short(row["Kernel_Name"])][int(row["Grid_Size"])].append(float(row["Counter_Value"]) * 1024.0)
    return per


def _mean(v):
    return sum(v) / len(v) if v else None


def main():
    args = sys.argv[1:]
    out = None
    if "--out" in args:
        i = args.index("--out")
        out = args[i + 1]
        args = args[:i] + args[i + 2:]
    fetch = _load(args[0], "FETCH_SIZE")
    write = _load(args[1], "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("bgcn::"):
            continue
        forms = {}
        for g in sorted(set(fetch.get(k, {})) | set(write.get(k, {}))):
            f, w = fetch.get(k, {}).get(g, []), write.get(k, {}).get(g, [])
            rd = 2.0 * _mean(f) if f else None          # gfx950: FETCH_SIZE = 1/2 of the bytes
            wr = _mean(w)
            forms[str(g)] = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes": (rd or 0.0) + (wr or 0.0),
                             "dispatches": max(len(f), len(w))}
        # the dominant form: of those reading at least half the most, the most dispatched
        # (k_prep_b: the in-step X pass, not the bench's few standalone launches)
        most = max((e["read_bytes"] or 0.0) for e in forms.values())
        top = max((e for e in forms.values() if (e["read_bytes"] or 0.0) >= 0.5 * most),
                  key=lambda e: e["dispatches"])
        res[k] = dict(top, forms=forms)
        for g, e in forms.items():
            print(f"{k:40s} grid {g:>8s} read {e['read_bytes'] or 0:14.0f} B  write {e['write_bytes'] or 0:14.0f} B"
                  f"  ({e['dispatches']} dispatches)")
    if out:
        with open(out, "w") as fh:
            json.dump({"correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE as is; KiB->B; "
                                     "per kernel the dominant launch form (grid size)",
                       "kernels": res}, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
