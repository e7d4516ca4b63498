"""Per-dispatch HBM traffic of libbgcn kernels from rocprofv3 PMC passes.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> [--out profiles/<name>.json]

<fetch_dir> / <write_dir>: output directories of separate passes
``rocprofv3 --pmc FETCH_SIZE --output-format csv`` and ``--pmc WRITE_SIZE`` (the two
counters do not fit one pass on gfx950).  Applies the MI355X_MICROARCH.md corrections:
FETCH_SIZE (KiB) reports half the bytes of a wide streaming read on gfx950 -> x2;
WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.  Prints and writes, per kernel,
the mean corrected bytes per dispatch."""
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
    per = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter:
                    per[_short(row["Kernel_Name"])].append(float(row["Counter_Value"]) * 1024.0)
    return per


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
        f = fetch.get(k, [])
        w = write.get(k, [])
        rd = 2.0 * sum(f) / len(f) if f else None          # gfx950: FETCH_SIZE = 1/2 of the bytes
        wr = sum(w) / len(w) if w else None
        res[k] = {"read_bytes": rd, "write_bytes": wr,
                  "hbm_bytes": (rd or 0.0) + (wr or 0.0), "dispatches": max(len(f), len(w))}
        print(f"{k:40s} read {rd or 0:14.0f} B  write {wr or 0:14.0f} B  ({max(len(f), len(w))} dispatches)")
    if out:
        with open(out, "w") as fh:
            json.dump({"correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE as is; KiB->B",
                       "kernels": res}, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
