"""Per-kernel mean of every counter in rocprofv3 --pmc passes (one row per kernel).

    python tools/pmc_summary.py <pmc_dir> [<pmc_dir> ...] [--match NAME]"""
from __future__ import annotations

import csv
import glob
import os
import re
import sys
from collections import defaultdict


def main():
    args = sys.argv[1:]
    match = None
    if "--match" in args:
        i = args.index("--match")
        match = args[i + 1]
        args = args[:i] + args[i + 2:]
    vals = defaultdict(lambda: defaultdict(list))
    for d in args:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)   # (dispatch, kernel, counter) summed over dimensions
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = re.sub(r"\(.*", "", re.sub(r"\(anonymous namespace\)::", "", row["Kernel_Name"]))
                    name = re.sub(r"^void ", "", name)
                    if not name.startswith("bgcn::") or (match and match not in name):
                        continue
                    per[(row["Dispatch_Id"], name, row["Counter_Name"])] += float(row["Counter_Value"])
            for (_, name, c), v in per.items():
                vals[name][c].append(v)
    for name, cs in sorted(vals.items()):
        print(name)
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {sum(v) / len(v):16.1f}   ({len(v)} dispatches)")


if __name__ == "__main__":
    main()
