"""Per-launch-form kernel durations from a rocprofv3 kernel trace.

    python tools/kernel_forms.py <run_kernel_trace.csv> [--match k_prep_b]

rocprofv3's --stats summary averages every dispatch of a kernel symbol, but k_prep_b runs in
several launch forms (the in-step X pass on the first preparation lane, the DropEdge / K1
roles on the second, the bench's standalone paced / unpaced passes), told apart by grid
size.  This prints, per (kernel, grid size), the dispatch count and the average / median
duration - the figure bench.py's roofline (device-side span of the X-pass launch) is
checked against."""
from __future__ import annotations

import csv
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
    forms = defaultdict(list)
    with open(args[0]) as fh:
        for row in csv.DictReader(fh):
            name = re.sub(r"\(.*", "", re.sub(r"\(anonymous namespace\)::", "", row["Kernel_Name"]))
            name = re.sub(r"^void ", "", name)
            if not name.startswith("bgcn::") or (match and match not in name):
                continue
            grid = int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"])
            forms[(name, grid)].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':44s} {'grid':>9s} {'blocks':>7s} {'n':>5s} {'avg us':>9s} {'median us':>10s}")
    for (name, grid), d in sorted(forms.items(), key=lambda kv: -sum(kv[1])):
        d = sorted(d)
        print(f"{name:44s} {grid:9d} {grid // 256:7d} {len(d):5d} {sum(d) / len(d):9.1f} {d[len(d) // 2]:10.1f}")


if __name__ == "__main__":
    main()
