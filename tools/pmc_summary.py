"""Per-kernel mean of every counter in rocprofv3 --pmc output dirs (tools/pmc_chain.sh).
    python tools/pmc_summary.py gpurun_out/pmc_chain"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"bgcn::\(anonymous namespace\)::", "", n)
    return re.sub(r"^void ", "", re.sub(r"\(.*", "", n))[:24]


def main():
    per = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    cols = sorted({c for k in per.values() for c in k})
    print(f"{'kernel':26s}" + "".join(f"{c[:14]:>16s}" for c in cols))
    for k, d in sorted(per.items()):
        if not k.startswith("k_"):
            continue
        print(f"{k:26s}" + "".join(f"{sum(d[c]) / len(d[c]):16.4g}" if d.get(c) else f"{'-':>16s}" for c in cols))


if __name__ == "__main__":
    main()
