"""Per-kernel average durations of several rocprofv3 --stats runs side by side
(tools/ab_libs.sh output dirs).  python tools/ab_stats.py gpurun_out/ab_base gpurun_out/ab_x ..."""
import csv
import os
import sys


def main():
    dirs = sys.argv[1:]
    res = {}
    for i, d in enumerate(dirs):
        for r in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
            nm = r["Name"].replace("bgcn::(anonymous namespace)::", "").replace("void ", "")[:34]
            res.setdefault(nm, {})[i] = (float(r["AverageNs"]) / 1e3, int(r["Calls"]))
    print(f"{'kernel':36s}" + "".join(f"{os.path.basename(d)[-14:]:>16s}" for d in dirs))
    for nm, v in sorted(res.items(), key=lambda kv: -max(x[0] for x in kv[1].values())):
        print(f"{nm:36s}" + "".join(f"{v[i][0]:9.1f} x{v[i][1]:<5d}" if i in v else f"{'-':>16s}"
                                    for i in range(len(dirs))))


if __name__ == "__main__":
    main()
