"""Per-position kernel durations of a repeated step from a rocprofv3 kernel trace:
the sequence of launches between consecutive occurrences of an anchor kernel is one
step; prints the median duration per position plus VGPR / scratch / grid of each.
    python tools/trace_seq.py run_kernel_trace.csv [--anchor k_prologue]"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="k_prologue")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur = [], None
    for r in rows:
        nm = r["Kernel_Name"].replace("bgcn::(anonymous namespace)::", "").replace("void ", "")
        nm = nm.split("(")[0]
        if a.anchor in nm:
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((nm, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r))
    L = statistics.mode(len(s) for s in steps)
    steps = [s for s in steps if len(s) == L][2:]
    for k in range(L):
        nm, _, r = steps[0][k]
        d = statistics.median(s[k][1] for s in steps)
        print(f"{k:2d} {nm:28s} {d:7.1f} us  vgpr {r['VGPR_Count']:>3s} agpr {r['Accum_VGPR_Count']:>3s} "
              f"scratch {r['Scratch_Size']:>4s} lds {r['LDS_Block_Size']:>6s} wg {r['Workgroup_Size_X']:>4s} "
              f"grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}")


if __name__ == "__main__":
    main()
