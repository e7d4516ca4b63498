"""Per-stream timeline of one training step from a rocprofv3 kernel trace.

    python tools/step_timeline.py <run_kernel_trace.csv> [--step 15]

Steps are delimited by the fused Adam kernel (or by --after KERNEL, e.g. the spin that
tools/trace_probe.py puts before every step).  Prints every kernel of the chosen step
(start / end relative to the previous Adam's end, stream) and per-stream busy time."""
import argparse
import collections
import csv
import re


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"bgcn::", "", n)
    return re.sub(r"\(.*", "", n)[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=15)
    ap.add_argument("--after", default="k_adam",
                    help="kernel that delimits steps (tools/trace_probe.py: k_alu, the spin before each step)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    adam = [i for i, r in enumerate(rows) if a.after in r["Kernel_Name"]]
    i0 = adam[a.step]
    if a.after == "k_adam":
        i1 = adam[a.step + 1]
    else:   # through the step's Adam
        i1 = next(i for i in range(i0 + 1, len(rows)) if "k_adam" in rows[i]["Kernel_Name"])
    t0 = int(rows[i0]["End_Timestamp"])
    busy = collections.defaultdict(float)
    for r in rows[i0 + 1:i1 + 1]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        busy[r["Stream_Id"]] += (e - s) / 1e3
        print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f}  s{r['Stream_Id']}  {short(r['Kernel_Name'])}")
    print("step", (int(rows[i1]["End_Timestamp"]) - t0) / 1e3, "us; busy per stream:",
          {k: round(v, 1) for k, v in busy.items()})


if __name__ == "__main__":
    main()
