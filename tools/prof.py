"""Readers for rocprofv3 CSV output (kernel traces and --pmc passes) of libbgcn runs.

    python tools/prof.py traffic <fetch_dir> <write_dir> [--out profiles/<name>.json]
    python tools/prof.py forms <run_kernel_trace.csv> [--match k_prep_b]
    python tools/prof.py counters <pmc_dir> [<pmc_dir> ...] [--match NAME]
    python tools/prof.py timeline <run_kernel_trace.csv> [--step 15] [--after KERNEL]

traffic   HBM bytes per dispatch from separate ``--pmc FETCH_SIZE`` / ``--pmc WRITE_SIZE``
          passes (they do not fit one pass on gfx950), with the MI355X_MICROARCH.md
          corrections: FETCH_SIZE (KiB) reports half the bytes of a wide streaming read on
          gfx950 -> x2; WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.  Per kernel the
          dominant launch form (the most dispatched of the forms reading at least half the
          most: k_prep_b's in-step X pass, its second-lane DropEdge / K1 launch and the
          bench's standalone passes are told apart by grid size) and every form under
          "forms" - the JSON bench.py's roofline.traffic reads from profiles/.
forms     per (kernel, grid size) the dispatch count and average / median duration: the
          figure bench.py's device-side span of the X pass is checked against.
counters  per kernel the mean of every counter of one or more --pmc passes (SQ summaries).
timeline  per-stream timeline of one training step: steps are delimited by the fused Adam
          (or by --after KERNEL, e.g. the spin tools/trace_probe.py puts before each step);
          every kernel of the step relative to the delimiter's end, and busy time per stream.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return re.sub(r"\(.*", "", name)


def _pmc_rows(d: str):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            yield from csv.DictReader(fh)


def _per_form(d: str, counter: str):
    per = collections.defaultdict(lambda: collections.defaultdict(list))   # kernel -> grid -> values
    for row in _pmc_rows(d):
        if row["Counter_Name"] == counter:
            per[short(row["Kernel_Name"])][int(row["Grid_Size"])].append(float(row["Counter_Value"]) * 1024.0)
    return per


def _mean(v):
    return sum(v) / len(v) if v else None


def cmd_traffic(a):
    fetch, write = _per_form(a.fetch_dir, "FETCH_SIZE"), _per_form(a.write_dir, "WRITE_SIZE")
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
        most = max((e["read_bytes"] or 0.0) for e in forms.values())
        top = max((e for e in forms.values() if (e["read_bytes"] or 0.0) >= 0.5 * most),
                  key=lambda e: e["dispatches"])
        res[k] = dict(top, forms=forms)
        for g, e in forms.items():
            print(f"{k:40s} grid {g:>8s} read {e['read_bytes'] or 0:14.0f} B  write {e['write_bytes'] or 0:14.0f} B"
                  f"  ({e['dispatches']} dispatches)")
    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"correction": "FETCH_SIZE x2 (gfx950 wide streaming reads), WRITE_SIZE as is; KiB->B; "
                                     "per kernel the dominant launch form (grid size)",
                       "kernels": res}, fh, indent=1, sort_keys=True)


def cmd_forms(a):
    forms = collections.defaultdict(list)
    with open(a.trace) as fh:
        for row in csv.DictReader(fh):
            name = short(row["Kernel_Name"])
            if not name.startswith("bgcn::") or (a.match and a.match not in name):
                continue
            grid = int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"])
            forms[(name, grid)].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':44s} {'grid':>9s} {'blocks':>7s} {'n':>5s} {'avg us':>9s} {'median us':>10s}")
    for (name, grid), d in sorted(forms.items(), key=lambda kv: -sum(kv[1])):
        d = sorted(d)
        print(f"{name:44s} {grid:9d} {grid // 256:7d} {len(d):5d} {sum(d) / len(d):9.1f} {d[len(d) // 2]:10.1f}")


def cmd_counters(a):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in a.dirs:
        per = collections.defaultdict(float)   # (dispatch, kernel, counter) summed over dimensions
        for row in _pmc_rows(d):
            name = short(row["Kernel_Name"])
            if not name.startswith("bgcn::") or (a.match and a.match not in name):
                continue
            per[(row["Dispatch_Id"], name, row["Counter_Name"])] += float(row["Counter_Value"])
        for (_, name, c), v in per.items():
            vals[name][c].append(v)
    for name, cs in sorted(vals.items()):
        print(name)
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {sum(v) / len(v):16.1f}   ({len(v)} dispatches)")


def cmd_timeline(a):
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.after in r["Kernel_Name"]]
    i0 = marks[a.step]
    if a.after == "k_adam":
        i1 = marks[a.step + 1]
    else:   # through the step's Adam (its own launch, or - fused - the main stream's last kernel
        # before the next mark)
        nxt = marks[a.step + 1] if a.step + 1 < len(marks) else len(rows)
        ia = [i for i in range(i0 + 1, nxt) if "k_adam" in rows[i]["Kernel_Name"]]
        if ia:
            i1 = ia[0]
        else:
            s0 = rows[i0 + 1]["Stream_Id"]
            i1 = max(i for i in range(i0 + 1, nxt) if rows[i]["Stream_Id"] == s0)
    t0 = int(rows[i0]["End_Timestamp"])
    busy = collections.defaultdict(float)
    for r in rows[i0 + 1:i1 + 1]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        busy[r["Stream_Id"]] += (e - s) / 1e3
        print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f}  s{r['Stream_Id']}  "
              f"{short(r['Kernel_Name']).replace('bgcn::', '')[:48]}")
    print("step", (int(rows[i1]["End_Timestamp"]) - t0) / 1e3, "us; busy per stream:",
          {k: round(v, 1) for k, v in busy.items()})


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("traffic")
    p.add_argument("fetch_dir")
    p.add_argument("write_dir")
    p.add_argument("--out")
    p.set_defaults(fn=cmd_traffic)
    p = sub.add_parser("forms")
    p.add_argument("trace")
    p.add_argument("--match")
    p.set_defaults(fn=cmd_forms)
    p = sub.add_parser("counters")
    p.add_argument("dirs", nargs="+")
    p.add_argument("--match")
    p.set_defaults(fn=cmd_counters)
    p = sub.add_parser("timeline")
    p.add_argument("trace")
    p.add_argument("--step", type=int, default=15)
    p.add_argument("--after", default="k_adam")
    p.set_defaults(fn=cmd_timeline)
    a = ap.parse_args()
    a.fn(a)


if __name__ == "__main__":
    main()
