"""Interleaved A/B runs of the bench (or a probe) over library variants and runtime knobs.

    python tools/ab.py [VARIANT ...] [--workloads twitter15 weibo_bf16] [--reps 2]
                       [--steps 200] [--warmup 10] [--bench-args "--feat-mode dense"]
                       [--probe "tools/agg_probe.py --graphs td"] [--out gpurun_out/ab.txt]

A VARIANT is ``base`` (the in-tree library, the default), or comma-separated items: a
library built with other compile-time knobs (a path ending in ``.so``, selected per run
through BGCN_LIB) and/or ``NAME=VALUE`` environment overrides the library reads per call
(``BGCN_PREP_LANES=1``, ``BGCN_X6_PIPE=0,BGCN_GEMM_X6=1``, ``v.so,BGCN_PREP_BLOCKS=256``).  Every (rep, workload, variant)
runs as its own child process with its own time limit - reps outermost, so box drift shows
up as spread rather than as a difference - and prints one line: the bench's trees/s,
ms/step, the roofline kernel's span and fraction, and the standalone pass's paced /
unpaced fractions (or the probe's output).  The bench runs light (no CPU baseline, no
comparison legs) unless --bench-args brings them back.  On the GPU box:

    gpurun -- 'python tools/ab.py base BGCN_PREP_LANES=1 --workloads "twitter15 weibo_bf16"'
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIGHT = ["--no-cpu-baseline", "--compare-dense", "0", "--compare-dropedge", "0", "--aggregation", "0",
         "--dropin", "0", "--host-fed", "0", "--eval-path", "0"]


def variant_env(v: str) -> dict:
    env = dict(os.environ)
    env.pop("BGCN_LIB", None)
    if v == "base":
        return env
    for kv in v.split(","):
        if kv.endswith(".so"):       # a library variant (may be combined with NAME=VALUE items)
            env["BGCN_LIB"] = os.path.abspath(kv)
            continue
        k, _, val = kv.partition("=")
        if not k or not _:
            raise SystemExit(f"bad variant {v!r}: base, a .so path or NAME=VALUE[,NAME=VALUE]")
        env[k] = val
    return env


def summary(out: str) -> str:
    d = json.loads(out.strip().splitlines()[-1])
    r = d.get("roofline") or {}
    c = d.get("compaction_standalone") or {}
    return " ".join(str(x) for x in (d["value"], d["ms_per_step"], r.get("avg_ms"), r.get("frac"),
                                     (c.get("paced") or {}).get("frac"), (c.get("unpaced") or {}).get("frac"),
                                     d.get("invalid_steps")))


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("variants", nargs="*", default=["base"])
    ap.add_argument("--workloads", default="twitter15", help="space-separated bench workloads")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--bench-args", default="", help="extra bench.py arguments")
    ap.add_argument("--probe", help="run this script (with its arguments) per variant instead of the bench")
    ap.add_argument("--timeout", type=int, default=200, help="seconds per run")
    ap.add_argument("--out", default=os.path.join("gpurun_out", "ab.txt"))
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    workloads = a.workloads.split() if not a.probe else ["-"]
    with open(a.out, "a") as log:
        for rep in range(1, a.reps + 1):
            for w in workloads:
                for v in a.variants:
                    if a.probe:
                        cmd = [sys.executable, *shlex.split(a.probe)]
                    else:
                        cmd = [sys.executable, "bench.py", "--workload", w, *LIGHT, "--steps", str(a.steps),
                               "--warmup", str(a.warmup), *shlex.split(a.bench_args)]
                    try:
                        p = subprocess.run(cmd, cwd=ROOT, env=variant_env(v), capture_output=True, text=True,
                                           timeout=a.timeout)
                    except subprocess.TimeoutExpired:
                        line = f"{rep} {w} {v} TIMEOUT"
                        print(line, flush=True)
                        log.write(line + "\n")
                        return 1   # no further GPU step after a time-out
                    if p.returncode != 0:
                        line = f"{rep} {w} {v} FAILED rc={p.returncode}: {p.stderr.strip()[-300:]}"
                        print(line, flush=True)
                        log.write(line + "\n")
                        return 1   # no further GPU step after a failure
                    line = f"{rep} {w} {v} " + (("\n" + p.stdout) if a.probe else summary(p.stdout))
                    print(line, flush=True)
                    log.write(line + "\n")
                    log.flush()
    return 0


if __name__ == "__main__":
    sys.exit(main())
