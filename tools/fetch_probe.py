"""Driver of tools/fetch_probe.hip (run under rocprofv3 --pmc FETCH_SIZE, and alone for the
times): each kernel reads a known number of distinct bytes; tools/prof.py counters (or the
summary this prints with --pmc-dir) gives FETCH_SIZE per dispatch to compare.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/fp -- python tools/fetch_probe.py
    python tools/fetch_probe.py --pmc-dir gpurun_out/fp      # the ratio table
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GIB = 1 << 30
# (kernel, piece bytes, bytes read): 512 MB distinct pieces of each size, the whole GiB streamed
CASES = [("k_fp_stream", 0, GIB), ("k_fp_gather<64>", 64, 512 << 20), ("k_fp_gather<128>", 128, 512 << 20),
         ("k_fp_gather<256>", 256, 512 << 20)]


def run(reps):
    import torch
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libfetchprobe.so"))
    dev = torch.device("cuda", 0)
    buf = torch.ones(GIB // 4, dtype=torch.int32, device=dev)
    out = torch.zeros(4, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    S = ctypes.c_void_p(s.cuda_stream)
    P = ctypes.c_void_p
    res = {}
    for name, piece, nbytes in CASES:
        ms = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            if piece == 0:
                rc = L.fp_stream(P(buf.data_ptr()), ctypes.c_int64(GIB), P(out.data_ptr()), S)
            else:
                rc = L.fp_gather(piece, P(buf.data_ptr()), ctypes.c_int64(GIB), ctypes.c_int64(nbytes // piece),
                                 P(out.data_ptr()), S)
            b.record(s)
            assert rc == 0, rc
            torch.cuda.synchronize()
            ms.append(a.elapsed_time(b))
        best = min(ms)
        res[name] = {"bytes": nbytes, "best_ms": round(best, 4), "gbs": round(nbytes / (best * 1e-3) / 1e9, 1)}
    print(json.dumps(res), flush=True)


def table(pmc_dir):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from prof import _per_form
    per = _per_form(pmc_dir, "FETCH_SIZE")
    out = {}
    for name, piece, nbytes in CASES:
        forms = per.get(name, {})
        vals = [v for g in forms.values() for v in g]
        if not vals:
            continue
        fetch = sum(vals) / len(vals)
        out[name] = {"bytes_read": nbytes, "fetch_size_bytes": round(fetch), "fetch_over_bytes": round(fetch / nbytes, 4),
                     "correction_to_bytes": round(nbytes / fetch, 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--pmc-dir")
    a = ap.parse_args()
    table(a.pmc_dir) if a.pmc_dir else run(a.reps)
