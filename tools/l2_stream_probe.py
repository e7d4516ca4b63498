"""Driver of tools/l2_stream_probe.hip: per-round latency of a dependent 256-byte-row gather chain
(the shape of the chain's aggregation / conv2 loads) with its rows in the XCD's own L2 or not,
alone and beside a non-temporal stream of the pass's size (the X window), and whether the L2
content survives a kernel boundary.

    python tools/l2_stream_probe.py [--part-rows 8192] [--steps 256] [--reps 3]

Cases (rows per XCD part: part_rows x 256 B):
  hot_in_launch   the chain's own launch warms its XCD's part, then gathers from it
  hot_after_boundary  a warm launch, then the chain launch on the part of the XCD it runs on
  other_xcd       warmed in the launch, gathers from the part another XCD warmed
  cold            a 600 MB sweep first (beyond L2 and the Infinity Cache), then the chain
each alone and with the stream running beside it ("+stream").
"""
import argparse
import ctypes
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
X_BYTES = 600 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--part-rows", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=256)
    ap.add_argument("--stream-blocks", type=int, default=384)
    ap.add_argument("--passes", type=int, default=12)
    ap.add_argument("--cu-every", type=int, default=0,
                    help="k > 1: the chain on the CUs i with i %% k == k - 1, the stream on the others")
    ap.add_argument("--cases", default="hot_in_launch,hot_after_boundary,other_xcd,cold")
    ap.add_argument("--out")
    a = ap.parse_args()
    assert a.part_rows & (a.part_rows - 1) == 0, "part_rows must be a power of two"
    import torch
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libl2streamprobe.so"))
    khz = L.l2_wallclock_khz()
    assert khz > 0, khz
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    table = torch.rand(8 * a.part_rows * 64, generator=g).to(dev)
    xbuf = torch.ones(X_BYTES // 4, dtype=torch.int32, device=dev)
    sink = torch.zeros(8, device=dev)
    out = torch.zeros(4, dtype=torch.int32, device=dev)
    waves = a.blocks * 4
    times = torch.zeros(waves, dtype=torch.int64, device=dev)
    P = ctypes.c_void_p
    h1, h2 = P(), P()
    assert L.l2_stream_create(a.cu_every, 0, ctypes.byref(h1)) == 0
    assert L.l2_stream_create(a.cu_every, 1, ctypes.byref(h2)) == 0
    s1 = torch.cuda.ExternalStream(h1.value, device=dev)
    s2 = torch.cuda.ExternalStream(h2.value, device=dev)
    S1, S2 = P(s1.cuda_stream), P(s2.cuda_stream)

    def chk(rc):
        assert rc == 0, rc

    def sweep(stream, passes, blocks):
        chk(L.l2_stream(P(xbuf.data_ptr()), ctypes.c_int64(X_BYTES), passes, blocks, P(out.data_ptr()), stream))

    def case(name, contended):
        with torch.cuda.stream(s1):
            if name == "cold":
                sweep(S1, 1, 4096)
            if name == "hot_after_boundary":
                chk(L.l2_warm(P(table.data_ptr()), a.part_rows, P(sink.data_ptr()), a.blocks, S1))
            start = torch.cuda.Event(enable_timing=True)
            start.record(s1)
        s2.wait_event(start)
        t_stream = torch.cuda.Event(enable_timing=True)
        if contended:
            with torch.cuda.stream(s2):
                sweep(S2, a.passes, a.stream_blocks)
                t_stream.record(s2)
        shift = 4 if name == "other_xcd" else 0
        warm = 1 if name in ("hot_in_launch", "other_xcd") else 0
        with torch.cuda.stream(s1):
            chk(L.l2_chain(P(table.data_ptr()), a.part_rows, shift, warm, a.steps, a.blocks, P(times.data_ptr()),
                           P(sink.data_ptr()), S1))
            t_chain = torch.cuda.Event(enable_timing=True)
            t_chain.record(s1)
        torch.cuda.synchronize()
        t = times.double().cpu() / (khz * 1e3) * 1e9 / a.steps   # ns per dependent round
        r = {"ns_per_round_p50": round(float(t.median()), 1),
             "ns_per_round_p90": round(float(t.quantile(0.9)), 1),
             "chain_launch_ms": round(start.elapsed_time(t_chain), 4)}
        if contended:
            r["stream_ms"] = round(start.elapsed_time(t_stream), 4)
            r["covered"] = r["stream_ms"] > r["chain_launch_ms"]
        return r

    res = {"part_bytes_per_xcd": a.part_rows * 256, "steps": a.steps, "chain_waves": waves,
           "stream": {"bytes": X_BYTES, "passes": a.passes, "blocks": a.stream_blocks}, "wallclock_khz": khz,
           "cu_every": a.cu_every}
    # the stream alone, for its rate
    with torch.cuda.stream(s2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s2)
        sweep(S2, a.passes, a.stream_blocks)
        e1.record(s2)
    torch.cuda.synchronize()
    res["stream_alone_tbs"] = round(X_BYTES * a.passes / (e0.elapsed_time(e1) * 1e-3) / 1e12, 2)
    for name in a.cases.split(","):
        for contended in (False, True):
            runs = [case(name, contended) for _ in range(a.reps + 1)][1:]
            best = min(runs, key=lambda r: r["ns_per_round_p50"])
            res[name + ("+stream" if contended else "")] = best
            print(name + ("+stream" if contended else ""), json.dumps(best), flush=True)
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
