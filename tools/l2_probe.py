"""Driver of tools/l2_probe.hip: same-XCD vs other-XCD reads of what the previous kernel
wrote (16 MB, 2 MB per XCD).  python tools/l2_probe.py"""
import ctypes
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    L = ctypes.CDLL(os.path.join(ROOT, "tools", "libl2probe.so"))
    dev = torch.device("cuda", 0)
    nbytes = 16 << 20
    buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    out = torch.zeros(4, device=dev)
    s = torch.cuda.current_stream()
    P = lambda t: ctypes.c_void_p(t.data_ptr())
    S = ctypes.c_void_p(s.cuda_stream)
    for shift in (0, 1, 0, 1):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        tot = 0.0
        for it in range(200):
            L.l2p_write(P(buf), ctypes.c_int64(nbytes), 32, ctypes.c_float(float(it)), S)
            e[0].record(s)
            L.l2p_read(P(buf), ctypes.c_int64(nbytes), 32, shift, P(out), S)
            e[1].record(s)
            torch.cuda.synchronize()
            if it >= 20:
                tot += e[0].elapsed_time(e[1])
        print(f"read after write, shift {shift}: {tot / 180 * 1e3:7.2f} us per 16 MB read", flush=True)


if __name__ == "__main__":
    main()
