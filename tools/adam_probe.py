"""Time the fused Adam launch alone (BiGCN twitter parameters) with and without the
weight images, for rocprofv3 --kernel-trace --stats: python tools/adam_probe.py plain|images [reps]."""
import sys

import torch

sys.path.insert(0, ".")
from bigcn_amd import BiGCN, _lib, optim  # noqa: E402
from bigcn_amd.optim import bigcn_adam  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "images"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    dev = torch.device("cuda:0")
    m = BiGCN(5000, 64, 64, 4).to(dev)
    opt = bigcn_adam(m)
    grads = [torch.randn_like(p) * 1e-3 for p in opt.params()]
    img = torch.empty(_lib.lib().bgcn_weight_images_size(5000), dtype=torch.uint8, device=dev)
    enc = list(m.encoder_params())
    roles = {id(enc[0]): optim.IMAGE_TD_W1, id(enc[4]): optim.IMAGE_BU_W1,
             id(enc[2]): optim.IMAGE_TD_W2, id(enc[6]): optim.IMAGE_BU_W2}
    for name, images in (("plain", None), ("images", (img, 5000, roles))):
        if name != mode:
            continue
        for _ in range(20):
            opt.step(grads=grads, images=images)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            opt.step(grads=grads, images=images)
        e1.record()
        torch.cuda.synchronize()
        print(f"adam {name} {1000 * e0.elapsed_time(e1) / reps:.2f} us/launch (host-bound if ~ launch rate)")


if __name__ == "__main__":
    main()
