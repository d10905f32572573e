"""Time every distinct Conv2d of a ResNet under MIOpen (F.conv2d forward and backward-data,
immediate mode as the engine runs it) to find the shapes MIOpen serves with its naive
fallback kernels.   python tools/probe_miopen.py [--arch resnet50] [--imagenet] [--batch B]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from data_diet_distributed_amd.resnet import build  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet50")
    ap.add_argument("--imagenet", action="store_true")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--classes", type=int, default=100)
    ap.add_argument("--benchmark", action="store_true")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = a.benchmark
    dev = torch.device("cuda:0")
    m = build(a.arch, a.classes, "imagenet" if a.imagenet else "cifar").to(dev)
    shapes = {}
    hooks = []
    for name, mod in m.named_modules():
        if isinstance(mod, torch.nn.Conv2d):
            def hook(mod, i, o, name=name):
                shapes.setdefault((tuple(i[0].shape[1:]), mod.out_channels, mod.kernel_size,
                                   mod.stride, mod.padding), (name, mod))
            hooks.append(mod.register_forward_hook(hook))
    with torch.no_grad():
        m(torch.randn(2, 3, 224 if a.imagenet else 32, 224 if a.imagenet else 32, device=dev))
    for h in hooks:
        h.remove()
    B = a.batch
    for (ishape, cout, k, s, p), (name, mod) in shapes.items():
        x = torch.randn((B,) + ishape, device=dev)
        w = mod.weight.detach()
        y = F.conv2d(x, w, None, s, p)
        dy = torch.randn_like(y)

        def fwd():
            return F.conv2d(x, w, None, s, p)

        def bwd():
            return torch.ops.aten.convolution_backward(dy, x, w, None, list(s), list(p), [1, 1],
                                                       False, [0, 0], 1, [True, False, False])[0]
        res = []
        for fn in (fwd, bwd):
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 3
            flop = 2.0 * B * y.shape[2] * y.shape[3] * cout * ishape[0] * k[0] * k[1]
            res.append((dt * 1e3, flop / dt / 1e12))
        print(f"{name:24s} in={ishape} cout={cout} k={k} s={s}  fwd {res[0][0]:8.2f} ms "
              f"{res[0][1]:6.1f} TF/s  bwd {res[1][0]:8.2f} ms {res[1][1]:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
