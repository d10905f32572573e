"""Interleaved in-process A/B of the EL2N forward with the unit tails fused into the next
convs' staging (el2n_fast.FUSE_UNIT_INPUT) against the separate dd_bn_apply passes: one
1024-row chunk (8 BN groups of 128), ResNet-18, median of per-round means.

    python tools/ab_unit_input.py [--rounds 9] [--iters 20] [--arch resnet18]"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from data_diet_distributed_amd import checkpoints, el2n_fast, synthetic  # noqa: E402
from oracle import pipeline as o_pipe  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    images, _ = synthetic.make_images(a.batch, 10, seed=1)
    sd = synthetic.make_checkpoint(a.arch, 10, seed=0)["net"]
    model = checkpoints.build_models([sd], a.arch, 10, device=dev)[0]
    model.eval()
    model.prepare_fast_convs()
    x = o_pipe.normalize(images).to(dev).contiguous()
    outs = {}
    times = {True: [], False: []}
    for r in range(a.rounds):
        for fuse in ((True, False) if r % 2 == 0 else (False, True)):
            el2n_fast.FUSE_UNIT_INPUT = fuse
            outs[fuse] = el2n_fast.forward_logits(model, x, 128, a.batch)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                el2n_fast.forward_logits(model, x, 128, a.batch)
            e1.record()
            torch.cuda.synchronize()
            times[fuse].append(e0.elapsed_time(e1) / a.iters)
    same = torch.equal(outs[True], outs[False])
    mf, mu = statistics.median(times[True]), statistics.median(times[False])
    print(f"EL2N forward {a.arch} B={a.batch}: separate apply {mu:.3f} ms (min "
          f"{min(times[False]):.3f}) | fused {mf:.3f} ms (min {min(times[True]):.3f}) | "
          f"speed {mu / mf:.3f} | logits bitwise equal: {same}")


if __name__ == "__main__":
    main()
