"""Diagnose GraNd GPU-vs-oracle differences on one example set: scores from every engine
variant (fast split-bf16 convs or MIOpen fp32, fused or tape, fp32 or bf16x3 norms) against
the CPU oracle, plus the oracle itself in float64."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from data_diet_distributed_amd import checkpoints, synthetic  # noqa: E402
from data_diet_distributed_amd.scoring import ScoreConfig, ScoringEngine  # noqa: E402
from oracle import pipeline as o_pipe  # noqa: E402


def main():
    cuda = torch.device("cuda:0")
    images, labels = synthetic.make_images(100, 10, seed=31)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=6)["net"]
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    ref = o_pipe.grand_scores(sd, images, labels, batch_size=50)
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    norm32 = o_pipe.normalize
    o_pipe.normalize = lambda u8: norm32(u8).double()
    try:
        ref64 = o_pipe.grand_scores(sd64, images, labels, batch_size=50)
    except Exception as exc:  # noqa: BLE001
        print("float64 oracle failed:", exc)
        ref64 = None
    o_pipe.normalize = norm32
    variants = {
        "fused_fast_bf16x3": dict(),
        "tape_fast_bf16x3": dict(fused_grand=False),
        "tape_miopen_bf16x3": dict(fused_grand=False, fast_convs=False),
        "tape_miopen_fp32": dict(fused_grand=False, fast_convs=False, pegrad_precision="fp32"),
        "tape_miopen_fp32_nofold": dict(fused_grand=False, fast_convs=False, fold_bn=False,
                                        pegrad_precision="fp32"),
    }
    print("oracle fp32 vs float64 max rel:",
          None if ref64 is None else float(np.max(np.abs(ref / ref64 - 1))))
    for name, kw in variants.items():
        eng = ScoringEngine(checkpoints.build_models([sd], device=cuda),
                            ScoreConfig(methods=("grand",), select_by="grand", grand_batch=64,
                                        **kw), cuda)
        got = eng.score_shard(img, lab, 0, 100)["grand"].cpu().numpy()
        rel = np.abs(got / ref - 1)
        i = int(np.argmax(rel))
        line = f"{name:28s} max rel vs oracle {rel[i]:.3e} at {i} (got {got[i]:.6g} ref {ref[i]:.6g})"
        if ref64 is not None:
            r64 = np.abs(got / ref64 - 1)
            line += f" | vs f64 max {r64.max():.3e} at {int(np.argmax(r64))}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
