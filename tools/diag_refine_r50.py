"""Config-4 parity case (ResNet-50 / CIFAR-100, N = 512): EL2N error vs the CPU oracle with
and without the near-threshold fp32 re-scoring, and which rows the re-scoring touched."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from data_diet_distributed_amd import checkpoints, synthetic  # noqa: E402
from data_diet_distributed_amd.scoring import ScoreConfig, ScoringEngine  # noqa: E402
from oracle import pipeline as o_pipe  # noqa: E402

dev = torch.device("cuda:0")
n = 512
images, labels = synthetic.make_images(n, 100, seed=41)
sd = synthetic.make_checkpoint("resnet50", 100, seed=5)["net"]
ref = o_pipe.el2n_scores(sd, images, labels, batch_size=128).astype(np.float64)
img, lab = torch.from_numpy(images).to(dev), torch.from_numpy(labels).to(dev)
rep = {}
for name, kw in (("split", {"refine": False}), ("refined", {}),
                 ("fp32", {"fast_convs": False, "fast_el2n": False, "refine": False})):
    eng = ScoringEngine(checkpoints.build_models([sd], "resnet50", 100, device=dev),
                        ScoreConfig(methods=("el2n",), **kw), dev)
    full, kept, k = eng.run(img, lab, 0.5)
    got = full["el2n"].cpu().numpy().astype(np.float64)
    err = np.abs(got / ref - 1)
    w = np.argsort(err)[::-1][:5]
    rep[name] = {"max_rel": float(err.max()), "worst_rows": w.tolist(),
                 "worst_errs": err[w].tolist(), "worst_scores": ref[w].tolist(),
                 "refine": eng.last_refine}
    print(name, json.dumps(rep[name]))
out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/diag_refine_r50.json"
with open(out, "w") as f:
    json.dump(rep, f, indent=1)
