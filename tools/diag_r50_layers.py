"""Which conv family carries the ResNet-50 split-bf16 EL2N error?  The config-4 parity case
(N = 512) scored with the hand-written grouped forward, then with one conv family at a time
moved to MIOpen fp32 (its packs removed): 1x1 (conv1x1 kernel), 3x3 stride 1 (conv3x3),
3x3 stride 2 (Bottleneck conv2 on the down kernel).  Max / row-14 relative error vs the oracle."""
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
for name in ("all_fast", "no_1x1", "no_3x3", "no_down3", "only_1x1"):
    models = checkpoints.build_models([sd], "resnet50", 100, device=dev)
    eng = ScoringEngine(models, ScoreConfig(methods=("el2n",), refine=False), dev)
    m = models[0]
    if name == "no_1x1":
        m._packs1 = {}
    if name in ("no_3x3", "only_1x1"):
        m._packs = {None: None}  # (non-empty: el2n_fast.applicable stays true)
        del m._gemm              # no implicit-GEMM fallback either: MIOpen fp32
    if name in ("no_down3", "only_1x1"):
        m._down3 = {}
        if hasattr(m, "_gemm"):
            del m._gemm
    got = eng.score_shard(img, lab, 0, n)["el2n"].cpu().numpy().astype(np.float64)
    err = np.abs(got / ref - 1)
    rep[name] = {"max_rel": float(err.max()), "row14": float(err[14]),
                 "p99": float(np.percentile(err, 99)), "median": float(np.median(err))}
    print(name, json.dumps(rep[name]), flush=True)
out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/diag_r50_layers.json"
with open(out, "w") as f:
    json.dump(rep, f, indent=1)
