"""Generate the golden EL2N fixtures by running the REFERENCE's own scoring code.

Runs in the build container only (needs /root/reference; never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [case names...]

For each case it
  1. makes synthetic inputs with data_diet_distributed_amd.synthetic (NumPy PCG64: the GPU
     box regenerates the same bytes; digests are stored to prove it),
  2. builds the reference's own ResNet (reference models/resnet.py) and loads a synthetic
     `{'net': state_dict}` checkpoint (the format of reference train.py:61-63),
  3. calls the reference `sparse_loader` (get_scores_and_prune.py:8-34) unmodified, with an
     UNSHUFFLED loader over the reference's `MyDataset` (the parity protocol),
     train-mode BN (the reference never calls .eval()), batch 128,
  4. records the scores the reference computed (logits captured by a forward hook, then the
     reference's own expression :16-18) and the kept indices read from the Subset the
     reference returned (:27), for several sparsities.
torchvision is absent, so tests/golden/torchvision_standin.py provides the few pieces used.
"""
import os
import sys

os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import torchvision_standin  # noqa: E402
from data_diet_distributed_amd import synthetic  # noqa: E402

CASES = [
    # name, N, ckpt seeds, data seed, sparsities
    ("r18_c10_n1024", 1024, [0], 0, [0.0, 0.5, 0.9]),
    ("r18_c10_n2000_ragged", 2000, [1], 3, [0.0, 0.5, 0.7, 0.8]),
    ("r18_c10_n640_k3", 640, [0, 1, 2], 5, [0.0, 0.5]),
    # the headline config's size (BASELINE config 1/2: N = 50 000, one checkpoint) at the
    # sparsities whose keep counts matter (0.9 -> 4999 by float truncation)
    ("r18_c10_n50000", 50000, [0], 0, [0.5, 0.7, 0.9]),
    # a K = 10 ensemble (north star: K = 10 seed checkpoints) at N = 4096
    ("r18_c10_n4096_k10", 4096, list(range(10)), 7, [0.5]),
]
BATCH = 128


def main():
    torchvision_standin.install()
    sys.path.insert(0, REF)
    import get_scores_and_prune as ref_gsp  # reference module, unmodified
    import models.resnet as ref_resnet
    from data.loader import MyDataset

    torch.set_num_threads(8)
    only = set(sys.argv[1:])  # optional: names of the cases to (re)generate
    for name, n, seeds, dseed, sparsities in CASES:
        if only and name not in only:
            continue
        images, labels = synthetic.make_images(n, 10, seed=dseed)
        torchvision_standin.SOURCE["train"] = (images, labels)
        torchvision_standin.SOURCE["test"] = (images[:10], labels[:10])
        out = {"images_digest": synthetic.digest(images, labels), "n": n, "data_seed": dseed,
               "ckpt_seeds": np.array(seeds), "batch_size": BATCH}
        per_ckpt = []
        for s in seeds:
            ck = synthetic.make_checkpoint("resnet18", 10, seed=s)
            out[f"ckpt{s}_digest"] = synthetic.state_digest(ck["net"])
            runs = {}
            for sp in sparsities:
                torch.manual_seed(0)
                net = ref_resnet.ResNet18()
                net.load_state_dict(ck["net"])  # train mode, as in train.py:59-63
                captured = []
                net.register_forward_hook(lambda m, i, o: captured.append(o.detach().clone()))
                ds = MyDataset(torchvision_standin.CIFAR10(train=True,
                                                           transform=_ref_transform()))
                loader = torch.utils.data.DataLoader(ds, batch_size=BATCH, shuffle=False,
                                                     num_workers=0)
                sub_loader, samples = ref_gsp.sparse_loader(loader, n, net, "cpu", sp, BATCH, 0)
                kept = np.array(sub_loader.dataset.indices, dtype=np.int64)
                logits = torch.cat(captured)
                y = torch.from_numpy(labels)
                preds = torch.nn.functional.softmax(logits, dim=1)
                e = preds - torch.nn.functional.one_hot(y, num_classes=10)
                scores = e.norm(dim=1, p=2).numpy().astype(np.float32)
                runs[sp] = (scores, kept, samples)
            s0 = runs[sparsities[0]][0]
            for sp, (sc, kept, samples) in runs.items():
                assert np.array_equal(sc, s0), "scores must not depend on sparsity"
                out[f"ckpt{s}_kept_{sp}"] = kept
                out[f"ckpt{s}_samples_{sp}"] = samples
            out[f"ckpt{s}_scores"] = s0
            per_ckpt.append(s0)
        if len(seeds) > 1:
            # K-checkpoint mean of the reference's per-checkpoint scores (north star (c)):
            # running fp32 sum in checkpoint order, then / K
            acc = np.zeros(n, np.float32)
            for sc in per_ckpt:
                acc += sc
            out["ensemble_scores"] = (acc / np.float32(len(seeds))).astype(np.float32)
        path = os.path.join(HERE, f"el2n_{name}.npz")
        np.savez_compressed(path, **out)
        print("wrote", path, {k: getattr(v, "shape", v) for k, v in out.items() if "digest" not in k})


def _ref_transform():
    # the reference's own transform object (data/loader.py:8-11) built on the stand-in
    from data.loader import transform
    return transform


if __name__ == "__main__":
    main()
