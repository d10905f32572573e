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
    # name, N, ckpt seeds, data seed, sparsities, classifier ("init": the random-init Linear
    # of synthetic.make_checkpoint; "probe": a Linear fitted to the set, see fit_probe)
    ("r18_c10_n1024", 1024, [0], 0, [0.0, 0.5, 0.9], "init"),
    ("r18_c10_n2000_ragged", 2000, [1], 3, [0.0, 0.5, 0.7, 0.8], "init"),
    ("r18_c10_n640_k3", 640, [0, 1, 2], 5, [0.0, 0.5], "init"),
    # the headline config's size (BASELINE config 1/2: N = 50 000, one checkpoint) at the
    # sparsities whose keep counts matter (0.9 -> 4999 by float truncation)
    ("r18_c10_n50000", 50000, [0], 0, [0.5, 0.7, 0.9], "init"),
    # a K = 10 ensemble (north star: K = 10 seed checkpoints) at N = 4096
    ("r18_c10_n4096_k10", 4096, list(range(10)), 7, [0.5], "init"),
    # the trained-checkpoint regime the reference's callers score (a ckpt_19 after training,
    # reference train.py:61-64): same backbone and set as r18_c10_n50000, classifier fitted
    # to the set, so most examples are confidently right and the thresholds sit among small,
    # softmax-saturated EL2N scores
    ("r18_c10_n50000_trained", 50000, [0], 0, [0.3, 0.5, 0.7, 0.9], "probe"),
]
# L2 strength of the fitted classifier (per example, on the raw pooled features); chosen so
# the fitted set's median EL2N is a few 1e-2, the regime of a trained CIFAR-10 ResNet
PROBE_L2 = 3e-4
BATCH = 128


def main():
    torchvision_standin.install()
    sys.path.insert(0, REF)
    import get_scores_and_prune as ref_gsp  # reference module, unmodified
    import models.resnet as ref_resnet
    from data.loader import MyDataset

    torch.set_num_threads(8)
    only = set(sys.argv[1:])  # optional: names of the cases to (re)generate
    for name, n, seeds, dseed, sparsities, classifier in CASES:
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
            if classifier == "probe":
                feats = probe_features(ref_resnet, MyDataset, ck["net"], n)
                w, b = fit_probe(feats, labels, PROBE_L2)
                ck["net"]["linear.weight"] = torch.from_numpy(w)
                ck["net"]["linear.bias"] = torch.from_numpy(b)
                out[f"ckpt{s}_linear_weight"], out[f"ckpt{s}_linear_bias"] = w, b
                out["probe_l2"] = PROBE_L2
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


def probe_features(ref_resnet, MyDataset, state, n):
    """The reference network's pooled features (the input of `linear`, reference
    models/resnet.py:93-96) on the parity partition: train-mode BN over the unshuffled
    128-example batches, exactly what the scoring pass will feed the classifier."""
    net = ref_resnet.ResNet18()
    net.load_state_dict(state)
    feats = []
    net.linear.register_forward_pre_hook(lambda m, i: feats.append(i[0].detach().clone()))
    ds = MyDataset(torchvision_standin.CIFAR10(train=True, transform=_ref_transform()))
    loader = torch.utils.data.DataLoader(ds, batch_size=BATCH, shuffle=False, num_workers=0)
    with torch.no_grad():
        for _, x, _ in loader:
            net(x)
    out = torch.cat(feats).numpy()
    assert out.shape[0] == n
    return out


def fit_probe(feats, labels, l2, iters=2000):
    """Multinomial logistic regression on the pooled features in float64 (L-BFGS, L2 penalty
    `l2` per example on the weights): the classifier of a network trained on this set.  The
    fit is deterministic (float64, fixed start), and the fitted float32 weights are stored in
    the fixture, so the GPU box rebuilds the exact checkpoint without refitting."""
    from scipy.optimize import minimize
    x = feats.astype(np.float64)
    n, d = x.shape
    c = int(labels.max()) + 1
    onehot = np.eye(c)[labels]

    def f(theta):
        w, b = theta[:c * d].reshape(c, d), theta[c * d:]
        z = x @ w.T + b
        z -= z.max(axis=1, keepdims=True)
        lse = np.log(np.exp(z).sum(axis=1))
        p = np.exp(z - lse[:, None])
        loss = (lse - (z * onehot).sum(axis=1)).mean() + 0.5 * l2 * (w * w).sum()
        g = (p - onehot) / n
        gw = g.T @ x + l2 * w
        return loss, np.concatenate([gw.ravel(), g.sum(axis=0)])

    r = minimize(f, np.zeros(c * d + c), jac=True, method="L-BFGS-B",
                 options={"maxiter": iters, "gtol": 1e-10})
    w = r.x[:c * d].reshape(c, d).astype(np.float32)
    b = r.x[c * d:].astype(np.float32)
    return w, b


def _ref_transform():
    # the reference's own transform object (data/loader.py:8-11) built on the stand-in
    from data.loader import transform
    return transform


if __name__ == "__main__":
    main()
