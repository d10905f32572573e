"""Where does GraNd's split-bf16 error come from?  For chosen rows of the bench-config GraNd
test (tests/test_gpu_pipeline.py::test_grand_at_bench_config_matches_float64_oracle), per
checkpoint and per layer: the squared norm from (a) the fused split-bf16 forward/backward with
the split-bf16 norm kernels (the engine), (b) the same activations / gradients with the fp32
norm kernels, (c) the fp32 path (MIOpen convs, autograd, fp32 norm kernels).  (a) vs (b)
isolates the norm kernels, (b) vs (c) the backbone's forward / backward convs.
Also: is the fp32 EL2N refinement path (MIOpen convs, grouped BN) bitwise reproducible?"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from data_diet_distributed_amd import _capi, checkpoints, grand_fast, synthetic  # noqa: E402
from data_diet_distributed_amd.scoring import MEAN, STD  # noqa: E402


def layer_norms(model, x, lab, fused, prec):
    G = x.shape[0]
    e = torch.empty((G, model.linear.out_features), device=x.device)
    if fused:
        pairs, feat = grand_fast.forward_backward(model, x, lab, e, None)
        work = [(m, inp, g, s) for (m, inp, g, s) in pairs]
    else:
        xin = x.detach().requires_grad_(True)
        tape = []
        with torch.enable_grad():
            logits = model.run(xin, bn="folded", tape=tape, fast=False)
            _capi.el2n(logits.detach().float().contiguous(), lab, e=e)
            convs = [t for t in tape if isinstance(t[0], torch.nn.Conv2d)]
            grads = torch.autograd.grad(logits, [t[2] for t in convs], grad_outputs=e)
        work = [(m, inp, g, s) for (m, inp, _, s), g in zip(convs, grads)]
        feat = tape[-1][1]
    out = {}
    names = {mod: name for name, mod in model.named_modules()}
    for (m, inp, g, s) in work:
        inp, g = inp.detach().contiguous(), g.contiguous()
        geom = _capi.conv_geom(inp, g, m.kernel_size, m.stride[0], m.padding[0])
        ws = torch.empty(max(1, _capi.conv_workspace_bytes(geom, "auto", prec)), dtype=torch.uint8,
                         device=x.device)
        sq = torch.zeros(G, device=x.device)
        _capi.conv_pegrad_sqnorm(inp, g, m.kernel_size, m.stride[0], m.padding[0], sq, ws,
                                 method="auto", col_scale=s, precision=prec)
        out[f"{names[m]} {tuple(inp.shape[1:])}->{g.shape[1]}"] = sq.double().cpu().numpy()
    sq = torch.zeros(G, device=x.device)
    _capi.linear_pegrad_sqnorm(feat.detach().contiguous(), e, sq, has_bias=True)
    out["linear"] = sq.double().cpu().numpy()
    return out


def main():
    dev = torch.device("cuda:0")
    n = 3 * 1024 - 40
    images, labels = synthetic.make_images(n, 10, seed=51)
    sds = [synthetic.make_checkpoint("resnet18", 10, seed=s)["net"] for s in (11, 12)]
    rows = np.array([1037, 701, 53, 2693, 1805, 1421, 5, 29])
    G = 64
    x = torch.zeros(G, 3, 32, 32, device=dev)
    _capi.normalize_u8(torch.from_numpy(images[rows]).to(dev), MEAN, STD, x[:rows.size])
    lab = torch.zeros(G, dtype=torch.int64, device=dev)
    lab[:rows.size] = torch.from_numpy(labels[rows]).to(dev)
    report = {}
    for ci, sd in enumerate(sds):
        model = checkpoints.build_models([sd], device=dev)[0]
        model.eval()
        for p in model.parameters():
            p.requires_grad_(False)
        model.fold_bn()
        model.prepare_fast_convs()
        a = layer_norms(model, x, lab, True, "bf16x3")
        b = layer_norms(model, x, lab, True, "fp32")
        c = layer_norms(model, x, lab, False, "fp32")
        for ri, r in enumerate(rows):
            tot = {k: float(np.sqrt(sum(v[ri] for v in d.values()))) for k, d in
                   (("split", a), ("split_act_fp32_norm", b), ("fp32", c))}
            lay = []
            for key in a:
                va, vb, vc = a[key][ri], b[key][ri], c[key][ri]
                lay.append({"layer": key, "share": vc / max(tot["fp32"] ** 2, 1e-300),
                            "norm_kernel_rel": (va - vb) / max(vc, 1e-300),
                            "backbone_rel": (vb - vc) / max(vc, 1e-300)})
            lay.sort(key=lambda d: -abs(d["norm_kernel_rel"] * d["share"]) - abs(d["backbone_rel"] * d["share"]))
            report[f"ckpt{ci}_row{r}"] = {"totals": tot,
                                          "rel_split_vs_fp32": tot["split"] / tot["fp32"] - 1,
                                          "rel_splitact_vs_fp32": tot["split_act_fp32_norm"] / tot["fp32"] - 1,
                                          "top_layers": lay[:5]}
    # determinism of the fp32 refinement path
    model = checkpoints.build_models([sds[0]], device=dev)[0]
    xs = torch.zeros(512, 3, 32, 32, device=dev)
    _capi.normalize_u8(torch.from_numpy(images[:512]).to(dev), MEAN, STD, xs)
    outs = []
    with torch.inference_mode():
        for rep in range(3):
            outs.append(model.run(xs, bn="groups", group=128, fast=False).clone())
        torch.backends.cudnn.deterministic = True
        for rep in range(2):
            outs.append(model.run(xs, bn="groups", group=128, fast=False).clone())
        one = model.run(xs[:128].contiguous(), bn="groups", group=128, fast=False).clone()
    report["refine_determinism"] = {
        "rep_equal": [bool(torch.equal(outs[0], o)) for o in outs[1:]],
        "max_rel_rep": [float(((outs[0] - o).abs().max() / outs[0].abs().max()).item()) for o in outs[1:]],
        "group1_vs_group4_equal": bool(torch.equal(one, outs[0][:128])),
        "group1_vs_group4_rel": float(((one - outs[0][:128]).abs().max() / one.abs().max()).item())}
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/diag_grand_rows.json"
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(report, f, indent=1)
    for k, v in report.items():
        if k.startswith("ckpt"):
            print(k, "split", f"{v['rel_split_vs_fp32']:.2e}", "split-act/fp32-norm",
                  f"{v['rel_splitact_vs_fp32']:.2e}", "top:", v["top_layers"][0]["layer"],
                  f"share {v['top_layers'][0]['share']:.3f} normk {v['top_layers'][0]['norm_kernel_rel']:.2e} "
                  f"bb {v['top_layers'][0]['backbone_rel']:.2e}")
    print(json.dumps(report["refine_determinism"]))


if __name__ == "__main__":
    main()
