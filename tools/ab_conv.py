"""In-process A/B of two libdd.so builds (tools/ab_build.sh) on the backbone conv shapes:
interleaved rounds, median and min per variant (cdna_hip_programming.md §5.4 rule 24).

    python tools/ab_conv.py [--rounds 7] [--iters 20] [--batch 512] [--kernel conv|down|bwd]"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from data_diet_distributed_amd import _capi  # noqa: E402


def load(path):
    L = ctypes.CDLL(path)
    P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    L.has_masks = hasattr(L, "dd_conv3x3_mask_bytes")
    L.dd_abi_version.restype = I32
    # ABI 7 added the operand halves (DD_OPERANDS_*) and the accumulator scale(s) before the
    # stream of the forward convs
    F32 = ctypes.c_float
    L.abi7 = L.dd_abi_version() >= 7
    L.ops = (lambda *pks: [_capi.pack_operands(pks[0])] + [_capi.pack_acc_scale(p) for p in pks]
             ) if L.abi7 else (lambda *pks: [])
    o7 = [I32, F32] if L.abi7 else []
    L.dd_conv3x3_forward.argtypes = [P, I64, I32, I32, I32, P, I32, P, P, P, I32, P, P, I32,
                                     I32, I64, P] + ([P, P] if L.has_masks else []) + [P] + o7 + [P]
    L.dd_conv3x3_forward.restype = I32
    L.dd_down_forward.argtypes = [P, I64, I32, I32, I32, P, P, I32, P, I32, P, P, P, I32, P, P,
                                  I32, I64] + o7 + ([F32] if L.abi7 else []) + [P]
    L.dd_down_forward.restype = I32
    L.dd_down_backward.argtypes = [P, P, I64, I32, I32, I32, P, P, I32, P] + \
        ([P] if L.dd_abi_version() >= 4 else []) + [P, P]
    L.dd_down_backward.restype = I32
    L.dd_conv_pegrad_sqnorm.argtypes = [P, P, P, P, I32, I32, P, P, ctypes.c_size_t, P]
    L.dd_conv_pegrad_sqnorm.restype = I32
    L.dd_conv_pegrad_workspace_bytes.argtypes = [P, I32, I32]
    L.dd_conv_pegrad_workspace_bytes.restype = ctypes.c_size_t
    if hasattr(L, "dd_conv1x1_forward"):
        L.dd_conv1x1_forward.argtypes = [P, I64, I32, I32, I32, I32, P, I32, P, P, P, P, I32,
                                         P, P, I32, I32, I64, P, P] + o7 + [P]
        L.dd_conv1x1_forward.restype = I32
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--kernel", default="conv")
    ap.add_argument("--epi", default="none", help="none | fwd (bias+relu+residual) | "
                    "fwdmask (fwd + mask_out in B) | bwd (residual + fp32 mask)")
    ap.add_argument("--lib-a", default="build/ab/libA.so")
    ap.add_argument("--lib-b", default="build/ab/libB.so")
    ap.add_argument("--operands", default="bf16x3", help="bf16x3 | f16x3 (ABI 7 builds)")
    a = ap.parse_args()
    ops = a.operands
    libs = {"A": load(os.path.join(ROOT, a.lib_a)), "B": load(os.path.join(ROOT, a.lib_b))}
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device=dev).manual_seed(0)
    B = a.batch
    cases = []
    keep = []
    if a.kernel == "conv":
        for cin, cout, H in ((3, 64, 32), (64, 64, 32), (128, 128, 16), (256, 256, 8),
                             (512, 512, 4)):
            x = torch.randn(B, cin, H, H, device=dev, generator=g)
            w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) / (3 * cin ** 0.5)
            pk = _capi.conv3x3_pack(w, operands=ops)
            y = torch.empty(B, cout, H, H, device=dev)
            fl = 2.0 * B * H * H * cin * cout * 9
            bias = torch.randn(cout, device=dev, generator=g)
            rsd = torch.randn(B, cout, H, H, device=dev, generator=g)
            keep.append((bias, rsd))  # the closures hold raw pointers: keep the tensors alive
            mk = torch.empty(_capi.conv3x3_mask_bytes(B, cout, H, H), dtype=torch.uint8,
                             device=dev)
            e = a.epi
            bp = bias.data_ptr() if e.startswith("fwd") else None
            rp = rsd.data_ptr() if e not in ("none", "stats") else None
            mp = rsd.data_ptr() if e == "bwd" else None
            relu = 1 if e.startswith("fwd") else 0
            # --epi stats: the EL2N forward (producer's grouped BN + ReLU staged, BN partial
            # statistics out), groups of 128; the partial buffer is sized for the finest
            # layout either build may write (one partial per 32 positions)
            gs = 128 if e == "stats" else 0
            G = (B + 127) // 128
            aff = torch.rand(2, G, cin, device=dev, generator=g) + 0.5
            sbuf = torch.zeros(G * cout * (128 * H * H // 32) * 2, device=dev)
            keep.append((aff, sbuf))
            sc_p = aff[0].data_ptr() if gs else None
            sh_p = aff[1].data_ptr() if gs else None
            sb_p = sbuf.data_ptr() if gs else None

            def run(L, x=x, pk=pk, y=y, cin=cin, cout=cout, H=H, bp=bp, rp=rp, mp=mp,
                    relu=relu, mk=mk, gs=gs, sc_p=sc_p, sh_p=sh_p, sb_p=sb_p):
                extra = [mk.data_ptr() if (e == "fwdmask" and L is libs["B"]) else None,
                         None] if L.has_masks else []
                rc = L.dd_conv3x3_forward(x.data_ptr(), B, cin, H, H, pk.data_ptr(), cout, bp,
                                          rp, mp, relu, sc_p, sh_p, 1, gs, B if gs else 0,
                                          sb_p, *extra, y.data_ptr(), *L.ops(pk), st)
                assert rc == 0
            cases.append((f"conv3x3 {cin}->{cout} {H}x{H}", fl, run, y))
    elif a.kernel == "c1x1":
        # the ResNet-50 1x1 shapes (B = --batch): --epi stats = grouped BN statistics
        for cin, cout, H, s_ in ((256, 64, 32, 1), (64, 256, 32, 1), (512, 128, 16, 1),
                                 (128, 512, 16, 1), (1024, 256, 8, 1), (2048, 512, 4, 1),
                                 (512, 2048, 4, 1), (256, 512, 32, 2)):
            x = torch.randn(B, cin, H, H, device=dev, generator=g)
            w = torch.randn(cout, cin, device=dev, generator=g) / cin ** 0.5
            pk = _capi.conv1x1_pack(w, operands=ops)
            Ho = H // s_
            y = torch.empty(B, cout, Ho, Ho, device=dev)
            fl = 2.0 * B * Ho * Ho * cin * cout
            gs = 128 if a.epi == "stats" else 0
            stb = None
            if gs:
                # sized for one partial per 32 positions: the finest layout either build
                # may write (the two builds' layouts can differ)
                tpg = gs * Ho * Ho // 32
                stb = torch.zeros((B + gs - 1) // gs * cout * tpg * 2, device=dev)
            keep.append(stb)

            # --epi fwd: bias + residual + ReLU (the GraNd forward of a Bottleneck conv3);
            # bwd: residual + ReLU-backward mask (the GraNd backward)
            bias = torch.randn(cout, device=dev, generator=g) if a.epi == "fwd" else None
            res = (torch.randn(B, cout, Ho, Ho, device=dev, generator=g)
                   if a.epi in ("fwd", "bwd") else None)
            msk = torch.randn(B, cout, Ho, Ho, device=dev, generator=g) if a.epi == "bwd" else None
            keep += [bias, res, msk]
            ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731

            def run(L, x=x, pk=pk, y=y, cin=cin, cout=cout, H=H, s_=s_, gs=gs, stb=stb,
                    bias=bias, res=res, msk=msk):
                rc = L.dd_conv1x1_forward(x.data_ptr(), B, cin, H, H, s_, pk.data_ptr(), cout,
                                          ptr(bias), ptr(res), None, ptr(msk),
                                          int(a.epi == "fwd"), None, None, 1, gs,
                                          B if gs else 0, stb.data_ptr() if stb is not None
                                          else None, y.data_ptr(), *L.ops(pk), st)
                assert rc == 0
            cases.append((f"c1x1 {cin}->{cout} {H}/{s_}", fl, run, y))
    elif a.kernel == "pegrad":
        # the GraNd per-example norms on the direct3x3 shapes (ResNet-18 layer1, layer2 and
        # the layer2 head), auto method, split-bf16
        for cin, H, cout, s_ in ((64, 32, 64, 1), (128, 16, 128, 1), (64, 32, 128, 2)):
            Ho = H // s_
            act = torch.relu(torch.randn(B, cin, H, H, device=dev, generator=g))
            gout = torch.randn(B, cout, Ho, Ho, device=dev, generator=g) * 1e-2
            geom = _capi.conv_geom(act, gout, (3, 3), s_, 1)
            # the two builds may tile differently: size the workspace for the larger plan
            nb = max(L_.dd_conv_pegrad_workspace_bytes(ctypes.byref(geom), _capi.DD_PEGRAD_AUTO,
                                                      _capi.PRECISIONS["bf16x3"])
                     for L_ in libs.values())
            ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
            sq = torch.zeros(B, device=dev)
            keep.append((act, gout, ws, geom))
            fl = 2.0 * B * Ho * Ho * 9 * cin * cout

            def run(L, act=act, gout=gout, geom=geom, ws=ws, sq=sq, nb=nb):
                sq.zero_()
                rc = L.dd_conv_pegrad_sqnorm(act.data_ptr(), gout.data_ptr(), ctypes.byref(geom),
                                             None, _capi.DD_PEGRAD_AUTO,
                                             _capi.PRECISIONS["bf16x3"], sq.data_ptr(),
                                             ws.data_ptr(), nb, st)
                assert rc == 0
            cases.append((f"pegrad {cin}->{cout} {H}/{s_}", fl, run, sq))
    elif a.kernel in ("down", "bwd"):
        for cin, cout, HI in ((64, 128, 32), (128, 256, 16), (256, 512, 8)):
            HO = HI // 2
            w3 = torch.randn(cout, cin, 3, 3, device=dev, generator=g) / (3 * cin ** 0.5)
            w1 = torch.randn(cout, cin, 1, 1, device=dev, generator=g) / cin ** 0.5
            fl = 2.0 * B * HO * HO * cin * cout * 10
            if a.kernel == "down":
                x = torch.randn(B, cin, HI, HI, device=dev, generator=g)
                p3 = _capi.conv3x3_pack(w3, operands=ops)
                p1 = _capi.conv1x1_pack(w1, operands=ops)
                y = torch.empty(B, cout, HO, HO, device=dev)
                ys = torch.empty_like(y)
                # --epi stats: grouped train-BN partial statistics of both outputs (the EL2N
                # forward); otherwise plain outputs
                st_m = st_s = None
                gs = 128 if a.epi == "stats" else 0
                if gs:
                    tpg = _capi.lib().dd_down_tiles_per_group(HO, HO, gs)
                    st_m = torch.zeros((B + gs - 1) // gs * cout * tpg * 2, device=dev)
                    st_s = torch.zeros_like(st_m)

                # --epi bias: bias + ReLU on the main output, bias on the shortcut (the GraNd
                # forward, folded eval BN)
                bm = bs = None
                if a.epi == "bias":
                    bm = torch.randn(cout, device=dev, generator=g)
                    bs = torch.randn(cout, device=dev, generator=g)
                    keep.append((bm, bs))

                def run(L, x=x, p3=p3, p1=p1, y=y, ys=ys, cin=cin, cout=cout, HO=HO,
                        st_m=st_m, st_s=st_s, gs=gs, bm=bm, bs=bs):
                    pm = st_m.data_ptr() if st_m is not None else None
                    ps = st_s.data_ptr() if st_s is not None else None
                    pbm = bm.data_ptr() if bm is not None else None
                    pbs = bs.data_ptr() if bs is not None else None
                    rc = L.dd_down_forward(x.data_ptr(), B, cin, HO, HO, p3.data_ptr(),
                                           p1.data_ptr(), cout, pbm, int(bm is not None), pm,
                                           y.data_ptr(), pbs, 0, ps, ys.data_ptr(), gs,
                                           B if gs else 0, *L.ops(p3, p1), st)
                    assert rc == 0
                cases.append((f"down {cin}->{cout} {HI}->{HO}", fl, run, y))
            else:
                p3t = _capi.conv3x3_pack(w3, transpose_flip=True)
                p1t = _capi.conv1x1_pack(w1, transpose=True)
                dh = torch.randn(B, cout, HO, HO, device=dev, generator=g)
                dz = torch.randn(B, cout, HO, HO, device=dev, generator=g)
                m = torch.randn(B, cin, HI, HI, device=dev, generator=g)
                dx = torch.empty_like(m)

                def run(L, dh=dh, dz=dz, p3t=p3t, p1t=p1t, m=m, dx=dx, cin=cin, cout=cout, HO=HO):
                    # ABI 4 added mask_bits after mask_src (None: the fp32 mask)
                    extra = [None] if L.dd_abi_version() >= 4 else []
                    rc = L.dd_down_backward(dh.data_ptr(), dz.data_ptr(), B, cout, HO, HO,
                                            p3t.data_ptr(), p1t.data_ptr(), cin, m.data_ptr(),
                                            *extra, dx.data_ptr(), st)
                    assert rc == 0
                cases.append((f"down_bwd {cout}->{cin} {HO}->{HI}", fl, run, dx))
    for name, fl, run, out in cases:
        res = {"A": [], "B": []}
        outs = {}
        for r in range(a.rounds):
            for v in ("A", "B") if r % 2 == 0 else ("B", "A"):
                L = libs[v]
                for _ in range(2):
                    run(L)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run(L)
                e1.record()
                torch.cuda.synchronize()
                res[v].append(e0.elapsed_time(e1) / a.iters * 1e3)
                outs[v] = out.clone()
        diff = (outs["A"] - outs["B"]).abs().max().item() / max(outs["A"].abs().max().item(), 1e-30)
        mA, mB = statistics.median(res["A"]), statistics.median(res["B"])
        print(f"{name:28s} A {mA:7.1f} us ({fl / mA / 1e6:5.1f} TF/s, min {min(res['A']):7.1f}) | "
              f"B {mB:7.1f} us ({fl / mB / 1e6:5.1f} TF/s, min {min(res['B']):7.1f}) | "
              f"B/A speed {mA / mB:5.3f} | max rel diff {diff:.1e}", flush=True)


if __name__ == "__main__":
    main()
