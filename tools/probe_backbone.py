"""GPU probe: MIOpen fp32 ResNet-18 throughput for the scoring passes (not product code)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from data_diet_distributed_amd.resnet import ResNet18

torch.backends.cudnn.benchmark = True
dev = "cuda:0"
m = ResNet18().to(dev)
for p in m.parameters():
    p.requires_grad_(False)


def timeit(fn, n=20, w=5):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


for cl in (False, True):
    mm = m.to(memory_format=torch.channels_last) if cl else m
    for B in (128, 512, 1024):
        x = torch.randn(B, 3, 32, 32, device=dev)
        if cl:
            x = x.to(memory_format=torch.channels_last)
        with torch.inference_mode():
            t = timeit(lambda: mm.run(x, bn="batch"))
        print(f"cl={cl} B={B} fwd-batchBN {t*1e3:.2f} ms  {B/t:.0f} ex/s  {1.111e9*B/t/1e12:.1f} TF", flush=True)
        with torch.inference_mode():
            t = timeit(lambda: mm.run(x, bn="running"))
        print(f"cl={cl} B={B} fwd-evalBN {t*1e3:.2f} ms  {B/t:.0f} ex/s", flush=True)

        def fb():
            xx = x.detach().requires_grad_(True)
            tape = []
            y = mm.run(xx, bn="running", tape=tape)
            outs = [t[2] for t in tape]
            torch.autograd.grad(y, outs, grad_outputs=torch.ones_like(y))
        t = timeit(fb, n=10, w=3)
        print(f"cl={cl} B={B} fwd+bwd(act) {t*1e3:.2f} ms  {B/t:.0f} ex/s", flush=True)

# bf16 reference point
mb = ResNet18().to(dev).to(torch.bfloat16)
x = torch.randn(1024, 3, 32, 32, device=dev, dtype=torch.bfloat16)
with torch.inference_mode():
    t = timeit(lambda: mb.run(x, bn="batch"))
print(f"bf16 B=1024 fwd {t*1e3:.2f} ms {1024/t:.0f} ex/s", flush=True)
