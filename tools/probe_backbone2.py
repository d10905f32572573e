"""GPU probe: MIOpen startup + throughput with cudnn.benchmark off (not product code)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from data_diet_distributed_amd.resnet import ResNet18
torch.backends.cudnn.benchmark = False
dev = "cuda:0"
t0 = time.time()
m = ResNet18().to(dev)
for p in m.parameters():
    p.requires_grad_(False)
def timeit(fn, n=20, w=3):
    for _ in range(w): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / n
for B in (128, 512):
    x = torch.randn(B, 3, 32, 32, device=dev)
    ts = time.time()
    with torch.inference_mode():
        t = timeit(lambda: m.run(x, bn="batch"))
    print(f"B={B} fwd-batchBN {t*1e3:.2f} ms {B/t:.0f} ex/s (first-use {time.time()-ts:.1f}s)", flush=True)
    def fb():
        xx = x.detach().requires_grad_(True); tape = []
        y = m.run(xx, bn="running", tape=tape)
        torch.autograd.grad(y, [t[2] for t in tape], grad_outputs=torch.ones_like(y))
    ts = time.time()
    t = timeit(fb, n=10)
    print(f"B={B} fwd+bwd {t*1e3:.2f} ms {B/t:.0f} ex/s (first-use {time.time()-ts:.1f}s)", flush=True)
print("total", time.time() - t0)
