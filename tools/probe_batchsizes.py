"""GPU probe: MIOpen immediate-mode time per batch size (which sizes fall back to naive)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from data_diet_distributed_amd.resnet import ResNet18
torch.backends.cudnn.benchmark = False
dev = "cuda:0"
m = ResNet18().to(dev).eval()
for p in m.parameters():
    p.requires_grad_(False)
def timeit(fn, n=5, w=2):
    for _ in range(w): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / n
for B in (16, 32, 64, 80, 96, 128, 192, 256, 336, 384, 512, 640, 768, 1024):
    x = torch.randn(B, 3, 32, 32, device=dev)
    with torch.inference_mode():
        tf = timeit(lambda: m.run(x, bn="batch"))
    def fb():
        xx = x.detach().requires_grad_(True); tape = []
        y = m.run(xx, bn="running", tape=tape)
        torch.autograd.grad(y, [t[2] for t in tape], grad_outputs=torch.ones_like(y))
    tb = timeit(fb)
    print(f"B={B:5d} fwd-batchBN {tf*1e3:8.2f} ms {tf/B*1e6:7.1f} us/ex | fwd+bwd {tb*1e3:8.2f} ms {tb/B*1e6:7.1f} us/ex", flush=True)
