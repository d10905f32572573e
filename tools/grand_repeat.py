"""Run-to-run determinism of the two GraNd paths on the inputs of tests/test_gpu_pipeline.py::
test_fused_grand_path_equals_autograd_tape_path: the fused schedule and the autograd tape
path, each repeated in one process (alternating), every score vector compared bitwise with
the path's first run.  DD_REPEAT_DET=1 sets torch.backends.cudnn.deterministic (MIOpen's
deterministic solvers) for the whole process.  python tools/grand_repeat.py [repeats]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from data_diet_distributed_amd import checkpoints, synthetic  # noqa: E402
from data_diet_distributed_amd.scoring import ScoreConfig, ScoringEngine  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    cuda = torch.device("cuda:0")
    if os.environ.get("DD_REPEAT_DET") == "1":
        torch.backends.cudnn.deterministic = True
        print("torch.backends.cudnn.deterministic = True", flush=True)
    images, labels = synthetic.make_images(100, 10, seed=31)
    sd = synthetic.make_checkpoint("resnet18", 10, seed=6)["net"]
    img, lab = torch.from_numpy(images).to(cuda), torch.from_numpy(labels).to(cuda)
    first, worst, nbad = {}, {True: 0.0, False: 0.0}, {True: 0, False: 0}
    for r in range(reps):
        for fused in (True, False):
            eng = ScoringEngine(checkpoints.build_models([sd], device=cuda),
                                ScoreConfig(methods=("grand",), select_by="grand", grand_batch=64,
                                            fused_grand=fused), cuda)
            s = eng.score_shard(img, lab, 0, 100)["grand"].cpu().numpy()
            del eng
            if not fused:
                print(f"rep {r} tape: example 10 {s[10]!r}, 69 {s[69]!r}", flush=True)
            if fused not in first:
                first[fused] = s
                continue
            d = np.abs(s / first[fused] - 1)
            if (s != first[fused]).any():
                nbad[fused] += 1
                i = int(d.argmax())
                print(f"rep {r} fused={fused}: {int((s != first[fused]).sum())} scores differ from "
                      f"run 0, worst example {i}: {s[i]!r} vs {first[fused][i]!r} ({d[i]:.2e})",
                      flush=True)
            worst[fused] = max(worst[fused], float(d.max()))
    rel = np.abs(first[True] / first[False] - 1)
    print(f"fused vs tape (run 0): max rel {rel.max():.2e} at example {int(rel.argmax())}")
    for fused in (True, False):
        print(f"fused={fused}: {nbad[fused]} of {reps - 1} repeats differ from run 0, "
              f"worst rel {worst[fused]:.2e}", flush=True)


if __name__ == "__main__":
    main()
