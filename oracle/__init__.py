"""ORACLE — CPU restatement of the reference's Data Diet scoring path.  TEST INFRASTRUCTURE.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import
anything under `oracle/`, and only as the checker / the timed CPU baseline — never as a
product code path.  The product (`data_diet_distributed_amd`) runs the HIP kernels through
`libdd.so` and fails loudly without it.

Contents (each function cites the reference file:line it restates; paths relative to the
reference repository TejasPote/data_diet_distributed):
  el2n.py      EL2N rows, keep-count, stable descending top-k    get_scores_and_prune.py:16-24
  pegrad.py    per-example Conv2d/Linear weight-gradient norms    (north star; no reference code)
  resnet_fn.py functional ResNet forward over a state_dict        models/resnet.py:7-97
  pipeline.py  the whole scoring path on CPU (EL2N train-BN over the pinned batch partition,
               GraNd eval-BN, K-checkpoint mean, keep-set)       get_scores_and_prune.py:8-34

Pinning: EL2N scores and keep-sets of this restatement are checked against golden vectors
produced by running the reference's own `sparse_loader` in the build container
(tests/golden/make_golden.py, fixtures tests/golden/*.npz; test tests/test_oracle_golden.py).
GraNd has no reference implementation: the hook/ghost restatement here is checked against
`torch.func` per-sample gradients (definition of GraNd), i.e. GraNd parity is pinned to the
definition, not to reference outputs.
"""
