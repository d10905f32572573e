"""Data Diet scoring engine: EL2N + GraNd over K checkpoints, sharded, globally selected.

Replaces the body of reference `sparse_loader` (get_scores_and_prune.py:8-34) with a
device-resident pipeline:

  per rank (one process per GPU), for its contiguous batch-aligned shard of the dataset
    for each of K checkpoints
      EL2N  : uint8 -> normalised fp32 (dd_normalize_u8) -> ResNet forward with batch-stat BN
              over the pinned partition [b*B, (b+1)*B) (MIOpen) -> dd_el2n accumulates into the
              ensemble buffer (no per-example host syncs; reference :19-20 did 2 per example)
      GraNd : eval-BN forward with a tape of Conv2d/Linear (input, output) -> dd_el2n emits the
              residual e = d(sum CE)/d(logits) -> autograd back to every conv output only
              (weights frozen: no weight-gradient GEMMs) -> dd_conv_pegrad_sqnorm per conv
              (direct or ghost on MFMA) + dd_linear_pegrad_sqnorm -> dd_sqrt_accumulate
    dd_ensemble_finalize (mean over K)
  RCCL all-gather of the fp32 score vectors (the one collective)
  dd_select_topk on the full vector -> keep indices (reference :22-24 order and tie rule)

Parity protocol: batch b = global indices [b*B, (b+1)*B), unshuffled, so
train-mode-BN EL2N scores are identical for any number of ranks.
"""
from __future__ import annotations

import dataclasses
import time
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch
import torch.distributed as dist

from . import _capi, el2n_fast, grand_fast
from .resnet import ResNet

MEAN = (0.4914, 0.4822, 0.4465)  # reference data/loader.py:10
STD = (0.2023, 0.1994, 0.2010)


@dataclasses.dataclass
class ScoreConfig:
    methods: Sequence[str] = ("el2n",)      # subset of {"el2n", "grand"}
    select_by: str = "el2n"                  # which ensemble score ranks the keep-set
    batch_size: int = 128                    # EL2N batch partition (config.yaml:7 batch_size)
    el2n_bn: str = "batch"                   # "batch" = reference semantics; "running" = eval
    grand_batch: int = 1024                  # GraNd chunk (eval BN: any size, same result)
    pegrad_method: str = "auto"              # auto | direct | ghost
    pegrad_precision: str = "bf16x3"         # fp32 (exact MFMA) | bf16x3 (split-bf16 MFMA)
    # GraNd parameter set: conv_linear = every Conv2d + Linear weight (north
    # star); all = also every BatchNorm gamma / beta (the per-sample-gradient definition)
    grand_params: str = "conv_linear"
    fold_bn: bool = True                     # GraNd forward with eval BN folded into convs
    fast_convs: bool = True                  # 3x3 stride-1 convs on the split-bf16 kernel
    fused_grand: bool = True                 # hand-scheduled fwd/bwd for BasicBlock ResNets
    fast_el2n: bool = True                   # hand-scheduled grouped train-BN EL2N forward
    # operand halves of the EL2N forward's split MFMA convs (include/dd_capi.h DD_OPERANDS_*):
    # "f16x3" (~2^-22 relative per product; its activations are batch-normalised) or "bf16x3"
    el2n_operands: str = "f16x3"
    # ... and of the GraNd forward's (BN folded into the weights; the backward and the
    # per-example norm products stay bf16x3: gradients span many octaves below fp16's range)
    grand_operands: str = "f16x3"
    el2n_chunk: int = 1024                   # examples per EL2N launch (whole BN groups)
    pad_ragged: bool = True                  # run ragged tails at the full batch/chunk size
    # chunk_plan(even=True): the round-4 launch plan (equal chunks, the tail padded to the
    # buffer size) instead of full chunks + a tail at its own size; for A/B runs
    even_chunks: bool = False
    # EL2N and GraNd passes on two HIP streams (they share only read-only inputs and weight
    # packs; same results: each pass accumulates into its own vector in order).  Measured
    # +0.4-0.6 % on config 2 (profiles/r02_s2/concurrent_passes.txt), within box noise, while
    # every per-kernel duration stretches under sharing: off by default
    concurrent_passes: bool = False
    # lanes > 1: the launch chunks of every pass are dealt round-robin to `lanes` HIP streams
    # and issued interleaved, so one chunk's kernels run beside another's (persistent-grid
    # tails, epilogues, the small BN / norm kernels leave the chip partly idle).  Every chunk
    # is computed exactly as on one stream and each example belongs to one lane, so scores are
    # bitwise those of lanes = 1.
    lanes: int = 1
    # Exact keep-set (reference get_scores_and_prune.py:18-24 ranks fp32 scores):
    # after the global select, the scores that lie within `refine_rel` (relative) of the
    # threshold are re-computed on the plain-fp32 path (EL2N: their whole pinned batches on
    # MIOpen convs with grouped fp32 BN; GraNd: those examples, eval BN, fp32 MFMA norms) for
    # all K checkpoints, and the keep-set is selected again.  The band then widens until the
    # expected number of examples left on the wrong side, from the split-vs-fp32 differences
    # seen on everything re-scored, is at most `refine_tol` (ScoringEngine._refine).
    # "auto" (default): refine where the ranking pass carries bf16-halves arithmetic (~2^-17 per
    # product: EL2N on bf16x3 operands, GraNd, whose backward is bf16x3), not where it is
    # fp32-grade (EL2N on f16x3 operands: its scores sit as close to the reference's as plain
    # fp32 on the GPU does -- 1.6e-5 vs MIOpen's 1.7e-5 at N = 50 000, 0 keep-set swaps
    # unrefined -- and the fp32 re-scoring's MIOpen first use costs a one-shot job ~9 s).
    # True / False force it.
    refine: Union[bool, str] = "auto"
    refine_rel: float = 1e-5
    refine_max_iter: int = 8
    refine_tol: float = 0.02                 # expected examples on the wrong side, at most
    # at most this fraction of the examples is re-scored: when the tolerance needs more (a
    # network whose split-bf16 error is wide relative to the score density near the threshold,
    # ResNet-50 at CIFAR-100 / ImageNet shape), the refinement stops at its first estimate and
    # last_refine reports the expected number of wrong sides it leaves
    refine_max_frac: float = 0.08
    refine_min_sample: int = 512             # rows in the first re-scored sample, at least
    refine_groups: int = 8                   # pinned batches per fp32 EL2N launch

    def __post_init__(self):
        self.methods = tuple(self.methods)
        for m in self.methods:
            if m not in ("el2n", "grand"):
                raise ValueError(f"unknown score method {m!r}")
        if self.select_by not in self.methods:
            raise ValueError(f"select_by={self.select_by!r} not among methods {self.methods}")
        if self.el2n_bn not in ("batch", "running"):
            raise ValueError("el2n_bn must be 'batch' or 'running'")
        if self.pegrad_method not in _capi.METHODS:
            raise ValueError(f"pegrad_method must be one of {sorted(_capi.METHODS)}")
        if self.grand_params not in ("conv_linear", "all"):
            raise ValueError("grand_params must be 'conv_linear' or 'all'")
        for name in ("el2n_operands", "grand_operands"):
            if getattr(self, name) not in _capi.OPERANDS:
                raise ValueError(f"{name} must be one of {sorted(_capi.OPERANDS)}")
        if self.pegrad_precision not in _capi.PRECISIONS:
            raise ValueError(f"pegrad_precision must be one of {sorted(_capi.PRECISIONS)}")
        if self.lanes < 1:
            raise ValueError("lanes must be >= 1")
        if self.batch_size <= 0 or self.grand_batch <= 0:
            raise ValueError("batch sizes must be positive")
        self.refine = normalize_refine(self.refine)
        if (self.refine_rel < 0 or self.refine_tol <= 0 or self.refine_groups < 1
                or not 0 < self.refine_max_frac <= 1):
            raise ValueError("refine_rel >= 0, refine_tol > 0, refine_groups >= 1")
        if self.el2n_chunk < self.batch_size:
            self.el2n_chunk = self.batch_size
        self.el2n_chunk -= self.el2n_chunk % self.batch_size


def normalize_refine(v) -> Union[bool, str]:
    """ScoreConfig.refine / sparse_loader(refine=) as True, False or "auto".  0 / 1 (an int
    from a CLI or environment override) map to False / True; anything else is rejected (the
    checks use identity, so an int left as it is would read differently in different places:
    ADVICE r05)."""
    if isinstance(v, str):
        if v == "auto":
            return v
    elif isinstance(v, (bool, int, np.integer)) and v in (0, 1):
        return bool(v)
    raise ValueError(f"refine must be True, False or 'auto' (got {v!r})")


def shard_bounds(n: int, batch_size: int, world: int, rank: int):
    """Contiguous, batch-aligned shard [lo, hi) of rank `rank`:
    rank r gets batches floor(r*nb/W) .. floor((r+1)*nb/W)-1 of nb = ceil(n/B)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    nb = -(-n // batch_size)
    b_lo = (rank * nb) // world
    b_hi = ((rank + 1) * nb) // world
    return min(n, b_lo * batch_size), min(n, b_hi * batch_size)


def all_shards(n: int, batch_size: int, world: int):
    return [shard_bounds(n, batch_size, world, r) for r in range(world)]


def gather_scores(local: torch.Tensor, n: int, batch_size: int, group=None) -> torch.Tensor:
    """All-gather per-rank score shards into the full [n] vector (every rank gets it).

    One collective: each rank contributes its shard padded to the longest shard; indices are
    implicit in the shard bounds.  On GPU with the "nccl" backend this is RCCL over xGMI."""
    if not dist.is_available() or not dist.is_initialized():
        if local.numel() != n:
            raise ValueError("single-process gather needs the whole score vector")
        return local
    world = dist.get_world_size(group)
    bounds = all_shards(n, batch_size, world)
    L = max(hi - lo for lo, hi in bounds)
    buf = torch.zeros(L, dtype=local.dtype, device=local.device)
    buf[:local.numel()] = local
    if dist.get_backend(group) == "gloo":
        # gloo (CPU tests; ranks sharing one GPU, where RCCL refuses a second communicator on
        # the device): device shards are staged through host memory
        host = buf.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        flat = torch.cat(parts).to(local.device)
    else:
        flat = torch.empty(world * L, dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(flat, buf, group=group)
    return torch.cat([flat[r * L: r * L + (hi - lo)] for r, (lo, hi) in enumerate(bounds)])


def _all_gather_same(t: torch.Tensor, group=None):
    """All-gather a same-shape tensor from every rank -> list in rank order (gloo: staged
    through host memory, as gather_scores)."""
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo":
        host = t.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host, group=group)
        return [p.to(t.device) for p in parts]
    flat = torch.empty((world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(flat, t.contiguous(), group=group)
    return list(flat.unbind(0))


def _all_reduce_sum(t: torch.Tensor, group=None):
    """In-place sum over ranks (gloo: staged through host memory)."""
    if dist.get_backend(group) == "gloo":
        host = t.cpu()
        dist.all_reduce(host, group=group)
        t.copy_(host)
    else:
        dist.all_reduce(t, group=group)


def chunk_plan(lo: int, hi: int, granule: int, chunk: int, even: bool = False):
    """Launch chunks [(c0, c1)] covering [lo, hi) in whole `granule`-row batches, and the
    buffer size.  Default: full `chunk`-row launches and one shorter tail, which runs at its
    own size rounded up to whole granules (run_rows), so a shard's launches are as full as the
    whole set's (a 195-batch W = 2 shard: 24 x 1024 rows + one of 384).

    even=True (the round-4 plan, kept for A/B runs): chunks as equal as possible, the tail run
    padded to the buffer size, the chunk count chosen (up to 4 above the minimum) to minimise
    that padding (the same shard: 28 x 896 rows)."""
    n = hi - lo
    if n <= 0:
        return [], 0
    granule = max(1, min(granule, chunk))
    if not even:
        rows = max(granule, chunk // granule * granule)
        rows = min(rows, run_rows(n, granule))
        return [(c0, min(hi, c0 + rows)) for c0 in range(lo, hi, rows)], rows
    nb = -(-n // granule)
    per_max = max(1, chunk // granule)
    nch0 = -(-nb // per_max)
    # among a few more chunks than the minimum, take the count whose padded work
    # nch * ceil(nb / nch) batches is least (a 98-batch shard: 14 chunks of 7 batches instead
    # of 13 of 8, 6 % less work)
    best = None
    for nch in range(nch0, min(nb, nch0 + 4) + 1):
        per = -(-nb // nch)
        cost = (-(-nb // per)) * per  # chunks actually produced x batches each
        if best is None or cost < best[0]:
            best = (cost, per)
    rows = best[1] * granule
    return [(c0, min(hi, c0 + rows)) for c0 in range(lo, hi, rows)], rows


def run_rows(n: int, granule: int) -> int:
    """Rows a launch of n valid rows runs at: whole granules (pinned BN batches)."""
    return -(-n // granule) * granule


def _world(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def world_of(group=None) -> int:
    return _world(group)[0]


def sharded_job(score_shard, n: int, batch_size: int, sparsity: float, select_by: str, select,
                keep_count, group=None, validate=None):
    """The whole job of one rank: score this rank's batch-aligned shard
    (`score_shard(lo, hi) -> {method: fp32 [hi - lo]}`), all-gather every score vector (the
    one collective), then the same deterministic global selection on every rank
    (`select(keys, k) -> kept indices`, `keep_count(n, sparsity)` = reference :22).
    `validate(full) -> full` runs on the gathered vectors before the selection: every rank
    holds the same vectors there, so a check that raises (or repairs) does so on all ranks
    together and none is left waiting in a collective.  Returns (full score dict, kept, k)."""
    world, rank = _world(group)
    lo, hi = shard_bounds(n, batch_size, world, rank)
    local = score_shard(lo, hi)
    full = {m: gather_scores(v, n, batch_size, group) for m, v in local.items()}
    if validate is not None:
        full = validate(full)
    k = keep_count(n, sparsity)
    if k < 0 or k > n:
        raise ValueError(f"sparsity {sparsity} gives keep count {k} outside [0, {n}]")
    return full, select(full[select_by], k), k


def check_bn_gammas(model: ResNet):
    """grand_params='all' recovers each BN's normalised input from its output,
    xhat = (v - beta) / gamma (dd_bn_pegrad_sqnorm: the folded forward never forms xhat), so
    a zero gamma has no per-example d/dgamma from this formulation: refuse it by name instead
    of returning NaN scores.  (Near-zero gammas stay accepted; their d/dgamma carries the
    rounding of v - beta divided by gamma.)"""
    for name, mod in model.named_modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            zero = (mod.weight.detach() == 0).nonzero().flatten()
            if zero.numel():
                raise ValueError(
                    f"grand_params='all': {name}.weight is exactly 0 in channel(s) "
                    f"{zero[:8].tolist()}; per-example BN-affine gradients are recovered from "
                    f"the BN output and need a non-zero gamma (use grand_params='conv_linear')")


def refine_keep_set(orig: torch.Tensor, k: int, unit: int, rescore, cfg: ScoreConfig,
                    check_nan: bool = True):
    """The exact keep-set from fast-path scores `orig` [N] (ScoreConfig.refine): re-score near
    the threshold on the fp32 path until the keep-set is settled.  Reference
    get_scores_and_prune.py:18-24 ranks exact fp32 scores; the split-bf16 fast path is ~1e-5
    relative off them, enough to swap a few examples at the threshold.

    Positions [u*unit, (u+1)*unit) form one re-scoring unit (EL2N: a pinned / visit batch,
    whose train-mode BN couples its rows; GraNd: unit 1); `rescore(rows)` returns the fp32
    scores of the position ranges `rows` (ascending, whole units), concatenated.

    The first round re-scores every unit with a score within `refine_rel` of the threshold (or
    the units of the `refine_min_sample` nearest rows where that band holds more).  Everything
    re-scored so far is a sample of the fast path's error e = |split - fp32| / |threshold|;
    an example left on the fast path at distance d from the threshold can be on the wrong side
    only if its error exceeds d, so the expected number of wrong sides is sum_j P(e > d_j) over
    the examples not re-scored, with P from the sample.  While that exceeds `refine_tol`, the
    band grows to the smallest one that brings it under, and those units are re-scored, within
    `refine_max_iter` rounds and `refine_max_frac` of N.  Returns (scores, keep-set, record)."""
    N = orig.numel()
    t0 = time.perf_counter()
    s = orig.clone()
    done = np.zeros(N, dtype=bool)
    band, rescored, its, expected, worst = cfg.refine_rel, 0, 0, None, 0.0
    capped, needed = False, None
    orig_h = orig.cpu().numpy().astype(np.float64)

    def estimate():
        """(distance of every score from the threshold / |threshold|, the examples still on
        the fast path, P(wrong side) for each of them, the largest error seen)"""
        _, thr, _ = _capi.select_topk(s, k, check_nan=False)
        s_h = s.cpu().numpy().astype(np.float64)
        t = max(abs(float(thr.item())), 1e-30)
        d = np.abs(s_h - float(thr.item())) / t
        if not done.any():
            return d, None, None, 0.0
        err = np.sort(np.abs(orig_h[done] - s_h[done]) / t)
        und = np.nonzero(~done)[0]
        # P(e > d_j) from the sample, per example still on the fast path
        p = 1.0 - np.searchsorted(err, d[und], side="right") / err.size
        return d, und, p, float(err[-1])

    stale = False  # re-scored since the last estimate
    for its in range(1, cfg.refine_max_iter + 1):
        d, und, p, worst = estimate()
        stale = False
        if und is not None:
            expected = float(p.sum())
            if expected <= cfg.refine_tol:
                break
            order = np.argsort(d[und], kind="stable")
            tail = np.cumsum(p[order][::-1])[::-1]  # tail[i] = sum of p over order[i:]
            i = int(np.argmax(tail <= cfg.refine_tol)) if (tail <= cfg.refine_tol).any() \
                else order.size
            band = max(band, float(d[und][order[i - 1]]) if i > 0 else band)
        else:
            # the first sample: the refine_min_sample rows of the nearest units (the start
            # band refine_rel only where it holds fewer: on a large set a fixed relative band
            # would already hold thousands of batches)
            m = min(N, -(-cfg.refine_min_sample // unit))
            band = min(band, float(np.partition(d, m - 1)[m - 1]))
        pos = np.nonzero((d <= band) & ~done)[0]
        units = np.unique(pos // unit)
        if units.size == 0:
            break
        usize = np.minimum(N, (units + 1) * unit) - units * unit
        budget = int(cfg.refine_max_frac * N) - rescored
        if rescored and int(usize.sum()) > budget:  # (the first sample always runs)
            # the tolerance needs more fp32 re-scoring than the budget allows (a network whose
            # split error is wide against the score density at the threshold): stop at the
            # estimate instead of spending the budget on a partial band, and say what the
            # band would have taken
            capped = True
            needed = rescored + int(usize.sum())
            break
        rows = [(u * unit, min(N, (u + 1) * unit)) for u in units.tolist()]
        new = rescore(rows)
        idx = torch.cat([torch.arange(r0, r1, device=s.device) for r0, r1 in rows])
        s = s.clone()
        s[idx] = new.to(s.device)
        for r0, r1 in rows:
            done[r0:r1] = True
        rescored += sum(r1 - r0 for r0, r1 in rows)
        stale = True
    if stale:
        # the loop ran out of refine_max_iter right after a re-scoring round: estimate what
        # that round left, so the record does not report the previous round's figure
        _, und, p, worst = estimate()
        expected = float(p.sum())
    kept = _capi.select_topk(s, k, check_nan=check_nan)[0]
    info = {"iterations": its, "band_rel": band, "max_rel_diff": worst,
            "expected_wrong_side": expected,
            "converged": expected is not None and expected <= cfg.refine_tol,
            "budget_capped": capped, "examples_rescored": rescored,
            "seconds": time.perf_counter() - t0}
    if capped:
        # examples the tolerance's band would re-score in all (whole units), and that as a
        # fraction of N: the refine_max_frac it would need
        info["rows_needed"] = needed
        info["max_frac_needed"] = needed / N
    return s, kept, info


class ScoringEngine:
    """Scores a device-resident uint8 dataset with K resident checkpoint models."""

    def __init__(self, models: List[ResNet], cfg: ScoreConfig, device):
        if not models:
            raise ValueError("need at least one checkpoint model")
        self.models = models
        self.cfg = cfg
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("the scoring engine runs on a GPU (libdd.so has no CPU path)")
        _capi.lib()  # fail loudly now if the HIP library is missing
        # per-checkpoint setup cost (bench.py reports it beside the steady-state step)
        self.setup_times = {"fold_s_per_ckpt": 0.0, "pack_s_per_ckpt": 0.0}
        for m in models:
            m.eval()  # BN mode is chosen per pass explicitly; eval() only stops dropout etc.
            for p in m.parameters():
                p.requires_grad_(False)
            t = time.perf_counter()
            if cfg.fold_bn:
                m.fold_bn()
            torch.cuda.synchronize(self.device)
            t1 = time.perf_counter()
            if cfg.fast_convs:
                m.prepare_fast_convs(cfg.el2n_operands, cfg.grand_operands)
            torch.cuda.synchronize(self.device)
            self.setup_times["fold_s_per_ckpt"] += (t1 - t) / len(models)
            self.setup_times["pack_s_per_ckpt"] += (time.perf_counter() - t1) / len(models)
        if cfg.grand_params == "all" and "grand" in cfg.methods:
            for m in models:
                check_bn_gammas(m)
        self._wss: Dict[int, torch.Tensor] = {}  # pegrad workspace per lane
        self.last_refine: Optional[dict] = None  # what the last run()'s _refine did
        # set when a GraNd forward on fp16 operand halves overflowed and the engine re-scored
        # on bf16 halves (run(); the engine keeps bf16 GraNd packs from then on)
        self.grand_fallback: Optional[str] = None
        self.fallback: Dict[str, str] = {}  # method -> why it was re-scored on bf16 halves
        self._bad = None  # dd_el2n's label counter of the current score_shard
        # optional heartbeat, called with a short message every `progress_every` launch chunks
        # (a long config-5 pass otherwise prints nothing for minutes)
        self.progress = None
        self.progress_every = 100
        self._side: Optional[torch.cuda.Stream] = None  # the concurrent pass stream
        self._lane_streams: List[torch.cuda.Stream] = []
        self._conv_meta = self._describe_convs(models[0])

    # ---- helpers ---------------------------------------------------------------------------
    @staticmethod
    def _describe_convs(model: ResNet):
        meta = {}
        for name, mod in model.named_modules():
            if isinstance(mod, torch.nn.Conv2d):
                if mod.groups != 1 or mod.bias is not None or mod.dilation != (1, 1):
                    raise ValueError(f"{name}: only dense, bias-free, undilated convs")
                if mod.stride[0] != mod.stride[1] or mod.padding[0] != mod.padding[1]:
                    raise ValueError(f"{name}: asymmetric stride/padding unsupported")
        return meta

    def _workspace(self, nbytes: int, lane: int = 0) -> torch.Tensor:
        ws = self._wss.get(lane)
        if ws is None or ws.numel() < nbytes:
            ws = self._wss[lane] = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8,
                                               device=self.device)
        return ws

    def _normalize(self, images_u8: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        return _capi.normalize_u8(images_u8, MEAN, STD, out)

    def _beat(self, what, ci, n):
        if self.progress is not None and ci % self.progress_every == self.progress_every - 1:
            self.progress(f"{what} chunk {ci + 1}/{n}")

    # ---- passes ----------------------------------------------------------------------------
    def el2n_pass(self, model: ResNet, images_u8, labels, lo, hi, accum):
        """accum[j] += EL2N(x_{lo+j}) for the shard, batch partition anchored at 0.

        A ragged final batch (N % B rows) is run padded to B rows with its BN statistics
        taken over the valid rows only (`n_valid`): identical scores, and MIOpen keeps the
        solvers it uses for full batches (at unusual batch sizes its immediate mode can fall
        back to naive kernels, SURVEY-era profile profiles/r01_v1)."""
        B = self.cfg.batch_size
        if (self.cfg.fast_el2n and self.cfg.fast_convs and self.cfg.el2n_bn == "batch"
                and el2n_fast.applicable(model)):
            return self._el2n_pass_grouped(model, images_u8, labels, lo, hi, accum)
        xbuf = torch.zeros((B,) + tuple(images_u8.shape[1:]), dtype=torch.float32,
                           device=self.device)
        with torch.inference_mode():
            for b0 in range(lo, hi, B):
                b1 = min(hi, b0 + B)
                n = b1 - b0
                pad = self.cfg.pad_ragged and n < B and self.cfg.el2n_bn == "batch"
                x = self._normalize(images_u8[b0:b1], xbuf[:n])
                if pad:
                    xbuf[n:].zero_()
                    x = xbuf
                logits = model.run(x, bn=self.cfg.el2n_bn, n_valid=n if pad else None,
                                   fast=self.cfg.fast_convs)
                logits = logits[:n].float().contiguous()
                _capi.el2n(logits, labels[b0:b1], accum=accum[b0 - lo:b1 - lo],
                           bad_labels=self._counter("el2n", model))

    def _el2n_pass_grouped(self, model: ResNet, images_u8, labels, lo, hi, accum):
        """el2n_pass on the hand-scheduled forward: `el2n_chunk` examples (whole pinned BN
        groups of batch_size) per launch; the tail chunk runs at full size, zero-padded, with
        its statistics over the valid rows only."""
        for _ in self._el2n_chunks(model, images_u8, labels, lo, hi, accum):
            pass

    def _el2n_chunks(self, model: ResNet, images_u8, labels, lo, hi, accum, lane=0, lanes=1):
        """The grouped EL2N pass as a generator: chunks lane, lane + lanes, ... of the plan,
        yielding after each (score_shard interleaves the lanes' chunks on their streams)."""
        B = self.cfg.batch_size
        even = self.cfg.even_chunks
        plan, CH = chunk_plan(lo, hi, B, self.cfg.el2n_chunk, even)
        if len(plan) <= lane:
            return
        # (a normal tensor, and inference mode per chunk: a context held across a yield would
        # leak into the other lanes' interleaved chunks)
        xbuf = torch.zeros((CH,) + tuple(images_u8.shape[1:]), dtype=torch.float32,
                           device=self.device)
        for ci in range(lane, len(plan), lanes):
            b0, b1 = plan[ci]
            self._beat("el2n", ci, len(plan))
            n = b1 - b0
            nr = CH if even else run_rows(n, B)  # whole pinned batches (a ragged one padded)
            with torch.inference_mode():
                xb = xbuf[:nr]
                if n < nr:
                    xb[n:].zero_()
                self._normalize(images_u8[b0:b1], xb[:n])
                logits = el2n_fast.forward_logits(model, xb, B, n)[:n]
                _capi.el2n(logits, labels[b0:b1], accum=accum[b0 - lo:b1 - lo],
                           bad_labels=self._counter("el2n", model))
            yield

    def grand_pass(self, model: ResNet, images_u8, labels, lo, hi, accum):
        for _ in self._grand_chunks(model, images_u8, labels, lo, hi, accum):
            pass

    def _grand_chunks(self, model: ResNet, images_u8, labels, lo, hi, accum, lane=0, lanes=1):
        """accum[j] += ||grad_W CE(x_{lo+j})|| (eval-mode BN, Conv2d + Linear weights).

        Chunks come from chunk_plan: whole `batch_size` granules, `grand_batch` rows each and
        a shorter tail run at its own size (whole granules; the padded rows discarded), so the
        launch sizes depend on the shard length.  Eval BN makes examples independent and every
        hand-written kernel of the fused schedule computes an example's norm from that
        example's rows alone, in a fixed order with no float atomics, so scores are bitwise
        independent of G and of the world size (tests/test_gpu_pipeline.py::
        test_grand_scores_independent_of_chunk_and_world).  The unfused autograd path runs
        convs on MIOpen, whose solver choice may vary with G (fp32 rounding only)."""
        gran = min(self.cfg.batch_size, self.cfg.grand_batch)
        even = self.cfg.even_chunks
        plan, G = chunk_plan(lo, hi, gran, self.cfg.grand_batch, even)
        if len(plan) <= lane:
            return
        bn = "folded" if self.cfg.fold_bn else "running"
        fused = (self.cfg.fused_grand and self.cfg.fold_bn and self.cfg.fast_convs
                 and grand_fast.applicable(model))
        shape = (G,) + tuple(images_u8.shape[1:])
        x = torch.zeros(shape, dtype=torch.float32, device=self.device)
        lab = torch.zeros(G, dtype=torch.int64, device=self.device)
        e = torch.empty((G, model.linear.out_features), dtype=torch.float32, device=self.device)
        sq = torch.empty(G, dtype=torch.float32, device=self.device)
        xfull, labfull, efull, sqfull = x, lab, e, sq
        for ci in range(lane, len(plan), lanes):
            b0, b1 = plan[ci]
            self._beat("grand", ci, len(plan))
            n = b1 - b0
            nr = G if even else run_rows(n, gran)  # rows this launch runs at
            x, lab, e, sq = xfull[:nr], labfull[:nr], efull[:nr], sqfull[:nr]
            if n < nr:
                x[n:].zero_()
                lab[n:].zero_()
            self._normalize(images_u8[b0:b1], x[:n])
            lab[:n].copy_(labels[b0:b1])
            bn_pairs = [] if self.cfg.grand_params == "all" else None
            if fused:
                pairs, feat = grand_fast.forward_backward(
                    model, x, lab, e, bn_pairs, bad_labels=self._counter("grand", model))
                work = [(m, inp, g, scale) for (m, inp, g, scale) in pairs]
                lin = model.linear
            elif bn_pairs is not None:
                raise NotImplementedError(
                    "grand_params='all' runs on the fused BasicBlock GraNd schedule "
                    "(ResNet-18/34 CIFAR); this model takes the autograd path")
            else:
                xin = x.detach().requires_grad_(True)
                tape = []
                with torch.enable_grad():
                    logits = model.run(xin, bn=bn, tape=tape, fast=self.cfg.fast_convs)
                    _capi.el2n(logits.detach().float().contiguous(), lab, e=e,
                               bad_labels=self._counter("grand", model))
                    convs = [t for t in tape if isinstance(t[0], torch.nn.Conv2d)]
                    grads = torch.autograd.grad(logits, [t[2] for t in convs], grad_outputs=e)
                work = [(m, inp, g, scale) for (m, inp, _, scale), g in zip(convs, grads)]
                lin, feat, _, _ = tape[-1]
                del tape, grads, convs, xin
            sq.zero_()
            for (m, inp, g, scale) in work:
                inp = inp.detach().contiguous()
                g = g.contiguous()
                geom = _capi.conv_geom(inp, g, m.kernel_size, m.stride[0], m.padding[0])
                prec = self.cfg.pegrad_precision
                ws = self._workspace(_capi.conv_workspace_bytes(geom, self.cfg.pegrad_method,
                                                                prec), lane)
                _capi.conv_pegrad_sqnorm(inp, g, m.kernel_size, m.stride[0], m.padding[0], sq, ws,
                                         method=self.cfg.pegrad_method, col_scale=scale,
                                         precision=prec)
            _capi.linear_pegrad_sqnorm(feat.detach().contiguous(), e, sq,
                                       has_bias=lin.bias is not None)
            for bnm, v, r, g in bn_pairs or ():
                _capi.bn_pegrad_sqnorm(v, g, bnm.weight, bnm.bias, sq, r=r)
            _capi.sqrt_accumulate(sq[:n], accum[b0 - lo:b1 - lo])
            del work, feat
            yield

    def _lanes_apply(self) -> bool:
        """Lanes interleave the chunk generators of the hand-scheduled passes."""
        c = self.cfg
        el2n_ok = "el2n" not in c.methods or (
            c.fast_el2n and c.fast_convs and c.el2n_bn == "batch"
            and all(el2n_fast.applicable(m) for m in self.models))
        return el2n_ok

    def score_shard(self, images_u8: torch.Tensor, labels: torch.Tensor, lo: int, hi: int,
                    check: bool = True) -> Dict[str, torch.Tensor]:
        """Ensemble-mean scores of examples [lo, hi) (device tensors [hi-lo]).

        check=True (a direct, single-rank call) raises here: LabelError for labels outside
        [0, C) (reference :17), ValueError for non-finite scores (a forward that left fp16's
        range).  run() passes check=False and checks the gathered vectors instead (_validate),
        so that on W > 1 ranks every rank raises (or falls back) together."""
        n = hi - lo
        K = len(self.models)
        self._bad = _capi.label_counter(self.device)
        # counted on the first pass over the shard only (the first method's first checkpoint
        # scores every row once), so the count is of rows, not of row-passes
        self._bad_pass = (self.cfg.methods[0], self.models[0])
        accs = {m: torch.zeros(n, dtype=torch.float32, device=self.device)
                for m in self.cfg.methods}

        def passes(method):
            for model in self.models:
                if method == "el2n":
                    self.el2n_pass(model, images_u8, labels, lo, hi, accs[method])
                else:
                    self.grand_pass(model, images_u8, labels, lo, hi, accs[method])

        lanes = self.cfg.lanes
        if lanes > 1 and self._lanes_apply():
            main = torch.cuda.current_stream(self.device)
            while len(self._lane_streams) < lanes:
                self._lane_streams.append(torch.cuda.Stream(self.device))
            streams = self._lane_streams[:lanes]
            for st in streams:
                st.wait_stream(main)  # inputs and accumulators are ready on the main stream
            for method in self.cfg.methods:
                gen = self._el2n_chunks if method == "el2n" else self._grand_chunks
                for model in self.models:
                    its = [gen(model, images_u8, labels, lo, hi, accs[method], lane=j,
                               lanes=lanes) for j in range(lanes)]
                    live = list(range(lanes))
                    while live:  # one chunk per lane in turn, each on its lane's stream
                        for j in list(live):
                            with torch.cuda.stream(streams[j]):
                                if next(its[j], StopIteration) is StopIteration:
                                    live.remove(j)
            for st in streams:
                for acc in accs.values():
                    acc.record_stream(st)
                main.wait_stream(st)
        elif self.cfg.concurrent_passes and len(self.cfg.methods) > 1:
            main = torch.cuda.current_stream(self.device)
            if self._side is None:
                self._side = torch.cuda.Stream(self.device)
            side = self._side
            side.wait_stream(main)  # inputs and accumulators are ready on the main stream
            with torch.cuda.stream(side):
                passes(self.cfg.methods[0])
            accs[self.cfg.methods[0]].record_stream(side)
            for m in self.cfg.methods[1:]:
                passes(m)
            main.wait_stream(side)
        else:
            for m in self.cfg.methods:
                passes(m)
        out = {}
        for method in self.cfg.methods:
            res = torch.empty_like(accs[method])
            _capi.ensemble_finalize(accs[method], K, res)
            out[method] = res
        if check and n:
            _capi.check_labels(self._bad, self.models[0].linear.out_features, "score_shard")
            fin = torch.stack([torch.isfinite(out[m]).all() for m in self.cfg.methods]).cpu()
            for m, ok in zip(self.cfg.methods, fin.tolist()):
                if not ok:
                    # e.g. an activation past fp16's range (65504) in a forward on fp16 operand
                    # halves: fail loudly rather than return non-finite scores (run() re-scores
                    # on bf16 halves by itself)
                    ops = "el2n_operands" if m == "el2n" else "grand_operands"
                    raise ValueError(f"non-finite {m} scores" + (
                        f": an activation of the forward may have left fp16's range; score "
                        f"with {ops}='bf16x3' (ScoreConfig), or through run(), which falls "
                        f"back to bf16 halves by itself" if self._f16_forward(m) else ""))
        return out

    def _counter(self, method: str, model) -> Optional[torch.Tensor]:
        """dd_el2n's label counter for the pass (method, model), or None (see score_shard)."""
        bp = getattr(self, "_bad_pass", None)
        return self._bad if bp is not None and bp[0] == method and bp[1] is model else None

    def _validate(self, full, score, N, B, group):
        """run()'s check of the gathered score vectors (sharded_job's `validate`), before the
        selection.  Every rank holds the same gathered vectors, so every rank takes the same
        branch (a raise on one rank only left the others blocked in the gather):
          all finite                      -> unchanged (one device -> host read);
          labels outside [0, C) anywhere  -> LabelError on every rank (the per-rank label
                                             counts are summed by one all-reduce, which only
                                             this failure branch issues);
          non-finite scores of a method whose forward ran on fp16 operand halves (an
          activation past 65504: the split gives inf / NaN, which the kernels' NaN-propagating
          ReLUs carry to the scores) -> every rank rebuilds that forward's packs on bf16
                                             halves (fp32's range), re-scores the method on its
                                             shard and gathers again; the engine keeps the bf16
                                             packs (`fallback` records it; EL2N on bf16 halves
                                             then takes the near-threshold fp32 re-scoring,
                                             refine "auto");
          anything else non-finite        -> ValueError (the selection would reject NaN)."""
        ms = list(full)
        if not ms or N == 0:
            return full
        fin = torch.stack([torch.isfinite(full[m]).all() for m in ms]).cpu()
        if bool(fin.all()):
            return full
        bad = self._bad.clone() if self._bad is not None else _capi.label_counter(self.device)
        if world_of(group) > 1:
            _all_reduce_sum(bad, group)
        _capi.check_labels(bad, self.models[0].linear.out_features, "run")
        redo = [m for i, m in enumerate(ms) if not bool(fin[i]) and self._f16_forward(m)]
        if redo:
            ops = {"el2n": "el2n_operands", "grand": "grand_operands"}
            self.cfg = dataclasses.replace(self.cfg, **{ops[m]: "bf16x3" for m in redo})
            self.fallback = {m: "a forward activation left fp16's range: re-scored on bf16 "
                                "operand halves" for m in redo}
            if "grand" in redo:
                self.grand_fallback = self.fallback["grand"]
            for mod in self.models:
                mod.prepare_fast_convs(self.cfg.el2n_operands, self.cfg.grand_operands)
            saved = self.cfg
            self.cfg = dataclasses.replace(saved, methods=tuple(redo), select_by=redo[0])
            try:
                world, rank = _world(group)
                lo, hi = shard_bounds(N, B, world, rank)
                local = score(lo, hi)
            finally:
                self.cfg = saved
            full = dict(full)
            for m in redo:
                full[m] = gather_scores(local[m], N, B, group)
        for m in ms:
            if not bool(torch.isfinite(full[m]).all()):
                raise ValueError(f"non-finite {m} scores" + (
                    " on bf16 operand halves too" if m in redo else ""))
        return full

    def _f16_forward(self, method: str) -> bool:
        """Whether `method`'s forward runs on fp16 operand halves (range 65504)."""
        c = self.cfg
        if not c.fast_convs:
            return False
        if method == "el2n":
            return c.el2n_operands == "f16x3"
        return c.grand_operands == "f16x3" and c.fold_bn

    def run(self, images_u8: torch.Tensor, labels: torch.Tensor, sparsity: float,
            group=None, check_nan: bool = True, n_total: int = None):
        """Score the whole dataset (sharded over the process group if initialised), gather,
        select.  Returns (full score dict on device, kept indices int64 on device, k).

        With `n_total` None, `images_u8`/`labels` hold every example (each rank reads its
        shard out of them).  With `n_total` given they hold ONLY this rank's shard
        [lo, hi) of the n_total examples (shard_bounds), so no rank needs the whole set in
        HBM (ImageNet shape: 193 GB of uint8)."""
        N = labels.numel() if n_total is None else int(n_total)
        B = self.cfg.batch_size
        world, rank = _world(group)
        lo, hi = shard_bounds(N, B, world, rank)
        off = 0 if n_total is None else lo  # global index g is local row g - off

        def score(lo, hi):
            if n_total is None:
                return self.score_shard(images_u8, labels, lo, hi, check=False)
            if labels.numel() != hi - lo or images_u8.shape[0] != hi - lo:
                raise ValueError(f"this rank's shard is [{lo}, {hi}) of {N}: got "
                                 f"{images_u8.shape[0]} images / {labels.numel()} labels")
            # shards are batch-aligned, so the partition anchored at 0 of the shard equals
            # the global one
            return self.score_shard(images_u8, labels, 0, hi - lo, check=False)

        def select(keys, k):
            return _capi.select_topk(keys, k, check_nan=check_nan)[0]

        full, kept, k = sharded_job(score, N, B, sparsity, self.cfg.select_by, select,
                                    _capi.keep_count, group,
                                    validate=lambda f: self._validate(f, score, N, B, group))
        self.last_refine = None
        if self._refines(self.cfg.select_by) and 0 < k < N:
            full, kept = self._refine(full, k, images_u8, labels, lo, hi, off, N, group,
                                      check_nan)
        return full, kept, k

    # ---- exact keep-set: fp32 re-scoring near the threshold --------------------------------
    def _refines(self, method: str) -> bool:
        """Whether `method`'s near-threshold scores are re-computed in plain fp32
        (ScoreConfig.refine: forced, or "auto" where the pass carries bf16-halves arithmetic)."""
        c = self.cfg
        if c.refine is False:
            return False
        if method == "el2n":
            if c.refine == "auto" and c.el2n_operands == "f16x3":
                return False
            return c.el2n_bn == "batch" and c.fast_convs
        # (grand_params "all" runs only on the fused split-bf16 schedule: no fp32 path to
        # re-score on)
        return c.grand_params == "conv_linear" and (c.fast_convs or c.pegrad_precision != "fp32")

    def _refine(self, full, k, images_u8, labels, lo, hi, off, N, group, check_nan):
        """Re-score near the threshold on the fp32 path until the keep-set is settled
        (ScoreConfig.refine; the loop is refine_keep_set).  The unit is EL2N's pinned batch
        (train-mode BN couples its rows) or one GraNd example.  Every rank holds the same
        gathered vectors (the fast-path scores and the current ones), so all take the same
        decisions; with W > 1 ranks the re-scoring is split by checkpoint
        (_rescore_fp32_ckpt_split).  Returns the updated score dict and the keep-set."""
        method = self.cfg.select_by
        world = world_of(group)

        def rescore(rows):
            if world > 1:
                return self._rescore_fp32_ckpt_split(method, images_u8, labels, rows, off, N,
                                                     group)
            return self._rescore_fp32(method, images_u8, labels, rows, off, N)

        torch.cuda.synchronize(self.device)
        s, kept, info = refine_keep_set(full[method], k,
                                        self.cfg.batch_size if method == "el2n" else 1,
                                        rescore, self.cfg, check_nan)
        torch.cuda.synchronize(self.device)
        self.last_refine = dict(method=method, **info)
        full = dict(full)
        full[method] = s
        return full, kept

    # bytes of images all-gathered per collective in the checkpoint-split refinement (its
    # memory does not grow with N: ImageNet rows are 150 KB each)
    refine_gather_bytes = 1 << 30

    def _rescore_fp32_ckpt_split(self, method, images_u8, labels, rows, off, N, group):
        """fp32 ensemble scores of the global row ranges `rows` on W > 1 ranks, split by
        checkpoint instead of by shard: the rows' images are all-gathered (each rank holds only
        its shard's), rank r runs checkpoints r, r + W, ... over all of them, and one all-reduce
        combines the per-checkpoint score vectors.  The refinement's cost per rank is then
        ~K / W forwards instead of K (it re-scores a few hundred rows: launch-bound, not
        row-bound), which is what keeps it from growing as a share of the step as W grows.

        Bitwise equal to the one-rank result: every rank runs the same `rows` through the same
        launches, each checkpoint's vector lands in its own row of a [K, rows] buffer (zeros
        elsewhere, so the all-reduce sum is exact), and the ensemble is accumulated in
        checkpoint order 0..K-1 as world 1 does.  The rows go in slices of at most
        `refine_gather_bytes` of images per collective."""
        world, rank = _world(group)
        B = self.cfg.batch_size
        K = len(self.models)
        # bytes per image from the shape every rank knows, even one whose shard is empty (a
        # per-rank cap would split the gathers differently on different ranks: ADVICE r05)
        per_img = max(1, int(np.prod(images_u8.shape[1:])) * images_u8.element_size())
        cap = max(B, self.refine_gather_bytes // per_img)
        slices, cur, c = [], [], 0
        for r in rows:  # whole units per slice (a pinned batch is never split)
            if cur and c + (r[1] - r[0]) > cap:
                slices.append(cur)
                cur, c = [], 0
            cur.append(r)
            c += r[1] - r[0]
        if cur:
            slices.append(cur)
        outs = []
        for part_rows in slices:
            per_rank = [[(r0, r1) for (r0, r1) in part_rows if blo <= r0 < bhi]
                        for blo, bhi in all_shards(N, B, world)]
            counts = [sum(r1 - r0 for r0, r1 in pr) for pr in per_rank]
            L = max(counts)
            shape = tuple(images_u8.shape[1:])
            img = torch.zeros((L,) + shape, dtype=images_u8.dtype, device=self.device)
            lab = torch.zeros(L, dtype=labels.dtype, device=self.device)
            c = 0
            for r0, r1 in per_rank[rank]:
                img[c:c + r1 - r0] = images_u8[r0 - off:r1 - off]
                lab[c:c + r1 - r0] = labels[r0 - off:r1 - off]
                c += r1 - r0
            img_all = torch.cat([t[:n] for t, n in zip(_all_gather_same(img, group), counts)])
            lab_all = torch.cat([t[:n] for t, n in zip(_all_gather_same(lab, group), counts)])
            del img, lab
            # rows ascend and the shards are contiguous and ascending: rank order is row order
            local, c = [], 0
            for r0, r1 in part_rows:
                local.append((c, c + r1 - r0))
                c += r1 - r0
            mine = [m for i, m in enumerate(self.models) if i % world == rank]
            per = torch.zeros((K, c), dtype=torch.float32, device=self.device)
            if mine:
                per[rank::world] = self._rescore_fp32(method, img_all, lab_all, local, 0, N,
                                                      models=mine, per_ckpt=True)
            del img_all, lab_all
            _all_reduce_sum(per, group)
            acc = torch.zeros(c, dtype=torch.float32, device=self.device)
            for kk in range(K):  # checkpoint order, as the one-rank accumulation
                acc += per[kk]
            out = torch.empty_like(acc)
            _capi.ensemble_finalize(acc, K, out)
            outs.append(out)
        return torch.cat(outs)

    def _rescore_fp32(self, method, images_u8, labels, rows, off, N, models=None,
                      per_ckpt=False):
        """fp32 ensemble scores of the global row ranges `rows` (this rank's), concatenated.
        models: the checkpoints to run (default all); per_ckpt=True returns each model's score
        vector instead ([len(models), rows]: 0 + s_k, bitwise the value the ensemble
        accumulation adds) of the ensemble mean over all K."""
        K = len(self.models)
        models = self.models if models is None else models
        if method == "grand":
            idx = torch.tensor([r0 - off for r0, _ in rows], dtype=torch.int64,
                               device=self.device)
            img, lab = images_u8[idx].contiguous(), labels[idx].contiguous()
            m = idx.numel()
            accs = [torch.zeros(m, dtype=torch.float32, device=self.device)
                    for _ in (models if per_ckpt else [None])]
            saved = self.cfg
            self.cfg = dataclasses.replace(saved, fast_convs=False, fused_grand=False,
                                           pegrad_precision="fp32", refine=False)
            try:
                for i, model in enumerate(models):
                    self.grand_pass(model, img, lab, 0, m, accs[i if per_ckpt else 0])
            finally:
                self.cfg = saved
            if per_ckpt:
                return torch.stack(accs)
            acc = accs[0]
            out = torch.empty_like(acc)
            _capi.ensemble_finalize(acc, K, out)
            return out
        # EL2N: whole pinned batches, `refine_groups` per launch (the count padded to a power of
        # two, so MIOpen sees few distinct batch sizes), ragged last batch last
        B = self.cfg.batch_size
        outs = []
        step = self.cfg.refine_groups
        shape = tuple(images_u8.shape[1:])
        with torch.inference_mode():
            for c in range(0, len(rows), step):
                part = rows[c:c + step]
                G = 1 << (len(part) - 1).bit_length()
                x = torch.zeros((G * B,) + shape, dtype=torch.float32, device=self.device)
                lab = torch.zeros(G * B, dtype=torch.int64, device=self.device)
                sel = []
                for gi, (r0, r1) in enumerate(part):
                    self._normalize(images_u8[r0 - off:r1 - off], x[gi * B:gi * B + (r1 - r0)])
                    lab[gi * B:gi * B + (r1 - r0)] = labels[r0 - off:r1 - off]
                    sel.append(torch.arange(gi * B, gi * B + (r1 - r0), device=self.device))
                sel = torch.cat(sel)
                r0, r1 = part[-1]
                n_valid = (len(part) - 1) * B + (r1 - r0)
                accs = [torch.zeros(sel.numel(), dtype=torch.float32, device=self.device)
                        for _ in (models if per_ckpt else [None])]
                for i, model in enumerate(models):
                    logits = el2n_fast.forward_logits_fp32(model, x, B, n_valid)
                    _capi.el2n(logits[sel].float().contiguous(), lab[sel].contiguous(),
                               accum=accs[i if per_ckpt else 0])
                if per_ckpt:
                    outs.append(torch.stack(accs))
                    continue
                out = torch.empty_like(accs[0])
                _capi.ensemble_finalize(accs[0], K, out)
                outs.append(out)
        return torch.cat(outs, dim=-1)
