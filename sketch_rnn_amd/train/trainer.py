"""Training drivers.

* :class:`ReferenceTrainer` -- the reference's epoch loop (``train.py:47-97``):
  per-epoch lr decay, reshuffle, zero state at epoch start, final state
  carried into the next batch (TBPTT), progress line in the reference format,
  divergence guard, periodic + final checkpoint, and (new) resume.
* :class:`VAETrainer` -- step loop for the seq2seq VAE with lr decay, KL
  annealing, per-element gradient clipping, periodic valid/test evaluation
  (recon NLL) and checkpointing; data-parallel over RCCL when
  ``torch.distributed`` is initialised.

Both can capture their step into a HIP graph on the GPU (:mod:`.graph`).
"""
from __future__ import annotations

import json
import math
import os
import time
from typing import Callable, Dict, Optional

import numpy as np
import torch

from ..ckpt import checkpoint as ckpt
from ..config import RefConfig, VAEConfig
from ..models.reference import SketchRNN
from ..models.vae import SketchVAE
from ..ops import gemm
from ..parallel import dp
from ..utils.trace import GpuPhaseTimer, PhaseTimes, phase
from . import schedules
from .graph import GraphedPhases, GraphedStep
from .optim import FlatAdam


class DivergenceError(RuntimeError):
    pass


def check_device_faults() -> None:
    """Raise when a kernel reported a fault through a device flag since the
    last check. Every kernel with in-launch waits on peer workgroups (the
    clustered LayerNorm cells, the persistent LSTM stack, the fused decoders,
    the hyper-fused GEMM) bounds its spins and sets the flag when one timed
    out -- that step's outputs are invalid. Under DP the flag is max-reduced
    over the ranks, so every rank raises at the same step instead of the
    healthy ones blocking in their next collective. Trainers call it at every
    log interval and before every checkpoint save (all ranks together)."""
    from ..ops import recurrent
    bad = 0
    for f in list(recurrent._ERR_FLAGS.values()):
        if int(f.item()) != 0:
            f.zero_()
            bad = 1
    if dp.max_scalar(float(bad)) != 0:
        raise DivergenceError("device fault: an in-launch wait on a peer workgroup timed out on %s "
                              "(workgroups not co-resident); the step's results are invalid"
                              % ("this rank" if bad else "another rank"))


def _to_device(a, device, dtype=torch.float32):
    if not torch.is_tensor(a):
        a = torch.as_tensor(np.ascontiguousarray(a))
    return a.to(device=device, dtype=dtype, non_blocking=True)


# =====================================================================================
# reference decoder-only model
# =====================================================================================
class ReferenceTrainer:
    def __init__(self, cfg: RefConfig, loader, device: str = "cpu", save_root: str = "save",
                 use_graph: Optional[bool] = None, log: Callable[[str], None] = print,
                 metrics_path: Optional[str] = None):
        self.cfg = cfg
        self.loader = loader
        self.device = torch.device(device)
        self.model = SketchRNN(cfg).to(self.device)
        # TF semantics (a NaN step is applied; the divergence guard then stops the run, train.py:93-94)
        self.opt = FlatAdam(self.model.parameters(), lr=cfg.learning_rate, eps=cfg.adam_eps,
                            clip_mode="global_norm", clip=cfg.grad_clip, nonfinite="apply")
        self.save_dir = os.path.join(save_root, cfg.dataset_name)
        self.log = log
        self.metrics_path = metrics_path
        self.b_processed = 0
        self.epoch = 0
        self.use_graph = (self.device.type == "cuda") if use_graph is None else use_graph
        self._graph = None
        B = cfg.batch_size
        self.state = self.model.zero_state(B, self.device)
        self.seed = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._in_epoch = False

    # ---------------------------------------------------------------------------------
    def _step_fn(self, x, y, state_flat):
        state = self._unflatten(state_flat)
        self.opt.zero_grad(set_to_none=True)
        cost, shape, pen, final = self.model.loss(x, y, state, train=True, drop_seed=self.seed)
        cost.backward()
        self.opt.gather_grads()
        self.opt.step()
        with torch.no_grad():
            for dst, src in zip(state_flat, self._flatten(final)):
                dst.copy_(src)
        return {"cost": cost.detach(), "shape": shape.detach(), "pen": pen.detach()}

    def _flatten(self, state):
        out = []
        for s in state:
            out.extend(s if isinstance(s, tuple) else (s,))
        return out

    def _unflatten(self, flat):
        if self.cfg.model == "lstm":
            return [(flat[2 * i], flat[2 * i + 1]) for i in range(len(flat) // 2)]
        return list(flat)

    def train_step(self, x: torch.Tensor, y: torch.Tensor) -> Dict[str, torch.Tensor]:
        gemm.invalidate_derived()   # weights change in place (possibly inside a graph replay)
        state_flat = self._flatten(self.state)
        if self.use_graph:
            if self._graph is None:
                static = {"x": x.clone(), "y": y.clone()}
                snap = [self.opt.flat, self.opt.m, self.opt.v, self.opt.scalars] + \
                       [s for s in state_flat]
                self._graph = GraphedStep(lambda x, y: self._step_fn(x, y, state_flat), static,
                                          snapshot=snap)
            out = self._graph(x=x, y=y)
        else:
            out = self._step_fn(x, y, state_flat)
        self.opt.step_count = int(self.opt.step_count)  # host mirror (device counter is authoritative)
        self.seed.add_(1)
        return out

    # ---------------------------------------------------------------------------------
    def save(self):
        st = {"s%d" % i: t for i, t in enumerate(self._flatten(self.state))}
        extra = {"epoch": self.epoch, "in_epoch": self._in_epoch, "b_processed": self.b_processed,
                 "seed": int(self.seed.item()),
                 "loader": self.loader.state_dict()}
        path = ckpt.save_checkpoint(self.save_dir, self.b_processed, self.model, self.opt, self.cfg,
                                    extra=extra, state=st)
        self.log("model saved to {}".format(path))
        return path

    def resume(self) -> bool:
        path = ckpt.latest_checkpoint(self.save_dir)
        if path is None:
            return False
        step, extra, st = ckpt.load_checkpoint(path, self.model, self.opt)
        self.b_processed = int(extra.get("b_processed", step))
        self.epoch = int(extra.get("epoch", 0))
        self.seed.fill_(int(extra.get("seed", self.b_processed)))
        for i, t in enumerate(self._flatten(self.state)):
            if "s%d" % i in st:
                t.copy_(st["s%d" % i])
        if "loader" in extra:
            # continue the interrupted epoch: same permutation, cursor, RNG and carried state
            self.loader.load_state_dict(extra["loader"])
            self._in_epoch = bool(extra.get("in_epoch", False))
        self.log("resumed from %s (epoch %d, batch %d)" % (path, self.epoch, self.b_processed))
        return True

    def train(self, num_epochs: Optional[int] = None, max_batches: Optional[int] = None):
        cfg, loader = self.cfg, self.loader
        num_epochs = cfg.num_epochs if num_epochs is None else num_epochs
        done = 0
        while self.epoch < num_epochs:
            e = self.epoch
            self.opt.set_lr(schedules.reference_lr(cfg, e))
            if not self._in_epoch:  # a resumed / interrupted epoch continues where it stopped
                loader.reset_index_pointer()
                for s in self._flatten(self.state):
                    s.zero_()
                self._in_epoch = True
            while self._in_epoch:
                t0 = time.time()
                x, y = loader.next_batch()
                out = self.train_step(_to_device(x, self.device), _to_device(y, self.device))
                cost, shape, pen = (float(out[k]) for k in ("cost", "shape", "pen"))
                dt = time.time() - t0
                self.b_processed += 1
                if loader.epoch_finished:
                    self._in_epoch = False
                    self.epoch += 1
                self.log("{}/{} (epoch {} batch {}), cost = {:.2f} ({:.2f}+{:.4f}), time/batch = {:.2f}".format(
                    loader.pointer + e * loader.num_samples, num_epochs * loader.num_samples,
                    e, self.b_processed, cost, shape, pen, dt))
                self._metrics({"step": self.b_processed, "epoch": e, "cost": cost, "shape": shape,
                               "pen": pen, "time": dt, "lr": self.opt.lr,
                               "strokes_per_s": cfg.batch_size * cfg.seq_length / max(dt, 1e-9)})
                check_device_faults()
                if not (cost < cfg.divergence_bound):  # NaN fails this too (train.py:93-94)
                    raise DivergenceError("training diverged: cost=%r" % cost)
                if self.b_processed % cfg.save_every == 0 and self.b_processed > 0:
                    self.save()
                done += 1
                if max_batches is not None and done >= max_batches:
                    return self.save()
        return self.save()

    def _metrics(self, rec):
        if self.metrics_path:
            with open(self.metrics_path, "a") as f:
                f.write(json.dumps(rec) + "\n")


# =====================================================================================
# seq2seq VAE
# =====================================================================================
class VAETrainer:
    def __init__(self, cfg: VAEConfig, train_set, valid_set=None, test_set=None, device: str = "cpu",
                 save_dir: str = "save/vae", use_graph: Optional[bool] = None,
                 log: Callable[[str], None] = print, metrics_path: Optional[str] = None,
                 compute_dtype: str = "fp32", max_skipped: int = 100, dp_wire_dtype: Optional[str] = None,
                 force_reducer: bool = False, dp_bucket_mb: float = 32.0):
        self.cfg = cfg
        self.train_set, self.valid_set, self.test_set = train_set, valid_set, test_set
        self.device = torch.device(device)
        self.rank, self.world = dp.rank(), dp.world_size()
        self.model = SketchVAE(cfg).to(self.device)
        from .. import ops
        ops.set_compute_dtype(compute_dtype)
        # arena order: parameters whose gradients are final once the decoder /
        # head backward is done, then the encoder's (computed last); with DP
        # the first part's all-reduce overlaps the encoder backward
        enc = self.model.encoder
        enc_ids = {id(p) for p in enc.parameters()} if enc is not None else set()
        self._early = [p for p in self.model.parameters() if id(p) not in enc_ids]
        self._late = [p for p in self.model.parameters() if id(p) in enc_ids]
        # a step with a non-finite gradient is dropped on the device and counted (FlatAdam)
        self.opt = FlatAdam(self._early + self._late, lr=cfg.learning_rate, eps=cfg.adam_eps,
                            clip_mode="value", clip=cfg.grad_clip, nonfinite="skip")
        self.max_skipped = max_skipped
        dp.broadcast_params(self.opt.flat)
        late = [p for p in self._late if p.requires_grad]
        # SKR_DP_OVERLAP: "1" on, "0" off, default on for RCCL only. gloo's
        # CUDA collectives stage through host threads that block on stream
        # syncs: the overlapped step measured 4.1 s/step against 20 ms for the
        # plain step (2 ranks on one GPU, vae_small; 41 ms with a device sync
        # between phases), so gloo keeps the plain step unless forced.
        # Concurrency decision (RCCL): overlap stays ON. The kernels that spin
        # on peer workgroups (lstm_persist_bwd of the encoder, the clustered
        # LayerNorm / HyperLSTM cells) never wait on a collective, so an RCCL
        # kernel holding CU slots only delays their unplaced workgroups until it
        # retires; the bounded spins last ~seconds, an all-reduce kernel's
        # residency milliseconds. Measured on MI355X with an occupancy hog on a
        # second stream (tests/test_dp_concurrency_gpu.py,
        # profiles/r3/dp_concurrency_hog.jsonl): 64x512-thread/32 KB-LDS and
        # whole-chip 256x1024 hogs for 20 ms, and a half-chip hog for 200 ms,
        # beside the encoder backward (solo 1.3 ms) and the H=2048 HyperLSTM
        # cells: every run finished right after the hog (20.2-21.7 / 200.2 ms),
        # no fault flag, outputs and gradients bit-identical to the solo run.
        ov = os.environ.get("SKR_DP_OVERLAP", "auto")
        if ov == "auto":
            ov = "1" if (self.world > 1 and dp.backend() == "nccl") or self.device.type == "cpu" else "0"
        # force_reducer: run the collectives even at world size 1 (RCCL path check on one GPU)
        reduce_on = self.world > 1 or (force_reducer and dp.is_dist())
        self.overlap = reduce_on and bool(late) and ov == "1"
        split = self.opt.offset_of[id(late[0])] if self.overlap else None
        # SKR_DP_WIRE=bf16: gradients cross the xGMI ring in bf16 (half the bytes)
        wire = dp_wire_dtype or os.environ.get("SKR_DP_WIRE", "fp32")
        # the arena plus its tail (this step's loss scalars, summed in the last
        # bucket); the 1/world average is folded into the clip + Adam kernels
        self.reducer = dp.GradReducer(self.opt.grad_full, bucket_mb=dp_bucket_mb, split=split, wire_dtype=wire,
                                      force=force_reducer, fold_scale=True, tail=FlatAdam.TAIL) if reduce_on else None
        if reduce_on:
            self.opt.set_grad_scale(1.0 / self.world)
        self._enc_pending = None
        self.save_dir = save_dir
        self.log = log
        self.metrics_path = metrics_path
        self.step = 0
        self.use_graph = (self.device.type == "cuda") if use_graph is None else use_graph
        self._graph = None
        # noise seed (dropout masks, reparameterisation eps): rank r uses
        # r, r + world, r + 2*world, ... so ranks draw independent noise
        self.seed = torch.full((1,), self.rank, dtype=torch.int64, device=self.device)
        self.kl_w = torch.zeros((), device=self.device)
        self.host_times = PhaseTimes()            # data / step / eval / save wall time
        self.gpu_times = GpuPhaseTimer(enabled=metrics_path is not None)

    # loss scalars packed into the gradient arena's tail (summed over ranks
    # with the last all-reduce bucket; the trainer logs their global mean)
    _TAIL_KEYS = ("cost", "r_cost", "kl_cost", "shape_cost", "pen_cost")

    def _pack_scalars(self, out, lengths):
        if self.reducer is None:
            return
        vals = [out[k].detach().reshape(()).float() for k in self._TAIL_KEYS if k in out]
        vals.append(lengths.sum().to(torch.float32))
        self.opt.tail[:len(vals)].copy_(torch.stack(vals))

    def reduced_scalars(self) -> Dict[str, float]:
        """The last step's loss scalars averaged over ranks and the global
        count of valid stroke points (from the reduced arena tail; one host
        read). Only meaningful with an active reducer."""
        keys = [k for k in self._TAIL_KEYS if k in self._last_keys]
        t = self.opt.tail[:len(keys) + 1].tolist()
        res = {k: v / self.world for k, v in zip(keys, t)}
        res["valid_points"] = t[len(keys)]
        return res

    def _fwd_bwd(self, strokes, lengths, labels):
        self.opt.zero_grad(set_to_none=True)
        out = self.model.loss(strokes, lengths, labels if self.cfg.num_classes > 0 else None,
                              kl_weight=self.kl_w, train=True, seed=self.seed)
        out["cost"].backward()
        self.opt.gather_grads()
        self._pack_scalars(out, lengths)
        self._last_keys = tuple(out)
        return {k: v.detach() for k, v in out.items()}

    def _opt_step(self):
        self.opt.step()
        return {}

    # two-phase backward (DP overlap): phase A = forward + backward down to
    # the encoder outputs, phase B = the encoder backward
    def _fwd_bwd_a(self, strokes, lengths, labels):
        self.opt.zero_grad(set_to_none=True)
        out = self.model.loss(strokes, lengths, labels if self.cfg.num_classes > 0 else None,
                              kl_weight=self.kl_w, train=True, seed=self.seed, split_encoder=True)
        enc, cut = out.pop("_enc")
        out["cost"].backward()
        self.opt.gather_grads(self._early)
        self._enc_pending = (enc, [t.grad for t in cut])
        self._pack_scalars(out, lengths)
        self._last_keys = tuple(out)
        return {k: v.detach() for k, v in out.items()}

    def _bwd_b(self):
        enc, grads = self._enc_pending
        self._enc_pending = None
        torch.autograd.backward(list(enc), grads)
        self.opt.gather_grads(self._late)
        return {}

    def _step_fn(self, strokes, lengths, labels):
        out = self._fwd_bwd(strokes, lengths, labels)
        if self.reducer is not None:
            self.reducer.all_reduce()
        self.opt.step()
        return out

    def train_step(self, strokes, lengths, labels):
        """One optimisation step. On the GPU the forward+backward is one
        captured HIP graph; with DP (and an encoder) the step runs as three
        graphs with the bucketed RCCL all-reduces issued between them, the
        decoder/head part overlapping the encoder backward
        (:meth:`_train_step_overlap`; ``SKR_DP_OVERLAP=0``: one all-reduce
        between the forward+backward graph and the clip+Adam graph).""" 
        gemm.invalidate_derived()   # weights change in place (possibly inside a graph replay)
        self.opt.set_lr(schedules.vae_lr(self.cfg, self.step))
        self.kl_w.fill_(schedules.kl_weight(self.cfg, self.step))
        if self.overlap:
            out = self._train_step_overlap(strokes, lengths, labels)
        elif self.use_graph:
            if self._graph is None:
                static = {"strokes": strokes.clone(), "lengths": lengths.clone(), "labels": labels.clone()}
                snap = [self.opt.flat, self.opt.m, self.opt.v, self.opt.scalars]
                if self.reducer is None:
                    self._graph = GraphedStep(self._step_fn, static, snapshot=snap)
                    self._graph_opt = None
                else:
                    self._graph = GraphedStep(self._fwd_bwd, static, snapshot=snap)
                    self._graph_opt = GraphedStep(self._opt_step, {}, snapshot=snap)
            with self.gpu_times.time("fwd_bwd" if self._graph_opt is not None else "step"):
                out = self._graph(strokes=strokes, lengths=lengths, labels=labels)
            if self._graph_opt is not None:
                with self.gpu_times.time("allreduce"):
                    self.reducer.all_reduce()
                with self.gpu_times.time("optimizer"):
                    self._graph_opt()
        else:
            with self.gpu_times.time("step"):
                out = self._step_fn(strokes, lengths, labels)
        self.seed.add_(self.world)
        self.step += 1
        return out

    def _train_step_overlap(self, strokes, lengths, labels):
        """DP step with the decoder/head gradient all-reduce in flight while
        the encoder backward runs: [phase A] -> all-reduce(part 0, async)
        -> [phase B] -> all-reduce(part 1, async) -> wait -> [clip + Adam].
        On the GPU each bracketed phase is a captured HIP graph."""
        if self.use_graph:
            if self._graph is None:
                static = {"strokes": strokes.clone(), "lengths": lengths.clone(), "labels": labels.clone()}
                snap = [self.opt.flat, self.opt.m, self.opt.v, self.opt.scalars]
                self._graph = GraphedPhases([self._fwd_bwd_a, self._bwd_b, self._opt_step], static, snapshot=snap)
            if os.environ.get("SKR_TRACE_PHASES"):
                import sys
                ts = [time.perf_counter()]

                def mark():
                    torch.cuda.synchronize()
                    ts.append(time.perf_counter())
                out = self._graph.replay(0, strokes=strokes, lengths=lengths, labels=labels)
                mark()
                w0 = self.reducer.start(0)
                mark()
                self._graph.replay(1)
                mark()
                w1 = self.reducer.start(1)
                mark()
                self.reducer.wait(w0 + w1)
                mark()
                self._graph.replay(2)
                mark()
                print("phases ms:", ["%.2f" % (1e3 * (b - a)) for a, b in zip(ts, ts[1:])], file=sys.stderr)
                return out
            with self.gpu_times.time("fwd_bwd"):
                out = self._graph.replay(0, strokes=strokes, lengths=lengths, labels=labels)
                w0 = self.reducer.start(0)
                self._graph.replay(1)
            with self.gpu_times.time("allreduce"):
                self.reducer.wait(w0 + self.reducer.start(1))
            with self.gpu_times.time("optimizer"):
                self._graph.replay(2)
            return out
        with self.gpu_times.time("step"):
            out = self._fwd_bwd_a(strokes, lengths, labels)
            w0 = self.reducer.start(0)
            self._bwd_b()
            self.reducer.wait(w0 + self.reducer.start(1))
            self.opt.step()
        return out

    def batch_to_device(self, batch):
        s, l, c = batch
        return (_to_device(s, self.device), _to_device(l, self.device, torch.int64),
                _to_device(c, self.device, torch.int64))

    @torch.no_grad()
    def evaluate(self, dataset, max_batches: Optional[int] = None) -> Dict[str, float]:
        """Mean cost / recon NLL / KL over the dataset (no dropout, fixed eps seed)."""
        tot = {"cost": 0.0, "r_cost": 0.0, "kl_cost": 0.0}
        n = dataset.num_batches if max_batches is None else min(max_batches, dataset.num_batches)
        gen = torch.Generator(device=self.device).manual_seed(1234)
        for b in range(n):
            s, l, c = self.batch_to_device(dataset.get_batch(b))
            eps = torch.randn(s.shape[0], self.cfg.z_size, device=self.device, generator=gen)
            out = self.model.loss(s, l, c if self.cfg.num_classes > 0 else None,
                                  kl_weight=self.cfg.kl_weight, train=False, eps=eps)
            for k in tot:
                tot[k] += float(out[k])
        res = {k: v / max(n, 1) for k, v in tot.items()}
        return dp.average_scalars(res)

    def save(self):
        if self.rank != 0:
            return None
        extra = {"step": self.step, "seed": int(self.seed.item())}
        pf = getattr(self, "_prefetch", None)
        if pf is not None and pf.consumed_state is not None:
            extra["data"] = pf.consumed_state     # batches still queued are regenerated on resume
        elif hasattr(self.train_set, "state_dict"):
            extra["data"] = self.train_set.state_dict()
        return ckpt.save_checkpoint(self.save_dir, self.step, self.model, self.opt, self.cfg, extra=extra)

    def resume(self) -> bool:
        """Weights, Adam moments/step, schedules (a function of the step),
        dropout seed and data RNG. With DP every rank loads the same file
        (rank 0 wrote it); the per-rank augmentation RNG restarts from the
        saved rank-0 stream offset by rank."""
        path = ckpt.latest_checkpoint(self.save_dir)
        if path is None:
            return False
        self.step, extra, _ = ckpt.load_checkpoint(path, self.model, self.opt)
        self.seed.fill_(int(extra.get("seed", self.step * self.world)) + self.rank)   # saved by rank 0
        if "data" in extra and hasattr(self.train_set, "load_state_dict"):
            self.train_set.load_state_dict(extra["data"])
            if self.rank:
                self.train_set.aug_rng.seed((self.cfg.seed * 7919 + 1 + self.rank + self.step) % (2 ** 32))
        return True

    def train(self, num_steps: Optional[int] = None, eval_every: int = 0, log_every: int = 20,
              prefetch: bool = True):
        """Step loop. ``prefetch``: batches are built ``2`` ahead on a
        background thread into pinned host memory (:mod:`..data.prefetch`);
        the same batches in the same order as without it."""
        from ..data.prefetch import Prefetcher
        self._prefetch = None
        if prefetch:
            self._prefetch = Prefetcher(lambda: self.train_set.random_batch(self.rank, self.world),
                                        getattr(self.train_set, "state_dict", None))
        try:
            return self._train_loop(num_steps, eval_every, log_every)
        finally:
            if self._prefetch is not None:
                consumed = self._prefetch.consumed_state
                self._prefetch.close()
                self._prefetch = None
                # the producer drew batches ahead of the consumer: rewind the
                # dataset to the last batch actually trained on, so a later
                # train() / save() continues the same sequence
                if consumed is not None and hasattr(self.train_set, "load_state_dict"):
                    self.train_set.load_state_dict(consumed)

    def _train_loop(self, num_steps, eval_every, log_every):
        cfg = self.cfg
        num_steps = cfg.num_steps if num_steps is None else num_steps
        pf = self._prefetch
        t0 = time.time()
        valid = 0.0     # this rank's non-padding stroke points since the last log line
        # every rank's points (DP): summed on the device from each step's reduced arena tail
        valid_glob = torch.zeros((), dtype=torch.float64, device=self.device)
        n_int = 0       # steps since the last log line (resume / repeated train() safe)
        while self.step < num_steps:
            with phase("data", self.host_times):
                raw = pf.get() if pf is not None else self.train_set.random_batch(self.rank, self.world)
                valid += float(np.asarray(raw[1]).sum())
                batch = self.batch_to_device(raw)
            with phase("step", self.host_times):
                out = self.train_step(*batch)
            if self.reducer is not None:
                # global point count of this step from the reduced arena tail,
                # accumulated on the device (no host sync, no collective)
                idx = len([k for k in self._TAIL_KEYS if k in self._last_keys])
                valid_glob.add_(self.opt.tail[idx].double())
            n_int += 1
            if self.step % log_every == 0 or self.step == num_steps:
                check_device_faults()
                if self.reducer is not None:   # global means, from the arena tail (no extra collective)
                    vals = self.reduced_scalars()
                    vals.pop("valid_points")
                    valid_all = float(valid_glob)           # summed per step from the reduced tails
                else:
                    vals = {k: float(v) for k, v in out.items()}
                    valid_all = valid                       # one rank: this rank's batches
                dt = (time.time() - t0) / n_int
                t0 = time.time()
                valid = 0.0
                valid_glob.zero_()
                if self.rank == 0:
                    self.log("step: %d, lr: %.6f, klw: %0.4f, cost: %.4f, recon: %.4f, kl: %.4f, time/step: %.4f" % (
                        self.step, self.opt.lr, schedules.kl_weight(cfg, self.step - 1), vals["cost"],
                        vals["r_cost"], vals["kl_cost"], dt))
                    vals["grad_norm"] = float(self.opt.scalars[2])
                    if self.metrics_path:
                        rec = dict(step=self.step, **vals, time=dt, lr=self.opt.lr,
                                   kl_weight=schedules.kl_weight(cfg, self.step - 1),
                                   strokes_per_s=valid_all / max(dt * n_int, 1e-9),      # valid points
                                   positions_per_s=self.world * cfg.batch_size * cfg.max_seq_len / max(dt, 1e-9),
                                   skipped=self.opt.skipped_steps(),
                                   host_ms=self.host_times.mean_ms(), gpu_ms=self.gpu_times.collect())
                        self.host_times.reset()
                        with open(self.metrics_path, "a") as f:
                            f.write(json.dumps(rec) + "\n")
                n_int = 0
                skipped = self.opt.skipped_steps()
                if skipped > self.max_skipped:
                    raise DivergenceError("%d steps with a non-finite gradient (last cost %r at step %d)"
                                          % (skipped, vals["cost"], self.step))
            if eval_every and self.step % eval_every == 0 and self.valid_set is not None:
                with phase("eval", self.host_times):
                    ev = self.evaluate(self.valid_set)
                if self.rank == 0:
                    self.log("valid: cost %.4f recon %.4f kl %.4f" % (ev["cost"], ev["r_cost"], ev["kl_cost"]))
            if cfg.save_every and self.step % cfg.save_every == 0:
                with phase("save", self.host_times):
                    check_device_faults()     # never checkpoint a step whose exchange timed out
                    self.save()
                    # every rank waits for rank 0's write: no rank starts the next
                    # step's collectives (whose kernels would then hold CUs waiting
                    # on rank 0) while rank 0 is still busy writing
                    dp.barrier()
        check_device_faults()
        path = self.save()
        dp.barrier()
        return path
