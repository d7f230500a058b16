"""One federated round on the engine (the body of ExperimentRunner.run_simulation,
experiments/run_experiments.py:188-259, minus evaluation and checkpointing).

  for each client: fresh model <- global; local SGD                (:193-240)
  malicious clients submit a poisoned update                       (malicious_client.py:103-115)
  aggregated = defense.aggregate(client_updates, num_examples)     (:243-254)
  global params <- aggregated                                      (:257-259)

The K clients are sharded over the GPUs (flr.dist); each GPU trains its rows
of the client matrix together.  The exchange is then either
* "alltoall" (default for FedAvg / Krum / trimmed mean / median): one
  all-to-all hands every GPU all K clients' values of its coordinate range
  (flr.shard), each GPU aggregates its range, and one all-gather of the
  P-vector slices rebuilds the global model; or
* "allgather": one all-gather assembles the whole K×P matrix on every GPU and
  the aggregation runs replicated (defenses that need whole rows).
Both give the bit-identical global model at every GPU count.
"""
from __future__ import annotations

import inspect
import logging
import os
from dataclasses import dataclass, field
from typing import Dict, Optional

import torch

from . import _capi
from . import dist as fdist
from . import ops
from .attacks import Backdoor, poison_batches_
from .defenses import get_defense
from .matrix import ClientMatrix
from .shard import PW_SLICES, Comm, CoordExchange, aligned_bounds
from .models.multimodal import ModelSpec, model_class, param_layout
from .train import ClientBatchTrainer, TrainConfig, make_dropout_masks, synthetic_batches


@dataclass
class RoundConfig:
    num_clients: int = 128
    batch: int = 32                      # run_experiments.py:40
    defense: str = "krum"
    defense_cfg: Dict = field(default_factory=dict)
    attack: str = "sign_flip"            # "sign_flip" (model_poisoning.py:274-276) | "backdoor" | "none"
    num_attackers: int = 25              # f = int(0.2 K), clients 0..f-1 (experiment_matrix.py:67-68)
    seed: int = 42                       # run_experiments.py:43
    exchange: str = "auto"               # "alltoall" | "allgather" | "auto" (alltoall when the defense shards)
    graph: bool = True                   # replay the training phase as one captured HIP graph (FLR_GRAPH=0: eager)
    fallback_fedavg: bool = False        # defense raises -> FedAvg of the round (robust_server.py:120-122)
    # with fallback_fedavg: also fall back on library / device errors (FlrError,
    # out of memory), as the reference's `except Exception` does (the default:
    # ADVICE r5, parity with robust_server.py:120-122).  At world > 1 a device
    # error is never swallowed — one rank falling back while the others wait in
    # the defense's next collective would hang the round instead of failing it;
    # False keeps device errors loud at world 1 too
    fallback_device_errors: bool = True


def initial_global(spec: ModelSpec, seed: int, device) -> torch.Tensor:
    """Global model init: the torch default init of the spec's model under seed."""
    torch.manual_seed(seed)
    m = model_class(spec)(spec)
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()]).to(device)


class _DeadFill:
    """The deferred dead-tap fill of a round (RoundEngine, FLR_DEFER_DEAD):
    side stream, the distances' 'X read for the last time' mark, the fill's
    done event, per-block dead-tap masks; state 0 idle, 1 due this round."""

    class _Mark:
        def __init__(self, device):
            self.event = torch.cuda.Event()
            self.event.record(torch.cuda.current_stream(device))  # created now: a handle to pass down
            self.recorded = False

    def __init__(self, device, masks):
        self.side = torch.cuda.Stream(device)
        self.mark = _DeadFill._Mark(device)
        self.done = torch.cuda.Event()
        self.masks = masks
        self.state = 0


class RoundEngine:
    def __init__(self, spec: ModelSpec, rcfg: RoundConfig, tcfg: TrainConfig = TrainConfig(), device="cuda",
                 rank: int = 0, world: int = 1):
        self.spec, self.rcfg, self.tcfg = spec, rcfg, tcfg
        self.device = torch.device(device)
        self.rank, self.world = rank, world
        K = rcfg.num_clients
        self.lo, self.hi = fdist.shard(K, world, rank)
        shapes = [s for _, s in param_layout(spec)]
        # the ResNet + GRU and ViT + BERT families train through one C entry
        # (flr_train_clients_ex / flr_train_vit_bert: no torch kernel in the
        # training phase); FLR_TRAINER=python: the autograd composition of the
        # same kernels (A/B; the CUB family)
        self.native = (spec.family in ("resnet_gru", "vit_bert") and self.device.type == "cuda"
                       and os.environ.get("FLR_TRAINER", "native") != "python")
        if self.native:
            from .native_trainer import NativeRoundTrainer
            self.trainer = NativeRoundTrainer(spec, self.hi - self.lo, self.device, tcfg, batch=rcfg.batch)
        else:
            self.trainer = ClientBatchTrainer(spec, self.hi - self.lo, self.device, tcfg)
        cfg = dict(rcfg.defense_cfg)
        if rcfg.defense in ("krum", "multi_krum", "krum_trimmed_mean"):  # run_experiments.py:155-162
            cfg.setdefault("num_malicious", rcfg.num_attackers)
            cfg.setdefault("multi_k", max(1, K // 2))
        self.defense = get_defense(rcfg.defense, cfg)
        mode = rcfg.exchange
        if mode == "auto":
            mode = "alltoall" if (self.defense.supports_sharded and PW_SLICES % world == 0) else "allgather"
        if mode not in ("alltoall", "allgather"):
            raise ValueError(f"unknown exchange mode {rcfg.exchange!r}")
        if mode == "alltoall" and not self.defense.supports_sharded:
            raise ValueError(f"{self.defense!r} needs whole client rows: use exchange='allgather'")
        self.exchange = mode
        self.full = None
        self.xchg = None
        self.slice = None
        self.global_flat = initial_global(spec, rcfg.seed, self.device)
        steps = tcfg.local_steps
        self.batches = synthetic_batches(spec, steps, range(self.lo, self.hi), rcfg.batch, self.device)
        self.masks = make_dropout_masks(spec, steps, range(self.lo, self.hi), rcfg.batch, self.device,
                                        seed=rcfg.seed + 7919)
        if rcfg.attack == "backdoor":  # data poisoning of the malicious clients (run_experiments.py:173-175)
            cols = [c - self.lo for c in range(self.lo, min(self.hi, rcfg.num_attackers))]
            poison_batches_(self.batches, cols, Backdoor(image_size=(spec.image_size, spec.image_size)))
        self.num_examples = [steps * rcfg.batch] * K  # len(client dataset) (run_experiments.py:240)
        self.losses: Optional[torch.Tensor] = None
        self.use_graph = (rcfg.graph and self.device.type == "cuda" and os.environ.get("FLR_GRAPH", "1") != "0")
        self._graph = None
        self._graph_losses: Optional[torch.Tensor] = None
        self._wants_global = "global_flat" in inspect.signature(self.defense.aggregate_flat).parameters
        # training-order rounds (BaseDefense.order_free): the client matrix is in
        # the trainer's coordinate order, written by the last optimizer step;
        # gtrain is the global model in that order (FLR_ORDER=torch: off)
        self.train_order = (getattr(self.defense, "order_free", False) and not self._wants_global
                            and os.environ.get("FLR_ORDER", "train") != "torch")
        bounds = None
        if self.train_order and getattr(self.defense, "needs_tap_blocks", False):
            # the reference-exact distances read the training-order matrix,
            # told which blocks are tap-major (no torch-order copy)
            ok, taps = self._tap_blocks()
            if ok and self.exchange == "alltoall" and world > 1:
                # the chains run through the ranks' coordinate ranges in torch
                # order: rank boundaries moved off the tap-major blocks, so each
                # range holds whole blocks (the same set in either order)
                bounds = aligned_bounds(self.trainer.P, world, taps)
                ok = bounds is not None
            self.train_order = ok
            self.defense.tap_blocks = taps if ok else None
        if mode == "alltoall":
            self.xchg = CoordExchange(K, self.hi - self.lo, self.trainer.P, self.device, Comm(), bounds=bounds)
        else:
            self.full = self.trainer.X if world == 1 else ClientMatrix.empty(K, shapes, self.device)
            if world > 1 and hasattr(self.defense, "comm"):
                # whole rows on every rank: the reference-exact Krum distances
                # split their pair tiles over the ranks (one 8·K² all-reduce)
                self.defense.comm = Comm()
        self.gtrain = self.trainer.to_train_order(self.global_flat) if self.train_order else None
        # FLR_DEFER_DEAD=1 (opt-in): the dead-tap slabs (copies of the global
        # model, 58 % of P at C3) written by a side stream under the Krum chains
        # instead of last in the training phase, the tap rewrite reading them from
        # gtrain meanwhile.  Bit-identical, but the chains slow by more than the
        # fill saves (profiles/r6_dead/): off by default
        # FLR_DEFER_DEAD=2 (default): never written at all — the distances read
        # them from the round's global vector, the Multi-Krum mean too
        # (flr_rows_mean_dead): C3 15.65-15.73 -> 15.94-15.99 rounds/s, the
        # same bits (profiles/r6_dead/); materialize() writes them for any other
        # reader of X; =0: written last in the training phase
        self._fill = None
        self._lazy = None
        self._x_stale = False
        defer = os.environ.get("FLR_DEFER_DEAD", "2")
        if (self.train_order and world == 1 and self.defense.__dict__.get("tap_blocks")
                and getattr(self.defense, "supports_dead_rows", False)
                and hasattr(self.trainer, "fill_dead") and defer in ("1", "2")):
            masks = self._dead_masks(self.defense.tap_blocks)
            if masks is not None and any(masks):
                self.trainer.defer_dead = True
                if defer == "1":
                    self._fill = _DeadFill(self.device, masks)
                else:
                    # the global vector the round trained from (gtrain is overwritten by the publish)
                    self._lazy = (masks, self.trainer.dead_ranges(),
                                  torch.empty(self.trainer.P, dtype=torch.float32, device=self.device))

        self.round_index = 0
        self.fell_back = False
        self.fallback_error: Optional[str] = None   # exception type of the last FedAvg fallback

    def _tap_blocks(self):
        """(ok, blocks): the training-order matrix's tap-major convolution
        weights [(off, Cout, Cin, KK), ...] (flr_pairwise_l2_reference_tap),
        checked once against the trainer's own reorder of a column-index
        vector (float32: exact below 2^24 coordinates; past that, or on any
        mismatch, ok=False: a torch-order round)."""
        from .models.multimodal import param_layout, tap_major_names
        P = self.trainer.P
        if P >= 1 << 24:
            return False, None
        tapn = tap_major_names(self.spec) if self.spec.family != "vit_bert" else frozenset()
        blocks, off = [], 0
        for name, shape in param_layout(self.spec):
            n = 1
            for d in shape:
                n *= int(d)
            if name in tapn:
                blocks.append((off, int(shape[0]), int(shape[1]), int(shape[2]) * int(shape[3])))
            off += n
        want = torch.arange(P, dtype=torch.int64, device=self.device)
        for o, co, ci, kk in blocks:
            u = torch.arange(co * ci * kk, dtype=torch.int64, device=self.device)
            want[o:o + co * ci * kk] = o + ((u % kk) * ci + (u // kk) % ci) * co + u // (ci * kk)
        got = self.trainer.to_torch_order(torch.arange(P, dtype=torch.float32, device=self.device))
        if not torch.equal(got.to(torch.int64), want):
            return False, None
        return True, blocks

    def _dead_masks(self, taps):
        """Per tap block the bitmask of its dead taps (the trainer's dead ranges,
        each a whole tap slab of one block), or None when a range is not (or a
        dead coordinate falls in the last P mod 8, which the distances read
        from X directly)."""
        ranges = self.trainer.dead_ranges()
        P = self.trainer.P
        masks = [0] * len(taps)
        for o, n in ranges:
            if o + n > P - P % 8:
                return None
            for b, (off, co, ci, kk) in enumerate(taps):
                slab = co * ci
                if off <= o and o + n <= off + kk * slab:
                    if (o - off) % slab or n % slab or kk > 64:
                        return None
                    for t in range((o - off) // slab, (o - off + n) // slab):
                        masks[b] |= 1 << t
                    break
            else:
                return None
        return masks

    def materialize(self) -> None:
        """X's dead-tap ranges written (FLR_DEFER_DEAD=2 leaves them out): call
        before reading the client matrix outside the round's own Krum."""
        if self._lazy is not None and self._x_stale:
            self.trainer.fill_dead(self._lazy[2], self._num_flipped())
            self._x_stale = False

    def _join_fill(self) -> None:
        """X whole on the current stream: this round's dead-tap fill launched
        if it is not yet (on the side stream, after the distances' last read
        of X when they marked it, else after everything so far) and waited for.
        Idempotent; a no-op without a pending fill."""
        f = self._fill
        if f is None or f.state == 0:
            return
        main = torch.cuda.current_stream(self.device)
        if f.state == 1:
            if f.mark.recorded:
                f.side.wait_event(f.mark.event)
            else:
                f.side.wait_stream(main)
            with torch.cuda.stream(f.side):
                self.trainer.fill_dead(self.gtrain, self._num_flipped())
                f.done.record(f.side)
        main.wait_event(f.done)
        f.state = 0

    def _num_flipped(self) -> int:
        """Local rows of sign-flip attackers (clients 0..f-1): they submit
        -update, the weights negated as the reference does (model_poisoning.py:
        274-276 via malicious_client.py:103-115) — written negated by the export."""
        f = self.rcfg.num_attackers if self.rcfg.attack == "sign_flip" else 0
        return max(0, min(self.hi, f) - self.lo)

    def _train_phase(self) -> torch.Tensor:
        """Every local client: global -> local SGD steps -> client-matrix rows
        (run_experiments.py:193-240), the attackers' poisoning in the export."""
        if self.train_order:
            self.trainer.load_global_train(self.gtrain)
            return self.trainer.local_update(self.batches, self.masks, negate_rows=self._num_flipped(),
                                             gtrain=self.gtrain)
        self.trainer.load_global(self.global_flat)
        return self.trainer.local_update(self.batches, self.masks, negate_rows=self._num_flipped())

    def _publish(self, agg: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The round's aggregate -> global_flat (torch order; and gtrain when
        training order is on, agg then being in training order)."""
        if self.train_order:
            if agg is not None:
                self.gtrain.copy_(agg)
            self.trainer.to_torch_order(self.gtrain, self.global_flat)
        elif agg is not None:
            self.global_flat.copy_(agg)
        self.round_index += 1
        return self.global_flat

    def _capture(self, keep_graph: bool = False) -> None:
        """Capture the training phase (~2.4k kernel launches per round at C3)
        as one HIP graph: replay removes the host launch cost, which dominates
        once a GPU holds few clients (K/G = 16 at 8 GPUs).  Inputs (global
        vector, batches, masks) and the training state live at fixed addresses,
        so the graph reads the current round's global model on every replay."""
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):  # warm-up on a side stream: library handles and workspaces
            self._train_phase()
        torch.cuda.current_stream(self.device).wait_stream(side)
        g = torch.cuda.CUDAGraph(keep_graph=keep_graph)  # keep_graph: the raw graph stays queryable (tools)
        with torch.cuda.graph(g):
            self._graph_losses = self._train_phase()
        self._graph = g

    def run_round(self) -> torch.Tensor:
        if self.use_graph:
            if self._graph is None:
                self._capture()
            self._graph.replay()
            self.losses = self._graph_losses
        else:
            self.losses = self._train_phase()
        if self._fill is not None:
            # the dead-tap slabs are written by the side stream under the Krum
            # chains (launched by _join_fill before the rows are read); until
            # then the distances read those taps from gtrain (ops.pairwise_l2 dead=)
            f = self._fill
            f.state, f.mark.recorded = 1, False
            self.defense.tap_dead = (f.masks, self.gtrain, self._num_flipped(), f.mark)
            self.defense.before_rows = self._join_fill
        if self._lazy is not None:
            masks, ranges, gprev = self._lazy
            _capi.call("flr_copy_rows", self.gtrain.data_ptr(), self.trainer.P, self.trainer.P, gprev.data_ptr(),
                       self.trainer.P, 1, torch.cuda.current_stream(self.device).cuda_stream)
            nneg = self._num_flipped()
            self._x_stale = True
            self.defense.tap_dead = (masks, gprev, nneg)
            self.defense.rows_dead = (ranges, gprev, nneg)
        try:
            return self._aggregate_phase()
        finally:
            self._join_fill()  # X is whole for every later reader
            if self._fill is not None:
                self.defense.tap_dead = self.defense.before_rows = None
            if self._lazy is not None:
                self.defense.tap_dead = self.defense.rows_dead = None

    def _aggregate_phase(self) -> torch.Tensor:
        kw = {"publish": False} if hasattr(self.defense, "publish") else {}
        self.fell_back = False
        self.fallback_error = None
        if self.exchange == "alltoall":
            self.slice = self.xchg.exchange(self.trainer.X.data)
            try:
                part = self.defense.aggregate_sharded(self.slice, self.num_examples, **kw)
            except Exception as e:  # noqa: BLE001 - the reference catches any exception
                part = self._fallback(e, self.slice.X)
            self._join_fill()  # gtrain is overwritten next: the fill has read it
            self.slice.gather_vector(part, self.gtrain if self.train_order else self.global_flat)
            return self._publish()
        fdist.allgather_rows(self.trainer.X.data, self.full.data)
        if self._wants_global:  # FLTrust: the server update starts from this round's global model
            kw["global_flat"] = self.global_flat.clone()  # global_flat is overwritten below
        try:
            agg = self.defense.aggregate_flat(self.full, self.num_examples, **kw)
        except Exception as e:  # noqa: BLE001
            agg = self._fallback(e, self.full.X)
        self._join_fill()
        return self._publish(agg)

    def _fallback(self, err: Exception, X: torch.Tensor) -> torch.Tensor:
        """robust_server.py:120-122: a failing defense falls back to FedAvg
        (only with RoundConfig.fallback_fedavg; otherwise the error propagates).
        The reference catches every Exception; RoundConfig.fallback_device_errors
        = False keeps device / library failures (kernel launch, workspace, HIP or
        RCCL errors, out of memory) loud instead."""
        from ._capi import FlrError
        self._join_fill()
        self.materialize()
        device_error = isinstance(err, (FlrError, torch.cuda.OutOfMemoryError))
        if not self.rcfg.fallback_fedavg or (device_error and (not self.rcfg.fallback_device_errors
                                                               or self.world > 1)):
            raise err
        logging.getLogger(__name__).error("Defense aggregation failed: %s, falling back to FedAvg", err)
        self.fell_back = True
        self.fallback_error = type(err).__name__
        return ops.fedavg(X, self.num_examples)

    # ---- checkpoint / resume (run_experiments.py:268-279) ----------------------
    def state_dict(self) -> Dict[str, torch.Tensor]:
        """The global model's state_dict: parameters() from the global vector,
        buffers (BatchNorm running statistics) at their initial values — the
        simulation never updates the global model's buffers (:257-259)."""
        m = model_class(self.spec)(self.spec)
        flat = self.global_flat.detach().cpu()
        off = 0
        with torch.no_grad():
            for p in m.parameters():
                n = p.numel()
                p.copy_(flat[off:off + n].view(p.shape))
                off += n
        return m.state_dict()

    def save_checkpoint(self, path: str, accuracy: Optional[float] = None, loss: Optional[float] = None) -> None:
        """torch.save({'round', 'model_state_dict', 'accuracy', 'loss'}) — the
        reference's checkpoint dict (run_experiments.py:273-279)."""
        torch.save({"round": self.round_index, "model_state_dict": self.state_dict(), "accuracy": accuracy,
                    "loss": loss}, path)

    def load_checkpoint(self, path: str) -> int:
        """Resume: the global vector and round index from save_checkpoint's file
        (weights_only load: nothing in the file is executed)."""
        ck = torch.load(path, map_location="cpu", weights_only=True)
        names = [n for n, _ in param_layout(self.spec)]
        sd = ck["model_state_dict"]
        flat = torch.cat([sd[n].reshape(-1).float() for n in names])
        self.global_flat.copy_(flat.to(self.global_flat.device))
        if self.train_order:
            self.gtrain.copy_(self.trainer.to_train_order(self.global_flat))
        self.round_index = int(ck["round"])
        return self.round_index

    # ---- per-round evaluation (run_experiments.py:261-266, 281-291) ------------
    def evaluator(self):
        """The GlobalEvaluator (flr.metrics) of this engine's model, created on
        first use; evaluate the current global model with
        ``eng.evaluator().load(eng.global_flat)`` then ``evaluate_model(...)`` /
        ``attack_success_rate(...)``."""
        if getattr(self, "_evaluator", None) is None:
            from .metrics import GlobalEvaluator
            self._evaluator = GlobalEvaluator(self.spec, self.device, batch_size=self.rcfg.batch)
        return self._evaluator

    def evaluate(self, images, text, labels):
        """evaluate_model(global_model, test_loader) of the reference's round
        loop (run_experiments.py:262) on the current global model."""
        ev = self.evaluator()
        ev.load(self.global_flat)
        return ev.evaluate_model(images, text, labels)
