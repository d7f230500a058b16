"""ORACLE (test infrastructure only) — the reference's local-training loop on CPU.

Restates experiments/run_experiments.py:195-240 (the fp32 CPU branch
:230-235) and the loss averaging of src/client/fl_client.py:129-149, for one
client at a time, on flr's MultimodalNet (the reference has no ResNet-18+GRU
model; its fusion-head structure is cub200_cnn.py:88-93).  Two deviations are
required for a deterministic comparison and are made explicit: fixed batches
instead of a shuffling DataLoader, and dropout applied through an explicit mask
(or p = 0) instead of torch's RNG stream.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


class _MaskDropout(nn.Module):
    def __init__(self):
        super().__init__()
        self.mask = None

    def forward(self, x):
        return x if self.mask is None else x * self.mask


def _mask_dropouts(model: nn.Module) -> List[_MaskDropout]:
    """Replace every nn.Dropout of the model (an attribute or a Sequential
    entry) by a module that applies an explicit mask."""
    out = []
    for mod in list(model.modules()):
        for cname, child in list(mod.named_children()):
            if isinstance(child, nn.Dropout):
                md = _MaskDropout()
                setattr(mod, cname, md)
                out.append(md)
    return out


class _TiedRelu(torch.autograd.Function):
    """F.relu with some gate decisions given instead of computed (m: the gate
    mask, (x > 0) except at the tie positions).  Forward where(m, x, 0),
    backward where(m, g, 0): torch's relu / threshold_backward wherever m is
    (x > 0)."""

    @staticmethod
    def forward(ctx, x, m):
        ctx.save_for_backward(m)
        return torch.where(m, x, torch.zeros((), dtype=x.dtype))

    @staticmethod
    def backward(ctx, g):
        (m,) = ctx.saved_tensors
        return torch.where(m, g, torch.zeros((), dtype=g.dtype)), None


@contextlib.contextmanager
def _relu_hooks(override: Optional[Dict[int, Tuple[torch.Tensor, torch.Tensor]]] = None,
                record: Optional[List[torch.Tensor]] = None):
    """Within the block, the n-th F.relu call of a forward (counted from 0 per
    forward: reset the counter list between forwards) takes the gate decisions
    override[n] = (flat element indices, decisions) at those elements; record,
    if given, collects every ReLU input."""
    if not override and record is None:
        yield [0]
        return
    orig = F.relu
    count = [0]

    def relu(x, *a, **kw):
        n = count[0]
        count[0] += 1
        if record is not None:
            record.append(x.detach().clone())
        if override and n in override:
            idx, on = override[n]
            m = (x > 0).reshape(-1).clone()
            m[idx] = on
            return _TiedRelu.apply(x, m.view_as(x))
        return orig(x, *a, **kw)

    F.relu = relu
    try:
        yield count
    finally:
        F.relu = orig


def relu_inputs(model_cls, spec, params_flat: torch.Tensor, images: torch.Tensor, tokens: torch.Tensor,
                dtype: torch.dtype = torch.float32) -> List[torch.Tensor]:
    """Every ReLU input of one train-mode forward of the reference model (the
    fp32 reference, or fp64 as the yardstick) from the flat parameters, in call
    order.  Test infrastructure: the gate-tie check of tests/parity.py."""
    model = model_cls(spec).to(dtype)
    off = 0
    with torch.no_grad():
        for p in model.parameters():
            p.copy_(params_flat[off:off + p.numel()].view(p.shape).to(dtype))
            off += p.numel()
    model.train()
    rec: List[torch.Tensor] = []
    with torch.no_grad(), _relu_hooks(record=rec):
        model(images.to(dtype), tokens)
    return rec


def local_update(model_cls, spec, global_flat: torch.Tensor, batches: Sequence, lr: float = 0.01,
                 momentum: float = 0.9, weight_decay: float = 0.0, max_norm: float = 1.0,
                 masks: Optional[Sequence[torch.Tensor]] = None, threads: Optional[int] = None,
                 dtype: torch.dtype = torch.float32, start_params: Optional[torch.Tensor] = None,
                 start_momentum: Optional[Sequence[torch.Tensor]] = None, return_momentum: bool = False,
                 relu_ties: Optional[Dict[int, Tuple[torch.Tensor, torch.Tensor]]] = None):
    """One client's local update.  Returns (params after training, mean loss).
    dtype=torch.float64 runs the same loop in double precision: not the
    reference (which trains in fp32), but the yardstick of how far the
    reference's own fp32 result is from exact (tests/parity.py
    check_conditioned).  start_params / start_momentum: continue a local
    update from another trainer's state (flat parameters, per-parameter
    momentum buffers) instead of the global model — one step of the reference
    from the GPU's own state; return_momentum: also return the buffers.
    relu_ties: {ReLU call index: (flat element indices, decisions)} — gate
    decisions given instead of computed at those elements of that ReLU's input
    (one batch only): the gate ties of tests/parity.py gate_ties, where the
    fp64 pre-activation lies inside the fp32 rounding band of zero and the
    engine's fp32 sums decided the other way.  Every other element, and every
    arithmetic operation, is the reference's."""
    if threads:
        torch.set_num_threads(threads)
    model = model_cls(spec).to(dtype)
    off = 0
    with torch.no_grad():
        for p in model.parameters():  # load_state_dict(global) for parameters() (:203)
            n = p.numel()
            src = global_flat if start_params is None else start_params
            p.copy_(src[off:off + n].view(p.shape).to(dtype))
            off += n
    drops = _mask_dropouts(model)
    optimizer = torch.optim.SGD(model.parameters(), lr=lr, momentum=momentum, weight_decay=weight_decay)  # :206-211
    if start_momentum is not None:
        for p, buf in zip(model.parameters(), start_momentum):
            optimizer.state[p]["momentum_buffer"] = buf.detach().clone().to(dtype)
    criterion = nn.CrossEntropyLoss()
    model.train()
    losses = []
    if relu_ties and len(batches) != 1:
        raise ValueError("relu_ties describe one forward: give one batch")
    for s, (images, tokens, labels) in enumerate(batches):
        for d in drops:
            d.mask = None if masks is None else masks[s]
        if dtype != torch.float32:
            images = images.to(dtype)
            for d in drops:
                d.mask = None if d.mask is None else d.mask.to(dtype)
        optimizer.zero_grad()
        with _relu_hooks(relu_ties):
            outputs = model(images, tokens)
            loss = criterion(outputs, labels)
            loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=max_norm)  # :234
        optimizer.step()
        losses.append(loss.item())
    update = [p.data.clone() for p in model.parameters()]  # :238
    if return_momentum:
        return update, sum(losses) / len(losses), [optimizer.state[p]["momentum_buffer"].clone()
                                                   for p in model.parameters()]
    return update, sum(losses) / len(losses)


def fl_client_train(model_cls, spec, global_flat: torch.Tensor, batches: Sequence, learning_rate: float = 0.01,
                    masks: Optional[Sequence[torch.Tensor]] = None) -> Tuple[List[torch.Tensor], float]:
    """FLClient._train (src/client/fl_client.py:109-149): SGD(lr, momentum=0.9),
    no weight decay and NO gradient clipping (only the simulation loop clips,
    run_experiments.py:234); loss = sum of batch losses / number of batches.
    clip_grad_norm_ with max_norm = inf scales by exactly 1, i.e. no clip."""
    return local_update(model_cls, spec, global_flat, batches, lr=learning_rate, momentum=0.9, weight_decay=0.0,
                        max_norm=float("inf"), masks=masks)
