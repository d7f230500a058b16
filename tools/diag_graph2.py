"""Replays of the captured training phase after replay 1 differ from eager (TINY):
which state carries over?  Writes gpurun_out/diag_graph2.log."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
import torch  # noqa: E402

from flr.models.multimodal import TINY  # noqa: E402
from flr.round import initial_global  # noqa: E402
from flr.train import ClientBatchTrainer, TrainConfig, make_dropout_masks, synthetic_batches  # noqa: E402


def main():
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = open(os.path.join(ROOT, "gpurun_out", "diag_graph2.log"), "w")
    spec, ids = TINY, list(range(8))
    g = initial_global(spec, 42, "cuda")
    tr = ClientBatchTrainer(spec, len(ids), "cuda", TrainConfig(local_steps=2))
    b = synthetic_batches(spec, 2, ids, 4, "cuda")
    bsave = [tuple(t.clone() for t in s) for s in b]
    m = make_dropout_masks(spec, 2, ids, 4, "cuda", seed=5)

    def phase():
        tr.load_global(g)
        return tr.local_update(b, m)

    def cmp(tag, ref):
        torch.cuda.synchronize()
        d = (tr.X.X - ref).abs().max().item()
        bd = max((a - c).abs().max().item() for s, s0 in zip(b, bsave) for a, c in zip(s, s0))
        print(f"{tag:40s} |X - ref| {d:.3e}  batches changed by {bd:.3e}", file=out, flush=True)

    phase()
    torch.cuda.synchronize()
    ref = tr.X.X.clone()
    phase()
    cmp("eager run 2", ref)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        phase()
    torch.cuda.current_stream().wait_stream(side)
    cmp("side-stream warm-up", ref)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        phase()
    gr.replay()
    cmp("replay 1", ref)
    gr.replay()
    cmp("replay 2", ref)
    tr._wbuf.fill_(float("nan"))
    tr._mbuf.fill_(float("nan"))
    gr.replay()
    cmp("replay 3 after W, M := NaN", ref)
    for n, w, mm in zip(tr.names, tr.W, tr.Mb):
        nw, nm = int(torch.isnan(w).sum()), int(torch.isnan(mm).sum())
        if nw or nm:
            print(f"   {n}: NaN in W {nw}/{w.numel()}, in M {nm}/{mm.numel()}", file=out, flush=True)
    for s, s0 in zip(b, bsave):
        for a, c in zip(s, s0):
            a.copy_(c)
    gr.replay()
    cmp("replay 4 after restoring batches", ref)
    phase()
    cmp("eager after replays", ref)
    print("done", file=out, flush=True)


if __name__ == "__main__":
    main()
