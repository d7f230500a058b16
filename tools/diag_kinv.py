"""Is client-batched training invariant to how clients are grouped into a launch?
Trains clients 0..7 as one batch of 8 and as two batches of 4 (0..3, 4..7), eager
and inside a captured HIP graph (as RoundEngine runs it), and compares rows.
Writes gpurun_out/diag_kinv.log."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
import torch  # noqa: E402

from flr.models.multimodal import TINY, ModelSpec, param_layout  # noqa: E402
from flr.round import initial_global  # noqa: E402
from flr.train import ClientBatchTrainer, TrainConfig, make_dropout_masks, synthetic_batches  # noqa: E402


def train(spec, ids, g, graph):
    tr = ClientBatchTrainer(spec, len(ids), "cuda", TrainConfig(local_steps=2))
    b = synthetic_batches(spec, 2, ids, 4, "cuda")
    m = make_dropout_masks(spec, 2, ids, 4, "cuda", seed=5)

    def phase():
        tr.load_global(g)
        return tr.local_update(b, m)
    if graph:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            phase()
        torch.cuda.current_stream().wait_stream(side)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            loss = phase()
        gr.replay()
    else:
        loss = phase()
    torch.cuda.synchronize()
    return tr.X.X.clone(), loss.clone()


def main():
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = open(os.path.join(ROOT, "gpurun_out", "diag_kinv.log"), "w")
    for spec, name in ((TINY, "tiny"), (ModelSpec(), "resnet18")):
        g = initial_global(spec, 42, "cuda")
        for graph in (False, True):
            X8, l8 = train(spec, list(range(8)), g, graph)
            Xa, la = train(spec, list(range(4)), g, graph)
            Xb, lb = train(spec, list(range(4, 8)), g, graph)
            X4 = torch.cat([Xa, Xb])
            d = (X8 - X4).abs().max(dim=1).values
            print(name, "graph" if graph else "eager", "per-client max|X8-X4|:", d.tolist(),
                  "loss diff", (l8 - torch.cat([la, lb])).abs().max().item(), file=out, flush=True)
            if d.max() > 0:
                k = int(d.argmax())
                diff = (X8[k] - X4[k]).abs()
                off = 0
                for n, s in param_layout(spec):
                    c = int(torch.Size(s).numel())
                    v = diff[off:off + c].max().item()
                    if v > 0:
                        print("   client", k, n, v, file=out, flush=True)
                    off += c
    print("done", file=out, flush=True)


if __name__ == "__main__":
    main()
