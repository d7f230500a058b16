"""Aggregation at the C4 / C5 shapes (BASELINE.json configs[3], [4]): the
client-matrix kernels on synthetic update matrices of the named size.
C4: trimmed mean, K = 256, P = 3.3e7 (ViT-S + BERT-mini), t = 25 (ratio 0.1);
C5: Krum (f = 102, multi_k = 256) + trimmed mean (t = 51, ratio 0.1) + median,
K = 512, P = 3.3e7.  Prints one JSON line per kernel (ms, GB/s, fraction of
8 TB/s) to stdout and gpurun_out/agg_c4c5.jsonl."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
import torch  # noqa: E402

from flr import ops  # noqa: E402
from flr.workload import update_matrix  # noqa: E402

P = int(os.environ.get("P", 33_000_000))


def timeit(fn, n=3):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = open(os.path.join(ROOT, "gpurun_out", "agg_c4c5.jsonl"), "w")
    for cfg, K in (("C4", 256), ("C5", 512)):
        X = update_matrix(K, P, f=int(0.2 * K), seed=K, device="cuda")[:, :P]
        t = int(0.1 * K)
        runs = [("trimmed_mean", lambda: ops.trimmed_mean(X, t), 4.0 * K * P + 4.0 * P),
                ("median", lambda: ops.median_lower(X), 4.0 * K * P + 4.0 * P)]
        if cfg == "C5":  # the C5 defense's second half: the trimmed mean of the 256 Multi-Krum rows
            rows = torch.randperm(K, generator=torch.Generator().manual_seed(5))[: K // 2].to(torch.int32).cuda()
            runs.append(("trimmed_mean_rows256", lambda: ops.trimmed_mean(X, int(0.1 * (K // 2)), rows=rows),
                         4.0 * (K // 2) * P + 4.0 * P))
        if cfg == "C5" or os.environ.get("GRAM_ALL"):
            runs.append(("krum_pairwise_gram", lambda: ops.pairwise_l2(X, "gram"), 4.0 * K * P + 8.0 * K * K))
        for name, fn, byts in runs:
            ms = timeit(fn)
            rec = {"config": cfg, "K": K, "P": P, "kernel": name, "ms": ms, "GBps": byts / ms / 1e6,
                   "frac_of_8TBps": byts / ms / 1e6 / 8000.0}
            print(json.dumps(rec), flush=True)
            print(json.dumps(rec), file=out, flush=True)
        if cfg == "C5":
            D = ops.pairwise_l2(X, "gram")
            _, order = ops.krum_select(D, int(0.2 * K))
            sel = set(order[: K // 2].tolist())
            print(json.dumps({"config": cfg, "attackers_selected": len(sel & set(range(int(0.2 * K))))}), file=out,
                  flush=True)
        del X
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
