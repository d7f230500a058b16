"""Krum Gram pairwise timing at the BASELINE shapes: C3 (K = 128, P = 11.8M),
C4 (K = 256, P = 3.3e7), C5 (K = 512, P = 3.3e7).  One line per shape: ms per
call (HIP events, 3 calls after a warm-up), GB/s of the 4*K*P algorithmic bytes
and the fraction of 8 TB/s.  SHAPES="K:P,..." overrides."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
import torch  # noqa: E402

from flr import ops  # noqa: E402
from flr.workload import update_matrix  # noqa: E402

shapes = [(128, 11_800_394), (256, 33_000_000), (512, 33_000_000)]
if os.environ.get("SHAPES"):
    shapes = [tuple(int(v) for v in s.split(":")) for s in os.environ["SHAPES"].split(",")]
for K, P in shapes:
    X = update_matrix(K, P, f=K // 5, seed=K, device="cuda")[:, :P]
    ops.pairwise_l2(X, "gram")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        ops.pairwise_l2(X, "gram")
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    gbs = 4.0 * K * P / (ms * 1e-3) / 1e9
    print(json.dumps({"K": K, "P": P, "ms": round(ms, 3), "GB/s": round(gbs, 1), "frac_8TBs": round(gbs / 8000, 3)}),
          flush=True)
    del X
    torch.cuda.empty_cache()
