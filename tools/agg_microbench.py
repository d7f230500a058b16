"""Quick timing of the aggregation kernels at the C3 shape (K=128, P=1e7)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
import torch
from flr import ops
from flr.workload import update_matrix

K = int(os.environ.get("K", 128)); P = int(os.environ.get("P", 10_000_000)); f = K // 5
X = update_matrix(K, P, f=f, device="cuda")[:, :P]
torch.cuda.synchronize()
def timeit(fn, n=10):
    fn(); torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n
gb = 4 * K * P / 1e9
for name, fn in [("pairwise_gram", lambda: ops.pairwise_l2(X, "gram")),
                 ("pairwise_direct", lambda: ops.pairwise_l2(X, "direct")),
                 ("fedavg", lambda: ops.fedavg(X, [1] * K)),
                 ("rows_mean64", lambda: ops.rows_mean(X, torch.arange(64, dtype=torch.int32))),
                 ("median", lambda: ops.median_lower(X)),
                 ("trimmed", lambda: ops.trimmed_mean(X, max(1, int(0.1 * K))))]:
    n = 3 if name == "pairwise_direct" else 10
    ms = timeit(fn, n)
    byt = gb * (0.5 if name == "rows_mean64" else 1.0)
    print(f"{name:16s} {ms:8.3f} ms  {byt/ms*1e3:8.1f} GB/s", flush=True)
D = ops.pairwise_l2(X, "gram"); D2 = ops.pairwise_l2(X, "direct")
print("gram vs direct max rel", ((D - D2).abs() / D2.clamp_min(1e-30)).max().item())
s, o = ops.krum_select(D, f)
print("selected attackers:", sorted(set(o[:K//2].tolist()) & set(range(f))))
for K2 in (256, 512):
    P2 = 2_000_000
    X2 = update_matrix(K2, P2, f=K2 // 5, device="cuda")[:, :P2]
    for name, fn in [("median", lambda: ops.median_lower(X2)), ("trimmed", lambda: ops.trimmed_mean(X2, int(0.1 * K2))),
                     ("pairwise", lambda: ops.pairwise_l2(X2))]:
        ms = timeit(fn, 5)
        print(f"K={K2} {name:10s} {ms:8.3f} ms  {4*K2*P2/1e9/ms*1e3:8.1f} GB/s", flush=True)
