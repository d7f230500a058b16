import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
import torch
from flr import ops
from flr.workload import update_matrix
K = int(os.environ.get("K", 128)); P = int(os.environ.get("P", 10_000_000))
X = update_matrix(K, P, f=K // 5, device="cuda")[:, :P]
for _ in range(10):
    D = ops.pairwise_l2(X, "gram")
torch.cuda.synchronize()
print("done", D[0, 1].item())
