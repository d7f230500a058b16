"""Diagnostic: Gram-path distance error vs the pair's cancellation factor."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
import torch, numpy as np
from flr import ops
from flr.workload import update_matrix

for P in [129, 1111, 4096, 65536, 1_000_000]:
    for K, f in [(64, 12), (128, 25)]:
        X = update_matrix(K, P, f=f, seed=P + K, device="cuda")[:, :P]
        D = ops.pairwise_l2(X, "gram").double()
        Xd = X.double()
        ex = torch.cdist(Xd, Xd)
        rel = ((D - ex).abs() / ex.clamp_min(1e-30)).fill_diagonal_(0).cpu().numpy()
        att = np.zeros(K, bool); att[:f] = True
        aa = rel[np.ix_(att, att)].max(); bb = rel[np.ix_(~att, ~att)].max(); ab = rel[np.ix_(att, ~att)].max()
        print(f"P={P:8d} K={K:3d} terms={os.environ.get('FLR_GRAM_TERMS','2')}  benign-benign {bb:.2e}  att-att {aa:.2e}  att-benign {ab:.2e}", flush=True)
