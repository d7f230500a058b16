"""Which pairs differ (K = 33, P = 2053): tile kind and super-blocks."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "multimodal-fl-security_amd")]
import numpy as np, torch
from oracle import normref
from flr import ops
from flr.matrix import padded_ld
for K, P in [(33, 2053), (33, 4099), (64, 2053), (40, 8200)]:
    g = torch.Generator().manual_seed(K * 1000 + P)
    X = torch.randn(K, P, generator=g) * 0.05
    data = torch.zeros((K, padded_ld(P)), dtype=torch.float32)
    data[:, :P] = X
    D = ops.pairwise_l2(data.cuda()[:, :P], "reference").cpu().numpy()
    want = normref.distance_matrix(X.numpy())
    bad = np.argwhere(D != want)
    bad = [(int(i), int(j)) for i, j in bad if i < j]
    kinds = {}
    for i, j in bad:
        key = "diag" if i // 32 == j // 32 else "off"
        kinds[key] = kinds.get(key, 0) + 1
    print(K, P, "bad pairs", len(bad), kinds, bad[:8])
