"""One steady-state round under rocprofv3: 2 warm-up rounds, a marker
(flr krum select on a 5x5 matrix), then the profiled round."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
import torch
from flr import ops
from flr.models.multimodal import ModelSpec
from flr.round import RoundConfig, RoundEngine
from flr.train import TrainConfig
K = int(os.environ.get("K", 128))
eng = RoundEngine(ModelSpec(), RoundConfig(num_clients=K, defense="krum", num_attackers=int(0.2 * K)),
                  TrainConfig(local_steps=5), "cuda")
for _ in range(2):
    eng.run_round()
torch.cuda.synchronize()
ops.median_lower(torch.rand(5, 64, device="cuda"))  # marker (orderstat_kernel)
torch.cuda.synchronize()
eng.run_round()
torch.cuda.synchronize()
print("profiled round done")
