"""Time one round of local training (K clients x 5 steps) under variants."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
import torch
if os.environ.get("BENCHMARK") == "1":
    torch.backends.cudnn.benchmark = True
from flr.models.multimodal import ModelSpec
from flr.round import initial_global
from flr.train import ClientBatchTrainer, TrainConfig, make_dropout_masks, synthetic_batches
K = int(os.environ.get("K", 128))
spec = ModelSpec()
tr = ClientBatchTrainer(spec, K, "cuda", TrainConfig(local_steps=5))
g = initial_global(spec, 42, "cuda")
b = synthetic_batches(spec, 5, range(K), 32, "cuda")
m = make_dropout_masks(spec, 5, K, 32, "cuda", 1)
for _ in range(2):
    tr.load_global(g); tr.local_update(b, m)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    tr.load_global(g); tr.local_update(b, m)
torch.cuda.synchronize()
print(os.environ.get("TAG", "base"), f"{(time.perf_counter()-t0)/3*1e3:.1f} ms/round", flush=True)
