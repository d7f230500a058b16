"""Bit-identity of library builds: one seeded round of the ResNet+GRU model (C3
shapes, K clients) and one of the ViT-S + BERT-mini model (C4 shapes, 2 clients
of 1 step), printing the sha256 of the client matrix X and the new global vector.
Run once per FLR_LIB and compare the lines (tools/archive/gpu_r3_y.sh).
usage: FLR_LIB=... python tools/lib_identity.py"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multimodal-fl-security_amd"))
import torch
from flr.models.multimodal import VIT_BERT, ModelSpec
from flr.round import RoundConfig, RoundEngine
from flr.train import TrainConfig


def sha(t: torch.Tensor) -> str:
    return hashlib.sha256(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()[:16]


def main():
    dev = torch.device("cuda")
    K = int(os.environ.get("K", 16))
    eng = RoundEngine(ModelSpec(), RoundConfig(num_clients=K, num_attackers=K // 5),
                      TrainConfig(local_steps=5), dev)
    g = eng.run_round()
    torch.cuda.synchronize()
    print("c3", "X", sha(eng.trainer.X.data), "global", sha(g), flush=True)
    eng = RoundEngine(VIT_BERT, RoundConfig(num_clients=2, batch=8, num_attackers=0, attack="none", defense="fedavg"),
                      TrainConfig(local_steps=1), dev)
    g = eng.run_round()
    torch.cuda.synchronize()
    print("c4", "X", sha(eng.trainer.X.data), "global", sha(g), flush=True)


if __name__ == "__main__":
    main()
