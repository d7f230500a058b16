"""In-process A/B of whole C3 rounds under kernel env switches: one RoundEngine
(and one captured HIP graph) per variant, replays interleaved, median ms.
usage: round_ab.py "A=1" "B=2,C=3" ...  (the first variant is the baseline {})"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multimodal-fl-security_amd"))
import torch
from flr.models.multimodal import ModelSpec
from flr.round import RoundConfig, RoundEngine
from flr.train import TrainConfig


def main():
    variants = [{}] + [dict(kv.split("=") for kv in a.split(",") if kv) for a in sys.argv[1:]]
    K = int(os.environ.get("K", 128))
    engines = []
    for var in variants:
        old = {k: os.environ.get(k) for k in var}
        os.environ.update(var)
        eng = RoundEngine(ModelSpec(), RoundConfig(num_clients=K, num_attackers=int(0.2 * K)),
                          TrainConfig(local_steps=5), torch.device("cuda"))
        eng.run_round()  # capture under this variant's env
        torch.cuda.synchronize()
        for k, v in old.items():
            os.environ.pop(k, None) if v is None else os.environ.__setitem__(k, v)
        engines.append(eng)
    times = [[] for _ in variants]
    for it in range(8):
        for i, eng in enumerate(engines):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng._graph.replay()
            torch.cuda.synchronize()
            times[i].append((time.perf_counter() - t0) * 1e3)
    for var, t in zip(variants, times):
        t = sorted(t)
        print(f"{str(var):40s} train phase median {t[len(t) // 2]:.2f} ms (min {t[0]:.2f})", flush=True)


if __name__ == "__main__":
    main()
