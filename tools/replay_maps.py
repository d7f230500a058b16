"""Diagnostic: capture a round's training-phase HIP graph,
write this process's /proc/self/maps next to the run's log, then replay it.
Run under `rocprofv3 --kernel-trace`: the native frames of a crash inside the
replay can then be mapped onto the libraries that hold them (same process,
same address space).  Usage: python tools/replay_maps.py C4 256 OUT.maps"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from flr.models.multimodal import CUB, VIT_BERT, ModelSpec  # noqa: E402
from flr.round import RoundConfig, RoundEngine  # noqa: E402
from flr.train import TrainConfig  # noqa: E402


def bench_mode(out, argv):
    """bench.py itself (runpy), with /proc/self/maps written before every round."""
    import runpy
    orig = RoundEngine.run_round

    def run_round(self):
        with open("/proc/self/maps") as src, open(out, "w") as dst:
            dst.write(src.read())
        print("round", flush=True)
        return orig(self)

    RoundEngine.run_round = run_round
    sys.argv = [os.path.join(ROOT, "bench.py"), *argv]
    runpy.run_path(sys.argv[0], run_name="__main__")


def main():
    if sys.argv[1] == "bench":
        return bench_mode(sys.argv[2], sys.argv[3:])
    cfg, K, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    model, _, defense, dcfg, attack, afrac = bench.PRESETS[cfg]
    spec = {"cub": CUB, "vit_bert": VIT_BERT}.get(model, ModelSpec())
    rc = RoundConfig(num_clients=K, defense=defense, defense_cfg=dict(dcfg), num_attackers=int(afrac * K),
                     attack=attack)
    eng = RoundEngine(spec, rc, TrainConfig(local_steps=5), torch.device("cuda:0"))
    eng._capture()
    torch.cuda.synchronize()
    with open("/proc/self/maps") as src, open(out, "w") as dst:
        dst.write(src.read())
    print(f"{cfg} K={K}: captured, maps written; replaying", flush=True)
    mode = sys.argv[4] if len(sys.argv) > 4 else "replay"
    for i in range(3):  # the bench crashed on its second replay
        if mode == "round":
            eng.run_round()  # replay + aggregation + write-back, as bench.py
        else:
            eng._graph.replay()
        torch.cuda.synchronize()
        print(f"{cfg} K={K}: replay {i} ok", flush=True)


if __name__ == "__main__":
    main()
