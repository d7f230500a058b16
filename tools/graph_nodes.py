"""Diagnostic: node count of a round's captured training-phase HIP graph
(RoundEngine._capture) for a BASELINE config preset and client count.
Usage: python tools/graph_nodes.py C4 256"""
import ctypes
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


def main():
    cfg, K = sys.argv[1], int(sys.argv[2])
    model, _, defense, dcfg, attack, afrac = bench.PRESETS[cfg]
    spec = {"cub": CUB, "vit_bert": VIT_BERT}.get(model, ModelSpec())
    rc = RoundConfig(num_clients=K, defense=defense, defense_cfg=dict(dcfg), num_attackers=int(afrac * K),
                     attack=attack)
    eng = RoundEngine(spec, rc, TrainConfig(local_steps=5), torch.device("cuda:0"))
    eng._capture(keep_graph=True)
    hip = ctypes.CDLL("libamdhip64.so.7")
    n = ctypes.c_size_t(0)
    st = hip.hipGraphGetNodes(ctypes.c_void_p(eng._graph.raw_cuda_graph()), None, ctypes.byref(n))
    nodes = (ctypes.c_void_p * n.value)()
    st2 = hip.hipGraphGetNodes(ctypes.c_void_p(eng._graph.raw_cuda_graph()), nodes, ctypes.byref(n))
    kinds = {}
    for i in range(n.value):
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t))
        kinds[t.value] = kinds.get(t.value, 0) + 1
    # hipGraphNodeType: 0 kernel, 1 memcpy, 2 memset, 3 host, 4 graph, 5 empty, 6 wait event, 7 event record
    print(f"{cfg} K={K}: graph nodes {n.value} (status {st}/{st2}) by type {kinds}", flush=True)
    eng._graph.instantiate()
    eng.run_round()
    torch.cuda.synchronize()
    print(f"{cfg} K={K}: replay ok", flush=True)


if __name__ == "__main__":
    main()
