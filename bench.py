#!/usr/bin/env python3
"""bench.py — FL rounds/sec + aggregate-ms (BASELINE.json metric).

Workload (BASELINE.json configs[2], "C3"): K = 128 clients, ResNet-18 image +
1-layer GRU text late-fusion model (P = 11,800,394 fp32 parameters), 5 local
SGD steps per client per round (batch 32, lr 0.01, momentum 0.9, clip 1.0),
20 % sign-flip attackers (f = 25), Multi-Krum aggregation (multi_k = 64).
One "step" = one full round: every client's local update + the exchange
(N > 1: one all-to-all of client rows -> coordinate ranges, flr.shard) +
Krum (pairwise distances, scores, selection, mean of each GPU's range) + the
all-gather of the aggregated vector (global write-back).  Synthetic inputs
are generated on the device before timing.

N = 1: python bench.py [--steps K --warmup W]
N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
  or   python bench.py --gpus N: with no torchrun environment (WORLD_SIZE
       unset) the process starts the N ranks itself — a fresh
       `python -m torch.distributed.run` child, before anything touches the
       GPU — relays their output and exits with their status.
Every rank checks that the process group's world size equals --gpus.
Clients shard over ranks (K/N each), so the total work per round is fixed
and the scaling is "strong".  Rank 0 prints one JSON line.
--exchange allgather selects the whole-matrix all-gather instead.
--backend gloo: the N-rank rehearsal on one GPU (collectives staged through
the host; every rank on cuda:(local_rank mod device count)).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "multimodal-fl-security_amd"))

METRIC = "FL rounds/sec + aggregate-ms, K=128 clients 10M-param multimodal, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# fp32 VALU issue peak in lane-operations/s: 256 CUs x 4 SIMD-32 x 32 lanes per cycle
# x 2.4 GHz (MI355X_MICROARCH.md: v_fma_f32 / v_add_f32 2 cycles per wave64 on a SIMD)
VALU_PEAK_OPS = 256 * 4 * 32 * 2.4e9

# The global model's sha256 after (warmup + steps) rounds of an unmodified
# preset, from a committed run of THIS library (the rounds are deterministic
# and bit-identical at every GPU count): (preset, pairwise method, rounds) ->
# sha.  bench prints sha_matches_reference_run against it (None: no entry).
REFERENCE_SHA = {}
_SHA_FILE = os.path.join(ROOT, "profiles", "reference_sha.json")
if os.path.exists(_SHA_FILE):
    REFERENCE_SHA = {tuple(k.split("|")[:2]) + (int(k.split("|")[2]),): v
                     for k, v in json.load(open(_SHA_FILE)).items() if not k.startswith("_")}


def gram_traffic(K: int, P: int):
    """HBM bytes per launch of the Gram kernel from the committed rocprofv3 PMC
    passes (profiles/gram_traffic.json: FETCH_SIZE and WRITE_SIZE in KiB per
    dispatch, separate passes, FETCH_SIZE doubled per MI355X_MICROARCH.md's
    gfx950 correction for wide streaming reads); None unless measured at this
    exact shape."""
    path = os.path.join(ROOT, "profiles", "gram_traffic.json")
    if not os.path.exists(path):
        return None
    t = json.load(open(path))
    if t.get("K") != K or t.get("P") != P:
        return None
    return (2.0 * t["fetch_kib"] + t["write_kib"]) * 1024.0


def ref_traffic(K: int, P: int):
    """HBM bytes of one reference-exact distance call (the transposes, the tap
    rewrite, the chains and the finish) from the committed rocprofv3 PMC
    passes (profiles/r6_ref/ref_traffic.json: FETCH_SIZE and WRITE_SIZE in KiB
    per call, separate passes, FETCH_SIZE doubled per MI355X_MICROARCH.md's
    gfx950 correction for 16-B-per-lane reads); None unless measured at this
    exact shape."""
    path = os.path.join(ROOT, "profiles", "r6_ref", "ref_traffic.json")
    if not os.path.exists(path):
        return None
    t = json.load(open(path))
    if t.get("K") != K or t.get("P") != P:
        return None
    return (2.0 * t["fetch_kib_per_call"] + t["write_kib_per_call"]) * 1024.0


COMMITTED_C3_STATS = "profiles/r6_prof/c3_kernel_stats_serial.txt"  # FLR_TEXT_STREAM=0 FLR_WGRAD_STREAM=0: per-kernel durations with nothing beside them
# the C4 bench's rocprofv3 summary (gemm_mfma_from_profile of an unmodified C4 line)
COMMITTED_C4_STATS = "profiles/r3_c4_kernel_stats.txt"


def _kernel_rows(path: str):
    """(name, calls, total ms) per kernel from a rocprofv3 --stats summary: the
    kernel_stats.csv it writes, or the fixed-width text summary committed under
    profiles/ (name in the first 90 columns)."""
    import csv
    import re
    if path.endswith(".csv"):
        with open(path) as fh:
            for r in csv.DictReader(fh):
                yield r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) * 1e-6
        return
    for line in open(path).read().splitlines()[2:]:
        m = re.match(r"(.{90})\s+(\d+)\s+([\d.]+)", line)
        if m:
            yield m.group(1), int(m.group(2)), float(m.group(3))


def conv_utilisation(spec, K: int, batch: int, steps: int, stats_path=None,
                     rounds_in_profile_key: str = "::ce_kernel("):
    """Convolution MFMA utilisation of the headline config from a rocprofv3
    summary of the C3 bench (NOT this run's kernels: the profiler wraps a
    separate bench run; --kernel-stats names it, else the newest committed
    summary): the round's useful conv FLOPs (fwd + dgrad + wgrad over the live
    taps; the stem has no dgrad) over the conv kernels' summed time per round,
    against the bf16x6 form's ceiling (2.5 PF/s dense bf16 / 6 products).
    None when the profile is absent or the spec has no convolutions."""
    from flr.models.multimodal import conv_geometry, live_taps, param_layout
    path = stats_path or os.path.join(ROOT, COMMITTED_C3_STATS)
    if not os.path.exists(path):
        path = os.path.join(ROOT, "profiles", "r2_c3_kernel_stats_final.txt")
    geo = conv_geometry(spec)
    if not geo or not os.path.exists(path):
        return None
    shapes = dict(param_layout(spec))
    flops = 0.0
    for name, (H, k, st, pd, Ho) in geo.items():
        cout, cin = shapes[name][0], shapes[name][1]
        f = 2.0 * batch * Ho * Ho * cout * cin * len(live_taps(H, k, st, pd))
        flops += f * (2 if name == "conv1.weight" else 3)
    flops *= K * steps
    conv_ms = sgd_calls = 0.0
    for name, calls, ms in _kernel_rows(path):
        if rounds_in_profile_key in name:
            sgd_calls += calls
        if "convt::" in name and any(t in name for t in ("FwdT", "DgradT", "WgtT")) or "stem::" in name \
                or "zero_taps" in name:
            conv_ms += ms
    if not sgd_calls or not conv_ms:
        return None
    rounds = sgd_calls / steps
    per_round = conv_ms / rounds
    achieved = flops / (per_round * 1e-3) / 1e12
    peak = 2500.0 / 6.0
    return {"source": os.path.relpath(path, ROOT), "measured_in_this_run": False,
            "flops_per_round": flops, "kernel_ms_per_round": per_round,
            "achieved_tflops": achieved, "peak_tflops": peak, "frac": achieved / peak,
            "peak_note": "bf16x6 form: 6 v_mfma_f32_32x32x16_bf16 products per fp32 product, 2.5 PF/s dense bf16"}


def cpu_model() -> str:
    """`lscpu` model name (from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def round_roofline(K: int, P: int, P_live: int, steps: int, ms_per_round: float, world: int):
    """SURVEY §8(d) round bytes: each client-step of the fused ideal moves 36 B
    per parameter (forward W read 4, backward W read 4 + grad write 4, norm read
    4, SGD read p, g, buf + write p, buf 20), plus 8 B per parameter per client
    per round for the global copy in and the update out:
        bytes = K (steps 36 P + 8 P).
    The engine trains only the live parameters (taps that read real pixels at
    32x32; dead taps have exactly zero gradient), so the achievable bound uses
    P_live for the per-step term.  Aggregated over all GPUs of the job."""
    full = K * (steps * 36.0 * P + 8.0 * P)
    live = K * (steps * 36.0 * P_live + 8.0 * P)
    sec = ms_per_round * 1e-3
    peak = HBM_PEAK_GBS * world
    # primary: the live parameters (the dead-tap slabs are never trained, so the
    # full-P figure would credit bytes no kernel moves)
    return {
        "bound": "hbm", "unit": "GB/s", "peak": peak,
        "bytes_per_round": live, "achieved": live / sec / 1e9, "frac": live / sec / 1e9 / peak,
        "bytes_per_round_full_P": full, "achieved_full_P": full / sec / 1e9, "frac_full_P": full / sec / 1e9 / peak,
        "P": P, "P_live": P_live, "formula": "K*(steps*36*P_live + 8*P) (SURVEY 8d, live parameters)",
        "note": "SURVEY 8d's HBM model omits the convolution / GEMM FLOPs; the conv_mfma / gemm_mfma fields "
                "give the compute side",
    }


def _median_time(fn, n: int, budget_s: float):
    """Median wall time of up to n calls of fn (at least one), stopping early
    once budget_s is spent; returns (median seconds, samples taken)."""
    import statistics
    ts = []
    t_all = time.perf_counter()
    while len(ts) < n:
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
        if time.perf_counter() - t_all > budget_s:
            break
    return statistics.median(ts), len(ts)


def cpu_baseline(spec, P, K, defense, f, multi_k, steps, batch, budget_s: float = 20.0, trim_ratio: float = 0.1):
    """The reference's CPU path (the oracle: run_experiments.py:195-240 loop,
    krum.py:55-192, trimmed_mean.py:48-166, base_defense.py:80-97 restated
    with the same torch/numpy calls) on this host's cores, BASELINE.md §2:
    (a) one client's local update (`steps` batches), (b) aggregate-ms of every
    hot-path aggregator at this K, (c) rounds/s of this config's defense =
    1 / (K * (a) + (b)[defense]).  Each figure is the median of up to 5 timed
    calls after one warm-up, inside a time budget (the sample text says how
    many were taken).  Bounded samples, stated: Krum's K(K-1)/2 pair norms are
    priced from pair norms at the full P; FedAvg, the trimmed mean, the median
    and the Multi-Krum mean from a reduced coordinate count P_s, scaled by
    P / P_s (each is linear in P)."""
    import numpy as np
    import torch
    sys.path.insert(0, ROOT)
    from oracle import aggregation as orc
    from oracle import training as otrain
    from flr.models.multimodal import model_class

    # the box's CPU share: OMP_NUM_THREADS (16 per GPU on the pool; os.cpu_count()
    # reports the whole host there, whose other cores belong to other jobs)
    host_cpus = os.cpu_count() or 1
    threads = min(host_cpus, int(os.environ.get("OMP_NUM_THREADS", host_cpus)))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(1000)
    batches = [(torch.randn(batch, spec.in_channels, spec.image_size, spec.image_size, generator=g),
                torch.randint(0, spec.vocab, (batch, spec.seq_len), generator=g),
                torch.randint(0, spec.num_classes, (batch,), generator=g)) for _ in range(steps)]
    torch.manual_seed(42)
    cls = model_class(spec)
    glob = torch.cat([p.detach().reshape(-1) for p in cls(spec).parameters()])
    otrain.local_update(cls, spec, glob, batches[:1])  # warm-up
    t_client, n_client = _median_time(lambda: otrain.local_update(cls, spec, glob, batches), 5, budget_s * 0.4)

    # (b) aggregation inputs: X[i] = g + sigma_i N(0,1), f sign-flipped
    P_s = min(P, 1 << 17)
    gs = torch.Generator().manual_seed(7)
    base = 0.05 * torch.randn(P_s, generator=gs)
    rows = []
    for i in range(K):
        r = base + 0.01 * (1 + 0.5 * i / K) * torch.randn(P_s, generator=gs)
        rows.append([-r if i < f else r])
    scale = P / P_s
    per = budget_s * 0.1
    nex = [steps * batch] * K
    agg = {}
    orc.fedavg(rows[:2], nex[:2])
    t, n_fa = _median_time(lambda: orc.fedavg(rows, nex), 5, per)
    agg["fedavg"] = t * scale
    orc.trimmed_mean(rows[:8], trim_ratio)
    t, n_tm = _median_time(lambda: orc.trimmed_mean(rows, trim_ratio), 5, per)
    agg["trimmed_mean"] = t * scale
    orc.median(rows[:8])
    t, n_md = _median_time(lambda: orc.median(rows), 5, per)
    agg["median"] = t * scale
    # Krum: pair norms at the full P (krum.py:95), scores + argsort on a K x K
    # matrix (krum.py:126-129, 174), the Multi-Krum mean of multi_k rows (:182-192)
    a = glob + 0.01 * torch.randn(P, generator=g)
    b = glob + 0.01 * torch.randn(P, generator=g)
    torch.norm(a - b).item()
    t_pair, n_pair = _median_time(lambda: torch.norm(a - b).item(), 5, per)
    del a, b
    D = np.abs(np.random.default_rng(0).standard_normal((K, K)))
    D = D + D.T
    np.fill_diagonal(D, 0.0)
    t_sel, _ = _median_time(lambda: np.argsort(orc.krum_scores(D, K - f - 2)), 5, per)
    mk = max(1, min(multi_k or K // 2, K))
    chosen = rows[:mk]
    t_mean, _ = _median_time(lambda: [sum(u[0] for u in chosen) / mk], 5, per)
    krum_s = K * (K - 1) / 2 * t_pair + t_sel + t_mean * scale
    agg["krum"] = krum_s
    mk_tm = max(1, int(mk * trim_ratio))
    sub = rows[:mk]
    t_ktm, _ = _median_time(lambda: orc.trimmed_mean(sub, trim_ratio), 3, per)
    agg["krum_trimmed_mean"] = K * (K - 1) / 2 * t_pair + t_sel + t_ktm * scale
    key = {"multi_krum": "krum", "none": "fedavg"}.get(defense, defense)
    agg_s = agg.get(key)
    round_s = K * t_client + (agg_s if agg_s is not None else 0.0)
    return {
        "value": 1.0 / round_s, "unit": "rounds/s", "cores": threads, "kind": "port",
        "cpu_model": cpu_model(), "host_cpus": host_cpus,
        "local_update_s_per_client": t_client, "local_update_s_all_clients": K * t_client,
        "aggregate_ms": {k: v * 1e3 for k, v in agg.items()},
        "aggregate_ms_this_defense": None if agg_s is None else agg_s * 1e3,
        "round_s": round_s,
        "sample": (f"oracle (reference loop restated, torch CPU fp32, {threads} threads = this job's CPU share "
                   f"(OMP_NUM_THREADS) of the host's {host_cpus} CPUs), medians after one warm-up: one client's "
                   f"local update x {steps} steps at batch {batch} ({n_client} timed, {t_client:.3f} s); "
                   f"FedAvg / trimmed mean (t = max(1, int({trim_ratio} K))) / median over K={K} rows at "
                   f"P_s={P_s} ({n_fa}/{n_tm}/{n_md} timed) scaled x{scale:.1f} to P={P}; Krum = "
                   f"{K * (K - 1) // 2} pair norms at the full P ({n_pair} timed, {t_pair * 1e3:.2f} ms/pair) + "
                   f"scores/argsort + the {mk}-row mean; round = K*client + aggregate({key}) = {round_s:.1f} s"),
    }


def gemm_flops_per_sample(spec) -> float:
    """Useful batched-GEMM FLOPs of one training sample (forward + input and
    weight gradients) of the model's nn.Linear layers, counted with forward
    hooks on one sample; the first layer on the raw input (the ViT patch
    embedding) has no input gradient."""
    import torch
    from flr.models.multimodal import model_class
    torch.manual_seed(0)
    m = model_class(spec)(spec)
    macs = []

    def hook(mod, inp, out):
        macs.append(inp[0].numel() // inp[0].shape[-1] * mod.in_features * mod.out_features)
    hs = [mod.register_forward_hook(hook) for mod in m.modules() if isinstance(mod, torch.nn.Linear)]
    with torch.no_grad():
        img = torch.randn(1, spec.in_channels, spec.image_size, spec.image_size)
        tok = torch.randint(0, spec.vocab, (1, spec.seq_len))
        m.eval()(img, tok)
    for h in hs:
        h.remove()
    return 2.0 * (3 * sum(macs) - (macs[0] if macs else 0))


def gemm_utilisation(spec, K: int, batch: int, steps: int, stats_path=None, chunk: int = 32):
    """Batched-GEMM MFMA utilisation for the encoder family (C4/C5): useful GEMM
    FLOPs per round (gemm_flops_per_sample) over the BGemm kernels' summed time
    per round in a rocprofv3 summary of that config's bench (--kernel-stats; the
    optimizer kernel's call count / local steps gives the rounds profiled),
    against the bf16x6 ceiling.  None without a summary."""
    if not stats_path or not os.path.exists(stats_path):
        return None
    flops = gemm_flops_per_sample(spec) * K * steps * batch
    ms = calls_ce = 0.0
    for name, calls, t in _kernel_rows(stats_path):
        if "BGemm" in name:
            ms += t
        if "::ce_kernel(" in name:
            calls_ce += calls
    if not calls_ce or not ms:
        return None
    # the cross-entropy kernel runs once per client chunk and local step (K = this GPU's clients)
    rounds = calls_ce / (steps * max(1, -(-K // max(1, chunk))))
    per_round = ms / rounds
    achieved = flops / (per_round * 1e-3) / 1e12
    peak = 2500.0 / 6.0
    return {"source": os.path.relpath(stats_path, ROOT), "measured_in_this_run": False,
            "flops_per_round": flops, "kernel_ms_per_round": per_round, "achieved_tflops": achieved,
            "peak_tflops": peak, "frac": achieved / peak,
            "peak_note": "bf16x6 form: 6 v_mfma_f32_32x32x16_bf16 products per fp32 product, 2.5 PF/s dense bf16"}


def round_collectives(eng, defense: str, K: int, P: int, world: int):
    """The per-round collectives of this configuration and the bytes each GPU
    sends (flr.shard / flr.ops.pairwise_l2_sharded / flr.dist), fp32 unless
    noted.  World 1: none."""
    if world == 1:
        return []
    from flr import _capi
    from flr.shard import PW_SLICES
    kl = K // world
    out = []
    if eng.exchange == "alltoall":
        ld = eng.xchg.plan.ld
        out.append({"op": "all_to_all", "what": "client rows -> coordinate ranges",
                    "bytes_sent_per_gpu": 4 * (world - 1) * kl * ld})
        if defense in ("krum", "multi_krum", "krum_trimmed_mean") and \
                getattr(eng.defense, "pairwise_method", "gram") == "reference":
            # the chains handed rank to rank (ops.pairwise_l2_reference_sharded), D broadcast
            out += [{"op": "send/recv", "what": "8 chain sums per pair [8, K, K] to the next rank",
                     "bytes_sent_per_gpu": 4 * 8 * K * K},
                    {"op": "broadcast", "what": "distance matrix [K, K] fp64 from the last rank",
                     "bytes_per_gpu": 8 * K * K}]
        elif defense in ("krum", "multi_krum", "krum_trimmed_mean"):
            S = int(_capi.lib().flr_pairwise_sample_len(P))
            glen = int(_capi.lib().flr_pairwise_gsum_len(K))
            out += [{"op": "all_reduce", "what": "pivot sample [K, S]",
                     "bytes_per_gpu": 4 * K * S},
                    {"op": "all_reduce", "what": "tail term [K, K] fp64", "bytes_per_gpu": 8 * K * K},
                    {"op": "all_gather", "what": "per-slice Gram records fp64",
                     "bytes_sent_per_gpu": 8 * glen * PW_SLICES // world}]
        out.append({"op": "all_gather", "what": "aggregated P-vector slices",
                    "bytes_sent_per_gpu": 4 * eng.xchg.plan.ld})
    else:
        out.append({"op": "all_gather", "what": "client matrix rows (replicated aggregation)",
                    "bytes_sent_per_gpu": 4 * kl * eng.full.data.stride(0)})
    return out


# BASELINE.json configs as presets: (model, clients, defense, defense_cfg, attack, attacker fraction)
PRESETS = {
    "C1": ("cub", 4, "fedavg", {}, "none", 0.0),
    "C2": ("resnet_gru", 32, "fedavg", {}, "none", 0.0),
    "C3": ("resnet_gru", 128, "krum", {}, "sign_flip", 0.2),
    "C4": ("vit_bert", 256, "trimmed_mean", {"trim_ratio": 0.1}, "none", 0.0),
    "C5": ("vit_bert", 512, "krum_trimmed_mean", {"trim_ratio": 0.1}, "backdoor", 0.2),
}
WORKLOAD = {
    "C1": "C1: FedAvg K=4, CUB200MultimodalCNN structure (conv img + attribute MLP over the BoW text)",
    "C2": "C2: FedAvg K=32, ResNet-18 img + 1-layer GRU text late fusion, 5 local SGD steps/round",
    "C3": "C3: Multi-Krum K=128, 20% sign-flip, ResNet-18 img + 1-layer GRU text late fusion, 5 local SGD steps/round",
    "C4": "C4: trimmed-mean K=256, ViT-S/4 img + BERT-mini text late fusion, 5 local SGD steps/round",
    "C5": "C5: backdoor K=512 (20% trigger-patch clients), ViT-S/4 + BERT-mini, Multi-Krum then trimmed-mean",
}


def launch_command(argv, n: int, port: int):
    """The child command that starts n ranks of this script on one node
    (torch.distributed.run, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def needs_launch(gpus: int, env=None) -> bool:
    """True when --gpus asks for more ranks than this process's torchrun
    environment provides and there is none: the parent then starts them.
    A torchrun environment whose WORLD_SIZE differs from --gpus is an error."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" not in env:
        return gpus > 1
    if int(env["WORLD_SIZE"]) != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={env['WORLD_SIZE']} but --gpus {gpus}")
    return False


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL over xGMI; gloo = one-GPU rehearsal)")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C3", choices=sorted(PRESETS),
                    help="BASELINE.json config preset (C3 = the headline metric's workload)")
    ap.add_argument("--clients", type=int, default=None)
    ap.add_argument("--local-steps", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--exchange", default="auto", choices=["auto", "alltoall", "allgather"])
    ap.add_argument("--pairwise", default="reference", choices=["gram", "reference"],
                    help="Krum distances: the reference-exact fp32 torch.norm accumulation (default: D "
                         "bit-identical to krum.py:89-97, so the selection is the reference's by construction; "
                         "whole rows: the all-gather exchange), or the centred Gram on MFMA (HBM-bound, "
                         "coordinate-sharded, selection equal only where the scores are well conditioned)")
    ap.add_argument("--defense", default=None, help="override the preset's defense (fedavg, krum, trimmed_mean, median)")
    ap.add_argument("--model", default=None, choices=["resnet_gru", "cub", "vit_bert"])
    ap.add_argument("--client-chunk", type=int, default=0, help="clients per forward/backward pass (0: automatic)")
    ap.add_argument("--kernel-stats", default=None,
                    help="rocprofv3 kernel_stats.csv (or the committed text summary) of THIS code's C3 bench, "
                         "for conv_mfma_from_profile (default: the newest committed profiles/*c3_kernel_stats*)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if needs_launch(args.gpus):
        # fresh child processes (never exec: nothing here has touched the GPU yet)
        import subprocess
        rc = subprocess.run(launch_command(sys.argv[1:], args.gpus, _free_port())).returncode
        sys.exit(rc)

    import torch
    from flr import dist as fdist
    from flr.models.multimodal import CUB, VIT_BERT, ModelSpec, num_params
    from flr.round import RoundConfig, RoundEngine
    from flr.timing import HipEventPair
    from flr.train import TrainConfig
    from flr import ops

    rank, world, local = fdist.init(args.backend)
    if world != args.gpus:
        raise SystemExit(f"bench.py: process group world size {world} != --gpus {args.gpus}")
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and local >= ndev:
        raise SystemExit(f"bench.py: local rank {local} but only {ndev} GPUs visible (use --backend gloo "
                         "to rehearse N ranks on fewer GPUs)")
    device = torch.device("cuda", local % max(1, ndev))
    torch.cuda.set_device(device)
    pg = None
    if world > 1:
        import torch.distributed as tdist
        pg = {"backend": tdist.get_backend(), "world_size": tdist.get_world_size()}
    model, K, defense, dcfg, attack, afrac = PRESETS[args.config]
    custom = any(v is not None for v in (args.clients, args.defense, args.model))
    model = args.model or model
    K = args.clients or K
    if args.defense:
        defense, dcfg = args.defense, ({"trim_ratio": 0.1} if "trimmed" in args.defense else {})
        attack, afrac = ("sign_flip", 0.2) if args.defense in ("krum", "multi_krum") else ("none", 0.0)
    spec = {"cub": CUB, "vit_bert": VIT_BERT}.get(model, ModelSpec())
    P = num_params(spec)
    krum = defense in ("krum", "multi_krum", "krum_trimmed_mean")
    if krum:
        dcfg = dict(dcfg, pairwise_method=args.pairwise)
    f = int(afrac * K)
    rcfg = RoundConfig(num_clients=K, defense=defense, defense_cfg=dict(dcfg), num_attackers=f,
                       exchange=args.exchange, attack=attack)
    tcfg = TrainConfig(local_steps=args.local_steps, client_chunk=args.client_chunk)
    eng = RoundEngine(spec, rcfg, tcfg, device, rank, world)
    multi_k = getattr(eng.defense, "multi_k", 0)
    workload = (WORKLOAD[args.config] if not custom else
                f"{defense} K={K}, {spec.name}, {args.local_steps} local SGD steps/round")
    if krum and args.pairwise == "reference":
        workload += "; Krum distances reference-exact"

    for _ in range(args.warmup):
        eng.run_round()
    torch.cuda.synchronize()
    fdist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.run_round()
    torch.cuda.synchronize()
    fdist.barrier()
    elapsed = fdist.max_over_ranks(time.perf_counter() - t0, device)

    # ---- untimed diagnostics after the timed region ----
    eng.materialize()  # (FLR_DEFER_DEAD=2: the client matrix's dead-tap ranges, for the diagnostics below)
    reps = 5
    sharded = eng.exchange == "alltoall"
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    kw = {"publish": False} if hasattr(eng.defense, "publish") else {}
    for _ in range(reps):  # Server.aggregate alone (sharded: this GPU's range + the P-vector all-gather)
        if sharded:
            eng.slice.gather_vector(eng.defense.aggregate_sharded(eng.slice, eng.num_examples, **kw),
                                    torch.empty_like(eng.global_flat))
        else:
            eng.defense.aggregate_flat(eng.full, eng.num_examples, **kw)
    ev1.record()
    torch.cuda.synchronize()
    aggregate_ms = ev0.elapsed_time(ev1) / reps
    # every hot-path aggregator on this round's client matrix
    from flr.defenses import get_defense
    aggregate_ms_all = {}
    for name in ("fedavg", "krum", "trimmed_mean", "median"):
        cfg = ({"num_malicious": f if krum else int(0.2 * K), "multi_k": max(1, K // 2),
                "pairwise_method": args.pairwise} if name == "krum" else
               {"trim_ratio": dcfg.get("trim_ratio", 0.1)} if name == "trimmed_mean" else {})
        d = get_defense(name, cfg)
        if name == "krum":  # the round's matrix order (a training-order round: the coordinate map)
            d.comm = getattr(eng.defense, "comm", None)
            d.tap_blocks = (eng.defense.tap_blocks if hasattr(eng.defense, "tap_blocks") else
                            eng._tap_blocks()[1] if eng.train_order else None)
        kwd = {"publish": False} if hasattr(d, "publish") else {}
        run = ((lambda: eng.slice.gather_vector(d.aggregate_sharded(eng.slice, eng.num_examples, **kwd),
                                                torch.empty_like(eng.global_flat))) if sharded else
               (lambda: d.aggregate_flat(eng.full, eng.num_examples, **kwd)))
        run()
        ev0.record()
        for _ in range(reps):
            run()
        ev1.record()
        torch.cuda.synchronize()
        aggregate_ms_all[name] = ev0.elapsed_time(ev1) / reps
    # the Gram path's kernel: centred-Gram pairwise
    # (HIP events around its launch, on the stream it runs on); sharded: this
    # GPU's coordinates.  Timed for every config (the Krum roofline line).
    kms = []
    # (not at tap-block-aligned rank boundaries: the Gram records need the canonical slices)
    gram_timed = not (sharded and eng.slice.plan.bounds is not None)
    for _ in range(reps if gram_timed else 0):
        ev = HipEventPair()
        if sharded:
            ops.pairwise_l2_sharded(eng.slice, events=ev.handles)
        else:
            ops.pairwise_l2(eng.full.X, "gram", events=ev.handles)
        kms.append(ev.elapsed_ms())
    kernel_ms = sum(kms) / len(kms) if kms else None
    # the whole Krum distance phase: every kernel that produces D —
    # Gram: pivot sample + Gram + far-cluster refine + reductions, HBM-bound;
    # reference: chain-major transposes + chains + finish, VALU-issue-bound
    phase = None
    if krum:
        method = getattr(eng.defense, "pairwise_method", "gram")
        pms = []
        for _ in range(reps):
            ev0.record()
            if sharded:
                eng.defense._sharded_distances(eng.slice)
            else:
                ops.pairwise_l2(eng.full.X, method, comm=getattr(eng.defense, "comm", None),
                                tap_blocks=getattr(eng.defense, "tap_blocks", None) if method == "reference" else None)
            ev1.record()
            torch.cuda.synchronize()
            pms.append(ev0.elapsed_time(ev1))
        pm = sorted(pms)[len(pms) // 2]
        nc = eng.slice.n if sharded else P
        byts = 4.0 * K * nc + 8.0 * K * K
        phase = {"method": method, "ms": pm, "algorithmic_bytes": byts,
                 "hbm_frac": byts / (pm * 1e-3) / (HBM_PEAK_GBS * 1e9)}
        if method == "reference":
            # 8 chains per pair, each a v_sub + v_fma per step over P/8 steps (this
            # rank's share of the pair tiles at world > 1)
            lane_ops = 2.0 * 8 * (K * (K - 1) / 2) * (P // 8) / world
            phase.update({"valu_lane_ops": lane_ops, "valu_peak_ops_per_s": VALU_PEAK_OPS,
                          "valu_frac": lane_ops / (pm * 1e-3) / VALU_PEAK_OPS,
                          "bound": "valu (issue)", "hbm_frac_note": "bytes of one read of X; the kernels also "
                          "rewrite X chain-major once (2x those bytes)"})
        else:
            phase["bound"] = "hbm"
    n_coords = eng.slice.n if sharded else P
    pair_bytes = 4.0 * K * n_coords + 8.0 * K * K
    achieved = pair_bytes / (kernel_ms * 1e-3) / 1e9 if kernel_ms else None
    traffic = gram_traffic(K, n_coords)
    gram_roofline = None if not gram_timed else {
        "kernel": "gram_partials_kernel (Krum pairwise, centred Gram on MFMA)" + (
            " — the --pairwise gram path, timed here beside the round" if phase and phase["method"] == "reference"
            else ""),
        "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
        "kernel_ms": kernel_ms, "algorithmic_bytes": pair_bytes, "coords_per_gpu": n_coords,
    }
    # the reference-exact distances (the default Krum path): VALU-issue bound —
    # every pair's 8 chains run the whole vector sequentially, one chain per
    # lane, one wave per SIMD; the phase (transposes + chains + finish) timed
    # live with HIP events; its chain kernel alone in profiles/ (rocprofv3)
    ref_roofline = None
    if phase is not None and phase["method"] == "reference":
        ref_roofline = {
            "kernel": "reference-exact distance phase (chain_transpose_kernel + tap_chain_kernel + ref_chain_kernel "
                      "+ ref_finish_kernel)",
            "bound": "valu", "unit": "Gop/s", "achieved": phase["valu_lane_ops"] / (phase["ms"] * 1e-3) / 1e9,
            "peak": VALU_PEAK_OPS / 1e9, "frac": phase["valu_frac"],
            "traffic": ref_traffic(K, P) if world == 1 else None,
            "kernel_ms": phase["ms"], "lane_ops": phase["valu_lane_ops"],
            "one_wave_issue_frac": phase["valu_frac"] * 2.0,
            "note": "lane-ops = 2 (v_sub + v_fma) x 8 chains x K(K-1)/2 pairs x P/8 steps; peak = fp32 VALU at "
                    "2 cycles per wave64 instruction per SIMD; one wave per SIMD issues at most every 4 cycles "
                    "(MI355X_MICROARCH.md), so one_wave_issue_frac = 2 x frac is this layout's ceiling "
                    "(the chains fill ~1 wave per SIMD at C3)",
        }
    # training-phase time (one round's local updates, this rank's clients)
    ev0.record()
    if eng._graph is not None:
        eng._graph.replay()
    else:
        eng._train_phase()
    ev1.record()
    torch.cuda.synchronize()
    train_ms = ev0.elapsed_time(ev1)
    attackers_selected = None
    if krum:
        eng.defense.publish()
        attackers_selected = sorted(set(eng.defense.selected_clients) & set(range(f)))
    # the global model after warmup + steps rounds (bit-identical at every N)
    import hashlib
    global_sha256 = hashlib.sha256(eng.global_flat.detach().cpu().numpy().tobytes()).hexdigest()
    ref_sha = None if custom else REFERENCE_SHA.get((args.config, args.pairwise, args.warmup + args.steps))

    out = {
        "metric": METRIC,
        "value": args.steps / elapsed,
        "unit": "rounds/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32 (bf16x6-split MFMA conv/GEMM = fp32 operands; Krum Gram bf16x4 hi/lo split, fp32 accumulate)",
        "data": "synthetic (SURVEY §8d: N(0,1) 3x32x32 images, U{0..999} 16-token texts, 10 classes; "
                "random-init weights, seed 42)",
        "config": {
            "workload": workload, "preset": None if custom else args.config, "model": spec.name,
            "clients": K, "params": P, "local_steps": args.local_steps, "batch": rcfg.batch,
            "defense": f"{defense}(f={f}, multi_k={multi_k})" if krum else defense, "attack": attack,
            "attackers": f, "client_chunk": eng.trainer.chunks[0][1] - eng.trainer.chunks[0][0],
            "parallelism": (f"clients sharded {K // world}/GPU x {world}; " + (
                "one all-to-all (client rows -> coordinate ranges), per-GPU aggregation of its range, "
                "all-gather of the aggregated vector" if sharded else "one all-gather of the client matrix")),
            "exchange": eng.exchange,
            "krum_distances": (None if not krum else "reference-exact (fp32 torch.norm accumulation, D bit-identical "
                               "to krum.py:89-97)" if args.pairwise == "reference" else
                               "centred Gram on MFMA + exact far-cluster refine"),
            "training_phase": ("one captured HIP graph per round" if eng.use_graph else "eager launches") + (
                ("; local updates = one flr_train_vit_bert call" if spec.family == "vit_bert" else
                 "; local updates = one flr_train_clients_ex call") if eng.native else
                "; local updates = the Python autograd composition of the kernels"),
        },
        "process_group": pg,
        "global_sha256": global_sha256,
        "sha_matches_reference_run": None if ref_sha is None else global_sha256 == ref_sha,
        "aggregate_ms": aggregate_ms,
        "aggregate_ms_by_defense": aggregate_ms_all,
        "train_ms_per_round": train_ms,
        "attackers_selected": attackers_selected,
        "round_roofline": round_roofline(K, P, eng.trainer.live_params, args.local_steps,
                                         elapsed / args.steps * 1e3, world),
        "conv_mfma_from_profile": conv_utilisation(spec, K, rcfg.batch, args.local_steps, args.kernel_stats)
        if args.config == "C3" and not custom else None,
        "gemm_mfma_from_profile": gemm_utilisation(
            spec, K // world, rcfg.batch, args.local_steps,
            args.kernel_stats or (os.path.join(ROOT, COMMITTED_C4_STATS) if args.config == "C4" and not custom
                                  else None), chunk=eng.trainer.chunks[0][1] - eng.trainer.chunks[0][0])
        if model == "vit_bert" else None,
        "collectives": round_collectives(eng, defense, K, P, world),
        "distance_phase": phase,
        "roofline": ref_roofline if ref_roofline is not None else gram_roofline,
        "roofline_gram": gram_roofline if ref_roofline is not None else None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(spec, P, K, defense, f, multi_k, args.local_steps, rcfg.batch,
                                           args.cpu_budget, dcfg.get("trim_ratio", 0.1))
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
