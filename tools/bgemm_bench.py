"""flr_bgemm timing at the encoder shapes of C4/C5 (32 clients per pass, batch
32: ViT rows M = 2080, BERT rows 512) and the GRU / head shapes of C3, in
useful TFLOP/s (2 M N R per client).  --variants "A=1;B=2": env settings timed
in the same process (the kernel reads FLR_BGEMM_TILE / FLR_GEMM per launch)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multimodal-fl-security_amd"))
import torch
from flr import nn as fnn

K = int(os.environ.get("K", 32))
ONLY = os.environ.get("ONLY")
SHAPES = [  # name, M, N, R, mode (fwd: x W^T | dx: dy W | dw: dy^T x)
    ("vit.qkv", 2080, 1152, 384, "fwd"), ("vit.fc1", 2080, 1536, 384, "fwd"), ("vit.fc2", 2080, 384, 1536, "fwd"),
    ("vit.fc1.dx", 2080, 384, 1536, "dx"), ("vit.fc1.dw", 1536, 384, 2080, "dw"), ("vit.qkv.dw", 1152, 384, 2080, "dw"),
    ("bert.fc1", 512, 1024, 256, "fwd"), ("bert.fc1.dw", 1024, 256, 512, "dw"),
    ("gru.hh", 32, 768, 256, "fwd"), ("gru.hh.dx", 32, 256, 768, "dx"), ("gru.ih", 512, 768, 128, "fwd"),
    ("gru.ih+b", 512, 768, 128, "fwdb"), ("gru.ih+add", 512, 768, 128, "fwda"),
]



def _set_knobs(env):
    """The library reads FLR_* switches once at load: variants go through flr_set_knob."""
    from flr import _capi
    for k, v in env.items():
        if k.startswith("FLR_"):
            _capi.set_knob(k, v)

def operands(M, N, R, mode):
    if mode in ("fwd", "fwdb", "fwda"):   # A = x [M, R], B = W [N, R] (fwdb: + bias [K, N]; fwda: + addend)
        return torch.randn(K, M, R, device="cuda"), torch.randn(K, N, R, device="cuda")
    if mode == "dx":    # A = dy [M, R], B = W^T view [N, R] of W [R, N]
        return torch.randn(K, M, R, device="cuda"), torch.randn(K, R, N, device="cuda").transpose(1, 2)
    # dw: A = dy^T [M, R] of dy [R, M], B = x^T [N, R] of x [R, N]
    return torch.randn(K, R, M, device="cuda").transpose(1, 2), torch.randn(K, R, N, device="cuda").transpose(1, 2)


def main():
    variants = [{}]
    if "--variants" in sys.argv:
        for v in sys.argv[sys.argv.index("--variants") + 1].split(";"):
            variants.append(dict(kv.split("=") for kv in v.split(",") if kv))
    print("K =", K, "variants:", variants, flush=True)
    for name, M, N, R, mode in SHAPES:
        if ONLY and not name.startswith(ONLY):
            continue
        A, B = operands(M, N, R, mode)
        out = torch.empty(K, M, N, device="cuda")
        bias = torch.randn(K, N, device="cuda") if mode == "fwdb" else None
        addt = torch.randn(K, M, N, device="cuda") if mode == "fwda" else None
        cells = []
        for var in variants:
            old = {k: os.environ.get(k) for k in var}
            os.environ.update(var)
            _set_knobs(var)
            for _ in range(3):
                fnn.bgemm(A, B, bias=bias, add=addt, out=out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record()
            for _ in range(reps):
                fnn.bgemm(A, B, bias=bias, add=addt, out=out)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            cells.append(f"{us:9.1f} us {2.0 * K * M * N * R / us / 1e6:6.1f} TF/s")
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            _set_knobs(old)
        print(f"{name:12s} {M:5d} {N:5d} {R:5d} {mode:4s} | " + " | ".join(cells), flush=True)


if __name__ == "__main__":
    main()
