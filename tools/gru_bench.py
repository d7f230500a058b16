"""Time the fused GRU step kernels (flr_gru_fwd_fused / flr_gru_bwd_fused) at
the C3 text-branch shape under each (waves, k-steps-per-group) variant.
usage: gru_bench.py [K B T H]"""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multimodal-fl-security_amd"))
import torch
from flr import _capi


def main():
    K, B, T, H = (int(a) for a in sys.argv[1:5]) if len(sys.argv) > 4 else (128, 32, 16, 256)
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=g) * 0.1
    gi, whh, bhh = r(K, B, T, 3 * H), r(K, 3 * H, H), r(K, 3 * H)
    hseq, gates = r(K, T + 1, B, H), r(K, T, B, 4 * H)
    from flr.nn import _gru_packed
    whhP, whhT = r(K, _gru_packed(3, H, H)), r(K, _gru_packed(1, H, 3 * H))
    dgh, dgi, dd = r(K, T, B, 3 * H), r(K, B, T, 3 * H), r(K, B, H)
    dd0 = dd.clone()
    lib = _capi.lib()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    P = lambda x: ctypes.c_void_p(x.data_ptr())
    fwd = lambda: lib.flr_gru_fwd_fused(P(gi), P(whhP), P(bhh), P(hseq), P(gates), K, B, T, H, 5, st)
    bwd = lambda: lib.flr_gru_bwd_fused(P(whhT), P(gates), P(hseq), P(dgh), P(dgi), P(dd), None, K, B, T, H, 6, st)
    wbytes = 4 * K * 3 * H * H
    pack = lambda: lib.flr_gru_pack(P(whh), K, 3, H, H, 0, P(whhP), st)
    packT = lambda: lib.flr_gru_pack(P(whh), K, 1, H, 3 * H, 1, P(whhT), st)

    def timeit(fn, n=50):
        for _ in range(5):
            assert fn() == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n * 1e3

    for name, fn in [("pack W_hh", pack), ("pack W_hh^T", packT)]:
        us = timeit(fn)
        print(f"{name:12s} {us:8.2f} us  {2 * wbytes / us / 1e6:6.2f} TB/s (read + write)", flush=True)
    outs = {"fwd": lambda: (hseq[:, 6].clone(), gates[:, 5].clone()),
            "bwd": lambda: (dgh[:, 5].clone(), dgi[:, :, 5].clone(), dd.clone())}
    for var, env, fn in [("fwd", "FLR_GRU_FW", fwd), ("bwd", "FLR_GRU_BW", bwd)]:
        cfgs = ["8,2", "8,2s", "4,4", "2,8"] if var == "fwd" else ["8,2", "8,2s", "8,6", "4,12", "16,3"]
        ref = None
        for c in cfgs:
            os.environ[env] = c
            if var == "bwd":
                dd.copy_(dd0)  # the bwd step rewrites dh_direct in place: same input for every variant
            assert fn() == 0
            torch.cuda.synchronize()
            o = outs[var]()
            same = "" if ref is None else ("  bit-identical" if all(torch.equal(a, b) for a, b in zip(o, ref))
                                            else "  DIFFERS")
            ref = ref if ref is not None else o
            us = timeit(fn)
            print(f"{var} NW,G={c:5s} {us:8.2f} us  W_hh stream {wbytes / us / 1e6:6.2f} TB/s{same}", flush=True)
        os.environ.pop(env)


if __name__ == "__main__":
    main()
