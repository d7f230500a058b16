"""Attention kernel timing at the C4/C5 encoder shapes (32 clients x batch 32):
ViT-S (T=65, 6 heads) and BERT-mini (T=16, 4 heads); fwd and bwd, us per
launch and the VALU FLOP rate (2*T*T*64 per product, 2 products fwd, 5 bwd)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "multimodal-fl-security_amd"))
import torch
from flr import _capi


def bench(KB, T, H, reps=20, threads=None):
    _capi.set_knob("FLR_ATT_THREADS", str(threads) if threads else None)
    torch.manual_seed(0)
    D = H * 64
    qkv = torch.randn(KB * T, 3 * D, device="cuda")
    ctx = torch.empty(KB * T, D, device="cuda")
    lse = torch.empty(KB * H * T, device="cuda")
    dctx = torch.randn_like(ctx)
    dqkv = torch.empty_like(qkv)
    st = torch.cuda.current_stream().cuda_stream
    f = lambda: _capi.call("flr_attention_fwd", qkv.data_ptr(), KB, T, H, 64, ctx.data_ptr(), lse.data_ptr(), st)
    b = lambda: _capi.call("flr_attention_bwd", qkv.data_ptr(), ctx.data_ptr(), dctx.data_ptr(), lse.data_ptr(), KB, T,
                           H, 64, dqkv.data_ptr(), st)
    out = []
    for fn, nprod in ((f, 2), (b, 5)):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        flops = KB * H * nprod * 2.0 * T * T * 64
        out.append((us, flops / us / 1e6))
    print(f"[threads {threads or 'default'}] KB={KB} T={T} H={H}: fwd {out[0][0]:8.1f} us {out[0][1]:6.1f} TF/s | bwd {out[1][0]:8.1f} us "
          f"{out[1][1]:6.1f} TF/s", flush=True)
    f()
    b()
    torch.cuda.synchronize()
    return ctx.cpu(), lse.cpu(), dqkv.cpu()



if __name__ == "__main__":
    for KB, T, H in ((32 * 32, 65, 6), (32 * 32, 16, 4), (64, 48, 2), (64, 96, 2)):
        r0 = bench(KB, T, H, threads=256)
        r1 = bench(KB, T, H, threads=512)
        same = all(torch.equal(a, b) for a, b in zip(r0, r1))
        print(f"  T={T}: 256- and 512-thread outputs bit-identical: {same}", flush=True)
