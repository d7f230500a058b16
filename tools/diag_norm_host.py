"""Diagnostic: which fp32 accumulation model does THIS host's torch.norm use?
(SURVEY App. C was probed on the build container's Xeon; the GPU box's EPYC
may dispatch a different CPU kernel.)"""
import ctypes, itertools, os, subprocess, sys
import torch
here = os.path.dirname(os.path.abspath(__file__))
so = "/tmp/norm_models.so"
subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-mfma", os.path.join(here, "norm_models.c"),
                "-o", so, "-lm"], check=True)
L = ctypes.CDLL(so)
L.norm_model.restype = ctypes.c_float
L.norm_model.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64] + [ctypes.c_int] * 4
print("torch", torch.__version__, "capability", torch.backends.cpu.get_cpu_capability(), "threads", torch.get_num_threads())
print(open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0])
cands = list(itertools.product([8, 16, 32], [1, 2, 4], [0, 1], [0, 1]))
ok = {c: 0 for c in cands}
tot = 0
for n in [8, 9, 15, 16, 17, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129, 255, 256, 257, 1000, 4099, 65537, 1 << 20]:
    for seed in range(4):
        g = torch.Generator().manual_seed(n * 10 + seed)
        a = torch.randn(n, generator=g) * (10.0 ** (seed - 2))
        b = a + torch.randn(n, generator=g) * 1e-3 * torch.exp(2 * torch.randn(n, generator=g))
        want = torch.norm(a - b).item()
        tot += 1
        for c in cands:
            if L.norm_model(a.data_ptr(), b.data_ptr(), n, *c) == want:
                ok[c] += 1
best = sorted(ok.items(), key=lambda kv: -kv[1])[:8]
print("trials", tot)
for c, k in best:
    print("lanes=%d unroll=%d tree=%d tailfma=%d : %d/%d" % (*c, k, tot))
