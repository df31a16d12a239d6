import os, sys, torch
sys.path.insert(0, "bitsandbytes-sycl_amd")
from python_src_quants import functional as F
def t_us(fn, it=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / it
dev = torch.device("cuda", 0); g = torch.Generator(device=dev).manual_seed(0); K = 11008
for (m, n) in ((4096, 512), (2048, 512), (4096, 1024), (2048, 1024), (2048, 2048)):
    A = torch.randint(-127, 128, (m, K), device=dev, dtype=torch.int8, generator=g)
    B = torch.randint(-127, 128, (n, K), device=dev, dtype=torch.int8, generator=g)
    rs = torch.rand(m, device=dev, generator=g) + 0.5; cs = torch.rand(n, device=dev, generator=g) + 0.5
    out = torch.empty(m, n, device=dev, dtype=torch.float16)
    fn = lambda: F.igemmlt_dequant(A, B, rs, cs, out=out)
    res = {}
    kss = (1, 2, 3, 4, 6, 8, 12, 16)
    for _ in range(3):
        for ks in kss:
            F.lib.cigemm_set_splitk(ks); res.setdefault(ks, []).append(t_us(fn))
    F.lib.cigemm_set_splitk(-1)
    print(f"{m}x{n}x{K} auto-bytes {F.lib.cigemmlt_workspace_bytes(m, n, K)}: " + "  ".join(f"ks{ks} {sorted(v)[1]:6.1f}" for ks, v in res.items()), flush=True)
