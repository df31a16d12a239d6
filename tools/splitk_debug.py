import ctypes as ct, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd")]
import torch
import python_src_quants.functional as F
dev = torch.device("cuda", 0)
m, n, k = 1024, 1536, 2048
X = (torch.rand(m, k, device=dev) * 2 - 1).to(torch.bfloat16)
W = (torch.rand(n, k, device=dev) * 2 - 1).to(torch.bfloat16)
nb = int(F.lib.chgemm_tn_workspace_bytes(m, n, k))
print("ws bytes", nb, nb / (m * n * 4))
ws = torch.zeros(nb // 4, dtype=torch.float32, device=dev)
out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
F.pre_call(dev)
rc = F.lib.chgemm_tn_ws_bf16(m, n, k, F.get_ptr(X), k, F.get_ptr(W), k, F.get_ptr(out), n, F.get_ptr(ws), ct.c_longlong(nb))
torch.cuda.synchronize()
exp = X.float() @ W.float().t()
S = nb // (m * n * 4)
part = ws.view(S, m, n)
print("rc", rc, "sum of partials vs exp max err", (part.sum(0) - exp).abs().max().item())
print("out vs exp max err", (out.float() - exp).abs().max().item())
print("partial[0][0,:8]", part[0, 0, :8].tolist())
print("exp[0,:8]", exp[0, :8].tolist())
print("out[0,:8]", out[0, :8].float().tolist())
nz = (part != 0).float().mean().item()
print("nonzero fraction of partials", nz)
