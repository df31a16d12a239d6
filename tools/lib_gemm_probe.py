"""Library GEMM layout probe at the metric shape: which bf16 operand layout hipBLASLt runs fastest for
Y[4096,4096] = X[4096,11008] @ W^T (W dequantised to [N,K] or [K,N]).  Interleaved reps, median."""
import statistics
import torch

M, N, K = 4096, 4096, 11008
dev = torch.device("cuda", 0)
X = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)      # [N, K] (dequantise output layout)
Wt = W.t().contiguous()                                              # [K, N]
Y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
cases = {
    "matmul(X, W.t()) NT": lambda: torch.matmul(X, W.t(), out=Y),
    "matmul(X, Wt) NN": lambda: torch.matmul(X, Wt, out=Y),
    "linear(X, W)": lambda: torch.nn.functional.linear(X, W),
    "mm(W, X.t()) -> Y^T": lambda: torch.mm(W, X.t()),
}
ev = {k: [] for k in cases}
for _ in range(3):
    for k, f in cases.items():
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        for _ in range(20):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(); f(); e.record()
            ev[k].append((s, e))
torch.cuda.synchronize()
for k, l in ev.items():
    t = statistics.median(s.elapsed_time(e) for s, e in l) * 1e3
    print(f"{k:28s} {t:8.1f} us  {2*M*N*K/t/1e6:8.1f} TFLOP/s")
