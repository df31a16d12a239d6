import sys, os, json
sys.path[:0] = ["/root/repo", "/root/repo/bitsandbytes-sycl_amd"]
os.chdir(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch, bench
dev = torch.device("cuda", 0)
for shape in ((4096, 4096, 11008), (4096, 4096, 4096)):
    r = bench.bench_int8(dev, *shape)
    print(shape, round(r["us"], 2), round(r["tops"], 1))
