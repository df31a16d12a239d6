import json, sys, os
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bitsandbytes-sycl_amd")]
import torch, bench
r = bench.bench_llama2_70b_shard(torch.device("cuda", 0))
print(json.dumps({k: r[k] for k in ("decode", "decode_fused", "prefill")}))
