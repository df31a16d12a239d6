"""Mismatch report of the optimizer kernels vs the oracle (debug aid): python tools/optim_debug.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bitsandbytes-sycl_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import python_src_quants.functional as F  # noqa: E402
from helpers import to_numpy, to_torch  # noqa: E402
from oracle import optim as oref  # noqa: E402
from oracle import ref  # noqa: E402

dev = torch.device("cuda", 0)
HP = {"adam": (0.9, 0.999, 1e-8, 1e-3), "momentum": (0.9, 0.0, 0.0, 1e-2), "rmsprop": (0.9, 0.0, 1e-8, 1e-2),
      "adagrad": (0.0, 0.0, 1e-10, 1e-2), "lion": (0.9, 0.99, 0.0, 1e-4)}
code1, code2 = F.create_dynamic_map(True), F.create_dynamic_map(False)
for name in HP:
    for kind in ("fp32", "bf16"):
        rng = np.random.default_rng(0)
        n = 2 * 2048
        b1, b2, eps, lr = HP[name]
        p = ref.cast_out((rng.standard_normal(n) * 0.1).astype(np.float32), kind)
        g = ref.cast_out((rng.standard_normal(n) * 0.01).astype(np.float32), kind)
        c1 = np.zeros(n, np.uint8); c2 = np.zeros(n, np.uint8)
        a1 = np.zeros(1 + n // 2048, np.float32)[:n // 2048]; a2 = a1.copy()
        tp = to_torch(p, kind, dev); t1 = torch.zeros(n, dtype=torch.uint8, device=dev)
        t2 = torch.zeros(n, dtype=torch.uint8, device=dev) if name == "adam" else None
        ta1 = torch.zeros(n // 2048, device=dev); ta2 = torch.zeros(n // 2048, device=dev) if name == "adam" else None
        F.optimizer_update_8bit_blockwise(name, to_torch(g, kind, dev), tp, t1, t2, b1, b2, eps, 1, lr, code1.to(dev),
                                          code2.to(dev) if t2 is not None else None, ta1, ta2)
        pe, c1e, c2e, a1e, a2e = oref.update_8bit_blockwise(name, g, p, c1, c2, code1.numpy(), code2.numpy(), a1, a2,
                                                            b1, b2, eps, 1, lr, 0.0, 1.0, False, kind)
        pg = ref.as_f32(to_numpy(tp, kind), kind); pe32 = ref.as_f32(pe, kind)
        bad = np.nonzero(pg.view(np.uint32) != pe32.view(np.uint32))[0]
        print(f"{name:8s} {kind}: p mismatches {bad.size}", end="")
        if bad.size:
            i = bad[0]
            print(f" e.g. i={i} gpu={pg[i]!r} oracle={pe32[i]!r} p0={ref.as_f32(p, kind)[i]!r} g={ref.as_f32(g, kind)[i]!r}", end="")
        print(f"; codes1 mism {(t1.cpu().numpy() != c1e).sum()}; absmax1 eq {np.array_equal(ta1.cpu().numpy(), a1e)}"
              f" gpu {ta1.cpu().numpy()[:2]} or {a1e[:2]}")
