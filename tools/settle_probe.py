#!/usr/bin/env python3
"""settle_probe.py MODE [log2 n] -- bench.py's timed loop (20 timed radix sorts after 5 warm-up
sorts, gsort_stats on) after one of these preconditionings (development tool):
  none      nothing
  copy      gsort_copy_ceiling for 100 ms (its two 1-GiB buffers allocated and freed per call)
  torch     torch device copies for 100 ms on buffers torch keeps (GPU load, no HIP malloc/free)
  alloc     1-GiB ctx.alloc / free 20 times (allocator churn, no GPU load)
  sorts     45 extra warm-up sorts
One JSON line: the mode and ms per timed step."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mpi-test_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import gsort  # noqa: E402

mode = sys.argv[1]
lg = int(sys.argv[2]) if len(sys.argv) > 2 else 28
n = 1 << lg
ctx = gsort.Context()
d_in = ctx.alloc(n * 4)
ctx.generate(gsort.UNIFORM, 42, 0, n, d_in)
ctx.reserve(n)
t_s = time.perf_counter()
warm = 5
if mode == "copy":
    while (time.perf_counter() - t_s) * 1e3 < 100:
        ctx.copy_ceiling(n * 4, 10)
elif mode == "torch":
    a = torch.empty(n, dtype=torch.int32, device="cuda")
    b = torch.empty_like(a)
    while (time.perf_counter() - t_s) * 1e3 < 100:
        for _ in range(10):
            b.copy_(a)
        torch.cuda.synchronize()
elif mode == "alloc":
    for _ in range(20):
        q = ctx.alloc(n * 4)
        ctx.free(q)
elif mode == "sorts":
    warm = 50
settle_ms = (time.perf_counter() - t_s) * 1e3
for _ in range(warm):
    ctx.radix(d_in, n)
torch.cuda.synchronize()
raw = [gsort.Stats() for _ in range(20)]
t0 = time.perf_counter()
for r in raw:
    ctx.radix(d_in, n, r)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) * 1e3 / 20
print(json.dumps({"mode": mode, "settle_ms": round(settle_ms, 1), "ms_per_step": round(ms, 4)}),
      flush=True)
ctx.free(d_in)
ctx.close()
