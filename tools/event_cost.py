#!/usr/bin/env python3
"""event_cost.py [log2 n] [reps] -- what instrumentation and buffer placement cost a sort
(development tool).  Times back-to-back radix sorts of the same resident keys, alternating
settings in one process, and prints the wall time per sort of each (host clock around a batch,
one synchronisation per batch):
  stats off / on  -- no gsort_stats (no events on the dispatches) vs. every kernel dispatch
                     carrying a stop event, as in bench.py's timed region;
  reserved        -- a second context that called gsort_reserve(n) first, as bench.py does
                     (S_TMP allocated before the sampled plan's region buffers)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mpi-test_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402
import gsort  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 28
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
n = 1 << lg
ctxs = []
for reserve in (False, True):
    ctx = gsort.Context()
    p = ctx.alloc(n * 4)
    ctx.generate(gsort.UNIFORM, 42, 0, n, p)
    if reserve:
        ctx.reserve(n)
    for _ in range(3):
        ctx.radix(p, n)
    ctxs.append((ctx, p))
settings = [("plain, stats off", 0, False), ("plain, stats on ", 0, True),
            ("reserved, stats off", 1, False), ("reserved, stats on ", 1, True)]
res = {s[0]: [] for s in settings}
for rnd in range(4):
    for name, ci, st in settings:
        ctx, p = ctxs[ci]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.radix(p, n, stats=st)
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) * 1e3 / reps)
for name, _, _ in settings:
    v = sorted(res[name])
    print(f"{name:20s} ms per sort: median {v[len(v) // 2]:.4f}  all "
          + " ".join(f"{x:.4f}" for x in res[name]), flush=True)
for ctx, p in ctxs:
    ctx.free(p)
    ctx.close()
