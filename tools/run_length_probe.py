#!/usr/bin/env python3
"""run_length_probe.py -- does a partition pass's time follow its digit-run length?  (development
tool, GPU).  Sorts 2^28 keys of 31 bits (the canonical stream: level 3 uses 128 digits, 64-key
runs per 8192-key tile) and of 32 bits (all 256 digits, 32-key runs) and prints the per-level
times from gsort_stats (K3r = level 3, K3a = level 2, K11)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mpi-test_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import gsort  # noqa: E402

n = 1 << 28
ctx = gsort.Context()
p = ctx.alloc(n * 4)
rng = np.random.default_rng(1)
for name, keys in (("31-bit", None),
                   ("32-bit", rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)),
                   ("30-bit", rng.integers(0, 2**30, n, dtype=np.int64).astype(np.int32))):
    if keys is None:
        ctx.generate(gsort.UNIFORM, 42, 0, n, p)
    else:
        ctx.to_device(keys, p)
    for _ in range(3):
        ctx.radix(p, n)
    st = [ctx.radix(p, n)[2] for _ in range(10)]
    avg = lambda f: sum(f(s) for s in st) / len(st)  # noqa: E731
    print(f"{name}: total {avg(lambda s: s['ms_total']):.4f} ms  K1h+plan {avg(lambda s: s['ms_hist']):.4f}"
          f"  K3r {avg(lambda s: s['ms_level'][0]):.4f}  K3a {avg(lambda s: s['ms_level'][1]):.4f}"
          f"  K11 {avg(lambda s: s['ms_bucket_sort']):.4f}", flush=True)
ctx.free(p)
ctx.close()
