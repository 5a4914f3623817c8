#!/usr/bin/env python3
"""dist_probe.py [log2 n] [case,case,...] -- local sort time across key distributions (development tool, GPU):
looks for performance cliffs of the MSD plan (bucket sizes that fall between K11 classes or
past kLocalMax, skewed digits, duplicates).  Prints ms per sort and the per-phase split."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mpi-test_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import gsort  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 28
n = 1 << lg
rng = np.random.default_rng(5)
ctx = gsort.Context()
p = ctx.alloc(n * 4)


def bits(b, signed=False):
    lo = -(1 << (b - 1)) if signed else 0
    hi = (1 << (b - 1)) if signed else (1 << b)
    return lambda: rng.integers(lo, hi, n, dtype=np.int64).astype(np.int32)


cases = {
    "uniform31 (canonical)": None,
    "zipf (canonical)": "zipf",
    "full32": bits(32, True),
    "bits30": bits(30), "bits29": bits(29), "bits28": bits(28), "bits24": bits(24),
    "bits20": bits(20), "bits16": bits(16), "bits8": bits(8),
    "all_equal": lambda: np.full(n, 12345, dtype=np.int32),
    "sorted": lambda: np.arange(n, dtype=np.int32),
    "reverse": lambda: np.arange(n, 0, -1, dtype=np.int32),
    "gauss": lambda: np.clip(rng.normal(0, 1e6, n), -2**31, 2**31 - 1).astype(np.int32),
}
only = set(sys.argv[2].split(",")) if len(sys.argv) > 2 else None  # e.g. zipf,bits16
for name, make in cases.items():
    if only and name.split()[0] not in only:
        continue
    if make is None:
        ctx.generate(gsort.UNIFORM, 42, 0, n, p)
    elif make == "zipf":
        ctx.generate(gsort.ZIPF, 42, 0, n, p)
    else:
        ctx.to_device(make(), p)
    ctx.radix(p, n)
    st = [ctx.radix(p, n)[2] for _ in range(5)]
    f = lambda k: sum(s[k] for s in st) / len(st)  # noqa: E731
    lv = [sum(s["ms_level"][i] for s in st) / len(st) for i in range(4)]
    print(f"{name:22s} {f('ms_total'):8.3f} ms  ({n / f('ms_total') / 1e6:6.1f} GKeys/s)  "
          f"hist {f('ms_hist'):.3f} levels {' '.join(f'{x:.3f}' for x in lv)} "
          f"K11 {f('ms_bucket_sort'):.3f} passes {st[-1]['passes_run']} plan {ctx.last_plan()}",
          flush=True)
ctx.free(p)
ctx.close()
