#!/usr/bin/env python3
"""recv_probe.py [log2 n [bits,bits..]] -- the distributed radix's per-GPU path on one GPU (development tool):
a one-rank group with GSORT_FORCE_DIST=1 runs sender grouping, radix select, the packed
self-exchange and the receive sort.  Key widths set the receive bucket size, i.e. the
weak-scaling shape at 2^28 keys per GPU: 31-bit keys give 8192-key 16-bit buckets (P = 1),
30-bit 16384 (P = 2), 29-bit 32768 (P = 4), 28-bit 65536 (P = 8), 27-bit 131072.
GSORT_RECV_CX picks the kernels (K11g classes vs K18c).  Prints ms per sort and phases;
run it under rocprofv3 --kernel-trace for the per-kernel split (the second argument keeps only the
listed key widths, e.g. 29 for the P = 4 shape alone: tools/profile_pipes.sh with PIPES_CMD)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "mpi-test_amd")):
    sys.path.insert(0, p)
os.environ["GSORT_FORCE_DIST"] = "1"

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import gsort  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 28
only = {int(b) for b in sys.argv[2].split(",")} if len(sys.argv) > 2 else None
n = 1 << lg
rng = np.random.default_rng(9)
grp = gsort.Group(1)
ctx = gsort.Context(group=grp)
p = ctx.alloc(n * 4)
for name, bits in [("uniform31 (8192-key buckets)", 31), ("bits30 (16384-key buckets)", 30),
                   ("bits29 (32768-key buckets)", 29), ("bits28 (65536-key buckets)", 28),
                   ("bits27 (131072-key buckets)", 27)]:
    if only is not None and bits not in only:
        continue
    if bits == 31:
        ctx.generate(gsort.UNIFORM, 42, 0, n, p)
    else:
        ctx.to_device(rng.integers(0, 1 << bits, n, dtype=np.int64).astype(np.int32), p)
    out, m, _ = ctx.radix(p, n)
    fp, fin = ctx.fingerprint(out, m), ctx.fingerprint(p, n)
    ok = fp["sorted"] and fp["sum"] == fin["sum"]
    st = [ctx.radix(p, n)[2] for _ in range(5)]
    f = lambda k: sum(s[k] for s in st) / len(st)  # noqa: E731
    print(f"{name:34s} {f('ms_total'):7.3f} ms  sender hist {f('ms_hist'):.3f} levels "
          f"{sum(s['ms_level'][0] for s in st) / 5:.3f} {sum(s['ms_level'][1] for s in st) / 5:.3f} "
          f"select {f('ms_sample'):.3f} exch {f('ms_exchange'):.3f} recv {f('ms_merge'):.3f} "
          f"(6 B/key: {n * 6 / (f('ms_merge') * 1e-3) / 1e9:.0f} GB/s)  ok {ok}", flush=True)
ctx.free(p)
ctx.close()
grp.close()
