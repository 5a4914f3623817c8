#!/usr/bin/env python3
"""k3_stamps.py [keys_log2] -- where K3r's and K3a's time goes, per phase.

Needs the diagnostic build: make -C mpi-test_amd VARIANT=stamps EXTRA=-DGSORT_STAMPS lib
(loaded through GSORT_LIB; the product build has no stamps).  Thread 0 of every K3r / K3a
workgroup of the sampled plan writes s_memrealtime (100 MHz) at 6 points, each behind a
workgroup barrier: entry, loads landed, ranked, reservations returned, scattered into LDS,
stores completed (gsort_kernels.hip, K3_STAMP).  Prints, per kernel, the mean / median
duration of every phase over the workgroups of the last sort, the workgroup lifetime, the
kernel span and the mean number of workgroups alive (lifetime sum / span)."""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-test_amd"))
os.environ.setdefault("GSORT_LIB", os.path.join(ROOT, "mpi-test_amd", "lib", "libgsort_stamps.so"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import gsort  # noqa: E402

WGS = 32768
PHASES = ["prologue", "load", "rank", "reserve", "scatter", "store"]


def main():
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 28
    n = 1 << lg
    with gsort.Context(device=0) as ctx:
        d_in = ctx.alloc(n * 4)
        ctx.generate(gsort.UNIFORM, 42, 0, n, d_in)
        ctx.reserve(n)
        buf = ctx.alloc(2 * WGS * 8 * 8)
        if gsort.lib().gsort_diag_stamps(ctypes.c_void_p(buf)) != 0:
            sys.exit("gsort_diag_stamps failed (not the stamps build?)")
        for _ in range(3):
            ctx.radix(d_in, n, stats=False)
        ctx.to_device(np.zeros(2 * WGS * 8, dtype=np.uint64).view(np.int32), buf)
        ctx.radix(d_in, n, stats=False)
        assert ctx.last_plan() == 1, "the sampled plan did not run"
        st = ctx.to_host(buf, 2 * WGS * 8 * 2).view(np.uint64).reshape(2, WGS, 8)
        ctx.free(buf)
        ctx.free(d_in)
    for ki, name in enumerate(["K3r (level 3, u32 out)", "K3a (level 2, u16 out)"]):
        s = st[ki]
        s = s[s[:, 5] > 0].astype(np.int64)
        if not len(s):
            print(name, "no stamps")
            continue
        t = s[:, [6, 0, 1, 2, 3, 4, 5]]  # entry, tile known, loads, rank, reserve, scatter, store
        d = np.diff(t, axis=1) * 10.0  # ns (100 MHz)
        life = (t[:, 6] - t[:, 0]) * 10.0
        span = (t[:, 6].max() - t[:, 0].min()) * 10.0
        print(f"{name}: {len(s)} workgroups, span {span / 1e3:.1f} us, "
              f"lifetime mean {life.mean() / 1e3:.2f} us median {np.median(life) / 1e3:.2f} us, "
              f"workgroups alive (mean) {life.sum() / span:.1f}")
        for j, ph in enumerate(PHASES):
            print(f"   {ph:8s} mean {d[:, j].mean() / 1e3:6.2f} us  median {np.median(d[:, j]) / 1e3:6.2f} us"
                  f"  share {d[:, j].sum() / life.sum():.3f}")


if __name__ == "__main__":
    main()
