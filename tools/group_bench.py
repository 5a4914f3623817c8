#!/usr/bin/env python3
"""group_bench.py -- P in-process ranks on ONE GPU (development tool, not the bench contract).

Runs the distributed radix / sample sort with P contexts of one process sharing one GPU (the
in-process rank group: device copies instead of RCCL) and reports the device time of every
phase summed over the ranks, i.e. the per-GPU work the distributed algorithm adds.  Usage:
    python group_bench.py [--ranks 8] [--keys-log2 25] [--algo radix] [--steps 5]
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-test_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--keys-log2", type=int, default=25)
    ap.add_argument("--algo", default="radix")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1, help="untimed calls per rank first")
    ap.add_argument("--local", default="msd")
    ap.add_argument("--dist", choices=["uniform", "zipf"], default="uniform")
    ap.add_argument("--detail", action="store_true",
                    help="stderr: every step's wall time and phases per rank (outlier hunting)")
    a = ap.parse_args()
    import torch  # noqa: F401
    import gsort
    P, n = a.ranks, 1 << a.keys_log2
    grp = gsort.Group(P)
    out = [None] * P
    out_walls = [None] * P
    barrier = threading.Barrier(P)

    def worker(r):
        with gsort.Context(rank=r, group=grp) as c:
            c.set_local_algo(gsort.LOCAL_MSD if a.local == "msd" else gsort.LOCAL_LSD)
            d = c.alloc(n * 4)
            c.generate(gsort.UNIFORM if a.dist == "uniform" else gsort.ZIPF, 42, r * n, n, d)
            c.reserve(n)
            fn = c.radix if a.algo == "radix" else c.sample
            for _ in range(a.warmup):
                barrier.wait()
                fn(d, n)
            sts, walls = [], []
            for _ in range(a.steps):  # each step between two barriers of all ranks
                barrier.wait()
                t0 = time.perf_counter()
                _, n_out, st = fn(d, n)
                sts.append(st)
                barrier.wait()
                walls.append(time.perf_counter() - t0)
            wall = sum(walls) / a.steps
            out_walls[r] = walls
            if a.detail:
                for i, (w_, st_) in enumerate(zip(walls, sts)):
                    print(f"step {i} rank {r}: wall {w_ * 1e3:.3f} total {st_['ms_total']:.3f} "
                          f"local {st_['ms_local_sort']:.3f} sample {st_['ms_sample']:.3f} "
                          f"exch {st_['ms_exchange']:.3f} merge {st_['ms_merge']:.3f}",
                          file=sys.stderr, flush=True)
            keys = ("ms_total", "ms_local_sort", "ms_sample", "ms_exchange", "ms_merge",
                    "ms_hist", "ms_bucket_sort")
            out[r] = {k: sum(s[k] for s in sts) / len(sts) for k in keys}
            out[r]["wall_ms"] = wall * 1e3
            c.free(d)

    th = [threading.Thread(target=worker, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    grp.close()
    tot = {k: round(sum(o[k] for o in out), 4) for k in out[0]}
    in_order = [round(max(w[i] for w in out_walls) * 1e3, 4) for i in range(a.steps)]
    steps = sorted(in_order)
    med = steps[len(steps) // 2]
    print(json.dumps({"ranks": P, "keys_per_rank": n, "algo": a.algo, "dist": a.dist,
                      "sum_over_ranks_ms": tot,
                      "wall_ms": round(max(o["wall_ms"] for o in out), 4),
                      "step_ms": [round(x, 4) for x in steps],
                      "step_ms_in_order": in_order, "warmup": a.warmup,
                      "median_step_ms": round(med, 4),
                      "median_ms_per_2p28_keys": round(med / P * (1 << 28) / n, 4)}))


if __name__ == "__main__":
    main()
