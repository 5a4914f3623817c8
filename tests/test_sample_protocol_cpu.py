"""The packed sample-sort protocol (gsort_dist.cpp sample_dist, round 6) over gloo, on CPU.

The GPU path never sorts a rank's block before the exchange: it groups the block by the top 16
bits of the ordered key (the radix sender's grouping; inside a group the keys stay in no
particular order), sorts only the groups holding the reference's regular samples and
splitters, and reads every quantity of mpi_sample_sort.c off the grouped block.  This test
restates that protocol step by step across world_size = 2 and 4 gloo processes and checks each
step against the reference's own definition on the fully sorted block:
  1. group the block (keys shuffled inside their groups), bounds gb;
  2. regular sample i = sorted[i * interval] (mpi_sample_sort.c:94-104): the group holding
     position i * interval sorted, the key read at that position;
  3. splitters on the root (:107-125: the gathered samples sorted, S[(i+1)k]), broadcast;
  4. the splitters' groups sorted, #keys <= s_j (and < s_j) by binary search in the group;
  5. the bucket matrix (the reference's "Bucket j=len" lines, :156-158) and the cut -- the
     reference's bucket rule (:148-155), or the duplicate-aware rule (gsort_plan_split,
     balanced) with the product's host planner;
  6. the packed exchange: low 16 bits per key + one count per (destination, 16-bit bucket)
     over the destination's bucket range [s_{q-1} >> 16, s_q >> 16];
and every rank checks that it ends up with exactly the keys the reference gives its bucket.
"""
import os
import socket

import numpy as np
import pytest

FLIP = np.uint64(0x80000000)


def _ordered(a):
    return (a.astype(np.int64).astype(np.uint64) & np.uint64(0xFFFFFFFF)) ^ FLIP


def _worker(rank, world, port, case, balanced, errq):
    try:
        import sys
        import torch
        import torch.distributed as dist
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, os.path.join(root, "mpi-test_amd"))
        import gsort
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        P, me = world, rank
        rng = np.random.default_rng(2000 + rank)
        n = 30000 + int(rng.integers(0, 5000))
        if case == "dups":    # few values: splitters repeat, groups hold every copy
            keys = rng.choice(np.array([-7, 0, 5, 65536, 2**31 - 1], np.int32), n)
        elif case == "narrow":  # every key in a handful of 16-bit groups
            keys = rng.integers(-3 * 65536, 3 * 65536, n).astype(np.int32)
        else:
            keys = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
        n_all = [None] * P
        dist.all_gather_object(n_all, n)
        N = sum(n_all)
        B = -(-N // P)
        k = 2 * P - 1
        S = P - 1
        interval = B // k
        # 1. grouped, unsorted inside a group
        u = _ordered(keys)
        top = (u >> np.uint64(16)).astype(np.int64)
        order = np.lexsort((rng.random(n), top))
        grouped = u[order].copy()
        gb = np.searchsorted(top[order], np.arange(65537), "left")
        sorted_u = np.sort(u)

        def sort_group(h):
            grouped[gb[h]:gb[h + 1]] = np.sort(grouped[gb[h]:gb[h + 1]])
        # 2. the regular samples from their groups
        pos = np.arange(k, dtype=np.int64) * interval
        hs = np.searchsorted(gb, pos, "right") - 1
        for h in np.unique(hs):
            sort_group(h)
        samp = grouped[pos]
        assert np.array_equal(samp, sorted_u[pos]), "regular samples"
        # 3. root: sort the P*k samples, splitters S[(i+1)*k]; broadcast
        alls = [None] * P
        dist.all_gather_object(alls, samp)
        spl = np.sort(np.concatenate(alls))[[(i + 1) * k for i in range(S)]]
        # 4. the splitters' groups sorted, counts by binary search inside the group
        for h in np.unique((spl >> np.uint64(16)).astype(np.int64)):
            sort_group(h)

        def count_below(x):  # keys < x (ordered u64), as k_count_below16
            h = int(x >> np.uint64(16))
            if h >= 65536:
                return n
            lo16 = int(x & np.uint64(0xFFFF))
            a, b = gb[h], gb[h + 1]
            return int(a + np.searchsorted(grouped[a:b] & np.uint64(0xFFFF), lo16, "left"))
        le = np.array([count_below(s + np.uint64(1)) for s in spl], np.uint64)
        lt = np.array([count_below(s) for s in spl], np.uint64)
        assert np.array_equal(le, np.searchsorted(sorted_u, spl, "right")), "keys <= s_j"
        rows = [None] * P
        dist.all_gather_object(rows, (le, lt))
        # 5. the bucket matrix and the cut
        M = np.zeros((P, P), np.int64)
        for p in range(P):
            if not balanced:
                b = np.concatenate([[0], rows[p][0].astype(np.int64), [n_all[p]]])
                M[p] = np.diff(b)
            else:
                LT = np.stack([r[1] for r in rows]).astype(np.uint64)
                LE = np.stack([r[0] for r in rows]).astype(np.uint64)
                snd, _ = gsort.plan_split(np.array(n_all, np.uint64), LT, LE, p, balanced=True)
                M[p] = snd
        # the reference's "Bucket j=len" counts (mpi_sample_sort.c:148-158) on the sorted block
        if not balanced:
            ref_b = np.zeros(P, np.int64)
            for v in sorted_u:
                j = next((j for j in range(S) if v <= spl[j]), S)
                ref_b[j] += 1
            assert np.array_equal(M[me], ref_b), "bucket matrix row"
        cut = np.concatenate([[0], np.cumsum(M[me])])
        recv = M[:, me]
        lo = [0 if q == 0 else int(spl[q - 1]) for q in range(P)]
        hi = [0xFFFFFFFF if q == S else int(spl[q]) for q in range(P)]
        hlo = [x >> 16 for x in lo]
        nh = [(hi[q] >> 16) - hlo[q] + 1 for q in range(P)]
        # 6. the packed exchange (all_gather_object stands in for the grouped send/recv)
        low16 = (grouped & np.uint64(0xFFFF)).astype(np.int64)
        sends = []
        for q in range(P):
            a, b = cut[q], cut[q + 1]
            h = np.arange(hlo[q], hlo[q] + nh[q])
            cnt = np.clip(np.minimum(gb[h + 1], b) - np.maximum(gb[h], a), 0, None)
            assert cnt.sum() == b - a, "destination's bucket range holds its run"
            sends.append((low16[a:b].copy(), cnt))
        allsend = [None] * P
        dist.all_gather_object(allsend, sends)
        rebuilt = []
        for p in range(P):
            pay, cnt = allsend[p][me]
            assert len(pay) == recv[p]
            h = np.repeat(np.arange(hlo[me], hlo[me] + nh[me], dtype=np.uint64), cnt)
            rebuilt.append((h << np.uint64(16)) | pay.astype(np.uint64))
        mine = np.sort(np.concatenate(rebuilt))
        allk = [None] * P
        dist.all_gather_object(allk, u)
        every = np.sort(np.concatenate(allk))
        if not balanced:  # the reference's bucket: (s_{me-1}, s_me]
            lo_ok = every > spl[me - 1] if me > 0 else np.ones(len(every), bool)
            hi_ok = every <= spl[me] if me < S else np.ones(len(every), bool)
            assert np.array_equal(mine, every[lo_ok & hi_ok]), (case, me)
        else:  # the global order cut at the planned sizes
            start = int(M[:, :me].sum())
            assert np.array_equal(mine, every[start:start + len(mine)]), (case, me)
        dist.destroy_process_group()
    except Exception:  # report to the parent
        import traceback
        errq.put((rank, traceback.format_exc()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("case,balanced", [("uniform", False), ("dups", False),
                                           ("narrow", False), ("dups", True)])
def test_packed_sample_protocol_gloo(world, case, balanced):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, balanced, errq))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, errs[0][1]
    assert all(p.exitcode == 0 for p in procs)
