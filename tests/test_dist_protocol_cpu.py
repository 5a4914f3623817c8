"""The distributed radix protocol over real multi-process communication, on CPU (gloo).

The product's N > 1 path (gsort_runtime.cpp, radix_dist_exact) runs on GPUs over RCCL; its
host-side protocol is restated here step by step and driven across world_size = 2 and 4 gloo
processes, with the product's own host planner (gsort_plan_split, C-ABI, no GPU) deciding the
cuts:
  1. every rank groups its block by the top 16 bits of the ordered key (here: sorts it);
  2. radix select of the boundary keys v_q: 4 rounds of 8 bits, each rank counts its keys below
     257 thresholds per boundary, the counts are all-gathered, every rank picks the same digit;
  3. gsort_plan_split turns the per-rank counts below / up to v_q into the cuts;
  4. the packed exchange: the low 16 bits of every key plus, per (destination, 16-bit bucket),
     a count -- the receiver rebuilds the keys from (bucket, low bits);
and every rank checks that it ends up with exactly its global block [qB, (q+1)B).
"""
import os
import socket

import numpy as np
import pytest

FLIP = np.uint64(0x80000000)


def _ordered(a):
    return (a.astype(np.int64).astype(np.uint64) & np.uint64(0xFFFFFFFF)) ^ FLIP


def _worker(rank, world, port, case, errq):
    try:
        import sys
        import torch
        import torch.distributed as dist
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, os.path.join(root, "mpi-test_amd"))
        import gsort
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        rng = np.random.default_rng(1000 + rank)
        n = int(rng.integers(0, 40000)) if case != "tiny" else int(rng.integers(0, 3))
        if case == "dups":
            keys = rng.choice(np.array([-7, 0, 5, 2**31 - 1], np.int32), n)
        else:
            keys = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
        P, me = world, rank
        block = np.sort(keys)                                   # step 1
        u = _ordered(block)
        n_all = torch.zeros(P, dtype=torch.int64)
        dist.all_gather_into_tensor(n_all, torch.tensor([n], dtype=torch.int64))
        n_all = n_all.numpy().astype(np.uint64)
        N = int(n_all.sum())
        B = -(-N // P) if N else 0
        nb = P - 1
        g = [min((q + 1) * B, N) for q in range(nb)]
        prefix = [0] * nb
        dsel = [0] * nb
        for k in range(4):                                       # step 2
            shift = 24 - 8 * k
            xs = np.array([[prefix[q] + (d << shift) for d in range(257)] for q in range(nb)],
                          dtype=np.uint64)
            mine = np.searchsorted(u, xs.ravel(), "left").astype(np.int64)
            allc = [torch.zeros(nb * 257, dtype=torch.int64) for _ in range(P)]
            dist.all_gather(allc, torch.from_numpy(mine))
            allc = np.stack([a.numpy() for a in allc]).reshape(P, nb, 257)
            for q in range(nb):
                if g[q] >= N:
                    continue
                tot = allc[:, q, :256].sum(axis=0)
                best = int(np.nonzero(tot <= g[q])[0].max())
                dsel[q] = best
                prefix[q] += best << shift
        lt = np.zeros((P, nb), np.uint64)
        le = np.zeros((P, nb), np.uint64)
        for p in range(P):
            for q in range(nb):
                lt[p, q] = n_all[p] if g[q] >= N else allc[p, q, dsel[q]]
                le[p, q] = n_all[p] if g[q] >= N else allc[p, q, dsel[q] + 1]
        send, recv = gsort.plan_split(n_all, lt, le, me)          # step 3
        cut = np.concatenate([[0], np.cumsum(send)]).astype(np.int64)
        lo = [0 if q == 0 else (0xFFFFFFFF if g[q - 1] >= N else prefix[q - 1]) for q in range(P)]
        hi = [0xFFFFFFFF if q == P - 1 else (0xFFFFFFFF if g[q] >= N else prefix[q])
              for q in range(P)]
        hlo = [x >> 16 for x in lo]
        nh = [(hi[q] >> 16) - hlo[q] + 1 for q in range(P)]
        gb = np.searchsorted(u, np.arange(65537, dtype=np.uint64) << np.uint64(16), "left")
        low16 = (u & np.uint64(0xFFFF)).astype(np.int64)
        sends = []                                               # step 4: payload + counts
        for q in range(P):
            a, b = cut[q], cut[q + 1]
            h = np.arange(hlo[q], hlo[q] + nh[q])
            cnt = np.clip(np.minimum(gb[h + 1], b) - np.maximum(gb[h], a), 0, None)
            sends.append((torch.from_numpy(low16[a:b].copy()),
                          torch.from_numpy(cnt.astype(np.int64))))
        got = []
        for step in range(P):  # pairwise exchange in a fixed schedule (gloo send/recv)
            for q in range(P):
                p = (q - step) % P                               # p sends to q at this step
                if me == p and me == q:
                    got.append((p, *sends[q]))
                elif me == p:
                    dist.send(torch.tensor([sends[q][0].numel()]), q)
                    if sends[q][0].numel():
                        dist.send(sends[q][0], q)
                        dist.send(sends[q][1], q)
                elif me == q:
                    m = torch.zeros(1, dtype=torch.int64)
                    dist.recv(m, p)
                    pay = torch.zeros(int(m.item()), dtype=torch.int64)
                    cnt = torch.zeros(nh[me], dtype=torch.int64)
                    if int(m.item()):
                        dist.recv(pay, p)
                        dist.recv(cnt, p)
                    got.append((p, pay, cnt))
        got.sort(key=lambda t: t[0])
        assert [int(t[1].numel()) for t in got] == [int(x) for x in recv]
        rebuilt = []
        for _, pay, cnt in got:
            if not pay.numel():
                continue
            h = np.repeat(np.arange(hlo[me], hlo[me] + nh[me], dtype=np.uint64), cnt.numpy())
            rebuilt.append(((h << np.uint64(16)) | pay.numpy().astype(np.uint64)) ^ FLIP)
        mine_keys = (np.sort(np.concatenate(rebuilt)).astype(np.int64) if rebuilt
                     else np.zeros(0, np.int64))
        mine_keys = ((mine_keys + 2**31) % 2**32 - 2**31).astype(np.int32)
        allk = [None] * P
        dist.all_gather_object(allk, keys)
        ref = np.sort(np.concatenate(allk))[me * B:(me + 1) * B] if N else np.zeros(0, np.int32)
        assert np.array_equal(np.sort(mine_keys), ref), (case, me)
        dist.destroy_process_group()
    except Exception as e:  # report to the parent
        import traceback
        errq.put((rank, traceback.format_exc()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("case", ["uniform", "dups", "tiny"])
def test_distributed_radix_protocol_gloo(world, case):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, errq)) for r in range(world)]
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
