"""bench.py's N > 1 output check (verify_rows) on CPU, with the rows a gloo all_gather of
world_size 2 delivers (tests/test_dist_protocol_cpu.py runs the protocol itself the same way)."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

M64 = (1 << 64) - 1


def mix64(z):
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9 & M64
    z = (z ^ (z >> 27)) * 0x94D049BB133111EB & M64
    return z ^ (z >> 31)


def s64(x):
    return x - (1 << 64) if x >= 1 << 63 else x


def row(inp, out):
    """A rank's row as bench.py builds it (K9's fingerprint restated in Python)."""
    fi = [mix64(int(v) & 0xFFFFFFFF) for v in inp]
    fo = [mix64(int(v) & 0xFFFFFFFF) for v in out]
    x_in = x_out = 0
    for v in fi:
        x_in ^= v
    for v in fo:
        x_out ^= v
    srt = bool(np.all(out[1:] >= out[:-1])) if len(out) else True
    return [s64(sum(fi) & M64), s64(sum(fo) & M64), s64(x_in), s64(x_out), int(srt), len(out),
            int(out[0]) if len(out) else 0, int(out[-1]) if len(out) else 0]


def blocks(seed=1, n=64, P=2):
    keys = np.random.default_rng(seed).integers(-2**31, 2**31, n * P, dtype=np.int64)
    ins = np.split(keys.astype(np.int32), P)
    outs = np.split(np.sort(keys).astype(np.int32), P)
    return ins, outs


def test_verify_rows_accepts_the_global_sort():
    ins, outs = blocks()
    assert bench.verify_rows([row(i, o) for i, o in zip(ins, outs)], 64, "radix")


def test_verify_rows_rejects_a_misrouted_exchange():
    """The ranks' pieces swapped: every rank sorted, same multiset, wrong global order."""
    ins, outs = blocks()
    assert not bench.verify_rows([row(ins[0], outs[1]), row(ins[1], outs[0])], 64, "radix")


def test_verify_rows_rejects_a_lost_key_and_an_unsorted_rank():
    ins, outs = blocks()
    bad = outs[1].copy()
    bad[5] = bad[4]  # one key replaced by a copy of its neighbour: still sorted
    assert not bench.verify_rows([row(ins[0], outs[0]), row(ins[1], bad)], 64, "radix")
    uns = outs[1][::-1].copy()
    assert not bench.verify_rows([row(ins[0], outs[0]), row(ins[1], uns)], 64, "radix")


def test_verify_rows_sample_sizes_may_differ():
    """Sample sort: ranks keep bucket-sized blocks; radix: exactly n_local each."""
    ins, outs = blocks()
    allk = np.concatenate(outs)
    o = [allk[:40], allk[40:]]
    rows = [row(ins[0], o[0]), row(ins[1], o[1])]
    assert bench.verify_rows(rows, 64, "sample")
    assert not bench.verify_rows(rows, 64, "radix")


def _gloo_rank(rank, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    ins, outs = blocks(seed=9)
    mine = torch.tensor(row(ins[rank], outs[rank]), dtype=torch.int64)
    rows = [torch.zeros_like(mine) for _ in range(2)]
    dist.all_gather(rows, mine)
    q.put((rank, bench.verify_rows([[int(x) for x in r.tolist()] for r in rows], 64, "radix")))
    dist.destroy_process_group()


def test_verify_rows_through_gloo_world_size_2():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_rank, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    res = dict(q.get(timeout=5) for _ in range(2))
    assert res == {0: True, 1: True}


def _stats(ms_exchange, exchanges, pair):
    return {"ms_exchange": ms_exchange, "exchanges": exchanges, "max_pair_bytes": pair}


def test_exchange_line_prices_the_largest_pair_on_one_link():
    """N > 1: per exchange, the largest (source, destination) pair over one xGMI link."""
    st = [_stats(2.0, 1, 153 * 10**6), _stats(2.0, 1, 153 * 10**6)]
    ex = bench.exchange_line(st)
    assert ex["bound"] == "xgmi" and ex["per_exchange_ms"] == 2.0
    assert ex["achieved_link_GBps"] == 76.5 and ex["frac"] == 0.5
    assert bench.exchange_line([_stats(0.0, 0, 0)]) is None  # one rank: no exchange


def test_strong_line_is_configs2_at_every_n():
    """The configs[2] block of an N > 1 line: 2^31 keys in total whatever N is (strong
    scaling), GKeys/s from the slowest rank's step time, its own verification flag."""
    for world in (2, 4, 8):
        st = [_stats(1.0, 1, 1 << 28)] * 3
        line = bench.strong_line(1 << 31, world, 10.0, True, st)
        assert line["total_keys"] == 1 << 31 and line["keys_per_gpu"] == (1 << 31) // world
        assert line["scaling"] == "strong" and line["n_gpus"] == world
        assert line["GKeys_s"] == round((1 << 31) / 10e-3 / 1e9, 3)
        assert line["verified"] is True and line["steps"] == 3
        assert line["exchange"]["bound"] == "xgmi"
        assert "configs[2]" in line["config"]
