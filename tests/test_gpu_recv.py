"""Receive side of the distributed sorts: K18c (one-read counting sort of a 16-bit bucket's low
16 bits) against np.sort, through in-process rank groups on one GPU.

GSORT_RECV_CX routes the receive buckets: 1 = every bucket through K18c (the K11g classes
too), 5 = only buckets past kLocalMax (the default), -1 = the round-2 kernels (K11g and the
two-read K18).  The cases reach what K18c must get right: pieces of P ranks starting at any
2-B / 4-B alignment, empty pieces, buckets of one value, and bins of >= 65 536 copies of one
value in buckets past 65 535 keys, whose u16 halves wrap (low half: the carry into the
neighbour bin; high half; both) -- and, with the default u8 bins, every bucket holding >= 256
copies of one key (redone with u16 bins).  The reference's own final order is the sorted multiset
(mpi_radix_sort.c:185-192, mpi_sample_sort.c:174), so np.sort is the oracle (bit-exact).
"""
import numpy as np
import pytest

from test_gpu_sort import run_group

pytestmark = pytest.mark.gpu


def _check(res, keys, P, algo):
    ref = np.sort(keys)
    got = np.concatenate([res[r][0] for r in range(P)])
    assert np.array_equal(got, ref)
    if algo == "radix":  # exact splitters: rank q holds [qB, (q+1)B)
        B = -(-keys.size // P)
        for q in range(P):
            assert np.array_equal(res[q][0], ref[q * B:(q + 1) * B]), q


def _wraps(rng, n):
    """Three 16-bit buckets: one with 150 000 copies of an even low half (two low-half wraps,
    carries into the odd neighbour) and 140 000 of that neighbour (high-half wraps, some
    carries landing on a full high half), one with 200 000 copies of an odd low half, one
    uniform; all under kHxMax = 2^20 keys per bucket and rank."""
    hot = np.concatenate([
        np.full(150000, 0x00070010, np.int64), np.full(140000, 0x00070011, np.int64),
        np.full(200000, -0x0003FFFF, np.int64),
        0x00090000 + rng.integers(0, 1 << 16, 120000)])
    rest = rng.integers(-2**31, 2**31, max(n - hot.size, 0))
    return np.concatenate([hot, rest]).astype(np.int32)


CASES = {
    # P = 8 weak-scaling shape: 65 536-key buckets (2^22 keys of 22 bits over 8 ranks)
    "bits22": lambda rng: rng.integers(0, 1 << 22, 1 << 22),
    # buckets of every K11g class and past kLocalMax (16-bit buckets of ~4K .. ~260K keys)
    "classes": lambda rng: rng.integers(-(1 << 22), 1 << 22, 3 << 20) >> rng.integers(0, 6, 3 << 20),
    "wraps": lambda rng: _wraps(rng, 1 << 20),
    "one_value": lambda rng: np.full(700001, -12345),
    "few_values": lambda rng: rng.choice(np.array([3, 4, 65539, -7]), 500000),
}


@pytest.mark.parametrize("cx", [1, 3, 4, 5, -1])
@pytest.mark.parametrize("algo", ["radix", "sample"])
@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("P", [2, 3, 8])
def test_receive_buckets(gsort, monkeypatch, case, algo, cx, P):
    monkeypatch.setenv("GSORT_RECV_CX", str(cx))
    rng = np.random.default_rng(hash((case, P)) % 2**32)
    keys = np.asarray(CASES[case](rng)).astype(np.int32)
    rng.shuffle(keys)
    if algo == "radix":  # uneven blocks: pieces at any alignment
        cuts = np.sort(rng.integers(0, keys.size + 1, P - 1))
    else:  # regular sampling wants the reference's equal blocks (mpi_sample_sort.c:82)
        B = -(-keys.size // P)
        cuts = np.arange(1, P) * B
    blocks = np.split(keys, cuts)
    res = run_group(gsort, blocks, algo)
    _check(res, keys, P, algo)


@pytest.mark.parametrize("algo", ["radix", "sample"])
@pytest.mark.parametrize("case", list(CASES))
@pytest.mark.parametrize("P", [2, 8])
def test_receive_buckets_u16_bins(gsort, monkeypatch, case, algo, P):
    """K18c's u16 bins (GSORT_RECV_CB=16; the default is u8 bins, whose buckets with >= 256
    copies of one key -- wraps, one_value, few_values -- are redone with u16 bins) on every
    bucket (GSORT_RECV_CX=1)."""
    monkeypatch.setenv("GSORT_RECV_CX", "1")
    monkeypatch.setenv("GSORT_RECV_CB", "16")
    rng = np.random.default_rng(hash((case, P, "u16")) % 2**32)
    keys = np.asarray(CASES[case](rng)).astype(np.int32)
    rng.shuffle(keys)
    B = -(-keys.size // P)
    res = run_group(gsort, np.split(keys, np.arange(1, P) * B), algo)
    _check(res, keys, P, algo)


@pytest.mark.parametrize("cx", [1, 5])
def test_receive_one_rank_forced(gsort, monkeypatch, cx):
    """A one-rank group on the distributed path (GSORT_FORCE_DIST, bench.py's dist_p1): one
    piece per bucket, 8192-key buckets (K11g class 2, or K18c with cx = 1)."""
    monkeypatch.setenv("GSORT_FORCE_DIST", "1")
    monkeypatch.setenv("GSORT_RECV_CX", str(cx))
    rng = np.random.default_rng(cx)
    keys = rng.integers(-2**31, 2**31, (1 << 22) + 77).astype(np.int32)
    res = run_group(gsort, [keys], "radix")
    _check(res, keys, 1, "radix")


def _run_group_seq(gsort, seq_blocks, algo):
    """Like run_group, but every rank's ONE context sorts the inputs of seq_blocks in turn (the
    receive launches of call i are shaped by call i-1's list counts: spec_recv_launch)."""
    import threading
    P = len(seq_blocks[0])
    grp = gsort.Group(P)
    res, errs = [[None] * P for _ in seq_blocks], []

    def worker(r):
        try:
            with gsort.Context(rank=r, group=grp) as c:
                fn = c.radix if algo == "radix" else c.sample
                for i, blocks in enumerate(seq_blocks):
                    p = c.alloc(max(blocks[r].size, 1) * 4)
                    c.to_device(blocks[r], p)
                    out, n, _ = fn(p, blocks[r].size)
                    res[i][r] = (c.to_host(out, n), None, None)
                    c.free(p)
        except Exception as e:
            errs.append((r, e))

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not [r for r, t in enumerate(th) if t.is_alive()], "group ranks hung"
    grp.close()
    if errs:
        raise errs[0][1]
    return res


@pytest.mark.parametrize("cx", [3, 4])
@pytest.mark.parametrize("algo", ["radix", "sample"])
@pytest.mark.parametrize("P", [2, 4])
def test_receive_launch_shapes_from_previous_call(gsort, monkeypatch, algo, cx, P):
    """The receive sort's launches are queued before the host reads the list counts, shaped by
    the previous call's counts: a context sorting inputs whose bucket classes
    differ call to call -- the guess too small, too large, for lists that are now empty or past
    kHxMax -- still sorts every bucket exactly once."""
    monkeypatch.setenv("GSORT_RECV_CX", str(cx))
    rng = np.random.default_rng(77 + P)
    order = ["classes", "bits22", "one_value", "classes", "few_values", "wraps", "bits22",
             "big_bucket", "classes"]
    gens = dict(CASES)
    # one 16-bit bucket past kHxMax (2^20 keys) on the receiving rank: list 0 goes to the MSD
    # levels (spec_recv_launch's K18c skips it on the device)
    gens["big_bucket"] = lambda r: np.concatenate([0x00050000 + r.integers(0, 1 << 16, 3 << 20),
                                                    r.integers(-2**31, 2**31, 1 << 20)])
    seq, keys_all = [], []
    for name in order:
        keys = np.asarray(gens[name](rng)).astype(np.int32)
        rng.shuffle(keys)
        B = -(-keys.size // P)
        seq.append(np.split(keys, np.arange(1, P) * B))
        keys_all.append(keys)
    res = _run_group_seq(gsort, seq, algo)
    for i, keys in enumerate(keys_all):
        _check(res[i], keys, P, algo)


@pytest.mark.parametrize("algo", ["radix", "sample"])
@pytest.mark.parametrize("P", [1, 2, 3, 12])
def test_receive_class3_packed_body(gsort, monkeypatch, algo, P):
    """16 384-key buckets (the P = 2 weak-scaling shape; 2^22 keys of 24 bits) on K11g class 3's
    packed body (sort_bucket16: two u16 keys per register, u16 LDS slots): one run straight from
    the entry (P = 1, forced distributed), pieces loaded directly (P = 2, 3) and gathered through
    LDS (P = 12 > kGatherDirectP); plus a few buckets of one value and a ragged tail."""
    if P == 1:
        monkeypatch.setenv("GSORT_FORCE_DIST", "1")
    rng = np.random.default_rng(300 + P)
    keys = np.concatenate([rng.integers(0, 1 << 24, (1 << 22) - 30011),
                           np.full(20000, 0x00A50000 + 7), np.full(10011, 0x00A60000)])
    keys = keys.astype(np.int32)
    rng.shuffle(keys)
    B = -(-keys.size // P)
    res = run_group(gsort, np.split(keys, np.arange(1, P) * B), algo)
    _check(res, keys, P, algo)
