"""GPU parity tests: libgsort's HIP path vs the CPU oracle and the reference's own outputs.

Bit-exact throughout (integer keys).  Small and medium sizes compare whole arrays with the
oracle / the golden fixtures; the 2^28 case (BASELINE config 2) checks size-independent
properties: output sorted, multiset fingerprint of output == input (K9), length preserved.
Multi-rank cases run the distributed algorithm with P ranks on ONE GPU through the
in-process rank group (gsort_create_in_group): same kernels, same routing, device copies in
place of RCCL transfers.
"""
import os
import threading

import numpy as np
import pytest

from conftest import case_input, case_output

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=["msd", "msd_segplan", "lsd"])
def ctx(gsort, request):
    """Both local-sort algorithms (MSD partitions + in-LDS buckets, and stable LSD passes); the
    MSD sort with its default two-level plan front end (K1h/K12h/K3a) and with the segmented
    level-2 plan (K12/K1s/K2s, GSORT_PLAN16=0) that levels 1 and 0 always use."""
    old = os.environ.get("GSORT_PLAN16")
    os.environ["GSORT_PLAN16"] = "0" if request.param == "msd_segplan" else "1"
    try:
        c = gsort.Context()
    finally:
        if old is None:
            os.environ.pop("GSORT_PLAN16")
        else:
            os.environ["GSORT_PLAN16"] = old
    c.set_local_algo(gsort.LOCAL_LSD if request.param == "lsd" else gsort.LOCAL_MSD)
    c.algo = "lsd" if request.param == "lsd" else "msd"
    yield c
    c.close()


def dev(ctx, a):
    p = ctx.alloc(max(a.size, 1) * 4)
    ctx.to_device(a, p)
    return p


def sort_on_gpu(ctx, keys, algo="radix"):
    p = dev(ctx, keys)
    try:
        fn = ctx.radix if algo == "radix" else ctx.sample
        out, n, st = fn(p, keys.size)
        assert n == keys.size
        return ctx.to_host(out, n), st
    finally:
        ctx.free(p)


def test_generator_matches_oracle(ctx, orc):
    for dist in (orc.UNIFORM, orc.ZIPF):
        for start, n in ((0, 1 << 20), (12345, 77777)):
            p = ctx.alloc(n * 4)
            ctx.generate(dist, 42, start, n, p)
            got = ctx.to_host(p, n)
            ctx.free(p)
            assert np.array_equal(got, orc.gen(dist, 42, n, start=start)), (dist, start)


EDGE_SIZES = [0, 1, 2, 3, 63, 64, 65, 1000, 8191, 8192, 8193, 3 * 8192 + 17, 1 << 16,
              (1 << 20) + 7]


@pytest.mark.parametrize("n", EDGE_SIZES)
def test_radix_one_gpu_matches_oracle_sizes(ctx, orc, n):
    keys = orc.gen(orc.UNIFORM, n + 1, n)
    got, st = sort_on_gpu(ctx, keys)
    assert np.array_equal(got, orc.lsd8(keys))


def test_radix_one_gpu_value_edge_cases(ctx, orc):
    rng = np.random.default_rng(1)
    cases = {
        "negatives": rng.integers(-2**31, 2**31, 50000, dtype=np.int64).astype(np.int32),
        "extremes": np.array([2**31 - 1, -2**31, 0, -1, 1, 2**31 - 1, -2**31] * 999,
                             dtype=np.int32),
        "all_equal": np.full(40000, 7, dtype=np.int32),
        "two_values": rng.choice(np.array([5, -5], dtype=np.int32), 30001),
        "sorted": np.arange(70000, dtype=np.int32),
        "reversed": np.arange(70000, 0, -1, dtype=np.int32),
        "low_byte_only": rng.integers(0, 256, 90000).astype(np.int32),
        "zipf": orc.gen(orc.ZIPF, 3, 1 << 18),
    }
    for name, keys in cases.items():
        got, st = sort_on_gpu(ctx, keys)
        assert np.array_equal(got, np.sort(keys)), name
    if ctx.algo == "lsd":  # a single non-trivial digit runs one pass
        _, st = sort_on_gpu(ctx, cases["low_byte_only"])
        assert st["passes_run"] == 1


def _one_hot_bucket(orc):
    rng = np.random.default_rng(7)
    half = np.concatenate([np.full(1 << 19, 123456, dtype=np.int32),
                           orc.gen(orc.UNIFORM, 9, 1 << 19)])
    rng.shuffle(half)
    return half


def _h16_wrap_pair(orc):
    """Two keys whose top 16 bits (ordered) share one packed K1h word, as its low (even) and
    high (odd) half, 2^25 copies each: every K1h workgroup counts > 65535 of both, so both
    halves wrap (and the word carries out) -- the repairs through fix[] must be exact."""
    rng = np.random.default_rng(8)
    a = np.int32(0x12340000)                   # ordered prefix 0x9234 (even)
    b = np.int32(0x12350005)                   # ordered prefix 0x9235 (odd)
    keys = np.where(rng.random(1 << 26) < 0.5, a, b).astype(np.int32)
    keys[::1009] = rng.integers(-2**31, 2**31, keys[::1009].size, dtype=np.int64)
    return keys


def _msd_cases(orc):
    rng = lambda s: np.random.default_rng(s)  # noqa: E731
    return {
        # one bucket / first level only
        # K11 class caps (kLocalCap: 4608, 9216, 16896, 32768; and older caps), one past each
        "n_cap2304": lambda: orc.gen(orc.UNIFORM, 15, 2304),
        "n_cap2304_plus1": lambda: orc.gen(orc.UNIFORM, 16, 2305),
        "n_cap6144": lambda: orc.gen(orc.UNIFORM, 17, 6144),
        "n_cap6144_plus1": lambda: orc.gen(orc.UNIFORM, 18, 6145),
        "n_cap8192": lambda: orc.gen(orc.UNIFORM, 19, 8192),
        "n_cap8192_plus1": lambda: orc.gen(orc.UNIFORM, 20, 8193),
        "n_cap8704": lambda: orc.gen(orc.UNIFORM, 21, 8704),
        "n_cap8704_plus1": lambda: orc.gen(orc.UNIFORM, 22, 8705),
        "n_cap1": lambda: orc.gen(orc.UNIFORM, 11, 4608),
        "n_cap1_plus1": lambda: orc.gen(orc.UNIFORM, 12, 4609),
        "n_cap2": lambda: orc.gen(orc.UNIFORM, 13, 9216),
        "n_cap2_plus1": lambda: orc.gen(orc.UNIFORM, 14, 9217),
        "n_16384": lambda: orc.gen(orc.UNIFORM, 1, 16384),
        "n_16385": lambda: orc.gen(orc.UNIFORM, 2, 16385),
        "n_cap3": lambda: orc.gen(orc.UNIFORM, 25, 16896),
        "n_cap3_plus1": lambda: orc.gen(orc.UNIFORM, 26, 16897),
        "n_localmax": lambda: orc.gen(orc.UNIFORM, 23, 32768),
        "n_localmax_plus1": lambda: orc.gen(orc.UNIFORM, 24, 32769),
        # level-2 children straddling 16 384 keys (class 3 / class 4 of K11)
        "children_16k_2p26_28bit": lambda: rng(9).integers(0, 1 << 28, 1 << 26).astype(np.int32),
        "children_32k_2p26_27bit": lambda: rng(10).integers(0, 1 << 27, 1 << 26).astype(np.int32),
        "uniform31_2p26": lambda: orc.gen(orc.UNIFORM, 6, 1 << 26),
        # top digits trivial: buckets stay oversized down to the last level (digit 0)
        "below_2p16": lambda: rng(7).integers(0, 1 << 16, 1 << 20).astype(np.int32),
        "below_2p24": lambda: rng(7).integers(0, 1 << 24, 1 << 21).astype(np.int32),
        "all_equal_big": lambda: np.full(1 << 20, -77, dtype=np.int32),
        # K1h: > 65535 equal 16-bit prefixes per workgroup (u16 wrap repairs)
        "all_equal_2p25": lambda: np.full(1 << 25, 1 << 20, dtype=np.int32),
        "h16_wrap_pair": lambda: _h16_wrap_pair(orc),
        "zipf_2p22": lambda: orc.gen(orc.ZIPF, 4, 1 << 22),
        "uniform_2p24": lambda: orc.gen(orc.UNIFORM, 5, 1 << 24),
        "one_hot_bucket": lambda: _one_hot_bucket(orc),
        "negatives_2p21": lambda: rng(7).integers(-2**31, 2**31, 1 << 21,
                                                  dtype=np.int64).astype(np.int32),
        "bucket_edges": lambda: np.repeat(np.arange(-600, 600, dtype=np.int32) * 65536, 8190),
        "full32_2p24": lambda: rng(7).integers(-2**31, 2**31, 1 << 24,
                                               dtype=np.int64).astype(np.int32),
    }


MSD_CASES = list(_msd_cases(None))


@pytest.mark.parametrize("name", MSD_CASES)
def test_radix_one_gpu_bucket_regimes(ctx, orc, name):
    """MSD level structure: single-bucket sorts, all-local first level, oversized buckets down
    to the digit-0 level, one huge bucket among normal ones, exact kLocalMax boundaries."""
    keys = _msd_cases(orc)[name]()
    got, st = sort_on_gpu(ctx, keys)
    assert np.array_equal(got, np.sort(keys)), name


def test_radix_matches_reference_golden_outputs(ctx, orc, ref_cases, ref_outputs):
    """The reference's own sorted dumps (oracle/_ref under mpirun) in the parity domain."""
    n = 0
    for c in ref_cases:
        spec = c["input"]
        if "gen" not in spec or c["P"] == 1 or c["rc"] != 0 or "mod" in spec:
            continue
        keys = case_input(orc, spec)
        for algo in ("radix", "sample"):
            got, _ = sort_on_gpu(ctx, keys, algo)
            assert np.array_equal(got, case_output(c, ref_outputs)), (c["id"], algo)
        n += 1
    assert n >= 15


def test_radix_2p28_properties(ctx, gsort, orc):
    """BASELINE config 2 (2^28 uniform keys, one GPU): sorted + same multiset as the input."""
    n = 1 << 28
    p = ctx.alloc(n * 4)
    try:
        ctx.generate(gsort.UNIFORM, 42, 0, n, p)
        fin = ctx.fingerprint(p, n)
        out, nout, st = ctx.radix(p, n)
        # MSD: the canonical keys use 31 bits: level 3 gives 128 buckets of ~2^21 keys,
        # level 2 buckets of ~8192 keys, all within kLocalMax -> two levels
        assert nout == n and st["passes_run"] == (4 if ctx.algo == "lsd" else 2)
        fout = ctx.fingerprint(out, n)
        assert fout["sorted"] and (fout["sum"], fout["xor"]) == (fin["sum"], fin["xor"])
        # spot-check a window against the oracle's sort of a generated slice bound
        head = ctx.to_host(out, 1 << 16)
        assert head[0] == fout["first"] and np.all(np.diff(head) >= 0)
        # the input is untouched (out-of-place)
        assert ctx.fingerprint(p, n) == fin
    finally:
        ctx.free(p)


def test_fingerprint_matches_oracle(ctx, orc):
    keys = orc.gen(orc.ZIPF, 5, 100003)
    p = dev(ctx, keys)
    f = ctx.fingerprint(p, keys.size)
    ctx.free(p)
    s, x, ok = orc.fingerprint(keys)
    assert (f["sum"], f["xor"], f["sorted"]) == (s, x, ok)


# ---------------------------------------------------------------------------------------
# multi-rank on one GPU (in-process rank group)
# ---------------------------------------------------------------------------------------
def run_group(gsort, blocks, algo, local="msd", balanced=False, setup=None):
    """P ranks as P threads of this process, one context each, on one GPU.  setup(ctx) runs
    on every rank's context before the sort."""
    P = len(blocks)
    grp = gsort.Group(P)
    res, errs = [None] * P, []

    def worker(r):
        try:
            with gsort.Context(rank=r, group=grp) as c:
                c.set_local_algo(gsort.LOCAL_MSD if local == "msd" else gsort.LOCAL_LSD)
                c.set_sample_balanced(balanced)
                if setup is not None:
                    setup(c)
                p = c.alloc(max(blocks[r].size, 1) * 4)
                c.to_device(blocks[r], p)
                fn = c.radix if algo == "radix" else c.sample
                out, n, st = fn(p, blocks[r].size)
                info = c.sample_info() if algo == "sample" else None
                res[r] = (c.to_host(out, n), st, info)
                c.free(p)
        except Exception as e:  # surface in the main thread
            errs.append((r, e))

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    hung = [r for r, t in enumerate(th) if t.is_alive()]
    if hung:
        # a worker may still be inside a group collective: leak the group rather than free
        # the state it is waiting on
        pytest.fail(f"in-process group ranks {hung} did not finish within 600 s")
    grp.close()
    if errs:
        if len(errs) > 1:  # every rank's failure, in the order they happened
            print("\n".join(f"rank {r}: {e}" for r, e in errs))
        raise errs[0][1]
    missing = [r for r in range(P) if res[r] is None]
    assert not missing, f"ranks {missing} returned no result"
    return res


@pytest.mark.parametrize("local", ["msd", "lsd"])
@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_radix_multirank_balanced_blocks(gsort, orc, P, local):
    """msd: exact splitters + one exchange; lsd: one exchange per digit (the reference's pass
    structure).  Both must leave rank q with global positions [qB, (q+1)B)."""
    for dist, n in ((orc.UNIFORM, 200003), (orc.ZIPF, 150000)):
        keys = orc.gen(dist, P, n)
        B = -(-n // P)
        blocks = [keys[r * B:(r + 1) * B] for r in range(P)]
        res = run_group(gsort, blocks, "radix", local)
        ref = np.sort(keys)
        for q in range(P):
            assert np.array_equal(res[q][0], ref[q * B:(q + 1) * B]), (P, dist, q)
        if local == "msd":
            assert all(r[1]["exchanges"] == 1 for r in res)


def test_radix_multirank_many_ranks(gsort, orc):
    """20 ranks (the packed exchange takes up to 64): 20 x 20 pieces, most destination ranges
    a few 16-bit buckets wide, exact at every rank."""
    P = 20
    for dist, n in ((orc.UNIFORM, 200003), (orc.ZIPF, 150001)):
        keys = orc.gen(dist, P, n)
        B = -(-n // P)
        blocks = [keys[r * B:(r + 1) * B] for r in range(P)]
        res = run_group(gsort, blocks, "radix")
        ref = np.sort(keys)
        for q in range(P):
            assert np.array_equal(res[q][0], ref[q * B:(q + 1) * B]), (dist, q)


@pytest.mark.parametrize("P", [1, 2, 4, 8])
def test_radix_multirank_mixed_inputs(gsort, orc, monkeypatch, P):
    """The packed exchange on uniform and Zipf keys, a few distinct values (destination ranges
    of very few buckets) and uneven blocks with empty ones; rank q gets [qB, (q+1)B)."""
    if P == 1:  # a one-rank group still takes the distributed path
        monkeypatch.setenv("GSORT_FORCE_DIST", "1")
    rng = np.random.default_rng(P * 10)
    cases = [orc.gen(orc.UNIFORM, P, 300007), orc.gen(orc.ZIPF, P + 1, 150000),
             rng.integers(-3, 4, 120000).astype(np.int32)]
    for keys in cases:
        B = -(-keys.size // P)
        blocks = [keys[r * B:(r + 1) * B] for r in range(P)]
        res = run_group(gsort, blocks, "radix")
        ref = np.sort(keys)
        for q in range(P):
            assert np.array_equal(res[q][0], ref[q * B:(q + 1) * B]), (P, q)
    if P > 2:
        keys = orc.gen(orc.UNIFORM, 7, 90000)
        blocks = [keys[:0], keys[:50000], keys[50000:50001]] + [keys[50001:]] + \
            [keys[:0]] * (P - 4)
        res = run_group(gsort, blocks, "radix")
        ref = np.sort(keys)
        B = -(-keys.size // P)
        for q in range(P):
            assert np.array_equal(res[q][0], ref[q * B:(q + 1) * B]), (P, q, "uneven")


@pytest.mark.parametrize("local", ["msd", "lsd"])
def test_radix_multirank_uneven_and_empty_inputs(gsort, orc, local):
    keys = orc.gen(orc.UNIFORM, 9, 50000) - (1 << 30)
    blocks = [keys[:0], keys[:31000], keys[31000:31001], keys[31001:]]
    res = run_group(gsort, blocks, "radix", local)
    ref = np.sort(keys)
    B = -(-keys.size // 4)
    for q in range(4):
        assert np.array_equal(res[q][0], ref[q * B:(q + 1) * B])


@pytest.mark.parametrize("case", ["all_equal", "two_values", "boundary_dups", "tiny",
                                  "extremes", "big_uniform", "big_groups", "wide_buckets"])
def test_radix_multirank_splitter_edges(gsort, orc, case):
    """Exact splitters where a boundary key repeats across ranks and blocks (copies split in
    rank order), fewer keys than ranks, INT_MIN/INT_MAX keys, and a 2^22-key sort."""
    rng = np.random.default_rng(sum(map(ord, case)))
    P = 5
    keys = {
        "all_equal": np.full(40003, 7, dtype=np.int32),
        "two_values": rng.choice(np.array([-3, 9], dtype=np.int32), 30011),
        "boundary_dups": np.repeat(np.arange(-4, 5, dtype=np.int32), 7777),
        "tiny": np.array([5, -1, 5], dtype=np.int32),
        "extremes": rng.choice(np.array([-2**31, 2**31 - 1, 0, -1], dtype=np.int32), 12345),
        "big_uniform": orc.gen(orc.UNIFORM, 77, 1 << 22),
        # three 16-bit groups of 60000 keys each: boundary groups larger than kLocalMax on the
        # sender (LSD group sort) and receive buckets larger than kLocalMax (gather + levels)
        "big_groups": (np.repeat(np.array([-5, 0, 7], dtype=np.int64) << 16, 60000) +
                       rng.integers(0, 1 << 16, 180000)).astype(np.int32),
        # 64 received 16-bit buckets of ~13000 keys per rank at P = 5 (the weak-scaling shape
        # of 2^28 keys per GPU at P = 8: receive buckets past kLocalMax, sorted by K18)
        "wide_buckets": rng.integers(0, 1 << 22, 1 << 22).astype(np.int32),
    }[case]
    rng.shuffle(keys)
    cuts = np.sort(rng.integers(0, keys.size + 1, P - 1))
    blocks = np.split(keys, cuts)
    res = run_group(gsort, blocks, "radix")
    ref = np.sort(keys)
    B = -(-keys.size // P)
    for q in range(P):
        assert np.array_equal(res[q][0], ref[q * B:(q + 1) * B]), (case, q)


@pytest.mark.parametrize("form", ["packed", "int32"])
@pytest.mark.parametrize("P", [2, 4, 8])
def test_sample_multirank_matches_reference_semantics(gsort, orc, ref_cases, ref_outputs, P, form,
                                                      monkeypatch):
    """Splitters, the P x P bucket matrix and the output equal the reference's own debug
    output (golden fixtures) and the oracle's restatement -- for the packed sample sort (the
    default: samples and bounds read off the 16-bit grouped block, 2 B/key exchange) and its
    int32 form (local sort first; GSORT_SAMPLE_INT32=1, what the LSD local algorithm and ranks
    past 2^32 keys take)."""
    monkeypatch.setenv("GSORT_SAMPLE_INT32", "1" if form == "int32" else "0")
    checked = 0
    for c in ref_cases:
        if c["prog"] != "sample_sort" or c["P"] != P or c["rc"] != 0:
            continue
        keys = case_input(orc, c["input"])
        B = -(-keys.size // P)
        blocks = [keys[r * B:(r + 1) * B] for r in range(P)]
        res = run_group(gsort, blocks, "sample")
        assert res[0][2][0].tolist() == c["splitters"], c["id"]
        mat = [res[r][2][1].astype(np.int64).tolist() for r in range(P)]
        assert mat == c["bucket_matrix"], c["id"]
        got = np.concatenate([res[r][0] for r in range(P)])
        assert np.array_equal(got, case_output(c, ref_outputs)), c["id"]
        checked += 1
    assert checked >= 2


def test_sample_not_enough_samples(gsort, orc):
    """mpi_sample_sort.c:94-99 aborts with "no enough sample" (Q9, N=9 P=4); every rank of
    the build returns GSORT_ENOSAMPLE instead of hanging."""
    keys = np.arange(9, 0, -1, dtype=np.int32)
    blocks = [keys[0:3], keys[3:6], keys[6:9], keys[9:]]
    with pytest.raises(gsort.GsortError) as ei:
        run_group(gsort, blocks, "sample")
    assert ei.value.status == gsort.ENOSAMPLE


@pytest.mark.parametrize("form", ["packed", "int32"])
def test_sample_multirank_zipf_skew(gsort, orc, form, monkeypatch):
    """Zipf at P=8 overflows the reference's fixed buckets (Q12); the build sizes receive
    buffers from the exchanged counts, so it sorts correctly with one rank holding ~30%.  (The
    packed form's giant 16-bit group takes the host path of the select, counted.)"""
    monkeypatch.setenv("GSORT_SAMPLE_INT32", "1" if form == "int32" else "0")
    P, n = 8, 1 << 18
    keys = orc.gen(orc.ZIPF, 11, n)
    assert orc.ref_sample(keys, P)[0] == orc.E_OVERFLOW
    B = n // P
    res = run_group(gsort, [keys[r * B:(r + 1) * B] for r in range(P)], "sample")
    got = np.concatenate([res[r][0] for r in range(P)])
    assert np.array_equal(got, np.sort(keys))
    assert max(res[r][0].size for r in range(P)) > 0.25 * n


@pytest.mark.parametrize("P", [2, 4, 8])
def test_sample_multirank_zipf_balanced(gsort, orc, P):
    """gsort_set_sample_balanced: the copies of a splitter value are shared out in rank order
    (gsort_plan_split_balanced), so Zipf no longer piles ~30% of the keys on one rank; the
    concatenated output is the same sorted array, and sample_info reports the balanced counts."""
    n = 1 << 18
    keys = orc.gen(orc.ZIPF, 11, n)
    B = n // P
    blocks = [keys[r * B:(r + 1) * B] for r in range(P)]
    res = run_group(gsort, blocks, "sample", balanced=True)
    got = np.concatenate([res[r][0] for r in range(P)])
    assert np.array_equal(got, np.sort(keys))
    assert max(res[r][0].size for r in range(P)) <= 2 * B
    if P == 8:
        assert max(res[r][0].size for r in range(P)) < 0.2 * n
    # uniform keys (distinct almost surely): identical to the reference's bucket rule
    ukeys = orc.gen(orc.UNIFORM, 5, n)
    ub = [ukeys[r * B:(r + 1) * B] for r in range(P)]
    a = run_group(gsort, ub, "sample", balanced=True)
    b = run_group(gsort, ub, "sample")
    for r in range(P):
        assert np.array_equal(a[r][0], b[r][0])


@pytest.mark.parametrize("algo", ["radix", "sample"])
@pytest.mark.parametrize("P,span,n", [(2, 1 << 22, 1 << 22), (4, 1 << 21, (1 << 22) + 3),
                                      (2, 1 << 16, (1 << 22) + 5), (3, 1 << 17, 3 << 20)])
def test_multirank_large_receive_buckets(gsort, P, span, n, algo):
    """Receive-side 16-bit buckets past kLocalMax: K18's counting sort from the pieces
    (<= kHxMax keys) and, for a bucket past kHxMax (span 2^16 at P = 2: one bucket of ~2M keys
    per rank), the gather + MSD levels fallback."""
    rng = np.random.default_rng(P * 1000 + span % 977 + n % 13)
    keys = (rng.integers(0, span, n) - span // 2).astype(np.int32)
    B = -(-n // P)
    blocks = [keys[r * B:(r + 1) * B] for r in range(P)]
    res = run_group(gsort, blocks, algo)
    got = np.concatenate([res[r][0] for r in range(P)])
    assert np.array_equal(got, np.sort(keys))
    if algo == "radix":
        ref = np.sort(keys)
        for q in range(P):
            assert np.array_equal(res[q][0], ref[q * B:(q + 1) * B]), q


def test_radix_multirank_h16_wraps(gsort, orc):
    """The distributed sender groups its block through the two-level plan (K1h 16-bit counts
    -> bucket bounds gb and the packed low-16 send buffer): a key repeated > 65535 times per
    K1h workgroup wraps its u16 counter; the bounds (and so the exchange) must stay exact."""
    P, n = 2, 1 << 26
    rng = np.random.default_rng(21)
    u = rng.random(n)
    keys = np.where(u < 0.7, np.int32(0x12340000),
                    np.where(u < 0.9, np.int32(0x12350005),
                             rng.integers(-2**31, 2**31, n, dtype=np.int64))).astype(np.int32)
    B = n // P
    res = run_group(gsort, [keys[r * B:(r + 1) * B] for r in range(P)], "radix")
    got = np.concatenate([res[r][0] for r in range(P)])
    assert all(res[r][0].size == B for r in range(P))
    assert np.array_equal(got, np.sort(keys))


@pytest.mark.parametrize("n", [0, 1000, 1 << 22, (40 << 20) + 3])
def test_drop_in_staged_round_trip(gsort, n):
    """The drop-in host path: pageable rank-0 array -> GPU (gsort_scatter_from_root, through
    the pinned staging chunks from 16 MiB on: exactly 16 MiB, and 160 MiB + 12 B, which ends
    in a partial chunk) -> gsort_radix -> host (gsort_gather_to_root, staged the same way)."""
    c = gsort.Context()
    try:
        rng = np.random.default_rng(n + 7)
        h = rng.integers(-(1 << 31), (1 << 31) - 1, size=n, dtype=np.int64).astype(np.int32)
        d, m = c.scatter_from_root(h, n)
        assert m == n
        if n:
            np.testing.assert_array_equal(c.to_host(d, n), h)  # the H2D half alone
        out, n_out, _ = c.radix(d, m)
        assert n_out == n
        back = c.gather_to_root(out, n_out, n)
        np.testing.assert_array_equal(back, np.sort(h))
    finally:
        c.close()


def test_ballot_rank_fallback(gsort, orc):
    """K11 / K11g with the 8-ballot stable ranks (wave_rank<false>): the path a context takes
    when its creation-time check of the LDS lane-order property fails, forced here with
    GSORT_BALLOT_RANK=1 (read at context creation)."""
    old = os.environ.get("GSORT_BALLOT_RANK")
    os.environ["GSORT_BALLOT_RANK"] = "1"
    try:
        ctx = gsort.Context()
        blocks = None
        cases = [orc.gen(orc.UNIFORM, 21, n) for n in (1, 777, 16384, 16385, (1 << 22) + 3)]
        cases += [orc.gen(orc.ZIPF, 22, 1 << 21), _h16_wrap_pair(orc)[: 1 << 22]]
        for keys in cases:
            for algo in ("radix", "sample"):
                got, _ = sort_on_gpu(ctx, keys, algo)
                assert np.array_equal(got, np.sort(keys)), (keys.size, algo)
        ctx.close()
        keys = orc.gen(orc.UNIFORM, 23, 300001)
        B = -(-keys.size // 4)
        blocks = [keys[r * B:(r + 1) * B] for r in range(4)]
        res = run_group(gsort, blocks, "radix")  # contexts created with the variable set
        assert np.array_equal(np.concatenate([r[0] for r in res]), np.sort(keys))
    finally:
        if old is None:
            os.environ.pop("GSORT_BALLOT_RANK")
        else:
            os.environ["GSORT_BALLOT_RANK"] = old
