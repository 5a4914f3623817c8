"""GPU parity tests of the sampled plan: levels 3 and 2 sized from a 1/64
sample, K11e into exact positions, and the exact-plan re-sort it falls back to.

Bit-exact against numpy's sort (integer keys).  Every case also states which plan ran
(gsort_last_plan), so a silent fallback cannot pass for the sampled path: uniform and
sorted inputs must stay on the sampled plan; skewed / dense inputs may be ineligible and
must then come back sorted through the exact plan; GSORT_EST_SLACK=0 (no sampling-error
margin) forces region overflows, which must be caught and re-sorted.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SAMPLED, FALLBACK, SHIFTED, GIANT = 1, 2, 3, 4


def _ctx(gsort, **env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return gsort.Context()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def ctx(gsort):
    c = _ctx(gsort, GSORT_EST=1, GSORT_EST_SLACK=1)
    yield c
    c.close()


def _sort(ctx, keys, algo="radix"):
    p = ctx.alloc(max(keys.size, 1) * 4)
    try:
        ctx.to_device(keys, p)
        out, n, st = (ctx.radix if algo == "radix" else ctx.sample)(p, keys.size)
        assert n == keys.size
        return ctx.to_host(out, n), st
    finally:
        ctx.free(p)


# the sampled plan starts at 2^22 keys (kEstMinKeys); odd sizes leave a partial last tile,
# sample block and segment
SIZES = [1 << 22, (1 << 22) + 12345, (1 << 23) + 8191, (1 << 24) + 1, 3 << 23]


@pytest.mark.parametrize("n", SIZES)
def test_sampled_plan_uniform(ctx, orc, n):
    keys = orc.gen(orc.UNIFORM, n % 1000 + 5, n)
    got, st = _sort(ctx, keys)
    assert ctx.last_plan() == SAMPLED
    assert np.array_equal(got, np.sort(keys))
    assert st["passes_run"] == 2


def test_sampled_plan_full_range_and_sample_sort(ctx):
    """Negative and positive keys over the whole int32 range (256 level-3 buckets); the one-rank
    sample sort takes the same plan."""
    rng = np.random.default_rng(11)
    keys = rng.integers(-2**31, 2**31, 1 << 23, dtype=np.int64).astype(np.int32)
    for algo in ("radix", "sample"):
        got, _ = _sort(ctx, keys, algo)
        assert ctx.last_plan() == SAMPLED, algo
        assert np.array_equal(got, np.sort(keys)), algo


def test_sampled_plan_below_threshold_is_exact(ctx, orc):
    keys = orc.gen(orc.UNIFORM, 3, (1 << 22) - 1)
    got, _ = _sort(ctx, keys)
    assert ctx.last_plan() == 0
    assert np.array_equal(got, np.sort(keys))


def _inputs(orc, n):
    rng = np.random.default_rng(5)
    u = orc.gen(orc.UNIFORM, 21, n)
    runs = np.sort(u)
    return {
        "sorted": runs,
        "reversed": runs[::-1].copy(),
        "sorted_blocks": np.concatenate([np.sort(b) for b in np.array_split(u, 64)]),
        "zipf": orc.gen(orc.ZIPF, 4, n),
        "all_equal": np.full(n, -77, dtype=np.int32),
        "bits16": (u & 0xFFFF).astype(np.int32),
        "bits24": (u & 0xFFFFFF).astype(np.int32),
        "bits28": (u & 0xFFFFFFF).astype(np.int32),
        "half_one_value": np.where(rng.random(n) < 0.5, np.int32(1 << 20), u).astype(np.int32),
        "two_clusters": np.where(rng.random(n) < 0.5, u >> 12, -(u >> 12)).astype(np.int32),
    }


@pytest.mark.parametrize("name", ["sorted", "reversed", "sorted_blocks", "zipf", "all_equal",
                                  "bits16", "bits24", "bits28", "half_one_value",
                                  "two_clusters"])
def test_sampled_plan_distributions(ctx, orc, name):
    n = 1 << 23
    keys = _inputs(orc, n)[name]
    got, _ = _sort(ctx, keys)
    plan = ctx.last_plan()
    assert plan in (SAMPLED, FALLBACK, SHIFTED, GIANT), plan
    if name in ("sorted", "reversed", "sorted_blocks"):  # uniform keys, position-correlated
        assert plan == SAMPLED, name
    if name in ("zipf", "bits16"):  # one 16-bit child holds (nearly) every key:
        assert plan == GIANT, name  # counted, not partitioned
    if name == "all_equal":  # every sample one value, min == max: the block is copied
        assert plan == SHIFTED, name
    if name == "half_one_value":  # the child holds about half: either way is right
        assert plan in (FALLBACK, GIANT), name
    if name == "bits24":  # a narrow key range: 256 children of ~32K keys, taken as they are
        assert plan in (SAMPLED, SHIFTED), name  # (K11e / K18c) or below the shared bits
    assert np.array_equal(got, np.sort(keys)), name


def test_sampled_plan_overflow_falls_back(gsort, orc):
    """No sampling margin: about half the regions overflow; every overflowed run went to the
    scratch tile, the runtime sees ovf and the exact plan sorts the block again."""
    c = _ctx(gsort, GSORT_EST=1, GSORT_EST_SLACK=0)
    try:
        for n in ((1 << 22) + 3, 1 << 24):
            keys = orc.gen(orc.UNIFORM, 99, n)
            got, _ = _sort(c, keys)
            assert c.last_plan() == FALLBACK
            assert np.array_equal(got, np.sort(keys))
    finally:
        c.close()


def test_sampled_plan_off(gsort, orc):
    c = _ctx(gsort, GSORT_EST=0)
    try:
        keys = orc.gen(orc.UNIFORM, 8, 1 << 23)
        got, _ = _sort(c, keys)
        assert c.last_plan() == 0
        assert np.array_equal(got, np.sort(keys))
    finally:
        c.close()


def test_sampled_plan_repeated_sorts_reuse_scratch(ctx, orc):
    """Back-to-back sorts of different sizes on one context (scratch reused, K1e re-zeroes the
    status words, the class counters are cleared by the front)."""
    for i, n in enumerate([1 << 24, (1 << 22) + 1, 1 << 24, 5 << 22]):
        keys = orc.gen(orc.UNIFORM, 100 + i, n)
        got, _ = _sort(ctx, keys)
        assert ctx.last_plan() == SAMPLED
        assert np.array_equal(got, np.sort(keys)), n


@pytest.mark.parametrize("bits,plan", [(27, SAMPLED), (26, SAMPLED), (25, SAMPLED)])
def test_sampled_plan_child_classes(ctx, bits, plan):
    """2^24 keys below 2^bits: 16-bit children of 2^(bits-8) keys -- K11e classes 2 and 3
    (8 192 / 16 384 keys) on the sampled plan; 32 768-key children (bits = 25) are past class
    3, so K12g lists them (and those past kLocalMax) for K18c's counting sort from Y (round 4;
    before it the block was retried with its digits below the 7 leading bits every key
    shares)."""
    rng = np.random.default_rng(bits)
    keys = rng.integers(0, 1 << bits, 1 << 24, dtype=np.int64).astype(np.int32)
    got, _ = _sort(ctx, keys)
    assert ctx.last_plan() == plan
    assert np.array_equal(got, np.sort(keys))


def test_sampled_plan_without_room_falls_back():
    """GSORT_ALLOC_LIMIT below the region buffers' size (but above the block's): the sampled
    plan cannot allocate Y, hands its memory back, and the exact plan sorts (one child
    process: the limit is read once per process)."""
    n = 1 << 23
    code = f"""
import sys, numpy as np
sys.path[:0] = {[os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                 os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                              "mpi-test_amd")]!r}
import torch, gsort
keys = np.random.default_rng(3).integers(-2**31, 2**31, {n}, dtype=np.int64).astype(np.int32)
with gsort.Context() as c:
    p = c.alloc(keys.size * 4); c.to_device(keys, p)
    out, m, _ = c.radix(p, keys.size)
    assert c.last_plan() == 2, c.last_plan()
    assert np.array_equal(c.to_host(out, m), np.sort(keys))
print("ok")
"""
    env = dict(os.environ, GSORT_EST="1", GSORT_ALLOC_LIMIT=str(n * 4 * 3 // 2))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("case", ["prefix_broken_late", "prefix_broken_first", "negative_16bit"])
def test_sampled_plan_shifted_prefix_check(ctx, case):
    """The shifted retry trusts the samples' common prefix only after K3r has checked it on every
    key: a block of 16-bit keys with a few keys outside the prefix (at unsampled positions or at
    position 0, the reference key) must still come back sorted (exact plan), and negative 16-bit
    keys (prefix 0x7fff after the sign flip) take the shifted plan."""
    rng = np.random.default_rng(17)
    n = 1 << 23
    keys = rng.integers(0, 1 << 16, n, dtype=np.int64).astype(np.int32)
    if case == "prefix_broken_late":
        keys[[n - 1, n // 2 + 3, 12345]] = [1 << 30, -5, 70000]
    elif case == "prefix_broken_first":
        keys[0] = 1 << 20
    else:
        keys = (keys - (1 << 16)).astype(np.int32)
    got, _ = _sort(ctx, keys)
    plan = ctx.last_plan()
    if case == "negative_16bit":  # every key in child 0x7fff: counted
        assert plan == GIANT
    else:  # one child holds all but a few keys: counted, the outliers sorted as cold keys
        assert plan == GIANT, plan
    assert np.array_equal(got, np.sort(keys)), case


@pytest.mark.parametrize("lo,hi,n,plans", [
    (0, 1 << 20, 1 << 23, (SAMPLED, SHIFTED)), (-(1 << 27), 0, 1 << 26, (SAMPLED, SHIFTED)),
    (5 << 24, (5 << 24) + (1 << 26), 1 << 26, (SAMPLED, SHIFTED)),
    (1 << 28, 3 << 27, 1 << 26, (SAMPLED, SHIFTED)),
    (0, 1 << 19, 1 << 24, (SHIFTED,)), (5 << 24, (5 << 24) + (1 << 20), 1 << 24, (SHIFTED,)),
    (-(1 << 14), 1 << 14, 1 << 23, (SHIFTED, GIANT))])
def test_sampled_plan_shifted_ranges(ctx, lo, hi, n, plans):
    """Key ranges narrower than int32 at any bit offset (20-, 27-, 26-, 27-, 19-bit spans, and
    one across zero: its ordered keys share no leading bit).  Children of up to kHxMax keys are
    taken by the first attempt (those past kLocalMax by K18c, round 4); past kHxMax (the 19- and
    20-bit spans at 2^24 keys: 8 / 16 children of ~1-2M keys) the retry shifts every digit by
    the samples' shared leading bits (not only whole bytes)."""
    rng = np.random.default_rng(hi & 0xffff)
    keys = rng.integers(lo, hi, n, dtype=np.int64).astype(np.int32)
    got, _ = _sort(ctx, keys)
    assert np.array_equal(got, np.sort(keys)), (lo, hi)
    # across zero the shared bits are the keys' minus the exact minimum: that read pass is spent
    # when the first sample's child counts are known, or -- as here, two children wrapped them
    # -- when the samples span at most 24 bits (a peaked block, round 4; before it this case
    # took the one-child count or the exact plan).  Its two children hold ~half of the keys
    # each, so the one-child count may take the larger one (>= n / 2 by the exact count).
    assert ctx.last_plan() in plans, (lo, hi, ctx.last_plan())


@pytest.mark.parametrize("case", ["gauss", "gauss_outliers", "two_values_across_zero"])
def test_sampled_plan_offset_retry(ctx, case):
    """Clustered keys around zero (no shared prefix) go through the offset retry: the exact
    min / max, every key taken minus the minimum.  Outliers the samples miss only widen that
    range (the plan still has to be right); two values across zero make many one-value
    children."""
    rng = np.random.default_rng(23)
    n = 1 << 24
    if case == "two_values_across_zero":
        keys = rng.choice(np.array([-3, 4], dtype=np.int32), n)
    else:
        keys = np.clip(rng.normal(0, 3e5, n), -2**31, 2**31 - 1).astype(np.int32)
        if case == "gauss_outliers":
            keys[[7, n // 3, n - 2]] = [-2**31, 2**31 - 1, 123456789]
    got, _ = _sort(ctx, keys)
    assert np.array_equal(got, np.sort(keys)), case
    assert ctx.last_plan() in (SAMPLED, FALLBACK, SHIFTED, GIANT), ctx.last_plan()
    if case == "gauss":  # ~55 children of ~300K keys: taken at once (K18c), or after the offset
        assert ctx.last_plan() in (SAMPLED, SHIFTED)


@pytest.mark.parametrize("case", ["arange", "arange_reversed", "full_span_reversed", "gauss_1e6"])
def test_dense_and_peaked_2p24(ctx, case):
    """tools/dist_probe.py's sorted / reverse / gauss shapes at 2^24:
    dense keys (every value of a range once, ascending or descending; or one key per 256
    values over the whole int32 range, descending) put a digit's run a fixed stride after the
    previous one in K11e's key array -- the padded layout -- and a Gaussian block goes through
    the offset retry guessed from its samples' range.  np.sort parity for both algorithms."""
    n = 1 << 24
    if case == "arange":
        keys = np.arange(n, dtype=np.int32)
    elif case == "arange_reversed":
        keys = np.arange(n, 0, -1, dtype=np.int32)
    elif case == "full_span_reversed":
        keys = (np.arange(n - 1, -1, -1, dtype=np.int64) * 256 - 2**31).astype(np.int32)
    else:
        keys = np.clip(np.random.default_rng(41).normal(0, 1e6, n), -2**31, 2**31 - 1).astype(np.int32)
    want = np.sort(keys)
    for algo in ("radix", "sample"):
        got, _ = _sort(ctx, keys, algo)
        assert np.array_equal(got, want), (case, algo)
        assert ctx.last_plan() in (SAMPLED, SHIFTED), (case, algo, ctx.last_plan())


@pytest.mark.parametrize("n", [(1 << 24) + 3, 1 << 25])
def test_sampled_plan_oversized_children(ctx, n):
    """A peak on a wide span (round 4): 60 % of the keys within +-5 120 of zero, the rest
    uniform over +-2^23.  The first sample wraps its counters on the peak; the offset retry
    (samples spanning <= 24 bits) shifts the digits 8 bits down, where the peak's ~40
    children hold ~250 K keys each -- past kLocalMax, so K12g lists them for K18c's counting
    sort from Y (list 0) instead of refusing the block."""
    rng = np.random.default_rng(n & 0xff)
    keys = np.where(rng.random(n) < 0.6, rng.integers(-5120, 5120, n),
                    rng.integers(-(1 << 23), 1 << 23, n)).astype(np.int32)
    keys[[0, n - 1]] = [-(1 << 23), (1 << 23) - 1]  # the span's ends
    got, st = _sort(ctx, keys)
    assert np.array_equal(got, np.sort(keys))
    assert ctx.last_plan() == SHIFTED, ctx.last_plan()


# ---- one dominant 16-bit child ("giant child") -------------------------------
def _giant_inputs(orc, n):
    rng = np.random.default_rng(31)
    u = orc.gen(orc.UNIFORM, 32, n)
    r = rng.random(n)
    return {
        # Zipf s = 1.5 (configs[4]'s distribution): ~99.6 % below 2^16, the rest cold
        "zipf": orc.gen(orc.ZIPF, 33, n),
        "bits8": (u & 0xFF).astype(np.int32),
        "bits16_negative": ((u & 0xFFFF) - (1 << 16)).astype(np.int32),
        # 60 % in one child, 20 % below it (negative keys) and 20 % above: the cold keys below
        # the child move to the front, those above go after it
        "child_in_middle": np.where(r < 0.6, (u & 0xFFFF) + (7 << 16),
                                    np.where(r < 0.8, -(u >> 8) - 1, u | (1 << 30))).astype(np.int32),
        "one_hot_value": np.where(r < 0.7, np.int32(-123456), u).astype(np.int32),
        "all_equal_min": np.full(n, -2**31, dtype=np.int32),
    }


@pytest.mark.parametrize("name", ["zipf", "bits8", "bits16_negative", "child_in_middle",
                                  "one_hot_value"])
@pytest.mark.parametrize("n", [1 << 22, (1 << 24) + 777])
def test_giant_child_counted(ctx, orc, name, n):
    keys = _giant_inputs(orc, n)[name]
    for algo in ("radix", "sample"):
        got, st = _sort(ctx, keys, algo)
        assert ctx.last_plan() == GIANT, (name, algo, ctx.last_plan())
        assert np.array_equal(got, np.sort(keys)), (name, algo)
        assert st["passes_run"] == 1 and st["buckets_local"] >= 1


@pytest.mark.parametrize("value", [-2**31, -77, 0, 2**31 - 1])
def test_one_value_block_copied(ctx, value):
    """All samples one value and min == max (checked by K20 before any counted child): the
    sorted block is the block, copied; the stats say one bucket and no partition level
    (the shortcut's stats)."""
    n = (1 << 22) + 9
    keys = np.full(n, value, dtype=np.int32)
    for algo in ("radix", "sample"):
        got, st = _sort(ctx, keys, algo)
        assert ctx.last_plan() == SHIFTED, (value, algo, ctx.last_plan())
        assert np.array_equal(got, keys)
        if algo == "radix":
            assert st["passes_run"] == 0 and st["buckets_local"] == 1
            assert st["keys_bucket_sort"] == n


def _k1m_positions(n):
    """K1m's 16 384 sample positions for n >= 16 384: 1024 groups of 16 consecutive keys, group
    g at g * floor(n / 1024) (gsort_kernels.hip, k_est_mode)."""
    i = np.arange(16384)
    return (i >> 4) * (n // 1024) + (i & 15)


def test_giant_child_sample_misjudged(ctx):
    """Every K1m sample lands on one value but only 1/256 of the keys hold it: the exact
    count after K1g sees the child is not dominant, writes nothing, and the block is sorted on
    another plan."""
    n = 1 << 22
    keys = np.random.default_rng(41).integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
    keys[_k1m_positions(n)] = 5  # exactly the K1m sample positions
    got, _ = _sort(ctx, keys)
    assert ctx.last_plan() in (SAMPLED, FALLBACK), ctx.last_plan()
    assert np.array_equal(got, np.sort(keys))


@pytest.mark.parametrize("extra", [0, 1], ids=["child_(n-1)/2", "child_(n+1)/2"])
def test_giant_child_half_of_odd_n(ctx, orc, extra):
    """odd n and a child of exactly (n - 1) / 2 keys would leave n_cold = n_child + 1
    cold keys, overlapping the cold-key sort's source and destination.  That child is not
    dominant (the block goes to another plan); one key more and it is (n_cold = n_child - 1)."""
    n = (1 << 22) + 1
    n_child = (n - 1) // 2 + extra
    rng = np.random.default_rng(43)
    u = orc.gen(orc.UNIFORM, 44, n)
    keys = (u | (1 << 30)).astype(np.int32)  # cold keys: top bits far from the child's
    pos = np.zeros(n, dtype=bool)
    pos[_k1m_positions(n)] = True  # every K1m sample position in the child
    rest = np.flatnonzero(~pos)
    pos[rng.choice(rest, n_child - int(pos.sum()), replace=False)] = True
    keys[pos] = ((u[pos] & 0xFFFF) + (7 << 16)).astype(np.int32)
    got, _ = _sort(ctx, keys)
    assert np.array_equal(got, np.sort(keys))
    assert (ctx.last_plan() == GIANT) == bool(extra), ctx.last_plan()


def test_giant_child_off(gsort, orc):
    c = _ctx(gsort, GSORT_GIANT=0)
    try:
        keys = orc.gen(orc.ZIPF, 34, 1 << 22)
        got, _ = _sort(c, keys)
        assert c.last_plan() == FALLBACK
        assert np.array_equal(got, np.sort(keys))
    finally:
        c.close()


def test_giant_then_sampled_reuses_scratch(ctx, orc):
    """Giant, uniform, giant on one context: K12m leaves K1h's wrap repairs zeroed, the region
    buffers and S_TMP are shared."""
    for i, (dist, n) in enumerate([(orc.ZIPF, 1 << 24), (orc.UNIFORM, 1 << 23),
                                   (orc.ZIPF, (1 << 22) + 5)]):
        keys = orc.gen(dist, 60 + i, n)
        got, _ = _sort(ctx, keys)
        assert ctx.last_plan() == (GIANT if dist == orc.ZIPF else SAMPLED)
        assert np.array_equal(got, np.sort(keys))


def test_region_buffers_reclaimed_for_a_later_call():
    """the sampled plan's region buffers outlive its call.  At 2^23 keys they take
    ~534 MB (X 64 MB + Y 470 MB: every one of the 65 536 child regions carries >= 2 sample
    blocks of slack, est_region_keys); with the block, the plan arrays and the lists a sampled
    sort fits under GSORT_ALLOC_TOTAL = 640 MB.  A following LSD sort of 2^24 keys needs a
    64 MB S_OUT and a 64 MB S_TMP on top: it fits only with the regions dropped on demand
    (reclaim_regions).  The third call (2^23 again) finds S_TMP held, so its regions may no
    longer fit and the exact plan may sort: either way the result must be exact."""
    code = f"""
import sys, numpy as np
sys.path[:0] = {[os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                 os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                              "mpi-test_amd")]!r}
import torch, gsort
rng = np.random.default_rng(4)
with gsort.Context() as c:
    # the third call finds S_TMP grown: its regions no longer fit, so it sorts on the exact plan
    for i, (n, algo) in enumerate(((1 << 23, gsort.LOCAL_MSD), (1 << 24, gsort.LOCAL_LSD),
                                   (1 << 23, gsort.LOCAL_MSD))):
        keys = rng.integers(-2**31, 2**31, n, dtype=np.int64).astype(np.int32)
        c.set_local_algo(algo)
        p = c.alloc(n * 4); c.to_device(keys, p)
        out, m, _ = c.radix(p, n)
        assert np.array_equal(c.to_host(out, m), np.sort(keys)), n
        if i == 0:
            assert c.last_plan() == 1, c.last_plan()
        c.free(p)
print("ok")
"""
    env = dict(os.environ, GSORT_EST="1", GSORT_ALLOC_TOTAL=str(640 << 20))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "ok" in r.stdout, r.stdout + r.stderr
