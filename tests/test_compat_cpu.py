"""Reference-compat radix order on the CPU: the host digit planner
(gsort_plan_ref_digits, product code) against the oracle's restatement of the reference's
number_digits / number_digit_at (oracle.c, mpi_radix_sort.c:48-58), and a numpy model of the
compat sort -- composite key from the planner's (mod, scale) exactly as K19 computes it, then a
stable sort -- against the reference's own outputs (tests/golden) and the oracle's simulated
reference run.  The GPU path is tests/test_gpu_compat.py.
"""
import numpy as np
import pytest

from conftest import case_input, case_output


@pytest.fixture(scope="module")
def gs():
    import gsort
    gsort.lib()
    return gsort


def x86_dtoi(x):
    x = np.asarray(x, dtype=np.float64)
    ok = (x > -2147483649.0) & (x < 2147483648.0)
    return np.where(ok, np.trunc(np.where(ok, x, 0)), -2**31).astype(np.int64)


def compat_keys(keys, P, gs):
    """The K19 key map in numpy (int64 arithmetic, C remainder semantics); None where the
    reference would index outside its buckets."""
    keys = np.asarray(keys, dtype=np.int64)
    vmax = max(-1, int(keys.max())) if keys.size else -1
    loop, mod, scale = gs.plan_ref_digits(P, vmax)
    mag = np.abs(keys)
    comp = np.zeros(keys.size, dtype=np.int64)
    w = 1
    for d in range(max(loop, 0)):
        m = int(mod[d])
        if m in (0, -1):
            rem = np.zeros_like(mag)
        else:
            rem = np.fmod(mag, m)  # C %: sign of the dividend
        dig = x86_dtoi(rem / scale[d])
        if np.any(dig < 0) or np.any(dig >= P):
            return None
        comp += dig * w
        w = min(w * P, 1 << 40)
    return comp


def compat_sort(keys, P, gs):
    k = compat_keys(keys, P, gs)
    if k is None:
        return None
    return np.asarray(keys)[np.argsort(k, kind="stable")]


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 7, 8, 16])
def test_plan_ref_digits_matches_oracle(gs, orc, P):
    L = orc.lib()
    rng = np.random.default_rng(P)
    maxes = [-1, 0, 1, 2, 3, 242, 243, 244, 255, 256, 1000, 65535, 65536, 2**31 - 1,
             *rng.integers(0, 2**31, 40).tolist()]
    for mx in maxes:
        loop, mod, scale = gs.plan_ref_digits(P, int(mx))
        assert loop == L.orc_ref_number_digits(int(mx), P), (P, mx)
        for v in rng.integers(0, 2**31, 64).tolist() + [0, 1, int(max(mx, 0))]:
            for d in range(max(loop, 0)):
                m = int(mod[d])
                rem = 0 if m in (0, -1) else int(np.fmod(v, m))
                dig = int(x86_dtoi(rem / scale[d]))
                assert dig == L.orc_ref_digit_at(int(v), P, d + 1), (P, mx, v, d)


def test_plan_ref_digits_quirks(gs):
    assert gs.plan_ref_digits(1, 1000)[0] < 1     # Q1: P = 1 runs no pass
    assert gs.plan_ref_digits(1, 0)[0] < 1
    assert gs.plan_ref_digits(3, 243)[0] == 5     # Q3: log(243)/log(3) rounds below 5
    assert gs.plan_ref_digits(2, -1)[0] == 1      # max_element starts at -1: one pass
    assert gs.plan_ref_digits(2, 2**31 - 1)[0] == 31
    with pytest.raises(gs.GsortError):
        gs.plan_ref_digits(2, 1000, cap=4)        # 10 digits do not fit 4 entries


def test_compat_model_matches_reference_golden(gs, orc, ref_cases, ref_outputs):
    """Every radix golden case the reference ran (uniform / Zipf at P = 2, 4, 8; P = 3 with
    the digit under-count; P = 1; negative keys; the reader's phantom element)."""
    n = 0
    for c in ref_cases:
        if c["prog"] != "radix_sort" or c["rc"] != 0:
            continue
        keys = case_input(orc, c["input"])
        if keys is None:  # text inputs: the reader quirks (q6 phantom, q7 wrap) are below
            continue
        got = compat_sort(keys, c["P"], gs)
        assert got is not None and np.array_equal(got, case_output(c, ref_outputs)), c["id"]
        n += 1
    assert n >= 15


def test_compat_model_matches_oracle_reference_run(gs, orc):
    """Negative-heavy random inputs at every P the reference supports, N % P != 0 included,
    against the oracle's simulated reference run (per-pass scatter / bucket / gather)."""
    rng = np.random.default_rng(3)
    for P in (2, 3, 4, 5, 8):
        for n, lo, hi in ((5000, -10**6, 10**6), (4099, -2**31 + 1, 2**31), (3001, -50, 50)):
            keys = rng.integers(lo, hi, n, dtype=np.int64).astype(np.int32)
            rc, ref, passes = orc.ref_radix(keys, P)
            assert rc == 0
            assert np.array_equal(compat_sort(keys, P, gs), ref), (P, n, lo)
