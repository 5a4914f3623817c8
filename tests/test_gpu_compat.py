"""GPU tests of the reference-compat radix order (gsort_set_ref_compat): outside
the parity domain the reference's radix sort is a stable sort of the values by the base-P digits
of |v| it extracts (mpi_radix_sort.c:48-58, :133-195).  The HIP path (K20 min/max, K19 key map,
stable key-value LSD passes; for P > 1 ranks through the distributed key-value exchange) is
checked bit-exactly against the reference's own outputs (tests/golden: negative keys at
P = 2, 4, 8, P = 3's digit under-count, P = 1's zero passes, the reader's phantom element) and
against the oracle's simulated reference run (orc.ref_radix) on larger negative-heavy inputs.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, case_input, case_output
from test_gpu_sort import run_group

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(gsort):
    c = gsort.Context()
    yield c
    c.close()


def compat_on_gpu(ctx, keys, P):
    ctx.set_ref_compat(P)
    p = ctx.alloc(max(keys.size, 1) * 4)
    try:
        ctx.to_device(keys, p)
        out, n, st = ctx.radix(p, keys.size)
        assert n == keys.size
        return ctx.to_host(out, n), st
    finally:
        ctx.free(p)
        ctx.set_ref_compat(0)


def test_compat_one_rank_matches_reference_golden(ctx, orc, ref_cases, ref_outputs):
    n = 0
    for c in ref_cases:
        if c["prog"] != "radix_sort" or c["rc"] != 0:
            continue
        keys = case_input(orc, c["input"])
        if keys is None:
            continue
        got, _ = compat_on_gpu(ctx, keys, c["P"])
        assert np.array_equal(got, case_output(c, ref_outputs)), c["id"]
        n += 1
    assert n >= 15


def test_compat_q2_literal(ctx):
    keys = np.array([5, -7, 3, -2, 0, 7, -3, 2], dtype=np.int32)
    for P in (2, 4, 8):
        got, _ = compat_on_gpu(ctx, keys, P)
        assert got.tolist() == [0, -2, 2, 3, -3, 5, -7, 7], P


@pytest.mark.parametrize("P", [2, 3, 4, 5, 8])
def test_compat_one_rank_matches_oracle(ctx, orc, P):
    rng = np.random.default_rng(P)
    for n, lo, hi in ((1 << 20, -2**31 + 1, 2**31), (300007, -70000, 70000),
                      ((1 << 16) + 3, -5, 6), (8193, 0, 1 << 20)):
        keys = rng.integers(lo, hi, n, dtype=np.int64).astype(np.int32)
        rc, ref, _ = orc.ref_radix(keys, P)
        assert rc == 0
        got, _ = compat_on_gpu(ctx, keys, P)
        assert np.array_equal(got, ref), (P, n, lo)


def test_compat_zero_pass_and_inside_domain(ctx, orc):
    keys = orc.gen(orc.UNIFORM, 42, 100000)
    got, _ = compat_on_gpu(ctx, keys, 1)            # Q1: input order
    assert np.array_equal(got, keys)
    got, _ = compat_on_gpu(ctx, keys, 8)            # inside the domain: the numeric sort
    assert np.array_equal(got, np.sort(keys))
    got, _ = compat_on_gpu(ctx, np.zeros(0, dtype=np.int32), 4)
    assert got.size == 0


def test_compat_rejects_undefined_reference_behaviour(ctx, gsort):
    with pytest.raises(gsort.GsortError) as e:      # Q5: abs(INT_MIN) indexes bucket -k
        compat_on_gpu(ctx, np.array([3, -2**31, 1, 2], dtype=np.int32), 2)
    assert e.value.status == gsort.EINVAL
    with pytest.raises(gsort.GsortError):            # Q8: N=5, P=4 -> empty last block
        compat_on_gpu(ctx, np.arange(5, dtype=np.int32), 4)
    got, _ = compat_on_gpu(ctx, np.arange(8, dtype=np.int32)[::-1].copy(), 4)
    assert got.tolist() == list(range(8))           # the context still works


@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_compat_multirank_matches_oracle(gsort, orc, ref_cases, ref_outputs, P):
    """P ranks (in-process group): the key-value passes through the distributed exchange; rank q
    ends with positions [qB, (q+1)B) of the reference's order."""
    rng = np.random.default_rng(10 + P)
    inputs = [rng.integers(-2**31 + 1, 2**31, 200003, dtype=np.int64).astype(np.int32),
              rng.integers(-3000, 3000, 150001, dtype=np.int64).astype(np.int32)]
    for c in ref_cases:
        if c["prog"] == "radix_sort" and c["P"] == P and c["rc"] == 0:
            k = case_input(orc, c["input"])
            if k is not None and k.size >= P:
                inputs.append(k)
    for keys in inputs:
        rc, ref, _ = orc.ref_radix(keys, P)
        assert rc == 0
        n = keys.size
        B = -(-n // P)
        blocks = [keys[r * B:(r + 1) * B] for r in range(P)]
        res = run_group(gsort, blocks, "radix", local="lsd",
                        setup=lambda c: c.set_ref_compat(-1))
        for q in range(P):
            assert np.array_equal(res[q][0], ref[q * B:(q + 1) * B]), (P, n, q)


def test_compat_cli_phantom_and_negatives(tmp_path):
    """GSORT_REF_COMPAT=1 radix_sort: the reference's reader phantom after a trailing newline
    (Q6) and its order of negative keys (Q2) -- here at one rank, the reference's P = 1 runs no
    pass (Q1), so the dump is the input order plus the phantom."""
    p = tmp_path / "q6.txt"
    p.write_text("5\n3\n9\n1\n")
    env = dict(os.environ, GSORT_REF_COMPAT="1")
    r = subprocess.run([os.path.join(ROOT, "mpi-test_amd", "bin", "radix_sort"), str(p), "3"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    dump = [ln for ln in r.stdout.splitlines() if "|" in ln and ln.split("|")[0].isdigit()]
    assert dump == ["0|5", "1|3", "2|9", "3|1", "4|1"]
    assert "The n/2-th sorted element: 3" in r.stdout
