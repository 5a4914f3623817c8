"""The benchmarked path pinned to the reference's own output at the sizes it runs at (VERDICT
r2): tests/golden/ref_large.json holds, for 2^22 / 2^24-key uniform and Zipf streams, the
sha256 of the reference's full sorted dump, its median / "Each bucket" lines, splitters, bucket
matrices and per-rank stdout contract digests (tests/golden/make_golden.py --large, from
`mpirun -np P` runs of the reference binaries).  One rank: the default local plan (the sampled
plan, gsort_last_plan() == 1 on uniform keys) on device-generated keys; P ranks: the whole
drop-in path (scatter, distributed sort, gather, report) in an in-process group."""
import hashlib

import numpy as np
import pytest

from conftest import GOLDEN_DEBUG
from test_gpu_dropin import check_contract, run_dropin

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<i4").tobytes()).hexdigest()


def streams(ref_large):
    seen = {}
    for c in ref_large:
        s = c["input"]
        seen[(s["gen"], s["n"], s["seed"])] = c
    return sorted(seen)


def reference_digest(ref_large, key):
    """sha256 of the reference's sorted output of a stream (any run that produced it)."""
    for c in ref_large:
        s = c["input"]
        if (s["gen"], s["n"], s["seed"]) == key and c.get("output_is_sorted_input"):
            return c["output_sha256"], c["median_line"]
    return None, None


def test_large_fixtures_cover_the_default_plan(ref_large):
    ns = {c["input"]["n"] for c in ref_large}
    assert min(ns) >= 1 << 22 and (1 << 24) in ns
    assert any(c["input"]["gen"] == "zipf" for c in ref_large)


@pytest.mark.parametrize("algo", ["radix", "sample"])
def test_one_rank_default_plan_equals_reference(gsort, ref_large, algo):
    for gen, n, seed in streams(ref_large):
        want, med = reference_digest(ref_large, (gen, n, seed))
        assert want, (gen, n, seed)
        with gsort.Context(device=0) as c:
            d = c.alloc(n * 4)
            c.generate(gsort.UNIFORM if gen == "uniform" else gsort.ZIPF, seed, 0, n, d)
            out, m, _ = (c.radix if algo == "radix" else c.sample)(d, n)
            plan = c.last_plan()
            h = c.to_host(out, m)
            c.free(d)
        if gen == "uniform":
            assert plan == c.PLAN_SAMPLED, (gen, n, plan)
        assert sha(h) == want, (gen, n, seed, algo, plan)
        assert f"The n/2-th sorted element: {h[n // 2 - 1]}" == med


def test_group_dropin_equals_reference_stdout(gsort, orc, ref_large):
    """Each reference run: the same P, the same stream, the whole drop-in path; every rank's
    stdout contract (for the sample sort: the reference's own splitters and bucket matrix) is
    compared byte for byte.  A run whose reference output is corrupt (the sample sort's fixed
    receive buffers overflow on Zipf) is compared on its splitter and bucket
    lines only."""
    done = 0
    for c in ref_large:
        if c["rc"] != 0:
            continue
        s = c["input"]
        keys = orc.gen(orc.UNIFORM if s["gen"] == "uniform" else orc.ZIPF, s["seed"], s["n"])
        algo = "radix" if c["prog"] == "radix_sort" else "sample"
        outs, g, infos = run_dropin(gsort, keys, c["P"], algo, GOLDEN_DEBUG[c["prog"]])
        assert np.array_equal(g, np.sort(keys)), c["id"]
        if c["output_is_sorted_input"]:
            check_contract(outs, c)
        else:
            for r, o in enumerate(outs):
                lines = o.decode().splitlines()
                assert [ln for ln in lines if "|" not in ln and "n/2-th" not in ln] == \
                    c["contract"][r]["head"], (c["id"], r)
        if algo == "sample":
            assert [list(map(int, i[1])) for i in infos] == c["bucket_matrix"], c["id"]
            assert list(map(int, infos[0][0])) == c["splitters"], c["id"]
        done += 1
    assert done >= 12
