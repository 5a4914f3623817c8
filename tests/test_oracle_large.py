"""The oracle and the stdout report pinned to the reference's own runs at >= 2^22 keys
(tests/golden/ref_large.json, made by tests/golden/make_golden.py --large from `mpirun -np P`
runs of the reference binaries): CPU only, at 2^22 keys to keep the suite short (the 2^24
cases are compared on the GPU, tests/test_gpu_golden_large.py)."""
import hashlib

import numpy as np
import pytest

from conftest import GOLDEN_DEBUG


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<i4").tobytes()).hexdigest()


def keys_of(orc, c):
    s = c["input"]
    return orc.gen(orc.UNIFORM if s["gen"] == "uniform" else orc.ZIPF, s["seed"], s["n"])


def small(ref_large):
    return [c for c in ref_large if c["input"]["n"] == 1 << 22]


def test_large_inputs_regenerate(orc, ref_large):
    seen = set()
    for c in ref_large:
        k = tuple(sorted(c["input"].items()))
        if k in seen:
            continue
        seen.add(k)
        assert sha(keys_of(orc, c)) == c["input_sha256"], c["id"]


def test_large_outputs_are_the_numeric_sort(orc, ref_large):
    """Every reference run at these sizes printed the ascending sort (the parity domain; the
    Zipf sample-sort runs did not overflow their buffers here) -- and the build's 8-bit LSD
    restatement gives the same array."""
    done = set()
    for c in ref_large:
        assert c["rc"] == 0 and c["output_is_sorted_input"], c["id"]
        s = c["input"]
        if s["n"] != 1 << 22 or (s["gen"], s["seed"]) in done:
            continue
        done.add((s["gen"], s["seed"]))
        keys = keys_of(orc, c)
        assert sha(orc.lsd8(keys)) == c["output_sha256"], c["id"]
    assert len(done) == 2


def test_large_sample_restatement(orc, ref_large):
    """The oracle's restatement of mpi_sample_sort.c (splitters :109-128, bucket matrix
    :148-158, output) against the reference's own run, at 2^22 keys, P = 2 / 4 / 8."""
    n = 0
    for c in small(ref_large):
        if c["prog"] != "sample_sort":
            continue
        rc, out, spl, mat, _ = orc.ref_sample(keys_of(orc, c), c["P"])
        assert rc == orc.OK, c["id"]
        assert spl.tolist() == c["splitters"] and mat.tolist() == c["bucket_matrix"], c["id"]
        assert sha(out) == c["output_sha256"], c["id"]
        n += 1
    assert n == 5


def test_large_radix_restatement_p8(orc, ref_large):
    """The oracle's restatement of mpi_radix_sort.c's base-P passes (11 passes at P = 8)."""
    c = next(x for x in small(ref_large) if x["prog"] == "radix_sort" and x["P"] == 8 and
             x["input"]["gen"] == "uniform")
    rc, out, passes = orc.ref_radix(keys_of(orc, c), 8)
    assert rc == orc.OK and passes == 11
    assert sha(out) == c["output_sha256"]


@pytest.mark.parametrize("prog", ["radix_sort", "sample_sort"])
def test_large_report_byte_for_byte(gsort, orc, ref_large, prog):
    """gsort_write_report on the reference's own splitters / bucket rows / sorted array
    reproduces every rank's stdout contract digest of the 2^22-key runs."""
    for c in small(ref_large):
        if c["prog"] != prog:
            continue
        keys = np.sort(keys_of(orc, c))
        P = c["P"]
        mat = c.get("bucket_matrix") or [[0] * P for _ in range(P)]
        for r in range(P):
            data = gsort.report_bytes(
                gsort.REPORT_SAMPLE if prog == "sample_sort" else gsort.REPORT_RADIX, r, P,
                GOLDEN_DEBUG[prog], keys.size, splitters=c.get("splitters") or None,
                bucket_counts=mat[r], sorted_keys=keys if r == 0 else None)
            assert hashlib.sha256(data).hexdigest() == c["contract"][r]["sha256"], (c["id"], r)
