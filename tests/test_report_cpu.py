"""The drop-in programs' stdout contract (gsort_write_report, include/gsort.h) against the
reference's own per-rank stdout, byte for byte (sha256 of the contract lines, captured by
tests/golden/make_golden.py from mpirun runs of the reference at P = 1..8).  CPU only: the
report is host code; its inputs here are the reference's own splitters, bucket matrix rows and
sorted dump from the fixtures (the GPU tests feed it the build's)."""
import hashlib

import numpy as np
import pytest

from conftest import GOLDEN_DEBUG, case_output, contract_split


def report(gsort, case, rank, sorted_keys, stage=0):
    P = case["P"]
    sample = case["prog"] == "sample_sort"
    mat = case.get("bucket_matrix") or [[0] * P for _ in range(P)]
    return gsort.report_bytes(gsort.REPORT_SAMPLE if sample else gsort.REPORT_RADIX, rank, P,
                              GOLDEN_DEBUG[case["prog"]], case["n_dump"],
                              splitters=case.get("splitters") or None,
                              bucket_counts=mat[rank], sorted_keys=sorted_keys, stage=stage)


def test_report_matches_reference_stdout_byte_for_byte(gsort, ref_cases, ref_outputs):
    done = 0
    for c in ref_cases:
        if c["rc"] != 0 or "output_sha256" not in c:
            continue
        out = case_output(c, ref_outputs)
        for r in range(c["P"]):
            data = report(gsort, c, r, out if r == 0 else None)
            want = c["contract"][r]
            head, nd, tail = contract_split(data)
            assert (head, nd, tail) == (want["head"], want["n_dump"], want["tail"]), (c["id"], r)
            assert hashlib.sha256(data).hexdigest() == want["sha256"], (c["id"], r)
            done += 1
    assert done >= 60


def test_report_stages_split_at_the_sort(gsort, ref_cases, ref_outputs):
    """stage 1 (before the sort) + stage 2 (after the gather) == the whole report."""
    c = next(x for x in ref_cases if x["prog"] == "sample_sort" and x["P"] == 4 and x["rc"] == 0)
    out = case_output(c, ref_outputs)
    whole = report(gsort, c, 0, out)
    a, b = report(gsort, c, 0, out, stage=1), report(gsort, c, 0, out, stage=2)
    assert a + b == whole and a.decode().startswith("Each bucket will be put ")
    assert a == f"Each bucket will be put {-(-c['n_dump'] // 4)} items.\n".encode()


def test_report_quirks(gsort):
    """N = 1: the median is element 0 (the reference reads int_buf[-1], Q14); negative keys
    print as %u in the dump (Q15) and %d in the median line; radix without debug: one line."""
    d = gsort.report_bytes(gsort.REPORT_RADIX, 0, 1, 3, 1, sorted_keys=np.array([-5], np.int32))
    assert d == b"0|4294967291\nThe n/2-th sorted element: -5\n"
    d = gsort.report_bytes(gsort.REPORT_RADIX, 0, 2, 0, 4, sorted_keys=np.arange(4, dtype=np.int32))
    assert d == b"The n/2-th sorted element: 1\n"
    assert gsort.report_bytes(gsort.REPORT_RADIX, 1, 2, 3, 4) == b""
    with pytest.raises(gsort.GsortError):  # sample debug needs the bucket counts
        gsort.report_bytes(gsort.REPORT_SAMPLE, 1, 2, 1, 4)
