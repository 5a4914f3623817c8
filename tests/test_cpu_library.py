"""CPU-only checks of the product library: it loads, exports every symbol include/gsort.h
declares, and its host-side planners agree with the oracle.  No compute call touches a GPU."""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, case_input


def header_symbols():
    src = open(os.path.join(ROOT, "include", "gsort.h")).read()
    return sorted(set(re.findall(r"\b(gsort_[a-z_]+)\s*\(", src)))


def test_library_exports_every_header_symbol(gsort):
    L = gsort.lib()
    declared = header_symbols()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(L, name), name
    assert set(declared) == set(gsort.EXPORTS)


def test_strerror_and_tile(gsort):
    L = gsort.lib()
    assert L.gsort_strerror(gsort.ENOSAMPLE).decode().startswith("not enough")
    assert gsort.onesweep_tile() % 64 == 0


def test_radix_route_matches_oracle(gsort, orc):
    rng = np.random.default_rng(0)
    for P in (1, 2, 3, 4, 8):
        for trial in range(4):
            n = int(rng.integers(0, 20000))
            keys = orc.gen(orc.ZIPF if trial % 2 else orc.UNIFORM, trial, n)
            B = -(-n // P) if n else 0
            blocks = [keys[r * B:(r + 1) * B] for r in range(P)]
            hist = np.stack([orc.digit_hist(b, trial % 4) for b in blocks])
            for me in range(P):
                s1, r1, g1 = gsort.plan_radix_route(hist, max(B, 1), me)
                s2, r2, g2 = orc.radix_route(hist, max(B, 1), me)
                assert np.array_equal(s1, s2) and np.array_equal(r1, r2)
                assert np.array_equal(g1, g2), (P, trial, me)


def test_splitters_match_reference_fixtures(gsort, orc, ref_cases):
    n = 0
    for c in ref_cases:
        if c["prog"] != "sample_sort" or c["rc"] != 0:
            continue
        P = c["P"]
        keys = case_input(orc, c["input"])
        B = -(-keys.size // P)
        k = 2 * P - 1
        samples = np.concatenate(
            [np.sort(keys[r * B:(r + 1) * B])[np.arange(k) * (B // k)] for r in range(P)])
        assert gsort.plan_splitters(samples, P).tolist() == c["splitters"], c["id"]
        n += 1
    assert n >= 8


def test_no_cpu_fallback_without_gpu(gsort):
    """The product must fail loudly (not silently compute on the CPU) when no GPU is usable."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(gsort.GsortError):
        gsort.Context()
