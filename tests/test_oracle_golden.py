"""Pin the CPU oracle against the reference programs' own outputs (tests/golden/).

The fixtures were produced by tests/golden/make_golden.py, which runs the unchanged reference
binaries (oracle/_ref, built from /root/reference) under mpirun.  Nothing here needs a GPU.
"""
import hashlib
import os
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import case_input, case_output


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<i4").tobytes()).hexdigest()


def test_generator_streams_match_fixture_checksums(orc, ref_cases):
    for c in ref_cases:
        spec = c["input"]
        if "gen" in spec:
            assert sha(case_input(orc, spec)) == c["input_sha256"], c["id"]


def test_generator_counter_based(orc):
    full = orc.gen(orc.UNIFORM, 42, 1000)
    part = orc.gen(orc.UNIFORM, 42, 300, start=700)
    assert np.array_equal(full[700:], part)
    z = orc.gen(orc.ZIPF, 7, 1 << 16)
    assert z.min() >= 1 and z.max() <= 2**31 - 1
    assert 0.25 < np.mean(z == 1) < 0.33  # P(key=1) ~ 29.3 %
    u = orc.gen(orc.UNIFORM, 42, 1 << 16)
    assert u.min() >= 0


def test_ref_radix_restatement_matches_reference(orc, ref_cases, ref_outputs):
    n_checked = 0
    for c in ref_cases:
        if c["prog"] != "radix_sort" or "text" in c["input"]:
            continue
        keys = case_input(orc, c["input"])
        rc, out, passes = orc.ref_radix(keys, c["P"])
        assert rc == orc.OK, c["id"]
        assert np.array_equal(out, case_output(c, ref_outputs)), c["id"]
        assert c["median_line"] == f"The n/2-th sorted element: {out[keys.size // 2 - 1]}"
        n_checked += 1
    assert n_checked >= 14


def test_ref_sample_restatement_matches_reference(orc, ref_cases, ref_outputs):
    n_checked = 0
    for c in ref_cases:
        if c["prog"] != "sample_sort":
            continue
        keys = case_input(orc, c["input"])
        rc, out, spl, mat, recv = orc.ref_sample(keys, c["P"])
        if c["rc"] != 0:
            assert rc == orc.E_NO_SAMPLE, c["id"]  # Q9
            continue
        assert rc == orc.OK, c["id"]
        assert np.array_equal(out, case_output(c, ref_outputs)), c["id"]
        assert spl.tolist() == c["splitters"], c["id"]
        assert mat.tolist() == c["bucket_matrix"], c["id"]
        B = -(-keys.size // c["P"])
        assert c["each_bucket_line"] == f"Each bucket will be put {B} items."
        n_checked += 1
    assert n_checked >= 8


def test_in_parity_domain_outputs_are_the_numeric_sort(orc, ref_cases, ref_outputs):
    """Inside the parity domain both references output the ascending sort; the
    build's 8-bit LSD restatement reproduces exactly that array."""
    for c in ref_cases:
        spec = c["input"]
        if "gen" not in spec or "mod" in spec or c["P"] == 1 or c["rc"] != 0:
            continue
        keys = case_input(orc, spec)
        ref = case_output(c, ref_outputs)
        assert np.array_equal(ref, np.sort(keys)), c["id"]
        assert np.array_equal(orc.lsd8(keys), ref), c["id"]


def test_quirks_pinned(orc, ref_cases, ref_outputs):
    by = {c["id"]: c for c in ref_cases}
    # Q1: radix at P=1 runs zero passes -> input order
    c = by["uniform1000s42__radix_sort__P1"]
    keys = case_input(orc, c["input"])
    assert np.array_equal(case_output(c, ref_outputs), keys)
    rc, out, passes = orc.ref_radix(keys, 1)
    assert passes < 1 and np.array_equal(out, keys)
    # Q2: negatives sort by |v| mod P^loop, stable
    for P in (2, 4, 8):
        assert case_output(by[f"q2_neg8__radix_sort__P{P}"], ref_outputs).tolist() == \
            [0, -2, 2, 3, -3, 5, -7, 7]
    # Q3: P=3 under-counts digits at 243 (top digit skipped)
    c = by["q3_max243__radix_sort__P3"]
    assert orc.lib().orc_ref_number_digits(243, 3) == 5  # exact would be 6
    rc, out, _ = orc.ref_radix(case_input(orc, c["input"]), 3)
    assert np.array_equal(out, case_output(c, ref_outputs))


def test_reader_semantics(orc, ref_cases, ref_outputs, tmp_path):
    by = {c["id"]: c for c in ref_cases}
    # Q6: trailing newline appends a phantom copy of the last value in ref-radix
    p = tmp_path / "q6.txt"
    p.write_text(by["q6_trailing_nl__radix_sort__P2"]["input"]["text"])
    assert orc.read_ints(str(p), with_phantom=True).tolist() == [5, 3, 9, 1, 1]
    assert orc.read_ints(str(p), with_phantom=False).tolist() == [5, 3, 9, 1]
    assert sorted([5, 3, 9, 1, 1]) == case_output(by["q6_trailing_nl__radix_sort__P2"],
                                                   ref_outputs).tolist()
    # Q7: %d wraps out-of-range text mod 2^32
    c = by["q7_wrap__radix_sort__P2"]
    p = tmp_path / "q7.txt"
    p.write_text(c["input"]["text"])
    keys = orc.read_ints(str(p))
    assert keys.tolist() == [-2**31, -1, 12, -5, 0, 0, 77, 1]
    rc, out, _ = orc.ref_radix(keys, 2)
    assert rc == orc.OK and np.array_equal(out, case_output(c, ref_outputs))


@pytest.mark.skipif(not os.path.exists("/opt/conda/bin/mpirun"), reason="no mpirun")
def test_reference_binary_live_small(orc, tmp_path):
    """If the reference binaries are present (oracle/_ref), re-run one small case live."""
    exe = os.path.join(orc.REF_DIR, "radix_sort")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built")
    keys = orc.gen(orc.UNIFORM, 9, 512)
    path = str(tmp_path / "k.txt")
    orc.write_text(path, keys)
    out = subprocess.run(["/opt/conda/bin/mpirun", "-np", "2", exe, path], capture_output=True,
                         text=True, timeout=60)
    assert out.returncode == 0
    assert f"The n/2-th sorted element: {np.sort(keys)[255]}" in out.stdout


def test_radix_route_restatement(orc):
    """The distributed placement (K8) restated: simulate P ranks, route, place, compare."""
    rng = np.random.default_rng(3)
    for P in (1, 2, 3, 4, 8):
        n = 5000
        keys = (orc.gen(orc.UNIFORM, 11, n) >> int(rng.integers(0, 20))).astype(np.int32)
        B = -(-n // P)
        blocks = [keys[r * B:(r + 1) * B].copy() for r in range(P)]
        for pas in range(4):
            hist = np.stack([orc.digit_hist(b, pas) for b in blocks])
            # local stable partition by digit (what one onesweep pass does)
            dig = [((b.view(np.uint32) ^ 0x80000000) >> (8 * pas)) & 0xFF for b in blocks]
            local = [b[np.argsort(d, kind="stable")] for b, d in zip(blocks, dig)]
            sends = [orc.radix_route(hist, B, r) for r in range(P)]
            new = []
            for q in range(P):
                send_q, recv_q, seg = sends[q]
                chunks = []
                for r in range(P):  # what r sends to q: contiguous slice of r's local order
                    s_r = sends[r][0]
                    off = int(s_r[:q].sum())
                    chunks.append(local[r][off: off + int(s_r[q])])
                assert [c.size for c in chunks] == recv_q.tolist()
                out = np.empty(int(recv_q.sum()), dtype=np.int32)
                for src, coff, doff, ln in seg:
                    out[doff: doff + ln] = chunks[src][coff: coff + ln]
                new.append(out)
            blocks = new
        assert np.array_equal(np.concatenate(blocks), np.sort(keys))


def test_sample_plan_restatement(orc, ref_cases):
    for c in ref_cases:
        if c["prog"] != "sample_sort" or c["rc"] != 0:
            continue
        P = c["P"]
        keys = case_input(orc, c["input"])
        B = -(-keys.size // P)
        k = 2 * P - 1
        blocks = [np.sort(keys[r * B:(r + 1) * B]) for r in range(P)]
        samples = np.concatenate([b[np.arange(k) * (B // k)] for b in blocks])
        mats = []
        for b in blocks:
            spl, bounds = orc.sample_plan(samples, b, P)
            mats.append(np.diff(np.concatenate([[0], bounds.astype(np.int64)])).tolist())
        assert spl.tolist() == c["splitters"]
        assert mats == c["bucket_matrix"]


def test_fingerprint(orc):
    a = orc.gen(orc.UNIFORM, 1, 4096)
    s1, x1, ok1 = orc.fingerprint(a)
    s2, x2, ok2 = orc.fingerprint(np.sort(a))
    assert (s1, x1) == (s2, x2) and not ok1 and ok2
    b = np.sort(a)
    b[5] += 1
    assert orc.fingerprint(b)[:2] != (s2, x2)
