"""GPU tests of the drop-in programs (mpi-test_amd/bin/radix_sort, sample_sort): same argv,
text input, stdout / stderr lines and sorted dump as the reference programs,
checked against the reference's own output captured in tests/golden/.  One rank (this box has
one GPU); multi-rank placement is covered by tests/test_gpu_sort.py's in-process groups."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, case_input, case_output

pytestmark = pytest.mark.gpu
BIN = os.path.join(ROOT, "mpi-test_amd", "bin")
DUMP = re.compile(r"^(\d+)\|(\d+)$")


def run(prog, path, debug=None, timeout=120):
    cmd = [os.path.join(BIN, prog), path] + ([str(debug)] if debug is not None else [])
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)


def dump_of(stdout):
    vals = {}
    for ln in stdout.splitlines():
        m = DUMP.match(ln)
        if m:
            u = int(m.group(2))
            vals[int(m.group(1))] = u - (1 << 32) if u >= 1 << 31 else u
    return np.array([vals[i] for i in sorted(vals)], dtype=np.int32)


@pytest.mark.parametrize("prog,debug", [("radix_sort", 3), ("sample_sort", 1)])
def test_cli_dump_matches_reference(orc, ref_cases, ref_outputs, tmp_path, prog, debug):
    done = 0
    for c in ref_cases:
        spec = c["input"]
        if "gen" not in spec or c["rc"] != 0 or c["P"] != 2 or c["prog"] != prog:
            continue
        keys = case_input(orc, spec)
        path = str(tmp_path / "in.txt")
        orc.write_text(path, keys)
        r = run(prog, path, debug)
        assert r.returncode == 0, r.stderr
        assert np.array_equal(dump_of(r.stdout), case_output(c, ref_outputs)), c["id"]
        assert c["median_line"] in r.stdout.splitlines()
        assert re.search(r"^Endtime\(\)-Starttime\(\) = \d+\.\d{5} sec$", r.stderr, re.M)
        if prog == "sample_sort":
            assert f"Each bucket will be put {keys.size} items." in r.stdout  # P = 1: B = N
        done += 1
    assert done >= 3


def test_cli_default_output_is_only_the_contract_lines(orc, tmp_path):
    keys = orc.gen(orc.UNIFORM, 42, 1 << 16)
    path = str(tmp_path / "in.txt")
    orc.write_text(path, keys)
    r = run("radix_sort", path)
    assert r.returncode == 0
    assert r.stdout.splitlines() == [f"The n/2-th sorted element: {np.sort(keys)[(1 << 15) - 1]}"]
    assert len(r.stderr.strip().splitlines()) >= 1
    r = run("sample_sort", path)
    assert r.stdout.splitlines() == [f"Each bucket will be put {1 << 16} items.",
                                     f"The n/2-th sorted element: {np.sort(keys)[(1 << 15) - 1]}"]


def test_cli_quirk_inputs(orc, tmp_path):
    """Q7: out-of-range text wraps like glibc %d; negative keys sort numerically (the build's
    contract; the reference sorts by |v| mod P^loop, Q2 -- a documented divergence)."""
    p = tmp_path / "q.txt"
    p.write_text("2147483648 4294967295 12 -5 0 4294967296 77 1\n")
    r = run("radix_sort", str(p), 3)
    assert r.returncode == 0
    assert dump_of(r.stdout).tolist() == sorted([-2**31, -1, 12, -5, 0, 0, 77, 1])
    assert "The n/2-th sorted element: 0" in r.stdout


def test_cli_large_text(orc, tmp_path):
    """2^22 keys through the text path (parallel reader, H2D, sort, D2H)."""
    n = 1 << 22
    path = str(tmp_path / "big.txt")
    subprocess.run([os.path.join(BIN, "gen_keys"), "zipf", str(n), "9", path], check=True)
    keys = orc.gen(orc.ZIPF, 9, n)
    r = run("sample_sort", path)
    assert r.returncode == 0
    assert f"The n/2-th sorted element: {np.sort(keys)[n // 2 - 1]}" in r.stdout
