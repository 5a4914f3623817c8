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


def _split_case(rng, P, kind):
    n_all = rng.integers(0, 3000, P)
    if kind == "empty_ranks":
        n_all[rng.integers(0, P, max(1, P // 2))] = 0
    if kind == "tiny":
        n_all = rng.integers(0, 2, P)
    hi = {"uniform": 2**31, "dups": 5, "one_value": 1, "empty_ranks": 100, "tiny": 3}[kind]
    blocks = [np.sort(rng.integers(-hi, hi, int(k)).astype(np.int32)) for k in n_all]
    return [int(k) for k in n_all], blocks


@pytest.mark.parametrize("kind", ["uniform", "dups", "one_value", "empty_ranks", "tiny"])
def test_plan_split_yields_the_global_blocks(gsort, kind):
    """gsort_plan_split (the distributed radix's one exchange): with lt/le taken at the exact
    boundary keys, the runs every rank receives concatenate to its global block
    [qB, (q+1)B) of the sorted multiset -- including duplicate-heavy and empty ranks."""
    rng = np.random.default_rng(sum(map(ord, kind)))
    for P in (2, 3, 4, 5, 8):
        for trial in range(6):
            n_all, blocks = _split_case(rng, P, kind)
            allk = np.sort(np.concatenate(blocks)) if sum(n_all) else np.zeros(0, np.int32)
            N = allk.size
            B = -(-N // P) if N else 0
            lt = np.zeros((P, P - 1), np.uint64)
            le = np.zeros((P, P - 1), np.uint64)
            for q in range(1, P):
                g = min(q * B, N)
                for p in range(P):
                    if g >= N:
                        lt[p, q - 1] = le[p, q - 1] = n_all[p]
                    else:
                        v = allk[g]
                        lt[p, q - 1] = np.searchsorted(blocks[p], v, "left")
                        le[p, q - 1] = np.searchsorted(blocks[p], v, "right")
            sends = [gsort.plan_split(n_all, lt, le, me) for me in range(P)]
            for q in range(P):
                # rank q receives, in rank order, the slice each p sends to q
                parts = []
                for p in range(P):
                    s_p = sends[p][0]
                    a = int(s_p[:q].sum())
                    parts.append(blocks[p][a:a + int(s_p[q])])
                    assert sends[q][1][p] == s_p[q]
                got = np.sort(np.concatenate(parts))
                assert np.array_equal(got, allk[q * B:(q + 1) * B]), (P, trial, q)


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


def test_text_parser_matches_glibc_fscanf(gsort, orc, tmp_path):
    """gsort_parse_text (the CLIs' rank-0 reader) == the reference's fscanf("%d") loop
    (mpi_radix_sort.c:85-97) without its trailing-delimiter phantom (Q6)."""
    rng = np.random.default_rng(5)
    toks = ["0", "-0", "+7", "2147483647", "2147483648", "-2147483648", "-2147483649",
            "4294967295", "4294967296", "99999999999999999999", "-99999999999999999999",
            "9223372036854775807", "9223372036854775808", "-9223372036854775809", "00012"]
    toks += [str(int(x)) for x in rng.integers(-2**40, 2**40, 300)]
    seps = [" ", "\n", "\t", "  \r\n", "\v", "\f"]
    for trial in range(20):
        picked = rng.choice(toks, 200)
        text = "".join(t + seps[int(rng.integers(0, len(seps)))] for t in picked)
        if trial % 2:
            text = text.rstrip()
        p = tmp_path / f"t{trial}.txt"
        p.write_text(text)
        want = orc.read_ints(str(p), with_phantom=False)
        for th in (1, 4):
            got = gsort.parse_text(text, threads=th)
            assert got is not None and np.array_equal(got, want), (trial, th)
    assert gsort.parse_text("1 2 x 3") is None
    assert gsort.parse_text("12,13") is None
    assert gsort.parse_text("") is not None and gsort.parse_text("").size == 0


def test_text_parser_parallel_large(gsort, orc):
    keys = orc.gen(orc.UNIFORM, 3, 1 << 20) - (1 << 30)
    text = "\n".join(map(str, keys.tolist()))
    assert np.array_equal(gsort.parse_text(text, threads=8), keys)


def test_dump_formatter_matches_printf(gsort, orc):
    """gsort_format_dump (the CLIs' sorted dump) == the reference's
    printf("%u|%u\n", i, int_buf[i]) lines (mpi_radix_sort.c:198-200), negatives as 2^32+v
    (Q15), on one and many threads and from a nonzero first index (the CLI's blocks)."""
    keys = np.concatenate([orc.gen(orc.UNIFORM, 4, 100000) - (1 << 30),
                           np.array([0, -1, 2**31 - 1, -2**31, 9, 10, 99, 100], np.int32)])
    for first in (0, 999_999_999_995):
        want = "".join(f"{first + i}|{int(v) & 0xFFFFFFFF}\n" for i, v in enumerate(keys.tolist()))
        for th in (1, 7, 16):
            assert gsort.format_dump(keys, first, th) == want.encode(), (first, th)
    assert gsort.format_dump(np.zeros(0, np.int32)) == b""


def test_cli_contract_without_gpu(tmp_path):
    """argv / invalid-file handling happens before any GPU call."""
    import subprocess
    exe = os.path.join(ROOT, "mpi-test_amd", "bin", "radix_sort")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and f"Usage: {exe} <file: Data file to read>" in r.stderr
    r = subprocess.run([exe, "a", "b", "c"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "Usage:" in r.stderr
    missing = str(tmp_path / "missing.txt")
    r = subprocess.run([exe, missing], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0
    assert f"sort(): '{missing}' is not a valid file for read." in r.stderr
    bad = tmp_path / "bad.txt"
    bad.write_text("1 2 three")
    r = subprocess.run([os.path.join(ROOT, "mpi-test_amd", "bin", "sample_sort"), str(bad)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "is not a valid file for read." in r.stderr


def test_uid_bytes_survive_marshalling(gsort):
    """An RCCL unique id holds NUL bytes (socket address, port): the ctypes struct must carry
    all 128 bytes both ways (a c_char array field stops at the first NUL)."""
    raw = bytes([2, 0, 0x1F, 0x90, 127, 0, 0, 1] + [0] * 56 + list(range(1, 65)))
    u = gsort.Uid.from_bytes(raw)
    assert u.to_bytes() == raw
    assert bytes(u.internal) == raw


def _balanced_cut_model(n_all, blocks, spl):
    """Python model of gsort_plan_split_balanced: boundary q sits at
    clamp(min(qB, N), LT + 1, LE) of splitter spl[q-1] (LT + 1 only when the value occurs);
    copies of the splitter value are taken in rank order."""
    P = len(blocks)
    N = sum(n_all)
    B = -(-N // P) if N else 0
    cut = [[0] * (P + 1) for _ in range(P)]
    for p in range(P):
        cut[p][P] = n_all[p]
    for q in range(1, P):
        v = spl[q - 1]
        lt = [int(np.searchsorted(b, v, "left")) for b in blocks]
        le = [int(np.searchsorted(b, v, "right")) for b in blocks]
        g = min(max(min(q * B, N), sum(lt) + (sum(le) > sum(lt))), sum(le))
        left = g - sum(lt)
        for p in range(P):
            take = min(max(left, 0), le[p] - lt[p])
            cut[p][q] = n_all[p] if g >= N else lt[p] + take
            left -= le[p] - lt[p]
    return cut


@pytest.mark.parametrize("kind", ["uniform", "dups", "one_value", "empty_ranks", "tiny"])
def test_plan_split_balanced_sample_buckets(gsort, kind):
    """gsort_plan_split_balanced (duplicate-aware sample-sort buckets): matches the model, the
    buckets concatenate to the sorted multiset (duplicate-heavy and empty ranks too), and a
    splitter value held once cuts exactly where the reference's rule does (keys <= s_j go to
    bucket j, mpi_sample_sort.c:148-155)."""
    rng = np.random.default_rng(7 + sum(map(ord, kind)))
    for P in (2, 3, 4, 8):
        for trial in range(6):
            n_all, blocks = _split_case(rng, P, kind)
            allk = np.sort(np.concatenate(blocks)) if sum(n_all) else np.zeros(0, np.int32)
            if allk.size == 0:
                continue
            spl = np.sort(rng.choice(allk, P - 1))
            lt = np.array([[np.searchsorted(b, v, "left") for v in spl] for b in blocks],
                          np.uint64).reshape(P, P - 1)
            le = np.array([[np.searchsorted(b, v, "right") for v in spl] for b in blocks],
                          np.uint64).reshape(P, P - 1)
            sends = [gsort.plan_split(n_all, lt, le, me, balanced=True) for me in range(P)]
            cut = _balanced_cut_model(n_all, blocks, spl)
            buckets = []
            for q in range(P):
                parts = []
                for p in range(P):
                    assert int(sends[p][0][q]) == cut[p][q + 1] - cut[p][q], (P, trial, p, q)
                    assert sends[q][1][p] == sends[p][0][q]
                    parts.append(blocks[p][cut[p][q]:cut[p][q + 1]])
                buckets.append(np.sort(np.concatenate(parts)))
            assert np.array_equal(np.concatenate(buckets), allk)
            for q in range(1, P):
                if int(le[:, q - 1].sum()) - int(lt[:, q - 1].sum()) == 1:
                    for p in range(P):
                        assert cut[p][q] == int(le[p, q - 1]) or cut[p][q] == n_all[p]


def test_kernels_isa_scc_hazard():
    """The gfx950 code object has no SCC consumer fed by an arithmetic SCC writer: the ROCm 7.2
    miscompile that made K1h read up to 32 KiB past its input (tools/isa_scc_check.py; K1h
    now computes tile lengths in 32-bit scalar arithmetic).  Disassembles the built library."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_scc_check.py")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]


def test_hot_kernels_use_no_scratch():
    """No hot-path kernel may spill VGPRs to scratch: a K18c restructure that ran into the
    128-VGPR limit of 1024-thread workgroups spilled 1480 B per lane and ran 4x slower.  Reads
    the built code object's notes (private_segment_fixed_size) for every kernel of the sort."""
    import subprocess
    import tempfile
    llvm = "/opt/rocm/lib/llvm/bin"
    lib = os.path.join(ROOT, "mpi-test_amd", "lib", "libgsort.so")
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "g.co")
        subprocess.run([f"{llvm}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib],
                       check=True)
        subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o",
                        f"--input={fat}", f"--output={co}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True)
        notes = subprocess.run([f"{llvm}/llvm-readelf", "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    name, spills = None, []
    for line in notes.splitlines():
        line = line.strip()
        if line.startswith(".name:"):
            name = line.split(":", 1)[1].strip()
        elif line.startswith(".private_segment_fixed_size:") and name:
            if int(line.split(":", 1)[1]) > 0:
                spills.append(name)
    hot = ("k_partition_res", "k_local_sort_e", "k_local_sort", "k_est_sample", "k_hist16",
           "k_count_expand", "k_gather_sort", "k_giant_hist", "k_giant_expand")
    bad = [n for n in spills if any(h in n for h in hot)]
    assert not bad, bad


def test_bench_roofline_traffic_takes_the_dominant_instantiation():
    """bench.py prices the dominant kernel's HBM traffic from the newest committed PMC summary:
    of K11e's size classes it must take the one holding the time (the 2^28 launches), not an
    average with the small class the bench's 2^24 reference check runs."""
    import importlib.util
    import json
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    got = bench.pmc_traffic("radix", 1 << 28, 1, ("k_local_sort_e",))
    assert got is not None
    d = json.load(open(os.path.join(root, got["source"])))["kernels"]
    k11e = [v for k, v in d.items() if k.startswith("k_local_sort_e")]
    top = max(k11e, key=lambda v: v["avg_us"] * v["calls"])
    assert got["hbm_bytes_per_launch"] == round(top["hbm_bytes"])
    # 2 B read + 4 B written per key at 2^28 keys, within the PMC's few % of overhead
    assert 0.95 < got["hbm_bytes_per_launch"] / (6 * (1 << 28)) < 1.15
