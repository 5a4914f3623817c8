"""The drop-in programs as the reference is run: `mpirun -np P radix_sort|sample_sort <file>
<debug>`, one process per rank.  This box has one GPU, so the P processes share it through the
same-node IPC process group (gsort_get_uid_ipc; RCCL refuses two ranks on one device): the
CLI's MPI bootstrap, per-process contexts, scatter / sort / gather across processes and the
report all run for real.  Each rank's stdout is compared byte for byte with the reference's
own (tests/golden: contract lines of `mpirun -np P` runs of the reference binaries)."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN_DEBUG, ROOT, case_input, contract_split

pytestmark = pytest.mark.gpu
BIN = os.path.join(ROOT, "mpi-test_amd", "bin")
MPIRUN = "/opt/conda/bin/mpirun"


def mpirun(prog, P, path, debug, tmp, timeout=150, env=None):
    cmd = [MPIRUN, "-np", str(P), "-outfile-pattern", f"{tmp}/o.%r", "-errfile-pattern",
           f"{tmp}/e.%r", os.path.join(BIN, prog), path] + ([str(debug)] if debug is not None else [])
    e = dict(os.environ, **(env or {}))
    r = subprocess.run(cmd, timeout=timeout, capture_output=True, text=True, env=e)
    outs, errs = [], []
    for q in range(P):
        p = os.path.join(tmp, f"o.{q}")
        outs.append(open(p, "rb").read() if os.path.exists(p) else b"")
        p = os.path.join(tmp, f"e.{q}")
        errs.append(open(p, errors="replace").read() if os.path.exists(p) else "")
    if r.returncode != 0:  # every rank's stderr and mpirun's own output, for the failure report
        print(f"mpirun rc={r.returncode}\nstdout: {r.stdout[-2000:]}\nstderr: {r.stderr[-2000:]}")
        for q in range(P):
            print(f"--- rank {q} stderr:\n{errs[q][-2000:]}")
    return r.returncode, outs, errs[0]


CASES = [("uniform65536s42", "radix_sort", P) for P in (2, 4, 8)] + \
        [("uniform65536s42", "sample_sort", P) for P in (2, 4, 8)] + \
        [("zipf65536s7", "radix_sort", 8), ("zipf65536s7", "sample_sort", 4),
         ("uniform1024s42", "sample_sort", 8)]


@pytest.mark.parametrize("name,prog,P", CASES)
def test_mpirun_stdout_equals_reference(orc, ref_cases, tmp_path, name, prog, P):
    c = next(x for x in ref_cases if x["id"] == f"{name}__{prog}__P{P}")
    keys = case_input(orc, c["input"])
    path = str(tmp_path / "in.txt")
    orc.write_text(path, keys)
    rc, outs, err0 = mpirun(prog, P, path, GOLDEN_DEBUG[prog], tmp_path)
    assert rc == 0, err0
    for r in range(P):
        want = c["contract"][r]
        assert contract_split(outs[r]) == (want["head"], want["n_dump"], want["tail"]), (c["id"], r)
        assert hashlib.sha256(outs[r]).hexdigest() == want["sha256"], (c["id"], r)
    assert err0.startswith("Endtime()-Starttime() = ") and err0.endswith(" sec\n")


@pytest.mark.parametrize("chunk", [None, 1 << 21])
@pytest.mark.parametrize("prog", ["radix_sort", "sample_sort"])
def test_mpirun_ipc_staging_regrowth_2p22(orc, ref_large, tmp_path, prog, chunk):
    """the IPC group's staging buffers start at 1 MiB and are re-allocated,
    re-exported and re-opened by the peers when a collective needs more -- the path on which
    per-collective export / open once failed.  The reference's 2^22-key uniform stream at P = 4
    moves ~1 M keys per rank (2-4 MiB payloads), so every rank's staging buffer grows mid-run;
    every rank's stdout must still equal the reference's own (tests/golden/ref_large.json).
    chunk: staging buffers exported as 2 MiB chunks (GSORT_IPC_CHUNK; the product's chunks are
    2^30 bytes -- one exported 2 GiB buffer hung both ranks in their first pull, 2^30 keys per
    rank at P = 2), so a 1 MiB chunk replaced by 2 MiB ones, growth by appended chunks (rank 0's
    16 MiB scatter: 8 chunks) and pulls across chunk boundaries all run here."""
    c = next(x for x in ref_large if x["id"] == f"uniform4194304s42__{prog}__P4")
    s = c["input"]
    keys = orc.gen(orc.UNIFORM, s["seed"], s["n"])
    path = str(tmp_path / "in.txt")
    orc.write_text(path, keys)
    env = {"GSORT_TRANSPORT": "ipc"}
    if chunk:
        env["GSORT_IPC_CHUNK"] = str(chunk)
    rc, outs, err0 = mpirun(prog, 4, path, GOLDEN_DEBUG[prog], tmp_path, timeout=300, env=env)
    assert rc == 0, err0
    for r in range(4):
        want = c["contract"][r]
        assert contract_split(outs[r]) == (want["head"], want["n_dump"], want["tail"]), r
        assert hashlib.sha256(outs[r]).hexdigest() == want["sha256"], r


def test_mpirun_default_debug_and_ragged(orc, tmp_path):
    """No debug argument, N % P != 0: only the median (radix) / "Each bucket" + median
    (sample) lines, from rank 0; the other ranks print nothing."""
    n = 100003
    keys = orc.gen(orc.UNIFORM, 3, n)
    path = str(tmp_path / "in.txt")
    orc.write_text(path, keys)
    med = f"The n/2-th sorted element: {np.sort(keys)[n // 2 - 1]}\n".encode()
    rc, outs, err0 = mpirun("radix_sort", 4, path, None, tmp_path)
    assert rc == 0, err0
    assert outs == [med, b"", b"", b""]
    rc, outs, err0 = mpirun("sample_sort", 4, path, None, tmp_path)
    assert rc == 0, err0
    assert outs[0] == f"Each bucket will be put {-(-n // 4)} items.\n".encode() + med
    assert outs[1:] == [b"", b"", b""]


def test_mpirun_no_enough_sample(orc, ref_cases, tmp_path):
    """N = 9 at P = 4: the reference prints "Each bucket" and aborts with "no enough sample"."""
    c = next(x for x in ref_cases if x["id"] == "q9_n9__sample_sort__P4")
    path = str(tmp_path / "in.txt")
    orc.write_text(path, case_input(orc, c["input"]))
    rc, outs, err0 = mpirun("sample_sort", 4, path, 1, tmp_path)
    assert rc != 0
    assert outs[0].decode().splitlines() == c["contract"][0]["head"]
    assert "no enough sample" in err0


def test_mpirun_sample_balanced(orc, ref_cases, tmp_path):
    """GSORT_SAMPLE_BALANCED=1 (duplicate-aware buckets): on Zipf keys the sorted dump and
    the median stay the reference's, the bucket lines differ (the copies of a splitter value
    are shared out instead of all going to the lower bucket)."""
    c = next(x for x in ref_cases if x["id"] == "zipf65536s7__sample_sort__P4")
    keys = case_input(orc, c["input"])
    path = str(tmp_path / "in.txt")
    orc.write_text(path, keys)
    rc, outs, err0 = mpirun("sample_sort", 4, path, 1, tmp_path,
                            env={"GSORT_SAMPLE_BALANCED": "1"})
    assert rc == 0, err0
    head, nd, tail = contract_split(outs[0])
    want = c["contract"][0]
    assert nd == want["n_dump"] and tail == want["tail"]
    lines = outs[0].decode().splitlines()
    dump = np.array([int(ln.split("|")[1]) for ln in lines if "|" in ln], dtype=np.int64)
    assert np.array_equal(dump.astype(np.uint32).view(np.int32), np.sort(keys))
    sizes = [sum(int(ln.split("=")[1]) for ln in o.decode().splitlines() if "Bucket" in ln)
             for o in outs]
    assert sum(sizes) == keys.size
    ref_sizes = [sum(c["bucket_matrix"][r]) for r in range(4)]
    assert sizes == ref_sizes  # each rank still sends its whole block
    recv = [sum(int(ln.split("=")[1]) for o in outs for ln in o.decode().splitlines()
                if f"Bucket {q}=" in ln) for q in range(4)]
    assert max(recv) < max(sum(c["bucket_matrix"][r][q] for r in range(4)) for q in range(4))
