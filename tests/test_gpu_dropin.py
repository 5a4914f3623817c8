"""The drop-in path at P > 1 ranks: rank 0's host array ->
gsort_scatter_from_root (the reference's MPI_Scatter, mpi_radix_sort.c:139 /
mpi_sample_sort.c:82) -> gsort_radix / gsort_sample -> gsort_gather_to_root (MPI_Gatherv,
radix:180-192 / sample:182-197) -> gsort_write_report, compared byte for byte with the
reference's own per-rank stdout (tests/golden, captured from `mpirun -np P` runs of the
reference).  P ranks run as P threads of one process (in-process group) on one GPU; the
multi-process form (mpirun + the IPC process group) is tests/test_gpu_cli_mpi.py."""
import hashlib
import threading

import numpy as np
import pytest

from conftest import GOLDEN_DEBUG, case_input, contract_split

pytestmark = pytest.mark.gpu


def run_dropin(gsort, keys, P, algo, debug=0, report=True):
    """Every rank: scatter from rank 0's array, sort, gather to rank 0, report.  Returns
    (per-rank stdout bytes, rank 0's gathered array, per-rank sample info)."""
    N = 0 if keys is None else keys.size
    grp = gsort.Group(P)
    outs, infos, errs = [None] * P, [None] * P, []
    gathered = [None]

    def worker(r):
        try:
            with gsort.Context(rank=r, group=grp) as c:
                d, n = c.scatter_from_root(keys if r == 0 else None, N)
                fn = c.radix if algo == "radix" else c.sample
                out, n_out, _ = fn(d, n, stats=False)
                spl, cnt = c.sample_info() if algo == "sample" else (None, None)
                infos[r] = (spl, cnt, n_out)
                g = c.gather_to_root(out, n_out, N)
                if r == 0:
                    gathered[0] = g
                if report:
                    outs[r] = gsort.report_bytes(
                        gsort.REPORT_RADIX if algo == "radix" else gsort.REPORT_SAMPLE, r, P,
                        debug, N, splitters=spl, bucket_counts=cnt,
                        sorted_keys=g if r == 0 else None)
        except Exception as e:
            errs.append((r, e))

    th = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    if any(t.is_alive() for t in th):
        pytest.fail("in-process group did not finish within 600 s")
    grp.close()
    if errs:
        raise errs[0][1]
    return outs, gathered[0], infos


def check_contract(outs, case):
    for r, data in enumerate(outs):
        want = case["contract"][r]
        head, nd, tail = contract_split(data)
        assert (head, nd, tail) == (want["head"], want["n_dump"], want["tail"]), (case["id"], r)
        assert hashlib.sha256(data).hexdigest() == want["sha256"], (case["id"], r)


@pytest.mark.parametrize("prog", ["radix_sort", "sample_sort"])
def test_dropin_group_stdout_equals_reference(gsort, orc, ref_cases, prog):
    """Every generated-input golden case at P = 2, 4, 8: each rank's stdout contract lines --
    the dump, median, "Each bucket", splitter and bucket lines -- equal the reference's."""
    done = 0
    for c in ref_cases:
        if c["prog"] != prog or c["rc"] != 0 or "gen" not in c["input"] or c["P"] < 2:
            continue
        keys = case_input(orc, c["input"])
        algo = "radix" if prog == "radix_sort" else "sample"
        outs, g, _ = run_dropin(gsort, keys, c["P"], algo, GOLDEN_DEBUG[prog])
        assert np.array_equal(g, np.sort(keys))
        check_contract(outs, c)
        done += 1
    assert done >= (9 if prog == "radix_sort" else 8)


@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("n", [0, 1, 3, 1001, 65539])
def test_dropin_group_radix_ragged_sizes(gsort, orc, P, n):
    """N % P != 0 (the reference over-reads / overflows there, Q8), N < P (empty blocks), N = 0:
    rank q still holds positions [qB, (q+1)B) and rank 0 gathers the sorted array."""
    keys = orc.gen(orc.UNIFORM, n + P, n) - (1 << 30) if n else np.zeros(0, np.int32)
    outs, g, infos = run_dropin(gsort, keys if n else None, P, "radix", 3)
    assert np.array_equal(g, np.sort(keys))
    B = -(-n // P)
    assert [i[2] for i in infos] == [max(0, min(B, n - q * B)) for q in range(P)]
    head, nd, tail = contract_split(outs[0])
    assert head == [] and nd == n
    assert tail == ([f"The n/2-th sorted element: {np.sort(keys)[max(n // 2 - 1, 0)]}"] if n else [])
    assert all(o == b"" for o in outs[1:])


@pytest.mark.parametrize("P", [2, 4, 8])
def test_dropin_group_sample_ragged_and_too_small(gsort, orc, P):
    n = 65539  # N % P != 0
    keys = orc.gen(orc.UNIFORM, P, n)
    outs, g, infos = run_dropin(gsort, keys, P, "sample", 1)
    assert np.array_equal(g, np.sort(keys))
    assert sum(i[2] for i in infos) == n
    head, nd, _ = contract_split(outs[0])
    assert head[0] == f"Each bucket will be put {-(-n // P)} items." and nd == n
    # a block too small for the 2P - 1 regular samples (N = P - 1: the last block is empty):
    # every rank fails with GSORT_ENOSAMPLE (the reference aborts with "no enough sample",
    # mpi_sample_sort.c:94-99)
    with pytest.raises(gsort.GsortError) as e:
        run_dropin(gsort, keys[: P - 1], P, "sample", 0, report=False)
    assert e.value.status == gsort.ENOSAMPLE


@pytest.mark.parametrize("P,algo", [(4, "radix"), (8, "sample"), (2, "sample")])
def test_dropin_group_2p26(gsort, orc, P, algo):
    """A 2^26-key drop-in run: staged H2D on rank 0, scatter, sort, gather, staged D2H."""
    n = 1 << 26
    keys = orc.gen(orc.UNIFORM, 26, n)
    outs, g, _ = run_dropin(gsort, keys, P, algo, 0)
    assert np.array_equal(g, np.sort(keys))
    med = f"The n/2-th sorted element: {g[n // 2 - 1]}\n".encode()
    assert outs[0].endswith(med)
