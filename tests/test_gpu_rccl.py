"""The distributed code path through a real communicator on a one-GPU machine.

RCCL refuses two ranks on one device, so multi-rank GPU tests use the in-process rank group;
these tests instead run a ONE-rank context with GSORT_FORCE_DIST=1, which makes
gsort_radix / gsort_sample take the distributed algorithms anyway: radix select, plan_split,
the packed 16-bit exchange (to self) and the receive-side sort -- over the in-process group
and over RCCL itself (ncclCommInitRank from a gsort_get_uid, ncclAllGather, grouped
ncclSend/ncclRecv, ncclBroadcast).  Output must equal the oracle's sort, bit for bit.

The cases run in ONE child process (this file with --child), as a real rank does: one process
per GPU and one communicator in it.  In the pytest process itself, an 8-rank in-process group
started after an RCCL communicator had lived and been destroyed there failed on the MI355X
box (first a failed 512 KiB hipMalloc, then an illegal-address fault surfacing at the next
launch; the same tests pass when the group runs first), so the RCCL communicator never shares
a process with the in-process groups.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DIST_CASES = [(t, a, d) for d in ("uniform", "zipf") for a in ("radix", "sample")
              for t in ("group", "rccl")]
SMALL_CASES = [0, 1, 5, 16384, 16385]


def _ctx(gsort, transport):
    if transport == "group":
        grp = gsort.Group(1)
        return gsort.Context(group=grp), grp
    return gsort.Context(rank=0, nranks=1, device=0, uid=gsort.get_uid()), None


def _case_distributed_path(gsort, orc, transport, algo, dist_name):
    n = (1 << 20) + 4321
    dist = orc.UNIFORM if dist_name == "uniform" else orc.ZIPF
    keys = orc.gen(dist, 11, n)
    ctx, grp = _ctx(gsort, transport)
    try:
        p = ctx.alloc(n * 4)
        ctx.generate(gsort.UNIFORM if dist_name == "uniform" else gsort.ZIPF, 11, 0, n, p)
        out, m, st = (ctx.radix if algo == "radix" else ctx.sample)(p, n)
        assert m == n
        assert st["exchanges"] == 1, "the distributed path ran"
        assert np.array_equal(ctx.to_host(out, m), np.sort(keys))
        # a second call on the same context reuses its buffers and communicator
        out, m, _ = (ctx.radix if algo == "radix" else ctx.sample)(p, n)
        assert np.array_equal(ctx.to_host(out, m), np.sort(keys))
        ctx.free(p)
    finally:
        ctx.close()
        if grp is not None:
            grp.close()


def _case_rccl_small(gsort, orc, n):
    keys = orc.gen(orc.UNIFORM, 5, n)
    ctx, _ = _ctx(gsort, "rccl")
    try:
        p = ctx.alloc(max(n, 1) * 4)
        if n:
            ctx.to_device(keys, p)
        out, m, _ = ctx.radix(p, n)
        assert m == n
        if n:
            assert np.array_equal(ctx.to_host(out, m), np.sort(keys))
        ctx.free(p)
    finally:
        ctx.close()


def _child():
    """Every case in this process; one JSON line of {case id: "ok" | error text}."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "mpi-test_amd")):
        sys.path.insert(0, p)
    import torch  # noqa: F401  (one HIP runtime per process, as conftest.gsort)
    import gsort
    from oracle import orc
    orc.lib()
    res = {}
    for c in DIST_CASES:
        try:
            _case_distributed_path(gsort, orc, *c)
            res["-".join(c)] = "ok"
        except Exception as e:  # reported per case by the parent
            res["-".join(c)] = repr(e)
        print("case", c, res["-".join(c)], file=sys.stderr, flush=True)
    for n in SMALL_CASES:
        try:
            _case_rccl_small(gsort, orc, n)
            res[f"small-{n}"] = "ok"
        except Exception as e:
            res[f"small-{n}"] = repr(e)
        print("case", n, res[f"small-{n}"], file=sys.stderr, flush=True)
    print("RCCL_RESULTS " + json.dumps(res), flush=True)


@pytest.fixture(scope="module")
def child_results():
    env = dict(os.environ, GSORT_FORCE_DIST="1")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env,
                       capture_output=True, text=True, timeout=300)
    for line in r.stdout.splitlines():
        if line.startswith("RCCL_RESULTS "):
            return json.loads(line[len("RCCL_RESULTS "):])
    pytest.fail(f"RCCL child exited {r.returncode} without results:\n{r.stderr[-4000:]}")


@pytest.mark.parametrize("case", DIST_CASES, ids=["-".join(c) for c in DIST_CASES])
def test_one_rank_distributed_path(child_results, case):
    assert child_results["-".join(case)] == "ok"


@pytest.mark.parametrize("n", SMALL_CASES)
def test_one_rank_rccl_small(child_results, n):
    assert child_results[f"small-{n}"] == "ok"


if __name__ == "__main__" and "--child" in sys.argv:
    _child()
