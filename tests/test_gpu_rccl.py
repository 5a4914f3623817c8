"""The distributed code path through a real communicator on a one-GPU machine.

RCCL refuses two ranks on one device, so multi-rank GPU tests use the in-process rank group;
these tests instead run a ONE-rank context with GSORT_FORCE_DIST=1, which makes
gsort_radix / gsort_sample take the distributed algorithms anyway: radix select, plan_split,
the packed 16-bit exchange (to self) and the receive-side sort -- over the in-process group
and over RCCL itself (ncclCommInitRank from a gsort_get_uid, ncclAllGather, grouped
ncclSend/ncclRecv, ncclBroadcast).  Output must equal the oracle's sort, bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ctx(gsort, transport):
    if transport == "group":
        grp = gsort.Group(1)
        return gsort.Context(group=grp), grp
    return gsort.Context(rank=0, nranks=1, device=0, uid=gsort.get_uid()), None


@pytest.mark.parametrize("transport", ["group", "rccl"])
@pytest.mark.parametrize("algo", ["radix", "sample"])
@pytest.mark.parametrize("dist_name", ["uniform", "zipf"])
def test_one_rank_distributed_path(gsort, orc, monkeypatch, transport, algo, dist_name):
    monkeypatch.setenv("GSORT_FORCE_DIST", "1")
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


@pytest.mark.parametrize("n", [0, 1, 5, 16384, 16385])
def test_one_rank_rccl_small(gsort, orc, monkeypatch, n):
    monkeypatch.setenv("GSORT_FORCE_DIST", "1")
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
