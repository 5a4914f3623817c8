"""bench.py's N > 1 flow on one GPU: the ranks share the card through the IPC process group, so
the path the driver's multi-GPU scaling runs take -- rank processes, uid broadcast, barriers,
max-over-ranks timing, the exchange, verify_rows (multiset, per-rank order, sizes) and the
strong-scaling block -- runs end to end here, under both launchers (torch.distributed.run and
bench.py's own spawn).  The numbers price nothing (two ranks on one GPU); the verification
fields must hold.  The RCCL transport itself needs one GPU per rank (tests/test_gpu_multigpu.py).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(args, ranks, torchrun, timeout=110, env=None):
    bench = os.path.join(ROOT, "bench.py")
    tail = ["--gpus", str(ranks), "--steps", "2", "--warmup", "1", "--settle-ms", "0"] + args
    if torchrun:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={ranks}", "--master-addr", "127.0.0.1",
               "--master-port", str(_port()), bench] + tail
    else:
        cmd = [sys.executable, bench] + tail
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0]), r.stderr


def _common(line, ranks, keys_log2):
    assert line["n_gpus"] == ranks and line["scaling"] == "weak"
    assert line["transport"].startswith("ipc")
    assert line["verified"] is True
    assert line["config"]["total_keys"] == ranks << keys_log2
    assert line["value"] > 0 and line["ms_per_step"] > 0


def test_bench_torchrun_radix_2_ranks_with_strong_block():
    """The driver's launcher: 2 ranks, 2^22 keys each, then configs[2]'s strong-scaling block
    (2^31 keys in total: 2^30 per rank -- the staging size that once hung the IPC group)."""
    line, err = _run(["--keys-log2", "22", "--strong"], 2, torchrun=True)
    _common(line, 2, 22)
    assert line["exchange"]["max_pair_bytes"] > 0
    st = line["strong_scaling_cfg2"]
    assert st["verified"] is True and st["scaling"] == "strong"
    assert st["total_keys"] == 1 << 31 and st["exchange"]["max_pair_bytes"] > 0
    assert "strong-scaling block done" in err


def test_bench_self_spawn_sample_2_ranks():
    """bench.py --gpus 2 without WORLD_SIZE spawns its own ranks; sample sort's exchange."""
    line, _ = _run(["--keys-log2", "21", "--algo", "sample"], 2, torchrun=False)
    _common(line, 2, 21)


def test_bench_torchrun_radix_3_ranks_zipf():
    """An odd world size and skewed keys (Zipf: most keys in a few 16-bit buckets); ranks
    sharing the GPU skip the strong-scaling block by default."""
    line, _ = _run(["--keys-log2", "20", "--dist", "zipf"], 3, torchrun=True)
    _common(line, 3, 20)
    assert "strong_scaling_cfg2" not in line


def test_bench_rccl_setup_failure_falls_back_to_ipc():
    """GSORT_TRANSPORT=rccl with two ranks on one GPU: RCCL refuses the communicator, every
    rank sees the failure (gloo all-reduce), the group re-forms over IPC, the run completes
    verified and the line names the fallback -- what bench.py does if RCCL cannot form on a
    multi-GPU node instead of ending without a line."""
    line, err = _run(["--keys-log2", "20", "--no-strong"], 2, torchrun=True,
                     env={"GSORT_TRANSPORT": "rccl"})
    assert line["verified"] is True
    assert "rccl communicator setup failed" in line["transport"], line["transport"]
    assert "re-forming over the IPC group" in err
