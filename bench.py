#!/usr/bin/env python3
"""bench.py -- sorted keys/sec of the MI355X-native distributed sorter (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--algo radix|sample]
                    [--keys-log2 28] [--dist uniform|zipf] [--no-cpu-baseline]

One step = one gsort_radix (or gsort_sample) call over keys already resident in HBM: at N = 1
this is BASELINE.json configs[1] ("Radix sort 2^28 uniform random 32-bit keys on 1 MI355X");
at N > 1 every GPU holds 2^28 keys (weak scaling: 2^28 * N keys sorted globally, with a per-pass
RCCL all-to-all over xGMI -- configs[2] is the N = 8 point, 2^31 keys).  Keys come from the
canonical splitmix64 generator on device (K10), so the data is synthetic and identical to what
the oracle and the reference CPU run see.

The timed region is K steps bracketed by a barrier + torch.cuda.synchronize() on both sides;
the slowest rank's time is reported.  Before the W warm-up steps every rank runs the library's
streaming copy for --settle-ms (default 100 ms; reported as `settle`): from idle the GPU needs
tens of ms of load to reach its sustained clocks, and 5 warm-up sorts (~7 ms) did not get
there -- the same build measured 1.364-1.369 ms per step without it, 1.331-1.335 ms with
30-300 ms of copies first, 1.353 ms with 50 warm-up sorts.

`roofline` prices the dominant kernel class (by total device time: on the sampled plan K3r, K3a or K11e -- 8, 6 and 6 B/key of algorithmic traffic; K3u, K11 or an LSD pass on the other plans)
with its average duration measured live by HIP events recorded on libgsort's own stream
around every launch; `traffic` is the HBM bytes per launch from the rocprofv3 PMC summary in
profiles/ (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction) when one exists for this
configuration, else null; `copy_ceiling` is a device-to-device copy of the same 2^k keys
timed on this GPU (the practical ceiling of a read + write pass).  `drop_in` (N = 1) times
the reference's own timer span -- rank-0 host array -> GPU -> sorted -> rank-0 host array --
PCIe included; it is reported beside `value`, never as it.  `cpu_baseline` runs the reference
radix_sort (oracle/_ref, built unchanged from its source) under mpirun on a bounded 2^24-key
sample of the same stream on the host's cores (rank 0, N = 1 only), before the GPU is touched.
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "mpi-test_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "sorted keys/sec (GKeys/s) at 1/2/4/8 GPUs + % HBM/xGMI roofline"
HBM_PEAK_GBPS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
XGMI_LINK_GBPS = 153.0      # one xGMI link, per direction
PASS_BYTES_PER_KEY = 8      # K3 pass: read 4 B + write 4 B per key


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="streaming copies for this long before the warm-up steps (0: none)")
    ap.add_argument("--algo", choices=["radix", "sample"], default="radix")
    ap.add_argument("--keys-log2", type=int, default=28)
    ap.add_argument("--dist", choices=["uniform", "zipf"], default="uniform")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cpu-large", action="store_true",
                    help="skip the reference's 2^28-key point (~1 min of host time)")
    ap.add_argument("--no-dist-p1", action="store_true",
                    help="skip the one-rank distributed-path block")
    ap.add_argument("--no-strong", action="store_true",
                    help="N > 1: skip the configs[2] strong-scaling block (2^31 keys in total)")
    ap.add_argument("--strong", action="store_true",
                    help="N > 1 with ranks sharing GPUs (the IPC rehearsal): run the "
                         "strong-scaling block anyway (off by default there: it prices nothing)")
    ap.add_argument("--no-stats", action="store_true",
                    help="experiment: time the steps without per-phase events")
    ap.add_argument("--local", choices=["msd", "lsd"], default="msd",
                    help="local sort algorithm (DESIGN.md 5)")
    ap.add_argument("--spawn", action="store_true",
                    help="launch the rank processes from this one even at --gpus 1 "
                         "(without WORLD_SIZE in the environment, --gpus N > 1 always does)")
    return ap.parse_args()


# ---------------------------------------------------------------------------------------
# Self-launch: `python bench.py --gpus N` without a launcher starts N rank processes itself
# (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment), before this
# process touches the GPU, and forwards rank 0's JSON line.  Under torch.distributed.run the
# environment is already set and this is skipped.
# ---------------------------------------------------------------------------------------
def spawn_ranks(a):
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr))
    line = procs[0].stdout.read().decode()
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    sys.stdout.write(line)
    sys.stdout.flush()
    return rc


# ---------------------------------------------------------------------------------------
# CPU baseline: the reference itself, on the host cores, before any GPU work
# ---------------------------------------------------------------------------------------
def host_cpu():
    """The box's CPU: model name and the logical CPUs this process may use."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return {"cpu_model": model, "host_logical_cpus": os.cpu_count(), "usable_cpus": usable}


def run_reference(prog, np_, path, mpirun, bind=True, timeout=300):
    """One reference program under mpirun; (program-timer seconds, wall seconds, stdout)."""
    ref = os.path.join(ROOT, "oracle", "_ref", prog)
    t0 = time.time()
    cmd = [mpirun] + (["-bind-to", "core"] if bind else []) + ["-np", str(np_), ref, path]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    wall = time.time() - t0
    m = re.search(r"Endtime\(\)-Starttime\(\) = ([0-9.]+) sec", r.stderr)
    if r.returncode != 0 or not m:
        raise RuntimeError(f"{prog} rc={r.returncode}: {r.stderr[-300:]}")
    return float(m.group(1)), wall, r.stdout.strip().splitlines()[-1]


def median3(prog, np_, path, mpirun, bind):
    """Median of 3 runs (program timer), with every run's figures."""
    runs = [run_reference(prog, np_, path, mpirun, bind) for _ in range(3)]
    ts = sorted(r[0] for r in runs)
    meds = {r[2] for r in runs}
    if len(meds) != 1:
        raise RuntimeError(f"{prog} median lines differ between runs: {meds}")
    return ts[1], [round(r[0], 4) for r in runs], round(sum(r[1] for r in runs) / 3, 2), meds.pop()


def cpu_baseline(dist, seed, large=True):
    """The reference itself (oracle/_ref: radix_sort and sample_sort built unchanged from their
    sources with their own flags, -O0) under `mpirun -bind-to core -np P`, P = 4 (BASELINE
    configs[0]) and 8, on 2^24 keys of the same stream, median of 3, timed by the programs' own
    stderr timers (mpi_radix_sort.c:98,197,203; mpi_sample_sort.c:61,201,207), which exclude
    the text read; then the largest feasible point, 2^28 keys, radix at P = 8, one run (the
    reference's int N stops at 2^31 - 1, mpi_radix_sort.c:65).  `value` is the P = 4 radix
    figure; `cores` the ranks it ran on (one core each)."""
    keys_log2, np_ = 24, 4  # BASELINE configs[0]: reference radix, mpirun -np 4, 2^24 keys
    n = 1 << keys_log2
    gen = os.path.join(PKG, "bin", "gen_keys")
    mpirun = shutil.which("mpirun") or "/opt/conda/bin/mpirun"
    tmp = tempfile.mkdtemp(prefix="gsort_cpu_")
    host = host_cpu()
    t_start = time.time()
    try:
        path = os.path.join(tmp, "keys.txt")
        subprocess.run([gen, dist, str(n), str(seed), path], check=True)
        if os.path.exists(os.path.join(ROOT, "oracle", "_ref", "radix_sort")) and \
                os.path.exists(mpirun):
            bind = True
            try:
                run_reference("radix_sort", 2, path, mpirun, True)
            except Exception:  # binding refused on this host: run unbound, and say so
                bind = False
            points = {}
            for prog in ("radix_sort", "sample_sort"):
                for p in (4, 8):
                    try:
                        t, runs, wall, med = median3(prog, p, path, mpirun, bind)
                        points[f"{prog}_np{p}"] = {"value": n / t / 1e9, "program_s": t,
                                                    "runs_s": runs, "wall_s_avg": wall,
                                                    "median_line": med}
                    except Exception as e:  # reported, never fatal
                        points[f"{prog}_np{p}"] = {"value": None, "error": repr(e)}
            r4 = points["radix_sort_np4"]
            if r4.get("value") is None:
                raise RuntimeError(r4.get("error"))
            out = {"value": r4["value"], "unit": "GKeys/s", "cores": np_, "kind": "reference",
                   "sample": f"reference radix_sort (oracle/_ref, -O0 as shipped) under mpirun "
                             f"{'-bind-to core ' if bind else '(unbound) '}-np {np_}, 2^{keys_log2} "
                             f"{dist} keys seed {seed}; median of 3 program timers "
                             f"{r4['runs_s']} s (exclude the text read)",
                   "median_line": r4["median_line"], "bind_to_core": bind,
                   "points_2p24": points, **host}
            if large and time.time() - t_start < 120:
                nl = 1 << 28
                try:
                    lpath = os.path.join(tmp, "keys28.txt")
                    os.remove(path)
                    subprocess.run([gen, dist, str(nl), str(seed), lpath], check=True)
                    t, wall, med = run_reference("radix_sort", 8, lpath, mpirun, bind, 600)
                    out["large_point"] = {"value": nl / t / 1e9, "keys": nl, "np": 8,
                                          "program_s": t, "wall_s": round(wall, 1),
                                          "median_line": med, "runs": 1}
                except Exception as e:
                    out["large_point"] = {"value": None, "error": repr(e)}
                finally:
                    shutil.rmtree(tmp, ignore_errors=True)
            else:
                out["large_point"] = {"value": None,
                                      "skipped": "--no-cpu-large" if not large else
                                      "2^24 points took > 120 s"}
            out["beyond_reference"] = ("N >= 2^31: n/a, the reference's int N overflows "
                                       "(mpi_radix_sort.c:65)")
            out["wall_s_total"] = round(time.time() - t_start, 1)
            return out
        # fallback: the oracle's scalar port of the build's algorithm, one core
        from oracle import orc
        keys = orc.read_ints(path, cap=n)
        t0 = time.perf_counter()
        orc.lsd8(keys)
        t = time.perf_counter() - t0
        return {"value": n / t / 1e9, "unit": "GKeys/s", "cores": 1, "kind": "port",
                "sample": f"oracle lsd8 (scalar C port), 2^{keys_log2} {dist} keys, {t:.3f} s",
                **host}
    except Exception as e:  # the baseline is reported, never fatal
        return {"value": None, "unit": "GKeys/s", "cores": None, "kind": None,
                "sample": f"cpu baseline failed: {e!r}"}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def median_check(ctx, fn, dist_id, seed, cpu):
    """The GPU's sort of the CPU baseline's 2^24-key stream (same generator, seed, order)
    against the reference's own output on it: its median line (measured beside us in
    cpu_baseline) and, when tests/golden/ref_large.json holds this stream, the sha256 of the
    reference's full sorted dump."""
    import hashlib
    import numpy as np
    n = 1 << 24
    d = ctx.alloc(n * 4)
    try:
        ctx.generate(dist_id, seed, 0, n, d)
        out, m, _ = fn(d, n, stats=False)
        plan = ctx.last_plan()
        h = ctx.to_host(out, m)
    finally:
        ctx.free(d)
    res = {"keys": n, "gpu_median_line": f"The n/2-th sorted element: {h[n // 2 - 1]}",
           "local_plan": plan}
    ref_med = (cpu or {}).get("median_line")
    res["reference_median_line"] = ref_med
    res["median_matches_reference"] = (None if ref_med is None
                                       else ref_med == res["gpu_median_line"])
    try:
        cases = json.load(open(os.path.join(ROOT, "tests", "golden", "ref_large.json")))["cases"]
        gen = "uniform" if dist_id == 0 else "zipf"
        want = [c["output_sha256"] for c in cases if c["input"] == {"gen": gen, "n": n,
                                                                     "seed": seed}
                and c.get("output_is_sorted_input")]
        if want:
            got = hashlib.sha256(np.ascontiguousarray(h, dtype="<i4").tobytes()).hexdigest()
            res["dump_sha256_matches_reference"] = got == want[0]
    except (OSError, ValueError, KeyError):
        pass
    return res


def dist_p1(gsort, n_local, dist_id, seed, steps=5, algo="radix", settle_ms=100.0):
    """The distributed path at N = 1 (one-rank RCCL communicator, GSORT_FORCE_DIST) -- the
    per-GPU cost the multi-GPU points pay before any xGMI time:
      radix:  sender grouping, radix select, packed self-exchange through RCCL, receive sort;
      sample: the same sender grouping (no local sort, round 6), regular samples and bucket
              bounds read off the grouped block, device splitter selection + broadcast, the
              same packed exchange and receive sort (mpi_sample_sort.c:85, 89-128, 148-174)."""
    os.environ["GSORT_FORCE_DIST"] = "1"
    try:
        ctx = gsort.Context(rank=0, nranks=1, device=0, uid=gsort.get_uid())
    finally:
        del os.environ["GSORT_FORCE_DIST"]
    fn = ctx.radix if algo == "radix" else ctx.sample
    try:
        d = ctx.alloc(n_local * 4)
        ctx.generate(dist_id, seed, 0, n_local, d)
        ctx.reserve(n_local)
        # settled like the headline (the communicator's setup idles the GPU: without this the
        # first timed steps ran 1.70-1.79 ms against 1.55-1.60 once the clocks were up)
        t_s = time.perf_counter()
        while (time.perf_counter() - t_s) * 1e3 < settle_ms:
            ctx.copy_ceiling(n_local * 4, 10)
        for _ in range(2):
            fn(d, n_local, stats=False)
        t0 = time.perf_counter()
        for _ in range(steps):
            fn(d, n_local, stats=False)
        ms = (time.perf_counter() - t0) * 1e3 / steps
        st = [fn(d, n_local)[2] for _ in range(3)]
        out, m, _ = fn(d, n_local, stats=False)
        fp, fin = ctx.fingerprint(out, m), ctx.fingerprint(d, n_local)
        ok = fp["sorted"] and fp["sum"] == fin["sum"] and fp["xor"] == fin["xor"] and m == n_local
        ctx.free(d)
    finally:
        ctx.close()
    avg = {k: round(sum(s[k] for s in st) / len(st), 4)
           for k in ("ms_total", "ms_hist", "ms_local_sort", "ms_sample", "ms_exchange",
                     "ms_place", "ms_merge", "ms_bucket_sort")}
    avg["ms_level"] = [round(sum(s["ms_level"][i] for s in st) / len(st), 4) for i in range(2)]
    merge = avg["ms_merge"]
    # both receive sides read the 2-B packed key (the sample sort's int32 exchange is only its
    # fallback for the LSD local algorithm and ranks past 2^32 keys) and write the 4-B key
    bpk = 6
    return {"algo": algo, "ms_per_step": round(ms, 4),
            "GKeys_s": round(n_local / (ms * 1e-3) / 1e9, 2),
            "phases_ms_avg": avg, "verified": bool(ok),
            "receive_sort": {"ms": merge, "bytes_per_key": bpk,
                             "achieved_GBps": (round(n_local * bpk / (merge * 1e-3) / 1e9, 1)
                                               if merge else None),
                             "frac": (round(n_local * bpk / (merge * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
                                      if merge else None),
                             "note": ("K11g (<= 9216-key buckets) + K18c (larger): read the "
                                      "received 2-B packed key, write the 4-B key")},
            "note": "GSORT_FORCE_DIST=1, one-rank RCCL communicator (self-exchange = HBM copy); "
                    "settled as the headline, untimed steps, then 3 timed for phases"}


def kernel_rooflines(stats, n_local, plan=0):
    """Per kernel class: total device time over the timed steps (HIP events recorded on
    libgsort's stream around every launch), launches, algorithmic bytes:
    K3 / K3u read + write every key of the launch (8 B/key), K11 reads and writes every key of
    its buckets once (8 B/key); in the sampled plan K3a writes and K11e reads only the low 16
    bits of every key (6 B/key each)."""
    out = []

    def add(kernel, prefixes, ms_list, keys_list, bpk):
        launches = sum(1 for m in ms_list if m > 0)
        tot_ms = sum(ms_list)
        if not launches or tot_ms <= 0:
            return
        tot_bytes = sum(k * bpk for m, k in zip(ms_list, keys_list) if m > 0)
        out.append({"kernel": kernel, "pmc_prefixes": prefixes, "total_ms": tot_ms,
                    "launches": launches, "avg_launch_ms": round(tot_ms / launches, 5),
                    "bytes_per_key": bpk,
                    "bytes_per_launch": round(tot_bytes / launches),
                    "achieved": round(tot_bytes / (tot_ms * 1e-3) / 1e9, 1)})

    add("k_scatter (K3: rank + stable scatter of one LSD pass)", ("k_scatter",),
        [x for s in stats for x in s["ms_pass"]],
        [n_local for s in stats for x in s["ms_pass"]], PASS_BYTES_PER_KEY)
    # MSD levels: ms_level[0] = level 3 (K3u k_partition); with the two-level plan (default,
    # GSORT_PLAN16 != 0) ms_level[0] = level 3 (K3r) and ms_level[1] = level 2 (K3a), runs reserved by atomics;
    # every other level is a segmented K3u (k_seg_partition)
    # The sampled plan (plan 1): K1e reads 1/64 of the keys (0.0625 B/key; the
    # phase also holds K12e-a/b), then K3r / K3a (EST) and K11e (k_local_sort_e) as below.
    plan16 = os.environ.get("GSORT_PLAN16", "1") != "0"
    seg_from = 2 if plan16 else 1
    if plan == 1:
        add("k_est_sample (K1e: 1/64 sample histogram; with K12e-a + K12e-b)",
            ("k_est_sample",), [s["ms_hist"] for s in stats], [n_local for s in stats], 0.0625)
    if plan16:  # K1h reads every key once (4 B/key); the phase also holds K12a/b/p (~27 us)
        if plan != 1:
            add("k_hist16 (K1h: 16-bit histogram; with K12a + K12b + K12p)",
                ("k_hist16",), [s["ms_hist"] if s["ms_level"][1] > 0 else 0.0 for s in stats],
                [n_local for s in stats], 4)
        add("k_partition_res L3 (K3r: level 3, runs reserved on per-XCD-shard cursors)",
            ("k_partition_res<1024, 8, true",), [s["ms_level"][0] for s in stats],
            [s["keys_level"][0] for s in stats], PASS_BYTES_PER_KEY)
        # the sampled plan's K3a stores only the low 16 bits of every key (its Y regions are
        # u16) and K11e reads those back: 4 + 2 and 2 + 4 B/key
        add("k_partition_res L2 (K3a: level 2, runs reserved on the child cursors; the span "
            "also holds K12f's tile descriptors)",
            ("k_partition_res<1024, 8, false",), [s["ms_level"][1] for s in stats],
            [s["keys_level"][1] for s in stats], 6 if plan == 1 else PASS_BYTES_PER_KEY)
    else:
        add("k_partition (K3u: level 3, unstable MSD partition of the whole block)",
            ("k_partition<",), [s["ms_level"][0] for s in stats],
            [s["keys_level"][0] for s in stats], PASS_BYTES_PER_KEY)
    add("k_seg_partition (K3u: segmented MSD level)", ("k_seg_partition",),
        [x for s in stats for x in s["ms_level"][seg_from:]],
        [k for s in stats for k in s["keys_level"][seg_from:]], PASS_BYTES_PER_KEY)
    if plan == 1:
        add("k_local_sort_e (K11e: in-LDS sort of every level-2 child into its exact place; "
            "span from K12g's end: K11e + one launch gap)", ("k_local_sort_e",),
            [s["ms_bucket_sort"] for s in stats], [s["keys_bucket_sort"] for s in stats], 6)
    else:
        add("k_local_sort (K11: in-LDS sort of the small buckets)", ("k_local_sort",),
            [s["ms_bucket_sort"] for s in stats], [s["keys_bucket_sort"] for s in stats],
            PASS_BYTES_PER_KEY)
    return out


def pmc_traffic(algo, n_local, n_gpus, prefixes=("k_scatter",)):
    """HBM bytes per launch of the dominant kernel (FETCH_SIZE x 2 + WRITE_SIZE,
    MI355X_MICROARCH.md §HBM) from the
    newest committed rocprofv3 PMC summary of this exact configuration
    (tools/profile_pmc.sh -> profiles/*_pmc_summary.json), else None."""
    import glob
    import re

    def version(path):  # newest round, then newest version (r02_v11 after r02_v8a)
        m = re.match(r"r(\d+)_v(\d+)", os.path.basename(path))
        return (int(m.group(1)), int(m.group(2))) if m else (0, 0)

    paths = [p for p in glob.glob(os.path.join(ROOT, "profiles", "*_pmc_summary.json"))
             if "fd_" not in os.path.basename(p)]  # forced-distributed runs price other kernels
    for path in sorted(paths, key=version, reverse=True):
        try:
            d = json.load(open(path))
            cfg = d["bench"]["config"]
            if cfg["algo"] != algo or cfg["keys_per_gpu"] != n_local or n_gpus != 1:
                continue
            # the instantiation holding most of the time (K11e's size classes are separate
            # kernels: the smaller classes come from the bench's other legs, e.g. the 2^24
            # reference check, and must not be averaged into the 2^28 launch)
            k3 = [v for k, v in d["kernels"].items()
                  if k.startswith(tuple(prefixes)) and "hbm_bytes" in v]
            if k3:
                top = max(k3, key=lambda v: v.get("avg_us", 0.0) * v.get("calls", 1))
                return {"hbm_bytes_per_launch": round(top["hbm_bytes"]),
                        "source": os.path.relpath(path, ROOT)}
        except (OSError, ValueError, KeyError):
            continue
    return None


def copy_ceiling(ctx, n_local, reps=10):
    """The practical HBM ceiling of one read + write pass: libgsort's 16-B-per-lane streaming
    copy kernel (gsort_copy_ceiling) over the same 4 * n_local bytes, HIP events on its stream,
    median of `reps` (MI355X_MICROARCH.md: 6.29 TB/s float4 copy; the variants measured are
    in tools/experiments/copy_ceiling.hip)."""
    ms, gbps = ctx.copy_ceiling(n_local * 4, reps)
    return {"ms": round(ms, 4), "GBps": round(gbps, 1),
            "how": "gsort_copy_ceiling: k_stream_copy (16-KiB chunk per block, 16 B per lane, "
                   f"nontemporal stores) of the same {n_local * 4} bytes, median of {reps}"}


def drop_in_e2e(ctx, fn, d_in, n, reps=3):
    """The reference's timer span at N = 1: pageable rank-0 host int32 array -> GPU
    (gsort_scatter_from_root) -> gsort_radix -> rank-0 host array (gsort_gather_to_root)."""
    import numpy as np
    h = ctx.to_host(d_in, n)
    ts, out = [], None
    for _ in range(reps):
        t0 = time.perf_counter()
        d, m = ctx.scatter_from_root(h, n)
        d_out, n_out, _ = fn(d, m)
        out = ctx.gather_to_root(d_out, n_out, n)
        ts.append(time.perf_counter() - t0)
    ok = bool(out.size == n and np.all(out[1:] >= out[:-1]))
    ts.sort()
    ms = ts[len(ts) // 2] * 1e3
    return {"ms": round(ms, 2), "GKeys_s": round(n / (ms * 1e-3) / 1e9, 3), "sorted": ok,
            "note": "pageable host array -> GPU -> sorted -> host (PCIe included), "
                    "median of 3; not the headline value"}


def s64(x):
    """u64 -> the int64 with the same bits (all-gathered fingerprint rows)."""
    return x - (1 << 64) if x >= 1 << 63 else x


def exchange_line(stats):
    """The exchange's xGMI roofline from the timed steps' gsort_stats: per exchange, the
    largest (source, destination) pair's bytes over one xGMI link's peak."""
    last = stats[-1]
    if not last["exchanges"]:
        return None
    ex = sum(s["ms_exchange"] for s in stats) / len(stats) / max(last["exchanges"], 1)
    pair = last["max_pair_bytes"]
    return {"bound": "xgmi", "per_exchange_ms": round(ex, 4), "max_pair_bytes": pair,
            "achieved_link_GBps": round(pair / (ex * 1e-3) / 1e9, 2) if ex else None,
            "peak_link_GBps": XGMI_LINK_GBPS,
            "frac": round(pair / (ex * 1e-3) / 1e9 / XGMI_LINK_GBPS, 4) if ex else None}


def strong_line(n_total, world, ms_step, verified, stats):
    """BASELINE configs[2] ("Radix sort 2^31 uniform 32-bit keys across 2/4/8 MI355X"): the
    same 2^31 keys at every N (strong scaling), beside the weak-scaling headline."""
    return {"config": "BASELINE configs[2]: radix sort, 2^31 uniform int32 keys in total "
                      f"across {world} GPUs ({n_total // world} per GPU)",
            "total_keys": n_total, "keys_per_gpu": n_total // world, "n_gpus": world,
            "scaling": "strong", "ms_per_step": round(ms_step, 4),
            "GKeys_s": round(n_total / (ms_step * 1e-3) / 1e9, 3), "steps": len(stats),
            "verified": bool(verified), "exchange": exchange_line(stats) if stats else None}


def verify_rows(rows, n_local, algo):
    """N > 1 output check from every rank's row [sum_in, sum_out, xor_in, xor_out, sorted, n_out,
    first, last] (64-bit figures as int64 bit patterns): the multiset of all outputs (sum and
    xor of mix64(key)) equals that of all inputs, every output is sorted, rank q's last key <=
    rank q+1's first (a misrouted exchange that keeps the multiset fails here), and the sizes
    add up (radix: rank q holds exactly its n_local global positions)."""
    m64 = (1 << 64) - 1
    sum_in = sum(r[0] for r in rows) & m64
    sum_out = sum(r[1] for r in rows) & m64
    x_in = x_out = 0
    for r in rows:
        x_in ^= r[2] & m64
        x_out ^= r[3] & m64
    full = [r for r in rows if r[5]]
    return bool(all(r[4] for r in rows) and sum_in == sum_out and x_in == x_out
                and sum(r[5] for r in rows) == n_local * len(rows)
                and all(x[7] <= y[6] for x, y in zip(full, full[1:]))
                and (algo != "radix" or all(r[5] == n_local for r in rows)))


def main():
    # stdout carries the one JSON line only: native libraries (RCCL prints a version banner
    # at communicator init) write to fd 1, so point it at stderr and keep the real stdout
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    a = parse()
    if "WORLD_SIZE" not in os.environ and (a.gpus > 1 or a.spawn):
        os.dup2(json_fd, 1)
        sys.exit(spawn_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        sys.exit(f"bench: --gpus {a.gpus} but WORLD_SIZE={world}")
    dist_name = a.dist

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(dist_name, a.seed, large=not a.no_cpu_large)

    import torch
    import torch.distributed as dist
    import gsort

    # More ranks than GPUs (a one-GPU box rehearsing the N > 1 path): the ranks share the GPUs
    # through the library's IPC transport (RCCL refuses two ranks on one device).  Such a run
    # checks the multi-process flow end to end -- exchange, verify_rows, the strong-scaling
    # block -- but its numbers price nothing (`transport` in the line says so).
    ndev = torch.cuda.device_count()  # (counting devices does not initialise the GPU)
    shared = world > max(ndev, 1)
    dev = local % max(ndev, 1)
    torch.cuda.set_device(dev)
    if world > 1:
        dist.init_process_group("gloo")  # bootstrap only: uid broadcast, barrier, max-time
    # GSORT_TRANSPORT=rccl|ipc overrides the choice (as in the drop-in CLIs)
    forced = os.environ.get("GSORT_TRANSPORT")
    use_ipc = (shared and forced != "rccl") or forced == "ipc"
    if world > 1:
        # preflight: every rank forms the same kind of group -- if any rank's view
        # (device count, GSORT_TRANSPORT) picks the IPC group, all of them do
        flag = torch.tensor([int(use_ipc), int(shared)], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
        use_ipc, shared = bool(flag[0].item()), bool(flag[1].item())

    def make_ctx(ipc):
        uid = None
        # GSORT_FORCE_DIST=1 (test hook, tests/test_gpu_rccl.py): one rank still runs the
        # distributed algorithm over a one-rank RCCL communicator
        if world > 1 or os.environ.get("GSORT_FORCE_DIST") == "1":
            buf = torch.zeros(128, dtype=torch.uint8)
            if rank == 0:
                u = gsort.get_uid(ipc_ranks=world) if ipc else gsort.get_uid()
                buf = torch.tensor(list(u), dtype=torch.uint8)
            if world > 1:
                dist.broadcast(buf, 0)
            uid = bytes(buf.tolist())
        return gsort.Context(rank=rank, nranks=world, device=dev, uid=uid)

    # An RCCL communicator that fails to form (on any rank: the ranks agree over gloo) is not
    # the end of the run: the ranks re-form over the IPC group and the line says so in
    # `transport` (a hang inside RCCL's setup is not caught here)
    fallback = None
    try:
        ctx, err = make_ctx(use_ipc), None
    except gsort.GsortError as e:
        ctx, err = None, e
    if world > 1:
        bad = torch.tensor([0 if ctx is not None else 1], dtype=torch.int32)
        dist.all_reduce(bad, op=dist.ReduceOp.MAX)
        if bad.item() and use_ipc:  # no second transport to try: every rank ends, non-zero
            if ctx is not None:
                ctx.close()
            dist.destroy_process_group()
            sys.exit(f"bench r{rank}: ipc group setup failed "
                     f"({err if err else 'on another rank'})")
        if bad.item() and not use_ipc:
            if ctx is not None:
                ctx.close()
            fallback = f"rccl communicator setup failed ({err if err else 'on another rank'})"
            print(f"[bench r{rank}] {fallback}; re-forming over the IPC group", file=sys.stderr,
                  flush=True)
            use_ipc = True
            ctx, err = make_ctx(True), None
    if ctx is None:
        raise err

    def barrier():
        if world > 1:
            dist.barrier()

    n_local = 1 << a.keys_log2
    d_in = ctx.alloc(n_local * 4)
    ctx.generate(gsort.UNIFORM if dist_name == "uniform" else gsort.ZIPF, a.seed,
                 rank * n_local, n_local, d_in)
    ctx.reserve(n_local)
    ctx.set_local_algo(gsort.LOCAL_MSD if a.local == "msd" else gsort.LOCAL_LSD)
    fn = ctx.radix if a.algo == "radix" else ctx.sample
    t_start = time.perf_counter()

    def log(msg):  # progress on stderr (the JSON line goes to stdout)
        print(f"[bench r{rank} +{time.perf_counter() - t_start:.1f}s] {msg}", file=sys.stderr,
              flush=True)

    log(f"context ready: {n_local} keys, transport {'ipc' if use_ipc else 'rccl' if world > 1 else 'none'}")
    settle = {"ms": 0.0, "copies": 0}
    if a.settle_ms > 0:  # (module docstring: from idle to the sustained clocks)
        t_s = time.perf_counter()
        while (time.perf_counter() - t_s) * 1e3 < a.settle_ms:
            ctx.copy_ceiling(n_local * 4, 10)
            settle["copies"] += 10
        settle["ms"] = round((time.perf_counter() - t_s) * 1e3, 1)
    settle["how"] = ("gsort_copy_ceiling's streaming copy of the 4 * n_local-byte buffer, "
                     "before the warm-up steps (untimed)")
    log("settled")
    for _ in range(a.warmup):
        fn(d_in, n_local)
    log("warm-up steps done")
    barrier()
    torch.cuda.synchronize()
    # one gsort_stats per step, filled in place and converted after the timed region
    raw = [gsort.Stats() if not a.no_stats else False for _ in range(a.steps)]
    t0 = time.perf_counter()
    for i in range(a.steps):
        fn(d_in, n_local, raw[i])
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    plan = ctx.last_plan()
    if a.no_stats:  # experiment: the un-instrumented step time; stats from extra steps
        stats = [fn(d_in, n_local)[2] for _ in range(a.steps)]
    else:
        stats = [r.as_dict() for r in raw]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    log("timed steps done")
    # correctness of the last step's output, checked on device (K9)
    out_ptr, n_out, _ = fn(d_in, n_local)
    fp = ctx.fingerprint(out_ptr, n_out)
    fin = ctx.fingerprint(d_in, n_local)
    ok = fp["sorted"]
    if world > 1:
        # every rank's figures to every rank: the multiset (sum and xor of mix64(key), 64-bit)
        # of all outputs == of all inputs, every output sorted, rank q's last key <= rank
        # q+1's first (a misrouted exchange that keeps the multiset fails here), and the sizes
        # (radix: rank q holds exactly its n_local global positions)
        mine = torch.tensor([s64(fin["sum"]), s64(fp["sum"]), s64(fin["xor"]), s64(fp["xor"]),
                             int(fp["sorted"]), n_out, fp["first"], fp["last"]], dtype=torch.int64)
        rows = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(rows, mine)
        ok = verify_rows([[int(x) for x in r.tolist()] for r in rows], n_local, a.algo)
    else:
        ok = ok and fp["sum"] == fin["sum"] and fp["xor"] == fin["xor"] and n_out == n_local

    n_total = n_local * world
    ms_step = elapsed * 1e3 / a.steps
    value = n_total / (ms_step / 1e3) / 1e9

    ceiling = copy_ceiling(ctx, n_local) if rank == 0 else None
    drop_in = drop_in_e2e(ctx, fn, d_in, n_local) if world == 1 else None
    dist_id = gsort.UNIFORM if dist_name == "uniform" else gsort.ZIPF
    med = median_check(ctx, fn, dist_id, a.seed, cpu) if world == 1 else None

    rooflines = kernel_rooflines(stats, n_local, plan)
    dom = max(rooflines, key=lambda r: r["total_ms"])
    pmc = pmc_traffic(a.algo, n_local, world, dom["pmc_prefixes"])
    traffic = pmc["hbm_bytes_per_launch"] if pmc else None
    last = stats[-1]
    phases = {k: round(sum(s[k] for s in stats) / len(stats), 4)
              for k in ("ms_total", "ms_hist", "ms_local_sort", "ms_exchange", "ms_place",
                        "ms_sample", "ms_merge")}
    phases["ms_pass"] = [round(sum(s["ms_pass"][i] for s in stats) / len(stats), 4)
                         for i in range(4)]
    phases["ms_level"] = [round(sum(s["ms_level"][i] for s in stats) / len(stats), 4)
                          for i in range(4)]
    phases["ms_bucket_sort"] = round(sum(s["ms_bucket_sort"] for s in stats) / len(stats), 4)
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GKeys/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "settle": settle,
        "transport": (None if world == 1 else
                      f"ipc, after {fallback}" + ("; ranks share GPUs (prices nothing)"
                                                  if shared else "")
                      if fallback else
                      "ipc: ranks share GPUs (a rehearsal of the N > 1 path; prices nothing)"
                      if use_ipc and shared else
                      "ipc over xGMI (GSORT_TRANSPORT=ipc)" if use_ipc else "rccl over xGMI"),
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": f"synthetic: splitmix64 {dist_name} keys (seed {a.seed}) generated on device",
        "config": {
            "workload": (f"{a.algo} sort, 2^{a.keys_log2} {dist_name} int32 keys per GPU "
                         f"(BASELINE configs[1] at N=1; 2^{a.keys_log2}*N keys sorted "
                         f"globally at N GPUs)"),
            "keys_per_gpu": n_local, "total_keys": n_total, "algo": a.algo,
            "parallelism": f"dp{world}", "onesweep_tile": gsort.onesweep_tile(),
        },
        "roofline": {"bound": "hbm", "kernel": dom["kernel"],
                     "achieved": dom["achieved"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(dom["achieved"] / HBM_PEAK_GBPS, 4),
                     "traffic": traffic,
                     "traffic_source": pmc["source"] if pmc else None,
                     "algorithmic_bytes_per_launch": dom["bytes_per_launch"],
                     "bytes_per_key": dom["bytes_per_key"],
                     "avg_launch_ms": dom["avg_launch_ms"],
                     "launches_timed": dom["launches"],
                     "copy_ceiling_GBps": ceiling["GBps"] if ceiling else None,
                     "frac_of_copy": (round(dom["achieved"] / ceiling["GBps"], 4)
                                      if ceiling else None)},
        "kernels": [{k: v for k, v in r.items() if k != "pmc_prefixes"} for r in rooflines],
        "cpu_baseline": cpu,
        "copy_ceiling": ceiling,
        "drop_in": drop_in,
        "phases_ms_avg": phases,
        "passes_run": last["passes_run"],
        "local_algo": "lsd" if last["local_algo"] == gsort.LOCAL_LSD else "msd",
        "local_plan": ("lsd passes" if a.local == "lsd" else
                       {0: "exact two-level", 1: "sampled", 2: "sampled, re-sorted exact",
                        3: "sampled below a constant key prefix",
                        4: "one dominant 16-bit child counted"}.get(
                           plan, str(plan))),
        "verified": bool(ok),
        "reference_check_2p24": med,
        # the HIP runtime / RCCL libgsort is bound to here (torch's bundled ones: torch is
        # imported first; the drop-in CLIs run on /opt/rocm's -- DESIGN.md 6)
        "runtime": gsort.runtime_info(),
    }
    if last["exchanges"]:
        line["exchange"] = exchange_line(stats)
    ctx.free(d_in)
    # (ranks sharing one GPU -- the IPC rehearsal -- skip it unless --strong: 2^31 keys plus
    # scratch on one GPU and 2 GiB of staging per rank, for a number that prices nothing)
    if world > 1 and a.algo == "radix" and not a.no_strong and (a.strong or not shared):
        # configs[2]'s strong-scaling point: 2^31 keys in total (the canonical stream, rank r's
        # block = its slice), a few timed steps bracketed like the headline's, max over ranks
        n_s = (1 << 31) // world
        log(f"strong-scaling block: {n_s} keys per rank")
        d_s = ctx.alloc(n_s * 4)
        ctx.generate(gsort.UNIFORM, a.seed, rank * n_s, n_s, d_s)
        ctx.reserve(n_s)
        fn(d_s, n_s)
        barrier()
        torch.cuda.synchronize()
        raw_s = [gsort.Stats() for _ in range(3)]
        t0 = time.perf_counter()
        for r_ in raw_s:
            fn(d_s, n_s, r_)
        torch.cuda.synchronize()
        barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        out_s, m_s, _ = fn(d_s, n_s)
        fo, fi = ctx.fingerprint(out_s, m_s), ctx.fingerprint(d_s, n_s)
        mine = torch.tensor([s64(fi["sum"]), s64(fo["sum"]), s64(fi["xor"]), s64(fo["xor"]),
                             int(fo["sorted"]), m_s, fo["first"], fo["last"]], dtype=torch.int64)
        rows = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(rows, mine)
        ok_s = verify_rows([[int(x) for x in r.tolist()] for r in rows], n_s, "radix")
        line["strong_scaling_cfg2"] = strong_line(n_s * world, world,
                                                  float(el.item()) * 1e3 / len(raw_s), ok_s,
                                                  [r_.as_dict() for r_ in raw_s])
        ctx.free(d_s)
        ok = ok and ok_s
        log("strong-scaling block done")
    ctx.close()
    if world == 1 and a.algo == "radix" and not a.no_dist_p1 and \
            os.environ.get("GSORT_FORCE_DIST") != "1":
        for key, algo in (("dist_p1", "radix"), ("dist_p1_sample", "sample")):
            try:
                line[key] = dist_p1(gsort, n_local, dist_id, a.seed, algo=algo,
                                    settle_ms=a.settle_ms)
            except Exception as e:  # reported, never fatal
                line[key] = {"error": repr(e)}
    if rank == 0:
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit("bench: output failed verification")


if __name__ == "__main__":
    main()
