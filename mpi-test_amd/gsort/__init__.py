"""Python binding of libgsort (include/gsort.h) over ctypes.

Host-side mirror of the reference's sort entry point for Python callers (tests, bench.py):
`Context.radix` / `Context.sample` are the device-resident hot paths that replace the pass
loops of sort() in mpi_radix_sort.c:60-205 / mpi_sample_sort.c:28-218; `run_sort` mirrors the
reference's `sort(rank, size, file, debug)` end to end (read on rank 0, scatter, sort, gather,
print).  Everything runs in libgsort.so's HIP kernels; there is no CPU fallback: if the library
is missing or no GPU is visible, calls raise.

Import torch BEFORE this module in processes that also use torch, so libgsort binds to the
same HIP runtime torch loaded (both resolve libamdhip64.so.7 by soname).
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
# GSORT_LIB (development, same-box A/B of two builds: tools/ab_lib.sh) loads another build
LIB_PATH = os.environ.get("GSORT_LIB") or os.path.join(PKG, "lib", "libgsort.so")

OK, EINVAL, ENOMEM, EHIP, ERCCL, ENOSAMPLE, ECOMM = range(7)
UNIFORM, ZIPF = 0, 1
LOCAL_MSD, LOCAL_LSD = 0, 1


class GsortError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"gsort status {status}: {msg}")
        self.status = status


class Stats(ctypes.Structure):
    _fields_ = [("ms_total", ctypes.c_double), ("ms_hist", ctypes.c_double),
                ("ms_pass", ctypes.c_double * 4), ("ms_local_sort", ctypes.c_double),
                ("ms_exchange", ctypes.c_double), ("ms_place", ctypes.c_double),
                ("ms_sample", ctypes.c_double), ("ms_merge", ctypes.c_double),
                ("keys_local_in", ctypes.c_uint64), ("keys_local_out", ctypes.c_uint64),
                ("bytes_sent", ctypes.c_uint64), ("max_pair_bytes", ctypes.c_uint64),
                ("passes_run", ctypes.c_int), ("exchanges", ctypes.c_int),
                ("ms_level", ctypes.c_double * 4), ("ms_bucket_sort", ctypes.c_double),
                ("keys_level", ctypes.c_uint64 * 4), ("keys_bucket_sort", ctypes.c_uint64),
                ("buckets_local", ctypes.c_uint64), ("local_algo", ctypes.c_int)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["ms_pass"] = list(self.ms_pass)
        d["ms_level"] = list(self.ms_level)
        d["keys_level"] = list(self.keys_level)
        return d


class Uid(ctypes.Structure):
    # raw bytes: a c_char array field would cut the id at its first NUL on read and write
    _fields_ = [("internal", ctypes.c_ubyte * 128)]

    @classmethod
    def from_bytes(cls, b):
        b = bytes(b)
        if len(b) != 128:
            raise ValueError(f"a gsort uid is 128 bytes, got {len(b)}")
        u = cls()
        ctypes.memmove(ctypes.addressof(u), b, 128)
        return u

    def to_bytes(self):
        return ctypes.string_at(ctypes.addressof(self), 128)


EXPORTS = [
    "gsort_get_uid", "gsort_get_uid_ipc", "gsort_visible_devices", "gsort_create", "gsort_group_create", "gsort_group_destroy",
    "gsort_create_in_group", "gsort_destroy", "gsort_reserve", "gsort_set_local_algo",
    "gsort_set_sample_balanced",
    "gsort_strerror",
    "gsort_last_error", "gsort_rank", "gsort_nranks", "gsort_radix", "gsort_sample",
    "gsort_sample_info", "gsort_scatter_from_root", "gsort_gather_to_root", "gsort_generate",
    "gsort_fingerprint", "gsort_device_alloc", "gsort_device_free", "gsort_copy_to_host",
    "gsort_copy_to_device", "gsort_onesweep_tile", "gsort_plan_radix_route",
    "gsort_plan_splitters", "gsort_plan_split", "gsort_plan_split_balanced", "gsort_parse_text",
    "gsort_format_dump", "gsort_copy_ceiling", "gsort_set_ref_compat", "gsort_plan_ref_digits",
    "gsort_last_plan", "gsort_write_report", "gsort_runtime_info",
]
REPORT_RADIX, REPORT_SAMPLE = 0, 1


class RuntimeInfo(ctypes.Structure):
    """gsort_runtime_info_t: the HIP runtime and RCCL libgsort is bound to in this process."""
    _fields_ = [("hip_runtime", ctypes.c_int), ("rccl", ctypes.c_int),
                ("hip_path", ctypes.c_char * 256), ("rccl_path", ctypes.c_char * 256)]


class Report(ctypes.Structure):
    """gsort_report: what one rank of the drop-in programs prints to stdout."""
    _fields_ = [("algo", ctypes.c_int), ("rank", ctypes.c_int), ("nranks", ctypes.c_int),
                ("debug", ctypes.c_int), ("n_total", ctypes.c_uint64),
                ("splitters", ctypes.c_void_p), ("bucket_counts", ctypes.c_void_p),
                ("sorted", ctypes.c_void_p), ("stage", ctypes.c_int)]

_lib = None


def lib():
    """Load libgsort.so (built by `make -C mpi-test_amd`); raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libgsort.so not built at {LIB_PATH}: run __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH)
    P, VP, SZ, I, U64 = (ctypes.POINTER, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                         ctypes.c_uint64)
    for name in EXPORTS:
        if os.environ.get("GSORT_LIB") and not hasattr(L, name):
            continue  # (an older build loaded for a same-box A/B: what it lacks stays unused)
        getattr(L, name).restype = ctypes.c_int
    L.gsort_strerror.restype = ctypes.c_char_p
    L.gsort_last_error.restype = ctypes.c_char_p
    L.gsort_onesweep_tile.restype = SZ
    L.gsort_get_uid.argtypes = [P(Uid)]
    L.gsort_get_uid_ipc.argtypes = [I, P(Uid)]
    L.gsort_visible_devices.argtypes = []
    if hasattr(L, "gsort_runtime_info"):
        L.gsort_runtime_info.argtypes = [P(RuntimeInfo)]
    L.gsort_write_report.argtypes = [P(Report), I]
    L.gsort_create.argtypes = [P(VP), I, I, I, P(Uid)]
    L.gsort_group_create.argtypes = [P(VP), I]
    L.gsort_group_destroy.argtypes = [VP]
    L.gsort_create_in_group.argtypes = [P(VP), VP, I, I]
    L.gsort_destroy.argtypes = [VP]
    L.gsort_reserve.argtypes = [VP, SZ]
    L.gsort_set_local_algo.argtypes = [VP, I]
    L.gsort_strerror.argtypes = [I]
    L.gsort_last_error.argtypes = [VP]
    L.gsort_rank.argtypes = [VP]
    L.gsort_nranks.argtypes = [VP]
    for fn in (L.gsort_radix, L.gsort_sample):
        fn.argtypes = [VP, VP, SZ, P(VP), P(SZ), P(Stats)]
    L.gsort_sample_info.argtypes = [VP, VP, VP]
    L.gsort_last_plan.argtypes = [VP]
    L.gsort_scatter_from_root.argtypes = [VP, VP, SZ, P(VP), P(SZ)]
    L.gsort_gather_to_root.argtypes = [VP, VP, SZ, VP]
    L.gsort_generate.argtypes = [VP, I, U64, U64, SZ, VP]
    L.gsort_fingerprint.argtypes = [VP, VP, SZ, P(U64), P(U64), P(I), P(ctypes.c_int32),
                                    P(ctypes.c_int32)]
    L.gsort_device_alloc.argtypes = [VP, SZ, P(VP)]
    L.gsort_device_free.argtypes = [VP, VP]
    L.gsort_copy_to_host.argtypes = [VP, VP, VP, SZ]
    L.gsort_copy_to_device.argtypes = [VP, VP, VP, SZ]
    L.gsort_copy_ceiling.argtypes = [VP, SZ, I, P(ctypes.c_double), P(ctypes.c_double)]
    L.gsort_plan_radix_route.argtypes = [I, VP, U64, I, VP, VP, VP, P(SZ)]
    L.gsort_plan_splitters.argtypes = [I, VP, VP]
    L.gsort_plan_split.argtypes = [I, VP, VP, VP, I, VP, VP]
    L.gsort_plan_split_balanced.argtypes = [I, VP, VP, VP, I, VP, VP]
    L.gsort_set_sample_balanced.argtypes = [VP, I]
    L.gsort_set_ref_compat.argtypes = [VP, I]
    L.gsort_plan_ref_digits.argtypes = [I, ctypes.c_int32, P(I), VP, VP, I]
    L.gsort_parse_text.argtypes = [ctypes.c_char_p, SZ, VP, SZ, I]
    L.gsort_parse_text.restype = ctypes.c_longlong
    L.gsort_format_dump.argtypes = [VP, SZ, U64, VP, SZ, I]
    L.gsort_format_dump.restype = ctypes.c_longlong
    _lib = L
    return L


def runtime_info():
    """{hip_runtime, rccl (e.g. '2.27.7'), hip_path, rccl_path}: what libgsort runs on in this
    process (under torch: torch's bundled HIP runtime and RCCL, loaded first; without torch and
    in the drop-in CLIs: /opt/rocm's) -- gsort_runtime_info."""
    r = RuntimeInfo()
    _check(lib().gsort_runtime_info(ctypes.byref(r)), None)
    v = r.rccl
    return {"hip_runtime": r.hip_runtime,
            "rccl": f"{v // 10000}.{v // 100 % 100}.{v % 100}" if v > 0 else None,
            "hip_path": r.hip_path.decode(), "rccl_path": r.rccl_path.decode()}


def get_uid(ipc_ranks=None):
    """An RCCL unique id, or with ipc_ranks=P the id of a P-process IPC group (any number of
    ranks per GPU; gsort_get_uid_ipc)."""
    u = Uid()
    if ipc_ranks is None:
        _check(lib().gsort_get_uid(ctypes.byref(u)), None)
    else:
        _check(lib().gsort_get_uid_ipc(ipc_ranks, ctypes.byref(u)), None)
    return u.to_bytes()


def write_report(fd, algo, rank, nranks, debug, n_total, splitters=None, bucket_counts=None,
                 sorted_keys=None, stage=0):
    """gsort_write_report: rank `rank`'s stdout contract lines (the drop-in programs' output)
    written to the file descriptor fd."""
    import numpy as np
    keep = []

    def arr(a, dt):
        if a is None:
            return None
        a = np.ascontiguousarray(a, dtype=dt)
        keep.append(a)
        return a.ctypes.data if a.size else None

    r = Report(algo, rank, nranks, debug, n_total, arr(splitters, np.int32),
               arr(bucket_counts, np.uint64), arr(sorted_keys, np.int32), stage)
    _check(lib().gsort_write_report(ctypes.byref(r), fd), None)


def report_bytes(*args, **kw):
    """write_report into a pipe-free temporary file; returns the bytes written."""
    import tempfile
    with tempfile.TemporaryFile() as f:
        write_report(f.fileno(), *args, **kw)
        f.seek(0)
        return f.read()


def _check(st, ctx):
    if st != OK:
        L = lib()
        msg = L.gsort_strerror(st).decode()
        if ctx:
            detail = L.gsort_last_error(ctx).decode()
            if detail:
                msg += ": " + detail
        raise GsortError(st, msg)


class Group:
    """In-process rank group: `nranks` contexts, one per thread, on one process."""

    def __init__(self, nranks):
        self.h = ctypes.c_void_p()
        _check(lib().gsort_group_create(ctypes.byref(self.h), nranks), None)
        self.nranks = nranks

    def close(self):
        if self.h:
            lib().gsort_group_destroy(self.h)
            self.h = ctypes.c_void_p()


class Context:
    """One rank == one GPU.  Not thread-safe; one thread per context."""

    def __init__(self, rank=0, nranks=1, device=0, uid=None, group=None):
        self.h = ctypes.c_void_p()
        L = lib()
        if group is not None:
            _check(L.gsort_create_in_group(ctypes.byref(self.h), group.h, rank, device), None)
        else:
            u = Uid.from_bytes(uid) if uid is not None else None
            _check(L.gsort_create(ctypes.byref(self.h), rank, nranks, device,
                                  ctypes.byref(u) if u is not None else None), None)
        self.rank, self.nranks, self.device = rank, (group.nranks if group else nranks), device

    def close(self):
        if self.h:
            lib().gsort_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _c(self, st):
        _check(st, self.h)

    def reserve(self, n):
        self._c(lib().gsort_reserve(self.h, n))

    def set_local_algo(self, algo):
        """LOCAL_MSD (default) or LOCAL_LSD for every later local sort of this context."""
        self._c(lib().gsort_set_local_algo(self.h, algo))

    def set_sample_balanced(self, on=True):
        """Duplicate-aware balanced sample-sort buckets (gsort_set_sample_balanced)."""
        self._c(lib().gsort_set_sample_balanced(self.h, 1 if on else 0))

    def set_ref_compat(self, radix_p=-1):
        """Reference-compat radix order (gsort_set_ref_compat): radix_p > 0 reproduces the
        reference's output order for an `mpirun -np radix_p` run, -1 uses this context's rank
        count, 0 restores the numeric sort."""
        self._c(lib().gsort_set_ref_compat(self.h, radix_p))

    def _sort(self, fn, d_keys, n, stats=True):
        out, nout = ctypes.c_void_p(), ctypes.c_size_t()
        st = stats if isinstance(stats, Stats) else Stats() if stats else None
        self._c(fn(self.h, ctypes.c_void_p(d_keys), n, ctypes.byref(out), ctypes.byref(nout),
                   ctypes.byref(st) if st is not None else None))
        if isinstance(stats, Stats):
            return out.value or 0, nout.value, stats  # filled in place, unconverted
        return out.value or 0, nout.value, st.as_dict() if st is not None else None

    def radix(self, d_keys, n, stats=True):
        """Device-resident radix sort: returns (d_out, n_out, stats); d_out is ctx-owned.
        stats=False passes no gsort_stats (no per-phase timing); a Stats instance is filled in
        place and returned as is (a timing loop converts it afterwards)."""
        return self._sort(lib().gsort_radix, d_keys, n, stats)

    def sample(self, d_keys, n, stats=True):
        return self._sort(lib().gsort_sample, d_keys, n, stats)

    def sample_info(self):
        import numpy as np
        spl = np.zeros(max(self.nranks - 1, 1), dtype=np.int32)
        cnt = np.zeros(self.nranks, dtype=np.uint64)
        self._c(lib().gsort_sample_info(self.h, spl.ctypes.data, cnt.ctypes.data))
        return spl[: self.nranks - 1], cnt

    PLAN_EXACT, PLAN_SAMPLED, PLAN_SAMPLED_THEN_EXACT, PLAN_SAMPLED_SHIFTED, PLAN_GIANT = \
        0, 1, 2, 3, 4

    def last_plan(self):
        """Plan of the last one-rank local sort (gsort_last_plan): 0 exact, 1 sampled,
        2 sampled then re-sorted on the exact plan (ineligible block or a region overflow),
        3 sampled on the digits below a constant key prefix, 4 one dominant 16-bit child
        counted (its low 16 bits), the other keys sorted apart."""
        return lib().gsort_last_plan(self.h)

    def generate(self, dist, seed, start, n, d_out):
        self._c(lib().gsort_generate(self.h, dist, seed, start, n, ctypes.c_void_p(d_out)))

    def fingerprint(self, d_keys, n):
        s, x, ok = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        f, l = ctypes.c_int32(), ctypes.c_int32()
        self._c(lib().gsort_fingerprint(self.h, ctypes.c_void_p(d_keys), n, ctypes.byref(s),
                                        ctypes.byref(x), ctypes.byref(ok), ctypes.byref(f),
                                        ctypes.byref(l)))
        return {"sum": s.value, "xor": x.value, "sorted": bool(ok.value), "first": f.value,
                "last": l.value}

    def alloc(self, nbytes):
        p = ctypes.c_void_p()
        self._c(lib().gsort_device_alloc(self.h, nbytes, ctypes.byref(p)))
        return p.value

    def free(self, p):
        self._c(lib().gsort_device_free(self.h, ctypes.c_void_p(p)))

    def copy_ceiling(self, nbytes, reps=10):
        """gsort_copy_ceiling: (ms, GB/s) of the in-library streaming copy of nbytes."""
        ms, gbps = ctypes.c_double(), ctypes.c_double()
        self._c(lib().gsort_copy_ceiling(self.h, nbytes, reps, ctypes.byref(ms),
                                         ctypes.byref(gbps)))
        return ms.value, gbps.value

    def to_host(self, d_ptr, n):
        import numpy as np
        a = np.empty(n, dtype=np.int32)
        if n:
            self._c(lib().gsort_copy_to_host(self.h, a.ctypes.data, ctypes.c_void_p(d_ptr),
                                             n * 4))
        return a

    def to_device(self, a, d_ptr):
        import numpy as np
        a = np.ascontiguousarray(a, dtype=np.int32)
        if a.size:
            self._c(lib().gsort_copy_to_device(self.h, ctypes.c_void_p(d_ptr), a.ctypes.data,
                                               a.size * 4))

    def scatter_from_root(self, h_root, n_total):
        import numpy as np
        ptr = None
        if h_root is not None:
            h_root = np.ascontiguousarray(h_root, dtype=np.int32)
            ptr = h_root.ctypes.data
        d, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._c(lib().gsort_scatter_from_root(self.h, ptr, n_total, ctypes.byref(d),
                                              ctypes.byref(n)))
        return d.value, n.value

    def gather_to_root(self, d_out, n_out, n_total):
        import numpy as np
        h = np.empty(max(n_total, 1), dtype=np.int32) if self.rank == 0 else None
        self._c(lib().gsort_gather_to_root(self.h, ctypes.c_void_p(d_out), n_out,
                                           h.ctypes.data if h is not None else None))
        return h[:n_total] if h is not None else None


def onesweep_tile():
    return lib().gsort_onesweep_tile()


def plan_radix_route(hist, B, me):
    """Host-only K8 routing (gsort_plan_radix_route): returns (send, recv, seg rows)."""
    import numpy as np
    hist = np.ascontiguousarray(hist, dtype=np.uint64)
    P = hist.shape[0]
    send = np.zeros(P, dtype=np.uint64)
    recv = np.zeros(P, dtype=np.uint64)
    seg = np.zeros(4 * P * 256, dtype=np.uint64)
    n = ctypes.c_size_t()
    _check(lib().gsort_plan_radix_route(P, hist.ctypes.data, B, me, send.ctypes.data,
                                        recv.ctypes.data, seg.ctypes.data, ctypes.byref(n)),
           None)
    return send, recv, seg[: 4 * n.value].reshape(-1, 4)


def plan_split(n_all, lt, le, me, balanced=False):
    """Host-only exact split of the distributed radix (gsort_plan_split): (send, recv);
    balanced: the sample sort's duplicate-aware cut (gsort_plan_split_balanced)."""
    import numpy as np
    n_all = np.ascontiguousarray(n_all, dtype=np.uint64)
    P = n_all.size
    lt = np.ascontiguousarray(lt, dtype=np.uint64).reshape(P, max(P - 1, 0))
    le = np.ascontiguousarray(le, dtype=np.uint64).reshape(P, max(P - 1, 0))
    send = np.zeros(P, dtype=np.uint64)
    recv = np.zeros(P, dtype=np.uint64)
    fn = lib().gsort_plan_split_balanced if balanced else lib().gsort_plan_split
    _check(fn(P, n_all.ctypes.data, lt.ctypes.data, le.ctypes.data, me,
              send.ctypes.data, recv.ctypes.data), None)
    return send, recv


def plan_splitters(samples, P):
    import numpy as np
    samples = np.ascontiguousarray(samples, dtype=np.int32)
    out = np.zeros(max(P - 1, 1), dtype=np.int32)
    _check(lib().gsort_plan_splitters(P, samples.ctypes.data, out.ctypes.data), None)
    return out[: P - 1]


def plan_ref_digits(P, max_element, cap=64):
    """Host-only reference digit plan (gsort_plan_ref_digits): (loop, mod, scale)."""
    import numpy as np
    loop = ctypes.c_int()
    mod = np.zeros(cap, dtype=np.int32)
    scale = np.zeros(cap, dtype=np.float64)
    _check(lib().gsort_plan_ref_digits(P, max_element, ctypes.byref(loop), mod.ctypes.data,
                                       scale.ctypes.data, cap), None)
    k = max(loop.value, 0)
    return loop.value, mod[:k], scale[:k]


def parse_text(data, threads=1):
    """gsort_parse_text: the rank-0 reader's %d-compatible parse.  Returns int32 array or None
    on a non-numeric token."""
    import numpy as np
    if isinstance(data, str):
        data = data.encode()
    n = lib().gsort_parse_text(data, len(data), None, 0, threads)
    if n < 0:
        return None
    out = np.empty(max(n, 1), dtype=np.int32)
    n2 = lib().gsort_parse_text(data, len(data), out.ctypes.data, n, threads)
    assert n2 == n
    return out[:n]


def format_dump(keys, first_index=0, threads=1):
    """gsort_format_dump: the reference's "%u|%u" sorted dump lines for keys (bytes)."""
    import numpy as np
    keys = np.ascontiguousarray(keys, dtype=np.int32)
    n = lib().gsort_format_dump(keys.ctypes.data, keys.size, first_index, None, 0, threads)
    buf = ctypes.create_string_buffer(max(n, 1))
    m = lib().gsort_format_dump(keys.ctypes.data, keys.size, first_index, buf, n, threads)
    assert m == n
    return buf.raw[:n]
