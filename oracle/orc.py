"""ctypes binding of oracle/liborcl.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; it is
the parity checker, never the measured or shipped path.  See oracle/oracle.c for what each
function restates (with /root/reference file:line cites).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liborcl.so")
REF_DIR = os.path.join(HERE, "_ref")

OK, E_OUTSIDE_PD, E_NO_SAMPLE, E_OVERFLOW, E_NOMEM = 0, 1, 2, 3, 4
UNIFORM, ZIPF = 0, 1

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P, U64, SZ, I = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_size_t, ctypes.c_int
        L.orc_gen.argtypes = [I, U64, U64, SZ, P]
        L.orc_gen_one.argtypes = [I, U64, U64]
        L.orc_gen_one.restype = ctypes.c_int32
        L.orc_read_ints.argtypes = [ctypes.c_char_p, P, ctypes.c_long, I]
        L.orc_read_ints.restype = ctypes.c_long
        L.orc_ref_number_digits.argtypes = [I, I]
        L.orc_ref_digit_at.argtypes = [I, I, I]
        L.orc_ref_radix.argtypes = [P, SZ, I, P, P]
        L.orc_ref_sample.argtypes = [P, SZ, I, P, P, P, P]
        L.orc_lsd8.argtypes = [P, SZ, P]
        L.orc_digit_hist.argtypes = [P, SZ, I, P]
        L.orc_radix_route.argtypes = [I, P, U64, I, P, P, P]
        L.orc_radix_route.restype = ctypes.c_long
        L.orc_sample_plan.argtypes = [I, P, P, U64, P, P]
        L.orc_fingerprint.argtypes = [P, SZ, P, P, P]
        L.orc_qsort_i32.argtypes = [P, SZ]
        L.orc_write_text.argtypes = [ctypes.c_char_p, P, SZ]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def gen(dist, seed, n, start=0):
    out = np.empty(n, dtype=np.int32)
    lib().orc_gen(dist, seed, start, n, _p(out))
    return out


def read_ints(path, with_phantom=False, cap=1 << 26):
    buf = np.empty(cap, dtype=np.int32)
    n = lib().orc_read_ints(path.encode(), _p(buf), cap, 1 if with_phantom else 0)
    if n < 0:
        raise FileNotFoundError(path)
    return buf[:n].copy()


def ref_radix(keys, P):
    keys = np.ascontiguousarray(keys, dtype=np.int32)
    out = np.empty_like(keys)
    passes = ctypes.c_int(0)
    rc = lib().orc_ref_radix(_p(keys), keys.size, P, _p(out), ctypes.byref(passes))
    return rc, out, passes.value


def ref_sample(keys, P):
    keys = np.ascontiguousarray(keys, dtype=np.int32)
    out = np.empty_like(keys)
    spl = np.zeros(max(P - 1, 1), dtype=np.int32)
    mat = np.zeros(P * P, dtype=np.int64)
    recv = np.zeros(P, dtype=np.int64)
    rc = lib().orc_ref_sample(_p(keys), keys.size, P, _p(out), _p(spl), _p(mat), _p(recv))
    return rc, out, spl[: P - 1], mat.reshape(P, P), recv


def lsd8(keys):
    keys = np.ascontiguousarray(keys, dtype=np.int32)
    out = np.empty_like(keys)
    rc = lib().orc_lsd8(_p(keys), keys.size, _p(out))
    assert rc == OK
    return out


def digit_hist(keys, pass_idx):
    keys = np.ascontiguousarray(keys, dtype=np.int32)
    h = np.zeros(256, dtype=np.uint64)
    lib().orc_digit_hist(_p(keys), keys.size, pass_idx, _p(h))
    return h


def radix_route(hist, B, me):
    """hist: (P, 256) uint64.  Returns (send[P], recv[P], seg rows (k,4))."""
    hist = np.ascontiguousarray(hist, dtype=np.uint64)
    P = hist.shape[0]
    send = np.zeros(P, dtype=np.uint64)
    recv = np.zeros(P, dtype=np.uint64)
    seg = np.zeros((P * 256 + P) * 4, dtype=np.uint64)
    rows = lib().orc_radix_route(P, _p(hist), B, me, _p(send), _p(recv), _p(seg))
    return send, recv, seg[: rows * 4].reshape(rows, 4)


def sample_plan(samples, blk, P):
    samples = np.ascontiguousarray(samples, dtype=np.int32)
    blk = np.ascontiguousarray(blk, dtype=np.int32)
    spl = np.zeros(max(P - 1, 1), dtype=np.int32)
    bounds = np.zeros(P, dtype=np.uint64)
    lib().orc_sample_plan(P, _p(samples), _p(blk), blk.size, _p(spl), _p(bounds))
    return spl[: P - 1], bounds


def fingerprint(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    s, x, ok = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_int(0)
    lib().orc_fingerprint(_p(a), a.size, ctypes.byref(s), ctypes.byref(x), ctypes.byref(ok))
    return s.value, x.value, bool(ok.value)


def qsort_inplace(a):
    lib().orc_qsort_i32(_p(a), a.size)


def write_text(path, a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    if lib().orc_write_text(path.encode(), _p(a), a.size) != 0:
        raise OSError(path)
