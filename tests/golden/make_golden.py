#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE programs.

The reference (/root/reference, acgrid/mpi-test) ships no tests and no fixtures,
so its own sorted output is captured here: oracle/Makefile compiles mpi_radix_sort.c and
mpi_sample_sort.c unchanged into oracle/_ref/, and this script runs them under MPICH's mpirun
on inputs from the repo's splitmix64 generator (oracle.orc.gen) plus a few hand-written quirk
inputs (SURVEY.md 8 Q-list).  Only data is committed: inputs are regenerable from their spec
(and carry a sha256 to prove it); outputs are the reference's full sorted dumps.

Capture: rank-0 lines matching ^[0-9]+\\|[0-9]+$ at debug 3 (radix) or
debug 1 (sample), values re-signed from %u; sample's "[MASTER] Splitter" and
"[COMMON] r: Bucket j=len" lines; the stdout median line and "Each bucket" line; exit status.

Run from the repo root:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import orc  # noqa: E402

MPIRUN = "/opt/conda/bin/mpirun"
OUT = os.path.join(ROOT, "tests", "golden")
DUMP = re.compile(r"^(\d+)\|(\d+)$")
SPLIT = re.compile(r"^\[MASTER\] Splitter: (\d+)\.$")
BUCKET = re.compile(r"^\[COMMON\] (\d+): Bucket (\d+)=(\d+)$")
# the program-contract lines of a rank's stdout: "Each bucket" (sample:74),
# splitters (sample:124), bucket lengths (sample:157), the sorted dump (radix:199, sample:203)
# and the median (radix:201, sample:205); every other line is free-form progress output
CONTRACT = re.compile(r"^(Each bucket will be put [0-9]+ items\.|\[MASTER\] Splitter: [0-9]+\.|"
                      r"\[COMMON\] [0-9]+: Bucket [0-9]+=[0-9]+|[0-9]+\|[0-9]+|"
                      r"The n/2-th sorted element: -?[0-9]+)$")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<i4").tobytes()).hexdigest()


def contract_of(lines):
    """{sha256 of the contract lines joined by '\\n' with a final '\\n', the lines before and
    after the dump block, dump length} for one rank's stdout lines"""
    keep = [ln for ln in lines if CONTRACT.match(ln)]
    h = hashlib.sha256()
    for ln in keep:
        h.update(ln.encode() + b"\n")
    is_dump = [bool(DUMP.match(ln)) for ln in keep]
    first = is_dump.index(True) if any(is_dump) else len(keep)
    last = len(keep) - is_dump[::-1].index(True) if any(is_dump) else len(keep)
    assert all(is_dump[first:last]), "dump lines are not one block"
    return {"sha256": h.hexdigest(), "head": keep[:first], "tail": keep[last:],
            "n_dump": last - first}


def resign(u):
    u = int(u)
    return u - (1 << 32) if u >= (1 << 31) else u


def run_ref(prog, P, path, debug, timeout=120):
    tmp = tempfile.mkdtemp(prefix="gold_")
    cmd = [MPIRUN, "-np", str(P), "-outfile-pattern", f"{tmp}/o.%r", "-errfile-pattern",
           f"{tmp}/e.%r", os.path.join(orc.REF_DIR, prog), path, str(debug)]
    try:
        rc = subprocess.run(cmd, timeout=timeout, stdout=subprocess.DEVNULL,
                            stderr=subprocess.DEVNULL).returncode
    except subprocess.TimeoutExpired:
        rc = "timeout"

    def rd(name):
        p = os.path.join(tmp, name)
        return open(p, errors="replace").read().splitlines() if os.path.exists(p) else []

    out0, err0 = rd("o.0"), rd("e.0")
    others = [rd(f"o.{r}") for r in range(1, P)]
    subprocess.run(["rm", "-rf", tmp])
    dump = {}
    for ln in out0:
        m = DUMP.match(ln)
        if m:
            dump[int(m.group(1))] = resign(m.group(2))
    res = {
        "rc": rc,
        "dump": np.array([dump[i] for i in sorted(dump)], dtype=np.int32),
        "median_line": next((l for l in out0 if l.startswith("The n/2-th")), None),
        "each_bucket_line": next((l for l in out0 if l.startswith("Each bucket")), None),
        "stderr0": [re.sub(r"= [0-9.]+ sec", "= <t> sec", l) for l in err0],
        "splitters": [resign(SPLIT.match(l).group(1)) for l in out0 if SPLIT.match(l)],
    }
    mat = {}
    for lines in [out0] + others:
        for ln in lines:
            m = BUCKET.match(ln)
            if m:
                mat[(int(m.group(1)), int(m.group(2)))] = int(m.group(3))
    if mat:
        res["bucket_matrix"] = [[mat.get((r, j), 0) for j in range(P)] for r in range(P)]
    res["contract"] = [contract_of(lines) for lines in [out0] + others]
    return res


def run_ref_stream(prog, P, path, debug, timeout=1800):
    """run_ref for large inputs: at debug 3 the reference's radix prints every key of every
    pass ("DUMP: LOOP", radix:175-178; ~13 GB of text at 2^24 keys, P = 2), so the merged
    stdout (-prepend-rank) is filtered to the contract lines by grep on the fly and only the
    filtered stream is parsed."""
    tmp = tempfile.mkdtemp(prefix="goldL_")
    filt, err = os.path.join(tmp, "f"), os.path.join(tmp, "e")
    cmd = (f"{MPIRUN} -prepend-rank -np {P} {os.path.join(orc.REF_DIR, prog)} {path} {debug} "
           f"2>{err} | LC_ALL=C grep -a -E '^\\[[0-9]+\\] ({CONTRACT.pattern[2:-2]})$' > {filt}")
    try:
        rc = subprocess.run(["bash", "-o", "pipefail", "-c", cmd], timeout=timeout).returncode
    except subprocess.TimeoutExpired:
        rc = "timeout"
    per = [[] for _ in range(P)]
    with open(filt, "rb") as f:
        for raw in f:
            r, _, ln = raw.decode().rstrip("\n").partition("] ")
            per[int(r[1:])].append(ln)
    err0 = [ln.partition("] ")[2] for ln in open(err, errors="replace").read().splitlines()
            if ln.startswith("[0] ")]
    subprocess.run(["rm", "-rf", tmp])
    out0 = per[0]
    dump = [DUMP.match(ln) for ln in out0]
    vals = np.array([int(m.group(2)) for m in dump if m], dtype=np.uint64)
    idx = np.array([int(m.group(1)) for m in dump if m], dtype=np.int64)
    assert idx.size == 0 or np.array_equal(idx, np.arange(idx.size)), "dump index order"
    res = {
        "rc": rc,
        "dump": vals.astype(np.uint32).view(np.int32),
        "median_line": next((l for l in out0 if l.startswith("The n/2-th")), None),
        "each_bucket_line": next((l for l in out0 if l.startswith("Each bucket")), None),
        "stderr0": [re.sub(r"= [0-9.]+ sec", "= <t> sec", l) for l in err0],
        "splitters": [resign(SPLIT.match(l).group(1)) for l in out0 if SPLIT.match(l)],
        "contract": [contract_of(lines) for lines in per],
    }
    mat = {}
    for lines in per:
        for ln in lines:
            m = BUCKET.match(ln)
            if m:
                mat[(int(m.group(1)), int(m.group(2)))] = int(m.group(3))
    if mat:
        res["bucket_matrix"] = [[mat.get((r, j), 0) for j in range(P)] for r in range(P)]
    return res


def main_large():
    """tests/golden/ref_large.json: the reference's output at the sizes the build's default
    (sampled) local plan runs at, >= 2^22 keys.  Data only: sha256 of the full
    sorted dump, median / "Each bucket" lines, splitters, bucket matrices and per-rank contract
    transcripts (sha256 + the non-dump lines); no arrays."""
    orc.build()
    tmpdir = tempfile.mkdtemp(prefix="goldLin_")
    cases = []
    plan = [(orc.UNIFORM, "uniform", 1 << 22, 42, (2, 4, 8), (2, 4, 8)),
            (orc.UNIFORM, "uniform", 1 << 24, 42, (2, 4, 8), (2, 4, 8)),
            (orc.ZIPF, "zipf", 1 << 22, 7, (2, 4, 8), (2, 4)),
            (orc.ZIPF, "zipf", 1 << 24, 7, (8,), (2,))]
    for dist, dname, n, seed, radix_ps, sample_ps in plan:
        keys = orc.gen(dist, seed, n)
        want = sha(np.sort(keys))
        path = os.path.join(tmpdir, "in.txt")
        orc.write_text(path, keys)
        spec = {"gen": dname, "n": n, "seed": seed}
        for prog, ps, debug in (("radix_sort", radix_ps, 3), ("sample_sort", sample_ps, 1)):
            for P in ps:
                r = run_ref_stream(prog, P, path, debug)
                c = {"id": f"{dname}{n}s{seed}__{prog}__P{P}", "prog": prog, "P": P,
                     "input": spec, "input_sha256": sha(keys), "rc": r["rc"],
                     "median_line": r["median_line"], "each_bucket_line": r["each_bucket_line"],
                     "stderr0": r["stderr0"], "n_dump": int(r["dump"].size),
                     "output_sha256": sha(r["dump"]) if r["dump"].size else None,
                     "contract": r["contract"]}
                # the reference's sample sort overflows its fixed receive buffers on skewed
                # inputs: record whether this run produced the sorted array
                c["output_is_sorted_input"] = c["output_sha256"] == want
                if prog == "sample_sort":
                    c["splitters"] = r["splitters"]
                    c["bucket_matrix"] = r.get("bucket_matrix")
                cases.append(c)
                print(c["id"], "rc", c["rc"], "n", c["n_dump"], "sorted",
                      c["output_is_sorted_input"], flush=True)
    with open(os.path.join(OUT, "ref_large.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py --large", "mpirun": MPIRUN,
                   "cases": cases}, f, indent=1)
    subprocess.run(["rm", "-rf", tmpdir])
    print("wrote", len(cases), "large cases")


def main():
    orc.build()
    tmpdir = tempfile.mkdtemp(prefix="goldin_")
    cases = []
    arrays = {}

    def add_case(name, prog, P, keys, spec, text=None):
        path = os.path.join(tmpdir, name + ".txt")
        if text is None:
            orc.write_text(path, keys)
        else:
            with open(path, "w") as f:
                f.write(text)
        debug = 3 if prog == "radix_sort" else 1
        r = run_ref(prog, P, path, debug)
        key = f"{name}__{prog}__P{P}"
        c = {"id": key, "prog": prog, "P": P, "input": spec, "rc": r["rc"],
             "median_line": r["median_line"], "each_bucket_line": r["each_bucket_line"],
             "stderr0": r["stderr0"], "n_dump": int(r["dump"].size)}
        if keys is not None:
            c["input_sha256"] = sha(keys)
        if r["dump"].size:
            c["output_sha256"] = sha(r["dump"])
            arrays[key] = r["dump"]
        if prog == "sample_sort":
            c["splitters"] = r["splitters"]
            c["bucket_matrix"] = r.get("bucket_matrix")
        c["contract"] = r["contract"]
        cases.append(c)
        print(key, "rc", r["rc"], "n", r["dump"].size, flush=True)

    # canonical generated inputs, inside the parity domain
    for dist, dname, n, seed in [(orc.UNIFORM, "uniform", 1 << 10, 42),
                                 (orc.UNIFORM, "uniform", 1 << 16, 42),
                                 (orc.ZIPF, "zipf", 1 << 16, 7)]:
        keys = orc.gen(dist, seed, n)
        spec = {"gen": dname, "n": n, "seed": seed}
        for P in (2, 4, 8):
            add_case(f"{dname}{n}s{seed}", "radix_sort", P, keys, spec)
        for P in ((2, 4, 8) if dist == orc.UNIFORM else (2, 4)):
            add_case(f"{dname}{n}s{seed}", "sample_sort", P, keys, spec)
    # P = 3 (Q3 pass-count under-count at 243) and P = 1 (Q1 zero passes)
    keys = orc.gen(orc.UNIFORM, 5, 999) % 1000
    keys[17] = 243
    add_case("u999mod1000", "radix_sort", 3, keys, {"gen": "uniform", "n": 999, "seed": 5,
                                                     "mod": 1000, "set": [[17, 243]]})
    keys = np.array([250, 7, 243, 1, 242, 9], dtype=np.int32)
    add_case("q3_max243", "radix_sort", 3, keys, {"literal": keys.tolist()})
    keys = orc.gen(orc.UNIFORM, 42, 1000)
    add_case("uniform1000s42", "radix_sort", 1, keys, {"gen": "uniform", "n": 1000, "seed": 42})
    # Q2 negative keys (ref-radix sorts by |v| mod P^loop, stable)
    neg = np.array([-7, 3, 7, -2, 2, -3, 5, 0], dtype=np.int32)
    for P in (2, 4, 8):
        add_case("q2_neg8", "radix_sort", P, neg, {"literal": neg.tolist()})
    # Q6 trailing newline phantom, Q7 %d wrap of out-of-range text
    add_case("q6_trailing_nl", "radix_sort", 2, None, {"text": "5\n3\n9\n1\n"},
             text="5\n3\n9\n1\n")
    add_case("q7_wrap", "radix_sort", 2, None,
             {"text": "2147483648 4294967295 12 -5 0 4294967296 77 1"},
             text="2147483648 4294967295 12 -5 0 4294967296 77 1")
    # Q9 "no enough sample" abort (N=9, P=4)
    k9 = np.arange(9, 0, -1, dtype=np.int32)
    add_case("q9_n9", "sample_sort", 4, k9, {"literal": k9.tolist()})

    with open(os.path.join(OUT, "ref_cases.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "mpirun": MPIRUN,
                   "cases": cases}, f, indent=1)
    # outputs are identical across P inside the parity domain: store each distinct array once
    uniq, index = {}, {}
    for k, a in arrays.items():
        h = sha(a)
        if h not in uniq:
            uniq[h] = a
        index[k] = h
    np.savez_compressed(os.path.join(OUT, "ref_outputs.npz"),
                        **{"h_" + h[:16]: a for h, a in uniq.items()})
    subprocess.run(["rm", "-rf", tmpdir])
    print("wrote", len(cases), "cases,", len(uniq), "distinct output arrays")


if __name__ == "__main__":
    main_large() if "--large" in sys.argv[1:] else main()
