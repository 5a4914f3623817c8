"""Which VMM-fenced buffer makes the CLI's 1-rank sort of zipf 65536 (seed 7) go wrong?"""
import os, subprocess, sys
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [ROOT, os.path.join(ROOT, "mpi-test_amd")]
import numpy as np
from oracle import orc
orc.lib()
keys = orc.gen(orc.ZIPF, 7, 65536)
want = np.sort(keys)
path = "/tmp/zipf65536.txt"
orc.write_text(path, keys)
def dump(out):
    v = [int(l.split("|")[1]) for l in out.splitlines() if "|" in l and l.split("|")[0].isdigit()]
    return np.array(v, dtype=np.int64).astype(np.uint32).astype(np.int32)
names = sys.argv[1].split(";") if len(sys.argv) > 1 else [""]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
for only in names:
    bad_runs = 0
    for rep in range(reps):
        env = dict(os.environ, GSORT_EFENCE="1", GSORT_EFENCE_ONLY=only)
        r = subprocess.run([os.path.join(ROOT, "mpi-test_amd/bin/radix_sort"), path, "3"],
                           env=env, capture_output=True, text=True, timeout=120)
        got = dump(r.stdout)
        if r.returncode != 0 or got.size != want.size or not np.array_equal(got, want):
            bad_runs += 1
    print(f"EFENCE_ONLY={only or 'ALL'}: {bad_runs}/{reps} wrong", flush=True)
