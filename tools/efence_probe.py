import os, sys, numpy as np
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"] if "GRAFT_REPO_ROOT" in os.environ else "/root/repo")
sys.path.insert(0, os.path.join(sys.path[0], "mpi-test_amd"))
import torch, gsort
from oracle import orc
orc.lib()
n = int(sys.argv[1])
keys = orc.gen(orc.UNIFORM, 11, n)
with gsort.Context() as c:
    p = c.alloc(n * 4)
    c.to_device(keys, p)
    f = c.fingerprint(p, n)
    print("fingerprint ok", f["sorted"], flush=True)
    out, m, st = c.radix(p, n)
    assert np.array_equal(c.to_host(out, m), np.sort(keys))
    c.free(p)
print("ok", n, os.environ.get("GSORT_EFENCE_SLACK"))
