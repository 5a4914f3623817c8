#!/usr/bin/env python3
"""dist_p1_trace.py [algo ...] -- bench.py's dist_p1 block alone (GSORT_FORCE_DIST one-rank RCCL
communicator, 2^28 uniform keys, untimed steps), for a rocprofv3 trace (development tool):
  rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -f csv -d D -o run -- \
      python3 tools/dist_p1_trace.py radix sample
then tools/step_timeline.py D/run_kernel_trace.csv k_hist16."""
import os
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(root, "mpi-test_amd"))
sys.path.insert(0, root)
import bench  # noqa: E402
import gsort  # noqa: E402

for algo in sys.argv[1:] or ["radix", "sample"]:
    r = bench.dist_p1(gsort, 1 << 28, gsort.UNIFORM, 42, steps=10, algo=algo)
    print(algo, r["ms_per_step"], r["phases_ms_avg"]["ms_total"], r["verified"], flush=True)
