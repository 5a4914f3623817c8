import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mpi-test_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")


@pytest.fixture(scope="session")
def orc():
    from oracle import orc as _orc
    _orc.lib()
    return _orc


@pytest.fixture(scope="session")
def ref_cases():
    with open(os.path.join(GOLDEN, "ref_cases.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def ref_outputs():
    z = np.load(os.path.join(GOLDEN, "ref_outputs.npz"))
    return {k: z[k] for k in z.files}


def case_input(orc, spec):
    """Rebuild a golden case's input from its spec (tests/golden/make_golden.py)."""
    if "literal" in spec:
        return np.array(spec["literal"], dtype=np.int32)
    if "text" in spec:
        return None
    dist = orc.UNIFORM if spec["gen"] == "uniform" else orc.ZIPF
    keys = orc.gen(dist, spec["seed"], spec["n"])
    if "mod" in spec:
        keys = keys % spec["mod"]
    for i, v in spec.get("set", []):
        keys[i] = v
    return keys


def case_output(case, ref_outputs):
    if "output_sha256" not in case:
        return None
    return ref_outputs["h_" + case["output_sha256"][:16]]


@pytest.fixture(scope="session")
def gsort():
    """The product's Python binding (ctypes over libgsort.so).  Loads torch first so both
    share one HIP runtime ('one runtime per process')."""
    import torch  # noqa: F401
    import gsort as _g
    return _g


@pytest.fixture(autouse=True)
def _gsort_memlog(request):
    """GSORT_MEMLOG=path: append each GPU test's device free/total bytes after it ran
    (diagnostics for device-memory growth across a test session)."""
    yield
    path = os.environ.get("GSORT_MEMLOG")
    if not path or request.node.get_closest_marker("gpu") is None:
        return
    import torch
    free, total = torch.cuda.mem_get_info()
    with open(path, "a") as f:
        f.write(f"{request.node.nodeid} {free} {total}\n")


@pytest.fixture(scope="session")
def ref_large():
    """Reference runs at >= 2^22 keys (tests/golden/make_golden.py --large): digests only."""
    path = os.path.join(GOLDEN, "ref_large.json")
    if not os.path.exists(path):
        pytest.skip("tests/golden/ref_large.json not generated")
    with open(path) as f:
        return json.load(f)["cases"]


GOLDEN_DEBUG = {"radix_sort": 3, "sample_sort": 1}  # the debug level every fixture was run at


def contract_split(data):
    """A rank's stdout bytes -> (lines before the dump, dump line count, lines after)."""
    lines = data.decode().splitlines()
    is_dump = [("|" in ln and ln.replace("|", "").isdigit()) for ln in lines]
    first = is_dump.index(True) if any(is_dump) else len(lines)
    last = len(lines) - is_dump[::-1].index(True) if any(is_dump) else len(lines)
    return lines[:first], last - first, lines[last:]
