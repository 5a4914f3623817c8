"""Resource guards on the built gfx950 code object (CPU-only: reads lib/libgsort.so, runs nothing).

Round 6 found several of the hot kernels' costs in their code generation rather than their
algorithm: register counts that decide how many workgroups share a CU,
spills, and flat memory instructions (which also count against the LDS wait counter, so every LDS
wait behind one waited for HBM).  These tests pin what the measured versions compiled to, so a
later edit that silently drops a kernel to fewer workgroups per CU, or back to flat accesses,
fails here instead of in a benchmark:
  * no flat loads or stores anywhere (the received runs go through ld_run / st_global);
  * no scratch (spills) in any kernel but the BALLOT fallback of K13g's 32 768-key boundary sort;
  * K3r / K3a (two 1024-thread workgroups per CU) within 64 VGPRs;
  * K11e / K11g class 2 (three 512-thread workgroups per CU, LDS-limited) within 64 VGPRs;
  * the packed class-3 bodies (three workgroups per CU) within 80 VGPRs (atomic-rank forms).
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mpi-test_amd", "lib", "libgsort.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _code_object(tmp):
    fat, co = os.path.join(tmp, "fat.bin"), os.path.join(tmp, "g.co")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, LIB],
                   check=True, capture_output=True)
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                    "--input=" + fat, "--output=" + co,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True, capture_output=True)
    return co


@pytest.fixture(scope="module")
def code():
    if not os.path.exists(LIB) or not os.path.exists(os.path.join(LLVM, "llvm-readelf")):
        pytest.skip("libgsort.so or the ROCm LLVM tools are missing")
    tmp = tempfile.mkdtemp()
    try:
        co = _code_object(tmp)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                               capture_output=True, text=True).stdout
        asm = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                             check=True, capture_output=True, text=True).stdout
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    kernels = {}
    for block in notes.split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", block)
        vg = re.search(r"\.vgpr_count:\s+(\d+)", block)
        sc = re.search(r"\.private_segment_fixed_size:\s+(\d+)", block)
        if name and vg and sc:
            kernels[name.group(1)] = (int(vg.group(1)), int(sc.group(1)))
    assert len(kernels) > 50, "kernel metadata not parsed"
    return kernels, asm


def _match(kernels, *parts):
    return {k: v for k, v in kernels.items() if all(p in k for p in parts)}


def test_no_flat_memory_instructions(code):
    _, asm = code
    cur, flat = None, {}
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
        if m:
            cur = m.group(1)
        elif cur and re.search(r"\bflat_(load|store|atomic)", line):
            flat[cur] = flat.get(cur, 0) + 1
    assert not flat, flat


def test_no_spills_outside_the_ballot_boundary_sort(code):
    kernels, _ = code
    spills = {k: v for k, v in kernels.items() if v[1] > 0 and "k_boundary_sort16ILb0E" not in k}
    assert not spills, spills


def test_partition_passes_keep_two_workgroups_per_cu(code):
    kernels, _ = code
    k3 = _match(kernels, "k_partition_resILi1024ELi8E")
    assert k3
    assert all(v[0] <= 64 for v in k3.values()), k3


def test_class2_sort_keeps_its_occupancy(code):
    kernels, _ = code
    c2 = {**_match(kernels, "k_local_sort_eILi512ELi18ELb1ELb0ELi2E"),
          **_match(kernels, "k_gather_sortILi512ELi18ELb1E")}
    assert len(c2) >= 3, c2
    assert all(v[0] <= 64 for v in c2.values()), c2


def test_packed_class3_bodies_fit_three_workgroups(code):
    kernels, _ = code
    c3 = {**_match(kernels, "k_local_sort_e16ILi512ELi33ELb1E"),
          **_match(kernels, "k_gather_sort16ILi512ELi33ELb1E")}
    assert len(c3) >= 3, c3
    assert all(v[0] <= 80 for v in c3.values()), c3
