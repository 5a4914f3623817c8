#!/usr/bin/env python3
"""isa_scc_check.py [libgsort.so] -- scan libgsort's gfx950 code object for an SCC hazard.

ROCm 7.2's backend miscompiled a uniform 64-bit min() in K1h (gsort_kernels.hip, k_counts_h16):
the compare was done in VCC for an s_cbranch_vccz, the `s_and_b64 vcc, vcc, exec` that also
sets SCC was removed in front of the branch, and the s_cselect after it read SCC from an
unrelated address add -- a tile-length select that silently became 8192, so K1h loaded up to
32 KiB past the end of its input (an intermittent page fault in the 8-rank group tests).

Rule checked here: every SCC consumer (s_cselect_*, s_cbranch_scc*) must be fed, in program
order within its function, by a compare (s_cmp*, s_bitcmp*) or by a logical op (s_and/s_or/...,
whose SCC is `result != 0`, the backend's lowering of a uniform VALU compare); an arithmetic
SCC writer (add/sub with carry, shifts, bfe, min/max) feeding a select is reported.  Listing
order is not control flow, so a report is a candidate to read, not a proof; the product has
none.  Prints the reports; exit status 1 if there are any.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mpi-test_amd", "lib", "libgsort.so")

SCC_ARITH = re.compile(r"^(s_add_u32|s_addc_u32|s_sub_u32|s_subb_u32|s_add_i32|s_sub_i32|"
                       r"s_lshl_b\d+|s_lshr_b\d+|s_ashr_i\d+|s_bfe_\w+|s_min_\w+|s_max_\w+|"
                       r"s_abs_i32|s_absdiff_i32|s_lshl\d_add_u32)$")
SCC_OK = re.compile(r"^(s_cmp\w*|s_bitcmp\w*|s_and_b\d+|s_or_b\d+|s_xor_b\d+|s_andn2_b\d+|"
                    r"s_orn2_b\d+|s_nand_b\d+|s_nor_b\d+|s_xnor_b\d+|s_not_b\d+|"
                    r"s_\w+_saveexec_b\d+)$")
SCC_USE = re.compile(r"^(s_cselect_b\d+|s_cbranch_scc[01])$")


def disassemble(lib):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "co.elf")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        f"--input={fat}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--output={co}"], check=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co],
                              check=True, capture_output=True, text=True).stdout


def scan(listing):
    reports, fn, last = [], None, None
    for line in listing.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:", line)
        if m:
            fn, last = m.group(1), None
            continue
        parts = line.strip().split(None, 1)
        if not parts:
            continue
        op = parts[0]
        if SCC_USE.match(op) and last is not None and SCC_ARITH.match(last[0]):
            reports.append(f"{fn}: {line.strip()}  <- SCC from: {last[1]}")
        # a `s_cselect_b64 x, -1, 0` materialising SCC is itself an SCC use, not a writer
        if SCC_ARITH.match(op) or SCC_OK.match(op):
            last = (op, line.strip())
    return reports


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else LIB
    reports = scan(disassemble(lib))
    for r in reports:
        print(r)
    print(f"{len(reports)} SCC hazard candidate(s) in {lib}")
    return 1 if reports else 0


if __name__ == "__main__":
    sys.exit(main())
