"""Per-kernel instruction counts of a HIP source's gfx950 ISA (scratch / global / LDS traffic sites).

    python tools/isa_stats.py cadence_amd/csrc/ingest_kernel.hip [substring ...]

Compiles device-only to assembly (hipcc -S) and counts, per function, the scratch loads / stores (spills
and private arrays), global loads / stores and LDS ops: a quick check that a hot kernel has no scratch
traffic before spending GPU time on it.
"""
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def isa(src):
    out = os.path.join(tempfile.mkdtemp(), "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                    "-I" + os.path.join(HERE, "include"), "-I" + os.path.join(HERE, "cadence_amd", "csrc"),
                    "--cuda-device-only", "-S", "-o", out, src], check=True)
    return open(out).read()


def main():
    src, subs = sys.argv[1], sys.argv[2:]
    s = isa(src)
    pats = {"scratch_ld": r"\bscratch_load|buffer_load\w* v\d+, off, s\[0:3\]",
            "scratch_st": r"\bscratch_store|buffer_store\w* v\d+, off, s\[0:3\]",
            "global_ld": r"\bglobal_load", "global_st": r"\bglobal_store", "lds": r"\bds_", "calls": r"\bs_swappc|\bs_setpc"}
    for m in re.finditer(r"^([_A-Za-z]\w*):[^\n]*\n(.*?)\.Lfunc_end", s, re.S | re.M):
        name, body = m.group(1), m.group(2)
        if subs and not any(k in name for k in subs):
            continue
        counts = " ".join(f"{k}={len(re.findall(p, body)):4d}" for k, p in pats.items())
        print(f"{name[:70]:70s} lines={body.count(chr(10)):6d} {counts}")


if __name__ == "__main__":
    main()
