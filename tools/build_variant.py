"""Profiling aid (not product code): the replay library rebuilt with extra -D switches, for A/B runs on
one box (tools/prof_kernel.py / tools/prof_longtail.py --lib).

    python tools/build_variant.py NAME [--src=FILE] -DCRR_WAVE_FIELDS=0 [...]   ->  tools/variants/NAME.so

Only replay_kernel.hip (or the --src= file, e.g. ingest_kernel.hip) is recompiled; the other objects come
from build/ (__graft_entry__.build()).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import __graft_entry__ as ge
    name, defs = sys.argv[1], sys.argv[2:]
    src = os.path.join(ROOT, "cadence_amd", "csrc", "replay_kernel.hip")
    if defs and defs[0].startswith("--src="):   # another version of the kernel source (e.g. the last commit's)
        src, defs = os.path.abspath(defs[0][6:]), defs[1:]
    outdir = os.path.join(ROOT, "tools", "variants")
    os.makedirs(outdir, exist_ok=True)
    obj = os.path.join(outdir, name + ".o")
    sched = os.environ.get("CRR_VARIANT_SCHED", "max-ilp")   # "default": the compiler's own scheduler
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
             *([] if sched == "default" else ["-mllvm", "-amdgpu-sched-strategy=" + sched]),
             "-I", os.path.join(ROOT, "include"), *defs]
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-I", os.path.join(ROOT, "cadence_amd", "csrc"), "-c", src, "-o", obj],
                   check=True)
    others = [os.path.join(ROOT, "build", os.path.basename(s) + ".o") for s in ge.HIP_SOURCES
              if os.path.basename(s) != os.path.basename(src)]
    out = os.path.join(outdir, name + ".so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", obj, *others, "-o", out], check=True)
    os.remove(obj)
    print(out)


if __name__ == "__main__":
    main()
