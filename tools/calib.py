"""Profiling aid: stream a known byte count at the replay kernels' access widths (tools/libcalib.so),
so a rocprofv3 --pmc pass can convert FETCH_SIZE / WRITE_SIZE into bytes for those widths.

    rocprofv3 --kernel-trace --pmc FETCH_SIZE -- python3 tools/calib.py [--mib 1024]
"""
import argparse
import ctypes
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KINDS = {1: "read u8/lane", 4: "read u32/lane", 8: "read u64/lane", 108: "write u64/lane",
         1014: "gather u64 per 112-B row/lane", 1026: "gather u64 per 208-B row/lane", 1002: "gather u64 per 16-B row/lane"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mib", type=int, default=1024, help="bytes streamed per dispatch (past the 256 MiB L3)")
    p.add_argument("--reps", type=int, default=2)
    a = p.parse_args()
    print(json.dumps(run(a.mib, a.reps)))


def run(mib, reps):
    import torch
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libcalib.so"))
    lib.calib_stream.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    nbytes = mib << 20
    buf = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    scratch = torch.zeros(4096 * 256, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    for kind in KINDS:
        for _ in range(reps):
            rc = lib.calib_stream(kind, buf.data_ptr(), nbytes, scratch.data_ptr(), s.cuda_stream)
            if rc != 0:
                raise RuntimeError(f"calib_stream({kind}) failed: {rc}")
            torch.cuda.synchronize()
    return {"bytes_per_dispatch": nbytes, "kinds": KINDS}


if __name__ == "__main__":
    main()
