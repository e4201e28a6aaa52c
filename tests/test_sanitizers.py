"""Host sanitizers on the native host code (no GPU): the history decoder under AddressSanitizer and
UBSan, fed intact and mutated persisted-history blobs, thriftrw and json (tests/cpp/decode_fuzz.cpp)."""
import os
import shutil
import struct
import subprocess

import pytest

from cadence_amd import synth_mixed
from cadence_amd.json_codec import serialize_history_json
from cadence_amd.thrift_codec import serialize_history

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_decoder_fuzz_under_asan_ubsan(tmp_path):
    exe = tmp_path / "decode_fuzz"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=undefined", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "decode_fuzz.cpp"),
                    os.path.join(ROOT, "cadence_amd", "csrc", "history_decode.cpp"),
                    os.path.join(ROOT, "cadence_amd", "csrc", "json_decode.cpp"), "-o", str(exe), "-lpthread"],
                   check=True)
    hs = synth_mixed.mixed_histories(60, 51, multi_version=True, invalid_rate=0.3)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    for mode, ser in (("thriftrw", serialize_history), ("json", serialize_history_json)):
        corpus = tmp_path / f"corpus_{mode}.bin"
        with open(corpus, "wb") as f:
            for h in hs:
                for b in ser(h):
                    f.write(struct.pack("<I", len(b)) + b)
        r = subprocess.run([str(exe), str(corpus), "1500", mode], capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "fuzz rounds=1500" in r.stdout
