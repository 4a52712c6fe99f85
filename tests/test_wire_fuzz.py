"""The certificate parsers (csrc/hsv_wire_parse.cpp) fuzzed under
AddressSanitizer + UndefinedBehaviorSanitizer on the host (race
detection / sanitizers on the host path).  They read untrusted network
bytes: the reference receives QC/TC frames over TCP
(network/src/receiver.rs:47-60, consensus/src/consensus.rs:32-39).  The
harness is tests/native/wire_fuzz.cpp; no GPU is involved."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG, ROOT

BIN = os.path.join(ROOT, "build", "wire_fuzz_asan")


@pytest.fixture(scope="module")
def fuzz_bin():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    csrc = os.path.join(PKG, "csrc")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-Wall", "-Wno-unknown-pragmas", "-I", csrc,
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "native", "wire_fuzz.cpp"), os.path.join(csrc, "hsv_wire_parse.cpp"),
                    "-o", BIN], check=True)
    return BIN


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_wire_parsers_fuzz_under_asan_ubsan(fuzz_bin, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([fuzz_bin, "60000", str(seed)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "wire fuzz ok" in r.stdout
