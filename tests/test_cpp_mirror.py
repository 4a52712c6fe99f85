"""The C++ mirror of the crypto crate (include/hsv_crypto.hpp) and its port of
the reference's crypto tests (tests/native/crypto_tests.cpp)."""
import os
import subprocess

import pytest

from conftest import PKG, ROOT

BIN = os.path.join(ROOT, "build", "crypto_tests")


@pytest.fixture(scope="module")
def crypto_tests_bin():
    from hsverify import _lib
    _lib.load(require=True)  # libhsv.so must exist (built by __graft_entry__.build)
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    libdir = os.path.join(PKG, "hsverify")
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wno-unknown-pragmas",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(PKG, "csrc"),
                    os.path.join(ROOT, "tests", "native", "crypto_tests.cpp"),
                    "-L", libdir, "-lhsv", f"-Wl,-rpath,{libdir}", "-lpthread", "-o", BIN], check=True)
    return BIN


def test_cpp_mirror_raises_infrastructure_error_without_gpu(crypto_tests_bin):
    from hsverify import _lib
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    r = subprocess.run([crypto_tests_bin], capture_output=True, text=True)
    assert r.returncode != 0
    assert "InfrastructureError" in r.stderr and "no HIP device" in r.stderr


@pytest.mark.gpu
def test_cpp_port_of_reference_crypto_tests(crypto_tests_bin, hsv):
    r = subprocess.run([crypto_tests_bin], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "all passed" in r.stdout
