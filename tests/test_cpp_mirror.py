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
    # the C oracle is linked in only as the --fallback stand-in for a host verifier
    oracle_o = BIN + "_oracle.o"
    subprocess.run(["gcc", "-O2", "-c", os.path.join(ROOT, "oracle", "ed25519_oracle.c"), "-o", oracle_o],
                   check=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-Wno-unknown-pragmas",
                    "-I", os.path.join(ROOT, "include"), "-I", os.path.join(PKG, "csrc"),
                    os.path.join(ROOT, "tests", "native", "crypto_tests.cpp"), oracle_o,
                    "-L", libdir, "-lhsv", f"-Wl,-rpath,{libdir}", "-lpthread", "-o", BIN], check=True)
    return BIN


def test_cpp_mirror_raises_infrastructure_error_without_gpu(crypto_tests_bin):
    from hsverify import _lib
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    r = subprocess.run([crypto_tests_bin], capture_output=True, text=True)
    assert r.returncode != 0
    assert "InfrastructureError" in r.stderr and "no HIP device" in r.stderr


def test_cpp_mirror_infrastructure_fallback_policy(crypto_tests_bin):
    """Caller-side policy for infrastructure errors:
    with a fallback verifier installed, a missing device does not take the
    caller down and does not turn into a rejection -- the reference's crypto
    tests pass through the fallback, and every verify used it."""
    from hsverify import _lib
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    r = subprocess.run([crypto_tests_bin, "--fallback"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "all passed" in r.stdout
    uses = int(r.stdout.split("infrastructure fallbacks:")[1].split()[0])
    assert uses >= 6, r.stdout  # every verify / verify_batch call of the port


@pytest.mark.gpu
def test_cpp_fallback_unused_on_gpu(crypto_tests_bin, hsv):
    """With a device the fallback is never consulted: every verdict is libhsv's."""
    r = subprocess.run([crypto_tests_bin, "--fallback"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "infrastructure fallbacks: 0" in r.stdout


@pytest.mark.gpu
def test_cpp_port_of_reference_crypto_tests(crypto_tests_bin, hsv):
    r = subprocess.run([crypto_tests_bin], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "all passed" in r.stdout


@pytest.mark.gpu
def test_cpp_mirror_repeated_with_concurrent_cache_build(crypto_tests_bin, hsv):
    """Regression: the reference's QC test (forged vote -> Err) while the
    automatic committee cache makes its first allocations on its build thread.
    Before launch workspaces came from the library's own memory pool, 8 of 16
    fresh processes accepted the forged vote (profiles/r02t_forgery/summary.txt);
    each run is a fresh process, so each gets that race."""
    for i in range(8):
        r = subprocess.run([crypto_tests_bin], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, f"run {i}: {r.stderr}"
