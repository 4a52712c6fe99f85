"""Shared fixtures for the hot-path tests.

Markers:
  gpu  -- needs an MI355X (runs through libhsv.so's C ABI on cuda:0)

CPU tests (-m "not gpu") cover the oracle against the golden vectors and
libsodium, the kernel's arithmetic compiled for the host, the C-ABI library's
exports and error paths, and the multi-rank sharding over gloo.
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD MI355X GPU (HIP)")


def _make(dirpath):
    subprocess.run(["make", "-s", "-j8"], cwd=dirpath, check=True)


@pytest.fixture(scope="session")
def oracle_lib():
    """The C restatement (oracle/_build/libhsv_oracle.so), built on demand."""
    so = os.path.join(ORACLE, "_build", "libhsv_oracle.so")
    if not os.path.exists(so):
        _make(ORACLE)
    lib = ctypes.CDLL(so)
    lib.oracle_verify_flags.restype = ctypes.c_uint8
    lib.oracle_verify_flags.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    lib.oracle_verify_many.restype = ctypes.c_int
    lib.oracle_verify_many.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
    lib.oracle_verify_batch.restype = ctypes.c_int
    lib.oracle_verify_batch.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    lib.oracle_verify_tx_many.restype = ctypes.c_int
    lib.oracle_verify_tx_many.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                          ctypes.c_void_p, ctypes.c_int]
    return lib


def oracle_tx_flags(lib, buf, offsets=None, tx_size=0, n=None, nthreads=None):
    """Transaction flags via the C oracle: buf u8, offsets u64 (n+1) or fixed tx_size."""
    buf = np.ascontiguousarray(buf, np.uint8)
    if n is None:
        n = len(offsets) - 1 if offsets is not None else buf.size // tx_size
    out = np.zeros(n, np.uint8)
    nt = nthreads or min(16, os.cpu_count() or 1)
    lib.oracle_verify_tx_many(buf.ctypes.data, offsets.ctypes.data if offsets is not None else None, tx_size, n,
                              out.ctypes.data, nt)
    return out


@pytest.fixture(scope="session")
def tx_golden():
    """Mempool transaction vectors (tests/golden/make_tx_golden.py): txs (list of
    bytes), flags (u8 array), cases."""
    with open(os.path.join(GOLDEN, "tx_vectors.json")) as f:
        vecs = json.load(f)["vectors"]
    return {"txs": [bytes.fromhex(v["tx"]) for v in vecs],
            "flags": np.array([v["flags"] for v in vecs], np.uint8),
            "cases": [v["case"] for v in vecs]}


def oracle_flags(lib, pk, sig, msg, nthreads=None):
    """Flags for arrays pk (n,32), sig (n,64), msg (n,32) via the C oracle."""
    pk = np.ascontiguousarray(pk, np.uint8)
    sig = np.ascontiguousarray(sig, np.uint8)
    msg = np.ascontiguousarray(msg, np.uint8)
    n = pk.shape[0]
    out = np.zeros(n, np.uint8)
    stride = 0 if msg.ndim == 1 else 32
    nt = nthreads or min(16, os.cpu_count() or 1)
    lib.oracle_verify_many(pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, stride, n, out.ctypes.data, nt)
    return out


@pytest.fixture(scope="session")
def golden():
    """All golden records: dict of arrays pk, sig, msg, flags and the edge labels."""
    with open(os.path.join(GOLDEN, "edge_vectors.json")) as f:
        edge = json.load(f)["vectors"]
    raw = np.fromfile(os.path.join(GOLDEN, "random_vectors.bin"), dtype=np.uint8).reshape(-1, 129)
    hx = lambda key, w: np.frombuffer(bytes.fromhex("".join(e[key] for e in edge)), np.uint8).reshape(-1, w)
    return {
        "pk": np.concatenate([hx("pk", 32), raw[:, :32]]),
        "sig": np.concatenate([hx("sig", 64), raw[:, 32:96]]),
        "msg": np.concatenate([hx("msg", 32), raw[:, 96:128]]),
        "flags": np.concatenate([np.array([e["flags"] for e in edge], np.uint8), raw[:, 128]]),
        "cases": [e["case"] for e in edge] + ["random"] * raw.shape[0],
        "n_edge": len(edge),
    }


@pytest.fixture(scope="session")
def fallback_records():
    """Records whose challenge takes the kernels' full-length fallback path
    (tests/golden/make_lattice_fallback.py): honest, corrupted-s, s + l and
    mixed-order-key variants."""
    raw = np.fromfile(os.path.join(GOLDEN, "lattice_fallback.bin"), dtype=np.uint8).reshape(-1, 129)
    return {"pk": raw[:, :32].copy(), "sig": raw[:, 32:96].copy(), "msg": raw[:, 96:128].copy(),
            "flags": raw[:, 128].copy()}


@pytest.fixture(scope="session")
def reference_fixtures():
    with open(os.path.join(GOLDEN, "reference_fixtures.json")) as f:
        return json.load(f)


def _gpu_available():
    try:
        from hsverify import _lib
        return _lib.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def hsv():
    """The product library on a GPU box; fails loudly if the build is missing."""
    from hsverify import _lib
    lib = _lib.load(require=True)
    if lib.hsv_device_count() <= 0:
        pytest.fail("gpu test collected but no HIP device is visible")
    return lib
