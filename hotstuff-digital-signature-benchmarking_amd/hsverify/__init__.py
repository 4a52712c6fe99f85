"""hsverify -- MI355X-native Ed25519 batch verification for the HotStuff crypto crate.

Layers (top to bottom):
  hsverify.crypto    mirror of the reference's crypto crate API (crypto/src/lib.rs)
  hsverify.verifier  array / device-tensor entry points
  hsverify.mempool   transaction-signature checks (mempool/src/batch_maker.rs:79-85)
  hsverify._lib      ctypes binding of libhsv.so (C ABI, include/hsv.h)
  csrc/              gfx950 HIP kernels + C ABI + host signing
"""
from ._lib import (A_OK, EQ_OK, PARSE_OK, R_OK, S_OK, SMALL_A, SMALL_R, STRICT_OK,  # noqa: F401
                   HsvLibraryError, LIB_PATH, device_count, load, version)

__all__ = ["crypto", "verifier", "mempool", "load", "device_count", "version", "HsvLibraryError",
           "STRICT_OK", "EQ_OK", "PARSE_OK", "SMALL_A", "SMALL_R", "S_OK", "A_OK", "R_OK"]
