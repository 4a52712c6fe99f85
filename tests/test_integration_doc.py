"""The Rust shim in INTEGRATION.md keeps the reference's public signatures.

north_star: the `crypto::Signature::verify_batch` / `Signature::verify`
signatures stay unchanged, so consensus, mempool and node compile untouched.
The reference lines (crypto/src/lib.rs:204 and 210-213) are hard-coded here:
/root/reference does not travel to the GPU box, and this test must fail if
the shim drifts from them (round 2 added `+ Clone` to the bound).
"""
import os
import re

from conftest import ROOT

# crypto/src/lib.rs:204
REF_VERIFY = "pub fn verify(&self, digest: &Digest, public_key: &PublicKey) -> Result<(), CryptoError> {"
# crypto/src/lib.rs:210-213
REF_VERIFY_BATCH = [
    "pub fn verify_batch<'a, I>(digest: &Digest, votes: I) -> Result<(), CryptoError>",
    "where",
    "I: IntoIterator<Item = &'a (PublicKey, Signature)>,",
    "{",
]


def _shim_lines():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```rust\n(.*?)```", text, flags=re.S)
    shim = next(b for b in blocks if "impl Signature" in b)
    lines = [l.strip() for l in shim.splitlines()]
    return lines[lines.index("impl Signature {"):]  # the crate's type, not the FFI block


def test_shim_verify_signature_is_the_reference_one():
    lines = _shim_lines()
    pubs = [l for l in lines if l.startswith("pub fn verify(")]
    assert pubs == [REF_VERIFY]


def test_shim_verify_batch_signature_is_the_reference_one():
    lines = _shim_lines()
    i = lines.index(REF_VERIFY_BATCH[0])
    assert lines[i:i + 4] == REF_VERIFY_BATCH
    # no other public fn or changed bound anywhere in the impl
    assert [l for l in lines if l.startswith("pub fn ")] == [REF_VERIFY, REF_VERIFY_BATCH[0]]
    assert not any("Clone" in l for l in lines if "IntoIterator" in l)
