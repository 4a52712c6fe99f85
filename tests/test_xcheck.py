"""The oracle pinned by two independent verifiers, over every committed record set.

* OpenSSL 3.0.2 answers the batch rule (PARSE_OK and EQ_OK) that
  `Signature::verify_batch` and so `QC::verify` depend on
  (`/root/reference/crypto/src/lib.rs:210-223` -> `consensus/src/messages.rs:197`;
  SURVEY Appendix A.2, A.3 rows 5-8).  libsodium only pins STRICT_OK, and it
  rejects small-order points by blocklist, so before round 4 "batch accepts a
  small-order A or R with e = O" rested on the oracle alone.
* libsodium 1.0.18 answers the strict rule (`lib.rs:204-208`), now over the C3
  and 2^15-random vectors too, not only the golden set.

Every disagreement must fall in a named class (tests/xcheck.py):
OpenSSL compares R by bytes, so an R whose bytes are not its point's canonical
encoding (y >= p, or x = 0 with the sign bit) is accepted by dalek's batch rule
and never by OpenSSL.  The committed columns (tests/golden/xcheck_verdicts.json,
tests/golden/make_xcheck.py) are checked against live runs of both libraries.
"""
import json
import os

import numpy as np
import pytest

import xcheck
from conftest import GOLDEN, oracle_flags


@pytest.fixture(scope="module")
def committed():
    with open(os.path.join(GOLDEN, "xcheck_verdicts.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def sets(oracle_lib):
    return xcheck.datasets(lambda pk, sig, msg: oracle_flags(oracle_lib, pk, sig, msg))


def _lib(cls):
    try:
        return cls()
    except OSError as e:
        pytest.skip(str(e))


SET_NAMES = ("golden", "lattice_fallback", "reference_fixtures", "tx_golden", "c3_qc", "c3_tc", "random_2p15")


def test_committed_sets_are_the_generated_records(committed, sets):
    assert set(committed["sets"]) == set(SET_NAMES) == set(sets)
    for name, (pk, sig, msg, _) in sets.items():
        c = committed["sets"][name]
        assert c["n"] == pk.shape[0], name
        assert c["records_sha256"] == xcheck.records_digest(pk, sig, msg), name


@pytest.mark.parametrize("name", SET_NAMES)
def test_openssl_pins_the_batch_rule(committed, sets, name):
    ossl = _lib(xcheck.OpenSSL)
    pk, sig, msg, flags = sets[name]
    got = xcheck.run(ossl, pk, sig, msg)
    c = committed["sets"][name]
    assert (got == xcheck.unpack_verdicts(c["openssl"], len(got))).all(), name
    cls = xcheck.classify_all(flags, pk, sig, ossl=got)["openssl"]
    unclassified = [(i, x) for i, x in enumerate(cls) if x not in xcheck.OPENSSL_CLASSES and x != "agree"]
    assert not unclassified, (name, unclassified[:5])
    assert {str(i): x for i, x in enumerate(cls) if x != "agree"} == c["openssl_divergent"]


@pytest.mark.parametrize("name", SET_NAMES)
def test_libsodium_pins_the_strict_rule(committed, sets, name):
    sodium = _lib(xcheck.Sodium)
    pk, sig, msg, flags = sets[name]
    got = xcheck.run(sodium, pk, sig, msg)
    c = committed["sets"][name]
    assert (got == xcheck.unpack_verdicts(c["sodium"], len(got))).all(), name
    cls = xcheck.classify_all(flags, pk, sig, sodium=got)["sodium"]
    # no divergence at all is expected for the strict bit (both classes need an
    # infeasible vector: a non-canonical large-order point in a valid signature)
    assert all(x == "agree" for x in cls), (name, [(i, x) for i, x in enumerate(cls) if x != "agree"][:5])


def test_committed_columns_classify_without_the_libraries(committed, sets):
    """The columns pin the oracle's flags on any box (no libcrypto needed)."""
    seen = set()
    confirmed_batch_only = 0
    for name, (pk, sig, msg, flags) in sets.items():
        c = committed["sets"][name]
        vo = xcheck.unpack_verdicts(c["openssl"], len(flags))
        vs = xcheck.unpack_verdicts(c["sodium"], len(flags))
        cls = xcheck.classify_all(flags, pk, sig, vo, vs)
        for i, x in enumerate(cls["openssl"]):
            if x != "agree":
                assert x in xcheck.OPENSSL_CLASSES, (name, i, x)
                seen.add(x)
        assert all(x == "agree" for x in cls["sodium"]), name
        batch = (flags & (xcheck.PARSE_OK | xcheck.EQ_OK)) == (xcheck.PARSE_OK | xcheck.EQ_OK)
        strict = (flags & xcheck.STRICT_OK) != 0
        confirmed_batch_only += int((batch & ~strict & vo).sum())
    # both classes are reached by the edge catalogue (non-canonical small-order R)
    assert seen == xcheck.OPENSSL_CLASSES
    # small-order A or R with e = O -- strict rejects, batch
    # accepts -- confirmed by OpenSSL on every canonically encoded instance
    assert confirmed_batch_only >= 9


def test_divergent_records_are_small_order_R():
    """Each divergent record is a decodable, small-order, non-canonically encoded R
    (no large-order point can carry a valid equation under a non-canonical
    encoding without its discrete log)."""
    with open(os.path.join(GOLDEN, "xcheck_verdicts.json")) as f:
        div = json.load(f)["sets"]["golden"]["openssl_divergent"]
    with open(os.path.join(GOLDEN, "edge_vectors.json")) as f:
        edge = json.load(f)["vectors"]
    assert div
    for i, cls in div.items():
        v = edge[int(i)]
        assert v["flags"] & xcheck.SMALL_R and v["flags"] & xcheck.R_OK
        assert xcheck.r_encoding_class(bytes.fromhex(v["sig"])[:32]) == cls
        assert not v["flags"] & xcheck.STRICT_OK
