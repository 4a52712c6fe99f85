"""The kernel's per-lane arithmetic, compiled for the host, against the oracle.

tests/native/core_host.cpp includes the same csrc/hsv_*.hpp headers the gfx950
kernel is built from and runs them with g++ (test infrastructure; the product
library never verifies on the CPU).  This pins field / scalar / SHA-512 /
window-geometry logic in this GPU-less container before a GPU run.
"""
import os
import random
import subprocess

import numpy as np
import pytest

import ed25519_ref as o
from conftest import PKG, ROOT

BIN = os.path.join(ROOT, "build", "core_host")


def _build(out, *defines):
    os.makedirs(os.path.dirname(out), exist_ok=True)
    src = os.path.join(ROOT, "tests", "native", "core_host.cpp")
    tmp = f"{out}.{os.getpid()}.tmp"  # parallel test workers build side by side
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wno-unknown-pragmas", *defines,
                    "-I", os.path.join(PKG, "csrc"), src, "-o", tmp], check=True)
    os.replace(tmp, out)
    return out


@pytest.fixture(scope="module")
def core_host():
    return _build(BIN)


@pytest.fixture(scope="module")
def core_host_checked():
    """-DHSV_CHECK_BOUNDS: every field multiply asserts its operand classes and
    that all 64-bit column sums are exact (checked in 128-bit arithmetic)."""
    return _build(BIN + "_checked", "-DHSV_CHECK_BOUNDS")


def _run(binary, args, lines):
    r = subprocess.run([binary] + args, input="\n".join(lines) + "\n", capture_output=True, text=True, check=True)
    return r.stdout.split()


def test_field_ops_match_python(core_host_checked):
    core_host = core_host_checked
    rnd = random.Random(5)
    lines, exp = [], []
    # operands enter through fe_from_words_masked (bit 255 dropped), so the domain is [0, 2^255)
    specials = [0, 1, 2, o.P - 1, o.P, o.P + 1, 2**255 - 1, 2**255 - 20, 19, 38, 2**26 - 1, 2**51]
    vals = specials + [rnd.randrange(2**255) for _ in range(120)]
    for a in vals:
        b = vals[rnd.randrange(len(vals))]
        for op, v in (("mul", a * b), ("sq", a * a), ("add", a + b), ("sub", a - b), ("canon", a)):
            lines.append(f"{op} {a:064x} {b:064x}")
            exp.append(v % o.P)
        lines.append(f"pow {a:064x} {b:064x}")
        exp.append(pow(a, (o.P - 5) // 8, o.P))
        if a % o.P:
            lines.append(f"inv {a:064x} {b:064x}")
            exp.append(pow(a, o.P - 2, o.P))
    got = _run(core_host, ["--field"], lines)
    bad = [lines[i] for i in range(len(exp)) if int(got[i], 16) != exp[i]]
    assert not bad, bad[:5]


def test_challenge_scalar_matches_python(core_host):
    rnd = random.Random(6)
    lines, exp = [], []
    for _ in range(200):
        r, a, m = rnd.randbytes(32), rnd.randbytes(32), rnd.randbytes(32)
        lines.append(f"{r.hex()} {a.hex()} {m.hex()}")
        exp.append(o.scalar_from_hash(o.sha512(r + a + m)))
    # extreme hashes are covered by construction of Barrett; also all-ones inputs
    lines.append(f"{'ff'*32} {'ff'*32} {'ff'*32}")
    exp.append(o.scalar_from_hash(o.sha512(b"\xff" * 96)))
    got = _run(core_host, ["--hashk"], lines)
    assert [int(g, 16) for g in got] == exp


@pytest.fixture(scope="module")
def core_host32():
    """The alternative radix-2^32 field representation (HSV_FE_RADIX=32)."""
    return _build(BIN + "32", "-DHSV_FE_RADIX=32", "-I", os.path.join(ROOT, "tests", "native"))


@pytest.mark.parametrize("variant", [0, 1, 10, 11, 12, 14, 16, 18, 20, 21])
def test_operand_bounds_hold_on_edge_and_sample(core_host_checked, golden, variant):
    """Bound-checked build over every edge vector and a random sample: no field
    operand leaves its class and no 64-bit column sum overflows."""
    idx = list(range(golden["n_edge"])) + list(range(golden["n_edge"], len(golden["flags"]), 7))
    lines = [f"{bytes(golden['pk'][i]).hex()} {bytes(golden['sig'][i]).hex()} {bytes(golden['msg'][i]).hex()}"
             for i in idx]
    got = np.array([int(x, 16) for x in _run(core_host_checked, ["--variant", str(variant)], lines)], np.uint8)
    assert (got == golden["flags"][idx]).all()


def test_radix32_field_matches_golden(core_host32, golden):
    lines = [f"{bytes(p).hex()} {bytes(s).hex()} {bytes(m).hex()}"
             for p, s, m in zip(golden["pk"], golden["sig"], golden["msg"])]
    got = np.array([int(x, 16) for x in _run(core_host32, ["--variant", "0"], lines)], np.uint8)
    assert (got == golden["flags"]).all()


@pytest.mark.parametrize("variant", [0, 1, 2, 4, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21])
def test_verify_core_all_geometries_match_golden(core_host, golden, variant):
    lines = [f"{bytes(p).hex()} {bytes(s).hex()} {bytes(m).hex()}"
             for p, s, m in zip(golden["pk"], golden["sig"], golden["msg"])]
    got = np.array([int(x, 16) for x in _run(core_host, ["--variant", str(variant)], lines)], np.uint8)
    bad = np.nonzero(got != golden["flags"])[0]
    assert bad.size == 0, [golden["cases"][i] for i in bad[:10]]


def test_committee_comb_path_matches_golden(core_host, golden):
    """Committee key cache (hsv_comb.hpp) built and verified on the host: every
    distinct golden key becomes a member (undecodable, small-order, mixed-order
    and non-canonical keys included); flags equal the generic path's."""
    idx = list(range(golden["n_edge"])) + list(range(golden["n_edge"], len(golden["flags"]), 25))
    keys = sorted({bytes(golden["pk"][i]).hex() for i in idx})
    kidx = {k: n for n, k in enumerate(keys)}
    lines = [str(len(keys))] + keys + [
        f"{kidx[bytes(golden['pk'][i]).hex()]} {bytes(golden['sig'][i]).hex()} {bytes(golden['msg'][i]).hex()}"
        for i in idx]
    got = np.array([int(x, 16) for x in _run(core_host, ["--comb"], lines)], np.uint8)
    bad = np.nonzero(got != golden["flags"][idx])[0]
    assert bad.size == 0, [golden["cases"][idx[i]] for i in bad[:10]]


@pytest.mark.parametrize("bits", [133, 138])
def test_lattice_reduction_properties(core_host, bits):
    """hsv_lattice.hpp: for challenges k < l the reduced pair satisfies
    c0 == c1 k (mod 8l), c1 odd and 0 < c1, |c0| < 2^bits (ok == 1), or reports
    ok == 0 (the kernel then takes the full-length path).  Includes k = 0, 1,
    l - 1, small and structured values.  133 is the register-table variants'
    bound, 138 the comb path's (kLatCombBits)."""
    rnd = random.Random(11)
    N = 8 * o.L
    ks = [0, 1, 2, 3, 8, o.L - 1, o.L - 2, 2**128, 2**128 - 1, 2**127 + 1, 2**252, (o.L - 1) // 2,
          (o.L + 1) // 2, (o.L - 1) // 3, 2**200 + 12345]
    ks += [rnd.randrange(o.L) for _ in range(3000)]
    got = _run(core_host, ["--lattice", str(bits)], [f"{k:064x}" for k in ks])
    assert len(got) == 4 * len(ks)
    n_ok = 0
    for i, k in enumerate(ks):
        ok, neg, c0, c1 = int(got[4 * i]), int(got[4 * i + 1]), int(got[4 * i + 2], 16), int(got[4 * i + 3], 16)
        if not ok:
            continue
        n_ok += 1
        c0s = -c0 if neg else c0
        assert c1 % 2 == 1 and 0 < c1 < 2**bits and c0 < 2**bits, k
        assert (c0s - c1 * k) % N == 0, k
    # the structured k (l - 1, 2^252, (l - 1) / 2 ...) have a tiny shortest vector
    # with an even cofactor: no short odd partner at any bound
    assert n_ok >= len(ks) - 8
    if bits == 138:
        assert all(int(got[4 * i]) for i in range(15, len(ks))), "a random challenge fell back at 138 bits"


@pytest.mark.parametrize("rcp_err", [None, "3e-6", "-3e-6"])
def test_lean_lehmer_equals_round1_lehmer(core_host, rcp_err):
    """The default reduction (lat_lehmer_lean_to_128: magnitude cofactors, the
    crossing step taken inside a round) stops at the same Euclid state as the
    round-1 form (-DHSV_LATTICE_LEHMER1), so every output is identical.  The
    rcp_err builds give the quotient estimate a relative error, as the device's
    hardware reciprocal does: the exactness checks must absorb it."""
    defs = [f"-DHSV_LAT_HOST_RCP_ERR=({rcp_err})"] if rcp_err else []
    tag = "" if rcp_err is None else ("_p" if rcp_err[0] != "-" else "_m")
    lean = _build(BIN + "_lean" + tag, *defs) if defs else core_host
    old = _build(BIN + "_lehmer1", "-DHSV_LATTICE_LEHMER1")
    rnd = random.Random(21)
    N = 8 * o.L
    ks = [0, 1, 2, 7, 8, o.L - 1, 2**128 - 1, 2**128, 2**128 + 1, 2**129, 2**252, 2**31 + 5]
    ks += [(N // d) % o.L for d in range(1, 120)] + [(N // d + 1) % o.L for d in range(1, 120)]
    ks += [(N >> e) for e in (30, 31, 40, 50, 60, 100)] + [2**e % o.L for e in range(0, 253, 3)]
    ks += [rnd.randrange(o.L) for _ in range(20000)]
    lines = [f"{k:064x}" for k in ks]
    for bits in ("138", "133"):
        assert _run(lean, ["--lattice", bits], lines) == _run(old, ["--lattice", bits], lines)


def test_lattice_comb_bound_accepts_fixture_challenges(core_host, fallback_records):
    """The challenges of tests/golden/lattice_fallback.bin have no pair below
    2^133 but all have one below the comb path's 2^138 (kLatCombBits): at the
    default bound none of them takes the full-length path."""
    fb = fallback_records
    ks = sorted({o.scalar_from_hash(o.sha512(bytes(s[:32]) + bytes(p) + bytes(m)))
                 for p, s, m in zip(fb["pk"], fb["sig"], fb["msg"])})
    got = _run(core_host, ["--lattice", "138"], [f"{k:064x}" for k in ks])
    oks = [int(got[4 * i]) for i in range(len(ks))]
    assert sum(oks) == len(ks), "a fixture challenge still falls back at 138 bits"
    got133 = _run(core_host, ["--lattice", "133"], [f"{k:064x}" for k in ks])
    assert sum(int(got133[4 * i]) for i in range(len(ks))) <= len(ks) - 24


@pytest.mark.parametrize("variant", [16, 17, 20, 21])
@pytest.mark.parametrize("bits", [133, 138])
def test_lattice_fallback_records(core_host, fallback_records, variant, bits):
    """Records built on challenges the lattice reduction rejects at 133 bits:
    under that bound the half-size path hands them to the full-length path
    (reported on stderr); at the comb path's default 138 they stay on the
    half-size path.  The flags equal the oracle's either way."""
    fb = fallback_records
    lines = [f"{bytes(p).hex()} {bytes(s).hex()} {bytes(m).hex()}" for p, s, m in zip(fb["pk"], fb["sig"], fb["msg"])]
    r = subprocess.run([core_host, "--variant", str(variant)], input="\n".join(lines) + "\n",
                       capture_output=True, text=True, check=True, env=dict(os.environ, HSV_LAT_BITS=str(bits)))
    got = np.array([int(x, 16) for x in r.stdout.split()], np.uint8)
    assert (got == fb["flags"]).all()
    if bits == 133:
        # 24 challenges x (honest, flipped s, s + l) keep k; the mixed-order key changes it
        assert r.stderr.count("fallback") >= 48
    else:
        assert r.stderr.count("fallback") == 0


def test_transaction_record_matches_hashlib(core_host):
    """Mempool transaction records (csrc/hsv_txhash.hpp):
    pk || sig || SHA-512(message)[..32] for tx = message || pk || sig
    (mempool/src/batch_maker.rs:79-85), over every SHA-512 padding boundary
    and every start alignment within a 16-byte chunk."""
    import hashlib
    rnd = random.Random(8)
    mlens = [0, 1, 7, 8, 9, 15, 16, 17, 63, 64, 110, 111, 112, 113, 127, 128, 129, 200, 238, 239, 240,
             241, 255, 256, 257, 416, 1000, 2048 + 5]
    lines, exp = [], []
    for mlen in mlens:
        for sh in (0, 1, 2, 3, 4, 5, 7, 8, 11, 12, 13, 15):
            tx = rnd.randbytes(mlen + 96)
            lines.append(f"{sh} {tx.hex()}")
            msg, pk, sig = tx[:mlen], tx[mlen:mlen + 32], tx[mlen + 32:]
            exp.append((pk + sig + hashlib.sha512(msg).digest()[:32]).hex())
    got = _run(core_host, ["--txrec"], lines)
    bad = [(lines[i][:12], len(lines[i])) for i in range(len(exp)) if got[i] != exp[i]]
    assert not bad, bad[:5]


def test_degenerate_accumulator_fails_closed(core_host):
    """(0 : 0 : 0 : 0) -- what an accumulator becomes when its table entries
    read back as zeros -- satisfies X == 0, Y == Z and X == xZ, Y == yZ; the
    final checks (ge_is_neutral, ge_eq_affine) also require Z != 0, so it is
    rejected, while the neutral point itself still compares equal."""
    assert _run(core_host, ["--degenerate"], []) == ["0", "0", "1", "1"]


def test_sanity_check_separates_points_from_corruption(core_host):
    """ge_is_sane, the device self-check on every final accumulator: curve
    points with Z != 0 pass (identity, B, [2^10]B); (0 : 0 : 0 : 0), an
    off-curve X and Z = 0 fail."""
    assert _run(core_host, ["--sanity"], []) == ["1", "0", "1", "0", "1", "0"]


@pytest.mark.parametrize("mode", [1, 3])
def test_injected_table_corruption_is_a_fault_not_a_verdict(core_host, golden, mode):
    """The kernel's fault injection (zeroed / bit-flipped table entries between
    the table build and the window loop) replayed on the host-built two-pass
    path: every record whose points decode reports the fault (the host turns
    it into HSV_ERR_DEVICE_FAULT); records whose A or R does not decode keep
    their flags (their verdict never depends on the equation)."""
    idx = list(range(golden["n_edge"])) + list(range(golden["n_edge"], len(golden["flags"]), 5))
    lines = [f"{bytes(golden['pk'][i]).hex()} {bytes(golden['sig'][i]).hex()} {bytes(golden['msg'][i]).hex()}"
             for i in idx]
    got = _run(core_host, ["--inject", str(mode)], lines)
    for i, g in zip(idx, got):
        f = int(golden["flags"][i])
        decoded = (f & o.A_OK) and (f & o.R_OK)
        if decoded:
            assert g == "fault", golden["cases"][i]
        else:
            assert int(g, 16) == f, golden["cases"][i]


@pytest.mark.parametrize("mode", [1, 3])
def test_injected_committee_table_corruption_is_a_fault(core_host, golden, mode):
    """Same for the committee kernels' key tables (verify_one_comb)."""
    idx = list(range(golden["n_edge"]))
    keys = sorted({bytes(golden["pk"][i]).hex() for i in idx})
    kidx = {k: n for n, k in enumerate(keys)}
    lines = [str(len(keys))] + keys + [
        f"{kidx[bytes(golden['pk'][i]).hex()]} {bytes(golden['sig'][i]).hex()} {bytes(golden['msg'][i]).hex()}"
        for i in idx]
    got = _run(core_host, ["--comb", str(mode)], lines)
    for i, g in zip(idx, got):
        f = int(golden["flags"][i])
        if (f & o.A_OK) and (f & o.R_OK):
            assert g == "fault", golden["cases"][i]
        else:
            assert int(g, 16) == f, golden["cases"][i]
