"""ISA-level checks of the persistent work loops (no GPU: hipcc -S only).

Round 1 hit a hang with strict bits enabled (commit 6e5c7e3): storing the
wave's ballot from lane 0 as two nested conditional stores made hipcc compile
the persistent point-pass loop as a DIVERGENT loop -- the back edge masks
exec (``s_andn2_b64 exec, exec, ...``) and the loop's exit mask is taken from
the exec left by the lane-0 region -- although its exit condition (the batch
base from lane 0's atomic, broadcast by readfirstlane) is wave-uniform.  A
wave of such a loop iterates while any lane has not "exited"; the base that
decides the exit comes from lane 0, so a wave whose remaining lanes exclude
lane 0 re-reads a stale base forever.

tools/repro_divergent_loop.hip keeps the two forms as a minimal reproducer;
here both are compiled and classified, and every product kernel whose work
loop takes batches from an atomic counter is checked to be uniform.  The GPU
side keeps a bits-enabled multi-round run (tests/test_c5.py: 2^22 + 4097
items, 21+ rounds of the persistent grid, with strict bits).
"""
import os
import re
import subprocess

import pytest

from conftest import PKG, ROOT

HIPCC = "/opt/rocm/bin/hipcc"
OUT = os.path.join(ROOT, "build", "isa")


def _compile(src, name, extra=()):
    os.makedirs(OUT, exist_ok=True)
    out = os.path.join(OUT, name)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-fno-slp-vectorize", "-std=c++17", "--cuda-device-only",
                    "-S", "-I", os.path.join(PKG, "csrc"), "-I", os.path.join(ROOT, "include"), *extra, src,
                    "-o", out], check=True, capture_output=True)
    return open(out).read().split("\n")


def _kernels(lines):
    """name -> instruction lines of each kernel body"""
    res = {}
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l)]
    for s in starts:
        e = next((i for i, l in enumerate(lines[s:]) if "s_endpgm" in l), None)
        if e is not None:  # kernels only (other _Z symbols are data)
            res[lines[s].split(":")[0]] = lines[s:s + e + 1]
    return res


def _block_loop(body):
    """per line: the Depth=1 loop header of the enclosing basic block (or None).
    A block's label line and the comment-only lines after it carry the loop
    comments: "This Loop Header: Depth=1", "in Loop: Header=BBx_y Depth=1" or,
    inside a nested loop, "Parent Loop BBx_y Depth=1"."""
    cur, res = None, []
    i = 0
    while i < len(body):
        l = body[i]
        if l.startswith(".LBB") or l.startswith("; %bb"):
            label = l.split(":")[0]
            text = l
            j = i + 1
            while j < len(body) and re.match(r"^\s+;", body[j]):
                text += body[j]
                j += 1
            m = re.search(r"(?:Header=|Parent Loop )(BB\d+_\d+) Depth=1", text)
            if "This Loop Header: Depth=1" in text:
                cur = "BB" + label.split("BB")[-1]
            elif m:
                cur = m.group(1)
            else:
                cur = None
        res.append(cur)
        i += 1
    return res


def work_loops(body):
    """{header: divergent?} for the Depth=1 loops that contain an atomic add"""
    loops = _block_loop(body)
    headers = {loops[i] for i, l in enumerate(body) if "global_atomic_add" in l and loops[i]}
    res = {}
    for h in headers:
        res[h] = any(loops[i] == h and re.match(r"^\s*s_andn2_b64\s+exec,\s*exec,", l) for i, l in enumerate(body))
    return res


@pytest.fixture(scope="module")
def hipcc():
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    return HIPCC


def test_reproducer_double_store_loop_is_divergent(hipcc):
    """The two store forms of tools/repro_divergent_loop.hip compile to a
    divergent and a uniform work loop respectively (the compiler behaviour
    behind the round-1 hang)."""
    ks = _kernels(_compile(os.path.join(ROOT, "tools", "repro_divergent_loop.hip"), "repro.s"))
    dbl = next(v for k, v in ks.items() if "k_double" in k)
    pair = next(v for k, v in ks.items() if "k_pair" in k)
    wd, wp = work_loops(dbl), work_loops(pair)
    assert len(wd) == 1 and len(wp) == 1, (wd, wp)
    assert list(wd.values()) == [True], "lane-0 double store: expected an exec-masked (divergent) work loop"
    assert list(wp.values()) == [False], "lanes-0/1 store: expected a uniform work loop"


@pytest.mark.parametrize("src", ["hsv_kernels.hip", "hsv_committee.hip", "hsv_mempool.hip"])
def test_product_work_loops_are_uniform(hipcc, src):
    """Every product kernel that deals batches from an atomic counter keeps its
    work loop uniform (no exec-masked back edge)."""
    ks = _kernels(_compile(os.path.join(PKG, "csrc", src), src + ".s", []))
    assert ks, "no kernels found"
    for name, body in ks.items():
        for h, divergent in work_loops(body).items():
            assert not divergent, f"{name}: work loop {h} compiled as a divergent loop"
    if src == "hsv_kernels.hip":
        assert any("hsv_verify_hp_kernel" in k and work_loops(v) for k, v in ks.items()), "point pass loop not found"


def test_fused_transaction_launch_hands_off_write_through(hipcc):
    """The fused transaction launch (hsv_verify_fused... in hsv_mempool.hip,
    DESIGN.md 4b) hands records from the waves that build them to other
    workgroups of the same launch.  Per-XCD L2s are not coherent, so in the
    record phase (between s_setprio 3 and s_setprio 0) every global or buffer
    store must be write-through (sc1) -- scratch spills are the lane's own --
    each record batch must be published by an atomic after an
    s_waitcnt vmcnt(0), and the point phase must acquire (buffer_inv sc1)."""
    ks = _kernels(_compile(os.path.join(PKG, "csrc", "hsv_mempool.hip"), "hsv_mempool_handoff.s", []))
    fused = [(k, v) for k, v in ks.items() if "fused_kernel" in k]
    assert fused, "fused transaction kernel not found"
    for name, body in fused:
        start = next(i for i, l in enumerate(body) if "s_setprio 3" in l)
        end = next(i for i, l in enumerate(body) if "s_setprio 0" in l and i > start)
        stores = [l.strip() for l in body[start:end] if re.search(r"\b(global|buffer|flat)_store", l)]
        assert stores and all(" sc1" in l for l in stores), [l for l in stores if " sc1" not in l][:4]
        assert any("buffer_store_dwordx4" in l for l in stores), "records not stored 16 B at a time"
        atomics = [i for i in range(start, end) if re.search(r"global_atomic_add\b", body[i])]
        waits = [i for i in range(start, end) if re.match(r"\s*s_waitcnt vmcnt\(0\)", body[i])]
        assert any(w < a for a in atomics for w in waits), "no drain before a publishing atomic"
        assert any("buffer_inv sc1" in l for l in body[end:]), "the point phase never acquires"
