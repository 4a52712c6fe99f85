#!/usr/bin/env python3
"""Benchmark: Ed25519 verifications/s at batch 2^20 per GPU (BASELINE.json metric).

python bench.py [--gpus N] [--steps K] [--warmup W] [--n ITEMS_PER_GPU] [--global-n ITEMS]

One process per GPU.  Launched under torch.distributed.run (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* in the environment), every rank runs its shard.  Run
directly with --gpus N > 1 and no WORLD_SIZE, this script starts
`python -m torch.distributed.run --nproc-per-node N` itself (the parent never
touches a GPU) and exits with its status; WORLD_SIZE != N is an error.

Workload (config C4 / C5 shards): each rank holds n = 2^20 independent
(public key, 32-byte digest, signature) triples in HBM, 5 % corrupted across
the SURVEY 8(d) corruption kinds.  A step is one verification launch over the
rank's whole batch (per-item flag bytes + packed STRICT_OK bits); consecutive
steps alternate over --streams (default 3) HIP streams with their own outputs,
so one batch's launch starts in the previous one's grid end.  Shards are
contiguous and independent: no collective touches the data path; the gloo
group only carries the timing barrier, the max-over-ranks reduction and the
final bitmask gather.  --global-n 16777216 runs C5 (2^24 split over the ranks,
strong scaling).  --dry-run exercises the launcher, sharding, timing and
gather on CPU (gloo, no GPU, no verification) for tests/test_bench_launcher.py.

Reported beside it:
  roofline         int32-VALU bound; achieved = 192,000 u32 MACs per verification
                   (SURVEY 8(d) convention) x items per launch / GPU time per step
                   from HIP events around the timed steps; isolated_launch_ms is
                   one launch alone on one stream (what rocprofv3 reports per
                   kernel pair); per rank with --global-n.
  cpu_baseline     rank 0, N = 1 only: the C restatement of ed25519-dalek's
                   verify_strict (oracle/ed25519_oracle.c, "port") on every host
                   core this job may use, over the full C4 batch, flag-for-flag
                   against the GPU; plus the batch way (verify_batch over chunks
                   of 64, verify_strict for failing chunks).
  qc_latency*      p50/p99 of the host-buffer QC call (C1/C2/C3), of one
                   verify_strict, of the C3 QC from bincode, and of C3 with 5 %
                   corrupted votes; C1 and C3 again paced 1 ms apart
                   (idle_gap_1ms, as consensus issues them).
  tc_latency       C3 TC (667 timeouts, per-vote digests) through the batched
                   strict API and from bincode, 0 % and 5 % corrupted.
  tc_dropin_sequential  C3 TC the way the unchanged caller verifies it: 667
                   sequential hsv_verify_strict calls (TC::verify's loop).
                   Single verifies and QCs of <= 4 cached-key votes take the
                   library's default route: the resident latency service.
  launched         a child process with HSV_QC_RESIDENT=0: one verify_strict, a
                   C1 QC and the sequential TC loop launched per call (the
                   service off), with the dalek port's single verify in the same
                   process.
  qc_cpu_baseline  one host core: the C port of dalek verify_batch (Straus /
                   Pippenger MSM) for C1-C3 QCs and the sequential TC::verify loop.
  mempool_tx       2^20 client transactions of 512 B in HBM.

Each rank binds its threads to its GPU's NUMA node before any measurement
(pin_to_gpu_node; the CPU baselines run on all the host's CPUs): calls from
the other socket of a two-socket host measured up to 9 us slower
(profiles/r05ac_numa.txt).

stdout carries ONE compact JSON line (< 4 KB: the C4 line, roofline,
cpu_baseline, and a `latency` object with every GPU latency next to the CPU
port's); the full record (every rep's phases and tails) goes to --detail.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hotstuff-digital-signature-benchmarking_amd"))

WORK_MACS = 192_000          # u32 MACs per verification
IO_BYTES = 129               # algorithmic HBM bytes per verification (128 in + 1 out)
# int32 VALU peak: 256 CUs x 4 SIMDs x 16 lanes/clk (v_mad_u64_u32 issues at
# half the f32 rate on gfx950, profiles/r01e_ubench) x 2.4 GHz max clock
# (MI355X_MICROARCH.md chip table) = 39.3 T MAC/s
PEAK_MACS = 256 * 4 * 16 * 2.4e9
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "latest_pmc_traffic.json")
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libhsv_oracle.so")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(variant, n):
    """HBM bytes per launch from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes (tools/pmc_traffic.sh), when they were taken on this kernel variant
    and batch size; gfx950 correction: FETCH_SIZE counts half the bytes of
    16-byte-per-lane reads (MI355X_MICROARCH.md), so it is doubled."""
    try:
        with open(PMC_TRAFFIC) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None
    # variant 21 runs variant 19's kernels above 2^13 items (its pair form is for small batches)
    same = {variant, 19} if (variant == 21 and n > (1 << 13)) else {variant}
    if t.get("variant") not in same or t.get("n") != n:
        return None, None
    return 2 * t["fetch_bytes_per_launch"] + t["write_bytes_per_launch"], t.get("source")


def host_cores():
    """CPU threads this job may use: the affinity mask, capped by a cgroup v2
    CPU quota (a GPU box grants each job a share of a larger machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(p)
            n = min(n, max(1, int(quota)))
    except (OSError, ValueError):
        pass
    return n, quota


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _oracle():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-s"], cwd=os.path.join(ROOT, "oracle"), check=True)
    lib = ctypes.CDLL(ORACLE_SO)
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.oracle_verify_many.argtypes = [vp, vp, vp, sz, sz, vp, ctypes.c_int]
    lib.oracle_verify_many_batch64.restype = ctypes.c_uint64
    lib.oracle_verify_many_batch64.argtypes = [vp, vp, vp, sz, vp, ctypes.c_int]
    lib.oracle_verify_batch_dalek.argtypes = [ctypes.c_char_p, vp, vp, sz, ctypes.c_uint64]
    lib.oracle_verify_batch.argtypes = [ctypes.c_char_p, vp, vp, sz]
    lib.oracle_tc_verify.argtypes = [vp, vp, vp, sz]
    lib.oracle_verify_flags.restype = ctypes.c_uint8
    lib.oracle_verify_flags.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, sz]
    lib.oracle_verify_tx_many.argtypes = [vp, vp, sz, sz, vp, ctypes.c_int]
    return lib


def dalek_probe():
    """BASELINE.md asks for ed25519-dalek itself as the CPU baseline when the
    GPU box can build it: record whether cargo / rustc and an offline crate
    registry exist here.  (They never have: the baseline is then the C port.)"""
    import shutil
    res = {"cargo": shutil.which("cargo"), "rustc": shutil.which("rustc")}
    for tool in ("cargo", "rustc"):
        if res[tool]:
            try:
                res[f"{tool}_version"] = subprocess.run([tool, "--version"], capture_output=True, text=True,
                                                        timeout=30).stdout.strip()
            except (OSError, subprocess.SubprocessError) as e:
                res[f"{tool}_version"] = f"error: {e}"
    home = os.environ.get("CARGO_HOME", os.path.expanduser("~/.cargo"))
    reg = os.path.join(home, "registry")
    res["registry"] = reg if os.path.isdir(reg) else None
    res["ed25519_dalek_in_registry"] = bool(res["registry"]) and any(
        "ed25519-dalek" in d for _, dirs, _ in os.walk(reg) for d in dirs)
    res["dalek_buildable"] = bool(res["cargo"] and res["ed25519_dalek_in_registry"])
    res["consequence"] = ("dalek buildable: not wired in this round" if res["dalek_buildable"] else
                          "no cargo / no offline ed25519-dalek crate on this box: the baseline is the C port "
                          "(oracle/ed25519_oracle.c), kind 'port'")
    return res


def cpu_baseline(w, gpu_flags, sample):
    """C4 on the host cores: the C port of dalek's verify_strict per item (the
    reference's Signature::verify, which gives the per-signature vector), and
    the batch way (verify_batch over chunks of 64 + verify_strict for chunks
    that fail).  Rank 0, N = 1 only, outside the timed region."""
    lib = _oracle()
    threads, quota = host_cores()
    m = min(sample, w.n)
    pk, sig, msg = (np.ascontiguousarray(a[:m]) for a in (w.pk, w.sig, w.msg))
    out = np.zeros(m, np.uint8)
    t0 = time.perf_counter()
    lib.oracle_verify_many(pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, 32, m, out.ctypes.data, threads)
    dt = time.perf_counter() - t0
    out64 = np.zeros(m, np.uint8)
    t0 = time.perf_counter()
    fb = lib.oracle_verify_many_batch64(pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, m, out64.ctypes.data,
                                        threads)
    dt64 = time.perf_counter() - t0
    # dalek's verify_batch draws random z_i: a chunk whose only failures are
    # pure torsion terms (a mixed-order key with k != 0 mod 8) is accepted with
    # some probability, so its items then read as accepted.  Any
    # other disagreement would be a bug; report which kinds disagree.
    miss = np.nonzero((out64 & 1) != (gpu_flags[:m] & 1))[0]
    from hsverify import synth
    miss_kinds = sorted({synth.CORRUPTIONS[k] if k >= 0 else "honest" for k in w.kind[miss]})
    return {
        "value": m / dt, "unit": "verif/s", "cores": threads, "kind": "port",
        "sample": f"first {m} triples of the same C4 workload (5 % corrupted); oracle/ed25519_oracle.c "
                  f"(C restatement of ed25519-dalek 1.0.1 verify_strict: radix-2^51 field, width-5/8 NAF "
                  f"double-scalar multiplication), {threads} threads, {dt:.2f} s wall",
        "sample_parity_vs_gpu": bool((out == gpu_flags[:m]).all()),
        "nproc": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": quota,
        "cpu_model": cpu_model(), "dalek_probe": dalek_probe(),
        "batch64": {"value": m / dt64, "unit": "verif/s", "cores": threads,
                    "algorithm": "dalek verify_batch (random linear combination, Straus MSM) over chunks of 64, "
                                 "verify_strict per item for the chunks that fail",
                    "failed_chunks": int(fb), "chunks": (m + 63) // 64,
                    "strict_ok_parity_vs_gpu": bool(miss.size == 0),
                    "strict_ok_mismatches": int(miss.size), "mismatch_kinds": miss_kinds,
                    "mismatch_note": "dalek verify_batch is randomised when a chunk's only failures are pure "
                                     "torsion (mixed-order key, k != 0 mod 8): such chunks may pass; the "
                                     "per-signature vector is verify_strict's (SURVEY A.2)"},
    }


def _p(ts):
    ts = np.array(ts) * 1e3
    return {"p50_ms": float(np.percentile(ts, 50)), "p99_ms": float(np.percentile(ts, 99)),
            "p999_ms": float(np.percentile(ts, 99.9)), "max_ms": float(ts.max()), "reps": len(ts)}


def _timed(fn, reps, warm=10):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return ts


def _timed_gap(fn, reps, gap_us, warm=5):
    """p50 / p99 of fn with gap_us of host busy-wait before every call: a
    consensus node verifies a QC every few milliseconds, not back to back, and
    an idle GPU takes ~5 us longer for the next launch (profiles/r05an_gap.txt)."""
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t_end = time.perf_counter() + gap_us * 1e-6
        while time.perf_counter() < t_end:
            pass
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return {"p50_ms": float(np.median(ts) * 1e3), "p99_ms": float(np.percentile(ts, 99) * 1e3), "reps": reps,
            "gap_us": gap_us}


MARKS = ("lookup", "slot", "staged", "launch", "sync", "done")  # hsv.h HSV_MARK_*


def _timed_lib(fn, reps, warm=10):
    """Latency of a libhsv call, with its attribution (round-3 VERDICT item 3).

    Every rep keeps its wall time and the library's host timeline of that call
    (hsv_host_call_marks: cache lookup, slot lease, staging, launch enqueue,
    stream synchronisation, exit; ms from the library's entry).  Python's
    cyclic garbage collector is paused while the reps run: the reference's
    callers are Rust and have no collector, and a gen-2 collection of this
    process (torch loaded) would land in a rep as a pause of its own.  The
    reps above p99 are returned with their phases next to the median rep's."""
    import ctypes
    import gc
    from hsverify import _lib
    lib = _lib.load()
    buf = (ctypes.c_double * 8)()
    gc.collect()  # before the warm-up: a collection between warm-up and reps left the first rep cold
    for _ in range(warm):
        fn()
    was = gc.isenabled()
    gc.disable()
    ts, marks = [], []
    try:
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
            n = lib.hsv_host_call_marks(buf, 8)
            marks.append([buf[i] for i in range(min(n, len(MARKS)))] if n == len(MARKS) else None)
    finally:
        if was:
            gc.enable()
    out = _p(ts)
    wall = np.array(ts) * 1e3
    if all(m is not None for m in marks):
        m = np.array(marks)                                   # (reps, 6), -1: mark not passed
        step = np.diff(np.concatenate([np.zeros((len(m), 1)), np.maximum(m, 0)], axis=1), axis=1)
        step[m < 0] = 0.0                                     # per-phase ms (a skipped phase is 0)
        lib_ms = m[:, -1]
        phases = lambda rows: {k: round(float(np.median(step[rows, j])), 4) for j, k in enumerate(MARKS)}
        cut = np.percentile(wall, 99)
        tail = np.nonzero(wall > cut)[0]
        out["lib_p50_ms"] = float(np.median(lib_ms))
        out["lib_p99_ms"] = float(np.percentile(lib_ms, 99))
        out["median_phases_ms"] = phases(np.arange(len(m)))
        out["tail"] = {
            "reps_above_p99": int(len(tail)),
            "phases_ms": phases(tail) if len(tail) else {},
            "outside_lib_ms": round(float(np.median(wall[tail] - lib_ms[tail])), 4) if len(tail) else None,
            "rep_index": tail.tolist()[:16],
            "wall_ms": [round(float(x), 4) for x in wall[tail][:16]],
        }
        out["outside_lib_p50_ms"] = round(float(np.median(wall - lib_ms)), 4)
    return out


def member_corrupted(make, committee, seed, frac=0.05):
    """A C3 certificate with `frac` corrupted votes whose keys all stay committee
    members: the reference rejects a vote by a non-member before any signature
    check (QC::verify / TC::verify stake lookups, consensus/src/messages.rs:186,296),
    so the kinds that swap the key (small-order and mixed-order A) are reverted
    to honest votes."""
    from hsverify import synth
    w = make(committee, seed=seed, corrupt_frac=frac)
    clean = make(committee, seed=seed)
    swap = np.isin(w.kind, [synth.CORRUPTIONS.index(k) for k in synth.KEY_KINDS])
    w.pk[swap], w.sig[swap] = clean.pk[swap], clean.sig[swap]
    w.honest[swap] = True
    w.accept[swap] = True
    return w


def tc_hqc(committee, seed, round_=1000):
    quorum = 2 * committee // 3 + 1
    return np.random.default_rng(seed + 29).integers(round_ - 10, round_, size=quorum)


def qc_latency(reps, auto=True):
    """auto: the drop-in default, hsv_verify_batch_packed with its automatic
    committee cache in steady state (the same keys every round, as consensus
    has); auto=False: the generic kernels only."""
    from hsverify import _lib, synth, wire
    import hashlib
    lib = _lib.load()
    lib.hsv_set_auto_committee(1 if auto else 0)
    res = {"automatic_committee_cache": bool(auto)}

    def settle(fn):  # two sightings queue the keys; wait for the background build
        for _ in range(3):
            fn()
        lib.hsv_auto_committee_wait(60000)

    gaps = {}
    for committee in (4, 100, 1000):
        w = synth.qc_votes(committee, seed=committee)
        packed = np.concatenate([w.pk, w.sig], axis=1).tobytes()
        digest = bytes(w.msg)
        call = lambda: lib.hsv_verify_batch_packed(digest, packed, w.n)
        settle(call)
        assert call() == 1
        res[f"n{committee}_votes{w.n}"] = _timed_lib(call, reps)
        if auto and committee != 100:  # the same calls 1 ms apart, as consensus issues them
            gaps[f"n{committee}_votes{w.n}"] = _timed_gap(call, min(reps, 200), 1000)
    # C3 with 5 % corrupted votes (member keys): Err, every flag computed
    w = member_corrupted(synth.qc_votes, 1000, seed=1000)
    packed = np.concatenate([w.pk, w.sig], axis=1).tobytes()
    digest = bytes(w.msg)
    call = lambda: lib.hsv_verify_batch_packed(digest, packed, w.n)
    settle(call)
    assert call() == 0
    res["n1000_votes667_corrupt5pct"] = dict(_timed_lib(call, reps), corrupted=int((~w.accept).sum()))
    # one strict verification (Vote::verify / Block::verify, consensus/src/messages.rs:136-146)
    w = synth.qc_votes(4, seed=4)
    pk0, sig0, d0 = bytes(w.pk[0]), bytes(w.sig[0]), bytes(w.msg)
    settle(lambda: lib.hsv_verify_batch_packed(d0, np.concatenate([w.pk, w.sig], 1).tobytes(), w.n))
    call = lambda: lib.hsv_verify_strict(d0, pk0, sig0)
    assert call() == 1
    res["single_verify_strict"] = _timed_lib(call, reps)
    res["single_verify_strict"]["route"] = call_route()
    if auto:
        gaps["single"] = _timed_gap(call, min(reps, 200), 1000)
    # the C3 QC handed over as its bincode wire bytes (hsv_qc_verify_bincode:
    # parse + base64 keys + qc.digest() on the host, verification on the GPU)
    w = synth.qc_votes(1000, seed=1000)
    block_hash = hashlib.sha512(b"block" + (1000).to_bytes(4, "little")).digest()[:32]
    buf = wire.encode_qc(block_hash, 1, [(bytes(p), bytes(q)) for p, q in zip(w.pk, w.sig)])
    nv = ctypes.c_size_t(0)
    call = lambda: lib.hsv_qc_verify_bincode(buf, len(buf), ctypes.byref(nv), None)
    settle(call)
    assert call() == 1
    res["n1000_votes667_bincode"] = dict(_timed_lib(call, reps), bytes=len(buf))
    if gaps:
        res["idle_gap_1ms"] = gaps
    return res


def call_route():
    """Which path answered the calling thread's last latency call: 'resident'
    (the resident service: the call leased no staging slot, HSV_MARK_SLOT not
    passed, but staged its request) or 'launch'."""
    from hsverify import _testing
    m = _testing.host_call_marks()
    return "resident" if (len(m) >= 3 and m[1] < 0 <= m[2]) else "launch"


def tc_latency(reps, auto=True):
    """C3 TC: 667 timeouts with per-vote digests SHA-512(round || hqc)[..32].
    TC::verify (consensus/src/messages.rs:307-313) calls Signature::verify per
    vote; the GPU form is the batched strict API (hsv_verify with per-item
    digests) and the certificate from its bincode bytes."""
    from hsverify import _lib, synth, wire
    lib = _lib.load()
    lib.hsv_set_auto_committee(1 if auto else 0)
    res = {"automatic_committee_cache": bool(auto)}
    for frac, tag in ((0.0, "clean"), (0.05, "corrupt5pct")):
        w = member_corrupted(synth.tc_votes, 1000, seed=1000, frac=frac) if frac else synth.tc_votes(1000, seed=1000)
        pk, sig, msg = (np.ascontiguousarray(a) for a in (w.pk, w.sig, w.msg))
        flags = np.zeros(w.n, np.uint8)
        if auto:  # the committee's keys were learnt from its QCs
            q = synth.qc_votes(1000, seed=1000)
            pq = np.concatenate([q.pk, q.sig], 1).tobytes()
            for _ in range(3):
                lib.hsv_verify_batch_packed(bytes(q.msg), pq, q.n)
            lib.hsv_auto_committee_wait(60000)
        call = lambda: lib.hsv_verify(pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, 32, w.n, flags.ctypes.data)
        res[f"n1000_votes667_{tag}_batched_strict"] = _timed_lib(call, reps)
        assert bool((flags & 1).all()) == (frac == 0)
        hqc = tc_hqc(1000, 1000)
        buf = wire.encode_tc(1000, [(bytes(p), bytes(s), int(h)) for p, s, h in zip(w.pk, w.sig, hqc)])
        nv = ctypes.c_size_t(0)
        call = lambda: lib.hsv_tc_verify_bincode(buf, len(buf), ctypes.byref(nv), None)
        rc = call()
        assert rc == (1 if frac == 0 else 0)
        res[f"n1000_votes667_{tag}_bincode"] = dict(_timed_lib(call, reps), bytes=len(buf))
    return res


def tc_dropin_sequential(reps):
    """C3 TC verified the way the unchanged caller does it: TC::verify
    (consensus/src/messages.rs:307-313) calls Signature::verify once per vote,
    in sequence, each over its own digest SHA-512(round || hqc)[..32].  Through
    the drop-in shim every call is one hsv_verify_strict (one vote, automatic
    committee cache warm).  Times the whole loop of 667 calls `reps` times, and
    the single calls inside it."""
    from hsverify import _lib, synth
    import gc
    lib = _lib.load()
    lib.hsv_set_auto_committee(1)
    q = synth.qc_votes(1000, seed=1000)
    pq = np.concatenate([q.pk, q.sig], 1).tobytes()
    for _ in range(3):
        lib.hsv_verify_batch_packed(bytes(q.msg), pq, q.n)
    lib.hsv_auto_committee_wait(60000)
    w = synth.tc_votes(1000, seed=1000)
    votes = [(bytes(w.msg[i]), bytes(w.pk[i]), bytes(w.sig[i])) for i in range(w.n)]
    vs = lib.hsv_verify_strict

    def loop(per_call=None):
        for d, p, s in votes:
            if per_call is None:
                if vs(d, p, s) != 1:
                    return False
            else:
                t0 = time.perf_counter()
                ok = vs(d, p, s)
                per_call.append(time.perf_counter() - t0)
                if ok != 1:
                    return False
        return True

    gc.collect()  # before the warm-up loop (as _timed_lib)
    assert loop()
    was = gc.isenabled()
    gc.disable()
    ts, calls = [], []
    try:
        for r in range(reps):
            t0 = time.perf_counter()
            ok = loop()
            ts.append(time.perf_counter() - t0)
            assert ok
        loop(calls)
    finally:
        if was:
            gc.enable()
    out = _p(ts)
    out.update(votes=w.n, call_p50_ms=float(np.median(calls) * 1e3), call_p99_ms=float(np.percentile(calls, 99) * 1e3),
               route=call_route())
    return out


def launched_child(reps, tc_reps):
    """Runs in a child process with HSV_QC_RESIDENT=0 (the library reads it
    once per process): one cached-key verify_strict, a C1 QC and the
    sequential TC loop launched per call, as without the resident service,
    and the dalek port's single verify_strict on one host core of the same
    process."""
    from hsverify import _lib, synth
    lib = _lib.load()
    lib.hsv_set_auto_committee(1)
    w = synth.qc_votes(4, seed=4)
    pk0, sig0, d0 = bytes(w.pk[0]), bytes(w.sig[0]), bytes(w.msg)
    packed = np.concatenate([w.pk, w.sig], 1).tobytes()
    for _ in range(3):
        lib.hsv_verify_batch_packed(d0, packed, w.n)
    lib.hsv_auto_committee_wait(60000)
    call = lambda: lib.hsv_verify_strict(d0, pk0, sig0)
    assert call() == 1
    res = {"single_verify_strict": _timed_lib(call, reps)}
    res["single_verify_strict"]["route"] = call_route()
    call = lambda: lib.hsv_verify_batch_packed(d0, packed, w.n)
    assert call() == 1
    res["n4_votes3"] = _timed_lib(call, reps)
    call = lambda: lib.hsv_verify_strict(d0, pk0, sig0)
    res["single_verify_strict_gap_1ms"] = _timed_gap(call, min(reps, 200), 1000)
    res["tc_dropin_sequential"] = tc_dropin_sequential(tc_reps)
    orc = _oracle()
    ts = _timed(lambda: orc.oracle_verify_flags(pk0, sig0, d0, 32), 200, warm=5)
    res["cpu_port_single_verify_strict_p50_ms"] = float(np.median(ts) * 1e3)
    return res


def launched_leg(reps, tc_reps):
    """launched_child in a fresh process (HSV_QC_RESIDENT=0); its JSON, or the error."""
    env = dict(os.environ, HSV_QC_RESIDENT="0")
    cmd = [sys.executable, os.path.abspath(__file__), "--launched-child", "--qc-reps", str(reps),
           "--tc-seq-reps", str(tc_reps)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
        if r.returncode == 0:
            return json.loads(r.stdout.strip().splitlines()[-1])
        return {"error": f"rc {r.returncode}: {r.stderr[-500:]}"}
    except (subprocess.SubprocessError, ValueError, IndexError) as e:
        return {"error": str(e)}


def committee_bench(reps, dev, n_votes=1 << 20):
    """Committee key cache: QC latency for C2/C3 through the
    cached tables, and throughput for 2^20 votes by a 1000-key committee."""
    import torch
    from hsverify import _lib, committee, synth
    from hsverify.verifier import sign_many
    lib = _lib.load()
    res = {}
    for size in (100, 1000):
        w = synth.qc_votes(size, seed=size)
        packed = np.concatenate([w.pk, w.sig], axis=1).tobytes()
        digest = bytes(w.msg)
        t0 = time.perf_counter()
        c = committee.Committee(synth.qc_votes(size, seed=size).pk)
        build_ms = (time.perf_counter() - t0) * 1e3
        h = c._h
        call = lambda: lib.hsv_committee_verify_batch_packed(h, digest, packed, w.n)
        assert call() == 1
        res[f"qc_n{size}_votes{w.n}"] = dict(_timed_lib(call, reps), table_build_ms=build_ms)
        c.close()
    # throughput: n_votes votes, each by one of 1000 members over its own digest
    seeds = synth.committee_seeds(1000, 7)
    rng = np.random.default_rng(7)
    who = rng.integers(0, 1000, n_votes)
    msgs = rng.integers(0, 256, (n_votes, 32), dtype=np.uint8)
    pks, sigs = sign_many(seeds[who], msgs)
    c = committee.Committee(sign_many(seeds, np.zeros((1000, 32), np.uint8))[0])
    idx = torch.from_numpy(who.astype(np.int32)).to(dev)
    sig = torch.from_numpy(sigs).to(dev)
    msg = torch.from_numpy(msgs).to(dev)
    flags = torch.zeros(n_votes, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    c.verify_device(idx, sig, msg, flags)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    steps = 5
    e0.record(stream)
    for _ in range(steps):
        c.verify_device(idx, sig, msg, flags)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    res["throughput"] = {"votes": n_votes, "committee": 1000, "kernel_ms": ms, "verif_per_s": n_votes / (ms * 1e-3),
                         "all_accepted": bool((flags.cpu().numpy() & 1).all())}
    c.close()
    return res


def qc_cpu(reps=5):
    """One host core: the reference's QC::verify crypto (dalek verify_batch:
    random linear combination, one Straus / Pippenger MSM of 2n+1 points,
    ported in oracle/ed25519_oracle.c) for C1 / C2 / C3, the strict-loop rule
    beside it, the sequential TC::verify loop (early exit) and one verify_strict."""
    from hsverify import synth
    lib = _oracle()
    res = {"cores": 1, "kind": "port", "cpu_model": cpu_model(),
           "algorithm": "C port of ed25519-dalek 1.0.1 verify_batch (curve25519-dalek 3.x: Straus below 190 "
                        "points, Pippenger w=6/7/8 above), radix-2^51 field"}
    for committee in (4, 100, 1000):
        w = synth.qc_votes(committee, seed=committee)
        pk, sig = np.ascontiguousarray(w.pk), np.ascontiguousarray(w.sig)
        ts = _timed(lambda: lib.oracle_verify_batch_dalek(bytes(w.msg), pk.ctypes.data, sig.ctypes.data, w.n, 1),
                    reps, warm=1)
        assert lib.oracle_verify_batch_dalek(bytes(w.msg), pk.ctypes.data, sig.ctypes.data, w.n, 2) == 1
        res[f"n{committee}_votes{w.n}_p50_ms"] = float(np.median(ts) * 1e3)
        ts = _timed(lambda: lib.oracle_verify_batch(bytes(w.msg), pk.ctypes.data, sig.ctypes.data, w.n), reps, warm=1)
        res[f"n{committee}_votes{w.n}_strict_loop_p50_ms"] = float(np.median(ts) * 1e3)
    w = member_corrupted(synth.qc_votes, 1000, seed=1000)
    pk, sig = np.ascontiguousarray(w.pk), np.ascontiguousarray(w.sig)
    ts = _timed(lambda: lib.oracle_verify_batch_dalek(bytes(w.msg), pk.ctypes.data, sig.ctypes.data, w.n, 3),
                reps, warm=1)
    assert lib.oracle_verify_batch_dalek(bytes(w.msg), pk.ctypes.data, sig.ctypes.data, w.n, 3) == 0
    res["n1000_votes667_corrupt5pct_p50_ms"] = float(np.median(ts) * 1e3)
    for frac, tag in ((0.0, "clean"), (0.05, "corrupt5pct")):
        w = member_corrupted(synth.tc_votes, 1000, seed=1000, frac=frac) if frac else synth.tc_votes(1000, seed=1000)
        pk, sig, msg = (np.ascontiguousarray(a) for a in (w.pk, w.sig, w.msg))
        ts = _timed(lambda: lib.oracle_tc_verify(pk.ctypes.data, sig.ctypes.data, msg.ctypes.data, w.n), reps, warm=1)
        res[f"tc_n1000_votes667_{tag}_p50_ms"] = float(np.median(ts) * 1e3)
    w = synth.qc_votes(4, seed=4)
    ts = _timed(lambda: lib.oracle_verify_flags(bytes(w.pk[0]), bytes(w.sig[0]), bytes(w.msg), 32), 50, warm=2)
    res["single_verify_strict_p50_ms"] = float(np.median(ts) * 1e3)
    return res


def mempool_bench(dev, n=1 << 20, tx_size=512, cpu_sample=1 << 17, nstreams=2, streams=None):
    """Mempool transactions: n client transactions of
    tx_size bytes (the reference benchmark's default, benchmark/fabfile.py),
    resident in HBM; one step = digest records + verification
    (hsv_verify_transactions_device).  Beside it: the C port on host threads
    over the first cpu_sample transactions, flag-for-flag against the GPU."""
    import torch
    from hsverify import mempool, synth
    w = synth.transactions(n, tx_size=tx_size, seed=9)
    d = torch.from_numpy(w.txs.reshape(-1)).to(dev)
    # Consecutive batches alternate over the given streams (main passes the
    # C4 line's first two), else over nstreams streams of their own.  Streams
    # created later can share a hardware queue with an earlier one (seen in
    # the round-4 traces, profiles/r04p_mempool_trace.txt); that did not change
    # the line's rate (r04w), but reusing the C4 line's streams keeps the two
    # lines' setups alike.
    if streams is None:
        stream = torch.cuda.current_stream(dev)
        streams = [stream] + [torch.cuda.Stream(dev) for _ in range(max(1, nstreams) - 1)]
    else:
        streams = list(streams)
        stream = streams[0]
    outs = [torch.zeros(n, dtype=torch.uint8, device=dev) for _ in streams]
    flags = outs[0]
    for j, s in enumerate(streams):
        mempool.verify_transactions_device(d, None, tx_size=tx_size, n=n, flags=outs[j], stream=s.cuda_stream)
    torch.cuda.synchronize(dev)
    steps = 10  # as many batches per round as the C4 line's default --steps
    rounds_ms = []
    # three timed rounds of `steps` batches, the median reported: one round
    # is ~100 ms, and one disturbed round once read 15.0 against 9.6-9.8 ms
    # (profiles/r03zz5_bench.json against r03zz6)
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for s in streams[1:]:
            s.wait_event(e0)
        for i in range(steps):
            j = i % len(streams)
            mempool.verify_transactions_device(d, None, tx_size=tx_size, n=n, flags=outs[j],
                                               stream=streams[j].cuda_stream)
        for s in streams[1:]:
            ev = torch.cuda.Event()
            ev.record(s)
            stream.wait_event(ev)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        rounds_ms.append(e0.elapsed_time(e1) / steps)
    ms = float(np.median(rounds_ms))
    f = flags.cpu().numpy()
    res = {"txs": n, "tx_size": tx_size, "ms_per_step": ms, "tx_per_s": n / (ms * 1e-3), "streams": len(streams),
           "rounds_ms_per_step": [round(x, 4) for x in rounds_ms],
           "outputs_identical_across_streams": all(bool(torch.equal(outs[0], o)) for o in outs[1:]),
           "honest_all_accepted": bool((f[w.accept] & 1).all()),
           "corrupted_all_rejected": bool(not (f[~w.accept] & 1).any())}
    sample = 1 << 17
    res["_check"] = (np.ascontiguousarray(w.txs[:sample]), tx_size, f[:sample].copy())  # for mempool_cpu
    if cpu_sample > 0:
        res["cpu_baseline"] = mempool_cpu(res.pop("_check"), cpu_sample)
    return res


def mempool_cpu(check, cpu_sample=1 << 17):
    """The C port on host threads over the first transactions of the mempool
    line's batch, flag-for-flag against the GPU's flags for them."""
    txs, tx_size, gpu = check
    lib = _oracle()
    m = min(cpu_sample, len(txs))
    threads, _ = host_cores()
    buf = np.ascontiguousarray(txs[:m])
    out = np.zeros(m, np.uint8)
    t0 = time.perf_counter()
    with all_host_cpus():
        lib.oracle_verify_tx_many(buf.ctypes.data, None, tx_size, m, out.ctypes.data, threads)
    dt = time.perf_counter() - t0
    return {"value": m / dt, "unit": "tx/s", "cores": threads, "kind": "port",
            "sample": f"first {m} transactions", "sample_parity_vs_gpu": bool((out == gpu[:m]).all())}


def host_api_bench(w, dev, reps=5):
    """The drop-in boundary hands over host buffers: hsv_verify on the C4 batch
    from numpy arrays, PCIe-inclusive (round 4: one streamed launch that reads
    the pinned records over PCIe as the host packs them).
    Beside it: the library's own account of the call (host time spent packing
    into pinned staging, bytes the kernel read from the host) and the link's
    H2D rate for the same bytes measured alone (one pinned 128 MiB copy)."""
    import torch
    from hsverify import _testing, verifier
    verifier.verify_flags(w.pk, w.sig, w.msg)
    ts, stats, marks = [], [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        f = verifier.verify_flags(w.pk, w.sig, w.msg)
        ts.append(time.perf_counter() - t0)
        stats.append(_testing.host_call_stats())
        marks.append(_testing.host_call_marks())
    k = int(np.argsort(ts)[len(ts) // 2])
    ms = float(ts[k] * 1e3)
    st = stats[k]
    nbytes = w.n * 128
    src = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        dst.copy_(src, non_blocking=True)
    e1.record()
    torch.cuda.synchronize(dev)
    h2d_ms = e0.elapsed_time(e1) / 3
    return {"items": int(w.n), "ms": ms, "verif_per_s": w.n / (ms * 1e-3), "reps": reps,
            "call_ms": st["call_ms"], "pack_ms": st["pack_ms"], "pack_threads": _testing.pack_threads() + 1,
            "h2d_bytes": st["h2d_bytes"], "input_rate_GBps": st["h2d_bytes"] / (ms * 1e-3) / 1e9,
            "h2d_alone_ms_for_128MiB": h2d_ms, "h2d_link_GBps": nbytes / (h2d_ms * 1e-3) / 1e9,
            "rep_ms": [round(t * 1e3, 3) for t in ts],
            # streamed path (run_streamed): ms from the call's entry to launch start,
            # launch enqueued, every piece packed, stream synchronised
            "median_call_marks_ms": dict(zip(("launch_start", "launch_enqueued", "packed", "synced"), marks[k]))
            if marks[k] and len(marks[k]) == 4 else marks[k],
            "honest_all_accepted": bool((f[w.accept] & 1).all()),
            "corrupted_all_rejected": bool(not (f[~w.accept] & 1).any())}


def _r(x, nd=4):
    """x rounded to nd significant digits (None passes through)."""
    if x is None:
        return None
    if isinstance(x, (bool, int)) and not isinstance(x, float):
        return x
    x = float(x)
    return 0.0 if x == 0 else float(f"{x:.{nd}g}")


def _pp(d, tail=False):
    """[p50, p99] ms of a latency record (plus the p50 of the library's own
    sync phase and of the tail reps' sync phase when tail=True)."""
    if not d:
        return None
    out = [_r(d.get("p50_ms")), _r(d.get("p99_ms"))]
    if tail and d.get("median_phases_ms") and d.get("tail", {}).get("phases_ms"):
        out += [_r(d["median_phases_ms"].get("sync")), _r(d["tail"]["phases_ms"].get("sync"))]
    return out


def compact(out):
    """The one stdout line (< 4 KB, so the driver's tail keeps it whole): the
    C4 throughput line with roofline and cpu_baseline, and BASELINE's second
    metric -- the QC verify p50 -- under `latency`, each GPU figure next to the
    CPU port's figure for the same call.  The full record goes to --detail."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data")
    c = {k: out[k] for k in keep}
    c["value"] = _r(out["value"], 6)
    c["ms_per_step"] = _r(out["ms_per_step"], 5)
    cfg = out["config"]
    c["config"] = {k: cfg[k] for k in ("workload", "batch_per_gpu", "global_batch", "parallelism", "kernel_variant",
                                       "streams", "host_affinity") if k in cfg}
    rf = out["roofline"]
    c["roofline"] = {"bound": rf["bound"], "achieved": _r(rf["achieved"]), "peak": _r(rf["peak"]), "unit": rf["unit"],
                     "frac": _r(rf["frac"]), "traffic": _r(rf["traffic"]),
                     "traffic_unit": "HBM B/launch (PMC FETCH_SIZEx2+WRITE_SIZE, committed pass)",
                     "kernel_ms": _r(rf["kernel_ms"]), "isolated_launch_ms": _r(rf["isolated_launch_ms"]),
                     "frac_isolated_launch": _r(rf["frac_isolated_launch"]),
                     "work": "192000 u32 MAC/verif; 129 B/verif algorithmic"}
    if len(rf.get("per_rank", [])) > 1:
        c["roofline"]["per_rank_kernel_ms"] = [_r(r["kernel_ms"]) for r in rf["per_rank"]]
    ck = out["checks"]
    c["checks"] = {k: ck[k] for k in ("honest_all_accepted", "corrupted_all_rejected", "outputs_identical_across_streams",
                                      "device_self_check_faults")}
    cb = out.get("cpu_baseline")
    if cb:
        c["cpu_baseline"] = {"value": _r(cb["value"]), "unit": cb["unit"], "cores": cb["cores"], "kind": cb["kind"],
                             "sample": cb["sample"].split(";")[0] + "; oracle/ed25519_oracle.c (dalek 1.0.1 "
                                                                     "verify_strict restated), all threads",
                             "sample_parity_vs_gpu": cb["sample_parity_vs_gpu"], "cpu_model": cb["cpu_model"],
                             "batch64_value": _r(cb["batch64"]["value"])}
    if "host_api" in out:
        h = out["host_api"]
        c["host_api"] = {"verif_per_s": _r(h["verif_per_s"]), "ms": _r(h["ms"]), "pack_ms": _r(h["pack_ms"]),
                         "checks_ok": bool(h["honest_all_accepted"] and h["corrupted_all_rejected"]),
                         "what": "hsv_verify on the C4 batch from host buffers, PCIe included"}
    ql, qg, tl = out.get("qc_latency"), out.get("qc_latency_generic"), out.get("tc_latency")
    if ql:
        qcpu = out.get("qc_cpu_baseline", {})
        cpu = lambda k: _r(qcpu.get(k))
        lat = {"unit": "ms", "form": "[p50, p99] (+ [sync p50, tail sync p50] for the cached QCs); cpu_p50: C port "
                                     "of dalek 1.0.1 on 1 host core, same inputs",
               "reps": ql["n4_votes3"]["reps"]}
        lat["qc_c1_3votes"] = {"gpu": _pp(ql["n4_votes3"], True), "cpu_p50": cpu("n4_votes3_p50_ms")}
        lat["qc_c2_67votes"] = {"gpu": _pp(ql["n100_votes67"], True), "cpu_p50": cpu("n100_votes67_p50_ms")}
        lat["qc_c3_667votes"] = {"gpu": _pp(ql["n1000_votes667"], True), "cpu_p50": cpu("n1000_votes667_p50_ms")}
        lat["qc_c3_corrupt5pct"] = {"gpu": _pp(ql["n1000_votes667_corrupt5pct"], True),
                                    "cpu_p50": cpu("n1000_votes667_corrupt5pct_p50_ms")}
        lat["qc_c3_bincode"] = {"gpu": _pp(ql["n1000_votes667_bincode"], True)}
        lat["verify_strict_single"] = {"gpu": _pp(ql["single_verify_strict"], True),
                                       "cpu_p50": cpu("single_verify_strict_p50_ms"),
                                       "route": ql["single_verify_strict"].get("route")}
        if qg:
            lat["cold_cache_off"] = {"c1": _pp(qg["n4_votes3"]), "c2": _pp(qg["n100_votes67"]),
                                     "c3": _pp(qg["n1000_votes667"]), "single": _pp(qg["single_verify_strict"])}
        if tl:
            lat["tc_c3_batched_strict"] = {"gpu": _pp(tl["n1000_votes667_clean_batched_strict"], True),
                                           "cpu_p50": cpu("tc_n1000_votes667_clean_p50_ms")}
            lat["tc_c3_corrupt5pct_bincode"] = {"gpu": _pp(tl["n1000_votes667_corrupt5pct_bincode"], True),
                                                "cpu_p50": cpu("tc_n1000_votes667_corrupt5pct_p50_ms")}
        seq = out.get("tc_dropin_sequential")
        if seq:
            lat["tc_c3_dropin_sequential"] = {"gpu": _pp(seq), "gpu_call_p50": _r(seq["call_p50_ms"]),
                                              "cpu_p50": cpu("tc_n1000_votes667_clean_p50_ms"), "route": seq.get("route"),
                                              "what": "667 sequential verify_strict calls, as TC::verify"}
        rs = out.get("launched", {})
        if "single_verify_strict" in rs:
            lat["launched_service_off"] = {
                "verify_strict_single": _pp(rs["single_verify_strict"], True),
                "qc_c1_3votes": _pp(rs["n4_votes3"], True),
                "tc_c3_dropin_sequential": _pp(rs["tc_dropin_sequential"]),
                "single_gap_1ms": _r(rs.get("single_verify_strict_gap_1ms", {}).get("p50_ms")),
                "cpu_p50_same_process": _r(rs["cpu_port_single_verify_strict_p50_ms"]),
                "what": "HSV_QC_RESIDENT=0 child process: one launch per call"}
        elif rs:
            lat["launched_service_off"] = {"error": str(rs.get("error"))[:200]}
        gq = (out.get("qc_latency") or {}).get("idle_gap_1ms")
        if gq:
            lat["idle_gap_1ms"] = {"c1": _r(gq["n4_votes3"]["p50_ms"]), "c3": _r(gq["n1000_votes667"]["p50_ms"]),
                                   "single": _r(gq.get("single", {}).get("p50_ms")),
                                   "what": "p50 with 1 ms of host idle before each call (consensus pacing)"}
        cc = out.get("committee_cache", {})
        if cc:
            lat["explicit_committee"] = {"c2": _pp(cc.get("qc_n100_votes67")), "c3": _pp(cc.get("qc_n1000_votes667"))}
        c["latency"] = lat
        if cc.get("throughput"):
            c["committee_throughput_verif_per_s"] = _r(cc["throughput"]["verif_per_s"])
    mp = out.get("mempool_tx")
    if mp:
        c["mempool_tx"] = {"tx_per_s": _r(mp["tx_per_s"]), "ms_per_step": _r(mp["ms_per_step"]),
                           "vs_c4": _r(mp["ms_per_step"] / out["roofline"]["kernel_ms"]),
                           "checks_ok": bool(mp["honest_all_accepted"] and mp["corrupted_all_rejected"]),
                           "cpu_tx_per_s": _r(mp.get("cpu_baseline", {}).get("value"))}
    if "qc_cpu_baseline" in out:
        c["qc_cpu_cores"] = out["qc_cpu_baseline"]["cores"]
    c["detail"] = out.get("detail_path")
    return c


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (one per GPU); default WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", "--per-gpu", dest="n", type=int, default=1 << 20, help="triples per GPU")
    ap.add_argument("--variant", type=int, default=None)
    ap.add_argument("--streams", type=int, default=3,
                    help="consecutive batches alternate over this many HIP streams, so a batch's launch can "
                         "start in the previous one's grid end (1: every batch on one stream)")
    ap.add_argument("--stream-priority", choices=("normal", "high"), default="normal",
                    help="priority of the C4 line's extra streams (measurement switch)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 20,
                    help="triples the CPU port verifies (default: the whole C4 batch)")
    ap.add_argument("--qc-reps", type=int, default=1000,
                    help="repetitions per latency figure (BASELINE.md: >= 1,000 for C2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-qc", action="store_true")
    ap.add_argument("--qc", action="store_true",
                    help="run the latency legs at N > 1 too (by default they run at N = 1 only: the QC p50 is a "
                         "one-GPU metric, and the other ranks would wait minutes at the final barrier)")
    ap.add_argument("--global-n", type=int, default=None,
                    help="C5 strong scaling: total triples split over the ranks (e.g. 16777216 = 2^24); "
                         "default: weak scaling with --n per GPU")
    ap.add_argument("--detail", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="file for the full record (every rep's phases, tails, probes); stdout gets the compact line")
    ap.add_argument("--tc-seq-reps", type=int, default=30,
                    help="repetitions of the 667-call sequential TC loop (tc_dropin_sequential)")
    ap.add_argument("--launched-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-launched", action="store_true", help="skip the service-off (launched) child leg")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU only: launcher, shards, timing and gather without a GPU or verification")
    return ap.parse_args(argv)


def launch_ranks(a):
    """Start one rank per GPU under torch.distributed.run; this process stays
    off the GPU and exits with the launcher's status."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    # torch.distributed.run's own parser rejects "--n" as an ambiguous prefix of
    # its options even after the script path: hand it on as --per-gpu
    args = ["--per-gpu" + x[3:] if x == "--n" or x.startswith("--n=") else x for x in sys.argv[1:]]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + args
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    log(f"[launcher] {' '.join(cmd)}")
    return subprocess.run(cmd, env=env).returncode


def dry_run(a, world, rank, dist):
    """Launcher / sharding / timing / gather path without a GPU: each rank owns
    its contiguous shard and runs a byte checksum over it as the 'step'."""
    strong = a.global_n is not None
    n = a.global_n // world if strong else a.n
    lo, hi = rank * n, (rank + 1) * n
    rng = np.random.default_rng(rank)
    data = rng.integers(0, 256, (n, 128), dtype=np.uint8)
    for _ in range(a.warmup):
        np.bitwise_xor.reduce(data, axis=1)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        flags = np.bitwise_xor.reduce(data, axis=1)
    elapsed = time.perf_counter() - t0
    import torch
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    shards = [None] * world
    dist.all_gather_object(shards, (rank, lo, hi, int(flags.size)))
    from hsverify import dist as hd
    gathered = hd.gather_strict(flags & 1, n * world)
    if rank == 0:
        el = float(t.item())
        print(json.dumps({
            "metric": "dry run (no GPU, no verification): launcher / shard / gather check",
            "value": n * world * a.steps / el, "unit": "items/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": el / a.steps * 1e3, "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "dry_run": True, "config": {"workload": "dry run", "batch_per_gpu": n, "global_batch": n * world,
                                        "parallelism": f"dp{world}"},
            "shards": [[r, l, h, m] for r, l, h, m in sorted(shards)], "gathered_items": int(gathered.size),
        }), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    a = parse_args()
    if a.launched_child:  # bench.py's own child (launched_leg): no ranks, one JSON line
        print(json.dumps(launched_child(a.qc_reps, a.tc_seq_reps)), flush=True)
        return
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus is not None and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(env_world or "1")
    if a.gpus is not None and a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    strong = a.global_n is not None
    if strong:
        if a.global_n % world:
            raise SystemExit("--global-n must be divisible by the number of ranks")
        a.n = a.global_n // world
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not a.qc:
        a.no_qc = True

    import torch.distributed as dist
    if a.dry_run:
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                init_method=None if world > 1 else "tcp://127.0.0.1:%d" % _free_port())
        return dry_run(a, world, rank, dist)

    import torch
    from hsverify import _lib, synth, verifier

    if world > 1:
        dist.init_process_group("gloo")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    affinity = pin_to_gpu_node(local_rank)
    _lib.load()
    if a.variant is not None:
        # a measurement run of another variant: every call goes to the test
        # library (the product libhsv.so exports no variant switch)
        _lib.set_override(_lib.load_test())
        log(f"--variant {a.variant}: measuring libhsv_test.so (the product objects plus the hooks)")
        verifier.set_variant(a.variant)
    verifier.bind_device(local_rank)  # this rank's host-buffer calls stay on its GPU

    host_threads = max(1, host_cores()[0] // max(1, world))
    t0 = time.perf_counter()
    # contiguous shard of the global batch: rank r owns items [r*n, (r+1)*n)
    w = synth.independent_triples(a.n, seed=0xC4 * 1000 + rank, corrupt_frac=0.05, nthreads=host_threads)
    log(f"[rank {rank}] synthesized {a.n} triples in {time.perf_counter() - t0:.1f}s")
    early_host_api = None
    if os.environ.get("HSV_BENCH_HOST_API_EARLY") and not a.no_qc:  # diagnosis: the same leg before any device work
        early_host_api = host_api_bench(w, torch.device("cuda", local_rank))
    pk, sig, msg = (torch.from_numpy(x).to(dev) for x in (w.pk, w.sig, w.msg))
    stream = torch.cuda.current_stream(dev)
    # Consecutive batches alternate over a.streams streams, each with its own
    # outputs: independent batches, as a verification pipeline would issue
    # them.  The next batch's prepass and point pass then fill the SIMDs the
    # previous point pass leaves idle at its grid end.
    nst = max(1, a.streams)
    prio = {"normal": 0, "high": -1}[a.stream_priority]
    streams = [stream] + [torch.cuda.Stream(dev, priority=prio) for _ in range(nst - 1)]
    outs = [(torch.zeros(a.n, dtype=torch.uint8, device=dev),
             torch.zeros((a.n + 31) // 32, dtype=torch.int32, device=dev)) for _ in range(nst)]
    flags, bits = outs[0]

    def step(i):
        o = outs[i % nst]
        verifier.verify_device(pk, sig, msg, o[0], o[1], stream=streams[i % nst].cuda_stream)

    for i in range(max(a.warmup, nst)):
        step(i)
    torch.cuda.synchronize(dev)

    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    e0.record(stream)
    for s in streams[1:]:
        s.wait_event(e0)
    for i in range(a.steps):
        step(i)
    for s in streams[1:]:
        ev = torch.cuda.Event()
        ev.record(s)
        stream.wait_event(ev)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    kernel_ms = e0.elapsed_time(e1) / a.steps
    # one launch alone on one stream (outside the timed region): the per-launch
    # duration rocprofv3 reports for the two kernels
    i0, i1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    i0.record(stream)
    for _ in range(3):
        verifier.verify_device(pk, sig, msg, flags, bits, stream=stream.cuda_stream)
    i1.record(stream)
    torch.cuda.synchronize(dev)
    isolated_ms = i0.elapsed_time(i1) / 3
    same_out = all(torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1]) for o in outs[1:])
    mine = {"rank": rank, "kernel_ms": kernel_ms, "isolated_launch_ms": isolated_ms, "elapsed_s": elapsed}
    per_rank = [mine]
    if world > 1:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    for r in per_rank:
        r["frac"] = a.n * WORK_MACS / (r["kernel_ms"] * 1e-3) / PEAK_MACS

    f = flags.cpu().numpy()
    honest_ok = bool((f[w.accept] & 1).all())
    corrupt_rejected = bool(not (f[~w.accept] & 1).any())
    faults = verifier.device_faults(local_rank)  # device self-checks of every launch above
    global_accepted = int((f & 1).sum())
    if world > 1:
        # host gather of the per-signature STRICT_OK bitmask (outside the timed region)
        from hsverify import dist as hd
        strict_all = hd.gather_strict(f, a.n * world)
        honest_all = hd.gather_strict(w.accept.astype(np.uint8), a.n * world)
        honest_ok = bool(strict_all[honest_all].all())
        corrupt_rejected = bool(not strict_all[~honest_all].any())
        global_accepted = int(strict_all.sum())

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    total = a.n * world * a.steps
    value = total / elapsed
    probe = verifier.measure_mad_peak()
    achieved = a.n * WORK_MACS / (kernel_ms * 1e-3)
    traffic, traffic_src = pmc_traffic(verifier.get_variant(), a.n)
    out = {
        "metric": "Ed25519 verifies/sec at batch 2^20 per GPU (bit-exact ed25519-dalek verify_strict flags)",
        "value": value,
        "unit": "verif/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (seeded keys/digests, RFC 8032 signatures, 5% corrupted)",
        "config": {
            "workload": (f"C5: {a.n * world} independent triples split over {world} GPU(s), inputs resident in HBM"
                         if strong else
                         "C4: 2^20 independent (pk, 32-B digest, sig) triples per GPU, inputs resident in HBM"),
            "batch_per_gpu": a.n,
            "global_batch": a.n * world,
            "parallelism": f"dp{world} (contiguous shards, no collective on the data path)",
            "host_affinity": affinity,
            "kernel_variant": verifier.get_variant(),
            "streams": nst,
        },
        "roofline": {
            "bound": "valu",
            "achieved": achieved / 1e12,
            "peak": PEAK_MACS / 1e12,
            "unit": "T u32-MAC/s",
            "frac": achieved / PEAK_MACS,
            "traffic": traffic,
            "traffic_unit": "HBM bytes per launch (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)",
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": a.n * IO_BYTES,
            "peak_probe": probe / 1e12,
            "work_per_verify": f"{WORK_MACS} u32 MACs (SURVEY 8(d)); {IO_BYTES} HBM bytes algorithmic",
            "kernel_ms": kernel_ms,
            "kernel_ms_is": (f"GPU time per step, HIP events around the {a.steps} steps "
                             f"(consecutive launches on {nst} alternating streams)"),
            "isolated_launch_ms": isolated_ms,
            "frac_isolated_launch": a.n * WORK_MACS / (isolated_ms * 1e-3) / PEAK_MACS,
            "kernels": "hsv_prep_kernel + hsv_verify_hp_kernel (one verify launch: scalar prepass, point pass)",
            "per_rank": per_rank,
        },
        "checks": {"honest_all_accepted": honest_ok, "corrupted_all_rejected": corrupt_rejected,
                   "strict_accepted_global": global_accepted, "outputs_identical_across_streams": same_out,
                   "device_self_check_faults": faults,
                   "expected_accept": "honest items and the mixed-order-A items with k = 0 mod 8"},
    }
    if not a.no_qc:
        # The two lines compared with the C4 line run right after it, in the same
        # conditions: the mempool line (the same point pass behind a message-hash
        # record kernel) first, then the drop-in boundary from host buffers.
        # After the latency legs -- a minute of other GPU work, and the resident
        # latency service's block on one CU -- the same mempool line read 7 %
        # slower than C4 (BENCH r05, r06a) against 4 % beside it
        # (profiles/r06/r06e_mp_analysis.json); the host call read 11.62 against
        # 11.21 ms (profiles/r03p_bench.json).
        # All three of the C4 line's streams: with the round-6 record kernel
        # (0.82 ms per 2^20, bitop3 message hash) three streams beat two, 9.61
        # against 9.66 ms (profiles/r06/r06l_nstreams_b3f.txt); round 4's
        # record kernel, 2.3x the C4 prepass's work, had been faster on two
        # (9.57 against 9.77 ms, profiles/r04z_mempool_streams2.txt).
        out["mempool_tx"] = mempool_bench(dev, nstreams=3, streams=streams if nst >= 2 else None,
                                          cpu_sample=0)
        out["host_api"] = host_api_bench(w, dev)
        if early_host_api is not None:
            out["host_api_early"] = early_host_api
    if world == 1 and not a.no_cpu_baseline:
        with all_host_cpus():
            out["cpu_baseline"] = cpu_baseline(w, f, a.cpu_sample)
    if not a.no_qc:
        out["qc_latency"] = qc_latency(a.qc_reps, auto=True)
        out["qc_latency_generic"] = qc_latency(a.qc_reps, auto=False)
        out["tc_latency"] = tc_latency(a.qc_reps, auto=True)
        out["tc_dropin_sequential"] = tc_dropin_sequential(a.tc_seq_reps)
        if not a.no_launched:
            out["launched"] = launched_leg(a.qc_reps, a.tc_seq_reps)
        _lib.load().hsv_set_auto_committee(1)
        out["committee_cache"] = committee_bench(a.qc_reps, dev)
        chk = out["mempool_tx"].pop("_check", None)
        if world == 1 and not a.no_cpu_baseline:
            with all_host_cpus():
                if chk is not None:
                    out["mempool_tx"]["cpu_baseline"] = mempool_cpu(chk)
                out["qc_cpu_baseline"] = qc_cpu()
    if a.detail:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(a.detail)), exist_ok=True)
            with open(a.detail, "w") as fh:
                json.dump(out, fh)
            out["detail_path"] = a.detail
        except OSError as e:
            log(f"detail record not written: {e}")
    print(json.dumps(compact(out), separators=(",", ":")), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if "-" in part:
            lo, hi = part.split("-")
            cpus.update(range(int(lo), int(hi) + 1))
        elif part:
            cpus.add(int(part))
    return cpus


_ALL_HOST_CPUS = None  # the process's CPU set before pin_to_gpu_node


class all_host_cpus:
    """The CPU baselines run on every CPU the process had before the GPU
    pinning (its worker threads, created inside the call, inherit the set)."""

    def __enter__(self):
        self.cur = os.sched_getaffinity(0)
        if _ALL_HOST_CPUS:
            os.sched_setaffinity(0, _ALL_HOST_CPUS)
        return self

    def __exit__(self, *exc):
        os.sched_setaffinity(0, self.cur)
        return False


def pin_to_gpu_node(device):
    """Bind this rank's threads to the CPUs of its GPU's NUMA node, the usual
    placement of one process per GPU.  The latency legs depend on it: a C3 QC
    called from the other socket of the box took 0.064 against 0.055 ms, C1
    +1 us, whichever node the library had allocated on
    (tools/qc_numa_probe.py, profiles/r05ac_numa.txt).  Threads the process
    starts later (the library's pack pool, the CPU baseline's workers) inherit
    the set.  Returns what was done, or None when the topology is not visible."""
    import torch
    try:
        p = torch.cuda.get_device_properties(device)
        bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
        with open(f"/sys/bus/pci/devices/{bdf}/numa_node") as fh:
            node = int(fh.read())
        if node < 0:
            return None
        with open(f"/sys/devices/system/node/node{node}/cpulist") as fh:
            cpus = _cpulist(fh.read()) & os.sched_getaffinity(0)
        if len(cpus) < host_cores()[0]:
            return None
        global _ALL_HOST_CPUS
        _ALL_HOST_CPUS = os.sched_getaffinity(0)
        os.sched_setaffinity(0, cpus)
        return {"numa_node": node, "cpus": len(cpus), "gpu_pci": bdf}
    except (OSError, ValueError, AttributeError, RuntimeError):
        return None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


if __name__ == "__main__":
    main()
