"""The record-light decoder's input hand-off (enet_amd/csrc/rc_slot.h) under a
seeded interleaving scheduler (tests/proto/slot_sched.cpp): a decoding lane
and its helper lane as two threads, one running at a time, switching at
every point between two LDS word accesses of the protocol -- including
between the decoder's h_ctl read and its slot read, and across packet
boundaries (one lane decodes a run of packets; generations count up).

Checks: every chunk the decoder takes from the slot is the packet's chunk,
and every packet the fast decoder finishes and its check passes (the bigram
count and the hand-off's check sums, rc_dec6_verify) decodes to the oracle's
bytes.  Two protocol mutants (SLOT_MUTANT=1: the generation published before
the packet index, as a torn 64-bit store could show it; =2: the helper's
announcement before its slot store) must take wrong chunks under the
scheduler -- it reaches the interleavings that matter -- and the check must
still leave no wrong packet: the sums catch every wrong chunk.  CPU only; no
reference needed at run time."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from enet_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "enet_amd", "csrc")
PROTO = os.path.join(ROOT, "tests", "proto")


def _build(mutant):
    so = os.path.join(PROTO, f"libslotsched{mutant}.so")
    src = [os.path.join(PROTO, "slot_sched.cpp")] + [os.path.join(CSRC, f) for f in (
        "rc_dec6.hip", "rc_dec6_rare.h", "rc_slot.h", "rc_lane_common.h", "rc_root3.h", "rc_udiv.h")]
    if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(s) for s in src):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", f"-DSLOT_MUTANT={mutant}",
                               "-I", CSRC, "-I", PROTO, "-o", so, src[0]])
    lib = C.CDLL(so)
    P = C.c_void_p
    lib.slot_sched_run.argtypes = [P, P, P, C.c_uint32, P, P, P, P, P, P, P, C.c_uint64, C.c_uint32,
                                   C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]
    lib.slot_sched_run.restype = C.c_uint32
    return lib


def _bigrams(x):
    if len(x) < 2:
        return 0
    return len(set(zip(x[:-1].tolist(), x[1:].tolist())))


def _workload(seed):
    """A lane's run of packets: short random ones (many packet boundaries per
    decoded byte), a few MTU-sized, odd alignments of the compressed streams."""
    from oracle.pyoracle import compress_batch
    rng = np.random.default_rng(seed)
    lens = np.concatenate([rng.integers(8, 120, 10), rng.integers(600, 1300, 2)]).astype(np.uint32)
    d, o, l = synth.random_batch(len(lens), int(lens.max()), seed=synth.SEED + seed)
    l = lens
    o = np.zeros(len(l), np.uint64)
    o[1:] = np.cumsum(l[:-1], dtype=np.uint64)
    d = d[: int(l.sum())].copy()
    out, oo, cap, ol = compress_batch(d, o, l, "port")
    # the compressed streams at ragged offsets (slot_init's alignment cases)
    pad = rng.integers(0, 16, len(l)).astype(np.uint64)
    coff = np.zeros(len(l), np.uint64)
    acc = 0
    for i in range(len(l)):
        acc += int(pad[i])
        coff[i] = acc
        acc += int(ol[i])
    comp = np.zeros(acc + 64, np.uint8)
    for i in range(len(l)):
        comp[int(coff[i]): int(coff[i]) + int(ol[i])] = out[int(oo[i]): int(oo[i]) + int(ol[i])]
    return d, o, l, comp, coff, ol.astype(np.uint32)


def _run(lib, wl, seed, p):
    d, o, l, comp, coff, clen = wl
    n = len(l)
    dout = np.zeros(int(l.sum()) + 64, np.uint8)
    dlen = np.zeros(n, np.uint32)
    claims = np.zeros(n, np.uint32)
    icks = np.zeros(n, np.uint32)
    hcks = np.zeros(2 * n, np.uint32)
    cap = l.astype(np.uint32)
    takes = C.c_uint32()
    sw = C.c_uint64()
    ptr = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    bad = lib.slot_sched_run(ptr(comp), ptr(coff), ptr(clen), n, ptr(dout), ptr(o), ptr(cap), ptr(dlen),
                             ptr(claims), ptr(icks), ptr(hcks), seed, {1.0: 0xFFFF, 2.0: 0xFFFE}.get(p, int(p * 65536)), C.byref(takes), C.byref(sw))
    wrong = 0
    done = 0
    for i in range(n):
        if claims[i] == 0xFFFFFFFF:
            continue                        # left to the lane kernels
        got = dout[int(o[i]): int(o[i]) + int(dlen[i])]
        ck = icks[i] == hcks[i] or icks[i] == (int(hcks[i]) - int(hcks[n + i])) & 0xFFFFFFFF
        if (claims[i] & 0x7FFFFFFF) != _bigrams(got) or not ck:
            continue                        # fails the check (rc_dec6_verify): decoded again by the lane kernels
        done += 1
        if int(dlen[i]) != int(l[i]) or not np.array_equal(got, d[int(o[i]): int(o[i]) + int(l[i])]):
            wrong += 1
    return bad, wrong, done, takes.value, sw.value


SEEDS = range(40)
# 0.0: log-uniform bursts; 1.0: per-site probabilities redrawn per run; 2.0: cooperative but for
# one preempting site per run (slot_sched.cpp switch_now)
PROBS = (0.0, 1.0, 2.0, 2.0, 2.0, 0.03, 0.3, 0.9)


def test_slot_handoff_interleavings():
    lib = _build(0)
    tot_takes = tot_sw = tot_done = 0
    for s in SEEDS:
        wl = _workload(s)
        for k, p in enumerate(PROBS):
            bad, wrong, done, takes, sw = _run(lib, wl, 1000 * s + k, p)
            assert bad == 0 and wrong == 0, (s, p, bad, wrong)
            tot_takes += takes
            tot_sw += sw
            tot_done += done
    # the runs exercised the slot: chunks taken through it, hand-overs, packets finished
    assert tot_takes > 5000 and tot_sw > 50000 and tot_done > 0.9 * len(SEEDS) * len(PROBS) * 12


@pytest.mark.parametrize("mutant", [1, 2])
def test_slot_mutants_are_caught(mutant):
    lib = _build(mutant)
    caught = 0
    for s in SEEDS:
        wl = _workload(s)
        for k, p in enumerate(PROBS):
            bad, wrong, done, takes, sw = _run(lib, wl, 1000 * s + k, p)
            caught += bad
            assert wrong == 0, (s, p, bad, wrong)
    assert caught > 0
