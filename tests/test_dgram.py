"""Datagram framing and batched socket I/O.

Oracle: oracle/pyoracle.datagram_{encode,decode}, a restatement of
protocol.c:1686-1718 (send) and :1022-1091 (receive).  It is pinned by real
ENet traffic: tests/golden/dgram_cases.json holds datagrams recorded from live
reference hosts (compress.c + enet_crc32; tests/golden/make_dgram_golden.py),
each of which the restatement must decode with a matching checksum and
re-encode to the exact wire bytes.

GPU: enet_rc_datagram_{encode,decode}_batch_{host,device} through the C ABI
against the fixture and the oracle (bit-exact bytes and lengths), and a
socket -> pinned buffer -> GPU decode pipeline over 127.0.0.1.
"""
import json
import os
import socket
import time

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _cases():
    with open(os.path.join(HERE, "golden", "dgram_cases.json")) as f:
        return json.load(f)["cases"]


def _port_coder():
    from oracle.pyoracle import Coder
    return Coder("port")


def _synthetic(rng, n):
    """Assembled datagrams: random header flags and session bits, game-state,
    random and tiny command payloads (some incompressible, some empty)."""
    from enet_amd import synth
    gd, go, gl = synth.gamestate_batch(max(1, n // 3), 1200)
    out = []
    for i in range(n):
        sent = bool(rng.integers(0, 2))
        peer = int(rng.integers(0, 0x1000))
        word = peer | (int(rng.integers(0, 4)) << 12) | (0x8000 if sent else 0)
        head = word.to_bytes(2, "big") + (int(rng.integers(0, 65536)).to_bytes(2, "big") if sent else b"")
        kind = i % 4
        if kind == 0:
            k = i // 4 % len(gl)
            cmds = gd[int(go[k]): int(go[k]) + int(rng.integers(1, 1200))].tobytes()
        elif kind == 1:
            cmds = rng.integers(0, 256, size=int(rng.integers(1, 1400)), dtype=np.uint8).tobytes()
        elif kind == 2:
            cmds = bytes(int(rng.integers(0, 64)))
        else:
            cmds = (rng.integers(0, 3, size=int(rng.integers(1, 3000)), dtype=np.uint8)).tobytes()
        out.append((head, cmds))
    return out


def _assemble(parts, checksum, rng):
    return [h + (int(rng.integers(0, 2**32)).to_bytes(4, "little") if checksum else b"") + c for h, c in parts]


# ------------------------------------------------------------------- CPU

def test_oracle_framing_pinned_by_real_datagrams():
    from oracle.pyoracle import datagram_decode, datagram_encode
    port = _port_coder()
    cases = _cases()
    assert len(cases) > 300 and sum(c["compressed"] for c in cases) > 100
    for c in cases:
        wire = bytes.fromhex(c["wire"])
        dec = datagram_decode(wire, bool(c["checksum"]), c["seed"], port)
        assert dec.hex() == c["decoded"]
        assert datagram_encode(dec, bool(c["checksum"]), c["seed"], port) == wire


def test_oracle_framing_drops():
    from oracle.pyoracle import datagram_decode
    port = _port_coder()
    c = next(c for c in _cases() if c["checksum"] and c["compressed"])
    wire = bytearray.fromhex(c["wire"])
    assert datagram_decode(bytes(wire), True, c["seed"], port)
    assert datagram_decode(bytes(wire), True, c["seed"] ^ 1, port) == b""     # wrong connectID
    hs = (4 if wire[0] & 0x80 else 2) + 4
    bad = bytearray(wire)
    bad[hs - 4] ^= 0x01                                                      # corrupt checksum field
    assert datagram_decode(bytes(bad), True, c["seed"], port) == b""
    assert datagram_decode(b"\x80", True, 0, port) == b""                   # shorter than 2 bytes
    assert datagram_decode(b"\x80\x01\x02", True, 0, port) == b""           # shorter than its header
    assert datagram_decode(b"\x40\x01", False, 0, port) == b""              # compressed, no commands


def test_socket_batch_loopback():
    from enet_amd import io
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
    rx.bind(("127.0.0.1", 0))
    rx.setblocking(False)
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    tx.bind(("127.0.0.1", 0))
    try:
        buf = np.zeros(4096 * 300, np.uint8)
        assert io.receive_batch(rx.fileno(), buf, 4096, 300)[0] == 0        # nothing queued: 0, no block
        dg = [bytes([i % 251]) * (1 + (i * 37) % 1400) for i in range(300)]
        assert io.send_batch(tx.fileno(), dg, rx.getsockname()) == 300
        got, t0 = [], time.time()
        while len(got) < 300 and time.time() - t0 < 5:
            n, lens, peers = io.receive_batch(rx.fileno(), buf, 4096, 300)
            got += [buf[i * 4096: i * 4096 + int(lens[i])].tobytes() for i in range(n)]
            assert all(p == tx.getsockname() for p in peers)
        assert got == dg
    finally:
        rx.close()
        tx.close()


# ------------------------------------------------------------------- GPU

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def coder():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from enet_amd import RangeCoder
    c = RangeCoder()
    yield c
    c.close()


@pytest.mark.gpu
def test_gpu_decode_encode_real_datagrams(coder):
    cases = _cases()
    for ck in (0, 1):
        sel = [c for c in cases if c["checksum"] == ck]
        wires = [bytes.fromhex(c["wire"]) for c in sel]
        seeds = [c["seed"] for c in sel]
        dec = coder.datagrams(True, wires, checksum=bool(ck), seeds=seeds)
        assert [d.hex() for d in dec] == [c["decoded"] for c in sel]
        enc = coder.datagrams(False, dec, checksum=bool(ck), seeds=seeds)
        assert enc == wires


@pytest.mark.gpu
def test_gpu_framing_vs_oracle_synthetic(coder):
    from oracle.pyoracle import datagram_decode, datagram_encode
    port = _port_coder()
    rng = np.random.default_rng(5)
    for ck in (False, True):
        dg = _assemble(_synthetic(rng, 400), ck, rng)
        dg += [b"", b"\x80", b"\x00\x01", b"\x80\x00\x01"]                 # shorter than their headers
        seeds = [int(s) for s in rng.integers(0, 2**32, size=len(dg))]
        enc = coder.datagrams(False, dg, checksum=ck, seeds=seeds)
        want = [datagram_encode(d, ck, s, port) for d, s in zip(dg, seeds)]
        assert enc == want
        wires = [w for w in want if w]
        ws = [s for w, s in zip(want, seeds) if w]
        # corrupt some: flipped bits in the stream or the checksum, wrong seeds
        for i in range(0, len(wires), 7):
            b = bytearray(wires[i])
            b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
            wires[i] = bytes(b)
        ws = [s ^ (1 if i % 11 == 3 else 0) for i, s in enumerate(ws)]
        dec = coder.datagrams(True, wires, checksum=ck, seeds=ws)
        assert dec == [datagram_decode(w, ck, s, port) for w, s in zip(wires, ws)]


@pytest.mark.gpu
def test_gpu_socket_to_device_decode_pipeline(coder):
    """Wire datagrams over UDP -> recvmmsg into pinned staging -> H2D -> one
    decode batch on the GPU (the host end of the path)."""
    from enet_amd import io
    cases = [c for c in _cases() if c["checksum"]][:256]
    wires = [bytes.fromhex(c["wire"]) for c in cases]
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
    rx.bind(("127.0.0.1", 0))
    rx.setblocking(False)
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    try:
        assert io.send_batch(tx.fileno(), wires, rx.getsockname()) == len(wires)
        stage = torch.zeros(4096 * len(wires), dtype=torch.uint8).pin_memory()
        buf = stage.numpy()
        n, t0, lens = 0, time.time(), []
        while n < len(wires) and time.time() - t0 < 5:
            k, ln, _ = io.receive_batch(rx.fileno(), buf[n * 4096:], 4096, len(wires) - n)
            lens += [int(x) for x in ln]
            n += k
        assert n == len(wires)
        dev = stage.cuda(non_blocking=True)
        off = torch.arange(n, dtype=torch.int64, device="cuda") * 4096
        ln = torch.tensor(lens, dtype=torch.int32, device="cuda")
        out = torch.zeros(4096 * n, dtype=torch.uint8, device="cuda")
        out_len = torch.zeros(n, dtype=torch.int32, device="cuda")
        seed = torch.tensor(np.array([c["seed"] for c in cases], np.uint32).view(np.int32), device="cuda")
        coder.datagram_decode_batch(dev, off, ln, out, off, out_len, checksum=True, seed=seed)
        torch.cuda.synchronize()
        ol = out_len.cpu().numpy()
        ob = out.cpu().numpy()
        got = [ob[i * 4096: i * 4096 + int(ol[i])].tobytes().hex() for i in range(n)]
        assert got == [c["decoded"] for c in cases]
    finally:
        rx.close()
        tx.close()
