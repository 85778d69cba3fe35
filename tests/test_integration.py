"""Drop-in check in live ENet hosts.

tests/integration/enet_loopback.c runs ENet hosts over 127.0.0.1 with
enet_host_compress_with_range_coder enabled.  oracle/Makefile links it twice:
  loopback_ref : reference library with its own compress.c
  loopback_amd : reference library WITHOUT compress.c + libenet_rc_amd.so
so the GPU coder is swapped in purely at link time, the way INTEGRATION.md
describes.  Mixed pairs prove wire compatibility: datagrams compressed on the
GPU are decompressed by compress.c and the other way round (the protocol drops
a datagram whose decompression fails, protocol.c:1067, so a mismatch shows up
as a missing or corrupted echo).
"""
import json
import os
import socket
import subprocess
import time

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = os.path.join(HERE, "..", "oracle", "_ref")
LOOP_REF = os.path.join(REF_DIR, "loopback_ref")
LOOP_AMD = os.path.join(REF_DIR, "loopback_amd")


def _port():
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _need(*paths):
    for p in paths:
        if not os.path.exists(p):
            pytest.skip(f"{os.path.basename(p)} not built (needs the reference sources at build time)")


def _run(binary, role, port, count, timeout=90):
    r = subprocess.run([binary, role, str(port), str(count)], capture_output=True, text=True, timeout=timeout)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


def _pair(server_bin, client_bin, count):
    port = _port()
    srv = subprocess.Popen([server_bin, "server", str(port), str(count)], stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True)
    try:
        time.sleep(0.5)
        crc, cres, cerr = _run(client_bin, "client", port, count)
        sout, serr = srv.communicate(timeout=90)
    finally:
        if srv.poll() is None:
            srv.kill()
    sres = json.loads([l for l in sout.splitlines() if l.startswith("{")][-1])
    assert crc == 0 and srv.returncode == 0, (cres, cerr, sres, serr)
    return cres, sres


def test_reference_loopback_harness():
    """The harness itself, with compress.c on both sides (CPU only)."""
    _need(LOOP_REF)
    rc, res, err = _run(LOOP_REF, "both", _port(), 200)
    assert rc == 0 and res["ok"], (res, err)
    assert res["wire_bytes_sent"] < res["payload_bytes"] / 2      # compression was in effect


@pytest.mark.gpu
def test_gpu_coder_in_live_hosts():
    _need(LOOP_AMD)
    rc, res, err = _run(LOOP_AMD, "both", _port(), 300)
    assert rc == 0 and res["ok"], (res, err)
    assert res["coder"].startswith("enet_rc_amd")
    assert res["wire_bytes_sent"] < res["payload_bytes"] / 2


@pytest.mark.gpu
def test_gpu_server_reference_client():
    _need(LOOP_AMD, LOOP_REF)
    c, s = _pair(LOOP_AMD, LOOP_REF, 300)
    assert c["ok"] and c["mismatches"] == 0 and s["coder"].startswith("enet_rc_amd")


@pytest.mark.gpu
def test_reference_server_gpu_client():
    _need(LOOP_AMD, LOOP_REF)
    c, s = _pair(LOOP_REF, LOOP_AMD, 300)
    assert c["ok"] and c["mismatches"] == 0 and c["coder"].startswith("enet_rc_amd")
