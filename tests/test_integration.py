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
LOOP_DEF = os.path.join(REF_DIR, "loopback_deferred")          # deferred-batch mode, GPU library
LOOP_DEF_CPU = os.path.join(REF_DIR, "loopback_deferred_cpu")  # same plumbing, CPU test double


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


def _env(checksum):
    env = dict(os.environ)
    env["ENET_LOOPBACK_CHECKSUM"] = "1" if checksum else "0"
    return env


def _run(binary, role, port, count, timeout=90, checksum=False, extra=()):
    r = subprocess.run([binary, role, str(port), str(count), *map(str, extra)], capture_output=True,
                       text=True, timeout=timeout, env=_env(checksum))
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


def _pair(server_bin, client_bin, count, checksum=False):
    port = _port()
    srv = subprocess.Popen([server_bin, "server", str(port), str(count)], stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True, env=_env(checksum))
    try:
        time.sleep(0.5)
        crc, cres, cerr = _run(client_bin, "client", port, count, checksum=checksum)
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


# ---------------------------------------------------------------------------
# Deferred-batch mode (include/enet_rc_deferred.h, enet_amd/csrc/rc_deferred.c):
# protocol.c unchanged, its socket calls routed by --wrap into one GPU batch
# per send / receive pass.  "fan" runs K peers between two hosts so that one
# pass carries many datagrams.

def _check_fan(res, peers, count):
    assert res["ok"] and res["mismatches"] == 0 and res["received"] == peers * count, res
    for side in ("server", "client"):
        st = res[side]
        assert st["send_compressed"] > 0 and st["recv_dropped"] == 0, res
        # the point of the mode: many datagrams per launch
        assert st["send_datagrams"] >= 4 * st["send_batches"], res
        assert st["recv_datagrams"] >= 4 * st["recv_batches"], res


@pytest.mark.parametrize("checksum", [False, True])
def test_deferred_plumbing_cpu_double(checksum):
    """The deferred queues and --wrap hooks in live hosts, with the four library
    calls served by the oracle (tests/integration/deferred_double.c): CPU only."""
    _need(LOOP_DEF_CPU)
    rc, res, err = _run(LOOP_DEF_CPU, "fan", _port(), 100, checksum=checksum, extra=(16,))
    assert rc == 0, (res, err)
    _check_fan(res, 16, 100)


@pytest.mark.parametrize("checksum", [False, True])
def test_deferred_cpu_double_talks_to_reference(checksum):
    _need(LOOP_DEF_CPU, LOOP_REF)
    c, s = _pair(LOOP_DEF_CPU, LOOP_REF, 200, checksum=checksum)
    assert c["ok"] and c["mismatches"] == 0
    c, s = _pair(LOOP_REF, LOOP_DEF_CPU, 200, checksum=checksum)
    assert c["ok"] and c["mismatches"] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("checksum", [False, True])
def test_deferred_host_gpu_batches(checksum):
    """32 peers, deferred mode on the GPU library: every echo matches and each
    send / receive pass is one batch launch of many datagrams."""
    _need(LOOP_DEF)
    rc, res, err = _run(LOOP_DEF, "fan", _port(), 200, checksum=checksum, extra=(32,))
    assert rc == 0, (res, err)
    assert res["coder"].startswith("enet_rc_amd")
    _check_fan(res, 32, 200)


@pytest.mark.gpu
@pytest.mark.parametrize("checksum", [False, True])
def test_deferred_gpu_host_talks_to_reference(checksum):
    """Wire compatibility: a deferred GPU host against compress.c + enet_crc32
    peers, in both roles."""
    _need(LOOP_DEF, LOOP_REF)
    c, s = _pair(LOOP_DEF, LOOP_REF, 300, checksum=checksum)
    assert c["ok"] and c["mismatches"] == 0 and s["coder"].startswith("enet_rc_amd")
    c, s = _pair(LOOP_REF, LOOP_DEF, 300, checksum=checksum)
    assert c["ok"] and c["mismatches"] == 0 and c["coder"].startswith("enet_rc_amd")


def test_deferred_header_symbols_defined():
    """Every function include/enet_rc_deferred.h declares, and the six --wrap
    entry points, are defined by rc_deferred.c as linked into the harness (the
    deferred module is linked into the application, not libenet_rc_amd.so)."""
    import re
    _need(LOOP_DEF_CPU)
    hdr = open(os.path.join(HERE, "..", "include", "enet_rc_deferred.h")).read()
    names = set(re.findall(r"^\w[\w\s\*]*?\b(enet_rc_deferred_\w+)\s*\(", hdr, re.M))
    assert {"enet_rc_deferred_attach", "enet_rc_deferred_flush", "enet_rc_deferred_detach",
            "enet_rc_deferred_checksum", "enet_rc_deferred_get_stats"} <= names
    wraps = {f"__wrap_enet_{f}" for f in ("socket_send", "socket_receive", "socket_wait",
                                           "host_service", "host_flush", "host_destroy")}
    out = subprocess.run(["nm", LOOP_DEF_CPU], capture_output=True, text=True, check=True).stdout
    defined = {l.split()[-1] for l in out.splitlines() if re.match(r"^[0-9a-f]+ T ", l)}
    assert names | wraps <= defined, sorted((names | wraps) - defined)
