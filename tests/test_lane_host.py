"""Host (CPU) build of the lane kernel's per-lane logic (enet_amd/csrc/rc_lane.hip
compiled with tests/proto/lane_host_shim.h) against the reference fixtures.

The lane kernel is scalar code per lane, so its model and coder logic can be
exercised here without a GPU; the -m gpu tests then check the real kernel."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from tests import golden_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tests", "proto", "liblanehost.so")


@pytest.fixture(scope="module", params=["v2", "v3"])
def lane(request):
    so = SO if request.param == "v2" else SO.replace("liblanehost", "liblanehost3")
    csrc = os.path.join(ROOT, "enet_amd", "csrc")
    src = [os.path.join(ROOT, "tests", "proto", "lane_host.cpp")] + \
        [os.path.join(csrc, f) for f in ("rc_lane.hip", "rc_lane3.hip", "rc_lane_common.h", "rc_root3.h")]
    if not os.path.exists(so) or os.path.getmtime(so) < max(os.path.getmtime(s) for s in src):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared"] +
                              (["-DLANE3"] if request.param == "v3" else []) +
                              ["-I", csrc, "-I", os.path.join(ROOT, "tests", "proto"), "-o", so, src[0]])
    lib = C.CDLL(so)
    lib.lane_host_run.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_uint32,
                                  C.POINTER(C.c_uint32)]
    ol = C.c_uint32()

    def run(dec, data, cap, max_len=None):
        a = np.frombuffer(bytes(data) + b"\0" * 16, dtype=np.uint8).copy()
        out = np.zeros(max(cap, 1) + 16, np.uint8)
        ml = max_len or max(len(data), 16)
        if lib.lane_host_run(dec, a.ctypes.data, len(data), out.ctypes.data, cap, ml, C.byref(ol)):
            return "exact", b""
        return ol.value, out[: ol.value].tobytes()
    run.version = request.param
    return run


def test_lane_logic_compress_fixtures(lane):
    for c in golden_io.compress_cases():
        if c["in_limit"] != len(c["input"]):
            continue
        r = lane(0, c["input"], c["out_limit"])
        if r[0] == "exact":      # (allowed only for packets long enough to reach the model reset)
            assert lane.version == "v3" and len(c["input"]) > 1919
            continue
        assert r[0] == c["ret"], (len(c["input"]), c["out_limit"])
        if c["ret"]:
            assert r[1] == c["expect"]


def test_lane_logic_decompress_fixtures(lane):
    exact = 0
    for c in golden_io.decompress_cases():
        r = lane(1, c["input"], c["out_limit"])
        if r[0] == "exact":      # corrupt stream pointing past symbol 255: exact path
            exact += 1
            assert c["ret"] >= 0
            continue
        assert r[0] == c["ret"]
        if c["ret"]:
            assert r[1] == c["expect"]
    assert 0 < exact < 2000


def test_lane_logic_region_overflow_routes_exact(lane):
    # a tiny region (max_len hint 16) cannot hold a 1200-byte random packet's model
    # (v3 keeps single-symbol order-2 contexts inline, so it needs a small
    # alphabet -- many order-2 contexts with several symbols -- to fill its arena)
    data = np.random.default_rng(3).integers(0, 256, 1200, dtype=np.uint8)
    if lane.version == "v3":
        data &= 15
    assert lane(0, data.tobytes(), 4096, max_len=16)[0] == "exact"
