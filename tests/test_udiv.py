"""The coder kernels' exact division (enet_amd/csrc/rc_udiv.h) against
integer division, on the GPU: ~1.3e10 operand pairs of random widths plus
exact multiples, one-below-multiples and a = 2^32 - 1."""
import ctypes as C
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "proto", "udiv_check.hip")
CSRC = os.path.join(HERE, "..", "enet_amd", "csrc")


@pytest.mark.gpu
def test_udiv_exact(tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    so = str(tmp_path / "libudiv.so")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                           "-I", CSRC, "-o", so, SRC])
    lib = C.CDLL(so)
    lib.udiv_run.restype = C.c_int
    lib.udiv_run.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.POINTER(C.c_ulonglong)]
    bad = C.c_ulonglong(0)
    assert lib.udiv_run(0x454E4554, 4096, 3200, C.byref(bad)) == 0
    assert bad.value == 0
