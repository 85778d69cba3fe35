"""The C-ABI library loads and exports every entry point include/enet_rc_amd.h declares.
CPU only: no compute calls (there is no GPU in the build container)."""
import ctypes as C
import os
import subprocess

from enet_amd._lib import LIB_PATH, header_symbols


def test_library_exports_header_symbols():
    syms = header_symbols()
    assert "enet_range_coder_compress" in syms and "enet_rc_compress_batch_device" in syms
    lib = C.CDLL(LIB_PATH)
    for s in syms:
        assert hasattr(lib, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(syms) <= exported


def test_reference_signatures_match_enet_h():
    # enet.h:603-606 and :574 -- the drop-in entry points keep the reference prototypes
    hdr = open(os.path.join(os.path.dirname(LIB_PATH), "..", "..", "include", "enet_rc_amd.h")).read()
    assert "void *enet_range_coder_create(void);" in hdr
    assert "void enet_range_coder_destroy(void *context);" in hdr
    assert "size_t enet_range_coder_compress(void *context, const ENetBuffer *inBuffers, size_t inBufferCount,\n" in hdr
    assert "size_t enet_range_coder_decompress(void *context, const enet_uint8 *inData, size_t inLimit,\n" in hdr
    assert "int enet_host_compress_with_range_coder(ENetHost *host);" in hdr


def test_no_cpu_coder_in_product():
    # the product library must not contain or load the oracle
    out = subprocess.run(["nm", "-D", LIB_PATH], capture_output=True, text=True).stdout
    assert "or_compress" not in out and "or_decompress" not in out
    deps = subprocess.run(["ldd", LIB_PATH], capture_output=True, text=True).stdout
    assert "liboracle" not in deps and "libenet_ref" not in deps
