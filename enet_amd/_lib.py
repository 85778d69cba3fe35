"""ctypes binding of libenet_rc_amd.so (the C ABI declared in include/enet_rc_amd.h).

The library is the product: HIP kernels + C host shim.  There is no Python or
CPU fallback; if the library is missing this module raises at import time.
"""
from __future__ import annotations

import ctypes as C
import os
import re

try:  # load torch's HIP runtime first so the library and torch share one runtime
    import torch  # noqa: F401
except ImportError:  # the C ABI itself does not need torch
    pass

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
# ENET_RC_LIB: diagnostic override (e.g. the -DRC_PROFILE build used by tools/lane_prof.py)
LIB_PATH = os.environ.get("ENET_RC_LIB") or os.path.join(HERE, "lib", "libenet_rc_amd.so")
HEADER = os.path.join(ROOT, "include", "enet_rc_amd.h")


class ENetBuffer(C.Structure):
    """include/enet/unix.h:30-34 (iovec layout)."""
    _fields_ = [("data", C.c_void_p), ("dataLength", C.c_size_t)]


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                          f"or `make -C enet_amd/csrc`")
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    vp, sz, u32 = C.c_void_p, C.c_size_t, C.c_uint32
    lib.enet_range_coder_create.restype = vp
    lib.enet_range_coder_create.argtypes = []
    lib.enet_range_coder_destroy.restype = None
    lib.enet_range_coder_destroy.argtypes = [vp]
    lib.enet_range_coder_compress.restype = sz
    lib.enet_range_coder_compress.argtypes = [vp, C.POINTER(ENetBuffer), sz, sz, vp, sz]
    lib.enet_range_coder_decompress.restype = sz
    lib.enet_range_coder_decompress.argtypes = [vp, vp, sz, vp, sz]
    lib.enet_host_compress_with_range_coder.restype = C.c_int
    lib.enet_host_compress_with_range_coder.argtypes = [vp]
    batch_dev = [vp, vp, vp, vp, sz, u32, vp, vp, vp, vp, vp]
    batch_host = [vp, vp, vp, vp, sz, vp, vp, vp, vp]
    for name, args in (("enet_rc_compress_batch_device", batch_dev),
                       ("enet_rc_decompress_batch_device", batch_dev),
                       ("enet_rc_compress_batch_host", batch_host),
                       ("enet_rc_decompress_batch_host", batch_host),
                       ("enet_rc_decompress_batch_device_bounded", batch_dev[:-1] + [u32, vp])):
        f = getattr(lib, name)
        f.restype = C.c_int
        f.argtypes = args
    lib.enet_rc_compress_gather_batch_host.restype = C.c_int
    lib.enet_rc_compress_gather_batch_host.argtypes = [vp, C.POINTER(ENetBuffer), vp, sz, vp, vp, vp, vp]
    lib.enet_rc_crc32_batch_device.restype = C.c_int
    lib.enet_rc_crc32_batch_device.argtypes = [vp, vp, vp, vp, sz, vp, vp]
    lib.enet_rc_crc32_batch_host.restype = C.c_int
    lib.enet_rc_crc32_batch_host.argtypes = [vp, vp, vp, vp, sz, vp]
    dg_dev = [vp, vp, vp, vp, sz, C.c_int, vp, vp, vp, vp, vp]
    dg_host = [vp, vp, vp, vp, sz, C.c_int, vp, vp, vp, vp]
    for name, args in (("enet_rc_datagram_encode_batch_device", dg_dev),
                       ("enet_rc_datagram_decode_batch_device", dg_dev),
                       ("enet_rc_datagram_encode_batch_host", dg_host),
                       ("enet_rc_datagram_decode_batch_host", dg_host)):
        f = getattr(lib, name)
        f.restype = C.c_int
        f.argtypes = args
    lib.enet_rc_socket_receive_batch.restype = C.c_int
    lib.enet_rc_socket_receive_batch.argtypes = [C.c_int, vp, sz, sz, vp, vp]
    lib.enet_rc_socket_send_batch.restype = C.c_int
    lib.enet_rc_socket_send_batch.argtypes = [C.c_int, vp, vp, vp, vp, sz]
    lib.enet_rc_crc32.restype = u32
    lib.enet_rc_crc32.argtypes = [C.POINTER(ENetBuffer), sz]
    lib.enet_rc_multi_create.restype = vp
    lib.enet_rc_multi_create.argtypes = [vp, sz]
    lib.enet_rc_multi_destroy.restype = None
    lib.enet_rc_multi_destroy.argtypes = [vp]
    lib.enet_rc_multi_devices.restype = sz
    lib.enet_rc_multi_devices.argtypes = [vp]
    lib.enet_rc_multi_split.restype = C.c_int
    lib.enet_rc_multi_split.argtypes = [vp, sz, sz, vp]
    for name in ("enet_rc_multi_plan", "enet_rc_multi_plan_device"):
        getattr(lib, name).restype = C.c_int
        getattr(lib, name).argtypes = [vp, vp, vp, vp, sz, sz, vp]
    for name, args in (("enet_rc_multi_compress_batch_host", batch_host),
                       ("enet_rc_multi_decompress_batch_host", batch_host),
                       ("enet_rc_multi_compress_batch_device", batch_dev[:-1]),
                       ("enet_rc_multi_decompress_batch_device", batch_dev[:-1]),
                       ("enet_rc_multi_compress_batch_device_stream", batch_dev),
                       ("enet_rc_multi_decompress_batch_device_stream", batch_dev)):
        f = getattr(lib, name)
        f.restype = C.c_int
        f.argtypes = args
    lib.enet_rc_pack_batch_device.restype = C.c_int
    lib.enet_rc_pack_batch_device.argtypes = [vp, vp, vp, vp, sz, vp, vp]
    lib.enet_rc_last_exact_count.restype = u32
    lib.enet_rc_last_exact_count.argtypes = [vp]
    lib.enet_rc_last_lane_count.restype = u32
    lib.enet_rc_last_lane_count.argtypes = [vp]
    lib.enet_rc_config_flags.restype = u32
    lib.enet_rc_config_flags.argtypes = [vp]
    lib.enet_rc_last_split.restype = u32
    lib.enet_rc_last_split.argtypes = [vp]
    lib.enet_rc_last_host_paths.restype = u32
    lib.enet_rc_last_host_paths.argtypes = [vp]
    lib.enet_rc_debug_counter.restype = u32
    lib.enet_rc_debug_counter.argtypes = [vp, u32]
    lib.enet_rc_version.restype = C.c_char_p
    lib.enet_rc_version.argtypes = []
    lib.rc_hip_lds_bytes.restype = u32
    lib.rc_hip_lds_bytes.argtypes = [u32]
    return lib


_LIB = None


def get_lib() -> C.CDLL:
    """Loads the product library on first use; raises if it is not built."""
    global _LIB
    if _LIB is None:
        _LIB = _load()
    return _LIB


def header_symbols() -> list:
    """Function names declared by include/enet_rc_amd.h."""
    with open(HEADER) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(\w+)\s*\(", text, flags=re.M)
    skip = {"compress", "decompress", "destroy", "if", "typedef"}
    return sorted({n for n in names if n not in skip and not n.startswith("_")})
