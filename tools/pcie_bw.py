"""PCIe / host-copy / registration rates on the GPU box (diagnostic for the
host-pointer path, rc_host.c run_host)."""
import ctypes as C, time
import numpy as np, torch
hip = C.CDLL("libamdhip64.so")
n = 80 << 20
a = np.random.randint(0, 255, n, dtype=np.uint8)
pin = torch.empty(n, dtype=torch.uint8).pin_memory()
dev = torch.empty(n, dtype=torch.uint8, device="cuda")
for _ in range(2):
    torch.cuda.synchronize(); t = time.perf_counter(); dev.copy_(pin, non_blocking=True); torch.cuda.synchronize()
    h2d = time.perf_counter() - t
    t = time.perf_counter(); pin.copy_(dev, non_blocking=True); torch.cuda.synchronize(); d2h = time.perf_counter() - t
    t = time.perf_counter(); np.copyto(pin.numpy(), a); cp = time.perf_counter() - t
print(f"pinned H2D {n/h2d/1e9:.1f} GB/s, D2H {n/d2h/1e9:.1f} GB/s, 1-thread host copy {n/cp/1e9:.1f} GB/s")
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
for _ in range(3):
    t = time.perf_counter(); r = hip.hipHostRegister(a.ctypes.data, n, 0); t1 = time.perf_counter()
    src = torch.from_numpy(a)
    torch.cuda.synchronize(); t2 = time.perf_counter(); dev.copy_(src, non_blocking=True); torch.cuda.synchronize(); t3 = time.perf_counter()
    hip.hipHostUnregister(a.ctypes.data); t4 = time.perf_counter()
    print(f"register rc={r} {1e3*(t1-t):.2f} ms, H2D from registered {n/(t3-t2)/1e9:.1f} GB/s, unregister {1e3*(t4-t3):.2f} ms")
t = time.perf_counter(); dev.copy_(torch.from_numpy(a)); torch.cuda.synchronize(); print(f"pageable H2D {n/(time.perf_counter()-t)/1e9:.1f} GB/s")
