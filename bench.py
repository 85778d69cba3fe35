#!/usr/bin/env python3
"""Device-resident range-coder throughput on MI355X (BASELINE.json metric).

One step = compress the whole packet batch, then decompress it back
(config C2: 65536 x 1200 B uniform-random packets per GPU, inputs resident in
HBM).  value = sum of uncompressed payload bytes of all ranks x steps / max
over ranks of the timed region, in GiB/s.

Multi-GPU (torchrun, one rank per GPU): every rank owns an independent
65536-packet shard (config C5, distinct seeds) and no collective runs inside
the timed region -- packets are independent (compress.c:252-265), so this is
weak scaling.  The RCCL scatter/gather of a batch from rank 0 is timed
separately and reported in "rccl_scatter_gather".

Extra fields: "roofline" (dominant kernel, algorithmic HBM bytes / measured
kernel time vs 8 TB/s), "cpu_baseline" (reference compress.c on host cores,
rank 0 only), "pcie_inclusive" (H2D + kernels + D2H from pinned memory),
"datagram_path" (whole ENet datagrams: GPU framing + checksum + coder, and the
UDP -> pinned staging -> GPU decode pipeline).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md); ~6.3 TB/s achievable
GIB = float(1 << 30)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", default="c2", choices=["c2", "c3", "c4"])
    p.add_argument("--packets", type=int, default=65536)
    p.add_argument("--size", type=int, default=1200)
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="cpu_baseline threads (0: every CPU in this process's affinity mask)")
    p.add_argument("--no-pcie", action="store_true")
    p.add_argument("--no-crc", action="store_true", help="skip the CRC-32 kernel line")
    p.add_argument("--no-rccl", action="store_true")
    p.add_argument("--no-dgram", action="store_true", help="skip the datagram-path leg")
    p.add_argument("--no-configs", action="store_true", help="skip the other BASELINE configs (C3, C4)")
    p.add_argument("--no-multi", action="store_true", help="skip the multi-GPU C-ABI leg")
    return p.parse_args()


def make_batch(kind, n, size, rank):
    from enet_amd import synth
    seed = synth.SEED + rank
    if kind == "c2":
        return synth.random_batch(n, size, seed=seed)
    if kind == "c3":
        return synth.gamestate_batch(n, size, seed=(synth.SEED ^ 0x47414D45) + rank)
    return synth.mixed_batch(n, seed=(synth.SEED ^ 0x4D495845) + rank)


def workload_name(kind, n=65536, size=1200):
    """The workload label; a packet count or size other than the config's is
    named as such (the C2/C3 shapes are 65536 x 1200 B)."""
    name = WORKLOADS[kind]
    if kind in ("c2", "c3") and (n, size) != (65536, 1200):
        name = name.replace("C2 65536x1200B", f"C2-shaped {n}x{size}B").replace("C3 65536x1200B",
                                                                               f"C3-shaped {n}x{size}B")
    return name


WORKLOADS = {"c2": "C2 65536x1200B uniform-random, compress+decompress round trip",
             "c3": "C3 65536x1200B game-state, compress+decompress round trip",
             "c4": "C4 1Mi mixed 64-1392B random, compress+decompress round trip"}


def run_workload(coder, dev, stream, kind, n, size, rank, steps, warmup, dist=None, world=1):
    """One workload: W untimed round trips, then K timed ones bracketed by
    (barrier +) synchronize.  Returns (raw timings, summary dict)."""
    import torch
    d, o, l = make_batch(kind, n, size, rank)
    n = len(l)
    max_len = int(l.max())
    din = torch.from_numpy(d).to(dev)
    doff = torch.from_numpy(o.astype(np.int64)).to(dev)
    dlen = torch.from_numpy(l.astype(np.int32)).to(dev)
    cap = (2 * dlen.to(torch.int64) + 64).to(torch.int32)
    coff = torch.zeros(n, dtype=torch.int64, device=dev)
    coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
    cout = torch.empty(int(coff[-1] + cap[-1]), dtype=torch.uint8, device=dev)
    clen = torch.zeros(n, dtype=torch.int32, device=dev)
    dout = torch.empty_like(din)
    dl = torch.zeros(n, dtype=torch.int32, device=dev)
    in_bytes = int(l.sum(dtype=np.uint64))

    # size the decoder's bound from the actual compressed lengths
    coder.compress_batch(din, doff, dlen, cout, coff, cap, clen, max_len=max_len, stream=stream)
    torch.cuda.synchronize()
    dec_max_len = int(clen.max().item())
    lanes = [0, 0]

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        coder.compress_batch(din, doff, dlen, cout, coff, cap, clen, max_len=max_len, stream=stream)
        if ev is not None:
            ev[1].record(stream)
        coder.decompress_batch(cout, coff, clen, dout, doff, dlen, dl, max_len=dec_max_len, stream=stream)
        if ev is not None:
            ev[2].record(stream)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    # correctness guard for the timed configuration, and the packets each
    # direction's fast kernel handed to the lane kernels
    ok = bool(torch.equal(dl, dlen)) and bool(torch.equal(dout, din))
    comp_bytes = int(clen.to(torch.int64).sum().item())
    lanes[1] = coder.last_lane_count()
    coder.compress_batch(din, doff, dlen, cout, coff, cap, clen, max_len=max_len, stream=stream)
    lanes[0] = coder.last_lane_count()

    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(events[k])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t_comp = sum(e[0].elapsed_time(e[1]) for e in events) / steps / 1e3
    t_dec = sum(e[1].elapsed_time(e[2]) for e in events) / steps / 1e3
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        okt = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())
    # roofline of the dominant kernel (whichever direction is slower): its
    # algorithmic bytes per launch -- compress reads N + offsets, writes C +
    # lengths; decompress reads C + offsets, writes N + lengths (SURVEY.md
    # §8d: 2(N+C) per round trip) -- over its HIP-event time on the stream
    # it runs on (the direction's fast kernel plus the empty lane/exact launches)
    meta = n * (8 + 4 + 8 + 4 + 4)
    alg = in_bytes + comp_bytes + meta
    dom_is_dec = t_dec >= t_comp
    t_dom = t_dec if dom_is_dec else t_comp
    achieved = alg / t_dom / 1e9
    kname = dominant_kernel(dom_is_dec, lanes[1] if dom_is_dec else lanes[0], n)
    roofline = {"kernel": kname, "bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 6), "alg_bytes_per_launch": alg,
                "launch_ms": round(t_dom * 1e3, 4)}
    traffic, tsrc = measured_traffic(kname, kind, n)
    roofline["traffic"] = traffic
    roofline["traffic_source"] = tsrc
    if traffic:
        # what the kernel actually moves: PMC HBM bytes per launch (separate
        # rocprofv3 --pmc passes of this workload) over this launch time
        rate = traffic / t_dom / 1e9
        roofline["traffic_GBps"] = round(rate, 1)
        roofline["traffic_frac_of_peak"] = round(rate / HBM_PEAK_GBPS, 4)
        roofline["traffic_over_alg"] = round(traffic / alg, 2)
    summary = {
        "workload": workload_name(kind, n, size), "packets": n, "value": round(in_bytes * world * steps / elapsed / GIB, 4),
        "unit": "GiB/s", "ms_per_step": round(elapsed / steps * 1e3, 4), "steps": steps, "warmup": warmup,
        "bit_exact_roundtrip": ok, "compression_ratio": round(comp_bytes / in_bytes, 5),
        "compress_GiBps": round(in_bytes / t_comp / GIB, 4), "decompress_GiBps": round(in_bytes / t_dec / GIB, 4),
        "compress_ms": round(t_comp * 1e3, 4), "decompress_ms": round(t_dec * 1e3, 4),
        "lane_handoff": {"compress": lanes[0], "decompress": lanes[1]},
        "roofline": roofline,
    }
    raw = dict(d=d, o=o, l=l, din=din, doff=doff, dlen=dlen, in_bytes=in_bytes, n=n, max_len=max_len,
               elapsed=elapsed, t_dom=t_dom, kname=kname)
    return raw, summary


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """`--gpus N` (N > 1) outside a torchrun job: one process per GPU, started
    here as torch.distributed.run's children before anything touches a GPU
    (the parent only counts devices, which does not initialise HIP), and the
    parent exits with their status.  Fewer than N visible GPUs: a message and
    exit status 2, never a one-GPU number under an N-GPU request.  Returns
    None when this process is to run the bench itself."""
    n = args.gpus
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if n > 1 and int(env_world) != n:
            print(f"bench.py: --gpus {n} but WORLD_SIZE={env_world}: launch one rank per requested GPU",
                  file=sys.stderr)
            return 2
        return None
    if n <= 1:
        return None
    if os.environ.get("ENET_BENCH_STUB") != "1":
        import torch
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} requested but {have} GPU(s) visible; refusing to report a "
                  f"{max(have, 1)}-GPU measurement as {n}-GPU", file=sys.stderr)
            return 2
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def stub_main(args):
    """ENET_BENCH_STUB=1 (CPU tests of the launcher, tests/test_bench_launch.py):
    the same rank/barrier/max-over-ranks reporting over gloo with a host
    memcpy in place of the coder; never a measurement of this library."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    src = np.full(1 << 16, rank, np.uint8)
    dst = np.empty_like(src)
    for _ in range(args.warmup):
        dst[:] = src
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dst[:] = src
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": "stub", "value": src.size * world * args.steps / max(float(t.item()), 1e-9) / GIB,
                          "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "data": "stub (launcher test: host memcpy, no coder)"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    rc = launch_ranks(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if os.environ.get("ENET_BENCH_STUB") == "1":
        return stub_main(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from enet_amd import RangeCoder

    coder = RangeCoder()
    stream = torch.cuda.current_stream(dev)
    raw, main_line = run_workload(coder, dev, stream, args.workload, args.packets, args.size, rank, args.steps,
                                  args.warmup, dist if world > 1 else None, world)
    d, o, l, din, doff, dlen = raw["d"], raw["o"], raw["l"], raw["din"], raw["doff"], raw["dlen"]
    n, in_bytes, max_len = raw["n"], raw["in_bytes"], raw["max_len"]
    roofline = main_line["roofline"]
    roofline["compress_ms"] = main_line["compress_ms"]
    roofline["decompress_ms"] = main_line["decompress_ms"]

    result = {
        "metric": "GiB/s device-resident range-coder (de)compress, 64Ki×1200B pkts, 1/2/4/8 GPU",
        "value": main_line["value"],
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": main_line["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": workload_name(args.workload, args.packets, args.size),
                   "packets_per_gpu": n, "packet_bytes": args.size if args.workload != "c4" else "64-1392",
                   "parallelism": f"shard{world}", "out_cap": "2N+64"},
        "bit_exact_roundtrip": main_line["bit_exact_roundtrip"],
        "compression_ratio": main_line["compression_ratio"],
        "compress_GiBps": main_line["compress_GiBps"],
        "decompress_GiBps": main_line["decompress_GiBps"],
        "lane_handoff": main_line["lane_handoff"],
        "roofline": roofline,
    }

    def leg(name, fn, *a):
        # side measurements never cost the main line: a failure is reported in place
        try:
            result[name] = fn(*a)
        except Exception as e:  # noqa: BLE001
            result[name] = {"error": f"{type(e).__name__}: {e}"}

    if world == 1 and not args.no_configs:
        # the other single-GPU BASELINE configs, measured in the same run
        # (C2 is the headline above); fewer steps: each is a full batch
        def other(kind, packets):
            del_keys = ("d", "o", "l", "din", "doff", "dlen")
            r, summ = run_workload(coder, dev, stream, kind, packets, 1200, rank, 3, 1)
            for k in del_keys:
                r.pop(k, None)
            torch.cuda.empty_cache()
            return summ
        cfg = {}
        for kind, packets in (("c2", 65536), ("c3", 65536), ("c4", 1 << 20)):
            if kind == args.workload:
                continue
            try:
                cfg[kind] = other(kind, packets)
            except Exception as e:  # noqa: BLE001
                cfg[kind] = {"error": f"{type(e).__name__}: {e}"}
        result["configs"] = cfg

    if not args.no_crc:
        leg("crc32", crc32_bench, coder, din, doff, dlen, in_bytes, n, stream)

    if rank == 0 and world == 1 and not args.no_pcie:
        leg("pcie_inclusive", pcie_inclusive, coder, d, o, l, args)

    if rank == 0 and world == 1 and not args.no_dgram:
        leg("datagram_path", datagram_path, coder, dev, stream)
        leg("per_datagram_call", per_datagram_call, coder, d, o, l)

    if not args.no_multi:
        # the single-process multi-GPU C entry (enet_rc_multi_*, rc_multi.c) over
        # every GPU of the job, driven from rank 0 (the other ranks wait)
        if world > 1:
            dist.barrier()
        if rank == 0:
            leg("multi_device_c_abi", multi_device_leg, list(range(world)), din, doff, dlen, max_len, in_bytes)
        if world > 1:
            dist.barrier()

    if world > 1 and not args.no_rccl:
        try:
            rs = rccl_scatter_gather(dist, dev, coder, din, doff, dlen, max_len, world, rank)
        except Exception as e:  # noqa: BLE001  (the main line is already measured)
            rs = {"error": f"{type(e).__name__}: {e}"}
        if rank == 0:
            result["rccl_scatter_gather"] = rs

    if rank == 0 and world == 1 and not args.no_cpu:
        leg("cpu_baseline", cpu_baseline, d, o, l, args.cpu_threads)

    if rank == 0:
        print(json.dumps(result), flush=True)
    coder.close()
    if world > 1:
        dist.destroy_process_group()


def multi_device_leg(devices, din, doff, dlen, max_len, in_bytes):
    """enet_rc_multi_{compress,decompress}_batch_device (rc_multi.c): the
    batch on devices[0], split by payload bytes, the other devices' ranges
    over the peer links (xGMI), coded, packed, gathered and unpacked back.
    Each call returns with its results in place; round trips timed on the host."""
    import torch
    from enet_amd import MultiCoder
    m = MultiCoder(devices)
    n = dlen.numel()
    cap = (2 * dlen.to(torch.int64) + 64).to(torch.int32)
    coff = torch.zeros(n, dtype=torch.int64, device=din.device)
    coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
    cout = torch.empty(int(coff[-1] + cap[-1]), dtype=torch.uint8, device=din.device)
    clen = torch.zeros(n, dtype=torch.int32, device=din.device)
    dout = torch.empty_like(din)
    dl = torch.zeros(n, dtype=torch.int32, device=din.device)
    m.batch_device(False, din, doff, dlen, cout, coff, cap, clen, max_len=max_len)
    dec_max_len = int(clen.max().item())         # (as the main line: known before the timed calls)
    torch.cuda.synchronize()
    best_c = best_d = None
    for it in range(4):
        t0 = time.perf_counter()
        m.batch_device(False, din, doff, dlen, cout, coff, cap, clen, max_len=max_len)
        t1 = time.perf_counter()
        m.batch_device(True, cout, coff, clen, dout, doff, dlen, dl, max_len=dec_max_len)
        t2 = time.perf_counter()
        if it:
            best_c = min(best_c or 1e9, t1 - t0)
            best_d = min(best_d or 1e9, t2 - t1)
    ok = bool(torch.equal(dl, dlen)) and bool(torch.equal(dout, din))
    m.close()
    return {"devices": devices, "value": round(in_bytes / (best_c + best_d) / GIB, 4), "unit": "GiB/s",
            "compress_GiBps": round(in_bytes / best_c / GIB, 4), "decompress_GiBps": round(in_bytes / best_d / GIB, 4),
            "bit_exact_roundtrip": ok,
            "note": "one process, one context per device; device pointers on devices[0], other ranges over "
                    "hipMemcpyPeerAsync (xGMI); the split computed on devices[0] (rc_multi_plan.hip, one "
                    "small D2H); includes the plan, copies and the closing syncs; best of 3"}


def crc32_bench(coder, din, doff, dlen, in_bytes, n, stream):
    """enet_crc32 of every packet of the same batch
    (rc_crc32_batch), device-resident.  Algorithmic bytes per launch: the
    payload + 12 B of offset/length read + 4 B written per packet."""
    import torch
    out = torch.empty(n, dtype=torch.int32, device=din.device)
    for _ in range(3):
        coder.crc32_batch(din, doff, dlen, out, stream=stream)
    reps = 20
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(stream)
    for _ in range(reps):
        coder.crc32_batch(din, doff, dlen, out, stream=stream)
    ev[1].record(stream)
    torch.cuda.synchronize()
    t = ev[0].elapsed_time(ev[1]) / reps / 1e3
    alg = in_bytes + 16 * n
    return {"kernel": "rc_crc32_batch", "ms": round(t * 1e3, 4), "GiBps": round(in_bytes / t / GIB, 3),
            "roofline": {"bound": "hbm", "achieved": round(alg / t / 1e9, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(alg / t / 1e9 / HBM_PEAK_GBPS, 4)}}


def datagram_path(coder, dev, stream):
    """whole ENet datagrams.  65536 assembled
    datagrams (4-B header with sentTime, 4-B checksum field, 1200 B of
    game-state commands; C3 payloads, so they compress) through
    enet_rc_datagram_encode_batch_device and back through _decode_ (protocol.c
    framing + range coder + enet_crc32), device-resident; then the host end:
    4096 wire datagrams over 127.0.0.1 -> recvmmsg into pinned staging -> H2D
    -> one decode batch -> D2H.  Rates count command (payload) bytes."""
    import socket
    import torch
    from enet_amd import io, synth
    n, size, hs = 65536, 1200, 8
    gd, go, gl = synth.gamestate_batch(n, size)
    dg = np.zeros((n, hs + size), np.uint8)
    dg[:, 0] = 0x80                                   # SENT_TIME, peer 0
    dg[:, 2:4] = 0x12
    dg[:, hs:] = gd.reshape(n, size)
    seeds = np.arange(n, dtype=np.uint32) * np.uint32(2654435761)
    din = torch.from_numpy(dg.reshape(-1)).to(dev)
    ln = torch.full((n,), hs + size, dtype=torch.int32, device=dev)
    off = torch.arange(n, dtype=torch.int64, device=dev) * (hs + size)
    seed = torch.from_numpy(seeds.view(np.int32)).to(dev)
    wire = torch.zeros_like(din)
    wl = torch.zeros(n, dtype=torch.int32, device=dev)
    back = torch.zeros(n * 4096, dtype=torch.uint8, device=dev)
    boff = torch.arange(n, dtype=torch.int64, device=dev) * 4096
    bl = torch.zeros(n, dtype=torch.int32, device=dev)

    def enc():
        coder.datagram_encode_batch(din, off, ln, wire, off, wl, checksum=True, seed=seed, stream=stream)

    def dec():
        coder.datagram_decode_batch(wire, off, wl, back, boff, bl, checksum=True, seed=seed, stream=stream)

    enc(); dec()
    torch.cuda.synchronize()
    ok = bool(torch.equal(bl, ln)) and bool(torch.equal(back.view(n, 4096)[:, hs:hs + size].reshape(-1),
                                                         din.view(n, hs + size)[:, hs:].reshape(-1)))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    reps = 3
    te = td = 0.0
    for _ in range(reps):
        ev[0].record(stream); enc(); ev[1].record(stream); dec(); ev[2].record(stream)
        torch.cuda.synchronize()
        te += ev[0].elapsed_time(ev[1]) / 1e3 / reps
        td += ev[1].elapsed_time(ev[2]) / 1e3 / reps
    cmd_bytes = n * size
    wire_bytes = int(wl.to(torch.int64).sum().item())
    res = {"datagrams": n, "command_bytes": size, "checksum": True,
           "encode_GiBps": round(cmd_bytes / te / GIB, 3), "decode_GiBps": round(cmd_bytes / td / GIB, 3),
           "wire_ratio": round(wire_bytes / (n * (hs + size)), 4), "roundtrip_ok": ok}
    # host end: UDP loopback -> recvmmsg into pinned staging -> GPU decode
    m = 4096
    wl_h = wl[:m].cpu().numpy()
    wire_h = wire.view(n, hs + size)[:m].cpu().numpy()
    pkts = [wire_h[i, :int(wl_h[i])].tobytes() for i in range(m)]
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 16 << 20)
    rx.bind(("127.0.0.1", 0))
    rx.setblocking(False)
    tx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    stage = torch.zeros(m * 4096, dtype=torch.uint8).pin_memory()
    sbuf = stage.numpy()
    out_h = torch.zeros(m * 4096, dtype=torch.uint8).pin_memory()
    ol_h = torch.zeros(m, dtype=torch.int32).pin_memory()
    best = None
    for _ in range(3):
        sent = 0
        for k in range(0, m, 512):                      # stay under the socket buffer
            sent += io.send_batch(tx.fileno(), pkts[k:k + 512], rx.getsockname())
        time.sleep(0.02)
        t0 = time.perf_counter()
        got, lens = 0, []
        while got < sent:
            r, lz, _ = io.receive_batch(rx.fileno(), sbuf[got * 4096:], 4096, min(256, sent - got))
            if r == 0:
                break
            lens += [int(x) for x in lz]
            got += r
        dv = stage[:got * 4096].to(dev, non_blocking=True)
        dl = torch.tensor(lens, dtype=torch.int32).to(dev, non_blocking=True)
        doff_ = boff[:got]
        coder.datagram_decode_batch(dv, doff_, dl, back, doff_, bl[:got], checksum=True, seed=seed[:got],
                                    stream=stream)
        out_h[:got * 4096].copy_(back[:got * 4096], non_blocking=True)
        ol_h[:got].copy_(bl[:got], non_blocking=True)
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        if got == m and (best is None or t < best):
            best = t
    rx.close()
    tx.close()
    ok_h = bool((ol_h.numpy() == hs + size).all())
    res["socket_pipeline"] = {"datagrams": m, "ok": ok_h,
                              "GiBps": round(m * size / best / GIB, 3) if best else None,
                              "note": "recvmmsg (256 per call) into pinned staging + H2D + GPU decode "
                                      "+ D2H of 4096-B slots, best of 3 (sender not timed)"}
    return res


def per_datagram_call(coder, d, o, l):
    """The drop-in surface as protocol.c uses it: one enet_range_coder_compress
    / _decompress call per 1200-B datagram (host memory in and out, one launch
    and two copies each).  Latency per call; the batch API is the throughput path."""
    import ctypes as C
    from enet_amd._lib import ENetBuffer
    lib = coder.lib
    m = 200
    src = [C.create_string_buffer(d[int(o[i]): int(o[i]) + int(l[i])].tobytes(), int(l[i])) for i in range(m)]
    bufs = [C.byref(ENetBuffer(C.cast(b, C.c_void_p), int(l[i]))) for i, b in enumerate(src)]
    out = C.create_string_buffer(4096)
    back = C.create_string_buffer(4096)
    for i in range(5):
        lib.enet_range_coder_compress(coder.ctx, bufs[i], 1, int(l[i]), out, 4096)
    t0 = time.perf_counter()
    sizes = [lib.enet_range_coder_compress(coder.ctx, bufs[i], 1, int(l[i]), out, 4096) for i in range(m)]
    t1 = time.perf_counter()
    packed = []
    for i in range(m):
        r = lib.enet_range_coder_compress(coder.ctx, bufs[i], 1, int(l[i]), out, 4096)
        packed.append(C.create_string_buffer(out.raw[:r], r))
    t2 = time.perf_counter()
    ok = True
    for i in range(m):
        r = lib.enet_range_coder_decompress(coder.ctx, packed[i], sizes[i], back, 4096)
        ok = ok and r == int(l[i]) and back.raw[:r] == src[i].raw
    t3 = time.perf_counter()
    return {"datagram_bytes": int(l[0]), "calls": m, "compress_us": round((t1 - t0) / m * 1e6, 1),
            "decompress_us": round((t3 - t2) / m * 1e6, 1), "roundtrip_ok": ok}


def pcie_inclusive(coder, d, o, l, args):
    """Rate including H2D of the input and D2H of the output (the reference
    path starts and ends in host memory): from ordinary pageable caller
    buffers (`value`), and from caller buffers that are page-locked already
    (`pinned_caller`: an application's long-lived receive / send buffers,
    allocated pinned once), which the library DMAs directly."""
    from enet_amd import get_lib
    import ctypes as C
    import torch
    lib = get_lib()
    n = len(l)
    cap = (2 * l.astype(np.int64) + 64).astype(np.uint32)
    coff = np.zeros(n, np.uint64)
    coff[1:] = np.cumsum(cap[:-1], dtype=np.uint64)
    lcap = l.astype(np.uint32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731

    def measure(alloc):
        src = alloc(d.size)
        src[:] = d
        cout = alloc(int(coff[-1] + cap[-1]))
        clen = np.zeros(n, np.uint32)
        dout = alloc(d.size)
        dlen = np.zeros(n, np.uint32)
        best_c = best_d = 1e9
        for _ in range(5):
            t0 = time.perf_counter()
            rc = lib.enet_rc_compress_batch_host(coder.ctx, p(src), p(o), p(lcap), n, p(cout), p(coff), p(cap), p(clen))
            t1 = time.perf_counter()
            rc |= lib.enet_rc_decompress_batch_host(coder.ctx, p(cout), p(coff), p(clen), n, p(dout), p(o), p(lcap),
                                                    p(dlen))
            t2 = time.perf_counter()
            assert rc == 0
            best_c, best_d = min(best_c, t1 - t0), min(best_d, t2 - t1)
        ok = bool(np.array_equal(dlen, lcap) and np.array_equal(dout, d))
        return best_c, best_d, ok

    nb = float(l.sum(dtype=np.uint64))
    bc, bd, ok = measure(lambda k: np.zeros(k, np.uint8))
    res = {"value": round(nb / (bc + bd) / GIB, 4), "unit": "GiB/s",
           "compress_GiBps": round(nb / bc / GIB, 4), "decompress_GiBps": round(nb / bd / GIB, 4),
           "bit_exact": ok, "note": "enet_rc_*_batch_host from pageable caller buffers, through the library's "
                   "pinned staging (host copies on the pieces' threads, DMA, kernels, DMA, host copies; caller "
                   "memory is not page-locked per call by default, DESIGN.md 2a); best of 5 (the first call "
                   "creates the pieces' contexts)"}
    pc, pd, pok = measure(lambda k: torch.zeros(k, dtype=torch.uint8).pin_memory().numpy())
    res["pinned_caller"] = {"value": round(nb / (pc + pd) / GIB, 4), "compress_GiBps": round(nb / pc / GIB, 4),
                            "decompress_GiBps": round(nb / pd / GIB, 4), "bit_exact": pok,
                            "note": "the same calls with the caller's data buffers page-locked beforehand "
                                    "(pinned host memory): a back-to-back input DMA'd directly, other gapped "
                                    "inputs gathered by a GPU kernel over PCIe; outputs that fill their slots "
                                    "DMA'd into place, others written into the caller's slots by a GPU kernel; "
                                    "best of 5"}
    return res


def rccl_scatter_gather(dist, dev, coder, din, doff, dlen, max_len, world, rank):
    """End-to-end sharded pipeline from one root GPU: rank 0 scatters a batch
    of world x (this shard's packets) over RCCL (grouped isend/irecv on the
    direct xGMI links), every rank compresses its shard, and the compressed
    packets are gathered back to rank 0 (enet_amd/shard.py).  Reported beside
    the device-resident number; not part of the timed region of `value`."""
    import torch
    from enet_amd import shard
    n = dlen.numel()
    if rank == 0:
        big = din.repeat(world)
        blen = dlen.repeat(world)
        boff = torch.zeros_like(blen, dtype=torch.int64)
        boff[1:] = torch.cumsum(blen[:-1].to(torch.int64), 0)
    else:
        big = boff = blen = None
    best = None
    for it in range(3):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pay, poff, pln = shard.scatter_batch(dist, big, boff, blen, device=dev)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        cap = (2 * pln.to(torch.int64) + 64).to(torch.int32)
        coff = torch.zeros(pln.numel(), dtype=torch.int64, device=dev)
        coff[1:] = torch.cumsum(cap[:-1].to(torch.int64), 0)
        cout = torch.empty(int(coff[-1] + cap[-1]), dtype=torch.uint8, device=dev)
        clen = torch.zeros_like(pln)
        coder.compress_batch(pay, poff, pln, cout, coff, cap, clen, max_len=max_len)
        res, rl = shard.pack_results(cout, coff, clen, coder=coder)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        parts = shard.gather_results(dist, res, rl)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        tt = torch.tensor([t1 - t0, t2 - t1, t3 - t2], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        if it > 0 and (best is None or tt.sum() < sum(best)):
            best = [float(x) for x in tt.tolist()]
    payload = float(dlen.to(torch.int64).sum().item()) * world
    sc, co, ga = best
    return {"scatter_ms": round(sc * 1e3, 3), "compress_ms": round(co * 1e3, 3), "gather_ms": round(ga * 1e3, 3),
            "end_to_end_GiBps": round(payload / (sc + co + ga) / GIB, 4),
            "scatter_GBps": round(payload * (world - 1) / world / sc / 1e9, 2),
            "packets": n * world,
            "note": "rank0 scatters world x shard over RCCL (xGMI), ranks compress, results gathered to rank0; "
                    "separate from the timed region of value"}


def dominant_kernel(decompress, handed_off=0, n=1):
    """The kernel that does most of a direction's work in the library's
    configuration (rc_host.c / rc_enc2.hip read the same environment): the
    fast kernel, or the lane kernel when the fast kernel handed most packets
    to it (C3 today)."""
    if os.environ.get("ENET_RC_KERNEL", "lane3") == "wave":
        return "rc_decompress_wave" if decompress else "rc_compress_wave"
    if decompress:
        fast = (os.environ.get("ENET_RC_DEC4", "1") != "0" and os.environ.get("ENET_RC_DEC", "1") != "0"
                and os.environ.get("ENET_RC_LANES", "64") == "64")
        return "rc_decompress_dec6s" if fast and 2 * handed_off < n else "rc_decompress_lane3"
    if os.environ.get("ENET_RC_ENC2", "1") == "0" or 2 * handed_off >= n:
        return "rc_compress_lane3"
    one = os.environ.get("ENET_RC_ENC2_CODE1") == "1" or os.environ.get("ENET_RC_ENC2_LANES") == "32"
    return "rc_enc2_code" if one else "rc_enc2_code2"


def measured_traffic(kernel, workload, packets):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary of this workload (profiles/traffic_<workload>.json, written by
    tools/traffic.py from separate --pmc passes of the same bench workload,
    tools/evidence.sh), or None."""
    path = os.path.join(ROOT, "profiles", f"traffic_{workload}.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None
    if t.get("workload") != workload or t.get("packets") != packets:
        return None, None
    k = t.get("kernels", {}).get(kernel)
    if not k:
        return None, None
    return k.get("hbm_bytes_per_launch"), f"profiles/traffic_{workload}.json (" + t.get("source", "") + ")"


def cpu_threads_available():
    """The host CPUs this process may use: its affinity mask, capped by the
    cgroup's CPU quota (cpu.max) -- the GPU box's CPU share, not
    os.cpu_count()'s whole machine."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
            if path.endswith("cpu.max") and parts and parts[0] != "max":
                n = min(n, max(1, int(int(parts[0]) // int(parts[1]))))
            elif path.endswith("cfs_quota_us") and parts and int(parts[0]) > 0:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as g:
                    n = min(n, max(1, int(parts[0]) // int(g.read().split()[0])))
            break
        except (OSError, ValueError, IndexError):
            continue
    return n


def cpu_baseline(d, o, l, threads):
    """Reference compress.c (oracle/_ref/libenet_ref.so, built from the
    reference sources by `make -C oracle ref` in the build container and
    shipped with the tree), timed round trip on host cores: on one thread over
    a bounded sample (the first 8192 packets of the batch), and on `threads`
    threads (default: every CPU in this process's affinity mask; one context
    each) over the whole batch.  ENET_RC_CPU_BASELINE=port times the oracle
    restatement instead; without either the leg fails rather than silently
    timing something else."""
    from oracle.pyoracle import cpu_roundtrip, have_reference
    want = os.environ.get("ENET_RC_CPU_BASELINE", "reference")
    if want == "reference" and not have_reference():
        raise RuntimeError("oracle/_ref/libenet_ref.so is missing: build it with `make -C oracle ref` "
                           "(or set ENET_RC_CPU_BASELINE=port to time the restatement)")
    kind = "reference" if want == "reference" else "port"
    avail = cpu_threads_available()
    threads = max(1, min(threads or avail, avail))
    try:
        model = [x for x in open("/proc/cpuinfo").read().splitlines() if x.startswith("model name")][0].split(":")[1].strip()
    except Exception:
        model = "unknown"

    def one(m, k):
        r = cpu_roundtrip(d, o[:m], l[:m], k, kind=kind)
        nb = float(l[:m].sum(dtype=np.uint64))
        t = r["t_compress"] + r["t_decompress"]
        return {"value": round(nb / t / GIB, 5), "cores": k, "packets": int(m),
                "compress_GiBps": round(nb / r["t_compress"] / GIB, 5),
                "decompress_GiBps": round(nb / r["t_decompress"] / GIB, 5),
                "mismatches": int(r["mismatches"])}

    single = one(min(len(l), 8192), 1)
    multi = one(len(l), threads)
    return {"value": multi["value"], "unit": "GiB/s", "cores": threads, "kind": kind,
            "sample": f"{len(l)} packets x {int(l.max())} B (the bench batch) on {threads} threads, one context "
                      f"per thread; single_thread: its first {single['packets']} packets on one thread",
            "compress_GiBps": multi["compress_GiBps"], "decompress_GiBps": multi["decompress_GiBps"],
            "mismatches": multi["mismatches"] + single["mismatches"], "single_thread": single,
            "host_cpus_available": avail, "host_cpus_visible": os.cpu_count(), "cpu": model}


if __name__ == "__main__":
    main()
