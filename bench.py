#!/usr/bin/env python3
"""Benchmark of the MI355X /tile pipeline (BASELINE.json metric).

Workload per GPU (weak scaling, one process per GPU, no collectives on the data path):
a 32768 x 32768 uint16 G_NOISE plane generated in HBM, and one batch = the 4096 tiles of
its 64 x 64 grid of 512 x 512 tiles, each encoded to PNG (APNGWriter layout, filter None
as the reference, zlib-compatible deflate).  A step = plan the 4096 requests on the host
(TileRequestHandler validation + descriptors) + descriptor upload + every kernel, outputs
left in HBM.  Inputs are resident before the timed region; D2H is reported separately.

    python bench.py [--gpus N] [--steps K] [--warmup W]

One rank per GPU.  Under torch.distributed.run (WORLD_SIZE set) this process is one rank.
Otherwise `--gpus N` with N > 1 makes this process a launcher that touches no GPU: it
starts N rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment),
and only rank 0 prints the JSON line.  Ranks only meet at the barrier and the max-over-ranks
of the step time (gloo, CPU tensors): no collective on the data path.  `--dry-run` runs the
rank plumbing (launch, barrier, max) without any HIP call (CPU test of the N > 1 path).
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402  (loads the HIP runtime the library then shares)
import torch.distributed as dist  # noqa: E402

import pbx  # noqa: E402

METRIC = "tiles/sec (512x512 uint16 PNG) + achieved HBM GB/s at 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
TILE, GRID = 512, 64
KSTREAMS, KSTAGGER = int(os.environ.get("PBX_KSTREAMS", "3")), int(os.environ.get("PBX_KSTAGGER", "1"))  # the library's defaults
PIPE_DEPTH = int(os.environ.get("PBX_BENCH_DEPTH", "2"))  # batches in flight
HEADLINE_SUB = int(os.environ.get("PBX_BENCH_SUB", "0"))  # headline sub-batch tiles (0: one batch per step)


def grid_ctxs(image_id, fmt, n=GRID * GRID, tile=TILE):
    return [pbx.TileCtx(image_id, 0, 0, 0, (i % GRID) * tile, (i // GRID) * tile, tile, tile,
                        format=fmt) for i in range(n)]


class StepStats:
    """pbx_batch_stats summed over the sub-batches of one step (counts, bytes and kernel ms)."""

    def __init__(self, parts):
        for f, _ in pbx.PbxBatchStats._fields_:
            setattr(self, f, sum(getattr(p, f) for p in parts))


def run_steps(svc, ctxs, steps, warmup, barrier, sub=0):
    """Warmup, then `steps` timed steps; returns (seconds, per-step stats, mean host ms).

    Steps are pipelined PIPE_DEPTH deep, as a server feeds its GPU: the host plans and
    launches batch k+1 (request validation, descriptors, upload) while earlier batches run,
    then waits for the oldest one (its own completion event).  The request arrays are built
    once.  sub > 0: a step's requests go as batches of `sub` tiles (PIPE_DEPTH steps' worth
    in flight); its stats are their sums."""
    parts = [ctxs] if sub <= 0 else [ctxs[i:i + sub] for i in range(0, len(ctxs), sub)]
    reqs = [pbx.make_reqs(p) for p in parts]
    depth = PIPE_DEPTH * len(parts)

    def one_pass(n, record):
        q = []
        host = 0.0
        out = []
        acc = []

        def retire():
            b = q.pop(0)
            b.sync()
            if record:
                acc.append(b.stats())
                if len(acc) == len(parts):
                    out.append(acc[0] if len(parts) == 1 else StepStats(acc))
                    acc.clear()
            b.close()

        for _ in range(n):
            for r in reqs:
                t0 = time.perf_counter()
                b = pbx.Batch(svc, reqs=r)
                b.launch()
                host += time.perf_counter() - t0
                q.append(b)
                if len(q) >= depth:
                    retire()
        while q:
            retire()
        return out, host

    if warmup:
        one_pass(warmup, False)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats, host = one_pass(steps, True)
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    return dt, stats, 1000.0 * host / len(stats)


def mean(stats, field):
    return sum(getattr(s, field) for s in stats) / len(stats)


def secondary_steps(svc, ctxs, steps, warmup, barrier):
    """run_steps for a secondary line: at least PIPE_DEPTH warmup batches, so that every
    batch the timed pass keeps in flight finds its device and pinned pool blocks already
    allocated (a fresh service with one warmup batch allocated the second in-flight batch's
    ~4 GB of blocks inside the timed region: BENCH_r02's adaptive line read 53k tiles/s for
    8 ms of kernels per 4096 tiles)."""
    return run_steps(svc, ctxs, steps, max(warmup, PIPE_DEPTH), barrier)


def wall_vs_kernels(dt, steps, stats, world=1):
    """Wall time per step next to the batch's own kernel time (HIP events, first to last
    kernel of one batch); a line whose wall time exceeds 1.5x its kernels is flagged: it is
    then measuring something other than the kernels it names."""
    wall = 1e3 * dt / steps
    kern = mean(stats, "ms_total")
    out = {"wall_ms_per_step": round(wall, 3), "kernel_ms_per_step": round(kern, 3),
           "wall_over_kernels": round(wall / kern, 3) if kern else None}
    if kern and wall > 1.5 * kern:
        out["flag"] = "wall time > 1.5x the batch's kernel time: not a kernel measurement"
    return out


def e2e_rate(svc, ctxs, batches=6):
    """End-to-end incl. D2H into pinned host memory (PCIe-inclusive; never the headline):
    batches pipelined two deep, batch k's D2H (copy stream) overlapping batch k+1's
    kernels, after two warmup batches (pinned pool populated)."""
    reqs = pbx.make_reqs(ctxs)
    q, nbytes, t0 = [], 0, None
    for k in range(batches + 2 + 1):
        if k == 2:
            torch.cuda.synchronize()
            t0, nbytes = time.perf_counter(), 0
        if k < batches + 2:
            b = pbx.Batch(svc, reqs=reqs)
            b.launch()
            q.append(b)
        if len(q) == 2 or (k == batches + 2 and q):
            f = q.pop(0)
            nbytes += f.fetch_into_host()
            f.close()
    while q:
        f = q.pop(0)
        nbytes += f.fetch_into_host()
        f.close()
    dt = time.perf_counter() - t0
    return len(ctxs) * batches / dt, nbytes / dt / 1e9


def load_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (profiles/*pmc*/traffic.json, written by scripts/pmc_summary.py: FETCH_SIZE doubled
    per the gfx950 rule + WRITE_SIZE, same workload as this bench's batch)."""
    import glob
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*", "traffic.json")), reverse=True):
        with open(fn) as f:
            k = json.load(f).get("kernels", {}).get(kernel)
        if k:  # the latest pass that profiled this kernel (filter-only passes hold no k_encode)
            return k["fetch_bytes"] + k["write_bytes"], os.path.relpath(fn, ROOT)
    return None, None


CHAIN_KERNELS = ("k_seg_map", "k_lz77", "k_huff", "k_seg_sizes", "k_scan_offsets", "k_encode", "k_frame")


def load_chain_traffic():
    """HBM bytes per launch of the whole deflate chain (every kernel of a headline batch) from
    the latest committed PMC passes that profiled it: (bytes, source)."""
    import glob
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*", "traffic.json")), reverse=True):
        with open(fn) as f:
            ks = json.load(f).get("kernels", {})
        if "k_lz77" in ks and "k_encode" in ks:
            return (sum(ks[k]["fetch_bytes"] + ks[k]["write_bytes"] for k in CHAIN_KERNELS if k in ks),
                    os.path.relpath(fn, ROOT))
    return None, None


def load_issue(kernels=("k_encode", "k_lz77")):
    """The issue roofline of the deflate kernels from the latest committed PMC passes
    (profiles/*pmc*/issue.json, scripts/pmc_summary.py: VALU busy = 2 cycles per wave64 VALU
    instruction per SIMD-cycle, SALU busy = 1 per CU-cycle, wave-time split), same workload."""
    import glob
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*", "issue.json")), reverse=True):
        with open(fn) as f:
            t = json.load(f)
        out = {k: t["kernels"][k] for k in kernels if k in t.get("kernels", {})}
        if out:  # the latest pass that profiled the deflate kernels
            out["source"] = os.path.relpath(fn, ROOT)
            out["rule"] = t.get("rule")
            return out
    return None


def load_rocprof_ms(kernel):
    """The rocprofv3 kernel-trace average (ms) of `kernel` in the latest committed summary of
    the headline's serial pass (profiles/*/kernel_stats.csv, PBX_KSTREAMS=1): (ms, source)."""
    import csv
    import glob
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "kernel_stats.csv")), reverse=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                name = row.get("Name", "")
                if f"::{kernel}<" in name or f"::{kernel}(" in name:
                    return float(row["AverageNs"]) * 1e-6, os.path.relpath(fn, ROOT)
    return None, None


def cpu_model():
    """The host CPU model string (quote the CPU with the baseline)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _timed_oracle(run, seconds, threads):
    """Calibrate on a short run, then time ~`seconds` of work: (items, seconds, bytes)."""
    n0 = 2 * threads
    sec, _ = run(n0)
    n = max(threads, int(n0 / sec * seconds))
    sec, nbytes = run(n)
    return n, sec, nbytes


def cpu_baseline(seconds=10.0, threads=16):
    """The C oracle (zlib-6 filter-None PNG, same region extraction) on host threads: the
    headline's 512x512 uint16 G_NOISE tiles on `threads` threads (the reported value), and on
    one thread, and G_FAKE tiles; the CPU model is stated."""
    import _oracle as O
    O.lib()
    pw = ph = 4096

    def grid(kind, th):
        return lambda n: O.bench(kind, O.UINT16, O.FMT_PNG, pw, ph, TILE, TILE, n, th)

    n, sec, nbytes = _timed_oracle(grid(O.GEN_NOISE, threads), seconds, threads)
    n1, sec1, _ = _timed_oracle(grid(O.GEN_NOISE, 1), seconds / 2, 1)
    nf, secf, nbf = _timed_oracle(grid(O.GEN_FAKE, threads), seconds / 4, threads)
    return {"value": round(n / sec, 2), "unit": "tiles/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(),
            "single_thread": {"value": round(n1 / sec1, 2), "unit": "tiles/s", "cores": 1,
                              "sample": f"{n1} G_NOISE tiles, {sec1:.1f} s"},
            "g_fake": {"value": round(nf / secf, 2), "unit": "tiles/s", "cores": threads,
                       "sample": f"{nf} 512x512 uint16 G_FAKE tiles -> PNG, {secf:.1f} s; "
                                 f"avg {nbf / nf:.0f} B/tile"},
            "sample": f"{n} tiles 512x512 uint16 G_NOISE -> PNG (filter None, zlib level 6) "
                      f"from a 4096x4096 plane, oracle/pbx_oracle.c on {threads} threads, "
                      f"{sec:.1f} s; avg {nbytes / n:.0f} B/tile"}


def c1_line(svc, rank, world, barrier, threads=16, reps=2000):
    """BASELINE configs[0] at its own workload: ONE 512x512 uint8 PNG request, tile (0, 0) of a
    4096^2 Bio-Formats-fake (G_FAKE) plane, repeated (TileRequestHandler.java:119-124,
    176-199).  GPU: (a) one caller in a loop through pbx_get_tile (the coalescer, D2H and the
    JNI-style body copy included; native loop), p50/p99 latency; (b) the request repeated 1024x
    in one device-resident batch, as the coalescer forms it under load.  CPU: the oracle for
    the same request on 1 thread and on `threads` threads, with the CPU model."""
    iid = 6
    side = 4096
    svc.register_plane(iid, 0, 0, 0, pbx.UINT8, side, side, generator="fake", plane_no=0)
    tc = pbx.TileCtx(iid, 0, 0, 0, 0, 0, TILE, TILE, format="png")
    one = serve_one(svc, [tc], 1, reps, 200)
    ctxs = [tc] * 1024
    dt, st, _ = secondary_steps(svc, ctxs, 5, 2, barrier)
    line = {"request": "tile (0,0,512,512) uint8 png of a 4096^2 G_FAKE plane",
            "single_caller_get_tile": one,
            "batched_1024_repeats": {"tiles_per_s": round(len(ctxs) * 5 * world / dt, 1),
                                     **wall_vs_kernels(dt, 5, st),
                                     "bytes_per_tile": round(st[-1].deflate_out_bytes / len(ctxs), 1)}}
    if rank == 0 and world == 1:
        import _oracle as O
        O.lib()
        cpu = {}
        for th in (1, threads):
            n, sec, nbytes = _timed_oracle(
                lambda k: O.bench_at(O.GEN_FAKE, O.UINT8, O.FMT_PNG, side, side, 0, 0, TILE, TILE, k, th),
                3.0, th)
            cpu[f"threads_{th}"] = {"tiles_per_s": round(n / sec, 1), "cores": th,
                                    "latency_ms": round(1e3 * sec * th / n, 3),
                                    "bytes_per_tile": round(nbytes / n, 1), "sample": f"{n} requests, {sec:.1f} s"}
        cpu["kind"] = "port"
        cpu["cpu_model"] = cpu_model()
        line["cpu_oracle"] = cpu
        line["gpu_over_cpu_1_thread_latency"] = round(cpu["threads_1"]["latency_ms"] / one["p50_ms"], 2)
    svc.release_plane(svc.lookup_plane(iid, 0, 0, 0)[0])
    return line


def zarr_lines(svc, rank, world, side=16384, chunk=512, reps=3):
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    import _zarr
    pid = svc.register_plane(20, 0, 0, 0, pbx.UINT16, side, side, generator="noise", plane_no=rank)
    plane = np.frombuffer(svc.read_plane_be(pid, side * side * 2), ">u2").reshape(side, side)
    svc.release_plane(pid)
    grid = _zarr.chunk_grid(plane, chunk, chunk)
    res = {}
    codecs = [("blosc_lz4", "blosc", {}), ("zlib1", "zlib", {"level": 1})]
    if _zarr.cblosc() is not None:  # chunks written by the real c-blosc 1.21
        codecs += [("blosc_zstd5", "blosc", {"cname": "zstd", "clevel": 5, "shuffle": 1}),
                   ("blosc_blosclz5", "blosc", {"cname": "blosclz", "clevel": 5, "shuffle": 1}),
                   ("blosc_lz4_bitshuffle", "blosc", {"cname": "lz4", "clevel": 5, "shuffle": 2})]

    def enc(c, comp, kw):
        if comp == "zlib":
            return _zarr.zlib_encode(c.tobytes(), 1)
        if "cname" in kw:
            return _zarr.cblosc_encode(c.tobytes(), 2, kw["cname"], kw["clevel"], kw["shuffle"])
        return _zarr.blosc_encode(c.tobytes(), 2)

    for name, comp, kw in codecs:
        with ThreadPoolExecutor(16) as ex:
            chunks = list(ex.map(lambda c: enc(c, comp, kw), grid))
        cbytes = sum(len(c) for c in chunks)
        packed = pbx.pack_chunks(chunks)  # the C-ABI's form: the chunk files back to back
        dec, plc, wall = [], [], []
        for r in range(reps + 1):
            t0 = time.perf_counter()
            pid, (md, mp) = svc.register_zarr_plane(21, 0, 0, 0, pbx.UINT16, side, side, chunk, chunk,
                                                    comp, packed, timing=True)
            t1 = time.perf_counter()
            if r:
                dec.append(md)
                plc.append(mp)
                wall.append(t1 - t0)
            svc.release_plane(pid)
        raw = side * side * 2
        md, mp = sum(dec) / reps, sum(plc) / reps
        line = {"chunks": len(chunks), "compressed_bytes": cbytes, "decoded_bytes": raw,
                "decode_ms": round(md, 3), "place_ms": round(mp, 3),
                "decoded_gbps": round(raw / ((md + mp) * 1e-3) / 1e9, 1),
                "chunks_per_s": round(len(chunks) * world / ((md + mp) * 1e-3), 1),
                "decode_alg_gbps": round((cbytes + raw) / (md * 1e-3) / 1e9, 1),
                "place_gbps": round(2 * raw / (mp * 1e-3) / 1e9, 1),
                "register_wall_ms_incl_upload": round(1e3 * sum(wall) / reps, 1)}
        if rank == 0 and world == 1:
            import _oracle as O
            L = O.lib()
            import ctypes
            L.pbxo_zarr_bench.restype = ctypes.c_double
            L.pbxo_zarr_bench.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_void_p,
                                          ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]
            n = 256  # bounded sample: a quarter of the chunks
            sub = chunks[:n]
            offs = np.concatenate([[0], np.cumsum([len(c) for c in sub])]).astype(np.uint64)
            sec = L.pbxo_zarr_bench({"blosc": 1, "zlib": 2}[comp], b"".join(sub), offs.ctypes.data,
                                    n, chunk * chunk * 2, 16)
            line["cpu_baseline"] = {"value": round(n * chunk * chunk * 2 / sec / 1e9, 2), "unit": "GB/s",
                                    "chunks_per_s": round(n / sec, 1), "cores": 16, "kind": "port",
                                    "sample": f"{n} of the same chunks, oracle/zarr_oracle.c "
                                              f"(c-blosc frame restatement / zlib 1.2.11) on 16 threads"}
        res[name] = line
    # compressible data: the FakeReader-like gradient plane (G_FAKE) in blosc-lz4 chunks
    pid = svc.register_plane(23, 0, 0, 0, pbx.UINT16, side, side, generator="fake", plane_no=rank)
    fake = np.frombuffer(svc.read_plane_be(pid, side * side * 2), ">u2").reshape(side, side)
    svc.release_plane(pid)
    with ThreadPoolExecutor(16) as ex:
        fchunks = list(ex.map(lambda c: _zarr.blosc_encode(c.tobytes(), 2),
                              _zarr.chunk_grid(fake, chunk, chunk)))
    dec, plc = [], []
    for r in range(reps + 1):
        pid, (md, mp) = svc.register_zarr_plane(24, 0, 0, 0, pbx.UINT16, side, side, chunk, chunk,
                                                "blosc", fchunks, timing=True)
        if r:
            dec.append(md)
            plc.append(mp)
        svc.release_plane(pid)
    md, mp = sum(dec) / reps, sum(plc) / reps
    res["blosc_lz4_fake_gradient"] = {
        "compressed_bytes": sum(len(c) for c in fchunks), "decode_ms": round(md, 3),
        "place_ms": round(mp, 3),
        "decoded_gbps": round(side * side * 2 / ((md + mp) * 1e-3) / 1e9, 1)}
    # the same chunks for 4 planes (4 x 512 MiB) in ONE pbx_planes_register_zarr call: 4x the
    # streams in flight hide the per-stream decode latency
    multi = [("blosc_lz4", "blosc", {}), ("zlib1", "zlib", {"level": 1})]
    if _zarr.cblosc() is not None:
        multi.append(("blosc_zstd5", "blosc", {"cname": "zstd", "clevel": 5, "shuffle": 1}))
    for name, comp, kw in multi:
        with ThreadPoolExecutor(16) as ex:
            chunks = list(ex.map(lambda c: enc(c, comp, kw), grid))
        specs = [dict(image_id=22, z=k, c=0, t=0, pixel_type=pbx.UINT16, size_x=side, size_y=side,
                      chunk_x=chunk, chunk_y=chunk, codec=comp, chunks=chunks) for k in range(4)]
        dec, plc = [], []
        for r in range(reps + 1):
            ids, (md, mp) = svc.register_zarr_planes(specs, timing=True)
            if r:
                dec.append(md)
                plc.append(mp)
            for pid in ids:
                svc.release_plane(pid)
        md, mp = sum(dec) / reps, sum(plc) / reps
        raw = 4 * side * side * 2
        res[name + "_4_planes_one_launch"] = {
            "chunks": 4 * len(chunks), "decoded_bytes": raw, "decode_ms": round(md, 3),
            "place_ms": round(mp, 3), "decoded_gbps": round(raw / ((md + mp) * 1e-3) / 1e9, 1),
            "chunks_per_s": round(4 * len(chunks) * world / ((md + mp) * 1e-3), 1)}
    return res


class ServeStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("requests", "ok", "bytes", "batches")] + \
               [(n, ctypes.c_double) for n in ("seconds", "p50_us", "p90_us", "p99_us", "max_us",
                                               "mean_us")]


def serve_one(svc, ctxs, threads, total, warmup):
    """T native caller threads, each blocking in one pbx_get_tile at a time over `ctxs`
    (lib/libpbx_servebench.so, no Python in the loop): tiles/s and latency percentiles."""
    L = ctypes.CDLL(os.path.join(ROOT, "omero-ms-pixel-buffer_amd", "lib", "libpbx_servebench.so"))
    L.pbx_serve_bench.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int,
                                  ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(ServeStats)]
    reqs = pbx.make_reqs(ctxs)
    s = ServeStats()
    rc = L.pbx_serve_bench(svc.handle, reqs, len(ctxs), threads, total, warmup, ctypes.byref(s))
    if rc != 0:
        raise RuntimeError(f"pbx_serve_bench: {rc}")
    return {"tiles_per_s": round(s.ok / s.seconds, 1), "requests": s.requests, "ok": s.ok,
            "requests_per_batch": round(s.requests / max(s.batches, 1), 1),
            "p50_ms": round(s.p50_us / 1e3, 3), "p90_ms": round(s.p90_us / 1e3, 3),
            "p99_ms": round(s.p99_us / 1e3, 3), "max_ms": round(s.max_us / 1e3, 3),
            "d2h_gbps": round(s.bytes / s.seconds / 1e9, 1)}


def serve_lines(svc, iid, threads=(32, 128, 512)):
    """The served path as the reference drives it: T worker threads (Vert.x
    worker_pool_size, PixelBufferMicroserviceVerticle.java:117-118,224-233), each blocking in
    one getTile at a time -> pbx_get_tile (coalesced into GPU batches), D2H and the JNI-style
    copy of every body included.  Native threads (lib/libpbx_servebench.so), no Python in the
    loop.  512x512 uint16 PNG tiles of the headline plane."""
    ctxs = grid_ctxs(iid, "png")
    return {f"threads_{t}": serve_one(svc, ctxs, t, max(8192, 32 * t), max(2048, 4 * t)) for t in threads}


def run_stream(svc, req_chunks, barrier, warmup=1, steps=1):
    """Timed passes over a request stream cut into batches (pipelined two deep: batch k+1
    planned and launched while k runs); returns (seconds for `steps` passes, last stats)."""
    def one_pass():
        stats, prev = [], None
        for r in list(req_chunks) + [None]:
            b = None
            if r is not None:
                b = pbx.Batch(svc, reqs=r)
                b.launch()
            if prev is not None:
                prev.sync()
                stats.append(prev.stats())
                prev.close()
            prev = b
        return stats
    for _ in range(warmup):
        one_pass()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        stats = one_pass()
    torch.cuda.synchronize()
    barrier()
    return (time.perf_counter() - t0) / steps, stats


C4_SIDE, C4_CHANNELS = 100000, 5


def c4_band(world, rank, side=C4_SIDE, tile=TILE):
    """configs[3] ownership: rank r owns the contiguous tile-row band
    [lo, hi) of every channel, i.e. plane rows [y0, y1)."""
    n = (side + tile - 1) // tile
    lo, hi = pbx.band_rows(n, world, rank)
    return lo, hi, tile * lo, min(side, tile * hi)


def wholeslide_line(svc, rank, world, barrier, steps=2, side=C4_SIDE, channels=C4_CHANNELS, tile=512,
                    band_batch_rows=49):
    """configs[3]: this rank's tile-row band of all 5 channels of a 100000^2 uint16 slide as
    TIFF (uncompressed = the reference's TiffWriter default, or Compression=8 when the
    service deflates TIFF), in batches of `band_batch_rows` tile rows (bounded arenas).  Each
    rank holds ONLY its band of each channel in HBM (pbx_plane_create with band_y0/band_rows:
    ~100 GB / N per rank); tiles of other bands would answer NOT_RESIDENT here."""
    n = (side + tile - 1) // tile
    lo, hi, y0, y1 = c4_band(world, rank, side, tile)
    before = svc.residency_stats()["resident_bytes"]
    pids = [svc.create_plane(4, 0, c, 0, pbx.UINT16, side, side, band=(y0, y1 - y0), generator="noise",
                             plane_no=c) for c in range(channels)]
    held = svc.residency_stats()["resident_bytes"] - before
    chunks, ntiles = [], 0
    for c in range(channels):
        for r0 in range(lo, hi, band_batch_rows):
            ctxs = [pbx.TileCtx(4, 0, c, 0, tile * tx, tile * ty, min(tile, side - tile * tx),
                                min(tile, side - tile * ty), format="tif")
                    for ty in range(r0, min(hi, r0 + band_batch_rows)) for tx in range(n)]
            ntiles += len(ctxs)
            chunks.append(pbx.make_reqs(ctxs))
    dt, stats = run_stream(svc, chunks, barrier, warmup=1, steps=steps)
    in_bytes = sum(s.in_bytes for s in stats)
    out_bytes = sum(s.out_bytes for s in stats)
    line = {"tiles_this_rank": ntiles, "tiles_all_ranks": n * n * channels,
            "tile_rows_this_rank": [lo, hi], "plane_rows_this_rank": [y0, y1],
            "hbm_plane_bytes_this_rank": held,
            "tiles_per_s": round(ntiles * world / dt, 1), "ms_per_pass": round(dt * 1e3, 2),
            "pixel_bytes": in_bytes, "response_bytes": out_bytes,
            "d2h_bytes_saved_vs_uncompressed": int(in_bytes + ntiles * 160 - out_bytes)}
    ext = sum(s.ms_extract for s in stats)
    if out_bytes >= in_bytes:  # uncompressed: the HBM-bound k_extract does all the work
        line["k_extract_gbps"] = round(2 * in_bytes / (ext * 1e-3) / 1e9, 1)
    # a tile of another rank's band is not resident here (world > 1)
    if world > 1:
        other = (hi % n) * tile if hi < n else 0
        (st, _), = svc.get_tiles([pbx.TileCtx(4, 0, 0, 0, 0, other, tile, tile, format="tif")])
        line["foreign_band_status"] = st
    for pid in pids:
        svc.release_plane(pid)
    return line


C5_SEED, C5_REQUESTS, C5_SIDE = 5, 16384, 16384


def c5_stream():
    """configs[4]: ONE common mixed request stream (the same in every rank: seeded RNG
    independent of the rank): uint8/int32/float32 planes of 16384^2, w, h in 256..2048,
    png/tif/raw."""
    import random
    rnd = random.Random(C5_SEED)
    reqs = []
    for _ in range(C5_REQUESTS):
        k = rnd.randrange(3)
        w, h = 256 * rnd.randint(1, 8), 256 * rnd.randint(1, 8)
        reqs.append(pbx.TileCtx(10 + k, 0, 0, 0, rnd.randrange(C5_SIDE - w + 1),
                                rnd.randrange(C5_SIDE - h + 1), w, h,
                                format=rnd.choice([None, "png", "tif"])))
    return reqs


def c5_shard(reqs, rank, world):
    """The requests rank `rank` serves: pbx_shard_of(req) == rank (hash of image, z, c, t and
    the 512-px tile cell), no collective."""
    return [i for i, c in enumerate(reqs) if world == 1 or pbx.shard_of(c, world) == rank]


def zlib6_sample(svc, pid, n=16):
    """The IDAT zlib stream of n grid tiles (512x512 uint16 PNG, filter None) against zlib
    level 6 of the same scanlines (java.util.zip.Deflater's default, the reference's ImageIO
    PNG writer): bytes per tile both ways and the ratio."""
    import zlib
    import numpy as np
    sample = [pbx.TileCtx(pid, 0, 0, 0, (j * 7 % GRID) * TILE, (j * 5 % GRID) * TILE, TILE, TILE)
              for j in range(n)]
    raw = [b for _, b in svc.get_tiles(sample)]
    png = [b for _, b in svc.get_tiles([pbx.TileCtx(pid, 0, 0, 0, c.region["x"], c.region["y"], TILE, TILE,
                                                    format="png") for c in sample])]
    z6 = sum(len(zlib.compress(np.concatenate([np.zeros((TILE, 1), np.uint8),
                                               np.frombuffer(b, np.uint8).reshape(TILE, 2 * TILE)], 1).tobytes(), 6))
             for b in raw)
    mine = sum(int.from_bytes(b[91:95], "big") for b in png)  # the single IDAT's length field
    return {"tiles": n, "idat_bytes_per_tile": round(mine / n, 1), "zlib6_bytes_per_tile": round(z6 / n, 1),
            "ratio": round(mine / z6, 4)}


def adaptive_filter_line(svc, rank, world, barrier, side):
    """PNG with the adaptive filter (cfg.png_filter = ADAPTIVE: k_adaptive_mode first decides
    per tile whether filtering pays -- if not, every row is None -- else the filter kernels pick
    None/Sub/Up/Avg/Paeth per row by minimum sum |residual|), on G_NOISE, G_FAKE and a
    Poisson-like plane: tiles/s (device-resident, like the headline) and bytes per tile
    against the filter-None path and zlib-6 of the filter-None stream (the reference's
    ImageIO PNG), the last two on a sample of 8 tiles fetched through the raw path."""
    import zlib
    import numpy as np
    out = {}
    # Poisson-like plane of the headline's size (4096 distinct tiles): lambda drifting 200..300
    # over the plane in 64-px steps, drawn on the GPU (torch.poisson), registered from host memory
    ps = side
    yy, xx = np.mgrid[0:ps:64, 0:ps:64]
    lam = 200.0 + 100.0 * (0.5 + 0.25 * np.sin(xx / 900.0) + 0.25 * np.cos(yy / 1300.0))
    gen = torch.Generator(device="cuda").manual_seed(1234 + rank)
    lam_t = torch.from_numpy(lam.astype(np.float32)).cuda().repeat_interleave(64, 0).repeat_interleave(64, 1)
    pois = torch.poisson(lam_t, generator=gen).to(torch.int16).cpu().numpy().view(np.uint16)
    del lam_t
    with pbx.PixelsService(device=torch.cuda.current_device(), png_filter=pbx.FILTER_ADAPTIVE) as sa:
        sa.set_kernel_streams(1, 0)  # serial: k_filter_ms is the kernel's own time
        for k, (name, gen, sz) in enumerate((("noise", "noise", side), ("fake", "fake", side),
                                            ("poisson", None, ps))):
            pid = 40 + k
            held = []
            for s_ in (sa, svc):
                if gen:
                    held.append((s_, s_.register_plane(pid, 0, 0, 0, pbx.UINT16, sz, sz, generator=gen,
                                                       plane_no=rank)))
                else:
                    held.append((s_, s_.register_plane(pid, 0, 0, 0, pbx.UINT16, sz, sz, data=pois,
                                                       big_endian=False)))
            # a 4096-tile batch like the headline's on every plane, 4096 distinct tiles
            g = sz // TILE
            ctxs = [pbx.TileCtx(pid, 0, 0, 0, (i % g) * TILE, (i // g % g) * TILE, TILE, TILE, format="png")
                    for i in range(GRID * GRID)]
            dt, st, _ = secondary_steps(sa, ctxs, 3, 1, barrier)
            sample = [pbx.TileCtx(pid, 0, 0, 0, (j * 7 % (sz // TILE)) * TILE,
                                  (j * 5 % (sz // TILE)) * TILE, TILE, TILE) for j in range(8)]
            raw = [b for _, b in svc.get_tiles(sample)]
            png_ad = [b for _, b in sa.get_tiles([pbx.TileCtx(c.imageId, 0, 0, 0, c.region["x"], c.region["y"],
                                                              TILE, TILE, format="png") for c in sample])]
            png_no = [b for _, b in svc.get_tiles([pbx.TileCtx(c.imageId, 0, 0, 0, c.region["x"], c.region["y"],
                                                               TILE, TILE, format="png") for c in sample])]
            z6 = 0
            for b in raw:  # filter-None scanlines (filter byte 0 + big-endian row), zlib level 6
                rows = np.frombuffer(b, np.uint8).reshape(TILE, TILE * 2)
                z6 += len(zlib.compress(np.concatenate([np.zeros((TILE, 1), np.uint8), rows], 1).tobytes(), 6))
            out[name] = {
                "tiles_per_s": round(len(ctxs) * 3 * world / dt, 1), "batch_tiles": len(ctxs),
                "distinct_tiles": g * g,
                **wall_vs_kernels(dt, 3, st),
                "k_filter_ms": round(mean(st, "ms_filter"), 3),
                # (the filter pass moves the bytes of the tiles it filters: None-mode tiles of
                # TF_DIRECT's geometry skip it, k_lz77 reads their rows from the plane)
                "k_filter_frac": (round((st[-1].in_bytes + st[-1].stream_bytes - st[-1].direct_bytes)
                                        / (mean(st, "ms_filter") * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
                                  if 2 * st[-1].direct_tiles < len(ctxs) else None),
                "none_mode_direct_tiles": st[-1].direct_tiles,
                **({"k_filter_note": "most tiles skip the filter pass (None mode, read from the plane by "
                                     "k_lz77): k_filter_ms is k_adaptive_mode and the idle launch"}
                   if 2 * st[-1].direct_tiles >= len(ctxs) else {}),
                "deflate_chain_ms": round(mean(st, "ms_deflate") + mean(st, "ms_assemble"), 3),
                "sample_bytes_per_tile": {"adaptive": round(sum(map(len, png_ad)) / 8, 1),
                                          "filter_none": round(sum(map(len, png_no)) / 8, 1),
                                          "zlib6_filter_none_idat": round(z6 / 8, 1)}}
            for s_, h in held:
                s_.release_plane(h)
    svc.release_cached()
    return out


def fixed_filter_line(rank, world, barrier, side):
    """PNG with one fixed filter for every row (cfg.png_filter = Sub / Up / Avg / Paeth:
    k_filter3), the headline's 4096 G_NOISE tiles, one kernel stream (k_filter_ms is the
    kernel's own HIP-event time).  Algorithmic bytes = the tiles read + the filtered stream
    written; gbps / frac against the 8 TB/s HBM peak."""
    out = {}
    for f, name in ((1, "sub"), (2, "up"), (3, "avg"), (4, "paeth")):
        with pbx.PixelsService(device=torch.cuda.current_device(), png_filter=f) as sf:
            sf.set_kernel_streams(1, 0)
            sf.register_plane(45, 0, 0, 0, pbx.UINT16, side, side, generator="noise", plane_no=rank)
            ctxs = grid_ctxs(45, "png")
            dt, st, _ = secondary_steps(sf, ctxs, 3, 1, barrier)
            ms = mean(st, "ms_filter")
            alg = st[-1].in_bytes + st[-1].stream_bytes
            out[name] = {"tiles_per_s": round(len(ctxs) * 3 * world / dt, 1), **wall_vs_kernels(dt, 3, st),
                         "k_filter_ms": round(ms, 3), "k_filter_alg_bytes": alg,
                         "k_filter_gbps": round(alg / (ms * 1e-3) / 1e9, 1),
                         "k_filter_frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                         "compressed_bytes_per_tile": round(st[-1].deflate_out_bytes / len(ctxs), 1)}
    return out


def progress(rank, msg):
    """A line on stderr per bench section (rank 0): long runs show they are alive."""
    if rank == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def extra(out, svc, rank, world, barrier, iid, side):
    """Secondary lines: the other BASELINE configs (parity-tested in tests/), each timed
    device-resident like the headline; and the PCIe-inclusive end-to-end rate."""
    # PCIe-inclusive end-to-end (D2H of every PNG into pinned host memory)
    progress(rank, "e2e with D2H")
    rate, gbs = e2e_rate(svc, grid_ctxs(iid, "png"))
    out["e2e_with_d2h"] = {"tiles_per_s": round(rate, 1), "d2h_gbps": round(gbs, 1)}
    # the served path: concurrent single-tile callers through the coalescer
    progress(rank, "served path")
    # (one node's ranks together: 512 callers per rank only on a single GPU)
    out["served_get_tile_512x512_u16_png"] = serve_lines(svc, iid, (32, 128, 512) if world == 1 else (32, 128))
    # configs[0]: the reference's own CPU case at its workload, GPU and CPU side by side
    progress(rank, "configs[0]")
    out["c1_png_512x512_u8_fake"] = c1_line(svc, rank, world, barrier)
    # configs[1]: raw path, extraction + byte swap (HBM-bound k_extract)
    progress(rank, "raw")
    raw = grid_ctxs(iid, None)
    dtr, sr, _ = secondary_steps(svc, raw, 5, 2, barrier)
    ms_ext = mean(sr, "ms_extract")
    out["raw_4096x512x512_u16"] = {
        "tiles_per_s": round(len(raw) * 5 * world / dtr, 1), **wall_vs_kernels(dtr, 5, sr),
        "k_extract_ms": round(ms_ext, 3),
        "k_extract_gbps": round(2 * sr[-1].in_bytes / (ms_ext * 1e-3) / 1e9, 1),
        "k_extract_frac": round(2 * sr[-1].in_bytes / (ms_ext * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
    # the same grid at an odd x (x * bpp mod 16 = 6, as most of the reference's arbitrary-x
    # requests, TileCtx.java:73-85): k_extract's realigned path
    progress(rank, "raw unaligned")
    rawu = [pbx.TileCtx(iid, 0, 0, 0, (i % GRID) * TILE + (3 if i % GRID < GRID - 1 else -5),
                        (i // GRID) * TILE, TILE, TILE) for i in range(GRID * GRID)]
    dtu, su, _ = secondary_steps(svc, rawu, 5, 2, barrier)
    ms_u = mean(su, "ms_extract")
    out["raw_unaligned_4096x512x512_u16"] = {
        "tiles_per_s": round(len(rawu) * 5 * world / dtu, 1), **wall_vs_kernels(dtu, 5, su),
        "x_times_bpp_mod_16": 6,
        "k_extract_ms": round(ms_u, 3),
        "k_extract_gbps": round(2 * su[-1].in_bytes / (ms_u * 1e-3) / 1e9, 1),
        "k_extract_frac": round(2 * su[-1].in_bytes / (ms_u * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
    # A/B: the same headline batch with the filter-None rows staged in a stream buffer by
    # k_rows first (cfg.stage_rows), instead of assembled from the plane inside k_lz77
    progress(rank, "staged rows")
    # (serial: one kernel stream, so the kernel times are the kernels' own; compare with
    # the headline's kernel_streams.serial_pass_tiles_per_s)
    with pbx.PixelsService(device=torch.cuda.current_device(), stage_rows=True) as ss:
        ss.set_kernel_streams(1, 0)
        ss.register_plane(iid, 0, 0, 0, pbx.UINT16, side, side, generator="noise", seed=0,
                          plane_no=rank)
        dts, sst, _ = secondary_steps(ss, grid_ctxs(iid, "png"), 5, 2, barrier)
        out["png_staged_rows_4096x512x512_u16"] = {
            "tiles_per_s": round(len(grid_ctxs(iid, "png")) * 5 * world / dts, 1),
            **wall_vs_kernels(dts, 5, sst),
            "k_rows_ms": round(mean(sst, "ms_filter"), 3),
            "k_lz77_ms": round(mean(sst, "ms_lz77"), 3)}
    # Row f3: on-GPU resolution pyramid of the headline plane (6 levels of 2x2 box means);
    # algorithmic bytes = every level read once + every lower level written once
    progress(rank, "pyramid")
    pid = svc.register_plane(5, 0, 0, 0, pbx.UINT16, side, side, generator="noise", plane_no=rank)
    _, pms = svc.build_pyramid(pid, 6, timing=True)
    pb, wl = 0, side
    for _ in range(6):
        pb += 2 * wl * wl + 2 * ((wl + 1) // 2) ** 2
        wl = (wl + 1) // 2
    out["pyramid_6_levels_32768sq_u16"] = {
        "kernel_ms": round(pms, 3), "alg_bytes": pb,
        "gbps": round(pb / (pms * 1e-3) / 1e9, 1),
        "frac": round(pb / (pms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
    # Row f2: NGFF/Zarr chunk decode into HBM (pbx_plane_register_zarr) of a 16384^2 uint16
    # G_NOISE plane stored as 512^2 chunks (1,024 chunks); blosc-lz4 (shuffle, the NGFF
    # writers' default) and zlib-1.  Timed: the decode kernels and the placement kernel
    # (HIP events); the chunk upload is PCIe and reported apart.
    progress(rank, "zarr")
    out["zarr_decode_16384sq_u16_512chunks"] = zarr_lines(svc, rank, world)
    # G_FAKE (FakeReader-like gradient) PNG, compressible data
    progress(rank, "fake")
    svc.register_plane(2, 0, 0, 0, pbx.UINT16, side, side, generator="fake", plane_no=rank)
    fk = grid_ctxs(2, "png")
    dtf, sf, _ = secondary_steps(svc, fk, 3, 2, barrier)
    out["png_fake_4096x512x512_u16"] = {
        "tiles_per_s": round(len(fk) * 3 * world / dtf, 1), **wall_vs_kernels(dtf, 3, sf),
        "compressed_bytes_per_tile": round(sf[-1].deflate_out_bytes / len(fk), 1),
        "vs_zlib6": zlib6_sample(svc, 2)}
    # the adaptive PNG filter (option; the reference writes filter None)
    progress(rank, "adaptive filter")
    out["png_adaptive_filter_512x512_u16"] = adaptive_filter_line(svc, rank, world, barrier, side)
    progress(rank, "fixed filters")
    out["png_fixed_filter_4096x512x512_u16"] = fixed_filter_line(rank, world, barrier, side)
    # configs[2]: 4096 x 1024^2 uint16 PNG from a 65536^2 plane (8 GiB)
    progress(rank, "configs[2]")
    svc.register_plane(3, 0, 0, 0, pbx.UINT16, 65536, 65536, generator="noise", plane_no=rank)
    c3 = grid_ctxs(3, "png", tile=1024)
    dt3, s3, _ = secondary_steps(svc, c3, 2, 2, barrier)
    out["c3_png_4096x1024x1024_u16"] = {
        "tiles_per_s": round(len(c3) * 2 * world / dt3, 1), **wall_vs_kernels(dt3, 2, s3),
        "compressed_bytes_per_tile": round(s3[-1].deflate_out_bytes / len(c3), 1)}
    # configs[3]: whole slide 100000^2 x 5 channels uint16, 512^2 tiles (edge 160 px) -> TIFF.
    # Every rank holds and serves its contiguous band of tile rows of the 5 channels
    # (SURVEY.md §8(e)); over all ranks the bands cover the whole slide (192,080 tiles).
    progress(rank, "configs[3]")
    # Each rank holds only its band (the one-GPU rehearsal's ranks share ~100 GB).
    out["c4_wholeslide_tif_100k_u16_5ch"] = wholeslide_line(svc, rank, world, barrier)
    svc.release_cached()  # the deflate-TIFF service below needs the HBM the caches hold
    with pbx.PixelsService(device=torch.cuda.current_device(), tiff_deflate=True) as sd:
        out["c4_wholeslide_tif_deflate_100k_u16_5ch"] = wholeslide_line(sd, rank, world, barrier,
                                                                        steps=1)
    # configs[4]: one common mixed stream of 16,384 requests (uint8/int32/float32 planes
    # 16384^2, w,h in 256..2048, png/tif/raw); each rank serves its pbx_shard_of share, in
    # batches of 2048
    progress(rank, "configs[4]")
    for k, pt in enumerate((pbx.UINT8, pbx.INT32, pbx.FLOAT)):
        svc.register_plane(10 + k, 0, 0, 0, pt, C5_SIDE, C5_SIDE, generator="noise")
    reqs5 = c5_stream()
    mine = [reqs5[i] for i in c5_shard(reqs5, rank, world)]
    chunks = [pbx.make_reqs(mine[j:j + 2048]) for j in range(0, len(mine), 2048)]

    def stream_pass():
        ok = err = 0
        prev = None
        for r in chunks + [None]:
            b = None
            if r is not None:
                b = pbx.Batch(svc, reqs=r)
                b.launch()
            if prev is not None:
                prev.sync()
                s = prev.stats()
                ok += s.ok_tiles
                err += s.tiles - s.ok_tiles
                prev.close()
            prev = b
        return ok, err

    stream_pass()  # warm: device pool blocks of every batch shape
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ok, err = stream_pass()
    torch.cuda.synchronize()
    barrier()
    dt5 = time.perf_counter() - t0
    tot = torch.tensor([ok, err, dt5], dtype=torch.float64)
    if world > 1:  # whole-stream totals over the ranks; time = the slowest rank's
        t_max = torch.tensor([dt5], dtype=torch.float64)
        dist.all_reduce(tot)
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        dt5 = float(t_max[0])
    out["c5_mixed_16384_requests"] = {"tiles_per_s": round(float(tot[0]) / dt5, 1),
                                      "ok": int(tot[0]), "errors_404": int(tot[1]),
                                      "requests_this_rank": len(mine),
                                      "stream": f"one common stream (seed {C5_SEED}), sharded by pbx_shard_of"}


def launch_ranks(n, argv):
    """`--gpus N` without a launcher: start N rank processes of this script and wait.

    This process never touches the GPU (it only imported torch; nothing here initialises
    HIP), so the ranks are plain child processes, not an exec.  If one rank fails, the
    others (which would wait at the barrier forever) are terminated by PID."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    while procs:
        time.sleep(0.2)
        for p in list(procs):
            c = p.poll()
            if c is None:
                continue
            procs.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in procs:
                    q.terminate()
    return rc


def dry_run(args, world, rank):
    """The N > 1 plumbing without HIP: rendezvous, barrier, timed no-op steps, max-over-ranks."""
    if world > 1:
        init_gloo()
    met = torch.ones(1, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(met)
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.barrier()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    # the data partitioning each rank would serve (host only: pbx_shard_of and the band
    # split are pure functions of the request / grid): C5's common stream by request hash,
    # C4's tile-row bands; rank 0 checks that the ranks' shares partition the whole
    reqs = c5_stream()
    shard = c5_shard(reqs, rank, world)
    band = c4_band(world, rank)
    parts = [(shard, band)]
    if world > 1:
        parts = [None] * world
        dist.all_gather_object(parts, (shard, band))
    if rank == 0:
        idx = [i for sh, _ in parts for i in sh]
        bands = [b for _, b in parts]
        n_rows = (C4_SIDE + TILE - 1) // TILE
        print(json.dumps({"metric": METRIC, "value": None, "unit": "tiles/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "dry_run": True,
                          "ranks_met": int(met[0]), "max_step_s": float(t[0]),
                          "c5_requests_per_rank": [len(sh) for sh, _ in parts],
                          "c5_shards_partition_stream": sorted(idx) == list(range(len(reqs))),
                          "c4_tile_row_bands": [[b[0], b[1]] for b in bands],
                          "c4_bands_partition_slide": bands[0][0] == 0 and bands[-1][1] == n_rows and
                          all(bands[i][1] == bands[i + 1][0] for i in range(world - 1))}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def init_gloo():
    """gloo's process group, its connection messages ("[Gloo] Rank r is connected ...", written
    to the C-level stdout) sent to stderr: rank 0's stdout carries the one JSON line only."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo", init_method="env://")
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--dry-run", action="store_true",
                    help="rank plumbing only (launch, barrier, max), no HIP call")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; measuring {world} rank(s)",
              file=sys.stderr)
    if args.dry_run:
        return dry_run(args, world, rank)
    if world > 1:
        init_gloo()
    # PBX_BENCH_ONE_GPU=1: every rank on GPU 0 (a rehearsal of the N-rank path on a one-GPU
    # box; per-rank numbers then share one device)
    dev = 0 if os.environ.get("PBX_BENCH_ONE_GPU") else local
    torch.cuda.set_device(dev)
    barrier = (lambda: dist.barrier()) if world > 1 else (lambda: None)

    svc = pbx.PixelsService(device=dev)
    side = GRID * TILE
    iid = 1
    svc.register_plane(iid, 0, 0, 0, pbx.UINT16, side, side, generator="noise", seed=0,
                       plane_no=rank)
    ctxs = grid_ctxs(iid, "png")
    dt, stats, host_ms = run_steps(svc, ctxs, args.steps, args.warmup, barrier, HEADLINE_SUB)
    t = torch.tensor([dt], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t[0])
    tiles_total = len(ctxs) * world * args.steps
    value = tiles_total / dt
    ms_per_step = 1000.0 * dt / args.steps
    st = stats[-1]
    # The timed pass overlaps consecutive batches on the library's kernel streams (default
    # 3, each batch's k_lz77 staggered behind the previous one's: pbx_set_kernel_streams),
    # which stretches each kernel's HIP-event duration over the others.  Per-kernel
    # durations therefore come from a second, serial pass (one kernel stream, batches in
    # launch order), the configuration the committed rocprofv3 kernel trace uses
    # (PBX_KSTREAMS=1); its tiles/s is reported beside the headline.
    svc.set_kernel_streams(1, 0)
    dts, stats, _ = run_steps(svc, ctxs, args.steps, 1, barrier, HEADLINE_SUB)
    svc.set_kernel_streams(KSTREAMS, KSTAGGER)
    serial_rate = len(ctxs) * args.steps / dts

    # Per-kernel algorithmic bytes per launch over the kernel's mean
    # HIP-event duration on the library's stream:
    #   k_lz77   tile bytes read from the plane (the filter-None stream is assembled in LDS:
    #            K1+K2 fused) + the stream written for k_encode + per-segment symbol
    #            histogram written (1280 B)
    #   k_huff   histograms read per segment + codes/header written per block (1280 + 1920 B)
    #   k_encode stream bytes read + compressed bytes written
    payload = st.deflate_out_bytes - len(ctxs) * 121  # zlib payload (minus PNG framing)
    seg = st.segments
    kern = {
        "k_lz77": (mean(stats, "ms_lz77"), st.in_bytes + st.stream_bytes + 1280 * seg),
        "k_huff": (mean(stats, "ms_huff"), 1280 * seg + 1920 * st.blocks),
        "k_encode": (mean(stats, "ms_encode"), st.stream_bytes + payload),
    }
    kernels = {k: {"ms": round(ms, 3), "alg_bytes": int(b),
                   "gbps": round(b / (ms * 1e-3) / 1e9, 1),
                   "frac": round(b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
               for k, (ms, b) in kern.items()}
    # the dominant kernel: the longest mean HIP-event time of the SERIAL pass (one kernel
    # stream: no overlap stretches a kernel), with its byte definition stated in the line
    byte_def = {"k_lz77": "plane tile bytes read + filtered stream written + 1280 B histogram per segment",
                "k_huff": "1280 B histogram read per segment + 1920 B codes/header written per block",
                "k_encode": "filtered stream read + zlib payload written"}
    dom = max(kern, key=lambda k: kern[k][0])
    dom_ms, dom_bytes = kern[dom]
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic, traffic_src = load_traffic(dom)
    chain_ms = mean(stats, "ms_deflate") + mean(stats, "ms_assemble")
    # SURVEY §8(d) "PNG end-to-end": the plane bytes the tiles read + the PNG bytes written,
    # per step, over the whole step's time (all kernels, launches and host planning)
    e2e_bytes = st.in_bytes + st.deflate_out_bytes
    chain_traffic, chain_src = load_chain_traffic()
    rp_ms, rp_src = load_rocprof_ms(dom)
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "tiles/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (G_NOISE seed 0 plane generated in HBM)",
        "config": {"workload": "4096 x 512x512 uint16 tiles -> PNG per GPU from a 32768^2 "
                               "uint16 plane (BASELINE configs[1] shape, metric's PNG format)",
                   "tiles_per_gpu": len(ctxs), "tile": "512x512", "pixel_type": "uint16",
                   "format": "png", "png_filter": "none (reference APNGWriter)",
                   "parallelism": f"dp{world} (request sharding, no collectives)",
                   "batches_per_step": 1 if HEADLINE_SUB <= 0 else -(-len(ctxs) // HEADLINE_SUB)},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": traffic, "traffic_source": traffic_src,
                     "limiter": "issue / latency, not HBM bandwidth: the deflate kernels wait on "
                                "dependent LDS and memory steps with VALU and SALU below saturation "
                                "(`issue`); `bound` names the roof the line is priced against (HBM)",
                     "kernel": dom, "kernel_ms": round(dom_ms, 3),
                     "kernel_ms_source": "HIP events around the kernel on its own stream, serial pass",
                     "rocprof_kernel_ms": round(rp_ms, 4) if rp_ms else None,
                     "rocprof_source": rp_src,
                     "hip_event_over_rocprof": round(dom_ms / rp_ms, 3) if rp_ms else None,
                     "frac_at_rocprof_ms": round(dom_bytes / (rp_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if rp_ms else None,
                     "kernel_choice": "longest mean HIP-event time of the serial pass",
                     "alg_bytes_per_launch": int(dom_bytes), "alg_bytes_definition": byte_def[dom],
                     "end_to_end_frac": round(e2e_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                     "end_to_end_bytes_per_step": int(e2e_bytes),
                     "chain_traffic_ratio": (round(chain_traffic / e2e_bytes, 3) if chain_traffic else None),
                     "chain_traffic_bytes": chain_traffic, "chain_traffic_source": chain_src,
                     "note": "deflate kernels are VALU-issue/latency-bound integer work, not "
                             "HBM-bound; the HBM-bound extraction kernel (k_extract) is in "
                             "raw_4096x512x512_u16; their issue roofline is in `issue`",
                     "issue": load_issue()},
        "kernels": kernels,
        "deflate_chain_ms": round(chain_ms, 3),
        "hbm_gbps_step": round((st.in_bytes + st.deflate_out_bytes) * world * args.steps / dt / 1e9, 1),
        "compressed_bytes_per_tile": round(st.deflate_out_bytes / len(ctxs), 1),
        "host_ms_per_step": round(host_ms, 3),
        "kernel_streams": {"timed_pass": KSTREAMS, "stagger": "k_lz77",
                           "serial_pass_tiles_per_s": round(serial_rate, 1),
                           "note": "kernels/roofline/deflate_chain_ms from the serial pass"},
    }

    if not args.no_extra:
        extra(out, svc, rank, world, barrier, iid, side)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress(rank, "cpu baseline")
        out["cpu_baseline"] = cpu_baseline(threads=args.cpu_threads)
        out["speedup_vs_cpu_baseline"] = round(value / out["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    svc.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
