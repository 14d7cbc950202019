#!/usr/bin/env python3
"""Benchmark of the MI355X /tile pipeline (BASELINE.json metric).

Workload per GPU (weak scaling, one process per GPU, no collectives on the data path):
a 32768 x 32768 uint16 G_NOISE plane generated in HBM, and one batch = the 4096 tiles of
its 64 x 64 grid of 512 x 512 tiles, each encoded to PNG (APNGWriter layout, filter None
as the reference, zlib-compatible deflate).  A step = plan the 4096 requests on the host
(TileRequestHandler validation + descriptors) + descriptor upload + every kernel, outputs
left in HBM.  Inputs are resident before the timed region; D2H is reported separately.

    python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1 is launched by torch.distributed.run (one rank per GPU); ranks only meet at the
barrier and the max-over-ranks of the step time (gloo, CPU tensors).
"""
import argparse
import ctypes
import json
import os
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


def grid_ctxs(image_id, fmt, n=GRID * GRID, tile=TILE):
    return [pbx.TileCtx(image_id, 0, 0, 0, (i % GRID) * tile, (i // GRID) * tile, tile, tile,
                        format=fmt) for i in range(n)]


def run_steps(svc, ctxs, steps, warmup, barrier):
    """Warmup, then `steps` timed steps; returns (seconds, last stats, mean deflate-chain ms,
    mean k_extract ms, mean host ms per step).

    Steps are pipelined two deep, as a server feeds its GPU: the host plans and launches
    batch k+1 (request validation, descriptors, upload) while batch k runs, then waits for
    batch k.  The request array is built once (the caller's TileCtx list)."""
    reqs = pbx.make_reqs(ctxs)

    def one_pass(n, record):
        prev = None
        host = 0.0
        out = []
        for _ in range(n):
            t0 = time.perf_counter()
            b = pbx.Batch(svc, reqs=reqs)
            b.launch()
            host += time.perf_counter() - t0
            if prev is not None:
                prev.sync()
                if record:
                    out.append(prev.stats())
                prev.close()
            prev = b
        prev.sync()
        if record:
            out.append(prev.stats())
        prev.close()
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
    n = len(stats)
    return (dt, stats[-1], sum(s.ms_deflate + s.ms_assemble for s in stats) / n,
            sum(s.ms_extract for s in stats) / n, 1000.0 * host / n)


def fetch_rate(svc, ctxs):
    """End-to-end incl. D2H to pinned host memory (PCIe-inclusive; never the headline)."""
    b = pbx.Batch(svc, ctxs)
    t0 = time.perf_counter()
    b.launch()
    res = b.fetch()
    dt = time.perf_counter() - t0
    b.close()
    return len(ctxs) / dt, sum(len(x) for _, x in res if x)


def cpu_baseline(seconds=10.0, threads=16):
    """The C oracle (zlib-6 filter-None PNG, same region extraction) on host threads."""
    import _oracle as O
    O.lib()
    pw = ph = 4096
    sec, _ = O.bench(O.GEN_NOISE, O.UINT16, O.FMT_PNG, pw, ph, TILE, TILE, 2 * threads, threads)
    rate = 2 * threads / sec
    n = max(threads, int(rate * seconds))
    sec, nbytes = O.bench(O.GEN_NOISE, O.UINT16, O.FMT_PNG, pw, ph, TILE, TILE, n, threads)
    return {"value": round(n / sec, 2), "unit": "tiles/s", "cores": threads, "kind": "port",
            "sample": f"{n} tiles 512x512 uint16 G_NOISE -> PNG (filter None, zlib level 6) "
                      f"from a 4096x4096 plane, oracle/pbx_oracle.c on {threads} threads, "
                      f"{sec:.1f} s; avg {nbytes / n:.0f} B/tile"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    torch.cuda.set_device(local)
    barrier = (lambda: dist.barrier()) if world > 1 else (lambda: None)

    svc = pbx.PixelsService(device=local)
    side = GRID * TILE
    iid = 1
    svc.register_plane(iid, 0, 0, 0, pbx.UINT16, side, side, generator="noise", seed=0,
                       plane_no=rank)
    ctxs = grid_ctxs(iid, "png")
    dt, st, ms_deflate, _, host_ms = run_steps(svc, ctxs, args.steps, args.warmup, barrier)
    t = torch.tensor([dt], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t[0])
    tiles_total = len(ctxs) * world * args.steps
    value = tiles_total / dt
    ms_per_step = 1000.0 * dt / args.steps

    # roofline of the dominant kernel (k_deflate): algorithmic bytes = tile bytes read
    # from the plane + compressed bytes written, per launch, / average launch duration
    deflate_payload = st.deflate_out_bytes - len(ctxs) * 121  # minus PNG framing bytes
    alg_bytes = st.in_bytes + deflate_payload
    achieved = alg_bytes / (ms_deflate * 1e-3) / 1e9
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "tiles/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (G_NOISE seed 0 plane generated in HBM)",
        "config": {"workload": "4096 x 512x512 uint16 tiles -> PNG per GPU from a 32768^2 "
                               "uint16 plane (BASELINE configs[1] shape, metric's PNG format)",
                   "tiles_per_gpu": len(ctxs), "tile": "512x512", "pixel_type": "uint16",
                   "format": "png", "png_filter": "none (reference APNGWriter)",
                   "parallelism": f"dp{world} (request sharding, no collectives)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": None,
                     "kernel": "deflate chain k_lz77+k_huff+k_seg_sizes+k_scan_offsets+k_encode+k_frame",
                     "kernel_ms": round(ms_deflate, 3),
                     "alg_bytes_per_launch": int(alg_bytes),
                     "alg_bytes_def": "PNG end-to-end w*h*bpp + out_len per tile (SURVEY 8d)"},
        "hbm_gbps_step": round((st.in_bytes + st.deflate_out_bytes) * world * args.steps / dt / 1e9, 1),
        "compressed_bytes_per_tile": round(st.deflate_out_bytes / len(ctxs), 1),
        "kernel_ms": {"extract": round(st.ms_extract, 3), "filter": round(st.ms_filter, 3),
                      "lz77": round(st.ms_lz77, 3), "huff": round(st.ms_huff, 3),
                      "encode": round(st.ms_encode, 3), "deflate": round(st.ms_deflate, 3),
                      "frame": round(st.ms_assemble, 3), "total": round(st.ms_total, 3)},
        "filter_gbps": round((st.in_bytes + st.stream_bytes) / (st.ms_filter * 1e-3) / 1e9, 1),
        "filter_frac": round((st.in_bytes + st.stream_bytes) / (st.ms_filter * 1e-3) / 1e9
                             / HBM_PEAK_GBPS, 4),
        "host_ms_per_step": round(host_ms, 3),
    }

    if not args.no_extra:
        # PCIe-inclusive end-to-end (D2H of every PNG to pinned memory)
        rate, nbytes = fetch_rate(svc, ctxs)
        out["e2e_with_d2h_tiles_per_s"] = round(rate, 1)
        # raw path (BASELINE configs[1]): extraction + byte swap, HBM-bound k_extract
        raw = grid_ctxs(iid, None)
        dtr, sr, _, ms_ext, _ = run_steps(svc, raw, 5, 1, barrier)
        out["raw_4096x512x512_u16"] = {
            "tiles_per_s": round(len(raw) * 5 * world / dtr, 1),
            "k_extract_ms": round(ms_ext, 3),
            "k_extract_gbps": round(2 * sr.in_bytes / (ms_ext * 1e-3) / 1e9, 1),
            "k_extract_frac": round(2 * sr.in_bytes / (ms_ext * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
        # G_FAKE (FakeReader-like gradient) PNG, compressible data
        svc.register_plane(2, 0, 0, 0, pbx.UINT16, side, side, generator="fake", plane_no=rank)
        fk = grid_ctxs(2, "png")
        dtf, sf, msf, _, _ = run_steps(svc, fk, 3, 1, barrier)
        out["png_fake_4096x512x512_u16"] = {
            "tiles_per_s": round(len(fk) * 3 * world / dtf, 1),
            "compressed_bytes_per_tile": round(sf.deflate_out_bytes / len(fk), 1),
            "k_deflate_ms": round(msf, 3)}

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(threads=args.cpu_threads)
        out["speedup_vs_cpu_baseline"] = round(value / out["cpu_baseline"]["value"], 1)
    if rank == 0:
        print(json.dumps(out), flush=True)
    svc.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
