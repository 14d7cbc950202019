"""Serving-path parity on the GPU:

* configs[0] at its own workload: 512x512 uint8 PNG tiles of a 4096^2 Bio-Formats-fake
  (G_FAKE) plane, the reference's CPU case (TileRequestHandler.java:119-124,176-199);
* the reference's 404s are answered before anything is loaded (:84, :100-103, :125-132);
* a device failure fails its batch with 500 and nothing else (PixelBufferVerticle.java:
  131-146; SURVEY.md §5 fault injection), through the coalescer and the batch paths;
* a batch that never completes answers 500 at the request deadline (the event-bus send
  timeout, PixelBufferMicroserviceVerticle.java:148-151,356-366) and nothing else;
* N device contexts in one process (the reference's one JVM, PixelBufferMicroserviceVerticle.
  java:117-118,224-233): requests routed by band ownership and pbx_shard_of.

Every body is checked against the CPU oracle (oracle/pbx_oracle.c).
"""
import itertools
import threading
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import pbx
import _emu

pytestmark = pytest.mark.gpu

_ids = itertools.count(650000, 10)  # disjoint from test_gpu_sweep (700000..)
FAKE, NOISE = 1, 2


# ------------------------------------------------------------------- configs[0]

C1_TILES = [(0, 0), (512, 0), (1536, 2048), (3584, 3584)]


def test_c1_png_512x512_u8_fake(service, oracle):
    """BASELINE configs[0]: 512x512 uint8 PNG tiles from a 4096^2 G_FAKE plane.  Each decodes
    to the oracle's pixels, its inflated IDAT is the oracle's filter-None scanlines, and its
    zlib stream is the CPU emulation of the deflate workgroups byte for byte; the single-tile
    path (pbx_get_tile through the coalescer, as one Vert.x worker calls it) returns the same
    bytes as the batch path on every repetition."""
    iid = next(_ids)
    pt, side = pbx.UINT8, 4096
    service.register_plane(iid, 0, 0, 0, pt, side, side, generator="fake")
    ctxs = [pbx.TileCtx(iid, 0, 0, 0, x, y, 512, 512, format="png") for x, y in C1_TILES]
    res = service.get_tiles(ctxs)
    z6 = []
    for (x, y), (st, body) in zip(C1_TILES, res):
        assert st == pbx.OK
        tile = oracle.gen_region(FAKE, pt, x, y, 512, 512)
        r, px, meta = oracle.png_decode(body)
        assert r == 0 and px == tile.tobytes(), (x, y)
        assert (meta["w"], meta["h"], meta["depth"], meta["color_type"]) == (512, 512, 8, 0)
        stream = oracle.png_filter_stream(tile, pt, 512, 512, 0).tobytes()
        r, idat = oracle.png_inflate_idat(body, len(stream))
        assert r == 0 and idat == stream
        z, _ = _emu.deflate(stream, 513)
        assert body[99:99 + len(z)] == z
        z6.append(len(zlib.compress(stream, 6)))
    # compressed size against the reference's zlib-6 (ImageIO) stream, recorded for DESIGN §2
    mine = [int.from_bytes(b[91:95], "big") for _, b in res]
    assert all(m <= 2 * max(z, 1024) for m, z in zip(mine, z6)), (mine, z6)
    # the served single-tile path: identical bytes, every time
    first = res[0][1]
    for _ in range(20):
        st, body = service.get_tile(pbx.TileCtx(iid, 0, 0, 0, 0, 0, 512, 512, format="png"))
        assert st == pbx.OK and body == first
    # and through the event-bus consumer: 200, the filename and Content-Type headers
    st, body, hdr = pbx.handle_get_tile(service, pbx.TileCtx(iid, 0, 0, 0, 0, 0, 512, 512,
                                                               format="png").to_json())
    assert st == 200 and body == first and hdr["Content-Type"] == "image/png"
    assert hdr["filename"] == "image%d_z0_c0_t0_x0_y0_w512_h512.png" % iid


# ------------------------------------------------------- 404 before NOT_RESIDENT

class CountingSource(pbx.PixelSource):
    def __init__(self, oracle, images):
        self.oracle, self.images = oracle, dict(images)
        self.lookups = self.reads = 0
        self.lock = threading.Lock()

    def get_pixels(self, image_id):
        with self.lock:
            self.lookups += 1
        return self.images.get(image_id)

    def read_rows(self, pixels, z, c, t, level, y0, rows):
        with self.lock:
            self.reads += 1
        return self.oracle.gen_region(NOISE, pixels.pixel_type, 0, y0, pixels.size_x, rows, seed=11,
                                      z=z, c=c, t=t).tobytes()


def test_cold_image_404s_load_nothing(service, oracle):
    """format=jpg, or a region no pixel type makes a Java byte[], on an image this context has
    never seen: the reference's 404 at once (TileRequestHandler.java:100-103,125-126), with no
    getPixels and no PixelSource read; a good request on the same cold image loads it."""
    iid = next(_ids)
    src = CountingSource(oracle, {iid: pbx.Pixels(iid, pbx.UINT16, 3000, 2000)})
    for tc in (pbx.TileCtx(iid, 0, 0, 0, 0, 0, 64, 64, format="jpg"),
               pbx.TileCtx(iid, 0, 0, 0, 0, 0, 64, 64, format="PNG"),
               pbx.TileCtx(iid, 0, 0, 0, 0, 0, 50000, 50000),
               pbx.TileCtx(iid, 0, 0, 0, 0, 0, -5, 64)):
        assert pbx.TileRequestHandler(service, tc, src).get_tile() is None
        st, _, _ = pbx.handle_get_tile(service, tc.to_json(), src)
        assert st == 404
    assert (src.lookups, src.reads) == (0, 0)
    tc = pbx.TileCtx(iid, 0, 0, 0, 100, 50, 64, 64)
    assert pbx.TileRequestHandler(service, tc, src).get_tile() == \
        oracle.gen_region(NOISE, pbx.UINT16, 100, 50, 64, 64, seed=11).tobytes()
    assert src.reads >= 1
    service.release_image(iid)


def test_stage_spans_under_the_reference_names(service, oracle):
    """The reference's tracing spans (TileRequestHandler.java:81 get_tile, :104 get_tile_direct,
    :147 create_metadata, :180 write_image): a cold PNG request records get_pixels and the
    region load, then the serving batch's device stages; a raw request's gather is its
    get_tile_direct, a PNG's is inside write_image."""
    iid = next(_ids)
    src = CountingSource(oracle, {iid: pbx.Pixels(iid, pbx.UINT16, 1500, 900)})
    seen = []
    tracer = lambda name, ms, tags: seen.append((name, ms, tags))
    tc = pbx.TileCtx(iid, 0, 0, 0, 64, 32, 512, 256, format="png")
    body = pbx.TileRequestHandler(service, tc, src, tracer=tracer).get_tile()
    r, px, _ = oracle.png_decode(body)
    assert r == 0 and px == oracle.gen_region(NOISE, pbx.UINT16, 64, 32, 512, 256, seed=11).tobytes()
    names = [n for n, _, _ in seen]
    assert names[-1] == "get_tile" and {"get_pixels", "load_region", "get_tile_direct",
                                        "create_metadata", "write_image", "d2h"} <= set(names)
    sp = {n: (ms, t) for n, ms, t in seen}
    assert sp["write_image"][0] > 0 and sp["create_metadata"][0] >= 0
    assert sp["write_image"][1]["batch_tiles"] >= 1
    assert sp["get_tile"][0] >= sp["write_image"][0]
    seen.clear()
    tc = pbx.TileCtx(iid, 0, 0, 0, 0, 0, 256, 256)
    body = pbx.TileRequestHandler(service, tc, src, tracer=tracer).get_tile()
    assert body == oracle.gen_region(NOISE, pbx.UINT16, 0, 0, 256, 256, seed=11).tobytes()
    sp = {n: ms for n, ms, _ in seen}
    assert "get_pixels" not in sp and sp["get_tile_direct"] > 0 and sp["write_image"] < 0.05
    # an error status has no body and no batch spans
    seen.clear()
    assert pbx.TileRequestHandler(service, pbx.TileCtx(iid, 0, 0, 0, 0, 0, 64, 64, format="jpg"),
                                  src, tracer=tracer).get_tile() is None
    assert [n for n, _, _ in seen] == ["get_tile"]
    # the event-bus consumer's own span closes the request
    seen.clear()
    st, _, _ = pbx.handle_get_tile(service, pbx.TileCtx(iid, 0, 0, 0, 0, 0, 128, 128).to_json(), src,
                                   tracer=tracer)
    assert st == 200 and [n for n, _, _ in seen][-2:] == ["get_tile", "handle_get_tile"]
    service.release_image(iid)


def test_eviction_between_load_and_retry_is_never_404(oracle):
    """a budget that holds ONE plane and concurrent requests to two planes: a plane
    evicted between its load and the retry is loaded again; every tile is served exactly, none
    answers 404."""
    pt, side = pbx.UINT16, 1024
    pbytes = (side * 2 + 255) // 256 * 256 * side + 256
    iid = next(_ids)
    src = CountingSource(oracle, {iid: pbx.Pixels(iid, pt, side, side, size_c=2)})
    with pbx.PixelsService() as svc:
        svc.set_residency_budget(int(1.5 * pbytes))
        ctxs = [pbx.TileCtx(iid, 0, k % 2, 0, 64 * (k % 7), 32 * (k % 5), 256, 256) for k in range(96)]
        errors = []

        def one(tc):
            try:
                body = pbx.TileRequestHandler(svc, tc, src).get_tile()
            except pbx.PbxError as e:  # a plane that cannot be held is a 500, never a 404
                assert e.status in (pbx.E_INTERNAL, pbx.E_NO_SPACE)  # both -> 500 (handle_get_tile)
                return "500"
            want = oracle.gen_region(NOISE, pt, tc.x, tc.y, 256, 256, seed=11, c=tc.c).tobytes()
            if body != want:
                errors.append((tc.c, tc.x, tc.y))
            return "ok"

        with ThreadPoolExecutor(16) as ex:
            outcomes = list(ex.map(one, ctxs))
        assert not errors, errors[:4]
        # a loaded plane is kept until its first read (the library's fresh protection) and a
        # loader that finds the budget held waits: (almost) nothing is given up
        assert outcomes.count("ok") >= len(ctxs) - 2, outcomes
        assert svc.residency_stats()["evictions"] >= 1


# ------------------------------------------------------------- fault injection

def test_failed_batch_is_500_for_its_requests_only(oracle):
    """PBX fault injection: the 3rd batch the coalescer launches fails on the device.  With 32
    concurrent callers, exactly that batch's requests answer 500 (a request that is the
    reference's 404 keeps its 404), every other response is exact, and the context serves
    normally afterwards (PixelBufferVerticle.java:131-146)."""
    iid = next(_ids)
    pt, side = pbx.UINT16, 4096
    with pbx.PixelsService() as svc:
        svc.register_plane(iid, 0, 0, 0, pt, side, side, generator="noise", seed=11)
        rng = np.random.default_rng(4)
        reqs = []
        for k in range(512):
            if k % 17 == 5:
                reqs.append(pbx.TileCtx(iid, 0, 0, 0, side - 10, 0, 64, 64, format="png"))  # 404
            else:
                x, y = (int(v) for v in rng.integers(0, side - 256, 2))
                reqs.append(pbx.TileCtx(iid, 0, 0, 0, x, y, 256, 256, format=["png", None, "tif"][k % 3]))
        b0, _ = svc.ctx_stats()
        svc.test_fail_batch(3)
        out = [None] * len(reqs)
        barrier = threading.Barrier(32)

        def worker(w):
            barrier.wait()
            for j in range(w, len(reqs), 32):
                out[j] = svc.get_tile(reqs[j])

        with ThreadPoolExecutor(32) as ex:
            list(ex.map(worker, range(32)))
        failed = [j for j, (st, _) in enumerate(out) if st == pbx.E_INTERNAL]
        assert 1 <= len(failed) <= 64, len(failed)  # one coalesced batch (<= 64 requests)
        for j, (st, body) in enumerate(out):
            tc = reqs[j]
            if tc.x == side - 10:
                assert st == 404 and body is None
                continue
            if j in failed:
                assert body is None
                continue
            assert st == pbx.OK, (j, st)
            want = oracle.gen_region(NOISE, pt, tc.x, tc.y, 256, 256, seed=11)
            if tc.format is None:
                assert body == want.tobytes()
            elif tc.format == "png":
                r, px, _ = oracle.png_decode(body)
                assert r == 0 and px == want.tobytes()
            else:
                assert body == oracle.tiff_encode(want, pt, 256, 256)[1]
        b1, _ = svc.ctx_stats()
        assert b1 - b0 >= 3
        # the context keeps serving, on every path; and the event-bus consumer maps 500
        st, body = svc.get_tile(reqs[0])
        assert st == pbx.OK
        svc.test_fail_batch(1)
        st, _, _ = pbx.handle_get_tile(svc, reqs[0].to_json())
        assert st == 500
        svc.test_fail_batch(1)  # pbx_get_tiles (one synchronous batch)
        res = svc.get_tiles(reqs[:8])
        assert all(s == (404 if r.x == side - 10 else 500) for r, (s, _) in zip(reqs[:8], res))
        svc.test_fail_batch(2)  # pbx_submit / pbx_wait: the second of two tickets fails
        t1, t2 = svc.submit(reqs[:8]), svc.submit(reqs[8:16])
        assert all(s == (404 if r.x == side - 10 else 0) for r, (s, _) in zip(reqs[:8], t1.wait()))
        assert all(s == (404 if r.x == side - 10 else 500) for r, (s, _) in zip(reqs[8:16], t2.wait()))
        assert [s for s, _ in svc.get_tiles(reqs[16:24])] == [404 if r.x == side - 10 else 0 for r in reqs[16:24]]


def _check_body(oracle, tc, st, body, pt, seed):
    assert st == pbx.OK, st
    want = oracle.gen_region(NOISE, pt, tc.x, tc.y, tc.w, tc.h, seed=seed)
    if tc.format is None:
        assert body == want.tobytes()
    elif tc.format == "png":
        r, px, _ = oracle.png_decode(body)
        assert r == 0 and px == want.tobytes()
    else:
        assert body == oracle.tiff_encode(want, pt, tc.w, tc.h)[1]


def test_stalled_batch_answers_500_at_deadline(oracle):
    """the reference bounds every getTile by the event-bus send timeout
    (PixelBufferMicroserviceVerticle.java:148-151; a timeout is a 500, :356-366).  A batch that
    never completes (pbx_test_stall_batch: its kernels queue behind a spinning wave) answers its
    caller 500 at pbx_config.request_timeout_us while 31 other callers, whose batches queue
    behind it on the device, get every body exact once the stall is released; no caller stays
    parked, and the context serves normally afterwards, on every path."""
    iid = next(_ids)
    pt, side, seed = pbx.UINT16, 4096, 12
    D = 1.5  # seconds
    with pbx.PixelsService(request_timeout_us=int(D * 1e6)) as svc:
        svc.register_plane(iid, 0, 0, 0, pt, side, side, generator="noise", seed=seed)
        rng = np.random.default_rng(6)
        reqs = []
        for k in range(256):
            x, y = (int(v) for v in rng.integers(0, side - 256, 2))
            reqs.append(pbx.TileCtx(iid, 0, 0, 0, x, y, 256, 256, format=["png", None, "tif"][k % 3]))
        st, body = svc.get_tile(reqs[0])  # warm: the first batch allocates the pools
        _check_body(oracle, reqs[0], st, body, pt, seed)
        svc.test_stall_batch(1)
        stalled = {}

        def caller_a():
            t = time.monotonic()
            stalled["res"] = svc.get_tile(reqs[1])
            stalled["s"] = time.monotonic() - t

        ta = threading.Thread(target=caller_a)
        ta.start()
        time.sleep(0.6)  # the stalled batch holds reqs[1] alone; the rest queue behind it
        out = [None] * len(reqs)

        def worker(w):
            for j in range(2 + w, len(reqs), 31):
                out[j] = svc.get_tile(reqs[j])

        with ThreadPoolExecutor(31) as ex:
            futs = [ex.submit(worker, w) for w in range(31)]
            ta.join(timeout=D + 5)
            assert not ta.is_alive(), "the stalled request's caller is still parked"
            svc.test_stall_batch(0)  # release: the late batch completes, the queue drains
            for f in futs:
                f.result(timeout=60)
        st, body = stalled["res"]
        assert st == pbx.E_INTERNAL and body is None
        assert D - 0.05 <= stalled["s"] < D + 1.0, stalled["s"]
        for j in range(2, len(reqs)):
            _check_body(oracle, reqs[j], *out[j], pt, seed)
        # the context serves on: coalescer, event-bus consumer, batches
        _check_body(oracle, reqs[1], *svc.get_tile(reqs[1]), pt, seed)
        st, _, _ = pbx.handle_get_tile(svc, reqs[2].to_json())
        assert st == 200
        svc.test_stall_batch(1)
        t = time.monotonic()
        st, _, _ = pbx.handle_get_tile(svc, reqs[3].to_json())  # the event-bus reply: 500
        assert st == 500 and time.monotonic() - t < D + 1.0
        svc.test_stall_batch(0)
        res = svc.get_tiles(reqs[:8])
        for tc, (st, body) in zip(reqs[:8], res):
            _check_body(oracle, tc, st, body, pt, seed)
    # one batch per call (coalesce off) and the node's routed call take the same deadline
    with pbx.PixelsService(coalesce=False, request_timeout_us=int(D * 1e6)) as svc:
        svc.register_plane(iid, 0, 0, 0, pt, side, side, generator="noise", seed=seed)
        _check_body(oracle, reqs[0], *svc.get_tile(reqs[0]), pt, seed)
        svc.test_stall_batch(1)
        t = time.monotonic()
        st, body = svc.get_tile(reqs[1])
        assert st == pbx.E_INTERNAL and body is None and D - 0.05 <= time.monotonic() - t < D + 1.0
        svc.test_stall_batch(0)
        for tc in reqs[2:6]:  # (the first of them also collects the late batch)
            _check_body(oracle, tc, *svc.get_tile(tc), pt, seed)
    with pbx.PixelsNode(1, devices=[0], request_timeout_us=int(D * 1e6)) as node:
        node.services[0].register_plane(iid, 0, 0, 0, pt, side, side, generator="noise", seed=seed)
        node.services[0].test_stall_batch(1)
        t = time.monotonic()
        st, body, k = node.get_tile(reqs[1])
        assert st == pbx.E_INTERNAL and body is None and time.monotonic() - t < D + 1.0
        node.services[0].test_stall_batch(0)
        st, body, k = node.get_tile(reqs[2])
        _check_body(oracle, reqs[2], st, body, pt, seed)


def test_direct_caller_keeps_deadline_while_run_mu_held(oracle):
    """a lone request that finds the coalescer idle is planned and launched
    by its own thread -- but only if the launch lock (run_mu) is free.  Here a batch submitted
    outside the coalescer stalls on the device and pbx_release_cached holds run_mu while it waits
    for the kernel streams; a lone pbx_get_tile must still answer 500 at its deadline
    (PixelBufferMicroserviceVerticle.java:148-151,356-366), and everything completes exactly once
    the stall is released."""
    iid = next(_ids)
    pt, side, seed = pbx.UINT16, 2048, 13
    D = 1.0
    with pbx.PixelsService(request_timeout_us=int(D * 1e6)) as svc:
        svc.register_plane(iid, 0, 0, 0, pt, side, side, generator="noise", seed=seed)
        reqs = [pbx.TileCtx(iid, 0, 0, 0, 100 * k, 37 * k, 256, 200, format=["png", None, "tif"][k % 3])
                for k in range(6)]
        _check_body(oracle, reqs[0], *svc.get_tile(reqs[0]), pt, seed)
        svc.test_stall_batch(1)
        ticket = svc.submit([reqs[1]])  # pbx_submit: stalled on the device, not the coalescer's
        holder = threading.Thread(target=svc.release_cached)  # takes run_mu, waits for the streams
        holder.start()
        time.sleep(0.3)
        assert holder.is_alive()
        t = time.monotonic()
        st, body = svc.get_tile(reqs[2])  # the coalescer is idle: the direct path
        took = time.monotonic() - t
        svc.test_stall_batch(0)
        holder.join(timeout=30)
        assert not holder.is_alive()
        assert st == pbx.E_INTERNAL and body is None
        assert D - 0.05 <= took < D + 0.5, took
        (s1, b1), = ticket.wait()
        _check_body(oracle, reqs[1], s1, b1, pt, seed)
        for tc in reqs[2:]:
            _check_body(oracle, tc, *svc.get_tile(tc), pt, seed)


def test_uncoalesced_late_batch_is_collected_while_idle(oracle):
    """an uncoalesced pbx_get_tile past its deadline parks its batch; the
    context's reaper thread collects it once it completes, with no later call on the context,
    so its plane pin goes: a plane released meanwhile gives its HBM back."""
    iid = next(_ids)
    pt, side, seed = pbx.UINT16, 2048, 14
    D = 0.5
    with pbx.PixelsService(coalesce=False, request_timeout_us=int(D * 1e6)) as svc:
        before = svc.residency_stats()["resident_bytes"]
        pid = svc.register_plane(iid, 0, 0, 0, pt, side, side, generator="noise", seed=seed)
        tc = pbx.TileCtx(iid, 0, 0, 0, 64, 64, 256, 256, format="png")
        _check_body(oracle, tc, *svc.get_tile(tc), pt, seed)
        svc.test_stall_batch(1)
        t = time.monotonic()
        st, body = svc.get_tile(tc)
        assert st == pbx.E_INTERNAL and body is None and D - 0.05 <= time.monotonic() - t < D + 0.5
        svc.release_plane(pid)  # the parked batch still pins it
        assert svc.residency_stats()["resident_bytes"] > before
        svc.test_stall_batch(0)
        deadline = time.monotonic() + 5
        while svc.residency_stats()["resident_bytes"] > before and time.monotonic() < deadline:
            time.sleep(0.02)
        assert svc.residency_stats()["resident_bytes"] == before


# ---------------------------------------------------------------- node routing

def test_node_two_contexts_one_device(oracle):
    """Two contexts in one process on device 0 (SURVEY §4.5 "fake device count"): a slide split
    into two row bands (context 0 holds rows [0, 2048), context 1 rows [2048, 4096)) and a plane
    replicated in both.  32 concurrent callers through pbx_node_get_tile: band requests land on
    their owner, replicated ones on their pbx_shard_of owner, and every body is exact."""
    pt, side = pbx.UINT16, 4096
    slide, rep = next(_ids), next(_ids)
    with pbx.PixelsNode(2, devices=[0, 0]) as node:
        for k, s_ in enumerate(node.services):
            s_.create_plane(slide, 0, 0, 0, pt, side, side, band=(2048 * k, 2048), generator="noise",
                            seed=11)
            s_.register_plane(rep, 0, 0, 0, pt, side, side, generator="noise", seed=11)
        rng = np.random.default_rng(8)
        reqs = []
        for k in range(640):
            img = slide if k % 2 else rep
            x = int(rng.integers(0, side // 512)) * 512
            y = int(rng.integers(0, side // 512)) * 512
            reqs.append(pbx.TileCtx(img, 0, 0, 0, x, y, 512, 512, format=["png", None][k % 4 == 1]))
        # a region straddling the two bands: no context holds it
        st, owner = node.route(pbx.TileCtx(slide, 0, 0, 0, 0, 2000, 512, 512))
        assert st == pbx.E_NOT_RESIDENT and owner == pbx.shard_of(pbx.TileCtx(slide, 0, 0, 0, 0, 2000, 512, 512), 2)
        out = [None] * len(reqs)
        barrier = threading.Barrier(32)

        def worker(w):
            barrier.wait()
            for j in range(w, len(reqs), 32):
                out[j] = node.get_tile(reqs[j])

        with ThreadPoolExecutor(32) as ex:
            list(ex.map(worker, range(32)))
        served = [0, 0]
        for tc, (st, body, k) in zip(reqs, out):
            assert st == pbx.OK
            if tc.imageId == slide:
                assert k == (0 if tc.y < 2048 else 1)
            else:
                assert k == pbx.shard_of(tc, 2)
            served[k] += 1
            want = oracle.gen_region(NOISE, pt, tc.x, tc.y, 512, 512, seed=11).tobytes()
            if tc.format is None:
                assert body == want
            else:
                r, px, _ = oracle.png_decode(body)
                assert r == 0 and px == want
        assert min(served) > 100
        stats = [s_.ctx_stats()[1] for s_ in node.services]
        assert sum(stats) == len(reqs) and min(stats) > 100
