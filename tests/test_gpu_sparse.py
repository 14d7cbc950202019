"""Region-proportional residency on the GPU: sparse planes.

The reference reads only the requested region per request — ``new byte[w*h*bpp]`` then
``getTileDirect(z, c, t, x, y, w, h)`` (TileRequestHandler.java:102-109).  A sparse plane
(pbx_plane_create_sparse) is registered at once but holds its rows as bands, each loaded on
demand when a request's rows cover it, pinned by the batches reading it and evicted on its own
under the HBM budget.  A region straddling bands is gathered into a per-batch bridge buffer on
the GPU and served bit-exact.  Every body is checked against the CPU oracle's generator.
"""
import itertools
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import pbx

pytestmark = pytest.mark.gpu

_ids = itertools.count(800000, 10)
NOISE = 2
SEED = 13


class RowSource(pbx.PixelSource):
    """PixelSource over the oracle generator that counts what it reads (rows and calls, per
    band-aligned start row)."""

    def __init__(self, oracle, images):
        self.oracle, self.images = oracle, dict(images)
        self.reads, self.rows = 0, 0
        self.starts = []
        self.lock = threading.Lock()

    def get_pixels(self, image_id):
        return self.images.get(image_id)

    def read_rows(self, pixels, z, c, t, level, y0, rows):
        with self.lock:
            self.reads += 1
            self.rows += rows
            self.starts.append(y0)
        return self.oracle.gen_region(NOISE, pixels.pixel_type, 0, y0, pixels.size_x, rows, seed=SEED,
                                      z=z, c=c, t=t).tobytes()


def want(oracle, pt, x, y, w, h, c=0):
    return oracle.gen_region(NOISE, pt, x, y, w, h, seed=SEED, c=c).tobytes()


def check(oracle, pt, tc, body):
    ref = want(oracle, pt, tc.x, tc.y, tc.w, tc.h, c=tc.c)
    if tc.format is None:
        assert body == ref, (tc.x, tc.y, tc.w, tc.h)
    elif tc.format == "png":
        r, px, _ = oracle.png_decode(body)
        assert r == 0 and px == ref, (tc.x, tc.y, tc.w, tc.h)
    else:
        r, px, _ = oracle.tiff_decode(body, len(ref))
        assert r == 0 and px == ref, (tc.x, tc.y, tc.w, tc.h)


def test_whole_slide_tile_reads_only_its_bands(oracle):
    """A 100000^2 uint16 image (20 GB per plane): one 512^2 PNG tile is served after reading
    the 2 bands of 512 rows its rows cover (~205 MB, not 20 GB); tiles straddling the band
    boundary (raw at odd columns, PNG, TIFF) are served bit-exact from the bridge; a taller
    region loads the bands it adds; resident bands hold no other rows."""
    pt, side, B = pbx.UINT16, 100000, 512
    iid = next(_ids)
    src = RowSource(oracle, {iid: pbx.Pixels(iid, pt, side, side)})
    pitch = (side * 2 + 255) // 256 * 256
    with pbx.PixelsService(sparse_band_rows=B) as svc:
        tc = pbx.TileCtx(iid, 0, 0, 0, 40000, 50000, 512, 512, format="png")  # bands 97, 98
        check(oracle, pt, tc, pbx.TileRequestHandler(svc, tc, src).get_tile())
        assert src.reads == 2 and src.rows == 2 * B and sorted(src.starts) == [97 * B, 98 * B]
        s = svc.residency_stats()
        assert s["bands"] == 2 and s["planes"] == 0
        assert s["resident_bytes"] == 2 * (B * pitch + 256)
        pid = svc.lookup_plane(iid, 0, 0, 0)[0]
        br, states = svc.band_info(pid)
        assert br == B and len(states) == -(-side // B)
        assert [k for k, v in enumerate(states) if v == pbx.BS_READY] == [97, 98]
        # more tiles inside the two resident bands, several straddling the boundary at 50176
        ctxs = [pbx.TileCtx(iid, 0, 0, 0, 7, 50100, 333, 97),                      # raw, odd x
                pbx.TileCtx(iid, 0, 0, 0, 99488, 49664, 512, 1024, format="png"),  # both bands whole
                pbx.TileCtx(iid, 0, 0, 0, 64, 50170, 1000, 11, format="tif"),
                pbx.TileCtx(iid, 0, 0, 0, 16, 50176, 512, 300, format="png"),      # band 98 only
                pbx.TileCtx(iid, 0, 0, 0, 3, 49700, 1, 900),                        # 1 column
                pbx.TileCtx(iid, 0, 0, 0, 5000, 50175, 256, 2, format="png")]       # 1 row each side
        for c, (st, body) in zip(ctxs, svc.get_tiles(ctxs)):
            assert st == pbx.OK
            check(oracle, pt, c, body)
        assert src.reads == 2
        # a region over four bands (96..99): loads the two it adds, and only those
        tall = pbx.TileCtx(iid, 0, 0, 0, 123, 49200, 300, 1500, format="png")  # rows 49200..50700
        check(oracle, pt, tall, pbx.TileRequestHandler(svc, tall, src).get_tile())
        assert src.reads == 4 and sorted(src.starts[2:]) == [96 * B, 99 * B]
        assert svc.residency_stats()["bands"] == 4
        # the last band of the plane (100000 = 195 * 512 + 160 rows)
        last = pbx.TileCtx(iid, 0, 0, 0, side - 512, side - 160, 512, 160, format="png")
        check(oracle, pt, last, pbx.TileRequestHandler(svc, last, src).get_tile())
        assert src.starts[-1] == 195 * B and src.rows == 4 * B + 160
        # outside the plane is the reference's 404, with nothing loaded
        out = pbx.TileCtx(iid, 0, 0, 0, side - 100, 0, 512, 512)
        assert pbx.TileRequestHandler(svc, out, src).get_tile() is None
        assert src.reads == 5


def test_band_eviction_under_budget(oracle):
    """Under a budget of three bands, requests in five band rows evict least-recently-used idle
    bands one at a time (the plane stays registered and READY); an evicted band is loaded again
    when a request needs it; resident bytes never exceed the budget; every tile is exact."""
    pt, side, B = pbx.UINT16, 16384, 256
    iid = next(_ids)
    src = RowSource(oracle, {iid: pbx.Pixels(iid, pt, side, side)})
    band_bytes = B * side * 2 + 256
    with pbx.PixelsService(sparse_band_rows=B) as svc:
        svc.set_residency_budget(3 * band_bytes + 1000)
        order = [3, 10, 20, 3, 30, 40, 10]
        reads = []
        for k in order:
            tc = pbx.TileCtx(iid, 0, 0, 0, 1024, k * B + 16, 512, 200, format="png")
            check(oracle, pt, tc, pbx.TileRequestHandler(svc, tc, src).get_tile())
            s = svc.residency_stats()
            assert s["resident_bytes"] <= s["budget"] and s["bands"] <= 3
            reads.append(src.reads)
        # 3, 10, 20 load; 3 hits; 30 evicts 10 (LRU: 3 was used again); 40 evicts 20; 10 reloads
        assert reads == [1, 2, 3, 3, 4, 5, 6]
        s = svc.residency_stats()
        assert s["band_evictions"] == 3 and s["evictions"] == 3
        pid = svc.lookup_plane(iid, 0, 0, 0)[0]
        assert svc.lookup_plane(iid, 0, 0, 0)[1] == pbx.PS_READY
        assert [k for k, v in enumerate(svc.band_info(pid)[1]) if v == pbx.BS_READY] == [10, 30, 40]


def test_foreign_rows_stay_not_resident(oracle):
    """A rank's share (own rows [0, 51200) of a 100000-row slide): regions that start in rows of
    another rank answer NOT_RESIDENT in the library and None in the handler, and nothing is read
    for them; requests in the share load their bands; a region that starts in the share and runs
    past its end is served here, its rows past the share loaded as a guest band (ADVICE r04:
    the reference's getTileDirect serves any region of the plane)."""
    pt, side, B = pbx.UINT16, 100000, 512
    iid = next(_ids)
    src = RowSource(oracle, {iid: pbx.Pixels(iid, pt, side, side)})
    own = (0, 100 * B)
    with pbx.PixelsService(sparse_band_rows=B) as svc:
        foreign = pbx.TileCtx(iid, 0, 0, 0, 0, 60000, 512, 512)
        assert pbx.TileRequestHandler(svc, foreign, src, band=own).get_tile() is None
        assert src.reads == 0
        mine = pbx.TileCtx(iid, 0, 0, 0, 512, 51200 - 512, 512, 512, format="png")
        check(oracle, pt, mine, pbx.TileRequestHandler(svc, mine, src, band=own).get_tile())
        assert src.reads == 1
        (st, _), = svc.get_tiles([foreign])
        assert st == pbx.E_NOT_RESIDENT
        edge = pbx.TileCtx(iid, 0, 0, 0, 0, 51200 - 100, 64, 200)  # half in the share
        (st, _), = svc.get_tiles([edge])
        assert st == pbx.E_NOT_RESIDENT  # its guest band is not loaded yet
        check(oracle, pt, edge, pbx.TileRequestHandler(svc, edge, src, band=own).get_tile())
        pid = svc.lookup_plane(iid, 0, 0, 0)[0]
        states = svc.band_info(pid)[1]
        assert states[99] == 2 and states[100] == 2  # the share's last band and one guest band
        assert sum(states) == 2 * 2 and src.reads == 2  # the guest band is the one more read
        (st, _), = svc.get_tiles([foreign])
        assert st == pbx.E_NOT_RESIDENT  # still another rank's region
        with pytest.raises(pbx.PbxError) as e:
            svc.band_write(pid, side - 100, 200, bytes(200 * side * 2))  # past the plane
        assert e.value.status == pbx.E_BADARG


def test_concurrent_requests_read_each_band_once(oracle):
    """32 Vert.x-style workers ask for tiles of a cold sparse plane: each band is read from the
    PixelSource exactly once (one loader per band), every tile is exact."""
    pt, side, B = pbx.UINT8, 20000, 1024
    iid = next(_ids)
    src = RowSource(oracle, {iid: pbx.Pixels(iid, pt, side, side, size_c=2)})
    rng = np.random.default_rng(3)
    ctxs = [pbx.TileCtx(iid, 0, int(rng.integers(2)), 0, int(rng.integers(0, side - 512)),
                        int(rng.integers(4 * B, 7 * B)), 512, 512, format=["png", None, "tif"][k % 3])
            for k in range(192)]
    with pbx.PixelsService(sparse_band_rows=B) as svc:
        errors = []
        barrier = threading.Barrier(32)

        def worker(w):
            barrier.wait()
            for j in range(w, len(ctxs), 32):
                try:
                    check(oracle, pt, ctxs[j], pbx.TileRequestHandler(svc, ctxs[j], src).get_tile())
                except AssertionError:
                    errors.append(j)

        with ThreadPoolExecutor(32) as ex:
            list(ex.map(worker, range(32)))
        assert not errors, errors[:5]
        needed = {(c.c, k) for c in ctxs for k in range(c.y // B, (c.y + 511) // B + 1)}
        assert src.reads == len(needed)


def test_generated_sparse_plane_and_release_under_batch(service, oracle):
    """A generator sparse plane (bands generated on the GPU by pbx_band_write with no data)
    serves the generator's tiles; a pbx_plane_release between plan and launch defers the free
    of the pinned bands to pbx_batch_destroy."""
    pt, side, B = pbx.UINT16, 8192, 1000
    iid = next(_ids)
    pid = service.create_sparse_plane(iid, 0, 0, 0, pt, side, side, B, generator="noise", seed=SEED)
    (st, _), = service.get_tiles([pbx.TileCtx(iid, 0, 0, 0, 0, 0, 64, 64)])
    assert st == pbx.E_NOT_RESIDENT
    for k in (2, 3):
        service.band_write(pid, k * B, B, None)
    with pytest.raises(pbx.PbxError) as e:
        service.band_write(pid, 2 * B, B, None)  # already resident
    assert e.value.status == pbx.E_EXISTS
    ctxs = [pbx.TileCtx(iid, 0, 0, 0, 512 * i, 2 * B + 700 * j, 512, 512, format=f)
            for i in range(4) for j in range(2) for f in ("png", None)]
    b = pbx.Batch(service, ctxs)
    before = service.residency_stats()["resident_bytes"]
    service.release_plane(pid)
    assert service.residency_stats()["resident_bytes"] == before  # pinned by the batch
    b.launch()
    res = b.fetch()
    b.close()
    for c, (st, body) in zip(ctxs, res):
        assert st == pbx.OK
        check(oracle, pt, c, body)
    assert service.residency_stats()["resident_bytes"] < before


def _rows(oracle, x_size, y0, rows, seed=SEED):
    return oracle.gen_region(NOISE, pbx.UINT16, 0, y0, x_size, rows, seed=seed).tobytes()


def test_band_load_failures_give_the_band_back(oracle, monkeypatch):
    """a band whose load fails part-way never keeps HBM nor stays loading.
    (1) A write that fails after another piece of the band was written resets the band: absent,
    its bytes returned; a reload serves exact pixels.  (2) A failure while a second writer of
    the same band is still uploading: the band is reset only when that writer leaves (no upload
    lands in freed HBM), and that writer is told its load is void.  (3) pbx_band_abort after a
    partial load (the JNI shim's path for a Java exception between pieces).  (4) A band left
    loading by a loader that went away is started over by the next writer after the stale
    time ($PBX_BAND_STALE_MS)."""
    monkeypatch.setenv("PBX_BAND_STALE_MS", "300")
    sx, sy, B = 4096, 2048, 512
    with pbx.PixelsService() as svc:
        iid = next(_ids)
        pid = svc.create_sparse_plane(iid, 0, 0, 0, pbx.UINT16, sx, sy, B)
        base = svc.residency_stats()["resident_bytes"]

        def tile_ok(y):
            st, body = svc.get_tile(pbx.TileCtx(iid, 0, 0, 0, 100, y, 512, 256))
            assert st == pbx.OK and body == oracle.gen_region(NOISE, pbx.UINT16, 100, y, 512, 256,
                                                                 seed=SEED).tobytes()

        # (1) piece 1 written, piece 2's upload fails
        svc.band_write(pid, 0, 256, _rows(oracle, sx, 0, 256))
        assert svc.band_info(pid)[1][0] == 1  # loading
        svc.test_fail_band_write(1)
        with pytest.raises(pbx.PbxError):
            svc.band_write(pid, 256, 256, _rows(oracle, sx, 256, 256))
        assert svc.band_info(pid)[1][0] == 0
        assert svc.residency_stats()["resident_bytes"] == base
        assert svc.get_tile(pbx.TileCtx(iid, 0, 0, 0, 0, 0, 64, 64))[0] == pbx.E_NOT_RESIDENT
        svc.band_write(pid, 0, 512, _rows(oracle, sx, 0, 512))
        tile_ok(100)

        # (2) two writers of band 1: the second fails while the first uploads 512 rows
        big = _rows(oracle, sx, 512, 512)
        svc.band_write(pid, 512, 8, big[:8 * sx * 2])  # the band exists (loading, allocated)
        errs = {}

        def first():
            try:
                svc.band_write(pid, 520, 504, big[8 * sx * 2:])
            except pbx.PbxError as e:
                errs["first"] = e.status
        th = threading.Thread(target=first)
        svc.test_fail_band_write(2)  # the first writer's call is write 1 from here, this one write 2
        th.start()
        try:
            svc.band_write(pid, 512, 8, big[:8 * sx * 2])
        except pbx.PbxError as e:
            errs["second"] = e.status
        th.join(timeout=60)
        # whichever ordering happened, the band is never published half-written: either both
        # writes failed and the band is absent, or the failed write came first, the band was
        # reset and the other write started it over (loading, its rows only)
        st1 = svc.band_info(pid)[1][1]
        assert "second" in errs or "first" in errs
        if st1 == 2:
            raise AssertionError("a band with a failed write was published")
        svc.band_abort(pid, 512)
        assert svc.band_info(pid)[1][1] == 0
        svc.band_write(pid, 512, 512, big)
        tile_ok(700)
        assert svc.residency_stats()["resident_bytes"] == base + 2 * (sx * 2 * B + 256)

        # (3) partial load, then the loader gives up: absent, bytes returned, reload works
        svc.band_write(pid, 1024, 100, _rows(oracle, sx, 1024, 100))
        svc.band_abort(pid, 1024)
        assert svc.band_info(pid)[1][2] == 0
        assert svc.residency_stats()["resident_bytes"] == base + 2 * (sx * 2 * B + 256)
        svc.band_write(pid, 1024, 512, _rows(oracle, sx, 1024, 512))
        tile_ok(1200)

        # (4) a loader that went away part-way: the band reads as loading within the stale time,
        # then as absent (its HBM returned), so a waiting binding loads it again
        svc.band_write(pid, 1536, 100, b"\xff" * (sx * 2 * 100))  # never finished
        assert svc.band_info(pid)[1][3] == 1
        time.sleep(0.5)
        assert svc.band_info(pid)[1][3] == 0
        assert svc.residency_stats()["resident_bytes"] == base + 3 * (sx * 2 * B + 256)
        svc.band_write(pid, 1536, 512, _rows(oracle, sx, 1536, 512))
        tile_ok(1700)
        assert svc.band_info(pid)[1] == [2, 2, 2, 2]

        # (5) ADVICE r05: a live loader whose pieces come more than the stale time apart has its
        # load reset under it; its next piece fails (500, load again from the band's first row)
        # instead of silently starting a load that could never complete
        pid2 = svc.create_sparse_plane(next(_ids), 0, 0, 0, pbx.UINT16, sx, 1024, B)
        svc.band_write(pid2, 0, 100, _rows(oracle, sx, 0, 100))
        time.sleep(0.5)
        with pytest.raises(pbx.PbxError) as ei:
            svc.band_write(pid2, 100, 412, _rows(oracle, sx, 100, 412))
        assert ei.value.status == pbx.E_INTERNAL
        assert svc.band_info(pid2)[1] == [0, 0]
        # the same after band_info did the reset: a piece past the first row still fails
        svc.band_write(pid2, 512, 64, _rows(oracle, sx, 512, 64))
        time.sleep(0.5)
        assert svc.band_info(pid2)[1] == [0, 0]
        with pytest.raises(pbx.PbxError):
            svc.band_write(pid2, 576, 448, _rows(oracle, sx, 576, 448))
        svc.band_write(pid2, 512, 512, _rows(oracle, sx, 512, 512))  # from the first row: loads
        svc.band_write(pid2, 0, 512, _rows(oracle, sx, 0, 512))
        assert svc.band_info(pid2)[1] == [2, 2]


class PoissonRows(pbx.PixelSource):
    """Poisson-like uint16 counts (lambda 250) row by row, each row seeded by its index: the
    rows the adaptive filter's tile mode sends to filter None."""

    def __init__(self, images):
        self.images = dict(images)

    def get_pixels(self, image_id):
        return self.images.get(image_id)

    @staticmethod
    def rows(size_x, y0, n):
        return np.concatenate([np.random.default_rng(1000 + y).poisson(250.0, size_x).astype(">u2")
                               for y in range(y0, y0 + n)]).view(np.uint8)

    def read_rows(self, pixels, z, c, t, level, y0, rows):
        return self.rows(pixels.size_x, y0, rows).tobytes()


@pytest.mark.parametrize("kind", ["poisson", "noise"])
def test_adaptive_filter_on_sparse_bands_and_bridges(oracle, kind):
    """The adaptive PNG filter on a sparse plane: tiles inside one band and tiles straddling
    bands (gathered into the batch's bridge buffer), at aligned and odd x, on Poisson-like
    rows (None mode: the direct path reads the band or the bridge) and on G_NOISE (the filter
    kernels): every IDAT equals the oracle's adaptive scanlines of the generator's tile."""
    pt, sx, sy, B = pbx.UINT16, 4096, 4096, 256
    iid = next(_ids)
    src = (PoissonRows({iid: pbx.Pixels(iid, pt, sx, sy)}) if kind == "poisson"
           else RowSource(oracle, {iid: pbx.Pixels(iid, pt, sx, sy)}))
    regions = [(0, 0, 512, 256), (512, 256, 512, 512), (1024, 200, 512, 112), (8, 250, 256, 10),
               (3, 700, 300, 77), (2048, 1020, 64, 8), (4000, 500, 96, 300), (17, 255, 33, 2)]
    with pbx.PixelsService(sparse_band_rows=B, png_filter=pbx.FILTER_ADAPTIVE) as svc:
        bodies = []
        for x, y, w, h in regions:
            tc = pbx.TileCtx(iid, 0, 0, 0, x, y, w, h, format="png")
            bodies.append(pbx.TileRequestHandler(svc, tc, src).get_tile())
        ctxs = [pbx.TileCtx(iid, 0, 0, 0, x, y, w, h, format="png") for x, y, w, h in regions]
        bodies2 = [b for st, b in svc.get_tiles(ctxs)]  # all at once: one batch, bridges included
    modes = []
    for (x, y, w, h), b1, b2 in zip(regions, bodies, bodies2):
        if kind == "poisson":
            tile = PoissonRows.rows(sx, y, h).reshape(h, sx * 2)[:, 2 * x:2 * (x + w)].reshape(-1).copy()
        else:
            tile = oracle.gen_region(NOISE, pt, x, y, w, h, seed=SEED)
        want_s = oracle.png_filter_stream(tile, pt, w, h, pbx.FILTER_ADAPTIVE).tobytes()
        for body in (b1, b2):
            r, idat = oracle.png_inflate_idat(bytes(body), len(want_s))
            assert r == 0 and idat == want_s, (kind, x, y, w, h)
        modes.append(oracle.adaptive_tile_none(tile, pt, w, h))
    if kind == "poisson":
        assert sum(modes) >= 6
