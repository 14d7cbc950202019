"""The JNI shim (jni/pbx_jni.c) driven against the REAL lib/libpbx.so on the GPU (VERDICT r03
item 2).  There is no JDK in this image, so the shim is compiled over the mock VM of
tests/jni_mock/mock_vm.h and driven by tests/jni_mock/jni_real.c through the sequence the
handler of INTEGRATION.md §2 runs (TileRequestHandler.java:84-128; PixelBufferVerticle.java:
109-146): declareImage, createPlane + writeRows in 64 MiB bands of a 33000^2 uint16 plane
(2.18 GB: more than a Java byte[] holds), commitPlane, getTile raw / png / tif (rows above
2 GiB), NOT_RESIDENT, the reference's 404s (region, format "jpg" on a resident and on a cold
image, Java-int overflow), registerZarr of a c-blosc 1.21 fixture, and an injected device
failure (RuntimeException -> 500) after which the context keeps serving, and a stalled batch
(RuntimeException -> 500 at the request deadline, then served again).  Every body is
checked against the CPU oracle."""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MOCK = os.path.join(ROOT, "tests", "jni_mock")
EXE = os.path.join(MOCK, "build", "jni_real")
ZARR = "blosc_lz4_u16_100x77"  # shape [100, 77] (rows, columns), dtype >u2
SX = SY = 33000
NOISE, SEED = 2, 3


def test_jni_shim_on_real_library(tmp_path, oracle):
    if not os.path.exists(EXE):  # built by __graft_entry__.build(); gcc is on the box as well
        subprocess.check_call(["make", "-s", "-C", MOCK])
    enc = os.path.join(ROOT, "tests", "golden", "zarr", ZARR + ".enc")
    env = dict(os.environ, PBX_REQUEST_TIMEOUT_US="3000000")  # the "stalled" request's deadline
    out = subprocess.run([EXE, str(tmp_path), enc, "77", "100"], capture_output=True, text=True,
                         timeout=240, env=env)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert "jni real ok" in out.stdout
    tiles, served_by = {}, {}
    for line in out.stdout.splitlines():
        if line.startswith("TILE "):
            _, name, st, n, w, h, served = line.split()
            body = None
            path = tmp_path / (name + ".bin")
            if path.exists():
                body = path.read_bytes()
                assert len(body) == int(n)
            tiles[name] = (int(st), body, int(w), int(h))
            served_by[name] = int(served)
    assert "BANDS 33" in out.stdout  # 64 MiB bands of 1016 rows

    def want(x, y, w, h):
        return oracle.gen_region(NOISE, oracle.UINT16, x, y, w, h, seed=SEED).tobytes()

    assert tiles["before_load"][0] == 460  # declared, not loaded: load and retry
    for name, (x, y, w, h) in (("raw_0", (0, 0, 512, 512)), ("raw_hi", (20000, 32488, 512, 512)),
                               ("raw_row", (100, 32999, 1000, 1))):
        st, body, ow, oh = tiles[name]
        assert st == 0 and body == want(x, y, w, h), name
        assert (ow, oh) == (w, h)
    for name, (x, y, w, h) in (("png_0", (0, 0, 512, 512)), ("png_hi", (32488, 32488, 512, 512)),
                               ("png_odd", (7, 16270, 333, 97))):
        st, body, _, _ = tiles[name]
        assert st == 0, name
        r, px, meta = oracle.png_decode(body)
        assert r == 0 and px == want(x, y, w, h), name
        assert (meta["w"], meta["h"], meta["depth"]) == (w, h, 16)
    for name, (x, y, w, h) in (("tif_0", (0, 0, 512, 512)), ("tif_hi", (1000, 31000, 700, 300))):
        st, body, _, _ = tiles[name]
        tile = np.frombuffer(want(x, y, w, h), np.uint8)
        assert st == 0 and body == oracle.tiff_encode(tile, oracle.UINT16, w, h)[1], name
    # the reference's answers for what it cannot serve
    assert tiles["not_resident"][0] == 460 and tiles["not_resident"][1] is None
    for name in ("outside", "jpg", "jpg_cold", "overflow"):
        assert tiles[name][0] == 404 and tiles[name][1] is None, name
    # registerZarr: the c-blosc 1.21 chunk decoded on the GPU equals the fixture's raw bytes
    raw = open(os.path.join(ROOT, "tests", "golden", "zarr", ZARR + ".raw"), "rb").read()
    st, body, ow, oh = tiles["zarr_raw"]
    assert st == 0 and body == raw and (ow, oh) == (77, 100)
    st, body, _, _ = tiles["zarr_png"]
    sub = np.frombuffer(raw, ">u2").reshape(100, 77)[5:, 3:]
    r, px, _ = oracle.png_decode(body)
    assert st == 0 and r == 0 and px == sub.astype(">u2").tobytes()
    # an injected device failure: RuntimeException (500); the next request is served
    assert tiles["failed"][0] == 500 and tiles["failed"][1] is None
    assert "EXC failed java/lang/RuntimeException" in out.stdout
    st, body, _, _ = tiles["after_failure"]
    r, px, _ = oracle.png_decode(body)
    assert st == 0 and r == 0 and px == want(512, 512, 512, 512)
    # a stalled batch: RuntimeException (500) at the 3 s deadline; released, the next is served
    assert tiles["stalled"][0] == 500 and tiles["stalled"][1] is None
    assert "EXC stalled java/lang/RuntimeException" in out.stdout
    stall_ms = int(out.stdout.split("STALL_MS ")[1].split()[0])
    assert 3000 <= stall_ms < 5000, stall_ms
    st, body, _, _ = tiles["after_stall"]
    r, px, _ = oracle.png_decode(body)
    assert st == 0 and r == 0 and px == want(1024, 1024, 512, 512)
    # the node: misses name the context owning the rows, the bands loaded there serve them
    assert tiles["node_a_miss"][0] == 460 and served_by["node_a_miss"] == 0
    assert tiles["node_b_miss"][0] == 460 and served_by["node_b_miss"] == 1
    # straddles the two owners' rows: routed to the owner of its first row, which loads the
    # other owner's band as a guest band and serves it
    assert tiles["node_c_miss"][0] == 460 and served_by["node_c_miss"] == 0
    st, body, _, _ = tiles["node_c"]
    tile = np.frombuffer(want(4000, 3900, 512, 512), np.uint8)
    assert st == 0 and served_by["node_c"] == 0 and body == oracle.tiff_encode(tile, oracle.UINT16, 512, 512)[1]
    st, body, _, _ = tiles["node_a"]
    assert st == 0 and served_by["node_a"] == 0 and body == want(512, 1000, 512, 512)
    st, body, _, _ = tiles["node_b"]
    r, px, _ = oracle.png_decode(body)
    assert st == 0 and served_by["node_b"] == 1 and r == 0 and px == want(2048, 6000, 512, 512)
    assert "BANDS1 00000220" in out.stdout  # context 1 holds bands 5 and 6 of the slide only
