"""Host logic and the C-ABI surface, on the CPU (no compute calls without a GPU)."""
import ctypes
import json
import os
import re

import pytest

import pbx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(ROOT, "include", "pbx.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pbx_[a-z_0-9]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    L = pbx.lib()
    declared = header_functions()
    assert declared == sorted(pbx.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name


def test_abi_struct_sizes_match_bindings():
    sizes = (ctypes.c_uint64 * 8)()
    assert pbx.lib().pbx_abi_sizes(sizes, 8) == 8
    assert list(sizes) == [ctypes.sizeof(t) for t in (pbx.PbxConfig, pbx.PbxPlaneDesc,
                                                      pbx.PbxTileReq, pbx.PbxResult,
                                                      pbx.PbxBatchStats, pbx.PbxImageDesc,
                                                      pbx.PbxResidencyStats, pbx.PbxSpans)]


def test_jni_shim_matches_abi():
    """jni/: every native method of PbxNative.java has its JNI function in pbx_jni.c, and
    every pbx_* call there is a symbol libpbx.so exports (no JDK here to compile it)."""
    java = open(os.path.join(ROOT, "jni", "PbxNative.java")).read()
    c = open(os.path.join(ROOT, "jni", "pbx_jni.c")).read()
    natives = set(re.findall(r"static native \S+ (\w+)\(", java))
    assert natives >= {"init", "shutdown", "registerPlane", "registerZarr", "getTile"}
    defined = set(re.findall(r"Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_(\w+)\(", c))
    assert natives == defined
    body = re.sub(r"/\*.*?\*/", "", c, flags=re.S)
    called = set(re.findall(r"\b(pbx_[a-z_0-9]+)\s*\(", body))
    assert called and called <= set(header_functions())


def test_enums_and_names():
    L = pbx.lib()
    assert L.pbx_abi_version() == 9
    assert L.pbx_format_from_string(None) == pbx.FMT_RAW
    assert L.pbx_format_from_string(b"png") == pbx.FMT_PNG
    assert L.pbx_format_from_string(b"tif") == pbx.FMT_TIF
    for bad in (b"PNG", b"tiff", b"jpg", b""):
        assert L.pbx_format_from_string(bad) == pbx.FMT_UNKNOWN
    for i, n in enumerate(pbx.PIXEL_TYPES):
        assert L.pbx_pixel_type_from_string(n.encode()) == i
        assert L.pbx_bytes_per_pixel(i) == pbx.BYTES_PER_PIXEL[i]
    assert L.pbx_pixel_type_from_string(b"bit") == -1


def test_content_type_matches_reference(oracle):
    for f in (None, "png", "tif", "jpg", "bin"):
        assert pbx.content_type(f) == oracle.content_type(f)


def test_filename_header(oracle):
    """PixelBufferVerticle.java:118-126, with the post-defaulting region."""
    ctx = pbx.TileCtx(123, 1, 2, 3, 0, 512, 256, 128, format="png")
    assert pbx.tile_filename(ctx) == "image123_z1_c2_t3_x0_y512_w256_h128.png"
    ctx = pbx.TileCtx(9, 0, 0, 0)
    assert pbx.tile_filename(ctx) == "image9_z0_c0_t0_x0_y0_w0_h0.bin"
    assert pbx.tile_filename(ctx) == oracle.tile_filename(9, 0, 0, 0, 0, 0, 0, 0, None)


def test_tilectx_from_params_java_semantics():
    """TileCtx(MultiMap, key) (TileCtx.java:67-90); bad numbers -> NumberFormatException."""
    c = pbx.TileCtx.from_params({"imageId": "5", "z": "1", "c": "0", "t": "2", "x": "10",
                                 "w": "256", "format": "png"}, "sess")
    assert (c.imageId, c.z, c.c, c.t, c.x, c.y, c.w, c.h) == (5, 1, 0, 2, 10, 0, 256, 0)
    assert c.resolution is None and c.format == "png" and c.omeroSessionKey == "sess"
    c = pbx.TileCtx.from_params({"imageId": "+7", "z": "-0", "c": "0", "t": "0",
                                 "resolution": "2"})
    assert c.imageId == 7 and c.resolution == 2 and c.format is None
    bad = [{"z": "0", "c": "0", "t": "0"},                                   # no imageId
           {"imageId": "1", "c": "0", "t": "0"},                             # no z
           {"imageId": "x", "z": "0", "c": "0", "t": "0"},
           {"imageId": "1", "z": "0.5", "c": "0", "t": "0"},
           {"imageId": "1", "z": " 1", "c": "0", "t": "0"},
           {"imageId": "1", "z": "2147483648", "c": "0", "t": "0"},           # int overflow
           {"imageId": "9223372036854775808", "z": "0", "c": "0", "t": "0"},  # long overflow
           {"imageId": "1", "z": "0", "c": "0", "t": "0", "w": ""}]
    for p in bad:
        with pytest.raises(ValueError):
            pbx.TileCtx.from_params(p)


def test_tilectx_json_roundtrip():
    c = pbx.TileCtx(5, 1, 2, 3, 4, 5, 6, 7, resolution=1, format="tif", omero_session_key="k")
    d = json.loads(c.to_json())
    assert d["region"] == {"x": 4, "y": 5, "width": 6, "height": 7}
    c2 = pbx.TileCtx.from_json(c.to_json())
    assert (c2.imageId, c2.z, c2.c, c2.t, c2.region, c2.resolution, c2.format) == \
        (5, 1, 2, 3, c.region, 1, "tif")


def test_event_bus_bad_json_is_400():
    """PixelBufferVerticle.java:91-100: an undecodable TileCtx fails with 400."""
    for body in ("{not json", "[]", json.dumps({"imageId": "x", "z": 0, "c": 0, "t": 0})):
        st, msg, hdr = pbx.handle_get_tile(None, body)
        assert st == 400 and msg == b"Illegal tile context"


def test_init_without_gpu_fails_loudly():
    """No CPU fallback: with no HIP device, init reports 500 and says why."""
    if pbx.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(pbx.PbxError) as e:
        pbx.PixelsService()
    assert e.value.status == pbx.E_INTERNAL and "no HIP device" in str(e.value)


def test_shard_of_is_deterministic_and_balanced():
    ctxs = [pbx.TileCtx(1, 0, c, 0, (i % 64) * 512, (i // 64) * 512, 512, 512)
            for c in range(2) for i in range(4096)]
    for world in (1, 2, 4, 8):
        counts = [0] * world
        for c in ctxs:
            r = pbx.shard_of(c, world)
            assert 0 <= r < world and r == pbx.shard_of(c, world)
            counts[r] += 1
        assert max(counts) - min(counts) < 0.1 * len(ctxs) / world + 16
    # band split covers every tile row once
    for world in (1, 3, 8):
        bands = [pbx.band_rows(196, world, r) for r in range(world)]
        assert bands[0][0] == 0 and bands[-1][1] == 196
        assert all(bands[i][1] == bands[i + 1][0] for i in range(world - 1))
