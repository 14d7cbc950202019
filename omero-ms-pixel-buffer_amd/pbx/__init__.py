"""pbx — Python host side of the MI355X /tile pipeline, mirroring the reference's interface.

The reference (glencoesoftware/omero-ms-pixel-buffer, Java) exposes the hot path as
``TileRequestHandler(pixelsService, tileCtx).getTile(client) -> byte[] | null``
(src/main/java/com/glencoesoftware/omero/ms/pixelbuffer/TileRequestHandler.java:74-139),
with the request parsed into a ``TileCtx`` (TileCtx.java:30-92) and replies built by
``PixelBufferVerticle.getTile`` (PixelBufferVerticle.java:90-147).  This module keeps the
same names, argument meanings and error behaviour:

* ``TileCtx.from_params`` raises ``ValueError`` for unparsable numbers (Java
  ``NumberFormatException`` -> HTTP 400, PixelBufferMicroserviceVerticle.java:344-348);
* ``TileRequestHandler.get_tile`` returns ``None`` for every failure the reference maps
  to ``null`` (unknown image, bad region, unsupported type/format: 404), and opens planes
  the GPU does not hold yet from a ``PixelSource`` (getPixels + getPixelBuffer);
* ``handle_get_tile`` reproduces the event-bus consumer: status, body and the
  ``filename`` header.

All compute runs in ``lib/libpbx.so`` (hand-written HIP kernels for gfx950) through the
plain C-ABI in include/pbx.h.  There is no CPU fallback: loading fails loudly if the
library is missing, and ``PixelsService`` raises if no HIP device is present.
"""
from __future__ import annotations

import ctypes
import json
import os
import time
from typing import Dict, Iterable, List, Mapping, Optional, Sequence, Tuple

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PBX_LIB") or os.path.join(os.path.dirname(_PKG_DIR), "lib", "libpbx.so")

# enum pbx_status — the HTTP status the reference ends with; E_NOT_RESIDENT (never sent to a
# client) = the context does not hold the plane: load it and retry (TileRequestHandler below)
OK, E_BADARG, E_NOTFOUND, E_INTERNAL, E_PENDING = 0, 400, 404, 500, 504
E_EXISTS, E_NOT_RESIDENT, E_NO_SPACE = 409, 460, 507
# plane states (pbx_plane_lookup); band states of sparse planes (pbx_plane_band_info)
PS_FILLING, PS_READY, PS_EVICTED = 0, 1, 2
BS_ABSENT, BS_LOADING, BS_READY = 0, 1, 2
# enum pbx_pixel_type (OMERO PixelType names)
PIXEL_TYPES = ["int8", "uint8", "int16", "uint16", "int32", "uint32", "float", "double"]
INT8, UINT8, INT16, UINT16, INT32, UINT32, FLOAT, DOUBLE = range(8)
BYTES_PER_PIXEL = [1, 1, 2, 2, 4, 4, 4, 8]
# enum pbx_format
FMT_RAW, FMT_PNG, FMT_TIF, FMT_UNKNOWN = range(4)
# enum pbx_source / byte order / png filter
SRC_HOST, SRC_GEN_FAKE, SRC_GEN_NOISE = range(3)
BIG_ENDIAN, LITTLE_ENDIAN = 0, 1
FILTER_NONE, FILTER_SUB, FILTER_UP, FILTER_AVG, FILTER_PAETH, FILTER_ADAPTIVE = range(6)


class PbxConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("png_filter", ctypes.c_int32),
                ("tiff_deflate", ctypes.c_int32), ("segment_bytes", ctypes.c_int32),
                ("max_batch_bytes", ctypes.c_uint64), ("coalesce", ctypes.c_int32),
                ("stage_rows", ctypes.c_int32), ("tiff_tile", ctypes.c_int32),
                ("request_timeout_us", ctypes.c_int32)]


class PbxPlaneDesc(ctypes.Structure):
    _fields_ = [("image_id", ctypes.c_int64), ("z", ctypes.c_int32), ("c", ctypes.c_int32),
                ("t", ctypes.c_int32), ("resolution", ctypes.c_int32),
                ("pixel_type", ctypes.c_int32), ("size_x", ctypes.c_int32),
                ("size_y", ctypes.c_int32), ("byte_order", ctypes.c_int32),
                ("source", ctypes.c_int32), ("host_data", ctypes.c_void_p),
                ("host_bytes", ctypes.c_uint64), ("seed", ctypes.c_uint64),
                ("plane_no", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class PbxImageDesc(ctypes.Structure):
    _fields_ = [("image_id", ctypes.c_int64), ("pixel_type", ctypes.c_int32),
                ("size_x", ctypes.c_int32), ("size_y", ctypes.c_int32), ("size_z", ctypes.c_int32),
                ("size_c", ctypes.c_int32), ("size_t_", ctypes.c_int32), ("levels", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class PbxResidencyStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("budget", "resident_bytes", "planes", "evicted_planes", "evictions", "evicted_bytes",
                 "bands", "band_evictions")]


class PbxZarrChunks(ctypes.Structure):
    _fields_ = [("chunk_x", ctypes.c_int32), ("chunk_y", ctypes.c_int32),
                ("codec", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("data", ctypes.c_void_p), ("offsets", ctypes.c_void_p),
                ("fill_bits", ctypes.c_uint64)]


ZARR_RAW, ZARR_BLOSC, ZARR_ZLIB = 0, 1, 2
ZARR_CODECS = {None: ZARR_RAW, "blosc": ZARR_BLOSC, "zlib": ZARR_ZLIB}
_ZARR_DTYPES = {"i1": INT8, "u1": UINT8, "i2": INT16, "u2": UINT16, "i4": INT32, "u4": UINT32,
                "f4": FLOAT, "f8": DOUBLE}


class PbxTileReq(ctypes.Structure):
    _fields_ = [("image_id", ctypes.c_int64), ("z", ctypes.c_int32), ("c", ctypes.c_int32),
                ("t", ctypes.c_int32), ("resolution", ctypes.c_int32), ("x", ctypes.c_int32),
                ("y", ctypes.c_int32), ("w", ctypes.c_int32), ("h", ctypes.c_int32),
                ("format", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class PbxResult(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("format", ctypes.c_int32), ("w", ctypes.c_int32),
                ("h", ctypes.c_int32), ("data", ctypes.POINTER(ctypes.c_uint8)),
                ("len", ctypes.c_uint64), ("owner", ctypes.c_void_p)]


class PbxBatchStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("tiles", "ok_tiles", "png_tiles", "raw_tiles", "tif_tiles", "in_bytes",
                 "stream_bytes", "out_bytes", "deflate_out_bytes", "segments")] + \
               [(n, ctypes.c_double) for n in
                ("ms_extract", "ms_filter", "ms_deflate", "ms_assemble", "ms_total",
                  "ms_lz77", "ms_huff", "ms_encode")] + \
               [(n, ctypes.c_uint64) for n in ("blocks", "direct_tiles", "direct_bytes")]


class PbxSpans(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in
                ("get_tile_direct_ms", "write_image_ms", "create_metadata_ms", "batch_ms", "d2h_ms")] + \
               [("batch_tiles", ctypes.c_uint64)]


# Every symbol include/pbx.h declares (tests check the library exports all of them).
EXPORTS = [
    "pbx_config_default", "pbx_init", "pbx_shutdown", "pbx_last_error", "pbx_abi_version",
    "pbx_device_count", "pbx_plane_register", "pbx_plane_release", "pbx_plane_read_be",
    "pbx_get_tile", "pbx_get_tiles", "pbx_results_release", "pbx_batch_plan",
    "pbx_batch_launch", "pbx_batch_sync", "pbx_batch_fetch", "pbx_batch_destroy",
    "pbx_batch_stats_get", "pbx_tile_filename", "pbx_content_type", "pbx_format_from_string",
    "pbx_pixel_type_from_string", "pbx_bytes_per_pixel", "pbx_device_synchronize",
    "pbx_abi_sizes", "pbx_shard_of", "pbx_test_huffman", "pbx_ctx_stats_get",
    "pbx_test_batch_lz77", "pbx_submit", "pbx_wait", "pbx_plane_build_pyramid",
    "pbx_plane_register_zarr", "pbx_planes_register_zarr", "pbx_release_cached",
    "pbx_set_kernel_streams", "pbx_image_declare", "pbx_image_release", "pbx_plane_create",
    "pbx_plane_write_rows", "pbx_plane_commit", "pbx_plane_lookup", "pbx_set_residency_budget",
    "pbx_residency_stats_get", "pbx_test_fail_batch", "pbx_node_init", "pbx_node_shutdown",
    "pbx_node_size", "pbx_node_context", "pbx_node_route", "pbx_node_get_tile",
    "pbx_plane_create_sparse", "pbx_band_write", "pbx_plane_band_info", "pbx_result_spans",
    "pbx_test_stall_batch", "pbx_band_abort", "pbx_test_fail_band_write",
]

_lib = None


def lib() -> ctypes.CDLL:
    """Load lib/libpbx.so (build it with `make -C omero-ms-pixel-buffer_amd`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"pbx: native library missing at {LIB_PATH}; run "
                           "`python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, u64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64
    L.pbx_last_error.restype = ctypes.c_char_p
    L.pbx_content_type.restype = ctypes.c_char_p
    L.pbx_content_type.argtypes = [ctypes.c_char_p]
    L.pbx_format_from_string.argtypes = [ctypes.c_char_p]
    L.pbx_pixel_type_from_string.argtypes = [ctypes.c_char_p]
    L.pbx_bytes_per_pixel.argtypes = [i32]
    L.pbx_config_default.argtypes = [ctypes.POINTER(PbxConfig)]
    L.pbx_init.argtypes = [ctypes.POINTER(PbxConfig), ctypes.POINTER(vp)]
    L.pbx_shutdown.argtypes = [vp]
    L.pbx_shutdown.restype = None
    L.pbx_device_synchronize.argtypes = [vp]
    L.pbx_set_kernel_streams.argtypes = [vp, i32, i32]
    L.pbx_release_cached.argtypes = [vp]
    L.pbx_plane_register.argtypes = [vp, ctypes.POINTER(PbxPlaneDesc), ctypes.POINTER(u64)]
    L.pbx_plane_release.argtypes = [vp, u64]
    L.pbx_image_declare.argtypes = [vp, ctypes.POINTER(PbxImageDesc)]
    L.pbx_image_release.argtypes = [vp, ctypes.c_int64]
    L.pbx_plane_create.argtypes = [vp, ctypes.POINTER(PbxPlaneDesc), i32, i32, ctypes.POINTER(u64)]
    L.pbx_plane_write_rows.argtypes = [vp, u64, i32, i32, vp, u64]
    L.pbx_plane_commit.argtypes = [vp, u64]
    L.pbx_plane_lookup.argtypes = [vp, ctypes.c_int64, i32, i32, i32, i32, ctypes.POINTER(u64),
                                   ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i32)]
    L.pbx_set_residency_budget.argtypes = [vp, u64]
    L.pbx_residency_stats_get.argtypes = [vp, ctypes.POINTER(PbxResidencyStats)]
    L.pbx_plane_read_be.argtypes = [vp, u64, vp, u64]
    L.pbx_plane_build_pyramid.argtypes = [vp, u64, i32, ctypes.POINTER(u64),
                                          ctypes.POINTER(ctypes.c_double)]
    L.pbx_plane_register_zarr.argtypes = [vp, ctypes.POINTER(PbxPlaneDesc),
                                          ctypes.POINTER(PbxZarrChunks), ctypes.POINTER(u64),
                                          ctypes.POINTER(ctypes.c_double)]
    L.pbx_planes_register_zarr.argtypes = [vp, u64, ctypes.POINTER(PbxPlaneDesc),
                                           ctypes.POINTER(PbxZarrChunks), ctypes.POINTER(u64),
                                           ctypes.POINTER(ctypes.c_double)]
    L.pbx_get_tile.argtypes = [vp, ctypes.POINTER(PbxTileReq), ctypes.POINTER(PbxResult)]
    L.pbx_test_batch_lz77.argtypes = [vp, vp, vp, vp, u64]
    L.pbx_ctx_stats_get.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]
    L.pbx_get_tiles.argtypes = [vp, ctypes.POINTER(PbxTileReq), u64, ctypes.POINTER(PbxResult)]
    L.pbx_submit.argtypes = [vp, ctypes.POINTER(PbxTileReq), u64, ctypes.POINTER(PbxResult),
                             ctypes.POINTER(vp)]
    L.pbx_wait.argtypes = [vp, vp, ctypes.c_int64]
    L.pbx_results_release.argtypes = [vp, ctypes.POINTER(PbxResult), u64]
    L.pbx_results_release.restype = None
    L.pbx_batch_plan.argtypes = [vp, ctypes.POINTER(PbxTileReq), u64, ctypes.POINTER(vp)]
    L.pbx_batch_launch.argtypes = [vp, vp]
    L.pbx_batch_sync.argtypes = [vp, vp]
    L.pbx_batch_fetch.argtypes = [vp, vp, ctypes.POINTER(PbxResult)]
    L.pbx_batch_destroy.argtypes = [vp, vp]
    L.pbx_batch_destroy.restype = None
    L.pbx_batch_stats_get.argtypes = [vp, vp, ctypes.POINTER(PbxBatchStats)]
    L.pbx_tile_filename.argtypes = [ctypes.POINTER(PbxTileReq), i32, i32, ctypes.c_char_p,
                                    ctypes.c_char_p, u64]
    L.pbx_abi_sizes.argtypes = [ctypes.POINTER(u64), ctypes.c_int]
    L.pbx_shard_of.argtypes = [ctypes.POINTER(PbxTileReq), i32, i32, i32]
    L.pbx_test_huffman.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 2 + [ctypes.c_uint32] + \
        [ctypes.c_void_p] * 2
    L.pbx_test_fail_batch.argtypes = [vp, u64]
    L.pbx_test_stall_batch.argtypes = [vp, u64]
    L.pbx_test_fail_band_write.argtypes = [vp, u64]
    L.pbx_plane_create_sparse.argtypes = [vp, ctypes.POINTER(PbxPlaneDesc), i32, i32, i32, ctypes.POINTER(u64)]
    L.pbx_band_write.argtypes = [vp, u64, i32, i32, vp, u64]
    L.pbx_band_abort.argtypes = [vp, u64, i32]
    L.pbx_plane_band_info.argtypes = [vp, u64, ctypes.POINTER(i32), ctypes.POINTER(i32), vp]
    L.pbx_node_init.argtypes = [ctypes.POINTER(PbxConfig), i32, ctypes.POINTER(i32), i32, ctypes.POINTER(vp)]
    L.pbx_node_shutdown.argtypes = [vp]
    L.pbx_node_shutdown.restype = None
    L.pbx_node_size.argtypes = [vp]
    L.pbx_node_context.argtypes = [vp, i32]
    L.pbx_node_context.restype = vp
    L.pbx_node_route.argtypes = [vp, ctypes.POINTER(PbxTileReq), ctypes.POINTER(i32)]
    L.pbx_node_get_tile.argtypes = [vp, ctypes.POINTER(PbxTileReq), ctypes.POINTER(PbxResult),
                                    ctypes.POINTER(i32)]
    L.pbx_result_spans.argtypes = [ctypes.POINTER(PbxResult), ctypes.POINTER(PbxSpans)]
    _lib = L
    return L


class PbxError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"pbx status {status}: {msg}")
        self.status = status


def _check(status: int) -> None:
    if status != OK:
        raise PbxError(status, lib().pbx_last_error().decode(errors="replace"))


def device_count() -> int:
    return lib().pbx_device_count()


# ------------------------------------------------------------------------- TileCtx

def _parse_int(v: str, bits: int) -> int:
    """Java Integer.parseInt / Long.parseLong: optional sign, ASCII digits, in range."""
    if v is None:
        raise ValueError("null")  # parseInt(null) -> NumberFormatException
    s = v[1:] if v[:1] in ("+", "-") else v
    if not s or not s.isascii() or not s.isdigit():
        raise ValueError(f'For input string: "{v}"')
    n = int(v)
    if not -(1 << (bits - 1)) <= n < (1 << (bits - 1)):
        raise ValueError(f'For input string: "{v}"')
    return n


RESOLUTION_NONE = -1  # PBX_RESOLUTION_NONE: TileCtx.resolution == null


def _req_resolution(r: Optional[int]) -> int:
    """TileCtx.resolution -> pbx_tile_req.resolution (OMERO numbering, include/pbx.h): null ->
    PBX_RESOLUTION_NONE; a given negative level (setResolutionLevel throws -> 404) -> -2."""
    if r is None:
        return RESOLUTION_NONE
    return r if r >= 0 else -2


class TileCtx:
    """TileCtx.java:30-92 — the request context and the event-bus JSON payload."""

    def __init__(self, image_id: int, z: int, c: int, t: int, x: int = 0, y: int = 0,
                 w: int = 0, h: int = 0, resolution: Optional[int] = None,
                 format: Optional[str] = None, omero_session_key: Optional[str] = None):
        self.imageId = image_id
        self.z, self.c, self.t = z, c, t
        self.region = {"x": x, "y": y, "width": w, "height": h}
        self.resolution = resolution
        self.format = format
        self.omeroSessionKey = omero_session_key

    @classmethod
    def from_params(cls, params: Mapping[str, str], omero_session_key: Optional[str] = None):
        """TileCtx(MultiMap, String) (TileCtx.java:67-90); ValueError == NumberFormatException."""
        opt = lambda k: _parse_int(params[k], 32) if params.get(k) is not None else None
        return cls(_parse_int(params.get("imageId"), 64), _parse_int(params.get("z"), 32),
                   _parse_int(params.get("c"), 32), _parse_int(params.get("t"), 32),
                   opt("x") or 0, opt("y") or 0, opt("w") or 0, opt("h") or 0,
                   opt("resolution"), params.get("format"), omero_session_key)

    def to_json(self) -> str:
        return json.dumps({"omeroSessionKey": self.omeroSessionKey, "imageId": self.imageId,
                           "z": self.z, "c": self.c, "t": self.t,
                           "resolution": self.resolution, "region": self.region,
                           "format": self.format})

    @classmethod
    def from_json(cls, body: str) -> "TileCtx":
        d = json.loads(body)
        r = d.get("region") or {}
        for k in ("imageId", "z", "c", "t"):
            if not isinstance(d.get(k), int):
                raise ValueError(f"bad {k}")
        return cls(d["imageId"], d["z"], d["c"], d["t"], r.get("x", 0), r.get("y", 0),
                   r.get("width", 0), r.get("height", 0), d.get("resolution"),
                   d.get("format"), d.get("omeroSessionKey"))

    @property
    def x(self): return self.region["x"]

    @property
    def y(self): return self.region["y"]

    @property
    def w(self): return self.region["width"]

    @property
    def h(self): return self.region["height"]

    def to_req(self) -> PbxTileReq:
        return PbxTileReq(self.imageId, self.z, self.c, self.t,
                          _req_resolution(self.resolution),
                          self.x, self.y, self.w, self.h,
                          lib().pbx_format_from_string(
                              self.format.encode() if self.format is not None else None), 0)


def tile_filename(ctx: TileCtx) -> str:
    """PixelBufferVerticle.java:118-126 (uses the region after w/h defaulting)."""
    buf = ctypes.create_string_buffer(512)
    req = ctx.to_req()
    lib().pbx_tile_filename(ctypes.byref(req), ctx.w, ctx.h,
                            ctx.format.encode() if ctx.format is not None else None, buf, 512)
    return buf.value.decode()


def shard_of(ctx: TileCtx, world: int, tile_w: int = 512, tile_h: int = 512) -> int:
    """Rank that serves this request when requests are sharded over `world` GPUs."""
    req = ctx.to_req()
    r = lib().pbx_shard_of(ctypes.byref(req), tile_w, tile_h, world)
    if r < 0:
        _check(E_BADARG)
    return r


def band_rows(n_rows: int, world: int, rank: int) -> Tuple[int, int]:
    """Whole-slide split: contiguous tile-row band [lo, hi) of a rank."""
    return (n_rows * rank) // world, (n_rows * (rank + 1)) // world


def content_type(fmt: Optional[str]) -> str:
    """PixelBufferMicroserviceVerticle.java:373-379."""
    return lib().pbx_content_type(fmt.encode() if fmt is not None else None).decode()


# --------------------------------------------------------------------- PixelsService

def zarr_array_meta(array_dir: str) -> dict:
    """The .zarray of a Zarr v2 array directory, checked for what the GPU decode supports."""
    import json
    with open(os.path.join(array_dir, ".zarray")) as f:
        meta = json.load(f)
    if meta.get("zarr_format") != 2 or meta.get("order", "C") != "C" or meta.get("filters"):
        raise PbxError(400, "only Zarr v2 C-order arrays without filters are supported")
    if meta["dtype"][1:] not in _ZARR_DTYPES:
        raise PbxError(400, "unsupported dtype %s" % meta["dtype"])
    if len(meta["shape"]) < 2 or len(meta["shape"]) > 5 or any(cs != 1 for cs in meta["chunks"][:-2]):
        raise PbxError(400, "need shape [..., y, x] with one plane per chunk")
    return meta


def _lead_axes(ndim: int, axes: Optional[Sequence[str]]) -> List[str]:
    """Names of the leading (non-y/x) axes of an array: the NGFF multiscales "axes" when given
    (0.4: time, then channel, then space), else t, c, z with missing ones dropped from the left."""
    if axes is not None:
        names = [a["name"] if isinstance(a, dict) else a for a in axes]
        if len(names) != ndim or [n.lower() for n in names[-2:]] != ["y", "x"]:
            raise PbxError(400, "axes %r do not end in y, x" % (names,))
        lead = [n.lower() for n in names[:-2]]
        if any(n not in ("t", "c", "z") for n in lead) or len(set(lead)) != len(lead):
            raise PbxError(400, "unsupported axes %r" % (names,))
        return lead
    return ["t", "c", "z"][3 - (ndim - 2):]


def zarr_plane_spec(array_dir: str, image_id: int, z: int, c: int, t: int, level: int = 0,
                    meta: Optional[dict] = None, axes: Optional[Sequence] = None) -> dict:
    """register_zarr_planes() arguments for plane (z, c, t) of an NGFF array directory (axes:
    the multiscales "axes" of the image, else NGFF order t, c, z, y, x with fewer leading axes
    dropped from the left): chunk files named by dimension_separator "." or "/", absent
    files = fill_value.  `level` is the stored pyramid level (0 = full resolution)."""
    import numpy as np
    meta = meta or zarr_array_meta(array_dir)
    shape, chunk, dt = meta["shape"], meta["chunks"], meta["dtype"]
    comp = meta.get("compressor")
    names = _lead_axes(len(shape), axes)
    want = {"t": t, "c": c, "z": z}
    lead = [want[n] for n in names]
    if any(want[n] for n in ("t", "c", "z") if n not in names):
        raise PbxError(404, "plane (z=%d, c=%d, t=%d) outside the array" % (z, c, t))
    for v, n in zip(lead, shape[:-2]):
        if not 0 <= v < n:
            raise PbxError(404, "plane (z=%d, c=%d, t=%d) outside the array" % (z, c, t))
    sep = meta.get("dimension_separator", ".")
    sy, sx, cy, cx = shape[-2], shape[-1], chunk[-2], chunk[-1]
    chunks = []
    for j in range(-(-sy // cy)):
        for i in range(-(-sx // cx)):
            path = os.path.join(array_dir, sep.join(str(v) for v in lead + [j, i]))
            chunks.append(open(path, "rb").read() if os.path.exists(path) else None)
    native = np.dtype(dt).newbyteorder("=")
    fill_bits = int(np.array([meta.get("fill_value") or 0], dtype=native).view("u%d" % native.itemsize)[0])
    return dict(image_id=image_id, z=z, c=c, t=t, level=level,
                pixel_type=_ZARR_DTYPES[dt[1:]], size_x=sx, size_y=sy, chunk_x=cx, chunk_y=cy,
                codec=None if comp is None else comp.get("id"), chunks=chunks,
                big_endian=dt[0] != "<", fill_bits=fill_bits)


def pack_chunks(chunks: Sequence[Optional[bytes]]):
    """Chunk files of one plane as the C-ABI takes them: (uint8 data, uint64 offsets[n+1]),
    the files concatenated in C order over the chunk grid (None / b"" = missing chunk)."""
    import numpy as np
    lens = np.array([len(b) if b else 0 for b in chunks], dtype=np.uint64)
    offsets = np.zeros(len(chunks) + 1, dtype=np.uint64)
    np.cumsum(lens, out=offsets[1:])
    data = np.frombuffer(b"".join(b for b in chunks if b) or b"\0", dtype=np.uint8)
    return data, offsets


def ngff_multiscales(image_dir: str):
    """(multiscales[0], image directory) of an NGFF image (.zattrs, NGFF 0.1-0.4); a
    bioformats2raw container root (attribute "bioformats2raw.layout") resolves to series 0."""
    import json
    with open(os.path.join(image_dir, ".zattrs")) as f:
        attrs = json.load(f)
    if "multiscales" not in attrs and "bioformats2raw.layout" in attrs:
        return ngff_multiscales(os.path.join(image_dir, "0"))
    ms = attrs.get("multiscales")
    if not ms or not ms[0].get("datasets"):
        raise PbxError(400, "no multiscales datasets in %s/.zattrs" % image_dir)
    return ms[0], image_dir


def make_config(device: Optional[int] = None, png_filter: int = FILTER_NONE,
                tiff_deflate: bool = False, coalesce: bool = True, stage_rows: bool = False,
                tiff_tile: Optional[int] = None, request_timeout_us: Optional[int] = None) -> PbxConfig:
    cfg = PbxConfig()
    _check(lib().pbx_config_default(ctypes.byref(cfg)))
    cfg.device = -1 if device is None else device
    cfg.png_filter = png_filter
    cfg.tiff_deflate = 1 if tiff_deflate else 0
    cfg.coalesce = 1 if coalesce else 0
    cfg.stage_rows = 1 if stage_rows else 0
    if tiff_tile is not None:  # else $PBX_TIFF_TILE or 0 (one strip, the reference's)
        cfg.tiff_tile = int(tiff_tile)
    if request_timeout_us is not None:  # else $PBX_REQUEST_TIMEOUT_US or 15 s (the event-bus send timeout)
        cfg.request_timeout_us = int(request_timeout_us)
    return cfg


class PixelsService:
    """Plane registry on one MI355X (the PixelsService / getPixels stand-in).

    Planes live in HBM.  ``register_plane`` takes a numpy array (any byte order) or a
    synthetic generator ("fake" = Bio-Formats FakeReader style, "noise" = G_NOISE).
    """

    def __init__(self, device: Optional[int] = None, png_filter: int = FILTER_NONE,
                 tiff_deflate: bool = False, coalesce: bool = True, stage_rows: bool = False,
                 tiff_tile: Optional[int] = None, sparse_band_rows: int = 0,
                 request_timeout_us: Optional[int] = None, _handle=None):
        """sparse_band_rows > 0: planes the handler opens on demand are sparse planes of bands
        of that many rows (region-proportional residency); 0: whole planes (or the handler's
        row band)."""
        import threading
        self.sparse_band_rows = int(sparse_band_rows)
        self._load_lock = threading.Lock()  # one loader per plane key / band
        self._loading: Dict[tuple, list] = {}  # key -> [lock, users]; removed with its last user
        self._owned = _handle is None
        if _handle is not None:  # a context owned by a PixelsNode
            self._h = ctypes.c_void_p(_handle)
            return
        L = lib()
        cfg = make_config(device, png_filter, tiff_deflate, coalesce, stage_rows, tiff_tile,
                          request_timeout_us)
        h = ctypes.c_void_p()
        _check(L.pbx_init(ctypes.byref(cfg), ctypes.byref(h)))
        self._h = h

    def close(self) -> None:
        if self._h and self._owned:
            lib().pbx_shutdown(self._h)
        self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def register_plane(self, image_id: int, z: int, c: int, t: int, pixel_type: int,
                       size_x: int, size_y: int, data=None, generator: Optional[str] = None,
                       seed: int = 0, plane_no: int = 0, level: int = 0,
                       big_endian: Optional[bool] = None) -> int:
        """``level`` is the STORED pyramid level (0 = full resolution, the NGFF dataset
        index); requests name levels in OMERO's numbering (TileCtx.resolution, levels-1 =
        full resolution)."""
        d = PbxPlaneDesc()
        d.image_id, d.z, d.c, d.t, d.resolution = image_id, z, c, t, level
        d.pixel_type, d.size_x, d.size_y = pixel_type, size_x, size_y
        keep = None
        if generator is not None:
            d.source = {"fake": SRC_GEN_FAKE, "noise": SRC_GEN_NOISE}[generator]
            d.seed, d.plane_no = seed, plane_no
        else:
            import numpy as np
            a = np.ascontiguousarray(data)
            if big_endian is None:
                big_endian = a.dtype.byteorder == ">" or (
                    a.dtype.byteorder == "=" and os.sys.byteorder == "big")
            keep = a.view(np.uint8).reshape(-1)
            d.source = SRC_HOST
            d.byte_order = BIG_ENDIAN if big_endian else LITTLE_ENDIAN
            d.host_data = keep.ctypes.data
            d.host_bytes = keep.nbytes
        pid = ctypes.c_uint64()
        _check(lib().pbx_plane_register(self._h, ctypes.byref(d), ctypes.byref(pid)))
        del keep
        return pid.value

    def register_zarr_plane(self, image_id: int, z: int, c: int, t: int, pixel_type: int,
                            size_x: int, size_y: int, chunk_x: int, chunk_y: int,
                            codec: Optional[str], chunks: Sequence[Optional[bytes]],
                            big_endian: bool = True, fill_bits: int = 0, level: int = 0,
                            timing: bool = False):
        """Register a plane from its Zarr v2 chunks (C order over the chunk grid; None or
        b"" = missing chunk -> fill; or pack_chunks()' (data, offsets) pair), decoded on the GPU
        (pbx_plane_register_zarr).  codec is
        the .zarray compressor id: None, "blosc" or "zlib".  Returns the plane id (and the
        decode / placement kernels' device ms with timing=True)."""
        if codec not in ZARR_CODECS:
            raise PbxError(400, "unsupported Zarr compressor %r" % (codec,))
        data, offsets = chunks if isinstance(chunks, tuple) else pack_chunks(chunks)
        d = PbxPlaneDesc()
        d.image_id, d.z, d.c, d.t, d.resolution = image_id, z, c, t, level
        d.pixel_type, d.size_x, d.size_y = pixel_type, size_x, size_y
        d.byte_order = BIG_ENDIAN if big_endian else LITTLE_ENDIAN
        zc = PbxZarrChunks()
        zc.chunk_x, zc.chunk_y, zc.codec = chunk_x, chunk_y, ZARR_CODECS[codec]
        zc.data, zc.offsets, zc.fill_bits = data.ctypes.data, offsets.ctypes.data, fill_bits
        pid = ctypes.c_uint64()
        ms = (ctypes.c_double * 2)()
        _check(lib().pbx_plane_register_zarr(self._h, ctypes.byref(d), ctypes.byref(zc),
                                             ctypes.byref(pid), ms))
        return (pid.value, (ms[0], ms[1])) if timing else pid.value

    def register_zarr_planes(self, planes: Sequence[dict], timing: bool = False):
        """Several Zarr planes decoded by one set of GPU launches (pbx_planes_register_zarr):
        each dict holds register_zarr_plane's arguments (image_id, z, c, t, pixel_type,
        size_x, size_y, chunk_x, chunk_y, codec, chunks[, big_endian, fill_bits,
        level]).  All are registered or none.  Returns the plane ids (and the kernels'
        device ms with timing=True)."""
        import numpy as np
        n = len(planes)
        descs = (PbxPlaneDesc * n)()
        zcs = (PbxZarrChunks * n)()
        keep = []
        for k, p in enumerate(planes):
            if p["codec"] not in ZARR_CODECS:
                raise PbxError(400, "unsupported Zarr compressor %r" % (p["codec"],))
            chunks = p["chunks"]
            data, offsets = chunks if isinstance(chunks, tuple) else pack_chunks(chunks)
            keep += [offsets, data]
            d = descs[k]
            d.image_id, d.z, d.c, d.t = p["image_id"], p["z"], p["c"], p["t"]
            d.resolution = p.get("level", 0)
            d.pixel_type, d.size_x, d.size_y = p["pixel_type"], p["size_x"], p["size_y"]
            d.byte_order = BIG_ENDIAN if p.get("big_endian", True) else LITTLE_ENDIAN
            zc = zcs[k]
            zc.chunk_x, zc.chunk_y, zc.codec = p["chunk_x"], p["chunk_y"], ZARR_CODECS[p["codec"]]
            zc.data, zc.offsets, zc.fill_bits = data.ctypes.data, offsets.ctypes.data, p.get("fill_bits", 0)
        ids = (ctypes.c_uint64 * n)()
        ms = (ctypes.c_double * 2)()
        _check(lib().pbx_planes_register_zarr(self._h, n, descs, zcs, ids, ms))
        del keep
        return (list(ids), (ms[0], ms[1])) if timing else list(ids)

    def register_zarr_array(self, array_dir: str, image_id: int, z: int, c: int, t: int,
                            level: int = 0) -> int:
        """One (t, c, z) plane of an NGFF multiscale dataset (a Zarr v2 array directory with
        shape [..., y, x], NGFF order t, c, z, y, x) — what ZarrPixelBuffer reads through
        JZarr (omero-zarr-pixel-buffer 0.6.1, build.gradle:57).  Chunks of the plane are read
        from disk here and decoded on the GPU."""
        sp = zarr_plane_spec(array_dir, image_id, z, c, t, level)
        return self.register_zarr_planes([sp])[0]

    @staticmethod
    def _array_planes(meta: dict, axes) -> List[Tuple[int, int, int]]:
        names = _lead_axes(len(meta["shape"]), axes)
        ext = {"t": 1, "c": 1, "z": 1}
        ext.update(dict(zip(names, meta["shape"][:-2])))
        return [(z, c, t) for t in range(ext["t"]) for c in range(ext["c"]) for z in range(ext["z"])]

    def register_zarr_array_planes(self, array_dir: str, image_id: int,
                                   planes: Optional[Sequence[Tuple[int, int, int]]] = None,
                                   level: int = 0, axes=None) -> Dict[Tuple[int, int, int], int]:
        """Every (z, c, t) plane of an NGFF array (or the given ones) decoded by ONE set of GPU
        launches (pbx_planes_register_zarr).  Returns {(z, c, t): plane id}."""
        meta = zarr_array_meta(array_dir)
        if planes is None:
            planes = self._array_planes(meta, axes)
        specs = [zarr_plane_spec(array_dir, image_id, z, c, t, level, meta, axes) for z, c, t in planes]
        ids = self.register_zarr_planes(specs)
        return dict(zip([tuple(p) for p in planes], ids))

    def register_ngff_image(self, image_dir: str, image_id: int,
                            planes: Optional[Sequence[Tuple[int, int, int]]] = None
                            ) -> Dict[int, Dict[Tuple[int, int, int], int]]:
        """A whole NGFF multiscale image -- what ZarrPixelsService opens for an image
        (omero-zarr-pixel-buffer 0.6.1, build.gradle:57; PixelBufferVerticle.java:29,56) -- in
        ONE set of GPU launches: .zattrs "multiscales"[0] lists the datasets from full
        resolution down; dataset k becomes stored level k of every (z, c, t) plane (or of the
        given ones).  A bioformats2raw container (root .zattrs with "bioformats2raw.layout")
        is opened at its series 0.  Requests then select levels with OMERO's numbering:
        TileCtx.resolution = levels - 1 - k (TileRequestHandler.java:89-91).  All levels are
        registered, or none.  Returns {level: {(z, c, t): plane id}}."""
        ms, root = ngff_multiscales(image_dir)
        axes = ms.get("axes")
        specs, keys = [], []
        for k, ds in enumerate(ms["datasets"]):
            adir = os.path.join(root, ds["path"])
            meta = zarr_array_meta(adir)
            for z, c, t in (planes if planes is not None else self._array_planes(meta, axes)):
                specs.append(zarr_plane_spec(adir, image_id, z, c, t, k, meta, axes))
                keys.append((k, (z, c, t)))
        ids = self.register_zarr_planes(specs)
        out: Dict[int, Dict[Tuple[int, int, int], int]] = {}
        for (k, p), pid in zip(keys, ids):
            out.setdefault(k, {})[p] = pid
        return out

    def release_plane(self, plane_id: int) -> None:
        _check(lib().pbx_plane_release(self._h, plane_id))

    # ---------------------------------------------------------------- plane residency
    def declare_image(self, pixels: "Pixels") -> None:
        """pbx_image_declare: the Pixels row (getPixels, TileRequestHandler.java:220-241) and
        the PixelBuffer's resolution level count, so that z/c/t/resolution outside the image
        answer the reference's 404 without loading anything."""
        d = PbxImageDesc(pixels.image_id, pixels.pixel_type, pixels.size_x, pixels.size_y,
                         pixels.size_z, pixels.size_c, pixels.size_t, pixels.levels, 0)
        _check(lib().pbx_image_declare(self._h, ctypes.byref(d)))

    def release_image(self, image_id: int) -> None:
        _check(lib().pbx_image_release(self._h, image_id))

    def create_plane(self, image_id: int, z: int, c: int, t: int, pixel_type: int, size_x: int,
                     size_y: int, level: int = 0, band: Optional[Tuple[int, int]] = None,
                     big_endian: bool = True, generator: Optional[str] = None, seed: int = 0,
                     plane_no: int = 0) -> int:
        """pbx_plane_create: allocate a plane, or only the row band (y0, rows) of it.  Host
        planes are filled with write_rows() and published by commit_plane(); generator
        planes are generated on the GPU and ready at once."""
        d = PbxPlaneDesc()
        d.image_id, d.z, d.c, d.t, d.resolution = image_id, z, c, t, level
        d.pixel_type, d.size_x, d.size_y = pixel_type, size_x, size_y
        d.byte_order = BIG_ENDIAN if big_endian else LITTLE_ENDIAN
        if generator is not None:
            d.source = {"fake": SRC_GEN_FAKE, "noise": SRC_GEN_NOISE}[generator]
            d.seed, d.plane_no = seed, plane_no
        y0, rows = band if band is not None else (0, 0)
        pid = ctypes.c_uint64()
        _check(lib().pbx_plane_create(self._h, ctypes.byref(d), y0, rows, ctypes.byref(pid)))
        return pid.value

    def write_rows(self, plane_id: int, y0: int, data) -> None:
        """pbx_plane_write_rows: packed rows (bytes or an array of rows x size_x samples, in
        the byte order given to create_plane) starting at plane row y0."""
        import numpy as np
        a = np.ascontiguousarray(data) if not isinstance(data, (bytes, bytearray, memoryview)) else \
            np.frombuffer(data, np.uint8)
        buf = a.view(np.uint8).reshape(-1)
        rows = a.shape[0] if a.ndim >= 2 else None
        if rows is None:
            raise ValueError("write_rows: pass a 2-D array of rows (or use write_rows_bytes)")
        _check(lib().pbx_plane_write_rows(self._h, plane_id, y0, rows, buf.ctypes.data, buf.nbytes))

    def write_rows_bytes(self, plane_id: int, y0: int, rows: int, data: bytes) -> None:
        buf = ctypes.create_string_buffer(bytes(data), len(data)) if not isinstance(data, bytes) else data
        _check(lib().pbx_plane_write_rows(self._h, plane_id, y0, rows, buf, len(data)))

    def commit_plane(self, plane_id: int) -> None:
        _check(lib().pbx_plane_commit(self._h, plane_id))

    def lookup_plane(self, image_id: int, z: int, c: int, t: int, level: int = 0):
        """(plane id, state, band_y0, band_rows) of the plane registered under a key, or None."""
        pid, st, y0, n = ctypes.c_uint64(), ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        r = lib().pbx_plane_lookup(self._h, image_id, z, c, t, level, ctypes.byref(pid),
                                   ctypes.byref(st), ctypes.byref(y0), ctypes.byref(n))
        if r == E_NOTFOUND:
            return None
        _check(r)
        return pid.value, st.value, y0.value, n.value

    def set_residency_budget(self, nbytes: int) -> None:
        """pbx_set_residency_budget: HBM for planes (0 = none); idle planes are evicted LRU."""
        _check(lib().pbx_set_residency_budget(self._h, nbytes))

    def residency_stats(self) -> Dict[str, int]:
        s = PbxResidencyStats()
        _check(lib().pbx_residency_stats_get(self._h, ctypes.byref(s)))
        return {n: getattr(s, n) for n, _ in PbxResidencyStats._fields_}

    # ------------------------------------------------------------- sparse (banded) planes
    def create_sparse_plane(self, image_id: int, z: int, c: int, t: int, pixel_type: int, size_x: int,
                            size_y: int, band_rows: int, level: int = 0,
                            own: Optional[Tuple[int, int]] = None, big_endian: bool = True,
                            generator: Optional[str] = None, seed: int = 0, plane_no: int = 0) -> int:
        """pbx_plane_create_sparse: a plane held as bands of `band_rows` rows, each loaded on
        demand (band_write) and evicted on its own; `own` = (y0, rows) limits the rows this
        context may hold (another context owns the rest)."""
        d = PbxPlaneDesc()
        d.image_id, d.z, d.c, d.t, d.resolution = image_id, z, c, t, level
        d.pixel_type, d.size_x, d.size_y = pixel_type, size_x, size_y
        d.byte_order = BIG_ENDIAN if big_endian else LITTLE_ENDIAN
        if generator is not None:
            d.source = {"fake": SRC_GEN_FAKE, "noise": SRC_GEN_NOISE}[generator]
            d.seed, d.plane_no = seed, plane_no
        y0, rows = own if own is not None else (0, 0)
        pid = ctypes.c_uint64()
        _check(lib().pbx_plane_create_sparse(self._h, ctypes.byref(d), band_rows, y0, rows, ctypes.byref(pid)))
        return pid.value

    def band_write(self, plane_id: int, y0: int, rows: int, data: Optional[bytes]) -> None:
        """pbx_band_write: rows [y0, y0 + rows) of one band (packed, the plane's byte order);
        data None generates them (generator planes)."""
        if data is None:
            _check(lib().pbx_band_write(self._h, plane_id, y0, rows, None, 0))
        else:
            _check(lib().pbx_band_write(self._h, plane_id, y0, rows, data, len(data)))

    def band_abort(self, plane_id: int, y0: int) -> None:
        """pbx_band_abort: give back the band holding row y0 when its load is abandoned."""
        _check(lib().pbx_band_abort(self._h, plane_id, y0))

    def band_info(self, plane_id: int) -> Tuple[int, List[int]]:
        """(band_rows, [state of band k]) of a sparse plane (BS_ABSENT / BS_LOADING / BS_READY)."""
        br, nb = ctypes.c_int32(), ctypes.c_int32()
        _check(lib().pbx_plane_band_info(self._h, plane_id, ctypes.byref(br), ctypes.byref(nb), None))
        st = (ctypes.c_uint8 * max(nb.value, 1))()
        _check(lib().pbx_plane_band_info(self._h, plane_id, ctypes.byref(br), ctypes.byref(nb), st))
        return br.value, list(st)[:nb.value]

    def test_fail_batch(self, ahead: int) -> None:
        """Fault injection: the `ahead`-th batch launched from now on fails (500s); 0 = off."""
        _check(lib().pbx_test_fail_batch(self._h, ahead))

    def test_fail_band_write(self, ahead: int) -> None:
        """Upload failure injection: the `ahead`-th band write from now on fails; 0 = off."""
        _check(lib().pbx_test_fail_band_write(self._h, ahead))

    def test_stall_batch(self, ahead: int) -> None:
        """Stall injection: the `ahead`-th batch launched from now on does not complete until
        test_stall_batch(0) releases it (its callers get 500 at their deadline)."""
        _check(lib().pbx_test_stall_batch(self._h, ahead))

    # ------------------------------------------------------------- opening planes on demand
    def _exclusive(self, key):
        """Context manager: one loader per key (plane, or (plane, band)); the lock entry goes
        with its last user."""
        import contextlib
        import threading

        @contextlib.contextmanager
        def cm():
            with self._load_lock:
                ent = self._loading.get(key)
                if ent is None:
                    ent = self._loading[key] = [threading.Lock(), 0]
                ent[1] += 1
            try:
                with ent[0]:
                    yield
            finally:
                with self._load_lock:
                    ent[1] -= 1
                    if ent[1] == 0:
                        del self._loading[key]
        return cm()

    def load_plane(self, source: "PixelSource", pixels: "Pixels", z: int, c: int, t: int,
                   level: int = 0, band: Optional[Tuple[int, int]] = None,
                   band_bytes: int = 64 << 20, timeout_s: float = 60.0) -> int:
        """Open a plane this context does not hold, as getPixelBuffer + getTileDirect would
        (TileRequestHandler.java:86,107-109,201-211): declare the image, create the plane (or
        only `band` = (y0, rows) of it), stream its rows from `source` in bands of about
        `band_bytes`, commit.  If another caller is loading the same key, wait for it."""
        self.declare_image(pixels)
        key = (pixels.image_id, z, c, t, level)
        with self._exclusive(key):
            found = self.lookup_plane(*key)
            if found is not None and found[1] == PS_READY:
                return found[0]
            sx, sy = source.level_size(pixels, level)
            y0, rows = band if band is not None else (0, sy)
            try:
                pid = self.create_plane(pixels.image_id, z, c, t, pixels.pixel_type, sx, sy, level,
                                        band=(y0, rows), big_endian=True)
            except PbxError as e:
                if e.status != E_EXISTS:
                    raise
                deadline = time.monotonic() + timeout_s  # another context user loads it
                while time.monotonic() < deadline:
                    found = self.lookup_plane(*key)
                    if found is None or found[1] != PS_FILLING:
                        return found[0] if found is not None else 0
                    time.sleep(0.001)
                raise
            step = max(1, band_bytes // max(1, sx * BYTES_PER_PIXEL[pixels.pixel_type]))
            try:
                for r in range(y0, y0 + rows, step):
                    n = min(step, y0 + rows - r)
                    self.write_rows_bytes(pid, r, n, source.read_rows(pixels, z, c, t, level, r, n))
                self.commit_plane(pid)
            except BaseException:
                self.release_plane(pid)
                raise
            return pid

    def load_bands(self, source: "PixelSource", pixels: "Pixels", z: int, c: int, t: int, level: int,
                   y: int, h: int, own: Optional[Tuple[int, int]] = None,
                   timeout_s: float = 60.0) -> int:
        """Region-proportional loading (TileRequestHandler.java:102-109 reads only the region):
        the sparse plane of the key (created if absent, bands of self.sparse_band_rows rows) gets
        the bands that rows [y, y + h) cover, each read from `source` once; bands another
        caller is loading are waited for.  Returns the plane id."""
        self.declare_image(pixels)
        key = (pixels.image_id, z, c, t, level)
        sx, sy = source.level_size(pixels, level)
        with self._exclusive(key):
            found = self.lookup_plane(*key)
            if found is None or found[1] == PS_EVICTED:
                try:
                    pid = self.create_sparse_plane(pixels.image_id, z, c, t, pixels.pixel_type, sx, sy,
                                                   self.sparse_band_rows, level, own=own)
                except PbxError as e:
                    if e.status != E_EXISTS:
                        raise
                    pid = self.lookup_plane(*key)[0]
            else:
                pid = found[0]
        B, states = self.band_info(pid)
        # every band the rows cover: the owned ones, and the guest bands past the owned rows that
        # a region starting in them covers (the reference's getTileDirect serves any region)
        y0, y1 = max(y, 0), min(y + h, sy)
        for k in range(y0 // B, (y1 + B - 1) // B) if y1 > y0 else ():
            if states[k] == BS_READY:
                continue
            with self._exclusive(key + (k,)):
                deadline = time.monotonic() + timeout_s
                while True:
                    st = self.band_info(pid)[1][k]
                    if st == BS_READY:
                        break
                    if st == BS_ABSENT:
                        r0, r1 = k * B, min((k + 1) * B, sy)
                        try:
                            self.band_write(pid, r0, r1 - r0,
                                            source.read_rows(pixels, z, c, t, level, r0, r1 - r0))
                            break
                        except PbxError as e:
                            if e.status != E_EXISTS:  # another binding loads it: wait
                                raise
                    if time.monotonic() > deadline:
                        raise PbxError(E_INTERNAL, "band %d of plane %d: timed out loading" % (k, pid))
                    time.sleep(0.001)
        return pid

    def build_pyramid(self, plane_id: int, levels: int, timing: bool = False):
        """Stored levels r+1 .. r+levels of a plane, built on the GPU (2x2 box means);
        returns their plane ids (and the kernels' device ms with timing=True).  With L
        stored levels, tiles of stored level k are TileCtx(..., resolution=L-1-k) (OMERO's
        numbering, include/pbx.h)."""
        ids = (ctypes.c_uint64 * max(levels, 1))()
        ms = ctypes.c_double(0.0)
        _check(lib().pbx_plane_build_pyramid(self._h, plane_id, levels, ids, ctypes.byref(ms)))
        return (list(ids)[:levels], ms.value) if timing else list(ids)[:levels]

    def read_plane_be(self, plane_id: int, nbytes: int) -> bytes:
        buf = ctypes.create_string_buffer(nbytes)
        _check(lib().pbx_plane_read_be(self._h, plane_id, buf, nbytes))
        return buf.raw

    def synchronize(self) -> None:
        _check(lib().pbx_device_synchronize(self._h))

    def set_kernel_streams(self, streams: int, stagger: int = 1) -> None:
        """Kernel streams for pipelined batches (pbx_set_kernel_streams); 1 = serial."""
        _check(lib().pbx_set_kernel_streams(self._h, streams, stagger))

    def release_cached(self) -> None:
        """Free cached batch buffers (device and pinned) no live batch uses."""
        _check(lib().pbx_release_cached(self._h))

    # One getTile (pbx_get_tile): safe to call from many threads at once; concurrent
    # calls are coalesced into batches by the library (ctypes releases the GIL).
    def get_tile(self, ctx: TileCtx, spans: Optional[dict] = None) -> Tuple[int, Optional[bytes]]:
        """(status, body).  ``spans``: a dict that receives the serving batch's stage timings
        (pbx_result_spans: get_tile_direct_ms, write_image_ms, create_metadata_ms, batch_ms,
        d2h_ms, batch_tiles) when the request has a body."""
        req = ctx.to_req()
        res = PbxResult()
        lib().pbx_get_tile(self._h, ctypes.byref(req), ctypes.byref(res))
        try:
            body = ctypes.string_at(res.data, res.len) if res.status == OK and res.len else (
                b"" if res.status == OK else None)
            ctx.region["width"], ctx.region["height"] = res.w, res.h
            if spans is not None and res.owner:
                sp = PbxSpans()
                if lib().pbx_result_spans(ctypes.byref(res), ctypes.byref(sp)) == OK:
                    spans.update({f: getattr(sp, f) for f, _ in PbxSpans._fields_})
        finally:
            lib().pbx_results_release(self._h, ctypes.byref(res), 1)
        return res.status, body

    def ctx_stats(self) -> Tuple[int, int]:
        """(batches launched, requests served) so far."""
        b, r = ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib().pbx_ctx_stats_get(self._h, ctypes.byref(b), ctypes.byref(r)))
        return b.value, r.value

    # Batched getTile: one set of GPU launches for many requests.
    def get_tiles(self, ctxs: Sequence[TileCtx]) -> List[Tuple[int, Optional[bytes]]]:
        n = len(ctxs)
        reqs = (PbxTileReq * max(n, 1))(*[c.to_req() for c in ctxs])
        res = (PbxResult * max(n, 1))()
        st = lib().pbx_get_tiles(self._h, reqs, n, res)
        out = []
        try:
            for i in range(n):
                r = res[i]
                body = ctypes.string_at(r.data, r.len) if r.status == OK and r.len else (
                    b"" if r.status == OK else None)
                ctxs[i].region["width"], ctxs[i].region["height"] = r.w, r.h
                out.append((r.status, body))
        finally:
            lib().pbx_results_release(self._h, res, n)
        if st != OK and not out:
            _check(st)
        return out


    # Batched async: submit returns at once, Ticket.wait() collects (pbx_submit / pbx_wait).
    def submit(self, ctxs: Sequence[TileCtx]) -> "Ticket":
        return Ticket(self, ctxs)


class PixelsNode:
    """N device contexts in ONE process (pbx_node_*): the reference runs all its worker
    verticles in one JVM (PixelBufferMicroserviceVerticle.java:117-118,224-233), so a node-wide
    drop-in holds one context per GPU and routes every getTile to the context holding its plane
    or row band, or (planes replicated on every GPU) to the pbx_shard_of owner among them.
    ``services[k]`` is context k as a PixelsService (register planes / bands there).  The same
    device may be listed several times (tests run two contexts on one GPU)."""

    def __init__(self, n: int, devices: Optional[Sequence[int]] = None, shard_tile: int = 512, **config):
        L = lib()
        cfg = make_config(**config)
        devs = (ctypes.c_int32 * n)(*devices) if devices is not None else None
        h = ctypes.c_void_p()
        _check(L.pbx_node_init(ctypes.byref(cfg), n, devs, shard_tile, ctypes.byref(h)))
        self._h = h
        self.services = [PixelsService(_handle=L.pbx_node_context(h, k)) for k in range(n)]

    def route(self, ctx: TileCtx) -> Tuple[int, int]:
        """(status the serving context would answer, its index); E_NOT_RESIDENT -> the index is
        the shard owner, where the binding should load the plane."""
        req = ctx.to_req()
        k = ctypes.c_int32()
        st = lib().pbx_node_route(self._h, ctypes.byref(req), ctypes.byref(k))
        if st == E_BADARG:
            _check(st)
        return st, k.value

    def get_tile(self, ctx: TileCtx) -> Tuple[int, Optional[bytes], int]:
        """(status, body, index of the context that served it)."""
        req = ctx.to_req()
        res = PbxResult()
        k = ctypes.c_int32(-1)
        lib().pbx_node_get_tile(self._h, ctypes.byref(req), ctypes.byref(res), ctypes.byref(k))
        try:
            body = ctypes.string_at(res.data, res.len) if res.status == OK and res.len else (
                b"" if res.status == OK else None)
            ctx.region["width"], ctx.region["height"] = res.w, res.h
        finally:
            lib().pbx_results_release(None, ctypes.byref(res), 1)
        return res.status, body, k.value

    def close(self) -> None:
        if self._h:
            for s_ in self.services:
                s_._h = None
            lib().pbx_node_shutdown(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Ticket:
    """A submitted batch of getTile requests (pbx_submit); wait() returns what get_tiles would."""

    def __init__(self, service: PixelsService, ctxs: Sequence[TileCtx]):
        self.service, self.ctxs, self.n = service, list(ctxs), len(ctxs)
        self._reqs = make_reqs(self.ctxs)
        self._res = (PbxResult * max(self.n, 1))()
        h = ctypes.c_void_p()
        _check(lib().pbx_submit(service._h, self._reqs, self.n, self._res, ctypes.byref(h)))
        self._t = h

    def wait(self, timeout_us: int = -1) -> Optional[List[Tuple[int, Optional[bytes]]]]:
        """Results, or None if the batch is still running after timeout_us (then call again)."""
        if self._t is None:
            raise RuntimeError("pbx: ticket already collected")
        st = lib().pbx_wait(self.service._h, self._t, timeout_us)
        if st == E_PENDING:
            return None
        self._t = None
        out = []
        try:
            for i in range(self.n):
                r = self._res[i]
                body = ctypes.string_at(r.data, r.len) if r.status == OK and r.len else (
                    b"" if r.status == OK else None)
                self.ctxs[i].region["width"], self.ctxs[i].region["height"] = r.w, r.h
                out.append((r.status, body))
        finally:
            lib().pbx_results_release(self.service._h, self._res, self.n)
        if st != OK and not out:
            _check(st)
        return out


def make_reqs(ctxs: Sequence[TileCtx]):
    """ctypes array of pbx_tile_req for a request list (reusable across batches)."""
    return (PbxTileReq * max(len(ctxs), 1))(*[c.to_req() for c in ctxs]) if ctxs else \
        (PbxTileReq * 1)()


class Batch:
    """Device-resident batch (plan once, launch many): outputs stay in HBM until fetch()."""

    def __init__(self, service: PixelsService, ctxs: Sequence[TileCtx] = (), reqs=None):
        """``ctxs``: TileCtx requests; or ``reqs``: a prebuilt ``make_reqs`` array."""
        self.service = service
        if reqs is None:
            self.n = len(ctxs)
            reqs = make_reqs(ctxs)
        else:
            self.n = len(reqs)
        self._reqs = reqs
        h = ctypes.c_void_p()
        _check(lib().pbx_batch_plan(service.handle, self._reqs, self.n, ctypes.byref(h)))
        self._h = h

    def launch(self) -> None:
        _check(lib().pbx_batch_launch(self.service.handle, self._h))

    def sync(self) -> None:
        _check(lib().pbx_batch_sync(self.service.handle, self._h))

    def stats(self) -> PbxBatchStats:
        s = PbxBatchStats()
        _check(lib().pbx_batch_stats_get(self.service.handle, self._h, ctypes.byref(s)))
        return s

    def fetch(self) -> List[Tuple[int, Optional[bytes]]]:
        res = (PbxResult * max(self.n, 1))()
        _check(lib().pbx_batch_fetch(self.service.handle, self._h, res))
        try:
            return [(res[i].status, ctypes.string_at(res[i].data, res[i].len)
                     if res[i].status == OK else None) for i in range(self.n)]
        finally:
            lib().pbx_results_release(self.service.handle, res, self.n)

    def lz77_records(self, nseg: int, hist_words: int, mrec_words: int):
        """Test hook: (hist, mrec) uint32 arrays of every segment from k_lz77."""
        import numpy as np
        h = np.zeros(nseg * hist_words, np.uint32)
        m = np.zeros(nseg * mrec_words, np.uint32)
        _check(lib().pbx_test_batch_lz77(self.service.handle, self._h, h.ctypes.data,
                                         m.ctypes.data, nseg))
        return h.reshape(nseg, hist_words), m.reshape(nseg, mrec_words)

    def fetch_into_host(self) -> int:
        """D2H of every result into library-owned pinned memory, then release it; returns
        the response bytes (bench: end-to-end rate without Python-side copies)."""
        res = (PbxResult * max(self.n, 1))()
        _check(lib().pbx_batch_fetch(self.service.handle, self._h, res))
        n = sum(res[i].len for i in range(self.n))
        lib().pbx_results_release(self.service.handle, res, self.n)
        return n

    def close(self) -> None:
        if self._h:
            lib().pbx_batch_destroy(self.service.handle, self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ----------------------------------------------------------------- plane sources

class Pixels:
    """The Pixels row getPixels returns (TileRequestHandler.java:220-241: pixelsType, sizeX..T)
    plus the PixelBuffer's getResolutionLevels()."""

    def __init__(self, image_id: int, pixel_type: int, size_x: int, size_y: int, size_z: int = 1,
                 size_c: int = 1, size_t: int = 1, levels: int = 1):
        self.image_id, self.pixel_type = image_id, pixel_type
        self.size_x, self.size_y = size_x, size_y
        self.size_z, self.size_c, self.size_t, self.levels = size_z, size_c, size_t, levels


class PixelSource:
    """Where a plane comes from when this context does not hold it: the reference's
    getPixels (TileRequestHandler.java:220-241) and getPixelBuffer(pixels) (:201-211) +
    PixelBuffer.getTileDirect (:107-109).  Subclass per storage (ROMIO files, Zarr, ...)."""

    def get_pixels(self, image_id: int) -> Optional[Pixels]:
        """The image's Pixels, or None if it does not exist (-> 404, :130-132)."""
        raise NotImplementedError

    def level_size(self, pixels: Pixels, level: int) -> Tuple[int, int]:
        """(size_x, size_y) of STORED level `level` (0 = full resolution)."""
        if level == 0:
            return pixels.size_x, pixels.size_y
        raise NotImplementedError

    def read_rows(self, pixels: Pixels, z: int, c: int, t: int, level: int, y0: int,
                  rows: int) -> bytes:
        """getTileDirect(z, c, t, 0, y0, sizeX, rows) at that level: packed big-endian rows."""
        raise NotImplementedError


# ----------------------------------------------------------------- TileRequestHandler

class TileRequestHandler:
    """TileRequestHandler.java:53-243 — ``get_tile()`` returns bytes, or None (-> 404).

    With a ``source`` (PixelSource), a plane the context does not hold (status
    E_NOT_RESIDENT) is opened as the reference opens it per request — getPixels (:84; None ->
    404), getPixelBuffer + getTileDirect (:86,107-109) — loaded into HBM, and the request
    retried.  The service's policy decides what is loaded: the whole plane, or (with
    ``sparse_band_rows``) only the bands the request's rows cover (region-proportional, as
    getTileDirect reads only the region).  ``band`` = (y0, rows) limits what this context
    holds (a rank's share of a whole slide); requests outside it are answered None here
    (another rank serves them).  Between a load and the retry another loader may evict what
    was loaded (a residency budget smaller than the working set): the load is retried, and a
    tile that still cannot be held is a 500, never the reference's 404.  Without a source the
    context is a closed registry: not resident -> None (404)."""

    LOAD_ATTEMPTS = 4
    NO_SPACE_WAIT_S = 30.0

    def _never_fits(self, pixels: "Pixels", level: int) -> bool:
        """The plane (or one band of it) is larger than the whole residency budget."""
        budget = self.pixels_service.residency_stats()["budget"]
        if not budget:
            return False
        sx, sy = self.source.level_size(pixels, level)
        rows = self.pixels_service.sparse_band_rows or sy
        pitch = (sx * BYTES_PER_PIXEL[pixels.pixel_type] + 255) // 256 * 256
        return pitch * min(rows, sy) + 256 > budget

    def __init__(self, pixels_service: PixelsService, tile_ctx: TileCtx,
                 source: Optional[PixelSource] = None, band: Optional[Tuple[int, int]] = None,
                 tracer=None):
        """``tracer``: optional ``tracer(name, ms, tags)`` called with the reference's span
        names (TileRequestHandler.java:81 get_tile, :104 get_tile_direct, :147 create_metadata,
        :180 write_image; :84 get_pixels and getTileDirect reads of a cold plane as
        get_pixels / load_region): the device stages are those of the batch that served the
        request (pbx_result_spans), get_tile is this call's wall time."""
        self.pixels_service = pixels_service
        self.tile_ctx = tile_ctx
        self.source = source
        self.band = band
        self.tracer = tracer

    def _span(self, name: str, ms: float, **tags) -> None:
        if self.tracer is not None:
            self.tracer(name, ms, tags)

    def _serve(self):
        """One pbx_get_tile with the batch's stage spans."""
        sp = {} if self.tracer is not None else None
        status, body = self.pixels_service.get_tile(self.tile_ctx, sp)
        if sp:
            tags = {"batch_tiles": sp["batch_tiles"]}
            self._span("get_tile_direct", sp["get_tile_direct_ms"], **tags)
            self._span("create_metadata", sp["create_metadata_ms"], **tags)
            self._span("write_image", sp["write_image_ms"], **tags)
            self._span("d2h", sp["d2h_ms"], **tags)
        return status, body

    @staticmethod
    def _answer(status: int, body: Optional[bytes]) -> Optional[bytes]:
        """The tile, None for every status the reference answers null (-> 404), and an
        exception (-> 500, PixelBufferVerticle.java:141-146) for a device failure."""
        if status == E_INTERNAL:
            raise PbxError(E_INTERNAL, "tile batch failed on the device: " +
                           lib().pbx_last_error().decode(errors="replace"))
        return body if status == OK else None

    def get_tile(self, client=None) -> Optional[bytes]:
        t0 = time.perf_counter()
        try:
            return self._get_tile()
        finally:
            self._span("get_tile", (time.perf_counter() - t0) * 1e3)

    def _get_tile(self) -> Optional[bytes]:
        svc, tc = self.pixels_service, self.tile_ctx
        status, body = self._serve()
        if status != E_NOT_RESIDENT or self.source is None:
            return self._answer(status, body)
        t1 = time.perf_counter()
        pixels = self.source.get_pixels(tc.imageId)
        self._span("get_pixels", (time.perf_counter() - t1) * 1e3)
        if pixels is None:
            return None  # :130-132 "Cannot find Image"
        level = 0
        if tc.resolution is not None:
            level = pixels.levels - 1 - tc.resolution  # OMERO numbering -> stored level (include/pbx.h)
        if not (0 <= level < pixels.levels and 0 <= tc.z < pixels.size_z and
                0 <= tc.c < pixels.size_c and 0 <= tc.t < pixels.size_t):
            svc.declare_image(pixels)  # the retry answers the reference's 404
            return self._answer(*svc.get_tile(tc))
        y, h = tc.y, (tc.h or pixels.size_y)  # :92-97 defaulting from the full-resolution size
        if self.band is not None and not (self.band[0] <= y < self.band[0] + self.band[1] and (
                svc.sparse_band_rows or y + h <= self.band[0] + self.band[1])):
            return None  # rows of another context's band (a sparse plane serves every region
            #              that starts in its rows, a whole-row band only those inside it)
        attempts, deadline = 0, time.monotonic() + self.NO_SPACE_WAIT_S
        while attempts < self.LOAD_ATTEMPTS:
            t1 = time.perf_counter()
            try:
                if svc.sparse_band_rows:
                    svc.load_bands(self.source, pixels, tc.z, tc.c, tc.t, level, y, h, own=self.band)
                else:
                    svc.load_plane(self.source, pixels, tc.z, tc.c, tc.t, level, self.band)
            except PbxError as e:
                # the budget is held by planes other requests are reading or have just loaded
                # (the library keeps a fresh plane until its first read): wait for them, unless
                # the plane could never fit
                if e.status != E_NO_SPACE or time.monotonic() > deadline or self._never_fits(pixels, level):
                    raise
                time.sleep(0.002)
                continue
            attempts += 1
            self._span("load_region", (time.perf_counter() - t1) * 1e3)
            status, body = self._serve()
            if status != E_NOT_RESIDENT:
                return self._answer(status, body)
        raise PbxError(E_INTERNAL, "Image:%d z=%d c=%d t=%d: the plane could not be held resident "
                       "(residency budget smaller than the working set)" % (tc.imageId, tc.z, tc.c, tc.t))

    getTile = get_tile


def handle_get_tile(service: PixelsService, body: str, source: Optional[PixelSource] = None, tracer=None):
    """PixelBufferVerticle.getTile (PixelBufferVerticle.java:90-147) over the JSON body.

    Returns (status, payload bytes or message, headers).  400 for an undecodable TileCtx,
    404 when the handler returns null, 500 for any other failure.  ``tracer``: as
    TileRequestHandler's, plus the consumer's own span "handle_get_tile" (:101-104).
    """
    t0 = time.perf_counter()
    try:
        return _handle_get_tile(service, body, source, tracer)
    finally:
        if tracer is not None:
            tracer("handle_get_tile", (time.perf_counter() - t0) * 1e3, {})


def _handle_get_tile(service, body, source, tracer):
    try:
        ctx = TileCtx.from_json(body)
    except Exception:
        return 400, b"Illegal tile context", {}
    try:
        tile = TileRequestHandler(service, ctx, source, tracer=tracer).get_tile()
    except PbxError as e:
        return (400 if e.status == E_BADARG else 500), b"Exception while retrieving tile", {}
    if tile is None:
        return 404, f"Cannot find Image:{ctx.imageId}".encode(), {}
    return 200, tile, {"filename": tile_filename(ctx),
                       "Content-Type": content_type(ctx.format),
                       "Content-Length": str(len(tile))}
