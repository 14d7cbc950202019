"""One 8192^2 uint16 plane of 512^2 chunks per codec through pbx_plane_register_zarr
(rocprofv3 kernel-trace / PMC workload for the k_zarr_* kernels)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "omero-ms-pixel-buffer_amd"), os.path.join(ROOT, "tests")]
import pbx  # noqa: E402
import _zarr  # noqa: E402

codecs = sys.argv[1:] or ["blosc", "zlib"]
plane = _zarr.noise_plane(8192, 8192, ">u2", seed=5)
with pbx.PixelsService(device=0) as svc:
    for k, comp in enumerate(codecs):
        chunks = _zarr.encode_chunks(plane, 512, 512, comp, **({"level": 1} if comp == "zlib" else {}))
        pid, ms = svc.register_zarr_plane(100 + k, 0, 0, 0, pbx.UINT16, 8192, 8192, 512, 512, comp,
                                          chunks, timing=True)
        print(comp, "decode %.3f ms place %.3f ms" % ms, flush=True)
        svc.release_plane(pid)
