"""Generate the Zarr chunk-codec golden fixtures (tests/golden/zarr/).

Run with an interpreter that has imagecodecs (c-blosc 1.21.0, zlib), e.g.
    /opt/conda/bin/python3.9 tests/golden/zarr/make_zarr_golden.py
Each case is a small 2-D array encoded the way a Zarr v2 writer stores one chunk
(numcodecs Blosc / Zlib = c-blosc frame / zlib stream of the C-order chunk bytes).
Writes <case>.enc (compressed chunk), <case>.raw (expected decoded bytes) and manifest.json.
"""
import json
import os

import imagecodecs as ic
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def image(h, w, dtype, seed, kind="noise"):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    if kind == "noise":  # G_NOISE-like: blocky background + 9-bit noise
        v = 256 + ((x >> 5) + (y >> 5)) % 16 * 48 + rng.integers(0, 512, size=(h, w))
    elif kind == "smooth":  # gradients with flat patches: long LZ matches
        v = (x // 7 + y // 5) % 200 + np.where((x // 40 + y // 40) % 3 == 0, 0, 1000)
    else:  # incompressible
        v = rng.integers(0, 1 << 30, size=(h, w))
    return v.astype(dtype)


CASES = [
    # name, shape, dtype, kind, codec, params
    ("blosc_lz4_u16_100x77", (100, 77), ">u2", "noise", "blosc", dict(compressor="lz4", level=5, shuffle=1)),
    ("blosc_lz4_u16_600x500", (600, 500), ">u2", "noise", "blosc", dict(compressor="lz4", level=5, shuffle=1)),
    ("blosc_lz4_u16_smooth_512x256", (512, 256), ">u2", "smooth", "blosc", dict(compressor="lz4", level=5, shuffle=1)),
    ("blosc_lz4_u8_256x256", (256, 256), "u1", "smooth", "blosc", dict(compressor="lz4", level=5, shuffle=1)),
    ("blosc_lz4_f32_128x128", (128, 128), ">f4", "noise", "blosc", dict(compressor="lz4", level=5, shuffle=1)),
    ("blosc_lz4_i32_le_96x96", (96, 96), "<i4", "smooth", "blosc", dict(compressor="lz4", level=9, shuffle=1)),
    ("blosc_lz4_noshuffle_u16_200x200", (200, 200), ">u2", "noise", "blosc", dict(compressor="lz4", level=5, shuffle=0)),
    ("blosc_lz4hc_u16_256x256", (256, 256), ">u2", "noise", "blosc", dict(compressor="lz4hc", level=5, shuffle=1)),
    ("blosc_lz4_memcpyed_u16_64x64", (64, 64), ">u2", "random", "blosc", dict(compressor="lz4", level=5, shuffle=1)),
    ("blosc_lz4_f64_64x40", (64, 40), ">f8", "smooth", "blosc", dict(compressor="lz4", level=5, shuffle=1)),
    ("blosc_zlib_u16_300x300", (300, 300), ">u2", "noise", "blosc", dict(compressor="zlib", level=5, shuffle=1)),
    ("zlib_l1_u16_256x200", (256, 200), ">u2", "noise", "zlib", dict(level=1)),
    ("zlib_l6_u16_smooth_256x256", (256, 256), ">u2", "smooth", "zlib", dict(level=6)),
    ("zlib_l9_u8_128x100", (128, 100), "u1", "smooth", "zlib", dict(level=9)),
    ("zlib_l6_u16_noise_128x128", (128, 128), ">u2", "noise", "zlib", dict(level=6)),
    # blosc-zstd, blosclz and bit shuffle (round 1 rejected these with 400; decoded since round 2)
    ("blosc_zstd_u16_64x64", (64, 64), ">u2", "smooth", "blosc", dict(compressor="zstd", level=5, shuffle=1)),
    ("blosc_blosclz_u16_128x128", (128, 128), ">u2", "smooth", "blosc", dict(compressor="blosclz", level=5, shuffle=1)),
    ("blosc_lz4_bitshuffle_u16_128x128", (128, 128), ">u2", "smooth", "blosc", dict(compressor="lz4", level=5, shuffle=2)),
    ("blosc_zstd_u16_600x500", (600, 500), ">u2", "noise", "blosc", dict(compressor="zstd", level=5, shuffle=1)),
    ("blosc_zstd_l1_f32_256x256", (256, 256), ">f4", "noise", "blosc", dict(compressor="zstd", level=1, shuffle=1)),
    ("blosc_zstd_l9_u8_300x200", (300, 200), "u1", "smooth", "blosc", dict(compressor="zstd", level=9, shuffle=0)),
    ("blosc_zstd_bitshuffle_u16_512x512", (512, 512), ">u2", "noise", "blosc", dict(compressor="zstd", level=5, shuffle=2)),
    ("blosc_blosclz_u16_600x500", (600, 500), ">u2", "noise", "blosc", dict(compressor="blosclz", level=5, shuffle=1)),
    ("blosc_blosclz_l9_u8_256x256", (256, 256), "u1", "smooth", "blosc", dict(compressor="blosclz", level=9, shuffle=0)),
    ("blosc_blosclz_i32_le_100x97", (100, 97), "<i4", "smooth", "blosc", dict(compressor="blosclz", level=5, shuffle=1)),
    ("blosc_blosclz_bitshuffle_f32_128x130", (128, 130), ">f4", "noise", "blosc", dict(compressor="blosclz", level=5, shuffle=2)),
    ("blosc_lz4_bitshuffle_u8_333x101", (333, 101), "u1", "noise", "blosc", dict(compressor="lz4", level=5, shuffle=2)),
    ("blosc_lz4_bitshuffle_f64_100x77", (100, 77), ">f8", "smooth", "blosc", dict(compressor="lz4", level=5, shuffle=2)),
    ("blosc_zlib_bitshuffle_u16_257x255", (257, 255), ">u2", "noise", "blosc", dict(compressor="zlib", level=5, shuffle=2)),
]


def main():
    manifest = {"generator": "imagecodecs %s, %s, %s" % (ic.__version__, ic.blosc_version(), ic.zstd_version()),
                "cases": []}
    for i, (name, shape, dtype, kind, codec, params) in enumerate(CASES):
        a = image(shape[0], shape[1], dtype, seed=i, kind=kind)
        raw = a.tobytes()
        if codec == "blosc":
            enc = ic.blosc_encode(raw, typesize=a.dtype.itemsize, numthreads=1, **params)
            assert ic.blosc_decode(enc) == raw
        else:
            enc = ic.zlib_encode(raw, level=params["level"])
        with open(os.path.join(HERE, name + ".enc"), "wb") as f:
            f.write(enc)
        with open(os.path.join(HERE, name + ".raw"), "wb") as f:
            f.write(raw)
        manifest["cases"].append({"name": name, "shape": list(shape), "dtype": dtype, "codec": codec,
                                  "params": params, "enc_bytes": len(enc), "raw_bytes": len(raw)})
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
