"""Generate tests/golden/ fixtures from the CPU oracle and pin them with independent tools.

Run in this container (not on the GPU box):  python tests/golden/make_golden.py
  * raw tiles: big-endian samples, also produced by the independent numpy generator
    (tests/_numpy_ref.py) — the two must agree byte for byte;
  * PNG (oracle = APNGWriter restatement, filter None + zlib 6): decoded by PIL
    (/usr/bin/python3) to the raw tile (int8/int16 after the sign flip);
  * TIFF (oracle = big-endian uncompressed): decoded by tifffile 2021.7.2
    (/opt/conda/bin/python3.9), independent of our C decoder.
The manifest records sha256 of every file and of the independently decoded pixels.
"""
import hashlib
import io
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import _numpy_ref  # noqa: E402
import _oracle as O  # noqa: E402

W, H, X0, Y0 = 64, 48, 3, 2
KINDS = {1: "fake", 2: "noise"}
CONDA_PY = "/opt/conda/bin/python3.9"


def sha(b):
    return hashlib.sha256(b).hexdigest()


def main():
    from PIL import Image
    manifest = {"tile": {"w": W, "h": H, "x": X0, "y": Y0}, "cases": []}
    tiff_jobs = []
    for kind, kname in KINDS.items():
        for pt in range(8):
            name = f"{O.TYPE_NAMES[pt]}_{kname}"
            raw = O.gen_region(kind, pt, X0, Y0, W, H).tobytes()
            ref = _numpy_ref.region(kind, pt, X0, Y0, W, H)
            assert raw == ref, f"oracle generator disagrees with numpy restatement: {name}"
            case = {"name": name, "pixel_type": pt, "kind": kind, "raw_sha256": sha(raw)}
            with open(os.path.join(HERE, f"raw_{name}.bin"), "wb") as f:
                f.write(raw)
            st, png = O.png_encode(np.frombuffer(raw, np.uint8), pt, W, H)
            if pt in (O.INT8, O.UINT8, O.INT16, O.UINT16):
                assert st == 0
                with open(os.path.join(HERE, f"png_{name}.png"), "wb") as f:
                    f.write(png)
                im = np.array(Image.open(io.BytesIO(png)))
                be = ">u2" if O.BPP[pt] == 2 else ">u1"
                dec = im.astype(be).tobytes()
                flipped = bytearray(raw)
                if pt in (O.INT8, O.INT16):
                    flipped[0::O.BPP[pt]] = bytes(b ^ 0x80 for b in flipped[0::O.BPP[pt]])
                assert dec == bytes(flipped), f"PIL decode mismatch {name}"
                case.update(png_sha256=sha(png), png_len=len(png),
                            png_pil_pixels_sha256=sha(dec))
            else:
                assert st == 404
                case["png_status"] = 404
            st, tif = O.tiff_encode(np.frombuffer(raw, np.uint8), pt, W, H)
            assert st == 0
            tpath = os.path.join(HERE, f"tif_{name}.tif")
            with open(tpath, "wb") as f:
                f.write(tif)
            case.update(tif_sha256=sha(tif), tif_len=len(tif))
            tiff_jobs.append((tpath, name))
            manifest["cases"].append(case)
    # independent TIFF decode with tifffile (python3.9 env)
    script = ("import sys,json,hashlib,tifffile\n"
              "out={}\n"
              "for p,n in json.loads(sys.argv[1]):\n"
              "    a=tifffile.imread(p); out[n]=[hashlib.sha256(a.astype(a.dtype.newbyteorder('>')).tobytes()).hexdigest(), str(a.dtype)]\n"
              "print(json.dumps(out))\n")
    r = subprocess.run([CONDA_PY, "-c", script, json.dumps(tiff_jobs)], capture_output=True,
                       text=True, check=True)
    dec = json.loads(r.stdout)
    for case in manifest["cases"]:
        h, dt = dec[case["name"]]
        assert h == case["raw_sha256"], f"tifffile decode mismatch {case['name']}"
        case["tif_tifffile_pixels_sha256"] = h
        case["tifffile_dtype"] = dt
    # reference-sized known answers (no files): sizes of the survey's measurements
    big = {}
    for kind, kname in KINDS.items():
        t = O.gen_region(kind, O.UINT16, 0, 0, 512, 512)
        s = O.png_filter_stream(t, O.UINT16, 512, 512, 0).tobytes()
        import zlib
        big[kname] = {"stream_sha256": sha(s), "zlib6_len": len(zlib.compress(s, 6)),
                      "raw_sha256": sha(t.tobytes())}
    manifest["u16_512_png"] = big
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", len(manifest["cases"]), "cases")


if __name__ == "__main__":
    main()
