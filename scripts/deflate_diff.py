"""Diagnostic: GPU zlib streams vs the CPU emulator for a set of tile shapes; prints the
first differing byte (and its segment) per shape."""
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "omero-ms-pixel-buffer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import _emu  # noqa: E402
import _oracle as O  # noqa: E402
import pbx  # noqa: E402

svc = pbx.PixelsService(device=0)
svc.register_plane(1, 0, 0, 0, pbx.UINT16, 4096, 4096, generator="noise", seed=0)
svc.register_plane(2, 0, 0, 0, pbx.UINT16, 4096, 4096, generator="fake")
shapes = [(w, h, g) for g in (1, 2) for (w, h) in
          [(512, 512), (1024, 1024), (64, 64), (1024, 64), (2048, 16), (700, 33), (1, 1)]]
for (w, h, g) in shapes:
    st, body = svc.get_tiles([pbx.TileCtx(g, 0, 0, 0, 0, 0, w, h, format="png")])[0]
    t = O.gen_region(2 if g == 1 else 1, O.UINT16, 0, 0, w, h)
    s = O.png_filter_stream(t, O.UINT16, w, h, 0).tobytes()
    z, segs = _emu.deflate(s, 1 + 2 * w)
    n = int.from_bytes(body[91:95], "big")
    gz = body[99:99 + n]
    ok = gz[:len(z)] == z and n == len(z)
    msg = ""
    if not ok:
        i = next((k for k in range(min(len(z), len(gz))) if z[k] != gz[k]), min(len(z), len(gz)))
        pos, seg = 2, 0
        for k, sg in enumerate(segs):
            if i < pos + sg.nbytes:
                seg = k
                break
            pos += sg.nbytes
        try:
            good = zlib.decompress(gz) == s
        except Exception as e:  # noqa: BLE001
            good = repr(e)[:60]
        msg = f"first diff at byte {i} (segment {seg} of {len(segs)}, seg offset {i - pos}); gpu len {n} emu len {len(z)}; gpu inflates ok: {good}"
    print(w, h, "gen", g, "OK" if ok else "DIFF", msg, flush=True)
svc.close()

# LZ77 stage: per-segment histogram and match records vs the emulator
svc = pbx.PixelsService(device=0)
svc.register_plane(1, 0, 0, 0, pbx.UINT16, 4096, 4096, generator="noise", seed=0)
svc.register_plane(2, 0, 0, 0, pbx.UINT16, 4096, 4096, generator="fake")
hw, mw = _emu.lib().pbxemu_hist_words(), _emu.lib().pbxemu_mrec_words()
for (w, h, g) in shapes:
    b = pbx.Batch(svc, [pbx.TileCtx(g, 0, 0, 0, 0, 0, w, h, format="png")])
    b.launch()
    b.sync()
    nseg = b.stats().segments
    gh, gm = b.lz77_records(nseg, hw, mw)
    b.close()
    t = O.gen_region(2 if g == 1 else 1, O.UINT16, 0, 0, w, h)
    s = O.png_filter_stream(t, O.UINT16, w, h, 0).tobytes()
    eh, em = _emu.lz77(s, 1 + 2 * w)
    for k in range(nseg):
        if not (gh[k] == eh[k]).all():
            d = np.nonzero(gh[k] != eh[k])[0]
            print(w, h, g, "seg", k, "HIST diff at", d[:8].tolist(), "gpu", gh[k][d[:8]].tolist(), "emu", eh[k][d[:8]].tolist())
        nw = _emu.lib().pbxemu_threads() // 64
        if not (gm[k][:nw] == em[k][:nw]).all():
            print(w, h, g, "seg", k, "match counts gpu", gm[k][:nw].tolist(), "emu", em[k][:nw].tolist())
            for wv in range(nw):
                gp = gm[k][nw + wv * 256: nw + wv * 256 + max(gm[k][wv], em[k][wv])]
                ep = em[k][nw + wv * 256: nw + wv * 256 + max(gm[k][wv], em[k][wv])]
                if not (gp == ep).all():
                    i = int(np.nonzero(gp != ep)[0][0])
                    print("   wave", wv, "first diff match", i, "gpu", hex(int(gp[i])), "emu", hex(int(ep[i])),
                          "prev", hex(int(gp[i - 1])) if i else None)
                    break
            break
    print(w, h, g, "lz77 checked", nseg, "segments", flush=True)
svc.close()
