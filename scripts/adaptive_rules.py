"""Adaptive PNG filter rules on the CPU: zlib-6 bytes of the filtered
streams of six 512^2 uint16 tiles per generator (G_NOISE, G_FAKE, Poisson-like lambda 200..300)
under per-row filter-selection rules:
  none      filter None on every row (the reference)
  plain     minimum sum |byte - prediction| (the product rule: oracle/pbx_oracle.c, k_filter*)
  signed    libpng's minimum sum |signed residual|
  second    minimum sum |residual - residual bpp back| (the residual's own variation)
  planes    per byte plane, sum of circular distances from the plane's median residual
  cnone_med plain for Sub..Paeth, None scored by the bytes' distance from their plane's median
  ccirc     the same with a circular centre
  entropy   minimum empirical entropy of the residual bytes, per byte plane (two histograms
            of 256 bins per candidate per row)
Output: profiles/r06h/adaptive_rules.txt.  CPU only."""
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RULES = sys.argv[1:] or ["none", "plain", "signed", "second", "planes", "cnone_med", "ccirc", "entropy"]
sys.path.insert(0, os.path.join(ROOT, "tests"))
import _oracle as O
T = 512
def tiles(kind):
    out = []
    if kind == "poisson":
        rng = np.random.default_rng(5)
        for j in range(6):
            lam = 200 + 100 * (0.5 + 0.25*np.sin((np.arange(T)+j*512)/900.0))[None, :] * np.ones((T, 1))
            out.append(rng.poisson(lam).astype(">u2").tobytes())
    else:
        k = 2 if kind == "noise" else 1
        for j in range(6):
            out.append(O.gen_region(k, O.UINT16, (j * 7 % 64) * T, (j * 5 % 64) * T, T, T).tobytes())
    return out
def preds(cur, prev, bpp=2):
    left = np.concatenate([np.zeros(bpp, np.int32), cur[:-bpp]])
    ul = np.concatenate([np.zeros(bpp, np.int32), prev[:-bpp]])
    up = prev
    p = left + up - ul
    pa, pb, pc = np.abs(p - left), np.abs(p - up), np.abs(p - ul)
    paeth = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, up, ul))
    return [np.zeros_like(cur), left, up, (left + up) >> 1, paeth]
def stream(tile, rule):
    a = np.frombuffer(tile, np.uint8).reshape(T, 2 * T).astype(np.int32)
    prev = np.zeros(2 * T, np.int32)
    rows = []
    for r in range(T):
        cur = a[r]
        P = preds(cur, prev)
        res = [((cur - p) & 255) for p in P]
        if rule == "none": f = 0
        elif rule == "plain": f = int(np.argmin([np.abs(cur - p).sum() for p in P]))
        elif rule == "signed": f = int(np.argmin([np.abs(((e + 128) & 255) - 128).sum() for e in res]))
        elif rule == "second":  # SAD of the residual's own left differences (per byte plane)
            f = int(np.argmin([np.abs(((e[2:] - e[:-2] + 128) & 255) - 128).sum() for e in res]))
        elif rule == "planes":  # per byte plane: signed distance from that plane's median residual
            sc = []
            for e in res:
                s = 0
                for ph in range(2):
                    v = e[ph::2]
                    m = int(np.median(v))
                    s += np.abs(((v - m + 128) & 255) - 128).sum()
                sc.append(s)
            f = int(np.argmin(sc))
        elif rule in ("ccirc", "ccirc_sub"):
            sc = [np.abs(cur - p).sum() for p in P]
            s0 = 0
            for ph in range(2):
                v = cur[ph::2]
                # circular centre: the byte value whose half-circle window holds most bytes
                c = np.bincount(v, minlength=256)
                win = np.convolve(np.concatenate([c, c]), np.ones(128, int), "valid")[:256]
                lo = int(np.argmax(win)); m = (lo + 64) & 255
                s0 += np.abs(((v - m + 128) & 255) - 128).sum()
            sc[0] = s0
            f = int(np.argmin(sc))
        elif rule in ("cnone", "cnone_med"):
            sc = [np.abs(cur - p).sum() for p in P]
            s0 = 0
            for ph in range(2):
                v = cur[ph::2]
                m = int(np.median(v)) if rule == "cnone_med" else (int(v.sum()) + len(v) // 2) // len(v)
                s0 += np.abs(v - m).sum()
            sc[0] = s0
            f = int(np.argmin(sc))
        elif rule == "entropy":
            def H(e):
                c = np.bincount(e, minlength=256); c = c[c > 0] / len(e)
                return -(c * np.log2(c)).sum()
            f = int(np.argmin([H(e[0::2]) + H(e[1::2]) for e in res]))
        rows.append(np.concatenate([[f], res[f]]).astype(np.uint8))
        prev = cur
    return np.concatenate(rows).tobytes()
for kind in ("noise", "fake", "poisson"):
    ts = tiles(kind)
    out = []
    for rule in RULES:
        n = sum(len(zlib.compress(stream(t, rule), 6)) for t in ts) / len(ts)
        out.append(f"{rule} {n:.0f}")
    print(kind, " | ".join(out), flush=True)
