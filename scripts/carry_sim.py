"""CPU model of k_lz77's cross-wave carry schedule, CPU only.

The serial parse (ph_parse_emu, deflate_seg.h): wave w walks its 2 KiB sub-segment from where
wave w-1's last recorded match ends.  The device walks every wave at once from a PREDICTED
start and repairs wrong starts in rounds.  This counts the rounds two schedules need per
segment on a tile stream:

  serial  (round 4): after round 0, waves from the first mispredicted one on walk again one per
          round, in wave order;
  jacobi  (round 5): every wave whose start is still wrong walks again in the same round from
          the previous wave's latest end; a round fixes at least the first wrong wave, and a
          wave whose end does not depend on its start (a row break inside it) fixes all.

Usage: python scripts/carry_sim.py [fake|noise] [filter 0..5] [tiles]
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/", 2)[0] + "/tests")
import _oracle as O  # noqa: E402

SEG, WIN, SUB, NW, CAP, MINCOV, MAXMW = 16384, 4096, 2048, 8, 32, 32, 256


def split(n):
    n0 = (n + SEG - 1) // SEG
    l = min(((n + n0 - 1) // n0 + 15) & ~15, SEG)
    return (n + l - 1) // l, l


def minlen(d):
    return 3 if d <= 256 else 4 if d <= 4096 else 6


def seg_parse(buf, wl, sl, rowlen):
    """Returns walk(w, start) -> (records, end-if-past-se-else-0) for one segment."""
    cands = [1, 2] + ([rowlen] if rowlen > 2 else [])

    def clen(p, se, d):
        a = wl + p
        if d > a or p >= se:
            return 0
        lim = min(se - p, CAP)
        n = 0
        while n < lim and buf[a + n] == buf[a - d + n]:
            n += 1
        return n

    def best(p, se):
        L = D = 0
        for d in cands:
            n = clen(p, se, d)
            if n >= minlen(d) and n > L:
                L, D = n, d
        return L, D

    def ext(p, L, D, lim):
        a = wl + p
        while L < lim and buf[a + L] == buf[a - D + L]:
            L += 1
        return L

    def walk(w, start):
        ss = w * SUB
        se = min(ss + SUB, sl)
        p, recs, cov = start, [], 0
        while p < se:
            L, D = best(p, se)
            if L < 3:
                p += 1
                continue
            L1, _ = best(p + 1, se)
            if L1 > L:
                p += 1
                continue
            if L >= CAP:
                L = ext(p, L, D, min(se - p, 258))
            if p + L == se and se < sl:
                L = ext(p, L, D, min(sl - p, 258))
            if len(recs) < MAXMW:
                recs.append((p, L, D))
                cov += L
            p += L
        if cov < MINCOV:
            recs = []
        end = recs[-1][0] + recs[-1][1] if recs else 0
        return recs, (end if end > se else 0)

    return walk


def schedule(walk, nw, reach, pred):
    """(serial rounds, jacobi rounds, records equal) for one segment."""
    # the serial parse
    true_start, ends, recs = [0] * nw, [0] * nw, []
    for w in range(nw):
        s = max(w * SUB, ends[w - 1]) if w else 0
        true_start[w] = s
        r, ends[w] = walk(w, s)
        recs.append(r)
    # round 0 from the predictions
    st = [pred(w) for w in range(nw)]
    en = [walk(w, st[w])[1] for w in range(nw)]
    if not any(reach):
        assert st == true_start
        return 0, 0
    # serial (round 4): first wrong wave f, then one wave per round from f on
    f = next((i for i in range(1, nw) if reach[i - 1] and max(en[i - 1], i * SUB) != st[i]), nw)
    serial = 0 if f == nw else nw - f
    # jacobi (round 5)
    jac = 0
    while True:
        f = next((i for i in range(1, nw) if max(en[i - 1], i * SUB) != st[i]), nw)
        if f == nw:
            break
        jac += 1
        new = list(en)
        for i in range(f, nw):
            a = max(en[i - 1], i * SUB)
            if a != st[i]:
                st[i] = a
                new[i] = walk(i, a)[1]
        en = new
        assert jac <= nw
    assert st == true_start, (st, true_start)
    return serial, jac


def main():
    gen = {"fake": O.GEN_FAKE, "noise": O.GEN_NOISE}[sys.argv[1] if len(sys.argv) > 1 else "fake"]
    filt = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    tiles = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    tot = {"segs": 0, "serial": 0, "jacobi": 0}
    for t in range(tiles):
        tile = O.gen_region(gen, O.UINT16, 512 * t, 512 * (t % 3), 512, 512)
        stream = O.png_filter_stream(np.frombuffer(tile.tobytes(), np.uint8), O.UINT16, 512, 512, filt).tobytes()
        rowlen = 1025
        nseg, sl_nom = split(len(stream))
        for k in range(nseg):
            s = k * sl_nom
            sl = min(len(stream) - s, sl_nom)
            wl = min(s, min((max(rowlen, 2) + 15) & ~15, WIN))
            buf = stream[s - wl:s + sl] + bytes(600)
            walk = seg_parse(buf, wl, sl, rowlen)
            nw = (sl + SUB - 1) // SUB
            # reachable boundaries: a paying run ends at the sub-segment's last byte
            reach = []
            for b in range(nw - 1):
                e = (b + 1) * SUB
                a = wl + e
                x = buf[a - 8:a]
                r = len(set(x[-4:])) == 1 or (x[-1] == x[-3] and x[-2] == x[-4] and x[-3] == x[-5])
                d = rowlen
                if a >= minlen(d) + d:
                    m = minlen(d)
                    r = r or buf[a - m:a] == buf[a - m - d:a - d]
                reach.append(r)

            def pred(j):
                sj = j * SUB
                return 258 * ((sj + 257) // 258) if j and reach[j - 1] else sj

            se, jc = schedule(walk, nw, reach, pred)
            tot["segs"] += 1
            tot["serial"] += se
            tot["jacobi"] += jc
    print(tot)


if __name__ == "__main__":
    main()
