"""Symbol histograms for Huffman-stage tests: realistic, degenerate and adversarial
(Fibonacci counts force code lengths past 15 bits -> zlib's overflow repair)."""
import numpy as np

SEG = 16384


def _fill(lit, dist=None):
    h = np.zeros(320, np.uint64)
    h[: len(lit)] = lit
    if dist is not None:
        h[288: 288 + len(dist)] = dist
    h[256] = 1  # end of block, always present
    return h


def cases(seed=0):
    rng = np.random.default_rng(seed)
    out = []
    # noise-like: five hot high bytes, flat low bytes, few matches
    lit = np.zeros(286, np.uint64)
    lit[1:6] = 1500
    lit[:256] += rng.integers(15, 40, 256).astype(np.uint64)
    lit[257:286] = rng.choice([0, 0, 1, 2, 5, 10, 30], 29)
    out.append(_fill(lit, rng.integers(0, 50, 30)))
    # smooth image: peaked literals, many matches
    b = np.arange(256)
    lit = np.zeros(286, np.uint64)
    lit[:256] = (3000 * 2.0 ** (-np.abs(b - 128) / 4.0)).astype(np.uint64)
    lit[257:286] = rng.choice([0, 1, 20, 100, 300], 29)
    out.append(_fill(lit, rng.choice([0, 1, 5, 80, 400], 30)))
    # single literal, no matches (trees completed by the forced symbols)
    lit = np.zeros(286, np.uint64)
    lit[77] = SEG
    out.append(_fill(lit))
    # nothing but the end of block
    out.append(_fill(np.zeros(286, np.uint64)))
    # all literals equal
    out.append(_fill(np.full(256, 64, np.uint64)))
    # Fibonacci counts: depth > 15 for literals, > 7 for the code-length code
    fib = [1, 1]
    while len(fib) < 24:
        fib.append(fib[-1] + fib[-2])
    lit = np.zeros(286, np.uint64)
    lit[: 24] = fib[:24]
    out.append(_fill(lit, fib[:12]))
    # spread Fibonacci over lengths and distances
    lit = np.zeros(286, np.uint64)
    idx = rng.permutation(286)[:22]
    lit[idx] = fib[:22]
    out.append(_fill(lit, np.array(fib[:20])))
    # random mixtures
    for _ in range(24):
        lit = rng.choice([0, 0, 1, 2, 3, 7, 50, 400, 3000], 286).astype(np.uint64)
        dist = rng.choice([0, 0, 1, 3, 10, 100, 1000], 30).astype(np.uint64)
        out.append(_fill(lit, dist))
    # every symbol once
    out.append(_fill(np.ones(286, np.uint64), np.ones(30, np.uint64)))
    return [h.astype(np.uint32) for h in out]


def stream_len(h):
    """A plausible segment length for the histogram (literals + 3 bytes per match)."""
    lit = int(h[:256].sum())
    matches = int(h[257:286].sum())
    return max(1, min(SEG, lit + 3 * matches))
