// pbx_config.h — the deflate configuration the library is built with, and the segment
// split of a stream (shared by the host planner, the kernels and the CPU emulator).
#pragma once
#include "deflate_seg.h"

namespace pbx {

// PBX_NT = 512 threads (8 waves) per segment of up to PBX_SEG = 16 KiB, with at most
// PBX_WIN look-back bytes (the longest candidate distance is one row); PBX_BLK consecutive
// segments of a tile form one deflate block with one Huffman code.  Overridable for
// experiments only.
#ifndef PBX_WIN
#define PBX_WIN 4096
#endif
#ifndef PBX_NT
#define PBX_NT 512
#endif
#ifndef PBX_SEG
#define PBX_SEG 16384
#endif
#ifndef PBX_BLK
#define PBX_BLK 64
#endif
using DeflateMainCfg = DeflateCfg<PBX_NT, PBX_SEG, PBX_WIN>;
constexpr uint32_t BLK_SEGS = PBX_BLK;  // segments per Huffman block at most (filter None, TIFF)
// Row-filtered tiles: at most 16 segments per block (a 512x512 uint16 tile's 33 segments: three
// blocks of 11).  Rounds 1-5 used 3, measured when blocks of more segments compressed worse (the
// merge's 16-bit weights wrapped, since fixed); round 6 re-measured 3 / 6 / 11 / 16 / 33 / 64 on
// the bench's filter lines (profiles/r06zq, r06zr): 16 writes fewer bytes than 3 on every
// generator and filter (adaptive: G_NOISE 374,988 vs 375,103, G_FAKE 1,785 vs 1,956, Poisson
// 283,283 vs 283,580 B/tile) in a third of the k_huff blocks (filter lines +8-12% tiles/s);
// one block per tile (33, 64) is 1% faster again but matches filter None's bytes on Poisson
// instead of beating them.  Without a filter one code per tile of up to 64 segments: the same
// bytes as blocks of 11 on noise (+0.005%), +0.3% on G_FAKE, and a third of the k_huff waves
// (0.208 -> 0.125 ms per 4096 tiles, profiles/r03_p22-23).
#ifndef PBX_BLK_FILT
#define PBX_BLK_FILT 16
#endif
constexpr uint32_t BLK_SEGS_FILTERED = PBX_BLK_FILT;
// The planner's longest segment.  A stored Huffman block is one stored block per segment
// (block_nbytes), so only a segment must fit a stored block's 65535 bytes.
constexpr uint32_t SPLIT_MAX = PBX_SEG;
static_assert(BLK_SEGS >= 1 && BLK_SEGS <= 64 && SPLIT_MAX <= 65535, "a stored block holds <= 65535 bytes");

// Huffman blocks of a tile of nseg segments.
PBX_HD uint32_t tile_blocks(uint32_t nseg, uint32_t cap = BLK_SEGS) { return (nseg + cap - 1) / cap; }
// Block j of a tile's nb blocks holds its segments [block_seg0(j, nseg, nb),
// block_seg0(j + 1, nseg, nb)): an even split (33 segments of a 512x512 uint16 PNG in
// one block of 33 at the default cap; three blocks of 11 at a cap of 16).
PBX_HD uint32_t block_seg0(uint32_t j, uint32_t nseg, uint32_t nb) {
    return (uint32_t)((uint64_t)j * nseg / nb);
}
// Per-segment HBM records between the deflate kernels (32-bit words).
constexpr uint32_t HIST_WORDS = 320;  // literal/length + distance histogram
constexpr uint32_t MREC_WORDS =       // per-wave match counts, positions|lengths, distances
    (DeflateMainCfg::NW + 2 * DeflateMainCfg::NW * DeflateMainCfg::MAXMW + 63) & ~63u;
constexpr uint32_t CODE_WORDS = 320 + DeflateMainCfg::HDRW;  // codes + block header bits

// Split of a stream of `len` bytes into segments of at most SEG bytes: an equal split
// rounded up to 16 bytes (segment starts stay 16-byte aligned for vector loads); the
// count is then recomputed so that the last segment is never empty.
inline void deflate_split(uint64_t len, uint32_t& nseg, uint32_t& seg_len) {
    const uint64_t S = (uint64_t)SPLIT_MAX;
    if (len == 0) { nseg = 1; seg_len = 16; return; }
    const uint64_t n0 = (len + S - 1) / S;
    uint64_t l = ((len + n0 - 1) / n0 + 15) & ~15ull;
    if (l > S) l = S;
    seg_len = (uint32_t)l;
    nseg = (uint32_t)((len + l - 1) / l);
}

}  // namespace pbx
