// pbx_config.h — the deflate configuration the library is built with, and the segment
// split of a stream (shared by the host planner, the kernels and the CPU emulator).
#pragma once
#include "deflate_seg.h"

namespace pbx {

// 512 threads (8 waves), 16 KiB segments with an 8 KiB look-back window, 4096-entry hash.
using DeflateMainCfg = DeflateCfg<512, 16384, 8192, 12>;

// Number of segments for a stream of `len` bytes: equal-sized segments of at most SEG.
inline uint32_t deflate_nsegs(uint64_t len) {
    const uint64_t seg = (uint64_t)DeflateMainCfg::SEG;
    return len == 0 ? 1u : (uint32_t)((len + seg - 1) / seg);
}
inline uint32_t deflate_seg_len(uint64_t len, uint32_t nseg) {
    return (uint32_t)((len + nseg - 1) / nseg);
}

}  // namespace pbx
