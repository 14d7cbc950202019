// pbx_kernels.h — host-side launchers of the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pbx_common.h"

namespace pbx {

// Synthetic plane (G_FAKE / G_NOISE) written little-endian into a pitched HBM plane.
hipError_t launch_gen_plane(hipStream_t st, uint8_t* out, int64_t pitch, int32_t sx, int32_t sy,
                            int32_t pixel_type, int32_t kind, uint64_t seed, int32_t plane_no,
                            int32_t z, int32_t c, int32_t t);

// K1: raw / uncompressed-TIFF tiles (getTileDirect + big-endian; TIFF header in front).
hipError_t launch_extract(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                          uint32_t nblocks, uint8_t* out);

// K1+K2: extract + byte swap + sign flip + PNG filter (or raw BE bytes for deflate-TIFF)
// into the per-tile byte streams the deflate kernel reads.  One workgroup per band.
hipError_t launch_filter(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                         uint32_t nblocks, uint8_t* stream);
uint32_t filter_band_rows();

// K3-K5: fused filter + LZ77 + Huffman + bit packing, one workgroup per segment.
hipError_t launch_deflate(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                          uint32_t nseg, const uint8_t* stream, uint8_t* slots,
                          uint32_t slot_stride, SegOut* segout, uint64_t* stamps = nullptr);

// K7: container sizes, exclusive scan into offsets[0..n] (offsets[n] = total).
hipError_t launch_sizes_scan(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                             const SegOut* segout, uint64_t* sizes, uint64_t* offsets);

// K5/K6: PNG (APNGWriter layout) or deflate-TIFF container, compacted at offsets[i].
hipError_t launch_assemble(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                           const SegOut* segout, const uint8_t* slots, uint32_t slot_stride,
                           const uint64_t* offsets, uint8_t* out);

uint32_t deflate_slot_stride();
uint32_t deflate_threads();
size_t deflate_lds_bytes();

}  // namespace pbx
