// pbx_kernels.h — host-side launchers of the gfx950 kernels (kernels_io.hip,
// kernels_deflate.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pbx_common.h"

namespace pbx {

// Synthetic plane (G_FAKE / G_NOISE) written little-endian into a pitched HBM plane.
// rows [y0, y0 + rows) of a synthetic plane, row y0 at `out`
hipError_t launch_gen_plane(hipStream_t st, uint8_t* out, int64_t pitch, int32_t sx, int32_t y0,
                            int32_t rows, int32_t pixel_type, int32_t kind, uint64_t seed,
                            int32_t plane_no, int32_t z, int32_t c, int32_t t);

// K1: raw / uncompressed-TIFF tiles (getTileDirect + big-endian; TIFF header in front).
// Resolution pyramid level: dst (dx x dy) = 2x2 box mean of src (sx x sy), edge samples
// repeated for odd sizes; samples big-endian in memory when `be`.
hipError_t launch_downsample(hipStream_t st, const uint8_t* src, int64_t spitch, int32_t sx, int32_t sy,
                             uint8_t* dst, int64_t dpitch, int32_t dx, int32_t dy, int32_t pixel_type,
                             bool be);
// test hook (pbx_test_stall_batch): one wave spinning until *flag == 0 or limit_ticks of the
// 100 MHz constant clock
hipError_t launch_stall(hipStream_t st, const uint32_t* flag, uint64_t limit_ticks);
hipError_t launch_extract(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                          uint32_t nblocks, uint8_t* out, bool unaligned);
// Tiled-TIFF headers (IFD + TileOffsets/TileByteCounts), one workgroup per response: after
// k_extract for uncompressed responses (in `fixed`), after k_frame for deflate ones (`zout`).
hipError_t launch_tiff_tiled(hipStream_t st, const TiledHdr* d_th, uint32_t nth, uint8_t* fixed,
                             const uint64_t* offs, uint8_t* zout);

// K1+K2: extract + byte swap + sign flip + PNG filter (or raw BE bytes for deflate-TIFF)
// into the per-tile byte streams the deflate kernels read.  One workgroup per band.
hipError_t launch_filter(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                         uint32_t nblocks, uint8_t* stream);
uint32_t filter_band_rows();
// PNG tiles with a Sub/Up/Avg/Paeth/adaptive filter and rows of whole dwords (<= 2 KiB,
// 16-byte aligned source): the same streams from dword-wide filter arithmetic (k_filter2).
hipError_t launch_filter2(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles, uint32_t nblocks,
                          uint32_t max_rb, uint8_t* stream);
uint32_t filter2_band_rows();
// PNG-filtered tiles with rows of whole 16-byte chunks (<= filter3_max_rb()): one wave per run
// of filter3_run_rows() rows, no LDS (k_filter3); nwaves = the runs of every tile; filter =
// the batch's PNG filter (1..4, 5 = adaptive), which every tile's d.filter holds
hipError_t launch_filter3(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles, uint32_t nwaves,
                          uint32_t max_rb, uint32_t filter, uint8_t* stream);
uint32_t filter3_run_rows(uint32_t filter);  // rows per wave for the PNG filter 1..5
// The adaptive option's tile mode, before the filter kernels: TF_ANONE of every adaptive PNG
// tile of d_tiles[0, ntiles) (one workgroup per tile; other tiles are left alone); max_rb: the
// widest of their rows in bytes.
hipError_t launch_adaptive_mode(hipStream_t st, TileDesc* d_tiles, uint32_t ntiles, uint32_t max_rb);
uint32_t filter3_max_rb();
uint32_t filter2_max_rb();

// K1+K2 for filter-None PNG rows and deflate-TIFF rows from 16-byte-aligned source rows:
// one workgroup per band of ROWS_BAND rows, staged in LDS, aligned 16-byte stream words.
constexpr uint32_t ROWS_BAND = 16;
constexpr uint32_t ROWS_MAX_RB = 8192;  // widest row (bytes) k_rows takes (LDS band <= 132 KB)
hipError_t launch_rows(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles, uint32_t nblocks,
                       uint32_t max_rb, uint8_t* stream);
inline uint32_t rows_blocks_for(uint32_t h) { return (h + ROWS_BAND - 1) / ROWS_BAND; }

// K3-K6: deflate of every tile's stream into its compacted container.
struct DeflateLaunch {
    const TileDesc* tiles;  // deflate tiles (seg_first / seg_count / out_off = stream offset)
    uint32_t ntiles, nseg;
    uint8_t* stream;        // filtered streams (16-byte aligned per tile, slack after); k_lz77
                            // writes those of TF_DIRECT tiles
    SegInfo* info;          // [nseg]
    uint32_t* hist;         // [nseg * HIST_WORDS]
    uint32_t* mrec;         // [nseg * MREC_WORDS]
    uint32_t* codes;        // [nblk * CODE_WORDS]
    BlkInfo* blk;           // [nblk] Huffman blocks
    uint32_t nblk;
    uint64_t* sizes;        // [ntiles] container bytes
    uint64_t* offs;         // [ntiles + 1] exclusive scan of sizes (offs[ntiles] = total)
    uint64_t* offs_host = nullptr;  // or a mapped pinned copy of offs, written by the scan
    uint8_t* out;           // compacted containers
    uint64_t* stamps;       // [nseg * 32] phase clocks (diagnostics) or nullptr
    uint32_t* seg_tile;     // [nseg] tile of every segment (k_seg_map)
    uint32_t cus = 256;     // compute units of the device (persistent grids)
    uint32_t uniform_nseg = 0;  // every tile has this many segments (tile = seg / it), or 0
    uint32_t uniform_rcp = 0;   // recip32(uniform_nseg)
    bool row_filtered = false;  // some tile's stream is PNG-row-filtered (k_lz77's VALU walk form)
};
// k_lz77, k_huff, k_seg_sizes + k_scan_offsets, k_encode, k_frame.
// ev[0..3] (and ev2[0..3] if given) are recorded after k_lz77, k_huff, k_scan_offsets, k_encode;
// with fine = false only ev[3] (the serving path's spans need no more).
hipError_t launch_deflate(hipStream_t st, const DeflateLaunch& a, hipEvent_t* ev = nullptr,
                          hipEvent_t* ev2 = nullptr, bool fine = true);
size_t deflate_lds_bytes(int kernel);  // 0 k_lz77, 1 k_huff, 2 k_encode
// k_huff alone (test hook): blk[].seg0 / .nseg and info[].sl / .last must be set.
hipError_t launch_huffman(hipStream_t st, uint32_t nblk, BlkInfo* blk, SegInfo* info,
                          const uint32_t* hist, uint32_t* codes);

// NGFF/Zarr chunk decode (kernels_zarr.hip).  One wave per stream.
enum : uint32_t { ZS_LZ4 = 0, ZS_ZLIB = 1, ZS_COPY = 2, ZS_BLOSCLZ = 3, ZS_ZSTD = 4, ZS_NKINDS = 5 };
struct ZStream {
    uint64_t src_off;  // compressed bytes in the uploaded chunk buffer
    uint64_t dst_off;  // decoded bytes in the scratch buffer
    uint32_t csize, dlen, kind, pad;
};
enum : uint32_t { ZC_MISSING = 1u, ZC_INPUT = 2u, ZC_BITSHUF = 4u };
struct ZChunk {
    uint64_t src;                         // decoded chunk: scratch offset (or input offset if ZC_INPUT)
    uint32_t nbytes, blocksize, typesize; // blosc geometry (typesize 1 = not byte-shuffled;
                                          // with ZC_BITSHUF the bit-shuffle element size)
    uint32_t flags;                       // ZC_*
    int32_t x0, y0;                       // chunk origin in the plane
    uint32_t plane, pad;                  // index into the ZPlane table of the launch
};
struct ZPlane {                           // a destination plane of one decode launch
    uint8_t* dev;
    int64_t pitch;
    int32_t sx, sy, cw, chh;              // plane and chunk shape
    uint32_t bpp, pad;
    uint64_t fill;                        // fill bytes in stored order (missing chunks)
};
// Streams ordered by kind (ZS_LZ4 | ZS_ZLIB | ZS_COPY | ZS_BLOSCLZ | ZS_ZSTD), counts[k] of
// kind k; err[i] = 0 or a decoder error code per stream.
// zstd_lit: zstd_scratch_bytes(counts[ZS_ZSTD]) bytes (a block's literals per zstd frame).
hipError_t launch_zarr_decode(hipStream_t st, const ZStream* d_streams, const uint32_t* counts,
                              const uint8_t* src, uint8_t* scratch, uint8_t* zstd_lit, uint32_t* err);
size_t zstd_scratch_bytes(uint32_t nstreams);
hipError_t launch_zarr_zstd(hipStream_t st, const ZStream* d_streams, uint32_t n, const uint8_t* src,
                            uint8_t* scratch, uint8_t* litbuf, uint32_t* err);
hipError_t launch_zarr_place(hipStream_t st, const ZChunk* d_chunks, uint32_t nchunks,
                             const ZPlane* d_planes, int32_t max_chunk_y, const uint8_t* scratch,
                             const uint8_t* input);

}  // namespace pbx
