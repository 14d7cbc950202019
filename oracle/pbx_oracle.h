/*
 * pbx_oracle — CPU restatement of the omero-ms-pixel-buffer /tile hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline).  The product library (libpbx.so) never links,
 * loads or calls it.
 *
 * Parity status: the reference (Java, /root/reference) has no tests, no golden
 * vectors and cannot be built or run here (no JDK, no Maven cache, no
 * network).  Its arithmetic lives in third-party jars (Bio-Formats APNGWriter /
 * TiffWriter, OMERO PixelBuffer, java.util.zip.Deflater = zlib).  This oracle
 * restates the reference call sites and the four upstream facts SURVEY.md §8(a)
 * lists; it is pinned by independent decoders (PIL for PNG, tifffile for TIFF)
 * and an independent numpy restatement of the generators (tests/golden/).
 * "Parity unpinned by the reference" — see DESIGN.md §Oracle.
 */
#ifndef PBX_ORACLE_H
#define PBX_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* OMERO pixel types (ome.xml.model.enums.PixelType names). Same numbering as include/pbx.h. */
enum { PBXO_INT8 = 0, PBXO_UINT8, PBXO_INT16, PBXO_UINT16, PBXO_INT32, PBXO_UINT32,
       PBXO_FLOAT, PBXO_DOUBLE, PBXO_NTYPES };
/* Output formats: TileCtx.format null / "png" / "tif" / anything else. */
enum { PBXO_FMT_RAW = 0, PBXO_FMT_PNG = 1, PBXO_FMT_TIF = 2, PBXO_FMT_UNKNOWN = 3 };
/* Synthetic plane generators. */
enum { PBXO_GEN_FAKE = 1, PBXO_GEN_NOISE = 2 };
/* Status codes = the HTTP status the reference ends with (PixelBufferVerticle.java:111-146). */
enum { PBXO_OK = 0, PBXO_E_BADARG = 400, PBXO_E_NOTFOUND = 404, PBXO_E_INTERNAL = 500 };

int pbxo_bpp(int pixel_type);
int pbxo_is_signed_int(int pixel_type);

/* One sample of a synthetic plane, as its raw bit pattern (zero-extended). */
uint64_t pbxo_gen_sample(int kind, uint64_t seed, int plane_no, int z, int c, int t,
                         int pixel_type, int64_t x, int64_t y);
/* Fill a w x h region (origin x0,y0) of a synthetic plane; big_endian selects the
 * byte order of the samples written to out (w*h*bpp bytes, row-major). */
void pbxo_gen_region(int kind, uint64_t seed, int plane_no, int z, int c, int t,
                     int pixel_type, int64_t x0, int64_t y0, int32_t w, int32_t h,
                     int big_endian, uint8_t* out);

/* PixelBuffer.getTileDirect semantics (TileRequestHandler.java:107-109): copy rows
 * y..y+h-1, cols x..x+w-1 of a plane into a row-major tile with BIG-ENDIAN samples.
 * plane_big_endian gives the byte order the plane is stored in. */
void pbxo_extract_be(const uint8_t* plane, int plane_big_endian, int pixel_type,
                     int64_t pitch_bytes, int32_t x, int32_t y, int32_t w, int32_t h,
                     uint8_t* out);

/* PNG filtered stream for a big-endian tile: h rows of (filter byte || row), with the
 * APNGWriter int8/int16 sign-bit flip.  filter: 0..4 fixed, 5 = adaptive (per tile: None on
 * every row when its middle row says filtering does not pay -- pbxo_adaptive_tile_none --
 * else per row the minimum sum of |byte - prediction|).  Returns bytes written (h*(1+w*bpp)). */
size_t pbxo_png_filter_stream(const uint8_t* tile_be, int pixel_type, int32_t w, int32_t h,
                              int filter, uint8_t* out);
/* The adaptive option's tile mode: 1 when the tile's rows all take filter None. */
int pbxo_adaptive_tile_none(const uint8_t* tile_be, int pixel_type, int32_t w, int32_t h);

/* Encoders.  Return PBXO_OK or PBXO_E_NOTFOUND (unsupported type -> getTile returns null).
 * *len receives the exact output length (TileRequestHandler.java:188-193). */
int pbxo_png_encode(const uint8_t* tile_be, int pixel_type, int32_t w, int32_t h,
                    int zlib_level, uint8_t* out, size_t cap, size_t* len);
int pbxo_tiff_encode(const uint8_t* tile_be, int pixel_type, int32_t w, int32_t h,
                     uint8_t* out, size_t cap, size_t* len);
size_t pbxo_png_max_size(int pixel_type, int32_t w, int32_t h);
size_t pbxo_tiff_size(int pixel_type, int32_t w, int32_t h);
/* Tiled TIFF of t x t tiles (t a multiple of 16; edge tiles zero-padded), compression 1
 * or 8 (zlib level 6 per tile), in the layout the tiled-TIFF option of the pipeline writes
 * (not part of the reference: its TiffWriter writes one strip). */
int pbxo_tiff_tiled_write(const uint8_t* tile_be, int32_t w, int32_t h, int32_t bpp, int32_t sf,
                          int32_t t, int32_t comp, uint8_t* out, size_t cap, size_t* len);

/* TileRequestHandler.getTile (TileRequestHandler.java:80-139) over one registered plane.
 * The plane is the whole (z,c,t) plane of an image of size_x x size_y.  Region w/h == 0
 * default to the plane size (:92-97).  Writes the response body; out_w and out_h receive
 * the post-defaulting region (used by the filename header). */
int pbxo_get_tile(const uint8_t* plane, int plane_big_endian, int pixel_type,
                  int32_t size_x, int32_t size_y, int32_t x, int32_t y, int32_t w, int32_t h,
                  int format, uint8_t* out, size_t cap, size_t* len,
                  int32_t* out_w, int32_t* out_h);

/* Decoders (independent of the encoders above; used to check GPU output). */
/* PNG: verifies signature and every chunk CRC, inflates IDAT, unfilters all 5 filter
 * types.  Writes big-endian samples (as stored in the PNG).  Returns 0 on success. */
int pbxo_png_decode(const uint8_t* png, size_t len, uint8_t* out, size_t cap,
                    int32_t* w, int32_t* h, int32_t* bit_depth, int32_t* color_type);
/* Inflate the concatenated IDAT payload: the filtered stream.  Returns 0 on success. */
int pbxo_png_inflate_idat(const uint8_t* png, size_t len, uint8_t* out, size_t cap,
                          size_t* out_len);
/* Baseline TIFF ("MM" or "II"), compression 1 or 8 (zlib), any strip layout or tiled
 * (TileWidth/TileLength/TileOffsets/TileByteCounts).  Writes samples in the file's byte
 * order.  Returns 0 on success. */
int pbxo_tiff_decode(const uint8_t* tif, size_t len, uint8_t* out, size_t cap,
                     int32_t* w, int32_t* h, int32_t* bits, int32_t* sample_format,
                     int32_t* compression, int32_t* big_endian);

/* zlib-format stream of the given bytes at a level (java.util.zip.Deflater semantics). */
int pbxo_zlib_compress(const uint8_t* in, size_t n, int level, uint8_t* out, size_t cap,
                       size_t* out_len);
int pbxo_zlib_inflate(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);
uint32_t pbxo_crc32(uint32_t crc, const uint8_t* p, size_t n);
uint32_t pbxo_adler32(uint32_t adler, const uint8_t* p, size_t n);

/* Response metadata (PixelBufferVerticle.java:118-126, PixelBufferMicroserviceVerticle.java:373-379). */
int pbxo_tile_filename(int64_t image_id, int32_t z, int32_t c, int32_t t, int32_t x, int32_t y,
                       int32_t w, int32_t h, const char* format, char* out, size_t cap);
const char* pbxo_content_type(const char* format);

/* CPU baseline: encode `tiles` tiles of w x h from a synthetic plane (generator kind,
 * pixel_type) to `format` on `threads` POSIX threads.  Tiles walk a grid on a plane of
 * plane_w x plane_h.  Returns wall seconds; *out_bytes receives the total output bytes. */
double pbxo_bench(int kind, int pixel_type, int format, int32_t plane_w, int32_t plane_h,
                  int32_t w, int32_t h, int tiles, int threads, uint64_t* out_bytes);
/* One request (x0, y0, w, h) of the plane `reps` times (BASELINE configs[0]). */
double pbxo_bench_at(int kind, int pt, int format, int32_t pw, int32_t ph, int32_t x0, int32_t y0,
                     int32_t w, int32_t h, int reps, int threads, uint64_t* out_bytes);

/* Zarr v2 chunk decode (oracle/zarr_oracle.c).  Codecs = include/pbx.h
 * enum pbx_zarr_codec. */
enum { PBXO_ZARR_RAW = 0, PBXO_ZARR_BLOSC = 1, PBXO_ZARR_ZLIB = 2 };
int pbxo_lz4_decode(const uint8_t* in, size_t ilen, uint8_t* out, size_t olen);
int pbxo_blosclz_decode(const uint8_t* in, size_t ilen, uint8_t* out, size_t olen);
/* -2 when the system libzstd cannot be loaded */
int pbxo_zstd_decode(const uint8_t* in, size_t ilen, uint8_t* out, size_t olen);
int pbxo_blosc_info(const uint8_t* in, size_t len, uint32_t* nbytes, uint32_t* blocksize,
                    uint32_t* typesize, uint32_t* flags);
int pbxo_blosc_decode(const uint8_t* in, size_t len, uint8_t* out, size_t cap, size_t* out_len);
int pbxo_zarr_decode_chunk(int codec, const uint8_t* in, size_t len, uint8_t* out, size_t nbytes);
/* Assemble a plane (row-major, size_x*bpp bytes per row) from the C-order chunk grid:
 * chunk i's bytes are data[offsets[i] .. offsets[i+1]); an empty range is a missing chunk
 * (every sample = the bpp bytes at fill).  Returns 0 on success. */
int pbxo_zarr_plane(int codec, int bpp, int32_t size_x, int32_t size_y, int32_t chunk_x,
                    int32_t chunk_y, const uint8_t* data, const uint64_t* offsets,
                    const uint8_t* fill, uint8_t* plane);
/* CPU baseline: decode every chunk on `threads` threads; returns wall seconds (-1 on error). */
double pbxo_zarr_bench(int codec, const uint8_t* data, const uint64_t* offsets, size_t nchunks,
                       size_t chunk_bytes, int threads);

#ifdef __cplusplus
}
#endif
#endif
