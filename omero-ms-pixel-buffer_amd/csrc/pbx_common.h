// pbx_common.h — types and helpers shared by the HIP kernels, the host runtime and the
// test-only CPU emulator of the deflate phases.  Plain C++ (no HIP headers): PBX_HD is
// `__host__ __device__` under hipcc and empty under g++.
//
// Reference anchors (paths under /root/reference/src/main/java/com/glencoesoftware/omero/ms/pixelbuffer/):
//   getTileDirect -> TileStream::be()            TileRequestHandler.java:107-109 (big-endian, :155)
//   writeImage("png") -> PNG framing constants    TileRequestHandler.java:176-199 (APNGWriter upstream)
//   writeImage("tif") -> TIFF header              TileRequestHandler.java:176-199 (TiffWriter upstream)
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define PBX_HD __host__ __device__ __forceinline__
#else
#define PBX_HD inline
#endif

namespace pbx {

// ----------------------------------------------------------------------------------- formats
enum : int32_t { FMT_RAW = 0, FMT_PNG = 1, FMT_TIF = 2, FMT_UNKNOWN = 3 };
enum : int32_t { PT_INT8 = 0, PT_UINT8, PT_INT16, PT_UINT16, PT_INT32, PT_UINT32, PT_FLOAT,
                 PT_DOUBLE, PT_N };

// Tile flags
enum : uint32_t {
    TF_SWAP = 1u,      // plane samples are little-endian -> swap to big-endian
    TF_FLIP = 2u,      // PNG int8/int16: flip the sign bit of the MS byte (APNGWriter)
    TF_PNGROWS = 4u,   // stream rows carry a leading PNG filter-type byte
    TF_TIFF = 8u,      // container is TIFF (else PNG) for deflate tiles
    TF_DIRECT = 16u,   // filter-None rows, 16-byte aligned source, bpp <= 4: k_lz77
                       // assembles the stream from the plane (no k_rows pass)
    TF_TILED = 32u,    // one T x T sub-tile of a tiled-TIFF response (header by k_tiff_tiled)
    TF_ANONE = 64u,    // adaptive PNG tile whose rows all take filter None (the tile mode: set
                       // or cleared on the device by k_adaptive_mode every launch)
    TF_DIRECT_OK = 128u,  // adaptive PNG tile of TF_DIRECT's geometry: in the None mode
                          // k_adaptive_mode sets TF_DIRECT on it (no filter pass; k_lz77 reads
                          // its rows from the plane)
    TF_BRIDGE = 1u << 30,  // host only, cleared before upload: `plane` is an offset into the
                           // batch's bridge buffer (a region straddling sparse-plane bands)
};

// PNG container layout (APNGWriter: sig, IHDR, acTL, fcTL, IDAT, IEND).
constexpr uint32_t PNG_SIG_BYTES = 8;
constexpr uint32_t PNG_IHDR_BYTES = 12 + 13;
constexpr uint32_t PNG_ACTL_BYTES = 12 + 8;
constexpr uint32_t PNG_FCTL_BYTES = 12 + 26;
constexpr uint32_t PNG_IDAT_DATA_OFF =
    PNG_SIG_BYTES + PNG_IHDR_BYTES + PNG_ACTL_BYTES + PNG_FCTL_BYTES + 8;  // 99
constexpr uint32_t ZLIB_HDR_BYTES = 2;
constexpr uint32_t PNG_TAIL_BYTES = 4 /*adler*/ + 4 /*IDAT crc*/ + 12 /*IEND*/;
// TIFF: header + 11-entry IFD, strip data at a 16-byte aligned offset.
constexpr uint32_t TIFF_NTAGS = 11;
constexpr uint32_t TIFF_DATA_OFFSET = 160;

// Per-tile descriptor (device side).  64-byte aligned POD, filled by the host planner.
// Division by a divisor known ahead (a tile's row length, a batch's segments per tile)
// without the ~20-instruction integer division sequence: recip32(d) = floor((2^32-1) / d) + 1
// makes umulhi(n, recip) floor(n / d) or one more (the error n * r / (d 2^32) < 1 for every
// 32-bit n), and the sign of n - q d (|n - q d| < d < 2^31) corrects it, all in 32-bit scalar
// arithmetic.  d <= 1: recip 0 (n / 1 = n).
PBX_HD uint32_t recip32(uint32_t d) { return d > 1 ? (uint32_t)(0xFFFFFFFFull / d) + 1u : 0u; }
PBX_HD uint32_t div_rcp(uint32_t n, uint32_t d, uint32_t rcp) {
    if (!rcp) return d ? n : 0u;
    const uint32_t q = (uint32_t)(((uint64_t)n * rcp) >> 32);
    return (int32_t)(n - q * d) < 0 ? q - 1u : q;
}

struct alignas(16) TileDesc {
    const uint8_t* plane;   // plane base in HBM
    int64_t pitch;          // bytes per plane row
    int32_t x, y, w, h;     // region (post-defaulting)
    int32_t bpp, lbpp;      // bytes per sample and log2
    uint32_t flags;         // TF_*
    int32_t filter;         // PNG filter 0..4, 5 = per-row choice in rowfilt
    int32_t pixel_type;
    uint32_t rowlen;        // stream bytes per row: (png?1:0) + w*bpp
    uint64_t stream_len;    // h * rowlen
    uint64_t out_off;       // raw/tif: offset in the fixed arena; deflate: offset of the stream
    uint32_t seg_first;     // deflate tiles: first segment index in the batch
    uint32_t seg_count;
    uint32_t seg_len;       // nominal segment length (the last may be shorter)
    uint32_t rowlen_rcp;    // deflate tiles: recip32(rowlen), divisions by rowlen on the device
    uint32_t blk_first;     // first workgroup of this tile (extract / filter bands)
    uint32_t rows_per_blk;  // extract: rows handled by one workgroup
    uint32_t hblk_first;    // deflate tiles: first Huffman block index in the batch
    uint32_t vw, vh;        // tiled-TIFF edge sub-tile: valid w x h inside the padded w x h
                            // geometry (bytes outside read as 0); 0 = no padding
    uint32_t tiff_hdr;      // tiled TIFF: header bytes before this sub-tile's data (first
                            // sub-tile of a response only)
};

// Segments per Huffman block at most for a deflate tile (pbx_config.h BLK_SEGS*).
#define PBX_TILE_BLK_CAP(d) ((d).filter != 0 ? BLK_SEGS_FILTERED : BLK_SEGS)

// Per-segment deflate result.
struct SegOut {
    uint32_t nbytes;        // compressed bytes in the slot
    uint32_t crc;           // CRC-32 of those bytes (standard, zlib crc32 convention)
    uint32_t crc_op;        // x^(8*nbytes) mod P, for crc32_combine
    uint32_t adler_s1;      // sum of stream bytes mod 65521
    uint32_t adler_s2;      // sum of (len - i) * byte_i mod 65521
    uint32_t len;           // stream bytes in this segment
    uint32_t btype;         // 0 stored, 1 fixed, 2 dynamic
    uint32_t bits;          // bits of the block (diagnostics)
};

// Per-segment record of the three deflate kernels (80 bytes, in HBM).
struct SegInfo {
    uint32_t sl, last, wl, rowlen;       // k_lz77: geometry (last: the tile's final segment)
    uint32_t adler_s1, adler_s2;         // k_lz77: Adler-32 partial sums of the sl bytes
    uint32_t btype, hdr_bits;            // k_huff: its block's type and header bits
    uint32_t bit0, bit1;                 // k_huff: the segment's bits [bit0, bit1) of its block
    uint32_t crc, crc_op;                // k_encode: CRC-32 of the bytes it owns, x^(8*owned)
    uint32_t blk, flags;                 // k_seg_map: block index; SF_FIRST / SF_LAST in block
    uint32_t part;                       // k_encode: head | tail << 8 | SP_HEAD | SP_TAIL
    uint32_t bitsum;                     // k_encode: token bits (diagnostics)
    uint32_t tile;                       // k_seg_map: the segment's tile
    uint32_t src_lo, src_hi;             // k_lz77: stream-buffer offset of the segment's first byte
    uint32_t zoff;                       // k_seg_map: container bytes before the zlib stream
};
constexpr uint32_t SF_FIRST = 1, SF_LAST = 2, SF_TIFF = 4;
constexpr uint32_t SP_HEAD = 1u << 16, SP_TAIL = 1u << 17;

// Per Huffman block (BLK_SEGS consecutive segments of one tile share a code).
struct BlkInfo {
    uint32_t seg0, nseg;                 // k_seg_map
    uint32_t nbytes, data_bits;          // k_huff: block bytes; data bits (EOB included)
    uint32_t off;                        // k_seg_sizes: byte offset in the tile's zlib payload
    uint32_t fin;                        // k_huff: the tile's final block (BFINAL)
    uint32_t pad[2];
};

PBX_HD uint32_t ceil_div_u32(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

PBX_HD void put_be32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
PBX_HD void put_be16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

// TIFF SampleFormat: 1 unsigned, 2 signed, 3 IEEE float.
PBX_HD uint32_t tiff_sample_format(int32_t pt) {
    return (pt == PT_FLOAT || pt == PT_DOUBLE) ? 3u
           : (pt == PT_INT8 || pt == PT_INT16 || pt == PT_INT32) ? 2u : 1u;
}

// Classic big-endian ("MM") TIFF header + 11-entry IFD; one strip of nbytes at
// TIFF_DATA_OFFSET (TiffWriter with PixelsBigEndian=true, TileRequestHandler.java:155,182-186).
// Writes exactly TIFF_DATA_OFFSET bytes.
PBX_HD void write_tiff_header(uint8_t* p, uint32_t w, uint32_t h, uint32_t bpp, uint32_t sf,
                              uint32_t compression, uint32_t nbytes) {
    for (uint32_t i = 0; i < TIFF_DATA_OFFSET; i++) p[i] = 0;
    p[0] = 'M'; p[1] = 'M'; put_be16(p + 2, 42); put_be32(p + 4, 8);
    put_be16(p + 8, TIFF_NTAGS);
    const uint16_t tag[TIFF_NTAGS] = {256, 257, 258, 259, 262, 273, 277, 278, 279, 284, 339};
    const uint16_t typ[TIFF_NTAGS] = {4, 4, 3, 3, 3, 4, 3, 4, 4, 3, 3};
    const uint32_t val[TIFF_NTAGS] = {w, h, 8 * bpp, compression, 1, TIFF_DATA_OFFSET, 1, h, nbytes, 1, sf};
    for (uint32_t k = 0; k < TIFF_NTAGS; k++) {
        uint8_t* e = p + 10 + 12 * k;
        put_be16(e, tag[k]); put_be16(e + 2, typ[k]); put_be32(e + 4, 1);
        if (typ[k] == 3) { put_be16(e + 8, val[k]); } else { put_be32(e + 8, val[k]); }
    }
    // next-IFD offset (0) is already zero
}

// Tiled TIFF (TIFF 6.0 section 15): header + 12-entry IFD at 8 (ends at 158); with n > 1
// sub-tiles the TileOffsets array at 160 and TileByteCounts at 160 + 4n; sub-tile data from
// the 16-byte aligned offset tiff_tiled_data_offset(n), row-major over the region, every
// sub-tile T x T samples (edge sub-tiles zero-padded), raw or one zlib stream each.
constexpr uint32_t TIFF_TILED_NTAGS = 12;
constexpr uint32_t TIFF_TILED_ARRAYS = 160;

PBX_HD uint64_t tiff_tiled_data_offset(uint64_t n) {
    return n > 1 ? (TIFF_TILED_ARRAYS + 8 * n + 15) & ~15ull : TIFF_TILED_ARRAYS;
}

// Header and IFD (bytes [0, 160)); for n == 1 the one offset / byte count sit in the entries,
// else the caller writes tiff_tiled_entry(k) for every sub-tile.
PBX_HD void write_tiff_tiled_ifd(uint8_t* p, uint32_t w, uint32_t h, uint32_t t, uint32_t bpp,
                                 uint32_t sf, uint32_t compression, uint32_t n, uint32_t off0,
                                 uint32_t cnt0) {
    for (uint32_t i = 0; i < TIFF_TILED_ARRAYS; i++) p[i] = 0;
    p[0] = 'M'; p[1] = 'M'; put_be16(p + 2, 42); put_be32(p + 4, 8);
    put_be16(p + 8, TIFF_TILED_NTAGS);
    const uint16_t tag[TIFF_TILED_NTAGS] = {256, 257, 258, 259, 262, 277, 284, 322, 323, 324, 325, 339};
    const uint16_t typ[TIFF_TILED_NTAGS] = {4, 4, 3, 3, 3, 3, 3, 4, 4, 4, 4, 3};
    const uint32_t val[TIFF_TILED_NTAGS] = {w, h, 8 * bpp, compression, 1, 1, 1, t, t,
                                            n > 1 ? TIFF_TILED_ARRAYS : off0,
                                            n > 1 ? TIFF_TILED_ARRAYS + 4 * n : cnt0, sf};
    for (uint32_t k = 0; k < TIFF_TILED_NTAGS; k++) {
        uint8_t* e = p + 10 + 12 * k;
        put_be16(e, tag[k]); put_be16(e + 2, typ[k]);
        put_be32(e + 4, (tag[k] == 324 || tag[k] == 325) ? n : 1u);
        if (typ[k] == 3) { put_be16(e + 8, val[k]); } else { put_be32(e + 8, val[k]); }
    }
}

// Sub-tile k's TileOffsets / TileByteCounts entries (n > 1).
PBX_HD void tiff_tiled_entry(uint8_t* p, uint32_t n, uint32_t k, uint32_t off, uint32_t cnt) {
    put_be32(p + TIFF_TILED_ARRAYS + 4 * k, off);
    put_be32(p + TIFF_TILED_ARRAYS + 4 * n + 4 * k, cnt);
}

// A tiled-TIFF response's header job (k_tiff_tiled).  comp 1: the response starts at `off`
// in the fixed arena and every sub-tile is t*t*bpp bytes; comp 8: its sub-tiles are deflate
// tiles first..first+n-1 and the response starts at their first container.
struct alignas(16) TiledHdr {
    uint64_t off;
    uint32_t first, n, w, h, t, bpp, sf, comp;
};

// ----------------------------------------------------------------------------- CRC-32 math
// Standard reflected CRC-32 (poly 0xEDB88320) with zlib's crc32_combine formulation:
// crc(A||B) = multmodp(x^(8|B|), crc(A)) ^ crc(B).
constexpr uint32_t CRC_POLY = 0xEDB88320u;

// a(x) * b(x) mod P for reflected 32-bit polynomials (zlib multmodp), branch-free.
PBX_HD uint32_t crc_multmodp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int i = 31; i >= 0; i--) {
        p ^= ((a >> i) & 1u) ? b : 0u;
        b = (b >> 1) ^ ((b & 1u) ? CRC_POLY : 0u);
    }
    return p;
}

constexpr uint32_t crc_multmodp_c(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int i = 31; i >= 0; i--) {
        if ((a >> i) & 1u) p ^= b;
        b = (b >> 1) ^ ((b & 1u) ? CRC_POLY : 0u);
    }
    return p;
}

// X8.v[k] = x^(8 * 2^k) mod P: the operator that appends 2^k zero bytes.
struct X8Table { uint32_t v[40]; };
constexpr X8Table make_x8() {
    X8Table t{};
    uint32_t p = 1u << 30;  // x^1
    p = crc_multmodp_c(p, p);
    p = crc_multmodp_c(p, p);
    p = crc_multmodp_c(p, p);  // x^8
    t.v[0] = p;
    for (int k = 1; k < 40; k++) t.v[k] = crc_multmodp_c(t.v[k - 1], t.v[k - 1]);
    return t;
}

// x^(8n) mod P (zlib x2nmodp(n, 3)), from compile-time constants.
PBX_HD uint32_t crc_x8n(uint64_t n) {
    constexpr X8Table t = make_x8();
    uint32_t p = 1u << 31;  // x^0
#pragma unroll
    for (int k = 0; k < 32; k++)
        if ((n >> k) & 1u) p = crc_multmodp(t.v[k], p);
    return p;
}

// Operator of 2^k zero bytes (k < 40), folded to a constant when k is.
PBX_HD uint32_t crc_x8pow2(int k) {
    constexpr X8Table t = make_x8();
    return t.v[k];
}

PBX_HD uint32_t crc_combine_op(uint32_t crc1, uint32_t crc2, uint32_t op2) {
    return crc_multmodp(op2, crc1) ^ crc2;
}

// c * x^4 mod P in one step: P's five low bits are zero, so the four bits shifted out decide
// alone (a chain of ~3 dependent operations instead of 4 x 3).  Latency forms for the
// single-request path (k_frame_wave); equal to crc_multmodp / the bitwise update.
PBX_HD uint32_t crc_x4(uint32_t c) {
    return (c >> 4) ^ ((c & 1u) ? (CRC_POLY >> 3) : 0u) ^ ((c & 2u) ? (CRC_POLY >> 2) : 0u) ^
           ((c & 4u) ? (CRC_POLY >> 1) : 0u) ^ ((c & 8u) ? CRC_POLY : 0u);
}
// a(x) * b(x) mod P by Horner over a's nibbles, highest powers first (b x^0..x^3 up front).
PBX_HD uint32_t crc_multmodp4(uint32_t a, uint32_t b) {
    const uint32_t b1 = (b >> 1) ^ ((b & 1u) ? CRC_POLY : 0u);
    const uint32_t b2 = (b >> 2) ^ ((b & 1u) ? (CRC_POLY >> 1) : 0u) ^ ((b & 2u) ? CRC_POLY : 0u);
    const uint32_t b3 = (b >> 3) ^ ((b & 1u) ? (CRC_POLY >> 2) : 0u) ^ ((b & 2u) ? (CRC_POLY >> 1) : 0u) ^
                        ((b & 4u) ? CRC_POLY : 0u);
    uint32_t p = 0;
#pragma unroll
    for (int s = 7; s >= 0; s--) {  // powers 4s .. 4s+3 <-> bits 31-4s .. 28-4s of a
        const uint32_t t = ((a >> (31 - 4 * s)) & 1u ? b : 0u) ^ ((a >> (30 - 4 * s)) & 1u ? b1 : 0u) ^
                           ((a >> (29 - 4 * s)) & 1u ? b2 : 0u) ^ ((a >> (28 - 4 * s)) & 1u ? b3 : 0u);
        p = crc_x4(p) ^ t;
    }
    return p;
}
// one byte into a (raw, reflected) CRC register
PBX_HD uint32_t crc_byte4(uint32_t c, uint32_t b) { return crc_x4(crc_x4(c ^ (b & 0xFFu))); }

// Bytewise CRC with a caller-provided 256-entry table (LDS on the device).
PBX_HD uint32_t crc_update(const uint32_t* table, uint32_t crc, uint8_t b) {
    return table[(crc ^ b) & 0xFF] ^ (crc >> 8);
}

PBX_HD uint32_t crc_table_entry(uint32_t n) {
    uint32_t c = n;
    for (int k = 0; k < 8; k++) c = (c & 1) ? CRC_POLY ^ (c >> 1) : c >> 1;
    return c;
}

// --------------------------------------------------------------------------- Adler-32 math
constexpr uint32_t ADLER_BASE = 65521u;

// Combine raw partial sums (s1 = sum b, s2 = sum (n-i) b) of L (left) and R (right, lenR bytes).
PBX_HD void adler_combine(uint32_t& s1L, uint32_t& s2L, uint32_t s1R, uint32_t s2R, uint64_t lenR) {
    // (all sums < ADLER_BASE: s2L + lr * s1L + s2R < 2^32, so 32-bit arithmetic suffices)
    const uint32_t lr = lenR < ADLER_BASE ? (uint32_t)lenR : (uint32_t)(lenR % ADLER_BASE);
    const uint32_t s2 = s2L + lr * s1L + s2R, s1 = s1L + s1R;
    s1L = s1 >= ADLER_BASE ? s1 - ADLER_BASE : s1;
    s2L = s2 % ADLER_BASE;
}

// Final adler32 value for a stream of total length n with raw sums s1, s2.
PBX_HD uint32_t adler_final(uint32_t s1, uint32_t s2, uint64_t n) {
    uint32_t a = (uint32_t)((1 + (uint64_t)s1) % ADLER_BASE);
    uint32_t b = (uint32_t)(((uint64_t)(n % ADLER_BASE) + s2) % ADLER_BASE);
    return (b << 16) | a;
}

// ---------------------------------------------------------------------- deflate code maps
// Length 3..258 -> symbol 257..285 and extra bits.
PBX_HD uint32_t ilog2_u32(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

PBX_HD void len_code(uint32_t len, uint32_t& sym, uint32_t& ebits, uint32_t& eval) {
    uint32_t l = len - 3;
    if (len == 258) { sym = 285; ebits = 0; eval = 0; return; }
    if (l < 8) { sym = 257 + l; ebits = 0; eval = 0; return; }
    uint32_t e = ilog2_u32(l) - 2;
    sym = 261 + 4 * e + (l >> e) - 4;
    ebits = e;
    eval = l & ((1u << e) - 1);
}

// Distance 1..32768 -> symbol 0..29 and extra bits.
PBX_HD void dist_code(uint32_t dist, uint32_t& sym, uint32_t& ebits, uint32_t& eval) {
    uint32_t d = dist - 1;
    if (d < 4) { sym = d; ebits = 0; eval = 0; return; }
    uint32_t e = ilog2_u32(d) - 1;
    sym = 2 * e + 2 + ((d >> e) & 1);
    ebits = e;
    eval = d & ((1u << e) - 1);
}

PBX_HD uint32_t len_sym_ebits(uint32_t sym) {
    if (sym < 265 || sym == 285) return 0;
    return (sym - 261) / 4;
}
PBX_HD uint32_t dist_sym_ebits(uint32_t sym) { return sym < 4 ? 0 : sym / 2 - 1; }

PBX_HD uint32_t fixed_lit_len(uint32_t sym) {
    return sym < 144 ? 8 : sym < 256 ? 9 : sym < 280 ? 7 : 8;
}

PBX_HD uint32_t bitrev(uint32_t code, uint32_t len) {
    uint32_t r = 0;
    for (uint32_t i = 0; i < len; i++) { r = (r << 1) | (code & 1); code >>= 1; }
    return r;
}

// ----------------------------------------------------------------------- tile byte source
// The byte stream a deflate segment reads: for PNG, h rows of (filter byte || filtered
// big-endian row); for deflate-TIFF, the big-endian tile bytes.  Reads the plane in HBM
// directly (getTileDirect fused with the filter: no intermediate tile buffer).
struct TileStream {
    const uint8_t* plane;
    int64_t pitch;
    int32_t x, y, bpp, lbpp;
    uint32_t rowlen, flags;
    int32_t filter;
    const uint8_t* rowfilt;
    uint32_t vrb, vh;  // valid row bytes / rows (tiled-TIFF edge sub-tiles; else unbounded)

    PBX_HD void init(const TileDesc& d, const uint8_t* rowfilt_base) {
        plane = d.plane; pitch = d.pitch; x = d.x; y = d.y; bpp = d.bpp; lbpp = d.lbpp;
        rowlen = d.rowlen; flags = d.flags; filter = d.filter;
        rowfilt = rowfilt_base;
        vrb = d.vw ? d.vw * (uint32_t)d.bpp : 0xFFFFFFFFu;
        vh = d.vw ? d.vh : 0xFFFFFFFFu;
    }
    // Big-endian byte i of tile row r, after the APNGWriter sign flip; 0 in the padding of
    // a tiled-TIFF edge sub-tile.
    PBX_HD uint32_t be(int64_t r, uint32_t i) const {
        if ((uint64_t)r >= vh || i >= vrb) return 0u;
        uint32_t s = i >> lbpp, b = i & (uint32_t)(bpp - 1);
        uint32_t sb = (flags & TF_SWAP) ? (uint32_t)(bpp - 1) - b : b;
        uint32_t v = plane[(int64_t)(y + r) * pitch + ((int64_t)x + s) * bpp + sb];
        if ((flags & TF_FLIP) && b == 0) v ^= 0x80u;
        return v;
    }
    PBX_HD int row_filter(int64_t r) const {
        return filter == 5 ? (int)rowfilt[r] : filter;
    }
    PBX_HD uint32_t filtered(int ft, int64_t r, uint32_t i) const {
        uint32_t cur = be(r, i);
        if (ft == 0) return cur;
        uint32_t left = i >= (uint32_t)bpp ? be(r, i - bpp) : 0u;
        uint32_t up = r > 0 ? be(r - 1, i) : 0u;
        if (ft == 1) return (cur - left) & 0xFF;
        if (ft == 2) return (cur - up) & 0xFF;
        if (ft == 3) return (cur - ((left + up) >> 1)) & 0xFF;
        uint32_t ul = (r > 0 && i >= (uint32_t)bpp) ? be(r - 1, i - bpp) : 0u;
        int p = (int)left + (int)up - (int)ul;
        int pa = p - (int)left, pb = p - (int)up, pc = p - (int)ul;
        pa = pa < 0 ? -pa : pa; pb = pb < 0 ? -pb : pb; pc = pc < 0 ? -pc : pc;
        uint32_t pr = (pa <= pb && pa <= pc) ? left : (pb <= pc ? up : ul);
        return (cur - pr) & 0xFF;
    }
    // Byte at (row r, column col) of the stream.
    PBX_HD uint32_t at(int64_t r, uint32_t col) const {
        if (flags & TF_PNGROWS) {
            int ft = row_filter(r);
            if (col == 0) return (uint32_t)ft;
            return filtered(ft, r, col - 1);
        }
        return be(r, col);
    }
    // Up to 4 stream bytes starting at stream position p0, packed little-endian.
    PBX_HD uint32_t fill_word(uint64_t p0, uint32_t nb) const {
        uint32_t p = (uint32_t)p0;  // tiles are < 2^31 bytes (TileRequestHandler.java:102)
        uint32_t r = p / rowlen, col = p - r * rowlen, v = 0;
        for (uint32_t b = 0; b < nb; b++) {
            v |= at(r, col) << (8 * b);
            if (++col == rowlen) { col = 0; r++; }
        }
        return v;
    }
};

// A stream in HBM whose words are read at 4-byte aligned offsets (segment starts and the
// window are multiples of 16; the buffer has slack after every tile).
struct WordStream {
    const uint8_t* p;
    PBX_HD uint32_t fill_word(uint64_t p0, uint32_t nb) const {
        const uint32_t v = *(const uint32_t*)(p + p0);
        return nb >= 4 ? v : v & ((1u << (8 * nb)) - 1u);
    }
};

// A stream already in memory (deflate-only callers and the CPU emulator).
struct MemStream {
    const uint8_t* p;
    PBX_HD uint32_t fill_word(uint64_t p0, uint32_t nb) const {
        uint32_t v = 0;
        for (uint32_t b = 0; b < nb; b++) v |= (uint32_t)p[p0 + b] << (8 * b);
        return v;
    }
};

// ------------------------------------------------------------------- synthetic planes
// G_FAKE: Bio-Formats FakeReader.openBytes (pixel = typeMin + x; rows y < 10 carry
// {series=0, planeNo, z, c, t} in 10-pixel boxes).  G_NOISE: SURVEY.md §8(d) counter-hash
// noise (12-bit-like 257..1486).  Returns the sample's bit pattern.
enum : int32_t { GEN_FAKE = 1, GEN_NOISE = 2 };

PBX_HD uint64_t splitmix64(uint64_t k) {
    uint64_t z = k + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

PBX_HD uint64_t cast_sample(int32_t pt, int64_t v) {
    switch (pt) {
    case PT_INT8: case PT_UINT8: return (uint64_t)v & 0xFFull;
    case PT_INT16: case PT_UINT16: return (uint64_t)v & 0xFFFFull;
    case PT_INT32: case PT_UINT32: return (uint64_t)v & 0xFFFFFFFFull;
    case PT_FLOAT: { float f = (float)v; return (uint64_t)__builtin_bit_cast(uint32_t, f); }
    default: { double d = (double)v; return __builtin_bit_cast(uint64_t, d); }
    }
}

PBX_HD uint64_t gen_sample(int32_t kind, uint64_t seed, int32_t plane_no, int32_t z, int32_t c,
                           int32_t t, int32_t pt, int64_t x, int64_t y) {
    if (kind == GEN_FAKE) {
        int64_t v = (pt == PT_INT8 ? -128 : pt == PT_INT16 ? -32768 : pt == PT_INT32 ? -2147483648LL : 0) + x;
        if (y < 10) {
            int64_t box = x / 10;
            if (box == 0) v = 0;
            else if (box == 1) v = plane_no;
            else if (box == 2) v = z;
            else if (box == 3) v = c;
            else if (box == 4) v = t;
        }
        return cast_sample(pt, v);
    }
    uint64_t k = (seed << 48) ^ ((uint64_t)(uint32_t)plane_no << 40) ^ ((uint64_t)y << 20) ^ (uint64_t)x;
    uint64_t r = splitmix64(k);
    int64_t v = 256 + (((x >> 5) + (y >> 5)) % 16) * 48 + (int64_t)(r & 0xFF) + (int64_t)((r >> 8) & 0xFF);
    return cast_sample(pt, v);
}

}  // namespace pbx
