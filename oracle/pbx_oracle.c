/*
 * pbx_oracle.c — CPU restatement of the /tile hot path of omero-ms-pixel-buffer.
 *
 * TEST INFRASTRUCTURE ONLY (see pbx_oracle.h).  Never linked into libpbx.so.
 *
 * What it restates (all file:line citations are into /root/reference,
 * src/main/java/com/glencoesoftware/omero/ms/pixelbuffer/):
 *   - TileRequestHandler.getTile            TileRequestHandler.java:80-139
 *       w/h == 0 -> full plane size          :92-97
 *       bpp = bitSize/8, tileSize int math   :100-103
 *       getTileDirect (big-endian samples)   :104-112, :155
 *       format null -> raw; png|tif -> writeImage; else null (404)   :119-128
 *       any exception -> null (404)          :133-138
 *   - createMetadata (BigEndian, gray, 1 sample, Z=C=T=1)            :145-170
 *   - writeImage by extension (ImageWriter -> APNGWriter / TiffWriter) :176-199
 *   - filename header / content type   PixelBufferVerticle.java:118-126,
 *                                      PixelBufferMicroserviceVerticle.java:373-379
 * Upstream (third-party, absent from /root/reference) facts restated, per SURVEY.md §8(a):
 *   1. raw tiles are big-endian;  2. APNGWriter flips the sign bit of int8/int16;
 *   3. APNGWriter rejects 32/64-bit types (-> exception -> 404);
 *   4. TiffWriter stores samples verbatim (uncompressed, "MM").
 * PNG = APNGWriter layout: signature, IHDR, acTL(1 frame), fcTL, IDAT, IEND; every
 * scanline filter byte 0 (None); zlib level 6 (java.util.zip.Deflater default -1 == 6).
 * zlib here is the system zlib 1.2.11 (the same algorithm the JDK binds).
 */
#include "pbx_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <zlib.h>

int pbxo_bpp(int pt) {
    switch (pt) {
    case PBXO_INT8: case PBXO_UINT8: return 1;
    case PBXO_INT16: case PBXO_UINT16: return 2;
    case PBXO_INT32: case PBXO_UINT32: case PBXO_FLOAT: return 4;
    case PBXO_DOUBLE: return 8;
    default: return 0;
    }
}

int pbxo_is_signed_int(int pt) {
    return pt == PBXO_INT8 || pt == PBXO_INT16 || pt == PBXO_INT32;
}

/* ------------------------------------------------------------------ generators */

static uint64_t splitmix64(uint64_t k) {
    uint64_t z = k + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint64_t cast_to_type(int pt, int64_t v) {
    union { float f; uint32_t u; } fu;
    union { double d; uint64_t u; } du;
    switch (pt) {
    case PBXO_INT8: case PBXO_UINT8: return (uint64_t)v & 0xFFull;
    case PBXO_INT16: case PBXO_UINT16: return (uint64_t)v & 0xFFFFull;
    case PBXO_INT32: case PBXO_UINT32: return (uint64_t)v & 0xFFFFFFFFull;
    case PBXO_FLOAT: fu.f = (float)v; return fu.u;
    case PBXO_DOUBLE: du.d = (double)v; return du.u;
    default: return 0;
    }
}

/* G_FAKE follows Bio-Formats FakeReader.openBytes: pixel = typeMin + x, truncated to the
 * type; rows y < 10 carry {series=0, planeNo, z, c, t} in 10-pixel boxes (x/10 = 0..4).
 * G_NOISE: SURVEY.md §8(d) counter-hash noise, 12-bit-like values 257..1486. */
uint64_t pbxo_gen_sample(int kind, uint64_t seed, int plane_no, int z, int c, int t,
                         int pt, int64_t x, int64_t y) {
    if (kind == PBXO_GEN_FAKE) {
        int64_t mn = 0;
        if (pt == PBXO_INT8) mn = -128;
        else if (pt == PBXO_INT16) mn = -32768;
        else if (pt == PBXO_INT32) mn = -2147483648LL;
        int64_t v = mn + x;
        if (y < 10) {
            switch (x / 10) {
            case 0: v = 0; break;
            case 1: v = plane_no; break;
            case 2: v = z; break;
            case 3: v = c; break;
            case 4: v = t; break;
            default: break;
            }
        }
        return cast_to_type(pt, v);
    }
    /* G_NOISE */
    uint64_t k = (seed << 48) ^ ((uint64_t)plane_no << 40) ^ ((uint64_t)y << 20) ^ (uint64_t)x;
    uint64_t r = splitmix64(k);
    int64_t v = 256 + (int64_t)(((x >> 5) + (y >> 5)) % 16) * 48 + (int64_t)(r & 0xFF) +
                (int64_t)((r >> 8) & 0xFF);
    return cast_to_type(pt, v);
}

static void put_sample(uint8_t* p, uint64_t v, int bpp, int big_endian) {
    for (int b = 0; b < bpp; b++) {
        uint8_t byte = (uint8_t)(v >> (8 * b));
        if (big_endian) p[bpp - 1 - b] = byte; else p[b] = byte;
    }
}

void pbxo_gen_region(int kind, uint64_t seed, int plane_no, int z, int c, int t, int pt,
                     int64_t x0, int64_t y0, int32_t w, int32_t h, int big_endian, uint8_t* out) {
    int bpp = pbxo_bpp(pt);
    for (int32_t yy = 0; yy < h; yy++)
        for (int32_t xx = 0; xx < w; xx++) {
            uint64_t v = pbxo_gen_sample(kind, seed, plane_no, z, c, t, pt, x0 + xx, y0 + yy);
            put_sample(out + ((size_t)yy * w + xx) * bpp, v, bpp, big_endian);
        }
}

/* ------------------------------------------------------------------ extraction */

void pbxo_extract_be(const uint8_t* plane, int plane_be, int pt, int64_t pitch, int32_t x,
                     int32_t y, int32_t w, int32_t h, uint8_t* out) {
    int bpp = pbxo_bpp(pt);
    for (int32_t r = 0; r < h; r++) {
        const uint8_t* src = plane + (int64_t)(y + r) * pitch + (int64_t)x * bpp;
        uint8_t* dst = out + (size_t)r * w * bpp;
        if (plane_be || bpp == 1) {
            memcpy(dst, src, (size_t)w * bpp);
        } else {
            for (int32_t i = 0; i < w; i++)
                for (int b = 0; b < bpp; b++) dst[i * bpp + b] = src[i * bpp + bpp - 1 - b];
        }
    }
}

/* ------------------------------------------------------------------ PNG */

static void be32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
static void be16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static uint32_t rd32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static int paeth(int a, int b, int c) {
    int p = a + b - c, pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    if (pb <= pc) return b;
    return c;
}

/* The byte filter ft predicts (None: 0). */
static int filt_pred(int ft, int left, int up, int ul) {
    switch (ft) {
    case 0: return 0;
    case 1: return left;
    case 2: return up;
    case 3: return (left + up) >> 1;
    default: return paeth(left, up, ul);
    }
}

static uint8_t filt_byte(int ft, int cur, int left, int up, int ul) {
    switch (ft) {
    case 0: return (uint8_t)cur;
    case 1: return (uint8_t)(cur - left);
    case 2: return (uint8_t)(cur - up);
    case 3: return (uint8_t)(cur - ((left + up) >> 1));
    default: return (uint8_t)(cur - paeth(left, up, ul));
    }
}

/* APNGWriter sign flip for int8/int16: the most significant byte of
 * each big-endian sample gets its top bit flipped (v + 2^(n-1) mod 2^n). */
static void png_row_bytes(const uint8_t* row_be, int pt, int32_t w, uint8_t* dst) {
    int bpp = pbxo_bpp(pt);
    size_t n = (size_t)w * bpp;
    memcpy(dst, row_be, n);
    if (pt == PBXO_INT8 || pt == PBXO_INT16)
        for (size_t i = 0; i < n; i += bpp) dst[i] ^= 0x80;
}

/* The adaptive option's tile mode (round 6): on microscope-like 16-bit data the
 * per-row rule below picks Sub/Paeth rows whose residuals cost more bytes than the raw rows,
 * because a distribution concentrated away from zero (the raw low bytes) scores a large
 * |byte - 0| sum.  So each tile first asks whether filtering pays at all, on its middle row
 * r* = h/2 (prediction row r* - 1, zeros above the tile): the best of Sub/Up/Avg/Paeth by the
 * plain-distance sum (the lowest on ties) against None, by the sum over the byte planes
 * ((i mod bpp) & 1) of the squared counts of the residual byte values -- a collision measure:
 * the larger, the more concentrated, the fewer bits.  None wins ties.  If None wins, every row
 * of the tile is filter None; otherwise every row takes the per-row rule.
 * scripts/adaptive_rules.py (zlib-6, six tiles each): G_NOISE 385,876 (None 390,421),
 * G_FAKE 1,572 (3,666), Poisson-like 266,701 (= None; the per-row rule alone: 290,636). */
static int adaptive_tile_none(const uint8_t* tile_be, int pt, int32_t w, int32_t h) {
    int bpp = pbxo_bpp(pt);
    size_t rb = (size_t)w * bpp;
    int32_t rs = h / 2;
    uint8_t* prev = (uint8_t*)calloc(rb + 1, 1);
    uint8_t* cur = (uint8_t*)calloc(rb + 1, 1);
    if (rs > 0) png_row_bytes(tile_be + (size_t)(rs - 1) * rb, pt, w, prev);
    png_row_bytes(tile_be + (size_t)rs * rb, pt, w, cur);
    uint64_t sad[5] = {0, 0, 0, 0, 0};
    for (size_t i = 0; i < rb; i++) {
        int left = i >= (size_t)bpp ? cur[i - bpp] : 0;
        int ul = i >= (size_t)bpp ? prev[i - bpp] : 0;
        for (int f = 1; f < 5; f++) {
            int v = (int)cur[i] - filt_pred(f, left, prev[i], ul);
            sad[f] += (uint64_t)(v < 0 ? -v : v);
        }
    }
    int fb = 1;
    for (int f = 2; f < 5; f++)
        if (sad[f] < sad[fb]) fb = f;
    uint32_t* cnt = (uint32_t*)calloc(2 * 2 * 256, sizeof(uint32_t));  /* [cand][plane][byte] */
    for (size_t i = 0; i < rb; i++) {
        int left = i >= (size_t)bpp ? cur[i - bpp] : 0;
        int ul = i >= (size_t)bpp ? prev[i - bpp] : 0;
        int pl = (int)(i % (size_t)bpp) & 1;
        cnt[(0 * 2 + pl) * 256 + cur[i]]++;
        cnt[(1 * 2 + pl) * 256 + filt_byte(fb, cur[i], left, prev[i], ul)]++;
    }
    uint64_t q0 = 0, q1 = 0;
    for (int k = 0; k < 512; k++) {
        q0 += (uint64_t)cnt[k] * cnt[k];
        q1 += (uint64_t)cnt[512 + k] * cnt[512 + k];
    }
    free(cnt);
    free(prev);
    free(cur);
    return q0 >= q1;
}

int pbxo_adaptive_tile_none(const uint8_t* tile_be, int pt, int32_t w, int32_t h) {
    return w > 0 && h > 0 ? adaptive_tile_none(tile_be, pt, w, h) : 0;
}

size_t pbxo_png_filter_stream(const uint8_t* tile_be, int pt, int32_t w, int32_t h, int filter,
                              uint8_t* out) {
    int bpp = pbxo_bpp(pt);
    size_t rb = (size_t)w * bpp, rl = rb + 1;
    const int tile_none = filter == 5 && w > 0 && h > 0 && adaptive_tile_none(tile_be, pt, w, h);
    uint8_t* prev = (uint8_t*)calloc(rb + 1, 1);
    uint8_t* cur = (uint8_t*)calloc(rb + 1, 1);
    for (int32_t r = 0; r < h; r++) {
        png_row_bytes(tile_be + (size_t)r * rb, pt, w, cur);
        int ft = filter;
        if (tile_none) {
            ft = 0;
        } else if (filter == 5) {
            /* adaptive (the pbx_config.png_filter option; the reference writes None): per row the
             * filter whose predictions are closest to the bytes, minimum sum of |byte -
             * prediction| (the plain byte distance, no mod-256 wrap: v_sad_u8 on the GPU), the
             * lowest filter on ties.  Measured against libpng's sum of |signed residual|: -1.6%
             * zlib-6 bytes on G_NOISE, equal on G_FAKE, +0.7% on Poisson-like data. */
            uint64_t best = UINT64_MAX;
            for (int f = 0; f < 5; f++) {
                uint64_t s = 0;
                for (size_t i = 0; i < rb; i++) {
                    int left = i >= (size_t)bpp ? cur[i - bpp] : 0;
                    int ul = i >= (size_t)bpp ? prev[i - bpp] : 0;
                    int v = (int)cur[i] - filt_pred(f, left, prev[i], ul);
                    s += (uint64_t)(v < 0 ? -v : v);
                }
                if (s < best) { best = s; ft = f; }
            }
        }
        uint8_t* o = out + (size_t)r * rl;
        o[0] = (uint8_t)ft;
        for (size_t i = 0; i < rb; i++) {
            int left = i >= (size_t)bpp ? cur[i - bpp] : 0;
            int ul = i >= (size_t)bpp ? prev[i - bpp] : 0;
            o[1 + i] = filt_byte(ft, cur[i], left, prev[i], ul);
        }
        uint8_t* tmp = prev; prev = cur; cur = tmp;
    }
    free(prev);
    free(cur);
    return (size_t)h * rl;
}

static size_t put_chunk(uint8_t* out, const char* type, const uint8_t* data, uint32_t n) {
    be32(out, n);
    memcpy(out + 4, type, 4);
    if (n) memcpy(out + 8, data, n);
    uint32_t crc = (uint32_t)crc32(0L, out + 4, 4 + n);
    be32(out + 8 + n, crc);
    return 12 + (size_t)n;
}

size_t pbxo_png_max_size(int pt, int32_t w, int32_t h) {
    size_t raw = (size_t)h * (1 + (size_t)w * pbxo_bpp(pt));
    return 8 + 25 + 20 + 38 + 12 + compressBound((uLong)raw) + 12 + 64;
}

int pbxo_png_encode(const uint8_t* tile_be, int pt, int32_t w, int32_t h, int level,
                    uint8_t* out, size_t cap, size_t* len) {
    /* APNGWriter supports int8/uint8/int16/uint16 only ("Unsupported image type"). */
    if (!(pt == PBXO_INT8 || pt == PBXO_UINT8 || pt == PBXO_INT16 || pt == PBXO_UINT16))
        return PBXO_E_NOTFOUND;
    if (w <= 0 || h <= 0) return PBXO_E_NOTFOUND;
    if (cap < pbxo_png_max_size(pt, w, h)) return PBXO_E_INTERNAL;
    int bpp = pbxo_bpp(pt);
    size_t raw_len = (size_t)h * (1 + (size_t)w * bpp);
    uint8_t* raw = (uint8_t*)malloc(raw_len);
    pbxo_png_filter_stream(tile_be, pt, w, h, 0, raw);
    uLongf zlen = compressBound((uLong)raw_len);
    uint8_t* z = (uint8_t*)malloc(zlen);
    int zr = compress2(z, &zlen, raw, (uLong)raw_len, level);
    free(raw);
    if (zr != Z_OK) { free(z); return PBXO_E_INTERNAL; }

    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    size_t o = 0;
    memcpy(out, sig, 8); o += 8;
    uint8_t ihdr[13];
    be32(ihdr, (uint32_t)w); be32(ihdr + 4, (uint32_t)h);
    ihdr[8] = (uint8_t)(8 * bpp); ihdr[9] = 0; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
    o += put_chunk(out + o, "IHDR", ihdr, 13);
    uint8_t actl[8];
    be32(actl, 1); be32(actl + 4, 0);
    o += put_chunk(out + o, "acTL", actl, 8);
    uint8_t fctl[26];
    memset(fctl, 0, sizeof fctl);
    be32(fctl, 0); be32(fctl + 4, (uint32_t)w); be32(fctl + 8, (uint32_t)h);
    o += put_chunk(out + o, "fcTL", fctl, 26);
    o += put_chunk(out + o, "IDAT", z, (uint32_t)zlen);
    o += put_chunk(out + o, "IEND", NULL, 0);
    free(z);
    *len = o;
    return PBXO_OK;
}

/* ------------------------------------------------------------------ TIFF */

#define TIFF_NTAGS 11
#define TIFF_DATA_OFFSET 160 /* 8 + 2 + 11*12 + 4 = 146, rounded up to 16 */

size_t pbxo_tiff_size(int pt, int32_t w, int32_t h) {
    return TIFF_DATA_OFFSET + (size_t)w * h * pbxo_bpp(pt);
}

static size_t tiff_tag(uint8_t* p, uint16_t tag, uint16_t type, uint32_t count, uint32_t v) {
    be16(p, tag); be16(p + 2, type); be32(p + 4, count);
    if (type == 3) { be16(p + 8, v); be16(p + 10, 0); } else be32(p + 8, v);
    return 12;
}

/* Classic big-endian TIFF (TiffWriter with PixelsBigEndian=true, TileRequestHandler.java:155),
 * Compression=1, one strip.  Strip layout is Bio-Formats' choice upstream (unpinned); the
 * decoded samples are what parity is defined on. */
int pbxo_tiff_encode(const uint8_t* tile_be, int pt, int32_t w, int32_t h, uint8_t* out,
                     size_t cap, size_t* len) {
    int bpp = pbxo_bpp(pt);
    if (bpp == 0 || w <= 0 || h <= 0) return PBXO_E_NOTFOUND;
    size_t n = (size_t)w * h * bpp;
    if (cap < TIFF_DATA_OFFSET + n) return PBXO_E_INTERNAL;
    memset(out, 0, TIFF_DATA_OFFSET);
    out[0] = 'M'; out[1] = 'M'; be16(out + 2, 42); be32(out + 4, 8);
    uint8_t* p = out + 8;
    be16(p, TIFF_NTAGS); p += 2;
    int sf = (pt == PBXO_FLOAT || pt == PBXO_DOUBLE) ? 3 : (pbxo_is_signed_int(pt) ? 2 : 1);
    p += tiff_tag(p, 256, 4, 1, (uint32_t)w);
    p += tiff_tag(p, 257, 4, 1, (uint32_t)h);
    p += tiff_tag(p, 258, 3, 1, (uint32_t)(8 * bpp));
    p += tiff_tag(p, 259, 3, 1, 1);
    p += tiff_tag(p, 262, 3, 1, 1);
    p += tiff_tag(p, 273, 4, 1, TIFF_DATA_OFFSET);
    p += tiff_tag(p, 277, 3, 1, 1);
    p += tiff_tag(p, 278, 4, 1, (uint32_t)h);
    p += tiff_tag(p, 279, 4, 1, (uint32_t)n);
    p += tiff_tag(p, 284, 3, 1, 1);
    p += tiff_tag(p, 339, 3, 1, (uint32_t)sf);
    be32(p, 0);
    memcpy(out + TIFF_DATA_OFFSET, tile_be, n);
    *len = TIFF_DATA_OFFSET + n;
    return PBXO_OK;
}

/* ------------------------------------------------------------------ getTile */

int pbxo_get_tile(const uint8_t* plane, int plane_be, int pt, int32_t size_x, int32_t size_y,
                  int32_t x, int32_t y, int32_t w, int32_t h, int format, uint8_t* out,
                  size_t cap, size_t* len, int32_t* out_w, int32_t* out_h) {
    if (w == 0) w = size_x; /* TileRequestHandler.java:92-94 */
    if (h == 0) h = size_y; /* :95-97 */
    if (out_w) *out_w = w;
    if (out_h) *out_h = h;
    int bpp = pbxo_bpp(pt);
    if (bpp == 0) return PBXO_E_NOTFOUND;
    /* int tileSize = width * height * bytesPerPixel (:102); Java int overflow -> negative
     * array size or a short buffer -> exception -> null (:133-138). */
    int64_t tile_size = (int64_t)w * h * bpp;
    if (w < 0 || h < 0 || tile_size > 2147483647LL) return PBXO_E_NOTFOUND;
    /* getTileDirect outside the plane throws (ext. PixelBuffer) -> 404 */
    if (x < 0 || y < 0 || (int64_t)x + w > size_x || (int64_t)y + h > size_y)
        return PBXO_E_NOTFOUND;
    if (tile_size == 0) return PBXO_E_NOTFOUND;
    uint8_t* tile = (uint8_t*)malloc((size_t)tile_size);
    pbxo_extract_be(plane, plane_be, pt, (int64_t)size_x * bpp, x, y, w, h, tile);
    int st = PBXO_OK;
    if (format == PBXO_FMT_RAW) {
        if (cap < (size_t)tile_size) st = PBXO_E_INTERNAL;
        else { memcpy(out, tile, (size_t)tile_size); *len = (size_t)tile_size; }
    } else if (format == PBXO_FMT_PNG) {
        st = pbxo_png_encode(tile, pt, w, h, 6, out, cap, len);
    } else if (format == PBXO_FMT_TIF) {
        st = pbxo_tiff_encode(tile, pt, w, h, out, cap, len);
    } else {
        st = PBXO_E_NOTFOUND; /* "Unknown output format" -> null (:125-126) */
    }
    free(tile);
    return st;
}

/* ------------------------------------------------------------------ decoders */

int pbxo_zlib_compress(const uint8_t* in, size_t n, int level, uint8_t* out, size_t cap,
                       size_t* out_len) {
    uLongf zl = (uLongf)cap;
    int r = compress2(out, &zl, in, (uLong)n, level);
    *out_len = zl;
    return r == Z_OK ? 0 : -1;
}

int pbxo_zlib_inflate(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    z_stream s;
    memset(&s, 0, sizeof s);
    if (inflateInit(&s) != Z_OK) return -1;
    s.next_in = (Bytef*)in; s.avail_in = (uInt)n;
    s.next_out = out; s.avail_out = (uInt)cap;
    int r = inflate(&s, Z_FINISH);
    *out_len = s.total_out;
    int ok = (r == Z_STREAM_END) && s.avail_in == 0;
    inflateEnd(&s);
    return ok ? 0 : -1;
}

uint32_t pbxo_crc32(uint32_t crc, const uint8_t* p, size_t n) { return (uint32_t)crc32(crc, p, (uInt)n); }
uint32_t pbxo_adler32(uint32_t a, const uint8_t* p, size_t n) { return (uint32_t)adler32(a, p, (uInt)n); }

/* Collect IDAT payload after validating signature + chunk CRCs. */
static int png_collect(const uint8_t* png, size_t len, uint8_t** idat, size_t* idat_len,
                       int32_t* w, int32_t* h, int32_t* depth, int32_t* ctype) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    if (len < 8 || memcmp(png, sig, 8) != 0) return -1;
    size_t o = 8, cap = 0, n = 0;
    uint8_t* buf = NULL;
    int seen_ihdr = 0, seen_iend = 0;
    while (o + 12 <= len) {
        uint32_t cl = rd32(png + o);
        if (o + 12 + (size_t)cl > len) { free(buf); return -2; }
        const uint8_t* type = png + o + 4;
        uint32_t crc = (uint32_t)crc32(0L, type, 4 + cl);
        if (crc != rd32(png + o + 8 + cl)) { free(buf); return -3; }
        if (!memcmp(type, "IHDR", 4)) {
            if (cl != 13) { free(buf); return -4; }
            *w = (int32_t)rd32(type + 4); *h = (int32_t)rd32(type + 8);
            *depth = type[12]; *ctype = type[13];
            if (type[14] || type[15] || type[16]) { free(buf); return -5; }
            seen_ihdr = 1;
        } else if (!memcmp(type, "IDAT", 4)) {
            if (n + cl > cap) { cap = (n + cl) * 2 + 1024; buf = (uint8_t*)realloc(buf, cap); }
            memcpy(buf + n, type + 4, cl); n += cl;
        } else if (!memcmp(type, "IEND", 4)) {
            seen_iend = 1;
            o += 12 + cl;
            break;
        }
        o += 12 + cl;
    }
    if (!seen_ihdr || !seen_iend || o != len) { free(buf); return -6; }
    *idat = buf; *idat_len = n;
    return 0;
}

int pbxo_png_inflate_idat(const uint8_t* png, size_t len, uint8_t* out, size_t cap, size_t* out_len) {
    uint8_t* idat = NULL; size_t il = 0; int32_t w, h, d, ct;
    int r = png_collect(png, len, &idat, &il, &w, &h, &d, &ct);
    if (r) return r;
    r = pbxo_zlib_inflate(idat, il, out, cap, out_len);
    free(idat);
    return r;
}

int pbxo_png_decode(const uint8_t* png, size_t len, uint8_t* out, size_t cap, int32_t* w,
                    int32_t* h, int32_t* depth, int32_t* ctype) {
    uint8_t* idat = NULL; size_t il = 0;
    int r = png_collect(png, len, &idat, &il, w, h, depth, ctype);
    if (r) return r;
    if (*ctype != 0 || (*depth != 8 && *depth != 16)) { free(idat); return -7; }
    int bpp = *depth / 8;
    size_t rb = (size_t)(*w) * bpp, rl = rb + 1, need = rl * (size_t)(*h);
    if (cap < rb * (size_t)(*h)) { free(idat); return -8; }
    uint8_t* raw = (uint8_t*)malloc(need + 1);
    size_t got = 0;
    r = pbxo_zlib_inflate(idat, il, raw, need + 1, &got);
    free(idat);
    if (r || got != need) { free(raw); return -9; }
    for (int32_t y = 0; y < *h; y++) {
        const uint8_t* f = raw + (size_t)y * rl;
        uint8_t* cur = out + (size_t)y * rb;
        const uint8_t* prev = y ? out + (size_t)(y - 1) * rb : NULL;
        int ft = f[0];
        if (ft > 4) { free(raw); return -10; }
        for (size_t i = 0; i < rb; i++) {
            int a = i >= (size_t)bpp ? cur[i - bpp] : 0;
            int b = prev ? prev[i] : 0;
            int c = (prev && i >= (size_t)bpp) ? prev[i - bpp] : 0;
            int x = f[1 + i], v;
            switch (ft) {
            case 0: v = x; break;
            case 1: v = x + a; break;
            case 2: v = x + b; break;
            case 3: v = x + ((a + b) >> 1); break;
            default: v = x + paeth(a, b, c); break;
            }
            cur[i] = (uint8_t)v;
        }
    }
    free(raw);
    return 0;
}

static uint32_t tget(const uint8_t* p, int be, int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; i++) v = be ? (v << 8) | p[i] : v | ((uint32_t)p[i] << (8 * i));
    return v;
}

static uint32_t tiff_value(const uint8_t* tif, size_t len, const uint8_t* e, int be, uint32_t idx) {
    uint16_t type = (uint16_t)tget(e + 2, be, 2);
    uint32_t count = tget(e + 4, be, 4);
    int sz = type == 3 ? 2 : 4;
    const uint8_t* base = e + 8;
    if ((uint64_t)count * sz > 4) {
        uint32_t off = tget(e + 8, be, 4);
        if ((size_t)off + (size_t)count * sz > len) return 0;
        base = tif + off;
    }
    return tget(base + (size_t)idx * sz, be, sz);
}

/* Tiled TIFF (TIFF 6.0 section 15: TileWidth 322, TileLength 323, TileOffsets 324,
 * TileByteCounts 325): tiles row-major over the image, each tw x tl samples (edge tiles
 * padded), raw or one zlib stream; only the part inside the image is kept. */
static int tiff_decode_tiles(const uint8_t* tif, size_t len, int be, uint8_t* out, size_t cap,
                             int32_t w, int32_t h, int32_t bits, int32_t comp, uint32_t spp,
                             uint32_t planar, uint32_t tw, uint32_t tl, uint32_t ntiles,
                             const uint8_t* toffs, const uint8_t* tcnts) {
    if (!toffs || !tcnts || !tw || !tl || spp != 1 || planar != 1 || bits % 8 || w <= 0 || h <= 0)
        return -4;
    if (tw % 16 || tl % 16) return -11;  /* TIFF 6.0: tile sizes are multiples of 16 */
    const size_t bpp = (size_t)bits / 8, rb = (size_t)w * bpp, trb = (size_t)tw * bpp;
    const uint32_t ntx = ((uint32_t)w + tw - 1) / tw, nty = ((uint32_t)h + tl - 1) / tl;
    if (ntiles != ntx * nty || tget(tcnts + 4, be, 4) != ntiles) return -12;
    if (cap < rb * (size_t)h) return -5;
    const size_t tbytes = trb * tl;
    uint8_t* tile = (uint8_t*)malloc(tbytes + 1);
    if (!tile) return -13;
    for (uint32_t k = 0; k < ntiles; k++) {
        uint32_t off = tiff_value(tif, len, toffs, be, k), cnt = tiff_value(tif, len, tcnts, be, k);
        if ((size_t)off + cnt > len) { free(tile); return -6; }
        if (comp == 1) {
            if (cnt < tbytes) { free(tile); return -7; }
            memcpy(tile, tif + off, tbytes);
        } else if (comp == 8 || comp == 32946) {
            size_t got = 0;
            if (pbxo_zlib_inflate(tif + off, cnt, tile, tbytes + 1, &got) || got != tbytes) {
                free(tile);
                return -8;
            }
        } else {
            free(tile);
            return -9;
        }
        const uint32_t tx = k % ntx, ty = k / ntx;
        const size_t x0 = (size_t)tx * tw, y0 = (size_t)ty * tl;
        const size_t vw = (size_t)w - x0 < tw ? (size_t)w - x0 : tw;
        const size_t vh = (size_t)h - y0 < tl ? (size_t)h - y0 : tl;
        for (size_t r = 0; r < vh; r++) memcpy(out + (y0 + r) * rb + x0 * bpp, tile + r * trb, vw * bpp);
    }
    free(tile);
    return 0;
}

static void wbe16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }
static void wbe32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

/* Tiled-TIFF writer: the layout DESIGN.md §3 specifies for tiled responses ("MM", 12-entry
 * IFD at 8, TileOffsets at 160 and TileByteCounts at 160 + 4n when n > 1, tile data from the
 * 16-byte aligned end of the arrays), tiles zero-padded to t x t, raw (comp 1) or each a
 * zlib stream at level 6 (comp 8).  Returns 0, -1 on bad arguments, -2 if cap is short. */
int pbxo_tiff_tiled_write(const uint8_t* tile_be, int32_t w, int32_t h, int32_t bpp, int32_t sf,
                          int32_t t, int32_t comp, uint8_t* out, size_t cap, size_t* out_len) {
    if (w <= 0 || h <= 0 || t <= 0 || t % 16 || (comp != 1 && comp != 8) || bpp <= 0) return -1;
    const uint32_t ntx = ((uint32_t)w + t - 1) / t, nty = ((uint32_t)h + t - 1) / t, n = ntx * nty;
    const size_t D = n > 1 ? (160 + 8 * (size_t)n + 15) & ~(size_t)15 : 160;
    const size_t rb = (size_t)w * bpp, trb = (size_t)t * bpp, tbytes = trb * t;
    if (cap < D) return -2;
    memset(out, 0, D);
    uint8_t* tile = (uint8_t*)malloc(tbytes);
    if (!tile) return -1;
    size_t pos = D;
    uint32_t off0 = 0, cnt0 = 0;
    for (uint32_t k = 0; k < n; k++) {
        const size_t x0 = (size_t)(k % ntx) * t, y0 = (size_t)(k / ntx) * t;
        const size_t vw = (size_t)w - x0 < (size_t)t ? (size_t)w - x0 : (size_t)t;
        const size_t vh = (size_t)h - y0 < (size_t)t ? (size_t)h - y0 : (size_t)t;
        memset(tile, 0, tbytes);
        for (size_t r = 0; r < vh; r++) memcpy(tile + r * trb, tile_be + (y0 + r) * rb + x0 * bpp, vw * bpp);
        size_t cnt;
        if (comp == 1) {
            if (pos + tbytes > cap) { free(tile); return -2; }
            memcpy(out + pos, tile, tbytes);
            cnt = tbytes;
        } else {
            uLongf dl = (uLongf)(cap - pos);
            if (compress2(out + pos, &dl, tile, (uLong)tbytes, 6) != Z_OK) { free(tile); return -2; }
            cnt = dl;
        }
        if (n > 1) {
            wbe32(out + 160 + 4 * (size_t)k, (uint32_t)pos);
            wbe32(out + 160 + 4 * (size_t)n + 4 * (size_t)k, (uint32_t)cnt);
        } else {
            off0 = (uint32_t)pos; cnt0 = (uint32_t)cnt;
        }
        pos += cnt;
    }
    free(tile);
    out[0] = 'M'; out[1] = 'M'; wbe16(out + 2, 42); wbe32(out + 4, 8); wbe16(out + 8, 12);
    const uint16_t tag[12] = {256, 257, 258, 259, 262, 277, 284, 322, 323, 324, 325, 339};
    const uint16_t typ[12] = {4, 4, 3, 3, 3, 3, 3, 4, 4, 4, 4, 3};
    const uint32_t val[12] = {(uint32_t)w, (uint32_t)h, 8u * bpp, (uint32_t)comp, 1, 1, 1, (uint32_t)t,
                              (uint32_t)t, n > 1 ? 160u : off0, n > 1 ? 160u + 4 * n : cnt0, (uint32_t)sf};
    for (int k = 0; k < 12; k++) {
        uint8_t* e = out + 10 + 12 * k;
        wbe16(e, tag[k]); wbe16(e + 2, typ[k]);
        wbe32(e + 4, (tag[k] == 324 || tag[k] == 325) ? n : 1u);
        if (typ[k] == 3) wbe16(e + 8, val[k]); else wbe32(e + 8, val[k]);
    }
    *out_len = pos;
    return 0;
}

int pbxo_tiff_decode(const uint8_t* tif, size_t len, uint8_t* out, size_t cap, int32_t* w,
                     int32_t* h, int32_t* bits, int32_t* sf, int32_t* comp, int32_t* big_endian) {
    if (len < 8) return -1;
    int be;
    if (tif[0] == 'M' && tif[1] == 'M') be = 1;
    else if (tif[0] == 'I' && tif[1] == 'I') be = 0;
    else return -1;
    if (tget(tif + 2, be, 2) != 42) return -2;
    uint32_t ifd = tget(tif + 4, be, 4);
    if ((size_t)ifd + 2 > len) return -3;
    uint32_t nt = tget(tif + ifd, be, 2);
    if ((size_t)ifd + 2 + nt * 12 + 4 > len) return -3;
    uint32_t rps = 0, nstrips = 0, spp = 1, planar = 1, tw = 0, tl = 0, ntiles = 0;
    const uint8_t *offs = NULL, *cnts = NULL, *toffs = NULL, *tcnts = NULL;
    *w = *h = 0; *bits = 0; *sf = 1; *comp = 1; *big_endian = be;
    for (uint32_t i = 0; i < nt; i++) {
        const uint8_t* e = tif + ifd + 2 + 12 * i;
        uint16_t tag = (uint16_t)tget(e, be, 2);
        switch (tag) {
        case 256: *w = (int32_t)tiff_value(tif, len, e, be, 0); break;
        case 257: *h = (int32_t)tiff_value(tif, len, e, be, 0); break;
        case 258: *bits = (int32_t)tiff_value(tif, len, e, be, 0); break;
        case 259: *comp = (int32_t)tiff_value(tif, len, e, be, 0); break;
        case 273: offs = e; nstrips = tget(e + 4, be, 4); break;
        case 277: spp = tiff_value(tif, len, e, be, 0); break;
        case 278: rps = tiff_value(tif, len, e, be, 0); break;
        case 279: cnts = e; break;
        case 284: planar = tiff_value(tif, len, e, be, 0); break;
        case 322: tw = tiff_value(tif, len, e, be, 0); break;
        case 323: tl = tiff_value(tif, len, e, be, 0); break;
        case 324: toffs = e; ntiles = tget(e + 4, be, 4); break;
        case 325: tcnts = e; break;
        case 339: *sf = (int32_t)tiff_value(tif, len, e, be, 0); break;
        default: break;
        }
    }
    if (toffs || tw || tl)
        return tiff_decode_tiles(tif, len, be, out, cap, *w, *h, *bits, *comp, spp, planar, tw, tl,
                                 ntiles, toffs, tcnts);
    if (!offs || !cnts || spp != 1 || planar != 1 || *bits % 8) return -4;
    if (rps == 0) rps = (uint32_t)*h;
    size_t rb = (size_t)(*w) * (*bits / 8), total = rb * (size_t)(*h), o = 0;
    if (cap < total) return -5;
    for (uint32_t s = 0; s < nstrips; s++) {
        uint32_t off = tiff_value(tif, len, offs, be, s);
        uint32_t cnt = tiff_value(tif, len, cnts, be, s);
        if ((size_t)off + cnt > len) return -6;
        size_t rows = rps;
        if ((size_t)s * rps + rows > (size_t)*h) rows = (size_t)*h - (size_t)s * rps;
        size_t want = rows * rb;
        if (*comp == 1) {
            if (cnt < want) return -7;
            memcpy(out + o, tif + off, want);
        } else if (*comp == 8 || *comp == 32946) {
            size_t got = 0;
            if (pbxo_zlib_inflate(tif + off, cnt, out + o, want, &got) || got != want) return -8;
        } else {
            return -9;
        }
        o += want;
    }
    return o == total ? 0 : -10;
}

/* ------------------------------------------------------------------ metadata */

int pbxo_tile_filename(int64_t id, int32_t z, int32_t c, int32_t t, int32_t x, int32_t y, int32_t w,
                       int32_t h, const char* format, char* out, size_t cap) {
    return snprintf(out, cap, "image%lld_z%d_c%d_t%d_x%d_y%d_w%d_h%d.%s", (long long)id, z, c, t,
                    x, y, w, h, format ? format : "bin");
}

const char* pbxo_content_type(const char* format) {
    if (format && !strcmp(format, "png")) return "image/png";
    if (format && !strcmp(format, "tif")) return "image/tiff";
    return "application/octet-stream";
}

/* ------------------------------------------------------------------ CPU baseline */

typedef struct {
    const uint8_t* plane; int pt, format; int32_t pw, ph, w, h; int first, step, tiles;
    uint64_t bytes;
    int32_t x0, y0; int single; /* pbxo_bench_at: the one region (x0, y0, w, h) every time */
} bench_arg;

static void* bench_worker(void* p) {
    bench_arg* a = (bench_arg*)p;
    int bpp = pbxo_bpp(a->pt);
    size_t cap = pbxo_png_max_size(a->pt, a->w, a->h) + pbxo_tiff_size(a->pt, a->w, a->h);
    uint8_t* out = (uint8_t*)malloc(cap);
    int gx = a->pw / a->w, gy = a->ph / a->h;
    (void)bpp;
    for (int i = a->first; i < a->tiles; i += a->step) {
        int tx = i % gx, ty = (i / gx) % gy;
        size_t len = 0;
        int32_t ow, oh;
        pbxo_get_tile(a->plane, 0, a->pt, a->pw, a->ph, a->single ? a->x0 : tx * a->w,
                      a->single ? a->y0 : ty * a->h, a->w, a->h, a->format, out, cap, &len, &ow, &oh);
        a->bytes += len;
    }
    free(out);
    return NULL;
}

static double bench_run(int kind, int pt, int format, int32_t pw, int32_t ph, int single, int32_t x0,
                        int32_t y0, int32_t w, int32_t h, int tiles, int threads, uint64_t* out_bytes);

double pbxo_bench(int kind, int pt, int format, int32_t pw, int32_t ph, int32_t w, int32_t h,
                  int tiles, int threads, uint64_t* out_bytes) {
    return bench_run(kind, pt, format, pw, ph, 0, 0, 0, w, h, tiles, threads, out_bytes);
}

/* BASELINE configs[0]: ONE request (x0, y0, w, h) of a pw x ph plane, `reps` times over
 * `threads` threads (TileRequestHandler.getTile repeated by the Vert.x worker pool). */
double pbxo_bench_at(int kind, int pt, int format, int32_t pw, int32_t ph, int32_t x0, int32_t y0,
                     int32_t w, int32_t h, int reps, int threads, uint64_t* out_bytes) {
    return bench_run(kind, pt, format, pw, ph, 1, x0, y0, w, h, reps, threads, out_bytes);
}

static double bench_run(int kind, int pt, int format, int32_t pw, int32_t ph, int single, int32_t x0,
                        int32_t y0, int32_t w, int32_t h, int tiles, int threads, uint64_t* out_bytes) {
    int bpp = pbxo_bpp(pt);
    uint8_t* plane = (uint8_t*)malloc((size_t)pw * ph * bpp);
    pbxo_gen_region(kind, 0, 0, 0, 0, 0, pt, 0, 0, pw, ph, 0, plane); /* little-endian plane */
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    bench_arg* args = (bench_arg*)calloc((size_t)threads, sizeof(bench_arg));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < threads; i++) {
        bench_arg a = {plane, pt, format, pw, ph, w, h, i, threads, tiles, 0, x0, y0, single};
        args[i] = a;
        pthread_create(&th[i], NULL, bench_worker, &args[i]);
    }
    uint64_t total = 0;
    for (int i = 0; i < threads; i++) { pthread_join(th[i], NULL); total += args[i].bytes; }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th); free(args); free(plane);
    if (out_bytes) *out_bytes = total;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
