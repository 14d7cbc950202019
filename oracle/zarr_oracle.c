/*
 * zarr_oracle.c — CPU restatement of the NGFF/Zarr chunk decode that feeds getTileDirect
 * (SURVEY.md §8f2).  TEST INFRASTRUCTURE ONLY (same rules as pbx_oracle.c: only tests/,
 * smoke() and bench.py's cpu_baseline leg load it).
 *
 * Reference anchors: the reference serves planes through ZarrPixelsService
 * (src/main/java/com/glencoesoftware/omero/ms/pixelbuffer/PixelBufferVerticle.java:29,56;
 * src/main/resources/beanRefContext.xml:51; src/dist/conf/config.yaml:18), implemented in
 * com.glencoesoftware.omero:omero-zarr-pixel-buffer:0.6.1 (build.gradle:57), which reads
 * Zarr v2 arrays through JZarr.  That jar is absent here; its decode is the published Zarr v2
 * chunk model plus the codec formats, restated below:
 *   - Zarr v2 (C order): chunk (i, j) of a 2-D plane holds a full chunk_y x chunk_x block of
 *     samples, row-major, edge chunks padded to the full chunk shape; a missing chunk file
 *     reads as fill_value.
 *   - compressor "zlib": the chunk is one zlib stream (RFC 1950/1951).
 *   - compressor "blosc" (c-blosc 1.x frame, version 2): 16-byte header
 *       [0] version, [1] versionlz, [2] flags, [3] typesize, [4..8) nbytes, [8..12) blocksize,
 *       [12..16) cbytes (little-endian);
 *     flags: 0x1 byte shuffle, 0x2 memcpyed (raw copy after the header), 0x4 bit shuffle,
 *     0x10 "don't split", bits 5..7 the codec (0 blosclz, 1 lz4/lz4hc, 2 snappy, 3 zlib,
 *     4 zstd).  Then nblocks int32 block starts, and per block `nsplits` streams of
 *     [int32 csize][csize bytes]; csize == the split's size means stored raw.  A block is
 *     split into typesize streams unless flagged "don't split", typesize > 16, the block is
 *     the leftover block, or blocksize / typesize < 128 (MIN_BUFFERSIZE).
 *     Byte shuffle within a block of bsize bytes: byte j of element i sits at j*(bsize/ts)+i.
 *   - LZ4 block format: sequences [token][lit-len ext][literals][offset u16 LE][match ext];
 *     match length = low nibble + 4 (+ ext bytes), the last sequence has literals only.
 *   - BloscLZ (c-blosc 1.21's internal codec, FastLZ-derived): a control byte; < 32: a run
 *     of ctrl + 1 literals; else a match of length (ctrl >> 5) + 2 (7 -> 255-terminated
 *     extension bytes added), distance ((ctrl & 31) << 8) + next byte + 1, or when those two
 *     are 31 and 255, a 16-bit big-endian distance + 8192.  The first control byte's top
 *     three bits carry the level.  A match is only copied when another control byte follows
 *     (streams end with literals).
 *   - Zstandard (RFC 8878) inside blosc: one zstd frame per split; decoded here with the
 *     system libzstd (1.4.8, loaded at run time), as zlib is with the system zlib.
 *   - Bit shuffle (flag 0x4, format version 2): a block of n = bsize / ts elements with
 *     n % 8 == 0 is stored as ts * 8 bit rows of n / 8 bytes: row j * 8 + k holds bit k of byte
 *     j of every element, element i at bit i % 8 of byte i / 8; other blocks are stored as is.
 * Pinned by fixtures encoded with c-blosc 1.21.0 / zlib via imagecodecs 2021.8.26
 * (tests/golden/zarr/make_zarr_golden.py), round trips through the system liblz4, and (CPU
 * tests) the c-blosc 1.21.0 library's own decoder on frames it encoded.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <zlib.h>

#include "pbx_oracle.h"

static uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

int pbxo_lz4_decode(const uint8_t* in, size_t ilen, uint8_t* out, size_t olen) {
    size_t ip = 0, op = 0;
    for (;;) {
        if (ip >= ilen) return -1;
        const unsigned tok = in[ip++];
        size_t ll = tok >> 4;
        if (ll == 15) {
            unsigned b;
            do {
                if (ip >= ilen) return -1;
                b = in[ip++];
                ll += b;
            } while (b == 255);
        }
        if (ip + ll > ilen || op + ll > olen) return -1;
        memcpy(out + op, in + ip, ll);
        ip += ll;
        op += ll;
        if (ip == ilen) break;  /* last sequence: literals only */
        if (ip + 2 > ilen) return -1;
        const size_t off = (size_t)in[ip] | (size_t)in[ip + 1] << 8;
        ip += 2;
        size_t ml = tok & 15;
        if (ml == 15) {
            unsigned b;
            do {
                if (ip >= ilen) return -1;
                b = in[ip++];
                ml += b;
            } while (b == 255);
        }
        ml += 4;
        if (off == 0 || off > op || op + ml > olen) return -1;
        for (size_t k = 0; k < ml; k++) out[op + k] = out[op + k - off];  /* overlap-safe */
        op += ml;
    }
    return op == olen ? 0 : -1;
}

int pbxo_blosclz_decode(const uint8_t* in, size_t ilen, uint8_t* out, size_t olen) {
    size_t ip = 0, op = 0;
    if (ilen == 0) return -1;
    uint32_t ctrl = in[ip++] & 31u;
    for (;;) {
        if (ctrl >= 32) {
            size_t len = (ctrl >> 5) - 1;
            size_t ofs = (size_t)(ctrl & 31u) << 8;
            if (len == 6) {
                unsigned code;
                do {
                    if (ip + 1 >= ilen) return -1;
                    code = in[ip++];
                    len += code;
                } while (code == 255);
            } else if (ip + 1 >= ilen) {
                return -1;
            }
            const unsigned code = in[ip++];
            len += 3;
            size_t dist = ofs + code + 1;
            if (code == 255 && ofs == (31u << 8)) {  /* 16-bit distance */
                if (ip + 1 >= ilen) return -1;
                dist = ((size_t)in[ip] << 8 | in[ip + 1]) + 8191 + 1;
                ip += 2;
            }
            if (op + len > olen || dist > op) return -1;
            if (ip >= ilen) break;  /* (c-blosc: a match is copied only if a control byte follows) */
            ctrl = in[ip++];
            for (size_t k = 0; k < len; k++) out[op + k] = out[op + k - dist];  /* overlap-safe */
            op += len;
        } else {
            const size_t n = ctrl + 1;
            if (op + n > olen || ip + n > ilen) return -1;
            memcpy(out + op, in + ip, n);
            op += n;
            ip += n;
            if (ip >= ilen) break;
            ctrl = in[ip++];
        }
    }
    return op == olen ? 0 : -1;
}

/* libzstd (system 1.4.8), resolved at run time: the oracle builds without its header. */
typedef size_t (*zstd_decompress_fn)(void*, size_t, const void*, size_t);
typedef unsigned (*zstd_iserror_fn)(size_t);
static zstd_decompress_fn p_zstd_decompress;
static zstd_iserror_fn p_zstd_iserror;

static int zstd_load(void) {
    if (p_zstd_decompress) return 0;
    void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return -1;
    p_zstd_iserror = (zstd_iserror_fn)dlsym(h, "ZSTD_isError");
    p_zstd_decompress = (zstd_decompress_fn)dlsym(h, "ZSTD_decompress");
    return p_zstd_decompress && p_zstd_iserror ? 0 : -1;
}

int pbxo_zstd_decode(const uint8_t* in, size_t ilen, uint8_t* out, size_t olen) {
    if (zstd_load()) return -2;
    const size_t n = p_zstd_decompress(out, olen, in, ilen);
    if (p_zstd_iserror(n)) return -1;
    return n == olen ? 0 : -1;
}

/* bit unshuffle of one block (format version 2): see the header comment */
static void bitunshuffle_block(const uint8_t* in, uint8_t* out, uint32_t bsize, uint32_t ts) {
    const uint32_t n = bsize / ts;
    if (n % 8) {
        memcpy(out, in, bsize);
        return;
    }
    const uint32_t row = n / 8;
    memset(out, 0, (size_t)n * ts);
    for (uint32_t j = 0; j < ts; j++)
        for (uint32_t k = 0; k < 8; k++) {
            const uint8_t* r = in + (size_t)(j * 8 + k) * row;
            for (uint32_t i = 0; i < n; i++)
                out[(size_t)i * ts + j] |= (uint8_t)(((r[i >> 3] >> (i & 7)) & 1u) << k);
        }
    memcpy(out + (size_t)n * ts, in + (size_t)n * ts, bsize - n * ts);
}

static int zlib_exact(const uint8_t* in, size_t ilen, uint8_t* out, size_t olen) {
    uLongf n = (uLongf)olen;
    if (uncompress(out, &n, in, (uLong)ilen) != Z_OK) return -1;
    return n == olen ? 0 : -1;
}

int pbxo_blosc_info(const uint8_t* in, size_t len, uint32_t* nbytes, uint32_t* blocksize,
                    uint32_t* typesize, uint32_t* flags) {
    if (len < 16) return -1;
    if (nbytes) *nbytes = rd32(in + 4);
    if (blocksize) *blocksize = rd32(in + 8);
    if (typesize) *typesize = in[3];
    if (flags) *flags = in[2];
    return 0;
}

int pbxo_blosc_decode(const uint8_t* in, size_t len, uint8_t* out, size_t cap, size_t* out_len) {
    if (len < 16) return -1;
    const uint32_t flags = in[2], ts = in[3] ? in[3] : 1;
    const uint32_t nbytes = rd32(in + 4), bs = rd32(in + 8), cbytes = rd32(in + 12);
    if (cbytes > len || nbytes > cap) return -1;
    if (out_len) *out_len = nbytes;
    if (nbytes == 0) return 0;
    if (flags & 0x2) {  /* memcpyed */
        if (16 + (size_t)nbytes > cbytes) return -1;
        memcpy(out, in + 16, nbytes);
        return 0;
    }
    if (bs == 0 || in[0] != 2) return -1;  /* c-blosc 1.x frames (format version 2) */
    const uint32_t codec = flags >> 5;
    if (codec != 0 && codec != 1 && codec != 3 && codec != 4) return -1;  /* no snappy */
    const uint32_t nblocks = (nbytes + bs - 1) / bs, leftover = nbytes % bs;
    if (16 + 4 * (size_t)nblocks > cbytes) return -1;
    const int bitshuf = (flags & 0x4) != 0, byteshuf = !bitshuf && (flags & 0x1) && ts > 1;
    uint8_t* tmp = byteshuf || bitshuf ? (uint8_t*)malloc(bs) : NULL;
    int rc = 0;
    for (uint32_t b = 0; b < nblocks && !rc; b++) {
        const int is_left = leftover && b == nblocks - 1;
        const uint32_t bsize = is_left ? leftover : bs;
        const int split = !(flags & 0x10) && ts <= 16 && bsize / ts >= 128 && !is_left;
        const uint32_t nsp = split ? ts : 1, neb = bsize / nsp;
        uint8_t* dst = tmp ? tmp : out + (size_t)b * bs;
        size_t pos = rd32(in + 16 + 4 * (size_t)b);
        for (uint32_t s = 0; s < nsp && !rc; s++) {
            if (pos + 4 > cbytes) { rc = -1; break; }
            const uint32_t cs = rd32(in + pos);
            pos += 4;
            if (pos + cs > cbytes || cs > neb) { rc = -1; break; }
            if (cs == neb) memcpy(dst + (size_t)s * neb, in + pos, neb);
            else if (codec == 0) rc = pbxo_blosclz_decode(in + pos, cs, dst + (size_t)s * neb, neb);
            else if (codec == 1) rc = pbxo_lz4_decode(in + pos, cs, dst + (size_t)s * neb, neb);
            else if (codec == 3) rc = zlib_exact(in + pos, cs, dst + (size_t)s * neb, neb);
            else rc = pbxo_zstd_decode(in + pos, cs, dst + (size_t)s * neb, neb);
            pos += cs;
        }
        if (!rc && bitshuf) {
            if (bsize >= ts) bitunshuffle_block(tmp, out + (size_t)b * bs, bsize, ts);
            else memcpy(out + (size_t)b * bs, tmp, bsize);
        } else if (!rc && tmp) {  /* byte unshuffle of this block */
            const uint32_t ne = bsize / ts;
            uint8_t* o = out + (size_t)b * bs;
            for (uint32_t j = 0; j < ts; j++)
                for (uint32_t i = 0; i < ne; i++) o[(size_t)i * ts + j] = tmp[(size_t)j * ne + i];
            memcpy(o + (size_t)ne * ts, tmp + (size_t)ne * ts, bsize - ne * ts);
        }
    }
    free(tmp);
    return rc;
}

int pbxo_zarr_decode_chunk(int codec, const uint8_t* in, size_t len, uint8_t* out, size_t nbytes) {
    if (codec == PBXO_ZARR_RAW) {
        if (len < nbytes) return -1;
        memcpy(out, in, nbytes);
        return 0;
    }
    if (codec == PBXO_ZARR_ZLIB) return zlib_exact(in, len, out, nbytes);
    if (codec == PBXO_ZARR_BLOSC) {
        size_t n = 0;
        if (pbxo_blosc_decode(in, len, out, nbytes, &n)) return -1;
        return n == nbytes ? 0 : -1;
    }
    return -1;
}

int pbxo_zarr_plane(int codec, int bpp, int32_t size_x, int32_t size_y, int32_t chunk_x,
                    int32_t chunk_y, const uint8_t* data, const uint64_t* offsets,
                    const uint8_t* fill, uint8_t* plane) {
    const int32_t gx = (size_x + chunk_x - 1) / chunk_x, gy = (size_y + chunk_y - 1) / chunk_y;
    const size_t cb = (size_t)chunk_x * chunk_y * bpp, row = (size_t)size_x * bpp;
    uint8_t* buf = (uint8_t*)malloc(cb);
    if (!buf) return -1;
    int rc = 0;
    for (int32_t cy = 0; cy < gy && !rc; cy++)
        for (int32_t cx = 0; cx < gx && !rc; cx++) {
            const size_t i = (size_t)cy * gx + cx;
            const size_t len = offsets[i + 1] - offsets[i];
            if (len == 0) {
                for (size_t k = 0; k < cb; k += bpp) memcpy(buf + k, fill, bpp);
            } else if (pbxo_zarr_decode_chunk(codec, data + offsets[i], len, buf, cb)) {
                rc = -1;
                break;
            }
            const int32_t w = size_x - cx * chunk_x < chunk_x ? size_x - cx * chunk_x : chunk_x;
            const int32_t h = size_y - cy * chunk_y < chunk_y ? size_y - cy * chunk_y : chunk_y;
            for (int32_t r = 0; r < h; r++)
                memcpy(plane + (size_t)(cy * chunk_y + r) * row + (size_t)cx * chunk_x * bpp,
                       buf + (size_t)r * chunk_x * bpp, (size_t)w * bpp);
        }
    free(buf);
    return rc;
}

struct zjob {
    int codec;
    const uint8_t* data;
    const uint64_t* offsets;
    size_t nchunks, nbytes;
    size_t next;
    pthread_mutex_t mu;
    int rc;
};

static void* zworker(void* arg) {
    struct zjob* j = (struct zjob*)arg;
    uint8_t* buf = (uint8_t*)malloc(j->nbytes);
    for (;;) {
        pthread_mutex_lock(&j->mu);
        const size_t i = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (i >= j->nchunks) break;
        const size_t len = j->offsets[i + 1] - j->offsets[i];
        if (len && pbxo_zarr_decode_chunk(j->codec, j->data + j->offsets[i], len, buf, j->nbytes))
            j->rc = -1;
    }
    free(buf);
    return NULL;
}

double pbxo_zarr_bench(int codec, const uint8_t* data, const uint64_t* offsets, size_t nchunks,
                       size_t chunk_bytes, int threads) {
    struct zjob j;
    j.codec = codec; j.data = data; j.offsets = offsets; j.nchunks = nchunks;
    j.nbytes = chunk_bytes; j.next = 0; j.rc = 0;
    pthread_mutex_init(&j.mu, NULL);
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int k = 0; k < threads; k++) pthread_create(&th[k], NULL, zworker, &j);
    for (int k = 0; k < threads; k++) pthread_join(th[k], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(th);
    pthread_mutex_destroy(&j.mu);
    if (j.rc) return -1.0;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
