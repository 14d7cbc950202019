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
 * Pinned by fixtures encoded with c-blosc 1.21.0 / zlib via imagecodecs 2021.8.26
 * (tests/golden/zarr/make_zarr_golden.py) and round trips through the system liblz4.
 */
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
    if (bs == 0 || (flags & 0x4)) return -1;  /* bit shuffle: not restated */
    const uint32_t codec = flags >> 5;
    if (codec != 1 && codec != 3) return -1;  /* lz4 / zlib only */
    const uint32_t nblocks = (nbytes + bs - 1) / bs, leftover = nbytes % bs;
    if (16 + 4 * (size_t)nblocks > cbytes) return -1;
    uint8_t* tmp = (flags & 0x1) && ts > 1 ? (uint8_t*)malloc(bs) : NULL;
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
            else if (codec == 1) rc = pbxo_lz4_decode(in + pos, cs, dst + (size_t)s * neb, neb);
            else rc = zlib_exact(in + pos, cs, dst + (size_t)s * neb, neb);
            pos += cs;
        }
        if (!rc && tmp) {  /* byte unshuffle of this block */
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
