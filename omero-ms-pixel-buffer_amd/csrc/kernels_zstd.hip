// kernels_zstd.hip — Zstandard frame decode (RFC 8878) on gfx950: the blosc-zstd splits of
// NGFF/Zarr chunks (c-blosc 1.21 codec 4, zstd 1.4.x frames; SURVEY.md §8f2: the reference's
// ZarrPixelsService decodes them on the CPU per getTileDirect, omero-zarr-pixel-buffer 0.6.1,
// build.gradle:57).  The CPU check is the system libzstd (oracle/zarr_oracle.c).
//
// One wave per frame, everything about the parse wave-uniform (SGPRs): the frame header, raw /
// RLE / compressed blocks; literals (raw, RLE, Huffman with 1 or 4 streams, tree descriptions
// as direct 4-bit weights or FSE-compressed weights; treeless = the previous tree), the
// sequence section (predefined, RLE, FSE-compressed or repeated tables for literal lengths,
// offsets and match lengths), the interleaved FSE state decode of the backward bitstream and
// the sequence execution with the three repeat offsets.  Decoded literals of a block go to a
// per-frame scratch buffer in HBM (64 bytes per wave store); the output goes through the
// same LDS ring as the other decoders (zarr_dev.h): matches up to 4 KiB back are LDS copies,
// longer ones read the already flushed output.  Table construction uses the wave's lanes.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dev_util.h"
#include "pbx_kernels.h"
#include "zarr_dev.h"

namespace pbx {

constexpr uint32_t ZSTD_WAVES = 2;           // waves (frames) per workgroup
constexpr uint32_t ZSTD_LITBUF = 128 * 1024; // Block_Maximum_Size: a block's literals
constexpr uint32_t ZSTD_LITSTRIDE = ZSTD_LITBUF + 64;  // + the masked-off lanes' trash bytes

// Per-wave LDS (byte offsets from the wave's base)
constexpr uint32_t ZD_RING = 0;                  // 4 KiB output ring
constexpr uint32_t ZD_WIN = ZD_RING + 4096;      // 1 KiB input window
constexpr uint32_t ZD_LL = ZD_WIN + ZWIN;        // FSE tables: u32 sym | nb << 8 | base << 16
constexpr uint32_t ZD_OF = ZD_LL + 512 * 4;
constexpr uint32_t ZD_ML = ZD_OF + 256 * 4;
constexpr uint32_t ZD_HUF = ZD_ML + 512 * 4;     // Huffman: u16 sym | nb << 8, 2^11 entries
constexpr uint32_t ZD_NORM = ZD_HUF + 2048 * 2;  // i16 normalized counts [256]
constexpr uint32_t ZD_NEXT = ZD_NORM + 512;      // u32 symbolNext [256]
constexpr uint32_t ZD_SPREAD = ZD_NEXT + 1024;   // u8 spread symbols [512]
constexpr uint32_t ZD_WGT = ZD_SPREAD + 512;     // u8 Huffman weights [256]
constexpr uint32_t ZD_WT = ZD_WGT + 256;         // FSE table of the weights (<= 64 entries)
constexpr uint32_t ZD_TRASH = ZD_WT + 64 * 4;    // the output ring's trash bytes (OutRing::put_if)
constexpr uint32_t ZD_FLAG = ZD_TRASH + 64;       // sequence-start flags of a batch step (+ trash)
constexpr uint32_t ZD_BYTES = ZD_FLAG + 128;

__device__ __forceinline__ uint32_t& zd32(uint32_t off) { return *(uint32_t*)(zlds + off); }
__device__ __forceinline__ uint16_t& zd16(uint32_t off) { return *(uint16_t*)(zlds + off); }
__device__ __forceinline__ int16_t& zdi16(uint32_t off) { return *(int16_t*)(zlds + off); }

// RFC 8878 3.1.1.3.2.1: literal-length / match-length codes -> baseline, extra bits
__constant__ uint32_t c_ll_base[36] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18, 20, 22,
                                       24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192,
                                       16384, 32768, 65536};
__constant__ uint32_t c_ll_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                      2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t c_ml_base[53] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20,
                                       21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 37,
                                       39, 41, 43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051,
                                       4099, 8195, 16387, 32771, 65539};
__constant__ uint32_t c_ml_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                      0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9,
                                      10, 11, 12, 13, 14, 15, 16};
// A decoding-table entry's payload (its low 13 bits): the symbol for offsets; for literal
// and match lengths the code's extra-bit count x (5 bits) and baseline: 1 << x (+ 3 for
// match lengths) when bit 5 is set, else bits 6..12 (every other baseline is < 128).  The
// sequence loop then needs no second lookup per length code.
__device__ __forceinline__ uint32_t len_payload(uint32_t base, uint32_t bits, uint32_t add) {
    return base == (1u << bits) + add ? bits | 32u : bits | (base << 6);
}
// predefined distributions (3.1.1.3.2.2)
__constant__ int16_t c_ll_def[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2,
                                     2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t c_ml_def[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                     1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t c_of_def[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                     -1, -1, -1, -1, -1};

__device__ __forceinline__ uint32_t hibit(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

// ---- XXH64 (seed 0) of a decoded frame: the optional Content_Checksum (RFC 8878 3.1.1; low
// 32 bits of XXH64 of the frame's content), which libzstd verifies.  The four stripe
// accumulators are inherently serial over the 32-byte stripes, so lanes 0..3 run them; the wave
// loads 1 KiB (32 stripes) at a time, one 16-byte word per lane, and lane k takes 8-byte word k
// of each stripe from the lane holding it (ds_bpermute).
constexpr uint64_t XP1 = 0x9E3779B185EBCA87ull, XP2 = 0xC2B2AE3D27D4EB4Full, XP3 = 0x165667B19E3779F9ull,
                   XP4 = 0x85EBCA77C2B2AE63ull, XP5 = 0x27D4EB2F165667C5ull;
__device__ __forceinline__ uint64_t xrotl(uint64_t x, uint32_t r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t in) { return xrotl(acc + in * XP2, 31) * XP1; }
__device__ __forceinline__ uint64_t xmerge(uint64_t h, uint64_t v) { return (h ^ xround(0, v)) * XP1 + XP4; }
__device__ __forceinline__ uint64_t gld64(const uint8_t* p) {  // 8 bytes, any alignment
    const uint32_t* q = (const uint32_t*)((uintptr_t)p & ~(uintptr_t)3);
    const uint32_t sh = ((uint32_t)(uintptr_t)p & 3u) * 8;
    const uint32_t a = q[0], b = q[1], c = q[2];
    const uint32_t lo = sh ? (a >> sh) | (b << (32 - sh)) : a, hi = sh ? (b >> sh) | (c << (32 - sh)) : b;
    return ((uint64_t)hi << 32) | lo;
}
__device__ uint64_t xxh64_wave(const uint8_t* p, uint32_t len, uint32_t lane) {
    const uint32_t nst = len / 32, k = lane & 3;
    uint64_t v = k == 0 ? XP1 + XP2 : k == 1 ? XP2 : k == 2 ? 0ull : 0ull - XP1;
    for (uint32_t b = 0; b < nst; b += 32) {
        const uint32_t at = 32 * b + 16 * lane;
        uint4 x = make_uint4(0, 0, 0, 0);
        if (at + 16 <= 32 * nst) {
            const uint64_t lo = gld64(p + at), hi = gld64(p + at + 8);
            x = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
        }
        const uint32_t ns = nst - b < 32 ? nst - b : 32;
        for (uint32_t j = 0; j < ns; j++) {
            const int src = (int)(2 * j + (k >> 1));
            const uint32_t a0 = (uint32_t)__shfl((int)x.x, src, 64), a1 = (uint32_t)__shfl((int)x.y, src, 64);
            const uint32_t a2 = (uint32_t)__shfl((int)x.z, src, 64), a3 = (uint32_t)__shfl((int)x.w, src, 64);
            const uint64_t in = (k & 1) ? ((uint64_t)a3 << 32) | a2 : ((uint64_t)a1 << 32) | a0;
            v = xround(v, in);
        }
    }
    auto rl = [](uint64_t x, int l) {
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), l) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
    };
    uint64_t h;
    if (nst) {
        const uint64_t v1 = rl(v, 0), v2 = rl(v, 1), v3 = rl(v, 2), v4 = rl(v, 3);
        h = xrotl(v1, 1) + xrotl(v2, 7) + xrotl(v3, 12) + xrotl(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = XP5;
    }
    h += len;
    uint32_t i = 32 * nst;
    for (; i + 8 <= len; i += 8) h = xrotl(h ^ xround(0, gld64(p + i)), 27) * XP1 + XP4;
    if (i + 4 <= len) {
        h = xrotl(h ^ ((uint64_t)(uint32_t)gld64(p + i) * XP1), 23) * XP2 + XP3;
        i += 4;
    }
    for (; i < len; i++) h = xrotl(h ^ ((uint64_t)p[i] * XP5), 11) * XP1;
    h ^= h >> 33;
    h *= XP2;
    h ^= h >> 29;
    h *= XP3;
    h ^= h >> 32;
    return h;
}

// Input bytes of the frame through the LDS window, read forward or backward: the window is
// reloaded so that it covers [q, q + n) with room in the direction of travel.
struct ZIn {
    InWin win;
    uint32_t len;  // frame bytes
    __device__ uint32_t byte(uint32_t q) { return win.byte(q); }
    // 8 bytes from q (little-endian), window placed to end just after them (backward reads)
    __device__ uint64_t le64_back(uint32_t q) {
        win.base = rfl(win.base);
        if (q < win.base || q + 8 > win.base + ZWIN) win.load(q + 8 > ZWIN ? q + 8 - ZWIN : 0u);
        uint32_t a, b;
        __builtin_memcpy(&a, zlds + win.wo + q - win.base, 4);
        __builtin_memcpy(&b, zlds + win.wo + q - win.base + 4, 4);
        return ((uint64_t)b << 32) | a;  // (every lane the same: no readfirstlane, see §10)
    }
    // 8 bytes from q (little-endian), window placed to start at q (forward reads)
    __device__ uint64_t le64_fwd(uint32_t q) {
        if (q < win.base || q + 8 > win.base + ZWIN) win.load(q);
        uint32_t a, b;
        __builtin_memcpy(&a, zlds + win.wo + q - win.base, 4);
        __builtin_memcpy(&b, zlds + win.wo + q - win.base + 4, 4);
        return ((uint64_t)rfl(b) << 32) | rfl(a);
    }
};

// Backward bitstream over frame bytes [lo, hi): the last byte's highest set bit is the end
// marker; reads take the highest remaining bits first; bits below the start read as zeros
// (pos < 0 afterwards = over-read).
// The bits are cached: cont holds stream bits [cb, cb + 64) (cb a multiple of 8), refilled
// from the LDS window when a read leaves it (about once per 32 bits instead of per read).
struct BitBack {
    uint32_t lo;
    int32_t pos;  // bits left, counted from lo * 8
    int32_t cb;   // first bit of cont
    uint64_t cont;
    __device__ bool init(ZIn& in, uint32_t lo_, uint32_t hi_) {
        lo = lo_;
        cb = 0x7FFFFFFF;  // nothing cached
        cont = 0;
        if (hi_ <= lo_) return false;
        const uint32_t last = in.byte(hi_ - 1);
        if (!last) return false;
        pos = (int32_t)((hi_ - lo_ - 1) * 8 + hibit(last));
        return true;
    }
    // the state is wave-uniform: pin it to SGPRs at the top of a decode loop (LLVM otherwise
    // carries it in VGPRs through the loop's phis)
    __device__ void pin() {
        lo = rfl(lo);
        pos = (int32_t)rfl((uint32_t)pos);
        cb = (int32_t)rfl((uint32_t)cb);
        cont = (uint64_t)rfl((uint32_t)(cont >> 32)) << 32 | rfl((uint32_t)cont);
    }
    __device__ uint32_t peek(ZIn& in, uint32_t n) {  // n <= 32
        if (n == 0) return 0;
        const int32_t q = pos - (int32_t)n;
        if (q < cb || pos > cb + 64) {  // refill: the 8 bytes ending at pos's byte
            const int32_t e = (pos + 7) >> 3;
            const int32_t sb = e >= 8 ? e - 8 : 0;
            cont = in.le64_back(lo + (uint32_t)sb);
            cb = 8 * sb;
        }
        // q >= cb, or q < 0 with cb == 0: the bits below the start read as zeros
        const uint64_t v = q >= cb ? cont >> (q - cb) : cont << (cb - q);
        return (uint32_t)v & (n == 32 ? 0xFFFFFFFFu : ((1u << n) - 1u));
    }
    __device__ uint32_t read(ZIn& in, uint32_t n) {
        const uint32_t v = peek(in, n);
        pos -= (int32_t)n;
        return v;
    }
    // n <= 56 bits at once (a refill leaves >= 57 cached bits below pos): the first field
    // read is the value's top bits
    __device__ uint64_t read64(ZIn& in, uint32_t n) {
        if (n == 0) return 0;
        const int32_t q = pos - (int32_t)n;
        if (q < cb || pos > cb + 64) {
            const int32_t e = (pos + 7) >> 3;
            const int32_t sb = e >= 8 ? e - 8 : 0;
            cont = in.le64_back(lo + (uint32_t)sb);
            cb = 8 * sb;
        }
        const uint64_t v = q >= cb ? cont >> (q - cb) : cont << (cb - q);
        pos = q;
        return v & ((1ull << n) - 1ull);
    }
};

// FSE table description (RFC 8878 4.1.1) at frame byte q: normalized counts into ZD_NORM;
// returns the bytes it took (0 on error) and the accuracy log / symbol count.
__device__ uint32_t read_ncount(ZIn& in, uint32_t wb, uint32_t q, uint32_t qend, uint32_t max_sym,
                                uint32_t max_log, uint32_t& log, uint32_t& nsym, uint32_t lane) {
    for (uint32_t s = lane; s < 256; s += 64) zdi16(wb + ZD_NORM + 2 * s) = 0;
    __builtin_amdgcn_wave_barrier();
    uint32_t bit = 0;
    bool over = false;
    auto rd = [&](uint32_t n) -> uint32_t {  // forward LSB-first bits; past qend: error
        if (q + (bit >> 3) >= qend) { over = true; return 0u; }
        const uint32_t v = (uint32_t)(in.le64_fwd(q + (bit >> 3)) >> (bit & 7)) & ((1u << n) - 1u);
        return v;
    };
    log = rd(4) + 5;
    bit += 4;
    if (log > max_log) return 0;
    int32_t remaining = (1 << log) + 1;
    uint32_t threshold = 1u << log, nb = log + 1, sym = 0;
    bool prev0 = false;
    while (remaining > 1 && sym <= max_sym && !over) {
        if (prev0) {
            uint32_t n0 = sym;
            uint32_t r;
            while ((r = rd(2)) == 3 && !over) { n0 += 3; bit += 2; }
            if (over) return 0;
            n0 += r;
            bit += 2;
            if (n0 > max_sym + 1) return 0;
            sym = n0;  // (counts are already zero)
            if (sym > max_sym) break;
        }
        const uint32_t maxv = (2 * threshold - 1) - (uint32_t)remaining;
        const uint32_t b = rd(nb);
        int32_t count;
        if ((b & (threshold - 1)) < maxv) {
            count = (int32_t)(b & (threshold - 1));
            bit += nb - 1;
        } else {
            count = (int32_t)(b & (2 * threshold - 1));
            if (count >= (int32_t)threshold) count -= (int32_t)maxv;
            bit += nb;
        }
        count--;  // -1: "less than 1" probability
        remaining -= count < 0 ? -count : count;
        if (lane == 0) zdi16(wb + ZD_NORM + 2 * sym) = (int16_t)count;
        sym++;
        prev0 = count == 0;
        while (remaining < (int32_t)threshold && nb > 1) { nb--; threshold >>= 1; }
    }
    __builtin_amdgcn_wave_barrier();
    if (over || remaining != 1 || sym > max_sym + 1) return 0;
    const uint32_t used = (bit + 7) >> 3;
    if (q + used > qend) return 0;
    nsym = sym;
    return used;
}

// The payload of symbol s of table kind (0 literal lengths, 1 offsets, 2 match lengths).
__device__ __forceinline__ uint32_t tab_payload(uint32_t kind, uint32_t s) {
    if (kind == 0) return len_payload(c_ll_base[s < 36 ? s : 35], c_ll_bits[s < 36 ? s : 35], 0);
    if (kind == 2) return len_payload(c_ml_base[s < 53 ? s : 52], c_ml_bits[s < 53 ? s : 52], 3);
    return s;
}

// FSE decoding table (RFC 8878 4.1.1, zstd FSE_buildDTable) from the counts in ZD_NORM:
// entries u32 payload(sym) | nbBits << 13 | baseline << 17 at LDS byte `tab`.
__device__ void build_fse(uint32_t wb, uint32_t tab, uint32_t log, uint32_t nsym, uint32_t lane, uint32_t kind) {
    const uint32_t size = 1u << log, mask = size - 1;
    uint32_t high = size - 1;
    // "less than 1" symbols at the top; symbolNext = count (1 for those)
    for (uint32_t s = 0; s < nsym; s++) {
        const int32_t c = zdi16(wb + ZD_NORM + 2 * s);
        if (c == -1) {
            if (lane == 0) zlds[wb + ZD_SPREAD + high] = (uint8_t)s;
            high--;
        }
        if (lane == 0) zd32(wb + ZD_NEXT + 4 * s) = (uint32_t)(c == -1 ? 1 : c);
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t step = (size >> 1) + (size >> 3) + 3;
    uint32_t p = 0;
    for (uint32_t s = 0; s < nsym; s++) {
        const int32_t c = zdi16(wb + ZD_NORM + 2 * s);
        for (int32_t i = 0; i < c; i++) {
            if (lane == 0) zlds[wb + ZD_SPREAD + p] = (uint8_t)s;
            do { p = (p + step) & mask; } while (p > high);
        }
    }
    __builtin_amdgcn_wave_barrier();
    // next states in position order: rank of u among the positions of its symbol, by ballots
    for (uint32_t g = 0; g < size; g += 64) {
        const uint32_t u = g + lane;
        const uint32_t s = u < size ? zlds[wb + ZD_SPREAD + u] : 0xFFFFu;
        uint32_t rank = 0;
        for (uint32_t j = 0; j < 64 && g + j < size; j++) {
            const uint32_t sj = rdl(s, j);
            rank += (j < lane && sj == s) ? 1u : 0u;
        }
        uint32_t ns = 0;
        if (u < size) ns = zd32(wb + ZD_NEXT + 4 * s) + rank;
        __builtin_amdgcn_wave_barrier();
        if (u < size) {
            const uint32_t nb = log - hibit(ns);
            const uint32_t base = (ns << nb) - size;
            zd32(tab + 4 * u) = tab_payload(kind, s) | (nb << 13) | (base << 17);
            atomicAdd(&zd32(wb + ZD_NEXT + 4 * s), 1u);  // this group's occurrences
        }
        __builtin_amdgcn_wave_barrier();
    }
    __builtin_amdgcn_wave_barrier();
}

// A sequence table for a Symbol_Compression_Mode: 0 predefined, 1 RLE, 2 FSE-compressed,
// 3 repeat (the table and log are left as they are).  Returns the bytes of the section used,
// or -1 on error.
__device__ int32_t seq_table(ZIn& in, uint32_t wb, uint32_t tab, uint32_t kind, uint32_t mode, uint32_t q,
                             uint32_t qend, const int16_t* def, uint32_t def_n, uint32_t def_log,
                             uint32_t max_sym, uint32_t max_log, uint32_t& log, bool& have, uint32_t lane) {
    if (mode == 0) {
        for (uint32_t s = lane; s < 256; s += 64)
            zdi16(wb + ZD_NORM + 2 * s) = s < def_n ? def[s] : (int16_t)0;
        __builtin_amdgcn_wave_barrier();
        log = def_log;
        build_fse(wb, tab, log, def_n, lane, kind);
        have = true;
        return 0;
    }
    if (mode == 1) {
        if (q >= qend) return -1;
        const uint32_t s = in.byte(q);
        if (s > max_sym) return -1;
        if (lane == 0) zd32(tab) = tab_payload(kind, s);  // nbBits 0, baseline 0
        __builtin_amdgcn_wave_barrier();
        log = 0;
        have = true;
        return 1;
    }
    if (mode == 2) {
        uint32_t l, n;
        const uint32_t used = read_ncount(in, wb, q, qend, max_sym, max_log, l, n, lane);
        if (!used) return -1;
        log = l;
        build_fse(wb, tab, log, n, lane, kind);
        have = true;
        return (int32_t)used;
    }
    return have ? 0 : -1;  // repeat
}

// Huffman tree description (RFC 8878 4.2.1) at q: builds the decode table in ZD_HUF and
// returns the bytes used (0 on error) and the table log.
__device__ uint32_t read_huf_tree(ZIn& in, uint32_t wb, uint32_t q, uint32_t qend, uint32_t& hlog, uint32_t lane) {
    if (q >= qend) return 0;
    const uint32_t hb = in.byte(q);
    uint32_t nw = 0, used = 0;
    for (uint32_t s = lane; s < 256; s += 64) zlds[wb + ZD_WGT + s] = 0;
    __builtin_amdgcn_wave_barrier();
    if (hb >= 128) {  // direct: 4-bit weights, two per byte, high nibble first
        nw = hb - 127;
        used = 1 + (nw + 1) / 2;
        if (q + used > qend) return 0;
        for (uint32_t i = 0; i < nw; i++) {
            const uint32_t b = in.byte(q + 1 + i / 2);
            if (lane == 0) zlds[wb + ZD_WGT + i] = (uint8_t)((i & 1) ? (b & 15) : (b >> 4));
        }
    } else {  // FSE-compressed weights: two interleaved states over one table (log <= 6)
        used = 1 + hb;
        if (hb == 0 || q + used > qend) return 0;
        uint32_t wlog, wn;
        const uint32_t nc = read_ncount(in, wb, q + 1, q + used, 255, 6, wlog, wn, lane);
        if (!nc) return 0;
        build_fse(wb, wb + ZD_WT, wlog, wn, lane, 1);
        BitBack br;
        if (!br.init(in, q + 1 + nc, q + used)) return 0;
        uint32_t s1 = br.read(in, wlog), s2 = br.read(in, wlog);
        for (;;) {
            uint32_t e = zd32(wb + ZD_WT + 4 * s1);
            if (nw >= 255) return 0;
            if (lane == 0) zlds[wb + ZD_WGT + nw] = (uint8_t)(e & 0xFF);
            nw++;
            s1 = (e >> 17) + br.read(in, (e >> 13) & 15);
            if (br.pos < 0) {
                e = zd32(wb + ZD_WT + 4 * s2);
                if (nw >= 255) return 0;
                if (lane == 0) zlds[wb + ZD_WGT + nw] = (uint8_t)(e & 0xFF);
                nw++;
                break;
            }
            e = zd32(wb + ZD_WT + 4 * s2);
            if (nw >= 255) return 0;
            if (lane == 0) zlds[wb + ZD_WGT + nw] = (uint8_t)(e & 0xFF);
            nw++;
            s2 = (e >> 17) + br.read(in, (e >> 13) & 15);
            if (br.pos < 0) {
                e = zd32(wb + ZD_WT + 4 * s1);
                if (nw >= 255) return 0;
                if (lane == 0) zlds[wb + ZD_WGT + nw] = (uint8_t)(e & 0xFF);
                nw++;
                break;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    // the last weight is implied: the weights' 2^(w-1) must sum to a power of two
    uint32_t total = 0;
    for (uint32_t g = 0; g < nw; g += 64) {
        const uint32_t i = g + lane, w = i < nw ? zlds[wb + ZD_WGT + i] : 0u;
        if (w > 12) return 0;
        uint32_t v = w ? 1u << (w - 1) : 0u;
        for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
        total += v;
    }
    total = rfl(total);
    if (total == 0) return 0;
    hlog = hibit(total) + 1;
    if (hlog > 11) return 0;
    const uint32_t rest = (1u << hlog) - total;
    if (rest & (rest - 1)) return 0;
    if (lane == 0) zlds[wb + ZD_WGT + nw] = (uint8_t)(hibit(rest) + 1);
    __builtin_amdgcn_wave_barrier();
    const uint32_t nsym = nw + 1;
    // table: weight 1 first, symbols in order within a weight; 2^(w-1) entries each
    uint32_t start[13];
    {
        uint32_t cnt[13];
        for (uint32_t w = 0; w < 13; w++) cnt[w] = 0;
        for (uint32_t s = 0; s < nsym; s++) cnt[zlds[wb + ZD_WGT + s]]++;
        uint32_t acc = 0;
        for (uint32_t w = 1; w <= hlog; w++) { start[w] = acc; acc += cnt[w] << (w - 1); }
    }
    for (uint32_t s = 0; s < nsym; s++) {
        const uint32_t w = zlds[wb + ZD_WGT + s];
        if (!w) continue;
        const uint32_t len = 1u << (w - 1), e = s | ((hlog + 1 - w) << 8);
        for (uint32_t k = lane; k < len; k += 64) zd16(wb + ZD_HUF + 2 * (start[w] + k)) = (uint16_t)e;
        start[w] += len;
    }
    __builtin_amdgcn_wave_barrier();
    return used;
}

// Decode `n` Huffman literals of one stream [lo, hi) into lit[0..n): 64 at a time, lane k
// holding the k-th of each group, stored by one byte store per lane.
__device__ bool huf_stream(ZIn& in, uint32_t wb, uint32_t hlog, uint32_t lo, uint32_t hi, uint8_t* lit,
                           uint32_t n, uint8_t* trash, uint32_t lane) {
    BitBack br;
    if (!br.init(in, lo, hi)) return false;
    uint32_t acc = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t e = rfl(zd16(wb + ZD_HUF + 2 * br.peek(in, hlog)));
        br.pos -= (int32_t)(e >> 8);
        acc = (lane == (i & 63)) ? (e & 0xFF) : acc;
        if ((i & 63) == 63 || i + 1 == n)  // (no lane branch: masked-off lanes write the trash bytes)
            *(lane <= (i & 63) ? lit + (i & ~63u) + lane : trash + lane) = (uint8_t)acc;
    }
    return br.pos == 0;
}

__global__ __launch_bounds__(64 * ZSTD_WAVES) void k_zarr_zstd(const ZStream* __restrict__ st, uint32_t n,
                                                              const uint8_t* __restrict__ src,
                                                              uint8_t* __restrict__ dst,
                                                              uint8_t* __restrict__ litbuf,
                                                              uint32_t* __restrict__ err) {
    const uint32_t lane = threadIdx.x & 63, w = rfl(threadIdx.x >> 6);
    const uint32_t si = blockIdx.x * ZSTD_WAVES + w;
    if (si >= n) return;
    const ZStream t = st[si];
    const uint32_t wb = w * ZD_BYTES;
    ZIn in{InWin{src + t.src_off, wb + ZD_WIN, 0, lane}, rfl(t.csize)};
    in.win.load(0);
    OutRing<4096> o{wb + ZD_RING, dst + t.dst_off, 0, 0, t.dlen, lane, wb + ZD_TRASH};
    uint8_t* lit = litbuf + (size_t)si * ZSTD_LITSTRIDE;
    const uint32_t ilen = in.len;
    uint32_t bad = 0, q = 0;
#ifdef PBX_ZARR_DIAG  // diagnostic build only: stream 0's clocks (printf)
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    uint64_t clit = 0, cseq = 0, ctab = 0;
    uint32_t nlits = 0, nseqs = 0, nblk = 0, nfar = 0, nlitrun = 0;
    uint64_t cread = 0, ccopy = 0, cmatch = 0;
#define ZSD(...) __VA_ARGS__
#else
#define ZSD(...)
#endif
    // ---- frame header
    if (ilen < 6) bad = 1;
    const uint32_t magic = bad ? 0u : (uint32_t)in.le64_fwd(0);
    if (!bad && magic != 0xFD2FB528u) bad = 2;
    q = 4;
    const uint32_t fhd = bad ? 0u : in.byte(q++);
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did = fhd & 3;
    if (!bad && (fhd & 8)) bad = 3;  // reserved bit
    if (!single) q++;                // window descriptor (the whole frame is the window here)
    q += did == 0 ? 0u : did == 1 ? 1u : did == 2 ? 2u : 4u;
    if (!bad && did) bad = 4;        // no dictionaries
    const uint32_t fcs_size = fcs_flag == 0 ? (single ? 1u : 0u) : fcs_flag == 1 ? 2u : fcs_flag == 2 ? 4u : 8u;
    if (!bad && fcs_size) {
        uint64_t fcs = in.le64_fwd(q) & (fcs_size == 8 ? ~0ull : ((1ull << (8 * fcs_size)) - 1));
        if (fcs_size == 2) fcs += 256;
        if (fcs != t.dlen) bad = 5;
    }
    q += fcs_size;
    // ---- blocks
    uint32_t rep1 = 1, rep2 = 4, rep3 = 8;
    uint32_t hlog = 0, ll_log = 0, of_log = 0, ml_log = 0;
    bool have_huf = false, have_ll = false, have_of = false, have_ml = false;
    bool last = false;
    while (!bad && !last) {
        if (q + 3 > ilen) { bad = 6; break; }
        const uint32_t bh = (uint32_t)in.le64_fwd(q) & 0xFFFFFFu;
        q += 3;
        last = bh & 1;
        const uint32_t btype = (bh >> 1) & 3, bsize = bh >> 3;
        if (btype == 3) { bad = 7; break; }
        if (btype == 0) {  // raw
            if (q + bsize > ilen || bsize > o.olen - o.op) { bad = 8; break; }
            for (uint32_t k = 0; k < bsize; k += 64) {
                const uint32_t nb = bsize - k < 64 ? bsize - k : 64;
                const uint32_t v = in.win.lane_byte(q + k);
                o.put_if(lane < nb, o.op + k + lane, v);
                o.flush(o.op + k + nb);
            }
            o.op += bsize;
            q += bsize;
            continue;
        }
        if (btype == 1) {  // RLE: one byte, bsize times
            if (q + 1 > ilen || bsize > o.olen - o.op) { bad = 9; break; }
            const uint32_t v = in.byte(q++);
            for (uint32_t k = 0; k < bsize; k += 64) {
                const uint32_t nb = bsize - k < 64 ? bsize - k : 64;
                o.put_if(lane < nb, o.op + k + lane, v);
                o.flush(o.op + k + nb);
            }
            o.op += bsize;
            continue;
        }
        // ---- compressed block [q, bend)
        ZSD(const uint64_t b0 = __builtin_amdgcn_s_memtime(); nblk++;)
        const uint32_t bend = q + bsize;
        if (bend > ilen || bsize > ZSTD_LITBUF) { bad = 10; break; }
        const uint64_t lh = in.le64_fwd(q);
        const uint32_t ltype = (uint32_t)lh & 3, sf = ((uint32_t)lh >> 2) & 3;
        uint32_t nlit = 0;
        if (ltype < 2) {  // raw / RLE literals
            uint32_t hs;
            if (sf == 0 || sf == 2) { nlit = ((uint32_t)lh & 0xFF) >> 3; hs = 1; }
            else if (sf == 1) { nlit = ((uint32_t)lh & 0xFFFF) >> 4; hs = 2; }
            else { nlit = ((uint32_t)lh & 0xFFFFFF) >> 4; hs = 3; }
            q += hs;
            if (nlit > ZSTD_LITBUF) { bad = 11; break; }
            if (ltype == 0) {
                if (q + nlit > bend) { bad = 12; break; }
                for (uint32_t k = 0; k < nlit; k += 64) {
                    const uint32_t v = in.win.lane_byte(q + k);
                    if (k + lane < nlit) lit[k + lane] = (uint8_t)v;
                }
                q += nlit;
            } else {
                if (q + 1 > bend) { bad = 13; break; }
                const uint32_t v = in.byte(q++);
                for (uint32_t k = lane; k < nlit; k += 64) lit[k] = (uint8_t)v;
            }
        } else {  // Huffman-coded literals (2: with a tree, 3: treeless)
            uint32_t hs, nbits;
            const bool four = sf != 0;
            if (sf < 2) { hs = 3; nbits = 10; } else if (sf == 2) { hs = 4; nbits = 14; } else { hs = 5; nbits = 18; }
            nlit = (uint32_t)(lh >> 4) & ((1u << nbits) - 1);
            const uint32_t csize = (uint32_t)(lh >> (4 + nbits)) & ((1u << nbits) - 1);
            q += hs;
            if (nlit > ZSTD_LITBUF || q + csize > bend) { bad = 14; break; }
            uint32_t lq = q;
            const uint32_t lend = q + csize;
            if (ltype == 2) {
                const uint32_t used = read_huf_tree(in, wb, lq, lend, hlog, lane);
                if (!used) { bad = 15; break; }
                lq += used;
                have_huf = true;
            } else if (!have_huf) {
                bad = 16;
                break;
            }
            if (!four) {
                if (!huf_stream(in, wb, hlog, lq, lend, lit, nlit, lit + ZSTD_LITBUF, lane)) { bad = 17; break; }
            } else {
                if (lq + 6 > lend) { bad = 18; break; }
                const uint64_t jt = in.le64_fwd(lq);
                const uint32_t s1 = (uint32_t)jt & 0xFFFF, s2 = (uint32_t)(jt >> 16) & 0xFFFF,
                               s3 = (uint32_t)(jt >> 32) & 0xFFFF;
                const uint32_t a = lq + 6, b2 = a + s1, c2 = b2 + s2, d2 = c2 + s3;
                if (d2 > lend) { bad = 19; break; }
                const uint32_t per = (nlit + 3) / 4;
                if (3 * per > nlit) { bad = 20; break; }
                if (!huf_stream(in, wb, hlog, a, b2, lit, per, lit + ZSTD_LITBUF, lane) ||
                    !huf_stream(in, wb, hlog, b2, c2, lit + per, per, lit + ZSTD_LITBUF, lane) ||
                    !huf_stream(in, wb, hlog, c2, d2, lit + 2 * per, per, lit + ZSTD_LITBUF, lane) ||
                    !huf_stream(in, wb, hlog, d2, lend, lit + 3 * per, nlit - 3 * per, lit + ZSTD_LITBUF, lane)) {
                    bad = 21;
                    break;
                }
            }
            q = lend;
        }
        // the literals just stored are read back by this wave below
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        ZSD(const uint64_t b1 = __builtin_amdgcn_s_memtime(); clit += b1 - b0; nlits += nlit;)
        // ---- sequences section
        if (q >= bend) { bad = 22; break; }
        uint32_t nseq = in.byte(q++);
        if (nseq >= 128) {
            if (nseq < 255) {
                if (q >= bend) { bad = 23; break; }
                nseq = ((nseq - 128) << 8) + in.byte(q++);
            } else {
                if (q + 2 > bend) { bad = 23; break; }
                nseq = in.byte(q) + (in.byte(q + 1) << 8) + 0x7F00;
                q += 2;
            }
        }
        uint32_t lp = 0;  // literals consumed
        // the literals through a register window: literals [lwb, lwb + 256) one dword per lane
        // in lcur, the next 256 in lnxt (loaded a window ahead: no HBM wait per sequence)
        auto lit_word = [&](uint32_t i) -> uint32_t {
            const uint32_t at = i + 4 * lane < ZSTD_LITBUF - 4 ? i + 4 * lane : ZSTD_LITBUF - 4;
            return *(const __attribute__((address_space(1))) uint32_t*)(lit + at);
        };
        uint32_t lwb = 0, lcur = lit_word(0), lnxt = lit_word(256);
        auto copy_lits = [&](uint32_t n2) -> bool {
            if (lp + n2 > nlit || n2 > o.olen - o.op) return false;
            for (uint32_t k = 0; k < n2; k += 64) {
                while (lp + k >= lwb + 256) {
                    lcur = lnxt;
                    lwb += 256;
                    lnxt = lit_word(lwb + 256);
                }
                const uint32_t nb = n2 - k < 64 ? n2 - k : 64;
                const uint32_t wi = lp + k + lane - lwb;  // < 320
                const uint32_t a = (uint32_t)__shfl((int)lcur, (int)((wi >> 2) & 63), 64);
                const uint32_t b = (uint32_t)__shfl((int)lnxt, (int)((wi >> 2) & 63), 64);
                const uint32_t v = ((wi < 256 ? a : b) >> ((wi & 3) * 8)) & 0xFFu;
                o.put_if(lane < nb, o.op + k + lane, v);
                o.flush(o.op + k + nb);
            }
            o.op += n2;
            lp += n2;
            return true;
        };
        if (nseq == 0) {
            if (q != bend || !copy_lits(nlit)) bad = 24;
            q = bend;
            continue;
        }
        if (q >= bend) { bad = 25; break; }
        const uint32_t modes = in.byte(q++);
        if (modes & 3) { bad = 26; break; }
        int32_t u = seq_table(in, wb, wb + ZD_LL, 0, modes >> 6, q, bend, c_ll_def, 36, 6, 35, 9, ll_log, have_ll, lane);
        if (u < 0) { bad = 27; break; }
        q += (uint32_t)u;
        u = seq_table(in, wb, wb + ZD_OF, 1, (modes >> 4) & 3, q, bend, c_of_def, 29, 5, 31, 8, of_log, have_of, lane);
        if (u < 0) { bad = 28; break; }
        q += (uint32_t)u;
        u = seq_table(in, wb, wb + ZD_ML, 2, (modes >> 2) & 3, q, bend, c_ml_def, 53, 6, 52, 9, ml_log, have_ml, lane);
        if (u < 0) { bad = 29; break; }
        q += (uint32_t)u;
        ZSD(const uint64_t b2 = __builtin_amdgcn_s_memtime(); ctab += b2 - b1; nseqs += nseq;)
        BitBack br;
        if (!br.init(in, q, bend)) { bad = 30; break; }
        uint32_t lls = br.read(in, ll_log), ofs = br.read(in, of_log), mls = br.read(in, ml_log);
        // the next sequence's three table entries are read as soon as its states are known
        // (the LDS latency overlaps the batch bookkeeping); uniform values, taken at the top
        uint32_t pe_l = zd32(wb + ZD_LL + 4 * lls), pe_o = zd32(wb + ZD_OF + 4 * ofs),
                 pe_m = zd32(wb + ZD_ML + 4 * mls);
        // Sequences are decoded into a batch (lane j: sequence j's literal length, match length
        // and offset) and a batch of up to 64 is executed byte-parallel: output offsets by prefix
        // sums, then 64 output bytes per step, each lane finding its sequence (start flags,
        // ballot, mbcnt) and its byte: a literal (register window), a ring byte, an HBM byte
        // (offsets beyond the ring) or, for a source inside the step, by pointer jumping.
        uint32_t bll = 0, bml = 0, boff = 0, bn = 0;
        auto exec_batch = [&]() -> bool {
            const uint32_t sll = lane < bn ? bll : 0u;
            const uint32_t lend = wave_incl_add(sll, lane), lst = lend - sll;  // literal index of each sequence
            const uint32_t TL = rdl(lend, 63);
            if (lp + TL > nlit) return false;
            const bool ok = seq_batch(o, wb + ZD_FLAG, lane, bn, bll, bml, boff, lst,
                                      [&](uint32_t li, uint32_t lfirst, bool any) -> uint32_t {
                // literal lp + li from the register window (the step's are consecutive)
                if (any)
                    while (lp + lfirst >= lwb + 256) {
                        lcur = lnxt;
                        lwb += 256;
                        lnxt = lit_word(lwb + 256);
                    }
                const uint32_t wi = lp + li - lwb;  // < 320 on literal lanes
                const uint32_t a = (uint32_t)__shfl((int)lcur, (int)((wi >> 2) & 63), 64);
                const uint32_t b2 = (uint32_t)__shfl((int)lnxt, (int)((wi >> 2) & 63), 64);
                return ((wi < 256 ? a : b2) >> ((wi & 3) * 8)) & 0xFFu;
            });
            lp += TL;
            bn = 0;
            return ok;
        };
        for (uint32_t i = 0; i < nseq; i++) {
            ZSD(const uint64_t s0 = __builtin_amdgcn_s_memtime();)
            // (The sequence state is wave-uniform but left where LLVM puts it, much of it in
            // VGPRs: pinning it all to SGPRs put the loop on the CU's one scalar unit, which
            // eight frames per CU saturate; 45.6 -> 54.7 GB/s without the pins.)
            const uint32_t le = pe_l, oe = pe_o, me = pe_m;  // (every lane the same)
            // (the tables hold only symbols read_ncount / the RLE mode checked against the
            // alphabets: offset codes <= 31, every length code valid)
            const uint32_t ofc = oe & 0x1F;
            // the four code tables up front (scalar loads, one wait)
            const uint32_t llx = le & 31, mlx = me & 31;
            const uint32_t llb = (le & 32) ? 1u << llx : (le >> 6) & 127;
            const uint32_t mlb = (me & 32) ? (1u << mlx) + 3 : (me >> 6) & 127;
            // every bit this sequence reads (offset, match and literal length extra bits, then
            // the three state updates) in one read when they fit 56 bits: the fields are
            // shifts of one value instead of six dependent reads
            const uint32_t nbl = (le >> 13) & 15, nbm = (me >> 13) & 15, nbo = (oe >> 13) & 15;
            const uint32_t nup = i + 1 < nseq ? nbl + nbm + nbo : 0u;
            const uint32_t T = ofc + mlx + llx + nup;
            uint32_t ofx, mlv, llv;
            uint64_t all = 0;
            if (T <= 56) {
                all = br.read64(in, T);
                ofx = (uint32_t)(all >> (T - ofc)) & ((1u << ofc) - 1u);
                mlv = (uint32_t)(all >> (T - ofc - mlx)) & ((1u << mlx) - 1u);
                llv = (uint32_t)(all >> (T - ofc - mlx - llx)) & ((1u << llx) - 1u);
            } else {
                ofx = br.read(in, ofc);
                mlv = br.read(in, mlx);
                llv = br.read(in, llx);
            }
            const uint32_t ofv = (1u << ofc) + ofx;
            const uint32_t ml = mlb + mlv;
            const uint32_t ll = llb + llv;
            uint32_t off;
            if (ofv > 3) {
                off = ofv - 3;
                rep3 = rep2; rep2 = rep1; rep1 = off;
            } else {
                const uint32_t idx = ofv - 1 + (ll == 0 ? 1u : 0u);  // 0..3
                if (idx == 0) {
                    off = rep1;
                } else if (idx == 1) {
                    off = rep2;
                    rep2 = rep1; rep1 = off;
                } else if (idx == 2) {
                    off = rep3;
                    rep3 = rep2; rep2 = rep1; rep1 = off;
                } else {
                    off = rep1 - 1;
                    rep3 = rep2; rep2 = rep1; rep1 = off;
                }
            }
            if (i + 1 < nseq) {  // state updates: literal lengths, match lengths, offsets
                if (T <= 56) {
                    lls = (le >> 17) + ((uint32_t)(all >> (nbm + nbo)) & ((1u << nbl) - 1u));
                    mls = (me >> 17) + ((uint32_t)(all >> nbo) & ((1u << nbm) - 1u));
                    ofs = (oe >> 17) + ((uint32_t)all & ((1u << nbo) - 1u));
                } else {
                    lls = (le >> 17) + br.read(in, nbl);
                    mls = (me >> 17) + br.read(in, nbm);
                    ofs = (oe >> 17) + br.read(in, nbo);
                }
                pe_l = zd32(wb + ZD_LL + 4 * lls);
                pe_o = zd32(wb + ZD_OF + 4 * ofs);
                pe_m = zd32(wb + ZD_ML + 4 * mls);
            }
            ZSD(cread += __builtin_amdgcn_s_memtime() - s0;)
            ZSD(const uint64_t s1 = __builtin_amdgcn_s_memtime(); nfar += off > 4096; nlitrun += ll > 0;)
            bll = lane == bn ? ll : bll;
            bml = lane == bn ? ml : bml;
            boff = lane == bn ? off : boff;
            bn++;
            if (bn == 64 || i + 1 == nseq) {
                bn = rfl(bn);
                if (!exec_batch()) { bad = 33; break; }
            }
            ZSD(cmatch += __builtin_amdgcn_s_memtime() - s1;)
        }
        if (bad) break;
        if (br.pos != 0) { bad = 34; break; }
        if (!copy_lits(nlit - lp)) { bad = 35; break; }
        ZSD(cseq += __builtin_amdgcn_s_memtime() - b2;)
        q = bend;
    }
    ZSD(if (si == 0 && lane == 0) printf("[zstd] total %lu literals %lu tables %lu sequences %lu (read %lu copy %lu match %lu) blocks %u nlit %u nseq %u far %u litruns %u dlen %u\n",
        (unsigned long)(__builtin_amdgcn_s_memtime() - c0), (unsigned long)clit, (unsigned long)ctab,
        (unsigned long)cseq, (unsigned long)cread, (unsigned long)ccopy, (unsigned long)cmatch, nblk, nlits, nseqs, nfar, nlitrun, t.dlen);)
    uint32_t want = 0;
    if (!bad && checksum) {
        if (q + 4 > ilen) bad = 36;
        else want = (uint32_t)in.le64_fwd(q);
        q += 4;
    }
    if (!bad && (o.op != o.olen || q > ilen)) bad = 36;
    o.finish();
    if (!bad && checksum) {
        // the content checksum over the output this wave stored: its stores complete and the
        // vector L1 invalidated (agent-scope fence), then read back
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        if ((uint32_t)xxh64_wave(dst + t.dst_off, t.dlen, lane) != want) bad = 37;
    }
    if (lane == 0) err[si] = bad;
}

size_t zstd_scratch_bytes(uint32_t nstreams) { return (size_t)nstreams * ZSTD_LITSTRIDE; }

hipError_t launch_zarr_zstd(hipStream_t st, const ZStream* d_streams, uint32_t n, const uint8_t* src,
                            uint8_t* scratch, uint8_t* litbuf, uint32_t* err) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_zarr_zstd, dim3((n + ZSTD_WAVES - 1) / ZSTD_WAVES), dim3(64 * ZSTD_WAVES),
                       ZSTD_WAVES * ZD_BYTES, st, d_streams, n, src, scratch, litbuf, err);
    return hipGetLastError();
}

}  // namespace pbx
