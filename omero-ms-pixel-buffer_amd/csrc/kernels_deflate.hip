// kernels_deflate.hip — gfx950 kernels of the zlib/PNG/TIFF encoder (writeImage,
// TileRequestHandler.java:176-199), one deflate block per <= 16 KiB segment of a tile's
// filtered stream (deflate_seg.h):
//
//   k_lz77        512 threads / segment: window + segment in LDS, first-occurrence hash,
//                 wave-serial greedy/lazy parse, symbol histogram, Adler-32 partials
//   k_huff        ONE WAVE / Huffman block of up to 64 segments (many per CU): code
//                 lengths and canonical codes, code-length RLE, the block header bits, the
//                 exact output size, every segment's bit range
//   k_seg_sizes   per tile: segment byte offsets and container size -> k_scan_offsets
//   k_encode      512 threads / segment: bit packing of every token into LDS, CRC-32, and
//                 the bytes stored straight into the compacted output at their final place
//   k_frame       per tile: zlib header + Adler-32 (combined), PNG chunks with the IDAT
//                 CRC-32 combined from the segments (APNGWriter layout), or the TIFF header
//
// LDS / ALU / latency-bound integer work; no MFMA.  Splitting the segment's work over three
// kernels gives each its own occupancy: k_lz77 and k_encode hold ~46-50 KB of LDS
// (4 workgroups per CU), k_huff 8.9 KB per wave, so the serial Huffman merge of many
// segments overlaps on every CU.
#include <mutex>
#include <hip/hip_runtime.h>

#include "deflate_seg.h"
#include "dev_util.h"
#include "pbx_common.h"
#include "pbx_config.h"
#include "pbx_kernels.h"

namespace pbx {

using DC = DeflateMainCfg;
constexpr uint32_t STAMP_STRIDE = 32;  // diagnostics: k_lz77 0.., k_huff 8.., k_encode 24..

// ------------------------------------------------------------------- LDS layouts
// A match record of k_lz77 in LDS: position in the wave's sub-segment (11 bits), length - 3
// (8 bits), candidate index (2 bits: distance 1, 2 or one row), unpacked into the mrec form
// (pos | (len - 3) << 16, dist - 1) when written to HBM.  4 KB less than two arrays: the room
// for 8 histogram copies at 4 workgroups per CU.
#ifndef PBX_LZ_HCOPIES
#define PBX_LZ_HCOPIES 8  // experiments: histogram copies (a power of two, >= 8)
#endif
constexpr uint32_t LZ_HCOPIES = PBX_LZ_HCOPIES;
template <class C>
struct LzSmem {
    static_assert(C::SUB == 2048, "11-bit sub-segment positions in the packed match records");
    alignas(16) uint32_t buf[C::BUFW];
    uint32_t mrl[C::NW * C::MAXMW];
    uint32_t w_nm[C::NW];
    // per repair round (double-buffered by round parity): a wave's last match end when it runs
    // into the next wave (else 0), and the start its current records were walked from
    // (0xFFFFFFFF: a wave whose walk is skipped, any start gives the same result)
    uint32_t w_end[2][C::NW];
    uint32_t reachw;  // PBX_LZ_REACH_MASKS: bit b = the boundary after wave b can be reached
    uint32_t dbg_walk, dbg_round;  // PBX_PHASE_PROFILE: walk steps of the workgroup, repair rounds
    uint32_t dbg_twalk, dbg_tsync;  // PBX_LZ_WALK_PROF: wave 0's cycles in walks / in the rounds' barriers and checks
    uint32_t w_st[2][C::NW];
    // literal/length histogram, LZ_HCOPIES interleaved copies (lane & 7): lanes of different
    // copies never share a bank, same-symbol atomics of one instruction spread over 8 words
    alignas(16) uint32_t h8[288 * LZ_HCOPIES];
    uint32_t hdummy[64];  // per-lane sink of the branch-free histogram (covered positions)
    uint32_t dfreq[32];
    uint32_t red[3 * C::NW];
#ifdef PBX_LZ_PAD_LDS  // experiments only: LDS a prefetch ring would take (occupancy probe)
    uint32_t pad[PBX_LZ_PAD_LDS / 4];
#endif
};

// Per-tree arrays of the literal/length tree (288 slots) and the distance tree (32 slots)
// back to back: a[T] is tree T's part, as with a [2][288] array, at 320 slots instead of 576.
template <class E, uint32_t N0, uint32_t N1>
struct Split2 {
    E v[N0 + N1];
    __device__ E* operator[](uint32_t T) { return v + (T ? N0 : 0u); }
    __device__ const E* operator[](uint32_t T) const { return v + (T ? N0 : 0u); }
};

// The tree-building scratch (keys, merge records, parents, depths, merge rounds) is dead
// once the code lengths exist; the code-length RLE, the code-length code, the header bits
// and the RLE counts then reuse its bytes.  The merge rounds' merged prefix (<= 288
// entries: the queue never holds more than the leaves) lives in leafpar, written only
// after the rounds.  8.9 KB: 18 one-wave workgroups per CU.
struct HuffScratchDev {
    uint32_t skey[KEYN];
    Split2<uint32_t, 288, 32> rec;      // step s: li0 | qi0 << 10 | cnt << 20
    Split2<uint16_t, 288, 32> leafpar;  // (merge rounds: the merged prefix)
    union {
        struct {
            Split2<uint16_t, 288, 32> aA, dB;
        };
        // merge rounds: the internal nodes' weights, 32-bit (a block of up to BLK_SEGS
        // segments counts far more than 65535 symbols); aA and dB are written after them
        Split2<uint32_t, 288, 32> iw;
    };
    Split2<uint16_t, 290, 34> rst;      // first internal node of every merge round (+ the end)
};

template <class C>
struct HuffSmem {
    uint32_t lfreq[288], dfreq[32];
    uint32_t lcode[288], dcode[32];
    uint32_t hblc[2][16], hover[2], hstart[2][16], hnext[2][16];
    uint32_t lbm[16 * 9], dbm[16];
    uint32_t misc[M_NMISC];
    uint32_t nrounds[2];
    uint32_t dk[BLK_SEGS];  // token bits of every segment of the block under its code
    uint32_t sls[BLK_SEGS];  // stream bytes of every segment
    union {
        HuffScratchDev hs;
        struct {  // from ph_rle_init on
            HuffWork hw;
            uint32_t rle[320], rboff[RLEN], rbm[10];
            uint32_t hdrw[C::HDRW];
            uint32_t rcnt[RLEN];
        };
    };
};

// The CRC combine tables of k_encode (words): per-lane distance operators x^(8*32*m) (TA,
// m = 0..7 chunks) and x^(8*256*m) (TB, 8-chunk steps), then the wave-distance operators
// x^(8*2048*2^k) (TW, k = 0..2), each as nibble tables (crc_lane_tables below).
constexpr uint32_t CRCX_TA = 0, CRCX_TB = 1024, CRCX_TW = 2048, CRCX_WORDS = 2048 + 3 * 128;
#ifndef PBX_CRC_SLICES
#define PBX_CRC_SLICES 4  // k_encode's CRC: slicing-by-4 (8: slicing-by-8, measured slower: r03_p7)
#endif
static_assert(PBX_CRC_SLICES == 4 || PBX_CRC_SLICES == 8, "slicing by 4 or 8");
template <class C>
struct EncSmem {
    union {
        struct {
            uint32_t mpos[C::NW * C::MAXMW];
            uint16_t mdist[C::NW * C::MAXMW];
        };
        alignas(16) uint32_t crcx[CRCX_WORDS];  // CRC combine tables once the slots are built
    };
    uint32_t w_nm[C::NW];
    uint32_t lcode[289], dcode[32];  // slot form; lcode[288] = no token
    alignas(16) uint32_t out[(C::OUTW + 3) & ~3];
    alignas(16) uint32_t crc_t[PBX_CRC_SLICES][256];
    uint32_t wtot[16];
    uint32_t red[C::NW];
    uint32_t crc_acc, ndone;  // PBX_ENC_LAST_WAVE: the waves' CRC terms XOR-ed, waves done
};
static_assert(CRCX_WORDS * 4 <= DC::NW * DC::MAXMW * 6, "the CRC combine tables fit the match lists' room");
static_assert(sizeof(EncSmem<DC>) * 512 <= 40 * 1024 * DC::NT, "32 encode waves per CU (160 KiB LDS)");

// Slicing-by-4 (or 8) CRC-32 tables, built at compile time into device memory (copied to LDS).
struct CrcTables {
    uint32_t t[PBX_CRC_SLICES][256];
};
constexpr uint32_t crc_entry_c(uint32_t n) {
    uint32_t c = n;
    for (int k = 0; k < 8; k++) c = (c & 1) ? CRC_POLY ^ (c >> 1) : c >> 1;
    return c;
}
constexpr CrcTables make_crc_tables() {
    CrcTables T{};
    for (uint32_t i = 0; i < 256; i++) T.t[0][i] = crc_entry_c(i);
    for (int k = 1; k < PBX_CRC_SLICES; k++)
        for (uint32_t i = 0; i < 256; i++) T.t[k][i] = (T.t[k - 1][i] >> 8) ^ T.t[0][T.t[k - 1][i] & 0xFF];
    return T;
}
__constant__ const CrcTables kCrcTables = make_crc_tables();

// The CRC combine multiplies by constant operators K mod P.  b -> K*b mod P is GF(2)-linear,
// so it is 8 lookups in nibble tables T[j][v] = K*(v << 4j) instead of a 32-step
// shift-and-reduce loop.  A thread's chunk CRC is moved to the end of its wave's 2 KiB by
// x^(8*32*dl), dl = 63 - lane = 8 mb + ma: TA (operator ma) then TB (operator mb), both laid
// out [j][v][m] (lanes of one lookup use different m: the layout spreads them over banks);
// the wave's XOR is moved to the segment end by TW levels k (x^(8*2048*2^k), [k][j][v]).
struct CrcLaneTables {
    uint32_t t[CRCX_WORDS];
};
constexpr uint32_t crc_pow_c(uint32_t base, uint32_t m) {  // base^m mod P
    uint32_t p = 1u << 31;
    for (uint32_t i = 0; i < m; i++) p = crc_multmodp_c(base, p);
    return p;
}
constexpr CrcLaneTables make_crc_lane_tables() {
    CrcLaneTables T{};
    const X8Table x = make_x8();
    static_assert(DC::CRCC == 32, "x.v[5] = 32 bytes, x.v[8] = 256, x.v[11] = 2048");
    for (uint32_t m = 0; m < 8; m++) {
        const uint32_t ka = crc_pow_c(x.v[5], m), kb = crc_pow_c(x.v[8], m);
        for (uint32_t j = 0; j < 8; j++)
            for (uint32_t v = 0; v < 16; v++) {
                T.t[CRCX_TA + j * 128 + v * 8 + m] = crc_multmodp_c(ka, v << (4 * j));
                T.t[CRCX_TB + j * 128 + v * 8 + m] = crc_multmodp_c(kb, v << (4 * j));
            }
    }
    for (uint32_t k = 0; k < 3; k++)
        for (uint32_t j = 0; j < 8; j++)
            for (uint32_t v = 0; v < 16; v++)
                T.t[CRCX_TW + k * 128 + j * 16 + v] = crc_multmodp_c(x.v[11 + k], v << (4 * j));
    return T;
}
__constant__ const CrcLaneTables kCrcLane = make_crc_lane_tables();

// x^(8n) mod P for n < 2^16 from two tables: x^(8v) and x^(8*256*v).
struct CrcPowTables {
    uint32_t lo[256], hi[256];
};
constexpr CrcPowTables make_crc_pow() {
    CrcPowTables T{};
    X8Table x = make_x8();
    for (uint32_t v = 0; v < 256; v++) {
        uint32_t p = 1u << 31;
        for (int k = 0; k < 8; k++)
            if ((v >> k) & 1u) p = crc_multmodp_c(x.v[k], p);
        T.lo[v] = p;
    }
    for (uint32_t v = 0; v < 256; v++) {
        uint32_t p = 1u << 31;
        for (int k = 0; k < 8; k++)
            if ((v >> k) & 1u) p = crc_multmodp_c(x.v[8 + k], p);
        T.hi[v] = p;
    }
    return T;
}
__constant__ const CrcPowTables kCrcPow = make_crc_pow();

// b * (operator m of a [j][v][m] table at t)
__device__ __forceinline__ uint32_t crc_mul_lane(const uint32_t* t, uint32_t m, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) r ^= t[j * 128 + ((b >> (4 * j)) & 0xFu) * 8 + m];
    return r;
}
// b * (the operator of a [j][v] table at t)
__device__ __forceinline__ uint32_t crc_mul_tab(const uint32_t* t, uint32_t b) {
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) r ^= t[j * 16 + ((b >> (4 * j)) & 0xFu)];
    return r;
}
// Sum of x over the wave (row scans by DPP shifts, then the four row totals), uniform.
__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 15) + (uint32_t)__builtin_amdgcn_readlane((int)x, 31) +
           (uint32_t)__builtin_amdgcn_readlane((int)x, 47) + (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
// XOR of x over the wave (row scans by DPP shifts, then the four row totals), uniform.
__device__ __forceinline__ uint32_t wave_xor(uint32_t x) {
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 15) ^ (uint32_t)__builtin_amdgcn_readlane((int)x, 31) ^
           (uint32_t)__builtin_amdgcn_readlane((int)x, 47) ^ (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

__device__ __forceinline__ uint32_t crc_x8n_small(uint32_t n) {  // n < 2^16
    return crc_multmodp(kCrcPow.lo[n & 0xFFu], kCrcPow.hi[(n >> 8) & 0xFFu]);
}
// Per byte count n < CRC_TAB_N (any segment's compressed bytes): x^(8n) mod P (the crc32_combine
// operator) and the standard CRC-32 of n bytes whose zero-init CRC is 0 (crc_from_raw's
// constant term), filled once per device by k_crc_tables.  k_encode's last step is then two
// loads instead of two 32-step carry-less products on one lane.
constexpr uint32_t CRC_TAB_N = 32768;
__device__ uint32_t g_crc_x8n[CRC_TAB_N];
__device__ uint32_t g_crc_fin[CRC_TAB_N];
__global__ __launch_bounds__(256) void k_crc_tables() {
    const uint32_t n = blockIdx.x * 256 + threadIdx.x;
    if (n >= CRC_TAB_N) return;
    const uint32_t op = crc_x8n_small(n);
    g_crc_x8n[n] = op;
    g_crc_fin[n] = crc_from_raw(0u, op);
}

// Segment geometry from the tile descriptor.
__device__ __forceinline__ SegParams seg_params(const TileDesc& d, uint32_t k) {
    SegParams sp;
    const uint64_t s = (uint64_t)k * d.seg_len;
    sp.sl = (uint32_t)((d.stream_len - s) < d.seg_len ? (d.stream_len - s) : d.seg_len);
    sp.wl = seg_window<DC>(s, d.rowlen);
    sp.base = s - sp.wl;
    sp.rowlen = d.rowlen;
    sp.last = (k + 1 == d.seg_count) ? 1u : 0u;
    return sp;
}

// 16-byte loads of nb stream bytes (16-byte aligned source, slack after every tile) into
// LDS words; bytes from nb up to nz (>= nb + 16, a multiple of 16) are zero.
template <int NT>
__device__ __forceinline__ void load_bytes16(uint32_t* dst, const uint8_t* src, uint32_t nb,
                                             uint32_t nz, uint32_t tid) {
    const uint32_t nv = (nb + 15) / 16;
    for (uint32_t k = tid; k < nz / 16; k += NT) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (k < nv) {
            v = *(const uint4*)(src + 16ull * k);
            const uint32_t rem = nb - 16 * k;
            if (rem < 16) {
                uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int keep = (int)rem - 4 * i;
                    w[i] = keep >= 4 ? w[i] : keep <= 0 ? 0u : w[i] & ((1u << (8 * keep)) - 1u);
                }
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
        }
        *(uint4*)(dst + 4 * k) = v;
    }
}

// Stream bytes of a TF_DIRECT tile assembled in LDS straight from the plane in HBM
// (getTileDirect + the APNGWriter scanline of filter None, TileRequestHandler.java:107-109,
// 176-199): the bytes k_rows would have written to a stream buffer.  Row r of the stream is
// [0] ++ the big-endian row (PNG) or the row alone (deflate-TIFF).  Source rows start 16-byte
// aligned (the planner checks x * bpp % 16; the pitch is a multiple of 256).
//
// One wave per (row, 64 chunks of 16 bytes): lane t loads chunk c = 64 g + t of the row
// (one coalesced 16-byte load, swapped / sign-flipped in registers) and stores it at LDS
// byte Q + 16 c, Q = the row's first data byte, with ONE unaligned ds_write_b128 (gfx950
// LDS takes byte-aligned accesses; chunks never share a byte).  Lanes at the buffer edges or
// with a partial last chunk write byte by byte; the filter bytes (0) go with chunk 0.  The
// loads of up to three rows are in flight at once.
struct DirectRows {
    const uint8_t* row0;  // region row 0 in the plane
    int64_t pitch;
    uint32_t rowlen, rb, fb, h, nc, ngrp;
    int32_t bpp;
    bool swap, flip, aligned;
    uint32_t rcp;  // recip32(rowlen): stream offset -> row without a division
    __device__ __forceinline__ void init(const TileDesc& d) {
        row0 = d.plane + (int64_t)d.y * d.pitch + (int64_t)d.x * d.bpp;
        pitch = d.pitch;
        fb = (d.flags & TF_PNGROWS) ? 1u : 0u;
        rowlen = d.rowlen;
        rcp = d.rowlen_rcp;
        rb = rowlen - fb;
        h = (uint32_t)d.h;
        nc = (rb + 15) >> 4;
        ngrp = (nc + 63) >> 6;
        bpp = d.bpp;
        swap = (d.flags & TF_SWAP) != 0;
        flip = (d.flags & TF_FLIP) != 0;
        aligned = (rb & 15u) == 0;  // rows of whole chunks: aligned stores (fill_stores)
    }
};

// LDS bytes [0, nb) = stream bytes [B, B + nb) of the tile, zero from nb up to nz (a
// multiple of 4).  NT threads; wave w takes tasks w, w + NW, ... of (row, chunk group), K
// tasks per batch (the loads of a batch are in flight together).  Split in two so that the
// first batch's loads can be issued one segment ahead (k_lz77's prefetch): fill_issue loads
// batch 0 into registers, fill_finish stores it and does the other batches.
template <uint32_t K>
struct FillPre {
    uint4 v[K];
    uint4 pv;  // aligned fill: lane 0's chunk before the first task's (prev group / row)
};

struct FillGeom {
    uint32_t ra, rz, ntask;
    __device__ __forceinline__ FillGeom(const DirectRows& dr, uint32_t B, uint32_t nb) {
        ra = div_rcp(B, dr.rowlen, dr.rcp);
        rz = div_rcp(B + nb - 1, dr.rowlen, dr.rcp);
        ntask = (rz - ra + 1) * dr.ngrp;
    }
};

// A wave's K tasks are consecutive (k0 .. k0+K-1): the chunk before a task's first is the
// previous task's last (a readlane), except for the first task, whose lane 0 loads it (pv).
template <int NT, uint32_t K>
__device__ __forceinline__ void fill_loads(uint4 (&v)[K], uint4& pv, const DirectRows& dr,
                                           const FillGeom& g, uint32_t k0, uint32_t lane) {
#pragma unroll
    for (uint32_t j = 0; j < K; j++) {
        const uint32_t k = k0 + j < g.ntask ? k0 + j : k0;
        const uint32_t i = dr.ngrp == 1 ? k : k / dr.ngrp;
        const uint32_t c0 = (k - i * dr.ngrp) * 64;
        const uint8_t* rp = dr.row0 + (int64_t)(g.ra + i) * dr.pitch + 16 * c0;
#ifdef PBX_LZ_FAKE_LOAD  // timing experiment only (scripts/variants.sh): hashed bytes, no plane reads
        {
            const uint64_t h = splitmix64((uint64_t)(uintptr_t)(rp + 16 * lane));
            v[j] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)(h * 3), (uint32_t)(h >> 17));
        }
#else
        v[j] = gload16(rp + 16 * (c0 + lane < dr.nc ? lane : 0u));
#endif
        if (j == 0 && dr.aligned) {  // lane 0: the chunk before (previous group, or the row above's last)
            pv = make_uint4(0, 0, 0, 0);
            if (lane == 0 && (c0 > 0 || g.ra + i > 0))
                pv = gload16(c0 > 0 ? rp - 16 : rp - dr.pitch + 16 * (dr.nc - 1));
        }
    }
}

// Bytes [16 - s, 16) of p followed by bytes [0, 16 - s) of x (little-endian 16-byte words),
// s uniform in 0..15.
__device__ __forceinline__ uint4 funnel16(const uint4& p, const uint4& x, uint32_t s) {
    const uint32_t z[8] = {p.x, p.y, p.z, p.w, x.x, x.y, x.z, x.w};
    const uint32_t q = (16 - s) >> 2, r = (16 - s) & 3;
    uint32_t o[4];
    switch (__builtin_amdgcn_readfirstlane(q)) {
    case 0:
#pragma unroll
        for (int k = 0; k < 4; k++) o[k] = __builtin_amdgcn_alignbyte(z[k + 1], z[k], r);
        break;
    case 1:
#pragma unroll
        for (int k = 0; k < 4; k++) o[k] = __builtin_amdgcn_alignbyte(z[k + 2], z[k + 1], r);
        break;
    case 2:
#pragma unroll
        for (int k = 0; k < 4; k++) o[k] = __builtin_amdgcn_alignbyte(z[k + 3], z[k + 2], r);
        break;
    case 3:
#pragma unroll
        for (int k = 0; k < 4; k++) o[k] = __builtin_amdgcn_alignbyte(z[k + 4], z[k + 3], r);
        break;
    default:  // s == 0
#pragma unroll
        for (int k = 0; k < 4; k++) o[k] = z[k + 4];
        break;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

template <int NT, uint32_t K>
__device__ __forceinline__ void fill_stores(const uint4 (&v)[K], const uint4& pv, uint8_t* bb,
                                            const DirectRows& dr, const FillGeom& g, uint32_t B,
                                            uint32_t nb, uint32_t k0, uint32_t lane) {
    uint4 xlast = make_uint4(0, 0, 0, 0);  // the previous task's last chunk (uniform)
#pragma unroll
    for (uint32_t j = 0; j < K; j++) {
        const uint32_t k = k0 + j;
        if (k >= g.ntask) break;  // uniform
        const uint32_t i = dr.ngrp == 1 ? k : k / dr.ngrp;
        const uint32_t c0 = (k - i * dr.ngrp) * 64;
        const int32_t q0 = (int32_t)((g.ra + i) * dr.rowlen + dr.fb) - (int32_t)B + 16 * (int32_t)c0;
        uint4 x = v[j];
        if (dr.swap) x = swap16(x, dr.bpp);
        if (dr.flip) x = flip_msb(x, dr.bpp);
        if (dr.aligned) {
            // Rows of whole 16-byte chunks: every lane stores the ALIGNED 16 bytes ending
            // where its chunk starts + 16 - s (s = q0 mod 16, uniform): the previous lane's
            // last s bytes (one wave shift) and its own first 16 - s; lane 0 takes the bytes
            // before the task's first chunk from the previous task (a readlane) or its extra
            // load (the filter byte 0 in front of a PNG row).  The task's last s bytes are the
            // next task's lane 0's word (or the word before it, when the filter byte makes
            // the next row start on a boundary); the buffer's last row writes them itself.
            // Bytes past nb are zero.
            uint4 p;
            p.x = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x.x, 0x138, 0xF, 0xF, false);  // wave_shr:1
            p.y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x.y, 0x138, 0xF, 0xF, false);
            p.z = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x.z, 0x138, 0xF, 0xF, false);
            p.w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x.w, 0x138, 0xF, 0xF, false);
            if (lane == 0) {
                uint4 y = xlast;
                if (j == 0) {
                    y = pv;
                    if (dr.swap) y = swap16(y, dr.bpp);
                    if (dr.flip) y = flip_msb(y, dr.bpp);
                }
                if (dr.fb && c0 == 0)  // the row above's last 15 bytes, then the filter byte
                    y = make_uint4((y.x >> 8) | (y.y << 24), (y.y >> 8) | (y.z << 24), (y.z >> 8) | (y.w << 24),
                                   y.w >> 8);
                p = y;
            }
            const uint32_t sft = (uint32_t)q0 & 15u;
            const int32_t A = q0 - (int32_t)sft;
            const uint32_t nct = dr.nc - c0 < 64 ? dr.nc - c0 : 64u;  // chunks of this task
            auto put = [&](int32_t at, uint4 w) {
                if (at < 0 || at >= (int32_t)nb) return;
                if (at + 16 > (int32_t)nb) {  // zero the bytes past the buffer
                    const uint32_t keep = (uint32_t)((int32_t)nb - at);
                    uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                    for (uint32_t q = 0; q < 4; q++) {
                        const int32_t kb = (int32_t)keep - 4 * (int32_t)q;
                        const uint32_t nbits = kb <= 0 ? 0u : kb >= 4 ? 32u : 8u * (uint32_t)kb;
                        ww[q] &= (uint32_t)((1ull << nbits) - 1ull);
                    }
                    w = make_uint4(ww[0], ww[1], ww[2], ww[3]);
                }
                *(uint4*)(bb + at) = w;
            };
            if (lane < nct) put(A + 16 * (int32_t)lane, funnel16(p, x, sft));
            // a PNG row starting on a word boundary: the word before (the row above's last 15
            // bytes and this row's filter byte) is this lane 0's too
            if (lane == 0 && dr.fb && c0 == 0 && sft == 0) put(A - 16, p);
            // the task's tail: the last chunk's last s bytes, when no task follows in the buffer
            if (lane == nct - 1 && sft && g.ra + i == g.rz && c0 + nct == dr.nc)
                put(A + 16 * (int32_t)nct, funnel16(x, make_uint4(0, 0, 0, 0), sft));
            const int ll = (int)nct - 1;
            xlast = make_uint4((uint32_t)__builtin_amdgcn_readlane((int)x.x, ll), (uint32_t)__builtin_amdgcn_readlane((int)x.y, ll),
                               (uint32_t)__builtin_amdgcn_readlane((int)x.z, ll), (uint32_t)__builtin_amdgcn_readlane((int)x.w, ll));
            continue;
        }
        const uint32_t c = c0 + lane;
        const int32_t dst = q0 + 16 * (int32_t)lane;  // LDS byte of the chunk's first byte
        const bool valid = c < dr.nc;
        if (valid && dst >= 0 && dst + 16 <= (int32_t)nb && 16 * (c + 1) <= dr.rb) {
            // one unaligned 16-byte LDS store (gfx950 DS access is unaligned-capable)
            __builtin_memcpy(bb + dst, &x, 16);
        } else if (valid && dst + 16 > 0 && dst < (int32_t)nb) {
            const uint32_t nbc = dr.rb - 16 * c < 16 ? dr.rb - 16 * c : 16u;
            for (uint32_t q = 0; q < nbc; q++) {
                const int32_t at = dst + (int32_t)q;
                const uint32_t lo = (q & 4u) ? x.y : x.x, hi = (q & 4u) ? x.w : x.z;
                if (at >= 0 && at < (int32_t)nb) bb[at] = (uint8_t)(((q & 8u) ? hi : lo) >> (8 * (q & 3u)));
            }
        }
        if (dr.fb && c == 0 && dst - 1 >= 0 && dst - 1 < (int32_t)nb) bb[dst - 1] = 0;
    }
}

template <int NT, uint32_t K>
__device__ __forceinline__ void fill_issue(FillPre<K>& pf, const DirectRows& dr, uint32_t B, uint32_t nb,
                                           uint32_t tid) {
    const FillGeom g(dr, B, nb);
    const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (w * K < g.ntask) fill_loads<NT, K>(pf.v, pf.pv, dr, g, w * K, tid & 63);
}

template <int NT, uint32_t K>
__device__ __forceinline__ void fill_finish(const FillPre<K>& pf, uint32_t* buf, const DirectRows& dr,
                                            uint32_t B, uint32_t nb, uint32_t nz, uint32_t tid) {
    constexpr uint32_t NW = NT / 64;
    uint8_t* bb = (uint8_t*)buf;
    const uint32_t lane = tid & 63;
    const FillGeom g(dr, B, nb);
    const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (w * K < g.ntask) fill_stores<NT, K>(pf.v, pf.pv, bb, dr, g, B, nb, w * K, lane);
    for (uint32_t k0 = (w + NW) * K; k0 < g.ntask; k0 += K * NW) {  // batches past the prefetched one
        uint4 v[K], pv;
        fill_loads<NT, K>(v, pv, dr, g, k0, lane);
        fill_stores<NT, K>(v, pv, bb, dr, g, B, nb, k0, lane);
    }
    // zero tail: bytes [nb, round4(nb)) and words up to nz
    const uint32_t nb4 = (nb + 3) & ~3u;
    if (tid < nb4 - nb) bb[nb + tid] = 0;
    for (uint32_t k = nb4 / 4 + tid; k < nz / 4; k += NT) buf[k] = 0;
}

// The common geometry, without per-task bookkeeping: rows of whole 16-byte chunks, at most
// 64 chunks (one wave per row), the sample conversion fixed at compile time (SB: bytes per
// swapped sample, 0 = none; FL: the PNG sign flip).  Wave w fills blocks of FR consecutive
// rows of the buffer, their loads in flight together.  Row r's
// lane l stores the aligned word ending where its chunk's first 16 - s bytes end (s = the
// row's start mod 16), lane 0's word holding the row above's tail and the filter byte (the
// layout fill_stores writes); the buffer's last row writes its own tail.  Only rows that
// cross the buffer's ends clip per lane.
#ifndef PBX_FF_FR
#define PBX_FF_FR 2  // fill_fast: consecutive rows per wave block
#endif
#ifndef PBX_FF_FR4
#define PBX_FF_FR4 3  // 16-bit samples without the sign flip (the headline): three rows, one load round for 18 rows
#endif
#ifndef PBX_NT_STREAM
#define PBX_NT_STREAM 0  // nontemporal accesses: 1 k_lz77's stream stores, 2 k_encode's stream loads, 4 its output stores
#endif
// gseg (optional): the segment's bytes (buffer bytes [wl, nb)) are also stored there, from
// the same registers (k_encode's input), instead of re-read from LDS after the fill.
template <int NT, uint32_t SB, bool FL, uint32_t FR = PBX_FF_FR>
__device__ void fill_fast(uint32_t* buf, const DirectRows& dr, uint32_t B, uint32_t nb, uint32_t nz,
                          uint32_t tid, uint32_t ra, uint32_t rz, uint8_t* gseg, uint32_t wl) {
    constexpr uint32_t NW = NT / 64;
    uint8_t* bb = (uint8_t*)buf;
    const uint32_t lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t nc = dr.nc, fb = dr.fb, rowlen = dr.rowlen, nrows = rz - ra + 1;
    const uint32_t flipm = dr.bpp == 1 ? 0x80808080u : 0x00800080u;
    const uint4 Z = make_uint4(0, 0, 0, 0);
    auto conv = [&](uint4 v) {
        if (SB) v = swap16(v, (int)SB);
        if (FL) { v.x ^= flipm; v.y ^= flipm; v.z ^= flipm; v.w ^= flipm; }
        return v;
    };
    // one 16-byte word at buffer byte `at` (aligned): skipped outside [0, nb), zero past nb
    auto put = [&](int32_t at, uint4 v) {
        if (at < 0 || at >= (int32_t)nb) return;
        if (at + 16 > (int32_t)nb) {
            const uint32_t keep = (uint32_t)((int32_t)nb - at);
            uint32_t ww[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (uint32_t q = 0; q < 4; q++) {
                const int32_t kb = (int32_t)keep - 4 * (int32_t)q;
                const uint32_t nbits = kb <= 0 ? 0u : kb >= 4 ? 32u : 8u * (uint32_t)kb;
                ww[q] &= (uint32_t)((1ull << nbits) - 1ull);
            }
            v = make_uint4(ww[0], ww[1], ww[2], ww[3]);
        }
        *(uint4*)(bb + at) = v;
        if (gseg && at >= (int32_t)wl) {
            if (PBX_NT_STREAM & 1) gstore16_nt(gseg + (at - (int32_t)wl), v); else gstore16(gseg + (at - (int32_t)wl), v);
        }
    };
    // interior word: no clipping in LDS, the global copy for segment bytes only
    auto put_in = [&](int32_t at, uint4 v) {
        *(uint4*)(bb + at) = v;
        if (gseg && at >= (int32_t)wl) {
            if (PBX_NT_STREAM & 1) gstore16_nt(gseg + (at - (int32_t)wl), v); else gstore16(gseg + (at - (int32_t)wl), v);
        }
    };
    // wave w: blocks of FR consecutive rows, w, w + NW, ...; the chunk before a block's first
    // row is one extra load, before its other rows the previous row's last chunk (a readlane)
    for (uint32_t i0 = w * FR; i0 < nrows; i0 += NW * FR) {
        uint4 x[FR];
#pragma unroll
        for (uint32_t j = 0; j < FR; j++) {  // unconditional loads (clamped row): exact counters
            const uint32_t r = ra + (i0 + j < nrows ? i0 + j : i0);
#ifdef PBX_LZ_FAKE_LOAD  // timing experiment only: hashed bytes, no plane reads
            {
                const uint64_t h = splitmix64((uint64_t)(uintptr_t)(dr.row0 + (int64_t)r * dr.pitch + 16 * lane));
                x[j] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)(h * 3), (uint32_t)(h >> 17));
            }
#else
            x[j] = gload16(dr.row0 + (int64_t)r * dr.pitch + 16 * (lane < nc ? lane : 0u));
#endif
        }
        const uint32_t r0 = ra + i0;
        const uint8_t* rp0 = dr.row0 + (int64_t)r0 * dr.pitch;
        uint4 y = gload16(r0 ? rp0 - dr.pitch + 16 * (nc - 1) : rp0);  // the row above's last chunk
        y = r0 ? conv(y) : Z;
#pragma unroll
        for (uint32_t j = 0; j < FR; j++) {
            if (i0 + j >= nrows) break;  // uniform
            const uint32_t r = r0 + j;
            const uint4 xc = conv(x[j]);
            uint4 yf = y;
            if (fb)  // the row above's last 15 bytes, then the filter byte (0)
                yf = make_uint4((y.x >> 8) | (y.y << 24), (y.y >> 8) | (y.z << 24), (y.z >> 8) | (y.w << 24), y.w >> 8);
            uint4 pv;  // the previous lane's chunk; lane 0: yf
            pv.x = (uint32_t)__builtin_amdgcn_update_dpp((int)yf.x, (int)xc.x, 0x138, 0xF, 0xF, false);  // wave_shr:1
            pv.y = (uint32_t)__builtin_amdgcn_update_dpp((int)yf.y, (int)xc.y, 0x138, 0xF, 0xF, false);
            pv.z = (uint32_t)__builtin_amdgcn_update_dpp((int)yf.z, (int)xc.z, 0x138, 0xF, 0xF, false);
            pv.w = (uint32_t)__builtin_amdgcn_update_dpp((int)yf.w, (int)xc.w, 0x138, 0xF, 0xF, false);
            const int32_t q0 = (int32_t)(r * rowlen + fb) - (int32_t)B;
            const uint32_t sft = (uint32_t)q0 & 15u;
            const int32_t A = q0 - (int32_t)sft;
            const uint4 wv = funnel16(pv, xc, sft);
            const bool last = r == rz && sft;  // the buffer's last row writes its own tail
            if (A >= 16 && A + 16 * (int32_t)(nc + 1) <= (int32_t)nb) {  // uniform: no clipping
                if (lane < nc) put_in(A + 16 * (int32_t)lane, wv);
                if (lane == 0 && fb && sft == 0) put_in(A - 16, pv);
                if (lane == nc - 1 && last) put_in(A + 16 * (int32_t)nc, funnel16(xc, Z, sft));
            } else {
                if (lane < nc) put(A + 16 * (int32_t)lane, wv);
                if (lane == 0 && fb && sft == 0) put(A - 16, pv);
                if (lane == nc - 1 && last) put(A + 16 * (int32_t)nc, funnel16(xc, Z, sft));
            }
            y = make_uint4((uint32_t)__builtin_amdgcn_readlane((int)xc.x, nc - 1), (uint32_t)__builtin_amdgcn_readlane((int)xc.y, nc - 1),
                           (uint32_t)__builtin_amdgcn_readlane((int)xc.z, nc - 1), (uint32_t)__builtin_amdgcn_readlane((int)xc.w, nc - 1));
        }
    }
    // zero tail: bytes [nb, round4(nb)) and words up to nz
    const uint32_t nb4 = (nb + 3) & ~3u;
    if (tid < nb4 - nb) bb[nb + tid] = 0;
    for (uint32_t k = nb4 / 4 + tid; k < nz / 4; k += NT) buf[k] = 0;
}

// fill_fast's sample conversion for a tile's geometry, + 1 (0: not its case -- rows not whole
// 16-byte chunks, more than 64 chunks a row, 8-byte samples, a flip with a swap of 4 bytes).
__device__ __forceinline__ uint32_t fast_fill_mode(const DirectRows& dr) {
    if (!dr.aligned || dr.ngrp != 1 || dr.bpp > 4) return 0u;
    const uint32_t sb = dr.swap ? (uint32_t)dr.bpp : 0u;
    const uint32_t mode = (sb == 1 ? 0u : sb) * 2 + (dr.flip ? 1u : 0u);
    return (mode == 0 || mode == 1 || mode == 4 || mode == 5 || mode == 8) ? mode + 1 : 0u;
}

// fill_fast for a mode of fast_fill_mode (!= 0)
template <int NT>
__device__ __forceinline__ void fill_fast_mode(uint32_t mode, uint32_t* buf, const DirectRows& dr, uint32_t B,
                                               uint32_t nb, uint32_t nz, uint32_t tid, uint32_t ra, uint32_t rz,
                                               uint8_t* gseg, uint32_t wl) {
    switch (mode) {
    case 1: fill_fast<NT, 0, false>(buf, dr, B, nb, nz, tid, ra, rz, gseg, wl); break;
    case 2: fill_fast<NT, 0, true>(buf, dr, B, nb, nz, tid, ra, rz, gseg, wl); break;
    case 5: fill_fast<NT, 2, false, PBX_FF_FR4>(buf, dr, B, nb, nz, tid, ra, rz, gseg, wl); break;
    case 6: fill_fast<NT, 2, true>(buf, dr, B, nb, nz, tid, ra, rz, gseg, wl); break;
    default: fill_fast<NT, 4, false>(buf, dr, B, nb, nz, tid, ra, rz, gseg, wl); break;
    }
}

// fill_fast for the tile's sample conversion; false when the geometry is not its case
template <int NT>
__device__ __forceinline__ bool fill_fast_any(uint32_t* buf, const DirectRows& dr, uint32_t B, uint32_t nb,
                                              uint32_t nz, uint32_t tid, uint8_t* gseg, uint32_t wl) {
    const uint32_t mode = fast_fill_mode(dr);
    if (!mode) return false;
    const uint32_t ra = div_rcp(B, dr.rowlen, dr.rcp), rz = div_rcp(B + nb - 1, dr.rowlen, dr.rcp);
    fill_fast_mode<NT>(mode, buf, dr, B, nb, nz, tid, ra, rz, gseg, wl);
    return true;
}

#ifndef PBX_LZ_FAST_FILL
#define PBX_LZ_FAST_FILL 1  // fill_fast for the common geometry (0: the general fill only)
#endif
// 1: for direct tiles of fill_fast's geometry k_encode rebuilds the segment's bytes from the
// plane (each wave its 2 KiB, through its part of the LDS output buffer) and k_lz77 writes no
// stream bytes for them -- the stream's HBM round trip (every byte written, read back) gone.
// Correct (every -m gpu test green) but slower: k_lz77 1.48 -> 1.36 ms, k_encode 1.57 ->
// 1.92 ms, the conversion's VALU in the issue-bound encoder (profiles/r03_p17/).  0 (default):
// k_lz77 stores the bytes from its fill registers and k_encode reads them back.
// 2: the same for 16-bit byte-swapped samples (fast-fill mode 5, the headline), each lane
// converting its own 32 bytes in registers: three 16-byte plane loads, the byte swap and a
// per-lane byte alignment (plane_words_swap16), no LDS.
#ifndef PBX_ENC_FROM_PLANE
#define PBX_ENC_FROM_PLANE 0
#endif

// Bytes [q, q + 32) of a row's converted data (16-bit samples byte-swapped) as 8 words; bytes
// outside [0, rb) are 0 (a PNG row's filter byte sits at q = -1).  rp: the row in the plane
// (nullptr: no row, all 0).  Chunks at 16-byte offsets inside the row only are loaded.
__device__ __forceinline__ void row_bytes32_swap16(const uint8_t* rp, int32_t q, uint32_t rb, uint32_t (&o)[8]) {
    const int32_t b16 = q & ~15;  // (floor for negative q)
    uint32_t z[12];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const int32_t off = b16 + 16 * k;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (rp && off >= 0 && off < (int32_t)rb) v = swap16(gload16(rp + off), 2);
        z[4 * k] = v.x; z[4 * k + 1] = v.y; z[4 * k + 2] = v.z; z[4 * k + 3] = v.w;
    }
    const uint32_t s = (uint32_t)(q - b16);  // 0..15: the first byte's offset in z
    // word selection by masks (a select the compiler would turn into a scratch-indexed array)
    const uint32_t m1 = 0u - ((s >> 2) & 1u), m2 = 0u - ((s >> 3) & 1u);
    uint32_t y[11];
#pragma unroll
    for (int i = 0; i < 11; i++) y[i] = z[i] ^ ((z[i] ^ z[i + 1]) & m1);
    uint32_t t[9];
#pragma unroll
    for (int i = 0; i < 9; i++) t[i] = y[i] ^ ((y[i] ^ y[i + 2]) & m2);
#pragma unroll
    for (int m = 0; m < 8; m++) o[m] = __builtin_amdgcn_alignbyte(t[m + 1], t[m], s & 3u);
}

// Stream bytes [B, B + 32) of a direct tile of fast-fill mode 5 (k_lz77 stored none): row r's
// bytes, then (a chunk that crosses into row r + 1: rows are longer than 32 bytes) row r + 1's
// from its filter byte on.  Rows past the tile's last are 0.
__device__ __forceinline__ void plane_words_swap16(const DirectRows& dr, uint32_t B, uint32_t (&cb)[8]) {
    const uint32_t r = div_rcp(B, dr.rowlen, dr.rcp);
    const uint32_t col = B - r * dr.rowlen;
    const uint8_t* rp = r < dr.h ? dr.row0 + (int64_t)r * dr.pitch : nullptr;
    row_bytes32_swap16(rp, (int32_t)col - (int32_t)dr.fb, dr.rb, cb);
    const uint32_t k = dr.rowlen - col;  // bytes of row r in the chunk
    if (k < 32) {
        const uint8_t* rn = r + 1 < dr.h ? dr.row0 + (int64_t)(r + 1) * dr.pitch : nullptr;
        uint32_t nb[8];
        row_bytes32_swap16(rn, -(int32_t)k - (int32_t)dr.fb, dr.rb, nb);
#pragma unroll
        for (uint32_t m = 0; m < 8; m++) {
            const int32_t a = (int32_t)k - 4 * (int32_t)m;  // bytes of word m from row r
            const uint32_t mask = a <= 0 ? 0u : a >= 4 ? 0xFFFFFFFFu : (1u << (8 * a)) - 1u;
            cb[m] = (cb[m] & mask) | (nb[m] & ~mask);
        }
    }
}

// ==================================================================== k_lz77
// Zero bytes of x as 4 bits (bit j: byte j of x is zero).
__device__ __forceinline__ uint32_t zero_nibble(uint32_t x) {
    const uint32_t t = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
    const uint32_t z = ~(t | x) & 0x80808080u;  // bit 8j+7: byte j == 0
    return ((z >> 7) | (z >> 14) | (z >> 21) | (z >> 28)) & 0xFu;
}

#ifndef PBX_LZ_DOT4PACK
#define PBX_LZ_DOT4PACK 1  // equality bits packed by v_dot4 (0: shifts and ORs per word)
#endif
// Zero bytes of the eight words x[j] as 32 bits (bit 4j + k: byte k of x[j] is zero).  Each
// word's zero-byte flags sit at bit 7 of its bytes (0 or 128 as a byte); one v_dot4_u32_u8
// against the weights 1, 2, 4, 8 (or 16 .. 128 for the second word of a pair) sums them into
// 128 x the pair's eight bits: two dot products, a shift and an OR per pair of words instead
// of four shifts and three ORs per word.
__device__ __forceinline__ uint32_t pack_zero_bytes8(const uint32_t (&x)[8]) {
    uint32_t e = 0;
#pragma unroll
    for (int p = 0; p < 4; p++) {
        const uint32_t za = ~(((x[2 * p] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x[2 * p]) & 0x80808080u;
        const uint32_t zb = ~(((x[2 * p + 1] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x[2 * p + 1]) & 0x80808080u;
        const uint32_t b = dot4_u8(za, 0x08040201u, dot4_u8(zb, 0x80402010u, 0u)) >> 7;
        e |= b << (8 * p);
    }
    return e;
}

// Parse of wave w's sub-segment (scalar twin: ph_parse_emu in deflate_seg.h).  Lane l holds
// positions p0 = ss + 32 l .. p0 + 31 (its thread chunk).  Per candidate distance d the lane
// builds E_d, bit i = (byte p0+i == byte p0+i-d), masked to valid positions (< se, d not
// before the window), and Ex_d = E_d | next lane's E_d << 32: the capped match length at
// position p0+i is ctz(~(Ex_d >> i)) (<= 64 - i), and the positions where a candidate pays
// (>= match_minlen(d) equal bytes) are E & E>>1 & E>>2 (& ...).  The wave walks only those
// positions (M), scalar: lengths at k and k+1 from readlane'd masks, the lazy rule, the
// wave-wide extension of a capped match.  Each lane also collects the positions of its
// chunk covered by recorded matches (cover), for the histogram.
template <class C, class SM, bool PROF = false, bool VC = false>
__device__ __forceinline__ void ph_parse_dev(uint32_t tid, SM& S, const SegParams& sp, const uint32_t (&cw)[9],
                             uint32_t& cover, uint32_t& smask) {
    uint32_t nsteps = 0;  // (PROF) walk steps of this wave
    const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const uint32_t ss = w * C::SUB;
    const uint32_t se = __builtin_amdgcn_readfirstlane(ss + C::SUB < sp.sl ? ss + C::SUB : sp.sl);
    const bool active = ss < se;  // (uniform) waves past the segment's end have nothing to parse
    cover = 0;
    smask = 0;
    const uint32_t p0 = ss + 32 * lane, a0 = sp.wl + p0;
    // Boundary after wave b (lane b < NW - 1): a paying run ends at that sub-segment's last byte
    // (ml equal bytes of a candidate there, ml = match_minlen), the only way a match of wave b
    // can run on into wave b + 1.  From the bytes alone, the same in every wave: a uniform
    // decision, no barrier (noise: almost never; then every wave's parse is final at once).
#ifndef PBX_LZ_REACH_LATE
#define PBX_LZ_REACH_LATE 1  // the boundary test after the candidate masks, loads unconditional
#endif
#ifndef PBX_LZ_REACH_MASKS
#define PBX_LZ_REACH_MASKS 0  // 1: each wave tests its own boundary from lane 63's candidate masks,
                              // the bits meet in LDS across one barrier (no LDS loads)
#endif
    auto reach_test = [&]() -> uint32_t {
        bool rb = false;
        const uint32_t e = (lane + 1) * (uint32_t)C::SUB;
        const bool ok = lane + 1 < (uint32_t)C::NW && e < sp.sl;
        if (PBX_LZ_REACH_LATE) {
            // every lane loads (clamped addresses, no divergent branch): the loads can issue
            // with the candidate masks' and are waited for once
            const uint32_t a = ok ? sp.wl + e : 8u;
            const uint2 v = *(const uint2*)&S.buf[(a >> 2) - 2];
            const uint64_t x = ((uint64_t)v.y << 32) | v.x;  // bytes a - 8 .. a - 1
            rb = ((x ^ (x << 8)) >> 40) == 0 || ((x ^ (x << 16)) >> 40) == 0;
            const uint32_t d = cand_dist(sp, 2), mlr = match_minlen(d);
            const bool okr = d && a >= mlr + d;
            const uint32_t ar = okr ? a : 8u + mlr + d;
            // the last mlr bytes (mlr = 3 for rows of <= 256 bytes: a 3-byte run pays)
            bool eq = ((v.y ^ lds_ld4(S, ar - 4 - d)) >> (mlr == 3 ? 8u : 0u)) == 0;
            if (mlr == 6) eq = eq && ((v.x >> 16) ^ (lds_ld4(S, ar - 6 - d) & 0xFFFFu)) == 0;
            rb = ok && (rb || (okr && eq));
        } else if (ok) {
            const uint32_t a = sp.wl + e;
            // the 8 bytes before the boundary: one aligned 8-byte LDS read (wl and e are
            // multiples of 16); distances 1 and 2 (ml = 3) compare them among themselves
            const uint2 v = *(const uint2*)&S.buf[(a >> 2) - 2];
            const uint64_t x = ((uint64_t)v.y << 32) | v.x;  // bytes a - 8 .. a - 1
            rb = ((x ^ (x << 8)) >> 40) == 0 || ((x ^ (x << 16)) >> 40) == 0;
            // one row up (ml = 4, or 6 past 4 KiB), when the run's sources are in the window
            const uint32_t d = cand_dist(sp, 2), mlr = match_minlen(d);
            if (d && a >= mlr + d) {
                bool eq = ((v.y ^ lds_ld4(S, a - 4 - d)) >> (mlr == 3 ? 8u : 0u)) == 0;
                if (mlr == 6) eq = eq && ((v.x >> 16) ^ (lds_ld4(S, a - 6 - d) & 0xFFFFu)) == 0;
                rb = rb || eq;
            }
        }
        uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)__ballot(rb));
#ifdef PBX_LZ_NOREACH  // timing bound only (variant build): no boundary reachable, wrong output on runs
        m = 0;
#endif
#ifdef PBX_LZ_REACH_DISCARD  // timing only (variant build): the test computed, its result dropped
        asm volatile("" ::"s"(m));
        m = 0;
#endif
        return m;
    };
    uint32_t reachm = PBX_LZ_REACH_LATE || PBX_LZ_REACH_MASKS ? 0u : reach_test();
    uint32_t exlo[NCAND] = {}, exhi[NCAND] = {}, ml[NCAND] = {3, 3, 3}, dd[NCAND] = {};
    uint32_t M = 0, cvb_n = 0;
    bool skip = true;
    if (active) {
        const uint32_t nval = se > p0 ? se - p0 : 0u;
        smask = nval >= 32 ? 0xFFFFFFFFu : (1u << nval) - 1u;
        uint32_t cvb_lo = 0, cvb_hi = 0;  // bytes inside some paying run (the walk's coverage bound, below)
#pragma unroll
        for (int c = 0; c < NCAND; c++) {
            const uint32_t d = __builtin_amdgcn_readfirstlane(cand_dist(sp, c));
            dd[c] = d;
            ml[c] = match_minlen(d);
            uint32_t e = 0;
            if (d) {
                if (c < 2) {  // d = 1, 2: the lane's own words shifted by d bytes
                    const uint32_t sh = 32 - 8 * d;
                    if (PBX_LZ_DOT4PACK) {
                        uint32_t xw[8];
#pragma unroll
                        for (int j = 0; j < 8; j++) xw[j] = cw[j + 1] ^ funnel32(cw[j + 1], cw[j], sh);
                        e = pack_zero_bytes8(xw);
                    } else {
#pragma unroll
                        for (int j = 0; j < 8; j++) e |= zero_nibble(cw[j + 1] ^ funnel32(cw[j + 1], cw[j], sh)) << (4 * j);
                    }
                } else {  // one row up: unaligned words at a0 - d
                    const int32_t b = (int32_t)a0 - (int32_t)d;
                    const int32_t r = b >> 2;
                    const uint32_t sh = (uint32_t)(b & 3) * 8;
                    // words r .. r+8 from three aligned 16-byte reads (lanes 32 bytes apart: a
                    // 2-way conflict per read instead of 8-way on 9 word reads); r mod 4 is the
                    // same in every lane (a0 - 32 lane is), so the selection is uniform.  Quads
                    // before the buffer (positions the window mask drops) read quad 0.
                    const int32_t r4 = r & ~3;
                    uint32_t q12[12];
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        const int32_t at = r4 + 4 * k;
                        const uint4 v = *(const uint4*)&S.buf[at > 0 ? at : 0];
                        q12[4 * k] = v.x; q12[4 * k + 1] = v.y; q12[4 * k + 2] = v.z; q12[4 * k + 3] = v.w;
                    }
                    uint32_t rw[9];
                    switch (__builtin_amdgcn_readfirstlane((uint32_t)(r - r4))) {
                    case 0:
#pragma unroll
                        for (int j = 0; j < 9; j++) rw[j] = q12[j];
                        break;
                    case 1:
#pragma unroll
                        for (int j = 0; j < 9; j++) rw[j] = q12[j + 1];
                        break;
                    case 2:
#pragma unroll
                        for (int j = 0; j < 9; j++) rw[j] = q12[j + 2];
                        break;
                    default:
#pragma unroll
                        for (int j = 0; j < 9; j++) rw[j] = q12[j + 3];
                        break;
                    }
                    if (PBX_LZ_DOT4PACK) {
                        uint32_t xw[8];
#pragma unroll
                        for (int j = 0; j < 8; j++) xw[j] = cw[j + 1] ^ funnel32(rw[j + 1], rw[j], sh);
                        e = pack_zero_bytes8(xw);
                    } else {
#pragma unroll
                        for (int j = 0; j < 8; j++) e |= zero_nibble(cw[j + 1] ^ funnel32(rw[j + 1], rw[j], sh)) << (4 * j);
                    }
                }
                const uint32_t vm = a0 >= d ? 0xFFFFFFFFu : (d - a0 >= 32 ? 0u : 0xFFFFFFFFu << (d - a0));
                e &= vm & smask;
            }
            // the next lane's E (wave_shl:1; lane 63: none, matches stay in the sub-segment)
            const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)e, 0x130, 0xF, 0xF, false);
            exlo[c] = e;
            exhi[c] = nx;
            if (d) {
                // (E | next lane's E << 32) >> k, low word: one funnel shift (v_alignbit) each
                uint32_t r = e & __builtin_amdgcn_alignbit(nx, e, 1) & __builtin_amdgcn_alignbit(nx, e, 2);
                if (ml[c] >= 4) r &= __builtin_amdgcn_alignbit(nx, e, 3);
                if (ml[c] >= 6) r &= __builtin_amdgcn_alignbit(nx, e, 4) & __builtin_amdgcn_alignbit(nx, e, 5);
                M |= r;
                // [j, j + ml) for every paying start j of the lane: bits inside the lane (lo) and
                // the ones past its end (hi)
                uint32_t dlo = r | (r << 1) | (r << 2), dhi = (r >> 31) | (r >> 30);
                if (ml[c] >= 4) { dlo |= r << 3; dhi |= r >> 29; }
                if (ml[c] >= 6) { dlo |= (r << 4) | (r << 5); dhi |= (r >> 28) | (r >> 27); }
                cvb_lo |= dlo;
                cvb_hi |= dhi;
            }
        }
#ifndef PBX_LZ_COVBOUND
#define PBX_LZ_COVBOUND 1  // skip the walk when its matches cannot reach MINCOV (0: always walk)
#endif
        // Every match the walk records lies inside a run of >= ml equal bytes of its candidate,
        // i.e. inside the union of [j, j + ml) over that candidate's paying starts j; a match
        // extended past CAP lies in a run of >= CAP >= MINCOV bytes.  So the walk's coverage is at
        // most the wave's count of such bytes (per lane, bytes past the lane's chunk counted too:
        // an overestimate), and below MINCOV the walk would drop all its matches (noise: most
        // waves hold a few 3-4 byte runs): the same result without the walk.  A match that reaches
        // the sub-segment's last byte may run on into the next one (extend_cross), past that
        // count: the bound then does not hold, and the wave walks.  Such a match lies in a run of
        // >= ml equal bytes ending at the last byte, so se - ml is a paying start and the last
        // byte is in the union above (this lane's bits, or the previous lane's bits past its
        // chunk): exactly the waves where a paying run reaches the last byte walk.
        cvb_n = wave_sum((uint32_t)__builtin_popcount(cvb_lo) + (uint32_t)__builtin_popcount(cvb_hi));
    }
    if (PBX_LZ_REACH_MASKS) {
        // the boundary after this wave: a paying run (ml equal bytes of a candidate) ends at
        // its last byte, i.e. the top ml bits of lane 63's equality mask are set (masked past
        // the segment's end and before the window, as the LDS form's conditions)
        uint32_t own = 0;
        if (active && w + 1 < (uint32_t)C::NW && se == ss + (uint32_t)C::SUB && se < sp.sl) {
            bool rb = false;
#pragma unroll
            for (int c = 0; c < NCAND; c++) {
                const uint32_t need = 0xFFFFFFFFu << (32 - ml[c]);
                rb = rb || (dd[c] != 0 && (exlo[c] & need) == need);
            }
            own = (uint32_t)__builtin_amdgcn_readlane((int)rb, 63);
        }
        if (lane == 0 && own) atomicOr(&S.reachw, 1u << w);
        __syncthreads();
        reachm = __builtin_amdgcn_readfirstlane(S.reachw);
    } else if (PBX_LZ_REACH_LATE) {
        reachm = reach_test();
    }
    if (active) skip = PBX_LZ_COVBOUND && !((reachm >> w) & 1u) && cvb_n < (uint32_t)C::MINCOV;
#ifndef PBX_LZ_EARLY_OUT
#define PBX_LZ_EARLY_OUT 1
#endif
    // (uniform) no boundary of the segment reachable and this wave's walk would keep nothing
    // (noise: most waves): no records, no walk, no carry rounds -- the round-3 early return
    if (PBX_LZ_EARLY_OUT && reachm == 0 && skip) {
        if (lane == 0) S.w_nm[w] = 0;
        return;
    }
    const uint64_t B = __ballot(M != 0);
    const uint32_t lsub = active ? se - ss : 0u;
#ifndef PBX_LZ_VCAND
#define PBX_LZ_VCAND 2  // the walk's candidate lengths in VALU, lane c for candidate c: 1 always, 2 in the
                        // run-dense waves of row-filtered batches (VC), 0 never
#endif
    // (2: row-filtered streams put runs in every wave, every wave of the CU walks at once and the
    // scalar unit is the bound; elsewhere -- filter None, noise -- the kernel keeps the scalar
    // loop only: the VALU form measured 1-9% slower there, profiles/r05zs, r05zt)
    const bool vcand = PBX_LZ_VCAND == 1 || (PBX_LZ_VCAND == 2 && VC && cvb_n >= (uint32_t)C::SUB / 2);
    // lane c < NCAND: candidate c's distance present and its match_minlen (the walk's VALU form)
    const bool vok = lane < (uint32_t)NCAND && (lane == 0 ? dd[0] : lane == 1 ? dd[1] : dd[2]) != 0;
    const uint32_t vml = lane == 0 ? ml[0] : lane == 1 ? ml[1] : ml[2];
    uint32_t nm = 0, cov = 0, last_end = 0;
    // The greedy walk over the paying positions from o0 (sub-segment offset): records, the
    // lane's covered positions, the end of the last match (uniform).
    auto walk = [&](uint32_t o0) {
        nm = 0;
        cov = 0;
        last_end = 0;
        cover = 0;
        uint32_t o = o0;
        while (o < lsub) {
            if (PROF) nsteps++;
            // the first position >= o where a match pays
            const uint32_t t0 = o >> 5;
            uint32_t k = 0xFFFFFFFFu;
            const uint32_t mt = __builtin_amdgcn_readlane(M, t0) & (0xFFFFFFFFu << (o & 31));
            if (mt) {
                k = (t0 << 5) + (uint32_t)__builtin_ctz(mt);
            } else if (t0 < 63) {
                const uint64_t bb = B & (~0ull << (t0 + 1));
                if (bb) {
                    const uint32_t t2 = (uint32_t)__builtin_ctzll(bb);
                    k = (t2 << 5) + (uint32_t)__builtin_ctz(__builtin_amdgcn_readlane(M, t2));
                }
            }
            k = __builtin_amdgcn_readfirstlane(k);
            if (k >= lsub) break;
            const uint32_t t = k >> 5, i = k & 31;
            uint32_t L = 0, D = 0, Dc = 0, L1 = 0;
            if (vcand) {
                // lane c (< NCAND) evaluates candidate c at k and k + 1 in VALU (the scalar unit
                // is the CU's bottleneck while every wave walks: run-heavy streams); the best
                // (length, then the earliest candidate) by a max over the quad of packed
                // (n0 << 2 | 3 - c), two DPP steps
                static_assert(NCAND == 3 && C::CAP == 32, "three candidates, 32-bit windows");
                const uint32_t l0 = (uint32_t)__builtin_amdgcn_readlane(exlo[0], t), h0 = (uint32_t)__builtin_amdgcn_readlane(exhi[0], t);
                const uint32_t l1 = (uint32_t)__builtin_amdgcn_readlane(exlo[1], t), h1 = (uint32_t)__builtin_amdgcn_readlane(exhi[1], t);
                const uint32_t l2 = (uint32_t)__builtin_amdgcn_readlane(exlo[2], t), h2 = (uint32_t)__builtin_amdgcn_readlane(exhi[2], t);
                const uint32_t xl = lane == 0 ? l0 : lane == 1 ? l1 : l2, xh = lane == 0 ? h0 : lane == 1 ? h1 : h2;
                const uint32_t q0 = ~__builtin_amdgcn_alignbit(xh, xl, i);
                const uint32_t q1 = ~(i < 31 ? __builtin_amdgcn_alignbit(xh, xl, i + 1) : xh);
                const uint32_t n0 = q0 ? (uint32_t)__builtin_ctz(q0) : 32u, n1 = q1 ? (uint32_t)__builtin_ctz(q1) : 32u;
                uint32_t v0 = vok && n0 >= vml ? (n0 << 2) | (3u - lane) : 0u;
                uint32_t v1 = vok && n1 >= vml ? n1 : 0u;
                auto qmax = [](uint32_t v) {  // over the quad: quad_perm 1,0,3,2 then 2,3,0,1
                    const uint32_t o = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
                    v = v > o ? v : o;
                    const uint32_t o2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
                    return v > o2 ? v : o2;
                };
                v0 = qmax(v0);
                v1 = qmax(v1);
                const uint32_t best = __builtin_amdgcn_readfirstlane(v0);
                L1 = __builtin_amdgcn_readfirstlane(v1);
                L = best >> 2;
                Dc = best ? 3u - (best & 3u) : 0u;
                D = best ? (Dc == 0 ? dd[0] : Dc == 1 ? dd[1] : dd[2]) : 0u;
            } else {
#pragma unroll
            for (int c = 0; c < NCAND; c++) {
                if (!dd[c]) continue;
                // (readlane returns int: cast through uint32_t, no sign extension)
                const uint64_t ex = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(exhi[c], t) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane(exlo[c], t);
                uint32_t n0 = (uint32_t)__builtin_ctzll(~(ex >> i));
                uint32_t n1 = (uint32_t)__builtin_ctzll(~(ex >> (i + 1)));
                n0 = n0 < (uint32_t)C::CAP ? n0 : (uint32_t)C::CAP;
                n1 = n1 < (uint32_t)C::CAP ? n1 : (uint32_t)C::CAP;
                if (n0 >= ml[c] && n0 > L) { L = n0; D = dd[c]; Dc = (uint32_t)c; }
                if (n1 >= ml[c] && n1 > L1) L1 = n1;
            }
            }
            L = __builtin_amdgcn_readfirstlane(L);
            D = __builtin_amdgcn_readfirstlane(D);
            Dc = __builtin_amdgcn_readfirstlane(Dc);
            L1 = __builtin_amdgcn_readfirstlane(L1);
            if (L < 3 || L1 > L) { o = k + 1; continue; }  // lazy: a longer match starts next
            const uint32_t p = ss + k;
            const uint32_t rem = se - p;
            const uint32_t maxlen = rem < 258 ? rem : 258;
#ifndef PBX_LZ_MASKEXT
#define PBX_LZ_MASKEXT 1  // extend capped matches from the lanes' equality masks (0: LDS compare)
#endif
            // one wave-wide compare of 4 bytes per lane extends the match from L up to lim
            auto extend_lds = [&](uint32_t lim) {
                const uint32_t a = sp.wl + p, off = L + 4 * lane;
                const uint32_t x = off < lim ? (lds_ld4(S, a - D + off) ^ lds_ld4(S, a + off)) : 0u;
                const uint64_t mm = __ballot(off >= lim || x != 0);
                // no lane stopped: the 256 bytes from L are all equal (L < 6 reaching lim = 258
                // from a sub-segment's last bytes), so the match runs to lim (ctz of 0 is no index)
                uint32_t l = lim;
                if (mm) {
                    const uint32_t f = (uint32_t)__builtin_ctzll(mm);
                    const uint32_t of = L + 4 * f;
                    if (of < lim) l = of + ((uint32_t)__builtin_ctz(__builtin_amdgcn_readlane(x, f) | 0x80000000u) >> 3);
                }
                L = __builtin_amdgcn_readfirstlane(l < lim ? l : lim);
            };
            uint32_t runk = 0;  // the chosen candidate's run of equal bytes from k (mask extension)
            if (PBX_LZ_MASKEXT && C::CAP == 32 && L >= (uint32_t)C::CAP && L < maxlen) {
                // the run of the chosen candidate's equality bits from position k over the wave's
                // masks: the rest of lane t, the whole lanes after it (a ballot of all-ones masks),
                // and the first bits of the next lane; masked bits (past se) end it, so capped at
                // maxlen it is the length the byte compare below finds
                static_assert(NCAND == 3, "three candidate masks");
                const uint32_t es = Dc == 0 ? exlo[0] : Dc == 1 ? exlo[1] : exlo[2];
                const uint64_t full = __ballot(es == 0xFFFFFFFFu);
                uint32_t run = 32 - i;  // a capped length of CAP = 32: the rest of lane t is equal
                if (t < 63) {
                    const uint32_t nf = (uint32_t)__builtin_ctzll(~(full >> (t + 1)));  // whole lanes after t
                    const uint32_t t2 = t + 1 + nf;  // the first lane that is not (all its bits < 32)
                    run += 32 * nf;
                    if (t2 < 64) run += (uint32_t)__builtin_ctz(~(uint32_t)__builtin_amdgcn_readlane(es, t2));
                }
                runk = __builtin_amdgcn_readfirstlane(run);
                L = __builtin_amdgcn_readfirstlane(run < maxlen ? run : maxlen);
            } else if (L >= (uint32_t)C::CAP && L < maxlen) {
                extend_lds(maxlen);
            }
            // a match reaching the end of the sub-segment runs on into the next one (extend_cross)
            if (p + L == se && se < sp.sl) {
                const uint32_t r2 = sp.sl - p;
                const uint32_t lim = r2 < 258 ? r2 : 258;
                if (L < lim) extend_lds(lim);
            }
            uint32_t adv = L;  // positions the recorded matches take
            if (nm < (uint32_t)C::MAXMW) {
                if (lane == 0) S.mrl[w * C::MAXMW + nm] = (p - ss) | ((L - 3) << 11) | (Dc << 19);
                nm++;
#ifndef PBX_LZ_CHAIN
#define PBX_LZ_CHAIN 1  // full 258-byte matches down a long run recorded together (0: one per step)
#endif
                // A run of the chosen candidate longer than two full matches: the walk would take
                // 258 more at k + 258 m (m = 1, 2, ...) while the run holds 258 more from there, the
                // match stays inside the sub-segment, and no earlier candidate (which wins ties) has
                // 32 equal bytes there -- the lazy rule cannot fire at the cap.  Lane m - 1 checks
                // chain position m (the earlier candidates' masks fetched by ds_bpermute); the
                // leading run of passing lanes is recorded at once (G_FAKE: a whole sub-segment in
                // one step instead of eight).
                if (PBX_LZ_CHAIN && L == 258 && runk >= 2 * 258) {
                    const uint32_t m = lane + 1, km = k + 258 * m;
                    bool ok = lane < 8 && runk >= 258 * (m + 1) && km + 258 < lsub;
                    const uint32_t tq = km >> 5 < 63 ? km >> 5 : 63u, iq = km & 31;
#pragma unroll
                    for (int c = 0; c < NCAND - 1; c++) {
                        if ((uint32_t)c >= Dc) break;  // (uniform)
                        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * tq), (int)exlo[c]);
                        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * tq), (int)exhi[c]);
                        const uint64_t ex = (((uint64_t)hi << 32) | lo) >> iq;
                        ok = ok && (uint32_t)ex != 0xFFFFFFFFu;
                    }
                    uint32_t nok = (uint32_t)__builtin_ctzll(~__ballot(ok));
                    if (nok > (uint32_t)C::MAXMW - nm) nok = (uint32_t)C::MAXMW - nm;
                    if (lane < nok) S.mrl[w * C::MAXMW + nm + lane] = km | (255u << 11) | (Dc << 19);
                    nm += nok;
                    adv += 258 * nok;
                }
                cov += adv;
                last_end = p + adv;
                // positions [p, p + adv) of this lane's chunk are covered
                const uint32_t lo = p > p0 ? p - p0 : 0u, hi = p + adv - p0;
                if (p + adv > p0 && p < p0 + 32) {
                    const uint32_t h = hi < 32 ? hi : 32u;
                    cover |= (h >= 32 ? 0xFFFFFFFFu : (1u << h) - 1u) & (0xFFFFFFFFu << lo);
                }
            }
            o = k + adv;
        }
        // ph_parse_emu's rule: matches covering < MINCOV bytes are dropped (literals only)
        if (cov < (uint32_t)C::MINCOV) {
            nm = 0;
            cover = 0;
            last_end = 0;
        }
    };
    // Matches cross the wave boundaries (ph_parse_emu: wave w parses from where wave w - 1's last
    // match ends, waves in order).  Round 0: every wave walks from a predicted start: its own
    // start when its boundary cannot be reached, else where a chain of 258-byte matches from
    // the segment start would cross it (one run over the whole segment, G_FAKE's repeated rows:
    // every prediction right).  Only if some boundary is reachable (reachm, uniform): one
    // barrier per round, then one lane per wave checks that wave's start against where the
    // previous wave's latest walk ends; while some start is wrong, EVERY wave whose start is
    // wrong walks again, all at once, from that end (round 4 repaired them one wave per round
    // in wave order).  The first wrong wave's predecessor walked from its final start (by
    // induction from wave 0), so each round fixes at least one more wave: at most NW - 1 repair
    // rounds, the records equal the serial parse's whatever the predictions.  Where a wave's
    // last match end does not depend on where it starts -- a run broken inside it, as at the
    // filter byte of every row of a filtered stream -- one round fixes every wave
    // (scripts/carry_sim.py: G_FAKE with the Up/Sub/adaptive filter, 6.9 serial rounds per
    // segment before, 1.5 now).  (One call site of the walk: two inlined copies spill
    // registers to scratch.)
    uint32_t st = ss;  // (uniform) the start of this wave's current records
#ifndef PBX_LZ_ROWPRED
#define PBX_LZ_ROWPRED 1  // row-filtered batches (VC): predict from the row start, not the segment start
#endif
    if (w && ((reachm >> (w - 1)) & 1u)) {
        if (VC && PBX_LZ_ROWPRED && sp.rowlen > 2) {
            // a row-filtered stream's runs break at every row's filter byte: predict where a chain
            // of 258-byte matches from the boundary's row start would cross it, capped at the next
            // row start (scripts/carry_sim.py, Up/Paeth/adaptive G_FAKE: 1.52 -> 0.15 repair rounds
            // per segment, Sub/Avg 1.42 -> 0.55)
            const uint32_t p = (uint32_t)((sp.base + sp.wl + ss) % sp.rowlen);
            uint32_t cand = 258u * ((p + 257u) / 258u);
            cand = cand < sp.rowlen ? cand : sp.rowlen;
            st = ss + cand - p;
        } else {
            st = 258u * ((ss + 257u) / 258u);
        }
    }
    uint32_t cur = 0, jr = 0;
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)C::NW; j++) {
        jr = j;
        bool go = j == 0 && active && !skip;
        uint32_t o0 = st - ss;
        if (j && w) {
            const uint32_t c = __builtin_amdgcn_readfirstlane(S.w_end[cur ^ 1u][w - 1]);
            const uint32_t a = c > ss ? c : ss;
            if (a != st) {
                st = a;
                go = active && !skip;
                o0 = a - ss;
            }
        }
#ifndef PBX_LZ_WALK_PROF
#define PBX_LZ_WALK_PROF 0  // diagnostics (variant build, PROF kernels): wave 0's walk / round cycles in phase slots 1 and 2
#endif
        const uint64_t tw0 = PROF && PBX_LZ_WALK_PROF ? __builtin_amdgcn_s_memtime() : 0;
        if (go) walk(o0);
        if (PROF && PBX_LZ_WALK_PROF && w == 0 && lane == 0) S.dbg_twalk += (uint32_t)(__builtin_amdgcn_s_memtime() - tw0);
        if (reachm == 0) break;  // (uniform) no match runs into another wave: no barrier at all
        if (lane == 0) {
            S.w_end[cur][w] = last_end > se ? last_end : 0u;
            S.w_st[cur][w] = active && !skip ? st : 0xFFFFFFFFu;
        }
        __syncthreads();
        // lane i (1 <= i < NW): is wave i's start where wave i - 1's latest walk ends?
        bool bad = false;
        if (lane && lane < (uint32_t)C::NW) {
            const uint32_t c = S.w_end[cur][lane - 1], si = lane * (uint32_t)C::SUB, sv = S.w_st[cur][lane];
            bad = sv != 0xFFFFFFFFu && (c > si ? c : si) != sv;
        }
        if (PROF && PBX_LZ_WALK_PROF && w == 0 && lane == 0) S.dbg_tsync += (uint32_t)(__builtin_amdgcn_s_memtime() - tw0);
        if (__ballot(bad) == 0 || j + 1 == (uint32_t)C::NW) break;  // (uniform) every start is final
        cur ^= 1u;
    }
    // the positions [ss, used) the previous wave's last match covers are not literals here
    // (w_end[cur][w - 1] holds that match's final end: written before the last barrier)
    uint32_t used = 0;
    if (reachm && w) {
        const uint32_t c = __builtin_amdgcn_readfirstlane(S.w_end[cur][w - 1]);
        used = c > ss ? c : 0u;
    }
    if (used > p0) {
        const uint32_t h = used - p0 < 32 ? used - p0 : 32u;
        cover |= h >= 32 ? 0xFFFFFFFFu : (1u << h) - 1u;
    }
    // the kept matches' length and distance symbols, one match per lane (this wave's own
    // records: LDS operations of one wave complete in order)
    __builtin_amdgcn_wave_barrier();
    for (uint32_t m = lane; m < nm; m += 64) {
        const uint32_t r = S.mrl[w * C::MAXMW + m], c = r >> 19;
        uint32_t sy, e, v;
        len_code(((r >> 11) & 255u) + 3, sy, e, v);
        atomicAdd(&S.h8[sy * LZ_HCOPIES + (lane & (LZ_HCOPIES - 1))], 1u);
        dist_code(c == 0 ? 1u : c == 1 ? 2u : sp.rowlen, sy, e, v);
        atomicAdd(&S.dfreq[sy], 1u);
    }
    if (lane == 0) S.w_nm[w] = nm;
    if (PROF && lane == 0) {
        atomicAdd(&S.dbg_walk, nsteps);
        if (w == 0) S.dbg_round = jr;
    }
}

// Container bytes before the zlib stream: TIFF header, PNG chunks up to the IDAT data, or
// (tiled TIFF) the response header in front of its first sub-tile only.
__device__ __forceinline__ uint32_t container_zoff(const TileDesc& d) {
    return (d.flags & TF_TILED) ? d.tiff_hdr : (d.flags & TF_TIFF) ? TIFF_DATA_OFFSET : PNG_IDAT_DATA_OFF;
}
__device__ __forceinline__ uint64_t container_bytes(const TileDesc& d, uint64_t payload) {
    return container_zoff(d) + ZLIB_HDR_BYTES + payload + ((d.flags & TF_TIFF) ? 4 : PNG_TAIL_BYTES);
}

// Segment g of tile i (descriptor d): its Huffman block by inverting block_seg0
// (j = ((k + 1) nb - 1) / n, checked for every n <= 300), the block's record from its first
// segment, and the segment's record fields the later kernels read (k_seg_map; k_lz77 itself
// in batches of equal segment counts).
__device__ __forceinline__ void seg_map_one(const TileDesc& d, uint32_t i, uint32_t g, SegInfo* __restrict__ info,
                                            BlkInfo* __restrict__ blk) {
    const uint32_t f = d.seg_first, n = d.seg_count, hb = d.hblk_first;
    const uint32_t nb = tile_blocks(n, PBX_TILE_BLK_CAP(d));
    const uint32_t k = g - f;
    const uint32_t j = (uint32_t)(((uint64_t)(k + 1) * nb - 1) / n);
    const uint32_t s0 = block_seg0(j, n, nb), s1 = block_seg0(j + 1, n, nb);
    if (k == s0) {
        blk[hb + j].seg0 = f + s0;
        blk[hb + j].nseg = s1 - s0;
    }
    info[g].blk = hb + j;
    info[g].tile = i;
    info[g].zoff = container_zoff(d);
    info[g].flags = (k == s0 ? SF_FIRST : 0u) | (k + 1 == s1 ? SF_LAST : 0u) | ((d.flags & TF_TIFF) ? SF_TIFF : 0u);
}

// The whole descriptor in one round of scalar loads: the fence keeps the compiler from
// sinking the plane fields' loads past the branches into a second dependent round.
__device__ __forceinline__ TileDesc load_desc(const TileDesc* p) {
    uint4 q[sizeof(TileDesc) / 16];
#pragma unroll
    for (uint32_t i = 0; i < sizeof(TileDesc) / 16; i++) q[i] = ((const uint4*)p)[i];
    asm volatile("" : "+s"(q[0].x), "+s"(q[0].y), "+s"(q[0].z), "+s"(q[0].w), "+s"(q[1].x), "+s"(q[1].y),
                 "+s"(q[1].z), "+s"(q[1].w), "+s"(q[2].x), "+s"(q[2].y), "+s"(q[2].z), "+s"(q[2].w),
                 "+s"(q[3].x), "+s"(q[3].y), "+s"(q[3].z), "+s"(q[3].w), "+s"(q[4].x), "+s"(q[4].y));
    TileDesc d;
    __builtin_memcpy(&d, q, sizeof d);
    return d;
}

constexpr uint32_t LZ_PF = 3;  // load tasks (rows x 64 chunks) per wave in flight at once

// A finished segment's results, from LDS to HBM: SegInfo (geometry, Adler-32 partials from
// S.red), the symbol histogram (the 8 copies summed), the match records (unpacked).
template <class C>
__device__ __forceinline__ void lz_write_out(const LzSmem<C>& S, uint32_t seg, const SegParams& sp, uint64_t src,
                                             SegInfo* __restrict__ info, uint32_t* __restrict__ hist,
                                             uint32_t* __restrict__ mrec, uint32_t tid) {
    if (tid < 64) {
        // the segment's Adler-32 sums from the waves' (s1_k, s2_k, n_k): s1 = sum s1_k,
        // s2 = sum (s2_k + s1_k * bytes after wave k) (adler_combine folded), lane k < NW
        // one term, reduced over the wave
        uint32_t t1 = 0, t2 = 0;
        if (tid < (uint32_t)C::NW) {
            uint32_t after = 0;
#pragma unroll
            for (int j = 1; j < C::NW; j++) after += (uint32_t)j > tid ? S.red[3 * j + 2] : 0u;
            t1 = S.red[3 * tid];
            t2 = (uint32_t)(((uint64_t)t1 * after + S.red[3 * tid + 1]) % ADLER_BASE);
        }
        const uint32_t a1 = wave_sum(t1) % ADLER_BASE, a2 = wave_sum(t2) % ADLER_BASE;  // lanes >= NW hold 0
        if (tid == 0) {
            SegInfo& g = info[seg];
            g.sl = sp.sl; g.last = sp.last; g.wl = sp.wl; g.rowlen = sp.rowlen;
            g.adler_s1 = a1; g.adler_s2 = a2;
            g.src_lo = (uint32_t)src; g.src_hi = (uint32_t)(src >> 32);
        }
    }
    uint32_t* hg = hist + (size_t)seg * HIST_WORDS;
    for (uint32_t i = tid; i < HIST_WORDS; i += C::NT) {
        uint32_t v;
        if (i < 288) {
            v = 0;
#pragma unroll
            for (uint32_t k = 0; k < LZ_HCOPIES; k += 8) {
                const uint4 a = *(const uint4*)&S.h8[i * LZ_HCOPIES + k];
                const uint4 b = *(const uint4*)&S.h8[i * LZ_HCOPIES + k + 4];
                v += (a.x + a.y) + (a.z + a.w) + (b.x + b.y) + (b.z + b.w);
            }
        } else {
            v = S.dfreq[i - 288];
        }
        hg[i] = v;
    }
    uint32_t* mg = mrec + (size_t)seg * MREC_WORDS;
    const uint32_t nmw = S.w_nm[tid & (uint32_t)(C::NW - 1)];
    if (tid < (uint32_t)C::NW) mg[tid] = nmw;
    if (__builtin_amdgcn_ballot_w64(nmw != 0) == 0) return;  // no wave kept a match (noise)
    for (uint32_t i = tid; i < (uint32_t)(C::NW * C::MAXMW); i += C::NT) {
        if (i % C::MAXMW < S.w_nm[i / C::MAXMW]) {
            const uint32_t r = S.mrl[i], c = r >> 19;
            const uint32_t pos = (i / C::MAXMW) * C::SUB + (r & 2047u);
            const uint32_t dist = c == 0 ? 1u : c == 1 ? 2u : sp.rowlen;
            mg[C::NW + i] = pos | (((r >> 11) & 255u) << 16);
            mg[C::NW + C::NW * C::MAXMW + i] = dist - 1;
        }
    }
}

// One workgroup per segment.  (A persistent variant -- a contiguous run of segments per
// workgroup, the next segment's plane rows prefetched into registers while the current one is
// parsed -- needed more registers than 8 waves per SIMD allow and spilled; the fill is
// issue-bound rather than latency-bound anyway: the same cycles with every plane read a cache
// hit, profiles/r01_s4_phase_direct_sametile.log.)
#ifndef PBX_LZ_MINB  // experiments only: the min-blocks launch bound of k_lz77 (0 = none)
#define PBX_LZ_MINB 8
#endif
#if PBX_LZ_MINB
#define PBX_LZ_BOUNDS __launch_bounds__(C::NT, PBX_LZ_MINB)
#else
#define PBX_LZ_BOUNDS __launch_bounds__(C::NT)
#endif
template <class C, bool PROF, bool VC = false>
__global__ PBX_LZ_BOUNDS void k_lz77(const TileDesc* __restrict__ dt,
                                                const uint32_t* __restrict__ seg_tile,
                                                uint32_t nseg, uint8_t* __restrict__ stream,
                                                SegInfo* __restrict__ info, BlkInfo* __restrict__ blk,
                                                uint32_t* __restrict__ hist,
                                                uint32_t* __restrict__ mrec, uint64_t* __restrict__ stamps,
                                                uint32_t uniform_nseg, uint32_t uniform_rcp, uint32_t self_map) {
    __shared__ LzSmem<C> S;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t seg = xcd_remap(blockIdx.x, gridDim.x);
    uint32_t nst = 0;
    auto stamp = [&]() {
        if (PROF && tid == 0) stamps[(size_t)seg * STAMP_STRIDE + nst] = __builtin_amdgcn_s_memtime();
        nst++;
    };
    stamp();
    // (tiles of equal segment counts: the tile by a division, one dependent load less)
    const uint32_t ti = uniform_nseg ? div_rcp(seg, uniform_nseg, uniform_rcp) : seg_tile[seg];
    const TileDesc d = load_desc(dt + ti);
    const SegParams sp = seg_params(d, seg - d.seg_first);
    if (self_map && tid == 0) seg_map_one(d, ti, seg, info, blk);  // (small batches: no k_seg_map launch)
    const bool direct = (d.flags & TF_DIRECT) != 0;
    DirectRows dr;  // (before the branch: one round of descriptor loads, not two)
    dr.init(d);
    const uint32_t nz = lz_fill_bytes<C>(sp) & ~15u;
#ifndef PBX_LZ_SKIP_STORE
#define PBX_LZ_SKIP_STORE 0  // timing experiments only (scripts/variants.sh): wrong output
#endif
#ifndef PBX_LZ_SKIP_FILL
#define PBX_LZ_SKIP_FILL 0  // timing experiments only (scripts/variants.sh): wrong output
#endif
    bool stored = false;  // the segment's stream bytes already written (fill_fast)
    if (PBX_LZ_SKIP_FILL) {
    } else if (direct && PBX_LZ_FAST_FILL &&
               fill_fast_any<C::NT>(S.buf, dr, (uint32_t)sp.base, sp.wl + sp.sl, nz, tid,
                                    PBX_LZ_SKIP_STORE || PBX_ENC_FROM_PLANE == 1 ||
                                            (PBX_ENC_FROM_PLANE == 2 && fast_fill_mode(dr) == 5u)
                                        ? nullptr
                                        : stream + d.out_off + sp.base + sp.wl,
                                    sp.wl)) {
        stored = true;  // (or not needed: k_encode reads the plane)
        if (PROF) stamp();
    } else if (direct) {
        FillPre<LZ_PF> pf;
        fill_issue<C::NT, LZ_PF>(pf, dr, (uint32_t)sp.base, sp.wl + sp.sl, tid);
        if (PROF) stamp();  // diagnostics: the first loads issued
        fill_finish<C::NT, LZ_PF>(pf, S.buf, dr, (uint32_t)sp.base, sp.wl + sp.sl, nz, tid);
    } else {
        load_bytes16<C::NT>(S.buf, stream + d.out_off + sp.base, sp.wl + sp.sl, nz, tid);
        if (PROF) stamp();
    }
    for (uint32_t k = tid; k < 288 * LZ_HCOPIES; k += C::NT) S.h8[k] = 0;
    if (tid < 32) S.dfreq[tid] = 0;
    if (tid == 0) S.reachw = 0;
    if (PROF && tid == 0) S.dbg_walk = S.dbg_twalk = S.dbg_tsync = 0;
    if (PROF) {  // diagnostics: wave 0's fill done
        __builtin_amdgcn_s_waitcnt(0);
        stamp();
    }
    __syncthreads();
    if (direct && !stored && !PBX_LZ_SKIP_STORE) {  // the segment's stream bytes for k_encode (16-byte words; slack after every tile)
        uint8_t* o = stream + d.out_off + sp.base + sp.wl;
        for (uint32_t k = tid; k < (sp.sl + 15) / 16; k += C::NT)
            *(uint4*)(o + 16 * k) = *(const uint4*)(S.buf + sp.wl / 4 + 4 * k);
    }
    stamp();
    // the thread's chunk words (and the word before it) from LDS
    // (wl is a multiple of 16: two aligned 16-byte reads; the word before the chunk is the
    // previous lane's last, one wave shift; lane 0 reads it)
    const uint32_t cs = tid * C::CH, wi = (sp.wl + cs) >> 2;
    uint32_t cw[9];
    {
        const uint4 q0 = *(const uint4*)&S.buf[wi], q1 = *(const uint4*)&S.buf[wi + 4];
        cw[1] = q0.x; cw[2] = q0.y; cw[3] = q0.z; cw[4] = q0.w;
        cw[5] = q1.x; cw[6] = q1.y; cw[7] = q1.z; cw[8] = q1.w;
        const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)cw[8], 0x138, 0xF, 0xF, false);  // wave_shr:1
        cw[0] = lane ? prev : (wi ? S.buf[wi - 1] : 0u);
    }
    uint32_t cover = 0, smask = 0xFFFFFFFFu;
#ifndef PBX_LZ_SKIP_PARSE
#define PBX_LZ_SKIP_PARSE 0  // timing experiments only: no matches (valid output, lower ratio)
#endif
    if (PBX_LZ_SKIP_PARSE) {
        if (lane == 0) S.w_nm[w] = 0;
        const uint32_t p0 = tid * C::CH;
        const uint32_t nval = sp.sl > p0 ? sp.sl - p0 : 0u;
        smask = nval >= 32 ? 0xFFFFFFFFu : (1u << nval) - 1u;
    } else {
        ph_parse_dev<C, LzSmem<C>, PROF, VC>(tid, S, sp, cw, cover, smask);
    }
    stamp();
    // the chunk's words for the histogram and Adler-32
    uint32_t cb[8];
#ifndef PBX_LZ_CBRELOAD  // experiment: reloaded (kept in registers: 0.08 ms faster, profiles/r04i/)
#pragma unroll
    for (int k = 0; k < 8; k++) cb[k] = cw[k + 1];
#else
    {
        const uint4 q0 = *(const uint4*)&S.buf[wi], q1 = *(const uint4*)&S.buf[wi + 4];
        cb[0] = q0.x; cb[1] = q0.y; cb[2] = q0.z; cb[3] = q0.w;
        cb[4] = q1.x; cb[5] = q1.y; cb[6] = q1.z; cb[7] = q1.w;
    }
#endif
    // literal histogram of the chunk (positions no recorded match covers), 8 interleaved
    // copies against same-address LDS atomics, branch-free: a covered position adds into the
    // lane's own sink word.  Adler-32 partial sums from the same words.
#ifndef PBX_LZ_SKIP_HIST
#define PBX_LZ_SKIP_HIST 0  // timing experiments only: wrong output
#endif
    if (!PBX_LZ_SKIP_HIST) {
        const uint32_t lit = ~cover & smask, cp = lane & (LZ_HCOPIES - 1);
        if (__builtin_amdgcn_ballot_w64(lit != 0xFFFFFFFFu) == 0) {
            // every position of the wave a literal (no kept match, whole chunks: most waves on
            // noisy data): the bin address only, no per-position select
#pragma unroll
            for (int j = 0; j < 32; j++) {
                const uint32_t bt = (cb[j >> 2] >> ((j & 3) * 8)) & 0xFFu;
                atomicAdd(&S.h8[bt * LZ_HCOPIES + cp], 1u);
            }
        } else {
            const uint32_t sink = (uint32_t)(&S.hdummy[lane] - S.h8);
#pragma unroll
            for (int j = 0; j < 32; j++) {
                const uint32_t bt = (cb[j >> 2] >> ((j & 3) * 8)) & 0xFFu;
                atomicAdd(&S.h8[((lit >> j) & 1u) ? bt * LZ_HCOPIES + cp : sink], 1u);
            }
        }
    }
    if (tid == 0) atomicAdd(&S.h8[256 * LZ_HCOPIES], 1u);  // end of block
    uint32_t s1 = 0, s2 = 0, n = 0;
    if (cs < sp.sl) {
        const uint32_t ce = cs + C::CH < sp.sl ? cs + C::CH : sp.sl;
        n = ce - cs;
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)C::CH / 4; k++) {
            const uint32_t v = cb[k];  // bytes past the segment are zero in buf
            const uint32_t e = (uint32_t)C::CH - 4 * k;
            s1 = dot4_u8(v, 0x01010101u, s1);
            s2 = dot4_u8(v, e | ((e - 1) << 8) | ((e - 2) << 16) | ((e - 3) << 24), s2);
        }
        s2 -= (cs + (uint32_t)C::CH - ce) * s1;
    }
    // Adler-32 partials of the wave on raw sums (one wave covers <= 2048 bytes: s1 < 2^20,
    // s2 < 2^31, no modular reduction needed): s1 = sum s1_l, s2 = sum (s2_l + s1_l * bytes
    // of the lanes after l), by DPP scans and sums (no ds_bpermute round trips)
    {
        const uint32_t ninc = wave_incl_scan_dpp(n);
        const uint32_t ntot = (uint32_t)__builtin_amdgcn_readlane((int)ninc, 63);
        const uint32_t w1 = wave_incl_scan_dpp(s1), w2 = wave_incl_scan_dpp(s2 + s1 * (ntot - ninc));
        if (lane == 63) { S.red[3 * w] = w1 % ADLER_BASE; S.red[3 * w + 1] = w2 % ADLER_BASE; S.red[3 * w + 2] = ntot; }
    }
    __syncthreads();
    stamp();
#ifndef PBX_LZ_SKIP_OUT
#define PBX_LZ_SKIP_OUT 0  // timing experiments only: wrong output
#endif
    if (!PBX_LZ_SKIP_OUT) lz_write_out<C>(S, seg, sp, d.out_off + sp.base + sp.wl, info, hist, mrec, tid);
    stamp();
    // (diagnostics: slot 7 = slot 6 + the walk steps, so the lz77 report's "7:" is their mean;
    // slots 30/31 (unused by k_encode) differ by 1 + 1000 x the repair rounds: encode "7:")
    if (PROF && tid == 0) {
        const uint64_t t6 = stamps[(size_t)seg * STAMP_STRIDE + 6];
        stamps[(size_t)seg * STAMP_STRIDE + 7] = t6 + S.dbg_walk;
        stamps[(size_t)seg * STAMP_STRIDE + 30] = t6;
        stamps[(size_t)seg * STAMP_STRIDE + 31] = t6 + 1 + 1000ull * S.dbg_round;
        if (PBX_LZ_WALK_PROF) {  // "1:" wave 0's walk cycles, "2:" its round cycles (walks included)
            const uint64_t t0 = stamps[(size_t)seg * STAMP_STRIDE];
            stamps[(size_t)seg * STAMP_STRIDE + 1] = t0 + 1 + S.dbg_twalk;
            stamps[(size_t)seg * STAMP_STRIDE + 2] = t0 + 2 + S.dbg_twalk + S.dbg_tsync;
        }
    }
}

// ==================================================================== k_huff
// x of lane (lane ^ M) without an LDS round trip: DPP quad permutes (1, 2), two row shifts
// and a select (4), a row rotate (8), gfx950's permlane swaps and a select (16, 32).
template <uint32_t M>
__device__ __forceinline__ uint32_t lane_xor(uint32_t x, uint32_t lane) {
    if constexpr (M == 1) {
        return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
    } else if constexpr (M == 2) {
        return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
    } else if constexpr (M == 4) {
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x104, 0xF, 0xF, false);  // row_shl:4
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
        return (lane & 4u) ? dn : up;
    } else if constexpr (M == 8) {
        return (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x128, 0xF, 0xF, false);  // row_ror:8
    } else if constexpr (M == 16) {
        const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return (lane & 16u) ? p[0] : p[1];
    } else {
        static_assert(M == 32, "lane distances 1 .. 32");
        const auto p = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return (lane & 32u) ? p[0] : p[1];
    }
}
// Wave sums of N per-lane values at once, the sum of value k landing in lane k (k < N <= 64):
// a transposing butterfly.  Slot k starts in register k; at each lane distance h = 32 .. 1
// the registers pair up (k, k + h) and trade halves so that one add leaves slot k's partial
// sums in the lanes whose bit h is clear and slot k + h's where it is set -- gfx950's lane
// swaps for 32 and 16, then DPP row mirror (8), half-row mirror (4) and quad permutes (2, 1),
// each folded into its add (a mirror partner differs in bit h and agrees in the bits already
// split; the mirrors' merged lane classes still cover each row once).  Registers that hold
// no slot below N are skipped at compile time: 17 values take 111 VALU instructions, 34 take
// 141, against 17 / 34 wave_sum row scans and lane reads.
__device__ constexpr bool lane_sums_nz(uint32_t n, uint32_t w, uint32_t j) {  // register j of w holds a slot < n
    for (uint32_t s = j; s < 64; s += w)
        if (s < n) return true;
    return false;
}
template <uint32_t H>
__device__ __forceinline__ uint32_t lane_sums_step(uint32_t x, uint32_t y, uint32_t lane) {
    const bool hi = (lane & H) != 0;
    const uint32_t keep = hi ? y : x, send = hi ? x : y;
    constexpr int ctl = H == 8 ? 0x140 : H == 4 ? 0x141 : H == 2 ? 0x4E : 0xB1;  // row_mirror, row_half_mirror, quad_perm
    return keep + (uint32_t)__builtin_amdgcn_update_dpp(0, (int)send, ctl, 0xF, 0xF, false);
}
template <uint32_t N>
__device__ __forceinline__ uint32_t wave_sums_to_lanes(const uint32_t (&v)[N], uint32_t lane) {
    static_assert(N >= 1 && N <= 64, "one slot per lane");
    uint32_t r[32];
#pragma unroll
    for (uint32_t j = 0; j < 32; j++) {
        if (lane_sums_nz(N, 64, j) || lane_sums_nz(N, 64, j + 32)) {
            const auto p = __builtin_amdgcn_permlane32_swap(v[j < N ? j : 0], j + 32 < N ? v[j + 32 < N ? j + 32 : 0] : 0u,
                                                            false, false);
            r[j] = p[0] + p[1];
        } else {
            r[j] = 0;
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < 16; j++) {
        if (lane_sums_nz(N, 32, j) || lane_sums_nz(N, 32, j + 16)) {
            const auto p = __builtin_amdgcn_permlane16_swap(r[j], r[j + 16], false, false);
            r[j] = p[0] + p[1];
        } else {
            r[j] = 0;
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < 8; j++) r[j] = lane_sums_nz(N, 16, j) || lane_sums_nz(N, 16, j + 8) ? lane_sums_step<8>(r[j], r[j + 8], lane) : 0u;
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) r[j] = lane_sums_nz(N, 8, j) || lane_sums_nz(N, 8, j + 4) ? lane_sums_step<4>(r[j], r[j + 4], lane) : 0u;
#pragma unroll
    for (uint32_t j = 0; j < 2; j++) r[j] = lane_sums_nz(N, 4, j) || lane_sums_nz(N, 4, j + 2) ? lane_sums_step<2>(r[j], r[j + 2], lane) : 0u;
    return lane_sums_step<1>(r[0], r[1], lane);
}

template <uint32_t M>
__device__ __forceinline__ void lane_xor8(const uint32_t (&v)[8], uint32_t (&o)[8], uint32_t lane) {
#pragma unroll
    for (int r = 0; r < 8; r++) o[r] = lane_xor<M>(v[r], lane);
}

// Ascending sort of the KEYN keys (padded to 512 with KEY_NONE) by one wave: 8 per lane (lane*8 + r), partners at distance
// j >= 8 by lane exchanges (lane_xor, no LDS), j < 8 inside the lane's registers.
__device__ __forceinline__ void sort512_wave(uint32_t* keys, uint32_t lane) {
    uint32_t v[8];
#pragma unroll
    for (int r = 0; r < 8; r++) v[r] = lane * 8 + r < KEYN ? keys[lane * 8 + r] : KEY_NONE;
#pragma unroll
    for (uint32_t k = 2; k <= 512; k <<= 1) {
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            if (j >= 8) {
                uint32_t ox[8];
                switch (j >> 3) {
                case 1: lane_xor8<1>(v, ox, lane); break;
                case 2: lane_xor8<2>(v, ox, lane); break;
                case 4: lane_xor8<4>(v, ox, lane); break;
                case 8: lane_xor8<8>(v, ox, lane); break;
                case 16: lane_xor8<16>(v, ox, lane); break;
                default: lane_xor8<32>(v, ox, lane); break;
                }
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    const uint32_t o = ox[r];
                    const uint32_t e = lane * 8 + r;
                    const bool up = (e & k) == 0, lower = (e & j) == 0;
                    v[r] = (lower == up) ? (v[r] < o ? v[r] : o) : (v[r] < o ? o : v[r]);
                }
            } else {
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    if (r & j) continue;
                    const int p = r | (int)j;
                    const uint32_t e = lane * 8 + r;
                    const uint32_t a = v[r], b = v[p], lo = a < b ? a : b, hi = a < b ? b : a;
                    if ((e & k) == 0) { v[r] = lo; v[p] = hi; } else { v[r] = hi; v[p] = lo; }
                }
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 8; r++)
        if (lane * 8 + r < KEYN) keys[lane * 8 + r] = v[r];
}

// LDS visibility among the lanes of ONE wave (its LDS operations complete in order): no
// workgroup barrier, so the waves of a workgroup can run different trees (k_huff<.., 2>).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <bool WS>
__device__ __forceinline__ void huff_sync() {
    if (WS) wave_lds_sync(); else __syncthreads();
}

// The Huffman merge of tree T on one wave, in rounds.  Internal nodes are created in
// non-decreasing weight order, so once node ni-1 (weight W) exists every node still to come
// weighs >= W: the remaining leaves of weight <= W and the internal nodes not yet consumed
// form a fixed prefix of the merged sequence (leaves first on ties), and its consecutive
// pairs are the next internal nodes, all built at once.  An odd last element waits for the
// next round; a lone element pairs with the next leaf.  About 16 rounds replace the ~285
// steps of the serial merge and give exactly its records (twoqueue_serial in deflate_seg.h,
// which the emulator runs): step s = li0 | qi0 << 10 | cnt << 20.
template <bool WS = false, class SM>
__device__ __forceinline__ void huff_rounds_wave(SM& S, uint32_t T, uint32_t lane) {
    const uint32_t n = __builtin_amdgcn_readfirstlane(S.misc[T ? M_ND : M_NL]);
    const uint32_t base = __builtin_amdgcn_readfirstlane(T ? S.misc[M_NL] : 0u);
    const uint32_t* sk = S.hs.skey + base;
    uint32_t* iq = S.hs.iw[T];        // internal weights (aA, dB are free until the parents)
    uint16_t* M = S.hs.leafpar[T];    // merged prefix: leaf index | 0x8000, or internal index
                                      // (<= n entries: tree T's own part, the trees may run at once)
    uint32_t* rq = S.hs.rec[T];
    uint16_t* rs = S.hs.rst[T];
    if (n < 2) {
        if (lane == 0) S.nrounds[T] = 0;
        return;
    }
    if (lane == 0) {
        iq[0] = key_weight(sk[0]) + key_weight(sk[1]);
        rq[0] = 2u << 20;
        rs[0] = 0;
    }
    uint32_t li = 2, qi = 0, ni = 1, nr = 1;
    huff_sync<WS>();
    while (ni + 1 < n) {
        if (lane == 0) rs[nr] = (uint16_t)ni;  // this round creates nodes ni..
        nr++;
        const uint32_t W = iq[ni - 1];
        uint32_t a = 0;
        for (uint32_t c = li; c < n; c += 64) {  // leaves are sorted: count those <= W
            const uint32_t i = c + lane;
            const uint64_t m = __ballot(i < n && key_weight(sk[i]) <= W);
            a += (uint32_t)__builtin_popcountll(m);
            if (~m) break;
        }
        a = __builtin_amdgcn_readfirstlane(a);
        const uint32_t b = ni - qi, P = a + b;
        if (P == 1) {  // the lone internal node qi pairs with the next leaf
            if (lane == 0) {
                iq[ni] = iq[qi] + key_weight(sk[li]);
                rq[ni] = li | (qi << 10) | (1u << 20);
            }
            li++; qi++; ni++;
            huff_sync<WS>();
            continue;
        }
        for (uint32_t e = lane; e < a; e += 64) {  // leaf li+e: after internal nodes < it
            const uint32_t w = key_weight(sk[li + e]);
            uint32_t lo = qi, hi = ni;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (iq[mid] < w) lo = mid + 1; else hi = mid;
            }
            M[e + lo - qi] = (uint16_t)((li + e) | 0x8000u);
        }
        for (uint32_t e = lane; e < b; e += 64) {  // internal qi+e: after leaves <= it
            const uint32_t w = iq[qi + e];
            uint32_t lo = li, hi = li + a;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (key_weight(sk[mid]) <= w) lo = mid + 1; else hi = mid;
            }
            M[e + lo - li] = (uint16_t)(qi + e);
        }
        huff_sync<WS>();
        const uint32_t m = P >> 1;
        // leaves among the first p merged elements, from the element at p
        auto leaves_before = [&](uint32_t p, uint32_t x) -> uint32_t {
            return (x & 0x8000u) ? (x & 0x7FFFu) - li : p - (x - qi);
        };
        for (uint32_t k = lane; k < m; k += 64) {
            const uint32_t x0 = M[2 * k], x1 = M[2 * k + 1];
            const uint32_t w0 = (x0 & 0x8000u) ? key_weight(sk[x0 & 0x7FFFu]) : iq[x0];
            const uint32_t w1 = (x1 & 0x8000u) ? key_weight(sk[x1 & 0x7FFFu]) : iq[x1];
            const uint32_t lb = leaves_before(2 * k, x0);
            const uint32_t cnt = (x0 >> 15) + (x1 >> 15);
            iq[ni + k] = w0 + w1;
            rq[ni + k] = (li + lb) | ((qi + 2 * k - lb) << 10) | (cnt << 20);
        }
        uint32_t lb = a;
        if (2 * m < P) lb = leaves_before(2 * m, M[2 * m]);
        lb = __builtin_amdgcn_readfirstlane(lb);
        li += lb;
        qi += 2 * m - lb;
        ni += m;
        huff_sync<WS>();
    }
    if (lane == 0) {
        rs[nr] = (uint16_t)ni;
        S.nrounds[T] = nr;
    }
}

// Parents from the merge records (ph_parents without the pointer-jumping depths, which the
// device does not use): leafpar of every leaf, aA of every internal node.
template <class SM>
__device__ __forceinline__ void parents_wave(SM& S, uint32_t tid) {
    for (uint32_t i = tid; i < 320; i += 64) {
        uint32_t T, s;
        tree_slot(i, T, s);
        const uint32_t n = tree_n(S.misc, T);
        if (s + 1 >= n) continue;
        const uint32_t r = S.hs.rec[T][s];
        const uint32_t li0 = r & 0x3FF, qi0 = (r >> 10) & 0x3FF, cnt = r >> 20;
        for (uint32_t j = li0; j < li0 + cnt; j++) S.hs.leafpar[T][j] = (uint16_t)s;
        for (uint32_t k = qi0; k < qi0 + 2 - cnt; k++) S.hs.aA[T][k] = (uint16_t)s;
        if (s + 2 == n) S.hs.aA[T][s] = (uint16_t)s;  // the root
    }
}

// Depth of every internal node, root first: a node's parent is created in a later merge
// round, so the rounds taken in reverse order each resolve in one parallel step (instead
// of pointer jumping).  Result in dB, as ph_jump leaves it.
template <bool WS = false, class SM>
__device__ __forceinline__ void depths_wave(SM& S, uint32_t T, uint32_t lane) {
    const uint32_t nr = __builtin_amdgcn_readfirstlane(S.nrounds[T]);
    if (nr == 0) return;
    uint16_t* dd = S.hs.dB[T];
    const uint16_t* par = S.hs.aA[T];
    const uint32_t root = S.hs.rst[T][nr] - 1u;  // the last round creates only the root
    if (lane == 0) dd[root] = 0;
    huff_sync<WS>();
    for (int32_t r = (int32_t)nr - 2; r >= 0; r--) {
        const uint32_t k0 = S.hs.rst[T][r], k1 = S.hs.rst[T][r + 1];
        for (uint32_t k = k0 + lane; k < k1; k += 64) dd[k] = (uint16_t)(dd[par[k]] + 1);
        huff_sync<WS>();
    }
}

// Code lengths of both trees from the repaired bit-length counts (ph_assign's result):
// leaf j of a tree gets the length L with end(L+1) <= j < end(L), end(L) = leaves of
// length >= L.  Sums and maxima by wave reductions instead of same-address LDS atomics.
template <class SM>
__device__ __forceinline__ void assign_wave(SM& S, uint32_t lane) {
    uint32_t e0[16], e1[16];
#pragma unroll
    for (int L = 1; L < 16; L++) {
        e0[L] = S.hstart[0][L] + S.hblc[0][L];
        e1[L] = S.hstart[1][L] + S.hblc[1][L];
    }
    const uint32_t nl = S.misc[M_NL], nd = S.misc[M_ND];
    uint32_t dyn = 0, fix = 0, hlit = 257, hdist = 1;
#pragma unroll
    for (int it = 0; it < 5; it++) {
        const uint32_t i = lane + 64 * it;
        const uint32_t T = i >= 288 ? 1u : 0u, j = T ? i - 288 : i;
        if (j >= (T ? nd : nl)) continue;
        const uint32_t key = S.hs.skey[(T ? nl : 0u) + j], sym = key & 0x1FF;
        uint32_t L = 0;
#pragma unroll
        for (int l = 1; l < 16; l++) L += j < (T ? e1[l] : e0[l]) ? 1u : 0u;
        if (T == 0) {
            S.lcode[sym] = L << 16;
            atomicOr(&S.lbm[L * 9 + (sym >> 5)], 1u << (sym & 31));
            const uint32_t f = S.lfreq[sym];
            const uint32_t eb = sym >= 257 ? len_sym_ebits(sym) : 0;
            dyn += f * (L + eb);
            fix += f * (fixed_lit_len(sym) + eb);
            hlit = sym + 1 > hlit ? sym + 1 : hlit;
        } else {
            S.dcode[sym] = L << 16;
            atomicOr(&S.dbm[L], 1u << sym);
            const uint32_t f = S.dfreq[sym];
            const uint32_t eb = dist_sym_ebits(sym);
            dyn += f * (L + eb);
            fix += f * (5 + eb);
            hdist = sym + 1 > hdist ? sym + 1 : hdist;
        }
    }
    auto xstep = [&](auto m) {  // one butterfly level of the sums and maxima (lane_xor, no LDS)
        constexpr uint32_t M = decltype(m)::value;
        dyn += lane_xor<M>(dyn, lane);
        fix += lane_xor<M>(fix, lane);
        const uint32_t h1 = lane_xor<M>(hlit, lane), h2 = lane_xor<M>(hdist, lane);
        hlit = h1 > hlit ? h1 : hlit;
        hdist = h2 > hdist ? h2 : hdist;
    };
    xstep(std::integral_constant<uint32_t, 32>{});
    xstep(std::integral_constant<uint32_t, 16>{});
    xstep(std::integral_constant<uint32_t, 8>{});
    xstep(std::integral_constant<uint32_t, 4>{});
    xstep(std::integral_constant<uint32_t, 2>{});
    xstep(std::integral_constant<uint32_t, 1>{});
    if (lane == 0) {
        S.misc[M_DYNBITS] = dyn; S.misc[M_FIXBITS] = fix;
        S.misc[M_HLIT] = hlit; S.misc[M_HDIST] = hdist;
    }
}

// The code-length RLE (ph_rle_mark / _count / the scan / _emit) on one wave, same symbols
// and counts: lane l holds code lengths l, l + 64, ..; run starts by DPP compares and five
// ballots (no run-start bitmask walked in LDS), every run's length from the next set bit of
// the masks, its symbol count in closed form, the offsets by a wave scan, then each run's
// first lane writes its symbols.
template <class SM>
__device__ __forceinline__ void rle_wave(SM& S, uint32_t lane) {
    const uint32_t hlit = S.misc[M_HLIT], ntot = hlit + S.misc[M_HDIST];
    uint32_t v[5];
    uint64_t M[5];
    uint32_t prev_last = 0xFFFFFFFFu;  // (position -1: no length)
#pragma unroll
    for (int it = 0; it < 5; it++) {
        const uint32_t i = lane + 64u * it;
        v[it] = i < ntot ? (i < hlit ? S.lcode[i] >> 16 : S.dcode[i - hlit] >> 16) : 0xFFu;
        const uint32_t pv = (uint32_t)__builtin_amdgcn_update_dpp((int)prev_last, (int)v[it], 0x138, 0xF, 0xF, false);  // wave_shr:1
        M[it] = __ballot(i < ntot && v[it] != pv);
        prev_last = (uint32_t)__builtin_amdgcn_readlane((int)v[it], 63);
    }
    uint32_t F[5];  // the first run start in the blocks after it (ntot: none)
    F[4] = ntot;
#pragma unroll
    for (int it = 3; it >= 0; it--) F[it] = M[it + 1] ? 64u * (it + 1) + (uint32_t)__builtin_ctzll(M[it + 1]) : F[it + 1];
    uint32_t cnt[5], run[5], base = 0, off[5];
#pragma unroll
    for (int it = 0; it < 5; it++) {
        const uint32_t i = lane + 64u * it;
        const bool st = (M[it] >> lane) & 1ull;
        const uint64_t hi = lane < 63 ? M[it] & (~0ull << (lane + 1)) : 0ull;
        const uint32_t nx = hi ? 64u * it + (uint32_t)__builtin_ctzll(hi) : F[it];
        run[it] = st ? (nx < ntot ? nx : ntot) - i : 0u;
        const uint32_t c = st ? rle_nsyms_closed(v[it], run[it]) : 0u;
        cnt[it] = c;
        const uint32_t incl = wave_incl_scan_dpp(c);
        off[it] = base + incl - c;
        base += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    }
    if (lane == 0) S.misc[M_NRLE] = base;
    uint32_t* cf = S.hw.clfreq;
#pragma unroll
    for (int it = 0; it < 5; it++) {
        if (!cnt[it]) continue;
        uint32_t k = off[it], r = run[it];
        const uint32_t x = v[it];
        if (x == 0) {
            while (r >= 11) {
                const uint32_t n = r < 138 ? r : 138;
                S.rle[k++] = 18u | ((n - 11) << 8); atomicAdd(&cf[18], 1u); r -= n;
            }
            if (r >= 3) { S.rle[k++] = 17u | ((r - 3) << 8); atomicAdd(&cf[17], 1u); r = 0; }
            while (r) { S.rle[k++] = 0; atomicAdd(&cf[0], 1u); r--; }
        } else {
            S.rle[k++] = x; atomicAdd(&cf[x], 1u); r--;
            while (r >= 3) {
                const uint32_t n = r < 6 ? r : 6;
                S.rle[k++] = 16u | ((n - 3) << 8); atomicAdd(&cf[16], 1u); r -= n;
            }
            while (r) { S.rle[k++] = x; atomicAdd(&cf[x], 1u); r--; }
        }
    }
}

// The 19-symbol code-length code on one wave (lane s = symbol s); same result as ph_clen:
// stable (freq, symbol) order, serial two-queue merge on lane-held arrays, depths, zlib's
// overflow repair at 7 bits, longest codes to the least frequent, canonical codes.
template <bool WS = false, class SM>
__device__ __forceinline__ void clen_wave(SM& S, uint32_t lane) {
    const bool sy = lane < 19;
    uint32_t f = sy ? S.hw.clfreq[lane] : 0u;
    {   // at least two used symbols: the first unused ones get frequency 1
        const uint64_t used = __ballot(sy && f != 0);
        const uint32_t nu = (uint32_t)__builtin_popcountll(used);
        if (nu < 2) {
            const uint64_t zero = __ballot(sy && f == 0);
            const uint32_t zr = (uint32_t)__builtin_popcountll(zero & ((1ull << lane) - 1ull));
            if (sy && f == 0 && zr < 2 - nu) f = 1;
        }
    }
    const bool used = sy && f != 0;
    const uint32_t ncl = (uint32_t)__builtin_popcountll(__ballot(used));
    uint32_t rank = 0;  // position in ascending (freq, symbol) order
    for (uint32_t t = 0; t < 19; t++) {
        const uint32_t ft = __builtin_amdgcn_readlane(f, t);
        rank += (ft != 0 && (ft < f || (ft == f && t < lane))) ? 1u : 0u;
    }
    // weights in sorted order: lane p holds the weight of the p-th used symbol
    uint32_t wv = 0;
    for (uint32_t t = 0; t < 19; t++) {
        const uint32_t ft = __builtin_amdgcn_readlane(f, t), rt = __builtin_amdgcn_readlane(rank, t);
        if (ft != 0 && rt == lane) wv = ft;
    }
    // serial two-queue merge (leaves 0..ncl, internal ncl..2ncl-2), parents lane-held
    uint32_t pv = 0;
    uint32_t li = 0, qi = ncl, nxt = ncl;
    for (uint32_t k = 0; k + 1 < ncl; k++) {
        uint32_t a, b;
        const uint32_t wl0 = __builtin_amdgcn_readlane(wv, li < 63 ? li : 63);
        const uint32_t wq0 = __builtin_amdgcn_readlane(wv, qi < 63 ? qi : 63);
        if (li < ncl && (qi >= nxt || wl0 <= wq0)) a = li++; else a = qi++;
        const uint32_t wl1 = __builtin_amdgcn_readlane(wv, li < 63 ? li : 63);
        const uint32_t wq1 = __builtin_amdgcn_readlane(wv, qi < 63 ? qi : 63);
        if (li < ncl && (qi >= nxt || wl1 <= wq1)) b = li++; else b = qi++;
        const uint32_t sum = __builtin_amdgcn_readlane(wv, a) + __builtin_amdgcn_readlane(wv, b);
        wv = lane == nxt ? sum : wv;
        pv = (lane == a || lane == b) ? nxt : pv;
        nxt++;
    }
    // depths: root 2ncl-2 at 0, then every node below its parent (parents have larger index)
    uint32_t dv = 0;
    if (ncl >= 2) {
        for (int32_t i = (int32_t)(2 * ncl) - 3; i >= 0; i--) {
            const uint32_t p = __builtin_amdgcn_readlane(pv, (uint32_t)i);
            const uint32_t d = __builtin_amdgcn_readlane(dv, p) + 1;
            dv = lane == (uint32_t)i ? d : dv;
        }
    }
    // bit-length counts (lane L holds blc[L]) and overflow repair
    const bool leaf = lane < ncl;
    // zlib counts every node deeper than 7, internal ones (lanes ncl..2ncl-3) included
    const uint32_t over = (uint32_t)__builtin_popcountll(__ballot(lane + 2 < 2 * ncl && dv > 7));
    const uint32_t dcl = dv > 7 ? 7u : dv;
    uint32_t blc = 0;
    for (uint32_t L = 1; L <= 7; L++) {
        const uint32_t c = (uint32_t)__builtin_popcountll(__ballot(leaf && dcl == L));
        blc = lane == L ? c : blc;
    }
    for (int32_t ov = (int32_t)over; ov > 0; ov -= 2) {
        const uint64_t nz = __ballot(lane >= 1 && lane <= 6 && blc != 0);
        const uint32_t bits = 63u - (uint32_t)__builtin_clzll(nz);
        blc += (lane == bits ? 0xFFFFFFFFu : 0u) + (lane == bits + 1 ? 2u : 0u) +
               (lane == 7 ? 0xFFFFFFFFu : 0u);
    }
    // end(L) = sum of blc[L..7]; sorted position p gets #{L : p < end(L)}
    uint32_t endv = 0;
    for (uint32_t L = 7; L >= 1; L--) {
        const uint32_t c = __builtin_amdgcn_readlane(blc, L);
        endv += lane <= L ? c : 0u;  // lane L accumulates blc[L..7]
    }
    // (cross-lane reads stay outside divergent code: a lane inactive in a branch may not
    // hold its value there)
    uint32_t len = 0;
    for (uint32_t L = 1; L <= 7; L++) {
        const uint32_t eL = __builtin_amdgcn_readlane(endv, L);
        len += (used && rank < eL) ? 1u : 0u;
    }
    // canonical codes (huff_codes)
    uint32_t code = 0, nextc = 0;
    for (uint32_t L = 1; L <= 7; L++) {
        const uint32_t prev = (uint32_t)__builtin_popcountll(__ballot(sy && len == L - 1 && L > 1));
        nextc = (nextc + prev) << 1;
        const uint64_t mL = __ballot(sy && len == L);
        if (len == L) code = nextc + (uint32_t)__builtin_popcountll(mL & ((1ull << lane) - 1ull));
    }
    if (sy) {
        S.hw.cllen[lane] = len;
        S.hw.clcode[lane] = len ? (bitrev(code, len) | (len << 16)) : 0u;
        S.hw.clfreq[lane] = f;
    }
    huff_sync<WS>();
    const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < 19; k++) o = lane == (uint32_t)k ? order[k] : o;
    const uint64_t nzo = __ballot(sy && S.hw.cllen[o] != 0);
    const uint32_t hclen = nzo ? 64u - (uint32_t)__builtin_clzll(nzo) : 0u;
    if (lane == 0) S.misc[M_HCLEN] = hclen < 4 ? 4u : hclen;
}

#ifndef PBX_HUFF_LDSEG
#define PBX_HUFF_LDSEG 17  // 4: 0.215 ms, 8: 0.213, 12: 0.208 (profiles/r03_p19/); one block per tile: 8: 0.131, 12: 0.124, 17: 0.119, 24: 0.158 (99 / 134 VGPRs: 4 / 3 waves per SIMD, profiles/r05r/)
#endif
constexpr uint32_t HUFF_LDSEG = PBX_HUFF_LDSEG;  // k_huff: segments whose histogram loads are in flight together
constexpr uint32_t HUFF_SMALL_BLKS = 256;   // batches of at most this many blocks: k_huff<.., 34>
#ifndef PBX_HUFF_SMALL_WAVES
#define PBX_HUFF_SMALL_WAVES 2  // k_huff<.., 34>'s waves: 2 = the distance tree on a second wave
#endif
constexpr uint32_t HUFF_SMALL_WAVES = PBX_HUFF_SMALL_WAVES;
constexpr uint32_t FRAME_WAVE_TILES = 256;  // batches of at most this many tiles: k_frame_wave
constexpr uint32_t LZ_SELF_MAP_SEGS = 2048;  // k_lz77 maps its segment in batches of at most this many

// One Huffman block = the BLK_SEGS (or fewer, at a tile's end) consecutive segments of
// one tile whose histograms it sums; one wave per block.
// LDSEG: segments whose histogram loads are in flight together.  Large batches take 17 (the
// registers of more would cut the kernel's occupancy, profiles/r05r/); a small batch (the
// single-request latency path: one block, one wave on the chip) loads up to 34 segments' at
// once, one round of loads instead of three for a 512x512 uint16 tile.
// NWV = 2 (small batches): a second wave builds the distance tree (merge rounds and depths)
// while the first builds the literal/length tree; everything else is the first wave's, with
// wave-level LDS syncs instead of workgroup barriers.
template <class C, bool PROF, uint32_t LDSEG = HUFF_LDSEG, uint32_t NWV = 1>
// solo (a batch of one tile in one block, the single-request path): the block also writes the
// tile's output offsets (and their mapped copy), so no k_sizes_scan launch follows.
__global__ __launch_bounds__(64 * NWV) void k_huff(uint32_t nblk, BlkInfo* __restrict__ blk,
                                             SegInfo* __restrict__ info,
                                             const uint32_t* __restrict__ hist,
                                             uint32_t* __restrict__ codes,
                                             uint64_t* __restrict__ stamps,
                                             const TileDesc* __restrict__ solo = nullptr,
                                             uint64_t* __restrict__ offs = nullptr,
                                             uint64_t* __restrict__ offs_host = nullptr,
                                             uint32_t solo_nseg = 0) {
    __shared__ HuffSmem<C> S;
    const uint32_t tid = threadIdx.x & 63;  // the lane (the code below is one wave's)
    const uint32_t wv = NWV > 1 ? __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0u;
    const bool w0 = wv == 0;
    // a sync among the lanes doing a phase: the workgroup's barrier when it is one wave
    auto bar = [&]() { huff_sync<(NWV > 1)>(); };
    const uint32_t b = xcd_remap(blockIdx.x, gridDim.x);
    // (solo: the block is the tile's segments 0..nseg-1, known at launch -- no dependent load of
    // its record before the histogram loads)
    const uint32_t seg0 = solo_nseg ? 0u : blk[b].seg0, nsg = solo_nseg ? solo_nseg : blk[b].nseg;
    uint32_t nst = 0;
    auto stamp = [&]() {
        if (PROF && threadIdx.x == 0) stamps[(size_t)seg0 * STAMP_STRIDE + 8 + nst] = __builtin_amdgcn_s_memtime();
        nst++;
    };
    stamp();
    // the segments' histograms summed (read again, L2-hot, for their bit counts at the end;
    // the small-batch variant keeps its first round in registers for that instead: one wave
    // on the CU has the registers, and a lone block waits on every load round)
    constexpr bool KEEP = LDSEG > 24;
    uint32_t hr0[KEEP ? LDSEG : 1][5];
    uint32_t hs[5] = {0, 0, 0, 0, 0};
    uint32_t sl = 0, last = 0;
    // the solo tile's container fields, for its output size at the end (loaded now: a lone
    // block would otherwise wait on one more load round there)
    uint32_t solo_flags = 0, solo_hdr = 0;
    if (solo) {
        solo_flags = solo->flags;
        solo_hdr = solo->tiff_hdr;
    }
    if (w0) {  // (NWV = 2: the second wave waits at the barrier after the sort)
    // the segments' lengths (lane k: segment k) and the last one's flag, issued with the
    // histogram loads (one round trip for all of them)
    const uint32_t my_sl = tid < nsg ? info[seg0 + tid].sl : 0u;
    last = info[seg0 + nsg - 1].last;
    for (uint32_t k0 = 0; k0 < nsg; k0 += LDSEG) {  // LDSEG segments' loads in flight
        uint32_t hr[LDSEG][5];
#pragma unroll
        for (uint32_t k = 0; k < LDSEG; k++)
#pragma unroll
            for (int j = 0; j < 5; j++)
                hr[k][j] = k0 + k < nsg ? hist[(size_t)(seg0 + k0 + k) * HIST_WORDS + tid + 64 * j] : 0u;
#pragma unroll
        for (uint32_t k = 0; k < LDSEG; k++)
#pragma unroll
            for (int j = 0; j < 5; j++) hs[j] += hr[k][j];
        if (KEEP && k0 == 0) {
#pragma unroll
            for (uint32_t k = 0; k < (KEEP ? LDSEG : 1); k++)
#pragma unroll
                for (int j = 0; j < 5; j++) hr0[k][j] = hr[k][j];
        }
    }
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t i = tid + 64 * j;
        const uint32_t v = i == 256 ? 1u : hs[j];  // one end of block (every segment counted one)
        if (i < 288) S.lfreq[i] = v; else S.dfreq[i - 288] = v;
    }
    if (tid < nsg) S.sls[tid] = my_sl;
    sl = wave_sum(my_sl);
    ph_huff_init<C>(tid, S);
    bar();
    ph_keys<C, DevOps>(tid, S);
    bar();
    stamp();
    sort512_wave(S.hs.skey, tid);
    }
    __syncthreads();
    stamp();
    if (NWV > 1) {
        huff_rounds_wave<true>(S, wv, tid);  // wave T builds tree T
    } else {
        huff_rounds_wave(S, 0, tid);
        huff_rounds_wave(S, 1, tid);
    }
    __syncthreads();
    stamp();
    if (w0) parents_wave(S, tid);
    __syncthreads();
    stamp();
    if (NWV > 1) {
        depths_wave<true>(S, wv, tid);
        __syncthreads();
        if (!w0) return;  // the rest is the first wave's (no workgroup barrier follows)
    } else {
        depths_wave(S, 0, tid);
        depths_wave(S, 1, tid);
    }
    stamp();
    ph_leafdepth<C, DevOps>(tid, S);
    bar();
    stamp();
    ph_fixblc<C>(tid, S);
    bar();
    stamp();
    assign_wave(S, tid);
    bar();
    ph_rle_init<C>(tid, S);
    bar();
    stamp();
#ifndef PBX_HUFF_RLE_WAVE
#define PBX_HUFF_RLE_WAVE 1  // 1: rle_wave (five ballots); 0: the generic phases of deflate_seg.h (the emulator's); 2: rle_wave in the batch variant only
#endif
    if (PBX_HUFF_RLE_WAVE == 1 || (PBX_HUFF_RLE_WAVE == 2 && !KEEP)) {
        rle_wave(S, tid);
        bar();
        stamp();
    } else {
        ph_rle_mark<C, DevOps>(tid, S);
        bar();
        ph_rle_count<C>(tid, S);
        bar();
        {
            const uint32_t nr = wave_scan_excl_add<RLEN>(S.rcnt, tid);
            if (tid == 0) S.misc[M_NRLE] = nr;
        }
        bar();
        stamp();
        ph_rle_emit<C, DevOps>(tid, S);
    }
    bar();
    stamp();
    clen_wave<(NWV > 1)>(S, tid);
    bar();
    stamp();
    ph_rle_bits<C>(tid, S);
    bar();
    {
        const uint32_t hb = wave_scan_excl_add<RLEN>(S.rboff, tid);
        if (tid == 0) S.misc[M_HDRBITS] = hb;
    }
    bar();
    ph_choose<C>(tid, S, sl, last, nsg);
    bar();
    stamp();
    ph_codes<C>(tid, S);
    ph_header<C, DevOps>(tid, S, last);
    bar();
    stamp();
    uint32_t* cg = codes + (size_t)b * CODE_WORDS;
    for (uint32_t i = tid; i < CODE_WORDS; i += 64)
        cg[i] = i < 288 ? S.lcode[i] : i < 320 ? S.dcode[i - 288] : S.hdrw[i - 320];
    // every segment's bit range in the block: [header] tokens of segment 0, 1, ... [EOB]
    // [empty stored block unless the tile ends here]; a stored block is byte-aligned
    // the segments' token bits under the block's code (wave-uniform), into LDS: the
    // per-symbol cost (code length + extra bits) of this lane's 5 symbols, then one dot
    // product per segment with its histogram
    uint32_t cost[5];
#pragma unroll
    for (int j = 0; j < 5; j++) {
        const uint32_t i = tid + 64 * j;
        const bool skip = i == 256 || (i >= 286 && i < 288) || i >= 318;
        const uint32_t L = (i < 288 ? S.lcode[i] : S.dcode[i < 320 ? i - 288 : 0]) >> 16;
        const uint32_t eb = i < 288 ? (i > 256 ? len_sym_ebits(i) : 0u) : dist_sym_ebits(i < 318 ? i - 288 : 0);
        cost[j] = skip ? 0u : L + eb;
    }
#ifndef PBX_HUFF_ONEREAD
#define PBX_HUFF_ONEREAD 0  // timing bound only (variant build): no second histogram read, wrong output
#endif
#ifndef PBX_HUFF_LANE_SUMS
#define PBX_HUFF_LANE_SUMS 1  // 1: the segments' dot products summed by one transposing butterfly (lane k: segment k); 0: a wave_sum each
#endif
    uint32_t dkl = 0;  // lane k: segment k's token bits
    for (uint32_t k0 = 0; k0 < nsg; k0 += LDSEG) {
        uint32_t hr[LDSEG][5];
#pragma unroll
        for (uint32_t k = 0; k < LDSEG; k++)
#pragma unroll
            for (int j = 0; j < 5; j++)
                hr[k][j] = KEEP && k0 == 0 ? hr0[KEEP ? k : 0][j]
                           : k0 + k < nsg && !PBX_HUFF_ONEREAD ? hist[(size_t)(seg0 + k0 + k) * HIST_WORDS + tid + 64 * j] : 0u;
        uint32_t dv[LDSEG];
#pragma unroll
        for (uint32_t k = 0; k < LDSEG; k++) {
            uint32_t d = 0;
#pragma unroll
            for (int j = 0; j < 5; j++) d += cost[j] * hr[k][j];
            dv[k] = d;
        }
        if (PBX_HUFF_LANE_SUMS) {
            uint32_t t = wave_sums_to_lanes(dv, tid);  // lane k: segment k0 + k (k < LDSEG)
            if (k0) {  // to lane k0 + k
                t = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((tid - k0) & 63u) << 2), (int)t);
                t = tid >= k0 && tid < k0 + LDSEG ? t : 0u;
            }
            dkl += t;
        } else {
#pragma unroll
            for (uint32_t k = 0; k < LDSEG; k++) {
                const uint32_t d = wave_sum(dv[k]);
                if (tid == 0 && k0 + k < nsg) S.dk[k0 + k] = d;
            }
        }
    }
    bar();
    if (!PBX_HUFF_LANE_SUMS) dkl = tid < nsg ? S.dk[tid] : 0u;
    // a segment's share of a Huffman-coded block must fit k_encode's output buffer
    // (deflate_seg.h seg_share_fits); else the block is stored
    uint32_t bt = S.misc[M_BTYPE], hdr = S.misc[M_HDRBITS], nbytes = S.misc[M_NBYTES];
    uint32_t dbits = S.misc[M_DATABITS];
    // (deflate_seg.h seg_shares_fit: lane k checks segment k's share, bit offsets by a scan)
    bool fits;
    {
        static_assert(BLK_SEGS <= 64, "one lane per segment of a block");
        const uint32_t incl = wave_incl_scan_dpp(dkl);
        const uint64_t run1 = (uint64_t)hdr + incl, run0 = run1 - dkl;
        const uint64_t b0 = tid == 0 ? 0 : run0;
        const uint64_t b1 = tid + 1 < nsg ? run1 : last ? run1 + (S.lcode[256] >> 16) : 8ull * nbytes;
        fits = __builtin_amdgcn_ballot_w64(tid < nsg && b1 - b0 > 8ull * (uint64_t)C::SEG) == 0;
    }
    if (bt != 0 && !fits) {
        bt = 0; hdr = 0; dbits = 0;
        nbytes = block_nbytes(0, 0, sl, last, nsg);
    }
    // stored: every segment is its own stored block (5-byte header + its bytes).  Lane k
    // writes segment k's bit range [bit0, bit1): the bits before it by a wave scan.
    static_assert(BLK_SEGS <= 64, "one lane per segment of a block");
    {
        const uint32_t k = tid;
        const uint32_t d = k < nsg ? (bt == 0 ? 8 * (5 + S.sls[k]) : dkl) : 0u;
        const uint32_t st = (bt == 0 ? 0u : hdr) + wave_incl_scan_dpp(d) - d;  // run before segment k
        if (k < nsg) {
            SegInfo& g = info[seg0 + k];
            g.btype = bt;
            g.hdr_bits = hdr;
            g.bit0 = k == 0 ? 0u : st;
            const uint32_t e = st + d;
            g.bit1 = k + 1 < nsg ? e : last ? (bt == 0 ? 8 * nbytes : e + (S.lcode[256] >> 16)) : 8 * nbytes;
        }
    }
    if (tid == 0) {
        blk[b].nbytes = nbytes;
        blk[b].data_bits = dbits;
        blk[b].fin = last;
        if (solo) {
            blk[b].pad[0] = 0;  // k_encode's count of finished workgroups (the last frames the tile)
            TileDesc sd{};
            sd.flags = solo_flags;
            sd.tiff_hdr = solo_hdr;
            const uint64_t sz = container_bytes(sd, nbytes);
            blk[b].off = 0;
            offs[0] = 0;
            offs[1] = sz;
            if (offs_host) {
                offs_host[0] = 0;
                offs_host[1] = sz;
            }
        }
    }
    stamp();
}

// ================================================================= k_seg_map
// Per tile (one thread): the tile of every segment, so the per-segment kernels find their
// tile descriptor with one load, and the tile's Huffman blocks.
// One thread per segment (one per tile left 4096 tiles on 16 workgroups: 23 us): its tile by
// the batch's reciprocal when every tile has the same segment count, else a binary search;
// its Huffman block by inverting block_seg0 (j = ((k + 1) nb - 1) / n, checked for every
// n <= 300); the block's first segment writes the block record.
__global__ __launch_bounds__(256) void k_seg_map(const TileDesc* __restrict__ dt, uint32_t ndt, uint32_t nseg,
                                                 uint32_t uniform_nseg, uint32_t uniform_rcp,
                                                 uint32_t* __restrict__ seg_tile,
                                                 SegInfo* __restrict__ info, BlkInfo* __restrict__ blk) {
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= nseg) return;
    const uint32_t i = uniform_nseg ? div_rcp(g, uniform_nseg, uniform_rcp)
                                    : upper_index(ndt, g, [&](uint32_t t) { return dt[t].seg_first; });
    seg_tile[g] = i;
    seg_map_one(dt[i], i, g, info, blk);
}

// ================================================================ k_seg_sizes

__global__ __launch_bounds__(256) void k_seg_sizes(const TileDesc* __restrict__ dt, uint32_t ndt,
                                                   BlkInfo* __restrict__ blk,
                                                   uint64_t* __restrict__ sizes) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= ndt) return;
    const TileDesc& d = dt[i];
    uint32_t off = 0;
    const uint32_t nb = tile_blocks(d.seg_count, PBX_TILE_BLK_CAP(d));
    for (uint32_t k = 0; k < nb; k++) {
        BlkInfo& g = blk[d.hblk_first + k];
        g.off = off;
        off += g.nbytes;
    }
    sizes[i] = container_bytes(d, off);
}

// A batch of at most 1024 tiles: k_seg_sizes and k_scan_offsets in one launch (thread t
// sizes tile t).  offs_host (or nullptr): a copy of the offsets in mapped pinned memory, so
// the serving path reads them without a D2H copy at the end of the launch.
__global__ __launch_bounds__(1024) void k_sizes_scan(const TileDesc* __restrict__ dt, uint32_t ndt,
                                                     BlkInfo* __restrict__ blk, uint64_t* __restrict__ offs,
                                                     uint64_t* __restrict__ offs_host) {
    __shared__ uint64_t part[1024];
    const uint32_t tid = threadIdx.x;
    uint64_t s = 0;
    if (tid < ndt) {
        const TileDesc& d = dt[tid];
        uint32_t off = 0;
        const uint32_t nb = tile_blocks(d.seg_count, PBX_TILE_BLK_CAP(d));
        for (uint32_t k = 0; k < nb; k++) {
            BlkInfo& g = blk[d.hblk_first + k];
            g.off = off;
            off += g.nbytes;
        }
        s = container_bytes(d, off);
    }
    part[tid] = s;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        const uint64_t v = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    if (tid < ndt) {
        offs[tid] = part[tid] - s;
        if (offs_host) offs_host[tid] = part[tid] - s;
    }
    if (tid == 1023) {
        offs[ndt] = part[1023];
        if (offs_host) offs_host[ndt] = part[1023];
    }
}

__global__ __launch_bounds__(1024) void k_scan_offsets(const uint64_t* __restrict__ sizes, uint32_t n,
                                                       uint64_t* __restrict__ offs, uint64_t* __restrict__ offs_host) {
    __shared__ uint64_t part[1024];
    const uint32_t tid = threadIdx.x;
    const uint32_t per = (n + 1023) / 1024;
    const uint32_t b = tid * per, e = b + per < n ? b + per : n;
    uint64_t s = 0;
    for (uint32_t i = b; i < e; i++) s += sizes[i];
    part[tid] = s;
    __syncthreads();
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint64_t v = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    uint64_t run = part[tid] - s;
    for (uint32_t i = b; i < e; i++) {
        offs[i] = run;
        if (offs_host) offs_host[i] = run;
        run += sizes[i];
    }
    if (tid == 1023) {
        offs[n] = part[1023];
        if (offs_host) offs_host[n] = part[1023];
    }
}

// ==================================================================== k_encode
// Output bytes j..j+3 (j = any byte offset) from the assembled words.
template <class SM>
__device__ __forceinline__ uint32_t out_word(const SM& S, uint32_t j) {
    const uint32_t w0 = S.out[j >> 2], w1 = S.out[(j >> 2) + 1], sh = (j & 3) * 8;
    return sh ? (w0 >> sh) | (w1 << (32 - sh)) : w0;
}
template <class SM>
__device__ __forceinline__ uint32_t out_byte_at(const SM& S, uint32_t j) {
    return (S.out[j >> 2] >> ((j & 3) * 8)) & 0xFFu;
}
template <class SM>
__device__ __forceinline__ uint8_t* out_byte_ptr(SM& S, uint32_t j) {
    return (uint8_t*)&S.out[j >> 2] + (j & 3);
}

// Bit writers over the LDS output words (deflate_seg.h RunWriter / BitWriter semantics:
// every word is OR'd into a zeroed buffer, so words shared with the neighbouring bit ranges
// need no special case).  (A branch-free put -- OR zero when no word completes -- measured
// slower: on compressible data many lanes then OR into the same few words.)
struct LdsRunWriter {
    uint32_t* out;
    uint32_t word, nacc;
    uint64_t acc;
    __device__ LdsRunWriter(uint32_t* o, uint32_t pos) : out(o), word(pos >> 5), nacc(pos & 31), acc(0) {}
    __device__ __forceinline__ void put(uint32_t v, uint32_t n) {
        acc |= (uint64_t)v << nacc;
        nacc += n;
        if (nacc >= 32) {
            atomicOr(&out[word], (uint32_t)acc);
            word++;
            acc >>= 32;
            nacc -= 32;
        }
    }
    __device__ __forceinline__ void finish() {
        if (acc) atomicOr(&out[word], (uint32_t)acc);
    }
};
struct LdsBitWriter {
    uint32_t* out;
    uint32_t pos;
    __device__ void put(uint32_t v, uint32_t n) {
        if (!n) return;
        const uint32_t w = pos >> 5, sh = pos & 31;
        atomicOr(&out[w], v << sh);
        if (sh + n > 32) atomicOr(&out[w + 1], v >> (32 - sh));
        pos += n;
    }
};

// Slicing-by-4 CRC step over one little-endian word.
// Slicing-by-8 CRC step over two little-endian words: the second word's four lookups do not
// depend on the running CRC, so a chain of 8 bytes is one round of dependent LDS reads, not two.
template <class SM>
__device__ __forceinline__ uint32_t crc_word2(const SM& S, uint32_t c, uint32_t v0, uint32_t v1) {
    static_assert(sizeof(S.crc_t) / sizeof(S.crc_t[0]) == 8, "slicing-by-8 tables");
    c ^= v0;
    return (S.crc_t[7][c & 0xFF] ^ S.crc_t[6][(c >> 8) & 0xFF] ^ S.crc_t[5][(c >> 16) & 0xFF] ^ S.crc_t[4][c >> 24]) ^
           (S.crc_t[3][v1 & 0xFF] ^ S.crc_t[2][(v1 >> 8) & 0xFF] ^ S.crc_t[1][(v1 >> 16) & 0xFF] ^ S.crc_t[0][v1 >> 24]);
}
template <class SM>
__device__ __forceinline__ uint32_t crc_word(const SM& S, uint32_t c, uint32_t v) {
    c ^= v;
    return S.crc_t[3][c & 0xFF] ^ S.crc_t[2][(c >> 8) & 0xFF] ^ S.crc_t[1][(c >> 16) & 0xFF] ^
           S.crc_t[0][c >> 24];
}

// ph_crc (deflate_seg.h) over out[0, 4 nv) with nv a multiple of 8 words: the segment's
// bytes sit after P leading zero bytes (P = -bytes mod 32), so every thread's right-aligned
// 32-byte chunk starts on a 32-byte boundary and is two 16-byte LDS reads (no realignment,
// no stride-8 word reads).  Byte zb (the head byte shared with the previous segment, or
// ~0u) reads as zero.
template <class C, class SM>
__device__ __forceinline__ uint32_t crc_chunk_aligned(uint32_t tid, const SM& S, uint32_t nv, uint32_t zb) {
    const int32_t hi = (int32_t)nv - (int32_t)(C::NT - 1 - tid) * (C::CRCC / 4);
    uint32_t c = 0;
    auto step = [&](uint32_t k) {  // words k..k+3
        const uint4 q = *(const uint4*)&S.out[k];
        uint32_t v[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (uint32_t j = 0; j < 4; j++)
            if (k + j == (zb >> 2)) v[j] &= ~(0xFFu << (8 * (zb & 3)));
#if PBX_CRC_SLICES == 8
        c = crc_word2(S, c, v[0], v[1]);
        c = crc_word2(S, c, v[2], v[3]);
#else
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) c = crc_word(S, c, v[j]);
#endif
    };
    if (tid == 0) {
        for (int32_t k = 0; k < hi; k += 4) step((uint32_t)k);  // its chunk and everything before
    } else if (hi >= (int32_t)(C::CRCC / 4)) {
        step((uint32_t)hi - 8);
        step((uint32_t)hi - 4);
    }
    return c;
}

// Timing experiments only (scripts/variants.sh): skip parts of k_encode (wrong output).
#ifndef PBX_ENC_SKIP_WRITE
#define PBX_ENC_SKIP_WRITE 0
#endif
#ifndef PBX_ENC_SKIP_PATCH
#define PBX_ENC_SKIP_PATCH 0
#endif
#ifndef PBX_ENC_SKIP_CRC
#define PBX_ENC_SKIP_CRC 0
#endif
#ifndef PBX_ENC_LIT_BF
#define PBX_ENC_LIT_BF 0  // literal-only waves: branch-free word puts
#endif
#ifndef PBX_ENC_SKIP_STORE
#define PBX_ENC_SKIP_STORE 0
#endif

// A token's bits packed in one register: value (<= 20 bits) | nbits << 27.  The LDS code
// tables hold literal/length and distance codes in this form (slot 288 = 0 bits).
__device__ __forceinline__ uint32_t slot_from_code(uint32_t c) { return (c & 0xFFFFu) | ((c >> 16) << 27); }
constexpr uint32_t SLOT_NONE = 288;

// The thread's CH positions as register slots, in stream order: slot i holds the literal
// or length code (+ extra bits) of a token starting at chunk position i; a match also
// fills slots i+1 (distance code) and i+2 (distance extra bits), positions it covers.
// Same tokens as walk_tokens (deflate_seg.h) over the same match lists.  Literals first,
// branch-free: covered positions read the empty slot; then the (few) matches starting in
// the chunk overwrite their three slots.
// Returns true (wave-uniform) when the wave's slots are literals only (no match, full
// chunks): slots 32 and 33 are then empty and every slot holds <= 15 bits.
template <class C, class SM>
__device__ __forceinline__ bool build_slots(uint32_t tid, const SM& S, const SegParams& sp,
                                            const uint32_t (&cb)[C::CH / 4],
                                            uint32_t (&slot)[C::CH + 2], uint32_t carry) {
    const uint32_t cs = tid * C::CH;
    const uint32_t ce = cs + C::CH < sp.sl ? cs + C::CH : sp.sl;
    const uint32_t w = (cs / C::SUB) < (uint32_t)C::NW ? cs / C::SUB : (uint32_t)C::NW - 1;
    const uint32_t* mp = S.mpos + w * C::MAXMW;
    const auto* md = S.mdist + w * C::MAXMW;
    const uint32_t nm = S.w_nm[w];
    uint32_t lo = 0, hi = nm;  // first match starting at or after cs
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((mp[mid] & 0xFFFFu) < cs) lo = mid + 1; else hi = mid;
    }
    // covered = positions of the chunk inside a match or past the segment
    const uint32_t nval = ce > cs ? ce - cs : 0u;
    uint32_t covered = nval >= 32 ? 0u : (0xFFFFFFFFu << nval);
    auto cover = [&](uint32_t a, uint32_t b) {  // stream positions [a, b) of the chunk
        const uint32_t l = a > cs ? a - cs : 0u, h = b - cs < 32 ? b - cs : 32u;
        if (b > cs && l < 32) covered |= (h >= 32 ? 0xFFFFFFFFu : (1u << h) - 1u) & (0xFFFFFFFFu << l);
    };
    if (lo > 0) {
        cover(mp[lo - 1] & 0xFFFFu, (mp[lo - 1] & 0xFFFFu) + (mp[lo - 1] >> 16) + 3);
    } else if (carry > cs) {  // the previous wave's last match runs into this chunk (walk_tokens)
        cover(cs, carry);
    }
    uint32_t m1 = lo;
    while (m1 < nm && (mp[m1] & 0xFFFFu) < ce) {
        cover(mp[m1] & 0xFFFFu, (mp[m1] & 0xFFFFu) + (mp[m1] >> 16) + 3);
        m1++;
    }
    // a wave without matches or partial chunks (most waves on noisy data): literals only
    if (__builtin_amdgcn_ballot_w64(lo < m1 || covered != 0) == 0) {
#pragma unroll
        for (int i = 0; i < C::CH; i++) slot[i] = S.lcode[(cb[i >> 2] >> ((i & 3) * 8)) & 0xFFu];
        slot[C::CH] = 0;
        slot[C::CH + 1] = 0;
        return true;
    }
    // the first match starting in the chunk goes in with the literals, branch-free; any
    // further ones (several short matches in 32 bytes) are patched in after
    uint32_t i0 = 0xFFu, A = 0, B = 0, Cx = 0;
    if (lo < m1) {
        const uint32_t len = (mp[lo] >> 16) + 3, dist = (uint32_t)md[lo] + 1;
        i0 = (mp[lo] & 0xFFFFu) - cs;
        uint32_t sy, e, v;
        len_code(len, sy, e, v);
        const uint32_t lc = S.lcode[sy];
        A = lc + (v << (lc >> 27)) + (e << 27);
        dist_code(dist, sy, e, v);
        B = S.dcode[sy];
        Cx = v | (e << 27);
    }
#pragma unroll
    for (int i = 0; i < C::CH + 2; i++) {
        uint32_t lit = 0;
        if (i < C::CH) {
            const uint32_t b = (cb[i >> 2] >> ((i & 3) * 8)) & 0xFFu;
            lit = S.lcode[((covered >> i) & 1u) ? SLOT_NONE : b];
        }
        // masks, not ?: chains: the compiler turns those into branches around the lookup
        const uint32_t di = (uint32_t)i - i0;
        const uint32_t k0 = 0u - (uint32_t)(di == 0), k1 = 0u - (uint32_t)(di == 1), k2 = 0u - (uint32_t)(di == 2);
        slot[i] = (lit & ~(k0 | k1 | k2)) | (A & k0) | (B & k1) | (Cx & k2);
    }
    for (uint32_t m = lo + 1; m < (PBX_ENC_SKIP_PATCH ? lo : m1); m++) {
        const uint32_t i = (mp[m] & 0xFFFFu) - cs, len = (mp[m] >> 16) + 3, dist = (uint32_t)md[m] + 1;
        uint32_t sy, e, v;
        len_code(len, sy, e, v);
        const uint32_t lc = S.lcode[sy];
        const uint32_t A = lc + (v << (lc >> 27)) + (e << 27);
        dist_code(dist, sy, e, v);
        const uint32_t B = S.dcode[sy], Cx = v | (e << 27);
#pragma unroll
        for (int j = 0; j < C::CH + 2; j++) {
            const uint32_t dj = (uint32_t)j - i;
            slot[j] = dj == 0 ? A : dj == 1 ? B : dj == 2 ? Cx : slot[j];
        }
    }
    return false;
}

// One segment's part of its block: the header (first segment), its tokens, and the end of
// block (+ the empty stored block of a non-final block; last segment) at the bits
// [bit0, bit1) k_huff assigned.  The bytes it owns entirely go straight to the compacted
// output; a byte it shares with the previous / next segment of the block (bit0 or bit1 not
// on a byte boundary) is left to k_frame (SegInfo.part), which ORs the two halves.
//
// Four barriers: (1) inputs in LDS and the output words zeroed (the block header already
// in them), (2) the bit offsets scanned, (3) every token written, (4) the waves' CRCs.
// Everything the segment needs is loaded up front in two dependent rounds (the record and
// the match counts, then the bytes, matches and codes); the CRC tables, needed last, are
// loaded while the slots are built.  The segment's bytes go P = -bytes mod 32 bytes into
// out[], so the CRC chunks are 32-byte aligned.
// k_frame_wave's work for one tile on one wave (below); the single-request path runs it at
// the end of k_encode, in the workgroup that finishes last
template <bool LR>
__device__ void frame_wave_tile(const TileDesc& d, uint8_t* __restrict__ base, const SegInfo* __restrict__ info,
                                const BlkInfo* __restrict__ blk, uint32_t lane);

// FRAME (the single-tile batch only: its own instantiation, so the framing code's registers
// never reach the batch kernel's allocation): the last workgroup frames the tile
template <class C, bool PROF, bool FRAME = false>
__global__ __launch_bounds__(C::NT, 8) void k_encode(const TileDesc* __restrict__ dt,
                                                  const uint32_t* __restrict__ seg_tile,
                                                  uint32_t nseg, const uint8_t* __restrict__ stream,
                                                  SegInfo* __restrict__ info,
                                                  const BlkInfo* __restrict__ blk,
                                                  const uint32_t* __restrict__ mrec,
                                                  const uint32_t* __restrict__ codes,
                                                  const uint64_t* __restrict__ offs,
                                                  uint8_t* __restrict__ out,
                                                  uint64_t* __restrict__ stamps,
                                                  uint32_t uniform_nseg, uint32_t uniform_rcp,
                                                  uint32_t* __restrict__ frame_ctr = nullptr) {
    static_assert(C::CH == 32 && C::CRCC == 32, "two 16-byte loads per thread chunk");
    static_assert(C::SUB == 64 * C::CH && C::NW * C::SUB <= 4 * C::OUTW, "a wave's bytes staged in its part of out[]");
    __shared__ EncSmem<C> S;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t seg = xcd_remap(blockIdx.x, gridDim.x);
    uint32_t nst = 0;
    auto stamp = [&]() {
        if (PROF && tid == 0) stamps[(size_t)seg * STAMP_STRIDE + 24 + nst] = __builtin_amdgcn_s_memtime();
        nst++;
    };
    stamp();
    // round 1: the segment record and this wave's match count (scalar loads, issued together:
    // the empty asm uses make the compiler wait for all of them at one point)
    const uint32_t* mg = mrec + (size_t)seg * MREC_WORDS;
    SegInfo gi;  // everything the encoder needs about its segment / tile
    uint32_t nmw, nmp;
    {
        nmw = mg[w];
        nmp = w ? mg[w - 1] : 0u;  // the previous wave's matches: its last may run into this wave
        static_assert(sizeof(SegInfo) == 80, "five 16-byte words");
        const uint4* src = (const uint4*)&info[seg];
        const uint4 g0 = src[0], g1 = src[1], g2 = src[2], g3 = src[3], g4 = src[4];
        asm volatile("" ::"s"(g0.x), "s"(g0.y), "s"(g0.z), "s"(g0.w), "s"(g1.x), "s"(g1.y), "s"(g1.z),
                     "s"(g1.w), "s"(g2.x), "s"(g2.y), "s"(g2.z), "s"(g2.w), "s"(g3.x), "s"(g3.y),
                     "s"(g3.z), "s"(g3.w), "s"(g4.x), "s"(g4.y), "s"(g4.z), "s"(g4.w));
        __builtin_memcpy((uint4*)&gi, &g0, 16);
        __builtin_memcpy((uint4*)&gi + 1, &g1, 16);
        __builtin_memcpy((uint4*)&gi + 2, &g2, 16);
        __builtin_memcpy((uint4*)&gi + 3, &g3, 16);
        __builtin_memcpy((uint4*)&gi + 4, &g4, 16);
    }
    // the tile (its plane rows, PBX_ENC_FROM_PLANE): in round 1 too when every tile has the
    // same number of segments
    const TileDesc d = PBX_ENC_FROM_PLANE
                           ? load_desc(dt + (uniform_nseg ? div_rcp(seg, uniform_nseg, uniform_rcp) : gi.tile))
                           : TileDesc{};
    const uint32_t ti = gi.tile;
    SegParams sp;  // the encoder holds the segment only (no window)
    sp.base = 0;
    sp.wl = 0;
    sp.sl = gi.sl;
    sp.last = gi.last;
    sp.rowlen = gi.rowlen;
    const uint64_t seg_off = ((uint64_t)gi.src_hi << 32) | gi.src_lo;
    const bool first = (gi.flags & SF_FIRST) != 0, lastb = (gi.flags & SF_LAST) != 0;
    const bool final_seg = sp.last != 0;          // the tile's stream ends in this segment
    const bool stored = gi.btype == 0;
    const uint32_t byte0 = gi.bit0 >> 3, lb = gi.bit0 & 7u;  // block byte byte0 = out[] byte P
    const uint32_t le = gi.bit1 - 8 * byte0;      // end bit, relative to byte P
    // bytes owned: [o0, o1) after byte P; a partial first byte (lb != 0) and a partial last
    // byte of a non-final segment are shared with the neighbours (k_frame joins them)
    const uint32_t o0 = lb ? 1u : 0u;
    uint32_t o1 = final_seg ? (le + 7) >> 3 : le >> 3;
    if (o1 < o0) o1 = o0;
    const uint32_t P = (0u - o1) & 31u, SH = 8 * P;  // leading zero bytes: P + o1 = 0 mod 32
    // round 2: the thread's chunk bytes (zero past the segment: loads past it read the
    // segment start instead, no branch), the wave's matches, the block's codes and header
    uint32_t cb[C::CH / 4];
    DirectRows dr;
    dr.init(d);
    const uint32_t fmode = PBX_ENC_FROM_PLANE == 1 && PBX_LZ_FAST_FILL && (d.flags & TF_DIRECT) ? fast_fill_mode(dr) : 0u;
    const bool rmode = PBX_ENC_FROM_PLANE == 2 && PBX_LZ_FAST_FILL && (d.flags & TF_DIRECT) && fast_fill_mode(dr) == 5u;
    if (rmode) {
        // k_lz77 stored no bytes: the lane's 32 bytes from the plane rows, converted in registers
        const uint32_t cs = tid * C::CH;
        plane_words_swap16(dr, (uint32_t)(seg_off - d.out_off) + cs, cb);
#pragma unroll
        for (int k = 0; k < C::CH / 4; k++) {  // mask bytes past the segment end, branch-free
            const int32_t keep = (int32_t)sp.sl - (int32_t)(cs + 4 * k);
            const uint32_t kb = keep <= 0 ? 0u : keep >= 4 ? 32u : 8u * (uint32_t)keep;
            cb[k] &= (uint32_t)((1ull << kb) - 1ull);
        }
    } else if (fmode) {
        // k_lz77 stored no bytes: the wave converts its 2 KiB of the segment from the plane
        // rows into its part of out[] (fill_fast as one 64-thread group, zero past the
        // segment), each lane reads its 32 bytes back and zeroes them.  Wave-local: the LDS
        // operations of one wave complete in order.
        uint32_t* wbuf = S.out + w * (C::SUB / 4);
        const uint32_t wb = w * C::SUB;
        if (wb < sp.sl) {
            const uint32_t nbw = sp.sl - wb < (uint32_t)C::SUB ? sp.sl - wb : (uint32_t)C::SUB;
            const uint32_t B = (uint32_t)(seg_off - d.out_off) + wb;  // tile stream offset
            const uint32_t ra = div_rcp(B, dr.rowlen, dr.rcp), rz = div_rcp(B + nbw - 1, dr.rowlen, dr.rcp);
            fill_fast_mode<64>(fmode, wbuf, dr, B, nbw, C::SUB, lane, ra, rz, nullptr, 0);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint4 q0 = *(const uint4*)&wbuf[8 * lane], q1 = *(const uint4*)&wbuf[8 * lane + 4];
            cb[0] = q0.x; cb[1] = q0.y; cb[2] = q0.z; cb[3] = q0.w;
            cb[4] = q1.x; cb[5] = q1.y; cb[6] = q1.z; cb[7] = q1.w;
        } else {
#pragma unroll
            for (int k = 0; k < C::CH / 4; k++) cb[k] = 0;
        }
        *(uint4*)&wbuf[8 * lane] = make_uint4(0, 0, 0, 0);
        *(uint4*)&wbuf[8 * lane + 4] = make_uint4(0, 0, 0, 0);
    } else {
        const uint32_t cs = tid * C::CH;
        const uint8_t* p0 = stream + seg_off + (cs < sp.sl ? cs : 0u);
        const uint8_t* p1 = stream + seg_off + (cs + 16 < sp.sl ? cs + 16 : 0u);
        const uint4 q0 = (PBX_NT_STREAM & 2) ? gload16_nt(p0) : *(const uint4*)p0;
        const uint4 q1 = (PBX_NT_STREAM & 2) ? gload16_nt(p1) : *(const uint4*)p1;
        cb[0] = q0.x; cb[1] = q0.y; cb[2] = q0.z; cb[3] = q0.w;
        cb[4] = q1.x; cb[5] = q1.y; cb[6] = q1.z; cb[7] = q1.w;
#ifndef PBX_ENC_MASK_TAIL
#define PBX_ENC_MASK_TAIL 1  // mask only in the chunks the segment ends in or past (0: every chunk)
#endif
        if (!PBX_ENC_MASK_TAIL || cs + C::CH > sp.sl) {  // (full waves skip it: ~50 VALU a lane)
#pragma unroll
            for (int k = 0; k < C::CH / 4; k++) {  // mask bytes past the segment end
                const int32_t keep = (int32_t)sp.sl - (int32_t)(cs + 4 * k);
                const uint32_t kb = keep <= 0 ? 0u : keep >= 4 ? 32u : 8u * (uint32_t)keep;
                cb[k] &= (uint32_t)((1ull << kb) - 1ull);
            }
        }
    }
    const BlkInfo bi = blk[gi.blk];       // scalar loads, needed at the end
    const uint64_t tile_off = offs[ti];
    const uint32_t* cg = codes + (size_t)gi.blk * CODE_WORDS;
    const uint32_t craw = cg[tid < 320 ? tid : 319u];  // unconditional: no branch, no early wait
    // the block header (first segment of a Huffman block): word tid, OR-ed in at bit SH + 32 tid
    const bool hdr = first && !stored;
    const uint32_t hraw = cg[320 + (tid < (uint32_t)C::HDRW ? tid : (uint32_t)C::HDRW - 1)];
    if (__builtin_amdgcn_readfirstlane(nmw) != 0) {  // uniform: most waves on noise keep no match
        static_assert(C::MAXMW == 256, "four match slots per lane");
        const uint32_t* gp = mg + C::NW + w * C::MAXMW;
        const uint32_t* gd = mg + C::NW + C::NW * C::MAXMW + w * C::MAXMW;
        uint32_t vp[4], vd[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            const uint32_t m = lane + 64 * j;
            vp[j] = m < nmw ? gp[m] : 0u;
            vd[j] = m < nmw ? gd[m] : 0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            const uint32_t m = lane + 64 * j;
            if (m < nmw) {
                S.mpos[w * C::MAXMW + m] = vp[j];
                S.mdist[w * C::MAXMW + m] = (uint16_t)vd[j];
            }
        }
    }
    if (lane == 0) S.w_nm[w] = nmw;
    if (tid < 288) S.lcode[tid] = slot_from_code(craw); else if (tid < 320) S.dcode[tid - 288] = slot_from_code(craw);
    if (tid == 0) {
        S.lcode[SLOT_NONE] = 0;
        S.crc_acc = 0;
        S.ndone = 0;
    }
    {   // zero the output words (with the bytes from the plane: past the waves' staging parts)
        uint4* o4 = (uint4*)S.out;
        const uint32_t k0 = fmode ? (uint32_t)(C::NW * C::SUB / 16) : 0u;
        for (uint32_t k = k0 + tid; k < (uint32_t)(sizeof(S.out) / 16); k += C::NT) o4[k] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    stamp();  // diagnostics: inputs in LDS
    uint32_t slot[C::CH + 2];
    uint32_t nbits = 0;
    bool lit_only = false;
    if (!stored) {
        // where the previous wave's last match ends when it runs into this wave (carry_end):
        // scalar loads of its last record, only when it kept matches (noise: almost never)
        uint32_t carry = 0;
        if (nmp) {
            const uint32_t r = mg[C::NW + (w - 1) * C::MAXMW + nmp - 1];
            const uint32_t e = (r & 0xFFFFu) + (r >> 16) + 3;
            carry = e > w * (uint32_t)C::SUB ? e : 0u;
        }
        lit_only = build_slots<C>(tid, S, sp, cb, slot, carry);
#pragma unroll
        for (int i = 0; i < C::CH + 2; i++) nbits = dot4_u8(slot[i], 0x01000000u, nbits);
        // (a slot's value is < 2^24, so its top byte is 8 x its bit count: one v_dot4 each)
        nbits >>= 3;
    }
    // the slicing tables (needed after barrier 3): loaded now, stored before barrier 2
    if (tid < 64 * PBX_CRC_SLICES) ((uint4*)&S.crc_t[0][0])[tid] = ((const uint4*)&kCrcTables.t[0][0])[tid];
    if (PROF) {  // diagnostics: slots built (wave 0)
        __builtin_amdgcn_s_waitcnt(0);
        stamp();
    }
    // exclusive scan of the token bits over the workgroup (one barrier)
    const uint32_t inc = wave_incl_scan_dpp(nbits);
    if (lane == 63) S.wtot[w] = inc;
    __syncthreads();
    stamp();
    uint32_t pre = 0, bitsum = 0;
#pragma unroll
    for (int i = 0; i < C::NW; i++) {
        const uint32_t x = S.wtot[i];
        pre += (uint32_t)i < w ? x : 0u;
        bitsum += x;
    }
    // the combine tables go where the match lists were (every wave is past build_slots)
    constexpr uint32_t NX4 = CRCX_WORDS / 4;
    static_assert(NX4 <= 2 * (uint32_t)C::NT, "two 16-byte table loads per thread");
    const uint4 tx0 = ((const uint4*)kCrcLane.t)[tid];
    const uint4 tx1 = ((const uint4*)kCrcLane.t)[tid + C::NT < NX4 ? tid + C::NT : tid];
    if (stored) {  // the segment's own stored block: BFINAL/BTYPE byte, LEN, NLEN, the bytes
        const uint32_t cs = tid * C::CH, o = P + 5u;
#pragma unroll
        for (uint32_t i = 0; i < (uint32_t)C::CH; i++)
            if (cs + i < sp.sl) *out_byte_ptr(S, o + cs + i) = (uint8_t)(cb[i >> 2] >> ((i & 3) * 8));
        if (tid == 0) {
            const uint32_t len = sp.sl;
            *out_byte_ptr(S, P) = (uint8_t)(final_seg ? 1 : 0);
            *out_byte_ptr(S, P + 1) = (uint8_t)len; *out_byte_ptr(S, P + 2) = (uint8_t)(len >> 8);
            *out_byte_ptr(S, P + 3) = (uint8_t)~len; *out_byte_ptr(S, P + 4) = (uint8_t)(~len >> 8);
        }
    } else if (!PBX_ENC_SKIP_WRITE) {
        if (hdr && tid < (uint32_t)C::HDRW && hraw) {  // header word tid at bit SH + 32 tid
            const uint32_t q = (SH >> 5) + tid, r = SH & 31;
            atomicOr(&S.out[q], hraw << r);
            if (r) atomicOr(&S.out[q + 1], hraw >> (32 - r));
        }
        const uint32_t tb = SH + lb + (first ? gi.hdr_bits : 0u);  // first token bit in out[]
        LdsRunWriter bw(S.out, tb + pre + inc - nbits);
        if (lit_only && PBX_ENC_LIT_BF) {
            // literal codes in pairs (<= 30 bits: at most one word completes per pair), no
            // branch: a pair that completes no word ORs zero into the current one
#pragma unroll
            for (int i = 0; i < C::CH; i += 2) {
                const uint32_t n0 = slot[i] >> 27;
                bw.acc |= (uint64_t)((slot[i] & 0x7FFFFFFu) | ((slot[i + 1] & 0x7FFFFFFu) << n0)) << bw.nacc;
                bw.nacc += n0 + (slot[i + 1] >> 27);
                const uint32_t full = bw.nacc >= 32 ? 1u : 0u;
                atomicOr(&S.out[bw.word], full ? (uint32_t)bw.acc : 0u);
                bw.acc = full ? bw.acc >> 32 : bw.acc;
                bw.word += full;
                bw.nacc -= 32 * full;
            }
        } else if (lit_only) {  // literal codes (<= 15 bits) put in pairs: half the puts
#pragma unroll
            for (int i = 0; i < C::CH; i += 2) {
                const uint32_t n0 = slot[i] >> 27;
                bw.put((slot[i] & 0x7FFFFFFu) | ((slot[i + 1] & 0x7FFFFFFu) << n0), n0 + (slot[i + 1] >> 27));
            }
        } else {
#pragma unroll
            for (int i = 0; i < C::CH + 2; i++) bw.put(slot[i] & 0x7FFFFFFu, slot[i] >> 27);
        }
        bw.finish();
        if (lastb && tid == 0) {  // end of block; a non-final block ends byte-aligned
            const uint32_t eob = S.lcode[256];
            LdsBitWriter ew{S.out, tb + bitsum};
            ew.put(eob & 0x7FFFFFFu, eob >> 27);
            if (!final_seg) {
                ew.put(0, 3);
                ew.pos = (ew.pos + 7) & ~7u;
                ew.put(0xFFFF0000u, 32);
            }
        }
    }
    ((uint4*)S.crcx)[tid] = tx0;
    if (tid + C::NT < NX4) ((uint4*)S.crcx)[tid + C::NT] = tx1;
    __syncthreads();
    stamp();
    // CRC-32 of out[P, P + o1) (the shared head byte as zero): raw CRC of the 32-byte chunks,
    // each moved to its wave's end by its own operator x^(8*32*(63-lane)) (two table
    // multiplies), XOR-ed over the wave, moved to the segment end by x^(8*2048*(NW-1-w)) and
    // XOR-ed over the waves by thread 0.  Waves whose chunks are all empty skip it.
    const uint32_t nv = (P + o1) >> 2;
    const bool wact = nv >= 8u * (uint32_t)(C::NT - 64 * w - 63);
    uint32_t c = 0;
    if (!PBX_ENC_SKIP_CRC && wact) {
        c = crc_chunk_aligned<C>(tid, S, nv, lb ? P : 0xFFFFFFFFu);
        const uint32_t dl = 63 - lane;
        c = crc_mul_lane(S.crcx + CRCX_TA, dl & 7u, c);
        c = crc_mul_lane(S.crcx + CRCX_TB, dl >> 3, c);
        c = wave_xor(c);
        const uint32_t d = (uint32_t)C::NW - 1 - w;  // waves after this one
#pragma unroll
        for (int k = 0; k < 3; k++)
            if ((d >> k) & 1u) c = crc_mul_tab(S.crcx + CRCX_TW + 128 * k, c);
    }
    if (lane == 0) S.red[w] = c;
    // owned bytes to their final place: unaligned head and tail bytes, aligned words between
    const uint32_t nbytes = o1 - o0;
    uint8_t* dst = out + tile_off + gi.zoff + ZLIB_HDR_BYTES + bi.off + byte0 + o0;
    const uint32_t b0 = P + o0;
#ifndef PBX_ENC_STORE16
#define PBX_ENC_STORE16 1  // 16-byte output stores (0: dword stores, the round-2 form)
#endif
    if (PBX_ENC_STORE16) {
        // aligned 16-byte units: two aligned LDS reads, a uniform word selection and byte
        // shift (the units' LDS offset mod 16 is the same for every thread)
        uint32_t head = (uint32_t)((16u - ((uintptr_t)dst & 15u)) & 15u);
        if (head > nbytes) head = nbytes;
        const uint32_t n16 = PBX_ENC_SKIP_STORE ? 0u : (nbytes - head) >> 4;
        if (tid < head) dst[tid] = (uint8_t)out_byte_at(S, b0 + tid);
        const uint32_t j0 = b0 + head, w0 = (j0 >> 2) & ~3u, sb = j0 & 3u;
        const uint32_t wq = __builtin_amdgcn_readfirstlane((j0 >> 2) & 3u);
        for (uint32_t k = tid; k < n16; k += C::NT) {
            const uint4 a = *(const uint4*)&S.out[w0 + 4 * k], b = *(const uint4*)&S.out[w0 + 4 * k + 4];
            const uint32_t z[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
            uint32_t q[5];
            switch (wq) {
            case 0:
#pragma unroll
                for (int i = 0; i < 5; i++) q[i] = z[i];
                break;
            case 1:
#pragma unroll
                for (int i = 0; i < 5; i++) q[i] = z[i + 1];
                break;
            case 2:
#pragma unroll
                for (int i = 0; i < 5; i++) q[i] = z[i + 2];
                break;
            default:
#pragma unroll
                for (int i = 0; i < 5; i++) q[i] = z[i + 3];
                break;
            }
            const uint4 ov =
                make_uint4(__builtin_amdgcn_alignbyte(q[1], q[0], sb), __builtin_amdgcn_alignbyte(q[2], q[1], sb),
                           __builtin_amdgcn_alignbyte(q[3], q[2], sb), __builtin_amdgcn_alignbyte(q[4], q[3], sb));
            if (PBX_NT_STREAM & 4) gstore16_nt(dst + head + 16 * k, ov); else *(uint4*)(dst + head + 16 * k) = ov;
        }
        for (uint32_t j = head + 16 * n16 + tid; j < nbytes; j += C::NT) dst[j] = (uint8_t)out_byte_at(S, b0 + j);
    } else {
        uint32_t head = (uint32_t)((4u - ((uintptr_t)dst & 3u)) & 3u);
        if (head > nbytes) head = nbytes;
        const uint32_t nwords = PBX_ENC_SKIP_STORE ? 0u : (nbytes - head) >> 2;
        if (tid < head) dst[tid] = (uint8_t)out_byte_at(S, b0 + tid);
        for (uint32_t k = tid; k < nwords; k += C::NT) *(uint32_t*)(dst + head + 4 * k) = out_word(S, b0 + head + 4 * k);
        for (uint32_t j = head + 4 * nwords + tid; j < nbytes; j += C::NT) dst[j] = (uint8_t)out_byte_at(S, b0 + j);
    }
#ifndef PBX_ENC_LAST_WAVE
#define PBX_ENC_LAST_WAVE 0  // 1: the last wave to finish joins the CRC, no workgroup barrier (measured 4-7% slower: profiles/r05zf/)
#endif
    // the segment's record: the waves' CRC terms joined by the last wave to get here (LDS
    // atomics of one wave complete in order: its XOR lands before its count), or by thread 0
    // after a barrier
    auto finish = [&](uint32_t raw) {
        const bool has_tail = !final_seg && (le & 7u) && !(lb && (le >> 3) == 0);
        uint32_t part = 0;
        if (lb) part |= out_byte_at(S, P) | SP_HEAD;
        if (has_tail) part |= (out_byte_at(S, P + (le >> 3)) << 8) | SP_TAIL;
        SegInfo& g = info[seg];
        if (nbytes < CRC_TAB_N) {
            g.crc = raw ^ g_crc_fin[nbytes];
            g.crc_op = g_crc_x8n[nbytes];
        } else {
            const uint32_t op = crc_x8n_small(nbytes);
            g.crc = crc_from_raw(raw, op);
            g.crc_op = op;
        }
        g.part = part;
        g.bitsum = bitsum;
    };
    if (PBX_ENC_LAST_WAVE) {
        if (lane == 0) {
            atomicXor(&S.crc_acc, c);
            if (atomicAdd(&S.ndone, 1u) == (uint32_t)C::NW - 1) finish(atomicOr(&S.crc_acc, 0u));
        }
    } else {
        __syncthreads();
        if (tid == 0) {
            uint32_t raw = 0;
#pragma unroll
            for (int k = 0; k < C::NW; k++) raw ^= S.red[k];
            finish(raw);
        }
    }
    // a single-tile batch (frame_ctr, zeroed by k_huff): the workgroup that finishes last
    // frames the tile -- k_frame_wave's work without its launch (wave 0: thread 0 wrote this
    // segment's record above; the fences order it before the count, and the others' before
    // the reads of theirs)
    if (FRAME && w == 0) {
        uint32_t lastw = 0;
        if (lane == 0) {
            __threadfence();
            lastw = atomicAdd(frame_ctr, 1u) == nseg - 1 ? 1u : 0u;
        }
        if (__builtin_amdgcn_readfirstlane(lastw)) {
            __threadfence();
            const TileDesc td = load_desc(dt);
            frame_wave_tile<true>(td, out + offs[0], info, blk, lane);
        }
    }
    stamp();
}

// ===================================================================== k_frame

// CRC-32 register updates from values (reflected, raw: the caller applies the pre/post xor)
__device__ __forceinline__ uint32_t crc_u8(uint32_t c, uint32_t b) { return crc_byte4(c, b); }
__device__ __forceinline__ uint32_t crc_be32(uint32_t c, uint32_t v) {  // v's 4 bytes, big-endian
    c = crc_u8(c, v >> 24); c = crc_u8(c, v >> 16); c = crc_u8(c, v >> 8);
    return crc_u8(c, v);
}

constexpr uint32_t FOURCC(char a, char b, char c, char d) {
    return ((uint32_t)(uint8_t)a << 24) | ((uint32_t)(uint8_t)b << 16) | ((uint32_t)(uint8_t)c << 8) | (uint8_t)d;
}

// A PNG chunk whose data are the words wd[0..NW) (big-endian) then nz zero bytes: length,
// type, data, and the CRC computed from the values (no read-back of the bytes just written).
template <int NW>
__device__ __forceinline__ uint32_t put_chunk_w(uint8_t* o, uint32_t type, const uint32_t (&wd)[NW], uint32_t nz) {
    const uint32_t n = 4 * NW + nz;
    put_be32(o, n);
    put_be32(o + 4, type);
    uint32_t c = crc_be32(0xFFFFFFFFu, type);
#pragma unroll
    for (int k = 0; k < NW; k++) {
        put_be32(o + 8 + 4 * k, wd[k]);
        c = crc_be32(c, wd[k]);
    }
    for (uint32_t k = 0; k < nz; k++) {
        o[8 + 4 * NW + k] = 0;
        c = crc_u8(c, 0);
    }
    put_be32(o + 8 + n, c ^ 0xFFFFFFFFu);
    return 12 + n;
}


// One tile: everything around the segments' bytes, and the bytes two segments of a block
// share (SegInfo.part), joined in stream order into the output and the IDAT CRC.
__device__ __forceinline__ void frame_tile(const TileDesc& d, uint8_t* __restrict__ base,
                                           const SegInfo* __restrict__ info, const BlkInfo* __restrict__ blk) {
    const bool tiff = (d.flags & TF_TIFF) != 0;
    const uint32_t zoff = container_zoff(d);
    uint32_t s1 = 0, s2 = 0, payload = 0;
#pragma unroll 4
    for (uint32_t k = 0; k < d.seg_count; k++) {  // (unrolled: four segments' loads in flight)
        const SegInfo& g = info[d.seg_first + k];
        adler_combine(s1, s2, g.adler_s1, g.adler_s2, g.sl);
    }
    const uint32_t nb = tile_blocks(d.seg_count, PBX_TILE_BLK_CAP(d));
    for (uint32_t k = 0; k < nb; k++) payload += blk[d.hblk_first + k].nbytes;
    const uint32_t adler = adler_final(s1, s2, d.stream_len);
    const uint64_t pos = zoff + ZLIB_HDR_BYTES + payload;
    base[zoff] = 0x78;      // CMF: deflate, 32 KiB window
    base[zoff + 1] = 0x9C;  // FLG: default level (Deflater -1 == 6), check bits
    put_be32(base + pos, adler);
    uint32_t o = 8;
    if (!tiff) {
        const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
        for (int j = 0; j < 8; j++) base[j] = sig[j];
        // IHDR: w, h, bit depth, then colour type / compression / filter / interlace 0
        const uint32_t ihdr[3] = {(uint32_t)d.w, (uint32_t)d.h, (8u * (uint32_t)d.bpp) << 24};
        o += put_chunk_w(base + o, FOURCC('I', 'H', 'D', 'R'), ihdr, 1);
        const uint32_t actl[2] = {1u, 0u};  // acTL: 1 frame, 0 plays
        o += put_chunk_w(base + o, FOURCC('a', 'c', 'T', 'L'), actl, 0);
        const uint32_t fctl[3] = {0u, (uint32_t)d.w, (uint32_t)d.h};  // fcTL: seq 0, w, h, offsets 0, delay 0/0, ops 0
        o += put_chunk_w(base + o, FOURCC('f', 'c', 'T', 'L'), fctl, 14);
        // IDAT: length, type, zlib stream
        put_be32(base + o, ZLIB_HDR_BYTES + payload + 4);
        put_be32(base + o + 4, FOURCC('I', 'D', 'A', 'T'));
    }
    // CRC over type + zlib stream (PNG), joined from the segments' CRCs and shared bytes
    uint32_t c = tiff ? 0u
                      : crc_u8(crc_u8(crc_be32(0xFFFFFFFFu, FOURCC('I', 'D', 'A', 'T')), 0x78), 0x9C) ^ 0xFFFFFFFFu;
    uint8_t* z = base + zoff + ZLIB_HDR_BYTES;
    for (uint32_t k = 0; k < nb; k++) {
        const BlkInfo bi = blk[d.hblk_first + k];
        bool pend = false;
        uint32_t pv = 0, pidx = 0;
        auto flush = [&]() {
            const uint8_t v = (uint8_t)pv;
            z[bi.off + pidx] = v;
            if (!tiff) c = crc_u8(c ^ 0xFFFFFFFFu, v) ^ 0xFFFFFFFFu;
            pend = false;
        };
        for (uint32_t q = 0; q < bi.nseg; q++) {
            const SegInfo& g = info[bi.seg0 + q];
            const uint32_t b0 = g.bit0 >> 3, le = g.bit1 - 8 * b0, o0 = (g.bit0 & 7u) ? 1u : 0u;
            uint32_t o1 = g.last ? (le + 7) >> 3 : le >> 3;
            if (o1 < o0) o1 = o0;
            if (g.part & SP_HEAD) {
                if (!pend) { pend = true; pv = 0; pidx = b0; }
                pv |= g.part & 0xFFu;
            }
            if (o1 > o0) {
                if (pend) flush();
                if (!tiff) c = crc_combine_op(c, g.crc, g.crc_op);
            }
            if (g.part & SP_TAIL) {
                if (pend) flush();
                pend = true;
                pv = (g.part >> 8) & 0xFFu;
                pidx = g.bit1 >> 3;
            }
        }
        if (pend) flush();
    }
    if (d.flags & TF_TILED) return;  // header and tile arrays: k_tiff_tiled
    if (tiff) {
        write_tiff_header(base, d.w, d.h, d.bpp, tiff_sample_format(d.pixel_type), 8,
                          ZLIB_HDR_BYTES + payload + 4);
        return;
    }
    c = crc_be32(c ^ 0xFFFFFFFFu, adler) ^ 0xFFFFFFFFu;
    put_be32(base + pos + 4, c);
    put_be32(base + pos + 8, 0);  // IEND: no data
    put_be32(base + pos + 12, FOURCC('I', 'E', 'N', 'D'));
    put_be32(base + pos + 16, 0xAE426082u);  // its CRC
}

// One thread per tile (large batches: 64 tiles' serial joins in lockstep per wave).
__global__ __launch_bounds__(64) void k_frame(const TileDesc* __restrict__ dt, uint32_t ndt,
                                              const SegInfo* __restrict__ info,
                                              const BlkInfo* __restrict__ blk,
                                              const uint64_t* __restrict__ offs,
                                              uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 64 + threadIdx.x;
    if (i >= ndt) return;
    const TileDesc d = dt[i];
    frame_tile(d, out + offs[i], info, blk);
}

// The same bytes for a small batch (the single-request latency path), one wave per tile: a
// tile's serial join is ~33 dependent CRC multiplies (~18 us for one tile on an idle chip).
// Lane k takes segment k (64 at a time): its Adler-32 term (bytes after it by a wave scan)
// and its CRC item -- the byte it shares with segment k - 1 when its bits start mid-byte,
// written here, then the bytes it owns: crc(v || own) = crc(v) x^(8 |own|) + crc(own).  The
// items are joined in stream order by a 6-level lane tree ((I1, O1) then (I2, O2) =
// (I1 O2 + I2, O1 O2)) with nibble-step multiplies; lanes 1-3 write the PNG chunks before
// IDAT.  A tile with a segment that owns no byte (all its bits inside one byte: the byte is
// then shared by three segments) takes frame_tile on lane 0.
// LR: low register use (loops not unrolled), for the copy inside k_encode's 64-VGPR budget
__device__ __forceinline__ uint32_t crc_multmodp4_lr(uint32_t a, uint32_t b) {
    const uint32_t b1 = (b >> 1) ^ ((b & 1u) ? CRC_POLY : 0u);
    const uint32_t b2 = (b >> 2) ^ ((b & 1u) ? (CRC_POLY >> 1) : 0u) ^ ((b & 2u) ? CRC_POLY : 0u);
    const uint32_t b3 = (b >> 3) ^ ((b & 1u) ? (CRC_POLY >> 2) : 0u) ^ ((b & 2u) ? (CRC_POLY >> 1) : 0u) ^
                        ((b & 4u) ? CRC_POLY : 0u);
    uint32_t p = 0;
#pragma unroll 1
    for (int s = 7; s >= 0; s--) {
        const uint32_t t = ((a >> (31 - 4 * s)) & 1u ? b : 0u) ^ ((a >> (30 - 4 * s)) & 1u ? b1 : 0u) ^
                           ((a >> (29 - 4 * s)) & 1u ? b2 : 0u) ^ ((a >> (28 - 4 * s)) & 1u ? b3 : 0u);
        p = crc_x4(p) ^ t;
    }
    return p;
}
template <bool LR>
__device__ void frame_wave_tile(const TileDesc& d, uint8_t* __restrict__ base, const SegInfo* __restrict__ info,
                                const BlkInfo* __restrict__ blk, uint32_t lane) {
    auto mul = [](uint32_t a, uint32_t b) { return LR ? crc_multmodp4_lr(a, b) : crc_multmodp4(a, b); };
    const bool tiff = (d.flags & TF_TIFF) != 0;
    const uint32_t zoff = container_zoff(d), n = d.seg_count, f = d.seg_first;
    // Two dependent rounds of loads (a lone tile waits on each, ~1 us): the descriptor, then
    // every segment's record, the part of the one before it and the tile's block records
    // (lane j: block j; a segment finds its block's offset in the lanes).
    const uint32_t nb = tile_blocks(n, PBX_TILE_BLK_CAP(d)), hb = d.hblk_first;
    uint32_t bnb = 0, boff = 0;
    if (lane < nb) {
        bnb = blk[hb + lane].nbytes;
        boff = blk[hb + lane].off;
    }
    uint32_t payload = bnb;
    for (uint32_t k = lane + 64; k < nb; k += 64) payload += blk[hb + k].nbytes;
    uint8_t* z = base + zoff + ZLIB_HDR_BYTES;
    constexpr uint32_t X0 = 1u << 31;  // the operator x^0
    const uint32_t X8 = crc_x8pow2(0);
    // raw Adler sums, and the IDAT CRC (conditioned) from "IDAT" 78 9C on
    uint32_t s1 = 0, s2 = 0;
    uint64_t before = 0;
    uint32_t c = crc_u8(crc_u8(crc_be32(0xFFFFFFFFu, FOURCC('I', 'D', 'A', 'T')), 0x78), 0x9C) ^ 0xFFFFFFFFu;
    for (uint32_t k0 = 0; k0 < n; k0 += 64) {
        const uint32_t k = k0 + lane;
        const bool v = k < n;
        const SegInfo& g = info[f + (v ? k : 0u)];
        const uint32_t sl = v ? g.sl : 0u, a1 = v ? g.adler_s1 : 0u, a2 = v ? g.adler_s2 : 0u;
        const uint32_t part = v ? g.part : 0u, bit0 = v ? g.bit0 : 0u, bit1 = v ? g.bit1 : 0u;
        const uint32_t last = v ? g.last : 0u, gb = v ? g.blk : hb, gcrc = v ? g.crc : 0u;
        const uint32_t gop = v ? g.crc_op : X0;
        const uint32_t pp = v && k ? info[f + k - 1].part : 0u;
        // every segment owns a byte (the tree's item form), else the serial join (the shared
        // bytes written so far are the values it writes too)
        {
            const uint32_t b0 = bit0 >> 3, le = bit1 - 8 * b0, o0 = (bit0 & 7u) ? 1u : 0u;
            const uint32_t o1 = last ? (le + 7) >> 3 : le >> 3;
            if (__builtin_amdgcn_ballot_w64(v && o1 <= o0)) {
                if (lane == 0) frame_tile(d, base, info, blk);
                return;
            }
        }
        // Adler: s2 gains a1 x (bytes after this segment)
        const uint32_t incl = wave_incl_scan_dpp(sl);
        const uint64_t after = d.stream_len - (before + incl);
        const uint32_t t2 = (uint32_t)(((uint64_t)a1 * (after % ADLER_BASE) + a2) % ADLER_BASE);
        s1 = (s1 + wave_sum(a1) % ADLER_BASE) % ADLER_BASE;
        s2 = (s2 + wave_sum(t2) % ADLER_BASE) % ADLER_BASE;
        before += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);  // (segments < 4 GiB)
        // the block's offset: from its lane (blocks 64.. from memory)
        const uint32_t bj = gb - hb;
        const uint32_t bo_l = (uint32_t)__shfl((int)boff, (int)(bj < 64 ? bj : 0u), 64);
        // the byte shared with segment k - 1 (its tail bits | this segment's head bits)
        uint32_t I = gcrc, O = gop;
        if (v && (part & SP_HEAD)) {
            const uint32_t sb = (part & 0xFFu) | ((pp & SP_TAIL) ? (pp >> 8) & 0xFFu : 0u);
            z[(bj < 64 ? bo_l : blk[gb].off) + (bit0 >> 3)] = (uint8_t)sb;
            if (!tiff) {
                const uint32_t cb = crc_byte4(0xFFFFFFFFu, sb) ^ 0xFFFFFFFFu;
                I = mul(O, cb) ^ I;
                O = mul(O, X8);
            }
        }
        if (!tiff) {
            // levels past the segments present combine identity items only: stop there
            const uint32_t nk = __builtin_amdgcn_readfirstlane(n - k0 < 64 ? n - k0 : 64u);
            // (I, O) of lanes [lane, lane + 2s) on lane % 2s == 0
            auto level = [&](uint32_t s) {
                const uint32_t I2 = (uint32_t)__shfl_down((int)I, s, 64), O2 = (uint32_t)__shfl_down((int)O, s, 64);
                const bool has = lane + s < 64;
                const uint32_t In = mul(O2, I) ^ I2, On = mul(O, O2);
                I = has ? In : I;
                O = has ? On : O;
            };
            if (LR) {
#pragma unroll 1
                for (uint32_t s = 1; s < nk; s <<= 1) level(s);
            } else {
#pragma unroll
                for (int s = 1; s < 64; s <<= 1) {
                    if ((uint32_t)s >= nk) break;
                    level((uint32_t)s);
                }
            }
            const uint32_t Ic = (uint32_t)__builtin_amdgcn_readfirstlane((int)I);
            const uint32_t Oc = (uint32_t)__builtin_amdgcn_readfirstlane((int)O);
            c = mul(Oc, c) ^ Ic;
        }
    }
    payload = wave_sum(payload);
    const uint32_t adler = adler_final(s1, s2, d.stream_len);
    const uint64_t pos = zoff + ZLIB_HDR_BYTES + payload;
    if (lane == 0) {
        z[-2] = 0x78;  // CMF: deflate, 32 KiB window
        z[-1] = 0x9C;  // FLG: default level, check bits
        put_be32(base + pos, adler);
    }
    if (d.flags & TF_TILED) return;  // header and tile arrays: k_tiff_tiled
    if (tiff) {
        if (lane == 0)
            write_tiff_header(base, d.w, d.h, d.bpp, tiff_sample_format(d.pixel_type), 8, ZLIB_HDR_BYTES + payload + 4);
        return;
    }
    if (lane == 0) {
        const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
        for (int j = 0; j < 8; j++) base[j] = sig[j];
        put_be32(base + PNG_IDAT_DATA_OFF - 8, ZLIB_HDR_BYTES + payload + 4);
        put_be32(base + PNG_IDAT_DATA_OFF - 4, FOURCC('I', 'D', 'A', 'T'));
        put_be32(base + pos + 4, crc_be32(c ^ 0xFFFFFFFFu, adler) ^ 0xFFFFFFFFu);
        put_be32(base + pos + 8, 0);  // IEND
        put_be32(base + pos + 12, FOURCC('I', 'E', 'N', 'D'));
        put_be32(base + pos + 16, 0xAE426082u);
    } else if (lane == 1) {  // IHDR: w, h, bit depth, colour type / compression / filter / interlace 0
        const uint32_t ihdr[3] = {(uint32_t)d.w, (uint32_t)d.h, (8u * (uint32_t)d.bpp) << 24};
        put_chunk_w(base + PNG_SIG_BYTES, FOURCC('I', 'H', 'D', 'R'), ihdr, 1);
    } else if (lane == 2) {  // acTL: 1 frame, 0 plays
        const uint32_t actl[2] = {1u, 0u};
        put_chunk_w(base + PNG_SIG_BYTES + PNG_IHDR_BYTES, FOURCC('a', 'c', 'T', 'L'), actl, 0);
    } else if (lane == 3) {  // fcTL: seq 0, w, h, offsets 0, delay 0/0, ops 0
        const uint32_t fctl[3] = {0u, (uint32_t)d.w, (uint32_t)d.h};
        put_chunk_w(base + PNG_SIG_BYTES + PNG_IHDR_BYTES + PNG_ACTL_BYTES, FOURCC('f', 'c', 'T', 'L'), fctl, 14);
    }
}

__global__ __launch_bounds__(64) void k_frame_wave(const TileDesc* __restrict__ dt, uint32_t ndt,
                                                   const SegInfo* __restrict__ info,
                                                   const BlkInfo* __restrict__ blk,
                                                   const uint64_t* __restrict__ offs,
                                                   uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x;
    if (i >= ndt) return;
    const TileDesc d = dt[i];
    frame_wave_tile<false>(d, out + offs[i], info, blk, threadIdx.x);
}

// ================================================================== launchers
size_t deflate_lds_bytes(int kernel) {
    return kernel == 0 ? sizeof(LzSmem<DC>) : kernel == 1 ? sizeof(HuffSmem<DC>) : sizeof(EncSmem<DC>);
}

hipError_t launch_huffman(hipStream_t st, uint32_t nblk, BlkInfo* blk, SegInfo* info,
                          const uint32_t* hist, uint32_t* codes) {
    if (nblk)
        hipLaunchKernelGGL((k_huff<DC, false>), dim3(nblk), dim3(64), 0, st, nblk, blk, info, hist,
                           codes, nullptr);
    return hipGetLastError();
}

// k_crc_tables once per device, finished before any deflate launch can use the tables
static hipError_t crc_tables_ready() {
    constexpr int kMaxDev = 64;
    static std::once_flag once[kMaxDev];
    static hipError_t res[kMaxDev];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
    std::call_once(once[dev], [&] {
        hipStream_t s = nullptr;
        res[dev] = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        if (res[dev] != hipSuccess) return;
        hipLaunchKernelGGL(k_crc_tables, dim3(CRC_TAB_N / 256), dim3(256), 0, s);
        res[dev] = hipGetLastError();
        const hipError_t e2 = hipStreamSynchronize(s);
        if (res[dev] == hipSuccess) res[dev] = e2;
        (void)hipStreamDestroy(s);
    });
    return res[dev];
}

#ifndef PBX_HUFF_SOLO_ARGS
#define PBX_HUFF_SOLO_ARGS 1  // a solo block's segment range as a launch argument (0: loaded from its record)
#endif
hipError_t launch_deflate(hipStream_t st, const DeflateLaunch& a, hipEvent_t* ev, hipEvent_t* ev2, bool fine) {
    if (!a.ntiles || !a.nseg) return hipSuccess;
    if (const hipError_t e = crc_tables_ready(); e != hipSuccess) return e;
    const bool prof = a.stamps != nullptr;
    // a small batch of equal segment counts: k_lz77 maps its own segment (one launch less on
    // the latency path; in large batches the mapping's divisions cost k_lz77 more than the
    // separate launch, profiles/r05k/)
    const uint32_t self_map = a.uniform_nseg && a.nseg <= LZ_SELF_MAP_SEGS ? 1u : 0u;
    const bool solo = !prof && a.ntiles == 1 && a.nblk == 1;  // one tile, one Huffman block
#ifndef PBX_ENC_FRAME_SOLO
#define PBX_ENC_FRAME_SOLO 0  // 1: a solo tile framed by k_encode's last workgroup, no k_frame_wave (measured: no gain, profiles/r05zk/)
#endif
    const bool solo_frame = solo && PBX_ENC_FRAME_SOLO;
    if (!self_map)
        hipLaunchKernelGGL(k_seg_map, dim3((a.nseg + 255) / 256), dim3(256), 0, st, a.tiles, a.ntiles, a.nseg,
                           a.uniform_nseg, a.uniform_rcp, a.seg_tile, a.info, a.blk);
    const uint32_t lz_grid = a.nseg;
#define PBX_LZ_LAUNCH(P, V)                                                                                  \
    hipLaunchKernelGGL((k_lz77<DC, P, V>), dim3(lz_grid), dim3(DC::NT), 0, st, a.tiles, a.seg_tile, a.nseg,   \
                       a.stream, a.info, a.blk, a.hist, a.mrec, a.stamps, a.uniform_nseg, a.uniform_rcp, self_map)
    if (prof) {
        if (a.row_filtered) PBX_LZ_LAUNCH(true, true); else PBX_LZ_LAUNCH(true, false);
    } else {
        if (a.row_filtered) PBX_LZ_LAUNCH(false, true); else PBX_LZ_LAUNCH(false, false);
    }
#undef PBX_LZ_LAUNCH
    if (ev && fine) (void)hipEventRecord(ev[0], st);
    if (ev2) (void)hipEventRecord(ev2[0], st);
    if (prof && a.nblk <= HUFF_SMALL_BLKS)  // (the phase profile of the variant that runs)
        hipLaunchKernelGGL((k_huff<DC, true, 34, HUFF_SMALL_WAVES>), dim3(a.nblk), dim3(64 * HUFF_SMALL_WAVES), 0, st,
                           a.nblk, a.blk, a.info, a.hist, a.codes, a.stamps);
    else if (prof)
        hipLaunchKernelGGL((k_huff<DC, true>), dim3(a.nblk), dim3(64), 0, st, a.nblk, a.blk, a.info,
                           a.hist, a.codes, a.stamps);
    else if (a.nblk <= HUFF_SMALL_BLKS)  // a small batch: every segment's histogram loads at once
        hipLaunchKernelGGL((k_huff<DC, false, 34, HUFF_SMALL_WAVES>), dim3(a.nblk), dim3(64 * HUFF_SMALL_WAVES), 0, st,
                           a.nblk, a.blk, a.info, a.hist, a.codes, a.stamps, solo ? a.tiles : nullptr, a.offs,
                           a.offs_host, solo && PBX_HUFF_SOLO_ARGS ? a.nseg : 0u);
    else
        hipLaunchKernelGGL((k_huff<DC, false>), dim3(a.nblk), dim3(64), 0, st, a.nblk, a.blk, a.info,
                           a.hist, a.codes, a.stamps);
    if (ev && fine) (void)hipEventRecord(ev[1], st);
    if (ev2) (void)hipEventRecord(ev2[1], st);
    if (solo) {  // (k_huff wrote the offsets)
    } else if (a.ntiles <= 1024) {
        hipLaunchKernelGGL(k_sizes_scan, dim3(1), dim3(1024), 0, st, a.tiles, a.ntiles, a.blk, a.offs, a.offs_host);
    } else {
        hipLaunchKernelGGL(k_seg_sizes, dim3((a.ntiles + 255) / 256), dim3(256), 0, st, a.tiles, a.ntiles,
                           a.blk, a.sizes);
        hipLaunchKernelGGL(k_scan_offsets, dim3(1), dim3(1024), 0, st, a.sizes, a.ntiles, a.offs, a.offs_host);
    }
    if (ev && fine) (void)hipEventRecord(ev[2], st);
    if (ev2) (void)hipEventRecord(ev2[2], st);
    if (prof)
        hipLaunchKernelGGL((k_encode<DC, true>), dim3(a.nseg), dim3(DC::NT), 0, st, a.tiles, a.seg_tile,
                           a.nseg, a.stream, a.info, a.blk, a.mrec, a.codes, a.offs, a.out, a.stamps,
                           a.uniform_nseg, a.uniform_rcp);
    else
        if (solo_frame)
            hipLaunchKernelGGL((k_encode<DC, false, true>), dim3(a.nseg), dim3(DC::NT), 0, st, a.tiles, a.seg_tile,
                               a.nseg, a.stream, a.info, a.blk, a.mrec, a.codes, a.offs, a.out, a.stamps,
                               a.uniform_nseg, a.uniform_rcp, &a.blk[0].pad[0]);
        else
            hipLaunchKernelGGL((k_encode<DC, false>), dim3(a.nseg), dim3(DC::NT), 0, st, a.tiles, a.seg_tile,
                               a.nseg, a.stream, a.info, a.blk, a.mrec, a.codes, a.offs, a.out, a.stamps,
                               a.uniform_nseg, a.uniform_rcp);
    if (ev) (void)hipEventRecord(ev[3], st);
    if (ev2) (void)hipEventRecord(ev2[3], st);
    if (solo_frame) {  // (k_encode's last workgroup framed the tile)
    } else if (a.ntiles <= FRAME_WAVE_TILES)  // small batch: a wave per tile (latency)
        hipLaunchKernelGGL(k_frame_wave, dim3(a.ntiles), dim3(64), 0, st, a.tiles, a.ntiles, a.info, a.blk,
                           a.offs, a.out);
    else
        hipLaunchKernelGGL(k_frame, dim3((a.ntiles + 63) / 64), dim3(64), 0, st, a.tiles, a.ntiles, a.info,
                           a.blk, a.offs, a.out);
    return hipGetLastError();
}

}  // namespace pbx

// The timing knobs that change the OUTPUT (they skip a phase to time the rest)
// are for variant builds only: `make OUT=lib/var_<name> EXTRA="-DPBX_TIMING_VARIANT ..."`
// (scripts/variants.sh).  Any other build that sets one refuses to compile, so the product
// library lib/libpbx.so can never ship corrupt PNGs (the Makefile refuses the variant flag for
// OUT=lib).
#if !defined(PBX_TIMING_VARIANT) && (PBX_LZ_SKIP_STORE || PBX_LZ_SKIP_FILL || PBX_LZ_SKIP_HIST || \
    PBX_LZ_SKIP_OUT || PBX_ENC_SKIP_WRITE || PBX_ENC_SKIP_PATCH || PBX_ENC_SKIP_CRC || PBX_ENC_SKIP_STORE || \
    PBX_HUFF_ONEREAD || defined(PBX_LZ_FAKE_LOAD) || defined(PBX_LZ_NOREACH) || defined(PBX_LZ_REACH_DISCARD))
#error "output-changing timing knobs (PBX_LZ_SKIP_*, PBX_ENC_SKIP_*, PBX_HUFF_ONEREAD, PBX_LZ_FAKE_LOAD) need a variant build (-DPBX_TIMING_VARIANT, OUT=lib/var_*)"
#endif
