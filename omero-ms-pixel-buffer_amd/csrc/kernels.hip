// kernels.hip — gfx950 (MI355X / CDNA4) kernels of the /tile pipeline.
//
//   k_gen_plane    synthetic planes in HBM (G_FAKE = Bio-Formats FakeReader, G_NOISE)
//   k_extract      K1  raw + uncompressed TIFF: PixelBuffer.getTileDirect + big-endian
//                      (TileRequestHandler.java:104-112,128; TiffWriter via :122-123)
//   k_filter       K1+K2 getTileDirect + big-endian + APNGWriter sign flip + PNG scanline
//                      filter (adaptive: min sum |residual|) -> per-tile streams in HBM
//   k_deflate      K3/K4 LZ77 (LDS hash + wave-serial greedy/lazy parse) + Huffman +
//                      bit packing, one workgroup per 16 KiB segment (writeImage, :176-199)
//   k_tile_sizes   K7  container size per tile  -> k_scan_offsets: exclusive scan
//   k_assemble     K5/K6 zlib framing (Adler-32 combine), PNG chunks (CRC-32 combine,
//                      APNGWriter layout) or deflate-TIFF header, compacted output
//
// All integer/byte work, HBM- or LDS/ALU-bound: no MFMA.  Kernels are written for wave64
// and use ballot/readlane for the serial parts of the parse.
#include <hip/hip_runtime.h>

#include "deflate_seg.h"
#include "pbx_common.h"
#include "pbx_config.h"
#include "pbx_kernels.h"

namespace pbx {

using DC = DeflateMainCfg;

struct DevOps {
    __device__ static void amin(uint32_t* p, uint32_t v) { atomicMin(p, v); }
    __device__ static void amax(uint32_t* p, uint32_t v) { atomicMax(p, v); }
    __device__ static void add(uint32_t* p, uint32_t v) { atomicAdd(p, v); }
    __device__ static void aor(uint32_t* p, uint32_t v) { atomicOr(p, v); }
};

// Bijective XCD-aware remap: consecutive logical ids land on the same XCD (shared L2),
// since workgroups are dealt round-robin over the 8 XCDs.  Speed only, never correctness.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t n) {
    const uint32_t q = n / 8, r = n % 8, x = b % 8, i = b / 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// Largest i with key(i) <= v, for a non-decreasing key (uniform across the workgroup).
template <class F>
__device__ __forceinline__ uint32_t upper_index(uint32_t n, uint32_t v, F key) {
    uint32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (key(mid) <= v) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Exclusive prefix sum of arr[0..NT) in place; returns the total.  Wave64 shuffles + LDS.
template <int NT>
__device__ uint32_t block_scan_excl_add(uint32_t* arr, uint32_t* wtot, uint32_t tid) {
    const uint32_t v = arr[tid], lane = tid & 63, w = tid >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(inc, off, 64);
        if (lane >= (uint32_t)off) inc += t;
    }
    if (lane == 63) wtot[w] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < NT / 64; i++) {
        const uint32_t x = wtot[i];
        pre += (uint32_t)i < w ? x : 0u;
        tot += x;
    }
    arr[tid] = pre + inc - v;
    __syncthreads();
    return tot;
}

// Wave-serial greedy parse of one sub-segment (scalar twin: ph_parse_emu in deflate_seg.h).
template <class C>
__device__ void ph_parse_dev(uint32_t tid, DeflateSmem<C>& S, const SegParams& sp) {
    const uint32_t w = tid >> 6, lane = tid & 63;
    const uint32_t ss = w * C::SUB;
    const uint32_t se = ss + C::SUB < sp.sl ? ss + C::SUB : sp.sl;
    uint32_t nm = 0, pos = ss;
    while (pos < se) {
        uint32_t L, D;
        eval_pos<C>(S, sp, pos + lane, se, L, D);
        const uint64_t mask = __ballot(L >= 3);
        uint32_t o = 0;
        while (o < 64) {
            const uint64_t m = mask >> o;
            if (!m) { o = 64; break; }
            const uint32_t k = o + (uint32_t)__builtin_ctzll(m);
            uint32_t Lk = __builtin_amdgcn_readlane(L, k);
            const uint32_t Dk = __builtin_amdgcn_readlane(D, k);
            if (k + 1 < 64) {
                const uint32_t L1 = __builtin_amdgcn_readlane(L, k + 1);
                if (L1 > Lk) { o = k + 1; continue; }  // lazy: a longer match starts next
            }
            const uint32_t p = pos + k;
            const uint32_t rem = se - p;
            const uint32_t maxlen = rem < 258 ? rem : 258;
            if (Lk >= (uint32_t)C::CAP && Lk < maxlen) {
                // one wave-wide compare of 4 bytes per lane extends the match past the cap
                const uint32_t a = sp.wl + p, off = Lk + 4 * lane;
                const uint32_t x = off < maxlen ? (lds_ld4(S, a - Dk + off) ^ lds_ld4(S, a + off)) : 0u;
                const uint64_t mm = __ballot(off >= maxlen || x != 0);
                const uint32_t f = (uint32_t)__builtin_ctzll(mm);
                const uint32_t xf = __builtin_amdgcn_readlane(x, f);
                const uint32_t of = Lk + 4 * f;
                uint32_t l = of >= maxlen ? maxlen : of + ((uint32_t)__builtin_ctz(xf | 0x80000000u) >> 3);
                Lk = l < maxlen ? l : maxlen;
            }
            if (nm < (uint32_t)C::MAXMW) {
                if (lane == 0) {
                    S.mpos[w * C::MAXMW + nm] = p | ((Lk - 3) << 16);
                    S.mdist[w * C::MAXMW + nm] = Dk - 1;
                }
                nm++;
            }
            o = k + Lk;
        }
        pos += o;
    }
    if (lane == 0) S.w_nm[w] = nm;
}

// Ascending bitonic sort of SORTN (= NT) keys, one per thread: wave shuffles for
// partners inside a wave, LDS + barriers for the 6 cross-wave steps.
template <class C>
__device__ void bitonic_sort_keys(uint32_t tid, uint32_t* keys) {
    static_assert(C::NT == (int)SORTN, "one key per thread");
    uint32_t v = keys[tid];
#pragma unroll
    for (uint32_t k = 2; k <= SORTN; k <<= 1) {
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            uint32_t o;
            if (j >= 64) {
                keys[tid] = v;
                __syncthreads();
                o = keys[tid ^ j];
                __syncthreads();
            } else {
                o = __shfl_xor(v, (int)j, 64);
            }
            const bool up = (tid & k) == 0, lower = (tid & j) == 0;
            v = (lower == up) ? (v < o ? v : o) : (v < o ? o : v);
        }
    }
    keys[tid] = v;
}

// The serial Huffman merge on one wave per tree (wave 0: literal/length, wave 1: distance).
// Queues live in LDS; the wave keeps 64-entry register windows over them (lane i = entry
// 64*block + i): the leaf read window, the internal-node write window and read window,
// and the step-record write window.  Every access is one readlane or one lane select;
// windows move (one LDS access per lane) every 64 entries.  Same records as
// twoqueue_serial in deflate_seg.h.
template <class C>
__device__ void ph_twoqueue_dev(uint32_t tid, DeflateSmem<C>& S) {
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    if (wv > 1) return;
    const uint32_t T = wv;
    const uint32_t n = __builtin_amdgcn_readfirstlane(S.misc[T ? M_ND : M_NL]);
    const uint32_t base = __builtin_amdgcn_readfirstlane(T ? S.misc[M_NL] : 0u);
    const uint32_t* sk = S.u.hs.skey + base;
    uint32_t* iq = S.u.hs.dB[T];  // internal weights (dB is free until the jump rounds)
    uint32_t* rq = S.u.hs.rec[T];
    const uint32_t INF = 0xFFFFFFFFu;
    uint32_t lblk = 0, iwblk = 0, irblk = 0xFFFFFFFFu, rblk = 0;
    uint32_t Wwin = lane < n ? key_weight(sk[lane]) : INF;
    uint32_t Iw = 0, Ir = 0, Rw = 0;
    uint32_t li = 0, qi = 0, ni = 0;
    uint32_t lw = __builtin_amdgcn_readlane(Wwin, 0), iw = INF;
    for (uint32_t s = 0; s + 1 < n; s++) {
        const uint32_t rec = li | (qi << 10);
        uint32_t cnt = 0, sum = 0;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if (lw <= iw) {
                sum += lw; li++; cnt++;
                if (li < n) {
                    if ((li >> 6) != lblk) {
                        lblk = li >> 6;
                        const uint32_t e = lblk * 64 + lane;
                        Wwin = e < n ? key_weight(sk[e]) : INF;
                    }
                    lw = __builtin_amdgcn_readlane(Wwin, li & 63);
                } else {
                    lw = INF;
                }
            } else {
                sum += iw; qi++;
                if (qi < ni) {
                    if ((qi >> 6) == iwblk) {
                        iw = __builtin_amdgcn_readlane(Iw, qi & 63);
                    } else {
                        if ((qi >> 6) != irblk) { irblk = qi >> 6; Ir = iq[irblk * 64 + lane]; }
                        iw = __builtin_amdgcn_readlane(Ir, qi & 63);
                    }
                } else {
                    iw = INF;
                }
            }
        }
        if ((ni >> 6) != iwblk) {  // the write window moves on: flush it
            if (iwblk * 64 + lane < 288) iq[iwblk * 64 + lane] = Iw;
            iwblk = ni >> 6;
        }
        Iw = lane == (ni & 63) ? sum : Iw;
        if (qi == ni) iw = sum;
        ni++;
        if ((s >> 6) != rblk) {
            if (rblk * 64 + lane < 288) rq[rblk * 64 + lane] = Rw;
            rblk = s >> 6;
        }
        Rw = lane == (s & 63) ? (rec | (cnt << 20)) : Rw;
    }
    if (n > 1 && rblk * 64 + lane < 288) rq[rblk * 64 + lane] = Rw;
}

// PROF: diagnostic build only (PBX_PHASE_PROFILE=1): thread 0 stamps s_memtime after each
// barrier into stamps[seg * 16 + phase]; no output value depends on a stamp.
template <class C, bool PROF>
__global__ __launch_bounds__(C::NT) void k_deflate(const TileDesc* __restrict__ dt, uint32_t ndt,
                                                   uint32_t nseg, const uint8_t* __restrict__ stream,
                                                   uint8_t* __restrict__ slots, uint32_t slot_stride,
                                                   SegOut* __restrict__ segout,
                                                   uint64_t* __restrict__ stamps) {
    __shared__ DeflateSmem<C> S;
    const uint32_t tid = threadIdx.x;
    uint32_t nst = 0;
    auto stamp = [&]() {
        if (PROF && tid == 0) stamps[(size_t)xcd_remap(blockIdx.x, gridDim.x) * 16 + nst] = __builtin_amdgcn_s_memtime();
        nst++;
    };
    stamp();
    const uint32_t seg = xcd_remap(blockIdx.x, gridDim.x);
    if (seg >= nseg) return;
    const uint32_t ti = upper_index(ndt, seg, [&](uint32_t i) { return dt[i].seg_first; });
    const TileDesc d = dt[ti];
    const WordStream src{stream + d.out_off};
    const uint32_t k = seg - d.seg_first;
    const uint64_t s = (uint64_t)k * d.seg_len;
    SegParams sp;
    sp.sl = (uint32_t)((d.stream_len - s) < d.seg_len ? (d.stream_len - s) : d.seg_len);
    sp.wl = (uint32_t)(s < (uint64_t)C::WIN ? s : (uint64_t)C::WIN);
    sp.base = s - sp.wl;
    sp.rowlen = d.rowlen;
    sp.last = (k + 1 == d.seg_count) ? 1u : 0u;

    ph_fill<C>(tid, S, src, sp);
    __syncthreads();
    stamp();
    ph_insert<C, DevOps>(tid, S, sp);
    __syncthreads();
    stamp();
    ph_parse_dev<C>(tid, S, sp);
    __syncthreads();
    stamp();
    ph_hist<C, DevOps>(tid, S, sp);
    __syncthreads();
    stamp();
    ph_keys<C, DevOps>(tid, S);
    __syncthreads();
    bitonic_sort_keys<C>(tid, S.u.hs.skey);
    __syncthreads();
    stamp();
    ph_twoqueue_dev<C>(tid, S);
    __syncthreads();
    stamp();
    ph_parents<C>(tid, S);
    __syncthreads();
#pragma unroll 1
    for (int r = 0; r < JUMP_ROUNDS; r++) {
        ph_jump<C>(tid, S, r);
        __syncthreads();
    }
    stamp();
    ph_leafdepth<C, DevOps>(tid, S);
    __syncthreads();
    ph_fixblc<C>(tid, S);
    __syncthreads();
    ph_assign<C, DevOps>(tid, S);
    __syncthreads();
    stamp();
    ph_rle_mark<C, DevOps>(tid, S);
    __syncthreads();
    ph_rle_count<C>(tid, S);
    __syncthreads();
    {
        const uint32_t nr = block_scan_excl_add<C::NT>(S.u.hs.rcnt, S.wtot, tid);
        if (tid == 0) S.misc[M_NRLE] = nr;
    }
    __syncthreads();
    ph_rle_emit<C, DevOps>(tid, S);
    __syncthreads();
    ph_clen<C>(tid, S);
    __syncthreads();
    ph_rle_bits<C>(tid, S);
    __syncthreads();
    {
        const uint32_t hb = block_scan_excl_add<C::NT>(S.rboff, S.wtot, tid);
        if (tid == 0) S.misc[M_HDRBITS] = hb;
    }
    __syncthreads();
    ph_choose<C>(tid, S, sp);
    __syncthreads();
    ph_codes<C>(tid, S);
    __syncthreads();
    stamp();
    ph_bits<C>(tid, S, sp);
    __syncthreads();
    stamp();
    const uint32_t total = block_scan_excl_add<C::NT>(S.t_a, S.wtot, tid);
    if (tid == 0) S.misc[M_DATABITS] = total;
    __syncthreads();
    stamp();
    ph_write<C, DevOps>(tid, S, sp);
    __syncthreads();
    stamp();
    ph_store<C>(tid, S, sp, slots + (size_t)seg * slot_stride);
    __syncthreads();
    stamp();
#pragma unroll
    for (int lv = 0; lv < C::LOGNT; lv++) {
        ph_tree<C>(tid, S, lv, crc_x8pow2(C::LOG2_CRCC + lv));
        __syncthreads();
    }
    stamp();
    ph_final<C>(tid, S, sp, &segout[seg]);
    stamp();
}

// ------------------------------------------------------------------- synthetic planes
__global__ __launch_bounds__(256) void k_gen_plane(uint8_t* __restrict__ out, int64_t pitch,
                                                   int32_t sx, int32_t sy, int32_t pt, int32_t bpp,
                                                   int32_t kind, uint64_t seed, int32_t plane_no,
                                                   int32_t z, int32_t c, int32_t t) {
    const uint64_t total = (uint64_t)sx * (uint64_t)sy;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += stride) {
        const uint64_t y = idx / (uint64_t)sx, x = idx - y * (uint64_t)sx;
        const uint64_t v = gen_sample(kind, seed, plane_no, z, c, t, pt, (int64_t)x, (int64_t)y);
        uint8_t* p = out + (int64_t)y * pitch + (int64_t)x * bpp;
        switch (bpp) {
        case 1: *p = (uint8_t)v; break;
        case 2: *(uint16_t*)p = (uint16_t)v; break;
        case 4: *(uint32_t*)p = (uint32_t)v; break;
        default: *(uint64_t*)p = v; break;
        }
    }
}

// ------------------------------------------------------------------------ extraction
__device__ __forceinline__ uint32_t bswap16x2(uint32_t v) {
    return ((v & 0x00FF00FFu) << 8) | ((v >> 8) & 0x00FF00FFu);
}

__device__ __forceinline__ uint4 swap16(uint4 q, int bpp) {
    if (bpp == 2) {
        q.x = bswap16x2(q.x); q.y = bswap16x2(q.y); q.z = bswap16x2(q.z); q.w = bswap16x2(q.w);
    } else if (bpp == 4) {
        q.x = __builtin_bswap32(q.x); q.y = __builtin_bswap32(q.y);
        q.z = __builtin_bswap32(q.z); q.w = __builtin_bswap32(q.w);
    } else if (bpp == 8) {
        const uint32_t a = __builtin_bswap32(q.x), b = __builtin_bswap32(q.y);
        const uint32_t c = __builtin_bswap32(q.z), d = __builtin_bswap32(q.w);
        q.x = b; q.y = a; q.z = d; q.w = c;
    }
    return q;
}

__global__ __launch_bounds__(256) void k_extract(const TileDesc* __restrict__ ft, uint32_t nft,
                                                 uint8_t* __restrict__ out) {
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const uint32_t ti = upper_index(nft, b, [&](uint32_t i) { return ft[i].blk_first; });
    const TileDesc d = ft[ti];
    const uint32_t rb = (uint32_t)d.w * (uint32_t)d.bpp;
    const uint32_t r0 = (b - d.blk_first) * d.rows_per_blk;
    const uint32_t r1 = r0 + d.rows_per_blk < (uint32_t)d.h ? r0 + d.rows_per_blk : (uint32_t)d.h;
    uint8_t* base = out + d.out_off;
    if (d.flags & TF_TIFF) {
        if (r0 == 0 && tid == 0)
            write_tiff_header(base, d.w, d.h, d.bpp, tiff_sample_format(d.pixel_type), 1, rb * d.h);
        base += TIFF_DATA_OFFSET;
    }
    const uint8_t* src0 = d.plane + (int64_t)d.y * d.pitch + (int64_t)d.x * d.bpp;
    const bool fast = (((uintptr_t)src0 | (uintptr_t)base | (uintptr_t)d.pitch | rb) & 15u) == 0;
    const bool swap = (d.flags & TF_SWAP) != 0;
    if (fast) {
        const uint32_t n16 = rb >> 4, nv = (r1 - r0) * n16;
        for (uint32_t i = tid; i < nv; i += 256) {
            const uint32_t r = r0 + i / n16, v = i % n16;
            uint4 q = *(const uint4*)(src0 + (int64_t)r * d.pitch + 16 * v);
            if (swap) q = swap16(q, d.bpp);
            *(uint4*)(base + (size_t)r * rb + 16 * v) = q;
        }
    } else {
        TileStream ts;
        ts.init(d, nullptr);
        const uint32_t nbytes = (r1 - r0) * rb;
        for (uint32_t i = tid; i < nbytes; i += 256) {
            const uint32_t r = r0 + i / rb, c = i % rb;
            base[(size_t)r * rb + c] = (uint8_t)ts.be(r, c);
        }
    }
}

// ------------------------------------------------------- K1+K2: extract + PNG filter
// One workgroup per band of FB_ROWS rows of a deflate tile: stage the band's source rows
// (plus the row above) in LDS as big-endian bytes (16-byte loads, byte swap, APNGWriter
// sign flip), choose each row's filter (adaptive mode: minimum sum of |signed residual|,
// one wave per row), then write the band's stream bytes as aligned 16-byte words:
// FB_ROWS * rowlen is a multiple of 16, so bands never share an output word.
constexpr int FB_ROWS = 16;
constexpr int FB_LDS = 64 * 1024;

__device__ __forceinline__ uint4 flip_msb(uint4 q, int bpp) {
    const uint32_t m = bpp == 1 ? 0x80808080u : 0x00800080u;  // MS byte of each BE sample
    q.x ^= m; q.y ^= m; q.z ^= m; q.w ^= m;
    return q;
}

__device__ __forceinline__ uint32_t filt_byte(int ft, uint32_t cur, uint32_t left, uint32_t up,
                                             uint32_t ul) {
    switch (ft) {
    case 0: return cur;
    case 1: return (cur - left) & 0xFF;
    case 2: return (cur - up) & 0xFF;
    case 3: return (cur - ((left + up) >> 1)) & 0xFF;
    default: {
        const int p = (int)left + (int)up - (int)ul;
        const int pa = abs(p - (int)left), pb = abs(p - (int)up), pc = abs(p - (int)ul);
        const uint32_t pr = (pa <= pb && pa <= pc) ? left : (pb <= pc ? up : ul);
        return (cur - pr) & 0xFF;
    }
    }
}

__device__ uint32_t block_min_filter(uint32_t (&sum)[5], uint32_t* red, uint32_t lane) {
    (void)red; (void)lane;
    int best = 0;
    for (int f = 1; f < 5; f++) if (sum[f] < sum[best]) best = f;
    return (uint32_t)best;
}

__global__ __launch_bounds__(256) void k_filter(const TileDesc* __restrict__ dt, uint32_t ndt,
                                                uint8_t* __restrict__ stream) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    const uint32_t b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t ti = upper_index(ndt, b, [&](uint32_t i) { return dt[i].blk_first; });
    const TileDesc d = dt[ti];
    const uint32_t r0 = (b - d.blk_first) * FB_ROWS;
    const uint32_t r1 = r0 + FB_ROWS < (uint32_t)d.h ? r0 + FB_ROWS : (uint32_t)d.h;
    const uint32_t bpp = d.bpp, rb = (uint32_t)d.w * bpp, rowlen = d.rowlen;
    const bool png = (d.flags & TF_PNGROWS) != 0;
    uint8_t* out = stream + d.out_off;
    const uint8_t* src0 = d.plane + (int64_t)d.y * d.pitch + (int64_t)d.x * bpp;
    const uint32_t rbp = ((rb + 15) & ~15u) + 16;
    uint32_t* ftype = (uint32_t*)(sm + FB_LDS - 256);
    const bool fast = (uint64_t)(FB_ROWS + 1) * rbp + 256 <= (uint64_t)FB_LDS &&
                      ((((uintptr_t)src0) | (uintptr_t)d.pitch) & 15) == 0;
    const uint32_t o0 = r0 * rowlen, o1 = r1 * rowlen;
    if (fast) {
        const uint32_t nq = r1 - r0 + 1, nc = (rb + 15) >> 4;
        const bool swap = (d.flags & TF_SWAP) != 0, flip = (d.flags & TF_FLIP) != 0;
        for (uint32_t i = tid; i < nq * nc; i += 256) {
            const uint32_t q = i / nc, c = i - q * nc;
            const int64_t row = (int64_t)r0 - 1 + q;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (row >= 0 && png) {
                v = *(const uint4*)(src0 + row * d.pitch + 16 * c);
                if (swap) v = swap16(v, bpp);
                if (flip) v = flip_msb(v, bpp);
            } else if (row >= 0) {
                v = *(const uint4*)(src0 + row * d.pitch + 16 * c);
                if (swap) v = swap16(v, bpp);
            }
            *(uint4*)(sm + q * rbp + 16 * c) = v;
        }
        __syncthreads();
        if (png && d.filter == 5) {
            for (uint32_t q = 1 + wv; q < nq; q += 4) {
                const uint8_t* L = sm + q * rbp;
                const uint8_t* U = L - rbp;
                uint32_t sum[5] = {0, 0, 0, 0, 0};
                for (uint32_t i = lane; i < rb; i += 64) {
                    const uint32_t cur = L[i], up = U[i];
                    const uint32_t left = i >= bpp ? L[i - bpp] : 0u, ul = i >= bpp ? U[i - bpp] : 0u;
#pragma unroll
                    for (int f = 0; f < 5; f++)
                        sum[f] += (uint32_t)abs((int)(int8_t)(uint8_t)filt_byte(f, cur, left, up, ul));
                }
#pragma unroll
                for (int f = 0; f < 5; f++)
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1) sum[f] += __shfl_xor(sum[f], off, 64);
                if (lane == 0) ftype[q - 1] = block_min_filter(sum, nullptr, 0);
            }
            __syncthreads();
        }
        for (uint32_t o = o0 + 16 * tid; o < o1; o += 16 * 256) {
            uint32_t row = o / rowlen, col = o - row * rowlen;
            uint32_t w4[4] = {0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < 16; k++) {
                uint32_t byte = 0;
                if (o + k < o1) {
                    const uint8_t* L = sm + (row - r0 + 1) * rbp;
                    if (png) {
                        const int ft = d.filter == 5 ? (int)ftype[row - r0] : d.filter;
                        if (col == 0) {
                            byte = (uint32_t)ft;
                        } else {
                            const uint32_t i = col - 1, cur = L[i];
                            if (ft == 0) {
                                byte = cur;
                            } else {
                                const uint8_t* U = L - rbp;
                                byte = filt_byte(ft, cur, i >= bpp ? L[i - bpp] : 0u, U[i],
                                                 i >= bpp ? U[i - bpp] : 0u);
                            }
                        }
                    } else {
                        byte = L[col];
                    }
                }
                w4[k >> 2] |= byte << (8 * (k & 3));
                if (++col == rowlen) { col = 0; row++; }
            }
            *(uint4*)(out + o) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
    } else {
        // wide rows or unaligned regions: bytes straight from the plane
        TileStream ts;
        ts.init(d, nullptr);
        uint32_t* red = (uint32_t*)sm;
        if (png && d.filter == 5) {
            for (uint32_t r = r0; r < r1; r++) {
                if (tid < 5) red[tid] = 0;
                __syncthreads();
                uint32_t sum[5] = {0, 0, 0, 0, 0};
                for (uint32_t i = tid; i < rb; i += 256) {
                    const uint32_t cur = ts.be(r, i), up = r > 0 ? ts.be(r - 1, i) : 0u;
                    const uint32_t left = i >= bpp ? ts.be(r, i - bpp) : 0u;
                    const uint32_t ul = (r > 0 && i >= bpp) ? ts.be(r - 1, i - bpp) : 0u;
                    for (int f = 0; f < 5; f++)
                        sum[f] += (uint32_t)abs((int)(int8_t)(uint8_t)filt_byte(f, cur, left, up, ul));
                }
                for (int f = 0; f < 5; f++) atomicAdd(&red[f], sum[f]);
                __syncthreads();
                if (tid == 0) {
                    int best = 0;
                    for (int f = 1; f < 5; f++) if (red[f] < red[best]) best = f;
                    ftype[r - r0] = (uint32_t)best;
                }
                __syncthreads();
            }
        }
        for (uint32_t o = o0 + tid; o < o1; o += 256) {
            const uint32_t row = o / rowlen, col = o - row * rowlen;
            uint32_t byte;
            if (png) {
                const int ft = d.filter == 5 ? (int)ftype[row - r0] : d.filter;
                byte = col == 0 ? (uint32_t)ft : ts.filtered(ft, row, col - 1);
            } else {
                byte = ts.be(row, col);
            }
            out[o] = (uint8_t)byte;
        }
    }
}

// ------------------------------------------------------------------- sizes + scan
__device__ __forceinline__ uint64_t container_bytes(const TileDesc& d, uint64_t payload) {
    return (d.flags & TF_TIFF) ? TIFF_DATA_OFFSET + ZLIB_HDR_BYTES + payload + 4
                               : PNG_IDAT_DATA_OFF + ZLIB_HDR_BYTES + payload + PNG_TAIL_BYTES;
}

__global__ __launch_bounds__(256) void k_tile_sizes(const TileDesc* __restrict__ dt, uint32_t ndt,
                                                    const SegOut* __restrict__ so,
                                                    uint64_t* __restrict__ sizes) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= ndt) return;
    const TileDesc& d = dt[i];
    uint64_t tot = 0;
    for (uint32_t k = 0; k < d.seg_count; k++) tot += so[d.seg_first + k].nbytes;
    sizes[i] = container_bytes(d, tot);
}

__global__ __launch_bounds__(1024) void k_scan_offsets(const uint64_t* __restrict__ sizes, uint32_t n,
                                                       uint64_t* __restrict__ offs) {
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
    for (uint32_t i = b; i < e; i++) { offs[i] = run; run += sizes[i]; }
    if (tid == 1023) offs[n] = part[1023];
}

// --------------------------------------------------------------------- assemble
// Standard CRC-32 register update, bitwise (only for the few header bytes).
__device__ uint32_t crc_bits(uint32_t c, const uint8_t* p, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        c ^= p[i];
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ CRC_POLY : c >> 1;
    }
    return c;
}

__device__ uint32_t put_chunk(uint8_t* o, const char* type, const uint8_t* data, uint32_t n) {
    put_be32(o, n);
    for (int i = 0; i < 4; i++) o[4 + i] = (uint8_t)type[i];
    for (uint32_t i = 0; i < n; i++) o[8 + i] = data[i];
    const uint32_t crc = crc_bits(0xFFFFFFFFu, o + 4, 4 + n) ^ 0xFFFFFFFFu;
    put_be32(o + 8 + n, crc);
    return 12 + n;
}

__global__ __launch_bounds__(256) void k_assemble(const TileDesc* __restrict__ dt, uint32_t ndt,
                                                  const SegOut* __restrict__ so,
                                                  const uint8_t* __restrict__ slots,
                                                  uint32_t slot_stride,
                                                  const uint64_t* __restrict__ offs,
                                                  uint8_t* __restrict__ out) {
    const uint32_t i = xcd_remap(blockIdx.x, gridDim.x), tid = threadIdx.x;
    if (i >= ndt) return;
    const TileDesc d = dt[i];
    uint8_t* base = out + offs[i];
    const bool tiff = (d.flags & TF_TIFF) != 0;
    const uint32_t zoff = tiff ? TIFF_DATA_OFFSET : PNG_IDAT_DATA_OFF;
    uint64_t pos = zoff + ZLIB_HDR_BYTES;
    for (uint32_t k = 0; k < d.seg_count; k++) {
        const uint32_t n = so[d.seg_first + k].nbytes;
        const uint8_t* src = slots + (size_t)(d.seg_first + k) * slot_stride;
        uint8_t* dst = base + pos;
        for (uint32_t j = tid; j < n; j += 256) dst[j] = src[j];
        pos += n;
    }
    if (tid != 0) return;
    const uint64_t payload = pos - zoff - ZLIB_HDR_BYTES;
    uint32_t s1 = 0, s2 = 0;
    for (uint32_t k = 0; k < d.seg_count; k++) {
        const SegOut& g = so[d.seg_first + k];
        adler_combine(s1, s2, g.adler_s1, g.adler_s2, g.len);
    }
    const uint32_t adler = adler_final(s1, s2, d.stream_len);
    base[zoff] = 0x78;      // CMF: deflate, 32 KiB window
    base[zoff + 1] = 0x9C;  // FLG: default level (Deflater -1 == 6), check bits
    put_be32(base + pos, adler);
    if (tiff) {
        write_tiff_header(base, d.w, d.h, d.bpp, tiff_sample_format(d.pixel_type), 8,
                          (uint32_t)(ZLIB_HDR_BYTES + payload + 4));
        return;
    }
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    for (int j = 0; j < 8; j++) base[j] = sig[j];
    uint32_t o = 8;
    uint8_t buf[26];
    put_be32(buf, d.w); put_be32(buf + 4, d.h);
    buf[8] = (uint8_t)(8 * d.bpp); buf[9] = 0; buf[10] = 0; buf[11] = 0; buf[12] = 0;
    o += put_chunk(base + o, "IHDR", buf, 13);
    put_be32(buf, 1); put_be32(buf + 4, 0);  // acTL: 1 frame, 0 plays
    o += put_chunk(base + o, "acTL", buf, 8);
    for (int j = 0; j < 26; j++) buf[j] = 0;  // fcTL: seq 0, w, h, offsets 0, delay 0/0, ops 0
    put_be32(buf + 4, d.w); put_be32(buf + 8, d.h);
    o += put_chunk(base + o, "fcTL", buf, 26);
    // IDAT: length, type, zlib stream; CRC over type + data combined from segment CRCs
    put_be32(base + o, (uint32_t)(ZLIB_HDR_BYTES + payload + 4));
    base[o + 4] = 'I'; base[o + 5] = 'D'; base[o + 6] = 'A'; base[o + 7] = 'T';
    uint32_t c = crc_bits(0xFFFFFFFFu, base + o + 4, 4 + ZLIB_HDR_BYTES) ^ 0xFFFFFFFFu;
    for (uint32_t k = 0; k < d.seg_count; k++) {
        const SegOut& g = so[d.seg_first + k];
        c = crc_combine_op(c, g.crc, g.crc_op);
    }
    c = crc_bits(c ^ 0xFFFFFFFFu, base + pos, 4) ^ 0xFFFFFFFFu;
    put_be32(base + pos + 4, c);
    put_chunk(base + pos + 8, "IEND", nullptr, 0);
}

// ------------------------------------------------------------------------ launchers
uint32_t deflate_slot_stride() { return (uint32_t)((DC::SEG + 64 + 255) & ~255); }
uint32_t deflate_threads() { return DC::NT; }
size_t deflate_lds_bytes() { return sizeof(DeflateSmem<DC>); }

hipError_t launch_gen_plane(hipStream_t st, uint8_t* out, int64_t pitch, int32_t sx, int32_t sy,
                            int32_t pt, int32_t kind, uint64_t seed, int32_t plane_no, int32_t z,
                            int32_t c, int32_t t) {
    static const int bpps[PT_N] = {1, 1, 2, 2, 4, 4, 4, 8};
    const uint64_t total = (uint64_t)sx * (uint64_t)sy;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_plane, dim3((uint32_t)blocks), dim3(256), 0, st, out, pitch, sx, sy, pt,
                       bpps[pt], kind, seed, plane_no, z, c, t);
    return hipGetLastError();
}

hipError_t launch_extract(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                          uint32_t nblocks, uint8_t* out) {
    if (!ntiles || !nblocks) return hipSuccess;
    hipLaunchKernelGGL(k_extract, dim3(nblocks), dim3(256), 0, st, d_tiles, ntiles, out);
    return hipGetLastError();
}

hipError_t launch_filter(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                         uint32_t nblocks, uint8_t* stream) {
    if (!ntiles || !nblocks) return hipSuccess;
    hipLaunchKernelGGL(k_filter, dim3(nblocks), dim3(256), FB_LDS, st, d_tiles, ntiles, stream);
    return hipGetLastError();
}

uint32_t filter_band_rows() { return FB_ROWS; }

hipError_t launch_deflate(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles, uint32_t nseg,
                          const uint8_t* stream, uint8_t* slots, uint32_t slot_stride,
                          SegOut* segout, uint64_t* stamps) {
    if (!ntiles || !nseg) return hipSuccess;
    if (stamps)
        hipLaunchKernelGGL((k_deflate<DC, true>), dim3(nseg), dim3(DC::NT), 0, st, d_tiles, ntiles,
                           nseg, stream, slots, slot_stride, segout, stamps);
    else
        hipLaunchKernelGGL((k_deflate<DC, false>), dim3(nseg), dim3(DC::NT), 0, st, d_tiles, ntiles,
                           nseg, stream, slots, slot_stride, segout, stamps);
    return hipGetLastError();
}

hipError_t launch_sizes_scan(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                             const SegOut* segout, uint64_t* sizes, uint64_t* offsets) {
    if (!ntiles) return hipSuccess;
    hipLaunchKernelGGL(k_tile_sizes, dim3((ntiles + 255) / 256), dim3(256), 0, st, d_tiles, ntiles,
                       segout, sizes);
    hipLaunchKernelGGL(k_scan_offsets, dim3(1), dim3(1024), 0, st, sizes, ntiles, offsets);
    return hipGetLastError();
}

hipError_t launch_assemble(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                           const SegOut* segout, const uint8_t* slots, uint32_t slot_stride,
                           const uint64_t* offsets, uint8_t* out) {
    if (!ntiles) return hipSuccess;
    hipLaunchKernelGGL(k_assemble, dim3(ntiles), dim3(256), 0, st, d_tiles, ntiles, segout, slots,
                       slot_stride, offsets, out);
    return hipGetLastError();
}

}  // namespace pbx
