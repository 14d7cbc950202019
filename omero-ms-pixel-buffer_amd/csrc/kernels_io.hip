// kernels_io.hip — gfx950 kernels that move pixels: synthetic planes, K1 (raw / TIFF
// extraction) and K1+K2 (extraction fused with the PNG scanline filter).
//
//   k_gen_plane  synthetic planes in HBM (G_FAKE = Bio-Formats FakeReader, G_NOISE)
//   k_extract    K1  PixelBuffer.getTileDirect + big-endian, raw tiles and uncompressed TIFF
//                    (TileRequestHandler.java:104-112,128; TiffWriter via :122-123)
//   k_filter     K1+K2 getTileDirect + big-endian + APNGWriter sign flip + PNG scanline
//                    filter (adaptive: min sum |residual|) -> per-tile streams in HBM
// HBM-bound byte work: 16-byte loads/stores, byte swaps in registers, no MFMA.
#include <hip/hip_runtime.h>

#include "dev_util.h"
#include "pbx_common.h"
#include "pbx_kernels.h"

namespace pbx {

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

// ------------------------------------------------------------------------ launchers
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

// ------------------------------------------------------- K1+K2 fast rows (filter None)
// The stream of a filter-None PNG tile is row r = [0] ++ big-endian row bytes, and of a
// deflate-TIFF tile the row bytes alone.  Each thread writes aligned 16-byte stream words:
// 16 bytes of one source row at byte offset s come from two aligned 16-byte loads (byte
// swap / sign flip applied on the aligned words, where sample boundaries are known) and a
// funnel shift by s & 15; the ~1/64 of words that straddle a row end are merged bytewise
// from both rows.  No LDS: neighbouring lanes share the overlapping loads in L1/L2.
constexpr int RW_NT = 256;
constexpr int RW_WPT = (int)ROWS_WORDS_PER_BLOCK / RW_NT;

struct Rows16 {
    const uint8_t* row;  // source row start (16-byte aligned), little- or big-endian samples
    uint32_t rb, bpp;
    bool swap, flip;
    __device__ __forceinline__ uint4 fix(uint4 v) const {
        if (swap) v = swap16(v, (int)bpp);
        if (flip) v = flip_msb(v, (int)bpp);
        return v;
    }
    // 16 big-endian row bytes starting at byte s (-16 <= s < rb); bytes outside [0, rb)
    // are unspecified
    __device__ __forceinline__ uint4 fetch(int32_t s) const {
        uint4 lo, hi;
        uint32_t sh;
        if (s < 0) {
            lo = make_uint4(0, 0, 0, 0);
            hi = fix(*(const uint4*)row);
            sh = (uint32_t)(s + 16);
        } else {
            const uint32_t a = (uint32_t)s & ~15u;
            lo = fix(*(const uint4*)(row + a));
            sh = (uint32_t)s & 15u;
            hi = (sh && a + 16 < rb) ? fix(*(const uint4*)(row + a + 16)) : make_uint4(0, 0, 0, 0);
        }
        if (!sh) return lo;
        const uint32_t q = sh >> 2, t = (sh & 3) * 8;
        const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        uint32_t v[5];
#pragma unroll
        for (int i = 0; i < 5; i++)
            v[i] = q == 0 ? w[i] : q == 1 ? w[i + 1] : q == 2 ? w[i + 2] : w[i + 3];
        if (!t) return make_uint4(v[0], v[1], v[2], v[3]);
        return make_uint4((v[0] >> t) | (v[1] << (32 - t)), (v[1] >> t) | (v[2] << (32 - t)),
                          (v[2] >> t) | (v[3] << (32 - t)), (v[3] >> t) | (v[4] << (32 - t)));
    }
};

__device__ __forceinline__ uint32_t byte_of(const uint4& v, uint32_t k) {
    const uint32_t w = k < 8 ? (k < 4 ? v.x : v.y) : (k < 12 ? v.z : v.w);
    return (w >> ((k & 3) * 8)) & 0xFFu;
}

__global__ __launch_bounds__(RW_NT) void k_rows(const TileDesc* __restrict__ dt, uint32_t ndt,
                                                uint8_t* __restrict__ stream) {
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const uint32_t ti = upper_index(ndt, b, [&](uint32_t i) { return dt[i].blk_first; });
    const TileDesc d = dt[ti];
    const uint32_t fb = (d.flags & TF_PNGROWS) ? 1u : 0u;
    const uint32_t rowlen = d.rowlen, len = (uint32_t)d.stream_len;
    const uint32_t nwords = (len + 15) >> 4;
    Rows16 R;
    R.rb = rowlen - fb;
    R.bpp = d.bpp;
    R.swap = (d.flags & TF_SWAP) != 0;
    R.flip = (d.flags & TF_FLIP) != 0;
    const uint8_t* src0 = d.plane + (int64_t)d.y * d.pitch + (int64_t)d.x * d.bpp;
    uint8_t* out = stream + d.out_off;
    const uint32_t w0 = (b - d.blk_first) * ROWS_WORDS_PER_BLOCK;
#pragma unroll
    for (int j = 0; j < RW_WPT; j++) {
        const uint32_t wi = w0 + (uint32_t)j * RW_NT + tid;
        if (wi >= nwords) break;
        const uint32_t o = wi << 4;
        const uint32_t r = o / rowlen, c = o - r * rowlen;
        R.row = src0 + (int64_t)r * d.pitch;
        const uint4 x1 = R.fetch((int32_t)c - (int32_t)fb);
        uint4 v = x1;
        if (c < fb || c + 16 > rowlen || o + 16 > len) {
            // filter byte at the row start, or the word runs into the next row / the end
            uint4 x2 = make_uint4(0, 0, 0, 0);
            const bool next = c + 16 > rowlen && r + 1 < (uint32_t)d.h;
            if (next) {
                Rows16 R2 = R;
                R2.row = R.row + d.pitch;
                x2 = R2.fetch((int32_t)c - (int32_t)rowlen - (int32_t)fb);
            }
            uint32_t wv[4] = {0, 0, 0, 0};
#pragma unroll
            for (uint32_t k = 0; k < 16; k++) {
                const uint32_t p = c + k;
                uint32_t byte = 0;
                if (o + k < len) {
                    if (p < rowlen) byte = p < fb ? 0u : byte_of(x1, k);
                    else byte = (p - rowlen) < fb ? 0u : byte_of(x2, k);
                }
                wv[k >> 2] |= byte << ((k & 3) * 8);
            }
            v = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        }
        *(uint4*)(out + o) = v;
    }
}

hipError_t launch_rows(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles, uint32_t nblocks,
                       uint8_t* stream) {
    if (!ntiles || !nblocks) return hipSuccess;
    hipLaunchKernelGGL(k_rows, dim3(nblocks), dim3(RW_NT), 0, st, d_tiles, ntiles, stream);
    return hipGetLastError();
}

hipError_t launch_filter(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                         uint32_t nblocks, uint8_t* stream) {
    if (!ntiles || !nblocks) return hipSuccess;
    hipLaunchKernelGGL(k_filter, dim3(nblocks), dim3(256), FB_LDS, st, d_tiles, ntiles, stream);
    return hipGetLastError();
}

uint32_t filter_band_rows() { return FB_ROWS; }

}  // namespace pbx
