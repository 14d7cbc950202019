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

#include <mutex>
#include <type_traits>

#include "dev_util.h"
#include "pbx_common.h"
#include "pbx_kernels.h"

namespace pbx {

// The tile of a workgroup: the scalar binary search (descriptor keys through the scalar cache)
// or, with -DPBX_IO_WAVE_SEARCH, the 64-probe wave search (upper_index_wave: 2 rounds of
// vector gathers for 4096 tiles) -- measured slower (profiles/r06f/).
#ifdef PBX_IO_WAVE_SEARCH
#define PBX_IO_UPPER_INDEX upper_index_wave
#else
#define PBX_IO_UPPER_INDEX upper_index
#endif

// ------------------------------------------------------------------- synthetic planes
// Rows [y0, y0 + rows) of the plane (a row band, or the whole plane), row y0 at `out`.
__global__ __launch_bounds__(256) void k_gen_plane(uint8_t* __restrict__ out, int64_t pitch,
                                                   int32_t sx, int32_t y0, int32_t rows, int32_t pt,
                                                   int32_t bpp, int32_t kind, uint64_t seed,
                                                   int32_t plane_no, int32_t z, int32_t c, int32_t t) {
    const uint64_t total = (uint64_t)sx * (uint64_t)rows;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += stride) {
        const uint64_t r = idx / (uint64_t)sx, x = idx - r * (uint64_t)sx;
        const uint64_t v = gen_sample(kind, seed, plane_no, z, c, t, pt, (int64_t)x, (int64_t)y0 + (int64_t)r);
        uint8_t* p = out + (int64_t)r * pitch + (int64_t)x * bpp;
        switch (bpp) {
        case 1: *p = (uint8_t)v; break;
        case 2: *(uint16_t*)p = (uint16_t)v; break;
        case 4: *(uint32_t*)p = (uint32_t)v; break;
        default: *(uint64_t*)p = v; break;
        }
    }
}

// ------------------------------------------------------------------ resolution pyramid
// One level of the on-GPU pyramid (the levels PixelBuffer.setResolutionLevel
// selects, TileRequestHandler.java:89-91): out(x, y) = mean of in(2x..2x+1, 2y..2y+1), the
// last column / row repeated when the input size is odd.  Integers: (sum + 2) >> 2 on the
// exact 64-bit sum (arithmetic shift for signed types: floor((sum + 2) / 4)); float/double:
// ((a + b) + (c + d)) * 0.25 in the sample's precision.
template <class T>
__device__ __forceinline__ T ds_swap(T v, bool be) {
    if constexpr (sizeof(T) == 1) {
        return v;
    } else if constexpr (sizeof(T) == 2) {
        if (!be) return v;
        const uint16_t u = __builtin_bit_cast(uint16_t, v);
        return __builtin_bit_cast(T, (uint16_t)((u >> 8) | (u << 8)));
    } else if constexpr (sizeof(T) == 4) {
        return be ? __builtin_bit_cast(T, __builtin_bswap32(__builtin_bit_cast(uint32_t, v))) : v;
    } else {
        return be ? __builtin_bit_cast(T, __builtin_bswap64(__builtin_bit_cast(uint64_t, v))) : v;
    }
}

template <class T>
__device__ __forceinline__ T ds_mean4(T a, T b, T c, T d) {
    if constexpr (std::is_floating_point<T>::value) {
        return ((a + b) + (c + d)) * (T)0.25;
    } else {
        const int64_t s = (int64_t)a + (int64_t)b + (int64_t)c + (int64_t)d;
        return (T)((s + 2) >> 2);
    }
}

// One level: a thread makes DS_G groups of N = 8 / sizeof(T) output samples of a row, each
// from one aligned 16-byte load per input row (input rows are 256-aligned, so group g starts
// at byte 16 g), all loads issued before the means; whole groups are stored as one 8-byte
// (DS_G = 1) or 16-byte (DS_G = 2) word; the last, partial group of a row goes sample by sample.
#ifndef PBX_DS_G
#define PBX_DS_G 1  // (2: 0.684, with nontemporal loads 0.652; profiles/r06zg/)
#endif
#ifndef PBX_DS_NT
#define PBX_DS_NT 1  // bit 0: nontemporal loads, bit 1: nontemporal stores (1: 0.697 -> 0.768 of HBM peak, profiles/r06zg/)
#endif
constexpr int DS_G = PBX_DS_G;
template <class T>
__global__ __launch_bounds__(256) void k_downsample(const uint8_t* __restrict__ src, int64_t spitch,
                                                    int32_t sx, int32_t sy, uint8_t* __restrict__ dst,
                                                    int64_t dpitch, int32_t dx, int32_t dy, bool be) {
    constexpr int N = 8 / sizeof(T);
    const uint64_t ngx = ((uint64_t)dx + N * DS_G - 1) / (N * DS_G), total = ngx * (uint64_t)dy;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int32_t y = (int32_t)(i / ngx), sg = (int32_t)(i - (uint64_t)y * ngx);
        const int32_t y0 = 2 * y, y1 = 2 * y + 1 < sy ? 2 * y + 1 : sy - 1;
        const uint8_t* r0 = src + (int64_t)y0 * spitch;
        const uint8_t* r1 = src + (int64_t)y1 * spitch;
        const int32_t g0 = sg * DS_G;
        T* out = (T*)(dst + (int64_t)y * dpitch) + g0 * N;
        if (2 * (g0 + DS_G) * N <= sx) {
            uint4 va[DS_G], vb[DS_G];
#pragma unroll
            for (int k = 0; k < DS_G; k++) {
                va[k] = (PBX_DS_NT & 1) ? gload16_nt(r0 + 16 * (g0 + k)) : gload16(r0 + 16 * (g0 + k));
                vb[k] = (PBX_DS_NT & 1) ? gload16_nt(r1 + 16 * (g0 + k)) : gload16(r1 + 16 * (g0 + k));
            }
            T m[N * DS_G];
#pragma unroll
            for (int k = 0; k < DS_G; k++) {
                T a[2 * N], b[2 * N];
                __builtin_memcpy(a, &va[k], 16);
                __builtin_memcpy(b, &vb[k], 16);
#pragma unroll
                for (int j = 0; j < N; j++)
                    m[k * N + j] = ds_swap(ds_mean4(ds_swap(a[2 * j], be), ds_swap(a[2 * j + 1], be),
                                                    ds_swap(b[2 * j], be), ds_swap(b[2 * j + 1], be)), be);
            }
            if constexpr (DS_G == 2) {
                uint4 w;
                __builtin_memcpy(&w, m, 16);
                if (PBX_DS_NT & 2) gstore16_nt(out, w);
                else gstore16(out, w);
            } else {
                uint2 w;
                __builtin_memcpy(&w, m, 8);
                *(uint2*)out = w;
            }
        } else {
            for (int32_t j = 0; j < N * DS_G && g0 * N + j < dx; j++) {
                const int32_t xa = 2 * (g0 * N + j), xb = xa + 1 < sx ? xa + 1 : sx - 1;
                const T* p0 = (const T*)r0;
                const T* p1 = (const T*)r1;
                out[j] = ds_swap(ds_mean4(ds_swap(p0[xa], be), ds_swap(p0[xb], be), ds_swap(p1[xa], be),
                                          ds_swap(p1[xb], be)), be);
            }
        }
    }
}

hipError_t launch_downsample(hipStream_t st, const uint8_t* src, int64_t spitch, int32_t sx, int32_t sy,
                             uint8_t* dst, int64_t dpitch, int32_t dx, int32_t dy, int32_t pixel_type,
                             bool be) {
    static const int bpps[PT_N] = {1, 1, 2, 2, 4, 4, 4, 8};
    const uint64_t n = 8 / bpps[pixel_type] * DS_G;
    const uint64_t total = ((uint64_t)dx + n - 1) / n * (uint64_t)dy;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (!blocks) return hipSuccess;
    const dim3 g((uint32_t)blocks), b(256);
    switch (pixel_type) {
    case PT_INT8: hipLaunchKernelGGL(k_downsample<int8_t>, g, b, 0, st, src, spitch, sx, sy, dst, dpitch, dx, dy, be); break;
    case PT_UINT8: hipLaunchKernelGGL(k_downsample<uint8_t>, g, b, 0, st, src, spitch, sx, sy, dst, dpitch, dx, dy, be); break;
    case PT_INT16: hipLaunchKernelGGL(k_downsample<int16_t>, g, b, 0, st, src, spitch, sx, sy, dst, dpitch, dx, dy, be); break;
    case PT_UINT16: hipLaunchKernelGGL(k_downsample<uint16_t>, g, b, 0, st, src, spitch, sx, sy, dst, dpitch, dx, dy, be); break;
    case PT_INT32: hipLaunchKernelGGL(k_downsample<int32_t>, g, b, 0, st, src, spitch, sx, sy, dst, dpitch, dx, dy, be); break;
    case PT_UINT32: hipLaunchKernelGGL(k_downsample<uint32_t>, g, b, 0, st, src, spitch, sx, sy, dst, dpitch, dx, dy, be); break;
    case PT_FLOAT: hipLaunchKernelGGL(k_downsample<float>, g, b, 0, st, src, spitch, sx, sy, dst, dpitch, dx, dy, be); break;
    default: hipLaunchKernelGGL(k_downsample<double>, g, b, 0, st, src, spitch, sx, sy, dst, dpitch, dx, dy, be); break;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------ extraction
// UA: the batch holds regions whose rows are not whole 16-byte words at 16-byte aligned
// sources (the host knows: x * bpp and w * bpp mod 16); without them the kernel is the aligned
// path alone (22 VGPRs instead of 54: configs[3]'s all-aligned pass read 5.29 TB/s with the
// unaligned path compiled in, 5.48 without, profiles/r06j/).
template <bool UA>
__global__ __launch_bounds__(256) void k_extract(const TileDesc* __restrict__ ft, uint32_t nft,
                                                 uint8_t* __restrict__ out) {
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const uint32_t ti = PBX_IO_UPPER_INDEX(nft, b, [&](uint32_t i) { return ft[i].blk_first; });
    const TileDesc d = ft[ti];
    const uint32_t rb = (uint32_t)d.w * (uint32_t)d.bpp;
    const uint32_t r0 = (b - d.blk_first) * d.rows_per_blk;
    const uint32_t r1 = r0 + d.rows_per_blk < (uint32_t)d.h ? r0 + d.rows_per_blk : (uint32_t)d.h;
    uint8_t* base = out + d.out_off;
    if ((d.flags & (TF_TIFF | TF_TILED)) == TF_TIFF) {  // tiled: header by k_tiff_tiled
        if (r0 == 0 && tid == 0)
            write_tiff_header(base, d.w, d.h, d.bpp, tiff_sample_format(d.pixel_type), 1, rb * d.h);
        base += TIFF_DATA_OFFSET;
    }
    const uint8_t* src0 = d.plane + (int64_t)d.y * d.pitch + (int64_t)d.x * d.bpp;
    // padded edge sub-tiles of a tiled TIFF go byte by byte (zeros outside the region)
    const bool fast = !d.vw && (((uintptr_t)src0 | (uintptr_t)base | (uintptr_t)d.pitch | rb) & 15u) == 0;
    const bool swap = (d.flags & TF_SWAP) != 0;
    if (fast) {
        // EXT_U loads per thread in flight before their stores (a block's ~16 KiB of rows is
        // one round: 4 KiB per wave in flight instead of 1)
#ifndef PBX_EXT_U
#define PBX_EXT_U 8  // all-aligned batches (k_extract<false>): configs[3] 5.29 -> 5.61 TB/s over 4 (profiles/r06r/)
#endif
#ifndef PBX_EXT_U_UA
#define PBX_EXT_U_UA 4  // k_extract<true>: 8 here costs its unaligned path 10% (registers)
#endif
        constexpr uint32_t EXT_U = UA ? PBX_EXT_U_UA : PBX_EXT_U;
#ifndef PBX_EXT_NT
#define PBX_EXT_NT 3  // bit 0: nontemporal loads, bit 1: nontemporal stores (both: the headline grid
                      // 5.55 -> 6.03-6.15 TB/s aligned, configs[4] 549k -> 570k tiles/s, profiles/r06zb/)
#endif
        const uint32_t n16 = rb >> 4, nv = (r1 - r0) * n16;
        for (uint32_t i0 = tid; i0 < nv; i0 += 256 * EXT_U) {
            uint4 q[EXT_U];
#pragma unroll
            for (uint32_t k = 0; k < EXT_U; k++) {
                const uint32_t i = i0 + 256 * k, r = r0 + i / n16, v = i - (i / n16) * n16;
                if (i < nv) q[k] = (PBX_EXT_NT & 1) ? gload16_nt(src0 + (int64_t)r * d.pitch + 16 * v)
                                                    : gload16(src0 + (int64_t)r * d.pitch + 16 * v);
            }
#pragma unroll
            for (uint32_t k = 0; k < EXT_U; k++) {
                const uint32_t i = i0 + 256 * k, r = r0 + i / n16, v = i - (i / n16) * n16;
                if (i >= nv) break;
                if (swap) q[k] = swap16(q[k], d.bpp);
                if (PBX_EXT_NT & 2) gstore16_nt(base + (size_t)r * rb + 16 * v, q[k]);
                else gstore16(base + (size_t)r * rb + 16 * v, q[k]);
            }
        }
    } else if (UA && !d.vw && rb >= 16) {
        // Any other region (x * bpp not a multiple of 16, or rows of a length that is not): the
        // output is one contiguous run of (r1 - r0) * rb bytes at a 16-byte aligned base, so
        // every whole 16-byte output word of this block is built from 16 source bytes loaded
        // as two aligned words and funnel-shifted (gload16u).  Its bytes lie in row r from
        // column c on, and -- when fewer than 16 remain in the row -- in row r + 1 from column
        // 0: that part is loaded from n1 bytes before row r + 1's start and merged by a byte
        // mask.  Rows hold whole samples and c is a multiple of bpp (16 and rb are), so the
        // byte swap is swap16 on the assembled word.  The up-to-15 bytes at each end of the
        // block's run share an output word with the neighbouring block: written singly.
        const uint32_t f0 = r0 * rb, f1 = r1 * rb;
        const uint32_t w0 = (f0 + 15) >> 4, w1 = f1 >> 4;
        // EXTU_U words per thread in flight; a lane's upper source word comes from its right
        // neighbour (uload_*), the second row's part of a row-crossing word by its own loads
#ifndef PBX_EXTU_U
#define PBX_EXTU_U 2
#endif
        constexpr uint32_t U = PBX_EXTU_U;
        for (uint32_t wb = w0 + tid; wb < w1; wb += 256 * U) {
            ULoad a[U];
            uint4 q2[U];
            uint32_t n1[U];
#pragma unroll
            for (uint32_t k = 0; k < U; k++) {
                const uint32_t wi = wb + 256 * k;
                if (wi >= w1) break;  // (the lanes past the end leave the later rounds together)
                const uint32_t o = wi << 4, r = o / rb, c = o - r * rb;
                n1[k] = rb - c;
                uload_issue<(PBX_EXT_NT & 1) != 0>(a[k], src0 + (int64_t)r * d.pitch + c);
                // the word runs into row r + 1: loaded from n1 bytes before that row's start
                if (n1[k] < 16) q2[k] = gload16u(src0 + (int64_t)(r + 1) * d.pitch - n1[k]);
            }
#pragma unroll
            for (uint32_t k = 0; k < U; k++) {
                const uint32_t wi = wb + 256 * k;
                if (wi >= w1) break;
                uint4 q = uload_finish(a[k]);
                if (n1[k] < 16) {
                    const uint32_t n = n1[k];
                    auto keep = [&](uint32_t j) {  // bytes of word j that come from row r
                        return n >= 4 * j + 4 ? 0xFFFFFFFFu : n <= 4 * j ? 0u : (1u << (8 * (n - 4 * j))) - 1u;
                    };
                    const uint32_t m0 = keep(0), m1 = keep(1), m2 = keep(2), m3 = keep(3);
                    q.x = (q.x & m0) | (q2[k].x & ~m0);
                    q.y = (q.y & m1) | (q2[k].y & ~m1);
                    q.z = (q.z & m2) | (q2[k].z & ~m2);
                    q.w = (q.w & m3) | (q2[k].w & ~m3);
                }
                if (swap) q = swap16(q, d.bpp);
                if (PBX_EXT_NT & 2) gstore16_nt(base + (wi << 4), q);
                else gstore16(base + (wi << 4), q);
            }
        }
        const uint32_t h_end = f1 < (w0 << 4) ? f1 : (w0 << 4);
        const uint32_t t_beg = (w1 << 4) > h_end ? (w1 << 4) : h_end;
        const uint32_t i = tid < 16 ? f0 + tid : t_beg + (tid - 16);
        if (tid < 32 && (tid < 16 ? i < h_end : i < f1)) {
            TileStream ts;
            ts.init(d, nullptr);
            const uint32_t r = i / rb, c = i - r * rb;
            base[i] = (uint8_t)ts.be(r, c);
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
// sign flip), choose each row's filter (adaptive mode: minimum sum of |byte - prediction|,
// one wave per row), then write the band's stream bytes as aligned 16-byte words:
// FB_ROWS * rowlen is a multiple of 16, so bands never share an output word.
constexpr int FB_ROWS = 16;
constexpr int FB_LDS = 64 * 1024;

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

// The byte a filter predicts (0 for None); the adaptive choice sums |cur - prediction| (the
// plain byte distance, v_sad_u8) over the row and takes the minimum, the first on ties.
__device__ __forceinline__ uint32_t filt_pred(int ft, uint32_t left, uint32_t up, uint32_t ul) {
    switch (ft) {
    case 0: return 0u;
    case 1: return left;
    case 2: return up;
    case 3: return (left + up) >> 1;
    default: {
        const int p = (int)left + (int)up - (int)ul;
        const int pa = abs(p - (int)left), pb = abs(p - (int)up), pc = abs(p - (int)ul);
        return (pa <= pb && pa <= pc) ? left : (pb <= pc ? up : ul);
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
    const uint32_t ti = PBX_IO_UPPER_INDEX(ndt, b, [&](uint32_t i) { return dt[i].blk_first; });
    const TileDesc d = dt[ti];
    if (d.flags & TF_DIRECT) return;  // an adaptive tile in the None mode: k_lz77 reads the plane
    const uint32_t r0 = (b - d.blk_first) * FB_ROWS;
    const uint32_t r1 = r0 + FB_ROWS < (uint32_t)d.h ? r0 + FB_ROWS : (uint32_t)d.h;
    const uint32_t bpp = d.bpp, rb = (uint32_t)d.w * bpp, rowlen = d.rowlen;
    const bool png = (d.flags & TF_PNGROWS) != 0;
    uint8_t* out = stream + d.out_off;
    const uint8_t* src0 = d.plane + (int64_t)d.y * d.pitch + (int64_t)d.x * bpp;
    const uint32_t rbp = ((rb + 15) & ~15u) + 16;
    uint32_t* ftype = (uint32_t*)(sm + FB_LDS - 256);
    // (source rows of any alignment: gload16u; the pitch of every plane, band and bridge is a
    // multiple of 256)
    const bool fast = !d.vw && (uint64_t)(FB_ROWS + 1) * rbp + 256 <= (uint64_t)FB_LDS;
    const uint32_t o0 = r0 * rowlen, o1 = r1 * rowlen;
    if (fast) {
        const uint32_t nq = r1 - r0 + 1, nc = (rb + 15) >> 4;
        const bool swap = (d.flags & TF_SWAP) != 0, flip = (d.flags & TF_FLIP) != 0;
        for (uint32_t i = tid; i < nq * nc; i += 256) {
            const uint32_t q = i / nc, c = i - q * nc;
            const int64_t row = (int64_t)r0 - 1 + q;
            // (every lane loads -- the row above the tile's first row from row 0, then zeroed --
            // so the realigned loads can share words between neighbouring lanes)
            ULoad u;
            uload_issue(u, src0 + (row >= 0 ? row : 0) * d.pitch + 16 * c);
            uint4 v = uload_finish(u);
            if (swap) v = swap16(v, bpp);
            if (png && flip) v = flip_msb(v, bpp);
            if (row < 0) v = make_uint4(0, 0, 0, 0);
            *(uint4*)(sm + q * rbp + 16 * c) = v;
        }
        __syncthreads();
        if (png && d.filter == 5) {  // (tile mode None: every ftype 0, sums unused)
            for (uint32_t q = 1 + wv; q < nq; q += 4) {
                const uint8_t* L = sm + q * rbp;
                const uint8_t* U = L - rbp;
                uint32_t sum[5] = {0, 0, 0, 0, 0};
                for (uint32_t i = lane; i < rb; i += 64) {
                    const uint32_t cur = L[i], up = U[i];
                    const uint32_t left = i >= bpp ? L[i - bpp] : 0u, ul = i >= bpp ? U[i - bpp] : 0u;
#pragma unroll
                    for (int f = 0; f < 5; f++)
                        sum[f] += (uint32_t)abs((int)cur - (int)filt_pred(f, left, up, ul));
                }
#pragma unroll
                for (int f = 0; f < 5; f++)
#pragma unroll
                    for (int off = 32; off > 0; off >>= 1) sum[f] += __shfl_xor(sum[f], off, 64);
                if (lane == 0) ftype[q - 1] = (d.flags & TF_ANONE) ? 0u : block_min_filter(sum, nullptr, 0);
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
                        sum[f] += (uint32_t)abs((int)cur - (int)filt_pred(f, left, up, ul));
                }
                for (int f = 0; f < 5; f++) atomicAdd(&red[f], sum[f]);
                __syncthreads();
                if (tid == 0) {
                    int best = 0;
                    for (int f = 1; f < 5; f++) if (red[f] < red[best]) best = f;
                    ftype[r - r0] = (d.flags & TF_ANONE) ? 0u : (uint32_t)best;
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

// ------------------------------------------------------- adaptive filter: the tile mode
// The pbx_config.png_filter = adaptive option first asks, per tile, whether filtering pays at
// all (on microscope-like 16-bit data the per-row minimum-distance rule picks
// Sub/Paeth rows that deflate worse than the raw rows).  On the tile's middle row r* = h/2
// (row r* - 1 above it, zeros above the tile): the best of Sub/Up/Avg/Paeth by the sum of
// |byte - prediction| (the first on ties), then None against it by the sum, over the two byte
// planes (i mod bpp) & 1, of the squared counts of the row's byte values -- the larger, the
// more concentrated the bytes, the fewer bits; None wins ties.  TF_ANONE sends every row of
// the tile to None (k_filter / k_filter2 / k_filter3 read it), and on a tile the host marked
// TF_DIRECT_OK the kernel also sets TF_DIRECT: the filter kernels skip it and k_lz77 reads its
// rows from the plane.  The oracle's adaptive_tile_none (oracle/pbx_oracle.c) is the same
// rule.  One workgroup per tile: the two rows staged in LDS by 16-byte loads (k_filter's
// staging), then the sums and 4 KiB of byte counters from LDS (~25 us per 4096 tiles).
// rows_cap: LDS bytes for the two staged rows (the batch's widest adaptive row; wider ones
// read their bytes from the plane)
#ifndef PBX_AM_NT
#define PBX_AM_NT 128  // (256: 28.5 us per 4096 tiles, 128: 24.8, 64: 25.0; profiles/r06ze/)
#endif
constexpr uint32_t AM_NT = PBX_AM_NT;  // threads per tile
__global__ __launch_bounds__(AM_NT) void k_adaptive_mode(TileDesc* __restrict__ dt, uint32_t ndt,
                                                       uint32_t rows_cap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    uint32_t* cnt = (uint32_t*)sm;  // [candidate][byte plane][byte]
    uint8_t* rows = sm + 4096;
    __shared__ uint32_t red[4];
    __shared__ unsigned long long q2[2];
    const uint32_t t = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    if (t >= ndt) return;
    const TileDesc d = dt[t];
    if (d.filter != 5 || !(d.flags & TF_PNGROWS)) return;  // uniform: the whole workgroup
    TileStream ts;
    ts.init(d, nullptr);
    const uint32_t bpp = (uint32_t)d.bpp, rb = (uint32_t)d.w * bpp;
    const int64_t rs = d.h / 2;
    const uint32_t rbp = ((rb + 15) & ~15u) + 16;
    const bool staged = !d.vw && 2 * rbp <= rows_cap;
    for (uint32_t k = tid; k < 1024; k += AM_NT) cnt[k] = 0;
    if (tid < 4) red[tid] = 0;
    if (tid < 2) q2[tid] = 0;
    if (staged) {  // rows r* - 1 (zeros above the tile) and r*: k_filter's staging (any alignment)
        const uint32_t nc = (rb + 15) >> 4;
        const uint8_t* src0 = d.plane + (int64_t)d.y * d.pitch + (int64_t)d.x * bpp;
        const bool swap = (d.flags & TF_SWAP) != 0, flip = (d.flags & TF_FLIP) != 0;
        for (uint32_t i = tid; i < 2 * nc; i += AM_NT) {
            const uint32_t q = i / nc, c = i - q * nc;
            const int64_t row = rs - 1 + q;
            ULoad u;
            uload_issue(u, src0 + (row >= 0 ? row : 0) * d.pitch + 16 * c);
            uint4 v = uload_finish(u);
            if (swap) v = swap16(v, bpp);
            if (flip) v = flip_msb(v, bpp);
            if (row < 0) v = make_uint4(0, 0, 0, 0);
            *(uint4*)(rows + q * rbp + 16 * c) = v;
        }
    }
    __syncthreads();
    const uint8_t* U = rows;
    const uint8_t* L = rows + rbp;
    auto bytes = [&](uint32_t i, uint32_t& cur, uint32_t& left, uint32_t& up, uint32_t& ul) {
        if (staged) {
            cur = L[i];
            up = U[i];
            left = i >= bpp ? L[i - bpp] : 0u;
            ul = i >= bpp ? U[i - bpp] : 0u;
        } else {
            cur = ts.be(rs, i);
            up = rs > 0 ? ts.be(rs - 1, i) : 0u;
            left = i >= bpp ? ts.be(rs, i - bpp) : 0u;
            ul = (rs > 0 && i >= bpp) ? ts.be(rs - 1, i - bpp) : 0u;
        }
    };
    uint32_t sum[4] = {0, 0, 0, 0};
    for (uint32_t i = tid; i < rb; i += AM_NT) {
        uint32_t cur, left, up, ul;
        bytes(i, cur, left, up, ul);
#pragma unroll
        for (int f = 1; f < 5; f++) sum[f - 1] += (uint32_t)abs((int)cur - (int)filt_pred(f, left, up, ul));
    }
#pragma unroll
    for (int f = 0; f < 4; f++) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sum[f] += __shfl_xor(sum[f], off, 64);
        if (lane == 0) atomicAdd(&red[f], sum[f]);
    }
    __syncthreads();
    int fb = 1;
    for (int f = 2; f < 5; f++)
        if (red[f - 1] < red[fb - 1]) fb = f;
    for (uint32_t i = tid; i < rb; i += AM_NT) {
        uint32_t cur, left, up, ul;
        bytes(i, cur, left, up, ul);
        const uint32_t pl = (i & (bpp - 1)) & 1u;
        atomicAdd(&cnt[pl * 256 + cur], 1u);
        atomicAdd(&cnt[512 + pl * 256 + filt_byte(fb, cur, left, up, ul)], 1u);
    }
    __syncthreads();
    unsigned long long a = 0, b = 0;
    for (uint32_t k = tid; k < 512; k += AM_NT) {
        a += (unsigned long long)cnt[k] * cnt[k];
        b += (unsigned long long)cnt[512 + k] * cnt[512 + k];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off, 64);
        b += __shfl_xor(b, off, 64);
    }
    if (lane == 0) {
        atomicAdd(&q2[0], a);
        atomicAdd(&q2[1], b);
    }
    __syncthreads();
    if (tid == 0) {
        const bool none = rb > 0 && d.h > 0 && q2[0] >= q2[1];
        const uint32_t f = d.flags & ~(TF_ANONE | TF_DIRECT);
        dt[t].flags = none ? (f | TF_ANONE | ((d.flags & TF_DIRECT_OK) ? TF_DIRECT : 0u)) : f;
    }
}

hipError_t launch_adaptive_mode(hipStream_t st, TileDesc* d_tiles, uint32_t ntiles, uint32_t max_rb) {
    if (!ntiles) return hipSuccess;
    // the two rows of the widest tile in LDS, up to 2 x 16 KiB (+ 4 KiB of counters): small
    // workgroups stay many to a CU
    const uint32_t rbp = ((max_rb + 15) & ~15u) + 16;
    const uint32_t rows_cap = 2 * rbp <= 32768u ? 2 * rbp : 0u;
    hipLaunchKernelGGL(k_adaptive_mode, dim3(ntiles), dim3(AM_NT), 4096 + rows_cap, st, d_tiles, ntiles, rows_cap);
    return hipGetLastError();
}

// ------------------------------------------------------------- tiled-TIFF headers
// One workgroup per tiled-TIFF response: header, IFD and the TileOffsets / TileByteCounts
// arrays (TIFF 6.0 section 15).  Uncompressed sub-tiles all hold t*t*bpp bytes; deflate
// sub-tiles k are the containers [offs[first+k], offs[first+k+1]) of the deflate arena, the
// first one preceded by the header.
__global__ __launch_bounds__(256) void k_tiff_tiled(const TiledHdr* __restrict__ th, uint32_t nth,
                                                    uint8_t* __restrict__ fixed,
                                                    const uint64_t* __restrict__ offs,
                                                    uint8_t* __restrict__ zout) {
    const TiledHdr j = th[blockIdx.x];
    const uint32_t tid = threadIdx.x;
    const uint64_t D = tiff_tiled_data_offset(j.n);
    const uint64_t sub = (uint64_t)j.t * j.t * j.bpp;
    uint8_t* p = j.comp == 1 ? fixed + j.off : zout + offs[j.first];
    auto entry = [&](uint32_t k, uint32_t& off, uint32_t& cnt) {
        if (j.comp == 1) {
            off = (uint32_t)(D + k * sub);
            cnt = (uint32_t)sub;
        } else {
            const uint64_t a = offs[j.first + k] - offs[j.first], e = offs[j.first + k + 1] - offs[j.first];
            off = (uint32_t)(k ? a : D);
            cnt = (uint32_t)(e - off);
        }
    };
    if (tid == 0) {
        uint32_t off0, cnt0;
        entry(0, off0, cnt0);
        write_tiff_tiled_ifd(p, j.w, j.h, j.t, j.bpp, j.sf, j.comp, j.n, off0, cnt0);
    }
    if (j.n > 1) {
        for (uint32_t k = tid; k < j.n; k += 256) {
            uint32_t off, cnt;
            entry(k, off, cnt);
            tiff_tiled_entry(p, j.n, k, off, cnt);
        }
        for (uint64_t i = TIFF_TILED_ARRAYS + 8ull * j.n + tid; i < D; i += 256) p[i] = 0;
    }
}

// ------------------------------------------------------------------------ launchers
hipError_t launch_tiff_tiled(hipStream_t st, const TiledHdr* d_th, uint32_t nth, uint8_t* fixed,
                             const uint64_t* offs, uint8_t* zout) {
    if (!nth) return hipSuccess;
    hipLaunchKernelGGL(k_tiff_tiled, dim3(nth), dim3(256), 0, st, d_th, nth, fixed, offs, zout);
    return hipGetLastError();
}

hipError_t launch_gen_plane(hipStream_t st, uint8_t* out, int64_t pitch, int32_t sx, int32_t y0,
                            int32_t rows, int32_t pt, int32_t kind, uint64_t seed, int32_t plane_no,
                            int32_t z, int32_t c, int32_t t) {
    static const int bpps[PT_N] = {1, 1, 2, 2, 4, 4, 4, 8};
    const uint64_t total = (uint64_t)sx * (uint64_t)rows;
    uint64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gen_plane, dim3((uint32_t)blocks), dim3(256), 0, st, out, pitch, sx, y0, rows, pt,
                       bpps[pt], kind, seed, plane_no, z, c, t);
    return hipGetLastError();
}

hipError_t launch_extract(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                          uint32_t nblocks, uint8_t* out, bool unaligned) {
    if (!ntiles || !nblocks) return hipSuccess;
#ifdef PBX_EXT_ALWAYS_UA  // A/B: every batch through the instantiation with the unaligned path
    unaligned = true;
#endif
    if (unaligned)
        hipLaunchKernelGGL(k_extract<true>, dim3(nblocks), dim3(256), 0, st, d_tiles, ntiles, out);
    else
        hipLaunchKernelGGL(k_extract<false>, dim3(nblocks), dim3(256), 0, st, d_tiles, ntiles, out);
    return hipGetLastError();
}

// ------------------------------------------------------- test hook: a batch that never completes
// pbx_test_stall_batch: one wave spins on a flag in mapped pinned host memory until the host
// clears it, or until `limit` ticks of the constant 100 MHz clock (s_memrealtime) have passed,
// so the spin always ends on its own.  The batch's kernels queue behind it on its stream: to
// its callers the batch is a wedged device (the reference's event-bus send timeout,
// PixelBufferMicroserviceVerticle.java:148-151,352-366).
__global__ void k_stall(const uint32_t* flag, uint64_t limit) {
    const uint64_t t0 = wall_clock64();
    for (;;) {
        const uint32_t v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v == 0 || wall_clock64() - t0 >= limit) break;
        __builtin_amdgcn_s_sleep(127);
    }
}

hipError_t launch_stall(hipStream_t st, const uint32_t* flag, uint64_t limit_ticks) {
    hipLaunchKernelGGL(k_stall, dim3(1), dim3(64), 0, st, flag, limit_ticks);
    return hipGetLastError();
}

// ------------------------------------------------------- K1+K2 fast rows (filter None)
// The stream of a filter-None PNG tile is row r = [0] ++ big-endian row bytes, and of a
// deflate-TIFF tile the row bytes alone.  One workgroup per band of RB_ROWS rows (whose
// stream bytes start and end 16-byte aligned, as RB_ROWS * rowlen is a multiple of 16):
// the band's source rows are loaded once as 16-byte words (realigned in registers when the
// region's x * bpp is not a multiple of 16; byte swap and sign flip applied there, where the
// sample boundaries are known) into LDS rows padded to
// 16 bytes, then every aligned 16-byte stream word is assembled from 5 LDS words with
// funnel shifts; the few words that straddle a row end merge two rows with byte masks.
constexpr int RB_NT = 256;
constexpr uint32_t RB_ROWS = 16;

__device__ __forceinline__ uint32_t lds_word4(const uint32_t* rowp, int32_t s, uint32_t i) {
    // dword i of the 16 bytes of an LDS row starting at byte s (s >= -17): bytes before the
    // row come from the previous row or the pad and are only ever masked out
    const int32_t b = s + 4 * (int32_t)i;
    const int32_t wdx = b >> 2;  // floor
    const uint32_t w0 = rowp[wdx], w1 = rowp[wdx + 1];
    return __builtin_amdgcn_alignbit(w1, w0, (uint32_t)(b & 3) * 8);
}

// bytes [lo, hi) of dword i (byte index within the 16-byte word) as a mask
__device__ __forceinline__ uint32_t byte_mask(int32_t lo, int32_t hi, uint32_t i) {
    const int32_t a = lo - 4 * (int32_t)i, b = hi - 4 * (int32_t)i;
    const uint32_t ma = a <= 0 ? 0xFFFFFFFFu : a >= 4 ? 0u : (0xFFFFFFFFu << (8 * a));
    const uint32_t mb = b >= 4 ? 0xFFFFFFFFu : b <= 0 ? 0u : (0xFFFFFFFFu >> (8 * (4 - b)));
    return ma & mb;
}

__global__ __launch_bounds__(RB_NT) void k_rows(const TileDesc* __restrict__ dt, uint32_t ndt,
                                                uint8_t* __restrict__ stream) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lrow[];
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const uint32_t ti = PBX_IO_UPPER_INDEX(ndt, b, [&](uint32_t i) { return dt[i].blk_first; });
    const TileDesc d = dt[ti];
    const uint32_t fb = (d.flags & TF_PNGROWS) ? 1u : 0u;
    const uint32_t rowlen = d.rowlen, rb = rowlen - fb, bpp = d.bpp;
    const uint32_t nc = (rb + 15) >> 4;          // 16-byte chunks per row
    const uint32_t rw = 4 * nc + 4;               // LDS row stride in words (+16 B pad)
    const uint32_t r0 = (b - d.blk_first) * RB_ROWS;
    const uint32_t nr = (uint32_t)d.h - r0 < RB_ROWS ? (uint32_t)d.h - r0 : RB_ROWS;
    const bool swap = (d.flags & TF_SWAP) != 0, flip = (d.flags & TF_FLIP) != 0;
    const uint8_t* src0 = d.plane + (int64_t)(d.y + r0) * d.pitch + (int64_t)d.x * bpp;
    // 1. band rows -> LDS (row q at word 4 + q*rw: one pad word before row 0)
    uint32_t* rows = lrow + 4;
    for (uint32_t i = tid; i < nr * nc; i += RB_NT) {
        const uint32_t q = i / nc, c = i - q * nc;
        // (source rows of any alignment: realigned loads; 16 c is a sample boundary)
        ULoad u;
        uload_issue(u, src0 + (int64_t)q * d.pitch + 16 * c);
        uint4 v = uload_finish(u);
        if (swap) v = swap16(v, (int)bpp);
        if (flip) v = flip_msb(v, (int)bpp);
        *(uint4*)(rows + q * rw + 4 * c) = v;
    }
    __syncthreads();
    // 2. aligned stream words of the band
    const uint32_t o0 = r0 * rowlen, nb = nr * rowlen, nw = (nb + 15) >> 4;
    const uint32_t magic = 0xFFFFFFFFu / rowlen;
    uint8_t* out = stream + d.out_off + o0;
    for (uint32_t k = tid; k < nw; k += RB_NT) {
        const uint32_t o = k << 4;
        uint32_t r = __umulhi(o, magic);
        if ((r + 1) * rowlen <= o) r++;
        const uint32_t c = o - r * rowlen;
        const int32_t s = (int32_t)c - (int32_t)fb;  // data byte of row r at word byte 0
        const uint32_t* rp = rows + r * rw;
        uint32_t w[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) w[i] = lds_word4(rp, s, i);
        const int32_t k1 = (int32_t)rowlen - (int32_t)c;  // bytes of row r in this word
        if (s < 0 || k1 < 16 || o + 16 > nb) {
            // filter byte (row start) / next row's filter byte and data / band end
            const bool nxt = k1 < 16 && r + 1 < nr;
            const uint32_t* rq = rows + (r + 1) * rw;
            const int32_t s2 = s - (int32_t)rowlen;  // data byte of row r+1 at word byte 0
            const int32_t end = (int32_t)(nb - o) < 16 ? (int32_t)(nb - o) : 16;
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const uint32_t m1 = byte_mask((int32_t)fb - (int32_t)c > 0 ? 1 : 0, k1 < end ? k1 : end, i);
                uint32_t v = w[i] & m1;
                if (nxt) v |= lds_word4(rq, s2, i) & byte_mask(k1 + (int32_t)fb, end, i);
                w[i] = v;
            }
        }
        *(uint4*)(out + o) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

size_t rows_lds_bytes(uint32_t rb) { return 16 + (size_t)RB_ROWS * (4 * ((rb + 15) / 16) + 4) * 4; }

hipError_t launch_rows(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles, uint32_t nblocks,
                       uint32_t max_rb, uint8_t* stream) {
    if (!ntiles || !nblocks) return hipSuccess;
    const size_t lds = rows_lds_bytes(max_rb);
    if (lds > 64 * 1024) {
        // bands of rows over 4 KiB: allow up to 160 KiB of LDS.  The attribute belongs to the
        // current device, so it is raised once per device (thread-safe).
        constexpr int kMaxDev = 64;
        static std::once_flag once[kMaxDev];
        static hipError_t res[kMaxDev];
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
        std::call_once(once[dev], [&] {
            res[dev] = hipFuncSetAttribute((const void*)k_rows, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           160 * 1024);
        });
        if (res[dev] != hipSuccess) return res[dev];
    }
    hipLaunchKernelGGL(k_rows, dim3(nblocks), dim3(RB_NT), lds, st, d_tiles, ntiles, stream);
    return hipGetLastError();
}

hipError_t launch_filter(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles,
                         uint32_t nblocks, uint8_t* stream) {
    if (!ntiles || !nblocks) return hipSuccess;
    hipLaunchKernelGGL(k_filter, dim3(nblocks), dim3(256), FB_LDS, st, d_tiles, ntiles, stream);
    return hipGetLastError();
}

uint32_t filter_band_rows() { return FB_ROWS; }

// ------------------------------------------- K1+K2: PNG filters on 4-byte words
// PNG tiles with a Sub/Up/Avg/Paeth or adaptive filter and rows of whole dwords (w*bpp % 4
// == 0, <= F2_MAX_RB bytes; 16-byte aligned source rows): one 256-thread workgroup per
// band of F2_ROWS rows.
//   A  the band's rows and the row above, big-endian, into LDS (16-byte loads; 16 zero bytes
//      before every row: the left neighbours of its first samples)
//   B  (adaptive) each row's filter: one wave per row, the five sums of |byte - prediction|
//      over dwords, four bytes at once (SWAR byte arithmetic; v_sad_u8 on the biased bytes
//      gives sum |residual| in one instruction; Paeth on packed 16-bit pairs), minimum first
//   C  every filtered dword of the band into LDS rows laid out as k_rows' staging rows
//   D  the stream words (filter byte + filtered row), 16-byte aligned, assembled from the
//      filtered rows with funnel shifts exactly as k_rows does, the filter bytes OR-ed in.
// Output identical to k_filter's (the same per-row choice; tests compare both to the oracle).
constexpr uint32_t F2_ROWS = 16;
constexpr uint32_t F2_NT = 256;
constexpr uint32_t F2_MAX_RB = 2048;

__device__ __forceinline__ uint32_t sub8(uint32_t a, uint32_t b) {  // bytewise a - b mod 256
    return ((a | 0x80808080u) - (b & 0x7F7F7F7Fu)) ^ ((a ^ ~b) & 0x80808080u);
}
// (a - b) ^ 0x80 per byte: the residual biased by 128 (sub8's last xor folded into its mask)
__device__ __forceinline__ uint32_t sub8m(uint32_t a, uint32_t b) {
    return ((a | 0x80808080u) - (b & 0x7F7F7F7Fu)) ^ ((a ^ b) & 0x80808080u);
}
__device__ __forceinline__ uint32_t avg8(uint32_t a, uint32_t b) {  // bytewise floor((a + b) / 2)
    return __builtin_amdgcn_lerp(a, b, 0u);  // v_lerp_u8: (a + b + round bit 0) >> 1 per byte
}
typedef short f2_s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2_s16x2 f2_abs(f2_s16x2 x) {
    const f2_s16x2 m = x >> 15;
    return (x ^ m) - m;
}
// PNG Paeth predictor (a = left, b = up, c = up-left): pa = |b - c|, pb = |a - c|,
// pc = |a + b - 2c| (<= 510); a if pa <= min(pb, pc), else b if pb <= pc, else c.
// Computed in packed f16.  A byte x in a 16-bit lane with 0x64 above it is the f16
// value 1024 + x (exponent of [1024, 2048): unit steps), so every difference and sum the
// predictor forms (within +-510) is exact; |d| is one AND of the sign bits; the signs of
// (min(pb, pc) - pa) and (pc - pb) are the f16 sign bits (never -0: x - x = +0), spread over
// their lane by one v_pk_ashrrev_i16 each (in asm: the compiler otherwise rewrites the masked
// selects as per-lane compares and v_cndmask).  The lanes are built by ONE v_perm_b32 per
// pair (two bytes of a word and the 0x64 bias), and the two results recombined by one more.
// Checked against the integer rule for all 2^24 (a, b, c) byte triples.
typedef _Float16 f3_h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_sign_mask(uint32_t y) {  // 0xFFFF per negative 16-bit lane
    // The shift counts come from an SGPR holding 15 in BOTH halves: an inline constant 15
    // reaches only the low lane of a packed operand (the high lane then reads its bits 31:16,
    // 0, and was not shifted at all: wrong Paeth choices in bytes 2 and 3 on the GPU).
    uint32_t m;
    asm("v_pk_ashrrev_i16 %0, %1, %2" : "=v"(m) : "s"(0x000F000Fu), "v"(y));
    return m;
}
__device__ __forceinline__ uint32_t paeth_pair_h(uint32_t a, uint32_t b, uint32_t c) {  // biased lanes
    const f3_h2 A = __builtin_bit_cast(f3_h2, a), B = __builtin_bit_cast(f3_h2, b), C = __builtin_bit_cast(f3_h2, c);
    const f3_h2 d1 = B - C, d2 = A - C, d3 = d1 + d2;
    const f3_h2 pa = __builtin_elementwise_max(d1, -d1), pb = __builtin_elementwise_max(d2, -d2),
                pc = __builtin_elementwise_max(d3, -d3);
    const uint32_t na = pk_sign_mask(__builtin_bit_cast(uint32_t, (f3_h2)(__builtin_elementwise_min(pb, pc) - pa)));
    const uint32_t nb = pk_sign_mask(__builtin_bit_cast(uint32_t, (f3_h2)(pc - pb)));
    const uint32_t t = (nb & c) | (~nb & b);
    return (na & t) | (~na & a);  // na = -1: pa > min(pb, pc)
}
__device__ __forceinline__ uint32_t paeth4(uint32_t l, uint32_t u, uint32_t ul) {
    constexpr uint32_t BIAS = 0x64646464u, LO = 0x00060004u, HI = 0x00070005u;  // [b0|b1, 64, b2|b3, 64]
    const uint32_t rl = paeth_pair_h(__builtin_amdgcn_perm(l, BIAS, LO), __builtin_amdgcn_perm(u, BIAS, LO),
                                     __builtin_amdgcn_perm(ul, BIAS, LO));
    const uint32_t rh = paeth_pair_h(__builtin_amdgcn_perm(l, BIAS, HI), __builtin_amdgcn_perm(u, BIAS, HI),
                                     __builtin_amdgcn_perm(ul, BIAS, HI));
    return __builtin_amdgcn_perm(rh, rl, 0x06020400u);  // [rl.b0, rh.b0, rl.b2, rh.b2]
}
// the bytes bpp before each byte of word k: from words k and k-1 (k-2 for 8-byte samples)
__device__ __forceinline__ uint32_t back_bytes(const uint32_t* row, int32_t k, uint32_t bpp) {
    if (bpp >= 4) return row[k - (int32_t)(bpp >> 2)];
    return __builtin_amdgcn_alignbyte(row[k], row[k - 1], 4 - bpp);
}
__device__ __forceinline__ uint32_t filt_word(uint32_t ft, uint32_t cur, uint32_t left, uint32_t up, uint32_t ul) {
    switch (ft) {
    case 0: return cur;
    case 1: return sub8(cur, left);
    case 2: return sub8(cur, up);
    case 3: return sub8(cur, avg8(left, up));
    default: return sub8(cur, paeth4(left, up, ul));
    }
}

size_t filter2_lds_bytes(uint32_t max_rb) {
    const uint32_t rbq = (max_rb + 15) & ~15u;
    return (size_t)(F2_ROWS + 1) * (rbq + 32) + 16 + (size_t)F2_ROWS * (rbq + 16) + 64;
}

__global__ __launch_bounds__(F2_NT) void k_filter2(const TileDesc* __restrict__ dt, uint32_t ndt,
                                                  uint32_t rbq_max, uint8_t* __restrict__ stream) {
    extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
    const uint32_t b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t ti = PBX_IO_UPPER_INDEX(ndt, b, [&](uint32_t i) { return dt[i].blk_first; });
    const TileDesc d = dt[ti];
    if (d.flags & TF_DIRECT) return;  // an adaptive tile in the None mode: k_lz77 reads the plane
    const uint32_t r0 = (b - d.blk_first) * F2_ROWS;
    const uint32_t nr = (uint32_t)d.h - r0 < F2_ROWS ? (uint32_t)d.h - r0 : F2_ROWS;
    const uint32_t bpp = (uint32_t)d.bpp, rb = (uint32_t)d.w * bpp, nw = rb >> 2;
    const uint32_t nc = (rb + 15) >> 4, sst = rbq_max + 32;
    uint8_t* SA = sm;                                         // staged rows, slot q at SA + q*sst
    uint32_t* FR = (uint32_t*)(sm + (F2_ROWS + 1) * sst + 16);  // filtered rows (k_rows layout)
    const uint32_t rw = 4 * nc + 4;
    uint32_t* ftype = (uint32_t*)(sm + (F2_ROWS + 1) * sst + 16 + F2_ROWS * (rbq_max + 16));
    const bool swap = (d.flags & TF_SWAP) != 0, flip = (d.flags & TF_FLIP) != 0;
    const uint8_t* src0 = d.plane + (int64_t)d.y * d.pitch + (int64_t)d.x * bpp;
    // A: rows r0-1 .. r0+nr-1 (zeros above the tile)
    for (uint32_t i = tid; i < (nr + 1) * nc; i += F2_NT) {
        const uint32_t q = i / nc, c = i - q * nc;
        const int64_t row = (int64_t)r0 - 1 + q;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (row >= 0) {
            v = gload16(src0 + row * d.pitch + 16 * c);
            if (swap) v = swap16(v, (int)bpp);
            if (flip) v = flip_msb(v, (int)bpp);
        }
        *(uint4*)(SA + q * sst + 16 + 16 * c) = v;
    }
    for (uint32_t q = tid; q < nr + 1; q += F2_NT) *(uint4*)(SA + q * sst) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    // B: the adaptive choice, one wave per row
    if (d.filter == 5) {
        for (uint32_t q = 1 + wv; q <= nr; q += F2_NT / 64) {
            const uint32_t* L = (const uint32_t*)(SA + q * sst + 16);
            const uint32_t* U = (const uint32_t*)(SA + (q - 1) * sst + 16);
            uint32_t s[5] = {0, 0, 0, 0, 0};
            for (uint32_t k = (d.flags & TF_ANONE) ? nw : lane; k < nw; k += 64) {
                const uint32_t cur = L[k], up = U[k];
                const uint32_t left = back_bytes(L, (int32_t)k, bpp), ul = back_bytes(U, (int32_t)k, bpp);
                s[0] = __builtin_amdgcn_sad_u8(cur, 0u, s[0]);
                s[1] = __builtin_amdgcn_sad_u8(cur, left, s[1]);
                s[2] = __builtin_amdgcn_sad_u8(cur, up, s[2]);
                s[3] = __builtin_amdgcn_sad_u8(cur, avg8(left, up), s[3]);
                s[4] = __builtin_amdgcn_sad_u8(cur, paeth4(left, up, ul), s[4]);
            }
#pragma unroll
            for (int f = 0; f < 5; f++)
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) s[f] += __shfl_xor(s[f], off, 64);
            if (lane == 0) {
                uint32_t best = 0;
                for (uint32_t f = 1; f < 5; f++) if (s[f] < s[best]) best = f;
                ftype[q - 1] = (d.flags & TF_ANONE) ? 0u : best;  // the tile mode: None on every row
            }
        }
        __syncthreads();
    }
    // C: filtered dwords of every row
    for (uint32_t i = tid; i < nr * nw; i += F2_NT) {
        const uint32_t q = i / nw, k = i - q * nw;
        const uint32_t* L = (const uint32_t*)(SA + (q + 1) * sst + 16);
        const uint32_t* U = (const uint32_t*)(SA + q * sst + 16);
        const uint32_t ft = d.filter == 5 ? ftype[q] : (uint32_t)d.filter;
        FR[4 + q * rw + k] = filt_word(ft, L[k], back_bytes(L, (int32_t)k, bpp), U[k], back_bytes(U, (int32_t)k, bpp));
    }
    __syncthreads();
    // D: the band's stream words (k_rows' assembly, filter bytes OR-ed in)
    const uint32_t rowlen = d.rowlen;
    const uint32_t o0 = r0 * rowlen, nb = nr * rowlen, nwo = (nb + 15) >> 4;
    const uint32_t magic = 0xFFFFFFFFu / rowlen;
    uint8_t* out = stream + d.out_off + o0;
    const uint32_t* rows = FR + 4;
    for (uint32_t kk = tid; kk < nwo; kk += F2_NT) {
        const uint32_t o = kk << 4;
        uint32_t r = __umulhi(o, magic);
        if ((r + 1) * rowlen <= o) r++;
        const uint32_t c = o - r * rowlen;
        const int32_t s = (int32_t)c - 1;  // data byte of row r at word byte 0
        const uint32_t* rp = rows + r * rw;
        uint32_t w[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) w[i] = lds_word4(rp, s, i);
        const int32_t k1 = (int32_t)rowlen - (int32_t)c;  // bytes of row r in this word
        const int32_t end = (int32_t)(nb - o) < 16 ? (int32_t)(nb - o) : 16;
        const bool nxt = k1 < end && r + 1 < nr;
        if (s < 0 || k1 < 16 || o + 16 > nb) {
            const uint32_t* rq = rows + (r + 1) * rw;
            const int32_t s2 = s - (int32_t)rowlen;
#pragma unroll
            for (uint32_t i = 0; i < 4; i++) {
                const uint32_t m1 = byte_mask(c == 0 ? 1 : 0, k1 < end ? k1 : end, i);
                uint32_t v = w[i] & m1;
                if (nxt) v |= lds_word4(rq, s2, i) & byte_mask(k1 + 1, end, i);
                w[i] = v;
            }
        }
        if (c == 0) w[0] |= d.filter == 5 ? ftype[r] : (uint32_t)d.filter;
        if (nxt) w[k1 >> 2] |= (d.filter == 5 ? ftype[r + 1] : (uint32_t)d.filter) << (8 * (k1 & 3));
        *(uint4*)(out + o) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

hipError_t launch_filter2(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles, uint32_t nblocks,
                          uint32_t max_rb, uint8_t* stream) {
    if (!ntiles || !nblocks) return hipSuccess;
    const size_t lds = filter2_lds_bytes(max_rb);
    if (lds > 64 * 1024) {
        constexpr int kMaxDev = 64;
        static std::once_flag once[kMaxDev];
        static hipError_t res[kMaxDev];
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
        std::call_once(once[dev], [&] {
            res[dev] = hipFuncSetAttribute((const void*)k_filter2, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           160 * 1024);
        });
        if (res[dev] != hipSuccess) return res[dev];
    }
    hipLaunchKernelGGL(k_filter2, dim3(nblocks), dim3(F2_NT), lds, st, d_tiles, ntiles,
                       (max_rb + 15) & ~15u, stream);
    return hipGetLastError();
}

uint32_t filter2_band_rows() { return F2_ROWS; }

// ------------------------------------------- K1+K2: streaming PNG filter rows
// PNG tiles with a Sub/Up/Avg/Paeth or adaptive filter, rows of whole 16-byte chunks
// (w * bpp % 16 == 0, <= 2 KiB; 16-byte aligned source rows).  No LDS and no barriers: one
// WAVE per run of f3_run_rows() consecutive rows of one tile holds a whole row in registers (lane l
// = 16-byte chunks l, 64 + l), keeps the row above in registers, and prefetches the next row
// while it filters the current one.  A sample's left neighbour is the previous lane's chunk
// (one DPP wave shift; lane 0: the previous 64-chunk group, or zero before the row).  The
// adaptive choice (minimum sum of |byte - prediction|, first filter on ties: the oracle's rule)
// needs the whole row: five per-lane sums reduced over the wave by DPP.  Stream words are
// stored 16-byte aligned: lane l writes the aligned word ending where its chunk's first 16 - s
// bytes end (s = the row's start offset mod 16), i.e. the previous chunk's last s bytes and its
// own first 16 - s (k_rows' layout); lane 0 of a row writes the word that holds the previous
// row's tail and the filter byte.  That word needs the previous row's filtered tail, so a run
// also filters the row before it (without storing it): 1/run extra reads, no cross-wave
// hand-off.
// Rows a wave filters, per filter.  Round 6 (profiles/r06j/): a fixed filter's wave loads its
// whole run (and the row before it) at once -- a ring of run + 1 row buffers, no load waits
// behind a filtered row -- and exits, like k_extract's workgroups: Sub / Up / Avg 0.59-0.62 ->
// 0.64 of HBM peak with runs of 24 rows (100 VGPRs of rows, three waves per SIMD), Paeth
// 0.60 -> 0.625 with runs of 12 (its forms need more registers a row); the adaptive choice
// keeps its 5-row ring, over runs of 24 rows (the run-at-once forms spill it: 0.47-0.53).
#ifndef PBX_F3_RUN
#define PBX_F3_RUN 24  // Sub, Up, Avg
#endif
#ifndef PBX_F3_RUN_P
#define PBX_F3_RUN_P 12  // Paeth
#endif
#ifndef PBX_F3_RUN_AD
#define PBX_F3_RUN_AD 24  // adaptive (32: 0.559-0.564, 16: 0.559-0.561, 48: 0.567, 24: 0.573-0.575 of HBM, profiles/r06n/)
#endif
#ifndef PBX_F3_NTS
#define PBX_F3_NTS 0
#endif
__host__ __device__ constexpr uint32_t f3_run_rows(uint32_t filter) {
    return filter == 4 ? PBX_F3_RUN_P : filter == 5 ? PBX_F3_RUN_AD : PBX_F3_RUN;
}
// stream stores: nontemporal (the stream is re-read only by the next kernel, from HBM anyway)
#ifndef PBX_F3_NTL
#define PBX_F3_NTL 0  // nontemporal plane loads in k_filter3 (Sub / Up / Paeth 11-16% slower, profiles/r06zb/)
#endif
__device__ __forceinline__ void f3_store(uint8_t* p, const uint4& v) {
    if (PBX_F3_NTS) {
        pbx_v4u x;
        x.x = v.x; x.y = v.y; x.z = v.z; x.w = v.w;
        __builtin_nontemporal_store(x, (__attribute__((address_space(1))) pbx_v4u*)p);
    } else {
        gstore16(p, v);
    }
}
constexpr uint32_t F3_NT = 256;
// row buffers per wave (up, cur and NB - 2 loads in flight), by the registers the variant has
#ifndef PBX_F3_NB
#define PBX_F3_NB 0
#endif
template <uint32_t G, uint32_t FT>
constexpr uint32_t F3_NB() {  // fixed filters, rows <= 1 KiB: the whole run and the row before it
    return PBX_F3_NB ? PBX_F3_NB : G == 1 ? (FT == 5 ? 5 : f3_run_rows(FT) + 1) : 4;
}

// Sum over the wave: row prefix sums (row_shr, zero shifted in), then row_bcast:15 / :31 carry
// the row totals up to lane 63.  bound_ctrl lets each step fold into one v_add_u32_dpp.
__device__ __forceinline__ uint32_t f3_wave_sum(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
// Sums over the wave of five per-lane values.  Four go through gfx950's lane swaps: the upper
// 32 lanes of one register trade places with the lower 32 of another (v_permlane32_swap), so
// one add leaves s0's 32-lane partials in lanes 0-31 and s1's in 32-63 (likewise s2 / s3);
// swapping odd 16-lane rows of that with even rows of the other (v_permlane16_swap) and one
// add leaves rows holding s0, s2, s1, s3; four row_shr steps finish all four at once (lane 15
// of each row).  s4 takes the plain path.  14 VALU operations fewer than five f3_wave_sums.
#ifndef PBX_F3_SWAP_SUMS
#define PBX_F3_SWAP_SUMS 1
#endif
__device__ __forceinline__ void f3_wave_sums5(const uint32_t (&s)[5], uint32_t (&t)[5]) {
    if (!PBX_F3_SWAP_SUMS) {
#pragma unroll
        for (int k = 0; k < 5; k++) t[k] = f3_wave_sum(s[k]);
        return;
    }
    const auto p01 = __builtin_amdgcn_permlane32_swap(s[0], s[1], false, false);
    const auto p23 = __builtin_amdgcn_permlane32_swap(s[2], s[3], false, false);
    const uint32_t a = p01[0] + p01[1], b = p23[0] + p23[1];  // [s0 | s1], [s2 | s3]
    const auto q = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    uint32_t x = q[0] + q[1];  // rows: s0, s2, s1, s3
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    t[0] = (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
    t[2] = (uint32_t)__builtin_amdgcn_readlane((int)x, 31);
    t[1] = (uint32_t)__builtin_amdgcn_readlane((int)x, 47);
    t[3] = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
    t[4] = f3_wave_sum(s[4]);
}
// The previous lane's chunk (wave shift right by one lane); lane 0 gets `first`.
__device__ __forceinline__ uint4 f3_prev_lane(const uint4& x, const uint4& first) {
    return make_uint4((uint32_t)__builtin_amdgcn_update_dpp((int)first.x, (int)x.x, 0x138, 0xF, 0xF, false),
                      (uint32_t)__builtin_amdgcn_update_dpp((int)first.y, (int)x.y, 0x138, 0xF, 0xF, false),
                      (uint32_t)__builtin_amdgcn_update_dpp((int)first.z, (int)x.z, 0x138, 0xF, 0xF, false),
                      (uint32_t)__builtin_amdgcn_update_dpp((int)first.w, (int)x.w, 0x138, 0xF, 0xF, false));
}
// The same with zero into lane 0 (bound_ctrl: no old value to set up)
__device__ __forceinline__ uint4 f3_prev_lane0(const uint4& x) {
    return make_uint4((uint32_t)__builtin_amdgcn_update_dpp(0, (int)x.x, 0x138, 0xF, 0xF, true),
                      (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x.y, 0x138, 0xF, 0xF, true),
                      (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x.z, 0x138, 0xF, 0xF, true),
                      (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x.w, 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ uint4 f3_readlane(const uint4& x, uint32_t l) {
    return make_uint4((uint32_t)__builtin_amdgcn_readlane((int)x.x, l), (uint32_t)__builtin_amdgcn_readlane((int)x.y, l),
                      (uint32_t)__builtin_amdgcn_readlane((int)x.z, l), (uint32_t)__builtin_amdgcn_readlane((int)x.w, l));
}
// The four words of the bytes bpp before each byte of chunk x (p = the chunk before it).
__device__ __forceinline__ void f3_left(const uint4& x, const uint4& p, uint32_t bpp, uint32_t (&l)[4]) {
    if (bpp == 8) {
        l[0] = p.z; l[1] = p.w; l[2] = x.x; l[3] = x.y;
    } else if (bpp == 4) {
        l[0] = p.w; l[1] = x.x; l[2] = x.y; l[3] = x.z;
    } else {
        const uint32_t sh = 4 - bpp;
        l[0] = __builtin_amdgcn_alignbyte(x.x, p.w, sh);
        l[1] = __builtin_amdgcn_alignbyte(x.y, x.x, sh);
        l[2] = __builtin_amdgcn_alignbyte(x.z, x.y, sh);
        l[3] = __builtin_amdgcn_alignbyte(x.w, x.z, sh);
    }
}

// v[g] for a uniform g < G, by masks (no dynamic register index: that would be scratch)
template <uint32_t G>
__device__ __forceinline__ uint4 f3_pick(const uint4 (&v)[G], uint32_t g) {
    uint4 r = v[0];
#pragma unroll
    for (uint32_t k = 1; k < G; k++) {
        const uint32_t m = 0u - (uint32_t)(g == k);
        r = make_uint4((r.x & ~m) | (v[k].x & m), (r.y & ~m) | (v[k].y & m), (r.z & ~m) | (v[k].z & m),
                       (r.w & ~m) | (v[k].w & m));
    }
    return r;
}

// Paeth's f16 lane forms of a row (paeth_pair_h): word j of chunk g as [0] = bytes 0, 1 and
// [1] = bytes 2, 3, each byte in a 16-bit lane under 0x64 (one v_perm_b32 each), and the same
// forms of the bytes bpp to their left.  In this layout the left forms are other words' forms
// (bpp 2: [0] = the previous word's [1], [1] = this word's [0]; bpp 4 / 8: the word one / two
// back), or one v_alignbyte each (bpp 1), so a row's forms are built once, reused as the next
// row's up forms, and only the previous lane's last words cross lanes (one DPP each; lane 0:
// the previous chunk group's lane 63, or zero bytes before the row).
constexpr uint32_t F3_PF_LO = 0x00050004u, F3_PF_HI = 0x00070006u, F3_PF_BIAS = 0x64646464u;
constexpr uint32_t F3_PF_ZERO = 0x64006400u;  // the form of two zero bytes
template <uint32_t G, uint32_t BPP>
__device__ __forceinline__ void f3_paeth_forms(const uint4 (&v)[G], uint32_t (&X)[G][4][2],
                                               uint32_t (&L)[G][4][2]) {
#pragma unroll
    for (uint32_t g = 0; g < G; g++) {
        const uint32_t w[4] = {v[g].x, v[g].y, v[g].z, v[g].w};
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) {
            X[g][j][0] = __builtin_amdgcn_perm(w[j], F3_PF_BIAS, F3_PF_LO);
            X[g][j][1] = __builtin_amdgcn_perm(w[j], F3_PF_BIAS, F3_PF_HI);
        }
    }
#pragma unroll
    for (uint32_t g = 0; g < G; g++) {
        // the previous lane's forms of words 2 and 3 (only those the sample size reads)
        uint32_t P[2][2];
#pragma unroll
        for (uint32_t j = 2; j < 4; j++)
#pragma unroll
            for (uint32_t s = 0; s < 2; s++) {
                const bool need = BPP == 8 || (j == 3 && (BPP == 4 || s == 1));
                if (!need) { P[j - 2][s] = 0; continue; }
                const uint32_t first = g ? (uint32_t)__builtin_amdgcn_readlane((int)X[g - 1][j][s], 63) : F3_PF_ZERO;
                P[j - 2][s] = (uint32_t)__builtin_amdgcn_update_dpp((int)first, (int)X[g][j][s], 0x138, 0xF, 0xF, false);
            }
        auto W = [&](int j, uint32_t s) -> uint32_t { return j >= 0 ? X[g][j][s] : P[j + 2][s]; };
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (BPP == 1) {
                L[g][j][0] = __builtin_amdgcn_alignbyte(X[g][j][0], W(j - 1, 1), 2);
                L[g][j][1] = __builtin_amdgcn_alignbyte(X[g][j][1], X[g][j][0], 2);
            } else if (BPP == 2) {
                L[g][j][0] = W(j - 1, 1);
                L[g][j][1] = X[g][j][0];
            } else if (BPP == 4) {
                L[g][j][0] = W(j - 1, 0);
                L[g][j][1] = W(j - 1, 1);
            } else {
                L[g][j][0] = W(j - 2, 0);
                L[g][j][1] = W(j - 2, 1);
            }
        }
    }
}
// Paeth's two decisions for a pair of bytes (paeth_pair_h without the selects): the f16 sign
// bit of each lane set where pa > min(pb, pc) (na) and where pb > pc (nb).
__device__ __forceinline__ void paeth_pair_signs(uint32_t a, uint32_t b, uint32_t c, uint32_t& na, uint32_t& nb) {
    const f3_h2 A = __builtin_bit_cast(f3_h2, a), B = __builtin_bit_cast(f3_h2, b), C = __builtin_bit_cast(f3_h2, c);
    const f3_h2 d1 = B - C, d2 = A - C, d3 = d1 + d2;
    const f3_h2 pa = __builtin_elementwise_max(d1, -d1), pb = __builtin_elementwise_max(d2, -d2),
                pc = __builtin_elementwise_max(d3, -d3);
    na = __builtin_bit_cast(uint32_t, (f3_h2)(__builtin_elementwise_min(pb, pc) - pa));
    nb = __builtin_bit_cast(uint32_t, (f3_h2)(pc - pb));
}
// Paeth's prediction of a word from the forms of its left, up and up-left bytes and the same
// bytes as words (a, b, c): the four lanes' sign bits become a byte mask in ONE v_perm_b32
// (selectors 8..11 replicate bits 15 / 31 of each source), and two bitwise selects pick
// c over b, then that over a, byte by byte.
__device__ __forceinline__ uint32_t f3_paeth_word(const uint32_t (&l)[2], const uint32_t (&u)[2], const uint32_t (&ul)[2],
                                                  uint32_t a, uint32_t b, uint32_t c) {
    uint32_t na0, nb0, na1, nb1;
    paeth_pair_signs(l[0], u[0], ul[0], na0, nb0);
    paeth_pair_signs(l[1], u[1], ul[1], na1, nb1);
    const uint32_t ma = __builtin_amdgcn_perm(na1, na0, 0x0B0A0908u), mb = __builtin_amdgcn_perm(nb1, nb0, 0x0B0A0908u);
    const uint32_t t = (mb & c) | (~mb & b);
    return (ma & t) | (~ma & a);
}
#ifndef PBX_F3_CARRY
#define PBX_F3_CARRY 1  // 1: a row's Paeth forms are kept for the next row; 0: rebuilt from it
#endif

// One wave's run of rows, specialised on the sample size (the left-neighbour shifts, the byte
// swap and the sign flip are then fixed: no per-row branches or register moves on bpp).
template <uint32_t G, uint32_t FT, uint32_t BPP, bool NONE>
__device__ __forceinline__ void f3_run(const TileDesc& d, uint32_t wi, uint32_t lane, uint8_t* __restrict__ stream) {
    constexpr uint32_t bpp = BPP;
    const uint32_t rb = (uint32_t)d.w * bpp, nc = rb >> 4, rowlen = d.rowlen;
    const uint32_t h = (uint32_t)d.h;
    // uniform row bounds: the row loop and its prefetch stay scalar branches
    constexpr uint32_t RUN = f3_run_rows(FT);
    const uint32_t r0 = __builtin_amdgcn_readfirstlane((wi - d.blk_first) * RUN);
    const uint32_t r1 = __builtin_amdgcn_readfirstlane(r0 + RUN < h ? r0 + RUN : h);
    const bool swap = (d.flags & TF_SWAP) != 0, flip = (d.flags & TF_FLIP) != 0;
    constexpr bool ADAPTIVE = FT == 5;
    constexpr uint32_t fixed = FT;  // the batch's filter: 1..4, 5 = adaptive (every tile's d.filter)
    const uint8_t* src0 = d.plane + (int64_t)d.y * d.pitch + (int64_t)d.x * bpp;
    uint8_t* out = stream + d.out_off;
    const uint4 Z = make_uint4(0, 0, 0, 0);
    auto load_row = [&](uint32_t r, uint4 (&v)[G]) {
        const uint8_t* rp = src0 + (int64_t)r * d.pitch;
#pragma unroll
        for (uint32_t g = 0; g < G; g++) {
            const uint32_t c = 64 * g + lane;
            v[g] = PBX_F3_NTL ? gload16_nt(rp + 16 * (c < nc ? c : 0u)) : gload16(rp + 16 * (c < nc ? c : 0u));
        }
    };
    auto conv = [&](uint4 (&v)[G]) {  // big-endian samples (and the sign flip), zero past the row
#pragma unroll
        for (uint32_t g = 0; g < G; g++) {
            uint4 q = v[g];
            if (swap) q = swap16(q, (int)bpp);
            if (flip) q = flip_msb(q, (int)bpp);
            // by a mask, not a select of the two vectors (which the compiler may turn into
            // a select between their stack slots: scratch); only a group the row ends in
            if (nc < 64 * (g + 1)) {
                const uint32_t m = 0u - (uint32_t)(64 * g + lane < nc);
                q = make_uint4(q.x & m, q.y & m, q.z & m, q.w & m);
            }
            v[g] = q;
        }
    };
    const uint32_t rs = r0 ? r0 - 1 : 0;  // first row filtered (the one before the run: not stored)
    const uint32_t rl = r1 - 1;
    uint4 tail = Z;  // the previous row's last filtered chunk (uniform)
    const uint32_t cl = nc - 1, gl = cl >> 6, ll = cl & 63;
    // Paeth's forms of the row above (PBX_F3_CARRY: the previous step's own, else rebuilt)
    // and (PBX_F3_CARRY) its left bytes as words
    uint32_t UF[G][4][2], ULF[G][4][2], ULB[G][4];
    // filter row r (cur, converted here) against up (already converted) and store it
    auto step = [&](const uint4 (&up)[G], uint4 (&cur)[G], uint32_t r) {
        conv(cur);
        uint4 lft[G];
#pragma unroll
        for (uint32_t g = 0; g < G; g++)
            lft[g] = g ? f3_prev_lane(cur[g], f3_readlane(cur[g - 1], 63)) : f3_prev_lane0(cur[g]);
        // the Paeth prediction of every word (forms of this row built here; the row above's
        // kept from the previous step, or rebuilt)
        auto paeth_row = [&](const uint32_t (&lw)[G][4], uint32_t (&pp)[G][4]) {  // lw: left bytes
            uint32_t XF[G][4][2], LF[G][4][2];
            f3_paeth_forms<G, BPP>(cur, XF, LF);
            if (!PBX_F3_CARRY) f3_paeth_forms<G, BPP>(up, UF, ULF);
#pragma unroll
            for (uint32_t g = 0; g < G; g++) {
                const uint32_t u[4] = {up[g].x, up[g].y, up[g].z, up[g].w};
#pragma unroll
                for (uint32_t j = 0; j < 4; j++) {
                    const uint32_t c = PBX_F3_CARRY ? ULB[g][j] : __builtin_amdgcn_perm(ULF[g][j][1], ULF[g][j][0], 0x06040200u);
                    pp[g][j] = f3_paeth_word(LF[g][j], UF[g][j], ULF[g][j], lw[g][j], u[j], c);
                }
            }
            if (PBX_F3_CARRY) {
#pragma unroll
                for (uint32_t g = 0; g < G; g++)
#pragma unroll
                    for (uint32_t j = 0; j < 4; j++) {
                        ULB[g][j] = lw[g][j];
#pragma unroll
                        for (uint32_t s = 0; s < 2; s++) {
                            UF[g][j][s] = XF[g][j][s];
                            ULF[g][j][s] = LF[g][j][s];
                        }
                    }
            }
        };
        uint4 f[G];
        uint32_t ft = fixed;
        if (NONE) {  // an adaptive tile in the None mode (k_adaptive_mode): the rows as they are
#pragma unroll
            for (uint32_t g = 0; g < G; g++) f[g] = cur[g];
            ft = 0;
        } else if (ADAPTIVE) {
            // every candidate's prediction ([0] Sub = left, [1] Up, [2] Avg, [3] Paeth) and the
            // row sums of |byte - prediction| (v_sad_u8; None: the bytes themselves); the chosen
            // filter's residuals are formed once, after the choice
            uint32_t pw[G][4][4];
            uint32_t sm[5] = {0, 0, 0, 0, 0};
            uint32_t pp[G][4], lw[G][4];
#pragma unroll
            for (uint32_t g = 0; g < G; g++) f3_left(cur[g], lft[g], bpp, lw[g]);
            paeth_row(lw, pp);
#pragma unroll
            for (uint32_t g = 0; g < G; g++) {
                const uint32_t(&l)[4] = lw[g];
                const uint32_t x[4] = {cur[g].x, cur[g].y, cur[g].z, cur[g].w};
                const uint32_t u[4] = {up[g].x, up[g].y, up[g].z, up[g].w};
#pragma unroll
                for (uint32_t j = 0; j < 4; j++) {
                    pw[g][0][j] = l[j];
                    pw[g][1][j] = u[j];
                    pw[g][2][j] = avg8(l[j], u[j]);
                    pw[g][3][j] = pp[g][j];
                }
                if (64 * g + lane < nc) {
#pragma unroll
                    for (uint32_t j = 0; j < 4; j++) {
                        sm[0] = __builtin_amdgcn_sad_u8(x[j], 0u, sm[0]);
#pragma unroll
                        for (uint32_t k = 0; k < 4; k++) sm[k + 1] = __builtin_amdgcn_sad_u8(x[j], pw[g][k][j], sm[k + 1]);
                    }
                }
            }
            uint32_t tot[5];
            f3_wave_sums5(sm, tot);
            uint32_t best = 0, bs = tot[0];
#pragma unroll
            for (uint32_t k = 1; k < 5; k++) {
                if (tot[k] < bs) { bs = tot[k]; best = k; }
            }
            ft = __builtin_amdgcn_readfirstlane(best);
#ifndef PBX_F3_ADAPT_SELECT
#define PBX_F3_ADAPT_SELECT 1  // 1: the chosen prediction by a uniform branch; 0: by masks in SGPRs
#endif
            if (PBX_F3_ADAPT_SELECT) {
                // ft is uniform (an SGPR): one scalar branch per row to the subtraction it
                // needs.  Each arm ends in its own (empty) asm statement: otherwise the
                // compiler sinks the four identical sub8 chains below the branch and selects
                // their operand per word (~100 scalar instructions and branches a row).
                auto resid = [&](auto kc) {  // kc: the candidate's index as a type (a constant)
                    constexpr uint32_t k = decltype(kc)::value;
#pragma unroll
                    for (uint32_t g = 0; g < G; g++) {
                        uint32_t o[4];
                        const uint32_t x[4] = {cur[g].x, cur[g].y, cur[g].z, cur[g].w};
#pragma unroll
                        for (uint32_t j = 0; j < 4; j++) o[j] = sub8(x[j], pw[g][k][j]);
                        f[g] = make_uint4(o[0], o[1], o[2], o[3]);
                    }
                };
                if (ft == 0) {
#pragma unroll
                    for (uint32_t g = 0; g < G; g++) f[g] = cur[g];
                    asm volatile("; f3 none");
                } else if (ft == 1) {
                    resid(std::integral_constant<uint32_t, 0>{});
                    asm volatile("; f3 sub");
                } else if (ft == 2) {
                    resid(std::integral_constant<uint32_t, 1>{});
                    asm volatile("; f3 up");
                } else if (ft == 3) {
                    resid(std::integral_constant<uint32_t, 2>{});
                    asm volatile("; f3 avg");
                } else {
                    resid(std::integral_constant<uint32_t, 3>{});
                    asm volatile("; f3 paeth");
                }
            } else {
                // the prediction by masks in SGPRs (None predicts 0), then one sub8
                const uint32_t m1 = 0u - (uint32_t)(ft == 1), m2 = 0u - (uint32_t)(ft == 2);
                const uint32_t m3 = 0u - (uint32_t)(ft == 3), m4 = 0u - (uint32_t)(ft == 4);
#pragma unroll
                for (uint32_t g = 0; g < G; g++) {
                    uint32_t o[4];
                    const uint32_t x[4] = {cur[g].x, cur[g].y, cur[g].z, cur[g].w};
#pragma unroll
                    for (uint32_t j = 0; j < 4; j++)
                        o[j] = sub8(x[j], (pw[g][0][j] & m1) | (pw[g][1][j] & m2) | (pw[g][2][j] & m3) | (pw[g][3][j] & m4));
                    f[g] = make_uint4(o[0], o[1], o[2], o[3]);
                }
            }
        } else {
            // one filter for every row: only it (ft is uniform: a scalar branch)
            uint32_t pp[G][4], lw[G][4];
            if (ft == 4) {
#pragma unroll
                for (uint32_t g = 0; g < G; g++) f3_left(cur[g], lft[g], bpp, lw[g]);
                paeth_row(lw, pp);
            }
#pragma unroll
            for (uint32_t g = 0; g < G; g++) {
                uint32_t l[4], o[4];
                const uint32_t x[4] = {cur[g].x, cur[g].y, cur[g].z, cur[g].w};
                const uint32_t u[4] = {up[g].x, up[g].y, up[g].z, up[g].w};
                if (ft == 2) {
#pragma unroll
                    for (uint32_t j = 0; j < 4; j++) o[j] = sub8(x[j], u[j]);
                } else {
                    f3_left(cur[g], lft[g], bpp, l);
                    if (ft == 1) {
#pragma unroll
                        for (uint32_t j = 0; j < 4; j++) o[j] = sub8(x[j], l[j]);
                    } else if (ft == 3) {
#pragma unroll
                        for (uint32_t j = 0; j < 4; j++) o[j] = sub8(x[j], avg8(l[j], u[j]));
                    } else {
#pragma unroll
                        for (uint32_t j = 0; j < 4; j++) o[j] = sub8(x[j], pp[g][j]);
                    }
                }
                f[g] = make_uint4(o[0], o[1], o[2], o[3]);
            }
        }
        if (r >= r0) {
            // stream words of row r: data chunk c at q = r * rowlen + 1 + 16 c, s = q mod 16
            const uint32_t q0 = r * rowlen + 1, s = q0 & 15u, A = q0 - s;
            // lane 0's word before its chunk: the previous row's last s - 1 bytes and the filter byte
            const uint4 y = make_uint4((tail.x >> 8) | (tail.y << 24), (tail.y >> 8) | (tail.z << 24),
                                       (tail.z >> 8) | (tail.w << 24), (tail.w >> 8) | (ft << 24));
#pragma unroll
            for (uint32_t g = 0; g < G; g++) {
                const uint32_t c = 64 * g + lane;
                const uint4 pf = f3_prev_lane(f[g], g ? f3_readlane(f[g - 1], 63) : y);
                uint4 wv = f[g];
                if (s) {
                    uint32_t ww[4];
                    funnel16(pf, f[g], 16 - s, ww);
                    wv = make_uint4(ww[0], ww[1], ww[2], ww[3]);
                }
                if (c < nc) f3_store(out + A + 16 * c, wv);
            }
            if (s == 0 && lane == 0) f3_store(out + A - 16, y);  // (r > 0: s == 1 at r == 0)
            if (r + 1 == h && s) {  // the tile's last row: its tail word (zeros after the stream)
                const uint4 fl = f3_pick(f, gl);
                if (lane == ll) {
                    uint32_t ww[4];
                    funnel16(fl, Z, 16 - s, ww);
                    f3_store(out + A + 16 * nc, make_uint4(ww[0], ww[1], ww[2], ww[3]));
                }
            }
        }
        tail = f3_readlane(f3_pick(f, gl), ll);
    };
    // A ring of NB row buffers, rotated by NAME (the loop is unrolled NB times): B[k] = up,
    // B[k + 1] = cur, the other NB - 2 = loads in flight.  Moving registers that a load is still
    // filling would make the compiler wait for every load (vmcnt(0)) each row; loads are
    // unconditional (clamped to the run's last row) so the counters stay exact.
    constexpr uint32_t NB = F3_NB<G, FT>();
    uint4 B[NB][G];
    load_row(rs ? rs - 1 : 0, B[0]);
#pragma unroll
    for (uint32_t k = 1; k < NB; k++) load_row(rs + k - 1 < rl ? rs + k - 1 : rl, B[k]);
    conv(B[0]);
    if (!rs) {
#pragma unroll
        for (uint32_t g = 0; g < G; g++) B[0][g] = Z;
    }
    if (PBX_F3_CARRY && !NONE && (ADAPTIVE || fixed == 4)) {
        f3_paeth_forms<G, BPP>(B[0], UF, ULF);
#pragma unroll
        for (uint32_t g = 0; g < G; g++)
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) ULB[g][j] = __builtin_amdgcn_perm(ULF[g][j][1], ULF[g][j][0], 0x06040200u);
    }
    const uint32_t nrow = r1 - rs, nfull = nrow - nrow % NB;
    uint32_t r = rs;
    for (; r < rs + nfull; r = __builtin_amdgcn_readfirstlane(r + NB)) {
#pragma unroll
        for (uint32_t k = 0; k < NB; k++) {
            step(B[k], B[(k + 1) % NB], r + k);
            const uint32_t rn = r + k + NB - 1;
            load_row(rn < rl ? rn : rl, B[k]);
        }
    }
#pragma unroll
    for (uint32_t k = 0; k + 1 < NB; k++)  // the last nrow % NB rows: already loaded
        if (r + k < r1) step(B[k], B[(k + 1) % NB], r + k);
}

template <uint32_t G, uint32_t FT>
__global__ __launch_bounds__(F3_NT) void k_filter3(const TileDesc* __restrict__ dt, uint32_t ndt,
                                                  uint32_t nwaves, uint8_t* __restrict__ stream) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wi = xcd_remap(blockIdx.x, gridDim.x) * (F3_NT / 64) +
                        __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wi >= nwaves) return;  // a whole wave: no barrier in this kernel
    const uint32_t ti = __builtin_amdgcn_readfirstlane(upper_index(ndt, wi, [&](uint32_t i) { return dt[i].blk_first; }));
    const TileDesc d = dt[ti];
    const uint32_t bpp = __builtin_amdgcn_readfirstlane((uint32_t)d.bpp);
    const uint32_t fl = __builtin_amdgcn_readfirstlane(d.flags);
    if (FT == 5 && (fl & TF_DIRECT)) return;  // None mode, read from the plane by k_lz77
    if (FT == 5 && (fl & TF_ANONE)) {  // uniform branches
        switch (bpp) {
        case 1: f3_run<G, FT, 1, true>(d, wi, lane, stream); break;
        case 2: f3_run<G, FT, 2, true>(d, wi, lane, stream); break;
        case 4: f3_run<G, FT, 4, true>(d, wi, lane, stream); break;
        default: f3_run<G, FT, 8, true>(d, wi, lane, stream); break;
        }
        return;
    }
    switch (bpp) {
    case 1: f3_run<G, FT, 1, false>(d, wi, lane, stream); break;
    case 2: f3_run<G, FT, 2, false>(d, wi, lane, stream); break;
    case 4: f3_run<G, FT, 4, false>(d, wi, lane, stream); break;
    default: f3_run<G, FT, 8, false>(d, wi, lane, stream); break;
    }
}

hipError_t launch_filter3(hipStream_t st, const TileDesc* d_tiles, uint32_t ntiles, uint32_t nwaves,
                          uint32_t max_rb, uint32_t filter, uint8_t* stream) {
    if (!ntiles || !nwaves) return hipSuccess;
    if (filter < 1 || filter > 5) return hipErrorInvalidValue;  // every tile's d.filter (the batch's)
    const uint32_t blocks = (nwaves + F3_NT / 64 - 1) / (F3_NT / 64);
    const dim3 g(blocks), b(F3_NT);
    // one body per filter: a fixed filter's kernel holds only its own registers
#define PBX_F3_LAUNCH(GG)                                                                                     \
    switch (filter) {                                                                                        \
    case 1: hipLaunchKernelGGL((k_filter3<GG, 1>), g, b, 0, st, d_tiles, ntiles, nwaves, stream); break;   \
    case 2: hipLaunchKernelGGL((k_filter3<GG, 2>), g, b, 0, st, d_tiles, ntiles, nwaves, stream); break;   \
    case 3: hipLaunchKernelGGL((k_filter3<GG, 3>), g, b, 0, st, d_tiles, ntiles, nwaves, stream); break;   \
    case 4: hipLaunchKernelGGL((k_filter3<GG, 4>), g, b, 0, st, d_tiles, ntiles, nwaves, stream); break;   \
    default: hipLaunchKernelGGL((k_filter3<GG, 5>), g, b, 0, st, d_tiles, ntiles, nwaves, stream); break;  \
    }
    if (max_rb <= 1024) {
        PBX_F3_LAUNCH(1)
    } else {
        PBX_F3_LAUNCH(2)
    }
#undef PBX_F3_LAUNCH
    return hipGetLastError();
}

uint32_t filter3_run_rows(uint32_t filter) { return f3_run_rows(filter); }
uint32_t filter3_max_rb() { return 2048; }
uint32_t filter2_max_rb() { return F2_MAX_RB; }

}  // namespace pbx
