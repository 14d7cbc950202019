// dev_util.h — small device helpers shared by the gfx950 kernels (wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pbx {

struct DevOps {
    __device__ static void amin(uint32_t* p, uint32_t v) { atomicMin(p, v); }
    __device__ static void amax(uint32_t* p, uint32_t v) { atomicMax(p, v); }
    __device__ static void add(uint32_t* p, uint32_t v) { atomicAdd(p, v); }
    __device__ static void aor(uint32_t* p, uint32_t v) { atomicOr(p, v); }
};

// Load through a pointer known to be in global memory (plane pointers come from tile
// descriptors, so the compiler cannot infer their address space and would emit FLAT loads,
// which also count against lgkmcnt and so stall every later LDS wait on HBM latency).
// (A native vector type: a uint4 struct copy is lowered to a memcpy that drops the cast.)
typedef unsigned int pbx_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gload16(const void* p) {
    const pbx_v4u v = *(const __attribute__((address_space(1))) pbx_v4u*)p;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gstore16(void* p, const uint4& v) {
    pbx_v4u x;
    x.x = v.x; x.y = v.y; x.z = v.z; x.w = v.w;
    *(__attribute__((address_space(1))) pbx_v4u*)p = x;
}

// Streaming forms (nontemporal: data read or written once, not kept in the caches).
__device__ __forceinline__ uint4 gload16_nt(const void* p) {
    const pbx_v4u v = __builtin_nontemporal_load((const __attribute__((address_space(1))) pbx_v4u*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gstore16_nt(void* p, const uint4& v) {
    pbx_v4u x;
    x.x = v.x; x.y = v.y; x.z = v.z; x.w = v.w;
    __builtin_nontemporal_store(x, (__attribute__((address_space(1))) pbx_v4u*)p);
}

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

// The same search by a whole wave (all 64 lanes active, the same n and v in every lane): each
// round probes 64 evenly spaced keys at once and keeps the span between the last probe <= v
// and the next, so 4096 keys take 2 dependent rounds of loads instead of 12.
template <class F>
__device__ __forceinline__ uint32_t upper_index_wave(uint32_t n, uint32_t v, F key) {
    const uint32_t lane = __lane_id();
    uint32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const uint32_t step = (hi - lo) / 64 + 1;  // 64 probes cover [lo, hi]
        const uint32_t p = lo + lane * step;
        const bool le = p <= hi && key(p) <= v;
        const uint64_t m = __ballot(le);           // lane 0 (p = lo) is always set
        const uint32_t t = 63u - (uint32_t)__builtin_clzll(m);
        const uint32_t nlo = lo + t * step;
        const uint32_t nhi = nlo + step - 1 < hi ? nlo + step - 1 : hi;
        lo = __builtin_amdgcn_readfirstlane(nlo);
        hi = __builtin_amdgcn_readfirstlane(nhi);
    }
    return lo;
}

// Inclusive prefix sum over the wave by DPP alone (no ds_bpermute round trips): row scans by
// row_shr (zero shifted in), then row_bcast:15 / :31 carry the row totals into the rows above.
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return x;
}

// (every lane active at the call, as DPP reads its source lanes' registers)
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t v, uint32_t /*lane*/) { return wave_incl_scan_dpp(v); }

// Exclusive prefix sum of arr[0..NT) in place (one element per thread); returns the total.
template <int NT>
__device__ uint32_t block_scan_excl_add(uint32_t* arr, uint32_t* wtot, uint32_t tid) {
    const uint32_t v = arr[tid], lane = tid & 63, w = tid >> 6;
    const uint32_t inc = wave_incl_add(v, lane);
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

// Exclusive prefix sum of arr[0..N) in place by ONE wave (N/64 consecutive elements per
// lane); returns the total.
template <int N>
__device__ uint32_t wave_scan_excl_add(uint32_t* arr, uint32_t lane) {
    constexpr int K = N / 64;
    uint32_t v[K], s = 0;
#pragma unroll
    for (int k = 0; k < K; k++) { v[k] = arr[lane * K + k]; s += v[k]; }
    const uint32_t inc = wave_incl_add(s, lane);
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    uint32_t run = inc - s;
#pragma unroll
    for (int k = 0; k < K; k++) { arr[lane * K + k] = run; run += v[k]; }
    return tot;
}

__device__ __forceinline__ uint32_t bswap16x2(uint32_t v) {
    return __builtin_amdgcn_perm(v, v, 0x02030001u);  // [b1, b0, b3, b2]: one v_perm_b32
}

// Swap each big-endian sample of a 16-byte vector to/from little-endian.
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

// APNGWriter's sign flip of int8 / int16 samples: the MS byte of each big-endian sample.
__device__ __forceinline__ uint4 flip_msb(uint4 q, int bpp) {
    const uint32_t m = bpp == 1 ? 0x80808080u : 0x00800080u;
    q.x ^= m; q.y ^= m; q.z ^= m; q.w ^= m;
    return q;
}

// Bytes [bs, bs + 16) of the 32 bytes lo || hi (bs < 16) as 4 words: two levels of mask
// selects pick the 5 source words, one alignbit each.  (Masks, not ?: over an array: the
// compiler turns `c ? a[k + 1] : a[k]` into a dynamic index, i.e. scratch memory.)
__device__ __forceinline__ void funnel16(const uint4& lo, const uint4& hi, uint32_t bs, uint32_t (&w)[4]) {
    const uint32_t m0 = 0u - ((bs >> 2) & 1u), m1 = 0u - ((bs >> 3) & 1u);
    auto sel = [](uint32_t m, uint32_t y, uint32_t x) { return (y & m) | (x & ~m); };
    const uint32_t u0 = sel(m0, lo.y, lo.x), u1 = sel(m0, lo.z, lo.y), u2 = sel(m0, lo.w, lo.z),
                   u3 = sel(m0, hi.x, lo.w), u4 = sel(m0, hi.y, hi.x), u5 = sel(m0, hi.z, hi.y),
                   u6 = sel(m0, hi.w, hi.z);
    const uint32_t t0 = sel(m1, u2, u0), t1 = sel(m1, u3, u1), t2 = sel(m1, u4, u2),
                   t3 = sel(m1, u5, u3), t4 = sel(m1, u6, u4);
    const uint32_t sh = (bs & 3u) * 8;
    w[0] = __builtin_amdgcn_alignbit(t1, t0, sh);
    w[1] = __builtin_amdgcn_alignbit(t2, t1, sh);
    w[2] = __builtin_amdgcn_alignbit(t3, t2, sh);
    w[3] = __builtin_amdgcn_alignbit(t4, t3, sh);
}

// 16 bytes from an address of any alignment in global memory: the aligned 16-byte word at or
// below it and (unless it is aligned) the next one, funnel-shifted.  Reads up to 31 bytes past
// `p`: callers stay inside a plane's pitched rows and its 256 B of over-read slack.
__device__ __forceinline__ uint4 gload16u(const uint8_t* p) {
    const uint32_t bs = (uint32_t)(uintptr_t)p & 15u;
    const uint8_t* a = p - bs;
    const uint4 lo = gload16(a);
    uint4 hi = lo;
    if (bs) hi = gload16(a + 16);
    uint32_t w[4];
    funnel16(lo, hi, bs, w);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Realigned 16-byte loads for a wave whose lanes read consecutive 16-byte pieces of a row (lane
// l + 1 at lane l's address + 16): a lane's upper aligned word is its right neighbour's lower
// one, so it is taken by one DPP wave shift instead of a second load.  Issue first (addresses
// shared by DPP before any load: the loads a lane still needs -- lane 63, a lane whose
// neighbour is inactive or elsewhere -- go out with the others), finish after.  Issue and
// finish must run with the same lanes active.
struct ULoad {
    uint4 lo, hi;
    uint32_t bs;
    bool own;
};
__device__ __forceinline__ uint32_t dpp_from_next(uint32_t x, uint32_t old) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, 0x130, 0xF, 0xF, false);  // wave_shl:1
}
template <bool NT = false>  // NT: nontemporal loads (source read once)
__device__ __forceinline__ void uload_issue(ULoad& u, const uint8_t* p) {
    u.bs = (uint32_t)(uintptr_t)p & 15u;
    const uint8_t* a = p - u.bs;
    const uint64_t ai = (uint64_t)(uintptr_t)a;
    const uint64_t na = (uint64_t)dpp_from_next((uint32_t)ai, 0u) |
                        ((uint64_t)dpp_from_next((uint32_t)(ai >> 32), 0u) << 32);
    u.own = u.bs != 0 && na != ai + 16;
    u.lo = NT ? gload16_nt(a) : gload16(a);
    u.hi = u.lo;
    if (u.own) u.hi = NT ? gload16_nt(a + 16) : gload16(a + 16);
}
__device__ __forceinline__ uint4 uload_finish(const ULoad& u) {
    const uint4 nlo = make_uint4(dpp_from_next(u.lo.x, 0u), dpp_from_next(u.lo.y, 0u),
                                 dpp_from_next(u.lo.z, 0u), dpp_from_next(u.lo.w, 0u));
    const uint4 hi = u.own ? u.hi : nlo;
    uint32_t w[4];
    funnel16(u.lo, hi, u.bs, w);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

}  // namespace pbx
