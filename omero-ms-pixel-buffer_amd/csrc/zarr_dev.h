// zarr_dev.h — device helpers shared by the Zarr chunk decoders (kernels_zarr.hip,
// kernels_zstd.hip): the per-wave LDS input window and output ring.  Everything about a
// stream's parse is wave-uniform and kept in SGPRs (readfirstlane).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dev_util.h"

namespace pbx {

constexpr uint32_t ZR_INF = 32768;           // inflate: the whole deflate window (no far match reads HBM)
constexpr uint32_t ZR_LZ4 = 4096;            // LZ4 / BloscLZ ring: more waves per CU
constexpr uint32_t ZWAVES = 4;              // waves per workgroup
constexpr uint32_t ZLUT = 9;                // inflate first-level lookup: codes of <= 9 bits

// Dynamic LDS of the decoders, addressed by offset (a pointer into LDS kept in a struct would
// become a FLAT pointer; a selected one, a stack slot).  Per wave: ring, then (inflate) tables.
extern __shared__ uint8_t zlds[];

__device__ __forceinline__ uint16_t& lds16(uint32_t byte_off) {
    return *(uint16_t*)(zlds + byte_off);
}
__device__ __forceinline__ uint32_t& lds32(uint32_t byte_off) {
    return *(uint32_t*)(zlds + byte_off);
}
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

__device__ __forceinline__ uint32_t ld_u32_unaligned(const uint8_t* p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}

__device__ __forceinline__ uint32_t rfl(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// Input window of ZWIN bytes in LDS (wave-uniform reads are LDS reads: a VGPR window would
// put an s_waitcnt vmcnt(0) -- which on gfx9 also waits for every pending flush store --
// in front of each use).  Reloaded by one 16-byte load per lane.  The device source buffer
// has ZSLACK bytes after its last stream, so window loads never leave the allocation.
constexpr uint32_t ZWIN = 1024;  // the runtime leaves 4 KiB of slack after the streams

struct InWin {
    const uint8_t* in;
    uint32_t wo, base, lane;  // LDS offset of the window, stream offset it starts at
    __device__ void load(uint32_t q) {
        base = q;
        uint4 v;
        __builtin_memcpy(&v, in + q + 16 * lane, 16);
        *(uint4*)(zlds + wo + 16 * lane) = v;
    }
    __device__ uint32_t byte(uint32_t q) {
        if (q - base > ZWIN - 1) load(q);
        return rfl(zlds[wo + q - base]);
    }
    // 32 bits starting at byte q (little-endian)
    __device__ uint32_t dword(uint32_t q) {
        if (q - base > ZWIN - 4) load(q);
        uint32_t v;
        __builtin_memcpy(&v, zlds + wo + q - base, 4);  // one unaligned ds_read_b32
        return rfl(v);
    }
    // bytes q .. q+15 as four little-endian words: one unaligned ds_read_b128 (gfx950 LDS
    // takes byte-aligned accesses)
    __device__ void peek16(uint32_t q, uint32_t (&d)[4]) {
        if (q - base > ZWIN - 16) load(q);
        uint4 v;
        __builtin_memcpy(&v, zlds + wo + q - base, 16);
        d[0] = rfl(v.x);
        d[1] = rfl(v.y);
        d[2] = rfl(v.z);
        d[3] = rfl(v.w);
    }
    // byte q + lane for every lane
    __device__ uint32_t lane_byte(uint32_t q) {
        if (q - base > ZWIN - 64) load(q);
        return zlds[wo + q - base + lane];
    }
};

// Output through the LDS ring (offset rb, 256-aligned); bytes [flushed, op) are in the ring
// only.  Completed 256-byte runs go to HBM as one dword store per lane.
// Partial-wave stores go through put_if: the lanes outside the predicate write a byte of their
// own in a 64-byte trash area instead of branching round the store.  A divergent branch
// anywhere inside a decoder's symbol loop makes LLVM structurize the whole loop with exec
// masks, which moves the (wave-uniform) stream state into VGPRs and every test on it into
// v_cmp + s_and_saveexec code: several times the instructions per symbol.
// With ADLER, every byte written to HBM also goes into the lane's Adler-32 partial sums
// (sum of bytes, sum of position * byte; adler32() reduces them over the wave).
template <uint32_t RING, bool ADLER = false>
struct OutRing {
    static constexpr uint32_t ZM = RING - 1, ZR = RING;
    uint32_t rb;
    uint8_t* out;
    uint32_t op, flushed, olen, lane;
    uint32_t trash;  // LDS offset of 64 bytes
    uint32_t asb = 0;  // (ADLER) this lane's bytes: sum
    uint64_t asi = 0;  //          sum of position * byte
    __device__ uint8_t& ring(uint32_t pos) const { return zlds[rb + (pos & ZM)]; }
    __device__ void put_if(bool pred, uint32_t pos, uint32_t v) const {
        zlds[pred ? rb + (pos & ZM) : trash + lane] = (uint8_t)v;
    }
    __device__ void flush(uint32_t upto) {
        uint32_t f = rfl(flushed);  // keep the ring state in SGPRs (scalar branches)
        upto = rfl(upto);
        while (upto - f >= 256u) {
            const uint32_t v = *(const uint32_t*)(zlds + rb + ((f + 4 * lane) & ZM));
            __builtin_memcpy(out + f + 4 * lane, &v, 4);
            if (ADLER) {
                const uint32_t s = __builtin_amdgcn_udot4(v, 0x01010101u, 0u, false);
                asb += s;
                asi += (uint64_t)(f + 4 * lane) * s + __builtin_amdgcn_udot4(v, 0x03020100u, 0u, false);
            }
            f += 256;
        }
        flushed = f;
    }
    __device__ void finish() {
        for (uint32_t k = flushed; k < op; k += 64) {
            const uint32_t b = k + lane < op ? ring(k + lane) : 0u;
            if (k + lane < op) out[k + lane] = (uint8_t)b;
            if (ADLER) {
                asb += b;
                asi += (uint64_t)(k + lane) * b;
            }
        }
        flushed = op;
    }
    // (ADLER, after finish) Adler-32 of out[0, op): A = 1 + sum b, B = n + sum (n - i) b_i
    __device__ uint32_t adler32() const {
        uint64_t sb = asb, si = asi;
        for (int o = 32; o > 0; o >>= 1) {
            sb += (uint64_t)__shfl_xor((long long)sb, o, 64);
            si += (uint64_t)__shfl_xor((long long)si, o, 64);
        }
        constexpr uint64_t M = 65521;
        const uint64_t n = op % M, a = (1 + sb) % M;
        const uint64_t b = (n + n * (sb % M) + M - si % M) % M;
        return (uint32_t)(b << 16 | a);
    }
    // out[op .. op+len) = out[op-off .. op-off+len) (overlapping: period off)
    // lane % off for off < 64 without an integer division: lane / off is exact to within 1/63
    // in float, so +0.001 never crosses an integer
    __device__ uint32_t period_lane(uint32_t off) const {
        if (off >= 64) return lane;
        const float inv = __builtin_amdgcn_rcpf((float)off);
        return lane - off * (uint32_t)((float)lane * inv + 0.001f);
    }
    __device__ bool match(uint32_t off, uint32_t len) {
        if (off == 0 || off > op || len > olen - op) return false;
        const uint32_t rep = period_lane(off);
        if (off > ZR) {
            // A far source lies well below `flushed`: read it back from HBM, 1 KiB per round
            // trip (16 bytes a lane; off > ZR >= 4096 > 1024, so a chunk never overlaps its
            // source).  Its bytes end before p - 3072 while the last 8 flush stores (one per
            // 256 bytes) cover bytes >= p - 2303: vmcnt(8) (in-order completion on gfx9)
            // waits for the stores of the source and not for the latest ones.
            static_assert(ZR >= 4096, "far chunks of 1 KiB behind the last 8 flushes");
            for (uint32_t k = 0; k < len; k += 1024) {
                const uint32_t p = op + k, n = len - k < 1024 ? len - k : 1024;
                __builtin_amdgcn_s_waitcnt(0xF78);  // vmcnt(8), expcnt / lgkmcnt unconstrained
                typedef unsigned int v4u __attribute__((ext_vector_type(4)));
                const v4u q = *(const __attribute__((address_space(1))) v4u*)(out + p - off + 16 * lane);
#pragma unroll
                for (uint32_t b = 0; b < 16; b++) {
                    const uint32_t wv = b < 4 ? q.x : b < 8 ? q.y : b < 12 ? q.z : q.w;
                    put_if(16 * lane + b < n, p + 16 * lane + b, wv >> ((b & 3) * 8));
                }
                flush(p + n);
            }
        } else {
            for (uint32_t k = 0; k < len; k += 64) {
                const uint32_t p = op + k, n = len - k < 64 ? len - k : 64;
                const uint32_t v = ring(p - off + rep);
                put_if(lane < n, p + lane, v);
                flush(p + n);
            }
        }
        op += len;
        return true;
    }
    __device__ void put1(uint32_t v) {
        ring(op) = (uint8_t)v;  // every lane: the same byte
        op = rfl(op) + 1;
        // `flushed` is a multiple of 256 and every other writer flushes as it goes, so a
        // single byte completes a run exactly when op reaches a multiple of 256
        if ((op & 255u) == 0) flush(op);
    }
};


// Byte-parallel execution of a batch of up to 64 LZ77 sequences (LZ4, zstd): lane j holds
// sequence j = bll literals (source positions bsrc, bsrc + 1, ...) then bml bytes copied from
// boff back; no sequence is empty.  Output offsets by a prefix sum, then 64 output bytes per
// step: each lane finds its sequence (start flags in LDS at `flag`, ballot, mbcnt) and its
// byte: a literal (lit(position, step's first literal position, any literal in the step),
// called by every lane), a ring byte, an HBM byte (offsets beyond the ring, one round trip
// for the step), or a byte of the same step (pointer jumping).  False if a match reaches
// before the stream start or the output overflows.
template <uint32_t RING, bool ADL, class LitF>
__device__ bool seq_batch(OutRing<RING, ADL>& o, uint32_t flag, uint32_t lane, uint32_t bn, uint32_t bll,
                          uint32_t bml, uint32_t boff, uint32_t bsrc, LitF&& lit) {
    const bool act = lane < bn;
    const uint32_t sl = act ? bll + bml : 0u;
    const uint32_t end = wave_incl_add(sl, lane), st0 = end - sl;
    const uint32_t T = rdl(end, 63);
    const uint32_t op0 = rfl(o.op);
    if (T > o.olen - op0) return false;
    if (__ballot(act && bml != 0 && (boff == 0 || boff > op0 + st0 + bll))) return false;
    uint32_t base = 0;
    for (uint32_t cb = 0; cb < T; cb += 64) {
        zlds[flag + lane] = 0;
        const uint32_t rs = st0 - cb;
        zlds[act && rs < 64 ? flag + rs : flag + 64 + lane] = 1;
        const uint32_t f = zlds[flag + lane];
        const uint64_t M = __ballot(f != 0);
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0));
        const uint32_t idx = base + below + f - 1;
        base += (uint32_t)__popcll(M);
        const uint32_t p = cb + lane;
        const bool valid = p < T;
        const uint32_t s_st = (uint32_t)__shfl((int)st0, (int)idx, 64), s_ll = (uint32_t)__shfl((int)bll, (int)idx, 64);
        const uint32_t s_off = (uint32_t)__shfl((int)boff, (int)idx, 64), s_src = (uint32_t)__shfl((int)bsrc, (int)idx, 64);
        const uint32_t r = p - s_st;
        const bool islit = valid && r < s_ll;
        const uint64_t L = __ballot(islit);
        const uint32_t lpos = s_src + r;
        const uint32_t lfirst = L ? rdl(lpos, (uint32_t)__builtin_ctzll(L)) : 0u;
        const uint32_t lv = lit(lpos, lfirst, L != 0);
        const bool mt = valid && !islit;
        // a match byte's source; for a period s_off < 64 the copy of it in the first period
        // (before the match), so that runs do not chain through the step byte by byte
        const uint32_t rm = r - s_ll;
        uint32_t rep = rm;
        if (__ballot(mt && s_off < 64)) {
            const uint32_t d = s_off ? s_off : 1u;
            const uint32_t qq = (uint32_t)((float)rm * __builtin_amdgcn_rcpf((float)d));
            int32_t rr = (int32_t)(rm - qq * d);
            rr = rr < 0 ? rr + (int32_t)d : rr;
            rr = rr < 0 ? rr + (int32_t)d : rr;
            rr = rr >= (int32_t)d ? rr - (int32_t)d : rr;
            rr = rr >= (int32_t)d ? rr - (int32_t)d : rr;
            rep = s_off < 64 ? (uint32_t)rr : rm;
        }
        const uint32_t src = s_st + s_ll + rep - s_off;  // from op0 (may be < 0: an earlier batch)
        // below the ring: in HBM, under `flushed` (< 256 bytes stay unflushed after a step).
        // The source ends before p - (RING - 64) <= cb - 3968 while the last 8 flush stores
        // cover bytes >= cb - 2303: vmcnt(8) (in-order completion) waits for its stores only.
        static_assert(RING >= 4096, "far sources behind the last 8 flushes");
        const bool far = mt && s_off > RING - 64;
        uint32_t v = o.ring(op0 + src);
        if (__ballot(far)) {
            __builtin_amdgcn_s_waitcnt(0xF78);  // vmcnt(8), expcnt / lgkmcnt unconstrained
            const uint32_t hv = *(const __attribute__((address_space(1))) uint8_t*)(o.out + (far ? op0 + src : 0u));
            v = far ? hv : v;
        }
        v = islit ? lv : v;
        bool pend = mt && (int32_t)src >= (int32_t)cb;
        uint32_t ptr = src - cb;
        while (__ballot(pend)) {
            const uint32_t nv = (uint32_t)__shfl((int)v, (int)ptr, 64);
            const uint32_t np = (uint32_t)__shfl((int)pend, (int)ptr, 64);
            const uint32_t nq = (uint32_t)__shfl((int)ptr, (int)ptr, 64);
            v = pend && !np ? nv : v;
            ptr = pend && np ? nq : ptr;
            pend = pend && np;
        }
        o.put_if(valid, op0 + p, v);
        o.flush(op0 + (T - cb < 64 ? T : cb + 64));
    }
    o.op = op0 + T;
    return true;
}

}  // namespace pbx
