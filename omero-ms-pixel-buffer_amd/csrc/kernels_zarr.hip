// kernels_zarr.hip — NGFF/Zarr v2 chunk decode into a resident HBM plane:
// the step before getTileDirect when the reference's pixels service is ZarrPixelsService
// (PixelBufferVerticle.java:29,56; beanRefContext.xml:51; omero-zarr-pixel-buffer 0.6.1,
// build.gradle:57).  Chunk formats are restated in oracle/zarr_oracle.c.
//
//   k_zarr_lz4      one wave per compressed stream (a blosc split): LZ4 block decode
//   k_zarr_inflate  one wave per zlib stream (Zarr "zlib" chunks, blosc-zlib splits)
//   k_zarr_copy     one wave per stored stream (blosc splits kept raw)
//   k_zarr_place    per chunk rows: blosc byte-unshuffle + placement into the pitched plane,
//                   fill value for missing chunks
//
// Decoders keep the wave's last 4 KiB of output in an LDS ring (the match source for every
// distance <= 4 KiB) and flush completed 256-byte runs to HBM (one dword store per lane), so
// a match never waits on the wave's own global stores; a longer distance reads HBM after a
// workgroup fence.  Parse state is wave-uniform and lives in SGPRs (the wave index goes
// through readfirstlane).  The input is an LDS window of 1 KiB (one 16-byte load per lane);
// an LZ4 sequence header is one unaligned ds_read_b128 peek.  A Huffman symbol comes from a
// 512-entry first-level table (codes <= 9 bits) or, for longer codes, from lanes 0..14 testing
// the 15 code lengths at once (canonical ranges) with one ballot picking the length.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "dev_util.h"
#include "pbx_common.h"
#include "pbx_kernels.h"
#include "zarr_dev.h"

namespace pbx {

constexpr uint32_t ZL_BYTES = ZR_LZ4 + ZWIN + 64 + 128 + 1024;  // LZ4 / BloscLZ per wave: ring, window, trash, flags, batch

// ------------------------------------------------------------------------------ LZ4
// Most LZ4 sequences of image data are short (a few literals, a 4..18-byte match): one wave
// walking them one by one spends ~900 cycles on each, two LDS round trips in a chain.  Here
// they are parsed 64 input offsets at a time: lane k reads the sequence that would start k
// bytes on (token, literal count, offset: one round of LDS reads), a scalar walk from offset 0
// picks the real ones (a readlane and an add each), and their fields go to an LDS batch of up
// to 64 sequences executed by seq_batch (byte-parallel output steps).  Sequences with
// length-extension bytes (long literal runs or matches) and the final literals take the
// per-sequence path after the pending batch.
__global__ __launch_bounds__(256) void k_zarr_lz4(const ZStream* __restrict__ st, uint32_t n,
                                                  const uint8_t* __restrict__ src,
                                                  uint8_t* __restrict__ dst, uint32_t* __restrict__ err) {
    const uint32_t lane = threadIdx.x & 63, w = rfl(threadIdx.x >> 6);  // wave-uniform (SGPR) state
    const uint32_t si = blockIdx.x * ZWAVES + w;
    if (si >= n) return;
    const ZStream t = st[si];
    const uint32_t ilen = rfl(t.csize);
    const uint32_t wb = w * ZL_BYTES;
    InWin win{src + t.src_off, wb + ZR_LZ4, 0, lane};
    win.load(0);
    OutRing<ZR_LZ4> o{wb, dst + t.dst_off, 0, 0, t.dlen, lane, wb + ZR_LZ4 + ZWIN};
    const uint32_t FLAG = wb + ZR_LZ4 + ZWIN + 64, BATCH = FLAG + 128;  // batch: ll, ml, off, src x 64
    uint32_t ip = 0, bad = 0, bn = 0;
#ifdef PBX_ZARR_CLOCKS  // diagnostic build: stream 0's clocks
    const uint64_t c0 = __builtin_amdgcn_s_memtime();
    uint64_t cexec = 0, cgen = 0;
    uint32_t nbat = 0, nseq = 0, ngen = 0, nround = 0;
#define ZLC(...) __VA_ARGS__
#else
#define ZLC(...)
#endif
    auto flush_batch = [&]() -> bool {
        bn = rfl(bn);
        if (!bn) return true;
        ZLC(const uint64_t x0 = __builtin_amdgcn_s_memtime(); nbat++;)
        const uint32_t bll = lds32(BATCH + 4 * lane), bml = lds32(BATCH + 256 + 4 * lane);
        const uint32_t boff = lds32(BATCH + 512 + 4 * lane), bsrc = lds32(BATCH + 768 + 4 * lane);
        const uint32_t wo = win.wo, wbase = win.base;
        const bool ok = seq_batch(o, FLAG, lane, bn, bll, bml, boff, bsrc,
                                  [&](uint32_t pos, uint32_t, bool) -> uint32_t {
            const uint32_t at = pos - wbase;  // literals of the batch lie in the LDS window
            return zlds[wo + (at < ZWIN ? at : 0u)];
        });
        bn = 0;
        ZLC(cexec += __builtin_amdgcn_s_memtime() - x0;)
        return ok;
    };
    for (;;) {
        ip = rfl(ip); bn = rfl(bn); o.op = rfl(o.op); o.flushed = rfl(o.flushed);
        if (ip >= ilen) { bad = 1; break; }
        // the LDS window covers the 64 candidate starts and their headers and literals
        // (<= 17 bytes each); the batch's literals lie behind ip in it
        if (ip + 64 + 20 > win.base + ZWIN) {
            if (!flush_batch()) { bad = 6; break; }
            win.load(ip);
        }
        // lane k: the sequence starting at ip + k, if it is a short one
        const uint32_t q = ip + lane, qa = q - win.base;
        const uint32_t h = ld_u32_unaligned(zlds + win.wo + (qa < ZWIN - 4 ? qa : ZWIN - 4));
        const uint32_t tok = h & 0xFFu, ll = tok >> 4, ml0 = tok & 15;
        const uint32_t oa = qa + 1 + ll;
        const uint32_t off = ld_u32_unaligned(zlds + win.wo + (oa < ZWIN - 4 ? oa : ZWIN - 4)) & 0xFFFFu;
        const bool ok = ll < 15 && ml0 < 15 && q + 3 + ll <= ilen && q + 1 + ll != ilen;
        const uint32_t nx = (lane + 3 + ll) | (ok ? 0u : 0x100u);
        // the walk: real sequence starts (at most 64 - bn of them)
        uint64_t M = 0;
        uint32_t p = 0, cnt = 0;
        const uint32_t cap = 64 - bn;
        while (p < 64 && cnt < cap) {
            const uint32_t v = rdl(nx, p);
            if (v & 0x100u) break;
            M |= 1ull << p;
            cnt++;
            p = v;
        }
        ZLC(nround++; nseq += cnt;)
        if (cnt) {
            const uint32_t rank = bn + __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0));
            const bool in = (M >> lane) & 1;
            const uint32_t slot = in ? BATCH + 4 * rank : FLAG + 64;  // (masked-off lanes: trash)
            lds32(slot) = ll;
            lds32(slot + (in ? 256u : 0u)) = ml0 + 4;
            lds32(slot + (in ? 512u : 0u)) = off;
            lds32(slot + (in ? 768u : 0u)) = q + 1;
            bn += cnt;
            ip += p;
            if (bn == 64 && !flush_batch()) { bad = 6; break; }
            continue;
        }
        // a sequence with length-extension bytes (or the final literals): parsed serially; it
        // joins the batch when it is short enough and its literals lie in the LDS window, else
        // (a long literal run or match, or the end) the batch is executed and it is copied here
        ZLC(const uint64_t g0 = __builtin_amdgcn_s_memtime(); ngen++;)
        auto sbyte = [&](uint32_t qq) -> uint32_t {  // (the batch's literals must stay in the window)
            if (qq - win.base > ZWIN - 1 && !flush_batch()) bad = 6;
            return win.byte(qq);
        };
        const uint32_t t0 = sbyte(ip);
        if (bad) break;
        uint32_t k = 1, lln = t0 >> 4;
        if (lln == 15) {
            uint32_t b;
            do {
                if (ip + k >= ilen) { bad = 2; break; }
                b = sbyte(ip + k++);
                lln += b;
            } while (b == 255);
            if (bad) break;
        }
        const uint32_t ls = ip + k;
        if (lln > ilen - ls || lln > o.olen - o.op) { bad = 3; break; }
        const bool final = ls + lln == ilen;
        uint32_t ml = t0 & 15, off2 = 0;
        if (!final) {
            if (ilen - (ls + lln) < 2) { bad = 4; break; }
            k += lln;  // offset at ip + k
            off2 = sbyte(ip + k) | sbyte(ip + k + 1) << 8;
            k += 2;
            if (ml == 15) {
                uint32_t b;
                do {
                    if (ip + k >= ilen) { bad = 5; break; }
                    b = sbyte(ip + k++);
                    ml += b;
                } while (b == 255);
                if (bad) break;
            }
            if (bad) break;
            // (long matches copy faster on the per-sequence path: 64 bytes a step without the
            // batch's bookkeeping, 1 KiB per HBM round trip when far)
            if (ml + 4 <= 256 && lln <= 256 && ls >= win.base && ls + lln + 24 <= win.base + ZWIN) {
                const uint32_t slot = lane == 0 ? BATCH + 4 * rfl(bn) : FLAG + 64;
                lds32(slot) = lln;
                lds32(slot + (lane == 0 ? 256u : 0u)) = ml + 4;
                lds32(slot + (lane == 0 ? 512u : 0u)) = off2;
                lds32(slot + (lane == 0 ? 768u : 0u)) = ls;
                bn++;
                ip += k;
                ZLC(cgen += __builtin_amdgcn_s_memtime() - g0;)
                if (bn == 64 && !flush_batch()) { bad = 6; break; }
                continue;
            }
        }
        if (!flush_batch()) { bad = 6; break; }
        for (uint32_t c = 0; c < lln; c += 64) {
            const uint32_t nb = lln - c < 64 ? lln - c : 64;
            const uint32_t v = win.lane_byte(ls + c);
            o.put_if(lane < nb, o.op + c + lane, v);
            o.flush(o.op + c + nb);
        }
        o.op += lln;
        if (final) { ip = ilen; break; }
        ip += k;
        if (!o.match(off2, ml + 4)) { bad = 6; break; }
        ZLC(cgen += __builtin_amdgcn_s_memtime() - g0;)
        if (ip < ilen && (ip < win.base || ip + 84 > win.base + ZWIN)) win.load(ip);
    }
    if (!bad && o.op != o.olen) bad = 7;
    o.finish();
    ZLC(if (lane == 0 && si < 2) printf("lz4 stream %u: total %lu exec %lu (%u batches, %u sequences, %u rounds) per-sequence path %lu (%u)\n", si,
        (unsigned long)(__builtin_amdgcn_s_memtime() - c0), (unsigned long)cexec, nbat, nseq, nround, (unsigned long)cgen, ngen);)
    if (lane == 0) err[si] = bad;
}

// --------------------------------------------------------------------------- BloscLZ
// c-blosc 1.21's internal codec (format restated in oracle/zarr_oracle.c): control byte < 32
// = ctrl + 1 literals; else a match of (ctrl >> 5) + 2 bytes (7: + 255-terminated extension
// bytes) at distance ((ctrl & 31) << 8) + next byte + 1, or 16-bit big-endian + 8192 when
// those are 31 and 255.  A match is only copied when another control byte follows.
__global__ __launch_bounds__(256) void k_zarr_blosclz(const ZStream* __restrict__ st, uint32_t n,
                                                      const uint8_t* __restrict__ src,
                                                      uint8_t* __restrict__ dst, uint32_t* __restrict__ err) {
    const uint32_t lane = threadIdx.x & 63, w = rfl(threadIdx.x >> 6);  // wave-uniform (SGPR) state
    const uint32_t si = blockIdx.x * ZWAVES + w;
    if (si >= n) return;
    const ZStream t = st[si];
    const uint32_t ilen = rfl(t.csize);
    const uint32_t wb = w * ZL_BYTES;
    InWin win{src + t.src_off, wb + ZR_LZ4, 0, lane};
    win.load(0);
    OutRing<ZR_LZ4> o{wb, dst + t.dst_off, 0, 0, t.dlen, lane, wb + ZR_LZ4 + ZWIN};
    uint32_t ip = 0, bad = ilen == 0 ? 1u : 0u;
    uint32_t ctrl = bad ? 0u : win.byte(ip++) & 31u;
    while (!bad) {
        if (ctrl >= 32) {
            uint32_t len = (ctrl >> 5) - 1, code = 0;
            const uint32_t ofs = (ctrl & 31u) << 8;
            if (len == 6) {
                do {
                    if (ip + 1 >= ilen) { bad = 2; break; }
                    code = win.byte(ip++);
                    len += code;
                } while (code == 255);
                if (bad) break;
            } else if (ip + 1 >= ilen) {
                bad = 3;
                break;
            }
            code = win.byte(ip++);
            len += 3;
            uint32_t dist = ofs + code + 1;
            if (code == 255 && ofs == (31u << 8)) {  // 16-bit distance
                if (ip + 1 >= ilen) { bad = 4; break; }
                dist = (win.byte(ip) << 8 | win.byte(ip + 1)) + 8192;
                ip += 2;
            }
            if (len > o.olen - o.op || dist > o.op) { bad = 5; break; }
            if (ip >= ilen) break;
            ctrl = win.byte(ip++);
            if (!o.match(dist, len)) { bad = 6; break; }
        } else {
            const uint32_t nl = ctrl + 1;  // <= 32 literals: one lane step
            if (nl > o.olen - o.op || ip + nl > ilen) { bad = 7; break; }
            const uint32_t v = win.lane_byte(ip);
            o.put_if(lane < nl, o.op + lane, v);
            o.op += nl;
            o.flush(o.op);
            ip += nl;
            if (ip >= ilen) break;
            ctrl = win.byte(ip++);
        }
    }
    if (!bad && o.op != o.olen) bad = 8;
    o.finish();
    if (lane == 0) err[si] = bad;
}

// ---------------------------------------------------------------------------- inflate
// Canonical Huffman table held by lanes 1..15 (code length L = lane + 1 for lane < 15):
// first code, count and the index of its first symbol in the sorted symbol list.
struct HTab {
    uint32_t first, count, offs;
    uint32_t syms;  // LDS byte offset of the sorted symbol list (uint16)
};

struct BitIn {
    InWin win;
    uint64_t buf;
    uint32_t cnt, ipos, ilen;
    __device__ void refill() {
        // the bit-stream state is wave-uniform: pin it to SGPRs (LLVM otherwise moves it to
        // VGPRs through a phi and turns every branch on it into exec-mask code)
        cnt = rfl(cnt);
        ipos = rfl(ipos);
        buf = (uint64_t)rfl((uint32_t)(buf >> 32)) << 32 | rfl((uint32_t)buf);
        if (cnt <= 32) {
            // past the stream's end (corrupt input) feed zeros instead of reading on: the
            // decoder stops at the output bound and the consumed-bytes check fails the stream
            if (ipos <= ilen + 8) buf |= (uint64_t)win.dword(ipos) << cnt;
            cnt += 32;
            ipos += 4;
        }
    }
    __device__ uint32_t bits(uint32_t k) {  // k <= 32 - (bits guaranteed by a refill)
        const uint32_t v = (uint32_t)buf & ((k == 32) ? 0xffffffffu : ((1u << k) - 1u));
        buf >>= k;
        cnt -= k;
        return v;
    }
    __device__ uint32_t consumed_bytes() const { return ipos - cnt / 8; }
};

// Build the table of n code lengths lens[0..n) (LDS); returns false if over-subscribed.
__device__ bool build_table(HTab& h, uint32_t lens /* LDS offset */, uint32_t n, uint32_t lane,
                            uint32_t next /* LDS offset of 16 counters */) {
    const uint32_t L = lane + 1;
    uint32_t cnt = 0;
    if (L <= 15)
        for (uint32_t s = 0; s < n; s++) cnt += zlds[lens + s] == L;
    // first code of length L: code = (code + count[L-1]) << 1 from L = 1; offs = sum count[<L]
    uint32_t code = 0, off = 0, left = 1;
    bool over = false;
    for (uint32_t l = 1; l <= 15; l++) {
        const uint32_t c = rdl(cnt, l - 1);
        left = (left << 1);
        if (c > left) over = true;
        left -= c > left ? left : c;
        if (l == L) { h.first = code; h.offs = off; }
        code = (code + c) << 1;
        off += c;
    }
    h.count = L <= 15 ? cnt : 0;
    if (L > 15) { h.first = 0; h.offs = 0; }
    if (lane < 16) lds32(next + 4 * lane) = 0;
    __builtin_amdgcn_wave_barrier();
    // sorted symbol list: rank of s among the symbols of its length, in symbol order
    for (uint32_t g = 0; g < n; g += 64) {
        const uint32_t s = g + lane;
        const uint32_t ln = s < n ? zlds[lens + s] : 0;
        const uint64_t lt = (lane ? (~0ull >> (64 - lane)) : 0ull);
        for (uint32_t l = 1; l <= 15; l++) {
            const uint64_t m = __ballot(ln == l);
            if (!m) continue;
            const uint32_t base = lds32(next + 4 * l);
            if (ln == l) lds16(h.syms + 2 * (rdl(h.offs, l - 1) + base + __popcll(m & lt))) = (uint16_t)s;
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) lds32(next + 4 * l) = base + (uint32_t)__popcll(m);
            __builtin_amdgcn_wave_barrier();
        }
    }
    __builtin_amdgcn_wave_barrier();
    return !over;
}

// Canonical decode of the code in the low bits of `bits` (>= 15 valid bits): the symbol, and
// its length in nb; -1 on an invalid code.
__device__ __forceinline__ int decode_bits(const HTab& h, uint32_t bits, uint32_t lane, uint32_t& nb) {
    const uint32_t rev = __builtin_bitreverse32(bits & 0x7fffu) >> 17;  // 15 bits, MSB-first
    const uint32_t L = lane + 1;
    const uint32_t code = L <= 15 ? rev >> (15 - L) : 0;
    const bool ok = L <= 15 && (code - h.first) < h.count;
    const uint64_t m = __ballot(ok);
    if (!m) return -1;
    const uint32_t l = (uint32_t)__builtin_ctzll(m);
    const uint32_t idx = rdl(h.offs + code - h.first, l);
    nb = l + 1;
    return (int)rfl(lds16(h.syms + 2 * idx));
}
// Decode one symbol (the bit buffer holds >= 15 bits); returns -1 on an invalid code.
__device__ int decode_sym(const HTab& h, BitIn& bi, uint32_t lane) {
    uint32_t nb = 0;
    const int sym = decode_bits(h, (uint32_t)bi.buf, lane, nb);
    if (sym >= 0) bi.bits(nb);
    return sym;
}

// First-level table of a built code: lut[next 9 stream bits] = sym | len << 9 for codes of
// <= 9 bits (every extension of the bit-reversed code), 0xFFFF (-> decode_sym) otherwise.
template <uint32_t LB = ZLUT>
__device__ void build_lut(const HTab& h, uint32_t lens, uint32_t lut, uint32_t lane) {
    for (uint32_t e = lane; e < (1u << LB); e += 64) lds16(lut + 2 * e) = 0xFFFF;
    __builtin_amdgcn_wave_barrier();
    const uint32_t total = rdl(h.offs + h.count, 14);  // symbols with a code
    for (uint32_t g = 0; g < total; g += 64) {  // uniform trip count: the shuffles see all lanes
        const uint32_t j = g + lane;
        const uint32_t sym = j < total ? lds16(h.syms + 2 * j) : 0u;
        const uint32_t len = j < total ? zlds[lens + sym] : 0u;
        const uint32_t src = len ? len - 1 : 0;
        const uint32_t first = (uint32_t)__shfl((int)h.first, (int)src, 64);
        const uint32_t offs = (uint32_t)__shfl((int)h.offs, (int)src, 64);
        if (len == 0 || len > LB) continue;
        const uint32_t rev = __builtin_bitreverse32(first + (j - offs)) >> (32 - len);
        for (uint32_t k = 0; k < (1u << (LB - len)); k++)
            lds16(lut + 2 * (rev | (k << len))) = (uint16_t)(sym | len << 9);
    }
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int decode_fast(const HTab& h, uint32_t lut, BitIn& bi, uint32_t lane) {
    const uint32_t e = rfl(lds16(lut + 2 * ((uint32_t)bi.buf & ((1u << ZLUT) - 1))));
    if (e != 0xFFFF) {
        bi.bits(e >> 9);
        return (int)(e & 511);
    }
    return decode_sym(h, bi, lane);
}

__constant__ uint16_t c_lbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                     35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_lext[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2,
                                   3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                     193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097,
                                     6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dext[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                   6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

constexpr uint32_t ZLENS = 352;

// Per-wave LDS of k_zarr_inflate (byte offsets from the wave's base)
constexpr uint32_t ZI_RING = 0, ZI_LSYMS = ZR_INF, ZI_DSYMS = ZI_LSYMS + 2 * 288,
                   ZI_LENS = ZI_DSYMS + 2 * 32, ZI_NEXT = ZI_LENS + ZLENS,
                   ZI_LLUT = ZI_NEXT + 64, ZI_DLUT = ZI_LLUT + 2 * (1u << ZLUT),
                   ZI_TRASH = ZI_DLUT + 2 * (1u << ZLUT), ZI_BYTES = ZI_TRASH + 64;

__global__ __launch_bounds__(256) void k_zarr_inflate(const ZStream* __restrict__ st, uint32_t n,
                                                      const uint8_t* __restrict__ src,
                                                      uint8_t* __restrict__ dst, uint32_t* __restrict__ err) {
    const uint32_t lane = threadIdx.x & 63, w = rfl(threadIdx.x >> 6);  // wave-uniform (SGPR) state
    const uint32_t si = blockIdx.x * ZWAVES + w;
    if (si >= n) return;
    const uint32_t wb = w * (ZI_BYTES + ZWIN);
    const uint32_t LENS = wb + ZI_LENS, NEXT = wb + ZI_NEXT;
    const ZStream t = st[si];
    BitIn bi{{src + t.src_off, wb + ZI_BYTES, 0, lane}, 0ull, 0, 0, rfl(t.csize)};
    bi.win.load(0);
    OutRing<ZR_INF> o{wb + ZI_RING, dst + t.dst_off, 0, 0, t.dlen, lane, wb + ZI_TRASH};
    HTab lt{0, 0, 0, wb + ZI_LSYMS}, dt{0, 0, 0, wb + ZI_DSYMS};
    uint32_t bad = 0;
    bi.refill();
    if (t.kind == ZS_ZLIB) {  // RFC 1950 header: CM = 8, CINFO <= 7, no preset dictionary
        const uint32_t cmf = bi.bits(8), flg = bi.bits(8);
        if ((cmf & 15) != 8 || (cmf >> 4) > 7 || (flg & 0x20) || ((cmf << 8) | flg) % 31) bad = 10;
    }
    uint32_t final = 0;
    while (!bad && !final) {
        bi.refill();
        final = bi.bits(1);
        const uint32_t type = bi.bits(2);
        if (type == 0) {  // stored
            bi.bits(bi.cnt & 7);
            bi.refill();
            const uint32_t len = bi.bits(16), nlen = bi.bits(16);
            if ((len ^ 0xffffu) != nlen) { bad = 11; break; }
            // the remaining whole bytes of the bit buffer come first
            uint32_t done = 0;
            while (done < len && bi.cnt >= 8 && o.op < o.olen) { o.put1(bi.bits(8)); done++; }
            if (done < len && bi.cnt >= 8) { bad = 12; break; }
            // a block shorter than the buffered bytes (LEN 0..3: e.g. the empty stored block
            // of a sync flush) leaves whole bytes of what FOLLOWS it in the buffer: rewind
            // the input over them (cnt is a multiple of 8 here) instead of dropping them
            const uint32_t q = bi.ipos - bi.cnt / 8, rest = len - done;
            if (q + rest > bi.ilen || rest > o.olen - o.op) { bad = 12; break; }
            for (uint32_t k = 0; k < rest; k += 64) {
                const uint32_t nb = rest - k < 64 ? rest - k : 64;
                const uint32_t v = bi.win.lane_byte(q + k);
                o.put_if(lane < nb, o.op + k + lane, v);
                o.flush(o.op + k + nb);
            }
            o.op += rest;
            bi.ipos = q + rest;
            bi.buf = 0;
            bi.cnt = 0;
            continue;
        }
        if (type == 3) { bad = 13; break; }
        if (type == 1) {  // fixed codes
            for (uint32_t s = lane; s < 320; s += 64)
                zlds[LENS + s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
            __builtin_amdgcn_wave_barrier();
            build_table(lt, LENS, 288, lane, NEXT);
            build_table(dt, LENS + 288, 30, lane, NEXT);
            build_lut(lt, LENS, wb + ZI_LLUT, lane);
            build_lut(dt, LENS + 288, wb + ZI_DLUT, lane);
        } else {  // dynamic
            bi.refill();
            const uint32_t hlit = bi.bits(5) + 257, hdist = bi.bits(5) + 1, hclen = bi.bits(4) + 4;
            if (hlit > 286 || hdist > 30) { bad = 14; break; }
            for (uint32_t s = lane; s < 19; s += 64) zlds[LENS + s] = 0;
            __builtin_amdgcn_wave_barrier();
            for (uint32_t k = 0; k < hclen; k++) {
                bi.refill();
                const uint32_t v = bi.bits(3);
                if (lane == 0) zlds[LENS + c_clord[k]] = (uint8_t)v;
            }
            __builtin_amdgcn_wave_barrier();
            HTab ct{0, 0, 0, wb + ZI_LSYMS};
            if (!build_table(ct, LENS, 19, lane, NEXT)) { bad = 15; break; }
            // code lengths for litlen + dist go to lens[19..] first, then move down
            uint32_t k = 0, prev = 0;
            while (k < hlit + hdist) {
                bi.refill();
                const int sym = decode_sym(ct, bi, lane);
                if (sym < 0) { bad = 16; break; }
                uint32_t rep = 1, val = (uint32_t)sym;
                if (sym == 16) {
                    if (k == 0) { bad = 17; break; }
                    rep = 3 + bi.bits(2); val = prev;
                } else if (sym == 17) { rep = 3 + bi.bits(3); val = 0; }
                else if (sym == 18) { rep = 11 + bi.bits(7); val = 0; }
                if (k + rep > hlit + hdist) { bad = 18; break; }
                for (uint32_t r = lane; r < rep; r += 64) zlds[LENS + 19 + k + r] = (uint8_t)val;
                __builtin_amdgcn_wave_barrier();
                k += rep;
                prev = val;
            }
            if (bad) break;
            for (uint32_t s = lane; s < 320; s += 64) {
                const uint8_t v = s < hlit + hdist ? zlds[LENS + 19 + s] : 0;
                __builtin_amdgcn_wave_barrier();
                zlds[LENS + s] = v;
            }
            __builtin_amdgcn_wave_barrier();
            // litlen = lens[0..hlit) zero-padded to 288; dist lengths moved to lens[288..320)
            {
                const uint8_t dv = lane < hdist ? zlds[LENS + hlit + lane] : 0;
                __builtin_amdgcn_wave_barrier();
                for (uint32_t s = hlit + lane; s < ZLENS; s += 64) zlds[LENS + s] = 0;
                __builtin_amdgcn_wave_barrier();
                if (lane < 32) zlds[LENS + 288 + lane] = dv;
                __builtin_amdgcn_wave_barrier();
            }
            if (!build_table(lt, LENS, 288, lane, NEXT)) { bad = 19; break; }
            if (!build_table(dt, LENS + 288, 30, lane, NEXT)) { bad = 20; break; }
            build_lut(lt, LENS, wb + ZI_LLUT, lane);
            build_lut(dt, LENS + 288, wb + ZI_DLUT, lane);
        }
        // block data
        for (;;) {
            bi.refill();
            // distance-table entries at every bit offset of the buffer, gathered in the same
            // LDS round trip as the literal/length lookup: a match's distance code then costs
            // a readlane instead of a second dependent round trip
            const uint32_t cnt0 = bi.cnt;
            const uint32_t dv = lds16(wb + ZI_DLUT + 2 * ((uint32_t)(bi.buf >> lane) & ((1u << ZLUT) - 1)));
            const int sym = decode_fast(lt, wb + ZI_LLUT, bi, lane);
            if (sym < 0) { bad = 21; break; }
            if (sym < 256) {
                if (o.op >= o.olen) { bad = 22; break; }
                o.put1((uint32_t)sym);
                continue;
            }
            if (sym == 256) break;
            const uint32_t ls = (uint32_t)sym - 257;
            if (ls >= 29) { bad = 23; break; }
            // >= 17 bits are left after a <= 15-bit code (refill leaves >= 32): no refill
            const uint32_t len = c_lbase[ls] + bi.bits(c_lext[ls]);
            int ds;
            const uint32_t de = rdl(dv, cnt0 - bi.cnt);
            if (de != 0xFFFF && (de >> 9) <= bi.cnt) {
                bi.bits(de >> 9);
                ds = (int)(de & 511);
            } else {
                bi.refill();
                ds = decode_fast(dt, wb + ZI_DLUT, bi, lane);
            }
            if (ds < 0 || ds >= 30) { bad = 24; break; }
            bi.refill();
            const uint32_t dist = c_dbase[ds] + bi.bits(c_dext[ds]);
            if (!o.match(dist, len)) { bad = 25; break; }
        }
        if (!bad && bi.consumed_bytes() > bi.ilen) bad = 26;
    }
    if (!bad && o.op != o.olen) bad = 27;
    o.finish();
    if (lane == 0) err[si] = bad;
}

// ------------------------------------------------------------ inflate, two-wave pipeline
// One zlib stream is one serial symbol chain, and a plane of 512^2 chunks gives only one
// stream per SIMD: the single-wave decoder above is bound by the latency of that chain
// (Huffman lookup -> bits consumed -> next lookup, plus the match copies).  Here each stream
// gets TWO waves of one workgroup, a pipeline through an LDS token FIFO:
//   producer  the bit stream: block headers and code tables serially, as above; a Huffman
//             block's data by self-synchronizing macro-rounds (zp_huff_block): 64 segments of
//             ~24 tokens each decoded at once, one per lane, from guessed starts, then stitched
//             where the chains meet.  Whole tokens (literal, or length + distance with their
//             extra bits) go to the FIFO at each lane's prefix-sum offset.
//   consumer  the output: batches of >= 32 tokens; offsets by a prefix sum, then 64 output
//             bytes per step, each lane finding its token and its byte (the literal, the ring,
//             or pointer jumping over sources inside the step); the ring flushes to HBM.
// Tokens: literal 0x01000000 | byte; match 0x40000000 | (len - 3) << 16 | (dist - 1);
// stored run 0x80000000 | len, then the run's input offset; end 0xC0000000 | error code.
constexpr uint32_t ZP_TOKQ = 2048;                  // FIFO tokens per stream (power of two)
// The consumer's output ring: half the deflate window.  Farther sources (1.2% of zlib-1's
// matches on noise) are read back from HBM; the LDS saved is the fourth stream per CU.
constexpr uint32_t ZP_RINGB = 16384;
constexpr uint32_t ZPLUT = 10;                      // producer's first-level tables: codes <= 10 bits
constexpr uint32_t ZP_WINB = 3072;                  // input window: a macro-round's 64 segments
constexpr uint32_t ZP_SMAX = 256;                   // longest segment (bits): 8 * ZP_SMAX + 24 <= ZP_WINB
constexpr uint32_t ZP_SEGTOK = 24;                  // tokens per segment aimed at
constexpr uint32_t ZP_WIN = 0, ZP_LLUT = ZP_WINB, ZP_DLUT = ZP_LLUT + 2 * (1u << ZPLUT),
                   ZP_LSYMS = ZP_DLUT + 2 * (1u << ZPLUT), ZP_DSYMS = ZP_LSYMS + 2 * 288,
                   ZP_LENS = ZP_DSYMS + 2 * 32, ZP_NEXT = ZP_LENS + ZLENS, ZP_FIFO = ZP_NEXT + 64,
                   ZP_RING = ZP_FIFO + 4 * ZP_TOKQ, ZP_CTRL = ZP_RING + ZP_RINGB,
                   ZP_TRASH = ZP_CTRL + 32,         // 4 bytes per lane: masked-off lanes' stores
                   ZP_FLAG = ZP_TRASH + 256 + 64,   // the consumer's token-start flags (+ trash)
                   ZP_BYTES = ZP_FLAG + 128;        // per stream
static_assert(ZP_BYTES <= 160 * 1024 / 4, "four streams (eight waves) per CU");
constexpr uint32_t ZP_STREAMS = 1;                  // streams (x 2 waves) per workgroup
enum : uint32_t { ZPC_TAIL = 0, ZPC_HEAD = 4, ZPC_ABORT = 8, ZPC_DONE = 12, ZPC_ADLER = 16 };
constexpr uint32_t ZP_BATCH = 32;  // the consumer waits for this many tokens (or the end)

__device__ __forceinline__ uint32_t zp_lext(uint32_t ls) { return ls < 8 || ls == 28 ? 0u : (ls - 4) >> 2; }
__device__ __forceinline__ uint32_t zp_lbase(uint32_t ls) {
    return ls < 8 ? 3 + ls : ls == 28 ? 258u : ((4 + (ls & 3)) << ((ls >> 2) - 1)) + 3;
}
__device__ __forceinline__ uint32_t zp_dext(uint32_t ds) { return ds < 4 ? 0u : (ds >> 1) - 1; }
__device__ __forceinline__ uint32_t zp_dbase(uint32_t ds) {
    return ds < 4 ? ds + 1 : ((2 + (ds & 1)) << ((ds >> 1) - 1)) + 1;
}
// The FIFO control words.  Both waves' LDS operations complete in issue order, so a plain
// (volatile, LDS-typed) store of `tail` after the token stores publishes them; no memory
// fence (a workgroup fence would also wait for every outstanding HBM store of the consumer).
typedef volatile __attribute__((address_space(3))) uint32_t lds_vu32_t;
__device__ __forceinline__ uint32_t lds_load_volatile(uint32_t off) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const uint32_t v = rfl(*(lds_vu32_t*)(zlds + off));
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    return v;
}
__device__ __forceinline__ void lds_store_volatile(uint32_t off, uint32_t v) {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    *(lds_vu32_t*)(zlds + off) = v;  // every lane: the same word
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

struct TokOut {  // the producer's side of the FIFO
    uint32_t tail, head, sb, lane;
    __device__ bool room(uint32_t k) {  // false if the consumer aborted
        while (tail + k - head > ZP_TOKQ) {
            head = lds_load_volatile(sb + ZP_CTRL + ZPC_HEAD);
            if (tail + k - head <= ZP_TOKQ) break;
            if (lds_load_volatile(sb + ZP_CTRL + ZPC_ABORT)) return false;
            __builtin_amdgcn_s_sleep(1);
        }
        return true;
    }
    // the tokens of the lanes in m, in lane order (stores without a lane branch: a divergent
    // branch anywhere in the symbol loop makes LLVM structurize it with exec masks)
    __device__ bool put_lanes(uint64_t m, uint32_t tok) {
        const uint32_t nt = (uint32_t)__popcll(m);
        if (!nt) return true;
        if (!room(nt)) return false;
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0));
        lds32((m >> lane) & 1 ? sb + ZP_FIFO + 4 * ((tail + rank) & (ZP_TOKQ - 1)) : sb + ZP_TRASH + 4 * lane) = tok;
        tail += nt;
        lds_store_volatile(sb + ZP_CTRL + ZPC_TAIL, tail);
        return true;
    }
    __device__ bool put(uint32_t tok) { return put_lanes(1ull, tok); }
};

#ifdef PBX_ZARR_DIAG  // diagnostic build only: per-stream clocks and token counts (printf, stream 0)
#define ZDIAG(...) __VA_ARGS__
#else
#define ZDIAG(...)
#endif
// Per-lane decode kinds of the lane-parallel round
enum : uint32_t { ZK_TOK = 0, ZK_EOB = 1, ZK_SLOW = 2, ZK_BAD = 3 };

// Per-lane decode of the whole token that starts at bit `pos` of the stream (the LDS window
// [wbase, wbase + ZP_WINB) must hold its bytes): literal, end of block, or length + extra bits +
// distance + extra bits.  Codes longer than the first-level tables take a per-lane canonical
// search over the remaining lengths (uniform loop, only when some lane needs it).
struct ZLane {
    uint32_t kind, adv, tok;  // ZK_*, bits, FIFO token (or the error code of ZK_BAD)
};
__device__ __forceinline__ uint32_t canon_lane(const HTab& h, uint32_t bits, bool need) {
    const uint32_t rev = __builtin_bitreverse32(bits & 0x7fffu) >> 17;
    uint32_t res = 0xFFFF, idx = 0;
    for (uint32_t L = ZPLUT + 1; L <= 15; L++) {
        const uint32_t f = rdl(h.first, L - 1), c = rdl(h.count, L - 1), o = rdl(h.offs, L - 1);
        const uint32_t code = rev >> (15 - L);
        const bool hit = need && res == 0xFFFF && code - f < c;
        idx = hit ? o + code - f : idx;
        res = hit ? L << 9 : res;
    }
    const uint32_t sym = lds16(h.syms + 2 * idx);
    return res == 0xFFFF ? res : res | sym;
}
__device__ __forceinline__ ZLane zp_decode_at(uint32_t pos, uint32_t win, uint32_t wbase, uint32_t LLUT,
                                              uint32_t DLUT, const HTab& lt, const HTab& dt) {
    constexpr uint32_t LM = (1u << ZPLUT) - 1;
    const uint32_t bo = win + (pos >> 3) - wbase;
    uint32_t w0, w1;
    __builtin_memcpy(&w0, zlds + bo, 4);
    __builtin_memcpy(&w1, zlds + bo + 4, 4);
    const uint64_t x = ((uint64_t)w1 << 32 | w0) >> (pos & 7);  // >= 57 valid bits
    uint32_t e = lds16(LLUT + 2 * ((uint32_t)x & LM));
    if (__ballot(e == 0xFFFF)) e = e == 0xFFFF ? canon_lane(lt, (uint32_t)x, true) : e;
    const uint32_t l = (e >> 9) & 15, sym = e & 511, ls = sym - 257;
    const uint32_t lsv = ls < 29 ? ls : 0u;  // in range for the arithmetic of every lane
    const uint32_t le = zp_lext(lsv), p2 = l + le;
    const uint32_t len = zp_lbase(lsv) + ((uint32_t)(x >> l) & ((1u << le) - 1));
    const uint32_t xd = (uint32_t)(x >> p2);
    uint32_t de = lds16(DLUT + 2 * (xd & LM));
    const bool need_d = sym > 256 && ls < 29 && de == 0xFFFF;
    if (__ballot(need_d)) de = need_d ? canon_lane(dt, xd, true) : de;
    const uint32_t dl = (de >> 9) & 15, ds = de & 511, dsv = ds < 30 ? ds : 0u;
    const uint32_t dx = zp_dext(dsv), p3 = p2 + dl;
    const uint32_t dist = zp_dbase(dsv) + ((uint32_t)(x >> p3) & ((1u << dx) - 1));
    const bool short_sym = sym <= 256;
    ZLane r;
    r.kind = e == 0xFFFF ? ZK_BAD : sym == 256 ? ZK_EOB : short_sym ? ZK_TOK
           : ls >= 29 ? ZK_BAD : de == 0xFFFF ? ZK_BAD : ds >= 30 ? ZK_BAD : ZK_TOK;
    r.adv = short_sym ? l : p3 + dx;
    r.tok = r.kind == ZK_BAD ? (e == 0xFFFF ? 21u : ls >= 29 ? 23u : 24u)
          : short_sym ? 0x01000000u | sym : 0x40000000u | ((len - 3) << 16) | (dist - 1);
    return r;
}

// Token starts met in a segment (<= ZP_SMAX bits): four words in VGPRs, indexed by selects (an
// array indexed by a lane-varying bit would live in scratch memory).
struct SegBits {
    uint64_t a = 0, b = 0, c = 0, d = 0;
    __device__ void set(uint32_t r) {
        const uint64_t m = 1ull << (r & 63);
        const uint32_t w = r >> 6;
        a |= w == 0 ? m : 0ull; b |= w == 1 ? m : 0ull; c |= w == 2 ? m : 0ull; d |= w == 3 ? m : 0ull;
    }
    __device__ bool test(uint32_t r) const {  // (masks: a ?: chain becomes a scratch-memory table)
        const uint32_t w = r >> 6;
        const uint64_t x = (a & (0ull - (uint64_t)(w == 0))) | (b & (0ull - (uint64_t)(w == 1))) |
                           (c & (0ull - (uint64_t)(w == 2))) | (d & (0ull - (uint64_t)(w == 3)));
        return (x >> (r & 63)) & 1;
    }
    __device__ uint32_t count_below(uint32_t r) const {  // set bits < r (r < 256)
        const uint32_t w = r >> 6;
        const uint64_t m = (1ull << (r & 63)) - 1;
        uint32_t n = (uint32_t)__popcll(w == 0 ? a & m : a);
        n += w >= 1 ? (uint32_t)__popcll(w == 1 ? b & m : b) : 0u;
        n += w >= 2 ? (uint32_t)__popcll(w == 2 ? c & m : c) : 0u;
        n += w >= 3 ? (uint32_t)__popcll(d & m) : 0u;
        return n;
    }
    // bits >= r of this, bits < r of o
    __device__ void splice(const SegBits& o, uint32_t r) {
        const uint32_t w = r >> 6;
        const uint64_t m = (1ull << (r & 63)) - 1;
        const uint64_t la = w > 0 ? ~0ull : m, lb = w > 1 ? ~0ull : w == 1 ? m : 0ull,
                       lc = w > 2 ? ~0ull : w == 2 ? m : 0ull, ld = w == 3 ? m : 0ull;
        a = (o.a & la) | (a & ~la);
        b = (o.b & lb) | (b & ~lb);
        c = (o.c & lc) | (c & ~lc);
        d = (o.d & ld) | (d & ~ld);
    }
};

// One Huffman block's data, self-synchronizing: a macro-round splits the next 64*S bits into
// 64 segments and lane i decodes from the START of segment i, which is probably not a token
// boundary (pass A), recording the token starts it meets in the segment.
// Pass B re-decodes each lane from where its left neighbour's chain left the segments before
// it, until that chain meets one of the recorded starts: from there the two chains are the
// same token sequence (decoding is a function of the bit position), so the lane's pass-A
// count and exit stand.  A chain that meets none decodes the whole segment, and its right
// neighbour is checked again.  Pass C re-decodes every lane from its true entry and
// writes its tokens to the FIFO at the lane's offset (a prefix sum of the counts).
// Returns the bit position after the block (or of the round's end when it stopped early).
__device__ __forceinline__ uint32_t zp_huff_block(uint32_t B, BitIn& bi, TokOut& to, uint32_t sb, uint32_t lane,
                                                  const HTab& lt, const HTab& dt, uint32_t& bad, bool& alive,
                                                  uint32_t& sbits ZDIAG(, uint32_t* dg)) {
    const uint32_t WIN = sb + ZP_WIN, LLUT = sb + ZP_LLUT, DLUT = sb + ZP_DLUT;
    bool loaded = false;  // the bit reader's window is 1 KiB: reload the whole window once
    for (;;) {
        // segment length: about 16 tokens per lane at the last round's bits per token
        const uint32_t S = sbits;
        const uint32_t q = B >> 3;
        if (q > bi.ilen) { bad = 26; return B; }  // (corrupt input: the window would leave the slack)
        if (!loaded || q < bi.win.base || q + 8 * S + 24 > bi.win.base + ZP_WINB) {
            loaded = true;
            uint4 v[ZP_WINB / 1024];
#pragma unroll
            for (uint32_t k = 0; k < ZP_WINB / 1024; k++) __builtin_memcpy(&v[k], bi.win.in + q + 1024 * k + 16 * lane, 16);
#pragma unroll
            for (uint32_t k = 0; k < ZP_WINB / 1024; k++) *(uint4*)(zlds + WIN + 1024 * k + 16 * lane) = v[k];
            bi.win.base = q;
        }
        const uint32_t wb = bi.win.base;
        const uint32_t b0 = B + lane * S, e0 = b0 + S;
        ZDIAG(dg[0]++;)
        // pass A
        uint32_t pos = b0, cs = 0, fl = ZK_TOK, ec = 0;
        SegBits vis;
        bool act = true;
        while (__ballot(act)) {
            ZDIAG(dg[1]++;)
            const ZLane d = zp_decode_at(act ? pos : B, WIN, wb, LLUT, DLUT, lt, dt);
            if (act) vis.set(pos - b0);
            const bool stop = d.kind != ZK_TOK;
            fl = act && stop ? d.kind : fl;
            ec = act && d.kind == ZK_BAD ? d.tok : ec;
            cs += act && !stop ? 1u : 0u;
            pos += act && d.kind != ZK_BAD ? d.adv : 0u;
            act = act && !stop && pos < e0;
        }
        // pass B
        uint32_t xs = pos, chk = b0;
        for (;;) {
            const uint32_t pe = (uint32_t)__shfl_up((int)xs, 1, 64), pf = (uint32_t)__shfl_up((int)fl, 1, 64);
            const uint32_t e = lane ? pe : B;
            const bool todo = lane && pf == ZK_TOK && e != chk;
            if (!__ballot(todo)) break;
            ZDIAG(dg[2]++;)
            uint32_t p = e, c = 0;
            bool walk = todo;  // from the entry until the old chain is met (or the segment ends)
            SegBits vn;
            while (__ballot(walk)) {
                ZDIAG(dg[3]++;)
                const uint32_t rel = p - b0;
                if (walk && vis.test(rel)) {  // the chains meet at p
                    cs = c + (cs - vis.count_below(rel));
                    vis.splice(vn, rel);
                    walk = false;
                }
                const ZLane d = zp_decode_at(walk ? p : B, WIN, wb, LLUT, DLUT, lt, dt);
                if (walk) {
                    vn.set(rel);
                    const bool stop = d.kind != ZK_TOK;
                    c += stop ? 0u : 1u;
                    p += d.kind != ZK_BAD ? d.adv : 0u;
                    if (stop || p >= e0) {  // the new chain is this lane's chain
                        xs = p;
                        cs = c;
                        fl = d.kind;
                        ec = d.kind == ZK_BAD ? d.tok : ec;
                        vis = vn;
                        walk = false;
                    }
                }
            }
            chk = todo ? e : chk;
        }
        // pass C: the lanes up to the first chain that ends the block (EOB or an error)
        const uint64_t ends = __ballot(fl != ZK_TOK);
        const uint32_t first = ends ? (uint32_t)__builtin_ctzll(ends) : 63u;
        const uint32_t cnt = lane <= first ? cs : 0u;
        const uint32_t incl = wave_incl_add(cnt, lane), off = incl - cnt;
        // as many lanes as the FIFO takes now (lane 0 always: <= S tokens <= the FIFO)
        to.head = lds_load_volatile(sb + ZP_CTRL + ZPC_HEAD);
        if (!(alive = to.room(rdl(cnt, 0)))) return B;
        const uint32_t room = ZP_TOKQ - (to.tail - to.head);
        const uint64_t fits = __ballot(lane <= first && incl <= room);
        const uint32_t last = 63u - (uint32_t)__builtin_clzll(fits);  // lanes 0..last (fits is a prefix)
        const uint32_t n = lane <= last ? cnt : 0u;
        const uint32_t total = rdl(incl, last);
        ZDIAG(dg[4] += total;)
        {
            const uint32_t pe = (uint32_t)__shfl_up((int)xs, 1, 64);
            uint32_t p = lane ? pe : B, j = 0;
            while (__ballot(j < n)) {
                ZDIAG(dg[5]++;)
                const ZLane d = zp_decode_at(j < n ? p : B, WIN, wb, LLUT, DLUT, lt, dt);
                lds32(j < n ? sb + ZP_FIFO + 4 * ((to.tail + off + j) & (ZP_TOKQ - 1)) : sb + ZP_TRASH + 4 * lane) = d.tok;
                p += j < n ? d.adv : 0u;
                j++;
            }
        }
        to.tail += total;
        lds_store_volatile(sb + ZP_CTRL + ZPC_TAIL, to.tail);
        const uint32_t nB = rdl(xs, last);
        // next segment length from this round's bits per token
        if (total) {
            const uint32_t bpt = ((nB - B) * ZP_SEGTOK + total - 1) / total;
            sbits = bpt < 64 ? 64u : bpt > ZP_SMAX ? ZP_SMAX : (bpt + 7) & ~7u;
        }
        if (last == first && (ends >> first) & 1) {  // this round reached the end of the block
            const uint32_t f = rdl(fl, first);
            if (f == ZK_BAD) bad = rdl(ec, first);
            return nB;
        }
        B = nB;
    }
}

__device__ __forceinline__ void zp_producer(const ZStream& t, const uint8_t* src, uint32_t sb, uint32_t lane, uint32_t si) {
    const uint32_t LENS = sb + ZP_LENS, NEXT = sb + ZP_NEXT, LLUT = sb + ZP_LLUT, DLUT = sb + ZP_DLUT;
    BitIn bi{{src + t.src_off, sb + ZP_WIN, 0, lane}, 0ull, 0, 0, rfl(t.csize)};
    bi.win.load(0);
    HTab lt{0, 0, 0, sb + ZP_LSYMS}, dt{0, 0, 0, sb + ZP_DSYMS};
    TokOut to{0, 0, sb, lane};
    uint32_t bad = 0, final = 0;
    bool alive = true;
    uint32_t sbits = 128;  // segment length of the next macro-round
    ZDIAG(const uint64_t c0 = __builtin_amdgcn_s_memtime(); uint64_t chdr = 0, cdata = 0; uint32_t nblocks = 0; uint32_t dg[6] = {0, 0, 0, 0, 0, 0};)
    bi.refill();
    if (t.kind == ZS_ZLIB) {
        const uint32_t cmf = bi.bits(8), flg = bi.bits(8);
        if ((cmf & 15) != 8 || (cmf >> 4) > 7 || (flg & 0x20) || ((cmf << 8) | flg) % 31) bad = 10;
    }
    while (!bad && !final && alive) {
        bi.refill();
        final = bi.bits(1);
        const uint32_t type = bi.bits(2);
        if (type == 0) {  // stored: the consumer copies the bytes from the input
            bi.bits(bi.cnt & 7);
            bi.refill();
            const uint32_t len = bi.bits(16), nlen = bi.bits(16);
            if ((len ^ 0xffffu) != nlen) { bad = 11; break; }
            const uint32_t q = bi.ipos - bi.cnt / 8;  // the next byte of the input (buffered ones rewound)
            if (q + len > bi.ilen) { bad = 12; break; }
            if (len) alive = to.put_lanes(3ull, lane ? q : (0x80000000u | len));
            bi.ipos = q + len;
            bi.buf = 0;
            bi.cnt = 0;
            continue;
        }
        if (type == 3) { bad = 13; break; }
        ZDIAG(const uint64_t ch0 = __builtin_amdgcn_s_memtime(); nblocks++;)
        if (type == 1) {
            for (uint32_t s2 = lane; s2 < 320; s2 += 64)
                zlds[LENS + s2] = s2 < 144 ? 8 : s2 < 256 ? 9 : s2 < 280 ? 7 : s2 < 288 ? 8 : 5;
            __builtin_amdgcn_wave_barrier();
            build_table(lt, LENS, 288, lane, NEXT);
            build_table(dt, LENS + 288, 30, lane, NEXT);
        } else {
            bi.refill();
            const uint32_t hlit = bi.bits(5) + 257, hdist = bi.bits(5) + 1, hclen = bi.bits(4) + 4;
            if (hlit > 286 || hdist > 30) { bad = 14; break; }
            for (uint32_t s2 = lane; s2 < 19; s2 += 64) zlds[LENS + s2] = 0;
            __builtin_amdgcn_wave_barrier();
            for (uint32_t k = 0; k < hclen; k++) {
                bi.refill();
                const uint32_t v = bi.bits(3);
                if (lane == 0) zlds[LENS + c_clord[k]] = (uint8_t)v;
            }
            __builtin_amdgcn_wave_barrier();
            HTab ct{0, 0, 0, sb + ZP_LSYMS};
            if (!build_table(ct, LENS, 19, lane, NEXT)) { bad = 15; break; }
            uint32_t k = 0, prev = 0;
            while (k < hlit + hdist) {
                bi.refill();
                const int sym = decode_sym(ct, bi, lane);
                if (sym < 0) { bad = 16; break; }
                uint32_t rep = 1, val = (uint32_t)sym;
                if (sym == 16) {
                    if (k == 0) { bad = 17; break; }
                    rep = 3 + bi.bits(2); val = prev;
                } else if (sym == 17) { rep = 3 + bi.bits(3); val = 0; }
                else if (sym == 18) { rep = 11 + bi.bits(7); val = 0; }
                if (k + rep > hlit + hdist) { bad = 18; break; }
                for (uint32_t r = lane; r < rep; r += 64) zlds[LENS + 19 + k + r] = (uint8_t)val;
                __builtin_amdgcn_wave_barrier();
                k += rep;
                prev = val;
            }
            if (bad) break;
            for (uint32_t s2 = lane; s2 < 320; s2 += 64) {
                const uint8_t v = s2 < hlit + hdist ? zlds[LENS + 19 + s2] : 0;
                __builtin_amdgcn_wave_barrier();
                zlds[LENS + s2] = v;
            }
            __builtin_amdgcn_wave_barrier();
            {
                const uint8_t dv = lane < hdist ? zlds[LENS + hlit + lane] : 0;
                __builtin_amdgcn_wave_barrier();
                for (uint32_t s2 = hlit + lane; s2 < ZLENS; s2 += 64) zlds[LENS + s2] = 0;
                __builtin_amdgcn_wave_barrier();
                if (lane < 32) zlds[LENS + 288 + lane] = dv;
                __builtin_amdgcn_wave_barrier();
            }
            if (!build_table(lt, LENS, 288, lane, NEXT)) { bad = 19; break; }
            if (!build_table(dt, LENS + 288, 30, lane, NEXT)) { bad = 20; break; }
        }
        build_lut<ZPLUT>(lt, LENS, LLUT, lane);
        build_lut<ZPLUT>(dt, LENS + 288, DLUT, lane);
        ZDIAG(const uint64_t cd0 = __builtin_amdgcn_s_memtime(); chdr += cd0 - ch0;)
        // block data: self-synchronizing macro-rounds
        const uint32_t bp = zp_huff_block(bi.ipos * 8 - bi.cnt, bi, to, sb, lane, lt, dt, bad, alive, sbits ZDIAG(, dg));
        ZDIAG(cdata += __builtin_amdgcn_s_memtime() - cd0;)
        // back to the bit reader at bp (block headers, stored blocks)
        bi.ipos = bp >> 3;
        bi.buf = 0;
        bi.cnt = 0;
        bi.refill();
        bi.bits(bp & 7);
        if (!bad && bi.consumed_bytes() > bi.ilen) bad = 26;
    }
    if (!bad) {  // RFC 1950 trailer: Adler-32 of the output, big-endian, at the next byte
        const uint32_t q = (bi.ipos * 8 - bi.cnt + 7) >> 3;
        if (q + 4 > bi.ilen) bad = 28;
        else lds_store_volatile(sb + ZP_CTRL + ZPC_ADLER, bi.win.byte(q) << 24 | bi.win.byte(q + 1) << 16 |
                                                              bi.win.byte(q + 2) << 8 | bi.win.byte(q + 3));
    }
    ZDIAG(if (si == 0 && lane == 0) printf("[zp producer] total %lu hdr %lu data %lu blocks %u rounds %u stepsA %u syncs %u stepsB %u tokens %u stepsC %u\n",
                                           (unsigned long)(__builtin_amdgcn_s_memtime() - c0), (unsigned long)chdr,
                                           (unsigned long)cdata, nblocks, dg[0], dg[1], dg[2], dg[3], dg[4], dg[5]);)
    if (alive) to.put(0xC0000000u | bad);
    lds_store_volatile(sb + ZP_CTRL + ZPC_DONE, 1);
}

__device__ __forceinline__ void zp_consumer(const ZStream& t, const uint8_t* src, uint8_t* dst, uint32_t sb, uint32_t lane,
                                            uint32_t* errp, uint32_t si) {
    OutRing<ZP_RINGB, true> o{sb + ZP_RING, dst + t.dst_off, 0, 0, t.dlen, lane, sb + ZP_TRASH + 256};
    const uint8_t* in = src + t.src_off;
    const uint32_t FLAG = sb + ZP_FLAG;
    uint32_t head = 0, code = 0;
    bool done = false;
    ZDIAG(const uint64_t c0 = __builtin_amdgcn_s_memtime(); uint64_t cwait = 0, cpar = 0; uint32_t nbatch = 0, nchunk = 0, njump = 0;)
    while (!done) {
        uint32_t tail;
        ZDIAG(const uint64_t w0 = __builtin_amdgcn_s_memtime();)
        // a batch of >= ZP_BATCH tokens: the output steps are 64 bytes whatever the batch
        while ((tail = lds_load_volatile(sb + ZP_CTRL + ZPC_TAIL)) - head < ZP_BATCH &&
               !lds_load_volatile(sb + ZP_CTRL + ZPC_DONE))
            __builtin_amdgcn_s_sleep(2);
        if (tail == head) tail = lds_load_volatile(sb + ZP_CTRL + ZPC_TAIL);  // DONE seen: the end token is in
        ZDIAG(const uint64_t w1 = __builtin_amdgcn_s_memtime(); cwait += w1 - w0; nbatch++;)
        const uint32_t n = tail - head < 64 ? tail - head : 64u;
        const uint32_t tq = lds32(sb + ZP_FIFO + 4 * ((head + lane) & (ZP_TOKQ - 1)));
        const uint32_t tok = lane < n ? tq : 0xC0000000u;
        const uint32_t typ = tok >> 30;
        const uint64_t special = __ballot(typ >= 2);  // stored runs, the end token, lanes >= n
        const uint32_t k = special ? (uint32_t)__builtin_ctzll(special) : 64u;
        if (k) {
            // tokens [0, k), literals and matches, all at once: output offsets by a prefix sum,
            // then 64 output bytes per step, each lane finding its token (a flag per token
            // start, ballot, mbcnt) and its byte (the literal, the ring below this step, or
            // a lane of this step: pointer jumping over in-step sources)
            const bool act = lane < k;
            const uint32_t len = !act ? 0u : typ == 0 ? 1u : ((tok >> 16) & 0x3FFFu) + 3;
            const uint32_t end = wave_incl_add(len, lane), start = end - len;
            const uint32_t T = rdl(end, 63);
            const uint32_t dist = (tok & 0xFFFFu) + 1;
            const uint32_t op0 = o.op;
            const bool far = act && typ == 1 && dist > op0 + start;  // before the stream start
            if (__ballot(far) || T > o.olen - op0) {
                code = __ballot(act && typ == 1) ? 25u : 22u;
                done = true;
            } else {
                uint32_t base = 0;
                for (uint32_t cb = 0; cb < T; cb += 64) {
                    ZDIAG(nchunk++;)
                    zlds[FLAG + lane] = 0;
                    const uint32_t rs = start - cb;
                    zlds[act && rs < 64 ? FLAG + rs : FLAG + 64 + lane] = 1;
                    const uint32_t f = zlds[FLAG + lane];
                    const uint64_t M = __ballot(f != 0);
                    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0));
                    const uint32_t idx = base + below + f - 1;
                    base += (uint32_t)__popcll(M);
                    const uint32_t p = cb + lane;
                    const uint32_t ttok = (uint32_t)__shfl((int)tok, (int)idx, 64);
                    const bool valid = p < T, ismatch = (ttok >> 30) == 1;
                    const uint32_t dist = (ttok & 0xFFFFu) + 1;
                    const uint32_t s = p - dist;  // source offset (from op0; may be < 0)
                    uint32_t rv = o.ring(op0 + s);
                    // a source more than a ring back lies below `flushed` (< 256 bytes stay
                    // unflushed after a step): wait for this wave's stores, read it from HBM
                    const bool far = valid && ismatch && dist > ZP_RINGB - 64;
                    if (__ballot(far)) {
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                        const uint32_t hv = *(const __attribute__((address_space(1))) uint8_t*)(o.out + (far ? op0 + s : 0u));
                        rv = far ? hv : rv;
                    }
                    uint32_t v = ismatch ? rv : (ttok & 255u);
                    bool pend = valid && ismatch && (int32_t)s >= (int32_t)cb;
                    uint32_t ptr = s - cb;
                    while (__ballot(pend)) {
                        ZDIAG(njump++;)
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
            }
        }
        ZDIAG(cpar += __builtin_amdgcn_s_memtime() - w1;)
        uint32_t used = k;
        if (!done && k < n) {
            const uint32_t tk = rdl(tok, k);
            if (tk >> 30 == 2) {  // a stored run: its input offset follows (in this batch unless k == 63)
                if (k + 1 < n) {
                    const uint32_t len = tk & 0xFFFFu, q = rdl(tok, k + 1);
                    if (len > o.olen - o.op) { code = 12; done = true; }
                    else {
                        for (uint32_t kk = 0; kk < len; kk += 64) {
                            const uint32_t nb = len - kk < 64 ? len - kk : 64;
                            const uint32_t v = in[q + kk + lane];  // (the input has slack after every stream)
                            o.put_if(lane < nb, o.op + kk + lane, v);
                            o.flush(o.op + kk + nb);
                        }
                        o.op += len;
                    }
                    used = k + 2;
                }
            } else {
                code = tk & 0xFFu;
                done = true;
                used = k + 1;
            }
        }
        head += used;
        lds_store_volatile(sb + ZP_CTRL + ZPC_HEAD, head);
        if (done && code) lds_store_volatile(sb + ZP_CTRL + ZPC_ABORT, 1);
    }
    if (!code && o.op != o.olen) code = 27;
    o.finish();
    // the zlib trailer (stored by the producer before its end token): java.util.zip's
    // Inflater fails such a stream too
    if (!code && o.adler32() != lds_load_volatile(sb + ZP_CTRL + ZPC_ADLER)) code = 29;
    if (lane == 0) *errp = code;
    ZDIAG(if (si == 0 && lane == 0) printf("[zp consumer] total %lu wait %lu parallel %lu batches %u chunks %u jumps %u\n",
                                           (unsigned long)(__builtin_amdgcn_s_memtime() - c0), (unsigned long)cwait,
                                           (unsigned long)cpar, nbatch, nchunk, njump);)
}

__global__ __launch_bounds__(64 * 2 * ZP_STREAMS) void k_zarr_inflate2(const ZStream* __restrict__ st, uint32_t n,
                                                                       const uint8_t* __restrict__ src,
                                                                       uint8_t* __restrict__ dst,
                                                                       uint32_t* __restrict__ err) {
    const uint32_t lane = threadIdx.x & 63, w = rfl(threadIdx.x >> 6);
    const uint32_t s = w >> 1, si = blockIdx.x * ZP_STREAMS + s;
    const uint32_t sb = s * ZP_BYTES;
    if (lane < 8) lds32(sb + ZP_CTRL + 4 * lane) = 0;
    __syncthreads();
    if (si >= n) return;
    const ZStream t = st[si];
    if (w & 1) zp_consumer(t, src, dst, sb, lane, err + si, si);
    else zp_producer(t, src, sb, lane, si);
}

// ------------------------------------------------------------------------------ stored
__global__ __launch_bounds__(256) void k_zarr_copy(const ZStream* __restrict__ st, uint32_t n,
                                                   const uint8_t* __restrict__ src,
                                                   uint8_t* __restrict__ dst, uint32_t* __restrict__ err) {
    const uint32_t lane = threadIdx.x & 63, w = rfl(threadIdx.x >> 6);  // wave-uniform (SGPR) state
    const uint32_t si = blockIdx.x * ZWAVES + w;
    if (si >= n) return;
    const ZStream t = st[si];
    const uint8_t* in = src + t.src_off;
    uint8_t* out = dst + t.dst_off;
    const uint32_t len = t.dlen;
    uint32_t k = 0;
    if ((((uintptr_t)out) & 3) == 0)
        for (; k + 256 <= len; k += 256) {
            const uint32_t v = ld_u32_unaligned(in + k + 4 * lane);
            *(uint32_t*)(out + k + 4 * lane) = v;
        }
    for (; k < len; k += 64)
        if (k + lane < len) out[k + lane] = in[k + lane];
    if (lane == 0) err[si] = t.csize < t.dlen ? 30u : 0u;
}

// ------------------------------------------------------------------------------- place
// One workgroup per (chunk, band of ZP_ROWS chunk rows).  Blosc byte-unshuffle (typesize ts
// within blocks of `blocksize` bytes) + copy into the pitched plane (samples stay in the
// array's byte order); missing chunks get the fill bytes.  Fast path: each thread makes one
// aligned 16-byte group of a plane row (16 / bpp samples): unshuffled chunks are one 16-byte
// load, shuffled ones one load of 16 / bpp bytes from each byte plane, interleaved with byte
// permutes (v_perm_b32).  Groups straddling a blosc block, row tails and unaligned rows take
// the sample-by-sample path.
constexpr uint32_t ZP_ROWS = 16;

__device__ __forceinline__ uint32_t zperm(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);  // bytes 0-3 of lo, 4-7 of hi
}

// byte j of sample e of the chunk (after unshuffling; bit: the bit-shuffle layout of
// oracle/zarr_oracle.c -- a block of n = bsize / ts elements, n % 8 == 0, is ts * 8 bit rows of
// n / 8 bytes, row j * 8 + k holding bit k of byte j of every element; other blocks are raw)
__device__ __forceinline__ uint32_t zsample_byte(const uint8_t* s, uint32_t ts, uint32_t bs, uint32_t nb,
                                                 uint32_t e, uint32_t bpp, uint32_t j, bool bit = false) {
    if (bit) {
        const uint32_t B = e * bpp + j, blk = B / bs, within = B - blk * bs;
        const uint32_t bsize = nb - blk * bs < bs ? nb - blk * bs : bs, ne = bsize / ts;
        if (bsize < ts || (ne & 7u) || within >= ne * ts) return s[B];
        const uint32_t i = within / ts, jj = within - i * ts, row = ne >> 3;
        const uint8_t* r = s + (size_t)blk * bs + (size_t)jj * 8 * row + (i >> 3);
        uint32_t v = 0;
        for (uint32_t k = 0; k < 8; k++) v |= ((r[(size_t)k * row] >> (i & 7u)) & 1u) << k;
        return v;
    }
    if (ts <= 1) return s[(size_t)e * bpp + j];
    const uint32_t B = e * bpp + j, blk = B / bs, within = B - blk * bs;
    const uint32_t bsize = nb - blk * bs < bs ? nb - blk * bs : bs;
    const uint32_t ne = bsize / ts;
    return s[within < ne * ts ? blk * bs + (within % ts) * ne + within / ts : B];
}

__global__ __launch_bounds__(256) void k_zarr_place(const ZChunk* __restrict__ ch, uint32_t bands,
                                                    const ZPlane* __restrict__ planes,
                                                    const uint8_t* __restrict__ scratch,
                                                    const uint8_t* __restrict__ input) {
    const ZChunk c = ch[blockIdx.x / bands];
    const ZPlane& zp = planes[c.plane];
    uint8_t* const plane = zp.dev;
    const int64_t pitch = zp.pitch;
    const int32_t sx = zp.sx, sy = zp.sy, cw = zp.cw, chh = zp.chh;
    const uint32_t bpp = zp.bpp;
    const uint64_t fill = zp.fill;
    const uint32_t band = blockIdx.x % bands;
    const int32_t r0 = (int32_t)(band * ZP_ROWS);
    if (r0 >= chh) return;  // bands cover the tallest chunk of the set
    const int32_t w = sx - c.x0 < cw ? sx - c.x0 : cw;
    const int32_t h = sy - c.y0 < chh ? sy - c.y0 : chh;
    const int32_t r1 = r0 + (int32_t)ZP_ROWS < h ? r0 + (int32_t)ZP_ROWS : h;
    const uint8_t* s = (c.flags & ZC_INPUT ? input : scratch) + c.src;
    const uint32_t ts = c.typesize, bs = c.blocksize, nb = c.nbytes;
    const bool missing = (c.flags & ZC_MISSING) != 0;
    const bool bit = (c.flags & ZC_BITSHUF) != 0;
    const uint32_t G = 16 / bpp;  // samples per 16-byte group
    uint8_t* const base = plane + (int64_t)c.y0 * pitch + (int64_t)c.x0 * bpp;
    const bool aligned = ((((uintptr_t)base) | (uintptr_t)pitch) & 15) == 0;
    if (bit && !missing) {
        // bit shuffle: a thread makes 8 samples of a row (8 elements share each bit-row byte):
        // per byte j of the sample, the 8 bit rows' bytes -> an 8 x 8 bit transpose
        const int32_t w8 = (ts == bpp && (cw & 7) == 0) ? (w & ~7) : 0;
        const int32_t groups = w8 >> 3, total = (r1 - r0) * groups;
        for (int32_t g = (int32_t)threadIdx.x; g < total; g += 256) {
            const int32_t rr = g / groups, r = r0 + rr, col = 8 * (g - rr * groups);
            const uint32_t e = (uint32_t)r * (uint32_t)cw + (uint32_t)col;
            const uint32_t B = e * bpp, blk = B / bs;
            const uint32_t bsize = nb - blk * bs < bs ? nb - blk * bs : bs, ne = bsize / ts;
            uint8_t* o = base + (int64_t)r * pitch + (int64_t)col * bpp;
            const uint32_t i = (B - blk * bs) / ts;  // element index in the block (multiple of 8)
            if (bsize < ts || (ne & 7u) || i + 8 > ne) {
                for (uint32_t q = 0; q < 8 * bpp; q++) o[q] = (uint8_t)zsample_byte(s, ts, bs, nb, e + q / bpp, bpp, q % bpp, true);
                continue;
            }
            const uint32_t row = ne >> 3;
            const uint8_t* rb = s + (size_t)blk * bs + (i >> 3);
            for (uint32_t j = 0; j < bpp; j++) {
                // x byte k = bit row (j, k)'s byte: bit m of it = bit k of element m's byte j
                uint64_t x = 0;
                for (uint32_t k = 0; k < 8; k++) x |= (uint64_t)rb[(size_t)(j * 8 + k) * row] << (8 * k);
                // 8 x 8 bit transpose (delta swaps): afterwards byte m, bit k = old byte k, bit m
                uint64_t tt = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull; x ^= tt ^ (tt << 7);
                tt = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull; x ^= tt ^ (tt << 14);
                tt = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull; x ^= tt ^ (tt << 28);
                for (uint32_t m = 0; m < 8; m++) o[m * bpp + j] = (uint8_t)(x >> (8 * m));
            }
        }
        for (int32_t r = r0; r < r1; r++) {  // row tails (and chunks whose width is not 8k)
            uint8_t* o = base + (int64_t)r * pitch;
            for (int32_t col = w8 + (int32_t)threadIdx.x; col < w; col += 256) {
                const uint32_t e = (uint32_t)r * (uint32_t)cw + (uint32_t)col;
                for (uint32_t j = 0; j < bpp; j++) o[(int64_t)col * bpp + j] = (uint8_t)zsample_byte(s, ts, bs, nb, e, bpp, j, true);
            }
        }
        return;
    }
    const bool fast = aligned && (ts <= 1 || ts == bpp) && bpp <= 4;
    const int32_t wg = fast ? (w / (int32_t)G) * (int32_t)G : 0;  // samples in whole groups
    if (wg > 0) {
        const int32_t groups = wg / (int32_t)G, total = (r1 - r0) * groups;
        for (int32_t g = (int32_t)threadIdx.x; g < total; g += 256) {
            const int32_t rr = g / groups, r = r0 + rr, col = (int32_t)G * (g - rr * groups);
            uint4 o;
            if (missing) {
                uint32_t f = 0;
                for (uint32_t j = 0; j < 4; j++) f |= (uint32_t)(fill >> (8 * (j % bpp)) & 0xffu) << (8 * j);
                o = make_uint4(f, f, f, f);
            } else {
                const uint32_t e = (uint32_t)r * (uint32_t)cw + (uint32_t)col;
                if (ts <= 1 || bpp == 1) {
                    __builtin_memcpy(&o, s + (size_t)e * bpp, 16);
                } else {
                    const uint32_t B = e * bpp, blk = B / bs;
                    const uint32_t bsize = nb - blk * bs < bs ? nb - blk * bs : bs;
                    const uint32_t ne = bsize / ts, ie = (B - blk * bs) / ts;
                    if (ie + G > ne) {  // the group straddles a block (or its leftover bytes)
                        uint32_t v[4] = {0, 0, 0, 0};
                        for (uint32_t q = 0; q < 16; q++)
                            v[q >> 2] |= zsample_byte(s, ts, bs, nb, e + q / bpp, bpp, q % bpp) << (8 * (q & 3));
                        o = make_uint4(v[0], v[1], v[2], v[3]);
                    } else {
                        const uint8_t* q = s + (size_t)blk * bs + ie;
                        if (bpp == 2) {  // 8 samples: 8 bytes of each byte plane
                            uint2 p0, p1;
                            __builtin_memcpy(&p0, q, 8);
                            __builtin_memcpy(&p1, q + ne, 8);
                            o = make_uint4(zperm(p1.x, p0.x, 0x05010400u), zperm(p1.x, p0.x, 0x07030602u),
                                           zperm(p1.y, p0.y, 0x05010400u), zperm(p1.y, p0.y, 0x07030602u));
                        } else {  // bpp == 4: 4 samples, a 4 x 4 byte transpose
                            uint32_t a, b2, c2, d;
                            __builtin_memcpy(&a, q, 4);
                            __builtin_memcpy(&b2, q + ne, 4);
                            __builtin_memcpy(&c2, q + 2 * ne, 4);
                            __builtin_memcpy(&d, q + 3 * ne, 4);
                            const uint32_t t0 = zperm(b2, a, 0x05010400u), t1 = zperm(d, c2, 0x05010400u);
                            const uint32_t t2 = zperm(b2, a, 0x07030602u), t3 = zperm(d, c2, 0x07030602u);
                            o = make_uint4(zperm(t1, t0, 0x05040100u), zperm(t1, t0, 0x07060302u),
                                           zperm(t3, t2, 0x05040100u), zperm(t3, t2, 0x07060302u));
                        }
                    }
                }
            }
            *(uint4*)(base + (int64_t)r * pitch + (int64_t)col * bpp) = o;
        }
    }
    for (int32_t r = r0; r < r1; r++) {  // the rest of every row, sample by sample
        uint8_t* o = base + (int64_t)r * pitch;
        for (int32_t col = wg + (int32_t)threadIdx.x; col < w; col += 256) {
            const uint32_t e = (uint32_t)r * (uint32_t)cw + (uint32_t)col;
            for (uint32_t j = 0; j < bpp; j++) {
                const uint32_t v = missing ? (uint32_t)(fill >> (8 * j)) & 0xffu : zsample_byte(s, ts, bs, nb, e, bpp, j);
                o[(int64_t)col * bpp + j] = (uint8_t)v;
            }
        }
    }
}

hipError_t launch_zarr_decode(hipStream_t st, const ZStream* d_streams, const uint32_t* counts,
                              const uint8_t* src, uint8_t* scratch, uint8_t* zstd_lit, uint32_t* err) {
    // streams are ordered by kind: lz4, inflate, copy, blosclz, zstd
    uint32_t first = 0;
    for (uint32_t k = 0; k < ZS_NKINDS; k++) {
        const uint32_t n = counts[k];
        const ZStream* s = d_streams + first;
        uint32_t* e = err + first;
        first += n;
        if (!n) continue;
        const dim3 g((n + ZWAVES - 1) / ZWAVES), b(64 * ZWAVES);
        switch (k) {
        case ZS_LZ4: hipLaunchKernelGGL(k_zarr_lz4, g, b, ZWAVES * ZL_BYTES, st, s, n, src, scratch, e); break;
        case ZS_ZLIB:
            if (getenv("PBX_INFLATE_1WAVE")) {  // the single-wave decoder (A/B)
                static std::once_flag once[64];
                int dev = 0;
                (void)hipGetDevice(&dev);
                std::call_once(once[dev & 63], [] {
                    (void)hipFuncSetAttribute((const void*)k_zarr_inflate,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                });
                hipLaunchKernelGGL(k_zarr_inflate, g, b, ZWAVES * (ZI_BYTES + ZWIN), st, s, n, src, scratch, e);
            } else
                hipLaunchKernelGGL(k_zarr_inflate2, dim3((n + ZP_STREAMS - 1) / ZP_STREAMS), dim3(128 * ZP_STREAMS),
                                   ZP_STREAMS * ZP_BYTES, st, s, n, src, scratch, e);
            break;
        case ZS_COPY: hipLaunchKernelGGL(k_zarr_copy, g, b, 0, st, s, n, src, scratch, e); break;
        case ZS_BLOSCLZ: hipLaunchKernelGGL(k_zarr_blosclz, g, b, ZWAVES * ZL_BYTES, st, s, n, src, scratch, e); break;
        default: {
            hipError_t r = launch_zarr_zstd(st, s, n, src, scratch, zstd_lit, e);
            if (r != hipSuccess) return r;
        }
        }
    }
    return hipGetLastError();
}

hipError_t launch_zarr_place(hipStream_t st, const ZChunk* d_chunks, uint32_t nchunks,
                             const ZPlane* d_planes, int32_t max_chunk_y, const uint8_t* scratch,
                             const uint8_t* input) {
    const uint32_t bands = ((uint32_t)max_chunk_y + ZP_ROWS - 1) / ZP_ROWS;
    if (!nchunks) return hipSuccess;
    hipLaunchKernelGGL(k_zarr_place, dim3(nchunks * bands), dim3(256), 0, st, d_chunks, bands,
                       d_planes, scratch, input);
    return hipGetLastError();
}

}  // namespace pbx
