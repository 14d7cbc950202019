// deflate_seg.h — one deflate segment per workgroup: LZ77 match finding in LDS, dynamic /
// fixed / stored block choice, Huffman code construction and parallel bit packing.
//
// Replaces the compression half of writeImage("png") (TileRequestHandler.java:176-199:
// Bio-Formats APNGWriter -> java.util.zip.DeflaterOutputStream, level 6).  Parity is at
// the decoded-pixel level (BASELINE.json north_star): the stream is valid RFC 1950/1951
// and inflates to exactly the filtered scanlines; the compressed bytes differ from zlib's.
//
// The workgroup's work is written as a sequence of PHASES separated by workgroup barriers.
// A phase is a function of (tid, LDS state) that only communicates with other threads
// through LDS atomics that commute (min / add / or) or through disjoint writes, so the
// phases are deterministic.  The HIP kernel runs them with __syncthreads() in between;
// tests/ also run them on the CPU (csrc/emu.cpp) thread by thread to check the algorithm
// without a GPU.  Scans between phases are implemented separately for each side
// (wave shuffles on the device, a loop in the emulator) with identical results.
//
// Parse: each wave owns a SUB-byte sub-segment and walks it greedily (with zlib-style
// one-step lazy matching) in batches of 64 positions: every lane evaluates the match at
// one position (capped at CAP bytes), the wave picks the greedy path through the batch with
// ballot/ctz, and a chosen match that reaches the cap is extended by one wave-wide compare
// of 256 bytes.  The result is exactly the sequential greedy parse of the sub-segment
// (ph_parse_emu is its scalar twin).  Matches end inside their sub-segment.  Tokens are
// kept as per-wave match lists; literals are the positions no match covers, so the later
// phases (histogram, bit counts, bit writing) walk fixed 32-position thread chunks.
#pragma once
#include "pbx_common.h"

namespace pbx {

template <int NT_, int SEG_, int WIN_, int HBITS_>
struct DeflateCfg {
    static constexpr int NT = NT_;        // threads per workgroup
    static constexpr int SEG = SEG_;      // max segment bytes
    static constexpr int WIN = WIN_;      // max window bytes before the segment
    static constexpr int HBITS = HBITS_;  // hash table bits
    static constexpr int CH = SEG / NT;   // positions per thread chunk (emission phases)
    static constexpr int NW = NT / 64;    // waves
    static constexpr int SUB = SEG / NW;  // positions parsed by one wave
    static constexpr int MAXMW = 256;     // matches kept per wave (then literals only)
    static constexpr int CAP = 32;        // per-lane match length before the wave extends it
    static constexpr int BUFW = (WIN + SEG + 16) / 4;
    static constexpr int OUTW = (SEG + 64) / 4;
    static constexpr int HSIZE = 1 << HBITS;
    static constexpr int LOGNT = NT == 1024 ? 10 : NT == 512 ? 9 : NT == 256 ? 8 : 7;
    static_assert(SEG % NT == 0, "SEG must be a multiple of NT");
    static_assert(SUB <= 65536 && SUB % CH == 0, "sub-segments hold whole thread chunks");
    static_assert(WIN + SEG <= 32768, "deflate distances are limited to 32768");
    static_assert((1 << LOGNT) == NT, "NT must be a power of two in 128..1024");
    static_assert(NT >= 320, "ph_rank needs one thread per literal/length and distance symbol");
};

enum : int {
    M_NL = 0, M_ND, M_HLIT, M_HDIST, M_HCLEN, M_NRLE, M_BTYPE, M_HDRBITS, M_DATABITS, M_NBYTES,
    M_CRCOP, M_BLKBITS, M_OPK0,  // M_OPK0 .. M_OPK0+9: x^(8*CC*2^k)
    M_NMISC = M_OPK0 + 11
};

struct HuffWork {
    uint32_t w[2 * 288];  // weights, then depths
    uint32_t parent[2 * 288];
    uint32_t blc[16], next[16];
    uint32_t cllen[19], clcode[19], clfreq[19], clsort[19];
};

template <class C>
struct DeflateSmem {
    uint32_t buf[C::BUFW];            // window + segment bytes, zero padded
    uint32_t mpos[C::NW * C::MAXMW];  // per-wave matches: segment position | (len-3) << 16
    uint32_t mdist[C::NW * C::MAXMW]; // distance - 1
    union {
        uint32_t head[C::HSIZE];      // hash -> first position (atomicMin)
        uint32_t out[C::OUTW];        // packed output bits
    } u;
    uint32_t w_nm[C::NW];             // matches found by each wave
    uint32_t wtot[16];                // block-scan wave totals (device)
    uint32_t t_a[C::NT];              // bits -> exclusive prefix sum; then CRC partials
    uint32_t t_s1[C::NT], t_s2[C::NT], t_len[C::NT];  // Adler partials
    uint32_t lfreq[288], dfreq[32];
    uint32_t lcode[288], dcode[32];   // bit-reversed code | len << 16
    uint32_t lsort[288], dsort[32];
    uint32_t crc_table[256];
    HuffWork hw;
    uint32_t rle[320];                // code-length RLE symbols: sym | extra << 8
    uint32_t misc[M_NMISC];
};

// Per-segment parameters (uniform across the workgroup).
struct SegParams {
    uint64_t base;   // stream position of buf[0] (= segment start - wl)
    uint32_t wl;     // window bytes in buf before the segment
    uint32_t sl;     // segment bytes
    uint32_t rowlen; // repeating-row candidate distance (0 = none)
    uint32_t last;   // 1 if this segment ends the stream (BFINAL)
};

template <class C>
PBX_HD uint32_t lds_byte(const DeflateSmem<C>& S, uint32_t i) {
    return (S.buf[i >> 2] >> ((i & 3) * 8)) & 0xFFu;
}

// Unaligned little-endian 32-bit read from the byte buffer.
template <class C>
PBX_HD uint32_t lds_ld4(const DeflateSmem<C>& S, uint32_t i) {
    uint32_t w0 = S.buf[i >> 2], w1 = S.buf[(i >> 2) + 1];
    uint32_t sh = (i & 3) * 8;
    return sh ? (w0 >> sh) | (w1 << (32 - sh)) : w0;
}

template <class C>
PBX_HD uint32_t hash3(uint32_t v) {
    return ((v & 0xFFFFFFu) * 2654435761u) >> (32 - C::HBITS);
}

// ------------------------------------------------------------------------- phase: fill
// Src provides fill_word(p0, nb) -> up to 4 stream bytes starting at stream position p0.
template <class C, class Src>
PBX_HD void ph_fill(uint32_t tid, DeflateSmem<C>& S, const Src& src, const SegParams& sp) {
    const uint32_t nb = sp.wl + sp.sl, nw = (nb + 3) / 4;
    for (uint32_t k = tid; k < nw + 4; k += C::NT) {
        uint32_t v = 0;
        if (k < nw) {
            uint32_t take = nb - 4 * k;
            v = src.fill_word(sp.base + 4ull * k, take < 4 ? take : 4);
        }
        S.buf[k] = v;
    }
    for (uint32_t k = tid; k < (uint32_t)C::HSIZE; k += C::NT) S.u.head[k] = 0xFFFFFFFFu;
    if (tid < 288) S.lfreq[tid] = 0;
    if (tid < 32) S.dfreq[tid] = 0;
    if (tid < 256) S.crc_table[tid] = crc_table_entry(tid);
}

// ----------------------------------------------------------------------- phase: insert
template <class C, class Ops>
PBX_HD void ph_insert(uint32_t tid, DeflateSmem<C>& S, const SegParams& sp) {
    const uint32_t nb = sp.wl + sp.sl;
    for (uint32_t i = tid; i + 3 <= nb; i += C::NT) Ops::amin(&S.u.head[hash3<C>(lds_ld4(S, i))], i);
}

template <class C>
PBX_HD uint32_t match_len(const DeflateSmem<C>& S, uint32_t j, uint32_t a, uint32_t cur4,
                          uint32_t maxlen) {
    uint32_t x = lds_ld4(S, j) ^ cur4;
    uint32_t l;
    if (x) {
        l = (uint32_t)__builtin_ctz(x) >> 3;
    } else {
        l = 4;
        while (l < maxlen) {
            x = lds_ld4(S, j + l) ^ lds_ld4(S, a + l);
            if (x) { l += (uint32_t)__builtin_ctz(x) >> 3; break; }
            l += 4;
        }
    }
    return l < maxlen ? l : maxlen;
}

// ------------------------------------------------------------------------ phase: parse
// Minimum length worth coding at a distance: a 3-byte match 16 KiB back costs more bits
// than three literals (zlib's TOO_FAR rule, extended one step).
PBX_HD bool match_pays(uint32_t len, uint32_t dist) {
    return len >= 6 || (len >= 4 && dist <= 4096) || (len >= 3 && dist <= 256);
}

// Best match at segment position p (capped at CAP): candidates, in order, the previous
// byte (runs), the previous 2-byte sample, the same column one row up, and the first
// occurrence of the 3-byte hash.  Longest capped length wins; the first wins ties.
template <class C>
PBX_HD void eval_pos(const DeflateSmem<C>& S, const SegParams& sp, uint32_t p, uint32_t se,
                     uint32_t& L, uint32_t& D) {
    L = 0; D = 0;
    if (p >= se || se - p < 3) return;
    const uint32_t rem = se - p;
    const uint32_t maxlen = rem < 258 ? rem : 258;
    const uint32_t cap = maxlen < (uint32_t)C::CAP ? maxlen : (uint32_t)C::CAP;
    const uint32_t a = sp.wl + p;
    const uint32_t cur4 = lds_ld4(S, a);
    uint32_t cand[4];
    cand[0] = 1;
    cand[1] = 2;
    cand[2] = sp.rowlen > 2 ? sp.rowlen : 0;
    const uint32_t j = S.u.head[hash3<C>(cur4)];
    cand[3] = j < a ? a - j : 0;
    for (int k = 0; k < 4; k++) {
        const uint32_t d = cand[k];
        if (d == 0 || d > a) continue;
        const uint32_t l = match_len(S, a - d, a, cur4, cap);
        if (l > L && match_pays(l, d)) { L = l; D = d; }
    }
}

// Full length of a match of distance D at position p that reached the cap (scalar form).
template <class C>
PBX_HD uint32_t extend_scalar(const DeflateSmem<C>& S, const SegParams& sp, uint32_t p,
                              uint32_t se, uint32_t L, uint32_t D) {
    const uint32_t rem = se - p;
    const uint32_t maxlen = rem < 258 ? rem : 258;
    if (L < (uint32_t)C::CAP || L >= maxlen) return L;
    const uint32_t a = sp.wl + p;
    // compare 4-byte words at offsets L + 4k, exactly like the wave-wide form
    for (uint32_t k = 0; k < 64; k++) {
        const uint32_t o = L + 4 * k;
        if (o >= maxlen) return maxlen;
        const uint32_t x = lds_ld4(S, a - D + o) ^ lds_ld4(S, a + o);
        if (x) {
            const uint32_t l = o + ((uint32_t)__builtin_ctz(x) >> 3);
            return l < maxlen ? l : maxlen;
        }
    }
    return maxlen;
}

template <class C>
PBX_HD void push_match(DeflateSmem<C>& S, uint32_t w, uint32_t& nm, uint32_t p, uint32_t L, uint32_t D) {
    if (nm < (uint32_t)C::MAXMW) {
        S.mpos[w * C::MAXMW + nm] = p | ((L - 3) << 16);
        S.mdist[w * C::MAXMW + nm] = D - 1;
        nm++;
    }
}

// Scalar twin of the wave parse (CPU emulator): identical batches, path and lazy rule.
template <class C>
PBX_HD void ph_parse_emu(uint32_t w, DeflateSmem<C>& S, const SegParams& sp) {
    const uint32_t ss = w * C::SUB;
    const uint32_t se = ss + C::SUB < sp.sl ? ss + C::SUB : sp.sl;
    uint32_t nm = 0, pos = ss;
    uint32_t Ls[64], Ds[64];
    while (pos < se) {
        uint64_t mask = 0;
        for (uint32_t l = 0; l < 64; l++) {
            eval_pos(S, sp, pos + l, se, Ls[l], Ds[l]);
            if (Ls[l] >= 3) mask |= 1ull << l;
        }
        uint32_t o = 0;
        while (o < 64) {
            const uint64_t m = mask >> o;
            if (!m) { o = 64; break; }
            const uint32_t k = o + (uint32_t)__builtin_ctzll(m);
            uint32_t L = Ls[k];
            const uint32_t D = Ds[k];
            if (k + 1 < 64 && Ls[k + 1] > L) { o = k + 1; continue; }  // lazy
            L = extend_scalar(S, sp, pos + k, se, L, D);
            push_match(S, w, nm, pos + k, L, D);
            o = k + L;
        }
        pos += o;
    }
    S.w_nm[w] = nm;
}

// Emit this thread's chunk of tokens in stream order: matches starting in the chunk
// (they may run past its end) and literals at positions no match covers.
template <class C, class F>
PBX_HD void walk_tokens(uint32_t tid, const DeflateSmem<C>& S, const SegParams& sp, F& f) {
    const uint32_t cs = tid * C::CH;
    if (cs >= sp.sl) return;
    const uint32_t ce = cs + C::CH < sp.sl ? cs + C::CH : sp.sl;
    const uint32_t w = cs / C::SUB;
    const uint32_t* mp = S.mpos + w * C::MAXMW;
    const uint32_t* md = S.mdist + w * C::MAXMW;
    const uint32_t nm = S.w_nm[w];
    // first match starting at or after cs
    uint32_t lo = 0, hi = nm;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((mp[mid] & 0xFFFFu) < cs) lo = mid + 1; else hi = mid;
    }
    uint32_t pos = cs;
    if (lo > 0) {
        const uint32_t pe = (mp[lo - 1] & 0xFFFFu) + (mp[lo - 1] >> 16) + 3;
        if (pe > pos) pos = pe;
    }
    for (uint32_t m = lo; m < nm && pos < ce; m++) {
        const uint32_t ms = mp[m] & 0xFFFFu;
        if (ms >= ce) break;
        for (; pos < ms; pos++) f.lit(lds_byte(S, sp.wl + pos));
        const uint32_t len = (mp[m] >> 16) + 3;
        f.match(len, md[m] + 1);
        pos = ms + len;
    }
    for (; pos < ce; pos++) f.lit(lds_byte(S, sp.wl + pos));
}

template <class C, class Ops>
struct HistF {
    DeflateSmem<C>& S;
    PBX_HD void lit(uint32_t b) { Ops::add(&S.lfreq[b], 1u); }
    PBX_HD void match(uint32_t len, uint32_t dist) {
        uint32_t s, e, v;
        len_code(len, s, e, v);
        Ops::add(&S.lfreq[s], 1u);
        dist_code(dist, s, e, v);
        Ops::add(&S.dfreq[s], 1u);
    }
};

// --------------------------------------------------------- phase: histogram + adler partial
template <class C, class Ops>
PBX_HD void ph_hist(uint32_t tid, DeflateSmem<C>& S, const SegParams& sp) {
    HistF<C, Ops> f{S};
    walk_tokens<C>(tid, S, sp, f);
    if (tid == 0) Ops::add(&S.lfreq[256], 1u);  // end of block
    // Adler-32 partial sums of this thread's chunk of the segment.
    const uint32_t cs = tid * C::CH;
    uint32_t s1 = 0, s2 = 0, n = 0;
    if (cs < sp.sl) {
        const uint32_t ce = cs + C::CH < sp.sl ? cs + C::CH : sp.sl;
        n = ce - cs;
        for (uint32_t p = cs; p < ce; p++) {
            uint32_t b = lds_byte(S, sp.wl + p);
            s1 += b;
            s2 += (ce - p) * b;
        }
        s1 %= ADLER_BASE;
        s2 %= ADLER_BASE;
    }
    S.t_s1[tid] = s1; S.t_s2[tid] = s2; S.t_len[tid] = n;
}

// Effective frequencies: every tree gets >= 2 used symbols (zlib's rule, so every decoder
// accepts the code): literal 0 and EOB, distances 0 and 1.
PBX_HD uint32_t eff_lfreq(const uint32_t* f, uint32_t s) {
    uint32_t v = f[s];
    return (s == 0 || s == 256) && v == 0 ? 1u : v;
}
PBX_HD uint32_t eff_dfreq(const uint32_t* f, uint32_t s) {
    uint32_t v = f[s];
    return s < 2 && v == 0 ? 1u : v;
}

// ------------------------------------------------------------ phase: rank (parallel sort)
template <class C>
PBX_HD void ph_rank(uint32_t tid, DeflateSmem<C>& S) {
    if (tid < 286) {
        const uint32_t s = tid, fs = eff_lfreq(S.lfreq, s);
        if (fs) {
            uint32_t rank = 0, nz = 0;
            for (uint32_t j = 0; j < 286; j++) {
                uint32_t fj = eff_lfreq(S.lfreq, j);
                nz += fj != 0;
                rank += fj != 0 && (fj < fs || (fj == fs && j < s));
            }
            S.lsort[rank] = s;
            if (s == 256) S.misc[M_NL] = nz;
        }
    } else if (tid >= 288 && tid < 288 + 30) {
        const uint32_t s = tid - 288, fs = eff_dfreq(S.dfreq, s);
        if (fs) {
            uint32_t rank = 0, nz = 0;
            for (uint32_t j = 0; j < 30; j++) {
                uint32_t fj = eff_dfreq(S.dfreq, j);
                nz += fj != 0;
                rank += fj != 0 && (fj < fs || (fj == fs && j < s));
            }
            S.dsort[rank] = s;
            if (s == 0) S.misc[M_ND] = nz;
        }
    }
}

// Length-limited Huffman code lengths (two-queue build + zlib's overflow repair).
// sorted: n >= 2 used symbols by ascending (freq, symbol).  lens[] is (re)written for
// the n symbols only; the caller zeroes the rest.
PBX_HD void huff_lengths(const uint32_t* freq_of_sorted_w, const uint32_t* sorted, uint32_t n,
                         uint32_t maxbits, uint32_t* lens, uint32_t lens_shift, HuffWork& hw) {
    uint32_t* w = hw.w;
    uint32_t* parent = hw.parent;
    for (uint32_t i = 0; i < n; i++) w[i] = freq_of_sorted_w[i];
    uint32_t li = 0, qi = n, nxt = n;
    for (uint32_t k = 0; k + 1 < n; k++) {
        uint32_t a, b;
        if (li < n && (qi >= nxt || w[li] <= w[qi])) a = li++; else a = qi++;
        if (li < n && (qi >= nxt || w[li] <= w[qi])) b = li++; else b = qi++;
        w[nxt] = w[a] + w[b];
        parent[a] = nxt;
        parent[b] = nxt;
        nxt++;
    }
    const uint32_t root = 2 * n - 2;
    w[root] = 0;
    for (uint32_t i = root; i-- > 0;) w[i] = w[parent[i]] + 1;  // depths
    for (uint32_t b = 0; b < 16; b++) hw.blc[b] = 0;
    int overflow = 0;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t d = w[i];
        if (d > maxbits) { d = maxbits; overflow++; }
        hw.blc[d]++;
    }
    while (overflow > 0) {
        uint32_t bits = maxbits - 1;
        while (hw.blc[bits] == 0) bits--;
        hw.blc[bits]--;
        hw.blc[bits + 1] += 2;
        hw.blc[maxbits]--;
        overflow -= 2;
    }
    uint32_t idx = 0;
    for (uint32_t bits = maxbits; bits >= 1; bits--)
        for (uint32_t c = hw.blc[bits]; c > 0; c--) lens[sorted[idx++]] = bits << lens_shift;
}

// Canonical codes from lengths stored as (len << 16) in codes[]; result: rev code | len << 16.
PBX_HD void huff_codes(uint32_t* codes, uint32_t nsym, uint32_t maxbits, HuffWork& hw) {
    for (uint32_t b = 0; b < 16; b++) hw.blc[b] = 0;
    for (uint32_t s = 0; s < nsym; s++) hw.blc[codes[s] >> 16]++;
    hw.blc[0] = 0;
    uint32_t code = 0;
    for (uint32_t b = 1; b <= maxbits; b++) {
        code = (code + hw.blc[b - 1]) << 1;
        hw.next[b] = code;
    }
    for (uint32_t s = 0; s < nsym; s++) {
        uint32_t l = codes[s] >> 16;
        if (l) codes[s] = bitrev(hw.next[l]++, l) | (l << 16);
    }
}

PBX_HD uint32_t rle_ebits(uint32_t sym) { return sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0; }

// ----------------------------------------------------------- phase: Huffman (one thread)
template <class C>
PBX_HD void ph_huff(uint32_t tid, DeflateSmem<C>& S, const SegParams& sp) {
    if (tid != 0) return;
    HuffWork& hw = S.hw;
    // literal/length tree
    const uint32_t nl = S.misc[M_NL], nd = S.misc[M_ND];
    for (uint32_t s = 0; s < 288; s++) S.lcode[s] = 0;
    for (uint32_t s = 0; s < 32; s++) S.dcode[s] = 0;
    // (weights are staged in hw.w itself; huff_lengths' copy is then a no-op)
    for (uint32_t i = 0; i < nl; i++) hw.w[i] = eff_lfreq(S.lfreq, S.lsort[i]);
    huff_lengths(hw.w, S.lsort, nl, 15, S.lcode, 16, hw);
    for (uint32_t i = 0; i < nd; i++) hw.w[i] = eff_dfreq(S.dfreq, S.dsort[i]);
    huff_lengths(hw.w, S.dsort, nd, 15, S.dcode, 16, hw);
    // data bits (dynamic and fixed)
    uint64_t dyn = 0, fix = 0;
    for (uint32_t s = 0; s < 286; s++) {
        uint32_t f = S.lfreq[s];
        if (!f) continue;
        uint32_t eb = s >= 257 ? len_sym_ebits(s) : 0;
        dyn += (uint64_t)f * ((S.lcode[s] >> 16) + eb);
        fix += (uint64_t)f * (fixed_lit_len(s) + eb);
    }
    for (uint32_t s = 0; s < 30; s++) {
        uint32_t f = S.dfreq[s];
        if (!f) continue;
        uint32_t eb = dist_sym_ebits(s);
        dyn += (uint64_t)f * ((S.dcode[s] >> 16) + eb);
        fix += (uint64_t)f * (5 + eb);
    }
    // HLIT / HDIST and the run-length coded code lengths
    uint32_t hlit = 286;
    while (hlit > 257 && (S.lcode[hlit - 1] >> 16) == 0) hlit--;
    uint32_t hdist = 30;
    while (hdist > 1 && (S.dcode[hdist - 1] >> 16) == 0) hdist--;
    const uint32_t ntot = hlit + hdist;
    for (uint32_t s = 0; s < 19; s++) hw.clfreq[s] = 0;
    uint32_t nr = 0;
    uint32_t i = 0;
    while (i < ntot) {
        uint32_t v = i < hlit ? S.lcode[i] >> 16 : S.dcode[i - hlit] >> 16;
        uint32_t run = 1;
        while (i + run < ntot) {
            uint32_t u = (i + run) < hlit ? S.lcode[i + run] >> 16 : S.dcode[i + run - hlit] >> 16;
            if (u != v) break;
            run++;
        }
        i += run;
        if (v == 0) {
            while (run >= 11) {
                uint32_t n = run < 138 ? run : 138;
                S.rle[nr++] = 18u | ((n - 11) << 8); hw.clfreq[18]++; run -= n;
            }
            if (run >= 3) { S.rle[nr++] = 17u | ((run - 3) << 8); hw.clfreq[17]++; run = 0; }
            while (run) { S.rle[nr++] = 0; hw.clfreq[0]++; run--; }
        } else {
            S.rle[nr++] = v; hw.clfreq[v]++; run--;
            while (run >= 3) {
                uint32_t n = run < 6 ? run : 6;
                S.rle[nr++] = 16u | ((n - 3) << 8); hw.clfreq[16]++; run -= n;
            }
            while (run) { S.rle[nr++] = v; hw.clfreq[v]++; run--; }
        }
    }
    // code-length code (19 symbols, max 7 bits); same two-symbol minimum as above
    uint32_t ncl = 0;
    for (uint32_t s = 0; s < 19; s++) hw.cllen[s] = 0;
    {
        uint32_t* cf = hw.clfreq;  // gets the dummies; only the code-length tree reads it
        uint32_t used = 0;
        for (uint32_t s = 0; s < 19; s++) used += cf[s] != 0;
        for (uint32_t s = 0; s < 19 && used < 2; s++) if (!cf[s]) { cf[s] = 1; used++; }
        // insertion sort by (freq, sym)
        for (uint32_t s = 0; s < 19; s++) {
            if (!cf[s]) continue;
            uint32_t k = ncl++;
            while (k > 0) {
                uint32_t t = hw.clsort[k - 1];
                if (cf[t] < cf[s] || (cf[t] == cf[s] && t < s)) break;
                hw.clsort[k] = t;
                k--;
            }
            hw.clsort[k] = s;
        }
        for (uint32_t k = 0; k < ncl; k++) hw.w[k] = cf[hw.clsort[k]];
        huff_lengths(hw.w, hw.clsort, ncl, 7, hw.clcode, 16, hw);
        for (uint32_t s = 0; s < 19; s++) if (!cf[s]) hw.clcode[s] = 0;
        huff_codes(hw.clcode, 19, 7, hw);
        for (uint32_t s = 0; s < 19; s++) hw.cllen[s] = hw.clcode[s] >> 16;
    }
    const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint32_t hclen = 19;
    while (hclen > 4 && hw.cllen[order[hclen - 1]] == 0) hclen--;
    uint64_t hdr = 3 + 5 + 5 + 4 + 3ull * hclen;
    for (uint32_t k = 0; k < nr; k++) {
        uint32_t sym = S.rle[k] & 0xFF;
        hdr += hw.cllen[sym] + rle_ebits(sym);
    }
    const uint64_t dyn_bits = hdr + dyn, fix_bits = 3 + fix;
    auto bytes_of = [&](uint64_t bits) -> uint64_t {
        return sp.last ? (bits + 7) / 8 : (bits + 3 + 7) / 8 + 4;
    };
    const uint64_t stored_bytes = 5ull + sp.sl;
    uint32_t btype = 2;
    uint64_t best = bytes_of(dyn_bits);
    if (bytes_of(fix_bits) <= best) { btype = 1; best = bytes_of(fix_bits); }
    if (stored_bytes <= best) { btype = 0; best = stored_bytes; }
    if (btype == 1) {
        for (uint32_t s = 0; s < 288; s++) S.lcode[s] = fixed_lit_len(s) << 16;
        for (uint32_t s = 0; s < 32; s++) S.dcode[s] = 5u << 16;
        huff_codes(S.lcode, 288, 15, hw);
        huff_codes(S.dcode, 32, 15, hw);
        S.misc[M_HDRBITS] = 3;
    } else if (btype == 2) {
        huff_codes(S.lcode, 288, 15, hw);
        huff_codes(S.dcode, 32, 15, hw);
        S.misc[M_HDRBITS] = (uint32_t)hdr;
    } else {
        S.misc[M_HDRBITS] = 0;
    }
    S.misc[M_BTYPE] = btype;
    S.misc[M_HLIT] = hlit;
    S.misc[M_HDIST] = hdist;
    S.misc[M_HCLEN] = hclen;
    S.misc[M_NRLE] = nr;
}

template <class C>
struct BitsF {
    const DeflateSmem<C>& S;
    uint32_t bits;
    PBX_HD void lit(uint32_t b) { bits += S.lcode[b] >> 16; }
    PBX_HD void match(uint32_t len, uint32_t dist) {
        uint32_t s, e, v;
        len_code(len, s, e, v);
        bits += (S.lcode[s] >> 16) + e;
        dist_code(dist, s, e, v);
        bits += (S.dcode[s] >> 16) + e;
    }
};

// --------------------------------------------------------- phase: per-thread bit counts
template <class C>
PBX_HD void ph_bits(uint32_t tid, DeflateSmem<C>& S, const SegParams& sp) {
    for (uint32_t k = tid; k < (uint32_t)C::OUTW; k += C::NT) S.u.out[k] = 0;
    uint32_t bits = 0;
    if (S.misc[M_BTYPE] != 0) {
        BitsF<C> f{S, 0};
        walk_tokens<C>(tid, S, sp, f);
        bits = f.bits;
    }
    S.t_a[tid] = bits;
}

template <class C, class Ops>
struct BitWriter {
    uint32_t* out;
    uint32_t pos;
    PBX_HD void put(uint32_t v, uint32_t n) {
        if (!n) return;
        const uint32_t w = pos >> 5, sh = pos & 31;
        Ops::aor(&out[w], v << sh);
        if (sh + n > 32) Ops::aor(&out[w + 1], v >> (32 - sh));
        pos += n;
    }
};

template <class C, class Ops>
struct WriteF {
    const DeflateSmem<C>& S;
    BitWriter<C, Ops> bw;
    PBX_HD void lit(uint32_t b) { uint32_t c = S.lcode[b]; bw.put(c & 0xFFFF, c >> 16); }
    PBX_HD void match(uint32_t len, uint32_t dist) {
        uint32_t s, e, v;
        len_code(len, s, e, v);
        uint32_t c = S.lcode[s];
        bw.put(c & 0xFFFF, c >> 16);
        bw.put(v, e);
        dist_code(dist, s, e, v);
        c = S.dcode[s];
        bw.put(c & 0xFFFF, c >> 16);
        bw.put(v, e);
    }
};

// Output bytes of the segment (every thread can evaluate it after the bit scan).
template <class C>
PBX_HD uint32_t seg_nbytes(const DeflateSmem<C>& S, const SegParams& sp) {
    const uint32_t bt = S.misc[M_BTYPE];
    if (bt == 0) return 5 + sp.sl;
    const uint32_t bits = S.misc[M_HDRBITS] + S.misc[M_DATABITS] + (S.lcode[256] >> 16);
    return sp.last ? (bits + 7) / 8 : (bits + 3 + 7) / 8 + 4;
}

// ---------------------------------------------------------------- phase: write bits
// Requires t_a = exclusive prefix of bit counts and misc[M_DATABITS] = their total.
template <class C, class Ops>
PBX_HD void ph_write(uint32_t tid, DeflateSmem<C>& S, const SegParams& sp) {
    const uint32_t bt = S.misc[M_BTYPE];
    const uint32_t nbytes = seg_nbytes(S, sp);
    if (bt != 0) {
        const uint32_t hdr = S.misc[M_HDRBITS];
        WriteF<C, Ops> f{S, {S.u.out, hdr + S.t_a[tid]}};
        walk_tokens<C>(tid, S, sp, f);
        if (tid == 0) {
            BitWriter<C, Ops> bw{S.u.out, 0};
            bw.put(sp.last ? 1u : 0u, 1);
            bw.put(bt, 2);
            if (bt == 2) {
                const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
                bw.put(S.misc[M_HLIT] - 257, 5);
                bw.put(S.misc[M_HDIST] - 1, 5);
                bw.put(S.misc[M_HCLEN] - 4, 4);
                for (uint32_t k = 0; k < S.misc[M_HCLEN]; k++) bw.put(S.hw.cllen[order[k]], 3);
                for (uint32_t k = 0; k < S.misc[M_NRLE]; k++) {
                    const uint32_t r = S.rle[k], sym = r & 0xFF;
                    const uint32_t c = S.hw.clcode[sym];
                    bw.put(c & 0xFFFF, c >> 16);
                    bw.put(r >> 8, rle_ebits(sym));
                }
            }
            // end of block, then (not last) an empty stored block to reach a byte boundary
            bw.pos = hdr + S.misc[M_DATABITS];
            const uint32_t eob = S.lcode[256];
            bw.put(eob & 0xFFFF, eob >> 16);
            S.misc[M_BLKBITS] = bw.pos;
            if (!sp.last) {
                bw.put(0, 3);
                bw.pos = (bw.pos + 7) & ~7u;
                bw.put(0xFFFF0000u, 32);
            }
        }
    }
    // CRC constants for the tree combine (chunks are right-aligned: every right operand
    // is full, so level k always shifts by x^(8*CC*2^k)).
    if (tid == C::NT - 1) {
        const uint32_t cc = (nbytes + C::NT - 1) / C::NT;
        uint32_t op = crc_x8n(cc);
        for (int k = 0; k <= C::LOGNT; k++) {
            S.misc[M_OPK0 + k] = op;
            op = crc_multmodp(op, op);
        }
    }
    if (tid == C::NT - 2) S.misc[M_CRCOP] = crc_x8n(nbytes);
    if (tid == 0 && bt == 0) S.misc[M_BLKBITS] = 8 * nbytes;
    if (tid == 0) S.misc[M_NBYTES] = nbytes;
}

template <class C>
PBX_HD uint32_t out_byte(const DeflateSmem<C>& S, const SegParams& sp, uint32_t j) {
    if (S.misc[M_BTYPE] != 0) return (S.u.out[j >> 2] >> ((j & 3) * 8)) & 0xFFu;
    if (j == 0) return sp.last ? 1u : 0u;
    if (j == 1) return sp.sl & 0xFF;
    if (j == 2) return (sp.sl >> 8) & 0xFF;
    if (j == 3) return (~sp.sl) & 0xFF;
    if (j == 4) return (~sp.sl >> 8) & 0xFF;
    return lds_byte(S, sp.wl + j - 5);
}

// ------------------------------------------------------ phase: store + CRC partials
template <class C>
PBX_HD void ph_store(uint32_t tid, DeflateSmem<C>& S, const SegParams& sp, uint8_t* slot) {
    const uint32_t nbytes = S.misc[M_NBYTES];
    if (S.misc[M_BTYPE] != 0) {
        uint32_t* s32 = (uint32_t*)slot;
        for (uint32_t k = tid; k < (nbytes + 3) / 4; k += C::NT) s32[k] = S.u.out[k];
    } else {
        for (uint32_t j = tid; j < nbytes; j += C::NT) slot[j] = (uint8_t)out_byte(S, sp, j);
    }
    // Raw CRC (register init 0, no final xor) of a right-aligned chunk: thread t covers
    // [n - (NT-t)*cc, n - (NT-1-t)*cc).  Leading zero bytes leave a raw CRC unchanged, so a
    // short or empty chunk counts as a full cc-byte one and every tree level shifts by the
    // same x^(8*cc*2^k).
    const uint32_t cc = (nbytes + C::NT - 1) / C::NT;
    const int64_t hi = (int64_t)nbytes - (int64_t)(C::NT - 1 - tid) * cc;
    int64_t lo = hi - cc;
    if (lo < 0) lo = 0;
    uint32_t c = 0;
    for (int64_t j = lo; j < hi; j++) c = crc_update(S.crc_table, c, (uint8_t)out_byte(S, sp, (uint32_t)j));
    S.t_a[tid] = c;
}

// ------------------------------------------------------- phase: tree combine level k
template <class C>
PBX_HD void ph_tree(uint32_t tid, DeflateSmem<C>& S, int k) {
    const uint32_t step = 1u << k;
    if ((tid & (2 * step - 1)) == 0 && tid + step < (uint32_t)C::NT) {
        const uint32_t r = tid + step;
        adler_combine(S.t_s1[tid], S.t_s2[tid], S.t_s1[r], S.t_s2[r], S.t_len[r]);
        S.t_len[tid] += S.t_len[r];
        S.t_a[tid] = crc_combine_op(S.t_a[tid], S.t_a[r], S.misc[M_OPK0 + k]);
    }
}

template <class C>
PBX_HD void ph_final(uint32_t tid, DeflateSmem<C>& S, const SegParams& sp, SegOut* out) {
    if (tid != 0) return;
    SegOut o;
    o.nbytes = S.misc[M_NBYTES];
    // raw CRC -> standard CRC-32: crc = raw ^ (0xFFFFFFFF shifted over n bytes) ^ 0xFFFFFFFF
    o.crc = S.t_a[0] ^ crc_multmodp(S.misc[M_CRCOP], 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
    o.crc_op = S.misc[M_CRCOP];
    o.adler_s1 = S.t_s1[0];
    o.adler_s2 = S.t_s2[0];
    o.len = sp.sl;
    o.btype = S.misc[M_BTYPE];
    o.bits = S.misc[M_BLKBITS];
    *out = o;
}

}  // namespace pbx
