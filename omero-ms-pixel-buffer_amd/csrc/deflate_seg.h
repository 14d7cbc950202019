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
    static constexpr int CRCC = 64;       // CRC chunk bytes per thread (NT*CRCC >= OUTW*4)
    static constexpr int LOG2_CRCC = 6;
    static constexpr int BUFW = (WIN + SEG + 16) / 4;
    static constexpr int OUTW = (SEG + 64) / 4;
    static constexpr int HSIZE = 1 << HBITS;
    static constexpr int LOGNT = NT == 1024 ? 10 : NT == 512 ? 9 : NT == 256 ? 8 : 7;
    static_assert(SEG % NT == 0, "SEG must be a multiple of NT");
    static_assert(SUB <= 65536 && SUB % CH == 0, "sub-segments hold whole thread chunks");
    static_assert(WIN + SEG <= 32768, "deflate distances are limited to 32768");
    static_assert((1 << LOGNT) == NT, "NT must be a power of two in 128..1024");
    static_assert(NT >= 320, "one thread per literal/length and distance symbol");
    static_assert(NT * CRCC >= OUTW * 4 && NT * CRCC >= SEG + 64, "CRC chunks cover the output");
};

enum : int {
    M_NL = 0, M_ND, M_HLIT, M_HDIST, M_HCLEN, M_NRLE, M_BTYPE, M_HDRBITS, M_DATABITS, M_NBYTES,
    M_CRCOP, M_BLKBITS, M_DYNBITS, M_FIXBITS,
    M_NMISC
};

struct HuffWork {  // the 19-symbol code-length code (one thread)
    uint32_t w[2 * 19];
    uint32_t parent[2 * 19];
    uint32_t blc[16], next[16];
    uint32_t cllen[19], clcode[19], clfreq[19], clsort[19];
};

constexpr uint32_t SORTN_ = 512;
struct HuffScratch {  // aliases the hash table (dead after the parse)
    uint32_t skey[SORTN_];
    uint32_t rcnt[SORTN_];      // RLE: symbols emitted by the run starting at i -> offsets
    uint32_t rec[2][288];       // step s: li0 | qi0 << 10 | cnt << 20
    uint32_t leafpar[2][288];
    uint32_t dA[2][288], aA[2][288], dB[2][288], aB[2][288];
};

template <class C>
struct DeflateSmem {
    uint32_t buf[C::BUFW];            // window + segment bytes, zero padded
    uint32_t mpos[C::NW * C::MAXMW];  // per-wave matches: segment position | (len-3) << 16
    uint32_t mdist[C::NW * C::MAXMW]; // distance - 1
    union {
        uint32_t head[C::HSIZE];      // hash -> first position (atomicMin)
        HuffScratch hs;               // Huffman construction (after the parse)
        uint32_t out[C::OUTW];        // packed output bits (after the codes)
    } u;
    uint32_t w_nm[C::NW];             // matches found by each wave
    uint32_t wtot[16];                // block-scan wave totals (device)
    uint32_t t_a[C::NT];              // bits -> exclusive prefix sum; then CRC partials
    uint32_t t_s1[C::NT], t_s2[C::NT], t_len[C::NT];  // Adler partials
    uint32_t lfreq[288], dfreq[32];
    uint32_t lcode[288], dcode[32];   // bit-reversed code | len << 16
    uint32_t hblc[2][16], hover[2], hstart[2][16], hnext[2][16];
    uint32_t lbm[16 * 9], dbm[16];    // per-length symbol bitmaps (canonical ranks)
    uint32_t crc_table[256];
    HuffWork hw;
    uint32_t rle[320];                // code-length RLE symbols: sym | extra << 8
    uint32_t rboff[512];              // bit offset of each RLE symbol inside the header
    uint32_t rbm[10];                 // run starts over the concatenated code lengths
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
    if (tid == 0) {
        S.misc[M_NL] = 0; S.misc[M_ND] = 0; S.misc[M_DYNBITS] = 0; S.misc[M_FIXBITS] = 0;
        S.misc[M_HLIT] = 257; S.misc[M_HDIST] = 1;
    }
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

// ====================================================================== Huffman codes
// Built in parallel phases; the result equals the classic sequential construction
// (sort by (freq, symbol), two-queue merge with leaves first on ties, zlib's overflow
// repair at 15 bits, longest codes to the least frequent leaves, canonical codes):
//   ph_keys     one key per symbol: (freq << 9 | sym), literal/length tree then distances
//   (sort)      ascending keys: bitonic with wave shuffles on the device, std-sort-like in
//               the emulator (any correct sort gives the same array)
//   (twoqueue)  the only serial step: per tree one wave (device: weights in registers,
//               readlane/writelane) records, per merge step, the queue positions and
//               how many leaves it took
//   ph_parents  every step's consumed leaves/internal nodes learn their parent step
//   ph_jump     pointer jumping (9 rounds): depth of every internal node
//   ph_leafdepth / ph_fixblc / ph_assign   bit-length counts, overflow repair, lengths
//   ph_rle      code-length RLE + code-length code + block type (one thread; short)
//   ph_codes    canonical codes: rank among same-length symbols from per-length bitmaps
constexpr uint32_t SORTN = SORTN_;
constexpr uint32_t KEY_NONE = 0xFFFFFFFFu;

PBX_HD uint32_t tree_n(const uint32_t* misc, uint32_t T) { return misc[T ? M_ND : M_NL]; }
PBX_HD uint32_t tree_base(const uint32_t* misc, uint32_t T) { return T ? misc[M_NL] : 0u; }
PBX_HD uint32_t key_weight(uint32_t key) { return (key >> 9) & 0x3FFFFFu; }

// (tree, index) handled by thread tid in the per-symbol / per-node phases
PBX_HD bool tree_slot(uint32_t tid, uint32_t& T, uint32_t& i) {
    if (tid < 288) { T = 0; i = tid; return true; }
    if (tid < 320) { T = 1; i = tid - 288; return true; }
    return false;
}

template <class C, class Ops>
PBX_HD void ph_keys(uint32_t tid, DeflateSmem<C>& S) {
    for (uint32_t t = tid; t < SORTN; t += C::NT) {
        uint32_t key = KEY_NONE;
        if (t < 286) {
            const uint32_t f = eff_lfreq(S.lfreq, t);
            if (f) { key = (f << 9) | t; Ops::add(&S.misc[M_NL], 1u); }
        } else if (t >= 288 && t < 318) {
            const uint32_t f = eff_dfreq(S.dfreq, t - 288);
            if (f) { key = (1u << 31) | (f << 9) | (t - 288); Ops::add(&S.misc[M_ND], 1u); }
        }
        S.u.hs.skey[t] = key;
    }
    if (tid < 288) S.lcode[tid] = 0;
    if (tid < 32) S.dcode[tid] = 0;
    if (tid < 32) { S.hblc[tid >> 4][tid & 15] = 0; }
    if (tid < 2) S.hover[tid] = 0;
    if (tid < 16 * 9) S.lbm[tid] = 0;
    if (tid < 16) S.dbm[tid] = 0;
    if (tid < 10) S.rbm[tid] = 0;
    if (tid < 19) S.hw.clfreq[tid] = 0;
}

// Serial two-queue merge over sorted leaf weights w(0..n): records every step.
template <class W>
PBX_HD void twoqueue_serial(W w, uint32_t n, uint32_t* iw, uint32_t* rec) {
    uint32_t li = 0, qi = 0, ni = 0;
    for (uint32_t s = 0; s + 1 < n; s++) {
        const uint32_t li0 = li, qi0 = qi;
        uint32_t cnt = 0, sum = 0;
        for (int k = 0; k < 2; k++) {
            if (li < n && (qi >= ni || w(li) <= iw[qi])) { sum += w(li); li++; cnt++; }
            else { sum += iw[qi]; qi++; }
        }
        iw[ni++] = sum;
        rec[s] = li0 | (qi0 << 10) | (cnt << 20);
    }
}

template <class C>
PBX_HD void ph_parents(uint32_t tid, DeflateSmem<C>& S) {
    uint32_t T, s;
    if (!tree_slot(tid, T, s)) return;
    const uint32_t n = tree_n(S.misc, T);
    if (s + 1 >= n) return;
    HuffScratch& H = S.u.hs;
    const uint32_t r = H.rec[T][s];
    const uint32_t li0 = r & 0x3FF, qi0 = (r >> 10) & 0x3FF, cnt = r >> 20;
    for (uint32_t j = li0; j < li0 + cnt; j++) H.leafpar[T][j] = s;
    for (uint32_t k = qi0; k < qi0 + 2 - cnt; k++) { H.aA[T][k] = s; H.dA[T][k] = 1; }
    if (s + 2 == n) { H.aA[T][s] = s; H.dA[T][s] = 0; }  // the root
}

// Round r of pointer jumping over internal nodes: depth = hops to the root.
template <class C>
PBX_HD void ph_jump(uint32_t tid, DeflateSmem<C>& S, int r) {
    uint32_t T, k;
    if (!tree_slot(tid, T, k)) return;
    const uint32_t n = tree_n(S.misc, T);
    if (k + 1 >= n) return;
    HuffScratch& H = S.u.hs;
    const uint32_t* sd = (r & 1) ? H.dB[T] : H.dA[T];
    const uint32_t* sa = (r & 1) ? H.aB[T] : H.aA[T];
    uint32_t* dd = (r & 1) ? H.dA[T] : H.dB[T];
    uint32_t* da = (r & 1) ? H.aA[T] : H.aB[T];
    const uint32_t a = sa[k];
    dd[k] = sd[k] + sd[a];
    da[k] = sa[a];
}
constexpr int JUMP_ROUNDS = 9;  // 2^9 > 287 internal nodes; result lands in dB

template <class C, class Ops>
PBX_HD void ph_leafdepth(uint32_t tid, DeflateSmem<C>& S) {
    uint32_t T, j;
    if (!tree_slot(tid, T, j)) return;
    if (j >= tree_n(S.misc, T)) return;
    HuffScratch& H = S.u.hs;
    uint32_t d = H.dB[T][H.leafpar[T][j]] + 1;
    if (d > 15) { d = 15; Ops::add(&S.hover[T], 1u); }
    Ops::add(&S.hblc[T][d], 1u);
}

// Per tree (thread 0: literal/length, thread 64: distance): overflow repair, the length
// assignment table and canonical first codes.
template <class C>
PBX_HD void ph_fixblc(uint32_t tid, DeflateSmem<C>& S) {
    if (tid != 0 && tid != 64) return;
    const uint32_t T = tid ? 1 : 0, maxbits = 15;
    uint32_t* blc = S.hblc[T];
    int overflow = (int)S.hover[T];
    while (overflow > 0) {  // zlib trees.c gen_bitlen
        uint32_t bits = maxbits - 1;
        while (blc[bits] == 0) bits--;
        blc[bits]--;
        blc[bits + 1] += 2;
        blc[maxbits]--;
        overflow -= 2;
    }
    uint32_t cum = 0;
    for (uint32_t L = maxbits; L >= 1; L--) { S.hstart[T][L] = cum; cum += blc[L]; }
    uint32_t code = 0;
    S.hnext[T][0] = 0;
    for (uint32_t L = 1; L <= maxbits; L++) {
        code = (code + (L > 1 ? blc[L - 1] : 0u)) << 1;
        S.hnext[T][L] = code;
    }
}

template <class C, class Ops>
PBX_HD void ph_assign(uint32_t tid, DeflateSmem<C>& S) {
    uint32_t T, j;
    if (!tree_slot(tid, T, j)) return;
    if (j >= tree_n(S.misc, T)) return;
    const uint32_t key = S.u.hs.skey[tree_base(S.misc, T) + j];
    const uint32_t sym = key & 0x1FF;
    uint32_t L = 15;
    while (L > 1 && j >= S.hstart[T][L] + S.hblc[T][L]) L--;
    if (T == 0) {
        S.lcode[sym] = L << 16;
        Ops::aor(&S.lbm[L * 9 + (sym >> 5)], 1u << (sym & 31));
        const uint32_t f = S.lfreq[sym];
        if (f) {
            const uint32_t eb = sym >= 257 ? len_sym_ebits(sym) : 0;
            Ops::add(&S.misc[M_DYNBITS], f * (L + eb));
            Ops::add(&S.misc[M_FIXBITS], f * (fixed_lit_len(sym) + eb));
        }
        Ops::amax(&S.misc[M_HLIT], sym + 1);
    } else {
        S.dcode[sym] = L << 16;
        Ops::aor(&S.dbm[L], 1u << sym);
        const uint32_t f = S.dfreq[sym];
        if (f) {
            const uint32_t eb = dist_sym_ebits(sym);
            Ops::add(&S.misc[M_DYNBITS], f * (L + eb));
            Ops::add(&S.misc[M_FIXBITS], f * (5 + eb));
        }
        Ops::amax(&S.misc[M_HDIST], sym + 1);
    }
}

// Length-limited Huffman lengths for a small alphabet (the 19-symbol code-length code).
PBX_HD void huff_lengths_small(const uint32_t* wsorted, const uint32_t* sorted, uint32_t n,
                               uint32_t maxbits, uint32_t* lens, HuffWork& hw) {
    uint32_t* w = hw.w;
    uint32_t* parent = hw.parent;
    for (uint32_t i = 0; i < n; i++) w[i] = wsorted[i];
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
    for (uint32_t i = root; i-- > 0;) w[i] = w[parent[i]] + 1;
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
        for (uint32_t c = hw.blc[bits]; c > 0; c--) lens[sorted[idx++]] = bits << 16;
}

// Canonical codes from lengths stored as (len << 16); result: rev code | len << 16.
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

// ----------------------------------------------- code-length RLE (parallel phases)
// The HLIT + HDIST code lengths are run-length coded (RFC 1951 3.2.7) run by run: a run
// of zeros becomes 18s (11..138), one 17 (3..10) and plain zeros; a run of v != 0 becomes
// v then 16s (3..6) and plain v's.  Runs may cross from the literal into the distance
// lengths.  ph_rle_mark flags run starts, ph_rle_count sizes each run's symbols, an
// exclusive scan places them, ph_rle_emit writes them.
template <class C>
PBX_HD uint32_t cl_len_at(const DeflateSmem<C>& S, uint32_t i) {
    const uint32_t hlit = S.misc[M_HLIT];
    return i < hlit ? S.lcode[i] >> 16 : S.dcode[i - hlit] >> 16;
}

template <class C, class Ops>
PBX_HD void ph_rle_mark(uint32_t tid, DeflateSmem<C>& S) {
    const uint32_t ntot = S.misc[M_HLIT] + S.misc[M_HDIST];
    if (tid < ntot && (tid == 0 || cl_len_at(S, tid) != cl_len_at(S, tid - 1)))
        Ops::aor(&S.rbm[tid >> 5], 1u << (tid & 31));
}

PBX_HD uint32_t rle_nsyms(uint32_t v, uint32_t run) {
    if (v == 0) {
        uint32_t n = 0;
        while (run >= 11) { run -= run < 138 ? run : 138; n++; }
        if (run >= 3) return n + 1;
        return n + run;
    }
    run--;
    return 1 + run / 6 + ((run % 6) >= 3 ? 1 : run % 6);
}

template <class C>
PBX_HD uint32_t rle_run_len(const DeflateSmem<C>& S, uint32_t i, uint32_t ntot) {
    uint32_t w = (i + 1) >> 5;
    uint32_t m = (i + 1) < 320 ? S.rbm[w] & ~((1u << ((i + 1) & 31)) - 1u) : 0u;
    while (!m && ++w < 10) m = S.rbm[w];
    const uint32_t nxt = m ? (w << 5) + (uint32_t)__builtin_ctz(m) : ntot;
    return (nxt < ntot ? nxt : ntot) - i;
}

template <class C>
PBX_HD void ph_rle_count(uint32_t tid, DeflateSmem<C>& S) {
    const uint32_t ntot = S.misc[M_HLIT] + S.misc[M_HDIST];
    uint32_t cnt = 0;
    if (tid < ntot && ((S.rbm[tid >> 5] >> (tid & 31)) & 1u))
        cnt = rle_nsyms(cl_len_at(S, tid), rle_run_len(S, tid, ntot));
    S.u.hs.rcnt[tid] = cnt;
}

// requires rcnt = exclusive prefix of the counts and misc[M_NRLE] = their total
template <class C, class Ops>
PBX_HD void ph_rle_emit(uint32_t tid, DeflateSmem<C>& S) {
    const uint32_t ntot = S.misc[M_HLIT] + S.misc[M_HDIST];
    if (!(tid < ntot && ((S.rbm[tid >> 5] >> (tid & 31)) & 1u))) return;
    const uint32_t v = cl_len_at(S, tid);
    uint32_t run = rle_run_len(S, tid, ntot), k = S.u.hs.rcnt[tid];
    uint32_t* cf = S.hw.clfreq;
    if (v == 0) {
        while (run >= 11) {
            const uint32_t n = run < 138 ? run : 138;
            S.rle[k++] = 18u | ((n - 11) << 8); Ops::add(&cf[18], 1u); run -= n;
        }
        if (run >= 3) { S.rle[k++] = 17u | ((run - 3) << 8); Ops::add(&cf[17], 1u); run = 0; }
        while (run) { S.rle[k++] = 0; Ops::add(&cf[0], 1u); run--; }
    } else {
        S.rle[k++] = v; Ops::add(&cf[v], 1u); run--;
        while (run >= 3) {
            const uint32_t n = run < 6 ? run : 6;
            S.rle[k++] = 16u | ((n - 3) << 8); Ops::add(&cf[16], 1u); run -= n;
        }
        while (run) { S.rle[k++] = v; Ops::add(&cf[v], 1u); run--; }
    }
}

// Code-length code (19 symbols, max 7 bits; at least two used symbols).  One thread.
template <class C>
PBX_HD void ph_clen(uint32_t tid, DeflateSmem<C>& S) {
    if (tid != 0) return;
    HuffWork& hw = S.hw;
    uint32_t* cf = hw.clfreq;
    uint32_t used = 0, ncl = 0;
    for (uint32_t s = 0; s < 19; s++) used += cf[s] != 0;
    for (uint32_t s = 0; s < 19 && used < 2; s++) if (!cf[s]) { cf[s] = 1; used++; }
    for (uint32_t s = 0; s < 19; s++) {
        hw.clcode[s] = 0;
        if (!cf[s]) continue;
        uint32_t k = ncl++;
        while (k > 0) {
            const uint32_t t = hw.clsort[k - 1];
            if (cf[t] < cf[s] || (cf[t] == cf[s] && t < s)) break;
            hw.clsort[k] = t;
            k--;
        }
        hw.clsort[k] = s;
    }
    uint32_t wsorted[19];
    for (uint32_t k = 0; k < ncl; k++) wsorted[k] = cf[hw.clsort[k]];
    huff_lengths_small(wsorted, hw.clsort, ncl, 7, hw.clcode, hw);
    huff_codes(hw.clcode, 19, 7, hw);
    for (uint32_t s = 0; s < 19; s++) hw.cllen[s] = hw.clcode[s] >> 16;
    const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    uint32_t hclen = 19;
    while (hclen > 4 && hw.cllen[order[hclen - 1]] == 0) hclen--;
    S.misc[M_HCLEN] = hclen;
}

// Bits of each RLE symbol (for the header offsets) into rboff[0..NT).
template <class C>
PBX_HD void ph_rle_bits(uint32_t tid, DeflateSmem<C>& S) {
    uint32_t b = 0;
    if (tid < S.misc[M_NRLE]) {
        const uint32_t sym = S.rle[tid] & 0xFF;
        b = S.hw.cllen[sym] + rle_ebits(sym);
    }
    S.rboff[tid] = b;
}

// Block type from the three sizes.  Requires rboff = exclusive prefix of RLE bits and
// misc[M_HDRBITS] = their total.  One thread.
template <class C>
PBX_HD void ph_choose(uint32_t tid, DeflateSmem<C>& S, const SegParams& sp) {
    if (tid != 0) return;
    const uint64_t hdr = 3 + 5 + 5 + 4 + 3ull * S.misc[M_HCLEN] + S.misc[M_HDRBITS];
    const uint64_t dyn_bits = hdr + S.misc[M_DYNBITS], fix_bits = 3ull + S.misc[M_FIXBITS];
    auto bytes_of = [&](uint64_t bits) -> uint64_t {
        return sp.last ? (bits + 7) / 8 : (bits + 3 + 7) / 8 + 4;
    };
    const uint64_t stored_bytes = 5ull + sp.sl;
    uint32_t btype = 2;
    uint64_t best = bytes_of(dyn_bits);
    if (bytes_of(fix_bits) <= best) { btype = 1; best = bytes_of(fix_bits); }
    if (stored_bytes <= best) { btype = 0; best = stored_bytes; }
    S.misc[M_HDRBITS] = btype == 2 ? (uint32_t)hdr : btype == 1 ? 3u : 0u;
    S.misc[M_BTYPE] = btype;
}

// Fixed Huffman codes (RFC 1951 3.2.6) in closed form: rev code | len << 16.
PBX_HD uint32_t fixed_lit_code(uint32_t s) {
    if (s < 144) return bitrev(0x30 + s, 8) | (8u << 16);
    if (s < 256) return bitrev(0x190 + (s - 144), 9) | (9u << 16);
    if (s < 280) return bitrev(s - 256, 7) | (7u << 16);
    return bitrev(0xC0 + (s - 280), 8) | (8u << 16);
}

// ------------------------------------------------------------ phase: canonical codes
template <class C>
PBX_HD void ph_codes(uint32_t tid, DeflateSmem<C>& S) {
    uint32_t T, sym;
    if (!tree_slot(tid, T, sym)) return;
    const uint32_t bt = S.misc[M_BTYPE];
    if (bt == 1) {
        if (T == 0) S.lcode[sym] = fixed_lit_code(sym);
        else S.dcode[sym] = bitrev(sym, 5) | (5u << 16);
        return;
    }
    if (bt == 0) return;
    uint32_t* codes = T ? S.dcode : S.lcode;
    const uint32_t L = codes[sym] >> 16;
    if (!L) return;
    uint32_t rank;
    if (T == 0) {
        const uint32_t* bm = S.lbm + L * 9;
        rank = (uint32_t)__builtin_popcount(bm[sym >> 5] & ((1u << (sym & 31)) - 1u));
        for (uint32_t w = 0; w < (sym >> 5); w++) rank += (uint32_t)__builtin_popcount(bm[w]);
    } else {
        rank = (uint32_t)__builtin_popcount(S.dbm[L] & ((1u << sym) - 1u));
    }
    codes[sym] = bitrev(S.hnext[T][L] + rank, L) | (L << 16);
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
        // header: fields by thread 0, code-length code lengths by threads < HCLEN,
        // RLE symbols by one thread each at their scanned offsets
        if (bt == 2) {
            const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
            const uint32_t hclen = S.misc[M_HCLEN];
            if (tid < hclen) {
                BitWriter<C, Ops> bw{S.u.out, 17 + 3 * tid};
                bw.put(S.hw.cllen[order[tid]], 3);
            }
            if (tid < S.misc[M_NRLE]) {
                const uint32_t r = S.rle[tid], sym = r & 0xFF, c = S.hw.clcode[sym];
                BitWriter<C, Ops> bw{S.u.out, 17 + 3 * hclen + S.rboff[tid]};
                bw.put(c & 0xFFFF, c >> 16);
                bw.put(r >> 8, rle_ebits(sym));
            }
        }
        if (tid == 0) {
            BitWriter<C, Ops> bw{S.u.out, 0};
            bw.put(sp.last ? 1u : 0u, 1);
            bw.put(bt, 2);
            if (bt == 2) {
                bw.put(S.misc[M_HLIT] - 257, 5);
                bw.put(S.misc[M_HDIST] - 1, 5);
                bw.put(S.misc[M_HCLEN] - 4, 4);
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
    if (tid == C::NT - 1) S.misc[M_CRCOP] = crc_x8n(nbytes);
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
    // Raw CRC (register init 0, no final xor) of a right-aligned CRCC-byte chunk: thread t
    // covers [n - (NT-t)*CRCC, n - (NT-1-t)*CRCC).  Leading zero bytes leave a raw CRC
    // unchanged, so a short or empty chunk counts as a full one and tree level k shifts by
    // the constant x^(8*CRCC*2^k).
    const uint32_t cc = (uint32_t)C::CRCC;
    const int64_t hi = (int64_t)nbytes - (int64_t)(C::NT - 1 - tid) * cc;
    int64_t lo = hi - cc;
    if (lo < 0) lo = 0;
    uint32_t c = 0;
    for (int64_t j = lo; j < hi; j++) c = crc_update(S.crc_table, c, (uint8_t)out_byte(S, sp, (uint32_t)j));
    S.t_a[tid] = c;
}

// ------------------------------------------------------- phase: tree combine level k
// op = x^(8 * CRCC * 2^k) = crc_x8pow2(LOG2_CRCC + k)
template <class C>
PBX_HD void ph_tree(uint32_t tid, DeflateSmem<C>& S, int k, uint32_t op) {
    const uint32_t step = 1u << k;
    if ((tid & (2 * step - 1)) == 0 && tid + step < (uint32_t)C::NT) {
        const uint32_t r = tid + step;
        adler_combine(S.t_s1[tid], S.t_s2[tid], S.t_s1[r], S.t_s2[r], S.t_len[r]);
        S.t_len[tid] += S.t_len[r];
        S.t_a[tid] = crc_combine_op(S.t_a[tid], S.t_a[r], op);
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
