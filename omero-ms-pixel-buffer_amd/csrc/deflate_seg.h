// deflate_seg.h — segment-parallel deflate: LZ77 in LDS, parallel Huffman construction and
// parallel bit packing.  Replaces the compression half of writeImage("png")
// (TileRequestHandler.java:176-199: Bio-Formats APNGWriter -> java.util.zip.
// DeflaterOutputStream, level 6).  Parity is at the decoded-pixel level (BASELINE.json
// north_star): the stream is valid RFC 1950/1951 and inflates to exactly the filtered
// scanlines; the compressed bytes differ from zlib's.
//
// A tile's byte stream is cut into segments of at most SEG bytes.  Every segment becomes one
// self-contained deflate block (stored / fixed / dynamic, whichever is smallest), followed
// by an empty stored block when it is not the last, so segments end byte-aligned and
// concatenate.  Matches reach up to WIN bytes back into the previous segment's bytes.
//
// Three GPU kernels share the work of one segment (kernels_deflate.hip):
//   LZ77     fill (window + segment in LDS), hash insert, wave-serial greedy/lazy parse,
//            symbol histogram and Adler-32 partial sums            -> matches, histogram
//   Huffman  one WAVE per segment: code lengths, canonical codes, the dynamic block
//            header and the exact output size                      -> code tables, header
//   encode   bit counts, scan, bit packing of every token, CRC-32  -> final output bytes
// The work of each kernel is written as PHASES separated by barriers.  A phase is a
// function of (thread id, LDS state) that only communicates through commuting LDS atomics
// (min / max / add / or) or disjoint writes, so the phases are deterministic.  The phases
// are templated on the LDS struct (SM): each kernel declares only the members its phases
// use, and tests/ run all phases on one CPU struct thread by thread (csrc/emu.cpp).  Scans
// and reductions between phases have a device form (wave shuffles) and an emulator form
// (loops) with identical results; GPU tests check the GPU bytes against the emulator's.
//
// Parse: each wave owns a SUB-byte sub-segment and parses it greedily with zlib-style
// one-step lazy matching.  The candidate matches at a position are fixed distances that
// image scanlines repeat at: the previous byte (runs), the previous 2-byte sample and the
// same column one row up.  On the device every lane holds 32 consecutive positions and
// builds, per candidate, a 64-bit mask of "byte equals the byte d back" (its positions
// plus the next lane's), so match lengths (capped at CAP) and the positions where a match
// pays are a few bit operations; the wave then walks only the positions that hold a
// paying match, scalar, and extends a capped match by one wave-wide compare.  The result
// is exactly the sequential greedy/lazy parse of ph_parse_emu (its scalar twin).  A match
// that reaches the end of its sub-segment runs on into the next one (up to 258 bytes, inside
// the segment), and the next wave parses from its end.  Tokens are kept as per-wave match lists; literals are the
// positions no match covers, so the later phases (histogram, bit counts, bit writing)
// walk fixed CH-position thread chunks.
#pragma once
#include "pbx_common.h"

#ifndef PBX_CAP
#define PBX_CAP 32
#endif

namespace pbx {

template <int NT_, int SEG_, int WIN_>
struct DeflateCfg {
    static constexpr int NT = NT_;        // threads per LZ77 / encode workgroup
    static constexpr int SEG = SEG_;      // max segment bytes
    static constexpr int WIN = WIN_;      // max window bytes before the segment
    static constexpr int HT = 64;         // threads of the Huffman workgroup (one wave)
    static constexpr int CH = SEG / NT;   // positions per thread chunk (emission phases)
    static constexpr int NW = NT / 64;    // waves
    static constexpr int SUB = SEG / NW;  // positions parsed by one wave
    static constexpr int MAXMW = 256;     // matches kept per wave (then literals only)
    static constexpr int MINCOV = 32;     // a wave keeps its matches only if they cover >= MINCOV bytes
    static constexpr int CAP = PBX_CAP;   // match length found by the masks before the wave extends it
    static constexpr int CRCC = 32;       // CRC chunk bytes per thread (thread 0: the rest too)
    static constexpr int LOG2_CRCC = 5;
    static constexpr int BUFW = (WIN + SEG + 32) / 4;
    static constexpr int SEGW = (SEG + 16) / 4;
    static constexpr int OUTW = (SEG + 64) / 4;
    static constexpr int HDRW = 160;      // dynamic block header bits (<= 17+57+316*14)
    static constexpr int LOGNT = NT == 1024 ? 10 : NT == 512 ? 9 : NT == 256 ? 8 : 7;
    static_assert(SEG % NT == 0, "SEG must be a multiple of NT");
    static_assert(CH == 32 && SUB == 64 * CH, "a lane's parse positions are its thread chunk");
    static_assert(CAP >= 6 && CAP <= 32, "capped lengths come from 64-bit equality masks");
    static_assert(SUB <= 65536 && SUB % CH == 0, "sub-segments hold whole thread chunks");
    static_assert(WIN <= 32768 && SEG <= 32768, "distances <= one row <= 32768; 16-bit positions");
    static_assert((1 << LOGNT) == NT, "NT must be a power of two in 128..1024");
    static_assert(CH % 4 == 0 && WIN % 16 == 0, "Adler chunks are whole aligned words");
    static_assert(HDRW * 32 >= 17 + 57 + 316 * 14, "header buffer holds any dynamic header");
};

enum : int {
    M_NL = 0, M_ND, M_HLIT, M_HDIST, M_HCLEN, M_NRLE, M_BTYPE, M_HDRBITS, M_DATABITS, M_NBYTES,
    M_CRCOP, M_BLKBITS, M_DYNBITS, M_FIXBITS,
    M_NMISC
};

// Per-segment parameters (uniform across the workgroup).
struct SegParams {
    uint64_t base;   // stream position of buf[0] (= segment start - wl)
    uint32_t wl;     // window bytes in buf before the segment
    uint32_t sl;     // segment bytes
    uint32_t rowlen; // repeating-row candidate distance (0 = none)
    uint32_t last;   // 1 if this segment ends the stream (BFINAL)
};

// Look-back bytes a segment starting at stream offset s keeps before it: enough for the
// longest candidate distance (one row), 16-byte aligned, at most WIN.
template <class C>
PBX_HD uint32_t seg_window(uint64_t s, uint32_t rowlen) {
    uint32_t need = ((rowlen > 2 ? rowlen : 2u) + 15u) & ~15u;
    if (need > (uint32_t)C::WIN) need = (uint32_t)C::WIN;
    return (uint32_t)(s < (uint64_t)need ? s : (uint64_t)need);
}

// c + sum of the four byte products of a and b (v_dot4_u32_u8 on the device).
PBX_HD uint32_t dot4_u8(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_udot4(a, b, c, false);
#else
    for (int i = 0; i < 4; i++) c += ((a >> (8 * i)) & 0xFFu) * ((b >> (8 * i)) & 0xFFu);
    return c;
#endif
}

template <class SM>
PBX_HD uint32_t lds_byte(const SM& S, uint32_t i) {
    return (S.buf[i >> 2] >> ((i & 3) * 8)) & 0xFFu;
}

// Low 32 bits of (hi:lo) >> sh, sh < 32 (v_alignbit_b32 on the device).
PBX_HD uint32_t funnel32(uint32_t hi, uint32_t lo, uint32_t sh) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh);
#endif
}

// Unaligned little-endian 32-bit read from the byte buffer: both words are always read
// (one ds_read2_b32, no branch on the alignment).
template <class SM>
PBX_HD uint32_t lds_ld4(const SM& S, uint32_t i) {
    const uint32_t w0 = S.buf[i >> 2], w1 = S.buf[(i >> 2) + 1];
    return funnel32(w1, w0, (i & 3) * 8);
}

// ============================================================================ LZ77
// Src provides fill_word(p0, nb) -> up to 4 stream bytes starting at stream position p0.
// Buffer bytes the LZ77 phases may read: the window and segment, zero up to the end of
// the last whole Adler chunk (CH) plus one 16-byte vector.
template <class C>
PBX_HD uint32_t lz_fill_bytes(const SegParams& sp) {
    const uint32_t z = sp.wl + (sp.sl + C::CH - 1) / C::CH * C::CH + 16;
    return z < (uint32_t)C::BUFW * 4 ? z : (uint32_t)C::BUFW * 4;
}

template <class C, class SM, class Src>
PBX_HD void ph_fill(uint32_t tid, SM& S, const Src& src, const SegParams& sp) {
    const uint32_t nb = sp.wl + sp.sl, nw = (nb + 3) / 4, nz = lz_fill_bytes<C>(sp) / 4;
    for (uint32_t k = tid; k < nz; k += C::NT) {
        uint32_t v = 0;
        if (k < nw) {
            const uint32_t take = nb - 4 * k;
            v = src.fill_word(sp.base + 4ull * k, take < 4 ? take : 4);
        }
        S.buf[k] = v;
    }
}

template <class C, class SM>
PBX_HD void ph_lz_init(uint32_t tid, SM& S) {
    for (uint32_t k = tid; k < 288; k += C::NT) S.lfreq[k] = 0;
    if (tid < 32) S.dfreq[tid] = 0;
}

// Candidate distances, in priority order (the first wins ties): previous byte, previous
// 2-byte sample, one row up (0 = none: rows too short to add anything).
constexpr int NCAND = 3;
PBX_HD uint32_t cand_dist(const SegParams& sp, int k) {
    return k == 0 ? 1u : k == 1 ? 2u : (sp.rowlen > 2 ? sp.rowlen : 0u);
}

// Shortest match worth coding at a distance: a 3-byte match far back costs more bits than
// three literals (zlib's TOO_FAR rule, extended one step).
PBX_HD uint32_t match_minlen(uint32_t dist) { return dist <= 256 ? 3u : dist <= 4096 ? 4u : 6u; }

// Length of the match of distance d at segment position p, capped at min(CAP, se - p);
// 0 when the distance reaches before the window.
template <class C, class SM>
PBX_HD uint32_t cand_len(const SM& S, const SegParams& sp, uint32_t p, uint32_t se, uint32_t d) {
    const uint32_t a = sp.wl + p;
    if (d == 0 || d > a || p >= se) return 0;
    const uint32_t lim = se - p < (uint32_t)C::CAP ? se - p : (uint32_t)C::CAP;
    uint32_t n = 0;
    while (n < lim && lds_byte(S, a + n) == lds_byte(S, a - d + n)) n++;
    return n;
}

// Best paying match at p: longest capped length among the candidates (first wins ties).
template <class C, class SM>
PBX_HD void best_match(const SM& S, const SegParams& sp, uint32_t p, uint32_t se, uint32_t& L,
                       uint32_t& D) {
    L = 0; D = 0;
    for (int k = 0; k < NCAND; k++) {
        const uint32_t d = cand_dist(sp, k);
        const uint32_t n = cand_len<C>(S, sp, p, se, d);
        if (n >= match_minlen(d) && n > L) { L = n; D = d; }
    }
}

// Length of a match of distance D at position p extended past L equal bytes by comparing
// 4-byte words at offsets L + 4k, up to maxlen (scalar form of the wave-wide compare).
template <class SM>
PBX_HD uint32_t extend_to(const SM& S, const SegParams& sp, uint32_t p, uint32_t L, uint32_t D, uint32_t maxlen) {
    if (L >= maxlen) return L;
    const uint32_t a = sp.wl + p;
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

// Full length of a match of distance D at position p that reached the cap, inside the
// sub-segment (up to min(258, se - p)).
template <class C, class SM>
PBX_HD uint32_t extend_scalar(const SM& S, const SegParams& sp, uint32_t p, uint32_t se,
                              uint32_t L, uint32_t D) {
    const uint32_t rem = se - p;
    const uint32_t maxlen = rem < 258 ? rem : 258;
    if (L < (uint32_t)C::CAP) return L;
    return extend_to(S, sp, p, L, D, maxlen);
}

// A match that reaches the end of its wave's sub-segment continues into the next one, up to
// min(258, sl - p) (segment end): runs are not cut at the 2 KiB wave boundaries (G_FAKE's
// repeated rows: one 258-byte match chain per segment instead of a short match per wave).
template <class C, class SM>
PBX_HD uint32_t extend_cross(const SM& S, const SegParams& sp, uint32_t p, uint32_t se, uint32_t L,
                             uint32_t D) {
    if (p + L != se || se >= sp.sl) return L;
    const uint32_t rem = sp.sl - p;
    return extend_to(S, sp, p, L, D, rem < 258 ? rem : 258);
}

// End (segment position) of wave w's last recorded match when it runs past the wave's
// sub-segment, else 0: wave w + 1 parses from there (its first positions are that match's).
template <class C, class SM>
PBX_HD uint32_t carry_end(const SM& S, uint32_t w) {
    const uint32_t nm = S.w_nm[w];
    if (!nm) return 0u;
    const uint32_t r = S.mpos[w * C::MAXMW + nm - 1];
    const uint32_t e = (r & 0xFFFFu) + (r >> 16) + 3;
    return e > (w + 1) * (uint32_t)C::SUB ? e : 0u;
}

// The parse of wave w's sub-segment, sequentially (the specification the device's
// bit-parallel parse reproduces): greedy, one-step lazy on capped lengths, from where the
// previous wave's last match ends if it runs into this sub-segment (waves in order).
template <class C, class SM>
PBX_HD void ph_parse_emu(uint32_t w, SM& S, const SegParams& sp) {
    const uint32_t ss = w * C::SUB;
    const uint32_t se = ss + C::SUB < sp.sl ? ss + C::SUB : sp.sl;
    uint32_t nm = 0, p = ss, cov = 0;
    if (w > 0) {
        const uint32_t c = carry_end<C>(S, w - 1);
        if (c > p) p = c;
    }
    while (p < se) {
        uint32_t L, D, L1, D1;
        best_match<C>(S, sp, p, se, L, D);
        if (L < 3) { p++; continue; }
        best_match<C>(S, sp, p + 1, se, L1, D1);
        if (L1 > L) { p++; continue; }  // lazy: a longer match starts at the next byte
        L = extend_scalar<C>(S, sp, p, se, L, D);
        L = extend_cross<C>(S, sp, p, se, L, D);
        if (nm < (uint32_t)C::MAXMW) {
            S.mpos[w * C::MAXMW + nm] = p | ((L - 3) << 16);
            S.mdist[w * C::MAXMW + nm] = (uint16_t)(D - 1);
            nm++;
            cov += L;
        }
        p += L;
    }
    // Matches covering fewer than MINCOV of the sub-segment's bytes (noise: a few 3-byte
    // runs, < 0.1% smaller) are dropped: the wave is then coded as literals only, which the
    // encoder does at half the cost (k_encode's literal-only path).
    S.w_nm[w] = cov < (uint32_t)C::MINCOV ? 0u : nm;
}

// Emit this thread's chunk of tokens in stream order: matches starting in the chunk
// (they may run past its end) and literals at positions no match covers.
template <class C, class SM, class F>
PBX_HD void walk_tokens(uint32_t tid, const SM& S, const SegParams& sp, F& f) {
    const uint32_t cs = tid * C::CH;
    if (cs >= sp.sl) return;
    const uint32_t ce = cs + C::CH < sp.sl ? cs + C::CH : sp.sl;
    const uint32_t w = cs / C::SUB;
    const uint32_t* mp = S.mpos + w * C::MAXMW;
    const auto* md = S.mdist + w * C::MAXMW;  // u16 or u32 distance - 1
    const uint32_t nm = S.w_nm[w];
    uint32_t lo = 0, hi = nm;  // first match starting at or after cs
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((mp[mid] & 0xFFFFu) < cs) lo = mid + 1; else hi = mid;
    }
    uint32_t pos = cs;
    if (lo > 0) {
        const uint32_t pe = (mp[lo - 1] & 0xFFFFu) + (mp[lo - 1] >> 16) + 3;
        if (pe > pos) pos = pe;
    } else if (w > 0) {  // the previous wave's last match may run into this chunk
        const uint32_t pe = carry_end<C>(S, w - 1);
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

template <class Ops, class SM>
struct HistF {
    SM& S;
    PBX_HD void lit(uint32_t b) { Ops::add(&S.lfreq[b], 1u); }
    PBX_HD void match(uint32_t len, uint32_t dist) {
        uint32_t s, e, v;
        len_code(len, s, e, v);
        Ops::add(&S.lfreq[s], 1u);
        dist_code(dist, s, e, v);
        Ops::add(&S.dfreq[s], 1u);
    }
};

// Histogram of the thread's tokens; returns the Adler-32 partial sums of its chunk
// (s1 = sum b, s2 = sum (n - i) b, both mod 65521; n bytes).
template <class C, class Ops, class SM>
PBX_HD void ph_hist(uint32_t tid, SM& S, const SegParams& sp, uint32_t& s1, uint32_t& s2,
                    uint32_t& n) {
    HistF<Ops, SM> f{S};
    walk_tokens<C>(tid, S, sp, f);
    if (tid == 0) Ops::add(&S.lfreq[256], 1u);  // end of block
    const uint32_t cs = tid * C::CH;
    s1 = 0; s2 = 0; n = 0;
    if (cs < sp.sl) {
        // whole words of the chunk (wl and cs are multiples of 4; bytes past the segment
        // are zero in buf): s2 with weights counted from the full chunk end, then shifted
        const uint32_t ce = cs + C::CH < sp.sl ? cs + C::CH : sp.sl;
        n = ce - cs;
        const uint32_t w0 = (sp.wl + cs) >> 2;
#pragma unroll
        for (uint32_t k = 0; k < (uint32_t)C::CH / 4; k++) {
            const uint32_t v = S.buf[w0 + k];
            const uint32_t e = (uint32_t)C::CH - 4 * k;  // weights e, e-1, e-2, e-3
            s1 = dot4_u8(v, 0x01010101u, s1);
            s2 = dot4_u8(v, e | ((e - 1) << 8) | ((e - 2) << 16) | ((e - 3) << 24), s2);
        }
        s2 -= (cs + (uint32_t)C::CH - ce) * s1;
        s1 %= ADLER_BASE;
        s2 %= ADLER_BASE;
    }
}

// ==================================================================== Huffman codes
// Built in parallel phases by one wave (C::HT threads); the result equals the classic
// sequential construction (sort by (freq, symbol), two-queue merge with leaves first on
// ties, zlib's overflow repair at 15 bits, longest codes to the least frequent leaves,
// canonical codes):
//   ph_keys     one key per symbol: (freq << 9 | sym), literal/length tree then distances
//   (sort)      ascending keys: register bitonic sort on the device, std::sort in the
//               emulator (any correct sort gives the same array)
//   (twoqueue)  the only serial step: per tree, the merge records, per step, the queue
//               positions and how many leaves it took
//   ph_parents  every step's consumed leaves/internal nodes learn their parent step
//   ph_jump     pointer jumping (9 rounds): depth of every internal node
//   ph_leafdepth / ph_fixblc / ph_assign   bit-length counts, overflow repair, lengths
//   ph_rle_*    code-length run-length coding; ph_clen: the code-length code
//   ph_choose   block type by exact size; ph_codes: canonical codes; ph_header: header bits
constexpr uint32_t SORTN = 512;  // sorting network width (the device sorts KEYN keys padded)
constexpr uint32_t KEYN = 320;   // sort keys: 288 literal/length slots, then 32 distance slots
constexpr uint32_t RLEN = 320;   // code-length RLE slots (HLIT + HDIST <= 316)
constexpr uint32_t KEY_NONE = 0xFFFFFFFFu;

struct HuffWork {  // the 19-symbol code-length code (one thread)
    uint32_t w[2 * 19];
    uint32_t parent[2 * 19];
    uint32_t blc[16], next[16];
    uint32_t cllen[19], clcode[19], clfreq[19], clsort[19];
};

// Node indices and depths fit 16 bits (internal weights, up to a block's symbol count, do not).  (The RLE counts,
// rcnt[RLEN], are a member of the phases' state struct itself.)
struct HuffScratch {
    uint32_t skey[KEYN];
    uint32_t rec[2][288];       // step s: li0 | qi0 << 10 | cnt << 20
    uint16_t leafpar[2][288];
    uint16_t dA[2][288], aA[2][288], dB[2][288], aB[2][288];
};

// Effective frequencies: every tree gets >= 2 used symbols (zlib's rule, so every decoder
// accepts the code): literal 0 and EOB, distances 0 and 1.
PBX_HD uint32_t eff_lfreq(const uint32_t* f, uint32_t s) {
    const uint32_t v = f[s];
    return (s == 0 || s == 256) && v == 0 ? 1u : v;
}
PBX_HD uint32_t eff_dfreq(const uint32_t* f, uint32_t s) {
    const uint32_t v = f[s];
    return s < 2 && v == 0 ? 1u : v;
}

PBX_HD uint32_t tree_n(const uint32_t* misc, uint32_t T) { return misc[T ? M_ND : M_NL]; }
PBX_HD uint32_t tree_base(const uint32_t* misc, uint32_t T) { return T ? misc[M_NL] : 0u; }
PBX_HD uint32_t key_weight(uint32_t key) { return (key >> 9) & 0x3FFFFFu; }

// item i of the 320 per-symbol / per-node slots -> (tree, index)
PBX_HD bool tree_slot(uint32_t i, uint32_t& T, uint32_t& k) {
    if (i < 288) { T = 0; k = i; return true; }
    if (i < 320) { T = 1; k = i - 288; return true; }
    return false;
}

template <class C, class SM>
PBX_HD void ph_huff_init(uint32_t tid, SM& S) {
    for (uint32_t t = tid; t < 288; t += C::HT) S.lcode[t] = 0;
    if (tid < 32) { S.dcode[tid] = 0; S.hblc[tid >> 4][tid & 15] = 0; S.dbm[tid & 15] = 0; }
    for (uint32_t t = tid; t < 16 * 9; t += C::HT) S.lbm[t] = 0;
    if (tid < 2) S.hover[tid] = 0;
    if (tid == 0) {
        S.misc[M_NL] = 0; S.misc[M_ND] = 0; S.misc[M_DYNBITS] = 0; S.misc[M_FIXBITS] = 0;
        S.misc[M_HLIT] = 257; S.misc[M_HDIST] = 1;
    }
}

// State of the code-length / header phases, initialised once the code lengths exist (on
// the device it shares LDS with the tree-building scratch, dead by then).
template <class C, class SM>
PBX_HD void ph_rle_init(uint32_t tid, SM& S) {
    for (uint32_t t = tid; t < (uint32_t)C::HDRW; t += C::HT) S.hdrw[t] = 0;
    if (tid < 10) S.rbm[tid] = 0;
    if (tid < 19) S.hw.clfreq[tid] = 0;
}

template <class C, class Ops, class SM>
PBX_HD void ph_keys(uint32_t tid, SM& S) {
    for (uint32_t t = tid; t < KEYN; t += C::HT) {
        uint32_t key = KEY_NONE;
        if (t < 286) {
            const uint32_t f = eff_lfreq(S.lfreq, t);
            if (f) { key = (f << 9) | t; Ops::add(&S.misc[M_NL], 1u); }
        } else if (t >= 288 && t < 318) {
            const uint32_t f = eff_dfreq(S.dfreq, t - 288);
            if (f) { key = (1u << 31) | (f << 9) | (t - 288); Ops::add(&S.misc[M_ND], 1u); }
        }
        S.hs.skey[t] = key;
    }
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

template <class C, class SM>
PBX_HD void ph_parents(uint32_t tid, SM& S) {
    for (uint32_t i = tid; i < 320; i += C::HT) {
        uint32_t T, s;
        tree_slot(i, T, s);
        const uint32_t n = tree_n(S.misc, T);
        if (s + 1 >= n) continue;
        auto& H = S.hs;
        const uint32_t r = H.rec[T][s];
        const uint32_t li0 = r & 0x3FF, qi0 = (r >> 10) & 0x3FF, cnt = r >> 20;
        for (uint32_t j = li0; j < li0 + cnt; j++) H.leafpar[T][j] = s;
        for (uint32_t k = qi0; k < qi0 + 2 - cnt; k++) { H.aA[T][k] = s; H.dA[T][k] = 1; }
        if (s + 2 == n) { H.aA[T][s] = s; H.dA[T][s] = 0; }  // the root
    }
}

// Round r of pointer jumping over internal nodes: depth = hops to the root.
template <class C, class SM>
PBX_HD void ph_jump(uint32_t tid, SM& S, int r) {
    for (uint32_t i = tid; i < 320; i += C::HT) {
        uint32_t T, k;
        tree_slot(i, T, k);
        const uint32_t n = tree_n(S.misc, T);
        if (k + 1 >= n) continue;
        auto& H = S.hs;
        const uint16_t* sd = (r & 1) ? H.dB[T] : H.dA[T];
        const uint16_t* sa = (r & 1) ? H.aB[T] : H.aA[T];
        uint16_t* dd = (r & 1) ? H.dA[T] : H.dB[T];
        uint16_t* da = (r & 1) ? H.aA[T] : H.aB[T];
        const uint32_t a = sa[k];
        dd[k] = (uint16_t)(sd[k] + sd[a]);
        da[k] = sa[a];
    }
}
constexpr int JUMP_ROUNDS = 9;  // 2^9 > 287 internal nodes; result lands in dB

template <class C, class Ops, class SM>
PBX_HD void ph_leafdepth(uint32_t tid, SM& S) {
    for (uint32_t i = tid; i < 320; i += C::HT) {
        uint32_t T, j;
        tree_slot(i, T, j);
        const uint32_t n = tree_n(S.misc, T);
        if (j >= n) continue;
        auto& H = S.hs;
        // zlib's overflow count (trees.c gen_bitlen) is over every node deeper than 15,
        // internal ones included: counting leaves only under-repairs deep trees
        if (j + 1 < n && H.dB[T][j] > 15) Ops::add(&S.hover[T], 1u);
        uint32_t d = H.dB[T][H.leafpar[T][j]] + 1;
        if (d > 15) { d = 15; Ops::add(&S.hover[T], 1u); }
        Ops::add(&S.hblc[T][d], 1u);
    }
}

// Per tree (thread 0: literal/length, thread 32: distance): overflow repair, the length
// assignment table and canonical first codes.
template <class C, class SM>
PBX_HD void ph_fixblc(uint32_t tid, SM& S) {
    if (tid != 0 && tid != 32) return;
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

template <class C, class Ops, class SM>
PBX_HD void ph_assign(uint32_t tid, SM& S) {
    for (uint32_t i = tid; i < 320; i += C::HT) {
        uint32_t T, j;
        tree_slot(i, T, j);
        if (j >= tree_n(S.misc, T)) continue;
        const uint32_t key = S.hs.skey[tree_base(S.misc, T) + j];
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
    int overflow = 0;  // every node deeper than maxbits, internal ones included (zlib)
    for (uint32_t i = n; i < root; i++) overflow += w[i] > maxbits ? 1 : 0;
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
        const uint32_t l = codes[s] >> 16;
        if (l) codes[s] = bitrev(hw.next[l]++, l) | (l << 16);
    }
}

PBX_HD uint32_t rle_ebits(uint32_t sym) { return sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0; }

// ------------------------------------------------ code-length RLE (parallel phases)
// The HLIT + HDIST code lengths are run-length coded (RFC 1951 3.2.7) run by run: a run
// of zeros becomes 18s (11..138), one 17 (3..10) and plain zeros; a run of v != 0 becomes
// v then 16s (3..6) and plain v's.  Runs may cross from the literal into the distance
// lengths.  ph_rle_mark flags run starts, ph_rle_count sizes each run's symbols, an
// exclusive scan places them, ph_rle_emit writes them.
template <class SM>
PBX_HD uint32_t cl_len_at(const SM& S, uint32_t i) {
    const uint32_t hlit = S.misc[M_HLIT];
    return i < hlit ? S.lcode[i] >> 16 : S.dcode[i - hlit] >> 16;
}

template <class C, class Ops, class SM>
PBX_HD void ph_rle_mark(uint32_t tid, SM& S) {
    const uint32_t ntot = S.misc[M_HLIT] + S.misc[M_HDIST];
    for (uint32_t i = tid; i < ntot; i += C::HT)
        if (i == 0 || cl_len_at(S, i) != cl_len_at(S, i - 1)) Ops::aor(&S.rbm[i >> 5], 1u << (i & 31));
}

// rle_nsyms without its loop (the device's wave-level RLE): 18s of 138 then the remainder
// (one more 18 from 11, one 17 from 3, else plain zeros); v, 16s of 6, then the remainder.
PBX_HD uint32_t rle_nsyms_closed(uint32_t v, uint32_t run) {
    if (v == 0) {
        const uint32_t q = run / 138, m = run % 138;
        return q + (m >= 3 ? 1u : m);
    }
    const uint32_t r1 = run - 1;
    return 1 + r1 / 6 + ((r1 % 6) >= 3 ? 1u : r1 % 6);
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

template <class SM>
PBX_HD uint32_t rle_run_len(const SM& S, uint32_t i, uint32_t ntot) {
    uint32_t w = (i + 1) >> 5;
    uint32_t m = (i + 1) < 320 ? S.rbm[w] & ~((1u << ((i + 1) & 31)) - 1u) : 0u;
    while (!m && ++w < 10) m = S.rbm[w];
    const uint32_t nxt = m ? (w << 5) + (uint32_t)__builtin_ctz(m) : ntot;
    return (nxt < ntot ? nxt : ntot) - i;
}

template <class C, class SM>
PBX_HD void ph_rle_count(uint32_t tid, SM& S) {
    const uint32_t ntot = S.misc[M_HLIT] + S.misc[M_HDIST];
    for (uint32_t i = tid; i < RLEN; i += C::HT) {
        uint32_t cnt = 0;
        if (i < ntot && ((S.rbm[i >> 5] >> (i & 31)) & 1u))
            cnt = rle_nsyms(cl_len_at(S, i), rle_run_len(S, i, ntot));
        S.rcnt[i] = cnt;
    }
}

// requires rcnt = exclusive prefix of the counts and misc[M_NRLE] = their total
template <class C, class Ops, class SM>
PBX_HD void ph_rle_emit(uint32_t tid, SM& S) {
    const uint32_t ntot = S.misc[M_HLIT] + S.misc[M_HDIST];
    for (uint32_t i = tid; i < ntot; i += C::HT) {
        if (!((S.rbm[i >> 5] >> (i & 31)) & 1u)) continue;
        const uint32_t v = cl_len_at(S, i);
        uint32_t run = rle_run_len(S, i, ntot), k = S.rcnt[i];
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
}

// Code-length code (19 symbols, max 7 bits; at least two used symbols).  One thread.
template <class C, class SM>
PBX_HD void ph_clen(uint32_t tid, SM& S) {
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

// Bits of each RLE symbol (for the header offsets) into rboff[0..RLEN).
template <class C, class SM>
PBX_HD void ph_rle_bits(uint32_t tid, SM& S) {
    for (uint32_t i = tid; i < RLEN; i += C::HT) {
        uint32_t b = 0;
        if (i < S.misc[M_NRLE]) {
            const uint32_t sym = S.rle[i] & 0xFF;
            b = S.hw.cllen[sym] + rle_ebits(sym);
        }
        S.rboff[i] = b;
    }
}

// Output bytes of a block of nsg segments (sl bytes in all) with the given block type and
// block bits (EOB included).  Stored, every segment is its own stored block (5-byte
// header): a block of many segments may hold more than a stored block's 65535 bytes.
PBX_HD uint32_t block_nbytes(uint32_t btype, uint64_t bits, uint32_t sl, uint32_t last, uint32_t nsg) {
    if (btype == 0) return 5 * nsg + sl;
    return last ? (uint32_t)((bits + 7) / 8) : (uint32_t)((bits + 3 + 7) / 8 + 4);
}

// Whether every segment's share of a Huffman-coded block (its bits [bit0, bit1): the header
// for the first, its tokens, the end of block and the empty stored block for the last)
// fits the encoder's per-segment output buffer: at most SEG bytes of bits.  With several
// segments per block one can exceed its stored size when the code was shaped by the
// others; such a block is stored instead (k_huff and the CPU emulation decide alike).
template <class C>
PBX_HD bool seg_shares_fit(const uint32_t* dk, uint32_t nsg, uint32_t hdr, uint32_t eob_len, uint32_t last,
                           uint32_t nbytes) {
    uint64_t run = hdr;
    for (uint32_t k = 0; k < nsg; k++) {
        const uint64_t b0 = k == 0 ? 0 : run;
        run += dk[k];
        const uint64_t b1 = k + 1 < nsg ? run : last ? run + eob_len : 8ull * nbytes;
        if (b1 - b0 > 8ull * (uint64_t)C::SEG) return false;
    }
    return true;
}

// Block type from the three sizes.  Requires rboff = exclusive prefix of RLE bits and
// misc[M_HDRBITS] = their total.  One thread.  Leaves M_HDRBITS = header bits of the
// chosen block, M_DATABITS = its data bits (EOB included) and M_NBYTES = the segment's
// exact output bytes.
template <class C, class SM>
PBX_HD void ph_choose(uint32_t tid, SM& S, uint32_t sl, uint32_t last, uint32_t nsg) {
    if (tid != 0) return;
    const uint64_t hdr = 3 + 5 + 5 + 4 + 3ull * S.misc[M_HCLEN] + S.misc[M_HDRBITS];
    const uint64_t dyn_bits = hdr + S.misc[M_DYNBITS], fix_bits = 3ull + S.misc[M_FIXBITS];
    const uint32_t dyn = block_nbytes(2, dyn_bits, sl, last, nsg), fix = block_nbytes(1, fix_bits, sl, last, nsg);
    const uint32_t sto = block_nbytes(0, 0, sl, last, nsg);
    uint32_t btype = 2, best = dyn;
    if (fix <= best) { btype = 1; best = fix; }
    if (sto <= best) { btype = 0; best = sto; }
    S.misc[M_HDRBITS] = btype == 2 ? (uint32_t)hdr : btype == 1 ? 3u : 0u;
    S.misc[M_DATABITS] = btype == 2 ? S.misc[M_DYNBITS] : btype == 1 ? S.misc[M_FIXBITS] : 0u;
    S.misc[M_BTYPE] = btype;
    S.misc[M_NBYTES] = best;
}

// Fixed Huffman codes (RFC 1951 3.2.6) in closed form: rev code | len << 16.
PBX_HD uint32_t fixed_lit_code(uint32_t s) {
    if (s < 144) return bitrev(0x30 + s, 8) | (8u << 16);
    if (s < 256) return bitrev(0x190 + (s - 144), 9) | (9u << 16);
    if (s < 280) return bitrev(s - 256, 7) | (7u << 16);
    return bitrev(0xC0 + (s - 280), 8) | (8u << 16);
}

template <class C, class SM>
PBX_HD void ph_codes(uint32_t tid, SM& S) {
    const uint32_t bt = S.misc[M_BTYPE];
    for (uint32_t i = tid; i < 320; i += C::HT) {
        uint32_t T, sym;
        tree_slot(i, T, sym);
        if (bt == 1) {
            if (T == 0) S.lcode[sym] = fixed_lit_code(sym);
            else S.dcode[sym] = bitrev(sym, 5) | (5u << 16);
            continue;
        }
        if (bt == 0) continue;
        uint32_t* codes = T ? S.dcode : S.lcode;
        const uint32_t L = codes[sym] >> 16;
        if (!L) continue;
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
}

template <class Ops>
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

// Block header bits into hdrw: BFINAL/BTYPE and, for a dynamic block, HLIT/HDIST/HCLEN,
// the code-length code lengths (one thread each) and the RLE symbols (one thread each, at
// their scanned offsets).
template <class C, class Ops, class SM>
PBX_HD void ph_header(uint32_t tid, SM& S, uint32_t last) {
    const uint32_t bt = S.misc[M_BTYPE];
    if (bt == 0) return;
    if (bt == 2) {
        const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
        const uint32_t hclen = S.misc[M_HCLEN];
        for (uint32_t k = tid; k < hclen; k += C::HT) {
            BitWriter<Ops> bw{S.hdrw, 17 + 3 * k};
            bw.put(S.hw.cllen[order[k]], 3);
        }
        for (uint32_t k = tid; k < S.misc[M_NRLE]; k += C::HT) {
            const uint32_t r = S.rle[k], sym = r & 0xFF, c = S.hw.clcode[sym];
            BitWriter<Ops> bw{S.hdrw, 17 + 3 * hclen + S.rboff[k]};
            bw.put(c & 0xFFFF, c >> 16);
            bw.put(r >> 8, rle_ebits(sym));
        }
    }
    if (tid == 0) {
        BitWriter<Ops> bw{S.hdrw, 0};
        bw.put(last ? 1u : 0u, 1);
        bw.put(bt, 2);
        if (bt == 2) {
            bw.put(S.misc[M_HLIT] - 257, 5);
            bw.put(S.misc[M_HDIST] - 1, 5);
            bw.put(S.misc[M_HCLEN] - 4, 4);
        }
    }
}

// =========================================================================== encode
// The encode workgroup holds the segment bytes (buf; wl may be 0), the match lists, the
// code tables, the block header (first HDRW words of out) and M_BTYPE / M_HDRBITS /
// M_DATABITS / M_NBYTES from the Huffman step.  The output bytes are assembled in out
// (a stored block is copied there too), then CRC'd and stored.
template <class C, class SM>
PBX_HD void ph_enc_init(uint32_t tid, SM& S, const uint32_t* hdrw) {
    for (uint32_t k = tid; k < (uint32_t)C::OUTW; k += C::NT) S.out[k] = k < (uint32_t)C::HDRW ? hdrw[k] : 0u;
    for (uint32_t k = tid; k < 256; k += C::NT) {  // slicing-by-4 CRC tables
        const uint32_t t0 = crc_table_entry(k);
        const uint32_t t1 = (t0 >> 8) ^ crc_table_entry(t0 & 0xFF);
        const uint32_t t2 = (t1 >> 8) ^ crc_table_entry(t1 & 0xFF);
        const uint32_t t3 = (t2 >> 8) ^ crc_table_entry(t2 & 0xFF);
        S.crc_t[0][k] = t0; S.crc_t[1][k] = t1; S.crc_t[2][k] = t2; S.crc_t[3][k] = t3;
    }
}

// Stored block (BTYPE 00) bytes into out: BFINAL/BTYPE byte, LEN, NLEN, the segment bytes.
template <class C, class SM>
PBX_HD void ph_stored(uint32_t tid, SM& S, const SegParams& sp) {
    const uint32_t n = 5 + sp.sl, nw = (n + 3) / 4;
    const uint32_t hdr0 = (sp.last ? 1u : 0u) | ((sp.sl & 0xFFFFu) << 8) | (((~sp.sl) & 0xFFu) << 24);
    const uint32_t hdr4 = ((~sp.sl) >> 8) & 0xFFu;
    for (uint32_t k = tid; k < nw; k += C::NT) {
        uint32_t v = 0;
        if (k == 0) {
            v = hdr0;
        } else {
            for (uint32_t i = 0; i < 4; i++) {
                const uint32_t j = 4 * k + i;
                const uint32_t b = j == 4 ? hdr4 : j < n ? lds_byte(S, sp.wl + j - 5) : 0u;
                v |= b << (8 * i);
            }
        }
        S.out[k] = v;
    }
}

template <class SM>
struct BitsF {
    const SM& S;
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

template <class C, class SM>
PBX_HD uint32_t ph_bits(uint32_t tid, const SM& S, const SegParams& sp) {
    if (S.misc[M_BTYPE] == 0) return 0;
    BitsF<SM> f{S, 0};
    walk_tokens<C>(tid, S, sp, f);
    return f.bits;
}

// Bit writer of one thread's contiguous bit range: every word is OR'd (the buffer starts zeroed), so the words shared with the neighbouring
// ranges need no special case and a put of 0 bits is a no-op.
template <class Ops>
struct RunWriter {
    uint32_t* out;
    uint32_t word;  // current word index
    uint32_t nacc;  // bits held in acc (including the leading bits of other ranges)
    uint64_t acc;
    PBX_HD RunWriter(uint32_t* o, uint32_t pos) : out(o), word(pos >> 5), nacc(pos & 31), acc(0) {}
    PBX_HD void put(uint32_t v, uint32_t n) {
        acc |= (uint64_t)v << nacc;
        nacc += n;
        if (nacc >= 32) {
            Ops::aor(&out[word], (uint32_t)acc);
            word++;
            acc >>= 32;
            nacc -= 32;
        }
    }
    PBX_HD void finish() {
        if (acc) Ops::aor(&out[word], (uint32_t)acc);  // < 32 bits left
    }
};

template <class Ops, class SM>
struct WriteF {
    const SM& S;
    RunWriter<Ops> bw;
    PBX_HD void lit(uint32_t b) { const uint32_t c = S.lcode[b]; bw.put(c & 0xFFFF, c >> 16); }
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

// Write this thread's tokens at hdr + bitoff; thread 0 adds the end of block and, for a
// non-final segment, an empty stored block that brings the stream to a byte boundary.
template <class C, class Ops, class SM>
PBX_HD void ph_write(uint32_t tid, SM& S, const SegParams& sp, uint32_t bitoff) {
    const uint32_t bt = S.misc[M_BTYPE];
    if (bt == 0) return;
    const uint32_t hdr = S.misc[M_HDRBITS];
    WriteF<Ops, SM> f{S, RunWriter<Ops>(S.out, hdr + bitoff)};
    walk_tokens<C>(tid, S, sp, f);
    f.bw.finish();
    if (tid == 0) {
        const uint32_t eob = S.lcode[256];
        BitWriter<Ops> bw{S.out, hdr + S.misc[M_DATABITS] - (eob >> 16)};
        bw.put(eob & 0xFFFF, eob >> 16);
        if (!sp.last) {
            bw.put(0, 3);
            bw.pos = (bw.pos + 7) & ~7u;
            bw.put(0xFFFF0000u, 32);
        }
    }
}

template <class SM>
PBX_HD uint32_t out_byte(const SM& S, uint32_t j) {
    return (S.out[j >> 2] >> ((j & 3) * 8)) & 0xFFu;
}

// Raw CRC (register init 0, no final xor) of this thread's right-aligned CRCC-byte chunk of
// the output left-padded with zero bytes to a multiple of 4 (leading zero bytes leave a raw
// CRC unchanged): thread t covers [V - (NT-t)*CRCC, V - (NT-1-t)*CRCC) of the padded V bytes,
// 4 bytes per slicing-by-4 step; thread 0 also takes everything before its chunk.  Short or
// empty chunks count as full ones and a chunk's operator only depends on the chunks after
// it, so combine level k shifts by the constant x^(8*CRCC*2^k).
template <class C, class SM>
PBX_HD uint32_t ph_crc(uint32_t tid, const SM& S) {
    const uint32_t nbytes = S.misc[M_NBYTES];
    const uint32_t pad = (4u - (nbytes & 3u)) & 3u, nv = (nbytes + pad) >> 2;
    const int64_t hi = (int64_t)nv - (int64_t)(C::NT - 1 - tid) * (C::CRCC / 4);
    int64_t lo = hi - C::CRCC / 4;
    if (lo < 0 || tid == 0) lo = 0;
    uint32_t c = 0;
    for (int64_t k = lo; k < hi; k++) {
        const uint32_t w1 = S.out[k];
        uint32_t v = w1;
        if (pad) {
            const uint32_t w0 = k > 0 ? S.out[k - 1] : 0u;
            v = (w1 << (8 * pad)) | (w0 >> (32 - 8 * pad));
        }
        c ^= v;
        c = S.crc_t[3][c & 0xFF] ^ S.crc_t[2][(c >> 8) & 0xFF] ^ S.crc_t[1][(c >> 16) & 0xFF] ^
            S.crc_t[0][c >> 24];
    }
    return c;
}

// Standard CRC-32 of n bytes from their raw CRC: raw ^ (0xFFFFFFFF shifted over n) ^ ~0.
PBX_HD uint32_t crc_from_raw(uint32_t raw, uint32_t op_n) {
    return raw ^ crc_multmodp(op_n, 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
}

}  // namespace pbx
