// emu.cpp — TEST-ONLY CPU emulation of the segment-deflate workgroup (deflate_seg.h).
//
// Builds libpbx_emu.so, which tests/ load to check the deflate algorithm on the CPU:
// every phase of k_lz77 / k_huff / k_encode is executed for tid = 0..NT-1 (HT for k_huff)
// in turn, with the barriers implied between phases.  The phases only communicate through
// commuting LDS atomics and disjoint writes, so this produces bit-for-bit the bytes the
// HIP kernels produce; GPU tests compare the two.  Never linked into libpbx.so and never used on the product path.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <vector>

#include "deflate_seg.h"
#include "pbx_config.h"

using namespace pbx;

namespace {

struct EmuOps {
    static void amin(uint32_t* p, uint32_t v) { if (v < *p) *p = v; }
    static void amax(uint32_t* p, uint32_t v) { if (v > *p) *p = v; }
    static void add(uint32_t* p, uint32_t v) { *p += v; }
    static void aor(uint32_t* p, uint32_t v) { *p |= v; }
};

using C = DeflateMainCfg;

// One CPU struct holding every member the phases of the three kernels touch.
struct Smem {
    uint32_t buf[C::BUFW];
    uint32_t mpos[C::NW * C::MAXMW];
    uint16_t mdist[C::NW * C::MAXMW];
    uint32_t w_nm[C::NW];
    uint32_t lfreq[288], dfreq[32];
    HuffScratch hs;
    uint32_t lcode[288], dcode[32];
    uint32_t hblc[2][16], hover[2], hstart[2][16], hnext[2][16];
    uint32_t lbm[16 * 9], dbm[16];
    HuffWork hw;
    uint32_t rle[320], rboff[RLEN], rbm[10], rcnt[RLEN];
    uint32_t hdrw[C::HDRW];
    uint32_t misc[M_NMISC];
    uint32_t out[C::OUTW];
    uint32_t crc_t[4][256];
    uint32_t t_a[C::NT];
};

uint32_t scan_excl_add(uint32_t* a, int n) {
    uint32_t run = 0;
    for (int t = 0; t < n; t++) { uint32_t v = a[t]; a[t] = run; run += v; }
    return run;
}

// k_huff (one wave of HT threads): needs lfreq / dfreq.
void run_huff(Smem& S, uint32_t sl, uint32_t last, uint32_t nsg) {
    for (int t = 0; t < C::HT; t++) ph_huff_init<C>(t, S);
    for (int t = 0; t < C::HT; t++) ph_keys<C, EmuOps>(t, S);
    std::sort(S.hs.skey, S.hs.skey + KEYN);
    {
        std::vector<uint32_t> iw(SORTN);
        const uint32_t nl = S.misc[M_NL], nd = S.misc[M_ND];
        const uint32_t* sk = S.hs.skey;
        twoqueue_serial([&](uint32_t i) { return key_weight(sk[i]); }, nl, iw.data(), S.hs.rec[0]);
        twoqueue_serial([&](uint32_t i) { return key_weight(sk[nl + i]); }, nd, iw.data(), S.hs.rec[1]);
    }
    for (int t = 0; t < C::HT; t++) ph_parents<C>(t, S);
    for (int r = 0; r < JUMP_ROUNDS; r++)
        for (int t = 0; t < C::HT; t++) ph_jump<C>(t, S, r);
    for (int t = 0; t < C::HT; t++) ph_leafdepth<C, EmuOps>(t, S);
    for (int t = 0; t < C::HT; t++) ph_fixblc<C>(t, S);
    for (int t = 0; t < C::HT; t++) ph_assign<C, EmuOps>(t, S);
    for (int t = 0; t < C::HT; t++) ph_rle_init<C>(t, S);
    for (int t = 0; t < C::HT; t++) ph_rle_mark<C, EmuOps>(t, S);
    for (int t = 0; t < C::HT; t++) ph_rle_count<C>(t, S);
    S.misc[M_NRLE] = scan_excl_add(S.rcnt, RLEN);
    for (int t = 0; t < C::HT; t++) ph_rle_emit<C, EmuOps>(t, S);
    for (int t = 0; t < C::HT; t++) ph_clen<C>(t, S);
    for (int t = 0; t < C::HT; t++) ph_rle_bits<C>(t, S);
    S.misc[M_HDRBITS] = scan_excl_add(S.rboff, RLEN);
    for (int t = 0; t < C::HT; t++) ph_choose<C>(t, S, sl, last, nsg);
    for (int t = 0; t < C::HT; t++) ph_codes<C>(t, S);
    for (int t = 0; t < C::HT; t++) ph_header<C, EmuOps>(t, S, last);
}

// Sequential bit writer of one block's tokens (the order k_encode's scan reproduces).
struct SeqWriter {
    const Smem& H;  // the block's codes (lcode / dcode: code | len << 16)
    BitWriter<EmuOps> bw;
    void lit(uint32_t b) { const uint32_t c = H.lcode[b]; bw.put(c & 0xFFFF, c >> 16); }
    void match(uint32_t len, uint32_t dist) {
        uint32_t s, e, v;
        len_code(len, s, e, v);
        uint32_t c = H.lcode[s];
        bw.put(c & 0xFFFF, c >> 16);
        bw.put(v, e);
        dist_code(dist, s, e, v);
        c = H.dcode[s];
        bw.put(c & 0xFFFF, c >> 16);
        bw.put(v, e);
    }
};

// k_lz77 of one segment, thread by thread (the phases' effects commute): matches, the
// histogram (one end of block counted) and the Adler-32 partial sums.
template <class Src>
void run_lz77(Smem& S, const Src& src, const SegParams& sp, uint32_t& a1, uint32_t& a2) {
    for (int t = 0; t < C::NT; t++) ph_fill<C>(t, S, src, sp);
    for (int t = 0; t < C::NT; t++) ph_lz_init<C>(t, S);
    for (int w = 0; w < C::NW; w++) ph_parse_emu<C>(w, S, sp);
    a1 = 0; a2 = 0;
    for (int t = 0; t < C::NT; t++) {
        uint32_t s1, s2, n;
        ph_hist<C, EmuOps>(t, S, sp, s1, s2, n);
        adler_combine(a1, a2, s1, s2, n);
    }
}

// One deflate block of nsg segments (k_lz77 per segment, k_huff on the summed histogram,
// k_encode of every segment into the block's bits); out gets the block's bytes.  -1 when
// cap is too small.
template <class Src>
int run_block(std::vector<std::unique_ptr<Smem>>& LZ, Smem& H, const Src& src, const SegParams* sps,
              uint32_t nsg, uint8_t* out, uint64_t cap, SegOut* so) {
    uint32_t sl = 0, a1 = 0, a2 = 0;
    for (uint32_t k = 0; k < nsg; k++) {
        memset(LZ[k].get(), 0xCD, sizeof(Smem));  // poison: phases must initialise what they read
        uint32_t s1, s2;
        run_lz77(*LZ[k], src, sps[k], s1, s2);
        adler_combine(a1, a2, s1, s2, sps[k].sl);
        sl += sps[k].sl;
    }
    const uint32_t last = sps[nsg - 1].last;
    memset(&H, 0xCD, sizeof(Smem));
    for (int i = 0; i < 288; i++) {
        uint32_t v = 0;
        for (uint32_t k = 0; k < nsg; k++) v += LZ[k]->lfreq[i];
        H.lfreq[i] = i == 256 ? 1u : v;
    }
    for (int i = 0; i < 32; i++) {
        uint32_t v = 0;
        for (uint32_t k = 0; k < nsg; k++) v += LZ[k]->dfreq[i];
        H.dfreq[i] = v;
    }
    run_huff(H, sl, last, nsg);
    if (H.misc[M_BTYPE] != 0) {  // k_huff's per-segment capacity rule (seg_shares_fit)
        uint32_t dk[BLK_SEGS];
        for (uint32_t k = 0; k < nsg; k++) {
            BitsF<Smem> f{H, 0};
            for (int t = 0; t < C::NT; t++) walk_tokens<C>((uint32_t)t, *LZ[k], sps[k], f);
            dk[k] = f.bits;
        }
        if (!seg_shares_fit<C>(dk, nsg, H.misc[M_HDRBITS], H.lcode[256] >> 16, last, H.misc[M_NBYTES])) {
            H.misc[M_BTYPE] = 0;
            H.misc[M_HDRBITS] = 0;
            H.misc[M_DATABITS] = 0;
            H.misc[M_NBYTES] = block_nbytes(0, 0, sl, last, nsg);
        }
    }
    for (uint32_t k = 0; k < 256; k++) H.crc_t[0][k] = crc_table_entry(k);
    const uint32_t bt = H.misc[M_BTYPE], nbytes = H.misc[M_NBYTES];
    if (nbytes > cap) return -1;
    std::vector<uint32_t> words((nbytes + 8) / 4 + 2, 0);
    if (bt == 0) {  // every segment its own stored block
        uint8_t* o = (uint8_t*)words.data();
        uint32_t p = 0;
        for (uint32_t k = 0; k < nsg; k++) {
            const uint32_t n = sps[k].sl;
            o[p] = (last && k + 1 == nsg) ? 1 : 0;
            o[p + 1] = (uint8_t)n; o[p + 2] = (uint8_t)(n >> 8); o[p + 3] = (uint8_t)~n; o[p + 4] = (uint8_t)(~n >> 8);
            p += 5;
            for (uint32_t j = 0; j < n; j++) o[p++] = (uint8_t)lds_byte(*LZ[k], sps[k].wl + j);
        }
    } else {
        const uint32_t hdr = H.misc[M_HDRBITS];
        for (uint32_t w = 0; w < (hdr + 31) / 32; w++) words[w] = H.hdrw[w];
        SeqWriter f{H, BitWriter<EmuOps>{words.data(), hdr}};
        for (uint32_t k = 0; k < nsg; k++)
            for (int t = 0; t < C::NT; t++) walk_tokens<C>((uint32_t)t, *LZ[k], sps[k], f);
        if (f.bw.pos != hdr + H.misc[M_DATABITS] - (H.lcode[256] >> 16)) return -2;
        const uint32_t eob = H.lcode[256];
        f.bw.put(eob & 0xFFFF, eob >> 16);
        if (!last) {
            f.bw.put(0, 3);
            f.bw.pos = (f.bw.pos + 7) & ~7u;
            f.bw.put(0xFFFF0000u, 32);
        }
    }
    memcpy(out, words.data(), nbytes);
    so->nbytes = nbytes;
    so->crc_op = crc_x8n(nbytes);
    uint32_t c = 0xFFFFFFFFu;
    for (uint32_t j = 0; j < nbytes; j++) c = crc_update(H.crc_t[0], c, out[j]);
    so->crc = c ^ 0xFFFFFFFFu;
    so->adler_s1 = a1;
    so->adler_s2 = a2;
    so->len = sl;
    so->btype = bt;
    so->bits = H.misc[M_HDRBITS] + H.misc[M_DATABITS];
    return 0;
}

}  // namespace

extern "C" {

int pbxemu_seg_bytes(void) { return C::SEG; }
int pbxemu_win_bytes(void) { return C::WIN; }
int pbxemu_threads(void) { return C::NT; }
int pbxemu_blk_segs(void) { return (int)BLK_SEGS; }
int pbxemu_split_max(void) { return (int)SPLIT_MAX; }
// The device's division by a precomputed reciprocal (pbx_common.h div_rcp), for the tests.
uint32_t pbxemu_div_rcp(uint32_t n, uint32_t d) { return div_rcp(n, d, recip32(d)); }

// Deflate `len` bytes into a zlib stream exactly as the batch pipeline does for one tile
// (segments of seg_len_for(len) bytes, window, per-segment blocks, combined Adler-32).
// rowlen: repeating-row candidate distance.  Per-segment results go to segs (may be NULL,
// else room for pbxemu_nsegs(len)).  Returns 0, -1 if cap is too small, -2 on a broken
// invariant.
uint32_t pbxemu_nsegs(uint64_t len) {
    uint32_t n, l;
    deflate_split(len, n, l);
    return n;
}

uint32_t pbxemu_nblocks(uint64_t len) { return tile_blocks(pbxemu_nsegs(len)); }

// Deflate `len` bytes into a zlib stream exactly as the batch pipeline does for one tile:
// segments of deflate_split, each with its row-sized window, BLK_SEGS segments per block
// sharing one Huffman code, combined Adler-32.  rowlen: the row-up candidate distance.
// Per-block results go to blks (may be NULL, else room for pbxemu_nblocks(len)).  Returns
// 0, -1 if cap is too small, -2 on a broken invariant.
int pbxemu_deflate(const uint8_t* stream, uint64_t len, uint32_t rowlen, uint8_t* out,
                   uint64_t cap, uint64_t* out_len, SegOut* blks) {
    uint32_t nseg, seg_len;
    deflate_split(len, nseg, seg_len);
    std::vector<std::unique_ptr<Smem>> LZ;
    for (uint32_t k = 0; k < BLK_SEGS; k++) LZ.emplace_back(new Smem());
    std::unique_ptr<Smem> H(new Smem());
    MemStream src{stream};
    uint64_t o = 0;
    if (cap < 2) return -1;
    out[o++] = 0x78;
    out[o++] = 0x9C;
    uint32_t s1 = 0, s2 = 0;
    const uint32_t nb = tile_blocks(nseg);
    for (uint32_t bi = 0; bi < nb; bi++) {
        const uint32_t k0 = block_seg0(bi, nseg, nb), nsg = block_seg0(bi + 1, nseg, nb) - k0;
        SegParams sps[BLK_SEGS];
        for (uint32_t q = 0; q < nsg; q++) {
            SegParams& sp = sps[q];
            const uint64_t s = (uint64_t)(k0 + q) * seg_len;
            sp.sl = (uint32_t)((len - s) < seg_len ? (len - s) : seg_len);
            sp.wl = seg_window<C>(s, rowlen);
            sp.base = s - sp.wl;
            sp.rowlen = rowlen;
            sp.last = k0 + q + 1 == nseg;
        }
        SegOut so;
        const int r = run_block(LZ, *H, src, sps, nsg, out + o, cap - o, &so);
        if (r) return r;
        o += so.nbytes;
        adler_combine(s1, s2, so.adler_s1, so.adler_s2, so.len);
        if (blks) blks[bi] = so;
    }
    if (o + 4 > cap) return -1;
    const uint32_t ad = adler_final(s1, s2, len);
    out[o++] = (uint8_t)(ad >> 24);
    out[o++] = (uint8_t)(ad >> 16);
    out[o++] = (uint8_t)(ad >> 8);
    out[o++] = (uint8_t)ad;
    *out_len = o;
    return 0;
}

// The LZ77 stage alone (k_lz77's outputs) for every segment of a stream: per segment
// HIST_WORDS histogram words and MREC_WORDS match-record words laid out as k_lz77 writes
// them (unused match slots are left 0).
int pbxemu_lz77(const uint8_t* stream, uint64_t len, uint32_t rowlen, uint32_t* hist, uint32_t* mrec) {
    uint32_t nseg, seg_len;
    deflate_split(len, nseg, seg_len);
    std::unique_ptr<Smem> S(new Smem());
    MemStream src{stream};
    for (uint32_t k = 0; k < nseg; k++) {
        SegParams sp;
        const uint64_t s = (uint64_t)k * seg_len;
        sp.sl = (uint32_t)((len - s) < seg_len ? (len - s) : seg_len);
        sp.wl = seg_window<C>(s, rowlen);
        sp.base = s - sp.wl;
        sp.rowlen = rowlen;
        sp.last = k + 1 == nseg;
        memset(S.get(), 0xCD, sizeof(Smem));
        for (int t = 0; t < C::NT; t++) ph_fill<C>(t, *S, src, sp);
        for (int t = 0; t < C::NT; t++) ph_lz_init<C>(t, *S);
        for (int w = 0; w < C::NW; w++) ph_parse_emu<C>(w, *S, sp);
        for (int t = 0; t < C::NT; t++) {
            uint32_t s1, s2, n;
            ph_hist<C, EmuOps>(t, *S, sp, s1, s2, n);
        }
        uint32_t* hg = hist + (size_t)k * HIST_WORDS;
        for (int i = 0; i < 288; i++) hg[i] = S->lfreq[i];
        for (int i = 0; i < 32; i++) hg[288 + i] = S->dfreq[i];
        uint32_t* mg = mrec + (size_t)k * MREC_WORDS;
        memset(mg, 0, MREC_WORDS * 4);
        for (int w = 0; w < C::NW; w++) {
            mg[w] = S->w_nm[w];
            for (uint32_t m = 0; m < S->w_nm[w]; m++) {
                mg[C::NW + w * C::MAXMW + m] = S->mpos[w * C::MAXMW + m];
                mg[C::NW + C::NW * C::MAXMW + w * C::MAXMW + m] = S->mdist[w * C::MAXMW + m];
            }
        }
    }
    return 0;
}

uint32_t pbxemu_hist_words(void) { return HIST_WORDS; }
uint32_t pbxemu_mrec_words(void) { return MREC_WORDS; }

// The Huffman stage alone on a given histogram (288 + 32 counts): codes 480 words as
// pbx_test_huffman returns them, info = block type, header bits, data bits, output bytes.
int pbxemu_huffman(const uint32_t* hist, uint32_t sl, uint32_t last, uint32_t* codes, uint32_t* info) {
    std::unique_ptr<Smem> S(new Smem());
    memset(S.get(), 0xCD, sizeof(Smem));
    for (int i = 0; i < 288; i++) S->lfreq[i] = i == 256 ? 1u : hist[i];  // one end of block
    for (int i = 0; i < 32; i++) S->dfreq[i] = hist[288 + i];
    run_huff(*S, sl, last, 1);
    for (int i = 0; i < 288; i++) codes[i] = S->lcode[i];
    for (int i = 0; i < 32; i++) codes[288 + i] = S->dcode[i];
    for (int i = 0; i < C::HDRW; i++) codes[320 + i] = S->hdrw[i];
    info[0] = S->misc[M_BTYPE];
    info[1] = S->misc[M_HDRBITS];
    info[2] = S->misc[M_DATABITS];
    info[3] = S->misc[M_NBYTES];
    return 0;
}

// Host check of the CRC combine math used by the assemble kernel.
uint32_t pbxemu_crc_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
    return crc_combine_op(crc1, crc2, crc_x8n(len2));
}

// The latency forms k_frame_wave uses (pbx_common.h) against zlib's bitwise ones: the number
// of the n seeded random pairs (and bytes) on which they differ.
// rle_nsyms_closed (the device's wave RLE) against rle_nsyms for every run of every length
// value: the number of mismatches.
uint32_t pbxemu_rle_closed_mismatches(void) {
    uint32_t bad = 0;
    for (uint32_t v = 0; v < 16; v++)
        for (uint32_t run = 1; run <= 320; run++) bad += rle_nsyms_closed(v, run) != rle_nsyms(v, run);
    return bad;
}

uint64_t pbxemu_crc_fast_mismatches(uint64_t n, uint64_t seed) {
    uint64_t x = seed | 1, bad = 0;
    auto next = [&]() {  // splitmix64
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return (uint32_t)(z ^ (z >> 31));
    };
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t a = (i % 7) ? next() : crc_x8n(next() & 0xFFFFFu), b = next(), v = next() & 0xFFu;
        if (crc_multmodp4(a, b) != crc_multmodp(a, b)) bad++;
        uint32_t c = b ^ v;
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ ((c & 1u) ? CRC_POLY : 0u);
        if (crc_byte4(b, v) != c) bad++;
    }
    return bad;
}

}  // extern "C"
