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
    uint32_t rle[320], rboff[SORTN], rbm[10];
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
void run_huff(Smem& S, uint32_t sl, uint32_t last) {
    for (int t = 0; t < C::HT; t++) ph_huff_init<C>(t, S);
    for (int t = 0; t < C::HT; t++) ph_keys<C, EmuOps>(t, S);
    std::sort(S.hs.skey, S.hs.skey + SORTN);
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
    for (int t = 0; t < C::HT; t++) ph_rle_mark<C, EmuOps>(t, S);
    for (int t = 0; t < C::HT; t++) ph_rle_count<C>(t, S);
    S.misc[M_NRLE] = scan_excl_add(S.hs.rcnt, SORTN);
    for (int t = 0; t < C::HT; t++) ph_rle_emit<C, EmuOps>(t, S);
    for (int t = 0; t < C::HT; t++) ph_clen<C>(t, S);
    for (int t = 0; t < C::HT; t++) ph_rle_bits<C>(t, S);
    S.misc[M_HDRBITS] = scan_excl_add(S.rboff, SORTN);
    for (int t = 0; t < C::HT; t++) ph_choose<C>(t, S, sl, last);
    for (int t = 0; t < C::HT; t++) ph_codes<C>(t, S);
    for (int t = 0; t < C::HT; t++) ph_header<C, EmuOps>(t, S, last);
}

// k_lz77, k_huff and k_encode of one segment, thread by thread; -2 if the encoder's bit
// count disagrees with the Huffman step's (a broken invariant).
template <class Src>
int run_segment(Smem& S, const Src& src, const SegParams& sp, uint8_t* slot, SegOut* so) {
    // ---- k_lz77
    for (int t = 0; t < C::NT; t++) ph_fill<C>(t, S, src, sp);
    for (int t = 0; t < C::NT; t++) ph_lz_init<C>(t, S);
    for (int w = 0; w < C::NW; w++) ph_parse_emu<C>(w, S, sp);
    uint32_t a1 = 0, a2 = 0;
    for (int t = 0; t < C::NT; t++) {
        uint32_t s1, s2, n;
        ph_hist<C, EmuOps>(t, S, sp, s1, s2, n);
        adler_combine(a1, a2, s1, s2, n);
    }
    run_huff(S, sp.sl, sp.last);
    // ---- k_encode
    for (int t = 0; t < C::NT; t++) ph_enc_init<C>(t, S, S.hdrw);
    if (S.misc[M_BTYPE] == 0)
        for (int t = 0; t < C::NT; t++) ph_stored<C>(t, S, sp);
    for (int t = 0; t < C::NT; t++) S.t_a[t] = ph_bits<C>(t, S, sp);
    const uint32_t bitsum = scan_excl_add(S.t_a, C::NT);
    if (S.misc[M_BTYPE] != 0 && bitsum != S.misc[M_DATABITS] - (S.lcode[256] >> 16)) return -2;
    for (int t = 0; t < C::NT; t++) ph_write<C, EmuOps>(t, S, sp, S.t_a[t]);
    const uint32_t nbytes = S.misc[M_NBYTES];
    for (uint32_t j = 0; j < nbytes; j++) slot[j] = (uint8_t)out_byte(S, j);
    uint32_t raw = 0;
    const uint32_t opc = crc_x8pow2(C::LOG2_CRCC);
    for (int t = 0; t < C::NT; t++) raw = crc_multmodp(opc, raw) ^ ph_crc<C>(t, S);
    so->nbytes = nbytes;
    so->crc_op = crc_x8n(nbytes);
    so->crc = crc_from_raw(raw, so->crc_op);
    so->adler_s1 = a1;
    so->adler_s2 = a2;
    so->len = sp.sl;
    so->btype = S.misc[M_BTYPE];
    so->bits = S.misc[M_HDRBITS] + S.misc[M_DATABITS];
    return 0;
}

}  // namespace

extern "C" {

int pbxemu_seg_bytes(void) { return C::SEG; }
int pbxemu_win_bytes(void) { return C::WIN; }
int pbxemu_threads(void) { return C::NT; }

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

int pbxemu_deflate(const uint8_t* stream, uint64_t len, uint32_t rowlen, uint8_t* out,
                   uint64_t cap, uint64_t* out_len, SegOut* segs) {
    uint32_t nseg, seg_len;
    deflate_split(len, nseg, seg_len);
    std::unique_ptr<Smem> S(new Smem());
    std::vector<uint8_t> slot(C::SEG + 256);
    MemStream src{stream};
    uint64_t o = 0;
    if (cap < 2) return -1;
    out[o++] = 0x78;
    out[o++] = 0x9C;
    uint32_t s1 = 0, s2 = 0;
    for (uint32_t k = 0; k < nseg; k++) {
        SegParams sp;
        const uint64_t s = (uint64_t)k * seg_len;
        sp.sl = (uint32_t)((len - s) < seg_len ? (len - s) : seg_len);
        sp.wl = seg_window<C>(s, rowlen);
        sp.base = s - sp.wl;
        sp.rowlen = rowlen;
        sp.last = k + 1 == nseg;
        memset(S.get(), 0xCD, sizeof(Smem));  // poison: phases must initialise what they read
        SegOut so;
        if (run_segment(*S, src, sp, slot.data(), &so)) return -2;
        if (o + so.nbytes > cap) return -1;
        memcpy(out + o, slot.data(), so.nbytes);
        o += so.nbytes;
        adler_combine(s1, s2, so.adler_s1, so.adler_s2, so.len);
        if (segs) segs[k] = so;
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
    for (int i = 0; i < 288; i++) S->lfreq[i] = hist[i];
    for (int i = 0; i < 32; i++) S->dfreq[i] = hist[288 + i];
    run_huff(*S, sl, last);
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

}  // extern "C"
