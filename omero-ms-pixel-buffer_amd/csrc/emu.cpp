// emu.cpp — TEST-ONLY CPU emulation of the segment-deflate workgroup (deflate_seg.h).
//
// Builds libpbx_emu.so, which tests/ load to check the deflate algorithm on the CPU:
// every phase is executed for tid = 0..NT-1 in turn, with the barriers implied between
// phases.  The phases only communicate through commuting LDS atomics and disjoint
// writes, so this produces bit-for-bit the bytes the HIP kernel produces; GPU tests
// compare the two.  Never linked into libpbx.so and never used on the product path.
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
using Smem = DeflateSmem<C>;

uint32_t scan_excl_add(uint32_t* a) {
    uint32_t run = 0;
    for (int t = 0; t < C::NT; t++) { uint32_t v = a[t]; a[t] = run; run += v; }
    return run;
}

template <class Src>
void run_segment(Smem& S, const Src& src, const SegParams& sp, uint8_t* slot, SegOut* so) {
    for (int t = 0; t < C::NT; t++) ph_fill<C>(t, S, src, sp);
    for (int t = 0; t < C::NT; t++) ph_insert<C, EmuOps>(t, S, sp);
    for (int w = 0; w < C::NW; w++) ph_parse_emu<C>(w, S, sp);
    for (int t = 0; t < C::NT; t++) ph_hist<C, EmuOps>(t, S, sp);
    for (int t = 0; t < C::NT; t++) ph_keys<C, EmuOps>(t, S);
    std::sort(S.u.hs.skey, S.u.hs.skey + SORTN);
    {
        std::vector<uint32_t> iw(SORTN);
        const uint32_t nl = S.misc[M_NL], nd = S.misc[M_ND];
        const uint32_t* sk = S.u.hs.skey;
        twoqueue_serial([&](uint32_t i) { return key_weight(sk[i]); }, nl, iw.data(), S.u.hs.rec[0]);
        twoqueue_serial([&](uint32_t i) { return key_weight(sk[nl + i]); }, nd, iw.data(), S.u.hs.rec[1]);
    }
    for (int t = 0; t < C::NT; t++) ph_parents<C>(t, S);
    for (int r = 0; r < JUMP_ROUNDS; r++)
        for (int t = 0; t < C::NT; t++) ph_jump<C>(t, S, r);
    for (int t = 0; t < C::NT; t++) ph_leafdepth<C, EmuOps>(t, S);
    for (int t = 0; t < C::NT; t++) ph_fixblc<C>(t, S);
    for (int t = 0; t < C::NT; t++) ph_assign<C, EmuOps>(t, S);
    for (int t = 0; t < C::NT; t++) ph_rle_mark<C, EmuOps>(t, S);
    for (int t = 0; t < C::NT; t++) ph_rle_count<C>(t, S);
    S.misc[M_NRLE] = scan_excl_add(S.u.hs.rcnt);
    for (int t = 0; t < C::NT; t++) ph_rle_emit<C, EmuOps>(t, S);
    for (int t = 0; t < C::NT; t++) ph_clen<C>(t, S);
    for (int t = 0; t < C::NT; t++) ph_rle_bits<C>(t, S);
    S.misc[M_HDRBITS] = scan_excl_add(S.rboff);
    for (int t = 0; t < C::NT; t++) ph_choose<C>(t, S, sp);
    for (int t = 0; t < C::NT; t++) ph_codes<C>(t, S);
    for (int t = 0; t < C::NT; t++) ph_bits<C>(t, S, sp);
    S.misc[M_DATABITS] = scan_excl_add(S.t_a);
    for (int t = 0; t < C::NT; t++) ph_write<C, EmuOps>(t, S, sp);
    for (int t = 0; t < C::NT; t++) ph_store<C>(t, S, sp, slot);
    for (int k = 0; k < C::LOGNT; k++)
        for (int t = 0; t < C::NT; t++) ph_tree<C>(t, S, k, crc_x8pow2(C::LOG2_CRCC + k));
    for (int t = 0; t < C::NT; t++) ph_final<C>(t, S, sp, so);
}

}  // namespace

extern "C" {

int pbxemu_seg_bytes(void) { return C::SEG; }
int pbxemu_win_bytes(void) { return C::WIN; }
int pbxemu_threads(void) { return C::NT; }

// Deflate `len` bytes into a zlib stream exactly as the batch pipeline does for one tile
// (segments of seg_len_for(len) bytes, window, per-segment blocks, combined Adler-32).
// rowlen: repeating-row candidate distance.  Per-segment results go to segs (may be NULL,
// else room for pbxemu_nsegs(len)).  Returns 0, or -1 if cap is too small.
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
        sp.wl = (uint32_t)(s < (uint64_t)C::WIN ? s : (uint64_t)C::WIN);
        sp.base = s - sp.wl;
        sp.rowlen = rowlen;
        sp.last = k + 1 == nseg;
        memset(S.get(), 0xCD, sizeof(Smem));  // poison: phases must initialise what they read
        SegOut so;
        run_segment(*S, src, sp, slot.data(), &so);
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

// Host check of the CRC combine math used by the assemble kernel.
uint32_t pbxemu_crc_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
    return crc_combine_op(crc1, crc2, crc_x8n(len2));
}

}  // extern "C"
