/* fake_pbx.h — TEST-ONLY: the scripted state of fake_pbx.c. */
#ifndef FAKE_PBX_H
#define FAKE_PBX_H
#include <stdint.h>
#include "pbx.h"
#define FAKE_MAX_WRITES 64
struct fake_state {
    int init_rc, declare_rc, create_rc, commit_rc, lookup_rc, lookup_state;
    int creates, commits, releases, nwrites, write_fail_at, band_aborts;
    int32_t abort_y0;
    int32_t w_y0[FAKE_MAX_WRITES], w_rows[FAKE_MAX_WRITES];
    uint64_t w_bytes[FAKE_MAX_WRITES];
    uint8_t w_first[FAKE_MAX_WRITES], w_last[FAKE_MAX_WRITES];
    int32_t create_y0, create_rows;
    pbx_plane_desc last_desc;
    pbx_image_desc last_image;
    uint64_t budget;
    int zarr_calls;
    uint64_t zarr_last_offset;
    pbx_tile_req last_req;
    int tile_fill, tile_status, tile_rc;
    const uint8_t* body;
    uint64_t body_len;
    int releases_results, bad_release;
    /* sparse planes and the node router */
    int32_t sparse_band_rows, sparse_own_y0, sparse_own_rows, band_exists, nbands;
    int node_n, node_dev0, served_by;
};
extern struct fake_state fake;
#endif
