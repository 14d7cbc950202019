/* fake_pbx.c — TEST-ONLY stand-in for libpbx.so's entry points the JNI shim calls, with
 * scripted results, so that jni/pbx_jni.c's argument checks, error mapping and result
 * handling can be unit-tested on a CPU (tests/test_jni_shim.py).  Records every call. */
#include <stdlib.h>
#include <string.h>

#include "pbx.h"
#include "fake_pbx.h"

struct fake_state fake;

const char* pbx_last_error(void) { return "fake error"; }
int pbx_pixel_type_from_string(const char* n) {
    static const char* names[8] = {"int8", "uint8", "int16", "uint16", "int32", "uint32", "float", "double"};
    for (int i = 0; n && i < 8; i++)
        if (!strcmp(n, names[i])) return i;
    return -1;
}
int pbx_bytes_per_pixel(int32_t pt) {
    static const int b[8] = {1, 1, 2, 2, 4, 4, 4, 8};
    return pt >= 0 && pt < 8 ? b[pt] : 0;
}
int pbx_format_from_string(const char* f) {
    if (!f) return PBX_FMT_RAW;
    if (!strcmp(f, "png")) return PBX_FMT_PNG;
    if (!strcmp(f, "tif")) return PBX_FMT_TIF;
    return PBX_FMT_UNKNOWN;
}
int pbx_config_default(pbx_config* c) { memset(c, 0, sizeof *c); c->device = -1; c->coalesce = 1; return 0; }
int pbx_init(const pbx_config* c, pbx_ctx** out) { (void)c; *out = (pbx_ctx*)0x1000; return fake.init_rc; }
void pbx_shutdown(pbx_ctx* ctx) { (void)ctx; }
int pbx_image_declare(pbx_ctx* ctx, const pbx_image_desc* d) { (void)ctx; fake.last_image = *d; return fake.declare_rc; }
int pbx_image_release(pbx_ctx* ctx, int64_t id) { (void)ctx; (void)id; return 0; }
int pbx_plane_create(pbx_ctx* ctx, const pbx_plane_desc* d, int32_t y0, int32_t rows, uint64_t* id) {
    (void)ctx;
    fake.creates++;
    fake.last_desc = *d;
    fake.create_y0 = y0;
    fake.create_rows = rows;
    if (fake.create_rc) return fake.create_rc;
    *id = 77;
    return 0;
}
int pbx_plane_write_rows(pbx_ctx* ctx, uint64_t id, int32_t y0, int32_t rows, const void* data, uint64_t bytes) {
    (void)ctx; (void)id;
    if (fake.nwrites < FAKE_MAX_WRITES) {
        fake.w_y0[fake.nwrites] = y0;
        fake.w_rows[fake.nwrites] = rows;
        fake.w_bytes[fake.nwrites] = bytes;
        fake.w_first[fake.nwrites] = bytes ? ((const uint8_t*)data)[0] : 0;
        fake.w_last[fake.nwrites] = bytes ? ((const uint8_t*)data)[bytes - 1] : 0;
    }
    fake.nwrites++;
    return fake.nwrites == fake.write_fail_at ? PBX_E_INTERNAL : 0;
}
int pbx_plane_commit(pbx_ctx* ctx, uint64_t id) { (void)ctx; (void)id; fake.commits++; return fake.commit_rc; }
int pbx_plane_lookup(pbx_ctx* ctx, int64_t image, int32_t z, int32_t c, int32_t t, int32_t level, uint64_t* id,
                     int32_t* state, int32_t* y0, int32_t* rows) {
    (void)ctx; (void)image; (void)z; (void)c; (void)t; (void)level; (void)id; (void)y0; (void)rows;
    if (fake.lookup_rc) return fake.lookup_rc;
    if (state) *state = fake.lookup_state;
    return 0;
}
int pbx_set_residency_budget(pbx_ctx* ctx, uint64_t b) { (void)ctx; fake.budget = b; return 0; }
int pbx_plane_release(pbx_ctx* ctx, uint64_t id) { (void)ctx; (void)id; fake.releases++; return 0; }
int pbx_plane_build_pyramid(pbx_ctx* ctx, uint64_t id, int32_t levels, uint64_t* ids, double* ms) {
    (void)ctx; (void)id; (void)ms;
    for (int i = 0; i < levels; i++) ids[i] = 100 + i;
    return 0;
}
int pbx_plane_register_zarr(pbx_ctx* ctx, const pbx_plane_desc* d, const pbx_zarr_chunks* z, uint64_t* id,
                            double* ms) {
    (void)ctx; (void)d; (void)ms;
    fake.zarr_calls++;
    fake.zarr_last_offset = z->offsets[1];
    *id = 55;
    return 0;
}
int pbx_get_tile(pbx_ctx* ctx, const pbx_tile_req* req, pbx_result* out) {
    (void)ctx;
    fake.last_req = *req;
    if (fake.tile_fill) {  /* a filled result: status, region, body */
        out->status = fake.tile_status;
        out->format = req->format;
        out->w = 512;
        out->h = 256;
        out->data = fake.body;
        out->len = fake.body_len;
        out->owner = fake.tile_status == 0 ? (void*)&fake : NULL;
        return fake.tile_status;
    }
    return fake.tile_rc;  /* a call-level failure: *out untouched */
}
void pbx_results_release(pbx_ctx* ctx, pbx_result* r, uint64_t n) {
    (void)ctx;
    for (uint64_t i = 0; i < n; i++) {
        if (r[i].owner != (void*)&fake) fake.bad_release++;
        fake.releases_results++;
    }
}

int pbx_plane_create_sparse(pbx_ctx* ctx, const pbx_plane_desc* d, int32_t band_rows, int32_t own_y0,
                            int32_t own_rows, uint64_t* id) {
    (void)ctx;
    fake.creates++;
    fake.last_desc = *d;
    fake.sparse_band_rows = band_rows;
    fake.sparse_own_y0 = own_y0;
    fake.sparse_own_rows = own_rows;
    if (fake.create_rc) return fake.create_rc;
    *id = 88;
    return 0;
}
int pbx_band_write(pbx_ctx* ctx, uint64_t id, int32_t y0, int32_t rows, const void* data, uint64_t bytes) {
    if (fake.band_exists) return PBX_E_EXISTS;
    return pbx_plane_write_rows(ctx, id, y0, rows, data, bytes);
}
int pbx_band_abort(pbx_ctx* ctx, uint64_t id, int32_t y0) {
    (void)ctx; (void)id;
    fake.band_aborts++;
    fake.abort_y0 = y0;
    return 0;
}
int pbx_plane_band_info(pbx_ctx* ctx, uint64_t id, int32_t* band_rows, int32_t* nbands, uint8_t* states) {
    (void)ctx; (void)id;
    if (band_rows) *band_rows = fake.sparse_band_rows;
    if (nbands) *nbands = fake.nbands;
    if (states)
        for (int32_t k = 0; k < fake.nbands; k++) states[k] = (uint8_t)(k % 3);
    return 0;
}
int pbx_node_init(const pbx_config* cfg, int32_t n, const int32_t* devices, int32_t shard_tile, pbx_node** out) {
    (void)cfg; (void)shard_tile;
    fake.node_n = n;
    fake.node_dev0 = devices ? devices[0] : -1;
    *out = (pbx_node*)0x2000;
    return fake.init_rc;
}
void pbx_node_shutdown(pbx_node* node) { (void)node; }
pbx_ctx* pbx_node_context(pbx_node* node, int32_t k) { (void)node; return k < fake.node_n ? (pbx_ctx*)0x1000 : NULL; }
int pbx_node_get_tile(pbx_node* node, const pbx_tile_req* req, pbx_result* out, int32_t* served_by) {
    (void)node;
    if (served_by) *served_by = fake.served_by;
    return pbx_get_tile(NULL, req, out);
}
