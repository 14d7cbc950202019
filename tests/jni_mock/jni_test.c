/* jni_test.c — TEST-ONLY driver of jni/pbx_jni.c against the minimal JNI environment
 * (jni.h here) and the scripted fake libpbx (fake_pbx.c): argument checks, error mapping,
 * the getTile status slot, piecewise row copies.  Built and run by tests/test_jni_shim.py. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fake_pbx.h"
#include "jni.h"
#include "mock_vm.h"

/* the shim's entry points (its own file has no header) */
jlong J(createPlane)(JNIEnv*, jclass, jlong, jlong, jint, jint, jint, jint, jstring, jint, jint, jboolean, jint, jint);
void J(writeRows)(JNIEnv*, jclass, jlong, jlong, jint, jint, jint, jbyteArray, jint);
void J(writeRowsDirect)(JNIEnv*, jclass, jlong, jlong, jint, jint, jobject);
void J(commitPlane)(JNIEnv*, jclass, jlong, jlong);
jint J(planeState)(JNIEnv*, jclass, jlong, jlong, jint, jint, jint, jint);
jlong J(registerPlane)(JNIEnv*, jclass, jlong, jlong, jint, jint, jint, jint, jstring, jint, jint, jboolean, jbyteArray);
jlong J(registerZarr)(JNIEnv*, jclass, jlong, jlong, jint, jint, jint, jint, jstring, jint, jint, jboolean, jint, jint,
                      jint, jbyteArray, jlongArray, jlong);
jbyteArray J(getTile)(JNIEnv*, jclass, jlong, jlong, jint, jint, jint, jint, jint, jint, jint, jint, jstring, jintArray);
void J(declareImage)(JNIEnv*, jclass, jlong, jlong, jstring, jint, jint, jint, jint, jint, jint);
jlong J(createSparsePlane)(JNIEnv*, jclass, jlong, jlong, jint, jint, jint, jint, jstring, jint, jint, jboolean, jint,
                           jint, jint);
jboolean J(writeBand)(JNIEnv*, jclass, jlong, jlong, jint, jint, jint, jbyteArray, jint);
jint J(bandInfo)(JNIEnv*, jclass, jlong, jlong, jbyteArray);
jlong J(nodeInit)(JNIEnv*, jclass, jint, jintArray, jint, jboolean, jint, jint);
jlong J(nodeContext)(JNIEnv*, jclass, jlong, jint);
jbyteArray J(nodeGetTile)(JNIEnv*, jclass, jlong, jlong, jint, jint, jint, jint, jint, jint, jint, jint, jstring,
                          jintArray);

static void reset(void) {
    memset(&fake, 0, sizeof fake);
    pending[0] = 0;
}

int main(void) {
    struct mock_obj u16 = str("uint16"), png = str("png");
    /* ---- getTile: a call-level failure (null ctx / shutdown) never releases a garbage owner */
    {
        reset();
        fake.tile_rc = PBX_E_BADARG;
        struct mock_obj so = arr(3, 3, 4);
        jbyteArray r = J(getTile)(env, NULL, 0, 1, 0, 0, 0, -1, 0, 0, 64, 64, &png, &so);
        CHECK(r == NULL && !pending[0]);
        CHECK(((jint*)so.data)[2] == PBX_E_BADARG);
        CHECK(fake.releases_results == 0);
        reset();
        fake.tile_rc = PBX_E_INTERNAL;
        r = J(getTile)(env, NULL, 1, 1, 0, 0, 0, -1, 0, 0, 64, 64, &png, &so);
        CHECK(r == NULL && threw("java/lang/RuntimeException"));
        CHECK(fake.releases_results == 0 && ((jint*)so.data)[2] == PBX_E_INTERNAL);
    }
    /* ---- getTile OK: exact-length body, the post-defaulting region, one release */
    {
        reset();
        static const uint8_t body[5] = {1, 2, 3, 4, 5};
        fake.tile_fill = 1;
        fake.tile_status = 0;
        fake.body = body;
        fake.body_len = 5;
        struct mock_obj so = arr(3, 3, 4);
        jbyteArray r = J(getTile)(env, NULL, 1, 9, 1, 2, 3, 4, 10, 20, 0, 0, &png, &so);
        CHECK(r && r->len == 5 && memcmp(r->data, body, 5) == 0 && !pending[0]);
        CHECK(((jint*)so.data)[0] == 512 && ((jint*)so.data)[1] == 256 && ((jint*)so.data)[2] == 0);
        CHECK(fake.releases_results == 1 && fake.bad_release == 0);
        CHECK(fake.last_req.image_id == 9 && fake.last_req.resolution == 4 && fake.last_req.format == PBX_FMT_PNG);
        /* a response a Java array cannot hold: IllegalArgumentException, still released */
        reset();
        fake.tile_fill = 1;
        fake.body = body;
        fake.body_len = 0x80000000ull;
        r = J(getTile)(env, NULL, 1, 9, 0, 0, 0, -1, 0, 0, 0, 0, NULL, &so);
        CHECK(r == NULL && threw("java/lang/IllegalArgumentException") && fake.releases_results == 1);
    }
    /* ---- getTile statuses: 404 -> null, NOT_RESIDENT -> null with the status for the handler */
    {
        struct mock_obj so = arr(3, 3, 4);
        int sts[2] = {PBX_E_NOTFOUND, PBX_E_NOT_RESIDENT};
        for (int k = 0; k < 2; k++) {
            reset();
            fake.tile_fill = 1;
            fake.tile_status = sts[k];
            jbyteArray r = J(getTile)(env, NULL, 1, 9, 0, 0, 0, -1, 0, 0, 8, 8, NULL, &so);
            CHECK(r == NULL && !pending[0] && ((jint*)so.data)[2] == sts[k] && fake.releases_results == 0);
        }
    }
    /* ---- writeRows: whole-row pieces of at most 16 MiB, every row once, bounds checked */
    {
        reset();
        const jint row = 65536 * 2, rows = 300;  /* 37.5 MiB */
        struct mock_obj a = arr(1, (size_t)row * rows + 7, 1);
        for (size_t i = 0; i < a.len; i++) ((uint8_t*)a.data)[i] = (uint8_t)(i / row);
        J(writeRows)(env, NULL, 1, 77, 1000, rows, row, &a, 7 - 7);
        CHECK(!pending[0]);
        int32_t y = 1000;
        uint64_t tot = 0;
        for (int i = 0; i < fake.nwrites; i++) {
            CHECK(fake.w_y0[i] == y && fake.w_bytes[i] == (uint64_t)fake.w_rows[i] * row);
            CHECK(fake.w_bytes[i] <= (16u << 20));
            CHECK(fake.w_first[i] == (uint8_t)(y - 1000));
            y += fake.w_rows[i];
            tot += fake.w_bytes[i];
        }
        CHECK(fake.nwrites == 3 && y == 1000 + rows && tot == (uint64_t)row * rows);
        reset();
        J(writeRows)(env, NULL, 1, 77, 0, rows + 1, row, &a, 0);  /* array too short */
        CHECK(threw("java/lang/IllegalArgumentException") && fake.nwrites == 0);
        reset();
        fake.write_fail_at = 2;
        J(writeRows)(env, NULL, 1, 77, 0, rows, row, &a, 0);  /* a library failure stops the copy */
        CHECK(threw("java/lang/RuntimeException") && fake.nwrites == 2);
        reset();
        struct mock_obj db = {4, 4096, calloc(4096, 1), NULL};
        J(writeRowsDirect)(env, NULL, 1, 77, 5, 2, &db);
        CHECK(!pending[0] && fake.nwrites == 1 && fake.w_bytes[0] == 4096);
        struct mock_obj notdirect = arr(1, 16, 1);
        reset();
        J(writeRowsDirect)(env, NULL, 1, 77, 5, 2, &notdirect);
        CHECK(threw("java/lang/IllegalArgumentException"));
    }
    /* ---- createPlane: 409 (another loader) is 0, not an exception; 507 throws */
    {
        reset();
        CHECK(J(createPlane)(env, NULL, 1, 9, 0, 1, 0, 0, &u16, 100, 200, 0, 64, 32) == 77 && !pending[0]);
        CHECK(fake.create_y0 == 64 && fake.create_rows == 32 && fake.last_desc.pixel_type == PBX_UINT16 &&
              fake.last_desc.byte_order == PBX_BIG_ENDIAN && fake.last_desc.source == PBX_SRC_HOST);
        reset();
        fake.create_rc = PBX_E_EXISTS;
        CHECK(J(createPlane)(env, NULL, 1, 9, 0, 1, 0, 0, &u16, 100, 200, 0, 0, 0) == 0 && !pending[0]);
        reset();
        fake.create_rc = PBX_E_NO_SPACE;
        CHECK(J(createPlane)(env, NULL, 1, 9, 0, 1, 0, 0, &u16, 100, 200, 0, 0, 0) == 0 &&
              threw("java/lang/RuntimeException") && strstr(pending, "pbx status 507: ") != NULL);
    }
    /* ---- planeState, declareImage */
    {
        reset();
        fake.lookup_rc = PBX_E_NOTFOUND;
        CHECK(J(planeState)(env, NULL, 1, 9, 0, 0, 0, 0) == -1 && !pending[0]);
        reset();
        fake.lookup_state = 2;
        CHECK(J(planeState)(env, NULL, 1, 9, 0, 0, 0, 0) == 2);
        reset();
        J(declareImage)(env, NULL, 1, 9, &u16, 10, 20, 3, 4, 5, 2);
        CHECK(!pending[0] && fake.last_image.size_z == 3 && fake.last_image.size_c == 4 &&
              fake.last_image.size_t_ == 5 && fake.last_image.levels == 2 && fake.last_image.pixel_type == 3);
    }
    /* ---- registerPlane: create + rows + commit; a failed copy releases the plane */
    {
        reset();
        struct mock_obj a = arr(1, 100 * 2 * 10, 1);
        CHECK(J(registerPlane)(env, NULL, 1, 9, 0, 0, 0, 0, &u16, 100, 10, 0, &a) == 77);
        CHECK(!pending[0] && fake.creates == 1 && fake.nwrites == 1 && fake.commits == 1 && fake.releases == 0);
        reset();
        struct mock_obj small = arr(1, 100 * 2 * 10 - 1, 1);
        CHECK(J(registerPlane)(env, NULL, 1, 9, 0, 0, 0, 0, &u16, 100, 10, 0, &small) == 0);
        CHECK(threw("java/lang/IllegalArgumentException") && fake.creates == 0);
        reset();
        fake.write_fail_at = 1;
        CHECK(J(registerPlane)(env, NULL, 1, 9, 0, 0, 0, 0, &u16, 100, 10, 0, &a) == 0);
        CHECK(threw("java/lang/RuntimeException") && fake.commits == 0 && fake.releases == 1);
    }
    /* ---- registerZarr: offsets checked against both Java arrays before the call */
    {
        struct mock_obj chunks = arr(1, 1000, 1);
        struct mock_obj offs = arr(2, 5, 8);  /* 2 x 2 chunks of 64 -> needs 5 entries */
        jlong* o = offs.data;
        o[0] = 0; o[1] = 100; o[2] = 100; o[3] = 600; o[4] = 1000;
        reset();
        CHECK(J(registerZarr)(env, NULL, 1, 9, 0, 0, 0, 0, &u16, 128, 128, 0, 64, 64, 1, &chunks, &offs, 0) == 55);
        CHECK(!pending[0] && fake.zarr_calls == 1);
        struct mock_obj shortoffs = arr(2, 4, 8);
        reset();
        CHECK(J(registerZarr)(env, NULL, 1, 9, 0, 0, 0, 0, &u16, 128, 128, 0, 64, 64, 1, &chunks, &shortoffs, 0) == 0);
        CHECK(threw("java/lang/IllegalArgumentException") && fake.zarr_calls == 0);
        o[4] = 1001;  /* past the chunk bytes */
        reset();
        CHECK(J(registerZarr)(env, NULL, 1, 9, 0, 0, 0, 0, &u16, 128, 128, 0, 64, 64, 1, &chunks, &offs, 0) == 0);
        CHECK(threw("java/lang/IllegalArgumentException") && fake.zarr_calls == 0);
        o[4] = 1000; o[2] = 50;  /* decreasing */
        reset();
        CHECK(J(registerZarr)(env, NULL, 1, 9, 0, 0, 0, 0, &u16, 128, 128, 0, 64, 64, 1, &chunks, &offs, 0) == 0);
        CHECK(threw("java/lang/IllegalArgumentException") && fake.zarr_calls == 0);
    }
    /* ---- sparse planes: createSparsePlane's arguments, writeBand's pieces and its 409 */
    {
        reset();
        CHECK(J(createSparsePlane)(env, NULL, 1, 9, 0, 0, 0, 0, &u16, 100000, 100000, 0, 512, 1024, 2048) == 88);
        CHECK(!pending[0] && fake.sparse_band_rows == 512 && fake.sparse_own_y0 == 1024 && fake.sparse_own_rows == 2048);
        reset();
        fake.create_rc = PBX_E_EXISTS;
        CHECK(J(createSparsePlane)(env, NULL, 1, 9, 0, 0, 0, 0, &u16, 100, 100, 0, 64, 0, 0) == 0 && !pending[0]);
        const jint row = 100000 * 2, rows = 512;  /* a 102 MB band: 7 pieces of <= 16 MiB */
        struct mock_obj a = arr(1, (size_t)row * rows, 1);
        reset();
        CHECK(J(writeBand)(env, NULL, 1, 88, 1024, rows, row, &a, 0) == 1 && !pending[0]);
        int32_t y = 1024;
        for (int i = 0; i < fake.nwrites; i++) {
            CHECK(fake.w_y0[i] == y && fake.w_bytes[i] <= (16u << 20));
            y += fake.w_rows[i];
        }
        CHECK(y == 1024 + rows && fake.nwrites == 7);
        reset();
        fake.band_exists = 1;  /* resident / being loaded: false, no exception */
        CHECK(J(writeBand)(env, NULL, 1, 88, 1024, rows, row, &a, 0) == 0 && !pending[0]);
        reset();
        CHECK(J(writeBand)(env, NULL, 1, 88, 1024, rows + 1, row, &a, 0) == 0 &&
              threw("java/lang/IllegalArgumentException"));
        /* a Java exception between pieces: the pieces written so far are given back
         * (pbx_band_abort), so the band does not stay loading */
        reset();
        region_fail_after = 3;
        CHECK(J(writeBand)(env, NULL, 1, 88, 1024, rows, row, &a, 0) == 0 && threw("java/lang/InternalError"));
        CHECK(fake.nwrites == 3 && fake.band_aborts == 1 && fake.abort_y0 == 1024);
        reset();  /* an exception before any piece: nothing to give back */
        region_fail_after = 0;
        CHECK(J(writeBand)(env, NULL, 1, 88, 1024, rows, row, &a, 0) == 0 && threw("java/lang/InternalError"));
        CHECK(fake.nwrites == 0 && fake.band_aborts == 0);
        free(a.data);
        reset();
        fake.sparse_band_rows = 512;
        fake.nbands = 5;
        struct mock_obj st = arr(1, 5, 1);
        CHECK(J(bandInfo)(env, NULL, 1, 88, &st) == 512);
        CHECK(((uint8_t*)st.data)[4] == 1 && ((uint8_t*)st.data)[2] == 2);
    }
    /* ---- the node: devices passed through, the serving context reported in statusOut[3] */
    {
        reset();
        struct mock_obj devs = arr(3, 2, 4);
        ((jint*)devs.data)[0] = 3;
        ((jint*)devs.data)[1] = 3;
        jlong node = J(nodeInit)(env, NULL, 2, &devs, 0, 0, 0, 512);
        CHECK(node != 0 && !pending[0] && fake.node_n == 2 && fake.node_dev0 == 3);
        CHECK(J(nodeContext)(env, NULL, node, 1) != 0 && !pending[0]);
        CHECK(J(nodeContext)(env, NULL, node, 2) == 0 && threw("java/lang/IllegalArgumentException"));
        reset();
        static const uint8_t body[3] = {7, 8, 9};
        fake.tile_fill = 1;
        fake.body = body;
        fake.body_len = 3;
        fake.served_by = 1;
        fake.node_n = 2;
        struct mock_obj so = arr(3, 4, 4);
        jbyteArray r = J(nodeGetTile)(env, NULL, node, 9, 0, 0, 0, -1, 0, 0, 8, 8, NULL, &so);
        CHECK(r && r->len == 3 && ((jint*)so.data)[2] == 0 && ((jint*)so.data)[3] == 1);
        CHECK(fake.releases_results == 1 && fake.bad_release == 0);
    }
    if (failures) {
        fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    printf("jni shim ok\n");
    return 0;
}
