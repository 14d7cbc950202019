/* pbx_jni.c — JNI side of jni/PbxNative.java over the C-ABI in include/pbx.h.
 *
 * Build (needs a JDK; there is none in this image): `make -C jni` with $JAVA_HOME set,
 * producing jni/libpbx_jni.so linked against omero-ms-pixel-buffer_amd/lib/libpbx.so.
 *
 * Error mapping follows the reference: PBX_E_NOTFOUND / PBX_E_BADARG statuses of a tile are
 * the nulls TileRequestHandler.getTile returns (-> 404, PixelBufferVerticle.java:132-136);
 * PBX_E_INTERNAL is an exception (-> 500, :141-146).  PBX_E_NOT_RESIDENT is reported through
 * getTile's status slot so that the handler can load the plane (getPixels + getPixelBuffer)
 * and retry.  Registration errors throw IllegalArgumentException (400) or
 * RuntimeException (500).
 *
 * No JNI critical section is ever held across library calls: Java arrays are copied out in
 * bounded pieces (GetByteArrayRegion) into native buffers, or read in place from direct
 * ByteBuffers, so the GPU work never stalls the JVM's garbage collector. */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pbx.h"

#define PBX_CTX(h) ((pbx_ctx*)(intptr_t)(h))
#define PIECE_BYTES (16u << 20) /* Java -> native copy granule of writeRows */

static void throw_class(JNIEnv* env, const char* cls, const char* msg) {
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, msg);
}

/* The message starts "pbx status <code>: " (e.g. 507: the residency budget is held; the
 * handler waits and loads again). */
static void throw_status(JNIEnv* env, int st) {
    char msg[512];
    const char* e = pbx_last_error();
    snprintf(msg, sizeof msg, "pbx status %d: %s", st, e ? e : "");
    throw_class(env, st == PBX_E_BADARG || st == PBX_E_NOTFOUND || st == PBX_E_EXISTS
                         ? "java/lang/IllegalArgumentException" : "java/lang/RuntimeException",
                msg);
}

static int pixel_type(JNIEnv* env, jstring s) {
    if (!s) return -1;
    const char* p = (*env)->GetStringUTFChars(env, s, NULL);
    int pt = p ? pbx_pixel_type_from_string(p) : -1;
    if (p) (*env)->ReleaseStringUTFChars(env, s, p);
    return pt;
}

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_init(
        JNIEnv* env, jclass cls, jint device, jint png_filter, jboolean tiff_deflate, jint tiff_tile) {
    (void)cls;
    pbx_config cfg;
    pbx_config_default(&cfg);
    cfg.device = device;
    cfg.png_filter = png_filter;
    cfg.tiff_deflate = tiff_deflate ? 1 : 0;
    cfg.tiff_tile = tiff_tile;
    pbx_ctx* ctx = NULL;
    int st = pbx_init(&cfg, &ctx);
    if (st != PBX_OK) {
        throw_status(env, st);
        return 0;
    }
    return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_shutdown(
        JNIEnv* env, jclass cls, jlong ctx) {
    (void)env; (void)cls;
    pbx_shutdown(PBX_CTX(ctx));
}

static void fill_desc(pbx_plane_desc* d, jlong image, jint z, jint c, jint t, jint level, int pt,
                      jint sx, jint sy, jboolean le) {
    memset(d, 0, sizeof *d);
    d->image_id = image; d->z = z; d->c = c; d->t = t; d->resolution = level;
    d->pixel_type = pt; d->size_x = sx; d->size_y = sy;
    d->byte_order = le ? PBX_LITTLE_ENDIAN : PBX_BIG_ENDIAN;
    d->source = PBX_SRC_HOST;
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_declareImage(
        JNIEnv* env, jclass cls, jlong ctx, jlong image, jstring ptype, jint sx, jint sy, jint sz, jint sc,
        jint st_, jint levels) {
    (void)cls;
    pbx_image_desc d;
    memset(&d, 0, sizeof d);
    d.image_id = image;
    d.pixel_type = pixel_type(env, ptype);
    d.size_x = sx; d.size_y = sy; d.size_z = sz; d.size_c = sc; d.size_t_ = st_;
    d.levels = levels;
    int st = pbx_image_declare(PBX_CTX(ctx), &d);
    if (st != PBX_OK) throw_status(env, st);
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_releaseImage(
        JNIEnv* env, jclass cls, jlong ctx, jlong image) {
    (void)cls;
    int st = pbx_image_release(PBX_CTX(ctx), image);
    if (st != PBX_OK && st != PBX_E_NOTFOUND) throw_status(env, st);
}

/* 0 when another caller holds the key (409: it is loading or has loaded the plane). */
JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_createPlane(
        JNIEnv* env, jclass cls, jlong ctx, jlong image, jint z, jint c, jint t, jint level,
        jstring ptype, jint sx, jint sy, jboolean le, jint band_y0, jint band_rows) {
    (void)cls;
    pbx_plane_desc d;
    fill_desc(&d, image, z, c, t, level, pixel_type(env, ptype), sx, sy, le);
    uint64_t id = 0;
    int st = pbx_plane_create(PBX_CTX(ctx), &d, band_y0, band_rows, &id);
    if (st == PBX_E_EXISTS) return 0;
    if (st != PBX_OK) {
        throw_status(env, st);
        return 0;
    }
    return (jlong)id;
}

/* Rows [y0, y0 + rows) from data[off .. off + rows * rowBytes): copied out of the Java array
 * in whole-row pieces of at most PIECE_BYTES (no critical section), each handed to
 * pbx_plane_write_rows (pinned staging, DMA). */
JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_writeRows(
        JNIEnv* env, jclass cls, jlong ctx, jlong plane, jint y0, jint rows, jint row_bytes, jbyteArray data,
        jint off) {
    (void)cls;
    if (!data || rows < 0 || row_bytes <= 0 || off < 0) {
        throw_class(env, "java/lang/IllegalArgumentException", "writeRows: bad arguments");
        return;
    }
    const jsize n = (*env)->GetArrayLength(env, data);
    if ((int64_t)off + (int64_t)rows * row_bytes > (int64_t)n) {
        throw_class(env, "java/lang/IllegalArgumentException", "writeRows: array shorter than rows * rowBytes");
        return;
    }
    if (!rows) return;
    int32_t per = (int32_t)(PIECE_BYTES / (uint32_t)row_bytes);
    if (per < 1) per = 1;
    if (per > rows) per = rows;
    jbyte* buf = malloc((size_t)per * (size_t)row_bytes);
    if (!buf) {
        throw_class(env, "java/lang/OutOfMemoryError", "writeRows: native staging buffer");
        return;
    }
    for (int32_t r = 0; r < rows; r += per) {
        const int32_t k = rows - r < per ? rows - r : per;
        (*env)->GetByteArrayRegion(env, data, off + r * row_bytes, k * row_bytes, buf);
        if ((*env)->ExceptionCheck(env)) break;
        int st = pbx_plane_write_rows(PBX_CTX(ctx), (uint64_t)plane, y0 + r, k, buf, (uint64_t)k * row_bytes);
        if (st != PBX_OK) {
            throw_status(env, st);
            break;
        }
    }
    free(buf);
}

/* The same from a direct ByteBuffer (no copy on the Java side). */
JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_writeRowsDirect(
        JNIEnv* env, jclass cls, jlong ctx, jlong plane, jint y0, jint rows, jobject buffer) {
    (void)cls;
    void* p = buffer ? (*env)->GetDirectBufferAddress(env, buffer) : NULL;
    const jlong cap = buffer ? (*env)->GetDirectBufferCapacity(env, buffer) : -1;
    if (!p || cap < 0) {
        throw_class(env, "java/lang/IllegalArgumentException", "writeRowsDirect: not a direct buffer");
        return;
    }
    int st = pbx_plane_write_rows(PBX_CTX(ctx), (uint64_t)plane, y0, rows, p, (uint64_t)cap);
    if (st != PBX_OK) throw_status(env, st);
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_commitPlane(
        JNIEnv* env, jclass cls, jlong ctx, jlong plane) {
    (void)cls;
    int st = pbx_plane_commit(PBX_CTX(ctx), (uint64_t)plane);
    if (st != PBX_OK) throw_status(env, st);
}

/* State of the plane under a key: 0 loading, 1 ready, 2 evicted; -1 not registered. */
JNIEXPORT jint JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_planeState(
        JNIEnv* env, jclass cls, jlong ctx, jlong image, jint z, jint c, jint t, jint level) {
    (void)cls;
    int32_t state = -1;
    int st = pbx_plane_lookup(PBX_CTX(ctx), image, z, c, t, level, NULL, &state, NULL, NULL);
    if (st == PBX_E_NOTFOUND) return -1;
    if (st != PBX_OK) {
        throw_status(env, st);
        return -1;
    }
    return state;
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_setResidencyBudget(
        JNIEnv* env, jclass cls, jlong ctx, jlong bytes) {
    (void)cls;
    int st = pbx_set_residency_budget(PBX_CTX(ctx), bytes < 0 ? 0 : (uint64_t)bytes);
    if (st != PBX_OK) throw_status(env, st);
}

/* A whole plane in one call, through the same create / writeRows / commit path (a plane
 * larger than a Java array is loaded with createPlane + writeRows bands instead). */
JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_registerPlane(
        JNIEnv* env, jclass cls, jlong ctx, jlong image, jint z, jint c, jint t, jint level,
        jstring ptype, jint sx, jint sy, jboolean le, jbyteArray plane) {
    const int pt = pixel_type(env, ptype);
    const int bpp = pbx_bytes_per_pixel(pt);
    if (!plane || bpp <= 0 || sx <= 0 || sy <= 0) {
        throw_class(env, "java/lang/IllegalArgumentException", "registerPlane: bad arguments");
        return 0;
    }
    const int64_t row = (int64_t)sx * bpp;
    if (row > 0x7fffffff || row * sy > (int64_t)(*env)->GetArrayLength(env, plane)) {
        throw_class(env, "java/lang/IllegalArgumentException", "registerPlane: array shorter than the plane");
        return 0;
    }
    pbx_plane_desc d;
    fill_desc(&d, image, z, c, t, level, pt, sx, sy, le);
    uint64_t id = 0;
    int st = pbx_plane_create(PBX_CTX(ctx), &d, 0, 0, &id);
    if (st != PBX_OK) {
        throw_status(env, st);
        return 0;
    }
    Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_writeRows(env, cls, ctx, (jlong)id, 0, sy,
                                                                      (jint)row, plane, 0);
    if (!(*env)->ExceptionCheck(env)) {
        st = pbx_plane_commit(PBX_CTX(ctx), id);
        if (st == PBX_OK) return (jlong)id;
        throw_status(env, st);
    }
    (void)pbx_plane_release(PBX_CTX(ctx), id);  /* all or nothing */
    return 0;
}

JNIEXPORT jlongArray JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_buildPyramid(
        JNIEnv* env, jclass cls, jlong ctx, jlong plane, jint levels) {
    (void)cls;
    if (levels <= 0) return (*env)->NewLongArray(env, 0);
    uint64_t* ids = calloc((size_t)levels, sizeof *ids);
    if (!ids) {
        throw_status(env, PBX_E_INTERNAL);
        return NULL;
    }
    int st = pbx_plane_build_pyramid(PBX_CTX(ctx), (uint64_t)plane, levels, ids, NULL);
    jlongArray out = NULL;
    if (st == PBX_OK) {
        out = (*env)->NewLongArray(env, levels);
        if (out) (*env)->SetLongArrayRegion(env, out, 0, levels, (const jlong*)ids);
    } else {
        throw_status(env, st);
    }
    free(ids);
    return out;
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_releasePlane(
        JNIEnv* env, jclass cls, jlong ctx, jlong plane) {
    (void)cls;
    int st = pbx_plane_release(PBX_CTX(ctx), (uint64_t)plane);
    if (st != PBX_OK) throw_status(env, st);
}

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_registerZarr(
        JNIEnv* env, jclass cls, jlong ctx, jlong image, jint z, jint c, jint t, jint level,
        jstring ptype, jint sx, jint sy, jboolean le, jint chunk_x, jint chunk_y, jint codec,
        jbyteArray chunks, jlongArray offsets, jlong fill_bits) {
    (void)cls;
    if (!chunks || !offsets || sx <= 0 || sy <= 0 || chunk_x <= 0 || chunk_y <= 0) {
        throw_class(env, "java/lang/IllegalArgumentException", "registerZarr: bad arguments");
        return 0;
    }
    /* the C-ABI reads offsets[0 .. gx*gy] and data[0 .. offsets[gx*gy]): check both against
     * the Java arrays before handing them over */
    const int64_t gx = ((int64_t)sx + chunk_x - 1) / chunk_x, gy = ((int64_t)sy + chunk_y - 1) / chunk_y;
    const jsize n_off = (*env)->GetArrayLength(env, offsets), n_data = (*env)->GetArrayLength(env, chunks);
    if ((int64_t)n_off < gx * gy + 1) {
        throw_class(env, "java/lang/IllegalArgumentException", "registerZarr: offsets needs gx*gy + 1 entries");
        return 0;
    }
    jlong* offs = (*env)->GetLongArrayElements(env, offsets, NULL);
    if (!offs) return 0;  /* OutOfMemoryError pending */
    for (int64_t i = 0; i < gx * gy; i++)
        if (offs[i] < 0 || offs[i + 1] < offs[i] || offs[i + 1] > (jlong)n_data) {
            (*env)->ReleaseLongArrayElements(env, offsets, offs, JNI_ABORT);
            throw_class(env, "java/lang/IllegalArgumentException",
                        "registerZarr: offsets must be non-decreasing and within chunks");
            return 0;
        }
    /* a copy (or a pinned view the VM chooses), never a critical section: the call below
     * uploads and decodes on the GPU */
    jbyte* data = (*env)->GetByteArrayElements(env, chunks, NULL);
    if (!data) {
        (*env)->ReleaseLongArrayElements(env, offsets, offs, JNI_ABORT);
        return 0;
    }
    pbx_plane_desc d;
    fill_desc(&d, image, z, c, t, level, pixel_type(env, ptype), sx, sy, le);
    pbx_zarr_chunks zc;
    memset(&zc, 0, sizeof zc);
    zc.chunk_x = chunk_x; zc.chunk_y = chunk_y; zc.codec = codec;
    zc.data = (const uint8_t*)data;
    zc.offsets = (const uint64_t*)offs;
    zc.fill_bits = (uint64_t)fill_bits;
    uint64_t id = 0;
    int st = pbx_plane_register_zarr(PBX_CTX(ctx), &d, &zc, &id, NULL);
    (*env)->ReleaseByteArrayElements(env, chunks, data, JNI_ABORT);
    (*env)->ReleaseLongArrayElements(env, offsets, offs, JNI_ABORT);
    if (st != PBX_OK) throw_status(env, st);   /* 400: corrupt / unsupported chunk */
    return (jlong)id;
}

/* One getTile through a context (node == 0) or a node's router. */
static jbyteArray tile_call(JNIEnv* env, jlong ctx, jlong node, jlong image, jint z, jint c, jint t, jint res,
                            jint x, jint y, jint w, jint h, jstring jfmt, jintArray status_out) {
    pbx_tile_req req;
    memset(&req, 0, sizeof req);
    req.image_id = image; req.z = z; req.c = c; req.t = t; req.resolution = res;
    req.x = x; req.y = y; req.w = w; req.h = h;
    const char* fmt = jfmt ? (*env)->GetStringUTFChars(env, jfmt, NULL) : NULL;
    if (jfmt && !fmt) return NULL;  /* OutOfMemoryError pending */
    req.format = pbx_format_from_string(fmt);
    if (fmt) (*env)->ReleaseStringUTFChars(env, jfmt, fmt);
    pbx_result r;
    memset(&r, 0, sizeof r);   /* pbx_get_tile may return before it writes the result */
    r.status = PBX_E_INTERNAL;
    int32_t served_by = -1;
    int st = node ? pbx_node_get_tile((pbx_node*)(intptr_t)node, &req, &r, &served_by)
                  : pbx_get_tile(PBX_CTX(ctx), &req, &r);
    /* a call-level failure (null ctx, shutdown, failed plan) leaves the result unfilled */
    const int status = r.owner || r.status == st ? r.status : st;
    if (status_out && (*env)->GetArrayLength(env, status_out) >= 3) {
        jint v[4] = {r.w, r.h, status, served_by};
        const jsize n = node && (*env)->GetArrayLength(env, status_out) >= 4 ? 4 : 3;
        (*env)->SetIntArrayRegion(env, status_out, 0, n, v);
    }
    jbyteArray out = NULL;
    if (status == PBX_OK) {
        if (r.len > 0x7fffffffu) {  /* a Java array cannot hold it */
            if (r.owner) pbx_results_release(PBX_CTX(ctx), &r, 1);
            throw_class(env, "java/lang/IllegalArgumentException", "tile response larger than 2^31-1 bytes");
            return NULL;
        }
        out = (*env)->NewByteArray(env, (jsize)r.len);   /* exact length, :188-193 */
        if (out && r.len) (*env)->SetByteArrayRegion(env, out, 0, (jsize)r.len, (const jbyte*)r.data);
    }
    if (r.owner) pbx_results_release(NULL, &r, 1);
    if (status == PBX_E_INTERNAL) {
        throw_status(env, status);   /* -> 500 */
        return NULL;
    }
    return out;   /* null for every status the reference answers null, and NOT_RESIDENT */
}

/* statusOut (length >= 3): [0] w, [1] h after the :92-97 defaulting, [2] the pbx status. */
JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_getTile(
        JNIEnv* env, jclass cls, jlong ctx, jlong image, jint z, jint c, jint t, jint res,
        jint x, jint y, jint w, jint h, jstring jfmt, jintArray status_out) {
    (void)cls;
    return tile_call(env, ctx, 0, image, z, c, t, res, x, y, w, h, jfmt, status_out);
}

/* ---- sparse (banded) planes: region-proportional residency */

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_createSparsePlane(
        JNIEnv* env, jclass cls, jlong ctx, jlong image, jint z, jint c, jint t, jint level,
        jstring ptype, jint sx, jint sy, jboolean le, jint band_rows, jint own_y0, jint own_rows) {
    (void)cls;
    pbx_plane_desc d;
    fill_desc(&d, image, z, c, t, level, pixel_type(env, ptype), sx, sy, le);
    uint64_t id = 0;
    int st = pbx_plane_create_sparse(PBX_CTX(ctx), &d, band_rows, own_y0, own_rows, &id);
    if (st == PBX_E_EXISTS) return 0;
    if (st != PBX_OK) {
        throw_status(env, st);
        return 0;
    }
    return (jlong)id;
}

/* Rows of one band, copied out of the Java array in whole-row pieces (no critical section). */
JNIEXPORT jboolean JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_writeBand(
        JNIEnv* env, jclass cls, jlong ctx, jlong plane, jint y0, jint rows, jint row_bytes, jbyteArray data,
        jint off) {
    (void)cls;
    if (!data || rows <= 0 || row_bytes <= 0 || off < 0) {
        throw_class(env, "java/lang/IllegalArgumentException", "writeBand: bad arguments");
        return JNI_FALSE;
    }
    if ((int64_t)off + (int64_t)rows * row_bytes > (int64_t)(*env)->GetArrayLength(env, data)) {
        throw_class(env, "java/lang/IllegalArgumentException", "writeBand: array shorter than rows * rowBytes");
        return JNI_FALSE;
    }
    int32_t per = (int32_t)(PIECE_BYTES / (uint32_t)row_bytes);
    if (per < 1) per = 1;
    if (per > rows) per = rows;
    jbyte* buf = malloc((size_t)per * (size_t)row_bytes);
    if (!buf) {
        throw_class(env, "java/lang/OutOfMemoryError", "writeBand: native staging buffer");
        return JNI_FALSE;
    }
    jboolean ok = JNI_TRUE;
    for (int32_t r = 0; r < rows; r += per) {
        const int32_t k = rows - r < per ? rows - r : per;
        (*env)->GetByteArrayRegion(env, data, off + r * row_bytes, k * row_bytes, buf);
        if ((*env)->ExceptionCheck(env)) {
            /* the pieces written so far would leave the band loading: give it back */
            if (r) (void)pbx_band_abort(PBX_CTX(ctx), (uint64_t)plane, y0);
            ok = JNI_FALSE;
            break;
        }
        int st = pbx_band_write(PBX_CTX(ctx), (uint64_t)plane, y0 + r, k, buf, (uint64_t)k * row_bytes);
        if (st == PBX_E_EXISTS && r == 0) {  /* resident, or another caller loads it */
            ok = JNI_FALSE;
            break;
        }
        if (st != PBX_OK) {  /* (a failed write has already reset the band) */
            throw_status(env, st);
            ok = JNI_FALSE;
            break;
        }
    }
    free(buf);
    return ok;
}

JNIEXPORT jint JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_bandInfo(
        JNIEnv* env, jclass cls, jlong ctx, jlong plane, jbyteArray states) {
    (void)cls;
    int32_t band_rows = 0, nbands = 0;
    int st = pbx_plane_band_info(PBX_CTX(ctx), (uint64_t)plane, &band_rows, &nbands, NULL);
    if (st != PBX_OK) {
        throw_status(env, st);
        return 0;
    }
    if (states && nbands > 0) {
        uint8_t* s = malloc((size_t)nbands);
        if (!s) {
            throw_class(env, "java/lang/OutOfMemoryError", "bandInfo");
            return 0;
        }
        st = pbx_plane_band_info(PBX_CTX(ctx), (uint64_t)plane, NULL, NULL, s);
        jsize n = (*env)->GetArrayLength(env, states);
        if (n > nbands) n = nbands;
        if (st == PBX_OK) (*env)->SetByteArrayRegion(env, states, 0, n, (const jbyte*)s);
        free(s);
        if (st != PBX_OK) throw_status(env, st);
    }
    return band_rows;
}

/* ---- a node: one context per GPU in this JVM, requests routed to the context holding them */

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_nodeInit(
        JNIEnv* env, jclass cls, jint n, jintArray devices, jint png_filter, jboolean tiff_deflate, jint tiff_tile,
        jint shard_tile) {
    (void)cls;
    pbx_config cfg;
    pbx_config_default(&cfg);
    cfg.png_filter = png_filter;
    cfg.tiff_deflate = tiff_deflate ? 1 : 0;
    cfg.tiff_tile = tiff_tile;
    int32_t* devs = NULL;
    if (devices) {
        if ((*env)->GetArrayLength(env, devices) < n) {
            throw_class(env, "java/lang/IllegalArgumentException", "nodeInit: fewer devices than contexts");
            return 0;
        }
        devs = malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
        if (!devs) {
            throw_class(env, "java/lang/OutOfMemoryError", "nodeInit");
            return 0;
        }
        (*env)->GetIntArrayRegion(env, devices, 0, n, (jint*)devs);
    }
    pbx_node* node = NULL;
    int st = pbx_node_init(&cfg, n, devs, shard_tile, &node);
    free(devs);
    if (st != PBX_OK) {
        throw_status(env, st);
        return 0;
    }
    return (jlong)(intptr_t)node;
}

JNIEXPORT void JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_nodeShutdown(
        JNIEnv* env, jclass cls, jlong node) {
    (void)env; (void)cls;
    pbx_node_shutdown((pbx_node*)(intptr_t)node);
}

JNIEXPORT jlong JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_nodeContext(
        JNIEnv* env, jclass cls, jlong node, jint k) {
    (void)cls;
    pbx_ctx* c = pbx_node_context((pbx_node*)(intptr_t)node, k);
    if (!c) throw_class(env, "java/lang/IllegalArgumentException", "nodeContext: no such context");
    return (jlong)(intptr_t)c;
}

/* statusOut (length >= 4): w, h, status, index of the context that served (or should load) it. */
JNIEXPORT jbyteArray JNICALL Java_com_glencoesoftware_omero_ms_pixelbuffer_PbxNative_nodeGetTile(
        JNIEnv* env, jclass cls, jlong node, jlong image, jint z, jint c, jint t, jint res,
        jint x, jint y, jint w, jint h, jstring jfmt, jintArray status_out) {
    (void)cls;
    if (!node) {
        throw_class(env, "java/lang/IllegalArgumentException", "nodeGetTile: null node");
        return NULL;
    }
    return tile_call(env, 0, node, image, z, c, t, res, x, y, w, h, jfmt, status_out);
}
