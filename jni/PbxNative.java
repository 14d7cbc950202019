/*
 * JNI facade over libpbx.so (include/pbx.h) for omero-ms-pixel-buffer.  Drop into
 * src/main/java/com/glencoesoftware/omero/ms/pixelbuffer/ next to TileRequestHandler.java;
 * the native side is jni/pbx_jni.c (build: `make -C jni` with $JAVA_HOME set).
 *
 * What it replaces (paths under the reference's pixelbuffer package):
 *   getTile            TileRequestHandler.getTile body, :98-128 (getTileDirect :107-109 +
 *                      writeImage :123, with the w/h defaulting of :92-97)
 *   init / shutdown    PixelBufferMicroserviceVerticle.start :114-233 / stop :298-308
 *   declareImage       the Pixels row getPixels returns (:84, :220-241)
 *   createPlane / writeRows / commitPlane
 *                      getPixelBuffer (:86, :201-211) + getTileDirect reads, done once per
 *                      (image, z, c, t, level) — or per row band — instead of once per tile
 *   registerZarr       ZarrPixelsService chunk reads (PixelBufferVerticle.java:29,56)
 */
package com.glencoesoftware.omero.ms.pixelbuffer;

import java.nio.ByteBuffer;

final class PbxNative {
    static { System.loadLibrary("pbx_jni"); }   // libpbx_jni.so, linked against libpbx.so

    private PbxNative() {}

    /** pbx_status values getTile reports in statusOut[2]. */
    static final int OK = 0, BADARG = 400, NOTFOUND = 404, NOT_RESIDENT = 460, INTERNAL = 500;
    /** planeState values. */
    static final int PLANE_ABSENT = -1, PLANE_LOADING = 0, PLANE_READY = 1, PLANE_EVICTED = 2;

    /** pbx_init.  device -1 = $PBX_DEVICE / $LOCAL_RANK / 0; tiffTile 0 = one strip. */
    static native long init(int device, int pngFilter, boolean tiffDeflate, int tiffTile);

    static native void shutdown(long ctx);

    /**
     * pbx_image_declare: the Pixels row (pixelsType value, sizeX..T) and the PixelBuffer's
     * getResolutionLevels().  Idempotent; throws IllegalArgumentException if it contradicts
     * an earlier declaration.
     */
    static native void declareImage(long ctx, long imageId, String pixelsType, int sizeX, int sizeY,
                                    int sizeZ, int sizeC, int sizeT, int levels);

    static native void releaseImage(long ctx, long imageId);

    /**
     * pbx_plane_create: an empty plane of STORED level `level` (0 = full resolution), or only
     * its rows [bandY0, bandY0 + bandRows) (bandRows 0 = whole plane), whose rows arrive by
     * writeRows in the given byte order.  Returns the plane id, or 0 when another caller
     * holds the key (it is loading the plane: wait until planeState is no longer LOADING).
     * Throws 507 (RuntimeException) when the plane does not fit the HBM residency budget.
     */
    static native long createPlane(long ctx, long imageId, int z, int c, int t, int level,
                                   String pixelsType, int sizeX, int sizeY, boolean littleEndian,
                                   int bandY0, int bandRows);

    /**
     * pbx_plane_write_rows: `rows` packed rows of rowBytes (= sizeX * bytesPerPixel) from
     * data[off ..], e.g. one PixelBuffer.getTileDirect(z, c, t, 0, y0, sizeX, rows, data).
     * Copied out in pieces (no JNI critical section), so a band of any size may be passed.
     */
    static native void writeRows(long ctx, long planeId, int y0, int rows, int rowBytes, byte[] data,
                                 int off);

    /** The same from a direct ByteBuffer (its capacity bounds what is read). */
    static native void writeRowsDirect(long ctx, long planeId, int y0, int rows, ByteBuffer data);

    /** pbx_plane_commit: the plane is served from now on (every row must be written). */
    static native void commitPlane(long ctx, long planeId);

    /** pbx_plane_lookup: PLANE_ABSENT / LOADING / READY / EVICTED for a key. */
    static native int planeState(long ctx, long imageId, int z, int c, int t, int level);

    /** pbx_set_residency_budget: HBM bytes for planes (0 = none); idle planes evicted LRU. */
    static native void setResidencyBudget(long ctx, long bytes);

    /**
     * A whole plane (< 2 GiB) in one call: createPlane + writeRows + commitPlane.  Planes
     * larger than a Java array are loaded in row bands with those three calls.
     */
    static native long registerPlane(long ctx, long imageId, int z, int c, int t, int level,
                                     String pixelsType, int sizeX, int sizeY, boolean littleEndian,
                                     byte[] plane);

    /** pbx_plane_build_pyramid: `levels` 2x2-mean levels below the plane; returns their ids. */
    static native long[] buildPyramid(long ctx, long planeId, int levels);

    static native void releasePlane(long ctx, long planeId);

    /**
     * pbx_plane_register_zarr: the concatenated chunk files of one plane (C order over the
     * chunk grid, offsets has gx*gy + 1 non-decreasing entries within chunks, an empty range
     * = missing chunk).  codec 0 null, 1 blosc, 2 zlib (.zarray "compressor").
     */
    static native long registerZarr(long ctx, long imageId, int z, int c, int t, int level,
                                    String pixelsType, int sizeX, int sizeY, boolean littleEndian,
                                    int chunkX, int chunkY, int codec, byte[] chunks,
                                    long[] offsets, long fillBits);

    /**
     * pbx_get_tile: the response body, or null.  statusOut (length 3) receives the
     * post-defaulting w, h (the filename header's) and the status: OK; NOTFOUND / BADARG
     * where TileRequestHandler.getTile returns null (-> 404); NOT_RESIDENT when this context
     * does not hold the plane (load it, then call again).  resolution: TileCtx.resolution in
     * OMERO's numbering, null -> RESOLUTION_NONE, a given negative value -> below -1
     * (resolutionArg).  A device failure throws RuntimeException (-> 500,
     * PixelBufferVerticle.java:141-146).
     */
    static native byte[] getTile(long ctx, long imageId, int z, int c, int t, int resolution,
                                 int x, int y, int w, int h, String format, int[] statusOut);

    /**
     * pbx_plane_create_sparse: a plane held as bands of bandRows rows, each loaded on demand
     * (writeBand) and evicted on its own under the residency budget — region-proportional
     * residency, as getTileDirect reads only the requested region (:102-109).  ownY0/ownRows
     * (0/0 = all): the rows this context may hold.  Returns 0 when the key is taken (409).
     */
    static native long createSparsePlane(long ctx, long imageId, int z, int c, int t, int level,
                                         String pixelsType, int sizeX, int sizeY, boolean littleEndian,
                                         int bandRows, int ownY0, int ownRows);

    /**
     * pbx_band_write: rows [y0, y0 + rows) of ONE band from data[off ..], e.g. one
     * getTileDirect(z, c, t, 0, y0, sizeX, rows, data); copied out in pieces.  Returns false
     * when the band is resident or being loaded by another caller (409).
     */
    static native boolean writeBand(long ctx, long planeId, int y0, int rows, int rowBytes, byte[] data,
                                    int off);

    /** pbx_plane_band_info: bandRows; states[k] = 0 absent, 1 loading, 2 resident (may be null). */
    static native int bandInfo(long ctx, long planeId, byte[] states);

    /**
     * pbx_node_init: `n` device contexts in this JVM (devices null = 0..n-1), one per GPU of the
     * node; nodeContext(node, k) is context k (declare / load planes there).  nodeGetTile routes
     * a request to the context holding its plane or row band (statusOut[3] = its index; on
     * NOT_RESIDENT the context to load into).  PixelBufferMicroserviceVerticle.java:224-233.
     */
    static native long nodeInit(int n, int[] devices, int pngFilter, boolean tiffDeflate, int tiffTile,
                                int shardTile);

    static native void nodeShutdown(long node);

    static native long nodeContext(long node, int k);

    static native byte[] nodeGetTile(long node, long imageId, int z, int c, int t, int resolution,
                                     int x, int y, int w, int h, String format, int[] statusOut);

    static final int RESOLUTION_NONE = -1;

    /** TileCtx.resolution (Integer, may be null) -> the int getTile takes. */
    static int resolutionArg(Integer resolution) {
        if (resolution == null) return RESOLUTION_NONE;
        return resolution < 0 ? Integer.MIN_VALUE : resolution;
    }
}
