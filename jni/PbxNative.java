/*
 * JNI facade over libpbx.so (include/pbx.h) for omero-ms-pixel-buffer.  Drop into
 * src/main/java/com/glencoesoftware/omero/ms/pixelbuffer/ next to TileRequestHandler.java;
 * the native side is jni/pbx_jni.c (build: `make -C jni` with $JAVA_HOME set).
 *
 * What it replaces (paths under the reference's pixelbuffer package):
 *   getTile            TileRequestHandler.getTile body, :98-128 (getTileDirect :107-109 +
 *                      writeImage :123, with the w/h defaulting of :92-97)
 *   init / shutdown    PixelBufferMicroserviceVerticle.start :114-233 / stop :298-308
 *   registerPlane      the PixelBuffer a deployment reads planes from (ROMIO / Zarr),
 *                      once per (image, z, c, t, level) instead of once per tile
 *   registerZarr       ZarrPixelsService chunk reads (PixelBufferVerticle.java:29,56)
 */
package com.glencoesoftware.omero.ms.pixelbuffer;

final class PbxNative {
    static { System.loadLibrary("pbx_jni"); }   // libpbx_jni.so, linked against libpbx.so

    private PbxNative() {}

    /** pbx_init.  device -1 = $PBX_DEVICE / $LOCAL_RANK / 0; tiffTile 0 = one strip. */
    static native long init(int device, int pngFilter, boolean tiffDeflate, int tiffTile);

    static native void shutdown(long ctx);

    /**
     * pbx_plane_register of one plane's samples as PixelBuffer returns them (big-endian
     * unless littleEndian).  level = STORED level, 0 = full resolution.  Returns the plane
     * id; throws IllegalArgumentException (400) / RuntimeException (500).
     */
    static native long registerPlane(long ctx, long imageId, int z, int c, int t, int level,
                                     String pixelsType /* Pixels.getPixelsType() value */,
                                     int sizeX, int sizeY, boolean littleEndian, byte[] plane);

    /** pbx_plane_build_pyramid: `levels` 2x2-mean levels below the plane; returns their ids. */
    static native long[] buildPyramid(long ctx, long planeId, int levels);

    static native void releasePlane(long ctx, long planeId);

    /**
     * pbx_plane_register_zarr: the concatenated chunk files of one plane (C order over the
     * chunk grid, offsets has gx*gy + 1 entries, an empty range = missing chunk).
     * codec 0 null, 1 blosc, 2 zlib (.zarray "compressor").
     */
    static native long registerZarr(long ctx, long imageId, int z, int c, int t, int level,
                                    String pixelsType, int sizeX, int sizeY, boolean littleEndian,
                                    int chunkX, int chunkY, int codec, byte[] chunks,
                                    long[] offsets, long fillBits);

    /**
     * pbx_get_tile: the response body, or null exactly where TileRequestHandler.getTile
     * returns null (-> 404).  resolution: TileCtx.resolution in OMERO's numbering, null
     * -> pass RESOLUTION_NONE; a given negative value must be passed as < -1 (it throws in
     * setResolutionLevel upstream -> null).  regionOut receives the post-defaulting w, h.
     * A device failure throws RuntimeException (-> 500, PixelBufferVerticle.java:141-146).
     */
    static native byte[] getTile(long ctx, long imageId, int z, int c, int t, int resolution,
                                 int x, int y, int w, int h, String format, int[] regionOut);

    static final int RESOLUTION_NONE = -1;

    /** TileCtx.resolution (Integer, may be null) -> the int getTile takes. */
    static int resolutionArg(Integer resolution) {
        if (resolution == null) return RESOLUTION_NONE;
        return resolution < 0 ? Integer.MIN_VALUE : resolution;
    }
}
