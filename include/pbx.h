/*
 * pbx.h — C-ABI of the MI355X-native /tile pipeline (drop-in for the
 * omero-ms-pixel-buffer tile hot path).
 *
 * Plain C: no exceptions, no torch/HIP types, plain pointers and sizes.  Every
 * entry point is thread-safe.  Each declaration cites the reference interface
 * it replaces; paths are relative to
 * /root/reference/src/main/java/com/glencoesoftware/omero/ms/pixelbuffer/.
 *
 * Mapping to the reference:
 *   TileCtx (TileCtx.java:30-92)                  -> pbx_tile_req
 *   TileRequestHandler.getTile (TileRequestHandler.java:80-139)
 *                                                 -> pbx_get_tile / pbx_get_tiles
 *   PixelBuffer.getTileDirect (:107-109)          -> kernel K1 (extract + big-endian)
 *   writeImage("png"|"tif") (:176-199)            -> kernels K2..K7 (filter/deflate/frame)
 *   PixelsService.getPixelBuffer (:201-211)       -> planes registered with pbx_plane_register
 *   getPixels (Ice HQL, :220-241)                 -> the plane registry's image records
 *   reply "filename" header (PixelBufferVerticle.java:116-126)  -> pbx_tile_filename
 *   Content-Type (PixelBufferMicroserviceVerticle.java:373-379)  -> pbx_content_type
 */
#ifndef PBX_H
#define PBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBX_ABI_VERSION 9

/* Status codes are the HTTP status the reference's event-bus consumer ends with:
 * getTile() == null -> message.fail(404) (PixelBufferVerticle.java:111-114);
 * IllegalArgumentException -> 400 (:137-140); any other exception -> 500 (:141-146).
 *
 * PBX_E_NOT_RESIDENT is never sent to a client.  It means "this context does not hold the
 * plane the request needs": the image is unknown here, its (z, c, t, level) plane was never
 * loaded or was evicted, or the region lies outside the row band this context owns.  The
 * reference would open the plane on demand (getPixels + getPixelBuffer,
 * TileRequestHandler.java:84-86,201-241); the binding does the same — look the image up,
 * load the plane with pbx_image_declare / pbx_plane_create / pbx_plane_write_rows /
 * pbx_plane_commit and retry.  A context answers 404 only for what the
 * reference itself answers 404. */
enum pbx_status {
    PBX_OK = 0,
    PBX_E_BADARG = 400,
    PBX_E_NOTFOUND = 404,
    PBX_E_EXISTS = 409,      /* registration: the (image, z, c, t, level) key is taken (loaded
                                or being loaded by another caller) */
    PBX_E_NOT_RESIDENT = 460,/* tile status: load the plane, then retry (see above) */
    PBX_E_INTERNAL = 500,
    PBX_E_PENDING = 504,     /* pbx_wait: the batch is still running (not a tile status) */
    PBX_E_NO_SPACE = 507     /* registration: the plane does not fit the HBM residency budget
                                even after evicting every idle plane */
};

/* OMERO pixel types (ome.xml.model.enums.PixelType; TileRequestHandler.java:100-101,164-165). */
enum pbx_pixel_type {
    PBX_INT8 = 0, PBX_UINT8, PBX_INT16, PBX_UINT16, PBX_INT32, PBX_UINT32, PBX_FLOAT, PBX_DOUBLE,
    PBX_NPIXEL_TYPES
};

/* TileCtx.format (TileCtx.java:89): null -> raw bytes (:128), "png"/"tif" -> writeImage
 * (:122-123), anything else -> null -> 404 (:125-126). */
enum pbx_format { PBX_FMT_RAW = 0, PBX_FMT_PNG = 1, PBX_FMT_TIF = 2, PBX_FMT_UNKNOWN = 3 };

/* Byte order of the samples of a registered plane as handed to pbx_plane_register. */
enum pbx_byte_order { PBX_BIG_ENDIAN = 0, PBX_LITTLE_ENDIAN = 1 };

/* Plane sources: host bytes (copied to HBM) or an on-device synthetic generator
 * (Bio-Formats FakeReader-style G_FAKE, counter-hash G_NOISE). */
enum pbx_source { PBX_SRC_HOST = 0, PBX_SRC_GEN_FAKE = 1, PBX_SRC_GEN_NOISE = 2 };

/* PNG scanline filter used by the encoder.  NONE is what the reference's APNGWriter
 * writes (filter byte 0 on every row); the others decode to identical pixels.  ADAPTIVE: per
 * tile, NONE on every row when the tile's middle row says filtering does not pay, else per row
 * the filter with the smallest sum of |byte - prediction|. */
enum pbx_png_filter {
    PBX_FILTER_NONE = 0, PBX_FILTER_SUB = 1, PBX_FILTER_UP = 2, PBX_FILTER_AVG = 3,
    PBX_FILTER_PAETH = 4, PBX_FILTER_ADAPTIVE = 5
};

typedef struct pbx_config {
    int32_t device;          /* HIP device ordinal; -1 = $PBX_DEVICE, else $LOCAL_RANK, else 0 */
    int32_t png_filter;      /* enum pbx_png_filter; default NONE (reference) */
    int32_t tiff_deflate;    /* 0 = uncompressed TIFF (reference default); 1 = Compression=8 */
    int32_t segment_bytes;   /* deflate segment size (bytes of filtered stream); 0 = default */
    uint64_t max_batch_bytes;/* device scratch budget per batch; 0 = default */
    int32_t coalesce;        /* 1 (default) = concurrent pbx_get_tile calls are coalesced into
                                batches (one per GPU-busy interval); 0 = one batch per call */
    int32_t stage_rows;      /* 0 (default) = the deflate kernels read filter-None rows straight
                                from the plane; 1 = stage them in a stream buffer first (k_rows) */
    int32_t tiff_tile;       /* 0 (reference) = TIFF as one strip; T = tiled TIFF (TIFF 6.0 s.15)
                                of T x T tiles, edge tiles zero-padded; T a multiple of 16 in
                                [16, 4096]; with tiff_deflate every tile is its own zlib stream */
    int32_t request_timeout_us; /* deadline of one pbx_get_tile / pbx_node_get_tile call: past it
                                the call answers PBX_E_INTERNAL (500), as the reference's
                                event-bus send timeout does (PixelBufferMicroserviceVerticle.java:
                                148-151 default 15 s, :356-366 timeout -> 500); the late batch's
                                results are released when it completes.  0 = $PBX_REQUEST_TIMEOUT_US,
                                else 15,000,000; < 0 = no deadline */
} pbx_config;

typedef struct pbx_ctx pbx_ctx;

/* Lifecycle (PixelBufferMicroserviceVerticle.start/deploy :114-233, stop :298-308). */
int pbx_config_default(pbx_config* cfg);
int pbx_init(const pbx_config* cfg, pbx_ctx** out);
void pbx_shutdown(pbx_ctx* ctx);
/* Last error message of the calling thread (never NULL). */
const char* pbx_last_error(void);
int pbx_abi_version(void);
int pbx_device_count(void);

/* A plane (z,c,t,resolution) of an image.  Registering a resolution-0 plane creates or
 * checks the image record (the `Pixels` row getPixels returns, TileRequestHandler.java:220-241):
 * size_x/size_y/pixel_type are the image's. */
typedef struct pbx_plane_desc {
    int64_t image_id;
    int32_t z, c, t;
    int32_t resolution;      /* STORED pyramid level: 0 = full resolution, k = k-th downsampled
                                level (the NGFF multiscales dataset index).  Requests use
                                OMERO's numbering instead: see pbx_tile_req.resolution. */
    int32_t pixel_type;      /* enum pbx_pixel_type */
    int32_t size_x, size_y;
    int32_t byte_order;      /* enum pbx_byte_order of host_data (ignored for generators) */
    int32_t source;          /* enum pbx_source */
    const void* host_data;   /* PBX_SRC_HOST: size_y rows of size_x samples, row-major */
    uint64_t host_bytes;
    uint64_t seed;           /* generators */
    int32_t plane_no;        /* generators: FakeReader plane number / noise plane index */
    int32_t reserved;
} pbx_plane_desc;

int pbx_plane_register(pbx_ctx* ctx, const pbx_plane_desc* desc, uint64_t* plane_id);
/* Frees the plane.  Batches planned before the call keep reading it: the HBM is returned
 * when the last of them is destroyed (pbx_batch_destroy), never under a running kernel. */
int pbx_plane_release(pbx_ctx* ctx, uint64_t plane_id);

/* ---- Plane residency: planes opened on demand, in row bands, under an HBM budget ----
 *
 * The reference opens an image's PixelBuffer per request (getPixels :220-241, then
 * getPixelBuffer :201-211 and getTileDirect :107-109).  Here the bytes of a plane are loaded
 * into HBM once and then serve every tile of it; a request for a plane this context does not
 * hold answers PBX_E_NOT_RESIDENT and the binding loads it.
 *
 * pbx_image_declare records the Pixels row getPixels returns (:84; pixelsType, sizeX/Y/Z/C/T)
 * and the PixelBuffer's getResolutionLevels().  With it a request for a z/c/t outside the
 * image, or a resolution outside its levels, is the reference's 404 without loading anything;
 * without it (planes registered directly) the image is described by its registered planes. */
typedef struct pbx_image_desc {
    int64_t image_id;
    int32_t pixel_type;          /* enum pbx_pixel_type (Pixels.pixelsType) */
    int32_t size_x, size_y;      /* full resolution (Pixels.sizeX / sizeY) */
    int32_t size_z, size_c, size_t_;
    int32_t levels;              /* PixelBuffer.getResolutionLevels(); >= 1 */
    int32_t reserved;
} pbx_image_desc;
/* Idempotent; 400 if it contradicts an earlier declaration or a registered plane. */
int pbx_image_declare(pbx_ctx* ctx, const pbx_image_desc* desc);
/* Releases every plane of the image and forgets its record (requests then answer
 * NOT_RESIDENT).  404 if the image is unknown. */
int pbx_image_release(pbx_ctx* ctx, int64_t image_id);

/* Allocates a plane — or only its rows [band_y0, band_y0 + band_rows) when band_rows > 0 (a
 * rank's tile-row band of a whole slide) — under the key desc->(image_id, z,
 * c, t, resolution).  desc->size_x / size_y are the plane's (the level's) full size; requests
 * for rows outside the band answer PBX_E_NOT_RESIDENT (another context owns them).
 * desc->source: PBX_SRC_HOST -> the plane is empty and not served until pbx_plane_commit;
 * its rows arrive by pbx_plane_write_rows in desc->byte_order.  Generators -> the band is
 * generated on the GPU and the plane is ready at once.  409 if the key is loaded or being
 * loaded; 507 if it does not fit the residency budget (pbx_set_residency_budget). */
int pbx_plane_create(pbx_ctx* ctx, const pbx_plane_desc* desc, int32_t band_y0, int32_t band_rows,
                     uint64_t* plane_id);
/* Rows [y0, y0 + rows) of a created plane (inside its band): `rows` rows of size_x samples,
 * packed (size_x * bpp bytes each), as PixelBuffer.getTileDirect(z, c, t, 0, y0, sizeX, rows)
 * returns them.  Copied through pooled pinned staging to HBM; the caller's buffer is free
 * again when the call returns.  Any number of calls, in any order, of any band size. */
int pbx_plane_write_rows(pbx_ctx* ctx, uint64_t plane_id, int32_t y0, int32_t rows, const void* data,
                         uint64_t bytes);
/* Publishes a created plane: from now on its tiles are served.  400 if a row of the band was
 * never written. */
int pbx_plane_commit(pbx_ctx* ctx, uint64_t plane_id);
/* The plane registered under a key (STORED level): its id and state (0 loading, 1 ready,
 * 2 evicted) and resident band; 404 if the key is not registered.  Lets a binding that got
 * NOT_RESIDENT tell "load it" from "another caller is loading it". */
int pbx_plane_lookup(pbx_ctx* ctx, int64_t image_id, int32_t z, int32_t c, int32_t t, int32_t level,
                     uint64_t* plane_id, int32_t* state, int32_t* band_y0, int32_t* band_rows);

/* Sparse planes: region-proportional residency.  The reference reads only the requested region
 * per request (new byte[w*h*bpp] then getTileDirect(z, c, t, x, y, w, h), TileRequestHandler.java:
 * 102-109); a whole-slide plane is far larger than one request.  A sparse plane is registered
 * under its key at once (READY) but holds its rows as bands of `band_rows` rows (band k = rows
 * [k*band_rows, (k+1)*band_rows)), each loaded on demand, pinned by the batches that read it and
 * evicted on its own, least recently used first, under the residency budget.  A request whose
 * rows cover a band that is not resident answers PBX_E_NOT_RESIDENT; the binding loads the
 * covering bands (rows y .. y+h-1, by pbx_band_write) and retries.  A region straddling bands is
 * served bit-exact (its rows are gathered into a per-batch bridge buffer on the GPU).
 * own_y0 / own_rows (0/0 = the whole plane): the rows this context may hold; own_y0 a multiple of
 * band_rows; rows outside answer PBX_E_NOT_RESIDENT (another context owns them).  Generator
 * sources generate each band on the GPU when it is written with data == NULL. */
int pbx_plane_create_sparse(pbx_ctx* ctx, const pbx_plane_desc* desc, int32_t band_rows, int32_t own_y0,
                            int32_t own_rows, uint64_t* plane_id);
/* Rows [y0, y0 + rows) of ONE band (packed, desc->byte_order), as getTileDirect(z, c, t, 0, y0,
 * sizeX, rows) returns them; the first write of an absent band allocates it (507 if it cannot be
 * made to fit), the write that completes it makes it resident.  409 if the band is resident (or
 * another caller is allocating it).  data == NULL: generate the rows (generator planes).  A
 * failed write fails the band's whole load (every writer of it: load it again). */
int pbx_band_write(pbx_ctx* ctx, uint64_t plane_id, int32_t y0, int32_t rows, const void* data,
                   uint64_t bytes);
/* A loader that gives up on the band holding row y0 part-way (a failed piece, a Java exception
 * between pieces): the band goes back to absent and its HBM is returned (at once, or by the last
 * write still in flight); a resident or absent band is left as it is.  A write that fails does
 * the same by itself, and a band left loading with no write for 10 s is started over by the
 * next writer (or evicted).  400 for a plane that is not sparse. */
int pbx_band_abort(pbx_ctx* ctx, uint64_t plane_id, int32_t y0);
/* band_rows and the number of bands of a sparse plane; states (may be NULL, nbands entries):
 * 0 absent (never loaded, or evicted), 1 loading, 2 resident.  A band whose load failed, or that
 * has been loading without a write for 10 s (a loader that went away), reads as 0 and its HBM is
 * returned.  400 for a plane that is not sparse. */
int pbx_plane_band_info(pbx_ctx* ctx, uint64_t plane_id, int32_t* band_rows, int32_t* nbands, uint8_t* states);

/* HBM residency budget for planes (bytes; 0 = none, the default, or $PBX_HBM_BUDGET_MB).  A
 * registration that would exceed it first evicts idle planes, least recently used first (a
 * plane is idle when no planned batch reads it).  With or without a budget, a plane
 * allocation that fails for lack of device memory evicts idle planes and retries.  An evicted
 * plane's requests answer PBX_E_NOT_RESIDENT until it is registered again. */
int pbx_set_residency_budget(pbx_ctx* ctx, uint64_t bytes);
typedef struct pbx_residency_stats {
    uint64_t budget;             /* 0 = none */
    uint64_t resident_bytes;     /* HBM held by planes and bands (incl. released ones still read) */
    uint64_t planes;             /* registered (non-sparse) planes resident in HBM */
    uint64_t evicted_planes;     /* registered keys whose plane was evicted */
    uint64_t evictions, evicted_bytes;  /* totals since pbx_init (planes and bands) */
    uint64_t bands;              /* resident bands of sparse planes */
    uint64_t band_evictions;     /* bands evicted since pbx_init */
} pbx_residency_stats;
int pbx_residency_stats_get(pbx_ctx* ctx, pbx_residency_stats* out);
/* Resolution pyramid on the GPU (the lower levels
 * PixelBuffer.setResolutionLevel selects, TileRequestHandler.java:89-91): registers `levels`
 * planes of the same (image, z, c, t) at resolutions r+1 .. r+levels (r = the plane's), each
 * the 2x2 box mean of the one above (sizes rounded up; the last column / row repeated for odd
 * sizes; integers (sum + 2) >> 2 on the exact sum, arithmetic for signed types; float/double
 * ((a + b) + (c + d)) * 0.25), in the plane's byte order.  ids[k] = the plane id of level
 * r+1+k (ids may be NULL).  Tiles of a level are served with pbx_tile_req.resolution.
 * kernel_ms (may be NULL): device time of the downsampling kernels (HIP events). */
int pbx_plane_build_pyramid(pbx_ctx* ctx, uint64_t plane_id, int32_t levels, uint64_t* ids,
                            double* kernel_ms);
/* NGFF / Zarr v2 planes: the reference's pixels service is ZarrPixelsService
 * (PixelBufferVerticle.java:29,56; beanRefContext.xml:51; config.yaml:18), which reads Zarr
 * chunks through omero-zarr-pixel-buffer 0.6.1 / JZarr (build.gradle:57) on every
 * getTileDirect.  Here the chunks of one (z, c, t, resolution) plane are uploaded once and
 * decoded on the GPU (one wave per compressed stream) straight into a resident HBM plane,
 * which then serves tiles like any registered plane.  Codec = the .zarray "compressor":
 * null, blosc (c-blosc 1.x frames: blosclz / lz4 / lz4hc / zlib / zstd, byte shuffle, bit
 * shuffle or none, split or not), zlib.  snappy and blosc2 frames -> 400. */
enum pbx_zarr_codec { PBX_ZARR_RAW = 0, PBX_ZARR_BLOSC = 1, PBX_ZARR_ZLIB = 2 };

typedef struct pbx_zarr_chunks {
    int32_t chunk_x, chunk_y;   /* .zarray "chunks" (the x and y extents; edge chunks are full) */
    int32_t codec;              /* enum pbx_zarr_codec */
    int32_t reserved;
    const uint8_t* data;        /* the chunk files concatenated, C order over the chunk grid */
    const uint64_t* offsets;    /* gx*gy + 1 entries (gx = ceil(size_x/chunk_x), ...); chunk
                                   i = cy*gx + cx is data[offsets[i] .. offsets[i+1]); an empty
                                   range is a missing chunk (every sample = fill) */
    uint64_t fill_bits;         /* .zarray fill_value as the sample's bit pattern */
} pbx_zarr_chunks;

/* desc: image/z/c/t/resolution/pixel_type/size as pbx_plane_register; byte_order = the
 * .zarray dtype's ('<' little, '>' / '|' big); source/host_data are ignored.
 * kernel_ms (may be NULL): [0] device ms of the decode kernels, [1] of the placement kernel.
 * A malformed or unsupported chunk fails the whole plane with 400 (nothing registered). */
int pbx_plane_register_zarr(pbx_ctx* ctx, const pbx_plane_desc* desc, const pbx_zarr_chunks* chunks,
                            uint64_t* plane_id, double* kernel_ms);
/* n planes (e.g. every (z, c, t) plane of an NGFF resolution level) decoded by ONE set of
 * launches: descs[k] / chunks[k] as above, plane_ids[k] receives plane k's id.  More planes
 * per call = more compressed streams in flight (one wave each), which is what hides the
 * serial decode latency.  All planes are registered, or none (400/500). */
int pbx_planes_register_zarr(pbx_ctx* ctx, uint64_t n, const pbx_plane_desc* descs,
                             const pbx_zarr_chunks* chunks, uint64_t* plane_ids, double* kernel_ms);
/* Copy a registered plane back to the host, samples in big-endian order (test hook). */
int pbx_plane_read_be(pbx_ctx* ctx, uint64_t plane_id, void* out, uint64_t bytes);

/* TileCtx.resolution == null (TileCtx.java:86-88): the pixel buffer's default level. */
#define PBX_RESOLUTION_NONE (-1)

/* TileCtx (TileCtx.java:36-54, parsed at :67-90). */
typedef struct pbx_tile_req {
    int64_t image_id;
    int32_t z, c, t;
    int32_t resolution;      /* OMERO PixelBuffer.setResolutionLevel numbering
                                (TileRequestHandler.java:89-91): with L stored levels,
                                L-1 = full resolution, 0 = the smallest level; stored level
                                = L-1-resolution.  PBX_RESOLUTION_NONE = not given (full
                                resolution).  Outside [0, L), or any other negative value:
                                setResolutionLevel throws -> getTile null -> 404.  A binding
                                maps a given negative Integer to a value < -1. */
    int32_t x, y, w, h;      /* w/h == 0 -> plane size (TileRequestHandler.java:92-97) */
    int32_t format;          /* enum pbx_format */
    int32_t reserved;
} pbx_tile_req;

/* One response: status plus the exact-length body (TileRequestHandler.java:188-193). */
typedef struct pbx_result {
    int32_t status;          /* enum pbx_status */
    int32_t format;
    int32_t w, h;            /* region after the w/h defaulting (used by the filename header) */
    const uint8_t* data;     /* library-owned; valid until pbx_results_release */
    uint64_t len;
    void* owner;             /* internal */
} pbx_result;

/* Synchronous single tile: TileRequestHandler.getTile (TileRequestHandler.java:80-139).
 * Called from many threads at once (the Vert.x worker pool, PixelBufferVerticle.java:109-110),
 * requests are coalesced: all requests that arrive while the GPU is busy become one batch. */
int pbx_get_tile(pbx_ctx* ctx, const pbx_tile_req* req, pbx_result* out);
/* Synchronous batch: n independent getTile calls executed as one set of GPU launches. */
int pbx_get_tiles(pbx_ctx* ctx, const pbx_tile_req* reqs, uint64_t n, pbx_result* out);
/* Results go back to the context that produced them (ctx may be NULL). */
void pbx_results_release(pbx_ctx* ctx, pbx_result* results, uint64_t n);

/* Stage timings under the reference's tracing span names (TileRequestHandler.java:81
 * "get_tile", :104 "get_tile_direct", :147 "create_metadata", :180 "write_image").  A request is
 * served inside a batch, so the stages are the batch's (HIP events on its kernel stream; the
 * caller times its own get_tile span around pbx_get_tile):
 *   get_tile_direct_ms  the region gather from HBM (raw/TIFF extract kernel); 0 for a PNG-only
 *                       batch, whose gather is fused into the filter/deflate kernels
 *   write_image_ms      PNG row filters + deflate (LZ77, Huffman, encode) of the whole batch
 *   create_metadata_ms  container framing: IHDR/IDAT/IEND or the TIFF IFD, chunk CRCs
 *   batch_ms            the batch's device time, first to last kernel
 *   d2h_ms              host wall time from queuing the batch's device->host copy to its end
 *   batch_tiles         requests in the batch
 * Returns PBX_E_BADARG for a result without a body (error statuses, released results). */
typedef struct pbx_spans {
    double get_tile_direct_ms, write_image_ms, create_metadata_ms, batch_ms, d2h_ms;
    uint64_t batch_tiles;
} pbx_spans;
int pbx_result_spans(const pbx_result* r, pbx_spans* out);

/* Batched async: pbx_submit plans and launches n independent getTile
 * requests and returns at once; pbx_wait blocks until the batch has finished (timeout_us < 0:
 * no limit; 0: poll), fills out[0..n) (the array given to pbx_submit) exactly like
 * pbx_get_tiles and frees the ticket.  On PBX_E_PENDING the ticket stays valid: call again.
 * Batches run in submission order on the context's stream; results are released with
 * pbx_results_release. */
typedef struct pbx_ticket pbx_ticket;
int pbx_submit(pbx_ctx* ctx, const pbx_tile_req* reqs, uint64_t n, pbx_result* out,
               pbx_ticket** ticket);
int pbx_wait(pbx_ctx* ctx, pbx_ticket* ticket, int64_t timeout_us);

/* Device-resident batches: plan once, launch asynchronously on the context's stream,
 * outputs stay in HBM until pbx_batch_fetch.  Used by callers that pipeline requests
 * (and by bench.py, whose timed region is plan+launch+sync of one batch). */
typedef struct pbx_batch pbx_batch;
int pbx_batch_plan(pbx_ctx* ctx, const pbx_tile_req* reqs, uint64_t n, pbx_batch** out);
int pbx_batch_launch(pbx_ctx* ctx, pbx_batch* b);
int pbx_batch_sync(pbx_ctx* ctx, pbx_batch* b);
int pbx_batch_fetch(pbx_ctx* ctx, pbx_batch* b, pbx_result* out);
void pbx_batch_destroy(pbx_ctx* ctx, pbx_batch* b);

typedef struct pbx_batch_stats {
    uint64_t tiles, ok_tiles, png_tiles, raw_tiles, tif_tiles;
    uint64_t in_bytes;       /* w*h*bpp summed over OK tiles */
    uint64_t stream_bytes;   /* bytes fed to deflate (PNG filtered streams, deflate-TIFF) */
    uint64_t out_bytes;      /* total response bytes */
    uint64_t deflate_out_bytes; /* compressed payload bytes (zlib streams) */
    uint64_t segments;
    /* HIP events of the last launch: extract (raw/TIFF), filter (PNG rows), deflate (LZ77 ..
     * encode, all segments), assemble (container framing), total; then the deflate parts */
    double ms_extract, ms_filter, ms_deflate, ms_assemble, ms_total;
    double ms_lz77, ms_huff, ms_encode;
    uint64_t blocks;         /* deflate blocks (segments sharing one Huffman code) */
    /* adaptive-filter PNG tiles in the None mode read by k_lz77 straight from the plane (no
     * filter pass), and their bytes as in_bytes + stream_bytes count them */
    uint64_t direct_tiles, direct_bytes;
} pbx_batch_stats;
int pbx_batch_stats_get(pbx_ctx* ctx, pbx_batch* b, pbx_batch_stats* out);

/* Reply metadata. */
/* "image%d_z%d_c%d_t%d_x%d_y%d_w%d_h%d.%s" (PixelBufferVerticle.java:118-126), ext "bin" when
 * format is raw.  format_str is the caller's original TileCtx.format (may be NULL). */
int pbx_tile_filename(const pbx_tile_req* req, int32_t w, int32_t h, const char* format_str,
                      char* out, uint64_t cap);
/* PixelBufferMicroserviceVerticle.java:373-379. */
const char* pbx_content_type(const char* format_str);
/* TileCtx.format string -> enum pbx_format (null -> RAW). */
int pbx_format_from_string(const char* format_str);
int pbx_pixel_type_from_string(const char* name);
int pbx_bytes_per_pixel(int32_t pixel_type);

/* Batches launched and requests served so far by this context (coalescing check). */
int pbx_ctx_stats_get(pbx_ctx* ctx, uint64_t* batches, uint64_t* requests);

/* Free the context's cached (currently unused) device and pinned batch buffers; buffers
 * of batches still alive stay (torch.cuda.empty_cache analogue). */
int pbx_release_cached(pbx_ctx* ctx);

/* Synchronise the context's device (bench/test hook). */
int pbx_device_synchronize(pbx_ctx* ctx);

/* Pipelined batches (pbx_batch_launch, pbx_submit) with deflate work alternate over
 * `streams` kernel streams (1..4; default 3, or $PBX_KSTREAMS), each starting behind the
 * previous batch's stage `stagger` (1 = after its k_lz77 (default), 2 k_huff, 3 the
 * offsets scan, 4 k_encode; 0 = no wait), so one batch's latency-bound phases overlap
 * the next batch's kernels.  streams = 1: every batch in launch order on one stream
 * (per-kernel timings then have no overlap).  Synchronous calls (pbx_get_tile(s)) and
 * batches without deflate work always use the one stream.  No reference counterpart
 * (the reference runs one request per worker thread). */
int pbx_set_kernel_streams(pbx_ctx* ctx, int32_t streams, int32_t stagger);

/* sizeof of the ABI structs, for bindings to check their layouts: pbx_config,
 * pbx_plane_desc, pbx_tile_req, pbx_result, pbx_batch_stats, pbx_image_desc,
 * pbx_residency_stats, pbx_spans (in that order).  Returns the number of structs (8). */
int pbx_abi_sizes(uint64_t* sizes, int n);

/* ---- A node: N device contexts in ONE process ----
 * The reference deploys its worker verticles in one JVM (PixelBufferMicroserviceVerticle.java:
 * 117-118,224-233: worker_pool_size threads calling TileRequestHandler.getTile).  A node-wide
 * drop-in therefore holds one context per GPU in that process and routes each request to the
 * context that holds its plane, or its row band (a whole slide split into tile-row bands over
 * the GPUs); where several hold it (planes replicated on every GPU) the
 * pbx_shard_of owner among them serves it.  devices: n HIP ordinals (NULL = 0 .. n-1; one
 * device may appear several times); shard_tile: the tile cell of the shard hash (0 = 512). */
typedef struct pbx_node pbx_node;
int pbx_node_init(const pbx_config* cfg, int32_t n, const int32_t* devices, int32_t shard_tile,
                  pbx_node** out);
void pbx_node_shutdown(pbx_node* node);
int32_t pbx_node_size(pbx_node* node);
/* Context k of the node (register planes / bands there; NULL if out of range). */
pbx_ctx* pbx_node_context(pbx_node* node, int32_t k);
/* The context that serves `req`: *index = a context that holds the plane (the status it would
 * answer is returned: PBX_OK, or the reference's 404 ...), else PBX_E_NOT_RESIDENT with *index =
 * the context the binding should load into: the one whose sparse plane owns the rows (bands not
 * loaded yet), else the pbx_shard_of owner. */
int pbx_node_route(pbx_node* node, const pbx_tile_req* req, int32_t* index);
/* pbx_get_tile on the routed context (served_by may be NULL); results are released with
 * pbx_results_release (any context of the node, or NULL). */
int pbx_node_get_tile(pbx_node* node, const pbx_tile_req* req, pbx_result* out, int32_t* served_by);

/* Fault injection (test hook): the `ahead`-th batch launched by this context from
 * now on (1 = the next) completes with a device failure: each of its requests answers 500
 * (PBX_E_INTERNAL, PixelBufferVerticle.java:141-146) unless it already had its own 4xx; the
 * context keeps serving.  0 disables.  $PBX_FAIL_BATCH=k does the same for the k-th launch
 * since pbx_init. */
int pbx_test_fail_batch(pbx_ctx* ctx, uint64_t ahead);
/* Stall injection (test hook): the `ahead`-th batch launched by this context from now on (1 =
 * the next) never completes until pbx_test_stall_batch(ctx, 0) releases it (a one-wave kernel
 * ahead of its kernels spins on a host flag; it also ends by itself after 30 s).  Later batches
 * queue behind it on the device, as behind a wedged one.  Callers of pbx_get_tile get 500 at
 * their deadline (pbx_config.request_timeout_us).  0 releases the stall and disarms. */
int pbx_test_stall_batch(pbx_ctx* ctx, uint64_t ahead);
/* Upload failure injection (test hook): the `ahead`-th pbx_band_write from now on fails after
 * joining its band's load, as a failed host-to-device copy would.  0 disables. */
int pbx_test_fail_band_write(pbx_ctx* ctx, uint64_t ahead);

/* Request sharding across GPUs (one process per GPU, no collectives): the rank that
 * owns a request, by hash of (image, z, c, t, tile column, tile row) for tile_w x tile_h
 * tiles.  Identical in every process. */
int pbx_shard_of(const pbx_tile_req* req, int32_t tile_w, int32_t tile_h, int32_t world);

/* Test hook: the Huffman stage of the deflate pipeline (k_huff) alone, on given symbol
 * histograms.  hist: nseg x 320 counts (288 literal/length, 32 distance); sl_last: nseg x 2
 * (segment bytes, final-segment flag).  Out: codes nseg x 480 (288 literal/length and 32
 * distance codes as bit-reversed code | length << 16, then 160 words of block header bits)
 * and info nseg x 4 (block type, header bits, data bits, output bytes).  Used by tests/ to
 * compare the GPU stage with the CPU emulator on adversarial histograms. */
int pbx_test_huffman(pbx_ctx* ctx, const uint32_t* hist, const uint32_t* sl_last, uint32_t nseg,
                     uint32_t* codes, uint32_t* info);

/* Test hook: the LZ77 stage's per-segment outputs of a launched batch (k_lz77: 320
 * histogram words and the match records per segment, segments in batch order), compared by
 * tests/ with the CPU emulator.  nseg must equal the batch's segment count. */
int pbx_test_batch_lz77(pbx_ctx* ctx, pbx_batch* b, uint32_t* hist, uint32_t* mrec, uint64_t nseg);

#ifdef __cplusplus
}
#endif
#endif /* PBX_H */
