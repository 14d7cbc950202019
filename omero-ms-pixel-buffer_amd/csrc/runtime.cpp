// runtime.cpp — host runtime behind include/pbx.h: device context, plane registry (the
// PixelsService / getPixels stand-in), request validation that mirrors
// TileRequestHandler.getTile, batch planning, kernel launches and result ownership.
//
// Paths below are relative to /root/reference/src/main/java/com/glencoesoftware/omero/ms/pixelbuffer/.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <functional>
#include <tuple>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "../../include/pbx.h"
#include "pbx_common.h"
#include "pbx_config.h"
#include "pbx_kernels.h"

using namespace pbx;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(PBX_E_INTERNAL, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                        __FILE__, __LINE__);                                            \
    } while (0)

const int kBpp[PBX_NPIXEL_TYPES] = {1, 1, 2, 2, 4, 4, 4, 8};

int bpp_of(int32_t pt) { return (pt >= 0 && pt < PBX_NPIXEL_TYPES) ? kBpp[pt] : 0; }
int log2i(int v) { int l = 0; while ((1 << l) < v) l++; return l; }

// A registered plane (the bytes getPixelBuffer + getTileDirect read, TileRequestHandler.java:
// 86,107-109) or the row band of one that this context owns.  Records live in
// pbx_ctx::planes and are heap-allocated so that batches can pin them.
enum PlaneState : int {
    PS_FILLING = 0,  // created (pbx_plane_create), rows arriving, not served yet
    PS_READY = 1,    // served
    PS_EVICTED = 2   // key still registered, HBM returned (NOT_RESIDENT until re-registered)
};

// One row band of a sparse plane (pbx_plane_create_sparse): rows [k*B, (k+1)*B) of the plane
// (clipped to the plane and to the context's owned rows), loaded on demand, pinned by the
// batches that read it and evicted on its own (region-proportional residency: a request
// loads only the bands its rows cover, as getTileDirect reads only the requested region,
// TileRequestHandler.java:102-109).
enum BandState : int { BS_ABSENT = 0, BS_LOADING = 1, BS_READY = 2 };

// A plane or band that has just been loaded is not evicted until a batch has read it, or
// FRESH_NS has passed (a loader that went away): otherwise, under a budget smaller than the
// working set, concurrent loaders evict each other's planes between the load and the retry
// that was to read them, and every request is loaded again and again.  A
// loader that finds only fresh or pinned memory gets PBX_E_NO_SPACE and retries later.
constexpr int64_t FRESH_NS = 2000000000;
// A band left BS_LOADING with no writer for this long (a loader that failed part-way or went
// away) is reclaimed: the next writer starts it over, and eviction may return its HBM
// (pbx_ctx::stale_ns; $PBX_BAND_STALE_MS for tests).
constexpr int64_t STALE_NS = 10000000000;
inline int64_t mono_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

struct Band {
    uint8_t* dev = nullptr;      // the band's rows at the plane's pitch + 256 B slack
    size_t bytes = 0;
    int state = BS_ABSENT;
    int64_t pins = 0;            // planned batches that read it
    uint64_t last_use = 0;
    int64_t fresh_until = 0;     // loaded, not served yet: not evicted before this (fresh_now)
    uint32_t rows_left = 0;      // BS_LOADING: rows not written yet
    int32_t writers = 0;         // pbx_band_write calls in flight
    bool failed = false;         // BS_LOADING: a write failed; the last writer out resets the band
    int64_t touched = 0;         // BS_LOADING: mono_ns of the last write activity
    // the last load went idle past stale_ns and was reset: the next load must start at the
    // band's first row, so a late piece of the reset load fails instead of starting a load
    // that could never complete
    bool stale_reset = false;
    std::vector<uint8_t> rows_done;
};

struct Plane {
    uint64_t id = 0;
    int64_t image_id = 0;
    int32_t z = 0, c = 0, t = 0, res = 0, pixel_type = 0, size_x = 0, size_y = 0;
    bool little_endian = false;
    uint8_t* dev = nullptr;      // allocation: rows [band_y0, band_y0 + band_rows) + 256 B slack
    int64_t pitch = 0;
    size_t bytes = 0;
    int32_t band_y0 = 0, band_rows = 0;  // resident rows (band_rows == size_y: the whole plane)
    // sparse planes: held as bands of sparse_rows rows (bands[k]), `dev` unused; band_y0 /
    // band_rows are then the rows this context owns: requests whose first row lies there are
    // served here (another context owns the rest), incl. the bands past the owned rows that a
    // region straddling their end covers (guest bands, loaded on demand like the owned ones)
    int32_t sparse_rows = 0;
    std::vector<Band> bands;
    int32_t gen_source = 0;      // sparse generator planes: bands are generated on demand
    uint64_t gen_seed = 0;
    int32_t gen_plane_no = 0;
    // registry state, under reg_mu
    int state = PS_FILLING;
    bool indexed = false;        // reachable from ctx->index (false once released)
    int64_t pins = 0;            // planned batches / running kernels that read the plane
    uint64_t last_use = 0;       // LRU tick of the last request served from it
    int64_t fresh_until = 0;     // loaded, not served yet: not evicted before this (fresh_now)
    std::vector<uint8_t> rows_done;  // PS_FILLING host planes: which band rows were written
    uint64_t rows_left = 0;
    int32_t writers = 0;         // pbx_plane_write_rows calls in flight (commit waits for none)
    // the kernels address rows by their index in the whole plane
    uint8_t* base() const { return dev - (int64_t)band_y0 * pitch; }
    bool whole() const { return !sparse_rows && band_y0 == 0 && band_rows == size_y; }
    // sparse: rows of band k, [y0, y1) (the owned rows start at a band start)
    int32_t band_lo(int32_t k) const { return k * sparse_rows; }
    int32_t band_hi(int32_t k) const { return (int32_t)std::min<int64_t>((int64_t)(k + 1) * sparse_rows, size_y); }
    uint8_t* band_base(int32_t k) const { return bands[(size_t)k].dev - (int64_t)band_lo(k) * pitch; }
    // every HBM block the record holds
    void memory(std::vector<std::pair<void*, size_t>>& out) const {
        if (dev) out.emplace_back(dev, bytes);
        for (const Band& b : bands)
            if (b.dev) out.emplace_back(b.dev, b.bytes);
    }
};

struct Image {
    int32_t pixel_type = 0, size_x = 0, size_y = 0;
    int32_t planes = 0;                       // registry keys (any state)
    std::map<int32_t, int32_t> level_planes;  // stored pyramid level -> registry keys
    // pbx_image_declare: the Pixels row and PixelBuffer.getResolutionLevels()
    bool declared = false;
    int32_t size_z = 0, size_c = 0, size_t_ = 0, nlevels = 0;
    // PixelBuffer.getResolutionLevels(): declared, else the number of stored levels (0 .. max)
    int32_t levels() const {
        if (declared) return nlevels;
        return level_planes.empty() ? 0 : level_planes.rbegin()->first + 1;
    }
};

// Grow-only caching allocator for device and pinned host blocks (power-of-two classes).
struct Pool {
    bool pinned = false;  // pinned host blocks: power-of-two classes from 4 MiB (few, reused)
    std::mutex mu;
    std::multimap<size_t, void*> free_blocks;
    std::unordered_map<void*, size_t> sizes;

    // size classes: 1 MiB, then 2^k x {1, 1.25, 1.5, 1.75} (at most 25% slack per block)
    size_t cls(size_t n) const {
        size_t c = pinned ? (4u << 20) : (1u << 20);
        if (n <= c) return c;
        if (pinned) {
            while (c < n) c <<= 1;
            return c;
        }
        while (c < n) c <<= 1;
        const size_t q = c >> 3;  // c/8: the steps between c/2 and c
        for (size_t k = 5; k <= 8; k++)
            if (k * q >= n) return k * q;
        return c;
    }
    void* get(size_t n, hipError_t* err) {
        const size_t c = cls(n);
        {
            std::lock_guard<std::mutex> g(mu);
            auto it = free_blocks.find(c);
            if (it != free_blocks.end()) {
                void* p = it->second;
                free_blocks.erase(it);
                return p;
            }
        }
        void* p = nullptr;
        *err = pinned ? hipHostMalloc(&p, c, hipHostMallocDefault) : hipMalloc(&p, c);
        if (*err != hipSuccess) {
            // drop cached blocks and retry once
            trim();
            *err = pinned ? hipHostMalloc(&p, c, hipHostMallocDefault) : hipMalloc(&p, c);
            if (*err != hipSuccess) return nullptr;
        }
        std::lock_guard<std::mutex> g(mu);
        sizes[p] = c;
        return p;
    }
    void put(void* p) {
        if (!p) return;
        std::lock_guard<std::mutex> g(mu);
        free_blocks.emplace(sizes[p], p);
    }
    void trim() {
        std::lock_guard<std::mutex> g(mu);
        for (auto& kv : free_blocks) {
            if (pinned) (void)hipHostFree(kv.second); else (void)hipFree(kv.second);
            sizes.erase(kv.second);
        }
        free_blocks.clear();
    }
    void release_all() {
        std::lock_guard<std::mutex> g(mu);
        for (auto& kv : sizes) {
            if (pinned) (void)hipHostFree(kv.first); else (void)hipFree(kv.first);
        }
        sizes.clear();
        free_blocks.clear();
    }
};

// Reused HIP events (a batch takes up to ten; creating and destroying them per batch cost
// the single-request path host time on every request).
struct EventPool {
    unsigned flags = hipEventDefault;
    std::mutex mu;
    std::vector<hipEvent_t> free_ev;
    hipError_t get(hipEvent_t* e) {
        {
            std::lock_guard<std::mutex> g(mu);
            if (!free_ev.empty()) {
                *e = free_ev.back();
                free_ev.pop_back();
                return hipSuccess;
            }
        }
        return hipEventCreateWithFlags(e, flags);
    }
    void put(hipEvent_t e) {
        if (!e) return;
        std::lock_guard<std::mutex> g(mu);
        free_ev.push_back(e);
    }
    void release_all() {
        std::lock_guard<std::mutex> g(mu);
        for (hipEvent_t e : free_ev) (void)hipEventDestroy(e);
        free_ev.clear();
    }
};

// Waits for an event: small batches (the single-request latency path) poll it for up to
// `spin_us` first -- a blocking wait wakes the thread tens of microseconds after the GPU is
// done -- then block.
// A spinning thread's pause between polls (spin loops without one take cores
// from the JVM's workers and storm the HIP runtime with queries).
inline void cpu_relax() {
    for (int k = 0; k < 8; k++) __builtin_ia32_pause();
}

hipError_t wait_event(hipEvent_t e, int64_t spin_us) {
    if (spin_us > 0) {
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin_us);
        for (;;) {
            const hipError_t q = hipEventQuery(e);
            if (q != hipErrorNotReady) return q;
            if (std::chrono::steady_clock::now() >= until) break;
            cpu_relax();
        }
    }
    return hipEventSynchronize(e);
}

}  // namespace

struct Coalescer;

// Returns plane HBM with hipFree on a thread of its own: hipFree waits for the whole device,
// so it must never run on a completer (pbx_batch_destroy of a batch holding the last pin of
// a released plane) or on the launch path, where it would stall every in-flight batch.
struct Reaper {
    std::mutex mu;
    std::condition_variable cv, cv_idle;
    std::deque<void*> q;
    int busy = 0;
    bool stop = false;
    std::thread th;
    int device = 0;
    // Housekeeping between frees: while `ticking`, tick() runs every few ms (outside mu) until
    // it reports nothing left -- the uncoalesced pbx_get_tile calls parked at their deadline
    // are collected here, so their pins and pool blocks go back even if the context goes idle
    // (ADVICE r05).  poke() starts it; pokes counts them so that a poke during a tick that
    // found nothing is not lost.
    std::function<bool()> tick;
    bool ticking = false, in_tick = false;
    uint64_t pokes = 0;

    void start(int dev) {
        device = dev;
        th = std::thread([this] { loop(); });
    }
    void loop() {
        (void)hipSetDevice(device);
        std::unique_lock<std::mutex> g(mu);
        for (;;) {
            auto ready = [&] { return stop || !q.empty(); };
            if (ticking) cv.wait_for(g, std::chrono::milliseconds(2), ready);
            else cv.wait(g, [&] { return ready() || ticking; });
            if (stop && q.empty()) break;  // stopping, nothing left
            if (!q.empty()) {
                std::vector<void*> take(q.begin(), q.end());
                q.clear();
                busy++;
                g.unlock();
                for (void* p : take) (void)hipFree(p);
                g.lock();
                busy--;
            }
            if (ticking && tick) {
                const uint64_t seen = pokes;
                in_tick = true;
                g.unlock();
                const bool more = tick();
                g.lock();
                in_tick = false;
                if (!more && pokes == seen) ticking = false;
            }
            cv_idle.notify_all();
        }
    }
    void put(void* p) {
        if (!p) return;
        {
            std::lock_guard<std::mutex> g(mu);
            q.push_back(p);
        }
        cv.notify_one();
    }
    void poke() {
        {
            std::lock_guard<std::mutex> g(mu);
            ticking = true;
            pokes++;
        }
        cv.notify_one();
    }
    // No further ticks (shutdown): waits for one in progress.
    void stop_ticking() {
        std::unique_lock<std::mutex> g(mu);
        tick = nullptr;
        ticking = false;
        cv_idle.wait(g, [&] { return !in_tick; });
    }
    // Waits until every handed-over block is back with the device (an allocation that ran out
    // of memory retries only after that).
    void drain() {
        std::unique_lock<std::mutex> g(mu);
        cv_idle.wait(g, [&] { return q.empty() && busy == 0; });
    }
    void finish() {
        if (!th.joinable()) return;
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        th.join();
    }
};

struct pbx_ctx {
    int device = 0;
    int cus = 256;                      // compute units (persistent kernel grids)
    pbx_config cfg{};
    hipStream_t stream = nullptr;       // kernels (planes, Zarr; batches on kstream[])
    // Batch kernel streams: batch k runs on kstream[k % nks], so one batch's latency-bound
    // phases (k_huff, the small compaction kernels, kernel tails) overlap the next batch's
    // kernels.  kstream[0] is `stream`.  PBX_KSTREAMS (1..4, default 3).
    hipStream_t kstream[4] = {};
    std::atomic<int> nks{1};
    std::atomic<uint32_t> kturn{0};
    // Stagger (PBX_KSTAGGER, 1..4): a batch's first kernel waits for the previous batch's
    // stage event (after k_lz77, k_huff, k_scan_offsets, k_encode); 0 = no wait.  Default 1:
    // a batch's k_lz77 starts when the previous batch's k_lz77 has ended, so it overlaps
    // that batch's k_huff and k_encode rather than competing with its k_lz77.
    std::atomic<int> stagger{1};
    hipEvent_t stage_ev[4][4] = {};     // [stream][stage]
    std::atomic<int> last_ks{-1};       // stream of the last overlapped deflate batch
    hipStream_t copy_stream = nullptr;  // D2H of finished batches, overlapping later kernels
    // Pipelined batches holding both raw / TIFF tiles and deflate tiles run their HBM-bound
    // k_extract on this stream, beside their own (and the previous batch's) issue-bound deflate
    // chain on the kernel stream; consecutive batches' extracts stay in order here.
    // $PBX_SPLIT_EXTRACT=0: one stream per batch, as before.
    hipStream_t xstream = nullptr;
    bool split_extract = true;
    hipStream_t upload_stream = nullptr;  // H2D of plane rows (pbx_plane_write_rows / register)
    std::mutex reg_mu;   // plane registry
    std::mutex run_mu;   // plan + launch of one batch at a time on the stream
    std::mutex copy_mu;  // one fetch at a time on the copy stream
    std::mutex upload_mu;  // one staged upload at a time on upload_stream
    Coalescer* coal = nullptr;
    std::atomic<uint64_t> n_batches{0}, n_requests{0};
    // registry (reg_mu): id -> record (every key's record, evicted ones included, plus
    // released records until their last pin goes), key -> id, image records
    std::unordered_map<uint64_t, Plane*> planes;
    std::map<std::tuple<int64_t, int32_t, int32_t, int32_t, int32_t>, uint64_t> index;
    std::unordered_map<int64_t, Image> images;
    uint64_t next_id = 1;
    // residency (reg_mu)
    uint64_t budget = 0, resident_bytes = 0, use_tick = 0, evictions = 0, evicted_bytes = 0, band_evictions = 0;
    Pool dpool, hpool;
    EventPool evpool, evpool_sync;  // timing events (batch stages), sync-only events (copies)
    // batches of at most this many requests poll their completion events (wait_event) for
    // up to spin_us before blocking ($PBX_SPIN_US, default 2000; 0 = always block)
    uint32_t spin_max_reqs = 8;
    int64_t spin_us = 2000;
    // lite batches whose output arenas fit this many bytes write them straight into pinned
    // host memory (pbx_batch::h_zc; $PBX_ZC_MAX, default 4 MiB, 0 = always D2H)
    uint64_t zc_max = 4u << 20;
    Reaper reaper;  // hipFree of plane HBM, off the serving threads
    // fault injection (tests): the batch launched with ordinal fail_at (1-based,
    // counted over every batch launch of this context; $PBX_FAIL_BATCH or
    // pbx_test_fail_batch) completes with a device failure (500 for its requests)
    std::atomic<uint64_t> launch_seq{0}, fail_at{0};
    // request deadline of pbx_get_tile (pbx_config.request_timeout_us resolved; <= 0: none)
    int64_t timeout_us = 15000000;
    std::atomic<uint64_t> late_requests{0};  // calls answered 500 at their deadline
    // stall injection (pbx_test_stall_batch): the batch launched with ordinal stall_at starts
    // behind k_stall, which spins while *stall_flag (mapped pinned host memory) is nonzero
    std::atomic<uint64_t> stall_at{0};
    uint32_t* stall_flag = nullptr;
    // uncoalesced pbx_get_tile calls past their deadline: their tickets and result slots,
    // finished and released by later calls and by pbx_shutdown
    std::mutex late_mu;
    std::vector<std::pair<pbx_ticket*, pbx_result*>> late;
    int64_t stale_ns = STALE_NS;  // a loading band without writers this long is reclaimed
    std::atomic<uint64_t> band_writes{0}, fail_band_write_at{0};  // pbx_test_fail_band_write
};

namespace {

// Waits for every batch kernel stream (before a plane or a pooled block is freed).
hipError_t sync_kernel_streams(pbx_ctx* ctx) {
    hipError_t r = hipSuccess;
    for (int k = 0; k < 4; k++) {
        if (k && !ctx->kstream[k]) continue;
        const hipError_t e = hipStreamSynchronize(k ? ctx->kstream[k] : ctx->stream);
        if (r == hipSuccess) r = e;
    }
    if (ctx->xstream) {
        const hipError_t e = hipStreamSynchronize(ctx->xstream);
        if (r == hipSuccess) r = e;
    }
    return r;
}

// Host-side result storage shared by the results of one batch fetch.
struct HostBlock {
    std::atomic<int> refs{0};
    pbx_ctx* ctx = nullptr;
    void* pinned = nullptr;
    pbx_spans spans{};  // the batch's stage timings (pbx_result_spans)
};

}  // namespace

struct pbx_batch {
    std::vector<pbx_tile_req> reqs;
    std::vector<int32_t> status, w, h;
    std::vector<TileDesc> ft, dt;          // fixed-size (raw / TIFF) and deflate tiles
    std::vector<uint32_t> ft_req, dt_req;  // request index of each
    std::vector<TiledHdr> th;              // tiled-TIFF responses (their sub-tiles carry TF_TILED)
    std::vector<uint32_t> th_req;
    uint32_t ext_blocks = 0, nseg = 0, nblk = 0, filt_blocks = 0;
    bool ext_unaligned = false;  // some k_extract tile is not whole aligned 16-byte words (k_extract<true>)
    // dt = [direct tiles | k_rows tiles | k_filter2 tiles | k_filter3 tiles | k_filter tiles |
    //       tiled-TIFF sub-tiles]
    uint32_t ndirect_tiles = 0, nrows_tiles = 0, rows_blocks = 0, rows_max_rb = 0;
    uint32_t nfilt2_tiles = 0, filt2_blocks = 0, filt2_max_rb = 0;  // k_filter2 group
    uint32_t nfilt3_tiles = 0, filt3_waves = 0, filt3_max_rb = 0;   // k_filter3 group
    uint32_t filt3_filter = 0;  // its PNG filter (the context's: every k_filter3 tile's d.filter)
    bool adaptive = false;      // some PNG tile takes the adaptive filter (k_adaptive_mode first)
    uint32_t adaptive_max_rb = 0;  // the widest row (bytes) of those tiles
    uint64_t fixed_bytes = 0, stream_cap = 0, png_cap = 0;
    uint64_t in_bytes = 0, stream_bytes = 0;
    // device buffers (pool blocks)
    void *d_ft = nullptr, *d_dt = nullptr, *d_fixed = nullptr, *d_stream = nullptr,
         *d_info = nullptr, *d_hist = nullptr, *d_mrec = nullptr, *d_codes = nullptr,
         *d_sizes = nullptr, *d_offs = nullptr, *d_png = nullptr, *d_stamps = nullptr,
         *d_segmap = nullptr, *d_blk = nullptr, *d_th = nullptr;
    void* h_desc = nullptr;  // pinned staging for descriptors (+ the tile offsets read back)
    uint64_t* h_offs_pin = nullptr;  // in h_desc: the deflate tiles' output offsets, D2H'd by the
    bool offs_ready = false;         // kernel stream at the end of a launch that will be fetched
    hipEvent_t ev_copy = nullptr;    // the fetch's D2H on the copy stream
    std::chrono::steady_clock::time_point t_done;  // the fetch saw the kernels complete (PBX_TIMELINE)
    // start, H2D, extract, filter, lz77, huff, offsets, encode, frame
    hipEvent_t ev[9] = {};
    // split launches (pbx_ctx::xstream): the extract kernel's completion on xstream (sync
    // event, recorded twice: descriptors uploaded on the kernel stream, then extract done) and
    // the kernel stream's own start of the row kernels (timing: ms_filter)
    bool split = false;
    hipEvent_t ev_x = nullptr, ev_fs = nullptr;
    // lite: a batch of the serving path (fetched by the coalescer) records only the events its
    // spans need (start, after the extract kernel, before k_frame, end): every event record is
    // a marker packet that costs the device a few microseconds between two kernels
    bool lite = false;
    // zero-copy output (small lite batches): the fixed and deflate output arenas live in one
    // pinned host block [fixed | png at zc_png_at] that the kernels write over PCIe, so the
    // results need no D2H round trip; the block becomes the results' HostBlock at the fetch
    void* h_zc = nullptr;
    uint64_t zc_png_at = 0;
    bool launched = false;
    bool attempted = false;  // batch_launch began enqueuing work (it may have failed midway)
    uint64_t ordinal = 0;    // launch ordinal in the context (fault injection)
    bool inject_fail = false;  // completes with an injected device failure (pbx_test_fail_batch)
    std::vector<uint64_t> h_offs;
    // planes this batch reads (pinned by pbx_batch_plan, unpinned by pbx_batch_destroy), with
    // the number of pins taken on each; the bands of sparse planes it reads, one pin each
    std::vector<std::pair<Plane*, int64_t>> pins;
    std::vector<std::pair<Plane*, int32_t>> band_pins;
    // regions of sparse planes that straddle bands: copied (D2D) into one bridge buffer at
    // launch, before the kernels; their descriptors address the bridge (TF_BRIDGE)
    struct Bridge {
        Plane* p;
        int32_t x, y, w, h, k0, k1;
        int64_t xo, bp;      // column offset (x*bpp mod 256, alignment kept) and row pitch
        uint64_t off;        // offset in the bridge buffer
    };
    std::vector<Bridge> bridges;
    uint64_t bridge_bytes = 0;
    void* d_bridge = nullptr;
};

namespace {

int ensure_device(pbx_ctx* ctx) {
    HIP_TRY(hipSetDevice(ctx->device));
    return PBX_OK;
}

using PlaneKey = std::tuple<int64_t, int32_t, int32_t, int32_t, int32_t>;
PlaneKey key_of(const Plane& p) { return std::make_tuple(p.image_id, p.z, p.c, p.t, p.res); }

// Checks, under reg_mu, that a plane may join the registry: its key is free (or holds an
// evicted plane, which the new one replaces) and it agrees with the image record (the
// Pixels row: pixel type; full-resolution size; declared z/c/t extents and levels).
int registry_check(pbx_ctx* ctx, const Plane& p) {
    auto it = ctx->index.find(key_of(p));
    if (it != ctx->index.end() && ctx->planes.at(it->second)->state != PS_EVICTED)
        return fail(PBX_E_EXISTS, "plane already registered");
    auto im = ctx->images.find(p.image_id);
    if (im == ctx->images.end()) return PBX_OK;
    const Image& I = im->second;
    if ((I.planes || I.declared) && I.pixel_type != p.pixel_type)
        return fail(PBX_E_BADARG, "pixel type differs from the image's");
    if (p.res == 0 && (I.level_planes.count(0) || I.declared) &&
        (I.size_x != p.size_x || I.size_y != p.size_y))
        return fail(PBX_E_BADARG, "plane size differs from the image's");
    if (I.declared && (p.z < 0 || p.z >= I.size_z || p.c < 0 || p.c >= I.size_c || p.t < 0 ||
                       p.t >= I.size_t_ || p.res >= I.nlevels))
        return fail(PBX_E_BADARG, "plane (z=%d c=%d t=%d level=%d) outside the declared image", p.z, p.c, p.t,
                    p.res);
    return PBX_OK;
}

// Drops an evicted record the key of `p` still points at (under reg_mu; it holds no HBM and
// no pins: only READY planes are pinned).  Returns true if the key was such an entry.
bool drop_evicted(pbx_ctx* ctx, const Plane& p) {
    auto it = ctx->index.find(key_of(p));
    if (it == ctx->index.end()) return false;
    auto pit = ctx->planes.find(it->second);
    Plane* old = pit->second;
    if (old->state != PS_EVICTED) return false;
    ctx->planes.erase(pit);
    ctx->index.erase(it);
    delete old;
    return true;
}

// Adds one record under reg_mu (its checks done): a new id, the index entry and the image
// record.  A key that held an evicted plane was already counted by its image.
Plane* registry_add(pbx_ctx* ctx, const Plane& p) {
    const bool replaced = drop_evicted(ctx, p);
    Plane* q = new Plane(p);
    q->id = ctx->next_id++;
    q->indexed = true;
    q->last_use = ++ctx->use_tick;
    ctx->planes[q->id] = q;
    ctx->index[key_of(*q)] = q->id;
    Image& im = ctx->images[q->image_id];
    if (!im.declared && (q->res == 0 || im.planes == 0)) {  // the Pixels row: full-resolution sizes
        im.pixel_type = q->pixel_type;
        im.size_x = q->size_x;
        im.size_y = q->size_y;
    }
    if (!replaced) {
        im.planes++;
        im.level_planes[q->res]++;
    }
    return q;
}

// Inserts finished planes into the registry, all or none, re-checking every key under reg_mu
// at insertion time (a concurrent registration of the same key loses with 409 instead of
// both succeeding).  On failure the caller still owns (and frees) the planes' memory.
int registry_insert(pbx_ctx* ctx, std::vector<Plane>& ps, uint64_t* ids) {
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    for (size_t k = 0; k < ps.size(); k++) {
        if (int rc = registry_check(ctx, ps[k])) return rc;
        for (size_t j = 0; j < k; j++)
            if (key_of(ps[j]) == key_of(ps[k])) return fail(PBX_E_BADARG, "the same plane twice in one call");
    }
    for (size_t k = 0; k < ps.size(); k++) {
        ps[k].state = PS_READY;
        ps[k].fresh_until = mono_ns() + FRESH_NS;
        Plane* q = registry_add(ctx, ps[k]);
        ps[k].id = q->id;
        if (ids) ids[k] = q->id;
    }
    return PBX_OK;
}

// Removes a record's key from the registry (release), under reg_mu.  The record itself goes
// when nothing pins it: its HBM (if any) is appended to `to_free` and the record deleted.
void registry_remove(pbx_ctx* ctx, Plane* p, std::vector<std::pair<void*, size_t>>& to_free) {
    ctx->planes.erase(p->id);
    ctx->index.erase(key_of(*p));
    p->indexed = false;
    auto im = ctx->images.find(p->image_id);
    if (im != ctx->images.end()) {
        if (--im->second.level_planes[p->res] == 0) im->second.level_planes.erase(p->res);
        if (--im->second.planes == 0 && !im->second.declared) ctx->images.erase(im);
    }
    if (p->pins == 0) {
        p->memory(to_free);
        delete p;
    }
}

// Drops `n` pins of a record (under reg_mu); a released record whose last pin goes is freed.
void unpin_locked(pbx_ctx* ctx, Plane* p, int64_t n, std::vector<std::pair<void*, size_t>>& to_free) {
    (void)ctx;
    p->pins -= n;
    if (p->pins == 0 && !p->indexed) {
        p->memory(to_free);
        delete p;
    }
}

// Returns plane HBM (outside reg_mu): the blocks go to the reaper thread, which hipFrees them
// (hipFree waits for the whole device).  Nothing reads them: their record had no pins, and it
// was unreachable from the index or evicted.  They stop counting as resident at once.
void free_planes(pbx_ctx* ctx, const std::vector<std::pair<void*, size_t>>& to_free) {
    if (to_free.empty()) return;
    uint64_t bytes = 0;
    for (auto& f : to_free) {
        ctx->reaper.put(f.first);
        bytes += f.second;
    }
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    ctx->resident_bytes -= bytes;
}

// Evicts the least recently used idle plane (READY, registered, no pins), under reg_mu.
// Its key stays registered (PS_EVICTED: requests answer NOT_RESIDENT).  Its HBM goes to
// `to_free` for a plain hipFree (no longer counted as resident).  False if none.
// Bands of sparse planes compete in the same LRU: a READY band no batch pins is evicted on its
// own (state back to BS_ABSENT; the plane stays registered and READY).
bool evict_one_locked(pbx_ctx* ctx, std::vector<std::pair<void*, size_t>>& to_free) {
    Plane* v = nullptr;
    Band* vb = nullptr;
    uint64_t best = UINT64_MAX;
    const int64_t now = mono_ns();
    for (auto& kv : ctx->planes) {
        Plane* p = kv.second;
        if (!p->indexed || p->state != PS_READY) continue;
        if (p->sparse_rows) {
            for (Band& b : p->bands) {
                const bool stale = b.state == BS_LOADING && b.writers == 0 && b.dev && now - b.touched > ctx->stale_ns;
                const uint64_t age = stale ? 0 : b.last_use;  // stale loads go first
                if (((b.state == BS_READY && b.pins == 0 && b.dev && b.fresh_until <= now) || stale) && age < best) {
                    best = age;
                    v = p;
                    vb = &b;
                }
            }
        } else if (p->pins == 0 && p->dev && p->fresh_until <= now && p->last_use < best) {
            best = p->last_use;
            v = p;
            vb = nullptr;
        }
    }
    if (!v) return false;
    uint8_t** dev = vb ? &vb->dev : &v->dev;
    const size_t bytes = vb ? vb->bytes : v->bytes;
    to_free.emplace_back(*dev, bytes);
    ctx->resident_bytes -= bytes;
    ctx->evictions++;
    ctx->evicted_bytes += bytes;
    *dev = nullptr;
    if (vb) {
        if (vb->state == BS_LOADING) vb->stale_reset = true;  // (a stale load: see Band)
        vb->state = BS_ABSENT;
        vb->rows_done.clear();
        vb->failed = false;
        ctx->band_evictions++;
    } else {
        v->state = PS_EVICTED;
    }
    return true;
}

// Bytes an eviction could return now (idle planes and idle bands), under reg_mu.
uint64_t idle_bytes_locked(pbx_ctx* ctx) {
    uint64_t idle = 0;
    const int64_t now = mono_ns();
    for (auto& kv : ctx->planes) {
        const Plane* p = kv.second;
        if (!p->indexed || p->state != PS_READY) continue;
        if (p->sparse_rows) {
            for (const Band& b : p->bands)
                if ((b.state == BS_READY && b.pins == 0 && b.dev && b.fresh_until <= now) ||
                    (b.state == BS_LOADING && b.writers == 0 && b.dev && now - b.touched > ctx->stale_ns))
                    idle += b.bytes;
        } else if (p->pins == 0 && p->dev && p->fresh_until <= now) {
            idle += p->bytes;
        }
    }
    return idle;
}

// HBM for a plane, within the residency budget: evicts idle planes (LRU) to make room, and
// again whenever hipMalloc runs out of device memory.  The bytes count as resident from here
// on; plane_free returns them.
int plane_alloc(pbx_ctx* ctx, size_t bytes, uint8_t** out) {
    *out = nullptr;
    std::vector<std::pair<void*, size_t>> victims;
    {
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        if (ctx->budget) {
            const uint64_t idle = idle_bytes_locked(ctx);
            if (ctx->resident_bytes + bytes > ctx->budget + idle)
                return fail(PBX_E_NO_SPACE, "plane of %zu bytes does not fit the residency budget (%llu of %llu "
                            "bytes held, %llu idle)", bytes, (unsigned long long)ctx->resident_bytes,
                            (unsigned long long)ctx->budget, (unsigned long long)idle);
            while (ctx->resident_bytes + bytes > ctx->budget)
                if (!evict_one_locked(ctx, victims)) break;
        }
        ctx->resident_bytes += bytes;
    }
    for (auto& v : victims) ctx->reaper.put(v.first);
    bool drained = false;
    for (;;) {
        const hipError_t e = hipMalloc((void**)out, bytes);
        if (e == hipSuccess) return PBX_OK;
        (void)hipGetLastError();
        if (e == hipErrorOutOfMemory && !drained) {  // blocks on their way back first
            ctx->reaper.drain();
            drained = true;
            continue;
        }
        std::vector<std::pair<void*, size_t>> one;
        {
            std::lock_guard<std::mutex> g(ctx->reg_mu);
            if (e != hipErrorOutOfMemory || !evict_one_locked(ctx, one)) {
                ctx->resident_bytes -= bytes;
                *out = nullptr;
                return fail(e == hipErrorOutOfMemory ? PBX_E_NO_SPACE : PBX_E_INTERNAL,
                            "plane of %zu bytes: hipMalloc: %s (no idle plane left to evict)", bytes,
                            hipGetErrorString(e));
            }
        }
        ctx->reaper.put(one[0].first);
        ctx->reaper.drain();
    }
}

void plane_free(pbx_ctx* ctx, void* dev, size_t bytes) {
    if (!dev) return;
    free_planes(ctx, {{dev, bytes}});
}

// Mirrors TileRequestHandler.getTile (TileRequestHandler.java:80-139) up to the dispatch:
// returns PBX_OK and the plane (pinned: the caller unpins it), the status the reference ends
// with, or PBX_E_NOT_RESIDENT where the reference would open a plane this context does not
// hold (getPixels + getPixelBuffer, :84-86).
// pin = false: a probe (node routing) that takes no pin and leaves the LRU stamps alone.
// kr (sparse planes): the first and last band the region covers, each pinned with the plane.
// owns (probes): set to true when the answer is NOT_RESIDENT only because bands of rows this
// context owns are not loaded yet (the node routes such a request to this context).
int validate(pbx_ctx* ctx, const pbx_tile_req& r, int32_t& w, int32_t& h, Plane*& plane, bool pin = true,
             int32_t* kr = nullptr, bool* owns = nullptr) {
    w = r.w;
    h = r.h;
    plane = nullptr;
    if (owns) *owns = false;
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    auto im = ctx->images.find(r.image_id);
    // :84 getPixels — the image's Pixels row is not known here; the binding looks it up
    // (null -> 404 there) and loads the plane.  What ends in null whatever the image holds is
    // answered first, so that nothing is loaded for it: an unknown format (:125-126) and a
    // region no pixel type makes a valid byte[] (negative, or w*h alone past 2^31-1, :100-103).
    if (im == ctx->images.end()) {
        if (r.format != PBX_FMT_RAW && r.format != PBX_FMT_PNG && r.format != PBX_FMT_TIF)
            return fail(PBX_E_NOTFOUND, "Unknown output format");
        if (r.w < 0 || r.h < 0 || (int64_t)r.w * (int64_t)r.h > 2147483647LL)
            return fail(PBX_E_NOTFOUND, "invalid tile size %dx%d", r.w, r.h);
        return fail(PBX_E_NOT_RESIDENT, "Image:%lld not resident", (long long)r.image_id);
    }
    // :89-91 — pixelBuffer.setResolutionLevel(resolution) when given.  OMERO numbers levels
    // the other way round from storage: resolution getResolutionLevels()-1 is the full
    // resolution and 0 the smallest (omero-zarr-pixel-buffer's ZarrPixelBuffer maps it to
    // NGFF dataset levels-1-resolution; a level outside [0, levels) throws
    // IllegalArgumentException, which getTile turns into null -> 404).  Stored level 0 is
    // the full resolution.  Not given (PBX_RESOLUTION_NONE): the buffer's default, full res.
    int32_t level = 0;
    if (r.resolution != PBX_RESOLUTION_NONE) {
        const int32_t nlev = im->second.levels();
        if (r.resolution < 0 || r.resolution >= nlev)
            return fail(PBX_E_NOTFOUND, "This image has only %d resolution levels", nlev);
        level = nlev - 1 - r.resolution;
    }
    // :92-97 — defaults come from the full-resolution Pixels sizes even with `resolution`
    if (w == 0) w = im->second.size_x;
    if (h == 0) h = im->second.size_y;
    const int bpp = bpp_of(im->second.pixel_type);
    // :100-103 — int tileSize = w*h*bpp; overflow / negative size -> exception -> null -> 404
    const int64_t tile_size = (int64_t)w * (int64_t)h * bpp;
    if (w < 0 || h < 0 || tile_size > 2147483647LL || tile_size <= 0)
        return fail(PBX_E_NOTFOUND, "invalid tile size %dx%d", w, h);
    // The format is decided after getTileDirect upstream, but both of its failures end in
    // null -> 404 whatever the plane holds, so they are checked before loading anything.
    switch (r.format) {
    case PBX_FMT_RAW:
    case PBX_FMT_TIF:
        break;
    case PBX_FMT_PNG:
        // APNGWriter accepts int8/uint8/int16/uint16 only ("Unsupported image type")
        if (bpp > 2) return fail(PBX_E_NOTFOUND, "png: unsupported pixel type");
        break;
    default:
        return fail(PBX_E_NOTFOUND, "Unknown output format");  // :125-126
    }
    const Image& I = im->second;
    auto it = ctx->index.find(std::make_tuple(r.image_id, r.z, r.c, r.t, level));
    if (it == ctx->index.end()) {
        // getTileDirect of a z/c/t outside the declared image throws -> 404; otherwise the
        // plane exists upstream and is not loaded here
        if (I.declared && (r.z < 0 || r.z >= I.size_z || r.c < 0 || r.c >= I.size_c || r.t < 0 ||
                           r.t >= I.size_t_))
            return fail(PBX_E_NOTFOUND, "no plane z=%d c=%d t=%d", r.z, r.c, r.t);
        return fail(PBX_E_NOT_RESIDENT, "plane z=%d c=%d t=%d level=%d not resident", r.z, r.c, r.t, level);
    }
    Plane* p = ctx->planes.at(it->second);
    if (p->state != PS_READY)
        return fail(PBX_E_NOT_RESIDENT, "plane z=%d c=%d t=%d level=%d %s", r.z, r.c, r.t, level,
                    p->state == PS_EVICTED ? "evicted" : "still loading");
    // getTileDirect outside the plane throws (upstream PixelBuffer) -> 404
    if (r.x < 0 || r.y < 0 || (int64_t)r.x + w > p->size_x || (int64_t)r.y + h > p->size_y)
        return fail(PBX_E_NOTFOUND, "region outside plane");
    // a row band: rows outside it belong to another context; a sparse plane serves every region
    // whose first row it owns (the bands past the owned rows such a region covers are loaded
    // here as guest bands: the reference's getTileDirect serves any region of the plane)
    if (r.y < p->band_y0 || r.y >= (int64_t)p->band_y0 + p->band_rows ||
        (!p->sparse_rows && (int64_t)r.y + h > (int64_t)p->band_y0 + p->band_rows))
        return fail(PBX_E_NOT_RESIDENT, "rows %d..%lld outside the resident band %d..%d", r.y,
                    (long long)r.y + h, p->band_y0, p->band_y0 + p->band_rows);
    if (p->sparse_rows) {  // every band the rows cover must be resident
        const int32_t k0 = r.y / p->sparse_rows, k1 = (int32_t)(((int64_t)r.y + h - 1) / p->sparse_rows);
        for (int32_t k = k0; k <= k1; k++)
            if (p->bands[(size_t)k].state != BS_READY) {
                if (owns) *owns = true;
                return fail(PBX_E_NOT_RESIDENT, "rows %d..%lld: band %d (rows %d..%d) of plane z=%d c=%d t=%d level=%d "
                            "not resident", r.y, (long long)r.y + h, k, p->band_lo(k), p->band_hi(k), r.z, r.c, r.t,
                            level);
            }
        if (kr) {
            kr[0] = k0;
            kr[1] = k1;
        }
        if (!pin) return PBX_OK;
        const uint64_t tick = ++ctx->use_tick;
        for (int32_t k = k0; k <= k1; k++) {
            p->bands[(size_t)k].pins++;
            p->bands[(size_t)k].last_use = tick;
            p->bands[(size_t)k].fresh_until = 0;
        }
    } else if (kr) {
        kr[0] = kr[1] = -1;
    }
    if (!pin) return PBX_OK;
    p->pins++;
    p->last_use = ++ctx->use_tick;
    p->fresh_until = 0;
    plane = p;
    return PBX_OK;
}

// Drops every pin a batch holds (its kernels have finished or never ran).
void batch_unpin(pbx_ctx* ctx, pbx_batch* b) {
    if (b->pins.empty()) return;
    std::vector<std::pair<void*, size_t>> to_free;
    {
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        for (auto& bp : b->band_pins) bp.first->bands[(size_t)bp.second].pins--;  // before the plane pins
        for (auto& pc : b->pins) unpin_locked(ctx, pc.first, pc.second, to_free);
    }
    b->band_pins.clear();
    b->pins.clear();
    free_planes(ctx, to_free);
}

void free_batch_device(pbx_ctx* ctx, pbx_batch* b) {
    if (b->zc_png_at || b->h_zc) {  // the output arenas were in the zero-copy block
        b->d_fixed = b->d_png = nullptr;
        if (b->h_zc) ctx->hpool.put(b->h_zc);
        b->h_zc = nullptr;
    }
    void** bufs[] = {&b->d_ft,   &b->d_dt,    &b->d_fixed, &b->d_stream, &b->d_info, &b->d_hist,
                     &b->d_mrec, &b->d_codes, &b->d_sizes, &b->d_offs,   &b->d_png,  &b->d_stamps,
                     &b->d_segmap, &b->d_blk, &b->d_th, &b->d_bridge};
    for (void** p : bufs) {
        ctx->dpool.put(*p);
        *p = nullptr;
    }
    if (b->h_desc) ctx->hpool.put(b->h_desc);
    b->h_desc = nullptr;
}

}  // namespace

// k_extract's aligned path takes the tile: no padding, and its rows start and end on 16-byte
// words (plane and bridge rows are 256-aligned and keep a region's column alignment, fixed
// arena offsets are 16-byte aligned)
static bool ext_aligned(const TileDesc& d) {
    return !d.vw && ((int64_t)d.x * d.bpp) % 16 == 0 && ((int64_t)d.w * d.bpp) % 16 == 0;
}

// Rows of one k_extract workgroup: about this many bytes ($PBX_EXT_BLK for aligned tiles,
// $PBX_EXT_BLK_UA for the realigned path; 16 KiB each).  32 KiB unaligned blocks move the
// headline grid at x*bpp mod 16 = 6 faster (0.824 -> 0.797 ms) but configs[4]'s stream of
// smaller launches slower (548k -> 535k tiles/s), profiles/r06t/: the baseline config wins.
static uint32_t ext_blk_bytes(bool aligned) {
    static const uint32_t v[2] = {[] {
        const char* e = getenv("PBX_EXT_BLK_UA");
        const long x = e ? atol(e) : 16384;
        return (uint32_t)std::min<long>(1 << 20, std::max<long>(1024, x));
    }(), [] {
        const char* e = getenv("PBX_EXT_BLK");
        const long x = e ? atol(e) : 16384;
        return (uint32_t)std::min<long>(1 << 20, std::max<long>(1024, x));
    }()};
    return v[aligned ? 1 : 0];
}

static int batch_launch(pbx_ctx* ctx, pbx_batch* b, bool overlap, bool fetch_follows);

// One synchronous batch: plan + launch under run_mu (launches stay in order on the
// kernel stream), then the fetch outside it, so that concurrent callers overlap one
// batch's D2H with the next batch's kernels.  A device failure fails every request of the
// batch with 500 (PixelBufferVerticle.java:141-146).
static int run_batch(pbx_ctx* ctx, const pbx_tile_req* reqs, uint64_t n, pbx_result* out) {
    pbx_batch* b = nullptr;
    int st;
    {
        std::lock_guard<std::mutex> run(ctx->run_mu);
        st = pbx_batch_plan(ctx, reqs, n, &b);
        if (st) return st;
        st = batch_launch(ctx, b, false, true);
    }
    ctx->n_batches++;
    ctx->n_requests += n;
    if (st == PBX_OK) st = pbx_batch_fetch(ctx, b, out);
    if (st != PBX_OK) {
        const std::string msg = g_err;
        for (uint64_t i = 0; i < n; i++) {
            out[i].status = b->status[i] == PBX_OK ? PBX_E_INTERNAL : b->status[i];
            out[i].format = reqs[i].format;
            out[i].w = b->w[i];
            out[i].h = b->h[i];
            out[i].data = nullptr;
            out[i].len = 0;
            out[i].owner = nullptr;
        }
        pbx_batch_destroy(ctx, b);
        g_err = msg;
        return st;
    }
    pbx_batch_destroy(ctx, b);
    return PBX_OK;
}

// A pbx_get_tile call past its deadline: 500, as the reference's event-bus reply timeout
// (PixelBufferMicroserviceVerticle.java:148-151,356-366).
static int deadline_result(pbx_ctx* ctx, const pbx_tile_req& r, pbx_result* out) {
    ctx->late_requests++;
    out->status = PBX_E_INTERNAL;
    out->format = r.format;
    out->w = r.w;
    out->h = r.h;
    out->data = nullptr;
    out->len = 0;
    out->owner = nullptr;
    return fail(PBX_E_INTERNAL, "request deadline of %lld us exceeded", (long long)ctx->timeout_us);
}

// Uncoalesced calls that passed their deadline: finish the batches that have completed (all
// of them when `block`), release their results and free their slots.
static void collect_late(pbx_ctx* ctx, bool block) {
    std::vector<std::pair<pbx_ticket*, pbx_result*>> todo, keep;
    {
        std::lock_guard<std::mutex> g(ctx->late_mu);
        todo.swap(ctx->late);
    }
    if (todo.empty()) return;
    const std::string err = g_err;  // (the caller's last error survives the collection)
    for (auto& tr : todo) {
        if (pbx_wait(ctx, tr.first, block ? -1 : 0) == PBX_E_PENDING) {
            keep.push_back(tr);
            continue;
        }
        pbx_results_release(ctx, tr.second, 1);
        delete[] tr.second;
    }
    g_err = err;
    if (keep.empty()) return;
    std::lock_guard<std::mutex> g(ctx->late_mu);
    ctx->late.insert(ctx->late.end(), keep.begin(), keep.end());
}

// Request coalescer behind pbx_get_tile: the reference runs getTile on up to
// worker_pool_size concurrent Vert.x worker threads, one request each
// (PixelBufferMicroserviceVerticle.java:117-118,224-233; PixelBufferVerticle.java:109-110).
// Callers block as before; a launcher thread turns every request queued while the GPU is
// busy into ONE batch (no fixed time window: an idle GPU takes a lone request at once),
// with at most DEPTH batches in flight, and completer threads ($PBX_COMPLETERS, default 2)
// fetch finished batches (D2H on the copy stream, the copies of two batches queued back to
// back) and wake their callers.
struct Coalescer {
    static constexpr size_t MAX_BATCH = 1 << 16;
    // Heap-allocated: a caller that gives up at its deadline leaves it to the completer, which
    // releases the late result and frees it (abandoned).
    using clk = std::chrono::steady_clock;
    struct Pending {
        pbx_tile_req req;
        pbx_result res{};
        std::atomic<bool> done{false};  // set under mu; a spinning caller polls it unlocked
        bool abandoned = false;
        // PBX_TIMELINE: submitted, taken by the launcher, planned, launched, kernels seen
        // complete, fetched (D2H done), caller woken
        clk::time_point t[7];
        int rc = PBX_OK;
        std::string err;
        std::condition_variable cv;  // this caller only: no thundering herd per batch
    };
    struct Flight {
        pbx_batch* b;
        std::vector<Pending*> reqs;
        int rc;
        std::string err;
    };
    pbx_ctx* ctx;
    std::mutex mu;
    std::condition_variable cv_launch, cv_complete;
    // Batches in flight (launched, not yet fetched): up to `depth` ($PBX_COALESCE_DEPTH), but
    // the k-th concurrent batch only once `launch_min[k]` requests wait, so that few callers
    // get few, larger batches and many callers get a deeper pipeline (measured:
    // scripts/serve_sweep.py).
    int depth = 4;
    // Requests per batch at most ($PBX_MAX_BATCH): with many callers, batches of <= 64 keep
    // the kernel / D2H pipeline fine-grained, so no caller waits behind one large batch's
    // copy (512 callers: p99 4.6 ms at 64, 15-46 ms uncapped; profiles/r03_sv).
    size_t max_batch = 64;
    size_t launch_min[8] = {1, 4, 32, 64, 128, 256, 512, 1024};
    bool may_launch() const { return !queue.empty() && inflight < depth && queue.size() >= launch_min[inflight]; }
    std::deque<Pending*> queue;
    std::deque<Flight> flights;
    int inflight = 0;
    bool stop = false;
    // PBX_TIMELINE=1: per-request stage durations (us), summarised on stderr at shutdown
    // (the configs[0] single-request latency breakdown, scripts/c1_latency.py)
    bool timeline = getenv("PBX_TIMELINE") != nullptr;
    // a request that finds the coalescer idle is launched by its own thread ($PBX_DIRECT=0: always
    // by the launcher thread)
    bool direct = !getenv("PBX_DIRECT") || atoi(getenv("PBX_DIRECT")) != 0;
    std::vector<std::array<double, 6>> tl;
    std::thread launcher;
    std::vector<std::thread> completers;

    explicit Coalescer(pbx_ctx* c) : ctx(c) {
        if (const char* d = getenv("PBX_COALESCE_DEPTH")) depth = std::min(8, std::max(1, atoi(d)));
        if (const char* m = getenv("PBX_MAX_BATCH")) max_batch = std::min<size_t>(MAX_BATCH, std::max(1, atoi(m)));
        int nc = 2;
        if (const char* c = getenv("PBX_COMPLETERS")) nc = std::min(8, std::max(1, atoi(c)));
        launcher = std::thread([this] { launch_loop(); });
        for (int k = 0; k < nc; k++) completers.emplace_back([this] { complete_loop(); });
    }
    ~Coalescer() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv_launch.notify_all();
        cv_complete.notify_all();
        launcher.join();
        for (auto& t : completers) t.join();
        if (timeline && !tl.empty()) {
            static const char* name[6] = {"queue_to_launcher", "plan", "launch_enqueue", "kernels_to_seen_done",
                                          "fetch_d2h", "wake_caller"};
            fprintf(stderr, "[pbx timeline] %zu requests, us p50/p90/p99:", tl.size());
            for (int k = 0; k < 6; k++) {
                std::vector<double> v;
                for (auto& a : tl) v.push_back(a[k]);
                std::sort(v.begin(), v.end());
                fprintf(stderr, " %s %.1f/%.1f/%.1f", name[k], v[v.size() / 2], v[v.size() * 9 / 10],
                        v[std::min(v.size() - 1, v.size() * 99 / 100)]);
            }
            fprintf(stderr, "\n");
        }
    }
    // One request, blocking until its batch is fetched or its deadline (ctx->timeout_us, the
    // reference's event-bus send timeout, PixelBufferMicroserviceVerticle.java:148-151) has
    // passed: then 500 (:356-366).  A request still queued is withdrawn; one whose batch is in
    // flight is abandoned to the completer, which releases its result when the batch ends.
    // `to` (us, <= 0: none) is the call's deadline, counted from entry: neither the plan and
    // launch of a direct request nor a wait for ctx->run_mu may run past it.
    int submit(const pbx_tile_req& r, pbx_result* out, int64_t to) {
        const auto t_in = clk::now();
        const auto until = t_in + std::chrono::microseconds(to > 0 ? to : 0);
        Pending* p = new Pending();
        p->req = r;
        if (timeline) p->t[0] = t_in;
        std::unique_lock<std::mutex> g(mu);
        if (stop) {
            delete p;
            return fail(PBX_E_INTERNAL, "context is shutting down");
        }
        bool launched = false;
        if (queue.empty() && inflight == 0 && direct) {
            // an idle coalescer: this thread plans and launches its own request (no hand-off
            // to the launcher thread, whose wake-up the lone request would wait for) -- but only
            // if run_mu is free now: a thread holding it (a release_cached syncing a wedged
            // device, a batch launch) could keep a direct caller past its deadline, so such a
            // request goes to the launcher and this thread waits on its deadline.  The
            // completer fetches a direct batch as any other, so the deadline below holds.
            std::unique_lock<std::mutex> run(ctx->run_mu, std::try_to_lock);
            if (run.owns_lock()) {
                inflight++;
                g.unlock();
                launch_take(std::vector<Pending*>{p}, &run);
                g.lock();
                launched = true;
            }
        }
        if (!launched) {
            queue.push_back(p);
            cv_launch.notify_one();
        }
        // a lone caller (an idle coalescer: the single-request latency path) polls for its
        // result before it blocks -- a condition-variable wake-up costs it ~15 us
        if (ctx->spin_us > 0 && queue.size() + (size_t)inflight <= 2) {
            g.unlock();
            auto spin_until = t_in + std::chrono::microseconds(ctx->spin_us);
            if (to > 0 && until < spin_until) spin_until = until;
            while (!p->done.load(std::memory_order_acquire) && clk::now() < spin_until) cpu_relax();
            g.lock();
        }
        if (to > 0) {
            if (!p->cv.wait_until(g, until, [&] { return p->done.load(); })) {
                const auto it = std::find(queue.begin(), queue.end(), p);
                if (it != queue.end()) {
                    queue.erase(it);
                    delete p;
                } else {
                    p->abandoned = true;
                }
                g.unlock();
                return deadline_result(ctx, r, out);
            }
        } else {
            p->cv.wait(g, [&] { return p->done.load(); });
        }
        *out = p->res;
        const int rc = p->rc;
        if (rc != PBX_OK) g_err = p->err;
        if (timeline) {
            p->t[6] = clk::now();
            std::array<double, 6> a;
            for (int k = 0; k < 6; k++) a[k] = std::chrono::duration<double, std::micro>(p->t[k + 1] - p->t[k]).count();
            tl.push_back(a);  // (under mu)
        }
        delete p;
        return rc;
    }
    void launch_loop() {
        (void)hipSetDevice(ctx->device);
        for (;;) {
            std::vector<Pending*> take;
            {
                std::unique_lock<std::mutex> g(mu);
                cv_launch.wait(g, [&] { return (stop && queue.empty()) || may_launch(); });
                if (queue.empty()) break;  // stopping, nothing left
                while (!queue.empty() && take.size() < max_batch) {
                    take.push_back(queue.front());
                    queue.pop_front();
                }
                inflight++;
            }
            launch_take(std::move(take));
        }
        std::lock_guard<std::mutex> g(mu);
        cv_complete.notify_all();
    }
    // Plans and launches one batch of taken requests (inflight already counts it) and hands
    // it to the completers.
    // `held`: run_mu already taken by the caller (the direct path); released here after the launch.
    void launch_take(std::vector<Pending*> take, std::unique_lock<std::mutex>* held = nullptr) {
        (void)hipSetDevice(ctx->device);
        {
            std::vector<pbx_tile_req> reqs(take.size());
            for (size_t i = 0; i < take.size(); i++) reqs[i] = take[i]->req;
            Flight f{nullptr, std::move(take), PBX_OK, {}};
            clk::time_point t1, t2, t3;
            if (timeline) t1 = clk::now();
            {
                std::unique_lock<std::mutex> own;
                if (!held) own = std::unique_lock<std::mutex>(ctx->run_mu);
                f.rc = pbx_batch_plan(ctx, reqs.data(), reqs.size(), &f.b);
                if (timeline) t2 = clk::now();
                if (f.rc == PBX_OK) f.rc = batch_launch(ctx, f.b, false, true);
                if (f.rc != PBX_OK) f.err = g_err;
                if (held) held->unlock();
            }
            if (timeline) {
                t3 = clk::now();
                for (Pending* p : f.reqs) { p->t[1] = t1; p->t[2] = t2; p->t[3] = t3; }
            }
            ctx->n_batches++;
            ctx->n_requests += reqs.size();
            {
                std::lock_guard<std::mutex> g(mu);
                flights.push_back(std::move(f));
            }
            cv_complete.notify_one();
        }
    }
    void complete_loop() {
        (void)hipSetDevice(ctx->device);
        for (;;) {
            Flight f;
            {
                std::unique_lock<std::mutex> g(mu);
                cv_complete.wait(g, [&] { return !flights.empty() || (stop && queue.empty() && inflight == 0); });
                if (flights.empty()) break;
                f = std::move(flights.front());
                flights.pop_front();
            }
            const size_t n = f.reqs.size();
            std::vector<pbx_result> res(n);
            if (f.rc == PBX_OK) {
                f.rc = pbx_batch_fetch(ctx, f.b, res.data());
                if (f.rc != PBX_OK) f.err = g_err;
            }
            if (timeline && f.b) {
                const clk::time_point t5 = clk::now();
                for (Pending* p : f.reqs) { p->t[4] = f.b->t_done; p->t[5] = t5; }
            }
            for (size_t i = 0; i < n; i++) {
                pbx_result& o = f.reqs[i]->res;
                if (f.rc == PBX_OK) {
                    o = res[i];
                } else {
                    const int32_t s = f.b ? f.b->status[i] : PBX_E_INTERNAL;
                    o.status = s == PBX_OK ? PBX_E_INTERNAL : s;
                    o.format = f.reqs[i]->req.format;
                    o.w = f.b ? f.b->w[i] : 0;
                    o.h = f.b ? f.b->h[i] : 0;
                    o.data = nullptr;
                    o.len = 0;
                    o.owner = nullptr;
                }
            }
            if (f.b) pbx_batch_destroy(ctx, f.b);
            std::vector<Pending*> late;  // callers gone at their deadline
            {
                std::lock_guard<std::mutex> g(mu);
                for (Pending* p : f.reqs) {
                    if (p->abandoned) {
                        late.push_back(p);
                        continue;
                    }
                    p->rc = f.rc;
                    p->err = f.err;
                    p->done.store(true, std::memory_order_release);
                    p->cv.notify_one();  // under mu: the caller cannot return (and free p) first
                }
                inflight--;
            }
            for (Pending* p : late) {
                pbx_results_release(ctx, &p->res, 1);
                delete p;
            }
            cv_launch.notify_one();
            cv_complete.notify_all();  // (shutdown: the other completers see inflight == 0)
        }
    }
};

// ============================================================================ C-ABI

extern "C" {

const char* pbx_last_error(void) { return g_err.c_str(); }
int pbx_abi_version(void) { return PBX_ABI_VERSION; }

int pbx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int pbx_bytes_per_pixel(int32_t pt) { return bpp_of(pt); }

int pbx_format_from_string(const char* f) {
    if (!f) return PBX_FMT_RAW;
    if (!strcmp(f, "png")) return PBX_FMT_PNG;
    if (!strcmp(f, "tif")) return PBX_FMT_TIF;
    return PBX_FMT_UNKNOWN;
}

int pbx_pixel_type_from_string(const char* n) {
    static const char* names[PBX_NPIXEL_TYPES] = {"int8", "uint8", "int16", "uint16",
                                                  "int32", "uint32", "float", "double"};
    if (!n) return -1;
    for (int i = 0; i < PBX_NPIXEL_TYPES; i++)
        if (!strcmp(n, names[i])) return i;
    return -1;
}

int pbx_tile_filename(const pbx_tile_req* r, int32_t w, int32_t h, const char* fmt, char* out,
                      uint64_t cap) {
    if (!r || !out) return fail(PBX_E_BADARG, "null argument");
    return snprintf(out, cap, "image%lld_z%d_c%d_t%d_x%d_y%d_w%d_h%d.%s", (long long)r->image_id,
                    r->z, r->c, r->t, r->x, r->y, w, h, fmt ? fmt : "bin");
}

const char* pbx_content_type(const char* f) {
    if (f && !strcmp(f, "png")) return "image/png";
    if (f && !strcmp(f, "tif")) return "image/tiff";
    return "application/octet-stream";
}

int pbx_config_default(pbx_config* cfg) {
    if (!cfg) return fail(PBX_E_BADARG, "null config");
    memset(cfg, 0, sizeof *cfg);
    cfg->device = -1;
    cfg->png_filter = PBX_FILTER_NONE;
    cfg->coalesce = 1;
    const char* co = getenv("PBX_COALESCE");
    if (co) cfg->coalesce = atoi(co);
    const char* sr = getenv("PBX_STAGE_ROWS");
    if (sr) cfg->stage_rows = atoi(sr);
    const char* f = getenv("PBX_PNG_FILTER");
    if (f) cfg->png_filter = atoi(f);
    const char* td = getenv("PBX_TIFF_DEFLATE");
    if (td) cfg->tiff_deflate = atoi(td);
    const char* tt = getenv("PBX_TIFF_TILE");
    if (tt) cfg->tiff_tile = atoi(tt);
    cfg->request_timeout_us = 15000000;  // the reference's event-bus send timeout (15 s)
    if (const char* rt = getenv("PBX_REQUEST_TIMEOUT_US")) cfg->request_timeout_us = atoi(rt);
    return PBX_OK;
}

int pbx_init(const pbx_config* cfg_in, pbx_ctx** out) {
    if (!out) return fail(PBX_E_BADARG, "null out");
    *out = nullptr;
    pbx_config cfg;
    if (cfg_in) cfg = *cfg_in; else pbx_config_default(&cfg);
    if (cfg.png_filter < PBX_FILTER_NONE || cfg.png_filter > PBX_FILTER_ADAPTIVE)
        return fail(PBX_E_BADARG, "bad png_filter %d", cfg.png_filter);
    if (cfg.tiff_tile && (cfg.tiff_tile < 16 || cfg.tiff_tile > 4096 || cfg.tiff_tile % 16))
        return fail(PBX_E_BADARG, "bad tiff_tile %d (0, or a multiple of 16 in [16, 4096])", cfg.tiff_tile);
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(PBX_E_INTERNAL, "no HIP device available (the tile pipeline runs on MI355X only)");
    int dev = cfg.device;
    if (dev < 0) {
        const char* e = getenv("PBX_DEVICE");
        const char* lr = getenv("LOCAL_RANK");
        dev = e ? atoi(e) : lr ? atoi(lr) : 0;
    }
    if (dev < 0 || dev >= n) return fail(PBX_E_BADARG, "device %d out of range (%d devices)", dev, n);
    pbx_ctx* ctx = new pbx_ctx();
    ctx->device = dev;
    ctx->cfg = cfg;
    ctx->hpool.pinned = true;
    ctx->evpool_sync.flags = hipEventDisableTiming;
    if (const char* su = getenv("PBX_SPIN_US")) ctx->spin_us = atoll(su);
    if (const char* zm = getenv("PBX_ZC_MAX")) ctx->zc_max = strtoull(zm, nullptr, 10);
    ctx->timeout_us = cfg.request_timeout_us;
    if (ctx->timeout_us == 0) {
        const char* rt = getenv("PBX_REQUEST_TIMEOUT_US");
        ctx->timeout_us = rt ? atoll(rt) : 15000000;
    }
    hipError_t e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&ctx->cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->upload_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->xstream, hipStreamNonBlocking);
    if (const char* sx = getenv("PBX_SPLIT_EXTRACT")) ctx->split_extract = atoi(sx) != 0;
    if (const char* hb = getenv("PBX_HBM_BUDGET_MB")) ctx->budget = (uint64_t)strtoull(hb, nullptr, 10) << 20;
    if (const char* ks = getenv("PBX_KSTREAMS")) ctx->nks = std::min(4, std::max(1, atoi(ks)));
    else ctx->nks = 3;
    ctx->kstream[0] = ctx->stream;
    for (int k = 1; k < 4 && e == hipSuccess; k++)
        e = hipStreamCreateWithFlags(&ctx->kstream[k], hipStreamNonBlocking);
    if (const char* sg = getenv("PBX_KSTAGGER")) ctx->stagger = std::min(4, std::max(0, atoi(sg)));
    for (int k = 0; k < 4 && e == hipSuccess; k++)
        for (int j = 0; j < 4 && e == hipSuccess; j++)
            e = hipEventCreateWithFlags(&ctx->stage_ev[k][j], hipEventDisableTiming);
    if (e != hipSuccess) {
        delete ctx;
        return fail(PBX_E_INTERNAL, "init: %s", hipGetErrorString(e));
    }
    if (const char* fb = getenv("PBX_FAIL_BATCH")) ctx->fail_at = strtoull(fb, nullptr, 10);
    if (const char* bs = getenv("PBX_BAND_STALE_MS")) ctx->stale_ns = (int64_t)atoll(bs) * 1000000;
    ctx->reaper.tick = [ctx] {
        collect_late(ctx, false);
        std::lock_guard<std::mutex> g(ctx->late_mu);
        return !ctx->late.empty();
    };
    ctx->reaper.start(dev);
    if (cfg.coalesce) ctx->coal = new Coalescer(ctx);
    *out = ctx;
    return PBX_OK;
}

void pbx_shutdown(pbx_ctx* ctx) {
    if (!ctx) return;
    if (ctx->stall_flag) __atomic_store_n(ctx->stall_flag, 0u, __ATOMIC_SEQ_CST);  // a stalled batch ends
    delete ctx->coal;  // drains queued requests, joins its threads
    ctx->coal = nullptr;
    ctx->reaper.stop_ticking();  // (no late collection on the reaper thread from here on)
    collect_late(ctx, true);
    (void)hipSetDevice(ctx->device);
    (void)sync_kernel_streams(ctx);
    (void)hipStreamSynchronize(ctx->copy_stream);
    (void)hipStreamSynchronize(ctx->upload_stream);
    ctx->reaper.finish();  // frees what it still holds
    for (auto& kv : ctx->planes) {  // records of released planes still pinned by undestroyed
        std::vector<std::pair<void*, size_t>> blocks;  // batches are leaked with those batches
        kv.second->memory(blocks);  // the whole plane's HBM, or every resident band's
        for (auto& m : blocks) (void)hipFree(m.first);
        delete kv.second;
    }
    ctx->planes.clear();
    ctx->dpool.release_all();
    ctx->hpool.release_all();
    ctx->evpool.release_all();
    ctx->evpool_sync.release_all();
    for (int k = 1; k < 4; k++)
        if (ctx->kstream[k]) (void)hipStreamDestroy(ctx->kstream[k]);
    for (auto& r : ctx->stage_ev)
        for (auto& x : r) if (x) (void)hipEventDestroy(x);
    (void)hipStreamDestroy(ctx->stream);
    (void)hipStreamDestroy(ctx->copy_stream);
    if (ctx->upload_stream) (void)hipStreamDestroy(ctx->upload_stream);
    if (ctx->xstream) (void)hipStreamDestroy(ctx->xstream);
    if (ctx->stall_flag) (void)hipHostFree(ctx->stall_flag);
    delete ctx;
}

int pbx_release_cached(pbx_ctx* ctx) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    std::lock_guard<std::mutex> run(ctx->run_mu);
    if (ensure_device(ctx)) return PBX_E_INTERNAL;
    HIP_TRY(sync_kernel_streams(ctx));
    HIP_TRY(hipStreamSynchronize(ctx->copy_stream));
    ctx->dpool.trim();
    ctx->hpool.trim();
    return PBX_OK;
}

int pbx_set_kernel_streams(pbx_ctx* ctx, int32_t streams, int32_t stagger) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    if (streams < 1 || streams > 4 || stagger < 0 || stagger > 4)
        return fail(PBX_E_BADARG, "kernel streams %d / stagger %d out of range", streams, stagger);
    std::lock_guard<std::mutex> run(ctx->run_mu);
    ctx->nks = streams;
    ctx->stagger = stagger;
    ctx->last_ks = -1;
    return PBX_OK;
}

int pbx_device_synchronize(pbx_ctx* ctx) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    if (ensure_device(ctx)) return PBX_E_INTERNAL;
    HIP_TRY(hipDeviceSynchronize());
    return PBX_OK;
}

// ------------------------------------------------------------- staged host -> HBM upload
}  // extern "C"
namespace {

// Copies `rows` packed host rows of `row` bytes (pageable caller memory) to HBM rows `pitch`
// apart, through pinned staging blocks of the context's pinned pool: each piece (whole rows,
// or a part of one row longer than a piece) is copied into a pinned block by several host
// threads (one thread's memcpy is the bottleneck otherwise) and DMA'd asynchronously on `st`
// while the next piece is being staged.  Returns once every piece is staged and its DMA has
// completed; the pinned blocks go back to the pool.
int upload_rows(pbx_ctx* ctx, uint8_t* dev, int64_t pitch, const uint8_t* host, uint64_t row, uint64_t rows,
                hipStream_t st) {
    constexpr uint64_t PIECE = 32ull << 20;
    constexpr int NBUF = 3;
    const uint64_t total = row * rows;
    if (!total) return PBX_OK;
    if (total < (4ull << 20)) {  // small: one pageable copy
        if ((uint64_t)pitch == row || rows == 1)
            HIP_TRY(hipMemcpyAsync(dev, host, total, hipMemcpyHostToDevice, st));
        else
            HIP_TRY(hipMemcpy2DAsync(dev, pitch, host, row, row, rows, hipMemcpyHostToDevice, st));
        HIP_TRY(hipStreamSynchronize(st));
        return PBX_OK;
    }
    // pieces: k whole rows (row <= PIECE), or [off, off + n) of one row (row > PIECE)
    const bool whole_rows = row <= PIECE;
    const uint64_t k_rows = whole_rows ? std::max<uint64_t>(1, PIECE / row) : 1;
    const uint64_t per_row = whole_rows ? 1 : (row + PIECE - 1) / PIECE;
    const uint64_t npieces = whole_rows ? (rows + k_rows - 1) / k_rows : rows * per_row;
    void* blk[NBUF] = {};
    hipEvent_t ev[NBUF] = {};
    bool used[NBUF] = {};
    hipError_t e = hipSuccess;
    for (int i = 0; i < NBUF && e == hipSuccess; i++) {
        blk[i] = ctx->hpool.get(PIECE, &e);
        if (blk[i]) e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
    }
    const unsigned nth = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
    for (uint64_t p = 0; p < npieces && e == hipSuccess; p++) {
        uint64_t r0, k, off, n;
        if (whole_rows) {
            r0 = p * k_rows;
            k = std::min(k_rows, rows - r0);
            off = 0;
            n = row;
        } else {
            r0 = p / per_row;
            k = 1;
            off = (p % per_row) * PIECE;
            n = std::min(PIECE, row - off);
        }
        const int b = (int)(p % NBUF);
        if (used[b]) e = hipEventSynchronize(ev[b]);  // the block's previous DMA is done
        if (e != hipSuccess) break;
        uint8_t* dst = (uint8_t*)blk[b];
        const uint8_t* src = host + r0 * row + off;
        const uint64_t bytes = k * n;  // contiguous on the host in both cases
        const uint64_t per = (bytes + nth - 1) / nth;
        std::vector<std::thread> th;
        for (unsigned t = 1; t < nth && t * per < bytes; t++)
            th.emplace_back([=] { memcpy(dst + t * per, src + t * per, std::min(per, bytes - t * per)); });
        memcpy(dst, src, std::min(per, bytes));
        for (auto& x : th) x.join();
        uint8_t* d = dev + (int64_t)r0 * pitch + off;
        if (k == 1 || (uint64_t)pitch == n)
            e = hipMemcpyAsync(d, dst, bytes, hipMemcpyHostToDevice, st);
        else
            e = hipMemcpy2DAsync(d, pitch, dst, n, n, k, hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipEventRecord(ev[b], st);
        used[b] = true;
    }
    for (int i = 0; i < NBUF; i++) {
        if (used[i]) (void)hipEventSynchronize(ev[i]);
        if (ev[i]) (void)hipEventDestroy(ev[i]);
        if (blk[i]) ctx->hpool.put(blk[i]);
    }
    if (e != hipSuccess) return fail(PBX_E_INTERNAL, "staged upload: %s", hipGetErrorString(e));
    return PBX_OK;
}

// Contiguous bytes (Zarr chunk data) to HBM, as one "row".
int upload_staged(pbx_ctx* ctx, uint8_t* dev, const uint8_t* host, uint64_t bytes, hipStream_t st) {
    return upload_rows(ctx, dev, (int64_t)bytes, host, bytes, 1, st);
}

// Pins the record of `id` if it is in one of `states` (bit mask of 1 << PlaneState); the
// caller unpins it with unpin_id.  Returns the record or sets the status.
Plane* pin_id(pbx_ctx* ctx, uint64_t id, unsigned states, int* rc) {
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    auto it = ctx->planes.find(id);
    if (it == ctx->planes.end()) {
        *rc = fail(PBX_E_NOTFOUND, "no plane %llu", (unsigned long long)id);
        return nullptr;
    }
    Plane* p = it->second;
    if (!((1u << p->state) & states)) {
        static const char* names[3] = {"still loading", "ready", "evicted"};
        *rc = fail(p->state == PS_READY ? PBX_E_EXISTS : p->state == PS_EVICTED ? PBX_E_NOT_RESIDENT : PBX_E_BADARG,
                   "plane %llu is %s", (unsigned long long)id, names[p->state]);
        return nullptr;
    }
    p->pins++;
    *rc = PBX_OK;
    return p;
}

void unpin_one(pbx_ctx* ctx, Plane* p) {
    std::vector<std::pair<void*, size_t>> to_free;
    {
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        unpin_locked(ctx, p, 1, to_free);
    }
    free_planes(ctx, to_free);
}

// pbx_plane_create: reserve the key (409 if taken), allocate the band within the budget,
// generate it for generator sources.  The new record is returned pinned.
int plane_create(pbx_ctx* ctx, const pbx_plane_desc* d, int32_t y0, int32_t nrows, Plane** out) {
    *out = nullptr;
    if (!d) return fail(PBX_E_BADARG, "null argument");
    const int bpp = bpp_of(d->pixel_type);
    if (!bpp) return fail(PBX_E_BADARG, "bad pixel type %d", d->pixel_type);
    if (d->size_x <= 0 || d->size_y <= 0) return fail(PBX_E_BADARG, "bad plane size");
    if (d->resolution < 0) return fail(PBX_E_BADARG, "bad resolution");
    if (d->source != PBX_SRC_HOST && d->source != PBX_SRC_GEN_FAKE && d->source != PBX_SRC_GEN_NOISE)
        return fail(PBX_E_BADARG, "bad source %d", d->source);
    if (nrows == 0) {
        if (y0 != 0) return fail(PBX_E_BADARG, "band_rows 0 (whole plane) needs band_y0 0");
        nrows = d->size_y;
    }
    if (y0 < 0 || nrows < 0 || (int64_t)y0 + nrows > d->size_y)
        return fail(PBX_E_BADARG, "band %d+%d outside the plane's %d rows", y0, nrows, d->size_y);
    if (ensure_device(ctx)) return PBX_E_INTERNAL;
    Plane p;
    p.image_id = d->image_id; p.z = d->z; p.c = d->c; p.t = d->t; p.res = d->resolution;
    p.pixel_type = d->pixel_type; p.size_x = d->size_x; p.size_y = d->size_y;
    p.band_y0 = y0;
    p.band_rows = nrows;
    const int64_t row = (int64_t)d->size_x * bpp;
    p.pitch = (row + 255) & ~(int64_t)255;
    p.bytes = (size_t)p.pitch * nrows + 256;
    p.little_endian = d->source == PBX_SRC_HOST ? (d->byte_order == PBX_LITTLE_ENDIAN && bpp > 1) : bpp > 1;
    p.state = PS_FILLING;
    Plane* q;
    {
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        if (int rc = registry_check(ctx, p)) return rc;
        q = registry_add(ctx, p);  // the key is ours: concurrent creators get 409
        q->pins = 1;
    }
    auto abandon = [&](int rc) {
        const std::string msg = g_err;
        std::vector<std::pair<void*, size_t>> to_free;
        {
            std::lock_guard<std::mutex> g(ctx->reg_mu);
            if (q->indexed) registry_remove(ctx, q, to_free);  // still pinned: not freed yet
            unpin_locked(ctx, q, 1, to_free);
        }
        free_planes(ctx, to_free);
        g_err = msg;
        return rc;
    };
    uint8_t* dev = nullptr;
    if (int rc = plane_alloc(ctx, p.bytes, &dev)) return abandon(rc);
    {
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        q->dev = dev;
        if (d->source == PBX_SRC_HOST) {
            q->rows_done.assign((size_t)nrows, 0);
            q->rows_left = (uint64_t)nrows;
        }
    }
    hipError_t e;
    {
        std::lock_guard<std::mutex> u(ctx->upload_mu);
        e = hipMemsetAsync(dev + (size_t)p.pitch * nrows, 0, 256, ctx->upload_stream);  // over-read slack
        if (e == hipSuccess && d->source != PBX_SRC_HOST)
            e = launch_gen_plane(ctx->upload_stream, dev, p.pitch, d->size_x, y0, nrows, d->pixel_type,
                                 d->source == PBX_SRC_GEN_FAKE ? GEN_FAKE : GEN_NOISE, d->seed, d->plane_no,
                                 d->z, d->c, d->t);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->upload_stream);
    }
    if (e != hipSuccess) return abandon(fail(PBX_E_INTERNAL, "plane create: %s", hipGetErrorString(e)));
    if (d->source != PBX_SRC_HOST) {
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        q->state = PS_READY;
        q->fresh_until = mono_ns() + FRESH_NS;
    }
    *out = q;
    return PBX_OK;
}

// The rows of a FILLING record that the caller has pinned.
int plane_write(pbx_ctx* ctx, Plane* q, int32_t y0, int32_t rows, const void* data, uint64_t bytes) {
    const int bpp = bpp_of(q->pixel_type);
    const uint64_t row = (uint64_t)q->size_x * bpp;
    if (rows < 0 || y0 < q->band_y0 || (int64_t)y0 + rows > (int64_t)q->band_y0 + q->band_rows)
        return fail(PBX_E_BADARG, "rows %d+%d outside the plane's band %d+%d", y0, rows, q->band_y0, q->band_rows);
    if (!rows) return PBX_OK;
    if (!data || bytes < row * (uint64_t)rows)
        return fail(PBX_E_BADARG, "%llu bytes for %d rows of %llu", (unsigned long long)bytes, rows,
                    (unsigned long long)row);
    if (ensure_device(ctx)) return PBX_E_INTERNAL;
    {   // a writer in flight: pbx_plane_commit refuses to publish the plane until it is done
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        if (q->state != PS_FILLING) return fail(PBX_E_BADARG, "plane %llu is not being loaded", (unsigned long long)q->id);
        q->writers++;
    }
    int rc;
    {
        std::lock_guard<std::mutex> u(ctx->upload_mu);
        rc = upload_rows(ctx, q->dev + (int64_t)(y0 - q->band_y0) * q->pitch, q->pitch, (const uint8_t*)data, row,
                         (uint64_t)rows, ctx->upload_stream);
    }
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    q->writers--;
    if (rc) return rc;
    if (q->state != PS_FILLING)  // cannot happen while we were a writer; kept as the invariant
        return fail(PBX_E_INTERNAL, "plane %llu was published during a write", (unsigned long long)q->id);
    for (int32_t r = y0 - q->band_y0; r < y0 - q->band_y0 + rows; r++)
        if (!q->rows_done[(size_t)r]) {
            q->rows_done[(size_t)r] = 1;
            q->rows_left--;
        }
    return PBX_OK;
}

int plane_commit(pbx_ctx* ctx, Plane* q) {
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    if (q->state != PS_FILLING) return fail(PBX_E_BADARG, "plane %llu is not being loaded", (unsigned long long)q->id);
    if (q->writers)  // rows may still be in flight on upload_stream: never publish them half-written
        return fail(PBX_E_EXISTS, "plane %llu: %d pbx_plane_write_rows calls still running", (unsigned long long)q->id,
                    q->writers);
    if (q->rows_left)
        return fail(PBX_E_BADARG, "plane %llu: %llu rows of its band were never written", (unsigned long long)q->id,
                    (unsigned long long)q->rows_left);
    q->rows_done.clear();
    q->rows_done.shrink_to_fit();
    q->state = PS_READY;
    q->last_use = ++ctx->use_tick;
    q->fresh_until = mono_ns() + FRESH_NS;
    return PBX_OK;
}

}  // namespace
extern "C" {

int pbx_plane_create(pbx_ctx* ctx, const pbx_plane_desc* d, int32_t band_y0, int32_t band_rows, uint64_t* plane_id) {
    if (!ctx || !d || !plane_id) return fail(PBX_E_BADARG, "null argument");
    Plane* q = nullptr;
    if (int rc = plane_create(ctx, d, band_y0, band_rows, &q)) return rc;
    *plane_id = q->id;
    unpin_one(ctx, q);
    return PBX_OK;
}

int pbx_plane_write_rows(pbx_ctx* ctx, uint64_t id, int32_t y0, int32_t rows, const void* data, uint64_t bytes) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    int rc;
    Plane* q = pin_id(ctx, id, 1u << PS_FILLING, &rc);
    if (!q) return rc;
    rc = plane_write(ctx, q, y0, rows, data, bytes);
    const std::string msg = g_err;
    unpin_one(ctx, q);
    g_err = msg;
    return rc;
}

int pbx_plane_commit(pbx_ctx* ctx, uint64_t id) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    int rc;
    Plane* q = pin_id(ctx, id, 1u << PS_FILLING, &rc);
    if (!q) return rc;
    rc = plane_commit(ctx, q);
    const std::string msg = g_err;
    unpin_one(ctx, q);
    g_err = msg;
    return rc;
}

int pbx_plane_register(pbx_ctx* ctx, const pbx_plane_desc* d, uint64_t* plane_id) {
    if (!ctx || !d || !plane_id) return fail(PBX_E_BADARG, "null argument");
    const int bpp = bpp_of(d->pixel_type);
    if (d->source == PBX_SRC_HOST && bpp && d->size_x > 0 && d->size_y > 0 &&
        (!d->host_data || d->host_bytes < (uint64_t)d->size_x * bpp * (uint64_t)d->size_y))
        return fail(PBX_E_BADARG, "host_data too small");
    Plane* q = nullptr;
    if (int rc = plane_create(ctx, d, 0, 0, &q)) return rc;
    int rc = PBX_OK;
    if (d->source == PBX_SRC_HOST) {
        rc = plane_write(ctx, q, 0, d->size_y, d->host_data, d->host_bytes);
        if (rc == PBX_OK) rc = plane_commit(ctx, q);
    }
    const std::string msg = g_err;
    std::vector<std::pair<void*, size_t>> to_free;
    {
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        if (rc != PBX_OK && q->indexed) registry_remove(ctx, q, to_free);  // all or nothing
        if (rc == PBX_OK) *plane_id = q->id;
        unpin_locked(ctx, q, 1, to_free);
    }
    free_planes(ctx, to_free);
    g_err = msg;
    return rc;
}

// ------------------------------------------------------------------ sparse (banded) planes

int pbx_plane_create_sparse(pbx_ctx* ctx, const pbx_plane_desc* d, int32_t band_rows, int32_t own_y0,
                            int32_t own_rows, uint64_t* plane_id) {
    if (!ctx || !d || !plane_id) return fail(PBX_E_BADARG, "null argument");
    const int bpp = bpp_of(d->pixel_type);
    if (!bpp) return fail(PBX_E_BADARG, "bad pixel type %d", d->pixel_type);
    if (d->size_x <= 0 || d->size_y <= 0) return fail(PBX_E_BADARG, "bad plane size");
    if (d->resolution < 0) return fail(PBX_E_BADARG, "bad resolution");
    if (d->source != PBX_SRC_HOST && d->source != PBX_SRC_GEN_FAKE && d->source != PBX_SRC_GEN_NOISE)
        return fail(PBX_E_BADARG, "bad source %d", d->source);
    if (band_rows <= 0) return fail(PBX_E_BADARG, "band_rows %d", band_rows);
    if (own_rows == 0) {
        if (own_y0 != 0) return fail(PBX_E_BADARG, "own_rows 0 (the whole plane) needs own_y0 0");
        own_rows = d->size_y;
    }
    if (own_y0 < 0 || own_rows < 0 || (int64_t)own_y0 + own_rows > d->size_y || own_y0 % band_rows)
        return fail(PBX_E_BADARG, "owned rows %d+%d: outside the plane or not at a band start", own_y0, own_rows);
    Plane p;
    p.image_id = d->image_id; p.z = d->z; p.c = d->c; p.t = d->t; p.res = d->resolution;
    p.pixel_type = d->pixel_type; p.size_x = d->size_x; p.size_y = d->size_y;
    p.band_y0 = own_y0;
    p.band_rows = own_rows;
    p.sparse_rows = band_rows;
    p.pitch = ((int64_t)d->size_x * bpp + 255) & ~(int64_t)255;
    p.little_endian = d->source == PBX_SRC_HOST ? (d->byte_order == PBX_LITTLE_ENDIAN && bpp > 1) : bpp > 1;
    p.gen_source = d->source;
    p.gen_seed = d->seed;
    p.gen_plane_no = d->plane_no;
    p.bands.resize((size_t)((d->size_y + (int64_t)band_rows - 1) / band_rows));
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    if (int rc = registry_check(ctx, p)) return rc;
    p.state = PS_READY;  // served at once: requests answer NOT_RESIDENT per missing band
    Plane* q = registry_add(ctx, p);
    *plane_id = q->id;
    return PBX_OK;
}

namespace {

// A loading band back to absent (under reg_mu); its HBM goes to `to_free`.
void band_reset_locked(Band& b, std::vector<std::pair<void*, size_t>>& to_free) {
    if (b.dev) to_free.emplace_back(b.dev, b.bytes);
    b.dev = nullptr;
    b.state = BS_ABSENT;
    b.rows_done.clear();
    b.rows_left = 0;
    b.failed = false;
}

// free_planes under reg_mu (the memory goes to the reaper, the bytes stop counting)
void free_planes_locked(pbx_ctx* ctx, const std::vector<std::pair<void*, size_t>>& to_free) {
    for (auto& f : to_free) {
        ctx->reaper.put(f.first);
        ctx->resident_bytes -= f.second;
    }
}

// Rows [y0, y0 + rows) of one band of a sparse plane: the first write of an absent band
// allocates it (within the budget, evicting idle planes / bands), the last one publishes it.
// data == NULL on a generator plane generates the rows on the GPU instead.
int band_write(pbx_ctx* ctx, Plane* q, int32_t y0, int32_t rows, const void* data, uint64_t bytes) {
    if (!q->sparse_rows) return fail(PBX_E_BADARG, "plane %llu is not a sparse plane", (unsigned long long)q->id);
    // any band of the plane: the owned ones, and guest bands that regions straddling the end of
    // the owned rows cover (validate routes a region by its first row)
    if (rows <= 0 || y0 < 0 || (int64_t)y0 + rows > q->size_y)
        return fail(PBX_E_BADARG, "rows %d+%d outside the plane (%d rows)", y0, rows, q->size_y);
    const int32_t k = y0 / q->sparse_rows;
    const int32_t lo = q->band_lo(k), hi = q->band_hi(k);
    if (y0 + rows > hi) return fail(PBX_E_BADARG, "rows %d+%d cross the end of band %d (rows %d..%d)", y0, rows, k, lo, hi);
    const int bpp = bpp_of(q->pixel_type);
    const uint64_t row = (uint64_t)q->size_x * bpp;
    const bool gen = data == nullptr;
    if (gen && q->gen_source == PBX_SRC_HOST) return fail(PBX_E_BADARG, "null data");
    if (!gen && bytes < row * (uint64_t)rows)
        return fail(PBX_E_BADARG, "%llu bytes for %d rows of %llu", (unsigned long long)bytes, rows, (unsigned long long)row);
    if (ensure_device(ctx)) return PBX_E_INTERNAL;
    Band& b = q->bands[(size_t)k];
    bool alloc = false;
    const size_t nbytes = (size_t)q->pitch * (size_t)(hi - lo) + 256;
    std::vector<std::pair<void*, size_t>> stale;
    {
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        if (b.state == BS_READY) return fail(PBX_E_EXISTS, "band %d is resident", k);
        // a load that failed part-way, or whose loader went away, starts over
        if (b.state == BS_LOADING && b.writers == 0 && (b.failed || mono_ns() - b.touched > ctx->stale_ns)) {
            if (!b.failed) b.stale_reset = true;
            band_reset_locked(b, stale);
        }
        if (b.state == BS_ABSENT && b.stale_reset && y0 != lo) {
            free_planes_locked(ctx, stale);
            return fail(PBX_E_INTERNAL, "band %d: its load was idle for more than %lld ms and was reset; "
                        "write it again from row %d", k, (long long)(ctx->stale_ns / 1000000), lo);
        }
        if (b.state == BS_ABSENT) {
            b.stale_reset = false;
            b.state = BS_LOADING;
            b.failed = false;
            b.rows_done.assign((size_t)(hi - lo), 0);
            b.rows_left = (uint32_t)(hi - lo);
            alloc = true;
        } else if (!b.dev || b.failed) {
            free_planes_locked(ctx, stale);
            return fail(PBX_E_EXISTS, "band %d is being allocated (or reset) by another caller", k);
        }
        b.writers++;
        b.touched = mono_ns();
        free_planes_locked(ctx, stale);
    }
    // A failed write fails the whole load: the band is reset (its HBM returned) by the last
    // writer to leave, never under another writer's upload.
    auto leave_failed = [&](int rc) {
        const std::string msg = g_err;
        std::vector<std::pair<void*, size_t>> to_free;
        {
            std::lock_guard<std::mutex> g(ctx->reg_mu);
            b.writers--;
            b.failed = true;
            b.touched = mono_ns();
            if (b.writers == 0) band_reset_locked(b, to_free);
            free_planes_locked(ctx, to_free);
        }
        g_err = msg;
        return rc;
    };
    if (alloc) {
        uint8_t* dev = nullptr;
        if (int rc = plane_alloc(ctx, nbytes, &dev)) return leave_failed(rc);
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        b.dev = dev;
        b.bytes = nbytes;
    }
    hipError_t e = hipSuccess;
    int rc = PBX_OK;
    if (++ctx->band_writes == ctx->fail_band_write_at.load())  // test hook: this write's upload fails
        return leave_failed(fail(PBX_E_INTERNAL, "injected upload failure in band write %llu",
                                 (unsigned long long)ctx->band_writes.load()));
    {
        std::lock_guard<std::mutex> u(ctx->upload_mu);
        if (alloc) e = hipMemsetAsync(b.dev + (size_t)q->pitch * (size_t)(hi - lo), 0, 256, ctx->upload_stream);
        uint8_t* dst = b.dev + (int64_t)(y0 - lo) * q->pitch;
        if (e == hipSuccess && gen) {
            e = launch_gen_plane(ctx->upload_stream, dst, q->pitch, q->size_x, y0, rows, q->pixel_type,
                                 q->gen_source == PBX_SRC_GEN_FAKE ? GEN_FAKE : GEN_NOISE, q->gen_seed,
                                 q->gen_plane_no, q->z, q->c, q->t);
            if (e == hipSuccess) e = hipStreamSynchronize(ctx->upload_stream);
        } else if (e == hipSuccess) {
            rc = upload_rows(ctx, dst, q->pitch, (const uint8_t*)data, row, (uint64_t)rows, ctx->upload_stream);
        }
    }
    if (e != hipSuccess) rc = fail(PBX_E_INTERNAL, "band write: %s", hipGetErrorString(e));
    if (rc) return leave_failed(rc);
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    if (b.failed || b.state != BS_LOADING || b.rows_done.size() != (size_t)(hi - lo)) {
        // another writer failed meanwhile: this load is void; the last writer out resets it
        std::vector<std::pair<void*, size_t>> to_free;
        b.writers--;
        if (b.writers == 0) band_reset_locked(b, to_free);
        free_planes_locked(ctx, to_free);
        return fail(PBX_E_INTERNAL, "band %d: another write of this load failed; load it again", k);
    }
    b.writers--;
    b.touched = mono_ns();
    for (int32_t r = y0 - lo; r < y0 - lo + rows; r++)
        if (!b.rows_done[(size_t)r]) {
            b.rows_done[(size_t)r] = 1;
            b.rows_left--;
        }
    if (b.rows_left == 0 && b.writers == 0) {  // the last write publishes it
        b.rows_done.clear();
        b.rows_done.shrink_to_fit();
        b.state = BS_READY;
        b.last_use = ++ctx->use_tick;
        b.fresh_until = mono_ns() + FRESH_NS;
    }
    return PBX_OK;
}

}  // namespace

int pbx_band_write(pbx_ctx* ctx, uint64_t id, int32_t y0, int32_t rows, const void* data, uint64_t bytes) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    int rc;
    Plane* q = pin_id(ctx, id, 1u << PS_READY, &rc);
    if (!q) return rc == PBX_E_EXISTS ? fail(PBX_E_BADARG, "plane %llu is not a sparse plane", (unsigned long long)id) : rc;
    rc = band_write(ctx, q, y0, rows, data, bytes);
    const std::string msg = g_err;
    unpin_one(ctx, q);
    g_err = msg;
    return rc;
}

int pbx_band_abort(pbx_ctx* ctx, uint64_t id, int32_t y0) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    std::vector<std::pair<void*, size_t>> to_free;
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    auto it = ctx->planes.find(id);
    if (it == ctx->planes.end() || !it->second->indexed) return fail(PBX_E_NOTFOUND, "no plane %llu", (unsigned long long)id);
    Plane* p = it->second;
    if (!p->sparse_rows) return fail(PBX_E_BADARG, "plane %llu is not a sparse plane", (unsigned long long)id);
    if (y0 < 0 || y0 >= p->size_y) return fail(PBX_E_BADARG, "row %d outside the plane", y0);
    Band& b = p->bands[(size_t)(y0 / p->sparse_rows)];
    if (b.state != BS_LOADING) return PBX_OK;
    b.failed = true;  // writers still in flight: the last one out resets the band
    if (b.writers == 0) band_reset_locked(b, to_free);
    free_planes_locked(ctx, to_free);
    return PBX_OK;
}

int pbx_plane_band_info(pbx_ctx* ctx, uint64_t id, int32_t* band_rows, int32_t* nbands, uint8_t* states) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    auto it = ctx->planes.find(id);
    if (it == ctx->planes.end() || !it->second->indexed) return fail(PBX_E_NOTFOUND, "no plane %llu", (unsigned long long)id);
    Plane* p = it->second;
    if (!p->sparse_rows) return fail(PBX_E_BADARG, "plane %llu is not a sparse plane", (unsigned long long)id);
    // bands left loading by a loader that failed or went away read as absent (and give their
    // HBM back): a binding waiting for them loads them again
    std::vector<std::pair<void*, size_t>> stale;
    const int64_t now = mono_ns();
    for (Band& b : p->bands)
        if (b.state == BS_LOADING && b.writers == 0 && (b.failed || now - b.touched > ctx->stale_ns)) {
            if (!b.failed) b.stale_reset = true;
            band_reset_locked(b, stale);
        }
    free_planes_locked(ctx, stale);
    if (band_rows) *band_rows = p->sparse_rows;
    if (nbands) *nbands = (int32_t)p->bands.size();
    if (states)
        for (size_t k = 0; k < p->bands.size(); k++) states[k] = (uint8_t)p->bands[k].state;
    return PBX_OK;
}

int pbx_plane_lookup(pbx_ctx* ctx, int64_t image_id, int32_t z, int32_t c, int32_t t, int32_t level,
                     uint64_t* plane_id, int32_t* state, int32_t* band_y0, int32_t* band_rows) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    auto it = ctx->index.find(std::make_tuple(image_id, z, c, t, level));
    if (it == ctx->index.end()) return fail(PBX_E_NOTFOUND, "no plane registered under that key");
    const Plane* p = ctx->planes.at(it->second);
    if (plane_id) *plane_id = p->id;
    if (state) *state = p->state;
    if (band_y0) *band_y0 = p->band_y0;
    if (band_rows) *band_rows = p->band_rows;
    return PBX_OK;
}

int pbx_image_declare(pbx_ctx* ctx, const pbx_image_desc* d) {
    if (!ctx || !d) return fail(PBX_E_BADARG, "null argument");
    if (!bpp_of(d->pixel_type)) return fail(PBX_E_BADARG, "bad pixel type %d", d->pixel_type);
    if (d->size_x <= 0 || d->size_y <= 0 || d->size_z <= 0 || d->size_c <= 0 || d->size_t_ <= 0 || d->levels <= 0 ||
        d->levels > 64)
        return fail(PBX_E_BADARG, "bad image extents");
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    auto it = ctx->images.find(d->image_id);
    if (it != ctx->images.end()) {
        const Image& I = it->second;
        if (I.declared) {
            if (I.pixel_type != d->pixel_type || I.size_x != d->size_x || I.size_y != d->size_y || I.size_z != d->size_z ||
                I.size_c != d->size_c || I.size_t_ != d->size_t_ || I.nlevels != d->levels)
                return fail(PBX_E_BADARG, "Image:%lld declared differently before", (long long)d->image_id);
            return PBX_OK;
        }
        if (I.planes && I.pixel_type != d->pixel_type)
            return fail(PBX_E_BADARG, "pixel type differs from the registered planes'");
        if (I.level_planes.count(0) && (I.size_x != d->size_x || I.size_y != d->size_y))
            return fail(PBX_E_BADARG, "size differs from the registered full-resolution planes'");
        if (I.levels() > d->levels) return fail(PBX_E_BADARG, "a plane is registered at level %d", I.levels() - 1);
        for (auto& kv : ctx->index) {
            if (std::get<0>(kv.first) != d->image_id) continue;
            const int32_t z = std::get<1>(kv.first), c = std::get<2>(kv.first), t = std::get<3>(kv.first);
            if (z < 0 || z >= d->size_z || c < 0 || c >= d->size_c || t < 0 || t >= d->size_t_)
                return fail(PBX_E_BADARG, "a plane is registered at z=%d c=%d t=%d", z, c, t);
        }
    }
    Image& I = ctx->images[d->image_id];
    I.declared = true;
    I.pixel_type = d->pixel_type;
    I.size_x = d->size_x;
    I.size_y = d->size_y;
    I.size_z = d->size_z;
    I.size_c = d->size_c;
    I.size_t_ = d->size_t_;
    I.nlevels = d->levels;
    return PBX_OK;
}

int pbx_image_release(pbx_ctx* ctx, int64_t image_id) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    std::vector<std::pair<void*, size_t>> to_free;
    {
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        auto im = ctx->images.find(image_id);
        if (im == ctx->images.end()) return fail(PBX_E_NOTFOUND, "Image:%lld unknown", (long long)image_id);
        std::vector<Plane*> ps;
        for (auto& kv : ctx->index)
            if (std::get<0>(kv.first) == image_id) ps.push_back(ctx->planes.at(kv.second));
        for (Plane* p : ps) registry_remove(ctx, p, to_free);
        ctx->images.erase(image_id);
    }
    free_planes(ctx, to_free);
    return PBX_OK;
}

int pbx_set_residency_budget(pbx_ctx* ctx, uint64_t bytes) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    std::vector<std::pair<void*, size_t>> victims;
    {
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        ctx->budget = bytes;
        while (bytes && ctx->resident_bytes > bytes)  // shrink now, as far as idle planes allow
            if (!evict_one_locked(ctx, victims)) break;
    }
    for (auto& v : victims) ctx->reaper.put(v.first);
    return PBX_OK;
}

int pbx_residency_stats_get(pbx_ctx* ctx, pbx_residency_stats* s) {
    if (!ctx || !s) return fail(PBX_E_BADARG, "null argument");
    memset(s, 0, sizeof *s);
    std::lock_guard<std::mutex> g(ctx->reg_mu);
    s->budget = ctx->budget;
    s->resident_bytes = ctx->resident_bytes;
    for (auto& kv : ctx->planes) {
        const Plane* p = kv.second;
        if (!p->indexed) continue;
        if (p->state == PS_EVICTED) s->evicted_planes++;
        else if (p->dev) s->planes++;
        for (const Band& b : p->bands) s->bands += b.state == BS_READY;
    }
    s->evictions = ctx->evictions;
    s->evicted_bytes = ctx->evicted_bytes;
    s->band_evictions = ctx->band_evictions;
    return PBX_OK;
}

int pbx_plane_build_pyramid(pbx_ctx* ctx, uint64_t id, int32_t levels, uint64_t* ids, double* kernel_ms) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    if (levels < 1 || levels > 30) return fail(PBX_E_BADARG, "bad level count %d", levels);
    // the source stays pinned from the lookup through the last kernel: a concurrent
    // pbx_plane_release cannot free it under the downsampling kernels
    int rc;
    Plane* sp = pin_id(ctx, id, 1u << PS_READY, &rc);
    if (!sp) return rc;
    const Plane src = *sp;
    std::vector<Plane> made;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    auto undo = [&](int code) {
        const std::string msg = g_err;
        for (Plane& q : made) plane_free(ctx, q.dev, q.bytes);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        unpin_one(ctx, sp);
        g_err = msg;
        return code;
    };
    if (!src.whole()) return undo(fail(PBX_E_BADARG, "plane %llu is a row band: no pyramid", (unsigned long long)id));
    {
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        for (int32_t k = 1; k <= levels; k++) {
            auto it = ctx->index.find(std::make_tuple(src.image_id, src.z, src.c, src.t, src.res + k));
            if (it != ctx->index.end() && ctx->planes.at(it->second)->state != PS_EVICTED)
                return undo(fail(PBX_E_EXISTS, "resolution %d already registered", src.res + k));
        }
    }
    if (ensure_device(ctx)) return undo(PBX_E_INTERNAL);
    const int bpp = bpp_of(src.pixel_type);
    hipError_t e = hipSuccess;
    if (kernel_ms) {
        e = hipEventCreate(&ev0);
        if (e == hipSuccess) e = hipEventCreate(&ev1);
        if (e != hipSuccess) return undo(fail(PBX_E_INTERNAL, "hipEventCreate: %s", hipGetErrorString(e)));
    }
    Plane prev = src;
    for (int32_t k = 1; k <= levels; k++) {
        Plane p;
        p.image_id = src.image_id; p.z = src.z; p.c = src.c; p.t = src.t;
        p.pixel_type = src.pixel_type;
        p.little_endian = src.little_endian;
        p.size_x = (prev.size_x + 1) / 2;
        p.size_y = (prev.size_y + 1) / 2;
        p.band_rows = p.size_y;
        p.pitch = ((int64_t)p.size_x * bpp + 255) & ~(int64_t)255;
        p.bytes = (size_t)p.pitch * p.size_y + 256;
        if (int rc2 = plane_alloc(ctx, p.bytes, &p.dev)) return undo(rc2);
        p.res = src.res + k;
        made.push_back(p);
        prev = p;
    }
    if (ev0) e = hipEventRecord(ev0, ctx->stream);
    prev = src;
    for (int32_t k = 1; k <= levels && e == hipSuccess; k++) {
        const Plane& p = made[k - 1];
        e = launch_downsample(ctx->stream, prev.dev, prev.pitch, prev.size_x, prev.size_y, p.dev, p.pitch,
                              p.size_x, p.size_y, p.pixel_type, !p.little_endian && bpp > 1);
        if (e == hipSuccess) e = hipMemsetAsync(p.dev + (size_t)p.pitch * p.size_y, 0, 256, ctx->stream);
        prev = p;
    }
    if (ev1 && e == hipSuccess) e = hipEventRecord(ev1, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) return undo(fail(PBX_E_INTERNAL, "downsample: %s", hipGetErrorString(e)));
    if (kernel_ms) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, ev0, ev1);
        *kernel_ms = ms;
    }
    if (int rc2 = registry_insert(ctx, made, ids)) return undo(rc2);  // keys re-checked here
    made.clear();
    return undo(PBX_OK);  // events and the source pin only
}

// ------------------------------------------------------------------ NGFF / Zarr planes
namespace {

uint32_t rd_le32(const uint8_t* p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

// Host plan of one plane's chunks: metadata only (blosc headers, block starts and split
// sizes); every byte of chunk data is decoded on the GPU.  Frame layout: oracle/zarr_oracle.c.
struct ZarrPlan {
    std::vector<ZStream> kind[ZS_NKINDS];  // streams by decoder (enum ZS_*)
    std::vector<ZChunk> chunks;
    uint64_t scratch = 0;
};

int zarr_plan(const pbx_plane_desc* d, const pbx_zarr_chunks* z, int bpp, uint64_t in_base,
              uint32_t plane_idx, ZarrPlan& P) {
    const int64_t gx = (d->size_x + z->chunk_x - 1) / z->chunk_x;
    const int64_t gy = (d->size_y + z->chunk_y - 1) / z->chunk_y;
    const uint64_t cb = (uint64_t)z->chunk_x * z->chunk_y * bpp;
    if (cb > 0x7fffffffull) return fail(PBX_E_BADARG, "chunk of %llu bytes too large", (unsigned long long)cb);
    const uint64_t total = z->offsets[gx * gy];
    for (int64_t i = 0; i < gx * gy; i++) {
        const uint64_t o = z->offsets[i], len = z->offsets[i + 1] - o;
        const uint64_t ob = o + in_base;  // device offset in the launch's upload buffer
        if (z->offsets[i + 1] < o || z->offsets[i + 1] > total)
            return fail(PBX_E_BADARG, "chunk %lld: bad offsets", (long long)i);
        ZChunk c{};
        c.plane = plane_idx;
        c.x0 = (int32_t)((i % gx) * z->chunk_x);
        c.y0 = (int32_t)((i / gx) * z->chunk_y);
        c.nbytes = (uint32_t)cb;
        c.blocksize = (uint32_t)cb;
        c.typesize = 1;
        if (len == 0) {
            c.flags = ZC_MISSING;
            P.chunks.push_back(c);
            continue;
        }
        if (z->codec == PBX_ZARR_RAW) {
            if (len < cb) return fail(PBX_E_BADARG, "chunk %lld: %llu bytes < %llu", (long long)i,
                                      (unsigned long long)len, (unsigned long long)cb);
            c.src = ob;
            c.flags = ZC_INPUT;
            P.chunks.push_back(c);
            continue;
        }
        const uint64_t dst = P.scratch;
        if (z->codec == PBX_ZARR_ZLIB) {
            if (len > 0xffffffffull) return fail(PBX_E_BADARG, "chunk %lld too large", (long long)i);
            P.kind[ZS_ZLIB].push_back(ZStream{ob, dst, (uint32_t)len, (uint32_t)cb, ZS_ZLIB, 0});
            c.src = dst;
            P.chunks.push_back(c);
            P.scratch += (cb + 255) & ~255ull;
            continue;
        }
        // blosc 1.x frame
        const uint8_t* f = z->data + o;
        if (len < 16) return fail(PBX_E_BADARG, "chunk %lld: short blosc header", (long long)i);
        const uint32_t ver = f[0], flags = f[2], ts = f[3] ? f[3] : 1;
        const uint32_t nbytes = rd_le32(f + 4), bs = rd_le32(f + 8), cbytes = rd_le32(f + 12);
        if (ver != 2) return fail(PBX_E_BADARG, "chunk %lld: blosc format version %u (c-blosc 1.x writes 2)", (long long)i, ver);
        if (nbytes != cb) return fail(PBX_E_BADARG, "chunk %lld: blosc nbytes %u != chunk bytes %llu",
                                      (long long)i, nbytes, (unsigned long long)cb);
        if (cbytes > len || cbytes < 16) return fail(PBX_E_BADARG, "chunk %lld: blosc cbytes %u", (long long)i, cbytes);
        if (flags & 0x2) {  // memcpyed: the unshuffled chunk follows the header
            if (16ull + nbytes > cbytes) return fail(PBX_E_BADARG, "chunk %lld: short memcpyed frame", (long long)i);
            c.src = ob + 16;
            c.flags = ZC_INPUT;
            P.chunks.push_back(c);
            continue;
        }
        const uint32_t codec = flags >> 5;  // 0 blosclz, 1 lz4 / lz4hc, 2 snappy, 3 zlib, 4 zstd
        if (codec != 0 && codec != 1 && codec != 3 && codec != 4)
            return fail(PBX_E_BADARG, "chunk %lld: blosc codec %u not supported (blosclz/lz4/lz4hc/zlib/zstd)",
                        (long long)i, codec);
        static const uint32_t kind_of[5] = {ZS_BLOSCLZ, ZS_LZ4, 0, ZS_ZLIB, ZS_ZSTD};
        if (bs == 0 || bs > nbytes || (bs % ts)) return fail(PBX_E_BADARG, "chunk %lld: blosc blocksize %u", (long long)i, bs);
        const uint32_t nblocks = (nbytes + bs - 1) / bs, leftover = nbytes % bs;
        if (16ull + 4ull * nblocks > cbytes) return fail(PBX_E_BADARG, "chunk %lld: short block table", (long long)i);
        for (uint32_t b = 0; b < nblocks; b++) {
            const bool is_left = leftover && b == nblocks - 1;
            const uint32_t bsize = is_left ? leftover : bs;
            const bool split = !(flags & 0x10) && ts <= 16 && bsize / ts >= 128 && !is_left;
            const uint32_t nsp = split ? ts : 1, neb = bsize / nsp;
            if (neb * nsp != bsize) return fail(PBX_E_BADARG, "chunk %lld: block %u not a multiple of typesize", (long long)i, b);
            uint64_t pos = rd_le32(f + 16 + 4 * b);
            for (uint32_t s = 0; s < nsp; s++) {
                if (pos + 4 > cbytes) return fail(PBX_E_BADARG, "chunk %lld: block %u truncated", (long long)i, b);
                const uint32_t cs = rd_le32(f + pos);
                pos += 4;
                if (pos + cs > cbytes || cs > neb || cs == 0)
                    return fail(PBX_E_BADARG, "chunk %lld: block %u split %u size %u", (long long)i, b, s, cs);
                const uint32_t k = cs == neb ? ZS_COPY : kind_of[codec];
                P.kind[k].push_back(ZStream{ob + pos, dst + (uint64_t)b * bs + (uint64_t)s * neb, cs, neb, k, 0});
                pos += cs;
            }
        }
        c.src = dst;
        c.blocksize = bs;
        if (flags & 0x4) {  // bit shuffle (takes precedence over the byte-shuffle bit)
            c.flags |= ZC_BITSHUF;
            c.typesize = ts;
        } else {
            c.typesize = (flags & 0x1) ? ts : 1;
        }
        P.chunks.push_back(c);
        P.scratch += (cb + 255) & ~255ull;
    }
    return PBX_OK;
}

}  // namespace

int pbx_planes_register_zarr(pbx_ctx* ctx, uint64_t n, const pbx_plane_desc* ds,
                             const pbx_zarr_chunks* zs, uint64_t* plane_ids, double* kernel_ms) {
    if (!ctx || !ds || !zs || !plane_ids || n == 0) return fail(PBX_E_BADARG, "null argument");
    std::vector<std::tuple<int64_t, int32_t, int32_t, int32_t, int32_t>> keys;
    for (uint64_t k = 0; k < n; k++) {
        const pbx_plane_desc* d = &ds[k];
        const pbx_zarr_chunks* z = &zs[k];
        if (!z->offsets || (!z->data && z->codec != PBX_ZARR_RAW)) return fail(PBX_E_BADARG, "null argument");
        if (!bpp_of(d->pixel_type)) return fail(PBX_E_BADARG, "bad pixel type %d", d->pixel_type);
        if (d->size_x <= 0 || d->size_y <= 0) return fail(PBX_E_BADARG, "bad plane size");
        if (d->resolution < 0) return fail(PBX_E_BADARG, "bad resolution");
        if (z->chunk_x <= 0 || z->chunk_y <= 0) return fail(PBX_E_BADARG, "bad chunk shape");
        if (z->codec < PBX_ZARR_RAW || z->codec > PBX_ZARR_ZLIB) return fail(PBX_E_BADARG, "bad codec %d", z->codec);
        keys.emplace_back(d->image_id, d->z, d->c, d->t, d->resolution);
    }
    {
        auto sorted = keys;
        std::sort(sorted.begin(), sorted.end());
        if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end())
            return fail(PBX_E_BADARG, "the same plane twice in one call");
        for (uint64_t a = 0; a < n; a++)  // planes of one image agree with each other too
            for (uint64_t b = a + 1; b < n; b++)
                if (ds[a].image_id == ds[b].image_id &&
                    (ds[a].pixel_type != ds[b].pixel_type ||
                     (ds[a].resolution == 0 && ds[b].resolution == 0 &&
                      (ds[a].size_x != ds[b].size_x || ds[a].size_y != ds[b].size_y))))
                    return fail(PBX_E_BADARG, "planes of image %lld disagree on type or size",
                                (long long)ds[a].image_id);
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        for (uint64_t k = 0; k < n; k++) {  // early: a taken key fails before any decoding
            Plane p;
            p.image_id = ds[k].image_id; p.z = ds[k].z; p.c = ds[k].c; p.t = ds[k].t;
            p.res = ds[k].resolution; p.pixel_type = ds[k].pixel_type;
            p.size_x = ds[k].size_x; p.size_y = ds[k].size_y;
            if (int rc = registry_check(ctx, p)) return rc;
        }
    }
    // host plan: metadata of every chunk of every plane, one upload buffer, one scratch
    ZarrPlan P;
    std::vector<uint64_t> in_base(n + 1, 0);
    int32_t max_cy = 0;
    for (uint64_t k = 0; k < n; k++) {
        const pbx_plane_desc* d = &ds[k];
        const pbx_zarr_chunks* z = &zs[k];
        const int64_t gx = (d->size_x + z->chunk_x - 1) / z->chunk_x, gy = (d->size_y + z->chunk_y - 1) / z->chunk_y;
        if (int rc = zarr_plan(d, z, bpp_of(d->pixel_type), in_base[k], (uint32_t)k, P)) return rc;
        in_base[k + 1] = in_base[k] + ((z->offsets[gx * gy] + 15) & ~15ull);
        max_cy = std::max(max_cy, z->chunk_y);
    }
    if (ensure_device(ctx)) return PBX_E_INTERNAL;
    const uint64_t in_bytes = in_base[n];
    std::vector<Plane> ps(n);
    std::vector<ZPlane> zp(n);
    for (uint64_t k = 0; k < n; k++) {
        const pbx_plane_desc* d = &ds[k];
        const int bpp = bpp_of(d->pixel_type);
        Plane& p = ps[k];
        p.image_id = d->image_id; p.z = d->z; p.c = d->c; p.t = d->t; p.res = d->resolution;
        p.pixel_type = d->pixel_type; p.size_x = d->size_x; p.size_y = d->size_y;
        p.little_endian = d->byte_order == PBX_LITTLE_ENDIAN && bpp > 1;
        p.pitch = ((int64_t)d->size_x * bpp + 255) & ~(int64_t)255;
        p.bytes = (size_t)p.pitch * d->size_y + 256;
        p.band_rows = d->size_y;
        uint64_t fill = 0;  // fill bytes in the stored byte order
        for (int j = 0; j < bpp; j++) {
            const uint64_t byte = (zs[k].fill_bits >> (8 * j)) & 0xff;
            fill |= byte << (8 * (p.little_endian || bpp == 1 ? j : bpp - 1 - j));
        }
        zp[k] = ZPlane{nullptr, p.pitch, d->size_x, d->size_y, zs[k].chunk_x, zs[k].chunk_y,
                       (uint32_t)bpp, 0, fill};
    }
    uint32_t counts[ZS_NKINDS], nstreams = 0;
    std::vector<ZStream> all;
    for (uint32_t k = 0; k < ZS_NKINDS; k++) {
        counts[k] = (uint32_t)P.kind[k].size();
        nstreams += counts[k];
        all.insert(all.end(), P.kind[k].begin(), P.kind[k].end());
    }
    uint8_t *d_in = nullptr, *d_scr = nullptr, *d_lit = nullptr;
    ZStream* d_st = nullptr;
    ZChunk* d_ch = nullptr;
    ZPlane* d_pl = nullptr;
    uint32_t* d_err = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    // launch scratch (input, decoded chunks, tables) comes from the context's device pool and
    // goes back to it: only the planes themselves are new allocations
    auto cleanup = [&](bool planes_too) {
        // queued copies, memsets or decoders may still write these blocks on an error path;
        // the pool hands them to other streams' batches as soon as they are back
        (void)hipStreamSynchronize(ctx->stream);
        for (void* q : {(void*)d_in, (void*)d_scr, (void*)d_lit, (void*)d_st, (void*)d_ch, (void*)d_pl, (void*)d_err})
            if (q) ctx->dpool.put(q);
        for (auto& x : ev) if (x) (void)hipEventDestroy(x);
        if (planes_too)
            for (Plane& p : ps) plane_free(ctx, p.dev, p.bytes);
    };
    hipError_t e = hipSuccess;
    auto dget = [&](auto*& ptr, size_t bytes) {
        if (e != hipSuccess) return;
        ptr = (std::remove_reference_t<decltype(ptr)>)ctx->dpool.get(std::max<size_t>(bytes, 256), &e);
    };
    for (uint64_t k = 0; k < n; k++) {
        if (int rc = plane_alloc(ctx, ps[k].bytes, &ps[k].dev)) {
            const std::string msg = g_err;
            cleanup(true);
            g_err = msg;
            return rc;
        }
        zp[k].dev = ps[k].dev;
    }
    dget(d_in, in_bytes + 4096);  // decoder window over-read slack
    if (P.scratch) dget(d_scr, P.scratch);
    if (counts[ZS_ZSTD]) dget(d_lit, zstd_scratch_bytes(counts[ZS_ZSTD]));
    if (nstreams) dget(d_st, sizeof(ZStream) * nstreams);
    dget(d_ch, sizeof(ZChunk) * P.chunks.size());
    dget(d_pl, sizeof(ZPlane) * n);
    dget(d_err, sizeof(uint32_t) * (nstreams + 1));
    for (auto& x : ev) if (e == hipSuccess) e = hipEventCreate(&x);
    if (e != hipSuccess) {
        cleanup(true);
        return fail(PBX_E_INTERNAL, "zarr decode: %s", hipGetErrorString(e));
    }
    for (uint64_t k = 0; k < n && e == hipSuccess; k++) {
        const uint64_t len = in_base[k + 1] - in_base[k];
        const int64_t gx = (ds[k].size_x + zs[k].chunk_x - 1) / zs[k].chunk_x;
        const int64_t gy = (ds[k].size_y + zs[k].chunk_y - 1) / zs[k].chunk_y;
        const uint64_t used = zs[k].offsets[gx * gy];
        if (used) {
            if (int rc = upload_staged(ctx, d_in + in_base[k], zs[k].data, used, ctx->stream)) {
                cleanup(true);
                return rc;
            }
        }
        if (len > used) e = hipMemsetAsync(d_in + in_base[k] + used, 0, len - used, ctx->stream);
    }
    if (e == hipSuccess) e = hipMemsetAsync(d_in + in_bytes, 0, 4096, ctx->stream);
    if (e == hipSuccess && nstreams)
        e = hipMemcpyAsync(d_st, all.data(), sizeof(ZStream) * nstreams, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(d_ch, P.chunks.data(), sizeof(ZChunk) * P.chunks.size(), hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(d_pl, zp.data(), sizeof(ZPlane) * n, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipMemsetAsync(d_err, 0, sizeof(uint32_t) * (nstreams + 1), ctx->stream);
    if (e == hipSuccess) e = hipEventRecord(ev[0], ctx->stream);
    if (e == hipSuccess)
        e = launch_zarr_decode(ctx->stream, d_st, counts, d_in, d_scr, d_lit, d_err);
    if (e == hipSuccess) e = hipEventRecord(ev[1], ctx->stream);
    if (e == hipSuccess)
        e = launch_zarr_place(ctx->stream, d_ch, (uint32_t)P.chunks.size(), d_pl, max_cy, d_scr, d_in);
    if (e == hipSuccess) e = hipEventRecord(ev[2], ctx->stream);
    for (uint64_t k = 0; k < n && e == hipSuccess; k++)
        e = hipMemsetAsync(ps[k].dev + (size_t)ps[k].pitch * ps[k].size_y, 0, 256, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    std::vector<uint32_t> err(nstreams + 1, 0);
    if (e == hipSuccess && nstreams)
        e = hipMemcpy(err.data(), d_err, sizeof(uint32_t) * nstreams, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        cleanup(true);
        return fail(PBX_E_INTERNAL, "zarr decode: %s", hipGetErrorString(e));
    }
    for (uint32_t s = 0; s < nstreams; s++)
        if (err[s]) {
            static const char* names[ZS_NKINDS] = {"lz4", "zlib", "stored", "blosclz", "zstd"};
            uint32_t k = 0, first = 0;
            while (s >= first + counts[k]) first += counts[k++];
            cleanup(true);
            return fail(PBX_E_BADARG, "corrupt chunk stream %u (%s, decoder code %u)", s, names[k], err[s]);
        }
    if (kernel_ms) {
        float a = 0, b = 0;
        (void)hipEventElapsedTime(&a, ev[0], ev[1]);
        (void)hipEventElapsedTime(&b, ev[1], ev[2]);
        kernel_ms[0] = a;
        kernel_ms[1] = b;
    }
    cleanup(false);
    if (int rc = registry_insert(ctx, ps, plane_ids)) {  // keys re-checked at insertion
        const std::string msg = g_err;
        for (Plane& p : ps) plane_free(ctx, p.dev, p.bytes);
        g_err = msg;
        return rc;
    }
    return PBX_OK;
}

int pbx_plane_register_zarr(pbx_ctx* ctx, const pbx_plane_desc* d, const pbx_zarr_chunks* z,
                            uint64_t* plane_id, double* kernel_ms) {
    return pbx_planes_register_zarr(ctx, 1, d, z, plane_id, kernel_ms);
}

int pbx_plane_release(pbx_ctx* ctx, uint64_t id) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    std::vector<std::pair<void*, size_t>> to_free;
    {
        std::lock_guard<std::mutex> g(ctx->reg_mu);
        auto it = ctx->planes.find(id);
        if (it == ctx->planes.end() || !it->second->indexed)
            return fail(PBX_E_NOTFOUND, "no plane %llu", (unsigned long long)id);
        // batches planned before this call hold pins: the HBM goes with their last one
        registry_remove(ctx, it->second, to_free);
    }
    free_planes(ctx, to_free);
    return PBX_OK;
}

int pbx_plane_read_be(pbx_ctx* ctx, uint64_t id, void* out, uint64_t bytes) {
    if (!ctx || !out) return fail(PBX_E_BADARG, "null argument");
    int rc;
    Plane* p = pin_id(ctx, id, 1u << PS_READY, &rc);
    if (!p) return rc;
    rc = [&]() -> int {
        if (p->sparse_rows) return fail(PBX_E_BADARG, "plane %llu is a sparse plane", (unsigned long long)id);
        const int bpp = bpp_of(p->pixel_type);
        const int64_t row = (int64_t)p->size_x * bpp;
        const int64_t rows = p->band_rows;  // a band plane: its rows only
        if (bytes < (uint64_t)row * rows) return fail(PBX_E_BADARG, "buffer too small");
        if (ensure_device(ctx)) return PBX_E_INTERNAL;
        HIP_TRY(hipMemcpy2D(out, row, p->dev, p->pitch, row, rows, hipMemcpyDeviceToHost));
        if (p->little_endian) {
            uint8_t* b = (uint8_t*)out;
            for (int64_t i = 0; i < row * rows; i += bpp) std::reverse(b + i, b + i + bpp);
        }
        return PBX_OK;
    }();
    const std::string msg = g_err;
    unpin_one(ctx, p);
    g_err = msg;
    return rc;
}

int pbx_batch_plan(pbx_ctx* ctx, const pbx_tile_req* reqs, uint64_t n, pbx_batch** out) {
    if (!ctx || !out || (!reqs && n)) return fail(PBX_E_BADARG, "null argument");
    if (n > (1u << 26)) return fail(PBX_E_BADARG, "batch too large");
    pbx_batch* b = new pbx_batch();
    b->reqs.assign(reqs, reqs + n);
    b->status.resize(n);
    b->w.resize(n);
    b->h.resize(n);
    const int filter = ctx->cfg.png_filter;
    const bool tiff_deflate = ctx->cfg.tiff_deflate != 0;
    const int32_t tiff_tile = ctx->cfg.tiff_tile;
    // deflate sub-tiles of a tiled TIFF stay consecutive (one response = one run of the
    // deflate arena): they go to k_filter, after the other banded tiles
    std::vector<TileDesc> dt_direct, dt_rows, dt_filt2, dt_filt3, dt_band, dt_tiled;
    std::vector<uint32_t> req_direct, req_rows, req_filt2, req_filt3, req_band, req_tiled;
    static const bool use_f3 = !getenv("PBX_FILTER3") || atoi(getenv("PBX_FILTER3")) != 0;
    for (uint64_t i = 0; i < n; i++) {
        const pbx_tile_req& r = reqs[i];
        Plane* pp = nullptr;
        int32_t w = 0, h = 0, kr[2] = {-1, -1};
        const int st = validate(ctx, r, w, h, pp, true, kr);
        b->status[i] = st;
        b->w[i] = w;
        b->h[i] = h;
        if (st != PBX_OK) continue;
        if (!b->pins.empty() && b->pins.back().first == pp) b->pins.back().second++;
        else b->pins.emplace_back(pp, 1);
        const Plane& pl = *pp;  // pinned until pbx_batch_destroy; its geometry never changes
        const int bpp = bpp_of(pl.pixel_type);
        TileDesc d;
        memset(&d, 0, sizeof d);
        d.plane = pl.base();
        d.pitch = pl.pitch;
        d.x = r.x; d.y = r.y; d.w = w; d.h = h;
        d.bpp = bpp; d.lbpp = log2i(bpp);
        d.pixel_type = pl.pixel_type;
        d.flags = pl.little_endian ? TF_SWAP : 0u;
        if (pl.sparse_rows) {  // its bands are pinned (validate); the kernels read one band, or the bridge
            for (int32_t k = kr[0]; k <= kr[1]; k++) b->band_pins.emplace_back(pp, k);
            if (kr[0] == kr[1]) {
                d.plane = pl.band_base(kr[0]);
            } else {
                pbx_batch::Bridge g;
                g.p = pp;
                g.x = r.x; g.y = r.y; g.w = w; g.h = h; g.k0 = kr[0]; g.k1 = kr[1];
                g.xo = ((int64_t)r.x * bpp) & 255;  // same alignment as in the plane rows
                g.bp = (g.xo + (int64_t)w * bpp + 32 + 255) & ~(int64_t)255;  // + vector over-read (gload16u: 31 B)
                g.off = b->bridge_bytes;
                b->bridge_bytes += (uint64_t)g.bp * (uint64_t)h + 256;
                b->bridges.push_back(g);
                d.plane = (const uint8_t*)(uintptr_t)((int64_t)g.off + g.xo - (int64_t)r.y * g.bp - (int64_t)r.x * bpp);
                d.pitch = g.bp;
                d.flags |= TF_BRIDGE;
            }
        }
        const uint64_t tile_bytes = (uint64_t)w * h * bpp;
        b->in_bytes += tile_bytes;
        const bool deflate = r.format == PBX_FMT_PNG || (r.format == PBX_FMT_TIF && tiff_deflate);
        if (r.format == PBX_FMT_TIF && tiff_tile) {
            // Tiled TIFF: the region as ntx x nty sub-tiles of T x T samples (edge ones
            // zero-padded), each raw or its own zlib stream, behind one header
            const uint32_t T = (uint32_t)tiff_tile;
            const uint32_t ntx = ((uint32_t)w + T - 1) / T, nty = ((uint32_t)h + T - 1) / T;
            const uint64_t nsub = (uint64_t)ntx * nty, sub = (uint64_t)T * T * bpp;
            const uint64_t D = tiff_tiled_data_offset(nsub);
            // The response must fit a Java byte[] (the reference's int tileSize rule, :100-103:
            // past 2^31-1 bytes getTile returns null -> 404); zero-padding the edge sub-tiles
            // can push it past the unpadded tile's size, and a deflated sub-tile is at most its
            // stored form (5 bytes per 16 KiB block) plus the zlib framing.
            const uint64_t sub_max = deflate ? sub + 5 * ((sub + 16383) / 16384) + 64 : sub;
            if (D + nsub * sub_max > 2147483647ull) {
                b->status[i] = fail(PBX_E_NOTFOUND, "tiled TIFF response over 2^31-1 bytes");
                b->in_bytes -= tile_bytes;
                continue;
            }
            TiledHdr th;
            memset(&th, 0, sizeof th);
            th.n = (uint32_t)nsub;
            th.w = (uint32_t)w; th.h = (uint32_t)h; th.t = T; th.bpp = (uint32_t)bpp;
            th.sf = tiff_sample_format(pl.pixel_type);
            th.comp = deflate ? 8u : 1u;
            if (!deflate) {
                th.off = b->fixed_bytes;
                b->fixed_bytes += (D + nsub * sub + 255) & ~255ull;
            } else {
                th.first = (uint32_t)dt_tiled.size();  // rebased below
            }
            d.flags |= TF_TIFF | TF_TILED;
            for (uint32_t ty = 0; ty < nty; ty++)
                for (uint32_t tx = 0; tx < ntx; tx++) {
                    TileDesc s = d;
                    const uint32_t k = ty * ntx + tx;
                    s.x = r.x + (int32_t)(tx * T);
                    s.y = r.y + (int32_t)(ty * T);
                    s.w = s.h = (int32_t)T;
                    const uint32_t vw = std::min<uint32_t>(T, (uint32_t)w - tx * T);
                    const uint32_t vh = std::min<uint32_t>(T, (uint32_t)h - ty * T);
                    if (vw < T || vh < T) { s.vw = vw; s.vh = vh; }
                    s.tiff_hdr = k == 0 ? (uint32_t)D : 0u;
                    if (!deflate) {
                        s.rows_per_blk = std::max<uint32_t>(1, (uint32_t)(16384 / (T * bpp)));
                        s.blk_first = b->ext_blocks;
                        b->ext_blocks += (T + s.rows_per_blk - 1) / s.rows_per_blk;
                        s.out_off = th.off + D + k * sub;
                        b->ft.push_back(s);
                        b->ext_unaligned |= !ext_aligned(s);
                        b->ft_req.push_back((uint32_t)i);
                    } else {
                        s.filter = 0;
                        s.rowlen = T * (uint32_t)bpp;
                        s.stream_len = (uint64_t)T * s.rowlen;
                        dt_tiled.push_back(s);
                        req_tiled.push_back((uint32_t)i);
                    }
                }
            b->th.push_back(th);
            b->th_req.push_back((uint32_t)i);
            continue;
        }
        if (!deflate) {
            if (r.format == PBX_FMT_TIF) d.flags |= TF_TIFF;
            const uint32_t rb = (uint32_t)w * bpp;
            d.rows_per_blk = std::max<uint32_t>(1, (uint32_t)(ext_blk_bytes(ext_aligned(d)) / std::max<uint32_t>(rb, 1)));
            const uint32_t blks = (uint32_t)((h + d.rows_per_blk - 1) / d.rows_per_blk);
            d.blk_first = b->ext_blocks;
            b->ext_blocks += blks;
            d.out_off = b->fixed_bytes;
            b->fixed_bytes += ((r.format == PBX_FMT_TIF ? TIFF_DATA_OFFSET : 0) + tile_bytes + 255) & ~255ull;
            b->ft.push_back(d);
            b->ext_unaligned |= !ext_aligned(d);
            b->ft_req.push_back((uint32_t)i);
        } else {
            if (r.format == PBX_FMT_PNG) {
                d.flags |= TF_PNGROWS;
                if (pl.pixel_type == PBX_INT8 || pl.pixel_type == PBX_INT16) d.flags |= TF_FLIP;
                d.filter = filter;
                if (filter == PBX_FILTER_ADAPTIVE) {
                    b->adaptive = true;
                    b->adaptive_max_rb = std::max<uint32_t>(b->adaptive_max_rb, (uint32_t)w * bpp);
                }
                d.rowlen = 1 + (uint32_t)w * bpp;
            } else {
                d.flags |= TF_TIFF;
                d.filter = 0;
                d.rowlen = (uint32_t)w * bpp;
            }
            d.stream_len = (uint64_t)h * d.rowlen;
            // Filter-None rows from 16-byte-aligned source rows are read by k_lz77 straight
            // from the plane (TF_DIRECT: no k_rows; k_lz77 writes the stream for k_encode);
            // cfg.stage_rows routes them through k_rows (vector funnel copy) instead.
            // Filtered or odd-shaped tiles go to the banded k_filter.
            // (k_rows reads source rows of any alignment; k_lz77's direct fill needs them aligned)
            const uint32_t rb = (uint32_t)w * bpp;
            const bool rows_ok = d.filter == 0 && d.rowlen >= 32 && rb <= ROWS_MAX_RB;
            const bool aligned = ((uint64_t)d.x * bpp % 16) == 0;
            // filtered PNG rows of whole dwords: dword-wide filter arithmetic (k_filter2)
            const bool filt2_ok = (d.flags & TF_PNGROWS) && d.filter != 0 && rb % 4 == 0 && rb >= 16 &&
                                  rb <= filter2_max_rb() && ((uint64_t)d.x * bpp % 16) == 0;
            // filtered PNG rows of whole 16-byte chunks: the streaming one-wave-per-run k_filter3
            const bool filt3_ok = use_f3 && filt2_ok && rb % 16 == 0 && rb <= filter3_max_rb();
            // adaptive tiles of the same geometry: direct when their tile mode says None
            if (d.filter == PBX_FILTER_ADAPTIVE && d.rowlen >= 32 && rb <= ROWS_MAX_RB && aligned && bpp <= 4 &&
                !ctx->cfg.stage_rows)
                d.flags |= TF_DIRECT_OK;
            if (rows_ok && aligned && bpp <= 4 && !ctx->cfg.stage_rows) {
                d.flags |= TF_DIRECT;
                dt_direct.push_back(d);
                req_direct.push_back((uint32_t)i);
            } else if (filt3_ok) {
                dt_filt3.push_back(d);
                req_filt3.push_back((uint32_t)i);
            } else if (filt2_ok) {
                dt_filt2.push_back(d);
                req_filt2.push_back((uint32_t)i);
            } else {
                (rows_ok ? dt_rows : dt_band).push_back(d);
                (rows_ok ? req_rows : req_band).push_back((uint32_t)i);
            }
        }
    }
    b->ndirect_tiles = (uint32_t)dt_direct.size();
    b->nrows_tiles = (uint32_t)dt_rows.size();
    b->dt = std::move(dt_direct);
    b->dt.insert(b->dt.end(), dt_rows.begin(), dt_rows.end());
    b->nfilt2_tiles = (uint32_t)dt_filt2.size();
    b->dt.insert(b->dt.end(), dt_filt2.begin(), dt_filt2.end());
    b->nfilt3_tiles = (uint32_t)dt_filt3.size();
    b->dt.insert(b->dt.end(), dt_filt3.begin(), dt_filt3.end());
    b->dt.insert(b->dt.end(), dt_band.begin(), dt_band.end());
    b->dt.insert(b->dt.end(), dt_tiled.begin(), dt_tiled.end());
    b->dt_req = std::move(req_direct);
    b->dt_req.insert(b->dt_req.end(), req_rows.begin(), req_rows.end());
    b->dt_req.insert(b->dt_req.end(), req_filt2.begin(), req_filt2.end());
    b->dt_req.insert(b->dt_req.end(), req_filt3.begin(), req_filt3.end());
    b->dt_req.insert(b->dt_req.end(), req_band.begin(), req_band.end());
    b->dt_req.insert(b->dt_req.end(), req_tiled.begin(), req_tiled.end());
    const uint32_t tiled0 = (uint32_t)(b->dt.size() - dt_tiled.size());
    for (TiledHdr& th : b->th)
        if (th.comp == 8) th.first += tiled0;
    for (size_t k = 0; k < b->dt.size(); k++) {
        TileDesc& d = b->dt[k];
        deflate_split(d.stream_len, d.seg_count, d.seg_len);
        d.rowlen_rcp = recip32(d.rowlen);
        d.seg_first = b->nseg;
        b->nseg += d.seg_count;
        d.hblk_first = b->nblk;
        b->nblk += tile_blocks(d.seg_count, PBX_TILE_BLK_CAP(d));
        b->stream_bytes += d.stream_len;
        b->png_cap += ((uint64_t)TIFF_DATA_OFFSET + d.tiff_hdr + 128 + d.stream_len + 16ull * d.seg_count + 255) &
                      ~255ull;
        d.out_off = b->stream_cap;  // the tile's filtered stream in the stream buffer
        b->stream_cap += (d.stream_len + 256 + 255) & ~255ull;
        if (k < b->ndirect_tiles) continue;  // k_lz77 assembles it from the plane
        if (k < b->ndirect_tiles + b->nrows_tiles) {
            d.blk_first = b->rows_blocks;
            b->rows_blocks += rows_blocks_for((uint32_t)d.h);
            b->rows_max_rb = std::max<uint32_t>(b->rows_max_rb, d.rowlen - ((d.flags & TF_PNGROWS) ? 1u : 0u));
        } else if (k < b->ndirect_tiles + b->nrows_tiles + b->nfilt2_tiles) {
            d.blk_first = b->filt2_blocks;
            b->filt2_blocks += (uint32_t)((d.h + filter2_band_rows() - 1) / filter2_band_rows());
            b->filt2_max_rb = std::max<uint32_t>(b->filt2_max_rb, d.rowlen - 1);
        } else if (k < b->ndirect_tiles + b->nrows_tiles + b->nfilt2_tiles + b->nfilt3_tiles) {
            d.blk_first = b->filt3_waves;  // first wave (run of rows) of the tile
            b->filt3_waves += (uint32_t)((d.h + filter3_run_rows(d.filter) - 1) / filter3_run_rows(d.filter));
            b->filt3_max_rb = std::max<uint32_t>(b->filt3_max_rb, d.rowlen - 1);
            b->filt3_filter = d.filter;
        } else {
            d.blk_first = b->filt_blocks;
            b->filt_blocks += (uint32_t)((d.h + filter_band_rows() - 1) / filter_band_rows());
        }
    }
    *out = b;
    return PBX_OK;
}

int pbx_batch_launch(pbx_ctx* ctx, pbx_batch* b) {
    if (!ctx || !b) return fail(PBX_E_BADARG, "null argument");
    std::lock_guard<std::mutex> run(ctx->run_mu);  // launches (and the stream turn) in order
    return batch_launch(ctx, b, true, false);
}

// overlap: the caller pipelines batches (pbx_batch_launch, pbx_submit), so a batch with
// deflate work goes to the next of the kernel streams, staggered behind the previous one;
// otherwise (synchronous calls, the coalescer, raw/TIFF-only batches) it runs on `stream`.
// fetch_follows: the results go to the host (pbx_batch_fetch): the tile offsets are read back
// by the kernel stream itself at the end of the launch, so the fetch needs no round trip for
// them before its data copy (the served path's per-batch latency).
static int batch_launch(pbx_ctx* ctx, pbx_batch* b, bool overlap, bool fetch_follows) {
    if (!ctx || !b) return fail(PBX_E_BADARG, "null argument");
    if (ensure_device(ctx)) return PBX_E_INTERNAL;
    hipError_t err = hipSuccess;
    auto dget = [&](void*& p, size_t n) -> bool {
        if (p) return true;
        p = ctx->dpool.get(std::max<size_t>(n, 256), &err);
        return p != nullptr;
    };
    const uint32_t nft = (uint32_t)b->ft.size(), ndt = (uint32_t)b->dt.size(), nth = (uint32_t)b->th.size();
    const size_t ft_bytes = nft * sizeof(TileDesc), dt_bytes = ndt * sizeof(TileDesc),
                 th_bytes = nth * sizeof(TiledHdr);
    const size_t offs_at = (ft_bytes + dt_bytes + th_bytes + 15) & ~(size_t)15;
    if (b->bridge_bytes && !dget(b->d_bridge, b->bridge_bytes))
        return fail(PBX_E_INTERNAL, "device alloc: %s", hipGetErrorString(err));
    if (!b->h_desc) {
        b->h_desc = ctx->hpool.get(offs_at + (ndt + 1) * sizeof(uint64_t) + 256, &err);
        if (!b->h_desc) return fail(PBX_E_INTERNAL, "pinned alloc: %s", hipGetErrorString(err));
        b->h_offs_pin = (uint64_t*)((uint8_t*)b->h_desc + offs_at);
        if (nft) memcpy(b->h_desc, b->ft.data(), ft_bytes);
        if (ndt) memcpy((uint8_t*)b->h_desc + ft_bytes, b->dt.data(), dt_bytes);
        if (nth) memcpy((uint8_t*)b->h_desc + ft_bytes + dt_bytes, b->th.data(), th_bytes);
        if (b->bridge_bytes) {  // bridged regions: their plane base is relative to the bridge buffer
            TileDesc* td = (TileDesc*)b->h_desc;
            for (uint32_t k = 0; k < nft + ndt; k++)
                if (td[k].flags & TF_BRIDGE) {
                    td[k].plane = (const uint8_t*)b->d_bridge + (intptr_t)td[k].plane;
                    td[k].flags &= ~(uint32_t)TF_BRIDGE;
                }
        }
    }
    const size_t ns = b->nseg;
    b->lite = fetch_follows && !overlap;
    if (b->lite && !b->h_zc && !b->d_fixed && !b->d_png && ctx->zc_max) {
        const uint64_t at = (b->fixed_bytes + 255) & ~(uint64_t)255;
        if (at + b->png_cap + 256 <= ctx->zc_max) {
            b->h_zc = ctx->hpool.get(at + b->png_cap + 256, &err);
            void* dp = nullptr;
            if (b->h_zc && hipHostGetDevicePointer(&dp, b->h_zc, 0) == hipSuccess) {
                b->d_fixed = dp;
                b->d_png = (uint8_t*)dp + at;
                b->zc_png_at = at | 1u;  // (bit 0: the block is in use even when at == 0)
            } else if (b->h_zc) {
                ctx->hpool.put(b->h_zc);
                b->h_zc = nullptr;
            }
        }
    }
    if (!dget(b->d_ft, ft_bytes) || !dget(b->d_dt, dt_bytes) || !dget(b->d_fixed, b->fixed_bytes) ||
        !dget(b->d_stream, b->stream_cap) || !dget(b->d_info, ns * sizeof(SegInfo)) ||
        !dget(b->d_hist, ns * HIST_WORDS * 4) || !dget(b->d_mrec, ns * MREC_WORDS * 4) ||
        !dget(b->d_codes, (size_t)b->nblk * CODE_WORDS * 4) || !dget(b->d_blk, b->nblk * sizeof(BlkInfo)) ||
        !dget(b->d_sizes, (ndt + 1) * sizeof(uint64_t)) ||
        !dget(b->d_offs, (ndt + 1) * sizeof(uint64_t)) || !dget(b->d_png, b->png_cap) ||
        !dget(b->d_segmap, ns * sizeof(uint32_t)) || !dget(b->d_th, th_bytes))
        return fail(PBX_E_INTERNAL, "device alloc: %s", hipGetErrorString(err));
    if (!b->ev[0])
        for (auto& e : b->ev) HIP_TRY(ctx->evpool.get(&e));
    const bool fine = !b->lite;  // every stage's event (the batch API: pbx_batch_stats_get)
    const int nks = ctx->nks.load();
    const bool multi = overlap && nks > 1 && b->nseg > 0;
    const int ks = multi ? (int)(ctx->kturn++ % (uint32_t)nks) : 0;
    hipStream_t st = ctx->kstream[ks];
    const int prev = ctx->last_ks.load(), stagger = ctx->stagger.load();
    if (multi && stagger && prev >= 0 && prev != ks)
        HIP_TRY(hipStreamWaitEvent(st, ctx->stage_ev[prev][stagger - 1], 0));
    b->attempted = true;
    b->ordinal = ++ctx->launch_seq;
    b->inject_fail = b->ordinal == ctx->fail_at.load();
    HIP_TRY(hipEventRecord(b->ev[0], st));
    if (b->ordinal == ctx->stall_at.load() && ctx->stall_flag)  // test hook: a wedged batch
        HIP_TRY(launch_stall(st, ctx->stall_flag, 30ull * 100000000ull));
    if (nft) HIP_TRY(hipMemcpyAsync(b->d_ft, b->h_desc, ft_bytes, hipMemcpyHostToDevice, st));
    if (ndt)
        HIP_TRY(hipMemcpyAsync(b->d_dt, (uint8_t*)b->h_desc + ft_bytes, dt_bytes, hipMemcpyHostToDevice, st));
    if (nth)
        HIP_TRY(hipMemcpyAsync(b->d_th, (uint8_t*)b->h_desc + ft_bytes + dt_bytes, th_bytes,
                               hipMemcpyHostToDevice, st));
    // regions straddling bands of sparse planes: their rows, band by band, into the bridge
    for (const pbx_batch::Bridge& g : b->bridges) {
        const Plane& p = *g.p;  // pinned, and so are its bands k0..k1
        const int64_t cb = (int64_t)g.w * bpp_of(p.pixel_type), xb = (int64_t)g.x * bpp_of(p.pixel_type);
        for (int32_t k = g.k0; k <= g.k1; k++) {
            const int32_t r0 = std::max(g.y, p.band_lo(k)), r1 = std::min(g.y + g.h, p.band_hi(k));
            if (r1 <= r0) continue;
            HIP_TRY(hipMemcpy2DAsync((uint8_t*)b->d_bridge + g.off + (int64_t)(r0 - g.y) * g.bp + g.xo, (size_t)g.bp,
                                     p.band_base(k) + (int64_t)r0 * p.pitch + xb, (size_t)p.pitch, (size_t)cb,
                                     (size_t)(r1 - r0), hipMemcpyDeviceToDevice, st));
        }
    }
    b->split = multi && nft && ndt && ctx->split_extract;
    if (b->split) {  // k_extract on xstream, once the descriptors (and bridges) are up
        if (!b->ev_x) HIP_TRY(ctx->evpool_sync.get(&b->ev_x));
        if (!b->ev_fs) HIP_TRY(ctx->evpool.get(&b->ev_fs));
        HIP_TRY(hipEventRecord(b->ev_x, st));
        HIP_TRY(hipStreamWaitEvent(ctx->xstream, b->ev_x, 0));
        HIP_TRY(hipEventRecord(b->ev[1], ctx->xstream));
        HIP_TRY(launch_extract(ctx->xstream, (const TileDesc*)b->d_ft, nft, b->ext_blocks, (uint8_t*)b->d_fixed,
                                b->ext_unaligned));
        HIP_TRY(hipEventRecord(b->ev[2], ctx->xstream));
        HIP_TRY(hipEventRecord(b->ev_x, ctx->xstream));
        HIP_TRY(hipEventRecord(b->ev_fs, st));
    } else {
        if (fine) HIP_TRY(hipEventRecord(b->ev[1], st));
        HIP_TRY(launch_extract(st, (const TileDesc*)b->d_ft, nft, b->ext_blocks, (uint8_t*)b->d_fixed,
                                b->ext_unaligned));
        if (fine || nft) HIP_TRY(hipEventRecord(b->ev[2], st));
    }
    const TileDesc* d_rows = (const TileDesc*)b->d_dt + b->ndirect_tiles;
    if (b->adaptive)  // the tile mode of every adaptive tile (the filtered ones follow k_rows')
        HIP_TRY(launch_adaptive_mode(st, (TileDesc*)b->d_dt + b->ndirect_tiles + b->nrows_tiles,
                                     ndt - b->ndirect_tiles - b->nrows_tiles, b->adaptive_max_rb));
    HIP_TRY(launch_rows(st, d_rows, b->nrows_tiles, b->rows_blocks, b->rows_max_rb, (uint8_t*)b->d_stream));
    HIP_TRY(launch_filter2(st, d_rows + b->nrows_tiles, b->nfilt2_tiles, b->filt2_blocks, b->filt2_max_rb,
                           (uint8_t*)b->d_stream));
    HIP_TRY(launch_filter3(st, d_rows + b->nrows_tiles + b->nfilt2_tiles, b->nfilt3_tiles, b->filt3_waves,
                           b->filt3_max_rb, b->filt3_filter, (uint8_t*)b->d_stream));
    HIP_TRY(launch_filter(st, d_rows + b->nrows_tiles + b->nfilt2_tiles + b->nfilt3_tiles,
                          ndt - b->ndirect_tiles - b->nrows_tiles - b->nfilt2_tiles - b->nfilt3_tiles,
                          b->filt_blocks, (uint8_t*)b->d_stream));
    if (fine) HIP_TRY(hipEventRecord(b->ev[3], st));
    // Diagnostic build of the deflate kernel: PBX_PHASE_PROFILE=1 stamps every phase.
    static const bool prof = getenv("PBX_PHASE_PROFILE") != nullptr;
    if (prof && !b->d_stamps && !dget(b->d_stamps, (size_t)b->nseg * 32 * sizeof(uint64_t)))
        return fail(PBX_E_INTERNAL, "device alloc: %s", hipGetErrorString(err));
    DeflateLaunch a;
    a.tiles = (const TileDesc*)b->d_dt;
    a.ntiles = ndt;
    a.nseg = b->nseg;
    a.stream = (uint8_t*)b->d_stream;
    a.info = (SegInfo*)b->d_info;
    a.hist = (uint32_t*)b->d_hist;
    a.mrec = (uint32_t*)b->d_mrec;
    a.codes = (uint32_t*)b->d_codes;
    a.sizes = (uint64_t*)b->d_sizes;
    a.offs = (uint64_t*)b->d_offs;
    a.out = (uint8_t*)b->d_png;
    a.stamps = prof ? (uint64_t*)b->d_stamps : nullptr;
    a.seg_tile = (uint32_t*)b->d_segmap;
    a.blk = (BlkInfo*)b->d_blk;
    a.nblk = b->nblk;
    a.cus = (uint32_t)ctx->cus;
    a.uniform_nseg = ndt ? b->dt[0].seg_count : 0u;
    for (uint32_t k = 1; k < ndt && a.uniform_nseg; k++)
        if (b->dt[k].seg_count != a.uniform_nseg) a.uniform_nseg = 0;
    a.uniform_rcp = recip32(a.uniform_nseg);
    for (uint32_t k = 0; k < ndt && !a.row_filtered; k++) a.row_filtered = b->dt[k].filter != 0;
    // the serving path reads the tile offsets from a mapped copy the scan writes (no D2H
    // copy at the end of the launch)
    void* offs_dev = nullptr;
    if (fetch_follows && ndt && b->lite && hipHostGetDevicePointer(&offs_dev, b->h_offs_pin, 0) == hipSuccess)
        a.offs_host = (uint64_t*)offs_dev;
    if (prof) HIP_TRY(hipMemsetAsync(b->d_stamps, 0, (size_t)b->nseg * 32 * sizeof(uint64_t), st));
    if (ndt) {
        HIP_TRY(launch_deflate(st, a, b->ev + 4, multi ? ctx->stage_ev[ks] : nullptr, fine));
        ctx->last_ks = multi ? ks : -1;
    } else {
        for (int k = fine ? 4 : 7; k < 8; k++) HIP_TRY(hipEventRecord(b->ev[k], st));
    }
    if (b->split) HIP_TRY(hipStreamWaitEvent(st, b->ev_x, 0));  // the batch ends when both are done
    HIP_TRY(launch_tiff_tiled(st, (const TiledHdr*)b->d_th, nth, (uint8_t*)b->d_fixed, (const uint64_t*)b->d_offs,
                              (uint8_t*)b->d_png));
    if (fetch_follows && ndt) {
        if (!a.offs_host)
            HIP_TRY(hipMemcpyAsync(b->h_offs_pin, b->d_offs, (ndt + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
        b->offs_ready = true;
    }
    HIP_TRY(hipEventRecord(b->ev[8], st));
    b->launched = true;
    return PBX_OK;
}

int pbx_batch_sync(pbx_ctx* ctx, pbx_batch* b) {
    if (!ctx || !b) return fail(PBX_E_BADARG, "null argument");
    if (ensure_device(ctx)) return PBX_E_INTERNAL;
    if (b->launched) HIP_TRY(wait_event(b->ev[8], b->reqs.size() <= ctx->spin_max_reqs ? ctx->spin_us : 0));
    if (b->inject_fail)
        return fail(PBX_E_INTERNAL, "injected device failure in batch %llu", (unsigned long long)b->ordinal);
    if (b->d_stamps && b->nseg) {  // PBX_PHASE_PROFILE diagnostic: mean cycles per phase
        std::vector<uint64_t> st((size_t)b->nseg * 32);
        HIP_TRY(hipMemcpy(st.data(), b->d_stamps, st.size() * 8, hipMemcpyDeviceToHost));
        const int base[3] = {0, 8, 24}, lim[3] = {8, 24, 32};
        const char* name[3] = {"lz77", "huff", "encode"};
        for (int kk = 0; kk < 3; kk++) {
            fprintf(stderr, "[pbx %s cycles/segment]", name[kk]);
            for (int k = base[kk] + 1; k < lim[kk]; k++) {
                double acc = 0;
                uint64_t cnt = 0;
                for (uint32_t s = 0; s < b->nseg; s++) {
                    const uint64_t a = st[(size_t)s * 32 + k - 1], c = st[(size_t)s * 32 + k];
                    if (a && c > a && c - a < (1ull << 40)) { acc += (double)(c - a); cnt++; }
                }
                if (cnt) fprintf(stderr, " %d:%.0f", k - base[kk], acc / cnt);
            }
            fprintf(stderr, "\n");
        }
    }
    return PBX_OK;
}

int pbx_batch_stats_get(pbx_ctx* ctx, pbx_batch* b, pbx_batch_stats* s) {
    if (!ctx || !b || !s) return fail(PBX_E_BADARG, "null argument");
    memset(s, 0, sizeof *s);
    s->tiles = b->reqs.size();
    for (size_t i = 0; i < b->reqs.size(); i++) {
        if (b->status[i] != PBX_OK) continue;
        s->ok_tiles++;
        if (b->reqs[i].format == PBX_FMT_PNG) s->png_tiles++;
        else if (b->reqs[i].format == PBX_FMT_TIF) s->tif_tiles++;
        else s->raw_tiles++;
    }
    s->in_bytes = b->in_bytes;
    s->stream_bytes = b->stream_bytes;
    s->segments = b->nseg;
    s->blocks = b->nblk;
    if (b->launched) {
        if (ensure_device(ctx)) return PBX_E_INTERNAL;
        if (b->lite) return fail(PBX_E_BADARG, "stage timings of a serving-path batch are not recorded");
        HIP_TRY(hipEventSynchronize(b->ev[8]));
        auto el = [&](int i, int j, double& out) -> int {
            float ms = 0;
            HIP_TRY(hipEventElapsedTime(&ms, b->ev[i], b->ev[j]));
            out = ms;
            return PBX_OK;
        };
        if (b->split) {  // the row kernels start on the kernel stream at ev_fs
            float ms = 0;
            HIP_TRY(hipEventElapsedTime(&ms, b->ev_fs, b->ev[3]));
            s->ms_filter = ms;
        }
        if (el(1, 2, s->ms_extract) || (!b->split && el(2, 3, s->ms_filter)) || el(3, 7, s->ms_deflate) ||
            el(7, 8, s->ms_assemble) || el(0, 8, s->ms_total) || el(3, 4, s->ms_lz77) ||
            el(4, 5, s->ms_huff) || el(6, 7, s->ms_encode))
            return PBX_E_INTERNAL;
        const uint32_t ndt = (uint32_t)b->dt.size();
        if (ndt) {
            std::vector<uint64_t> offs(ndt + 1);
            HIP_TRY(hipMemcpy(offs.data(), b->d_offs, (ndt + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost));
            s->deflate_out_bytes = offs[ndt];
            if (b->adaptive) {  // the tile modes k_adaptive_mode wrote into the descriptors
                std::vector<TileDesc> dd(ndt);
                HIP_TRY(hipMemcpy(dd.data(), b->d_dt, ndt * sizeof(TileDesc), hipMemcpyDeviceToHost));
                for (const TileDesc& d : dd)
                    if (d.filter == PBX_FILTER_ADAPTIVE && (d.flags & TF_DIRECT)) {
                        s->direct_tiles++;
                        s->direct_bytes += (uint64_t)d.w * d.h * d.bpp + d.stream_len;
                    }
            }
        }
        s->out_bytes = s->deflate_out_bytes;
        for (size_t k = 0; k < b->ft.size(); k++)
            s->out_bytes += (uint64_t)b->ft[k].w * b->ft[k].h * b->ft[k].bpp +
                            ((b->ft[k].flags & TF_TILED) ? b->ft[k].tiff_hdr
                             : (b->ft[k].flags & TF_TIFF) ? TIFF_DATA_OFFSET : 0);
    }
    return PBX_OK;
}

int pbx_batch_fetch(pbx_ctx* ctx, pbx_batch* b, pbx_result* out) {
    if (!ctx || !b || !out) return fail(PBX_E_BADARG, "null argument");
    const size_t n = b->reqs.size();
    for (size_t i = 0; i < n; i++) {
        out[i].status = b->status[i];
        out[i].format = b->reqs[i].format;
        out[i].w = b->w[i];
        out[i].h = b->h[i];
        out[i].data = nullptr;
        out[i].len = 0;
        out[i].owner = nullptr;
    }
    if (!b->launched) return PBX_OK;
    if (ensure_device(ctx)) return PBX_E_INTERNAL;
    // Wait for this batch only (later batches may already run on the kernel stream) and
    // copy on the copy stream, so the D2H overlaps the next batch's kernels.
    const int64_t spin = n <= ctx->spin_max_reqs ? ctx->spin_us : 0;
    HIP_TRY(wait_event(b->ev[8], spin));
    b->t_done = std::chrono::steady_clock::now();
    // a device failure shows when the batch's completion is collected (hipErrorLaunchFailure
    // at the event); the injected one takes the same way (PixelBufferVerticle.java:141-146: 500)
    if (b->inject_fail)
        return fail(PBX_E_INTERNAL, "injected device failure in batch %llu", (unsigned long long)b->ordinal);
    const uint32_t ndt = (uint32_t)b->dt.size();
    b->h_offs.assign(ndt + 1, 0);
    if (ndt && b->offs_ready) {
        memcpy(b->h_offs.data(), b->h_offs_pin, (ndt + 1) * sizeof(uint64_t));  // read back at launch
    } else if (ndt) {
        std::lock_guard<std::mutex> cg(ctx->copy_mu);
        HIP_TRY(hipMemcpyAsync(b->h_offs.data(), b->d_offs, (ndt + 1) * sizeof(uint64_t),
                               hipMemcpyDeviceToHost, ctx->copy_stream));
        HIP_TRY(hipStreamSynchronize(ctx->copy_stream));
    }
    const uint64_t png_total = ndt ? b->h_offs[ndt] : 0;
    hipError_t err = hipSuccess;
    HostBlock* hb = new HostBlock();
    hb->ctx = ctx;
    const bool zc = b->h_zc != nullptr;  // the kernels wrote the outputs into host memory
    if (zc) {
        hb->pinned = b->h_zc;
        b->h_zc = nullptr;  // the results own it now
    } else {
        hb->pinned = ctx->hpool.get(b->fixed_bytes + png_total + 256, &err);
    }
    if (!hb->pinned) {
        delete hb;
        return fail(PBX_E_INTERNAL, "pinned alloc: %s", hipGetErrorString(err));
    }
    uint8_t* h = (uint8_t*)hb->pinned;
    uint8_t* hp = h + (zc ? (b->zc_png_at & ~(uint64_t)1) : b->fixed_bytes);  // the deflate outputs
    auto fail_hb = [&](hipError_t e) {
        ctx->hpool.put(hb->pinned);
        delete hb;
        return fail(PBX_E_INTERNAL, "fetch: %s", hipGetErrorString(e));
    };
    if (!b->ev_copy && !zc) {
        const hipError_t e = ctx->evpool_sync.get(&b->ev_copy);
        if (e != hipSuccess) return fail_hb(e);
    }
    const auto t_copy = std::chrono::steady_clock::now();
    if (!zc) {  // the copies are queued back to back on the copy stream (several completers may have
        // theirs in flight: the link never waits for a host round trip); the wait is outside
        std::lock_guard<std::mutex> cg(ctx->copy_mu);
        hipError_t e = hipSuccess;
        if (b->fixed_bytes)
            e = hipMemcpyAsync(h, b->d_fixed, b->fixed_bytes, hipMemcpyDeviceToHost, ctx->copy_stream);
        if (e == hipSuccess && png_total)
            e = hipMemcpyAsync(h + b->fixed_bytes, b->d_png, png_total, hipMemcpyDeviceToHost, ctx->copy_stream);
        if (e == hipSuccess) e = hipEventRecord(b->ev_copy, ctx->copy_stream);
        if (e != hipSuccess) return fail_hb(e);
    }
    if (!zc)
        if (const hipError_t e = wait_event(b->ev_copy, spin)) return fail_hb(e);
    {   // the span timings (events of a finished batch: no wait); a lite batch recorded only
        // start (0), after the extract (2, when it had one), before k_frame (7) and end (8)
        float ms[5] = {0, 0, 0, 0, 0};
        const bool ext = !b->lite || !b->ft.empty();
        const int w0 = b->lite ? (ext ? 2 : 0) : 2;
        const int ij[5][2] = {{b->lite ? 0 : 1, 2}, {w0, b->lite ? 7 : 3}, {3, 7}, {7, 8}, {0, 8}};
        for (int q = 0; q < 5; q++) {
            if ((q == 0 && !ext) || (q == 2 && b->lite)) continue;
            (void)hipEventElapsedTime(&ms[q], b->ev[ij[q][0]], b->ev[ij[q][1]]);
        }
        if (b->split) (void)hipEventElapsedTime(&ms[1], b->ev_fs, b->ev[3]);  // (extract on xstream)
        pbx_spans& sp = hb->spans;
        sp.get_tile_direct_ms = ms[0];
        sp.write_image_ms = (double)ms[1] + ms[2];
        sp.create_metadata_ms = ms[3];
        sp.batch_ms = ms[4];
        sp.d2h_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_copy).count();
        sp.batch_tiles = n;
    }
    int refs = 0;
    for (size_t k = 0; k < b->ft.size(); k++) {
        const TileDesc& d = b->ft[k];
        if (d.flags & TF_TILED) continue;
        pbx_result& r = out[b->ft_req[k]];
        r.data = h + d.out_off;
        r.len = (uint64_t)d.w * d.h * d.bpp + ((d.flags & TF_TIFF) ? TIFF_DATA_OFFSET : 0);
        r.owner = hb;
        refs++;
    }
    for (uint32_t k = 0; k < ndt; k++) {
        if (b->dt[k].flags & TF_TILED) continue;
        pbx_result& r = out[b->dt_req[k]];
        r.data = hp + b->h_offs[k];
        r.len = b->h_offs[k + 1] - b->h_offs[k];
        r.owner = hb;
        refs++;
    }
    for (size_t k = 0; k < b->th.size(); k++) {  // tiled TIFF: header + all sub-tiles
        const TiledHdr& t = b->th[k];
        pbx_result& r = out[b->th_req[k]];
        if (t.comp == 1) {
            r.data = h + t.off;
            r.len = tiff_tiled_data_offset(t.n) + (uint64_t)t.n * t.t * t.t * t.bpp;
        } else {
            r.data = hp + b->h_offs[t.first];
            r.len = b->h_offs[t.first + t.n] - b->h_offs[t.first];
        }
        r.owner = hb;
        refs++;
    }
    if (refs == 0) {
        ctx->hpool.put(hb->pinned);
        delete hb;
    } else {
        hb->refs.store(refs);
    }
    return PBX_OK;
}

void pbx_batch_destroy(pbx_ctx* ctx, pbx_batch* b) {
    if (!ctx || !b) return;
    (void)hipSetDevice(ctx->device);
    if (b->launched) (void)hipEventSynchronize(b->ev[8]);
    else if (b->attempted) (void)sync_kernel_streams(ctx);  // a launch that failed midway
    if (b->ev_copy) (void)hipEventSynchronize(b->ev_copy);
    batch_unpin(ctx, b);
    free_batch_device(ctx, b);
    for (auto& e : b->ev) ctx->evpool.put(e);
    ctx->evpool_sync.put(b->ev_copy);
    ctx->evpool_sync.put(b->ev_x);
    ctx->evpool.put(b->ev_fs);
    delete b;
}

void pbx_results_release(pbx_ctx* ctx, pbx_result* res, uint64_t n) {
    if (!res) return;
    for (uint64_t i = 0; i < n; i++) {
        HostBlock* hb = (HostBlock*)res[i].owner;
        res[i].owner = nullptr;
        res[i].data = nullptr;
        if (!hb) continue;
        if (hb->refs.fetch_sub(1) == 1) {
            (void)ctx;  // the block goes back to the pool of the context that filled it
            hb->ctx->hpool.put(hb->pinned);
            delete hb;
        }
    }
}

int pbx_result_spans(const pbx_result* r, pbx_spans* out) {
    if (!r || !out) return fail(PBX_E_BADARG, "null argument");
    const HostBlock* hb = (const HostBlock*)r->owner;
    if (!hb) return fail(PBX_E_BADARG, "result without a body (status %d, or released)", r->status);
    *out = hb->spans;
    return PBX_OK;
}

int pbx_get_tiles(pbx_ctx* ctx, const pbx_tile_req* reqs, uint64_t n, pbx_result* out) {
    if (!ctx || !out || (!reqs && n)) return fail(PBX_E_BADARG, "null argument");
    return run_batch(ctx, reqs, n, out);
}

struct pbx_ticket {
    pbx_batch* b = nullptr;
    pbx_result* out = nullptr;
    int launch_status = PBX_OK;
    std::string launch_err;
};

int pbx_submit(pbx_ctx* ctx, const pbx_tile_req* reqs, uint64_t n, pbx_result* out, pbx_ticket** ticket) {
    if (!ctx || !out || !ticket || (!reqs && n)) return fail(PBX_E_BADARG, "null argument");
    *ticket = nullptr;
    pbx_batch* b = nullptr;
    int st;
    {
        std::lock_guard<std::mutex> run(ctx->run_mu);
        st = pbx_batch_plan(ctx, reqs, n, &b);
        if (st) return st;
        st = batch_launch(ctx, b, true, true);
    }
    ctx->n_batches++;
    ctx->n_requests += n;
    pbx_ticket* t = new pbx_ticket();
    t->b = b;
    t->out = out;
    t->launch_status = st;
    if (st != PBX_OK) t->launch_err = g_err;
    *ticket = t;
    return PBX_OK;
}

int pbx_wait(pbx_ctx* ctx, pbx_ticket* t, int64_t timeout_us) {
    if (!ctx || !t) return fail(PBX_E_BADARG, "null argument");
    pbx_batch* b = t->b;
    if (t->launch_status == PBX_OK && b->launched && timeout_us >= 0) {
        if (ensure_device(ctx)) return PBX_E_INTERNAL;
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us);
        for (;;) {
            const hipError_t q = hipEventQuery(b->ev[8]);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) {
                t->launch_status = fail(PBX_E_INTERNAL, "hipEventQuery: %s", hipGetErrorString(q));
                t->launch_err = g_err;
                break;
            }
            if (std::chrono::steady_clock::now() >= until) return PBX_E_PENDING;
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    }
    int st = t->launch_status;
    if (st == PBX_OK) st = pbx_batch_fetch(ctx, b, t->out);
    if (st != PBX_OK) {  // every request of the batch fails with 500 (or its own 4xx)
        const std::string msg = t->launch_status != PBX_OK ? t->launch_err : g_err;
        for (size_t i = 0; i < b->reqs.size(); i++) {
            pbx_result& r = t->out[i];
            r.status = b->status[i] == PBX_OK ? PBX_E_INTERNAL : b->status[i];
            r.format = b->reqs[i].format;
            r.w = b->w[i];
            r.h = b->h[i];
            r.data = nullptr;
            r.len = 0;
            r.owner = nullptr;
        }
        g_err = msg;
    }
    pbx_batch_destroy(ctx, b);
    delete t;
    return st;
}

int pbx_abi_sizes(uint64_t* sizes, int n) {
    const uint64_t v[8] = {sizeof(pbx_config), sizeof(pbx_plane_desc), sizeof(pbx_tile_req),
                           sizeof(pbx_result), sizeof(pbx_batch_stats), sizeof(pbx_image_desc),
                           sizeof(pbx_residency_stats), sizeof(pbx_spans)};
    if (!sizes || n < 0) return fail(PBX_E_BADARG, "null argument");
    for (int i = 0; i < n && i < 8; i++) sizes[i] = v[i];
    return 8;
}

int pbx_test_huffman(pbx_ctx* ctx, const uint32_t* hist, const uint32_t* sl_last, uint32_t nseg,
                     uint32_t* codes, uint32_t* info) {
    if (!ctx || !hist || !sl_last || !codes || !info) return fail(PBX_E_BADARG, "null argument");
    if (!nseg) return PBX_OK;
    if (ensure_device(ctx)) return PBX_E_INTERNAL;
    std::lock_guard<std::mutex> g(ctx->run_mu);
    std::vector<SegInfo> si(nseg);
    std::vector<BlkInfo> bl(nseg);
    memset(si.data(), 0, nseg * sizeof(SegInfo));
    memset(bl.data(), 0, nseg * sizeof(BlkInfo));
    for (uint32_t k = 0; k < nseg; k++) {  // one segment per block
        si[k].sl = sl_last[2 * k];
        si[k].last = sl_last[2 * k + 1];
        si[k].flags = SF_FIRST | SF_LAST;
        bl[k].seg0 = k;
        bl[k].nseg = 1;
    }
    hipError_t err = hipSuccess;
    void* d_info = ctx->dpool.get(nseg * sizeof(SegInfo), &err);
    void* d_blk = d_info ? ctx->dpool.get(nseg * sizeof(BlkInfo), &err) : nullptr;
    void* d_hist = d_blk ? ctx->dpool.get((size_t)nseg * HIST_WORDS * 4, &err) : nullptr;
    void* d_codes = d_hist ? ctx->dpool.get((size_t)nseg * CODE_WORDS * 4, &err) : nullptr;
    int rc = PBX_OK;
    if (!d_codes) {
        rc = fail(PBX_E_INTERNAL, "device alloc: %s", hipGetErrorString(err));
    } else {
        rc = [&]() -> int {
            HIP_TRY(hipMemcpy(d_info, si.data(), nseg * sizeof(SegInfo), hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(d_blk, bl.data(), nseg * sizeof(BlkInfo), hipMemcpyHostToDevice));
            HIP_TRY(hipMemcpy(d_hist, hist, (size_t)nseg * HIST_WORDS * 4, hipMemcpyHostToDevice));
            HIP_TRY(launch_huffman(ctx->stream, nseg, (BlkInfo*)d_blk, (SegInfo*)d_info,
                                   (const uint32_t*)d_hist, (uint32_t*)d_codes));
            HIP_TRY(hipStreamSynchronize(ctx->stream));
            HIP_TRY(hipMemcpy(codes, d_codes, (size_t)nseg * CODE_WORDS * 4, hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(si.data(), d_info, nseg * sizeof(SegInfo), hipMemcpyDeviceToHost));
            HIP_TRY(hipMemcpy(bl.data(), d_blk, nseg * sizeof(BlkInfo), hipMemcpyDeviceToHost));
            return PBX_OK;
        }();
    }
    for (void* p : {d_info, d_blk, d_hist, d_codes}) if (p) ctx->dpool.put(p);
    if (rc) return rc;
    for (uint32_t k = 0; k < nseg; k++) {
        info[4 * k] = si[k].btype;
        info[4 * k + 1] = si[k].hdr_bits;
        info[4 * k + 2] = bl[k].data_bits;
        info[4 * k + 3] = bl[k].nbytes;
    }
    return PBX_OK;
}

int pbx_test_batch_lz77(pbx_ctx* ctx, pbx_batch* b, uint32_t* hist, uint32_t* mrec, uint64_t nseg) {
    if (!ctx || !b || !hist || !mrec) return fail(PBX_E_BADARG, "null argument");
    if (!b->launched) return fail(PBX_E_BADARG, "batch not launched");
    if (nseg != b->nseg) return fail(PBX_E_BADARG, "segment count %llu != %u", (unsigned long long)nseg, b->nseg);
    if (ensure_device(ctx)) return PBX_E_INTERNAL;
    HIP_TRY(hipEventSynchronize(b->ev[8]));
    HIP_TRY(hipMemcpy(hist, b->d_hist, nseg * HIST_WORDS * 4, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(mrec, b->d_mrec, nseg * MREC_WORDS * 4, hipMemcpyDeviceToHost));
    return PBX_OK;
}

int pbx_shard_of(const pbx_tile_req* r, int32_t tw, int32_t th, int32_t world) {
    if (!r || world <= 0 || tw <= 0 || th <= 0) return fail(PBX_E_BADARG, "bad argument"), -1;
    uint64_t k = (uint64_t)r->image_id;
    const uint64_t parts[5] = {(uint64_t)(uint32_t)r->z, (uint64_t)(uint32_t)r->c,
                               (uint64_t)(uint32_t)r->t, (uint64_t)(uint32_t)(r->x / tw),
                               (uint64_t)(uint32_t)(r->y / th)};
    for (uint64_t p : parts) k = splitmix64(k ^ (p * 0x9E3779B97F4A7C15ull));
    return (int)(k % (uint64_t)world);
}

}  // extern "C"

// One getTile with a deadline of `to` us from now (<= 0: none).  Uncoalesced contexts plan and
// launch the lite single-request batch themselves (as run_batch; run_mu waited for only until the
// deadline), poll its completion until the deadline, and past it park the batch for the reaper
// thread's collector (the ticket's pins and pool blocks return even if the context
// then goes idle).
static int get_tile_within(pbx_ctx* ctx, const pbx_tile_req* req, pbx_result* out, int64_t to) {
    int st;
    if (ctx->coal) {
        st = ctx->coal->submit(*req, out, to);
    } else if (to <= 0) {
        st = run_batch(ctx, req, 1, out);
    } else {
        using clk = std::chrono::steady_clock;
        const auto until = clk::now() + std::chrono::microseconds(to);
        pbx_batch* b = nullptr;
        {
            std::unique_lock<std::mutex> run(ctx->run_mu, std::defer_lock);
            while (!run.try_lock()) {
                if (clk::now() >= until) return deadline_result(ctx, *req, out);
                std::this_thread::sleep_for(std::chrono::microseconds(20));
            }
            st = pbx_batch_plan(ctx, req, 1, &b);
            if (st) return st;
            st = batch_launch(ctx, b, false, true);
        }
        ctx->n_batches++;
        ctx->n_requests++;
        if (st == PBX_OK) {
            if (ensure_device(ctx)) return PBX_E_INTERNAL;
            const auto spin_until = clk::now() + std::chrono::microseconds(ctx->spin_us);
            int64_t nap = 5;
            for (;;) {
                const hipError_t q = hipEventQuery(b->ev[8]);
                if (q == hipSuccess) break;
                if (q != hipErrorNotReady) break;  // the fetch reports the device error
                const auto now = clk::now();
                if (now >= until) {  // parked: the reaper's collector releases it when it ends
                    pbx_ticket* t = new pbx_ticket();
                    t->b = b;
                    t->out = new pbx_result[1]();
                    {
                        std::lock_guard<std::mutex> g(ctx->late_mu);
                        ctx->late.emplace_back(t, t->out);
                    }
                    ctx->reaper.poke();
                    return deadline_result(ctx, *req, out);
                }
                if (now < spin_until) {
                    cpu_relax();
                } else {
                    std::this_thread::sleep_for(std::chrono::microseconds(nap));
                    nap = std::min<int64_t>(nap * 2, 200);
                }
            }
            st = pbx_batch_fetch(ctx, b, out);
        }
        if (st != PBX_OK) {  // as run_batch: a device failure is this request's 500
            const std::string msg = g_err;
            out->status = b->status[0] == PBX_OK ? PBX_E_INTERNAL : b->status[0];
            out->format = req->format;
            out->w = b->w[0];
            out->h = b->h[0];
            out->data = nullptr;
            out->len = 0;
            out->owner = nullptr;
            pbx_batch_destroy(ctx, b);
            g_err = msg;
            return st;
        }
        pbx_batch_destroy(ctx, b);
    }
    if (st) return st;
    return out->status;
}

extern "C" {

int pbx_get_tile(pbx_ctx* ctx, const pbx_tile_req* req, pbx_result* out) {
    if (!ctx || !req || !out) return fail(PBX_E_BADARG, "null argument");
    return get_tile_within(ctx, req, out, ctx->timeout_us);
}

int pbx_test_fail_band_write(pbx_ctx* ctx, uint64_t ahead) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    ctx->fail_band_write_at = ahead ? ctx->band_writes.load() + ahead : 0;
    return PBX_OK;
}

int pbx_test_stall_batch(pbx_ctx* ctx, uint64_t ahead) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    if (!ahead) {  // release: no lock, a launch may be waiting behind the stalled batch
        ctx->stall_at = 0;
        if (ctx->stall_flag) __atomic_store_n(ctx->stall_flag, 0u, __ATOMIC_SEQ_CST);
        return PBX_OK;
    }
    std::lock_guard<std::mutex> run(ctx->run_mu);  // launches are ordered under run_mu
    if (ensure_device(ctx)) return PBX_E_INTERNAL;
    if (!ctx->stall_flag) {
        void* p = nullptr;
        HIP_TRY(hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent));
        ctx->stall_flag = (uint32_t*)p;
    }
    __atomic_store_n(ctx->stall_flag, 1u, __ATOMIC_SEQ_CST);
    ctx->stall_at = ctx->launch_seq.load() + ahead;
    return PBX_OK;
}

int pbx_test_fail_batch(pbx_ctx* ctx, uint64_t ahead) {
    if (!ctx) return fail(PBX_E_BADARG, "null ctx");
    std::lock_guard<std::mutex> run(ctx->run_mu);  // launches are ordered under run_mu
    ctx->fail_at = ahead ? ctx->launch_seq.load() + ahead : 0;
    return PBX_OK;
}

// ------------------------------------------------------------------ node: N contexts
}  // extern "C"

// Several device contexts in one process: the reference runs all its worker verticles in one
// JVM (PixelBufferMicroserviceVerticle.java:117-118,224-233), so a node-wide drop-in routes
// each getTile to the context that holds its plane (or row band), or, when several do (planes
// replicated on every GPU), to the pbx_shard_of owner among them.
struct pbx_node {
    std::vector<pbx_ctx*> ctxs;
    int32_t tile = 512;
};

extern "C" {

int pbx_node_init(const pbx_config* cfg, int32_t n, const int32_t* devices, int32_t shard_tile, pbx_node** out) {
    if (!out) return fail(PBX_E_BADARG, "null out");
    *out = nullptr;
    if (n < 1 || n > 64) return fail(PBX_E_BADARG, "node of %d contexts", n);
    if (shard_tile < 0) return fail(PBX_E_BADARG, "bad shard tile %d", shard_tile);
    pbx_config base;
    if (cfg) base = *cfg; else pbx_config_default(&base);
    pbx_node* node = new pbx_node();
    node->tile = shard_tile ? shard_tile : 512;
    for (int32_t k = 0; k < n; k++) {
        pbx_config c = base;
        c.device = devices ? devices[k] : k;  // the same device may appear several times
        pbx_ctx* ctx = nullptr;
        if (int rc = pbx_init(&c, &ctx)) {
            const std::string msg = g_err;
            pbx_node_shutdown(node);
            g_err = msg;
            return rc;
        }
        node->ctxs.push_back(ctx);
    }
    *out = node;
    return PBX_OK;
}

void pbx_node_shutdown(pbx_node* node) {
    if (!node) return;
    for (pbx_ctx* c : node->ctxs) pbx_shutdown(c);
    delete node;
}

int32_t pbx_node_size(pbx_node* node) { return node ? (int32_t)node->ctxs.size() : 0; }

pbx_ctx* pbx_node_context(pbx_node* node, int32_t k) {
    if (!node || k < 0 || k >= (int32_t)node->ctxs.size()) return nullptr;
    return node->ctxs[(size_t)k];
}

int pbx_node_route(pbx_node* node, const pbx_tile_req* req, int32_t* index) {
    if (!node || !req || !index) return fail(PBX_E_BADARG, "null argument");
    const int32_t n = (int32_t)node->ctxs.size();
    const int32_t owner = n == 1 ? 0 : pbx_shard_of(req, node->tile, node->tile, n);
    if (owner < 0) return PBX_E_BADARG;
    int32_t owning = -1;
    for (int32_t k = 0; k < n; k++) {  // the owner first, then the others in ring order
        const int32_t c = (owner + k) % n;
        int32_t w = 0, h = 0;
        Plane* p = nullptr;
        bool owns = false;
        const int st = validate(node->ctxs[(size_t)c], *req, w, h, p, false, nullptr, &owns);
        if (st != PBX_E_NOT_RESIDENT) {
            *index = c;
            return st;
        }
        if (owns && owning < 0) owning = c;
    }
    // nobody holds it: the binding loads it where it belongs and retries — into the context
    // whose sparse plane owns those rows (their bands are not loaded yet), else the shard owner
    *index = owning >= 0 ? owning : owner;
    return fail(PBX_E_NOT_RESIDENT, "no context of the node holds the plane (load it into context %d)", *index);
}

int pbx_node_get_tile(pbx_node* node, const pbx_tile_req* req, pbx_result* out, int32_t* served_by) {
    if (!node || !req || !out) return fail(PBX_E_BADARG, "null argument");
    // One deadline for the whole call: the retry gets what the first attempt left.
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    int st = PBX_E_NOT_RESIDENT;
    for (int attempt = 0; attempt < 2; attempt++) {  // a plane evicted between route and get
        int32_t k = 0;
        const int r = pbx_node_route(node, req, &k);
        if (r == PBX_E_BADARG) return r;
        if (served_by) *served_by = k;
        pbx_ctx* c = node->ctxs[(size_t)k];
        int64_t to = c->timeout_us;
        if (to > 0 && attempt) {
            to -= std::chrono::duration_cast<std::chrono::microseconds>(clk::now() - t0).count();
            if (to <= 0) return deadline_result(c, *req, out);
        }
        st = get_tile_within(c, req, out, to);
        if (st != PBX_E_NOT_RESIDENT || r == PBX_E_NOT_RESIDENT) break;
    }
    return st;
}

int pbx_ctx_stats_get(pbx_ctx* ctx, uint64_t* batches, uint64_t* requests) {
    if (!ctx || !batches || !requests) return fail(PBX_E_BADARG, "null argument");
    *batches = ctx->n_batches.load();
    *requests = ctx->n_requests.load();
    return PBX_OK;
}

}  // extern "C"
