// serve_bench.cpp — BENCH-ONLY load generator for the served path (lib/libpbx_servebench.so;
// not part of libpbx.so, nothing in the product loads it).
//
// The reference serves one request per Vert.x worker thread, `worker_pool_size` workers
// (default 2 x cores) blocking in TileRequestHandler.getTile
// (PixelBufferMicroserviceVerticle.java:117-118,224-233; PixelBufferVerticle.java:109-110).
// This driver reproduces that closed loop against the C-ABI: T native threads, each calling
// pbx_get_tile (the coalesced single-request entry point) back to back, copying every body
// into a fresh exact-length buffer (what the JNI shim's NewByteArray + SetByteArrayRegion
// does) and releasing the result.  Reports requests/s, bytes and the latency distribution.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/pbx.h"

extern "C" {

typedef struct pbx_serve_stats {
    uint64_t requests, ok, bytes, batches;
    double seconds, p50_us, p90_us, p99_us, max_us, mean_us;
} pbx_serve_stats;

// n requests reqs[0..n) are served round robin by `threads` threads (each one request at a
// time), closed loop, the threads started once: the first `warmup` calls are not recorded,
// the next `total` are, and the threads keep the load on until every recorded call has
// returned (no ramp-up or ramp-down inside the measurement).  Rate = total / (the last
// recorded call's return - the first recorded call's issue).
int pbx_serve_bench(pbx_ctx* ctx, const pbx_tile_req* reqs, uint64_t n, int threads,
                    uint64_t total, uint64_t warmup, pbx_serve_stats* out) {
    if (!ctx || !reqs || !n || threads < 1 || !out || !total) return PBX_E_BADARG;
    using clk = std::chrono::steady_clock;
    const auto base = clk::now();
    auto us = [&](clk::time_point t) { return std::chrono::duration<double, std::micro>(t - base).count(); };
    std::atomic<uint64_t> next{0}, done_rec{0}, ok{0}, bytes{0};
    std::atomic<double> t_first{-1.0}, t_last{0.0};
    std::vector<std::vector<float>> lat(threads);
    for (auto& v : lat) v.reserve(total / threads + 16);
    uint64_t b0 = 0, r0 = 0, b1 = 0, r1 = 0;
    std::atomic<bool> stats0{false};
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++)
        th.emplace_back([&, t] {
            std::vector<uint8_t> body;
            for (;;) {
                if (done_rec.load() >= total) break;
                const uint64_t i = next.fetch_add(1);
                const bool rec = i >= warmup && i < warmup + total;
                pbx_result r;
                memset(&r, 0, sizeof r);
                const auto c0 = clk::now();
                if (i == warmup) {
                    pbx_ctx_stats_get(ctx, &b0, &r0);
                    stats0 = true;
                    t_first = us(c0);
                }
                const int st = pbx_get_tile(ctx, &reqs[i % n], &r);
                if (st == PBX_OK && r.data) {
                    body.resize(r.len);
                    memcpy(body.data(), r.data, r.len);  // the JNI byte[] copy
                }
                pbx_results_release(ctx, &r, 1);
                const auto c1 = clk::now();
                if (rec) {
                    lat[t].push_back(std::chrono::duration<float, std::micro>(c1 - c0).count());
                    if (st == PBX_OK) {
                        ok.fetch_add(1);
                        bytes.fetch_add(r.len);
                    }
                    double e = us(c1), cur = t_last.load();
                    while (e > cur && !t_last.compare_exchange_weak(cur, e)) {
                    }
                    if (done_rec.fetch_add(1) + 1 == total) pbx_ctx_stats_get(ctx, &b1, &r1);
                }
            }
        });
    for (auto& x : th) x.join();
    std::vector<float> all;
    all.reserve(total);
    for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    auto pct = [&](double p) { return all.empty() ? 0.0 : (double)all[(size_t)(p * (all.size() - 1))]; };
    double sum = 0;
    for (float v : all) sum += v;
    out->requests = total;
    out->ok = ok.load();
    out->bytes = bytes.load();
    out->batches = stats0 ? b1 - b0 : 0;
    out->seconds = (t_last.load() - t_first.load()) * 1e-6;
    out->p50_us = pct(0.50);
    out->p90_us = pct(0.90);
    out->p99_us = pct(0.99);
    out->max_us = all.empty() ? 0.0 : (double)all.back();
    out->mean_us = all.empty() ? 0.0 : sum / all.size();
    return PBX_OK;
}

}  // extern "C"
