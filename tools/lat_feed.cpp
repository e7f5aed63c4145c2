// lat_feed.cpp -- per-read latency of fws_rx_session_feed (the drop-in hook's
// hot call, GpuRxHook -> feed per read) on one masked BIN frame per read, by
// frame size, buffer kind (registered host memory: decoded in place; plain
// malloc: staged through the session's pinned block) and receive path (a
// kernel launch per read, or the persistent decode grid with W workers).
// Splits the ~16 us hooked-read RTT of the echo A/B into its fixed part (a
// 0-byte payload) and its size-dependent part. One JSON line per case.
//
// usage: lat_feed [iters]          (built by tools/build_lat_feed.sh)
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "fws_gpu.h"

extern "C" int fws_internal_rx_service_trace(int on, int device, unsigned long long *out12);

static size_t make_frame(uint8_t *out, size_t payload, uint32_t key) {
    size_t h = 0;
    out[h++] = 0x82;                                     // FIN | BIN
    if (payload < 126) {
        out[h++] = (uint8_t)(0x80 | payload);
    } else if (payload < 65536) {
        out[h++] = 0x80 | 126;
        out[h++] = (uint8_t)(payload >> 8);
        out[h++] = (uint8_t)payload;
    } else {
        out[h++] = 0x80 | 127;
        for (int i = 7; i >= 0; --i) out[h++] = (uint8_t)((uint64_t)payload >> (8 * i));
    }
    memcpy(out + h, &key, 4);
    h += 4;
    const uint8_t *k = out + h - 4;
    for (size_t i = 0; i < payload; ++i) out[h + i] = (uint8_t)((i * 131u + 7u) ^ k[i & 3]);
    return h + payload;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 3000;
    const size_t sizes[] = {0, 4096, 65536};
    const uint32_t workers_list[] = {0, 16};
    const size_t cap = 1 << 20;
    uint8_t *reg = (uint8_t *)aligned_alloc(4096, cap), *plain = (uint8_t *)aligned_alloc(4096, cap);
    uint8_t *frame = (uint8_t *)malloc(cap);
    if (!reg || !plain || !frame || fws_gpu_host_register(reg, cap)) {
        fprintf(stderr, "alloc/register failed\n");
        return 1;
    }
    const bool trace = getenv("LAT_TRACE") && atoi(getenv("LAT_TRACE"));
    unsigned long long tr[12];
    if (trace) fws_internal_rx_service_trace(1, 0, tr);
    for (uint32_t workers : workers_list) {
        fws_gpu_ctx *ctx = nullptr;
        if (fws_gpu_ctx_create(0, &ctx) || fws_gpu_ctx_set_rx_persistent(ctx, workers)) return 1;
        for (int registered = 1; registered >= 0; --registered) {
            for (size_t pl : sizes) {
                fws_rx_session *s = nullptr;
                if (fws_rx_session_create(ctx, 1, &s)) return 1;
                if (trace) fws_internal_rx_service_trace(1, 0, tr);       // zero the sums
                const size_t n = make_frame(frame, pl, 0x5A3C96E1u);
                uint8_t *buf = registered ? reg : plain;
                std::vector<double> us;
                us.reserve(iters);
                for (int i = 0; i < iters + 200; ++i) {
                    memcpy(buf, frame, n);
                    const fws_rx_event *ev;
                    const uint8_t *ctl;
                    uint64_t nev = 0, used = 0;
                    const auto t0 = std::chrono::steady_clock::now();
                    const int r = fws_rx_session_feed_view(s, buf, n, cap, &ev, &nev, &ctl, &used);
                    const auto t1 = std::chrono::steady_clock::now();
                    if (r || (pl && (nev != 1 || ev[0].size != pl))) {
                        fprintf(stderr, "feed failed: r=%d nev=%llu\n", r, (unsigned long long)nev);
                        return 1;
                    }
                    if (i >= 200) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
                }
                for (size_t i = 0; i < pl; ++i)
                    if (buf[n - pl + i] != (uint8_t)(i * 131u + 7u)) {
                        fprintf(stderr, "payload differs at %zu\n", i);
                        return 1;
                    }
                std::sort(us.begin(), us.end());
                printf("{\"workers\": %u, \"buffer\": \"%s\", \"payload\": %zu, \"p10_us\": %.2f, \"p50_us\": %.2f, "
                       "\"p90_us\": %.2f, \"p99_us\": %.2f}\n",
                       workers, registered ? "registered" : "plain", pl, us[us.size() / 10], us[us.size() / 2],
                       us[us.size() * 9 / 10], us[us.size() * 99 / 100]);
                if (trace && workers) {
                    fws_internal_rx_service_trace(1, 0, tr);
                    const double n = tr[0] ? (double)tr[0] : 1.0, tpu = tr[8] ? (double)tr[8] : 100.0;
                    const double hn = tr[9] ? (double)tr[9] : 1.0;
                    printf("{\"trace\": true, \"payload\": %zu, \"buffer\": \"%s\", \"gpu_requests\": %llu, "
                           "\"acquire_us\": %.2f, \"staged_us\": %.2f, \"walked_us\": %.2f, \"unmasked_us\": %.2f, "
                           "\"stores_drained_us\": %.2f, \"flag_stored_us\": %.2f, \"host_publish_us\": %.2f, "
                           "\"host_wait_us\": %.2f}\n",
                           pl, registered ? "registered" : "plain", tr[0], tr[1] / n / tpu, tr[2] / n / tpu,
                           tr[3] / n / tpu, tr[4] / n / tpu, tr[6] / n / tpu, tr[5] / n / tpu, tr[10] / hn / 1000.0,
                           tr[11] / hn / 1000.0);
                }
                fflush(stdout);
                fws_rx_session_destroy(s);
            }
        }
        fws_gpu_ctx_destroy(ctx);
    }
    // mux rounds (the batched hook's call per loop step): k reads of 4 KiB, one
    // per connection, in registered memory, decoded in place
    const uint32_t mux_workers[] = {0, 16, 64};
    for (uint32_t workers : mux_workers) {
        fws_gpu_ctx *ctx = nullptr;
        if (fws_gpu_ctx_create(0, &ctx) || fws_gpu_ctx_set_rx_persistent(ctx, workers)) return 1;
        for (uint32_t k : {1u, 8u, 32u, 64u}) {
            fws_rx_mux *m = nullptr;
            if (fws_rx_mux_create(ctx, k, &m)) return 1;
            const size_t n = make_frame(frame, 4096, 0x1B2C3D4Eu);
            const size_t slot = 8192;
            std::vector<fws_rx_read> rd(k);
            std::vector<fws_rx_read_result> res(k);
            std::vector<double> us;
            for (int i = 0; i < iters / 4 + 100; ++i) {
                for (uint32_t c = 0; c < k; ++c) {
                    memcpy(reg + c * slot, frame, n);
                    rd[c] = fws_rx_read{c, 0u, reg + c * slot, n, slot};
                }
                const auto t0 = std::chrono::steady_clock::now();
                const int r = fws_rx_mux_feed(m, rd.data(), k, res.data());
                const auto t1 = std::chrono::steady_clock::now();
                if (r) {
                    fprintf(stderr, "mux feed failed: %d\n", r);
                    return 1;
                }
                for (uint32_t c = 0; c < k; ++c)
                    if (res[c].ret || res[c].n_events != 1) {
                        fprintf(stderr, "mux read %u: ret %d events %llu\n", c, res[c].ret,
                                (unsigned long long)res[c].n_events);
                        return 1;
                    }
                if (i >= 100) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            }
            std::sort(us.begin(), us.end());
            printf("{\"mux\": true, \"workers\": %u, \"reads\": %u, \"p10_us\": %.2f, \"p50_us\": %.2f, "
                   "\"p90_us\": %.2f}\n", workers, k, us[us.size() / 10], us[us.size() / 2], us[us.size() * 9 / 10]);
            fflush(stdout);
            fws_rx_mux_destroy(m);
        }
        fws_gpu_ctx_destroy(ctx);
    }
    fws_gpu_host_unregister(reg);
    return 0;
}
