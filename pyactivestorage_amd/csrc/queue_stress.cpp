// queue_stress.cpp — host-only stress of pyas_queue.hpp, the coalescer's
// ring / FIFO / hand-off logic, built under -fsanitize=address,undefined and
// -fsanitize=thread by `make -C pyactivestorage_amd/csrc sanitize` and run
// by tests/test_sanitizers.py.
//
// 30 caller threads (active.py:557's pool size) each make requests of random
// size: reserve ring space, write a pattern derived from (caller, request)
// into it without the lock (the pread of pyas_coalesced_reduce), sometimes
// fail the fill (a short read), and wait.  A dispatcher thread batches the
// filled prefix; a completer thread "reduces" every submitted request by
// checksumming its ring bytes (the kernels' reads) and hands the sum back.
// Every caller checks that it got the checksum of exactly what it wrote: two
// requests sharing ring bytes, or a completion before the bytes were read,
// shows up as a wrong sum; a lost wake-up as a hang (the test's timeout).
//
// Usage: queue_stress [callers] [requests per caller] [ring bytes] [slots]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <random>
#include <thread>
#include <vector>

#include "pyas_queue.hpp"

namespace {

struct Req : pyas::QItem {
    uint64_t want = 0;       // checksum of what the caller wrote
    uint64_t got = 0;        // checksum the completer computed
    bool filled = false;
};

struct Slot {
    std::vector<Req *> batch;
};

uint64_t pattern(uint64_t seed, int64_t i) {
    uint64_t x = seed * 0x9E3779B97F4A7C15ull + (uint64_t)i * 0xBF58476D1CE4E5B9ull;
    x ^= x >> 31;
    return x;
}

}  // namespace

int main(int argc, char **argv) {
    const int callers = argc > 1 ? atoi(argv[1]) : 30;
    const int per = argc > 2 ? atoi(argv[2]) : 400;
    const int64_t ring_bytes = argc > 3 ? atoll(argv[3]) : (int64_t)1 << 16;
    const int n_slots = argc > 4 ? atoi(argv[4]) : 2;
    std::vector<uint8_t> ring((size_t)ring_bytes);
    pyas::BatchQueue<Req, Slot> q(ring_bytes, 64);
    std::vector<Slot> slots((size_t)n_slots);
    for (Slot &s : slots) q.add_slot(&s);
    std::atomic<int64_t> bad{0}, done{0}, skipped{0}, batches{0};

    std::thread disp([&] {
        Slot *sl = nullptr;
        while (q.next_batch(sl)) q.launched(sl, [&] { batches.fetch_add(1, std::memory_order_relaxed); });
        q.dispatcher_done();
    });
    std::thread comp([&] {
        Slot *sl = nullptr;
        while (q.next_done(sl)) {
            for (Req *r : sl->batch) {   // the "kernel": read the submitted bytes
                if (r->state != pyas::kSubmitted) continue;
                uint64_t s = 0;
                for (int64_t i = 0; i < r->span; ++i) s = s * 1315423911ull + ring[(size_t)(r->ring_off + i)];
                r->got = s;
            }
            q.complete(sl, [] {});
        }
    });
    std::vector<std::thread> ts;
    for (int t = 0; t < callers; ++t) {
        ts.emplace_back([&, t] {
            std::mt19937_64 rng((uint64_t)t * 7919u + 1u);
            for (int k = 0; k < per; ++k) {
                Req r;
                const int64_t cap = ring_bytes / 4 > 1 ? ring_bytes / 4 : 1;
                r.span = 1 + (int64_t)(rng() % (uint64_t)cap);
                if (!q.reserve(&r)) {
                    bad.fetch_add(1);
                    return;
                }
                const uint64_t seed = ((uint64_t)t << 32) | (uint64_t)k;
                uint64_t s = 0;
                for (int64_t i = 0; i < r.span; ++i) {
                    const uint8_t b = (uint8_t)pattern(seed, i);
                    ring[(size_t)(r.ring_off + i)] = b;
                    s = s * 1315423911ull + b;
                }
                r.want = s;
                const bool ok = rng() % 16 != 0;   // 1 in 16 fills fails (a short read)
                q.finish(&r, ok, [] {});
                if (ok && r.got != r.want) bad.fetch_add(1);
                if (!ok) skipped.fetch_add(1);
                done.fetch_add(1);
            }
        });
    }
    for (auto &th : ts) th.join();
    q.stop();
    disp.join();
    comp.join();
    printf("queue_stress: callers %d, requests %lld (%lld failed fills), batches %lld, ring %lld B, bad %lld\n",
           callers, (long long)done.load(), (long long)skipped.load(), (long long)batches.load(),
           (long long)ring_bytes, (long long)bad.load());
    return bad.load() == 0 && done.load() == (int64_t)callers * per ? 0 : 1;
}
