// pyas_queue.hpp — the host-side concurrency of the coalesced drop-in
// (pyas_coalesce.hip): ring reservation, the FIFO of requests in ring order,
// and the hand-offs between caller threads, the dispatcher and the
// completer.  It contains no HIP, so it also builds on its own under
// -fsanitize=address,undefined and -fsanitize=thread (csrc/queue_stress.cpp
// drives it from 30 caller threads, the reference's pool size at
// activestorage/active.py:557-589; tests/test_sanitizers.py runs it).
//
// Protocol (all state under `mu`):
//   caller     : reserve() a span of the ring (waits while the ring is full),
//                fill its bytes without the lock, then finish() with ok or
//                skip, which wakes the dispatcher and sleeps until its batch
//                has completed;
//   dispatcher : next_batch() takes the longest prefix of unsubmitted
//                requests whose fills are done (at most max_batch) into a
//                free slot, launched() hands the slot to the completer;
//   completer  : next_done() takes the oldest launched slot, complete()
//                marks its requests done, frees their ring space (batches
//                complete in FIFO order), wakes exactly those callers and
//                frees the slot.
#pragma once

#include <stdint.h>

#include <condition_variable>
#include <deque>
#include <mutex>
#include <vector>

namespace pyas {

enum QState { kReserved = 0, kFilled = 1, kSkip = 2, kSubmitted = 3, kDone = 4 };

// One caller's request; the coalescer's request type derives from it.
struct QItem {
    int64_t ring_off = 0, span = 0;
    int state = kReserved;
    std::condition_variable cv;   // state == kDone (waited on with the queue's mutex)
};

// Slot: one batch in flight; it must hold `std::vector<Item *> batch`.
template <class Item, class Slot>
class BatchQueue {
  public:
    BatchQueue(int64_t ring_bytes, int32_t max_batch) : ring_bytes_(ring_bytes), max_batch_(max_batch) {}

    std::mutex mu;

    int64_t ring_bytes() const { return ring_bytes_; }

    void add_slot(Slot *sl) {
        std::lock_guard<std::mutex> lk(mu);
        free_slots_.push_back(sl);
    }

    // -- callers ------------------------------------------------------------
    // Reserve it->span bytes and queue `it` in ring order.  False when the
    // queue is stopping or the span can never fit.
    bool reserve(Item *it) {
        std::unique_lock<std::mutex> lk(mu);
        const int64_t off = ring_reserve(lk, it->span);
        if (off < 0) return false;
        it->ring_off = off;
        it->state = kReserved;
        fifo_.push_back(it);
        return true;
    }

    // The request's bytes are in place (ok) or it cannot run: hand it to
    // the dispatcher and wait until its batch has completed.  `after` runs
    // under the lock once it has.
    template <class F>
    void finish(Item *it, bool ok, F &&after) {
        std::unique_lock<std::mutex> lk(mu);
        it->state = ok ? kFilled : kSkip;
        cv_disp_.notify_one();
        it->cv.wait(lk, [&] { return it->state == kDone; });
        after();
    }

    // -- dispatcher -----------------------------------------------------------
    // The next batch in a free slot (its requests move to kSubmitted); false
    // when stopping with nothing unsubmitted.
    bool next_batch(Slot *&out) {
        std::unique_lock<std::mutex> lk(mu);
        auto ready = [&] { return (int64_t)fifo_.size() > n_sub_ && fifo_[n_sub_]->state != kReserved; };
        cv_disp_.wait(lk, [&] { return ready() || (stop_ && (int64_t)fifo_.size() == n_sub_); });
        if (!ready()) return false;
        cv_slot_.wait(lk, [&] { return !free_slots_.empty(); });
        Slot *sl = free_slots_.front();
        free_slots_.pop_front();
        sl->batch.clear();
        for (int64_t i = n_sub_; i < (int64_t)fifo_.size(); ++i) {
            Item *r = fifo_[i];
            if ((int32_t)sl->batch.size() >= max_batch_) break;
            if (r->state != kFilled && r->state != kSkip) break;
            sl->batch.push_back(r);
        }
        for (Item *r : sl->batch)
            if (r->state == kFilled) r->state = kSubmitted;
        n_sub_ += (int64_t)sl->batch.size();
        out = sl;
        return true;
    }

    // The batch is enqueued on the device; `under` runs under the lock.
    template <class F>
    void launched(Slot *sl, F &&under) {
        std::lock_guard<std::mutex> lk(mu);
        under();
        inflight_.push_back(sl);
        cv_comp_.notify_one();
    }

    void dispatcher_done() {
        std::lock_guard<std::mutex> lk(mu);
        disp_done_ = true;
        cv_comp_.notify_one();
    }

    // -- completer --------------------------------------------------------------
    // The oldest launched batch; false once the dispatcher has stopped and
    // every batch completed.
    bool next_done(Slot *&out) {
        std::unique_lock<std::mutex> lk(mu);
        cv_comp_.wait(lk, [&] { return !inflight_.empty() || disp_done_; });
        if (inflight_.empty()) return false;
        out = inflight_.front();
        inflight_.pop_front();
        return true;
    }

    // Complete `sl`: `under` runs under the lock first (it sees the requests'
    // states before they become kDone); then the requests are done, their
    // ring space is free, their callers wake and the slot is free.
    template <class F>
    void complete(Slot *sl, F &&under) {
        std::lock_guard<std::mutex> lk(mu);
        under();
        for (Item *r : sl->batch) r->state = kDone;
        // batches complete in submission order == the FIFO's order
        for (size_t i = 0; i < sl->batch.size(); ++i) fifo_.pop_front();
        n_sub_ -= (int64_t)sl->batch.size();
        // wake exactly this batch's callers (one condition variable each: a
        // shared notify_all would wake every waiting caller per batch)
        for (Item *r : sl->batch) r->cv.notify_one();
        sl->batch.clear();
        free_slots_.push_back(sl);
        cv_slot_.notify_one();
        cv_space_.notify_all();
    }

    // -- owner --------------------------------------------------------------------
    // Stop accepting reservations; the dispatcher drains what is queued.
    void stop() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop_ = true;
        }
        cv_disp_.notify_all();
        cv_space_.notify_all();
    }

  private:
    // Reserve `span` ring bytes (lock held): -1 if it can never fit or the
    // queue stops while waiting for space.
    int64_t ring_reserve(std::unique_lock<std::mutex> &lk, int64_t span) {
        if (span > ring_bytes_ || span <= 0) return -1;
        for (;;) {
            if (stop_) return -1;
            if (fifo_.empty()) {       // everything free: restart at 0
                head_ = span;
                return 0;
            }
            // in use: [front, head) when head > front, else [front, R) + [0, head)
            // (head == front with requests queued means full)
            const int64_t front = fifo_.front()->ring_off;
            if (head_ > front) {       // free: [head, R) and [0, front)
                if (ring_bytes_ - head_ >= span) {
                    const int64_t off = head_;
                    head_ += span;
                    return off;
                }
                if (front >= span) {   // wrap
                    head_ = span;
                    return 0;
                }
            } else if (head_ < front && front - head_ >= span) {   // free: [head, front)
                const int64_t off = head_;
                head_ += span;
                return off;
            }
            cv_space_.wait(lk);
        }
    }

    int64_t ring_bytes_;
    int32_t max_batch_;
    int64_t head_ = 0;             // next free byte
    std::deque<Item *> fifo_;      // reservation order == ring order
    int64_t n_sub_ = 0;            // fifo_[0, n_sub_) are submitted, in flight
    std::deque<Slot *> free_slots_, inflight_;
    std::condition_variable cv_disp_, cv_space_, cv_comp_, cv_slot_;
    bool stop_ = false;
    bool disp_done_ = false;
};

}  // namespace pyas
