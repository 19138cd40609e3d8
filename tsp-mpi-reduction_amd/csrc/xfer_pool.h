// Pinned-slot bookkeeping of the small-transfer path (xfer.hip), without HIP:
// the slot claim and release logic is plain C++ over an event backend B, so
// the host-only thread test (host/check_xfer.cpp, ThreadSanitizer) runs the
// same code as the library.
//
// One pool per device.  The pool's mutex is held only to look at slot flags
// and to query events (non-blocking); no thread ever waits on a stream or an
// event while holding it.  A copy waits only on work of its OWN stream: it
// takes a free slot whose last copy has completed, else a free slot whose
// still-pending last copy was enqueued on the caller's stream (the caller
// waits on that event after the lock is released — in-order work it queued
// itself), else no slot at all (the caller uses the runtime copy path).  So a
// slot whose event sits behind another thread's collective can never block a
// copy on a different stream (round-5 ADVICE: the old single pool held one
// process-wide mutex across hipEventSynchronize / hipStreamSynchronize).
//
// Backend B: types Event and Stream (Stream equality-comparable);
//   bool alloc(Slot &)  pinned host buffer + event for a slot (false: broken)
//   bool done(Event)    non-blocking completion query
#pragma once
#include <cstddef>
#include <mutex>

namespace tspgpu {

template <class B, int kSlots = 8>
class XferPool {
public:
    using Event = typename B::Event;
    using Stream = typename B::Stream;
    struct Slot {
        char *h = nullptr;
        Event ev{};
        Stream st{};           // stream of the last copy through the slot
        bool pending = false;  // ev (behind that copy) not yet seen complete
        bool busy = false;     // claimed by a thread
    };

    explicit XferPool(B b = B()) : b_(b) {}

    // A slot for a copy on stream st, or null.  *wait: the slot's last copy
    // was on st and may still run — wait on s->ev (outside the pool) first.
    Slot *claim(Stream st, bool *wait)
    {
        std::lock_guard<std::mutex> g(mu_);
        *wait = false;
        if (broken_) return nullptr;
        Slot *same = nullptr;
        for (int i = 0; i < kSlots; ++i) {
            Slot &s = s_[(next_ + i) % kSlots];
            if (s.busy) continue;
            if (!s.h && !b_.alloc(s)) {
                broken_ = true;
                return nullptr;
            }
            if (s.pending && b_.done(s.ev)) s.pending = false;
            if (!s.pending) {
                s.busy = true;
                next_ = (next_ + i + 1) % kSlots;
                return &s;
            }
            if (!same && s.st == st) same = &s;
        }
        if (same) {
            same->busy = true;
            *wait = true;
        }
        return same;
    }
    // Hands the slot back; pending: an event behind this copy was recorded on st.
    void release(Slot *s, Stream st, bool pending)
    {
        std::lock_guard<std::mutex> g(mu_);
        s->st = st;
        s->pending = pending;
        s->busy = false;
    }
    bool broken()
    {
        std::lock_guard<std::mutex> g(mu_);
        return broken_;
    }

private:
    std::mutex mu_;
    Slot s_[kSlots];
    int next_ = 0;
    bool broken_ = false;  // a pinned allocation failed once: the runtime path from then on
    B b_;
};

}  // namespace tspgpu
