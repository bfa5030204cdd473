// Process-wide launch knobs of libclipembed (internal).
//
// The §8(b) threading contract (include/clipembed.h): one handle per device, any host thread,
// several handles driven from several threads at once (train_pacl.py:95 wraps the model in
// nn.DataParallel: one host thread per replica).  The only state outside the handles is the set of
// A/B knobs below (kernel variants, schedules) and per-device facts (CU count).  Each knob is an
// atomic int: its first reader publishes the environment's value with a compare-exchange from the
// "unset" sentinel, setters store atomically, and a launch reads each knob once and carries the
// value in its parameter block, so concurrent launches on any handles never race on them.  Per-device
// facts are cached per device ordinal, never "whichever device was current first".
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <climits>
#include <cstdlib>

namespace ce {

constexpr int kKnobUnset = INT_MIN;
constexpr int kMaxDevices = 64;

// Value of knob k; `init` (called at most once per losing race, result discarded unless it wins)
// gives the environment's value on first use.
template <class F>
inline int knob_get(std::atomic<int>& k, F&& init) {
    int v = k.load(std::memory_order_acquire);
    if (v == kKnobUnset) {
        int expect = kKnobUnset;
        const int want = init();
        k.compare_exchange_strong(expect, want, std::memory_order_acq_rel);
        v = k.load(std::memory_order_acquire);
    }
    return v;
}

// Atomically replace knob k (resolved first, so the previous value is the effective one).
template <class F>
inline int knob_set(std::atomic<int>& k, int v, F&& init) {
    knob_get(k, init);
    return k.exchange(v, std::memory_order_acq_rel);
}

inline int env_int(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return e ? std::atoi(e) : dflt;
}

inline int current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) dev = 0;
    return dev;
}

// Compute units of the current device (cached per device).
inline int device_cus() {
    static std::atomic<int> cache[kMaxDevices];
    const int dev = current_device();
    int n = cache[dev].load(std::memory_order_acquire);
    if (n <= 0) {
        int q = 0;
        if (hipDeviceGetAttribute(&q, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || q <= 0) q = 256;
        cache[dev].store(q, std::memory_order_release);
        n = q;
    }
    return n;
}

}  // namespace ce
