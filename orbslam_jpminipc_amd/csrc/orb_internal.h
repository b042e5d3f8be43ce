// orb_internal.h — host-side plumbing shared by the translation units of liborb_hip.so
// (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

// Records `msg` as the calling thread's orb_last_error() and returns `code`.
__attribute__((visibility("hidden"))) int orb_internal_set_error(int code, const std::string& msg);

// Per-thread, per-device state of the synchronous host-buffer entry points (matcher family,
// single-pair SearchForInitialization): a private non-blocking stream, a grow-only device
// arena and a grow-only pinned host staging buffer.  Each calling thread gets its own (the
// reference runs matchers concurrently from Tracking, LocalMapping and LoopClosing,
// main.cc:164-193), so calls from different threads overlap on the device instead of
// serialising; a context is returned to a pool when its thread exits and reused by the next
// thread (no HIP call at thread exit).  Calls only ever synchronise their own stream.
struct OrbHostCtx {
    int device = -1;
    hipStream_t stream = nullptr;
    uint8_t* buf = nullptr;     // device arena
    size_t cap = 0;
    uint8_t* pinned = nullptr;  // host staging (hipHostMalloc)
    size_t pcap = 0;
    // Grow the arena / staging to at least the given sizes (contents not preserved); creates
    // the stream on first use.  ORB_OK or ORB_EDEVICE (message set).
    int reserve(size_t dev_bytes, size_t host_bytes);
};
__attribute__((visibility("hidden"))) OrbHostCtx* orb_internal_thread_ctx(int device);
