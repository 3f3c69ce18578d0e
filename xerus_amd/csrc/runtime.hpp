// Internal runtime of libxerus_amd: handle (stream + caching allocator + profiler), error plumbing.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/xerus_amd.h"

namespace xrs {

// ---------------------------------------------------------------------------------------------
// Errors: the C-ABI returns int status codes; internally we throw and convert at the boundary.
struct Error {
    int code;
    std::string msg;
};

void set_last_error(const std::string& msg);

#define XRS_REQUIRE(cond, msg)                                                          \
    do {                                                                                \
        if (!(cond)) {                                                                  \
            throw ::xrs::Error{XRS_EINVAL, std::string(__func__) + ": " + (msg)};      \
        }                                                                               \
    } while (0)

#define XRS_HIP(call)                                                                   \
    do {                                                                                \
        hipError_t e_ = (call);                                                         \
        if (e_ != hipSuccess) {                                                         \
            throw ::xrs::Error{XRS_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)}; \
        }                                                                               \
    } while (0)

// Run `body` and translate exceptions into C status codes.
template <class F>
int guarded(F&& body) {
    try {
        body();
        return XRS_OK;
    } catch (const Error& e) {
        set_last_error(e.msg);
        return e.code;
    } catch (const std::exception& e) {
        set_last_error(e.what());
        return XRS_EINVAL;
    }
}

// ---------------------------------------------------------------------------------------------
// Stream-ordered caching allocator. All work of a handle runs on one stream, so a block freed on
// the host may be handed to a later launch on the same stream immediately.
class Pool {
   public:
    explicit Pool(int device) : device_(device) {}
    ~Pool();
    void* alloc(size_t bytes);
    void release(void* p);
    size_t held_bytes() const { return held_; }
    void trim();

   private:
    int device_;
    std::multimap<size_t, void*> free_;
    std::unordered_map<void*, size_t> live_;
    size_t held_ = 0;
};

struct ProfRecord {
    hipEvent_t start, stop;
    double flops, bytes;
};

}  // namespace xrs

namespace xrs {
class DotWorker;
void destroy_dot_worker(xrs_handle_t h);   // tt.hip
}  // namespace xrs

struct xrs_handle_s {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    xrs::Pool* pool = nullptr;
    // pinned host scratch for returning scalars / statuses
    void* host_scratch = nullptr;
    // device scratch for reductions / statuses (64 KiB)
    void* dev_scratch = nullptr;
    // side streams (each with its own stream-ordered pool) for independent work forked from `stream`
    static constexpr int kSides = 3;
    hipStream_t side_stream[kSides] = {};
    xrs::Pool* side_pool[kSides] = {};
    hipEvent_t ev_fork = nullptr, ev_join[kSides] = {};
    hipEvent_t ev_aux = nullptr;   // one extra cross-stream dependency inside a fork (see tt.hip chain_pass)
    // split-K arrival tickets (zero between launches; the last arriving slice resets its word), one
    // array per stream so concurrent launches never share a word; `tickets` follows `stream`
    static constexpr int kTicketCap = 4096;
    int* ticket_base = nullptr;
    int* tickets = nullptr;
    int* side_tickets[kSides] = {};
    // algorithm of the last TT round (XRS_ROUND_*)
    int last_round_path = 0;
    // asynchronous TT inner product (xrs_tt_dot_async): enqueued by a worker thread on a child handle
    // whose streams are side streams 1 and 2 of this one (forked at ev_dot from the main stream), so the
    // caller's thread goes on enqueueing the next work at once; while `reader_pending`, releases of the
    // handle's blocks first wait until the product has finished (fence_readers)
    hipEvent_t ev_dot = nullptr, ev_dot_join = nullptr;
    bool reader_pending = false;
    bool dot_pending = false;
    xrs::DotWorker* dot_worker = nullptr;
    bool borrowed_streams = false;   // child handle: streams belong to the parent
    // profiler
    uint32_t prof_mask = 0;
    std::vector<xrs::ProfRecord> prof;
    std::vector<hipEvent_t> event_cache;
};

namespace xrs {

// RAII device buffer from the handle's pool.
struct DevBuf {
    xrs_handle_t h = nullptr;
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(xrs_handle_t h_, size_t bytes_) : h(h_), bytes(bytes_) { p = bytes_ ? h_->pool->alloc(bytes_) : nullptr; }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : h(o.h), p(o.p), bytes(o.bytes) { o.p = nullptr; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        reset();
        h = o.h; p = o.p; bytes = o.bytes; o.p = nullptr;
        return *this;
    }
    ~DevBuf() { reset(); }
    void reset() {
        if (p) h->pool->release(p);
        p = nullptr;
    }
    double* d() const { return static_cast<double*>(p); }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

// Kernel-duration instrumentation (xrs_prof_begin/end).
class KernelTimer {
   public:
    // dispatch = true: the caller launches with hipExtLaunchKernelGGL(..., start(), stop(), 0, ...), so the
    // events carry the dispatch's own begin / end timestamps (the kernel-trace duration a profiler reports)
    // instead of marker packets around it (which add the dispatch latency: ~6 us per TT-shape GEMM)
    KernelTimer(xrs_handle_t h, uint32_t family, double flops, double bytes, bool dispatch = false);
    ~KernelTimer();
    hipEvent_t start() const { return on_ ? rec_.start : nullptr; }
    hipEvent_t stop() const { return on_ ? rec_.stop : nullptr; }

   private:
    xrs_handle_t h_;
    bool on_, dispatch_;
    ProfRecord rec_{};
};

void check_launch(const char* what);

// Diagnostic cycle / time stamps (stderr), off by default: XRS_STAMPS is a comma-separated list of
// "round" (host phase marks of round()), "svd" (block Jacobi phase cycles of xrs_svd_rows_vt), "syev"
// (tridiagonalisation column-step cycles), or "all".
bool stamps_enabled(const char* what);

// Runs the handle's launches on another stream for one scope (the main stream is restored on scope exit,
// also when a launch throws). The caller orders the two streams (events).
class StreamSwap {
   public:
    StreamSwap(xrs_handle_t h, hipStream_t s) : h_(h), saved_(h->stream) { h_->stream = s; }
    ~StreamSwap() { h_->stream = saved_; }
    StreamSwap(const StreamSwap&) = delete;
    StreamSwap& operator=(const StreamSwap&) = delete;
   private:
    xrs_handle_t h_;
    hipStream_t saved_;
};

// Host wait for everything enqueued on h->stream so far (the read-backs of a TT call: a scalar, the round's
// check values). (Polling an event instead measured no difference: 1.3361 vs 1.3305 ms/step.)
void host_wait(xrs_handle_t h);

// Order the current stream after an in-flight asynchronous reader of the handle's blocks (the async
// TT inner product): a host wait for it (opening its gate first); no-op when none is pending. Called
// before a block is released and by every C-ABI entry point that writes caller memory (xrs_scal,
// xrs_axpy, xrs_copy, xrs_upload, xrs_memset_zero, xrs_scale_rows, xrs_gemm*, xrs_permute, the
// factorisations and solves), so an in-place write to a core never races the product.
void fence_readers(xrs_handle_t h);
// blocks until the handle's asynchronous inner product (if any) has finished on the device (tt.hip)
void wait_dot_done(xrs_handle_t h);
// the worker's child handle (null before the first asynchronous inner product; tt.hip)
xrs_handle_t dot_child(xrs_handle_t h);

// Child handle for a worker thread: own pools, scratch, events and split-K tickets; main stream = the
// parent's side stream 1, side stream 0 = the parent's side stream 2 (borrowed, not destroyed).
xrs_handle_t create_child_handle(xrs_handle_t parent);

// Fork/join of independent work onto the handle's side stream. While `side()` is active every launch
// and DevBuf of the handle goes to the side stream / side pool (stream-ordered reuse stays valid);
// buffers shared across the fork must be allocated before it and released after join().
class StreamFork {
   public:
    explicit StreamFork(xrs_handle_t h, int sides = 1);
    ~StreamFork();
    void side(int i = 0);   // switch to side stream i < sides (after the fork point)
    void lane(int i);       // 0 = main stream, 1..sides = side stream i-1 (round-robin helper)
    void main();            // switch back
    void join();            // main stream waits for every side stream's work
    int lanes() const { return sides_ + 1; }
   private:
    xrs_handle_t h_;
    int sides_;
    hipStream_t main_stream_;
    Pool* main_pool_;
    int* main_tickets_;
    bool joined_ = false;
};

// an xrs_comm_emulate communicator (comm.cpp): its all-reduce is nranks x the local value
bool comm_is_emulated(const void* ctx);

}  // namespace xrs
