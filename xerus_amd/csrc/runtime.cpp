// Handle, stream, caching allocator, profiler and the runtime part of the C-ABI.
#include "runtime.hpp"

#include <algorithm>

#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace xrs {

static thread_local std::string g_last_error;

void set_last_error(const std::string& msg) { g_last_error = msg; }

Pool::~Pool() { trim(); }

static size_t round_size(size_t bytes) {
    if (bytes <= (1u << 20)) {
        size_t s = 256;
        while (s < bytes) s <<= 1;
        return s;
    }
    return (bytes + (1u << 20) - 1) & ~size_t((1u << 20) - 1);
}

void* Pool::alloc(size_t bytes) {
    const size_t sz = round_size(bytes);
    auto it = free_.lower_bound(sz);
    if (it != free_.end() && it->first <= sz + sz / 4) {
        void* p = it->second;
        live_[p] = it->first;
        free_.erase(it);
        return p;
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, sz);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        // give cached blocks back and retry once
        trim();
        e = hipMalloc(&p, sz);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            throw Error{XRS_ENOMEM, "device allocation of " + std::to_string(sz) + " bytes failed"};
        }
    }
    live_[p] = sz;
    held_ += sz;
    return p;
}

void Pool::release(void* p) {
    auto it = live_.find(p);
    if (it == live_.end()) throw Error{XRS_EINVAL, "xrs_free: pointer not owned by this handle"};
    free_.emplace(it->second, p);
    live_.erase(it);
}

void Pool::trim() {
    if (free_.empty()) return;
    (void)hipDeviceSynchronize();
    for (auto& kv : free_) {
        (void)hipFree(kv.second);
        held_ -= kv.first;
    }
    free_.clear();
}

KernelTimer::KernelTimer(xrs_handle_t h, uint32_t family, double flops, double bytes, bool dispatch)
    : h_(h), on_((h->prof_mask & family) != 0), dispatch_(dispatch) {
    if (!on_) return;
    auto get = [&]() {
        hipEvent_t e;
        if (!h_->event_cache.empty()) {
            e = h_->event_cache.back();
            h_->event_cache.pop_back();
        } else {
            XRS_HIP(hipEventCreate(&e));
        }
        return e;
    };
    rec_.start = get();
    rec_.stop = get();
    rec_.flops = flops;
    rec_.bytes = bytes;
    if (!dispatch_) XRS_HIP(hipEventRecord(rec_.start, h_->stream));
}

KernelTimer::~KernelTimer() {
    if (!on_) return;
    if (!dispatch_) (void)hipEventRecord(rec_.stop, h_->stream);
    h_->prof.push_back(rec_);
}

static int sync_debug() {
    static int v = [] {
        const char* e = std::getenv("XRS_SYNC_DEBUG");
        return (e && *e && *e != '0') ? 1 : 0;
    }();
    return v;
}

void host_wait(xrs_handle_t h) { XRS_HIP(hipStreamSynchronize(h->stream)); }

void fence_readers(xrs_handle_t h) {
    if (!h->reader_pending) return;
    // the worker thread has synchronised the product's streams when it reports done: afterwards no
    // device work reads the handle's blocks any more (a host wait, normally already satisfied: the
    // round releases x's old cores after its own check synchronisation)
    wait_dot_done(h);
    h->reader_pending = false;
}

bool stamps_enabled(const char* what) {
    const char* e = std::getenv("XRS_STAMPS");
    if (!e || !*e) return false;
    const std::string list = std::string(",") + e + ",";
    return list.find(",all,") != std::string::npos || list.find(std::string(",") + what + ",") != std::string::npos;
}

void check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw Error{XRS_EHIP, std::string(what) + ": " + hipGetErrorString(e)};
    if (sync_debug()) {
        std::fprintf(stderr, "[xrs] launched %s\n", what);
        std::fflush(stderr);
        e = hipDeviceSynchronize();
        std::fprintf(stderr, "[xrs]   done %s: %s\n", what, hipGetErrorString(e));
        std::fflush(stderr);
        if (e != hipSuccess) throw Error{XRS_EHIP, std::string(what) + ": " + hipGetErrorString(e)};
    }
}

}  // namespace xrs

using namespace xrs;

extern "C" {

const char* xrs_last_error(void) { return g_last_error.c_str(); }
const char* xrs_version(void) { return "xerus_amd 0.1 (gfx950)"; }

// Cross-stream dependencies: hipEventRecord + hipStreamWaitEvent. (Stream write-value / wait-value
// packets measured 8.7 vs 17.7 us for one isolated hop, tools/boundary_bench.hip, but the bench step did not
// get faster, 1.46 vs 1.43 ms, so events stay.)
static void stream_signal(hipStream_t producer, hipStream_t consumer, hipEvent_t ev) {
    XRS_HIP(hipEventRecord(ev, producer));
    XRS_HIP(hipStreamWaitEvent(consumer, ev, 0));
}

StreamFork::StreamFork(xrs_handle_t h, int sides)
    : h_(h), sides_(std::max(1, std::min(sides, int(xrs_handle_s::kSides)))), main_stream_(h->stream), main_pool_(h->pool),
      main_tickets_(h->tickets) {
    XRS_HIP(hipEventRecord(h_->ev_fork, main_stream_));
    for (int i = 0; i < sides_; ++i) XRS_HIP(hipStreamWaitEvent(h_->side_stream[i], h_->ev_fork, 0));
}

void StreamFork::side(int i) {
    // while kernels are being timed (xrs_prof_begin), the fork's lanes all stay on the main stream: every
    // event pair then brackets exactly one kernel (with concurrent lanes it also spans the time a kernel
    // waits for CUs held by the other lane's kernels), so the event durations agree with a kernel trace
    if (h_->prof_mask) return;
    h_->stream = h_->side_stream[i];
    h_->pool = h_->side_pool[i];
    h_->tickets = h_->side_tickets[i];
}

void StreamFork::lane(int i) {
    if (i <= 0) main();
    else side((i - 1) % sides_);
}

void StreamFork::main() {
    h_->stream = main_stream_;
    h_->pool = main_pool_;
    h_->tickets = main_tickets_;
}

void StreamFork::join() {
    if (joined_) return;
    joined_ = true;
    main();
    for (int i = 0; i < sides_; ++i) stream_signal(h_->side_stream[i], main_stream_, h_->ev_join[i]);
}

StreamFork::~StreamFork() {
    try {
        join();
    } catch (...) {
    }
}

static void init_handle_resources(xrs_handle_t h);

int xrs_create(xrs_handle_t* handle, int device) {
    return guarded([&] {
        XRS_REQUIRE(handle != nullptr, "null handle pointer");
        int count = 0;
        XRS_HIP(hipGetDeviceCount(&count));
        XRS_REQUIRE(device >= 0 && device < count, "device index out of range");
        XRS_HIP(hipSetDevice(device));
        auto* h = new xrs_handle_s();
        h->device = device;
        XRS_HIP(hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking));
        h->stream = h->own_stream;
        // side streams 1 and 2 carry the asynchronous inner product at the lowest queue priority, so the
        // work enqueued beside it (the round on the main stream) is dispatched first and the product
        // fills the gaps (bench step 1.19 -> 1.16 ms)
        int prio_least = 0, prio_greatest = 0;
        (void)hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
        for (int i = 0; i < xrs_handle_s::kSides; ++i) {
            if (i >= 1 && prio_least != prio_greatest)
                XRS_HIP(hipStreamCreateWithPriority(&h->side_stream[i], hipStreamNonBlocking, prio_least));
            else
                XRS_HIP(hipStreamCreateWithFlags(&h->side_stream[i], hipStreamNonBlocking));
        }
        init_handle_resources(h);
        *handle = h;
    });
}

}  // extern "C"

xrs_handle_t xrs::create_child_handle(xrs_handle_t parent) {
    auto* h = new xrs_handle_s();
    h->device = parent->device;
    h->borrowed_streams = true;
    h->own_stream = parent->side_stream[1];
    h->stream = h->own_stream;
    h->side_stream[0] = parent->side_stream[2];
    h->side_stream[1] = parent->side_stream[1];   // (never forked to: the child forks with one side)
    h->side_stream[2] = parent->side_stream[2];
    try {
        init_handle_resources(h);
    } catch (...) {
        delete h;
        throw;
    }
    return h;
}

static void init_handle_resources(xrs_handle_t h) {
    {
        const int device = h->device;
        h->pool = new Pool(device);
        for (int i = 0; i < xrs_handle_s::kSides; ++i) {
            h->side_pool[i] = new Pool(device);
            XRS_HIP(hipEventCreateWithFlags(&h->ev_join[i], hipEventDisableTiming));
        }
        XRS_HIP(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
        XRS_HIP(hipEventCreateWithFlags(&h->ev_aux, hipEventDisableTiming));
        XRS_HIP(hipEventCreateWithFlags(&h->ev_dot, hipEventDisableTiming));
        XRS_HIP(hipEventCreateWithFlags(&h->ev_dot_join, hipEventDisableTiming));
        XRS_HIP(hipHostMalloc(&h->host_scratch, 1 << 16, hipHostMallocDefault));
        XRS_HIP(hipMalloc(&h->dev_scratch, 1 << 16));
        const size_t tbytes = size_t(1 + xrs_handle_s::kSides) * xrs_handle_s::kTicketCap * sizeof(int);
        XRS_HIP(hipMalloc(&h->ticket_base, tbytes));
        XRS_HIP(hipMemset(h->ticket_base, 0, tbytes));
        h->tickets = h->ticket_base;
        for (int i = 0; i < xrs_handle_s::kSides; ++i)
            h->side_tickets[i] = h->ticket_base + size_t(1 + i) * xrs_handle_s::kTicketCap;
        // the zeroed tickets must be in place before any (non-blocking) stream uses them
        XRS_HIP(hipDeviceSynchronize());
    }
}

extern "C" {

int xrs_destroy(xrs_handle_t h) {
    return guarded([&] {
        if (!h) return;
        (void)hipSetDevice(h->device);
        destroy_dot_worker(h);   // (joins the worker thread and destroys its child handle)
        (void)hipStreamSynchronize(h->stream);
        for (auto& r : h->prof) {
            (void)hipEventDestroy(r.start);
            (void)hipEventDestroy(r.stop);
        }
        for (auto e : h->event_cache) (void)hipEventDestroy(e);
        for (auto s : h->side_stream)
            if (s) (void)hipStreamSynchronize(s);
        delete h->pool;
        for (int i = 0; i < xrs_handle_s::kSides; ++i) {
            delete h->side_pool[i];
            if (h->side_stream[i] && !h->borrowed_streams) (void)hipStreamDestroy(h->side_stream[i]);
            if (h->ev_join[i]) (void)hipEventDestroy(h->ev_join[i]);
        }
        if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
        if (h->ev_aux) (void)hipEventDestroy(h->ev_aux);
        if (h->ev_dot) (void)hipEventDestroy(h->ev_dot);
        if (h->ev_dot_join) (void)hipEventDestroy(h->ev_dot_join);
        (void)hipHostFree(h->host_scratch);
        (void)hipFree(h->dev_scratch);
        (void)hipFree(h->ticket_base);
        if (h->own_stream && !h->borrowed_streams) (void)hipStreamDestroy(h->own_stream);
        delete h;
    });
}

int xrs_set_stream(xrs_handle_t h, void* s) {
    return guarded([&] {
        XRS_REQUIRE(h, "null handle");
        hipStream_t next = s ? static_cast<hipStream_t>(s) : h->own_stream;
        // the pool and the split-K tickets are stream-ordered: drain the old stream before switching
        if (next != h->stream) XRS_HIP(hipStreamSynchronize(h->stream));
        h->stream = next;
    });
}

void* xrs_get_stream(xrs_handle_t h) { return h ? static_cast<void*>(h->stream) : nullptr; }

int xrs_synchronize(xrs_handle_t h) {
    return guarded([&] {
        XRS_REQUIRE(h, "null handle");
        XRS_HIP(hipStreamSynchronize(h->stream));
    });
}

int xrs_malloc(xrs_handle_t h, void** ptr, size_t bytes) {
    return guarded([&] {
        XRS_REQUIRE(h && ptr, "null argument");
        *ptr = bytes ? h->pool->alloc(bytes) : nullptr;
    });
}

int xrs_free(xrs_handle_t h, void* ptr) {
    return guarded([&] {
        XRS_REQUIRE(h, "null handle");
        if (!ptr) return;
        fence_readers(h);
        h->pool->release(ptr);
    });
}

size_t xrs_pool_bytes(xrs_handle_t h) { return h ? h->pool->held_bytes() : 0; }

int xrs_upload(xrs_handle_t h, double* dst, const double* src, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && (n == 0 || (dst && src)), "null argument");
        if (n == 0) return;
        fence_readers(h);
        XRS_HIP(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
        XRS_HIP(hipStreamSynchronize(h->stream));
    });
}

int xrs_download(xrs_handle_t h, double* dst, const double* src, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && (n == 0 || (dst && src)), "null argument");
        if (n == 0) return;
        XRS_HIP(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
        XRS_HIP(hipStreamSynchronize(h->stream));
    });
}

int xrs_memset_zero(xrs_handle_t h, double* dst, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && (n == 0 || dst), "null argument");
        if (n) fence_readers(h);
        if (n) XRS_HIP(hipMemsetAsync(dst, 0, n * sizeof(double), h->stream));
    });
}

int xrs_copy(xrs_handle_t h, double* dst, const double* src, size_t n) {
    return guarded([&] {
        XRS_REQUIRE(h && (n == 0 || (dst && src)), "null argument");
        if (n) fence_readers(h);
        if (n) XRS_HIP(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToDevice, h->stream));
    });
}

int xrs_prof_begin(xrs_handle_t h, uint32_t mask) {
    return guarded([&] {
        XRS_REQUIRE(h, "null handle");
        h->prof_mask = mask;
    });
}

int xrs_prof_end(xrs_handle_t h, size_t* launches, double* total_ms, double* flops, double* bytes) {
    return guarded([&] {
        XRS_REQUIRE(h, "null handle");
        h->prof_mask = 0;
        XRS_HIP(hipStreamSynchronize(h->stream));
        // records of the asynchronous inner product's worker (its child handle), once it has finished
        if (xrs_handle_t c = dot_child(h)) {
            wait_dot_done(h);
            c->prof_mask = 0;
            h->prof.insert(h->prof.end(), c->prof.begin(), c->prof.end());
            c->prof.clear();
        }
        double ms = 0, f = 0, b = 0;
        for (auto& r : h->prof) {
            float t = 0;
            XRS_HIP(hipEventElapsedTime(&t, r.start, r.stop));
            ms += t;
            f += r.flops;
            b += r.bytes;
            h->event_cache.push_back(r.start);
            h->event_cache.push_back(r.stop);
        }
        if (launches) *launches = h->prof.size();
        if (total_ms) *total_ms = ms;
        if (flops) *flops = f;
        if (bytes) *bytes = b;
        h->prof.clear();
    });
}

}  // extern "C"
