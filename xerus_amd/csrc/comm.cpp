// RCCL communicator for the mode-sharded TT entry points (xerus itself is single-process).
//
// xrs_comm_allreduce is an xrs_allreduce_fn whose ctx is an xrs_comm_t: it ENQUEUES ncclAllReduce (sum,
// fp64, in place) on the handle's current stream and returns -- the TT drivers recognise it and skip the
// host synchronisation a host-side hook needs, so a sharded round is a stream-ordered chain of kernels and
// collectives over xGMI with no host round trip per edge. RCCL is loaded at run time (dlopen): the
// library stays loadable where no RCCL is installed, and inside a PyTorch process the already-loaded copy
// is reused. The unique id is exchanged by the caller (xerus_amd.dist: torch.distributed broadcast).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>

#include "elementwise.hpp"
#include "runtime.hpp"

struct xrs_comm_s {
    ncclComm_t comm = nullptr;
    xrs_handle_t h = nullptr;
    int nranks = 1, rank = 0;
    size_t calls = 0, bytes = 0;
    bool emulated = false;   // xrs_comm_emulate: no RCCL; the sum over ranks is nranks x the local value
};

namespace xrs {
namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    bool ok = false;
    std::string why;
};

const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* lib = nullptr;
        for (const char* name : {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so.1"}) {
            lib = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (lib) break;
        }
        if (!lib) {
            x.why = std::string("cannot load librccl: ") + dlerror();
            return x;
        }
        x.get_unique_id = reinterpret_cast<decltype(x.get_unique_id)>(dlsym(lib, "ncclGetUniqueId"));
        x.init_rank = reinterpret_cast<decltype(x.init_rank)>(dlsym(lib, "ncclCommInitRank"));
        x.all_reduce = reinterpret_cast<decltype(x.all_reduce)>(dlsym(lib, "ncclAllReduce"));
        x.all_gather = reinterpret_cast<decltype(x.all_gather)>(dlsym(lib, "ncclAllGather"));
        x.destroy = reinterpret_cast<decltype(x.destroy)>(dlsym(lib, "ncclCommDestroy"));
        x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(lib, "ncclGetErrorString"));
        x.ok = x.get_unique_id && x.init_rank && x.all_reduce && x.all_gather && x.destroy && x.error_string;
        if (!x.ok) x.why = "librccl lacks the nccl* entry points";
        return x;
    }();
    return r;
}

void check_nccl(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw Error{XRS_EHIP, std::string(what) + ": " + rccl().error_string(r)};
}

}  // namespace

// an xrs_comm_emulate communicator (the per-rank timing probe): its all-reduce is nranks x the local value,
// so a zero-padded core "gathered" through it is not the TT's core (tt_trunc.hip: shard_layout)
bool comm_is_emulated(const void* ctx) { return ctx && static_cast<const xrs_comm_s*>(ctx)->emulated; }

}  // namespace xrs

using namespace xrs;

extern "C" {

int xrs_comm_unique_id(void* id_out) {
    return guarded([&] {
        XRS_REQUIRE(id_out, "null id buffer");
        XRS_REQUIRE(rccl().ok, rccl().why);
        ncclUniqueId id;
        check_nccl(rccl().get_unique_id(&id), "ncclGetUniqueId");
        std::memcpy(id_out, &id, sizeof(id));
    });
}

int xrs_comm_create(xrs_handle_t h, int nranks, int rank, const void* id, xrs_comm_t* out) {
    return guarded([&] {
        XRS_REQUIRE(h && id && out, "null argument");
        XRS_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "invalid rank / world size");
        XRS_REQUIRE(rccl().ok, rccl().why);
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof(uid));
        XRS_HIP(hipSetDevice(h->device));
        auto* c = new xrs_comm_s;
        c->h = h;
        c->nranks = nranks;
        c->rank = rank;
        const ncclResult_t r = rccl().init_rank(&c->comm, nranks, uid, rank);
        if (r != ncclSuccess) {
            delete c;
            check_nccl(r, "ncclCommInitRank");
        }
        *out = c;
    });
}

int xrs_comm_emulate(xrs_handle_t h, int nranks, xrs_comm_t* out) {
    return guarded([&] {
        XRS_REQUIRE(h && out, "null argument");
        XRS_REQUIRE(nranks >= 1, "invalid world size");
        auto* c = new xrs_comm_s;
        c->h = h;
        c->nranks = nranks;
        c->emulated = true;
        *out = c;
    });
}

int xrs_comm_destroy(xrs_comm_t c) {
    return guarded([&] {
        if (!c) return;
        if (c->comm) check_nccl(rccl().destroy(c->comm), "ncclCommDestroy");
        delete c;
    });
}

size_t xrs_comm_calls(xrs_comm_t c) { return c ? c->calls : 0; }

int xrs_comm_allreduce(void* ctx, double* buf, size_t count) {
    auto* c = static_cast<xrs_comm_s*>(ctx);
    if (!c || !(c->comm || c->emulated) || (count && !buf)) return 1;
    ++c->calls;
    c->bytes += count * 8;
    if (count == 0) return 0;
    if (c->emulated) {   // nranks identical slices: the sum is nranks x the local value, in stream order
        try {
            xrs::scal(c->h, buf, double(c->nranks), count);
        } catch (...) {
            return 1;
        }
        return 0;
    }
    return rccl().all_reduce(buf, buf, count, ncclDouble, ncclSum, c->comm, c->h->stream) == ncclSuccess ? 0 : 1;
}

int xrs_comm_allgather(void* ctx, const double* send, double* recv, size_t count) {
    auto* c = static_cast<xrs_comm_s*>(ctx);
    if (!c || !c->comm || c->emulated || (count && !(send && recv))) return 1;
    ++c->calls;
    c->bytes += count * 8 * size_t(c->nranks);
    if (count == 0) return 0;
    return rccl().all_gather(send, recv, count, ncclDouble, c->comm, c->h->stream) == ncclSuccess ? 0 : 1;
}

}  // extern "C"
