// Device-side gather / re-shard of mode-sharded TTs (xerus itself is single-process).
//
// Layout (xerus_amd.dist.mode_partition): rank p holds, of every component k (r_k, n_k, r_{k+1}), the
// contiguous mode block [s_p, s_p + m_p) with m_p = n_k / P (+1 for the first n_k % P ranks). The gather
// pads every rank's slices to the largest block, concatenates them for all components into ONE buffer,
// runs ONE all-gather over it (xrs_allgather_fn: ncclAllGather on the handle's stream for the library's
// RCCL communicator, or a torch.distributed hook), and scatters the blocks into full cores with strided
// device copies: the fallback of a sharded round whose certificate fails (round the gathered TT on every
// rank, then re-shard locally) never moves core data through the host.
#include <algorithm>
#include <vector>

#include "runtime.hpp"

namespace xrs {
namespace {

void partition(size_t n, int world, int rank, size_t& start, size_t& count) {
    const size_t base = n / size_t(world), extra = n % size_t(world);
    start = size_t(rank) * base + std::min(size_t(rank), extra);
    count = base + (size_t(rank) < extra ? 1 : 0);
}

}  // namespace
}  // namespace xrs

using namespace xrs;

extern "C" {

int xrs_tt_gather_sharded(xrs_handle_t h, size_t d, const size_t* n_global, int world, int rank, const size_t* r,
                          const double* const* local, double** full_out, xrs_allgather_fn allgather, void* ctx) {
    return guarded([&] {
        XRS_REQUIRE(h && n_global && r && local && full_out, "null argument");
        XRS_REQUIRE(world >= 1 && rank >= 0 && rank < world, "invalid rank / world size");
        XRS_REQUIRE(world == 1 || allgather, "an all-gather hook is needed for more than one rank");
        XRS_REQUIRE(d >= 1 && r[0] == 1 && r[d] == 1, "boundary ranks must be 1");
        fence_readers(h);
        // per component: padded block (r_k, mmax_k, r_{k+1}) at offset off[k] of every rank's segment
        std::vector<size_t> off(d + 1, 0), mmax(d);
        for (size_t k = 0; k < d; ++k) {
            XRS_REQUIRE(n_global[k] >= 1, "mode sizes must be positive");
            mmax[k] = (n_global[k] + size_t(world) - 1) / size_t(world);
            off[k + 1] = off[k] + r[k] * mmax[k] * r[k + 1];
        }
        const size_t seg = std::max<size_t>(off[d], 1);
        DevBuf send(h, seg * 8), recv(h, seg * size_t(world) * 8);
        XRS_HIP(hipMemsetAsync(send.d(), 0, seg * 8, h->stream));
        for (size_t k = 0; k < d; ++k) {
            size_t s, m;
            partition(n_global[k], world, rank, s, m);
            if (m == 0) continue;
            XRS_REQUIRE(local[k], "null local core");
            // (r, m, r') into the (r, mmax, r') block: r rows of m r' doubles
            XRS_HIP(hipMemcpy2DAsync(send.d() + off[k], mmax[k] * r[k + 1] * 8, local[k], m * r[k + 1] * 8, m * r[k + 1] * 8, r[k],
                                     hipMemcpyDeviceToDevice, h->stream));
        }
        if (world == 1) {
            XRS_HIP(hipMemcpyAsync(recv.d(), send.d(), seg * 8, hipMemcpyDeviceToDevice, h->stream));
        } else {
            if (allgather != &xrs_comm_allgather) XRS_HIP(hipStreamSynchronize(h->stream));
            XRS_REQUIRE(allgather(ctx, send.d(), recv.d(), seg) == 0, "all-gather callback failed");
        }
        for (size_t k = 0; k < d; ++k) {
            const size_t n = n_global[k], rb = r[k + 1];
            double* full = static_cast<double*>(h->pool->alloc(std::max<size_t>(r[k] * n * rb, 1) * 8));
            full_out[k] = full;
            for (int p = 0; p < world; ++p) {
                size_t s, m;
                partition(n, world, p, s, m);
                if (m == 0) continue;
                const double* src = recv.d() + size_t(p) * seg + off[k];
                XRS_HIP(hipMemcpy2DAsync(full + s * rb, n * rb * 8, src, mmax[k] * rb * 8, m * rb * 8, r[k], hipMemcpyDeviceToDevice,
                                         h->stream));
            }
        }
        XRS_HIP(hipStreamSynchronize(h->stream));   // (the hook's buffers are released on return)
    });
}

int xrs_tt_shard(xrs_handle_t h, size_t d, const size_t* n_global, int world, int rank, const size_t* r, const double* const* full,
                 double** local_out) {
    return guarded([&] {
        XRS_REQUIRE(h && n_global && r && full && local_out, "null argument");
        XRS_REQUIRE(world >= 1 && rank >= 0 && rank < world, "invalid rank / world size");
        fence_readers(h);
        for (size_t k = 0; k < d; ++k) {
            size_t s, m;
            partition(n_global[k], world, rank, s, m);
            const size_t rb = r[k + 1];
            double* loc = static_cast<double*>(h->pool->alloc(std::max<size_t>(r[k] * m * rb, 1) * 8));
            local_out[k] = loc;
            if (m) XRS_HIP(hipMemcpy2DAsync(loc, m * rb * 8, full[k] + s * rb, n_global[k] * rb * 8, m * rb * 8, r[k], hipMemcpyDeviceToDevice,
                                            h->stream));
        }
    });
}

}  // extern "C"
