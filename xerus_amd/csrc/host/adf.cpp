// ADF (reference src/xerus/algorithms/adf.cpp:35-611) on the GPU. The algorithm, step by step, is the
// reference's InternalSolver:
//   solve (:566-604): canonicalize_left, one run at the current ranks, then -- while the residual is above
//     the target, the ranks below maxRanks and sweeps are left -- x += 1e-6 ||x|| r / ||r|| for a random
//     rank-1 TT r, round(maxRanks), and another run;
//   solve_with_current_ranks (:489-542): per sweep move_core(0, keepRank), rebuild the backward stacks,
//     the residual at component 0 and the stopping rule (target, or the product of the last four residual
//     ratios above minimalDecrease^4); then for every component: residual, projected gradient
//     E(A^T(b - Ax)), slice-wise ||A(E(grad))||^2, the component update, move_core(k + 1, keepRank) and the
//     forward stack.
// The stacks are dense M x r device matrices (adf.hip); the reference's de-duplication of equal position
// prefixes (construct_stacks :102-191) only shares identical products, so every measurement's stack entry
// is computed here and the values are the same. Residuals are evaluated with the component and both
// neighbouring stacks (F_{k-1} C B_{k+1}) instead of through whichever stack has fewer unique entries
// (:291-312): the same contraction in another order.
#include <cmath>
#include <limits>

#include "measurement_device.hpp"
#include "xerus/algorithms/adf.h"

namespace xerus {

namespace {

template <class F>
auto guard(F&& f) -> decltype(f()) {
    try {
        return f();
    } catch (const xrs::Error& e) {
        throw misc::generic_error(e.msg);
    }
}

class AdfSolver {
   public:
    AdfSolver(TTTensor& _x, const std::vector<size_t>& _maxRanks, internal::DeviceMeasurements& _dm, const ADFVariant& _v)
        : x(_x),
          d(_x.degree()),
          maxRanks(TTTensor::reduce_to_maximal_ranks(_maxRanks, _x.dimensions)),
          dm(_dm),
          M(_dm.M),
          var(_v),
          h(gpu::handle()) {
        _x.require_correct_format();
        XERUS_REQUIRE(d >= 1, "ADF needs a TT of degree >= 1");
        XERUS_REQUIRE(_x.dimensions == _dm.n, "Measurment dimensions must coincide with x dimensions.");
        XERUS_REQUIRE(maxRanks.size() + 1 == d, "maxRanks must have degree - 1 entries");
        double s = 0.0;   // calculate_norm_of_measured_values (:37-43)
        for (double v : _dm.hvals) s += v * v;
        normMeasured = std::sqrt(s);
        fwd.resize(d + 1);   // fwd[k + 1] = F_k (after components 0..k), fwd[0] = ones
        bwd.resize(d + 1);   // bwd[k] = B_k (components k..d-1), bwd[d] = ones
        fwd[0] = Tensor::ones({M, 1});
        bwd[d] = Tensor::ones({M, 1});
        res = Tensor({M}, Tensor::Representation::Dense, Tensor::Initialisation::None);
        scratch = Tensor({M}, Tensor::Representation::Dense, Tensor::Initialisation::None);
    }

    double solve() {
        x.canonicalize_left();   // :582
        solve_with_current_ranks();
        while (residualNorm > var.targetResidualNorm && x.ranks() != maxRanks &&
               (var.maxIterations == 0 || iteration < var.maxIterations)) {   // :590-602
            x.move_core(0, true);
            const TTTensor rnd = TTTensor::random(x.dimensions, std::vector<size_t>(d - 1, 1));
            const TTTensor diff = (1e-6 * frob_norm(x)) * rnd / frob_norm(rnd);
            x = x + diff;
            x.round(maxRanks);
            solve_with_current_ranks();
        }
        return residualNorm;
    }

   private:
    TTTensor& x;
    const size_t d;
    const std::vector<size_t> maxRanks;
    internal::DeviceMeasurements& dm;
    const size_t M;
    const ADFVariant& var;
    xrs_handle_t h;
    double normMeasured = 0.0;
    size_t iteration = 0;
    double residualNorm = std::numeric_limits<double>::max(), lastResidualNorm = std::numeric_limits<double>::max();
    std::vector<Tensor> fwd, bwd;
    Tensor res, scratch;

    struct Dims {
        size_t a, n, b;
    };
    Dims dims_of(size_t k) const {
        const Tensor& C = x.get_component(k);
        return {C.dimensions[0], C.dimensions[1], C.dimensions[2]};
    }

    void update_backward(size_t k) {   // B_k = C_k B_{k+1} (:217-251)
        const Dims c = dims_of(k);
        Tensor out({M, c.a}, Tensor::Representation::Dense, Tensor::Initialisation::None);
        xrs::adf::stack_backward(h, M, x.component(k).device_data_applied(), dm.mode(k), bwd[k + 1].device_data(), c.a, c.n, c.b,
                                 out.device_data_for_write());
        bwd[k] = std::move(out);
    }

    void update_forward(size_t k) {   // F_k = F_{k-1} C_k (:254-288)
        const Dims c = dims_of(k);
        Tensor out({M, c.b}, Tensor::Representation::Dense, Tensor::Initialisation::None);
        xrs::adf::stack_forward(h, M, fwd[k].device_data(), x.component(k).device_data_applied(), dm.mode(k), c.a, c.n, c.b,
                                out.device_data_for_write());
        fwd[k + 1] = std::move(out);
    }

    void calculate_residual(size_t k) {   // res = b - A(x) (:290-312)
        const Dims c = dims_of(k);
        xrs::adf::evaluate(h, M, fwd[k].device_data(), x.component(k).device_data_applied(), dm.mode(k), bwd[k + 1].device_data(), c.a,
                           c.n, c.b, dm.values(), res.device_data_for_write());
    }

    double residual_norm_sqr() {
        Tensor out({1}, Tensor::Representation::Dense, Tensor::Initialisation::None);
        xrs::adf::sum_squares(h, M, res.device_data(), out.device_data_for_write());
        return out[0];
    }

    void sweep_component(size_t k) {
        const Dims c = dims_of(k);
        if (k > 0) calculate_residual(k);   // (for k = 0 done with the stopping test)
        // projected gradient component (a, n, b) (:359-396)
        Tensor D({c.a, c.n, c.b}, Tensor::Representation::Dense, Tensor::Initialisation::None);
        xrs::adf::projected_gradient(h, M, fwd[k].device_data(), bwd[k + 1].device_data(), res.device_data(), dm.mode(k), dm.perm_of(k),
                                     dm.seg_of(k), c.a, c.n, c.b, D.device_data_for_write());
        // slice-wise ||A(E(grad))||^2 (:413-465)
        Tensor nrm({c.n}, Tensor::Representation::Dense, Tensor::Initialisation::None);
        xrs::adf::evaluate(h, M, fwd[k].device_data(), D.device_data(), dm.mode(k), bwd[k + 1].device_data(), c.a, c.n, c.b, nullptr,
                           scratch.device_data_for_write());
        xrs::adf::slice_square_sums(h, M, scratch.device_data(), dm.mode(k), dm.perm_of(k), dm.seg_of(k), c.n, nrm.device_data_for_write());
        // x_k += step (D) (:468-487)
        xrs::adf::update_component(h, x.component(k).device_data_applied(), D.device_data(), nrm.device_data(), dm.single_point, c.a, c.n,
                                   c.b);
        if (k + 1 < d) {   // :536-539
            x.move_core(k + 1, true);
            update_forward(k);
        }
    }

    void solve_with_current_ranks() {   // :489-542
        double resDec1 = 0.0, resDec2 = 0.0, resDec3 = 0.0;
        for (; var.maxIterations == 0 || iteration < var.maxIterations; ++iteration) {
            x.move_core(0, true);
            for (size_t k = d - 1; k > 0; --k) update_backward(k);
            calculate_residual(0);
            lastResidualNorm = residualNorm;
            residualNorm = std::sqrt(residual_norm_sqr()) / normMeasured;
            const double resDec4 = resDec3;
            resDec3 = resDec2;
            resDec2 = resDec1;
            resDec1 = residualNorm / lastResidualNorm;
            if (residualNorm < var.targetResidualNorm ||
                resDec1 * resDec2 * resDec3 * resDec4 > std::pow(var.minimalResidualNormDecrease, 4)) {
                break;
            }
            for (size_t k = 0; k < d; ++k) sweep_component(k);
        }
    }
};

template <class Set>
double run_adf(const ADFVariant& _v, TTTensor& _x, const Set& _meas, const std::vector<size_t>& _maxRanks) {
    return guard([&] {
        internal::DeviceMeasurements dm(_meas, _x.dimensions);
        AdfSolver solver(_x, _maxRanks, dm, _v);
        return solver.solve();
    });
}

}  // namespace

double ADFVariant::operator()(TTTensor& _x, const SinglePointMeasurementSet& _m) const { return run_adf(*this, _x, _m, _x.ranks()); }
double ADFVariant::operator()(TTTensor& _x, const RankOneMeasurementSet& _m) const { return run_adf(*this, _x, _m, _x.ranks()); }
double ADFVariant::operator()(TTTensor& _x, const SinglePointMeasurementSet& _m, const std::vector<size_t>& _maxRanks) const {
    return run_adf(*this, _x, _m, _maxRanks);
}
double ADFVariant::operator()(TTTensor& _x, const RankOneMeasurementSet& _m, const std::vector<size_t>& _maxRanks) const {
    return run_adf(*this, _x, _m, _maxRanks);
}

const ADFVariant ADF(0, 1e-8, 0.999);

}  // namespace xerus
