// Measurement sets (reference src/xerus/measurments.cpp:38-607): the host-side containers, random
// generation with the reference's draws from misc::randomEngine (so seeded runs give the reference's
// positions), and evaluation. Dense-Tensor evaluation reads the host mirror as the reference reads its
// tensor; TTTensor evaluation runs all measurements at once on the GPU (adf.hip stacks) where the
// reference re-contracts a TensorNetwork per position.
#include <algorithm>
#include <cmath>
#include <numeric>
#include <set>

#include "measurement_device.hpp"

namespace xerus {

namespace internal {

int comp(const Tensor& _a, const Tensor& _b) {
    XERUS_REQUIRE(_a.dimensions == _b.dimensions, "Compared Tensors must have the same dimensions.");
    for (size_t k = 0; k < _a.size; ++k) {
        if (_a.cat(k) < _b.cat(k)) return 1;
        if (_a.cat(k) > _b.cat(k)) return -1;
    }
    return 0;
}

DeviceMeasurements::DeviceMeasurements(const SinglePointMeasurementSet& _set, const std::vector<size_t>& _dims)
    : M(_set.size()), d(_dims.size()), single_point(true), n(_dims) {
    XERUS_REQUIRE(M > 0, "Need at very least one measurment.");
    XERUS_REQUIRE(_set.degree() == d, "Measurment degree must coincide with the tensor degree.");
    xrs_handle_t h = gpu::handle();
    hpos.resize(d * M);
    hperm.resize(d);
    hseg.resize(d);
    for (size_t k = 0; k < d; ++k) {
        std::vector<int>& sg = hseg[k];
        sg.assign(n[k] + 1, 0);
        for (size_t m = 0; m < M; ++m) {
            const size_t p = _set.positions[m][k];
            XERUS_REQUIRE(p < n[k], "measurement position out of range");
            hpos[k * M + m] = int(p);
            ++sg[p + 1];
        }
        for (size_t t = 0; t < n[k]; ++t) sg[t + 1] += sg[t];
        std::vector<int> fill(sg.begin(), sg.end() - 1);
        hperm[k].resize(M);
        for (size_t m = 0; m < M; ++m) hperm[k][size_t(fill[size_t(hpos[k * M + m])]++)] = int(m);
    }
    hvals = _set.measuredValues;
    pos = xrs::DevBuf(h, d * M * sizeof(int));
    vals = xrs::DevBuf(h, M * 8);
    XRS_HIP(hipMemcpyAsync(pos.p, hpos.data(), d * M * sizeof(int), hipMemcpyHostToDevice, h->stream));
    XRS_HIP(hipMemcpyAsync(vals.p, hvals.data(), M * 8, hipMemcpyHostToDevice, h->stream));
    for (size_t k = 0; k < d; ++k) {
        perm.emplace_back(h, M * sizeof(int));
        seg.emplace_back(h, (n[k] + 1) * sizeof(int));
        XRS_HIP(hipMemcpyAsync(perm.back().p, hperm[k].data(), M * sizeof(int), hipMemcpyHostToDevice, h->stream));
        XRS_HIP(hipMemcpyAsync(seg.back().p, hseg[k].data(), (n[k] + 1) * sizeof(int), hipMemcpyHostToDevice, h->stream));
    }
}

DeviceMeasurements::DeviceMeasurements(const RankOneMeasurementSet& _set, const std::vector<size_t>& _dims)
    : M(_set.size()), d(_dims.size()), single_point(false), n(_dims) {
    XERUS_REQUIRE(M > 0, "Need at very least one measurment.");
    XERUS_REQUIRE(_set.degree() == d, "Measurment degree must coincide with the tensor degree.");
    xrs_handle_t h = gpu::handle();
    voff.assign(d + 1, 0);
    for (size_t k = 0; k < d; ++k) voff[k + 1] = voff[k] + M * n[k];
    hvec.resize(voff[d]);
    for (size_t m = 0; m < M; ++m)
        for (size_t k = 0; k < d; ++k) {
            const Tensor& v = _set.positions[m][k];
            XERUS_REQUIRE(v.size == n[k], "measurement vector of mode " << k << " has " << v.size << " entries, expected " << n[k]);
            for (size_t t = 0; t < n[k]; ++t) hvec[voff[k] + m * n[k] + t] = v.cat(t);
        }
    hvals = _set.measuredValues;
    vec = xrs::DevBuf(h, voff[d] * 8);
    vals = xrs::DevBuf(h, M * 8);
    XRS_HIP(hipMemcpyAsync(vec.p, hvec.data(), voff[d] * 8, hipMemcpyHostToDevice, h->stream));
    XRS_HIP(hipMemcpyAsync(vals.p, hvals.data(), M * 8, hipMemcpyHostToDevice, h->stream));
}

xrs::adf::Mode DeviceMeasurements::mode(size_t _k) const {
    xrs::adf::Mode md;
    if (single_point) md.pos = pos.as<int>() + _k * M;
    else md.vec = vec.d() + voff[_k];
    return md;
}

std::vector<value_t> evaluate_tt(const TTTensor& _x, const DeviceMeasurements& _dm) {
    XERUS_REQUIRE(_x.degree() == _dm.d, "Degrees of solution and measurements must match!");
    XERUS_REQUIRE(_x.dimensions == _dm.n, "Dimensions of solution and measurements must match!");
    xrs_handle_t h = gpu::handle();
    const size_t M = _dm.M;
    Tensor F = Tensor::ones({M, 1});
    for (size_t k = 0; k < _dm.d; ++k) {
        Tensor C = _x.get_component(k);   // (shares the buffer; a pending factor is applied to a private copy)
        const size_t a = C.dimensions[0], nk = C.dimensions[1], b = C.dimensions[2];
        Tensor Fn({M, b}, Tensor::Representation::Dense, Tensor::Initialisation::None);
        xrs::adf::stack_forward(h, M, F.device_data(), C.device_data_applied(), _dm.mode(k), a, nk, b, Fn.device_data_for_write());
        F = std::move(Fn);
    }
    std::vector<value_t> out = F.to_host();
    return out;
}

}  // namespace internal

// ------------------------------------------------------------------------------ SinglePointMeasurementSet
SinglePointMeasurementSet SinglePointMeasurementSet::random(const size_t _numMeasurements, const std::vector<size_t>& _dimensions) {
    SinglePointMeasurementSet result;
    result.create_random_positions(_numMeasurements, _dimensions);
    result.measuredValues.assign(_numMeasurements, 0.0);
    return result;
}

SinglePointMeasurementSet SinglePointMeasurementSet::random(const size_t _numMeasurements, const Tensor& _solution) {
    SinglePointMeasurementSet result;
    result.create_random_positions(_numMeasurements, _solution.dimensions);
    result.measure(_solution);
    return result;
}

SinglePointMeasurementSet SinglePointMeasurementSet::random(const size_t _numMeasurements, const TTTensor& _solution) {
    SinglePointMeasurementSet result;
    result.create_random_positions(_numMeasurements, _solution.dimensions);
    result.measure(_solution);
    return result;
}

SinglePointMeasurementSet SinglePointMeasurementSet::random(const size_t _numMeasurements, const TensorNetwork& _solution) {
    SinglePointMeasurementSet result;
    result.create_random_positions(_numMeasurements, _solution.dimensions);
    result.measure(_solution);
    return result;
}

SinglePointMeasurementSet SinglePointMeasurementSet::random(const size_t _numMeasurements, const std::vector<size_t>& _dimensions,
                                                            std::function<value_t(const std::vector<size_t>&)> _callback) {
    SinglePointMeasurementSet result;
    result.create_random_positions(_numMeasurements, _dimensions);
    result.measure(_callback);
    return result;
}

size_t SinglePointMeasurementSet::size() const {
    XERUS_REQUIRE(positions.size() == measuredValues.size(), "Inconsitend SinglePointMeasurementSet encountered.");
    return positions.size();
}

size_t SinglePointMeasurementSet::degree() const { return positions.empty() ? 0 : positions[0].size(); }

void SinglePointMeasurementSet::add(std::vector<size_t> _position, const value_t _measuredValue) {
    XERUS_REQUIRE(positions.empty() || _position.size() == positions.back().size(),
                  "Given _position has incorrect degree " << _position.size() << ". Expected " << positions.back().size() << ".");
    positions.emplace_back(std::move(_position));
    measuredValues.emplace_back(_measuredValue);
}

void SinglePointMeasurementSet::sort(const bool _positionsOnly) {
    const auto less = [](const std::vector<size_t>& _l, const std::vector<size_t>& _r) {
        XERUS_REQUIRE(_l.size() == _r.size(), "Inconsistent degrees in measurment positions.");
        return std::lexicographical_compare(_l.begin(), _l.end(), _r.begin(), _r.end());
    };
    if (_positionsOnly) {
        std::sort(positions.begin(), positions.end(), less);
        return;
    }
    XERUS_REQUIRE(positions.size() == measuredValues.size(), "Inconsitend SinglePointMeasurementSet encountered.");
    std::vector<size_t> order(positions.size());
    std::iota(order.begin(), order.end(), size_t(0));
    std::sort(order.begin(), order.end(), [&](size_t _a, size_t _b) { return less(positions[_a], positions[_b]); });
    std::vector<std::vector<size_t>> p(positions.size());
    std::vector<value_t> v(positions.size());
    for (size_t i = 0; i < order.size(); ++i) {
        p[i] = std::move(positions[order[i]]);
        v[i] = measuredValues[order[i]];
    }
    positions = std::move(p);
    measuredValues = std::move(v);
}

value_t SinglePointMeasurementSet::frob_norm() const {
    double norm = 0.0;
    for (size_t i = 0; i < size(); ++i) norm += measuredValues[i] * measuredValues[i];
    return std::sqrt(norm);
}

void SinglePointMeasurementSet::measure(const Tensor& _solution) {
    for (size_t i = 0; i < size(); ++i) measuredValues[i] = _solution[positions[i]];
}

void SinglePointMeasurementSet::measure(const TTTensor& _solution) {
    XERUS_REQUIRE(_solution.degree() == degree(), "Degrees of solution and measurements must match!");
    internal::DeviceMeasurements dm(*this, _solution.dimensions);
    measuredValues = internal::evaluate_tt(_solution, dm);
}

namespace {
// A network whose full tensor is small next to the work of contracting it once per entry (TensorNetwork::
// operator[], a slice copy per external mode and a contraction per entry) is contracted once and every entry
// read from the full tensor: at most 2^22 entries, or 64 per measurement.
bool contract_whole(const TensorNetwork& _net, size_t _count) {
    const size_t limit = std::max<size_t>(size_t(1) << 22, 64 * _count);
    size_t s = 1;
    for (const size_t d : _net.dimensions) {
        if (d != 0 && s > limit / d) return false;
        s *= d;
    }
    return true;
}
}  // namespace

void SinglePointMeasurementSet::measure(const TensorNetwork& _solution) {
    XERUS_REQUIRE(_solution.degree() == degree(), "Degrees of solution and measurements must match!");
    if (contract_whole(_solution, size())) {
        measure(_solution.to_tensor());
        return;
    }
    for (size_t i = 0; i < size(); ++i) measuredValues[i] = _solution[positions[i]];
}

void SinglePointMeasurementSet::measure(std::function<value_t(const std::vector<size_t>&)> _callback) {
    for (size_t i = 0; i < size(); ++i) measuredValues[i] = _callback(positions[i]);
}

double SinglePointMeasurementSet::test(const Tensor& _solution) const {
    double error = 0.0, norm = 0.0;
    for (size_t i = 0; i < size(); ++i) {
        const double e = measuredValues[i] - _solution[positions[i]];
        error += e * e;
        norm += measuredValues[i] * measuredValues[i];
    }
    return std::sqrt(error / norm);
}

double SinglePointMeasurementSet::test(const TensorNetwork& _solution) const {
    XERUS_REQUIRE(_solution.degree() == degree(), "Degrees of solution and measurements must match!");
    if (contract_whole(_solution, size())) return test(_solution.to_tensor());
    double error = 0.0, norm = 0.0;
    for (size_t i = 0; i < size(); ++i) {
        const double e = measuredValues[i] - _solution[positions[i]];
        error += e * e;
        norm += measuredValues[i] * measuredValues[i];
    }
    return std::sqrt(error / norm);
}

double SinglePointMeasurementSet::test(const TTTensor& _solution) const {
    XERUS_REQUIRE(_solution.degree() == degree(), "Degrees of solution and measurements must match!");
    internal::DeviceMeasurements dm(*this, _solution.dimensions);
    const std::vector<value_t> got = internal::evaluate_tt(_solution, dm);
    double error = 0.0, norm = 0.0;
    for (size_t i = 0; i < size(); ++i) {
        const double e = measuredValues[i] - got[i];
        error += e * e;
        norm += measuredValues[i] * measuredValues[i];
    }
    return std::sqrt(error / norm);
}

double SinglePointMeasurementSet::test(std::function<value_t(const std::vector<size_t>&)> _callback) const {
    double error = 0.0, norm = 0.0;
    for (size_t i = 0; i < size(); ++i) {
        const double e = measuredValues[i] - _callback(positions[i]);
        error += e * e;
        norm += measuredValues[i] * measuredValues[i];
    }
    return std::sqrt(error / norm);
}

void SinglePointMeasurementSet::create_random_positions(const size_t _numMeasurements, const std::vector<size_t>& _dimensions) {
    size_t total = 1;
    for (size_t n : _dimensions) total = (total > ~size_t(0) / std::max<size_t>(n, 1)) ? ~size_t(0) : total * n;
    XERUS_REQUIRE(total >= _numMeasurements,
                  "It's impossible to perform as many measurements as requested. " << _numMeasurements << " > " << total);
    std::vector<std::uniform_int_distribution<size_t>> indexDist;
    for (size_t n : _dimensions) indexDist.emplace_back(0, n - 1);
    std::set<size_t> measured;
    std::vector<size_t> multIdx(_dimensions.size());
    while (positions.size() < _numMeasurements) {
        size_t pos = 0;
        for (size_t i = 0; i < _dimensions.size(); ++i) {
            multIdx[i] = indexDist[i](misc::randomEngine);
            pos = pos * _dimensions[i] + multIdx[i];
        }
        if (measured.insert(pos).second) positions.push_back(multIdx);
    }
    sort(true);
    measuredValues.resize(_numMeasurements);
}

// ---------------------------------------------------------------------------------- RankOneMeasurementSet
RankOneMeasurementSet::RankOneMeasurementSet(const SinglePointMeasurementSet& _other, const std::vector<size_t>& _dimensions) {
    XERUS_REQUIRE(_other.degree() == _dimensions.size(), "Inconsistent degrees.");
    for (size_t i = 0; i < _other.size(); ++i) {
        std::vector<Tensor> pos;
        pos.reserve(_dimensions.size());
        for (size_t j = 0; j < _dimensions.size(); ++j) pos.push_back(Tensor::dirac({_dimensions[j]}, _other.positions[i][j]));
        add(pos, _other.measuredValues[i]);
    }
}

RankOneMeasurementSet RankOneMeasurementSet::random(const size_t _numMeasurements, const std::vector<size_t>& _dimensions) {
    RankOneMeasurementSet result;
    result.create_random_positions(_numMeasurements, _dimensions);
    result.measuredValues.assign(_numMeasurements, 0.0);
    return result;
}

RankOneMeasurementSet RankOneMeasurementSet::random(const size_t _numMeasurements, const Tensor& _solution) {
    RankOneMeasurementSet result;
    result.create_random_positions(_numMeasurements, _solution.dimensions);
    result.measure(_solution);
    return result;
}

RankOneMeasurementSet RankOneMeasurementSet::random(const size_t _numMeasurements, const TTTensor& _solution) {
    RankOneMeasurementSet result;
    result.create_random_positions(_numMeasurements, _solution.dimensions);
    result.measure(_solution);
    return result;
}

RankOneMeasurementSet RankOneMeasurementSet::random(const size_t _numMeasurements, const std::vector<size_t>& _dimensions,
                                                    std::function<value_t(const std::vector<Tensor>&)> _callback) {
    RankOneMeasurementSet result;
    result.create_random_positions(_numMeasurements, _dimensions);
    result.measure(_callback);
    return result;
}

size_t RankOneMeasurementSet::size() const {
    XERUS_REQUIRE(positions.size() == measuredValues.size(), "Inconsitend SinglePointMeasurementSet encountered.");
    return positions.size();
}

size_t RankOneMeasurementSet::degree() const { return positions.empty() ? 0 : positions[0].size(); }

void RankOneMeasurementSet::add(const std::vector<Tensor>& _position, const value_t _measuredValue) {
    if (!positions.empty()) {
        XERUS_REQUIRE(_position.size() == positions.back().size(), "Inconsitend degree obtained.");
        for (size_t i = 0; i < _position.size(); ++i)
            XERUS_REQUIRE(positions.back()[i].dimensions == _position[i].dimensions, "Inconsitend dimensions obtained.");
    }
    for (const Tensor& t : _position) XERUS_REQUIRE(t.degree() == 1, "Illegal measurement.");
    positions.push_back(_position);
    measuredValues.push_back(_measuredValue);
}

void RankOneMeasurementSet::sort(const bool _positionsOnly) {
    // host copies of the vectors once (comp reads entries through the host mirror)
    const size_t M = positions.size();
    std::vector<std::vector<std::vector<value_t>>> hv(M);
    for (size_t m = 0; m < M; ++m)
        for (const Tensor& t : positions[m]) hv[m].push_back(t.to_host());
    const auto less = [&](size_t _a, size_t _b) {
        for (size_t i = 0; i < hv[_a].size(); ++i) {
            const std::vector<value_t>& x = hv[_a][i];
            const std::vector<value_t>& y = hv[_b][i];
            for (size_t k = 0; k < x.size(); ++k) {   // internal::comp: the larger entry sorts first
                if (x[k] > y[k]) return true;
                if (x[k] < y[k]) return false;
            }
        }
        return false;
    };
    std::vector<size_t> order(M);
    std::iota(order.begin(), order.end(), size_t(0));
    std::sort(order.begin(), order.end(), less);
    std::vector<std::vector<Tensor>> p(M);
    std::vector<value_t> v(measuredValues.size());
    for (size_t i = 0; i < M; ++i) {
        p[i] = std::move(positions[order[i]]);
        if (!_positionsOnly) v[i] = measuredValues[order[i]];
    }
    positions = std::move(p);
    if (!_positionsOnly) measuredValues = std::move(v);
}

void RankOneMeasurementSet::normalize() {
    for (size_t i = 0; i < size(); ++i)
        for (size_t j = 0; j < degree(); ++j) {
            const value_t norm = positions[i][j].frob_norm();
            positions[i][j] /= norm;
            positions[i][j].apply_factor();
            measuredValues[i] /= norm;
        }
}

value_t RankOneMeasurementSet::frob_norm() const {
    double norm = 0.0;
    for (size_t i = 0; i < size(); ++i) norm += measuredValues[i] * measuredValues[i];
    return std::sqrt(norm);
}

namespace {
// <T, v_0 (x) ... (x) v_{d-1}> on the host mirror, contracting the first mode each time
// (contract(stack[i+1], positions[j][i], false, stack[i], false, 1), measurments.cpp:374-390)
value_t rank_one_value(const std::vector<value_t>& _t, const std::vector<size_t>& _dims, const std::vector<Tensor>& _v) {
    std::vector<value_t> cur = _t, nxt;
    size_t rest = cur.size();
    for (size_t k = 0; k < _dims.size(); ++k) {
        const size_t n = _dims[k];
        rest /= n;
        nxt.assign(rest, 0.0);
        for (size_t i = 0; i < n; ++i) {
            const value_t w = _v[k].cat(i);
            for (size_t r = 0; r < rest; ++r) nxt[r] += w * cur[i * rest + r];
        }
        cur.swap(nxt);
    }
    return cur[0];
}
}  // namespace

void RankOneMeasurementSet::measure(const Tensor& _solution) {
    XERUS_REQUIRE(_solution.degree() == degree(), "Degrees of solution and measurements must match!");
    const std::vector<value_t> t = _solution.to_host();
    for (size_t i = 0; i < size(); ++i) measuredValues[i] = rank_one_value(t, _solution.dimensions, positions[i]);
}

void RankOneMeasurementSet::measure(const TTTensor& _solution) {
    XERUS_REQUIRE(_solution.degree() == degree(), "Degrees of solution and measurements must match!");
    internal::DeviceMeasurements dm(*this, _solution.dimensions);
    measuredValues = internal::evaluate_tt(_solution, dm);
}

void RankOneMeasurementSet::measure(std::function<value_t(const std::vector<Tensor>&)> _callback) {
    for (size_t i = 0; i < size(); ++i) measuredValues[i] = _callback(positions[i]);
}

double RankOneMeasurementSet::test(const Tensor& _solution) const {
    XERUS_REQUIRE(_solution.degree() == degree(), "Degrees of solution and measurements must match!");
    const std::vector<value_t> t = _solution.to_host();
    double error = 0.0, norm = 0.0;
    for (size_t i = 0; i < size(); ++i) {
        const double e = measuredValues[i] - rank_one_value(t, _solution.dimensions, positions[i]);
        error += e * e;
        norm += measuredValues[i] * measuredValues[i];
    }
    return std::sqrt(error / norm);
}

double RankOneMeasurementSet::test(const TTTensor& _solution) const {
    XERUS_REQUIRE(_solution.degree() == degree(), "Degrees of solution and measurements must match!");
    internal::DeviceMeasurements dm(*this, _solution.dimensions);
    const std::vector<value_t> got = internal::evaluate_tt(_solution, dm);
    double error = 0.0, norm = 0.0;
    for (size_t i = 0; i < size(); ++i) {
        const double e = measuredValues[i] - got[i];
        error += e * e;
        norm += measuredValues[i] * measuredValues[i];
    }
    return std::sqrt(error / norm);
}

double RankOneMeasurementSet::test(std::function<value_t(const std::vector<Tensor>&)> _callback) const {
    double error = 0.0, norm = 0.0;
    for (size_t i = 0; i < size(); ++i) {
        const double e = measuredValues[i] - _callback(positions[i]);
        error += e * e;
        norm += measuredValues[i] * measuredValues[i];
    }
    return std::sqrt(error / norm);
}

void RankOneMeasurementSet::create_random_positions(const size_t _numMeasurements, const std::vector<size_t>& _dimensions) {
    size_t total = 1;
    for (size_t n : _dimensions) total = (total > ~size_t(0) / std::max<size_t>(n, 1)) ? ~size_t(0) : total * n;
    XERUS_REQUIRE(total >= _numMeasurements,
                  "It's impossible to perform as many measurements as requested. " << _numMeasurements << " > " << total);
    std::vector<Tensor> pos(_dimensions.size());
    while (positions.size() < _numMeasurements) {
        for (size_t i = 0; i < _dimensions.size(); ++i) pos[i] = Tensor::random({_dimensions[i]});
        positions.push_back(pos);
    }
    sort(true);
    measuredValues.resize(_numMeasurements);
}

}  // namespace xerus
