// TTTensor on HBM. The components are xerus::Tensors whose device buffers are handed to the TT drivers
// of tt.hip for move_core / round (ownership moves into the driver's core array and back, no copies)
// and read in place for <x,y>. Reference: ttNetwork.cpp (constructors :57-160, move_core :582-640,
// round :644-684, frob_norm :782-789, sums :797-847, scaling :860-873).
#include <algorithm>
#include <cmath>
#include <limits>

#include "../tt_internal.hpp"
#include "xerus.h"

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

// device cores of a TT, released from their Tensors (factor applied) for the duration of a driver call
struct Handoff {
    std::vector<size_t> n, r;
    std::vector<double*> cores;
    TTTensor* tt;
    bool done = false;

    explicit Handoff(TTTensor& _tt) : tt(&_tt) {
        const size_t d = _tt.degree();
        n = _tt.dimensions;
        r.assign(d + 1, 1);
        for (size_t k = 0; k < d; ++k) r[k + 1] = _tt.components[k].dimensions[2];
        cores.resize(d);
        for (size_t k = 0; k < d; ++k) cores[k] = _tt.components[k].release_device();
    }
    void give_back() {
        for (size_t k = 0; k < cores.size(); ++k) tt->components[k] = Tensor::adopt_device({r[k], n[k], r[k + 1]}, cores[k]);
        done = true;
    }
    ~Handoff() {
        if (done) return;
        // a failed driver call leaves the cores in an unspecified gauge; return the buffers and zero the TT
        xrs_handle_t h = gpu::handle();
        for (double* p : cores)
            if (p) h->pool->release(p);
        *tt = TTTensor(tt->dimensions);
    }
};

}  // namespace

TTTensor::TTTensor() : components(1), dimensions(), canonicalized(true), corePosition(0) {}

TTTensor::TTTensor(size_t _degree) : TTTensor(Tensor::DimensionTuple(_degree, 1)) {}

TTTensor::TTTensor(const Tensor::DimensionTuple& _dimensions) : dimensions(_dimensions), canonicalized(true), corePosition(0) {
    XERUS_REQUIRE(std::find(dimensions.begin(), dimensions.end(), size_t(0)) == dimensions.end(), "Zero is no valid dimension.");
    if (dimensions.empty()) {
        components.resize(1);
        return;
    }
    for (size_t i = 0; i < dimensions.size(); ++i) components.push_back(Tensor::dirac({1, dimensions[i], 1}, 0));
    components[0][0] = 0.0;   // zero tensor, core at 0 (ttNetwork.cpp:104-105)
}

TTTensor TTTensor::ones(const std::vector<size_t>& _dimensions) {
    XERUS_REQUIRE(std::find(_dimensions.begin(), _dimensions.end(), size_t(0)) == _dimensions.end(),
                  "Trying to construct a TTTensor with dimension 0 is not possible.");
    if (_dimensions.empty()) {
        TTTensor r(size_t(0));
        r.components[0] = Tensor::ones({});
        return r;
    }
    TTTensor result(_dimensions);
    for (size_t i = 0; i < _dimensions.size(); ++i) result.set_component(i, Tensor::ones({1, _dimensions[i], 1}));
    result.canonicalized = false;
    result.canonicalize_left();
    return result;
}

TTTensor::TTTensor(const Tensor& _tensor, const double _eps, const size_t _maxRank)
    : TTTensor(_tensor, _eps, std::vector<size_t>(_tensor.degree() == 0 ? 0 : _tensor.degree() - 1, _maxRank)) {}

// TT-SVD, right to left (ttNetwork.cpp:111-160)
TTTensor::TTTensor(const Tensor& _tensor, const double _eps, const std::vector<size_t>& _maxRanks) : TTTensor(_tensor.degree()) {
    XERUS_REQUIRE(_eps >= 0 && _eps < 1, "_eps must be positive and smaller than one. " << _eps << " was given.");
    const size_t d = _tensor.degree();
    XERUS_REQUIRE(_maxRanks.size() == (d == 0 ? 0 : d - 1), "We need " << (d == 0 ? 0 : d - 1) << " ranks but " << _maxRanks.size() << " where given");
    XERUS_REQUIRE(std::find(_maxRanks.begin(), _maxRanks.end(), size_t(0)) == _maxRanks.end(), "Maximal ranks must be strictly positive.");
    if (d == 0) {
        components[0] = _tensor;
        return;
    }
    dimensions = _tensor.dimensions;
    Tensor remains = _tensor;
    std::vector<size_t> ext{1};
    ext.insert(ext.end(), dimensions.begin(), dimensions.end());
    ext.push_back(1);
    remains.reinterpret_dimensions(ext);
    Tensor S, node;
    for (size_t position = d - 1; position > 0; --position) {
        calculate_svd(remains, S, node, remains, 1 + position, _maxRanks[position - 1], _eps);
        set_component(position, std::move(node));
        node.reset();
        contract(remains, remains, false, S, false, 1);
    }
    set_component(0, remains);
    assume_core_position(0);
}

std::vector<size_t> TTTensor::reduce_to_maximal_ranks(std::vector<size_t> _ranks, const std::vector<size_t>& _dimensions) {
    const size_t numComponents = _dimensions.size();
    XERUS_REQUIRE(numComponents == _ranks.size() + 1,
                  "Invalid number of ranks (" << _ranks.size() << ") or dimensions (" << _dimensions.size() << ") given.");
    size_t cur = 1;
    for (size_t i = 0; i + 1 < numComponents; ++i) {
        cur *= _dimensions[i];
        if (cur < _ranks[i]) _ranks[i] = cur;
        else cur = _ranks[i];
    }
    cur = 1;
    for (size_t i = 1; i < numComponents; ++i) {
        cur *= _dimensions[numComponents - i];
        if (cur < _ranks[numComponents - i - 1]) _ranks[numComponents - i - 1] = cur;
        else cur = _ranks[numComponents - i - 1];
    }
    return _ranks;
}

std::vector<size_t> TTTensor::ranks() const {
    std::vector<size_t> r;
    for (size_t k = 0; k + 1 < degree(); ++k) r.push_back(components[k].dimensions.back());
    return r;
}

size_t TTTensor::rank(const size_t _i) const {
    XERUS_REQUIRE(_i + 1 < degree(), "Requested illegal rank " << _i);
    return components[_i].dimensions.back();
}

Tensor& TTTensor::component(const size_t _idx) {
    XERUS_REQUIRE(_idx == 0 || _idx < degree(), "Illegal index " << _idx << " in TTNetwork::component");
    return components[_idx];
}

void TTTensor::set_component(const size_t _idx, Tensor _T) {
    if (degree() == 0) {
        XERUS_REQUIRE(_idx == 0 && _T.degree() == 0, "Component of degree zero TTNetwork must have degree zero.");
        components[0] = std::move(_T);
        return;
    }
    XERUS_REQUIRE(_idx < degree(), "Illegal index " << _idx << " in TTNetwork::set_component");
    XERUS_REQUIRE(_T.degree() == 3, "Component " << _idx << " must have degree 3. Given: " << _T.degree());
    dimensions[_idx] = _T.dimensions[1];
    components[_idx] = std::move(_T);
    canonicalized = canonicalized && corePosition == _idx;   // ttNetwork.cpp:491
}

bool TTTensor::exceeds_maximal_ranks() const {
    for (size_t i = 0; i < degree(); ++i) {
        const auto& c = components[i].dimensions;
        if (c.front() > c[1] * c.back() || c.back() > c[1] * c.front()) return true;
    }
    return false;
}

void TTTensor::require_correct_format() const {
    const size_t d = degree();
    if (d == 0) {
        XERUS_REQUIRE(components.size() == 1 && components[0].degree() == 0, "degree-0 TT must hold one scalar");
        return;
    }
    XERUS_REQUIRE(components.size() == d, "TT has " << components.size() << " components for degree " << d);
    for (size_t k = 0; k < d; ++k) {
        const auto& c = components[k].dimensions;
        XERUS_REQUIRE(c.size() == 3, "Component " << k << " must have degree 3");
        XERUS_REQUIRE(c[1] == dimensions[k], "Component " << k << " has external dimension " << c[1] << " instead of " << dimensions[k]);
        XERUS_REQUIRE(k == 0 ? c[0] == 1 : c[0] == components[k - 1].dimensions[2], "Rank mismatch left of component " << k);
    }
    XERUS_REQUIRE(components[d - 1].dimensions[2] == 1, "last rank must be 1");
}

void TTTensor::assume_core_position(const size_t _pos) {
    XERUS_REQUIRE(_pos < degree() || (degree() == 0 && _pos == 0), "Invalid core position.");
    corePosition = _pos;
    canonicalized = true;
}

void TTTensor::move_core(const size_t _position, const bool _keepRank) {
    XERUS_REQUIRE(_position < degree() || (_position == 0 && degree() == 0),
                  "Illegal core-position " << _position << " chosen for TTNetwork with " << degree() << " components");
    require_correct_format();
    if (degree() > 0) {
        Handoff H(*this);
        guard([&] {
            xrs::tt::move_core(gpu::handle(), degree(), H.n.data(), H.r.data(), H.cores.data(), canonicalized, corePosition, _position,
                               _keepRank);
        });
        H.give_back();
    }
    canonicalized = true;
    corePosition = _position;
}

void TTTensor::round(const std::vector<size_t>& _maxRanks, const double _eps) {
    require_correct_format();
    XERUS_REQUIRE(_eps < 1, "_eps must be smaller than one. " << _eps << " was given.");
    XERUS_REQUIRE(_maxRanks.size() + 1 == degree() || (_maxRanks.empty() && degree() == 0),
                  "There must be exactly degree/N-1 maxRanks. Here " << _maxRanks.size() << " instead of " << degree() - 1 << " are given.");
    XERUS_REQUIRE(std::find(_maxRanks.begin(), _maxRanks.end(), size_t(0)) == _maxRanks.end(),
                  "Trying to round a TTTensor to rank 0 is not possible.");
    if (degree() == 0) return;
    const bool initialCanonicalization = canonicalized;
    const size_t initialCorePosition = corePosition;
    {
        Handoff H(*this);
        guard([&] {
            xrs::tt::round(gpu::handle(), degree(), H.n.data(), H.r.data(), H.cores.data(), canonicalized, corePosition, _maxRanks.data(),
                           _eps);
        });
        H.give_back();
    }
    // the sweep ends with the core at 0 (ttNetwork.cpp:660-664)
    assume_core_position(0);
    if (initialCanonicalization && initialCorePosition != 0) move_core(initialCorePosition);
}

void TTTensor::round(const size_t _maxRank) { round(std::vector<size_t>(degree() == 0 ? 0 : degree() - 1, _maxRank), EPSILON); }

void TTTensor::round(const int _maxRank) {
    XERUS_REQUIRE(_maxRank > 0, "MaxRank must be positive");
    round(size_t(_maxRank));
}

void TTTensor::round(const value_t _eps) {
    round(std::vector<size_t>(degree() == 0 ? 0 : degree() - 1, std::numeric_limits<size_t>::max()), _eps);
}

void TTTensor::soft_threshold(const std::vector<double>& _taus, const bool /*_preventZero*/) {
    const size_t d = degree();
    XERUS_REQUIRE(_taus.size() + 1 == d || (_taus.empty() && d == 0),
                  "There must be exactly degree/N-1 taus. Here " << _taus.size() << " instead of " << d - 1 << " are given.");
    require_correct_format();
    if (d == 0) return;
    const bool initialCanonicalization = canonicalized;
    const size_t initialCorePosition = corePosition;
    {
        Handoff H(*this);
        guard([&] {
            xrs::tt::soft_threshold(gpu::handle(), d, H.n.data(), H.r.data(), H.cores.data(), canonicalized, corePosition,
                                    _taus.data());
        });
        H.give_back();
    }
    assume_core_position(0);
    if (initialCanonicalization) move_core(initialCorePosition);
}

void TTTensor::soft_threshold(const double _tau, const bool _preventZero) {
    soft_threshold(std::vector<double>(degree() == 0 ? 0 : degree() - 1, _tau), _preventZero);
}

value_t TTTensor::frob_norm() const {
    require_correct_format();
    if (canonicalized) return components[corePosition].frob_norm();
    return std::sqrt(std::max(0.0, dot(*this, *this)));
}

TTTensor& TTTensor::operator*=(const value_t _factor) {
    components[canonicalized ? corePosition : 0] *= _factor;
    return *this;
}

TTTensor& TTTensor::operator/=(const value_t _divisor) { return *this *= 1 / _divisor; }

// block-diagonal cores (ttNetwork.cpp:797-847); a canonical TT is re-canonicalised to its core position
// (move_core with the rank-revealing QC, :841-843), which may cut the summed ranks
TTTensor& TTTensor::operator+=(const TTTensor& _other) {
    XERUS_REQUIRE(dimensions == _other.dimensions, "The dimensions in TT sum must coincide.");
    require_correct_format();
    _other.require_correct_format();
    const size_t d = degree();
    const bool initialCanonicalization = canonicalized;
    const size_t initialCorePosition = corePosition;
    if (d <= 1) {
        components[0] += _other.components[0];
        return *this;
    }
    for (size_t k = 0; k < d; ++k) {
        const Tensor& A = components[k];
        const Tensor& B = _other.components[k];
        Tensor C({k == 0 ? 1 : A.dimensions[0] + B.dimensions[0], A.dimensions[1], k + 1 == d ? 1 : A.dimensions[2] + B.dimensions[2]},
                 Tensor::Representation::Dense, Tensor::Initialisation::Zero);
        C.offset_add(A, {0, 0, 0});
        C.offset_add(B, {k == 0 ? 0 : A.dimensions[0], 0, k + 1 == d ? 0 : A.dimensions[2]});
        components[k] = std::move(C);
    }
    canonicalized = false;
    if (initialCanonicalization) move_core(initialCorePosition);
    return *this;
}

TTTensor& TTTensor::operator-=(const TTTensor& _other) {
    *this *= -1.0;
    *this += _other;
    *this *= -1.0;
    return *this;
}

TTTensor operator+(TTTensor _lhs, const TTTensor& _rhs) { return _lhs += _rhs; }
TTTensor operator-(TTTensor _lhs, const TTTensor& _rhs) { return _lhs -= _rhs; }
TTTensor operator*(const value_t _factor, TTTensor _tt) { return _tt *= _factor; }
TTTensor operator*(TTTensor _tt, const value_t _factor) { return _tt *= _factor; }
TTTensor operator/(TTTensor _tt, const value_t _divisor) { return _tt /= _divisor; }

Tensor TTTensor::to_tensor() const {
    require_correct_format();
    if (degree() == 0) return components[0];
    Tensor result = components[0];
    for (size_t k = 1; k < degree(); ++k) contract(result, result, false, components[k], false, 1);
    result.reinterpret_dimensions(dimensions);
    return result;
}

TTTensor::operator Tensor() const { return to_tensor(); }

value_t dot(const TTTensor& _x, const TTTensor& _y) {
    XERUS_REQUIRE(_x.dimensions == _y.dimensions, "dot of TTs with different dimensions");
    _x.require_correct_format();
    _y.require_correct_format();
    const size_t d = _x.degree();
    if (d == 0) return _x.components[0][0] * _y.components[0][0];
    std::vector<size_t> rx(d + 1, 1), ry(d + 1, 1);
    std::vector<const double*> X(d), Y(d);
    value_t f = 1.0;
    for (size_t k = 0; k < d; ++k) {
        rx[k + 1] = _x.components[k].dimensions[2];
        ry[k + 1] = _y.components[k].dimensions[2];
        X[k] = _x.components[k].device_data();
        Y[k] = _y.components[k].device_data();
        f *= _x.components[k].factor * _y.components[k].factor;
    }
    return f * guard([&] { return xrs::tt::dot(gpu::handle(), d, _x.dimensions.data(), rx.data(), X.data(), ry.data(), Y.data()); });
}

bool approx_equal(const TTTensor& _a, const TTTensor& _b, const value_t _eps) {
    XERUS_REQUIRE(_a.dimensions == _b.dimensions, "The dimensions of the compared tensors don't match");
    TTTensor diff = _a - _b;
    diff.move_core(0);
    return diff.frob_norm() <= _eps * (_a.frob_norm() + _b.frob_norm()) / 2.0;
}

IndexedTensor<TTTensor> TTTensor::operator()(const std::vector<Index>& _indices) const {
    IndexedTensor<TTTensor> r;
    r.tt = this;
    r.indices = _indices;
    return r;
}

IndexedTTProduct operator*(const IndexedTensor<TTTensor>& _a, const IndexedTensor<TTTensor>& _b) {
    IndexedTTProduct p;
    p.x = _a.tt;
    p.y = _b.tt;
    p.ix = _a.indices;
    p.iy = _b.indices;
    return p;
}

// value_t(x(i&0)*y(i&0)): identical index lists contract mode by mode = the TT zipper on the GPU; any
// other index pattern goes through the dense expression engine.
IndexedTTProduct::operator value_t() const {
    const size_t d = x->degree();
    bool zipper = y->degree() == d && ix.size() == iy.size();
    size_t spanSum = 0;
    for (size_t k = 0; zipper && k < ix.size(); ++k) {
        const size_t s = ix[k].actual_span(d);
        zipper = !ix[k].fixed() && ix[k] == iy[k] && s == iy[k].actual_span(d);
        for (size_t j = 0; zipper && j < k; ++j) zipper = ix[j] != ix[k];
        spanSum += s;
    }
    zipper = zipper && spanSum == d;
    if (zipper) return scale * dot(*x, *y);
    const Tensor X = x->to_tensor(), Y = y->to_tensor();
    return scale * value_t(X(ix) * Y(iy));
}

}  // namespace xerus
