// TTOperator on HBM and the TTStack contraction (operator application). A TTOperator's cores
// (r, n, m, r') are, byte for byte, the cores (r, n m, r') of a TTTensor with merged modes, so
// move_core / round / sums / norms run through the TT drivers on that view (the reference's TTNetwork
// code is the same template for N = 1 and N = 2: ttNetwork.cpp:57-160, 582-684, 797-847).
// Application: xrs_tt_operator_apply (ttop.hip) per core, then the canonicalisation the reference's
// TTStack performs when the operator was canonical (ttStack.cpp:160-168, ttNetwork.cpp:1075-1093).
#include <algorithm>
#include <cmath>

#include "../runtime.hpp"
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

size_t half(const std::vector<size_t>& _dims) { return _dims.size() / 2; }

// the positions where an index list splits into two halves of `_half` modes each, or npos
size_t split_point(const std::vector<Index>& _idx, size_t _degree) {
    if (_degree == 0) return _idx.size() % 2 == 0 ? _idx.size() / 2 : std::string::npos;   // A(i/2, j/2) of order 0
    size_t span = 0, k = 0;
    while (k < _idx.size() && span < _degree / 2) span += _idx[k++].actual_span(_degree);
    return span == _degree / 2 ? k : std::string::npos;
}

bool same_indices(const std::vector<Index>& _a, size_t _aDeg, size_t _a0, size_t _a1, const std::vector<Index>& _b, size_t _bDeg) {
    if (_a1 - _a0 != _b.size()) return false;
    for (size_t k = 0; k < _b.size(); ++k) {
        if (_a[_a0 + k].fixed() || _b[k].fixed()) return false;
        if (!(_a[_a0 + k] == _b[k]) || _a[_a0 + k].actual_span(_aDeg) != _b[k].actual_span(_bDeg)) return false;
    }
    return true;
}

}  // namespace

// ------------------------------------------------------------------------------ construction / views
std::vector<size_t> TTOperator::merged_dimensions(const std::vector<size_t>& _dimensions) {
    XERUS_REQUIRE(_dimensions.size() % 2 == 0, "Illegal number of dimensions for ttOperator");
    const size_t d = _dimensions.size() / 2;
    std::vector<size_t> m(d);
    for (size_t k = 0; k < d; ++k) m[k] = _dimensions[k] * _dimensions[d + k];
    return m;
}

TTTensor TTOperator::to_tt() && {
    const size_t d = half(dimensions);
    TTTensor t(merged_dimensions(dimensions));
    if (d == 0) {
        t.components[0] = std::move(components[0]);
    } else {
        for (size_t k = 0; k < d; ++k) {
            Tensor c = std::move(components[k]);
            const auto& cd = c.dimensions;
            c.reinterpret_dimensions({cd[0], cd[1] * cd[2], cd[3]});
            t.components[k] = std::move(c);
        }
    }
    t.canonicalized = canonicalized;
    t.corePosition = corePosition;
    return t;
}

TTOperator TTOperator::from_tt(TTTensor&& _tt, const std::vector<size_t>& _dimensions) {
    TTOperator o;
    o.dimensions = _dimensions;
    const size_t d = half(_dimensions);
    o.components.clear();
    if (d == 0) {
        o.components.push_back(std::move(_tt.components[0]));
    } else {
        for (size_t k = 0; k < d; ++k) {
            Tensor c = std::move(_tt.components[k]);
            const auto cd = c.dimensions;
            c.reinterpret_dimensions({cd[0], _dimensions[k], _dimensions[d + k], cd[2]});
            o.components.push_back(std::move(c));
        }
    }
    o.canonicalized = _tt.canonicalized;
    o.corePosition = _tt.corePosition;
    return o;
}

TTOperator::TTOperator() : components(1), dimensions(), canonicalized(true), corePosition(0) {}

TTOperator::TTOperator(size_t _degree) : TTOperator(Tensor::DimensionTuple(_degree, 1)) {}

TTOperator::TTOperator(const Tensor::DimensionTuple& _dimensions) : dimensions(_dimensions), canonicalized(true), corePosition(0) {
    XERUS_REQUIRE(dimensions.size() % 2 == 0, "Illegal degree for TTOperator.");
    XERUS_REQUIRE(std::find(dimensions.begin(), dimensions.end(), size_t(0)) == dimensions.end(), "Zero is no valid dimension.");
    const size_t d = half(dimensions);
    if (d == 0) {
        components.resize(1);
        return;
    }
    for (size_t i = 0; i < d; ++i) components.push_back(Tensor::dirac({1, dimensions[i], dimensions[d + i], 1}, 0));
    components[0][0] = 0.0;   // zero tensor, core at 0 (ttNetwork.cpp:104-107)
}

TTOperator::TTOperator(const Tensor& _tensor, const double _eps, const size_t _maxRank)
    : TTOperator(_tensor, _eps, std::vector<size_t>(_tensor.degree() < 2 ? 0 : _tensor.degree() / 2 - 1, _maxRank)) {}

// TT-SVD with the modes interleaved (i_0, j_0, i_1, j_1, ...) first (ttNetwork.cpp:128-136): the
// splits 1 + 2 position of the reference are the merged-mode splits 1 + position
TTOperator::TTOperator(const Tensor& _tensor, const double _eps, const std::vector<size_t>& _maxRanks) : TTOperator() {
    XERUS_REQUIRE(_tensor.degree() % 2 == 0, "Number of indicis must be even for TTOperator");
    XERUS_REQUIRE(_eps >= 0 && _eps < 1, "_eps must be positive and smaller than one. " << _eps << " was given.");
    const size_t d = _tensor.degree() / 2;
    XERUS_REQUIRE(_maxRanks.size() == (d == 0 ? 0 : d - 1), "We need " << (d == 0 ? 0 : d - 1) << " ranks but " << _maxRanks.size() << " where given");
    if (d == 0) {
        components[0] = _tensor;
        return;
    }
    std::vector<size_t> shuffle(2 * d);
    for (size_t i = 0; i < d; ++i) {
        shuffle[i] = 2 * i;
        shuffle[d + i] = 2 * i + 1;
    }
    Tensor inter = reshuffle(_tensor, shuffle);
    inter.reinterpret_dimensions(merged_dimensions(_tensor.dimensions));
    *this = from_tt(TTTensor(inter, _eps, _maxRanks), _tensor.dimensions);
}

TTOperator TTOperator::identity(const std::vector<size_t>& _dimensions) {
    XERUS_REQUIRE(_dimensions.size() % 2 == 0, "Illegal number of dimensions for ttOperator");
    XERUS_REQUIRE(std::find(_dimensions.begin(), _dimensions.end(), size_t(0)) == _dimensions.end(),
                  "Trying to construct a TTTensor with dimension 0 is not possible.");
    if (_dimensions.empty()) {
        TTOperator r;
        r.components[0] = Tensor::ones({});
        return r;
    }
    const size_t d = half(_dimensions);
    TTOperator result(_dimensions);
    for (size_t i = 0; i < d; ++i)
        result.set_component(i, Tensor({1, _dimensions[i], _dimensions[d + i], 1},
                                       [](const Tensor::MultiIndex& _idx) { return _idx[1] == _idx[2] ? 1.0 : 0.0; }));
    result.canonicalized = false;
    result.canonicalize_left();
    return result;
}

TTOperator TTOperator::ones(const std::vector<size_t>& _dimensions) {
    XERUS_REQUIRE(_dimensions.size() % 2 == 0, "Illegal number of dimensions for ttOperator");
    if (_dimensions.empty()) {
        TTOperator r;
        r.components[0] = Tensor::ones({});
        return r;
    }
    const size_t d = half(_dimensions);
    TTOperator result(_dimensions);
    for (size_t i = 0; i < d; ++i) result.set_component(i, Tensor::ones({1, _dimensions[i], _dimensions[d + i], 1}));
    result.canonicalized = false;
    result.canonicalize_left();
    return result;
}

// ------------------------------------------------------------------------------ structure
std::vector<size_t> TTOperator::ranks() const {
    std::vector<size_t> r;
    for (size_t k = 0; k + 1 < half(dimensions); ++k) r.push_back(components[k].dimensions.back());
    return r;
}

size_t TTOperator::rank(const size_t _i) const {
    XERUS_REQUIRE(_i + 1 < half(dimensions), "Requested illegal rank " << _i);
    return components[_i].dimensions.back();
}

Tensor& TTOperator::component(const size_t _idx) {
    XERUS_REQUIRE(_idx == 0 || _idx < half(dimensions), "Illegal index " << _idx << " in TTNetwork::component");
    return components[_idx];
}

void TTOperator::set_component(const size_t _idx, Tensor _T) {
    const size_t d = half(dimensions);
    if (d == 0) {
        XERUS_REQUIRE(_idx == 0 && _T.degree() == 0, "Component of degree zero TTNetwork must have degree zero.");
        components[0] = std::move(_T);
        return;
    }
    XERUS_REQUIRE(_idx < d, "Illegal index " << _idx << " in TTNetwork::set_component");
    XERUS_REQUIRE(_T.degree() == 4, "Component " << _idx << " must have degree 4. Given: " << _T.degree());
    dimensions[_idx] = _T.dimensions[1];
    dimensions[d + _idx] = _T.dimensions[2];
    components[_idx] = std::move(_T);
    canonicalized = canonicalized && corePosition == _idx;
}

void TTOperator::require_correct_format() const {
    XERUS_REQUIRE(dimensions.size() % 2 == 0, "Illegal degree for TTOperator.");
    const size_t d = half(dimensions);
    if (d == 0) {
        XERUS_REQUIRE(components.size() == 1 && components[0].degree() == 0, "degree-0 TTOperator must hold one scalar");
        return;
    }
    XERUS_REQUIRE(components.size() == d, "TTOperator has " << components.size() << " components for " << d << " modes");
    for (size_t k = 0; k < d; ++k) {
        const auto& c = components[k].dimensions;
        XERUS_REQUIRE(c.size() == 4, "Component " << k << " must have degree 4");
        XERUS_REQUIRE(c[1] == dimensions[k] && c[2] == dimensions[d + k], "Component " << k << " has wrong external dimensions");
        XERUS_REQUIRE(k == 0 ? c[0] == 1 : c[0] == components[k - 1].dimensions[3], "Rank mismatch left of component " << k);
    }
    XERUS_REQUIRE(components[d - 1].dimensions[3] == 1, "last rank must be 1");
}

void TTOperator::assume_core_position(const size_t _pos) {
    XERUS_REQUIRE(_pos < half(dimensions) || (dimensions.empty() && _pos == 0), "Invalid core position.");
    corePosition = _pos;
    canonicalized = true;
}

// ------------------------------------------------------------------------------ TT-view operations
void TTOperator::move_core(const size_t _position, const bool _keepRank) {
    require_correct_format();
    const std::vector<size_t> dims = dimensions;
    TTTensor t = std::move(*this).to_tt();
    try {
        t.move_core(_position, _keepRank);
    } catch (...) {
        *this = from_tt(std::move(t), dims);
        throw;
    }
    *this = from_tt(std::move(t), dims);
}

void TTOperator::round(const std::vector<size_t>& _maxRanks, const double _eps) {
    require_correct_format();
    const std::vector<size_t> dims = dimensions;
    TTTensor t = std::move(*this).to_tt();
    try {
        t.round(_maxRanks, _eps);
    } catch (...) {
        *this = from_tt(std::move(t), dims);
        throw;
    }
    *this = from_tt(std::move(t), dims);
}

void TTOperator::round(const size_t _maxRank) { round(std::vector<size_t>(half(dimensions) < 1 ? 0 : half(dimensions) - 1, _maxRank), EPSILON); }

void TTOperator::round(const int _maxRank) {
    XERUS_REQUIRE(_maxRank > 0, "MaxRank must be positive");
    round(size_t(_maxRank));
}

void TTOperator::round(const value_t _eps) {
    round(std::vector<size_t>(half(dimensions) < 1 ? 0 : half(dimensions) - 1, std::numeric_limits<size_t>::max()), _eps);
}

value_t TTOperator::frob_norm() const {
    require_correct_format();
    if (canonicalized) return components[corePosition].frob_norm();
    TTOperator c = *this;
    return std::move(c).to_tt().frob_norm();
}

void TTOperator::transpose() {
    const size_t d = half(dimensions);
    for (size_t k = 0; k < d; ++k) components[k] = reshuffle(components[k], {0, 2, 1, 3});
    for (size_t k = 0; k < d; ++k) std::swap(dimensions[k], dimensions[d + k]);
}

TTOperator& TTOperator::operator+=(const TTOperator& _other) {
    XERUS_REQUIRE(dimensions == _other.dimensions, "The dimensions in TT sum must coincide.");
    const std::vector<size_t> dims = dimensions;
    TTOperator o = _other;
    TTTensor t = std::move(*this).to_tt();
    t += std::move(o).to_tt();
    *this = from_tt(std::move(t), dims);
    return *this;
}

TTOperator& TTOperator::operator-=(const TTOperator& _other) {
    *this *= -1.0;
    *this += _other;
    *this *= -1.0;
    return *this;
}

TTOperator& TTOperator::operator*=(const value_t _factor) {
    components[canonicalized ? corePosition : 0] *= _factor;
    return *this;
}

TTOperator& TTOperator::operator/=(const value_t _divisor) { return *this *= 1 / _divisor; }

TTOperator operator+(TTOperator _lhs, const TTOperator& _rhs) { return _lhs += _rhs; }
TTOperator operator-(TTOperator _lhs, const TTOperator& _rhs) { return _lhs -= _rhs; }
TTOperator operator*(const value_t _factor, TTOperator _op) { return _op *= _factor; }
TTOperator operator*(TTOperator _op, const value_t _factor) { return _op *= _factor; }
TTOperator operator/(TTOperator _op, const value_t _divisor) { return _op /= _divisor; }

Tensor TTOperator::to_tensor() const {
    require_correct_format();
    const size_t d = half(dimensions);
    if (d == 0) return components[0];
    TTOperator c = *this;
    Tensor inter = std::move(c).to_tt().to_tensor();   // modes (n_0 m_0, ..., n_{d-1} m_{d-1})
    std::vector<size_t> idims, shuffle(2 * d);
    for (size_t k = 0; k < d; ++k) {
        idims.push_back(dimensions[k]);
        idims.push_back(dimensions[d + k]);
        shuffle[2 * k] = k;
        shuffle[2 * k + 1] = d + k;
    }
    inter.reinterpret_dimensions(idims);
    return reshuffle(inter, shuffle);
}

TTOperator::operator Tensor() const { return to_tensor(); }

// ------------------------------------------------------------------------------ indexed expressions
IndexedTensor<TTOperator> TTOperator::operator()(const std::vector<Index>& _indices) const {
    IndexedTensor<TTOperator> r;
    r.op = this;
    r.indices = _indices;
    return r;
}

IndexedTensor<TTOperator> TTOperator::operator()(const std::vector<Index>& _indices) {
    IndexedTensor<TTOperator> r;
    r.op = this;
    r.mut = this;
    r.indices = _indices;
    return r;
}

IndexedTensor<TTTensor> TTTensor::operator()(const std::vector<Index>& _indices) {
    IndexedTensor<TTTensor> r;
    r.tt = this;
    r.mut = this;
    r.indices = _indices;
    return r;
}

IndexedTTStack operator*(const IndexedTensor<TTOperator>& _a, const IndexedTensor<TTTensor>& _x) {
    const size_t D = _a.op->degree();
    const size_t mid = split_point(_a.indices, D);
    IndexedTTStack s;
    s.op = _a.op;
    s.vec = _x.tt;
    if (mid != std::string::npos && same_indices(_a.indices, D, mid, _a.indices.size(), _x.indices, _x.tt->degree())) {
        s.indices.assign(_a.indices.begin(), _a.indices.begin() + long(mid));   // A x
    } else if (mid != std::string::npos && same_indices(_a.indices, D, 0, mid, _x.indices, _x.tt->degree())) {
        s.transposed = true;   // A(i/2, j/2) * x(i&0) = x^T A
        s.indices.assign(_a.indices.begin() + long(mid), _a.indices.end());
    } else {
        XERUS_REQUIRE(false, "TTOperator * TTTensor: the vector's indices must be one half of the operator's");
    }
    return s;
}

IndexedTTStack operator*(const IndexedTensor<TTTensor>& _x, const IndexedTensor<TTOperator>& _a) {
    IndexedTTStack s = _a * _x;   // same contraction, operand order does not matter for the value
    return s;
}

IndexedTTStack operator*(const IndexedTensor<TTOperator>& _a, const IndexedTensor<TTOperator>& _b) {
    const size_t DA = _a.op->degree(), DB = _b.op->degree();
    const size_t ma = split_point(_a.indices, DA), mb = split_point(_b.indices, DB);
    XERUS_REQUIRE(ma != std::string::npos && mb != std::string::npos, "TTOperator * TTOperator: an index spans both halves");
    std::vector<Index> bFirst(_b.indices.begin(), _b.indices.begin() + long(mb));
    XERUS_REQUIRE(same_indices(_a.indices, DA, ma, _a.indices.size(), bFirst, DB),
                  "TTOperator * TTOperator: A's column indices must be B's row indices");
    IndexedTTStack s;
    s.op = _a.op;
    s.rhsOp = _b.op;
    s.indices.assign(_a.indices.begin(), _a.indices.begin() + long(ma));
    s.indices.insert(s.indices.end(), _b.indices.begin() + long(mb), _b.indices.end());
    return s;
}

namespace {

// the cores' device pointers and ranks of an operator / TT (factors applied)
struct CoreView {
    std::vector<size_t> r;
    std::vector<const double*> p;
    double factor = 1.0;
};

CoreView view_op(const TTOperator& _o) {
    CoreView v;
    const size_t d = _o.degree() / 2;
    v.r.assign(d + 1, 1);
    for (size_t k = 0; k < d; ++k) {
        v.r[k + 1] = _o.components[k].dimensions[3];
        v.p.push_back(_o.components[k].device_data());
        v.factor *= _o.components[k].factor;
    }
    return v;
}

CoreView view_tt(const TTTensor& _t) {
    CoreView v;
    const size_t d = _t.degree();
    v.r.assign(d + 1, 1);
    for (size_t k = 0; k < d; ++k) {
        v.r[k + 1] = _t.components[k].dimensions[2];
        v.p.push_back(_t.components[k].device_data());
        v.factor *= _t.components[k].factor;
    }
    return v;
}

}  // namespace

TTTensor IndexedTTStack::evaluate_tt() const {
    XERUS_REQUIRE(op && vec && !rhsOp, "not an operator-vector product");
    op->require_correct_format();
    vec->require_correct_format();
    const size_t d = op->degree() / 2;
    XERUS_REQUIRE(vec->degree() == d, "TTOperator and TTTensor orders differ");
    std::vector<size_t> n(op->dimensions.begin(), op->dimensions.begin() + long(d));
    std::vector<size_t> m(op->dimensions.begin() + long(d), op->dimensions.end());
    XERUS_REQUIRE(std::vector<size_t>(vec->dimensions) == (transposed ? n : m), "TTOperator * TTTensor: mode sizes differ");
    if (d == 0) {   // order 0: the product of the two scalars
        TTTensor result(std::vector<size_t>{});
        Tensor c = op->components[0];
        c *= vec->components[0][size_t(0)];
        result.components[0] = std::move(c);
        return result;
    }
    const CoreView A = view_op(*op), X = view_tt(*vec);
    std::vector<double*> out(d, nullptr);
    guard([&] {
        const int st = xrs_tt_operator_apply(gpu::handle(), d, n.data(), m.data(), nullptr, A.r.data(), A.p.data(), X.r.data(),
                                             X.p.data(), transposed ? 1 : 0, out.data());
        if (st != XRS_OK) throw xrs::Error{st, xrs_last_error()};
    });
    TTTensor result(transposed ? m : n);
    for (size_t k = 0; k < d; ++k)
        result.components[k] = Tensor::adopt_device({A.r[k] * X.r[k], transposed ? m[k] : n[k], A.r[k + 1] * X.r[k + 1]}, out[k]);
    result.components[0] *= A.factor * X.factor;
    result.canonicalized = false;
    if (op->canonicalized) result.move_core(op->corePosition);   // ttStack.cpp:163-166
    return result;
}

TTOperator IndexedTTStack::evaluate_op() const {
    XERUS_REQUIRE(op && rhsOp, "not an operator-operator product");
    op->require_correct_format();
    rhsOp->require_correct_format();
    const size_t d = op->degree() / 2;
    XERUS_REQUIRE(rhsOp->degree() / 2 == d, "TTOperator orders differ");
    std::vector<size_t> n(op->dimensions.begin(), op->dimensions.begin() + long(d));
    std::vector<size_t> m(op->dimensions.begin() + long(d), op->dimensions.end());
    std::vector<size_t> mb(rhsOp->dimensions.begin(), rhsOp->dimensions.begin() + long(d));
    std::vector<size_t> p(rhsOp->dimensions.begin() + long(d), rhsOp->dimensions.end());
    XERUS_REQUIRE(m == mb, "TTOperator * TTOperator: mode sizes differ");
    if (d == 0) {
        TTOperator result(std::vector<size_t>{});
        Tensor c = op->components[0];
        c *= rhsOp->components[0][size_t(0)];
        result.components[0] = std::move(c);
        return result;
    }
    const CoreView A = view_op(*op), B = view_op(*rhsOp);
    std::vector<double*> out(d, nullptr);
    guard([&] {
        const int st = xrs_tt_operator_apply(gpu::handle(), d, n.data(), m.data(), p.data(), A.r.data(), A.p.data(), B.r.data(),
                                             B.p.data(), 0, out.data());
        if (st != XRS_OK) throw xrs::Error{st, xrs_last_error()};
    });
    std::vector<size_t> dims = n;
    dims.insert(dims.end(), p.begin(), p.end());
    TTOperator result(dims);
    for (size_t k = 0; k < d; ++k) result.components[k] = Tensor::adopt_device({A.r[k] * B.r[k], n[k], p[k], A.r[k + 1] * B.r[k + 1]}, out[k]);
    result.components[0] *= A.factor * B.factor;
    result.canonicalized = false;
    if (op->canonicalized) result.move_core(op->corePosition);
    return result;
}

IndexedTensor<TTTensor>& IndexedTensor<TTTensor>::operator=(const IndexedTTStack& _stack) {
    XERUS_REQUIRE(mut, "assignment to a const TTTensor");
    XERUS_REQUIRE(!_stack.rhsOp, "an operator product cannot be assigned to a TTTensor");
    XERUS_REQUIRE(same_indices(indices, _stack.op->degree() / 2, 0, indices.size(), _stack.indices, _stack.op->degree()),
                  "TTTensor assignment: the indices must be the free indices of the product in order");
    *mut = _stack.evaluate_tt();
    return *this;
}

IndexedTensor<TTOperator>& IndexedTensor<TTOperator>::operator=(const IndexedTTStack& _stack) {
    XERUS_REQUIRE(mut, "assignment to a const TTOperator");
    XERUS_REQUIRE(_stack.rhsOp, "a vector product cannot be assigned to a TTOperator");
    const size_t D = _stack.op->degree();
    XERUS_REQUIRE(indices.size() == _stack.indices.size(), "TTOperator assignment: the indices must be the free indices of the product");
    for (size_t k = 0; k < indices.size(); ++k) XERUS_REQUIRE(indices[k] == _stack.indices[k], "TTOperator assignment: index order differs");
    (void)D;
    *mut = _stack.evaluate_op();
    return *this;
}

value_t operator*(const IndexedTTStack& _s, const IndexedTensor<TTTensor>& _y) {
    XERUS_REQUIRE(_s.vec && !_s.rhsOp, "scalar product needs an operator-vector product");
    XERUS_REQUIRE(same_indices(_s.indices, _s.op->degree(), 0, _s.indices.size(), _y.indices, _y.tt->degree()),
                  "the TTTensor's indices must be the product's free indices");
    return dot(_s.evaluate_tt(), *_y.tt);
}

}  // namespace xerus
