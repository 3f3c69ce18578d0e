// TT operations around rounding: named constructors (kronecker, dirac), fix_mode / resize_mode / chop, and
// the products whose results are the canonical inputs of round() (entrywise product: rank r_A r_B;
// dyadic product). Reference: ttNetwork.cpp:224-283 (constructors), :432-446 (fix_mode, resize_mode),
// :515-580 (chop), :748-778 (contract_unconnected_subnetworks), :1209-1309 (entrywise_product),
// :1319-1445 (dyadic_product); tensor.cpp:1708-1740 (dense entrywise_product).
// The core products run on the GPU (xrs_tt_entrywise_product, ttop.hip); the structural operations move
// device buffers (slices, 2-D copies and GEMMs of the existing Tensor operations).
#include <algorithm>
#include <limits>

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

// component product of two TT core trains (r, ext, r') on the device, alpha into core 0
std::vector<double*> entrywise_cores(const std::vector<const Tensor*>& _A, const std::vector<const Tensor*>& _B,
                                     std::vector<size_t>& _ext, std::vector<size_t>& _ra, std::vector<size_t>& _rb) {
    const size_t d = _A.size();
    std::vector<const double*> pa(d), pb(d);
    value_t alpha = 1.0;
    for (size_t k = 0; k < d; ++k) {
        pa[k] = _A[k]->device_data();
        pb[k] = _B[k]->device_data();
        alpha *= _A[k]->factor * _B[k]->factor;
    }
    std::vector<double*> out(d, nullptr);
    guard([&] {
        const int st = xrs_tt_entrywise_product(gpu::handle(), d, _ext.data(), _ra.data(), pa.data(), _rb.data(), pb.data(), alpha,
                                                out.data());
        if (st != XRS_OK) throw xrs::Error{st, xrs_last_error()};
    });
    return out;
}

size_t min_dim(const std::vector<size_t>& _d) { return *std::min_element(_d.begin(), _d.end()); }

// Tensor::kronecker of the component dims (ranks min(dims) inside), boundary modes of size 1 added
Tensor kronecker_component(size_t _i, size_t _numNodes, size_t _minN, const std::vector<size_t>& _ext) {
    std::vector<size_t> dims;
    if (_i > 0) dims.push_back(_minN);
    dims.insert(dims.end(), _ext.begin(), _ext.end());
    if (_i + 1 < _numNodes) dims.push_back(_minN);
    Tensor c = Tensor::kronecker(dims);
    if (_i == 0) dims.insert(dims.begin(), 1);
    if (_i + 1 == _numNodes) dims.push_back(1);
    c.reinterpret_dimensions(dims);
    return c;
}

using Link = TensorNetwork::Link;
constexpr size_t kNoNode = std::numeric_limits<size_t>::max();

// the chain of components [first, last) as a TensorNetwork: the left part (_left: a ghost node ones({1})
// before component `first` = 0, the last rank external) or the right part (the first rank external, a ghost
// node after the last component). External order: rank (right part), row modes, column modes, rank (left
// part) -- TTNetwork::chop (ttNetwork.cpp:515-580). N = 1 (TTTensor) or 2 (TTOperator) external modes per core.
TensorNetwork chain_network(const std::vector<Tensor>& _comps, size_t _first, size_t _last, size_t _N, bool _left) {
    TensorNetwork net{TensorNetwork::Structure{}};
    const size_t nc = _last - _first;
    if (nc == 0) {   // the ghost node alone, its rank-1 link external
        net.nodes.emplace_back(std::unique_ptr<Tensor>(new Tensor(Tensor::ones({1}))), std::vector<Link>{Link(kNoNode, 0, 1, true)});
        net.dimensions = {1};
        net.externalLinks = {Link(0, 0, 1, false)};
        return net;
    }
    const size_t ghost = _left ? 0 : nc;          // node id of the ghost
    const size_t base = _left ? 1 : 0;            // node id of component _first
    const size_t lastMode = _N + 1;
    const size_t numExt = 1 + _N * nc;
    net.nodes.resize(nc + 1);
    net.dimensions.assign(numExt, 0);
    net.externalLinks.assign(numExt, Link());
    auto ext = [&](size_t slot, size_t node, size_t mode, size_t dim) {
        net.dimensions[slot] = dim;
        net.externalLinks[slot] = Link(node, mode, dim, false);
        return Link(kNoNode, slot, dim, true);
    };
    const size_t off = _left ? 0 : 1;             // external slots of the modes (after the rank on the right)
    for (size_t q = 0; q < nc; ++q) {
        const Tensor& c = _comps[_first + q];
        const size_t id = base + q;
        std::vector<Link> nb(c.degree());
        const size_t rl = c.dimensions.front(), rr = c.dimensions.back();
        if (q == 0) nb[0] = _left ? Link(ghost, 0, rl, false) : ext(0, id, 0, rl);
        else nb[0] = Link(id - 1, lastMode, rl, false);
        for (size_t e = 0; e < _N; ++e) nb[1 + e] = ext(off + e * nc + q, id, 1 + e, c.dimensions[1 + e]);
        if (q + 1 < nc) nb[lastMode] = Link(id + 1, 0, rr, false);
        else nb[lastMode] = _left ? ext(numExt - 1, id, lastMode, rr) : Link(ghost, 0, rr, false);
        net.nodes[id] = TensorNetwork::TensorNode(std::unique_ptr<Tensor>(new Tensor(c)), std::move(nb));
    }
    net.nodes[ghost] = TensorNetwork::TensorNode(std::unique_ptr<Tensor>(new Tensor(Tensor::ones({1}))),
                                                 {_left ? Link(base, 0, 1, false) : Link(base + nc - 1, lastMode, 1, false)});
    net.require_valid_network();
    return net;
}

}  // namespace

// ------------------------------------------------------------------------------------------ Tensor
Tensor::MultiIndex Tensor::position_to_multiIndex(size_t _position, const DimensionTuple& _dimensions) {
    MultiIndex idx(_dimensions.size());
    for (size_t k = _dimensions.size(); k-- > 0;) {
        idx[k] = _position % _dimensions[k];
        _position /= _dimensions[k];
    }
    XERUS_REQUIRE(_position == 0, "Invalid position for the given dimensions");
    return idx;
}

Tensor entrywise_product(const Tensor& _A, const Tensor& _B) {
    XERUS_REQUIRE(_A.dimensions == _B.dimensions, "Entrywise product ill-defined for non-equal dimensions.");
    if (_A.size == 0) return _A;
    std::vector<size_t> ext{_A.size}, r{1, 1};
    std::vector<double*> out = entrywise_cores({&_A}, {&_B}, ext, r, r);
    return Tensor::adopt_device(_A.dimensions, out[0]);
}

// ------------------------------------------------------------------------------------------ TTTensor
TTTensor TTTensor::kronecker(const std::vector<size_t>& _dimensions) {
    XERUS_REQUIRE(std::find(_dimensions.begin(), _dimensions.end(), size_t(0)) == _dimensions.end(),
                  "Trying to construct a TTNetwork with dimension 0 is not possible.");
    if (_dimensions.empty()) return TTTensor(Tensor::kronecker({}));
    const size_t d = _dimensions.size(), minN = min_dim(_dimensions);
    TTTensor result(_dimensions);
    for (size_t i = 0; i < d; ++i) result.set_component(i, kronecker_component(i, d, minN, {_dimensions[i]}));
    result.canonicalized = false;
    result.canonicalize_left();
    return result;
}

TTTensor TTTensor::dirac(std::vector<size_t> _dimensions, const std::vector<size_t>& _position) {
    XERUS_REQUIRE(std::find(_dimensions.begin(), _dimensions.end(), size_t(0)) == _dimensions.end(),
                  "Trying to construct a TTTensor with dimension 0 is not possible.");
    XERUS_REQUIRE(_dimensions.size() == _position.size(), "Inconsitend number of entries in _dimensions and _position.");
    if (_dimensions.size() <= 1) return TTTensor(Tensor::dirac(_dimensions, _position));
    TTTensor result(_dimensions);
    for (size_t i = 0; i < _dimensions.size(); ++i) result.set_component(i, Tensor::dirac({1, _dimensions[i], 1}, _position[i]));
    return result;
}

TTTensor TTTensor::dirac(std::vector<size_t> _dimensions, const size_t _position) {
    return dirac(_dimensions, Tensor::position_to_multiIndex(_position, _dimensions));
}

void TTTensor::fix_mode(const size_t _mode, const size_t _slatePosition) {
    require_correct_format();
    const size_t d = degree();
    XERUS_REQUIRE(_mode < d, "Invalid dimension to remove");
    XERUS_REQUIRE(_slatePosition < dimensions[_mode], "Invalide _slatePosition to choose");
    Tensor M = components[_mode];
    M.fix_mode(1, _slatePosition);                       // (r_k, r_{k+1})
    dimensions.erase(dimensions.begin() + long(_mode));
    if (d == 1) {                                        // degree 0: the scalar (contract everything)
        M.reinterpret_dimensions({});
        components.assign(1, std::move(M));
        canonicalized = false;
        corePosition = 0;
        return;
    }
    if (_mode + 1 < d) {   // contracted into the right neighbour, which takes the removed component's place
        Tensor next;
        contract(next, M, false, components[_mode + 1], false, 1);
        components[_mode + 1] = std::move(next);
        if (corePosition == _mode + 1) corePosition = _mode;
        else if (corePosition != _mode) canonicalized = false;
    } else {               // the last component: into its left neighbour
        Tensor prev;
        contract(prev, components[_mode - 1], false, M, false, 1);
        components[_mode - 1] = std::move(prev);
        if (corePosition == _mode) corePosition = _mode - 1;
        else if (corePosition != _mode - 1) canonicalized = false;
    }
    components.erase(components.begin() + long(_mode));
    if (!canonicalized) corePosition = 0;
    require_correct_format();
}

void TTTensor::resize_mode(const size_t _mode, const size_t _newDim, const size_t _cutPos) {
    require_correct_format();
    XERUS_REQUIRE(_mode < degree(), "Invalid dimension given for resize_mode");
    components[_mode].resize_mode(1, _newDim, _cutPos);
    dimensions[_mode] = _newDim;
    // (the reference compares the new dimension with the core position here, ttNetwork.cpp:440)
    if (canonicalized && _newDim != corePosition) {
        const size_t oldCorePosition = corePosition;
        move_core(_mode);
        move_core(oldCorePosition);
    }
}

std::pair<TensorNetwork, TensorNetwork> TTTensor::chop(const size_t _position) const {
    require_correct_format();
    const size_t d = degree();
    XERUS_REQUIRE(_position < d, "Can't split a " << d << " component TTNetwork at position " << _position);
    return {chain_network(components, 0, _position, 1, true), chain_network(components, _position + 1, d, 1, false)};
}

TTTensor entrywise_product(const TTTensor& _A, const TTTensor& _B) {
    XERUS_REQUIRE(_A.dimensions == _B.dimensions, "Entrywise_product ill-defined for different external dimensions.");
    _A.require_correct_format();
    _B.require_correct_format();
    const size_t d = _A.degree();
    if (d == 0) {
        TTTensor result(_A);
        result *= _B.components[0][0];
        return result;
    }
    std::vector<size_t> ext(_A.dimensions), ra(d + 1, 1), rb(d + 1, 1);
    std::vector<const Tensor*> ca(d), cb(d);
    for (size_t k = 0; k < d; ++k) {
        ra[k + 1] = _A.components[k].dimensions[2];
        rb[k + 1] = _B.components[k].dimensions[2];
        ca[k] = &_A.components[k];
        cb[k] = &_B.components[k];
    }
    std::vector<double*> out = entrywise_cores(ca, cb, ext, ra, rb);
    TTTensor result(_A.dimensions);
    for (size_t k = 0; k < d; ++k) result.components[k] = Tensor::adopt_device({ra[k] * rb[k], ext[k], ra[k + 1] * rb[k + 1]}, out[k]);
    result.canonicalized = false;
    if (_A.canonicalized && _B.canonicalized) result.move_core(_A.corePosition);
    return result;
}

namespace {

// the component train of lhs then rhs, canonicalised as ttNetwork.cpp:1402-1425 (both cores at the left end:
// the rhs core becomes the core, the lhs core's factor moves there, then move_core(0); both at the right end:
// symmetric); `numL` / `numR` components
template <class TT>
void dyadic_canonicalise(TT& _result, const TT& _lhs, const TT& _rhs, size_t _numL, size_t _numR) {
    _result.canonicalized = false;
    if (!(_lhs.canonicalized && _rhs.canonicalized)) return;
    if (_lhs.corePosition == 0 && _rhs.corePosition == 0) {
        _result.canonicalized = true;
        _result.corePosition = _numL;
        if (_result.components[0].has_factor()) {
            _result.components[_numL] *= _result.components[0].factor;
            _result.components[0].factor = 1.0;
        }
        _result.move_core(0);
    } else if (_lhs.corePosition == _numL - 1 && _rhs.corePosition == _numR - 1) {
        const size_t lastIdx = _numL + _numR - 1;
        _result.canonicalized = true;
        _result.corePosition = _numL - 1;
        if (_result.components[lastIdx].has_factor()) {
            _result.components[_numL - 1] *= _result.components[lastIdx].factor;
            _result.components[lastIdx].factor = 1.0;
        }
        _result.move_core(lastIdx);
    }
}

}  // namespace

TTTensor dyadic_product(const TTTensor& _lhs, const TTTensor& _rhs) {
    _lhs.require_correct_format();
    _rhs.require_correct_format();
    if (_lhs.degree() == 0) {
        TTTensor result(_rhs);
        result *= _lhs.components[0][0];
        return result;
    }
    if (_rhs.degree() == 0) {
        TTTensor result(_lhs);
        result *= _rhs.components[0][0];
        return result;
    }
    const size_t nl = _lhs.degree(), nr = _rhs.degree();
    TTTensor result(_lhs);
    result.dimensions.insert(result.dimensions.end(), _rhs.dimensions.begin(), _rhs.dimensions.end());
    result.components.insert(result.components.end(), _rhs.components.begin(), _rhs.components.end());
    dyadic_canonicalise(result, _lhs, _rhs, nl, nr);
    result.require_correct_format();
    return result;
}

TTTensor dyadic_product(const std::vector<TTTensor>& _tensors) {
    if (_tensors.empty()) return TTTensor();
    TTTensor result(_tensors.back());
    for (size_t i = _tensors.size() - 1; i > 0; --i) result = dyadic_product(_tensors[i - 1], result);
    return result;
}

// ------------------------------------------------------------------------------------------ TTOperator
TTOperator TTOperator::kronecker(const std::vector<size_t>& _dimensions) {
    XERUS_REQUIRE(_dimensions.size() % 2 == 0, "Illegal number of dimensions for ttOperator");
    XERUS_REQUIRE(std::find(_dimensions.begin(), _dimensions.end(), size_t(0)) == _dimensions.end(),
                  "Trying to construct a TTNetwork with dimension 0 is not possible.");
    if (_dimensions.empty()) return TTOperator(Tensor::kronecker({}));
    const size_t d = _dimensions.size() / 2, minN = min_dim(_dimensions);
    TTOperator result(_dimensions);
    for (size_t i = 0; i < d; ++i) result.components[i] = kronecker_component(i, d, minN, {_dimensions[i], _dimensions[d + i]});
    result.canonicalized = false;
    result.canonicalize_left();
    return result;
}

TTOperator TTOperator::dirac(std::vector<size_t> _dimensions, const std::vector<size_t>& _position) {
    XERUS_REQUIRE(_dimensions.size() % 2 == 0, "Illegal number of dimensions for ttOperator");
    XERUS_REQUIRE(std::find(_dimensions.begin(), _dimensions.end(), size_t(0)) == _dimensions.end(),
                  "Trying to construct a TTTensor with dimension 0 is not possible.");
    XERUS_REQUIRE(_dimensions.size() == _position.size(), "Inconsitend number of entries in _dimensions and _position.");
    const size_t d = _dimensions.size() / 2;
    if (d <= 1) return TTOperator(Tensor::dirac(_dimensions, _position));
    TTOperator result(_dimensions);
    for (size_t i = 0; i < d; ++i)
        result.set_component(i, Tensor::dirac({1, _dimensions[i], _dimensions[d + i], 1}, _position[i] * _dimensions[d + i] + _position[d + i]));
    return result;
}

TTOperator TTOperator::dirac(std::vector<size_t> _dimensions, const size_t _position) {
    return dirac(_dimensions, Tensor::position_to_multiIndex(_position, _dimensions));
}

void TTOperator::fix_mode(const size_t, const size_t) {
    XERUS_REQUIRE(false, "fix_mode(), does not work for TTOperators, if applicable cast to TensorNetwork first");
}

void TTOperator::resize_mode(const size_t _mode, const size_t _newDim, const size_t _cutPos) {
    require_correct_format();
    const size_t d = degree() / 2;
    XERUS_REQUIRE(_mode < degree(), "Invalid dimension given for resize_mode");
    components[_mode % d].resize_mode(_mode < d ? 1 : 2, _newDim, _cutPos);
    dimensions[_mode] = _newDim;
    if (canonicalized && _newDim != corePosition) {   // (as the reference, ttNetwork.cpp:440)
        const size_t oldCorePosition = corePosition;
        move_core(_mode % d);
        move_core(oldCorePosition);
    }
}

std::pair<TensorNetwork, TensorNetwork> TTOperator::chop(const size_t _position) const {
    require_correct_format();
    const size_t d = degree() / 2;
    XERUS_REQUIRE(_position < d, "Can't split a " << d << " component TTNetwork at position " << _position);
    return {chain_network(components, 0, _position, 2, true), chain_network(components, _position + 1, d, 2, false)};
}

TTOperator entrywise_product(const TTOperator& _A, const TTOperator& _B) {
    XERUS_REQUIRE(_A.dimensions == _B.dimensions, "Entrywise_product ill-defined for different external dimensions.");
    TTOperator A(_A), B(_B);
    const std::vector<size_t> dims = _A.dimensions;
    return TTOperator::from_tt(entrywise_product(std::move(A).to_tt(), std::move(B).to_tt()), dims);
}

TTOperator dyadic_product(const TTOperator& _lhs, const TTOperator& _rhs) {
    _lhs.require_correct_format();
    _rhs.require_correct_format();
    if (_lhs.degree() == 0) {
        TTOperator result(_rhs);
        result *= _lhs.components[0][0];
        return result;
    }
    if (_rhs.degree() == 0) {
        TTOperator result(_lhs);
        result *= _rhs.components[0][0];
        return result;
    }
    const size_t nl = _lhs.degree() / 2, nr = _rhs.degree() / 2;
    TTOperator result(_lhs);
    // rows of lhs, rows of rhs, columns of lhs, columns of rhs (ttNetwork.cpp:1377-1400)
    std::vector<size_t> dims(_lhs.dimensions.begin(), _lhs.dimensions.begin() + long(nl));
    dims.insert(dims.end(), _rhs.dimensions.begin(), _rhs.dimensions.begin() + long(nr));
    dims.insert(dims.end(), _lhs.dimensions.begin() + long(nl), _lhs.dimensions.end());
    dims.insert(dims.end(), _rhs.dimensions.begin() + long(nr), _rhs.dimensions.end());
    result.dimensions = dims;
    result.components.insert(result.components.end(), _rhs.components.begin(), _rhs.components.end());
    dyadic_canonicalise(result, _lhs, _rhs, nl, nr);
    result.require_correct_format();
    return result;
}

TTOperator dyadic_product(const std::vector<TTOperator>& _tensors) {
    if (_tensors.empty()) return TTOperator();
    TTOperator result(_tensors.back());
    for (size_t i = _tensors.size() - 1; i > 0; --i) result = dyadic_product(_tensors[i - 1], result);
    return result;
}

}  // namespace xerus
