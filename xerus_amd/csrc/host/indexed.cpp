// Indexed expressions on Tensors: A(i,j) = B(i,k,l)*C(k,j,l), A(i^2) = B(i^2)+C(i^2), traces, slices.
//
// Evaluation follows the reference's lowering (indexedTensorWritable.cpp:68-119, tensorNetwork.cpp:553-675):
//   1. per factor: spans are resolved against the factor's degree (index.cpp:64-92), then fixed
//      indices and traces inside one factor are applied in ONE strided-gather kernel pass
//      (internal::evaluate, indexedTensor_tensor_evaluate.cpp:248-390; k_strided_eval);
//   2. indices shared by two factors become network links, indices occurring once stay open (in order
//      of appearance); a third occurrence is an error;
//   3. components without open indices contract to a scalar factor, the rest through
//      TensorNetwork::contract(set) (pairwise permute+GEMM in the reference's heuristic order);
//   4. the result is permuted once into the order of the left-hand side.
// Factors and the product's scale are carried as lazy Tensor::factor and land in the GEMM alpha.
#include <algorithm>
#include <map>
#include <set>

#include "../elementwise.hpp"
#include "xerus.h"

namespace xerus {

IndexedTensor<Tensor> Tensor::operator()(const std::vector<Index>& _indices) { return IndexedTensor<Tensor>(this, _indices, true); }

IndexedTensor<Tensor> Tensor::operator()(std::vector<Index>&& _indices) { return IndexedTensor<Tensor>(this, std::move(_indices), true); }

IndexedTensor<Tensor> Tensor::operator()(const std::vector<Index>& _indices) const {
    return IndexedTensor<Tensor>(const_cast<Tensor*>(this), _indices, false);
}

namespace internal {
namespace {

struct OpenIndex {
    Index idx;      // span resolved
    size_t first;   // first mode in the reduced tensor
};

struct Reduced {
    Tensor tensor;
    std::vector<OpenIndex> open;
};

std::vector<size_t> row_strides(const std::vector<size_t>& _dims) {
    std::vector<size_t> s(_dims.size());
    size_t acc = 1;
    for (size_t k = _dims.size(); k-- > 0;) {
        s[k] = acc;
        acc *= _dims[k];
    }
    return s;
}

// spans resolved against _degree, span-0 indices removed (indexedTensorReadOnly.cpp:81-115)
std::vector<Index> resolve(const std::vector<Index>& _indices, size_t _degree) {
    std::vector<Index> out;
    size_t count = 0;
    for (const Index& i : _indices) {
        Index r(i.valueId, i.actual_span(_degree), i.flags & Index::FIXED);
        count += r.span;
        if (r.span) out.push_back(r);
    }
    XERUS_REQUIRE(count >= _degree, "Order determined by Indices is to small. Order according to the indices " << count
                                                                                                              << ", according to the tensor " << _degree);
    XERUS_REQUIRE(count <= _degree, "Order determined by Indices is to large. Order according to the indices " << count
                                                                                                              << ", according to the tensor " << _degree);
    return out;
}

Reduced reduce_term(const IndexedTerm& _term) {
    const Tensor& T = *_term.tensor;
    const std::vector<Index> idx = resolve(_term.indices, T.degree());
    const std::vector<size_t> str = row_strides(T.dimensions);

    std::vector<size_t> outDims, inStr, trDims, trStr;
    size_t base = 0;
    bool work = false;
    Reduced r;
    size_t mode = 0;
    std::vector<size_t> firstMode(idx.size());
    for (size_t k = 0; k < idx.size(); ++k) {
        firstMode[k] = mode;
        mode += idx[k].span;
    }
    for (size_t k = 0; k < idx.size(); ++k) {
        const Index& I = idx[k];
        const size_t m0 = firstMode[k];
        if (I.fixed()) {
            XERUS_REQUIRE(I.fixed_position() < T.dimensions[m0],
                          "Fixed index position " << I.fixed_position() << " out of range for dimension " << T.dimensions[m0]);
            base += I.fixed_position() * str[m0];
            work = true;
            continue;
        }
        size_t other = idx.size();
        for (size_t j = 0; j < idx.size(); ++j)
            if (j != k && idx[j] == I) {
                XERUS_REQUIRE(other == idx.size(), "An index must not appere more than twice!");
                other = j;
            }
        if (other == idx.size()) {   // open
            r.open.push_back(OpenIndex{I, outDims.size()});
            for (size_t s = 0; s < I.span; ++s) {
                outDims.push_back(T.dimensions[m0 + s]);
                inStr.push_back(str[m0 + s]);
            }
            continue;
        }
        work = true;
        if (other < k) continue;   // trace handled at its first occurrence
        XERUS_REQUIRE(I.span == idx[other].span, "Index spans do not coincide " << I << " vs " << idx[other]);
        for (size_t s = 0; s < I.span; ++s) {
            XERUS_REQUIRE(T.dimensions[m0 + s] == T.dimensions[firstMode[other] + s], "The dimensions of the traced modes must coincide");
            trDims.push_back(T.dimensions[m0 + s]);
            trStr.push_back(str[m0 + s] + str[firstMode[other] + s]);
        }
    }
    if (!work) {
        r.tensor = T;
        return r;
    }
    Tensor out(outDims, Tensor::Representation::Dense, Tensor::Initialisation::None);
    const double* src = T.device_data();
    double* dst = out.device_data_for_write();
    try {
        xrs::strided_eval(gpu::handle(), dst, src, outDims.size(), outDims.data(), inStr.data(), trDims.size(), trDims.data(),
                          trStr.data(), base);
    } catch (const xrs::Error& e) {
        throw misc::generic_error(e.msg);
    }
    out.factor = T.factor;
    r.tensor = std::move(out);
    return r;
}

struct Lowered {
    TensorNetwork net;
    std::vector<Index> openIndices;   // external indices in slot order (span resolved)
};

Lowered lower(const IndexedProduct& _p) {
    // an index occurs at most twice over the whole product, traces inside one factor included (the
    // reference's network assembly rejects E(i2) = A(i1,i1,i2) * B(i2,i2): tensorNetwork.cxx:193-218)
    {
        std::map<uint64, size_t> count;
        for (const IndexedTerm& t : _p.terms)
            for (const Index& I : t.indices)
                if (!I.fixed()) XERUS_REQUIRE(++count[I.valueId] <= 2, "Index must not appear three (or more) times.");
    }
    std::vector<Reduced> terms;
    terms.reserve(_p.terms.size());
    for (const IndexedTerm& t : _p.terms) terms.push_back(reduce_term(t));

    // occurrences of every open index over all factors
    std::map<uint64, std::vector<std::pair<size_t, size_t>>> occ;   // id -> (term, open#)
    for (size_t t = 0; t < terms.size(); ++t)
        for (size_t k = 0; k < terms[t].open.size(); ++k) occ[terms[t].open[k].idx.valueId].emplace_back(t, k);

    Lowered L;
    TensorNetwork& net = L.net;
    net.nodes.clear();
    net.dimensions.clear();
    net.externalLinks.clear();
    for (size_t t = 0; t < terms.size(); ++t) {
        std::vector<TensorNetwork::Link> links(terms[t].tensor.degree());
        net.nodes.emplace_back(std::unique_ptr<Tensor>(new Tensor(std::move(terms[t].tensor))), std::move(links));
    }
    for (size_t t = 0; t < terms.size(); ++t) {
        for (size_t k = 0; k < terms[t].open.size(); ++k) {
            const OpenIndex& oi = terms[t].open[k];
            const auto& o = occ[oi.idx.valueId];
            XERUS_REQUIRE(o.size() <= 2, "Index must not appear three (or more) times.");
            const std::vector<size_t>& dims = net.nodes[t].tensorObject->dimensions;
            if (o.size() == 1) {
                L.openIndices.push_back(oi.idx);
                for (size_t s = 0; s < oi.idx.span; ++s) {
                    const size_t slot = net.externalLinks.size();
                    net.nodes[t].neighbors[oi.first + s] = TensorNetwork::Link(~size_t(0), slot, dims[oi.first + s], true);
                    net.externalLinks.emplace_back(t, oi.first + s, dims[oi.first + s], false);
                    net.dimensions.push_back(dims[oi.first + s]);
                }
                continue;
            }
            const auto& partner = (o[0].first == t && o[0].second == k) ? o[1] : o[0];
            const OpenIndex& po = terms[partner.first].open[partner.second];
            XERUS_REQUIRE(oi.idx.span == po.idx.span, "Index spans do not coincide " << oi.idx << " vs " << po.idx);
            const std::vector<size_t>& pdims = net.nodes[partner.first].tensorObject->dimensions;
            for (size_t s = 0; s < oi.idx.span; ++s) {
                XERUS_REQUIRE(dims[oi.first + s] == pdims[po.first + s],
                              "Index dimensions do not coincide: [" << s << "] " << dims[oi.first + s] << " vs " << pdims[po.first + s]);
                net.nodes[t].neighbors[oi.first + s] = TensorNetwork::Link(partner.first, po.first + s, dims[oi.first + s], false);
            }
        }
    }
    return L;
}

// nodes not reachable from an external link contract to one scalar (tensorNetwork.cpp:134-198)
value_t contract_unconnected(TensorNetwork& _net) {
    if (_net.degree() == 0) return 1.0;
    std::vector<char> seen(_net.nodes.size(), 0);
    std::vector<size_t> stack;
    for (const auto& el : _net.externalLinks)
        if (!seen[el.other]) {
            seen[el.other] = 1;
            stack.push_back(el.other);
        }
    while (!stack.empty()) {
        const size_t cur = stack.back();
        stack.pop_back();
        for (const auto& l : _net.nodes[cur].neighbors)
            if (!l.external && !seen[l.other]) {
                seen[l.other] = 1;
                stack.push_back(l.other);
            }
    }
    std::set<size_t> rest;
    for (size_t i = 0; i < _net.nodes.size(); ++i)
        if (!seen[i] && !_net.nodes[i].erased) rest.insert(i);
    if (rest.empty()) return 1.0;
    const size_t r = _net.contract(rest);
    const value_t v = (*_net.nodes[r].tensorObject)[0];
    _net.nodes[r].erased = true;
    _net.nodes[r].tensorObject.reset();
    _net.sanitize();
    return v;
}

}  // namespace

std::vector<Index> resolve_indices(const std::vector<Index>& _indices, size_t _degree) { return resolve(_indices, _degree); }

// external slot -> position in the output index order (indexedTensorWritable.cpp:97-118)
static std::vector<size_t> output_slots(const Lowered& L, const std::vector<Index>& _out) {
    const size_t E = L.net.degree();
    const std::vector<Index> out = resolve(_out, E);
    std::vector<size_t> slotOf(E);
    std::vector<size_t> firstSlot(L.openIndices.size());
    size_t s = 0;
    for (size_t k = 0; k < L.openIndices.size(); ++k) {
        firstSlot[k] = s;
        s += L.openIndices[k].span;
    }
    std::vector<char> used(L.openIndices.size(), 0);
    size_t pos = 0;
    for (const Index& I : out) {
        XERUS_REQUIRE(!I.fixed(), "Traces and fixed indices are not allowed in the target of evaluation.");
        size_t k = 0;
        while (k < L.openIndices.size() && L.openIndices[k] != I) ++k;
        XERUS_REQUIRE(k < L.openIndices.size(), "Every index on the LHS must appear somewhere on the RHS, here: " << I);
        XERUS_REQUIRE(!used[k], "Traces and fixed indices are not allowed in the target of evaluation.");
        XERUS_REQUIRE(L.openIndices[k].span == I.span, "The indexSpans in the target and base of evaluation must coincide.");
        used[k] = 1;
        for (size_t q = 0; q < I.span; ++q) slotOf[firstSlot[k] + q] = pos++;
    }
    for (size_t k = 0; k < used.size(); ++k)
        XERUS_REQUIRE(used[k], "All indices of evalutation base must either be fixed, appear in the target or be part of a trace. Missing: "
                                   << L.openIndices[k]);
    return slotOf;
}

TensorNetwork product_network(const IndexedProduct& _p, const std::vector<Index>& _out) {
    XERUS_REQUIRE(!_p.terms.empty(), "empty product");
    Lowered L = lower(_p);
    const std::vector<size_t> slotOf = output_slots(L, _out);
    TensorNetwork& net = L.net;
    net.require_valid_network();
    // components without an external mode contract to one scalar, folded with the product's factor into a node
    const value_t scalar = contract_unconnected(net) * _p.scale;
    const size_t E = net.degree();
    std::vector<TensorNetwork::Link> ext(E);
    std::vector<size_t> dims(E);
    for (size_t s = 0; s < E; ++s) {
        ext[slotOf[s]] = net.externalLinks[s];
        dims[slotOf[s]] = net.dimensions[s];
    }
    for (TensorNetwork::TensorNode& node : net.nodes)
        for (TensorNetwork::Link& l : node.neighbors)
            if (l.external) l.indexPosition = slotOf[l.indexPosition];
    net.externalLinks = std::move(ext);
    net.dimensions = std::move(dims);
    if (scalar != 1.0) {
        for (TensorNetwork::TensorNode& node : net.nodes)
            if (!node.erased && node.tensorObject) {
                node.tensorObject->factor *= scalar;
                break;
            }
    }
    net.require_valid_network();
    return std::move(net);
}

Tensor evaluate_product(const IndexedProduct& _p, const std::vector<Index>& _out) {
    XERUS_REQUIRE(!_p.terms.empty(), "empty product");
    Lowered L = lower(_p);
    TensorNetwork& net = L.net;
    net.require_valid_network();
    const value_t scalar = contract_unconnected(net);

    std::set<size_t> all;
    for (size_t i = 0; i < net.nodes.size(); ++i)
        if (!net.nodes[i].erased) all.insert(i);
    const size_t res = net.contract(all);
    Tensor& R = *net.nodes[res].tensorObject;

    // output order (indexedTensorWritable.cpp:97-118)
    const std::vector<size_t> slotOf = output_slots(L, _out);
    std::vector<size_t> shuffle(R.degree());
    bool identity = true;
    for (size_t d = 0; d < R.degree(); ++d) {
        const auto& l = net.nodes[res].neighbors[d];
        XERUS_REQUIRE(l.external, "Internal Error: open link left after full contraction");
        shuffle[d] = slotOf[l.indexPosition];
        identity &= shuffle[d] == d;
    }
    Tensor result = identity ? std::move(R) : reshuffle(R, shuffle);
    result.factor *= _p.scale * scalar;
    return result;
}

}  // namespace internal

// ---------------------------------------------------------------------------------------------- products
IndexedProduct IndexedTensor<Tensor>::as_product() const {
    IndexedProduct p;
    p.terms.push_back(IndexedTerm{std::make_shared<const Tensor>(*tensorObject), indices});
    return p;
}

IndexedProduct::operator value_t() const {
    const Tensor t = internal::evaluate_product(*this, {});
    XERUS_REQUIRE(t.degree() == 0, "cannot cast tensors of degree > 0 to value_t. did you mean frob_norm() or similar?");
    return t[0];
}

IndexedTensor<Tensor>::operator value_t() const { return value_t(as_product()); }

IndexedTensor<Tensor>& IndexedTensor<Tensor>::operator=(const IndexedProduct& _rhs) {
    XERUS_REQUIRE(writable, "cannot assign to a const tensor");
    Tensor r = internal::evaluate_product(_rhs, indices);
    *tensorObject = std::move(r);
    return *this;
}

IndexedTensor<Tensor>& IndexedTensor<Tensor>::operator=(const IndexedTensor<Tensor>& _rhs) { return *this = _rhs.as_product(); }

IndexedTensor<Tensor>& IndexedTensor<Tensor>::operator=(const IndexedSum& _rhs) {
    XERUS_REQUIRE(writable, "cannot assign to a const tensor");
    XERUS_REQUIRE(!_rhs.summands.empty(), "empty sum");
    Tensor r = internal::evaluate_product(_rhs.summands[0], indices);
    for (size_t k = 1; k < _rhs.summands.size(); ++k) {
        const Tensor t = internal::evaluate_product(_rhs.summands[k], indices);
        r += t;
    }
    *tensorObject = std::move(r);
    return *this;
}

IndexedTensor<Tensor>& IndexedTensor<Tensor>::operator+=(const IndexedProduct& _rhs) {
    XERUS_REQUIRE(writable, "cannot assign to a const tensor");
    const Tensor t = internal::evaluate_product(_rhs, indices);
    *tensorObject += t;
    return *this;
}

IndexedTensor<Tensor>& IndexedTensor<Tensor>::operator-=(const IndexedProduct& _rhs) {
    XERUS_REQUIRE(writable, "cannot assign to a const tensor");
    const Tensor t = internal::evaluate_product(_rhs, indices);
    *tensorObject -= t;
    return *this;
}

IndexedTensor<Tensor>& IndexedTensor<Tensor>::operator+=(const IndexedTensor<Tensor>& _rhs) { return *this += _rhs.as_product(); }
IndexedTensor<Tensor>& IndexedTensor<Tensor>::operator-=(const IndexedTensor<Tensor>& _rhs) { return *this -= _rhs.as_product(); }

IndexedProduct operator*(IndexedProduct _a, const IndexedProduct& _b) {
    _a.terms.insert(_a.terms.end(), _b.terms.begin(), _b.terms.end());
    _a.scale *= _b.scale;
    return _a;
}
IndexedProduct operator*(const IndexedTensor<Tensor>& _a, const IndexedTensor<Tensor>& _b) { return _a.as_product() * _b.as_product(); }
IndexedProduct operator*(IndexedProduct _a, const IndexedTensor<Tensor>& _b) { return std::move(_a) * _b.as_product(); }
IndexedProduct operator*(const IndexedTensor<Tensor>& _a, IndexedProduct _b) { return _a.as_product() * _b; }
IndexedProduct operator*(const value_t _f, IndexedProduct _a) {
    _a.scale *= _f;
    return _a;
}
IndexedProduct operator*(IndexedProduct _a, const value_t _f) { return _f * std::move(_a); }
IndexedProduct operator*(const value_t _f, const IndexedTensor<Tensor>& _a) { return _f * _a.as_product(); }
IndexedProduct operator*(const IndexedTensor<Tensor>& _a, const value_t _f) { return _f * _a.as_product(); }
IndexedProduct operator/(IndexedProduct _a, const value_t _f) {
    _a.scale /= _f;
    return _a;
}
IndexedProduct operator/(const IndexedTensor<Tensor>& _a, const value_t _f) { return _a.as_product() / _f; }

// x(orderX) = b / A (indexedTensor_tensor_solve.cpp:31-75): A's indices shared with b come first (rows, in A's
// order), A's others are x's leading indices; b's indices not in A are extra trailing dimensions of both b
// and x. A and b are reshuffled into that order and solve() (tensor.cpp: LU / least squares) runs on them.
IndexedProduct operator/(const IndexedTensor<Tensor>& _b, const IndexedTensor<Tensor>& _A) {
    const std::vector<Index> ia = internal::resolve_indices(_A.indices, _A.tensorObject->degree());
    const std::vector<Index> ib = internal::resolve_indices(_b.indices, _b.tensorObject->degree());
    std::vector<Index> orderA, orderB, orderX;
    size_t extraDims = 0;
    for (const Index& idx : ia) {
        if (std::find(ib.begin(), ib.end(), idx) != ib.end()) orderA.push_back(idx);
        else orderX.push_back(idx);
    }
    orderB = orderA;
    orderA.insert(orderA.end(), orderX.begin(), orderX.end());
    for (const Index& idx : ib) {
        if (std::find(ia.begin(), ia.end(), idx) == ia.end()) {
            orderB.push_back(idx);
            orderX.push_back(idx);
            extraDims += idx.span;
        }
    }
    Tensor A, B;
    A(orderA) << _A.as_product();
    B(orderB) << _b.as_product();
    auto X = std::make_shared<Tensor>();
    solve(*X, A, B, extraDims);
    IndexedProduct p;
    p.terms.push_back(IndexedTerm{X, orderX});
    return p;
}
IndexedProduct operator-(IndexedProduct _a) { return -1.0 * std::move(_a); }
IndexedProduct operator-(const IndexedTensor<Tensor>& _a) { return -1.0 * _a.as_product(); }

IndexedSum operator+(IndexedSum _a, const IndexedProduct& _b) {
    _a.summands.push_back(_b);
    return _a;
}
IndexedSum operator-(IndexedSum _a, const IndexedProduct& _b) { return std::move(_a) + (-1.0 * _b); }
IndexedSum operator+(const IndexedProduct& _a, const IndexedProduct& _b) { return IndexedSum{{_a}} + _b; }
IndexedSum operator-(const IndexedProduct& _a, const IndexedProduct& _b) { return IndexedSum{{_a}} - _b; }
IndexedSum operator+(const IndexedTensor<Tensor>& _a, const IndexedTensor<Tensor>& _b) { return _a.as_product() + _b.as_product(); }
IndexedSum operator-(const IndexedTensor<Tensor>& _a, const IndexedTensor<Tensor>& _b) { return _a.as_product() - _b.as_product(); }
IndexedSum operator+(const IndexedTensor<Tensor>& _a, const IndexedProduct& _b) { return _a.as_product() + _b; }
IndexedSum operator-(const IndexedTensor<Tensor>& _a, const IndexedProduct& _b) { return _a.as_product() - _b; }
IndexedSum operator+(const IndexedProduct& _a, const IndexedTensor<Tensor>& _b) { return _a + _b.as_product(); }
IndexedSum operator-(const IndexedProduct& _a, const IndexedTensor<Tensor>& _b) { return _a - _b.as_product(); }
IndexedSum operator+(IndexedSum _a, const IndexedTensor<Tensor>& _b) { return std::move(_a) + _b.as_product(); }
IndexedSum operator-(IndexedSum _a, const IndexedTensor<Tensor>& _b) { return std::move(_a) - _b.as_product(); }

value_t frob_norm(const IndexedTensor<Tensor>& _idxTensor) { return _idxTensor.tensorObject->frob_norm(); }

// ---------------------------------------------------------------------------------------------- networks
IndexedNetwork& IndexedNetwork::operator=(const IndexedProduct& _rhs) {
    *network = internal::product_network(_rhs, indices);
    return *this;
}

IndexedNetwork& IndexedNetwork::operator=(const IndexedTensor<Tensor>& _rhs) { return *this = _rhs.as_product(); }

}  // namespace xerus
