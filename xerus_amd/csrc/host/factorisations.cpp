// Indexed factorisation expressions: (U(i,r), S(r,s), Vt(s,j)) = SVD(A(i,j), ...), QR / RQ / QC / CQ.
//
// Reference: prepare_split (indexedTensor_tensor_factorisations.cpp:36-140), SVD::operator() with the
// soft threshold (:142-192), QR / RQ / QC / CQ (:195-264), the ',' tuple (indexedTensorList.cpp:33-53).
// The base is permuted once into (row indices, column indices) order by the indexed-assignment engine
// (one k_strided_eval / permutation pass on the GPU, fixed indices and traces applied there too), the
// matrix factorisation runs on the device (calculate_*), and each factor is permuted into the order in
// which its indices are written.
#include <algorithm>

#include "xerus.h"

namespace xerus {

namespace {

struct Split {
    Tensor base;                        // the base with its modes in (lhs, rhs) order
    size_t splitPos = 0;                // number of row modes
    std::vector<Index> lhsPreliminary;  // the row indices in base order + the new (auxiliary) index
    std::vector<Index> rhsPreliminary;  // the new index + the column indices
};

bool contains(const std::vector<Index>& _v, const Index& _i) { return std::find(_v.begin(), _v.end(), _i) != _v.end(); }

// prepare_split (:36-140): sorts the base's open indices into the two outputs, finds each output's one
// index that is not in the base, and evaluates the base in (lhs, rhs) index order
Split prepare_split(const IndexedProduct& _base, IndexedTensor<Tensor>& _lhs, IndexedTensor<Tensor>& _rhs) {
    // open indices of the base in order of appearance: not fixed and occurring once over all its factors
    // (traces and fixed positions are applied by the evaluation below and leave no mode)
    std::vector<Index> all;
    for (const IndexedTerm& t : _base.terms) {
        const std::vector<Index> r = internal::resolve_indices(t.indices, t.tensor->degree());
        all.insert(all.end(), r.begin(), r.end());
    }
    std::vector<Index> baseIdx;
    for (size_t k = 0; k < all.size(); ++k) {
        if (all[k].fixed()) continue;
        size_t count = 0;
        for (const Index& o : all) count += (o == all[k]);
        if (count == 1) baseIdx.push_back(all[k]);
    }
    size_t lhsOrder = 1, rhsOrder = 1;   // one new mode each
    for (const Index& idx : baseIdx) {
        if (contains(_lhs.indices, idx)) {
            lhsOrder += idx.span;
        } else {
            XERUS_REQUIRE(contains(_rhs.indices, idx), "Every open index of factorisation base must be contained in one of the targets");
            rhsOrder += idx.span;
        }
    }
    Split sp;
    sp.splitPos = lhsOrder - 1;
    const std::vector<Index> lhsIdx = internal::resolve_indices(_lhs.indices, lhsOrder);
    const std::vector<Index> rhsIdx = internal::resolve_indices(_rhs.indices, rhsOrder);

    std::vector<Index> reordered;
    auto collect = [&](const std::vector<Index>& _out, std::vector<Index>& _prelim, const char* _side) {
        bool foundAux = false;
        Index aux;
        for (const Index& idx : _out) {
            size_t j = 0;
            while (j < baseIdx.size() && idx != baseIdx[j]) ++j;
            if (j < baseIdx.size()) {
                _prelim.push_back(baseIdx[j]);
                reordered.push_back(baseIdx[j]);
            } else {
                XERUS_REQUIRE(!foundAux, _side << " part of factorization must have exactly one index that is not contained in base. Here it is more than one.");
                foundAux = true;
                aux = idx;
            }
        }
        XERUS_REQUIRE(foundAux, _side << " part of factorization must have exactly one index that is not contained in base.");
        return aux;
    };
    const Index lhsAux = collect(lhsIdx, sp.lhsPreliminary, "Left");
    sp.lhsPreliminary.push_back(lhsAux);
    const Index rhsAux = collect(rhsIdx, sp.rhsPreliminary, "Right");
    sp.rhsPreliminary.insert(sp.rhsPreliminary.begin(), rhsAux);

    // the permuted base (evaluate(reorderedBaseTensor, base), :126-127)
    Tensor reordered_base;
    reordered_base(reordered) = _base;   // (the whole product contracted, factor and scale carried)
    sp.base = std::move(reordered_base);
    return sp;
}

// U(user order) = U(preliminary order): the "post evaluate" of every factorisation (:179-181)
void post_evaluate(IndexedTensor<Tensor>& _out, Tensor&& _value, const std::vector<Index>& _prelim) {
    const Tensor value = std::move(_value);
    _out = value(_prelim);
}

}  // namespace

void SVD::operator()(const std::vector<IndexedTensor<Tensor>*>& _output) const {
    XERUS_REQUIRE(_output.size() == 3, "SVD requires two output tensors, not " << _output.size());
    XERUS_REQUIRE(epsilon < 1, "Epsilon must be smaller than one.");
    XERUS_REQUIRE(maxRank > 0, "maxRank must be larger than zero.");
    IndexedTensor<Tensor>& U = *_output[0];
    IndexedTensor<Tensor>& S = *_output[1];
    IndexedTensor<Tensor>& Vt = *_output[2];
    Split sp = prepare_split(input, U, Vt);

    Tensor u, s, vt;
    calculate_svd(u, s, vt, std::move(sp.base), sp.splitPos, maxRank, epsilon);

    if (softThreshold > 0.0) {   // (:150-176)
        const size_t oldRank = s.dimensions[0];
        std::vector<value_t> sv(oldRank);
        for (size_t i = 0; i < oldRank; ++i) sv[i] = s[i * oldRank + i];
        size_t rank = oldRank;
        sv[0] = std::max(sv[0] - softThreshold, preventZero ? EPSILON * sv[0] : 0.0);
        for (size_t i = 1; i < oldRank; ++i) {
            if (sv[i] < softThreshold) {
                rank = i;
                break;
            }
            sv[i] -= softThreshold;
        }
        Tensor newS({rank, rank}, Tensor::Representation::Sparse, Tensor::Initialisation::Zero);
        for (size_t i = 0; i < rank; ++i) newS[i * rank + i] = sv[i];
        s = std::move(newS);
        if (rank != oldRank) {
            u.resize_mode(u.degree() - 1, rank);
            vt.resize_mode(0, rank);
        }
    }

    const std::vector<Index> mid{sp.lhsPreliminary.back(), sp.rhsPreliminary.front()};
    post_evaluate(U, std::move(u), sp.lhsPreliminary);
    post_evaluate(S, std::move(s), mid);
    post_evaluate(Vt, std::move(vt), sp.rhsPreliminary);
}

void QR::operator()(const std::vector<IndexedTensor<Tensor>*>& _output) const {
    XERUS_REQUIRE(_output.size() == 2, "QR factorisation requires two output tensors, not " << _output.size());
    IndexedTensor<Tensor>& Q = *_output[0];
    IndexedTensor<Tensor>& R = *_output[1];
    Split sp = prepare_split(input, Q, R);
    Tensor q, r;
    calculate_qr(q, r, std::move(sp.base), sp.splitPos);
    post_evaluate(Q, std::move(q), sp.lhsPreliminary);
    post_evaluate(R, std::move(r), sp.rhsPreliminary);
}

void RQ::operator()(const std::vector<IndexedTensor<Tensor>*>& _output) const {
    XERUS_REQUIRE(_output.size() == 2, "RQ factorisation requires two output tensors, not " << _output.size());
    IndexedTensor<Tensor>& R = *_output[0];
    IndexedTensor<Tensor>& Q = *_output[1];
    Split sp = prepare_split(input, R, Q);
    Tensor r, q;
    calculate_rq(r, q, std::move(sp.base), sp.splitPos);
    post_evaluate(R, std::move(r), sp.lhsPreliminary);
    post_evaluate(Q, std::move(q), sp.rhsPreliminary);
}

void QC::operator()(const std::vector<IndexedTensor<Tensor>*>& _output) const {
    XERUS_REQUIRE(_output.size() == 2, "QC factorisation requires two output tensors, not " << _output.size());
    IndexedTensor<Tensor>& Q = *_output[0];
    IndexedTensor<Tensor>& C = *_output[1];
    Split sp = prepare_split(input, Q, C);
    Tensor q, c;
    calculate_qc(q, c, std::move(sp.base), sp.splitPos);
    post_evaluate(Q, std::move(q), sp.lhsPreliminary);
    post_evaluate(C, std::move(c), sp.rhsPreliminary);
}

void CQ::operator()(const std::vector<IndexedTensor<Tensor>*>& _output) const {
    XERUS_REQUIRE(_output.size() == 2, "CQ factorisation requires two output tensors, not " << _output.size());
    IndexedTensor<Tensor>& C = *_output[0];
    IndexedTensor<Tensor>& Q = *_output[1];
    Split sp = prepare_split(input, C, Q);
    Tensor c, q;
    calculate_cq(c, q, std::move(sp.base), sp.splitPos);
    post_evaluate(C, std::move(c), sp.lhsPreliminary);
    post_evaluate(Q, std::move(q), sp.rhsPreliminary);
}

internal::IndexedTensorList operator,(IndexedTensor<Tensor>&& _first, IndexedTensor<Tensor>&& _second) {
    return internal::IndexedTensorList(std::move(_first), std::move(_second));
}

internal::IndexedTensorList operator,(internal::IndexedTensorList&& _first, IndexedTensor<Tensor>&& _second) {
    _first.tensors.push_back(&_second);
    return std::move(_first);
}

}  // namespace xerus
