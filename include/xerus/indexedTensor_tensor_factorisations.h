// Indexed factorisation expressions (reference include/xerus/indexedTensor_tensor_factorisations.h:40-131,
// src/xerus/indexedTensor_tensor_factorisations.cpp:36-266, include/xerus/indexedTensorList.h:36-80):
//
//     (U(i,r1), S(r1,r2), Vt(r2,j)) = SVD(A(i,j));            (Q(i,k), R(k,j)) = QR(A(i,j));
//     (U(i,j,r1), S(r1,r2), Vt(r2,k)) = SVD(A(j,k,i), maxRank, eps);   ... = SVD(A(i,j), softThreshold);
//
// The open indices of the base that appear on the left output span its rows, those on the right output
// its columns; each output has exactly one index not in the base (the new rank mode). The base is
// permuted once into (left indices, right indices) order on the GPU (prepare_split), factorised by
// calculate_svd / _qr / _rq / _qc / _cq (device kernels), and each result is permuted into the order its
// indices are written in.
#pragma once
#include <limits>
#include <vector>

#include "indexedTensor.h"

namespace xerus {

class TensorFactorisation {
   public:
    virtual void operator()(const std::vector<IndexedTensor<Tensor>*>& _output) const = 0;
    virtual ~TensorFactorisation() = default;

   protected:
    // the base: an indexed tensor or any indexed product (e.g. SVD(-1 * A(i,j)), the reference's
    // IndexedTensorReadOnly covers both); its open indices are the ones occurring once
    static IndexedProduct base(const IndexedTensor<Tensor>& _in) { return _in.as_product(); }
    static IndexedProduct base(const IndexedProduct& _in) { return _in; }
};

/// (U, S, Vt) = SVD(A): rank cut at maxRank, then at the first sigma_j <= epsilon sigma_0
/// (calculate_svd); softThreshold > 0 subtracts it from every singular value and drops those below it
/// (indexedTensor_tensor_factorisations.cpp:150-176; sigma_0 is kept, at least EPSILON sigma_0 with
/// preventZero).
class SVD : public TensorFactorisation {
   public:
    IndexedProduct input;
    const double epsilon;
    const double softThreshold;
    const size_t maxRank;
    const bool preventZero;

    template <class In>
    SVD(const In& _input)
        : input(base(_input)), epsilon(EPSILON), softThreshold(0.0), maxRank(std::numeric_limits<size_t>::max()), preventZero(false) {}
    template <class In>
    SVD(const In& _input, const double _softThreshold, const bool _preventZero = false)
        : input(base(_input)), epsilon(0.0), softThreshold(_softThreshold), maxRank(std::numeric_limits<size_t>::max()),
          preventZero(_preventZero) {}
    template <class In>
    SVD(const In& _input, const size_t _maxRank, const double _epsilon = EPSILON)
        : input(base(_input)), epsilon(_epsilon), softThreshold(0.0), maxRank(_maxRank), preventZero(false) {}
    template <class In>
    SVD(const In& _input, const size_t _maxRank, const double _epsilon, const double _softThreshold, const bool _preventZero)
        : input(base(_input)), epsilon(_epsilon), softThreshold(_softThreshold), maxRank(_maxRank), preventZero(_preventZero) {}

    void operator()(const std::vector<IndexedTensor<Tensor>*>& _output) const override;
};

/// (Q, R) = QR(A): unpivoted QR (calculate_qr)
class QR : public TensorFactorisation {
   public:
    IndexedProduct input;
    template <class In>
    QR(const In& _input) : input(base(_input)) {}
    void operator()(const std::vector<IndexedTensor<Tensor>*>& _output) const override;
};

/// (R, Q) = RQ(A) (calculate_rq)
class RQ : public TensorFactorisation {
   public:
    IndexedProduct input;
    template <class In>
    RQ(const In& _input) : input(base(_input)) {}
    void operator()(const std::vector<IndexedTensor<Tensor>*>& _output) const override;
};

/// (Q, C) = QC(A): rank-revealing (pivoted QR rank rule, calculate_qc)
class QC : public TensorFactorisation {
   public:
    IndexedProduct input;
    template <class In>
    QC(const In& _input) : input(base(_input)) {}
    void operator()(const std::vector<IndexedTensor<Tensor>*>& _output) const override;
};

/// (C, Q) = CQ(A) (calculate_cq)
class CQ : public TensorFactorisation {
   public:
    IndexedProduct input;
    template <class In>
    CQ(const In& _input) : input(base(_input)) {}
    void operator()(const std::vector<IndexedTensor<Tensor>*>& _output) const override;
};

namespace internal {
/// A tuple of writable indexed tensors, the target of a factorisation (indexedTensorList.h:40-63). It
/// points at the temporaries of the full expression `(U(i,r), S(r,s), Vt(s,j)) = SVD(...)`.
class IndexedTensorList {
   public:
    std::vector<IndexedTensor<Tensor>*> tensors;
    IndexedTensorList() = delete;
    IndexedTensorList(const IndexedTensorList&) = delete;
    IndexedTensorList(IndexedTensorList&& _old) noexcept = default;
    IndexedTensorList(IndexedTensor<Tensor>&& _first, IndexedTensor<Tensor>&& _second) : tensors{&_first, &_second} {}
    void operator=(TensorFactorisation&& _factorisation) const { _factorisation(tensors); }
};
}  // namespace internal

internal::IndexedTensorList operator,(IndexedTensor<Tensor>&& _first, IndexedTensor<Tensor>&& _second);
internal::IndexedTensorList operator,(internal::IndexedTensorList&& _first, IndexedTensor<Tensor>&& _second);

}  // namespace xerus
