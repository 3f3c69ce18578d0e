// Indexed expressions on Tensors: A(i,j) = B(i,k,l)*C(k,j,l), A(i^2) = B(i^2) + C(i^2), A() = B(i&0)*C(i&0)...
//
// Same semantics as the reference's IndexedTensor* family (indexedTensorReadOnly.cpp:81-324,
// indexedTensorWritable.cpp:68-119): indices are resolved per tensor (spans, fixed positions), an index
// appearing twice within one tensor is a trace, twice across tensors a contraction, once an open mode.
// A product is lowered to a TensorNetwork, contracted pairwise in a greedy order (the reference's
// contraction heuristics) with each pairwise step = at most one permutation + one GEMM on the GPU, and
// finally permuted into the order of the left-hand side.
#pragma once
#include <memory>
#include <vector>

#include "index.h"

namespace xerus {

class Tensor;

/// One factor of a product: a (shared, copy-on-write) tensor with its indices.
struct IndexedTerm {
    std::shared_ptr<const Tensor> tensor;
    std::vector<Index> indices;
};

class IndexedProduct {
   public:
    std::vector<IndexedTerm> terms;
    value_t scale = 1.0;
    /// evaluates a full contraction (no open index) to a scalar
    operator value_t() const;
    /// open indices of the product in order of first appearance (after span resolution)
};

class IndexedSum {
   public:
    std::vector<IndexedProduct> summands;
};

template <class T>
class IndexedTensor;

template <>
class IndexedTensor<Tensor> {
   public:
    Tensor* tensorObject;
    std::vector<Index> indices;
    bool writable;

    IndexedTensor(Tensor* _t, std::vector<Index> _indices, bool _writable)
        : tensorObject(_t), indices(std::move(_indices)), writable(_writable) {}
    IndexedTensor(const IndexedTensor&) = default;

    IndexedTensor& operator=(const IndexedTensor<Tensor>& _rhs);   // permutation / trace / slice
    IndexedTensor& operator=(const IndexedProduct& _rhs);
    IndexedTensor& operator=(const IndexedSum& _rhs);
    IndexedTensor& operator+=(const IndexedProduct& _rhs);
    IndexedTensor& operator-=(const IndexedProduct& _rhs);
    IndexedTensor& operator+=(const IndexedTensor<Tensor>& _rhs);
    IndexedTensor& operator-=(const IndexedTensor<Tensor>& _rhs);
    /// python-binding style assignment (reference python/indexedTensor.cpp: __lshift__)
    IndexedTensor& operator<<(const IndexedProduct& _rhs) { return *this = _rhs; }
    IndexedTensor& operator<<(const IndexedSum& _rhs) { return *this = _rhs; }
    IndexedTensor& operator<<(const IndexedTensor<Tensor>& _rhs) { return *this = _rhs; }

    IndexedProduct as_product() const;
    operator value_t() const;
};

IndexedProduct operator*(const IndexedTensor<Tensor>& _a, const IndexedTensor<Tensor>& _b);
IndexedProduct operator*(IndexedProduct _a, const IndexedTensor<Tensor>& _b);
IndexedProduct operator*(const IndexedTensor<Tensor>& _a, IndexedProduct _b);
IndexedProduct operator*(IndexedProduct _a, const IndexedProduct& _b);
IndexedProduct operator*(const value_t _f, const IndexedTensor<Tensor>& _a);
IndexedProduct operator*(const IndexedTensor<Tensor>& _a, const value_t _f);
IndexedProduct operator*(const value_t _f, IndexedProduct _a);
IndexedProduct operator*(IndexedProduct _a, const value_t _f);
IndexedProduct operator/(const IndexedTensor<Tensor>& _a, const value_t _f);
/// x(i...) = b(j...) / A(j..., i...): the (least-squares) solution of A x = b (indexedTensor_tensor_solve.cpp:31-75)
IndexedProduct operator/(const IndexedTensor<Tensor>& _b, const IndexedTensor<Tensor>& _A);
IndexedProduct operator/(IndexedProduct _a, const value_t _f);
IndexedProduct operator-(const IndexedTensor<Tensor>& _a);
IndexedProduct operator-(IndexedProduct _a);

IndexedSum operator+(const IndexedProduct& _a, const IndexedProduct& _b);
IndexedSum operator-(const IndexedProduct& _a, const IndexedProduct& _b);
IndexedSum operator+(IndexedSum _a, const IndexedProduct& _b);
IndexedSum operator-(IndexedSum _a, const IndexedProduct& _b);
IndexedSum operator+(const IndexedTensor<Tensor>& _a, const IndexedTensor<Tensor>& _b);
IndexedSum operator-(const IndexedTensor<Tensor>& _a, const IndexedTensor<Tensor>& _b);
IndexedSum operator+(const IndexedTensor<Tensor>& _a, const IndexedProduct& _b);
IndexedSum operator-(const IndexedTensor<Tensor>& _a, const IndexedProduct& _b);
IndexedSum operator+(const IndexedProduct& _a, const IndexedTensor<Tensor>& _b);
IndexedSum operator-(const IndexedProduct& _a, const IndexedTensor<Tensor>& _b);
IndexedSum operator+(IndexedSum _a, const IndexedTensor<Tensor>& _b);
IndexedSum operator-(IndexedSum _a, const IndexedTensor<Tensor>& _b);

value_t frob_norm(const IndexedTensor<Tensor>& _idxTensor);

namespace internal {
/// Evaluates a product into a tensor whose modes follow `_out` (LHS indices; resolved against the
/// product's open degree). Used by the assignment operators.
Tensor evaluate_product(const IndexedProduct& _p, const std::vector<Index>& _out);
/// spans resolved against a tensor of the given degree (index.cpp:64-92), span-0 indices dropped
std::vector<Index> resolve_indices(const std::vector<Index>& _indices, size_t _degree);
}  // namespace internal

}  // namespace xerus
