// TTTensor (= TTNetwork<false>) for the MI355X build: the cores stay in HBM; move_core, round,
// frob_norm and <x,y> run on the GPU (xerus_amd TT drivers).
// API surface of the reference's TTNetwork (include/xerus/ttNetwork.h:46-519, src/xerus/ttNetwork.cpp).
#pragma once
#include <vector>

#include "tensor.h"
#include "tensorNetwork.h"

namespace xerus {

class TTTensor;
template <>
class IndexedTensor<TTTensor>;

class TTTensor {
   public:
    /// component k has dims (r_k, n_k, r_{k+1}), r_0 = r_d = 1 (ttNetwork.cpp:57-108)
    std::vector<Tensor> components;
    std::vector<size_t> dimensions;
    bool canonicalized = false;
    size_t corePosition = 0;

    TTTensor();
    /// all-zero TT of rank 1 (ttNetwork.cpp:57-108)
    explicit TTTensor(const Tensor::DimensionTuple& _dimensions);
    explicit TTTensor(size_t _degree);
    /// TT-SVD of a dense tensor (ttNetwork.cpp:111-160)
    explicit TTTensor(const Tensor& _tensor, const double _eps = EPSILON,
                      const size_t _maxRank = std::numeric_limits<size_t>::max());
    TTTensor(const Tensor& _tensor, const double _eps, const std::vector<size_t>& _maxRanks);

    /// raw N(0,1) cores of the capped ranks (reduce_to_maximal_ranks), then move_core(0) (ttNetwork.h:129-157)
    template <class distribution = std::normal_distribution<value_t>, class generator = std::mt19937_64>
    static TTTensor random(std::vector<size_t> _dimensions, const std::vector<size_t>& _ranks,
                           distribution& _dist = misc::defaultNormalDistribution, generator& _rnd = misc::randomEngine) {
        TTTensor result = random_raw(_dimensions, _ranks, _dist, _rnd);
        result.move_core(0);
        return result;
    }
    template <class distribution = std::normal_distribution<value_t>, class generator = std::mt19937_64>
    static TTTensor random(std::vector<size_t> _dimensions, const size_t _rank,
                           distribution& _dist = misc::defaultNormalDistribution, generator& _rnd = misc::randomEngine) {
        return random(_dimensions, std::vector<size_t>(_dimensions.empty() ? 0 : _dimensions.size() - 1, _rank), _dist, _rnd);
    }
    template <class distribution = std::normal_distribution<value_t>, class generator = std::mt19937_64>
    static TTTensor random_raw(std::vector<size_t> _dimensions, const std::vector<size_t>& _ranks,
                               distribution& _dist = misc::defaultNormalDistribution, generator& _rnd = misc::randomEngine) {
        XERUS_REQUIRE(_ranks.size() + 1 == _dimensions.size(), "Non-matching amount of ranks given to TTNetwork::random.");
        const std::vector<size_t> target = reduce_to_maximal_ranks(_ranks, _dimensions);
        TTTensor result(_dimensions.size());
        result.dimensions = _dimensions;
        const size_t d = _dimensions.size();
        for (size_t i = 0; i < d; ++i) {
            const size_t l = (i == 0) ? 1 : target[i - 1];
            const size_t r = (i + 1 == d) ? 1 : target[i];
            result.components[i] = Tensor::random({l, _dimensions[i], r}, _dist, _rnd);
        }
        result.canonicalized = false;
        return result;
    }
    static std::vector<size_t> reduce_to_maximal_ranks(std::vector<size_t> _ranks, const std::vector<size_t>& _dimensions);
    /// all-ones rank-1 TT, then canonicalize_left (ttNetwork.cpp:170-191)
    static TTTensor ones(const std::vector<size_t>& _dimensions);
    /// the Kronecker delta (1 where all indices are equal): cores are delta tensors of rank min(dims), then
    /// canonicalize_left (ttNetwork.cpp:224-254)
    static TTTensor kronecker(const std::vector<size_t>& _dimensions);
    /// rank-1 unit tensor at _position (ttNetwork.cpp:257-283); not canonical for d >= 2
    static TTTensor dirac(std::vector<size_t> _dimensions, const std::vector<size_t>& _position);
    static TTTensor dirac(std::vector<size_t> _dimensions, const size_t _position);

    size_t degree() const { return dimensions.size(); }
    std::vector<size_t> ranks() const;
    size_t rank(const size_t _i) const;
    const Tensor& get_component(const size_t _idx) const { return components.at(_idx); }
    Tensor& component(const size_t _idx);
    void set_component(const size_t _idx, Tensor _T);
    bool exceeds_maximal_ranks() const;

    void move_core(const size_t _position, const bool _keepRank = false);
    void canonicalize_left() { move_core(0); }
    void canonicalize_right() { move_core(degree() == 0 ? 0 : degree() - 1); }
    void assume_core_position(const size_t _pos);

    void round(const std::vector<size_t>& _maxRanks, const double _eps = EPSILON);
    void round(const size_t _maxRank);
    void round(const int _maxRank);
    void round(const value_t _eps);
    /// TTNetwork::soft_threshold (ttNetwork.cpp:688-713): per edge sigma -> max(0, sigma - tau);
    /// _taus[0] applies to the last edge, as in the reference; _preventZero is unused there too
    void soft_threshold(const std::vector<double>& _taus, const bool _preventZero = false);
    void soft_threshold(const double _tau, const bool _preventZero = false);

    value_t frob_norm() const;

    /// fixes mode _mode to _slatePosition: the sliced core (a matrix) is contracted into its right
    /// neighbour (the left one for the last mode), as TensorNetwork::fix_mode + contract_unconnected_subnetworks
    /// (ttNetwork.cpp:432-435, 748-778, tensorNetwork.cpp:912-951)
    void fix_mode(const size_t _mode, const size_t _slatePosition);
    /// Tensor::resize_mode on the core holding _mode, then the reference's re-canonicalisation
    /// (ttNetwork.cpp:438-446)
    void resize_mode(const size_t _mode, const size_t _newDim, const size_t _cutPos = ~0ul);
    /// the networks left and right of component _position, each with the cut rank as an extra external
    /// index (last on the left, first on the right), ghost nodes as the reference's (ttNetwork.cpp:515-580)
    std::pair<TensorNetwork, TensorNetwork> chop(const size_t _position) const;

    TTTensor& operator+=(const TTTensor& _other);
    TTTensor& operator-=(const TTTensor& _other);
    TTTensor& operator*=(const value_t _factor);
    TTTensor& operator/=(const value_t _divisor);

    /// full contraction to a dense tensor
    operator Tensor() const;
    Tensor to_tensor() const;

    IndexedTensor<TTTensor> operator()(const std::vector<Index>& _indices) const;
    template <typename... args>
    IndexedTensor<TTTensor> operator()(args... _args) const;
    IndexedTensor<TTTensor> operator()(const std::vector<Index>& _indices);
    template <typename... args>
    IndexedTensor<TTTensor> operator()(args... _args);

    void require_correct_format() const;
};

TTTensor operator+(TTTensor _lhs, const TTTensor& _rhs);
TTTensor operator-(TTTensor _lhs, const TTTensor& _rhs);
TTTensor operator*(const value_t _factor, TTTensor _tt);
TTTensor operator*(TTTensor _tt, const value_t _factor);
TTTensor operator/(TTTensor _tt, const value_t _divisor);
inline value_t frob_norm(const TTTensor& _tt) { return _tt.frob_norm(); }
/// <x, y> on the GPU (left-to-right zipper, no permutations)
value_t dot(const TTTensor& _x, const TTTensor& _y);
bool approx_equal(const TTTensor& _a, const TTTensor& _b, const value_t _eps = EPSILON);
/// entrywise (Hadamard) product, rank r_A r_B (ttNetwork.cpp:1275-1309): one HBM-bound kernel per core
/// (xrs_tt_entrywise_product); moved to A's core position when both inputs are canonical
TTTensor entrywise_product(const TTTensor& _A, const TTTensor& _B);
/// the tensor product of two TTs: components of _lhs, then of _rhs (ttNetwork.cpp:1319-1429)
TTTensor dyadic_product(const TTTensor& _lhs, const TTTensor& _rhs);
/// repeated dyadic_product, right to left (ttNetwork.cpp:1435-1445)
TTTensor dyadic_product(const std::vector<TTTensor>& _tensors);

/// Indexed TT, supporting the full contraction value_t(x(i&0) * y(i&0)) of the reference.
template <>
class IndexedTensor<TTTensor> {
   public:
    const TTTensor* tt;
    TTTensor* mut = nullptr;   // set when indexed through a non-const TTTensor (assignment target)
    std::vector<Index> indices;
    /// y(i&0) = A(i/2, j/2) * x(j&0) (and the transposed x^T A form), ttNetwork.cpp:1075-1093
    IndexedTensor& operator=(const class IndexedTTStack& _stack);
};

class IndexedTTProduct {
   public:
    const TTTensor* x;
    const TTTensor* y;
    std::vector<Index> ix, iy;
    value_t scale = 1.0;
    operator value_t() const;
};
IndexedTTProduct operator*(const IndexedTensor<TTTensor>& _a, const IndexedTensor<TTTensor>& _b);

template <typename... args>
IndexedTensor<TTTensor> TTTensor::operator()(args... _args) const {
    return (*this)(std::vector<Index>({Index(_args)...}));
}
template <typename... args>
IndexedTensor<TTTensor> TTTensor::operator()(args... _args) {
    return (*this)(std::vector<Index>({Index(_args)...}));
}

using TTNetwork = TTTensor;

// ------------------------------------------------------------------------------------------ TTOperator
class TTOperator;
template <>
class IndexedTensor<TTOperator>;

/// TTOperator (= TTNetwork<true>, ttNetwork.h:46-519 with N = 2): component k has dims
/// (r_k, n_k, m_k, r_{k+1}); dimensions = (n_0..n_{d-1}, m_0..m_{d-1}). Storage-wise a TTOperator is the
/// TTTensor with modes n_k m_k (the same row-major cores), so canonicalisation, rounding, sums and norms
/// run through the TT drivers on that view; application to a TTTensor / TTOperator is the TTStack
/// contraction (xrs_tt_operator_apply).
class TTOperator {
   public:
    std::vector<Tensor> components;
    std::vector<size_t> dimensions;
    bool canonicalized = true;
    size_t corePosition = 0;

    TTOperator();
    /// all-zero operator of rank 1 (ttNetwork.cpp:57-108)
    explicit TTOperator(const Tensor::DimensionTuple& _dimensions);
    explicit TTOperator(size_t _degree);
    /// TT-SVD of a dense operator tensor (i_0..i_{d-1}, j_0..j_{d-1}) (ttNetwork.cpp:111-160, N = 2)
    explicit TTOperator(const Tensor& _tensor, const double _eps = EPSILON,
                        const size_t _maxRank = std::numeric_limits<size_t>::max());
    TTOperator(const Tensor& _tensor, const double _eps, const std::vector<size_t>& _maxRanks);

    template <class distribution = std::normal_distribution<value_t>, class generator = std::mt19937_64>
    static TTOperator random(std::vector<size_t> _dimensions, const std::vector<size_t>& _ranks,
                             distribution& _dist = misc::defaultNormalDistribution, generator& _rnd = misc::randomEngine) {
        TTOperator result = from_tt(TTTensor::random(merged_dimensions(_dimensions), _ranks, _dist, _rnd), _dimensions);
        return result;
    }
    template <class distribution = std::normal_distribution<value_t>, class generator = std::mt19937_64>
    static TTOperator random(std::vector<size_t> _dimensions, const size_t _rank,
                             distribution& _dist = misc::defaultNormalDistribution, generator& _rnd = misc::randomEngine) {
        return random(_dimensions, std::vector<size_t>(_dimensions.size() < 2 ? 0 : _dimensions.size() / 2 - 1, _rank), _dist, _rnd);
    }
    /// identity operator, cores delta(i, j), then canonicalize_left (ttNetwork.cpp:194-221)
    static TTOperator identity(const std::vector<size_t>& _dimensions);
    /// all-ones operator (ttNetwork.cpp:169-191)
    static TTOperator ones(const std::vector<size_t>& _dimensions);
    /// Kronecker delta over all 2d indices (ttNetwork.cpp:224-254)
    static TTOperator kronecker(const std::vector<size_t>& _dimensions);
    /// rank-1 unit operator (ttNetwork.cpp:257-283)
    static TTOperator dirac(std::vector<size_t> _dimensions, const std::vector<size_t>& _position);
    static TTOperator dirac(std::vector<size_t> _dimensions, const size_t _position);

    size_t degree() const { return dimensions.size(); }
    std::vector<size_t> ranks() const;
    size_t rank(const size_t _i) const;
    const Tensor& get_component(const size_t _idx) const { return components.at(_idx); }
    Tensor& component(const size_t _idx);
    void set_component(const size_t _idx, Tensor _T);

    void move_core(const size_t _position, const bool _keepRank = false);
    void canonicalize_left() { move_core(0); }
    void canonicalize_right() { move_core(degree() < 2 ? 0 : degree() / 2 - 1); }
    void assume_core_position(const size_t _pos);
    void round(const std::vector<size_t>& _maxRanks, const double _eps = EPSILON);
    void round(const size_t _maxRank);
    void round(const int _maxRank);
    void round(const value_t _eps);
    value_t frob_norm() const;
    /// swaps row and column modes (ttNetwork.h:443-448)
    void transpose();
    /// not available for operators (ttNetwork.cpp:433: REQUIRE)
    void fix_mode(const size_t _mode, const size_t _slatePosition);
    /// row modes 0..d-1, column modes d..2d-1 (ttNetwork.cpp:438-446)
    void resize_mode(const size_t _mode, const size_t _newDim, const size_t _cutPos = ~0ul);
    /// left / right networks of component _position (externals: row modes, column modes, then the cut rank
    /// on the left; the cut rank, row modes, column modes on the right; ttNetwork.cpp:515-580)
    std::pair<TensorNetwork, TensorNetwork> chop(const size_t _position) const;

    TTOperator& operator+=(const TTOperator& _other);
    TTOperator& operator-=(const TTOperator& _other);
    TTOperator& operator*=(const value_t _factor);
    TTOperator& operator/=(const value_t _divisor);

    operator Tensor() const;
    Tensor to_tensor() const;

    IndexedTensor<TTOperator> operator()(const std::vector<Index>& _indices) const;
    IndexedTensor<TTOperator> operator()(const std::vector<Index>& _indices);
    template <typename... args>
    IndexedTensor<TTOperator> operator()(args... _args) const;
    template <typename... args>
    IndexedTensor<TTOperator> operator()(args... _args);

    void require_correct_format() const;

    // the TTTensor view (modes n_k m_k) and back
    static std::vector<size_t> merged_dimensions(const std::vector<size_t>& _dimensions);
    TTTensor to_tt() &&;
    static TTOperator from_tt(TTTensor&& _tt, const std::vector<size_t>& _dimensions);
};

TTOperator operator+(TTOperator _lhs, const TTOperator& _rhs);
TTOperator operator-(TTOperator _lhs, const TTOperator& _rhs);
TTOperator operator*(const value_t _factor, TTOperator _op);
TTOperator operator*(TTOperator _op, const value_t _factor);
TTOperator operator/(TTOperator _op, const value_t _divisor);
inline value_t frob_norm(const TTOperator& _op) { return _op.frob_norm(); }
TTOperator entrywise_product(const TTOperator& _A, const TTOperator& _B);
TTOperator dyadic_product(const TTOperator& _lhs, const TTOperator& _rhs);
TTOperator dyadic_product(const std::vector<TTOperator>& _tensors);

template <>
class IndexedTensor<TTOperator> {
   public:
    const TTOperator* op;
    TTOperator* mut = nullptr;
    std::vector<Index> indices;
    /// C(i/2, k/2) = A(i/2, j/2) * B(j/2, k/2)
    IndexedTensor& operator=(const class IndexedTTStack& _stack);
};

/// A lazily contracted operator application (reference: TTStack, ttStack.h / ttStack.cpp): A x,
/// x^T A (x(i&0) * A(i/2, j/2)) or A B. Evaluated on assignment, or as a scalar against a TTTensor.
class IndexedTTStack {
   public:
    const TTOperator* op = nullptr;
    const TTTensor* vec = nullptr;        // A x / x^T A
    const TTOperator* rhsOp = nullptr;    // A B
    bool transposed = false;              // x^T A
    std::vector<Index> indices;           // the free indices of the result
    /// the contracted TTStack (TTTensor result), canonicalised at the operator's core (ttStack.cpp:160-168)
    TTTensor evaluate_tt() const;
    TTOperator evaluate_op() const;
};
IndexedTTStack operator*(const IndexedTensor<TTOperator>& _a, const IndexedTensor<TTTensor>& _x);
IndexedTTStack operator*(const IndexedTensor<TTTensor>& _x, const IndexedTensor<TTOperator>& _a);
IndexedTTStack operator*(const IndexedTensor<TTOperator>& _a, const IndexedTensor<TTOperator>& _b);
/// value_t(x(i&0) * A(i/2, j/2) * y(j&0)) and value_t(A(i/2, j/2) * x(j&0) * y(i&0))
value_t operator*(const IndexedTTStack& _s, const IndexedTensor<TTTensor>& _y);

template <typename... args>
IndexedTensor<TTOperator> TTOperator::operator()(args... _args) const {
    return (*this)(std::vector<Index>({Index(_args)...}));
}
template <typename... args>
IndexedTensor<TTOperator> TTOperator::operator()(args... _args) {
    return (*this)(std::vector<Index>({Index(_args)...}));
}

}  // namespace xerus
