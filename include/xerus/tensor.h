// xerus::Tensor for the MI355X build: a dense row-major fp64 tensor whose data lives in HBM.
//
// API surface of the reference's Tensor (include/xerus/tensor.h:98-1073). Differences by design:
//   - storage is always dense and device resident (a ref-counted device buffer from the calling
//     thread's xerus_amd handle, copy-on-write like the reference's shared_ptr, tensor.cpp:1158-1216);
//     the Representation argument is accepted and ignored (is_sparse() is always false);
//   - element access through operator[] goes through a host mirror that is synchronised lazily:
//     writes mark the device copy stale and the next device operation uploads once, reads download
//     once while the device copy is unchanged (SURVEY §7 "explicit boundaries");
//   - the lazy scalar `factor` (tensor.h:105) is kept and applied exactly where the reference applies it.
#pragma once

#include <functional>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "basic.h"
#include "misc/random.h"

namespace xerus {

class Index;
template <class T> class IndexedTensor;
class TensorNetwork;

namespace internal {
class Storage;
}

class Tensor {
   public:
    using DimensionTuple = std::vector<size_t>;
    using MultiIndex = std::vector<size_t>;
    enum class Representation { Dense, Sparse };
    enum class Initialisation { Zero, None };

    DimensionTuple dimensions;
    size_t size = 1;
    value_t factor = 1.0;
    Representation representation = Representation::Dense;

    /// Order-0 tensor with value 0 (reference default is a sparse zero scalar).
    explicit Tensor(const Representation _representation = Representation::Sparse);
    Tensor(const Tensor&) = default;
    Tensor(Tensor&&) noexcept = default;
    /// Zero-initialised (or uninitialised) dense tensor of the given dimensions.
    explicit Tensor(DimensionTuple _dimensions, const Representation _representation = Representation::Sparse,
                    const Initialisation _init = Initialisation::Zero);
    /// Takes host data (row-major) and uploads it.
    explicit Tensor(DimensionTuple _dimensions, std::unique_ptr<value_t[]>&& _data);
    explicit Tensor(DimensionTuple _dimensions, const std::function<value_t()>& _f);
    explicit Tensor(DimensionTuple _dimensions, const std::function<value_t(const size_t)>& _f);
    explicit Tensor(DimensionTuple _dimensions, const std::function<value_t(const MultiIndex&)>& _f);

    /// Entries drawn in row-major order from _dist(_rnd) on the host, then uploaded (tensor.h:212-220).
    template <class distribution = std::normal_distribution<value_t>, class generator = std::mt19937_64>
    static Tensor random(DimensionTuple _dimensions, distribution& _dist = misc::defaultNormalDistribution,
                         generator& _rnd = misc::randomEngine) {
        size_t n = 1;
        for (size_t d : _dimensions) n *= d;
        std::unique_ptr<value_t[]> data(new value_t[n]);
        for (size_t i = 0; i < n; ++i) data[i] = _dist(_rnd);
        return Tensor(std::move(_dimensions), std::move(data));
    }
    static Tensor ones(DimensionTuple _dimensions);
    static Tensor identity(DimensionTuple _dimensions);
    static Tensor kronecker(DimensionTuple _dimensions);
    static Tensor dirac(DimensionTuple _dimensions, const MultiIndex& _position);
    static Tensor dirac(DimensionTuple _dimensions, const size_t _position);

    Tensor dense_copy() const { return *this; }

    Tensor& operator=(const Tensor&) = default;
    Tensor& operator=(Tensor&&) = default;
    Tensor& operator=(const TensorNetwork& _network);

    size_t degree() const { return dimensions.size(); }
    bool has_factor() const { return factor != 1.0; }
    bool is_dense() const { return true; }
    bool is_sparse() const { return false; }
    size_t sparsity() const { return size; }
    value_t frob_norm() const;
    value_t one_norm() const;

    Tensor& operator+=(const Tensor& _other);
    Tensor& operator-=(const Tensor& _other);
    Tensor& operator*=(const value_t _factor);
    Tensor& operator/=(const value_t _divisor);

    /// Host access (through the lazily synchronised host mirror; applies the factor first).
    value_t& operator[](const size_t _position);
    value_t operator[](const size_t _position) const;
    value_t& operator[](const MultiIndex& _positions);
    value_t operator[](const MultiIndex& _positions) const;
    value_t& at(const size_t _position) { return (*this)[_position]; }
    value_t cat(const size_t _position) const { return (*this)[_position]; }

    /// Host pointer to the factor-applied data (valid until the next device operation).
    value_t* get_dense_data();
    /// Host copy of the entries with the factor applied.
    std::vector<value_t> to_host() const;

    /// Device pointer to the (factor-free) data, synchronised for reading.
    const value_t* device_data() const;
    /// Device pointer for writing: own data (COW), host mirror invalidated.
    value_t* device_data_for_write();
    /// Device pointer with the factor applied into the data (factor becomes 1).
    value_t* device_data_applied();

    void reset(DimensionTuple _newDim, const Representation _representation, const Initialisation _init = Initialisation::Zero);
    void reset(DimensionTuple _newDim, const Initialisation _init = Initialisation::Zero);
    void reset();
    void reinterpret_dimensions(DimensionTuple _newDimensions);
    void resize_mode(const size_t _mode, const size_t _newDim, size_t _cutPos = ~0ul);
    void fix_mode(const size_t _mode, const size_t _slatePosition);
    void remove_slate(const size_t _mode, const size_t _pos);
    void perform_trace(size_t _firstMode, size_t _secondMode);
    void modify_diagonal_entries(const std::function<void(value_t&)>& _f);
    void modify_diagonal_entries(const std::function<void(value_t&, const size_t)>& _f);
    void modify_entries(const std::function<void(value_t&)>& _f);
    void modify_entries(const std::function<void(value_t&, const size_t)>& _f);
    void offset_add(const Tensor& _other, const std::vector<size_t>& _offsets);
    void use_dense_representation() {}
    void use_dense_representation_if_desirable() {}
    void use_sparse_representation(const value_t = 0) {}
    std::string to_string() const;

    static size_t multiIndex_to_position(const MultiIndex& _multiIndex, const DimensionTuple& _dimensions);
    /// the inverse (row-major, last index fastest): tensor.cpp position_to_multiIndex
    static MultiIndex position_to_multiIndex(size_t _position, const DimensionTuple& _dimensions);

    void ensure_own_data();
    void apply_factor();

    // indexed expressions: A(i,j) = B(i,k)*C(k,j)
    IndexedTensor<Tensor> operator()(const std::vector<Index>& _indices);
    IndexedTensor<Tensor> operator()(std::vector<Index>&& _indices);
    template <typename... args>
    IndexedTensor<Tensor> operator()(args... _args);
    IndexedTensor<Tensor> operator()(const std::vector<Index>& _indices) const;
    template <typename... args>
    IndexedTensor<Tensor> operator()(args... _args) const;

    // internal: shares storage identity for aliasing checks
    const internal::Storage* storage_id() const { return store.get(); }
    /// Adopt a device buffer allocated from the thread's pool (takes ownership).
    static Tensor adopt_device(DimensionTuple _dimensions, value_t* _dev);
    /// Give up ownership of the device buffer (factor applied first); the tensor becomes empty.
    value_t* release_device();

   private:
    std::shared_ptr<internal::Storage> store;
    friend class internal::Storage;
};

// ---- free functions (tensor.h:56-66, 869-1000)
void contract(Tensor& _result, const Tensor& _lhs, const bool _lhsTrans, const Tensor& _rhs, const bool _rhsTrans,
              const size_t _numModes);
Tensor contract(const Tensor& _lhs, const bool _lhsTrans, const Tensor& _rhs, const bool _rhsTrans, const size_t _numModes);
inline void contract(Tensor& _result, const Tensor& _lhs, const Tensor& _rhs, const size_t _numModes) {
    contract(_result, _lhs, false, _rhs, false, _numModes);
}
inline Tensor contract(const Tensor& _lhs, const Tensor& _rhs, const size_t _numModes) {
    return contract(_lhs, false, _rhs, false, _numModes);
}
void reshuffle(Tensor& _out, const Tensor& _base, const std::vector<size_t>& _shuffle);
Tensor reshuffle(const Tensor& _base, const std::vector<size_t>& _shuffle);

Tensor operator+(Tensor _lhs, const Tensor& _rhs);
Tensor operator-(Tensor _lhs, const Tensor& _rhs);
Tensor operator*(const value_t _factor, Tensor _tensor);
Tensor operator*(Tensor _tensor, const value_t _factor);
Tensor operator/(Tensor _tensor, const value_t _divisor);
/// entrywise (Hadamard) product of equal-dimension tensors (tensor.cpp:1708-1740), one device kernel
Tensor entrywise_product(const Tensor& _A, const Tensor& _B);

inline value_t frob_norm(const Tensor& _tensor) { return _tensor.frob_norm(); }

/// A X = B with the first B.degree() - extraDegree modes of A contracted against B (tensor.cpp:1654-1704);
/// dispatch of blasWrapper::solve (blasLapackWrapper.cpp:540-640)
void solve(Tensor& _X, const Tensor& _A, const Tensor& _B, const size_t _extraDegree = 0);
/// minimum-norm least-squares solution (tensor.cpp:1583-1651, dgelsd semantics)
void solve_least_squares(Tensor& _X, const Tensor& _A, const Tensor& _B, const size_t _extraDegree = 0);
void calculate_svd(Tensor& _U, Tensor& _S, Tensor& _Vt, Tensor _input, const size_t _splitPos, const size_t _maxRank,
                   const value_t _eps);
void calculate_qr(Tensor& _Q, Tensor& _R, Tensor _input, const size_t _splitPos);
void calculate_rq(Tensor& _R, Tensor& _Q, Tensor _input, const size_t _splitPos);
void calculate_qc(Tensor& _Q, Tensor& _C, Tensor _input, const size_t _splitPos);
void calculate_cq(Tensor& _C, Tensor& _Q, Tensor _input, const size_t _splitPos);
void pseudo_inverse(Tensor& _inverse, const Tensor& _input, const size_t _splitPos);
Tensor pseudo_inverse(const Tensor& _input, const size_t _splitPos);

/// ||a-b||_F <= eps*(||a||_F+||b||_F)/2 (tensor.cpp:1738-1743)
bool approx_equal(const Tensor& _a, const Tensor& _b, const value_t _eps = EPSILON);
bool approx_entrywise_equal(const Tensor& _a, const Tensor& _b, const value_t _eps = EPSILON);
bool approx_entrywise_equal(const Tensor& _tensor, const std::vector<value_t>& _values, const value_t _eps = EPSILON);

std::ostream& operator<<(std::ostream& _out, const Tensor& _tensor);

namespace misc {
enum class FileFormat { BINARY, TSV };
}  // namespace misc

}  // namespace xerus

#include "indexedTensor.h"

namespace xerus {
template <typename... args>
IndexedTensor<Tensor> Tensor::operator()(args... _args) {
    return (*this)(std::vector<Index>({Index(_args)...}));
}
template <typename... args>
IndexedTensor<Tensor> Tensor::operator()(args... _args) const {
    return (*this)(std::vector<Index>({Index(_args)...}));
}
}  // namespace xerus
