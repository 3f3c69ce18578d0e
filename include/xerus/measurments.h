// Measurement sets for tensor recovery / completion (reference include/xerus/measurments.h:38-151,
// src/xerus/measurments.cpp). Positions and values live on the host, as in the reference; the ADF solver
// and the TTTensor overloads of measure / test upload them once and evaluate on the GPU.
#pragma once
#include <functional>
#include <vector>

#include "tensor.h"

namespace xerus {

class TTTensor;
class TensorNetwork;

/// Point evaluations x[i_0, ..., i_{d-1}] of a tensor.
class SinglePointMeasurementSet {
   public:
    std::vector<std::vector<size_t>> positions;
    std::vector<value_t> measuredValues;

    SinglePointMeasurementSet() = default;

    /// _numMeasurements distinct positions drawn with misc::randomEngine (one uniform_int_distribution per
    /// mode), sorted lexicographically; values 0 (measurments.cpp:41-45, 211-236)
    static SinglePointMeasurementSet random(const size_t _numMeasurements, const std::vector<size_t>& _dimensions);
    static SinglePointMeasurementSet random(const size_t _numMeasurements, const Tensor& _solution);
    static SinglePointMeasurementSet random(const size_t _numMeasurements, const TTTensor& _solution);
    static SinglePointMeasurementSet random(const size_t _numMeasurements, const TensorNetwork& _solution);
    static SinglePointMeasurementSet random(const size_t _numMeasurements, const std::vector<size_t>& _dimensions,
                                            std::function<value_t(const std::vector<size_t>&)> _callback);

    size_t size() const;
    size_t degree() const;
    value_t frob_norm() const;

    void add(std::vector<size_t> _position, const value_t _measuredValue);
    /// lexicographic order of the positions (values permuted along unless _positionsOnly)
    void sort(const bool _positionsOnly = false);

    void measure(const Tensor& _solution);
    /// all positions at once on the GPU (the core-by-core evaluation stack of the ADF solver)
    void measure(const TTTensor& _solution);
    /// entry by entry through TensorNetwork::operator[] (the reference's fixed-mode stack, measurments.cpp:125-173,
    /// computes the same values sharing prefixes)
    void measure(const TensorNetwork& _solution);
    void measure(std::function<value_t(const std::vector<size_t>&)> _callback);

    /// ||values - solution[positions]|| / ||values|| (measurments.cpp:151-199)
    double test(const Tensor& _solution) const;
    double test(const TTTensor& _solution) const;
    double test(const TensorNetwork& _solution) const;
    double test(std::function<value_t(const std::vector<size_t>&)> _callback) const;

   private:
    void create_random_positions(const size_t _numMeasurements, const std::vector<size_t>& _dimensions);
};

/// Rank-one measurements <x, v_0 (x) ... (x) v_{d-1}> (each position is one vector per mode).
class RankOneMeasurementSet {
   public:
    std::vector<std::vector<Tensor>> positions;
    std::vector<value_t> measuredValues;

    RankOneMeasurementSet() = default;
    /// unit vectors e_{i_k} from a single point set (measurments.cpp:244-257)
    RankOneMeasurementSet(const SinglePointMeasurementSet& _other, const std::vector<size_t>& _dimensions);

    /// random N(0,1) vectors per mode (Tensor::random), sorted (measurments.cpp:561-582)
    static RankOneMeasurementSet random(const size_t _numMeasurements, const std::vector<size_t>& _dimensions);
    static RankOneMeasurementSet random(const size_t _numMeasurements, const Tensor& _solution);
    static RankOneMeasurementSet random(const size_t _numMeasurements, const TTTensor& _solution);
    static RankOneMeasurementSet random(const size_t _numMeasurements, const std::vector<size_t>& _dimensions,
                                        std::function<value_t(const std::vector<Tensor>&)> _callback);

    size_t size() const;
    size_t degree() const;
    value_t frob_norm() const;

    void add(const std::vector<Tensor>& _position, const value_t _measuredValue);
    /// order of internal::comp, mode by mode (measurments.cpp:330-347)
    void sort(const bool _positionsOnly = false);
    /// every position vector scaled to unit norm, the value divided by the norms (measurments.cpp:349-358)
    void normalize();

    void measure(const Tensor& _solution);
    void measure(const TTTensor& _solution);
    void measure(std::function<value_t(const std::vector<Tensor>&)> _callback);

    double test(const Tensor& _solution) const;
    double test(const TTTensor& _solution) const;
    double test(std::function<value_t(const std::vector<Tensor>&)> _callback) const;

   private:
    void create_random_positions(const size_t _numMeasurements, const std::vector<size_t>& _dimensions);
};

namespace internal {
/// -1 / 0 / 1 ordering of two equally sized vectors (measurments.cpp:543-607; a larger entry sorts first)
int comp(const Tensor& _a, const Tensor& _b);
}  // namespace internal

}  // namespace xerus
