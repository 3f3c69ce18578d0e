// Device copy of a measurement set for the ADF solver and the TTTensor overloads of measure / test
// (host/measurements.cpp). Internal to the library.
#pragma once
#include <vector>

#include "../adf.hpp"
#include "xerus.h"
#include "xerus/measurments.h"

namespace xerus {
namespace internal {

struct DeviceMeasurements {
    size_t M = 0, d = 0;
    bool single_point = true;
    std::vector<size_t> n;
    // host staging, kept alive for the asynchronous uploads
    std::vector<int> hpos;               // d x M, mode-major (single point)
    std::vector<double> hvec, hvals;     // per mode M x n_k concatenated (rank one); the M values
    std::vector<size_t> voff;            // offset of mode k in hvec
    std::vector<std::vector<int>> hperm, hseg;
    xrs::DevBuf pos, vec, vals;
    // single point, per mode: measurement indices grouped by coordinate (ascending index within a group)
    // and the n_k + 1 group offsets
    std::vector<xrs::DevBuf> perm, seg;

    DeviceMeasurements(const SinglePointMeasurementSet& _set, const std::vector<size_t>& _dims);
    DeviceMeasurements(const RankOneMeasurementSet& _set, const std::vector<size_t>& _dims);
    DeviceMeasurements(const DeviceMeasurements&) = delete;
    DeviceMeasurements& operator=(const DeviceMeasurements&) = delete;

    xrs::adf::Mode mode(size_t _k) const;
    const int* perm_of(size_t _k) const { return single_point ? perm[_k].as<int>() : nullptr; }
    const int* seg_of(size_t _k) const { return single_point ? seg[_k].as<int>() : nullptr; }
    const double* values() const { return vals.d(); }
};

/// x evaluated at every measurement (a forward stack over all components), downloaded to the host
std::vector<value_t> evaluate_tt(const TTTensor& _x, const DeviceMeasurements& _dm);

}  // namespace internal
}  // namespace xerus
