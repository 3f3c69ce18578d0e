// Alternating directional fitting (reference include/xerus/algorithms/adf.h:36-268,
// src/xerus/algorithms/adf.cpp:35-611): recovers a low-rank TT from point or rank-one measurements by
// projected-gradient steps on one component at a time, the others kept orthogonal (move_core with keepRank),
// and raises the ranks towards maxRanks when the residual stalls.
//
// MI355X realisation: the measurement stacks (per measurement the contraction of the components left /
// right of the current one with the measurement operator) are M x r matrices in HBM, one per position,
// built by one gather-GEMV kernel launch per component for all measurements at once; residuals, the
// projected gradient (a segmented, fixed-order reduction over the measurements of each slice), the
// slice-wise norms of A(E(grad)) and the component update are kernels too. The host only reads the
// residual norm once per sweep (the termination rule).
#pragma once
#include <vector>

#include "../measurments.h"
#include "../ttNetwork.h"

namespace xerus {

class ADFVariant {
   public:
    size_t maxIterations;                ///< maximal number of sweeps (0: no limit)
    double targetResidualNorm;           ///< stop below this relative residual ||A(x) - b|| / ||b||
    double minimalResidualNormDecrease;  ///< stop (or raise ranks) when the product of the last four residual ratios exceeds its 4th power

    ADFVariant(const size_t _maxIteration, const double _targetResidual, const double _minimalResidualDecrease)
        : maxIterations(_maxIteration), targetResidualNorm(_targetResidual), minimalResidualNormDecrease(_minimalResidualDecrease) {}

    /// recovery at the current ranks of _x (adf.h:240-243); returns the final relative residual
    double operator()(TTTensor& _x, const SinglePointMeasurementSet& _measurments) const;
    double operator()(TTTensor& _x, const RankOneMeasurementSet& _measurments) const;
    /// recovery with rank increases up to _maxRanks (adf.h:253-256)
    double operator()(TTTensor& _x, const SinglePointMeasurementSet& _measurments, const std::vector<size_t>& _maxRanks) const;
    double operator()(TTTensor& _x, const RankOneMeasurementSet& _measurments, const std::vector<size_t>& _maxRanks) const;
};

/// default variant: no sweep limit, target residual 1e-8, minimal decrease 0.999 (adf.cpp:610)
extern const ADFVariant ADF;

}  // namespace xerus
