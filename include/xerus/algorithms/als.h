// Alternating least squares on TT tensors (reference include/xerus/algorithms/als.h:37-226,
// src/xerus/algorithms/als.cpp:35-565): solves A x = b (or minimises ||A x - b|| / ||x - b||) by
// optimising one component at a time while the others are kept orthogonal (move_core with keepRank).
//
// Local systems are built from the cached left/right environments as dense tensors in HBM (each
// environment update is one indexed product: permutations + MFMA GEMMs) and solved on the GPU
// (xerus::solve: blocked Cholesky for the symmetric positive definite local operators of every variant).
#pragma once
#include <functional>
#include <utility>
#include <vector>

#include "../ttNetwork.h"

namespace xerus {

class ALSVariant {
   public:
    enum Direction { Increasing, Decreasing };

    /// state of one ALS run (als.h:44-84)
    struct ALSAlgorithmicData {
        const ALSVariant& ALS;
        const TTOperator* A;
        TTTensor& x;
        const TTTensor& b;
        std::vector<size_t> targetRank;
        std::vector<Tensor> opLeft, opRight;     ///< environments of the local operator (x A x, or x A^T A x)
        std::vector<Tensor> rhsLeft, rhsRight;   ///< environments of the right-hand side (b x, or b A x)
        value_t normB;
        std::pair<size_t, size_t> optimizedRange;
        bool canonicalizeAtTheEnd;
        size_t corePosAtTheEnd;
        size_t currIndex = 0;
        value_t lastEnergy2 = 1e102, lastEnergy = 1e101, energy = 1e100;
        size_t halfSweepCount = 0;
        Direction direction = Increasing;

        ALSAlgorithmicData(const ALSVariant& _ALS, const TTOperator* _A, TTTensor& _x, const TTTensor& _b);
        void prepare_x_for_als();
        void prepare_stacks();
        void move_to_next_index();
        Tensor op_step_left(const Tensor& _env, size_t _pos) const;
        Tensor op_step_right(const Tensor& _env, size_t _pos) const;
        Tensor rhs_step_left(const Tensor& _env, size_t _pos) const;
        Tensor rhs_step_right(const Tensor& _env, size_t _pos) const;
        value_t energy_f() const;
        value_t residual_f() const;
    };

    /// (local operator as a tensor (rL, n.., rR, rL', n'.., rR') over the window's sites, local solution(s),
    /// local rhs (rL, n.., rR), state)
    using LocalSolver = std::function<void(const Tensor&, std::vector<Tensor>&, const Tensor&, const ALSAlgorithmicData&)>;

    static void lapack_solver(const Tensor& _A, std::vector<Tensor>& _x, const Tensor& _b, const ALSAlgorithmicData& _data);
    static void ASD_solver(const Tensor& _A, std::vector<Tensor>& _x, const Tensor& _b, const ALSAlgorithmicData& _data);

    unsigned sites;
    size_t numHalfSweeps;
    value_t convergenceEpsilon;
    bool useResidualForEndCriterion;
    bool preserveCorePosition;
    bool assumeSPD;
    LocalSolver localSolver;

    ALSVariant(unsigned _sites, size_t _numHalfSweeps, LocalSolver _localSolver, bool _assumeSPD, bool _useResidual = false);

    double operator()(const TTOperator& _A, TTTensor& _x, const TTTensor& _b, value_t _convergenceEpsilon) const {
        return solve(&_A, _x, _b, numHalfSweeps, _convergenceEpsilon);
    }
    double operator()(const TTOperator& _A, TTTensor& _x, const TTTensor& _b, size_t _numHalfSweeps) const {
        return solve(&_A, _x, _b, _numHalfSweeps, convergenceEpsilon);
    }
    double operator()(const TTOperator& _A, TTTensor& _x, const TTTensor& _b) const {
        return solve(&_A, _x, _b, numHalfSweeps, convergenceEpsilon);
    }
    double operator()(TTTensor& _x, const TTTensor& _b, value_t _convergenceEpsilon) const {
        return solve(nullptr, _x, _b, numHalfSweeps, _convergenceEpsilon);
    }
    double operator()(TTTensor& _x, const TTTensor& _b, size_t _numHalfSweeps) const {
        return solve(nullptr, _x, _b, _numHalfSweeps, convergenceEpsilon);
    }
    double operator()(TTTensor& _x, const TTTensor& _b) const { return solve(nullptr, _x, _b, numHalfSweeps, convergenceEpsilon); }

    /// the ALS loop (als.cpp:475-553); returns the last value of the energy functional
    double solve(const TTOperator* _Ap, TTTensor& _x, const TTTensor& _b, size_t _numHalfSweeps, value_t _convergenceEpsilon) const;

   private:
    Tensor construct_local_operator(const ALSAlgorithmicData& _data) const;
    Tensor construct_local_RHS(const ALSAlgorithmicData& _data) const;
    bool check_for_end_of_sweep(ALSAlgorithmicData& _data, size_t _numHalfSweeps, value_t _convergenceEpsilon) const;
};

/// the reference's predefined variants (als.cpp:556-563)
extern const ALSVariant ALS;
extern const ALSVariant ALS_SPD;
/// two-site DMRG (merged component of two neighbours, split by an SVD truncated to the initial ranks)
extern const ALSVariant DMRG;
extern const ALSVariant DMRG_SPD;
extern const ALSVariant ASD;
extern const ALSVariant ASD_SPD;

}  // namespace xerus
