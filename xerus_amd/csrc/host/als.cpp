// ALS / DMRG / ASD on TT tensors (reference src/xerus/algorithms/als.cpp:35-565). The algorithm
// is the reference's: full-rank boundary components are folded away (prepare_x_for_als, :109-187),
// left/right environments are cached as stacks (:226-257, :354-392), the local operator and right-hand
// side are assembled from them (:394-449), solved (lapack_solver :37-69 / ASD_solver :72-91), and the
// core moves with keepRank (unpivoted QR/RQ) to the next site; a half sweep ends at the range
// boundary and the run stops on the sweep budget or when the energy changes by less than epsilon
// (:451-471).
// MI355X realisation: every environment update, local assembly and energy is ONE indexed product
// (permutations + MFMA GEMMs in the reference's heuristic contraction order) on HBM-resident tensors;
// the local systems are solved by xerus::solve (blocked Cholesky: all local operators here are
// symmetric positive definite for SPD operators, and A^T A otherwise). Multi-site variants (DMRG: two
// sites) optimise the merged component of `sites` neighbours and split it again with the indexed SVD
// (lapack_solver, :43-69), truncated to the initial ranks.
//
// Deviation: in the reference's move_to_next_index the decreasing direction extends the right stacks by
// the slice of currIndex (als.cpp:371-379), which is the site that enters the next window when sites > 1
// (dimensionally consistent only for equal ranks); here the site that LEAVES the window,
// currIndex + sites - 1, is contracted -- identical for sites == 1, the mathematically correct
// environment for DMRG (checked against dense solutions and the oracle's restatement, which makes the
// same choice).
#include <cmath>

#include "xerus.h"
#include "xerus/algorithms/als.h"

namespace xerus {

ALSVariant::ALSVariant(unsigned _sites, size_t _numHalfSweeps, LocalSolver _localSolver, bool _assumeSPD, bool _useResidual)
    : sites(_sites),
      numHalfSweeps(_numHalfSweeps),
      convergenceEpsilon(1e-6),
      useResidualForEndCriterion(_useResidual),
      preserveCorePosition(true),
      assumeSPD(_assumeSPD),
      localSolver(std::move(_localSolver)) {
    XERUS_REQUIRE(_sites >= 1, "at least one site must be optimised");
}

// ---------------------------------------------------------------------------------------- solvers
void ALSVariant::lapack_solver(const Tensor& _A, std::vector<Tensor>& _x, const Tensor& _b, const ALSAlgorithmicData& _data) {
    Tensor x;
    xerus::solve(x, _A, _b);
    // several sites: split the merged component by SVDs truncated to the initial ranks (als.cpp:50-68)
    Index i, j, k, l;
    const size_t sites = _data.ALS.sites;
    if (_data.direction == Increasing) {
        for (size_t p = 0; p + 1 < sites; ++p) {
            Tensor U, S;
            (U(i ^ 2, j), S(j, k), x(k, l & 1)) = SVD(x(i ^ 2, l & 2), _data.targetRank[_data.currIndex + p]);
            _x[p] = std::move(U);
            x(j, l & 1) = S(j, k) * x(k, l & 1);
        }
        _x.back() = std::move(x);
    } else {
        for (size_t p = sites - 1; p > 0; --p) {
            Tensor S, Vt;
            (x(i & 1, j), S(j, k), Vt(k, l & 1)) = SVD(x(i & 2, l ^ 2), _data.targetRank[_data.currIndex + p - 1]);
            _x[p] = std::move(Vt);
            x(i & 1, k) = x(i & 1, j) * S(j, k);
        }
        _x[0] = std::move(x);
    }
}

void ALSVariant::ASD_solver(const Tensor& _A, std::vector<Tensor>& _x, const Tensor& _b, const ALSAlgorithmicData& _data) {
    XERUS_REQUIRE(_data.ALS.sites == 1, "ASD only defined for single site alternation at the moment");
    Index i, j;
    Tensor grad;
    grad(i & 0) = _b(i & 0) - _A(i / 2, j / 2) * _x[0](j & 0);
    value_t alpha;
    if (_data.ALS.assumeSPD) {
        const value_t ng = frob_norm(grad);
        alpha = ng * ng / value_t(grad(i & 0) * _A(i / 2, j / 2) * grad(j & 0));
    } else {
        Tensor g2;
        g2(i & 0) = _A(j / 2, i / 2) * grad(j & 0);
        Tensor Ag;
        Ag(i & 0) = _A(i / 2, j / 2) * g2(j & 0);
        alpha = frob_norm(g2) / frob_norm(Ag);
        grad = std::move(g2);
    }
    _x[0] += alpha * grad;
}

// ---------------------------------------------------------------------------------------- state
ALSVariant::ALSAlgorithmicData::ALSAlgorithmicData(const ALSVariant& _ALS, const TTOperator* _A, TTTensor& _x, const TTTensor& _b)
    : ALS(_ALS),
      A(_A),
      x(_x),
      b(_b),
      targetRank(_x.ranks()),
      normB(frob_norm(_b)),
      canonicalizeAtTheEnd(_x.canonicalized),
      corePosAtTheEnd(_x.corePosition) {
    prepare_x_for_als();
    prepare_stacks();
    currIndex = optimizedRange.first;
}

// components whose left (right) unfolding already has full rank carry no freedom: they are replaced by
// the identity isometry and their content pushed into the neighbour (als.cpp:109-187)
void ALSVariant::ALSAlgorithmicData::prepare_x_for_als() {
    const size_t d = x.degree();
    Index r1, r2, n1, cr1;
    size_t first = 0, dimProd = 1;
    while (first + 1 < d) {
        const size_t localDim = x.dimensions[first];
        const size_t newProd = dimProd * localDim;
        if (x.rank(first) < newProd) break;
        Tensor cur = x.get_component(first);
        cur.reinterpret_dimensions({cur.dimensions[0] * cur.dimensions[1], cur.dimensions[2]});
        Tensor merged;
        merged(r1, n1, r2) = cur(r1, cr1) * x.get_component(first + 1)(cr1, n1, r2);
        x.set_component(first + 1, std::move(merged));
        x.set_component(first, Tensor({dimProd, localDim, newProd},
                                      [&](const Tensor::MultiIndex& _idx) { return _idx[0] * localDim + _idx[1] == _idx[2] ? 1.0 : 0.0; }));
        x.require_correct_format();
        ++first;
        dimProd = newProd;
    }
    size_t firstNot = d;
    dimProd = 1;
    while (firstNot > first + ALS.sites) {
        const size_t localDim = x.dimensions[firstNot - 1];
        const size_t newProd = dimProd * localDim;
        if (x.rank(firstNot - 2) < newProd) break;
        Tensor cur = x.get_component(firstNot - 1);
        cur.reinterpret_dimensions({cur.dimensions[0], cur.dimensions[1] * cur.dimensions[2]});
        Tensor merged;
        merged(r1, n1, r2) = x.get_component(firstNot - 2)(r1, n1, cr1) * cur(cr1, r2);
        x.set_component(firstNot - 2, std::move(merged));
        x.set_component(firstNot - 1, Tensor({newProd, localDim, dimProd},
                                             [&](const Tensor::MultiIndex& _idx) { return _idx[0] == _idx[1] * dimProd + _idx[2] ? 1.0 : 0.0; }));
        x.require_correct_format();
        --firstNot;
        dimProd = newProd;
    }
    if (canonicalizeAtTheEnd && corePosAtTheEnd < first) {
        x.assume_core_position(first);
    } else {
        if (canonicalizeAtTheEnd && corePosAtTheEnd >= firstNot) x.assume_core_position(firstNot - 1);
        x.move_core(first, true);
    }
    optimizedRange = {first, firstNot};
}

// environment updates (the reference's localOperatorSlice / localRhsSlice contracted into the stack,
// :190-223, 240-256): one product each
Tensor ALSVariant::ALSAlgorithmicData::op_step_left(const Tensor& _env, size_t _pos) const {
    Index r1, r2, r3, r4, c1, c2, c3, c4, n1, n2, n3;
    const Tensor& xk = x.get_component(_pos);
    const Tensor& Ak = A->get_component(_pos);
    Tensor res;
    if (ALS.assumeSPD) res(c1, c2, c3) = _env(r1, r2, r3) * xk(r1, n1, c1) * Ak(r2, n1, n2, c2) * xk(r3, n2, c3);
    else res(c1, c2, c3, c4) = _env(r1, r2, r3, r4) * xk(r1, n1, c1) * Ak(r2, n2, n1, c2) * Ak(r3, n2, n3, c3) * xk(r4, n3, c4);
    return res;
}

Tensor ALSVariant::ALSAlgorithmicData::op_step_right(const Tensor& _env, size_t _pos) const {
    Index r1, r2, r3, r4, c1, c2, c3, c4, n1, n2, n3;
    const Tensor& xk = x.get_component(_pos);
    const Tensor& Ak = A->get_component(_pos);
    Tensor res;
    if (ALS.assumeSPD) res(r1, r2, r3) = xk(r1, n1, c1) * Ak(r2, n1, n2, c2) * xk(r3, n2, c3) * _env(c1, c2, c3);
    else res(r1, r2, r3, r4) = xk(r1, n1, c1) * Ak(r2, n2, n1, c2) * Ak(r3, n2, n3, c3) * xk(r4, n3, c4) * _env(c1, c2, c3, c4);
    return res;
}

Tensor ALSVariant::ALSAlgorithmicData::rhs_step_left(const Tensor& _env, size_t _pos) const {
    Index r1, r2, r3, c1, c2, c3, n1, n2;
    const Tensor& xk = x.get_component(_pos);
    const Tensor& bk = b.get_component(_pos);
    Tensor res;
    if (ALS.assumeSPD || A == nullptr) res(c1, c2) = _env(r1, r2) * bk(r1, n1, c1) * xk(r2, n1, c2);
    else res(c1, c2, c3) = _env(r1, r2, r3) * bk(r1, n1, c1) * A->get_component(_pos)(r2, n1, n2, c2) * xk(r3, n2, c3);
    return res;
}

Tensor ALSVariant::ALSAlgorithmicData::rhs_step_right(const Tensor& _env, size_t _pos) const {
    Index r1, r2, r3, c1, c2, c3, n1, n2;
    const Tensor& xk = x.get_component(_pos);
    const Tensor& bk = b.get_component(_pos);
    Tensor res;
    if (ALS.assumeSPD || A == nullptr) res(r1, r2) = bk(r1, n1, c1) * xk(r2, n1, c2) * _env(c1, c2);
    else res(r1, r2, r3) = bk(r1, n1, c1) * A->get_component(_pos)(r2, n1, n2, c2) * xk(r3, n2, c3) * _env(c1, c2, c3);
    return res;
}

void ALSVariant::ALSAlgorithmicData::prepare_stacks() {
    const size_t d = x.degree();
    const bool plain = ALS.assumeSPD || A == nullptr;
    const Tensor opOne = plain ? Tensor::ones({1, 1, 1}) : Tensor::ones({1, 1, 1, 1});
    const Tensor rhsOne = plain ? Tensor::ones({1, 1}) : Tensor::ones({1, 1, 1});
    opLeft.assign(1, opOne);
    opRight.assign(1, opOne);
    rhsLeft.assign(1, rhsOne);
    rhsRight.assign(1, rhsOne);
    for (size_t i = d - 1; i > optimizedRange.first + ALS.sites - 1; --i) {
        if (A) opRight.push_back(op_step_right(opRight.back(), i));
        rhsRight.push_back(rhs_step_right(rhsRight.back(), i));
    }
    for (size_t i = 0; i < optimizedRange.first; ++i) {
        if (A) opLeft.push_back(op_step_left(opLeft.back(), i));
        rhsLeft.push_back(rhs_step_left(rhsLeft.back(), i));
    }
}

void ALSVariant::ALSAlgorithmicData::move_to_next_index() {
    // (sites > 1: the solver's SVD split has already moved the core)
    if (direction == Increasing) {
        if (ALS.sites == 1) x.move_core(currIndex + 1, true);
        if (A) {
            opRight.pop_back();
            opLeft.push_back(op_step_left(opLeft.back(), currIndex));
        }
        rhsRight.pop_back();
        rhsLeft.push_back(rhs_step_left(rhsLeft.back(), currIndex));
        ++currIndex;
    } else {
        if (ALS.sites == 1) x.move_core(currIndex - 1, true);
        const size_t leaving = currIndex + ALS.sites - 1;   // (see the deviation note at the top)
        if (A) {
            opLeft.pop_back();
            opRight.push_back(op_step_right(opRight.back(), leaving));
        }
        rhsLeft.pop_back();
        rhsRight.push_back(rhs_step_right(rhsRight.back(), leaving));
        --currIndex;
    }
}

// the energy functionals of choose_energy_functional (:259-320), over the window currIndex ..
// currIndex + sites - 1: <x, A x> / <x, A^T A x> and <b, x> / <b, A x> as one product each
namespace {
// opLeft * [x_p A_p x_p]_p * opRight (spd) or with A^T A (4-index environments), contracted to a scalar
IndexedProduct window_op(const ALSVariant::ALSAlgorithmicData& _d) {
    const size_t s = _d.ALS.sites, c = _d.currIndex;
    const bool spd = _d.ALS.assumeSPD;
    std::vector<Index> rx(s + 1), ra(s + 1), rb(s + 1), ry(s + 1);
    IndexedProduct p = spd ? _d.opLeft.back()(rx[0], ra[0], ry[0]).as_product() : _d.opLeft.back()(rx[0], ra[0], rb[0], ry[0]).as_product();
    for (size_t q = 0; q < s; ++q) {
        Index m1, m2, m3;
        const Tensor& xk = _d.x.get_component(c + q);
        const Tensor& Ak = _d.A->get_component(c + q);
        if (spd) p = p * xk(rx[q], m1, rx[q + 1]) * Ak(ra[q], m1, m2, ra[q + 1]) * xk(ry[q], m2, ry[q + 1]);
        else p = p * xk(rx[q], m1, rx[q + 1]) * Ak(ra[q], m2, m1, ra[q + 1]) * Ak(rb[q], m2, m3, rb[q + 1]) * xk(ry[q], m3, ry[q + 1]);
    }
    return spd ? p * _d.opRight.back()(rx[s], ra[s], ry[s]) : p * _d.opRight.back()(rx[s], ra[s], rb[s], ry[s]);
}
// rhsLeft * [b_p x_p]_p * rhsRight (plain) or [b_p A_p x_p]_p
IndexedProduct window_rhs(const ALSVariant::ALSAlgorithmicData& _d) {
    const size_t s = _d.ALS.sites, c = _d.currIndex;
    const bool plain = _d.ALS.assumeSPD || _d.A == nullptr;
    std::vector<Index> rb(s + 1), ra(s + 1), rx(s + 1);
    IndexedProduct p = plain ? _d.rhsLeft.back()(rb[0], rx[0]).as_product() : _d.rhsLeft.back()(rb[0], ra[0], rx[0]).as_product();
    for (size_t q = 0; q < s; ++q) {
        Index m1, m2;
        const Tensor& xk = _d.x.get_component(c + q);
        const Tensor& bk = _d.b.get_component(c + q);
        if (plain) p = p * bk(rb[q], m1, rb[q + 1]) * xk(rx[q], m1, rx[q + 1]);
        else p = p * bk(rb[q], m1, rb[q + 1]) * _d.A->get_component(c + q)(ra[q], m1, m2, ra[q + 1]) * xk(rx[q], m2, rx[q + 1]);
    }
    return plain ? p * _d.rhsRight.back()(rb[s], rx[s]) : p * _d.rhsRight.back()(rb[s], ra[s], rx[s]);
}
}  // namespace

value_t ALSVariant::ALSAlgorithmicData::residual_f() const {
    Index n1, n2;
    if (A == nullptr) return frob_norm(x - b);
    if (ALS.assumeSPD) {
        TTTensor Ax;
        Ax(n1 & 0) = (*A)(n1 / 2, n2 / 2) * x(n2 & 0);
        return frob_norm(Ax - b) / normB;
    }
    const value_t xAtAx = value_t(window_op(*this));
    const value_t bAx = value_t(window_rhs(*this));
    return std::sqrt(xAtAx - 2 * bAx + normB * normB) / normB;
}

value_t ALSVariant::ALSAlgorithmicData::energy_f() const {
    if (ALS.useResidualForEndCriterion || (A && !ALS.assumeSPD)) return residual_f();
    const value_t bx = value_t(window_rhs(*this));
    if (A == nullptr) {
        Index r1;
        const Tensor& xk = x.get_component(currIndex);
        return 0.5 * value_t(xk(r1 & 0) * xk(r1 & 0)) - bx;
    }
    return std::abs(0.5 * value_t(window_op(*this)) - bx);
}

// ---------------------------------------------------------------------------------------- local problem
// local operator (als.cpp:383-400) as one product: modes (rL, n_0 .. n_{s-1}, rR, rL', n'_0 .. n'_{s-1}, rR')
Tensor ALSVariant::construct_local_operator(const ALSAlgorithmicData& _data) const {
    const size_t s = sites, c = _data.currIndex;
    Index a, bb, a2, b2;
    std::vector<Index> iv(s), jv(s), r1(s + 1), r2(s + 1);
    IndexedProduct p = assumeSPD ? _data.opLeft.back()(a, r1[0], a2).as_product() : _data.opLeft.back()(a, r1[0], r2[0], a2).as_product();
    for (size_t q = 0; q < s; ++q) {
        const Tensor& Ak = _data.A->get_component(c + q);
        if (assumeSPD) {
            p = p * Ak(r1[q], iv[q], jv[q], r1[q + 1]);
        } else {
            Index y;
            p = p * Ak(r1[q], y, iv[q], r1[q + 1]) * Ak(r2[q], y, jv[q], r2[q + 1]);
        }
    }
    p = assumeSPD ? p * _data.opRight.back()(bb, r1[s], b2) : p * _data.opRight.back()(bb, r1[s], r2[s], b2);
    std::vector<Index> out{a};
    out.insert(out.end(), iv.begin(), iv.end());
    out.push_back(bb);
    out.push_back(a2);
    out.insert(out.end(), jv.begin(), jv.end());
    out.push_back(b2);
    Tensor res;
    res(out) = p;
    return res;
}

// local right-hand side (als.cpp:404-423): modes (rL, n_0 .. n_{s-1}, rR)
Tensor ALSVariant::construct_local_RHS(const ALSAlgorithmicData& _data) const {
    const size_t s = sites, c = _data.currIndex;
    const bool plain = assumeSPD || _data.A == nullptr;
    Index a, bb;
    std::vector<Index> iv(s), r1(s + 1), r2(s + 1);
    IndexedProduct p = plain ? _data.rhsLeft.back()(r1[0], a).as_product() : _data.rhsLeft.back()(r1[0], r2[0], a).as_product();
    for (size_t q = 0; q < s; ++q) {
        const Tensor& bk = _data.b.get_component(c + q);
        if (plain) {
            p = p * bk(r1[q], iv[q], r1[q + 1]);
        } else {
            Index y;
            p = p * bk(r1[q], y, r1[q + 1]) * _data.A->get_component(c + q)(r2[q], y, iv[q], r2[q + 1]);
        }
    }
    p = plain ? p * _data.rhsRight.back()(r1[s], bb) : p * _data.rhsRight.back()(r1[s], r2[s], bb);
    std::vector<Index> out{a};
    out.insert(out.end(), iv.begin(), iv.end());
    out.push_back(bb);
    Tensor res;
    res(out) = p;
    return res;
}

bool ALSVariant::check_for_end_of_sweep(ALSAlgorithmicData& _data, size_t _numHalfSweeps, value_t _convergenceEpsilon) const {
    const bool atEnd = (_data.direction == Decreasing && _data.currIndex == _data.optimizedRange.first) ||
                       (_data.direction == Increasing && _data.currIndex == _data.optimizedRange.second - sites);
    if (!atEnd) return false;
    _data.halfSweepCount += 1;
    _data.lastEnergy2 = _data.lastEnergy;
    _data.lastEnergy = _data.energy;
    _data.energy = _data.energy_f();
    if (_data.halfSweepCount == _numHalfSweeps || std::abs(_data.lastEnergy - _data.energy) < _convergenceEpsilon ||
        std::abs(_data.lastEnergy2 - _data.energy) < _convergenceEpsilon ||
        (_data.optimizedRange.second - _data.optimizedRange.first <= sites)) {
        if (_data.canonicalizeAtTheEnd && preserveCorePosition) _data.x.move_core(_data.corePosAtTheEnd, true);
        return true;
    }
    _data.direction = _data.direction == Increasing ? Decreasing : Increasing;
    return false;
}

double ALSVariant::solve(const TTOperator* _Ap, TTTensor& _x, const TTTensor& _b, size_t _numHalfSweeps, value_t _convergenceEpsilon) const {
    _x.require_correct_format();
    _b.require_correct_format();
    XERUS_REQUIRE(_x.degree() > 0, "");
    XERUS_REQUIRE(_x.dimensions == _b.dimensions, "");
    if (_Ap) {
        _Ap->require_correct_format();
        XERUS_REQUIRE(_Ap->dimensions.size() == _b.dimensions.size() * 2, "");
        for (size_t i = 0; i < _x.dimensions.size(); ++i) {
            XERUS_REQUIRE(_Ap->dimensions[i] == _x.dimensions[i], "");
            XERUS_REQUIRE(_Ap->dimensions[i + _Ap->degree() / 2] == _x.dimensions[i], "");
        }
    }
    ALSAlgorithmicData data(*this, _Ap, _x, _b);
    data.energy = data.energy_f();
    while (true) {
        if (_Ap) {
            std::vector<Tensor> tmpX;
            for (size_t p = 0; p < sites; ++p) tmpX.push_back(_x.get_component(data.currIndex + p));
            localSolver(construct_local_operator(data), tmpX, construct_local_RHS(data), data);
            for (size_t p = 0; p < sites; ++p) _x.set_component(data.currIndex + p, std::move(tmpX[p]));
        } else {
            XERUS_REQUIRE(sites == 1, "approximation dmrg not implemented yet");
            _x.component(data.currIndex) = construct_local_RHS(data);
        }
        if (check_for_end_of_sweep(data, _numHalfSweeps, _convergenceEpsilon)) return data.energy;
        data.move_to_next_index();
    }
}

const ALSVariant ALS(1, 0, ALSVariant::lapack_solver, false);
const ALSVariant ALS_SPD(1, 0, ALSVariant::lapack_solver, true);
const ALSVariant DMRG(2, 0, ALSVariant::lapack_solver, false);
const ALSVariant DMRG_SPD(2, 0, ALSVariant::lapack_solver, true);
const ALSVariant ASD(1, 0, ALSVariant::ASD_solver, false);
const ALSVariant ASD_SPD(1, 0, ALSVariant::ASD_solver, true);

}  // namespace xerus
