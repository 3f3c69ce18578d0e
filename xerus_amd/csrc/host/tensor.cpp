// xerus::Tensor on HBM (see include/xerus/tensor.h). Every numeric operation runs on the GPU through the
// kernels of libxerus_amd; the host only plans shapes and holds a lazily synchronised mirror for
// operator[] access.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <numeric>

#include "../smallla.hpp"
#include "xerus.h"

namespace xerus {

namespace misc {
thread_local std::mt19937_64 randomEngine(std::random_device{}());
thread_local std::normal_distribution<double> defaultNormalDistribution;
}  // namespace misc

// ------------------------------------------------------------------------------------------------ gpu context
namespace gpu {
namespace {
thread_local int tl_device = -1;
thread_local xrs_handle_t tl_handle = nullptr;  // intentionally never destroyed (tensors may outlive threads)
}  // namespace

void set_device(int _device) {
    XERUS_REQUIRE(tl_handle == nullptr || tl_device == _device, "set_device must be called before the first GPU use");
    tl_device = _device;
}

int device() {
    if (tl_device < 0) {
        const char* e = std::getenv("XERUS_DEVICE");
        tl_device = e ? std::atoi(e) : 0;
    }
    return tl_device;
}

xrs_handle_t handle() {
    if (!tl_handle) {
        xrs_handle_t h = nullptr;
        const int st = xrs_create(&h, device());
        XERUS_REQUIRE(st == 0, "cannot create the GPU context: " << xrs_last_error());
        tl_handle = h;
    }
    return tl_handle;
}

void synchronize() {
    XERUS_REQUIRE(xrs_synchronize(handle()) == 0, xrs_last_error());
}
}  // namespace gpu

// xrs::Error -> generic_error at the C++ API boundary
template <class F>
static auto guard(F&& f) -> decltype(f()) {
    try {
        return f();
    } catch (const xrs::Error& e) {
        throw misc::generic_error(e.msg);
    }
}

// ------------------------------------------------------------------------------------------------ storage
namespace internal {
class Storage {
   public:
    xrs_handle_t h;
    size_t n;
    double* dev = nullptr;
    std::vector<double> host;
    bool devValid = false, hostValid = false;

    Storage(size_t _n, bool _zero) : h(gpu::handle()), n(_n) {
        dev = static_cast<double*>(h->pool->alloc(std::max<size_t>(n, 1) * 8));
        if (_zero) {
            XRS_HIP(hipMemsetAsync(dev, 0, std::max<size_t>(n, 1) * 8, h->stream));
        }
        devValid = true;
    }
    Storage(size_t _n, double* _adopt) : h(gpu::handle()), n(_n), dev(_adopt), devValid(true) {}
    ~Storage() {
        if (dev) {
            try {
                h->pool->release(dev);
            } catch (...) {
            }
        }
    }
    double* device_ro() {
        if (!devValid) {
            XRS_HIP(hipMemcpyAsync(dev, host.data(), n * 8, hipMemcpyHostToDevice, h->stream));
            devValid = true;
        }
        return dev;
    }
    double* device_rw() {
        device_ro();
        hostValid = false;
        return dev;
    }
    const double* host_ro() {
        if (!hostValid) {
            host.resize(n);
            if (n) {
                XRS_HIP(hipMemcpyAsync(host.data(), dev, n * 8, hipMemcpyDeviceToHost, h->stream));
                XRS_HIP(hipStreamSynchronize(h->stream));
            }
            hostValid = true;
        }
        return host.data();
    }
    double* host_rw() {
        host_ro();
        devValid = false;
        return host.data();
    }
    std::shared_ptr<Storage> clone() {
        auto c = std::make_shared<Storage>(n, false);
        if (devValid) {
            if (n) XRS_HIP(hipMemcpyAsync(c->dev, dev, n * 8, hipMemcpyDeviceToDevice, h->stream));
        } else {
            c->host = host;
            c->hostValid = true;
            c->devValid = false;
        }
        return c;
    }
    double* detach() {
        device_ro();
        double* p = dev;
        dev = nullptr;
        return p;
    }
};
}  // namespace internal

using internal::Storage;

static size_t product(const std::vector<size_t>& v, size_t from = 0, size_t to = ~size_t(0)) {
    to = std::min(to, v.size());
    size_t p = 1;
    for (size_t i = from; i < to; ++i) p *= v[i];
    return p;
}

// ------------------------------------------------------------------------------------------------ construction
Tensor::Tensor(const Representation) : dimensions(), size(1), store(std::make_shared<Storage>(1, true)) {}

Tensor::Tensor(DimensionTuple _dimensions, const Representation, const Initialisation _init)
    : dimensions(std::move(_dimensions)), size(product(dimensions)) {
    store = guard([&] { return std::make_shared<Storage>(size, _init == Initialisation::Zero); });
}

Tensor::Tensor(DimensionTuple _dimensions, std::unique_ptr<value_t[]>&& _data)
    : dimensions(std::move(_dimensions)), size(product(dimensions)) {
    store = guard([&] { return std::make_shared<Storage>(size, false); });
    store->host.assign(_data.get(), _data.get() + size);
    store->hostValid = true;
    store->devValid = false;
}

Tensor::Tensor(DimensionTuple _dimensions, const std::function<value_t()>& _f) : Tensor(std::move(_dimensions), Representation::Dense, Initialisation::None) {
    double* h = store->host_rw();
    for (size_t i = 0; i < size; ++i) h[i] = _f();
}

Tensor::Tensor(DimensionTuple _dimensions, const std::function<value_t(const size_t)>& _f)
    : Tensor(std::move(_dimensions), Representation::Dense, Initialisation::None) {
    double* h = store->host_rw();
    for (size_t i = 0; i < size; ++i) h[i] = _f(i);
}

Tensor::Tensor(DimensionTuple _dimensions, const std::function<value_t(const MultiIndex&)>& _f)
    : Tensor(std::move(_dimensions), Representation::Dense, Initialisation::None) {
    double* h = store->host_rw();
    MultiIndex idx(degree(), 0);
    for (size_t i = 0; i < size; ++i) {
        h[i] = _f(idx);
        for (size_t k = degree(); k-- > 0;) {
            if (++idx[k] < dimensions[k]) break;
            idx[k] = 0;
        }
    }
}

Tensor Tensor::ones(DimensionTuple _dimensions) {
    Tensor t(std::move(_dimensions), Representation::Dense, Initialisation::None);
    double* h = t.store->host_rw();
    std::fill(h, h + t.size, 1.0);
    return t;
}

Tensor Tensor::identity(DimensionTuple _dimensions) {
    XERUS_REQUIRE(_dimensions.size() % 2 == 0, "Identity tensor must have even degree, here: " << _dimensions.size());
    const size_t d = _dimensions.size();
    Tensor t(std::move(_dimensions), Representation::Dense, Initialisation::Zero);
    double* h = t.store->host_rw();
    MultiIndex idx(d, 0);
    for (size_t i = 0; i < t.size; ++i) {
        bool diag = true;
        for (size_t k = 0; k < d / 2; ++k) diag &= idx[k] == idx[k + d / 2];
        h[i] = diag ? 1.0 : 0.0;
        for (size_t k = d; k-- > 0;) {
            if (++idx[k] < t.dimensions[k]) break;
            idx[k] = 0;
        }
    }
    return t;
}

Tensor Tensor::kronecker(DimensionTuple _dimensions) {
    const size_t d = _dimensions.size();
    Tensor t(std::move(_dimensions), Representation::Dense, Initialisation::Zero);
    double* h = t.store->host_rw();
    std::fill(h, h + t.size, 0.0);
    if (d == 0) {
        h[0] = 1.0;
        return t;
    }
    const size_t mn = *std::min_element(t.dimensions.begin(), t.dimensions.end());
    for (size_t i = 0; i < mn; ++i) h[multiIndex_to_position(MultiIndex(d, i), t.dimensions)] = 1.0;
    return t;
}

Tensor Tensor::dirac(DimensionTuple _dimensions, const MultiIndex& _position) {
    Tensor t(std::move(_dimensions), Representation::Dense, Initialisation::Zero);
    double* h = t.store->host_rw();
    std::fill(h, h + t.size, 0.0);
    h[multiIndex_to_position(_position, t.dimensions)] = 1.0;
    return t;
}

Tensor Tensor::dirac(DimensionTuple _dimensions, const size_t _position) {
    Tensor t(std::move(_dimensions), Representation::Dense, Initialisation::Zero);
    XERUS_REQUIRE(_position < t.size, "Invalid dirac position");
    double* h = t.store->host_rw();
    std::fill(h, h + t.size, 0.0);
    h[_position] = 1.0;
    return t;
}

Tensor Tensor::adopt_device(DimensionTuple _dimensions, value_t* _dev) {
    Tensor t;
    t.dimensions = std::move(_dimensions);
    t.size = product(t.dimensions);
    t.store = std::make_shared<Storage>(t.size, _dev);
    return t;
}

value_t* Tensor::release_device() {
    apply_factor();
    ensure_own_data();
    value_t* p = store->detach();
    store = std::make_shared<Storage>(1, true);
    dimensions.clear();
    size = 1;
    return p;
}

size_t Tensor::multiIndex_to_position(const MultiIndex& _idx, const DimensionTuple& _dims) {
    XERUS_REQUIRE(_idx.size() == _dims.size(), "MultiIndex has wrong degree: " << _idx.size() << " vs " << _dims.size());
    size_t pos = 0;
    for (size_t i = 0; i < _dims.size(); ++i) {
        XERUS_REQUIRE(_idx[i] < _dims[i], "Index " << i << " out of bounds: " << _idx[i] << " >= " << _dims[i]);
        pos = pos * _dims[i] + _idx[i];
    }
    return pos;
}

// ------------------------------------------------------------------------------------------------ data access
void Tensor::ensure_own_data() {
    if (store.use_count() > 1) store = guard([&] { return store->clone(); });
}

void Tensor::apply_factor() {
    if (factor == 1.0) return;
    ensure_own_data();
    guard([&] { xrs::scal(store->h, store->device_rw(), factor, size); });
    factor = 1.0;
}

const value_t* Tensor::device_data() const { return guard([&] { return store->device_ro(); }); }

value_t* Tensor::device_data_for_write() {
    ensure_own_data();
    return guard([&] { return store->device_rw(); });
}

value_t* Tensor::device_data_applied() {
    apply_factor();
    return device_data_for_write();
}

value_t& Tensor::operator[](const size_t _position) {
    XERUS_REQUIRE(_position < size, "Position " << _position << " does not exist in Tensor of size " << size);
    apply_factor();
    ensure_own_data();
    return guard([&] { return store->host_rw(); })[_position];
}

value_t Tensor::operator[](const size_t _position) const {
    XERUS_REQUIRE(_position < size, "Position " << _position << " does not exist in Tensor of size " << size);
    return factor * guard([&] { return store->host_ro(); })[_position];
}

value_t& Tensor::operator[](const MultiIndex& _positions) { return (*this)[multiIndex_to_position(_positions, dimensions)]; }

value_t Tensor::operator[](const MultiIndex& _positions) const { return (*this)[multiIndex_to_position(_positions, dimensions)]; }

value_t* Tensor::get_dense_data() {
    apply_factor();
    ensure_own_data();
    return guard([&] { return store->host_rw(); });
}

std::vector<value_t> Tensor::to_host() const {
    const double* h = guard([&] { return store->host_ro(); });
    std::vector<value_t> out(h, h + size);
    if (factor != 1.0)
        for (auto& v : out) v *= factor;
    return out;
}

void Tensor::reset(DimensionTuple _newDim, const Representation, const Initialisation _init) { reset(std::move(_newDim), _init); }

void Tensor::reset(DimensionTuple _newDim, const Initialisation _init) {
    dimensions = std::move(_newDim);
    size = product(dimensions);
    factor = 1.0;
    store = guard([&] { return std::make_shared<Storage>(size, _init == Initialisation::Zero); });
}

void Tensor::reset() {
    dimensions.clear();
    size = 1;
    factor = 1.0;
    store = guard([&] { return std::make_shared<Storage>(1, true); });
}

void Tensor::reinterpret_dimensions(DimensionTuple _newDimensions) {
    XERUS_REQUIRE(product(_newDimensions) == size, "New dimensions must not change the size of the tensor in reinterpretation");
    dimensions = std::move(_newDimensions);
}

// ------------------------------------------------------------------------------------------------ norms/arith
value_t Tensor::frob_norm() const {
    return std::abs(factor) * guard([&] { return xrs::reduce_to_host(store->h, 0, store->device_ro(), nullptr, size); });
}

value_t Tensor::one_norm() const {
    return std::abs(factor) * guard([&] { return xrs::reduce_to_host(store->h, 2, store->device_ro(), nullptr, size); });
}

Tensor& Tensor::operator+=(const Tensor& _other) {
    XERUS_REQUIRE(dimensions == _other.dimensions, "The dimensions in Tensor addition must coincide");
    apply_factor();
    const double* o = _other.device_data();
    double* me = device_data_for_write();
    guard([&] { xrs::axpy(store->h, me, _other.factor, o, size); });
    return *this;
}

Tensor& Tensor::operator-=(const Tensor& _other) {
    XERUS_REQUIRE(dimensions == _other.dimensions, "The dimensions in Tensor subtraction must coincide");
    apply_factor();
    const double* o = _other.device_data();
    double* me = device_data_for_write();
    guard([&] { xrs::axpy(store->h, me, -_other.factor, o, size); });
    return *this;
}

Tensor& Tensor::operator*=(const value_t _factor) {
    factor *= _factor;
    return *this;
}

Tensor& Tensor::operator/=(const value_t _divisor) {
    factor /= _divisor;
    return *this;
}

Tensor operator+(Tensor _lhs, const Tensor& _rhs) { return _lhs += _rhs; }
Tensor operator-(Tensor _lhs, const Tensor& _rhs) { return _lhs -= _rhs; }
Tensor operator*(const value_t _factor, Tensor _tensor) { return _tensor *= _factor; }
Tensor operator*(Tensor _tensor, const value_t _factor) { return _tensor *= _factor; }
Tensor operator/(Tensor _tensor, const value_t _divisor) { return _tensor /= _divisor; }

// ------------------------------------------------------------------------------------------------ mode operations
// (pre, dim, post) decomposition of a mode
static void mode_split(const Tensor& t, size_t mode, size_t& pre, size_t& post) {
    pre = product(t.dimensions, 0, mode);
    post = product(t.dimensions, mode + 1);
}

void Tensor::resize_mode(const size_t _mode, const size_t _newDim, size_t _cutPos) {
    XERUS_REQUIRE(_mode < degree(), "Can't resize mode " << _mode << " as the tensor is only order " << degree());
    const size_t oldDim = dimensions[_mode];
    if (_newDim == oldDim) return;
    _cutPos = std::min(_cutPos, oldDim);
    XERUS_REQUIRE(_newDim > 0, "Dimension must be larger than 0! Is " << _newDim);
    XERUS_REQUIRE(_newDim > oldDim || _cutPos >= oldDim - _newDim,
                  "Cannot remove " << oldDim - _newDim << " slates starting (exclusivly) at position " << _cutPos);
    size_t pre, post;
    mode_split(*this, _mode, pre, post);
    DimensionTuple nd = dimensions;
    nd[_mode] = _newDim;
    Tensor out(nd, Representation::Dense, _newDim > oldDim ? Initialisation::Zero : Initialisation::None);
    const double* src = device_data();
    double* dst = out.device_data_for_write();
    xrs_handle_t h = store->h;
    // slates [0, front) stay; growing inserts zero slates at the cut, shrinking drops the slates in
    // [cut - removed, cut) (tensor.cpp:626-729)
    const size_t front = _newDim > oldDim ? _cutPos : _cutPos - (oldDim - _newDim);
    const size_t back = oldDim - _cutPos;
    const size_t dstBack = _newDim - back;
    guard([&] {
        if (pre && post && front)
            XRS_HIP(hipMemcpy2DAsync(dst, _newDim * post * 8, src, oldDim * post * 8, front * post * 8, pre, hipMemcpyDeviceToDevice,
                                     h->stream));
        if (pre && post && back)
            XRS_HIP(hipMemcpy2DAsync(dst + dstBack * post, _newDim * post * 8, src + _cutPos * post, oldDim * post * 8, back * post * 8,
                                     pre, hipMemcpyDeviceToDevice, h->stream));
    });
    out.factor = factor;
    *this = std::move(out);
}

void Tensor::fix_mode(const size_t _mode, const size_t _slatePosition) {
    XERUS_REQUIRE(_mode < degree(), "Can't fix mode " << _mode << " of an order " << degree() << " tensor");
    XERUS_REQUIRE(_slatePosition < dimensions[_mode], "Can't fix mode at " << _slatePosition);
    size_t pre, post;
    mode_split(*this, _mode, pre, post);
    const size_t dim = dimensions[_mode];
    DimensionTuple nd = dimensions;
    nd.erase(nd.begin() + long(_mode));
    Tensor out(nd, Representation::Dense, Initialisation::None);
    const double* src = device_data();
    double* dst = out.device_data_for_write();
    xrs_handle_t h = store->h;
    guard([&] {
        if (pre && post)
            XRS_HIP(hipMemcpy2DAsync(dst, post * 8, src + _slatePosition * post, dim * post * 8, post * 8, pre,
                                     hipMemcpyDeviceToDevice, h->stream));
    });
    out.factor = factor;
    *this = std::move(out);
}

void Tensor::remove_slate(const size_t _mode, const size_t _pos) {
    XERUS_REQUIRE(_mode < degree() && _pos < dimensions[_mode], "invalid slate");
    resize_mode(_mode, dimensions[_mode] - 1, _pos + 1);
}

void Tensor::perform_trace(size_t _firstMode, size_t _secondMode) {
    XERUS_REQUIRE(_firstMode != _secondMode, "Given indices must not coincide");
    XERUS_REQUIRE(_firstMode < degree() && _secondMode < degree(), "invalid trace modes");
    XERUS_REQUIRE(dimensions[_firstMode] == dimensions[_secondMode], "The dimensions of the traced modes must coincide");
    if (_firstMode > _secondMode) std::swap(_firstMode, _secondMode);
    // move the two traced modes to the back, then sum the diagonal
    std::vector<size_t> shuffle(degree());
    size_t pos = 0;
    for (size_t i = 0; i < degree(); ++i)
        if (i != _firstMode && i != _secondMode) shuffle[i] = pos++;
    shuffle[_firstMode] = degree() - 2;
    shuffle[_secondMode] = degree() - 1;
    Tensor tmp = reshuffle(*this, shuffle);
    DimensionTuple nd;
    for (size_t i = 0; i < degree(); ++i)
        if (i != _firstMode && i != _secondMode) nd.push_back(dimensions[i]);
    const size_t m = dimensions[_firstMode];
    Tensor out(nd, Representation::Dense, Initialisation::None);
    const double* src = tmp.device_data();
    double* dst = out.device_data_for_write();
    guard([&] { xrs::diag_sum(store->h, dst, src, out.size, m); });
    out.factor = tmp.factor;
    *this = std::move(out);
}

void Tensor::modify_diagonal_entries(const std::function<void(value_t&)>& _f) {
    modify_diagonal_entries([&](value_t& v, const size_t) { _f(v); });
}

void Tensor::modify_diagonal_entries(const std::function<void(value_t&, const size_t)>& _f) {
    XERUS_REQUIRE(degree() == 0 || degree() % 2 == 0, "Diagonal modification only for even degree");
    double* h = get_dense_data();
    if (degree() == 0) {
        _f(h[0], 0);
        return;
    }
    const size_t half = product(dimensions, 0, degree() / 2);
    const size_t other = product(dimensions, degree() / 2);
    const size_t n = std::min(half, other);
    for (size_t i = 0; i < n; ++i) _f(h[i * other + i], i);
}

void Tensor::modify_entries(const std::function<void(value_t&)>& _f) {
    double* h = get_dense_data();
    for (size_t i = 0; i < size; ++i) _f(h[i]);
}

void Tensor::modify_entries(const std::function<void(value_t&, const size_t)>& _f) {
    double* h = get_dense_data();
    for (size_t i = 0; i < size; ++i) _f(h[i], i);
}

void Tensor::offset_add(const Tensor& _other, const std::vector<size_t>& _offsets) {
    XERUS_REQUIRE(degree() == _other.degree() && _offsets.size() == degree(), "Degrees and offsets must match");
    for (size_t i = 0; i < degree(); ++i)
        XERUS_REQUIRE(_offsets[i] + _other.dimensions[i] <= dimensions[i], "offset_add out of range in mode " << i);
    apply_factor();
    const double* src = _other.device_data();
    double* dst = device_data_for_write();
    guard([&] { xrs::offset_add(store->h, dst, dimensions.data(), src, _other.dimensions.data(), degree(), _offsets.data(), _other.factor); });
}

std::string Tensor::to_string() const {
    std::ostringstream s;
    const auto v = to_host();
    if (degree() == 0) {
        s << v[0];
        return s.str();
    }
    const size_t last = dimensions.back();
    for (size_t i = 0; i < size; ++i) {
        s << v[i] << ((i + 1) % last == 0 ? "\n" : " ");
    }
    return s.str();
}

std::ostream& operator<<(std::ostream& _out, const Tensor& _tensor) { return _out << _tensor.to_string(); }

// ------------------------------------------------------------------------------------------------ contract / reshuffle
void reshuffle(Tensor& _out, const Tensor& _base, const std::vector<size_t>& _shuffle) {
    XERUS_REQUIRE(_shuffle.size() == _base.degree(), "IE: shuffle has wrong size");
    std::vector<size_t> outDims(_base.degree());
    std::vector<char> seen(_base.degree(), 0);
    for (size_t i = 0; i < _base.degree(); ++i) {
        XERUS_REQUIRE(_shuffle[i] < _base.degree(), _shuffle[i] << " is no valid new position!");
        XERUS_REQUIRE(!seen[_shuffle[i]], _shuffle[i] << " illegally appeared twice.");
        seen[_shuffle[i]] = 1;
        outDims[_shuffle[i]] = _base.dimensions[i];
    }
    bool identity = true;
    for (size_t i = 0; i < _base.degree(); ++i) identity &= _shuffle[i] == i;
    if (identity) {
        _out = _base;
        return;
    }
    Tensor result(outDims, Tensor::Representation::Dense, Tensor::Initialisation::None);
    const double* src = _base.device_data();
    double* dst = result.device_data_for_write();
    guard([&] {
        xrs_handle_t h = gpu::handle();
        if (_base.degree() == 0) {
            XRS_HIP(hipMemcpyAsync(dst, src, 8, hipMemcpyDeviceToDevice, h->stream));
        } else {
            xrs::permute(h, dst, src, _base.degree(), _base.dimensions.data(), _shuffle.data());
        }
    });
    result.factor = _base.factor;
    _out = std::move(result);
}

Tensor reshuffle(const Tensor& _base, const std::vector<size_t>& _shuffle) {
    Tensor r;
    reshuffle(r, _base, _shuffle);
    return r;
}

void contract(Tensor& _result, const Tensor& _lhs, const bool _lhsTrans, const Tensor& _rhs, const bool _rhsTrans,
              const size_t _numModes) {
    XERUS_REQUIRE(_numModes <= _lhs.degree() && _numModes <= _rhs.degree(),
                  "Cannot contract more indices than both tensors have. we have: " << _lhs.degree() << " and " << _rhs.degree()
                                                                                   << " but want to contract: " << _numModes);
    const size_t lo = _lhs.degree() - _numModes, ro = _rhs.degree() - _numModes;
    const size_t lRemStart = _lhsTrans ? _numModes : 0, lConStart = _lhsTrans ? 0 : lo;
    const size_t rRemStart = _rhsTrans ? 0 : _numModes, rConStart = _rhsTrans ? ro : 0;
    for (size_t i = 0; i < _numModes; ++i)
        XERUS_REQUIRE(_lhs.dimensions[lConStart + i] == _rhs.dimensions[rConStart + i],
                      "Dimensions of the be contracted indices do not coincide.");
    const size_t left = product(_lhs.dimensions, lRemStart, lRemStart + lo);
    const size_t mid = product(_lhs.dimensions, lConStart, lConStart + _numModes);
    const size_t right = product(_rhs.dimensions, rRemStart, rRemStart + ro);
    Tensor::DimensionTuple rd(_lhs.dimensions.begin() + long(lRemStart), _lhs.dimensions.begin() + long(lRemStart + lo));
    rd.insert(rd.end(), _rhs.dimensions.begin() + long(rRemStart), _rhs.dimensions.begin() + long(rRemStart + ro));
    Tensor result(rd, Tensor::Representation::Dense, Tensor::Initialisation::None);   // never aliases lhs/rhs
    const double* A = _lhs.device_data();
    const double* B = _rhs.device_data();
    double* C = result.device_data_for_write();
    guard([&] {
        xrs::gemm(gpu::handle(), C, left, right, _lhs.factor * _rhs.factor, A, _lhsTrans ? left : mid, _lhsTrans, mid, B,
                  _rhsTrans ? mid : right, _rhsTrans);
    });
    _result = std::move(result);
}

Tensor contract(const Tensor& _lhs, const bool _lhsTrans, const Tensor& _rhs, const bool _rhsTrans, const size_t _numModes) {
    Tensor r;
    contract(r, _lhs, _lhsTrans, _rhs, _rhsTrans, _numModes);
    return r;
}

// ------------------------------------------------------------------------------------------------ factorisations
static void factorization_sizes(const Tensor& t, size_t split, size_t& lhs, size_t& rhs) {
    XERUS_REQUIRE(split <= t.degree(), "Split position must be in range.");
    lhs = product(t.dimensions, 0, split);
    rhs = product(t.dimensions, split);
}

static Tensor::DimensionTuple dims_with(const Tensor::DimensionTuple& d, size_t from, size_t to, size_t rank, bool rankFirst) {
    Tensor::DimensionTuple r;
    if (rankFirst) r.push_back(rank);
    r.insert(r.end(), d.begin() + long(from), d.begin() + long(to));
    if (!rankFirst) r.push_back(rank);
    return r;
}

// tensor.cpp:1424-1489
namespace {
// shared shape logic of solve / solve_least_squares (tensor.cpp:1585-1606, 1659-1681)
void solve_impl(Tensor& _X, const Tensor& _A, const Tensor& _B, const size_t _extraDegree, bool _ls) {
    XERUS_REQUIRE(&_X != &_B && &_X != &_A, "Not supportet yet");
    XERUS_REQUIRE(_B.degree() >= _extraDegree, "Inconsistent dimensions.");
    const size_t degM = _B.degree() - _extraDegree;
    XERUS_REQUIRE(_A.degree() >= degM, "Inconsistent dimensions.");
    const size_t degN = _A.degree() - degM;
    for (size_t i = 0; i < degM; ++i) XERUS_REQUIRE(_A.dimensions[i] == _B.dimensions[i], "Inconsistent dimensions.");
    Tensor::DimensionTuple newDimX(_A.dimensions.begin() + long(degM), _A.dimensions.end());
    newDimX.insert(newDimX.end(), _B.dimensions.begin() + long(degM), _B.dimensions.end());
    size_t m = 1, n = 1, p = 1;
    for (size_t i = 0; i < degM; ++i) m *= _A.dimensions[i];
    for (size_t i = degM; i < degM + degN; ++i) n *= _A.dimensions[i];
    for (size_t i = degM; i < _B.degree(); ++i) p *= _B.dimensions[i];
    Tensor X(newDimX, Tensor::Representation::Dense, Tensor::Initialisation::None);
    xrs_handle_t h = gpu::handle();
    const double* Ad = _A.device_data();
    const double* Bd = _B.device_data();
    double* Xd = X.device_data_for_write();
    guard([&] {
        if (_ls) xrs::svd_solve(h, Xd, Ad, m, n, Bd, p);
        else xrs::solve_dense(h, Xd, Ad, m, n, Bd, p);
    });
    X.factor = _B.factor / _A.factor;   // (:1703)
    _X = std::move(X);
}
}  // namespace

void solve(Tensor& _X, const Tensor& _A, const Tensor& _B, const size_t _extraDegree) { solve_impl(_X, _A, _B, _extraDegree, false); }

void solve_least_squares(Tensor& _X, const Tensor& _A, const Tensor& _B, const size_t _extraDegree) {
    solve_impl(_X, _A, _B, _extraDegree, true);
}

void calculate_svd(Tensor& _U, Tensor& _S, Tensor& _Vt, Tensor _input, const size_t _splitPos, const size_t _maxRank,
                   const value_t _eps) {
    XERUS_REQUIRE(0 <= _eps && _eps < 1, "Epsilon must be fullfill 0 <= _eps < 1.");
    size_t m, n;
    factorization_sizes(_input, _splitPos, m, n);
    const size_t k = std::min(m, n);
    xrs_handle_t h = gpu::handle();
    xrs::DevBuf U(h, m * k * 8), S(h, k * 8), Vt(h, k * n * 8);
    const double* A = _input.device_data();
    guard([&] { xrs::svd(h, A, m, n, U.d(), S.d(), Vt.d()); });
    std::vector<double> s(k);
    guard([&] {
        XRS_HIP(hipMemcpyAsync(s.data(), S.d(), k * 8, hipMemcpyDeviceToHost, h->stream));
        XRS_HIP(hipStreamSynchronize(h->stream));
    });
    size_t rank = k;
    if (_maxRank != 0) rank = std::min(rank, _maxRank);
    for (size_t j = 1; j < rank; ++j) {
        if (s[j] <= _eps * s[0]) {
            rank = j;
            break;
        }
    }
    Tensor Ut(dims_with(_input.dimensions, 0, _splitPos, rank, false), Tensor::Representation::Dense, Tensor::Initialisation::None);
    Tensor Vtt(dims_with(_input.dimensions, _splitPos, _input.degree(), rank, true), Tensor::Representation::Dense,
               Tensor::Initialisation::None);
    guard([&] {
        XRS_HIP(hipMemcpy2DAsync(Ut.device_data_for_write(), rank * 8, U.d(), k * 8, rank * 8, m, hipMemcpyDeviceToDevice, h->stream));
        XRS_HIP(hipMemcpyAsync(Vtt.device_data_for_write(), Vt.d(), rank * n * 8, hipMemcpyDeviceToDevice, h->stream));
    });
    if (!(s[0] > 0.0)) {
        // the zero matrix: rank 1 with sigma 0; dgesdd's factors are still orthonormal (e_0 columns / rows)
        const double one = 1.0;
        guard([&] {
            XRS_HIP(hipMemsetAsync(Ut.device_data_for_write(), 0, m * rank * 8, h->stream));
            XRS_HIP(hipMemsetAsync(Vtt.device_data_for_write(), 0, rank * n * 8, h->stream));
            XRS_HIP(hipMemcpyAsync(Ut.device_data_for_write(), &one, 8, hipMemcpyHostToDevice, h->stream));
            XRS_HIP(hipMemcpyAsync(Vtt.device_data_for_write(), &one, 8, hipMemcpyHostToDevice, h->stream));
            XRS_HIP(hipStreamSynchronize(h->stream));
        });
    }
    Tensor St({rank, rank}, Tensor::Representation::Dense, Tensor::Initialisation::Zero);
    {
        double* hs = St.get_dense_data();
        for (size_t i = 0; i < rank; ++i) hs[i * rank + i] = std::abs(_input.factor) * s[i];
    }
    if (_input.factor < 0.0) Vtt *= -1;
    _U = std::move(Ut);
    _S = std::move(St);
    _Vt = std::move(Vtt);
}

void calculate_qr(Tensor& _Q, Tensor& _R, Tensor _input, const size_t _splitPos) {
    size_t m, n;
    factorization_sizes(_input, _splitPos, m, n);
    const size_t k = std::min(m, n);
    Tensor Q(dims_with(_input.dimensions, 0, _splitPos, k, false), Tensor::Representation::Dense, Tensor::Initialisation::None);
    Tensor R(dims_with(_input.dimensions, _splitPos, _input.degree(), k, true), Tensor::Representation::Dense,
             Tensor::Initialisation::None);
    const double* A = _input.device_data();
    guard([&] { xrs::qr(gpu::handle(), A, m, n, Q.device_data_for_write(), R.device_data_for_write()); });
    R.factor = _input.factor;
    _Q = std::move(Q);
    _R = std::move(R);
}

void calculate_rq(Tensor& _R, Tensor& _Q, Tensor _input, const size_t _splitPos) {
    size_t m, n;
    factorization_sizes(_input, _splitPos, m, n);
    const size_t k = std::min(m, n);
    Tensor R(dims_with(_input.dimensions, 0, _splitPos, k, false), Tensor::Representation::Dense, Tensor::Initialisation::None);
    Tensor Q(dims_with(_input.dimensions, _splitPos, _input.degree(), k, true), Tensor::Representation::Dense,
             Tensor::Initialisation::None);
    const double* A = _input.device_data();
    guard([&] { xrs::rq(gpu::handle(), A, m, n, R.device_data_for_write(), Q.device_data_for_write()); });
    R.factor = _input.factor;
    _R = std::move(R);
    _Q = std::move(Q);
}

void calculate_qc(Tensor& _Q, Tensor& _C, Tensor _input, const size_t _splitPos) {
    size_t m, n;
    factorization_sizes(_input, _splitPos, m, n);
    const size_t k = std::min(m, n);
    xrs_handle_t h = gpu::handle();
    xrs::DevBuf Q(h, m * k * 8), C(h, k * n * 8);
    const double* A = _input.device_data();
    const size_t rank = guard([&] { return xrs::qc(h, A, m, n, Q.d(), C.d()); });
    Tensor Qt(dims_with(_input.dimensions, 0, _splitPos, rank, false), Tensor::Representation::Dense, Tensor::Initialisation::None);
    Tensor Ct(dims_with(_input.dimensions, _splitPos, _input.degree(), rank, true), Tensor::Representation::Dense,
              Tensor::Initialisation::None);
    guard([&] {
        XRS_HIP(hipMemcpyAsync(Qt.device_data_for_write(), Q.d(), m * rank * 8, hipMemcpyDeviceToDevice, h->stream));
        XRS_HIP(hipMemcpyAsync(Ct.device_data_for_write(), C.d(), rank * n * 8, hipMemcpyDeviceToDevice, h->stream));
    });
    Ct.factor = _input.factor;
    _Q = std::move(Qt);
    _C = std::move(Ct);
}

void calculate_cq(Tensor& _C, Tensor& _Q, Tensor _input, const size_t _splitPos) {
    size_t m, n;
    factorization_sizes(_input, _splitPos, m, n);
    const size_t k = std::min(m, n);
    xrs_handle_t h = gpu::handle();
    xrs::DevBuf C(h, m * k * 8), Q(h, k * n * 8);
    const double* A = _input.device_data();
    const size_t rank = guard([&] { return xrs::cq(h, A, m, n, C.d(), Q.d()); });
    Tensor Ct(dims_with(_input.dimensions, 0, _splitPos, rank, false), Tensor::Representation::Dense, Tensor::Initialisation::None);
    Tensor Qt(dims_with(_input.dimensions, _splitPos, _input.degree(), rank, true), Tensor::Representation::Dense,
              Tensor::Initialisation::None);
    guard([&] {
        XRS_HIP(hipMemcpyAsync(Ct.device_data_for_write(), C.d(), m * rank * 8, hipMemcpyDeviceToDevice, h->stream));
        XRS_HIP(hipMemcpyAsync(Qt.device_data_for_write(), Q.d(), rank * n * 8, hipMemcpyDeviceToDevice, h->stream));
    });
    Ct.factor = _input.factor;
    _C = std::move(Ct);
    _Q = std::move(Qt);
}

void pseudo_inverse(Tensor& _inverse, const Tensor& _input, const size_t _splitPos) {
    Tensor U, S, Vt;
    calculate_svd(U, S, Vt, _input, _splitPos, 0, EPSILON);
    S.modify_diagonal_entries([](value_t& _a) { _a = 1 / _a; });
    // inverse = Vt^T S^-1 U^T : contract(Vt, true, S, true) then with U transposed
    Tensor tmp = contract(Vt, true, S, true, 1);
    _inverse = contract(tmp, false, U, true, 1);
}

Tensor pseudo_inverse(const Tensor& _input, const size_t _splitPos) {
    Tensor r;
    pseudo_inverse(r, _input, _splitPos);
    return r;
}

// ------------------------------------------------------------------------------------------------ comparisons
bool approx_equal(const Tensor& _a, const Tensor& _b, const value_t _eps) {
    XERUS_REQUIRE(_a.dimensions == _b.dimensions, "The dimensions of the compared tensors don't match: " << _a.dimensions.size()
                                                                                                        << " vs " << _b.dimensions.size());
    const Tensor diff = _a - _b;
    return diff.frob_norm() <= _eps * (_a.frob_norm() + _b.frob_norm()) / 2.0;
}

bool approx_entrywise_equal(const Tensor& _a, const Tensor& _b, const value_t _eps) {
    if (_a.dimensions != _b.dimensions) return false;
    const auto x = _a.to_host(), y = _b.to_host();
    for (size_t i = 0; i < x.size(); ++i) {
        const double d = std::abs(x[i] - y[i]);
        if (d > _eps * std::max({1.0, std::abs(x[i]), std::abs(y[i])})) return false;
    }
    return true;
}

bool approx_entrywise_equal(const Tensor& _tensor, const std::vector<value_t>& _values, const value_t _eps) {
    if (_tensor.size != _values.size()) return false;
    const auto x = _tensor.to_host();
    for (size_t i = 0; i < x.size(); ++i) {
        const double d = std::abs(x[i] - _values[i]);
        if (d > _eps * std::max({1.0, std::abs(x[i]), std::abs(_values[i])})) return false;
    }
    return true;
}


}  // namespace xerus
