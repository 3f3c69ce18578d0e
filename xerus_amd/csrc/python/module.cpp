// Python bindings of the xerus hot-path API (module xerus_amd.xerus), mirroring the names and call
// patterns of the reference's Python module (src/xerus/python/{tensor,indexedTensor,ttnetwork,misc}.cpp):
//     import xerus_amd.xerus as xe
//     i, j, k = xe.indices(3)
//     A(i, j) << B(i, k) * C(k, j)
// Everything computes on the GPU through libxerus_amd; numpy arrays are only the host interchange format.
#include <limits>
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/operators.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "xerus.h"

namespace py = pybind11;
using namespace xerus;

namespace {

std::vector<Index> to_indices(const py::args& _args) {
    std::vector<Index> out;
    for (const auto& a : _args) {
        if (py::isinstance<Index>(a)) out.push_back(a.cast<Index>());
        else if (py::isinstance<py::int_>(a)) out.emplace_back(int64(a.cast<long long>()));
        else if (py::isinstance<py::list>(a) || py::isinstance<py::tuple>(a)) {
            for (const auto& b : a) out.push_back(b.cast<Index>());
        } else throw py::type_error("indices must be xerus Index objects or integers");
    }
    return out;
}

Tensor from_ndarray(py::array_t<double, py::array::c_style | py::array::forcecast> _a) {
    Tensor::DimensionTuple dims(_a.shape(), _a.shape() + _a.ndim());
    size_t n = 1;
    for (size_t d : dims) n *= d;
    std::unique_ptr<value_t[]> data(new value_t[n]);
    if (n) std::memcpy(data.get(), _a.data(), n * sizeof(double));
    return Tensor(dims, std::move(data));
}

py::array_t<double> to_ndarray(const Tensor& _t) {
    const auto v = _t.to_host();
    py::array_t<double> a(std::vector<py::ssize_t>(_t.dimensions.begin(), _t.dimensions.end()));
    if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(double));
    return a;
}

}  // namespace

PYBIND11_MODULE(xerus, m) {
    m.doc() = "MI355X-native xerus hot path: dense tensors, indexed contractions, TT rounding and inner products on HBM";
    py::register_exception<misc::generic_error>(m, "generic_error", PyExc_RuntimeError);

    m.attr("EPSILON") = EPSILON;
    m.def("set_device", &gpu::set_device);
    m.def("synchronize", &gpu::synchronize);
    m.def("seed", [](uint64 _s) {
        misc::randomEngine.seed(_s);
        misc::defaultNormalDistribution.reset();
    }, "reseed the thread's mt19937_64 (and reset the normal distribution's cached value)");

    // ------------------------------------------------------------------ Index
    py::class_<Index>(m, "Index")
        .def(py::init<>())
        .def(py::init([](long long _i) { return Index(int64(_i)); }))
        .def("__xor__", &Index::operator^)
        .def("__pow__", [](const Index& _i, size_t _s) { return _i ^ _s; })
        .def("__and__", &Index::operator&)
        .def("__truediv__", &Index::operator/)
        .def_readonly("valueId", &Index::valueId)
        .def_readonly("span", &Index::span)
        .def("fixed", &Index::fixed)
        .def("__eq__", [](const Index& _a, const Index& _b) { return _a == _b; })
        .def("__hash__", [](const Index& _a) { return py::hash(py::int_(_a.valueId)); })
        .def("__repr__", [](const Index& _i) {
            std::ostringstream s;
            s << _i;
            return s.str();
        });
    py::implicitly_convertible<py::int_, Index>();
    m.def("indices", [](size_t _n) { return indices(_n); }, py::arg("n") = 1);

    // ------------------------------------------------------------------ indexed expressions
    py::class_<IndexedProduct>(m, "IndexedProduct")
        .def("__mul__", [](const IndexedProduct& _a, const IndexedProduct& _b) { return _a * _b; })
        .def("__mul__", [](const IndexedProduct& _a, const IndexedTensor<Tensor>& _b) { return _a * _b; })
        .def("__mul__", [](const IndexedProduct& _a, value_t _f) { return _a * _f; })
        .def("__rmul__", [](const IndexedProduct& _a, value_t _f) { return _f * _a; })
        .def("__truediv__", [](const IndexedProduct& _a, value_t _f) { return _a / _f; })
        .def("__neg__", [](const IndexedProduct& _a) { return -_a; })
        .def("__add__", [](const IndexedProduct& _a, const IndexedProduct& _b) { return _a + _b; })
        .def("__add__", [](const IndexedProduct& _a, const IndexedTensor<Tensor>& _b) { return _a + _b; })
        .def("__sub__", [](const IndexedProduct& _a, const IndexedProduct& _b) { return _a - _b; })
        .def("__sub__", [](const IndexedProduct& _a, const IndexedTensor<Tensor>& _b) { return _a - _b; })
        .def("__float__", [](const IndexedProduct& _a) { return value_t(_a); });

    py::class_<IndexedSum>(m, "IndexedSum")
        .def("__add__", [](const IndexedSum& _a, const IndexedProduct& _b) { return _a + _b; })
        .def("__add__", [](const IndexedSum& _a, const IndexedTensor<Tensor>& _b) { return _a + _b; })
        .def("__sub__", [](const IndexedSum& _a, const IndexedProduct& _b) { return _a - _b; })
        .def("__sub__", [](const IndexedSum& _a, const IndexedTensor<Tensor>& _b) { return _a - _b; });

    py::class_<IndexedTensor<Tensor>>(m, "IndexedTensor")
        .def("__lshift__", [](IndexedTensor<Tensor>& _l, const IndexedTensor<Tensor>& _r) { _l << _r; })
        .def("__lshift__", [](IndexedTensor<Tensor>& _l, const IndexedProduct& _r) { _l << _r; })
        .def("__lshift__", [](IndexedTensor<Tensor>& _l, const IndexedSum& _r) { _l << _r; })
        .def("__iadd__", [](IndexedTensor<Tensor>& _l, const IndexedProduct& _r) { return _l += _r; })
        .def("__iadd__", [](IndexedTensor<Tensor>& _l, const IndexedTensor<Tensor>& _r) { return _l += _r; })
        .def("__isub__", [](IndexedTensor<Tensor>& _l, const IndexedProduct& _r) { return _l -= _r; })
        .def("__isub__", [](IndexedTensor<Tensor>& _l, const IndexedTensor<Tensor>& _r) { return _l -= _r; })
        .def("__mul__", [](const IndexedTensor<Tensor>& _a, const IndexedTensor<Tensor>& _b) { return _a * _b; })
        .def("__mul__", [](const IndexedTensor<Tensor>& _a, const IndexedProduct& _b) { return _a * _b; })
        .def("__mul__", [](const IndexedTensor<Tensor>& _a, value_t _f) { return _a * _f; })
        .def("__rmul__", [](const IndexedTensor<Tensor>& _a, value_t _f) { return _f * _a; })
        .def("__truediv__", [](const IndexedTensor<Tensor>& _a, value_t _f) { return _a / _f; })
        .def("__truediv__", [](const IndexedTensor<Tensor>& _b, const IndexedTensor<Tensor>& _A) { return _b / _A; })
        .def("__neg__", [](const IndexedTensor<Tensor>& _a) { return -_a; })
        .def("__add__", [](const IndexedTensor<Tensor>& _a, const IndexedTensor<Tensor>& _b) { return _a + _b; })
        .def("__add__", [](const IndexedTensor<Tensor>& _a, const IndexedProduct& _b) { return _a + _b; })
        .def("__sub__", [](const IndexedTensor<Tensor>& _a, const IndexedTensor<Tensor>& _b) { return _a - _b; })
        .def("__sub__", [](const IndexedTensor<Tensor>& _a, const IndexedProduct& _b) { return _a - _b; })
        .def("frob_norm", [](const IndexedTensor<Tensor>& _a) { return frob_norm(_a); })
        .def("__float__", [](const IndexedTensor<Tensor>& _a) { return value_t(_a); });

    // ------------------------------------------------------------------ Tensor
    py::class_<Tensor>(m, "Tensor")
        .def(py::init<>())
        .def(py::init([](const TTTensor& _tt) { return _tt.to_tensor(); }))
        .def(py::init([](const TTOperator& _op) { return _op.to_tensor(); }))
        .def(py::init([](const std::vector<size_t>& _dims) { return Tensor(_dims); }))
        .def_static("from_ndarray", &from_ndarray)
        .def("to_ndarray", &to_ndarray)
        .def_static("random", [](const std::vector<size_t>& _dims) { return Tensor::random(_dims); })
        .def_static("ones", &Tensor::ones)
        .def_static("identity", &Tensor::identity)
        .def_static("kronecker", &Tensor::kronecker)
        .def_static("dirac", py::overload_cast<Tensor::DimensionTuple, const Tensor::MultiIndex&>(&Tensor::dirac))
        .def_static("dirac", py::overload_cast<Tensor::DimensionTuple, const size_t>(&Tensor::dirac))
        .def_readonly("dimensions", &Tensor::dimensions)
        .def_readonly("size", &Tensor::size)
        .def_readwrite("factor", &Tensor::factor)
        .def("degree", &Tensor::degree)
        .def("has_factor", &Tensor::has_factor)
        .def("is_dense", &Tensor::is_dense)
        .def("is_sparse", &Tensor::is_sparse)
        .def("frob_norm", &Tensor::frob_norm)
        .def("one_norm", &Tensor::one_norm)
        .def("reinterpret_dimensions", &Tensor::reinterpret_dimensions)
        .def("resize_mode", &Tensor::resize_mode, py::arg("mode"), py::arg("newDim"), py::arg("cutPos") = ~0ul)
        .def("fix_mode", &Tensor::fix_mode)
        .def("remove_slate", &Tensor::remove_slate)
        .def("perform_trace", &Tensor::perform_trace)
        .def("offset_add", &Tensor::offset_add)
        .def("apply_factor", &Tensor::apply_factor)
        .def("ensure_own_data", &Tensor::ensure_own_data)
        .def("dense_copy", &Tensor::dense_copy)
        .def_static("multiIndex_to_position", &Tensor::multiIndex_to_position)
        .def("__call__", [](Tensor& _t, py::args _a) { return _t(to_indices(_a)); }, py::keep_alive<0, 1>())
        .def("__getitem__", [](const Tensor& _t, size_t _i) { return _t[_i]; })
        .def("__getitem__", [](const Tensor& _t, const std::vector<size_t>& _i) { return _t[_i]; })
        .def("__setitem__", [](Tensor& _t, size_t _i, value_t _v) { _t[_i] = _v; })
        .def("__setitem__", [](Tensor& _t, const std::vector<size_t>& _i, value_t _v) { _t[_i] = _v; })
        .def("__str__", &Tensor::to_string)
        .def(py::self + py::self)
        .def(py::self - py::self)
        .def(py::self += py::self)
        .def(py::self -= py::self)
        .def(py::self * value_t())
        .def(value_t() * py::self)
        .def(py::self / value_t())
        .def("__copy__", [](const Tensor& _t) { return Tensor(_t); });

    // factorisation expressions (reference python/factorizations.cpp): (U(i,r), S(r,s), Vt(s,j)) << SVD(A(i,j))
    py::class_<TensorFactorisation>(m, "TensorFactorisation")
        .def("__rlshift__", [](const TensorFactorisation& _f, const py::tuple& _lhs) {
            std::vector<IndexedTensor<Tensor>*> out;
            for (const auto& o : _lhs) out.push_back(o.cast<IndexedTensor<Tensor>*>());
            _f(out);
        });
    py::class_<SVD, TensorFactorisation>(m, "SVD_temporary");
    py::class_<QR, TensorFactorisation>(m, "QR_temporary");
    py::class_<RQ, TensorFactorisation>(m, "RQ_temporary");
    py::class_<QC, TensorFactorisation>(m, "QC_temporary");
    py::class_<CQ, TensorFactorisation>(m, "CQ_temporary");
    // eps defaults to EPSILON, or to 0 with a soft threshold (the C++ SVD(A, softThreshold) constructor)
    auto def_factorisations = [&m](auto _tag) {
        using In = decltype(_tag);
        m.def("SVD", [](const In& _a, size_t _maxRank, py::object _eps, double _soft, bool _preventZero) {
            const double eps = _eps.is_none() ? (_soft > 0.0 ? 0.0 : EPSILON) : _eps.cast<double>();
            return new SVD(_a, _maxRank, eps, _soft, _preventZero);
        }, py::arg("source"), py::arg("maxRank") = std::numeric_limits<size_t>::max(), py::arg("eps") = py::none(),
              py::arg("softThreshold") = 0.0, py::arg("preventZero") = false, py::keep_alive<0, 1>());
        m.def("QR", [](const In& _a) { return new QR(_a); }, py::keep_alive<0, 1>());
        m.def("RQ", [](const In& _a) { return new RQ(_a); }, py::keep_alive<0, 1>());
        m.def("QC", [](const In& _a) { return new QC(_a); }, py::keep_alive<0, 1>());
        m.def("CQ", [](const In& _a) { return new CQ(_a); }, py::keep_alive<0, 1>());
    };
    def_factorisations(IndexedTensor<Tensor>(nullptr, {}, false));
    def_factorisations(IndexedProduct());

    m.def("contract", py::overload_cast<const Tensor&, bool, const Tensor&, bool, size_t>(&contract));
    m.def("reshuffle", py::overload_cast<const Tensor&, const std::vector<size_t>&>(&reshuffle));
    m.def("frob_norm", [](const Tensor& _t) { return _t.frob_norm(); });
    m.def("frob_norm", [](const TTTensor& _t) { return _t.frob_norm(); });
    m.def("frob_norm", [](const IndexedTensor<Tensor>& _t) { return frob_norm(_t); });
    m.def("one_norm", [](const Tensor& _t) { return _t.one_norm(); });
    m.def("pseudo_inverse", py::overload_cast<const Tensor&, size_t>(&pseudo_inverse));
    m.def("approx_equal", py::overload_cast<const Tensor&, const Tensor&, value_t>(&approx_equal), py::arg("a"), py::arg("b"),
          py::arg("eps") = EPSILON);
    m.def("approx_equal", py::overload_cast<const TTTensor&, const TTTensor&, value_t>(&approx_equal), py::arg("a"), py::arg("b"),
          py::arg("eps") = EPSILON);
    m.def("approx_entrywise_equal", py::overload_cast<const Tensor&, const Tensor&, value_t>(&approx_entrywise_equal), py::arg("a"),
          py::arg("b"), py::arg("eps") = EPSILON);
    m.def("approx_entrywise_equal", py::overload_cast<const Tensor&, const std::vector<value_t>&, value_t>(&approx_entrywise_equal),
          py::arg("a"), py::arg("values"), py::arg("eps") = EPSILON);
    m.def("calculate_svd", [](const Tensor& _A, size_t _split, size_t _maxRank, value_t _eps) {
        Tensor U, S, Vt;
        calculate_svd(U, S, Vt, _A, _split, _maxRank, _eps);
        return py::make_tuple(U, S, Vt);
    }, py::arg("A"), py::arg("splitPos"), py::arg("maxRank") = 0, py::arg("eps") = EPSILON);
    m.def("calculate_qr", [](const Tensor& _A, size_t _split) {
        Tensor Q, R;
        calculate_qr(Q, R, _A, _split);
        return py::make_tuple(Q, R);
    });
    m.def("calculate_rq", [](const Tensor& _A, size_t _split) {
        Tensor R, Q;
        calculate_rq(R, Q, _A, _split);
        return py::make_tuple(R, Q);
    });
    m.def("calculate_qc", [](const Tensor& _A, size_t _split) {
        Tensor Q, C;
        calculate_qc(Q, C, _A, _split);
        return py::make_tuple(Q, C);
    });
    m.def("calculate_cq", [](const Tensor& _A, size_t _split) {
        Tensor C, Q;
        calculate_cq(C, Q, _A, _split);
        return py::make_tuple(C, Q);
    });
    m.def("save_to_file", [](const Tensor& _t, const std::string& _f, bool _tsv) {
        misc::save_to_file(_t, _f, _tsv ? misc::FileFormat::TSV : misc::FileFormat::BINARY);
    }, py::arg("tensor"), py::arg("filename"), py::arg("tsv") = false);
    m.def("save_to_file", [](const TTTensor& _t, const std::string& _f, bool _tsv) {
        misc::save_to_file(_t, _f, _tsv ? misc::FileFormat::TSV : misc::FileFormat::BINARY);
    }, py::arg("tt"), py::arg("filename"), py::arg("tsv") = false);
    m.def("save_to_file", [](const TensorNetwork& _t, const std::string& _f, bool _tsv) {
        misc::save_to_file(_t, _f, _tsv ? misc::FileFormat::TSV : misc::FileFormat::BINARY);
    }, py::arg("network"), py::arg("filename"), py::arg("tsv") = false);
    // misc::load_from_file<TensorNetwork> / <TTTensor> / <Tensor> (misc/fileIO.h:139-163): the stored type must match
    m.def("load_network_from_file", &misc::load_network_from_file);
    m.def("load_tt_from_file", &misc::load_tt_from_file);
    m.def("load_tensor_from_file", &misc::load_tensor_from_file);
    // the object type is read from the file's header (Tensor, TTTensor; a TensorNetwork file loads as its
    // contracted Tensor)
    m.def("load_from_file", [](const std::string& _f) -> py::object {
        const std::string type = misc::file_type(_f);
        if (type == "xerus::TTNetwork<false>") return py::cast(misc::load_tt_from_file(_f));
        if (type == "xerus::TensorNetwork") return py::cast(misc::load_network_from_file(_f).to_tensor());
        return py::cast(misc::load_tensor_from_file(_f));
    });
    m.def("file_type", &misc::file_type);

    // ------------------------------------------------------------------ TensorNetwork (results of chop)
    py::class_<IndexedNetwork>(m, "IndexedNetwork")
        .def("__lshift__", [](IndexedNetwork& _l, const IndexedProduct& _r) { _l = _r; })
        .def("__lshift__", [](IndexedNetwork& _l, const IndexedTensor<Tensor>& _r) { _l = _r; });
    py::class_<TensorNetwork>(m, "TensorNetwork")
        .def(py::init<>())
        .def(py::init<Tensor>())
        .def(py::init<const TensorNetwork&>())
        .def_readonly("dimensions", &TensorNetwork::dimensions)
        .def("degree", &TensorNetwork::degree)
        .def("num_nodes", &TensorNetwork::num_nodes)
        .def("frob_norm", &TensorNetwork::frob_norm)
        .def("to_tensor", &TensorNetwork::to_tensor)
        .def("require_valid_network", &TensorNetwork::require_valid_network)
        .def("__call__", [](TensorNetwork& _t, py::args _a) { return _t(to_indices(_a)); }, py::keep_alive<0, 1>())
        .def("__getitem__", [](const TensorNetwork& _t, size_t _i) { return _t[_i]; })
        .def("__getitem__", [](const TensorNetwork& _t, const std::vector<size_t>& _i) { return _t[_i]; });

    // ------------------------------------------------------------------ TTTensor
    py::class_<IndexedTTStack>(m, "IndexedTTStack")
        .def("__mul__", [](const IndexedTTStack& _s, const IndexedTensor<TTTensor>& _y) { return _s * _y; });
    py::class_<IndexedTensor<TTOperator>>(m, "IndexedTTOperator")
        .def("__mul__", [](const IndexedTensor<TTOperator>& _a, const IndexedTensor<TTTensor>& _x) { return _a * _x; })
        .def("__mul__", [](const IndexedTensor<TTOperator>& _a, const IndexedTensor<TTOperator>& _b) { return _a * _b; })
        .def("__lshift__", [](IndexedTensor<TTOperator>& _l, const IndexedTTStack& _r) { _l = _r; });
    py::class_<IndexedTensor<TTTensor>>(m, "IndexedTTTensor")
        .def("__mul__", [](const IndexedTensor<TTTensor>& _a, const IndexedTensor<TTTensor>& _b) { return _a * _b; })
        .def("__mul__", [](const IndexedTensor<TTTensor>& _x, const IndexedTensor<TTOperator>& _a) { return _x * _a; })
        .def("__lshift__", [](IndexedTensor<TTTensor>& _l, const IndexedTTStack& _r) { _l = _r; });
    py::class_<IndexedTTProduct>(m, "IndexedTTProduct")
        .def("__float__", [](const IndexedTTProduct& _p) { return value_t(_p); });

    py::class_<TTTensor>(m, "TTTensor")
        .def(py::init<>())
        .def(py::init<const TTTensor&>())
        .def(py::init([](const Tensor& _t, value_t _eps, size_t _maxRank) { return TTTensor(_t, _eps, _maxRank); }), py::arg("tensor"),
             py::arg("eps") = EPSILON, py::arg("maxRank") = std::numeric_limits<size_t>::max())
        .def(py::init([](const Tensor& _t, value_t _eps, const std::vector<size_t>& _maxRanks) { return TTTensor(_t, _eps, _maxRanks); }))
        .def(py::init([](const std::vector<size_t>& _dims) { return TTTensor(_dims); }))
        .def(py::init([](size_t _degree) { return TTTensor(_degree); }))
        .def_static("random", [](const std::vector<size_t>& _dims, const std::vector<size_t>& _ranks) { return TTTensor::random(_dims, _ranks); })
        .def_static("random", [](const std::vector<size_t>& _dims, size_t _rank) { return TTTensor::random(_dims, _rank); })
        .def_static("random_raw",
                    [](const std::vector<size_t>& _dims, const std::vector<size_t>& _ranks) { return TTTensor::random_raw(_dims, _ranks); })
        .def_static("reduce_to_maximal_ranks", &TTTensor::reduce_to_maximal_ranks)
        .def_static("ones", &TTTensor::ones)
        .def_static("kronecker", &TTTensor::kronecker)
        .def_static("dirac", py::overload_cast<std::vector<size_t>, const std::vector<size_t>&>(&TTTensor::dirac))
        .def_static("dirac", py::overload_cast<std::vector<size_t>, const size_t>(&TTTensor::dirac))
        .def("fix_mode", &TTTensor::fix_mode)
        .def("resize_mode", &TTTensor::resize_mode, py::arg("mode"), py::arg("newDim"), py::arg("cutPos") = ~0ul)
        .def("chop", &TTTensor::chop)
        .def("require_correct_format", &TTTensor::require_correct_format)
        .def_readonly("dimensions", &TTTensor::dimensions)
        .def_readonly("canonicalized", &TTTensor::canonicalized)
        .def_readonly("corePosition", &TTTensor::corePosition)
        .def("degree", &TTTensor::degree)
        .def("ranks", &TTTensor::ranks)
        .def("rank", &TTTensor::rank)
        .def("get_component", &TTTensor::get_component)
        .def("set_component", &TTTensor::set_component)
        .def("move_core", &TTTensor::move_core, py::arg("position"), py::arg("keepRank") = false)
        .def("assume_core_position", &TTTensor::assume_core_position)
        .def("canonicalize_left", &TTTensor::canonicalize_left)
        .def("canonicalize_right", &TTTensor::canonicalize_right)
        .def("round", py::overload_cast<const std::vector<size_t>&, const double>(&TTTensor::round), py::arg("maxRanks"),
             py::arg("eps") = EPSILON)
        .def("round", py::overload_cast<const size_t>(&TTTensor::round))
        .def("round", py::overload_cast<const value_t>(&TTTensor::round))
        .def("soft_threshold", py::overload_cast<const std::vector<double>&, const bool>(&TTTensor::soft_threshold), py::arg("taus"),
             py::arg("preventZero") = false)
        .def("soft_threshold", py::overload_cast<const double, const bool>(&TTTensor::soft_threshold), py::arg("tau"),
             py::arg("preventZero") = false)
        .def("frob_norm", &TTTensor::frob_norm)
        .def("exceeds_maximal_ranks", &TTTensor::exceeds_maximal_ranks)
        .def("__call__", [](TTTensor& _t, py::args _a) { return _t(to_indices(_a)); }, py::keep_alive<0, 1>())
        .def(py::self + py::self)
        .def(py::self - py::self)
        .def(py::self += py::self)
        .def(py::self -= py::self)
        .def(py::self * value_t())
        .def(value_t() * py::self)
        .def(py::self / value_t())
        .def("__copy__", [](const TTTensor& _t) { return TTTensor(_t); });
    m.def("dot", [](const TTTensor& _x, const TTTensor& _y) { return dot(_x, _y); });
    m.def("entrywise_product", py::overload_cast<const Tensor&, const Tensor&>(&entrywise_product));
    m.def("entrywise_product", py::overload_cast<const TTTensor&, const TTTensor&>(&entrywise_product));
    m.def("entrywise_product", py::overload_cast<const TTOperator&, const TTOperator&>(&entrywise_product));
    m.def("dyadic_product", py::overload_cast<const TTTensor&, const TTTensor&>(&dyadic_product));
    m.def("dyadic_product", py::overload_cast<const std::vector<TTTensor>&>(&dyadic_product));
    m.def("dyadic_product", py::overload_cast<const TTOperator&, const TTOperator&>(&dyadic_product));
    m.def("dyadic_product", py::overload_cast<const std::vector<TTOperator>&>(&dyadic_product));
    m.def("position_to_multiIndex", &Tensor::position_to_multiIndex);

    // ------------------------------------------------------------------ ALS (algorithms/als.h)
    py::class_<ALSVariant>(m, "ALSVariant")
        .def_readwrite("sites", &ALSVariant::sites)
        .def_readwrite("numHalfSweeps", &ALSVariant::numHalfSweeps)
        .def_readwrite("convergenceEpsilon", &ALSVariant::convergenceEpsilon)
        .def_readwrite("useResidualForEndCriterion", &ALSVariant::useResidualForEndCriterion)
        .def_readwrite("preserveCorePosition", &ALSVariant::preserveCorePosition)
        .def_readwrite("assumeSPD", &ALSVariant::assumeSPD)
        .def("__call__", [](const ALSVariant& _s, const TTOperator& _A, TTTensor& _x, const TTTensor& _b, value_t _eps) {
            return _s(_A, _x, _b, _eps);
        })
        .def("__call__", [](const ALSVariant& _s, const TTOperator& _A, TTTensor& _x, const TTTensor& _b, size_t _n) {
            return _s(_A, _x, _b, _n);
        })
        .def("__call__", [](const ALSVariant& _s, const TTOperator& _A, TTTensor& _x, const TTTensor& _b) { return _s(_A, _x, _b); })
        .def("__call__", [](const ALSVariant& _s, TTTensor& _x, const TTTensor& _b, value_t _eps) { return _s(_x, _b, _eps); })
        .def("__call__", [](const ALSVariant& _s, TTTensor& _x, const TTTensor& _b, size_t _n) { return _s(_x, _b, _n); })
        .def("__call__", [](const ALSVariant& _s, TTTensor& _x, const TTTensor& _b) { return _s(_x, _b); })
        .def("__copy__", [](const ALSVariant& _s) { return ALSVariant(_s); });
    m.attr("ALS") = py::cast(ALSVariant(ALS));
    m.attr("ALS_SPD") = py::cast(ALSVariant(ALS_SPD));
    m.attr("DMRG") = py::cast(ALSVariant(DMRG));
    m.attr("DMRG_SPD") = py::cast(ALSVariant(DMRG_SPD));
    m.attr("ASD") = py::cast(ALSVariant(ASD));
    m.attr("ASD_SPD") = py::cast(ALSVariant(ASD_SPD));

    // ------------------------------------------------------------------ measurements + ADF (measurments.h, algorithms/adf.h)
    py::class_<SinglePointMeasurementSet>(m, "SinglePointMeasurementSet")
        .def(py::init<>())
        .def(py::init<const SinglePointMeasurementSet&>())
        .def_readwrite("positions", &SinglePointMeasurementSet::positions)
        .def_readwrite("measuredValues", &SinglePointMeasurementSet::measuredValues)
        .def_static("random", [](size_t _n, const std::vector<size_t>& _dims) { return SinglePointMeasurementSet::random(_n, _dims); })
        .def_static("random", [](size_t _n, const Tensor& _t) { return SinglePointMeasurementSet::random(_n, _t); })
        .def_static("random", [](size_t _n, const TTTensor& _t) { return SinglePointMeasurementSet::random(_n, _t); })
        .def("size", &SinglePointMeasurementSet::size)
        .def("degree", &SinglePointMeasurementSet::degree)
        .def("frob_norm", &SinglePointMeasurementSet::frob_norm)
        .def("add", &SinglePointMeasurementSet::add)
        .def("sort", &SinglePointMeasurementSet::sort, py::arg("positionsOnly") = false)
        .def("measure", py::overload_cast<const Tensor&>(&SinglePointMeasurementSet::measure))
        .def("measure", py::overload_cast<const TTTensor&>(&SinglePointMeasurementSet::measure))
        .def("measure", py::overload_cast<const TensorNetwork&>(&SinglePointMeasurementSet::measure))
        .def("measure", py::overload_cast<std::function<value_t(const std::vector<size_t>&)>>(&SinglePointMeasurementSet::measure))
        .def("test", py::overload_cast<const Tensor&>(&SinglePointMeasurementSet::test, py::const_))
        .def("test", py::overload_cast<const TTTensor&>(&SinglePointMeasurementSet::test, py::const_))
        .def("test", py::overload_cast<const TensorNetwork&>(&SinglePointMeasurementSet::test, py::const_));
    py::class_<RankOneMeasurementSet>(m, "RankOneMeasurementSet")
        .def(py::init<>())
        .def(py::init<const RankOneMeasurementSet&>())
        .def(py::init<const SinglePointMeasurementSet&, const std::vector<size_t>&>())
        .def_readwrite("positions", &RankOneMeasurementSet::positions)
        .def_readwrite("measuredValues", &RankOneMeasurementSet::measuredValues)
        .def_static("random", [](size_t _n, const std::vector<size_t>& _dims) { return RankOneMeasurementSet::random(_n, _dims); })
        .def_static("random", [](size_t _n, const Tensor& _t) { return RankOneMeasurementSet::random(_n, _t); })
        .def_static("random", [](size_t _n, const TTTensor& _t) { return RankOneMeasurementSet::random(_n, _t); })
        .def("size", &RankOneMeasurementSet::size)
        .def("degree", &RankOneMeasurementSet::degree)
        .def("frob_norm", &RankOneMeasurementSet::frob_norm)
        .def("add", &RankOneMeasurementSet::add)
        .def("sort", &RankOneMeasurementSet::sort, py::arg("positionsOnly") = false)
        .def("normalize", &RankOneMeasurementSet::normalize)
        .def("measure", py::overload_cast<const Tensor&>(&RankOneMeasurementSet::measure))
        .def("measure", py::overload_cast<const TTTensor&>(&RankOneMeasurementSet::measure))
        .def("test", py::overload_cast<const Tensor&>(&RankOneMeasurementSet::test, py::const_))
        .def("test", py::overload_cast<const TTTensor&>(&RankOneMeasurementSet::test, py::const_));
    py::class_<ADFVariant>(m, "ADFVariant")
        .def(py::init<size_t, double, double>(), py::arg("maxIteration"), py::arg("targetResidual"), py::arg("minimalResidualDecrease"))
        .def_readwrite("maxIterations", &ADFVariant::maxIterations)
        .def_readwrite("targetResidualNorm", &ADFVariant::targetResidualNorm)
        .def_readwrite("minimalResidualNormDecrease", &ADFVariant::minimalResidualNormDecrease)
        .def("__call__", [](const ADFVariant& _v, TTTensor& _x, const SinglePointMeasurementSet& _m) { return _v(_x, _m); })
        .def("__call__", [](const ADFVariant& _v, TTTensor& _x, const RankOneMeasurementSet& _m) { return _v(_x, _m); })
        .def("__call__", [](const ADFVariant& _v, TTTensor& _x, const SinglePointMeasurementSet& _m, const std::vector<size_t>& _r) {
            return _v(_x, _m, _r);
        })
        .def("__call__", [](const ADFVariant& _v, TTTensor& _x, const RankOneMeasurementSet& _m, const std::vector<size_t>& _r) {
            return _v(_x, _m, _r);
        });
    m.attr("ADF") = py::cast(ADFVariant(ADF));
    m.def("solve", [](const Tensor& _A, const Tensor& _B, size_t _extra) {
        Tensor X;
        solve(X, _A, _B, _extra);
        return X;
    }, py::arg("A"), py::arg("B"), py::arg("extraDegree") = 0);
    m.def("solve_least_squares", [](const Tensor& _A, const Tensor& _B, size_t _extra) {
        Tensor X;
        solve_least_squares(X, _A, _B, _extra);
        return X;
    }, py::arg("A"), py::arg("B"), py::arg("extraDegree") = 0);

    // ------------------------------------------------------------------ TTOperator (TTNetwork<true>)
    py::class_<TTOperator>(m, "TTOperator")
        .def(py::init<>())
        .def(py::init<const TTOperator&>())
        .def(py::init([](const Tensor& _t, value_t _eps, size_t _maxRank) { return TTOperator(_t, _eps, _maxRank); }), py::arg("tensor"),
             py::arg("eps") = EPSILON, py::arg("maxRank") = std::numeric_limits<size_t>::max())
        .def(py::init([](const Tensor& _t, value_t _eps, const std::vector<size_t>& _maxRanks) { return TTOperator(_t, _eps, _maxRanks); }))
        .def(py::init([](const std::vector<size_t>& _dims) { return TTOperator(_dims); }))
        .def(py::init([](size_t _degree) { return TTOperator(_degree); }))
        .def_static("random", [](const std::vector<size_t>& _dims, const std::vector<size_t>& _ranks) { return TTOperator::random(_dims, _ranks); })
        .def_static("random", [](const std::vector<size_t>& _dims, size_t _rank) { return TTOperator::random(_dims, _rank); })
        .def_static("identity", &TTOperator::identity)
        .def_static("ones", &TTOperator::ones)
        .def_static("kronecker", &TTOperator::kronecker)
        .def_static("dirac", py::overload_cast<std::vector<size_t>, const std::vector<size_t>&>(&TTOperator::dirac))
        .def_static("dirac", py::overload_cast<std::vector<size_t>, const size_t>(&TTOperator::dirac))
        .def("fix_mode", &TTOperator::fix_mode)
        .def("resize_mode", &TTOperator::resize_mode, py::arg("mode"), py::arg("newDim"), py::arg("cutPos") = ~0ul)
        .def("chop", &TTOperator::chop)
        .def("require_correct_format", &TTOperator::require_correct_format)
        .def_readonly("dimensions", &TTOperator::dimensions)
        .def_readonly("canonicalized", &TTOperator::canonicalized)
        .def_readonly("corePosition", &TTOperator::corePosition)
        .def("degree", &TTOperator::degree)
        .def("ranks", &TTOperator::ranks)
        .def("rank", &TTOperator::rank)
        .def("get_component", &TTOperator::get_component)
        .def("set_component", &TTOperator::set_component)
        .def("move_core", &TTOperator::move_core, py::arg("position"), py::arg("keepRank") = false)
        .def("canonicalize_left", &TTOperator::canonicalize_left)
        .def("canonicalize_right", &TTOperator::canonicalize_right)
        .def("round", py::overload_cast<const std::vector<size_t>&, const double>(&TTOperator::round), py::arg("maxRanks"),
             py::arg("eps") = EPSILON)
        .def("round", py::overload_cast<const size_t>(&TTOperator::round))
        .def("round", py::overload_cast<const value_t>(&TTOperator::round))
        .def("frob_norm", &TTOperator::frob_norm)
        .def("transpose", &TTOperator::transpose)
        .def("__call__", [](TTOperator& _t, py::args _a) { return _t(to_indices(_a)); }, py::keep_alive<0, 1>())
        .def(py::self + py::self)
        .def(py::self - py::self)
        .def(py::self += py::self)
        .def(py::self -= py::self)
        .def(py::self * value_t())
        .def(value_t() * py::self)
        .def(py::self / value_t())
        .def("__copy__", [](const TTOperator& _t) { return TTOperator(_t); });

    // ------------------------------------------------------------------ generic TensorNetwork path of <x,y>
    // (contraction order of the reference's heuristics on the 2d+4-node network; host-only planning)
    m.def("tt_dot_contraction_order", [](const std::vector<size_t>& _n, const std::vector<size_t>& _rx, const std::vector<size_t>& _ry) {
        return internal::greedy_contraction_order(internal::tt_pair_network(_n, _rx, _ry));
    });
    // value_t(x(i&0) * y(i&0)) contracted as a generic TensorNetwork (heuristic order, permutation + GEMM per
    // pair on the GPU) instead of the TT zipper
    m.def("tt_dot_network", [](const TTTensor& _x, const TTTensor& _y) {
        XERUS_REQUIRE(_x.dimensions == _y.dimensions, "dot of TTs with different dimensions");
        const size_t d = _x.degree();
        std::vector<size_t> rx(d + 1, 1), ry(d + 1, 1);
        for (size_t k = 0; k < d; ++k) {
            rx[k + 1] = _x.components[k].dimensions[2];
            ry[k + 1] = _y.components[k].dimensions[2];
        }
        TensorNetwork net = internal::tt_pair_network(_x.dimensions, rx, ry, &_x, &_y);
        std::set<size_t> all;
        for (size_t i = 0; i < net.nodes.size(); ++i) all.insert(i);
        const size_t res = net.contract(all);
        return (*net.nodes[res].tensorObject)[0];
    });
}
