// xerus data files for Tensor, TensorNetwork and TTTensor (misc/fileIO.h:103-163).
//
// Header line "Xerus <demangled type> datafile." + "Format: Binary" / "Format: TSV", then the object's
// stream (every scalar raw in BINARY, "value\t" in TSV; vectors as size + elements):
//   Tensor        (tensor.cpp:1781-1845):        version 1, dims, representation 1 (dense), values
//   TensorNetwork (tensorNetwork.cpp:1429-1466): version 1, dims, external links (other, indexPosition,
//                  dimension), node count, per node its links (external, other, indexPosition, dimension),
//                  then every node's Tensor
//   TTNetwork     (ttNetwork.cpp:1455-1487):     version 1, canonicalized, corePosition, TensorNetwork
// A TTTensor is written with the reference's node layout (ghost ones({1}) node 0, components 1..d, ghost
// node d+1, ttNetwork.cpp:57-108), so files interchange with the reference in both directions. Device data
// crosses PCIe only here (explicit host boundary). Sparse payloads (representation 2, the reference's files of
// sparse tensors) are read into dense tensors; files are written dense (the build is dense-only).
#include <cstdint>
#include <fstream>
#include <iomanip>
#include <limits>
#include <sstream>

#include "xerus.h"

namespace xerus {
namespace misc {

namespace {

constexpr size_t kExternal = ~size_t(0);   // Link::other of an external link (the reference's -1)

const char* type_name(int kind) {
    switch (kind) {
        case 0: return "xerus::Tensor";
        case 1: return "xerus::TensorNetwork";
        default: return "xerus::TTNetwork<false>";
    }
}

struct Writer {
    std::ostream& s;
    FileFormat f;
    template <class T>
    void put(const T& v) {
        if (f == FileFormat::TSV) s << v << '\t';
        else s.write(reinterpret_cast<const char*>(&v), std::streamsize(sizeof(T)));
    }
    void put_dims(const std::vector<size_t>& v) {
        put<size_t>(v.size());
        for (size_t x : v) put<size_t>(x);
    }
    void nl(const char* t = "\n") {
        if (f == FileFormat::TSV) s << t;
    }
    void tensor(const Tensor& t) {
        put<size_t>(1);
        put_dims(t.dimensions);
        put<size_t>(1);   // dense
        const std::vector<value_t> v = t.to_host();
        if (f == FileFormat::TSV)
            for (value_t x : v) s << x << '\t';
        else s.write(reinterpret_cast<const char*>(v.data()), std::streamsize(v.size() * sizeof(value_t)));
    }
};

struct Reader {
    std::istream& s;
    FileFormat f;
    template <class T>
    T get() {
        T v{};
        if (f == FileFormat::TSV) s >> v;
        else s.read(reinterpret_cast<char*>(&v), sizeof(T));
        XERUS_REQUIRE(s, "Unexpected end of stream.");
        return v;
    }
    std::vector<size_t> get_dims() {
        const size_t count = get<size_t>();
        XERUS_REQUIRE(count <= 4096, "Malformed stream: " << count << " dimensions");
        std::vector<size_t> v(count);
        for (size_t& x : v) x = get<size_t>();
        return v;
    }
    Tensor tensor() {
        const size_t ver = get<size_t>();
        XERUS_REQUIRE(ver == 1, "Unknown stream version to open (" << ver << ")");
        Tensor::DimensionTuple dims = get_dims();
        const size_t rep = get<size_t>();
        XERUS_REQUIRE(rep == 1 || rep == 2, "Unknown tensor representation " << rep << " in stream");
        // a malformed size must not wrap: check every product, and (binary) that the payload is in the stream
        size_t n = 1;
        for (size_t d : dims) {
            XERUS_REQUIRE(d == 0 || n <= (std::numeric_limits<size_t>::max() / sizeof(value_t)) / d,
                          "Malformed stream: the tensor size overflows");
            n *= d;
        }
        if (rep == 2) {
            // sparse payload (tensor.cpp:1796-1803 / 1826-1840): entry count, then (flat position, value) pairs
            // with the factor applied; read into a dense tensor (this build's only representation)
            const size_t num = get<size_t>();
            XERUS_REQUIRE(num <= n, "Malformed stream: " << num << " sparse entries for " << n << " positions");
            std::unique_ptr<value_t[]> data(new value_t[std::max<size_t>(n, 1)]());
            for (size_t i = 0; i < num; ++i) {
                const size_t pos = get<size_t>();
                const value_t val = get<value_t>();
                XERUS_REQUIRE(pos < n, "Malformed stream: sparse position " << pos << " beyond " << n);
                data[pos] = val;
            }
            return Tensor(std::move(dims), std::move(data));
        }
        if (f != FileFormat::TSV) {
            const std::streampos here = s.tellg();
            if (here != std::streampos(-1)) {
                s.seekg(0, std::ios::end);
                const std::streampos end = s.tellg();
                s.seekg(here);
                XERUS_REQUIRE(end != std::streampos(-1) && size_t(end - here) >= n * sizeof(value_t),
                              "Malformed stream: " << n << " entries announced, fewer in the stream");
            }
        }
        std::unique_ptr<value_t[]> data(new value_t[std::max<size_t>(n, 1)]);
        if (f == FileFormat::TSV)
            for (size_t i = 0; i < n; ++i) s >> data[i];
        else s.read(reinterpret_cast<char*>(data.get()), std::streamsize(n * sizeof(value_t)));
        XERUS_REQUIRE(s, "Unexpected end of stream in reading dense Tensor.");
        return Tensor(std::move(dims), std::move(data));
    }
};

void write_network(Writer& w, const TensorNetwork& net) {
    w.put<size_t>(1);
    w.put_dims(net.dimensions);
    w.nl();
    for (const TensorNetwork::Link& el : net.externalLinks) {
        w.put<size_t>(el.other);
        w.put<size_t>(el.indexPosition);
        w.put<size_t>(el.dimension);
    }
    w.nl("\n\n");
    w.put<size_t>(net.nodes.size());
    w.nl();
    for (const TensorNetwork::TensorNode& node : net.nodes) {
        w.put<size_t>(node.neighbors.size());
        for (const TensorNetwork::Link& l : node.neighbors) {
            w.put<bool>(l.external);
            w.put<size_t>(l.external ? kExternal : l.other);
            w.put<size_t>(l.indexPosition);
            w.put<size_t>(l.dimension);
        }
    }
    w.nl();
    for (const TensorNetwork::TensorNode& node : net.nodes) {
        XERUS_REQUIRE(node.tensorObject, "cannot save a network node without data");
        w.tensor(*node.tensorObject);
        w.nl();
    }
}

TensorNetwork read_network(Reader& r) {
    const size_t ver = r.get<size_t>();
    XERUS_REQUIRE(ver == 1, "Unknown stream version to open (" << ver << ")");
    TensorNetwork net{TensorNetwork::Structure{}};
    net.dimensions = r.get_dims();
    for (size_t i = 0; i < net.dimensions.size(); ++i) {
        const size_t other = r.get<size_t>(), pos = r.get<size_t>(), dim = r.get<size_t>();
        net.externalLinks.emplace_back(other, pos, dim, false);
    }
    net.nodes.resize(r.get<size_t>());
    for (auto& node : net.nodes) {
        node.neighbors.resize(r.get<size_t>());
        for (auto& l : node.neighbors) {
            l.external = r.get<bool>();
            l.other = r.get<size_t>();
            l.indexPosition = r.get<size_t>();
            l.dimension = r.get<size_t>();
        }
    }
    for (auto& node : net.nodes) node.tensorObject.reset(new Tensor(r.tensor()));
    net.require_valid_network();
    return net;
}

// the reference's TTNetwork<false> node layout around the components
TensorNetwork tt_network(const TTTensor& tt) {
    const size_t d = tt.degree();
    TensorNetwork net{TensorNetwork::Structure{}};
    net.dimensions = tt.dimensions;
    if (d == 0) {
        net.nodes.emplace_back(std::unique_ptr<Tensor>(new Tensor(tt.components[0])), std::vector<TensorNetwork::Link>());
        return net;
    }
    for (size_t i = 0; i < d; ++i) net.externalLinks.emplace_back(i + 1, 1, tt.dimensions[i], false);
    net.nodes.emplace_back(std::unique_ptr<Tensor>(new Tensor(Tensor::ones({1}))),
                           std::vector<TensorNetwork::Link>{TensorNetwork::Link(1, 0, 1, false)});
    for (size_t i = 0; i < d; ++i) {
        const Tensor& c = tt.components[i];
        std::vector<TensorNetwork::Link> nb{TensorNetwork::Link(i, i == 0 ? 0 : 2, c.dimensions[0], false),
                                            TensorNetwork::Link(kExternal, i, c.dimensions[1], true),
                                            TensorNetwork::Link(i + 2, 0, c.dimensions[2], false)};
        net.nodes.emplace_back(std::unique_ptr<Tensor>(new Tensor(c)), std::move(nb));
    }
    net.nodes.emplace_back(std::unique_ptr<Tensor>(new Tensor(Tensor::ones({1}))),
                           std::vector<TensorNetwork::Link>{TensorNetwork::Link(d, 2, 1, false)});
    return net;
}

TTTensor tt_from_network(TensorNetwork&& net, bool canonicalized, size_t corePosition) {
    const size_t d = net.dimensions.size();
    TTTensor tt(d);
    if (d == 0) {
        XERUS_REQUIRE(net.nodes.size() == 1, "a degree-0 TT file holds one node");
        tt.components[0] = *net.nodes[0].tensorObject;
        return tt;
    }
    XERUS_REQUIRE(net.nodes.size() == d + 2, "not a TTTensor file: " << net.nodes.size() << " nodes for degree " << d);
    for (size_t i = 0; i < d; ++i) {
        const Tensor& c = *net.nodes[i + 1].tensorObject;
        XERUS_REQUIRE(c.degree() == 3, "Component " << i << " must have degree 3");
        tt.set_component(i, c);
    }
    // the ghost nodes are ones({1}) in the reference; fold any other scalar into the first component
    const value_t g = (*net.nodes[0].tensorObject)[0] * (*net.nodes[d + 1].tensorObject)[0];
    if (g != 1.0) tt.components[0] *= g;
    tt.require_correct_format();
    tt.canonicalized = canonicalized;
    tt.corePosition = corePosition;
    XERUS_REQUIRE(!canonicalized || corePosition < d, "Invalid core position " << corePosition);
    return tt;
}

template <class F>
void write_file(const std::string& _filename, int kind, FileFormat _format, F&& body) {
    std::ofstream out(_filename, std::ios::binary);
    XERUS_REQUIRE(out.good(), "cannot open " << _filename);
    out << "Xerus " << type_name(kind) << " datafile.\nFormat: " << (_format == FileFormat::TSV ? "TSV" : "Binary") << "\n";
    if (_format == FileFormat::TSV) out << std::setprecision(std::numeric_limits<value_t>::digits10 + 1);
    Writer w{out, _format};
    body(w);
    XERUS_REQUIRE(out.good(), "error occured while writing to file " << _filename);
}

// opens the file, checks the header type, returns the reader positioned after "Format: ...\n"
struct FileIn {
    std::ifstream in;
    FileFormat format;
    std::string type;
};

FileIn open_file(const std::string& _filename) {
    FileIn f;
    f.in.open(_filename, std::ios::binary);
    XERUS_REQUIRE(f.in.good(), "cannot open " << _filename);
    std::string l1, l2;
    std::getline(f.in, l1);
    std::getline(f.in, l2);
    const std::string pre = "Xerus ", post = " datafile.";
    XERUS_REQUIRE(l1.size() > pre.size() + post.size() && l1.compare(0, pre.size(), pre) == 0 &&
                      l1.compare(l1.size() - post.size(), post.size(), post) == 0,
                  "Invalid input file " << _filename << ". DBG: " << l1);
    f.type = l1.substr(pre.size(), l1.size() - pre.size() - post.size());
    XERUS_REQUIRE(l2 == "Format: Binary" || l2 == "Format: TSV", "Invalid Sytax detected in file " << _filename << ". DBG: " << l2);
    f.format = l2 == "Format: TSV" ? FileFormat::TSV : FileFormat::BINARY;
    return f;
}

}  // namespace

void save_to_file(const Tensor& _tensor, const std::string& _filename, const FileFormat _format) {
    write_file(_filename, 0, _format, [&](Writer& w) { w.tensor(_tensor); });
}

void save_to_file(const TensorNetwork& _network, const std::string& _filename, const FileFormat _format) {
    write_file(_filename, 1, _format, [&](Writer& w) { write_network(w, _network); });
}

void save_to_file(const TTTensor& _tt, const std::string& _filename, const FileFormat _format) {
    _tt.require_correct_format();
    write_file(_filename, 2, _format, [&](Writer& w) {
        w.put<size_t>(1);
        w.put<bool>(_tt.canonicalized);
        w.put<size_t>(_tt.corePosition);
        write_network(w, tt_network(_tt));
    });
}

std::string file_type(const std::string& _filename) { return open_file(_filename).type; }

Tensor load_tensor_from_file(const std::string& _filename) {
    FileIn f = open_file(_filename);
    XERUS_REQUIRE(f.type == type_name(0), "Invalid binary input file " << _filename << ": holds a " << f.type);
    Reader r{f.in, f.format};
    return r.tensor();
}

TensorNetwork load_network_from_file(const std::string& _filename) {
    FileIn f = open_file(_filename);
    XERUS_REQUIRE(f.type == type_name(1), "Invalid binary input file " << _filename << ": holds a " << f.type);
    Reader r{f.in, f.format};
    return read_network(r);
}

TTTensor load_tt_from_file(const std::string& _filename) {
    FileIn f = open_file(_filename);
    XERUS_REQUIRE(f.type == type_name(2), "Invalid binary input file " << _filename << ": holds a " << f.type);
    Reader r{f.in, f.format};
    const size_t ver = r.get<size_t>();
    XERUS_REQUIRE(ver == 1, "Unknown stream version to open (" << ver << ")");
    const bool canon = r.get<bool>();
    const size_t core = r.get<size_t>();
    return tt_from_network(read_network(r), canon, core);
}

}  // namespace misc
}  // namespace xerus
