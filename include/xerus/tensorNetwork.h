// TensorNetwork: graph of tensors connected by links (reference include/xerus/tensorNetwork.h:50-574).
// Used by the indexed-expression engine; pairwise contraction = (at most one) permutation + one GEMM on
// the GPU (tensorNetwork.cpp:1037-1229), multi-node contraction order from the reference's greedy
// heuristics with cost m*n*r (contractionHeuristic.cpp:35-381).
#pragma once
#include <memory>
#include <set>
#include <vector>

#include "tensor.h"

namespace xerus {

class TensorNetwork;

/// T(i,j,...) = A(...) * B(...) for a TensorNetwork T: the product kept as a network (no contraction), its
/// external modes in the order of T's indices (the reference's IndexedTensor<TensorNetwork> assignment,
/// indexedTensorWritable.cpp:68-119 with tensorNetwork.cpp:224-296).
struct IndexedNetwork {
    TensorNetwork* network;
    std::vector<Index> indices;
    IndexedNetwork& operator=(const IndexedProduct& _rhs);
    IndexedNetwork& operator=(const IndexedTensor<Tensor>& _rhs);
};

class TensorNetwork {
   public:
    struct Link {
        size_t other;           // node id, or (for external links) the external index position
        size_t indexPosition;   // position of the mode in the other node (or external slot)
        size_t dimension;
        bool external;
        Link() = default;
        Link(size_t _other, size_t _indexPos, size_t _dim, bool _external)
            : other(_other), indexPosition(_indexPos), dimension(_dim), external(_external) {}
        bool links(size_t _other) const { return !external && other == _other; }
    };
    struct TensorNode {
        std::unique_ptr<Tensor> tensorObject;
        std::vector<Link> neighbors;
        bool erased = false;
        TensorNode() = default;
        TensorNode(std::unique_ptr<Tensor>&& _t, std::vector<Link> _n) : tensorObject(std::move(_t)), neighbors(std::move(_n)) {}
        TensorNode(const TensorNode& _o)
            : tensorObject(_o.tensorObject ? new Tensor(*_o.tensorObject) : nullptr), neighbors(_o.neighbors), erased(_o.erased) {}
        TensorNode(TensorNode&&) = default;
        TensorNode& operator=(const TensorNode& _o) {
            tensorObject.reset(_o.tensorObject ? new Tensor(*_o.tensorObject) : nullptr);
            neighbors = _o.neighbors;
            erased = _o.erased;
            return *this;
        }
        TensorNode& operator=(TensorNode&&) = default;
        size_t degree() const { return neighbors.size(); }
    };

    std::vector<size_t> dimensions;        // external dimensions
    std::vector<TensorNode> nodes;
    std::vector<Link> externalLinks;       // external slot -> (node, mode)

    TensorNetwork();
    explicit TensorNetwork(Tensor _tensor);
    /// an empty graph (no nodes, no tensors): structural copies for contraction planning
    struct Structure {};
    explicit TensorNetwork(Structure) {}
    TensorNetwork(const TensorNetwork&) = default;
    TensorNetwork(TensorNetwork&&) = default;
    TensorNetwork& operator=(const TensorNetwork&) = default;
    TensorNetwork& operator=(TensorNetwork&&) = default;

    size_t degree() const { return dimensions.size(); }
    size_t num_nodes() const;
    /// Contracts nodes id1 and id2 into id1 (id2 erased); GPU permutation + GEMM.
    void contract(const size_t _nodeId1, const size_t _nodeId2);
    /// Contracts a set of nodes (greedy heuristics for > 3 nodes) and returns the remaining node id.
    size_t contract(const std::set<size_t>& _ids);
    /// Full contraction to a dense tensor in external-index order.
    Tensor to_tensor() const;
    value_t frob_norm() const;
    /// Estimated flops (m*n*r) of contracting everything in the heuristic's order.
    double contraction_cost(const std::set<size_t>& _ids) const;

    /// Entry at a flat / multi index (tensorNetwork.cpp:310-370): every node's external modes are fixed to the
    /// position (Tensor::fix_mode on the GPU), the remaining network is contracted to a scalar.
    value_t operator[](const size_t _position) const;
    value_t operator[](const std::vector<size_t>& _positions) const;

    IndexedNetwork operator()(const std::vector<Index>& _indices) { return IndexedNetwork{this, _indices}; }
    template <class... args>
    IndexedNetwork operator()(args... _args) { return IndexedNetwork{this, std::vector<Index>{_args...}}; }

    void require_valid_network() const;
    void sanitize();   // drop erased nodes, renumber
};

class TTTensor;

namespace internal {
/// the network of a product with its externals in the order of _out (IndexedNetwork's assignment)
TensorNetwork product_network(const IndexedProduct& _p, const std::vector<Index>& _out);
/// best greedy contraction order over the reference's five score functions (contractionHeuristic.cpp)
std::vector<std::pair<size_t, size_t>> greedy_contraction_order(const TensorNetwork& _net, double* _cost = nullptr);
/// the 2d+4-node network of value_t(x(i&0) * y(i&0)) in the reference's numbering (x: ghost 0, cores
/// 1..d, ghost d+1; y: the same + d+2); with null TTs the nodes carry no data (order planning only)
TensorNetwork tt_pair_network(const std::vector<size_t>& _n, const std::vector<size_t>& _rx, const std::vector<size_t>& _ry,
                              const TTTensor* _x = nullptr, const TTTensor* _y = nullptr);
}  // namespace internal

}  // namespace xerus
