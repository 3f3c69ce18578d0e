// TensorNetwork: node graph + pairwise GPU contraction + the reference's contraction-order heuristics.
//
// Pairwise contraction (tensorNetwork.cpp:1037-1229): the common modes of both nodes are brought to
// adjacent blocks with at most one permutation (LDS-tiled permute kernel) and the product is a single
// GEMM whose transpose flags absorb every other layout; the open modes keep their relative order
// (node 1's, then node 2's). Multi-node order (tensorNetwork.cpp:1253-1333): 2 nodes direct, 3 nodes the
// closed-form cost comparison, more nodes the best of the five greedy scores plus the exchange
// heuristic (contractionHeuristic.cpp:35-381), cost model m*n*r.
#include <algorithm>
#include <functional>
#include <limits>
#include <tuple>

#include "xerus.h"

namespace xerus {

using Link = TensorNetwork::Link;
using TensorNode = TensorNetwork::TensorNode;

static constexpr size_t NO_NODE = ~size_t(0);

static double node_size(const TensorNode& _n) {
    double s = 1;
    for (const Link& l : _n.neighbors) s *= double(l.dimension);
    return s;
}

TensorNetwork::TensorNetwork() {
    nodes.emplace_back(std::unique_ptr<Tensor>(new Tensor()), std::vector<Link>());
}

TensorNetwork::TensorNetwork(Tensor _tensor) : dimensions(_tensor.dimensions) {
    std::vector<Link> links;
    for (size_t d = 0; d < dimensions.size(); ++d) {
        externalLinks.emplace_back(0, d, dimensions[d], false);
        links.emplace_back(NO_NODE, d, dimensions[d], true);
    }
    nodes.emplace_back(std::unique_ptr<Tensor>(new Tensor(std::move(_tensor))), std::move(links));
}

size_t TensorNetwork::num_nodes() const {
    size_t n = 0;
    for (const auto& node : nodes) n += node.erased ? 0 : 1;
    return n;
}

void TensorNetwork::require_valid_network() const {
    XERUS_REQUIRE(externalLinks.size() == dimensions.size(), "externalLinks.size() != dimensions.size()");
    XERUS_REQUIRE(!nodes.empty(), "There must always be at least one node!");
    for (size_t n = 0; n < externalLinks.size(); ++n) {
        const Link& el = externalLinks[n];
        XERUS_REQUIRE(el.other < nodes.size(), "External link " << n << " is inconsistent");
        XERUS_REQUIRE(el.dimension == dimensions[n], "External link " << n << " has a wrong dimension");
        const TensorNode& node = nodes[el.other];
        XERUS_REQUIRE(el.indexPosition < node.degree(), "External link " << n << " points to a missing mode");
        const Link& back = node.neighbors[el.indexPosition];
        XERUS_REQUIRE(back.external && back.indexPosition == n && back.dimension == el.dimension,
                      "External link " << n << " is not mirrored by its node");
    }
    for (size_t n = 0; n < nodes.size(); ++n) {
        const TensorNode& node = nodes[n];
        if (node.erased) continue;
        if (node.tensorObject)
            XERUS_REQUIRE(node.degree() == node.tensorObject->degree(), "Node " << n << " has a wrong number of links");
        for (size_t i = 0; i < node.neighbors.size(); ++i) {
            const Link& l = node.neighbors[i];
            if (node.tensorObject) XERUS_REQUIRE(l.dimension == node.tensorObject->dimensions[i], "n=" << n << " i=" << i);
            if (l.external) continue;
            XERUS_REQUIRE(l.other < nodes.size() && !nodes[l.other].erased, "Link from node " << n << " to a missing node");
            const TensorNode& other = nodes[l.other];
            XERUS_REQUIRE(l.indexPosition < other.degree(), "Link from node " << n << " to a missing mode");
            const Link& back = other.neighbors[l.indexPosition];
            XERUS_REQUIRE(!back.external && back.other == n && back.indexPosition == i && back.dimension == l.dimension,
                          "Link from node " << n << " mode " << i << " is not mirrored");
        }
    }
}

void TensorNetwork::sanitize() {
    std::vector<size_t> idMap(nodes.size(), NO_NODE);
    size_t newId = 0;
    for (size_t oldId = 0; oldId < nodes.size(); ++oldId) {
        if (nodes[oldId].erased) continue;
        idMap[oldId] = newId;
        if (newId != oldId) std::swap(nodes[newId], nodes[oldId]);
        ++newId;
    }
    nodes.resize(newId);
    for (TensorNode& n : nodes)
        for (Link& l : n.neighbors)
            if (!l.external) l.other = idMap[l.other];
    for (Link& l : externalLinks) l.other = idMap[l.other];
}

// self-links (traces) of one node: GPU trace over both modes, then relink (tensorNetwork.cpp:222-255)
static void perform_traces(TensorNetwork& _net, size_t _id) {
    TensorNode& node = _net.nodes[_id];
    for (size_t i = 0; i < node.degree(); ++i) {
        const Link link = node.neighbors[i];
        if (link.external || link.other != _id) continue;
        const size_t j = link.indexPosition;   // j > i as i is the first occurrence
        if (node.tensorObject) node.tensorObject->perform_trace(i, j);
        node.neighbors.erase(node.neighbors.begin() + long(j));
        node.neighbors.erase(node.neighbors.begin() + long(i));
        for (size_t k = 0; k < node.degree(); ++k) {
            const Link& l = node.neighbors[k];
            if (l.external) _net.externalLinks[l.indexPosition].indexPosition = k;
            else _net.nodes[l.other].neighbors[l.indexPosition].indexPosition = k;
        }
        i = size_t(-1);   // restart: positions changed
    }
}

void TensorNetwork::contract(const size_t _nodeId1, const size_t _nodeId2) {
    XERUS_REQUIRE(_nodeId1 < nodes.size() && !nodes[_nodeId1].erased, "It appears node1 = " << _nodeId1 << " was already contracted?");
    XERUS_REQUIRE(_nodeId2 < nodes.size() && !nodes[_nodeId2].erased, "It appears node2 = " << _nodeId2 << " was already contracted?");
    XERUS_REQUIRE(_nodeId1 != _nodeId2, "cannot contract a node with itself");
    TensorNode& n1 = nodes[_nodeId1];
    TensorNode& n2 = nodes[_nodeId2];
    auto to2 = [&](const Link& l) { return !l.external && l.other == _nodeId2; };
    auto to1 = [&](const Link& l) { return !l.external && l.other == _nodeId1; };

    std::vector<Link> newLinks;
    size_t common = 0;
    for (const Link& l : n1.neighbors) {
        if (to2(l)) ++common;
        else newLinks.push_back(l);
    }
    for (const Link& l : n2.neighbors)
        if (!to1(l)) newLinks.push_back(l);

    if (n1.tensorObject) {
        XERUS_REQUIRE(n2.tensorObject, "cannot contract a stripped node with a full one");
        // common modes a prefix or suffix of the mode list (the reference's "at most one switch")
        auto separated = [&](const TensorNode& n, const std::function<bool(const Link&)>& isCommon) {
            if (n.degree() <= 1 || common == 0) return true;
            size_t switches = 0;
            bool prev = isCommon(n.neighbors[0]);
            for (const Link& l : n.neighbors) {
                if (isCommon(l) != prev) {
                    ++switches;
                    prev = !prev;
                }
            }
            return switches < 2;
        };
        bool sep1 = separated(n1, to2);
        bool sep2 = separated(n2, to1);
        bool matching = true;   // node 2 visits the common modes in node 1's order
        {
            size_t last = 0;
            bool first = true;
            for (const Link& l : n2.neighbors) {
                if (!to1(l)) continue;
                if (!first && l.indexPosition < last) matching = false;
                last = l.indexPosition;
                first = false;
            }
        }
        if (!matching && sep1 && sep2) {
            if (n1.tensorObject->size < n2.tensorObject->size) sep1 = false;
            else sep2 = false;
        }
        if (!sep1) {   // node 1 -> (open..., common in node 2's order)
            std::vector<size_t> shuffle(n1.degree());
            size_t pos = 0;
            for (size_t d = 0; d < n1.degree(); ++d)
                if (!to2(n1.neighbors[d])) shuffle[d] = pos++;
            for (const Link& l : n2.neighbors)
                if (to1(l)) shuffle[l.indexPosition] = pos++;
            reshuffle(*n1.tensorObject, Tensor(*n1.tensorObject), shuffle);
            matching = true;
        }
        if (!sep2) {   // node 2 -> (common..., open...)
            std::vector<size_t> shuffle(n2.degree());
            size_t pos = 0;
            if (matching) {
                for (size_t d = 0; d < n2.degree(); ++d)
                    if (to1(n2.neighbors[d])) shuffle[d] = pos++;
            } else {
                for (const Link& l : n1.neighbors)
                    if (to2(l)) shuffle[l.indexPosition] = pos++;
            }
            for (size_t d = 0; d < n2.degree(); ++d)
                if (!to1(n2.neighbors[d])) shuffle[d] = pos++;
            reshuffle(*n2.tensorObject, Tensor(*n2.tensorObject), shuffle);
        }
        const bool trans1 = sep1 && !n1.neighbors.empty() && to2(n1.neighbors[0]);
        const bool trans2 = sep2 && !n2.neighbors.empty() && !to1(n2.neighbors[0]);
        Tensor result;
        xerus::contract(result, *n1.tensorObject, trans1, *n2.tensorObject, trans2, common);
        *n1.tensorObject = std::move(result);
    }

    n1.neighbors = std::move(newLinks);
    n2.erased = true;
    n2.tensorObject.reset();
    n2.neighbors.clear();
    for (size_t d = 0; d < n1.neighbors.size(); ++d) {
        const Link& l = n1.neighbors[d];
        if (l.external) {
            externalLinks[l.indexPosition].other = _nodeId1;
            externalLinks[l.indexPosition].indexPosition = d;
        } else {
            nodes[l.other].neighbors[l.indexPosition].other = _nodeId1;
            nodes[l.other].neighbors[l.indexPosition].indexPosition = d;
        }
    }
}

namespace internal {

static double contraction_cost(double _m, double _n, double _r) { return _m * _n * _r; }

// pair cost as TensorNetwork::contraction_cost(id1, id2) (tensorNetwork.cpp:1232-1250)
static double pair_cost(const TensorNetwork& _net, size_t _a, size_t _b) {
    double cost = node_size(_net.nodes[_a]);
    for (const Link& l : _net.nodes[_b].neighbors)
        if (l.external || l.other != _a) cost *= double(l.dimension);
    return cost;
}

using Order = std::vector<std::pair<size_t, size_t>>;

template <double (*score)(double, double, double)>
static void greedy_heuristic(double& _bestCost, Order& _order, TensorNetwork _net) {
    double numNodes = 0, numEdges = 0;
    for (const auto& n : _net.nodes)
        if (!n.erased) {
            numNodes += 1;
            numEdges += double(n.degree());
        }
    if (_bestCost < 2 * 2 * numNodes * numEdges) return;
    double ourCost = 0, finalCost = 0, bestScore;
    Order ours;
    size_t best1 = 0, best2 = 0;
    do {
        bestScore = std::numeric_limits<double>::max();
        for (size_t i = 0; i < _net.nodes.size(); ++i) {
            if (_net.nodes[i].erased) continue;
            const TensorNode& ni = _net.nodes[i];
            for (size_t j = i + 1; j < _net.nodes.size(); ++j) {
                if (_net.nodes[j].erased) continue;
                const TensorNode& nj = _net.nodes[j];
                double m = 1, n = 1, r = 1;
                for (const Link& l : ni.neighbors) {
                    if (!l.external && l.other == j) r *= double(l.dimension);
                    else m *= double(l.dimension);
                }
                for (const Link& l : nj.neighbors)
                    if (l.external || l.other != i) n *= double(l.dimension);
                const double s = score(m, n, r);
                if (s < bestScore) {
                    bestScore = s;
                    ourCost = contraction_cost(m, n, r);
                    best1 = i;
                    best2 = j;
                }
            }
        }
        if (bestScore < std::numeric_limits<double>::max()) {
            finalCost += ourCost;
            if (finalCost > _bestCost) return;
            ours.emplace_back(best1, best2);
            _net.contract(best1, best2);
        }
    } while (bestScore < std::numeric_limits<double>::max());
    if (finalCost < _bestCost) {
        _bestCost = finalCost;
        _order = std::move(ours);
    }
}

static double score_size(double m, double n, double r) { return n * m - (n + m) * r; }
static double score_mn(double m, double n, double) { return m * n; }
static double score_speed(double m, double n, double r) { return (n * m - (n + m) * r) / (n * m * r); }
static double score_big_tensor(double m, double n, double r) {
    if (n * m < (n + m) * r) return -1e10 + n * m * r;
    return n * m - (n + m) * r;
}
static double score_littlestep(double m, double n, double r) {
    if (n * m < (n + m) * r) return -std::max(n, m) * r;
    return n * m - (n + m) * r;
}

// which two of three nodes to contract first (contractionHeuristic.cpp:138-177)
static std::tuple<size_t, size_t, size_t, double> best_of_three(const TensorNetwork& _net, size_t _a, size_t _b, size_t _c) {
    double sa = 1, sb = 1, sc = 1, sab = 1, sbc = 1, sac = 1;
    auto links = [](const Link& l, size_t id) { return !l.external && l.other == id; };
    for (const Link& l : _net.nodes[_a].neighbors) {
        if (links(l, _b)) sab *= double(l.dimension);
        else if (links(l, _c)) sac *= double(l.dimension);
        else sa *= double(l.dimension);
    }
    for (const Link& l : _net.nodes[_b].neighbors) {
        if (links(l, _c)) sbc *= double(l.dimension);
        else if (!links(l, _a)) sb *= double(l.dimension);
    }
    for (const Link& l : _net.nodes[_c].neighbors)
        if (!links(l, _a) && !links(l, _b)) sc *= double(l.dimension);
    const double costAB = sa * sb * sac * sbc * (sab + sc);
    const double costAC = sa * sc * sab * sbc * (sac + sb);
    const double costBC = sb * sc * sab * sac * (sbc + sa);
    if (costAB < costAC && costAB < costBC) return std::make_tuple(_a, _b, _c, sa * sb * sac * sbc * sab);
    if (costAC < costBC) return std::make_tuple(_a, _c, _b, sa * sc * sab * sbc * sac);
    return std::make_tuple(_b, _c, _a, sb * sc * sab * sac * sbc);
}

// re-pair consecutive steps of the best order found so far (contractionHeuristic.cpp:278-369)
static void exchange_heuristic(double& _bestCost, Order& _order, TensorNetwork _net) {
    if (_order.empty()) return;
    const TensorNetwork copy(_net);
    double numEdges = 0;
    for (const auto& n : _net.nodes)
        if (!n.erased) numEdges += double(n.degree());
    const double heuristicCost = 3 * numEdges;
    if (_bestCost < 2 * heuristicCost) return;

    Order openPairs{_order.front()};
    double finalCost = 0;
    Order ours;
    std::vector<size_t> idMap(_net.nodes.size());
    for (size_t i = 0; i < idMap.size(); ++i) idMap[i] = i;
    auto root = [&](size_t id) {
        while (id != idMap[id]) id = idMap[id];
        return id;
    };
    for (size_t i = 1; i < _order.size(); ++i) {
        std::pair<size_t, size_t> next(root(_order[i].first), root(_order[i].second));
        Order newOpen;
        for (const auto& p : openPairs) {
            const size_t id1 = root(p.first), id2 = root(p.second);
            const bool firstIn = next.first == id1 || next.first == id2;
            const bool secondIn = next.second == id1 || next.second == id2;
            if (!firstIn && !secondIn) {
                newOpen.emplace_back(id1, id2);
                continue;
            }
            XERUS_REQUIRE(!(firstIn && secondIn), "internal error in exchange heuristic");
            const size_t third = firstIn ? next.second : next.first;
            const auto c = best_of_three(_net, id1, id2, third);
            const size_t a = std::get<0>(c), b = std::get<1>(c);
            idMap[b] = a;
            finalCost += std::get<3>(c);
            ours.emplace_back(a, b);
            _net.contract(a, b);
            next = {a, std::get<2>(c)};
        }
        newOpen.push_back(next);
        openPairs = std::move(newOpen);
    }
    XERUS_REQUIRE(openPairs.size() == 1, "internal error in exchange heuristic");
    finalCost += pair_cost(_net, openPairs.front().first, openPairs.front().second);
    ours.push_back(openPairs.front());
    if (finalCost < _bestCost) {
        const bool repeat = _bestCost - finalCost > heuristicCost * 2;
        _bestCost = finalCost;
        _order = std::move(ours);
        if (repeat) exchange_heuristic(_bestCost, _order, copy);
    }
}

// structural copy of the given nodes (no tensors); links leaving the set become external
static TensorNetwork stripped_subnet(const TensorNetwork& _net, const std::set<size_t>& _ids) {
    TensorNetwork s{TensorNetwork::Structure{}};
    s.nodes.resize(_net.nodes.size());
    for (size_t id = 0; id < _net.nodes.size(); ++id) {
        if (!_ids.count(id)) {
            s.nodes[id].erased = true;
            continue;
        }
        s.nodes[id].neighbors = _net.nodes[id].neighbors;
        for (size_t i = 0; i < s.nodes[id].neighbors.size(); ++i) {
            Link& l = s.nodes[id].neighbors[i];
            if (l.external || !_ids.count(l.other)) {
                l.external = true;
                l.other = NO_NODE;
                l.indexPosition = s.externalLinks.size();
                s.dimensions.push_back(l.dimension);
                s.externalLinks.emplace_back(id, i, l.dimension, false);
            }
        }
    }
    return s;
}

Order greedy_contraction_order(const TensorNetwork& _net, double* _cost) {
    std::set<size_t> ids;
    for (size_t i = 0; i < _net.nodes.size(); ++i)
        if (!_net.nodes[i].erased) ids.insert(i);
    const TensorNetwork s = stripped_subnet(_net, ids);
    double best = std::numeric_limits<double>::max();
    Order order;
    greedy_heuristic<&score_size>(best, order, s);
    greedy_heuristic<&score_mn>(best, order, s);
    greedy_heuristic<&score_speed>(best, order, s);
    greedy_heuristic<&score_big_tensor>(best, order, s);
    greedy_heuristic<&score_littlestep>(best, order, s);
    exchange_heuristic(best, order, s);
    if (_cost) *_cost = best;
    return order;
}

// The network value_t(x(i&0) * y(i&0)) is contracted over, in the reference's node numbering: x's TT
// network (ghost ones({1}) node 0, components 1..d, ghost d+1; ttNetwork.cpp:57-108), then y's appended
// by add_network_to_network (ids + d + 2, tensorNetwork.cpp:553-595), the d mode links joined by
// link_traces_and_fix (:598-675). Without TT data the nodes are stripped (planning only).
TensorNetwork tt_pair_network(const std::vector<size_t>& _n, const std::vector<size_t>& _rx, const std::vector<size_t>& _ry,
                              const TTTensor* _x, const TTTensor* _y) {
    const size_t d = _n.size();
    XERUS_REQUIRE(d >= 1 && _rx.size() == d + 1 && _ry.size() == d + 1, "tt_pair_network: need d dims and d+1 ranks per TT");
    TensorNetwork net{TensorNetwork::Structure{}};
    net.nodes.resize(2 * d + 4);
    auto build = [&](size_t base, size_t other, const std::vector<size_t>& r, const TTTensor* tt) {
        net.nodes[base].neighbors = {Link(base + 1, 0, 1, false)};
        for (size_t k = 0; k < d; ++k) {
            const size_t id = base + 1 + k;
            net.nodes[id].neighbors = {Link(id - 1, k == 0 ? 0 : 2, r[k], false), Link(other + 1 + k, 1, _n[k], false),
                                       Link(id + 1, 0, r[k + 1], false)};
        }
        net.nodes[base + d + 1].neighbors = {Link(base + d, 2, 1, false)};
        if (tt) {
            net.nodes[base].tensorObject.reset(new Tensor(Tensor::ones({1})));
            net.nodes[base + d + 1].tensorObject.reset(new Tensor(Tensor::ones({1})));
            for (size_t k = 0; k < d; ++k) net.nodes[base + 1 + k].tensorObject.reset(new Tensor(tt->components[k]));
        }
    };
    build(0, d + 2, _rx, _x);
    build(d + 2, 0, _ry, _y);
    net.require_valid_network();
    return net;
}

}  // namespace internal

size_t TensorNetwork::contract(const std::set<size_t>& _ids) {
    for (const size_t id : _ids) perform_traces(*this, id);
    if (_ids.empty()) return NO_NODE;
    if (_ids.size() == 1) return *_ids.begin();
    auto it = _ids.begin();
    if (_ids.size() == 2) {
        const size_t a = *it++;
        contract(a, *it);
        return a;
    }
    if (_ids.size() == 3) {
        const size_t a = *it++, b = *it++, c = *it;
        const auto t = internal::best_of_three(*this, a, b, c);
        // same decision as tensorNetwork.cpp:1269-1313 (ab, ac or bc first; a survives)
        if (std::get<0>(t) == a && std::get<1>(t) == b) {
            contract(a, b);
            contract(a, c);
        } else if (std::get<0>(t) == a) {
            contract(a, c);
            contract(a, b);
        } else {
            contract(b, c);
            contract(a, b);
        }
        return a;
    }
    std::set<size_t> sub = _ids;
    TensorNetwork s = internal::stripped_subnet(*this, sub);
    double best = std::numeric_limits<double>::max();
    internal::Order order;
    internal::greedy_heuristic<&internal::score_size>(best, order, s);
    internal::greedy_heuristic<&internal::score_mn>(best, order, s);
    internal::greedy_heuristic<&internal::score_speed>(best, order, s);
    internal::greedy_heuristic<&internal::score_big_tensor>(best, order, s);
    internal::greedy_heuristic<&internal::score_littlestep>(best, order, s);
    internal::exchange_heuristic(best, order, s);
    XERUS_REQUIRE(!order.empty(), "Internal Error: no contraction order found");
    for (const auto& c : order) contract(c.first, c.second);
    return order.back().first;
}

double TensorNetwork::contraction_cost(const std::set<size_t>& _ids) const {
    if (_ids.size() <= 1) return 0;
    TensorNetwork s = internal::stripped_subnet(*this, _ids);
    double cost = 0;
    internal::greedy_contraction_order(s, &cost);
    return cost;
}

Tensor TensorNetwork::to_tensor() const {
    require_valid_network();
    TensorNetwork cpy(*this);
    std::set<size_t> all;
    for (size_t i = 0; i < cpy.nodes.size(); ++i)
        if (!cpy.nodes[i].erased) all.insert(i);
    const size_t res = cpy.contract(all);
    const TensorNode& node = cpy.nodes[res];
    std::vector<size_t> shuffle(node.degree());
    bool identity = true;
    for (size_t i = 0; i < node.degree(); ++i) {
        XERUS_REQUIRE(node.neighbors[i].external, "Internal Error: the fully contracted network has an internal link");
        shuffle[i] = node.neighbors[i].indexPosition;
        identity &= shuffle[i] == i;
    }
    // unconnected components multiply in as scalars (degree-0 nodes are never linked)
    Tensor result = identity ? *node.tensorObject : reshuffle(*node.tensorObject, shuffle);
    return result;
}

value_t TensorNetwork::frob_norm() const { return to_tensor().frob_norm(); }

value_t TensorNetwork::operator[](const size_t _position) const {
    require_valid_network();
    if (degree() == 0) {
        XERUS_REQUIRE(_position == 0, "Tried to access non-existing entry of TN");
        value_t value = 1.0;
        for (const TensorNode& node : nodes)
            if (!node.erased) value *= (*node.tensorObject)[0];
        return value;
    }
    std::vector<size_t> positions(degree());
    size_t remains = _position;
    for (size_t i = degree(); i > 1; --i) {
        positions[i - 1] = remains % dimensions[i - 1];
        remains /= dimensions[i - 1];
    }
    positions[0] = remains;
    return (*this)[positions];
}

value_t TensorNetwork::operator[](const std::vector<size_t>& _positions) const {
    require_valid_network();
    XERUS_REQUIRE(_positions.size() == degree(), "Wrong number of positions: " << _positions.size() << " for degree " << degree());
    for (size_t i = 0; i < degree(); ++i)
        XERUS_REQUIRE(_positions[i] < dimensions[i], "Position " << _positions[i] << " out of range in mode " << i);
    // the reference's partial copy (tensorNetwork.cpp:331-370): fix every node's external modes (slices of the
    // device tensors), drop the external links, renumber the internal ones, contract what remains.
    // Cost per entry: the node copies are copy-on-write handles (no device copy); each external mode is one
    // strided slice copy, then the network of slices is contracted (one launch chain per entry). Callers that
    // need many entries of a TT -- the measurement sets of ADF -- go through the batched M x r stacks of
    // adf.hip instead (host/adf.cpp), not through this operator.
    TensorNetwork partial{Structure{}};
    partial.nodes = nodes;
    for (TensorNode& node : partial.nodes) {
        if (node.erased) continue;
        size_t killed = 0;
        for (size_t i = 0; i < node.neighbors.size(); ++i)
            if (node.neighbors[i].external) {
                node.tensorObject->fix_mode(i - killed, _positions[node.neighbors[i].indexPosition]);
                ++killed;
            }
        node.neighbors.erase(std::remove_if(node.neighbors.begin(), node.neighbors.end(), [](const Link& _l) { return _l.external; }),
                             node.neighbors.end());
        for (size_t i = 0; i < node.neighbors.size(); ++i)
            partial.nodes[node.neighbors[i].other].neighbors[node.neighbors[i].indexPosition].indexPosition = i;
    }
    std::set<size_t> all;
    for (size_t i = 0; i < partial.nodes.size(); ++i)
        if (!partial.nodes[i].erased) all.insert(i);
    if (all.empty()) return 1.0;
    const size_t res = partial.contract(all);
    return (*partial.nodes[res].tensorObject)[0];
}

Tensor& Tensor::operator=(const TensorNetwork& _network) { return *this = _network.to_tensor(); }

}  // namespace xerus
