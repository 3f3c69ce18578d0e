// xerus::Index (index.cpp:33-178 of the reference): thread-local unique ids with the thread number in
// the top 10 bits, integer indices are fixed positions, ^ / & / "/" give span, inverse span and
// fractional span.
#include <atomic>

#include "xerus.h"

namespace xerus {

namespace {
std::atomic<uint64> idThreadInitCounter(0);
thread_local uint64 idCounter = (idThreadInitCounter++) << 54;
}  // namespace

Index::Index() : valueId(idCounter++), span(1), flags(0) {}

Index::Index(const int32 _i) : Index(static_cast<uint64>(_i)) { XERUS_REQUIRE(_i >= 0, "Negative valueId= " << _i << " given"); }

Index::Index(const uint32 _i) noexcept : valueId(_i), span(1), flags(FIXED) {}

Index::Index(const int64 _i) : Index(static_cast<uint64>(_i)) { XERUS_REQUIRE(_i >= 0, "Negative valueId= " << _i << " given"); }

Index::Index(const uint64 _i) noexcept : valueId(_i), span(1), flags(FIXED) {}

size_t Index::actual_span(const size_t _degree) const {
    if (flags & INVERSE_SPAN) {
        XERUS_REQUIRE(!(flags & FIXED), "Fixed indices must not have inverse span.");
        XERUS_REQUIRE(span <= _degree, "Index with inverse span would have negative actual span. Tensor degree: " << _degree
                                                                                                                 << ", inverse span " << span);
        return _degree - span;
    }
    if (flags & FRACTIONAL_SPAN) {
        XERUS_REQUIRE(!(flags & FIXED), "Fixed indices must not have fractional span.");
        XERUS_REQUIRE(span != 0 && _degree % span == 0,
                      "Fractional span must divide the tensor degree. Here tensor degree = " << _degree << ", span = " << span);
        return _degree / span;
    }
    XERUS_REQUIRE(!(flags & FIXED) || span == 1, "Fixed indices must have span one.");
    return span;
}

size_t Index::fixed_position() const {
    XERUS_REQUIRE(fixed(), "fixed_position() must only be called for fixed indices.");
    return size_t(valueId);
}

Index Index::operator^(const size_t _span) const {
    XERUS_REQUIRE(flags == 0, "Cannot apply ^ operator to an index that has any flag set.");
    return Index(valueId, _span);
}

Index Index::operator&(const size_t _span) const {
    XERUS_REQUIRE(flags == 0, "Cannot apply & operator to an index that has any flag set.");
    return Index(valueId, _span, INVERSE_SPAN);
}

Index Index::operator/(const size_t _span) const {
    XERUS_REQUIRE(flags == 0, "Cannot apply / operator to an index that has any flag set.");
    return Index(valueId, _span, FRACTIONAL_SPAN);
}

bool operator==(const Index& _a, const Index& _b) { return _a.valueId == _b.valueId && !_a.fixed() && !_b.fixed(); }

bool operator!=(const Index& _a, const Index& _b) { return !(_a == _b); }

std::ostream& operator<<(std::ostream& _out, const Index& _idx) {
    _out << "index#" << _idx.valueId << ((_idx.flags & Index::INVERSE_SPAN) ? "&" : ((_idx.flags & Index::FRACTIONAL_SPAN) ? "/" : "^"))
         << _idx.span;
    return _out;
}

std::vector<Index> indices(size_t _n) { return std::vector<Index>(_n); }

}  // namespace xerus
