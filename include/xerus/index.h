// Index objects of indexed expressions (reference include/xerus/index.h:43-158, src/xerus/index.cpp).
// An Index covers `span` consecutive modes; i^n spans n modes, i&n spans all but n modes of the tensor
// it indexes, i/n spans degree/n modes; an integer is a fixed index (slice).
#pragma once
#include <ostream>
#include <vector>

#include "basic.h"

namespace xerus {

class Index {
   public:
    enum Flag : unsigned { FIXED = 1u, INVERSE_SPAN = 2u, FRACTIONAL_SPAN = 4u };
    /// unique id (or the fixed position for FIXED indices)
    uint64 valueId;
    size_t span = 1;
    unsigned flags = 0;

    Index();
    Index(const Index&) noexcept = default;
    Index& operator=(const Index&) = default;
    Index(const int32 _i);
    Index(const uint32 _i) noexcept;
    Index(const int64 _i);
    Index(const uint64 _i) noexcept;
    explicit Index(const uint64 _valueId, const size_t _span, const unsigned _flags = 0) noexcept
        : valueId(_valueId), span(_span), flags(_flags) {}

    /// span this index covers in a tensor of the given degree
    size_t actual_span(const size_t _degree) const;
    bool fixed() const { return (flags & FIXED) != 0; }
    size_t fixed_position() const;

    Index operator^(const size_t _span) const;
    Index operator&(const size_t _span) const;
    Index operator/(const size_t _span) const;
};

/// Two indices are equal if their ids coincide; fixed indices are never equal.
bool operator==(const Index& _a, const Index& _b);
bool operator!=(const Index& _a, const Index& _b);
std::ostream& operator<<(std::ostream& _out, const Index& _idx);

/// convenience for bindings: n fresh indices
std::vector<Index> indices(size_t _n);

}  // namespace xerus
