// xerus-compatible basics for the MI355X build: value type, EPSILON, the error type thrown by REQUIRE.
// Mirrors include/xerus/basic.h:44,51 and misc/exceptions.h / misc/check.h:60-65 of the reference
// (XERUS_REQUIRE -> LOG(error) -> throw xerus::misc::generic_error).
#pragma once

#include <cstddef>
#include <cstdint>
#include <exception>
#include <limits>
#include <sstream>
#include <string>

namespace xerus {

using value_t = double;
using int32 = int32_t;
using int64 = int64_t;
using uint32 = uint32_t;
using uint64 = uint64_t;

/// 8 * DBL_EPSILON, the default relative cut of round() and SVDs (reference basic.h:51).
constexpr value_t EPSILON = 8 * std::numeric_limits<value_t>::epsilon();

namespace misc {
/// The exception every failed precondition throws (reference misc/exceptions.h).
class generic_error : public std::exception {
   public:
    std::string error_info;
    generic_error() = default;
    explicit generic_error(std::string msg) : error_info(std::move(msg)) {}
    const char* what() const noexcept override { return error_info.c_str(); }
    template <class T>
    generic_error& operator<<(const T& v) {
        std::ostringstream s;
        s << v;
        error_info += s.str();
        return *this;
    }
};
}  // namespace misc

}  // namespace xerus

#define XERUS_REQUIRE(cond, msg)                                                                  \
    do {                                                                                          \
        if (!(cond)) {                                                                            \
            std::ostringstream xerus_msg_;                                                        \
            xerus_msg_ << __FILE__ << ":" << __LINE__ << " " << msg;                              \
            throw ::xerus::misc::generic_error(xerus_msg_.str());                                 \
        }                                                                                         \
    } while (0)
