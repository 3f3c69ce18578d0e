// Thread-local input generator (reference misc/random.h:33-34, misc/random.cpp:29-30): the same
// std::mt19937_64 + std::normal_distribution<double> pair, so Tensor::random / TTTensor::random draw
// bit-identical streams to the reference for the same seed.
#pragma once
#include <random>

namespace xerus {
namespace misc {
extern thread_local std::mt19937_64 randomEngine;
extern thread_local std::normal_distribution<double> defaultNormalDistribution;
}  // namespace misc
}  // namespace xerus
