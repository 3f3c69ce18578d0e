// Generates tests/golden/rng_baadf00d.json: the first values libstdc++'s
// std::normal_distribution<double> draws from std::mt19937_64 seeded 0xBAADF00D (the reference's
// test seed, src/xerus/test/test.cpp:105; Tensor::random draw order, include/xerus/tensor.h:212-220).
// Build: g++ -O2 make_rng_fixture.cpp -o /tmp/mk && /tmp/mk > rng_baadf00d.json
#include <cstdio>
#include <random>
int main() {
    std::mt19937_64 g(0xBAADF00D);
    std::normal_distribution<double> d;
    std::printf("{\"seed\": %llu, \"generator\": \"libstdc++ std::mt19937_64 + std::normal_distribution<double>\",\n \"normal\": [",
                0xBAADF00DULL);
    for (int i = 0; i < 64; ++i) std::printf("%s%.17g", i ? ", " : "", d(g));
    std::mt19937_64 g2(0xBAADF00D);
    std::printf("],\n \"raw_u64\": [");
    for (int i = 0; i < 8; ++i) std::printf("%s\"%llu\"", i ? ", " : "", (unsigned long long)g2());
    std::printf("]}\n");
}
