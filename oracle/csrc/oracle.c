/*
 * CPU restatement of two byte/integer-exact pieces of the reference, used ONLY as a test checker
 * (tests/, __graft_entry__.smoke(), bench.py cpu_baseline). Never linked into the product.
 *
 *  1. reshuffle — mode permutation with the reference's block/odometer structure
 *     (/root/reference/src/xerus/indexedTensor_tensor_evaluate.cpp:39-49 increase_indices,
 *      :55-113 reshuffle, dense branch). shuffle[i] = new position of old mode i (:52-53, :80-82).
 *  2. the input generator of Tensor::random (include/xerus/tensor.h:212-220): std::mt19937_64
 *     (misc/random.cpp:29) feeding libstdc++'s std::normal_distribution<double> (Marsaglia polar
 *     method with one cached value; generate_canonical<double,53> = double(g())/2^64).
 *     Restated from the published algorithms, so fixtures can be regenerated bit-identically.
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>
#include <string.h>

/* ------------------------------------------------------------------ reshuffle */
void orc_reshuffle(double* out, const double* in, size_t ndim, const size_t* dims, const size_t* shuffle) {
    /* trailing modes that do not move form one contiguous block (evaluate.cpp:64-72) */
    long last = -1;
    for (size_t i = 0; i < ndim; ++i)
        if (shuffle[i] != i) last = (long)i;
    size_t nshuf = (size_t)(last + 1);
    size_t total = 1, block = 1;
    for (size_t i = 0; i < ndim; ++i) total *= dims[i];
    for (size_t i = nshuf; i < ndim; ++i) block *= dims[i];
    if (block == total) { memcpy(out, in, total * sizeof(double)); return; }
    size_t odims[64], step[64], idx[64];
    for (size_t i = 0; i < ndim; ++i) odims[shuffle[i]] = dims[i];
    for (size_t i = 0; i < nshuf; ++i) {       /* output stride of old mode i (evaluate.cpp:86-89) */
        size_t s = block;
        for (size_t k = shuffle[i] + 1; k < nshuf; ++k) s *= odims[k];
        step[i] = s;
        idx[i] = 0;
    }
    size_t nblocks = total / block, pos = 0;
    for (size_t b = 0; b < nblocks; ++b) {
        memcpy(out + pos, in + b * block, block * sizeof(double));
        /* odometer over the old modes 0..nshuf-1 in row-major order */
        for (long k = (long)nshuf - 1; k >= 0; --k) {
            pos += step[k];
            if (++idx[k] < dims[k]) break;
            pos -= dims[k] * step[k];
            idx[k] = 0;
        }
    }
}

/* ------------------------------------------------------------------ mt19937_64 + normal */
typedef struct {
    uint64_t mt[312];
    int mti;
    int saved_available;
    double saved;
} orc_rng;

void orc_rng_seed(orc_rng* r, uint64_t seed) {
    r->mt[0] = seed;
    for (int i = 1; i < 312; ++i)
        r->mt[i] = 6364136223846793005ULL * (r->mt[i - 1] ^ (r->mt[i - 1] >> 62)) + (uint64_t)i;
    r->mti = 312;
    r->saved_available = 0;
    r->saved = 0.0;
}

/* reseed the engine only (the reference's distribution object survives engine reseeds) */
void orc_rng_seed_engine(orc_rng* r, uint64_t seed) {
    int sa = r->saved_available;
    double sv = r->saved;
    orc_rng_seed(r, seed);
    r->saved_available = sa;
    r->saved = sv;
}

uint64_t orc_rng_next(orc_rng* r) {
    static const uint64_t MAG01[2] = {0ULL, 0xB5026F5AA96619E9ULL};
    const uint64_t UM = 0xFFFFFFFF80000000ULL, LM = 0x7FFFFFFFULL;
    if (r->mti >= 312) {
        int i;
        for (i = 0; i < 312 - 156; ++i) {
            uint64_t x = (r->mt[i] & UM) | (r->mt[i + 1] & LM);
            r->mt[i] = r->mt[i + 156] ^ (x >> 1) ^ MAG01[(int)(x & 1ULL)];
        }
        for (; i < 311; ++i) {
            uint64_t x = (r->mt[i] & UM) | (r->mt[i + 1] & LM);
            r->mt[i] = r->mt[i + (156 - 312)] ^ (x >> 1) ^ MAG01[(int)(x & 1ULL)];
        }
        uint64_t x = (r->mt[311] & UM) | (r->mt[0] & LM);
        r->mt[311] = r->mt[155] ^ (x >> 1) ^ MAG01[(int)(x & 1ULL)];
        r->mti = 0;
    }
    uint64_t x = r->mt[r->mti++];
    x ^= (x >> 29) & 0x5555555555555555ULL;
    x ^= (x << 17) & 0x71D67FFFEDA60000ULL;
    x ^= (x << 37) & 0xFFF7EEE000000000ULL;
    x ^= (x >> 43);
    return x;
}

static double canonical(orc_rng* r) {
    double u = (double)orc_rng_next(r) / 18446744073709551616.0; /* 2^64 */
    if (u >= 1.0) u = nextafter(1.0, 0.0);
    return u;
}

double orc_rng_normal(orc_rng* r) {
    if (r->saved_available) {
        r->saved_available = 0;
        return r->saved;
    }
    double x, y, r2;
    do {
        x = 2.0 * canonical(r) - 1.0;
        y = 2.0 * canonical(r) - 1.0;
        r2 = x * x + y * y;
    } while (r2 > 1.0 || r2 == 0.0);
    double mult = sqrt(-2.0 * log(r2) / r2);
    r->saved = x * mult;
    r->saved_available = 1;
    return y * mult;
}

void orc_rng_fill_normal(orc_rng* r, double* out, size_t n) {
    for (size_t i = 0; i < n; ++i) out[i] = orc_rng_normal(r);
}

size_t orc_rng_state_bytes(void) { return sizeof(orc_rng); }
