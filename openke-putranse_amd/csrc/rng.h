// Random streams of the reference, restated for the GPU path.
//
//  * GlibcRand: glibc's srand()/rand() (TYPE_3 additive feedback, stdlib/random_r.c) with PRIVATE
//    state. The reference draws its sampler seeds and its universe walk from the process-global
//    glibc generator (Random.h:10-15, :32-45, UniverseConstructor.h:336-342); a private copy lets
//    every universe own its stream, so universes can be built concurrently with identical output.
//  * Lcg: the per-sampler-thread 64-bit LCG x <- x*25214903917 + 11 (Random.h:18-21) with an O(log n)
//    affine jump, so any GPU lane can start at any point of a thread's stream.
#pragma once
#include <cstdint>

#ifndef __HIPCC__
#define PT_HD
#else
#define PT_HD __host__ __device__
#endif

namespace pt {

struct GlibcRand {
    int32_t s[31];
    int f = 3, r = 0;
    explicit GlibcRand(uint32_t seed = 1) { seed_with(seed); }
    void seed_with(uint32_t seed) {
        if (seed == 0) seed = 1;
        int32_t w = (int32_t)seed;
        s[0] = w;
        for (int i = 1; i < 31; ++i) {   // 16807 * w mod (2^31 - 1), Schrage's decomposition
            long hi = w / 127773, lo = w % 127773;
            w = (int32_t)(16807 * lo - 2836 * hi);
            if (w < 0) w += 2147483647;
            s[i] = w;
        }
        f = 3;
        r = 0;
        for (int i = 0; i < 310; ++i) next();
    }
    int32_t next() {
        uint32_t v = (uint32_t)s[f] + (uint32_t)s[r];
        s[f] = (int32_t)v;
        if (++f >= 31) {
            f = 0;
            ++r;
        } else if (++r >= 31) {
            r = 0;
        }
        return (int32_t)(v >> 1);
    }
    // rand(a,b) of Random.h:32-34
    int64_t range(int64_t a, int64_t b) { return (int64_t)next() % (b - a) + a; }
};

constexpr uint64_t kLcgA = 25214903917ULL;
constexpr uint64_t kLcgC = 11ULL;

struct Affine {   // x -> a*x + c  (mod 2^64)
    uint64_t a, c;
};

// n-step affine map of the LCG
PT_HD inline Affine lcg_power(uint64_t n) {
    Affine acc{1, 0}, p{kLcgA, kLcgC};
    while (n) {
        if (n & 1) acc = Affine{acc.a * p.a, acc.c * p.a + p.c};   // apply acc first, then p
        p = Affine{p.a * p.a, p.c * p.a + p.c};
        n >>= 1;
    }
    return acc;
}
PT_HD inline uint64_t lcg_jump(uint64_t x, uint64_t n) {
    Affine m = lcg_power(n);
    return m.a * x + m.c;
}
PT_HD inline uint64_t lcg_next(uint64_t &x) {
    x = x * kLcgA + kLcgC;
    return x;
}

}  // namespace pt
