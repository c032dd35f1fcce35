// rng_pin.cpp — pins the oracle's RNG restatement against rocThrust (the implementation of the
// reference's third-party RNG dependency, THRUST_VERSION 200805 in this image).
// Host-only use of thrust::default_random_engine + uniform_real_distribution<float>(0,1),
// seeded exactly as pathtrace.cu:51-56 does.  utilhash (intersections.h:13-22) cannot be
// included from the reference (its header pulls in cuda_runtime.h), so it is restated here.
// Output: JSON {"cases": [[iter, index, depth, h, [u32 bits of 8 draws]], ...]} on stdout.
#include <thrust/random.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

static unsigned int utilhash(unsigned int a) {
    a = (a + 0x7ed55d16) + (a << 12);
    a = (a ^ 0xc761c23c) ^ (a >> 19);
    a = (a + 0x165667b1) + (a << 5);
    a = (a + 0xd3a2646c) ^ (a << 9);
    a = (a + 0xfd7046c5) + (a << 3);
    a = (a ^ 0xb55a4f09) ^ (a >> 16);
    return a;
}

int main() {
    const int iters[] = {1, 2, 3, 8, 17, 100, 4999, 5000};
    const int depths[] = {0, 1, 4, 7, 8, 12};
    uint32_t lcg = 12345u;
    std::printf("{\"thrust_version\": %d, \"cases\": [\n", THRUST_VERSION);
    bool first = true;
    for (int it : iters)
        for (int d : depths)
            for (int k = 0; k < 12; ++k) {
                lcg = lcg * 1664525u + 1013904223u;
                int index = (k < 4) ? k : (k < 8 ? 639996 + k : (int)(lcg % 2560000u));
                int h = utilhash((1 << 31) | (d << 22) | it) ^ utilhash(index);
                thrust::default_random_engine rng(h);
                thrust::uniform_real_distribution<float> u01(0, 1);
                std::printf("%s[%d, %d, %d, %u, [", first ? "" : ",\n", it, index, d, (unsigned)h);
                first = false;
                for (int j = 0; j < 8; ++j) {
                    float f = u01(rng);
                    uint32_t b; std::memcpy(&b, &f, 4);
                    std::printf("%s%u", j ? ", " : "", b);
                }
                std::printf("]]");
            }
    // engine edge cases: seeds that reduce to 0 mod m, and the largest outputs
    const uint32_t seeds[] = {0u, 2147483647u, 4294967294u, 1u, 2147483646u, 4294967295u};
    std::printf("\n], \"engine\": [\n");
    for (int s = 0; s < 6; ++s) {
        thrust::default_random_engine rng(seeds[s]);
        std::printf("%s[%u, [", s ? ",\n" : "", seeds[s]);
        for (int j = 0; j < 4; ++j) std::printf("%s%u", j ? ", " : "", (unsigned)rng());
        std::printf("]]");
    }
    std::printf("\n]}\n");
    return 0;
}
