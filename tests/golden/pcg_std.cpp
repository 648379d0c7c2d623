// Fixture generator (compiled by make_golden.py with the system g++ /
// libstdc++ 11): the draws jql::random_point_in_unit_sphere makes, using the
// REAL std::uniform_real_distribution<float> of libstdc++ over a PCG engine
// restated from VRT/graphics_math.h:821-857.  Output: text lines
//   U seed v0 v1 ... v(n-1)      (raw uniform(-1,1) draws, %a hex floats)
//   P seed x y z                 (accepted unit-sphere points in order)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <random>

struct PCG {
        using result_type = uint32_t;
        uint64_t state_;
        explicit PCG(uint64_t seed) : state_{ seed } {}
        static constexpr uint32_t min() { return 0; }
        static constexpr uint32_t max() { return std::numeric_limits<uint32_t>::max(); }
        uint32_t operator()()
        {
                state_ = state_ * 6364136223846793005ULL + 1442695040888963407ULL;
                auto xorshift = static_cast<uint32_t>((state_ ^ (state_ >> 18u)) >> 27u);
                uint64_t shift = state_ >> 59u;
                int32_t s32 = static_cast<int32_t>(static_cast<uint32_t>(shift));
                return (xorshift >> shift) | (xorshift << ((-s32) & 31u));
        }
};

int main(int argc, char **argv)
{
        const int nseeds = argc > 1 ? std::atoi(argv[1]) : 64;
        const int ndraw = argc > 2 ? std::atoi(argv[2]) : 48;
        const int npts = argc > 3 ? std::atoi(argv[3]) : 64;
        for (int k = 0; k < nseeds; ++k) {
                const uint64_t seed = 0xc01dbeefULL ^ (uint64_t)(k * 7919ULL + (k & 3) * 1920ULL * 1080ULL);
                PCG g(seed);
                std::printf("U %llu", (unsigned long long)seed);
                for (int i = 0; i < ndraw; ++i) {
                        std::uniform_real_distribution<float> d{ -1, 1 };
                        std::printf(" %a", (double)d(g));
                }
                std::printf("\n");
                PCG h(seed);
                for (int i = 0; i < npts; ++i) {
                        for (;;) {
                                auto d = std::uniform_real_distribution<float>{ -1, 1 };
                                float x = d(h), y = d(h), z = d(h);
                                float l = 0.f;
                                l += x * x;
                                l += y * y;
                                l += z * z;
                                if (__builtin_sqrtf(l) < 1.f) {
                                        std::printf("P %llu %a %a %a\n", (unsigned long long)seed, (double)x,
                                                    (double)y, (double)z);
                                        break;
                                }
                        }
                }
        }
        return 0;
}
