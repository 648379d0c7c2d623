// Fixture generator (compiled by make_golden.py with the system g++ /
// libstdc++ 11): the REAL std::sort and std::min_element, called exactly as
// the reference calls them --
//   travorder        VRT/voxel_octree.cc:82-96  (Item {int ci; float dist},
//                    std::sort(items, items + 8, lhs.dist < rhs.dist))
//   ray_march_isect  VRT/voxel_octree.cc:101-125 (Record {..., float depth,
//                    int i}, std::min_element(.., lhs.depth < rhs.depth))
// on input arrays read from stdin (hex floats, so every bit pattern --
// +-0, +-inf, NaN, denormals -- survives the round trip).
// Input lines:   S d0 .. d7        ->  output "S c0 .. c7" (child order)
//                M n d0 .. d(n-1)  ->  output "M k" (min_element index, -1 if n == 0)
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static float read_float(const char *tok)
{
        // %a-formatted doubles (exact for every float) or "nan"/"-nan"
        // with an explicit payload in hex: "nanx7fc00001"
        if (std::strncmp(tok, "nanx", 4) == 0) {
                unsigned int u = (unsigned int)std::strtoul(tok + 4, nullptr, 16);
                float f;
                std::memcpy(&f, &u, 4);
                return f;
        }
        return (float)std::strtod(tok, nullptr);
}

int main()
{
        char line[4096];
        while (std::fgets(line, sizeof line, stdin)) {
                char *save = nullptr;
                char *tok = strtok_r(line, " \n", &save);
                if (!tok)
                        continue;
                if (tok[0] == 'S') {
                        struct Item {
                                int ci;
                                float dist;
                        } items[8];
                        for (int ci = 0; ci < 8; ++ci) {
                                items[ci].ci = ci;
                                items[ci].dist = read_float(strtok_r(nullptr, " \n", &save));
                        }
                        std::sort(items, items + 8,
                                  [](const Item &lhs, const Item &rhs) { return lhs.dist < rhs.dist; });
                        std::printf("S");
                        for (int i = 0; i < 8; ++i)
                                std::printf(" %d", items[i].ci);
                        std::printf("\n");
                } else if (tok[0] == 'M') {
                        struct Record {
                                float depth;
                                int i;
                        };
                        const int n = std::atoi(strtok_r(nullptr, " \n", &save));
                        std::vector<Record> records;
                        for (int i = 0; i < n; ++i)
                                records.push_back({ read_float(strtok_r(nullptr, " \n", &save)), i });
                        int k = -1;
                        if (!records.empty()) {
                                auto p = std::min_element(records.begin(), records.end(),
                                                          [](const Record &lhs, const Record &rhs) {
                                                                  return lhs.depth < rhs.depth;
                                                          });
                                k = p->i;
                        }
                        std::printf("M %d\n", k);
                }
        }
        return 0;
}
