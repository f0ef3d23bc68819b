// Host-side check of the device S2 helpers (compiled by hipcc as host code):
// prints values the pytest compares with the CPU oracle.
#include <cstdio>
#include <cstdlib>

#include "../../dss_amd/csrc/loopdev.cuh"

using namespace dss::s2;

int main(int argc, char **argv)
{
    // mode 0: cell ids from (face, i, j, level)
    unsigned long long seed = 12345;
    auto rnd = [&]() { seed = seed * 6364136223846793005ull + 1442695040888963407ull; return (unsigned)(seed >> 33); };
    for (int k = 0; k < 2000; k++) {
        int face = rnd() % 6, level = rnd() % 31;
        int i = rnd() & ((1 << 30) - 1), j = rnd() & ((1 << 30) - 1);
        int o;
        unsigned long long id = cell_from_face_ij_level(face, i, j, level, o);
        printf("%d %d %d %d %llu %d\n", face, i, j, level, id, o);
    }
    return 0;
}
