// Generates tests/golden/philox_kat.txt from ROCm rocrand host engine (Philox4x32-10 ten_rounds).
// Build: hipcc -x hip --offload-arch=gfx950 -O1 make_philox_kat.cpp -o /tmp/philox_kat && /tmp/philox_kat > philox_kat.txt
// The first three lines are also the published Random123 known-answer vectors.
#include <rocrand/rocrand_philox4x32_10.h>
#include <cstdio>
#include <cstdint>
struct E : rocrand_device::philox4x32_10_engine {
    uint4 tr(uint4 c, uint2 k) { return ten_rounds(c, k); }
};
int main() {
    E e;
    uint32_t vec[][6] = {{0,0,0,0,0,0},{0xffffffffu,0xffffffffu,0xffffffffu,0xffffffffu,0xffffffffu,0xffffffffu},
                         {0x243f6a88u,0x85a308d3u,0x13198a2eu,0x03707344u,0xa4093822u,0x299f31d0u}};
    for (auto& v : vec) { uint4 c = {v[0],v[1],v[2],v[3]}; uint2 k = {v[4],v[5]}; uint4 r = e.tr(c,k);
        printf("%08x %08x %08x %08x  %08x %08x -> %08x %08x %08x %08x\n", v[0],v[1],v[2],v[3],v[4],v[5], r.x,r.y,r.z,r.w); }
    uint32_t s = 12345;
    for (int i = 0; i < 8; ++i) {
        uint32_t w[6]; for (int j = 0; j < 6; ++j) { s = s * 1664525u + 1013904223u; w[j] = s; }
        uint4 c = {w[0],w[1],w[2],w[3]}; uint2 k = {w[4],w[5]}; uint4 r = e.tr(c,k);
        printf("%08x %08x %08x %08x  %08x %08x -> %08x %08x %08x %08x\n", w[0],w[1],w[2],w[3],w[4],w[5], r.x,r.y,r.z,r.w);
    }
}
