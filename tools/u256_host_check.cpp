// Host build of mythril_amd/csrc/u256.h (clang, x86) to fuzz the limb arithmetic before GPU runs.
// __ballot(x) is the lane's own predicate here (one lane per "wave").
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#define __device__
#define __forceinline__ inline
static inline unsigned long long __ballot(int p) { return p ? 1ull : 0ull; }
struct uint2 { uint32_t x, y; };
static inline uint2 make_uint2(uint32_t x, uint32_t y) { return uint2{x, y}; }
#define PF_HOST_MAC
#include "../mythril_amd/csrc/u256.h"
using pf::u256;
int main() {
    // reads lines: op a(64 hex) b(64 hex) ; prints results
    char op[16], as[80], bs[80];
    while (scanf("%15s %79s %79s", op, as, bs) == 3) {
        u256 a, b;
        for (int i = 0; i < 8; i++) {
            char t[9]; for (int k = 0; k < 8; k++) t[k] = as[56 - 8 * i + k]; t[8] = 0; a.l[i] = strtoul(t, 0, 16);
            for (int k = 0; k < 8; k++) t[k] = bs[56 - 8 * i + k]; b.l[i] = strtoul(t, 0, 16);
        }
        u256 q, r;
        pf::udivrem256(a, b, &q, &r);
        u256 m = pf::mul256(a, b);
        u256 sq = pf::sqr256(a);
        uint2 tbl[32];
        u256 ex = pf::exp256(a, b, (a.l[0] & 1u) ? 256u : 256u - pf::clz256(b), tbl, 1u);
        u256 ex2 = pf::exp256_split(a, b, tbl, 1u);
        for (int i = 7; i >= 0; i--) printf("%08x", q.l[i]); printf(" ");
        for (int i = 7; i >= 0; i--) printf("%08x", r.l[i]); printf(" ");
        for (int i = 7; i >= 0; i--) printf("%08x", m.l[i]); printf(" ");
        for (int i = 7; i >= 0; i--) printf("%08x", sq.l[i]); printf(" ");
        for (int i = 7; i >= 0; i--) printf("%08x", ex.l[i]); printf(" ");
        for (int i = 7; i >= 0; i--) printf("%08x", ex2.l[i]); printf("\n");
    }
}
