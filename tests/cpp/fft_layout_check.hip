// Host-side exhaustive check of the FFT tile's index algebra (lphy_fft.h):
//  * pos / first-pass input index split into lane bits | element bits;
//  * lbase ^ cpart reproduces addr for every (slot, lane, element);
//  * addr is a bijection of (slot, position) onto the tile's LDS slots;
//  * every pass touches each position of a symbol exactly once.
#include "../../lora-sdr-lightweight-standalone-library-clean_amd/csrc/lphy_fft.h"
#include <cstdio>
#include <set>
#include <vector>
using namespace lphy;

template <int SF, int PI>
int check_pass() {
    using G = Geo<SF>;
    constexpr Passes<SF> PS{};
    if constexpr (PI >= PS.n) return 0;
    else {
        constexpr int HI = PS.hi[PI], LO = PS.lo[PI];
        using Gr = Group<SF, HI, LO>;
        int bad = 0;
        std::vector<int> seen_pos(G::N, 0), seen_in(G::N, 0);
        for (int lam = 0; lam < G::LPS; ++lam)
            for (int e = 0; e < G::E; ++e) {
                int p = Gr::pos(e, lam);
                if (p != (Gr::pos(0, lam) ^ Gr::pos(e, 0)) || (Gr::pos(0, lam) & Gr::pos(e, 0))) ++bad;
                int q = Gr::inidx(e, lam);
                if (PI == 0 && (q != (Gr::inidx(0, lam) ^ Gr::inidx(e, 0)) || (Gr::inidx(0, lam) & Gr::inidx(e, 0)))) ++bad;
                if (p < 0 || p >= G::N) { ++bad; continue; }
                seen_pos[p]++;
                if (PI == 0) seen_in[q]++;
                for (int slot = 0; slot < G::T; ++slot) {
                    if (G::at(G::lbase(slot, Gr::pos(0, lam)), G::cpart(Gr::pos(e, 0))) != G::addr(slot, p)) ++bad;
                    if (PI == 0 && G::at(G::lbase(slot, Gr::inidx(0, lam)), G::cpart(Gr::inidx(e, 0))) != G::addr(slot, q)) ++bad;
                }
            }
        for (int p = 0; p < G::N; ++p) {
            if (seen_pos[p] != 1) ++bad;
            if (PI == 0 && seen_in[p] != 1) ++bad;
        }
        return bad + check_pass<SF, PI + 1>();
    }
}

template <int SF>
int check_sf() {
    using G = Geo<SF>;
    int bad = check_pass<SF, 0>();
    std::set<int> addrs;
    for (int slot = 0; slot < G::T; ++slot)
        for (int p = 0; p < G::N; ++p) {
            int a = G::addr(slot, p);
            if (a < 0 || a >= G::T * G::SSTRIDE) ++bad;
            addrs.insert(a);
        }
    if ((int)addrs.size() != G::T * G::N) ++bad;
    for (int lam = 0; lam < G::LPS; ++lam)  // staging split
        for (int e = 0; e < G::E; ++e)
            for (int slot = 0; slot < G::T; ++slot)
                if (G::at(G::lbase(slot, lam), G::cpart(e * G::LPS)) != G::addr(slot, lam + e * G::LPS)) ++bad;
    printf("SF%d: %s (%d issues)\n", SF, bad ? "FAIL" : "ok", bad);
    return bad;
}

int main() {
    int bad = check_sf<1>() + check_sf<2>() + check_sf<3>() + check_sf<4>() + check_sf<5>() +
              check_sf<6>() + check_sf<7>() + check_sf<8>() + check_sf<9>() + check_sf<10>() +
              check_sf<11>() + check_sf<12>();
    return bad ? 1 : 0;
}
