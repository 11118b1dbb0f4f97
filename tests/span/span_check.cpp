// Host brute-force check of makeGraph's span arithmetic (depthmapx_amd/csrc/kernels/span.hpp) against the
// sieve's per-cell rules (PointMap::sieve2, salalib/pointdata.cpp:1512-1565): for random gap lists,
// sources, octants and depth windows, every row's visible depths (visited by a gap, inside its centre)
// computed cell by cell equal the per-row intervals; and every row's class boundaries equal the per-cell
// bin decisions.  Built and run by tests/test_span_math.py (g++, -ffp-contract=off).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../depthmapx_amd/csrc/kernels/span.hpp"

using namespace dmx;

int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 2000;
    std::mt19937_64 rng(argc > 2 ? atoll(argv[2]) : 2026);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long long rows_checked = 0, cells = 0, bad = 0, class_checked = 0;
    for (int t = 0; t < trials; t++) {
        // a gap list inside [0, 1]: sorted cut points, alternate gap / block, gaps longer than 1e-10
        const int ng = 1 + (int)(rng() % 6);
        std::vector<double> cut;
        for (int i = 0; i < 2 * ng; i++) {
            double v = U(rng);
            if (rng() % 8 == 0) v = (double)(rng() % 5) / 4.0;   // exact quarters (0, 1/4, ..., 1)
            if (rng() % 16 == 0) v = 1.0 / (1 + rng() % 7);       // 1/k
            cut.push_back(v);
        }
        std::sort(cut.begin(), cut.end());
        if (rng() % 3 == 0) cut.front() = 0.0;
        if (rng() % 3 == 0) cut.back() = 1.0;
        std::vector<double> gs, ge;
        for (int i = 0; i < ng; i++)
            if (cut[2 * i + 1] > cut[2 * i] + 1e-10 && (gs.empty() || cut[2 * i] > ge.back())) {
                gs.push_back(cut[2 * i]);
                ge.push_back(cut[2 * i + 1]);
            }
        if (gs.empty()) continue;
        const int n = (int)gs.size();
        const int d0 = 1 + (int)(rng() % 1500), d1 = d0 + (int)(rng() % 300);
        // sieve2 per cell: visits[ind][d] = gap index that adds it (centre) or -1
        const int R = d1 + 2;
        std::vector<std::vector<int>> vis(R, std::vector<int>(d1 - d0 + 1, -1));
        for (int d = d0; d <= d1; d++) {
            int firstind = 0;
            for (int g = 0; g < n; g++)
                for (int ind = gap_lo(gs[g], d); ind <= gap_hi(ge[g], d); ind++) {
                    if (ind < firstind) continue;
                    if (ind > d) break;
                    firstind = ind;
                    const bool centre = (double)ind >= gs[g] * d && (double)ind <= ge[g] * d;
                    if (centre) {
                        if (vis[ind][d - d0] != -1) { bad++; fprintf(stderr, "row %d depth %d added twice\n", ind, d); }
                        vis[ind][d - d0] = g;
                    }
                }
        }
        for (int ind = 0; ind < R; ind++) {
            std::vector<int> got(d1 - d0 + 1, -1);
            int last_r = d0 - 1;
            for (int g = n - 1; g >= 0; g--) {
                int p, r;
                span_row_gap(ind, gs[g], ge[g], g > 0, g > 0 ? ge[g - 1] : 0.0, d0, d1, p, r);
                if (p <= r && p <= last_r) { bad++; fprintf(stderr, "gap intervals out of depth order\n"); }
                for (int d = p; d <= r; d++) got[d - d0] = g;
                if (p <= r) last_r = r;
            }
            for (int d = d0; d <= d1; d++) {
                cells += got[d - d0] >= 0;
                if (got[d - d0] != vis[ind][d - d0]) {
                    if (bad < 20)
                        fprintf(stderr, "trial %d row %d depth %d: span %d, sieve %d (gaps %d, d %d..%d)\n", t, ind, d,
                                got[d - d0], vis[ind][d - d0], n, d0, d1);
                    bad++;
                }
            }
            rows_checked++;
        }
        // class boundaries of random rows against the per-cell bins
        SpanOct o;
        o.q = (int)(rng() % 8);
        o.cx = (int)(rng() % 2000);
        o.cy = (int)(rng() % 2000);
        o.sp = (rng() % 2) ? 1.0 : 0.1 + U(rng);
        o.blx = (rng() % 2) ? 0.0 : -1000.0 * U(rng);
        o.bly = (rng() % 2) ? 0.0 : 1000.0 * U(rng);
        o.c0x = o.blx + o.sp * 1.0 * (double)o.cx;
        o.c0y = o.bly + o.sp * 1.0 * (double)o.cy;
        o.obinp = octant_bins(o.q);
        for (int k = 0; k < 40; k++) {
            const int ind = 1 + (int)(rng() % 1200);
            const int t3 = class_last(o, ind, 3, 0.5773502691896257), t2 = class_last(o, ind, 2, 0.2679491924311227);
            for (int d = ind + 1; d <= 5000; d++) {
                const int c = cell_class(o, d, ind);
                const int want = d <= t3 ? 3 : (d <= t2 ? 2 : 1);
                if (c != want) {
                    if (bad < 20) fprintf(stderr, "class: q %d row %d depth %d: cell %d, span %d (t3 %d t2 %d)\n", o.q, ind, d, c, want, t3, t2);
                    bad++;
                }
                class_checked++;
            }
        }
    }
    printf("rows %lld, visible cells %lld, class cells %lld, mismatches %lld\n", rows_checked, cells, class_checked, bad);
    return bad ? 1 : 0;
}
