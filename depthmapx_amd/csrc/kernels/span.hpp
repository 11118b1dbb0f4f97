// span.hpp -- makeGraph's occluder-free depth spans: the per-row arithmetic, shared by the kernel
// (makegraph.hip) and a host brute-force test (tests/test_span_math.py builds tests/span_check.cpp).
//
// The reference's sieve (PointMap::sieve2, salalib/pointdata.cpp:1512-1565) visits, at depth d and for
// each gap [s, e] of the octant in order, the rows
//     ind in [max(lo(s, d), F), min(hi(e, d), d)]      lo = ceil(s (d - 1/2) - 1/2), hi = floor(e (d + 1/2) + 1/2)
// (F: the last row visited by the earlier gaps, the reference's `firstind`), and adds a visited cell when
// it is FILLED, unblocked and inside the gap's centre (`centregap`, :1541-1542):
//     cl(s, d) = ceil(s d) <= ind <= floor(e d) = ch(e, d).
// A cell's blocks (sparkSieve2::block, sparksieve2.cpp:67-87) change the gap list only if it holds an
// occluder piece.  So over depths where every visited cell is FILLED and holds no piece, the gap list is
// frozen and a row's visible depths, gap by gap, are intervals:
//   * cl(s, d) and ch(e, d) are non-decreasing in d (IEEE products are monotone), so ind >= cl holds on a
//     prefix of depths and ind <= ch on a suffix;
//   * every gap visits at least one row at every depth (hi >= lo: the window [s(d-1/2)-1/2, e(d+1/2)+1/2]
//     is longer than 1; lo <= d - 1 for s <= 1), and b = min(hi, d) is non-decreasing in e, so F before gap g
//     is b(e_{g-1}, d) -- non-decreasing in d, so ind >= F holds on a prefix;
//   * cl >= lo and ch <= min(hi, d), so a cell in the centre of gap g and at or past F is visited by g.
// Hence row ind is visible in gap g exactly on [first d with ch(e_g, d) >= ind,
//                                               last d with cl(s_g, d) <= ind and b(e_{g-1}, d) <= ind],
// and the gaps give disjoint intervals, later gaps first (a row's ratio ind/d falls as d grows).
//
// Each boundary is found from a floating estimate and settled with the exact predicate (monotone, so a few
// steps from an estimate within one of the answer).  All expressions are the kernel's own, in the same
// operation order (-ffp-contract=off): any difference from the per-cell path would show in the bit-exact
// makeGraph parity tests.
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#define DMX_SPAN_HD __host__ __device__
#else
#define DMX_SPAN_HD
#endif

namespace dmx {

// whichbin (pointdata.h:432-520)
DMX_SPAN_HD inline int whichbin(double gx, double gy) {
    int bin;
    double ratio;
    if (!(fabs(gy) > fabs(gx))) {
        ratio = fabs(gy) / fabs(gx);
        if (gx > 0.0) bin = (gy >= 0.0) ? 0 : -32;
        else bin = (gy >= 0.0) ? -16 : 16;
    } else {
        ratio = fabs(gx) / fabs(gy);
        if (gy > 0.0) bin = (gx >= 0.0) ? -8 : 8;
        else bin = (gx >= 0.0) ? 24 : -24;
    }
    if (ratio < 1e-12) {
    } else if (ratio < 0.2679491924311227) bin += 1;
    else if (ratio < 0.5773502691896257) bin += 2;
    else if (ratio < 1.0 - 1e-12) bin += 3;
    else bin += 4;
    if (bin < 0) bin = -bin;
    return bin % 32;
}

// cell (depth, ind) of octant q around (cx, cy) (pointdata.cpp:1536-1540)
DMX_SPAN_HD inline void octant_xy(int q, int cx, int cy, int depth, int ind, int& hx, int& hy) {
    const int x = (q >= 4 ? ind : depth);
    const int y = (q >= 4 ? depth : ind);
    hx = (short)(cx + ((q & 1) ? x : -x));
    hy = (short)(cy + ((q <= 1 || q >= 6) ? y : -y));
}

// The octant's geometry and its 5 bins by ratio class (0 axis, 1 below tan 15, 2 below tan 30, 3 below 1,
// 4 diagonal), 6 bits a class: whichbin of a representative direction of each class.
struct SpanOct {
    int q, cx, cy;
    double blx, bly, sp, c0x, c0y;
    unsigned obinp;
};

DMX_SPAN_HD inline unsigned octant_bins(int q) {
    const double rr[5] = {0.0, 0.1, 0.4, 0.8, 1.0};
    unsigned p = 0;
    for (int k = 0; k < 5; k++) {
        const double mj = 10.0, mn = 10.0 * rr[k];
        const double ax = (q >= 4 ? mn : mj), ay = (q >= 4 ? mj : mn);
        p |= (unsigned)whichbin((q & 1) ? ax : -ax, (q <= 1 || q >= 6) ? ay : -ay) << (6 * k);
    }
    return p;
}
DMX_SPAN_HD inline int obin(unsigned obinp, int k) { return (int)((obinp >> (6 * k)) & 63u); }

// The bin of visible cell (depth, ind): the makeGraph chunk loop's decision, verbatim -- the exact ratio
// ind/depth decides axis and diagonal; a float test with a 1e-6 margin decides the tan 15 / tan 30 classes;
// cells inside the margin take the FP64 whichbin of depixelate(cell) - centre.
DMX_SPAN_HD inline int cell_bin(const SpanOct& o, int depth, int ind) {
    const float fd = (float)depth, fi = (float)ind, mg = 1e-6f * fd;
    const float e15 = fi - 0.267949192f * fd, e30 = fi - 0.577350269f * fd;
    int k = 1 + (e15 >= 0.0f) + (e30 >= 0.0f);
    k = (ind == depth) ? 4 : k;
    k = (ind == 0) ? 0 : k;
    const bool amb = (ind != 0) & (ind != depth) & ((fabsf(e15) < mg) | (fabsf(e30) < mg));
    if (amb) {
        int hx, hy;
        octant_xy(o.q, o.cx, o.cy, depth, ind, hx, hy);
        const double px = o.blx + o.sp * 1.0 * (double)hx, py = o.bly + o.sp * 1.0 * (double)hy;
        return whichbin(px - o.c0x, py - o.c0y);
    }
    return obin(o.obinp, k);
}
// its ratio class (the bins of an octant are distinct)
DMX_SPAN_HD inline int cell_class(const SpanOct& o, int depth, int ind) {
    const int b = cell_bin(o, depth, ind);
    int k = 0;
    for (int j = 1; j < 5; j++)
        if (obin(o.obinp, j) == b) k = j;
    return k;
}

// Last depth d > ind with class >= kmin (kmin 2: ratio >= tan 15, tan = 0.2679...; kmin 3: ratio >= tan 30),
// or ind if there is none.  The class is non-increasing in d.  Off the float test's margin (|ind - tan d| >=
// 1e-6 d) the float decides, and d <= t - 1 (t = floor(ind / tan)) is far above the boundary, d >= t + 2 far
// below it, so only t and t + 1 are evaluated.
DMX_SPAN_HD inline int class_last(const SpanOct& o, int ind, int kmin, double tanv) {
    const double x = (double)ind / tanv;
    const int t = (int)floor(x);
    if (t + 1 > ind && cell_class(o, t + 1, ind) >= kmin) return t + 1;
    if (t > ind && cell_class(o, t, ind) >= kmin) return t;
    return (t - 1 > ind) ? t - 1 : ind;
}

// the sieve's per-gap integer bounds, the kernel's expressions
DMX_SPAN_HD inline int gap_lo(double s, int d) { return (int)ceil(s * (d - 0.5) - 0.5); }
DMX_SPAN_HD inline int gap_hi(double e, int d) { return (int)floor(e * (d + 0.5) + 0.5); }
DMX_SPAN_HD inline int gap_b(double e, int d) { const int h = gap_hi(e, d); return h < d ? h : d; }
DMX_SPAN_HD inline int gap_cl(double s, int d) { return (int)ceil(s * d); }
DMX_SPAN_HD inline int gap_ch(double e, int d) { return (int)floor(e * d); }

// an estimate clamped to [a, b] (x may be huge or infinite)
DMX_SPAN_HD inline int clamp_est(double x, int a, int b) {
    if (!(x >= (double)a)) return a;
    if (x >= (double)b) return b;
    return (int)x;
}

// Visible depths [p, r] of row ind in gap (s, e) within [d0, d1] (p > r: none); ep = end of the gap before
// (has_prev false for the first gap).  The row's exclusions (the axis row in 4 octants, the diagonal cell in
// the V octants) are applied by the caller.
DMX_SPAN_HD inline void span_row_gap(int ind, double s, double e, bool has_prev, double ep, int d0, int d1, int& p, int& r) {
    // p: first d with ch(e, d) >= ind  (e d >= ind)
    int a = (ind == 0) ? d0 : clamp_est(ceil((double)ind / e), d0, d1 + 1);
    while (a > d0 && gap_ch(e, a - 1) >= ind) a--;
    while (a <= d1 && gap_ch(e, a) < ind) a++;
    p = a;
    // last d with cl(s, d) <= ind  (s d <= ind)
    int c = (s > 0.0) ? clamp_est(floor((double)ind / s), d0 - 1, d1) : d1;
    while (c < d1 && gap_cl(s, c + 1) <= ind) c++;
    while (c >= d0 && gap_cl(s, c) > ind) c--;
    r = c;
    if (has_prev) {   // last d with b(ep, d) <= ind (the row is at or past the earlier gaps' last visited row)
        int f = clamp_est(floor(((double)ind + 0.5) / ep - 0.5), d0 - 1, d1);
        const int m = ind < d1 ? ind : d1;   // b(ep, d) <= d <= ind holds up to depth ind
        if (f < m) f = m;
        while (f < d1 && gap_b(ep, f + 1) <= ind) f++;
        while (f >= d0 && gap_b(ep, f) > ind) f--;
        if (f < r) r = f;
    }
}

}  // namespace dmx
