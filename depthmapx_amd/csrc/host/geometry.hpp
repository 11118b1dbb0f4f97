// geometry.hpp -- IEEE-double 2-D primitives of the visibility path, shared by the host model and
// the HIP kernels (all functions are __host__ __device__).  Every operation keeps the exact
// operation order of the reference so results are bit-identical; compile with -ffp-contract=off.
//
// Reference: genlib/p2dpoly.{h,cpp} (orange-vertex/depthmapX).
#pragma once
#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#define DMX_HD __host__ __device__ inline
#else
#define DMX_HD inline
#endif

namespace dmx {

struct Vec2 {
    double x, y;
};

// QtRegion (p2dpoly.h:288-330) -- bottom-left / top-right corners.
struct Rect {
    double blx, bly, trx, tr_y;
    DMX_HD double width() const { return fabs(trx - blx); }   // p2dpoly.h:317
    DMX_HD double height() const { return fabs(tr_y - bly); } // p2dpoly.h:306
};

// Line = region + parity bit (p2dpoly.h:398-481).  parity 1: start at bottom-left.
struct Seg {
    Rect r;
    int parity;
    DMX_HD double ax() const { return r.blx; }
    DMX_HD double bx() const { return r.trx; }
    DMX_HD double ay() const { return parity ? r.bly : r.tr_y; }
    DMX_HD double by() const { return parity ? r.tr_y : r.bly; }
    DMX_HD double sign() const { return parity ? 1.0 : -1.0; }
    DMX_HD Vec2 start() const { return Vec2{r.blx, ay()}; }
    DMX_HD Vec2 end() const { return Vec2{r.trx, by()}; }
    DMX_HD double length() const { // p2dpoly.h:476-479
        return sqrt((r.trx - r.blx) * (r.trx - r.blx) + (r.tr_y - r.bly) * (r.tr_y - r.bly));
    }
};

// Line::Line(a, b) (p2dpoly.cpp:291-336); the direction bit is not needed on this path.
DMX_HD Seg make_seg(Vec2 a, Vec2 b) {
    Seg s;
    if (a.x == b.x) {
        s.r.blx = a.x; s.r.trx = b.x; s.parity = 1;
        if (a.y <= b.y) { s.r.bly = a.y; s.r.tr_y = b.y; }
        else { s.r.bly = b.y; s.r.tr_y = a.y; }
    } else if (a.x < b.x) {
        s.r.blx = a.x; s.r.trx = b.x;
        if (a.y <= b.y) { s.r.bly = a.y; s.r.tr_y = b.y; s.parity = 1; }
        else { s.r.bly = b.y; s.r.tr_y = a.y; s.parity = 0; }
    } else {
        s.r.blx = b.x; s.r.trx = a.x;
        if (b.y <= a.y) { s.r.bly = b.y; s.r.tr_y = a.y; s.parity = 1; }
        else { s.r.bly = a.y; s.r.tr_y = b.y; s.parity = 0; }
    }
    return s;
}

// intersect_region with tolerance, touching counts (p2dpoly.cpp:247-279).
DMX_HD bool rects_touch(const Rect& a, const Rect& b, double tol) {
    bool ox = (a.blx > b.blx) ? (b.trx >= a.blx - tol) : (a.trx >= b.blx - tol);
    if (!ox) return false;
    return (a.bly > b.bly) ? (b.tr_y >= a.bly - tol) : (a.tr_y >= b.bly - tol);
}

// intersect_line: product-of-cross-products test, touching counts (p2dpoly.cpp:350-363).
DMX_HD bool segs_cross(const Seg& a, const Seg& b, double tol) {
    double p1 = ((a.ay() - a.by()) * (b.ax() - a.ax()) + (a.bx() - a.ax()) * (b.ay() - a.ay())) *
                ((a.ay() - a.by()) * (b.bx() - a.ax()) + (a.bx() - a.ax()) * (b.by() - a.ay()));
    if (!(p1 <= tol)) return false;
    double p2 = ((b.ay() - b.by()) * (a.ax() - b.ax()) + (b.bx() - b.ax()) * (a.ay() - b.ay())) *
                ((b.ay() - b.by()) * (a.bx() - b.ax()) + (b.bx() - b.ax()) * (a.by() - b.ay()));
    return p2 <= tol;
}

// intersect_line_no_touch (p2dpoly.cpp:368-381).
DMX_HD bool segs_cross_strict(const Seg& a, const Seg& b, double tol) {
    double p1 = ((a.ay() - a.by()) * (b.ax() - a.ax()) + (a.bx() - a.ax()) * (b.ay() - a.ay())) *
                ((a.ay() - a.by()) * (b.bx() - a.ax()) + (a.bx() - a.ax()) * (b.by() - a.ay()));
    if (!(p1 < -tol)) return false;
    double p2 = ((b.ay() - b.by()) * (a.ax() - b.ax()) + (b.bx() - b.ax()) * (a.ay() - b.ay())) *
                ((b.ay() - b.by()) * (a.bx() - b.ax()) + (b.bx() - b.ax()) * (a.by() - b.ay()));
    return p2 < -tol;
}

// Line::crop (p2dpoly.cpp:626-667); false if the segment misses the rectangle.
DMX_HD bool clip_seg(Seg& l, const Rect& c) {
    double& ay = l.parity ? l.r.bly : l.r.tr_y;
    double& by = l.parity ? l.r.tr_y : l.r.bly;
    if (!(l.r.trx >= c.blx)) return false;
    if (l.r.blx < c.blx) {
        ay += l.sign() * (l.r.height() * (c.blx - l.r.blx) / l.r.width());
        l.r.blx = c.blx;
    }
    if (!(l.r.blx <= c.trx)) return false;
    if (l.r.trx > c.trx) {
        by -= l.sign() * l.r.height() * (l.r.trx - c.trx) / l.r.width();
        l.r.trx = c.trx;
    }
    if (!(l.r.tr_y >= c.bly)) return false;
    if (l.r.bly < c.bly) {
        if (l.parity) l.r.blx += l.r.width() * (c.bly - l.r.bly) / l.r.height();
        else l.r.trx -= l.r.width() * (c.bly - l.r.bly) / l.r.height();
        l.r.bly = c.bly;
    }
    if (!(l.r.bly <= c.tr_y)) return false;
    if (l.r.tr_y > c.tr_y) {
        if (l.parity) l.r.trx -= l.r.width() * (l.r.tr_y - c.tr_y) / l.r.height();
        else l.r.blx += l.r.width() * (l.r.tr_y - c.tr_y) / l.r.height();
        l.r.tr_y = c.tr_y;
    }
    return true;
}

// int(floor(v)) as the reference's x86-64 build evaluates it (cvttsd2si): NaN and out-of-range values
// give INT_MIN.  pixelateLineTouching meets NaN on zero-length lines (0/0 gradient); C++ leaves the
// conversion undefined and the GPU's own conversion gives 0, so both paths spell it out.
DMX_HD int cvt_i32_x86(double v) { return (v >= -2147483648.0 && v < 2147483648.0) ? (int)v : (int)(-2147483647 - 1); }

// Point::m_state bits (salalib/point.h:32-38).
enum CellState : int32_t {
    CELL_EMPTY = 0x0001, CELL_FILLED = 0x0002, CELL_BLOCKED = 0x0004, CELL_CONTEXTFILLED = 0x0008,
    CELL_SELECTED = 0x0010, CELL_EDGE = 0x0020, CELL_MERGED = 0x0040, CELL_AUGMENTED = 0x8000
};

} // namespace dmx
