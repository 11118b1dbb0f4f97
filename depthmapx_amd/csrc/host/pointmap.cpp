// pointmap.cpp -- see pointmap.hpp.
#include "pointmap.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace dmx {

PointMapHost::PointMapHost(const Rect& region, double spacing, const double* lines, int64_t nlines)
    : parent_(region), spacing_(spacing), draw_(lines, lines + 4 * nlines) {
    // PointMap::setGrid(spacing, Point2f(0,0)) -- pointdata.cpp:122-171
    double xoffset = fmod(parent_.blx + 0.0, spacing_);
    double yoffset = fmod(parent_.bly + 0.0, spacing_);
    if (xoffset < spacing_ / 2.0) xoffset += spacing_;
    if (xoffset > spacing_ / 2.0) xoffset -= spacing_;
    if (yoffset < spacing_ / 2.0) yoffset += spacing_;
    if (yoffset > spacing_ / 2.0) yoffset -= spacing_;
    cols_ = (int)floor((xoffset + parent_.width()) / spacing_ + 0.5) + 1;
    rows_ = (int)floor((yoffset + parent_.height()) / spacing_ + 0.5) + 1;
    bl_ = Vec2{parent_.blx + -xoffset, parent_.bly + -yoffset};
    region_ = Rect{bl_.x - spacing_ / 2.0, bl_.y - spacing_ / 2.0,
                   bl_.x + double(cols_ - 1) * spacing_ + spacing_ / 2.0,
                   bl_.y + double(rows_ - 1) * spacing_ + spacing_ / 2.0};
    state_.assign((size_t)cells(), CELL_EMPTY);
    seg_off_.assign((size_t)cells() + 1, 0);
}

void PointMapHost::load_state(int cols, int rows, double spacing, Vec2 bl, const int32_t* state) {
    cols_ = cols;
    rows_ = rows;
    spacing_ = spacing;
    bl_ = bl;
    region_ = Rect{bl_.x - spacing_ / 2.0, bl_.y - spacing_ / 2.0, bl_.x + double(cols_ - 1) * spacing_ + spacing_ / 2.0,
                   bl_.y + double(rows_ - 1) * spacing_ + spacing_ / 2.0};
    state_.assign(state, state + (size_t)cells());
    seg_off_.assign((size_t)cells() + 1, 0);
    segs_.clear();
    draw_.clear();
    blocked_ = true;
    filled_ = 0;
    for (int32_t s : state_) filled_ += (s & CELL_FILLED) ? 1 : 0;
}

void PointMapHost::restore_fill(const int32_t* state) {
    // PointMap::read keeps MERGED as well (pointdata.cpp:1128); unmake clears the link, not the bit
    const int32_t keep = CELL_FILLED | CELL_EDGE | CELL_CONTEXTFILLED | CELL_EMPTY | CELL_MERGED;
    filled_ = 0;
    for (int64_t c = 0; c < cells(); c++) {
        state_[c] = (state_[c] & ~keep) | (state[c] & keep);
        filled_ += (state_[c] & CELL_FILLED) ? 1 : 0;
    }
}

Rect PointMapHost::cell_rect(int x, int y, double border) const {
    return Rect{bl_.x + spacing_ * (double(x) - 0.5 - border), bl_.y + spacing_ * (double(y) - 0.5 - border),
                bl_.x + spacing_ * (double(x) + 0.5 + border), bl_.y + spacing_ * (double(y) + 0.5 + border)};
}

// PixelBase::pixelateLineTouching(l, 1e-10) -- spacepix.cpp:144-214.  Appends (x,y) pairs.
void PointMapHost::rasterise(const Seg& in, std::vector<int32_t>& out) const {
    const double tol = 1e-10;
    Seg l = in;
    // normalScale to the grid region (top_right first, then bottom_left), then scale to cells
    double rw = region_.width(), rh = region_.height();
    l.r.trx = rw ? (l.r.trx - region_.blx) / rw : 0.0;
    l.r.tr_y = rh ? (l.r.tr_y - region_.bly) / rh : 0.0;
    l.r.blx = rw ? (l.r.blx - region_.blx) / rw : 0.0;
    l.r.bly = rh ? (l.r.bly - region_.bly) / rh : 0.0;
    l.r.trx *= double(cols_); l.r.tr_y *= double(rows_);
    l.r.blx *= double(cols_); l.r.bly *= double(rows_);
    auto emit = [&](int x, int y) {
        short sx = (short)x, sy = (short)y; // PixelRef(short, short), PixelRef::encloses
        if (sx >= 0 && sx < (short)cols_ && sy >= 0 && sy < (short)rows_) {
            out.push_back(sx);
            out.push_back(sy);
        }
    };
    const bool along_x = l.r.width() > l.r.height();
    const double grad = along_x ? l.sign() * l.r.height() / l.r.width() : l.sign() * l.r.width() / l.r.height();
    const double constant = along_x ? l.ay() - grad * l.ax() : l.ax() - grad * l.ay();
    const double lo = along_x ? l.ax() : l.r.bly, hi = along_x ? l.bx() : l.r.tr_y;
    int first = cvt_i32_x86(floor(lo - tol)), last = cvt_i32_x86(floor(hi + tol));
    for (int i = first; i <= last; i++) {
        int j1 = cvt_i32_x86(floor((first == i ? lo : double(i)) * grad + constant - l.sign() * tol));
        int j2 = cvt_i32_x86(floor((last == i ? hi : double(i + 1)) * grad + constant + l.sign() * tol));
        int js[3] = {j1, j2, (int)(((long long)j1 + j2) / 2)};
        int nj = (j1 != j2) ? (std::abs(j2 - j1) == 2 ? 3 : 2) : 1;
        for (int k = 0; k < nj; k++) {
            if (along_x) emit(i, js[k]);
            else emit(js[k], i);
        }
    }
}

// PointMap::blockLines / blockLine (pointdata.cpp:296-357): every drawing line is appended to each
// touched cell (cells become BLOCKED), then each cell crops its copies to regionate(cell, 1e-10).
void PointMapHost::block_lines() {
    if (blocked_) return;
    const int64_t C = cells();
    const int64_t L = (int64_t)draw_.size() / 4;
    std::vector<Seg> dl((size_t)L);
    std::vector<std::vector<int32_t>> touched((size_t)L);
    std::vector<int64_t> count((size_t)C + 1, 0);
    for (int64_t k = 0; k < L; k++) {
        dl[k] = make_seg(Vec2{draw_[4 * k], draw_[4 * k + 1]}, Vec2{draw_[4 * k + 2], draw_[4 * k + 3]});
        rasterise(dl[k], touched[k]);
        for (size_t i = 0; i < touched[k].size(); i += 2) count[index(touched[k][i], touched[k][i + 1]) + 1]++;
    }
    for (int64_t c = 0; c < C; c++) count[c + 1] += count[c];
    std::vector<int64_t> cursor(count.begin(), count.end() - 1);
    std::vector<int32_t> raw((size_t)count[C]);
    for (int64_t k = 0; k < L; k++)
        for (size_t i = 0; i < touched[k].size(); i += 2) {
            int64_t c = index(touched[k][i], touched[k][i + 1]);
            raw[cursor[c]++] = (int32_t)k;
            state_[c] |= CELL_BLOCKED;
        }
    segs_.clear();
    for (int x = 0; x < cols_; x++)
        for (int y = 0; y < rows_; y++) {
            int64_t c = index(x, y);
            seg_off_[c] = (int32_t)(segs_.size() / 4);
            Rect cell = cell_rect(x, y, 1e-10);
            for (int64_t i = count[c]; i < count[c + 1]; i++) {
                Seg s = dl[raw[i]];
                if (clip_seg(s, cell)) {
                    Vec2 a = s.start(), b = s.end();
                    segs_.push_back(a.x); segs_.push_back(a.y);
                    segs_.push_back(b.x); segs_.push_back(b.y);
                }
            }
        }
    seg_off_[C] = (int32_t)(segs_.size() / 4);
    blocked_ = true;
}

// PointMap::expand (pointdata.cpp:483-514): 1 off-grid, 2 already filled, 4 blocked, 8 filled now.
int PointMapHost::expand_test(int x1, int y1, int x2, int y2) const {
    if ((short)x2 < 0 || (short)x2 >= (short)cols_ || (short)y2 < 0 || (short)y2 >= (short)rows_) return 1;
    const int64_t c1 = index(x1, y1), c2 = index(x2, y2);
    if (state_[c2] & CELL_FILLED) return 2;
    Seg l = make_seg(cell_centre(x1, y1), cell_centre(x2, y2));
    const double tol = spacing_ * 1e-10;
    for (int64_t c : {c1, c2})
        for (int32_t k = seg_off_[c]; k < seg_off_[c + 1]; k++) {
            Seg s = seg_at(k);
            if (rects_touch(l.r, s.r, tol) && segs_cross(l, s, tol)) return 4;
        }
    return 8;
}

int PointMapHost::expand(int x1, int y1, int x2, int y2, std::vector<int32_t>& next) {
    const int r = expand_test(x1, y1, x2, y2);
    if (r != 8) return r;
    const int64_t c2 = index(x2, y2);
    state_[c2] = fill_state_ | (state_[c2] & CELL_BLOCKED); // Point::set keeps BLOCKED
    filled_++;
    next.push_back(x2);
    next.push_back(y2);
    return 8;
}

int32_t PointMapHost::fill_state_of(int fill_type) {
    switch (fill_type) {
    case 0: return CELL_FILLED;                       // FULLFILL
    case 1: return CELL_FILLED | CELL_CONTEXTFILLED;  // SEMIFILL
    case 2: return CELL_AUGMENTED;                    // AUGMENT
    default: return -1;
    }
}

// makePoints' expand order (pointdata.cpp:457-464): up, down, left, right, up-left, up-right, down-left,
// down-right (PixelRef::up() is y+1).
static const int k_expand_dx[8] = {0, 0, -1, 1, -1, 1, -1, 1};
static const int k_expand_dy[8] = {1, -1, 0, 0, 1, 1, -1, -1};

bool PointMapHost::seed_can_expand(int sx, int sy) const {
    for (int k = 0; k < 8; k++)
        if (expand_test(sx, sy, sx + k_expand_dx[k], sy + k_expand_dy[k]) == 8) return true;
    return false;
}

int PointMapHost::fill_seed(double px, double py, int* psx, int* psy) const {
    // fillGraph: graph.getRegion().contains(point) -- strict (p2dpoly.h:338-340)
    if (!(px > parent_.blx && px < parent_.trx && py > parent_.bly && py < parent_.tr_y)) return 1;
    // PointMap::pixelate(p, false) (pointdata.cpp:283-305) into PixelRef(short, short)
    int sx = (short)(int)floor((px - bl_.x + (spacing_ / 2.0)) / (spacing_ / 1.0));
    int sy = (short)(int)floor((py - bl_.y + (spacing_ / 2.0)) / (spacing_ / 1.0));
    if (!includes(sx, sy) || (state_[index(sx, sy)] & CELL_FILLED)) return 2;
    if (blocked_) { // seed must see its own cell centre (only once lines are blocked: pointdata.cpp:422-428)
        Seg ls = make_seg(Vec2{px, py}, cell_centre(sx, sy));
        int64_t c = index(sx, sy);
        for (int32_t k = seg_off_[c]; k < seg_off_[c + 1]; k++)
            if (segs_cross_strict(seg_at(k), ls, 0.0)) return 2;
    }
    *psx = sx;
    *psy = sy;
    return 0;
}

void PointMapHost::adopt_blocked(std::vector<int32_t>&& seg_off, std::vector<double>&& segs) {
    seg_off_ = std::move(seg_off);
    segs_ = std::move(segs);
    blocked_ = true;
}

void PointMapHost::adopt_state(std::vector<int32_t>&& state) {
    // m_filled_point_count counts set() calls, not FILLED bits (an AUGMENT seed counts too): add the
    // cells the adopted fill filled
    int64_t before = 0, after = 0;
    for (int32_t s : state_) before += (s & CELL_FILLED) ? 1 : 0;
    for (int32_t s : state) after += (s & CELL_FILLED) ? 1 : 0;
    state_ = std::move(state);
    filled_ += after - before;
}

int PointMapHost::fill(double px, double py, int fill_type) {
    const int32_t fs = fill_state_of(fill_type);
    if (fs < 0) return 2;
    int sx = 0, sy = 0;
    const int r = fill_seed(px, py, &sx, &sy);
    if (r) return r;
    block_lines();
    int64_t c0 = index(sx, sy);
    if (fs == CELL_AUGMENTED) {
        // AUGMENT sets AUGMENTED without FILLED, and expand only stops at FILLED cells
        // (pointdata.cpp:489): the first neighbour it fills re-queues the seed, which re-queues that
        // neighbour, and the reference's loop never ends.  It ends only when the seed expands nowhere;
        // then the seed alone is set (and counted, :444) and gets EDGE like any fill's cell (:466-468).
        if (seed_can_expand(sx, sy)) return 3;
        int res = 0;
        for (int k = 0; k < 8; k++) res |= expand_test(sx, sy, sx + k_expand_dx[k], sy + k_expand_dy[k]);
        state_[c0] = fs | (state_[c0] & CELL_BLOCKED);
        filled_++;
        if ((res & 4) || (state_[c0] & CELL_BLOCKED)) state_[c0] |= CELL_EDGE;
        return 0;
    }
    fill_state_ = fs;
    state_[c0] = fs | (state_[c0] & CELL_BLOCKED);
    filled_++;
    // pflipper flood fill: pop from the back of the current layer, push into the next layer
    std::vector<int32_t> layer[2];
    int cur = 0;
    layer[0] = {sx, sy};
    while (!layer[cur].empty()) {
        int x = layer[cur][layer[cur].size() - 2], y = layer[cur].back();
        std::vector<int32_t>& nxt = layer[cur ^ 1];
        int res = 0;
        for (int k = 0; k < 8; k++) res |= expand(x, y, x + k_expand_dx[k], y + k_expand_dy[k], nxt);
        int64_t c = index(x, y);
        if ((res & 4) || (state_[c] & CELL_BLOCKED)) state_[c] |= CELL_EDGE;
        layer[cur].pop_back();
        layer[cur].pop_back();
        if (layer[cur].empty()) cur ^= 1;
    }
    fill_state_ = CELL_FILLED;
    return 0;
}

void PointMapHost::keep_edges_only() {
    for (auto& s : state_)
        if ((s & CELL_FILLED) && !(s & CELL_EDGE)) {
            s &= ~CELL_FILLED;
            filled_--;
        }
}

} // namespace dmx
