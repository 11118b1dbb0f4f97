// pointmap.hpp -- host-side VISPREP data model: the grid, occluder rasterisation and flood fill
// that precede makeGraph.  Mirrors salalib PointMap (pointdata.cpp:122-171 setGrid, :296-371
// blockLines/blockLine, :402-514 makePoints/expand) and PixelBase::pixelateLineTouching
// (spacepix.cpp:144-214).  O(cells + line length) work; the O(N * visible) sweep runs on the GPU.
//
// Layout (what is uploaded to HBM):
//   state[C]      int32 Point::m_state, x-major cell index c = x * rows + y  (ColumnMatrix order)
//   seg_off[C+1]  int32 CSR into segs: the occluder pieces cropped to each cell
//   segs[S]       4 doubles (start.x, start.y, end.x, end.y) per cropped piece
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "geometry.hpp"

namespace dmx {

class PointMapHost {
  public:
    // region = MetaGraph::getRegion(); lines = drawing lines (x1,y1,x2,y2) as blockLines sees them.
    PointMapHost(const Rect& region, double spacing, const double* lines, int64_t nlines);

    int cols() const { return cols_; }
    int rows() const { return rows_; }
    double spacing() const { return spacing_; }
    Vec2 bottom_left() const { return bl_; }
    const Rect& grid_region() const { return region_; }
    const Rect& parent_region() const { return parent_; }
    int64_t cells() const { return (int64_t)cols_ * rows_; }
    int64_t index(int x, int y) const { return (int64_t)x * rows_ + y; }
    bool includes(int x, int y) const { return x >= 0 && x < cols_ && y >= 0 && y < rows_; }
    Vec2 cell_centre(int x, int y) const { // PointMap::depixelate (pointdata.h:353-357)
        return Vec2{bl_.x + spacing_ * 1.0 * double(x), bl_.y + spacing_ * 1.0 * double(y)};
    }
    Rect cell_rect(int x, int y, double border) const; // PointMap::regionate (pointdata.h:359-367)

    // runmethods.cpp:269-277 fillGraph + PointMap::makePoints(seed, fill_type) (pointdata.cpp:402-481).
    // fill_type 0 FULLFILL (FILLED), 1 SEMIFILL (FILLED | CONTEXTFILLED), 2 AUGMENT (AUGMENTED: not
    // FILLED, so the reference's expand re-queues every augmented neighbour and the fill only ends
    // when the seed cannot expand at all; see fill()).
    // Returns 0 = filled, 1 = point outside region, 2 = makePoints refused (off-grid, already
    // filled, or seed hidden from its cell centre), 3 = an AUGMENT fill that would never end in the
    // reference (nothing changed but the line blocking).
    int fill(double x, double y, int fill_type = 0);
    // Point::m_state a fill of this type sets (pointdata.cpp:434-441); -1 for an unknown type.
    static int32_t fill_state_of(int fill_type);
    // The AUGMENT pre-check: true if some neighbour of (sx, sy) passes PointMap::expand's tests.
    bool seed_can_expand(int sx, int sy) const;
    // fill's checks on the seed alone (region, pixelate, already filled, seed hidden from its cell
    // centre once lines are blocked): 0 = a fill may start at cell (*sx, *sy), else fill's code.
    int fill_seed(double x, double y, int* sx, int* sy) const;
    // Results of a fill computed elsewhere (the GPU path): lines blocked into these per-cell pieces,
    // and/or the cell states after the fill.
    void adopt_blocked(std::vector<int32_t>&& seg_off, std::vector<double>&& segs);
    void adopt_state(std::vector<int32_t>&& state);
    const std::vector<double>& drawing() const { return draw_; }
    // A map restored from a .graph PointMap chunk: grid geometry and cell states as stored
    // (PointMap::read, pointdata.cpp:1073-1156).  No occluder pieces: such a map can run VGA and
    // step depth on its graph but not makeGraph.
    void load_state(int cols, int rows, double spacing, Vec2 bl, const int32_t* state);
    // Fill states of a saved map of this same grid (FILLED / EDGE / CONTEXTFILLED bits).
    void restore_fill(const int32_t* state);
    // PointMap::sparkGraph2's boundary-graph pre-pass (pointdata.cpp:1254-1264).
    void keep_edges_only();
    void block_lines(); // idempotent (m_blockedlines)

    int64_t filled_count() const { return filled_; }
    std::vector<int32_t>& state() { return state_; }
    const std::vector<int32_t>& state() const { return state_; }
    const std::vector<int32_t>& seg_off() const { return seg_off_; }
    const std::vector<double>& segs() const { return segs_; }
    bool lines_blocked() const { return blocked_; }
    // Point::m_merge of every cell: the merge partner (x-major cell) or -1; empty when the map has no
    // merge links (PointMap::mergePixels, pointdata.cpp:1653-1680: both ends point at each other).
    const std::vector<int32_t>& merge() const { return merge_; }
    void set_merge(std::vector<int32_t>&& m) { merge_ = std::move(m); }

  private:
    void rasterise(const Seg& l, std::vector<int32_t>& out) const;
    int expand(int x1, int y1, int x2, int y2, std::vector<int32_t>& next);
    int expand_test(int x1, int y1, int x2, int y2) const;   // expand's result without filling
    Seg seg_at(int64_t k) const {
        return make_seg(Vec2{segs_[4 * k], segs_[4 * k + 1]}, Vec2{segs_[4 * k + 2], segs_[4 * k + 3]});
    }

    Rect parent_{};
    double spacing_ = 0;
    int cols_ = 0, rows_ = 0;
    Vec2 bl_{};
    Rect region_{};
    std::vector<double> draw_;
    std::vector<int32_t> state_;
    std::vector<int32_t> seg_off_;
    std::vector<double> segs_;
    bool blocked_ = false;
    int64_t filled_ = 0;
    int32_t fill_state_ = CELL_FILLED;   // the state the running fill sets
    std::vector<int32_t> merge_;
};

} // namespace dmx
