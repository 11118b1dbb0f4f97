// graphio.cpp -- the PointMap chunk of a depthmapX .graph file (host side, byte-exact).
//
// Writer: PointMap::write (salalib/pointdata.cpp:1158-1188) with AttributeTable::write
// (salalib/attributetable.cpp:427-456, columns alphabetically, rows x-major), LayerManagerImpl::write
// (salalib/layermanagerimpl.cpp:107-150), Point::write (salalib/point.cpp:51-73), Node::write /
// Bin::write / PixelVec::write (salalib/ngraph.cpp:209-220, :447-472, :517-583, 4-bit ShiftLength).
// Column statistics are replayed in the reference's setValue order (attributetable.cpp:65-84,
// :155-166) so min / max / total come out bit-identical.
//
// Reader: the inverse (PointMap::read pointdata.cpp:1073-1156, Bin::read ngraph.cpp:420-445,
// PixelVec::read ngraph.cpp:491-563) including the lossy 4-bit row shift: runs whose row jumps by
// more than 15 come back moved, exactly like the graph the reference CLI's VGA step analyses.
#include "graphio.hpp"

#include <algorithm>
#include <cstring>
#include <numeric>

namespace dmx {

namespace {
enum : uint8_t { DIR_NODIR = 0, DIR_H = 1, DIR_V = 2, DIR_PD = 4, DIR_ND = 8, DIR_DIAG = 12 };

struct Writer {
    std::vector<uint8_t>& b;
    template <typename T> void put(const T& v) {
        const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
        b.insert(b.end(), p, p + sizeof(T));
    }
    void str(const std::string& s) { // dXstring::writeString (genlib/stringutils.cpp:52-58)
        put<uint32_t>((uint32_t)s.size());
        b.insert(b.end(), s.begin(), s.end());
    }
};

struct Reader {
    const uint8_t* p;
    size_t n, o = 0;
    bool ok = true;
    template <typename T> T get() {
        T v{};
        if (o + sizeof(T) > n) { ok = false; return v; }
        std::memcpy(&v, p + o, sizeof(T));
        o += sizeof(T);
        return v;
    }
    std::string str() {
        const uint32_t len = get<uint32_t>();
        if (!ok || o + len > n) { ok = false; return std::string(); }
        std::string s(reinterpret_cast<const char*>(p + o), len);
        o += len;
        return s;
    }
};

inline int32_t pixref(int x, int y) { return (int32_t)(((uint32_t)(int16_t)x << 16) + ((uint32_t)(int16_t)y & 0xffffu)); }

// ShiftLength {unsigned short shift:4; unsigned short runlength:12;} (ngraph.cpp:536-539)
inline uint16_t shift_length(int shift, int runlength) {
    return (uint16_t)(((unsigned)shift & 0xFu) | (((unsigned)runlength & 0xFFFu) << 4));
}

// Bin direction of bin i (Node::make, ngraph.cpp:43-54); empty bins keep NODIR.
inline uint8_t bin_dir(int b) {
    if (b == 4 || b == 20) return DIR_PD;
    if (b == 12 || b == 28) return DIR_ND;
    if ((b > 4 && b < 12) || (b > 20 && b < 28)) return DIR_V;
    return DIR_H;
}

struct Stats { double min = -1.0, max = -1.0, total = -1.0; };

// AttributeRowImpl::setValue + AttributeColumnImpl::updateStats on a fresh column (every value -1),
// for the rows the analysis actually set (x-major order).
Stats replay_stats(const float* v, const uint8_t* set, int64_t n) {
    Stats s;
    for (int64_t i = 0; i < n; i++) {
        if (set && !set[i]) continue;
        const float val = v[i];
        const float old = 0.0f;   // the previous value is -1, clamped to 0
        if (s.total < 0) s.total = val;
        else { s.total += val; s.total -= old; }
        if (val > s.max) s.max = val;
        if (s.min < 0 || val < s.min) s.min = val;
    }
    return s;
}
} // namespace

int write_pointmap_chunk(const PointMapHost& h, int64_t nnodes, const int32_t* bins, const int16_t* runs, int64_t nruns,
                         const uint8_t* gridconn, const std::vector<ChunkColumn>& cols, int displayed, bool boundary,
                         std::vector<uint8_t>& out, std::string& err) {
    out.clear();
    Writer w{out};
    const int C_cols = h.cols(), C_rows = h.rows();
    // ---- PointMap header (pointdata.cpp:1160-1176)
    w.str("VGA Map");
    w.put<double>(h.spacing());
    w.put<int32_t>(C_rows);
    w.put<int32_t>(C_cols);
    w.put<int32_t>((int32_t)h.filled_count());
    w.put<double>(h.bottom_left().x);
    w.put<double>(h.bottom_left().y);
    // no graph (VISPREP without -pm): no Node records, an empty attribute table (rows are added by
    // sparkGraph2, pointdata.cpp:1294), m_processed false, displayed attribute -2
    const bool graph = bins != nullptr;
    if (!graph) nnodes = 0;
    std::vector<int> order(cols.size());
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return cols[a].name < cols[b].name; });
    int sorted_disp = -1;
    for (size_t i = 0; i < order.size(); i++)
        if (order[i] == displayed) sorted_disp = (int)i;
    if (displayed < 0) sorted_disp = displayed;
    if (!graph) sorted_disp = -2;
    w.put<int32_t>(sorted_disp);
    // ---- AttributeTable::write: layer manager with the single "Everything" layer
    w.put<int64_t>(0xC0000000LL);   // availableLayers = 0xffffffff << (32 + 0xfffffffe) (unsigned wrap: << 30)
    w.put<int64_t>(1);              // visible layers
    w.put<int32_t>(1);              // layer count
    w.put<int64_t>(1);              // layer key
    w.str("Everything");
    w.put<int32_t>((int32_t)cols.size());
    for (int ci : order) {
        const ChunkColumn& c = cols[ci];
        const Stats s = replay_stats(c.values.data(), c.set.empty() ? nullptr : c.set.data(), nnodes);
        w.str(c.name);
        w.put<float>((float)s.min);
        w.put<float>((float)s.max);
        w.put<double>(s.total);
        w.put<int32_t>(ci);           // physical column = insertion order
        w.put<uint8_t>(0);            // hidden
        w.put<uint8_t>(c.locked ? 1 : 0);
        w.put<float>(0.0f);           // DisplayParams {blue, red, colorscale}
        w.put<float>(1.0f);
        w.put<int32_t>(0);
        w.str("");                    // formula
    }
    w.put<int32_t>((int32_t)nnodes);
    const auto& st = h.state();
    if (graph) {
        int64_t k = 0;
        for (int x = 0; x < C_cols; x++)
            for (int y = 0; y < C_rows; y++) {
                if (!(st[h.index(x, y)] & CELL_FILLED)) continue;
                if (k >= nnodes) { err = "more filled cells than nodes"; return -1; }
                w.put<int32_t>(pixref(x, y));   // AttributeKey
                w.put<int64_t>(1);              // row layer key
                w.put<uint32_t>((uint32_t)cols.size());
                for (const ChunkColumn& c : cols) w.put<float>(c.values[k]);
                k++;
            }
        if (k != nnodes) { err = "node count does not match the filled cells"; return -1; }
    }
    w.put<float>(0.0f);   // table DisplayParams
    w.put<float>(1.0f);
    w.put<int32_t>(0);
    // ---- points, x-major (ColumnMatrix storage order)
    int64_t k = 0, ro = 0;
    for (int x = 0; x < C_cols; x++)
        for (int y = 0; y < C_rows; y++) {
            const int32_t s = st[h.index(x, y)];
            const bool node = graph && (s & CELL_FILLED) != 0;
            w.put<int32_t>(s);
            w.put<int32_t>(0);   // m_block
            w.put<int32_t>(0);   // dummy
            w.put<int8_t>(node ? (int8_t)gridconn[k] : 0);
            // m_merge: PixelRef {short x, short y} of the partner, NoPixel = (-1, -1)
            const int32_t mc = h.merge().empty() ? -1 : h.merge()[(size_t)h.index(x, y)];
            w.put<int16_t>(mc >= 0 ? (int16_t)(mc / C_rows) : (int16_t)-1);
            w.put<int16_t>(mc >= 0 ? (int16_t)(mc % C_rows) : (int16_t)-1);
            w.put<uint8_t>(node ? 1 : 0);
            if (node) {
                for (int b = 0; b < 32; b++) {
                    const int32_t* bn = bins + ((size_t)k * 32 + b) * 4;
                    const uint8_t dir = (uint8_t)bn[0];
                    const uint16_t count = (uint16_t)bn[1];
                    float dist;
                    std::memcpy(&dist, &bn[2], 4);
                    const int nr = bn[3];
                    w.put<uint8_t>(dir);
                    w.put<uint16_t>(count);
                    w.put<float>(dist);
                    w.put<float>(0.0f);   // m_occ_distance
                    const int16_t* r = runs + ro * 4;
                    if (count) {
                        if (nr == 0) { err = "bin with a node count but no runs"; return -1; }
                        if (dir & DIR_DIAG) {
                            w.put<int16_t>(r[0]);
                            w.put<int16_t>(r[1]);
                            w.put<uint16_t>((uint16_t)(r[2] - r[0]));
                        } else {
                            const uint16_t len = (uint16_t)nr;
                            w.put<uint16_t>(len);
                            w.put<int16_t>(r[0]);
                            w.put<int16_t>(r[1]);
                            w.put<uint16_t>((uint16_t)((dir & DIR_V) ? r[3] - r[1] : r[2] - r[0]));
                            for (int i = 1; i < len; i++) {
                                const int16_t* c = r + 4 * i;
                                const int16_t* p = r + 4 * (i - 1);
                                if (dir & DIR_V) {
                                    w.put<int16_t>(c[1]);
                                    w.put<uint16_t>(shift_length(c[0] - p[0], c[3] - c[1]));
                                } else {
                                    w.put<int16_t>(c[0]);
                                    w.put<uint16_t>(shift_length(c[1] - p[1], c[2] - c[0]));
                                }
                            }
                        }
                    }
                    ro += nr;
                }
                for (int b = 0; b < 32; b++) w.put<uint32_t>(0);   // empty occlusion bins
                k++;
            }
            const Vec2 loc = h.cell_centre(x, y);
            w.put<double>(loc.x);
            w.put<double>(loc.y);
        }
    if (graph && ro != nruns) { err = "run count does not match the bins"; return -1; }
    w.put<uint8_t>(graph ? 1 : 0);     // m_processed
    w.put<uint8_t>(graph && boundary ? 1 : 0);  // m_boundarygraph
    return 0;
}

int write_parsed_chunk(const ParsedChunk& pc, std::vector<uint8_t>& out, std::string& err) {
    out.clear();
    Writer w{out};
    const int ncols = (int)pc.columns.size();
    const int64_t nrows = (int64_t)pc.row_keys.size();
    for (const auto& c : pc.columns)
        if ((int64_t)c.values.size() != nrows) { err = "column length does not match the attribute rows"; return -1; }
    w.str(pc.name);
    w.put<double>(pc.spacing);
    w.put<int32_t>(pc.rows);
    w.put<int32_t>(pc.cols);
    w.put<int32_t>(pc.filled);
    w.put<double>(pc.blx);
    w.put<double>(pc.bly);
    std::vector<int> order(ncols);
    std::iota(order.begin(), order.end(), 0);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return pc.columns[a].name < pc.columns[b].name; });
    // AttributeTable::getColumnSortedIndex (attributetable.cpp:479-485)
    int32_t sd = pc.displayed_phys;
    if (sd >= 0) {
        if (sd >= ncols) sd = -1;
        else
            for (int i = 0; i < ncols; i++)
                if (order[i] == pc.displayed_phys) sd = i;
    }
    w.put<int32_t>(sd);
    out.insert(out.end(), pc.layers_raw.begin(), pc.layers_raw.end());
    w.put<int32_t>(ncols);
    for (int ci : order) {
        const ChunkColumn& c = pc.columns[ci];
        float mn = c.min, mx = c.max;
        double tot = c.total;
        if (!c.from_file) {
            const Stats s = replay_stats(c.values.data(), c.set.empty() ? nullptr : c.set.data(), nrows);
            mn = (float)s.min;
            mx = (float)s.max;
            tot = s.total;
        }
        w.str(c.name);
        w.put<float>(mn);
        w.put<float>(mx);
        w.put<double>(tot);
        w.put<int32_t>(ci);
        w.put<uint8_t>(c.hidden);
        w.put<uint8_t>(c.locked ? 1 : 0);
        out.insert(out.end(), c.display, c.display + 12);
        w.str(c.formula);
    }
    w.put<int32_t>((int32_t)nrows);
    for (int64_t i = 0; i < nrows; i++) {
        w.put<int32_t>(pc.row_keys[i]);
        w.put<int64_t>(i < (int64_t)pc.row_layers.size() ? pc.row_layers[i] : 1);
        w.put<uint32_t>((uint32_t)ncols);
        for (const ChunkColumn& c : pc.columns) w.put<float>(c.values[i]);
    }
    out.insert(out.end(), pc.table_display, pc.table_display + 12);
    out.insert(out.end(), pc.points_raw.begin(), pc.points_raw.end());
    w.put<uint8_t>(pc.processed ? 1 : 0);
    w.put<uint8_t>(pc.boundary ? 1 : 0);
    return 0;
}

int chunk_set_column(ParsedChunk& pc, const std::string& name, const float* values, const uint8_t* set, bool locked) {
    const int64_t nrows = (int64_t)pc.row_keys.size();
    int idx = -1;
    for (size_t i = 0; i < pc.columns.size(); i++)
        if (pc.columns[i].name == name) idx = (int)i;
    if (idx < 0) {   // addColumnInternal: appended, default display params, every row -1
        ChunkColumn c;
        c.name = name;
        pc.columns.push_back(c);
        idx = (int)pc.columns.size() - 1;
    }
    ChunkColumn& c = pc.columns[idx];   // reset: stats default, values -1, lock as asked
    c.from_file = false;
    c.locked = locked;
    c.values.assign((size_t)nrows, -1.0f);
    c.set.assign((size_t)nrows, 0);
    for (int64_t i = 0; i < nrows; i++)
        if (!set || set[i]) {
            c.values[i] = values[i];
            c.set[i] = 1;
        }
    return idx;
}

int chunk_unmake(ParsedChunk& pc, bool remove_links, std::string& err) {
    std::vector<uint8_t> pts;
    const size_t C = (size_t)pc.cols * pc.rows;
    if (pc.point_off.size() != C + 1) { err = "chunk has no point records"; return -1; }
    std::vector<uint64_t> off(C + 1, 0);
    for (size_t i = 0; i < C; i++) {
        const uint8_t* rec = pc.points_raw.data() + pc.point_off[i];
        const size_t len = (size_t)(pc.point_off[i + 1] - pc.point_off[i]);
        off[i] = pts.size();
        int32_t st;
        std::memcpy(&st, rec, 4);
        if (!(st & CELL_FILLED)) {
            pts.insert(pts.end(), rec, rec + len);
            continue;
        }
        st &= ~CELL_BLOCKED;                            // setBlock(false)
        const size_t at = pts.size();
        pts.insert(pts.end(), rec, rec + 18);           // state, block, dummy, grid conn, merge, has_node
        std::memcpy(&pts[at], &st, 4);
        pts[at + 12] = 0;                               // m_grid_connections
        if (remove_links) std::memset(&pts[at + 13], 0xFF, 4);   // m_merge = NoPixel
        pts[at + 17] = 0;                               // m_node = nullptr
        pts.insert(pts.end(), rec + len - 16, rec + len);   // m_location
    }
    off[C] = pts.size();
    pc.points_raw.swap(pts);
    pc.point_off.swap(off);
    pc.columns.clear();                                 // m_attributes->clear(): columns and rows
    pc.row_keys.clear();
    pc.row_layers.clear();
    pc.processed = false;
    pc.boundary = false;
    pc.displayed_phys = -2;
    pc.gridconn.clear();
    pc.bins.clear();
    pc.runs.clear();
    for (size_t i = 0; i < C; i++) pc.state[i] &= ~CELL_BLOCKED;
    return 0;
}

int read_pointmap_chunk(const uint8_t* buf, size_t size, ParsedChunk& pc, std::string& err) {
    Reader r{buf, size};
    pc = ParsedChunk();
    pc.name = r.str();
    pc.spacing = r.get<double>();
    pc.rows = r.get<int32_t>();
    pc.cols = r.get<int32_t>();
    pc.filled = r.get<int32_t>();
    pc.blx = r.get<double>();
    pc.bly = r.get<double>();
    pc.displayed_sorted = r.get<int32_t>();
    pc.displayed_phys = pc.displayed_sorted;   // PointMap::read: setDisplayedAttribute(value read)
    const size_t lay0 = r.o;
    (void)r.get<int64_t>();
    (void)r.get<int64_t>();
    const int32_t nlayers = r.get<int32_t>();
    for (int i = 0; i < nlayers && r.ok; i++) {
        (void)r.get<int64_t>();
        (void)r.str();
    }
    if (!r.ok || nlayers < 0) { err = "not a PointMap chunk"; return -1; }
    pc.layers_raw.assign(buf + lay0, buf + r.o);
    const int32_t ncols = r.get<int32_t>();
    if (!r.ok || ncols < 0 || ncols > 4096 || pc.rows <= 0 || pc.cols <= 0) { err = "not a PointMap chunk"; return -1; }
    std::vector<ChunkColumn> sorted(ncols);
    std::vector<int> phys(ncols);
    for (int i = 0; i < ncols && r.ok; i++) {
        sorted[i].name = r.str();
        sorted[i].min = r.get<float>();
        sorted[i].max = r.get<float>();
        sorted[i].total = r.get<double>();
        phys[i] = r.get<int32_t>();
        sorted[i].hidden = r.get<uint8_t>();
        sorted[i].locked = r.get<uint8_t>() != 0;
        if (r.o + 12 <= size) std::memcpy(sorted[i].display, buf + r.o, 12);
        r.o += 12;
        sorted[i].formula = r.str();
        sorted[i].from_file = true;
    }
    pc.columns.assign(ncols, ChunkColumn());
    for (int i = 0; i < ncols; i++) {
        if (phys[i] < 0 || phys[i] >= ncols) { err = "bad physical column"; return -1; }
        pc.columns[phys[i]] = sorted[i];
    }
    const int32_t nrows = r.get<int32_t>();
    // a row takes >= 16 bytes: a count beyond what is left is damage, not an allocation
    if (!r.ok || nrows < 0 || (size_t)nrows * 16 > size - r.o) { err = "truncated attribute table"; return -1; }
    for (auto& c : pc.columns) c.values.assign(nrows, -1.0f);
    pc.row_keys.resize(nrows);
    pc.row_layers.resize(nrows);
    for (int32_t i = 0; i < nrows && r.ok; i++) {
        pc.row_keys[i] = r.get<int32_t>();
        pc.row_layers[i] = r.get<int64_t>();
        const uint32_t n = r.get<uint32_t>();
        for (uint32_t j = 0; j < n && r.ok; j++) {
            const float v = r.get<float>();
            if ((int)j < ncols) pc.columns[j].values[i] = v;
        }
    }
    if (r.o + 12 <= size) std::memcpy(pc.table_display, buf + r.o, 12);
    r.o += 12;
    const int64_t C = (int64_t)pc.cols * pc.rows;
    // Point::write takes >= 30 bytes per cell
    if (r.o > size || (uint64_t)C * 30 > (uint64_t)(size - r.o)) { err = "truncated point records"; return -1; }
    pc.state.resize(C);
    pc.gridconn.clear();
    pc.bins.clear();
    pc.runs.clear();
    pc.points_raw.clear();
    pc.point_off.assign((size_t)C + 1, 0);
    pc.merges = 0;
    pc.merge_pairs.clear();
    for (int x = 0; x < pc.cols && r.ok; x++)
        for (int y = 0; y < pc.rows && r.ok; y++) {
            const size_t rec0 = r.o;
            pc.state[(int64_t)x * pc.rows + y] = r.get<int32_t>();
            (void)r.get<int32_t>();
            (void)r.get<int32_t>();
            const int8_t gc = r.get<int8_t>();
            const int32_t merge = r.get<int32_t>();
            if (merge != -1) {   // PixelRef NoPixel = (-1, -1); {short x, short y} little-endian
                pc.merges++;
                const int mx = (int16_t)(merge & 0xFFFF), my = (int16_t)((uint32_t)merge >> 16);
                pc.merge_pairs.push_back((int32_t)((int64_t)x * pc.rows + y));
                pc.merge_pairs.push_back((int32_t)((int64_t)mx * pc.rows + my));
            }
            const bool node = r.get<uint8_t>() != 0;
            if (node) {
                pc.gridconn.push_back((uint8_t)gc);
                for (int b = 0; b < 32 && r.ok; b++) {
                    const uint8_t dir = r.get<uint8_t>();
                    const uint16_t count = r.get<uint16_t>();
                    const float dist = r.get<float>();
                    (void)r.get<float>();
                    int32_t bn[4] = {dir, count, 0, 0};
                    std::memcpy(&bn[2], &dist, 4);
                    if (count) {
                        if (dir & DIR_DIAG) {
                            const int16_t sx = r.get<int16_t>(), sy = r.get<int16_t>();
                            const uint16_t len = r.get<uint16_t>();
                            const int16_t ey = (dir == DIR_PD) ? (int16_t)(sy + len) : (int16_t)(sy - len);
                            pc.runs.insert(pc.runs.end(), {sx, sy, (int16_t)(sx + len), ey});
                            bn[3] = 1;
                        } else {
                            const uint16_t n = r.get<uint16_t>();
                            int16_t px = r.get<int16_t>(), py = r.get<int16_t>();
                            const uint16_t len0 = r.get<uint16_t>();
                            if (dir & DIR_V) pc.runs.insert(pc.runs.end(), {px, py, px, (int16_t)(py + len0)});
                            else pc.runs.insert(pc.runs.end(), {px, py, (int16_t)(px + len0), py});
                            for (int i = 1; i < n && r.ok; i++) {
                                const int16_t primary = r.get<int16_t>();
                                const uint16_t sl = r.get<uint16_t>();
                                const int shift = sl & 0xF, len = sl >> 4;
                                if (dir & DIR_V) {
                                    px = (int16_t)(px + shift);
                                    py = primary;
                                    pc.runs.insert(pc.runs.end(), {px, py, px, (int16_t)(py + len)});
                                } else {
                                    px = primary;
                                    py = (int16_t)(py + shift);
                                    pc.runs.insert(pc.runs.end(), {px, py, (int16_t)(px + len), py});
                                }
                            }
                            bn[3] = n;
                        }
                    }
                    pc.bins.insert(pc.bins.end(), bn, bn + 4);
                }
                for (int b = 0; b < 32 && r.ok; b++) {
                    const uint32_t n = r.get<uint32_t>();
                    r.o += (size_t)n * 4;   // occlusion bins (PixelRef entries)
                }
            }
            (void)r.get<double>();
            (void)r.get<double>();
            if (!r.ok) break;
            // the record as Point::write re-emits it: PointMap::read masks the state (pointdata.cpp:1128)
            // and Point::write writes a zero dummy (point.cpp:57-58)
            const size_t at = pc.points_raw.size();
            pc.point_off[(size_t)x * pc.rows + y] = at;
            pc.points_raw.insert(pc.points_raw.end(), buf + rec0, buf + r.o);
            int32_t st = pc.state[(int64_t)x * pc.rows + y] & (CELL_EMPTY | CELL_FILLED | CELL_MERGED | CELL_BLOCKED |
                                                               CELL_CONTEXTFILLED | CELL_EDGE);
            std::memcpy(&pc.points_raw[at], &st, 4);
            std::memset(&pc.points_raw[at + 8], 0, 4);
        }
    pc.point_off[(size_t)C] = pc.points_raw.size();
    pc.processed = r.get<uint8_t>() != 0;
    pc.boundary = r.get<uint8_t>() != 0;
    if (!r.ok) { err = "truncated PointMap chunk"; return -1; }
    pc.bytes_used = r.o;
    return 0;
}

} // namespace dmx
