// dmx_salalib.cpp -- salalib-side binding of libdmx.so (see dmx_salalib.h).
//
// Compiled against the reference headers (integration/Makefile: -I/root/reference), it uses only the
// reference's public interface plus one pointer-to-member read of PointMap::m_parentRegion (protected,
// reached through a derived accessor, legal C++).  The engine and the reference exchange a map as the
// PointMap::write image (pointdata.cpp:1158-1188): the engine's writer is byte-identical to the
// reference's (tests/test_graphfile.py), and the reference's own PointMap::read (:1073-1156) turns it
// back into Points, Nodes, the attribute table and its statistics.
#include "dmx_salalib.h"

#include <cstdint>
#include <cstring>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "dmx.h"
#include "genlib/comm.h"
#include "genlib/exceptions.h"
#include "salalib/pointdata.h"

namespace dmxsala {
namespace {

// PointMap keeps the MetaGraph region it was made for by pointer (protected); a derived class may
// name the member, and the pointer-to-member then reads it from any PointMap.
struct RegionAccess : PointMap {
    static const QtRegion* parent(const PointMap& m) { return m.*(&RegionAccess::m_parentRegion); }
};

void check(int status) {
    if (status == DMX_ERR_CANCELLED) throw Communicator::CancelledException();
    if (status != DMX_OK) throw depthmapX::RuntimeException(std::string("libdmx: ") + dmx_last_error());
}

// One engine context per process (one process per GPU).  nullptr when no device is usable: the
// caller falls back to the reference's CPU code.
dmx_ctx* context() {
    static dmx_ctx* ctx = nullptr;
    static bool tried = false;
    if (!tried) {
        tried = true;
        if (dmx_ctx_create(0, &ctx) != DMX_OK) ctx = nullptr;
    }
    return ctx;
}

// Communicator bridge: NUM_RECORDS / CURRENT_RECORD posts and IsCancelled polls, every 0.5 s as the
// reference's qtimer(atime, 500) loops do (pointdata.cpp:1301-1316, vgavisualglobal.cpp:195-202).
struct Progress {
    Communicator* comm;
    bool posted_total = false;
    static int32_t fn(void* user, int32_t, int64_t done, int64_t total) {
        Progress* p = static_cast<Progress*>(user);
        if (!p->posted_total) {
            p->comm->CommPostMessage(Communicator::NUM_RECORDS, (int)total);
            p->posted_total = true;
        }
        p->comm->CommPostMessage(Communicator::CURRENT_RECORD, (int)done);
        return p->comm->IsCancelled() ? 1 : 0;
    }
};

struct ScopedProgress {
    dmx_ctx* ctx;
    Progress p;
    ScopedProgress(dmx_ctx* c, Communicator* comm) : ctx(c), p{comm} {
        if (comm) check(dmx_ctx_set_progress(ctx, &Progress::fn, &p, 0.5));
    }
    ~ScopedProgress() { dmx_ctx_set_progress(ctx, nullptr, nullptr, 0.0); }
};

template <class T, int (*F)(T*)>
struct Owned {
    T* p = nullptr;
    ~Owned() {
        if (p) F(p);
    }
};

std::string serialize(const dmx_chunk* c) {
    int64_t size = 0;
    check(dmx_chunk_serialize(c, nullptr, 0, &size));
    std::string out((size_t)size, '\0');
    check(dmx_chunk_serialize(c, reinterpret_cast<uint8_t*>(&out[0]), size, &size));
    return out;
}

std::string save(PointMap& map) {
    std::ostringstream os(std::ios::out | std::ios::binary);
    map.write(os);
    return os.str();
}

// PointMap::read fills a map object from scratch (MetaGraph::readPointMaps reads into a new map):
// read into a fresh map on the same region and drawing, then move it over `map`.
bool load(PointMap& map, const std::string& bytes) {
    const QtRegion* region = RegionAccess::parent(map);
    PointMap fresh(*region, map.getDrawingFiles(), map.getName());
    std::istringstream is(bytes, std::ios::in | std::ios::binary);
    if (!fresh.read(is)) return false;
    map = std::move(fresh);
    return true;
}

// The drawing lines PointMap::blockLines rasterises (pointdata.cpp:311-321): every shown layer.
std::vector<double> drawing_lines(PointMap& map) {
    std::vector<double> lines;
    for (const auto& file : map.getDrawingFiles())
        for (const auto& layer : file.m_spacePixels)
            if (layer.isShown())
                for (const auto& l : layer.getAllShapesAsLines()) {
                    lines.push_back(l.start().x);
                    lines.push_back(l.start().y);
                    lines.push_back(l.end().x);
                    lines.push_back(l.end().y);
                }
    return lines;
}

}  // namespace

bool saveMap(PointMap& map, void* bytes_out) {
    *static_cast<std::string*>(bytes_out) = save(map);
    return true;
}

bool loadMap(PointMap& map, const void* bytes) { return load(map, *static_cast<const std::string*>(bytes)); }

bool sparkGraph2(PointMap& map, Communicator* comm, bool boundarygraph, double maxdist) {
    dmx_ctx* ctx = context();
    // a processed map keeps the reference path (its sparkGraph2 re-adds attribute rows that exist and
    // throws, attributetable.cpp:278)
    if (!ctx || map.isProcessed()) return false;
    const QtRegion* parent = RegionAccess::parent(map);
    const double region[4] = {parent->bottom_left.x, parent->bottom_left.y, parent->top_right.x, parent->top_right.y};
    const std::vector<double> lines = drawing_lines(map);
    Owned<dmx_pointmap, dmx_pointmap_free> pm;
    check(dmx_pointmap_create(region, map.getSpacing(), lines.data(), (int64_t)lines.size() / 4, &pm.p));
    // the engine's grid is PointMap::setGrid(spacing, (0,0)) on the MetaGraph region (the CLI's grid);
    // a map gridded with another offset stays on the reference path
    int32_t cols = 0, rows = 0;
    double blx = 0, bly = 0;
    check(dmx_pointmap_info(pm.p, &cols, &rows, &blx, &bly, nullptr));
    const Point2f bl = map.depixelate(PixelRef(0, 0));
    if ((size_t)cols != map.getCols() || (size_t)rows != map.getRows() || blx != bl.x || bly != bl.y) return false;
    std::vector<int32_t> state((size_t)cols * rows);
    for (int32_t x = 0; x < cols; x++)
        for (int32_t y = 0; y < rows; y++)
            state[(size_t)x * rows + y] = map.getPoint(PixelRef((short)x, (short)y)).getState();
    check(dmx_pointmap_set_state(pm.p, state.data()));
    // merge links stay on the points and are written back with them (Point::write, point.cpp:51-73)
    std::vector<int32_t> links;
    for (const auto& pr : map.getMergedPixelPairs()) {
        links.push_back((int32_t)pr.first.x * rows + pr.first.y);
        links.push_back((int32_t)pr.second.x * rows + pr.second.y);
    }
    if (!links.empty()) check(dmx_pointmap_set_merges(pm.p, links.data(), (int64_t)links.size() / 2));
    // makeGraph on the GPU
    Owned<dmx_graph, dmx_graph_free> g;
    {
        ScopedProgress sp(ctx, comm);
        check(dmx_makegraph(ctx, pm.p, maxdist, boundarygraph ? 1 : 0, 0, -1, &g.p));
    }
    int64_t n = 0, nb = 0, ne = 0, nruns = 0;
    check(dmx_graph_info(g.p, &n, &nb, &ne, &nruns));
    std::vector<float> attrs((size_t)n * 3);
    std::vector<int32_t> bins((size_t)n * 32 * 4);
    std::vector<int16_t> runs((size_t)std::max<int64_t>(nruns, 1) * 4);
    std::vector<uint8_t> gridconn((size_t)n);
    check(dmx_graph_copy(g.p, attrs.data(), bins.data(), runs.data(), gridconn.data()));
    // the columns sparkGraph2 creates (pointdata.cpp:1266-1270: Connectivity locked), displayed =
    // Connectivity, then the image the reference would write for the made map
    const char* names[3] = {"Connectivity", "Point First Moment", "Point Second Moment"};
    std::vector<float> values((size_t)n * 3);
    for (int j = 0; j < 3; j++)
        for (int64_t k = 0; k < n; k++) values[(size_t)j * n + k] = attrs[(size_t)k * 3 + j];
    const uint8_t locked[3] = {1, 0, 0};
    int64_t size = 0;
    check(dmx_chunk_write(pm.p, n, bins.data(), runs.data(), nruns, gridconn.data(), 3, names, values.data(), locked,
                          nullptr, 0, boundarygraph ? 1 : 0, nullptr, 0, &size));
    std::string img((size_t)size, '\0');
    check(dmx_chunk_write(pm.p, n, bins.data(), runs.data(), nruns, gridconn.data(), 3, names, values.data(), locked,
                          nullptr, 0, boundarygraph ? 1 : 0, reinterpret_cast<uint8_t*>(&img[0]), size, &size));
    Owned<dmx_chunk, dmx_chunk_free> c;
    check(dmx_chunk_parse(reinterpret_cast<const uint8_t*>(img.data()), (int64_t)img.size(), &c.p));
    check(dmx_chunk_set_name(c.p, map.getName().c_str()));
    return load(map, serialize(c.p));
}

bool vgaVisualGlobal(PointMap& map, Communicator* comm, double radius, bool gates_only, bool simple_version) {
    dmx_ctx* ctx = context();
    if (!ctx || !map.isProcessed()) return false;
    const std::string img = save(map);
    Owned<dmx_chunk, dmx_chunk_free> c;
    check(dmx_chunk_parse(reinterpret_cast<const uint8_t*>(img.data()), (int64_t)img.size(), &c.p));
    const QtRegion* parent = RegionAccess::parent(map);
    const double region[4] = {parent->bottom_left.x, parent->bottom_left.y, parent->top_right.x, parent->top_right.y};
    Owned<dmx_pointmap, dmx_pointmap_free> pm;
    Owned<dmx_graph, dmx_graph_free> g;
    check(dmx_chunk_load(ctx, c.p, region, &pm.p, &g.p));
    int64_t n = 0, nb = 0, ne = 0, nruns = 0;
    check(dmx_graph_info(g.p, &n, &nb, &ne, &nruns));
    std::vector<float> out((size_t)n * 7);
    {
        ScopedProgress sp(ctx, comm);
        const int rc = dmx_vga_global(ctx, g.p, radius, gates_only ? 1 : 0, 0, -1, out.data(), nullptr);
        // a configuration the engine does not take (none on this path since round 5: the searches whose result
        // depends on the reference's pop order are re-run in that order, vga_ordered.hip): the reference path
        if (rc == DMX_ERR_UNSUPPORTED) return false;
        check(rc);
    }
    // VGAVisualGlobal::run's columns (vgavisualglobal.cpp:31-63), alphabetical, " R<r>" suffix for a
    // finite radius; a source the reference skips sets nothing, and the HH / P-value / Tekl values need
    // more than one node; displayed = Visual Integration [HH] (:212)
    const std::string suffix = radius != -1 ? " R" + std::to_string((int)radius) : std::string();
    struct Col {
        const char* name;
        int k;
        bool in_simple;
    };
    const Col cols[7] = {{"Visual Entropy", 0, false},         {"Visual Integration [HH]", 1, true},
                         {"Visual Integration [P-value]", 2, false}, {"Visual Integration [Tekl]", 3, false},
                         {"Visual Mean Depth", 4, false},      {"Visual Node Count", 5, false},
                         {"Visual Relativised Entropy", 6, false}};
    std::vector<float> v((size_t)n);
    std::vector<uint8_t> set((size_t)n);
    for (const Col& col : cols) {
        if (simple_version && !col.in_simple) continue;
        for (int64_t i = 0; i < n; i++) {
            const float nodes = out[(size_t)i * 7 + 5];
            const bool ran = nodes >= 1.0f;
            set[i] = (ran && (col.k < 1 || col.k > 3 || nodes > 1.0f)) ? 1 : 0;
            v[i] = out[(size_t)i * 7 + col.k];
        }
        check(dmx_chunk_set_column(c.p, (std::string(col.name) + suffix).c_str(), v.data(), set.data(), 0, col.k == 1));
    }
    return load(map, serialize(c.p));
}

}  // namespace dmxsala
