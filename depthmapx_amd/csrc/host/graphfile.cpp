// graphfile.cpp -- the depthmapX .graph container (see graphfile.hpp for the reference map).
#include "graphfile.hpp"

#include <algorithm>
#include <cstring>

namespace dmx {

namespace {

struct Rd {
    const uint8_t* p;
    size_t n, o = 0;
    bool ok = true;
    template <typename T> T get() {
        T v{};
        if (sizeof(T) > n - o) { ok = false; o = n; return v; }
        std::memcpy(&v, p + o, sizeof(T));
        o += sizeof(T);
        return v;
    }
    void skip(size_t k) {   // (o <= n always: the tests cannot overflow)
        if (k > n - o) { ok = false; o = n; return; }
        o += k;
    }
    std::string str() {   // dXstring::readString: u32 length + bytes
        const uint32_t len = get<uint32_t>();
        if (!ok || len > n - o) { ok = false; o = n; return std::string(); }
        std::string s(reinterpret_cast<const char*>(p + o), len);
        o += len;
        return s;
    }
    bool eof() const { return o >= n; }
};

struct Wr {
    std::vector<uint8_t>& b;
    template <typename T> void put(const T& v) {
        const uint8_t* q = reinterpret_cast<const uint8_t*>(&v);
        b.insert(b.end(), q, q + sizeof(T));
    }
    void str(const std::string& s) {
        put<uint32_t>((uint32_t)s.size());
        b.insert(b.end(), s.begin(), s.end());
    }
    void raw(const std::vector<uint8_t>& v) { b.insert(b.end(), v.begin(), v.end()); }
};

// AttributeTable::read (attributetable.cpp:397-425): layer manager, columns, rows, display params
bool skip_attribute_table(Rd& r) {
    r.get<int64_t>();
    r.get<int64_t>();
    const int32_t nl = r.get<int32_t>();
    if (!r.ok || nl < 0) return false;
    for (int i = 0; i < nl && r.ok; i++) {
        r.get<int64_t>();
        r.str();
    }
    const int32_t nc = r.get<int32_t>();
    if (!r.ok || nc < 0) return false;
    for (int i = 0; i < nc && r.ok; i++) {
        r.str();
        r.skip(4 + 4 + 8 + 4 + 1 + 1 + 12);   // min, max, total, physical column, hidden, locked, DisplayParams
        r.str();                               // formula
    }
    const int32_t nr = r.get<int32_t>();
    if (!r.ok || nr < 0) return false;
    for (int i = 0; i < nr && r.ok; i++) {
        r.skip(4 + 8);                         // key, layer key
        const uint32_t k = r.get<uint32_t>();
        r.skip((size_t)k * 4);
    }
    r.skip(12);
    return r.ok;
}

// ShapeMap::read (shapemap.cpp:2273-2383)
bool read_layer(Rd& r, GfLayer& L) {
    L.name = r.str();
    L.map_type = r.get<int32_t>();
    L.show = r.get<uint8_t>();
    L.editable = r.get<uint8_t>();
    for (int i = 0; i < 4; i++) L.region[i] = r.get<double>();
    L.rows = r.get<int32_t>();
    L.cols = r.get<int32_t>();
    L.obj_ref = r.get<int32_t>();
    r.get<int32_t>();   // largest shape ref (recomputed on write)
    const int32_t ns = r.get<int32_t>();
    // a stored shape takes >= 81 bytes: counts beyond what is left are damage, not an allocation
    if (!r.ok || ns < 0 || (size_t)ns * 81 > r.n - r.o) return false;
    L.shapes.resize((size_t)ns);
    for (auto& s : L.shapes) {
        s.key = r.get<int32_t>();
        s.type = r.get<uint8_t>();
        for (int i = 0; i < 4; i++) s.region[i] = r.get<double>();
        s.bits[0] = r.get<uint8_t>();
        s.bits[1] = r.get<uint8_t>();
        for (int i = 0; i < 6; i++) s.pad[i] = r.get<uint8_t>();   // padding of Line (sizeof 40)
        s.centroid[0] = r.get<double>();
        s.centroid[1] = r.get<double>();
        s.area = r.get<double>();
        s.perimeter = r.get<double>();
        const uint32_t np = r.get<uint32_t>();
        if (!r.ok || (size_t)np * 16 > r.n - r.o) return false;
        s.pts.resize((size_t)np * 2);
        for (auto& v : s.pts) v = r.get<double>();
    }
    std::stable_sort(L.shapes.begin(), L.shapes.end(), [](const GfShape& a, const GfShape& b) { return a.key < b.key; });
    // object data (unused): skipped, written back as an empty list
    const int32_t nobj = r.get<int32_t>();
    for (int i = 0; i < nobj && r.ok; i++) {
        r.get<int32_t>();
        const uint32_t sz = r.get<uint32_t>();
        r.skip((size_t)sz * 4);
    }
    const size_t t0 = r.o;
    if (!skip_attribute_table(r)) return false;
    L.table_raw.assign(r.p + t0, r.p + r.o);
    L.displayed = r.get<int32_t>();
    const size_t c0 = r.o;
    const int32_t nconn = r.get<int32_t>();   // Connector::read (connector.cpp:28-43)
    for (int i = 0; i < nconn && r.ok; i++) {
        const uint32_t nc = r.get<uint32_t>();
        r.skip((size_t)nc * 4);
        r.get<int32_t>();
        for (int m = 0; m < 2 && r.ok; m++) {
            const uint32_t ne = r.get<uint32_t>();
            r.skip((size_t)ne * 12);   // std::map<SegmentRef(8 B), float>
        }
    }
    for (int m = 0; m < 2 && r.ok; m++) {   // m_links, m_unlinks: OrderedIntPair vectors
        const uint32_t ne = r.get<uint32_t>();
        r.skip((size_t)ne * 8);
    }
    if (!r.ok) return false;
    L.links_raw.assign(r.p + c0, r.p + r.o);
    const size_t m0 = r.o;
    const uint8_t x = r.get<uint8_t>();
    if (x == 'm') {   // MapInfoData::read (parsers/mapinfodata.cpp:558-567)
        r.str();
        r.str();
        r.skip(1);
        r.str();
        r.str();
        r.str();
        L.mapinfo_raw.assign(r.p + m0, r.p + r.o);
    } else {
        L.mapinfo_raw.assign(1, (uint8_t)'x');   // ShapeMap::write puts 'x' when there is none
    }
    return r.ok;
}

void write_layer(Wr& w, const GfLayer& L) {   // ShapeMap::write (shapemap.cpp:2385-2449)
    w.str(L.name);
    w.put<int32_t>(L.map_type);
    w.put<uint8_t>(L.show);
    w.put<uint8_t>(L.editable);
    for (int i = 0; i < 4; i++) w.put<double>(L.region[i]);
    w.put<int32_t>(L.rows);
    w.put<int32_t>(L.cols);
    w.put<int32_t>(L.obj_ref);
    w.put<int32_t>(L.shapes.empty() ? -1 : L.shapes.back().key);
    w.put<int32_t>((int32_t)L.shapes.size());
    for (const auto& s : L.shapes) {
        w.put<int32_t>(s.key);
        w.put<uint8_t>(s.type);   // SalaShape::write (shapemap.cpp:68-76) of a copied shape
        for (int i = 0; i < 4; i++) w.put<double>(s.region[i]);
        w.put<uint8_t>(s.bits[0]);
        w.put<uint8_t>(s.bits[1]);
        // The 6 padding bytes after Line::bits are whatever the copy in `for (auto shape : m_shapes)`
        // holds: measured on the reference build, a line shape's copy carries the bytes it was read
        // with and every other shape's copy comes out zeroed (gallery_empty, gallery_connected,
        // turns_connected, polygons_drawing, barnsbury_drawing, rect1x1).
        for (int i = 0; i < 6; i++) w.put<uint8_t>(s.type == 0x02 ? s.pad[i] : 0);
        w.put<double>(s.centroid[0]);
        w.put<double>(s.centroid[1]);
        w.put<double>(s.area);
        w.put<double>(s.perimeter);
        w.put<uint32_t>((uint32_t)(s.pts.size() / 2));
        for (double v : s.pts) w.put<double>(v);
    }
    w.put<int32_t>(0);   // object data
    w.raw(L.table_raw);
    w.put<int32_t>(L.displayed);
    w.raw(L.links_raw);
    w.raw(L.mapinfo_raw);
}

bool read_pointmap_extent(Rd& r);

} // namespace

int32_t view_vga_top(int32_t vc) {
    if (vc & MG_VIEWAXIAL) return MG_VIEWBACKAXIAL | MG_VIEWVGA;
    if (vc & MG_VIEWDATA) return MG_VIEWBACKDATA | MG_VIEWVGA;
    return MG_VIEWVGA | (vc & (MG_VIEWBACKAXIAL | MG_VIEWBACKDATA));
}

std::string new_pointmap_name(const GraphFile& gf, const std::string& base) {
    std::vector<std::string> names;
    for (const auto& c : gf.pointmaps) {
        Rd r{c.data(), c.size()};
        names.push_back(r.str());
    }
    std::string name = base;
    int counter = 1;
    while (std::find(names.begin(), names.end(), name) != names.end()) name = base + " " + std::to_string(counter++);
    return name;
}

std::vector<double> graphfile_lines(const GraphFile& gf) {
    std::vector<double> out;
    for (const auto& f : gf.drawing)
        for (const auto& L : f.layers) {
            if (!L.show) continue;   // ShapeMap::isShown
            for (const auto& s : L.shapes) {
                if (s.type == 0x02) {
                    // SHAPE_LINE: SimpleLine(getLine()) takes Line::t_start() / t_end() (p2dpoly.h:462-467,
                    // 500-507): x from the direction bit, y from direction == parity
                    const bool right = s.bits[1] == 1, up = s.bits[1] == s.bits[0];
                    out.insert(out.end(), {right ? s.region[0] : s.region[2], up ? s.region[1] : s.region[3],
                                           right ? s.region[2] : s.region[0], up ? s.region[3] : s.region[1]});
                } else if ((s.type & (0x04 | 0x40)) == 0x04 || (s.type & (0x04 | 0x40)) == (0x04 | 0x40)) {
                    const size_t np = s.pts.size() / 2;   // polyline / polygon: consecutive segments
                    for (size_t k = 0; k + 1 < np; k++)
                        out.insert(out.end(), {s.pts[2 * k], s.pts[2 * k + 1], s.pts[2 * k + 2], s.pts[2 * k + 3]});
                    if ((s.type & 0x40) && np >= 1)   // closed: back to the first point
                        out.insert(out.end(), {s.pts[2 * np - 2], s.pts[2 * np - 1], s.pts[0], s.pts[1]});
                }
            }
        }
    return out;
}

int read_graphfile(const uint8_t* buf, size_t size, GraphFile& gf, std::string& err) {
    gf = GraphFile();
    Rd r{buf, size};
    if (size < 3 || buf[0] != 'g' || buf[1] != 'r' || buf[2] != 'f') { err = "not a graph file"; return -1; }
    r.o = 3;
    gf.version = r.get<int32_t>();
    if (!r.ok) { err = "not a graph file"; return -1; }
    if (gf.version != 440) {
        err = "graph file version " + std::to_string(gf.version) + " (only METAGRAPH_VERSION 440 is read here)";
        return -2;
    }
    int32_t state = r.get<int32_t>();
    gf.view_class = r.get<int32_t>();
    gf.showgrid = r.get<uint8_t>();
    gf.showtext = r.get<uint8_t>();
    uint8_t type = r.get<uint8_t>();
    if (!r.ok) { err = "damaged file header"; return -1; }
    if (type == 'd') { err = "deprecated data layers (legacy reader)"; return -2; }
    if (type == 'x') {
        for (auto& s : gf.props) s = r.str();
        if (!r.ok) { err = "damaged file properties"; return -1; }
        if (r.eof()) { gf.state = state; return 0; }
        type = r.get<uint8_t>();
    } else {
        gf.props[0] = gf.props[1] = gf.props[2] = gf.props[3] = "<unknown>";
    }
    if (r.eof() && type != 'l' && type != 'p') { gf.state = state; return 0; }
    if (type == 'v') {   // skipVirtualMem (mgraph.cpp:2760-2774)
        const int32_t nodes = r.get<int32_t>();
        if (nodes < 0) r.ok = false;
        for (int64_t i = 0; i < (int64_t)nodes * 2 && r.ok; i++) {
            const int32_t c = r.get<int32_t>();
            if (c < 0) { r.ok = false; break; }
            r.skip((size_t)c * 4);
        }
        if (!r.ok || r.eof()) { err = "damaged virtual graph section"; return -1; }
        type = r.get<uint8_t>();
    }
    if (type == 'l') {
        gf.name = r.str();
        for (int i = 0; i < 4; i++) gf.region[i] = r.get<double>();
        const int32_t nf = r.get<int32_t>();
        if (!r.ok || nf < 0 || (size_t)nf * 40 > r.n - r.o) { err = "damaged drawing section"; return -1; }
        gf.drawing.resize((size_t)nf);
        for (auto& f : gf.drawing) {
            f.name = r.str();
            for (int i = 0; i < 4; i++) f.region[i] = r.get<double>();
            const int32_t nl = r.get<int32_t>();
            if (!r.ok || nl < 0 || (size_t)nl * 8 > r.n - r.o) { err = "damaged drawing file"; return -1; }
            f.layers.resize((size_t)nl);
            for (auto& L : f.layers)
                if (!read_layer(r, L)) { err = "damaged drawing layer"; return -1; }
            if (f.name.empty()) f.name = "<unknown>";   // SpacePixelFile::read (spacepixfile.cpp:39-41)
        }
        if (gf.name.empty()) gf.name = "<unknown>";     // readFromStream (mgraph.cpp:2603-2605)
        state |= MG_LINEDATA;
        type = r.eof() ? 0 : r.get<uint8_t>();
    }
    if (type == 'p') {
        gf.displayed_pointmap = r.get<int32_t>();
        const int32_t n = r.get<int32_t>();
        if (!r.ok || n < 0) { err = "damaged point map section"; return -1; }
        for (int i = 0; i < n; i++) {
            const size_t p0 = r.o;
            if (!read_pointmap_extent(r)) { err = "damaged point map"; return -1; }
            gf.pointmaps.emplace_back(buf + p0, buf + r.o);
        }
        state |= MG_POINTMAPS;
        type = r.eof() ? 0 : r.get<uint8_t>();
    }
    if (type == 'g') {   // legacy marker: the last point map is processed
        if (!gf.pointmaps.empty()) gf.pointmaps.back()[gf.pointmaps.back().size() - 2] = 1;
        type = r.eof() ? 0 : r.get<uint8_t>();
    }
    if (type == 'a') {
        state |= MG_ANGULARGRAPH;
        type = r.eof() ? 0 : r.get<uint8_t>();
    }
    if (type == 'x' || type == 's') {
        gf.tail.assign(buf + r.o - 1, buf + size);
        gf.tail_flags = type == 'x' ? MG_SHAPEGRAPHS : MG_DATAMAPS;
        state |= gf.tail_flags;
        // a data maps section after the shape graphs cannot be located without parsing the shape
        // graphs; its flag is kept from the file's own state
    }
    gf.state = state;
    return 0;
}

int write_graphfile(const GraphFile& gf, std::vector<uint8_t>& out, std::string& err) {
    out.clear();
    Wr w{out};
    out.insert(out.end(), {'g', 'r', 'f'});
    w.put<int32_t>(440);
    w.put<int32_t>(gf.state);
    w.put<int32_t>(gf.view_class);
    w.put<uint8_t>(gf.showgrid);
    w.put<uint8_t>(gf.showtext);
    w.put<uint8_t>('x');
    for (const auto& s : gf.props) w.str(s);
    if (gf.state & MG_LINEDATA) {
        w.put<uint8_t>('l');
        w.str(gf.name);
        for (int i = 0; i < 4; i++) w.put<double>(gf.region[i]);
        w.put<int32_t>((int32_t)gf.drawing.size());
        for (const auto& f : gf.drawing) {   // SpacePixelFile::write (spacepixfile.cpp:45-57)
            w.str(f.name);
            for (int i = 0; i < 4; i++) w.put<double>(f.region[i]);
            w.put<int32_t>((int32_t)f.layers.size());
            for (const auto& L : f.layers) write_layer(w, L);
        }
    }
    if (gf.state & MG_POINTMAPS) {
        w.put<uint8_t>('p');
        w.put<int32_t>(gf.displayed_pointmap);
        w.put<int32_t>((int32_t)gf.pointmaps.size());
        for (const auto& c : gf.pointmaps) w.raw(c);
    }
    if (!gf.tail.empty() && (gf.state & gf.tail_flags)) w.raw(gf.tail);
    (void)err;
    return 0;
}

namespace {
// The extent of one PointMap record (PointMap::read pointdata.cpp:1073-1156 without decoding).
bool read_pointmap_extent(Rd& r) {
    r.str();
    r.get<double>();
    const int32_t rows = r.get<int32_t>(), cols = r.get<int32_t>();
    r.get<int32_t>();
    r.skip(16);
    r.get<int32_t>();
    if (!r.ok || rows < 0 || cols < 0) return false;
    if (!skip_attribute_table(r)) return false;
    for (int64_t i = 0; i < (int64_t)rows * cols && r.ok; i++) {
        r.skip(4 + 4 + 4 + 1 + 4);   // state, block, dummy, grid connections, merge
        const uint8_t node = r.get<uint8_t>();
        if (node) {
            for (int b = 0; b < 32 && r.ok; b++) {   // Bin::read (ngraph.cpp:420-445)
                const uint8_t dir = r.get<uint8_t>();
                const uint16_t count = r.get<uint16_t>();
                r.skip(8);
                if (count) {
                    if (dir & 12) r.skip(6);
                    else {
                        const uint16_t n = r.get<uint16_t>();
                        r.skip(6 + 4 * (size_t)(n > 0 ? n - 1 : 0));
                    }
                }
            }
            for (int b = 0; b < 32 && r.ok; b++) {
                const uint32_t n = r.get<uint32_t>();
                r.skip((size_t)n * 4);
            }
        }
        r.skip(16);
    }
    r.skip(2);
    return r.ok;
}
} // namespace

} // namespace dmx
