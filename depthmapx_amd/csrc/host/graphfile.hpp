// graphfile.hpp -- the depthmapX .graph container (MetaGraph file, METAGRAPH_VERSION 440), host side.
//
// Reader: MetaGraph::readFromStream (salalib/mgraph.cpp:2492-2654).  Writer: MetaGraph::write
// (mgraph.cpp:2656-2757) as the CLI calls it (currentlayer = false).  The drawing layers are parsed
// structurally (SpacePixelFile::read/write spacepixfile.cpp:28-57, ShapeMap::read/write
// shapemap.cpp:2273-2449, SalaShape::read/write shapemap.cpp:49-76) so that they are re-emitted the way
// the reference re-emits them, and so that PointMap::blockLines gets the visible drawing lines
// (pointdata.cpp:308-320 via ShapeMap::getAllShapesAsLines shapemap.cpp:3275-3292).  Point maps stay
// raw chunks (graphio.hpp parses and rewrites them).  Shape graphs and data maps are carried through
// verbatim.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace dmx {

// MetaGraph::m_state bits (mgraph.h:71-73) and view classes / show commands (mgraph.h:333-334)
enum : int32_t {
    MG_POINTMAPS = 0x0002, MG_LINEDATA = 0x0004, MG_ANGULARGRAPH = 0x0010, MG_DATAMAPS = 0x0020,
    MG_SHAPEGRAPHS = 0x0100
};
enum : int32_t {
    MG_VIEWVGA = 0x01, MG_VIEWBACKVGA = 0x02, MG_VIEWAXIAL = 0x04, MG_VIEWBACKAXIAL = 0x08, MG_VIEWDATA = 0x20,
    MG_VIEWBACKDATA = 0x40
};

struct GfShape {                 // SalaShape
    int32_t key = 0;
    uint8_t type = 0;
    double region[4] = {0, 0, 0, 0};   // Line m_region: bottom_left, top_right
    uint8_t bits[2] = {0, 0};          // Line::bits {parity, direction}
    uint8_t pad[6] = {0, 0, 0, 0, 0, 0};   // the Line's padding bytes as read
    double centroid[2] = {0, 0};
    double area = 0, perimeter = 0;
    std::vector<double> pts;           // [n][2]
};

struct GfLayer {                 // ShapeMap of a drawing file
    std::string name;
    int32_t map_type = 0;
    uint8_t show = 1, editable = 0;
    double region[4] = {0, 0, 0, 0};
    int32_t rows = 0, cols = 0, obj_ref = 0;
    std::vector<GfShape> shapes;       // key order (std::map)
    std::vector<uint8_t> table_raw;    // AttributeTable (layer manager, columns, rows, display params)
    int32_t displayed = -1;            // sorted index, as read and as written
    std::vector<uint8_t> links_raw;    // connectors, links, unlinks
    std::vector<uint8_t> mapinfo_raw;  // 'x', or 'm' + MapInfoData
};

struct GfDrawingFile {           // SpacePixelFile
    std::string name;
    double region[4] = {0, 0, 0, 0};
    std::vector<GfLayer> layers;
};

struct GraphFile {
    int32_t version = 440;
    int32_t state = 0, view_class = 0;
    uint8_t showgrid = 0, showtext = 0;
    std::string props[7];              // FileProperties (person, organization, date, program, title, location, description)
    std::string name;                  // MetaGraph m_name (drawing section)
    double region[4] = {0, 0, 0, 0};   // MetaGraph m_region
    std::vector<GfDrawingFile> drawing;
    int32_t displayed_pointmap = -1;
    std::vector<std::vector<uint8_t>> pointmaps;   // PointMap chunks (PointMap::write bytes)
    std::vector<uint8_t> tail;         // shape graphs / data maps sections, type byte included
    int32_t tail_flags = 0;            // MG_SHAPEGRAPHS / MG_DATAMAPS present in `tail`
};

// 0 on success; -1 not a graph / damaged (err says), -2 a version this reader does not handle
// (files older than 440 go through the reference's legacy mgraph440 reader, not on this path).
int read_graphfile(const uint8_t* buf, size_t size, GraphFile& gf, std::string& err);
int write_graphfile(const GraphFile& gf, std::vector<uint8_t>& out, std::string& err);
// PointMap::blockLines input: the lines of every shown layer, [n][4] x1,y1,x2,y2.
std::vector<double> graphfile_lines(const GraphFile& gf);
// MetaGraph::setViewClass(SHOWVGATOP) (mgraph.cpp:167-177)
int32_t view_vga_top(int32_t view_class);
// MetaGraph::addNewPointMap default naming (mgraph.cpp:2791-2809): "VGA Map", "VGA Map 1", ...
std::string new_pointmap_name(const GraphFile& gf, const std::string& base);

} // namespace dmx
