// graphio.hpp -- byte-exact PointMap chunk of the depthmapX .graph format (see graphio.cpp).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "pointmap.hpp"

namespace dmx {

struct ChunkColumn {
    std::string name;
    bool locked = false;
    std::vector<float> values;      // node (x-major) order
    std::vector<uint8_t> set;       // rows the analysis called setValue on (empty: all rows)
    float min = -1.0f, max = -1.0f; // as read
    double total = -1.0;
    // AttributeColumnImpl fields kept through a read / write (attributetable.cpp:91-124)
    bool from_file = false;         // true: stats as read; false: replayed from values / set
    uint8_t hidden = 0;
    uint8_t display[12] = {0, 0, 0, 0, 0, 0, 0x80, 0x3f, 0, 0, 0, 0};   // DisplayParams {0.0f, 1.0f, 0}
    std::string formula;
};

struct ParsedChunk {
    std::string name;
    double spacing = 0, blx = 0, bly = 0;
    int32_t rows = 0, cols = 0, filled = 0, displayed_sorted = -1;
    std::vector<ChunkColumn> columns;   // physical (insertion) order
    std::vector<int32_t> row_keys;      // PixelRef ints, x-major
    std::vector<int32_t> state;         // [cols*rows] x-major
    std::vector<uint8_t> gridconn;      // [N]
    std::vector<int32_t> bins;          // [N][32][4] dir, node count, distance bits, runs
    std::vector<int16_t> runs;          // [R][4] as decoded (4-bit shift quirk applied)
    bool processed = false, boundary = false;
    size_t bytes_used = 0;
    // structural pieces for a faithful rewrite (PointMap::read then ::write, pointdata.cpp:1073-1188)
    int32_t displayed_phys = -1;        // the reference keeps the value read as a physical index
    std::vector<uint8_t> layers_raw;    // LayerManagerImpl bytes (layermanagerimpl.cpp:90-150)
    std::vector<int64_t> row_layers;    // AttributeRowImpl::m_layerKey per row
    uint8_t table_display[12] = {0, 0, 0, 0, 0, 0, 0x80, 0x3f, 0, 0, 0, 0};
    std::vector<uint8_t> points_raw;    // Point records as Point::write re-emits them (state masked, dummy 0)
    std::vector<uint64_t> point_off;    // [cols*rows + 1] start of each Point record in points_raw (x-major)
    int64_t merges = 0;                 // points with a merge link (m_merge != NoPixel)
    std::vector<int32_t> merge_pairs;   // [merges][2] (cell, merge partner cell), x-major indices
};

// PointMap::write for the map `h` and the graph given as host arrays (node order).  cols are in
// insertion (physical) order; `displayed` indexes them (-1/-2 as in the reference).
int write_pointmap_chunk(const PointMapHost& h, int64_t nnodes, const int32_t* bins, const int16_t* runs, int64_t nruns,
                         const uint8_t* gridconn, const std::vector<ChunkColumn>& cols, int displayed, bool boundary,
                         std::vector<uint8_t>& out, std::string& err);
int read_pointmap_chunk(const uint8_t* buf, size_t size, ParsedChunk& pc, std::string& err);
// PointMap::write of a chunk read earlier and edited through the helpers below: header, attribute
// table (columns alphabetically; read columns keep their stats, set columns replay them), the point
// records as read (state bits masked as PointMap::read masks them), processed / boundary flags.
int write_parsed_chunk(const ParsedChunk& pc, std::vector<uint8_t>& out, std::string& err);
// AttributeTable::insertOrResetColumn / insertOrResetLockedColumn (attributetable.cpp:303-326) followed
// by setValue on the rows in `set` (empty: every row); returns the physical column index.
int chunk_set_column(ParsedChunk& pc, const std::string& name, const float* values, const uint8_t* set, bool locked);
// PointMap::unmake(removeLinks) (pointdata.cpp:1343-1374) on the parsed records.
int chunk_unmake(ParsedChunk& pc, bool remove_links, std::string& err);

} // namespace dmx
