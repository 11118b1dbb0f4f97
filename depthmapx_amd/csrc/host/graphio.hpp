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
};

// PointMap::write for the map `h` and the graph given as host arrays (node order).  cols are in
// insertion (physical) order; `displayed` indexes them (-1/-2 as in the reference).
int write_pointmap_chunk(const PointMapHost& h, int64_t nnodes, const int32_t* bins, const int16_t* runs, int64_t nruns,
                         const uint8_t* gridconn, const std::vector<ChunkColumn>& cols, int displayed, bool boundary,
                         std::vector<uint8_t>& out, std::string& err);
int read_pointmap_chunk(const uint8_t* buf, size_t size, ParsedChunk& pc, std::string& err);

} // namespace dmx
