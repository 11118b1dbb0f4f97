// san_host.cpp -- host-side code of libdmx under AddressSanitizer + UndefinedBehaviorSanitizer (no GPU).
//
// Built by tests/test_sanitizers.py with g++ -fsanitize=address,undefined from the product's host
// sources (host/graphfile.cpp, host/graphio.cpp, host/pointmap.cpp).  For every .graph given:
//   - MetaGraph read -> write -> read -> write: the second write equals the first (stable re-emit);
//   - every PointMap chunk: read -> write_parsed_chunk reproduces the chunk's bytes;
//   - the drawing's lines go through the VISPREP host model (setGrid, blockLines, fill) at two
//     spacings;
//   - damaged copies (truncations, byte overwrites) are read again: any status is fine, a crash or a
//     sanitizer report is not (the reader takes untrusted files).
// Exit status 0 when every check holds; the sanitizers abort on the first report.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include "../../depthmapx_amd/csrc/host/graphfile.hpp"
#include "../../depthmapx_amd/csrc/host/graphio.hpp"
#include "../../depthmapx_amd/csrc/host/pointmap.hpp"

using namespace dmx;

static int fails = 0;
#define CHECK(c, ...)                                   \
    do {                                                \
        if (!(c)) {                                     \
            fprintf(stderr, "FAIL %s: ", #c);           \
            fprintf(stderr, __VA_ARGS__);               \
            fprintf(stderr, "\n");                      \
            fails++;                                    \
        }                                               \
    } while (0)

static void damaged_reads(const std::vector<uint8_t>& buf, std::mt19937_64& rng, int n) {
    std::string err;
    for (int i = 0; i < n; i++) {
        std::vector<uint8_t> b = buf;
        if (i % 2 == 0) {
            b.resize(rng() % (buf.size() + 1));
        } else {
            const int k = 1 + (int)(rng() % 8);
            for (int j = 0; j < k && !b.empty(); j++) b[rng() % b.size()] = (uint8_t)rng();
        }
        GraphFile gf;
        if (read_graphfile(b.data(), b.size(), gf, err) == 0) {
            std::vector<uint8_t> out;
            (void)write_graphfile(gf, out, err);
            for (auto& ch : gf.pointmaps) {
                ParsedChunk pc;
                if (read_pointmap_chunk(ch.data(), ch.size(), pc, err) == 0) {
                    std::vector<uint8_t> o2;
                    (void)write_parsed_chunk(pc, o2, err);
                }
            }
        }
    }
}

int main(int argc, char** argv) {
    std::mt19937_64 rng(2026);
    const int nfuzz = argc > 1 ? atoi(argv[1]) : 200;
    for (int a = 2; a < argc; a++) {
        std::ifstream f(argv[a], std::ios::binary);
        std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        std::string err;
        GraphFile gf;
        int rc = read_graphfile(buf.data(), buf.size(), gf, err);
        CHECK(rc == 0, "%s: %s", argv[a], err.c_str());
        if (rc) continue;
        std::vector<uint8_t> w1, w2;
        CHECK(write_graphfile(gf, w1, err) == 0, "%s: %s", argv[a], err.c_str());
        GraphFile gf2;
        CHECK(read_graphfile(w1.data(), w1.size(), gf2, err) == 0, "%s re-read: %s", argv[a], err.c_str());
        CHECK(write_graphfile(gf2, w2, err) == 0, "%s: %s", argv[a], err.c_str());
        CHECK(w1 == w2, "%s: re-emit not stable (%zu vs %zu bytes)", argv[a], w1.size(), w2.size());
        for (size_t i = 0; i < gf.pointmaps.size(); i++) {
            ParsedChunk pc;
            const auto& ch = gf.pointmaps[i];
            CHECK(read_pointmap_chunk(ch.data(), ch.size(), pc, err) == 0, "%s chunk %zu: %s", argv[a], i, err.c_str());
            std::vector<uint8_t> o;
            CHECK(write_parsed_chunk(pc, o, err) == 0, "%s chunk %zu: %s", argv[a], i, err.c_str());
            CHECK(o == ch, "%s chunk %zu: bytes differ", argv[a], i);
        }
        const std::vector<double> lines = graphfile_lines(gf);
        const Rect region{gf.region[0], gf.region[1], gf.region[2], gf.region[3]};
        const double w = region.trx - region.blx, h = region.tr_y - region.bly;
        if (!lines.empty() && w > 0 && h > 0) {
            for (double div : {60.0, 150.0}) {
                PointMapHost pm(region, std::max(w, h) / div, lines.data(), (int64_t)lines.size() / 4);
                for (int k = 0; k < 5; k++) {
                    const double x = region.blx + w * (0.1 + 0.2 * k), y = region.bly + h * (0.9 - 0.2 * k);
                    (void)pm.fill(x, y);
                }
                int64_t filled = 0;
                for (int32_t s : pm.state()) filled += (s & CELL_FILLED) ? 1 : 0;
                CHECK(filled == pm.filled_count(), "%s: filled count", argv[a]);
                CHECK(pm.seg_off().back() * 4 == (int64_t)pm.segs().size(), "%s: pieces", argv[a]);
            }
        }
        damaged_reads(buf, rng, nfuzz);
        printf("%s: %zu bytes, %zu point maps, %zu lines ok\n", argv[a], buf.size(), gf.pointmaps.size(), lines.size() / 4);
    }
    printf("%s\n", fails ? "FAILED" : "all ok");
    return fails ? 1 : 0;
}
