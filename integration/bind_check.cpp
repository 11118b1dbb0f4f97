// bind_check.cpp -- builds and exercises the salalib binding (dmx_salalib.cpp) against the REAL
// reference library compiled from /root/reference (oracle/_ref/libsalaref.a).  Test driver only: in
// this container (no GPU) it proves the binding type-checks and links against the reference, and that
// the map image round trip it is built on (reference PointMap::write -> engine chunk parse/serialize ->
// reference PointMap::read) is lossless; with a GPU it also checks that the binding's makeGraph and
// VGA global leave the reference map byte-identical (makeGraph) / equal within 1e-6 (VGA columns) to
// the reference's own sparkGraph2 / VGAVisualGlobal::run.
//
// Usage: bind_check <drawing.graph> <spacing> <x,y>     (VISPREP -pg spacing -pp x,y -pm, then VGA -vg)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <sstream>
#include <string>

#include "dmx.h"
#include "dmx_salalib.h"
#include "salalib/entityparsing.h"
#include "salalib/mgraph.h"
#include "salalib/vgamodules/vgavisualglobal.h"

static std::unique_ptr<MetaGraph> prepared(const char* path, double spacing, const Point2f& p) {
    std::unique_ptr<MetaGraph> g(new MetaGraph);
    if (g->readFromFile(path) != MetaGraph::OK) return nullptr;
    g->addNewPointMap();
    g->setGrid(spacing, Point2f(0.0, 0.0));
    g->makePoints(p, 0, nullptr);
    return g;
}

static std::string image(PointMap& m) {
    std::string s;
    dmxsala::saveMap(m, &s);
    return s;
}

// the engine's chunk reader/writer on a reference image: parse and serialize, untouched
static std::string through_engine(const std::string& img) {
    dmx_chunk* c = nullptr;
    if (dmx_chunk_parse(reinterpret_cast<const uint8_t*>(img.data()), (int64_t)img.size(), &c) != DMX_OK) return "";
    int64_t size = 0;
    dmx_chunk_serialize(c, nullptr, 0, &size);
    std::string out((size_t)size, '\0');
    dmx_chunk_serialize(c, reinterpret_cast<uint8_t*>(&out[0]), size, &size);
    dmx_chunk_free(c);
    return out;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: bind_check <drawing.graph> <spacing> <x,y>\n");
        return 2;
    }
    const double spacing = std::atof(argv[2]);
    Point2f p;
    if (std::sscanf(argv[3], "%lf,%lf", &p.x, &p.y) != 2) return 2;
    int failures = 0;

    // reference: VISPREP -pm and VGA -vg on its own code
    auto ref = prepared(argv[1], spacing, p);
    if (!ref) return 2;
    ref->makeGraph(nullptr, 0, -1.0);
    PointMap& rm = ref->getDisplayedPointMap();
    const std::string made = image(rm);

    // 1. image round trip through the engine and back into the reference's PointMap::read
    const std::string eng = through_engine(made);
    std::printf("engine chunk parse/serialize: %s\n", eng == made ? "identical" : "DIFFERS");
    failures += eng != made;
    dmxsala::loadMap(rm, &eng);
    const std::string back = image(rm);
    std::printf("reference PointMap::read of the engine image: %s (%zu bytes)\n", back == made ? "identical" : "DIFFERS",
                made.size());
    failures += back != made;

    // 2. the binding's makeGraph on the GPU, against the reference's sparkGraph2
    auto gpu = prepared(argv[1], spacing, p);
    PointMap& gm = gpu->getDisplayedPointMap();
    if (!dmxsala::sparkGraph2(gm, nullptr, false, -1.0)) {
        std::printf("binding makeGraph: no usable device, the reference path runs (declined)\n");
        return failures ? 1 : 0;
    }
    const std::string gmade = image(gm);
    std::printf("binding makeGraph vs reference sparkGraph2: %s\n", gmade == made ? "identical" : "DIFFERS");
    failures += gmade != made;

    // 3. the binding's VGA global vs VGAVisualGlobal::run, column by column
    VGAVisualGlobal(-1, false).run(nullptr, rm, false);
    if (!dmxsala::vgaVisualGlobal(gm, nullptr, -1, false, false)) {
        std::printf("binding VGA global: declined\n");
        return 1;
    }
    AttributeTable& ra = rm.getAttributeTable();
    AttributeTable& ga = gm.getAttributeTable();
    double worst = 0.0;
    for (size_t c = 0; c < ra.getNumColumns(); c++) {
        const std::string& name = ra.getColumnName(c);
        const size_t gc = ga.getColumnIndex(name);
        for (auto it = ra.begin(); it != ra.end(); ++it) {
            const float a = it->getRow().getValue(c);
            const float b = ga.getRow(it->getKey()).getValue(gc);
            const double d = std::fabs((double)a - (double)b) / std::fmax(1.0, std::fabs((double)a));
            if (d > worst) worst = d;
        }
    }
    std::printf("binding VGA global vs VGAVisualGlobal::run: max rel diff %.3g over %zu columns\n", worst,
                ra.getNumColumns());
    failures += worst > 1e-6;
    return failures ? 1 : 0;
}
