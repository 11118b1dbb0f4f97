// ref_probe.cpp -- TEST INFRASTRUCTURE ONLY (this container; never shipped, never run on the GPU box).
//
// Our own driver, linked against the REAL reference library (oracle/_ref/libsalaref.a, compiled by
// oracle/Makefile from /root/reference sources).  It replays the depthmapXcli VISPREP/VGA sequence
// (depthmapXcli/runmethods.cpp:279-341 runVisualPrep, :227-267 runVga) on one input and dumps every
// intermediate the MI355X engine must reproduce, as raw little-endian arrays:
//
//   <out>/grid.txt        spacing, cols, rows, bottom_left, region, filled count
//   <out>/lines.bin       float64 [L][4]   drawing lines as PointMap::blockLines sees them
//   <out>/state.bin       int32   [cols*rows]  Point::m_state after fill+makeGraph (x-major: i*rows+j)
//   <out>/celllines_n.bin int32   [cols*rows]  per-cell cropped line count (before makeGraph unblocks)
//   <out>/celllines.bin   float64 [*][4]   per-cell cropped lines (start.x,start.y,end.x,end.y)
//   <out>/attrs.bin       float32 [N][3]   Connectivity, Point First Moment, Point Second Moment
//   <out>/bins.bin        int32   [N][32][4]  dir, node_count(u16), far dist (f32 bits), nruns
//   <out>/runs.bin        int16   [R][4]   x0,y0,x1,y1 in reference order
//   <out>/gridconn.bin    uint8   [N]
//   <out>/vga.bin         float32 [N][7]   VGA global columns in table (alphabetical) order
//   <out>/vga_rt.bin      float32 [N][7]   same, after the .graph write/read round trip (CLI path)
//
// Usage:
//   ref_probe --lines L.csv | --graph G.graph  --spacing s --fill x,y [--fill x,y ...]
//             [--maxdist d] [--boundary] [--vga] [--radius r] [--roundtrip] [--out DIR]
//             [--write-graph out.graph] [--sources K]   (K>0: time makeGraph on K sources only)
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <list>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <vector>
#include <deque>
#include <functional>
#include <unordered_map>
#include <unordered_set>
#define protected public
#define private public
#include "salalib/mgraph.h"
#include "salalib/ngraph.h"
#include "salalib/importutils.h"
#include "salalib/vgamodules/vgavisualglobal.h"
#undef protected
#undef private

template <typename T> static void dump(const std::string& path, const std::vector<T>& v) {
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) { perror(path.c_str()); exit(2); }
    if (!v.empty()) fwrite(v.data(), sizeof(T), v.size(), f);
    fclose(f);
}

static void dumpVga(PointMap& pm, const std::string& path) {
    AttributeTable& at = pm.getAttributeTable();
    std::vector<float> out;
    // VGAVisualGlobal column names (vgavisualglobal.cpp:38-63), dumped in a fixed order.
    const char* names[7] = {"Visual Entropy", "Visual Integration [HH]", "Visual Integration [P-value]",
                            "Visual Integration [Tekl]", "Visual Mean Depth", "Visual Node Count",
                            "Visual Relativised Entropy"};
    std::vector<int> cols;
    for (auto n : names) cols.push_back((int)at.getColumnIndex(n));
    for (auto it = at.begin(); it != at.end(); ++it)
        for (int c : cols) out.push_back(it->getRow().getValue(c));
    dump(path, out);
}

int main(int argc, char** argv) {
    std::string linesCsv, graphIn, outDir = ".", writeGraph;
    double spacing = -1, maxdist = -1, radius = -1;
    bool boundary = false, vga = false, roundtrip = false, vlocal = false, vmetric = false, vangular = false;
    double mradius = -1;
    long sources = 0;
    std::vector<Point2f> fills, stepPoints;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto next = [&]() { if (i + 1 >= argc) { fprintf(stderr, "missing arg for %s\n", a.c_str()); exit(2);} return std::string(argv[++i]); };
        if (a == "--lines") linesCsv = next();
        else if (a == "--graph") graphIn = next();
        else if (a == "--spacing") spacing = atof(next().c_str());
        else if (a == "--fill") { std::string p = next(); double x, y; sscanf(p.c_str(), "%lf,%lf", &x, &y); fills.push_back(Point2f(x, y)); }
        else if (a == "--maxdist") maxdist = atof(next().c_str());
        else if (a == "--radius") radius = atof(next().c_str());
        else if (a == "--boundary") boundary = true;
        else if (a == "--vga") vga = true;
        else if (a == "--roundtrip") roundtrip = true;
        else if (a == "--vlocal") vlocal = true;
        else if (a == "--vmetric") { vmetric = true; mradius = atof(next().c_str()); }
        else if (a == "--vangular") { vangular = true; mradius = atof(next().c_str()); }
        else if (a == "--out") outDir = next();
        else if (a == "--write-graph") writeGraph = next();
        else if (a == "--sources") sources = atol(next().c_str());
        else if (a == "--stepdepth") { std::string p = next(); double x, y; sscanf(p.c_str(), "%lf,%lf", &x, &y); stepPoints.push_back(Point2f(x, y)); }
        else { fprintf(stderr, "unknown arg %s\n", a.c_str()); return 2; }
    }
    MetaGraph mg;
    if (!graphIn.empty()) {
        int r = mg.readFromFile(graphIn);
        if (r != MetaGraph::OK) { fprintf(stderr, "readFromFile failed %d\n", r); return 1; }
    } else {
        std::ifstream f(linesCsv);
        if (!depthmapX::importFile(mg, f, nullptr, linesCsv, depthmapX::ImportType::DRAWINGMAP,
                                   depthmapX::ImportFileType::CSV)) {
            fprintf(stderr, "import failed\n"); return 1;
        }
    }
    QtRegion reg = mg.getRegion();
    mg.addNewPointMap();
    mg.setGrid(spacing, Point2f(0.0, 0.0));
    for (auto& p : fills) {
        if (!reg.contains(p)) { fprintf(stderr, "Point outside of target region\n"); return 1; }
        mg.makePoints(p, 0, nullptr);
    }
    PointMap& pm = mg.getDisplayedPointMap();
    pm.blockLines();
    const size_t cols = pm.getCols(), rows = pm.getRows();

    // drawing lines exactly as blockLines() consumes them (pointdata.cpp:308-320)
    std::vector<double> lines;
    for (const auto& pixelGroup : *pm.m_drawingFiles)
        for (const auto& pixel : pixelGroup.m_spacePixels)
            if (pixel.isShown())
                for (const auto& l : pixel.getAllShapesAsLines()) {
                    lines.push_back(l.start().x); lines.push_back(l.start().y);
                    lines.push_back(l.end().x); lines.push_back(l.end().y);
                }
    dump(outDir + "/lines.bin", lines);
    std::vector<int> cln(cols * rows);
    std::vector<double> cl;
    for (size_t i = 0; i < cols; i++)
        for (size_t j = 0; j < rows; j++) {
            Point& pt = pm.getPoint(PixelRef(i, j));
            cln[i * rows + j] = (int)pt.m_lines.size();
            for (auto& l : pt.m_lines) {
                cl.push_back(l.start().x); cl.push_back(l.start().y);
                cl.push_back(l.end().x); cl.push_back(l.end().y);
            }
        }
    dump(outDir + "/celllines_n.bin", cln);
    dump(outDir + "/celllines.bin", cl);

    if (sources > 0) {
        // timing probe: run sparkPixel2 for the first K filled sources (x-major) only
        pm.getAttributeTable().insertOrResetLockedColumn("Connectivity");
        pm.getAttributeTable().insertOrResetColumn("Point First Moment");
        pm.getAttributeTable().insertOrResetColumn("Point Second Moment");
        pm.tagState(true);
        long done = 0;
        auto t0 = std::chrono::steady_clock::now();
        for (size_t i = 0; i < cols && done < sources; i++)
            for (size_t j = 0; j < rows && done < sources; j++) {
                PixelRef c(i, j);
                if (!pm.getPoint(c).filled()) continue;
                pm.getPoint(c).m_node.reset(new Node());
                pm.getAttributeTable().addRow(AttributeKey(c));
                pm.sparkPixel2(c, 1, maxdist);
                done++;
            }
        auto t1 = std::chrono::steady_clock::now();
        printf("probe_sources %ld seconds %.6f\n", done, std::chrono::duration<double>(t1 - t0).count());
        return 0;
    }

    auto t0 = std::chrono::steady_clock::now();
    bool ok = mg.makeGraph(nullptr, boundary ? 1 : 0, maxdist);
    auto t1 = std::chrono::steady_clock::now();
    if (!ok) { fprintf(stderr, "makeGraph failed\n"); return 1; }

    std::vector<int> state(cols * rows);
    for (size_t i = 0; i < cols; i++)
        for (size_t j = 0; j < rows; j++) state[i * rows + j] = pm.getPoint(PixelRef(i, j)).m_state;
    dump(outDir + "/state.bin", state);

    AttributeTable& at = pm.getAttributeTable();
    int cc = at.getColumnIndex("Connectivity"), c1 = at.getColumnIndex("Point First Moment"),
        c2 = at.getColumnIndex("Point Second Moment");
    std::vector<float> attrs;
    std::vector<int> bins;
    std::vector<short> runs;
    std::vector<unsigned char> gconn;
    long nodes = 0;
    for (auto it = at.begin(); it != at.end(); ++it) {
        PixelRef p = it->getKey().value;
        attrs.push_back(it->getRow().getValue(cc));
        attrs.push_back(it->getRow().getValue(c1));
        attrs.push_back(it->getRow().getValue(c2));
        Point& pt = pm.getPoint(p);
        gconn.push_back((unsigned char)pt.m_grid_connections);
        for (int b = 0; b < 32; b++) {
            Bin& bin = pt.m_node->bin(b);
            float d = bin.distance();
            int dbits; memcpy(&dbits, &d, 4);
            bins.push_back((int)bin.m_dir);
            bins.push_back((int)bin.count());
            bins.push_back(dbits);
            bins.push_back((int)bin.m_pixel_vecs.size());
            for (auto& pv : bin.m_pixel_vecs) {
                runs.push_back(pv.m_start.x); runs.push_back(pv.m_start.y);
                runs.push_back(pv.m_end.x); runs.push_back(pv.m_end.y);
            }
        }
        nodes++;
    }
    {
        // the PointMap chunk of the .graph file exactly as MetaGraph::write emits it after VISPREP
        // (PointMap::write, salalib/pointdata.cpp:1158-1188)
        std::ofstream cf(outDir + "/pm_chunk_mk.bin", std::ios::binary);
        pm.write(cf);
    }
    dump(outDir + "/attrs.bin", attrs);
    dump(outDir + "/bins.bin", bins);
    dump(outDir + "/runs.bin", runs);
    dump(outDir + "/gridconn.bin", gconn);

    double tsd = 0, tvsd = 0;
    if (!stepPoints.empty()) {
        // dm_runmethods::runStepDepth (depthmapXcli/runmethods.cpp:735-778), metric step type
        for (auto& p : stepPoints) {
            if (!reg.contains(p)) { fprintf(stderr, "Point outside of target region\n"); return 1; }
            QtRegion r(p, p);
            mg.setCurSel(r, true);
        }
        std::vector<int> sel(pm.getSelSet().begin(), pm.getSelSet().end());
        dump(outDir + "/stepdepth_sel.bin", sel);
        Options opt;
        opt.global = 0;
        opt.point_depth_selection = 2;
        auto a = std::chrono::steady_clock::now();
        bool done = mg.analyseGraph(nullptr, opt, false);
        auto b = std::chrono::steady_clock::now();
        tsd = std::chrono::duration<double>(b - a).count();
        std::vector<float> sd;
        const char* names[3] = {"Metric Step Shortest-Path Angle", "Metric Step Shortest-Path Length",
                                "Metric Straight-Line Distance"};
        std::vector<int> cols3;
        for (auto n : names) cols3.push_back(done && at.hasColumn(n) ? (int)at.getColumnIndex(n) : -1);
        for (auto it = at.begin(); it != at.end(); ++it)
            for (int c : cols3) sd.push_back(c >= 0 ? it->getRow().getValue(c) : -1.0f);
        dump(outDir + "/stepdepth.bin", sd);
        // the same selection, -sdt visual (runmethods.cpp:767-769 -> VGAVisualGlobalDepth::run)
        Options vopt;
        vopt.global = 0;
        vopt.point_depth_selection = 1;
        a = std::chrono::steady_clock::now();
        bool vdone = mg.analyseGraph(nullptr, vopt, false);
        b = std::chrono::steady_clock::now();
        tvsd = std::chrono::duration<double>(b - a).count();
        std::vector<float> vsd;
        const int vcol = vdone && at.hasColumn("Visual Step Depth") ? (int)at.getColumnIndex("Visual Step Depth") : -1;
        for (auto it = at.begin(); it != at.end(); ++it) vsd.push_back(vcol >= 0 ? it->getRow().getValue(vcol) : -1.0f);
        dump(outDir + "/vstepdepth.bin", vsd);
        // and -sdt angular (runmethods.cpp:770-772 -> VGAAngularDepth::run, mgraph.cpp:334-336)
        Options aopt;
        aopt.global = 0;
        aopt.point_depth_selection = 3;
        bool adone = mg.analyseGraph(nullptr, aopt, false);
        std::vector<float> asd;
        const int acol = adone && at.hasColumn("Angular Step Depth") ? (int)at.getColumnIndex("Angular Step Depth") : -1;
        for (auto it = at.begin(); it != at.end(); ++it) asd.push_back(acol >= 0 ? it->getRow().getValue(acol) : -1.0f);
        dump(outDir + "/astepdepth.bin", asd);
        pm.clearSel();
    }

    double tv = 0, tvrt = 0;
    if (vga) {
        Options opt;
        opt.output_type = Options::OUTPUT_VISUAL;
        opt.local = 0;
        opt.global = 1;
        opt.radius = radius;
        auto a = std::chrono::steady_clock::now();
        mg.analyseGraph(nullptr, opt, false);
        auto b = std::chrono::steady_clock::now();
        tv = std::chrono::duration<double>(b - a).count();
        dumpVga(pm, outDir + "/vga.bin");
    }
    if (!writeGraph.empty() || roundtrip) {
        std::string g = writeGraph.empty() ? outDir + "/rt.graph" : writeGraph;
        mg.write(g, METAGRAPH_VERSION, false);
        if (roundtrip && vga) {
            MetaGraph mg2;
            int r = mg2.readFromFile(g);
            if (r != MetaGraph::OK) { fprintf(stderr, "re-read failed %d\n", r); return 1; }
            Options opt;
            opt.output_type = Options::OUTPUT_VISUAL;
            opt.local = 0;
            opt.global = 1;
            opt.radius = radius;
            auto a = std::chrono::steady_clock::now();
            mg2.analyseGraph(nullptr, opt, false);
            auto b = std::chrono::steady_clock::now();
            tvrt = std::chrono::duration<double>(b - a).count();
            dumpVga(mg2.getDisplayedPointMap(), outDir + "/vga_rt.bin");
        }
        if (writeGraph.empty()) remove(g.c_str());
    }

    // VGA visual local (-vl: mgraph.cpp:349-353 -> VGAVisualLocal::run), last so that its columns do
    // not travel through the round trip above
    double tvl = 0;
    if (vlocal) {
        Options opt;
        opt.output_type = Options::OUTPUT_VISUAL;
        opt.local = 1;
        opt.global = 0;
        opt.radius = -1;
        auto a = std::chrono::steady_clock::now();
        mg.analyseGraph(nullptr, opt, false);
        auto b = std::chrono::steady_clock::now();
        tvl = std::chrono::duration<double>(b - a).count();
        AttributeTable& at = pm.getAttributeTable();
        const char* names[3] = {"Visual Clustering Coefficient", "Visual Control", "Visual Controllability"};
        std::vector<float> out;
        for (auto it = at.begin(); it != at.end(); ++it)
            for (auto n : names) out.push_back(it->getRow().getValue((int)at.getColumnIndex(n)));
        dump(outDir + "/vlocal.bin", out);
    }

    // VGA metric (-vm metric -vr r: mgraph.cpp:359-361 -> VGAMetric::run), after everything else
    double tvm = 0;
    if (vmetric || vangular) {
        Options opt;
        opt.output_type = vmetric ? Options::OUTPUT_METRIC : Options::OUTPUT_ANGULAR;
        opt.radius = mradius;
        auto a = std::chrono::steady_clock::now();
        mg.analyseGraph(nullptr, opt, false);
        auto b = std::chrono::steady_clock::now();
        tvm = std::chrono::duration<double>(b - a).count();
        AttributeTable& at = pm.getAttributeTable();
        std::vector<int> mc;
        for (size_t i = 0; i < at.getNumColumns(); i++)
            if (at.getColumnName(i).rfind(vmetric ? "Metric " : "Angular ", 0) == 0) mc.push_back((int)i);
        std::vector<float> out;
        for (auto it = at.begin(); it != at.end(); ++it)
            for (int c : mc) out.push_back(it->getRow().getValue(c));
        dump(outDir + (vmetric ? "/vmetric.bin" : "/vangular.bin"), out);
        FILE* fn = fopen((outDir + (vmetric ? "/vmetric_cols.txt" : "/vangular_cols.txt")).c_str(), "w");
        for (int c : mc) fprintf(fn, "%s\n", at.getColumnName(c).c_str());
        fclose(fn);
    }

    FILE* f = fopen((outDir + "/grid.txt").c_str(), "w");
    fprintf(f, "spacing %.17g\ncols %zu\nrows %zu\n", pm.m_spacing, cols, rows);
    fprintf(f, "bottom_left %.17g %.17g\n", pm.m_bottom_left.x, pm.m_bottom_left.y);
    fprintf(f, "region %.17g %.17g %.17g %.17g\n", reg.bottom_left.x, reg.bottom_left.y, reg.top_right.x,
            reg.top_right.y);
    fprintf(f, "filled %d\nnodes %ld\nruns %zu\n", pm.m_filled_point_count, nodes, runs.size() / 4);
    fprintf(f, "t_makegraph %.6f\nt_vga %.6f\nt_vga_rt %.6f\nt_stepdepth %.6f\nt_vstepdepth %.6f\nt_vlocal %.6f\nt_vmetric %.6f\n",
            std::chrono::duration<double>(t1 - t0).count(), tv, tvrt, tsd, tvsd, tvl, tvm);
    fclose(f);
    printf("ok nodes %ld runs %zu t_makegraph %.3f t_vga %.3f\n", nodes, runs.size() / 4,
           std::chrono::duration<double>(t1 - t0).count(), tv);
    return 0;
}
