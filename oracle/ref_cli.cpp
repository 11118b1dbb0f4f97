// ref_cli.cpp -- TEST INFRASTRUCTURE ONLY (this container; never shipped, never run on the GPU box).
//
// Our own restatement of the reference CLI's run methods for the accelerated modes, linked against
// the REAL reference library (oracle/_ref/libsalaref.a, built by oracle/Makefile from /root/reference
// sources).  The reference's depthmapXcli itself is not built: commandlineparser.cpp needs the
// generated version header.  This driver replays, on the reference's own MetaGraph:
//   loadGraph            depthmapXcli/runmethods.cpp:33-45
//   runVisualPrep        :279-341 (fillGraph :269-277, GridProperties check, addNewPointMap, setGrid,
//                        makePoints, makeGraph, PointMap::unmake)
//   runVga               :227-267 (RadiusConverter radiusconverter.cpp:24-61)
//   runStepDepth         :735-778
//   linkGraph            :116-190 (LINK mode, point maps, coordinate links: -lnk x1,y1,x2,y2)
// Fixture-only extensions (not depthmapXcli flags): -pps / -ppa fill a point with makePoints'
// fill_type 1 (SEMIFILL) / 2 (AUGMENT), the GUI's other fill modes (depthmapview.h:75); -pen / -unpen
// x,y apply the GUI's pencil tool (PointMap::fillPoint(p, add), pointdata.cpp:375-394); all in the
// order given together with -pp.
// and writes the .graph exactly as the CLI does (MetaGraph::write(out, METAGRAPH_VERSION, false)).
// tests/golden/make_golden_graphfiles.py turns its outputs into fixtures (sha256 + section digests).
//
// Usage: ref_cli -f IN -o OUT -m VISPREP|VGA|STEPDEPTH [-s] [mode flags as depthmapXcli]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "salalib/entityparsing.h"
#include "salalib/gridproperties.h"
#include "salalib/linkutils.h"
#include "salalib/mgraph.h"

static std::vector<Point2f> parse_points(const std::vector<std::string>& pts) {
    std::stringstream ss;
    ss << "x,y";
    for (auto& p : pts) ss << "\n" << p;
    return EntityParsing::parsePoints(ss, ',');
}

static int die(const std::string& m) {
    std::cout << m << std::endl;
    return 1;
}

int main(int argc, char** argv) {
    std::string in, out, mode, vm, vr, sdt;
    bool simple = false, pm = false, pb = false, pu = false, pl = false, vg = false, vl = false;
    double pg = -1, pr = -1;
    std::vector<std::string> sdp, lnk;
    std::vector<std::pair<int, std::string>> pp;   // (fill_type, point)
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto next = [&]() { return std::string(argv[++i]); };
        if (a == "-f") in = next();
        else if (a == "-o") out = next();
        else if (a == "-m") mode = next();
        else if (a == "-s") simple = true;
        else if (a == "-pg") pg = atof(next().c_str());
        else if (a == "-pp") pp.push_back({0, next()});
        else if (a == "-pps") pp.push_back({1, next()});
        else if (a == "-ppa") pp.push_back({2, next()});
        else if (a == "-pen") pp.push_back({10, next()});
        else if (a == "-unpen") pp.push_back({11, next()});
        else if (a == "-lnk") lnk.push_back(next());
        else if (a == "-pr") pr = atof(next().c_str());
        else if (a == "-pm") pm = true;
        else if (a == "-pb") pb = true;
        else if (a == "-pu") pu = true;
        else if (a == "-pl") pl = true;
        else if (a == "-vm") vm = next();
        else if (a == "-vg") vg = true;
        else if (a == "-vl") vl = true;
        else if (a == "-vr") vr = next();
        else if (a == "-sdt") sdt = next();
        else if (a == "-sdp") sdp.push_back(next());
        else return die("unknown arg " + a);
    }
    std::unique_ptr<MetaGraph> g(new MetaGraph);
    if (g->readFromFile(in) != MetaGraph::OK) return die("Failed to load graph from file " + in);
    if (mode == "VISPREP") {
        if (~g->getState() & MetaGraph::LINEDATA) return die("Graph must have line data before preparing VGA");
        if (pg > 0) {
            QtRegion r = g->getRegion();
            GridProperties gp(__max(r.width(), r.height()));
            if (pg > gp.getMax() || pg < gp.getMin()) return die("Chosen grid spacing is outside of the expected interval");
            g->addNewPointMap();
            g->setGrid(pg, Point2f(0.0, 0.0));
        } else if (g->getPointMaps().empty()) {
            return die("No map exists to use. Please create a new one by providing a grid size");
        }
        if (pu) {
            if (!g->getDisplayedPointMap().isProcessed()) return die("Current map has not had its graph made");
            g->getDisplayedPointMap().unmake(pl);
        } else {
            for (auto& tp : pp) {
                Point2f p = parse_points({tp.second}).at(0);
                if (!g->getRegion().contains(p)) return die("Point outside of target region");
                if (tp.first >= 10) g->getDisplayedPointMap().fillPoint(p, tp.first == 10);
                else g->makePoints(p, tp.first, nullptr);
            }
            if (pm) g->makeGraph(nullptr, pb ? 1 : 0, pr);
        }
    } else if (mode == "VGA") {
        Options o;
        if (vm == "visibility") {
            o.output_type = Options::OUTPUT_VISUAL;
            o.local = vl;
            o.global = vg;
            if (vg) o.radius = vr == "n" ? -1.0 : (double)atoi(vr.c_str());
        } else if (vm == "metric") {
            o.output_type = Options::OUTPUT_METRIC;
            o.radius = vr == "n" ? -1.0 : atof(vr.c_str());
        } else if (vm == "angular") {
            o.output_type = Options::OUTPUT_ANGULAR;
        } else {
            return die("unsupported -vm " + vm);
        }
        g->analyseGraph(nullptr, o, simple);
    } else if (mode == "LINK") {
        std::stringstream ss;
        ss << "x1,y1,x2,y2";
        for (auto& l : lnk) ss << "\n" << l;
        std::vector<Line> lines = EntityParsing::parseLines(ss, ',');
        PointMap& map = g->getDisplayedPointMap();
        depthmapX::mergePixelPairs(depthmapX::pixelateMergeLines(lines, map), map);
    } else if (mode == "STEPDEPTH") {
        for (auto& p : parse_points(sdp)) {
            if (!g->getRegion().contains(p)) return die("Point outside of target region");
            QtRegion r(p, p);
            g->setCurSel(r, true);
        }
        Options o;
        o.global = 0;
        o.point_depth_selection = sdt == "angular" ? 3 : sdt == "metric" ? 2 : 1;
        g->analyseGraph(nullptr, o, false);
    } else {
        return die("unknown mode " + mode);
    }
    if (g->write(out.c_str(), METAGRAPH_VERSION, false) != MetaGraph::OK) return die("write failed");
    std::cout << "ok" << std::endl;
    return 0;
}
