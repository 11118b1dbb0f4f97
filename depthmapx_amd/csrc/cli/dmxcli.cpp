// dmxcli -- command-line front-end of the MI355X engine with the depthmapXcli mode-parser surface
// for the accelerated path: VISPREP (grid, fill, makeGraph), VGA (-vm visibility -vg -vr) and
// STEPDEPTH (-sdt metric, -sdt visual).  Flags, validation messages, the "-t" timing CSV and the exit status
// follow the reference CLI:
//   depthmapXcli/main.cpp:22-54, commandlineparser.cpp:51-142, visprepparser.cpp:26-172,
//   vgaparser.cpp:29-106, radiusconverter.cpp:24-61, stepdepthparser.cpp:26-100,
//   runmethods.cpp:33-45 (loadGraph), :227-267 (runVga), :279-341 (runVisualPrep),
//   :735-778 (runStepDepth), performancewriter.cpp:60-76, salalib/gridproperties.cpp:4-13.
// Host code over the C ABI (include/dmx.h); every analysis runs on the GPU.
//
// Files: a depthmapX .graph (MetaGraph::readFromFile / write, mgraph.cpp:2475-2757, through
// dmx_graphfile_*), written back as .graph; or a drawing as a CSV of lines (header x1,y1,x2,y2; what
// "depthmapXcli -m IMPORT -it drawing" ingests) whose output container (".dmxg") holds the region, the
// lines and one PointMap chunk of the .graph format.
#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/dmx.h"

namespace {

struct CommandLineException : std::runtime_error { using std::runtime_error::runtime_error; };
struct RuntimeException : std::runtime_error { using std::runtime_error::runtime_error; };

bool has_only_digits(const std::string& s) { return s.find_first_not_of("0123456789") == std::string::npos; }
bool has_only_digits_dots_commas(const std::string& s) { return s.find_first_not_of("0123456789,.-") == std::string::npos; }

// ENFORCE_ARGUMENT (depthmapXcli/parsingutils.h:19-25)
void enforce_argument(const char* flag, int& i, int argc, char** argv) {
    if (++i >= argc || (argv[i][0] == '-' && !isdigit((unsigned char)argv[i][1]) && argv[i][1] != '.'))
        throw CommandLineException(std::string(flag) + " requires an argument");
}

void check(int rc) {
    if (rc != DMX_OK) throw RuntimeException(dmx_last_error());
}

// PerformanceWriter (performancewriter.cpp:60-76) + DO_TIMED (runmethods.h:37-40)
struct Perf {
    std::string file;
    std::vector<std::string> lines;
    void add(const std::string& action, double s) {
        std::stringstream ss;
        ss << "\"" << action << "\"," << s << "\n";
        lines.push_back(ss.str());
    }
    void write() const {
        if (file.empty()) return;
        std::ofstream f(file);
        f << "\"action\",\"duration\"\n";
        for (auto& l : lines) f << l;
    }
};
template <typename F> void timed(Perf& perf, const char* action, F&& f) {
    const auto t0 = std::chrono::steady_clock::now();
    f();
    perf.add(action, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
}

// EntityParsing::parsePoints (salalib/entityparsing.cpp:116-170): header naming x and y columns
std::vector<std::pair<double, double>> parse_points(std::istream& in, char delim) {
    std::string line;
    std::getline(in, line);
    std::vector<std::string> head;
    {
        std::stringstream ss(line);
        std::string t;
        while (std::getline(ss, t, delim)) {
            std::transform(t.begin(), t.end(), t.begin(), ::tolower);
            head.push_back(t);
        }
    }
    if (head.size() < 2) throw RuntimeException("Badly formatted header (should contain x and y)");
    int xc = -1, yc = -1;
    for (size_t i = 0; i < head.size(); i++) {
        if (head[i] == "x") xc = (int)i;
        else if (head[i] == "y") yc = (int)i;
    }
    if (xc < 0 || yc < 0) throw RuntimeException("Badly formatted header (should contain x and y)");
    std::vector<std::pair<double, double>> pts;
    while (std::getline(in, line)) {
        if (line.empty()) continue;
        std::vector<std::string> f;
        std::stringstream ss(line);
        std::string t;
        while (std::getline(ss, t, delim)) f.push_back(t);
        if ((int)f.size() <= std::max(xc, yc)) throw RuntimeException("Error parsing line: " + line);
        pts.emplace_back(std::stod(f[xc]), std::stod(f[yc]));
    }
    return pts;
}

std::vector<std::pair<double, double>> points_from_args(const std::vector<std::string>& pts, const std::string& file) {
    if (!file.empty()) {
        std::ifstream f(file);
        if (!f) {
            std::stringstream m;
            m << "Failed to load file " << file << ", error " << std::strerror(errno);
            throw RuntimeException(m.str());
        }
        return parse_points(f, '\t');
    }
    std::stringstream ss;
    ss << "x,y";
    for (auto& p : pts) ss << "\n" << p;
    return parse_points(ss, ',');
}

// ---------------------------------------------------------------- the document
// A depthmapX .graph file (MetaGraph container, read and written through dmx_graphfile_*), or this
// tool's ".dmxg" container for a drawing imported from CSV (region, lines and one PointMap chunk of the
// .graph format).  Output goes out in the input's container.
const char kMagic[4] = {'D', 'M', 'X', 'G'};
// MetaGraph m_state bits (mgraph.h:71-73)
enum { MG_POINTMAPS = 0x0002, MG_LINEDATA = 0x0004, MG_ANGULARGRAPH = 0x0010 };

struct Document {
    double region[4] = {0, 0, 0, 0};
    std::vector<double> lines;        // [L][4] as PointMap::blockLines reads them
    dmx_graphfile* gf = nullptr;      // .graph input
    bool has_map = false;             // .dmxg: one point map
    std::vector<uint8_t> chunk;
    int32_t state = 0, view = 0;
    Document() {}
    Document(const Document&) = delete;
    Document& operator=(const Document&) = delete;
    ~Document() { if (gf) dmx_graphfile_free(gf); }
    bool line_data() const { return gf ? (state & MG_LINEDATA) != 0 : !lines.empty(); }
    bool any_map() const {
        if (!gf) return has_map;
        int32_t n = 0;
        check(dmx_graphfile_info(gf, nullptr, nullptr, nullptr, nullptr, &n, nullptr));
        return n > 0;
    }
    // the displayed point map (MetaGraph::getDisplayedPointMap)
    std::vector<uint8_t> displayed_chunk() const {
        if (!gf) return chunk;
        int32_t disp = -1;
        check(dmx_graphfile_info(gf, nullptr, nullptr, nullptr, nullptr, nullptr, &disp));
        const uint8_t* p = nullptr;
        int64_t n = 0;
        check(dmx_graphfile_pointmap(gf, disp, &p, &n));
        return std::vector<uint8_t>(p, p + n);
    }
    void put_displayed(const std::vector<uint8_t>& c, bool new_map) {
        if (!gf) { chunk = c; has_map = true; return; }
        int32_t disp = -1;
        check(dmx_graphfile_info(gf, nullptr, nullptr, nullptr, nullptr, nullptr, &disp));
        check(dmx_graphfile_put_pointmap(gf, new_map ? -1 : disp, c.data(), (int64_t)c.size()));
    }
    std::string new_map_name() const {
        if (!gf) return "VGA Map";
        char name[256];
        check(dmx_graphfile_new_pointmap_name(gf, name, sizeof(name)));
        return name;
    }
};

void read_document(const std::string& path, Document& d) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw RuntimeException("Failed to load graph from file " + path + ", error -1");
    char magic[4] = {0, 0, 0, 0};
    f.read(magic, 4);
    if (magic[0] == 'g' && magic[1] == 'r' && magic[2] == 'f') {
        f.close();
        const int rc = dmx_graphfile_read(path.c_str(), &d.gf);
        if (rc) throw RuntimeException("Failed to load graph from file " + path + ", error " + std::to_string(rc) + " (" +
                                       dmx_last_error() + ")");
        int64_t nl = 0;
        check(dmx_graphfile_info(d.gf, &d.state, &d.view, d.region, &nl, nullptr, nullptr));
        d.lines.resize((size_t)nl * 4);
        check(dmx_graphfile_lines(d.gf, d.lines.data()));
        return;
    }
    if (std::memcmp(magic, kMagic, 4) != 0) {
        // a drawing: CSV of lines x1,y1,x2,y2 (the reference's IMPORT -it drawing input)
        f.close();
        std::ifstream t(path);
        std::string line;
        std::getline(t, line);
        double mn[2] = {1e300, 1e300}, mx[2] = {-1e300, -1e300};
        while (std::getline(t, line)) {
            if (line.empty()) continue;
            double v[4];
            if (std::sscanf(line.c_str(), "%lf,%lf,%lf,%lf", &v[0], &v[1], &v[2], &v[3]) != 4)
                throw RuntimeException("Failed to load graph from file " + path + ", error -1");
            for (int i = 0; i < 4; i++) d.lines.push_back(v[i]);
            for (int i = 0; i < 2; i++) {
                mn[0] = std::min(mn[0], v[2 * i]); mx[0] = std::max(mx[0], v[2 * i]);
                mn[1] = std::min(mn[1], v[2 * i + 1]); mx[1] = std::max(mx[1], v[2 * i + 1]);
            }
        }
        if (d.lines.empty()) throw RuntimeException("Failed to load graph from file " + path + ", error -1");
        d.region[0] = mn[0]; d.region[1] = mn[1]; d.region[2] = mx[0]; d.region[3] = mx[1];
        return;
    }
    uint32_t version = 0;
    f.read((char*)&version, 4);
    f.read((char*)d.region, sizeof(d.region));
    int64_t nl = 0;
    f.read((char*)&nl, 8);
    d.lines.resize((size_t)nl * 4);
    if (nl) f.read((char*)d.lines.data(), (std::streamsize)(nl * 32));
    uint8_t hm = 0;
    f.read((char*)&hm, 1);
    d.has_map = hm != 0;
    if (d.has_map) {
        int64_t n = 0;
        f.read((char*)&n, 8);
        d.chunk.resize((size_t)n);
        f.read((char*)d.chunk.data(), (std::streamsize)n);
    }
    if (!f) throw RuntimeException("Failed to load graph from file " + path + ", error -1");
}

void write_document(const std::string& path, Document& d) {
    if (d.gf) {
        check(dmx_graphfile_set_view(d.gf, d.state, d.view));
        check(dmx_graphfile_write(d.gf, path.c_str()));
        return;
    }
    std::ofstream f(path, std::ios::binary | std::ios::trunc);
    if (!f) throw RuntimeException("Failed to write " + path);
    f.write(kMagic, 4);
    const uint32_t version = 1;
    f.write((const char*)&version, 4);
    f.write((const char*)d.region, sizeof(d.region));
    const int64_t nl = (int64_t)d.lines.size() / 4;
    f.write((const char*)&nl, 8);
    if (nl) f.write((const char*)d.lines.data(), (std::streamsize)(nl * 32));
    const uint8_t hm = d.has_map ? 1 : 0;
    f.write((const char*)&hm, 1);
    if (d.has_map) {
        const int64_t n = (int64_t)d.chunk.size();
        f.write((const char*)&n, 8);
        f.write((const char*)d.chunk.data(), (std::streamsize)n);
    }
}

// -p: the PrintCommunicator's record lines (depthmapXcli/printcommunicator.cpp:19-38), posted by the library's
// progress callback every 0.5 s (the Communicator contract, genlib/comm.h)
bool g_print_progress = false;
int print_progress(void*, int32_t, int64_t done, int64_t total) {
    std::cout << "step: 1/1 record: " << std::min(done, total) << "/" << total << std::endl;
    return 0;
}

struct Context {
    dmx_ctx* ctx = nullptr;
    Context() {
        check(dmx_ctx_create(0, &ctx));
        if (g_print_progress) check(dmx_ctx_set_progress(ctx, print_progress, nullptr, 0.5));
    }
    ~Context() { dmx_ctx_free(ctx); }
};

// A parsed point map chunk (library-owned) with its graph uploaded to the GPU: what the reference's
// VGA / STEPDEPTH steps analyse after loadGraph (runmethods.cpp:33-45).
struct LoadedMap {
    dmx_chunk* chunk = nullptr;
    dmx_pointmap* pm = nullptr;
    dmx_graph* g = nullptr;
    int64_t nnodes = 0;
    ~LoadedMap() {
        if (g) dmx_graph_free(g);
        if (pm) dmx_pointmap_free(pm);
        if (chunk) dmx_chunk_free(chunk);
    }
    // add / reset a column of the analysis (values and set mask in node = attribute row order)
    void column(const std::string& name, const float* values, const uint8_t* set, bool locked, bool displayed) {
        check(dmx_chunk_set_column(chunk, name.c_str(), values, set, locked ? 1 : 0, displayed ? 1 : 0));
    }
    std::vector<uint8_t> bytes() const {
        int64_t size = 0;
        check(dmx_chunk_serialize(chunk, nullptr, 0, &size));
        std::vector<uint8_t> out((size_t)size);
        check(dmx_chunk_serialize(chunk, out.data(), size, &size));
        return out;
    }
};

void load_map(Context& C, const Document& d, LoadedMap& m) {
    if (!d.any_map()) throw RuntimeException("No map exists to use. Please create a new one by providing a grid size");
    const std::vector<uint8_t> bytes = d.displayed_chunk();
    check(dmx_chunk_parse(bytes.data(), (int64_t)bytes.size(), &m.chunk));
    check(dmx_chunk_info(m.chunk, nullptr, nullptr, nullptr, nullptr, &m.nnodes, nullptr, nullptr, nullptr, nullptr));
    int64_t nrows = 0;
    check(dmx_chunk_flags(m.chunk, nullptr, nullptr, nullptr, &nrows));
    if (nrows != m.nnodes) throw RuntimeException("attribute rows do not match the graph's nodes");
    check(dmx_chunk_load(C.ctx, m.chunk, d.region, &m.pm, &m.g));
}

// PointMap::write of a freshly built map (dmx_chunk_write), named like the map it replaces / adds
std::vector<uint8_t> write_chunk(dmx_pointmap* pm, int64_t n, const int32_t* bins, const int16_t* runs, int64_t nruns,
                                 const uint8_t* gc, const std::vector<std::string>& names,
                                 const std::vector<std::vector<float>>& cols, const std::vector<uint8_t>& locked,
                                 int displayed, bool boundary, const std::string& map_name) {
    std::vector<const char*> nm;
    std::vector<float> vals;
    for (size_t i = 0; i < names.size(); i++) {
        nm.push_back(names[i].c_str());
        vals.insert(vals.end(), cols[i].begin(), cols[i].end());
    }
    int64_t size = 0;
    check(dmx_chunk_write(pm, n, bins, runs, nruns, gc, (int)names.size(), nm.data(), vals.data(), locked.data(), nullptr,
                          displayed, boundary ? 1 : 0, nullptr, 0, &size));
    std::vector<uint8_t> out((size_t)size);
    check(dmx_chunk_write(pm, n, bins, runs, nruns, gc, (int)names.size(), nm.data(), vals.data(), locked.data(), nullptr,
                          displayed, boundary ? 1 : 0, out.data(), size, &size));
    if (map_name == "VGA Map") return out;
    dmx_chunk* c = nullptr;
    check(dmx_chunk_parse(out.data(), size, &c));
    std::unique_ptr<dmx_chunk, int (*)(dmx_chunk*)> guard(c, dmx_chunk_free);
    check(dmx_chunk_set_name(c, map_name.c_str()));
    check(dmx_chunk_serialize(c, nullptr, 0, &size));
    out.resize((size_t)size);
    check(dmx_chunk_serialize(c, out.data(), size, &size));
    return out;
}

// ---------------------------------------------------------------- modes (IModeParser, imodeparser.h:24-32)
struct Args {
    std::string file, out, timing;
    bool simple = false, progress = false;
};

struct Mode {
    virtual ~Mode() {}
    virtual std::string name() const = 0;
    virtual void parse(int argc, char** argv) = 0;
    virtual void run(const Args& a, Perf& perf) = 0;
};

// VisPrepParser (visprepparser.cpp:26-172) + runVisualPrep (runmethods.cpp:279-341)
struct VisPrep : Mode {
    double grid = -1, maxvis = -1;
    bool boundary = false, make = false, unmake = false, removeLinks = false;
    std::vector<std::pair<double, double>> fills;
    std::string name() const override { return "VISPREP"; }
    void parse(int argc, char** argv) override {
        std::vector<std::string> points;
        std::string pointFile;
        for (int i = 1; i < argc; ++i) {
            if (!std::strcmp("-pg", argv[i])) {
                if (grid >= 0) throw CommandLineException("-pg can only be used once");
                enforce_argument("-pg", i, argc, argv);
                grid = std::atof(argv[i]);
                if (grid <= 0) throw CommandLineException(std::string("-pg must be a number >0, got ") + argv[i]);
            } else if (!std::strcmp("-pp", argv[i])) {
                if (!pointFile.empty()) throw CommandLineException("-pp cannot be used together with -pf");
                enforce_argument("-pp", i, argc, argv);
                if (!has_only_digits_dots_commas(argv[i])) {
                    std::stringstream m;
                    m << "Invalid fill point provided (" << argv[i] << "). Should only contain digits dots and commas";
                    throw CommandLineException(m.str());
                }
                points.push_back(argv[i]);
            } else if (!std::strcmp("-pf", argv[i])) {
                if (!points.empty()) throw CommandLineException("-pf cannot be used together with -pp");
                enforce_argument("-pf", i, argc, argv);
                pointFile = argv[i];
            } else if (!std::strcmp("-pr", argv[i])) {
                enforce_argument("-pr", i, argc, argv);
                maxvis = std::atof(argv[i]);
                if (maxvis == 0.0) {
                    std::stringstream m;
                    m << "Restricted visibility of '" << argv[i] << "' makes no sense, use a positive number or -1 for unrestricted";
                    throw CommandLineException(m.str());
                }
            } else if (!std::strcmp("-pb", argv[i])) {
                boundary = true;
            } else if (!std::strcmp("-pm", argv[i])) {
                if (unmake) throw CommandLineException("-pm cannot be used together with -pu");
                make = true;
            } else if (!std::strcmp("-pu", argv[i])) {
                if (make) throw CommandLineException("-pu cannot be used together with -pm");
                unmake = true;
            } else if (!std::strcmp("-pl", argv[i])) {
                removeLinks = true;
            }
        }
        if (!make && !unmake && grid <= 0 && pointFile.empty() && points.empty()) throw CommandLineException("Nothing to do");
        if (grid > 0 && make && pointFile.empty() && points.empty())
            throw CommandLineException("Creating a graph for an unfilled grid is not possible. Either -pp or -pf must be given");
        if (!pointFile.empty() || !points.empty()) fills = points_from_args(points, pointFile);
        if (unmake && (grid > 0 || !fills.empty()))
            throw CommandLineException("-pu can not be used with any other option apart from -pl");
        if (removeLinks && !unmake) throw CommandLineException("-pl can only be used together with -pu");
    }
    void run(const Args& a, Perf& perf) override {
        Document d;
        timed(perf, "Load graph file", [&] { read_document(a.file, d); });
        std::cout << "Initial checks... " << std::flush;
        if (!d.line_data()) throw RuntimeException("Graph must have line data before preparing VGA");
        dmx_pointmap* pm = nullptr;
        std::unique_ptr<dmx_pointmap, int (*)(dmx_pointmap*)> pmguard(nullptr, dmx_pointmap_free);
        std::unique_ptr<dmx_chunk, int (*)(dmx_chunk*)> existing(nullptr, dmx_chunk_free);
        std::string map_name = "VGA Map";
        bool new_map = false;
        if (grid > 0) {
            // GridProperties (salalib/gridproperties.cpp:4-13)
            const double maxdim = std::max(d.region[2] - d.region[0], d.region[3] - d.region[1]);
            const int maxexp = (int)std::floor(std::log10(maxdim)) - 1, minexp = maxexp - 2;
            const int mant = (int)std::floor(maxdim / std::pow(10.0, double(maxexp + 1)));
            const double gmax = (double)2 * mant * std::pow(10.0, double(maxexp));
            const double gmin = (double)mant * std::pow(10.0, double(minexp));
            if (grid > gmax || grid < gmin) {
                std::stringstream m;
                m << "Chosen grid spacing " << grid << " is outside of the expected interval of " << gmin
                  << " <= spacing <= " << gmax;
                throw RuntimeException(m.str());
            }
            std::cout << "ok\nSetting up grid... " << std::flush;
            // MetaGraph::addNewPointMap + setGrid (mgraph.cpp:2791-2809, :222-234)
            map_name = d.new_map_name();
            new_map = true;
            timed(perf, "Setting grid", [&] {
                check(dmx_pointmap_create(d.region, grid, d.lines.data(), (int64_t)d.lines.size() / 4, &pm));
            });
            pmguard.reset(pm);
            d.state |= MG_POINTMAPS;
            d.view = dmx_view_vga_top(d.view);
        } else {
            if (!d.any_map()) throw RuntimeException("No map exists to use. Please create a new one by providing a grid size");
            const std::vector<uint8_t> bytes = d.displayed_chunk();
            dmx_chunk* ch = nullptr;
            check(dmx_chunk_parse(bytes.data(), (int64_t)bytes.size(), &ch));
            existing.reset(ch);
            int32_t cols = 0, rows = 0;
            double spacing = 0;
            check(dmx_chunk_info(ch, &cols, &rows, &spacing, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr));
            std::vector<int32_t> st((size_t)cols * rows);
            check(dmx_chunk_arrays(ch, st.data(), nullptr, nullptr, nullptr));
            check(dmx_pointmap_create(d.region, spacing, d.lines.data(), (int64_t)d.lines.size() / 4, &pm));
            pmguard.reset(pm);
            check(dmx_pointmap_set_state(pm, st.data()));
            char nm[512];
            (void)nm;
            int processed = 0;
            check(dmx_chunk_flags(ch, &processed, nullptr, nullptr, nullptr));
            if (unmake) {
                if (!processed)
                    throw RuntimeException("Current map has not had its graph made so there's nothing to unmake");
            } else if (processed && (!fills.empty() || make)) {
                // the reference re-runs sparkGraph2 / makePoints on a map whose attribute rows exist:
                // AttributeTable::addRow throws a pointer (`throw new std::invalid_argument("Duplicate key")`,
                // salalib/attributetable.cpp:278) that main's catch (std::exception&) does not catch, so
                // depthmapXcli aborts; here it is an error with the CLI's exit code
                throw RuntimeException("The point map already has a graph: unmake it first (-pu)");
            }
            // merge links stay on the points (PointMap::read keeps m_merge, pointdata.cpp:1133-1137) and
            // are written back with them
            int64_t nlinks = 0;
            check(dmx_chunk_merges(ch, nullptr, &nlinks));
            if (nlinks) {
                std::vector<int32_t> links((size_t)nlinks * 2);
                check(dmx_chunk_merges(ch, links.data(), &nlinks));
                check(dmx_pointmap_set_merges(pm, links.data(), nlinks));
            }
            // the map keeps its name: read it back from the chunk header (dXstring: u32 length + bytes)
            uint32_t len = 0;
            std::memcpy(&len, bytes.data(), 4);
            map_name.assign((const char*)bytes.data() + 4, len);
        }
        if (unmake) {
            // PointMap::unmake (runmethods.cpp:319-325 -> pointdata.cpp:1343-1374)
            timed(perf, "Unmaking graph", [&] { check(dmx_chunk_unmake(existing.get(), removeLinks ? 1 : 0)); });
            std::cout << " ok\nWriting out result..." << std::flush;
            timed(perf, "Writing graph", [&] {
                int64_t size = 0;
                check(dmx_chunk_serialize(existing.get(), nullptr, 0, &size));
                std::vector<uint8_t> out((size_t)size);
                check(dmx_chunk_serialize(existing.get(), out.data(), size, &size));
                d.put_displayed(out, false);
                write_document(a.out, d);
            });
            std::cout << " ok" << std::endl;
            return;
        }
        std::unique_ptr<Context> C;   // the GPU: makeGraph, and the fill with DMX_FILL=device
        if (!fills.empty()) {
            // DMX_FILL=device: blockLines + the flood fill on the GPU (dmx_pointmap_fill_device)
            const char* fe = getenv("DMX_FILL");
            const bool on_device = fe && std::string(fe) == "device";
            if (on_device) C.reset(new Context());
            std::cout << "ok\nFilling grid... " << std::flush;
            timed(perf, "Filling grid", [&] {
                for (auto& p : fills) {
                    int made = 0;
                    // fillGraph (runmethods.cpp:269-277)
                    if (on_device) check(dmx_pointmap_fill_device(C->ctx, pm, p.first, p.second, &made));
                    else check(dmx_pointmap_fill(pm, p.first, p.second, &made));
                }
            });
        }
        dmx_graph* g = nullptr;
        if (make) {
            std::cout << "ok\nMaking graph... " << std::flush;
            d.state |= MG_ANGULARGRAPH;   // MetaGraph::makeGraph (mgraph.cpp:264-284)
            if (!C) C.reset(new Context());
            timed(perf, "Making graph", [&] { check(dmx_makegraph(C->ctx, pm, maxvis, boundary ? 1 : 0, 0, -1, &g)); });
            d.view = dmx_view_vga_top(d.view);
        }
        std::cout << " ok\nWriting out result..." << std::flush;
        timed(perf, "Writing graph", [&] {
            std::vector<uint8_t> out;
            if (g) {
                int64_t n = 0, b, e, nr = 0;
                check(dmx_graph_info(g, &n, &b, &e, &nr));
                std::vector<float> attrs((size_t)n * 3);
                std::vector<int32_t> bins((size_t)n * 128);
                std::vector<int16_t> runs((size_t)std::max<int64_t>(nr, 1) * 4);
                std::vector<uint8_t> gc((size_t)n);
                check(dmx_graph_copy(g, attrs.data(), bins.data(), runs.data(), gc.data()));
                dmx_graph_free(g);
                // sparkGraph2 columns (pointdata.cpp:1268-1270), displayed = Connectivity
                const std::vector<std::string> names = {"Connectivity", "Point First Moment", "Point Second Moment"};
                std::vector<std::vector<float>> cols(3, std::vector<float>((size_t)n));
                for (int j = 0; j < 3; j++)
                    for (int64_t k = 0; k < n; k++) cols[j][k] = attrs[k * 3 + j];
                out = write_chunk(pm, n, bins.data(), runs.data(), nr, gc.data(), names, cols, {1, 0, 0}, 0, boundary,
                                  map_name);
            } else {
                out = write_chunk(pm, 0, nullptr, nullptr, 0, nullptr, {}, {}, {}, -2, false, map_name);
            }
            d.put_displayed(out, new_map);
            write_document(a.out, d);
        });
        std::cout << " ok" << std::endl;
    }
};

// VgaParser (vgaparser.cpp:29-106), RadiusConverter (radiusconverter.cpp:24-37), runVga (runmethods.cpp:227-267)
struct Vga : Mode {
    enum { NONE, ISOVIST, VISIBILITY, METRIC, ANGULAR, THRU } mode = NONE;
    bool local = false, global = false;
    std::string radius;
    std::string name() const override { return "VGA"; }
    void parse(int argc, char** argv) override {
        for (int i = 1; i < argc;) {
            if (!std::strcmp("-vm", argv[i])) {
                if (mode != NONE) throw CommandLineException("-vm can only be used once, modes are mutually exclusive");
                enforce_argument("-vm", i, argc, argv);
                if (!std::strcmp(argv[i], "isovist")) mode = ISOVIST;
                else if (!std::strcmp(argv[i], "visibility")) mode = VISIBILITY;
                else if (!std::strcmp(argv[i], "metric")) mode = METRIC;
                else if (!std::strcmp(argv[i], "angular")) mode = ANGULAR;
                else if (!std::strcmp(argv[i], "thruvision")) mode = THRU;
                else throw CommandLineException(std::string("Invalid VGA mode: ") + argv[i]);
            } else if (!std::strcmp(argv[i], "-vg")) {
                global = true;
            } else if (!std::strcmp(argv[i], "-vl")) {
                local = true;
            } else if (!std::strcmp(argv[i], "-vr")) {
                enforce_argument("-vr", i, argc, argv);
                radius = argv[i];
            }
            ++i;
        }
        if (mode == NONE) mode = ISOVIST;
        if (mode == VISIBILITY && global) {
            if (radius.empty())
                throw CommandLineException("Global measures in VGA/visibility analysis require a radius, use -vr <radius>");
            if (radius != "n" && !has_only_digits(radius))
                throw CommandLineException(std::string("Radius must be a positive integer number or n, got ") + radius);
        } else if (mode == METRIC) {
            if (radius.empty()) throw CommandLineException("Metric vga requires a radius, use -vr <radius>");
        }
    }
    // runVga METRIC branch (runmethods.cpp:245-248, RadiusConverter::ConvertForMetric
    // radiusconverter.cpp:39-60) -> VGAMetric::run (vgametric.cpp:26-136)
    // runVga ANGULAR branch (runmethods.cpp:249-251: no radius option, so -1) -> VGAAngular::run
    // (vgaangular.cpp:26-133) shares the writer below.
    void run_metric(const Args& a, Perf& perf, Document& d, Context& C, LoadedMap& m) {
        const bool ang = mode == ANGULAR;
        double r = -1.0;
        if (!ang && radius != "n") {
            char* end = nullptr;
            r = std::strtod(radius.c_str(), &end);
            if (r <= 0)
                throw RuntimeException(std::string("Radius for metric vga must be n for the whole range or a positive "
                                                   "number. Got ") + radius);
            if (std::isnan(r)) throw RuntimeException("Radius NaN?! Really?");
            if (std::isinf(r)) throw RuntimeException("Radius inf?! Who are you kidding?");
        }
        std::cout << " ok\nAnalysing graph..." << std::flush;
        const int nc = ang ? 3 : 4;
        std::vector<float> out((size_t)m.nnodes * nc, -1.0f);
        timed(perf, "Run VGA", [&] {
            check(ang ? dmx_vga_angular(C.ctx, m.g, r, 0, 0, -1, out.data())
                      : dmx_vga_metric(C.ctx, m.g, r, 0, 0, -1, out.data()));
        });
        std::cout << " ok\nWriting out result..." << std::flush;
        timed(perf, "Writing graph", [&] {
            // radius suffix (vgametric.cpp:34-43) from the PointMap region (pointdata.cpp:151-154)
            std::string suffix;
            if (r != -1.0) {
                int32_t cols_ = 0, rows_ = 0;
                double blx = 0, bly = 0;
                check(dmx_pointmap_info(m.pm, &cols_, &rows_, &blx, &bly, nullptr));
                double sp = 0;
                check(dmx_chunk_info(m.chunk, nullptr, nullptr, &sp, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr));
                const double width = (blx + double(cols_ - 1) * sp + sp / 2.0) - (blx - sp / 2.0);
                char buf[64];
                snprintf(buf, sizeof(buf), r > 100.0 ? "%.f" : (width < 1.0 ? "%.4f" : "%.2f"), r);
                suffix = std::string(" R") + buf;
            }
            const char* mnames[4] = {"Metric Mean Shortest-Path Angle", "Metric Mean Shortest-Path Distance",
                                     "Metric Mean Straight-Line Distance", "Metric Node Count"};
            // VGAAngular inserts Mean Depth, Total Depth, Node Count (vgaangular.cpp:43-48)
            const char* anames[3] = {"Angular Mean Depth", "Angular Total Depth", "Angular Node Count"};
            std::vector<float> v((size_t)m.nnodes);
            for (int j = 0; j < nc; j++) {
                for (int64_t i = 0; i < m.nnodes; i++) v[i] = out[i * nc + j];
                // setDisplayedAttribute(mspl_col) / (mean_depth_col)
                m.column(std::string(ang ? anames[j] : mnames[j]) + suffix, v.data(), nullptr, false, j == (ang ? 0 : 1));
            }
            d.put_displayed(m.bytes(), false);
            write_document(a.out, d);
        });
        std::cout << " ok" << std::endl;
    }
    void run(const Args& a, Perf& perf) override {
        Document d;
        // the reference's loadGraph reads and parses the whole file: the chunk decode and the upload count in
        // "Load graph file" too (the device context's creation does not)
        const auto t0 = std::chrono::steady_clock::now();
        read_document(a.file, d);
        const auto t1 = std::chrono::steady_clock::now();
        Context C;
        LoadedMap m;
        const auto t2 = std::chrono::steady_clock::now();
        load_map(C, d, m);
        // the document's drawing: VGA global on the re-read (asymmetric) graph takes the asymmetric mode with it
        if (!d.lines.empty()) check(dmx_graph_set_drawing(m.g, d.lines.data(), (int64_t)d.lines.size() / 4));
        perf.add("Load graph file", std::chrono::duration<double>((t1 - t0) + (std::chrono::steady_clock::now() - t2)).count());
        std::cout << "Getting options..." << std::flush;
        if (mode == METRIC || mode == ANGULAR) {
            run_metric(a, perf, d, C, m);
            return;
        }
        if (mode != VISIBILITY)
            throw RuntimeException("Only -vm visibility, metric and angular are part of the accelerated path");
        double r = -1.0;
        if (global) {
            if (radius != "n") {
                const long rad = std::strtol(radius.c_str(), nullptr, 10);
                if (rad < 1 || rad > 99)
                    throw RuntimeException(std::string("Radius for visibility analysis must be n for the whole range or an "
                                                       "integer between 1 and 99 inclusive. Got ") + radius);
                r = (double)rad;
            }
        }
        std::cout << " ok\nAnalysing graph..." << std::flush;
        std::vector<float> out((size_t)m.nnodes * 7, -1.0f), lout;
        // analyseGraph runs VGAVisualLocal before VGAVisualGlobal (mgraph.cpp:349-356), one "Run VGA" span
        timed(perf, "Run VGA", [&] {
            if (local) {
                lout.assign((size_t)m.nnodes * 3, -1.0f);
                check(dmx_vga_local(C.ctx, m.g, 0, 0, -1, lout.data()));
            }
            if (global) check(dmx_vga_global(C.ctx, m.g, r, 0, 0, -1, out.data(), nullptr));
        });
        std::cout << " ok\nWriting out result..." << std::flush;
        timed(perf, "Writing graph", [&] {
            // VGAVisualGlobal::run column insertion order and setValue pattern (vgavisualglobal.cpp:38-193)
            const std::string suffix = r != -1.0 ? " R" + std::to_string((int)r) : std::string();
            struct Spec { const char* name; int outcol; bool simple; };
            const Spec specs[7] = {{"Visual Entropy", 0, false}, {"Visual Integration [HH]", 1, true},
                                   {"Visual Integration [P-value]", 2, false}, {"Visual Integration [Tekl]", 3, false},
                                   {"Visual Mean Depth", 4, false}, {"Visual Node Count", 5, false},
                                   {"Visual Relativised Entropy", 6, false}};
            std::vector<float> v((size_t)m.nnodes);
            std::vector<uint8_t> set((size_t)m.nnodes);
            if (local && !a.simple) {
                // VGAVisualLocal: three columns (vgavisuallocal.cpp:31-35), set for every source it does
                // not skip (context-filled odd cells), displayed = clustering coefficient (:109-112)
                int32_t cols_ = 0, rows_ = 0;
                check(dmx_pointmap_info(m.pm, &cols_, &rows_, nullptr, nullptr, nullptr));
                std::vector<int32_t> st((size_t)cols_ * rows_);
                check(dmx_pointmap_state(m.pm, st.data()));
                std::vector<uint8_t> ran((size_t)m.nnodes, 0);
                int64_t k = 0;
                for (int64_t c = 0; c < (int64_t)st.size() && k < m.nnodes; c++) {
                    if (!(st[c] & 0x2)) continue;   // Point::FILLED; nodes are the filled cells, x-major
                    const int64_t x = c / rows_, y = c % rows_;
                    ran[k++] = !((st[c] & 0x8) && !(x % 2 == 0 && y % 2 == 0));   // Point::CONTEXTFILLED
                }
                const char* lnames[3] = {"Visual Clustering Coefficient", "Visual Control", "Visual Controllability"};
                for (int j = 0; j < 3; j++) {
                    for (int64_t i = 0; i < m.nnodes; i++) v[i] = lout[i * 3 + j];
                    m.column(lnames[j], v.data(), ran.data(), false, j == 0);
                }
            }
            if (global)
                for (auto& sp : specs) {
                    if (a.simple && !sp.simple) continue;
                    for (int64_t k = 0; k < m.nnodes; k++) {
                        const float tn = out[k * 7 + 5];
                        const bool ran = tn >= 1.0f;   // skipped sources set nothing
                        bool on = ran;
                        if (sp.outcol >= 1 && sp.outcol <= 3) on = ran && tn > 1.0f;   // HH / P / Tekl need > 1 node
                        v[k] = out[k * 7 + sp.outcol];
                        set[k] = on ? 1 : 0;
                    }
                    m.column(sp.name + suffix, v.data(), set.data(), false, sp.outcol == 1);
                }
            d.put_displayed(m.bytes(), false);
            write_document(a.out, d);
        });
        std::cout << " ok" << std::endl;
    }
};

// StepDepthParser (stepdepthparser.cpp:26-100) + runStepDepth (runmethods.cpp:735-778)
struct StepDepth : Mode {
    enum { NONE, ANGULAR, METRIC, VISUAL } type = NONE;
    std::vector<std::pair<double, double>> points;
    std::string name() const override { return "STEPDEPTH"; }
    void parse(int argc, char** argv) override {
        std::vector<std::string> pts;
        std::string pointFile;
        for (int i = 1; i < argc; ++i) {
            if (!std::strcmp("-sdp", argv[i])) {
                if (!pointFile.empty()) throw CommandLineException("-sdp cannot be used together with -sdf");
                enforce_argument("-sdp", i, argc, argv);
                if (!has_only_digits_dots_commas(argv[i])) {
                    std::stringstream m;
                    m << "Invalid step depth point provided (" << argv[i] << "). Should only contain digits dots and commas";
                    throw CommandLineException(m.str());
                }
                pts.push_back(argv[i]);
            } else if (!std::strcmp("-sdf", argv[i])) {
                if (!pts.empty()) throw CommandLineException("-sdf cannot be used together with -sdp");
                enforce_argument("-sdf", i, argc, argv);
                pointFile = argv[i];
            } else if (!std::strcmp("-sdt", argv[i])) {
                enforce_argument("-sdt", i, argc, argv);
                if (!std::strcmp(argv[i], "angular")) type = ANGULAR;
                else if (!std::strcmp(argv[i], "metric")) type = METRIC;
                else if (!std::strcmp(argv[i], "visual")) type = VISUAL;
                else throw CommandLineException(std::string("Invalid step type: ") + argv[i]);
            }
        }
        if (pointFile.empty() && pts.empty()) throw CommandLineException("Either -sdp or -sdf must be given");
        points = points_from_args(pts, pointFile);
        if (type == NONE) throw CommandLineException("Step depth type (-sdt) must be provided");
    }
    void run(const Args& a, Perf& perf) override {
        Document d;
        timed(perf, "Load graph file", [&] { read_document(a.file, d); });
        Context C;
        LoadedMap m;
        load_map(C, d, m);
        std::cout << "ok\nSelecting cells... " << std::flush;
        int32_t cols = 0, rows = 0;
        double spacing = 0, bl[2] = {0, 0};
        check(dmx_chunk_info(m.chunk, &cols, &rows, &spacing, bl, nullptr, nullptr, nullptr, nullptr, nullptr));
        std::vector<int32_t> sel;
        for (auto& p : points) {
            if (!(p.first >= d.region[0] && p.first <= d.region[2] && p.second >= d.region[1] && p.second <= d.region[3]))
                throw RuntimeException("Point outside of target region");
            // PointMap::pixelate(p, constrain=true) (pointdata.cpp:263-283)
            int x = (int)std::floor((p.first - bl[0] + spacing / 2.0) / spacing);
            int y = (int)std::floor((p.second - bl[1] + spacing / 2.0) / spacing);
            x = std::min(std::max(x, 0), cols - 1);
            y = std::min(std::max(y, 0), rows - 1);
            sel.push_back(x * rows + y);
        }
        std::cout << "ok\nCalculating step-depth... " << std::flush;
        std::vector<float> out((size_t)m.nnodes * 3, -1.0f);
        int rc = DMX_OK;
        timed(perf, "Calculating step-depth", [&] {
            rc = type == METRIC   ? dmx_metric_stepdepth(C.ctx, m.g, sel.data(), (int64_t)sel.size(), out.data())
                 : type == ANGULAR ? dmx_angular_stepdepth(C.ctx, m.g, sel.data(), (int64_t)sel.size(), out.data())
                                   : dmx_visual_stepdepth(C.ctx, m.g, sel.data(), (int64_t)sel.size(), out.data());
        });
        if (rc != DMX_OK && rc != DMX_ERR_STATE) check(rc);   // no selection: analyseGraph returns false
        std::cout << " ok\nWriting out result..." << std::flush;
        timed(perf, "Writing graph", [&] {
            std::vector<float> v((size_t)m.nnodes);
            std::vector<uint8_t> set((size_t)m.nnodes);
            if (rc == DMX_OK && (type == VISUAL || type == ANGULAR)) {
                // VGAVisualGlobalDepth::run / VGAAngularDepth::run: one column, reset to -1, set on every
                // reached cell (vgavisualglobaldepth.cpp:28, :49; vgaangulardepth.cpp:27, :53-55)
                for (int64_t k = 0; k < m.nnodes; k++) {
                    v[k] = out[k];
                    set[k] = out[k] >= 0.0f ? 1 : 0;
                }
                m.column(type == VISUAL ? "Visual Step Depth" : "Angular Step Depth", v.data(), set.data(), false, true);
            } else if (rc == DMX_OK) {
                // VGAMetricDepth::run column order (vgametricdepth.cpp:27-33); cells it never pops keep -1
                const bool single = [&] {   // PointMap::setCurSel keeps FILLED cells only
                    std::vector<int32_t> st((size_t)cols * rows);
                    check(dmx_chunk_arrays(m.chunk, st.data(), nullptr, nullptr, nullptr));
                    std::vector<int32_t> s;
                    for (int32_t c : sel)
                        if (st[c] & 2) s.push_back(c);
                    std::sort(s.begin(), s.end());
                    s.erase(std::unique(s.begin(), s.end()), s.end());
                    return s.size() == 1;
                }();
                const char* names[3] = {"Metric Step Shortest-Path Angle", "Metric Step Shortest-Path Length",
                                        "Metric Straight-Line Distance"};
                for (int j = 0; j < (single ? 3 : 2); j++) {
                    for (int64_t k = 0; k < m.nnodes; k++) {
                        v[k] = out[k * 3 + j];
                        set[k] = out[k * 3 + 1] >= 0.0f ? 1 : 0;
                    }
                    m.column(names[j], v.data(), set.data(), false, j == 1);
                }
            }
            // the selection stays on the map the CLI writes (Point::SELECTED)
            check(dmx_chunk_select_cells(m.chunk, sel.data(), (int64_t)sel.size()));
            d.put_displayed(m.bytes(), false);
            write_document(a.out, d);
        });
        std::cout << " ok" << std::endl;
    }
};

void print_help() {
    std::cout << "Usage: dmxcli -m <mode> -f <filename> -o <output file> [-t <times.csv>] [-s] [-p] [mode options]\n"
                 "Modes (the accelerated depthmapXcli path):\n"
                 "  VISPREP   -pg <grid spacing> -pp <x,y> | -pf <points file> [-pr <max visibility>] [-pb] [-pm]\n"
                 "  VGA       -vm visibility [-vl] [-vg -vr <radius|n>] | -vm metric -vr <radius|n> | -vm angular\n"
                 "  STEPDEPTH -sdt metric|visual|angular -sdp <x,y> | -sdf <points file>\n"
                 "Input: a depthmapX .graph (written back as .graph), or a CSV drawing (x1,y1,x2,y2) / a .dmxg\n"
                 "written by this tool (written as .dmxg)\n";
}

} // namespace

int main(int argc, char* argv[]) {
    std::vector<std::unique_ptr<Mode>> modes;
    modes.emplace_back(new VisPrep());
    modes.emplace_back(new Vga());
    modes.emplace_back(new StepDepth());
    try {
        // CommandLineParser::parse (commandlineparser.cpp:51-133)
        if (argc <= 1) throw CommandLineException("No commandline parameters provided - don't know what to do");
        Mode* mode = nullptr;
        Args a;
        for (int i = 1; i < argc;) {
            if (!std::strcmp("-h", argv[i])) { print_help(); return 0; }
            if (!std::strcmp("-v", argv[i])) { std::cout << "dmxcli (depthmapX VISPREP/VGA/STEPDEPTH on MI355X)\n"; return 0; }
            if (!std::strcmp("-m", argv[i])) {
                if (mode) throw CommandLineException("-m can only be used once");
                enforce_argument("-m", i, argc, argv);
                for (auto& m : modes)
                    if (m->name() == argv[i]) mode = m.get();
                if (!mode) throw CommandLineException(std::string("Invalid mode: ") + argv[i]);
            } else if (!std::strcmp("-f", argv[i])) {
                enforce_argument("-f", i, argc, argv);
                a.file = argv[i];
            } else if (!std::strcmp("-o", argv[i])) {
                enforce_argument("-o", i, argc, argv);
                a.out = argv[i];
            } else if (!std::strcmp("-t", argv[i])) {
                enforce_argument("-t", i, argc, argv);
                a.timing = argv[i];
            } else if (!std::strcmp("-s", argv[i])) {
                a.simple = true;
            } else if (!std::strcmp("-p", argv[i])) {
                a.progress = true;
                g_print_progress = true;
            }
            ++i;
        }
        if (!mode) throw CommandLineException("-m for mode is required");
        if (a.file.empty()) throw CommandLineException("-f for input file is required");
        if (a.out.empty()) throw CommandLineException("-o for output file is required");
        mode->parse(argc, argv);
        Perf perf;
        perf.file = a.timing;
        mode->run(a, perf);
        perf.write();
    } catch (std::exception& e) {
        std::cout << e.what() << "\n"
                  << "Type 'depthmapXcli -h' for help" << std::endl;
        return -1;
    }
    return 0;
}
