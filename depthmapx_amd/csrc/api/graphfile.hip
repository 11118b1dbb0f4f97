// api/graphfile.hip -- the .graph file (MetaGraph container).
// Part of the dmx_api.hip unity build: included inside its extern "C" block, after the context and the
// internal types (dmx_ctx, dmx_pointmap, dmx_graph); not compiled on its own.

// ---------------------------------------------------------------- .graph file (MetaGraph container)
struct dmx_graphfile {
    GraphFile gf;
    std::vector<double> lines;
};

int dmx_graphfile_read(const char* path, dmx_graphfile** out) {
    if (!path || !out) return fail(DMX_ERR_ARG, "bad arguments");
    FILE* f = fopen(path, "rb");
    if (!f) return fail(DMX_ERR_ARG, std::string("cannot open ") + path);
    std::vector<uint8_t> buf;
    uint8_t tmp[1 << 16];
    size_t k;
    while ((k = fread(tmp, 1, sizeof(tmp), f)) > 0) buf.insert(buf.end(), tmp, tmp + k);
    fclose(f);
    std::unique_ptr<dmx_graphfile> g(new dmx_graphfile());
    std::string err;
    const int rc = read_graphfile(buf.data(), buf.size(), g->gf, err);
    if (rc == -2) return fail(DMX_ERR_UNSUPPORTED, err);
    if (rc) return fail(DMX_ERR_ARG, err);
    g->lines = graphfile_lines(g->gf);
    *out = g.release();
    return DMX_OK;
}

int dmx_graphfile_free(dmx_graphfile* g) {
    delete g;
    return DMX_OK;
}

int dmx_graphfile_write(const dmx_graphfile* g, const char* path) {
    if (!g || !path) return fail(DMX_ERR_ARG, "bad arguments");
    std::vector<uint8_t> out;
    std::string err;
    if (write_graphfile(g->gf, out, err)) return fail(DMX_ERR_STATE, err);
    FILE* f = fopen(path, "wb");
    if (!f) return fail(DMX_ERR_ARG, std::string("cannot write ") + path);
    const size_t w = fwrite(out.data(), 1, out.size(), f);
    fclose(f);
    if (w != out.size()) return fail(DMX_ERR_ARG, std::string("short write to ") + path);
    return DMX_OK;
}

int dmx_graphfile_info(const dmx_graphfile* g, int32_t* state, int32_t* view_class, double* region, int64_t* nlines,
                       int32_t* npointmaps, int32_t* displayed) {
    if (!g) return fail(DMX_ERR_ARG, "graph file is NULL");
    if (state) *state = g->gf.state;
    if (view_class) *view_class = g->gf.view_class;
    if (region) std::memcpy(region, g->gf.region, sizeof(g->gf.region));
    if (nlines) *nlines = (int64_t)g->lines.size() / 4;
    if (npointmaps) *npointmaps = (int32_t)g->gf.pointmaps.size();
    if (displayed) *displayed = g->gf.displayed_pointmap;
    return DMX_OK;
}

int dmx_graphfile_lines(const dmx_graphfile* g, double* lines) {
    if (!g || (!lines && !g->lines.empty())) return fail(DMX_ERR_ARG, "bad arguments");
    if (!g->lines.empty()) std::memcpy(lines, g->lines.data(), g->lines.size() * sizeof(double));
    return DMX_OK;
}

int dmx_graphfile_set_view(dmx_graphfile* g, int32_t state, int32_t view_class) {
    if (!g) return fail(DMX_ERR_ARG, "graph file is NULL");
    g->gf.state = state;
    g->gf.view_class = view_class;
    return DMX_OK;
}

int dmx_graphfile_pointmap(const dmx_graphfile* g, int i, const uint8_t** chunk, int64_t* size) {
    if (!g || !chunk || !size || i < 0 || i >= (int)g->gf.pointmaps.size()) return fail(DMX_ERR_ARG, "bad point map index");
    *chunk = g->gf.pointmaps[i].data();
    *size = (int64_t)g->gf.pointmaps[i].size();
    return DMX_OK;
}

int dmx_graphfile_put_pointmap(dmx_graphfile* g, int i, const uint8_t* chunk, int64_t size) {
    if (!g || !chunk || size <= 0 || i < -1 || i >= (int)g->gf.pointmaps.size()) return fail(DMX_ERR_ARG, "bad arguments");
    if (i < 0) {   // MetaGraph::addNewPointMap: appended and displayed
        g->gf.pointmaps.emplace_back(chunk, chunk + size);
        g->gf.displayed_pointmap = (int32_t)g->gf.pointmaps.size() - 1;
    } else {
        g->gf.pointmaps[i].assign(chunk, chunk + size);
    }
    return DMX_OK;
}

int dmx_graphfile_new_pointmap_name(const dmx_graphfile* g, char* name, int cap) {
    if (!g || !name || cap <= 0) return fail(DMX_ERR_ARG, "bad arguments");
    const std::string n = new_pointmap_name(g->gf, "VGA Map");
    if ((int)n.size() + 1 > cap) return fail(DMX_ERR_ARG, "buffer too small");
    std::memcpy(name, n.c_str(), n.size() + 1);
    return DMX_OK;
}

int32_t dmx_view_vga_top(int32_t view_class) { return view_vga_top(view_class); }
