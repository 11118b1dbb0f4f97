// api/chunk.hip -- the .graph PointMap chunk: parse, load, columns, serialise.
// Part of the dmx_api.hip unity build: included inside its extern "C" block, after the context and the
// internal types (dmx_ctx, dmx_pointmap, dmx_graph); not compiled on its own.

// ---------------------------------------------------------------- .graph PointMap chunk
struct dmx_chunk {
    ParsedChunk pc;
};

int dmx_graph_from_runs(dmx_ctx* ctx, dmx_pointmap* pm, int64_t nnodes, const int32_t* bins, const int16_t* runs,
                        int64_t nruns, const uint8_t* gridconn, const float* attrs, dmx_graph** out) {
    if (!ctx || !pm || !out || nnodes < 0 || nruns < 0 || (nnodes && !bins) || (nruns && !runs))
        return fail(DMX_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(ctx->device));
    int rc = upload_pointmap(ctx, pm);
    if (rc) return rc;
    if (nnodes != pm->nnodes) return fail(DMX_ERR_ARG, "node count does not match the filled cells of the map");
    const int64_t N = nnodes;
    std::vector<int32_t> bn((size_t)std::max<int64_t>(N, 1) * 32), nr((size_t)std::max<int64_t>(N, 1));
    std::vector<uint16_t> bc((size_t)std::max<int64_t>(N, 1) * 32);
    std::vector<float> bd((size_t)std::max<int64_t>(N, 1) * 32);
    std::vector<int64_t> st((size_t)std::max<int64_t>(N, 1));
    int64_t acc = 0;
    for (int64_t k = 0; k < N; k++) {
        int s = 0;
        for (int b = 0; b < 32; b++) {
            const int32_t* r = bins + (k * 32 + b) * 4;
            bn[k * 32 + b] = r[3];
            bc[k * 32 + b] = (uint16_t)r[1];
            std::memcpy(&bd[k * 32 + b], &r[2], 4);
            s += r[3];
        }
        nr[k] = s;
        st[k] = acc;
        acc += s;
    }
    if (acc != nruns) return fail(DMX_ERR_ARG, "bins do not account for the runs");
    std::unique_ptr<dmx_graph> g(new dmx_graph());
    g->ctx = ctx; g->pm = pm; g->nnodes = N; g->node_begin = 0; g->node_end = N; g->nruns = nruns;
    inherit_merges(g.get());
    HIPCHK(g->pool.alloc(std::max<int64_t>(nruns, 1)));
    HIPCHK(g->node_run_start.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(g->node_nruns.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(g->bin_nruns.alloc(std::max<int64_t>(N, 1) * 32));
    HIPCHK(g->bin_count.alloc(std::max<int64_t>(N, 1) * 32));
    HIPCHK(g->bin_dist.alloc(std::max<int64_t>(N, 1) * 32));
    HIPCHK(g->attrs.alloc(std::max<int64_t>(N, 1) * 3));
    HIPCHK(g->gridconn.alloc(std::max<int64_t>(N, 1)));
    hipStream_t s = ctx->stream;
    if (nruns) HIPCHK(hipMemcpyAsync(g->pool.p, runs, nruns * 8, hipMemcpyHostToDevice, s));
    if (N) {
        HIPCHK(hipMemcpyAsync(g->node_run_start.p, st.data(), N * 8, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(g->node_nruns.p, nr.data(), N * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(g->bin_nruns.p, bn.data(), N * 32 * 4, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(g->bin_count.p, bc.data(), N * 32 * 2, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(g->bin_dist.p, bd.data(), N * 32 * 4, hipMemcpyHostToDevice, s));
        if (attrs) HIPCHK(hipMemcpyAsync(g->attrs.p, attrs, N * 12, hipMemcpyHostToDevice, s));
        else HIPCHK(hipMemsetAsync(g->attrs.p, 0, N * 12, s));
        if (gridconn) HIPCHK(hipMemcpyAsync(g->gridconn.p, gridconn, N, hipMemcpyHostToDevice, s));
        else HIPCHK(hipMemsetAsync(g->gridconn.p, 0, N, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    *out = g.release();
    return DMX_OK;
}

int dmx_chunk_write(const dmx_pointmap* pm, int64_t nnodes, const int32_t* bins, const int16_t* runs, int64_t nruns,
                    const uint8_t* gridconn, int ncols, const char* const* names, const float* values,
                    const uint8_t* locked, const uint8_t* setmask, int displayed, int boundary, uint8_t* buf, int64_t cap,
                    int64_t* size) {
    if (!pm || !size || nnodes < 0 || ncols < 0 || (ncols && (!names || !values))) return fail(DMX_ERR_ARG, "bad arguments");
    std::vector<ChunkColumn> cols((size_t)ncols);
    for (int i = 0; i < ncols; i++) {
        cols[i].name = names[i];
        cols[i].locked = locked ? locked[i] != 0 : false;
        cols[i].values.assign(values + (size_t)i * nnodes, values + (size_t)(i + 1) * nnodes);
        if (setmask) cols[i].set.assign(setmask + (size_t)i * nnodes, setmask + (size_t)(i + 1) * nnodes);
    }
    std::vector<uint8_t> out;
    std::string err;
    if (write_pointmap_chunk(*pm->host, nnodes, bins, runs, nruns, gridconn, cols, displayed, boundary != 0, out, err))
        return fail(DMX_ERR_ARG, err);
    *size = (int64_t)out.size();
    if (buf) {
        if (cap < (int64_t)out.size()) return fail(DMX_ERR_ARG, "buffer too small");
        std::memcpy(buf, out.data(), out.size());
    }
    return DMX_OK;
}

int dmx_chunk_parse(const uint8_t* buf, int64_t size, dmx_chunk** out) {
    if (!buf || !out || size <= 0) return fail(DMX_ERR_ARG, "bad arguments");
    std::unique_ptr<dmx_chunk> c(new dmx_chunk());
    std::string err;
    if (read_pointmap_chunk(buf, (size_t)size, c->pc, err)) return fail(DMX_ERR_ARG, err);
    *out = c.release();
    return DMX_OK;
}

int dmx_chunk_free(dmx_chunk* c) {
    delete c;
    return DMX_OK;
}

int dmx_chunk_info(const dmx_chunk* c, int32_t* cols, int32_t* rows, double* spacing, double* bl, int64_t* nnodes,
                   int64_t* nruns, int32_t* ncols, int32_t* displayed_sorted, int64_t* bytes_used) {
    if (!c) return fail(DMX_ERR_ARG, "chunk is NULL");
    const ParsedChunk& p = c->pc;
    if (cols) *cols = p.cols;
    if (rows) *rows = p.rows;
    if (spacing) *spacing = p.spacing;
    if (bl) { bl[0] = p.blx; bl[1] = p.bly; }
    if (nnodes) *nnodes = (int64_t)p.gridconn.size();
    if (nruns) *nruns = (int64_t)p.runs.size() / 4;
    if (ncols) *ncols = (int32_t)p.columns.size();
    if (displayed_sorted) *displayed_sorted = p.displayed_sorted;
    if (bytes_used) *bytes_used = (int64_t)p.bytes_used;
    return DMX_OK;
}

int dmx_chunk_column(const dmx_chunk* c, int i, char* name, int name_cap, float* values, int* locked) {
    if (!c || i < 0 || i >= (int)c->pc.columns.size()) return fail(DMX_ERR_ARG, "bad column");
    const ChunkColumn& col = c->pc.columns[i];
    if (name && name_cap > 0) {
        const size_t n = std::min<size_t>(col.name.size(), (size_t)name_cap - 1);
        std::memcpy(name, col.name.data(), n);
        name[n] = 0;
    }
    if (values && !col.values.empty()) std::memcpy(values, col.values.data(), col.values.size() * 4);
    if (locked) *locked = col.locked ? 1 : 0;
    return DMX_OK;
}

int dmx_chunk_arrays(const dmx_chunk* c, int32_t* state, int32_t* bins, int16_t* runs, uint8_t* gridconn) {
    if (!c) return fail(DMX_ERR_ARG, "chunk is NULL");
    const ParsedChunk& p = c->pc;
    if (state) std::memcpy(state, p.state.data(), p.state.size() * 4);
    if (bins && !p.bins.empty()) std::memcpy(bins, p.bins.data(), p.bins.size() * 4);
    if (runs && !p.runs.empty()) std::memcpy(runs, p.runs.data(), p.runs.size() * 2);
    if (gridconn && !p.gridconn.empty()) std::memcpy(gridconn, p.gridconn.data(), p.gridconn.size());
    return DMX_OK;
}

int dmx_pointmap_set_state(dmx_pointmap* pm, const int32_t* state) {
    if (!pm || !state) return fail(DMX_ERR_ARG, "bad arguments");
    PointMapHost& h = *pm->host;
    h.restore_fill(state);
    pm->version++;
    return DMX_OK;
}

int dmx_chunk_load(dmx_ctx* ctx, const dmx_chunk* c, const double* region, dmx_pointmap** pm_out, dmx_graph** g_out) {
    if (!ctx || !c || !region || !pm_out || !g_out) return fail(DMX_ERR_ARG, "bad arguments");
    const ParsedChunk& p = c->pc;
    if (!p.processed) return fail(DMX_ERR_STATE, "the point map has no graph (run VISPREP -pm first)");
    Rect r{region[0], region[1], region[2], region[3]};
    std::unique_ptr<dmx_pointmap> pm(new dmx_pointmap());
    pm->host.reset(new PointMapHost(r, p.spacing, nullptr, 0));
    pm->host->load_state(p.cols, p.rows, p.spacing, Vec2{p.blx, p.bly}, p.state.data());
    const int64_t N = (int64_t)p.gridconn.size();
    std::vector<float> attrs((size_t)std::max<int64_t>(N, 1) * 3, 0.0f);
    const char* mk[3] = {"Connectivity", "Point First Moment", "Point Second Moment"};
    for (int j = 0; j < 3; j++)
        for (const auto& col : p.columns)
            if (col.name == mk[j] && (int64_t)col.values.size() == N)
                for (int64_t k = 0; k < N; k++) attrs[k * 3 + j] = col.values[k];
    dmx_graph* g = nullptr;
    int rc = dmx_graph_from_runs(ctx, pm.get(), N, p.bins.data(), p.runs.data(), (int64_t)p.runs.size() / 4,
                                 p.gridconn.data(), attrs.data(), &g);
    if (rc) return rc;
    std::unique_ptr<dmx_graph> gg(g);
    {
        std::vector<int32_t> per_cell, uniq;
        rc = normalize_merges(pm->host->cells(), p.merge_pairs.data(), (int64_t)p.merge_pairs.size() / 2, per_cell, uniq,
                              true);
        if (rc) return rc;
        pm->host->set_merge(std::move(per_cell));
    }
    inherit_merges(g);
    *pm_out = pm.release();
    *g_out = gg.release();
    return DMX_OK;
}

int dmx_pointmap_set_merges(dmx_pointmap* pm, const int32_t* cell_pairs, int64_t n) {
    if (!pm || n < 0 || (n && !cell_pairs)) return fail(DMX_ERR_ARG, "bad arguments");
    std::vector<int32_t> per_cell, uniq;
    if (int rc = normalize_merges(pm->host->cells(), cell_pairs, n, per_cell, uniq)) return rc;
    pm->host->set_merge(std::move(per_cell));
    return DMX_OK;
}

int dmx_graph_set_merges(dmx_graph* g, const int32_t* cell_pairs, int64_t n) {
    if (!g || n < 0 || (n && !cell_pairs)) return fail(DMX_ERR_ARG, "bad arguments");
    std::vector<int32_t> per_cell, uniq;
    if (int rc = normalize_merges(g->pm->host->cells(), cell_pairs, n, per_cell, uniq)) return rc;
    // the links belong to the points (Point::m_merge): the map gets them too, so a chunk written from it
    // saves them and a graph made from it again follows them
    g->pm->host->set_merge(std::move(per_cell));
    g->merges = std::move(uniq);
    g->merges_ready = false;
    if (g->merges.empty()) {   // prepare_merges returns early on no links: drop the previous links' device state
        g->nmamb = 0;
        g->d_mamb.reset();
        g->d_mpairs.reset();
        g->d_merge_cell.reset();
    }
    return DMX_OK;
}

int dmx_chunk_merges(const dmx_chunk* c, int32_t* cell_pairs, int64_t* n) {
    if (!c || !n) return fail(DMX_ERR_ARG, "bad arguments");
    std::vector<int32_t> per_cell, uniq;
    const ParsedChunk& p = c->pc;
    if (int rc = normalize_merges((int64_t)p.cols * p.rows, p.merge_pairs.data(), (int64_t)p.merge_pairs.size() / 2,
                                  per_cell, uniq, true))
        return rc;
    const int64_t m = (int64_t)uniq.size() / 2;
    if (cell_pairs) {
        if (*n < m) return fail(DMX_ERR_ARG, "buffer too small");
        std::memcpy(cell_pairs, uniq.data(), uniq.size() * 4);
    }
    *n = m;
    return DMX_OK;
}

int dmx_chunk_flags(const dmx_chunk* c, int* processed, int* boundary, int64_t* merges, int64_t* nrows) {
    if (!c) return fail(DMX_ERR_ARG, "chunk is NULL");
    if (processed) *processed = c->pc.processed ? 1 : 0;
    if (boundary) *boundary = c->pc.boundary ? 1 : 0;
    if (merges) *merges = c->pc.merges;
    if (nrows) *nrows = (int64_t)c->pc.row_keys.size();
    return DMX_OK;
}

int dmx_chunk_set_column(dmx_chunk* c, const char* name, const float* values, const uint8_t* setmask, int locked,
                         int make_displayed) {
    if (!c || !name || (!values && !c->pc.row_keys.empty())) return fail(DMX_ERR_ARG, "bad arguments");
    const int idx = chunk_set_column(c->pc, name, values, setmask, locked != 0);
    if (make_displayed) c->pc.displayed_phys = idx;
    return DMX_OK;
}

int dmx_chunk_set_displayed(dmx_chunk* c, int physical_column) {
    if (!c) return fail(DMX_ERR_ARG, "chunk is NULL");
    c->pc.displayed_phys = physical_column;
    return DMX_OK;
}

int dmx_chunk_set_name(dmx_chunk* c, const char* name) {
    if (!c || !name) return fail(DMX_ERR_ARG, "bad arguments");
    c->pc.name = name;
    return DMX_OK;
}

int dmx_chunk_select_cells(dmx_chunk* c, const int32_t* cells, int64_t n) {
    if (!c || (n && !cells)) return fail(DMX_ERR_ARG, "bad arguments");
    ParsedChunk& p = c->pc;
    const int64_t C = (int64_t)p.cols * p.rows;
    if ((int64_t)p.point_off.size() != C + 1) return fail(DMX_ERR_STATE, "chunk has no point records");
    for (int64_t i = 0; i < n; i++) {
        const int64_t cell = cells[i];
        if (cell < 0 || cell >= C) return fail(DMX_ERR_ARG, "cell outside the grid");
        if (!(p.state[cell] & CELL_FILLED)) continue;   // PointMap::setCurSel keeps filled cells only
        int32_t st;
        std::memcpy(&st, &p.points_raw[p.point_off[cell]], 4);
        st |= CELL_SELECTED;
        std::memcpy(&p.points_raw[p.point_off[cell]], &st, 4);
    }
    return DMX_OK;
}

int dmx_chunk_unmake(dmx_chunk* c, int remove_links) {
    if (!c) return fail(DMX_ERR_ARG, "chunk is NULL");
    std::string err;
    if (chunk_unmake(c->pc, remove_links != 0, err)) return fail(DMX_ERR_STATE, err);
    return DMX_OK;
}

int dmx_chunk_serialize(const dmx_chunk* c, uint8_t* buf, int64_t cap, int64_t* size) {
    if (!c || !size) return fail(DMX_ERR_ARG, "bad arguments");
    std::vector<uint8_t> out;
    std::string err;
    if (write_parsed_chunk(c->pc, out, err)) return fail(DMX_ERR_STATE, err);
    *size = (int64_t)out.size();
    if (buf) {
        if (cap < (int64_t)out.size()) return fail(DMX_ERR_ARG, "buffer too small");
        std::memcpy(buf, out.data(), out.size());
    }
    return DMX_OK;
}
