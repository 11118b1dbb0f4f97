// api/stepdepth.hip -- metric / angular / visual step depth.
// Part of the dmx_api.hip unity build: included inside its extern "C" block, after the context and the
// internal types (dmx_ctx, dmx_pointmap, dmx_graph); not compiled on its own.

// ---------------------------------------------------------------- metric step depth
// Batched metric search (stepdepth.hip): key/mdist/cum/lastpix are left in the VGAMetricDepth end
// state.  Returns DMX_OK, a negative status on a HIP error, or 1 when a batch capacity overflowed
// (the caller then re-runs the selection with the serial kernel).
static int stepdepth_batched(dmx_ctx* ctx, dmx_graph* g, const std::vector<uint8_t>& flags,
                             const std::vector<int32_t>& sel, const uint8_t* d_flags, const int32_t* d_sel,
                             unsigned long long* d_key, float* d_mdist, float* d_cum, int32_t* d_last) {
    PointMapHost& h = *g->pm->host;
    const int rows = h.rows();
    const int64_t C = (int64_t)h.cols() * rows;
    hipStream_t s = ctx->stream;
    std::vector<int32_t> ex;
    for (int64_t c = 0; c < C; c++)
        if (flags[(size_t)c] & SDF_EXPAND) ex.push_back((int32_t)c);
    const int64_t E = (int64_t)ex.size();
    // work units: ceil(runs / SDB_UNIT) per expander
    std::vector<int32_t> nr((size_t)g->nnodes);
    HIPCHK(hipStreamSynchronize(s));
    if (g->nnodes) HIPCHK(copy_sync(ctx->stream, nr.data(), g->node_nruns.p, g->nnodes * 4, hipMemcpyDeviceToHost));
    int64_t units = 0;
    const auto& nc = g->pm->node_cell;   // ascending cell index = node order
    for (int32_t c : ex) {
        const size_t node = (size_t)(std::lower_bound(nc.begin(), nc.end(), c) - nc.begin());
        units += (nr[node] + SDB_UNIT - 1) / SDB_UNIT;
    }
    const unsigned amb_cap = 1u << 16, ent_cap = 1u << 22;
    DevBuf<int32_t> d_ex, d_uown, d_win, d_ambid, d_touch, d_amb, d_ahead, d_enext;
    DevBuf<uint8_t> d_done;
    DevBuf<SdbExp> d_bq;
    DevBuf<unsigned long long> d_best;
    DevBuf<unsigned> d_nnear;
    DevBuf<int2> d_ent;
    DevBuf<SdbCtl> d_ctl;
    HIPCHK(d_ex.alloc(std::max<int64_t>(E, 1)));
    HIPCHK(d_done.alloc(std::max<int64_t>(E, 1)));
    HIPCHK(d_bq.alloc(std::max<int64_t>(E, 1)));
    HIPCHK(d_uown.alloc(std::max<int64_t>(units, 1)));
    HIPCHK(d_best.alloc(C));
    HIPCHK(d_nnear.alloc(C));
    HIPCHK(d_win.alloc(C));
    HIPCHK(d_ambid.alloc(C));
    HIPCHK(d_touch.alloc(C));
    HIPCHK(d_amb.alloc(amb_cap));
    HIPCHK(d_ent.alloc(ent_cap));
    HIPCHK(d_ahead.alloc(amb_cap));
    HIPCHK(d_enext.alloc(ent_cap));
    HIPCHK(hipMemsetAsync(d_ahead.p, 0xFF, (size_t)amb_cap * 4, s));
    HIPCHK(d_ctl.alloc(1));
    if (E) HIPCHK(hipMemcpyAsync(d_ex.p, ex.data(), E * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(d_done.p, 0, std::max<int64_t>(E, 1), s));
    HIPCHK(hipMemsetAsync(d_best.p, 0xFF, C * 8, s));
    HIPCHK(hipMemsetAsync(d_nnear.p, 0, C * 4, s));
    HIPCHK(hipMemsetAsync(d_ambid.p, 0xFF, C * 4, s));
    HIPCHK(hipMemsetAsync(d_key, 0xFF, C * 8, s));
    std::vector<float> m1((size_t)C, -1.0f);
    HIPCHK(hipMemcpyAsync(d_mdist, m1.data(), C * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(d_cum, 0, C * 4, s));
    HIPCHK(hipMemsetAsync(d_last, 0xFF, C * 4, s));
    SdbCtl c0;
    memset(&c0, 0, sizeof(c0));
    c0.gcur = 0ull;            // the selected cells' distance 0
    c0.gnext = SD_INF;
    HIPCHK(hipMemcpyAsync(d_ctl.p, &c0, sizeof(c0), hipMemcpyHostToDevice, s));
    SdbParams P;
    P.rows = rows; P.E = E; P.flags = d_flags; P.cell_node = g->pm->d_cell_node.p;
    P.node_run_start = g->node_run_start.p; P.node_nruns = g->node_nruns.p; P.pool = g->pool.p;
    P.key = d_key; P.mdist = d_mdist; P.cum = d_cum; P.lastpix = d_last;
    P.ex_cells = d_ex.p; P.ex_done = d_done.p; P.bq = d_bq.p; P.uown = d_uown.p;
    P.best = d_best.p; P.nnear = d_nnear.p; P.win = d_win.p; P.ambid = d_ambid.p; P.touch = d_touch.p;
    P.amb = d_amb.p; P.ent = d_ent.p; P.ahead = d_ahead.p; P.enext = d_enext.p; P.ent_cap = ent_cap; P.amb_cap = amb_cap; P.ctl = d_ctl.p;
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipEventRecord(ctx->ev0, s));
    hipLaunchKernelGGL(sdb_init_kernel, dim3((unsigned)((sel.size() + 255) / 256)), dim3(256), 0, s, P, d_sel,
                       (int)sel.size());
    HIPCHK(hipGetLastError());
    const unsigned gs = (unsigned)std::max<int64_t>(1, (E + 255) / 256);
    const unsigned gr = (unsigned)std::max(64, ctx->num_cu * 4);
    SdbCtl hc;
    // Batches advance the smallest live distance by >= 1 - 2^-18; the number of batches is bounded
    // by the longest path length, itself < C grid units.
    const int64_t max_it = 2 * C + 64;
    int64_t it = 0;
    for (;;) {
        for (int k = 0; k < 32; k++, it++) {
            hipLaunchKernelGGL(sdb_select_kernel, dim3(gs), dim3(256), 0, s, P);
            hipLaunchKernelGGL(sdb_relax_kernel<1>, dim3(gr), dim3(SDB_THREADS), 0, s, P);
            hipLaunchKernelGGL(sdb_relax_kernel<2>, dim3(gr), dim3(SDB_THREADS), 0, s, P);
            hipLaunchKernelGGL(sdb_apply_kernel, dim3(gr), dim3(256), 0, s, P);
            hipLaunchKernelGGL(sdb_relax_kernel<3>, dim3(gr), dim3(SDB_THREADS), 0, s, P);
            hipLaunchKernelGGL(sdb_fold_kernel, dim3(256), dim3(SDB_THREADS), 0, s, P);
            hipLaunchKernelGGL(sdb_finish_kernel, dim3(1), dim3(1), 0, s, P);
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(&hc, d_ctl.p, sizeof(hc), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (hc.done) break;
        CANCEL_POINT(ctx);
        if (it > max_it) return fail(DMX_ERR_STATE, "batched step depth did not terminate");
    }
    HIPCHK(hipEventRecord(ctx->ev1, s));
    HIPCHK(hipEventSynchronize(ctx->ev1));
    if (hc.error) return 1;
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last_sd_s = ms * 1e-3;
    ctx->last_sd_stats[0] = (long long)hc.popped;
    ctx->last_sd_stats[1] = (long long)hc.relaxed;
    ctx->last_sd_stats[2] = (long long)hc.batches;
    ctx->last_sd_extra[0] = (long long)hc.improved;
    ctx->last_sd_extra[1] = (long long)hc.ambiguous;
    return DMX_OK;
}

// STEPDEPTH -sdt metric (VGAMetricDepth) or, with ANG, -sdt angular (VGAAngularDepth): one search
// from the selection; out [N][3] (metric) or [N] (angular).
extern "C++" template <bool ANG>
static int stepdepth_impl(dmx_ctx* ctx, dmx_graph* g, const int32_t* sel_cells, int64_t nsel, float* out) {
    if (!ctx || !g || !out || (nsel > 0 && !sel_cells)) return fail(DMX_ERR_ARG, "bad arguments");
    if (g->node_begin != 0 || g->node_end != g->nnodes)
        return fail(DMX_ERR_STATE, "step depth needs the whole graph (assemble the shards first)");
    HIPCHK(hipSetDevice(ctx->device));
    CANCEL_POINT(ctx);   // a cancel requested while nothing ran stops this call (dmx.h)
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int64_t C = (int64_t)cols * rows, N = g->nnodes;
    const auto& st = h.state();
    // selection: filled cells only, std::set<int> PixelRef order, no duplicates
    std::vector<int32_t> sel;
    for (int64_t i = 0; i < nsel; i++) {
        const int32_t c = sel_cells[i];
        if (c < 0 || c >= C) return fail(DMX_ERR_ARG, "selected cell outside the grid");
        if (st[c] & CELL_FILLED) sel.push_back(c);
    }
    std::sort(sel.begin(), sel.end(), [&](int32_t a, int32_t b) {
        return ((a / rows) << 16) + (a % rows) < ((b / rows) << 16) + (b % rows);
    });
    sel.erase(std::unique(sel.begin(), sel.end()), sel.end());
    if (sel.empty()) return fail(DMX_ERR_STATE, "no filled cell selected");
    // expanders: selected, BLOCKED or next to a BLOCKED cell (ngraph.cpp:67-76, pointdata.cpp:1016-1068)
    std::vector<uint8_t> flags((size_t)C, 0);
    int64_t nexp = 0;
    for (int x = 0; x < cols; x++)
        for (int y = 0; y < rows; y++) {
            const int64_t c = h.index(x, y);
            if (!(st[c] & CELL_FILLED)) continue;
            uint8_t f = SDF_FILLED;
            bool ex = (st[c] & CELL_BLOCKED) != 0;
            for (int dx = -1; dx <= 1 && !ex; dx++)
                for (int dy = -1; dy <= 1 && !ex; dy++)
                    if ((dx || dy) && h.includes(x + dx, y + dy) && (st[h.index(x + dx, y + dy)] & CELL_BLOCKED)) ex = true;
            if (ex) { f |= SDF_EXPAND; nexp++; }
            flags[c] = f;
        }
    for (int32_t c : sel) flags[c] |= SDF_EXPAND;
    for (size_t i = 0; i < g->merges.size(); i++) { flags[g->merges[i]] |= SDF_MERGE; nexp++; }
    hipStream_t s = ctx->stream;
    DevBuf<uint8_t> d_flags;
    DevBuf<unsigned long long> d_key, d_over;
    DevBuf<float> d_mdist, d_cum, d_out;
    DevBuf<int32_t> d_last, d_sel;
    HIPCHK(d_flags.alloc(C));
    HIPCHK(d_key.alloc(C));
    HIPCHK(d_mdist.alloc(C));
    HIPCHK(d_cum.alloc(C));
    HIPCHK(d_last.alloc(C));
    HIPCHK(d_sel.alloc(sel.size()));
    HIPCHK(d_out.alloc(std::max<int64_t>(N, 1) * 3));
    HIPCHK(hipMemcpyAsync(d_flags.p, flags.data(), C, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_sel.p, sel.data(), sel.size() * 4, hipMemcpyHostToDevice, s));
    int64_t cap = 8 * (nexp + (int64_t)sel.size()) + SD_WIN + 1024 + (ANG ? 8 * N : 0);
    // metric: the batched search over the whole GPU (stepdepth.hip, "batched metric step depth");
    // DMX_SD_KERNEL=serial forces the one-workgroup kernel, which is also the fallback
    // (merge links: the serial kernel, which extracts a partner at its link's pop)
    bool batched = !ANG && g->merges.empty();
    if (const char* e = getenv("DMX_SD_KERNEL")) batched = batched && strcmp(e, "serial") != 0;
    ctx->last_sd_mode = 0;
    if (batched) {
        int rc = stepdepth_batched(ctx, g, flags, sel, d_flags.p, d_sel.p, d_key.p, d_mdist.p, d_cum.p, d_last.p);
        if (rc < 0) return rc;
        if (rc == DMX_OK) {
            const int single = sel.size() == 1 ? 1 : 0;
            if (N) {
                hipLaunchKernelGGL(stepdepth_out_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, rows,
                                   h.spacing(), g->pm->d_node_cell.p, N, d_key.p, d_cum.p, single, sel[0] / rows,
                                   sel[0] % rows, d_out.p);
                HIPCHK(hipGetLastError());
                HIPCHK(hipMemcpyAsync(out, d_out.p, N * 3 * 4, hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
            }
            ctx->last_sd_mode = 1;
            return DMX_OK;
        }
        // rc > 0: a batch capacity overflowed; the serial search below redoes the whole selection
        ctx->last_sd_mode = 2;
    }
    for (int attempt = 0; attempt < 4; attempt++) {
        HIPCHK(d_over.alloc(cap));
        HIPCHK(hipMemsetAsync(d_key.p, 0xFF, C * 8, s));
        std::vector<float> m1((size_t)C, -1.0f);
        HIPCHK(hipMemcpyAsync(d_mdist.p, m1.data(), C * 4, hipMemcpyHostToDevice, s));
        if (ANG) HIPCHK(hipMemcpyAsync(d_cum.p, m1.data(), C * 4, hipMemcpyHostToDevice, s));
        else HIPCHK(hipMemsetAsync(d_cum.p, 0, C * 4, s));
        HIPCHK(hipMemsetAsync(d_last.p, 0xFF, C * 4, s));
        HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 16 * sizeof(int), s));
        HIPCHK(hipMemsetAsync(ctx->stats.p, 0, 32 * sizeof(unsigned long long), s));
        StepDepthParams P;
        P.cols = cols; P.rows = rows; P.flags = d_flags.p; P.cell_node = g->pm->d_cell_node.p;
        P.node_run_start = g->node_run_start.p; P.node_nruns = g->node_nruns.p; P.pool = g->pool.p;
        P.key = d_key.p; P.mdist = d_mdist.p; P.cum = d_cum.p; P.lastpix = d_last.p;
        P.over = d_over.p; P.over_cap = cap; P.error = ctx->counters.p + 1; P.stats = ctx->stats.p;
        P.merge = g->merges.empty() ? nullptr : g->d_merge_cell.p;
        HIPCHK(hipEventRecord(ctx->ev0, s));
        hipLaunchKernelGGL(stepdepth_kernel<ANG>, dim3(1), dim3(SD_THREADS), 0, s, P, d_sel.p, (int)sel.size());
        HIPCHK(hipGetLastError());
        const int single = sel.size() == 1 ? 1 : 0;
        if (!ANG) {
            hipLaunchKernelGGL(stepdepth_out_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, rows,
                               h.spacing(), g->pm->d_node_cell.p, N, d_key.p, d_cum.p, single, sel[0] / rows,
                               sel[0] % rows, d_out.p);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipEventRecord(ctx->ev1, s));
        HIPCHK(hipStreamSynchronize(s));
        int hc[2];
        HIPCHK(copy_sync(ctx->stream, hc, ctx->counters.p, sizeof(hc), hipMemcpyDeviceToHost));
        if (hc[1] & KERR_FRONTIER) { cap *= 4; continue; }
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        ctx->last_sd_s = ms * 1e-3;
        unsigned long long st3[3];
        HIPCHK(copy_sync(ctx->stream, st3, ctx->stats.p, sizeof(st3), hipMemcpyDeviceToHost));
        for (int i = 0; i < 3; i++) ctx->last_sd_stats[i] = (long long)st3[i];
        if (ANG) {
            // "Angular Step Depth" = m_cumangle of every cell the search resolved (vgaangulardepth.cpp:53-55)
            std::vector<unsigned long long> kh((size_t)C);
            std::vector<float> ch((size_t)C);
            HIPCHK(copy_sync(ctx->stream, kh.data(), d_key.p, C * 8, hipMemcpyDeviceToHost));
            HIPCHK(copy_sync(ctx->stream, ch.data(), d_cum.p, C * 4, hipMemcpyDeviceToHost));
            for (int64_t k = 0; k < N; k++) {
                const int c = g->pm->node_cell[k];
                out[k] = kh[c] != SD_INF ? ch[c] : -1.0f;
            }
        } else if (N) {
            HIPCHK(copy_sync(ctx->stream, out, d_out.p, N * 3 * 4, hipMemcpyDeviceToHost));
        }
        return DMX_OK;
    }
    return fail(DMX_ERR_CAPACITY, "step depth queue overflow after retries");
}

int dmx_metric_stepdepth(dmx_ctx* ctx, dmx_graph* g, const int32_t* sel_cells, int64_t nsel, float* out) {
    SAME_DEVICE(ctx, g);
    release_sym_scatter(g);
    if (int rc = prepare_merges(g)) return rc;
    return stepdepth_impl<false>(ctx, g, sel_cells, nsel, out);
}

int dmx_angular_stepdepth(dmx_ctx* ctx, dmx_graph* g, const int32_t* sel_cells, int64_t nsel, float* out) {
    SAME_DEVICE(ctx, g);
    release_sym_scatter(g);
    if (int rc = prepare_merges(g)) return rc;
    return stepdepth_impl<true>(ctx, g, sel_cells, nsel, out);
}

// The nodes the symmetry pass found asymmetric (their in-set differs from their run-length out-set; the
// BFS kernels route them through exact Extra / Missing lists).  Runs the VGA preparation if needed.
int dmx_graph_special_nodes(dmx_graph* g, int32_t* nodes, int64_t* n) {
    if (!g || !n) return fail(DMX_ERR_ARG, "bad arguments");
    if (g->node_begin != 0 || g->node_end != g->nnodes) return fail(DMX_ERR_STATE, "needs the whole graph");
    HIPCHK(hipSetDevice(g->ctx->device));
    if (int rc = prepare_uf(g)) return rc;
    if (int rc = prepare_symmetry(g)) return rc;
    const int64_t m = (int64_t)g->special_nodes.size();
    if (nodes) {
        if (*n < m) return fail(DMX_ERR_ARG, "buffer too small");
        std::memcpy(nodes, g->special_nodes.data(), (size_t)m * 4);
    }
    *n = m;
    return DMX_OK;
}

int dmx_ctx_last_mk_reruns(dmx_ctx* ctx, int64_t* nodes, int64_t cap, int64_t* n) {
    if (!ctx || !n || cap < 0 || (cap > 0 && !nodes)) return fail(DMX_ERR_ARG, "bad arguments");
    *n = (int64_t)ctx->last_mk_reruns.size();
    for (int64_t i = 0; i < *n && i < cap; i++) nodes[i] = ctx->last_mk_reruns[(size_t)i];
    return DMX_OK;
}

int dmx_ctx_last_phase_cycles(dmx_ctx* ctx, int64_t* out5) {
    if (!ctx || !out5) return fail(DMX_ERR_ARG, "bad arguments");
    for (int i = 0; i < 5; i++) out5[i] = ctx->phase_cycles[i];
    return DMX_OK;
}

// STEPDEPTH -sdt visual: MetaGraph::analyseGraph(point_depth_selection = 1) -> VGAVisualGlobalDepth::run
// (depthmapXcli/runmethods.cpp:767-769, salalib/vgamodules/vgavisualglobaldepth.cpp:23-77).  One
// breadth-first search from every selected filled cell at once (level 0, always expanded); cells are
// discovered through run membership (Bin::extractUnseen, ngraph.cpp:308-326: set semantics, the
// extent short-cut only skips already-covered suffixes); contextfilled odd cells get their level but
// are not expanded.  Runs on the tile-resolved BFS in seed mode (one workgroup).
// Visual step depth for grids above 1024^2 or asymmetric graphs: the level-synchronous top-down
// search of kernels/vstep.hip over the whole GPU.
static int visual_stepdepth_topdown(dmx_ctx* ctx, dmx_graph* g, const std::vector<int32_t>& seeds, int tw, int th,
                                    float* out, const std::vector<int32_t>& sel_cells) {
    PointMapHost& h = *g->pm->host;
    const int rows = h.rows();
    const int64_t C = h.cells(), N = g->nnodes, nt = (int64_t)tw * th;
    hipStream_t s = ctx->stream;
    DevBuf<unsigned long long> vis, cnt;
    DevBuf<int32_t> level, fr[2], pend[2];
    DevBuf<int> err;
    HIPCHK(vis.alloc(nt));
    HIPCHK(cnt.alloc(2));   // next frontier, pending extractions
    HIPCHK(err.alloc(1));
    HIPCHK(hipMemsetAsync(err.p, 0, sizeof(int), ctx->stream));
    const int nmp = (int)(g->merges.size() / 2);
    if (g->nmamb) {
        HIPCHK(pend[0].alloc(g->nmamb));
        HIPCHK(pend[1].alloc(g->nmamb));
    }
    HIPCHK(level.alloc(C));
    HIPCHK(fr[0].alloc(std::max<int64_t>(N, 1)));
    HIPCHK(fr[1].alloc(std::max<int64_t>(N, 1)));
    std::vector<unsigned long long> v0((size_t)nt, 0ull);
    std::vector<int32_t> lv((size_t)C, -1);
    for (int32_t k : seeds) {
        const int c = g->pm->node_cell[k], x = c / rows, y = c % rows;
        v0[(size_t)(y >> 3) * tw + (x >> 3)] |= 1ull << ((y & 7) * 8 + (x & 7));
        lv[c] = 0;
    }
    HIPCHK(hipMemcpyAsync(vis.p, v0.data(), nt * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(level.p, lv.data(), C * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(fr[0].p, seeds.data(), seeds.size() * 4, hipMemcpyHostToDevice, s));
    HIPCHK(hipEventRecord(ctx->ev0, s));
    int64_t nf = (int64_t)seeds.size(), npend = 0;
    int cur = 0, L = 0;
    while (nf > 0) {
        HIPCHK(hipMemsetAsync(cnt.p, 0, 16, s));
        const int64_t blocks = std::min<int64_t>((nf + 3) / 4, (int64_t)ctx->num_cu * 16);
        hipLaunchKernelGGL(vsd_level_kernel, dim3((unsigned)blocks), dim3(VSD_THREADS), 0, s, rows, tw,
                           (const int32_t*)fr[cur].p, nf, g->node_run_start.p, g->node_nruns.p, g->pool.p,
                           g->pm->d_cell_node.p, g->pm->d_node_flags.p, L + 1, vis.p, level.p, fr[cur ^ 1].p, cnt.p);
        HIPCHK(hipGetLastError());
        if (nmp) {
            hipLaunchKernelGGL(vsd_merge_kernel, dim3((unsigned)((nmp + 255) / 256)), dim3(256), 0, s, rows, tw,
                               (const int2*)g->d_mpairs.p, nmp, g->pm->d_cell_node.p, g->pm->d_node_flags.p, L + 1,
                               vis.p, level.p, fr[cur ^ 1].p, cnt.p, pend[cur ^ 1].p, cnt.p + 1);
            HIPCHK(hipGetLastError());
        }
        if (npend) {   // the previous level's pending extractions, now that this level is complete
            hipLaunchKernelGGL(vsd_pending_kernel, dim3((unsigned)((npend + 3) / 4)), dim3(VSD_THREADS), 0, s, rows, tw,
                               (const int32_t*)pend[cur].p, npend, g->node_run_start.p, g->node_nruns.p, g->pool.p,
                               g->pm->d_cell_node.p, (const unsigned long long*)vis.p, err.p);
            HIPCHK(hipGetLastError());
        }
        unsigned long long n_next[2] = {0, 0};
        HIPCHK(copy_sync(s, n_next, cnt.p, 16, hipMemcpyDeviceToHost));
        cur ^= 1;
        nf = (int64_t)n_next[0];
        npend = (int64_t)n_next[1];
        L++;
    }
    int herr = 0;
    HIPCHK(copy_sync(s, &herr, err.p, sizeof(int), hipMemcpyDeviceToHost));
    HIPCHK(hipEventRecord(ctx->ev1, s));
    if (herr & KERR_ORDER) {
        // an unexpanded link end whose extraction depends on the pop order reached an unseen cell: the whole
        // search in the reference's order (vga_ordered.hip), from the selection in PixelRef order
        HIPCHK(hipMemsetAsync(level.p, 0xFF, C * 4, s));
        if (int rc = ordered_search(ctx, g, -1.0, {}, sel_cells, nullptr, nullptr, level.p)) return rc;
        HIPCHK(hipEventRecord(ctx->ev1, s));
        ctx->last_stats[38] = 1;
    } else {
        ctx->last_stats[38] = 0;
    }
    HIPCHK(copy_sync(s, lv.data(), level.p, C * 4, hipMemcpyDeviceToHost));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last_vga_s = ms * 1e-3;
    for (int64_t k = 0; k < N; k++) {
        const int v = lv[g->pm->node_cell[k]];
        out[k] = v >= 0 ? (float)v : -1.0f;
    }
    VLOG("visual step depth: top-down, %d levels, %.3f s\n", L, ms * 1e-3);
    return DMX_OK;
}

int dmx_visual_stepdepth(dmx_ctx* ctx, dmx_graph* g, const int32_t* sel_cells, int64_t nsel, float* out) {
    SAME_DEVICE(ctx, g);
    if (!ctx || !g || !out || (nsel > 0 && !sel_cells)) return fail(DMX_ERR_ARG, "bad arguments");
    if (int rc = prepare_merges(g)) return rc;
    if (g->node_begin != 0 || g->node_end != g->nnodes)
        return fail(DMX_ERR_STATE, "step depth needs the whole graph (assemble the shards first)");
    HIPCHK(hipSetDevice(ctx->device));
    CANCEL_POINT(ctx);   // (before any output is written)
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int64_t C = (int64_t)cols * rows, N = g->nnodes;
    for (int64_t k = 0; k < N; k++) out[k] = -1.0f;
    ctx->last_stats[38] = 0;
    const auto& st = h.state();
    std::vector<int32_t> seeds;   // nodes, selection order = std::set<int> PixelRef order, unique
    std::vector<int32_t> sel;     // the selected filled cells in that order
    {
        for (int64_t i = 0; i < nsel; i++) {
            const int32_t c = sel_cells[i];
            if (c < 0 || c >= C) return fail(DMX_ERR_ARG, "selected cell outside the grid");
            if (st[c] & CELL_FILLED) sel.push_back(c);
        }
        std::sort(sel.begin(), sel.end());
        sel.erase(std::unique(sel.begin(), sel.end()), sel.end());
        const auto& nc = g->pm->node_cell;   // ascending x-major cell index = node order
        for (int32_t c : sel) {
            const auto it = std::lower_bound(nc.begin(), nc.end(), c);
            if (it != nc.end() && *it == c) seeds.push_back((int32_t)(it - nc.begin()));
        }
    }
    if (seeds.empty()) return fail(DMX_ERR_STATE, "no filled cell selected");
    // a selected cell's merge pixel takes level 0 and is extracted with it (vgavisualglobaldepth.cpp:55-63)
    if (!g->merges.empty()) {
        const auto& nc = g->pm->node_cell;
        std::vector<int32_t> add;
        for (size_t i = 0; i < g->merges.size(); i += 2) {
            const int32_t a = g->merges[i], b = g->merges[i + 1];
            const int32_t na = (int32_t)(std::lower_bound(nc.begin(), nc.end(), a) - nc.begin());
            const int32_t nb = (int32_t)(std::lower_bound(nc.begin(), nc.end(), b) - nc.begin());
            const bool sa = std::binary_search(seeds.begin(), seeds.end(), na);
            const bool sb = std::binary_search(seeds.begin(), seeds.end(), nb);
            if (sa && !sb) add.push_back(nb);
            if (sb && !sa) add.push_back(na);
        }
        seeds.insert(seeds.end(), add.begin(), add.end());
        std::sort(seeds.begin() + 1, seeds.end());   // seeds[0] stays the first selected cell
    }
    const int tw = (cols + 7) / 8, th = (rows + 7) / 8, nt = tw * th;
    // links with a context-filled odd end need the top-down search's pending-extraction check
    bool tile = nt <= 16 * 1024 && !getenv("DMX_VSD_TOPDOWN") && g->nmamb == 0;
    int rc = DMX_OK;
    if (tile) {
        rc = prepare_uf(g);
        if (rc) return rc;
        rc = prepare_symmetry(g);
        if (rc) return rc;
        tile = g->symmetric == 1;
    }
    if (!tile) return visual_stepdepth_topdown(ctx, g, seeds, tw, th, out, sel);
    DevBuf<int32_t> d_seeds, d_level;
    HIPCHK(d_seeds.alloc(seeds.size()));
    HIPCHK(d_level.alloc((size_t)nt * 64));
    HIPCHK(hipMemcpyAsync(d_seeds.p, seeds.data(), seeds.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemsetAsync(d_level.p, 0xFF, (size_t)nt * 64 * 4, ctx->stream));
    std::vector<float> dummy(7);
    rc = vga_tile_impl(ctx, g, -1.0, 0, 0, 1, dummy.data(), false, nullptr, tw, th, d_seeds.p, (int)seeds.size(), d_level.p);
    if (rc == DMX_ERR_CAPACITY) return visual_stepdepth_topdown(ctx, g, seeds, tw, th, out, sel);
    if (rc) return rc;
    std::vector<int32_t> lv((size_t)nt * 64);
    HIPCHK(copy_sync(ctx->stream, lv.data(), d_level.p, lv.size() * 4, hipMemcpyDeviceToHost));
    for (int64_t k = 0; k < N; k++) {
        const int c = g->pm->node_cell[k];
        const int x = c / rows, y = c % rows;
        const int v = lv[(size_t)((((y >> 3) * tw + (x >> 3)) << 6) | ((y & 7) << 3) | (x & 7))];
        if (v >= 0) out[k] = (float)v;
    }
    for (int32_t k : seeds) out[k] = 0.0f;
    return DMX_OK;
}

int dmx_ctx_last_stepdepth(dmx_ctx* ctx, double* seconds, int64_t* expanders_popped, int64_t* cells_relaxed) {
    if (!ctx) return fail(DMX_ERR_ARG, "ctx is NULL");
    if (seconds) *seconds = ctx->last_sd_s;
    if (expanders_popped) *expanders_popped = ctx->last_sd_stats[0];
    if (cells_relaxed) *cells_relaxed = ctx->last_sd_stats[1];
    return DMX_OK;
}

int dmx_ctx_last_stepdepth_detail(dmx_ctx* ctx, int64_t* out4) {
    if (!ctx || !out4) return fail(DMX_ERR_ARG, "bad arguments");
    out4[0] = ctx->last_sd_mode;
    out4[1] = ctx->last_sd_stats[2];
    out4[2] = ctx->last_sd_extra[0];
    out4[3] = ctx->last_sd_extra[1];
    return DMX_OK;
}
