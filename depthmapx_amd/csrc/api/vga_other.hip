// api/vga_other.hip -- VGA metric / angular (all sources), VGA visual local, the preparation shard.
// Part of the dmx_api.hip unity build: included inside its extern "C" block, after the context and the
// internal types (dmx_ctx, dmx_pointmap, dmx_graph); not compiled on its own.

// ---------------------------------------------------------------- VGA metric (all sources)
// VGAMetric::run / VGAAngular::run for every source: one search per workgroup (stepdepth.hip).
extern "C++" template <bool ANG>
static int vga_search_all(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se, float* out) {
    constexpr int NO = ANG ? 3 : 4;
    if (!ctx || !g || !out) return fail(DMX_ERR_ARG, "bad arguments");
    if (g->node_begin != 0 || g->node_end != g->nnodes)
        return fail(DMX_ERR_STATE, "VGA needs the whole graph (assemble the shards first)");
    HIPCHK(hipSetDevice(ctx->device));
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int64_t C = (int64_t)cols * rows, N = g->nnodes;
    if (se < 0 || se > N) se = N;
    if (sb < 0 || sb > se) return fail(DMX_ERR_ARG, "source range out of bounds");
    const auto& st = h.state();
    // expanders: BLOCKED or next to a BLOCKED cell (ngraph.cpp:67-76, pointdata.cpp:1016-1068); the
    // source expands at distance 0 whatever its flags
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
    for (size_t i = 0; i < g->merges.size(); i++) { flags[g->merges[i]] |= SDF_MERGE; nexp++; }
    hipStream_t s = ctx->stream;
    int occ = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vga_metric_kernel<ANG>, SD_THREADS, 0));
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(se - sb, (int64_t)ctx->num_cu * std::max(occ, 1)));
    DevBuf<uint8_t> d_flags;
    DevBuf<unsigned long long> d_key, d_over, d_comp, d_srt;
    DevBuf<float> d_mdist, d_cum, d_out;
    DevBuf<int32_t> d_last;
    HIPCHK(d_flags.alloc(C));
    HIPCHK(d_key.alloc((size_t)nb * C));
    HIPCHK(d_mdist.alloc((size_t)nb * C));
    HIPCHK(d_cum.alloc((size_t)nb * C));
    HIPCHK(d_last.alloc((size_t)nb * C));
    HIPCHK(d_comp.alloc((size_t)nb * 2 * std::max<int64_t>(N, 1)));
    HIPCHK(d_srt.alloc((size_t)nb * std::max<int64_t>(N, 1)));
    HIPCHK(d_out.alloc((size_t)std::max<int64_t>(N, 1) * NO));
    HIPCHK(hipMemcpyAsync(d_flags.p, flags.data(), C, hipMemcpyHostToDevice, s));
    // Per-workgroup overflow list.  A source whose search outgrows it stops, is listed, and only the
    // listed sources run again with a 4x list on fewer workgroups (bounded by free device memory).
    int64_t cap = 8 * (nexp + 1) + SD_WIN + 1024;
    if (ANG) cap += 32 * N;   // cells reached at angle 0 are queued too (and re-queued on improvement)
    if (const char* e = getenv("DMX_SD_CAP")) cap = std::max<int64_t>(64, atoll(e));   // test hook: retries
    DevBuf<int64_t> d_list[2];
    DevBuf<int> d_nfail;
    HIPCHK(d_list[0].alloc(std::max<int64_t>(se - sb, 1)));
    HIPCHK(d_list[1].alloc(std::max<int64_t>(se - sb, 1)));
    HIPCHK(d_nfail.alloc(1));
    HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 16 * sizeof(int), s));
    HIPCHK(hipMemsetAsync(ctx->stats.p, 0, 32 * sizeof(unsigned long long), s));
    double kernel_s = 0.0;
    int64_t todo = se - sb, rerun = 0;
    const int64_t* list = nullptr;   // first pass: the range; then the failed sources
    int cur = 0;
    for (int attempt = 0; todo > 0; attempt++) {
        const int64_t nbl = std::max<int64_t>(1, std::min<int64_t>(nb, todo));
        size_t free_b = 0, total_b = 0;
        HIPCHK(hipMemGetInfo(&free_b, &total_b));
        free_b += cached_bytes() + d_over.n * sizeof(unsigned long long);
        const int64_t cap_max = (int64_t)(free_b * 0.8 / 8.0 / (double)nbl);
        if (attempt > 0 && cap > cap_max) return fail(DMX_ERR_CAPACITY, "VGA metric/angular: search queue exceeds device memory");
        if (attempt >= 10) return fail(DMX_ERR_CAPACITY, "VGA metric/angular: queue overflow after retries");
        d_over.reset();
        HIPCHK(d_over.alloc((size_t)nbl * std::min(cap, std::max<int64_t>(cap_max, 1))));
        const int64_t cap_used = std::min(cap, std::max<int64_t>(cap_max, 1));
        HIPCHK(hipMemsetAsync(d_nfail.p, 0, sizeof(int), s));
        StepDepthParams P;
        P.cols = cols; P.rows = rows; P.flags = d_flags.p; P.cell_node = g->pm->d_cell_node.p;
        P.node_run_start = g->node_run_start.p; P.node_nruns = g->node_nruns.p; P.pool = g->pool.p;
        P.key = d_key.p; P.mdist = d_mdist.p; P.cum = d_cum.p; P.lastpix = d_last.p;
        P.over = d_over.p; P.over_cap = cap_used; P.error = ctx->counters.p + 1; P.stats = ctx->stats.p;
        P.merge = g->merges.empty() ? nullptr : g->d_merge_cell.p;
        HIPCHK(hipEventRecord(ctx->ev0, s));
        hipLaunchKernelGGL(vga_metric_kernel<ANG>, dim3((unsigned)nbl), dim3(SD_THREADS), 0, s, P, C, g->pm->d_node_cell.p,
                           list ? 0 : sb, list ? todo : se, gates_only, h.spacing(), radius < 0 ? -1.0 : radius, d_comp.p,
                           d_srt.p, std::max<int64_t>(N, 1), d_out.p, list, d_list[cur].p, d_nfail.p);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ctx->ev1, s));
        HIPCHK(hipStreamSynchronize(s));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        kernel_s += ms * 1e-3;
        int hc[2], nfail = 0;
        HIPCHK(copy_sync(ctx->stream, hc, ctx->counters.p, sizeof(hc), hipMemcpyDeviceToHost));
        HIPCHK(copy_sync(ctx->stream, &nfail, d_nfail.p, sizeof(int), hipMemcpyDeviceToHost));
        if (hc[1] & ~KERR_FRONTIER) return fail(DMX_ERR_CAPACITY, "VGA metric/angular search failed");
        VLOG("vga %s: attempt %d, %lld sources, list %lld per workgroup x %lld: %.3f s, %d to re-run\n",
             ANG ? "angular" : "metric", attempt, (long long)todo, (long long)cap_used, (long long)nbl, ms * 1e-3, nfail);
        if (nfail > 0 && cap_used < cap) return fail(DMX_ERR_CAPACITY, "VGA metric/angular: search queue exceeds device memory");
        HIPCHK(hipMemsetAsync(ctx->counters.p + 1, 0, sizeof(int), s));
        rerun += nfail;
        todo = nfail;
        list = d_list[cur].p;
        cur ^= 1;
        cap *= 4;
    }
    ctx->last_vga_s = kernel_s;   // every attempt counted
    if (se > sb)
        HIPCHK(copy_sync(ctx->stream, out + sb * NO, d_out.p + sb * NO, (size_t)(se - sb) * NO * 4, hipMemcpyDeviceToHost));
    unsigned long long stv[3];
    HIPCHK(copy_sync(ctx->stream, stv, ctx->stats.p, sizeof(stv), hipMemcpyDeviceToHost));
    ctx->last_sd_stats[0] = (long long)stv[0];
    ctx->last_sd_stats[1] = (long long)stv[1];
    ctx->last_stats[7] = se - sb;
    ctx->last_stats[8] = rerun;   // sources re-run with a larger overflow list
    return DMX_OK;
}

// The symmetry scatter a whole-graph makeGraph did as it published (sym_diff 4*C*8 B, sym_ho N*8 B: ~160 MB at
// 2000^2) serves only the VGA BFS's preparation.  The analyses that do not use it release it; a VGA call after
// them runs the separate scatter pass instead (prepare_symmetry).
static void release_sym_scatter(dmx_graph* g) {
    if (g && g->sym_fused && !g->scan_ready) {
        g->sym_diff.reset();
        g->sym_ho.reset();
        g->sym_fused = false;
    }
}

int dmx_vga_metric(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se, float* out) {
    SAME_DEVICE(ctx, g);
    release_sym_scatter(g);
    if (int rc = prepare_merges(g)) return rc;
    return vga_search_all<false>(ctx, g, radius, gates_only, sb, se, out);
}

int dmx_vga_angular(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se, float* out) {
    SAME_DEVICE(ctx, g);
    release_sym_scatter(g);
    if (int rc = prepare_merges(g)) return rc;
    return vga_search_all<true>(ctx, g, radius, gates_only, sb, se, out);
}

// ---------------------------------------------------------------- VGA visual local
int dmx_vga_local(dmx_ctx* ctx, dmx_graph* g, int gates_only, int64_t sb, int64_t se, float* out) {
    SAME_DEVICE(ctx, g);
    release_sym_scatter(g);
    if (!ctx || !g || !out) return fail(DMX_ERR_ARG, "bad arguments");
    if (g->node_begin != 0 || g->node_end != g->nnodes)
        return fail(DMX_ERR_STATE, "VGA needs the whole graph (assemble the shards first)");
    HIPCHK(hipSetDevice(ctx->device));
    const int64_t N = g->nnodes;
    if (se < 0 || se > N) se = N;
    if (sb < 0 || sb > se) return fail(DMX_ERR_ARG, "source range out of bounds");
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int tw = (cols + 7) / 8, th = (rows + 7) / 8, nt = tw * th;
    const size_t bm_bytes = (size_t)2 * nt * 8;
    const bool gbm = bm_bytes > policy::kLdsPassBudget || getenv("DMX_VL_GBM");   // the env forces the HBM variant (tests)
    const size_t lds = gbm ? 0 : bm_bytes;
    hipStream_t s = ctx->stream;
    DevBuf<int32_t> nsz;
    DevBuf<float> d_out;
    DevBuf<unsigned long long> d_bm;
    HIPCHK(nsz.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(d_out.alloc((size_t)std::max<int64_t>(N, 1) * 3));
    HIPCHK(hipMemsetAsync(ctx->stats.p, 0, 32 * 8, s));
    HIPCHK(hipEventRecord(ctx->ev0, s));
    if (se > sb) {
        hipLaunchKernelGGL(node_size_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, s, N, g->node_run_start.p,
                           g->node_nruns.p, g->pool.p, nsz.p);
        HIPCHK(hipGetLastError());
        int occ = 0;
        auto kern = gbm ? vga_local_kernel<true> : vga_local_kernel<false>;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, VL_THREADS, lds));
        int64_t nb = std::min<int64_t>(se - sb, (int64_t)ctx->num_cu * std::max(occ, 1));
        if (gbm) {
            // bitmap slices within a quarter of the free memory
            size_t fr = 0, tot = 0;
            HIPCHK(hipMemGetInfo(&fr, &tot));
            nb = std::max<int64_t>(1, std::min<int64_t>(nb, (int64_t)((fr + cached_bytes()) / policy::kMemShareDiv / bm_bytes)));
            HIPCHK(d_bm.alloc((size_t)nb * 2 * nt));
        }
        hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(VL_THREADS), lds, s, cols, rows, tw, th,
                           g->pm->d_node_cell.p, g->pm->d_cell_node.p, g->pm->d_node_flags.p, g->node_run_start.p,
                           g->node_nruns.p, g->pool.p, nsz.p, sb, se, gates_only, d_out.p, ctx->stats.p, d_bm.p);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(ctx->ev1, s));
    HIPCHK(hipStreamSynchronize(s));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last_vga_s = ms * 1e-3;
    if (se > sb)
        HIPCHK(copy_sync(ctx->stream, out + sb * 3, d_out.p + sb * 3, (size_t)(se - sb) * 3 * 4, hipMemcpyDeviceToHost));
    unsigned long long st0 = 0;
    HIPCHK(copy_sync(ctx->stream, &st0, ctx->stats.p, 8, hipMemcpyDeviceToHost));
    ctx->last_stats[4] = (long long)st0;   // neighbour runs walked
    ctx->last_stats[7] = se - sb;
    return DMX_OK;
}

int dmx_graph_set_prep_shard(dmx_graph* g, int64_t node_begin, int64_t node_end, dmx_allreduce_fn fn, void* user) {
    if (!g) return fail(DMX_ERR_ARG, "bad arguments");
    if (fn && (node_begin < 0 || node_end < node_begin || node_end > g->nnodes))
        return fail(DMX_ERR_ARG, "prep node range out of bounds");
    if (g->uf_count >= 0 || g->symmetric >= 0 || g->tiles_ready)
        return fail(DMX_ERR_STATE, "VGA preparation already done on this graph");
    g->prep_fn = fn;
    g->prep_user = fn ? user : nullptr;
    g->prep_b = fn ? node_begin : 0;
    g->prep_e = fn ? node_end : -1;
    return DMX_OK;
}
