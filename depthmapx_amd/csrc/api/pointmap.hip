// api/pointmap.hip -- point maps: VISPREP grid, rasterisation and fill (dmx_pointmap_*), on the host model or the GPU (fill.hip).
// Part of the dmx_api.hip unity build: included inside its extern "C" block, after the context and the
// internal types (dmx_ctx, dmx_pointmap, dmx_graph); not compiled on its own.

int dmx_pointmap_create(const double* region, double spacing, const double* lines, int64_t nlines, dmx_pointmap** out) {
    if (!region || !out || (nlines > 0 && !lines) || nlines < 0) return fail(DMX_ERR_ARG, "bad arguments");
    if (!(spacing > 0)) return fail(DMX_ERR_ARG, "spacing must be > 0");
    Rect r{region[0], region[1], region[2], region[3]};
    auto* pm = new dmx_pointmap();
    pm->host.reset(new PointMapHost(r, spacing, lines, nlines));
    if (pm->host->cols() > 16000 || pm->host->rows() > 16000) {
        delete pm;
        return fail(DMX_ERR_UNSUPPORTED, "grid larger than 16000 cells per side");
    }
    *out = pm;
    return DMX_OK;
}

int dmx_pointmap_free(dmx_pointmap* pm) {
    delete pm;
    return DMX_OK;
}

int dmx_pointmap_make_points(dmx_pointmap* pm, double x, double y, int fill_type, int* made) {
    if (!pm) return fail(DMX_ERR_ARG, "pointmap is NULL");
    if (made) *made = 0;
    if (PointMapHost::fill_state_of(fill_type) < 0) return fail(DMX_ERR_ARG, "fill_type must be 0, 1 or 2");
    int r = pm->host->fill(x, y, fill_type);
    pm->version++;
    if (made) *made = (r == 0);
    if (r == 1) return fail(DMX_ERR_OUTSIDE, "Point outside of target region");
    if (r == 3)
        return fail(DMX_ERR_UNSUPPORTED, "an AUGMENT fill from this seed never ends in the reference (expand re-queues "
                                         "augmented cells, pointdata.cpp:489)");
    return DMX_OK;
}

int dmx_pointmap_fill(dmx_pointmap* pm, double x, double y, int* made) {
    return dmx_pointmap_make_points(pm, x, y, 0, made);
}

namespace {
// scratch for scan_excl: per level, the tile sums and the tile offsets (+ total)
int64_t scan_scratch_size(int64_t n) {
    int64_t s = 1;
    for (;;) {
        const int64_t t = (n + SCAN_TILE - 1) / SCAN_TILE;
        s += 2 * t + 1;
        if (t <= 1) break;
        n = t;
    }
    return s;
}
// out[0..n) = exclusive prefix of in, out[n] = total; out must not alias in.
void scan_excl(hipStream_t st, const int64_t* in, int64_t n, int64_t* out, int64_t* scratch) {
    if (n <= 0) {
        (void)hipMemsetAsync(out, 0, sizeof(int64_t), st);
        return;
    }
    const int64_t t = (n + SCAN_TILE - 1) / SCAN_TILE;
    int64_t* tsum = scratch;
    int64_t* toff = scratch + t;
    hipLaunchKernelGGL(scan_tile_kernel, dim3((unsigned)t), dim3(SCAN_THREADS), 0, st, in, n, out, tsum);
    if (t == 1) {
        hipLaunchKernelGGL(scan_total_kernel, dim3(1), dim3(1), 0, st, out, n, (const int64_t*)tsum);
        return;
    }
    scan_excl(st, tsum, t, toff, scratch + 2 * t + 1);
    hipLaunchKernelGGL(scan_add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, n, (const int64_t*)toff);
    hipLaunchKernelGGL(scan_total_kernel, dim3(1), dim3(1), 0, st, out, n, (const int64_t*)(toff + t));
}
unsigned fill_blocks(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + FILL_THREADS - 1) / FILL_THREADS); }
} // namespace

// PointMap::makePoints on the GPU (kernels/fill.hip): blockLines on the first fill, then the ordered
// level-synchronous flood fill.  The host model stays the owner of the results (cell states,
// cropped pieces), so makeGraph and the .graph writer see exactly what the host fill would leave.
int dmx_pointmap_fill_device(dmx_ctx* ctx, dmx_pointmap* pm, double x, double y, int* made) {
    return dmx_pointmap_make_points_device(ctx, pm, x, y, 0, made);
}

int dmx_pointmap_make_points_device(dmx_ctx* ctx, dmx_pointmap* pm, double x, double y, int fill_type, int* made) {
    if (!ctx || !pm) return fail(DMX_ERR_ARG, "bad arguments");
    PointMapHost& h = *pm->host;
    if (made) *made = 0;
    const int32_t fill_state = PointMapHost::fill_state_of(fill_type);
    if (fill_state < 0) return fail(DMX_ERR_ARG, "fill_type must be 0, 1 or 2");
    // AUGMENT changes the seed cell alone or never ends (PointMapHost::fill): nothing to flood
    if (fill_state == CELL_AUGMENTED) return dmx_pointmap_make_points(pm, x, y, fill_type, made);
    int sx = 0, sy = 0;
    const int r = h.fill_seed(x, y, &sx, &sy);
    if (r == 1) return fail(DMX_ERR_OUTSIDE, "Point outside of target region");
    if (r) return DMX_OK;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const double t0 = now_s();
    const int64_t C = h.cells();
    FillGrid G;
    G.cols = h.cols();
    G.rows = h.rows();
    G.spacing = h.spacing();
    G.blx = h.bottom_left().x;
    G.bly = h.bottom_left().y;
    G.region = h.grid_region();
    DevBuf<int32_t> d_state, d_segoff;
    DevBuf<double> d_segs;
    DevBuf<int64_t> cnt, off, scratch;
    HIPCHK(d_state.alloc(C));
    HIPCHK(d_segoff.alloc(C + 1));
    HIPCHK(cnt.alloc(C + 1));
    HIPCHK(off.alloc(C + 1));
    HIPCHK(scratch.alloc(scan_scratch_size(C + 1)));
    HIPCHK(hipMemcpyAsync(d_state.p, h.state().data(), C * sizeof(int32_t), hipMemcpyHostToDevice, st));
    int64_t npieces = 0;
    if (!h.lines_blocked()) {
        // blockLines: count / scan / emit per line, place / sort / crop per cell
        const std::vector<double>& draw = h.drawing();
        const int64_t L = (int64_t)draw.size() / 4;
        DevBuf<double> d_draw;
        DevBuf<int64_t> line_off, cursor;
        DevBuf<int32_t> em_cell, cell_lines;
        HIPCHK(d_draw.alloc(std::max<int64_t>(4 * L, 1)));
        HIPCHK(line_off.alloc(L + 1));
        if (L) HIPCHK(hipMemcpyAsync(d_draw.p, draw.data(), 4 * L * sizeof(double), hipMemcpyHostToDevice, st));
        HIPCHK(hipMemsetAsync(cnt.p, 0, (C + 1) * sizeof(int64_t), st));
        DevBuf<int64_t> lcnt, lscratch;
        HIPCHK(lcnt.alloc(std::max<int64_t>(L, 1)));
        HIPCHK(lscratch.alloc(scan_scratch_size(L)));
        if (L) hipLaunchKernelGGL(rast_count_kernel, dim3(fill_blocks(L)), dim3(FILL_THREADS), 0, st, G, (const double*)d_draw.p, L, lcnt.p);
        scan_excl(st, lcnt.p, L, line_off.p, lscratch.p);
        int64_t E = 0;
        HIPCHK(copy_sync(st, &E, line_off.p + L, sizeof(int64_t), hipMemcpyDeviceToHost));
        HIPCHK(em_cell.alloc(std::max<int64_t>(E, 1)));
        HIPCHK(cell_lines.alloc(std::max<int64_t>(E, 1)));
        HIPCHK(cursor.alloc(C + 1));
        HIPCHK(hipMemsetAsync(cursor.p, 0, C * sizeof(int64_t), st));
        if (L) hipLaunchKernelGGL(rast_emit_kernel, dim3(fill_blocks(L)), dim3(FILL_THREADS), 0, st, G, (const double*)d_draw.p, L,
                                  (const int64_t*)line_off.p, em_cell.p, cnt.p);
        scan_excl(st, cnt.p, C, off.p, scratch.p);   // off = per-cell line lists
        if (E) hipLaunchKernelGGL(rast_place_kernel, dim3(fill_blocks(E)), dim3(FILL_THREADS), 0, st, (const int64_t*)line_off.p, L,
                                  (const int32_t*)em_cell.p, E, (const int64_t*)off.p, cursor.p, cell_lines.p);
        // cnt is reused for the surviving pieces per cell; cursor (int64) holds their offsets
        hipLaunchKernelGGL(rast_crop_count_kernel, dim3(fill_blocks(C)), dim3(FILL_THREADS), 0, st, G, (const double*)d_draw.p, C,
                           (const int64_t*)off.p, cell_lines.p, d_state.p, cnt.p);
        scan_excl(st, cnt.p, C, cursor.p, scratch.p);
        HIPCHK(copy_sync(st, &npieces, cursor.p + C, sizeof(int64_t), hipMemcpyDeviceToHost));
        if (npieces >= (int64_t)INT32_MAX / 4) return fail(DMX_ERR_UNSUPPORTED, "too many occluder pieces");
        HIPCHK(d_segs.alloc(std::max<int64_t>(4 * npieces, 1)));
        hipLaunchKernelGGL(rast_crop_write_kernel, dim3(fill_blocks(C)), dim3(FILL_THREADS), 0, st, G, (const double*)d_draw.p, C,
                           (const int64_t*)off.p, (const int32_t*)cell_lines.p, (const int64_t*)cursor.p, d_segs.p);
        std::vector<int64_t> off64((size_t)C + 1);
        std::vector<int32_t> seg_off((size_t)C + 1);
        std::vector<double> segs((size_t)(4 * npieces));
        HIPCHK(hipMemcpyAsync(off64.data(), cursor.p, (C + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, st));
        if (npieces) HIPCHK(hipMemcpyAsync(segs.data(), d_segs.p, 4 * npieces * sizeof(double), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (int64_t c = 0; c <= C; c++) seg_off[c] = (int32_t)off64[c];
        HIPCHK(hipMemcpyAsync(d_segoff.p, seg_off.data(), (C + 1) * sizeof(int32_t), hipMemcpyHostToDevice, st));
        h.adopt_blocked(std::move(seg_off), std::move(segs));
        VLOG("fill: blockLines on the GPU (%lld lines, %lld cell touches, %lld pieces) %.3f s\n", (long long)L, (long long)E,
             (long long)npieces, now_s() - t0);
    } else {
        npieces = (int64_t)h.segs().size() / 4;
        HIPCHK(d_segs.alloc(std::max<int64_t>(4 * npieces, 1)));
        HIPCHK(hipMemcpyAsync(d_segoff.p, h.seg_off().data(), (C + 1) * sizeof(int32_t), hipMemcpyHostToDevice, st));
        if (npieces) HIPCHK(hipMemcpyAsync(d_segs.p, h.segs().data(), 4 * npieces * sizeof(double), hipMemcpyHostToDevice, st));
    }
    // the ordered flood fill, one level per round
    const double t1 = now_s();
    DevBuf<int32_t> layer[2];
    DevBuf<uint32_t> owner;
    DevBuf<uint8_t> blocked, children;
    HIPCHK(layer[0].alloc(C));
    HIPCHK(layer[1].alloc(C));
    HIPCHK(owner.alloc(C));
    HIPCHK(blocked.alloc(C));
    HIPCHK(children.alloc(C));
    HIPCHK(hipMemsetAsync(owner.p, 0xFF, C * sizeof(uint32_t), st));
    const int64_t c0 = h.index(sx, sy);
    G.fill_state = fill_state;
    const int32_t seed_state = fill_state | (h.state()[c0] & CELL_BLOCKED);
    const int32_t seed_cell = (int32_t)c0;
    HIPCHK(hipMemcpyAsync(d_state.p + c0, &seed_state, sizeof(int32_t), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(layer[0].p, &seed_cell, sizeof(int32_t), hipMemcpyHostToDevice, st));
    int64_t n = 1, levels = 0;
    int cur = 0;
    DevBuf<long long> io;
    HIPCHK(io.alloc(3));
    const bool wg_on = !getenv("DMX_FILL_GRID");   // test hook: every level grid-wide
    while (n > 0) {
        if (wg_on && n <= FILL_WG_CAP) {
            // small layers: one workgroup runs levels until the fill ends or a layer outgrows the cap
            long long h_io[3] = {(long long)n, (long long)cur, 0};
            HIPCHK(hipMemcpyAsync(io.p, h_io, sizeof(h_io), hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(fill_levels_wg_kernel, dim3(1), dim3(FILL_WG_THREADS), 0, st, G, (const int32_t*)d_segoff.p,
                               (const double*)d_segs.p, d_state.p, layer[0].p, layer[1].p, owner.p, io.p);
            HIPCHK(hipGetLastError());
            HIPCHK(copy_sync(st, h_io, io.p, sizeof(h_io), hipMemcpyDeviceToHost));
            n = h_io[0];
            cur = (int)h_io[1];
            levels += h_io[2];
            if (n == 0) break;
        }
        hipLaunchKernelGGL(fill_claim_kernel, dim3(fill_blocks(n)), dim3(FILL_THREADS), 0, st, G, (const int32_t*)d_segoff.p,
                           (const double*)d_segs.p, (const int32_t*)d_state.p, (const int32_t*)layer[cur].p, n, owner.p, blocked.p);
        hipLaunchKernelGGL(fill_resolve_kernel, dim3(fill_blocks(n)), dim3(FILL_THREADS), 0, st, G, d_state.p,
                           (const int32_t*)layer[cur].p, n, (const uint32_t*)owner.p, (const uint8_t*)blocked.p, children.p, cnt.p);
        scan_excl(st, cnt.p, n, off.p, scratch.p);
        int64_t n_next = 0;
        HIPCHK(copy_sync(st, &n_next, off.p + n, sizeof(int64_t), hipMemcpyDeviceToHost));
        if (n_next)
            hipLaunchKernelGGL(fill_push_kernel, dim3(fill_blocks(n)), dim3(FILL_THREADS), 0, st, G, d_state.p,
                               (const int32_t*)layer[cur].p, n, (const uint8_t*)children.p, (const int64_t*)off.p, n_next,
                               layer[cur ^ 1].p);
        HIPCHK(hipGetLastError());
        cur ^= 1;
        n = n_next;
        levels++;
    }
    std::vector<int32_t> state((size_t)C);
    HIPCHK(copy_sync(st, state.data(), d_state.p, C * sizeof(int32_t), hipMemcpyDeviceToHost));
    h.adopt_state(std::move(state));
    pm->version++;
    ctx->last_fill_s[0] = t1 - t0;
    ctx->last_fill_s[1] = now_s() - t1;
    ctx->last_fill_levels = levels;
    VLOG("fill: flood fill on the GPU, %lld levels, %lld filled, %.3f s\n", (long long)levels, (long long)h.filled_count(),
         now_s() - t1);
    if (made) *made = 1;
    return DMX_OK;
}

int dmx_ctx_last_fill(dmx_ctx* ctx, double* block_s, double* fill_s, int64_t* levels) {
    if (!ctx) return fail(DMX_ERR_ARG, "ctx is NULL");
    if (block_s) *block_s = ctx->last_fill_s[0];
    if (fill_s) *fill_s = ctx->last_fill_s[1];
    if (levels) *levels = ctx->last_fill_levels;
    return DMX_OK;
}

int dmx_pointmap_info(const dmx_pointmap* pm, int32_t* cols, int32_t* rows, double* bx, double* by, int64_t* filled) {
    if (!pm) return fail(DMX_ERR_ARG, "pointmap is NULL");
    if (cols) *cols = pm->host->cols();
    if (rows) *rows = pm->host->rows();
    if (bx) *bx = pm->host->bottom_left().x;
    if (by) *by = pm->host->bottom_left().y;
    if (filled) *filled = pm->host->filled_count();
    return DMX_OK;
}

int dmx_pointmap_state(const dmx_pointmap* pm, int32_t* out) {
    if (!pm || !out) return fail(DMX_ERR_ARG, "bad arguments");
    std::memcpy(out, pm->host->state().data(), pm->host->state().size() * 4);
    return DMX_OK;
}

int dmx_pointmap_cell_lines(dmx_pointmap* pm, int32_t* counts, double* pieces, int64_t* total) {
    if (!pm) return fail(DMX_ERR_ARG, "pointmap is NULL");
    pm->host->block_lines();
    const auto& off = pm->host->seg_off();
    const auto& segs = pm->host->segs();
    if (total) *total = (int64_t)segs.size() / 4;
    if (counts)
        for (size_t c = 0; c + 1 < off.size(); c++) counts[c] = off[c + 1] - off[c];
    if (pieces && !segs.empty()) std::memcpy(pieces, segs.data(), segs.size() * 8);
    return DMX_OK;
}
