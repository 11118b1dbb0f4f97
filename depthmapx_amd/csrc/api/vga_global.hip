// api/vga_global.hip -- VGA global: the O(R) preparation (symmetry certificate, scan order, tile summaries, partial-tile masks), the tile search, the fallbacks and the reference-order re-run.
// Part of the dmx_api.hip unity build: included inside its extern "C" block, after the context and the
// internal types (dmx_ctx, dmx_pointmap, dmx_graph); not compiled on its own.

// ---------------------------------------------------------------- VGA global
// Node range of this rank's share of the preparation scatters ([0, N) when not sharded).
static void prep_range(const dmx_graph* g, int64_t& b, int64_t& e) {
    b = 0; e = g->nnodes;
    if (g->prep_fn && g->prep_e >= 0) { b = g->prep_b; e = g->prep_e; }
}
// Sum a partial device buffer over the ranks (no-op when not sharded).  The stream is drained first:
// the caller's collective runs on its own stream and returns only once the sum is in place.
static int prep_allreduce(dmx_graph* g, void* p, int64_t count, int dtype) {
    if (!g->prep_fn || count <= 0) return DMX_OK;
    HIPCHK(hipStreamSynchronize(g->ctx->stream));
    if (g->prep_fn(p, count, dtype, g->prep_user) != 0)
        return fail(DMX_ERR_STATE, "prep all-reduce callback failed");
    return DMX_OK;
}
// U_f (filled cells that appear in some run: the early-exit universe of every BFS) by range counts,
// plus the longest-first scan pool.  O(runs) with a few line-prefix passes.
static int prepare_symmetry(dmx_graph* g);
static int build_scan_order(dmx_graph* g);
static int prepare_uf(dmx_graph* g) {
    if (g->scan_ready) return DMX_OK;
    // the symmetry pass computes U_f from its in-set hashes; coverage counting only when it is skipped
    if (int rc = prepare_symmetry(g)) return rc;
    dmx_ctx* ctx = g->ctx;
    hipStream_t s = ctx->stream;
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int tw = (cols + 7) / 8, th = (rows + 7) / 8;
    const int64_t C = (int64_t)cols * rows, N = g->nnodes;
    DevBuf<int> cov;
    DevBuf<unsigned long long> cnt;
    HIPCHK(cnt.alloc(1));
    HIPCHK(hipMemsetAsync(cnt.p, 0, 8, s));
    const bool have_uf = g->uf_count >= 0;
    if (!have_uf) {
        HIPCHK(cov.alloc((size_t)4 * C));
        HIPCHK(g->uf_tiles.alloc((size_t)tw * th));
        HIPCHK(g->notuf_tiles.alloc((size_t)tw * th));
        HIPCHK(hipMemsetAsync(cov.p, 0, (size_t)4 * C * 4, s));
        int64_t pb, pe;
        prep_range(g, pb, pe);
        if (pe > pb) {
            hipLaunchKernelGGL(cov_scatter_kernel, dim3((unsigned)std::min<int64_t>(pe - pb, 4096)), dim3(256), 0, s,
                               cols, rows, pe - pb, g->node_run_start.p + pb, g->node_nruns.p + pb, g->pool.p, cov.p);
            HIPCHK(hipGetLastError());
        }
        if (int rc = prep_allreduce(g, cov.p, (int64_t)4 * C, DMX_I32)) return rc;
        hipLaunchKernelGGL(cov_lines_kernel, dim3((cols + rows + 127) / 128, 4), dim3(128), 0, s, cols, rows, cov.p);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(cov_tiles_kernel, dim3((tw * th + 255) / 256), dim3(256), 0, s, cols, rows, tw, th,
                           g->pm->d_cell_node.p, cov.p, g->uf_tiles.p, g->notuf_tiles.p, cnt.p);
        HIPCHK(hipGetLastError());
    }
    unsigned long long ufc = have_uf ? (unsigned long long)g->uf_count : 0ull;
    if (!have_uf) HIPCHK(copy_sync(s, &ufc, cnt.p, 8, hipMemcpyDeviceToHost));
    if (int rc = build_scan_order(g)) return rc;
    g->uf_count = (int64_t)ufc;
    g->scan_ready = true;
    return DMX_OK;
}

// The scan order: every node's runs longest-first (scan_pool, node order), with per-node and per-cell starts.
static int build_scan_order(dmx_graph* g) {
    dmx_ctx* ctx = g->ctx;
    hipStream_t s = ctx->stream;
    PointMapHost& h = *g->pm->host;
    const int rows = h.rows();
    const int64_t C = (int64_t)h.cols() * rows, N = g->nnodes;
    std::vector<int32_t> nr((size_t)std::max<int64_t>(N, 1));
    if (N) HIPCHK(copy_sync(s, nr.data(), g->node_nruns.p, N * 4, hipMemcpyDeviceToHost));
    std::vector<int64_t> ss((size_t)std::max<int64_t>(N, 1));
    int64_t acc = 0;
    for (int64_t k = 0; k < N; k++) { ss[k] = acc; acc += nr[k]; }
    DevBuf<int64_t>& d_ss = g->scan_start;
    HIPCHK(d_ss.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(g->scan_pool.alloc(std::max<int64_t>(acc, 1)));
    HIPCHK(g->cell_scan_start.alloc(C));
    HIPCHK(g->cell_nruns.alloc(C));
    HIPCHK(hipMemsetAsync(g->cell_nruns.p, 0, C * 4, s));
    if (N) {
        HIPCHK(hipMemcpyAsync(d_ss.p, ss.data(), N * 8, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(scan_pool_kernel, dim3((unsigned)std::min<int64_t>(N, 8192)), dim3(256), 0, s, rows,
                           g->pm->d_node_cell.p, N, g->node_run_start.p, g->node_nruns.p, g->bin_nruns.p, g->pool.p, d_ss.p,
                           g->scan_pool.p, g->cell_scan_start.p, g->cell_nruns.p);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(s));
    g->scan_released = false;
    return DMX_OK;
}

// The wide-grid partial-tile masks take the scan order's place (prepare_tiles): the searches that read the
// scan order itself (vga_do, a tile search without the masks) free the tile-visibility data and rebuild it.
static int restore_scan_order(dmx_graph* g) {
    if (!g->scan_released) return DMX_OK;
    g->pmask.reset(); g->ppre.reset(); g->poff.reset();
    g->tvis.reset(); g->ftvis.reset(); g->tvsum.reset(); g->tvnz.reset(); g->ttvis.reset();
    g->tvw = 0;
    g->tiles_ready = false;
    return build_scan_order(g);
}

// In-set corrections for bottom-up BFS (vga_do.hip, "symmetry / in-set corrections").
static int prepare_symmetry(dmx_graph* g) {
    if (g->symmetric >= 0) return DMX_OK;
    const char* force = getenv("DMX_VGA_KERNEL");
    if (force && std::string(force) == "topdown") {
        g->symmetric = 0;
        g->sym_diff.reset(); g->sym_ho.reset(); g->sym_fused = false;
        return DMX_OK;
    }
    dmx_ctx* ctx = g->ctx;
    hipStream_t s = ctx->stream;
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int64_t C = (int64_t)cols * rows, N = g->nnodes;
    const int kSpecLimit = 4096;
    DevBuf<unsigned long long> prefix, diff_own, ho_own;
    DevBuf<int32_t> flist;
    DevBuf<int> fcount;
    HIPCHK(flist.alloc(kSpecLimit));
    HIPCHK(fcount.alloc(1));
    HIPCHK(hipMemsetAsync(fcount.p, 0, 4, s));
    const int maxlines = cols + rows;
    unsigned long long *diff = nullptr, *ho = nullptr;
    if (g->sym_fused) {
        // makeGraph did the scatter over the whole graph as it published the runs: complete on every rank,
        // so no all-reduce either
        diff = g->sym_diff.p;
        ho = g->sym_ho.p;
        ctx->last_stats[39] = 0;
    } else {
        const double t_sym = now_s();   // the scatter a sharded or assembled graph pays here (last_stats[39])
        HIPCHK(prefix.alloc((size_t)4 * C));
        HIPCHK(diff_own.alloc((size_t)4 * C));
        HIPCHK(ho_own.alloc(std::max<int64_t>(N, 1)));
        diff = diff_own.p;
        ho = ho_own.p;
        HIPCHK(hipMemsetAsync(diff, 0, (size_t)4 * C * 8, s));
        HIPCHK(hipMemsetAsync(ho, 0, (size_t)std::max<int64_t>(N, 1) * 8, s));
        hipLaunchKernelGGL(sym_lines_kernel, dim3((maxlines + 127) / 128, 4), dim3(128), 0, s, cols, rows,
                           g->pm->d_cell_node.p, prefix.p, 0);
        HIPCHK(hipGetLastError());
        int64_t pb, pe;
        prep_range(g, pb, pe);
        if (pe > pb) {
            hipLaunchKernelGGL(sym_scatter_kernel, dim3((unsigned)std::min<int64_t>(pe - pb, 4096)), dim3(256), 0, s,
                               cols, rows, g->pm->d_node_cell.p + pb, pe - pb, g->node_run_start.p + pb,
                               g->node_nruns.p + pb, g->pool.p, prefix.p, diff, ho + pb);
            HIPCHK(hipGetLastError());
        }
        if (int rc = prep_allreduce(g, diff, (int64_t)4 * C, DMX_I64)) return rc;
        if (int rc = prep_allreduce(g, ho, N, DMX_I64)) return rc;
        HIPCHK(hipStreamSynchronize(s));
        ctx->last_stats[39] = (long long)((now_s() - t_sym) * 1e6);
    }
    hipLaunchKernelGGL(sym_lines_kernel, dim3((maxlines + 127) / 128, 4), dim3(128), 0, s, cols, rows,
                       g->pm->d_cell_node.p, diff, 1);
    HIPCHK(hipGetLastError());
    if (N) {
        hipLaunchKernelGGL(sym_flag_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, rows,
                           g->pm->d_node_cell.p, N, C, diff, ho, fcount.p, flist.p, kSpecLimit);
        HIPCHK(hipGetLastError());
    }
    // U_f straight from the in-set hashes (uf_hi_tiles_kernel): no separate coverage pass
    const int tw = (cols + 7) / 8, th = (rows + 7) / 8;
    DevBuf<unsigned long long> ufcnt;
    HIPCHK(ufcnt.alloc(1));
    HIPCHK(hipMemsetAsync(ufcnt.p, 0, 8, s));
    HIPCHK(g->uf_tiles.alloc((size_t)tw * th));
    HIPCHK(g->notuf_tiles.alloc((size_t)tw * th));
    hipLaunchKernelGGL(uf_hi_tiles_kernel, dim3((tw * th + 255) / 256), dim3(256), 0, s, cols, rows, tw, th,
                       g->pm->d_cell_node.p, diff, g->uf_tiles.p, g->notuf_tiles.p, ufcnt.p);
    HIPCHK(hipGetLastError());
    int nspec = 0;
    unsigned long long ufc = 0;
    HIPCHK(hipMemcpyAsync(&nspec, fcount.p, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&ufc, ufcnt.p, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    g->sym_diff.reset(); g->sym_ho.reset(); g->sym_fused = false;   // consumed
    g->uf_count = (int64_t)ufc;
    g->nspecial = nspec;
    if (nspec == 0) { g->symmetric = 1; return DMX_OK; }
    if (nspec > kSpecLimit) { g->symmetric = 0; return DMX_OK; }
    std::vector<int32_t> specs((size_t)nspec);
    HIPCHK(copy_sync(g->ctx->stream, specs.data(), flist.p, nspec * 4, hipMemcpyDeviceToHost));
    std::sort(specs.begin(), specs.end());
    g->special_nodes = specs;
    std::vector<uint8_t> is_spec((size_t)N, 0);
    std::vector<int32_t> sidx((size_t)N, -1);
    for (int i = 0; i < nspec; i++) { is_spec[specs[i]] = 1; sidx[specs[i]] = i; }
    DevBuf<uint8_t> d_is;
    DevBuf<int32_t> d_specs, d_out;
    DevBuf<int> d_outn;
    HIPCHK(d_is.alloc(N));
    HIPCHK(d_specs.alloc(nspec));
    HIPCHK(d_out.alloc((size_t)nspec * nspec));
    HIPCHK(d_outn.alloc(nspec));
    HIPCHK(copy_sync(g->ctx->stream, d_is.p, is_spec.data(), N, hipMemcpyHostToDevice));
    HIPCHK(copy_sync(g->ctx->stream, d_specs.p, specs.data(), nspec * 4, hipMemcpyHostToDevice));
    // on the context stream: a null-stream hipMemset is not ordered before the kernel on this
    // non-blocking stream, and under load the kernel then counted from stale memory (the 4-rank
    // one-GPU rehearsal's heap abort)
    HIPCHK(hipMemsetAsync(d_outn.p, 0, nspec * 4, s));
    hipLaunchKernelGGL(sym_special_out_kernel, dim3(nspec), dim3(256), 0, s, rows, d_specs.p, nspec,
                       g->pm->d_node_cell.p, g->pm->d_cell_node.p, d_is.p, g->node_run_start.p, g->node_nruns.p,
                       g->pool.p, d_out.p, d_outn.p, nspec);
    HIPCHK(hipGetLastError());
    std::vector<int32_t> outn((size_t)nspec), out((size_t)nspec * nspec);
    HIPCHK(hipMemcpyAsync(outn.data(), d_outn.p, nspec * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out.data(), d_out.p, (size_t)nspec * nspec * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    // A[a][b] = b in cells(a), over special nodes (asymmetric pairs only involve special nodes)
    std::vector<std::vector<char>> A((size_t)nspec, std::vector<char>((size_t)nspec, 0));
    for (int a = 0; a < nspec; a++) {
        if (outn[a] < 0) return fail(DMX_ERR_STATE, "internal: special-node list count out of range");
        for (int j = 0; j < std::min(outn[a], nspec); j++) {
            const int32_t v = out[(size_t)a * nspec + j];
            if (v < 0 || v >= N || sidx[v] < 0) return fail(DMX_ERR_STATE, "internal: special-node list entry out of range");
            A[a][sidx[v]] = 1;
        }
    }
    std::vector<std::vector<int32_t>> extra((size_t)nspec), missing((size_t)nspec);
    for (int a = 0; a < nspec; a++)
        for (int b = 0; b < nspec; b++)
            if (A[a][b] && !A[b][a]) {          // b in cells(a), a not in cells(b)
                extra[b].push_back(specs[a]);   // a is an in-neighbour of b outside cells(b)
                missing[a].push_back(specs[b]); // b sits in cells(a) but is not an in-neighbour of a
            }
    std::vector<int32_t> eoff(1, 0), moff(1, 0), ev, mv;
    for (int i = 0; i < nspec; i++) {
        ev.insert(ev.end(), extra[i].begin(), extra[i].end());
        mv.insert(mv.end(), missing[i].begin(), missing[i].end());
        eoff.push_back((int32_t)ev.size());
        moff.push_back((int32_t)mv.size());
    }
    HIPCHK(g->spec_index.alloc(N));
    HIPCHK(g->extra_off.alloc(eoff.size()));
    HIPCHK(g->missing_off.alloc(moff.size()));
    HIPCHK(g->extra.alloc(std::max<size_t>(ev.size(), 1)));
    HIPCHK(g->missing.alloc(std::max<size_t>(mv.size(), 1)));
    HIPCHK(copy_sync(g->ctx->stream, g->spec_index.p, sidx.data(), N * 4, hipMemcpyHostToDevice));
    HIPCHK(copy_sync(g->ctx->stream, g->extra_off.p, eoff.data(), eoff.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(copy_sync(g->ctx->stream, g->missing_off.p, moff.data(), moff.size() * 4, hipMemcpyHostToDevice));
    if (!ev.empty()) HIPCHK(copy_sync(g->ctx->stream, g->extra.p, ev.data(), ev.size() * 4, hipMemcpyHostToDevice));
    if (!mv.empty()) HIPCHK(copy_sync(g->ctx->stream, g->missing.p, mv.data(), mv.size() * 4, hipMemcpyHostToDevice));
    g->symmetric = 1;
    return DMX_OK;
}

// Partial-tile masks for phase C's exact test (vga_tile.hip pmask_hit): counts from the full rows
// (every rank after the rows' all-reduce), an exclusive scan into per-cell offsets, then the masks of every
// node.  Each rank builds all of them itself, with no collective: the pass costs ~0.07 s at 1000^2, where
// all-reducing its ~10 GB over the ranks would cost more, and whether a rank has them does not change
// its results (phase C scans runs without them), so the ranks need not agree.  Skipped when they would
// take more than a quarter of the free memory.
static int prepare_pmask(dmx_graph* g, int rows, int tw, int th, int tvw, int64_t Ct, bool wide) {
    dmx_ctx* ctx = g->ctx;
    hipStream_t s = ctx->stream;
    DevBuf<int64_t> cnt, scratch;
    HIPCHK(cnt.alloc(Ct));
    HIPCHK(g->poff.alloc(Ct + 1));
    HIPCHK(g->ppre.alloc((size_t)Ct * tvw));
    HIPCHK(scratch.alloc(scan_scratch_size(Ct)));
    hipLaunchKernelGGL(tile_pcount_kernel, dim3((unsigned)((Ct + 3) / 4)), dim3(256), 0, s, Ct, tvw, g->tvis.p, g->ftvis.p,
                       cnt.p, g->ppre.p);
    HIPCHK(hipGetLastError());
    scan_excl(s, cnt.p, Ct, g->poff.p, scratch.p);
    HIPCHK(hipGetLastError());
    int64_t total = 0;
    HIPCHK(copy_sync(s, &total, g->poff.p + Ct, 8, hipMemcpyDeviceToHost));
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const size_t mask_b = (size_t)total * 8;
    bool build = total > 0 && mask_b <= free_b / policy::kMemShareDiv;
    const int pmcap = wide ? PM_CAP_WIDE : PM_CAP;
    if (wide && total > 0 && tile_pmask_lds(tvw, pmcap) <= policy::kLdsPassBudget) {
        // Above 1024 cells a side the masks (~80 GB at 2000^2) fit only in the scan order's place: the runs
        // are then scanned in pool order (the heads and tile-common runs stay, built from the scan order;
        // only special nodes still scan, from the first run; every regular cell phase C sees takes the masks)
        const size_t reserve = 16ull << 30;   // the search's per-workgroup buffers
        const size_t free_all = free_b + cached_bytes();
        const size_t scan_b = g->scan_pool.p ? g->scan_pool.n * sizeof(Run) + (size_t)g->nnodes * 8 +
                                                   (size_t)g->cell_scan_start.n * 12 : 0;
        if (mask_b + reserve <= free_all) {
            build = true;
        } else if (g->scan_pool.p && mask_b + reserve <= free_all + scan_b) {
            g->scan_pool.reset(); g->scan_start.reset(); g->cell_scan_start.reset(); g->cell_nruns.reset();
            g->scan_released = true;
            hipLaunchKernelGGL(tile_pool_order_kernel, dim3((unsigned)((g->nnodes + 255) / 256)), dim3(256), 0, s, rows, tw,
                               g->pm->d_node_cell.p, g->nnodes, g->node_run_start.p, g->tscan_start.p);
            HIPCHK(hipGetLastError());
            VLOG("vga prep: scan order released for %.1f GB of partial-tile masks\n", mask_b / 1e9);
            build = true;
            if (getenv("DMX_VGA_PMASK_FAIL"))   // test hook: a failure after the release (the next call recovers)
                return fail(DMX_ERR_HIP, "injected failure after the scan order was released");
        } else {
            build = false;
        }
    }
    if (!build) {
        g->poff.reset();
        g->ppre.reset();
        return DMX_OK;
    }
    HIPCHK(g->pmask.alloc((size_t)total));
    HIPCHK(hipMemsetAsync(g->pmask.p, 0, mask_b, s));
    const int64_t N = g->nnodes;
    if (N > 0) {
        const int64_t nb = std::min<int64_t>(N, (int64_t)ctx->num_cu * 16);
        hipLaunchKernelGGL(tile_pmask_kernel, dim3((unsigned)nb), dim3(64 * TV_WAVES), tile_pmask_lds(tvw, pmcap), s, rows,
                           tw, th, g->pm->d_node_cell.p, N, g->node_run_start.p, g->node_nruns.p, g->pool.p, g->tvis.p,
                           g->ftvis.p, g->poff.p, g->pmask.p, pmcap);
        HIPCHK(hipGetLastError());
    }
    return DMX_OK;
}

// Which memory-dependent VGA preparation structures the graph holds (last_stats[40..42]; bench.py prints them):
// the search a call takes depends on what fitted next to the graph (DESIGN.md sections 1 and 5).
static void prep_state_stats(dmx_ctx* ctx, const dmx_graph* g) {
    long long f = 0;
    if (g->scan_pool.p) f |= 1;          // the BFS scan order
    if (g->scan_released) f |= 2;        // ... released for the masks (runs read in pool order)
    if (g->tvis.p) f |= 4;               // tile-visibility rows
    if (g->ftvis.p) f |= 8;              // fully-seen tile rows
    if (g->ttvis.p) f |= 16;             // tile-to-tile rows
    if (g->pmask.p) f |= 32;             // partial-tile masks
    if (g->tvsum.p || g->tvnz.p) f |= 64;   // row summaries
    ctx->last_stats[40] = f;
    ctx->last_stats[41] = (long long)((g->tvis.p ? g->tvis.n * 8 : 0) + (g->ftvis.p ? g->ftvis.n * 8 : 0) +
                                      (g->ttvis.p ? g->ttvis.n * 8 : 0) + (g->tvsum.p ? g->tvsum.n * 8 : 0) + (g->tvnz.p ? g->tvnz.n * 8 : 0));
    ctx->last_stats[42] = (long long)(g->scan_pool.p ? g->scan_pool.n * sizeof(Run) : 0);
}

// LDS of the tile BFS workgroup: the frontier bitmap (unless FG), the tile-row summary Fsr, then either the
// per-tile column summary Fsc or the line-resolved summaries RB / CB, then the level histogram.  Returns the
// bytes (0: does not fit) and the variant: *fg the frontier in HBM, *rbm the line summaries.
static size_t tile_lds_layout(int tw, int th, bool* fg, bool* rbm) {
    const size_t nt = (size_t)tw * th, wr_ = (tw + 63) / 64, wc_ = (th + 63) / 64;
    const size_t lds_f = nt * 8, lds_h = (size_t)VGA_HMAX * 4;
    const size_t lds_sc = (size_t)(th * wr_ + tw * wc_) * 8, lds_rbcb = (size_t)(th * wr_ + th * 8 * wr_ + tw * 8 * wc_) * 8;
    const size_t lds_cap = (size_t)160 * 1024 - 1024;
    const char* rb_env = getenv("DMX_VGA_RB");
    const bool rb_ok = !(rb_env && atoi(rb_env) == 0);
    *fg = false;
    *rbm = false;
    if (rb_ok && lds_f + lds_rbcb + lds_h <= lds_cap) { *rbm = true; return lds_f + lds_rbcb + lds_h; }
    if (lds_f + lds_sc + lds_h <= lds_cap) return lds_f + lds_sc + lds_h;
    if (rb_ok && lds_rbcb + lds_h <= lds_cap) { *fg = true; *rbm = true; return lds_rbcb + lds_h; }
    if (lds_sc + lds_h <= lds_cap) { *fg = true; return lds_sc + lds_h; }
    return 0;
}

// Tile-ordered per-cell arrays, head runs and tile-common runs for vga_tile_kernel (O(runs)).
static int prepare_tiles(dmx_graph* g) {
    if (g->tiles_ready) return DMX_OK;
    // a preparation that released the scan order for the masks and then failed (prepare_pmask) left the tile data
    // half built: rebuild the scan order before the heads and the tile-common runs read it
    if (g->scan_released)
        if (int rc = restore_scan_order(g)) return rc;
    dmx_ctx* ctx = g->ctx;
    hipStream_t s = ctx->stream;
    PointMapHost& h = *g->pm->host;
    const int cols = h.cols(), rows = h.rows();
    const int tw = (cols + 7) / 8, th = (rows + 7) / 8, nt = tw * th;
    const int64_t N = g->nnodes, Ct = (int64_t)nt * 64;
    HIPCHK(g->tscan_start.alloc(Ct));
    HIPCHK(g->tnruns.alloc(Ct));
    HIPCHK(g->heads.alloc((size_t)KH * Ct));
    HIPCHK(g->cr.alloc((size_t)CRK * nt));
    HIPCHK(g->regular_tiles.alloc(nt));
    HIPCHK(hipMemsetAsync(g->tnruns.p, 0, Ct * 4, s));
    HIPCHK(hipMemsetAsync(g->tscan_start.p, 0, Ct * 8, s));
    HIPCHK(hipMemsetAsync(g->heads.p, 0xFF, (size_t)KH * Ct * sizeof(Run), s));
    // regular = U_f minus the special (asymmetric) nodes
    std::vector<unsigned long long> uf((size_t)nt);
    HIPCHK(hipMemcpyAsync(uf.data(), g->uf_tiles.p, nt * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    for (int32_t k : g->special_nodes) {
        const int c = g->pm->node_cell[k];
        const int x = c / rows, y = c % rows;
        uf[(size_t)(y >> 3) * tw + (x >> 3)] &= ~(1ull << ((y & 7) * 8 + (x & 7)));
    }
    HIPCHK(hipMemcpyAsync(g->regular_tiles.p, uf.data(), nt * 8, hipMemcpyHostToDevice, s));
    if (N) {
        hipLaunchKernelGGL(tile_heads_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, rows, tw,
                           g->pm->d_node_cell.p, N, g->node_nruns.p, g->scan_pool.p, g->scan_start.p,
                           g->tscan_start.p, g->tnruns.p, g->heads.p, (size_t)Ct);
        HIPCHK(hipGetLastError());
    }
    const int dmax = std::max(cols, rows);
    const size_t lds = (size_t)8 * (dmax + 2) * 4;
    // a capacity of the tile path: the callers fall back to the direction-optimising / top-down searches
    if (lds > policy::kLdsPassBudget) return fail(DMX_ERR_CAPACITY, "grid too long for the tile-common-run pass");
    hipLaunchKernelGGL(tile_cr_kernel, dim3((unsigned)std::min<int64_t>(nt, (int64_t)ctx->num_cu * 8)), dim3(CR_THREADS),
                       lds, s, cols, rows, tw, th, g->regular_tiles.p, g->pm->d_cell_node.p, g->node_run_start.p,
                       g->node_nruns.p, g->scan_start.p, g->scan_pool.p, g->pool.p, dmax, g->cr.p);
    HIPCHK(hipGetLastError());
    // tile-visibility rows (phase C rejects cells with no frontier tile in view); ~2 KB per cell at
    // 1000^2, skipped when they would not fit comfortably
    const int tvw = th * ((tw + 63) / 64);
    const size_t tv_bytes = (size_t)Ct * tvw * 8;
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const char* tv_env = getenv("DMX_VGA_TVIS");
    const bool tv_on = !(tv_env && atoi(tv_env) == 0);
    const char* ftv_env = getenv("DMX_VGA_FTVIS");
    const bool ftv_on = !(ftv_env && atoi(ftv_env) == 0);
    // Grids up to 1024 cells a side (tvw <= 256: the masks' row test reads 4 words a lane): tvis, ftvis, the
    // tile rows and the partial-tile masks when they take at most a quarter of the free memory.  Wider grids
    // (2000^2: 8 KB a row, 32 GB) keep tvis, the phase-C miss certificate in front of the run scan, when it takes
    // at most a third of what is free next to the graph and its scan order, and ftvis too (the certain-hit
    // test) when both leave 24 GiB free for the search's own buffers.
    const bool wide = tvw > 256;
    const size_t free_all = free_b + cached_bytes();
    // (the wide-grid ftvis, tile rows and masks serve the HBM-frontier variant, whose code reads wide rows; a
    // wide grid whose frontier fits the LDS -- a few tiles high, very long -- keeps tvis alone)
    bool fg_grid = false, rbm_grid = false;
    tile_lds_layout(tw, th, &fg_grid, &rbm_grid);
    bool ftv = ftv_on && (!wide || (fg_grid && 2 * tv_bytes + (24ull << 30) <= free_all));
    bool tv_build = tv_on && N && tv_bytes <= (32ull << 30) &&
                    (wide ? tv_bytes <= free_all / policy::kMemShareWideDiv : tv_bytes * (ftv ? 2 : 1) <= free_b / policy::kMemShareDiv);
    if (g->prep_fn) {
        // every rank must take the same branches (the rows are all-reduced): build only what all can
        DevBuf<int64_t> veto;
        HIPCHK(veto.alloc(1));
        const int64_t v = (tv_build ? 0 : 1) + (ftv ? 0 : (1ll << 20));
        HIPCHK(hipMemcpyAsync(veto.p, &v, 8, hipMemcpyHostToDevice, s));
        if (int rc = prep_allreduce(g, veto.p, 1, DMX_I64)) return rc;
        int64_t vs = 0;
        HIPCHK(copy_sync(g->ctx->stream, &vs, veto.p, 8, hipMemcpyDeviceToHost));
        tv_build = (vs & ((1ll << 20) - 1)) == 0;
        ftv = (vs >> 20) == 0;
    }
    if (tv_build) {
        HIPCHK(g->tvis.alloc(Ct * tvw));
        HIPCHK(hipMemsetAsync(g->tvis.p, 0, tv_bytes, s));
        if (ftv) {
            HIPCHK(g->ftvis.alloc(Ct * tvw));
            HIPCHK(hipMemsetAsync(g->ftvis.p, 0, tv_bytes, s));
        }
        const int ncw = (nt + 3) / 4;
        const size_t tv_lds = ((size_t)(ncw + 1) / 2 + (size_t)(tvw + (ncw + 1) / 2)) * 8;   // one node per workgroup
        if (tv_lds > policy::kLdsPassBudget) return fail(DMX_ERR_CAPACITY, "grid too large for the tile-visibility pass");
        int64_t pb, pe;
        prep_range(g, pb, pe);
        if (pe > pb) {
            const int64_t nb = std::min<int64_t>(pe - pb, (int64_t)ctx->num_cu * 16);
            hipLaunchKernelGGL(tile_vis_kernel, dim3((unsigned)nb), dim3(64 * TV_WAVES), tv_lds, s, rows, tw, th,
                               g->pm->d_node_cell.p + pb, pe - pb, g->node_run_start.p + pb, g->node_nruns.p + pb,
                               g->pool.p, g->notuf_tiles.p, g->tvis.p, ftv ? g->ftvis.p : nullptr);
            HIPCHK(hipGetLastError());
        }
        // rows of distinct nodes are disjoint: the sum over ranks is their union
        if (int rc = prep_allreduce(g, g->tvis.p, Ct * tvw, DMX_I64)) return rc;
        if (ftv)
            if (int rc = prep_allreduce(g, g->ftvis.p, Ct * tvw, DMX_I64)) return rc;
        const char* tt_env = getenv("DMX_VGA_TTVIS");
        if (ftv && !(tt_env && atoi(tt_env) == 0)) {
            HIPCHK(g->ttvis.alloc((size_t)2 * nt * tvw));   // ttvis, then ttany
            hipLaunchKernelGGL(tile_tt_kernel, dim3((unsigned)((nt + 3) / 4)), dim3(256), 0, s, nt, tvw, g->regular_tiles.p,
                               g->ftvis.p, g->tvis.p, g->ttvis.p, g->ttvis.p + (size_t)nt * tvw);
            HIPCHK(hipGetLastError());
        }
        const char* pm_env = getenv("DMX_VGA_PMASK");
        // (wide grids: the masks need the row summaries, at most 64 words of them, and a 16-bit row prefix)
        if (ftv && !(pm_env && atoi(pm_env) == 0) && (!wide || ((tvw + 63) / 64 <= 64 && nt <= 65535)))
            if (int rc = prepare_pmask(g, rows, tw, th, tvw, Ct, wide)) return rc;
        // the row summaries keep word k in lane k (vga_tile.hip reads them with readlane): at most 64 words
        if (wide && (tvw + 63) / 64 <= 64) {
            HIPCHK(g->tvsum.alloc((size_t)Ct * ((tvw + 63) / 64)));
            hipLaunchKernelGGL(tile_vsum_kernel, dim3((unsigned)((Ct + 3) / 4)), dim3(256), 0, s, Ct, tvw, g->tvis.p,
                               g->tvsum.p);
            HIPCHK(hipGetLastError());
        }
        // narrow grids with the masks: phase C's row loads skip the cell's zero words (1000^2: 61 % of the words
        // under a frontier tile row are zero; 32 B a cell)
        const char* nz_env = getenv("DMX_VGA_TVNZ");
        if (VGA_TVNZ && !wide && ftv && g->pmask.p && !(nz_env && atoi(nz_env) == 0)) {
            HIPCHK(g->tvnz.alloc((size_t)Ct * ((tvw + 63) / 64)));
            hipLaunchKernelGGL(tile_vsum_kernel, dim3((unsigned)((Ct + 3) / 4)), dim3(256), 0, s, Ct, tvw, g->tvis.p,
                               g->tvnz.p);
            HIPCHK(hipGetLastError());
        }
        g->tvw = tvw;
    }
    HIPCHK(hipStreamSynchronize(s));
    g->tiles_ready = true;
    return DMX_OK;
}

// threads of the tile BFS workgroup on grids above 4096 tiles (one workgroup per CU either way: F takes the
// LDS); A/B builds: -DVGA_NT_BIG=512
#ifndef VGA_NT_BIG
#define VGA_NT_BIG 1024
#endif
// The reference's own level order (vga_ordered.hip) for the searches the level-synchronous kernels cannot
// answer (merge links with a context-filled odd end found together with the other end at one level).
// VGA global: one search per listed source node, its level histogram into the measures kernel (rows of `outp`,
// levels into d_levels).  Visual step depth (seed_cells non-empty, PixelRef order): one search, the level of
// every cell it reaches into d_cell_level [C].
static int ordered_search(dmx_ctx* ctx, dmx_graph* g, double radius, const std::vector<int32_t>& src,
                          const std::vector<int32_t>& seed_cells, float* outp, int64_t* d_levels, int32_t* d_cell_level) {
    const PointMapHost& h = *g->pm->host;
    const int64_t C = h.cells(), N = g->nnodes;
    const bool vsd = !seed_cells.empty();
    const int64_t nsearch = vsd ? 1 : (int64_t)src.size();
    if (nsearch == 0) return DMX_OK;
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const size_t per = (size_t)C * 5 + (size_t)N * 8;   // misc, extents, two level vectors
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>({nsearch, (int64_t)ctx->num_cu,
                                                                    (int64_t)((free_b + cached_bytes()) / policy::kMemShareDiv / per)}));
    DevBuf<uint8_t> misc;
    DevBuf<int16_t> ext;
    DevBuf<int32_t> vec, d_src, d_seeds, hist, nlev;
    DevBuf<unsigned long long> junk;
    HIPCHK(misc.alloc((size_t)blocks * C));
    HIPCHK(ext.alloc((size_t)blocks * 2 * C));
    HIPCHK(vec.alloc((size_t)blocks * 2 * std::max<int64_t>(N, 1)));
    OrderedParams P;
    P.rows = h.rows(); P.C = C; P.N = N;
    P.node_run_start = g->node_run_start.p; P.node_nruns = g->node_nruns.p; P.pool = g->pool.p;
    P.cell_node = g->pm->d_cell_node.p; P.node_cell = g->pm->d_node_cell.p; P.node_flags = g->pm->d_node_flags.p;
    P.merge_cell = g->merges.empty() ? nullptr : g->d_merge_cell.p;
    P.src = nullptr; P.nsrc = 0; P.radius = (int)radius; P.hist_all = nullptr; P.nlev_all = nullptr;
    // levels kept per search: a radius r search has at most r + 2 (the cells at level r are counted, not
    // expanded); radius n as deep as the direction-optimising kernel follows (vga_do: 4096 levels)
    P.hmax = (radius == -1.0) ? 4096 : (int)std::min<double>(4096.0, radius + 2.0);
    P.seeds = nullptr; P.nseeds = 0; P.cell_level = d_cell_level;
    P.misc = misc.p; P.ext = ext.p; P.vec = vec.p;
    P.error = ctx->counters.p + 1;
    P.work_counter = ctx->counters.p + 0;
    P.ctl = ctx->d_ctl;
    ctx->h_ctl->progress = 0;
    HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 2 * sizeof(int), ctx->stream));
    if (vsd) {
        HIPCHK(d_seeds.alloc(seed_cells.size()));
        HIPCHK(hipMemcpyAsync(d_seeds.p, seed_cells.data(), seed_cells.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        P.seeds = d_seeds.p; P.nseeds = (int)seed_cells.size();
    } else {
        HIPCHK(d_src.alloc(src.size()));
        HIPCHK(hist.alloc((size_t)nsearch * P.hmax));
        HIPCHK(nlev.alloc(nsearch));
        HIPCHK(hipMemcpyAsync(d_src.p, src.data(), src.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        P.src = d_src.p; P.nsrc = (int)src.size(); P.hist_all = hist.p; P.nlev_all = nlev.p;
    }
    DevBuf<OrderedParams> dP;
    HIPCHK(dP.alloc(1));
    HIPCHK(hipMemcpyAsync(dP.p, &P, sizeof(P), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(vga_ordered_kernel, dim3((unsigned)blocks), dim3(ORD_NT), 0, ctx->stream, (const OrderedParams*)dP.p);
    HIPCHK(hipGetLastError());
    HIPCHK(wait_progress(ctx, DMX_PHASE_VGA, nsearch, 1));   // progress posts, the cancel flag
    CANCEL_POINT(ctx);
    int err = 0;
    HIPCHK(copy_sync(ctx->stream, &err, ctx->counters.p + 1, sizeof(int), hipMemcpyDeviceToHost));
    // deeper than the reference-order search keeps (the engine's own deepest search): declined, so that a
    // caller with a CPU path (integration/dmx_salalib.cpp) can take it
    if (err) return fail(DMX_ERR_UNSUPPORTED, "VGA BFS in the reference's order deeper than 4096 levels");
    if (!vsd) {
        HIPCHK(junk.alloc(32));
        hipLaunchKernelGGL(vga_measures_kernel, dim3((unsigned)((nsearch + 255) / 256)), dim3(256), 0, ctx->stream,
                           (int64_t)0, nsearch, hist.p, nlev.p, outp, d_levels, junk.p, (const int32_t*)d_src.p, P.hmax, true);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    VLOG("reference-order searches: %lld on %lld workgroups\n", (long long)nsearch, (long long)blocks);
    return DMX_OK;
}

// The sources a level-synchronous kernel marked in d_oflag, run again in the reference's order.
static int vga_order_rerun(dmx_ctx* ctx, dmx_graph* g, double radius, const uint8_t* d_oflag, float* outp,
                           int64_t* d_levels) {
    const int64_t N = g->nnodes;
    std::vector<uint8_t> fl((size_t)N);
    HIPCHK(copy_sync(ctx->stream, fl.data(), d_oflag, (size_t)N, hipMemcpyDeviceToHost));
    std::vector<int32_t> src;
    for (int64_t k = 0; k < N; k++)
        if (fl[k]) src.push_back((int32_t)k);
    const double t0 = now_s();
    int rc = ordered_search(ctx, g, radius, src, {}, outp, d_levels, nullptr);
    ctx->last_vga_s += now_s() - t0;
    ctx->last_stats[38] = (int64_t)src.size();
    return rc;
}

extern "C++" template <int NT, bool SPECIAL, bool RBM, bool FG>
static int launch_tile(dmx_ctx* ctx, const VgaTileParams& Q, int64_t nsrc, size_t lds, int64_t* blocks_out,
                       DevBuf<unsigned long long>& xg, DevBuf<int4>& queue, DevBuf<int32_t>& list) {
    // The shapes the kernel and its grid assume, checked before the launch: a tile grid that covers
    // the cells, the frontier (FG false) and the summaries inside the dynamic LDS, row words the fused phase-C
    // test covers (4 a lane: 256), the 32-bit narrow hint's tile (15 bits) and mask slot (16 bits; a cell's
    // partial tiles are at most nt), the asymmetric-mode list capacity.
    {
        const int64_t nt = (int64_t)Q.tw * Q.th;
        const char* why = nullptr;
        if (Q.tw != (Q.cols + 7) / 8 || Q.th != (Q.rows + 7) / 8 || nt <= 0) why = "tile grid does not cover the cells";
        else if (lds > (size_t)160 * 1024) why = "dynamic LDS above 160 KiB";
        else if (!FG && (size_t)nt * 8 > lds) why = "frontier bitmap larger than the dynamic LDS";
        else if (Q.tvis && Q.tvw != Q.th * ((Q.tw + 63) / 64)) why = "tile-visibility row width differs from the tile grid";
        else if (!FG && Q.pmask && Q.tvw > 256) why = "row words past the fused phase-C test (256)";
        else if (Q.tvnz && (FG || Q.tvw > 256)) why = "narrow row summaries on a wide grid";
        else if (Q.pmask && !FG && nt > 32767) why = "narrow mask hint: tile index above 15 bits";
        else if (Q.asym_tiles && Q.alist_cap <= 0) why = "asymmetric mode without an A-cell list";
        if (why) return fail(DMX_ERR_STATE, (std::string("VGA tile launch: ") + why).c_str());
    }
    int occ = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vga_tile_kernel<NT, SPECIAL, RBM, FG>, NT, lds));
    if (occ < 1) occ = 1;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((int64_t)ctx->num_cu * occ, nsrc));
    const int64_t nt = (int64_t)Q.tw * Q.th;
    HIPCHK(xg.alloc((size_t)blocks * (FG ? 3 : 2) * nt));   // V, X [, F]
    HIPCHK(queue.alloc((size_t)blocks * nt));
    HIPCHK(list.alloc((size_t)blocks * nt * 64 * 2));
    DevBuf<int32_t> tlist;   // per workgroup: the two unvisited-tile lists
    HIPCHK(tlist.alloc((size_t)blocks * nt * 2));
    DevBuf<uint32_t> hint;
    HIPCHK(hint.alloc((size_t)nt * 64));
    HIPCHK(hipMemsetAsync(hint.p, 0xFF, (size_t)nt * 64 * 4, ctx->stream));
    DevBuf<uint32_t> hint2;   // (narrow grids with the masks) the second, fully-seen-tile hint
    DevBuf<int32_t> mseen;   // per workgroup: merge_order_check stamps
    DevBuf<int32_t> alist;   // asymmetric mode: per workgroup, the frontier's A cells
    VgaTileParams P = Q;
    P.hint2 = nullptr;
    if (VGA_H2 > 0 && Q.pmask && !FG && !getenv("DMX_VGA_NOHINT2")) {
        HIPCHK(hint2.alloc((size_t)nt * 64 * VGA_H2));
        HIPCHK(hipMemsetAsync(hint2.p, 0xFF, (size_t)nt * 64 * 4 * VGA_H2, ctx->stream));
        P.hint2 = hint2.p;
    }
    if (Q.asym_tiles) {
        HIPCHK(alist.alloc((size_t)blocks * Q.alist_cap));
        P.alist = alist.p;
    }
    P.fg = FG ? xg.p + (size_t)blocks * 2 * nt : nullptr;   // per workgroup [nt] after every V / X pair
    if (Q.nmamb) {
        HIPCHK(mseen.alloc((size_t)blocks * Q.nmamb));
        HIPCHK(hipMemsetAsync(mseen.p, 0, (size_t)blocks * Q.nmamb * 4, ctx->stream));
        P.mseen = mseen.p;
    }
    P.xg = xg.p;
    P.queue = queue.p;
    P.list = list.p;
    P.tlist = tlist.p;
    P.hint = hint.p;
    DevBuf<unsigned long long> hintw;   // (wide grids with the masks) mask hints
    P.hintw = nullptr;
    if (P.pmask && P.tvsum) {
        HIPCHK(hintw.alloc((size_t)nt * 64));
        HIPCHK(hipMemsetAsync(hintw.p, 0, (size_t)nt * 64 * 8, ctx->stream));
        P.hintw = hintw.p;
    }
    // chunks of consecutive sources per workgroup, small enough to balance the tail
    // concurrent workgroups on neighbouring sources share L2 lines and hints
    P.chunk = std::max(1, policy::hook_int("DMX_VGA_CHUNK", policy::kVgaSourceChunk));
    P.nwork = (int)((P.src_end - P.src_begin + P.chunk - 1) / P.chunk);
    HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
    P.ctl = ctx->d_ctl;
    ctx->h_ctl->progress = 0;
    DevBuf<VgaTileParams> dP;
    HIPCHK(dP.alloc(1));
    HIPCHK(hipMemcpyAsync(dP.p, &P, sizeof(P), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL((vga_tile_kernel<NT, SPECIAL, RBM, FG>), dim3((unsigned)blocks), dim3(NT), lds, ctx->stream,
                       (const VgaTileParams*)dP.p);
    HIPCHK(hipGetLastError());
    HIPCHK(wait_progress(ctx, DMX_PHASE_VGA, nsrc, P.chunk));   // hint freed on return
    *blocks_out = blocks;
    return DMX_OK;
}

static int vga_tile_impl(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se, float* out,
                         bool out_on_device, int64_t* levels, int tw, int th, const int32_t* d_seeds = nullptr,
                         int nseeds = 0, int32_t* d_cell_level = nullptr, const int32_t* d_src_list = nullptr,
                         dmx_graph* pg = nullptr) {
    // pg (asymmetric mode): the graph analysed; g is its symmetric reference (prepare_asym)
    int rc = prepare_tiles(g);
    if (rc) return rc;
    PointMapHost& h = *g->pm->host;
    const int64_t N = g->nnodes, nsrc = se - sb;
    const int nt = tw * th;
    const int maxlev = 1024;
    DevBuf<float> d_out;
    float* outp = out;
    if (!out_on_device) {
        HIPCHK(d_out.alloc(std::max<int64_t>(N, 1) * 7));
        outp = d_out.p;
    }
    DevBuf<int64_t> d_lv;
    if (levels) HIPCHK(d_lv.alloc(std::max<int64_t>(N, 1) * 3));
    HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 16 * sizeof(int), ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->stats.p, 0, 32 * sizeof(unsigned long long), ctx->stream));
    VgaTileParams Q;
    Q.cols = h.cols(); Q.rows = h.rows(); Q.tw = tw; Q.th = th;
    Q.seed_tiles = g->notuf_tiles.p; Q.regular_tiles = g->regular_tiles.p; Q.nonexp_tiles = g->pm->d_nonexp_tiles.p;
    Q.cr = g->cr.p; Q.heads = g->heads.p; Q.tscan_start = g->tscan_start.p; Q.tnruns = g->tnruns.p;
    Q.scan_pool = g->scan_released ? g->pool.p : g->scan_pool.p;   // (tscan_start then indexes the pool)
    Q.tvis = g->tvw ? g->tvis.p : nullptr; Q.tvw = g->tvw;
    Q.tvsum = (g->tvw && g->tvsum.p) ? g->tvsum.p : nullptr;
    Q.tvnz = (g->tvw && g->tvnz.p) ? g->tvnz.p : nullptr;
    Q.ftvis = (g->tvw && g->ftvis.p) ? g->ftvis.p : nullptr;
    Q.ttvis = (g->tvw && g->ttvis.p) ? g->ttvis.p : nullptr;
    Q.ttany = Q.ttvis ? g->ttvis.p + (size_t)tw * th * g->tvw : nullptr;
    const char* pmk_env = getenv("DMX_VGA_PMASK");   // also a launch-time switch (the masks stay built), except
    // where the masks replaced the scan order (phase C's scan of the regular cells reads the scan order)
    Q.pmask = (Q.ftvis && g->pmask.p && (g->scan_released || !(pmk_env && atoi(pmk_env) == 0))) ? g->pmask.p : nullptr;
    Q.poff = Q.pmask ? g->poff.p : nullptr;
    Q.ppre = Q.pmask ? g->ppre.p : nullptr;
    Q.node_cell = g->pm->d_node_cell.p; Q.cell_node = g->pm->d_cell_node.p; Q.node_flags = g->pm->d_node_flags.p;
    Q.node_run_start = g->node_run_start.p; Q.node_nruns = g->node_nruns.p; Q.pool = g->pool.p;
    const bool corr = g->nspecial > 0;
    Q.spec_index = corr ? g->spec_index.p : nullptr;
    Q.extra_off = corr ? g->extra_off.p : nullptr;
    Q.extra = corr ? g->extra.p : nullptr;
    Q.missing_off = corr ? g->missing_off.p : nullptr;
    Q.missing = corr ? g->missing.p : nullptr;
    Q.src_begin = sb; Q.src_end = se; Q.radius = (int)radius; Q.gates_only = gates_only;
    Q.uf_count = g->uf_count;
    Q.seeds = d_seeds; Q.nseeds = nseeds; Q.cell_level = d_cell_level;
    Q.nmp = (int)(g->merges.size() / 2);
    Q.mpairs = Q.nmp ? g->d_mpairs.p : nullptr;
    Q.nmamb = Q.nmp && radius != -1.0 ? g->nmamb : 0;
    Q.mamb = Q.nmamb ? g->d_mamb.p : nullptr;
    Q.mseen = nullptr;
    DevBuf<uint8_t> oflag;   // sources whose result depends on the reference's pop order (merge_order_check)
    Q.oflag = nullptr;
    if (Q.nmamb) {
        HIPCHK(oflag.alloc(std::max<int64_t>(N, 1)));
        HIPCHK(hipMemsetAsync(oflag.p, 0, (size_t)std::max<int64_t>(N, 1), ctx->stream));
        Q.oflag = oflag.p;
    }
    Q.src_list = d_src_list;   // [sb, se) index this list of source nodes (out must be on the device)
    Q.asym_tiles = nullptr; Q.asym_uf = nullptr; Q.apool = nullptr; Q.arun_start = nullptr; Q.anruns = nullptr;
    Q.alist = nullptr; Q.alist_cap = 0;
    if (pg) {   // asymmetric mode: pg's own universe (pre-visited cells, early-exit count) and runs for A's pushes
        Q.seed_tiles = pg->notuf_tiles.p;
        Q.uf_count = pg->uf_count;
        Q.asym_tiles = pg->asym_tiles.p;
        Q.asym_uf = g->uf_tiles.p;
        Q.apool = pg->pool.p; Q.arun_start = pg->node_run_start.p; Q.anruns = pg->node_nruns.p;
        Q.alist_cap = (int)std::max<int64_t>(pg->nasym, 1);
    }
    // Beamer's direction test on cell counts (top-down levels run on the LDS frontier bitmap)
    // top-down costs a frontier cell its whole run list (~R/N runs): keep it rare
    Q.alpha = policy::hook_int("DMX_VGA_ALPHA", policy::kVgaTileAlpha);
    Q.bext = BEXT_DEFAULT;
    if (const char* b = getenv("DMX_VGA_BEXT")) Q.bext = std::max(0, atoi(b));
    Q.crk = std::min(CRK, std::max(0, policy::hook_int("DMX_VGA_CRK", policy::kVgaTileCommonRuns)));
    Q.work_counter = ctx->counters.p + 0; Q.error = ctx->counters.p + 1;
    DevBuf<int32_t> d_hist, d_nlev;
    HIPCHK(d_hist.alloc((size_t)std::max<int64_t>(N, 1) * VGA_HMAX));
    HIPCHK(d_nlev.alloc(std::max<int64_t>(N, 1)));
    Q.maxlev = maxlev; Q.hist_out = d_hist.p; Q.nlev_out = d_nlev.p; Q.stats = ctx->stats.p;
    bool fg = false, rbm = false;
    const size_t L = tile_lds_layout(tw, th, &fg, &rbm);
    if (!L) return fail(DMX_ERR_CAPACITY, "grid too large for the tile BFS's LDS summaries");
    // With the frontier in HBM a top-down level's run rasterisation takes global atomics: past level 1 the
    // bottom-up levels win (2000^2 interior block: alpha 60 -> 200: 2.70 -> 2.28 s, identical output;
    // 1000 and 100000 the same, profiles/r5_vga2000_alpha.jsonl)
    if (fg && !policy::hook("DMX_VGA_ALPHA")) Q.alpha = policy::kVgaTileAlphaHbm;
    DevBuf<unsigned long long> xg;
    DevBuf<int4> queue;
    DevBuf<int32_t> list;
    int64_t blocks = 0;
    int kt = 0, ntpb = 0;
    (void)kt;
    if (nsrc > 0) {
        const bool sp = g->nspecial > 0;
        if (fg) {
            rc = sp ? (rbm ? launch_tile<1024, true, true, true>(ctx, Q, nsrc, L, &blocks, xg, queue, list)
                           : launch_tile<1024, true, false, true>(ctx, Q, nsrc, L, &blocks, xg, queue, list))
                    : (rbm ? launch_tile<1024, false, true, true>(ctx, Q, nsrc, L, &blocks, xg, queue, list)
                           : launch_tile<1024, false, false, true>(ctx, Q, nsrc, L, &blocks, xg, queue, list));
            ntpb = 1024;
        } else if (nt <= 4096) {
            rc = sp ? (rbm ? launch_tile<256, true, true, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list)
                           : launch_tile<256, true, false, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list))
                    : (rbm ? launch_tile<256, false, true, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list)
                           : launch_tile<256, false, false, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list));
            ntpb = 256;
        } else {
            rc = sp ? (rbm ? launch_tile<VGA_NT_BIG, true, true, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list)
                           : launch_tile<VGA_NT_BIG, true, false, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list))
                    : (rbm ? launch_tile<VGA_NT_BIG, false, true, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list)
                           : launch_tile<VGA_NT_BIG, false, false, false>(ctx, Q, nsrc, L, &blocks, xg, queue, list));
            ntpb = VGA_NT_BIG;
        }
        if (rc) return rc;
        CANCEL_POINT(ctx);
        if (nseeds == 0) {
            hipLaunchKernelGGL(vga_measures_kernel, dim3((unsigned)((nsrc + 255) / 256)), dim3(256), 0, ctx->stream, sb,
                               se, d_hist.p, d_nlev.p, outp, levels ? d_lv.p : nullptr, ctx->stats.p, d_src_list);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
    } else {
        HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
        HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last_vga_s = ms * 1e-3;
    int hc[2];
    HIPCHK(copy_sync(ctx->stream, hc, ctx->counters.p, sizeof(hc), hipMemcpyDeviceToHost));
    if (hc[1] & ~KERR_ORDER) return fail(DMX_ERR_CAPACITY, "VGA BFS exceeded its level capacity");
    ctx->last_stats[38] = 0;
    if ((hc[1] & KERR_ORDER) && nseeds == 0)
        if (int rc2 = vga_order_rerun(ctx, g, radius, oflag.p, outp, levels ? d_lv.p : nullptr)) return rc2;
    unsigned long long st[32];
    HIPCHK(copy_sync(ctx->stream, st, ctx->stats.p, sizeof(st), hipMemcpyDeviceToHost));
    for (int i = 0; i < 5; i++) ctx->phase_cycles[i] = (long long)st[8 + i];
    ctx->last_stats[18] = (long long)st[16];                          // phase-C hits by a fully seen tile
    ctx->last_stats[19] = (long long)st[17];                          // clocks of top-down levels > 1
    ctx->last_stats[20] = (long long)st[18];                          // phase-B tiles
    ctx->last_stats[21] = (long long)st[19];                          // phase-B cells
    ctx->last_stats[22] = (long long)st[20];                          // phase-B tiles resolved by ttvis
    ctx->last_stats[27] = (long long)st[25];                          // phase-B tiles pruned by ttany
    ctx->last_stats[28] = (long long)st[26];                          // phase-B row-test clocks (not collected: 0)
    ctx->last_stats[29] = (long long)st[27];                          // phase-B tiles with cell tests
    ctx->last_stats[30] = (long long)st[28];                          // phase-B cell-test clocks (not collected: 0)
    ctx->last_stats[31] = (long long)st[29];                          // phase-B cells past hint + 4 heads
    ctx->last_stats[23] = (long long)st[21];                          // phase-C busy clocks summed over waves
    ctx->last_stats[24] = (long long)st[22];                          // phase-C per-cell clocks (not collected: 0)
    ctx->last_stats[25] = (long long)st[23];                          // phase-C special-node clocks (not collected: 0)
    ctx->last_stats[26] = (long long)st[24];                          // phase-C special-node tests
    ctx->last_stats[3] = 3 | ((long long)g->nspecial << 8);
    ctx->last_stats[4] = (long long)st[0];
    ctx->last_stats[5] = (long long)(st[3] | (st[4] << 32));
    ctx->last_stats[6] = (long long)st[2];
    ctx->last_stats[7] = nsrc;
    ctx->last_stats[8] = (long long)st[5];
    ctx->last_stats[9] = (long long)st[6];
    ctx->last_stats[10] = 0;
    ctx->last_stats[11] = (long long)st[7];
    ctx->last_stats[12] = blocks | ((long long)kt << 32) | ((long long)ntpb << 40) | ((long long)fg << 56);
    ctx->last_stats[13] = (long long)st[13];
    ctx->last_stats[14] = (long long)st[14] * g->tvw * 8;   // bytes of tile-visibility rows read
    ctx->last_stats[15] = (long long)st[15];                          // runs scanned in phase C
    ctx->last_stats[16] = (long long)st[1];                           // phase-C cells that hit
    ctx->last_stats[17] = (long long)st[14];                          // phase-C cells (regular)
    ctx->last_stats[35] = (long long)st[30];                          // phase-C partial-tile masks read
    ctx->last_stats[36] = (long long)st[31];                          // phase-C cells tested by masks
    ctx->last_stats[37] = (long long)(g->pmask.p ? g->pmask.n * 8 : 0);  // bytes of partial-tile masks held
    prep_state_stats(ctx, g);
    if (pg) {   // asymmetric mode (bit 7) and |A|
        ctx->last_stats[40] |= 128;
        ctx->last_stats[43] = pg->nasym;
    }
    if (nseeds > 0) return DMX_OK;
    if (!out_on_device && nsrc > 0)
        HIPCHK(copy_sync(ctx->stream, out + sb * 7, d_out.p + sb * 7, nsrc * 7 * 4, hipMemcpyDeviceToHost));
    if (levels && nsrc > 0)
        HIPCHK(copy_sync(ctx->stream, levels + sb * 3, d_lv.p + sb * 3, nsrc * 3 * 8, hipMemcpyDeviceToHost));
    return DMX_OK;
}

// Asymmetric mode (vga_tile.hip): a graph whose runs are not symmetric at scale -- a map re-read from a .graph file,
// where PixelVec's 4-bit row shift (ngraph.cpp:536-583) moved the runs after a jump of more than 15 rows and a bin
// of 65536 k cells lost its runs (Bin::write's unsigned short count) -- has almost every node asymmetric, beyond
// the in-set correction lists.  Made again from the drawing, the map's graph R is symmetric but for a few nodes;
// A = the nodes whose runs differ between the graph and R, plus R's asymmetric nodes.  Every edge between two
// nodes outside A is in both graphs and in both directions, so the search runs bottom-up on R with the frontier
// limited to cells outside A, and the A cells of each frontier push the graph's own runs top-down.  Needs the
// drawing (dmx_graph_set_drawing), the whole graph, no merge links, R on the same grid and |A| <= N/4.
static int prepare_asym(dmx_ctx* ctx, dmx_graph* g) {
    if (g->asym_state) return g->asym_state > 0 ? DMX_OK : DMX_ERR_UNSUPPORTED;
    g->asym_state = -1;
    if (!g->has_drawing) { g->asym_why = "no drawing"; return DMX_ERR_UNSUPPORTED; }
    if (!g->merges.empty()) { g->asym_why = "merge links"; return DMX_ERR_UNSUPPORTED; }
    if (g->node_begin != 0 || g->node_end != g->nnodes) { g->asym_why = "a shard"; return DMX_ERR_UNSUPPORTED; }
    const PointMapHost& h = *g->pm->host;
    std::unique_ptr<dmx_pointmap> pm(new dmx_pointmap());
    pm->host.reset(new PointMapHost(h.parent_region(), h.spacing(), g->drawing.data(), (int64_t)g->drawing.size() / 4));
    PointMapHost& hr = *pm->host;
    if (hr.cols() != h.cols() || hr.rows() != h.rows() || hr.bottom_left().x != h.bottom_left().x ||
        hr.bottom_left().y != h.bottom_left().y) {
        g->asym_why = "the drawing's grid differs from the map's";
        return DMX_ERR_UNSUPPORTED;
    }
    hr.block_lines();
    hr.restore_fill(h.state().data());
    pm->version++;
    const double t0 = now_s();
    // (makeGraph's timing and counters are the reference graph's from here on)
    dmx_graph* r = nullptr;
    if (int rc = makegraph_impl(ctx, pm.get(), -1.0, 0, 0, -1, nullptr, nullptr, &r)) {
        g->asym_why = "makeGraph of the reference failed";
        return rc;
    }
    std::unique_ptr<dmx_graph> R(r);
    if (R->nnodes != g->nnodes) { g->asym_why = "the reference has other nodes"; return DMX_ERR_UNSUPPORTED; }
    if (int rc = prepare_uf(R.get())) return rc;
    if (int rc = prepare_symmetry(R.get())) return rc;
    if (R->symmetric != 1) { g->asym_why = "the reference is not symmetric enough"; return DMX_ERR_UNSUPPORTED; }
    const int64_t N = g->nnodes;
    DevBuf<uint8_t> d_flag;
    HIPCHK(d_flag.alloc(std::max<int64_t>(N, 1)));
    if (N) {
        hipLaunchKernelGGL(node_runs_differ_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, ctx->stream, N,
                           g->bin_nruns.p, g->node_run_start.p, g->node_nruns.p, g->pool.p, R->bin_nruns.p,
                           R->node_run_start.p, R->node_nruns.p, R->pool.p, d_flag.p);
        HIPCHK(hipGetLastError());
    }
    std::vector<uint8_t> flag((size_t)std::max<int64_t>(N, 1));
    HIPCHK(copy_sync(ctx->stream, flag.data(), d_flag.p, (size_t)N, hipMemcpyDeviceToHost));
    for (int32_t k : R->special_nodes) flag[k] = 1;
    const int tw = (h.cols() + 7) / 8, th = (h.rows() + 7) / 8;
    std::vector<unsigned long long> at((size_t)tw * th, 0ull);
    int64_t na = 0;
    for (int64_t k = 0; k < N; k++)
        if (flag[k]) {
            const int c = g->pm->node_cell[k], x = c / h.rows(), y = c % h.rows();
            at[(size_t)(y >> 3) * tw + (x >> 3)] |= 1ull << ((y & 7) * 8 + (x & 7));
            na++;
        }
    if (na > N / 4) { g->asym_why = "too many nodes differ from the reference"; return DMX_ERR_UNSUPPORTED; }
    HIPCHK(g->asym_tiles.alloc(at.size()));
    HIPCHK(copy_sync(ctx->stream, g->asym_tiles.p, at.data(), at.size() * 8, hipMemcpyHostToDevice));
    g->nasym = na;
    g->aref = std::move(R);
    g->aref_pm = std::move(pm);
    g->asym_state = 1;
    VLOG("asymmetric mode: reference graph %.2f s, %lld of %lld nodes differ (%zu asymmetric in the reference)\n",
         now_s() - t0, (long long)na, (long long)N, g->aref->special_nodes.size());
    return DMX_OK;
}

int dmx_graph_set_drawing(dmx_graph* g, const double* lines, int64_t nlines) {
    if (!g || nlines < 0 || (nlines > 0 && !lines)) return fail(DMX_ERR_ARG, "bad arguments");
    g->drawing.assign(lines, lines + 4 * nlines);
    g->has_drawing = true;
    g->asym_state = 0;
    g->aref.reset();
    g->aref_pm.reset();
    g->asym_tiles.reset();
    return DMX_OK;
}

static int vga_impl(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se, float* out,
                    bool out_on_device, int64_t* levels) {
    if (!ctx || !g || !out) return fail(DMX_ERR_ARG, "bad arguments");
    if (g->node_begin != 0 || g->node_end != g->nnodes)
        return fail(DMX_ERR_STATE, "VGA needs the whole graph (assemble the shards first)");
    HIPCHK(hipSetDevice(ctx->device));
    const int64_t N = g->nnodes;
    if (se < 0 || se > N) se = N;
    if (sb < 0 || sb > se) return fail(DMX_ERR_ARG, "bad source range");
    int rc = prepare_uf(g);
    if (rc) return rc;
    rc = prepare_symmetry(g);
    if (rc) return rc;
    ctx->last_stats[40] = 0;   // (the tile search sets its preparation flags; the other searches leave none)
    ctx->last_stats[43] = 0;
    PointMapHost& h = *g->pm->host;
    const int tw = (h.cols() + 7) / 8, th = (h.rows() + 7) / 8;
    const int maxlev = 4096;
    {
        const char* fk = getenv("DMX_VGA_KERNEL");
        const bool forced_other = fk && (std::string(fk) == "v1" || std::string(fk) == "do" || std::string(fk) == "topdown");
        const int nt = tw * th;
        // DMX_VGA_ASYM (test hook): the asymmetric mode also for a graph whose few asymmetric nodes the in-set
        // correction lists handle (small re-read maps), so that both exact paths can be compared
        const bool force_asym = getenv("DMX_VGA_ASYM") && g->has_drawing && g->symmetric == 1 && g->nspecial > 0;
        if (!forced_other && g->symmetric == 1 && !ctx->tile_disabled && !force_asym) {
            int rc2 = vga_tile_impl(ctx, g, radius, gates_only, sb, se, out, out_on_device, levels, tw, th);
            if (rc2 != DMX_ERR_CAPACITY) return rc2;   // capacity (level histogram): retry with vga_do
        } else if (!forced_other && (g->symmetric == 0 || force_asym) && !ctx->tile_disabled && !getenv("DMX_VGA_NOASYM") &&
                   prepare_asym(ctx, g) == DMX_OK) {
            // asymmetric at scale (a re-read .graph): the tile search on the reference graph, A pushing its own runs
            int rc2 = vga_tile_impl(ctx, g->aref.get(), radius, gates_only, sb, se, out, out_on_device, levels, tw, th,
                                    nullptr, 0, nullptr, nullptr, g);
            if (rc2 != DMX_ERR_CAPACITY) return rc2;
        }
    }
    if (int rc3 = restore_scan_order(g)) return rc3;   // (vga_do reads the scan order)
    const size_t lds_do = (size_t)tw * th * 8 * 3 + (maxlev + 4) * 4 + 64;
    const char* force = getenv("DMX_VGA_KERNEL");
    const bool want_v1 = force && std::string(force) == "v1";
    const bool gbm = !want_v1 && lds_do > 160 * 1024;   // bitmaps in HBM
    const bool use_do = !want_v1;
    const size_t lds = gbm ? (size_t)(maxlev + 4) * 4 + 64 : use_do ? lds_do : (size_t)tw * th * 8 + (maxlev + 4) * 4 + 64;
    if (lds > 160 * 1024) return fail(DMX_ERR_UNSUPPORTED, "grid too large for the LDS visited bitmap (v1 limit)");
    int occ = 0;
    if (gbm) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vga_do_kernel<true>, DO_THREADS, lds));
    else if (use_do) HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vga_do_kernel<false>, DO_THREADS, lds));
    else HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vga_global_kernel, VGA_THREADS, lds));
    if (occ < 1) occ = 1;
    const int64_t nsrc = se - sb;
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((int64_t)ctx->num_cu * occ, nsrc));
    DevBuf<int32_t> frontier;
    HIPCHK(frontier.alloc((size_t)blocks * 2 * std::max<int64_t>(N, 1)));
    DevBuf<unsigned long long> gbm_buf;
    if (gbm) HIPCHK(gbm_buf.alloc((size_t)blocks * 3 * tw * th));
    DevBuf<float> d_out;
    float* outp = out;
    if (!out_on_device) {
        HIPCHK(d_out.alloc(std::max<int64_t>(N, 1) * 7));
        outp = d_out.p;
    }
    DevBuf<int64_t> d_lv;
    if (levels) HIPCHK(d_lv.alloc(std::max<int64_t>(N, 1) * 3));
    HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 16 * sizeof(int), ctx->stream));
    HIPCHK(hipMemsetAsync(ctx->stats.p, 0, 32 * sizeof(unsigned long long), ctx->stream));
    VgaParams P;
    P.cols = h.cols(); P.rows = h.rows(); P.tw = tw; P.th = th;
    P.seed_tiles = g->pm->d_seed_tiles.p; P.uf_tiles = g->uf_tiles.p; P.uf_count = g->uf_count;
    P.node_cell = g->pm->d_node_cell.p; P.cell_node = g->pm->d_cell_node.p; P.node_flags = g->pm->d_node_flags.p;
    P.node_run_start = g->node_run_start.p; P.node_nruns = g->node_nruns.p; P.pool = g->pool.p;
    P.src_begin = sb; P.src_end = se; P.radius = (int)radius; P.gates_only = gates_only;
    P.work_counter = ctx->counters.p + 0; P.error = ctx->counters.p + 1;
    P.frontier = frontier.p; P.nnodes = N; P.maxlev = maxlev;
    P.out = outp; P.levels_out = levels ? d_lv.p : nullptr;
    P.stats = ctx->stats.p;
    VgaDoParams Q;
    Q.cols = h.cols(); Q.rows = h.rows(); Q.tw = tw; Q.th = th;
    Q.seed_tiles = g->notuf_tiles.p; Q.uf_tiles = g->uf_tiles.p; Q.nonexp_tiles = g->pm->d_nonexp_tiles.p;
    Q.node_cell = P.node_cell; Q.cell_node = P.cell_node; Q.node_flags = P.node_flags;
    Q.node_run_start = P.node_run_start; Q.node_nruns = P.node_nruns; Q.pool = P.pool;
    Q.cell_scan_start = g->cell_scan_start.p; Q.cell_nruns = g->cell_nruns.p; Q.scan_pool = g->scan_pool.p;
    Q.src_begin = sb; Q.src_end = se; Q.radius = P.radius; Q.gates_only = gates_only;
    Q.uf_count = g->uf_count; Q.symmetric = g->symmetric;
    const bool corr = g->symmetric == 1 && g->nspecial > 0;
    Q.spec_index = corr ? g->spec_index.p : nullptr;
    Q.extra_off = corr ? g->extra_off.p : nullptr;
    Q.extra = corr ? g->extra.p : nullptr;
    Q.missing_off = corr ? g->missing_off.p : nullptr;
    Q.missing = corr ? g->missing.p : nullptr;
    Q.alpha = policy::hook_int("DMX_VGA_ALPHA", policy::kVgaDoAlpha);
    Q.kshort = policy::hook_int("DMX_VGA_KSHORT", policy::kVgaDoShortList);
    Q.work_counter = P.work_counter; Q.scratch = frontier.p; Q.nnodes = N; Q.maxlev = maxlev;
    Q.out = outp; Q.levels_out = P.levels_out; Q.error = P.error; Q.stats = P.stats;
    Q.gbm = gbm ? gbm_buf.p : nullptr;
    Q.nmp = (int)(g->merges.size() / 2);
    Q.mpairs = Q.nmp ? g->d_mpairs.p : nullptr;
    if (!use_do && Q.nmp) return fail(DMX_ERR_UNSUPPORTED, "the top-down v1 kernel does not follow merge links");
    Q.nmamb = Q.nmp && radius != -1.0 ? g->nmamb : 0;
    Q.mamb = Q.nmamb ? g->d_mamb.p : nullptr;
    DevBuf<int32_t> mseen;
    DevBuf<uint8_t> oflag;
    if (Q.nmamb) {
        HIPCHK(mseen.alloc((size_t)blocks * Q.nmamb));
        HIPCHK(hipMemsetAsync(mseen.p, 0, (size_t)blocks * Q.nmamb * 4, ctx->stream));
        Q.mseen = mseen.p;
        HIPCHK(oflag.alloc(N));
        HIPCHK(hipMemsetAsync(oflag.p, 0, (size_t)N, ctx->stream));
        Q.oflag = oflag.p;
    }
    HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
    if (nsrc > 0) {
        if (gbm) hipLaunchKernelGGL(vga_do_kernel<true>, dim3((unsigned)blocks), dim3(DO_THREADS), lds, ctx->stream, Q);
        else if (use_do) hipLaunchKernelGGL(vga_do_kernel<false>, dim3((unsigned)blocks), dim3(DO_THREADS), lds, ctx->stream, Q);
        else hipLaunchKernelGGL(vga_global_kernel, dim3((unsigned)blocks), dim3(VGA_THREADS), lds, ctx->stream, P);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
    ctx->h_ctl->progress = 0;   // these kernels do not poll: a cancel takes effect when they finish
    HIPCHK(wait_progress(ctx, DMX_PHASE_VGA, nsrc, 1));
    CANCEL_POINT(ctx);
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->last_vga_s = ms * 1e-3;
    int hc[2];
    HIPCHK(copy_sync(ctx->stream, hc, ctx->counters.p, sizeof(hc), hipMemcpyDeviceToHost));
    if (hc[1] & ~KERR_ORDER) return fail(DMX_ERR_CAPACITY, "VGA BFS exceeded its level/frontier capacity");
    ctx->last_stats[38] = 0;
    if (hc[1] & KERR_ORDER)
        if (int rc2 = vga_order_rerun(ctx, g, radius, oflag.p, outp, P.levels_out)) return rc2;
    unsigned long long st[8];
    HIPCHK(copy_sync(ctx->stream, st, ctx->stats.p, sizeof(st), hipMemcpyDeviceToHost));
    ctx->last_stats[8] = (long long)st[5];   // bottom-up cells that scanned all their runs without a hit
    ctx->last_stats[9] = (long long)st[6];   // runs read by those
    ctx->last_stats[10] = gbm ? 1 : 0;
    for (int i = 13; i < 24; i++) ctx->last_stats[i] = 0;
    ctx->last_stats[3] = (long long)(use_do ? (g->symmetric ? 2 : 1) : 0) | ((long long)g->nspecial << 8);
    ctx->last_stats[4] = (long long)st[0];
    ctx->last_stats[5] = (long long)(st[3] | (st[4] << 32));                 // bottom-up | top-down levels
    ctx->last_stats[6] = (long long)st[2];
    ctx->last_stats[7] = nsrc;
    if (!out_on_device && nsrc > 0)
        HIPCHK(copy_sync(ctx->stream, out + sb * 7, d_out.p + sb * 7, nsrc * 7 * 4, hipMemcpyDeviceToHost));
    if (levels && nsrc > 0)
        HIPCHK(copy_sync(ctx->stream, levels + sb * 3, d_lv.p + sb * 3, nsrc * 3 * 8, hipMemcpyDeviceToHost));
    return DMX_OK;
}

int dmx_vga_global(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se, float* out,
                   int64_t* levels) {
    SAME_DEVICE(ctx, g);
    if (int rc = prepare_merges(g)) return rc;
    return vga_impl(ctx, g, radius, gates_only, sb, se, out, false, levels);
}

int dmx_vga_global_device(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t sb, int64_t se,
                          float* out_device) {
    SAME_DEVICE(ctx, g);
    if (int rc = prepare_merges(g)) return rc;
    return vga_impl(ctx, g, radius, gates_only, sb, se, out_device, true, nullptr);
}

// VGA global for an arbitrary set of source nodes (multi-GPU shards interleaved over the grid so that
// every rank gets the same mix of cheap and expensive sources).  The tile-resolved BFS takes the list
// in one launch; otherwise runs of consecutive nodes go through vga_impl one by one.
int dmx_vga_global_device_list(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, const int64_t* nodes,
                               int64_t n, float* out_device) {
    SAME_DEVICE(ctx, g);
    if (!ctx || !g || !out_device || (n > 0 && !nodes)) return fail(DMX_ERR_ARG, "bad arguments");
    if (int rc = prepare_merges(g)) return rc;
    if (g->node_begin != 0 || g->node_end != g->nnodes)
        return fail(DMX_ERR_STATE, "VGA needs the whole graph (assemble the shards first)");
    HIPCHK(hipSetDevice(ctx->device));
    const int64_t N = g->nnodes;
    std::vector<int32_t> lst((size_t)std::max<int64_t>(n, 1));
    for (int64_t i = 0; i < n; i++) {
        if (nodes[i] < 0 || nodes[i] >= N) return fail(DMX_ERR_ARG, "source node out of range");
        lst[i] = (int32_t)nodes[i];
    }
    int rc = prepare_uf(g);
    if (rc) return rc;
    rc = prepare_symmetry(g);
    if (rc) return rc;
    PointMapHost& h = *g->pm->host;
    const int tw = (h.cols() + 7) / 8, th = (h.rows() + 7) / 8;
    if (g->symmetric == 1 && !ctx->tile_disabled) {
        DevBuf<int32_t> d_list;
        HIPCHK(d_list.alloc(lst.size()));
        HIPCHK(hipMemcpyAsync(d_list.p, lst.data(), lst.size() * 4, hipMemcpyHostToDevice, ctx->stream));
        rc = vga_tile_impl(ctx, g, radius, gates_only, 0, n, out_device, true, nullptr, tw, th, nullptr, 0, nullptr, d_list.p);
        if (rc != DMX_ERR_CAPACITY) return rc;
    }
    // Grids above 1024^2, asymmetric graphs or a capacity retry: the other BFS kernels take contiguous
    // source ranges, so each maximal run of consecutive listed nodes is one call (the preparation, and
    // with it every collective of a sharded preparation, is already done: the ranks may differ in the
    // number of calls from here on).  Kernel times add up; the work counters are the last call's.
    const bool was_disabled = ctx->tile_disabled;
    ctx->tile_disabled = true;
    double total = 0.0;
    for (int64_t i = 0; i < n;) {
        int64_t j = i + 1;
        while (j < n && lst[j] == lst[j - 1] + 1) j++;
        rc = vga_impl(ctx, g, radius, gates_only, lst[i], (int64_t)lst[j - 1] + 1, out_device, true, nullptr);
        if (rc) break;
        total += ctx->last_vga_s;
        i = j;
    }
    ctx->tile_disabled = was_disabled;
    if (rc) return rc;
    ctx->last_vga_s = total;
    return DMX_OK;
}
