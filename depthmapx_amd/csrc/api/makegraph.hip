// api/makegraph.hip -- makeGraph (dmx_makegraph, dmx_makegraph_balance) and the made graph (dmx_graph_info / copy).
// Part of the dmx_api.hip unity build: included inside its extern "C" block, after the context and the
// internal types (dmx_ctx, dmx_pointmap, dmx_graph); not compiled on its own.

// makeGraph kernel variants (makegraph.hip).  VGPR budget: 5 waves per SIMD.  The kernel is latency-bound
// (one wave walks one source's sieve depth by depth), so waves beat registers: at 1000^2, 3 waves/SIMD
// 6.9 s, 4: 5.4 s, 5: 4.9 s (96 VGPRs, some cold spills), 6: 5.4 s.  fixed: the first pass (LDS
// capacities, certified moment sums and the maxdist test compiled in); count: the cost-sample counters.
typedef void (*mk_kernel_t)(const MakeGraphParams*);
// waves per SIMD the makeGraph register allocation targets (A/B builds: -DDMX_MK_WPE=n).  Measured round 4
// (profiles/r4_makegraph_wpe_ab.jsonl, configs[2] / configs[4]): 5 -> 4.62 / 10.65 s, 6 -> 5.20 / 11.99 s,
// 8 -> 9.10 / 19.31 s: fewer registers spill more than the extra waves hide
#ifndef DMX_MK_WPE
#define DMX_MK_WPE 5
#endif
#define MKK(PROF, FIXED, COUNT, MAXD, FAR) makegraph_kernel<DMX_MK_WPE, PROF, FIXED, COUNT, MAXD, FAR>
static mk_kernel_t mk_kernel(bool fixed, bool count, bool maxd, bool far) {
    if (count) {       // the cost sample of dmx_makegraph_balance: always counts (its bounds depend on it)
        if (!fixed || maxd) return MKK(false, false, true, false, false);
        return far ? MKK(false, true, true, false, true) : MKK(false, true, true, false, false);
    }
    if (verbose()) {   // per-phase clocks (maxdist runs take the generic kernel)
        if (!fixed || maxd) return MKK(true, false, false, false, false);
        return far ? MKK(true, true, false, false, true) : MKK(true, true, false, false, false);
    }
    if (!fixed) return MKK(false, false, false, false, false);
    if (maxd) return far ? MKK(false, true, false, true, true) : MKK(false, true, false, true, false);
    return far ? MKK(false, true, false, false, true) : MKK(false, true, false, false, false);
}
#undef MKK

// The largest relative error of makeGraph's moment square root (MK_SQRT) over the integers 1..nmax, measured
// exhaustively on the device (once per context and range): the certificate of the moment sums rests on it.
static int mk_sqrt_err(dmx_ctx* ctx, long long nmax, double* err) {
    if (ctx->sqrt_err_nmax < nmax) {
        DevBuf<unsigned long long> e;
        HIPCHK(e.alloc(1));
        HIPCHK(hipMemsetAsync(e.p, 0, 8, ctx->stream));
        hipLaunchKernelGGL(sqrt_err_kernel, dim3((unsigned)std::min<long long>((nmax + 255) / 256, 4096)), dim3(256), 0,
                           ctx->stream, nmax, e.p);
        HIPCHK(hipGetLastError());
        unsigned long long bits = 0;
        HIPCHK(copy_sync(ctx->stream, &bits, e.p, 8, hipMemcpyDeviceToHost));
        double v;
        std::memcpy(&v, &bits, 8);
        // a device square root worse than 2^-30: no source can pass the moment certificate, so every source runs the
        // serial chains (which do not use it) from the first pass (makegraph_impl)
        if (!(v >= 0.0 && v < 0x1p-30)) {
            VLOG("makegraph: square-root error %.3g over 1..%lld: certified moment sums off\n", v, nmax);
            v = INFINITY;
        }
        ctx->sqrt_err = v;
        ctx->sqrt_err_nmax = nmax;
        VLOG("makegraph: square-root error bound %.3g over 1..%lld\n", v, nmax);
    }
    *err = ctx->sqrt_err;
    return DMX_OK;
}

// makeGraph over [node_begin, node_end), or only over the listed nodes of that range (`only`: the cost
// sample of dmx_makegraph_balance; the graph's other nodes stay unset).  d_work (optional, [n][2]) receives
// each published source's sieve depth steps and candidate chunks.
static int makegraph_impl(dmx_ctx* ctx, dmx_pointmap* pm, double maxdist, int boundary, int64_t node_begin,
                          int64_t node_end, const std::vector<int64_t>* only, uint32_t* d_work, dmx_graph** out) {
    if (!ctx || !pm || !out) return fail(DMX_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(ctx->device));
    const double t_start = now_s();
    PointMapHost& h = *pm->host;
    if (!h.lines_blocked()) h.block_lines();
    if (boundary) { h.keep_edges_only(); pm->version++; }
    int rc = upload_pointmap(ctx, pm);
    if (rc) return rc;
    VLOG("makegraph: host prep + upload %.3f s\n", now_s() - t_start);
    const int64_t N = pm->nnodes;
    if (node_end < 0 || node_end > N) node_end = N;
    if (node_begin < 0 || node_begin > node_end) return fail(DMX_ERR_ARG, "bad node range");
    const int64_t n = node_end - node_begin;
    std::unique_ptr<dmx_graph> g(new dmx_graph());
    g->ctx = ctx;
    g->pm = pm;
    g->nnodes = N;
    g->node_begin = node_begin;
    g->node_end = node_end;
    inherit_merges(g.get());
    const int D = std::max(h.cols(), h.rows());
    HIPCHK(g->node_run_start.alloc(std::max<int64_t>(n, 1)));
    HIPCHK(g->node_nruns.alloc(std::max<int64_t>(n, 1)));
    HIPCHK(g->bin_nruns.alloc(std::max<int64_t>(n, 1) * 32));
    HIPCHK(g->bin_count.alloc(std::max<int64_t>(n, 1) * 32));
    HIPCHK(g->bin_dist.alloc(std::max<int64_t>(n, 1) * 32));
    HIPCHK(g->attrs.alloc(std::max<int64_t>(n, 1) * 3));
    HIPCHK(g->gridconn.alloc(std::max<int64_t>(n, 1)));

    // capacities (retried on overflow)
    // LDS gap / block lists: small lists keep the per-wave LDS near 12 KB at 1000^2 (13 waves per CU
    // instead of 10 with 64-entry lists: 8.27 s -> 6.6 s); longer block lists spill to HBM, longer gap
    // lists re-run the source with larger capacities
    int gcap = MK_GCAP0, bcap = MK_BCAP0;
    int spill_cap = 4096;      // per-wave HBM blocks past bcap
    int64_t capB = 32 * (int64_t)D + 2048;
    if (const char* e = getenv("DMX_MK_GCAP")) gcap = std::max(2, atoi(e));   // test hooks for the retry path
    if (const char* e = getenv("DMX_MK_BCAP")) bcap = std::max(2, atoi(e));
    if (const char* e = getenv("DMX_MK_SPILL")) spill_cap = std::max(1, atoi(e));
    size_t free_b = 0, total_b = 0;
    HIPCHK(hipMemGetInfo(&free_b, &total_b));
    const int64_t n_src = only ? (int64_t)only->size() : n;   // sources this call sweeps
    if (only)
        for (int64_t v : *only)
            if (v < node_begin || v >= node_end) return fail(DMX_ERR_ARG, "sample node outside the range");
    int64_t pool_cap = std::max<int64_t>(n_src * std::max<int64_t>(64, 6 * (int64_t)D), 1024);
    // A whole-graph build does the VGA symmetry certificate's scatter as it publishes each source's runs
    // (the runs are in the L2 then, and the memory-side atomics overlap the sweep), instead of a later pass
    // over the 36 GB pool (0.38 s at 1000^2).  Ranges, samples and cost counts leave it to prepare_symmetry.
    const bool fuse_sym = !only && d_work == nullptr && node_begin == 0 && node_end == N && N > 0 &&
                          !getenv("DMX_MK_NOSYM");
    const int64_t Cc = (int64_t)h.cols() * h.rows();
    if (fuse_sym) {
        HIPCHK(g->sym_prefix.alloc((size_t)4 * Cc));
        HIPCHK(g->sym_diff.alloc((size_t)4 * Cc));
        HIPCHK(g->sym_ho.alloc(N));
        const int maxlines = h.cols() + h.rows();
        hipLaunchKernelGGL(sym_lines_kernel, dim3((maxlines + 127) / 128, 4), dim3(128), 0, ctx->stream, h.cols(),
                           h.rows(), pm->d_cell_node.p, g->sym_prefix.p, 0);
        HIPCHK(hipGetLastError());
    }
    ctx->last_mk_s = 0;
    double sqrt_err = 0.0;
    if (int rc2 = mk_sqrt_err(ctx, 2ll * D * D, &sqrt_err)) return rc2;
    DevBuf<int64_t> fail_list, node_list;
    DevBuf<MakeGraphParams> dP;   // kernel parameters in device memory (see makegraph_kernel)
    HIPCHK(fail_list.alloc(std::max<int64_t>(n, 1)));
    HIPCHK(node_list.alloc(std::max<int64_t>(n, 1)));
    // Run pool size.  The worst case above (6 runs per depth per source) is ~1.4x the real count at
    // 1000^2; at 2000^2 it exceeds the device, and clamping it to the free memory would leave nothing
    // for the scan order a following VGA needs.  When the worst case takes more than 40 % of the free
    // memory, a first pass over an evenly spaced sample of sources measures the runs per source and
    // the pool takes 1.25x that plus 64 per source (0.08 s at 1000^2, so skipped there).  An overflow
    // still re-runs everything with a doubled pool.
    const int64_t kSample = policy::kMkSample;
    const bool big_pool = (double)pool_cap * sizeof(Run) > 0.4 * (double)(free_b + cached_bytes());
    bool sampling = !only && !getenv("DMX_MK_NOSAMPLE") &&
                    ((n >= 16 * kSample && big_pool) || (n >= kSample && getenv("DMX_MK_SAMPLE")));   // test hook
    double mk_total_s = 0.0;
    int64_t reruns = 0;   // sources re-run after a first-pass capacity or certification failure
    std::vector<int64_t> mk_reruns;
    for (int restart = 0; restart < 4; restart++) {
        // one full pass, then re-runs of only the sources that overflowed an LDS / staging capacity
        double kernel_s = 0.0;
        int64_t list_n = -1;   // -1: the whole range
        if (only) {
            list_n = n_src;
            if (list_n)
                HIPCHK(hipMemcpyAsync(node_list.p, only->data(), list_n * 8, hipMemcpyHostToDevice, ctx->stream));
        }
        bool pool_over = false;
        const int64_t pool_cap_full = pool_cap;
        if (fuse_sym) {   // every pass publishes each source once; a restarted pass starts over
            HIPCHK(hipMemsetAsync(g->sym_diff.p, 0, (size_t)4 * Cc * 8, ctx->stream));
            HIPCHK(hipMemsetAsync(g->sym_ho.p, 0, (size_t)N * 8, ctx->stream));
        }
        if (sampling) {
            std::vector<int64_t> sl((size_t)kSample);
            for (int64_t i = 0; i < kSample; i++) sl[i] = node_begin + (i * n) / kSample + n / (2 * kSample);
            HIPCHK(hipMemcpyAsync(node_list.p, sl.data(), kSample * 8, hipMemcpyHostToDevice, ctx->stream));
            list_n = kSample;
            pool_cap = kSample * std::max<int64_t>(64, 6 * (int64_t)D);
        }
        HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 16 * sizeof(int), ctx->stream));
        HIPCHK(hipMemsetAsync(ctx->stats.p, 0, 32 * sizeof(unsigned long long), ctx->stream));
        size_t lds0 = makegraph_lds(gcap, bcap, D);
        int occ0 = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ0, mk_kernel(false, d_work != nullptr, false, false), 64, lds0));
        {
            const int64_t waves0 = std::min<int64_t>((int64_t)ctx->num_cu * std::max(occ0, 1), std::max<int64_t>(n, 1));
            const size_t stage0 = (size_t)waves0 * (capB * 16 + (3 * ((size_t)D + 1) + 4) * 4) * 4;   // headroom for retries
            HIPCHK(hipMemGetInfo(&free_b, &total_b));
            free_b += cached_bytes();   // released by cached_malloc if the fresh allocation needs them
            const size_t pool_bytes_max = free_b > stage0 + (1ull << 30) ? (free_b - stage0 - (1ull << 30)) : 0;
            if ((size_t)pool_cap * sizeof(Run) > pool_bytes_max) pool_cap = (int64_t)(pool_bytes_max / sizeof(Run));
            if (pool_cap <= 0) return fail(DMX_ERR_HIP, "not enough device memory for the run pool");
            double ta = now_s();
            HIPCHK(g->pool.alloc(pool_cap));
            VLOG("makegraph: pool alloc %.3f GB %.3f s\n", pool_cap * 8.0 / 1e9, now_s() - ta);
        }
        for (int attempt = 0; attempt < 8; attempt++) {
            size_t lds = makegraph_lds(gcap, bcap, D);
            if (lds > 160 * 1024) return fail(DMX_ERR_CAPACITY, "makegraph LDS requirement exceeds 160 KiB");
            // re-runs (and every pass when the device square root is not accurate enough): the serial moment chains
            const bool exact_pass = attempt > 0 || getenv("DMX_MK_EXACT") || !(sqrt_err < 0x1p-30) || getenv("DMX_MK_SQRT_BAD");
            const mk_kernel_t kern = mk_kernel(gcap == MK_GCAP0 && bcap == MK_BCAP0 && !exact_pass &&
                                                   !getenv("DMX_MK_NOFIXED"),
                                               d_work != nullptr, maxdist != -1.0, D + 4 > MK_OPEN_LDS);
            int occ = 0;
            HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, 64, lds));
            if (occ < 1) occ = 1;
            const int64_t todo = list_n < 0 ? n : list_n;
            const int64_t waves = std::min<int64_t>((int64_t)ctx->num_cu * occ, std::max<int64_t>(todo, 1));
            const int64_t capA = capB;
            DevBuf<unsigned long long> stA;
            DevBuf<Run> stB;
            DevBuf<uint32_t> pref, rcnt;
            HIPCHK(stA.alloc((size_t)waves * capA));
            HIPCHK(stB.alloc((size_t)waves * capB));
            HIPCHK(pref.alloc((size_t)waves * (3 * ((size_t)D + 1) + 4)));
            HIPCHK(rcnt.alloc((size_t)waves * (3 * ((size_t)D + 1) + 4)));
            HIPCHK(hipMemsetAsync(rcnt.p, 0, (size_t)waves * (3 * ((size_t)D + 1) + 4) * 4, ctx->stream));
            const int openh_n = std::max(0, D + 4 - MK_OPEN_LDS);
            DevBuf<uint32_t> openh;
            HIPCHK(openh.alloc(std::max<size_t>((size_t)waves * openh_n, 1)));
            HIPCHK(hipMemsetAsync(openh.p, 0, std::max<size_t>((size_t)waves * openh_n, 1) * 4, ctx->stream));
            DevBuf<double2> bsp;
            DevBuf<int> bspf;
            HIPCHK(bsp.alloc((size_t)waves * 2 * spill_cap));
            HIPCHK(bspf.alloc((size_t)waves * spill_cap));
            // work counter, error word and failure count restart; the pool cursor carries on
            HIPCHK(hipMemsetAsync(ctx->counters.p, 0, 2 * sizeof(int), ctx->stream));
            HIPCHK(hipMemsetAsync(ctx->counters.p + 4, 0, sizeof(int), ctx->stream));
            MakeGraphParams P;
            P.cols = h.cols(); P.rows = h.rows();
            P.spacing = h.spacing(); P.blx = h.bottom_left().x; P.bly = h.bottom_left().y;
            P.maxdist = maxdist;
            P.cellw = pm->d_cellw.p; P.segs = pm->d_segs.p; P.node_cell = pm->d_node_cell.p;
            P.sqrt_err = sqrt_err;
            P.node_begin = node_begin; P.node_end = node_end;
            P.work_counter = ctx->counters.p + 0;
            P.ctl = ctx->d_ctl;
            ctx->h_ctl->progress = 0;
            P.error = ctx->counters.p + 1;
            P.pool_cursor = (unsigned long long*)(ctx->counters.p + 2);
            P.pool_capacity = pool_cap; P.pool = g->pool.p;
            P.node_run_start = g->node_run_start.p; P.bin_nruns = g->bin_nruns.p; P.bin_count = g->bin_count.p;
            P.bin_dist = g->bin_dist.p; P.attrs = g->attrs.p;
            P.stageA = stA.p; P.stageB = stB.p; P.prefix = pref.p; P.runcnt = rcnt.p;
            P.capA = (int)capA; P.capB = (int)capB; P.gcap = gcap; P.bcap = bcap; P.dmax = D;
            P.bspill = bsp.p; P.bspill_flag = bspf.p; P.spill_cap = spill_cap;
            P.stats = ctx->stats.p;
            P.node_list = list_n < 0 ? nullptr : node_list.p;
            P.list_n = list_n < 0 ? 0 : list_n;
            P.fail_list = fail_list.p;
            P.fail_count = ctx->counters.p + 4;
            P.profile = verbose() ? 1 : 0;
            // the first pass certifies parallel moment sums; re-runs of failed sources use the serial chains
            P.exact_moments = exact_pass ? 1 : 0;
            P.src_work = d_work;
            P.openh = openh.p; P.openh_n = openh_n;
            const bool sym_pass = fuse_sym && !sampling;   // the sampling pass's runs are thrown away
            P.sym_prefix = sym_pass ? g->sym_prefix.p : nullptr;
            P.sym_diff = sym_pass ? g->sym_diff.p : nullptr;
            P.sym_ho = sym_pass ? g->sym_ho.p : nullptr;
            // the shortest span taken (DMX_MK_SPAN: A/B hook; DMX_MK_NOSPAN: every depth cell by cell)
            P.spans = getenv("DMX_MK_NOSPAN") ? 0 : (getenv("DMX_MK_SPAN") ? std::max(1, atoi(getenv("DMX_MK_SPAN"))) : MK_SPAN_MIN);
            HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
            if (todo > 0) {
                HIPCHK(dP.alloc(1));
                HIPCHK(hipMemcpyAsync(dP.p, &P, sizeof(P), hipMemcpyHostToDevice, ctx->stream));
                hipLaunchKernelGGL(kern, dim3((unsigned)waves), dim3(64), lds, ctx->stream,
                                   (const MakeGraphParams*)dP.p);
                HIPCHK(hipGetLastError());
            }
            HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
            HIPCHK(wait_progress(ctx, DMX_PHASE_MAKEGRAPH, todo, 1));
            CANCEL_POINT(ctx);
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
            kernel_s += ms * 1e-3;
            int hc[5] = {0, 0, 0, 0, 0};
            HIPCHK(copy_sync(ctx->stream, hc, ctx->counters.p, sizeof(hc), hipMemcpyDeviceToHost));
            const int err = hc[1], nfail = hc[4];
            VLOG("makegraph: attempt %d (%lld sources, gcap %d bcap %d spill %d capB %lld, occupancy %d): %.3f s, %d failed, "
                 "err %d\n", attempt, (long long)todo, gcap, bcap, spill_cap, (long long)capB, occ, ms * 1e-3, nfail, err);
            if (err & KERR_BIN_MISMATCH) return fail(DMX_ERR_STATE, "internal: whichbin outside octant");
            if (err & KERR_POOL_CAPACITY) {
                unsigned long long used = 0;
                std::memcpy(&used, &hc[2], 8);
                pool_cap = std::max<int64_t>(pool_cap * 2, (int64_t)used + 1024);
                pool_over = true;
                break;
            }
            if (nfail == 0) break;
            if (!sampling) {
                reruns += nfail;
                std::vector<int64_t> fl((size_t)nfail);
                HIPCHK(copy_sync(ctx->stream, fl.data(), fail_list.p, (size_t)nfail * 8, hipMemcpyDeviceToHost));
                mk_reruns.insert(mk_reruns.end(), fl.begin(), fl.end());
            }
            if (err & KERR_GAP_CAPACITY) gcap *= 2;
            if (err & KERR_BLOCK_CAPACITY) spill_cap *= 4;
            if (err & KERR_STAGE_CAPACITY) capB *= 2;
            HIPCHK(hipMemcpyAsync(node_list.p, fail_list.p, (size_t)nfail * 8, hipMemcpyDeviceToDevice, ctx->stream));
            list_n = nfail;
            if (attempt == 7) return fail(DMX_ERR_CAPACITY, "makegraph capacities exceeded after retries");
        }
        if (sampling) {
            unsigned long long used = 0;
            HIPCHK(copy_sync(ctx->stream, &used, ctx->counters.p + 2, 8, hipMemcpyDeviceToHost));
            sampling = false;
            mk_total_s += kernel_s;
            if (pool_over) { pool_cap = pool_cap_full; continue; }   // no estimate: the worst-case pool
            const double per_src = (double)used / (double)kSample;
            pool_cap = std::min<int64_t>(pool_cap_full, (int64_t)(1.25 * per_src * (double)n) + 64 * n + 4096);
            VLOG("makegraph: sample of %lld sources, %.1f runs each -> pool %.3f GB\n", (long long)kSample, per_src,
                 pool_cap * 8.0 / 1e9);
            continue;
        }
        if (pool_over) { mk_total_s += kernel_s; mk_reruns.clear(); reruns = 0; continue; }
        HIPCHK(hipEventRecord(ctx->ev0, ctx->stream));
        if (n > 0 && !only) {   // (a sample leaves the other nodes' run starts unset)
            hipLaunchKernelGGL(gridconn_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, h.rows(),
                               pm->d_node_cell.p + node_begin, n, g->node_run_start.p, g->bin_nruns.p, g->pool.p,
                               g->gridconn.p);
            HIPCHK(hipGetLastError());
            hipLaunchKernelGGL(node_nruns_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream,
                               g->bin_nruns.p, n, g->node_nruns.p);
            HIPCHK(hipGetLastError());
        }
        HIPCHK(hipEventRecord(ctx->ev1, ctx->stream));
        HIPCHK(hipStreamSynchronize(ctx->stream));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
        kernel_s += ms * 1e-3;
        int hc[4] = {0, 0, 0, 0};
        HIPCHK(copy_sync(ctx->stream, hc, ctx->counters.p, sizeof(hc), hipMemcpyDeviceToHost));
        unsigned long long used = 0;
        std::memcpy(&used, &hc[2], 8);
        unsigned long long st[32];
        HIPCHK(copy_sync(ctx->stream, st, ctx->stats.p, sizeof(st), hipMemcpyDeviceToHost));
        if (verbose()) {
            st[22] += st[26] + st[27] + st[28];   // the span block's clocks, all parts
            double tot = (double)st[22];
            for (int i = 8; i < 18; i++) tot += (double)st[i];
            VLOG("makegraph phases (wave clocks): garbage %.1f%%, ranges %.1f%%, candidates %.1f%%, bins %.1f%%, "
                 "moments %.1f%%, run tracking %.1f%%, placement %.1f%%, publish %.1f%%, depth tail %.1f%%, "
                 "octant setup %.1f%% (%.3g total; %llu depth steps, %llu chunks, %llu candidates)\n", 100 * st[8] / tot,
                 100 * st[9] / tot, 100 * st[10] / tot, 100 * st[11] / tot, 100 * st[12] / tot, 100 * st[13] / tot,
                 100 * st[14] / tot, 100 * st[15] / tot, 100 * st[16] / tot, 100 * st[17] / tot, tot, st[2], st[3], st[0]);
            VLOG("makegraph merges: %llu (%llu with one block), %.2f blocks and %.2f gaps a merge\n", st[18], st[19],
                 st[18] ? (double)st[20] / st[18] : 0.0, st[18] ? (double)st[21] / st[18] : 0.0);
            VLOG("makegraph spans: %.1f%% of the clocks; %llu spans over %llu depths (%.1f each), %llu of %llu visible cells "
                 "(%.1f%%)\n", 100 * st[22] / tot, st[23], st[24], st[23] ? (double)st[24] / st[23] : 0.0, st[25], st[1],
                 st[1] ? 100.0 * st[25] / st[1] : 0.0);
            VLOG("makegraph span parts: rows' class ends and open state %.1f%%, gap depth searches %.1f%%, class pieces "
                 "%.1f%%, the rest (setup, examined, sums) %.1f%% of the clocks; %llu row chunks, %llu (chunk, gap) pairs, "
                 "%llu of them with no visible row\n", 100 * st[26] / tot, 100 * st[27] / tot, 100 * st[28] / tot,
                 100 * (st[22] - st[26] - st[27] - st[28]) / tot, st[29], st[30], st[31]);
        }
        ctx->last_stats[0] = (long long)st[0];
        ctx->last_stats[1] = (long long)st[1];
        ctx->last_stats[2] = (long long)used;
        ctx->last_stats[32] = (long long)st[2];   // sieve depth steps
        ctx->last_stats[33] = (long long)st[3];   // 64-candidate chunks
        ctx->last_stats[34] = (long long)reruns;
        ctx->last_mk_reruns = std::move(mk_reruns);
        ctx->last_mk_s = mk_total_s + kernel_s;   // every pass counted (sample, overflow re-runs)
        g->nruns = (int64_t)used;
        if (fuse_sym) { g->sym_fused = true; g->sym_prefix.reset(); }   // the prefix sums are no longer needed
        VLOG("makegraph: kernels %.3f s, total %.3f s\n", kernel_s, now_s() - t_start);
        *out = g.release();
        return DMX_OK;
    }
    return fail(DMX_ERR_CAPACITY, "makegraph capacities exceeded after retries");
}

int dmx_makegraph(dmx_ctx* ctx, dmx_pointmap* pm, double maxdist, int boundary, int64_t node_begin, int64_t node_end,
                  dmx_graph** out) {
    return makegraph_impl(ctx, pm, maxdist, boundary, node_begin, node_end, nullptr, nullptr, out);
}

// Cost model of one source's sweep, in units of one depth step: a source pays a fixed setup, one unit per
// sieve depth step (collectgarbage + visit ranges) and kMkChunkCost per 64-candidate chunk (tests, bins,
// moments, run tracking).  Fitted to per-strip kernel times on MI355X.
using policy::kMkSourceCost;
using policy::kMkChunkCost;

int dmx_makegraph_balance(dmx_ctx* ctx, dmx_pointmap* pm, double maxdist, int boundary, int32_t world, int64_t stride,
                          int64_t* bounds) {
    if (!ctx || !pm || !bounds || world < 1 || stride < 1) return fail(DMX_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(ctx->device));
    PointMapHost& h = *pm->host;
    if (!h.lines_blocked()) h.block_lines();
    if (boundary) { h.keep_edges_only(); pm->version++; }
    int rc = upload_pointmap(ctx, pm);
    if (rc) return rc;
    const int64_t N = pm->nnodes;
    bounds[0] = 0;
    for (int r = 1; r <= world; r++) bounds[r] = N;
    if (N == 0 || world == 1) return DMX_OK;
    // sample j stands for the nodes [j*stride, (j+1)*stride): its middle node is swept
    const int64_t ns = (N + stride - 1) / stride;
    std::vector<int64_t> sample((size_t)ns);
    for (int64_t j = 0; j < ns; j++) sample[j] = std::min<int64_t>(N - 1, j * stride + stride / 2);
    DevBuf<uint32_t> d_work;
    HIPCHK(d_work.alloc((size_t)N * 2));
    HIPCHK(hipMemsetAsync(d_work.p, 0xFF, (size_t)N * 2 * 4, ctx->stream));   // unwritten entries stay ~0u
    dmx_graph* g = nullptr;
    rc = makegraph_impl(ctx, pm, maxdist, 0, 0, N, &sample, d_work.p, &g);   // boundary already applied
    if (rc) return rc;
    dmx_graph_free(g);
    std::vector<uint32_t> w2((size_t)N * 2);
    HIPCHK(copy_sync(ctx->stream, w2.data(), d_work.p, (size_t)N * 2 * 4, hipMemcpyDeviceToHost));
    // cumulative modelled cost at the interval ends; bounds at equal shares (same doubles on every rank)
    std::vector<double> cum((size_t)ns + 1, 0.0);
    for (int64_t j = 0; j < ns; j++) {
        const int64_t v = sample[j];
        if (w2[2 * v] == ~0u || w2[2 * v + 1] == ~0u)
            return fail(DMX_ERR_STATE, "internal: the makeGraph cost sample did not record every sampled source");
        const double w = kMkSourceCost + (double)w2[2 * v] + kMkChunkCost * (double)w2[2 * v + 1];
        const int64_t cnt = std::min<int64_t>(N, (j + 1) * stride) - j * stride;
        cum[j + 1] = cum[j] + w * (double)cnt;
    }
    int64_t j = 0;
    for (int r = 1; r < world; r++) {
        const double target = cum[ns] * (double)r / (double)world;
        while (j < ns - 1 && cum[j + 1] < target) j++;
        const double per = (cum[j + 1] - cum[j]) / (double)(std::min<int64_t>(N, (j + 1) * stride) - j * stride);
        int64_t b = j * stride + (per > 0.0 ? (int64_t)((target - cum[j]) / per) : 0);
        b = std::max<int64_t>(b, bounds[r - 1]);
        bounds[r] = std::min<int64_t>(b, N);
    }
    return DMX_OK;
}

int dmx_graph_free(dmx_graph* g) {
    if (g && g->ctx) (void)hipSetDevice(g->ctx->device);
    delete g;
    return DMX_OK;
}

int dmx_graph_info(const dmx_graph* g, int64_t* nnodes, int64_t* nb, int64_t* ne, int64_t* nruns) {
    if (!g) return fail(DMX_ERR_ARG, "graph is NULL");
    if (nnodes) *nnodes = g->nnodes;
    if (nb) *nb = g->node_begin;
    if (ne) *ne = g->node_end;
    if (nruns) *nruns = g->nruns;
    return DMX_OK;
}

int dmx_graph_copy_range(dmx_graph* g, int64_t kb, int64_t ke, float* attrs, int32_t* bins, int16_t* runs,
                         int64_t runs_cap, int64_t* nruns_out, uint8_t* gridconn) {
    if (!g) return fail(DMX_ERR_ARG, "graph is NULL");
    const int64_t nl = g->node_end - g->node_begin;
    if (ke < 0) ke = nl;
    if (kb < 0 || kb > ke || ke > nl) return fail(DMX_ERR_ARG, "node range outside the graph");
    HIPCHK(hipSetDevice(g->ctx->device));
    hipStream_t st = g->ctx->stream;
    const int64_t n = ke - kb;
    if (nruns_out) *nruns_out = 0;
    if (n == 0) return DMX_OK;
    if (attrs) HIPCHK(copy_sync(st, attrs, g->attrs.p + kb * 3, n * 3 * 4, hipMemcpyDeviceToHost));
    if (gridconn) HIPCHK(copy_sync(st, gridconn, g->gridconn.p + kb, n, hipMemcpyDeviceToHost));
    std::vector<int32_t> bn((size_t)n * 32);
    HIPCHK(copy_sync(st, bn.data(), g->bin_nruns.p + kb * 32, n * 32 * 4, hipMemcpyDeviceToHost));
    if (bins) {
        std::vector<uint16_t> bc((size_t)n * 32);
        std::vector<float> bd((size_t)n * 32);
        HIPCHK(copy_sync(st, bc.data(), g->bin_count.p + kb * 32, n * 32 * 2, hipMemcpyDeviceToHost));
        HIPCHK(copy_sync(st, bd.data(), g->bin_dist.p + kb * 32, n * 32 * 4, hipMemcpyDeviceToHost));
        for (int64_t k = 0; k < n; k++)
            for (int b = 0; b < 32; b++) {
                const int64_t i = k * 32 + b;
                int dir; // Node::make (ngraph.cpp:43-54); empty bins keep NODIR
                if (b == 4 || b == 20) dir = 4;
                else if (b == 12 || b == 28) dir = 8;
                else if ((b > 4 && b < 12) || (b > 20 && b < 28)) dir = 2;
                else dir = 1;
                bins[i * 4 + 0] = bn[i] > 0 ? dir : 0;
                bins[i * 4 + 1] = bc[i];
                std::memcpy(&bins[i * 4 + 2], &bd[i], 4);
                bins[i * 4 + 3] = bn[i];
            }
    }
    int64_t acc = 0;
    std::vector<int64_t> dst((size_t)n);
    for (int64_t k = 0; k < n; k++) {
        int sum = 0;
        for (int b = 0; b < 32; b++) sum += bn[k * 32 + b];
        dst[k] = acc;
        acc += sum;
    }
    if (nruns_out) *nruns_out = acc;
    if (runs) {
        if (runs_cap >= 0 && acc > runs_cap) return fail(DMX_ERR_ARG, "runs buffer too small for the node range");
        // node-ordered copy (the pool is in completion order), gathered in node batches of at most
        // kChunk runs so that the staging buffer stays small next to a 90 GB graph
        const int64_t kChunk = (int64_t)1 << 29;   // 4 GiB of runs
        DevBuf<int64_t> d_dst;
        DevBuf<Run> d_runs;
        HIPCHK(d_dst.alloc(n));
        HIPCHK(d_runs.alloc(std::max<int64_t>(std::min(acc, kChunk), 1)));
        int64_t k0 = 0;
        while (k0 < n) {
            int64_t k1 = k0;
            const int64_t base = dst[k0];
            while (k1 < n && (k1 == k0 || (k1 + 1 < n ? dst[k1 + 1] : acc) - base <= kChunk)) k1++;
            const int64_t cnt = (k1 < n ? dst[k1] : acc) - base;
            std::vector<int64_t> rel((size_t)(k1 - k0));
            for (int64_t k = k0; k < k1; k++) rel[k - k0] = dst[k] - base;
            if (cnt > (int64_t)d_runs.n) HIPCHK(d_runs.alloc(cnt));   // one node above the chunk size
            HIPCHK(copy_sync(st, d_dst.p, rel.data(), (k1 - k0) * 8, hipMemcpyHostToDevice));
            hipLaunchKernelGGL(gather_runs_kernel, dim3((unsigned)(k1 - k0)), dim3(256), 0, st, g->pool.p,
                               g->node_run_start.p + kb + k0, g->node_nruns.p + kb + k0, d_dst.p, k1 - k0, d_runs.p);
            HIPCHK(hipGetLastError());
            if (cnt) HIPCHK(copy_sync(st, runs + base * 4, d_runs.p, cnt * sizeof(Run), hipMemcpyDeviceToHost));
            k0 = k1;
        }
    }
    return DMX_OK;
}

int dmx_graph_copy(dmx_graph* g, float* attrs, int32_t* bins, int16_t* runs, uint8_t* gridconn) {
    return dmx_graph_copy_range(g, 0, -1, attrs, bins, runs, -1, nullptr, gridconn);
}
