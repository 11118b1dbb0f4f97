// api/shard.hip -- shard blobs: a makeGraph range serialised on the device, and the assembly of a whole graph from them.
// Part of the dmx_api.hip unity build: included inside its extern "C" block, after the context and the
// internal types (dmx_ctx, dmx_pointmap, dmx_graph); not compiled on its own.

// ---------------------------------------------------------------- shard blobs
// layout: int64 header[4] {node_begin, node_end, nruns, magic}, then (8-byte aligned sections)
// bin_nruns i32[n*32], bin_count u16[n*32], bin_dist f32[n*32], attrs f32[n*3], gridconn u8[n],
// runs (node order).
static const int64_t kBlobMagic = 0x31424d58444d44LL;
static inline int64_t al8(int64_t x) { return (x + 7) & ~7LL; }
static void blob_layout(int64_t n, int64_t nruns, int64_t* off /*7*/) {
    off[0] = 32;
    off[1] = off[0] + al8(n * 32 * 4);
    off[2] = off[1] + al8(n * 32 * 2);
    off[3] = off[2] + al8(n * 32 * 4);
    off[4] = off[3] + al8(n * 3 * 4);
    off[5] = off[4] + al8(n);
    off[6] = off[5] + nruns * 8;
}

int dmx_graph_blob_size(dmx_graph* g, int64_t* bytes) {
    if (!g || !bytes) return fail(DMX_ERR_ARG, "bad arguments");
    int64_t off[7];
    blob_layout(g->node_end - g->node_begin, g->nruns, off);
    *bytes = off[6];
    return DMX_OK;
}

int dmx_graph_blob_write_device(dmx_graph* g, void* dst, int64_t bytes) {
    if (!g || !dst) return fail(DMX_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(g->ctx->device));
    const int64_t n = g->node_end - g->node_begin;
    int64_t off[7];
    blob_layout(n, g->nruns, off);
    if (bytes < off[6]) return fail(DMX_ERR_ARG, "blob buffer too small");
    char* d = (char*)dst;
    hipStream_t s = g->ctx->stream;
    int64_t hdr[4] = {g->node_begin, g->node_end, g->nruns, kBlobMagic};
    HIPCHK(hipMemcpyAsync(d, hdr, 32, hipMemcpyHostToDevice, s));
    if (n) {
        HIPCHK(hipMemcpyAsync(d + off[0], g->bin_nruns.p, n * 32 * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(d + off[1], g->bin_count.p, n * 32 * 2, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(d + off[2], g->bin_dist.p, n * 32 * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(d + off[3], g->attrs.p, n * 3 * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(d + off[4], g->gridconn.p, n, hipMemcpyDeviceToDevice, s));
        std::vector<int32_t> nr((size_t)n);
        HIPCHK(hipMemcpyAsync(nr.data(), g->node_nruns.p, n * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        std::vector<int64_t> dsto((size_t)n);
        int64_t acc = 0;
        for (int64_t k = 0; k < n; k++) { dsto[k] = acc; acc += nr[k]; }
        DevBuf<int64_t> d_dst;
        HIPCHK(d_dst.alloc(n));
        HIPCHK(hipMemcpyAsync(d_dst.p, dsto.data(), n * 8, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(gather_runs_kernel, dim3((unsigned)n), dim3(256), 0, s, g->pool.p, g->node_run_start.p,
                           g->node_nruns.p, d_dst.p, n, (Run*)(d + off[5]));
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipStreamSynchronize(s));
    return DMX_OK;
}

int dmx_graph_assemble_device(dmx_ctx* ctx, dmx_pointmap* pm, const void* const* blobs, const int64_t* sizes,
                              int nshards, dmx_graph** out) {
    if (!ctx || !pm || !blobs || !out || nshards <= 0) return fail(DMX_ERR_ARG, "bad arguments");
    HIPCHK(hipSetDevice(ctx->device));
    int rc = upload_pointmap(ctx, pm);
    if (rc) return rc;
    const int64_t N = pm->nnodes;
    std::vector<std::array<int64_t, 4>> hdr((size_t)nshards);
    int64_t total_runs = 0;
    for (int i = 0; i < nshards; i++) {
        HIPCHK(copy_sync(ctx->stream, hdr[i].data(), blobs[i], 32, hipMemcpyDeviceToHost));
        if (hdr[i][3] != kBlobMagic) return fail(DMX_ERR_ARG, "not a dmx graph blob");
        total_runs += hdr[i][2];
    }
    std::unique_ptr<dmx_graph> g(new dmx_graph());
    g->ctx = ctx; g->pm = pm; g->nnodes = N; g->node_begin = 0; g->node_end = N; g->nruns = total_runs;
    inherit_merges(g.get());
    HIPCHK(g->node_run_start.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(g->node_nruns.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(g->bin_nruns.alloc(std::max<int64_t>(N, 1) * 32));
    HIPCHK(g->bin_count.alloc(std::max<int64_t>(N, 1) * 32));
    HIPCHK(g->bin_dist.alloc(std::max<int64_t>(N, 1) * 32));
    HIPCHK(g->attrs.alloc(std::max<int64_t>(N, 1) * 3));
    HIPCHK(g->gridconn.alloc(std::max<int64_t>(N, 1)));
    HIPCHK(g->pool.alloc(std::max<int64_t>(total_runs, 1)));
    hipStream_t s = ctx->stream;
    std::vector<char> covered((size_t)N, 0);
    // shards are placed in node order; runs of a shard are contiguous in node order
    std::vector<int> order(nshards);
    for (int i = 0; i < nshards; i++) order[i] = i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return hdr[a][0] < hdr[b][0]; });
    int64_t run_base = 0;
    for (int oi = 0; oi < nshards; oi++) {
        const int i = order[oi];
        const int64_t b = hdr[i][0], e = hdr[i][1], n = e - b, nr = hdr[i][2];
        if (b < 0 || e > N || b > e) return fail(DMX_ERR_ARG, "blob node range does not fit the point map");
        int64_t off[7];
        blob_layout(n, nr, off);
        if (sizes && sizes[i] < off[6]) return fail(DMX_ERR_ARG, "blob shorter than its header says");
        for (int64_t k = b; k < e; k++) {
            if (covered[k]) return fail(DMX_ERR_ARG, "overlapping shards");
            covered[k] = 1;
        }
        const char* d = (const char*)blobs[i];
        if (n) {
            HIPCHK(hipMemcpyAsync(g->bin_nruns.p + b * 32, d + off[0], n * 32 * 4, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(g->bin_count.p + b * 32, d + off[1], n * 32 * 2, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(g->bin_dist.p + b * 32, d + off[2], n * 32 * 4, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(g->attrs.p + b * 3, d + off[3], n * 3 * 4, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(g->gridconn.p + b, d + off[4], n, hipMemcpyDeviceToDevice, s));
        }
        if (nr) HIPCHK(hipMemcpyAsync(g->pool.p + run_base, d + off[5], nr * 8, hipMemcpyDeviceToDevice, s));
        run_base += nr;
    }
    for (int64_t k = 0; k < N; k++)
        if (!covered[k]) return fail(DMX_ERR_ARG, "shards do not cover every node");
    if (N) {
        hipLaunchKernelGGL(node_nruns_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, g->bin_nruns.p, N,
                           g->node_nruns.p);
        HIPCHK(hipGetLastError());
        std::vector<int32_t> nr((size_t)N);
        HIPCHK(hipMemcpyAsync(nr.data(), g->node_nruns.p, N * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        std::vector<int64_t> st((size_t)N);
        int64_t acc = 0;
        for (int64_t k = 0; k < N; k++) { st[k] = acc; acc += nr[k]; }
        if (acc != total_runs) return fail(DMX_ERR_ARG, "blob run counts inconsistent");
        HIPCHK(hipMemcpyAsync(g->node_run_start.p, st.data(), N * 8, hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    *out = g.release();
    return DMX_OK;
}
