/* dmx.h -- C ABI of the MI355X visibility-graph engine (libdmx.so).
 *
 * Drop-in boundary for the depthmapX VISPREP makeGraph + VGA global path.  Every entry point is
 * extern "C", takes plain pointers and sizes, never throws, and returns an int status
 * (DMX_OK = 0, negative on error; dmx_last_error() explains).  The reference interface each one
 * replaces is cited as file:line in orange-vertex/depthmapX.
 *
 * Ownership: the library owns contexts, point maps and graphs (device buffers included); callers
 * release them with the matching *_free.  Host arrays passed in are copied; host arrays passed out
 * are caller-allocated with the sizes the *_info calls report.  Device pointers (dmx_*_device)
 * must be valid on the context's device.  One context per device; one process per GPU.
 */
#ifndef DMX_H
#define DMX_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DMX_ABI_VERSION 1

enum {
    DMX_OK = 0,
    DMX_ERR_ARG = -1,          /* invalid argument / handle */
    DMX_ERR_HIP = -2,          /* HIP runtime error (no device, launch failure, OOM) */
    DMX_ERR_CAPACITY = -3,     /* a kernel capacity was exceeded even after retries */
    DMX_ERR_STATE = -4,        /* call sequence not allowed (e.g. makegraph on an unfilled map) */
    DMX_ERR_UNSUPPORTED = -5,  /* feature of the reference not (yet) implemented on this path */
    DMX_ERR_OUTSIDE = -6,      /* fill point outside the region ("Point outside of target region") */
    DMX_ERR_CANCELLED = -7     /* dmx_ctx_cancel / the progress callback stopped the operation
                                  (the reference throws Communicator::CancelledException, genlib/comm.h:61-65) */
};

/* Phases reported to the progress callback. */
enum {
    DMX_PHASE_MAKEGRAPH = 1,   /* sources of PointMap::sparkGraph2 (pointdata.cpp:1293-1322) */
    DMX_PHASE_VGA = 2          /* sources of VGAVisualGlobal::run (vgavisualglobal.cpp:195-202) */
};

typedef struct dmx_ctx dmx_ctx;
typedef struct dmx_pointmap dmx_pointmap;
typedef struct dmx_graph dmx_graph;

/* ---- library / device ------------------------------------------------------------------ */
int dmx_abi_version(void);
/* Thread-local message for the last failing call on this thread. */
const char* dmx_last_error(void);
/* Bind a context to HIP device `device` (the process-local ordinal).  No reference counterpart:
 * salalib is single-threaded CPU code. */
int dmx_ctx_create(int device, dmx_ctx** out);
int dmx_ctx_free(dmx_ctx* ctx);
/* Return the device blocks the engine keeps cached for reuse by the next graph of the same size
 * (run pool, scan order, visibility rows) to the HIP runtime.  Optional; allocation failures do it
 * automatically. */
int dmx_release_cached_memory(void);

/* Progress and cancellation, the Communicator contract (genlib/comm.h:59-142): the reference posts the
 * record count and polls IsCancelled every 500 ms inside makeGraph (pointdata.cpp:1301-1316) and VGA
 * (vgavisualglobal.cpp:195-202).  While a makegraph / VGA-global kernel runs, the calling thread
 * calls fn(user, phase, done, total) every interval_s seconds (<= 0: 0.5 s) and once with
 * done == total when the phase completes; a non-zero return requests cancellation.  fn NULL: no
 * polling (the default).  The kernels read the cancel word between sources, so a cancelled call
 * returns DMX_ERR_CANCELLED within one source's time; its outputs are not written (device outputs
 * are undefined).  A context's callback runs on the thread that made the call. */
typedef int32_t (*dmx_progress_fn)(void* user, int32_t phase, int64_t done, int64_t total);
int dmx_ctx_set_progress(dmx_ctx* ctx, dmx_progress_fn fn, void* user, double interval_s);
/* Request cancellation of the operation running on ctx (callable from any thread).  The request is
 * consumed by the operation that observes it; one made while no operation runs cancels the next
 * makegraph, VGA-global or step-depth (metric, angular, visual) call at its first poll -- before that
 * call writes any output.  VGA local / metric / angular do not poll (a pending request waits). */
int dmx_ctx_cancel(dmx_ctx* ctx);
/* Wall time of the kernels of the last makegraph / vga call, measured with HIP events on the
 * context stream (seconds); kernel_ms receives per-kernel averages. */
int dmx_ctx_last_timing(dmx_ctx* ctx, double* makegraph_s, double* vga_s);
/* Work counters of the last calls (for roofline accounting), up to 40 entries (engine.py names them):
 * [0] sieve cells examined, [1] visible (source,target) pairs, [2] runs written,
 * [3] VGA kernel used (0 top-down v1, 1 direction-optimising restricted to top-down,
 *     2 direction-optimising, 3 tile-resolved) | nodes needing exact in-set corrections << 8,
 * [4] runs read by the BFS, [5] bottom-up levels | top-down levels << 32, [6] cells reached (sum
 * over sources), [7] sources run, [8] bottom-up cells that found no hit, [9] their runs,
 * [10] bitmaps in HBM (direction-optimising), [11] tiles resolved by common runs, [12] launch
 * shape, [13] hard cells rejected by their tile-visibility row, [14] bytes of those rows read,
 * [15] runs scanned by hard cells, [16] hard cells that hit, [17] hard cells, ... [38] searches the last VGA
 * global / visual step depth call ran again in the reference's level order (vga_ordered.hip), [39] microseconds
 * the last VGA preparation spent on the symmetry scatter and its all-reduces (0 when makeGraph did it), [40] the
 * memory-dependent VGA preparation the last tile search ran with (bits: 0 scan order, 1 scan order released for
 * the partial-tile masks, 2 tile-visibility rows, 3 fully-seen rows, 4 tile-to-tile rows, 5 partial-tile masks,
 * 6 row summaries, 7 asymmetric mode), [41] bytes of tile-visibility rows held, [42] bytes of the scan order
 * held, [43] asymmetric mode: nodes whose runs differ from the reference graph (dmx_graph_set_drawing).  n <= 48. */
int dmx_ctx_last_stats(dmx_ctx* ctx, int64_t* out, int n);

/* The sources the last makeGraph swept a second time (graph node indices, in the order the passes listed
 * them; a source can appear once per pass): bit 62 set for a capacity overflow (gap list, block spill,
 * staging), clear for a moment-sum certificate that did not decide the float.  Writes
 * min(cap, *n) entries; *n receives the count. */
int dmx_ctx_last_mk_reruns(dmx_ctx* ctx, int64_t* nodes, int64_t cap, int64_t* n);

/* Diagnostics of the last tile-resolved VGA launch: core-clock cycles spent (workgroup leader,
 * summed over workgroups) in level 1, phase A (tile-common runs), B (head runs), C (hard cells)
 * and level bookkeeping. */
int dmx_ctx_last_phase_cycles(dmx_ctx* ctx, int64_t* out5);

/* ---- VISPREP preparation (host model) ----------------------------------------------------- */
/* MetaGraph::addNewPointMap + PointMap::setGrid(spacing, (0,0)) (salalib/pointdata.cpp:122-171),
 * with the drawing `lines` ([n][4] = x1,y1,x2,y2 as PointMap::blockLines reads them,
 * pointdata.cpp:308-320) inside `region` (= MetaGraph::getRegion(), [4] = blx,bly,trx,try). */
int dmx_pointmap_create(const double* region, double spacing, const double* lines, int64_t nlines,
                        dmx_pointmap** out);
int dmx_pointmap_free(dmx_pointmap* pm);
/* dm_runmethods::fillGraph -> PointMap::makePoints(p, FULLFILL) (depthmapXcli/runmethods.cpp:269-277,
 * salalib/pointdata.cpp:402-481).  DMX_ERR_OUTSIDE if the point is outside the region;
 * *made = 0 where makePoints returns false. */
int dmx_pointmap_fill(dmx_pointmap* pm, double x, double y, int* made);
/* The same fill computed on the context's GPU (kernels/fill.hip): PointMap::blockLines
 * (pointdata.cpp:296-357, spacepix.cpp:144-214, p2dpoly.cpp:626-667) on the first fill, then the
 * makePoints/expand flood fill (pointdata.cpp:402-514) in the reference's exact expand order, so
 * the FILLED and order-dependent EDGE bits equal the host fill's.  Same return codes and *made. */
int dmx_pointmap_fill_device(dmx_ctx* ctx, dmx_pointmap* pm, double x, double y, int* made);
/* Seconds of the last dmx_pointmap_fill_device: blockLines (0 when lines were already blocked),
 * flood fill, and the number of fill levels. */
int dmx_ctx_last_fill(dmx_ctx* ctx, double* block_s, double* fill_s, int64_t* levels);
/* PointMap::makePoints(seed, fill_type) (salalib/pointdata.cpp:402-481; MetaGraph::makePoints,
 * mgraph.cpp:237-247), the GUI's three fill modes (depthmapX/views/depthmapview/depthmapview.h:75):
 * 0 FULLFILL (Point::FILLED, what the CLI uses), 1 SEMIFILL (FILLED | CONTEXTFILLED: such cells at odd
 * PixelRefs are skipped as VGA sources and not expanded under a radius or in visual step depth), 2 AUGMENT
 * (Point::AUGMENTED without FILLED).  The reference's AUGMENT fill only ends when the seed expands nowhere
 * (expand stops at FILLED cells only, pointdata.cpp:489, so augmented neighbours re-queue each other
 * forever): that case sets the seed alone, any other returns DMX_ERR_UNSUPPORTED with no cell filled
 * (the occluders are blocked, as before any fill).
 * The _device form runs FULLFILL / SEMIFILL on the context's GPU as dmx_pointmap_fill_device does. */
int dmx_pointmap_make_points(dmx_pointmap* pm, double x, double y, int fill_type, int* made);
int dmx_pointmap_make_points_device(dmx_ctx* ctx, dmx_pointmap* pm, double x, double y, int fill_type, int* made);
/* Restore the FILLED / EDGE / CONTEXTFILLED cell states of a map saved earlier (e.g. the state
 * array of a PointMap chunk of the same grid), as PointMap::read does before makeGraph. */
int dmx_pointmap_set_state(dmx_pointmap* pm, const int32_t* state);
/* cols, rows, bottom-left cell centre, filled count. */
int dmx_pointmap_info(const dmx_pointmap* pm, int32_t* cols, int32_t* rows, double* bl_x, double* bl_y,
                      int64_t* filled);
/* Point::m_state per cell, x-major (cell = x*rows + y, ColumnMatrix order, simplematrix.h:193-218). */
int dmx_pointmap_state(const dmx_pointmap* pm, int32_t* out);
/* Cropped occluder pieces per cell after blockLines: counts[C], pieces[total][4]. */
int dmx_pointmap_cell_lines(dmx_pointmap* pm, int32_t* counts, double* pieces, int64_t* total);

/* ---- makeGraph (GPU) ---------------------------------------------------------------------- */
/* MetaGraph::makeGraph(comm, boundary, maxdist) -> PointMap::sparkGraph2 (salalib/mgraph.cpp:264-284,
 * pointdata.cpp:1246-1341).  Builds nodes [node_begin, node_end) of the filled cells in x-major
 * order (node_end < 0: all) -- a sub-range is one rank's shard.  maxdist = -1: unrestricted. */
int dmx_makegraph(dmx_ctx* ctx, dmx_pointmap* pm, double maxdist, int boundary, int64_t node_begin,
                  int64_t node_end, dmx_graph** out);
/* Shard bounds for `world` ranks (no reference counterpart: the reference builds the graph on one
 * host, pointdata.cpp:1246-1341).  Sweeps every stride-th source (the middle node of each run of
 * `stride` nodes), models each source's cost from its sieve depth steps and candidate chunks, and writes
 * bounds[0..world] (bounds[0] = 0, bounds[world] = nodes) so that the contiguous ranges
 * [bounds[r], bounds[r+1]) carry equal modelled makeGraph cost.  The counts are deterministic: every rank
 * computes the same bounds without communicating.  boundary as for dmx_makegraph (applied to pm here). */
int dmx_makegraph_balance(dmx_ctx* ctx, dmx_pointmap* pm, double maxdist, int boundary, int32_t world,
                          int64_t stride, int64_t* bounds);
int dmx_graph_free(dmx_graph* g);
/* nodes in the whole map, first/last node built here, runs held. */
int dmx_graph_info(const dmx_graph* g, int64_t* nnodes, int64_t* node_begin, int64_t* node_end, int64_t* nruns);
/* Copies in reference layout (rows for the built range only, node order):
 *   attrs[n][3]  Connectivity, Point First Moment, Point Second Moment (pointdata.cpp:1494-1497)
 *   bins[n][32][4]  Bin::m_dir, m_node_count (u16), m_distance (f32 bits), runs in bin (ngraph.h:48-60)
 *   runs[R][4]   PixelVec start.x,start.y,end.x,end.y in Bin order (ngraph.cpp:234-304)
 *   gridconn[n]  Point::m_grid_connections (pointdata.cpp:1735-1768)
 * Any pointer may be NULL. */
int dmx_graph_copy(dmx_graph* g, float* attrs, int32_t* bins, int16_t* runs, uint8_t* gridconn);
/* The same for the local nodes [node_b, node_e) only (node_e < 0: to the end): bins/attrs/gridconn
 * sized for the range, runs node-ordered (capacity runs_cap entries, < 0: unchecked); *nruns_out
 * = the range's run count (runs may be NULL to query it). */
int dmx_graph_copy_range(dmx_graph* g, int64_t node_b, int64_t node_e, float* attrs, int32_t* bins, int16_t* runs,
                         int64_t runs_cap, int64_t* nruns_out, uint8_t* gridconn);

/* Shard exchange for multi-GPU runs: a graph's built range serialises into one flat blob
 * (device memory) that another rank's dmx_graph_assemble can consume. */
int dmx_graph_blob_size(dmx_graph* g, int64_t* bytes);
int dmx_graph_blob_write_device(dmx_graph* g, void* dst_device, int64_t bytes);
/* Build the whole-map graph from nshards blobs (device pointers, any order of ranges). */
int dmx_graph_assemble_device(dmx_ctx* ctx, dmx_pointmap* pm, const void* const* blobs, const int64_t* sizes,
                              int nshards, dmx_graph** out);

/* ---- VGA global (GPU) ----------------------------------------------------------------------- */
/* MetaGraph::analyseGraph(OUTPUT_VISUAL, global) -> VGAVisualGlobal(radius, gates_only).run
 * (salalib/mgraph.cpp:349-359, vgamodules/vgavisualglobal.cpp:23-216) for source nodes
 * [src_begin, src_end) (src_end < 0: all).  radius = -1 for "n".  The graph must hold every node
 * (dmx_graph_assemble_device for shards).  out: host [N][7] or device (dmx_vga_global_device), rows
 * outside the range untouched, columns in table (alphabetical) order: Visual Entropy, Visual
 * Integration [HH], [P-value], [Tekl], Visual Mean Depth, Visual Node Count, Visual Relativised
 * Entropy.  levels (optional, host [N][3]): total nodes, total depth, BFS levels.
 * The first call on a graph builds its search structures (scan order, tile-visibility rows and, when
 * they take at most a quarter of the free device memory, the partial-tile masks: about 10 GB next to
 * the 36 GB graph at 1000^2); they stay with the graph until dmx_graph_free.  Results do not depend on
 * which of them fit. */
int dmx_vga_global(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t src_begin, int64_t src_end,
                   float* out, int64_t* levels);
int dmx_vga_global_device(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t src_begin,
                          int64_t src_end, float* out_device);
/* The same for an arbitrary list of source nodes (host array of n node indices); rows of other
 * nodes in out_device are left untouched.  Used to interleave multi-GPU shards over the grid. */
int dmx_vga_global_device_list(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, const int64_t* nodes,
                               int64_t n, float* out_device);
/* Diagnostics of the VGA preparation (no reference counterpart): the nodes whose visible set is not
 * symmetric (a cell in the node's runs that does not see the node back), found by 64-bit random-weight
 * range hashes and routed through exact in-set corrections.  *n in = capacity, out = count; nodes NULL:
 * only *n.  Builds the preparation on the graph's context if no VGA call has. */
int dmx_graph_special_nodes(dmx_graph* g, int32_t* nodes, int64_t* n);
/* ---- VGA metric (GPU) ----------------------------------------------------------------------- */
/* MetaGraph::analyseGraph(OUTPUT_METRIC) -> VGAMetric(radius, gates_only).run (salalib/mgraph.cpp:
 * 359-361, vgamodules/vgametric.cpp:26-136) for source nodes [src_begin, src_end) (src_end < 0:
 * all); radius < 0 for "n" (otherwise in drawing units, compared with dist * spacing).  out: host
 * [N][4] in node order, rows outside the range untouched: Metric Mean Shortest-Path Angle, Metric
 * Mean Shortest-Path Distance, Metric Mean Straight-Line Distance, Metric Node Count (-1 rows with
 * gates_only). */
int dmx_vga_metric(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t src_begin, int64_t src_end,
                   float* out);
/* ---- VGA angular (GPU) ---------------------------------------------------------------------- */
/* MetaGraph::analyseGraph(OUTPUT_ANGULAR) -> VGAAngular(radius, gates_only).run (salalib/mgraph.cpp:
 * 362-364, vgamodules/vgaangular.cpp:26-133) for source nodes [src_begin, src_end); radius < 0 for
 * "n" (otherwise compared with the cumulative angle).  out: host [N][3] in node order: Angular Mean
 * Depth, Angular Total Depth, Angular Node Count (-1 rows with gates_only). */
int dmx_vga_angular(dmx_ctx* ctx, dmx_graph* g, double radius, int gates_only, int64_t src_begin, int64_t src_end,
                    float* out);
/* ---- VGA visual local (GPU) ----------------------------------------------------------------- */
/* MetaGraph::analyseGraph(OUTPUT_VISUAL, local) -> VGAVisualLocal(gates_only).run
 * (salalib/mgraph.cpp:349-353, vgamodules/vgavisuallocal.cpp:23-117) for source nodes
 * [src_begin, src_end) (src_end < 0: all).  out: host [N][3] in node order, rows outside the range
 * untouched: Visual Clustering Coefficient, Visual Control, Visual Controllability (-1 for skipped
 * sources and neighbourhoods of <= 1 cell).  The two tile bitmaps per source live in LDS up to ~780^2
 * cells and in per-workgroup HBM slices above that (no grid-size limit). */
int dmx_vga_local(dmx_ctx* ctx, dmx_graph* g, int gates_only, int64_t src_begin, int64_t src_end, float* out);
/* Multi-GPU share of the VGA preparation (no reference counterpart: the reference prepares nothing;
 * this splits our own O(runs) pre-passes).  Every rank holds the whole graph; the per-node scatters
 * (in-set hash sums, tile-visibility rows) then run over nodes [node_begin, node_end)
 * only and each partial device buffer is handed to fn, which must sum it in place over all ranks
 * (an all-reduce SUM of `count` elements of dtype DMX_I32 / DMX_I64, returning 0 on success) before
 * returning.  Every rank must call this with the same fn semantics before its first VGA call on g;
 * fn is called the same number of times, in the same order, on every rank.  fn = NULL undoes it. */
#define DMX_I32 0
#define DMX_I64 1
typedef int (*dmx_allreduce_fn)(void* device_ptr, int64_t count, int dtype, void* user);
int dmx_graph_set_prep_shard(dmx_graph* g, int64_t node_begin, int64_t node_end, dmx_allreduce_fn fn, void* user);

/* ---- VGA metric step depth (GPU) ----------------------------------------------------------- */
/* dm_runmethods::runStepDepth with -sdt metric -> MetaGraph::analyseGraph(point_depth_selection=2)
 * -> VGAMetricDepth::run (depthmapXcli/runmethods.cpp:735-778, salalib/mgraph.cpp:327-330,
 * vgamodules/vgametricdepth.cpp:23-92).  sel_cells: x-major cell indices of the selection
 * (PointMap::setCurSel keeps FILLED cells only; order and duplicates do not matter).  out: host
 * [N][3] in node order: Metric Step Shortest-Path Angle, Metric Step Shortest-Path Length,
 * Metric Straight-Line Distance (single selected cell only, else -1); unreached cells -1.
 * DMX_ERR_STATE if no filled cell is selected (the reference then skips the analysis). */
int dmx_metric_stepdepth(dmx_ctx* ctx, dmx_graph* g, const int32_t* sel_cells, int64_t nsel, float* out);
/* ---- VGA angular step depth (GPU) ---------------------------------------------------------- */
/* dm_runmethods::runStepDepth with -sdt angular -> MetaGraph::analyseGraph(point_depth_selection=3)
 * -> VGAAngularDepth::run (depthmapXcli/runmethods.cpp:770-772, salalib/mgraph.cpp:334-336,
 * vgamodules/vgaangulardepth.cpp:23-75).  sel_cells as for dmx_metric_stepdepth.  out: host [N]
 * "Angular Step Depth" in node order (unreached cells -1).  DMX_ERR_STATE if no filled cell is
 * selected. */
int dmx_angular_stepdepth(dmx_ctx* ctx, dmx_graph* g, const int32_t* sel_cells, int64_t nsel, float* out);
/* ---- VGA visual step depth (GPU) ----------------------------------------------------------- */
/* dm_runmethods::runStepDepth with -sdt visual -> MetaGraph::analyseGraph(point_depth_selection=1)
 * -> VGAVisualGlobalDepth::run (depthmapXcli/runmethods.cpp:767-769, salalib/mgraph.cpp:312-314,
 * vgamodules/vgavisualglobaldepth.cpp:23-77).  sel_cells as for dmx_metric_stepdepth.  out: host
 * [N] "Visual Step Depth" in node order (unreached cells -1).  DMX_ERR_STATE if no filled cell is
 * selected.  Grids up to 1024^2 with a symmetric graph take the tile-resolved BFS; others the
 * level-synchronous top-down search (kernels/vstep.hip). */
int dmx_visual_stepdepth(dmx_ctx* ctx, dmx_graph* g, const int32_t* sel_cells, int64_t nsel, float* out);
/* Kernel time of the last step-depth call, expanders popped, cells relaxed. */
int dmx_ctx_last_stepdepth(dmx_ctx* ctx, double* seconds, int64_t* expanders_popped, int64_t* cells_relaxed);
/* How the last metric step depth ran: out4 = {mode (0 serial, 1 batched over the whole GPU, 2 a
 * batch capacity overflowed and the serial kernel re-ran the search), batches (serial: queue
 * refills), cells improved, ambiguous cells folded sequentially}. */
int dmx_ctx_last_stepdepth_detail(dmx_ctx* ctx, int64_t* out4);

/* ---- .graph PointMap chunk (host) ------------------------------------------------------------ */
/* The bytes PointMap::write emits into a .graph file (salalib/pointdata.cpp:1158-1188, with
 * AttributeTable::write attributetable.cpp:427-456, Point::write point.cpp:51-73, Node/Bin/PixelVec
 * write ngraph.cpp:209-220,447-472,517-583): header, attribute table (columns alphabetical, stats
 * replayed in setValue order), every cell x-major with its run-length node (4-bit ShiftLength).
 * bins/runs/gridconn as dmx_graph_copy returns them; values [ncols][nnodes] in insertion order;
 * displayed indexes the columns.  buf NULL (or cap too small): only *size is set. */
int dmx_chunk_write(const dmx_pointmap* pm, int64_t nnodes, const int32_t* bins, const int16_t* runs, int64_t nruns,
                    const uint8_t* gridconn, int ncols, const char* const* names, const float* values,
                    const uint8_t* locked, const uint8_t* setmask, int displayed, int boundary, uint8_t* buf, int64_t cap,
                    int64_t* size);
/* setmask (optional, [ncols][nnodes]): rows the analysis called setValue on (column statistics
 * skip the others, like the reference's AttributeColumnImpl::updateStats). */
/* PointMap::read (pointdata.cpp:1073-1156, ngraph.cpp:420-445,491-563): decode a chunk; runs come
 * back with the reference's lossy 4-bit row shift applied. */
typedef struct dmx_chunk dmx_chunk;
int dmx_chunk_parse(const uint8_t* buf, int64_t size, dmx_chunk** out);
int dmx_chunk_free(dmx_chunk* c);
int dmx_chunk_info(const dmx_chunk* c, int32_t* cols, int32_t* rows, double* spacing, double* bl, int64_t* nnodes,
                   int64_t* nruns, int32_t* ncols, int32_t* displayed_sorted, int64_t* bytes_used);
int dmx_chunk_column(const dmx_chunk* c, int i, char* name, int name_cap, float* values, int* locked);
int dmx_chunk_arrays(const dmx_chunk* c, int32_t* state, int32_t* bins, int16_t* runs, uint8_t* gridconn);
/* A state-only point map (region = MetaGraph::getRegion()) and its device graph from a chunk: what
 * the reference CLI's VGA / STEPDEPTH steps analyse after loadGraph (runmethods.cpp:33). */
int dmx_chunk_load(dmx_ctx* ctx, const dmx_chunk* c, const double* region, dmx_pointmap** pm, dmx_graph** g);
/* Device graph from host node records (e.g. a graph the reference itself built or loaded). */
int dmx_graph_from_runs(dmx_ctx* ctx, dmx_pointmap* pm, int64_t nnodes, const int32_t* bins, const int16_t* runs,
                        int64_t nruns, const uint8_t* gridconn, const float* attrs, dmx_graph** out);
/* Merge links (Point::m_merge, set by the LINK mode / PointMap::mergePixels, salalib/pointdata.cpp:1653-1680):
 * n pairs (cell, partner cell) of x-major indices; a pair may be listed in both directions (as
 * PointMap::write stores it on both points); a cell belongs to at most one link (DMX_ERR_ARG otherwise).
 * dmx_chunk_load sets them from the chunk.  Every search that follows merge links in the reference
 * follows them here, with the reference's bookkeeping of the partner: VGA global (vgavisualglobal.cpp:
 * 113-122), visual step depth (vgavisualglobaldepth.cpp:55-63), metric / angular all sources
 * (vgametric.cpp:97-105, vgaangular.cpp:95-104) and metric / angular step depth (vgametricdepth.cpp:68-83,
 * vgaangulardepth.cpp:57-67).  Both ends must be filled cells of the graph (DMX_ERR_ARG at the analysis).
 * A link with one end CONTEXTFILLED at an odd PixelRef is followed exactly too: where the reference's result
 * depends on its pop order inside a level (VGA global with a radius where a source finds both ends at one
 * level; visual step depth where extracting the unexpanded end would reach a new cell) that source or search
 * is run again in the reference's own level order (kernels/vga_ordered.hip).  VGA visual local has no merge
 * logic.  The links are set on the
 * graph's point map as well (they belong to the points: a chunk written from it saves them).  A chunk
 * (dmx_chunk_merges, dmx_chunk_load) must store every link on both of its points (DMX_ERR_ARG otherwise). */
int dmx_graph_set_merges(dmx_graph* g, const int32_t* cell_pairs, int64_t n);
/* The drawing ([n][4] lines x1,y1,x2,y2, the MetaGraph's drawing layers) the graph's point map was made from.  A
 * graph read back from a .graph file is asymmetric at scale: PixelVec::write stores each run after a bin's first
 * as a 4-bit row shift (salalib/ngraph.cpp:536-583), so a jump of more than 15 rows moves every later run of the
 * bin, and Bin::write's unsigned short node count drops the runs of a bin of 65536 k cells (:447-472).  With the
 * drawing, VGA global makes the map's graph again as a symmetric reference and runs the tile search on it, the
 * nodes whose runs differ pushing their own runs (exact; DESIGN.md section 2, asymmetric mode); without it, such
 * a graph takes the top-down search.  Replaces nothing in the reference: its VGA walks the re-read runs as they
 * are (vgavisualglobal.cpp:96-128), which this reproduces. */
int dmx_graph_set_drawing(dmx_graph* g, const double* lines, int64_t nlines);
/* The same links on a point map: written into its PointMap chunk (Point::write, point.cpp:51-73) and
 * followed by the graphs made from it (dmx_makegraph, dmx_graph_assemble_device, dmx_graph_from_runs). */
int dmx_pointmap_set_merges(dmx_pointmap* pm, const int32_t* cell_pairs, int64_t n);
/* The merge links stored in a chunk, one entry per link (cell < partner cell): *n in = capacity of
 * cell_pairs ([n][2]), out = number of links; cell_pairs NULL: only *n. */
int dmx_chunk_merges(const dmx_chunk* c, int32_t* cell_pairs, int64_t* n);
/* Editing a parsed chunk the way the reference edits a PointMap it read (PointMap::read then ::write,
 * pointdata.cpp:1073-1188): columns that are not set keep their bytes (stats, display parameters,
 * formula), point records are re-emitted with the state bits PointMap::read keeps.
 * processed / boundary flags, points with merge links, attribute rows. */
int dmx_chunk_flags(const dmx_chunk* c, int* processed, int* boundary, int64_t* merges, int64_t* nrows);
/* AttributeTable::insertOrResetColumn / insertOrResetLockedColumn (attributetable.cpp:303-326) + setValue on
 * the rows of setmask (NULL: all; values [nrows] in row = node order); make_displayed: the analysis's
 * setDisplayedAttribute.  The chunk's dmx_chunk_column / dmx_chunk_info views are not refreshed. */
int dmx_chunk_set_column(dmx_chunk* c, const char* name, const float* values, const uint8_t* setmask, int locked,
                         int make_displayed);
int dmx_chunk_set_displayed(dmx_chunk* c, int physical_column);
int dmx_chunk_set_name(dmx_chunk* c, const char* name);
/* PointMap::setCurSel(r, add) of the STEPDEPTH selection (runmethods.cpp:745-753): Point::SELECTED on the
 * filled cells among `cells` (x-major indices); MetaGraph::write then saves it. */
int dmx_chunk_select_cells(dmx_chunk* c, const int32_t* cells, int64_t n);
/* PointMap::unmake(removeLinks) (pointdata.cpp:1343-1374): VISPREP -pu [-pl]. */
int dmx_chunk_unmake(dmx_chunk* c, int remove_links);
/* PointMap::write of the (edited) chunk; buf NULL or cap too small: only *size. */
int dmx_chunk_serialize(const dmx_chunk* c, uint8_t* buf, int64_t cap, int64_t* size);

/* ---- .graph file (host) ---------------------------------------------------------------------- */
/* The MetaGraph container, METAGRAPH_VERSION 440: MetaGraph::readFromFile / readFromStream
 * (salalib/mgraph.cpp:2475-2654) and MetaGraph::write(file, 440, false) (mgraph.cpp:2656-2757, as
 * depthmapXcli calls it, runmethods.cpp:113,265,339,776).  Drawing layers (SpacePixelFile / ShapeMap /
 * SalaShape, spacepixfile.cpp:28-57, shapemap.cpp:49-76,2273-2449) are parsed and re-emitted as the
 * reference re-emits them; point maps are PointMap chunks (dmx_chunk_*); shape graphs and data maps are
 * carried through unchanged.  Older file versions need the reference's legacy mgraph440 reader:
 * DMX_ERR_UNSUPPORTED. */
typedef struct dmx_graphfile dmx_graphfile;
int dmx_graphfile_read(const char* path, dmx_graphfile** out);
int dmx_graphfile_free(dmx_graphfile* g);
int dmx_graphfile_write(const dmx_graphfile* g, const char* path);
/* MetaGraph m_state / m_view_class, m_region ([4] blx, bly, trx, try), the drawing lines PointMap::blockLines
 * reads (every shown layer, pointdata.cpp:308-320), point map count, displayed point map. */
int dmx_graphfile_info(const dmx_graphfile* g, int32_t* state, int32_t* view_class, double* region, int64_t* nlines,
                       int32_t* npointmaps, int32_t* displayed);
int dmx_graphfile_lines(const dmx_graphfile* g, double* lines /* [nlines][4] */);
int dmx_graphfile_set_view(dmx_graphfile* g, int32_t state, int32_t view_class);
/* Point map i (the pointer stays valid until the next put on the same file). */
int dmx_graphfile_pointmap(const dmx_graphfile* g, int i, const uint8_t** chunk, int64_t* size);
/* Replace point map i, or (i = -1) append it and make it the displayed one (MetaGraph::addNewPointMap). */
int dmx_graphfile_put_pointmap(dmx_graphfile* g, int i, const uint8_t* chunk, int64_t size);
/* The name addNewPointMap gives the next map ("VGA Map", then "VGA Map 1", ...; mgraph.cpp:2791-2809). */
int dmx_graphfile_new_pointmap_name(const dmx_graphfile* g, char* name, int cap);
/* MetaGraph::setViewClass(SHOWVGATOP) applied to a view class (mgraph.cpp:167-177). */
int32_t dmx_view_vga_top(int32_t view_class);

#ifdef __cplusplus
}
#endif
#endif
