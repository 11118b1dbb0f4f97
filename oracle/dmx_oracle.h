/* dmx_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement (plain C) of the depthmapX VISPREP makeGraph + VGA global path, used
 * as the parity checker for the MI355X engine and as the "port" CPU baseline in bench.py.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.  Every function
 * cites the reference file:line it restates (paths relative to orange-vertex/depthmapX).
 *
 * Pinned against the real reference: tests/test_oracle_golden.py compares it with the outputs of
 * oracle/_ref/ref_probe (the reference salalib compiled from source) committed under tests/golden/.
 */
#ifndef DMX_ORACLE_H
#define DMX_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct dmxo_map dmxo_map;

/* MetaGraph region + PointMap::setGrid(spacing, (0,0)) (pointdata.cpp:122-171), drawing lines as
 * blockLines() sees them (pointdata.cpp:308-320). lines: [L][4] = x1,y1,x2,y2. */
dmxo_map* dmxo_create(const double region[4], double spacing, const double* lines, int64_t nlines);
void dmxo_free(dmxo_map* m);
/* A grid as a .graph PointMap chunk stores it (PointMap::read, pointdata.cpp:1073-1156), no drawing;
 * dmxo_set_state then gives the cell states and dmxo_set_graph the nodes. */
dmxo_map* dmxo_create_grid(int cols, int rows, double spacing, double bl_x, double bl_y);
void dmxo_set_state(dmxo_map* m, const int32_t* state);
void dmxo_grid_info(const dmxo_map* m, int32_t* cols, int32_t* rows, double* bl_x, double* bl_y);

/* PointMap::makePoints(seed, FULLFILL) (pointdata.cpp:402-481). Returns 1 on success, 0 if the
 * reference would return false. */
int dmxo_fill(dmxo_map* m, double x, double y);
/* makePoints with fill_type 0/1/2 (pointdata.cpp:402-481); -1: an AUGMENT fill that does not end. */
int dmxo_fill_type(dmxo_map* m, double x, double y, int fill_type);
/* Test knob: VGA global / visual step depth walk each level front to back (1) or, as the reference, back
 * to front (0, the default).  Shows which results depend on the pop order inside a level. */
void dmxo_set_pop_forward(int forward);

/* Per-cell state (x-major, cols*rows) and cropped cell lines (after blockLines). */
void dmxo_get_state(const dmxo_map* m, int32_t* out);
int64_t dmxo_cell_lines_count(const dmxo_map* m);
void dmxo_get_cell_lines(const dmxo_map* m, int32_t* counts /*C*/, double* lines /*[total][4]*/);

/* PointMap::sparkGraph2 (pointdata.cpp:1246-1341) for filled nodes [node_begin, node_end) in
 * x-major order (node_end < 0: all).  nthreads > 1 runs sources in parallel (OpenMP); results are
 * identical to the sequential order because each source is independent. */
int dmxo_makegraph(dmxo_map* m, double maxdist, int boundary, int64_t node_begin, int64_t node_end,
                   int nthreads);
int64_t dmxo_num_nodes(const dmxo_map* m);
int64_t dmxo_num_runs(const dmxo_map* m);
/* attrs [N][3] (Connectivity, First, Second Moment); bins [N][32][4] (dir, count, dist bits, nruns);
 * runs [R][4] int16 (x0,y0,x1,y1) in reference order; gridconn [N]. */
void dmxo_get_graph(const dmxo_map* m, float* attrs, int32_t* bins, int16_t* runs, uint8_t* gridconn);
/* Merge links (Point::m_merge, PointMap::mergePixels pointdata.cpp:1653-1680): n pairs of distinct
 * x-major cells.  VGA global, visual / metric / angular step depth and VGA metric / angular then
 * follow them as the reference does (getMergePixel blocks of the vgamodules).  Returns -1 on a bad pair. */
int dmxo_set_merges(dmxo_map* m, const int32_t* cell_pairs, int64_t n);
/* Replace the graph with externally supplied bins/runs (e.g. a reference dump), same layout. */
int dmxo_set_graph(dmxo_map* m, const int32_t* bins, const int16_t* runs, int64_t nruns);
/* same, borrowing `runs` (kept alive by the caller) instead of copying it */
int dmxo_set_graph_view(dmxo_map* m, const int32_t* bins, const int16_t* runs, int64_t nruns);

/* VGAVisualGlobal::run (vgamodules/vgavisualglobal.cpp:23-216) for source nodes
 * [node_begin, node_end).  out [N][7] in column order: Visual Entropy, Integration [HH],
 * Integration [P-value], Integration [Tekl], Mean Depth, Node Count, Relativised Entropy
 * (rows outside the range are left untouched).  levels_out (optional, [N][3]) receives
 * total_nodes, total_depth, number of levels. */
int dmxo_vga_global(dmxo_map* m, double radius, int gates_only, int64_t node_begin, int64_t node_end,
                    int nthreads, float* out, int64_t* levels_out);

/* VGAMetricDepth::run (vgamodules/vgametricdepth.cpp:23-92) from the selected cells (x-major cell
 * indices, in std::set<int> PixelRef order, all FILLED).  out [N][3]: Metric Step Shortest-Path
 * Angle, Metric Step Shortest-Path Length, Metric Straight-Line Distance (single selection only;
 * otherwise -1); unreached cells keep -1.  Returns -1 for an empty selection. */
int dmxo_metric_stepdepth(dmxo_map* m, const int32_t* sel_cells, int64_t nsel, float* out);
/* VGAMetric::run (vgamodules/vgametric.cpp:26-136) for source nodes [node_begin, node_end),
 * radius < 0 for "n".  out [N][4]: Metric Mean Shortest-Path Angle, Metric Mean Shortest-Path
 * Distance, Metric Mean Straight-Line Distance, Metric Node Count (-1 rows with gates_only). */
int dmxo_vga_metric(dmxo_map* m, double radius, int gates_only, int64_t node_begin, int64_t node_end, int nthreads,
                    float* out);
/* VGAAngularDepth::run (vgamodules/vgaangulardepth.cpp:23-75): out [N] Angular Step Depth, -1
 * unreached.  Returns -1 for an empty selection. */
int dmxo_angular_stepdepth(dmxo_map* m, const int32_t* sel_cells, int64_t nsel, float* out);
/* VGAAngular::run (vgamodules/vgaangular.cpp:26-133), radius < 0 for "n".  out [N][3]: Angular Mean
 * Depth, Angular Total Depth, Angular Node Count (-1 rows with gates_only). */
int dmxo_vga_angular(dmxo_map* m, double radius, int gates_only, int64_t node_begin, int64_t node_end, int nthreads,
                     float* out);
/* VGAVisualGlobalDepth::run (vgamodules/vgavisualglobaldepth.cpp:23-77): out [N], -1 unreached. */
int dmxo_visual_stepdepth(dmxo_map* m, const int32_t* sel_cells, int64_t nsel, float* out);
/* VGAVisualLocal::run (vgamodules/vgavisuallocal.cpp:23-117) for source nodes [node_begin,
 * node_end).  out [N][3]: Visual Clustering Coefficient, Visual Control, Visual Controllability;
 * -1 for skipped sources (context-filled odd cells, gates_only) and for neighbourhoods of <= 1 cell;
 * rows outside the range untouched. */
int dmxo_vga_local(dmxo_map* m, int gates_only, int64_t node_begin, int64_t node_end, int nthreads, float* out);
/* CPU-baseline sampling (bench.py): makeGraph / VGA global for a list of nodes, one node per thread,
 * per-node wall seconds in secs[n]. */
int dmxo_makegraph_sample(dmxo_map* m, double maxdist, const int64_t* nodes, int64_t n, int nthreads, double* secs);
/* Chunked whole-map sweep (tests/golden/gen_mk_digests.py): sparkGraph2 + addGridConnections of nodes
 * [nb, ne) into the map's node arrays (allocated on first use), read back in dmxo_get_graph's layout, and
 * the chunk's runs freed again. */
int dmxo_makegraph_range(dmxo_map* m, double maxdist, int64_t nb, int64_t ne, int nthreads);
int64_t dmxo_num_runs_range(const dmxo_map* m, int64_t nb, int64_t ne);
void dmxo_get_graph_range(const dmxo_map* m, int64_t nb, int64_t ne, float* attrs, int32_t* bins, int16_t* runs,
                          uint8_t* gridconn);
void dmxo_release_range(dmxo_map* m, int64_t nb, int64_t ne);
int dmxo_vga_global_sample(dmxo_map* m, double radius, const int64_t* nodes, int64_t n, int nthreads, float* out,
                           double* secs);

#ifdef __cplusplus
}
#endif
#endif
