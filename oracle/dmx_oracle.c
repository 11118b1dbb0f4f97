/* dmx_oracle.c -- TEST INFRASTRUCTURE ONLY (see dmx_oracle.h).
 *
 * Clean-room plain-C restatement of the depthmapX visibility-graph path.  It is the checker the
 * MI355X engine is compared against and the "port" CPU baseline; the product never links it.
 * All arithmetic follows the reference's IEEE-double operation order (compiled with
 * -ffp-contract=off).  Reference citations are file:line in orange-vertex/depthmapX.
 */
#include "dmx_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define M_1_LN2_ 1.4426950408889634073599246810019
#define M_PI_ 3.14159265358979323846

/* Point::m_state bits (salalib/point.h:32-38) */
/* Test knob (dmxo_set_pop_forward): walk each BFS level front to back instead of the reference's back
 * to front (rbegin, vgavisualglobal.cpp:99, vgavisualglobaldepth.cpp:46).  Used only to show which
 * results depend on the pop order inside a level; 0 (the reference's order) by default. */
static int g_pop_forward = 0;
void dmxo_set_pop_forward(int forward) { g_pop_forward = forward; }

enum { ST_EMPTY = 0x1, ST_FILLED = 0x2, ST_BLOCKED = 0x4, ST_CONTEXTFILLED = 0x8, ST_EDGE = 0x20, ST_AUGMENTED = 0x8000 };
/* PixelRef directions (salalib/pixelref.h:46) */
enum { D_NODIR = 0, D_H = 1, D_V = 2, D_PD = 4, D_ND = 8, D_DIAG = 12, D_NH = 16, D_NV = 32 };

/* ---------------------------------------------------------------- geometry (genlib/p2dpoly) */
typedef struct { double x, y; } P2;
typedef struct { double blx, bly, trx, try_; } Reg;            /* QtRegion */
typedef struct { Reg r; char parity, direction; } Line;        /* Line : QtRegion (p2dpoly.h:398) */

static Line line_make(P2 a, P2 b) { /* Line::Line (p2dpoly.cpp:291-336) */
    Line l;
    if (a.x == b.x) {
        l.r.blx = a.x; l.r.trx = b.x;
        if (a.y <= b.y) { l.r.bly = a.y; l.r.try_ = b.y; l.parity = 1; l.direction = 1; }
        else { l.r.bly = b.y; l.r.try_ = a.y; l.parity = 1; l.direction = 0; }
    } else if (a.x < b.x) {
        l.r.blx = a.x; l.r.trx = b.x;
        if (a.y <= b.y) { l.r.bly = a.y; l.r.try_ = b.y; l.parity = 1; l.direction = 1; }
        else { l.r.bly = b.y; l.r.try_ = a.y; l.parity = 0; l.direction = 1; }
    } else {
        l.r.blx = b.x; l.r.trx = a.x;
        if (b.y <= a.y) { l.r.bly = b.y; l.r.try_ = a.y; l.parity = 1; l.direction = 0; }
        else { l.r.bly = a.y; l.r.try_ = b.y; l.parity = 0; l.direction = 0; }
    }
    return l;
}
/* accessors p2dpoly.h:452-470 */
static inline double L_ax(const Line* l) { return l->r.blx; }
static inline double L_bx(const Line* l) { return l->r.trx; }
static inline double L_ay(const Line* l) { return l->parity ? l->r.bly : l->r.try_; }
static inline double L_by(const Line* l) { return l->parity ? l->r.try_ : l->r.bly; }
static inline double* L_ayp(Line* l) { return l->parity ? &l->r.bly : &l->r.try_; }
static inline double* L_byp(Line* l) { return l->parity ? &l->r.try_ : &l->r.bly; }
static inline double R_w(const Reg* r) { return fabs(r->trx - r->blx); }  /* p2dpoly.h:306-318 */
static inline double R_h(const Reg* r) { return fabs(r->try_ - r->bly); }
static inline double L_sign(const Line* l) { return l->parity ? 1.0 : -1.0; }
static inline P2 L_start(const Line* l) { P2 p = {l->r.blx, L_ay(l)}; return p; }
static inline P2 L_end(const Line* l) { P2 p = {l->r.trx, L_by(l)}; return p; }
static inline double L_len(const Line* l) { /* p2dpoly.h:476 */
    return sqrt((l->r.trx - l->r.blx) * (l->r.trx - l->r.blx) + (l->r.try_ - l->r.bly) * (l->r.try_ - l->r.bly));
}

static int overlap_x(const Reg* a, const Reg* b, double tol) { /* p2dpoly.cpp:255-266 */
    if (a->blx > b->blx) return b->trx >= a->blx - tol;
    return a->trx >= b->blx - tol;
}
static int overlap_y(const Reg* a, const Reg* b, double tol) { /* p2dpoly.cpp:268-279 */
    if (a->bly > b->bly) return b->try_ >= a->bly - tol;
    return a->try_ >= b->bly - tol;
}
static int intersect_region(const Reg* a, const Reg* b, double tol) { /* p2dpoly.cpp:247-253 */
    return overlap_x(a, b, tol) && overlap_y(a, b, tol);
}
static int intersect_line(const Line* a, const Line* b, double tol) { /* p2dpoly.cpp:350-363 */
    if (((L_ay(a) - L_by(a)) * (L_ax(b) - L_ax(a)) + (L_bx(a) - L_ax(a)) * (L_ay(b) - L_ay(a))) *
                ((L_ay(a) - L_by(a)) * (L_bx(b) - L_ax(a)) + (L_bx(a) - L_ax(a)) * (L_by(b) - L_ay(a))) <= tol &&
        ((L_ay(b) - L_by(b)) * (L_ax(a) - L_ax(b)) + (L_bx(b) - L_ax(b)) * (L_ay(a) - L_ay(b))) *
                ((L_ay(b) - L_by(b)) * (L_bx(a) - L_ax(b)) + (L_bx(b) - L_ax(b)) * (L_by(a) - L_ay(b))) <= tol)
        return 1;
    return 0;
}
static int intersect_line_no_touch(const Line* a, const Line* b, double tol) { /* p2dpoly.cpp:368-381 */
    if (((L_ay(a) - L_by(a)) * (L_ax(b) - L_ax(a)) + (L_bx(a) - L_ax(a)) * (L_ay(b) - L_ay(a))) *
                ((L_ay(a) - L_by(a)) * (L_bx(b) - L_ax(a)) + (L_bx(a) - L_ax(a)) * (L_by(b) - L_ay(a))) < -tol &&
        ((L_ay(b) - L_by(b)) * (L_ax(a) - L_ax(b)) + (L_bx(b) - L_ax(b)) * (L_ay(a) - L_ay(b))) *
                ((L_ay(b) - L_by(b)) * (L_bx(a) - L_ax(b)) + (L_bx(b) - L_ax(b)) * (L_by(a) - L_ay(b))) < -tol)
        return 1;
    return 0;
}
static int line_crop(Line* l, const Reg* r) { /* Line::crop (p2dpoly.cpp:626-667) */
    if (L_bx(l) >= r->blx) {
        if (L_ax(l) < r->blx) {
            *L_ayp(l) += L_sign(l) * (R_h(&l->r) * (r->blx - L_ax(l)) / R_w(&l->r));
            l->r.blx = r->blx;
        }
        if (L_ax(l) <= r->trx) {
            if (L_bx(l) > r->trx) {
                *L_byp(l) -= L_sign(l) * R_h(&l->r) * (L_bx(l) - r->trx) / R_w(&l->r);
                l->r.trx = r->trx;
            }
            if (l->r.try_ >= r->bly) {
                if (l->r.bly < r->bly) {
                    if (l->parity) l->r.blx += R_w(&l->r) * (r->bly - l->r.bly) / R_h(&l->r);
                    else l->r.trx -= R_w(&l->r) * (r->bly - l->r.bly) / R_h(&l->r);
                    l->r.bly = r->bly;
                }
                if (l->r.bly <= r->try_) {
                    if (l->r.try_ > r->try_) {
                        if (l->parity) l->r.trx -= R_w(&l->r) * (l->r.try_ - r->try_) / R_h(&l->r);
                        else l->r.blx += R_w(&l->r) * (l->r.try_ - r->try_) / R_h(&l->r);
                        l->r.try_ = r->try_;
                    }
                    return 1;
                }
            }
        }
    }
    return 0;
}

/* ---------------------------------------------------------------- growable arrays */
typedef struct { void* p; int64_t n, cap; } Vec;
static void* vec_push(Vec* v, size_t sz) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 16;
        v->p = realloc(v->p, (size_t)v->cap * sz);
    }
    return (char*)v->p + (size_t)(v->n++) * sz;
}

/* ---------------------------------------------------------------- map */
typedef struct { int16_t x0, y0, x1, y1; } Run;
typedef struct {
    char dir[32];
    uint16_t count[32];
    float dist[32];
    int32_t nruns[32];
    Run* runs; /* concatenated over bins 0..31 */
    int64_t total_runs;
} NodeG;

struct dmxo_map {
    Reg parent;          /* MetaGraph region */
    double spacing;
    int cols, rows;
    P2 bl;               /* m_bottom_left */
    Reg region;          /* PixelBase::m_region */
    int32_t* state;      /* x-major */
    int blocked_lines;   /* m_blockedlines */
    const double* draw;  /* copy of drawing lines */
    int64_t ndraw;
    int64_t* cl_off;     /* cell lines CSR (C+1) */
    Line* cl;
    int32_t* node_of_cell; /* -1 if not a node */
    int64_t nnodes;
    int32_t* node_cell;  /* node -> cell index */
    NodeG* nodes;
    float* attrs;        /* [N][3] */
    uint8_t* gridconn;
    int runs_borrowed;   /* nodes[].runs point into a caller's array (dmxo_set_graph_view) */
    int32_t* merge;      /* Point::m_merge per cell: partner cell (x-major) or -1 (point.h:56) */
};

static inline int64_t cidx(const dmxo_map* m, int x, int y) { return (int64_t)x * m->rows + y; }
static inline int incl(const dmxo_map* m, int x, int y) { /* spacepix.h:48-49 */
    return x >= 0 && x < m->cols && y >= 0 && y < m->rows;
}
static inline P2 depixelate(const dmxo_map* m, int x, int y) { /* pointdata.h:353-357 */
    P2 p = {m->bl.x + m->spacing * 1.0 * (double)x, m->bl.y + m->spacing * 1.0 * (double)y};
    return p;
}
static inline Reg regionate(const dmxo_map* m, int x, int y, double border) { /* pointdata.h:359-367 */
    Reg r;
    r.blx = m->bl.x + m->spacing * ((double)x - 0.5 - border);
    r.bly = m->bl.y + m->spacing * ((double)y - 0.5 - border);
    r.trx = m->bl.x + m->spacing * ((double)x + 0.5 + border);
    r.try_ = m->bl.y + m->spacing * ((double)y + 0.5 + border);
    return r;
}

dmxo_map* dmxo_create(const double region[4], double spacing, const double* lines, int64_t nlines) {
    dmxo_map* m = (dmxo_map*)calloc(1, sizeof(dmxo_map));
    m->parent.blx = region[0]; m->parent.bly = region[1]; m->parent.trx = region[2]; m->parent.try_ = region[3];
    /* PointMap::setGrid (pointdata.cpp:122-171), offset (0,0) as runVisualPrep passes */
    m->spacing = spacing;
    double xoffset = fmod(m->parent.blx + 0.0, spacing);
    double yoffset = fmod(m->parent.bly + 0.0, spacing);
    if (xoffset < spacing / 2.0) xoffset += spacing;
    if (xoffset > spacing / 2.0) xoffset -= spacing;
    if (yoffset < spacing / 2.0) yoffset += spacing;
    if (yoffset > spacing / 2.0) yoffset -= spacing;
    double offx = -xoffset, offy = -yoffset;
    m->cols = (int)floor((xoffset + R_w(&m->parent)) / spacing + 0.5) + 1;
    m->rows = (int)floor((yoffset + R_h(&m->parent)) / spacing + 0.5) + 1;
    m->bl.x = m->parent.blx + offx;
    m->bl.y = m->parent.bly + offy;
    m->region.blx = m->bl.x - spacing / 2.0;
    m->region.bly = m->bl.y - spacing / 2.0;
    m->region.trx = m->bl.x + (double)(m->cols - 1) * spacing + spacing / 2.0;
    m->region.try_ = m->bl.y + (double)(m->rows - 1) * spacing + spacing / 2.0;
    int64_t C = (int64_t)m->cols * m->rows;
    m->state = (int32_t*)malloc(C * sizeof(int32_t));
    for (int64_t i = 0; i < C; i++) m->state[i] = ST_EMPTY;
    double* d = (double*)malloc((nlines > 0 ? nlines : 1) * 4 * sizeof(double));
    memcpy(d, lines, nlines * 4 * sizeof(double));
    m->draw = d;
    m->ndraw = nlines;
    m->merge = (int32_t*)malloc(C * sizeof(int32_t));
    for (int64_t i = 0; i < C; i++) m->merge[i] = -1;
    return m;
}

static void release_nodes(dmxo_map* m);
static void index_nodes(dmxo_map* m);

/* A map read back from a .graph PointMap chunk (PointMap::read, pointdata.cpp:1073-1156): the grid as
 * stored (cols, rows, spacing, bottom-left cell centre) and no drawing -- enough to analyse a graph
 * handed over with dmxo_set_state + dmxo_set_graph. */
dmxo_map* dmxo_create_grid(int cols, int rows, double spacing, double blx, double bly) {
    const double region[4] = {blx - spacing / 2.0, bly - spacing / 2.0, blx + spacing * (cols - 0.5),
                              bly + spacing * (rows - 0.5)};
    dmxo_map* m = dmxo_create(region, spacing, NULL, 0);
    if (!m) return NULL;
    free(m->state);
    free(m->merge);
    m->cols = cols;
    m->rows = rows;
    m->bl.x = blx;
    m->bl.y = bly;
    m->region.blx = region[0]; m->region.bly = region[1]; m->region.trx = region[2]; m->region.try_ = region[3];
    const int64_t C = (int64_t)cols * rows;
    m->state = (int32_t*)malloc(C * sizeof(int32_t));
    m->merge = (int32_t*)malloc(C * sizeof(int32_t));
    for (int64_t i = 0; i < C; i++) { m->state[i] = ST_EMPTY; m->merge[i] = -1; }
    return m;
}

/* Cell states as stored (x-major); re-indexes the nodes (filled cells, x-major). */
void dmxo_set_state(dmxo_map* m, const int32_t* state) {
    const int64_t C = (int64_t)m->cols * m->rows;
    memcpy(m->state, state, C * sizeof(int32_t));
    release_nodes(m);
    index_nodes(m);
}

/* PointMap::mergePixels (pointdata.cpp:1653-1680) for each pair: both cells point at each other.
 * Pairs must join two distinct filled cells; a cell in two pairs keeps the last one. */
int dmxo_set_merges(dmxo_map* m, const int32_t* pairs, int64_t n) {
    const int64_t C = (int64_t)m->cols * m->rows;
    for (int64_t i = 0; i < C; i++) m->merge[i] = -1;
    for (int64_t i = 0; i < n; i++) {
        const int32_t a = pairs[2 * i], b = pairs[2 * i + 1];
        if (a < 0 || b < 0 || a >= C || b >= C || a == b) return -1;
        m->merge[a] = b;
        m->merge[b] = a;
    }
    return 0;
}

static void release_nodes(dmxo_map* m) {
    if (m->nodes) {
        if (!m->runs_borrowed)
            for (int64_t i = 0; i < m->nnodes; i++) free(m->nodes[i].runs);
        free(m->nodes);
    }
    m->nodes = NULL;
    m->runs_borrowed = 0;
}

void dmxo_free(dmxo_map* m) {
    if (!m) return;
    free(m->state); free((void*)m->draw); free(m->cl_off); free(m->cl);
    free(m->node_of_cell); free(m->node_cell); free(m->attrs); free(m->gridconn); free(m->merge);
    release_nodes(m);
    free(m);
}

void dmxo_grid_info(const dmxo_map* m, int32_t* cols, int32_t* rows, double* bx, double* by) {
    *cols = m->cols; *rows = m->rows; *bx = m->bl.x; *by = m->bl.y;
}

/* PixelBase::pixelateLineTouching (spacepix.cpp:144-214); emits cell indices via callback arrays */
static int64_t pixelate_touching(const dmxo_map* m, Line l, double tol, int32_t* outx, int32_t* outy) {
    int64_t n = 0;
    const Reg* r = &m->region;
    /* l.normalScale(m_region): top_right then bottom_left (p2dpoly.h:321-324, :370-379) */
    double rw = R_w(r), rh = R_h(r);
    if (rw) l.r.trx = (l.r.trx - r->blx) / rw; else l.r.trx = 0.0;
    if (rh) l.r.try_ = (l.r.try_ - r->bly) / rh; else l.r.try_ = 0.0;
    if (rw) l.r.blx = (l.r.blx - r->blx) / rw; else l.r.blx = 0.0;
    if (rh) l.r.bly = (l.r.bly - r->bly) / rh; else l.r.bly = 0.0;
    /* l.scale(Point2f(cols, rows)) */
    l.r.trx *= (double)m->cols; l.r.try_ *= (double)m->rows;
    l.r.blx *= (double)m->cols; l.r.bly *= (double)m->rows;
    double grad, constant;
    int dirx;
    if (R_w(&l.r) > R_h(&l.r)) {
        dirx = 1;
        grad = L_sign(&l) * R_h(&l.r) / R_w(&l.r);           /* grad(YAXIS) p2dpoly.h:468 */
        constant = L_ay(&l) - grad * L_ax(&l);               /* constant(YAXIS) */
    } else {
        dirx = 0;
        grad = L_sign(&l) * R_w(&l.r) / R_h(&l.r);           /* grad(XAXIS) */
        constant = L_ax(&l) - grad * L_ay(&l);               /* constant(XAXIS) */
    }
#define ENCL(X, Y) ((short)(X) >= 0 && (short)(X) < (short)m->cols && (short)(Y) >= 0 && (short)(Y) < (short)m->rows)
#define PUSH(X, Y) do { if (ENCL(X, Y)) { if (outx) { outx[n] = (short)(X); outy[n] = (short)(Y); } n++; } } while (0)
    if (dirx) {
        int first = (int)floor(L_ax(&l) - tol);
        int last = (int)floor(L_bx(&l) + tol);
        for (int i = first; i <= last; i++) {
            int j1 = (int)floor((first == i ? L_ax(&l) : (double)i) * grad + constant - L_sign(&l) * tol);
            int j2 = (int)floor((last == i ? L_bx(&l) : (double)(i + 1)) * grad + constant + L_sign(&l) * tol);
            PUSH(i, j1);
            if (j1 != j2) {
                PUSH(i, j2);
                if (abs(j2 - j1) == 2) { int j3 = (j1 + j2) / 2; PUSH(i, j3); }
            }
        }
    } else {
        int first = (int)floor(l.r.bly - tol);
        int last = (int)floor(l.r.try_ + tol);
        for (int i = first; i <= last; i++) {
            int j1 = (int)floor((first == i ? l.r.bly : (double)i) * grad + constant - L_sign(&l) * tol);
            int j2 = (int)floor((last == i ? l.r.try_ : (double)(i + 1)) * grad + constant + L_sign(&l) * tol);
            PUSH(j1, i);
            if (j1 != j2) {
                PUSH(j2, i);
                if (abs(j2 - j1) == 2) { int j3 = (j1 + j2) / 2; PUSH(j3, i); }
            }
        }
    }
#undef PUSH
#undef ENCL
    return n;
}

/* PointMap::blockLines + blockLine (pointdata.cpp:296-357) */
static void block_lines(dmxo_map* m) {
    if (m->blocked_lines) return;
    int64_t C = (int64_t)m->cols * m->rows;
    int64_t* cnt = (int64_t*)calloc(C + 1, sizeof(int64_t));
    int64_t maxn = 0;
    Line* dl = (Line*)malloc((m->ndraw ? m->ndraw : 1) * sizeof(Line));
    for (int64_t k = 0; k < m->ndraw; k++) {
        P2 a = {m->draw[4 * k], m->draw[4 * k + 1]}, b = {m->draw[4 * k + 2], m->draw[4 * k + 3]};
        dl[k] = line_make(a, b);
        int64_t n = pixelate_touching(m, dl[k], 1e-10, NULL, NULL);
        if (n > maxn) maxn = n;
    }
    int32_t* px = (int32_t*)malloc((maxn + 1) * sizeof(int32_t));
    int32_t* py = (int32_t*)malloc((maxn + 1) * sizeof(int32_t));
    for (int64_t k = 0; k < m->ndraw; k++) {
        int64_t n = pixelate_touching(m, dl[k], 1e-10, px, py);
        for (int64_t i = 0; i < n; i++) cnt[cidx(m, px[i], py[i]) + 1]++;
    }
    for (int64_t c = 0; c < C; c++) cnt[c + 1] += cnt[c];
    Line* raw = (Line*)malloc((cnt[C] ? cnt[C] : 1) * sizeof(Line));
    int64_t* fillp = (int64_t*)malloc(C * sizeof(int64_t));
    memcpy(fillp, cnt, C * sizeof(int64_t));
    for (int64_t k = 0; k < m->ndraw; k++) {
        int64_t n = pixelate_touching(m, dl[k], 1e-10, px, py);
        for (int64_t i = 0; i < n; i++) {
            int64_t c = cidx(m, px[i], py[i]);
            raw[fillp[c]++] = dl[k];
            m->state[c] |= ST_BLOCKED; /* Point::setBlock */
        }
    }
    /* crop to regionate(cell, 1e-10), dropping lines outside (pointdata.cpp:323-340) */
    m->cl_off = (int64_t*)calloc(C + 1, sizeof(int64_t));
    m->cl = (Line*)malloc((cnt[C] ? cnt[C] : 1) * sizeof(Line));
    int64_t out = 0;
    for (int x = 0; x < m->cols; x++)
        for (int y = 0; y < m->rows; y++) {
            int64_t c = cidx(m, x, y);
            Reg vp = regionate(m, x, y, 1e-10);
            m->cl_off[c] = out;
            for (int64_t i = cnt[c]; i < cnt[c + 1]; i++) {
                Line l = raw[i];
                if (line_crop(&l, &vp)) m->cl[out++] = l;
            }
        }
    m->cl_off[C] = out;
    free(cnt); free(raw); free(fillp); free(px); free(py); free(dl);
    m->blocked_lines = 1;
}

/* PointMap::expand (pointdata.cpp:483-514); fill_state is makePoints' filltype (:434-441) */
static int expand(dmxo_map* m, int x1, int y1, int x2, int y2, Vec* list, int32_t fill_state) {
    if ((short)x2 < 0 || (short)x2 >= (short)m->cols || (short)y2 < 0 || (short)y2 >= (short)m->rows) return 1;
    int64_t c2 = cidx(m, x2, y2), c1 = cidx(m, x1, y1);
    if (m->state[c2] & ST_FILLED) return 2;
    Line l = line_make(depixelate(m, x1, y1), depixelate(m, x2, y2));
    double tol = m->spacing * 1e-10;
    for (int64_t i = m->cl_off[c1]; i < m->cl_off[c1 + 1]; i++)
        if (intersect_region(&l.r, &m->cl[i].r, tol) && intersect_line(&l, &m->cl[i], tol)) return 4;
    for (int64_t i = m->cl_off[c2]; i < m->cl_off[c2 + 1]; i++)
        if (intersect_region(&l.r, &m->cl[i].r, tol) && intersect_line(&l, &m->cl[i], tol)) return 4;
    m->state[c2] = fill_state | (m->state[c2] & ST_BLOCKED); /* Point::set (point.h:121-125) */
    int32_t* p = (int32_t*)vec_push(list, 2 * sizeof(int32_t));
    p[0] = x2; p[1] = y2;
    return 8;
}

int dmxo_fill(dmxo_map* m, double sx, double sy) { return dmxo_fill_type(m, sx, sy, 0); }

/* PointMap::makePoints(seed, fill_type) (pointdata.cpp:402-481): 0 FULLFILL, 1 SEMIFILL, 2 AUGMENT.
 * The loop is the reference's literal pflipper loop.  An AUGMENT fill sets AUGMENTED without FILLED,
 * which expand does not stop at (:489), so it can run forever: the loop is cut after 64 pops per cell
 * and -1 returned (the state is then garbage; callers discard the map). */
int dmxo_fill_type(dmxo_map* m, double sx, double sy, int fill_type) {
    int32_t fill_state = fill_type == 0 ? ST_FILLED : fill_type == 1 ? (ST_FILLED | ST_CONTEXTFILLED) : ST_AUGMENTED;
    /* runmethods.cpp:269-277 fillGraph: region.contains(point) */
    if (!(sx > m->parent.blx && sx < m->parent.trx && sy > m->parent.bly && sy < m->parent.try_)) return 0;
    /* PointMap::pixelate(p, false) (pointdata.cpp:283-305) */
    double sp = m->spacing / 1.0;
    int px = (short)(int)floor((sx - m->bl.x + (m->spacing / 2.0)) / sp);
    int py = (short)(int)floor((sy - m->bl.y + (m->spacing / 2.0)) / sp);
    if (!incl(m, px, py) || (m->state[cidx(m, px, py)] & ST_FILLED)) return 0;
    /* the seed-visibility test only sees lines once blockLines has run (pointdata.cpp:422-428) */
    if (m->blocked_lines) {
        int64_t c = cidx(m, px, py);
        P2 s = {sx, sy};
        Line ls = line_make(s, depixelate(m, px, py));
        for (int64_t i = m->cl_off[c]; i < m->cl_off[c + 1]; i++)
            if (intersect_line_no_touch(&m->cl[i], &ls, 0.0)) return 0;
    }
    block_lines(m);
    int64_t c0 = cidx(m, px, py);
    m->state[c0] = fill_state | (m->state[c0] & ST_BLOCKED);
    Vec lists[2] = {{0}, {0}};
    const int64_t max_pops = 64 * (int64_t)m->cols * m->rows + 64;
    int64_t pops = 0;
    int par = 0;
    int32_t* p0 = (int32_t*)vec_push(&lists[0], 2 * sizeof(int32_t));
    p0[0] = px; p0[1] = py;
    while (lists[par].n > 0) { /* pflipper surface (pointdata.cpp:450-479) */
        int32_t* cur = (int32_t*)lists[par].p + 2 * (lists[par].n - 1);
        int x = cur[0], y = cur[1];
        Vec* b = &lists[par ^ 1];
        int res = 0;
        res |= expand(m, x, y, x, y + 1, b, fill_state);          /* up */
        res |= expand(m, x, y, x, y - 1, b, fill_state);          /* down */
        res |= expand(m, x, y, x - 1, y, b, fill_state);          /* left */
        res |= expand(m, x, y, x + 1, y, b, fill_state);          /* right */
        res |= expand(m, x, y, x - 1, y + 1, b, fill_state);      /* up-left */
        res |= expand(m, x, y, x + 1, y + 1, b, fill_state);      /* up-right */
        res |= expand(m, x, y, x - 1, y - 1, b, fill_state);      /* down-left */
        res |= expand(m, x, y, x + 1, y - 1, b, fill_state);      /* down-right */
        int64_t c = cidx(m, x, y);
        if ((res & 4) || (m->state[c] & ST_BLOCKED)) m->state[c] |= ST_EDGE;
        lists[par].n--;
        if (lists[par].n == 0) par ^= 1;
        if (++pops > max_pops) {
            free(lists[0].p); free(lists[1].p);
            return -1;
        }
    }
    free(lists[0].p); free(lists[1].p);
    return 1;
}

void dmxo_get_state(const dmxo_map* m, int32_t* out) {
    memcpy(out, m->state, (size_t)m->cols * m->rows * sizeof(int32_t));
}
int64_t dmxo_cell_lines_count(const dmxo_map* m) {
    return m->cl_off ? m->cl_off[(int64_t)m->cols * m->rows] : 0;
}
void dmxo_get_cell_lines(const dmxo_map* m, int32_t* counts, double* lines) {
    int64_t C = (int64_t)m->cols * m->rows;
    for (int64_t c = 0; c < C; c++) {
        counts[c] = m->cl_off ? (int32_t)(m->cl_off[c + 1] - m->cl_off[c]) : 0;
    }
    int64_t n = dmxo_cell_lines_count(m);
    for (int64_t i = 0; i < n; i++) {
        P2 s = L_start(&m->cl[i]), e = L_end(&m->cl[i]);
        lines[4 * i] = s.x; lines[4 * i + 1] = s.y; lines[4 * i + 2] = e.x; lines[4 * i + 3] = e.y;
    }
}

/* ---------------------------------------------------------------- spark sieve (sparksieve2.cpp) */
typedef struct { double start, end; } Zone;
typedef struct {
    P2 centre;
    double maxdist;
    Zone* gaps; int ng, capg;
    Zone* blocks; int nb, capb;
} Sieve;

static double tanify(const Sieve* s, P2 p, int q) { /* sparksieve2.cpp:143-173 */
    switch (q) {
    case 0: return (p.y - s->centre.y) / (s->centre.x - p.x);
    case 1: return (p.y - s->centre.y) / (p.x - s->centre.x);
    case 2: return (s->centre.y - p.y) / (s->centre.x - p.x);
    case 3: return (s->centre.y - p.y) / (p.x - s->centre.x);
    case 4: return (s->centre.x - p.x) / (s->centre.y - p.y);
    case 5: return (p.x - s->centre.x) / (s->centre.y - p.y);
    case 6: return (s->centre.x - p.x) / (p.y - s->centre.y);
    case 7: return (p.x - s->centre.x) / (p.y - s->centre.y);
    }
    return -1.0;
}
static void sieve_block(Sieve* s, const Line* lines, int64_t n, int q) { /* sparksieve2.cpp:67-87 */
    for (int64_t i = 0; i < n; i++) {
        double a = tanify(s, L_start(&lines[i]), q);
        double b = tanify(s, L_end(&lines[i]), q);
        if (s->nb == s->capb) { s->capb = s->capb ? 2 * s->capb : 64; s->blocks = (Zone*)realloc(s->blocks, s->capb * sizeof(Zone)); }
        Zone z;
        if (a < b) { z.start = a - 1e-10; z.end = b + 1e-10; }
        else { z.start = b - 1e-10; z.end = a + 1e-10; }
        s->blocks[s->nb++] = z;
    }
}
static int zone_less(const Zone* a, const Zone* b) { /* sparksieve2.h:72-75 */
    return (a->start == b->start) ? (a->end > b->end) : (a->start < b->start);
}
static int zone_cmp(const void* pa, const void* pb) {
    const Zone* a = (const Zone*)pa; const Zone* b = (const Zone*)pb;
    if (zone_less(a, b)) return -1;
    if (zone_less(b, a)) return 1;
    return 0;
}
/* std::sort + std::unique of the accumulated blocks, then the gap merge (sparksieve2.cpp:89-132) */
static void sieve_collectgarbage(Sieve* s) {
    if (s->nb > 1) {
        qsort(s->blocks, s->nb, sizeof(Zone), zone_cmp);
        int w = 1;
        for (int i = 1; i < s->nb; i++)
            if (!(s->blocks[i].start == s->blocks[w - 1].start && s->blocks[i].end == s->blocks[w - 1].end))
                s->blocks[w++] = s->blocks[i];
        s->nb = w;
    }
    /* gaps live in an array; erase/insert shift the tail (std::list semantics preserved) */
    int gi = 0, bi = 0;
    while (bi < s->nb && gi < s->ng) {
        Zone* blk = &s->blocks[bi];
        Zone* g = &s->gaps[gi];
        if (blk->end < g->start) { bi++; continue; }
        int create = 1;
        if (blk->start <= g->start) {
            create = 0;
            if (blk->end > g->start) g->start = blk->end;
        }
        if (blk->end >= g->end) {
            create = 0;
            if (blk->start < g->end) g->end = blk->start;
        }
        if (g->end <= g->start + 1e-10) {
            memmove(&s->gaps[gi], &s->gaps[gi + 1], (s->ng - gi - 1) * sizeof(Zone));
            s->ng--;
            continue;
        } else if (blk->end > g->end) {
            gi++;
            continue;
        } else if (create) {
            if (s->ng == s->capg) { s->capg *= 2; s->gaps = (Zone*)realloc(s->gaps, s->capg * sizeof(Zone)); g = &s->gaps[gi]; }
            memmove(&s->gaps[gi + 1], &s->gaps[gi], (s->ng - gi) * sizeof(Zone));
            s->ng++;
            s->gaps[gi].start = s->gaps[gi + 1].start;
            s->gaps[gi].end = blk->start;
            gi++;
            s->gaps[gi].start = blk->end;
        }
        bi++;
    }
    s->nb = 0;
}
static int sieve_testblock(const Sieve* s, P2 pt, const Line* lines, int64_t n, double tol) { /* :45-63 */
    Line l = line_make(s->centre, pt);
    if (s->maxdist != -1.0 && L_len(&l) > s->maxdist) return 1;
    for (int64_t i = 0; i < n; i++)
        if (intersect_region(&l.r, &lines[i].r, tol) && intersect_line(&l, &lines[i], tol)) return 1;
    return 0;
}

/* whichbin (pointdata.h:432-520) */
static int whichbin(P2 grad) {
    int bin = 0;
    double ratio;
    if (fabs(grad.y) > fabs(grad.x)) bin = 1;
    if (bin == 0) {
        ratio = fabs(grad.y) / fabs(grad.x);
        if (grad.x > 0.0) bin = (grad.y >= 0.0) ? 0 : -32;
        else bin = (grad.y >= 0.0) ? -16 : 16;
    } else {
        ratio = fabs(grad.x) / fabs(grad.y);
        if (grad.y > 0.0) bin = (grad.x >= 0.0) ? -8 : 8;
        else bin = (grad.x >= 0.0) ? 24 : -24;
    }
    if (ratio < 1e-12) {
    } else if (ratio < 0.2679491924311227) bin += 1;
    else if (ratio < 0.5773502691896257) bin += 2;
    else if (ratio < 1.0 - 1e-12) bin += 3;
    else bin += 4;
    if (bin < 0) bin = -bin;
    bin = bin % 32;
    return bin;
}

/* per-thread scratch for one source */
typedef struct { int32_t x, y; } Pix;
typedef struct {
    Sieve sv;
    Vec bins[32];   /* Pix */
    Vec add;        /* Pix */
    Vec sortbuf;    /* Pix */
    Line* lines0; int cap0;
} Work;

static int pixH_cmp(const void* a, const void* b) { /* PixelRefH (ngraph.h:153-170): (y, x) */
    const Pix* p = (const Pix*)a; const Pix* q = (const Pix*)b;
    if (p->y != q->y) return p->y < q->y ? -1 : 1;
    if (p->x != q->x) return p->x < q->x ? -1 : 1;
    return 0;
}
static int pixV_cmp(const void* a, const void* b) { /* PixelRefV: (x, y) */
    const Pix* p = (const Pix*)a; const Pix* q = (const Pix*)b;
    if (p->x != q->x) return p->x < q->x ? -1 : 1;
    if (p->y != q->y) return p->y < q->y ? -1 : 1;
    return 0;
}

/* Bin::make (ngraph.cpp:234-304); appends runs to rv, returns nruns */
static int bin_make(Work* w, const Pix* px, int64_t n, char dir, Vec* rv, uint16_t* count) {
    if (n == 0) return 0;
    *count = (uint16_t)n;
    if (dir & D_DIAG) {
        Pix s = px[0], e = px[0];
        if (px[n - 1].x < s.x) s = px[n - 1];
        if (px[n - 1].x > e.x) e = px[n - 1];
        Run* r = (Run*)vec_push(rv, sizeof(Run));
        r->x0 = s.x; r->y0 = s.y; r->x1 = e.x; r->y1 = e.y;
        return 1;
    }
    w->sortbuf.n = 0;
    for (int64_t i = 0; i < n; i++) *(Pix*)vec_push(&w->sortbuf, sizeof(Pix)) = px[i];
    Pix* b = (Pix*)w->sortbuf.p;
    qsort(b, n, sizeof(Pix), dir == D_H ? pixH_cmp : pixV_cmp);
    int64_t u = 1; /* std::set dedup */
    for (int64_t i = 1; i < n; i++) if (b[i].x != b[u - 1].x || b[i].y != b[u - 1].y) b[u++] = b[i];
    int nr = 0;
    Run* cur = (Run*)vec_push(rv, sizeof(Run)); nr++;
    cur->x0 = b[0].x; cur->y0 = b[0].y;
    Pix prev = b[0];
    for (int64_t i = 1; i < u; i++) {
        int brk = (dir == D_H) ? (prev.y != b[i].y || prev.x + 1 != b[i].x) : (prev.x != b[i].x || prev.y + 1 != b[i].y);
        if (brk) {
            cur = (Run*)rv->p + (rv->n - 1);
            cur->x1 = prev.x; cur->y1 = prev.y;
            cur = (Run*)vec_push(rv, sizeof(Run)); nr++;
            cur->x0 = b[i].x; cur->y0 = b[i].y;
        }
        prev = b[i];
    }
    cur = (Run*)rv->p + (rv->n - 1);
    cur->x1 = b[u - 1].x; cur->y1 = b[u - 1].y;
    return nr;
}

/* PointMap::sieve2 (pointdata.cpp:1512-1565) */
static int sieve2(const dmxo_map* m, Sieve* sv, Vec* addlist, int q, int depth, int cx, int cy) {
    int hasgaps = 0;
    int firstind = 0;
    for (int g = 0; g < sv->ng; g++) {
        double st = sv->gaps[g].start, en = sv->gaps[g].end;
        for (int ind = (int)ceil(st * (depth - 0.5) - 0.5); ind <= (int)floor(en * (depth + 0.5) + 0.5); ind++) {
            if (ind < firstind) continue;
            if (ind > depth) break;
            firstind = ind;
            int x = (q >= 4 ? ind : depth);
            int y = (q >= 4 ? depth : ind);
            int hx = (short)(cx + ((q % 2) ? x : -x));
            int hy = (short)(cy + ((q <= 1 || q >= 6) ? y : -y));
            if (incl(m, hx, hy)) {
                hasgaps = 1;
                int centregap = ((double)ind >= st * depth && (double)ind <= en * depth);
                int64_t hc = cidx(m, hx, hy);
                const Line* hl = m->cl + m->cl_off[hc];
                int64_t nl = m->cl_off[hc + 1] - m->cl_off[hc];
                if (centregap && (m->state[hc] & ST_FILLED)) {
                    if ((ind != 0 || q == 0 || q == 1 || q == 5 || q == 6) && (ind != depth || q < 4)) {
                        if (!sieve_testblock(sv, depixelate(m, hx, hy), hl, nl, m->spacing * 1e-10)) {
                            Pix* p = (Pix*)vec_push(addlist, sizeof(Pix));
                            p->x = hx; p->y = hy;
                        }
                    }
                }
                sieve_block(sv, hl, nl, q);
            }
        }
    }
    sieve_collectgarbage(sv);
    return hasgaps;
}

/* PointMap::sparkPixel2 (pointdata.cpp:1380-1510) + Node::make (ngraph.cpp:27-58) */
static void spark_pixel(dmxo_map* m, Work* w, int cx, int cy, double maxdist, NodeG* nd, float* attr) {
    float far[32];
    for (int i = 0; i < 32; i++) { far[i] = 0.0f; w->bins[i].n = 0; }
    int nsize = 0;
    double tdist = 0.0, tdist2 = 0.0;
    P2 c0 = depixelate(m, cx, cy);
    int64_t cc = cidx(m, cx, cy);
    for (int q = 0; q < 8; q++) {
        Sieve* sv = &w->sv;
        sv->centre = c0; sv->maxdist = maxdist;
        sv->ng = 1; sv->gaps[0].start = 0.0; sv->gaps[0].end = 1.0; sv->nb = 0;
        double border = m->spacing * 1e-10;
        Reg vp = regionate(m, cx, cy, 1e-10);
        switch (q) {
        case 0: vp.trx = c0.x; vp.bly = c0.y - border; break;
        case 6: vp.trx = c0.x + border; vp.bly = c0.y; break;
        case 1: vp.blx = c0.x; vp.bly = c0.y - border; break;
        case 7: vp.blx = c0.x - border; vp.bly = c0.y; break;
        case 2: vp.trx = c0.x; vp.try_ = c0.y + border; break;
        case 4: vp.trx = c0.x + border; vp.try_ = c0.y; break;
        case 3: vp.blx = c0.x; vp.try_ = c0.y + border; break;
        case 5: vp.blx = c0.x - border; vp.try_ = c0.y; break;
        }
        int64_t nl = m->cl_off[cc + 1] - m->cl_off[cc];
        if (nl > w->cap0) { w->cap0 = (int)nl; w->lines0 = (Line*)realloc(w->lines0, nl * sizeof(Line)); }
        int n0 = 0;
        for (int64_t i = 0; i < nl; i++) {
            Line l = m->cl[m->cl_off[cc] + i];
            if (line_crop(&l, &vp)) w->lines0[n0++] = l;
        }
        sieve_block(sv, w->lines0, n0, q);
        sieve_collectgarbage(sv);
        for (int depth = 1; sv->ng > 0; depth++) {
            w->add.n = 0;
            if (!sieve2(m, sv, &w->add, q, depth, cx, cy)) break;
            Pix* ad = (Pix*)w->add.p;
            for (int64_t n = 0; n < w->add.n; n++) {
                if (m->state[cidx(m, ad[n].x, ad[n].y)] & ST_FILLED) {
                    P2 pa = depixelate(m, ad[n].x, ad[n].y);
                    P2 g = {pa.x - c0.x, pa.y - c0.y};
                    int bin = whichbin(g);
                    double dx = (double)(ad[n].x - cx), dy = (double)(ad[n].y - cy);
                    double this_dist = sqrt(dx * dx + dy * dy) * m->spacing;
                    if (this_dist > far[bin]) far[bin] = (float)this_dist;
                    tdist += this_dist;
                    tdist2 += this_dist * this_dist;
                    nsize++;
                    *(Pix*)vec_push(&w->bins[bin], sizeof(Pix)) = ad[n];
                }
            }
        }
    }
    Vec rv = {0};
    nd->total_runs = 0;
    for (int i = 0; i < 32; i++) {
        char dir;
        if (i == 4 || i == 20) dir = D_PD;
        else if (i == 12 || i == 28) dir = D_ND;
        else if ((i > 4 && i < 12) || (i > 20 && i < 28)) dir = D_V;
        else dir = D_H;
        nd->dist[i] = far[i];
        nd->count[i] = 0;
        nd->dir[i] = w->bins[i].n ? dir : D_NODIR;
        nd->nruns[i] = bin_make(w, (Pix*)w->bins[i].p, w->bins[i].n, dir, &rv, &nd->count[i]);
    }
    nd->runs = (Run*)rv.p;
    nd->total_runs = rv.n;
    attr[0] = (float)nsize;
    attr[1] = (float)tdist;
    attr[2] = (float)tdist2;
}

static void free_work(Work* w) {
    free(w->sv.gaps); free(w->sv.blocks);
    for (int i = 0; i < 32; i++) free(w->bins[i].p);
    free(w->add.p); free(w->sortbuf.p); free(w->lines0);
}

static void index_nodes(dmxo_map* m) {
    int64_t C = (int64_t)m->cols * m->rows;
    free(m->node_of_cell); free(m->node_cell);
    m->node_of_cell = (int32_t*)malloc(C * sizeof(int32_t));
    int64_t n = 0;
    for (int64_t c = 0; c < C; c++) m->node_of_cell[c] = (m->state[c] & ST_FILLED) ? (int32_t)(n++) : -1;
    m->nnodes = n;
    m->node_cell = (int32_t*)malloc((n ? n : 1) * sizeof(int32_t));
    for (int64_t c = 0; c < C; c++) if (m->node_of_cell[c] >= 0) m->node_cell[m->node_of_cell[c]] = (int32_t)c;
}

/* does the node's bin contain pixel (x,y) -- Bin cursor iteration (ngraph.cpp:395-416) */
static int bin_contains(const NodeG* nd, const Run* br, int b, int x, int y) {
    char dir = nd->dir[b];
    for (int r = 0; r < nd->nruns[b]; r++) {
        int px = br[r].x0, py = br[r].y0;
        int endc = (dir & D_V) ? br[r].y1 : br[r].x1;
        for (;;) {
            int col = (dir & D_V) ? py : px;
            if (col > endc) break;
            if (px == x && py == y) return 1;
            switch (dir) {
            case D_PD: px++; py++; break;
            case D_ND: px++; py--; break;
            case D_H: px++; break;
            case D_V: py++; break;
            default: px++; break;
            }
        }
    }
    return 0;
}

/* addGridConnections (pointdata.cpp:1735-1768) for node k */
static uint8_t grid_connections(const dmxo_map* m, int64_t k) {
    static const int mv[8][2] = {{0, 1}, {-1, 0}, {-1, 0}, {0, -1}, {0, -1}, {1, 0}, {1, 0}, {0, 0}};
    int32_t c = m->node_cell[k];
    int cx = c / m->rows, cy = c % m->rows;
    int nx = cx + 1, ny = cy;
    const NodeG* nd = &m->nodes[k];
    uint8_t gc = 0;
    for (int i = 0; i < 32; i += 4) {
        const Run* br = nd->runs;
        for (int b = 0; b < i; b++) br += nd->nruns[b];
        if (bin_contains(nd, br, i, nx, ny)) gc |= (uint8_t)(1 << (i / 4));
        nx += mv[i / 4][0]; ny += mv[i / 4][1];
    }
    return gc;
}

int dmxo_makegraph(dmxo_map* m, double maxdist, int boundary, int64_t nb, int64_t ne, int nthreads) {
    if (!m->blocked_lines) block_lines(m);
    int64_t C = (int64_t)m->cols * m->rows;
    if (boundary) { /* pointdata.cpp:1254-1264 */
        for (int64_t c = 0; c < C; c++)
            if ((m->state[c] & ST_FILLED) && !(m->state[c] & ST_EDGE)) m->state[c] &= ~ST_FILLED;
    }
    index_nodes(m);
    int64_t N = m->nnodes;
    release_nodes(m);
    m->nodes = (NodeG*)calloc(N ? N : 1, sizeof(NodeG));
    free(m->attrs); m->attrs = (float*)calloc((N ? N : 1) * 3, sizeof(float));
    free(m->gridconn); m->gridconn = (uint8_t*)calloc(N ? N : 1, 1);
    if (ne < 0 || ne > N) ne = N;
    if (nb < 0) nb = 0;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
#endif
    {
        Work w;
        memset(&w, 0, sizeof(w));
        w.sv.capg = 64; w.sv.gaps = (Zone*)malloc(64 * sizeof(Zone));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
        for (int64_t k = nb; k < ne; k++) {
            int32_t c = m->node_cell[k];
            spark_pixel(m, &w, (int)(c / m->rows), (int)(c % m->rows), maxdist, &m->nodes[k], &m->attrs[3 * k]);
        }
        free_work(&w);
    }
    for (int64_t k = nb; k < ne; k++) m->gridconn[k] = grid_connections(m, k);
    return 0;
}

/* Whole-map digests (tests/golden/gen_mk_digests.py): sparkGraph2 + addGridConnections for the nodes
 * [nb, ne) only, keeping the graph arrays of the map between calls, so a caller can sweep the map in
 * chunks, read each chunk back (dmxo_get_graph_range) and free its runs (dmxo_release_range) without
 * ever holding the whole 36-90 GB graph. */
int dmxo_makegraph_range(dmxo_map* m, double maxdist, int64_t nb, int64_t ne, int nthreads) {
    if (!m->blocked_lines) block_lines(m);
    if (m->runs_borrowed) release_nodes(m);
    if (!m->nodes) {
        index_nodes(m);
        int64_t N = m->nnodes;
        m->nodes = (NodeG*)calloc(N ? N : 1, sizeof(NodeG));
        free(m->attrs); m->attrs = (float*)calloc((N ? N : 1) * 3, sizeof(float));
        free(m->gridconn); m->gridconn = (uint8_t*)calloc(N ? N : 1, 1);
    }
    if (nb < 0 || ne > m->nnodes || nb > ne) return -1;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
#endif
    {
        Work w;
        memset(&w, 0, sizeof(w));
        w.sv.capg = 64; w.sv.gaps = (Zone*)malloc(64 * sizeof(Zone));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
        for (int64_t k = nb; k < ne; k++) {
            free(m->nodes[k].runs);
            memset(&m->nodes[k], 0, sizeof(NodeG));
            int32_t c = m->node_cell[k];
            spark_pixel(m, &w, (int)(c / m->rows), (int)(c % m->rows), maxdist, &m->nodes[k], &m->attrs[3 * k]);
            m->gridconn[k] = grid_connections(m, k);
        }
        free_work(&w);
    }
    return 0;
}

int64_t dmxo_num_runs_range(const dmxo_map* m, int64_t nb, int64_t ne) {
    int64_t r = 0;
    for (int64_t k = nb; k < ne; k++) r += m->nodes[k].total_runs;
    return r;
}

/* dmxo_get_graph's layout for the nodes [nb, ne): attrs [n][3], bins [n][32][4], runs of those nodes. */
void dmxo_get_graph_range(const dmxo_map* m, int64_t nb, int64_t ne, float* attrs, int32_t* bins, int16_t* runs,
                          uint8_t* gridconn) {
    int64_t ro = 0;
    for (int64_t k = nb; k < ne; k++) {
        const NodeG* nd = &m->nodes[k];
        const int64_t i = k - nb;
        if (attrs) memcpy(attrs + 3 * i, m->attrs + 3 * k, 3 * sizeof(float));
        if (gridconn) gridconn[i] = m->gridconn[k];
        if (bins)
            for (int b = 0; b < 32; b++) {
                int32_t* o = bins + (i * 32 + b) * 4;
                o[0] = nd->dir[b]; o[1] = nd->count[b];
                memcpy(&o[2], &nd->dist[b], 4);
                o[3] = nd->nruns[b];
            }
        if (runs) memcpy(runs + 4 * ro, nd->runs, nd->total_runs * sizeof(Run));
        ro += nd->total_runs;
    }
}

void dmxo_release_range(dmxo_map* m, int64_t nb, int64_t ne) {
    if (m->runs_borrowed) return;
    for (int64_t k = nb; k < ne; k++) {
        free(m->nodes[k].runs);
        m->nodes[k].runs = NULL;
        m->nodes[k].total_runs = 0;
    }
}

/* bench.py cpu_baseline: makeGraph (sparkPixel2) of a sample of nodes, each on one thread, its wall
 * time in secs[i].  The graph arrays of the map are allocated on first use (no boundary graph). */
int dmxo_makegraph_sample(dmxo_map* m, double maxdist, const int64_t* nodes, int64_t n, int nthreads, double* secs) {
    if (!m->blocked_lines) block_lines(m);
    if (m->runs_borrowed) release_nodes(m);
    if (!m->nodes) {
        index_nodes(m);
        int64_t N = m->nnodes;
        m->nodes = (NodeG*)calloc(N ? N : 1, sizeof(NodeG));
        free(m->attrs); m->attrs = (float*)calloc((N ? N : 1) * 3, sizeof(float));
        free(m->gridconn); m->gridconn = (uint8_t*)calloc(N ? N : 1, 1);
    }
    for (int64_t i = 0; i < n; i++)
        if (nodes[i] < 0 || nodes[i] >= m->nnodes) return -1;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
#endif
    {
        Work w;
        memset(&w, 0, sizeof(w));
        w.sv.capg = 64; w.sv.gaps = (Zone*)malloc(64 * sizeof(Zone));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t i = 0; i < n; i++) {
            const int64_t k = nodes[i];
            const double t0 = omp_get_wtime();
            free(m->nodes[k].runs);
            memset(&m->nodes[k], 0, sizeof(NodeG));
            int32_t c = m->node_cell[k];
            spark_pixel(m, &w, (int)(c / m->rows), (int)(c % m->rows), maxdist, &m->nodes[k], &m->attrs[3 * k]);
            secs[i] = omp_get_wtime() - t0;
        }
        free_work(&w);
    }
    return 0;
}

int64_t dmxo_num_nodes(const dmxo_map* m) { return m->nnodes; }
int64_t dmxo_num_runs(const dmxo_map* m) {
    int64_t r = 0;
    for (int64_t k = 0; k < m->nnodes; k++) r += m->nodes[k].total_runs;
    return r;
}
void dmxo_get_graph(const dmxo_map* m, float* attrs, int32_t* bins, int16_t* runs, uint8_t* gridconn) {
    int64_t ro = 0;
    for (int64_t k = 0; k < m->nnodes; k++) {
        const NodeG* nd = &m->nodes[k];
        if (attrs) memcpy(attrs + 3 * k, m->attrs + 3 * k, 3 * sizeof(float));
        if (gridconn) gridconn[k] = m->gridconn[k];
        for (int b = 0; b < 32; b++) {
            if (bins) {
                int32_t* o = bins + (k * 32 + b) * 4;
                o[0] = nd->dir[b]; o[1] = nd->count[b];
                memcpy(&o[2], &nd->dist[b], 4);
                o[3] = nd->nruns[b];
            }
        }
        if (runs) memcpy(runs + 4 * ro, nd->runs, nd->total_runs * sizeof(Run));
        ro += nd->total_runs;
    }
}

int dmxo_set_graph(dmxo_map* m, const int32_t* bins, const int16_t* runs, int64_t nruns) {
    if (!m->node_of_cell) index_nodes(m);
    int64_t N = m->nnodes, ro = 0;
    if (m->runs_borrowed) release_nodes(m);
    if (!m->nodes) m->nodes = (NodeG*)calloc(N ? N : 1, sizeof(NodeG));
    for (int64_t k = 0; k < N; k++) {
        NodeG* nd = &m->nodes[k];
        free(nd->runs);
        int64_t t = 0;
        for (int b = 0; b < 32; b++) {
            const int32_t* o = bins + (k * 32 + b) * 4;
            nd->dir[b] = (char)o[0]; nd->count[b] = (uint16_t)o[1];
            memcpy(&nd->dist[b], &o[2], 4);
            nd->nruns[b] = o[3];
            t += o[3];
        }
        if (ro + t > nruns) return -1;
        nd->runs = (Run*)malloc((t ? t : 1) * sizeof(Run));
        memcpy(nd->runs, runs + 4 * ro, t * sizeof(Run));
        nd->total_runs = t;
        ro += t;
    }
    return 0;
}

/* As dmxo_set_graph, without copying the runs: nodes[].runs point into `runs`, which the caller keeps
 * alive and unchanged until the next set_graph / makegraph / free (bench.py's CPU leg on a 36 GB graph). */
int dmxo_set_graph_view(dmxo_map* m, const int32_t* bins, const int16_t* runs, int64_t nruns) {
    if (!m->node_of_cell) index_nodes(m);
    int64_t N = m->nnodes, ro = 0;
    release_nodes(m);
    m->nodes = (NodeG*)calloc(N ? N : 1, sizeof(NodeG));
    m->runs_borrowed = 1;
    for (int64_t k = 0; k < N; k++) {
        NodeG* nd = &m->nodes[k];
        int64_t t = 0;
        for (int b = 0; b < 32; b++) {
            const int32_t* o = bins + (k * 32 + b) * 4;
            nd->dir[b] = (char)o[0]; nd->count[b] = (uint16_t)o[1];
            memcpy(&nd->dist[b], &o[2], 4);
            nd->nruns[b] = o[3];
            t += o[3];
        }
        if (ro + t > nruns) { release_nodes(m); return -1; }
        nd->runs = (Run*)(runs + 4 * ro);
        nd->total_runs = t;
        ro += t;
    }
    return 0;
}

/* ---------------------------------------------------------------- VGA global */
static inline double plog2(double a) { return log(a) * M_1_LN2_; } /* pafmath.h:61 */
static inline double dvalue(double k) { /* pafmath.h:72 */
    return 2.0 * (k * (plog2((k + 2.0) / 3.0) - 1.0) + 1.0) / ((k - 1.0) * (k - 2.0));
}
static inline double pvalue(double k) { return 2.0 * (k - plog2(k) - 1.0) / ((k - 1.0) * (k - 2.0)); } /* :75 */
static inline double teklinteg(double nc, double td) { return log(0.5 * (nc - 2.0)) / log((double)(td - nc + 1)); }

/* VGAVisualGlobal::extractUnseen (vgavisualglobal.cpp:218-240), misc/extent row-major x + y*cols */
static void extract_unseen(const dmxo_map* m, const NodeG* nd, Vec* out, int32_t* miscs, int16_t* extx, int16_t* exty) {
    const Run* r = nd->runs;
    for (int b = 0; b < 32; b++) {
        char dir = nd->dir[b];
        for (int k = 0; k < nd->nruns[b]; k++, r++) {
            int px = r->x0, py = r->y0;
            int endc = (dir & D_V) ? r->y1 : r->x1;
            for (;;) {
                int col = (dir & D_V) ? py : px;
                if (col > endc) break;
                int64_t idx = (int64_t)px + (int64_t)py * m->cols;
                if (miscs[idx] == 0) {
                    Pix* p = (Pix*)vec_push(out, sizeof(Pix));
                    p->x = px; p->y = py;
                    miscs[idx] |= (1 << b);
                }
                if (!(dir & D_DIAG)) {
                    int16_t* ext = (dir & D_V) ? &exty[idx] : &extx[idx];
                    if (*ext >= endc) break;
                    *ext = (int16_t)endc;
                }
                switch (dir) {
                case D_PD: px++; py++; break;
                case D_ND: px++; py--; break;
                case D_H: px++; break;
                case D_V: py++; break;
                }
            }
        }
    }
}

int dmxo_vga_global(dmxo_map* m, double radius, int gates_only, int64_t nb, int64_t ne, int nthreads,
                    float* out, int64_t* lv) {
    int64_t N = m->nnodes, C = (int64_t)m->cols * m->rows;
    if (ne < 0 || ne > N) ne = N;
    if (nb < 0) nb = 0;
    int rad = (int)radius;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
#endif
    {
        int32_t* miscs = (int32_t*)malloc(C * sizeof(int32_t));
        int16_t* extx = (int16_t*)malloc(C * sizeof(int16_t));
        int16_t* exty = (int16_t*)malloc(C * sizeof(int16_t));
        Vec levels[4096];
        int nlev_alloc = 0;
        memset(levels, 0, sizeof(levels));
        int64_t* dist = (int64_t*)malloc(4096 * sizeof(int64_t));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t k = nb; k < ne; k++) {
            float* o = out + 7 * k;
            for (int i = 0; i < 7; i++) o[i] = -1.0f;
            int32_t c = m->node_cell[k];
            int cx = c / m->rows, cy = c % m->rows;
            int st = m->state[c];
            if (((st & ST_CONTEXTFILLED) && !(cx % 2 == 0 && cy % 2 == 0)) || gates_only) continue;
            for (int x = 0; x < m->cols; x++)
                for (int y = 0; y < m->rows; y++) {
                    int64_t idx = (int64_t)x + (int64_t)y * m->cols;
                    miscs[idx] = 0; extx[idx] = (int16_t)x; exty[idx] = (int16_t)y;
                }
            int64_t total_depth = 0, total_nodes = 0;
            int nd = 0;
            for (int i = 0; i < nlev_alloc; i++) levels[i].n = 0;
            if (nlev_alloc == 0) nlev_alloc = 1;
            Pix* p0 = (Pix*)vec_push(&levels[0], sizeof(Pix));
            p0->x = cx; p0->y = cy;
            int level = 0;
            while (levels[level].n) {
                if (level + 1 >= 4096) break;
                if (nlev_alloc < level + 2) nlev_alloc = level + 2;
                levels[level + 1].n = 0;
                dist[nd++] = 0;
                const int64_t nl = levels[level].n;
                for (int64_t i = nl - 1; i >= 0; i--) {
                    Pix cur = ((Pix*)levels[level].p)[g_pop_forward ? nl - 1 - i : i];
                    int64_t idx = (int64_t)cur.x + (int64_t)cur.y * m->cols;
                    int64_t cc = cidx(m, cur.x, cur.y);
                    if ((m->state[cc] & ST_FILLED) && miscs[idx] != ~0) {
                        total_depth += level;
                        total_nodes += 1;
                        dist[nd - 1] += 1;
                        int pst = m->state[cc];
                        if (rad == -1 || (level < rad && (!(pst & ST_CONTEXTFILLED) || (cur.x % 2 == 0 && cur.y % 2 == 0)))) {
                            extract_unseen(m, &m->nodes[m->node_of_cell[cc]], &levels[level + 1], miscs, extx, exty);
                            miscs[idx] = ~0;
                            /* the merge pixel's node is extracted at the same level, uncounted
                               (vgavisualglobal.cpp:113-122) */
                            const int32_t mc = m->merge[cc];
                            if (mc >= 0) {
                                const int64_t midx = (int64_t)(mc / m->rows) + (int64_t)(mc % m->rows) * m->cols;
                                if (miscs[midx] != ~0) {
                                    if (m->node_of_cell[mc] >= 0)
                                        extract_unseen(m, &m->nodes[m->node_of_cell[mc]], &levels[level + 1], miscs, extx, exty);
                                    miscs[midx] = ~0;
                                }
                            }
                        } else {
                            miscs[idx] = ~0;
                        }
                    }
                }
                levels[level].n = 0;
                level++;
            }
            if (lv) { lv[3 * k] = total_nodes; lv[3 * k + 1] = total_depth; lv[3 * k + 2] = nd; }
            o[5] = (float)total_nodes;
            if (total_nodes > 1) {
                double mean_depth = (double)total_depth / (double)(total_nodes - 1);
                o[4] = (float)mean_depth;
                if (total_nodes > 2 && mean_depth > 1.0) {
                    double ra = 2.0 * (mean_depth - 1.0) / (double)(total_nodes - 2);
                    double rra_d = ra / dvalue((double)total_nodes);
                    double rra_p = ra / pvalue((double)total_nodes);
                    double integ_tk = teklinteg((double)total_nodes, (double)total_depth);
                    o[1] = (float)(1.0 / rra_d);
                    o[2] = (float)(1.0 / rra_p);
                    o[3] = (total_depth - total_nodes + 1 > 1) ? (float)integ_tk : -1.0f;
                } else {
                    o[1] = -1.0f; o[2] = -1.0f; o[3] = -1.0f;
                }
                double entropy = 0.0, rel_entropy = 0.0, factorial = 1.0;
                for (int kk = 1; kk < nd; kk++) {
                    if (dist[kk] > 0) {
                        double prob = (double)dist[kk] / (double)(total_nodes - 1);
                        entropy -= prob * plog2(prob);
                        factorial *= (double)(kk + 1);
                        double qq = (pow(mean_depth, (double)kk) / factorial) * exp(-mean_depth);
                        rel_entropy += (float)prob * plog2(prob / qq);
                    }
                }
                o[0] = (float)entropy;
                o[6] = (float)rel_entropy;
            } else {
                o[4] = -1.0f; o[0] = -1.0f; o[6] = -1.0f;
            }
        }
        for (int i = 0; i < 4096; i++) free(levels[i].p);
        free(miscs); free(extx); free(exty); free(dist);
    }
    return 0;
}

/* ---------------------------------------------------------------- VGA metric step depth */
/* MetricTriple (salalib/pointdata.h:377-399): std::set ordered by (dist, pixel); two triples with
 * equal dist and pixel are the same key, so a second insert keeps the first lastpixel. */
typedef struct { float dist; int32_t pix; int32_t last; } MTrip;
static int mt_less(const MTrip* a, const MTrip* b) {
    return a->dist < b->dist || (a->dist == b->dist && a->pix < b->pix);
}
typedef struct { MTrip* a; int64_t n, cap; } MHeap;
static void mh_push(MHeap* h, MTrip t) {
    if (h->n == h->cap) { h->cap = h->cap ? 2 * h->cap : 1024; h->a = (MTrip*)realloc(h->a, h->cap * sizeof(MTrip)); }
    int64_t i = h->n++;
    while (i > 0) {
        int64_t p = (i - 1) / 2;
        if (!mt_less(&t, &h->a[p])) break;
        h->a[i] = h->a[p];
        i = p;
    }
    h->a[i] = t;
}
static MTrip mh_pop(MHeap* h) {
    MTrip top = h->a[0], last = h->a[--h->n];
    int64_t i = 0;
    for (;;) {
        int64_t c = 2 * i + 1;
        if (c >= h->n) break;
        if (c + 1 < h->n && mt_less(&h->a[c + 1], &h->a[c])) c++;
        if (!mt_less(&h->a[c], &last)) break;
        h->a[i] = h->a[c];
        i = c;
    }
    if (h->n) h->a[i] = last;
    return top;
}
static inline int32_t pix_int(int x, int y) { return (int32_t)(((uint32_t)x << 16) + ((uint32_t)y & 0xffff)); } /* pixelref.h:81 */
static inline double pix_dist(int ax, int ay, int bx, int by) { /* pixelref.h:116-119 */
    int dx = ax - bx, dy = ay - by;
    return sqrt((double)(dx * dx + dy * dy));
}
static inline double pix_angle(int ax, int ay, int bx, int by, int cx, int cy) { /* pixelref.h:121-131 */
    return acos((double)((ax - bx) * (bx - cx) + (ay - by) * (by - cy)) /
                (sqrt((double)((ax - bx) * (ax - bx) + (ay - by) * (ay - by))) *
                     sqrt((double)((bx - cx) * (bx - cx) + (by - cy) * (by - cy))) + 1e-12));
}
/* PointMap::blockedAdjacent (pointdata.cpp:1016-1068) */
static int blocked_adjacent(const dmxo_map* m, int x, int y) {
    static const int dx[8] = {1, 1, 0, -1, -1, -1, 0, 1}, dy[8] = {0, 1, 1, 1, 0, -1, -1, -1};
    for (int i = 0; i < 8; i++) {
        int nx = x + dx[i], ny = y + dy[i];
        if (incl(m, nx, ny) && (m->state[cidx(m, nx, ny)] & ST_BLOCKED)) return 1;
    }
    return 0;
}

/* The std::set<MetricTriple> search shared by VGAMetricDepth::run (vgametricdepth.cpp:45-84) and
 * VGAMetric::run (vgametric.cpp:82-112): every selected cell enters at dist 0; popped triples of
 * FILLED, not yet visited cells expand through Node::extractMetric when they are the search roots,
 * BLOCKED or blocked-adjacent; `visit` sees every resolved cell in pop order.  radius >= 0 stops the
 * search at the first popped triple with dist * spacing > radius (vgametric.cpp:86-88). */
typedef void (*metric_visit_fn)(void* ctx, const dmxo_map* m, int64_t cell, float dist, float cum, int merged);
/* Node::extractMetric / Bin::extractMetric (ngraph.cpp:67-76, :330-345) of the node at cell hc for
 * the triple (dist, hc, last): relaxes only when dist == 0 or hc is BLOCKED / blocked-adjacent. */
static void metric_relax(dmxo_map* m, int64_t hc, float dist, int32_t last, float* mdist, float* cum, int32_t* misc,
                         Vec* ins, MHeap* h) {
    const int hx = (int)(hc / m->rows), hy = (int)(hc % m->rows);
    if (!(dist == 0.0f || (m->state[hc] & ST_BLOCKED) || blocked_adjacent(m, hx, hy))) return;
    if (m->node_of_cell[hc] < 0) return;
    const NodeG* nd = &m->nodes[m->node_of_cell[hc]];
    const Run* r = nd->runs;
    const int lx = last >> 16, ly = last & 0xffff;
    const int32_t hpix = pix_int(hx, hy);
    for (int b = 0; b < 32; b++) {
        char dir = nd->dir[b];
        for (int k = 0; k < nd->nruns[b]; k++, r++) {
            int px = r->x0, py = r->y0;
            int endc = (dir & D_V) ? r->y1 : r->x1;
            for (;;) {
                int col = (dir & D_V) ? py : px;
                if (col > endc) break;
                int64_t pc = cidx(m, px, py);
                /* non-filled cells (diagonal gaps) can be queued but never resolve */
                if ((m->state[pc] & ST_FILLED) && misc[pc] == 0) {
                    double dd = pix_dist(px, py, hx, hy);
                    if (mdist[pc] == -1.0 || (double)dist + dd < (double)mdist[pc]) {
                        mdist[pc] = dist + (float)dd;
                        cum[pc] = cum[hc] + (last == -1 ? 0.0f : (float)(pix_angle(px, py, hx, hy, lx, ly) / (M_PI_ * 0.5)));
                        int dup = 0;
                        for (int64_t q = 0; q < ins[pc].n; q++)
                            if (((float*)ins[pc].p)[q] == mdist[pc]) { dup = 1; break; }
                        if (!dup) {
                            float* d = (float*)vec_push(&ins[pc], sizeof(float));
                            *d = mdist[pc];
                            MTrip t = {mdist[pc], pix_int(px, py), hpix};
                            mh_push(h, t);
                        }
                    }
                }
                switch (dir) {
                case D_PD: px++; py++; break;
                case D_ND: px++; py--; break;
                case D_H: px++; break;
                case D_V: py++; break;
                }
            }
        }
    }
}

/* The std::set<MetricTriple> search shared by VGAMetricDepth::run (vgametricdepth.cpp:45-84) and
 * VGAMetric::run (vgametric.cpp:82-112): every selected cell enters at dist 0; a popped triple of a
 * FILLED, not yet visited cell relaxes through Node::extractMetric, is marked visited and visited
 * (`visit`, merged = 0, in pop order); then a merge pixel not yet visited takes the popped cell's
 * cumulative angle, is visited (merged = 1: VGAMetricDepth writes its row, VGAMetric does not count
 * it), relaxes from (here.dist, merge pixel, NoPixel) and is marked visited (vgametricdepth.cpp:68-83,
 * vgametric.cpp:97-105).  radius >= 0 stops the search at the first popped triple with
 * dist * spacing > radius (vgametric.cpp:86-88). */
static void metric_search(dmxo_map* m, const int32_t* sel_cells, int64_t nsel, double radius, metric_visit_fn visit,
                          void* vctx, float* mdist, float* cum, int32_t* misc, Vec* ins) {
    const int64_t C = (int64_t)m->cols * m->rows;
    for (int64_t c = 0; c < C; c++) { mdist[c] = -1.0f; cum[c] = 0.0f; misc[c] = 0; ins[c].n = 0; }
    MHeap h = {0, 0, 0};
    for (int64_t i = 0; i < nsel; i++) {
        int32_t c = sel_cells[i];
        int x = c / m->rows, y = c % m->rows;
        MTrip t = {0.0f, pix_int(x, y), -1};
        float* d = (float*)vec_push(&ins[c], sizeof(float));
        *d = 0.0f;
        mh_push(&h, t);
    }
    while (h.n) {
        MTrip here = mh_pop(&h);
        if (radius >= 0.0 && ((double)here.dist * m->spacing) > radius) break;
        int hx = here.pix >> 16, hy = here.pix & 0xffff;
        int64_t hc = cidx(m, hx, hy);
        if (!(m->state[hc] & ST_FILLED) || misc[hc] == ~0) continue;
        metric_relax(m, hc, here.dist, here.last, mdist, cum, misc, ins, &h);
        misc[hc] = ~0;
        visit(vctx, m, hc, here.dist, cum[hc], 0);
        const int32_t mc = m->merge[hc];
        if (mc >= 0 && misc[mc] != ~0) {
            cum[mc] = cum[hc];
            visit(vctx, m, mc, here.dist, cum[mc], 1);
            metric_relax(m, mc, here.dist, -1, mdist, cum, misc, ins, &h);
            misc[mc] = ~0;
        }
    }
    free(h.a);
}

typedef struct { float* out; int64_t nsel; int sx0, sy0; } StepVisit;
static void stepdepth_visit(void* vctx, const dmxo_map* m, int64_t hc, float dist, float cumv, int merged) {
    (void)merged;   /* the merge pixel's row is written like the popped cell's (vgametricdepth.cpp:71-80) */
    StepVisit* v = (StepVisit*)vctx;
    float* o = v->out + 3 * m->node_of_cell[hc];
    o[0] = cumv;
    o[1] = (float)(m->spacing * dist);
    if (v->nsel == 1) o[2] = (float)(m->spacing * pix_dist((int)(hc / m->rows), (int)(hc % m->rows), v->sx0, v->sy0));
}

int dmxo_metric_stepdepth(dmxo_map* m, const int32_t* sel_cells, int64_t nsel, float* out) {
    const int64_t N = m->nnodes, C = (int64_t)m->cols * m->rows;
    for (int64_t i = 0; i < 3 * N; i++) out[i] = -1.0f;
    if (nsel <= 0) return -1;
    float* mdist = (float*)malloc(C * sizeof(float));
    float* cum = (float*)malloc(C * sizeof(float));
    int32_t* misc = (int32_t*)malloc(C * sizeof(int32_t));
    Vec* ins = (Vec*)calloc(C, sizeof(Vec)); /* dists inserted per cell (std::set key dedupe) */
    /* std::set<int> getSelSet() order; every selected cell enters at dist 0 (vgametricdepth.cpp:45-47) */
    StepVisit v = {out, nsel, sel_cells[0] / m->rows, sel_cells[0] % m->rows};
    metric_search(m, sel_cells, nsel, -1.0, stepdepth_visit, &v, mdist, cum, misc, ins);
    for (int64_t c = 0; c < C; c++) free(ins[c].p);
    free(ins); free(mdist); free(cum); free(misc);
    return 0;
}

/* VGAMetric::run (vgametric.cpp:26-136): per FILLED source, the metric search from it alone, with
 * float totals accumulated in pop order: total_depth += float(dist * spacing), total_angle +=
 * cumangle, euclid_depth += float(spacing * dist(pixel, source)), total_nodes++.  out [N][4]:
 * Metric Mean Shortest-Path Angle, Mean Shortest-Path Distance, Mean Straight-Line Distance,
 * Node Count (-1 for every source when gates_only). */
typedef struct { float ftd, fta, fte; int64_t tn; int sx, sy; } MetricVisit;
static void metric_visit(void* vctx, const dmxo_map* m, int64_t hc, float dist, float cumv, int merged) {
    if (merged) return;   /* merge pixels are not counted (vgametric.cpp:97-110) */
    MetricVisit* v = (MetricVisit*)vctx;
    v->ftd += (float)(dist * m->spacing);
    v->fta += cumv;
    v->fte += (float)(m->spacing * pix_dist((int)(hc / m->rows), (int)(hc % m->rows), v->sx, v->sy));
    v->tn += 1;
}

int dmxo_vga_metric(dmxo_map* m, double radius, int gates_only, int64_t nb, int64_t ne, int nthreads, float* out) {
    const int64_t N = m->nnodes, C = (int64_t)m->cols * m->rows;
    if (ne < 0 || ne > N) ne = N;
    if (nb < 0) nb = 0;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
#endif
    {
        float* mdist = (float*)malloc(C * sizeof(float));
        float* cum = (float*)malloc(C * sizeof(float));
        int32_t* misc = (int32_t*)malloc(C * sizeof(int32_t));
        Vec* ins = (Vec*)calloc(C, sizeof(Vec));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t k = nb; k < ne; k++) {
            float* o = out + 4 * k;
            for (int i = 0; i < 4; i++) o[i] = -1.0f;
            if (gates_only) continue;
            const int32_t c = m->node_cell[k];
            MetricVisit v;
            memset(&v, 0, sizeof(v));
            v.sx = c / m->rows; v.sy = c % m->rows;
            metric_search(m, &c, 1, radius, metric_visit, &v, mdist, cum, misc, ins);
            o[0] = (float)((double)v.fta / (double)v.tn);
            o[1] = (float)((double)v.ftd / (double)v.tn);
            o[2] = (float)((double)v.fte / (double)v.tn);
            o[3] = (float)v.tn;
        }
        for (int64_t c = 0; c < C; c++) free(ins[c].p);
        free(ins); free(mdist); free(cum); free(misc);
    }
    return 0;
}

/* Node::extractAngular / Bin::extractAngular (ngraph.cpp:78-85, :348-366) of the node at cell hc for
 * the triple (angle, hc, last): relaxes when angle == 0 or hc is BLOCKED / blocked-adjacent. */
static void angular_relax(dmxo_map* m, int64_t hc, float angle, int32_t last, float* cum, int32_t* misc, Vec* ins,
                          MHeap* h) {
    const int hx = (int)(hc / m->rows), hy = (int)(hc % m->rows);
    if (!(angle == 0.0f || (m->state[hc] & ST_BLOCKED) || blocked_adjacent(m, hx, hy))) return;
    if (m->node_of_cell[hc] < 0) return;
    const NodeG* nd = &m->nodes[m->node_of_cell[hc]];
    const Run* r = nd->runs;
    const int lx = last >> 16, ly = last & 0xffff;
    const int32_t hpix = pix_int(hx, hy);
    for (int b = 0; b < 32; b++) {
        char dir = nd->dir[b];
        for (int k = 0; k < nd->nruns[b]; k++, r++) {
            int px = r->x0, py = r->y0;
            int endc = (dir & D_V) ? r->y1 : r->x1;
            for (;;) {
                int col = (dir & D_V) ? py : px;
                if (col > endc) break;
                int64_t pc = cidx(m, px, py);
                if (misc[pc] == 0) {
                    float ang = last == -1 ? 0.0f : (float)(pix_angle(px, py, hx, hy, lx, ly) / (M_PI_ * 0.5));
                    if (cum[pc] == -1.0 || angle + ang < cum[pc]) {
                        cum[pc] = cum[hc] + ang;
                        int dup = 0;
                        for (int64_t q = 0; q < ins[pc].n; q++)
                            if (((float*)ins[pc].p)[q] == cum[pc]) { dup = 1; break; }
                        if (!dup) {
                            float* d = (float*)vec_push(&ins[pc], sizeof(float));
                            *d = cum[pc];
                            MTrip t = {cum[pc], pix_int(px, py), hpix};
                            mh_push(h, t);
                        }
                    }
                }
                switch (dir) {
                case D_PD: px++; py++; break;
                case D_ND: px++; py--; break;
                case D_H: px++; break;
                case D_V: py++; break;
                }
            }
        }
    }
}

/* The std::set<AngularTriple> search shared by VGAAngularDepth::run (vgaangulardepth.cpp:23-75) and
 * VGAAngular::run (vgaangular.cpp:26-133): selected cells enter with cumangle 0; a popped FILLED,
 * unvisited cell expands through Node::extractAngular (ngraph.cpp:78-85) when its angle is 0 or it is
 * BLOCKED / blocked-adjacent; Bin::extractAngular (ngraph.cpp:348-366) relaxes every unvisited cell
 * of its runs (no FILLED test) with ang = angle(pix, here, last)/(pi/2) when cumangle == -1 or
 * here.angle + ang < cumangle.  cum[] starts at -1 for every cell (VGAAngular resets all points;
 * VGAAngularDepth only the filled ones, but unfilled cells are never counted nor expanded).
 * A merge pixel not yet visited takes the popped cell's cumangle, is visited (merged = 1), relaxes
 * from (here.angle, merge pixel, NoPixel) and is marked visited (vgaangular.cpp:95-104,
 * vgaangulardepth.cpp:57-67).  radius >= 0 stops at the first popped triple with angle > radius
 * (vgaangular.cpp:86-88). */
static void angular_search(dmxo_map* m, const int32_t* sel_cells, int64_t nsel, double radius, metric_visit_fn visit,
                           void* vctx, float* cum, int32_t* misc, Vec* ins) {
    const int64_t C = (int64_t)m->cols * m->rows;
    for (int64_t c = 0; c < C; c++) { cum[c] = -1.0f; misc[c] = 0; ins[c].n = 0; }
    MHeap h = {0, 0, 0};
    for (int64_t i = 0; i < nsel; i++) {
        int32_t c = sel_cells[i];
        int x = c / m->rows, y = c % m->rows;
        MTrip t = {0.0f, pix_int(x, y), -1};
        int dup = 0;
        for (int64_t q = 0; q < ins[c].n; q++)
            if (((float*)ins[c].p)[q] == 0.0f) dup = 1;
        if (!dup) {
            float* d = (float*)vec_push(&ins[c], sizeof(float));
            *d = 0.0f;
            mh_push(&h, t);
        }
        cum[c] = 0.0f;
    }
    while (h.n) {
        MTrip here = mh_pop(&h);
        if (radius >= 0.0 && (double)here.dist > radius) break;
        int hx = here.pix >> 16, hy = here.pix & 0xffff;
        int64_t hc = cidx(m, hx, hy);
        if (!(m->state[hc] & ST_FILLED) || misc[hc] == ~0) continue;
        angular_relax(m, hc, here.dist, here.last, cum, misc, ins, &h);
        misc[hc] = ~0;
        visit(vctx, m, hc, here.dist, cum[hc], 0);
        const int32_t mc = m->merge[hc];
        if (mc >= 0 && misc[mc] != ~0) {
            cum[mc] = cum[hc];
            visit(vctx, m, mc, here.dist, cum[mc], 1);
            angular_relax(m, mc, here.dist, -1, cum, misc, ins, &h);
            misc[mc] = ~0;
        }
    }
    free(h.a);
}

static void angular_step_visit(void* vctx, const dmxo_map* m, int64_t hc, float dist, float cumv, int merged) {
    (void)dist; (void)merged;   /* the merge pixel's row is written too (vgaangulardepth.cpp:60-62) */
    ((float*)vctx)[m->node_of_cell[hc]] = cumv;
}

int dmxo_angular_stepdepth(dmxo_map* m, const int32_t* sel_cells, int64_t nsel, float* out) {
    const int64_t N = m->nnodes, C = (int64_t)m->cols * m->rows;
    for (int64_t i = 0; i < N; i++) out[i] = -1.0f;
    if (nsel <= 0) return -1;
    float* cum = (float*)malloc(C * sizeof(float));
    int32_t* misc = (int32_t*)malloc(C * sizeof(int32_t));
    Vec* ins = (Vec*)calloc(C, sizeof(Vec));
    angular_search(m, sel_cells, nsel, -1.0, angular_step_visit, out, cum, misc, ins);
    for (int64_t c = 0; c < C; c++) free(ins[c].p);
    free(ins); free(cum); free(misc);
    return 0;
}

typedef struct { float total; int64_t n; } AngularVisit;
static void angular_visit(void* vctx, const dmxo_map* m, int64_t hc, float dist, float cumv, int merged) {
    (void)m; (void)hc; (void)dist;
    if (merged) return;   /* merge pixels are not counted (vgaangular.cpp:95-106) */
    AngularVisit* v = (AngularVisit*)vctx;
    v->total += cumv;
    v->n += 1;
}

/* VGAAngular::run (vgaangular.cpp:26-133): out [N][3] Angular Mean Depth, Angular Total Depth,
 * Angular Node Count (-1 rows with gates_only). */
int dmxo_vga_angular(dmxo_map* m, double radius, int gates_only, int64_t nb, int64_t ne, int nthreads, float* out) {
    const int64_t N = m->nnodes, C = (int64_t)m->cols * m->rows;
    if (ne < 0 || ne > N) ne = N;
    if (nb < 0) nb = 0;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
#endif
    {
        float* cum = (float*)malloc(C * sizeof(float));
        int32_t* misc = (int32_t*)malloc(C * sizeof(int32_t));
        Vec* ins = (Vec*)calloc(C, sizeof(Vec));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t k = nb; k < ne; k++) {
            float* o = out + 3 * k;
            for (int i = 0; i < 3; i++) o[i] = -1.0f;
            if (gates_only) continue;
            const int32_t c = m->node_cell[k];
            AngularVisit v = {0.0f, 0};
            angular_search(m, &c, 1, radius, angular_visit, &v, cum, misc, ins);
            if (v.n > 0) o[0] = (float)((double)v.total / (double)v.n);
            o[1] = v.total;
            o[2] = (float)v.n;
        }
        for (int64_t c = 0; c < C; c++) free(ins[c].p);
        free(ins); free(cum); free(misc);
    }
    return 0;
}

/* VGAVisualGlobalDepth::run (salalib/vgamodules/vgavisualglobaldepth.cpp:23-77) with
 * Node::extractUnseen -> Bin::extractUnseen (ngraph.cpp:60-65, :308-326): one search tree from the
 * whole selection (std::set<int> PixelRef order), each level walked in reverse; Point::m_misc and
 * m_extent are reset for the attribute rows (filled cells) only (:31-35) -- every other point keeps
 * its freshly loaded state (misc 0, extent PixelRef() = (-1, -1), point.h:67). */
int dmxo_visual_stepdepth(dmxo_map* m, const int32_t* sel_cells, int64_t nsel, float* out) {
    const int64_t N = m->nnodes, C = (int64_t)m->cols * m->rows;
    for (int64_t i = 0; i < N; i++) out[i] = -1.0f;
    if (nsel <= 0) return -1;
    int32_t* miscs = (int32_t*)calloc(C, sizeof(int32_t));
    int16_t* extx = (int16_t*)malloc(C * sizeof(int16_t));
    int16_t* exty = (int16_t*)malloc(C * sizeof(int16_t));
    for (int x = 0; x < m->cols; x++)
        for (int y = 0; y < m->rows; y++) {
            const int64_t idx = (int64_t)x + (int64_t)y * m->cols;
            const int filled = (m->state[cidx(m, x, y)] & ST_FILLED) != 0;
            extx[idx] = (int16_t)(filled ? x : -1);
            exty[idx] = (int16_t)(filled ? y : -1);
        }
    Vec cur = {0, 0, 0}, next = {0, 0, 0};
    for (int64_t i = 0; i < nsel; i++) {
        Pix* p = (Pix*)vec_push(&cur, sizeof(Pix));
        p->x = sel_cells[i] / m->rows;
        p->y = sel_cells[i] % m->rows;
    }
    int level = 0;
    while (cur.n) {
        next.n = 0;
        for (int64_t i = cur.n - 1; i >= 0; i--) {
            const Pix pc = ((Pix*)cur.p)[g_pop_forward ? cur.n - 1 - i : i];
            const int64_t cc = cidx(m, pc.x, pc.y), idx = (int64_t)pc.x + (int64_t)pc.y * m->cols;
            if ((m->state[cc] & ST_FILLED) && miscs[idx] != ~0) {
                out[m->node_of_cell[cc]] = (float)level;
                if (!(m->state[cc] & ST_CONTEXTFILLED) || (pc.x % 2 == 0 && pc.y % 2 == 0) || level == 0) {
                    extract_unseen(m, &m->nodes[m->node_of_cell[cc]], &next, miscs, extx, exty);
                    miscs[idx] = ~0;
                    /* the merge pixel takes this level and is extracted now (vgavisualglobaldepth.cpp:55-63) */
                    const int32_t mc = m->merge[cc];
                    if (mc >= 0) {
                        const int64_t midx = (int64_t)(mc / m->rows) + (int64_t)(mc % m->rows) * m->cols;
                        if (miscs[midx] != ~0) {
                            if (m->node_of_cell[mc] >= 0) {
                                out[m->node_of_cell[mc]] = (float)level;
                                extract_unseen(m, &m->nodes[m->node_of_cell[mc]], &next, miscs, extx, exty);
                            }
                            miscs[midx] = ~0;
                        }
                    }
                }
                miscs[idx] = ~0;
            }
        }
        Vec t = cur; cur = next; next = t;
        level++;
    }
    free(cur.p); free(next.p); free(miscs); free(extx); free(exty);
    return 0;
}

/* ---------------------------------------------------------------- VGA visual local */
/* Visit the cells of node nd in Node::first/next order (ngraph.cpp:158-190, Bin::first/next
 * ngraph.cpp:392-416): bins 0..31, runs in order, each run from its start along the bin direction
 * until col(dir) passes the run end (col = y for vertical bins, x otherwise). */
#define WALK_NODE_CELLS(m, nd, CELL_BODY)                                                          \
    do {                                                                                           \
        const Run* r_ = (nd)->runs;                                                                \
        for (int b_ = 0; b_ < 32; b_++) {                                                          \
            const char dir_ = (nd)->dir[b_];                                                       \
            for (int k_ = 0; k_ < (nd)->nruns[b_]; k_++, r_++) {                                   \
                int px = r_->x0, py = r_->y0;                                                      \
                const int endc_ = (dir_ & D_V) ? r_->y1 : r_->x1;                                  \
                while (((dir_ & D_V) ? py : px) <= endc_) {                                        \
                    const int64_t cell = cidx((m), px, py);                                        \
                    CELL_BODY;                                                                     \
                    switch (dir_) {                                                                \
                    case D_PD: px++; py++; break;                                                  \
                    case D_ND: px++; py--; break;                                                  \
                    case D_V: py++; break;                                                         \
                    default: px++; break;                                                          \
                    }                                                                              \
                }                                                                                  \
            }                                                                                      \
        }                                                                                          \
    } while (0)

static int cmp_i64(const void* a, const void* b) {
    const int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return x < y ? -1 : x > y;
}

/* VGAVisualLocal::run (vgavisuallocal.cpp:23-117).  Per source: neighbourhood = Node::contents
 * (ngraph.cpp:184-191: cells of every run, addIfNotExists), sorted by PixelRef (x-major cell order,
 * pixelref.h:95-98).  For each neighbour that is FILLED with a node: retro_size = cells iterated in
 * its node, intersect_size = those in the neighbourhood, totalneighbourhood gains the ones not yet
 * in it; control += 1.0f/float(retro_size) (float, sorted order), cluster += intersect_size (int).
 * The std::find membership tests are restated with per-cell marks (same sets, same counts). */
int dmxo_vga_local(dmxo_map* m, int gates_only, int64_t nb, int64_t ne, int nthreads, float* out) {
    const int64_t N = m->nnodes, C = (int64_t)m->cols * m->rows;
    if (ne < 0 || ne > N) ne = N;
    if (nb < 0) nb = 0;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
#endif
    {
        uint8_t* inhood = (uint8_t*)calloc(C, 1);
        uint8_t* intotal = (uint8_t*)calloc(C, 1);
        int64_t* hood = (int64_t*)malloc((C + 1) * sizeof(int64_t));
        int64_t* total = (int64_t*)malloc((C + 1) * sizeof(int64_t));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t k = nb; k < ne; k++) {
            float* o = out + 3 * k;
            for (int i = 0; i < 3; i++) o[i] = -1.0f;
            const int32_t c = m->node_cell[k];
            const int cx = c / m->rows, cy = c % m->rows;
            if (((m->state[c] & ST_CONTEXTFILLED) && !(cx % 2 == 0 && cy % 2 == 0)) || gates_only) continue;
            int64_t nh = 0, ntot = 0;
            WALK_NODE_CELLS(m, &m->nodes[k], {
                if (!inhood[cell]) { inhood[cell] = 1; hood[nh++] = cell; }
            });
            qsort(hood, (size_t)nh, sizeof(int64_t), cmp_i64);
            int32_t cluster = 0;   /* int in the reference; wraps like it past 2^31 */
            float control = 0.0f;
            for (int64_t i = 0; i < nh; i++) {
                const int64_t nc = hood[i];
                if (!(m->state[nc] & ST_FILLED) || m->node_of_cell[nc] < 0) continue;
                int32_t retro = 0, inter = 0;
                WALK_NODE_CELLS(m, &m->nodes[m->node_of_cell[nc]], {
                    retro++;
                    if (inhood[cell]) inter++;
                    if (!intotal[cell]) { intotal[cell] = 1; total[ntot++] = cell; }
                });
                control += 1.0f / (float)retro;
                cluster = (int32_t)((uint32_t)cluster + (uint32_t)inter);
            }
            if (nh > 1) {
                o[0] = (float)(cluster / ((double)nh * ((double)nh - 1.0)));
                o[1] = control;
                o[2] = (float)((double)nh / (double)ntot);
            }
            for (int64_t i = 0; i < nh; i++) inhood[hood[i]] = 0;
            for (int64_t i = 0; i < ntot; i++) intotal[total[i]] = 0;
        }
        free(inhood); free(intotal); free(hood); free(total);
    }
    return 0;
}

/* bench.py cpu_baseline: VGA global BFS of a sample of source nodes, each on one thread (the graph must
 * be set: dmxo_set_graph), its wall time in secs[i]; out [N][7] rows of the sample. */
int dmxo_vga_global_sample(dmxo_map* m, double radius, const int64_t* nodes, int64_t n, int nthreads, float* out,
                           double* secs) {
    for (int64_t i = 0; i < n; i++)
        if (nodes[i] < 0 || nodes[i] >= m->nnodes) return -1;
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads)
#endif
    for (int64_t i = 0; i < n; i++) {
        const double t0 = omp_get_wtime();
        dmxo_vga_global(m, radius, 0, nodes[i], nodes[i] + 1, 1, out, NULL);
        secs[i] = omp_get_wtime() - t0;
    }
    return 0;
}
