// policy.hpp -- the engine's tuning and memory decisions in one place (DESIGN.md §9 "Policy").
//
// Every constant here was chosen by an A/B measurement on MI355X at BASELINE.json configs[2] (1000^2) and,
// where it matters, configs[4] (2000^2/5000); the record each one rests on is named next to it.  None of them
// changes a result: every path they choose between is exact (the parity tests run every one of them).
//
// Run-time overrides are test hooks (DMX_* environment variables, read through hook() / hook_int()).  The
// suite runs with the defaults; the hooks exist for the A/B records and to force fallbacks in tests.
#pragma once
#include <cstdint>
#include <cstdlib>

namespace dmx {
namespace policy {

// ---- makeGraph (makegraph.hip)
// sources of the pool-sizing sample pass (run when the worst-case pool would not fit)
constexpr int64_t kMkSample = 4096;
// makeGraph cost model of one source for the balanced shard ranges (dmx_makegraph_balance): chunks of 64
// candidates weigh 0.7 of a depth step (profiles/r4_balance_config*.log)
constexpr double kMkSourceCost = 0.0, kMkChunkCost = 0.7;
// (the shortest occluder-free span, MK_SPAN_MIN = 4 depths, is a kernel constant: makegraph.hip)

// ---- VGA global, tile search (vga_tile.hip)
// Beamer's alpha: a level goes top-down when the frontier's runs are fewer than the unvisited cells / alpha.
// 60 with the frontier in LDS (r5_vga1000_knobs_ab.jsonl, r6 knobs.jsonl: 30 / 60 / 120 within 3 %), 1000 with
// the frontier in HBM (grids above ~1010^2: top-down levels there cost a global pass; r5 probe_vga2000)
constexpr int kVgaTileAlpha = 60;
constexpr int kVgaTileAlphaHbm = 1000;
// tile-common runs tested in phase A (all 4: the last two save ~20 % of the phase-B cell tests)
constexpr int kVgaTileCommonRuns = 4;
// consecutive sources a workgroup takes per grab (neighbouring sources share L2 lines and hit hints)
constexpr int kVgaSourceChunk = 1;
// ---- VGA global, direction-optimising fallback (vga_do.hip)
constexpr int kVgaDoAlpha = 15;
constexpr int kVgaDoShortList = 16;

// ---- memory: optional summaries are built only within a share of the free device memory, so a graph
// that fills the GPU still runs (on the slower exact path that needs no summary)
// tile rows (tvis / ftvis) and partial-tile masks on narrow grids: a quarter of the free memory
constexpr int kMemShareDiv = 4;
// tile rows on wide grids (above 1024^2), where the scan order's place is released for them: a third
constexpr int kMemShareWideDiv = 3;
// a per-workgroup LDS budget above which a preparation pass takes its HBM variant (of the 160 KiB a CU)
constexpr int kLdsPassBudget = 150 * 1024;

// ---- test hooks
inline const char* hook(const char* name) { return std::getenv(name); }
inline int hook_int(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return e ? std::atoi(e) : dflt;
}

}  // namespace policy
}  // namespace dmx
