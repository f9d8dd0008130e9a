// Shape-keyed kernel routing for the three convolution GEMMs (conv_route.hip).
//
// Every default "which kernel / which tile configuration" decision of conv_fwd_launch,
// conv_dgrad_launch and conv_wgrad_plan is a row of one ordered table: the first row whose
// shape window (filter taps, stride, input / output channels, GEMM rows, tiles) and feature
// flags (fused statistics, residual join, folded BN, fp8, …) match the problem — and whose
// kernel then accepts it (alignment, instantiation, LDS budget) — runs.  The launchers keep only
// those hard eligibility checks; every threshold that came from a measurement lives here, next to
// the profile that chose it.  Overrides act on rows by name (TDL_ROUTE_OFF / TDL_ROUTE_ON /
// TDL_ROUTE_CFG, conv_route_force) and are validated against the configurations each kernel
// family instantiates, so an override can no longer select a tile config the launcher does not
// have (the round-4 "output tiles left unwritten" bug).
#pragma once
#include <stdexcept>
#include <string>

#include "kernels.h"

namespace tdl {

enum RouteImpl { RT_GEMM = 0, RT_GLDS = 1, RT_PC = 2, RT_HALO = 3, RT_ASFWD = 4 };

// problem features that select instantiations (need / forbid masks of a rule)
enum RouteFlag {
  RF_STATS = 1,   // fused BN statistics (FWD Σy, Σy²; DGRAD Σg, Σg·x) the kernel can take
  RF_JOIN = 2,    // DGRAD residual join (dx += …)
  RF_AFF = 4,     // folded BN + ReLU on the input (ConvArgs::aff)
  RF_FP8 = 8,     // fp8 operands
  RF_RES = 16,    // FWD residual epilogue
  RF_BIAS = 32,   // FWD bias
  RF_WFLIP = 64,  // DGRAD: the flipped filter is available (dgrad as a forward conv)
  RF_STATS_JOIN = 128,  // DGRAD: statistics together with a join (only the 8-wave stats tiles)
  RF_STRIDED = 256,     // DGRAD: stride > 1 without dilation (parity classes)
};

struct RouteRule {
  const char* name;      // stable id: overrides, tests, conv_last_route
  int op;                // convk FWD / DGRAD / WGRAD
  int impl;              // RouteImpl
  int taps_min, taps_max;
  int stride1;           // 1: stride-1 problems only
  int cin_min, cin_max;  // C: input channels of the forward conv (DGRAD: dx's)
  int cout_min, cout_max;  // K: output channels of the forward conv (WGRAD: dW rows)
  long rows_min;         // GEMM rows (FWD / DGRAD: output pixels; WGRAD: reduction pixels)
  int tile_m, tile_n;    // tile of the rule's config (tiles_min is counted in these)
  int tiles_min;
  int need, forbid;      // RouteFlag masks
  int cfg;               // the family's tile configuration (ASFWD: the forward loop's — glds
                         // 0 / 4, 100 the halo loader, 102 the producer/consumer kernel)
  bool on;               // default state (off: opt-in rows, TDL_ROUTE_ON)
  bool test;             // active only when its family is forced onto every aligned problem
                         // (conv_set_glds_mode / conv_set_halo_mode 2: the kernel tests)
  const char* evidence;  // the measurement behind the row
};

struct RouteProblem {
  int op, taps, stride, cin, cout;
  long rows;  // GEMM rows (DGRAD: Σ over the parity classes with taps)
  int flags;
  // DGRAD parity classes (0: one class of `rows`): tiles are counted per class
  int ncls = 0;
  long cls_rows[MAX_DG_CLASSES] = {};
};

// the problem of a launcher's ConvArgs (op: 0 FWD, 1 DGRAD, 2 WGRAD)
RouteProblem route_problem(int op, const ConvArgs& a, int flags);

int route_count();
const RouteRule& route_rule(int i);
// index of the first enabled rule after `after` (−1: from the start) that matches `p`; −1 if
// none.  glds_mode / halo_mode 0 skip those families, 2 ignore their size thresholds (tests).
int route_next(const RouteProblem& p, int after);
// the row a launcher ran (per op, this thread) — tests and conv_last_route
void route_record(int op, int idx);
int route_last(int op);
// launches per row since the last reset (HIP-graph replays do not pass through the launchers)
long route_count_of(int idx);
void route_counts_reset();
// force one row for `op` (name; "" clears): route_next then yields only that row (its shape
// window still applies, its size thresholds do not), and a launcher that cannot run it throws
void route_force(int op, const char* name);
int route_forced(int op);
// per-row state after overrides (TDL_ROUTE_OFF / TDL_ROUTE_ON / TDL_ROUTE_CFG=name:cfg,…, then
// route_set): validated against route_cfg_instantiated
int route_cfg(int idx);
bool route_on(int idx);
// in-process A/B: enable / disable a row and / or set its cfg (cfg < 0 keeps it); throws on an
// unknown row or a configuration its kernel does not instantiate
void route_set(const char* name, int on, int cfg);
void route_reset();  // back to the table defaults + environment
// does kernel family `impl` instantiate tile config `cfg` for `op` with these flags?
bool route_cfg_instantiated(int impl, int op, int cfg, int flags);
// the mode (0 off / 1 default / 2 every aligned problem) that governs row `r`'s family
int route_family_mode(const RouteRule& r);

}  // namespace tdl
