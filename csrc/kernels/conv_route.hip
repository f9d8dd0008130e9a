// The convolution routing table (conv_route.h): one ordered row per measured default, the
// matcher, per-row overrides and the record of which row ran.
#include "conv_route.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace tdl {

namespace {
constexpr int FWD = 0, DGRAD = 1, WGRAD = 2;
constexpr int INF = 1 << 30;
constexpr int TAPS = 1 << 20;  // no upper bound on filter taps
constexpr int HT = 16;         // the halo kernel's tap table (conv_halo.hip HALO_MAXTAP)
constexpr int ASF_HALO = 100, ASF_RW = 101, ASF_PC = 102;

// Rows are tried in order; the first whose window matches and whose kernel takes the problem
// runs.  `test` rows are live only while their family is forced onto every aligned problem
// (conv_set_glds_mode / conv_set_halo_mode 2), which also drops every row's rows / tiles minimum.
// clang-format off
// name                           op     impl      taps      s1 cin          cout         rows   tile      tiles need                forbid                                cfg   on     test
const RouteRule kRoutes[] = {
  // -------------------------------------------------------------------------------- forward
  {"fwd.glds.fp8",                FWD,   RT_GLDS,  1, TAPS,  0, 16, INF,     128, INF,    0,     0, 0,     0,  RF_FP8,             0,                                    0,    true,  false,
   "fp8 forward: LDS-DMA kernel only (e4m3 x e4m3, per-tensor scales)"},
  {"fwd.glds.fp8.n64",            FWD,   RT_GLDS,  1, TAPS,  0, 16, INF,     8, 127,      0,     0, 0,     0,  RF_FP8,             0,                                    1,    true,  false,
   "fp8 forward with < 128 outputs: 4-wave 256x64 tiles"},
  {"fwd.pc.folded_bn",            FWD,   RT_PC,    1, TAPS,  0, 64, INF,     128, INF,    4096,  256, 128, 128, RF_AFF,           RF_BIAS | RF_RES | RF_FP8,            0,    true,  false,
   "opt-in BN+ReLU fold: the producer waves stage the transformed A tile (profiles/r05_bnconv_fold_ab.txt)"},
  {"fwd.halo.rw64",               FWD,   RT_HALO,  9, 9,     1, 64, 64,      64, 64,      4096,  0, 0,     0,  0,                  RF_AFF | RF_RES | RF_FP8,             1,    true,  false,
   "stride-1 3x3 64->64: filter resident in LDS, one barrier per 8-row halo tile (conv_halo.hip conv_rw_kernel)"},
  {"fwd.halo.narrow",             FWD,   RT_HALO,  3, HT,    1, 64, INF,     1, 64,       4096,  0, 0,     0,  0,                  RF_AFF | RF_RES | RF_FP8,             0,    true,  false,
   "stride-1 3x3 with <= 64 outputs: halo tiles, ResNet layer1 683 -> 520 us at b1024 (profiles/r04_halo_ab.txt)"},
  {"fwd.halo.aligned",            FWD,   RT_HALO,  3, HT,    1, 64, INF,     1, INF,      0,     0, 0,     0,  0,                  RF_AFF | RF_RES | RF_FP8,             0,    true,  true,
   "tests: every eligible problem on the halo kernel"},
  {"fwd.pc.wide3x3",              FWD,   RT_PC,    2, TAPS,  0, 256, INF,    128, INF,    4096,  256, 128, 128, 0,                RF_AFF | RF_RES | RF_FP8,             0,    true,  false,
   "producer/consumer waves 14-20 % faster on 3x3 with >= 256 inputs (profiles/r04_conv_pc_ab.txt)"},
  {"fwd.glds.wide",               FWD,   RT_GLDS,  1, TAPS,  0, 8, INF,      128, INF,    4096,  256, 128, 128, 0,                RF_AFF | RF_FP8,                      0,    true,  false,
   "LDS-DMA 256x128 tiles for >= 128 outputs; < 128 tiles stay on the GEMM (DeepLab 13x13x1024->256 b64: 20.6 vs 25.0 us)"},
  {"fwd.glds.1x1n64",             FWD,   RT_GLDS,  1, 1,     0, 8, INF,      49, 64,      4096,  256, 64,  128, 0,                RF_AFF | RF_FP8,                      4,    true,  false,
   "1x1 with 64 outputs: 8-wave 256x64 tiles, 35 vs 53 us on 56x56 64->64 (profiles/r02_conv_n64_configs.txt)"},
  {"fwd.glds.stem",               FWD,   RT_GLDS,  2, TAPS,  0, 8, 32,       49, 64,      65536, 256, 64,  128, 0,                RF_AFF | RF_FP8,                      4,    false, false,
   "opt-in: row-packed ResNet stem (7 taps x 24 channels -> 64) on 8-wave 256x64 tiles, 914 vs 1017 us alone at b1024 but no step gain (13,386 / 13,398 vs 13,396 / 13,435 img/s; profiles/r05_stem_ab.txt)"},
  {"fwd.glds.narrow3x3",          FWD,   RT_GLDS,  9, 9,     0, 8, 32,       49, 64,      65536, 256, 64,  128, 0,                RF_AFF | RF_FP8,                      4,    true,  false,
   "3x3 with <= 32 inputs and <= 64 outputs: 8-wave 256x64 LDS-DMA tiles, 256 vs 307 us on the GEMM (Xception-41 150x150 32->64 b128, profiles/r06_narrow_rows.txt)"},
  {"fwd.pc.aligned.aff",          FWD,   RT_PC,    1, TAPS,  0, 64, INF,     65, INF,     0,     0, 0,     0,  RF_AFF,             RF_BIAS | RF_RES | RF_FP8,            0,    true,  true,
   "tests: folded-BN forwards of any size"},
  {"fwd.pc.aligned",              FWD,   RT_PC,    2, TAPS,  0, 256, INF,    65, INF,     0,     0, 0,     0,  0,                  RF_AFF | RF_RES | RF_FP8,             0,    true,  true,
   "tests: every aligned problem on the LDS-DMA family"},
  {"fwd.glds.aligned",            FWD,   RT_GLDS,  1, TAPS,  0, 8, INF,      65, INF,     0,     0, 0,     0,  0,                  RF_AFF | RF_FP8,                      0,    true,  true,
   "tests: every aligned problem on the LDS-DMA family"},
  {"fwd.glds.aligned.n64",        FWD,   RT_GLDS,  1, TAPS,  0, 8, INF,      1, 64,       0,     0, 0,     0,  0,                  RF_AFF | RF_FP8,                      4,    true,  true,
   "tests: every aligned problem on the LDS-DMA family"},
  {"fwd.gemm",                    FWD,   RT_GEMM,  1, TAPS,  0, 1, INF,      1, INF,      0,     0, 0,     0,  0,                  RF_RES | RF_FP8,                      0,    true,  false,
   "register-staged implicit GEMM: small, unaligned and everything else"},
  // -------------------------------------------------------------------------------- input gradient
  {"dgrad.asfwd.fp8",             DGRAD, RT_ASFWD, 1, TAPS,  1, 8, INF,      128, INF,    0,     0, 0,     0,  RF_FP8 | RF_WFLIP,  RF_AFF | RF_STRIDED,                  0,    true,  false,
   "stride-1 fp8 dgrad as the forward conv of e5m2 dy with the e4m3 flipped filter: +0.3 % ResNet-152 fp8 (profiles/r05_fp8_dgrad_as_fwd_ab.txt)"},
  {"dgrad.glds.fp8.n64",          DGRAD, RT_GLDS,  1, TAPS,  0, 8, 64,       128, INF,    0,     0, 0,     0,  RF_FP8,             0,                                    1,    true,  false,
   "fp8 dgrad (e5m2 dy x e4m3 W^T): LDS-DMA kernel only"},
  {"dgrad.glds.fp8",              DGRAD, RT_GLDS,  1, TAPS,  0, 65, INF,     128, INF,    0,     0, 0,     0,  RF_FP8,             0,                                    0,    true,  false,
   "fp8 dgrad (e5m2 dy x e4m3 W^T): LDS-DMA kernel only"},
  {"dgrad.asfwd.rw64",            DGRAD, RT_ASFWD, 9, 9,     1, 64, 64,      64, 64,      4096,  0, 0,     0,  RF_WFLIP,           RF_AFF | RF_FP8 | RF_STRIDED,         ASF_RW, true, false,
   "stride-1 3x3 64->64 dgrad as the forward conv on the resident-filter halo kernel (mask, join, BN-backward sums)"},
  {"dgrad.asfwd.glds.n32",        DGRAD, RT_ASFWD, 1, TAPS,  1, 8, 32,       64, INF,     4096,  256, 64,  128, RF_WFLIP,         RF_STATS_JOIN | RF_AFF | RF_FP8,      4,    true,  false,
   "<= 32-wide dx: the LDS-DMA 8-wave tiles, not the halo loader: 361 vs 714 us (Xception-41 150x150 32<-64 b128, profiles/r06_narrow_rows.txt)"},
  {"dgrad.asfwd.halo",            DGRAD, RT_ASFWD, 3, HT,    1, 8, 64,       64, INF,     4096,  0, 0,     0,  RF_WFLIP,           RF_STATS | RF_AFF | RF_FP8,           ASF_HALO, true, false,
   "<= 64-wide dx as the forward conv of dy on the halo loader: 698 -> 503 us (bench/dgrad_paths.py, profiles/r05_dgrad_as_fwd.txt)"},
  {"dgrad.asfwd.halo.aligned",    DGRAD, RT_ASFWD, 3, HT,    1, 8, INF,      64, INF,     0,     0, 0,     0,  RF_WFLIP,           RF_STATS | RF_AFF | RF_FP8,           ASF_HALO, true, true,
   "tests: every eligible dgrad as a forward on the halo loader"},
  {"dgrad.asfwd.pc",              DGRAD, RT_ASFWD, 2, TAPS,  1, 65, INF,     256, INF,    4096,  256, 128, 128, RF_WFLIP,         RF_STATS | RF_AFF | RF_FP8,           ASF_PC, true,  false,
   "3x3 dgrad as the forward conv on the producer/consumer kernel, 22-31 % (profiles/r05_dgrad_as_fwd.txt)"},
  {"dgrad.asfwd.glds.join.wide",  DGRAD, RT_ASFWD, 1, TAPS,  1, 65, INF,     64, INF,     4096,  256, 128, 128, RF_WFLIP | RF_STATS | RF_JOIN, RF_AFF | RF_FP8,      0,    true,  false,
   "statistics + residual join on the 256x128 tiles, epilogue operands in two halves (229 VGPRs, no spill; conv_common.h store_tile_bf16 RG)"},
  {"dgrad.asfwd.glds.join",       DGRAD, RT_ASFWD, 1, TAPS,  1, 8, INF,      64, INF,     4096,  256, 64,  128, RF_WFLIP | RF_STATS | RF_JOIN, RF_AFF | RF_FP8,      4,    true,  false,
   "statistics + residual join on the forward K loop's 8-wave 256x64 tiles (narrow dx: the wide row takes C >= 65)"},
  {"dgrad.asfwd.glds.n64",        DGRAD, RT_ASFWD, 1, TAPS,  1, 8, 64,       64, INF,     4096,  256, 64,  128, RF_WFLIP,         RF_STATS_JOIN | RF_AFF | RF_FP8,      4,    true,  false,
   "stride-1 dgrad as the forward conv: LDS-DMA K loop, DGRAD epilogue (profiles/r05_dgrad_as_fwd.txt)"},
  {"dgrad.asfwd.glds",            DGRAD, RT_ASFWD, 1, TAPS,  1, 65, INF,     64, INF,     4096,  256, 128, 128, RF_WFLIP,         RF_STATS_JOIN | RF_AFF | RF_FP8,      0,    true,  false,
   "stride-1 dgrad as the forward conv: LDS-DMA K loop, DGRAD epilogue (profiles/r05_dgrad_as_fwd.txt)"},
  {"dgrad.asfwd.strided.n64",     DGRAD, RT_ASFWD, 1, TAPS,  0, 8, 64,       64, INF,     4096,  256, 64,  128, RF_WFLIP | RF_STRIDED, RF_STATS_JOIN | RF_AFF | RF_FP8, 4, true, false,
   "strided dgrad as one forward conv of dy per parity class (bench/dgrad_strided.py)"},
  {"dgrad.asfwd.strided",         DGRAD, RT_ASFWD, 1, TAPS,  0, 65, INF,     64, INF,     4096,  256, 128, 128, RF_WFLIP | RF_STRIDED, RF_STATS_JOIN | RF_AFF | RF_FP8, 0, true, false,
   "strided dgrad as one forward conv of dy per parity class: 3x3/s2 1.2-1.8x, 1x1/s2 1.9-2.2x (bench/dgrad_strided.py)"},
  {"dgrad.halo",                  DGRAD, RT_HALO,  3, HT,    1, 8, INF,      64, INF,     0,     0, 0,     0,  0,                  RF_AFF | RF_FP8,                      0,    true,  true,
   "tests only: the halo dgrad lost to the implicit GEMMs on every measured shape (profiles/r04_halo_ab.txt)"},
  {"dgrad.glds.stats.aff.n64",    DGRAD, RT_GLDS,  1, TAPS,  1, 49, 64,      8, INF,      4096,  256, 64,  128, RF_STATS | RF_AFF, RF_FP8,                              4,    true,  false,
   "folded-BN ReLU mask on the statistics epilogue, 8-wave 256x64"},
  {"dgrad.glds.stats.aff",        DGRAD, RT_GLDS,  1, TAPS,  0, 128, INF,    8, INF,      4096,  256, 128, 128, RF_STATS | RF_AFF, RF_FP8,                              6,    true,  false,
   "folded-BN mask: 8-wave 128x128 tiles (256x128 spills with the coefficient registers)"},
  {"dgrad.glds.1x1n64",           DGRAD, RT_GLDS,  1, 1,     0, 49, 64,      8, INF,      4096,  256, 64,  128, 0,                RF_AFF | RF_FP8,                      4,    true,  false,
   "1x1 with 64-wide dx: 8-wave 256x64 tiles, 49 vs 88 us on 56x56 64->64 (profiles/r02_conv_n64_configs.txt)"},
  {"dgrad.glds.n64.stats",        DGRAD, RT_GLDS,  1, TAPS,  1, 49, 64,      8, INF,      4096,  256, 64,  128, RF_STATS,         RF_AFF | RF_FP8,                      4,    true,  false,
   "64-wide 3x3 dgrads with fused BN sums: within 5 % of the GEMM, saves the BN's reduce pass (profiles/r02_bnstat_fuse_ab.txt)"},
  {"dgrad.glds.stats.join",       DGRAD, RT_GLDS,  1, TAPS,  0, 128, INF,    8, INF,      4096,  256, 128, 128, RF_STATS | RF_JOIN, RF_AFF | RF_FP8,                    6,    true,  false,
   "statistics + join: 8-wave 32x64 wave tiles (256x128 spills; profiles/r02_bnstat_fuse_ab.txt)"},
  {"dgrad.glds.stats",            DGRAD, RT_GLDS,  1, TAPS,  0, 128, INF,    8, INF,      4096,  256, 128, 128, RF_STATS,         RF_JOIN | RF_AFF | RF_FP8,            0,    true,  false,
   "fused BN-backward sums on 256x128 tiles (profiles/r02_bnstat_fuse_ab.txt)"},
  {"dgrad.glds.wide",             DGRAD, RT_GLDS,  1, TAPS,  0, 128, INF,    8, INF,      4096,  256, 128, 128, 0,                RF_AFF | RF_FP8,                      0,    true,  false,
   "LDS-DMA dgrad for >= 128-wide dx (profiles/r01_conv_bench_resnet50_b256_modes.txt)"},
  {"dgrad.glds.aligned.n64",      DGRAD, RT_GLDS,  1, TAPS,  0, 1, 64,       8, INF,      0,     0, 0,     0,  0,                  RF_FP8,                               4,    true,  true,
   "tests: every aligned problem on the LDS-DMA family"},
  {"dgrad.glds.aligned.stats.aff",DGRAD, RT_GLDS,  1, TAPS,  0, 65, INF,     8, INF,      0,     0, 0,     0,  RF_STATS | RF_AFF, RF_FP8,                              6,    true,  true,
   "tests: every aligned problem on the LDS-DMA family"},
  {"dgrad.glds.aligned.stats.join",DGRAD,RT_GLDS,  1, TAPS,  0, 65, INF,     8, INF,      0,     0, 0,     0,  RF_STATS | RF_JOIN, RF_AFF | RF_FP8,                    6,    true,  true,
   "tests: every aligned problem on the LDS-DMA family"},
  {"dgrad.glds.aligned",          DGRAD, RT_GLDS,  1, TAPS,  0, 65, INF,     8, INF,      0,     0, 0,     0,  0,                  RF_FP8,                               0,    true,  true,
   "tests: every aligned problem on the LDS-DMA family"},
  {"dgrad.gemm",                  DGRAD, RT_GEMM,  1, TAPS,  0, 1, INF,      1, INF,      0,     0, 0,     0,  0,                  RF_FP8,                               0,    true,  false,
   "register-staged implicit GEMM over the stride parity classes"},
  // -------------------------------------------------------------------------------- weight gradient
  {"wgrad.glds.fp8",              WGRAD, RT_GLDS,  1, TAPS,  0, 16, INF,    129, INF,    0,     0, 0,     0,  RF_FP8,             0,                                    0,    true,  false,
   "fp8 weight gradient (e5m2 dy x e4m3 x, transposed 8-bit LDS reads): LDS-DMA kernel only"},
  {"wgrad.glds.fp8.m128",         WGRAD, RT_GLDS,  1, TAPS,  0, 16, INF,    16, 128,     0,     0, 0,     0,  RF_FP8,             0,                                    2,    true,  false,
   "fp8 weight gradient with <= 128 output channels: 128x128 tiles"},
  {"wgrad.halo.wide3x3",          WGRAD, RT_HALO,  9, 9,     1, 128, INF,    8, INF,      32768, 0, 0,     0,  0,                  RF_AFF | RF_FP8,                               0,    true,  false,
   "3x3 with >= 128 inputs: halo weight gradient, ResNet-50 layers 2-4 362 -> 295 us at b1024 (profiles/r04_halo_ab.txt); 7x7x512 b1024 287 vs 375 us on the GEMM (profiles/r06_wgrad3x3.txt)"},
  {"wgrad.halo.c64",              WGRAD, RT_HALO,  9, 9,     1, 64, 127,     8, INF,      1000000, 0, 0,   0,  0,                  RF_AFF | RF_FP8,                               0,    true,  false,
   "3x3 weight gradients of 64-127 input channels over >= 1M pixels on the halo kernel: 441 vs 481 us on the register GEMM after its swizzle change (ResNet-50 b1024 56x56x64; profiles/r06_halo_wgrad_swizzle.txt)"},
  {"wgrad.halo.aligned",          WGRAD, RT_HALO,  9, 9,     1, 64, INF,     8, INF,      0,     0, 0,     0,  0,                  RF_AFF | RF_FP8,                               0,    true,  true,
   "tests: every eligible problem on the halo kernel"},
  {"wgrad.glds.stem",             WGRAD, RT_GLDS,  1, TAPS,  0, 1, 32,       1, 64,       65536, 0, 0,     0,  0,                  RF_AFF | RF_FP8,                               7,    false, false,
   "opt-in: one 64x256 tile column for the row-packed stem — slower (r03: 1120 vs 1040 us; r05: 11.6 vs 0.97 ms, profiles/r05_stem_ab.txt)"},
  {"wgrad.glds.1x1",              WGRAD, RT_GLDS,  1, 1,     0, 8, INF,      256, INF,    4096,  0, 0,     0,  0,                  RF_AFF | RF_FP8,                               0,    true,  false,
   "1x1 with >= 256 outputs on the LDS-DMA kernel (3x3 gathers of x favour the others; README round-4 A/B)"},
  {"wgrad.glds.aligned.m128",     WGRAD, RT_GLDS,  1, TAPS,  0, 8, INF,      1, 128,      0,     0, 0,     0,  0,                  RF_AFF | RF_FP8,                               2,    true,  true,
   "tests: every aligned problem on the LDS-DMA family"},
  {"wgrad.glds.aligned",          WGRAD, RT_GLDS,  1, TAPS,  0, 8, INF,      129, INF,    0,     0, 0,     0,  0,                  RF_AFF | RF_FP8,                               0,    true,  true,
   "tests: every aligned problem on the LDS-DMA family"},
  {"wgrad.gemm",                  WGRAD, RT_GEMM,  1, TAPS,  0, 1, INF,      1, INF,      0,     0, 0,     0,  0,                  RF_FP8,                               0,    true,  false,
   "register-staged split-K weight gradient"},
};
// clang-format on
constexpr int kNum = sizeof(kRoutes) / sizeof(kRoutes[0]);

struct State {
  bool on[kNum];
  int cfg[kNum];
};

int find(const char* name) {
  for (int i = 0; i < kNum; ++i)
    if (strcmp(kRoutes[i].name, name) == 0) return i;
  return -1;
}

std::vector<std::string> split_list(const char* s) {
  std::vector<std::string> out;
  std::string cur;
  for (const char* p = s; p && *p; ++p) {
    if (*p == ',' || *p == ' ') {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur += *p;
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

int env_i(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

void set_row(State& s, const char* name, int on, int cfg, const char* who) {
  const int i = find(name);
  if (i < 0) throw std::runtime_error(std::string(who) + ": unknown conv route '" + name + "'");
  if (on >= 0) s.on[i] = on != 0;
  if (cfg >= 0) {
    const RouteRule& r = kRoutes[i];
    if (!route_cfg_instantiated(r.impl, r.op, cfg, r.need))
      throw std::runtime_error(std::string(who) + ": tile config " + std::to_string(cfg) +
                               " is not instantiated for route '" + name + "'");
    s.cfg[i] = cfg;
  }
}

State defaults() {
  State s;
  for (int i = 0; i < kNum; ++i) {
    s.on[i] = kRoutes[i].on;
    s.cfg[i] = kRoutes[i].cfg;
  }
  // knobs of earlier rounds, now row overrides
  if (env_i("TDL_DGSTAT_N64", 1) == 0) set_row(s, "dgrad.glds.n64.stats", 0, -1, "TDL_DGSTAT_N64");
  if (env_i("TDL_GLDS_STEM_WGRAD", 0) != 0) set_row(s, "wgrad.glds.stem", 1, -1, "TDL_GLDS_STEM_WGRAD");
  if (env_i("TDL_DGRAD_AS_FWD", 1) == 0)
    for (const char* n : {"dgrad.asfwd.halo", "dgrad.asfwd.halo.aligned", "dgrad.asfwd.pc",
                          "dgrad.asfwd.glds.n64", "dgrad.asfwd.glds"})
      set_row(s, n, 0, -1, "TDL_DGRAD_AS_FWD");
  for (const auto& n : split_list(getenv("TDL_ROUTE_OFF"))) set_row(s, n.c_str(), 0, -1, "TDL_ROUTE_OFF");
  for (const auto& n : split_list(getenv("TDL_ROUTE_ON"))) set_row(s, n.c_str(), 1, -1, "TDL_ROUTE_ON");
  for (const auto& kv : split_list(getenv("TDL_ROUTE_CFG"))) {
    const size_t c = kv.find(':');
    if (c == std::string::npos) throw std::runtime_error("TDL_ROUTE_CFG: expected name:cfg, got " + kv);
    set_row(s, kv.substr(0, c).c_str(), -1, atoi(kv.c_str() + c + 1), "TDL_ROUTE_CFG");
  }
  return s;
}

State& state() {
  static State s = defaults();
  return s;
}

thread_local int g_last[3] = {-1, -1, -1};
int g_forced[3] = {-1, -1, -1};
long g_count[kNum] = {};  // launches per row since route_counts_reset (host-side bookkeeping)

bool in_window(const RouteRule& r, const RouteProblem& p, bool relax) {
  if (p.taps < r.taps_min || p.taps > r.taps_max) return false;
  if (r.stride1 && p.stride != 1) return false;
  if (p.cin < r.cin_min || p.cin > r.cin_max) return false;
  if (p.cout < r.cout_min || p.cout > r.cout_max) return false;
  if ((p.flags & r.need) != r.need || (p.flags & r.forbid)) return false;
  if (relax) return true;
  if (p.rows < r.rows_min) return false;
  if (r.tiles_min > 0) {
    // FWD: output pixels × output channels; DGRAD: dx pixels (per parity class) × dx channels
    const long cols = p.op == DGRAD ? p.cin : p.cout;
    const long ntn = (cols + r.tile_n - 1) / r.tile_n;
    long ntm = 0;
    if (p.ncls <= 0) {
      ntm = (p.rows + r.tile_m - 1) / r.tile_m;
    } else {
      for (int c = 0; c < p.ncls; ++c) ntm += (p.cls_rows[c] + r.tile_m - 1) / r.tile_m;
    }
    if (ntm * ntn < r.tiles_min) return false;
  }
  return true;
}
}  // namespace

RouteProblem route_problem(int op, const ConvArgs& a, int flags) {
  RouteProblem p;
  p.op = op;
  p.taps = a.R * a.S;
  p.stride = std::max(a.sh, a.sw);
  p.cin = a.C;
  p.cout = a.K;
  p.rows = op == DGRAD ? (long)a.N * a.H * a.W : (long)a.N * a.Ho * a.Wo;
  p.flags = flags;
  return p;
}

int route_count() { return kNum; }
const RouteRule& route_rule(int i) { return kRoutes[i]; }
int route_cfg(int i) { return state().cfg[i]; }
bool route_on(int i) { return state().on[i]; }

void route_set(const char* name, int on, int cfg) { set_row(state(), name, on, cfg, "conv_route_set"); }
void route_reset() { state() = defaults(); }

bool route_cfg_instantiated(int impl, int op, int cfg, int flags) {
  switch (impl) {
    case RT_GEMM:
    case RT_PC:
      return cfg == 0;
    case RT_HALO:  // 1: the resident-filter 3x3 64 -> 64 forward
      return cfg == 0 || (op == FWD && cfg == 1 && !(flags & (RF_AFF | RF_RES | RF_FP8)));
    case RT_ASFWD:
      if (flags & RF_FP8) return op == DGRAD && cfg == 0;
      return op == DGRAD && (cfg == 0 || cfg == 4 || cfg == ASF_HALO || cfg == ASF_RW || cfg == ASF_PC);
    case RT_GLDS:
      if (flags & RF_FP8) return op == WGRAD ? (cfg == 0 || cfg == 2) : (cfg == 0 || cfg == 1);
      if (op == FWD) return (flags & RF_RES) ? (cfg == 0 || cfg == 4) : (cfg >= 0 && cfg <= 5);
      if (op == DGRAD) {
        if (flags & RF_AFF) return cfg == 4 || cfg == 6;
        if (flags & RF_STATS) return cfg >= 0 && cfg <= 6;
        return cfg >= 0 && cfg <= 5;
      }
      return (cfg >= 0 && cfg <= 5) || cfg == 7;
    default:
      return false;
  }
}

int route_family_mode(const RouteRule& r) {
  const int glds = conv_glds_mode(), halo = conv_halo_mode();
  switch (r.impl) {
    case RT_GEMM:
      return 1;
    case RT_HALO:
      return halo;
    case RT_PC:
      // conv_set_pc(0) / TDL_CONV_PC=0: the producer/consumer forward off (the folded BN has no
      // other LDS-DMA kernel, so its rows stay)
      if (conv_pc() == 0 && !(r.need & RF_AFF)) return 0;
      return glds;
    case RT_ASFWD:
      if (glds == 0) return 0;
      return r.cfg == ASF_HALO || r.cfg == ASF_RW ? halo : glds;
    default:
      // fp8 operands exist only on the LDS-DMA kernel: its rows ignore the mode switch
      return (r.need & RF_FP8) ? 1 : glds;
  }
}

int route_next(const RouteProblem& p, int after) {
  const int forced = g_forced[p.op];
  if (forced >= 0) {
    if (after >= forced) return -1;
    return in_window(kRoutes[forced], p, true) ? forced : -1;
  }
  const State& s = state();
  for (int i = after + 1; i < kNum; ++i) {
    const RouteRule& r = kRoutes[i];
    if (r.op != p.op || !s.on[i]) continue;
    const int mode = route_family_mode(r);
    if (mode == 0 || (r.test && mode != 2)) continue;
    if (in_window(r, p, mode == 2)) return i;
  }
  return -1;
}

void route_record(int op, int idx) {
  g_last[op] = idx;
  if (idx >= 0 && idx < kNum) __atomic_fetch_add(&g_count[idx], 1L, __ATOMIC_RELAXED);
}
long route_count_of(int idx) { return __atomic_load_n(&g_count[idx], __ATOMIC_RELAXED); }
void route_counts_reset() {
  for (int i = 0; i < kNum; ++i) __atomic_store_n(&g_count[i], 0L, __ATOMIC_RELAXED);
}
int route_last(int op) { return g_last[op]; }
int route_forced(int op) { return g_forced[op]; }

void route_force(int op, const char* name) {
  if (op < 0 || op > 2) throw std::runtime_error("route_force: op 0 (fwd), 1 (dgrad), 2 (wgrad)");
  if (name == nullptr || !*name) {
    g_forced[op] = -1;
    return;
  }
  const int i = find(name);
  if (i < 0 || kRoutes[i].op != op)
    throw std::runtime_error(std::string("route_force: no route '") + name + "' for this op");
  g_forced[op] = i;
}

}  // namespace tdl
