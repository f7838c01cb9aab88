// Launch-planner knobs: ONE table of tested defaults, compiled in.  The library never reads the environment; the
// product uses these values as they are.  Tests and measurement scripts switch an entry through fd_set_knob (C ABI,
// include/faithdiff_hip.h) to compare kernel variants in one process (e.g. gemm256 vs gemm8 bitwise, the e4m3 tile
// shapes); fd_reset_knobs restores the table.  Every bitwise batching invariant the GPU suite certifies is certified
// for these defaults.
#include <string.h>

#include "fd_common.h"

namespace {
struct KnobDef {
  const char* name;
  int dflt;
};
// order = enum fd_knob_id (fd_common.h)
const KnobDef kDefs[FDK_COUNT] = {
    {"FD_GEMM8", 1},          // eight-wave 256-row kernels on (0: everything on the 4-wave kernel)
    {"FD_GEMM8_S", 0},        // force the split count (0: planner)
    {"FD_GEMM8_GM", 0},       // force the tile-walk group height (0: planner)
    {"FD_GEMM8_W160", 3},     // bit 0: 256 x 160 tiles where faster; bit 1: take N = 320 from the 4-wave kernel
    {"FD_GEMM8_LNP", 1},      // LN-fold producers with K >= 4096 on the eight-wave 128 x 160 pairwise split
    {"FD_GEMM8_MIDK", 3},     // K splits for the mid-K launches of the 32^2 level (0: off)
    {"FD_F8_TILE", 0},        // force the e4m3 eight-wave tile (256160 / 256128 / 128160 / 64160; 0: planner)
    {"FD_GEMM_CFG", -1},      // 4-wave kernel: force the tile config (-1: planner)
    {"FD_GEMM_SWZ", 1},       // 4-wave kernel: XCD-aware tile order
    {"FD_GEMM_MODE", 0},      // 4-wave kernel diagnostic build mode (1 loads only, 2 MFMA only; probes only)
    {"FD_GEMV", 1},           // few-row GEMV for M <= 4
    {"FD_GEMM256", 1},        // 256 x 256 kernel where it applies (0: gemm8, bitwise-equal reference in tests)
    {"FD_GEMM256_MIN_TILES", 192},
    {"FD_GN_MIN_CHUNKS", 256},     // GroupNorm row-chunk floor for small images
    {"FD_GN_APPLY_V", 2},          // GroupNorm apply: 2 register scale/shift kernel, 1 LDS-table kernel
    {"FD_GN_APPLY_BLOCKS", 1024},  // GroupNorm apply grid cap
    {"FD_GN_APPLY_U", 4},          // GroupNorm apply vectors in flight per thread
    {"FD_FLASH_SWZ", 1},           // flash attention XCD-aware block order
    {"FD_FLASH_WAVES", 4},         // flash attention waves per workgroup (2, 4, 8)
    {"FD_FLASH_QPW", 0},           // flash attention queries per wave (0: by launch size, 16, 32)
    {"FD_CONV_HALO", 1},           // 3x3 stride-1 convs on the halo-staged kernel where eligible (1: not the gemm256 ones; 2: all)
    {"FD_CONV_HALO_MIN_TILES", 192},  // ... when it has at least this many tiles (per TLC tile's rows, m_ref)
    {"FD_CONV_HALO_SPLIT", 1},     // ... or twice that many with the input channels split in two (pairwise combine)
    {"FD_GEMM_GMP", 1},            // 4-wave kernel: tile-row group height planned per launch (0: fixed 4)
    {"FD_CONV_HALO_PT", 3},        // halo conv persistent over tiles (next tile's chunk 0 DMA'd in the K loop) for launches
                                   // of >= 2 tiles per CU: 3 GroupNorm-folded convs without residual, 1 all, 2 also the
                                   // gemm256-eligible ones, 0 off
    {"FD_CONV_HALO_NS16", 3},      // weight-ring depth of its 256 x 128 tiles (3 or 4)
    {"FD_CONV_HALO_SPLIT16", 1},   // 256-row tiles with a pairwise input-channel split before 128-row tiles
    {"FD_CONV_HALO_PP", 1},        // halo conv per-tile forms on the two-group ping-pong K loop (0: one-barrier loop)
};
int g_knobs[FDK_COUNT];
bool g_init = false;

void init_knobs() {
  if (g_init) return;
  for (int i = 0; i < FDK_COUNT; ++i) g_knobs[i] = kDefs[i].dflt;
  g_init = true;
}
}  // namespace

int fd_knob(int id) {
  init_knobs();
  return g_knobs[id];
}

extern "C" int fd_set_knob(const char* name, int value, int* previous) {
  init_knobs();
  if (!name) return FD_ERR_ARG;
  for (int i = 0; i < FDK_COUNT; ++i) {
    if (strcmp(name, kDefs[i].name) == 0) {
      if (previous) *previous = g_knobs[i];
      g_knobs[i] = value;
      return FD_OK;
    }
  }
  return FD_ERR_ARG;
}

extern "C" int fd_get_knob(const char* name, int* value, int* dflt) {
  init_knobs();
  if (!name) return FD_ERR_ARG;
  for (int i = 0; i < FDK_COUNT; ++i) {
    if (strcmp(name, kDefs[i].name) == 0) {
      if (value) *value = g_knobs[i];
      if (dflt) *dflt = kDefs[i].dflt;
      return FD_OK;
    }
  }
  return FD_ERR_ARG;
}

extern "C" const char* fd_knob_name(int id) { return (id >= 0 && id < FDK_COUNT) ? kDefs[id].name : nullptr; }

extern "C" void fd_reset_knobs(void) {
  g_init = false;
  init_knobs();
}

// Split-K hand-off health (include/faithdiff_hip.h): the pairwise split-K waits (gemm8, halo conv) that timed out
// since the last reset.  Synchronous (reads device symbols); the host calls it at its own sync points.
extern "C" int fd_splitk_health(unsigned* timeouts, int reset) {
  if (!timeouts) return FD_ERR_ARG;
  *timeouts = 0;
  int rc = g8_splitk_health(timeouts, reset, -1);
  if (rc == FD_OK) rc = halo_splitk_health(timeouts, reset, -1);
  return rc;
}

// Test hook only: drop = 1 makes every pairwise split-K publisher skip its flag, so the waiting split times out
// (~1 s per tile wave), poisons its tile with NaN and counts the timeout; 0 restores the product behaviour.
extern "C" int fd_splitk_test_drop(int drop) {
  if (drop < 0) return FD_ERR_ARG;
  int rc = g8_splitk_health(nullptr, 0, drop);
  if (rc == FD_OK) rc = halo_splitk_health(nullptr, 0, drop);
  return rc;
}
