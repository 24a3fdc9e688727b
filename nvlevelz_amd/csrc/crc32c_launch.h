// nvlevelz_amd/csrc/crc32c_launch.h -- host-side helpers shared by the
// kernel TUs (grids, the head kernel launcher, cross-TU launchers).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "crc32c_dev_heads.h"

namespace nvl {

inline uint32_t grid_for(int num_cu, uint64_t T) {
  uint64_t g = (T + dev::kWavesPerWG - 1) / dev::kWavesPerWG;
  if (g > (uint64_t)num_cu) g = (uint64_t)num_cu;
  return g ? (uint32_t)g : 1u;
}

inline uint32_t chunks_of(uint64_t len) { return dev::chunks_for(len); }

// The head kernel over a geometry's n buffers; its dispatch records
// ev_start when given (it is then the call's first kernel).
constexpr uint32_t kHeadGridMult = 1;  // head kernel workgroups per CU (A/B'd; the fused plan takes <= 1023 tiles)
inline uint32_t head_grid(int num_cu, uint64_t n) {
  const uint64_t per_wg = 8u * dev::kWavesPerWG;  // at least ~8 buffers per wave
  const uint64_t cap = std::min<uint64_t>((uint64_t)num_cu * kHeadGridMult, dev::kMaxTiles);
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(cap, (n + per_wg - 1) / per_wg));
}

template <class G>
hipError_t launch_heads(const LaunchCtx& lc, const G& g, uint32_t* out, uint32_t flags, uint32_t* hc,
                               hipEvent_t ev_start, uint64_t* lpre = nullptr, uint64_t* tiles = nullptr,
                               bool short_ok = false, hipEvent_t ev_stop = nullptr) {
  const uint32_t grid = head_grid(lc.num_cu, g.n);
  dev::KArgs ka{out, flags, nullptr, lc.tables, nullptr, hc};
  ka.short_ok = short_ok ? 1u : 0u;
  if (lpre) {  // tiles of the variable-length plan: one per workgroup
    ka.lpre = lpre;
    ka.tiles = tiles;
    ka.tile_G = grid;
    ka.tile_S = (g.n + grid - 1) / grid;
  }
  if (ev_start || ev_stop)
    hipExtLaunchKernelGGL(dev::crc32c_head_kernel<G>, dim3(grid), dim3(dev::kThreads), 0, lc.stream, ev_start,
                          ev_stop, 0u, g, ka);
  else
    hipLaunchKernelGGL(dev::crc32c_head_kernel<G>, dim3(grid), dim3(dev::kThreads), 0, lc.stream, g, ka);
  return hipGetLastError();
}

// crc32c_fixed.hip: the fix-up kernel over scheduler B's unit records.
hipError_t launch_fixup(const Rec* recs, uint32_t nw, uint32_t* out, uint32_t flags, hipStream_t st,
                        hipEvent_t ev_stop = nullptr);
// crc32c_batch.hip: the routed call's third launch (crc32c_var_fused_kernel over the
// route's verdict), launched by crc32c_region.hip's launch_routed.
hipError_t launch_var_body(const LaunchCtx& lc, const dev::VarGeom& g, const dev::KArgs& ka);

inline size_t align256(size_t v) { return (v + 255u) / 256u * 256u; }

}  // namespace nvl
