// rle_coop_limits.h — the largest single buffers the cooperative kernels (rle_coop.hip) take in one
// workgroup: rounds of 16 one-wave tiles (1024 input bytes per encode tile, 1008 stream bytes per
// decode tile) and a decode staging of at most 64 KiB of output (LDS).  The drop-in
// (rle_dropin.cpp) sends zero-copy calls within them to the sized launch, where they run as one
// workgroup, instead of the segmented kernels.
#pragma once
#include <stdint.h>

namespace rle {
constexpr uint32_t kCoopMaxWaves = 16;
constexpr uint32_t kCoopEncRounds = 4, kCoopDecRounds = 5;
constexpr uint64_t kCoopEncMaxBytes = 1024ull * kCoopMaxWaves * kCoopEncRounds;   // 64 KiB
constexpr uint64_t kCoopDecMaxIn = 1008ull * kCoopMaxWaves * kCoopDecRounds;      // 80640
constexpr uint64_t kCoopDecUmax = 65536;
}  // namespace rle
