// Layout constants of the frame-sharded driver's packed per-rank result (shard.cpp writes it on
// the device, shard_host.cpp reads the all-gathered rows on rank 0's host).  Host-only header.
#pragma once

#include <cstdint>

namespace rpt {
constexpr int kGidShift = 40;                     // point id = (rank << 40) | own index
constexpr int64_t kPackMagic = 0x5250545332LL;  // "RPTS2"
constexpr int kHdr = 8;                           // int64 header words of a packed result
}  // namespace rpt
