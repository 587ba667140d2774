// Internal helpers shared by trace.hip and rt_host.cpp (not part of the ABI).
#pragma once
#include <cstdint>
#include <string>

#include "../../include/rt.h"

namespace rtclj {

// Thread-local last-error slot behind rt_last_error().
int set_error(int code, const std::string& msg);
void clear_error();

// RNG keying shared by host and device (see trace.hip, "RNG").
//   lowbias32 integer hash (C. Wellons' hash-prospector result).
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Per-call key folded from the 64-bit seed on the host.
inline uint32_t seed_key(uint64_t seed) {
  return mix32(static_cast<uint32_t>(seed) ^
               mix32(static_cast<uint32_t>(seed >> 32) ^ 0x85ebca6bu));
}

// Rows produced by a row selection (contiguous or interleaved tiles).
int rows_out(const rt_params& p);

// rt_render's contexts own their streams: before one destroys its stream
// (already synchronised) it drops that stream's adaptive-schedule and
// split-sum entries from the device scenes it launched on (`scenes`, n of
// them; those no longer live are skipped), so the scenes' per-stream slots do
// not fill up with dead streams -- and a direct rt_launch user's entries on a
// stream the context shared (the NULL stream) are left alone (trace.hip).
void release_stream_schedules(void* stream, const void* const* scenes, int n);
// A context that moves from the NULL stream to a stream of its own keeps its
// adaptive tile orders: the entries of `from` in those scenes become `to`'s
// (both streams idle; a scene that already has an entry for `to` keeps it).
void rebind_stream_schedules(void* from, void* to, const void* const* scenes, int n);

}  // namespace rtclj
