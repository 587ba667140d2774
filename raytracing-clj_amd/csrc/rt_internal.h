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
// Scenes are named by their upload id (scene_uid), never by address: a freed
// scene's address can come back for a new one.
void release_stream_schedules(void* stream, const uint64_t* scene_uids, int n);
// A context that moves from the NULL stream to a stream of its own keeps its
// adaptive tile orders: the entries of `from` in those scenes become `to`'s
// (both streams idle; a scene that already has an entry for `to` keeps it).
void rebind_stream_schedules(void* from, void* to, const uint64_t* scene_uids, int n);
// A device scene's upload id: unique for the process's lifetime.
uint64_t scene_uid(const rt_dscene* ds);

// rt_quantize's byte of one channel as 255 thresholds: t[q] (q = 1..255) is
// the smallest float whose byte is >= q (t[0] unused), so a channel's byte is
// the number of thresholds <= it -- exact for every float, NaN included
// (no comparison holds).  Built once from rt_quantize's own arithmetic
// (rt_host.cpp); the device quantiser (trace.hip) searches it.
const float* quantize_thresholds();
// Enqueue the library's fill kernel (trace.hip): `bytes` (a multiple of 4)
// of p set to byte_value, on `stream` -- in place of hipMemsetAsync, whose
// runtime blit kernel a fresh process would load on its first frame.
// Returns the launch's hipError_t (0: enqueued).
int fill_async(void* p, int byte_value, size_t bytes, void* stream);
// Enqueue the device quantiser: d_out[i] = rt_quantize's byte of d_lin[i].
// Returns the launch's hipError_t (0: enqueued).
int quantize_launch(const float* d_lin, uint8_t* d_out, size_t n, void* stream);

}  // namespace rtclj
