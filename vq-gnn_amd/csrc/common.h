// Shared helpers for the vqgnn HIP library (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../include/vqgnn.h"

namespace vqgnn {

constexpr int kWave = 64;     // CDNA wavefront
constexpr int kNumXcd = 8;    // MI355X: 8 XCDs, private L2 each

// Thread-local last-error text (reentrant: no shared mutable state).
void set_error(const char* fmt, ...);
void clear_error();

inline hipStream_t as_stream(vqgnn_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Launch-status check: turns a HIP error into a VQGNN_ERR_LAUNCH with text.
int check_launch(const char* what);

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// XCD-aware remap of a 1-D workgroup id: blocks b and b+8 share an XCD under
// the observed round-robin dispatch (MI355X_MICROARCH.md §Workgroup dispatch);
// returns an id such that each XCD receives a contiguous range.  Bijective for
// any n (the variant of cdna_hip_programming.md §5, "XCD swizzle").  Speed only.
__device__ __forceinline__ int xcd_remap(int orig, int n) {
  const int q = n / kNumXcd, r = n % kNumXcd;
  const int xcd = orig % kNumXcd, local = orig / kNumXcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
}

// Environment of the alternative-implementation knobs the test suite drives
// (VQGNN_SPMM_FAR, VQGNN_EMA_GLOBAL, VQGNN_ASSIGN_EXACT): each selects another
// kernel whose results are identical to the default's (tested both ways).
inline int path_env(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}

}  // namespace vqgnn

// Measurement knobs (other schedules, chunk sizes, work cut short for timing)
// exist only in builds compiled with -DVQGNN_EXPERIMENTS
// (scripts/build_variant.sh); the default library never reads them, so no
// environment variable can truncate or drop its work.
#ifdef VQGNN_EXPERIMENTS
#define VQGNN_KNOB(name, dflt) (::vqgnn::path_env(name, dflt))
#else
#define VQGNN_KNOB(name, dflt) (dflt)
#endif

#define VQGNN_REQUIRE(cond, ...)                    \
  do {                                              \
    if (!(cond)) {                                  \
      ::vqgnn::set_error(__VA_ARGS__);              \
      return VQGNN_ERR_INVALID;                     \
    }                                               \
  } while (0)
