// Common definitions for the channel_gpu_amd native core (gfx950 / MI355X only).
//
// Error handling replaces the reference's check.cu (check.cu:3-79), which printed and called
// exit(1) on the failing rank only (so peers hung in the next collective).  Here every
// failure throws a channel::Error; the driver catches it and aborts the whole job (RCCL abort +
// MPI_Abort), and the Python bindings turn it into a RuntimeError.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <sstream>
#include <stdexcept>
#include <string>

namespace channel {

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

[[noreturn]] inline void fail(const std::string& msg, const char* file, int line) {
  std::ostringstream os;
  os << "channel error at " << file << ":" << line << ": " << msg;
  throw Error(os.str());
}

// Debug mode: synchronise after every launch so asynchronous faults are attributed to the kernel
// that caused them (the reference's kernelCheck ran cudaGetLastError without a sync, check.cu:7).
bool debug_sync_enabled();
// version of the HIP runtime this process is bound to (hipRuntimeGetVersion; torch imports bring their own)
int hip_runtime_version();
void set_debug_sync(bool on);
// LDS poison-fill debug mode (CHANNEL_LDS_POISON=1 or set_lds_poison): the hot kernels fill their
// shared memory with NaN bit patterns before any use, so a read of an LDS slot that the kernel
// never wrote turns the result into NaN instead of silently reusing stale data
bool lds_poison_enabled();
void set_lds_poison(bool on);
// SIGSEGV/SIGBUS/SIGABRT handler that writes the native backtrace (execinfo) to stderr before the
// process dies (failure diagnosis on boxes without a debugger); CHANNEL_CRASH_TRACE=1 installs it
// at library load
void install_crash_handler();

// Number of blocks of `kernel` (with `threads` per block and `dyn_lds` dynamic LDS) that are
// resident on the current device at once: CUs x occupancy.  Persistent kernels size their grid
// with it.  Cached per (device, kernel).
int resident_blocks(const void* kernel, int threads, size_t dyn_lds = 0);

}  // namespace channel

#define CH_CHECK(cond, msg)                                          \
  do {                                                               \
    if (!(cond)) {                                                   \
      std::ostringstream _os;                                        \
      _os << msg;                                                    \
      ::channel::fail(_os.str(), __FILE__, __LINE__);                \
    }                                                                \
  } while (0)

#define HIP_CHECK(expr)                                                                   \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess) {                                                               \
      ::channel::fail(std::string(#expr) + " -> " + hipGetErrorString(_e), __FILE__, __LINE__); \
    }                                                                                     \
  } while (0)

// After a kernel launch: catch launch-configuration errors immediately, and in debug mode also
// execution faults.
#define HIP_LAUNCH_CHECK(stream)                                                          \
  do {                                                                                    \
    HIP_CHECK(hipGetLastError());                                                         \
    if (::channel::debug_sync_enabled()) HIP_CHECK(hipStreamSynchronize(stream));         \
  } while (0)
