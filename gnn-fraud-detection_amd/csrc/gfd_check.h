// gfd_check.h -- the bounds-checked diagnostic build ("a debug
// build with index-bounds asserts").  Compiled in only with -DGFD_CHECKED
// (GFD_BUILD_VARIANT=checked GFD_EXTRA_FLAGS=-DGFD_CHECKED python -m gfd.build
// -> libgfd_checked.so; load it with GFD_LIB_PATH).  Every forward / backward
// entry point then first validates, on the device, every index array its
// kernels gather through -- rowptr monotone with rowptr[0] = 0 and
// rowptr[n] = E', col in [0, N), slot descriptors inside their rows, hub
// chunks inside their hubs, CSC arrays inside [0, N) / [0, E') -- and the
// first violation is recorded (array, position, value, printed once) and the
// entry point returns GFD_ERR_INDEX before any gather kernel is launched,
// instead of a kernel faulting somewhere inside a gather.  This build
// synchronises the stream once per call to read the record (the product
// library never does), and its one record per device makes concurrent calls
// from several host threads serialise on a host mutex.  The product library
// contains none of this.
#pragma once

#include "gfd_common.h"

namespace gfd {

#ifdef GFD_CHECKED
// first violation of the current check_graph call: {flag, pos, value}
struct CheckRecord {
  int flag;
  int pad;
  long long pos, val;
};
extern __device__ CheckRecord g_check;
__device__ __forceinline__ void check_fail(const char* what, long long pos, long long val,
                                           long long lo, long long hi) {
  if (atomicCAS(&g_check.flag, 0, 1) == 0) {  // one report per call
    g_check.pos = pos;
    g_check.val = val;
    printf("gfd checked build: %s[%lld] = %lld outside [%lld, %lld)\n", what, pos, val, lo, hi);
  }
}
// in a check kernel's body: record and leave the thread (nothing after a bad
// index reads through it)
#define GFD_DCHECK(what, pos, val, lo, hi)                                               \
  do {                                                                                   \
    const long long _v = (long long)(val);                                               \
    if (_v < (long long)(lo) || _v >= (long long)(hi)) {                                 \
      ::gfd::check_fail(what, (long long)(pos), _v, (long long)(lo), (long long)(hi));   \
      return;                                                                            \
    }                                                                                    \
  } while (0)
#endif

// Host entry: validate the index arrays of one destination range (rowptr has
// num_dst + 1 entries, absolute positions into col; sources index [0, N)).
// No-op unless GFD_CHECKED.  csc_* nullable (forward calls).
gfd_status check_graph(const int32_t* rowptr, const int32_t* col, int64_t num_dst, int64_t N,
                       const gfd_plan* plan, const int32_t* colptr, const int32_t* csc_dst,
                       const int32_t* csc_eid, int64_t num_messages, hipStream_t stream);

}  // namespace gfd
