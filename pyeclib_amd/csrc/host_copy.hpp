// Parallel host memcpy for the single-object calls (liberasurecode_encode /
// _decode: one object per call, pageable caller memory on both sides).
//
// A call moves its object through host memory three times -- into the pinned,
// device-mapped staging buffer the kernels read over PCIe, into the k data
// fragments liberasurecode hands back (prepare_fragments_for_encode's copy),
// and the parity (or the decoded object) back out -- and at 4 MiB one core
// copying at ~20 GB/s spends ~0.5 ms on that alone, several times the GPU's
// share.  Copies of 256 KiB or more are therefore cut into 64-KiB-aligned
// pieces and run by a small pool of worker threads together with the calling
// thread (ctypes releases the GIL around the call, so the pool is not held up
// by Python).  Smaller copies stay on the calling thread.
#pragma once

#include <cstddef>
#include <cstdint>

namespace ecamd {

struct CopyJob {
  void* dst;
  const void* src;  // null: zero-fill
  size_t n;
};

// Run every job (any mix of copies and zero-fills) and return when all are done.
void host_copy(const CopyJob* jobs, int count);

inline void host_copy(void* dst, const void* src, size_t n) {
  const CopyJob j{dst, src, n};
  host_copy(&j, 1);
}

// Worker threads of the pool (ECAMD_COPY_THREADS, read once; default a
// quarter of the CPUs in the affinity mask, 2..8,
// 0 = the calling thread only).
int host_copy_threads();

}  // namespace ecamd
