// Host memory: pinned, page-aligned arrays visible to every GPU — the
// MI355X-native replacement for the reference's aligned native arrays
// (CSpaceArrays.cs:108-147 createArray/alignedArrHead/deleteArray/copyMemory,
// FastArr<T> :234-322) and for CL_MEM_USE_HOST_PTR zero-copy buffers
// (ClBuffer.cs:294-300).  Without a GPU runtime (CPU-only host) the same API
// falls back to posix_memalign.
#pragma once
#include "common.h"

namespace cek {

// Allocate `bytes` aligned to `align` (>= 4096 recommended).  Pinned +
// mapped + portable when a HIP device exists.
void* host_alloc(uint64_t bytes, uint64_t align, bool* pinned);
void host_free(void* p);
bool host_is_pinned(const void* p);

// Page-lock an existing host range (e.g. a numpy buffer); refcounted.
bool host_register(void* p, uint64_t bytes);
void host_unregister(void* p);
// Device-visible pointer of pinned/registered host memory (zero-copy).
void* host_device_ptr(void* p);

void copy_memory(void* dst, const void* src, uint64_t bytes);

}  // namespace cek
