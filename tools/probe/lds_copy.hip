// tools/probe/lds_copy.hip -- diagnostic only (never part of libcbgpu): a copy kernel with RCCL's device footprint
// on gfx950 (ncclDevKernel_Generic: 512 threads, 37,664 B of static LDS -- llvm-readelf --notes of librccl's gfx950
// code object), staging every 16-byte word through LDS as RCCL's primitives do.  tools/coresidency_probe.py launches
// it on a second stream beside the SpGEMM to see whether such a kernel can start while the persistent heavy grid
// holds every CU's LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

constexpr int kThreads = 512;
constexpr int kLdsWords = 37664 / 16;   // uint4 words

__global__ void __launch_bounds__(kThreads) k_lds_copy(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                       uint64_t n16) {
  __shared__ uint4 stage[kLdsWords];
  const uint64_t stride = (uint64_t)gridDim.x * kThreads;
  for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < n16; i += stride) {
    const int s = threadIdx.x + (int)((i / stride) & 3) * kThreads;
    stage[s % kLdsWords] = src[i];
    __builtin_amdgcn_s_waitcnt(0);
    dst[i] = stage[s % kLdsWords];
  }
}

extern "C" int probe_copy(void* stream, const void* src, void* dst, uint64_t bytes, int nwg) {
  if (nwg <= 0 || !src || !dst) return 1;
  k_lds_copy<<<nwg, kThreads, 0, (hipStream_t)stream>>>((const uint4*)src, (uint4*)dst, bytes / 16);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int probe_lds_bytes(int* out) {
  hipFuncAttributes a;
  if (hipFuncGetAttributes(&a, (const void*)k_lds_copy) != hipSuccess) return 1;
  *out = (int)a.sharedSizeBytes;
  return 0;
}
