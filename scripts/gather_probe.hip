// Diagnostic (scripts/gather_probe.py): random-row gather rate of a plain
// wave-per-batch kernel (lane <-> feature, 8 rows per batch, KF = 3 dword
// loads per row), to separate footprint (TLB / DRAM page) effects from bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <typename T>
__global__ void __launch_bounds__(256) k_probe(const T* __restrict__ x, int64_t ldx, int F,
                                               const int32_t* __restrict__ idx, int64_t batches,
                                               float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  const int64_t nw = (int64_t(gridDim.x) * blockDim.x) >> 6;
  float acc[3] = {0.f, 0.f, 0.f};
  for (int64_t b = w0; b < batches; b += nw) {
    const int j = idx[b * 8 + (lane & 7)];
    float v[8][3];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int jk = __builtin_amdgcn_readlane(j, k);
      const T* r = x + int64_t(jk) * ldx;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int f = lane + 64 * q;
        T t = r[f < F ? f : F - 1];
        if constexpr (sizeof(T) == 4) v[k][q] = t; else v[k][q] = __uint_as_float(uint32_t(t) << 16);
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int q = 0; q < 3; ++q) acc[q] += v[k][q];
  }
  out[w0 * 64 + lane] = acc[0] + acc[1] + acc[2];
}

extern "C" int probe_gather(const void* x, int bf16, int64_t ldx, int F, const int32_t* idx,
                            int64_t batches, float* out, int blocks, void* stream) {
  if (bf16)
    k_probe<uint16_t><<<blocks, 256, 0, (hipStream_t)stream>>>((const uint16_t*)x, ldx, F, idx,
                                                               batches, out);
  else
    k_probe<float><<<blocks, 256, 0, (hipStream_t)stream>>>((const float*)x, ldx, F, idx, batches,
                                                            out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
