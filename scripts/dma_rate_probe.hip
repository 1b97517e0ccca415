// dma_rate_probe.hip -- diagnostic: how fast can one CU gather random x rows
// (672 B = 42 x 16 B, fp32 F = 166 at pitch 168) into LDS, and what does the
// issue cost the issuing wave?  Standalone:
//   hipcc --offload-arch=gfx950 -O3 dma_rate_probe.hip -o dma_rate_probe && ./dma_rate_probe
// Variants (one block of W waves per CU, every wave gathers R rows per round,
// round = issue R rows, then wait for all):
//   mode 0  LDS-DMA  buffer_load_dwordx4 ... lds, 42 lanes per row
//   mode 1  register staging: buffer_load_dwordx4 (42 lanes) -> ds_write_b128
//   mode 2  LDS-DMA with R rows issued, then a wait for the rows of the
//           previous round only (two rounds in flight)
// Prints chip-wide GB/s and the issuing wave's cycles per row (s_memtime).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :: "v"(voff), "s"(rs), "s"(lds) : "memory", "m0");
}

template <int MODE, int R>
__global__ void __launch_bounds__(1024) kgather(const float* __restrict__ x, long ldx,
                                                const int* __restrict__ idx, long rounds,
                                                float* __restrict__ out,
                                                unsigned long long* __restrict__ cyc) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const unsigned base = (unsigned)(size_t)lds;
  const long gw = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * nw + wave));  // uniform: s_load
  float acc = 0.f;
  unsigned long long ic = 0;
  for (long rd = 0; rd < rounds; ++rd) {
    const int* ix = idx + ((gw * rounds + rd) * R) % (1L << 26);
    int j[R];
#pragma unroll
    for (int r = 0; r < R; ++r) j[r] = __builtin_amdgcn_readfirstlane(ix[r]);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const int slot0 = ((rd & 1) * nw + wave) * R;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(x + (size_t)(unsigned)j[r] * ldx), 0, 664, 0x00020000);
      const unsigned la = base + (unsigned)((slot0 + r) * 688);
      if (MODE == 0 || MODE == 2) {
        if (lane < 42) dma16(rs, lane * 16, __builtin_amdgcn_readfirstlane(la));
      } else {
        if (lane < 42) {
          float4 d = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, 0, 0));
          *(float4*)(lds + (slot0 + r) * 688 + lane * 16) = d;
        }
      }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    ic += t1 - t0;
    if (MODE == 2) {
      // keep one round in flight: wait for the previous round only (R younger ops)
      if (R == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if (R == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    acc += *(float*)(lds + (slot0 * 688) + lane * 4);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (lane == 0) atomicAdd(cyc, ic);
}

template <int MODE, int R>
void run(const float* x, const int* idx, float* out, unsigned long long* cyc, int cus, int waves,
         long rounds) {
  const size_t lds = size_t(2) * waves * R * 688;
  if (lds > 160 * 1024) { printf("mode %d R %d waves %d: LDS %zu too large\n", MODE, R, waves, lds); return; }
  hipFuncSetAttribute((const void*)kgather<MODE, R>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipMemset(cyc, 0, 8);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL((kgather<MODE, R>), dim3(cus), dim3(64 * waves), lds, 0, x, 168L, idx, 2L, out, cyc);
  hipMemset(cyc, 0, 8);
  hipEventRecord(a);
  hipLaunchKernelGGL((kgather<MODE, R>), dim3(cus), dim3(64 * waves), lds, 0, x, 168L, idx, rounds, out, cyc);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  unsigned long long c = 0;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  const double rows = double(cus) * waves * rounds * R;
  printf("mode %d  R %d  waves %2d: %7.1f GB/s (%.0f B rows, 664 B used)  issue %6.1f cyc/row/wave  %.3f ms\n",
         MODE, R, waves, rows * 664 / (ms * 1e-3) / 1e9, 672.0, double(c) / rows, ms);
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const long N = 10000000, ld = 168;
  float* x; int* idx; float* out; unsigned long long* cyc;
  if (hipMalloc(&x, sizeof(float) * N * ld) != hipSuccess) return 2;
  hipMemset(x, 0, sizeof(float) * N * ld);
  std::vector<int> h(1 << 26);
  srand(1);
  for (auto& v : h) v = (int)(((unsigned long)rand() * 2654435761ul) % N);
  hipMalloc(&idx, sizeof(int) * (h.size() + 64));
  hipMemcpy(idx, h.data(), sizeof(int) * h.size(), hipMemcpyHostToDevice);
  hipMalloc(&out, sizeof(float) * cus * 1024);
  hipMalloc(&cyc, 8);
  const long rounds = 400;
  run<0, 4>(x, idx, out, cyc, cus, 8, rounds);
  run<0, 8>(x, idx, out, cyc, cus, 8, rounds);
  run<0, 4>(x, idx, out, cyc, cus, 16, rounds);
  run<2, 4>(x, idx, out, cyc, cus, 8, rounds);
  run<2, 8>(x, idx, out, cyc, cus, 8, rounds / 2);
  run<1, 4>(x, idx, out, cyc, cus, 8, rounds);
  run<1, 8>(x, idx, out, cyc, cus, 8, rounds);
  run<1, 4>(x, idx, out, cyc, cus, 16, rounds);
  return 0;
}
