// lds_dma_probe.hip -- hardware facts the LDS-gathered light kernel relies on
// (diagnostic; standalone: hipcc --offload-arch=gfx950 -O2 lds_dma_probe.hip -o lds_dma_probe):
//  1. buffer_load_dwordx4 ... lds writes lane i's 16 B at M0 + 16 i, and
//     EXEC-masked lanes write nothing;
//  2. the raw-buffer range check on a 16-B access that straddles num_records:
//     per dword (in-range dwords kept) or per access (all four dwords zero);
//  3. the same for a 4-B access (buffer_load_dword ... lds).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :: "v"(voff), "s"(rs), "s"(lds) : "memory", "m0");
}
__device__ __forceinline__ void dma4(__amdgpu_buffer_rsrc_t rs, unsigned voff, unsigned lds) {
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dword %0, %1, 0 offen lds"
               :: "v"(voff), "s"(rs), "s"(lds) : "memory", "m0");
}

__global__ void __launch_bounds__(64) kprobe(const float* src, float* out, int nrec, int nact, int wide) {
  __shared__ __attribute__((aligned(16))) float buf[64 * 4 + 64];
  const int lane = threadIdx.x;
  for (int i = lane; i < 64 * 4 + 64; i += 64) buf[i] = -1.0f;  // sentinel
  __syncthreads();
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, nrec, 0x00020000);
  const unsigned base = (unsigned)(size_t)&buf[16];  // 64-B offset into the array
  if (lane < nact) {
    if (wide) dma16(rs, lane * 16, __builtin_amdgcn_readfirstlane(base));
    else dma4(rs, lane * 4, __builtin_amdgcn_readfirstlane(base));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = lane; i < 64 * 4 + 64; i += 64) out[i] = buf[i];
}

int main() {
  const int n = 64 * 4 + 64;
  float h[n], *ds, *dout;
  for (int i = 0; i < n; ++i) h[i] = float(i + 1);
  hipMalloc(&ds, n * sizeof(float));
  hipMalloc(&dout, n * sizeof(float));
  hipMemcpy(ds, h, sizeof(h), hipMemcpyHostToDevice);
  struct Case { int nrec, nact, wide; const char* what; } cases[] = {
      {1024, 64, 1, "dwordx4, all lanes, all in range"},
      {1024, 42, 1, "dwordx4, lanes < 42 active"},
      {664, 42, 1, "dwordx4, num_records 664 (lane 41 straddles: 656..671)"},
      {664, 64, 0, "dword, num_records 664"},
      {662, 64, 0, "dword, num_records 662 (lane 165/4 straddles)"},
  };
  int bad = 0;
  for (const Case& c : cases) {
    float o[n];
    hipLaunchKernelGGL(kprobe, dim3(1), dim3(64), 0, 0, ds, dout, c.nrec, c.nact, c.wide);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
    hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
    // o[16 + k] is LDS dword k of the image; expected src dword k when in range
    const int elem = c.wide ? 4 : 1;
    int lanes_ok = 1, last_in = -1, first_zero = -1, writes_past = 0;
    for (int k = 0; k < 64 * elem; ++k) {
      const int lane = k / elem;
      const float v = o[16 + k];
      const bool act = lane < c.nact;
      if (!act) { if (v != -1.0f) writes_past++; continue; }
      if (4 * (k + 1) <= c.nrec) { if (v != float(k + 1)) lanes_ok = 0; else last_in = k; }
      else if (first_zero < 0) first_zero = k;
    }
    printf("%-55s in-range ok=%d last_ok_dword=%d ", c.what, lanes_ok, last_in);
    if (first_zero >= 0) {
      printf("| dwords %d..%d (straddling access):", (first_zero / elem) * elem, (first_zero / elem) * elem + elem - 1);
      for (int k = (first_zero / elem) * elem; k < (first_zero / elem) * elem + elem; ++k) printf(" %g", o[16 + k]);
    }
    printf(" | masked-lane writes %d | before image %g after image %g\n", writes_past, o[15],
           o[16 + 64 * elem]);
    if (!lanes_ok || writes_past) bad = 1;
  }
  return bad;
}
