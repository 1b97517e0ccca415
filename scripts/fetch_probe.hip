// fetch_probe.hip -- calibration of rocprofv3 FETCH_SIZE on gfx950 for the
// access widths the GATConv kernels use (MI355X_MICROARCH.md §HBM: FETCH_SIZE
// reports 1/2 of a 16-B-per-lane streaming read; "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
// Every kernel reads a known set of bytes once, from buffers far larger than
// the 256 MiB Infinity Cache; compare its FETCH_SIZE with the byte count:
//   hipcc --offload-arch=gfx950 -O3 fetch_probe.hip -o fetch_probe
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d out -o run -- ./fetch_probe
// Kernels (each launched once, in this order):
//   k_stream<16|4|2>   sweep of a 2 GiB buffer, 16 / 4 / 2 bytes per lane
//   k_gather<bf16,b16> rows of 166 bf16 at a 336-B pitch (C5's x) in a random
//                      permutation, 2 B per lane (gfd_fwd.h row_regs, bf16)
//   k_gather<bf16,b32> the same rows as 4-B feature pairs
//   k_gather<f32,b32>  rows of 166 fp32 at a 672-B pitch (C4's x), 4 B per lane
// The program prints each kernel's byte counts (the 128-B lines its rows touch,
// counted per row; the rows' own bytes) and its rate, and the gather buffers'
// unique lines (the count if no shared boundary line is fetched twice).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

template <int W>
__global__ void __launch_bounds__(256) k_stream(const char* __restrict__ p, int64_t bytes,
                                                float* __restrict__ out) {
  const int64_t tid = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  const int64_t nt = int64_t(gridDim.x) * blockDim.x;
  float acc = 0.f;
  for (int64_t o = tid * W; o < bytes; o += nt * W) {
    if constexpr (W == 16) {
      const float4 v = *reinterpret_cast<const float4*>(p + o);
      acc += v.x + v.y + v.z + v.w;
    } else if constexpr (W == 4) {
      acc += *reinterpret_cast<const float*>(p + o);
    } else {
      acc += float(*reinterpret_cast<const uint16_t*>(p + o));
    }
  }
  out[tid] = acc;
}

// one wave per row, rows idx[w], idx[w + nw], ...; lane <-> feature (B = 2: one
// bf16 per lane and load, f = lane + 64 q; B = 4: one dword per lane and load,
// a bf16 pair or an fp32 feature)
template <int ES, int B>
__global__ void __launch_bounds__(256) k_gather(const char* __restrict__ x, int64_t pitch, int F,
                                                const int32_t* __restrict__ idx, int64_t rows,
                                                float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  const int64_t nw = (int64_t(gridDim.x) * blockDim.x) >> 6;
  const int units = (F * ES + B - 1) / B;  // B-byte units per row
  float acc = 0.f;
  for (int64_t r = w0; r < rows; r += nw) {
    const char* row = x + int64_t(idx[r]) * pitch;
    for (int u = lane; u < units; u += 64) {
      if constexpr (B == 2)
        acc += float(*reinterpret_cast<const uint16_t*>(row + 2 * u));
      else
        acc += float(*reinterpret_cast<const uint32_t*>(row + 4 * u) & 0xffff);
    }
  }
  out[w0 * 64 + lane] = acc;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int64_t SB = int64_t(2) << 30;  // streamed bytes
  const int64_t R = 6000000;            // gathered rows
  const int F = 166;
  const int64_t pb = 336, pf = 672;     // bf16 / fp32 row pitches (ldx = 168)
  char* buf;
  CK(hipMalloc(&buf, std::max(SB, R * pf)));
  CK(hipMemset(buf, 1, std::max(SB, R * pf)));
  float* out;
  CK(hipMalloc(&out, sizeof(float) * cus * 8 * 256));
  std::vector<int32_t> h(R);
  std::iota(h.begin(), h.end(), 0);
  std::shuffle(h.begin(), h.end(), std::mt19937(7));
  int32_t* idx;
  CK(hipMalloc(&idx, sizeof(int32_t) * R));
  CK(hipMemcpy(idx, h.data(), sizeof(int32_t) * R, hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timed = [&](const char* name, double bytes_lines, double bytes_used, auto launch) {
    (void)hipEventRecord(a);
    launch();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("%-22s lines %.4e B  used %.4e B  %.3f ms  %.2f TB/s (used)\n", name, bytes_lines,
           bytes_used, ms, bytes_used / (ms * 1e-3) / 1e12);
  };
  const dim3 g(cus * 8), t(256);
  timed("k_stream<16>", double(SB), double(SB), [&] { k_stream<16><<<g, t>>>(buf, SB, out); });
  timed("k_stream<4>", double(SB), double(SB), [&] { k_stream<4><<<g, t>>>(buf, SB, out); });
  timed("k_stream<2>", double(SB), double(SB), [&] { k_stream<2><<<g, t>>>(buf, SB, out); });
  // a 336-B row spans whole 128-B lines only at line-aligned starts: count the
  // lines the rows touch (rows share boundary lines with their neighbours)
  auto lines = [&](int64_t pitch, int64_t used) {
    double s = 0;
    for (int64_t r = 0; r < R; ++r) {
      const int64_t b0 = r * pitch, b1 = b0 + used - 1;
      s += double(b1 / 128 - b0 / 128 + 1) * 128;
    }
    return s;
  };
  printf("gather buffers: unique lines bf16 %.4e B, fp32 %.4e B (each line once)\n",
         double((R * pb + 127) / 128 * 128), double((R * pf + 127) / 128 * 128));
  timed("k_gather<bf16,b16>", lines(pb, 2 * F), double(R) * 2 * F,
        [&] { k_gather<2, 2><<<g, t>>>(buf, pb, F, idx, R, out); });
  timed("k_gather<bf16,b32>", lines(pb, 2 * F), double(R) * 2 * F,
        [&] { k_gather<2, 4><<<g, t>>>(buf, pb, F, idx, R, out); });
  timed("k_gather<f32,b32>", lines(pf, 4 * F), double(R) * 4 * F,
        [&] { k_gather<4, 4><<<g, t>>>(buf, pf, F, idx, R, out); });
  CK(hipDeviceSynchronize());
  return 0;
}
