// gfd_light_lds.hip -- the light destinations (2..kLightMax messages, self
// loop included; with dropout also the self-loop-only ones) of the PyG
// GATConv forward (/root/reference/src/models/gat.py:80): the bulk of a
// power-law graph's destinations.  Two kernels:
//
// k_light_alpha: one wave per 16-slot tile: the softmax weights of every
// light destination (PyG softmax: max, exp, sum + 1e-16; dropout on alpha;
// times the launch's Z scale 2^erg) as alpha[slot][message][head] for the
// slot's messages, the training statistics, and the tile's largest message
// count.  Gathers 32 B of source logits per message.
//
// k_light_lds: the gathered x rows go to LDS, not to VGPRs, and the K
// dimension (8 heads x F features) is sliced across the waves instead of the
// output columns, so the aggregation is done in the MFMA A-fragment layout and
// never goes through a Z tile.
//  * Rows (and the alpha rows of k_light_alpha) land by LDS-DMA
//    (buffer_load_dwordx4 ... lds, one instruction per gathered row, per-row
//    buffer descriptor whose per-dword range check zero-fills the row's tail):
//    a tile's 16 destinations x kmax messages are issued one tile ahead into a
//    two-region ring (even tiles at the bottom, odd at the top), so the bytes
//    in flight are LDS, not registers.
//  * KQ = ceil(F / 4) k-steps = 8 KB + kx: wave w owns full k-steps
//    [w KB, w KB + KB) for all 4 column tiles (W stationary in VGPRs as fp16
//    hi / lo fragments) and, when w < 4 kx, the piece (k-step 8 KB + w / 4,
//    column tile w % 4) of the kx extra ones -- every wave issues the same 12
//    KB + 3 MFMAs at F = 166 (KB = 5, kx = 2).  Lane (r, g) of a k-step holds
//    destination r's z for heads 2 g, 2 g + 1 of features 4 s .. 4 s + 3 (the
//    head-pair fragment order of k_pack_frag_q): one ds_read of 4 features per
//    message (identical across g: broadcast), 4 v_pk_fma with the lane's own
//    (alpha_2g, alpha_2g+1) -- no v_readlane per message -- then the fp16
//    hi / lo' split and the MFMAs (3 terms per column tile).
//  * The 8 waves' partial [16 x 64] tiles are summed through LDS (the tile's
//    own ring region, free once every wave has finished its MFMAs).
//  * When the launch's one Z scale is not available (max |x| past 2^20: erg =
//    127) both kernels do nothing and k_stream's light instance takes the
//    class (all three are launched; each checks erg on the device).
//
// Per tile (iteration v):
//   B1  x(v), alpha(v), rid(v) visible
//   D   records(v + 2) load; DMA of alpha(v + 1); rid(v + 1)
//   M   this wave's k-steps of tile v -> acc[4 ct]; between them the DMA of
//       x(v + 1), a few rows per k-step (the LDS-DMA issue rate is about the
//       CU's share of HBM bandwidth: issued in one burst it stalls the wave)
//   B2a every wave done with x(v)
//   P   acc -> LDS (region of tile v)
//   B2b
//   W   s_waitcnt vmcnt(0): x(v + 1), alpha(v + 1), records(v + 2) landed
//   S   8 partials summed, scaled, bias / epilogue, out rows stored
// LDS ownership:
//  * ring region of tile t (parity t & 1): written by DMA / zero fill in D of
//    iteration t - 1 (after B1(t - 1): S(t - 2), the region's last reader, is
//    done), read by M(t), partials of tile t between B2a(t) and B1(t + 1).
//  * alpha[t & 1], rid[t & 1]: written in D of iteration t - 1, read by M(t) /
//    S(t); next written in D of iteration t + 1 (after B1(t + 1)).
// The LDS-DMA is inline asm, invisible to the compiler's wait-count pass (its
// own handling waits vmcnt(0) before every LDS read that might alias); the
// explicit vmcnt(0) of W is the only wait on it, and every ds_read of x(v)
// follows B1(v).  Between D and W no compiler-visible load is consumed (its
// counted wait would not know the DMA is younger and would drain it).
#include "gfd_fwd.h"

using namespace gfd;
using namespace gfd::fwd;

namespace {

constexpr int kLW = 8;                // waves per block
constexpr int kAS = 272;              // alpha row stride in LDS (bytes): [8 msgs][8 heads] f32 + pad
constexpr int kAG = kLightMax * H;    // alpha row stride in HBM (floats)
constexpr int kPartBytes = kLW * 4 * 64 * 16;  // the 8 waves' partial tiles
static_assert(kLightMax <= 6, "ring regions and alpha rows hold 6 messages");

#ifdef GFD_PROF
// Diagnostic build only: per-wave s_memtime cycles of the loop phases summed
// over waves: 0 D, 1 M, 2 B2a, 3 P + B2b, 4 W, 5 S, 6 (unused), 7 B1; 8 tiles
// (wave 0).  Read by gfd_prof_lds_read (scripts/prof_phases.py).
__device__ unsigned long long g_prof_lds[9];
#define GFD_STAMP(i)                                                  \
  do {                                                                \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();       \
    pc[i] += t_ - tp;                                                 \
    tp = t_;                                                          \
  } while (0)
#else
#define GFD_STAMP(i) do {} while (0)
#endif

struct Geom {   // LDS geometry of one launch (bytes unless noted)
  int SB;       // slot bytes: one gathered row, 16 x odd (conflict-free 16-row reads)
  int NC;       // 16-B chunks per row
  int R;        // ring slots
  int PS;       // minimum slots per tile region (the partial sums reuse it)
  int off_alpha, off_rid, off_pw, total;
};

// One LDS-DMA wave-instruction: lane i's 16 B at voff (range-checked against
// nbytes from base) to LDS byte address lds + 16 i.  base, nbytes and lds are
// wave-uniform (made scalar here: the asm needs SGPRs).
__device__ __forceinline__ void dma16(const void* base, uint32_t nbytes, uint32_t voff,
                                      uint32_t lds) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  // (readfirstlane returns int: zero-extend each half, never sign-extend)
  const uint64_t bu =
      (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(b >> 32)))) << 32) |
      uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(b))));
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<void*>(bu), 0, __builtin_amdgcn_readfirstlane(nbytes), 0x00020000);
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :: "v"(voff), "s"(rs), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory", "m0");
}

struct LightRange {  // the light slots' tiles [tb, te) and the last live slot + 1
  int64_t tb, te, lim;
};
__device__ __forceinline__ LightRange light_range(const int64_t* split, int64_t num_dst,
                                                  int to_end) {
  LightRange r;
  r.lim = to_end ? num_dst : split[1];
  r.tb = (split[0] + kTile - 1) / kTile;
  r.te = (r.lim + kTile - 1) / kTile;
  return r;
}

// ---------------------------------------------------------------------------
// k_light_alpha
__global__ void __launch_bounds__(256) k_light_alpha(
    int64_t num_dst, int64_t dst_offset, const int4* __restrict__ desc,
    const int32_t* __restrict__ cols8, const float* __restrict__ st, float slope, float dp,
    uint64_t seed, float* __restrict__ stats, const float* __restrict__ xmax,
    const int64_t* __restrict__ split, int to_end, float* __restrict__ lalpha,
    int32_t* __restrict__ tkmax) {
  const int erg = global_scale_exp(xmax, dp);
  if (erg == 127) return;  // k_stream's light instance runs the class
  const LightRange lr = light_range(split, num_dst, to_end);
  const int lane = threadIdx.x & 63;
  const int h = lane & 7, km = lane >> 3;
  const float sc = ldexpf(1.0f, erg);
  const int64_t nw = int64_t(gridDim.x) * (blockDim.x >> 6);
  for (int64_t t = lr.tb + ((int64_t(blockIdx.x) * blockDim.x + threadIdx.x) >> 6); t < lr.te;
       t += nw) {
    const int64_t sb = t * kTile;
    const int rem = int(min(num_dst - 1 - sb, int64_t(kTile - 1)));  // last valid slot offset
    // lane l: dword l & 3 of slot l >> 2's {row, e_begin, e_end, hub}
    const int dv = reinterpret_cast<const int32_t*>(desc + sb)[min(lane >> 2, rem) * 4 + (lane & 3)];
    // sources: message k of slot r at lane 8 (r & 7) + k of c[r >> 3]
    const int c0 = cols8[(sb + min(lane >> 3, rem)) * 8 + (lane & 7)];
    const int c1 = cols8[(sb + min(8 + (lane >> 3), rem)) * 8 + (lane & 7)];
    // t_i of head h: slot r at lane 8 (r & 7) + h of tv[r >> 3]
    const int rw0 = __builtin_amdgcn_ds_bpermute((4 * (lane >> 3)) << 2, dv);
    const int rw1 = __builtin_amdgcn_ds_bpermute((4 * (8 + (lane >> 3))) << 2, dv);
    const float tv0 = st[(dst_offset + rw0) * 16 + H + h];
    const float tv1 = st[(dst_offset + rw1) * 16 + H + h];
    float sj[kTile];
#pragma unroll
    for (int r = 0; r < kTile; ++r) {
      const int j = __builtin_amdgcn_ds_bpermute((8 * (r & 7) + km) << 2, r < 8 ? c0 : c1);
      sj[r] = st[int64_t(j) * 16 + h];
    }
    int kmax = 1;
#pragma unroll
    for (int r = 0; r < kTile; ++r) {
      if (sb + r >= lr.lim) break;  // wave-uniform; slots past the light range
      const int row = __builtin_amdgcn_readlane(dv, 4 * r);
      const int e0 = __builtin_amdgcn_readlane(dv, 4 * r + 1);
      const int n = min(max(__builtin_amdgcn_readlane(dv, 4 * r + 2) - e0, 0), kLightMax);
      kmax = max(kmax, n);
      const float t_h = __int_as_float(
          __builtin_amdgcn_ds_bpermute((8 * (r & 7) + h) << 2, __float_as_int(r < 8 ? tv0 : tv1)));
      const float v = leaky01(sj[r] + t_h, slope);
      const bool valid = km < n;
      const float m = max_xor8_16_32(valid ? v : -INFINITY);
      const float p = valid ? __expf(v - m) : 0.f;
      const float l = sum_xor8_16_32(p);
      if (__builtin_expect(stats != nullptr, 0) && lane < 8) {  // training only
        float* sr = stats + int64_t(row) * 16 + lane;
        sr[0] = m;
        sr[8] = l;
      }
      float pd = p;
      if (__builtin_expect(dp > 0.f, 0))
        pd = dropout_keep(seed, uint32_t(e0 + km), uint32_t(h), dp) ? p * (1.0f / (1.0f - dp)) : 0.f;
      if (valid) lalpha[(sb + r) * kAG + lane] = pd * (__builtin_amdgcn_rcpf(l + kSoftmaxEps) * sc);
    }
    if (lane == 0) tkmax[t] = kmax;
  }
}

// ---------------------------------------------------------------------------
// k_light_lds

// The records of tile t for rows r0, r0 + 1 as one dword per lane: lanes 0..7
// / 8..15 the sources of messages 0..7 (slot_cols), 16/17 the rows, 18/19
// e_begin, 20/21 e_end, 22 (and the rest) the tile's largest message count;
// slots past num_dst read a clamped copy of the last one.
__device__ __forceinline__ int tile_rec(int64_t t, int r0, int64_t num_dst,
                                        const int4* __restrict__ desc,
                                        const int32_t* __restrict__ cols8,
                                        const int32_t* __restrict__ tkmax, int lane) {
  const int64_t sb = t * kTile;
  const int rem = int(min(num_dst - 1 - sb, int64_t(kTile - 1)));
  const int h = (lane >> 3) & 1;
  if (lane < 16) return cols8[(sb + min(r0 + h, rem)) * 8 + (lane & 7)];
  if (lane < 22) {
    const int q = (lane - 16) >> 1, hh = lane & 1;
    return reinterpret_cast<const int32_t*>(desc + sb)[min(r0 + hh, rem) * 4 + q];
  }
  return tkmax[t];
}

struct TileInfo {
  int kmax;        // messages per slot of the tile (>= 1)
  int reg;         // first ring slot of the tile's region
  int n[2];        // messages of rows r0, r0 + 1 (0: past the end)
  int row[2];      // their rows (local to dst_offset), -1 past the end
};

__device__ __forceinline__ TileInfo tile_info(int rec, int64_t t, int64_t v, int r0, int64_t lim,
                                              const Geom& g) {
  TileInfo ti;
  const int64_t sb = t * kTile;
  ti.kmax = min(max(__builtin_amdgcn_readlane(rec, 22), 1), kLightMax);
  const int need = max(kTile * ti.kmax, g.PS);
  ti.reg = (v & 1) ? g.R - need : 0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const bool lv = sb + r0 + h < lim;
    const int n = __builtin_amdgcn_readlane(rec, 20 + h) - __builtin_amdgcn_readlane(rec, 18 + h);
    ti.n[h] = lv ? min(max(n, 0), ti.kmax) : 0;
    ti.row[h] = lv ? __builtin_amdgcn_readlane(rec, 16 + h) : -1;
  }
  return ti;
}

// D, part 1 (before the k-steps): the alpha rows of tile t for this wave's
// two destinations, zeros into the ring slots and alpha rows of messages
// n .. kmax - 1, the output rows.
template <typename XT>
__device__ __forceinline__ void tile_issue_pre(const TileInfo& ti, int64_t t, int r0,
                                               const float* __restrict__ lalpha, char* ssm,
                                               char* alp, int* rid, const Geom& g, int lane) {
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int r = r0 + hh;
    const int n = ti.n[hh];
    char* ar = alp + r * kAS;
    if (n > 0 && lane < 2 * n)
      dma16(lalpha + (t * kTile + r) * kAG, uint32_t(n * H * 4), uint32_t(lane * 16),
            uint32_t(reinterpret_cast<uintptr_t>(ar)));
    if (lane >= 2 * n && lane < 2 * ti.kmax)
      *reinterpret_cast<uint4*>(ar + lane * 16) = make_uint4(0, 0, 0, 0);
    for (int k = n; k < ti.kmax; ++k) {
      if (lane < g.NC)
        *reinterpret_cast<uint4*>(ssm + size_t(ti.reg + k * kTile + r) * g.SB + lane * 16) =
            make_uint4(0, 0, 0, 0);
    }
    if (lane == 0) rid[r] = ti.row[hh];
  }
}

// D, part 2 (spread over the k-steps): x rows of items [i0, i1) of the
// wave's n0 + n1 gathered rows (item q: row r0 + (q >= n0), message q or
// q - n0) into the ring.
template <typename XT>
__device__ __forceinline__ void tile_issue_rows(const TileInfo& ti, int rec, int r0, int i0,
                                                int i1, const void* x, int64_t ldx, int F,
                                                uint32_t lbase, const Geom& g, int lane) {
  const uint32_t nrec = uint32_t((F * XT::kBytes + 3) & ~3);  // the row's dwords
  const int n0 = ti.n[0], cnt = ti.n[0] + ti.n[1];
  for (int q = i0; q < i1 && q < cnt; ++q) {
    const int hh = q >= n0 ? 1 : 0;
    const int k = q - hh * n0;
    const int j = __builtin_amdgcn_readlane(rec, 8 * hh + k);
    const uint32_t la = lbase + uint32_t((ti.reg + k * kTile + r0 + hh) * g.SB);
#ifndef GFD_LLDS_NODMA  // timing experiment only: no row gather (wrong results)
    if (lane < g.NC) dma16(xrow<XT>(x, j, ldx), nrec, uint32_t(lane * 16), la);
#else
    (void)j; (void)la;
#endif
  }
}

// 4 features of one gathered row as loaded (fp32: 4 dwords; bf16: 2 dwords,
// widened where they are used)
template <typename XT>
struct XRaw {
  typedef typename std::conditional<XT::kBytes == 4, f32x4, uint2>::type T;
};
template <typename XT>
__device__ __forceinline__ float x_feat(const typename XRaw<XT>::T& r, int u) {
  if constexpr (XT::kBytes == 4) {
    return r[u];
  } else {
    const uint32_t w = (u < 2) ? r.x : r.y;
    return __uint_as_float((u & 1) ? (w & 0xffff0000u) : (w << 16));
  }
}

// M: this wave's KB full k-steps and (hp) its piece of the tile, KM messages
// per slot, software-pipelined by hand: the FMAs and fp16 split of k-step i + 1
// run between the MFMAs of k-step i (sched_group_barrier interleave: the two
// waves of a SIMD are in the same phase, so a wave must fill its own MFMA
// gaps), and k-step i + 2's x reads are issued after that.  The aggregation
// uses plain v_fma_f32 (packed f32 VALU beside MFMAs costs more than two plain
// ones; this file is built with -fno-slp-vectorize).
template <typename XT, int KM>
struct ZStep {  // one k-step's A fragments: z of heads (2g, 2g + 1) x 4 features
  typedef typename XRaw<XT>::T XR;
  __device__ __forceinline__ static void fma_split(const XR (&xr)[KM], const f32x2 (&a)[KM],
                                                   bool tail, int s, int F, f16x8& hi,
                                                   f16x8& lo) {
    float z0[4] = {0.f, 0.f, 0.f, 0.f}, z1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KM; ++k)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float xf = x_feat<XT>(xr[k], u);
        if constexpr (XT::kBytes == 2) {
          if (u > 0 && tail && 4 * s + u >= F) xf = 0.f;
        }
        z0[u] = __builtin_fmaf(a[k].x, xf, z0[u]);
        z1[u] = __builtin_fmaf(a[k].y, xf, z1[u]);
      }
    union { f16x8 v; f16x2 p[4]; uint32_t u[4]; } h, l;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x2 z = {z0[u], z1[u]};
      h.p[u] = __builtin_convertvector(z, f16x2);
      l.u[u] = split_lo(z, h.u[u]);
    }
    hi = h.v;
    lo = l.v;
  }
};

template <typename XT, int KM, int KB, bool HP, typename STEP>
__device__ __forceinline__ void tile_mfma(f32x4 (&acc)[4], const char* __restrict__ xs,
                                          const char* __restrict__ as, int SB, int s0, int sp,
                                          int ctp, int KQ, int F,
                                          const f16x8 (&bh)[KB][4], const f16x8 (&bl)[KB][4],
                                          const uint4* __restrict__ pw, STEP&& step) {
  typedef typename XRaw<XT>::T XR;
  constexpr int XB = XT::kBytes * 4;  // bytes of 4 features
  auto kst = [&](int i) { return i < KB ? s0 + i : sp; };
  auto rd = [&](int i, XR (&xr)[KM]) {
#pragma unroll
    for (int k = 0; k < KM; ++k)
      xr[k] = *reinterpret_cast<const XR*>(xs + k * kTile * SB + kst(i) * XB);
  };
  // features past F read as 0 from the per-dword range check, except the
  // odd tail feature of a bf16 row (its dword is in range): masked
  auto tailf = [&](int i) { return XT::kBytes == 2 && (F & 1) && kst(i) == KQ - 1; };
  constexpr int S = KB + (HP ? 1 : 0);  // k-steps of this wave
  f32x2 a[KM];
  XR xr[KM];
  f16x8 hA, lA, hB, lB;
#pragma unroll
  for (int k = 0; k < KM; ++k) a[k] = *reinterpret_cast<const f32x2*>(as + k * 32);
  rd(0, xr);
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) acc[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  ZStep<XT, KM>::fma_split(xr, a, tailf(0), kst(0), F, hA, lA);
  __builtin_amdgcn_sched_barrier(0);
  if (1 < S) rd(1, xr);
  step(0);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < S; ++i) {
    // the fragments of k-step i are in (hA, lA) for even i, (hB, lB) for odd i
    const f16x8& hc = (i & 1) ? hB : hA;
    const f16x8& lc = (i & 1) ? lB : lA;
    f16x8& hn = (i & 1) ? hA : hB;
    f16x8& ln = (i & 1) ? lA : lB;
    if (i < KB) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hc, bh[i < KB ? i : 0][ct], acc[ct], 0, 0, 0);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hc, bl[i < KB ? i : 0][ct], acc[ct], 0, 0, 0);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(lc, bh[i < KB ? i : 0][ct], acc[ct], 0, 0, 0);
    } else {  // the piece: its W from LDS (kept out of the register budget)
      const uint4 wh = pw[0], wo = pw[64];
      const f16x8 ph = *reinterpret_cast<const f16x8*>(&wh);
      const f16x8 pl = *reinterpret_cast<const f16x8*>(&wo);
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        if (ct == ctp) {  // wave-uniform
          acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hc, ph, acc[ct], 0, 0, 0);
          acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hc, pl, acc[ct], 0, 0, 0);
          acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(lc, ph, acc[ct], 0, 0, 0);
        }
      }
    }
    if (i + 1 < S) {
      ZStep<XT, KM>::fma_split(xr, a, tailf(i + 1), kst(i + 1), F, hn, ln);
      if (i < KB) {  // 12 MFMAs: interleave the FMA / split VALU into their gaps
        constexpr int V = (8 * KM + 12 + 11) / 12;
#pragma unroll
        for (int g = 0; g < 12; ++g) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
          __builtin_amdgcn_sched_group_barrier(0x002, V, 0);  // VALU
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (i + 2 < S) rd(i + 2, xr);
    step(i + 1);  // the next tile's DMA pieces of this k-step
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <typename XT, int KB>
__global__ void __launch_bounds__(kLW * 64, 2) k_light_lds(
    const void* __restrict__ x, int F, int64_t ldx, int64_t num_dst,
    const int4* __restrict__ desc, const int32_t* __restrict__ cols8,
    const float* __restrict__ lalpha, const int32_t* __restrict__ tkmax,
    const PackHeader* __restrict__ hdr, const uint4* __restrict__ wqh,
    const uint4* __restrict__ wql, const float* __restrict__ bias, float dp,
    float* __restrict__ out, const float* __restrict__ xmax, const int64_t* __restrict__ split,
    int to_end, Epi ep, Geom g) {
  extern __shared__ __attribute__((aligned(16))) char ssm[];
  const int erg = global_scale_exp(xmax, dp);
  if (erg == 127) return;  // k_stream's light instance runs this launch's class
  const uint32_t lbase = uint32_t(reinterpret_cast<uintptr_t>(ssm));
  char* alpha0 = ssm + g.off_alpha;                       // [2][16][kAS]
  int* rid0 = reinterpret_cast<int*>(ssm + g.off_rid);     // [2][16]

  const int wave = wave_uniform(threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  const int r0 = 2 * wave;
  const int KQ = (F + 3) / 4;
  const int kx = KQ - kLW * KB;  // extra k-steps (0..2), as 4 kx (k-step, column tile) pieces
  const int s0 = wave * KB;
  const bool hp = wave < 4 * kx;
  const int sp = kLW * KB + (wave >> 2), ctp = wave & 3;
  const LightRange lr = light_range(split, num_dst, to_end);
  const int64_t G = gridDim.x;
  const int64_t t0 = blockIdx.x;
  const int64_t nv = t0 < lr.te - lr.tb ? (lr.te - lr.tb - 1 - t0) / G + 1 : 0;
  auto tile = [&](int64_t v) { return lr.tb + t0 + v * G; };

  // kernel-lifetime constants: W of this wave's k-steps, all 4 column tiles,
  // and of its piece
  const float wu = hdr->w_unscale;
  const int ctw = wave & 3, ipw = wave >> 2;  // S: column tile, row pair of the partials
  const float bcol = bias ? bias[ctw * 16 + (lane & 15)] : 0.f;
  f16x8 bh[KB][4], bl[KB][4];
#pragma unroll
  for (int i = 0; i < KB; ++i)
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int idx = ((s0 + i) * 4 + ct) * 64 + lane;
      const uint4 vh = wqh[idx], vl = wql[idx];
      bh[i][ct] = *reinterpret_cast<const f16x8*>(&vh);
      bl[i][ct] = *reinterpret_cast<const f16x8*>(&vl);
    }
  uint4* pw = reinterpret_cast<uint4*>(ssm + g.off_pw) + wave * 2 * 64 + lane;  // [8][hi, lo][64]
  if (hp) {
    const int idx = (sp * 4 + ctp) * 64 + lane;
    pw[0] = wqh[idx];
    pw[64] = wql[idx];
  }
  if (nv == 0) return;  // uniform per block

  // prologue: records of tiles 0 and 1, tile 0 issued
  int rec_n = tile_rec(tile(0), r0, num_dst, desc, cols8, tkmax, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  TileInfo tc = tile_info(rec_n, tile(0), 0, r0, lr.lim, g);
  tile_issue_pre<XT>(tc, tile(0), r0, lalpha, ssm, alpha0, rid0, g, lane);
  tile_issue_rows<XT>(tc, rec_n, r0, 0, 2 * kLightMax, x, ldx, F, lbase, g, lane);
  if (nv > 1) rec_n = tile_rec(tile(1), r0, num_dst, desc, cols8, tkmax, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const float osc = ldexpf(1.0f, -erg) * wu;

#ifdef GFD_PROF
  unsigned long long pc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tp = __builtin_amdgcn_s_memtime();
#endif
  for (int64_t v = 0; v < nv; ++v) {
    // an opaque lane: per-lane values derived from it are recomputed in the
    // loop instead of being hoisted and pinned in VGPRs next to W
    lane = opaque(threadIdx.x & 63);
    const int par = int(v & 1);
    __syncthreads();  // B1: x(v), alpha(v), rid(v); S(v - 1) done with its region
    GFD_STAMP(7);
    // D: tile v + 1 (records loaded last iteration), records of v + 2
    // (records first: nothing the compiler waits for may follow the DMA)
    const bool more = v + 1 < nv;
    const int rec_1 = rec_n;
    if (v + 2 < nv) rec_n = tile_rec(tile(v + 2), r0, num_dst, desc, cols8, tkmax, lane);
    TileInfo tn = tc;
    if (more) {
      tn = tile_info(rec_1, tile(v + 1), v + 1, r0, lr.lim, g);
      tile_issue_pre<XT>(tn, tile(v + 1), r0, lalpha, ssm, alpha0 + (par ^ 1) * kTile * kAS,
                         rid0 + (par ^ 1) * kTile, g, lane);
    } else {
      tn.n[0] = tn.n[1] = 0;  // nothing to issue
    }
    GFD_STAMP(0);
    // M, with the x rows of tile v + 1 issued piece by piece between the k-steps
    f32x4 acc[4];
    {
      const char* xs = ssm + size_t(tc.reg + (lane & 15)) * g.SB;
      const char* as = alpha0 + par * kTile * kAS + (lane & 15) * kAS + 8 * (lane >> 4);
      constexpr int QS = (2 * kLightMax + KB) / (KB + 1);  // rows per k-step
      auto step = [&](int i) {  // i = 0 .. S (<= KB + 1): the last call issues the rest
        tile_issue_rows<XT>(tn, rec_1, r0, QS * i, i >= KB ? 2 * kLightMax : QS * (i + 1), x, ldx,
                            F, lbase, g, lane);
      };
#define GFD_M(KM)                                                                       \
  (hp ? tile_mfma<XT, KM, KB, true>(acc, xs, as, g.SB, s0, sp, ctp, KQ, F, bh, bl, pw, step) \
      : tile_mfma<XT, KM, KB, false>(acc, xs, as, g.SB, s0, sp, ctp, KQ, F, bh, bl, pw, step))
      switch (tc.kmax) {
        case 1: GFD_M(1); break;
        case 2: GFD_M(2); break;
        case 3: GFD_M(3); break;
        case 4: GFD_M(4); break;
        case 5: GFD_M(5); break;
        default: GFD_M(6); break;
      }
#undef GFD_M
    }
    GFD_STAMP(1);
    __syncthreads();  // B2a: every wave done with x(v)
    GFD_STAMP(2);
    f32x4* P = reinterpret_cast<f32x4*>(ssm + size_t(tc.reg) * g.SB);
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) P[(wave * 4 + ct) * 64 + lane] = acc[ct];
    __syncthreads();  // B2b: partials visible
    GFD_STAMP(3);
    // W: tile v + 1's rows and alpha and the records of v + 2 landed.  Before
    // S: no load the compiler waits for (the epilogue's) may be consumed while
    // the DMA is in flight -- its wait counts do not know the DMA is there.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    GFD_STAMP(4);
    {
      f32x2 sum = {0.f, 0.f};
#pragma unroll
      for (int w = 0; w < kLW; ++w)
        sum += *reinterpret_cast<const f32x2*>(
            reinterpret_cast<const char*>(P + (w * 4 + ctw) * 64 + lane) + 8 * ipw);
      const int* rid = rid0 + par * kTile;
      const int n = ctw * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int ri = rid[4 * (lane >> 4) + 2 * ipw + e];
        if (ri >= 0) out[int64_t(ri) * C + n] = epi_store_value(sum[e] * osc, bcol, n, ri, ep);
      }
    }
    GFD_STAMP(5);
    tc = tn;
  }
#ifdef GFD_PROF
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) atomicAdd(&g_prof_lds[i], pc[i]);
    if (wave == 0) atomicAdd(&g_prof_lds[8], (unsigned long long)nv);
  }
#endif
}

Geom light_geom(int F, int eb) {
  Geom g;
  g.NC = (F * eb + 15) / 16;
  g.SB = 16 * (g.NC | 1);
  g.PS = (kPartBytes + g.SB - 1) / g.SB;
  const int region = max(kTile * kLightMax, g.PS);
  const int rest = 2 * kTile * kAS + 2 * kTile * int(sizeof(int)) + kLW * 2 * 64 * 16;
  g.R = int((kLdsBytes - size_t(rest)) / size_t(g.SB));
  if (g.R < 2 * region) g.R = -1;
  // ring first (slot addresses from 0), then alpha and rid
  g.off_alpha = g.R * g.SB;
  g.off_rid = g.off_alpha + 2 * kTile * kAS;
  g.off_pw = g.off_rid + 2 * kTile * int(sizeof(int));  // the pieces' W: [8 waves][hi, lo][64]
  g.total = g.off_pw + kLW * 2 * 64 * 16;
  return g;
}

// KQ = 8 KB + kx with KB in {4, 5} and kx <= 2 (F in 125..136 and 157..168)
int light_kb(int F) {
  const int KQ = (F + 3) / 4;
  for (int kb = 4; kb <= 5; ++kb)
    if (KQ >= kLW * kb && KQ - kLW * kb <= 2) return kb;
  return 0;
}

}  // namespace

namespace gfd {
namespace fwd {

size_t light_alpha_bytes(int64_t num_dst) { return size_t(num_dst) * kAG * sizeof(float); }
size_t light_tkmax_bytes(int64_t num_dst) { return size_t((num_dst + kTile - 1) / kTile) * 4; }

bool light_lds_supported(const AggArgs& a, const PackLayout& L) {
  (void)L;
  const int eb = a.xdt == GFD_DTYPE_BF16 ? 2 : 4;
  const uintptr_t base = reinterpret_cast<uintptr_t>(a.x);
  if (!light_kb(a.F) || !a.xmax || !a.lalpha || !a.tkmax) return false;
  if (base % 16 != 0 || (a.ldx * eb) % 16 != 0) return false;
  if (!a.plan.slot_desc || !a.plan.slot_cols || !a.plan.class_split) return false;
  if (!(a.slope >= 0.f && a.slope <= 1.f)) return false;
  const Geom g = light_geom(a.F, eb);
  return g.R > 0 && size_t(g.total) <= kLdsBytes;
}

gfd_status launch_light_lds(const AggArgs& a, const PackLayout& L, bool to_end,
                            hipStream_t stream) {
  const int eb = a.xdt == GFD_DTYPE_BF16 ? 2 : 4;
  const Geom g = light_geom(a.F, eb);
  const gfd_plan& p = a.plan;
  const int64_t tiles = (a.num_dst + kTile - 1) / kTile;
  {
    int64_t grid = int64_t(cu_count()) * 8;
    if (grid > (tiles + 3) / 4) grid = (tiles + 3) / 4;
    if (grid < 1) return GFD_OK;
    k_light_alpha<<<int(grid), 256, 0, stream>>>(
        a.num_dst, a.dst_offset, reinterpret_cast<const int4*>(p.slot_desc), p.slot_cols, a.st,
        a.slope, a.dp, a.seed, a.stats, a.xmax, p.class_split, to_end ? 1 : 0, a.lalpha, a.tkmax);
    GFD_LAUNCH_CHECK();
  }
  int64_t grid = cu_count();
  if (grid > tiles) grid = tiles;
  auto launch = [&](auto kern) -> gfd_status {
    if (!ensure_lds(reinterpret_cast<const void*>(kern), size_t(g.total))) return GFD_ERR_HIP;
    kern<<<int(grid), kLW * 64, size_t(g.total), stream>>>(
        a.x, a.F, a.ldx, a.num_dst, reinterpret_cast<const int4*>(p.slot_desc), p.slot_cols,
        a.lalpha, a.tkmax, reinterpret_cast<const PackHeader*>(a.packed + L.hdr_off),
        reinterpret_cast<const uint4*>(a.packed + L.wqh_off),
        reinterpret_cast<const uint4*>(a.packed + L.wql_off), a.bias, a.dp, a.out, a.xmax,
        p.class_split, to_end ? 1 : 0, a.ep, g);
    GFD_LAUNCH_CHECK();
    return GFD_OK;
  };
  const bool bf = a.xdt == GFD_DTYPE_BF16;
  switch (light_kb(a.F)) {
    case 4: return bf ? launch(&k_light_lds<XBF16, 4>) : launch(&k_light_lds<XF32, 4>);
    case 5: return bf ? launch(&k_light_lds<XBF16, 5>) : launch(&k_light_lds<XF32, 5>);
    default: return GFD_ERR_UNSUPPORTED;
  }
}

}  // namespace fwd
}  // namespace gfd

#ifdef GFD_PROF
extern "C" int gfd_prof_lds_read(unsigned long long* out9, int reset) {
  if (hipMemcpyFromSymbol(out9, HIP_SYMBOL(g_prof_lds), sizeof(g_prof_lds)) != hipSuccess) return 1;
  if (reset) {
    static const unsigned long long zero[9] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof_lds), zero, sizeof(zero)) != hipSuccess) return 1;
  }
  return 0;
}
#endif
