// gfd_light.hip -- the light destinations (2..kLightMax messages, self loop
// included; with dropout also the self-loop-only ones) of the PyG GATConv
// forward (/root/reference/src/models/gat.py:80) for F in 161..168: the bulk
// of a power-law graph's destinations.
//
// k_light_fs ("feature split"): the 16-destination tile's K = 8 heads x 168
// features is split into two halves by FEATURE (K half g = features
// 84 g .. 84 g + 83, all heads), and each half is one wave group's whole job:
// group g (waves 4 g .. 4 g + 3, one per SIMD) aggregates half-rows of its
// features for all 16 destinations into its own Z half-tile, and projects
// that half-tile against its half of W (W stationary in VGPRs / LDS exactly as
// in k_stream: wave = column tile ct x K half g).  The groups run one phase
// apart, so on every SIMD one wave is on the matrix pipe while its partner is
// on the VALU, instead of both waves of a SIMD doing MFMA (VALU idle) and then
// both aggregating (matrix pipe idle) as in k_stream:
//
//   phase 1 of tile v:  group 1  MFMA(v) over Z1(v)      | group 0  aggregate(v) -> Z0(v)
//   phase 2 of tile v:  group 0  MFMA(v) over Z0(v),      | group 1  aggregate(v+1) -> Z1(v+1)
//                       adds group 1's partial, stores out |
//
// One barrier per phase.  Each group issues the rows of the tile it
// aggregates next during its MFMA phase (one phase ahead).  Aggregation lane
// map: a wave owns 4 destinations in 2 pairs; lane = (pair member lane >> 5,
// feature 84 g + (lane & 31) + 32 q, q = 0..2), so one register holds a
// feature of BOTH destinations of a pair and a gathered half-row costs 3
// loads per pair; the softmax weights come from a per-wave LDS scratch with a
// per-half broadcast read (no v_readlane).
//
// LDS ownership:
//  * Z0: written by group 0 in phase 1 (tile v), read by group 0 in phase 2.
//  * Z1: written by group 1 in phase 2 (tile v + 1), read by group 1 in the
//    next phase 1.
//  * ring[g][t & 1][slot]: tile t's slot descriptors as issued by group g,
//    read when group g aggregates tile t (two phases later at most).
//  * rsc[t & 1][g][row]: the Z row scales of group g for tile t (written when
//    aggregated, read in that group's MFMA phase of the tile).
//  * rid[t & 1][row], red[ct]: group 0 writes rid in phase 1 and reads it in
//    phase 2; group 1 writes its scaled partial to red in phase 1, group 0
//    reads it in phase 2.
//  * P[wave]: the wave's own softmax weights (wave-private scratch).
//
// Measured (C4, MI355X, scripts/gpu_ab_parity.sh + scripts/prof_phases.py):
// light 8.2 ms against k_stream's 6.1 ms, parity green.  Per tile and wave:
// MFMA phase 5.8-6.4k cycles, aggregation 4.4-5.3k.  The premise fails on
// CDNA4's issue model: one wave alone issues vector instructions at half the
// rate two waves reach (4 vs 2 cycles per v_fma), and an MFMA holds the SIMD's
// vector issue for 8 of its 16 cycles, so an aggregating wave beside an MFMA
// wave runs its ~700 VALU instructions per phase at the single-wave rate --
// longer than the pair of waves aggregating together in k_stream.  Kept
// opt-in (-DGFD_LIGHT_FS=1) as the record of that experiment.
#include "gfd_fwd.h"

using namespace gfd;
using namespace gfd::fwd;

namespace {

constexpr int kFW = 8;              // waves per block
constexpr int kKH = 21;             // k-steps per K half (Fp = 168)
constexpr int kFH = 84;             // features per K half
constexpr int kZH = 8 * kFH + 8;    // Z half-row stride in halves (16-B pad)
constexpr int kLoL = 8;             // W_lo k-steps kept in LDS per wave
constexpr int kNR = kKH - kLoL;     // W_lo k-steps in VGPRs
constexpr int kNL = kLightMax;      // rows per light slot
static_assert(kNL <= 7, "message 7's logit lanes carry t_i");

#ifdef GFD_PROF
// Diagnostic build only: per-group s_memtime cycles summed over waves,
// [g][0] MFMA phase, [g][1] barrier after it, [g][2] aggregation phase,
// [g][3] barrier after it; [0][4] tiles; [g][5] the MFMA phase's slot heads,
// [g][6] its k-step loop.  Read by gfd_prof_fs_read.
__device__ unsigned long long g_prof_fs[2][8];  // [g][5..7]: MFMA phase split (heads, k-loop, rest)
#endif

// LDS layout (bytes)
constexpr size_t kOffZ = 0;                                            // [2 g][2 plane][16][kZH] f16
constexpr size_t kOffWL = kOffZ + sizeof(_Float16) * 2 * 2 * kTile * kZH;  // [8][kLoL][64] uint4
constexpr size_t kOffRed = kOffWL + sizeof(uint4) * kFW * kLoL * 64;   // [4 ct][64] f32x4
constexpr size_t kOffRing = kOffRed + sizeof(f32x4) * 4 * 64;          // [2 g][2 par][16] int4
constexpr size_t kOffRsc = kOffRing + sizeof(int4) * 2 * 2 * kTile;    // [2 par][2 g][16] float
constexpr size_t kOffRid = kOffRsc + sizeof(float) * 2 * 2 * kTile;    // [2 par][16] int
constexpr size_t kOffP = kOffRid + sizeof(int) * 2 * kTile;            // [8][2][64] float
constexpr size_t kOffCol = kOffP + sizeof(float) * kFW * 2 * 64;      // [3][64] bias, BN a, BN b
constexpr size_t kFsLds = kOffCol + sizeof(float) * 3 * 64;

// One slot record as loaded, in both wave halves (a pair's two records are
// merged by half): lanes 0..3 / 32..35 {row, e_begin, e_end, hub_rank},
// lanes 8..15 / 40..47 the sources of messages 0..7, other lanes a desc
// word (slots past num_dst: a clamped copy of the last one)
__device__ __forceinline__ int fs_rec(int64_t slot, int64_t num_dst,
                                      const int4* __restrict__ desc,
                                      const int32_t* __restrict__ cols8, int lane) {
  const int64_t sl = slot < num_dst ? slot : num_dst - 1;
  const int32_t* a = reinterpret_cast<const int32_t*>(desc + sl) + (lane & 3);
  const int32_t* b = cols8 + sl * 8 + (lane & 7);
  return *((lane & 24) == 8 ? b : a);
}

template <typename XT>
__device__ __forceinline__ float xload(const char* p) {
  if constexpr (XT::kBytes == 4) return *reinterpret_cast<const float*>(p);
  else return __uint_as_float(uint32_t(*reinterpret_cast<const uint16_t*>(p)) << 16);
}

template <typename XT>
__global__ void __launch_bounds__(kFW * 64, 2) k_light_fs(
    const void* __restrict__ x, int F, int64_t ldx, const int32_t* __restrict__ col,
    int64_t num_dst, int64_t dst_offset, const int4* __restrict__ desc,
    const int32_t* __restrict__ cols8, const float* __restrict__ st,
    const PackHeader* __restrict__ hdr, const uint4* __restrict__ wsh,
    const uint4* __restrict__ wsl, const float* __restrict__ bias, float slope, float dp,
    uint64_t seed, float* __restrict__ out, float* __restrict__ stats,
    const float* __restrict__ xmax, const int64_t* __restrict__ split, int to_end, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char ssm[];
  _Float16* Zb = reinterpret_cast<_Float16*>(ssm + kOffZ);
  uint4* WL = reinterpret_cast<uint4*>(ssm + kOffWL);
  f32x4* red = reinterpret_cast<f32x4*>(ssm + kOffRed);
  int4* ring = reinterpret_cast<int4*>(ssm + kOffRing);
  float* rsc = reinterpret_cast<float*>(ssm + kOffRsc);
  int* rid = reinterpret_cast<int*>(ssm + kOffRid);
  float* Pw = reinterpret_cast<float*>(ssm + kOffP);

  const int wave = wave_uniform(threadIdx.x >> 6);
  const int g = wave >> 2, ct = wave & 3;
  const int sb = 4 * ct;                      // this wave's 4 slots: sb .. sb + 3
  const int64_t G = gridDim.x;
  const int64_t t0 = blockIdx.x;
  const int64_t tb = (split[0] + kTile - 1) / kTile;
  const int64_t te = ((to_end ? num_dst : split[1]) + kTile - 1) / kTile;
  const int64_t nv = t0 < te - tb ? (te - tb - 1 - t0) / G + 1 : 0;
  const int64_t lim = to_end ? num_dst : split[1];
  int lane = opaque(threadIdx.x & 63);
  auto slot = [&](int64_t v, int r) { return (tb + t0 + v * G) * kTile + r; };
  _Float16* Zh = Zb + (g * 2 + 0) * kTile * kZH;   // this group's half-tile, hi plane
  _Float16* Zl = Zb + (g * 2 + 1) * kTile * kZH;   // lo plane
  float* P = Pw + wave * 2 * 64;

  // per-column epilogue constants (bias, BN affine) parked in LDS: no VGPRs
  // for the launch, and no global load behind the next tile's rows (which an
  // in-order vmcnt would make the store wait for)
  float* colc = reinterpret_cast<float*>(ssm + kOffCol);
  if (wave == 0) {
    colc[lane] = bias ? bias[lane] : 0.f;
    colc[64 + lane] = ep.ab ? ep.ab[lane] : 1.f;
    colc[128 + lane] = ep.ab ? ep.ab[C + lane] : 0.f;
  }
  const float wu = hdr->w_unscale;
  const int erg = global_scale_exp(xmax, dp);
  const float keep =  // 1 / (1 - p), kept scalar
      __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f)));
  const float sg = erg != 127 ? ldexpf(1.0f, erg) : 1.0f;
  const char* xb = static_cast<const char*>(x);
  const uint32_t pitch = uint32_t(ldx) * uint32_t(XT::kBytes);
  f16x8 bh[kKH], bl[kNR];
#pragma unroll
  for (int u = 0; u < kKH; ++u) {
    const int idx = ((g * kKH + u) * 4 + ct) * 64 + lane;
    const uint4 vh = wsh[idx], vl = wsl[idx];
    bh[u] = *reinterpret_cast<const f16x8*>(&vh);
    if (u < kNR) bl[u < kNR ? u : 0] = *reinterpret_cast<const f16x8*>(&vl);
    else WL[(wave * kLoL + (u - kNR)) * 64 + lane] = vl;
  }
  if (nv == 0) return;  // block-uniform: no barrier below is reached by anyone

  int rec[4];                    // records of the tile this wave issues next
  unsigned live = 0;             // bit i: slot i of that tile is < lim
  float sj[4];                   // its logits: s_j (message lane >> 3, head lane & 7),
                                 // t_i in lanes 56..63
  float xv[2][kNL][3];           // its half-rows: pair, message, feature chunk

  // ---- issue pieces: part 0 (descriptor, logits) of slot i; row k of pair pr ----
  // The records are merged per pair first (comb: lanes 0..31 the first
  // slot's record, 32..63 the second's), at the start of an issue, so every
  // piece reads registers that are already complete: the in-order vmcnt never
  // makes a piece wait for the loads the pieces before it issued.
  int comb[2];
  auto merge_recs = [&]() {
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      // a bit select, not ?: (which the compiler turns into a lane-indexed
      // read of rec: a scratch array)
      const int m = -((lane >> 5) & 1);
      comb[pr] = (rec[2 * pr + 1] & m) | (rec[2 * pr] & ~m);
    }
    // pinned here: sunk to its first use, the merge would wait (in-order
    // vmcnt) for the loads the pieces before that use issued
    asm volatile("" : "+v"(comb[0]), "+v"(comb[1]));
  };
  auto issue_head = [&](int i, int tpar) {
    const int c = comb[i >> 1], lb = 32 * (i & 1);
    const int h = lane & 7;
    const int row = __builtin_amdgcn_readlane(c, lb + 0);
    const int e0 = __builtin_amdgcn_readlane(c, lb + 1);
    const int e1 = __builtin_amdgcn_readlane(c, lb + 2);
    const int hw = __builtin_amdgcn_readlane(c, lb + 3);
    const int jm = __builtin_amdgcn_ds_bpermute((lb + 8 + (lane >> 3)) << 2, c);
    // one load: s_j of message lane >> 3 in lanes 0..47, the destination's
    // t_i in lanes 56..63 (message 7: past every light slot)
    const int64_t si = lane >= 56 ? (dst_offset + row) * 16 + H + h : int64_t(jm) * 16 + h;
    sj[i] = st[si];
    if (lane == 0) ring[(g * 2 + tpar) * kTile + sb + i] = make_int4((live >> i) & 1 ? row : -1, e0, e1, hw);
  };
  auto issue_row = [&](int pr, int k) {
    const int fl = lane & 31;
    // sources through scalar reads (a bpermute here would wait on lgkmcnt
    // for the MFMA loop's A-fragment reads in flight)
    const int ja = __builtin_amdgcn_readlane(comb[pr], 8 + k);
    const int jb = __builtin_amdgcn_readlane(comb[pr], 40 + k);
    const int j = (lane & 32) ? jb : ja;
    // no branch or select at the loads (a select right behind a load waits
    // for it): features past F read feature F - 1 of the same row, messages
    // past the slot's end the repeated last source; the aggregation masks both
    const char* rp = xb + uint64_t(uint32_t(j)) * pitch;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int f = kFH * g + fl + 32 * q;
      xv[pr][k][q] = xload<XT>(rp + uint32_t(f < F ? f : F - 1) * uint32_t(XT::kBytes));
    }
  };

  // softmax of slot i (descriptor dd): p (message lane >> 3, head lane & 7;
  // dropout applied; the global scale folded in when erg < 127), 1 / (sum + eps)
  auto softmax = [&](const int4 dd, int i, float& p, float& inv) {
    const int kk = lane >> 3;
    const int n = dd.z - dd.y;
    const float th = __int_as_float(
        __builtin_amdgcn_ds_bpermute((56 + (lane & 7)) << 2, __float_as_int(sj[i])));
    const float vv = leaky01(sj[i] + th, slope);
    // constants through opaque copies: rematerialised at each use instead of
    // hoisted into VGPRs for the launch (the kernel is at 256)
    const float m = max_xor8_16_32(kk < n ? vv : __int_as_float(opaque(int(0xff800000u))));
    const float pe = kk < n ? __expf(vv - m) : 0.f;
    const float l = sum_xor8_16_32(pe);
    if (__builtin_expect(stats != nullptr, 0) && g == 0 && lane < 8 && dd.x >= 0) {
      float* sr = stats + int64_t(dd.x) * 16 + lane;
      sr[0] = m;
      sr[8] = l;
    }
    inv = __builtin_amdgcn_rcpf(l + kSoftmaxEps);
    float pd = pe;
    if (__builtin_expect(dp > 0.f, 0))
      pd = dropout_keep(seed, uint32_t(dd.y + kk), uint32_t(lane & 7), dp)
               ? pe * keep : 0.f;
    p = erg != 127 ? pd * (inv * sg) : pd;
  };

  // aggregate pair pr of the tile in ring parity tpar into this group's Z half
  auto agg_pair = [&](int pr, int tpar) {
    const int ia = 2 * pr, ib = ia + 1;
    const int4 da = uni4(ring[(g * 2 + tpar) * kTile + sb + ia]);
    const int4 db = uni4(ring[(g * 2 + tpar) * kTile + sb + ib]);
    const int kmax = max(da.z - da.y, db.z - db.y);  // wave-uniform
    float pa, pb, ia_, ib_;
    softmax(da, ia, pa, ia_);
    softmax(db, ib, pb, ib_);
    P[lane] = pa;          // [member][message][head] = the logit lane order
    P[64 + lane] = pb;
    const int half = lane >> 5, fl = lane & 31;
    const float* Ph = P + 64 * half;
    f32x2 z[4][3];
#pragma unroll
    for (int g2 = 0; g2 < 4; ++g2)
#pragma unroll
      for (int q = 0; q < 3; ++q) z[g2][q] = f32x2{0.f, 0.f};
    // rows past this lane's slot's messages (and features past F) were loaded
    // from clamped addresses: replaced by 0 here (p is 0 there too, but 0 x
    // inf would be NaN)
    const int nown = half ? db.z - db.y : da.z - da.y;
    const bool f2ok = kFH * g + fl + 64 < F;
#pragma unroll
    for (int k = 0; k < kNL; ++k) {
      if (k < kmax) {
        float xk[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          const bool ok = (k == 0 || k < nown) && (q < 2 || f2ok);
          xk[q] = (k == 0 && q < 2) ? xv[pr][k][q] : (ok ? xv[pr][k][q] : 0.f);
        }
#pragma unroll
        for (int g2 = 0; g2 < 4; ++g2) {
          const f32x2 p2 = *reinterpret_cast<const f32x2*>(Ph + 8 * k + 2 * g2);
#pragma unroll
          for (int q = 0; q < 3; ++q)
            z[g2][q] = __builtin_elementwise_fma(p2, f32x2{xk[q], xk[q]}, z[g2][q]);
        }
      }
    }
    // this lane's destination (pair member half)
    const int4 dd = half ? db : da;
    const float inv = half ? ib_ : ia_;
    int er = erg;
    if (erg == 127) {  // per-row scale: max |z| over the half's 32 lanes (normalised)
      float zm = 0.f;
#pragma unroll
      for (int g2 = 0; g2 < 4; ++g2) {
        const float ia2 = __int_as_float(__builtin_amdgcn_ds_bpermute(
            ((lane & 32) + 2 * g2) << 2, __float_as_int(half ? ib_ : ia_)));
        const float ib2 = __int_as_float(__builtin_amdgcn_ds_bpermute(
            ((lane & 32) + 2 * g2 + 1) << 2, __float_as_int(half ? ib_ : ia_)));
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          z[g2][q] *= f32x2{ia2, ib2};
          zm = fmaxf(zm, fmaxf(fabsf(z[g2][q].x), fabsf(z[g2][q].y)));
        }
      }
      zm = fmaxf(zm, dpp_mov<0x121>(zm));  // row_ror:1 .. 8, then the other row
      zm = fmaxf(zm, dpp_mov<0x122>(zm));
      zm = fmaxf(zm, dpp_mov<0x124>(zm));
      zm = fmaxf(zm, dpp_mov<0x128>(zm));
      {
        auto pz = __builtin_amdgcn_permlane16_swap(__float_as_uint(zm), __float_as_uint(zm),
                                                   false, false);
        zm = fmaxf(__uint_as_float(pz[0]), __uint_as_float(pz[1]));
      }
      {  // scale_exp with the clamp bounds rematerialised
        int ex = 0;
        if (zm > 0.f) frexpf(zm, &ex);
        er = min(max(14 - ex, -opaque(100)), opaque(100));
      }
      const float rs = ldexpf(1.0f, er);
#pragma unroll
      for (int g2 = 0; g2 < 4; ++g2)
#pragma unroll
        for (int q = 0; q < 3; ++q) z[g2][q] *= f32x2{rs, rs};
    }
    (void)inv;
    const int r = sb + ia + half;  // tile row of this lane's destination
    _Float16* zh = Zh + r * kZH;
    _Float16* zl = Zl + r * kZH;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int fh = fl + 32 * q;
      if (fh < kFH) {
        union { f16x8 v; f16x2 p[4]; uint32_t u[4]; } a, b;
#pragma unroll
        for (int g2 = 0; g2 < 4; ++g2) {
          a.p[g2] = __builtin_convertvector(z[g2][q], f16x2);
          b.u[g2] = split_lo(z[g2][q], a.u[g2]);
        }
        *reinterpret_cast<f16x8*>(zh + 8 * fh) = a.v;
        *reinterpret_cast<f16x8*>(zl + 8 * fh) = b.v;
      }
    }
    if (fl == 0) {
      rsc[(tpar * 2 + g) * kTile + r] = ldexpf(1.0f, -er);
      if (g == 0) rid[tpar * kTile + r] = dd.x;
    }
  };

#ifdef GFD_PROF
  unsigned long long pq[2] = {0ull, 0ull};
#endif
  // MFMA of this group's half-tile (tile parity tpar) with the issue of the
  // next tile (records in rec, ring parity npar) spread over the k-steps when
  // issue_next; returns the unscaled 16 x 16 partial of column tile ct
  auto mfma_phase = [&](bool issue_next, int npar) -> f32x4 {
    const int aoff = (lane & 15) * kZH + 8 * (lane >> 4);
    const _Float16* ah = Zh + aoff;
    const _Float16* al = Zl + aoff;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    f16x8 phi = *reinterpret_cast<const f16x8*>(ah), plo = *reinterpret_cast<const f16x8*>(al);
    f16x8 pwl = phi;
#ifdef GFD_PROF
    const unsigned long long tq0 = __builtin_amdgcn_s_memtime();
#endif
    if (issue_next) {  // the 4 slot heads first: their bpermutes share one LDS wait
      merge_recs();
#pragma unroll
      for (int i = 0; i < 4; ++i) issue_head(i, npar);
    }
#ifdef GFD_PROF
    const unsigned long long tq1 = __builtin_amdgcn_s_memtime();
#endif
    constexpr int NP = 2 * kNL;  // row pieces: 2 pairs x kNL rows
#pragma unroll
    for (int u = 0; u < kKH; ++u) {
      if (issue_next) {
#pragma unroll
        for (int i = 0; i < NP; ++i)
          if (u == 1 + i * (kKH - 2) / NP) issue_row(i / kNL, i % kNL);
      }
      const f16x8 ahi = phi, alo = plo;
      if (u + 1 < kKH) {
        phi = *reinterpret_cast<const f16x8*>(ah + 32 * (u + 1));
        plo = *reinterpret_cast<const f16x8*>(al + 32 * (u + 1));
      }
      const f16x8 blo = u < kNR ? bl[u < kNR ? u : 0] : pwl;
      if (u + 1 >= kNR && u + 1 < kKH) {  // LDS-resident W_lo one k-step ahead
        const uint4 w = WL[(wave * kLoL + (u + 1 - kNR)) * 64 + lane];
        pwl = *reinterpret_cast<const f16x8*>(&w);
      }
      f32x4& acc = (u & 1) ? acc1 : acc0;
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bh[u], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, blo, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bh[u], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
#ifdef GFD_PROF
    const f32x4 r = acc0 + acc1;
    asm volatile("" : "+v"(r));
    const unsigned long long tq2 = __builtin_amdgcn_s_memtime();
    pq[0] += tq1 - tq0;
    pq[1] += tq2 - tq1;
    return r;
#else
    return acc0 + acc1;
#endif
  };
  auto load_recs = [&](int64_t v) {
    live = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      rec[i] = fs_rec(slot(v, sb + i), num_dst, desc, cols8, lane);
      live |= unsigned(slot(v, sb + i) < lim) << i;
    }
  };
  auto issue_all = [&](int tpar) {
    merge_recs();
#pragma unroll
    for (int i = 0; i < 4; ++i) issue_head(i, tpar);
#pragma unroll
    for (int pr = 0; pr < 2; ++pr)
#pragma unroll
      for (int k = 0; k < kNL; ++k) issue_row(pr, k);
  };

  // ---- prologue: tile 0 issued by both groups; group 1 aggregates it ----
  load_recs(0);
  issue_all(0);
  load_recs(1);
  if (g == 1) {
    agg_pair(0, 0);
    agg_pair(1, 0);
  }
  __syncthreads();

#ifdef GFD_PROF
  unsigned long long pc[4] = {0ull, 0ull, 0ull, 0ull};
#define GFD_TS(t) const unsigned long long t = __builtin_amdgcn_s_memtime()
#else
#define GFD_TS(t)
#endif
  // One loop per group (g is wave-uniform; both loops pass the same barriers
  // in the same order): with one loop, the compiler's vmcnt model merges the
  // groups' paths at the loop head and makes each group wait for the other
  // group's rows before reusing their registers.
  if (g == 1) {
    for (int64_t v = 0; v < nv; ++v) {
      lane = opaque(threadIdx.x & 63);
      const int par = int(v & 1), pn = par ^ 1;
      const bool more = v + 1 < nv;
      GFD_TS(ts0);
      // ---- phase 1: project tile v (group 0 aggregates it) ----
      const f32x4 acc = mfma_phase(more, pn);
      if (more) load_recs(v + 2);
      f32x4 sc;
#pragma unroll
      for (int q = 0; q < 4; ++q) sc[q] = acc[q] * rsc[(par * 2 + 1) * kTile + (lane >> 4) * 4 + q];
      red[ct * 64 + lane] = sc;
      GFD_TS(ts1);
      __syncthreads();
      GFD_TS(ts2);
      // ---- phase 2: aggregate tile v + 1 (group 0 projects and stores v) ----
      if (more) {
        agg_pair(0, pn);
        agg_pair(1, pn);
      }
      GFD_TS(ts3);
      __syncthreads();
#ifdef GFD_PROF
      GFD_TS(ts4);
      pc[0] += ts1 - ts0;
      pc[1] += ts2 - ts1;
      pc[2] += ts3 - ts2;
      pc[3] += ts4 - ts3;
#endif
    }
  } else {
    for (int64_t v = 0; v < nv; ++v) {
      lane = opaque(threadIdx.x & 63);
      const int par = int(v & 1), pn = par ^ 1;
      const bool more = v + 1 < nv;
      GFD_TS(ts0);
      // ---- phase 1: aggregate tile v ----
      agg_pair(0, par);
      agg_pair(1, par);
      GFD_TS(ts1);
      __syncthreads();
      GFD_TS(ts2);
      // ---- phase 2: project tile v, add group 1's partial, store ----
      const f32x4 acc = mfma_phase(more, pn);
      if (more) load_recs(v + 2);
      const f32x4 other = red[ct * 64 + lane];
      const int n = ct * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = (lane >> 4) * 4 + q;
        const int ri = rid[par * kTile + r];
        const float sum = fmaf(acc[q], rsc[(par * 2 + 0) * kTile + r], other[q]);
        if (ri >= 0) {
          float y = fmaf(sum, wu, colc[n]);
          if (ep.ab) {  // gat.py:82-91 eval body: BN affine, relu, residual
            y = fmaf(y, colc[64 + n], colc[128 + n]);
            if (ep.relu) y = fmaxf(y, 0.f);
            if (ep.res) y += ep.res[int64_t(ri) * ep.ldr + n];
          }
          out[int64_t(ri) * C + n] = y;
        }
      }
      GFD_TS(ts3);
      __syncthreads();
#ifdef GFD_PROF
      GFD_TS(ts4);
      pc[2] += ts1 - ts0;
      pc[3] += ts2 - ts1;
      pc[0] += ts3 - ts2;
      pc[1] += ts4 - ts3;
#endif
    }
  }
#ifdef GFD_PROF
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) atomicAdd(&g_prof_fs[g][i], pc[i]);
    atomicAdd(&g_prof_fs[g][5], pq[0]);
    atomicAdd(&g_prof_fs[g][6], pq[1]);
    if (wave == 0) atomicAdd(&g_prof_fs[0][4], (unsigned long long)nv);
  }
#endif
#undef GFD_TS
}

}  // namespace

namespace gfd {
namespace fwd {

bool light_fs_supported(const AggArgs& a, const PackLayout& L) {
  return L.Fp == 168 && L.KS / 2 == kKH && a.plan.slot_desc && a.plan.slot_cols &&
         a.plan.class_split && a.slope >= 0.f && a.slope <= 1.f;
}

gfd_status launch_light_fs(const AggArgs& a, const PackLayout& L, bool to_end,
                           hipStream_t stream) {
  if (!light_fs_supported(a, L)) return GFD_ERR_UNSUPPORTED;
  const bool bf = a.xdt == GFD_DTYPE_BF16;
  const void* kern = bf ? reinterpret_cast<const void*>(&k_light_fs<XBF16>)
                        : reinterpret_cast<const void*>(&k_light_fs<XF32>);
  if (!ensure_lds(kern, kFsLds)) return GFD_ERR_HIP;
  const int64_t tiles = (a.num_dst + kTile - 1) / kTile;
  int64_t grid = cu_count();
  if (grid > tiles) grid = tiles;
  const gfd_plan& p = a.plan;
#define GFD_FS_ARGS                                                                           \
  a.x, a.F, a.ldx, a.col, a.num_dst, a.dst_offset, reinterpret_cast<const int4*>(p.slot_desc), \
      p.slot_cols, a.st, reinterpret_cast<const PackHeader*>(a.packed + L.hdr_off),           \
      reinterpret_cast<const uint4*>(a.packed + L.wsh_off),                                   \
      reinterpret_cast<const uint4*>(a.packed + L.wsl_off), a.bias, a.slope, a.dp, a.seed,     \
      a.out, a.stats, a.xmax, p.class_split, to_end ? 1 : 0, a.ep
  if (bf)
    k_light_fs<XBF16><<<int(grid), kFW * 64, kFsLds, stream>>>(GFD_FS_ARGS);
  else
    k_light_fs<XF32><<<int(grid), kFW * 64, kFsLds, stream>>>(GFD_FS_ARGS);
#undef GFD_FS_ARGS
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

}  // namespace fwd
}  // namespace gfd

#ifdef GFD_PROF
extern "C" int gfd_prof_fs_read(unsigned long long* out16, int reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_prof_fs), sizeof(g_prof_fs)) != hipSuccess) return 1;
  if (reset) {
    static const unsigned long long zero[2][8] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof_fs), zero, sizeof(zero)) != hipSuccess) return 1;
  }
  return 0;
}
#endif
