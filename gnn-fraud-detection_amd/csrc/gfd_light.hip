// gfd_light.hip -- the light class (destinations of 2 .. kLightMax messages,
// self loop included) for fp32 and bf16 rows, 64 + Fp/2 <= F <= 168: the PyG
// GATConv.forward softmax-aggregate-project of /root/reference/src/models/gat.py:80
// (and tgn.py:94) as a PAIRED-PHASE tile kernel.
//
// Why: k_stream<LIGHT> runs all 8 waves of a block
// through the same two phases per 16-row tile -- MFMA, barrier, aggregation,
// barrier -- so the two waves of a SIMD (waves w and w + 4) are always in the
// same phase and matrix and vector work never execute side by side.
//
// Here the two K halves of the projection are ALSO the two feature halves of
// the aggregation: K position p = 8 f + h, so K half g holds features
// [g FH, g FH + FH) (FH = Fp / 2) of all 8 heads.  Wave group g (waves 4g ..
// 4g + 3, one per SIMD, column tile ct = wave & 3) aggregates ITS feature half
// of all 16 rows of a tile into its own Z half and runs the MFMAs of that K
// half, so the groups share nothing but the partial outputs and the softmax
// weights, and group 1 runs half a tile behind group 0:
//
//   step 2v - 1:  group 0 aggregates tile v        group 1 MFMA, tile v - 1
//   step 2v    :  group 0 MFMA, tile v             group 1 aggregates tile v
//   (one block barrier per step)
//
// so on every SIMD one wave issues MFMAs while its partner issues the
// aggregation's VALU work.  Per step each LDS region has one writer phase and
// one reader phase, separated by the step barrier:
//  * Z[g] (16 rows x 4 Fp halves, f16 hi / lo planes): written by group g in
//    its aggregation step, read by group g's MFMAs in its next step.
//  * P[16 slots][48] (normalised message weights, message k, head h at 8 k + h):
//    slots 4 ct, 4 ct + 1 of a tile are written by wave (0, ct) when it
//    aggregates the tile, slots 4 ct + 2, 4 ct + 3 by wave (1, ct) one step
//    BEFORE group 0 aggregates it; each slot is read by waves (0, ct) and
//    (1, ct) only, and rewritten for the next tile only after both read it
//    (group 1 aggregates first, then computes the next tile's weights).
//  * red[4 ct][64] (group 0's f32x4 partial outputs): written at the end of
//    group 0's MFMA step, read at the end of group 1's (the next step).
//  * rid[2 parity][16], rsc[2 g][2 parity][16]: destination rows and (when x
//    is too large for one launch-wide scale) per-row per-half scales, written
//    with the weights / the Z half, read by the MFMA steps of that tile.
//
// Aggregation layout: each wave aggregates slots 4 ct .. 4 ct + 3 in two
// passes of two slots (lanes 0..31: slot 4 ct + 2 pass, lanes 32..63: the
// next); lane li = lane & 31 holds local features li, 32 + li, 64 + li of
// its slot, all 8 heads (z: 12 f32x2).  Rows are gathered with 64-bit lane
// addresses (structured buffer loads would range-check rows and features for
// free, but a descriptor reaches only 4 GiB: scripts/sbuf_probe.hip); rows
// past a slot's messages and features past F are masked loads reading 0.  A
// pass's rows for the NEXT tile are issued right after the pass consumed
// this tile's, so a row has two steps to arrive.
//
// Results are bit-identical to k_stream<LIGHT> while one launch-wide scale
// covers x (max |x| <= 2^20): same weights, same FMA order, same f16 split,
// same MFMA k-step order and partial-sum order.
#include "gfd_fwd.h"

using namespace gfd;
using namespace gfd::fwd;

namespace {

constexpr int kLW = 8;                 // waves per block: 2 groups x 4 column tiles
constexpr int kLR = kLightMax;         // rows (messages) per slot
constexpr int kLZPad = 16;             // Z row pad (halves): conflict-free A-fragment reads
// bf16 rows (config C5) through this kernel as well
#ifndef GFD_LIGHT_PAIR_BF16
#define GFD_LIGHT_PAIR_BF16 1
#endif


struct Logits {  // a softmax owner's two slots: s_j of message lane >> 3, t_i (head lane & 7)
  float sv[2];
  float th[2];
};

// max over the 32 lanes of each half of the wave
__device__ __forceinline__ float max_half32(float v) {
  v = fmaxf(v, dpp_mov<0x121>(v));  // row_ror:1
  v = fmaxf(v, dpp_mov<0x122>(v));  // row_ror:2
  v = fmaxf(v, dpp_mov<0x124>(v));  // row_ror:4
  v = fmaxf(v, dpp_mov<0x128>(v));  // row_ror:8
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
}

// acc += ahi.bh + ahi.bl + alo.bh (the 3-term split) IN PLACE.  Inline asm,
// because with the builtins the register allocator gave these chains
// destination quads partially overlapping their srcC quads (v[2:5] <- ..,
// v[0:3]) in this kernel -- 168 such MFMAs, and rows of the tile came out
// wrong at random (round 6; the k_stream listing has none).  The first
// k-step of a chain takes srcC = 0 (no vector write of the accumulator ahead
// of it); a chain's own back-to-back MFMAs on one quad need no wait states.
__device__ __forceinline__ void mfma3(f32x4& acc, f16x8 ahi, f16x8 alo, f16x8 bh, f16x8 bl,
                                      bool first) {
  if (first) {
    asm volatile(
        "v_mfma_f32_16x16x32_f16 %0, %1, %3, 0\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %2, %3, %0"
        : "=&v"(acc)
        : "v"(ahi), "v"(alo), "v"(bh), "v"(bl));
  } else {
    asm volatile(
        "v_mfma_f32_16x16x32_f16 %0, %1, %3, %0\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %1, %4, %0\n\t"
        "v_mfma_f32_16x16x32_f16 %0, %2, %3, %0"
        : "+v"(acc)
        : "v"(ahi), "v"(alo), "v"(bh), "v"(bl));
  }
}

#ifdef GFD_LP_PROF
// Diagnostic build only (GFD_BUILD_VARIANT=lpprof GFD_EXTRA_FLAGS=-DGFD_LP_PROF):
// per-wave s_memtime cycles summed over waves, [group][i]: 0 aggregation-step
// work, 1 of it waiting for the step's rows, 2 MFMA-step work, 3 barrier after
// an aggregation step, 4 barrier after an MFMA step, 5 aggregation steps,
// 6 MFMA steps (scripts/prof_light_pair.py)
__device__ unsigned long long g_lprof[2][16];
#endif

size_t light_pair_smem(int Fp, int lo) {
  const int ZSH = 4 * Fp + kLZPad;
  return sizeof(_Float16) * 4 * kTile * ZSH + sizeof(uint4) * kLW * lo * 64 +
         sizeof(float) * kTile * 64 + sizeof(f32x4) * 4 * 64 + sizeof(int) * 2 * kTile +
         sizeof(float) * 4 * kTile;
}

template <typename XT, int KHM, int LO, bool EXACT, bool EPI>
__global__ void __launch_bounds__(kLW * 64, 2) k_light_pair(
    const void* __restrict__ x, int64_t N, int F, int Fp, int64_t ldx, int64_t num_dst,
    const int4* __restrict__ desc, const int32_t* __restrict__ cols8,
    const float* __restrict__ s, int lds, const float* __restrict__ t, int ldt,
    const PackHeader* __restrict__ hdr, const uint4* __restrict__ wsh,
    const uint4* __restrict__ wsl, const float* __restrict__ bias, float slope, float dp,
    uint64_t seed, float* __restrict__ out, float* __restrict__ stats,
    const float* __restrict__ xmax, const int64_t* __restrict__ split, int to_end, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char ssm[];
  const int FH = Fp / 2;
  const int ZSH = 4 * Fp + kLZPad;                                // halves per Z row
  _Float16* Zh = reinterpret_cast<_Float16*>(ssm);                // [2 g][16][ZSH]
  _Float16* Zl = Zh + 2 * kTile * ZSH;                            // [2 g][16][ZSH]
  uint4* WL = reinterpret_cast<uint4*>(Zl + 2 * kTile * ZSH);     // [8 waves][LO][64]
  float* P = reinterpret_cast<float*>(WL + kLW * LO * 64);        // [16][48]
#ifdef GFD_LP_DIAG_P64
  f32x4* red = reinterpret_cast<f32x4*>(P + kTile * 64);          // [4 ct][64]
#else
  f32x4* red = reinterpret_cast<f32x4*>(P + kTile * 48);          // [4 ct][64]
#endif
  int* rid = reinterpret_cast<int*>(red + 4 * 64);                // [2 par][16]
  float* rsc = reinterpret_cast<float*>(rid + 2 * kTile);         // [2 g][2 par][16]

  const int wave = wave_uniform(threadIdx.x >> 6);
  const int g = wave >> 2, ct = wave & 3;
  // lane is re-derived opaquely every step: addresses built from it are then
  // recomputed where used instead of being hoisted out of the persistent loop
  // and pinned in VGPRs (which spilled 48 of them)
  int lane = opaque(threadIdx.x & 63);
  const int64_t G = gridDim.x;
  const int64_t t0 = blockIdx.x;
  const int64_t tb = (split[0] + kTile - 1) / kTile;
  const int64_t te = ((to_end ? num_dst : split[1]) + kTile - 1) / kTile;
  const int64_t nv = t0 < te - tb ? (te - tb - 1 - t0) / G + 1 : 0;
  // not to the end: the slots of the last tile past split[1] are lone rows
  // another kernel writes -- taken as empty here
  const int64_t lim = to_end ? num_dst : split[1];
  auto slot = [&](int64_t v, int r) { return (tb + t0 + v * G) * kTile + r; };

  // Z positions no lane writes (features F .. Fp - 1 of half 1) must read 0
  for (int i = threadIdx.x; i < 4 * kTile * ZSH / 8; i += kLW * 64)
    reinterpret_cast<uint4*>(Zh)[i] = make_uint4(0u, 0u, 0u, 0u);

  // kernel-lifetime constants first
  const float bcol = bias ? bias[ct * 16 + (lane & 15)] : 0.f;
  const float wu = hdr->w_unscale;
  const int erg = global_scale_exp(xmax, dp);
  const float ergs = erg != 127 ? ldexpf(1.0f, erg) : 1.0f;   // folded into the weights
  const float rs_glob = erg != 127 ? ldexpf(1.0f, -erg) * wu : 0.f;
  const int KH = EXACT ? KHM : Fp / 8;
  constexpr int NR = KHM - LO;
  f16x8 bh[KHM], bl[NR > 0 ? NR : 1];
#pragma unroll
  for (int u = 0; u < KHM; ++u) {
    uint4 vh = make_uint4(0, 0, 0, 0), vl = vh;
    if (u < KH) {
      const int idx = ((g * KH + u) * 4 + ct) * 64 + lane;
      vh = wsh[idx];
      vl = wsl[idx];
    }
    bh[u] = *reinterpret_cast<const f16x8*>(&vh);
    if (u < NR) bl[u < NR ? u : 0] = *reinterpret_cast<const f16x8*>(&vl);
    else WL[(wave * LO + (u - NR)) * 64 + lane] = vl;
  }
  if (nv == 0) return;  // uniform per block: no barrier below is reached by anyone

  const int64_t pitch = ldx * XT::kBytes;      // row pitch in bytes (< 2^32: host check)
  const int fg = g * FH;                       // first feature of this half

  // slot records, one VGPR per tile: lanes 8 q + k = source k of slot 4 ct + q;
  // lanes 32 + 4 q + f = field f of its descriptor {row, e_begin, e_end, hub},
  // e_end = -1 for a slot past the class (empty)
  auto rec_load = [&](int64_t v) -> int {
    const int q = lane < 32 ? (lane >> 3) : min((lane - 32) >> 2, 3);
    const int64_t sl0 = slot(v, 4 * ct + q);
    const int64_t sl = sl0 < num_dst ? sl0 : num_dst - 1;
    const int32_t* a = lane < 32 ? cols8 + sl * 8 + (lane & 7)
                                 : reinterpret_cast<const int32_t*>(desc + sl) + (lane & 3);
    const int val = *a;
    return (lane >= 32 && (lane & 3) == 2 && sl0 >= lim) ? -1 : val;
  };
  auto n_of = [&](int Cr, int64_t, int q) -> int {  // messages of slot 4 ct + q (0: empty)
    const int e0 = __builtin_amdgcn_readlane(Cr, 33 + 4 * q);
    const int e1 = __builtin_amdgcn_readlane(Cr, 34 + 4 * q);
    return e1 < 0 ? 0 : e1 - e0;
  };

#ifdef GFD_LP_PROF
  unsigned long long pw = 0ull;  // cycles waiting for rows (aggregation)
  unsigned long long pv[4] = {0ull, 0ull, 0ull, 0ull};  // softmax, aggregate, rows issue, logits
#endif
  float xr[2][kLR][3];  // a pass's rows for the next tile (lane <-> its slot's three features)
  Logits lg;            // logits of the wave's next softmax
  int Cq[4];            // records of tiles v .. v + 3 (of the wave's next aggregation v)

  // ---- pieces ----
  auto rows_issue = [&](int Cn, int64_t vn, int p) {
    if (vn >= nv) return;
    const int hf = lane >> 5, li = lane & 31;
    constexpr int eb = XT::kBytes;
    const bool v2 = 64 + li < FH && fg + 64 + li < F;   // third feature of the lane exists
    const int q = 2 * p + hf;
    const int na = n_of(Cn, vn, 2 * p), nb = n_of(Cn, vn, 2 * p + 1);
    const int R = max(na, nb), nmin = min(na, nb);
    const int nl = hf ? nb : na;
    const char* xl = reinterpret_cast<const char*>(x) + (fg + li) * eb;
    // all sources of the pass first (one LDS wait), then the row loads
    int jr[kLR];
#pragma unroll
    for (int k = 0; k < kLR; ++k)
      if (k < R) jr[k] = __builtin_amdgcn_ds_bpermute((8 * q + k) << 2, Cn);
#pragma unroll
    for (int k = 0; k < kLR; ++k) {
      if (k < R) {
        // the lane's first feature of row j (64-bit: x exceeds the 4 GiB a
        // buffer descriptor reaches -- scripts/sbuf_probe.hip)
        const typename XT::T* ra = reinterpret_cast<const typename XT::T*>(
            xl + uint64_t(uint32_t(jr[k])) * uint64_t(uint32_t(pitch)));
        float x0 = 0.f, x1 = 0.f, x2 = 0.f;
        if (k < nmin || k < nl) {  // (uniform, or this half's slot has message k)
          x0 = xcvt(ra[0]);
          x1 = xcvt(ra[32]);
          if (v2) x2 = xcvt(ra[64]);
        }
        xr[p][k][0] = x0;
        xr[p][k][1] = x1;
        xr[p][k][2] = x2;
      }
    }
  };
  auto logits_issue = [&](int Cr, int64_t vt) {  // the wave's softmax slots 2 g, 2 g + 1 of tile vt
    if (vt >= nv) return;
    const int h = lane & 7;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int q = 2 * g + e;
      const int j = __builtin_amdgcn_ds_bpermute((8 * q + (lane >> 3)) << 2, Cr);
      const int row = __builtin_amdgcn_readlane(Cr, 32 + 4 * q);
      lg.sv[e] = lrow(s, j, lds)[h];
      lg.th[e] = lrow(t, row, ldt)[h];
    }
  };
  // normalised message weights of slots 4 ct + 2 g, + 1 of tile v -> P, rid
  auto softmax = [&](int Cr, int64_t v) {
    const int par = int(v & 1);
    const int kk = lane >> 3, h = lane & 7;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int q = 2 * g + e;
      const int r = 4 * ct + q;
      const int row = __builtin_amdgcn_readlane(Cr, 32 + 4 * q);
      const int e0 = __builtin_amdgcn_readlane(Cr, 33 + 4 * q);
      const int n = n_of(Cr, v, q);
      const float val = leaky01(lg.sv[e] + lg.th[e], slope);
      const float mx = max_xor8_16_32(kk < n ? val : -INFINITY);
      const float pe = kk < n ? __expf(val - mx) : 0.f;
      const float l = sum_xor8_16_32(pe);
      if (__builtin_expect(stats != nullptr, 0) && n > 0 && lane < 8) {  // training only
        float* sr = stats + int64_t(row) * 16 + lane;
        sr[0] = mx;
        sr[8] = l;
      }
      const float inv = __builtin_amdgcn_rcpf(l + kSoftmaxEps);
      float pd = pe;
      if (__builtin_expect(dp > 0.f, 0))  // kernel-uniform
        pd = dropout_keep(seed, uint32_t(e0 + kk), uint32_t(h), dp) ? pe * (1.0f / (1.0f - dp)) : 0.f;
      const float ps = pd * (inv * ergs);
#ifdef GFD_LP_DIAG_P64
      P[r * 64 + lane] = ps;
      rid[par * kTile + r] = n > 0 ? row : -1;
#else
      if (lane < 48) P[r * 48 + lane] = ps;
      if (lane == 0) rid[par * kTile + r] = n > 0 ? row : -1;
#endif
    }
  };
  // the wave's feature half of slots 4 ct + 2 p (lanes 0..31) and + 1 (32..63)
  // of tile v, from the rows in xr[p] and the weights in P -> Z[g]
  auto aggregate = [&](int Cr, int64_t v, int p) {
    const int par = int(v & 1);
    const int hf = lane >> 5, li = lane & 31;
    const bool w2 = 64 + li < FH;                // the lane's third feature is in this half
    const int r = 4 * ct + 2 * p + hf;
    const int R = max(max(n_of(Cr, v, 2 * p), n_of(Cr, v, 2 * p + 1)), 1);
#ifdef GFD_LP_DIAG_P64
    const float* pr = P + r * 64;
#else
    const float* pr = P + r * 48;
#endif
#ifdef GFD_LP_DIAG_WAIT
    __builtin_amdgcn_s_waitcnt(0);
#endif
#ifdef GFD_LP_PROF
    {
      const unsigned long long w0 = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_s_waitcnt(0);
      pw += __builtin_amdgcn_s_memtime() - w0;
    }
#endif
    // plain FMAs, not v_pk_fma_f32: beside the partner wave's MFMAs a packed
    // FMA costs far more than two plain ones (MI355X_MICROARCH.md, fillers
    // beside MFMAs).  Same arithmetic per element.  The next round's weights
    // are read one round ahead.
    float z[H][3];
    f32x4 w0 = *reinterpret_cast<const f32x4*>(pr), w1 = *reinterpret_cast<const f32x4*>(pr + 4);
#pragma unroll
    for (int k = 0; k < kLR; ++k) {
      if (k == 0 || k < R) {
        const float pk[H] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        if (k + 1 < kLR && k + 1 < R) {
          w0 = *reinterpret_cast<const f32x4*>(pr + 8 * (k + 1));
          w1 = *reinterpret_cast<const f32x4*>(pr + 8 * (k + 1) + 4);
        }
#pragma unroll
        for (int h = 0; h < H; ++h)
#pragma unroll
          for (int m = 0; m < 3; ++m)
            z[h][m] = k == 0 ? pk[h] * xr[p][k][m] : fmaf(pk[h], xr[p][k][m], z[h][m]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if (erg == 127) {  // kernel-uniform: a scale for this row's half from its own max |z|
      float zm = 0.f;
#pragma unroll
      for (int h = 0; h < H; ++h)
#pragma unroll
        for (int m = 0; m < 3; ++m) zm = fmaxf(zm, fabsf(z[h][m]));
      const int er = scale_exp(max_half32(zm));
      const float sc = ldexpf(1.0f, er);
#pragma unroll
      for (int h = 0; h < H; ++h)
#pragma unroll
        for (int m = 0; m < 3; ++m) z[h][m] *= sc;
      if (li == 0) rsc[(g * 2 + par) * kTile + r] = ldexpf(1.0f, -er);
    }
    _Float16* zh = Zh + (g * kTile + r) * ZSH;
    _Float16* zl = Zl + (g * kTile + r) * ZSH;
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      union { f16x8 v; f16x2 p[4]; uint32_t u[4]; } a, b;
#pragma unroll
      for (int hp = 0; hp < 4; ++hp) {
        const f32x2 zz = f32x2{z[2 * hp][m], z[2 * hp + 1][m]};
        a.p[hp] = __builtin_convertvector(zz, f16x2);
        b.u[hp] = split_lo(zz, a.u[hp]);
      }
      if (m < 2 || w2) {
        const int f = 32 * m + li;
        *reinterpret_cast<f16x8*>(zh + 8 * f) = a.v;
        *reinterpret_cast<f16x8*>(zl + 8 * f) = b.v;
      }
    }
  };
  // MFMAs of tile v over this group's K half; group 0 parks its partial
  // outputs, group 1 adds them and stores the rows
  auto mfma = [&](int64_t v) {
    const int par = int(v & 1);
    const int aoff = (g * kTile + (lane & 15)) * ZSH + 8 * (lane >> 4);
    const _Float16* ah = Zh + aoff;
    const _Float16* al = Zl + aoff;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    f16x8 phi = *reinterpret_cast<const f16x8*>(ah);
    f16x8 plo = *reinterpret_cast<const f16x8*>(al);
    f16x8 pwl;
    if (NR == 0) {
      const uint4 w = WL[(wave * LO) * 64 + lane];
      pwl = *reinterpret_cast<const f16x8*>(&w);
    }
#pragma unroll
    for (int u = 0; u < KHM; ++u) {
      if (u < KH) {
        const f16x8 ahi = phi, alo = plo;
        const f16x8 blo = u < NR ? bl[u < NR ? u : 0] : pwl;
        if (u + 1 < KH) {
          phi = *reinterpret_cast<const f16x8*>(ah + 32 * (u + 1));
          plo = *reinterpret_cast<const f16x8*>(al + 32 * (u + 1));
          if (u + 1 >= NR) {
            const uint4 w = WL[(wave * LO + (u + 1 - NR)) * 64 + lane];
            pwl = *reinterpret_cast<const f16x8*>(&w);
          }
        }
        f32x4& acc = (u & 1) ? acc1 : acc0;
        mfma3(acc, ahi, alo, bh[u], blo, u < 2);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // the MFMA results are read by vector instructions next: the inline-asm
    // chains carry no hazard information for the compiler, so wait out the
    // last MFMA's passes here (16 wait states)
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    acc0 += acc1;
    if (g == 0) {
      if (erg == 127) {
#pragma unroll
        for (int q = 0; q < 4; ++q) acc0[q] *= rsc[par * kTile + (lane >> 4) * 4 + q];
      }
      red[ct * 64 + lane] = acc0;
    } else {
      const f32x4 pr = red[ct * 64 + lane];
      const int n = ct * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = (lane >> 4) * 4 + q;
        const int ri = rid[par * kTile + r];
        const float vs = erg != 127 ? (acc0[q] + pr[q]) * rs_glob
                                    : (pr[q] + acc0[q] * rsc[(2 + par) * kTile + r]) * wu;
        if (ri >= 0) out[int64_t(ri) * ep.ldo + n] = epi_store_value<EPI>(vs, bcol, n, ri, ep);
      }
    }
  };
  // a wave's aggregation step: group 0 -- weights of its slots of tile v, then
  // both passes; group 1 -- both passes of tile v, then the weights of its
  // slots of tile v + 1 (P holds one tile: each slot's weights are read by
  // waves (0, ct) and (1, ct) before group 1 replaces them)
#ifdef GFD_LP_PROF
#define GFD_LP_STAMP(i)                                          \
  do {                                                           \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();  \
    pv[i] += _t - tv;                                            \
    tv = _t;                                                     \
  } while (0)
#else
#define GFD_LP_STAMP(i) do {} while (0)
#endif
  auto valu_step = [&](int64_t v) {
#ifdef GFD_LP_PROF
    unsigned long long tv = __builtin_amdgcn_s_memtime();
#endif
    Cq[3] = rec_load(v + 3);
    if (g == 0) {
      softmax(Cq[0], v);
      // this wave reads back the weights it just wrote: the hardware runs a
      // wave's LDS operations in order, but the compiler must not hoist the
      // reads above the writes (it did: stale weights in slot 4 ct + 1)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    GFD_LP_STAMP(0);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if (v >= 0) aggregate(Cq[0], v, p);
      GFD_LP_STAMP(1);
      rows_issue(Cq[1], v + 1, p);
      GFD_LP_STAMP(2);
    }
    if (g == 1 && v + 1 < nv) softmax(Cq[1], v + 1);
    GFD_LP_STAMP(0);
    logits_issue(g == 0 ? Cq[1] : Cq[2], v + 1 + g);
    GFD_LP_STAMP(3);
  };
  auto rotate = [&]() {
    Cq[0] = Cq[1];
    Cq[1] = Cq[2];
    Cq[2] = Cq[3];
  };

  // ---- prologue: records, the first weights' logits, group 0's first rows ----
  if (g == 0) {
    Cq[0] = rec_load(0);
    Cq[1] = rec_load(1);
    Cq[2] = rec_load(2);
    logits_issue(Cq[0], 0);
    rows_issue(Cq[0], 0, 0);
    rows_issue(Cq[0], 0, 1);
  } else {  // group 1's first aggregation step is tile -1 (weights of tile 0 only)
    Cq[1] = rec_load(0);
    Cq[0] = Cq[1];
    Cq[2] = rec_load(1);
    logits_issue(Cq[1], 0);
  }
  __syncthreads();  // Z zeroed

#ifdef GFD_LP_PROF
  unsigned long long pc[7] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
#endif
  for (int64_t st = -2; st < 2 * nv; ++st) {
    lane = opaque(threadIdx.x & 63);
    const bool odd = (st & 1) != 0;
#ifdef GFD_LP_PROF
    const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
    const unsigned long long pw0 = pw;
    const bool vstep = (g == 0) ? odd : !odd;
#endif
    if (g == 0) {
      if (odd) {
        const int64_t v = (st + 1) / 2;
        if (v < nv) valu_step(v);
      } else if (st >= 0) {
        mfma(st / 2);
        rotate();
      }
    } else {
      if (!odd) {
        valu_step(st / 2);
      } else {
        const int64_t v = (st - 1) / 2;
        if (v >= 0) mfma(v);
        rotate();
      }
    }
#ifdef GFD_LP_PROF
    const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();
#ifdef GFD_LP_PROF
    const unsigned long long ts2 = __builtin_amdgcn_s_memtime();
    if (st >= 0) {
      pc[vstep ? 0 : 2] += ts1 - ts0;
      pc[1] += pw - pw0;
      pc[vstep ? 3 : 4] += ts2 - ts1;
      pc[vstep ? 5 : 6] += 1;
    }
#endif
  }
#ifdef GFD_LP_PROF
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 7; ++i) atomicAdd(&g_lprof[g][i], pc[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) atomicAdd(&g_lprof[g][8 + i], pv[i]);
  }
#endif
}

template <typename XT, int KHM, int LO, bool EXACT>
gfd_status launch_pair_k(const AggArgs& a, const PackLayout& L, bool to_end, hipStream_t stream) {
  const bool epi = a.ep.ab != nullptr;
  auto kern = epi ? &k_light_pair<XT, KHM, LO, EXACT, true>
                  : &k_light_pair<XT, KHM, LO, EXACT, false>;
  const size_t lds = light_pair_smem(L.Fp, LO);
  if (lds > kLdsBytes) return GFD_ERR_UNSUPPORTED;
  if (!ensure_lds(reinterpret_cast<const void*>(kern), lds)) return GFD_ERR_HIP;
  const int64_t tiles = (a.num_dst + kTile - 1) / kTile;
  int64_t grid = cu_count();
  if (grid > tiles) grid = tiles;
  const gfd_plan& p = a.plan;
  kern<<<int(grid), kLW * 64, lds, stream>>>(
      a.x, a.N, a.F, L.Fp, a.ldx, a.num_dst,
      reinterpret_cast<const int4*>(p.slot_desc), p.slot_cols, a.s, a.lds, a.t, a.ldt,
      reinterpret_cast<const PackHeader*>(a.packed + L.hdr_off),
      reinterpret_cast<const uint4*>(a.packed + L.wsh_off),
      reinterpret_cast<const uint4*>(a.packed + L.wsl_off), a.bias, a.slope, a.dp, a.seed, a.out,
      a.stats, a.xmax, p.class_split, to_end ? 1 : 0, a.ep);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

}  // namespace

namespace gfd {
namespace fwd {

bool light_pair_supported(const AggArgs& a, const PackLayout& L) {
  const int eb = a.xdt == GFD_DTYPE_BF16 ? 2 : 4;
  return (a.xdt == GFD_DTYPE_F32 || (GFD_LIGHT_PAIR_BF16 && a.xdt == GFD_DTYPE_BF16)) &&
         kf_for(a.F) == 3 && a.F >= 64 + L.Fp / 2 && a.ldx * eb <= 0x7fffffffLL &&
         a.ep.hout == nullptr && a.N <= 0x7fffffff &&
         a.plan.slot_desc && a.plan.slot_cols && a.plan.class_split;
}

gfd_status launch_light_pair(const AggArgs& a, const PackLayout& L, bool to_end,
                             hipStream_t stream) {
  if (!light_pair_supported(a, L)) return GFD_ERR_UNSUPPORTED;
  if (!(a.slope >= 0.f && a.slope <= 1.f)) return GFD_ERR_UNSUPPORTED;  // leaky01
  const bool exact = L.KS / 2 == 21;
  if (a.xdt == GFD_DTYPE_BF16)
    return exact ? launch_pair_k<XBF16, 21, 8, true>(a, L, to_end, stream)
                 : launch_pair_k<XBF16, 21, 8, false>(a, L, to_end, stream);
  return exact ? launch_pair_k<XF32, 21, 8, true>(a, L, to_end, stream)
               : launch_pair_k<XF32, 21, 8, false>(a, L, to_end, stream);
}

}  // namespace fwd
}  // namespace gfd

#ifdef GFD_LP_PROF
extern "C" int gfd_lprof_read(unsigned long long* out16, int reset) {
  if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_lprof), sizeof(g_lprof)) != hipSuccess) return 1;
  if (reset) {
    static const unsigned long long zero[2][16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_lprof), zero, sizeof(zero)) != hipSuccess) return 1;
  }
  return 0;
}
#endif
