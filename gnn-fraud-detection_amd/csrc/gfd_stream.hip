// gfd_stream.hip -- general (hub rows and 7+ messages) and light (2..kLightMax
// = 6 messages incl. the self loop) destinations: the PyG GATConv.forward
// softmax-aggregate-project of /root/reference/src/models/gat.py:80 for the
// bulk of a power-law graph.  One kernel template, two instances (LIGHT).
//
// Weight-stationary streaming tile kernel (persistent, one 8-wave block per
// CU, two waves per SIMD at up to 256 VGPRs):
//  * The projection weights stay on chip for the launch: wave w owns column
//    tile ct = w & 3 over K half kh = w >> 2 (k-steps [kh*KH, kh*KH + KH)):
//    W_hi of its k-steps in VGPRs, W_lo of the first KH - LO in VGPRs and of
//    the last LO in LDS.  Only x rows, logits and slot records stream per tile.
//  * Z goes through LDS once per 16-row tile in the feature-major K order
//    p = 8 f + h, so a lane stores all 8 heads of its feature with one 16-B
//    write per (hi, lo).  acc += Zhi.Whi + Zhi.Wlo + Zlo.Whi (lo unscaled).
//  * Two destinations per wave (rows 2w, 2w+1).  The first 4 x rows of a
//    general slot (all kLightMax of a light slot's) are issued one tile
//    ahead, between the MFMA k-steps of the current tile; records are loaded
//    two tiles ahead.
//  * General slots (LIGHT = false) continue with an online softmax over
//    batches of 8 messages: the sources of messages 8..71 come with the
//    record (one 64-wide window of the CSR columns), so the logits and all 8
//    rows of the next batch are issued together at the end of the current one
//    (one memory round trip per batch); hub rows load their merged z.
//  * Per tile: MFMA -> kh = 1 partials to LDS -> barrier -> kh = 0 waves reduce
//    and store out (during the next tile's MFMA); every wave aggregates its
//    next rows into Z -> barrier.
//
// LDS ownership (the invariant every access below keeps):
//  * ring[par][r] (slot records: descriptor and, general only, the first 8
//    sources) is private to the wave that owns slot r
//    (r = 2w, 2w + 1): written by that wave when it issues tile v + 1 (during
//    MFMA(v), parity (v + 1) & 1) and read by the same wave after barrier 1 of
//    iteration v.  The next write of that parity happens at iteration v + 2,
//    two barriers later.  No other wave touches it.
//  * Z tile: written after barrier 1 (tile v + 1), read by MFMA(v + 1) after
//    barrier 2; MFMA(v) reads complete before barrier 1.
//  * rsc/rid[par]: written with Z (parity of the tile), read by kh = 0 waves in
//    reduce_store(tile v - 1) during MFMA(v), before barrier 1; the next write
//    of that parity is after barrier 1 of iteration v.
//  * red[par]: written by kh = 1 waves after MFMA(v), read by kh = 0 waves
//    during MFMA(v + 1) (after barriers 1 and 2 of v), next written after
//    MFMA(v + 2).
#include "gfd_fwd.h"

using namespace gfd;
using namespace gfd::fwd;

namespace {

// The epilogue (BN affine / ReLU / residual, gfd.fused) and the folded model
// head are compiled into EPI instances only: the plain layer's tile loop then
// carries none of their code (C4 -0.2 ms against one instance with run-time
// checks: profiles/r5z_epi_instances.txt)
#define GFD_HOUT(ep) (EPI && ep.hout)

constexpr int kSWaves = 8;
// s_setprio 1 once for one half of the block (1: waves 4-7, 2: waves 0-3):
// within box noise either way (C4 13.14-13.16 / 13.00-13.03 vs 13.09-13.19 ms,
// profiles/r6_stream_knobs_ab.txt), off
#ifndef GFD_STREAM_SETPRIO
#define GFD_STREAM_SETPRIO 0
#endif
// Z tile row pad (halves): 8 gives the A-fragment ds_read_b128 reads a 2-way
// bank conflict in one of their 16-lane groups, 16 none (scripts/bank_pad.py;
// C4 13.09 / 13.19 -> 12.99 / 13.00 ms, profiles/r6_stream_knobs_ab.txt)
#ifndef GFD_STREAM_ZPAD
#define GFD_STREAM_ZPAD 16
#endif
// Light slots: message weights broadcast through LDS (fma_k_lds: 2 broadcast
// reads per message instead of 8 v_readlane; the light kernel's VALU count
// -25 %) -- measured neutral (C4 light 6.34-6.61 vs 6.36-6.51 ms across three
// box pairs, C5 34.3 vs 33.7 ms: profiles/r5c_light_ablation.txt), so off by
// default: the kernel is not bound by its VALU count
#ifndef GFD_LIGHT_ALDS
#define GFD_LIGHT_ALDS 0
#endif
#ifndef GFD_LIGHT_AP
#define GFD_LIGHT_AP 1
#endif
#ifndef GFD_LIGHT_AP_BF16
#define GFD_LIGHT_AP_BF16 2
#endif
#ifndef GFD_GENERAL_AP
#define GFD_GENERAL_AP 1
#endif
// short light tiles (every slot at most kLightLo messages: LIGHT = 2): kLightLo
// rows per slot in flight instead of kLightMax, so the A fragments can be read
// further ahead
#ifndef GFD_LIGHT_LO_AP
#define GFD_LIGHT_LO_AP 2
#endif
#ifndef GFD_LIGHT_LO_AP_BF16
#define GFD_LIGHT_LO_AP_BF16 2
#endif
#ifndef GFD_LIGHT_LO_WL
#define GFD_LIGHT_LO_WL 8
#endif
// bf16 rows held as RowL pairs (2 VGPRs a row instead of 3) where they allow it
#ifndef GFD_STREAM_PAIRS
#define GFD_STREAM_PAIRS 1
#endif
// A-fragment k-steps read ahead in the MFMA loop (general; light fp32 / bf16
// rows).  Light fp32: 1 keeps the kernel spill-free with 6 rows per slot in
// flight (C4 light 6.73 -> 6.22 ms against 2); light bf16: 2 (C5 33.3 vs 33.7 ms)
// LIGHT: 0 general tiles, 1 light tiles (2..kLightMax messages), 2 short
// light tiles (at most kLightLo)
template <int LIGHT, typename XT>
constexpr int ap_of() {
  return LIGHT == 2 ? (XT::kBytes == 2 ? GFD_LIGHT_LO_AP_BF16 : GFD_LIGHT_LO_AP)
       : LIGHT ? (XT::kBytes == 2 ? GFD_LIGHT_AP_BF16 : GFD_LIGHT_AP) : GFD_GENERAL_AP;
}
// x rows of a general slot issued one tile ahead (the rest of batch 0 is
// issued when its aggregation starts).  fp32 rows: 4 since round 6 (the two
// slots sharing their batch registers left room: spill-free at 255 VGPRs;
// C4 general -0.04..-0.07 ms, profiles/r6q_hub_pairs_general_nl4_ab.txt --
// until then 0: 3.13 -> 3.00 ms against the spilling 4 of round 2); bf16 rows:
// 4 (without them C5's general stage 35.8 -> 56.2 ms: the half-size rows
// issued during the MFMA phase hide most of a round trip)
#ifndef GFD_GENERAL_NL_F32
#define GFD_GENERAL_NL_F32 4
#endif
#ifndef GFD_GENERAL_NL_BF16
#define GFD_GENERAL_NL_BF16 4
#endif
// ... bf16 rows held as RowL pairs (2 VGPRs a row)
#ifndef GFD_GENERAL_NL_BF16P
#define GFD_GENERAL_NL_BF16P 4
#endif
template <int LIGHT, typename XT, bool PR = false>
constexpr int nl_of() {
  return LIGHT == 2 ? kLightLo
       : LIGHT ? (XT::kBytes == 2 ? kLightMaxBf16 : kLightMax)
       : (XT::kBytes == 2 ? (PR ? GFD_GENERAL_NL_BF16P : GFD_GENERAL_NL_BF16) : GFD_GENERAL_NL_F32);
}

#ifdef GFD_PROF
// Diagnostic build only (GFD_BUILD_VARIANT=prof GFD_EXTRA_FLAGS=-DGFD_PROF):
// per-wave s_memtime cycles of the tile loop phases, summed over waves,
// [LIGHT: 0 general, 1 light, 2 short light][phase]: 0 MFMA + next-tile issue, 1 barrier 1, 2 aggregation,
// 3 barrier 2; [light][4] tiles; [light][5] cycles of the aggregation spent
// waiting for the loads in flight at its start (an explicit vmcnt(0) wait).
// Read by gfd_prof_read (scripts/prof_phases.py).
__device__ unsigned long long g_prof[3][6];
#endif

struct SlotRec {  // one tile slot as loaded (vector loads: no SMEM in the lgkm queue)
  int v;          // lanes 0..3: {row, e_begin, e_end, hub_rank}; lanes 8..15: sources of
                  // messages 0..7 (slot_cols); other lanes: row
  bool live;      // slot < num_dst (otherwise v is a clamped copy, row taken as -1)
};

struct SlotRing {  // a slot record parked in LDS between issue and aggregation
  int4 d;          // {row (-1: empty), e_begin, e_end, hub_rank}
  int j[8];        // sources of messages 0..7 (general slots)
};

template <int KF, int NRW = 4, int W = KF>
struct SlotRows {  // a slot's first (and, for light slots, only) batch in flight
  float th;        // t_i of head lane & 7
  float sj;        // s_j of the lane's message (lane >> 3)
  int cj;          // general: source of message 8 + lane (0 past the end)
  int n;           // messages of the slot (wave-uniform; set with the logits)
  float xv[NRW][W];  // x rows of messages 0 .. NRW - 1 (RowL layout, W registers a row)
};

// live: slot < lim (<= num_dst): the light launch stops at the first lone slot
// when the lone rows are written elsewhere (k_lone, k_logits_lone)
__device__ __forceinline__ void sl_rec(SlotRec& p, int64_t slot, int64_t num_dst, int64_t lim,
                                       const int4* __restrict__ desc,
                                       const int32_t* __restrict__ cols8, int lane) {
  const int64_t sl = slot < num_dst ? slot : num_dst - 1;
  const int32_t* a = reinterpret_cast<const int32_t*>(desc + sl) + (lane & 3);
  const int32_t* b = cols8 + sl * 8 + (lane & 7);
  p.v = *((lane & 56) == 8 ? b : a);  // one dword per lane, one VGPR per slot
  p.live = slot < lim;
}

// One piece of the issue of a slot: part 0 = logits (t_i, s_j), the source
// window (general) and the ring record; part 1 + k = x row k.  Issued
// unconditionally (past the last slot: clamped, ignored records), so no
// branch joins in-flight loads.
template <int PART, typename XT, int KF, int LIGHT, typename RL, int NRW>
__device__ __forceinline__ void sl_issue_part(const SlotRec& p, SlotRows<KF, NRW, RL::W>& q,
                                              const void* __restrict__ x, int64_t ldx, int F,
                                              const int32_t* __restrict__ col,
                                              const float* __restrict__ s, int lds,
                                              const float* __restrict__ t, int ldt,
                                              SlotRing* __restrict__ ring, int lane) {
  if constexpr (PART == 0) {
    const int h = lane & 7;
    const int row = __builtin_amdgcn_readlane(p.v, 0);  // >= 0: clamped slots are real rows
    const int e0 = __builtin_amdgcn_readlane(p.v, 1);
    const int e1 = __builtin_amdgcn_readlane(p.v, 2);
    const int hw = __builtin_amdgcn_readlane(p.v, 3);
    const int jm = __builtin_amdgcn_ds_bpermute((8 + (lane >> 3)) << 2, p.v);  // message lane >> 3
    q.n = e1 - e0;
    q.th = lrow(t, row, ldt)[h];
    q.sj = lrow(s, jm, lds)[h];
    if constexpr (!LIGHT) {
      // sources of messages 8 .. 71 (one per lane), range-checked: light, hub
      // and empty slots fetch nothing
      const int nx = (p.live && hw < 0 && e1 - e0 > 8) ? e1 - e0 - 8 : 0;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<int32_t*>(col) + e0 + 8, 0, nx * 4, 0x00020000);
      q.cj = int(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, 0, 0));
      if ((lane & 56) == 8) ring->j[lane & 7] = p.v;
    }
    if (lane == 0) ring->d = make_int4(p.live ? row : -1, e0, e1, hw);
  } else {
    // messages past the slot's end (light slots of 2 or 3 messages; the
    // padding sources repeat the last one) fetch nothing and read zeros
    constexpr int k = PART - 1;
    const int jk = __builtin_amdgcn_readlane(p.v, 8 + k);
    RL::load(xrow<XT>(x, jk, ldx), F, lane, k < q.n, q.xv[k]);
  }
}

// z = sum of the first kmax (2 .. NR, wave-uniform) rows, one straight-line
// block per count (K = 2 .. NR)
template <int KF, int NR, typename RL, int K = 2>
__device__ __forceinline__ void light_fma(f32x2 (&z)[4][KF], const float (&xv)[NR][RL::W],
                                          float p, int kmax) {
  static_assert(NR >= 2 && NR <= 7, "light slots: 2 .. 7 messages");
  if constexpr (K >= NR) {
    fma_k<KF, NR, NR, RL>(z, xv, p);
  } else {
    if (kmax <= K) fma_k<KF, K, NR, RL>(z, xv, p);
    else light_fma<KF, NR, RL, K + 1>(z, xv, p, kmax);
  }
}

// light_fma with the weights from the wave's LDS buffer (fma_k_lds)
template <int KF, int NR, typename RL, int K = 2>
__device__ __forceinline__ void light_fma_lds(f32x2 (&z)[4][KF], const float (&xv)[NR][RL::W],
                                              const float* __restrict__ ab, int kmax) {
  if constexpr (K >= NR) {
    fma_k_lds<KF, NR, NR, RL>(z, xv, ab);
  } else {
    if (kmax <= K) fma_k_lds<KF, K, NR, RL>(z, xv, ab);
    else light_fma_lds<KF, NR, RL, K + 1>(z, xv, ab, kmax);
  }
}

// A slot with at most kLightMax messages (all rows prefetched), not a hub
// (with dropout also the self-loop-only slots: their heads are masked one by
// one, so the head-mean shortcut of k_lone does not apply): straight-line
// code, the softmax sum and reciprocal independent of the FMA block.  kmax:
// messages to run (wave-uniform, >= n).
template <int KF, typename RL, int NR>
__device__ __forceinline__ void sl_light(const int4 d, const SlotRows<KF, NR, RL::W>& q, int kmax,
                                         float slope, float dp, uint64_t seed, int Fp,
                                         float* __restrict__ stats,
                                         _Float16* __restrict__ zh, _Float16* __restrict__ zl,
                                         float* __restrict__ rsc, int* __restrict__ rid, int r,
                                         int erg, float* __restrict__ ab, int lane) {
  if (d.x < 0) {  // past the last destination
    if (lane == 0) rid[r] = -1;
    return;
  }
  const int kk = lane >> 3;
  const int n = d.z - d.y;
  const float v = leaky01(q.sj + q.th, slope);
  const float m = max_xor8_16_32(kk < n ? v : -INFINITY);
  const float p = kk < n ? __expf(v - m) : 0.f;
  const float l = sum_xor8_16_32(p);
  if (__builtin_expect(stats != nullptr, 0) && lane < 8) {  // training only
    float* sr = stats + int64_t(d.x) * 16 + lane;
    sr[0] = m;
    sr[8] = l;
  }
  const float inv = __builtin_amdgcn_rcpf(l + kSoftmaxEps);
  // training: dropout on alpha after the softmax (the statistics above are the
  // undropped ones), the counter-based mask of (seed, CSR position, head) that
  // the general / hub kernels and the backward use
  float pd = p;
  if (__builtin_expect(dp > 0.f, 0))  // kernel-uniform
    pd = dropout_keep(seed, uint32_t(d.y + kk), uint32_t(lane & 7), dp) ? p * (1.0f / (1.0f - dp))
                                                                        : 0.f;
  f32x2 z[4][KF];
  f16x8 hi[KF], lo[KF];
  int er = erg;
  if (erg != 127) {
    // one scale for every row: fold 1 / (sum + eps) and 2^erg into the
    // weights, so z comes out normalised and scaled and only needs the split
    const float ps = pd * (inv * ldexpf(1.0f, erg));
#if GFD_LIGHT_ALDS
    ab[lane] = ps;  // this wave's own buffer: its LDS operations run in order
    light_fma_lds<KF, NR, RL>(z, q.xv, ab, kmax);
#else
    light_fma<KF, NR, RL>(z, q.xv, ps, kmax);
#endif
    split_zrow<KF>(z, hi, lo);
  } else {
#if GFD_LIGHT_ALDS
    ab[lane] = pd;
    light_fma_lds<KF, NR, RL>(z, q.xv, ab, kmax);
#else
    light_fma<KF, NR, RL>(z, q.xv, pd, kmax);
#endif
    er = pack_zrow<KF>(z, inv, erg, hi, lo);
  }
  write_zrow<KF, RL>(hi, lo, Fp, lane, zh, zl);
  if (lane == 0) {
    rsc[r] = ldexpf(1.0f, -er);
    rid[r] = d.x;
  }
}

// A general slot (record in the ring, first 4 rows in q): un-normalised z
// (head pairs, lane <-> feature) by an online softmax over batches of 8
// messages, then normalised, scaled, split and written into the Z tile.
//  * batch 0: logits and rows 0..3 were issued one tile ahead; rows 4..7 are
//    issued on entry.
//  * batches 1..: sources come from the cj window (lane i = message cb + i),
//    so the logits and all 8 rows of the next batch are issued together at
//    the end of the current one (one memory round trip per batch; a col ->
//    st -> rows chain would be three).
//  * hub rows: the merged, normalised z of k_hub_fin.
//  * xa / xb (8 rows of a batch) belong to the caller: the wave's two slots
//    share them, which keeps the bf16 instance (4 rows a tile ahead) spill-free
//    (C5 general stage 34.4 -> 25.9 ms; profiles/r6p_general_rows_ab.txt).
template <typename XT, int KF, typename RL, int NRW, int NRA>
__device__ __forceinline__ void sl_general(const SlotRing* __restrict__ ring,
                                           const SlotRows<KF, NRA, RL::W>& q,
                                           const void* __restrict__ x,
                                           int64_t ldx, int F, int Fp,
                                           const int32_t* __restrict__ col,
                                           const float* __restrict__ s, int lds, float slope, float dp,
                                           uint64_t seed, const float* __restrict__ zhub,
                                           float* __restrict__ stats, _Float16* __restrict__ zh,
                                           _Float16* __restrict__ zl, float* __restrict__ rsc,
                                           int* __restrict__ rid, int r, int erg, int lane,
                                           float (&xa)[4][RL::W], float (&xb)[4][RL::W]) {
  const int4 d = uni4(ring->d);
  const int j0 = ring->j[lane >> 3];
  const int h = lane & 7, kk = lane >> 3;
  // batch 0 of a slot: rows 0..3 (4..7 when it has more than 4 messages)
  auto issue0 = [&](int ja, int na) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
      RL::load(xrow<XT>(x, __builtin_amdgcn_readlane(ja, 8 * k), ldx), F, lane, k < na, xa[k]);
    if (na > 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        RL::load(xrow<XT>(x, __builtin_amdgcn_readlane(ja, 8 * (4 + k)), ldx), F, lane,
                 4 + k < na, xb[k]);
    }
  };
  f32x2 z[4][KF];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int qq = 0; qq < KF; ++qq) z[g][qq] = f32x2{0.f, 0.f};
  float inv = 1.0f;
  if (d.x < 0) {  // past the last destination
    if (lane == 0) rid[r] = -1;
    return;
  }
  if (d.w >= 0) {  // hub: merged row (already normalised)
    const float* src = zhub + int64_t(d.w) * (H * Fp);
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int qq = 0; qq < KF; ++qq) {
        const int f = RL::feat(qq, lane);
        if (f < Fp) z[g][qq] = f32x2{src[2 * g * Fp + f], src[(2 * g + 1) * Fp + f]};
      }
  } else {
    const int e0 = d.y, e1 = d.z;
    const int n = e1 - e0;
    const float keep = dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f;
    float m, l;
    {  // batch 0
      if constexpr (NRW == 0) issue0(j0, n);  // rows 0..7 issued here, before the softmax
      const bool valid = kk < n;
      const float v = leaky01(q.sj + q.th, slope);
      m = max_xor8_16_32(valid ? v : -INFINITY);
      float pv = valid ? __expf(v - m) : 0.f;
      l = pv;
      if (dp > 0.f) pv = dropout_keep(seed, uint32_t(e0 + kk), uint32_t(h), dp) ? pv * keep : 0.f;
      if constexpr (NRW == 0) {
        fma_rows<KF, 4, RL>(z, xa, pv, 0, min(4, n));
        if (n > 4) fma_rows<KF, 4, RL>(z, xb, pv, 4, min(4, n - 4));
      } else if constexpr (NRW == 8) {  // the whole batch issued a tile ahead
        fma_rows<KF, 8, RL>(z, q.xv, pv, 0, min(8, n));
      } else {
        static_assert(NRW == 4, "general slots: 0, 4 or 8 rows a tile ahead");
        fma_rows<KF, 4, RL>(z, q.xv, pv, 0, min(4, n));
      }
      if (NRW == 4 && n > 4) {  // rows 4..7
#pragma unroll
        for (int k = 0; k < 4; ++k)
          RL::load(xrow<XT>(x, __builtin_amdgcn_readlane(j0, 8 * (4 + k)), ldx), F, lane,
                   4 + k < n, xb[k]);
        fma_rows<KF, 4, RL>(z, xb, pv, 4, min(4, n - 4));
      }
    }
    // batches 1..: loads of batch b issued at the end of batch b - 8
    int cj = q.cj, cb = 8;  // cj window: lane i = message cb + i
    float sv = 0.f;
    auto issue = [&](int b) {
      if (b - cb >= 64) {  // past the window (more than 72 messages): next 64 sources
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<int32_t*>(col) + e0 + b, 0, (n - b) * 4, 0x00020000);
        cj = int(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, 0, 0));
        cb = b;
      }
      const int jl = __builtin_amdgcn_ds_bpermute((b - cb + kk) << 2, cj);
      sv = lrow(s, jl, lds)[h];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        RL::load(xrow<XT>(x, __builtin_amdgcn_readlane(cj, b - cb + k), ldx), F, lane,
                 b + k < n, xa[k]);
      if (n - b > 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          RL::load(xrow<XT>(x, __builtin_amdgcn_readlane(cj, b - cb + 4 + k), ldx), F,
                   lane, b + 4 + k < n, xb[k]);
      }
    };
    if (n > 8) issue(8);
    for (int b = 8; b < n; b += 8) {
      const bool valid = b + kk < n;
      const float v = leaky01(sv + q.th, slope);
      const float mn = fmaxf(m, max_xor8_16_32(valid ? v : -INFINITY));
      const float sc = __expf(m - mn);
      float pv = valid ? __expf(v - mn) : 0.f;
      l = fmaf(l, sc, pv);
      {  // rescale (unconditional: a wave-uniform branch here costs the register
         // allocator more than the 12 multiplies it would skip)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x2 s2 = bcast2(sc, 2 * g);
#pragma unroll
          for (int qq = 0; qq < KF; ++qq) z[g][qq] *= s2;
        }
      }
      m = mn;
      if (dp > 0.f)
        pv = dropout_keep(seed, uint32_t(e0 + b + kk), uint32_t(h), dp) ? pv * keep : 0.f;
      fma_rows<KF, 4, RL>(z, xa, pv, 0, min(4, n - b));
      if (n - b > 4) fma_rows<KF, 4, RL>(z, xb, pv, 4, min(4, n - b - 4));
      if (b + 8 < n) issue(b + 8);
    }
    l = sum_xor8_16_32(l);
    if (__builtin_expect(stats != nullptr, 0) && lane < 8) {  // training only
      float* sr = stats + int64_t(d.x) * 16 + lane;
      sr[0] = m;
      sr[8] = l;
    }
    inv = __builtin_amdgcn_rcpf(l + kSoftmaxEps);
  }
  f16x8 hi[KF], lo[KF];
  const int er = pack_zrow<KF>(z, inv, erg, hi, lo);
  write_zrow<KF, RL>(hi, lo, Fp, lane, zh, zl);
  if (lane == 0) {
    rsc[r] = ldexpf(1.0f, -er);
    rid[r] = d.x;
  }
}

// PR: bf16 rows held as RowL pairs (2 VGPRs a row; 128 < F <= 192, 4-B aligned rows)
template <typename XT, int KF, int KHM, int LO, bool EXACT, int LIGHT, bool EPI, bool PR>
__global__ void __launch_bounds__(kSWaves * 64, 2) k_stream(
    const void* __restrict__ x, int F, int Fp, int64_t ldx, const int32_t* __restrict__ col,
    int64_t num_dst, const int4* __restrict__ desc,
    const int32_t* __restrict__ cols8, const float* __restrict__ s, int lds,
    const float* __restrict__ t, int ldt, const PackHeader* __restrict__ hdr, const uint4* __restrict__ wsh,
    const uint4* __restrict__ wsl, const float* __restrict__ bias, float slope, float dp,
    uint64_t seed, const float* __restrict__ zhub, float* __restrict__ out,
    float* __restrict__ stats, const float* __restrict__ xmax,
    const int64_t* __restrict__ split, int to_end, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char ssm[];
  const int ZS = 8 * Fp + GFD_STREAM_ZPAD;                      // row stride (fp16)
  const int KH = EXACT ? KHM : Fp / 8;                          // k-steps per K half (<= KHM)
  _Float16* Zh = reinterpret_cast<_Float16*>(ssm);              // [16][ZS]
  _Float16* Zl = Zh + kTile * ZS;                               // [16][ZS]
  f32x4* red0 = reinterpret_cast<f32x4*>(Zl + kTile * ZS);      // [2 parity][4 ct][64]
  SlotRing* ring0 = reinterpret_cast<SlotRing*>(red0 + 2 * 4 * 64);  // [2 parity][16]
  float* rsc0 = reinterpret_cast<float*>(ring0 + 2 * kTile);    // [2][16] by tile parity
  int* rid0 = reinterpret_cast<int*>(rsc0 + 2 * kTile);         // [2][16]
  uint4* WL = reinterpret_cast<uint4*>(rid0 + 2 * kTile);       // [8 waves][LO][64]
  // model head (ep.hout): per-tile row-dot partials of the 4 column tiles and
  // the rows, by tile parity (written by the kh = 0 waves in reduce_store,
  // summed by wave 4 after the next barrier 1)
  float* hpart = reinterpret_cast<float*>(WL + kSWaves * LO * 64);  // [2][4 ct][16]
  int* hrow = reinterpret_cast<int*>(hpart + 2 * 4 * kTile);         // [2][16]

  const int wave = wave_uniform(threadIdx.x >> 6);
  const int ct = wave & 3, kh = wave >> 2;
  const int r0 = 2 * wave, r1 = r0 + 1;
  const int64_t G = gridDim.x;
  const int64_t t0 = blockIdx.x;
  // general tiles: [0, ceil(split[g] / 16)), every tile without a split;
  // light tiles: [ceil(split[g] / 16), ceil(split[2] / 16)); short light
  // tiles: [ceil(split[2] / 16), ceil(split[1] / 16)) (to_end: up to the last
  // tile, when k_lone does not run); this block takes tiles t0 + v G.  g = 0
  // (light bound kLightMax) for fp32 rows, 3 (kLightMaxBf16) for bf16 rows
  constexpr int kG = XT::kBytes == 2 ? 3 : 0;
  const int64_t all = (num_dst + kTile - 1) / kTile;
  const int64_t tb = LIGHT ? (split[LIGHT == 2 ? 2 : kG] + kTile - 1) / kTile : 0;
  const int64_t te = LIGHT == 2 ? ((to_end ? num_dst : split[1]) + kTile - 1) / kTile
                   : LIGHT ? (split[2] + kTile - 1) / kTile
                           : (split ? (split[kG] + kTile - 1) / kTile : all);
  const int64_t nv = t0 < te - tb ? (te - tb - 1 - t0) / G + 1 : 0;
  // light, not to the end: the slots of the last tile past split[1] are lone
  // rows another kernel writes -- taken as empty here
  const int64_t lim = (LIGHT && !to_end) ? split[1] : num_dst;
  int lane = opaque(threadIdx.x & 63);
  auto slot = [&](int64_t v, int r) { return (tb + t0 + v * G) * kTile + r; };

  // kernel-lifetime constants first: nothing the loop waits on may be loaded
  // after the first rows are issued
  const float bcol = bias ? bias[ct * 16 + (lane & 15)] : 0.f;
  const float wu = hdr->w_unscale;
  const int erg = global_scale_exp(xmax, dp);
  constexpr int NR = KHM - LO;  // k-steps (of KHM) with W_lo in registers
  f16x8 bh[KHM], bl[NR > 0 ? NR : 1];
#pragma unroll
  for (int u = 0; u < KHM; ++u) {
    uint4 vh = make_uint4(0, 0, 0, 0), vl = vh;
    if (u < KH) {
      const int idx = ((kh * KH + u) * 4 + ct) * 64 + lane;
      vh = wsh[idx];
      vl = wsl[idx];
    }
    bh[u] = *reinterpret_cast<const f16x8*>(&vh);
    if (u < NR) bl[u < NR ? u : 0] = *reinterpret_cast<const f16x8*>(&vl);
    else WL[(wave * LO + (u - NR)) * 64 + lane] = vl;
  }
  if (nv == 0) return;  // uniform per block: no barrier below is reached by anyone
#if GFD_STREAM_SETPRIO == 1
  // static priority for the second-dispatched half (waves 4-7), once, before
  // the loop (MI355X_MICROARCH.md, two waves per SIMD, item 4)
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#elif GFD_STREAM_SETPRIO == 2
  if (wave < 4) __builtin_amdgcn_s_setprio(1);
#endif

  SlotRec n0, n1;
  constexpr int NL = nl_of<LIGHT, XT, PR>();  // rows issued one tile ahead per slot
  constexpr int NA = NL > 0 ? NL : 1;      // (register arrays of at least one row)
  using RL = RowL<XT, KF, PR>;
  SlotRows<KF, NA, RL::W> d0, d1;
  // prologue: tile 0 issued and aggregated; records of tile 1 loading
  sl_rec(n0, slot(0, r0), num_dst, lim, desc, cols8, lane);
  sl_rec(n1, slot(0, r1), num_dst, lim, desc, cols8, lane);
#define GFD_ISSUE(P, n, d, ring) \
  sl_issue_part<P, XT, KF, LIGHT, RL>(n, d, x, ldx, F, col, s, lds, t, ldt, ring, lane)
#define GFD_ROW(k, n, d, ring) \
  if constexpr (NL >= k) GFD_ISSUE((NL >= k ? k : 0), n, d, ring)
  GFD_ISSUE(0, n0, d0, ring0 + r0);
  GFD_ROW(1, n0, d0, ring0 + r0); GFD_ROW(2, n0, d0, ring0 + r0); GFD_ROW(3, n0, d0, ring0 + r0);
  GFD_ROW(4, n0, d0, ring0 + r0); GFD_ROW(5, n0, d0, ring0 + r0); GFD_ROW(6, n0, d0, ring0 + r0);
  GFD_ROW(7, n0, d0, ring0 + r0); GFD_ROW(8, n0, d0, ring0 + r0);
  GFD_ISSUE(0, n1, d1, ring0 + r1);
  GFD_ROW(1, n1, d1, ring0 + r1); GFD_ROW(2, n1, d1, ring0 + r1); GFD_ROW(3, n1, d1, ring0 + r1);
  GFD_ROW(4, n1, d1, ring0 + r1); GFD_ROW(5, n1, d1, ring0 + r1); GFD_ROW(6, n1, d1, ring0 + r1);
  GFD_ROW(7, n1, d1, ring0 + r1); GFD_ROW(8, n1, d1, ring0 + r1);
  sl_rec(n0, slot(1, r0), num_dst, lim, desc, cols8, lane);
  sl_rec(n1, slot(1, r1), num_dst, lim, desc, cols8, lane);
  auto aggregate = [&](int tpar) {  // this wave's two slots of the tile in parity tpar
    SlotRing* rg = ring0 + tpar * kTile;
    float* rsc = rsc0 + tpar * kTile;
    int* rid = rid0 + tpar * kTile;
    if constexpr (LIGHT) {
      const int4 da = uni4(rg[r0].d), db = uni4(rg[r1].d);
      const int kmax = max(da.z - da.y, db.z - db.y);  // wave-uniform
      // message-weight buffers: the kh = 1 partials region of this tile's
      // parity, free between barrier 1 and the next MFMA phase (its last
      // reader, reduce_store of tile v - 1, ran before barrier 1); 2 x 256 B per wave
      float* ab = reinterpret_cast<float*>(red0 + tpar * 4 * 64) + wave * 128;
      sl_light<KF, RL>(da, d0, kmax, slope, dp, seed, Fp, stats, Zh + r0 * ZS, Zl + r0 * ZS, rsc, rid,
                   r0, erg, ab, lane);
      sl_light<KF, RL>(db, d1, kmax, slope, dp, seed, Fp, stats, Zh + r1 * ZS, Zl + r1 * ZS, rsc, rid,
                   r1, erg, ab + 64, lane);
    } else {
      float xa[4][RL::W], xb[4][RL::W];  // the two slots' batch registers (sl_general)
      sl_general<XT, KF, RL, NL, NA>(rg + r0, d0, x, ldx, F, Fp, col, s, lds, slope, dp, seed, zhub,
                                 stats, Zh + r0 * ZS, Zl + r0 * ZS, rsc, rid, r0, erg, lane, xa, xb);
      sl_general<XT, KF, RL, NL, NA>(rg + r1, d1, x, ldx, F, Fp, col, s, lds, slope, dp, seed, zhub,
                                 stats, Zh + r1 * ZS, Zl + r1 * ZS, rsc, rid, r1, erg, lane, xa, xb);
    }
  };
  aggregate(0);
  __syncthreads();

  // out rows of a finished tile (waves kh = 0): own K-half partial + the other
  // half's from LDS, row scale, bias
  auto reduce_store = [&](const f32x4& acc, int tpar) {
    const float* rsc = rsc0 + tpar * kTile;
    const int* rid = rid0 + tpar * kTile;
    const f32x4 sum = acc + red0[(tpar * 4 + ct) * 64 + lane];
    const int n = ct * 16 + (lane & 15);
    if (GFD_HOUT(ep)) {  // kernel-uniform: the head's dot over this wave's 16 columns
      const float w = ep.hw[n];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = (lane >> 4) * 4 + q;
        const int ri = rid[r];
        const float v = ri >= 0 ? epi_store_value<EPI>(sum[q] * (rsc[r] * wu), bcol, n, ri, ep) * w
                                : 0.f;
        const float d = row16_sum(v);  // lanes 16 k .. 16 k + 15 hold row 4 k + q
        if ((lane & 15) == 0) {
          hpart[(tpar * 4 + ct) * kTile + r] = d;
          if (ct == 0) hrow[tpar * kTile + r] = ri;
        }
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (lane >> 4) * 4 + q;
      const int ri = rid[r];
      if (ri >= 0) out[int64_t(ri) * ep.ldo + n] = epi_store_value<EPI>(sum[q] * (rsc[r] * wu), bcol, n, ri, ep);
    }
  };
  // the head's outputs of a finished tile: the four column tiles' partials in
  // a fixed order (wave 4, after the barrier that follows reduce_store)
  auto head_out = [&](int tpar) {
    if (wave == 4 && lane < kTile) {
      const int ri = hrow[tpar * kTile + lane];
      const float* hp = hpart + tpar * 4 * kTile + lane;
      if (ri >= 0)
        ep.hout[ri] = ((hp[0] + hp[kTile]) + (hp[2 * kTile] + hp[3 * kTile])) +
                      (ep.hb ? ep.hb[0] : 0.f);
    }
  };
  f32x4 acc_prev = {0.f, 0.f, 0.f, 0.f};  // kh = 0: tile v - 1, stored during MFMA(v)
#ifdef GFD_PROF
  unsigned long long pc[5] = {0ull, 0ull, 0ull, 0ull, 0ull};
#endif
  for (int64_t v = 0; v < nv; ++v) {
#ifdef GFD_PROF
    const unsigned long long ts0 = __builtin_amdgcn_s_memtime();
#endif
    lane = opaque(threadIdx.x & 63);
    const int par = int(v & 1);
    // ---- MFMA: out[16 x 16] of column tile ct over K half kh ----
    const int aoff = (lane & 15) * ZS + 8 * (lane >> 4) + 32 * kh * KH;
    const _Float16* ah = Zh + aoff;
    const _Float16* al = Zl + aoff;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    // A fragments (and LDS-resident W_lo) kAP k-steps ahead; the scheduling
    // barriers keep the compiler from hoisting every LDS read of the tile
    // (registers belong to W)
    constexpr int kAP = ap_of<LIGHT, XT>();
    f16x8 phi[kAP], plo[kAP], pwl[kAP];
#pragma unroll
    for (int u = 0; u < kAP; ++u) {
      phi[u] = *reinterpret_cast<const f16x8*>(ah + 32 * u);
      plo[u] = *reinterpret_cast<const f16x8*>(al + 32 * u);
      if (u >= NR) {
        const uint4 w = WL[(wave * LO + (u - NR)) * 64 + lane];
        pwl[u] = *reinterpret_cast<const f16x8*>(&w);
      }
    }
    const int pn = par ^ 1;
    const bool more = v + 1 < nv;
#pragma unroll
    for (int u = 0; u < KHM; ++u) {
      // the next tile's rows are issued between the k-steps (the vector memory
      // pipe is idle in this phase): 2 NL + 2 pieces (per slot: header, NL
      // rows) spread evenly, piece i in k-step i * KHM / (2 NL + 2)
      SlotRing* rg = ring0 + pn * kTile;
#define GFD_PIECE(i) (u == (i) * KHM / (2 * NL + 2))
#define GFD_PROW(i, k, n, d, ring) \
  if constexpr (NL >= k) if (GFD_PIECE(i)) GFD_ISSUE((NL >= k ? k : 0), n, d, ring)
      if (GFD_PIECE(0)) GFD_ISSUE(0, n0, d0, rg + r0);
      GFD_PROW(1, 1, n0, d0, rg + r0); GFD_PROW(2, 2, n0, d0, rg + r0);
      GFD_PROW(3, 3, n0, d0, rg + r0); GFD_PROW(4, 4, n0, d0, rg + r0);
      GFD_PROW(5, 5, n0, d0, rg + r0); GFD_PROW(6, 6, n0, d0, rg + r0);
      GFD_PROW(7, 7, n0, d0, rg + r0); GFD_PROW(8, 8, n0, d0, rg + r0);
      if (GFD_PIECE(NL)) sl_rec(n0, slot(v + 2, r0), num_dst, lim, desc, cols8, lane);
      if (GFD_PIECE(NL + 1)) GFD_ISSUE(0, n1, d1, rg + r1);
      GFD_PROW(NL + 2, 1, n1, d1, rg + r1); GFD_PROW(NL + 3, 2, n1, d1, rg + r1);
      GFD_PROW(NL + 4, 3, n1, d1, rg + r1); GFD_PROW(NL + 5, 4, n1, d1, rg + r1);
      GFD_PROW(NL + 6, 5, n1, d1, rg + r1); GFD_PROW(NL + 7, 6, n1, d1, rg + r1);
      GFD_PROW(NL + 8, 7, n1, d1, rg + r1); GFD_PROW(NL + 9, 8, n1, d1, rg + r1);
#undef GFD_PROW
      if (GFD_PIECE(2 * NL + 1)) sl_rec(n1, slot(v + 2, r1), num_dst, lim, desc, cols8, lane);
#undef GFD_PIECE
      if (u == KHM - 2 && !kh && v > 0) reduce_store(acc_prev, pn);  // tile v - 1
      if (u < KH) {
        const f16x8 ahi = phi[u % kAP], alo = plo[u % kAP];
        f16x8 blo = u < NR ? bl[u < NR ? u : 0] : pwl[u % kAP];
        if (u + kAP < KH) {
          phi[u % kAP] = *reinterpret_cast<const f16x8*>(ah + 32 * (u + kAP));
          plo[u % kAP] = *reinterpret_cast<const f16x8*>(al + 32 * (u + kAP));
          if (u + kAP >= NR) {
            const uint4 w = WL[(wave * LO + (u + kAP - NR)) * 64 + lane];
            pwl[u % kAP] = *reinterpret_cast<const f16x8*>(&w);
          }
        }
        f32x4& acc = (u & 1) ? acc1 : acc0;
        {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bh[u], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, blo, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bh[u], acc, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    acc0 += acc1;
    if (kh) red0[(par * 4 + ct) * 64 + lane] = acc0;
    acc_prev = acc0;
#ifdef GFD_PROF
    const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();  // partials visible; every Z read of this tile done
#ifdef GFD_PROF
    const unsigned long long ts2 = __builtin_amdgcn_s_memtime();
    // the wait for every load in flight (the next tile's rows, issued during
    // the MFMA phase) before the aggregation: [5] (this stamp's own wait moves
    // the aggregation's first waits here)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pc[4] += __builtin_amdgcn_s_memtime() - ts2;
#endif

    // ---- tile v + 1: aggregate its rows into Z ----
    if (GFD_HOUT(ep) && v > 0) head_out(pn);  // tile v - 1 (its partials: before barrier 1)
    if (more) aggregate(pn);
#ifdef GFD_PROF
    const unsigned long long ts3 = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();  // Z of the next tile complete
#ifdef GFD_PROF
    const unsigned long long ts4 = __builtin_amdgcn_s_memtime();
    pc[0] += ts1 - ts0;
    pc[1] += ts2 - ts1;
    pc[2] += ts3 - ts2;
    pc[3] += ts4 - ts3;
#endif
  }
#ifdef GFD_PROF
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) atomicAdd(&g_prof[LIGHT][i], pc[i]);
    if (wave == 0) atomicAdd(&g_prof[LIGHT][4], (unsigned long long)nv);
    atomicAdd(&g_prof[LIGHT][5], pc[4]);
  }
#endif
#undef GFD_ROW
#undef GFD_ISSUE
  if (!kh) reduce_store(acc_prev, int((nv - 1) & 1));  // last tile
  if (GFD_HOUT(ep)) {  // kernel-uniform
    __syncthreads();
    head_out(int((nv - 1) & 1));
  }
}

size_t stream_smem(int Fp, int lo) {
  return sizeof(_Float16) * 2 * kTile * (8 * Fp + GFD_STREAM_ZPAD) + sizeof(f32x4) * 2 * 4 * 64 +
         sizeof(SlotRing) * 2 * kTile + sizeof(float) * 4 * kTile +
         sizeof(uint4) * kSWaves * lo * 64 + sizeof(float) * 2 * 4 * kTile +
         sizeof(int) * 2 * kTile;
}

template <typename XT, int KF, int KHM, int LO, bool EXACT, int LIGHT, bool PR = false>
gfd_status launch_stream_k(const AggArgs& a, const PackLayout& L, bool to_end,
                           hipStream_t stream) {
  const bool epi = a.ep.ab != nullptr || a.ep.hout != nullptr;
  auto kern = epi ? &k_stream<XT, KF, KHM, LO, EXACT, LIGHT, true, PR>
                  : &k_stream<XT, KF, KHM, LO, EXACT, LIGHT, false, PR>;
  if (EXACT && L.KS / 2 != KHM) return GFD_ERR_UNSUPPORTED;
  const size_t lds = stream_smem(L.Fp, LO);
  if (L.KS / 2 > KHM || lds > kLdsBytes) return GFD_ERR_UNSUPPORTED;
  if (!ensure_lds(reinterpret_cast<const void*>(kern), lds)) return GFD_ERR_HIP;
  const int64_t tiles = (a.num_dst + kTile - 1) / kTile;
  int64_t grid = cu_count();
  if (grid > tiles) grid = tiles;
  const gfd_plan& p = a.plan;
  // general: the slots before the light class (every tile without a class split)
  const int64_t* split = p.class_split;
  kern<<<int(grid), kSWaves * 64, lds, stream>>>(
      a.x, a.F, L.Fp, a.ldx, a.col, a.num_dst,
      reinterpret_cast<const int4*>(p.slot_desc), p.slot_cols, a.s, a.lds, a.t, a.ldt,
      reinterpret_cast<const PackHeader*>(a.packed + L.hdr_off),
      reinterpret_cast<const uint4*>(a.packed + L.wsh_off),
      reinterpret_cast<const uint4*>(a.packed + L.wsl_off), a.bias, a.slope, a.dp, a.seed,
      a.zhub, a.out, a.stats, a.xmax, split, to_end ? 1 : 0, a.ep);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

// Instance for this K: KH = KS / 2 k-steps per wave, at most KHM = 8 / 16 / 21
// for one / two / three feature chunks (F <= 64 / 128 / 168).  KF = 3 keeps
// W_lo of 8 k-steps per wave in LDS.
template <typename XT, int LIGHT>
gfd_status launch_stream_x(const AggArgs& a, const PackLayout& L, bool to_end,
                           hipStream_t stream) {
  const int KF = kf_for(a.F);
  const bool exact = L.KS / 2 == (KF == 1 ? 8 : KF == 2 ? 16 : 21);
  switch (KF) {
    case 1: return exact ? launch_stream_k<XT, 1, 8, 0, true, LIGHT>(a, L, to_end, stream)
                         : launch_stream_k<XT, 1, 8, 0, false, LIGHT>(a, L, to_end, stream);
    case 2: return exact ? launch_stream_k<XT, 2, 16, 0, true, LIGHT>(a, L, to_end, stream)
                         : launch_stream_k<XT, 2, 16, 0, false, LIGHT>(a, L, to_end, stream);
    case 3: {
      // W_lo k-steps in LDS: 8 (the registers go to rows in flight); the short
      // light tiles have registers to spare, but 4 (GFD_LIGHT_LO_WL) measured
      // the same (profiles/r6q_hub_pairs_general_nl4_ab.txt)
      constexpr int LO = LIGHT == 2 ? GFD_LIGHT_LO_WL : 8;
      // bf16 rows with F > 128 and 4-B aligned row starts: RowL pairs
      constexpr bool kB = XT::kBytes == 2;
      const bool pr = GFD_STREAM_PAIRS && kB && a.F > 128 &&
                      reinterpret_cast<uintptr_t>(a.x) % 4 == 0 && a.ldx % 2 == 0;
      if (pr)
        return exact ? launch_stream_k<XT, 3, 21, LO, true, LIGHT, kB>(a, L, to_end, stream)
                     : launch_stream_k<XT, 3, 21, LO, false, LIGHT, kB>(a, L, to_end, stream);
      return exact ? launch_stream_k<XT, 3, 21, LO, true, LIGHT>(a, L, to_end, stream)
                   : launch_stream_k<XT, 3, 21, LO, false, LIGHT>(a, L, to_end, stream);
    }
    default: return GFD_ERR_UNSUPPORTED;
  }
}

}  // namespace

namespace gfd {
namespace fwd {

gfd_status launch_general(const AggArgs& a, const PackLayout& L, hipStream_t stream) {
  const gfd_plan& p = a.plan;
  if (!p.slot_desc || !p.slot_cols) return GFD_ERR_UNSUPPORTED;
  if (!(a.slope >= 0.f && a.slope <= 1.f)) return GFD_ERR_UNSUPPORTED;  // leaky01
  return a.xdt == GFD_DTYPE_BF16 ? launch_stream_x<XBF16, 0>(a, L, false, stream)
                                 : launch_stream_x<XF32, 0>(a, L, false, stream);
}

gfd_status launch_light(const AggArgs& a, const PackLayout& L, bool to_end,
                        hipStream_t stream) {
  const gfd_plan& p = a.plan;
  if (!p.slot_desc || !p.slot_cols || !p.class_split) return GFD_ERR_UNSUPPORTED;
  if (!(a.slope >= 0.f && a.slope <= 1.f)) return GFD_ERR_UNSUPPORTED;  // leaky01
  // the light tiles, then the short light tiles (two persistent launches)
  const gfd_status st = a.xdt == GFD_DTYPE_BF16 ? launch_stream_x<XBF16, 1>(a, L, to_end, stream)
                                                : launch_stream_x<XF32, 1>(a, L, to_end, stream);
  if (st != GFD_OK) return st;
  return a.xdt == GFD_DTYPE_BF16 ? launch_stream_x<XBF16, 2>(a, L, to_end, stream)
                                 : launch_stream_x<XF32, 2>(a, L, to_end, stream);
}

}  // namespace fwd
}  // namespace gfd

#ifdef GFD_PROF
extern "C" int gfd_prof_read(unsigned long long* out18, int reset) {
  if (hipMemcpyFromSymbol(out18, HIP_SYMBOL(g_prof), sizeof(g_prof)) != hipSuccess) return 1;
  if (reset) {
    static const unsigned long long zero[3][6] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), zero, sizeof(zero)) != hipSuccess) return 1;
  }
  return 0;
}
#endif
