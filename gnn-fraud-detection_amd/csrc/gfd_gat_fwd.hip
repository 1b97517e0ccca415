// gfd_gat_fwd.hip -- GATConv forward entry points (PyG GATConv.forward,
// concat=False; /root/reference/src/models/gat.py:80 and tgn.py:94): argument
// checks, workspace layout and the per-class dispatch of the tile stage.
//
//   stage HUBS   k_hub_partial + k_hub_fin (gfd_hub.hip)
//   stage TILES  with a slot plan and F <= 168:
//                  general slots  k_stream<LIGHT = false>  (gfd_stream.hip)
//                  light slots    k_stream<LIGHT = true>
//                  lone slots     k_lone    (gfd_lone.hip)
//                otherwise        k_fused   (gfd_fused.hip)
// Classes come from the plan's class_split (gfd_plan_desc); with no class
// split every slot goes to the general kernel; with dropout the lone slots go
// to the light kernel (per-head masks).  No runtime switch changes what a
// call computes.
#include <map>
#include <mutex>
#include <utility>

#include "gfd_check.h"
#include "gfd_fwd.h"

using namespace gfd;
using namespace gfd::fwd;

namespace gfd {
namespace fwd {

int cu_count() {
  int dev = 0, v = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  static std::mutex mu;
  static std::map<int, int> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
    v = 256;
  cache[dev] = v;
  return v;
}

bool ensure_lds(const void* kernel, size_t bytes) {
  if (bytes <= 64 * 1024) return true;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, size_t> cache;  // largest size set per device
  std::lock_guard<std::mutex> g(mu);
  size_t& have = cache[{dev, kernel}];
  if (have >= bytes) return true;
  if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, int(bytes)) !=
      hipSuccess)
    return false;
  have = bytes;
  return true;
}

}  // namespace fwd
}  // namespace gfd

namespace {

bool check_hc(int heads, int channels, int F) {
  return heads == H && channels == C && F >= 1 && F <= 256;
}

bool dtype_ok(int xdt) { return xdt == GFD_DTYPE_F32 || xdt == GFD_DTYPE_BF16; }

// Tile classes to run: GFD_STAGE_TILES = all three, or any of the single-class
// bits (profiling: the same launches, split over calls).
constexpr int kMidBit = GFD_STAGE_TILES_GENERAL, kLightBit = GFD_STAGE_TILES_LIGHT,
              kLoneBit = GFD_STAGE_TILES_LONE;

gfd_status tiles_impl(const AggArgs& a, const PackLayout& L, hipStream_t stream) {
  const gfd_plan& p = a.plan;
  const int cls = (a.stages & GFD_STAGE_TILES) ? (kMidBit | kLightBit | kLoneBit)
                                               : (a.stages & (kMidBit | kLightBit | kLoneBit));
  const bool plan_path = kf_for(a.F) <= 3 && p.slot_desc && p.slot_cols &&
                         a.slope >= 0.f && a.slope <= 1.f;
  if (!plan_path) return (cls & kMidBit) ? launch_fused(a, L, stream) : GFD_OK;
  if (cls & kMidBit) {
    const gfd_status s = launch_general(a, L, stream);
    if (s == GFD_ERR_UNSUPPORTED) return launch_fused(a, L, stream);
    if (s != GFD_OK) return s;
  }
  if (!p.class_split) return GFD_OK;  // the general kernel took every tile
  // lone slots need 16-B aligned rows and no dropout (k_lone projects with the
  // head mean; a dropout mask differs per head); otherwise the light kernel
  // runs to the end and takes them as one-message slots -- unless the lone
  // class is not asked for (the logits pass produced it: gfd_gat_fwd_ep)
  const uintptr_t base = reinterpret_cast<uintptr_t>(a.x);
  const int eb = a.xdt == GFD_DTYPE_BF16 ? 2 : 4;
  const bool lone = base % 16 == 0 && (a.ldx * eb) % 16 == 0 && L.KB <= 6 && a.dp == 0.f;
  if (cls & kLightBit) {
    const gfd_status s = launch_light(a, L, !lone && (cls & kLoneBit), stream);
    if (s != GFD_OK) return s;  // the class split promised a light kernel for this F
  }
  return (lone && (cls & kLoneBit)) ? launch_lone(a, L, stream) : GFD_OK;
}

// The whole-graph forward may take the lone class out of the tile stage and
// into the logits pass (k_logits_lone): exactly when the tile stage would run
// the class-scheduled kernels with a lone class.
bool lone_fusable(const AggArgs& a, const PackLayout& L) {
  const gfd_plan& p = a.plan;
  return kf_for(a.F) <= 3 && L.KB <= 6 && p.slot_desc && p.slot_cols && p.class_split &&
         a.dp == 0.f && a.slope >= 0.f && a.slope <= 1.f && a.dst_offset == 0 &&
         a.num_dst == a.N && logits_lone_supported(a.x, a.xdt, a.F, a.ldx);
}

gfd_status aggregate_impl(const AggArgs& a, hipStream_t stream) {
  const PackLayout L = pack_layout(a.F);
  if (a.stages & GFD_STAGE_HUBS) {
    const gfd_status s = launch_hubs(a, L, stream);
    if (s != GFD_OK) return s;
  }
  if (!(a.stages & ~GFD_STAGE_HUBS) || a.num_dst == 0) return GFD_OK;
  return tiles_impl(a, L, stream);
}

gfd_status check_agg_args(const void* x, int xdt, int64_t N, int F, int64_t ldx,
                          const int32_t* rowptr, const int32_t* col, int64_t num_dst,
                          int64_t dst_offset, float dp, const gfd_plan& p, float* out) {
  if (!dtype_ok(xdt)) return GFD_ERR_ARGUMENT;
  if (N <= 0 || num_dst < 0 || dst_offset < 0 || dst_offset + num_dst > N) return GFD_ERR_ARGUMENT;
  if (!x || !rowptr || !col || !out || ldx < F) return GFD_ERR_ARGUMENT;
  if (!(dp >= 0.f && dp < 1.f)) return GFD_ERR_ARGUMENT;
  if (p.num_hubs < 0 || p.num_chunks < 0 || p.num_hubs > 0x7fffffff) return GFD_ERR_ARGUMENT;
  if (p.num_hubs > 0 &&
      (!p.hub_rank || !p.hub_chunk || !p.hub_chunk_ptr || !p.hub_dst || p.num_chunks <= 0))
    return GFD_ERR_ARGUMENT;
  if ((p.class_split || p.slot_cols) && !p.slot_desc) return GFD_ERR_ARGUMENT;
  // 32-bit row byte offsets in the gather kernels (xrow): ldx * elem < 2^32
  if (ldx > (int64_t(1) << 29)) return GFD_ERR_UNSUPPORTED;
  if ((num_dst + kTile - 1) / kTile > 0x7fffffff) return GFD_ERR_UNSUPPORTED;
  return GFD_OK;
}

gfd_plan plan_or_empty(const gfd_plan* p) {
  if (p) return *p;
  gfd_plan e;
  e.row_order = e.slot_desc = e.slot_cols = e.hub_rank = e.hub_chunk = e.hub_chunk_ptr = e.hub_dst =
      nullptr;
  e.class_split = nullptr;
  e.num_hubs = e.num_chunks = 0;
  return e;
}

void hub_ws_layout(Carve* c, int64_t num_hubs, int64_t num_chunks, const PackLayout& L,
                   float** part, float** zhub) {
  *part = c->take<float>(size_t(num_chunks) * (16 + L.KP));
  *zhub = c->take<float>(size_t(num_hubs) * L.KP);
}

}  // namespace

extern "C" {

size_t gfd_gat_fwd_workspace_size(int64_t num_nodes, int64_t num_dst, int F, int heads,
                                  int channels, int64_t num_hubs, int64_t num_chunks) {
  if (!check_hc(heads, channels, F)) return 0;
  (void)num_dst;
  const PackLayout L = pack_layout(F);
  Sizer s;
  s.take<float>(size_t(num_chunks) * (16 + L.KP));    // hub partials
  s.take<float>(size_t(num_hubs) * L.KP);             // merged hub z rows
  s.take<char>(L.bytes);                              // packed weights (gfd_gat_fwd only)
  s.take<float>(size_t(num_nodes) * 16);              // st (gfd_gat_fwd when st == NULL)
  s.take<float>(1);                                   // max |x| (gfd_gat_fwd)
  return s.off;
}

gfd_status gfd_gat_aggregate_split(const void* x, int x_dtype, int64_t N, int F, int64_t ldx,
                                   const int32_t* rowptr, const int32_t* col, int64_t num_dst,
                                   int64_t dst_offset, const float* s_log, int64_t s_stride,
                                   const float* t_log, int64_t t_stride, const float* xmax,
                                   const void* packed, const float* bias, int heads, int channels,
                                   float slope, float dp, uint64_t seed, const gfd_plan* plan,
                                   int stages, const gfd_epilogue* ep, float* out,
                                   int64_t out_stride, float* stats, void* ws, size_t ws_bytes,
                                   gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!check_hc(heads, channels, F)) return GFD_ERR_UNSUPPORTED;
  const gfd_plan p = plan_or_empty(plan);
  if (!out && ep && ep->head_out) out = ep->head_out;  // rows not written: the head replaces them
  gfd_status s =
      check_agg_args(x, x_dtype, N, F, ldx, rowptr, col, num_dst, dst_offset, dp, p, out);
  if (s != GFD_OK) return s;
  if (!s_log || !t_log || !packed || stages < 1 || stages > 31) return GFD_ERR_ARGUMENT;
  if (s_stride < H || t_stride < H || s_stride > (1 << 20) || t_stride > (1 << 20) ||
      out_stride < channels)
    return GFD_ERR_ARGUMENT;
  Epi e{nullptr, 0, nullptr, 0};
  if (ep) {  // inference epilogue (see gfd_gat_fwd_ep); residual rows indexed like out
    if (!ep->scale_shift || stats || dp > 0.f) return GFD_ERR_ARGUMENT;
    if (ep->residual && ep->residual_stride < channels) return GFD_ERR_ARGUMENT;
    e = Epi{ep->scale_shift, ep->relu ? 1 : 0, ep->residual, ep->residual_stride};
    e.hw = ep->head_weight;
    e.hb = ep->head_bias;
    e.hout = ep->head_out;
    if (e.hout && !e.hw) return GFD_ERR_ARGUMENT;
  }
  e.ldo = out_stride;
  if (num_dst == 0) return GFD_OK;
  const PackLayout L = pack_layout(F);
  s = check_graph(rowptr, col, num_dst, N, plan, nullptr, nullptr, nullptr, 0, stream);
  if (s != GFD_OK) return s;
  AggArgs a{x, x_dtype, F, ldx, N, rowptr, col, num_dst, dst_offset, s_log, int(s_stride),
            t_log, int(t_stride), static_cast<const char*>(packed), bias, slope, dp, seed, p,
            stages, out, stats, nullptr, nullptr, xmax, e};
  Carve c(ws, ws_bytes);
  hub_ws_layout(&c, p.num_hubs, p.num_chunks, L, &a.part, &a.zhub);
  if (!c.ok && p.num_hubs > 0) return GFD_ERR_WORKSPACE;
  return aggregate_impl(a, stream);
}

gfd_status gfd_gat_aggregate_ep(const void* x, int x_dtype, int64_t N, int F, int64_t ldx,
                                const int32_t* rowptr, const int32_t* col, int64_t num_dst,
                                int64_t dst_offset, const float* st, const float* xmax,
                                const void* packed, const float* bias, int heads, int channels,
                                float slope, float dp, uint64_t seed, const gfd_plan* plan,
                                int stages, const gfd_epilogue* ep, float* out, float* stats,
                                void* ws, size_t ws_bytes, gfd_stream_t stream_) {
  // [N, 16] table: s = columns 0..7 of every row, t = columns 8..15 of the
  // destination range's rows
  if (!st || dst_offset < 0) return GFD_ERR_ARGUMENT;
  return gfd_gat_aggregate_split(x, x_dtype, N, F, ldx, rowptr, col, num_dst, dst_offset, st, 16,
                                 st + dst_offset * 16 + H, 16, xmax, packed, bias, heads,
                                 channels, slope, dp, seed, plan, stages, ep, out, C, stats, ws,
                                 ws_bytes, stream_);
}

gfd_status gfd_gat_aggregate_ex(const void* x, int x_dtype, int64_t N, int F, int64_t ldx,
                                const int32_t* rowptr, const int32_t* col, int64_t num_dst,
                                int64_t dst_offset, const float* st, const float* xmax,
                                const void* packed, const float* bias, int heads, int channels,
                                float slope, float dp, uint64_t seed, const gfd_plan* plan,
                                int stages, float* out, float* stats, void* ws, size_t ws_bytes,
                                gfd_stream_t stream_) {
  return gfd_gat_aggregate_ep(x, x_dtype, N, F, ldx, rowptr, col, num_dst, dst_offset, st, xmax,
                              packed, bias, heads, channels, slope, dp, seed, plan, stages,
                              nullptr, out, stats, ws, ws_bytes, stream_);
}

gfd_status gfd_gat_aggregate(const void* x, int x_dtype, int64_t N, int F, int64_t ldx,
                             const int32_t* rowptr, const int32_t* col, int64_t num_dst,
                             int64_t dst_offset, const float* st, const void* packed,
                             const float* bias, int heads, int channels, float slope, float dp,
                             uint64_t seed, const gfd_plan* plan, int stages, float* out,
                             float* stats, void* ws, size_t ws_bytes, gfd_stream_t stream_) {
  return gfd_gat_aggregate_ex(x, x_dtype, N, F, ldx, rowptr, col, num_dst, dst_offset, st,
                              nullptr, packed, bias, heads, channels, slope, dp, seed, plan,
                              stages, out, stats, ws, ws_bytes, stream_);
}

// gfd_gat_fwd_ep with the packed weights either built here (packed_in NULL:
// weight / att_* packed into the workspace) or supplied (gfd_gat_fwd_ep_packed)
static gfd_status fwd_ep_impl(const void* x, int x_dtype, int64_t N, int F, int64_t ldx,
                          const int32_t* rowptr, const int32_t* col, const float* weight,
                          const float* att_src, const float* att_dst, const float* bias,
                          int heads, int channels, float slope, float dp, uint64_t seed,
                          const gfd_plan* plan, const gfd_epilogue* ep, float* out, float* st,
                          float* stats, void* ws, size_t ws_bytes, const void* packed_in,
                          gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!check_hc(heads, channels, F)) return GFD_ERR_UNSUPPORTED;
  const gfd_plan p = plan_or_empty(plan);
  if (!out && ep && ep->head_out) out = ep->head_out;  // rows not written: the head replaces them
  gfd_status s = check_agg_args(x, x_dtype, N, F, ldx, rowptr, col, N, 0, dp, p, out);
  if (s != GFD_OK) return s;
  if (!packed_in && (!weight || !att_src || !att_dst)) return GFD_ERR_ARGUMENT;
  Epi e{nullptr, 0, nullptr, 0};
  if (ep) {  // inference epilogue: no training statistics, no dropout
    if (!ep->scale_shift || stats || dp > 0.f) return GFD_ERR_ARGUMENT;
    if (ep->residual && ep->residual_stride < channels) return GFD_ERR_ARGUMENT;
    e = Epi{ep->scale_shift, ep->relu ? 1 : 0, ep->residual, ep->residual_stride};
    e.hw = ep->head_weight;
    e.hb = ep->head_bias;
    e.hout = ep->head_out;
    if (e.hout && !e.hw) return GFD_ERR_ARGUMENT;
  }
  if (ws_bytes < gfd_gat_fwd_workspace_size(N, N, F, heads, channels, p.num_hubs, p.num_chunks))
    return GFD_ERR_WORKSPACE;
  const PackLayout L = pack_layout(F);
  Carve c(ws, ws_bytes);
  AggArgs a{x, x_dtype, F, ldx, N, rowptr, col, N, 0, st, 16, st ? st + H : nullptr, 16, nullptr,
            bias, slope, dp, seed, p, GFD_STAGE_ALL, out, stats, nullptr, nullptr, nullptr, e};
  hub_ws_layout(&c, p.num_hubs, p.num_chunks, L, &a.part, &a.zhub);
  void* packed_ws = c.take<char>(L.bytes);
  const void* packed = packed_in ? packed_in : packed_ws;
  float* st_ws = c.take<float>(size_t(N) * 16);
  float* xmax = c.take<float>(1);
  if (!c.ok) return GFD_ERR_WORKSPACE;
  if (st == nullptr) st = st_ws;
  a.s = st;
  a.t = st + H;
  a.packed = static_cast<const char*>(packed);
  a.xmax = xmax;
  s = check_graph(rowptr, col, N, N, plan, nullptr, nullptr, nullptr, 0, stream);
  if (s != GFD_OK) return s;
  if (!packed_in) {
    s = gfd_gat_pack_weights(weight, att_src, att_dst, F, heads, channels, packed_ws, stream_);
    if (s != GFD_OK) return s;
  }
  if (hipMemsetAsync(xmax, 0, sizeof(float), stream) != hipSuccess) return GFD_ERR_HIP;
  if (lone_fusable(a, L)) {
    // the lone destinations' outputs come out of the logits pass; the tile
    // stage runs the general and light classes only
    s = launch_logits_lone(x, x_dtype, N, F, ldx, L, a.packed, rowptr, bias, slope, st, 16,
                           st + H, 16, xmax, out, stats, a.ep, stream);
    if (s != GFD_OK) return s;
    a.stages = GFD_STAGE_HUBS | GFD_STAGE_TILES_GENERAL | GFD_STAGE_TILES_LIGHT;
  } else {
    s = gfd_gat_logits_ex(x, x_dtype, N, F, ldx, packed, heads, channels, st, xmax, stream_);
    if (s != GFD_OK) return s;
  }
  return aggregate_impl(a, stream);
}

gfd_status gfd_gat_fwd_ep(const void* x, int x_dtype, int64_t N, int F, int64_t ldx,
                          const int32_t* rowptr, const int32_t* col, const float* weight,
                          const float* att_src, const float* att_dst, const float* bias,
                          int heads, int channels, float slope, float dp, uint64_t seed,
                          const gfd_plan* plan, const gfd_epilogue* ep, float* out, float* st,
                          float* stats, void* ws, size_t ws_bytes, gfd_stream_t stream_) {
  return fwd_ep_impl(x, x_dtype, N, F, ldx, rowptr, col, weight, att_src, att_dst, bias, heads,
                     channels, slope, dp, seed, plan, ep, out, st, stats, ws, ws_bytes, nullptr,
                     stream_);
}

gfd_status gfd_gat_fwd_ep_packed(const void* x, int x_dtype, int64_t N, int F, int64_t ldx,
                                 const int32_t* rowptr, const int32_t* col, const void* packed,
                                 const float* bias, int heads, int channels, float slope,
                                 float dp, uint64_t seed, const gfd_plan* plan,
                                 const gfd_epilogue* ep, float* out, float* st, float* stats,
                                 void* ws, size_t ws_bytes, gfd_stream_t stream_) {
  if (!packed) return GFD_ERR_ARGUMENT;
  return fwd_ep_impl(x, x_dtype, N, F, ldx, rowptr, col, nullptr, nullptr, nullptr, bias, heads,
                     channels, slope, dp, seed, plan, ep, out, st, stats, ws, ws_bytes, packed,
                     stream_);
}

gfd_status gfd_gat_fwd(const void* x, int x_dtype, int64_t N, int F, int64_t ldx,
                       const int32_t* rowptr, const int32_t* col, const float* weight,
                       const float* att_src, const float* att_dst, const float* bias, int heads,
                       int channels, float slope, float dp, uint64_t seed, const gfd_plan* plan,
                       float* out, float* st, float* stats, void* ws, size_t ws_bytes,
                       gfd_stream_t stream_) {
  return gfd_gat_fwd_ep(x, x_dtype, N, F, ldx, rowptr, col, weight, att_src, att_dst, bias, heads,
                        channels, slope, dp, seed, plan, nullptr, out, st, stats, ws, ws_bytes,
                        stream_);
}

}  // extern "C"
