// Host-side construction of a ChainSet: packing tables (weight element ->
// reference tensor element), activation-workspace layout, dW problem setup.
// Included by the per-configuration translation units.
#pragma once
#include <algorithm>
#include "chain.hip"
#include "chain_extern.h"
#include "chain_inst.h"
#include "dw_args.h"
#include "latent.hip"

namespace cn {

template <int SB>
constexpr int real_in_width(int L, int TB) {
  // reference input width of forward layer L (src/model.py:19-34)
  return L == 0 ? 63 : (L == SB + 2 ? 256 + 27 : (L == SB + TB + 4 ? 128 : 256));
}

inline int32_t src_idx(int tensor, int offset) { return (int32_t)(((uint32_t)tensor << 24) | (uint32_t)offset); }
// flag of a pack-table entry: store rn(w - rn(w)) (the W_lo of bf16x3), pack_kernel
constexpr int32_t kPackLo = 1 << 23;

template <int P, int SB, int TB, bool BWD>
std::vector<int32_t> build_pack_table() {
  using S = Sched<P, SB, TB, BWD>;
  using N = Net<SB, TB>;
  constexpr bool bf16 = P != CN_P_FP32;
  constexpr int EPL = S::elems_per_lane();
  std::vector<int32_t> tab((size_t)S::kChunks * kChunkBlocks * 64 * EPL, -1);
  for (int g = 0; g < S::kBlocks; ++g) {
    const int li = S::layer_of(g);
    const Layer l = S::L(li);
    const int lb = g - S::first_block(li);
    const int t = lb / S::bpt(li), kb = (lb % S::bpt(li)) / S::kAmul;
    const bool lo = (lb % S::bpt(li)) % S::kAmul == 1;     // bf16x3: the W_lo fragment
    for (int lane = 0; lane < 64; ++lane) {
      const int n = lane & 31, h = lane >> 5;
      const int row = 32 * t + n;
      for (int e = 0; e < EPL; ++e) {
        int32_t v = -1;
        if (!BWD) {
          const int in_real = real_in_width<SB>(li, TB);
          const int out_real = li == N::kFwdLayers - 1 ? 3 : l.T * 32;
          int f = -1;
          if (bf16) {
            const int q = kb, j = e;
            if (l.in_kind == IN_PE) f = pe_slot_feature(h, 8 * q + j);
            else if (l.in_kind == IN_ACC_DIR && q >= 16) {
              const int d = dir_slot_feature(h, 8 * (q - 16) + j);
              f = d < 0 ? -1 : 256 + d;
            } else f = bf16_acc_feature(q, h, j);
          } else {
            const int q = 4 * kb + e;
            if (l.in_kind == IN_PE) f = pe_slot_feature(h, q);
            else if (l.in_kind == IN_ACC_DIR && q >= 128) {
              const int d = dir_slot_feature(h, q - 128);
              f = d < 0 ? -1 : 256 + d;
            } else f = f32_acc_feature(q, h);
          }
          if (f >= 0 && f < in_real && row < out_real) v = src_idx(l.w, row * in_real + f);
        } else {
          // transposed: output row = forward input feature, k = forward output feature
          const int fl = li == 0 ? N::kFwdLayers - 1 : N::kFwdLayers - 1 - li;
          const int in_f = real_in_width<SB>(fl, TB);
          const int out_f = fl == N::kFwdLayers - 1 ? 3 : N::fwd(fl).T * 32;
          int kf;
          if (li == 0) kf = bf16 ? 8 * h + e : 2 * (4 * kb + e) + h;   // drgb component
          else kf = bf16 ? bf16_acc_feature(kb, h, e) : f32_acc_feature(4 * kb + e, h);
          if (kf < out_f && row < in_f) v = src_idx(l.w, kf * in_f + row);
        }
        tab[((size_t)g * 64 + lane) * EPL + e] = (v >= 0 && lo) ? (v | kPackLo) : v;
      }
    }
  }
  return tab;
}

template <int P, int SB, int TB>
ActLayout act_layout(size_t Mp) {
  using N = Net<SB, TB>;
  const size_t es = P != CN_P_FP32 ? 2 : 4;
  ActLayout L;
  size_t off = 0;
  auto take = [&](size_t n) { size_t o = off; off += (n + 255) & ~(size_t)255; return o; };
  L.pe = take(Mp * 64 * es);
  L.dir = take(Mp * 32 * es);
  // planes the kernels do not write (N::stored) take no space: width 0
  for (int p = 0; p < N::kPlanes; ++p) {
    L.Yw[p] = N::stored(p) ? N::plane_width(p) : 0;
    L.Y[p] = take(Mp * L.Yw[p] * es);
  }
  for (int p = 0; p < N::kPlanes; ++p) {
    L.dAw[p] = N::stored(p) ? N::dplane_width(p) : 0;
    L.dA[p] = take(Mp * L.dAw[p] * es);
  }
  L.d8 = take(Mp * 32 * es);
  L.spre = take(Mp * 4);
  L.mask_bytes_per_slab = (size_t)N::kMasks * 64 * 16;
  L.masks = take(Mp / 32 * L.mask_bytes_per_slab);
  if constexpr (P == CN_P_BF16X3) {
    // the X operands' lo parts, after everything else (the planes above keep
    // their offsets in every precision)
    L.pelo = take(Mp * 64 * es);
    for (int p = 0; p < N::kPlanes; ++p) L.Ylo[p] = L.Yw[p] ? take(Mp * L.Yw[p] * es) : 0;
  }
  L.bytes = off;
  return L;
}

// dW schedule for M samples: nwg persistent workgroups (default kDwWorkgroups,
// one per CU) each take an equal byte share of the (layer, slab) stream.
// Fewer workgroups leave CUs to a dX chain running beside the dW pass.
constexpr int kDwWorkgroups = 256;

constexpr size_t dw_part_bytes() {
  return (size_t)kDwWorkgroups * 2 * ((size_t)kPartRows * kPartCols + kPartRows) * sizeof(float);
}

// The schedule's unit is a slab's COST (DwArgs::wprefix / pbytes).  bf16 dW
// is HBM-bound: cost = operand bytes.  The exact-fp32 pass is MFMA-bound and
// its bodies differ 16x in MFMAs per byte (DW_VIEWDIR 1,280 v_mfma_f32_32x32x2
// per 72 KiB slab, DW_RGB2 64 per 20 KiB), so equal byte shares left the
// workgroups holding viewdir / 256x256 slabs ~1.25x the mean while the
// others idled: cost = CU cycles, max(MFMA cycles over 4 SIMDs -- 64 per
// MFMA --, bytes at ~9 B per CU-cycle of HBM) + a barrier's ~512.
constexpr int dw_f32_slab_cost(int kind, int bytes) {
  const int mfma = kind == DW_FULL ? 1024 : kind == DW_PE ? 256 : kind == DW_VIEWDIR ? 1280
                 : kind == DW_RGB0 ? 512 : 64;                 // per slab, all waves (dw.hip DwShape)
  const int mc = mfma * 16, bc = bytes / 9;
  return (mc > bc ? mc : bc) + 512;
}

template <int P, int SB, int TB>
size_t dw_ws_bytes(int) {
  return dw_part_bytes() + (size_t)kFoldRows * kFoldCols * sizeof(float);   // + the fold operand Gx
}

// Rows [row0, row0 + pad(M)) of a workspace laid out for act_M samples
// (row0 a multiple of 256): the coarse and fine row ranges of one step can
// then be reduced by two launches, each overlapping the other range's dX chain.
template <int P, int SB, int TB>
int dw_setup_cost(char* act, int act_M, int row0, int M, int nwg_req, const float* zvec, float* dbuf, char* ws,
                  DwArgs* dw, DwRedArgs* red, bool cost) {
  using N = Net<SB, TB>;
  constexpr ParamIdx PI{SB, TB};
  constexpr int ES = P != CN_P_FP32 ? 2 : 4;
  const int Mp = ((M + 255) / 256) * 256;
  const int Ma = ((act_M + 255) / 256) * 256;
  if (row0 < 0 || row0 % 256 || row0 + Mp > Ma) return -1;
  const ActLayout A = act_layout<P, SB, TB>(Ma);
  const size_t r0 = (size_t)row0 * ES;      // byte offset per element of plane width
  static_assert(N::kFwdLayers - 1 <= kDwMaxProblems, "dw problems");
  static_assert(!N::stored(SB + 1) && N::stored(SB), "the fold assumes encoding_shape's planes are the unstored ones");
  *dw = DwArgs{};
  *red = DwRedArgs{};
  // one problem per forward layer except encoding_shape (L = SB + 1), whose
  // gradients come out of the viewdir problem's fold (dw_fold_kernel)
  constexpr int NP = N::kFwdLayers - 1;
  auto layer_of = [](int k) { return k <= SB ? k : k + 1; };
  dw->nprob = red->nprob = NP;
  dw->total_tiles = Mp / 32;
  int ep = 0;
  long long wsum = 0, min_total = -1;
  for (int k = 0; k < NP; ++k) {
    const int L = layer_of(k);
    const bool last = L == N::kFwdLayers - 1;
    const bool vd = L == SB + 2;
    DwProblem& p = dw->p[k];
    p.a_width = last ? 32 : N::dplane_width(L);
    p.A = act + (last ? A.d8 : A.dA[L]) + r0 * p.a_width;
    p.a_tiles = p.a_width / 32;
    p.out_tiles = last ? 1 : N::fwd(L).T;
    // viewdir: X = Y of the last shape layer (encoding_shape's INPUT), the fold
    // maps the accumulated dA_viewdir (x) Y_shape through encoding_shape
    const int xin = vd ? SB : L - 1;
    if (L == 0) { p.X0 = act + A.pe + r0 * 64; p.x0_width = 64; }
    else { p.x0_width = N::plane_width(xin); p.X0 = act + A.Y[xin] + r0 * p.x0_width; }
    p.x0_tiles = p.x0_width / 32;
    if (vd) { p.X1 = act + A.dir + r0 * 32; p.x1_width = 32; p.x1_tiles = 1; }
    // bf16x3: X0's lo parts (the training forward stored them, act_layout)
    const size_t lo_off = L == 0 ? A.pelo : A.Ylo[xin];
    if (lo_off) {
      p.X0lo = act + lo_off + r0 * p.x0_width;
      p.lo = 1;
    }
    p.sigma_head = vd ? 1 : 0;
    p.kind = L == 0 ? DW_PE : vd ? DW_VIEWDIR : last ? DW_RGB2 : (L == N::kFwdLayers - 2 ? DW_RGB0 : DW_FULL);
    {
      // the bf16 bodies are compiled for exactly these operand shapes
      static constexpr int shape[5][4] = {{8, 8, 0, 8}, {8, 2, 0, 8}, {9, 8, 1, 8}, {4, 8, 0, 4}, {1, 4, 0, 1}};
      const int* e = shape[p.kind];
      if (p.a_tiles != e[0] || p.x0_tiles != e[1] || p.x1_tiles != e[2] || p.out_tiles != e[3]) return -1;
    }
    dw->pbytes[k] = (p.a_tiles + p.x0_tiles * (1 + p.lo) + p.x1_tiles) * 1024 * ES;
    if (cost) dw->pbytes[k] = dw_f32_slab_cost(p.kind, dw->pbytes[k]);
    dw->wprefix[k] = wsum;
    const long long tot = (long long)dw->pbytes[k] * dw->total_tiles;
    wsum += tot;
    if (min_total < 0 || tot < min_total) min_total = tot;

    DwRedProblem& r = red->p[k];
    r.out_real = last ? 3 : N::fwd(L).T * 32;
    r.in_real = real_in_width<SB>(L, TB);
    r.cols = (p.x0_tiles + p.x1_tiles) * 32;
    r.map = L == 0 ? MAP_PE : (vd ? MAP_VIEWDIR : MAP_PLAIN);
    r.w = N::fwd(L).w;
    r.b = N::fwd(L).b;
    r.w2 = PI.sigma_w();
    r.b2 = PI.sigma_w() + 1;
    const int inj = L >= 1 ? N::fwd(L - 1).inj : -1;
    r.z = inj >= 0 ? zvec + inj * 256 : nullptr;
    r.dbout = inj >= 0 ? dbuf + inj * 256 : nullptr;
    r.elems = (r.out_real + (vd ? 1 : 0)) * r.cols;
    r.pbytes = dw->pbytes[k];
    red->prefix[k] = ep;
    ep += r.elems;
    red->wprefix[k] = dw->wprefix[k];
  }
  dw->wprefix[NP] = red->wprefix[NP] = wsum;
  red->prefix[NP] = ep;
  // a share (wsum / nwg bytes) never exceeds the smallest problem, so it
  // holds slabs of at most two problems; and it spans at least
  // 1.5 slabs of the largest, so every workgroup between a problem's first
  // and last holds some of its slabs (the reduction sums exactly those
  // workgroups' partials: small M runs fewer workgroups instead of leaving
  // empty ones in between)
  long long max_pbytes = 0;
  for (int k = 0; k < NP; ++k) max_pbytes = std::max<long long>(max_pbytes, dw->pbytes[k]);
  long long nwg = nwg_req > 0 ? std::min(nwg_req, kDwWorkgroups) : kDwWorkgroups;
  nwg = std::min(nwg, std::max(1LL, 2 * wsum / (3 * max_pbytes)));
  if ((wsum + min_total - 1) / min_total >= nwg) return -1;
  dw->nwg = red->nwg = (int)nwg;
  // which partial slots hold each problem (the kernel's own segment walk)
  for (int k = 0; k < NP; ++k) red->gfirst[k] = -1;
  for (int g = 0; g < (int)nwg; ++g) {
    const long long b0 = dw_share_begin(g, wsum, (int)nwg), b1 = dw_share_begin(g + 1, wsum, (int)nwg);
    int seg = 0;
    for (int k = 0; k < NP && seg < 2; ++k) {
      int t0, t1;
      dw_slab_range(dw->wprefix, dw->pbytes, dw->total_tiles, k, b0, b1, t0, t1);
      if (t1 <= t0) continue;
      if (red->gfirst[k] < 0) { red->gfirst[k] = g; red->gseg[k] = seg; }
      else if (seg != 0) return -1;      // only a problem's first workgroup may hold it second
      red->glast[k] = g;
      ++seg;
    }
  }
  for (int k = 0; k < NP; ++k)
    if (red->gfirst[k] < 0) return -1;
  dw->part = (float*)ws;
  dw->dbpart = (float*)(ws + (size_t)kDwWorkgroups * 2 * kPartRows * kPartCols * sizeof(float));
  red->part = dw->part;
  red->dbpart = dw->dbpart;
  red->fold = (float*)(ws + dw_part_bytes());
  return (int)nwg;
}

// fp32: MFMA-cost shares (dw_f32_slab_cost); a small call whose cost shares
// cannot satisfy the segment rules above (a share larger than the cheapest
// problem) falls back to byte shares
template <int P, int SB, int TB>
int dw_setup(char* act, int act_M, int row0, int M, int nwg_req, const float* zvec, float* dbuf, char* ws,
             DwArgs* dw, DwRedArgs* red) {
  if constexpr (P == CN_P_FP32) {
    const int n = dw_setup_cost<P, SB, TB>(act, act_M, row0, M, nwg_req, zvec, dbuf, ws, dw, red, true);
    if (n > 0) return n;
  }
  return dw_setup_cost<P, SB, TB>(act, act_M, row0, M, nwg_req, zvec, dbuf, ws, dw, red, false);
}

// The encoding_shape fold (see Net::stored): the viewdir problem accumulates
// Gx[n][k] = sum_m dA_vd[m][n] * Y_s[m][k] with Y_s the last shape layer's
// output (n < 256: viewdir rows, n = 256: the sigma head), plus column
// k = 256 = sum_m dA_vd[m][n] (the bias gradients).  encoding_shape is
// Y_e = W_e Y_s + b_e, so with Wx_e = [W_e | b_e] (256 x 257) and
// Wx_v[n][f] = W_v[n][f] (n < 256, the y columns of encoding_viewdir) or
// w_sigma[f] (n = 256):
//   d[W_v y-part ; w_sigma][n][f] = sum_k Gx[n][k] Wx_e[f][k]
//   d[W_e | b_e][f][k]            = sum_n Wx_v[n][f] Gx[n][k]
template <int SB, int TB>
DwFoldArgs fold_args() {
  constexpr ParamIdx PI{SB, TB};
  DwFoldArgs f{};
  f.w_shape = PI.enc_shape_w();
  f.w_view = PI.viewdir_w();
  f.view_cols = real_in_width<SB>(SB + 2, TB);
  f.w_sigma = PI.sigma_w();
  return f;
}

template <int P, int SB, int TB>
int db_setup(char* act, int act_M, int M, float* dbuf, char* ws, DbArgs* db) {
  // rows [0, pad(M)) of a workspace laid out for act_M samples
  using N = Net<SB, TB>;
  const int Mp = ((M + 255) / 256) * 256;
  const int Ma = ((act_M + 255) / 256) * 256;
  if (Mp > Ma) return -1;
  const ActLayout A = act_layout<P, SB, TB>(Ma);
  static_assert(N::kInject <= kDbMaxInject, "injections");
  *db = DbArgs{};
  db->total_slabs = Mp / 32;
  db->slabs_per_blk = (db->total_slabs + kDbBlocks - 1) / kDbBlocks;
  int n = 0;
  for (int L = 1; L < N::kFwdLayers; ++L) {
    const int inj = N::fwd(L - 1).inj;
    if (inj < 0) continue;
    db->A[inj] = act + A.dA[L];
    db->a_width[inj] = N::dplane_width(L);
    if (db->a_width[inj] != 256) return -1;     // db_kernel streams 256-wide planes
    ++n;
  }
  db->ninj = n;
  db->part = (float*)ws;
  db->dbout = dbuf;
  return n;
}

template <int P, int SB, int TB>
ChainSet make_chain_set() {
  using N = Net<SB, TB>;
  // bf16: 8-wave workgroups (two waves per SIMD, one workgroup per CU) by
  // default; fp32 (bin operand of 144 VGPRs) and bf16x3 (hi + lo operands,
  // 2 x 72 VGPRs, beside 128 accumulator registers): 4 waves, one per SIMD
  // (round 5 measured a 16-sample, two-waves-per-SIMD bf16x3 layout and kept
  // this one: DESIGN.md section 7, Round 5)
  constexpr int WF = P == CN_P_BF16 ? 8 : 4;
  constexpr int WB = P == CN_P_BF16 ? 8 : 4;
  ChainSet s;
  s.prec = P != CN_P_FP32;     // activation-plane element type: 1 = bf16 (bf16, bf16x3)
  s.x3 = P == CN_P_BF16X3;
  s.SB = SB;
  s.TB = TB;
  s.waves_fwd = WF;
  s.waves_bwd = WB;
  s.tile = 256;
  s.n_params = ParamIdx{SB, TB}.count();
  s.n_inject = N::kInject;
  s.n_fwd_layers = N::kFwdLayers;
  s.blob_floats = BiasBlob<SB, TB>::kFloats;
  s.pack_fwd_bytes = Sched<P, SB, TB, false>::packed_bytes();
  s.pack_bwd_bytes = Sched<P, SB, TB, true>::packed_bytes();
  s.fwd_train = chain_kernel<P, SB, TB, false, WF, CN_MODE_TRAIN>;
  s.fwd_infer = chain_kernel<P, SB, TB, false, WF, CN_MODE_INFER>;
  s.fwd_codes = chain_kernel<P, SB, TB, false, WF, CN_MODE_CODES>;
  s.bwd = chain_kernel<P, SB, TB, true, WB, CN_MODE_TRAIN>;
  s.bwd_codes = chain_kernel<P, SB, TB, true, WB, CN_MODE_CODES>;
  s.fwd_table = build_pack_table<P, SB, TB, false>;
  s.bwd_table = build_pack_table<P, SB, TB, true>;
  s.latent_fwd = latent_fwd_kernel<SB, TB>;
  s.latent_bwd = latent_bwd_kernel<SB, TB>;
  s.code_grad = code_grad_kernel<SB, TB>;
  s.layout = act_layout<P, SB, TB>;
  s.dw_setup = dw_setup<P, SB, TB>;
  s.dw_ws_bytes = dw_ws_bytes<P, SB, TB>;
  s.fold_args = fold_args<SB, TB>;
  s.db_setup = db_setup<P, SB, TB>;
  return s;
}

// CN_P_BF16X3F: the bf16x3 forward chains (rgb within ~5e-7 of the fp32
// reference) with the CN_P_BF16 backward: the training forward stores the hi
// planes only (CN_MODE_TRAIN_HI -- exactly the bf16 plan's planes: the same
// layout, masks and rounding rn(x)), which the bf16 dX chain (8 waves) and the
// bf16 dW pass read.  Weight packs: forward = bf16x3 (W_hi, W_lo fragments),
// backward = bf16.
template <int SB, int TB>
ChainSet make_chain_set_x3f() {
  using N = Net<SB, TB>;
  constexpr int X3 = CN_P_BF16X3, B16 = CN_P_BF16;
  ChainSet s;
  s.prec = 1;                 // bf16 planes and dW
  s.x3 = 1;                   // forward chains in bf16x3
  s.SB = SB;
  s.TB = TB;
  s.waves_fwd = 4;            // as the bf16x3 plan
  s.waves_bwd = 8;            // as the bf16 plan
  s.tile = 256;
  s.n_params = ParamIdx{SB, TB}.count();
  s.n_inject = N::kInject;
  s.n_fwd_layers = N::kFwdLayers;
  s.blob_floats = BiasBlob<SB, TB>::kFloats;
  s.pack_fwd_bytes = Sched<X3, SB, TB, false>::packed_bytes();
  s.pack_bwd_bytes = Sched<B16, SB, TB, true>::packed_bytes();
  s.fwd_train = chain_kernel<X3, SB, TB, false, 4, CN_MODE_TRAIN_HI>;
  s.fwd_infer = chain_kernel<X3, SB, TB, false, 4, CN_MODE_INFER>;
  s.fwd_codes = chain_kernel<X3, SB, TB, false, 4, CN_MODE_CODES>;
  s.bwd = chain_kernel<B16, SB, TB, true, 8, CN_MODE_TRAIN>;
  s.bwd_codes = chain_kernel<B16, SB, TB, true, 8, CN_MODE_CODES>;
  s.fwd_table = build_pack_table<X3, SB, TB, false>;
  s.bwd_table = build_pack_table<B16, SB, TB, true>;
  s.latent_fwd = latent_fwd_kernel<SB, TB>;
  s.latent_bwd = latent_bwd_kernel<SB, TB>;
  s.code_grad = code_grad_kernel<SB, TB>;
  s.layout = act_layout<B16, SB, TB>;
  s.dw_setup = dw_setup<B16, SB, TB>;
  s.dw_ws_bytes = dw_ws_bytes<B16, SB, TB>;
  s.fold_args = fold_args<SB, TB>;
  s.db_setup = db_setup<B16, SB, TB>;
  return s;
}

}  // namespace cn
