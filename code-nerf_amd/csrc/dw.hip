// Weight gradients of the CodeNeRF MLP: dW_L = sum_m dA_L[m] (x) X_L[m].
//
// The reduction runs over samples (K = M ~ 2e6): a persistent workgroup (one
// per CU) owns the WHOLE (<= 288 x 288) gradient of one layer over one
// byte-balanced slice of the (layer, slab) stream, so every operand byte is
// read from HBM exactly once.  This pass is HBM-bound: 8,000 B of bf16
// operands per sample against 0.9 MFLOP.  A 32-sample slab of a plane is one
// contiguous run (cn_layout.h); it lands in LDS unchanged and is read back
// transposed.
//   bf16 (DwBf16<KIND>): one compile-time body per operand shape (DwKind),
//     4-slot LDS-DMA ring (three slabs in flight while one is consumed),
//     ds_read_b64_tr_b16 (conflict-free by the pair-block rotation) feeding
//     v_mfma_f32_32x32x16_bf16; the sigma head (ds x y_shape) is an extra
//     MFMA tile of the viewdir body;
//   fp32 (DwF32): exact fp32 parity path, register-staged double buffer,
//     ds_read_b32 + v_mfma_f32_32x32x2_f32.
// Bias gradients (row sums of dA) come from the A fragments.  Workgroups write
// fp32 partials; dw_reduce sums them (deterministic, no atomics), maps padded /
// permuted columns back to the reference tensors, adds the code-injection
// correction db (x) z and accumulates into .grad.
#include "cn_common.h"
#include "chain_args.h"
#include "dw_args.h"

namespace cn {

typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <int ES>
CN_DEV int img_off(int s, int f) {
  // byte offset, inside a staged slab image, of features f..f+3 of sample s
  return slab_off(s, f, ES);
}

// ------------------------------------------------------------ fp32 body
// The exact-fp32 parity path: one generic body for every operand shape (the
// shape is read from the problem at run time), slabs staged through
// registers into a double-buffered LDS image, v_mfma_f32_32x32x2_f32 with
// K = samples.  8 waves: wave w owns rows 64 (w >> 1) .. +63 and columns
// 128 (w & 1) .. +127 (+ the 9th, dir-PE, column tile on the (w & 1) == 0
// waves); the sigma head (ds x y_shape) is a VALU side product.
struct DwF32 {
  static constexpr int ES = 4;
  static constexpr int kTileB = 1024 * ES;                // one 32-sample x 32-feature tile
  static constexpr int kStage = 18 * kTileB;              // A (<= 9 tiles) + X (<= 9 tiles)
  static constexpr int kLoads = 9;                        // 16-B pieces per thread per slab
  static constexpr int kSmem = 2 * kStage;

  __device__ static void run(const DwProblem& pr, int t0, int t1, int rot, float* part, float* dbpart, char* smem) {
    const int nst = t1 - t0;
    // slab visited at step st: rotated so that the workgroups streaming one
    // plane do not walk it in lockstep (HBM channel camping); the sum does
    // not depend on the order.
    rot %= nst;
    auto slab = [&](int st) { const int t = st + rot; return t0 + (t >= nst ? t - nst : t); };
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wo = w >> 1, wi = w & 1;
    const int h = lane >> 5;
    const int xt = pr.x0_tiles + pr.x1_tiles;
    const bool extra = (wi == 0) && xt > 8;
    const int a_bytes = pr.a_tiles * kTileB;
    const int x0_bytes = pr.x0_tiles * kTileB;
    const int x1_bytes = pr.x1_tiles * kTileB;
    const int stage_pieces = (a_bytes + x0_bytes + x1_bytes) >> 4;
    const bool row0_live = 64 * wo < pr.out_tiles * 32;
    const bool row1_live = 64 * wo + 32 < pr.out_tiles * 32;
    const bool cols_live = 128 * wi < min(xt, 8) * 32;
    const bool live = row0_live && (cols_live || extra);
    const bool sigma_head = pr.sigma_head;

    f32x16 acc[2][5];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j) acc[i][j] = f32x16{};
    float dbacc[2] = {0.f, 0.f};
    float sg = 0.f, sgb = 0.f;                   // sigma head: ds x y (feature tid & 255), sum ds

    const char* pa0 = (const char*)pr.A;
    const char* p00 = (const char*)pr.X0;
    const char* p10 = pr.X1 ? (const char*)pr.X1 : p00;
    auto src_of = [&](int tile, int b) -> const char* {
      // byte b of the slab of wave tile `tile`: [A tiles | X0 tiles | X1 tiles]
      if (b < a_bytes) return pa0 + (size_t)tile * pr.a_width * 32 * ES + b;
      if (b < a_bytes + x0_bytes) return p00 + (size_t)tile * pr.x0_width * 32 * ES + (b - a_bytes);
      return p10 + (size_t)tile * pr.x1_width * 32 * ES + (b - a_bytes - x0_bytes);
    };
    u32x4 rg[kLoads];
    auto gload = [&](int tile) {
#pragma unroll
      for (int k = 0; k < kLoads; ++k) {
        const int b = (threadIdx.x + 512 * k) << 4;
        rg[k] = (threadIdx.x + 512 * k) < stage_pieces ? *(const u32x4*)src_of(tile, b) : u32x4{};
      }
    };
    auto lstore = [&](int buf) {
      char* dst = smem + buf * kStage;
#pragma unroll
      for (int k = 0; k < kLoads; ++k)
        if ((threadIdx.x + 512 * k) < stage_pieces) *(u32x4*)(dst + ((threadIdx.x + 512 * k) << 4)) = rg[k];
    };

    gload(slab(0));
    lstore(0);
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
      if (st + 1 < nst) gload(slab(st + 1));
      const char* A = smem + (st & 1) * kStage;
      const char* X = A + a_bytes;
      if (live) {
        const int c = lane & 31;
#pragma unroll 4
        for (int q = 0; q < 16; ++q) {
          const int s = 2 * q + h;
          float fa[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int f = 64 * wo + 32 * i + c;
            fa[i] = *(const float*)(A + img_off<ES>(s, f & ~3) + (f & 3) * 4);
            dbacc[i] += fa[i];
          }
#pragma unroll
          for (int j = 0; j < 5; ++j) {
            if (j < 4 ? !cols_live : !extra) continue;
            const int f = (j < 4 ? 128 * wi + 32 * j : 256) + c;
            const float fx = *(const float*)(X + img_off<ES>(s, f & ~3) + (f & 3) * 4);
            acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[0], fx, acc[0][j], 0, 0, 0);
            if (row1_live) acc[1][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[1], fx, acc[1][j], 0, 0, 0);
          }
        }
      }
      if (sigma_head) {
        // d w_sigma[f] += sum_s ds[s] * y[s][f];  ds = A[s][256] + A[s][257]
        const int f = threadIdx.x & 255;
        const int s0 = (threadIdx.x >> 8) * 16;
#pragma unroll 4
        for (int s = s0; s < s0 + 16; ++s) {
          const float* dsp = (const float*)(A + img_off<ES>(s, 256));
          const float ds = dsp[0] + dsp[1];
          const float y = ((const float*)(X + img_off<ES>(s, f & ~3)))[f & 3];
          sg = __builtin_fmaf(ds, y, sg);
          sgb += ds;
        }
      }
      if (st + 1 < nst) lstore((st + 1) & 1);
      __syncthreads();
    }

    // ---- fp32 partial: row n (out feature), column c (in feature)
    if (live) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if (i == 1 && !row1_live) continue;
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          if (j < 4 ? !cols_live : !extra) continue;
          const int col = (j < 4 ? 128 * wi + 32 * j : 256) + (lane & 31);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = 64 * wo + 32 * i + acc_row(r, h);
            part[(size_t)row * kPartCols + col] = acc[i][j][r];
          }
        }
      }
    }
    if (wi == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float tot = dbacc[i] + __shfl_xor(dbacc[i], 32);
        const bool rl = i == 0 ? row0_live : row1_live;
        if (h == 0 && rl) dbpart[64 * wo + 32 * i + (lane & 31)] = tot;
      }
    }
    if (sigma_head) {
      // combine the two sample halves through LDS (the staging buffers are free now)
      float* red = (float*)smem;
      red[threadIdx.x] = sg;
      red[512 + threadIdx.x] = sgb;
      __syncthreads();
      if (threadIdx.x < 256) {
        part[(size_t)256 * kPartCols + threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + 256];
        if (threadIdx.x == 0) dbpart[256] = red[512] + red[512 + 256];
      }
    }
    __syncthreads();
  }
};

// ------------------------------------------------------------ bf16 bodies
// One compile-time body per operand shape (DwKind): every wave's tiles, LDS
// reads, MFMAs and piece counts are constants, so the slab loop has no
// runtime branches beyond wave-uniform role tests.  Staging: a 4-slot LDS-DMA
// ring of 36 KiB slots, three slabs in flight while the fourth is consumed.
template <int KIND> struct DwShape;
//                                      A tiles, X0, X1, row tiles/wave, col tiles/wave
template <> struct DwShape<DW_FULL>    { static constexpr int kA = 8, kX0 = 8, kX1 = 0, NI = 2, NJ = 4; };
template <> struct DwShape<DW_PE>      { static constexpr int kA = 8, kX0 = 2, kX1 = 0, NI = 1, NJ = 2; };
template <> struct DwShape<DW_VIEWDIR> { static constexpr int kA = 9, kX0 = 8, kX1 = 1, NI = 2, NJ = 4; };
template <> struct DwShape<DW_RGB0>    { static constexpr int kA = 4, kX0 = 8, kX1 = 0, NI = 2, NJ = 2; };
template <> struct DwShape<DW_RGB2>    { static constexpr int kA = 1, kX0 = 4, kX1 = 0, NI = 1, NJ = 1; };

// LDS ring per shape: 256x256 slabs (32 KiB stages, no padding pieces) and
// the other shapes (36 KiB = the viewdir stage, + an 8 KiB landing area for
// padding pieces) both keep 4 slots, 3 slabs in flight: a 5-slot ring for the
// 256x256 bodies measured 0.2 ms slower per C2 step.
constexpr int kDwSmemBf16 = 160 * 1024;

template <int KIND>
struct DwBf16 {
  using Sh = DwShape<KIND>;
  static constexpr int kA = Sh::kA, kX0 = Sh::kX0, kX1 = Sh::kX1, NI = Sh::NI, NJ = Sh::NJ;
  static constexpr int kPieces = 2 * (kA + kX0 + kX1);     // 1 KiB pieces per slab
  static constexpr int kG = (kPieces + 7) / 8;              // pieces per wave per slab
  static constexpr bool kVD = KIND == DW_VIEWDIR;
#ifndef CN_DW_RING_FULL
#define CN_DW_RING_FULL 4
#endif
  static constexpr int kDwSlot = KIND == DW_FULL ? 32 * 1024 : 36 * 1024;
  static constexpr int kDwRing = KIND == DW_FULL ? CN_DW_RING_FULL : 4;
  static constexpr int kDwDepth = kDwRing - 1;        // slabs in flight while one is consumed
  static constexpr int kDwDummy = kDwRing * kDwSlot;  // landing area of padding pieces
  static_assert(kPieces * 1024 <= kDwSlot, "dw stage");
  static_assert(kDwDummy + (8 * kG - kPieces) * 1024 <= kDwSmemBf16, "dw LDS");

  // wave w's row tile i / column tile j (wave-uniform)
  static CN_DEV int row_tile(int w, int i) {
    if constexpr (KIND == DW_FULL || KIND == DW_VIEWDIR) return 2 * (w >> 1) + i;
    else if constexpr (KIND == DW_PE) return w;
    else if constexpr (KIND == DW_RGB0) return 2 * (w >> 2) + i;
    else return 0;
  }
  static CN_DEV int col_tile(int w, int j) {
    if constexpr (KIND == DW_FULL || KIND == DW_VIEWDIR) return 4 * (w & 1) + j;
    else if constexpr (KIND == DW_PE) return j;
    else if constexpr (KIND == DW_RGB0) return 2 * (w & 3) + j;
    else return w;
  }
  static CN_DEV bool wave_live(int w) { return KIND != DW_RGB2 || w < 4; }
  // the one wave per row tile that also sums the bias gradient (row sums of A)
  static CN_DEV bool wave_db(int w) {
    if constexpr (KIND == DW_FULL || KIND == DW_VIEWDIR) return (w & 1) == 0;
    else if constexpr (KIND == DW_PE) return true;
    else if constexpr (KIND == DW_RGB0) return (w & 3) == 0;
    else return w == 0;
  }

  __device__ static void run(const DwProblem& pr, int t0, int t1, int rot, float* part, float* dbpart, char* smem) {
    const int nst = t1 - t0;
    rot %= nst;
    auto slab = [&](int st) { const int t = st + rot; return t0 + (t >= nst ? t - nst : t); };
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int h = lane >> 5;
    const bool live = wave_live(w);
    const bool do_db = wave_db(w);

    f32x16 acc[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x16{};
    f32x16 acc_e1 = f32x16{}, acc_e2 = f32x16{};     // viewdir: (row w, dir tile), (sigma tile, col)
    float dbacc[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) dbacc[i] = 0.f;
    float dbsig = 0.f;

    const char* pa = (const char*)pr.A;
    const char* px0 = (const char*)pr.X0;
    const char* px1 = kX1 ? (const char*)pr.X1 : px0;
    auto issue = [&](int st, auto slotc) {
      const size_t t = (size_t)slab(st);
#pragma unroll
      for (int k = 0; k < kG; ++k) {
        const int piece = w * kG + k;            // wave-uniform
        const char* src;
        uint32_t dst = lds_addr(smem + decltype(slotc)::value * kDwSlot + piece * 1024);
        if (piece < 2 * kA) src = pa + t * (kA * 2048) + piece * 1024;
        else if (piece < 2 * (kA + kX0)) src = px0 + t * (kX0 * 2048) + (piece - 2 * kA) * 1024;
        else if (piece < kPieces) src = px1 + t * (kX1 * 2048) + (piece - 2 * (kA + kX0)) * 1024;
        else {
          src = pa + t * (kA * 2048);            // padding piece: re-read, never consumed
          dst = lds_addr(smem + kDwDummy + (piece - kPieces) * 1024);
        }
        glds16_opaque(src + lane * 16, dst);
      }
    };
    static_for<0, kDwDepth>([&](auto i) {
      if (i < nst) issue(i, i);
    });

    const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    auto frag = [&](const char* base, int tile, int s) -> bf16x8 {
      const int f = 32 * tile + 16 * (G & 1) + 4 * p;
      s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + img_off<2>(s, f)));
      s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + img_off<2>(s + 4, f)));
      return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    auto rowsum = [](bf16x8 v) {
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += (float)v[j];
      return sum;
    };

    auto body = [&](int st, auto slotc) {
      constexpr int SL = decltype(slotc)::value;
      const int ahead = min(kDwDepth - 1, nst - 1 - st);
      static_for<0, kDwDepth>([&](auto n) {
        if (n == ahead) wait_vmcnt<n * kG>();
      });
      block_barrier();
      if (st + kDwDepth < nst) issue(st + kDwDepth, std::integral_constant<int, (SL + kDwDepth) % kDwRing>{});
      const char* A = smem + SL * kDwSlot;
      const char* X = A + kA * 2048;
      if (!live) return;
#pragma unroll
      for (int kk = 0; kk < 32; kk += 16) {
        const int s = kk + 8 * h + q;
        bf16x8 fa[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          fa[i] = frag(A, row_tile(w, i), s);
          if (do_db) dbacc[i] += rowsum(fa[i]);
        }
        bf16x8 fs{};
        if constexpr (kVD) {
          fs = frag(A, 8, s);                    // sigma-head columns 256.. of the dA plane
          if (w == 0) dbsig += rowsum(fs);
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const bf16x8 fx = frag(X, col_tile(w, j), s);
#pragma unroll
          for (int i = 0; i < NI; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fx, acc[i][j], 0, 0, 0);
          if constexpr (kVD) {
            if (j == (w >> 1)) acc_e2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fs, fx, acc_e2, 0, 0, 0);
          }
        }
        if constexpr (kVD) {
          const bf16x8 fd = frag(X, 8, s);       // dir-PE input tile
          const bf16x8 fr = (w & 1) ? fa[1] : fa[0];
          acc_e1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr, fd, acc_e1, 0, 0, 0);
        }
      }
    };
    for (int base = 0; base < nst; base += kDwRing)
      static_for<0, kDwRing>([&](auto k) {
        if (base + k < nst) body(base + k, k);
      });
    __syncthreads();

    // ---- fp32 partial: row n (out feature), column c (in feature)
    if (live) {
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int col = 32 * col_tile(w, j) + (lane & 31);
#pragma unroll
          for (int r = 0; r < 16; ++r)
            part[(size_t)(32 * row_tile(w, i) + acc_row(r, h)) * kPartCols + col] = acc[i][j][r];
        }
      if constexpr (kVD) {
        const int col = 256 + (lane & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) part[(size_t)(32 * w + acc_row(r, h)) * kPartCols + col] = acc_e1[r];
        // sigma head: d w_sigma = sum_s (dA[256] + dA[257]) x y: rows 0 and 1 of the sigma tile
        if (h == 0) part[(size_t)256 * kPartCols + 32 * (4 * (w & 1) + (w >> 1)) + (lane & 31)] = acc_e2[0] + acc_e2[1];
      }
    }
    if (do_db && live) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const float tot = dbacc[i] + __shfl_xor(dbacc[i], 32);
        if (h == 0) dbpart[32 * row_tile(w, i) + (lane & 31)] = tot;
      }
    }
    if constexpr (kVD) {
      if (w == 0) {
        const float tot = dbsig + __shfl_xor(dbsig, 32);
        const float both = tot + __shfl(tot, 1);
        if (lane == 0) dbpart[256] = both;
      }
    }
    __syncthreads();
  }
};

template <int P>
__global__ __launch_bounds__(512, 2) void dw_kernel(DwArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[P == CN_P_BF16 ? kDwSmemBf16 : DwF32::kSmem];
  const int g = blockIdx.x;
  const long long total = a.wprefix[a.nprob];
  const long long b0 = dw_share_begin(g, total, a.nwg), b1 = dw_share_begin(g + 1, total, a.nwg);
  int seg = 0;
  for (int p = 0; p < a.nprob && seg < 2; ++p) {
    int t0, t1;
    dw_slab_range(a.wprefix, a.pbytes, a.total_tiles, p, b0, b1, t0, t1);
    if (t1 <= t0) continue;
    const size_t slot = (size_t)g * 2 + seg;
    const DwProblem& pr = a.p[p];
    float* part = a.part + slot * kPartRows * kPartCols;
    float* dbpart = a.dbpart + slot * kPartRows;
    if constexpr (P == CN_P_BF16) {
      switch (pr.kind) {
        case DW_FULL: DwBf16<DW_FULL>::run(pr, t0, t1, g * 613, part, dbpart, smem); break;
        case DW_PE: DwBf16<DW_PE>::run(pr, t0, t1, g * 613, part, dbpart, smem); break;
        case DW_VIEWDIR: DwBf16<DW_VIEWDIR>::run(pr, t0, t1, g * 613, part, dbpart, smem); break;
        case DW_RGB0: DwBf16<DW_RGB0>::run(pr, t0, t1, g * 613, part, dbpart, smem); break;
        default: DwBf16<DW_RGB2>::run(pr, t0, t1, g * 613, part, dbpart, smem); break;
      }
    } else {
      DwF32::run(pr, t0, t1, g * 613, part, dbpart, smem);
    }
    ++seg;
  }
}

// ---------------------------------------------------------------- reduction
__device__ __forceinline__ int pe_feature(int c) { return pe_slot_feature(col_half(c), col_slot(c)); }
__device__ __forceinline__ int dir_feature(int c) { return dir_slot_feature(col_half(c), col_slot(c)); }

__global__ __launch_bounds__(256) void dw_reduce_kernel(DwRedArgs a) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  if (gid >= a.prefix[a.nprob]) return;
  int pi = 0;
  while (pi + 1 < a.nprob && a.prefix[pi + 1] <= gid) ++pi;
  const DwRedProblem& p = a.p[pi];
  const int e = gid - a.prefix[pi];
  const int n = e / p.cols, c = e % p.cols;
  float v = 0.f, db = 0.f;
  const bool need_db = (c == 0) || p.z;
  const int gf = a.gfirst[pi], gl = a.glast[pi];
  for (int g = gf; g <= gl; ++g) {
    const size_t slot = (size_t)g * 2 + (g == gf ? a.gseg[pi] : 0);
    v += a.part[slot * kPartRows * kPartCols + (size_t)n * kPartCols + c];
    if (need_db) db += a.dbpart[slot * kPartRows + n];
  }
  if (p.map == MAP_VIEWDIR && n == p.out_real) {          // sigma-head row
    if (c < 256) a.grads[p.w2][c] += v;
    if (c == 0) a.grads[p.b2][0] += db;
    return;
  }
  if (p.z && n < p.out_real && c < p.in_real) v += db * p.z[c];
  if (n >= p.out_real) return;
  int f = c;
  if (p.map == MAP_PE) f = pe_feature(c);
  else if (p.map == MAP_VIEWDIR && c >= 256) {
    const int d = dir_feature(c - 256);
    f = d < 0 ? -1 : 256 + d;
  }
  if (f >= 0 && f < p.in_real) a.grads[p.w][(size_t)n * p.in_real + f] += v;
  if (c == 0) {
    a.grads[p.b][n] += db;
    if (p.dbout) p.dbout[n] = db;
  }
}

// ---------------------------------------------------------------- bias only
template <int P>
__global__ __launch_bounds__(256) void db_kernel(DbArgs a) {
  using E = std::conditional_t<P == CN_P_BF16, __bf16, float>;
  constexpr int ES = sizeof(E);
  const int j = blockIdx.y, blk = blockIdx.x, f = threadIdx.x;
  const int s0 = blk * a.slabs_per_blk, s1 = min(a.total_slabs, s0 + a.slabs_per_blk);
  const char* A = (const char*)a.A[j];
  const size_t slab_bytes = (size_t)a.a_width[j] * 32 * ES;
  const int foff = f & ~3, fe = (f & 3) * ES;
  float sum = 0.f;
  for (int t = s0; t < s1; ++t) {
    const char* base = A + (size_t)t * slab_bytes + fe;
#pragma unroll 8
    for (int s = 0; s < 32; ++s) sum += (float)*(const E*)(base + img_off<ES>(s, foff));
  }
  a.part[((size_t)j * kDbBlocks + blk) * 256 + f] = sum;
}

__global__ __launch_bounds__(256) void db_reduce_kernel(DbArgs a) {
  const int j = blockIdx.x, f = threadIdx.x;
  double sum = 0.0;
  for (int b = 0; b < kDbBlocks; ++b) sum += a.part[((size_t)j * kDbBlocks + b) * 256 + f];
  a.dbout[j * 256 + f] = (float)sum;
}

}  // namespace cn
