// Weight gradients of the CodeNeRF MLP: dW_L = sum_m dA_L[m] (x) X_L[m].
//
// The reduction runs over samples (K = M ~ 2e6): a persistent workgroup (one
// per CU) owns the WHOLE (<= 288 x 288) gradient of one layer over one
// byte-balanced slice of the (layer, slab) stream, so every operand byte is
// read from HBM exactly once.  This pass is HBM-bound: 6,976 B of bf16
// operands per sample (srncar net; encoding_shape folded, chain_set.h)
// against 0.77 MFLOP.  A 32-sample slab of a plane is one
// contiguous run (cn_layout.h); it lands in LDS unchanged and is read back
// transposed.
//   bf16 (DwBf16<KIND>): one compile-time body per operand shape (DwKind),
//     4-slot LDS-DMA ring (three slabs in flight while one is consumed),
//     ds_read_b64_tr_b16 (conflict-free by the pair-block rotation) feeding
//     v_mfma_f32_32x32x16_bf16; the sigma head (ds x y_shape) is an extra
//     MFMA tile of the viewdir body;
//   fp32: exact fp32 parity path, 2-slot LDS-DMA ring of 72 KiB slots,
//     ds_read_b32 + v_mfma_f32_32x32x2_f32; MFMA-bound, so the schedule
//     balances MFMA cost instead of bytes (chain_set.h dw_f32_slab_cost).
// Every body reads its X fragments one column tile ahead of the MFMAs that
// use them (round 4: the LDS latency had sat between the MFMA groups).
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

// ------------------------------------------------------------ bodies
// One compile-time body per (precision, operand shape): every wave's tiles,
// LDS reads, MFMAs and piece counts are constants, so the slab loop has no
// runtime branches beyond wave-uniform role tests.  Staging by LDS-DMA:
//   bf16: 4-slot ring of 32 / 36 KiB slots, three slabs in flight;
//   fp32: 2-slot ring of 72 KiB slots, one slab in flight (this path is
//         MFMA-bound: 16 K SIMD cycles of v_mfma_f32_32x32x2_f32 per slab).
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
constexpr int kDwSmem = 160 * 1024;

// LO (bf16x3 planes): the slab also stages X0's lo parts (after X1), and every
// X0 fragment's MFMA is followed by one with the lo fragment, so dW sums
// A (x) (X0_hi + X0_lo) -- the X operand at ~16 significant bits, as the
// bf16x3 chains used it.  The dir-PE tile (X1) stays hi only.
template <int P, int KIND, bool LO = false>
struct DwBody {
  using Sh = DwShape<KIND>;
  static constexpr bool kBf16 = P == CN_P_BF16;
  static_assert(kBf16 || !LO, "lo planes exist for bf16 planes only");
  static constexpr int ES = kBf16 ? 2 : 4;
  static constexpr int TB = 1024 * ES;                      // one 32-sample x 32-feature tile
  static constexpr int kA = Sh::kA, kX0 = Sh::kX0, kX1 = Sh::kX1, NI = Sh::NI, NJ = Sh::NJ;
  static constexpr int kXl = LO ? kX0 : 0;                  // lo tiles of X0
  static constexpr int kPA = kA * TB / 1024, kPX0 = kX0 * TB / 1024;   // 1 KiB pieces of A / X0
  static constexpr int kPX1 = kX1 * TB / 1024;
  static constexpr int kPieces = (kA + kX0 + kX1 + kXl) * TB / 1024;     // 1 KiB pieces per slab
  static constexpr int kG = (kPieces + 7) / 8;              // pieces per wave per slab
  static constexpr bool kVD = KIND == DW_VIEWDIR;
  // hi-only bf16: 32 / 36 KiB slots, 4-slot ring (measured best); LO: the
  // slab itself, as many slots (<= 4) as fit beside the padding pieces
  static constexpr int kLoRing = (kDwSmem - (8 * kG - kPieces) * 1024) / (kPieces * 1024);
  static constexpr int kDwSlot = LO ? kPieces * 1024 : kBf16 ? (KIND == DW_FULL ? 32 * 1024 : 36 * 1024) : 72 * 1024;
  // Paired staging (the bf16 256 x 256 bodies): one barrier and one 64 KiB
  // DMA batch per TWO slabs over a 5-slot ring (three slabs in flight while
  // two are consumed) -- the LO bodies' 48 KiB batches streamed at 6.2 TB/s
  // where per-slab 32 KiB batches stream at 5.5 (profiles/r04c, r04e)
  static constexpr bool kPair = kBf16 && !LO && KIND == DW_FULL;
  static constexpr int kDwRing = kPair ? 5 : LO ? (kLoRing < 4 ? kLoRing : 4) : kBf16 ? 4 : 2;
  static_assert(!LO || kDwRing >= 3, "a LO slab must leave a 3-slot ring");
  static constexpr int kDwDepth = kPair ? 3 : kDwRing - 1;   // slabs issued before the first barrier
  static constexpr int kDwDummy = kDwRing * kDwSlot;  // landing area of padding pieces
  static_assert(kPieces * 1024 <= kDwSlot, "dw stage");
  static_assert(kDwDummy + (8 * kG - kPieces) * 1024 <= kDwSmem, "dw LDS");

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
    const char* px0l = LO ? (const char*)pr.X0lo : px0;
    auto issue = [&](int st, auto slotc) {
      const size_t t = (size_t)slab(st);
#pragma unroll
      for (int k = 0; k < kG; ++k) {
        const int piece = w * kG + k;            // wave-uniform
        const char* src;
        uint32_t dst = lds_addr(smem + decltype(slotc)::value * kDwSlot + piece * 1024);
        if (piece < kPA) src = pa + t * (kA * TB) + piece * 1024;
        else if (piece < kPA + kPX0) src = px0 + t * (kX0 * TB) + (piece - kPA) * 1024;
        else if (piece < kPA + kPX0 + kPX1) src = px1 + t * (kX1 * TB) + (piece - kPA - kPX0) * 1024;
        else if (piece < kPieces) src = px0l + t * (kX0 * TB) + (piece - kPA - kPX0 - kPX1) * 1024;
        else {
          src = pa + t * (kA * TB);              // padding piece: re-read, never consumed
          dst = lds_addr(smem + kDwDummy + (piece - kPieces) * 1024);
        }
        // non-temporal: a once-read stream (measured 3.24 -> 3.13 ms per C2 dW
        // against the default policy)
        glds16_opaque_nt(src + lane * 16, dst);
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
      if constexpr (kPair) {
        // even slab: slabs st and st + 1 must have landed (only st + 2 may
        // still be in flight); then st + 3 and st + 4 go into the slots of
        // st - 2 and st - 1, which every wave finished before this barrier
        if ((st & 1) == 0) {
          if (st + 2 < nst) wait_vmcnt<kG>();
          else wait_vmcnt<0>();
          block_barrier();
          if (st + 3 < nst) issue(st + 3, std::integral_constant<int, (SL + 3) % kDwRing>{});
          if (st + 4 < nst) issue(st + 4, std::integral_constant<int, (SL + 4) % kDwRing>{});
        }
      } else {
        const int ahead = min(kDwDepth - 1, nst - 1 - st);
        static_for<0, kDwDepth>([&](auto n) {
          if (n == ahead) wait_vmcnt<n * kG>();
        });
        block_barrier();
        if (st + kDwDepth < nst) issue(st + kDwDepth, std::integral_constant<int, (SL + kDwDepth) % kDwRing>{});
      }
      const char* A = smem + SL * kDwSlot;
      const char* X = A + kA * TB;
      const char* Xl = X + (kX0 + kX1) * TB;     // LO: X0's lo tiles
      if (!live) return;
      if constexpr (!kBf16) {
        // exact fp32: K = 2 samples per MFMA; lane l reads feature l & 31 of
        // sample 2 qq + (l >> 5) (A: rows = out features, B: cols = inputs)
        const int c = lane & 31;
        auto val = [&](const char* base, int tile, int s) {
          const int f = 32 * tile + c;
          return *(const float*)(base + img_off<4>(s, f & ~3) + (f & 3) * 4);
        };
#pragma unroll 4
        for (int qq = 0; qq < 16; ++qq) {
          const int s = 2 * qq + h;
          float fa[NI];
#pragma unroll
          for (int i = 0; i < NI; ++i) fa[i] = val(A, row_tile(w, i), s);
          float fs = 0.f;
          if constexpr (kVD) fs = val(A, 8, s);
          // X values read one column tile ahead of their MFMAs (as the bf16
          // bodies below)
          float fx = val(X, col_tile(w, 0), s);
#pragma unroll
          for (int i = 0; i < NI; ++i)
            if (do_db) dbacc[i] += fa[i];
          if constexpr (kVD) {
            if (w == 0) dbsig += fs;
          }
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            float nx = 0.f;
            if (j + 1 < NJ) nx = val(X, col_tile(w, j + 1), s);
            else if constexpr (kVD) nx = val(X, 8, s);          // the dir-PE input tile
#pragma unroll
            for (int i = 0; i < NI; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fx, acc[i][j], 0, 0, 0);
            fx = nx;
          }
          if constexpr (kVD) {
            const float fr = (w & 1) ? fa[1] : fa[0];
            acc_e1 = __builtin_amdgcn_mfma_f32_32x32x2f32(fr, fx, acc_e1, 0, 0, 0);   // fx = the dir-PE value
            // the sigma-head row against column tile w >> 1 (no branch in the loop)
            acc_e2 = __builtin_amdgcn_mfma_f32_32x32x2f32(fs, val(X, 4 * (w & 1) + (w >> 1), s), acc_e2, 0, 0, 0);
          }
        }
        return;
      }
#pragma unroll
      for (int kk = 0; kk < 32; kk += 16) {
        const int s = kk + 8 * h + q;
        // every X fragment is read one column tile ahead of the MFMAs that
        // use it (the compiler otherwise waits lgkmcnt(0) right behind each
        // read: the LDS latency stood between every pair of MFMA groups)
        bf16x8 fa[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) fa[i] = frag(A, row_tile(w, i), s);
        bf16x8 fs{};
        if constexpr (kVD) fs = frag(A, 8, s);   // sigma-head columns 256.. of the dA plane
        bf16x8 fx = frag(X, col_tile(w, 0), s);
        bf16x8 fxl{};
        if constexpr (LO) fxl = frag(Xl, col_tile(w, 0), s);
        // bias sums (VALU) while the reads are in flight
#pragma unroll
        for (int i = 0; i < NI; ++i)
          if (do_db) dbacc[i] += rowsum(fa[i]);
        if constexpr (kVD) {
          if (w == 0) dbsig += rowsum(fs);
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          bf16x8 nx{}, nxl{};
          if (j + 1 < NJ) {
            nx = frag(X, col_tile(w, j + 1), s);
            if constexpr (LO) nxl = frag(Xl, col_tile(w, j + 1), s);
          } else if constexpr (kVD) {
            nx = frag(X, 8, s);                  // the dir-PE input tile, for acc_e1 below
          }
#pragma unroll
          for (int i = 0; i < NI; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fx, acc[i][j], 0, 0, 0);
          if constexpr (kVD && LO) {      // (LO: no registers left for a re-read after the loop)
            if (j == (w >> 1)) acc_e2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fs, fx, acc_e2, 0, 0, 0);
          }
          if constexpr (LO) {
#pragma unroll
            for (int i = 0; i < NI; ++i)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fxl, acc[i][j], 0, 0, 0);
            if constexpr (kVD) {
              if (j == (w >> 1)) acc_e2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fs, fxl, acc_e2, 0, 0, 0);
            }
          }
          fx = nx;
          fxl = nxl;
        }
        if constexpr (kVD) {
          const bf16x8 fr = (w & 1) ? fa[1] : fa[0];
          acc_e1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr, fx, acc_e1, 0, 0, 0);   // fx = the dir-PE tile
          // the sigma-head tile against this wave's column tile w >> 1 of its
          // half, read once more instead of a wave-uniform branch inside the
          // unrolled column loop (each branch target cost hazard NOPs)
          if constexpr (!LO)
            acc_e2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fs, frag(X, 4 * (w & 1) + (w >> 1), s), acc_e2, 0, 0, 0);
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
  __shared__ __attribute__((aligned(16))) char smem[kDwSmem];
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
    // bf16x3 planes: the X0 lo parts ride along (pr.lo, DwBody<..., true>)
    auto body = [&](auto kind) {
      constexpr int K = decltype(kind)::value;
      if constexpr (P == CN_P_BF16) {
        if (pr.lo) {
          DwBody<P, K, true>::run(pr, t0, t1, g * 613, part, dbpart, smem);
          return;
        }
      }
      DwBody<P, K>::run(pr, t0, t1, g * 613, part, dbpart, smem);
    };
    switch (pr.kind) {
      case DW_FULL: body(std::integral_constant<int, DW_FULL>{}); break;
      case DW_PE: body(std::integral_constant<int, DW_PE>{}); break;
      case DW_VIEWDIR: body(std::integral_constant<int, DW_VIEWDIR>{}); break;
      case DW_RGB0: body(std::integral_constant<int, DW_RGB0>{}); break;
      default: body(std::integral_constant<int, DW_RGB2>{}); break;
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
  if (p.map == MAP_VIEWDIR) {
    // columns < 256 are the last shape layer's features: Gx of the
    // encoding_shape fold (dw_fold_kernel maps them); row out_real = sigma head
    if (c < 256) a.fold[n * kFoldCols + c] = v;
    if (c == 0) a.fold[n * kFoldCols + 256] = db;
    if (n == p.out_real) {
      if (c == 0) a.grads[p.b2][0] += db;
      return;
    }
    if (c < 256) {
      if (c == 0) a.grads[p.b][n] += db;
      return;
    }
  }
  if (p.z && n < p.out_real && c < p.in_real) v += db * p.z[c];
  if (n >= p.out_real) return;
  int f = c;
  if (p.map == MAP_PE) f = pe_feature(c);
  else if (p.map == MAP_VIEWDIR) {
    const int d = dir_feature(c - 256);
    f = d < 0 ? -1 : 256 + d;
  }
  if (f >= 0 && f < p.in_real) a.grads[p.w][(size_t)n * p.in_real + f] += v;
  if (c == 0) {
    a.grads[p.b][n] += db;
    if (p.dbout) p.dbout[n] = a.db_accum ? p.dbout[n] + db : db;
  }
}

// ---------------------------------------------------------------- fold
// The encoding_shape fold (chain_set.h fold_args), two small fp32 GEMMs over
// the reduced Gx (257 x 257), one 16 x 16 output tile per workgroup:
//   z = 0: d[W_v y-part ; w_sigma] (257 x 256)  = Gx . Wx_e^T
//   z = 1: d[W_e | b_e]            (256 x 257)  = Wx_v^T . Gx
// ~34 M FMAs per dW launch.
__global__ __launch_bounds__(256) void dw_fold_kernel(DwFoldArgs a) {
  // one 16 x 16 output tile per workgroup (grid 17 x 17 x 2: ~570 live
  // workgroups, one output per thread -- 32 x 32 tiles left ~160 workgroups
  // on 256 CUs running 257-long LDS-latency-bound chains: 28 us per fold);
  // the workgroup's whole K = 257 strips of both operands staged at once
  __shared__ float As[16][kFoldCols + 3];     // [i][k]
  __shared__ float Bs[kFoldCols][17];         // [k][j]
  const int z = blockIdx.z;
  const int rows = z == 0 ? kFoldRows : 256, cols = z == 0 ? 256 : kFoldCols;
  const int i0 = blockIdx.y * 16, j0 = blockIdx.x * 16;
  if (i0 >= rows || j0 >= cols) return;
  const float* G = a.fold;
  const float* We = a.params[a.w_shape];
  const float* be = a.params[a.w_shape + 1];
  const float* Wv = a.params[a.w_view];
  const float* ws = a.params[a.w_sigma];
  const int VC = a.view_cols;
  // consecutive threads read consecutive addresses of each operand
  if (z == 0) {
    // A = Gx rows i0.. (contiguous), B(k, j) = [W_e | b_e][j][k]
    for (int e = threadIdx.x; e < 16 * kFoldCols; e += 256) {
      const int ii = e / kFoldCols, k = e - ii * kFoldCols;
      As[ii][k] = i0 + ii < rows ? G[(size_t)(i0 + ii) * kFoldCols + k] : 0.f;
    }
    for (int e = threadIdx.x; e < 16 * 256; e += 256) {
      const int jj = e >> 8, k = e & 255;
      Bs[k][jj] = We[(size_t)(j0 + jj) * 256 + k];
    }
    if (threadIdx.x < 16) Bs[256][threadIdx.x] = be[j0 + threadIdx.x];
  } else {
    // A(i, k) = [W_v ; w_sigma][k][i] (rows of W_v contiguous in i), B = Gx
    for (int e = threadIdx.x; e < kFoldRows * 16; e += 256) {
      const int k = e >> 4, ii = e & 15;
      As[ii][k] = k < 256 ? Wv[(size_t)k * VC + i0 + ii] : ws[i0 + ii];
      Bs[k][ii] = j0 + ii < cols ? G[(size_t)k * kFoldCols + j0 + ii] : 0.f;
    }
  }
  __syncthreads();
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;   // 16 x 16
  // one FMA chain in k order: the fp32 parity path's sums stay in the order
  // the trajectory tests were pinned with (tiling changes no sum)
  float acc = 0.f;
#pragma unroll 8
  for (int k = 0; k < kFoldCols; ++k) acc = __builtin_fmaf(As[ty][k], Bs[k][tx], acc);
  const int i = i0 + ty, j = j0 + tx;
  if (i >= rows || j >= cols) return;
  if (z == 0) {
    if (i < 256) a.grads[a.w_view][i * VC + j] += acc;
    else a.grads[a.w_sigma][j] += acc;
  } else {
    if (j < 256) a.grads[a.w_shape][i * 256 + j] += acc;
    else a.grads[a.w_shape + 1][i] += acc;
  }
}

// ---------------------------------------------------------------- bias only
// Column sums of the 256-wide dA planes of the code-fed layers, streamed in
// 16-B chunks: in a slab, thread t reads chunks t + 256 k, which always hold
// the same sample's 8 (bf16: two quads, cn_layout.h) / 4 (fp32) features of
// tiles advancing with k; each lane sums its sample over the workgroup's slabs, then
// the 32 lanes of a half-wave (the 32 samples) are combined by an xor tree.
template <int P>
__global__ __launch_bounds__(256) void db_kernel(DbArgs a) {
  constexpr bool kBf16 = P == CN_P_BF16;
  constexpr int EPC = kBf16 ? 8 : 4;                // elements per 16-B chunk
  constexpr int NK = 256 * (kBf16 ? 2 : 4) / 128;   // chunks per thread per slab (256-wide plane)
  const int j = blockIdx.y, blk = blockIdx.x, t = threadIdx.x, lane = t & 63;
  const int s0 = blk * a.slabs_per_blk, s1 = min(a.total_slabs, s0 + a.slabs_per_blk);
  const u32x4* A = (const u32x4*)a.A[j];
  float acc[NK][EPC];
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int e = 0; e < EPC; ++e) acc[k][e] = 0.f;
  for (int sl = s0; sl < s1; ++sl) {
    const u32x4* base = A + (size_t)sl * (256 * NK) + t;
    u32x4 v[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) v[k] = base[256 * k];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      if constexpr (kBf16) {
        const bf16x8 x = __builtin_bit_cast(bf16x8, v[k]);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[k][e] += (float)x[e];
      } else {
        const f32x4 x = __builtin_bit_cast(f32x4, v[k]);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[k][e] += x[e];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NK; ++k)
#pragma unroll
    for (int e = 0; e < EPC; ++e) {
      float x = acc[k][e];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) x += __shfl_xor(x, o);
      acc[k][e] = x;
    }
  if ((lane & 31) == 0) {
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c = t + 256 * k;
      // bf16 chunk (tile, pair block gp, lane half hh): features 16 gp + 4 hh
      // + (e & 3) + 8 (e >> 2); fp32 chunk: 4 consecutive features
      const int f0 = kBf16 ? 32 * (c >> 7) + 16 * ((c >> 6) & 1) + 4 * ((c >> 5) & 1)
                           : 32 * (c >> 8) + 8 * ((c >> 6) & 3) + 4 * ((c >> 5) & 1);
#pragma unroll
      for (int e = 0; e < EPC; ++e)
        a.part[((size_t)j * kDbBlocks + blk) * 256 + f0 + (kBf16 ? (e & 3) + 8 * (e >> 2) : e)] = acc[k][e];
    }
  }
}

__global__ __launch_bounds__(256) void db_reduce_kernel(DbArgs a) {
  const int j = blockIdx.x, f = threadIdx.x;
  double sum = 0.0;
  for (int b = 0; b < kDbBlocks; ++b) sum += a.part[((size_t)j * kDbBlocks + b) * 256 + f];
  a.dbout[j * 256 + f] = (float)sum;
}

}  // namespace cn
