// Weight gradients of the CodeNeRF MLP: dW_L = sum_m dA_L[m] (x) X_L[m].
//
// The reduction runs over samples (K = M, ~1e6), so each workgroup owns one
// 128 x 128 output tile of one layer over one slice of the samples and writes
// an fp32 partial; dw_reduce sums the slices (deterministic, no atomics),
// maps padded / permuted columns back to the reference tensors, adds the
// code-injection correction db (x) z (the forward folds y + z into the bias)
// and accumulates into .grad.  Bias gradients (row sums of dA) are computed in
// the same pass from the A fragments.
//
// Operands are sample-major planes written by the chain kernels.  A 32-sample
// slab of each operand is staged through LDS (register staging, double
// buffered) and read back transposed:
//   bf16: ds_read_b64_tr_b16 (4 samples x 1 feature per lane per read) feeding
//         v_mfma_f32_32x32x16_bf16 with K = samples;
//   fp32: ds_read_b32 feeding v_mfma_f32_32x32x2_f32 (exact fp32).
#include "cn_common.h"
#include "chain_args.h"
#include "dw_args.h"

namespace cn {

template <int P>
struct DwCfg;
template <> struct DwCfg<CN_P_BF16> {
  using E = __bf16;
  static constexpr int kRow = 128 * 2 + 64;     // padded LDS row bytes (conflict-free tr reads)
  static constexpr int kPieces = 2;             // 16-byte pieces per thread per tile
};
template <> struct DwCfg<CN_P_FP32> {
  using E = float;
  static constexpr int kRow = 128 * 4;
  static constexpr int kPieces = 4;
};

typedef __attribute__((ext_vector_type(4))) short s16x4;

template <int P>
__global__ __launch_bounds__(256, 2) void dw_kernel(DwArgs a) {
  using C = DwCfg<P>;
  using E = typename C::E;
  constexpr bool kBf16 = P == CN_P_BF16;
  constexpr int kTile = 32 * C::kRow;            // one 32-sample x 128-feature slab
  constexpr int kEPP = 16 / sizeof(E);           // elements per 16-byte piece
  constexpr int kPPR = 128 / kEPP;               // pieces per row
  __shared__ __attribute__((aligned(16))) char smem[4 * kTile];   // [buf][A|X]

  // ---- job decode: problem, output tile, input tile, sample slice
  const int tiles_total = a.tile_prefix[a.nprob];
  const int job = blockIdx.x;
  const int slice = job / tiles_total;
  int rem = job - slice * tiles_total;
  int pi = 0;
  while (pi + 1 < a.nprob && a.tile_prefix[pi + 1] <= rem) ++pi;
  rem -= a.tile_prefix[pi];
  const DwProblem& pr = a.p[pi];
  const int to = rem / pr.in_tiles, ti = rem % pr.in_tiles;
  const int m0 = slice * a.mchunk;
  const int m1 = min(a.M, m0 + a.mchunk);

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int wo = w >> 1, wi = w & 1;   // wave sub-tile: rows 64*wo, cols 64*wi
  const int h = lane >> 5;

  // source descriptors of this job's A columns and X columns
  const int a_col0 = to * 128;
  const int a_cols = min(128, pr.a_valid - a_col0);
  const int x_col0 = ti * 128;
  const E* xsrc;
  int ldx, x_cols;
  if (x_col0 < pr.x0_cols) {
    xsrc = (const E*)pr.X0 + x_col0; ldx = pr.ldx0; x_cols = min(128, pr.x0_cols - x_col0);
  } else {
    xsrc = (const E*)pr.X1 + (x_col0 - pr.x0_cols); ldx = pr.ldx1;
    x_cols = min(128, pr.in_valid - x_col0);
  }
  const E* asrc = (const E*)pr.A + a_col0;
  const bool wave_live = (64 * wo < a_cols) && (64 * wi < x_cols);

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
  float dbacc[2] = {0.f, 0.f};

  u32x4 ra[C::kPieces], rx[C::kPieces];
  auto gload = [&](int mb) {
#pragma unroll
    for (int k = 0; k < C::kPieces; ++k) {
      const int piece = threadIdx.x + 256 * k;
      const int row = piece / kPPR, cp = piece % kPPR;
      const int mm = mb + row;
      const bool rok = mm < m1;
      ra[k] = (rok && cp * kEPP < a_cols) ? *(const u32x4*)(asrc + (size_t)mm * pr.lda + cp * kEPP) : u32x4{};
      rx[k] = (rok && cp * kEPP < x_cols) ? *(const u32x4*)(xsrc + (size_t)mm * ldx + cp * kEPP) : u32x4{};
    }
  };
  auto lstore = [&](int buf) {
    char* A = smem + buf * 2 * kTile;
    char* X = A + kTile;
#pragma unroll
    for (int k = 0; k < C::kPieces; ++k) {
      const int piece = threadIdx.x + 256 * k;
      const int row = piece / kPPR, cp = piece % kPPR;
      *(u32x4*)(A + row * C::kRow + cp * 16) = ra[k];
      *(u32x4*)(X + row * C::kRow + cp * 16) = rx[k];
    }
  };

  const int nsteps = (m1 - m0 + 31) / 32;
  if (nsteps > 0) {
    gload(m0);
    lstore(0);
  }
  __syncthreads();
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    if (st + 1 < nsteps) gload(m0 + 32 * (st + 1));
    const char* A = smem + buf * 2 * kTile;
    const char* X = A + kTile;
    if (wave_live) {
      if constexpr (kBf16) {
        const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
#pragma unroll
        for (int kk = 0; kk < 32; kk += 16) {
          bf16x8 fa[2], fx[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int col = 64 * wo + 32 * i + 16 * (g & 1) + 4 * p;
            const int row = kk + 8 * h + q;
            const char* base = A + row * C::kRow + col * 2;
            s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)base);
            s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(base + 4 * C::kRow));
            fa[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            const int colx = 64 * wi + 32 * i + 16 * (g & 1) + 4 * p;
            const char* bx = X + row * C::kRow + colx * 2;
            s16x4 xl = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)bx);
            s16x4 xh = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4*)(bx + 4 * C::kRow));
            fx[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(xl, xh, 0, 1, 2, 3, 4, 5, 6, 7));
          }
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < 8; ++j) s += (float)fa[i][j];
            dbacc[i] += s;
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fx[j], acc[i][j], 0, 0, 0);
          }
        }
      } else {
        const int c = lane & 31;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int row = 2 * q + h;
          float fa[2], fx[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            fa[i] = *(const float*)(A + row * C::kRow + (64 * wo + 32 * i + c) * 4);
            fx[i] = *(const float*)(X + row * C::kRow + (64 * wi + 32 * i + c) * 4);
          }
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            dbacc[i] += fa[i];
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fx[j], acc[i][j], 0, 0, 0);
          }
        }
      }
    }
    if (st + 1 < nsteps) lstore(buf ^ 1);
    __syncthreads();
  }

  // ---- write the fp32 partial tile: row n (out feature), column c (in feature)
  const int ldp = pr.in_tiles * 128;
  float* part = pr.part + ((size_t)slice * pr.out_tiles * 128) * ldp;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = ti * 128 + 64 * wi + 32 * j + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = to * 128 + 64 * wo + 32 * i + acc_row(r, h);
        part[(size_t)row * ldp + col] = acc[i][j][r];
      }
    }
  if (wi == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float tot = dbacc[i] + __shfl_xor(dbacc[i], 32);
      if (h == 0)
        pr.dbpart[(size_t)slice * pr.out_tiles * 128 + to * 128 + 64 * wo + 32 * i + (lane & 31)] = tot;
    }
  }
}

__device__ __forceinline__ int pe_feature(int slot) { return pe_slot_feature(slot >> 5, slot & 31); }
__device__ __forceinline__ int dir_feature(int slot) { return dir_slot_feature(slot >> 4, slot & 15); }

__global__ __launch_bounds__(256) void dw_reduce_kernel(DwRedArgs a) {
  const int gid = blockIdx.x * 256 + threadIdx.x;
  if (gid >= a.prefix[a.nprob]) return;
  int pi = 0;
  while (pi + 1 < a.nprob && a.prefix[pi + 1] <= gid) ++pi;
  const DwRedProblem& p = a.p[pi];
  const int e = gid - a.prefix[pi];
  const int n = e / p.cols, c = e % p.cols;
  const size_t slice_stride = (size_t)p.rows_pad * p.ldp;
  float v = 0.f;
  for (int s = 0; s < a.slices; ++s) v += p.part[s * slice_stride + (size_t)n * p.ldp + c];
  float db = 0.f;
  const bool need_db = (c == 0) || p.z;
  if (need_db)
    for (int s = 0; s < a.slices; ++s) db += p.dbpart[(size_t)s * p.rows_pad + n];
  if (p.z && n < p.out_real && c < p.in_real) v += db * p.z[c];
  // destination
  if (p.map == MAP_VIEWDIR && n >= p.out_real) {          // sigma-head rows (value, residual)
    if (n == p.out_real) {
      // combine both rows here so the accumulation into .grad stays race-free
      float v2 = 0.f, db2 = 0.f;
      for (int s = 0; s < a.slices; ++s) v2 += p.part[s * slice_stride + (size_t)(n + 1) * p.ldp + c];
      if (c == 0)
        for (int s = 0; s < a.slices; ++s) db2 += p.dbpart[(size_t)s * p.rows_pad + n + 1];
      if (c < 256) a.grads[p.w2][c] += v + v2;
      if (c == 0) a.grads[p.b2][0] += db + db2;
    }
    return;
  }
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

}  // namespace cn
