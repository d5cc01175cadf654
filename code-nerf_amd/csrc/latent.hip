// Per-object latent-code layers (reference src/model.py:22-23,30-31,41,49).
//
// Forward: z_j = ReLU(L_j code + c_j) for every shape / texture block, then
// the injection y + z_j that feeds layer W_j is folded into that layer's bias:
// b'_j = b_j + W_j z_j (one 256x256 GEMV per block per call).  The result is
// the per-call bias blob the chain kernels load into LDS.
//
// Backward: dz_j = W_j^T db_j (db_j = this call's bias gradient of the layer
// z_j is injected into = sum over samples of its pre-activation gradient),
// dpre_j = dz_j * [z_j > 0], d L_j += dpre_j code^T, d c_j += dpre_j, and
// d code = sum_j L_j^T dpre_j (+ the regulariser of src/trainer.py:77-78).
#include "cn_common.h"
#include "chain_args.h"
#include "latent_args.h"

namespace cn {

template <int SB, int TB>
__global__ __launch_bounds__(256) void latent_fwd_kernel(LatentArgs a) {
  using N = Net<SB, TB>;
  constexpr ParamIdx P{SB, TB};
  __shared__ float z[256];
  __shared__ float code[256];
  const int L = blockIdx.x;
  const int i = threadIdx.x;
  if (L == N::kFwdLayers) {   // sigma head weight + bias
    a.blob[BiasBlob<SB, TB>::kWs + i] = a.params[P.sigma_w()][i];
    if (i < 4) a.blob[BiasBlob<SB, TB>::kMisc + i] = i == 0 ? a.params[P.sigma_w() + 1][0] : 0.f;
    return;
  }
  const Layer l = N::fwd(L);
  const int out_real = L == N::kFwdLayers - 1 ? 3 : l.T * 32;
  const int inj = L >= 1 ? N::fwd(L - 1).inj : -1;
  float b = i < out_real ? a.params[l.b][i] : 0.f;
  if (inj >= 0) {
    const bool shape = inj < SB;
    const int lw = shape ? P.shape_latent_w(inj) : P.tex_latent_w(inj - SB);
    code[i] = (shape ? a.shape_code : a.texture_code)[i];
    __syncthreads();
    const float* Lw = a.params[lw] + (size_t)i * 256;
    float acc = 0.f;
    for (int k = 0; k < 256; ++k) acc = __builtin_fmaf(Lw[k], code[k], acc);
    acc += a.params[lw + 1][i];
    const float zi = acc > 0.f ? acc : 0.f;
    z[i] = zi;
    a.zvec[inj * 256 + i] = zi;
    __syncthreads();
    // row i of W_j (256 x 256): b'_i = b_i + sum_k W[i][k] z[k]
    const float* W = a.params[l.w] + (size_t)i * 256;
    float s = 0.f;
    for (int k = 0; k < 256; ++k) s = __builtin_fmaf(W[k], z[k], s);
    b += s;
  }
  a.blob[L * 256 + i] = b;
}

template <int SB, int TB>
__global__ __launch_bounds__(256) void latent_bwd_kernel(LatentBwdArgs a) {
  constexpr ParamIdx P{SB, TB};
  __shared__ float db[256];
  __shared__ float dp[256];
  // grid (kInject, kLatentRowBlocks): block (j, r) recomputes dz_j (a GEMV
  // over W_j, L2-resident) and updates rows [32 r, 32 r + 32) of d L_j, so the
  // 256 KB read-modify-write of each latent weight gradient is spread over
  // kLatentRowBlocks workgroups; block r == 0 also writes dpre and d c_j
  const int j = blockIdx.x;
  const int rb = blockIdx.y;
  const int i = threadIdx.x;
  // code_grad_kernel (next on the stream) adds both codes' regulariser terms
  if (j == 0 && rb == 0 && i == 0 && a.reg_out) *a.reg_out = 0.f;
  const bool shape = j < SB;
  const int wl = shape ? P.shape_w(j) : P.tex_w(j - SB);          // layer fed by z_j
  const int lw = shape ? P.shape_latent_w(j) : P.tex_latent_w(j - SB);
  db[i] = a.dbuf[j * 256 + i];
  __syncthreads();
  // dz_i = sum_n W[n][i] db[n]  (coalesced over i)
  const float* W = a.params[wl];
  float dz = 0.f;
  for (int n = 0; n < 256; ++n) dz = __builtin_fmaf(W[(size_t)n * 256 + i], db[n], dz);
  const float d = a.zvec[j * 256 + i] > 0.f ? dz : 0.f;
  dp[i] = d;
  if (rb == 0) {
    a.dpre[j * 256 + i] = d;
    a.grads[lw + 1][i] += d;
  }
  __syncthreads();
  const float* code = shape ? a.shape_code : a.texture_code;
  const float ck = code[i];
  float* gL = a.grads[lw];
  constexpr int kRows = 256 / kLatentRowBlocks;
#pragma unroll 8
  for (int r = rb * kRows; r < (rb + 1) * kRows; ++r) gL[(size_t)r * 256 + i] += dp[r] * ck;
}

template <int SB, int TB>
__global__ __launch_bounds__(1024) void code_grad_kernel(LatentBwdArgs a) {
  // 4 groups of 256 threads each take a quarter of the rows i of every L_j;
  // their partial sums are added in a fixed order (deterministic)
  constexpr ParamIdx P{SB, TB};
  __shared__ float red[256];
  __shared__ float part[4][256];
  const bool shape = blockIdx.x == 0;
  const int k = threadIdx.x & 255, q = threadIdx.x >> 8;
  const float* code = shape ? a.shape_code : a.texture_code;
  const int j0 = shape ? 0 : SB, j1 = shape ? SB : SB + TB;
  float gq = 0.f;
  for (int j = j0; j < j1; ++j) {
    const int lw = shape ? P.shape_latent_w(j) : P.tex_latent_w(j - SB);
    const float* L = a.params[lw];
    const float* d = a.dpre + j * 256;
#pragma unroll 8
    for (int i = 64 * q; i < 64 * q + 64; ++i) gq = __builtin_fmaf(L[(size_t)i * 256 + k], d[i], gq);
  }
  part[q][k] = gq;
  // regulariser reg_coef * mean(|s| + |t|) over the (1, 256) codes; every
  // thread of the block passes every barrier, group 0 does the work
  const float c = code[k];
  if (q == 0) red[k] = c * c;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (q == 0 && k < s) red[k] += red[k + s];
    __syncthreads();
  }
  if (q != 0) return;
  float g = (part[0][k] + part[1][k]) + (part[2][k] + part[3][k]);
  const float nrm = sqrtf(red[0]);
  if (a.reg_coef != 0.f && nrm > 0.f) g += a.reg_coef * (c / nrm);
  (shape ? a.d_shape_code : a.d_texture_code)[k] += g;
  if (k == 0 && a.reg_out) atomicAdd(a.reg_out, a.reg_coef * nrm);
}

}  // namespace cn
