// Parameter packing and the AdamW step.
//
// pack:  gathers the reference-layout fp32 parameters into the chain kernels'
//        fragment-ordered blobs (fp32 or bf16) through a precomputed index
//        table (built once per plan on the host, plan.cpp).
// adamw: torch.optim.AdamW (reference src/trainer.py:116-120, defaults
//        betas 0.9/0.999, eps 1e-8, weight_decay 0.01) for every tensor of a
//        parameter group in one launch, in torch's single-tensor update order:
//          p *= 1 - lr*wd;  m = lerp(m, g, 1-b1);  v = v*b2 + (1-b2)*g*g;
//          p += ((-lr/bc1) * m) / (sqrt(v)/sqrt(bc2) + eps)
#include "cn_common.h"

namespace cn {

// idx: (tensor << 24) | (lo << 23) | offset, or -1 for a zero; lo (bf16x3):
// the element is w_lo = rn(w - rn(w)) instead of rn(w)
__global__ __launch_bounds__(256) void pack_kernel(const float* const* params, const int32_t* __restrict__ idx,
                                                   int n, void* out, int bf16) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int e = idx[i];
  const float v = e < 0 ? 0.f : params[(uint32_t)e >> 24][e & 0x7FFFFF];
  if (bf16) {
    const __bf16 hi = (__bf16)v;
    ((__bf16*)out)[i] = (e >= 0 && (e & 0x800000)) ? (__bf16)(v - (float)hi) : hi;
  } else {
    ((float*)out)[i] = v;
  }
}

constexpr int kAdamMaxSeg = 48;
struct AdamSeg {
  float* p;
  float* g;
  float* m;
  float* v;
  int n;
  float decay;        // 1 - lr * wd
  float step_neg;     // -lr / bc1
};
struct AdamArgs {
  AdamSeg s[kAdamMaxSeg];
  int nseg;
  int prefix[kAdamMaxSeg + 1];   // cumulative element counts
  float lerp_w;       // 1 - beta1
  float beta2, one_m_beta2;
  float bc2_sqrt;     // sqrt(1 - beta2^t)
  float eps;
  int zero_grad;      // write g = 0 after reading it (the next step's zero_grad, for free)
};

__global__ __launch_bounds__(256) void adamw_kernel(AdamArgs a) {
  const int total = a.prefix[a.nseg];
  for (int gid = blockIdx.x * 256 + threadIdx.x; gid < total; gid += gridDim.x * 256) {
    int si = 0;
    while (si + 1 < a.nseg && a.prefix[si + 1] <= gid) ++si;
    const AdamSeg& s = a.s[si];
    const int i = gid - a.prefix[si];
    const float g = s.g[i];
    float p = fmul_rn(s.p[i], s.decay);
    float m = s.m[i];
    // torch lerp with weight < 0.5: m + w * (g - m)
    m = fadd_rn(m, fmul_rn(a.lerp_w, fadd_rn(g, -m)));
    float v = fmul_rn(s.v[i], a.beta2);
    v = fadd_rn(v, fmul_rn(fmul_rn(a.one_m_beta2, g), g));
    const float denom = fadd_rn(sqrtf(v) / a.bc2_sqrt, a.eps);
    // ATen addcdiv: self + value * t1 / t2, evaluated left to right
    p = fadd_rn(p, fmul_rn(s.step_neg, m) / denom);
    s.p[i] = p;
    s.m[i] = m;
    s.v[i] = v;
    if (a.zero_grad) s.g[i] = 0.f;
  }
}

__global__ __launch_bounds__(256) void zero_kernel(float* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = 0.f;
}

}  // namespace cn
