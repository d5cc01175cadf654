// Ray generation, alpha compositing (+ backward) and the image loss.
//
//   get_rays            reference src/utils.py:10-19
//   composite fwd/bwd   reference src/utils.py:34-47 and its autograd
//   render_loss         composite + chunk-mean MSE (src/trainer.py:75) + the
//                       composite backward, fused per ray for training
//
// One wave per ray: lane l owns a contiguous run of samples, the exclusive
// transmittance product and the reverse cumulative sum are wave scans.  Both
// accumulate in float64, as torch's CPU cumprod/cumsum do (acc_type<float> is
// double on the CPU), so the rounded float results match the reference.
#include "cn_common.h"

namespace cn {

// ---------------------------------------------------------------- rays
__global__ __launch_bounds__(256) void get_rays_kernel(int H, int W, double focal, int focal_f64,
                                                       const float* __restrict__ c2w,
                                                       float* __restrict__ ro, float* __restrict__ vd) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= H * W) return;
  const int row = p / W, col = p - row * W;
  float dx, dy;
  if (focal_f64) {   // (i - W/2) / focal formed in float64, then cast (type promotion)
    dx = (float)(((double)col - W * 0.5) / focal);
    dy = (float)(-(((double)row - H * 0.5) / focal));
  } else {
    const float f = (float)focal;
    dx = ((float)col - W * 0.5f) / f;
    dy = -(((float)row - H * 0.5f) / f);
  }
  float d[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    // sum_b dirs[b] * c2w[a][b], summed in order, no fma
    float s = fmul_rn(dx, c2w[4 * a + 0]);
    s = fadd_rn(s, fmul_rn(dy, c2w[4 * a + 1]));
    s = fadd_rn(s, fmul_rn(-1.f, c2w[4 * a + 2]));
    d[a] = s;
  }
  // torch.norm(dim=-1) of a float32 3-vector on the CPU (src/utils.py:16):
  // sqrt(fma(d2, d2, fma(d1, d1, d0 * d0))) -- matched bit for bit against
  // torch 2.10's CPU kernel over 2e5 random vectors
  const float nrm = sqrtf(__builtin_fmaf(d[2], d[2], __builtin_fmaf(d[1], d[1], fmul_rn(d[0], d[0]))));
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    vd[3 * p + a] = d[a] / nrm;
    ro[3 * p + a] = c2w[4 * a + 3];
  }
}

// ---------------------------------------------------------------- scans
CN_DEV double shfl_up_d(double v, int k) {
  const int lo = __shfl_up(__double2loint(v), k);
  const int hi = __shfl_up(__double2hiint(v), k);
  return __hiloint2double(hi, lo);
}
CN_DEV double shfl_down_d(double v, int k) {
  const int lo = __shfl_down(__double2loint(v), k);
  const int hi = __shfl_down(__double2hiint(v), k);
  return __hiloint2double(hi, lo);
}
// exclusive product over lanes (lane 0 gets 1)
CN_DEV double wave_exclusive_prod(double v) {
  const int lane = threadIdx.x & 63;
  double incl = v;
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const double o = shfl_up_d(incl, k);
    if (lane >= k) incl *= o;
  }
  double ex = shfl_up_d(incl, 1);
  return lane == 0 ? 1.0 : ex;
}
// exclusive suffix sum over lanes (lane 63 gets 0)
CN_DEV double wave_exclusive_suffix_sum(double v) {
  const int lane = threadIdx.x & 63;
  double incl = v;
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const double o = shfl_down_d(incl, k);
    if (lane + k < 64) incl += o;
  }
  double ex = shfl_down_d(incl, 1);
  return lane == 63 ? 0.0 : ex;
}
CN_DEV float wave_sum(float v) {
#pragma unroll
  for (int k = 32; k > 0; k >>= 1) v += __shfl_xor(v, k);
  return v;
}

constexpr int kMaxPer = 4;   // samples per lane: N <= 256

struct RayState {
  int n0, cnt;                // this lane's sample range
  float sig[kMaxPer], z[kMaxPer], delta[kMaxPer], e[kMaxPer], alpha[kMaxPer], trans[kMaxPer];
  float T[kMaxPer], w[kMaxPer], c[kMaxPer][3];
};

// Forward of one ray (src/utils.py:35-43), lane-local part + scan.
CN_DEV void ray_forward(RayState& st, const float* sig, const float* rgb, const float* z, int N) {
  const int lane = threadIdx.x & 63;
  const int per = (N + 63) / 64;
  st.n0 = lane * per;
  st.cnt = max(0, min(per, N - st.n0));
  double prod = 1.0;
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    if (k < st.cnt) {
      const int s = st.n0 + k;
      st.sig[k] = sig[s];
      st.z[k] = z[s];
      st.delta[k] = s + 1 < N ? fadd_rn(z[s + 1], -z[s]) : 1e10f;
      st.e[k] = expf(-fmul_rn(st.sig[k], st.delta[k]));
      st.alpha[k] = 1.f - st.e[k];
      st.trans[k] = fadd_rn(1.f - st.alpha[k], 1e-10f);
      if (rgb) {
        st.c[k][0] = rgb[3 * s + 0];
        st.c[k][1] = rgb[3 * s + 1];
        st.c[k][2] = rgb[3 * s + 2];
      }
      prod *= (double)st.trans[k];
    }
  }
  double run = wave_exclusive_prod(prod);
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    if (k < st.cnt) {
      st.T[k] = (float)run;
      run *= (double)st.trans[k];
      st.w[k] = fmul_rn(st.alpha[k], st.T[k]);
    }
  }
}

// rgb (3), depth, weight sum of a ray (sums in float64, rounded once)
CN_DEV void ray_reduce(const RayState& st, float out[5]) {
  double acc[5] = {0, 0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    if (k < st.cnt) {
      acc[0] += (double)fmul_rn(st.w[k], st.c[k][0]);
      acc[1] += (double)fmul_rn(st.w[k], st.c[k][1]);
      acc[2] += (double)fmul_rn(st.w[k], st.c[k][2]);
      acc[3] += (double)fmul_rn(st.w[k], st.z[k]);
      acc[4] += (double)st.w[k];
    }
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    double v = acc[i];
#pragma unroll
    for (int k = 32; k > 0; k >>= 1) v += __hiloint2double(__shfl_xor(__double2hiint(v), k),
                                                           __shfl_xor(__double2loint(v), k));
    out[i] = (float)v;
  }
}

// Backward of one ray given d rgb_final (3) and d depth, as torch autograd.
CN_DEV void ray_backward(const RayState& st, const float g[3], float gd, int white_bg,
                         float* dsig, float* drgb) {
  const float gw_bg = white_bg ? -(g[0] + g[1] + g[2]) : 0.f;
  float dw[kMaxPer], wdT[kMaxPer];
  double part = 0.0;
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    if (k < st.cnt) {
      // d weights = sum_c g_c c_c  + d(wsum) + gd * z
      float v = fadd_rn(fadd_rn(fmul_rn(g[0], st.c[k][0]), fmul_rn(g[1], st.c[k][1])), fmul_rn(g[2], st.c[k][2]));
      v = fadd_rn(v, gw_bg);
      v = fadd_rn(v, fmul_rn(gd, st.z[k]));
      dw[k] = v;
      // grad of cumprod output T_k is dw_k * alpha_k; reversed cumsum of T_k * dT_k
      wdT[k] = fmul_rn(st.T[k], fmul_rn(v, st.alpha[k]));
      part += (double)wdT[k];
    }
  }
  // suffix sums strictly after each sample: across lanes, then within the lane
  double after = wave_exclusive_suffix_sum(part);
#pragma unroll
  for (int k = kMaxPer - 1; k >= 0; --k) {
    if (k < st.cnt) {
      const int s = st.n0 + k;
      // d trans_k = (sum_{j > k} T_j dT_j) / trans_k
      const float dtrans = (float)after / st.trans[k];
      after += (double)wdT[k];
      const float dalpha = fadd_rn(fmul_rn(dw[k], st.T[k]), -dtrans);
      dsig[s] = fmul_rn(fmul_rn(dalpha, st.e[k]), st.delta[k]);
      drgb[3 * s + 0] = fmul_rn(st.w[k], g[0]);
      drgb[3 * s + 1] = fmul_rn(st.w[k], g[1]);
      drgb[3 * s + 2] = fmul_rn(st.w[k], g[2]);
    }
  }
}

// rgb_out (R,3), depth (R): volume_rendering forward
__global__ __launch_bounds__(256) void composite_fwd_kernel(const float* __restrict__ sig, const float* __restrict__ rgb,
                                                            const float* __restrict__ z, int z_stride, int R, int N,
                                                            int white_bg, float* __restrict__ out_rgb,
                                                            float* __restrict__ out_depth, float* __restrict__ out_w) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  RayState st;
  ray_forward(st, sig + (size_t)r * N, rgb + (size_t)r * N * 3, z + (size_t)r * z_stride, N);
  float o[5];
  ray_reduce(st, o);
  if ((threadIdx.x & 63) == 0) {
    for (int c = 0; c < 3; ++c) out_rgb[3 * r + c] = white_bg ? fadd_rn(o[c] + 1.f, -o[4]) : o[c];
    out_depth[r] = o[3];
  }
  if (out_w)
    for (int k = 0; k < st.cnt; ++k) out_w[(size_t)r * N + st.n0 + k] = st.w[k];
}

__global__ __launch_bounds__(256) void composite_bwd_kernel(const float* __restrict__ sig, const float* __restrict__ rgb,
                                                            const float* __restrict__ z, int z_stride, int R, int N,
                                                            int white_bg, const float* __restrict__ g_rgb,
                                                            const float* __restrict__ g_depth,
                                                            float* __restrict__ dsig, float* __restrict__ drgb) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  RayState st;
  ray_forward(st, sig + (size_t)r * N, rgb + (size_t)r * N * 3, z + (size_t)r * z_stride, N);
  const float g[3] = {g_rgb[3 * r], g_rgb[3 * r + 1], g_rgb[3 * r + 2]};
  const float gd = g_depth ? g_depth[r] : 0.f;
  ray_backward(st, g, gd, white_bg, dsig + (size_t)r * N, drgb + (size_t)r * N * 3);
}

// Training: composite, per-ray squared error, d rgb of the chunk-mean MSE
// (chunk = `chunk` consecutive rays, src/trainer.py:69,75), composite backward.
__global__ __launch_bounds__(256) void render_loss_kernel(const float* __restrict__ sig, const float* __restrict__ rgb,
                                                          const float* __restrict__ z, int z_stride, int R, int N,
                                                          int white_bg, const float* __restrict__ gt, int chunk,
                                                          float* __restrict__ out_rgb, float* __restrict__ ray_se,
                                                          float* __restrict__ dsig, float* __restrict__ drgb) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  RayState st;
  ray_forward(st, sig + (size_t)r * N, rgb + (size_t)r * N * 3, z + (size_t)r * z_stride, N);
  float o[5];
  ray_reduce(st, o);
  float col[3], g[3];
  const int c0 = (r / chunk) * chunk;
  const int nb = min(chunk, R - c0);
  const float inv = 1.f / (float)(3 * nb);
  float se = 0.f;
  for (int c = 0; c < 3; ++c) {
    col[c] = white_bg ? fadd_rn(o[c] + 1.f, -o[4]) : o[c];
    const float diff = col[c] - gt[3 * r + c];
    se += diff * diff;
    // d mean(diff^2) = 2 * diff / numel
    g[c] = fmul_rn(fmul_rn(inv, 2.f), diff);
  }
  if ((threadIdx.x & 63) == 0) {
    for (int c = 0; c < 3; ++c) out_rgb[3 * r + c] = col[c];
    ray_se[r] = se;
  }
  ray_backward(st, g, 0.f, white_bg, dsig + (size_t)r * N, drgb + (size_t)r * N * 3);
}

// chunk-mean MSE values from per-ray squared errors (one block per chunk)
__global__ __launch_bounds__(256) void chunk_loss_kernel(const float* __restrict__ ray_se, int R, int chunk,
                                                         float* __restrict__ loss) {
  __shared__ double red[256];
  const int c = blockIdx.x;
  const int a = c * chunk, b = min(R, a + chunk);
  double s = 0.0;
  for (int r = a + threadIdx.x; r < b; r += 256) s += ray_se[r];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[c] = (float)(red[0] / (3.0 * (b - a)));
}

// ---------------------------------------------------------------- fine pass
// Hierarchical ("coarse + fine") sampling: the BASELINE configs' 64 + 64
// samples.  The reference has no fine pass, so this
// follows NeRF's sample_pdf with the CodeNeRF MLP shared by both passes;
// oracle: oracle/ref_cpu.py sample_pdf / fine_render_loss (parity unpinned).

// Importance samples of one ray per wave: bins = midpoints of the coarse z,
// pdf = (w[1:-1] + 1e-5) / sum, cdf = [0, cumsum] (float64, rounded once),
// u_j = (j + rnd_j) / Nf (stratified, so z_f comes out sorted), z_f = inverse
// cdf with NeRF's degenerate-bin rule (denom < 1e-5 -> 1).
constexpr int kMaxRaySamples = 64 * kMaxPer;

__global__ __launch_bounds__(256) void sample_pdf_kernel(const float* __restrict__ sig, const float* __restrict__ z,
                                                         int z_stride, int R, int Nc,
                                                         const float* __restrict__ rnd, int Nf,
                                                         float* __restrict__ zf) {
  __shared__ float cdf_s[4][kMaxRaySamples], bin_s[4][kMaxRaySamples];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + wv;
  if (r >= R) return;                       // wave-uniform; no block barriers below
  const float* zr = z + (size_t)r * z_stride;
  RayState st;
  ray_forward(st, sig + (size_t)r * Nc, nullptr, zr, Nc);
  // interior weights s = 1 .. Nc-2, +1e-5 (float, as torch: weights + 1e-5)
  float wv_[kMaxPer];
  double part = 0.0;
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    const int s = st.n0 + k;
    wv_[k] = 0.f;
    if (k < st.cnt && s >= 1 && s <= Nc - 2) {
      wv_[k] = st.w[k] + 1e-5f;
      part += (double)wv_[k];
    }
  }
  // exclusive prefix over lanes
  double incl = part;
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const double o = shfl_up_d(incl, k);
    if (lane >= k) incl += o;
  }
  double total = incl;
  total = __hiloint2double(__shfl(__double2hiint(total), 63), __shfl(__double2loint(total), 63));
  double run = incl - part;
  float* cdf = cdf_s[wv];
  float* bins = bin_s[wv];
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    const int s = st.n0 + k;
    if (k < st.cnt) {
      run += (double)wv_[k];
      // cdf[i] = sum_{s=1..i} / total for i = 1 .. Nc-2; cdf[0] = 0
      if (s >= 1 && s <= Nc - 2) cdf[s] = (float)(run / total);
      if (s == 0) cdf[0] = 0.f;
      if (s + 1 < Nc) bins[s] = fmul_rn(0.5f, fadd_rn(zr[s], zr[s + 1]));
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int nb = Nc - 1;                    // cdf / bin entries
  for (int j = lane; j < Nf; j += 64) {
    const float u = (float)j + rnd[(size_t)r * Nf + j];
    const float uu = u / (float)Nf;
    // searchsorted(cdf, uu, right=True): first index with cdf > uu
    int lo = 0, hi = nb;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf[mid] <= uu) lo = mid + 1; else hi = mid;
    }
    const int below = max(0, lo - 1), above = min(nb - 1, lo);
    const float cb = cdf[below], ca = cdf[above];
    const float bb = bins[below], ba = bins[above];
    float denom = fadd_rn(ca, -cb);
    if (denom < 1e-5f) denom = 1.f;
    const float t = fadd_rn(uu, -cb) / denom;
    zf[(size_t)r * Nf + j] = fadd_rn(bb, fmul_rn(t, fadd_rn(ba, -bb)));
  }
}

// Fine composite + chunk-mean MSE + backward over the union of the coarse
// and fine samples of each ray (merged by z; a coarse sample precedes a fine
// one at equal z).  dsig_c / drgb_c are ACCUMULATED into (they already hold
// the coarse loss's gradient); dsig_f / drgb_f are written.
__global__ __launch_bounds__(256) void fine_render_loss_kernel(
    const float* __restrict__ sig_c, const float* __restrict__ rgb_c, const float* __restrict__ zc, int zc_stride,
    int Nc, const float* __restrict__ sig_f, const float* __restrict__ rgb_f, const float* __restrict__ zf, int Nf,
    int R, int white_bg, const float* __restrict__ gt, int chunk, float* __restrict__ out_rgb,
    float* __restrict__ ray_se, float* __restrict__ dsig_c, float* __restrict__ drgb_c,
    float* __restrict__ dsig_f, float* __restrict__ drgb_f) {
  __shared__ float m_sig[4][kMaxRaySamples], m_z[4][kMaxRaySamples], m_rgb[4][kMaxRaySamples * 3];
  __shared__ float m_dsig[4][kMaxRaySamples], m_drgb[4][kMaxRaySamples * 3];
  __shared__ int m_src[4][kMaxRaySamples];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + wv;
  if (r >= R) return;                       // wave-uniform; only wave-level sync below
  const int N = Nc + Nf;
  const float* zcr = zc + (size_t)r * zc_stride;
  const float* zfr = zf + (size_t)r * Nf;
  auto wave_sync = [] {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  // Every merged slot starts as "no source": with non-finite z (diverged
  // weights) the two rank computations below need not form a permutation, and
  // an unwritten slot must not scatter through an undefined index.
  for (int p = lane; p < N; p += 64) m_src[wv][p] = -1;
  // the ray's coarse and fine z staged in LDS (m_dsig is written only by the
  // backward below): the rank searches' dependent reads then cost LDS, not
  // global-memory, latency
  float* zs = m_dsig[wv];
  for (int i = lane; i < Nc; i += 64) zs[i] = zcr[i];
  for (int j = lane; j < Nf; j += 64) zs[Nc + j] = zfr[j];
  wave_sync();
  // merged position = own index + number of the other list's samples before it
  for (int i = lane; i < Nc; i += 64) {
    const float v = zs[i];
    int lo = 0, hi = Nf;                    // count zf < v
    while (lo < hi) { const int mid = (lo + hi) >> 1; if (zs[Nc + mid] < v) lo = mid + 1; else hi = mid; }
    const int p = i + lo;
    const size_t g = (size_t)r * Nc + i;
    m_sig[wv][p] = sig_c[g];
    m_z[wv][p] = v;
    m_rgb[wv][3 * p + 0] = rgb_c[3 * g + 0];
    m_rgb[wv][3 * p + 1] = rgb_c[3 * g + 1];
    m_rgb[wv][3 * p + 2] = rgb_c[3 * g + 2];
    m_src[wv][p] = i;
  }
  for (int j = lane; j < Nf; j += 64) {
    const float v = zs[Nc + j];
    int lo = 0, hi = Nc;                    // count zc <= v
    while (lo < hi) { const int mid = (lo + hi) >> 1; if (zs[mid] <= v) lo = mid + 1; else hi = mid; }
    const int p = j + lo;
    const size_t g = (size_t)r * Nf + j;
    m_sig[wv][p] = sig_f[g];
    m_z[wv][p] = v;
    m_rgb[wv][3 * p + 0] = rgb_f[3 * g + 0];
    m_rgb[wv][3 * p + 1] = rgb_f[3 * g + 1];
    m_rgb[wv][3 * p + 2] = rgb_f[3 * g + 2];
    m_src[wv][p] = Nc + j;
  }
  wave_sync();
  RayState st;
  ray_forward(st, m_sig[wv], m_rgb[wv], m_z[wv], N);
  float o[5];
  ray_reduce(st, o);
  float col[3], gr[3];
  const int c0 = (r / chunk) * chunk;
  const int nbr = min(chunk, R - c0);
  const float inv = 1.f / (float)(3 * nbr);
  float se = 0.f;
  for (int c = 0; c < 3; ++c) {
    col[c] = white_bg ? fadd_rn(o[c] + 1.f, -o[4]) : o[c];
    const float diff = col[c] - gt[3 * r + c];
    se += diff * diff;
    gr[c] = fmul_rn(fmul_rn(inv, 2.f), diff);
  }
  if (lane == 0) {
    for (int c = 0; c < 3; ++c) out_rgb[3 * r + c] = col[c];
    ray_se[r] = se;
  }
  ray_backward(st, gr, 0.f, white_bg, m_dsig[wv], m_drgb[wv]);
  wave_sync();
  for (int p = lane; p < N; p += 64) {
    const int src = m_src[wv][p];
    if (src < 0) continue;
    if (src < Nc) {
      const size_t g = (size_t)r * Nc + src;
      dsig_c[g] += m_dsig[wv][p];
      for (int c = 0; c < 3; ++c) drgb_c[3 * g + c] += m_drgb[wv][3 * p + c];
    } else {
      const size_t g = (size_t)r * Nf + (src - Nc);
      dsig_f[g] = m_dsig[wv][p];
      for (int c = 0; c < 3; ++c) drgb_f[3 * g + c] = m_drgb[wv][3 * p + c];
    }
  }
}

// ---------------------------------------------------------------- misc
__global__ __launch_bounds__(256) void stratified_points_kernel(const float* __restrict__ ro, const float* __restrict__ vd,
                                                                const float* __restrict__ z, int z_stride, int R, int N,
                                                                float* __restrict__ xyz, float* __restrict__ vrep) {
  const int m = blockIdx.x * 256 + threadIdx.x;
  if (m >= R * N) return;
  const int r = m / N, s = m - r * N;
  const float zz = z[(size_t)r * z_stride + s];
  for (int a = 0; a < 3; ++a) {
    const float d = vd[3 * r + a];
    xyz[3 * m + a] = fadd_rn(ro[3 * r + a], fmul_rn(d, zz));
    vrep[3 * m + a] = d;
  }
}

}  // namespace cn
