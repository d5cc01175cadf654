// C ABI of the CodeNeRF gfx950 hot path (include/codenerf.h).
#include <stdio.h>
#include <string.h>
#include <algorithm>
#include <mutex>
#include <cmath>
#include <string>
#include <vector>
#include <hip/hip_ext.h>

#include "../../include/codenerf.h"
#include "chain_inst.h"
#include "latent_args.h"
#include "dw.hip"
#include "optim.hip"
#include "render.hip"
#include "probe.hip"

using namespace cn;

struct cn_plan {
  ChainSet cs;
  // packing tables (host), uploaded to the device by the first cn_pack_weights
  // so that creating a plan and querying sizes / validating arguments needs no
  // device
  std::vector<int32_t> h_fwd_idx, h_bwd_idx;
  int32_t* d_fwd_idx = nullptr;
  int32_t* d_bwd_idx = nullptr;
  int fwd_n = 0, bwd_n = 0;
  std::mutex upload_mu;
};

namespace {
thread_local std::string g_err;

int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}
int check(hipError_t e, const char* what) {
  if (e != hipSuccess) return fail(std::string(what) + ": " + hipGetErrorString(e));
  return 0;
}
int launch_check(const char* what) { return check(hipGetLastError(), what); }
hipStream_t S(void* s) { return (hipStream_t)s; }
int grid_for(long n, int per) { return (int)((n + per - 1) / per); }

// cn_time_next_launch: the next hot kernel (chain, dW, bias-sum) launched by
// this thread records these events from its own dispatch packet
// (hipExtLaunchKernel) -- no marker packets between kernels, whose ~7 us
// each the bench's per-kernel timers otherwise added to the step
thread_local hipEvent_t g_ev_start = nullptr, g_ev_stop = nullptr;
template <typename K, typename... A>
void launch_hot(K kernel, dim3 grid, dim3 block, hipStream_t s, A... args) {
  if (g_ev_start) {
    hipExtLaunchKernelGGL(kernel, grid, block, 0, s, g_ev_start, g_ev_stop, 0, args...);
    g_ev_start = g_ev_stop = nullptr;
  } else {
    hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
  }
}
// Armed events belong to the NEXT hot entry call only: every entry point that
// may launch a hot kernel holds one of these, so an error return, a call with
// nothing to launch (cn_mlp_dbias without injections) or a failed dW setup
// disarms them instead of leaving them for an unrelated later launch.
struct HotCallScope {
  ~HotCallScope() { g_ev_start = g_ev_stop = nullptr; }
};
}  // namespace

extern "C" {

int cn_abi_version(void) { return CN_ABI_VERSION; }
const char* cn_last_error(void) { return g_err.c_str(); }

int cn_stream_wait(void* waiter, void* signaller) {
  // a ring of fence-less events per thread AND per device (an event must be
  // recorded on a stream of the device it was created on): hipStreamWaitEvent
  // captures the event's current record, so reusing one 16 records later is
  // safe.  The event is created with the signaller's device current.
  constexpr int kRing = 16, kDevs = 64;
  thread_local hipEvent_t ring[kDevs][kRing] = {};
  thread_local int next[kDevs] = {};
  hipDevice_t dev = 0;
  if (signaller) {
    if (check(hipStreamGetDevice(S(signaller), &dev), "cn_stream_wait: hipStreamGetDevice")) return -1;
  } else if (check(hipGetDevice(&dev), "cn_stream_wait: hipGetDevice")) {
    return -1;
  }
  if (dev < 0 || dev >= kDevs) return fail("cn_stream_wait: device index out of range");
  hipEvent_t& e = ring[dev][next[dev]];
  next[dev] = (next[dev] + 1) % kRing;
  if (!e) {
    int cur = 0;
    if (check(hipGetDevice(&cur), "cn_stream_wait: hipGetDevice")) return -1;
    if (cur != dev && check(hipSetDevice(dev), "cn_stream_wait: hipSetDevice")) return -1;
    const int rc = check(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventDisableSystemFence),
                         "cn_stream_wait: hipEventCreateWithFlags");
    if (cur != dev) (void)hipSetDevice(cur);
    if (rc) {
      e = nullptr;
      return -1;
    }
  }
  if (check(hipEventRecord(e, S(signaller)), "cn_stream_wait: hipEventRecord")) return -1;
  return check(hipStreamWaitEvent(S(waiter), e, 0), "cn_stream_wait: hipStreamWaitEvent");
}

int cn_time_next_launch(void* start_event, void* stop_event) {
  if ((start_event == nullptr) != (stop_event == nullptr)) return fail("cn_time_next_launch: give both events or none");
  g_ev_start = (hipEvent_t)start_event;
  g_ev_stop = (hipEvent_t)stop_event;
  return 0;
}

int cn_plan_create(int shape_blocks, int texture_blocks, int W, int num_xyz_freq, int num_dir_freq,
                   int latent_dim, int precision, cn_plan** out) {
  if (!out) return fail("cn_plan_create: out is NULL");
  *out = nullptr;
  if (W != 256 || latent_dim != 256 || num_xyz_freq != 10 || num_dir_freq != 4)
    return fail("cn_plan_create: unsupported net (need W=latent_dim=256, num_xyz_freq=10, num_dir_freq=4)");
  if (precision != CN_FP32 && precision != CN_BF16 && precision != CN_BF16X3 && precision != CN_BF16X3F)
    return fail("cn_plan_create: precision must be CN_FP32, CN_BF16, CN_BF16X3 or CN_BF16X3F");
  ChainSet cs;
  if (shape_blocks == 3 && texture_blocks == 1)
    cs = precision == CN_BF16X3F ? chain_set_bf16x3f_3_1() : precision == CN_BF16X3 ? chain_set_bf16x3_3_1()
       : precision ? chain_set_bf16_3_1() : chain_set_fp32_3_1();
  else if (shape_blocks == 2 && texture_blocks == 1)
    cs = precision == CN_BF16X3F ? chain_set_bf16x3f_2_1() : precision == CN_BF16X3 ? chain_set_bf16x3_2_1()
       : precision ? chain_set_bf16_2_1() : chain_set_fp32_2_1();
  else return fail("cn_plan_create: unsupported (shape_blocks, texture_blocks); built: (3,1), (2,1)");
  cn_plan* p = new cn_plan();
  p->cs = cs;
  p->h_fwd_idx = cs.fwd_table();
  p->h_bwd_idx = cs.bwd_table();
  p->fwd_n = (int)p->h_fwd_idx.size();
  p->bwd_n = (int)p->h_bwd_idx.size();
  *out = p;
  return 0;
}

static int upload_tables(cn_plan* p) {
  std::lock_guard<std::mutex> lk(p->upload_mu);
  if (p->d_fwd_idx) return 0;
  int32_t *f = nullptr, *b = nullptr;
  if (check(hipMalloc(&f, p->h_fwd_idx.size() * 4), "hipMalloc") ||
      check(hipMalloc(&b, p->h_bwd_idx.size() * 4), "hipMalloc") ||
      check(hipMemcpy(f, p->h_fwd_idx.data(), p->h_fwd_idx.size() * 4, hipMemcpyHostToDevice), "hipMemcpy") ||
      check(hipMemcpy(b, p->h_bwd_idx.data(), p->h_bwd_idx.size() * 4, hipMemcpyHostToDevice), "hipMemcpy")) {
    if (f) (void)hipFree(f);
    if (b) (void)hipFree(b);
    return -1;
  }
  p->d_bwd_idx = b;
  p->d_fwd_idx = f;
  return 0;
}

// Sample-count guard shared by every per-sample entry point: sample indices
// (3 m, 4 m) are 32-bit in the kernels.  The activation planes themselves
// have no size limit (each wave addresses its own slab through a 64-bit
// descriptor base, chain.hip slab_rsrc).
static int check_samples(long long M, const char* who) {
  if (M <= 0) return fail(std::string(who) + ": M must be positive");
  if (M > CN_MAX_SAMPLES)
    return fail(std::string(who) + ": " + std::to_string(M) + " samples exceed CN_MAX_SAMPLES (" +
                std::to_string((long long)CN_MAX_SAMPLES) + ") per call; split the rays into parts");
  return 0;
}

void cn_plan_destroy(cn_plan* p) {
  if (!p) return;
  if (p->d_fwd_idx) (void)hipFree(p->d_fwd_idx);
  if (p->d_bwd_idx) (void)hipFree(p->d_bwd_idx);
  delete p;
}

int cn_plan_num_params(const cn_plan* p) { return p ? p->cs.n_params : -1; }
int cn_plan_num_inject(const cn_plan* p) { return p ? p->cs.n_inject : -1; }
int cn_pad_samples(const cn_plan* p, int M) {
  return p && M >= 0 && M <= CN_MAX_SAMPLES ? ((M + 255) / 256) * 256 : -1;
}
int cn_max_samples(void) { return CN_MAX_SAMPLES; }
size_t cn_packed_bytes(const cn_plan* p, int bwd) { return p ? (bwd ? p->cs.pack_bwd_bytes : p->cs.pack_fwd_bytes) : 0; }
size_t cn_blob_floats(const cn_plan* p) { return p ? (size_t)p->cs.blob_floats : 0; }
size_t cn_act_bytes(const cn_plan* p, int M) {
  return p && M > 0 && M <= CN_MAX_SAMPLES ? p->cs.layout(cn_pad_samples(p, M)).bytes : 0;
}
size_t cn_act_bytes_per_sample(const cn_plan* p) {
  return p ? p->cs.layout(1 << 20).bytes >> 20 : 0;
}
size_t cn_dw_ws_bytes(const cn_plan* p, int M) { return p ? p->cs.dw_ws_bytes(M) : 0; }

long long cn_act_plane(const cn_plan* p, int M, int kind, int index, int* width) {
  if (!p || M <= 0 || M > CN_MAX_SAMPLES) return -1;
  const ActLayout L = p->cs.layout(cn_pad_samples(p, M));
  int w = 0;
  long long off = -1;
  if ((kind == CN_PLANE_Y || kind == CN_PLANE_DA) && index >= 0 && index < kMaxPlanes) {
    w = (int)(kind == CN_PLANE_Y ? L.Yw[index] : L.dAw[index]);
    if (w > 0) off = (long long)(kind == CN_PLANE_Y ? L.Y[index] : L.dA[index]);
  } else if (kind == CN_PLANE_PE) {
    w = 64, off = (long long)L.pe;
  } else if (kind == CN_PLANE_DIR) {
    w = 32, off = (long long)L.dir;
  } else if (kind == CN_PLANE_MASKS) {
    w = (int)(L.mask_bytes_per_slab / 32), off = (long long)L.masks;
  } else if (kind == CN_PLANE_YLO && index >= 0 && index < kMaxPlanes && L.Ylo[index]) {
    w = (int)L.Yw[index], off = (long long)L.Ylo[index];
  } else if (kind == CN_PLANE_PELO && L.pelo) {
    w = 64, off = (long long)L.pelo;
  }
  if (width) *width = w;
  return off;
}

int cn_pack_weights(const cn_plan* p, const float* const* d_params, void* d_fwd, void* d_bwd, void* stream) {
  if (!p || !d_params) return fail("cn_pack_weights: NULL argument");
  if (!p->d_fwd_idx && upload_tables(const_cast<cn_plan*>(p))) return -1;
  const int bf16 = p->cs.prec;
  if (d_fwd) {
    hipLaunchKernelGGL(pack_kernel, dim3(grid_for(p->fwd_n, 256)), dim3(256), 0, S(stream), d_params,
                       p->d_fwd_idx, p->fwd_n, d_fwd, bf16);
    if (launch_check("pack_kernel(fwd)")) return -1;
  }
  if (d_bwd) {
    hipLaunchKernelGGL(pack_kernel, dim3(grid_for(p->bwd_n, 256)), dim3(256), 0, S(stream), d_params,
                       p->d_bwd_idx, p->bwd_n, d_bwd, bf16);
    if (launch_check("pack_kernel(bwd)")) return -1;
  }
  return 0;
}

int cn_latent_fwd(const cn_plan* p, const float* const* d_params, const float* d_shape, const float* d_tex,
                  float* d_blob, float* d_zvec, void* stream) {
  if (!p || !d_params || !d_shape || !d_tex || !d_blob || !d_zvec) return fail("cn_latent_fwd: NULL argument");
  LatentArgs a{d_params, d_shape, d_tex, d_blob, d_zvec};
  hipLaunchKernelGGL(p->cs.latent_fwd, dim3(p->cs.n_fwd_layers + 1), dim3(256), 0, S(stream), a);
  return launch_check("latent_fwd_kernel");
}

static int mlp_fwd_impl(int codes, const cn_plan* p, const void* d_pack, const float* d_blob, int M,
                        const float* d_xyz, const float* d_viewdir, const float* d_rays_o, const float* d_rays_d,
                        const float* d_z, int z_stride, int n_samples, float* d_sigma, float* d_rgb, void* d_act,
                        int act_M, int act_row0, void* stream) {
  HotCallScope hot;
  if (codes && !d_act) return fail("cn_mlp_fwd_codes: the activation workspace is required");
  if (!p || !d_pack || !d_blob || !d_sigma || !d_rgb) return fail("cn_mlp_fwd: NULL argument");
  if (check_samples(M, "cn_mlp_fwd")) return -1;
  ChainArgs a{};
  a.wpack = d_pack;
  a.bias = d_blob;
  a.M = M;
  if (d_xyz) {
    if (!d_viewdir) return fail("cn_mlp_fwd: xyz given without viewdir");
    a.mode = 0;
    a.xyz = d_xyz;
    a.vdir = d_viewdir;
    a.nsamp = 1;
  } else {
    if (!d_rays_o || !d_rays_d || !d_z || n_samples <= 0) return fail("cn_mlp_fwd: ray mode needs rays_o, rays_d, z, n_samples");
    if (M % n_samples) return fail("cn_mlp_fwd: M must be a multiple of n_samples in ray mode");
    if (z_stride != 0 && z_stride != n_samples) return fail("cn_mlp_fwd: z_stride must be 0 or n_samples");
    a.mode = 1;
    a.rays_o = d_rays_o;
    a.rays_d = d_rays_d;
    a.zvals = d_z;
    a.z_stride = z_stride;
    a.nsamp = n_samples;
  }
  a.sigma = d_sigma;
  a.rgb = d_rgb;
  const int Mp = cn_pad_samples(p, M);
  if (d_act) {
    // the workspace may be sized for act_M samples, this launch filling rows
    // [act_row0, act_row0 + Mp) of it (coarse and fine passes share one
    // workspace, so one backward / dW covers both)
    if (act_M <= 0) act_M = M;
    if (check_samples(act_M, "cn_mlp_fwd (act_M)")) return -1;
    if (act_row0 < 0 || act_row0 % p->cs.tile) return fail("cn_mlp_fwd: act_row0 must be a multiple of the tile");
    const int Ma = cn_pad_samples(p, act_M);
    if (act_row0 + Mp > Ma) return fail("cn_mlp_fwd: rows exceed the activation workspace");
    const ActLayout L = p->cs.layout(Ma);
    const size_t es = p->cs.prec ? 2 : 4;
    const size_t r0 = (size_t)act_row0;
    char* b = (char*)d_act;
    a.pe = b + L.pe + r0 * 64 * es;
    a.dir = b + L.dir + r0 * 32 * es;
    for (int i = 0; i < kMaxPlanes; ++i) {
      a.Y[i] = b + L.Y[i] + r0 * L.Yw[i] * es;
      a.dA[i] = b + L.dA[i] + r0 * L.dAw[i] * es;
    }
    a.d8 = b + L.d8 + r0 * 32 * es;
    a.spre = (float*)(b + L.spre) + r0;
    a.masks = (uint32_t*)(b + L.masks + (r0 / 32) * L.mask_bytes_per_slab);
    a.pelo = L.pelo ? b + L.pelo + r0 * 64 * es : nullptr;
    for (int i = 0; i < kMaxPlanes; ++i) a.Ylo[i] = L.Ylo[i] ? b + L.Ylo[i] + r0 * L.Yw[i] * es : nullptr;
  }
  const int grid = (Mp + p->cs.waves_fwd * 32 - 1) / (p->cs.waves_fwd * 32);
  launch_hot(d_act ? (codes ? p->cs.fwd_codes : p->cs.fwd_train) : p->cs.fwd_infer, dim3(grid),
             dim3(p->cs.waves_fwd * 64), S(stream), a);
  return launch_check("chain_kernel(fwd)");
}

int cn_mlp_fwd(const cn_plan* p, const void* d_pack, const float* d_blob, int M, const float* d_xyz,
               const float* d_viewdir, const float* d_rays_o, const float* d_rays_d, const float* d_z,
               int z_stride, int n_samples, float* d_sigma, float* d_rgb, void* d_act, int act_M, int act_row0,
               void* stream) {
  return mlp_fwd_impl(0, p, d_pack, d_blob, M, d_xyz, d_viewdir, d_rays_o, d_rays_d, d_z, z_stride, n_samples,
                      d_sigma, d_rgb, d_act, act_M, act_row0, stream);
}

int cn_mlp_fwd_codes(const cn_plan* p, const void* d_pack, const float* d_blob, int M, const float* d_xyz,
                     const float* d_viewdir, const float* d_rays_o, const float* d_rays_d, const float* d_z,
                     int z_stride, int n_samples, float* d_sigma, float* d_rgb, void* d_act, int act_M,
                     int act_row0, void* stream) {
  return mlp_fwd_impl(1, p, d_pack, d_blob, M, d_xyz, d_viewdir, d_rays_o, d_rays_d, d_z, z_stride, n_samples,
                      d_sigma, d_rgb, d_act, act_M, act_row0, stream);
}

static int mlp_bwd_impl(int codes, const cn_plan* p, const void* d_pack, const float* d_blob, int M,
                        const float* d_dsigma, const float* d_drgb, void* d_act, int act_M, int act_row0,
                        void* stream) {
  HotCallScope hot;
  if (!p || !d_pack || !d_blob || !d_dsigma || !d_drgb || !d_act) return fail("cn_mlp_bwd: NULL argument");
  if (check_samples(M, "cn_mlp_bwd")) return -1;
  ChainArgs a{};
  a.wpack = d_pack;
  a.bias = d_blob;
  a.M = M;
  a.dsigma = d_dsigma;
  a.drgb = d_drgb;
  const int Mp = cn_pad_samples(p, M);
  // rows [act_row0, act_row0 + Mp) of a workspace laid out for act_M samples
  if (act_M <= 0) act_M = M;
  if (check_samples(act_M, "cn_mlp_bwd (act_M)")) return -1;
  if (act_row0 < 0 || act_row0 % p->cs.tile) return fail("cn_mlp_bwd: act_row0 must be a multiple of the tile");
  const int Ma = cn_pad_samples(p, act_M);
  if (act_row0 + Mp > Ma) return fail("cn_mlp_bwd: rows exceed the activation workspace");
  const ActLayout L = p->cs.layout(Ma);
  const size_t es = p->cs.prec ? 2 : 4;
  const size_t r0 = (size_t)act_row0;
  char* b = (char*)d_act;
  a.pe = b + L.pe + r0 * 64 * es;
  a.dir = b + L.dir + r0 * 32 * es;
  for (int i = 0; i < kMaxPlanes; ++i) {
    a.Y[i] = b + L.Y[i] + r0 * L.Yw[i] * es;
    a.dA[i] = b + L.dA[i] + r0 * L.dAw[i] * es;
  }
  a.d8 = b + L.d8 + r0 * 32 * es;
  a.spre = (float*)(b + L.spre) + r0;
  a.masks = (uint32_t*)(b + L.masks + (r0 / 32) * L.mask_bytes_per_slab);
  launch_hot(codes ? p->cs.bwd_codes : p->cs.bwd, dim3((Mp + p->cs.waves_bwd * 32 - 1) / (p->cs.waves_bwd * 32)),
             dim3(p->cs.waves_bwd * 64), S(stream), a);
  return launch_check("chain_kernel(bwd)");
}

int cn_mlp_bwd(const cn_plan* p, const void* d_pack, const float* d_blob, int M, const float* d_dsigma,
               const float* d_drgb, void* d_act, void* stream) {
  return mlp_bwd_impl(0, p, d_pack, d_blob, M, d_dsigma, d_drgb, d_act, M, 0, stream);
}

int cn_mlp_bwd_rows(const cn_plan* p, const void* d_pack, const float* d_blob, int M, const float* d_dsigma,
                    const float* d_drgb, void* d_act, int act_M, int act_row0, void* stream) {
  return mlp_bwd_impl(0, p, d_pack, d_blob, M, d_dsigma, d_drgb, d_act, act_M, act_row0, stream);
}

int cn_mlp_bwd_codes(const cn_plan* p, const void* d_pack, const float* d_blob, int M, const float* d_dsigma,
                     const float* d_drgb, void* d_act, int act_M, int act_row0, void* stream) {
  return mlp_bwd_impl(1, p, d_pack, d_blob, M, d_dsigma, d_drgb, d_act, act_M, act_row0, stream);
}

static int mlp_dw_impl(const cn_plan* p, void* d_act, int act_M, int act_row0, int M, const float* d_zvec,
                       const float* const* d_params, float* const* d_grads, float* d_dbuf, int db_accum, int nwg_req,
                       void* d_ws, void* stream) {
  HotCallScope hot;
  if (!p || !d_act || !d_zvec || !d_params || !d_grads || !d_dbuf || !d_ws) return fail("cn_mlp_dw: NULL argument");
  if (check_samples(M, "cn_mlp_dw")) return -1;
  if (act_M <= 0) act_M = M;
  if (check_samples(act_M, "cn_mlp_dw (act_M)")) return -1;
  if (act_row0 < 0 || act_row0 % 256 || act_row0 + cn_pad_samples(p, M) > cn_pad_samples(p, act_M))
    return fail("cn_mlp_dw: rows exceed the activation workspace (act_row0 must be a multiple of 256)");
  DwArgs dw;
  DwRedArgs red;
  if (nwg_req < 0 || nwg_req > 256) return fail("cn_mlp_dw_rows: n_workgroups must be in [0, 256]");
  const int nwg = p->cs.dw_setup((char*)d_act, act_M, act_row0, M, nwg_req, d_zvec, d_dbuf, (char*)d_ws, &dw, &red);
  if (nwg <= 0) return fail("cn_mlp_dw: schedule does not fit (too few workgroups for the layer sizes?)");
  red.grads = d_grads;
  red.db_accum = db_accum ? 1 : 0;
  if (p->cs.prec) launch_hot(dw_kernel<CN_P_BF16>, dim3(nwg), dim3(512), S(stream), dw);
  else launch_hot(dw_kernel<CN_P_FP32>, dim3(nwg), dim3(512), S(stream), dw);
  if (launch_check("dw_kernel")) return -1;
  hipLaunchKernelGGL(dw_reduce_kernel, dim3(grid_for(red.prefix[red.nprob], 256)), dim3(256), 0, S(stream), red);
  if (launch_check("dw_reduce_kernel")) return -1;
  DwFoldArgs f = p->cs.fold_args();
  f.fold = red.fold;
  f.params = d_params;
  f.grads = d_grads;
  hipLaunchKernelGGL(dw_fold_kernel, dim3(17, 17, 2), dim3(256), 0, S(stream), f);
  return launch_check("dw_fold_kernel");
}

int cn_mlp_dw(const cn_plan* p, void* d_act, int M, const float* d_zvec, const float* const* d_params,
              float* const* d_grads, float* d_dbuf, void* d_ws, void* stream) {
  return mlp_dw_impl(p, d_act, M, 0, M, d_zvec, d_params, d_grads, d_dbuf, 0, 0, d_ws, stream);
}

int cn_mlp_dw_rows(const cn_plan* p, void* d_act, int act_M, int act_row0, int M, const float* d_zvec,
                   const float* const* d_params, float* const* d_grads, float* d_dbuf, int db_accum,
                   int n_workgroups, void* d_ws, void* stream) {
  return mlp_dw_impl(p, d_act, act_M, act_row0, M, d_zvec, d_params, d_grads, d_dbuf, db_accum, n_workgroups, d_ws,
                     stream);
}

int cn_mlp_dbias(const cn_plan* p, void* d_act, int act_M, int M, float* d_dbuf, void* d_ws, void* stream) {
  HotCallScope hot;
  if (!p || !d_act || !d_dbuf || !d_ws) return fail("cn_mlp_dbias: NULL argument");
  if (check_samples(M, "cn_mlp_dbias")) return -1;
  if (act_M <= 0) act_M = M;
  if (check_samples(act_M, "cn_mlp_dbias (act_M)")) return -1;
  DbArgs db;
  if (p->cs.db_setup((char*)d_act, act_M, M, d_dbuf, (char*)d_ws, &db) < 0)
    return fail("cn_mlp_dbias: rows exceed the workspace or unsupported plane width");
  if (db.ninj <= 0) return 0;
  if (p->cs.prec) launch_hot(db_kernel<CN_P_BF16>, dim3(kDbBlocks, db.ninj), dim3(256), S(stream), db);
  else launch_hot(db_kernel<CN_P_FP32>, dim3(kDbBlocks, db.ninj), dim3(256), S(stream), db);
  if (launch_check("db_kernel")) return -1;
  hipLaunchKernelGGL(db_reduce_kernel, dim3(db.ninj), dim3(256), 0, S(stream), db);
  return launch_check("db_reduce_kernel");
}

int cn_latent_bwd(const cn_plan* p, const float* const* d_params, float* const* d_grads, const float* d_shape,
                  const float* d_tex, const float* d_zvec, const float* d_dbuf, float* d_scratch, float* d_dshape,
                  float* d_dtex, float reg_coef, float* d_reg_out, void* stream) {
  if (!p || !d_params || !d_grads || !d_shape || !d_tex || !d_zvec || !d_dbuf || !d_scratch || !d_dshape || !d_dtex)
    return fail("cn_latent_bwd: NULL argument");
  LatentBwdArgs a{d_params, d_grads, d_shape, d_tex, d_zvec, d_dbuf, d_scratch, d_dshape, d_dtex, reg_coef, d_reg_out};
  hipLaunchKernelGGL(p->cs.latent_bwd, dim3(p->cs.n_inject, kLatentRowBlocks), dim3(256), 0, S(stream), a);
  if (launch_check("latent_bwd_kernel")) return -1;
  hipLaunchKernelGGL(p->cs.code_grad, dim3(2), dim3(1024), 0, S(stream), a);
  return launch_check("code_grad_kernel");
}

int cn_get_rays(int H, int W, double focal, int focal_is_f64, const float* d_c2w, float* d_ro, float* d_vd,
                void* stream) {
  if (!d_c2w || !d_ro || !d_vd || H <= 0 || W <= 0) return fail("cn_get_rays: bad argument");
  if (check_samples((long long)H * W, "cn_get_rays")) return -1;
  hipLaunchKernelGGL(get_rays_kernel, dim3(grid_for((long)H * W, 256)), dim3(256), 0, S(stream), H, W, focal,
                     focal_is_f64, d_c2w, d_ro, d_vd);
  return launch_check("get_rays_kernel");
}

int cn_sample_points(const float* d_ro, const float* d_vd, const float* d_z, int z_stride, int R, int N,
                     float* d_xyz, float* d_vrep, void* stream) {
  if (!d_ro || !d_vd || !d_z || !d_xyz || !d_vrep || R <= 0 || N <= 0) return fail("cn_sample_points: bad argument");
  if (check_samples((long long)R * N, "cn_sample_points")) return -1;
  hipLaunchKernelGGL(stratified_points_kernel, dim3(grid_for((long)R * N, 256)), dim3(256), 0, S(stream), d_ro,
                     d_vd, d_z, z_stride, R, N, d_xyz, d_vrep);
  return launch_check("stratified_points_kernel");
}

static int check_rn(int R, int N, const char* who) {
  if (R <= 0 || N <= 0) return fail(std::string(who) + ": R and N must be positive");
  if (N > 64 * kMaxPer) return fail(std::string(who) + ": at most 256 samples per ray");
  if (check_samples((long long)R * N, who)) return -1;
  return 0;
}

int cn_composite_fwd(const float* d_sigma, const float* d_rgb, const float* d_z, int z_stride, int R, int N,
                     int white_bg, float* d_out_rgb, float* d_out_depth, float* d_w, void* stream) {
  if (!d_sigma || !d_rgb || !d_z || !d_out_rgb || !d_out_depth) return fail("cn_composite_fwd: NULL argument");
  if (check_rn(R, N, "cn_composite_fwd")) return -1;
  hipLaunchKernelGGL(composite_fwd_kernel, dim3(grid_for(R, 4)), dim3(256), 0, S(stream), d_sigma, d_rgb, d_z,
                     z_stride, R, N, white_bg, d_out_rgb, d_out_depth, d_w);
  return launch_check("composite_fwd_kernel");
}

int cn_composite_bwd(const float* d_sigma, const float* d_rgb, const float* d_z, int z_stride, int R, int N,
                     int white_bg, const float* d_grgb, const float* d_gdepth, float* d_dsig, float* d_drgb,
                     void* stream) {
  if (!d_sigma || !d_rgb || !d_z || !d_grgb || !d_dsig || !d_drgb) return fail("cn_composite_bwd: NULL argument");
  if (check_rn(R, N, "cn_composite_bwd")) return -1;
  hipLaunchKernelGGL(composite_bwd_kernel, dim3(grid_for(R, 4)), dim3(256), 0, S(stream), d_sigma, d_rgb, d_z,
                     z_stride, R, N, white_bg, d_grgb, d_gdepth, d_dsig, d_drgb);
  return launch_check("composite_bwd_kernel");
}

int cn_render_loss(const float* d_sigma, const float* d_rgb, const float* d_z, int z_stride, int R, int N,
                   int white_bg, const float* d_gt, int chunk, float* d_out_rgb, float* d_ray_se,
                   float* d_chunk_loss, float* d_dsig, float* d_drgb, void* stream) {
  if (!d_sigma || !d_rgb || !d_z || !d_gt || !d_out_rgb || !d_ray_se || !d_chunk_loss || !d_dsig || !d_drgb)
    return fail("cn_render_loss: NULL argument");
  if (check_rn(R, N, "cn_render_loss")) return -1;
  if (chunk <= 0) return fail("cn_render_loss: chunk must be positive");
  hipLaunchKernelGGL(render_loss_kernel, dim3(grid_for(R, 4)), dim3(256), 0, S(stream), d_sigma, d_rgb, d_z,
                     z_stride, R, N, white_bg, d_gt, chunk, d_out_rgb, d_ray_se, d_dsig, d_drgb);
  if (launch_check("render_loss_kernel")) return -1;
  hipLaunchKernelGGL(chunk_loss_kernel, dim3(grid_for(R, chunk)), dim3(256), 0, S(stream), d_ray_se, R, chunk,
                     d_chunk_loss);
  return launch_check("chunk_loss_kernel");
}

int cn_sample_pdf(const float* d_sigma_c, const float* d_z_c, int zc_stride, int R, int Nc, const float* d_rand,
                  int Nf, float* d_z_f, void* stream) {
  if (!d_sigma_c || !d_z_c || !d_rand || !d_z_f) return fail("cn_sample_pdf: NULL argument");
  if (check_rn(R, Nc, "cn_sample_pdf")) return -1;
  if (Nc < 3) return fail("cn_sample_pdf: need at least 3 coarse samples");
  if (Nf <= 0) return fail("cn_sample_pdf: Nf must be positive");
  if (zc_stride != 0 && zc_stride != Nc) return fail("cn_sample_pdf: zc_stride must be 0 or Nc");
  hipLaunchKernelGGL(sample_pdf_kernel, dim3(grid_for(R, 4)), dim3(256), 0, S(stream), d_sigma_c, d_z_c, zc_stride,
                     R, Nc, d_rand, Nf, d_z_f);
  return launch_check("sample_pdf_kernel");
}

int cn_render_loss_fine(const float* d_sigma_c, const float* d_rgb_c, const float* d_z_c, int zc_stride, int Nc,
                        const float* d_sigma_f, const float* d_rgb_f, const float* d_z_f, int Nf, int R,
                        int white_bg, const float* d_gt, int chunk, float* d_out_rgb, float* d_ray_se,
                        float* d_chunk_loss, float* d_dsig_c, float* d_drgb_c, float* d_dsig_f, float* d_drgb_f,
                        void* stream) {
  if (!d_sigma_c || !d_rgb_c || !d_z_c || !d_sigma_f || !d_rgb_f || !d_z_f || !d_gt || !d_out_rgb || !d_ray_se ||
      !d_chunk_loss || !d_dsig_c || !d_drgb_c || !d_dsig_f || !d_drgb_f)
    return fail("cn_render_loss_fine: NULL argument");
  if (Nc <= 0 || Nf <= 0) return fail("cn_render_loss_fine: Nc and Nf must be positive");
  if (check_rn(R, Nc + Nf, "cn_render_loss_fine")) return -1;
  if (zc_stride != 0 && zc_stride != Nc) return fail("cn_render_loss_fine: zc_stride must be 0 or Nc");
  if (chunk <= 0) return fail("cn_render_loss_fine: chunk must be positive");
  hipLaunchKernelGGL(fine_render_loss_kernel, dim3(grid_for(R, 4)), dim3(256), 0, S(stream), d_sigma_c, d_rgb_c,
                     d_z_c, zc_stride, Nc, d_sigma_f, d_rgb_f, d_z_f, Nf, R, white_bg, d_gt, chunk, d_out_rgb,
                     d_ray_se, d_dsig_c, d_drgb_c, d_dsig_f, d_drgb_f);
  if (launch_check("fine_render_loss_kernel")) return -1;
  hipLaunchKernelGGL(chunk_loss_kernel, dim3(grid_for(R, chunk)), dim3(256), 0, S(stream), d_ray_se, R, chunk,
                     d_chunk_loss);
  return launch_check("chunk_loss_kernel");
}

static int adamw_impl(int nseg, float* const* p, float* const* g, float* const* m, float* const* v, const int* n,
                      const double* lr, double wd, double beta1, double beta2, double eps, int step, int zero_grad,
                      void* stream) {
  if (nseg <= 0 || !p || !g || !m || !v || !n || !lr) return fail("cn_adamw_step: bad argument");
  if (step < 1) return fail("cn_adamw_step: step must be >= 1");
  const double bc1 = 1.0 - std::pow(beta1, step);
  const double bc2 = 1.0 - std::pow(beta2, step);
  for (int base = 0; base < nseg; base += kAdamMaxSeg) {
    AdamArgs a{};
    a.nseg = std::min(kAdamMaxSeg, nseg - base);
    long total = 0;
    for (int i = 0; i < a.nseg; ++i) {
      const int k = base + i;
      a.s[i] = AdamSeg{p[k], g[k], m[k], v[k], n[k], (float)(1.0 - lr[k] * wd), (float)(-(lr[k] / bc1))};
      a.prefix[i] = (int)total;
      total += n[k];
    }
    a.prefix[a.nseg] = (int)total;
    a.lerp_w = (float)(1.0 - beta1);
    a.beta2 = (float)beta2;
    a.one_m_beta2 = (float)(1.0 - beta2);
    a.bc2_sqrt = (float)std::sqrt(bc2);
    a.eps = (float)eps;
    a.zero_grad = zero_grad;
    const int grid = std::min(2048, grid_for(total, 256));
    hipLaunchKernelGGL(adamw_kernel, dim3(grid), dim3(256), 0, S(stream), a);
    if (launch_check("adamw_kernel")) return -1;
  }
  return 0;
}

int cn_adamw_step(int nseg, float* const* p, const float* const* g, float* const* m, float* const* v,
                  const int* n, const double* lr, double wd, double beta1, double beta2, double eps, int step,
                  void* stream) {
  return adamw_impl(nseg, p, const_cast<float* const*>(g), m, v, n, lr, wd, beta1, beta2, eps, step, 0, stream);
}

int cn_adamw_step_zero_grad(int nseg, float* const* p, float* const* g, float* const* m, float* const* v,
                            const int* n, const double* lr, double wd, double beta1, double beta2, double eps,
                            int step, void* stream) {
  return adamw_impl(nseg, p, g, m, v, n, lr, wd, beta1, beta2, eps, step, 1, stream);
}

int cn_clock_probe(unsigned int* d_out, int n_workgroups, int iters, unsigned int seed, void* stream) {
  if (!d_out || n_workgroups <= 0 || iters <= 0) return fail("cn_clock_probe: bad argument");
  hipLaunchKernelGGL(clock_probe_kernel, dim3(n_workgroups), dim3(kProbeWaves * 64), 0, S(stream), d_out, iters, seed);
  return launch_check("clock_probe_kernel");
}

}  // extern "C"
