// mjw_dense.hip -- the dense factor / solve / integrate kernel (device code in mjw_dense.h), its
// launcher and the device self-checks of its wave primitives.

#include "mjw_dense.h"

#include <cstdlib>

namespace mjw {

// NB = 32: 3 waves/SIMD (up to 168 VGPRs, 12 worlds/CU).  NB <= 28: 4 (128 VGPRs, 16 worlds/CU, which
// the 9.7 KB of LDS also allows): since the unrolled J products (round 5) the NB = 28 instance spills
// the same 20 B/lane at 128 VGPRs as at 166, and the humanoid dense kernel measured 0.313 -> 0.305 ms
// (driver window) and 0.273 -> 0.264 ms (200 steps) at 4 (round 4: 0.295 -> 0.288 ms at 3, 0.287 at 2)
// ELL: elliptic friction cones (opt.cone = ELLIPTIC), a separate instantiation so that the pyramidal
// kernels keep their registers
// NB: the compile-time bound of the factor / substitution loops (>= nv; 16, 28 or 32, mjw_dense.h).
// The NB = 16 instances fit 128 VGPRs (4 waves/SIMD, 16 worlds/CU); the Euler-only one (5.9 KB of LDS,
// 27 worlds/CU) fits 64.
#ifndef MJW_DENSE_WPE
#define MJW_DENSE_WPE 4  // NB = 28 (A/B builds: 3)
#endif
// (Newton keeps 3: at 4 its NB = 28 instances allocate more registers, not fewer -- apollo's dense
// kernel measured 0.153 -> 0.173 ms; again with the LDL' Hessian solve in round 6, MJW_DENSE_WPE_NEWTON=4:
// humanoid Newton 0.182 -> 0.193 ms, apollo 0.133 -> 0.136 ms, profiles/r06_ab_newton_wpe.log)
#ifndef MJW_DENSE_WPE_NEWTON
#define MJW_DENSE_WPE_NEWTON 3
#endif
template <int FLAGS, bool NEWTON, int NB>
constexpr int dense_waves_per_eu() { return FLAGS == DF_EULER ? 6 : (NB <= 16 ? 4 : (NB <= 28 ? (NEWTON ? MJW_DENSE_WPE_NEWTON : MJW_DENSE_WPE) : 3)); }
template <int FLAGS, bool NEWTON, bool ELL, int NB>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(dense_waves_per_eu<FLAGS, NEWTON, NB>())))
dense_kernel(const mjw_model_t m, const mjw_data_t d, int w0) {
  __shared__ __attribute__((aligned(16))) float sm[dense_lds_words<FLAGS, NEWTON, ELL, NB>()];
  const int b = w0 + (int)blockIdx.x;
  if (b >= d.nworld) return;
  // d.sched set: worlds in the counter-reset kernel's longest-first order (world_order is a permutation)
  const int wid = d.sched ? d.world_order[b] : b;
  WLOG_T0();
  dense_world<FLAGS, NEWTON, ELL, NB>(m, d, wid, sm);
  if (!MJW_SCHED_EARLY && (FLAGS & DF_SOLVE) && d.sched && (threadIdx.x & 63) == 0) {
    // the next step's order: bucket by this step's iterations, most iterations first
    d.world_key[wid] = MJW_SCHED_BUCKETS - 1 - min(d.solver_niter[wid] >> 1, MJW_SCHED_BUCKETS - 1);
  }
  WLOG_END(wid, (FLAGS & DF_SOLVE) ? d.solver_niter[wid] : 0);
}

// device self-checks of the primitives above (mjw_selftest): which = 0 -> per-wave dsum and
// xhalf_add of 64-lane chunks; which = 1 -> spd_inverse of 32x32 row-major SPD matrices; which = 2 ->
// the same with the factor bound NB = 16 (matrices that are the identity past row / column 16);
// which = 3 / 4 -> ldl_factor + ldl_solve (NB = 32 / 28) of one right-hand side per matrix
__global__ void __launch_bounds__(64) selftest_kernel(int which, const float* in, float* out, int n) {
  __shared__ __attribute__((aligned(16))) float S[DS_WORDS];
  const int w = blockIdx.x, lane = threadIdx.x;
  if (w >= n) return;
  if (which == 0) {
    float x = in[w * 64 + lane];
    float t = dsum(x);
    if (lane == 0) out[w] = t;
    out[n + w * 64 + lane] = xhalf_add(x);
  } else if (which == 3 || which == 4) {
    // ldl_factor + ldl_solve of (32x32 SPD, 32-vector) pairs, 1056 floats each; which = 4: NB = 28 (input
    // identity past 28, right-hand side 0 there)
    float a[32];
    f32x16 M;
    const float* g = in + (long)w * 1056;
    stage_spd(g, 32, 32, nullptr, 0.0f, S, lane, a, M);
    const float b = g[1024 + (lane & 31)];
    float x;
    if (which == 4) {
      ldl_factor<28>(a, lane, S);
      x = ldl_solve<28>(a, S, lane, b);
    } else {
      ldl_factor<32>(a, lane, S);
      x = ldl_solve<32>(a, S, lane, b);
    }
    if (lane < 32) out[(long)w * 32 + lane] = x;
  } else {
    float a[32];
    f32x16 M;
    stage_spd(in + (long)w * 1024, 32, 32, nullptr, 0.0f, S, lane, a, M);
    // which = 2: the NB = 16 bound (input identity past 16)
    f32x16 Mi = which == 2 ? spd_inverse<false, 16>(a, lane) : spd_inverse(a, lane);
    const int c = lane & 31, h = lane >> 5;
#pragma unroll
    for (int r = 0; r < 16; r++) out[(long)w * 1024 + acc_row(r, h) * 32 + c] = Mi[r];
  }
}

template <int FLAGS, int NB>
void launch_nb(bool newton, const mjw_model_t* m, const mjw_data_t* d, hipStream_t s, int w0, int count) {
  if (newton) hipLaunchKernelGGL((dense_kernel<FLAGS, true, false, NB>), dim3(count), dim3(64), 0, s, *m, *d, w0);
  else hipLaunchKernelGGL((dense_kernel<FLAGS, false, false, NB>), dim3(count), dim3(64), 0, s, *m, *d, w0);
}

template <int FLAGS>
hipError_t launch_flags(const mjw_model_t* m, const mjw_data_t* d, hipStream_t s, int w0, int count) {
  const bool newton = m->opt_solver == SOLVER_NEWTON;
  // the cone only matters to the solve; Euler-only / factor-only launches use the pyramidal kernels
  const bool ell = (FLAGS & DF_SOLVE) && m->opt_cone == CONE_ELLIPTIC;
  int nbi = 0;  // factor bound: 0 -> 32, 1 -> 16, 2 -> 28 (the kernel id and name carry it)
  static const int nb_max = [] {  // MJW_DENSE_NB=32 / 28: never use the smaller bounds (A/B runs)
    const char* e = getenv("MJW_DENSE_NB");
    return e ? atoi(e) : 0;
  }();
  if (ell) {
    if (newton) hipLaunchKernelGGL((dense_kernel<FLAGS, true, true, 32>), dim3(count), dim3(64), 0, s, *m, *d, w0);
    else hipLaunchKernelGGL((dense_kernel<FLAGS, false, true, 32>), dim3(count), dim3(64), 0, s, *m, *d, w0);
  } else if (nb_max == 32) {
    launch_nb<FLAGS, 32>(newton, m, d, s, w0, count);
  } else if (m->nv <= 16 && nb_max != 28) {
    launch_nb<FLAGS, 16>(newton, m, d, s, w0, count);
    nbi = 1;
  } else if (m->nv <= 28) {
    launch_nb<FLAGS, 28>(newton, m, d, s, w0, count);
    nbi = 2;
  } else {
    launch_nb<FLAGS, 32>(newton, m, d, s, w0, count);
  }
  trace_launch(s, K_DENSE + 32 * nbi + 4 * FLAGS + (ell ? 2 : 0) + (newton ? 1 : 0));
  return hipGetLastError();
}

int dense_launch(int flags, const mjw_model_t* m, const mjw_data_t* d, hipStream_t s, int w0, int count) {
  if (count < 0) count = d->nworld - w0;
  if (count <= 0) return 0;
  const int fl = m->opt_disableflags;
  const bool implicit_int = m->opt_integrator == INT_IMPLICITFAST
                                ? (fl & (DSBL_ACTUATION | DSBL_SPRING | DSBL_DAMPER)) != (DSBL_ACTUATION | DSBL_SPRING | DSBL_DAMPER)
                                : !(fl & (DSBL_EULERDAMP | DSBL_DAMPER));
  if ((flags & DF_EULER) && flags != DF_EULER && implicit_int) {
    int rc = dense_launch(flags & ~DF_EULER, m, d, s, w0, count);
    return rc ? rc : dense_launch(DF_EULER, m, d, s, w0, count);
  }
  switch (flags) {
    case DF_FACTOR | DF_SOLVE | DF_EULER: return (int)launch_flags<DF_FACTOR | DF_SOLVE | DF_EULER>(m, d, s, w0, count);
    case DF_FACTOR | DF_SOLVE: return (int)launch_flags<DF_FACTOR | DF_SOLVE>(m, d, s, w0, count);
    case DF_FACTOR: return (int)launch_flags<DF_FACTOR>(m, d, s, w0, count);
    case DF_SOLVE: return (int)launch_flags<DF_SOLVE>(m, d, s, w0, count);
    case DF_EULER: return (int)launch_flags<DF_EULER>(m, d, s, w0, count);
    default: return (int)hipErrorInvalidValue;
  }
}

}  // namespace mjw

MJW_PROF_READER(mjw_prof_read_dense)
MJW_WLOG_SETTER(mjw_prof_wlog_dense)

extern "C" int mjw_selftest(int which, const float* in, float* out, int n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(mjw::selftest_kernel, dim3(n), dim3(64), 0, (hipStream_t)stream, which, in, out, n);
  return (int)hipGetLastError();
}
