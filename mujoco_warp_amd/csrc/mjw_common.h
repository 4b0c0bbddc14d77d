// mjw_common.h -- constants and helpers shared by the generic (mjw_step.hip) and dense
// (mjw_dense.hip) world-per-wavefront kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "mjw_amd.h"
#include "mjw_math.h"

namespace mjw {

constexpr int LPW = 64;   // lanes per world (one wavefront)
constexpr int CREC = 33;  // words per staged contact record (odd: lane-per-record access is bank-conflict free)
constexpr int CMAX = 32;  // staged contacts per collision round

// ST_POOL (with ST_POS): the position stage with the contacts read back from the pool instead of the
// narrowphase -- the constraint rows after a contactfilter callback edited d.contact (mjw_contact_rows)
enum : int { ST_POS = 1, ST_VEL = 2, ST_ACT = 4, ST_ACC = 8, ST_SOLVE = 16, ST_EULER = 32, ST_NOFACTOR = 64, ST_POOL = 128 };
enum : int { JNT_FREE = 0, JNT_BALL = 1, JNT_SLIDE = 2, JNT_HINGE = 3 };
enum : int { GEOM_PLANE = 0, GEOM_HFIELD = 1, GEOM_SPHERE = 2, GEOM_CAPSULE = 3, GEOM_ELLIPSOID = 4, GEOM_CYLINDER = 5, GEOM_BOX = 6, GEOM_MESH = 7 };
enum : int { EQ_CONNECT = 0, EQ_WELD = 1, EQ_JOINT = 2, EQ_TENDON = 3 };
enum : int { INT_EULER = 0, INT_RK4 = 1, INT_IMPLICIT = 2, INT_IMPLICITFAST = 3 };
enum : int { GAIN_FIXED = 0, GAIN_AFFINE = 1, GAIN_MUSCLE = 2 };
enum : int { BIAS_NONE = 0, BIAS_AFFINE = 1, BIAS_MUSCLE = 2 };
enum : int { DYN_NONE = 0, DYN_INTEGRATOR = 1, DYN_FILTER = 2, DYN_FILTEREXACT = 3, DYN_MUSCLE = 4, DYN_USER = 5 };
enum : int {
  DSBL_CONSTRAINT = 1, DSBL_EQUALITY = 2, DSBL_FRICTIONLOSS = 4, DSBL_LIMIT = 8, DSBL_CONTACT = 16, DSBL_SPRING = 32,
  DSBL_DAMPER = 64, DSBL_GRAVITY = 128, DSBL_CLAMPCTRL = 256, DSBL_WARMSTART = 512, DSBL_ACTUATION = 2048,
  DSBL_REFSAFE = 4096, DSBL_SENSOR = 8192, DSBL_EULERDAMP = 1 << 15
};
enum : int { TRN_JOINT = 0, TRN_JOINTINPARENT = 1, TRN_SLIDERCRANK = 2, TRN_TENDON = 3, TRN_SITE = 4, TRN_BODY = 5 };
enum : int { OBJ_UNKNOWN = 0, OBJ_BODY = 1, OBJ_XBODY = 2, OBJ_GEOM = 5, OBJ_SITE = 6, OBJ_CAMERA = 7 };
enum : int { DATATYPE_REAL = 0, DATATYPE_POSITIVE = 1 };
enum : int { STAGE_POS = 1, STAGE_VEL = 2, STAGE_ACC = 3 };
enum : int {
  SENS_ACCELEROMETER = 1, SENS_VELOCIMETER = 2, SENS_GYRO = 3, SENS_FORCE = 4, SENS_TORQUE = 5, SENS_MAGNETOMETER = 6,
  SENS_JOINTPOS = 9, SENS_JOINTVEL = 10, SENS_ACTUATORPOS = 13, SENS_ACTUATORVEL = 14, SENS_ACTUATORFRC = 15,
  SENS_JOINTACTFRC = 16, SENS_BALLQUAT = 18, SENS_BALLANGVEL = 19, SENS_FRAMEPOS = 26, SENS_FRAMEQUAT = 27,
  SENS_FRAMEXAXIS = 28, SENS_FRAMEYAXIS = 29, SENS_FRAMEZAXIS = 30, SENS_FRAMELINVEL = 31, SENS_FRAMEANGVEL = 32,
  SENS_FRAMELINACC = 33, SENS_FRAMEANGACC = 34, SENS_SUBTREECOM = 35, SENS_CLOCK = 45,
  SENS_TOUCH = 0, SENS_TENDONPOS = 11, SENS_TENDONVEL = 12, SENS_TENDONACTFRC = 17, SENS_JOINTLIMITPOS = 20,
  SENS_JOINTLIMITVEL = 21, SENS_JOINTLIMITFRC = 22, SENS_TENDONLIMITPOS = 23, SENS_TENDONLIMITVEL = 24,
  SENS_TENDONLIMITFRC = 25, SENS_SUBTREELINVEL = 36, SENS_SUBTREEANGMOM = 37, SENS_E_POTENTIAL = 43, SENS_E_KINETIC = 44,
  SENS_INSIDESITE = 38, SENS_GEOMDIST = 39, SENS_GEOMNORMAL = 40, SENS_GEOMFROMTO = 41, SENS_CAMPROJECTION = 8, SENS_CONTACT = 42, SENS_TACTILE = 46
};
enum : int { ENBL_ENERGY = 2, ENBL_MULTICCD = 16 };
enum : int { CNSTR_EQUALITY = 0, CNSTR_FRICTION_DOF = 1, CNSTR_FRICTION_TENDON = 2, CNSTR_LIMIT_JOINT = 3, CNSTR_LIMIT_TENDON = 4, CNSTR_CONTACT_FRICTIONLESS = 5, CNSTR_CONTACT_PYRAMIDAL = 6,
             CNSTR_CONTACT_ELLIPTIC = 7 };
enum : int { CONE_PYRAMIDAL = 0, CONE_ELLIPTIC = 1 };
enum : int { STATE_SATISFIED = 0, STATE_QUADRATIC = 1, STATE_LINEARNEG = 2, STATE_LINEARPOS = 3, STATE_CONE = 4 };
enum : int { SOLVER_CG = 1, SOLVER_NEWTON = 2 };
enum : int { CAM_FIXED = 0, CAM_TRACK = 1, CAM_TRACKCOM = 2, CAM_TARGETBODY = 3, CAM_TARGETBODYCOM = 4 };
enum : int { FILTER_PLANE = 1, FILTER_SPHERE = 2, FILTER_AABB = 4, FILTER_OBB = 8 };

// The kernel arguments as a struct `A` mirroring the kernel's parameter list (same order, so the same
// layout as the kernarg segment), seen through an opaque copy of the segment pointer: loads of its
// fields after this point cannot be merged with loads before it, so a field is re-read (s_load from the
// kernarg segment, scalar cache) in each stage that uses it instead of being held in an SGPR across the
// whole kernel.  Without it the forward kernel kept ~1000 field values live and spilled 946 SGPRs into
// VGPR lanes (v_writelane / v_readlane: VALU work in every stage).
template <class A>
__device__ __forceinline__ const A& fresh_args() {
  typedef const __attribute__((address_space(4))) char* kptr;
  kptr p = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return *(const A*)p;
}

// batched model field base pointer for world w (types.py "*" semantics: worldid % nb)
__device__ __forceinline__ const float* mb(const float* p, int nb, int cnt, int w) {
  return nb <= 1 ? p : p + (long)(w % nb) * cnt;
}
#define MR(name) mb(m.name, m.name##_nb, m.name##_cnt, wid)

// solver.py:325-327 _log_scale: step size i of the parallel linesearch, log-spaced in [min_step, 1]
__device__ __forceinline__ float ls_parallel_alpha(float min_step, int n, int i) {
  const float lmin = logf(min_step);
  const float step = (logf(1.0f) - lmin) / fmaxf(1.0f, (float)(n - 1));
  return expf(lmin + (float)i * step);
}

// support.py:38-64 next_act: one activation advanced by scale * act_dot over the timestep dt
// (FILTEREXACT integrates the first-order filter exactly; USER activations are left to the user)
__device__ __forceinline__ float next_act(float dt, int dyntype, float tau_prm, const float* actrange, float act, float act_dot,
                                          float scale, bool clamp) {
  float a;
  if (dyntype == DYN_FILTEREXACT) {
    const float tau = fmaxf(MJW_MINVAL, tau_prm);
    a = act + scale * act_dot * tau * (1.0f - expf(-dt / tau));
  } else if (dyntype == DYN_USER) {
    return act;
  } else {
    a = act + scale * act_dot * dt;
  }
  return clamp ? clampf(a, actrange[0], actrange[1]) : a;
}

// ---- muscles (util_misc.py:454-600): prm = (range[2], force, scale, lmin, lmax, vmax, fpmax, fvmax),
// dynprm = (tau_act, tau_deact, tausmooth); acc0 / lengthrange are the actuator's model constants
__device__ __forceinline__ float muscle_gain_length(float L, float lmin, float lmax) {
  if (lmin > L || L > lmax) return 0.0f;
  const float a = 0.5f * (lmin + 1.0f), b = 0.5f * (1.0f + lmax);
  if (L <= a) {
    const float x = (L - lmin) / fmaxf(MJW_MINVAL, a - lmin);
    return 0.5f * x * x;
  }
  if (L <= 1.0f) {
    const float x = (1.0f - L) / fmaxf(MJW_MINVAL, 1.0f - a);
    return 1.0f - 0.5f * x * x;
  }
  if (L <= b) {
    const float x = (L - 1.0f) / fmaxf(MJW_MINVAL, b - 1.0f);
    return 1.0f - 0.5f * x * x;
  }
  const float x = (lmax - L) / fmaxf(MJW_MINVAL, lmax - b);
  return 0.5f * x * x;
}

__device__ __forceinline__ float muscle_gain(float len, float vel, const float* lr, float acc0, const float* prm) {
  float force = prm[2];
  if (force < 0.0f) force = prm[3] / fmaxf(MJW_MINVAL, acc0);
  const float L0 = (lr[1] - lr[0]) / fmaxf(MJW_MINVAL, prm[1] - prm[0]);
  const float L = prm[0] + (len - lr[0]) / fmaxf(MJW_MINVAL, L0);
  const float V = vel / fmaxf(MJW_MINVAL, L0 * prm[6]);
  const float FL = muscle_gain_length(L, prm[4], prm[5]);
  const float fvmax = prm[8], y = fvmax - 1.0f;
  float FV;
  if (V <= -1.0f) FV = 0.0f;
  else if (V <= 0.0f) FV = (V + 1.0f) * (V + 1.0f);
  else if (V <= y) FV = fvmax - (y - V) * (y - V) / fmaxf(MJW_MINVAL, y);
  else FV = fvmax;
  return -force * FL * FV;
}

__device__ __forceinline__ float muscle_bias(float len, const float* lr, float acc0, const float* prm) {
  float force = prm[2];
  if (force < 0.0f) force = prm[3] / fmaxf(MJW_MINVAL, acc0);
  const float L0 = (lr[1] - lr[0]) / fmaxf(MJW_MINVAL, prm[1] - prm[0]);
  const float L = prm[0] + (len - lr[0]) / fmaxf(MJW_MINVAL, L0);
  const float b = 0.5f * (1.0f + prm[5]), fpmax = prm[7];
  if (L <= 1.0f) return 0.0f;
  if (L <= b) {
    const float x = (L - 1.0f) / fmaxf(MJW_MINVAL, b - 1.0f);
    return -force * fpmax * 0.5f * x * x;
  }
  const float x = (L - b) / fmaxf(MJW_MINVAL, b - 1.0f);
  return -force * fpmax * (0.5f + x);
}

__device__ __forceinline__ float muscle_dynamics(float ctrl, float act, const float* prm) {
  const float ctrlclamp = fminf(fmaxf(ctrl, 0.0f), 1.0f), actclamp = fminf(fmaxf(act, 0.0f), 1.0f);
  const float tau_act = prm[0] * (0.5f + 1.5f * actclamp), tau_deact = prm[1] / (0.5f + 1.5f * actclamp);
  const float smooth = prm[2], dctrl = ctrlclamp - act;
  float tau;
  if (smooth < MJW_MINVAL) {
    tau = dctrl > 0.0f ? tau_act : tau_deact;
  } else {
    const float x = dctrl / smooth + 0.5f;
    const float sig = x <= 0.0f ? 0.0f : (x >= 1.0f ? 1.0f : x * x * x * (3.0f * x * (2.0f * x - 5.0f) + 10.0f));
    tau = tau_deact + (tau_act - tau_deact) * sig;
  }
  return dctrl / fmaxf(MJW_MINVAL, tau);
}

// derivative.py:36-107 (_qderiv_actuator_passive_vel): d force / d velocity scale of actuator a
__device__ __forceinline__ float actuator_vel_deriv(const mjw_model_t& m, const mjw_data_t& d, int wid, int a) {
  const float* gainprm = MR(actuator_gainprm) + 10 * a;
  const float* biasprm = MR(actuator_biasprm) + 10 * a;
  float gain = m.actuator_gaintype[a] == GAIN_AFFINE ? gainprm[2] : 0.0f;
  float bias = m.actuator_biastype[a] == BIAS_AFFINE ? biasprm[2] : 0.0f;
  if (bias == 0.0f && gain == 0.0f) return 0.0f;
  if (m.actuator_forcelimited[a]) {
    float f = d.actuator_force[(long)wid * m.nu + a];
    const float* fr = MR(actuator_forcerange) + 2 * a;
    if (f <= fr[0] || f >= fr[1]) return 0.0f;
  }
  float vel = bias;
  if (m.actuator_dyntype[a] != DYN_NONE) {
    if (gain != 0.0f) {  // derivative.py:86-101: actearly differentiates at the next activation
      const long ga = (long)wid * m.na + m.actuator_actadr[a] + m.actuator_actnum[a] - 1;
      vel += gain * (m.actuator_actearly[a] ? next_act(MR(opt_timestep)[0], m.actuator_dyntype[a], MR(actuator_dynprm)[10 * a], MR(actuator_actrange) + 2 * a,
                                                       d.act[ga], d.act_dot[ga], 1.0f, m.actuator_actlimited[a] != 0)
                                            : d.act[ga]);
    }
  } else if (gain != 0.0f) {
    vel += gain * d.ctrl[(long)wid * m.nu + a];
  }
  return vel;
}


// ---- wave primitives ------------------------------------------------------------------------
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ float dpp_src(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, ROWMASK, 0xf, false));
}

__device__ __forceinline__ float rdlane(float x, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l)); }

// full 64-lane sum, wave-uniform result (must be called with all lanes active)
__device__ __forceinline__ float dsum(float x) {
  x += dpp_src<0xb1>(x);        // quad_perm [1,0,3,2]
  x += dpp_src<0x4e>(x);        // quad_perm [2,3,0,1]  -> quad sums
  x += dpp_src<0x124>(x);       // row_ror:4
  x += dpp_src<0x128>(x);       // row_ror:8            -> row (16-lane) sums
  x += dpp_src<0x142, 0xa>(x);  // row_bcast:15 into rows 1,3
  x += dpp_src<0x143, 0xc>(x);  // row_bcast:31 into rows 2,3 -> lane 63 holds the total
  return rdlane(x, 63);
}

// the sums of x over lanes 0-31 and over lanes 32-63, wave-uniform (all lanes active): dsum without its
// last (cross-half) step, so two 32-lane sums cost one reduction
__device__ __forceinline__ void dsum_halves(float x, float& lo, float& hi) {
  x += dpp_src<0xb1>(x);        // quad_perm [1,0,3,2]
  x += dpp_src<0x4e>(x);        // quad_perm [2,3,0,1]
  x += dpp_src<0x124>(x);       // row_ror:4
  x += dpp_src<0x128>(x);       // row_ror:8            -> row (16-lane) sums
  x += dpp_src<0x142, 0xa>(x);  // row_bcast:15 into rows 1,3 -> lanes 31 / 63 hold the half sums
  lo = rdlane(x, 31);
  hi = rdlane(x, 63);
}

// the full 64-lane sums of a and b in one reduction: v_permlane32_swap leaves a's two halves in
// lanes 0-31 and b's in lanes 32-63 of the two results (their sum pairs the halves), then dsum_halves
__device__ __forceinline__ void dsum2(float a, float b, float& sa, float& sb) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  dsum_halves(__uint_as_float(r[0]) + __uint_as_float(r[1]), sa, sb);
}

// opt-in phase timers (build with -DMJW_PROFILE): per-phase s_memtime deltas summed over
// all waves into the translation unit's own g_prof[] (phase ids below), read back with
// mjw_prof_read (generic kernel) and mjw_prof_read_dense (dense kernel)
enum : int {
  PH_LOAD = 0, PH_KIN, PH_COM, PH_CAM, PH_CRB, PH_COLL, PH_TRN, PH_VEL, PH_ACT, PH_ACC, PH_GSOLVE, PH_GEULER,
  PH_DFACTOR, PH_DSOLVE, PH_DEULER,
  // sub-phases of PH_COLL (reported separately, not added to the total)
  PH_C_ROWS0, PH_C_BROAD, PH_C_NARROW, PH_C_POOL, PH_C_JROWS, PH_C_SCAL, PH_C_TAIL,
  // parts of PH_DSOLVE (counted in it as well): Newton's Hessian build (MFMA over row pairs) and its
  // Cholesky factor + solve, per solver iteration
  PH_NT_H, PH_NT_CHOL, PH_N
};
#ifdef MJW_PROFILE
// PROF_COPIES copies of every phase counter, a wave adding into copy (workgroup id mod PROF_COPIES): with
// one counter per phase, 8192 waves' same-address atomics serialised and the profile build ran the humanoid
// step 2.5x slower than the product build, inflating whichever phase followed each mark (round 6)
constexpr int PROF_COPIES = 64;
static __device__ unsigned long long g_prof[PH_N * PROF_COPIES];
#define PROF_SLOT(ph) (&g_prof[(ph) * PROF_COPIES + (blockIdx.x & (PROF_COPIES - 1))])
#define PROF_T0() unsigned long long _pt = __builtin_amdgcn_s_memtime()
#define PROF_T0_SUB() unsigned long long _pts = __builtin_amdgcn_s_memtime()
#define PROF_MARK_SUB(ph)                                                        \
  do {                                                                           \
    unsigned long long _nt = __builtin_amdgcn_s_memtime();                       \
    if ((threadIdx.x & 63) == 0) atomicAdd(PROF_SLOT(ph), _nt - _pts);           \
    _pts = _nt;                                                                  \
  } while (0)
#define PROF_MARK(ph)                                                            \
  do {                                                                           \
    unsigned long long _nt = __builtin_amdgcn_s_memtime();                       \
    if ((threadIdx.x & 63) == 0) atomicAdd(PROF_SLOT(ph), _nt - _pt);            \
    _pt = _nt;                                                                   \
  } while (0)
#define MJW_PROF_READER(fname)                                                                  \
  extern "C" int fname(unsigned long long* out, int reset) {                                    \
    static unsigned long long c[mjw::PH_N * mjw::PROF_COPIES];                                  \
    hipError_t e = hipMemcpyFromSymbol(c, HIP_SYMBOL(mjw::g_prof), sizeof(c));                  \
    for (int p = 0; p < mjw::PH_N; p++) {                                                       \
      unsigned long long t = 0;                                                                 \
      for (int k = 0; k < mjw::PROF_COPIES; k++) t += c[p * mjw::PROF_COPIES + k];              \
      out[p] = t;                                                                               \
    }                                                                                           \
    if (e == hipSuccess && reset) {                                                             \
      for (auto& v : c) v = 0;                                                                  \
      e = hipMemcpyToSymbol(HIP_SYMBOL(mjw::g_prof), c, sizeof(c));                              \
    }                                                                                           \
    return (int)e;                                                                              \
  }
#else
#define MJW_PROF_READER(fname)
#define PROF_T0() (void)0
#define PROF_MARK(ph) (void)0
#define PROF_T0_SUB() (void)0
#define PROF_MARK_SUB(ph) (void)0
#endif

// per-wave lifetime log (tools/wave_log.py; -DMJW_WAVELOG alone, or with MJW_PROFILE): 4 x u64 per
// world, {start, end} s_memrealtime (100 MHz, one clock for the whole chip), HW_ID | XCC_ID << 32,
// solver iterations; set with the translation unit's setter
#if defined(MJW_PROFILE) || defined(MJW_WAVELOG)
static __device__ unsigned long long* g_wlog = nullptr;
#define WLOG_T0() const unsigned long long _wt0 = __builtin_amdgcn_s_memrealtime()
#define WLOG_END(wid, niter)                                                                         \
  do {                                                                                               \
    if (g_wlog && (threadIdx.x & 63) == 0) {                                                         \
      unsigned long long* r = g_wlog + 4 * (long)(wid);                                              \
      r[0] = _wt0;                                                                                   \
      r[1] = __builtin_amdgcn_s_memrealtime();                                                       \
      r[2] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |                         \
             ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);                 \
      r[3] = (unsigned long long)(niter);                                                            \
    }                                                                                                \
  } while (0)
#define MJW_WLOG_SETTER(fname)                                                                       \
  extern "C" int fname(unsigned long long* buf) {                                                    \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(mjw::g_wlog), &buf, sizeof(buf));                         \
  }
#else
#define WLOG_T0() (void)0
#define WLOG_END(wid, niter) (void)0
#define MJW_WLOG_SETTER(fname)
#endif

// ---- launch trace (mjw_step_trace): one HIP event recorded after every kernel launch of a step,
// tagged with a kernel id (mjw_kernel_name gives its name), so that a host can time each kernel
// of the step on the stream the kernels run on
enum : int {
  K_RESET = 0, K_CTRL_NOISE, K_CCD, K_SENSOR, K_RK4,
  K_SP_POS, K_SP_CCD, K_SP_COLL, K_SP_CON, K_SP_VEL, K_SP_INDEX, K_SP_SOLVE, K_SP_SOLVE_LDS, K_SP_EULER,
  K_CCD_HF, K_SENSOR_COLL, K_SP_CCD_HF,
  K_STEP = 17,  // + NEWTON + 2 * BOX + 4 * nbi  (step_kernel<79, BOX, 7, NEWTON, NB>, NB = 28 / 16 for nbi 0 / 1)
  K_DENSE = 32,  // + 32 * nbi + 4 * FLAGS + 2 * ELL + NEWTON  (dense_kernel<FLAGS, NEWTON, ELL, NB>, NB = 32 / 16 / 28 for nbi 0 / 1 / 2)
  K_FWD = 256,   // + 4 * STAGES + 2 * box + tendon    (mjw_kernel<STAGES, box, tendon>)
  K_END = 256 + 4 * 256
};
struct LaunchTrace {
  hipEvent_t* ev;  // ev[0] recorded by the caller before the step; ev[i + 1] after launch i
  int* ids;        // ids[i]: kernel id of launch i
  int cap, n;
};
extern thread_local LaunchTrace* g_trace;
__host__ inline void trace_launch(hipStream_t s, int id) {
  LaunchTrace* t = g_trace;
  if (!t || t->n >= t->cap) return;
  (void)hipEventRecord(t->ev[t->n + 1], s);
  t->ids[t->n++] = id;
}

// dense (register-resident) factor / solve / euler kernel launcher, mjw_dense.hip
enum : int { DF_FACTOR = 1, DF_SOLVE = 2, DF_EULER = 4 };
// worlds [w0, w0 + count) of d (count < 0: all from w0)
int dense_launch(int flags, const mjw_model_t* m, const mjw_data_t* d, hipStream_t s, int w0 = 0, int count = -1);
// post-solve sensors of every stage + rne_postconstraint, mjw_sensor.hip (no-op without sensors)
enum : int { RK_BEGIN = 0, RK_PERTURB = 1, RK_ACCUM = 2, RK_END = 3 };
int rk4_launch(const mjw_model_t* m, const mjw_data_t* d, hipStream_t s, int op, float scale);
int sensor_launch(const mjw_model_t* m, const mjw_data_t* d, hipStream_t s, int stages = 7, int w0 = 0, int count = -1);
// workgroup-per-world pipeline of sparse / flex models (m->is_sparse), mjw_sparse.hip; ST_* stage bits
int sparse_launch(int stages, const mjw_model_t* m, const mjw_data_t* d, hipStream_t s);
// per-world slot ranges of the contact pool (d->ncon_world) on the dense path, mjw_step.hip
int pool_ranges_launch(const mjw_data_t* d, hipStream_t s);

}  // namespace mjw
