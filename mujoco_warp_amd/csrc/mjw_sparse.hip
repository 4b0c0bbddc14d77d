// mjw_sparse.hip -- workgroup-per-world step for large, sparse and flex models (m.is_sparse).
//
// The world-per-wavefront kernels (mjw_step.hip / mjw_dense.hip) keep a whole world in LDS and
// registers, which stops at nv ~ 64.  Models past that -- the reference's sparse path
// (io.py:67-74: jacobian=sparse or nv > 32), e.g. the cloth benchmarks with a 30x30 flexcomp
// (nv = 2706, ~2600 constraint rows) -- run here instead:
//
//   * one 256-thread workgroup owns one world; per-world state stays in HBM (L2 resident while
//     the workgroup runs); threads stride over bodies / dofs / trees / pairs / rows;
//   * tree recursions avoid level launches: subtree sums walk DFS subtree ranges, velocity and
//     acceleration propagation walk the ancestor chain, so no atomics and no per-level sync
//     beyond the kinematics levels;
//   * M and its factor use the ancestor-row sparse layout (M_rowadr / M_colind, diagonal last);
//     the L'DL factor and solves run one kinematic tree per thread (smooth.py:1003-1064, 2813-2846);
//   * constraint Jacobian rows are sparse (efc_J_colind / efc_J_rownnz, njrow slots per row) and
//     stored slot-major (ELL: slot k of every row contiguous, (nworld, njrow, njmax_pad)), so the
//     row-parallel passes read only the slots a row uses, coalesced across the wave;
//     the solver builds the transposed (column) index once per solve, so J'f is a deterministic
//     per-dof gather instead of atomics;
//   * contacts and rows are emitted in a deterministic per-world order with block scans.
//
// Stages restate the reference (file:line per function) and oracle/oracle.c restates the same
// algorithms on the CPU for the parity tests.

#include "mjw_common.h"

#include <cstdlib>
#include <mutex>

#include "mjw_ccd.h"
#include "mjw_narrow.h"
#include "mjw_flexcol.h"
#include "mjw_passive.h"
#include "mjw_tendon.h"
#include "mjw_trn.h"

namespace mjw {
namespace sp {

#define MR_W(name) (MR(name)[0])

// 256 threads per world: measured best on aloha_cloth (512, with or without an 80 / 64 VGPR cap on
// the solve, and 256 with a 64 VGPR cap were 12-25 % slower; so was capping the solve's residency
// to fit the per-world row state in the 256 MB MALL: DESIGN 3.6)
constexpr int BLK = 256;
// Round-6 A/B switches of the CG passes (tools/build_variants.py, same-box lines in profiles/r06_sparse_ab.log
// and r06_sparse_ab2.log): the small-tree register path (+4 %: aloha_cloth 42.9 -> 45.2 K env-steps/s) and
// the solve's 4-worlds-per-CU register cap (without it the inlined CG loop takes 152 VGPRs, 3 worlds per CU,
// 34.0 K).  Measured and removed (the code is in commit 5781637): loading a jv batch's J slots / a J'f
// column's entries up front, whole (43.4 K / 38.4 K) or in chunks (4- / 2-slot jv chunks 41.8 K / 43.9 K,
// 8-entry J'f chunks 40.3 K, against 45.1 K): every form that puts more loads in flight per thread is slower
// -- the passes are bound by the memory pipeline's throughput, not by the latency of one thread's chain
#ifndef MJW_SP_TREE
#define MJW_SP_TREE 1
#endif
#ifndef MJW_SP_SOLVE_MINBLK
#define MJW_SP_SOLVE_MINBLK 4
#endif
constexpr int SOLVE_LDS_THREADS = 1024;
constexpr int SP_LDS_SEARCH_MAX = 8192;  // the CG search direction lives in LDS up to this nv
constexpr int SORTN = 32;  // J-transpose segments up to this length are sorted in registers
constexpr int SP_LDS_CNT_MAX = 8192;  // column counters of the J transpose live in LDS up to this nv + 1
constexpr int SP_LDS_ITEMS_MAX = 48 * 1024;  // per-item contact counts of the collision pass in LDS up to this

// opt-in phase timers of this path (build with -DMJW_PROFILE; tools/sparse_prof.py): s_memtime
// deltas summed over waves, read back with mjw_prof_read_sparse
// SPH_NPASS / SPH_NITER (counts, not cycles): the row passes of the line searches (the jv + alpha = 0
// pass, the Newton-step pass and one per bracketing iteration) and the CG iterations, summed over worlds
// SPH_S_*: sub-phases of the CG iteration (also counted in SPH_SLS / SPH_SUPD): the line search's M x search
// (mul_m_trees), its jv + alpha = 0 pass, its remaining row passes; update_constraint's row pass, its J'f
// (transposed-index gathers); update_gradient's preconditioner (solve_trees / the Newton direction)
enum : int { SPH_KIN = 0, SPH_FLEX, SPH_CRB, SPH_COLL, SPH_CON, SPH_VEL, SPH_ACT, SPH_ACC, SPH_SINIT, SPH_SLS, SPH_SUPD, SPH_SCG, SPH_NPASS, SPH_NITER,
             SPH_S_MULM, SPH_S_JV, SPH_S_LSP, SPH_S_UCR, SPH_S_JTF, SPH_S_TREES, SPH_N };
#ifdef MJW_PROFILE
// SPROF_COPIES copies per counter, a workgroup adding into copy (world mod SPROF_COPIES): same-address
// atomics from every wave would serialise and distort the phases they follow (as in mjw_common.h)
constexpr int SPROF_COPIES = 64;
static __device__ unsigned long long g_sprof[SPH_N * SPROF_COPIES];
#define SPROF_SLOT(ph) (&g_sprof[(ph) * SPROF_COPIES + (blockIdx.x & (SPROF_COPIES - 1))])
#define SPROF_T0() unsigned long long _spt = __builtin_amdgcn_s_memtime()
#define SPROF_MARK(ph)                                                           \
  do {                                                                           \
    unsigned long long _nt = __builtin_amdgcn_s_memtime();                       \
    if ((threadIdx.x & 63) == 0) atomicAdd(SPROF_SLOT(ph), _nt - _spt);          \
    _spt = _nt;                                                                  \
  } while (0)
#define SPROF_COUNT(ph, n)                                  \
  do {                                                      \
    if (threadIdx.x == 0) atomicAdd(SPROF_SLOT(ph), (unsigned long long)(n)); \
  } while (0)
#define SPROF_T0_SUB() unsigned long long _spts = __builtin_amdgcn_s_memtime()
#define SPROF_MARK_SUB(ph)                                                       \
  do {                                                                           \
    unsigned long long _nt = __builtin_amdgcn_s_memtime();                       \
    if ((threadIdx.x & 63) == 0) atomicAdd(SPROF_SLOT(ph), _nt - _spts);         \
    _spts = _nt;                                                                 \
  } while (0)
#else
#define SPROF_T0_SUB() (void)0
#define SPROF_MARK_SUB(ph) (void)0
#define SPROF_T0() (void)0
#define SPROF_MARK(ph) (void)0
#define SPROF_COUNT(ph, n) (void)0
#endif
constexpr int NWAVE = BLK / 64;
enum : int { EQ_FLEX = 4 };

constexpr int SP_FBOX = 4;  // flexes whose bounding box the collision pass keeps (culls triangle-geom items)

constexpr int NWAVE_MAX = 16;  // the LDS-resident solve runs 1024-thread worlds

struct Smem {
  float red[NWAVE_MAX][16];
  float red2[2][NWAVE_MAX][16];  // double-buffered partials of block_sum_db
  int iscan[NWAVE_MAX];
  int ival[8];
  float fbox[SP_FBOX][6];  // per flex: min xyz, max xyz of its vertices
};

__device__ __forceinline__ int tid() { return (int)threadIdx.x; }
// threads per world of the running kernel (BLK, or 1024 for the LDS-resident solve)
__device__ __forceinline__ int nthr() { return (int)blockDim.x; }

// block-wide sums of N <= 16 floats; every thread gets the same (bitwise) totals
template <int N>
__device__ __forceinline__ void block_sum(float (&v)[N], Smem& sm) {
  const int lane = tid() & 63, wv = tid() >> 6;
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = dsum(v[k]);
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < N; k++) sm.red[wv][k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; k++) {
    float s = 0.0f;
    for (int w = 0; w < (nthr() >> 6); w++) s += sm.red[w][k];
    v[k] = s;
  }
}

__device__ __forceinline__ float block_sum1(float x, Smem& sm) {
  float v[1] = {x};
  block_sum<1>(v, sm);
  return v[0];
}

// block_sum with one barrier: consecutive calls alternate between two partial buffers (`phase`,
// uniform over the block), so a wave that runs ahead into the next call never overwrites partials
// another wave is still reading -- that would take a second buffer-reuse barrier per call.  The
// remaining barrier still orders every memory operation issued before the call.
template <int N>
__device__ __forceinline__ void block_sum_db(float (&v)[N], Smem& sm, int& phase) {
  const int lane = tid() & 63, wv = tid() >> 6;
#pragma unroll
  for (int k = 0; k < N; k++) v[k] = dsum(v[k]);
  float(*red)[16] = sm.red2[phase];
  phase ^= 1;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < N; k++) red[wv][k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < N; k++) {
    float t = 0.0f;
    for (int w = 0; w < (nthr() >> 6); w++) t += red[w][k];
    v[k] = t;
  }
}

__device__ __forceinline__ float block_sum1_db(float x, Smem& sm, int& phase) {
  float v[1] = {x};
  block_sum_db<1>(v, sm, phase);
  return v[0];
}

// exclusive block scan of ints; `total` gets the block total (uniform)
__device__ __forceinline__ int block_scan(int v, int& total, Smem& sm) {
  const int lane = tid() & 63, wv = tid() >> 6;
  int incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    int t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  __syncthreads();
  if (lane == 63) sm.iscan[wv] = incl;
  __syncthreads();
  int off = 0;
  total = 0;
  for (int w = 0; w < (nthr() >> 6); w++) {  // every wave of the block (1024-thread solve blocks too)
    if (w < wv) off += sm.iscan[w];
    total += sm.iscan[w];
  }
  return off + incl - v;
}

// ---------------------------------------------------------------------------------------------
// smooth.py:44-224 kinematics (level passes over bodies, then frames of geoms / sites / flex verts)
// ---------------------------------------------------------------------------------------------
__device__ void kinematics(const mjw_model_t& m, const mjw_data_t& d, int wid) {
  const int nb = m.nbody;
  float* xpos = d.xpos + (long)wid * nb * 3;
  float* xquat = d.xquat + (long)wid * nb * 4;
  const float* qpos = d.qpos + (long)wid * m.nq;
  const float* body_pos = MR(body_pos);
  const float* body_quat = MR(body_quat);
  const float* qpos0 = MR(qpos0);
  const float* jnt_axis = MR(jnt_axis);
  const float* jnt_pos = MR(jnt_pos);
  float* xanchor = d.xanchor + (long)wid * m.njnt * 3;
  float* xaxis = d.xaxis + (long)wid * m.njnt * 3;
  if (tid() == 0) {
    xpos[0] = xpos[1] = xpos[2] = 0.0f;
    xquat[0] = 1.0f;
    xquat[1] = xquat[2] = xquat[3] = 0.0f;
  }
  __syncthreads();
  for (int lev = 1; lev < m.nlevel; lev++) {
    for (int k = m.level_adr[lev] + tid(); k < m.level_adr[lev + 1]; k += BLK) {
      const int b = m.level_body[k];
      const int pid = m.body_parentid[b], ja = m.body_jntadr[b], jn = m.body_jntnum[b];
      if (jn == 1 && m.jnt_type[ja] == JNT_FREE) {
        const int qa = m.jnt_qposadr[ja];
        float q[4] = {qpos[qa + 3], qpos[qa + 4], qpos[qa + 5], qpos[qa + 6]};
        normalize4(q);
        for (int i = 0; i < 3; i++) {
          xpos[3 * b + i] = qpos[qa + i];
          xanchor[3 * ja + i] = qpos[qa + i];
          xaxis[3 * ja + i] = jnt_axis[3 * ja + i];
        }
        for (int i = 0; i < 4; i++) xquat[4 * b + i] = q[i];
        continue;
      }
      float pos[3], quat[4];
      const int mid = m.body_mocapid[b];
      if (mid >= 0) {
        for (int i = 0; i < 3; i++) pos[i] = d.mocap_pos[((long)wid * m.nmocap + mid) * 3 + i];
        for (int i = 0; i < 4; i++) quat[i] = d.mocap_quat[((long)wid * m.nmocap + mid) * 4 + i];
      } else {
        for (int i = 0; i < 3; i++) pos[i] = body_pos[3 * b + i];
        for (int i = 0; i < 4; i++) quat[i] = body_quat[4 * b + i];
      }
      float t[3];
      rot_vec_quat(t, pos, xquat + 4 * pid);
      for (int i = 0; i < 3; i++) pos[i] = t[i] + xpos[3 * pid + i];
      mul_quat(quat, xquat + 4 * pid, quat);
      for (int j = ja; j < ja + jn; j++) {
        const int qa = m.jnt_qposadr[j], jt = m.jnt_type[j];
        const float* axis = jnt_axis + 3 * j;
        const float* jp = jnt_pos + 3 * j;
        float xa[3], xx[3];
        rot_vec_quat(t, jp, quat);
        for (int i = 0; i < 3; i++) xa[i] = t[i] + pos[i];
        rot_vec_quat(xx, axis, quat);
        if (jt == JNT_BALL) {
          float ql[4] = {qpos[qa], qpos[qa + 1], qpos[qa + 2], qpos[qa + 3]};
          normalize4(ql);
          mul_quat(quat, quat, ql);
          rot_vec_quat(t, jp, quat);
          for (int i = 0; i < 3; i++) pos[i] = xa[i] - t[i];
        } else if (jt == JNT_SLIDE) {
          const float dq = qpos[qa] - qpos0[qa];
          for (int i = 0; i < 3; i++) pos[i] += xx[i] * dq;
        } else if (jt == JNT_HINGE) {
          float ql[4];
          axis_angle_to_quat(ql, axis, qpos[qa] - qpos0[qa]);
          mul_quat(quat, quat, ql);
          rot_vec_quat(t, jp, quat);
          for (int i = 0; i < 3; i++) pos[i] = xa[i] - t[i];
        }
        for (int i = 0; i < 3; i++) {
          xanchor[3 * j + i] = xa[i];
          xaxis[3 * j + i] = xx[i];
        }
      }
      normalize4(quat);
      for (int i = 0; i < 3; i++) xpos[3 * b + i] = pos[i];
      for (int i = 0; i < 4; i++) xquat[4 * b + i] = quat[i];
    }
    __syncthreads();
  }
  const float* body_ipos = MR(body_ipos);
  const float* body_iquat = MR(body_iquat);
  for (int b = tid(); b < nb; b += BLK) {
    float q[4], t[3];
    quat_to_mat(d.xmat + ((long)wid * nb + b) * 9, xquat + 4 * b);
    rot_vec_quat(t, body_ipos + 3 * b, xquat + 4 * b);
    for (int i = 0; i < 3; i++) d.xipos[((long)wid * nb + b) * 3 + i] = xpos[3 * b + i] + t[i];
    mul_quat(q, xquat + 4 * b, body_iquat + 4 * b);
    quat_to_mat(d.ximat + ((long)wid * nb + b) * 9, q);
  }
  const float* geom_pos = MR(geom_pos);
  const float* geom_quat = MR(geom_quat);
  for (int g = tid(); g < m.ngeom; g += BLK) {
    const int b = m.geom_bodyid[g];
    float q[4], t[3];
    rot_vec_quat(t, geom_pos + 3 * g, xquat + 4 * b);
    for (int i = 0; i < 3; i++) d.geom_xpos[((long)wid * m.ngeom + g) * 3 + i] = xpos[3 * b + i] + t[i];
    mul_quat(q, xquat + 4 * b, geom_quat + 4 * g);
    quat_to_mat(d.geom_xmat + ((long)wid * m.ngeom + g) * 9, q);
  }
  const float* site_pos = MR(site_pos);
  const float* site_quat = MR(site_quat);
  for (int s = tid(); s < m.nsite; s += BLK) {
    const int b = m.site_bodyid[s];
    float q[4], t[3];
    rot_vec_quat(t, site_pos + 3 * s, xquat + 4 * b);
    for (int i = 0; i < 3; i++) d.site_xpos[((long)wid * m.nsite + s) * 3 + i] = xpos[3 * b + i] + t[i];
    mul_quat(q, xquat + 4 * b, site_quat + 4 * s);
    quat_to_mat(d.site_xmat + ((long)wid * m.nsite + s) * 9, q);
  }
  // smooth.py:228-258 _flex_vertices (flexcomp vertices are centered on their bodies)
  for (int v = tid(); v < m.nflexvert; v += BLK) {
    const int b = m.flex_vertbodyid[v];
    for (int i = 0; i < 3; i++) d.flexvert_xpos[((long)wid * m.nflexvert + v) * 3 + i] = xpos[3 * b + i];
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// smooth.py:463-632 com_pos: subtree com (DFS subtree-range sums), cinert, cdof
// ---------------------------------------------------------------------------------------------
__device__ void com_pos(const mjw_model_t& m, const mjw_data_t& d, int wid, Smem& sm) {
  const int nb = m.nbody;
  const float* xipos = d.xipos + (long)wid * nb * 3;
  const float* body_mass = MR(body_mass);
  const float* body_subtreemass = MR(body_subtreemass);
  float* sc = d.subtree_com + (long)wid * nb * 3;
  // subtrees of up to BIG bodies: one thread each, serial; larger ones (the world body's spans every
  // flex vertex, ~900 on the cloth) as block-wide sums: a serial fp32 running sum over them drifted to
  // 1.5e-5 of the oracle's fp64 value and sat on the critical path of the whole block
  constexpr int BIG = 64, NBIG = 16;
  __shared__ int big[NBIG];
  __shared__ int nbig;
  if (tid() == 0) nbig = 0;
  __syncthreads();
  for (int b = tid(); b < nb; b += BLK) {
    if (m.body_subtree_end[b] - b > BIG) {  // (past NBIG of them: serial here after all)
      const int k = atomicAdd(&nbig, 1);
      if (k < NBIG) {
        big[k] = b;
        continue;
      }
    }
    float s[3] = {0.0f, 0.0f, 0.0f};
    for (int c = b; c < m.body_subtree_end[b]; c++)
      for (int i = 0; i < 3; i++) s[i] += xipos[3 * c + i] * body_mass[c];
    const float mass = body_subtreemass[b];
    for (int i = 0; i < 3; i++) sc[3 * b + i] = mass != 0.0f ? s[i] / mass : s[i];
  }
  __syncthreads();
  const int nbg = min(nbig, NBIG);
  for (int j = 0; j < nbg; j++) {  // uniform: the big subtrees, one block sum each
    const int b = big[j], e = m.body_subtree_end[b];
    float v[3] = {0.0f, 0.0f, 0.0f};
    for (int c = b + tid(); c < e; c += BLK)
      for (int i = 0; i < 3; i++) v[i] += xipos[3 * c + i] * body_mass[c];
    block_sum<3>(v, sm);
    const float mass = body_subtreemass[b];
    if (tid() == 0)
      for (int i = 0; i < 3; i++) sc[3 * b + i] = mass != 0.0f ? v[i] / mass : v[i];
  }
  __syncthreads();
  const float* body_inertia = MR(body_inertia);
  for (int b = tid(); b < nb; b += BLK) {
    const float* mat = d.ximat + ((long)wid * nb + b) * 9;
    const float* inert = body_inertia + 3 * b;
    const float mass = body_mass[b];
    const int root = m.body_rootid[b];
    float dif[3], tmp[9];
    for (int i = 0; i < 3; i++) dif[i] = xipos[3 * b + i] - sc[3 * root + i];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        float s = 0.0f;
        for (int k = 0; k < 3; k++) s += mat[3 * i + k] * inert[k] * mat[3 * j + k];
        tmp[3 * i + j] = s;
      }
    float* r = d.cinert + ((long)wid * nb + b) * 10;
    r[0] = tmp[0] + mass * (dif[1] * dif[1] + dif[2] * dif[2]);
    r[1] = tmp[4] + mass * (dif[0] * dif[0] + dif[2] * dif[2]);
    r[2] = tmp[8] + mass * (dif[0] * dif[0] + dif[1] * dif[1]);
    r[3] = tmp[1] - mass * dif[0] * dif[1];
    r[4] = tmp[2] - mass * dif[0] * dif[2];
    r[5] = tmp[5] - mass * dif[1] * dif[2];
    r[6] = mass * dif[0];
    r[7] = mass * dif[1];
    r[8] = mass * dif[2];
    r[9] = mass;
  }
  float* cd = d.cdof + (long)wid * m.nv * 6;
  for (int j = tid(); j < m.njnt; j += BLK) {
    const int b = m.jnt_bodyid[j], da = m.jnt_dofadr[j], jt = m.jnt_type[j];
    const float* xaxis = d.xaxis + ((long)wid * m.njnt + j) * 3;
    const float* xmat = d.xmat + ((long)wid * nb + b) * 9;
    float off[3];
    for (int i = 0; i < 3; i++) off[i] = sc[3 * m.body_rootid[b] + i] - d.xanchor[((long)wid * m.njnt + j) * 3 + i];
    if (jt == JNT_FREE || jt == JNT_BALL) {
      int rot0 = da;
      if (jt == JNT_FREE) {
        for (int k = 0; k < 3; k++)
          for (int i = 0; i < 6; i++) cd[6 * (da + k) + i] = (i == 3 + k) ? 1.0f : 0.0f;
        rot0 = da + 3;
      }
      for (int k = 0; k < 3; k++) {
        float ax[3] = {xmat[k], xmat[3 + k], xmat[6 + k]};
        float* r = cd + 6 * (rot0 + k);
        r[0] = ax[0];
        r[1] = ax[1];
        r[2] = ax[2];
        cross3(r + 3, ax, off);
      }
    } else if (jt == JNT_SLIDE) {
      float* r = cd + 6 * da;
      r[0] = r[1] = r[2] = 0.0f;
      r[3] = xaxis[0];
      r[4] = xaxis[1];
      r[5] = xaxis[2];
    } else {
      float* r = cd + 6 * da;
      r[0] = xaxis[0];
      r[1] = xaxis[1];
      r[2] = xaxis[2];
      cross3(r + 3, xaxis, off);
    }
  }
  __syncthreads();
}

// smooth.py:635-803 camlight
__device__ void camlight(const mjw_model_t& m, const mjw_data_t& d, int wid) {
  const float* xpos = d.xpos + (long)wid * m.nbody * 3;
  const float* xquat = d.xquat + (long)wid * m.nbody * 4;
  const float* sc = d.subtree_com + (long)wid * m.nbody * 3;
  const float* cam_pos = MR(cam_pos);
  const float* cam_quat = MR(cam_quat);
  const float* cam_pos0 = MR(cam_pos0);
  const float* cam_poscom0 = MR(cam_poscom0);
  const float* cam_mat0 = MR(cam_mat0);
  for (int c = tid(); c < m.ncam; c += BLK) {
    const int mode = m.cam_mode[c], b = m.cam_bodyid[c], tgt = m.cam_targetbodyid[c];
    const bool is_target = mode == CAM_TARGETBODY || mode == CAM_TARGETBODYCOM;
    float* cx = d.cam_xpos + ((long)wid * m.ncam + c) * 3;
    float* cm = d.cam_xmat + ((long)wid * m.ncam + c) * 9;
    if ((is_target && tgt < 0) || mode == CAM_FIXED) {
      float t[3], q[4];
      rot_vec_quat(t, cam_pos + 3 * c, xquat + 4 * b);
      for (int i = 0; i < 3; i++) cx[i] = xpos[3 * b + i] + t[i];
      mul_quat(q, xquat + 4 * b, cam_quat + 4 * c);
      quat_to_mat(cm, q);
    } else if (mode == CAM_TRACK) {
      for (int i = 0; i < 9; i++) cm[i] = cam_mat0[9 * c + i];
      for (int i = 0; i < 3; i++) cx[i] = xpos[3 * b + i] + cam_pos0[3 * c + i];
    } else if (mode == CAM_TRACKCOM) {
      for (int i = 0; i < 9; i++) cm[i] = cam_mat0[9 * c + i];
      for (int i = 0; i < 3; i++) cx[i] = sc[3 * b + i] + cam_poscom0[3 * c + i];
    } else {
      float t[3], m1[3], m2[3], m3[3];
      rot_vec_quat(t, cam_pos + 3 * c, xquat + 4 * b);
      for (int i = 0; i < 3; i++) cx[i] = xpos[3 * b + i] + t[i];
      const float* tp = mode == CAM_TARGETBODYCOM ? sc + 3 * tgt : xpos + 3 * tgt;
      for (int i = 0; i < 3; i++) m3[i] = cx[i] - tp[i];
      normalize3(m3);
      float z[3] = {0.0f, 0.0f, 1.0f};
      cross3(m1, z, m3);
      normalize3(m1);
      cross3(m2, m3, m1);
      normalize3(m2);
      for (int i = 0; i < 3; i++) {
        cm[3 * i] = m1[i];
        cm[3 * i + 1] = m2[i];
        cm[3 * i + 2] = m3[i];
      }
    }
  }
  const float* light_pos = MR(light_pos);
  const float* light_dir = MR(light_dir);
  const float* light_pos0 = MR(light_pos0);
  const float* light_poscom0 = MR(light_poscom0);
  const float* light_dir0 = MR(light_dir0);
  for (int l = tid(); l < m.nlight; l += BLK) {
    const int mode = m.light_mode[l], b = m.light_bodyid[l], tgt = m.light_targetbodyid[l];
    const bool is_target = mode == CAM_TARGETBODY || mode == CAM_TARGETBODYCOM;
    float lx[3], ld[3];  // built in registers, stored once (smooth.py:703-758)
    bool norm = true;
    if ((is_target && tgt < 0) || mode == CAM_FIXED) {
      float t[3];
      rot_vec_quat(t, light_pos + 3 * l, xquat + 4 * b);
      for (int i = 0; i < 3; i++) lx[i] = xpos[3 * b + i] + t[i];
      rot_vec_quat(ld, light_dir + 3 * l, xquat + 4 * b);
      norm = !(is_target && tgt < 0);  // smooth.py:726-732 returns before normalize
    } else if (mode == CAM_TRACK) {
      for (int i = 0; i < 3; i++) {
        ld[i] = light_dir0[3 * l + i];
        lx[i] = xpos[3 * b + i] + light_pos0[3 * l + i];
      }
    } else if (mode == CAM_TRACKCOM) {
      for (int i = 0; i < 3; i++) {
        ld[i] = light_dir0[3 * l + i];
        lx[i] = sc[3 * b + i] + light_poscom0[3 * l + i];
      }
    } else {
      float t[3];
      rot_vec_quat(t, light_pos + 3 * l, xquat + 4 * b);
      for (int i = 0; i < 3; i++) lx[i] = xpos[3 * b + i] + t[i];
      const float* tp = mode == CAM_TARGETBODYCOM ? sc + 3 * tgt : xpos + 3 * tgt;
      for (int i = 0; i < 3; i++) ld[i] = tp[i] - lx[i];
    }
    if (norm) normalize3(ld);
    float* gx = d.light_xpos + ((long)wid * m.nlight + l) * 3;
    float* gd = d.light_xdir + ((long)wid * m.nlight + l) * 3;
    for (int i = 0; i < 3; i++) {
      gx[i] = lx[i];
      gd[i] = ld[i];
    }
  }
}

// smooth.py:261-355 _flex_edges: length, velocity, d(length)/dq over the vertex bodies' own dofs
__device__ void flex_edges(const mjw_model_t& m, const mjw_data_t& d, int wid) {
  const float* fx = d.flexvert_xpos + (long)wid * m.nflexvert * 3;
  const float* sc = d.subtree_com + (long)wid * m.nbody * 3;
  const float* cdof = d.cdof + (long)wid * m.nv * 6;
  const float* qvel = d.qvel + (long)wid * m.nv;
  for (int f = 0; f < m.nflex; f++) {
    const int ea = m.flex_edgeadr[f], vb = m.flex_vertadr[f];
    for (int e = ea + tid(); e < ea + m.flex_edgenum[f]; e += BLK) {
      const int v[2] = {vb + m.flex_edge[2 * e], vb + m.flex_edge[2 * e + 1]};
      float vec[3], dir[3];
      for (int i = 0; i < 3; i++) vec[i] = fx[3 * v[1] + i] - fx[3 * v[0] + i];
      float len = sqrtf(dot3(vec, vec));
      for (int i = 0; i < 3; i++) dir[i] = len == 0.0f ? vec[i] : vec[i] / len;
      float J[6] = {0, 0, 0, 0, 0, 0}, vel = 0.0f;
      int slot = 0;
      for (int s2 = 0; s2 < 2; s2++) {
        const int b = m.flex_vertbodyid[v[s2]];
        float off[3];
        for (int i = 0; i < 3; i++) off[i] = fx[3 * v[s2] + i] - sc[3 * m.body_rootid[b] + i];
        for (int k = 0; k < m.body_dofnum[b] && slot < 6; k++) {
          const int dof = m.body_dofadr[b] + k;
          const float* c = cdof + 6 * dof;
          float cr[3], jp[3];
          cross3(cr, c, off);
          for (int i = 0; i < 3; i++) jp[i] = c[3 + i] + cr[i];
          const float jv = s2 ? dot3(jp, dir) : -dot3(jp, dir);
          vel += jv * qvel[dof];
          J[slot++] = jv;
        }
      }
      d.flexedge_length[(long)wid * m.nflexedge + e] = len;
      d.flexedge_velocity[(long)wid * m.nflexedge + e] = vel;
      for (int k = 0; k < 6; k++) d.flexedge_J[((long)wid * m.nflexedge + e) * 6 + k] = J[k];
    }
  }
}

// smooth.py:806-912 crb (subtree-range sums) + sparse qM rows (ancestors ascending, diagonal last)
__device__ void crb_qM(const mjw_model_t& m, const mjw_data_t& d, int wid) {
  const int nb = m.nbody;
  const float* cinert = d.cinert + (long)wid * nb * 10;
  float* crb = d.crb + (long)wid * nb * 10;
  for (int b = tid(); b < nb; b += BLK) {
    float s[10];
    for (int i = 0; i < 10; i++) s[i] = cinert[10 * b + i];
    if (b > 0)
      for (int c = b + 1; c < m.body_subtree_end[b]; c++)
        for (int i = 0; i < 10; i++) s[i] += cinert[10 * c + i];
    for (int i = 0; i < 10; i++) crb[10 * b + i] = s[i];
  }
  __syncthreads();
  const float* cdof = d.cdof + (long)wid * m.nv * 6;
  const float* armature = MR(dof_armature);
  float* qM = d.qM + (long)wid * m.nM;
  for (int i = tid(); i < m.nv; i += BLK) {
    float buf[6];
    inert_vec(buf, crb + 10 * m.dof_bodyid[i], cdof + 6 * i);
    const int adr = m.M_rowadr[i], nnz = m.M_rownnz[i];
    float s = armature[i];
    for (int k = 0; k < 6; k++) s += cdof[6 * i + k] * buf[k];
    qM[adr + nnz - 1] = s;
    int j = m.dof_parentid[i];
    for (int p = nnz - 2; p >= 0; p--, j = m.dof_parentid[j]) {
      float q = 0.0f;
      for (int k = 0; k < 6; k++) q += cdof[6 * j + k] * buf[k];
      qM[adr + p] = q;
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// tendons (fixed and spatial; mjw_tendon.h restates smooth.py:3085-3465 for both paths): lengths and
// Jacobian rows into the Data, then armature into the sparse M rows (smooth.py:916-1000)
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ TenFrames ten_frames(const mjw_model_t& m, const mjw_data_t& d, int wid) {
  return TenFrames{d.site_xpos + (long)wid * m.nsite * 3, d.geom_xpos + (long)wid * m.ngeom * 3, d.geom_xmat + (long)wid * m.ngeom * 9,
                   d.subtree_com + (long)wid * m.nbody * 3, d.cdof + (long)wid * m.nv * 6};
}

// position of M[i][j] (j = i or an ancestor dof of i) in the ancestor-row layout, or -1
__device__ __forceinline__ int m_pos(const mjw_model_t& m, int i, int j) {
  const int adr = m.M_rowadr[i], rn = m.M_rownnz[i];
  if (i == j) return adr + rn - 1;
  for (int q = 0; q < rn - 1; q++)
    if (m.M_colind[adr + q] == j) return adr + q;
  return -1;
}

__device__ void tendons(const mjw_model_t& m, const mjw_data_t& d, int wid) {
  tendon_pos(m, d, d.qpos + (long)wid * m.nq, ten_frames(m, d, wid), wid, tid(), BLK);
  __syncthreads();
  const float* arm = MR(tendon_armature);
  float* qM = d.qM + (long)wid * m.nM;
  for (int t = 0; t < m.ntendon; t++) {  // uniform: one tendon's (i >= j) pairs per round
    if (arm[t] == 0.0f) continue;
    const int rn = m.ten_J_rownnz[t], ra = m.ten_J_rowadr[t];
    const float* J = d.ten_J + (long)wid * m.nJten + ra;
    for (int p = tid(); p < rn * rn; p += BLK) {
      const int k1 = p / rn, k2 = p - k1 * rn;
      if (k2 > k1) continue;
      const int pos = m_pos(m, m.ten_J_colind[ra + k1], m.ten_J_colind[ra + k2]);
      if (pos >= 0) qM[pos] += arm[t] * J[k1] * J[k2];
    }
    __syncthreads();
  }
}

// M = L' D L per kinematic tree (smooth.py:1003-1064, mj_factorM order): LD = factor(M + diag(add))
__device__ void factor_trees(const mjw_model_t& m, const float* M, float* LD, const float* add, float add_scale) {
  for (int t = tid(); t < m.ntree; t += BLK) {
    const int a = m.tree_dofadr[t], e = m.tree_dofadr[t + 1];
    for (int k = a; k < e; k++) {
      const int adr = m.M_rowadr[k], nnz = m.M_rownnz[k];
      for (int p = 0; p < nnz; p++) LD[adr + p] = M[adr + p];
      if (add) LD[adr + nnz - 1] += add_scale * add[k];
    }
    for (int k = e - 1; k >= a; k--) {
      const int adr = m.M_rowadr[k], nnz = m.M_rownnz[k];
      const float dk = LD[adr + nnz - 1];
      for (int p = nnz - 2; p >= 0; p--) {
        const int i = m.M_colind[adr + p];
        const float tmp = LD[adr + p] / dk;
        const int adri = m.M_rowadr[i];
        for (int q = 0; q <= p; q++) LD[adri + q] -= tmp * LD[adr + q];
        LD[adr + p] = tmp;
      }
    }
  }
}

// chain trees of at most 4 dofs (each dof's parent is the previous one: a flex vertex's slide x/y/z)
// run in registers with every load issued up front; row k of such a tree holds columns a..a+k
constexpr int CHAIN = 4;
__device__ __forceinline__ bool chain_tree(const mjw_model_t& m, int a, int e) {
  if (e - a > CHAIN) return false;
  for (int k = a + 1; k < e; k++)
    if (m.dof_parentid[k] != k - 1) return false;
  return true;
}

// the tree's lower triangle (L[k][p], p <= k, diagonal at p = k) and x into registers
__device__ __forceinline__ void chain_load(const mjw_model_t& m, const float* A, const float* x, int a, int n, float (&L)[CHAIN][CHAIN],
                                           float (&xs)[CHAIN]) {
#pragma unroll
  for (int k = 0; k < CHAIN; k++) {
    xs[k] = k < n ? x[a + k] : 0.0f;
    const int adr = k < n ? m.M_rowadr[a + k] : 0;
#pragma unroll
    for (int p = 0; p <= k; p++) L[k][p] = k < n ? A[adr + p] : 0.0f;
  }
}

// branched trees of at most TREE dofs (an arm whose two fingers hang off the wrist): x (and y) in registers,
// the sparse loops of the general path below unchanged, each indexed access to a dof of the tree done as a
// compare-select over the tree's TREE registers (no register array indexed at run time, no stack).  The
// updates are the general path's, in its order, so the result is bitwise its result -- without its chain of
// dependent global read-modify-writes (one tree's thread walked ~60 per call: aloha_cloth's preconditioner
// measured 10.7 % of the step's wave-cycles, profiles/r06_sparse_prof.json)
constexpr int TREE = 8;
template <int T>
__device__ __forceinline__ float tree_get(const float (&v)[T], int j) {
  float g = 0.0f;
#pragma unroll
  for (int i = 0; i < T; i++) g = j == i ? v[i] : g;
  return g;
}
// x = (L' D L)^-1 x for the tree of dofs [a, a + n), n <= T (smooth.py:2813-2846, as solve_trees)
template <int T>
__device__ __forceinline__ void tree_solve_small(const mjw_model_t& m, const float* LD, float* x, int a, int n) {
  float xs[T];
#pragma unroll
  for (int k = 0; k < T; k++) xs[k] = k < n ? x[a + k] : 0.0f;
#pragma unroll
  for (int k = T - 1; k >= 0; k--) {
    if (k >= n) continue;
    const int adr = m.M_rowadr[a + k], nnz = m.M_rownnz[a + k];
    const float xk = xs[k];
#pragma unroll
    for (int p = 0; p < T - 1; p++) {
      if (p >= nnz - 1) break;
      const int cj = m.M_colind[adr + p] - a;
      const float v = LD[adr + p];
#pragma unroll
      for (int j = 0; j < k; j++)
        if (cj == j) xs[j] -= v * xk;
    }
  }
#pragma unroll
  for (int k = 0; k < T; k++)
    if (k < n) xs[k] /= LD[m.M_rowadr[a + k] + m.M_rownnz[a + k] - 1];
#pragma unroll
  for (int k = 0; k < T; k++) {
    if (k >= n) continue;
    const int adr = m.M_rowadr[a + k], nnz = m.M_rownnz[a + k];
    float sk = xs[k];
#pragma unroll
    for (int p = 0; p < T - 1; p++) {
      if (p >= nnz - 1) break;
      sk -= LD[adr + p] * tree_get<T>(xs, m.M_colind[adr + p] - a);
    }
    xs[k] = sk;
  }
#pragma unroll
  for (int k = 0; k < T; k++)
    if (k < n) x[a + k] = xs[k];
}
// y = M x for the tree of dofs [a, a + n), n <= T (support.py:67-101, as mul_m_trees' general path)
template <int T>
__device__ __forceinline__ void tree_mul_small(const mjw_model_t& m, const float* M, const float* x, float* y, int a, int n) {
  float xs[T], ys[T];
#pragma unroll
  for (int k = 0; k < T; k++) {
    xs[k] = k < n ? x[a + k] : 0.0f;
    ys[k] = 0.0f;
  }
#pragma unroll
  for (int k = 0; k < T; k++) {
    if (k >= n) continue;
    const int adr = m.M_rowadr[a + k], nnz = m.M_rownnz[a + k];
    float sk = M[adr + nnz - 1] * xs[k];
#pragma unroll
    for (int p = 0; p < T - 1; p++) {
      if (p >= nnz - 1) break;
      const int i = m.M_colind[adr + p] - a;
      const float v = M[adr + p];
      sk += v * tree_get<T>(xs, i);
#pragma unroll
      for (int j = 0; j < k; j++)
        if (i == j) ys[j] += v * xs[k];
    }
    ys[k] += sk;
  }
#pragma unroll
  for (int k = 0; k < T; k++)
    if (k < n) y[a + k] = ys[k];
}

// x = (L' D L)^-1 x of one chain tree held dense in registers (chain_load)
template <int T>
__device__ __forceinline__ void tree_solve_regs(const float (&L)[T][T], float (&xs)[T], int n) {
#pragma unroll
  for (int k = T - 1; k >= 0; k--)
    if (k < n) {
#pragma unroll
      for (int p = 0; p < k; p++) xs[p] -= L[k][p] * xs[k];
    }
#pragma unroll
  for (int k = 0; k < T; k++)
    if (k < n) xs[k] /= L[k][k];
#pragma unroll
  for (int k = 0; k < T; k++)
    if (k < n) {
      float sk = xs[k];
#pragma unroll
      for (int p = 0; p < k; p++) sk -= L[k][p] * xs[p];
      xs[k] = sk;
    }
}

// x = (L' D L)^-1 x in place, per tree (smooth.py:2813-2846)
__device__ __forceinline__ void solve_trees(const mjw_model_t& m, const float* LD, float* x) {
  for (int t = tid(); t < m.ntree; t += nthr()) {
    const int a = m.tree_dofadr[t], e = m.tree_dofadr[t + 1];
    const int n = e - a;
    if (chain_tree(m, a, e)) {
      float L[CHAIN][CHAIN], xs[CHAIN];
      chain_load(m, LD, x, a, n, L, xs);
      tree_solve_regs<CHAIN>(L, xs, n);
#pragma unroll
      for (int k = 0; k < CHAIN; k++)
        if (k < n) x[a + k] = xs[k];
      continue;
    }
    if (MJW_SP_TREE && n <= TREE) {
      tree_solve_small<TREE>(m, LD, x, a, n);
      continue;
    }
    for (int k = e - 1; k >= a; k--) {
      const int adr = m.M_rowadr[k], nnz = m.M_rownnz[k];
      const float xk = x[k];
      for (int p = 0; p < nnz - 1; p++) x[m.M_colind[adr + p]] -= LD[adr + p] * xk;
    }
    for (int k = a; k < e; k++) x[k] /= LD[m.M_rowadr[k] + m.M_rownnz[k] - 1];
    for (int k = a; k < e; k++) {
      const int adr = m.M_rowadr[k], nnz = m.M_rownnz[k];
      float s = x[k];
      for (int p = 0; p < nnz - 1; p++) s -= LD[adr + p] * x[m.M_colind[adr + p]];
      x[k] = s;
    }
  }
}

// y = M x of one tree held dense in registers (rows k < n of y)
template <int T>
__device__ __forceinline__ void tree_mul_regs(const float (&L)[T][T], const float (&xs)[T], int n, float* y) {
#pragma unroll
  for (int k = 0; k < T; k++)
    if (k < n) {
      float sk = L[k][k] * xs[k];
#pragma unroll
      for (int p = 0; p < k; p++) sk += L[k][p] * xs[p];
#pragma unroll
      for (int j = k + 1; j < T; j++)
        if (j < n) sk += L[j][k] * xs[j];
      y[k] = sk;
    }
}

// y = M x (support.py:67-101 sparse mul_m), per tree: lower rows plus their transposes
__device__ __forceinline__ void mul_m_trees(const mjw_model_t& m, const float* M, const float* x, float* y) {
  for (int t = tid(); t < m.ntree; t += nthr()) {
    const int a = m.tree_dofadr[t], e = m.tree_dofadr[t + 1];
    const int n = e - a;
    if (chain_tree(m, a, e)) {
      float L[CHAIN][CHAIN], xs[CHAIN];
      chain_load(m, M, x, a, n, L, xs);
      tree_mul_regs<CHAIN>(L, xs, n, y + a);
      continue;
    }
    if (MJW_SP_TREE && n <= TREE) {
      tree_mul_small<TREE>(m, M, x, y, a, n);
      continue;
    }
    for (int k = a; k < e; k++) y[k] = 0.0f;
    for (int k = a; k < e; k++) {
      const int adr = m.M_rowadr[k], nnz = m.M_rownnz[k];
      float s = M[adr + nnz - 1] * x[k];
      for (int p = 0; p < nnz - 1; p++) {
        const int i = m.M_colind[adr + p];
        s += M[adr + p] * x[i];
        y[i] += M[adr + p] * x[k];
      }
      y[k] += s;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// collision: geom pairs (collision_driver.py:697-789 + primitive narrowphase), flex triangles vs
// geoms (collision_flex.py:381-529) and flex vertices vs planes (:261-378)
// ---------------------------------------------------------------------------------------------
// collision_driver.py:274-321 on global frames
__device__ bool broadphase(const mjw_model_t& m, int wid, const float* gx, const float* gm, int g1, int g2) {
  const float* geom_aabb = MR(geom_aabb);
  const float* geom_rbound = MR(geom_rbound);
  const float* geom_margin = MR(geom_margin);
  const float rb1 = geom_rbound[g1], rb2 = geom_rbound[g2], mg1 = geom_margin[g1], mg2 = geom_margin[g2];
  const float *xp1 = gx + 3 * g1, *xp2 = gx + 3 * g2, *xm1 = gm + 9 * g1, *xm2 = gm + 9 * g2;
  const int filt = m.opt_broadphase_filter;
  if (rb1 == 0.0f || rb2 == 0.0f) {
    if (filt & FILTER_PLANE) {
      if (rb1 == 0.0f) {
        float dif[3] = {xp2[0] - xp1[0], xp2[1] - xp1[1], xp2[2] - xp1[2]}, n[3] = {xm1[2], xm1[5], xm1[8]};
        return dot3(dif, n) <= rb2 + mg1 + mg2;
      }
      float dif[3] = {xp1[0] - xp2[0], xp1[1] - xp2[1], xp1[2] - xp2[2]}, n[3] = {xm2[2], xm2[5], xm2[8]};
      return dot3(dif, n) <= rb1 + mg1 + mg2;
    }
    return true;
  }
  if (filt & FILTER_SPHERE) {
    const float bound = rb1 + rb2 + mg1 + mg2;
    float dif[3] = {xp2[0] - xp1[0], xp2[1] - xp1[1], xp2[2] - xp1[2]};
    if (!(dot3(dif, dif) <= bound * bound)) return false;
  }
  if (filt & FILTER_AABB)
    if (!aabb_filter(geom_aabb + 6 * g1, geom_aabb + 6 * g2, geom_aabb + 6 * g1 + 3, geom_aabb + 6 * g2 + 3, mg1 + mg2, xp1, xp2, xm1, xm2))
      return false;
  if (filt & FILTER_OBB)
    if (!obb_filter(geom_aabb + 6 * g1, geom_aabb + 6 * g2, geom_aabb + 6 * g1 + 3, geom_aabb + 6 * g2 + 3, mg1 + mg2, xp1, xp2, xm1, xm2))
      return false;
  return true;
}

struct ConOut {
  float margin, includemargin;
  int condim, g1, g2, flex, vert;
  float friction[5], solref[2], solreffriction[2], solimp[5];
};

// `frame` (9, optional) keeps the narrowphase's own tangents (plane_capsule / capsule_capsule align
// them with the capsule axis, collision_primitive.py); otherwise make_frame(nrm) (math.py:246-257)
__device__ void write_contact(const mjw_model_t& m, const mjw_data_t& d, int wid, int slot, int lim, const ConOut& o, float dist,
                              const float* pos, const float* nrm, const float* frame = nullptr) {
  if (slot < 0 || slot >= lim || slot >= d.naconmax) return;
  d.contact_dist[slot] = dist;
  for (int i = 0; i < 3; i++) d.contact_pos[3 * (long)slot + i] = pos[i];
  float fr[9];
  if (frame) {
    for (int i = 0; i < 9; i++) fr[i] = frame[i];
  } else {
    make_frame(fr, nrm);
  }
  for (int i = 0; i < 9; i++) d.contact_frame[9 * (long)slot + i] = fr[i];
  d.contact_includemargin[slot] = o.includemargin;
  for (int i = 0; i < 5; i++) d.contact_friction[5 * (long)slot + i] = o.friction[i];
  for (int i = 0; i < 2; i++) d.contact_solref[2 * (long)slot + i] = o.solref[i];
  for (int i = 0; i < 2; i++) d.contact_solreffriction[2 * (long)slot + i] = o.solreffriction[i];
  for (int i = 0; i < 5; i++) d.contact_solimp[5 * (long)slot + i] = o.solimp[i];
  d.contact_dim[slot] = o.condim;
  d.contact_geom[2 * (long)slot] = o.g1;
  d.contact_geom[2 * (long)slot + 1] = o.g2;
  d.contact_flex[2 * (long)slot] = -1;
  d.contact_flex[2 * (long)slot + 1] = o.flex;
  d.contact_vert[2 * (long)slot] = -1;
  d.contact_vert[2 * (long)slot + 1] = o.vert;
  for (int i = 0; i < m.nmaxpyramid; i++) d.contact_efc_address[(long)slot * m.nmaxpyramid + i] = -1;
  d.contact_worldid[slot] = wid;
  d.contact_type[slot] = 1;
  d.contact_geomcollisionid[slot] = 0;
}

// out-of-line copies of the (force-inlined, shared with the dense kernel) primitive narrowphase:
// collide_item runs three ways per step, and inlining every pair type into it spilled to scratch
__device__ __noinline__ void nl_capsule_capsule(Con2& c, const float* p1, const float* n1, float r1, float h1, const float* p2,
                                                const float* n2, float r2, float h2, float margin) {
  capsule_capsule(c, p1, n1, r1, h1, p2, n2, r2, h2, margin);
}
__device__ __noinline__ void nl_capsule_box(Con2& c, const float* p1, const float* n1, float r1, float h1, const float* p2,
                                            const float* r2, const float* s2) {
  capsule_box(c, p1, n1, r1, h1, p2, r2, s2);
}
__device__ __noinline__ void nl_plane_capsule(Con2& c, const float* n1, const float* p1, const float* p2, const float* n2, float r,
                                              float h) {
  plane_capsule(c, n1, p1, p2, n2, r, h);
}
__device__ __noinline__ float nl_sphere_box(float* pos, float* nrm, const float* p1, float r, const float* p2, const float* r2,
                                            const float* s2) {
  return sphere_box(pos, nrm, p1, r, p2, r2, s2);
}

__device__ __noinline__ float nl_plane_ellipsoid(float* pos, const float* n1, const float* p1, const float* p2, const float* r2,
                                                 const float* s2) {
  return plane_ellipsoid(pos, n1, p1, p2, r2, s2);
}
__device__ __noinline__ float nl_sphere_cylinder(float* pos, float* nrm, const float* p1, float r, const float* p2, const float* n2,
                                                 float rc, float hc) {
  return sphere_cylinder(pos, nrm, p1, r, p2, n2, rc, hc);
}
__device__ __noinline__ void nl_plane_cylinder_k(int k, const float* n1, const float* p1, const float* p2, const float* n2, float r,
                                                 float h, float* dist, float* pos) {
  plane_cylinder_k(k, n1, p1, p2, n2, r, h, dist, pos);
}

// one collision item: a geom pair, a (flex element, collidable geom) pair or a (flex vertex, plane)
// pair.  Returns the number of contacts; writes them from pool slot `base` when base >= 0.
__device__ __forceinline__ int collide_item(const mjw_model_t& m, const mjw_data_t& d, int wid, int item, int base, int* npassed, int lim = 0x7fffffff,
                                        const float* fbox = nullptr) {
  const float* gx = d.geom_xpos + (long)wid * m.ngeom * 3;
  const float* gm = d.geom_xmat + (long)wid * m.ngeom * 9;
  const float* geom_size = MR(geom_size);
  int cnt = 0;
  if (item < m.nxn) {
    int g1 = m.nxn_geom_pair[2 * item], g2 = m.nxn_geom_pair[2 * item + 1];
    if (!(broadphase(m, wid, gx, gm, g1, g2) || m.nxn_pairid[2 * item + 1] >= 0)) return 0;
    if (npassed) (*npassed)++;
    ConOut o;
    float gap;
    contact_params(m, wid, g1, g2, m.nxn_pairid[2 * item], &o.margin, &gap, &o.condim, o.friction, o.solref, o.solimp, o.solreffriction);
    o.includemargin = o.margin - gap;
    o.g1 = g1;
    o.g2 = g2;
    o.flex = o.vert = -1;
    const int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
    const float *p1 = gx + 3 * g1, *p2 = gx + 3 * g2, *r1 = gm + 9 * g1, *r2 = gm + 9 * g2;
    const float *s1 = geom_size + 3 * g1, *s2 = geom_size + 3 * g2;
    const float n1[3] = {r1[2], r1[5], r1[8]}, n2[3] = {r2[2], r2[5], r2[8]};
    const int ccdslot = m.nxn_ccdid[item];
    if (ccdslot >= 0) {
      // convex pair: results of the CCD pre-pass (ccd_kernel below), n contacts, each with its distance and
      // frame make_frame(normal) (collision_convex.py:763-852; heightfields :495-695)
      const float* out = d.ccd_out + ((long)wid * m.nxn_ccd + ccdslot) * CCD_OUT;
      const int n = (int)out[0];
      if (m.nxn_pairid[2 * item] < -1) return 0;
      for (int k = 0; k < n; k++) {
        if (!(out[4 + 4 * k] < o.margin)) continue;
        if (base >= 0) write_contact(m, d, wid, base + cnt, lim, o, out[4 + 4 * k], out + 5 + 4 * k, out + 20 + 3 * k);
        cnt++;
      }
      return cnt;
    }
    if (t1 == GEOM_PLANE && t2 == GEOM_MESH) {
      float pd[4], pp[4][3];
      const int mid = m.geom_dataid[g2];
      const int n = plane_mesh(n1, p1, p2, r2, MR(mesh_vert) + 3 * (long)m.mesh_vertadr[mid], m.mesh_vertnum[mid], pd, pp);
      for (int k = 0; k < n; k++) {
        if (!(pd[k] < o.margin) || m.nxn_pairid[2 * item] < -1) continue;
        if (base >= 0) write_contact(m, d, wid, base + cnt, lim, o, pd[k], pp[k], n1);
        cnt++;
      }
      return cnt;
    }
    const int ncand = (t1 == GEOM_PLANE && t2 == GEOM_BOX) ? 8 : ((t1 == GEOM_PLANE && t2 == GEOM_CYLINDER) ? 4 : 2);
    Con2 c;
    c.n = 0;
    if (t1 == GEOM_PLANE && t2 == GEOM_SPHERE) {
      c.dist[0] = plane_sphere(c.pos[0], n1, p1, p2, s2[0]);
      make_frame(c.frame[0], n1);
      c.n = 1;
    } else if (t1 == GEOM_PLANE && t2 == GEOM_CAPSULE) {
      nl_plane_capsule(c, n1, p1, p2, n2, s2[0], s2[1]);
    } else if (t1 == GEOM_SPHERE && t2 == GEOM_SPHERE) {
      float nrm[3];
      c.dist[0] = sphere_sphere(c.pos[0], nrm, p1, s1[0], p2, s2[0]);
      make_frame(c.frame[0], nrm);
      c.n = 1;
    } else if (t1 == GEOM_SPHERE && t2 == GEOM_CAPSULE) {
      float a[3], b[3], pt[3], nrm[3];
      for (int i = 0; i < 3; i++) { a[i] = p2[i] - n2[i] * s2[1]; b[i] = p2[i] + n2[i] * s2[1]; }
      closest_segment_point(pt, a, b, p1);
      c.dist[0] = sphere_sphere(c.pos[0], nrm, p1, s1[0], pt, s2[0]);
      make_frame(c.frame[0], nrm);
      c.n = 1;
    } else if (t1 == GEOM_CAPSULE && t2 == GEOM_CAPSULE) {
      nl_capsule_capsule(c, p1, n1, s1[0], s1[1], p2, n2, s2[0], s2[1], o.margin);
    } else if (t1 == GEOM_SPHERE && t2 == GEOM_BOX) {
      float nrm[3];
      c.dist[0] = nl_sphere_box(c.pos[0], nrm, p1, s1[0], p2, r2, s2);
      make_frame(c.frame[0], nrm);
      c.n = 1;
    } else if (t1 == GEOM_CAPSULE && t2 == GEOM_BOX) {
      nl_capsule_box(c, p1, n1, s1[0], s1[1], p2, r2, s2);
    } else if (t1 == GEOM_PLANE && t2 == GEOM_ELLIPSOID) {  // collision_primitive.py:665-733
      c.dist[0] = nl_plane_ellipsoid(c.pos[0], n1, p1, p2, r2, s2);
      make_frame(c.frame[0], n1);
      c.n = 1;
    } else if (t1 == GEOM_SPHERE && t2 == GEOM_CYLINDER) {  // collision_primitive.py:882-960
      float nrm[3];
      c.dist[0] = nl_sphere_cylinder(c.pos[0], nrm, p1, s1[0], p2, n2, s2[0], s2[1]);
      make_frame(c.frame[0], nrm);
      c.n = 1;
    }
    const int nk = ncand == 2 ? c.n : ncand;
    for (int k = 0; k < nk; k++) {
      float dist, pos[3], nrm[3];
      if (ncand == 8) {
        dist = plane_box_corner(k, n1, p1, p2, r2, s2, pos);
        for (int i = 0; i < 3; i++) nrm[i] = n1[i];
      } else if (ncand == 4) {
        nl_plane_cylinder_k(k, n1, p1, p2, n2, s2[0], s2[1], &dist, pos);
        for (int i = 0; i < 3; i++) nrm[i] = n1[i];
      } else {
        dist = c.dist[k];
        for (int i = 0; i < 3; i++) { pos[i] = c.pos[k][i]; nrm[i] = c.frame[k][i]; }
      }
      if (!(dist < o.margin) || m.nxn_pairid[2 * item] < -1) continue;
      if (base >= 0) write_contact(m, d, wid, base + cnt, lim, o, dist, pos, nrm, ncand == 2 ? c.frame[k] : nullptr);
      cnt++;
    }
    return cnt;
  }
  item -= m.nxn;
  const float* fx = d.flexvert_xpos + (long)wid * m.nflexvert * 3;
  for (int f = 0; f < m.nflex; f++) {
    const int ncg = m.flex_cgeomadr[f + 1] - m.flex_cgeomadr[f];
    // dim 2: the elements; dim 3: the boundary (shell) triangles (collision_flex.py:531-683); dim 1: none
    const bool shell = m.flex_dim[f] == 3;
    const int nitem = (m.flex_dim[f] == 2 ? m.flex_elemnum[f] : (shell ? m.flex_shellnum[f] : 0)) * ncg;
    if (item >= nitem) {
      item -= nitem;
      continue;
    }
    const int el = item / ncg, g = m.flex_cgeom[m.flex_cgeomadr[f] + item % ncg];
    if (fbox && f < SP_FBOX) {
      // flex-level cull (exact: every candidate lies within the flex's vertex box grown by the
      // radius, the margin and the geom's bounding sphere)
      const float* b = fbox + 6 * f;
      const float grow = MR(geom_rbound)[g] + MR(flex_radius)[f] + fmaxf(MR(geom_margin)[g] + MR(flex_margin)[f], 0.0f) + 1e-5f;
      const float* gp = gx + 3 * g;
      if (gp[0] < b[0] - grow || gp[1] < b[1] - grow || gp[2] < b[2] - grow || gp[0] > b[3] + grow || gp[1] > b[4] + grow ||
          gp[2] > b[5] + grow)
        return 0;
    }
    const int* ev = shell ? m.flex_shell + m.flex_shelldataadr[f] + 3 * el : m.flex_elem + m.flex_elemdataadr[f] + 3 * el;
    const float* t[3];
    float cen[3] = {0.0f, 0.0f, 0.0f}, rad = 0.0f;
    for (int k = 0; k < 3; k++) {
      t[k] = fx + 3 * (m.flex_vertadr[f] + ev[k]);
      for (int i = 0; i < 3; i++) cen[i] += t[k][i] * (1.0f / 3.0f);
    }
    for (int k = 0; k < 3; k++) {
      float dv[3] = {t[k][0] - cen[0], t[k][1] - cen[1], t[k][2] - cen[2]};
      rad = fmaxf(rad, sqrtf(dot3(dv, dv)));
    }
    const float tr = MR(flex_radius)[f];
    const float margin = MR(geom_margin)[g] + MR(flex_margin)[f];
    // exact bounding-sphere cull: every candidate distance is at least the sphere gap
    float dg[3] = {gx[3 * g] - cen[0], gx[3 * g + 1] - cen[1], gx[3 * g + 2] - cen[2]};
    const float bound = MR(geom_rbound)[g] + rad + tr + fmaxf(margin, 0.0f) + 1e-5f;
    if (dot3(dg, dg) > bound * bound) return 0;
    Cand c[2];
    const int n = geom_triangle(c, m.geom_type[g], gx + 3 * g, gm + 9 * g, geom_size + 3 * g, t, tr);
    ConOut o;
    const float* gf = MR(geom_friction) + 3 * g;
    o.friction[0] = o.friction[1] = fmaxf(MJW_MINMU, gf[0]);
    o.friction[2] = fmaxf(MJW_MINMU, gf[1]);
    o.friction[3] = o.friction[4] = fmaxf(MJW_MINMU, gf[2]);
    for (int i = 0; i < 2; i++) { o.solref[i] = MR(geom_solref)[2 * g + i]; o.solreffriction[i] = 0.0f; }
    for (int i = 0; i < 5; i++) o.solimp[i] = MR(geom_solimp)[5 * g + i];
    o.margin = o.includemargin = margin;
    o.condim = m.geom_condim[g];
    o.g1 = g;
    o.g2 = -1;
    o.flex = f;
    o.vert = ev[0];
    for (int k = 0; k < n; k++) {
      if (!(c[k].dist < margin) || c[k].dist >= MJW_MAXVAL) continue;
      if (base >= 0) write_contact(m, d, wid, base + cnt, lim, o, c[k].dist, c[k].pos, c[k].nrm);
      cnt++;
    }
    return cnt;
  }
  // flex vertex vs plane
  const int v = item / max(m.nplane, 1), g = m.plane_geom[item % max(m.nplane, 1)];
  const int f = m.flex_vertflexid[v];
  const float *pp = gx + 3 * g, *pr = gm + 9 * g;
  const float n[3] = {pr[2], pr[5], pr[8]};
  const float* x = fx + 3 * v;
  const float df[3] = {x[0] - pp[0], x[1] - pp[1], x[2] - pp[2]};
  const float margin = MR(geom_margin)[g] + MR(flex_margin)[f];
  const float fr = MR(flex_radius)[f];
  const float dist = dot3(df, n) - fr;
  if (!(dist < margin)) return 0;
  if (base >= 0) {
    ConOut o;
    const float *gf = MR(geom_friction) + 3 * g, *ff = MR(flex_friction) + 3 * f;
    const float f0 = fmaxf(gf[0], ff[0]), f1 = fmaxf(gf[1], ff[1]), f2 = fmaxf(gf[2], ff[2]);
    o.friction[0] = o.friction[1] = fmaxf(MJW_MINMU, f0);
    o.friction[2] = fmaxf(MJW_MINMU, f1);
    o.friction[3] = o.friction[4] = fmaxf(MJW_MINMU, f2);
    for (int i = 0; i < 2; i++) { o.solref[i] = MR(geom_solref)[2 * g + i]; o.solreffriction[i] = 0.0f; }
    for (int i = 0; i < 5; i++) o.solimp[i] = MR(geom_solimp)[5 * g + i];
    o.margin = o.includemargin = margin;
    o.condim = max(m.geom_condim[g], m.flex_condim[f]);
    o.g1 = g;
    o.g2 = -1;
    o.flex = f;
    o.vert = v - m.flex_vertadr[f];
    float pos[3];
    for (int i = 0; i < 3; i++) pos[i] = x[i] - n[i] * (dist * 0.5f + fr);
    write_contact(m, d, wid, base, lim, o, dist, pos, n);
  }
  return 1;
}

__device__ int ncollide_items(const mjw_model_t& m) {
  int n = m.nxn + m.nflexvert * m.nplane;
  for (int f = 0; f < m.nflex; f++)
    n += (m.flex_dim[f] == 2 ? m.flex_elemnum[f] : (m.flex_dim[f] == 3 ? m.flex_shellnum[f] : 0)) * (m.flex_cgeomadr[f + 1] - m.flex_cgeomadr[f]);
  return n;
}

// count, reserve one contiguous pool range per world, then write in item order
__device__ void collision(const mjw_model_t& m, const mjw_data_t& d, int wid, Smem& sm) {
  int* ncw = d.ncon_world + 2 * (long)wid;
  if (m.opt_disableflags & (DSBL_CONSTRAINT | DSBL_CONTACT)) {
    if (tid() == 0) { ncw[0] = 0; ncw[1] = 0; }
    __syncthreads();
    return;
  }
  const int nitem = ncollide_items(m);
  // per-item contact counts kept in LDS (forward_kernel's dynamic LDS, sized by sparse_launch), so
  // the scan pass needs no second narrowphase evaluation; larger models recount
  extern __shared__ unsigned char s_items[];
  // vertex bounding box of each (of the first SP_FBOX) flex: block min-reduction of (min, -max)
  const float* fbox = nullptr;
  if (m.nflex > 0) {
    const float* fx = d.flexvert_xpos + (long)wid * m.nflexvert * 3;
    for (int f = 0; f < min(m.nflex, SP_FBOX); f++) {
      float v[6] = {MJW_MAXVAL, MJW_MAXVAL, MJW_MAXVAL, MJW_MAXVAL, MJW_MAXVAL, MJW_MAXVAL};
      const int v0 = m.flex_vertadr[f], v1 = f + 1 < m.nflex ? m.flex_vertadr[f + 1] : m.nflexvert;
      for (int i = v0 + tid(); i < v1; i += BLK)
        for (int k = 0; k < 3; k++) {
          v[k] = fminf(v[k], fx[3 * i + k]);
          v[3 + k] = fminf(v[3 + k], -fx[3 * i + k]);
        }
      const int lane = tid() & 63, wv = tid() >> 6;
#pragma unroll
      for (int k = 0; k < 6; k++)
        for (int o = 32; o > 0; o >>= 1) v[k] = fminf(v[k], __shfl_xor(v[k], o, 64));
      __syncthreads();
      if (lane == 0)
        for (int k = 0; k < 6; k++) sm.red[wv][k] = v[k];
      __syncthreads();
      if (tid() < 6) {
        float r = sm.red[0][tid()];
        for (int w = 1; w < (nthr() >> 6); w++) r = fminf(r, sm.red[w][tid()]);
        sm.fbox[f][tid()] = tid() < 3 ? r : -r;
      }
      __syncthreads();
    }
    fbox = &sm.fbox[0][0];
  }
  // the same bound sparse_launch sizes the LDS with (>= nitem)
  const bool cached = (long)m.nxn + (long)m.nflexvert * m.nplane + ((long)m.nflexelem + m.nflexshelldata / 3) * m.nflexcg <= SP_LDS_ITEMS_MAX;
  int cnt = 0, passed = 0;
  for (int it = tid(); it < nitem; it += BLK) {
    const int n = collide_item(m, d, wid, it, -1, &passed, 0x7fffffff, fbox);
    cnt += n;
    if (cached) s_items[it] = (unsigned char)n;
  }
  float v[2] = {(float)cnt, (float)passed};
  block_sum<2>(v, sm);
  // one global pool of naconmax contacts shared by all worlds, as the reference's (collision_core.py:
  // 212-231: nacon counts every contact found, contacts past the pool are dropped): the world
  // reserves its contiguous block with one atomic and keeps the part of it inside the pool, its
  // contacts in item order.  Which world overflows depends on the atomics' order, as there.
  const int total = (int)v[0];
  if (tid() == 0) {
    // the broadphase count rides in the same 64-bit atomic when ncollision follows nacon (io.py), as in
    // the dense step kernel
    const int passed = (int)v[1];
    const bool cnt64 = d.ncollision == d.nacon + 1;
    int base = 0;
    if (total && cnt64)
      base = (int)(unsigned)atomicAdd(reinterpret_cast<unsigned long long*>(d.nacon), ((unsigned long long)passed << 32) | (unsigned)total);
    else if (total)
      base = atomicAdd(d.nacon, total);
    sm.ival[0] = base;
    sm.ival[1] = total ? max(0, min(total, d.naconmax - base)) : 0;
    if (passed > 0 && !(total && cnt64)) atomicAdd(d.ncollision, passed);
    ncw[0] = base;
    ncw[1] = sm.ival[1];
  }
  __syncthreads();
  const int keep = sm.ival[1];
  const int start = sm.ival[0], lim = start + keep;
  int run = start;
  if (keep) {
    for (int c0 = 0; c0 < nitem && run < lim; c0 += BLK) {
      const int it = c0 + tid();
      const int n = it < nitem ? (cached ? (int)s_items[it] : collide_item(m, d, wid, it, -1, nullptr, 0x7fffffff, fbox)) : 0;
      int chunk;
      const int off = block_scan(n, chunk, sm);
      if (n && run + off < lim) collide_item(m, d, wid, it, run + off, nullptr, lim, fbox);
      run += chunk;
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// constraint.py make_constraint (joint / flex equality, friction, limits, pyramidal contacts)
// ---------------------------------------------------------------------------------------------
__device__ void put_row_scalars(const mjw_model_t& m, const mjw_data_t& d, int wid, int r, float vel, float pos_aref, float pos_imp,
                                float invweight, const float* solref, const float* solimp, float margin, float frictionloss, int type,
                                int id);

// constraint.py:52-121 _efc_row (scalars) + the sparse J row
__device__ void put_row(const mjw_model_t& m, const mjw_data_t& d, int wid, int r, int nnz, const int* cols, const float* vals, float pos_aref,
                        float pos_imp, float invweight, const float* solref, const float* solimp, float margin, float frictionloss, int type,
                        int id) {
  const float* qvel = d.qvel + (long)wid * m.nv;
  const long jb = (long)wid * m.njrow * d.njmax_pad + r, P = d.njmax_pad;
  float vel = 0.0f;
  for (int k = 0; k < nnz; k++) {
    d.efc_J[jb + k * P] = vals[k];
    d.efc_J_colind[jb + k * P] = cols[k];
    vel += vals[k] * qvel[cols[k]];
  }
  d.efc_J_rownnz[(long)wid * d.njmax + r] = nnz;
  put_row_scalars(m, d, wid, r, vel, pos_aref, pos_imp, invweight, solref, solimp, margin, frictionloss, type, id);
}

// constraint.py:52-121 _efc_row: the row scalars for a J row already written (its J qvel in vel)
__device__ void put_row_scalars(const mjw_model_t& m, const mjw_data_t& d, int wid, int r, float vel, float pos_aref, float pos_imp,
                                float invweight, const float* solref, const float* solimp, float margin, float frictionloss, int type,
                                int id) {
  const float timestep = MR(opt_timestep)[0];
  float timeconst = solref[0], dampratio = solref[1];
  float dmin = solimp[0], dmax = solimp[1], width = solimp[2], mid = solimp[3], power = solimp[4];
  if (!(m.opt_disableflags & DSBL_REFSAFE)) timeconst = fmaxf(timeconst, 2.0f * timestep);
  dmin = clampf(dmin, MJW_MINIMP, MJW_MAXIMP);
  dmax = clampf(dmax, MJW_MINIMP, MJW_MAXIMP);
  width = fmaxf(MJW_MINVAL, width);
  mid = clampf(mid, MJW_MINIMP, MJW_MAXIMP);
  power = fmaxf(1.0f, power);
  const float dmax_sq = dmax * dmax;
  float k = 1.0f / (dmax_sq * timeconst * timeconst * dampratio * dampratio);
  float b = 2.0f / (dmax * timeconst);
  if (solref[0] <= 0.0f) k = -solref[0] / dmax_sq;
  if (solref[1] <= 0.0f) b = -solref[1] / dmax;
  const float imp_x = fabsf(pos_imp) / width;
  float imp = dmin + imp_shape(imp_x, mid, power) * (dmax - dmin);
  imp = clampf(imp, dmin, dmax);
  if (imp_x > 1.0f) imp = dmax;
  const long gr = (long)wid * d.njmax + r;
  d.efc_D[(long)wid * d.njmax_pad + r] = 1.0f / fmaxf(invweight * (1.0f - imp) / imp, MJW_MINVAL);
  d.efc_vel[gr] = vel;
  d.efc_aref[gr] = -k * imp * pos_aref - b * vel;
  d.efc_pos[gr] = pos_aref + margin;
  d.efc_margin[gr] = margin;
  d.efc_frictionloss[gr] = frictionloss;
  d.efc_type[gr] = type;
  d.efc_id[gr] = id;
}

// constraint.py:124-365 (_equality_connect) and :792-1110 (_equality_weld), equality e: 3 (6) rows from
// r0 on, J over the union of the two bodies' dof chains (descending, as the contact rows), one thread
__device__ void eq_connect_weld_rows(const mjw_model_t& m, const mjw_data_t& d, int wid, int e, int r0, bool weld) {
  const float* data = MR(eq_data) + 11 * e;
  const int o1 = m.eq_obj1id[e], o2 = m.eq_obj2id[e];
  const bool site = m.eq_objtype[e] == OBJ_SITE && m.nsite > 0;
  const long wb = (long)wid * m.nbody;
  const float* xpos = d.xpos + wb * 3;
  const float* xquat = d.xquat + wb * 4;
  const float* xmat = d.xmat + wb * 9;
  int b1, b2;
  float p1[3], p2[3], q[4] = {1, 0, 0, 0}, q1[4] = {1, 0, 0, 0};
  if (site) {
    const float* site_quat = MR(site_quat);
    const float* sx = d.site_xpos + (long)wid * m.nsite * 3;
    b1 = m.site_bodyid[o1];
    b2 = m.site_bodyid[o2];
    for (int k = 0; k < 3; k++) { p1[k] = sx[3 * o1 + k]; p2[k] = sx[3 * o2 + k]; }
    if (weld) {
      float t[4];
      mul_quat(q, xquat + 4 * b1, site_quat + 4 * o1);
      mul_quat(t, xquat + 4 * b2, site_quat + 4 * o2);
      q1[0] = t[0]; q1[1] = -t[1]; q1[2] = -t[2]; q1[3] = -t[3];
    }
  } else {
    b1 = o1;
    b2 = o2;
    const float* a1 = weld ? data + 3 : data;  // the weld reads its anchors swapped (constraint.py:855-856)
    const float* a2 = weld ? data : data + 3;
    matvec3(p1, xmat + 9 * b1, a1);
    matvec3(p2, xmat + 9 * b2, a2);
    for (int k = 0; k < 3; k++) { p1[k] += xpos[3 * b1 + k]; p2[k] += xpos[3 * b2 + k]; }
    if (weld) {
      mul_quat(q, xquat + 4 * b1, data + 6);
      q1[0] = xquat[4 * b2]; q1[1] = -xquat[4 * b2 + 1]; q1[2] = -xquat[4 * b2 + 2]; q1[3] = -xquat[4 * b2 + 3];
    }
  }
  const float ts = data[10];
  const int nrow = weld ? 6 : 3;
  const float* sc = d.subtree_com + wb * 3;
  const float* cdof = d.cdof + (long)wid * m.nv * 6;
  const float* qvel = d.qvel + (long)wid * m.nv;
  float off1[3], off2[3];
  for (int x = 0; x < 3; x++) {
    off1[x] = p1[x] - sc[3 * m.body_rootid[b1] + x];
    off2[x] = p2[x] - sc[3 * m.body_rootid[b2] + x];
  }
  const int w1 = m.body_weldid[b1], w2 = m.body_weldid[b2];
  const long P = d.njmax_pad;
  float jq[6] = {0, 0, 0, 0, 0, 0};
  int i1 = w1 > 0 ? m.body_dofadr[w1] + m.body_dofnum[w1] - 1 : -1;
  int i2 = w2 > 0 ? m.body_dofadr[w2] + m.body_dofnum[w2] - 1 : -1;
  int nnz = 0;
  while ((i1 >= 0 || i2 >= 0) && nnz < m.njrow) {
    const int dof = max(i1, i2);
    const float* c = cdof + 6 * dof;
    float v[6] = {0, 0, 0, 0, 0, 0}, dr[3] = {0, 0, 0}, cr[3];
    if (dof == i1) {
      cross3(cr, c, off1);
      for (int x = 0; x < 3; x++) { v[x] += c[3 + x] + cr[x]; dr[x] += c[x]; }
      i1 = m.dof_parentid[i1];
    }
    if (dof == i2) {
      cross3(cr, c, off2);
      for (int x = 0; x < 3; x++) { v[x] -= c[3 + x] + cr[x]; dr[x] -= c[x]; }
      i2 = m.dof_parentid[i2];
    }
    if (weld) {
      float t[4], u[4];
      for (int x = 0; x < 3; x++) dr[x] *= ts;
      quat_mul_axis(t, q1, dr);
      mul_quat(u, t, q);
      for (int x = 0; x < 3; x++) v[3 + x] = 0.5f * u[1 + x];
    }
    for (int k = 0; k < nrow; k++) {
      if (r0 + k >= d.njmax) break;
      const long jb = (long)wid * m.njrow * P + r0 + k;
      d.efc_J[jb + nnz * P] = v[k];
      d.efc_J_colind[jb + nnz * P] = dof;
      jq[k] += v[k] * qvel[dof];
    }
    nnz++;
  }
  float cpos[6], pos_imp;
  for (int k = 0; k < 3; k++) cpos[k] = p1[k] - p2[k];
  if (weld) {
    float cq[4];
    mul_quat(cq, q1, q);
    for (int k = 0; k < 3; k++) cpos[3 + k] = cq[1 + k] * ts;
    pos_imp = sqrtf(dot3(cpos, cpos) + dot3(cpos + 3, cpos + 3));
  } else {
    pos_imp = sqrtf(dot3(cpos, cpos));
  }
  const float* biw = MR(body_invweight0);
  for (int k = 0; k < nrow && r0 + k < d.njmax; k++) {
    const int cc = k < 3 ? 0 : 1;
    d.efc_J_rownnz[(long)wid * d.njmax + r0 + k] = nnz;
    put_row_scalars(m, d, wid, r0 + k, jq[k], cpos[k], pos_imp, biw[2 * b1 + cc] + biw[2 * b2 + cc], MR(eq_solref) + 2 * e,
                    MR(eq_solimp) + 5 * e, 0.0f, 0.0f, CNSTR_EQUALITY, e);
  }
}

// constraint.py:1940-2207 (_contact_elliptic): contact i's condim rows from r0 on -- row dimid projects
// the relative Jacobian on frame row dimid (translational below 3, rotational after); the friction rows
// scale invweight by impratio^-1 and (fri0 / frii)^2, use solreffriction when set, and have no position
// term.  J over the union of the two weld bodies' dof chains, as the pyramidal rows.
__device__ void contact_elliptic_rows(const mjw_model_t& m, const mjw_data_t& d, int wid, int i, int r0, int condim, float pos,
                                      float includemargin) {
  const int g1 = d.contact_geom[2 * (long)i], g2 = d.contact_geom[2 * (long)i + 1];
  const int body1 = g1 >= 0 ? m.geom_bodyid[g1] : m.flex_vertbodyid[m.flex_vertadr[d.contact_flex[2 * (long)i]] + d.contact_vert[2 * (long)i]];
  const int body2 =
    g2 >= 0 ? m.geom_bodyid[g2] : m.flex_vertbodyid[m.flex_vertadr[d.contact_flex[2 * (long)i + 1]] + d.contact_vert[2 * (long)i + 1]];
  const float* biw = MR(body_invweight0);
  const float iw_base = biw[2 * body1] + biw[2 * body2];
  const int w1 = m.body_weldid[body1], w2 = m.body_weldid[body2];
  const float* frame = d.contact_frame + 9 * (long)i;
  const float* cpos = d.contact_pos + 3 * (long)i;
  const float* sc = d.subtree_com + (long)wid * m.nbody * 3;
  const float* cdof = d.cdof + (long)wid * m.nv * 6;
  const float* qvel = d.qvel + (long)wid * m.nv;
  const float* fr = d.contact_friction + 5 * (long)i;
  const float iri = MR(opt_impratio_invsqrt)[0];
  float off1[3], off2[3];
  for (int x = 0; x < 3; x++) {
    off1[x] = cpos[x] - sc[3 * m.body_rootid[w1] + x];
    off2[x] = cpos[x] - sc[3 * m.body_rootid[w2] + x];
  }
  const long P = d.njmax_pad;
  for (int dimid = 0; dimid < condim; dimid++) {
    const int r = r0 + dimid;
    if (r >= d.njmax) {
      d.contact_efc_address[(long)i * m.nmaxpyramid + dimid] = -1;
      continue;
    }
    d.contact_efc_address[(long)i * m.nmaxpyramid + dimid] = r;
    const long jb = (long)wid * m.njrow * P + r;
    int i1 = w1 > 0 ? m.body_dofadr[w1] + m.body_dofnum[w1] - 1 : -1;
    int i2 = w2 > 0 ? m.body_dofadr[w2] + m.body_dofnum[w2] - 1 : -1;
    int nnz = 0;
    float vel = 0.0f;
    const float* fv = frame + 3 * (dimid < 3 ? dimid : dimid - 3);
    while ((i1 >= 0 || i2 >= 0) && nnz < m.njrow) {
      const int dof = max(i1, i2);
      const float* c = cdof + 6 * dof;
      float jd[3] = {0, 0, 0}, cr[3];
      if (dof == i1) {
        if (dimid < 3) {
          cross3(cr, c, off1);
          for (int x = 0; x < 3; x++) jd[x] -= c[3 + x] + cr[x];
        } else {
          for (int x = 0; x < 3; x++) jd[x] -= c[x];
        }
        i1 = m.dof_parentid[i1];
      }
      if (dof == i2) {
        if (dimid < 3) {
          cross3(cr, c, off2);
          for (int x = 0; x < 3; x++) jd[x] += c[3 + x] + cr[x];
        } else {
          for (int x = 0; x < 3; x++) jd[x] += c[x];
        }
        i2 = m.dof_parentid[i2];
      }
      const float Jval = fv[0] * jd[0] + fv[1] * jd[1] + fv[2] * jd[2];
      d.efc_J[jb + nnz * P] = Jval;
      d.efc_J_colind[jb + nnz * P] = dof;
      vel += Jval * qvel[dof];
      nnz++;
    }
    d.efc_J_rownnz[(long)wid * d.njmax + r] = nnz;
    float invw = iw_base, pos_aref = pos;
    const float* sr = d.contact_solref + 2 * (long)i;
    if (dimid > 0) {
      const float* srf = d.contact_solreffriction + 2 * (long)i;
      if (srf[0] != 0.0f || srf[1] != 0.0f) sr = srf;
      invw = invw * iri * iri;
      if (dimid > 1) {
        const float fri0 = fr[0], frii = fr[dimid - 1];
        invw *= fri0 * fri0 / (frii * frii);
      }
      pos_aref = 0.0f;
    }
    put_row_scalars(m, d, wid, r, vel, pos_aref, pos, invw, sr, d.contact_solimp + 5 * (long)i, includemargin, 0.0f, CNSTR_CONTACT_ELLIPTIC, i);
  }
}

// rows contributed by item i of a category (cat: 0 eq joint, 1 flex edge of eq e, 2 friction dof,
// 3 limit joint, 4 contact, 5-7 tendon equality / friction / limit, 8 eq connect, 9 eq weld, 10 ball
// joint limit); writes them from row r0 when r0 >= 0
__device__ int make_rows(const mjw_model_t& m, const mjw_data_t& d, int wid, int cat, int i, int e, int r0) {
  const float* qpos = d.qpos + (long)wid * m.nq;
  const float* qpos0 = MR(qpos0);
  const float* dof_invweight0 = MR(dof_invweight0);
  const int njmax = d.njmax;
  if (cat == 8 || cat == 9) {
    if (m.eq_type[i] != (cat == 9 ? EQ_WELD : EQ_CONNECT) || !d.eq_active[(long)wid * m.neq + i]) return 0;
    const int nrow = cat == 9 ? 6 : 3;
    if (r0 < 0) return nrow;
    if (r0 < njmax) eq_connect_weld_rows(m, d, wid, i, r0, cat == 9);
    return nrow;
  }
  if (cat == 10) {  // constraint.py:1421-1543: one row on the ball joint's 3 dofs along -axis
    if (!m.jnt_limited[i] || m.jnt_type[i] != JNT_BALL) return 0;
    const float* qp = qpos + m.jnt_qposadr[i];
    float q[4] = {qp[0], qp[1], qp[2], qp[3]}, aa[3], axis[3];
    normalize4(q);
    quat_to_vel(aa, q);
    const float angle = sqrtf(dot3(aa, aa));  // math.py:261-265 normalize_with_norm
    for (int k = 0; k < 3; k++) axis[k] = angle == 0.0f ? aa[k] : aa[k] / angle;
    const float* rng = MR(jnt_range) + 2 * i;
    const float margin = MR(jnt_margin)[i];
    const float pos = fmaxf(rng[0], rng[1]) - angle - margin;
    if (!(pos < 0.0f)) return 0;
    if (r0 < 0 || r0 >= njmax) return 1;
    const int da = m.jnt_dofadr[i];
    const int cols[3] = {da + 2, da + 1, da};  // descending, as the chain rows
    const float vals[3] = {-axis[2], -axis[1], -axis[0]};
    put_row(m, d, wid, r0, 3, cols, vals, pos, pos, dof_invweight0[da], MR(jnt_solref) + 2 * i, MR(jnt_solimp) + 5 * i, margin, 0.0f,
            CNSTR_LIMIT_JOINT, i);
    return 1;
  }
  if (cat == 0) {
    if (m.eq_type[i] != EQ_JOINT || !d.eq_active[(long)wid * m.neq + i]) return 0;
    if (r0 < 0 || r0 >= njmax) return 1;
    const int j1 = m.eq_obj1id[i], j2 = m.eq_obj2id[i];
    const float* data = MR(eq_data) + 11 * i;
    const int da1 = m.jnt_dofadr[j1], qa1 = m.jnt_qposadr[j1];
    int cols[2] = {da1, 0};
    float vals[2] = {1.0f, 0.0f}, pos, iw;
    int nnz = 1;
    if (j2 > -1) {
      const int qa2 = m.jnt_qposadr[j2], da2 = m.jnt_dofadr[j2];
      const float dif = qpos[qa2] - qpos0[qa2];
      const float rhs = data[0] + dif * (data[1] + dif * (data[2] + dif * (data[3] + dif * data[4])));
      const float deriv_2 = data[1] + dif * (2.0f * data[2] + dif * (3.0f * data[3] + dif * 4.0f * data[4]));
      pos = qpos[qa1] - qpos0[qa1] - rhs;
      iw = dof_invweight0[da1] + dof_invweight0[da2];
      cols[1] = da2;
      vals[1] = -deriv_2;
      nnz = 2;
    } else {
      pos = qpos[qa1] - qpos0[qa1] - data[0];
      iw = dof_invweight0[da1];
    }
    put_row(m, d, wid, r0, nnz, cols, vals, pos, pos, iw, MR(eq_solref) + 2 * i, MR(eq_solimp) + 5 * i, 0.0f, 0.0f, CNSTR_EQUALITY, i);
    return 1;
  }
  if (cat == 1) {  // constraint.py:677-790, edge i of the flex of equality e
    if (r0 < 0 || r0 >= njmax) return 1;
    const int f = m.eq_obj1id[e];
    const int v[2] = {m.flex_vertadr[f] + m.flex_edge[2 * i], m.flex_vertadr[f] + m.flex_edge[2 * i + 1]};
    int cols[6];
    float vals[6];
    int nnz = 0;
    for (int s2 = 0; s2 < 2; s2++) {
      const int b = m.flex_vertbodyid[v[s2]];
      for (int k = 0; k < m.body_dofnum[b] && nnz < 6; k++) {
        cols[nnz] = m.body_dofadr[b] + k;
        vals[nnz] = d.flexedge_J[((long)wid * m.nflexedge + i) * 6 + nnz];
        nnz++;
      }
    }
    const float pos = d.flexedge_length[(long)wid * m.nflexedge + i] - MR(flexedge_length0)[i];
    put_row(m, d, wid, r0, nnz, cols, vals, pos, pos, MR(flexedge_invweight0)[i], MR(eq_solref) + 2 * e, MR(eq_solimp) + 5 * e, 0.0f, 0.0f,
            CNSTR_EQUALITY, e);
    return 1;
  }
  if (cat == 2) {  // constraint.py:1113-1190
    const float fl = MR(dof_frictionloss)[i];
    if (fl <= 0.0f) return 0;
    if (r0 < 0 || r0 >= njmax) return 1;
    const float one = 1.0f;
    put_row(m, d, wid, r0, 1, &i, &one, 0.0f, 0.0f, dof_invweight0[i], MR(dof_solref) + 2 * i, MR(dof_solimp) + 5 * i, 0.0f, fl,
            CNSTR_FRICTION_DOF, i);
    return 1;
  }
  if (cat == 3) {  // constraint.py:1316-1418
    const int jt = m.jnt_type[i];
    if (!m.jnt_limited[i] || !(jt == JNT_SLIDE || jt == JNT_HINGE)) return 0;
    const float* rng = MR(jnt_range) + 2 * i;
    const float q = qpos[m.jnt_qposadr[i]];
    const float dmn = q - rng[0], dmx = rng[1] - q;
    const float margin = MR(jnt_margin)[i];
    const float pos = fminf(dmn, dmx) - margin;
    if (!(pos < 0.0f)) return 0;
    if (r0 < 0 || r0 >= njmax) return 1;
    const int da = m.jnt_dofadr[i];
    const float Jv = (float)(dmn < dmx) * 2.0f - 1.0f;
    put_row(m, d, wid, r0, 1, &da, &Jv, pos, pos, dof_invweight0[da], MR(jnt_solref) + 2 * i, MR(jnt_solimp) + 5 * i, margin, 0.0f,
            CNSTR_LIMIT_JOINT, i);
    return 1;
  }
  if (cat >= 5) {  // tendon rows: 5 equality (constraint.py:498-674), 6 friction (:1204-1313), 7 limit (:1547-1665)
    const float* qv = d.qvel + (long)wid * m.nv;
    const float* tiw = MR(tendon_invweight0);
    int t1 = i, t2 = -1;
    float pos = 0.0f, deriv = 0.0f, scl = 1.0f, margin = 0.0f, fl = 0.0f, iw;
    const float *sref, *simp;
    int type;
    if (cat == 5) {
      if (m.eq_type[i] != EQ_TENDON || !d.eq_active[(long)wid * m.neq + i]) return 0;
      if (r0 < 0 || r0 >= njmax) return 1;
      const float* data = MR(eq_data) + 11 * i;
      const float* len0 = MR(tendon_length0);
      t1 = m.eq_obj1id[i];
      t2 = m.eq_obj2id[i];
      pos = ten_len(m, d, wid, qpos, t1) - len0[t1];
      iw = tiw[t1];
      if (t2 > -1) {
        iw += tiw[t2];
        const float dif = ten_len(m, d, wid, qpos, t2) - len0[t2];
        pos -= data[0] + data[1] * dif + data[2] * dif * dif + data[3] * dif * dif * dif + data[4] * dif * dif * dif * dif;
        deriv = data[1] + 2.0f * data[2] * dif + 3.0f * data[3] * dif * dif + 4.0f * data[4] * dif * dif * dif;
      } else {
        pos -= data[0];
      }
      if (deriv == 0.0f) t2 = -1;
      sref = MR(eq_solref) + 2 * i;
      simp = MR(eq_solimp) + 5 * i;
      type = CNSTR_EQUALITY;
    } else if (cat == 6) {
      fl = MR(tendon_frictionloss)[i];
      if (fl <= 0.0f) return 0;
      if (r0 < 0 || r0 >= njmax) return 1;
      iw = tiw[i];
      sref = MR(tendon_solref_fri) + 2 * i;
      simp = MR(tendon_solimp_fri) + 5 * i;
      type = CNSTR_FRICTION_TENDON;
    } else {
      if (!m.tendon_limited[i]) return 0;
      const float* rng = MR(tendon_range) + 2 * i;
      const float L = ten_len(m, d, wid, qpos, i);
      const float dmn = L - rng[0], dmx = rng[1] - L;
      margin = MR(tendon_margin)[i];
      pos = fminf(dmn, dmx) - margin;
      if (!(pos < 0.0f)) return 0;
      if (r0 < 0 || r0 >= njmax) return 1;
      scl = (float)(dmn < dmx) * 2.0f - 1.0f;
      iw = tiw[i];
      sref = MR(tendon_solref_lim) + 2 * i;
      simp = MR(tendon_solimp_lim) + 5 * i;
      type = CNSTR_LIMIT_TENDON;
    }
    // J = scl J1 - deriv J2 over the merged (ascending) columns of the two tendon rows
    const long jb = (long)wid * m.njrow * d.njmax_pad + r0, P = d.njmax_pad;
    const int n1 = m.ten_J_rownnz[t1], a1 = m.ten_J_rowadr[t1];
    const int n2 = t2 >= 0 ? m.ten_J_rownnz[t2] : 0, a2 = t2 >= 0 ? m.ten_J_rowadr[t2] : 0;
    const float* J1 = d.ten_J + (long)wid * m.nJten + a1;
    const float* J2 = d.ten_J + (long)wid * m.nJten + a2;
    int p1 = 0, p2 = 0, nnz = 0;
    float vel = 0.0f;
    while ((p1 < n1 || p2 < n2) && nnz < m.njrow) {
      const int c1 = p1 < n1 ? m.ten_J_colind[a1 + p1] : 0x7fffffff, c2 = p2 < n2 ? m.ten_J_colind[a2 + p2] : 0x7fffffff;
      const int col = min(c1, c2);
      float v = 0.0f;
      if (c1 == col) v += scl * J1[p1++];
      if (c2 == col) v -= deriv * J2[p2++];
      d.efc_J[jb + nnz * P] = v;
      d.efc_J_colind[jb + nnz * P] = col;
      vel += v * qv[col];
      nnz++;
    }
    d.efc_J_rownnz[(long)wid * njmax + r0] = nnz;
    put_row_scalars(m, d, wid, r0, vel, pos, pos, iw, sref, simp, margin, fl, type, i);
    return 1;
  }
  // cat 4: contact pyramidal (constraint.py:1668-1936); i = pool slot; contacts a contactfilter took the
  // CONSTRAINT bit from get no rows (constraint.py:1731)
  if (!(d.contact_type[i] & 1)) {
    if (r0 < 0)  // the counting pass visits every contact once
      for (int k = 0; k < m.nmaxpyramid; k++) d.contact_efc_address[(long)i * m.nmaxpyramid + k] = -1;
    return 0;
  }
  const int condim = d.contact_dim[i];
  const bool ell = m.opt_cone == CONE_ELLIPTIC && condim > 1;
  const int nrow = condim == 1 ? 1 : (ell ? condim : 2 * (condim - 1));
  const float includemargin = d.contact_includemargin[i];
  const float pos = d.contact_dist[i] - includemargin;
  if (!(pos < 0.0f)) return 0;
  if (r0 < 0) return nrow;
  if (ell) {
    contact_elliptic_rows(m, d, wid, i, r0, condim, pos, includemargin);
    return nrow;
  }
  const int g1 = d.contact_geom[2 * (long)i], g2 = d.contact_geom[2 * (long)i + 1];
  const int body1 = g1 >= 0 ? m.geom_bodyid[g1] : m.flex_vertbodyid[m.flex_vertadr[d.contact_flex[2 * (long)i]] + d.contact_vert[2 * (long)i]];
  const int body2 =
    g2 >= 0 ? m.geom_bodyid[g2] : m.flex_vertbodyid[m.flex_vertadr[d.contact_flex[2 * (long)i + 1]] + d.contact_vert[2 * (long)i + 1]];
  const float* biw = MR(body_invweight0);
  const float iw_base = biw[2 * body1] + biw[2 * body2];
  const int w1 = m.body_weldid[body1], w2 = m.body_weldid[body2];
  const float* frame = d.contact_frame + 9 * (long)i;
  const float* cpos = d.contact_pos + 3 * (long)i;
  const float* sc = d.subtree_com + (long)wid * m.nbody * 3;
  const float* cdof = d.cdof + (long)wid * m.nv * 6;
  float off1[3], off2[3];
  for (int x = 0; x < 3; x++) {
    off1[x] = cpos[x] - sc[3 * m.body_rootid[w1] + x];
    off2[x] = cpos[x] - sc[3 * m.body_rootid[w2] + x];
  }
  const float* fr = d.contact_friction + 5 * (long)i;
  const float iri = MR(opt_impratio_invsqrt)[0];
  for (int dimid = 0; dimid < nrow; dimid++) {
    const int r = r0 + dimid;
    if (r >= njmax) {
      d.contact_efc_address[(long)i * m.nmaxpyramid + dimid] = -1;
      continue;
    }
    d.contact_efc_address[(long)i * m.nmaxpyramid + dimid] = r;
    float invweight = iw_base, frii = 0.0f;
    const int dimid2 = dimid / 2 + 1;
    if (condim > 1) {
      const float fri0 = fr[0];
      frii = fr[dimid2 - 1];
      invweight = invweight + fri0 * fri0 * invweight;
      invweight = invweight * 2.0f * fri0 * fri0 * iri * iri;
    }
    // union of the two weld bodies' dof chains, descending
    const long jb = (long)wid * m.njrow * d.njmax_pad + r, P = d.njmax_pad;
    int i1 = w1 > 0 ? m.body_dofadr[w1] + m.body_dofnum[w1] - 1 : -1;
    int i2 = w2 > 0 ? m.body_dofadr[w2] + m.body_dofnum[w2] - 1 : -1;
    int nnz = 0;
    float vel = 0.0f;
    const float* qvel = d.qvel + (long)wid * m.nv;
    while ((i1 >= 0 || i2 >= 0) && nnz < m.njrow) {
      const int dof = max(i1, i2);
      const bool in1 = dof == i1, in2 = dof == i2;
      const float* c = cdof + 6 * dof;
      float j1p[3] = {0, 0, 0}, j2p[3] = {0, 0, 0}, j1r[3] = {0, 0, 0}, j2r[3] = {0, 0, 0}, cr[3];
      if (in1) {
        cross3(cr, c, off1);
        for (int x = 0; x < 3; x++) { j1p[x] = c[3 + x] + cr[x]; j1r[x] = c[x]; }
        i1 = m.dof_parentid[i1];
      }
      if (in2) {
        cross3(cr, c, off2);
        for (int x = 0; x < 3; x++) { j2p[x] = c[3 + x] + cr[x]; j2r[x] = c[x]; }
        i2 = m.dof_parentid[i2];
      }
      float Jval = 0.0f, Ji = 0.0f;
      for (int x = 0; x < 3; x++) {
        const float jd = j2p[x] - j1p[x];
        Jval += frame[x] * jd;
        if (condim > 1) {
          if (dimid2 < 3) Ji += frame[3 * dimid2 + x] * jd;
          else Ji += frame[3 * (dimid2 - 3) + x] * (j2r[x] - j1r[x]);
        }
      }
      if (condim > 1) Jval += (dimid % 2 == 0) ? Ji * frii : -Ji * frii;
      d.efc_J[jb + nnz * P] = Jval;
      d.efc_J_colind[jb + nnz * P] = dof;
      vel += Jval * qvel[dof];
      nnz++;
    }
    d.efc_J_rownnz[(long)wid * njmax + r] = nnz;
    const int type = condim == 1 ? CNSTR_CONTACT_FRICTIONLESS : CNSTR_CONTACT_PYRAMIDAL;
    const float* sr = d.contact_solref + 2 * (long)i;
    const float* si = d.contact_solimp + 5 * (long)i;
    // same scalar math as put_row, keeping the J row written above
    const float timestep = MR(opt_timestep)[0];
    float timeconst = sr[0], dampratio = sr[1];
    float dmin = si[0], dmax = si[1], width = si[2], mid = si[3], power = si[4];
    if (!(m.opt_disableflags & DSBL_REFSAFE)) timeconst = fmaxf(timeconst, 2.0f * timestep);
    dmin = clampf(dmin, MJW_MINIMP, MJW_MAXIMP);
    dmax = clampf(dmax, MJW_MINIMP, MJW_MAXIMP);
    width = fmaxf(MJW_MINVAL, width);
    mid = clampf(mid, MJW_MINIMP, MJW_MAXIMP);
    power = fmaxf(1.0f, power);
    const float dmax_sq = dmax * dmax;
    float kk = 1.0f / (dmax_sq * timeconst * timeconst * dampratio * dampratio);
    float bb = 2.0f / (dmax * timeconst);
    if (sr[0] <= 0.0f) kk = -sr[0] / dmax_sq;
    if (sr[1] <= 0.0f) bb = -sr[1] / dmax;
    const float imp_x = fabsf(pos) / width;
    float imp = dmin + imp_shape(imp_x, mid, power) * (dmax - dmin);
    imp = clampf(imp, dmin, dmax);
    if (imp_x > 1.0f) imp = dmax;
    const long gr = (long)wid * njmax + r;
    d.efc_D[(long)wid * d.njmax_pad + r] = 1.0f / fmaxf(invweight * (1.0f - imp) / imp, MJW_MINVAL);
    d.efc_vel[gr] = vel;
    d.efc_aref[gr] = -kk * imp * pos - bb * vel;
    d.efc_pos[gr] = pos + includemargin;
    d.efc_margin[gr] = includemargin;
    d.efc_frictionloss[gr] = 0.0f;
    d.efc_type[gr] = type;
    d.efc_id[gr] = i;
  }
  return nrow;
}

__device__ void make_constraint(const mjw_model_t& m, const mjw_data_t& d, int wid, Smem& sm) {
  int run = 0, ne = 0, nf = 0, nl = 0;
  const int dsbl = m.opt_disableflags;
  if (!(dsbl & DSBL_CONSTRAINT)) {
    const int ncon_base = d.ncon_world[2 * (long)wid], ncon = d.ncon_world[2 * (long)wid + 1];
    // the reference's row order (constraint.py:2209-2779 launch order): equality (connect, weld, joint,
    // tendon, flex), friction (dof, tendon), limits (ball, slide / hinge, tendon), contacts
    const int order[11] = {8, 9, 0, 5, 1, 2, 6, 10, 3, 7, 4};
    for (int oi = 0; oi < 11; oi++) {
      const int cat = order[oi];
      const bool eq = cat <= 1 || cat == 5 || cat == 8 || cat == 9, lim = cat == 3 || cat == 7 || cat == 10;
      if (eq && (dsbl & DSBL_EQUALITY)) continue;
      if ((cat == 2 || cat == 6) && (dsbl & DSBL_FRICTIONLOSS)) continue;
      if (lim && (dsbl & DSBL_LIMIT)) continue;
      if (cat == 4 && (dsbl & DSBL_CONTACT)) continue;
      if (cat >= 5 && cat <= 7 && m.ntendon == 0) continue;
      if ((cat == 8 || cat == 9) && m.neq_cw == 0) continue;
      if (cat == 10 && m.nlimited_ball == 0) continue;
      const int start = run;
      const int neqs = cat == 1 ? m.neq : 1;
      for (int e = 0; e < neqs; e++) {
        int n_items, i0 = 0;
        if (cat == 0 || cat == 8 || cat == 9) n_items = m.neq;
        else if (cat == 10) n_items = m.njnt;
        else if (cat == 1) {
          if (m.eq_type[e] != EQ_FLEX || !d.eq_active[(long)wid * m.neq + e]) continue;
          const int f = m.eq_obj1id[e];
          i0 = m.flex_edgeadr[f];
          n_items = m.flex_edgenum[f];
        } else if (cat == 2) n_items = m.nv;
        else if (cat == 3) n_items = m.njnt;
        else if (cat == 5) n_items = m.neq;
        else if (cat >= 6) n_items = m.ntendon;
        else {
          i0 = ncon_base;
          n_items = min(ncon, max(d.naconmax - ncon_base, 0));
        }
        for (int c0 = 0; c0 < n_items; c0 += BLK) {
          const int it = c0 + tid();
          const int n = it < n_items ? make_rows(m, d, wid, cat, i0 + it, e, -1) : 0;
          int chunk;
          const int off = block_scan(n, chunk, sm);
          if (n) make_rows(m, d, wid, cat, i0 + it, e, run + off);
          run += chunk;
        }
      }
      if (eq) ne += run - start;
      else if (cat == 2 || cat == 6) nf += run - start;
      else if (lim) nl += run - start;
    }
  }
  if (tid() == 0) {
    d.ne[wid] = ne;
    d.nf[wid] = nf;
    d.nl[wid] = nl;
    d.nefc[wid] = run;
  }
  __syncthreads();
}

// smooth.py:2448-2602: BODY (adhesion) transmissions.  Moment = minus the mean, over the world's
// contacts touching the body (flex contacts excepted), of n . (J(pos, b2) - J(pos, b1)) -- what the
// reference reads back from the contact's constraint rows or, outside the margin, from the Jacobian
// difference (mjw_trn.h).  The block splits the dofs; each thread walks the world's contacts in order.
__device__ void body_transmission(const mjw_model_t& m, const mjw_data_t& d, int wid) {
  const int cbase = d.ncon_world[2 * (long)wid], nc = d.ncon_world[2 * (long)wid + 1];
  const float* sc = d.subtree_com + (long)wid * m.nbody * 3;
  const float* cdof = d.cdof + (long)wid * m.nv * 6;
  for (int a = 0; a < m.nu; a++) {
    if (m.actuator_trntype[a] != TRN_BODY) continue;
    const int body = m.actuator_trnid[2 * a];
    int ncon = 0;
    for (int c = cbase; c < cbase + nc; c++) {
      const int g1 = d.contact_geom[2 * (long)c], g2 = d.contact_geom[2 * (long)c + 1];
      if (g1 >= 0 && g2 >= 0 && (m.geom_bodyid[g1] == body || m.geom_bodyid[g2] == body)) ncon++;
    }
    const long gu = (long)wid * m.nu + a;
    float* gm = d.actuator_moment + (long)wid * m.nJmom + d.moment_rowadr[gu];
    int* gc = d.moment_colind + (long)wid * m.nJmom + d.moment_rowadr[gu];
    for (int i = tid(); i < m.nv; i += BLK) {
      float q = 0.0f;
      for (int c = cbase; c < cbase + nc && ncon > 0; c++) {
        const int g1 = d.contact_geom[2 * (long)c], g2 = d.contact_geom[2 * (long)c + 1];
        if (g1 < 0 || g2 < 0) continue;
        const int b1 = m.geom_bodyid[g1], b2 = m.geom_bodyid[g2];
        if (b1 != body && b2 != body) continue;
        const float* pos = d.contact_pos + 3 * (long)c;
        const float* n = d.contact_frame + 9 * (long)c;
        float j1[3], j2[3], r[3];
        trn_jac_dof(m, sc, cdof, pos, b1, i, j1, r);
        trn_jac_dof(m, sc, cdof, pos, b2, i, j2, r);
        q += n[0] * (j2[0] - j1[0]) + n[1] * (j2[1] - j1[1]) + n[2] * (j2[2] - j1[2]);
      }
      gm[i] = ncon > 0 ? q * (-1.0f / (float)ncon) : 0.0f;
      gc[i] = i;
    }
  }
  __syncthreads();
}

// smooth.py:2041-2147 joint transmissions (packed moment rows, actuator order)
__device__ void transmission(const mjw_model_t& m, const mjw_data_t& d, int wid, Smem& sm) {
  const float* gear_all = MR(actuator_gear);
  const float* qpos = d.qpos + (long)wid * m.nq;
  int carry = 0;
  for (int a0 = 0; a0 < m.nu; a0 += BLK) {
    const int a = a0 + tid();
    int nnz = 0;
    if (a < m.nu) {
      if (m.actuator_trntype[a] == TRN_TENDON) {
        nnz = m.ten_J_rownnz[m.actuator_trnid[2 * a]];
      } else if (m.actuator_trntype[a] == TRN_SITE || m.actuator_trntype[a] == TRN_SLIDERCRANK || m.actuator_trntype[a] == TRN_BODY) {
        nnz = trn_site_nnz(m, a);
      } else {
        const int jt0 = m.jnt_type[m.actuator_trnid[2 * a]];
        nnz = jt0 == JNT_FREE ? 6 : (jt0 == JNT_BALL ? 3 : 1);
      }
    }
    int chunk;
    const int rowadr = carry + block_scan(nnz, chunk, sm);
    carry += chunk;
    if (a >= m.nu) continue;
    const float* gear = gear_all + 6 * a;
    const int trn = m.actuator_trntype[a], j = m.actuator_trnid[2 * a];
    if (trn == TRN_TENDON) {  // smooth.py:2242-2259: length = ten_length gear0, moment row = gear0 ten_J
      const long gu = (long)wid * m.nu + a;
      const float* J = d.ten_J + (long)wid * m.nJten + m.ten_J_rowadr[j];
      d.actuator_length[gu] = ten_len(m, d, wid, qpos, j) * gear[0];
      d.moment_rownnz[gu] = nnz;
      d.moment_rowadr[gu] = rowadr;
      for (int k = 0; k < nnz; k++) {
        d.actuator_moment[(long)wid * m.nJmom + rowadr + k] = gear[0] * J[k];
        d.moment_colind[(long)wid * m.nJmom + rowadr + k] = m.ten_J_colind[m.ten_J_rowadr[j] + k];
      }
      continue;
    }
    if (trn == TRN_BODY) {  // a dense row over every dof, filled below once all rows are placed
      const long gu = (long)wid * m.nu + a;
      d.actuator_length[gu] = 0.0f;
      d.moment_rownnz[gu] = nnz;
      d.moment_rowadr[gu] = rowadr;
      continue;
    }
    if (trn == TRN_SITE || trn == TRN_SLIDERCRANK) {  // smooth.py:2150-2241, 2274-2442 (mjw_trn.h)
      const long gu = (long)wid * m.nu + a;
      float* gm = d.actuator_moment + (long)wid * m.nJmom + rowadr;
      int* gc = d.moment_colind + (long)wid * m.nJmom + rowadr;
      d.actuator_length[gu] = trn_site(m, wid, a, nnz, d.site_xpos + (long)wid * m.nsite * 3, d.site_xmat + (long)wid * m.nsite * 9,
                                       d.xquat + (long)wid * m.nbody * 4, d.subtree_com + (long)wid * m.nbody * 3,
                                       d.cdof + (long)wid * m.nv * 6, gm, gc, gm, gc);
      d.moment_rownnz[gu] = nnz;
      d.moment_rowadr[gu] = rowadr;
      continue;
    }
    const int jt = m.jnt_type[j], qa = m.jnt_qposadr[j], va = m.jnt_dofadr[j];
    float mom[6] = {0, 0, 0, 0, 0, 0}, length;
    if (jt == JNT_FREE) {
      length = 0.0f;
      if (trn == 1) {
        float q[4] = {qpos[qa + 3], qpos[qa + 4], qpos[qa + 5], qpos[qa + 6]}, ga[3];
        normalize4(q);
        float qn[4] = {q[0], -q[1], -q[2], -q[3]};
        rot_vec_quat(ga, gear + 3, qn);
        for (int i = 0; i < 3; i++) { mom[i] = gear[i]; mom[3 + i] = ga[i]; }
      } else {
        for (int i = 0; i < 6; i++) mom[i] = gear[i];
      }
    } else if (jt == JNT_BALL) {
      float q[4] = {qpos[qa], qpos[qa + 1], qpos[qa + 2], qpos[qa + 3]}, aa[3];
      normalize4(q);
      quat_to_vel(aa, q);
      float ga[3] = {gear[0], gear[1], gear[2]};
      if (trn == 1) {
        float qn[4] = {q[0], -q[1], -q[2], -q[3]};
        rot_vec_quat(ga, ga, qn);
      }
      length = dot3(aa, ga);
      for (int i = 0; i < 3; i++) mom[i] = ga[i];
    } else {
      length = qpos[qa] * gear[0];
      mom[0] = gear[0];
    }
    const long gu = (long)wid * m.nu + a;
    d.actuator_length[gu] = length;
    d.moment_rownnz[gu] = nnz;
    d.moment_rowadr[gu] = rowadr;
    for (int k = 0; k < nnz; k++) {
      d.actuator_moment[(long)wid * m.nJmom + rowadr + k] = mom[k];
      d.moment_colind[(long)wid * m.nJmom + rowadr + k] = va + k;
    }
  }
  __syncthreads();
  if (m.nbodytrn) body_transmission(m, d, wid);
}

// ---------------------------------------------------------------------------------------------
// velocity: actuator velocity, com_vel (smooth.py:1935-2038), passive (passive.py:70-179, 566-725),
// rne (smooth.py:1112-1274)
// ---------------------------------------------------------------------------------------------
__device__ void fwd_velocity(const mjw_model_t& m, const mjw_data_t& d, int wid) {
  const int nb = m.nbody, nv = m.nv;
  const float* qvel = d.qvel + (long)wid * nv;
  const float* cdof = d.cdof + (long)wid * nv * 6;
  for (int a = tid(); a < m.nu; a += BLK) {
    const long gu = (long)wid * m.nu + a;
    float v = 0.0f;
    for (int k = 0; k < d.moment_rownnz[gu]; k++) {
      const long p = (long)wid * m.nJmom + d.moment_rowadr[gu] + k;
      v += d.actuator_moment[p] * qvel[d.moment_colind[p]];
    }
    d.actuator_velocity[gu] = v;
  }
  // com_vel: cvel of the parent = sum over the ancestors' dofs; then this body's joints in order
  float* cvel_all = d.cvel + (long)wid * nb * 6;
  float* cdot = d.cdof_dot + (long)wid * nv * 6;
  for (int b = tid(); b < nb; b += BLK) {
    float cv[6] = {0, 0, 0, 0, 0, 0};
    for (int p = m.body_parentid[b]; p > 0; p = m.body_parentid[p])
      for (int k = 0; k < m.body_dofnum[p]; k++) {
        const int dof = m.body_dofadr[p] + k;
        for (int i = 0; i < 6; i++) cv[i] += cdof[6 * dof + i] * qvel[dof];
      }
    if (b > 0) {
      int dof = m.body_dofadr[b];
      for (int j = m.body_jntadr[b]; j < m.body_jntadr[b] + m.body_jntnum[b]; j++) {
        const int jt = m.jnt_type[j];
        if (jt == JNT_FREE) {
          for (int k = 0; k < 3; k++) {
            for (int i = 0; i < 6; i++) { cv[i] += cdof[6 * (dof + k) + i] * qvel[dof + k]; cdot[6 * (dof + k) + i] = 0.0f; }
          }
          for (int k = 3; k < 6; k++) motion_cross(cdot + 6 * (dof + k), cv, cdof + 6 * (dof + k));
          for (int k = 3; k < 6; k++)
            for (int i = 0; i < 6; i++) cv[i] += cdof[6 * (dof + k) + i] * qvel[dof + k];
          dof += 6;
        } else if (jt == JNT_BALL) {
          for (int k = 0; k < 3; k++) motion_cross(cdot + 6 * (dof + k), cv, cdof + 6 * (dof + k));
          for (int k = 0; k < 3; k++)
            for (int i = 0; i < 6; i++) cv[i] += cdof[6 * (dof + k) + i] * qvel[dof + k];
          dof += 3;
        } else {
          motion_cross(cdot + 6 * dof, cv, cdof + 6 * dof);
          for (int i = 0; i < 6; i++) cv[i] += cdof[6 * dof + i] * qvel[dof];
          dof += 1;
        }
      }
    }
    for (int i = 0; i < 6; i++) cvel_all[6 * b + i] = cv[i];
  }
  // passive: joint springs / dampers
  const int dsbl_spring = m.opt_disableflags & DSBL_SPRING, dsbl_damper = m.opt_disableflags & DSBL_DAMPER;
  float* qs = d.qfrc_spring + (long)wid * nv;
  float* qd = d.qfrc_damper + (long)wid * nv;
  const float* qpos = d.qpos + (long)wid * m.nq;
  const float* stiffness = MR(jnt_stiffness);
  const float* damping = MR(dof_damping);
  const float* qpos_spring = MR(qpos_spring);
  for (int j = tid(); j < m.njnt; j += BLK) {
    const int da = m.jnt_dofadr[j], qa = m.jnt_qposadr[j], jt = m.jnt_type[j];
    const int nd = jt == JNT_FREE ? 6 : (jt == JNT_BALL ? 3 : 1);
    for (int k = 0; k < nd; k++) qs[da + k] = qd[da + k] = 0.0f;
    if (dsbl_spring && dsbl_damper) continue;
    const float stiff = stiffness[j], damp = damping[da];
    const bool has_s = stiff != 0.0f && !dsbl_spring, has_d = damp != 0.0f && !dsbl_damper;
    if (jt == JNT_FREE) {
      if (has_s) {
        for (int i = 0; i < 3; i++) qs[da + i] = -stiff * (qpos[qa + i] - qpos_spring[qa + i]);
        float rot[4] = {qpos[qa + 3], qpos[qa + 4], qpos[qa + 5], qpos[qa + 6]}, dif[3];
        normalize4(rot);
        quat_sub(dif, rot, qpos_spring + qa + 3);
        for (int i = 0; i < 3; i++) qs[da + 3 + i] = -stiff * dif[i];
      }
      if (has_d) for (int i = 0; i < 6; i++) qd[da + i] = -damp * qvel[da + i];
    } else if (jt == JNT_BALL) {
      if (has_s) {
        float rot[4] = {qpos[qa], qpos[qa + 1], qpos[qa + 2], qpos[qa + 3]}, dif[3];
        normalize4(rot);
        quat_sub(dif, rot, qpos_spring + qa);
        for (int i = 0; i < 3; i++) qs[da + i] = -stiff * dif[i];
      }
      if (has_d) for (int i = 0; i < 3; i++) qd[da + i] = -damp * qvel[da + i];
    } else {
      if (has_s) qs[da] = -stiff * (qpos[qa] - qpos_spring[qa]);
      if (has_d) qd[da] = -damp * qvel[da];
    }
  }
  // flex elasticity (per element) and bending (per edge) into scratch, gathered per vertex below
  float* frc = d.flex_frc + (long)wid * (m.nflexelem * 12 + m.nflexedge * 12);
  const float* fx = d.flexvert_xpos + (long)wid * m.nflexvert * 3;
  if (!(dsbl_spring && dsbl_damper) && !dsbl_spring) {
    const float dt = MR(opt_timestep)[0];
    const float* stiff = MR(flex_stiffness);
    // the local edges of a segment / triangle / tetrahedron (passive.py:606-613)
    const int le[4][6][2] = {{{0, 0}}, {{0, 1}}, {{1, 2}, {2, 0}, {0, 1}}, {{0, 1}, {1, 2}, {2, 0}, {2, 3}, {0, 3}, {1, 3}}};
    for (int f = 0; f < m.nflex; f++) {
      const int dim = m.flex_dim[f], nve = dim + 1, ne = dim == 1 ? 1 : (dim == 2 ? 3 : 6);
      const float kD = (dt > 0.0f && !dsbl_damper) ? MR(flex_damping)[f] / dt : 0.0f;
      const int vb = m.flex_vertadr[f];
      for (int el = tid(); el < m.flex_elemnum[f]; el += BLK) {
        const int elemid = m.flex_elemadr[f] + el;
        const int* ev = m.flex_elem + m.flex_elemdataadr[f] + nve * el;
        float grad[6][6], elong[6], force[4][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
        for (int e = 0; e < ne; e++) {
          const float* x0 = fx + 3 * (vb + ev[le[dim][e][0]]);
          const float* x1 = fx + 3 * (vb + ev[le[dim][e][1]]);
          for (int i = 0; i < 3; i++) { grad[e][i] = x0[i] - x1[i]; grad[e][3 + i] = x1[i] - x0[i]; }
          const int idx = m.flex_edgeadr[f] + m.flex_elemedge[m.flex_elemedgeadr[f] + ne * el + e];
          const float vel = d.flexedge_velocity[(long)wid * m.nflexedge + idx];
          const float def = d.flexedge_length[(long)wid * m.nflexedge + idx], ref = MR(flexedge_length0)[idx];
          const float prev = def - vel * dt;
          elong[e] = def * def - ref * ref + (def * def - prev * prev) * kD;
        }
        float metric[6][6];
        int id = 0;
        for (int a = 0; a < ne; a++)
          for (int b = a; b < ne; b++) { metric[a][b] = metric[b][a] = stiff[21 * elemid + id]; id++; }
        for (int a = 0; a < ne; a++)
          for (int b = 0; b < ne; b++)
            for (int s2 = 0; s2 < 2; s2++)
              for (int x = 0; x < 3; x++) force[le[dim][b][s2]][x] -= elong[a] * grad[b][3 * s2 + x] * metric[a][b];
        for (int k = 0; k < nve; k++)
          for (int x = 0; x < 3; x++) frc[12 * elemid + 3 * k + x] = force[k][x];
      }
      for (int e = m.flex_edgeadr[f] + tid(); e < m.flex_edgeadr[f] + m.flex_edgenum[f]; e += BLK) {
        float* out = frc + 12 * m.nflexelem + 12 * e;
        if (m.flex_edgeflap[2 * e + 1] == -1) {
          for (int k = 0; k < 12; k++) out[k] = 0.0f;
          continue;
        }
        const int v[4] = {vb + m.flex_edge[2 * e], vb + m.flex_edge[2 * e + 1], vb + m.flex_edgeflap[2 * e], vb + m.flex_edgeflap[2 * e + 1]};
        const float* B = MR(flex_bending) + 17 * e;
        float fr4[4][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
        if (B[16] != 0.0f) {
          float a1[3], a2[3], a3[3];
          for (int i = 0; i < 3; i++) {
            a1[i] = fx[3 * v[1] + i] - fx[3 * v[0] + i];
            a2[i] = fx[3 * v[2] + i] - fx[3 * v[0] + i];
            a3[i] = fx[3 * v[3] + i] - fx[3 * v[0] + i];
          }
          cross3(fr4[1], a2, a3);
          cross3(fr4[2], a3, a1);
          cross3(fr4[3], a1, a2);
          for (int i = 0; i < 3; i++) fr4[0][i] = -(fr4[1][i] + fr4[2][i] + fr4[3][i]);
        }
        for (int i = 0; i < 4; i++)
          for (int x = 0; x < 3; x++) {
            float s = 0.0f;
            for (int j = 0; j < 4; j++) s -= B[4 * i + j] * fx[3 * v[j] + x];
            out[3 * i + x] = s - B[16] * fr4[i][x];
          }
      }
    }
  }
  __syncthreads();
  // per-vertex gather in a fixed order (flexvert_inc: encoded contributions)
  if (!(dsbl_spring && dsbl_damper) && !dsbl_spring) {
    for (int v = tid(); v < m.nflexvert; v += BLK) {
      const int b = m.flex_vertbodyid[v];
      if (m.body_dofnum[b] == 0) continue;
      float s[3] = {0.0f, 0.0f, 0.0f};
      for (int p = m.flexvert_incadr[v]; p < m.flexvert_incadr[v + 1]; p++) {
        const int code = m.flexvert_inc[p];  // 4*elem + k (element vertex slot) or 4*nflexelem + 4*edge + k
        const float* src = code < 4 * m.nflexelem ? frc + 3 * code : frc + 12 * m.nflexelem + 3 * (code - 4 * m.nflexelem);
        for (int x = 0; x < 3; x++) s[x] += src[x];
      }
      for (int x = 0; x < 3; x++) qs[m.body_dofadr[b] + x] += s[x];
    }
  }
  __syncthreads();
  // passive.py:183-252: tendon velocity, spring (dead band between lengthspring[0] and [1]) and damper; one
  // tendon per round (rows may share dofs), threads over its Jacobian row
  if (m.ntendon) {
    __syncthreads();
    const float* tst = MR(tendon_stiffness);
    const float* tdp = MR(tendon_damping);
    const float* tls = MR(tendon_lengthspring);
    for (int t = tid(); t < m.ntendon; t += BLK) d.ten_velocity[(long)wid * m.ntendon + t] = ten_vel(m, d, wid, qvel, t);
    for (int t = 0; t < m.ntendon; t++) {
      const bool hs = tst[t] != 0.0f && !dsbl_spring, hd = tdp[t] != 0.0f && !dsbl_damper;
      if (!hs && !hd) continue;
      const float L = ten_len(m, d, wid, qpos, t), v = ten_vel(m, d, wid, qvel, t);
      const float lo = tls[2 * t], hi = tls[2 * t + 1];
      const float fs = L > hi ? tst[t] * (hi - L) : (L < lo ? tst[t] * (lo - L) : 0.0f);
      const float fd = -tdp[t] * v;
      const float* J = d.ten_J + (long)wid * m.nJten + m.ten_J_rowadr[t];
      for (int k = tid(); k < m.ten_J_rownnz[t]; k += BLK) {
        const int dof = m.ten_J_colind[m.ten_J_rowadr[t] + k];
        if (hs) qs[dof] += J[k] * fs;
        if (hd) qd[dof] += J[k] * fd;
      }
      __syncthreads();
    }
  }
  // passive.py:829-869: gravity compensation and fluid forces (mjw_passive.h), per-body wrenches in the
  // sp_body / cacc scratch (rne fills both afterwards), then per dof over its body's subtree
  float* qp = d.qfrc_passive + (long)wid * nv;
  float* qg = d.qfrc_gravcomp + (long)wid * nv;
  float* qf = d.qfrc_fluid + (long)wid * nv;
  const bool gc_on = m.ngravcomp && !(m.opt_disableflags & DSBL_GRAVITY) && !(dsbl_spring && dsbl_damper);
  const bool fl_on = m.has_fluid && !(dsbl_spring && dsbl_damper);
  if (gc_on || fl_on) {
    float* Wg = d.sp_body + (long)wid * nb * 6;
    float* Wf = d.cacc + (long)wid * nb * 6;
    const float* xipos = d.xipos + (long)wid * nb * 3;
    const float* ximat = d.ximat + (long)wid * nb * 9;
    const float* sc = d.subtree_com + (long)wid * nb * 3;
    const float* gxpos = d.geom_xpos + (long)wid * m.ngeom * 3;
    const float* gxmat = d.geom_xmat + (long)wid * m.ngeom * 9;
    const float zero3[3] = {0.0f, 0.0f, 0.0f};
    for (int b = tid(); b < nb; b += BLK) {
      const float* sr = sc + 3 * m.body_rootid[b];
      float f[3], t[3];
      if (gc_on) {
        gravcomp_force(m, wid, b, f);
        body_wrench(Wg + 6 * b, f, zero3, xipos + 3 * b, sr);
      }
      if (fl_on) {
        fluid_force(m, wid, b, xipos + 3 * b, ximat + 9 * b, cvel_all + 6 * b, sr, gxpos, gxmat, f, t);
        body_wrench(Wf + 6 * b, f, t, xipos + 3 * b, sr);
      }
    }
    __syncthreads();
    for (int i = tid(); i < nv; i += BLK) {
      const float* cd = cdof + 6 * i;
      const int db = m.dof_bodyid[i], end = m.body_subtree_end[db];
      float g = 0.0f, fl = 0.0f;
      for (int b = db; b < end; b++) {
        if (gc_on) g += cd[0] * Wg[6 * b] + cd[1] * Wg[6 * b + 1] + cd[2] * Wg[6 * b + 2] + cd[3] * Wg[6 * b + 3] + cd[4] * Wg[6 * b + 4] + cd[5] * Wg[6 * b + 5];
        if (fl_on) fl += cd[0] * Wf[6 * b] + cd[1] * Wf[6 * b + 1] + cd[2] * Wf[6 * b + 2] + cd[3] * Wf[6 * b + 3] + cd[4] * Wf[6 * b + 4] + cd[5] * Wf[6 * b + 5];
      }
      qg[i] = g;
      qf[i] = fl;
    }
  } else {
    for (int i = tid(); i < nv; i += BLK) qg[i] = qf[i] = 0.0f;
  }
  __syncthreads();
  // passive.py:555-561: gravcomp unless routed to the actuators (forward.py:824-826), then the fluid force
  for (int i = tid(); i < nv; i += BLK) {
    float p = qs[i] + qd[i];
    if (gc_on && !m.jnt_actgravcomp[m.dof_jntid[i]]) p += qg[i];
    if (fl_on) p += qf[i];
    qp[i] = p;
  }
  // rne: cacc by ancestor walk, body forces into scratch, subtree sums, projection on cdof
  float* cacc = d.cacc + (long)wid * nb * 6;
  float* body_f = d.sp_body + (long)wid * nb * 6;
  const float* cinert = d.cinert + (long)wid * nb * 10;
  const float* grav = MR(opt_gravity);
  const bool gravity = !(m.opt_disableflags & DSBL_GRAVITY);
  for (int b = tid(); b < nb; b += BLK) {
    float acc[6] = {0, 0, 0, 0, 0, 0};
    if (gravity) for (int i = 0; i < 3; i++) acc[3 + i] = -grav[i];
    for (int p = b; p > 0; p = m.body_parentid[p])
      for (int k = 0; k < m.body_dofnum[p]; k++) {
        const int dof = m.body_dofadr[p] + k;
        for (int i = 0; i < 6; i++) acc[i] += cdot[6 * dof + i] * qvel[dof];
      }
    for (int i = 0; i < 6; i++) cacc[6 * b + i] = acc[i];
    if (b == 0) {
      for (int i = 0; i < 6; i++) body_f[i] = 0.0f;
      continue;
    }
    float f1[6], iv[6], f2[6];
    inert_vec(f1, cinert + 10 * b, acc);
    inert_vec(iv, cinert + 10 * b, cvel_all + 6 * b);
    motion_cross_force(f2, cvel_all + 6 * b, iv);
    for (int i = 0; i < 6; i++) body_f[6 * b + i] = f1[i] + f2[i];
  }
  __syncthreads();
  float* cfrc = d.cfrc_int + (long)wid * nb * 6;
  for (int b = tid(); b < nb; b += BLK) {
    float s[6] = {0, 0, 0, 0, 0, 0};
    for (int c = b; c < m.body_subtree_end[b]; c++)
      for (int i = 0; i < 6; i++) s[i] += body_f[6 * c + i];
    for (int i = 0; i < 6; i++) cfrc[6 * b + i] = s[i];
  }
  __syncthreads();
  float* bias = d.qfrc_bias + (long)wid * nv;
  for (int i = tid(); i < nv; i += BLK) {
    const float* c = cfrc + 6 * m.dof_bodyid[i];
    float s = 0.0f;
    for (int k = 0; k < 6; k++) s += cdof[6 * i + k] * c[k];
    bias[i] = s;
  }
  __syncthreads();
  // smooth.py:1878-1932 tendon_bias: armature J (Jdot qvel) of the spatial tendons, BLK tendons per round
  if (m.nten_spatial) {
    __shared__ float coef[BLK];
    const TenFrames f = ten_frames(m, d, wid);
    for (int base = 0; base < m.ntendon; base += BLK) {
      const int t = base + tid();
      coef[tid()] = t < m.ntendon ? tendon_bias_coef(m, wid, t, qvel, f, cvel_all, cdot) : 0.0f;
      __syncthreads();
      for (int q = 0; q < BLK && base + q < m.ntendon; q++) {
        if (coef[q] == 0.0f) continue;
        const int tq = base + q, ra = m.ten_J_rowadr[tq];
        for (int k = tid(); k < m.ten_J_rownnz[tq]; k += BLK)
          bias[m.ten_J_colind[ra + k]] += coef[q] * d.ten_J[(long)wid * m.nJten + ra + k];
        __syncthreads();
      }
    }
  }
}

// forward.py:616-927 actuation (gain / bias / activation dynamics, joint actuator force limits)
__device__ void fwd_actuation(const mjw_model_t& m, const mjw_data_t& d, int wid) {
  const int nv = m.nv;
  float* qa = d.qfrc_actuator + (long)wid * nv;
  if (!m.nu || (m.opt_disableflags & DSBL_ACTUATION)) {
    for (int i = tid(); i < nv; i += BLK) qa[i] = 0.0f;
    for (int a = tid(); a < m.na; a += BLK) d.act_dot[(long)wid * m.na + a] = 0.0f;
    __syncthreads();
    return;
  }
  const float* ctrlrange = MR(actuator_ctrlrange);
  const float* forcerange = MR(actuator_forcerange);
  const float* gainprm = MR(actuator_gainprm);
  const float* biasprm = MR(actuator_biasprm);
  const float* dynprm = MR(actuator_dynprm);
  for (int a = tid(); a < m.nu; a += BLK) {
    float ctrl = d.ctrl[(long)wid * m.nu + a];
    if (m.actuator_ctrllimited[a] && !(m.opt_disableflags & DSBL_CLAMPCTRL)) ctrl = clampf(ctrl, ctrlrange[2 * a], ctrlrange[2 * a + 1]);
    float ctrl_act = ctrl;
    const int act_first = m.actuator_actadr[a];
    if (m.na && act_first >= 0) {
      const int last = act_first + m.actuator_actnum[a] - 1, dt = m.actuator_dyntype[a];
      const float act = d.act[(long)wid * m.na + last];
      float act_dot = 0.0f;
      if (dt == DYN_INTEGRATOR) act_dot = ctrl;
      else if (dt == DYN_FILTER || dt == DYN_FILTEREXACT) act_dot = (ctrl - act) / fmaxf(dynprm[10 * a], MJW_MINVAL);
      else if (dt == DYN_MUSCLE) act_dot = muscle_dynamics(ctrl, act, dynprm + 10 * a);
      d.act_dot[(long)wid * m.na + last] = act_dot;
      ctrl_act = m.actuator_actearly[a]
                   ? next_act(MR(opt_timestep)[0], dt, dynprm[10 * a], MR(actuator_actrange) + 2 * a, act, act_dot, 1.0f, m.actuator_actlimited[a] != 0)
                   : act;
    }
    const long gu = (long)wid * m.nu + a;
    const float len = d.actuator_length[gu], vel = d.actuator_velocity[gu];
    const float *gp = gainprm + 10 * a, *bp = biasprm + 10 * a;
    float gain = 0.0f, bias = 0.0f;
    if (m.actuator_gaintype[a] == GAIN_FIXED) gain = gp[0];
    else if (m.actuator_gaintype[a] == GAIN_AFFINE) gain = gp[0] + gp[1] * len + gp[2] * vel;
    if (m.actuator_biastype[a] == BIAS_AFFINE) bias = bp[0] + bp[1] * len + bp[2] * vel;
    if (m.actuator_gaintype[a] == GAIN_MUSCLE) gain = muscle_gain(len, vel, MR(actuator_lengthrange) + 2 * a, MR(actuator_acc0)[a], gp);
    if (m.actuator_biastype[a] == BIAS_MUSCLE) bias = muscle_bias(len, MR(actuator_lengthrange) + 2 * a, MR(actuator_acc0)[a], bp);
    float force = gain * ctrl_act + bias;
    if (m.actuator_forcelimited[a]) force = clampf(force, forcerange[2 * a], forcerange[2 * a + 1]);
    d.actuator_force[gu] = force;
  }
  __syncthreads();
  // forward.py:739-779: the total force of the actuators on a force-limited tendon scaled into its range
  if (m.ntendon) {
    const float* rng = MR(tendon_actfrcrange);
    float* force = d.actuator_force + (long)wid * m.nu;
    for (int t = tid(); t < m.ntendon; t += BLK) {
      if (!m.tendon_actfrclimited[t]) continue;
      float tot = 0.0f;
      for (int a = 0; a < m.nu; a++)
        if (m.actuator_trntype[a] == TRN_TENDON && m.actuator_trnid[2 * a] == t) tot += force[a];
      const float sc = tot < rng[2 * t] ? rng[2 * t] / tot : (tot > rng[2 * t + 1] ? rng[2 * t + 1] / tot : 1.0f);
      if (sc != 1.0f)
        for (int a = 0; a < m.nu; a++)
          if (m.actuator_trntype[a] == TRN_TENDON && m.actuator_trnid[2 * a] == t) force[a] *= sc;
    }
    __syncthreads();
  }
  const float* jfr = MR(jnt_actfrcrange);
  for (int i = tid(); i < nv; i += BLK) {
    float q = 0.0f;
    for (int a = 0; a < m.nu; a++) {
      const long gu = (long)wid * m.nu + a;
      const int adr = d.moment_rowadr[gu];
      for (int k = 0; k < d.moment_rownnz[gu]; k++)
        if (d.moment_colind[(long)wid * m.nJmom + adr + k] == i) q += d.actuator_moment[(long)wid * m.nJmom + adr + k] * d.actuator_force[gu];
    }
    const int j = m.dof_jntid[i];
    if (m.ngravcomp && m.jnt_actgravcomp[j]) q += d.qfrc_gravcomp[(long)wid * nv + i];  // forward.py:824-826
    if (m.jnt_actfrclimited[j]) q = clampf(q, jfr[2 * j], jfr[2 * j + 1]);
    qa[i] = q;
  }
  __syncthreads();
}

// forward.py:930-969 + support.py:174-237 (xfrc over the dof's subtree) + tree factor / solve
__device__ void fwd_acceleration(const mjw_model_t& m, const mjw_data_t& d, int wid) {
  const int nv = m.nv;
  const float* cdof = d.cdof + (long)wid * nv * 6;
  const float* xfrc = d.xfrc_applied + (long)wid * m.nbody * 6;
  const float* xipos = d.xipos + (long)wid * m.nbody * 3;
  const float* sc = d.subtree_com + (long)wid * m.nbody * 3;
  float* qs = d.qfrc_smooth + (long)wid * nv;
  float* qacc_s = d.qacc_smooth + (long)wid * nv;
  for (int i = tid(); i < nv; i += BLK) {
    float v = d.qfrc_passive[(long)wid * nv + i] - d.qfrc_bias[(long)wid * nv + i] + d.qfrc_actuator[(long)wid * nv + i] +
              d.qfrc_applied[(long)wid * nv + i];
    const float* cd = cdof + 6 * i;
    const int db = m.dof_bodyid[i];
    for (int b = db; b < m.body_subtree_end[db]; b++) {
      const float* ft = xfrc + 6 * b;
      if (ft[0] == 0.0f && ft[1] == 0.0f && ft[2] == 0.0f && ft[3] == 0.0f && ft[4] == 0.0f && ft[5] == 0.0f) continue;
      float off[3], c[3];
      for (int k = 0; k < 3; k++) off[k] = xipos[3 * b + k] - sc[3 * m.body_rootid[b] + k];
      cross3(c, cd, off);
      v += cd[3] * ft[0] + cd[4] * ft[1] + cd[5] * ft[2] + cd[0] * ft[3] + cd[1] * ft[4] + cd[2] * ft[5] + dot3(c, ft);
    }
    qs[i] = v;
    qacc_s[i] = v;
  }
  factor_trees(m, d.qM + (long)wid * m.nM, d.qLD + (long)wid * m.nM, nullptr, 0.0f);
  __syncthreads();
  solve_trees(m, d.qLD + (long)wid * m.nM, qacc_s);
  __syncthreads();
}

// The forward stages as separate kernels (one instantiation per group): every stage already keeps
// its state in HBM, so splitting costs a launch, while one fused kernel took the register maximum of
// all stages (248 VGPRs, 3.4 KB scratch per lane, 2 waves / SIMD).  POS_A: frames to qM; COLL:
// collision; CON: constraint rows + transmission; the convex pre-pass runs between POS_A and COLL.
enum : int { SP_POS_A = 1 << 8, SP_POS_B = 1 << 9, SP_COLL = 1 << 10, SP_CON = 1 << 11 };
// mjw_kernel_name (mjw_step.hip) spells these launches with the numeric template arguments
static_assert(SP_POS_A == 256 && SP_COLL == 1024 && SP_CON == 2048 && ST_VEL == 2, "kernel names");

template <int S>
__global__ void __launch_bounds__(BLK, 4) forward_kernel(const mjw_model_t m, const mjw_data_t d, int stages) {
  __shared__ Smem sm;
  const int wid = blockIdx.x;
  SPROF_T0();
  if constexpr ((S & SP_POS_A) != 0) {
    kinematics(m, d, wid);
    com_pos(m, d, wid, sm);
    camlight(m, d, wid);
    SPROF_MARK(SPH_KIN);
    flex_edges(m, d, wid);
    SPROF_MARK(SPH_FLEX);
    crb_qM(m, d, wid);
    if (m.ntendon) tendons(m, d, wid);
    SPROF_MARK(SPH_CRB);
  }
  if constexpr ((S & SP_COLL) != 0) {
    collision(m, d, wid, sm);
    SPROF_MARK(SPH_COLL);
  }
  if constexpr ((S & SP_CON) != 0) {
    make_constraint(m, d, wid, sm);
    transmission(m, d, wid, sm);
    SPROF_MARK(SPH_CON);
  }
  if constexpr ((S & ST_VEL) != 0) {
    if (stages & ST_VEL) fwd_velocity(m, d, wid);
    SPROF_MARK(SPH_VEL);
    if (stages & ST_ACT) fwd_actuation(m, d, wid);
    SPROF_MARK(SPH_ACT);
    if (stages & ST_ACC) fwd_acceleration(m, d, wid);
    SPROF_MARK(SPH_ACC);
  }
}

// convex pre-pass (collision_convex.py:701-890): one wave per world applies the broadphase to the
// convex pairs 64 at a time, then runs GJK / EPA (mjw_ccd.h) on each survivor with the whole wave in
// lockstep over an LDS workspace; mesh supports are wave-parallel vertex scans.  Results go to
// d.ccd_out, which collide_item reads for the same (broadphase-passing) pairs.
template <bool HF>  // HF: with the heightfield pairs (see the dense pre-pass)
__device__ __forceinline__ void ccd_body(const mjw_model_t& m, const mjw_data_t& d) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wid = blockIdx.x, lane = (int)threadIdx.x;
  const CcdLay CL = ccd_layout(m.ccd_epa_iterations, HF && m.nhfield > 0, m.nmaxpolygon, m.nmaxmeshdeg);
  float* W = smem;
  int* list = reinterpret_cast<int*>(smem + CL.total);
  const MeshPoly MP = mesh_poly(m);
  const float* gx = d.geom_xpos + (long)wid * m.ngeom * 3;
  const float* gm = d.geom_xmat + (long)wid * m.ngeom * 9;
  const float* gsize = MR(geom_size);
  const float* gmargin = MR(geom_margin);
  const float* mesh_vert = MR(mesh_vert);
  for (int p0 = 0; p0 < m.nxn; p0 += 64) {
    const int p = p0 + lane;
    bool pass = false;
    if (p < m.nxn && m.nxn_ccdid[p] >= 0)
      pass = m.nxn_pairid[2 * p + 1] >= 0 || broadphase(m, wid, gx, gm, m.nxn_geom_pair[2 * p], m.nxn_geom_pair[2 * p + 1]);
    const unsigned long long bal = __ballot(pass);
    if (pass) list[__popcll(bal & ((1ull << lane) - 1ull))] = p;
    __syncthreads();
    const int nsurv = __popcll(bal);
    for (int k = 0; k < nsurv; k++) {
      const int q = list[k];
      const int g1 = m.nxn_geom_pair[2 * q], g2 = m.nxn_geom_pair[2 * q + 1];
      const int t1 = m.geom_type[g1], t2 = m.geom_type[g2];
      const int md1 = t1 == GEOM_MESH ? m.geom_dataid[g1] : -1, md2 = t2 == GEOM_MESH ? m.geom_dataid[g2] : -1;
      if (HF && t1 == GEOM_HFIELD) {
        // heightfield-convex pair (collision_convex.py:158-697): the record is built whole in the workspace
        const int hid = m.geom_dataid[g1], pid = m.nxn_pairid[2 * q];
        CcdWS cw;
        cw.W = W;
        cw.L = CL;
        hfield_pair(cw, m.ccd_epa_iterations, MR(opt_ccd_tolerance)[0], m.opt_ccd_iterations, gmargin[g1] + gmargin[g2],
                    pid > -1 ? MR(pair_margin)[pid] : gmargin[g1] + gmargin[g2], gx + 3 * g1, gm + 9 * g1, MR(hfield_size) + 4 * hid,
                    m.hfield_nrow[hid], m.hfield_ncol[hid], MR(hfield_data) + m.hfield_adr[hid], gx + 3 * g2, gm + 9 * g2, gsize + 3 * g2,
                    MR(geom_rbound)[g2], t2, md2 >= 0 ? mesh_vert + 3 * (long)m.mesh_vertadr[md2] : nullptr,
                    md2 >= 0 ? m.mesh_vertnum[md2] : 0, W + CL.out);
        float* out = d.ccd_out + ((long)wid * m.nxn_ccd + m.nxn_ccdid[q]) * CCD_OUT;
        if (lane < CCD_OUT) out[lane] = W[CL.out + lane];
        __syncthreads();
        continue;
      }
      put_cgeom(W + CL.geoms, gx + 3 * g1, gm + 9 * g1, gsize + 3 * g1, t1, md1 >= 0 ? m.mesh_vertadr[md1] : 0, md1 >= 0 ? m.mesh_vertnum[md1] : 0,
                md1);
      put_cgeom(W + CL.geoms + CGEOM_WORDS, gx + 3 * g2, gm + 9 * g2, gsize + 3 * g2, t2, md2 >= 0 ? m.mesh_vertadr[md2] : 0,
                md2 >= 0 ? m.mesh_vertnum[md2] : 0, md2);
      __syncthreads();
      const int pid = m.nxn_pairid[2 * q];  // explicit <pair>: its own margin (collision_core.py:271)
      const int nc = ccd_pair(W, m.ccd_epa_iterations, MR(opt_ccd_tolerance)[0], m.opt_ccd_iterations,
                              pid > -1 ? MR(pair_margin)[pid] : gmargin[g1] + gmargin[g2], mesh_vert, 0.0f, &MP,
                              (m.opt_enableflags & ENBL_MULTICCD) != 0, m.nmaxpolygon, m.nmaxmeshdeg);
      float* out = d.ccd_out + ((long)wid * m.nxn_ccd + m.nxn_ccdid[q]) * CCD_OUT;
      if (lane < CCD_OUT) out[lane] = ccd_record_word(lane, nc, W + CL.out);
      __syncthreads();
    }
  }
}
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) ccd_kernel(const mjw_model_t m, const mjw_data_t d) { ccd_body<false>(m, d); }
__global__ void __launch_bounds__(64) ccd_hf_kernel(const mjw_model_t m, const mjw_data_t d) { ccd_body<true>(m, d); }

// ---------------------------------------------------------------------------------------------
// solver.py CG (primal, pyramidal): init_context :3257-3293, iteration :3187-3254, exact
// iterative linesearch :886-1341, update_constraint :2154-2219, update_gradient :2879-3008
// ---------------------------------------------------------------------------------------------
struct SolveCtx {
  int nv, nefc, ne, nf, njrow, P;
  const float* J;     // slot-major: slot k of row r at J[k * P + r]
  const int* Jcol;
  const unsigned short* Jcol16;  // 16-bit copy of Jcol for the CG passes (solve_kernel<0> writes it)
  const int* Jnnz;
  const int* JT_adr;  // J transposed (CSR by dof): rows JT16[p] (16 bit), values JT_val[p]
  const unsigned short* JT16;
  const float* JT_val;
  const float* D;
  const float* fl;
  const float* aref;
  float* force;
  int* state;
  float *Jaref, *jv;
  float* Dq;   // Newton: D of the rows in the quadratic state, 0 for the others (sp_row's third block)
  float* H;    // Newton: the dense nv x nv Hessian / its Cholesky factor (sp_H), null for CG
  bool newton;
  float *qacc, *Ma, *qfrc_c;
  const float *qfrc_s, *qacc_s;
  float *grad, *Mgrad, *search, *mv, *pgrad, *pMgrad;
  const float *M, *LD;
  float cost, prev_cost, gauss, search_dot, grad_dot;
  int rphase;  // block_sum_db buffer parity (uniform)
  const struct EllCtx* ell;  // elliptic cones (solve_kernel<3> only)
};

// row types / ids, and the contacts' first rows, dims and frictions, for the cone rows
struct EllCtx {
  const int* type;
  const int* id;
  const int* con_adr;  // contact_efc_address (nmaxpyramid per contact)
  const int* con_dim;
  const float* con_fr;
  int nmaxpyr;
  float iri;  // opt.impratio_invsqrt
};

// ---- elliptic cones (solver.py:263-323 _eval_elliptic, 1550-1611 quad, 1886-1942 update) ----------
// the contact of elliptic row r: its first row, dim, friction and mu; false when its rows run past
// njmax (the oracle and the reference then leave the contact out)
struct ConeRow {
  int r0, dim, con;
  float mu;
  const float* fr;
};
__device__ __forceinline__ bool cone_of(const SolveCtx& c, int r, ConeRow& k) {
  const EllCtx& e = *c.ell;
  k.con = e.id[r];
  k.r0 = e.con_adr[(long)k.con * e.nmaxpyr];
  k.dim = e.con_dim[k.con];
  k.fr = e.con_fr + 5 * (long)k.con;
  k.mu = k.fr[0] * e.iri;
  return k.r0 >= 0 && k.r0 + k.dim <= c.nefc;
}

// quad, quad1, quad2 of the contact whose first row is r (solver.py:1550-1611), at the current Jaref / jv
__device__ __forceinline__ void ell_quad(const SolveCtx& c, const ConeRow& k, float* q) {
  const int r = k.r0;
  const float D0 = c.D[r], ja = c.Jaref[r], jv = c.jv[r];
  q[0] = 0.5f * ja * ja * D0; q[1] = jv * ja * D0; q[2] = 0.5f * jv * jv * D0;
  float uu = 0.0f, uv = 0.0f, vv = 0.0f;
  for (int j = 1; j < k.dim; j++) {
    const int rj = r + j;
    const float jaj = c.Jaref[rj], jvj = c.jv[rj], dj = c.D[rj], DJj = dj * jaj;
    q[0] += 0.5f * jaj * DJj; q[1] += jvj * DJj; q[2] += 0.5f * jvj * dj * jvj;
    const float uj = jaj * k.fr[j - 1], vj = jvj * k.fr[j - 1];
    uu += uj * uj; uv += uj * vj; vv += vj * vj;
  }
  q[3] = ja * k.mu; q[4] = jv * k.mu; q[5] = uu;
  q[6] = uv; q[7] = vv; q[8] = D0 / (k.mu * k.mu * (1.0f + k.mu * k.mu));
}

// (cost, grad, hess) of one contact's cone at alpha (solver.py:263-323), added into o
__device__ __forceinline__ void ell_eval(const float* q, float mu, float alpha, float* o) {
  const float u0 = q[3], v0 = q[4], uu = q[5], uv = q[6], vv = q[7], dm = q[8];
  const float N = u0 + alpha * v0;
  const float Tsqr = uu + alpha * (2.0f * uv + alpha * vv);
  bool bottom = false;
  if (Tsqr <= 0.0f) {
    if (!(N < 0.0f)) return;
    bottom = true;
  } else {
    const float T = sqrtf(Tsqr);
    if (N >= mu * T) return;
    if (mu * N + T <= 0.0f) {
      bottom = true;
    } else {
      const float N1 = v0, T1 = (uv + alpha * vv) / T;
      const float T2 = vv / T - (uv + alpha * vv) * T1 / (T * T);
      const float nmt = N - mu * T, d1 = N1 - mu * T1;
      o[0] += 0.5f * dm * nmt * nmt;
      o[1] += dm * nmt * d1;
      o[2] += dm * (d1 * d1 + nmt * (-mu * T2));
      return;
    }
  }
  if (bottom) {
    const float aq2 = alpha * q[2];
    o[0] += alpha * aq2 + alpha * q[1] + q[0];
    o[1] += 2.0f * aq2 + q[1];
    o[2] += 2.0f * q[2];
  }
}

// force / cost / state of elliptic row r at the current Jaref (solver.py:1886-1942); every row of the
// contact must be current
__device__ __forceinline__ float ell_force(const SolveCtx& c, int r, float jaref, float& cost, int& state) {
  ConeRow k;
  cost = 0.0f;
  if (!cone_of(c, r, k)) { state = STATE_SATISFIED; return 0.0f; }
  const float N = c.Jaref[k.r0] * k.mu;
  float TT = 0.0f, uf = 0.0f;
  for (int j = 1; j < k.dim; j++) {
    const float uj = c.Jaref[k.r0 + j] * k.fr[j - 1];
    TT += uj * uj;
    if (k.r0 + j == r) uf = uj * k.fr[j - 1];
  }
  const float T = TT <= 0.0f ? 0.0f : sqrtf(TT);
  const float D = c.D[r];
  if (N >= k.mu * T || (T <= 0.0f && N >= 0.0f)) {
    state = STATE_SATISFIED;
    return 0.0f;
  }
  if (k.mu * N + T <= 0.0f || (T <= 0.0f && N < 0.0f)) {
    state = STATE_QUADRATIC;
    cost = 0.5f * D * jaref * jaref;
    return -D * jaref;
  }
  const float dm = safe_div(c.D[k.r0], k.mu * k.mu * (1.0f + k.mu * k.mu));
  const float nmt = N - k.mu * T;
  const float f0 = -dm * nmt * k.mu;
  state = STATE_CONE;
  if (r == k.r0) {
    cost = 0.5f * dm * nmt * nmt;
    return f0;
  }
  return -safe_div(f0, T) * uf;
}

__device__ __forceinline__ void eval_row_v(const SolveCtx& c, int r, float D, float jaref, float jv, float alpha, float* o) {
  const float x = jaref + alpha * jv;
  if (r >= c.ne + c.nf) {
    if (x < 0.0f) {
      const float jvD = jv * D;
      o[0] += 0.5f * D * x * x;
      o[1] += jvD * x;
      o[2] += jv * jvD;
    }
    return;
  }
  if (r >= c.ne) {
    const float f = c.fl[r], rf = safe_div(f, D);
    if (-rf < x && x < rf) {
      const float jvD = jv * D;
      o[0] += 0.5f * D * x * x;
      o[1] += jvD * x;
      o[2] += jv * jvD;
    } else if (x <= -rf) {
      o[0] += f * (-0.5f * rf - x);
      o[1] += -f * jv;
    } else {
      o[0] += f * (-0.5f * rf + x);
      o[1] += f * jv;
    }
    return;
  }
  const float jvD = jv * D;
  o[0] += 0.5f * D * x * x;
  o[1] += jvD * x;
  o[2] += jv * jvD;
}

__device__ __forceinline__ void eval_row(const SolveCtx& c, int r, float alpha, float* o) {
  eval_row_v(c, r, c.D[r], c.Jaref[r], c.jv[r], alpha, o);
}

// eval_row at NA step sizes over every row (o: NA x 3 sums).  The row passes are latency bound, so
// each thread loads RU rows (r0, r0 + nthr(), ...: the same per-thread order as a plain strided loop,
// hence the same sums) before evaluating any of them.
constexpr int RU = 4;  // 8 and 16 rows in flight per thread measured 14 % and 73 % slower on aloha_cloth, 2 and 1
                       // 3 % and 5 % slower (round 6, profiles/r06_sparse_ab_ru.log)
template <int NA, bool ELL = false>
__device__ __forceinline__ void eval_rows(const SolveCtx& c, const float* alphas, float* o) {
  if (ELL) {
    // elliptic models: contact rows of the cone type are evaluated per contact, at its first row
    for (int r = c.ne + tid(); r < c.nefc; r += nthr()) {
      if (r >= c.ne + c.nf && c.ell->type[r] == CNSTR_CONTACT_ELLIPTIC) {
        ConeRow k;
        if (!cone_of(c, r, k) || k.r0 != r) continue;
        float q[9];
        ell_quad(c, k, q);
#pragma unroll
        for (int a = 0; a < NA; a++) ell_eval(q, k.mu, alphas[a], o + 3 * a);
        continue;
      }
#pragma unroll
      for (int a = 0; a < NA; a++) eval_row(c, r, alphas[a], o + 3 * a);
    }
    return;
  }
  for (int r0 = c.ne + tid(); r0 < c.nefc; r0 += RU * nthr()) {  // equality rows: folded into the quadratic
    float D[RU], ja[RU], jv[RU];
#pragma unroll
    for (int u = 0; u < RU; u++) {
      const int r = r0 + u * nthr();
      const bool ok = r < c.nefc;
      D[u] = ok ? c.D[r] : 0.0f;
      ja[u] = ok ? c.Jaref[r] : 0.0f;
      jv[u] = ok ? c.jv[r] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < RU; u++) {
      const int r = r0 + u * nthr();
      if (r < c.nefc) {
#pragma unroll
        for (int a = 0; a < NA; a++) eval_row_v(c, r, D[u], ja[u], jv[u], alphas[a], o + 3 * a);
      }
    }
  }
}

// `alpha`: the linesearch step still to be applied to Jaref (fused here: Jaref += alpha * jv)
template <bool ELL = false>
__device__ __forceinline__ void update_constraint(SolveCtx& c, Smem& sm, float alpha = 0.0f) {
  SPROF_T0_SUB();
  float cost = 0.0f;
  if (ELL) {
    // a cone row reads its contact's other rows: Jaref is advanced for every row first
    if (alpha != 0.0f) {
      for (int r = tid(); r < c.nefc; r += nthr()) c.Jaref[r] += alpha * c.jv[r];
      __syncthreads();
    }
    for (int r = tid(); r < c.nefc; r += nthr()) {
      const float D = c.D[r], jaref = c.Jaref[r];
      float f;
      if (r < c.ne) {
        f = -D * jaref;
        cost += 0.5f * D * jaref * jaref;
      } else if (r < c.ne + c.nf) {
        const float fl = c.fl[r], rf = safe_div(fl, D);
        if (jaref <= -rf) { f = fl; cost += -fl * (0.5f * rf + jaref); }
        else if (jaref >= rf) { f = -fl; cost += -fl * (0.5f * rf - jaref); }
        else { f = -D * jaref; cost += 0.5f * D * jaref * jaref; }
      } else if (c.ell->type[r] == CNSTR_CONTACT_ELLIPTIC) {
        float rc;
        int st;
        f = ell_force(c, r, jaref, rc, st);
        cost += rc;
      } else {
        if (jaref >= 0.0f) { f = 0.0f; }
        else { f = -D * jaref; cost += 0.5f * D * jaref * jaref; }
      }
      c.force[r] = f;
    }
    alpha = 0.0f;
  }
  for (int r0 = ELL ? c.nefc : tid(); r0 < c.nefc; r0 += RU * nthr()) {
  float Du[RU], jau[RU];
#pragma unroll
  for (int u = 0; u < RU; u++) {
    const int r = r0 + u * nthr();
    const bool ok = r < c.nefc;
    Du[u] = ok ? c.D[r] : 0.0f;
    jau[u] = ok ? c.Jaref[r] : 0.0f;
    if (ok && alpha != 0.0f) jau[u] += alpha * c.jv[r];
  }
#pragma unroll
  for (int u = 0; u < RU; u++) {
    const int r = r0 + u * nthr();
    if (r >= c.nefc) break;
    const float D = Du[u];
    const float jaref = jau[u];
    if (alpha != 0.0f) c.Jaref[r] = jaref;
    float f;
    if (r < c.ne) {
      f = -D * jaref;
      cost += 0.5f * D * jaref * jaref;
    } else if (r < c.ne + c.nf) {
      const float fl = c.fl[r], rf = safe_div(fl, D);
      if (jaref <= -rf) { f = fl; cost += -fl * (0.5f * rf + jaref); }
      else if (jaref >= rf) { f = -fl; cost += -fl * (0.5f * rf - jaref); }
      else { f = -D * jaref; cost += 0.5f * D * jaref * jaref; }
    } else {
      if (jaref >= 0.0f) { f = 0.0f; }
      else { f = -D * jaref; cost += 0.5f * D * jaref * jaref; }
    }
    c.force[r] = f;
  }
  }
  __syncthreads();
  SPROF_MARK_SUB(SPH_S_UCR);
  float g = 0.0f;
  for (int i = tid(); i < c.nv; i += nthr()) {
    float s = 0.0f;
    // 4 entries in flight (index loads, then the dependent force gathers), same summation order
    const int pa = c.JT_adr[i], pb = c.JT_adr[i + 1];
    int p = pa;
    for (; p + 4 <= pb; p += 4) {
      const int r0 = c.JT16[p], r1 = c.JT16[p + 1], r2 = c.JT16[p + 2], r3 = c.JT16[p + 3];
      const float v0 = c.JT_val[p], v1 = c.JT_val[p + 1], v2 = c.JT_val[p + 2], v3 = c.JT_val[p + 3];
      const float f0 = c.force[r0], f1 = c.force[r1], f2 = c.force[r2], f3 = c.force[r3];
      s += v0 * f0;
      s += v1 * f1;
      s += v2 * f2;
      s += v3 * f3;
    }
    for (; p < pb; p++) s += c.JT_val[p] * c.force[c.JT16[p]];
    c.qfrc_c[i] = s;
    g += (c.Ma[i] - c.qfrc_s[i]) * (c.qacc[i] - c.qacc_s[i]);
  }
  float v[2] = {cost, g};
  block_sum_db<2>(v, sm, c.rphase);
  SPROF_MARK_SUB(SPH_S_JTF);
  c.prev_cost = c.cost;
  c.gauss = 0.5f * v[1];
  c.cost = v[0] + 0.5f * v[1];
}

// efc_state of the final Jaref (solver.py:2154-2219), written once after the iterations: the CG itself
// never reads it, so update_constraint does not store it every iteration
template <bool ELL = false>
__device__ void write_states(const SolveCtx& c) {
  for (int r = tid(); r < c.nefc; r += nthr()) {
    const float D = c.D[r], jaref = c.Jaref[r];
    int st = STATE_QUADRATIC;
    if (ELL && r >= c.ne + c.nf && c.ell->type[r] == CNSTR_CONTACT_ELLIPTIC) {
      float rc;
      (void)ell_force(c, r, jaref, rc, st);
    } else if (r >= c.ne && r < c.ne + c.nf) {
      const float fl = c.fl[r], rf = safe_div(fl, D);
      st = jaref <= -rf ? STATE_LINEARNEG : (jaref >= rf ? STATE_LINEARPOS : STATE_QUADRATIC);
    } else if (r >= c.ne + c.nf) {
      st = jaref >= 0.0f ? STATE_SATISFIED : STATE_QUADRATIC;
    }
    c.state[r] = st;
  }
}

// Newton direction (solver.py:2879-3008): H = M + J' diag(D quadratic) J (dense, nv x nv, lower
// triangle, row-major; solver.py:2367-2425 builds the same H for the reference's sparse models),
// factored in place (right-looking Cholesky, one column per round) and solved for Mgrad = H^-1 grad.
// J'DJ entries come from the transposed index: rows common to columns i and j, merged in ascending
// row order -- a fixed summation order, so replicas stay bitwise equal
template <bool ELL = false>
__device__ void newton_direction(const mjw_model_t& m, SolveCtx& c) {
  const int nv = c.nv;
  float* H = c.H;
  for (int r = c.ne + tid(); r < c.nefc; r += nthr()) {  // equality rows are always quadratic
    const float D = c.D[r], ja = c.Jaref[r];
    bool quad = true;
    if (ELL && r >= c.ne + c.nf && c.ell->type[r] == CNSTR_CONTACT_ELLIPTIC) {
      float rc;
      int st;
      (void)ell_force(c, r, ja, rc, st);
      quad = st == STATE_QUADRATIC;
    } else if (r < c.ne + c.nf) {
      const float rf = safe_div(c.fl[r], D);
      quad = -rf < ja && ja < rf;
    } else {
      quad = ja < 0.0f;
    }
    c.Dq[r] = quad ? D : 0.0f;
  }
  for (int r = tid(); r < min(c.ne, c.nefc); r += nthr()) c.Dq[r] = c.D[r];
  __syncthreads();
  for (int i = tid(); i < nv; i += nthr()) {
    const int ai = c.JT_adr[i], bi = c.JT_adr[i + 1];
    for (int j = 0; j <= i; j++) {
      float s = 0.0f;
      int p = ai, q = c.JT_adr[j];
      const int bj = c.JT_adr[j + 1];
      while (p < bi && q < bj) {
        const int rp = c.JT16[p], rq = c.JT16[q];
        if (rp == rq) {
          s += c.Dq[rp] * c.JT_val[p] * c.JT_val[q];
          p++;
          q++;
        } else if (rp < rq) {
          p++;
        } else {
          q++;
        }
      }
      H[i * nv + j] = s;
    }
    if (ELL) {
      // + J_c' C J_c of every contact in the cone state (solver.py:2430-2585), row i of H by this thread:
      // C[a][b] J[ra][i] J[rb][j] over the contact's rows a, b and the columns j <= i of row rb
      for (int r = c.ne + c.nf; r < c.nefc; r++) {
        if (c.ell->type[r] != CNSTR_CONTACT_ELLIPTIC) continue;
        ConeRow k;
        if (!cone_of(c, r, k) || k.r0 != r) continue;
        const float mu2 = k.mu * k.mu;
        const float dm = safe_div(c.D[r], mu2 * (1.0f + mu2));
        float u[6], fri[6], tt = 0.0f;
        u[0] = c.Jaref[r] * k.mu;
        fri[0] = k.mu;
        for (int j = 1; j < k.dim; j++) {
          u[j] = c.Jaref[r + j] * k.fr[j - 1];
          fri[j] = k.fr[j - 1];
          tt += u[j] * u[j];
        }
        const float T = tt <= 0.0f ? 0.0f : sqrtf(tt), N = u[0];
        // the cone state of the contact (ell_force's zones)
        if (N >= k.mu * T || (T <= 0.0f && N >= 0.0f) || k.mu * N + T <= 0.0f || (T <= 0.0f && N < 0.0f) || dm == 0.0f) continue;
        const float t = fmaxf(T, MJW_MINVAL), ttt = fmaxf(t * t * t, MJW_MINVAL);
        const float mu_over_t = safe_div(k.mu, t), mu_n_over_ttt = k.mu * safe_div(N, ttt), diag = mu2 - k.mu * safe_div(N, t);
        for (int a = 0; a < k.dim; a++) {
          // J[r + a][i]
          const int ra = r + a;
          float jai = 0.0f;
          for (int q = 0; q < c.Jnnz[ra]; q++)
            if (c.Jcol[(long)q * c.P + ra] == i) jai = c.J[(long)q * c.P + ra];
          if (jai == 0.0f) continue;
          for (int b = 0; b < k.dim; b++) {
            float h;
            if (a == 0 && b == 0) h = 1.0f;
            else if (a == 0) h = -mu_over_t * u[b];
            else if (b == 0) h = -mu_over_t * u[a];
            else h = mu_n_over_ttt * u[a] * u[b] + (a == b ? diag : 0.0f);
            h *= dm * fri[a] * fri[b];
            if (h == 0.0f) continue;
            const int rb = r + b;
            for (int q = 0; q < c.Jnnz[rb]; q++) {
              const int j = c.Jcol[(long)q * c.P + rb];
              if (j <= i) H[i * nv + j] += h * jai * c.J[(long)q * c.P + rb];
            }
          }
        }
      }
    }
  }
  __syncthreads();
  for (int i = tid(); i < nv; i += nthr()) {  // + M on its ancestor rows (diagonal last)
    const int adr = m.M_rowadr[i], nnz = m.M_rownnz[i];
    for (int p = 0; p < nnz - 1; p++) H[i * nv + m.M_colind[adr + p]] += c.M[adr + p];
    H[i * nv + i] += c.M[adr + nnz - 1];
  }
  for (int k = 0; k < nv; k++) {
    __syncthreads();
    const float piv = sqrtf(fmaxf(H[k * nv + k], MJW_MINVAL));
    __syncthreads();
    if (tid() == 0) H[k * nv + k] = piv;
    for (int i = k + 1 + tid(); i < nv; i += nthr()) H[i * nv + k] /= piv;
    __syncthreads();
    for (int i = k + 1 + tid(); i < nv; i += nthr()) {
      const float lik = H[i * nv + k];
      for (int j = k + 1; j <= i; j++) H[i * nv + j] -= lik * H[j * nv + k];
    }
  }
  __syncthreads();
  // L y = grad, then L' x = y, in Mgrad (one pivot per round, the updates in parallel)
  float* x = c.Mgrad;
  for (int k = 0; k < nv; k++) {
    const float yk = x[k] / H[k * nv + k];
    __syncthreads();
    if (tid() == 0) x[k] = yk;
    for (int i = k + 1 + tid(); i < nv; i += nthr()) x[i] -= H[i * nv + k] * yk;
    __syncthreads();
  }
  for (int k = nv - 1; k >= 0; k--) {
    const float xk = x[k] / H[k * nv + k];
    __syncthreads();
    if (tid() == 0) x[k] = xk;
    for (int i = tid(); i < k; i += nthr()) x[i] -= H[k * nv + i] * xk;
    __syncthreads();
  }
}

template <bool ELL = false>
__device__ __forceinline__ void update_gradient(const mjw_model_t& m, SolveCtx& c, Smem& sm) {
  SPROF_T0_SUB();
  float gd = 0.0f;
  for (int i = tid(); i < c.nv; i += nthr()) {
    const float g = c.Ma[i] - c.qfrc_s[i] - c.qfrc_c[i];
    c.grad[i] = g;
    c.Mgrad[i] = g;
    gd += g * g;
  }
  c.grad_dot = block_sum1_db(gd, sm, c.rphase);  // syncs
  if (c.newton) newton_direction<ELL>(m, c);
  else solve_trees(m, c.LD, c.Mgrad);
  __syncthreads();
  SPROF_MARK_SUB(SPH_S_TREES);
}

__device__ __forceinline__ bool in_bracket(const float* x, const float* y) {
  return (x[1] < y[1] && y[1] < 0.0f) || (x[1] > y[1] && y[1] > 0.0f);
}

// returns the step; qacc / Ma are updated here, Jaref by update_constraint
template <bool ELL = false>
__device__ __forceinline__ float linesearch(const mjw_model_t& m, SolveCtx& c, int wid, Smem& sm) {
  SPROF_T0_SUB();
  mul_m_trees(m, c.M, c.search, c.mv);
#ifdef MJW_PROFILE
  __syncthreads();  // (profile build only: the sub-phase ends when every tree is done)
#endif
  SPROF_MARK_SUB(SPH_S_MULM);
  // jv = J search, fused with the alpha = 0 evaluation of each row (same thread)
  // equality rows are quadratic for every step size: their cost 0.5 D (Jaref + a jv)^2 is folded
  // into the Gauss quadratic once here (v5[5..7]), and the line-search passes skip them
  float v5[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int r0 = tid(); r0 < c.nefc; r0 += RU * nthr()) {
    // RU rows interleaved so their (column -> search) gathers overlap; per-row order unchanged
    int nz[RU], kmax = 0;
    float acc[RU];
#pragma unroll
    for (int u = 0; u < RU; u++) {
      const int r = r0 + u * nthr();
      nz[u] = r < c.nefc ? c.Jnnz[r] : 0;
      kmax = max(kmax, nz[u]);
      acc[u] = 0.0f;
    }
    for (int k = 0; k < kmax; k++) {
      float v[RU];
      int col[RU];
#pragma unroll
      for (int u = 0; u < RU; u++) {
        const long q = (long)k * c.P + r0 + u * nthr();
        v[u] = k < nz[u] ? c.J[q] : 0.0f;
        col[u] = k < nz[u] ? c.Jcol16[q] : 0;
      }
#pragma unroll
      for (int u = 0; u < RU; u++)
        if (k < nz[u]) acc[u] += v[u] * c.search[col[u]];
    }
#pragma unroll
    for (int u = 0; u < RU; u++) {
    const int r = r0 + u * nthr();
    if (r >= c.nefc) continue;
    const float s = acc[u];
    c.jv[r] = s;
    if (r < c.ne) {
      const float D = c.D[r], ja = c.Jaref[r];
      v5[5] += 0.5f * D * ja * ja;
      v5[6] += D * ja * s;
      v5[7] += 0.5f * D * s * s;
    } else if (!ELL || r < c.ne + c.nf || c.ell->type[r] != CNSTR_CONTACT_ELLIPTIC) {
      eval_row(c, r, 0.0f, v5);
    }
    }
  }
  __syncthreads();
  SPROF_MARK_SUB(SPH_S_JV);
  if (ELL) {  // the cones at alpha = 0, once every row's jv is in
    for (int r = c.ne + c.nf + tid(); r < c.nefc; r += nthr()) {
      if (c.ell->type[r] != CNSTR_CONTACT_ELLIPTIC) continue;
      ConeRow k;
      if (!cone_of(c, r, k) || k.r0 != r) continue;
      float q[9];
      ell_quad(c, k, q);
      ell_eval(q, k.mu, 0.0f, v5);
    }
  }
  const float snorm = sqrtf(c.search_dot);
  const float scale = MR_W(stat_meaninertia) * (float)c.nv;
  const float gtol = fmaxf(MR_W(opt_tolerance) * MR_W(opt_ls_tolerance) * snorm * scale, 1e-6f);
  for (int i = tid(); i < c.nv; i += nthr()) {
    v5[3] += c.search[i] * (c.Ma[i] - c.qfrc_s[i]);
    v5[4] += 0.5f * c.search[i] * c.mv[i];
  }
  block_sum_db<8>(v5, sm, c.rphase);
  const float qg0 = c.gauss + v5[5], qg1 = v5[3] + v5[6], qg2 = v5[4] + v5[7];
  const float p0[3] = {qg0 + v5[0], qg1 + v5[1], 2.0f * qg2 + v5[2]};
  auto gauss_at = [&](float a, float* o) {
    o[0] = a * a * qg2 + a * qg1 + qg0;
    o[1] = 2.0f * a * qg2 + qg1;
    o[2] = 2.0f * qg2;
  };
  float alpha;
  if (m.opt_ls_parallel) {
    // solver.py:325-478 parallel linesearch: the cheapest of ls_iterations log-spaced step sizes in
    // [ls_parallel_min_step, 1] (the first one on ties), three per row pass
    alpha = 0.0f;
    float best = MJW_MAXVAL;
    const int n = m.opt_ls_iterations;
    for (int i0 = 0; i0 < n; i0 += 3) {
      float al[3], v9[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      for (int k = 0; k < 3; k++) al[k] = ls_parallel_alpha(MR_W(opt_ls_parallel_min_step), n, min(i0 + k, n - 1));
      eval_rows<3, ELL>(c, al, v9);
      block_sum_db<9>(v9, sm, c.rphase);
      for (int k = 0; k < 3 && i0 + k < n; k++) {
        float g[3];
        gauss_at(al[k], g);
        const float cst = v9[3 * k] + g[0];
        if (cst < best) { best = cst; alpha = al[k]; }
      }
    }
  } else {
  const float lo_alpha_in = -safe_div(p0[1], p0[2]);
  float lo_in[3] = {0, 0, 0};
  SPROF_COUNT(SPH_NPASS, 2);  // the jv + alpha = 0 pass above and this one
  eval_rows<1, ELL>(c, &lo_alpha_in, lo_in);
  block_sum_db<3>(lo_in, sm, c.rphase);
  {
    float g[3];
    gauss_at(lo_alpha_in, g);
    for (int k = 0; k < 3; k++) lo_in[k] += g[k];
  }
  if (!(fabsf(lo_in[1]) < gtol && lo_in[0] < p0[0])) {
    alpha = 0.0f;
    float lo[3], hi[3], lo_alpha, hi_alpha;
    if (lo_in[1] < p0[1]) {
      for (int k = 0; k < 3; k++) { lo[k] = lo_in[k]; hi[k] = p0[k]; }
      lo_alpha = lo_alpha_in;
      hi_alpha = 0.0f;
    } else {
      for (int k = 0; k < 3; k++) { lo[k] = p0[k]; hi[k] = lo_in[k]; }
      lo_alpha = 0.0f;
      hi_alpha = lo_alpha_in;
    }
    for (int it = 0; it < m.opt_ls_iterations; it++) {
      const float lo_next_alpha = lo_alpha - safe_div(lo[1], lo[2]);
      const float hi_next_alpha = hi_alpha - safe_div(hi[1], hi[2]);
      const float mid_alpha = 0.5f * (lo_alpha + hi_alpha);
      float v9[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      const float al[3] = {lo_next_alpha, hi_next_alpha, mid_alpha};
      SPROF_COUNT(SPH_NPASS, 1);
      eval_rows<3, ELL>(c, al, v9);
      block_sum_db<9>(v9, sm, c.rphase);
      float lo_next[3], hi_next[3], mid[3], g[3];
      gauss_at(lo_next_alpha, g);
      for (int k = 0; k < 3; k++) lo_next[k] = g[k] + v9[k];
      gauss_at(hi_next_alpha, g);
      for (int k = 0; k < 3; k++) hi_next[k] = g[k] + v9[3 + k];
      gauss_at(mid_alpha, g);
      for (int k = 0; k < 3; k++) mid[k] = g[k] + v9[6 + k];
      const bool s1 = in_bracket(lo, lo_next);
      if (s1) { for (int k = 0; k < 3; k++) lo[k] = lo_next[k]; lo_alpha = lo_next_alpha; }
      const bool s2 = in_bracket(lo, mid);
      if (s2) { for (int k = 0; k < 3; k++) lo[k] = mid[k]; lo_alpha = mid_alpha; }
      const bool s3 = in_bracket(lo, hi_next);
      if (s3) { for (int k = 0; k < 3; k++) lo[k] = hi_next[k]; lo_alpha = hi_next_alpha; }
      const bool h1 = in_bracket(hi, hi_next);
      if (h1) { for (int k = 0; k < 3; k++) hi[k] = hi_next[k]; hi_alpha = hi_next_alpha; }
      const bool h2 = in_bracket(hi, mid);
      if (h2) { for (int k = 0; k < 3; k++) hi[k] = mid[k]; hi_alpha = mid_alpha; }
      const bool h3 = in_bracket(hi, lo_next);
      if (h3) { for (int k = 0; k < 3; k++) hi[k] = lo_next[k]; hi_alpha = lo_next_alpha; }
      const bool done = (!(s1 || s2 || s3) && !(h1 || h2 || h3)) || (lo[1] < 0.0f && lo[1] > -gtol) || (hi[1] > 0.0f && hi[1] < gtol);
      const bool improved = lo[0] < p0[0] || hi[0] < p0[0];
      if (improved) alpha = lo[0] < hi[0] ? lo_alpha : hi_alpha;
      if (done) break;
    }
  } else {
    alpha = lo_alpha_in;
  }
  }
  SPROF_MARK_SUB(SPH_S_LSP);
  for (int i = tid(); i < c.nv; i += nthr()) {
    c.qacc[i] += alpha * c.search[i];
    c.Ma[i] += alpha * c.mv[i];
  }
  __syncthreads();
  return alpha;
}

// PART 0: qacc from the warmstart, Jaref, and the transposed index of J; PART 1: the CG iterations.
// Two launches so that the index build (register-resident segment sorts) and the solver loop each
// get their own register budget.  PART 2 is PART 1 with the per-row line-search state (Jaref, jv)
// in LDS and SOLVE_LDS_THREADS threads per world: the line-search passes, which re-read that state
// several times per CG iteration, then stop streaming it through HBM (sparse_launch picks it when
// 2 * njmax floats fit the LDS of a CU).
template <int PART>
__global__ void __launch_bounds__(PART == 2 ? SOLVE_LDS_THREADS : BLK, PART == 2 ? 1 : MJW_SP_SOLVE_MINBLK) solve_kernel(const mjw_model_t m, const mjw_data_t d) {
  // PART 3: PART 1 for elliptic-cone models (the cone rows of a contact are evaluated together)
  constexpr bool ELL = PART == 3;
  __shared__ Smem sm;
  const int wid = blockIdx.x;
  const int nv = m.nv, njmax = d.njmax;
  float* qacc = d.qacc + (long)wid * nv;
  const float* qacc_s = d.qacc_smooth + (long)wid * nv;
  if (njmax == 0 || nv == 0) {
    if (PART == 0) return;
    for (int i = tid(); i < nv; i += nthr()) qacc[i] = qacc_s[i];
    if (tid() == 0) d.solver_niter[wid] = 0;
    return;
  }
  SPROF_T0();
  SolveCtx c;
  c.rphase = 0;
  c.nv = nv;
  c.nefc = min(d.nefc[wid], njmax);
  c.ne = d.ne[wid];
  c.nf = d.nf[wid];
  c.njrow = m.njrow;
  const long P = d.njmax_pad;
  c.P = (int)P;
  c.J = d.efc_J + (long)wid * d.njmax_pad * m.njrow;
  c.Jcol = d.efc_J_colind + (long)wid * d.njmax_pad * m.njrow;
  c.Jnnz = d.efc_J_rownnz + (long)wid * njmax;
  int* JT_adr = d.efc_JT_adr + (long)wid * (nv + 1);
  int* JT_ind = d.efc_JT_rowind + (long)wid * d.njmax_pad * m.njrow;
  // column counters in LDS when they fit (sparse_launch sizes the dynamic LDS), else in HBM
  extern __shared__ int s_cnt[];
  int* cnt = (nv + 1) <= SP_LDS_CNT_MAX ? s_cnt : d.sp_cnt + (long)wid * (nv + 1);
  float* JT_val = d.efc_JT_val + (long)wid * d.njmax_pad * m.njrow;
  c.JT_adr = JT_adr;
  c.JT_val = JT_val;
  // 16-bit indices (rows < 65536 and dofs < 65535, io.make_data checks): half the index bytes that every
  // CG iteration streams twice (the jv pass's columns, the J'f gathers' rows)
  unsigned short* idx16 = reinterpret_cast<unsigned short*>(d.sp_idx16 + (long)wid * d.njmax_pad * m.njrow);
  unsigned short* Jcol16 = idx16;
  unsigned short* JT16 = idx16 + P * m.njrow;
  c.Jcol16 = Jcol16;
  c.JT16 = JT16;
  c.D = d.efc_D + (long)wid * d.njmax_pad;
  c.fl = d.efc_frictionloss + (long)wid * njmax;
  c.aref = d.efc_aref + (long)wid * njmax;
  c.force = d.efc_force + (long)wid * njmax;
  c.state = d.efc_state + (long)wid * d.njmax_pad;
  c.Jaref = d.sp_row + (long)wid * njmax * 3;
  c.jv = c.Jaref + njmax;
  c.Dq = c.Jaref + 2 * njmax;
  EllCtx ell;
  if (ELL) {
    ell.type = d.efc_type + (long)wid * njmax;
    ell.id = d.efc_id + (long)wid * njmax;
    ell.con_adr = d.contact_efc_address;
    ell.con_dim = d.contact_dim;
    ell.con_fr = d.contact_friction;
    ell.nmaxpyr = m.nmaxpyramid;
    ell.iri = MR_W(opt_impratio_invsqrt);
  }
  c.ell = ELL ? &ell : nullptr;
  c.newton = m.opt_solver == SOLVER_NEWTON && m.sp_nH == nv;
  c.H = c.newton ? d.sp_H + (long)wid * nv * nv : nullptr;
  if constexpr (PART == 2) {
    float* rows = reinterpret_cast<float*>(s_cnt);
    for (int r = tid(); r < c.nefc; r += nthr()) rows[r] = c.Jaref[r];
    c.Jaref = rows;
    c.jv = rows + njmax;
    __syncthreads();
  }
  c.qacc = qacc;
  c.Ma = d.efc_Ma + (long)wid * nv;
  c.qfrc_c = d.qfrc_constraint + (long)wid * nv;
  c.qfrc_s = d.qfrc_smooth + (long)wid * nv;
  c.qacc_s = qacc_s;
  float* vec = d.sp_vec + (long)wid * nv * 10;
  c.grad = vec;
  c.Mgrad = vec + nv;
  c.search = vec + 2 * nv;
  c.mv = vec + 3 * nv;
  c.pgrad = vec + 4 * nv;
  c.pMgrad = vec + 5 * nv;
  if constexpr (PART != 0) {
    // the search direction in LDS when it fits: the jv pass gathers it by column every CG iteration
    if (nv <= SP_LDS_SEARCH_MAX) c.search = reinterpret_cast<float*>(s_cnt) + (PART == 2 ? 2 * njmax : 0);
  }
  c.M = d.qM + (long)wid * m.nM;
  c.LD = d.qLD + (long)wid * m.nM;
  const float* warm = d.qacc_warmstart + (long)wid * nv;
  const bool ws = !(m.opt_disableflags & DSBL_WARMSTART);
  if constexpr (PART == 0) {
  // transposed index of J: counts, scan, fill, per-column sort (deterministic J'f)
  for (int i = tid(); i <= nv; i += nthr()) cnt[i] = 0;
  for (int i = tid(); i < nv; i += nthr()) qacc[i] = ws ? warm[i] : qacc_s[i];
  __syncthreads();
  for (int r = tid(); r < c.nefc; r += nthr())
    for (int k = 0; k < c.Jnnz[r]; k++) atomicAdd(&cnt[c.Jcol[k * P + r]], 1);
  __syncthreads();
  int run = 0;
  for (int c0 = 0; c0 < nv; c0 += nthr()) {
    const int i = c0 + tid();
    const int n = i < nv ? cnt[i] : 0;
    int chunk;
    const int off = block_scan(n, chunk, sm);
    if (i < nv) { JT_adr[i] = run + off; cnt[i] = run + off; }
    run += chunk;
  }
  if (tid() == 0) JT_adr[nv] = run;
  __syncthreads();
  // fill carries the values (and computes Jaref on the way); the per-column sort of the
  // (row * njrow + slot) codes then fixes the summation order of J'f whatever the atomics did
  for (int r = tid(); r < c.nefc; r += nthr()) {
    float s = 0.0f;
    for (int k = 0; k < c.Jnnz[r]; k++) {
      const float v = c.J[k * P + r];
      const int col = c.Jcol[k * P + r];
      Jcol16[k * P + r] = (unsigned short)col;
      const int pos = atomicAdd(&cnt[col], 1);
      JT_ind[pos] = r * m.njrow + k;
      JT_val[pos] = v;
      s += v * qacc[col];
    }
    c.Jaref[r] = s - c.aref[r];
  }
  __syncthreads();
  for (int i = tid(); i < nv; i += nthr()) {
    const int a = JT_adr[i], b = JT_adr[i + 1];
    if (b - a <= SORTN) {
      // short segment: loaded at once, odd-even transposition network in registers
      const int n = b - a;
      int key[SORTN];
      float val[SORTN];
#pragma unroll
      for (int j = 0; j < SORTN; j++) {
        key[j] = j < n ? JT_ind[a + j] : 0x7fffffff;
        val[j] = j < n ? JT_val[a + j] : 0.0f;
      }
#pragma unroll
      for (int r = 0; r < SORTN; r++) {
#pragma unroll
        for (int j = r & 1; j + 1 < SORTN; j += 2) {
          const bool sw = key[j] > key[j + 1];
          const int k0 = key[j], k1 = key[j + 1];
          const float v0 = val[j], v1 = val[j + 1];
          key[j] = sw ? k1 : k0;
          key[j + 1] = sw ? k0 : k1;
          val[j] = sw ? v1 : v0;
          val[j + 1] = sw ? v0 : v1;
        }
      }
#pragma unroll
      for (int j = 0; j < SORTN; j++)
        if (j < n) {
          JT16[a + j] = (unsigned short)(key[j] / m.njrow);  // code -> row
          JT_val[a + j] = val[j];
        }
      continue;
    }
    for (int p = a + 1; p < b; p++) {
      const int key = JT_ind[p];
      const float kv = JT_val[p];
      int q = p - 1;
      while (q >= a && JT_ind[q] > key) { JT_ind[q + 1] = JT_ind[q]; JT_val[q + 1] = JT_val[q]; q--; }
      JT_ind[q + 1] = key;
      JT_val[q + 1] = kv;
    }
    for (int p = a; p < b; p++) JT16[p] = (unsigned short)(JT_ind[p] / m.njrow);  // code -> row
  }
  return;
  }
  mul_m_trees(m, c.M, qacc, c.Ma);
  __syncthreads();
  c.cost = MJW_MAXVAL;
  update_constraint<ELL>(c, sm);
  update_gradient<ELL>(m, c, sm);
  float sd = 0.0f;
  for (int i = tid(); i < nv; i += nthr()) {
    c.search[i] = -c.Mgrad[i];
    sd += c.Mgrad[i] * c.Mgrad[i];
  }
  c.search_dot = block_sum1_db(sd, sm, c.rphase);
  const float scale = 1.0f / (MR_W(stat_meaninertia) * (float)nv);
  const float tol = MR_W(opt_tolerance);
  int niter = 0;
  SPROF_MARK(SPH_SINIT);
  if (m.opt_iterations != 0) {
    for (;;) {
      const float alpha = linesearch<ELL>(m, c, wid, sm);
      SPROF_MARK(SPH_SLS);
      for (int i = tid(); i < nv; i += nthr()) {
        c.pgrad[i] = c.grad[i];
        c.pMgrad[i] = c.Mgrad[i];
      }
      __syncthreads();
      update_constraint<ELL>(c, sm, alpha);
      update_gradient<ELL>(m, c, sm);
      SPROF_MARK(SPH_SUPD);
      float nd[2] = {0.0f, 0.0f};
      for (int i = tid(); i < nv; i += nthr()) {
        nd[0] += c.grad[i] * (c.Mgrad[i] - c.pMgrad[i]);
        nd[1] += c.pgrad[i] * c.pMgrad[i];
      }
      block_sum_db<2>(nd, sm, c.rphase);
      // Polak-Ribiere for CG; Newton steps along -H^-1 grad (solver.py:3141-3144)
      const float beta = c.newton ? 0.0f : fmaxf(0.0f, nd[0] / fmaxf(MJW_MINVAL, nd[1]));
      float s2 = 0.0f;
      for (int i = tid(); i < nv; i += nthr()) {
        const float v = -c.Mgrad[i] + beta * c.search[i];
        c.search[i] = v;
        s2 += v * v;
      }
      c.search_dot = block_sum1_db(s2, sm, c.rphase);
      niter++;
      SPROF_MARK(SPH_SCG);
      SPROF_COUNT(SPH_NITER, 1);
      const float improvement = (c.prev_cost - c.cost) * scale;
      const float gradient = sqrtf(c.grad_dot) * scale;
      if (improvement < tol || gradient < tol || niter == m.opt_iterations) break;
    }
  }
  write_states<ELL>(c);
  if (tid() == 0) d.solver_niter[wid] = niter;
}

// forward.py:326-354 euler with implicit damping (sparse: factor M + dt*diag(damping) per tree), and
// implicitfast (forward.py:494-510): M - dt qDeriv with qDeriv = sum_a vel_a m_a m_a' - diag(damping)
// (derivative.py:320-416) on the ancestor rows of the sparse M, which hold exactly that pattern
__global__ void __launch_bounds__(BLK) euler_kernel(const mjw_model_t m, const mjw_data_t d) {
  const int wid = blockIdx.x;
  const int nv = m.nv;
  const float dt = MR_W(opt_timestep);
  float* qvel = d.qvel + (long)wid * nv;
  float* qpos = d.qpos + (long)wid * m.nq;
  const float* qacc = d.qacc + (long)wid * nv;
  const float* adv = qacc;
  const int fl = m.opt_disableflags;
  const bool implicitfast = m.opt_integrator == INT_IMPLICITFAST;
  const bool need_implicit = implicitfast ? (fl & (DSBL_ACTUATION | DSBL_SPRING | DSBL_DAMPER)) != (DSBL_ACTUATION | DSBL_SPRING | DSBL_DAMPER)
                                          : !(fl & (DSBL_EULERDAMP | DSBL_DAMPER));
  if (need_implicit) {
    float* LD2 = d.sp_LD + (long)wid * m.nM;
    float* q = d.sp_vec + (long)wid * nv * 10 + 6 * nv;
    const float* M = d.qM + (long)wid * m.nM;
    const float* damping = MR(dof_damping);
    const bool damp = !(fl & DSBL_DAMPER);
    for (int i = tid(); i < nv; i += BLK) {
      const int adr = m.M_rowadr[i], nnz = m.M_rownnz[i];
      for (int p = 0; p < nnz; p++) LD2[adr + p] = M[adr + p];
      if (damp) LD2[adr + nnz - 1] += dt * damping[i];
    }
    __syncthreads();
    if (implicitfast && m.nu > 0 && !(fl & DSBL_ACTUATION)) {
      for (int u = 0; u < m.nu; u++) {  // uniform: one actuator's (i >= j) moment pairs per round
        const float vel = actuator_vel_deriv(m, d, wid, u);
        if (vel == 0.0f) continue;
        const long gu = (long)wid * m.nu + u;
        const int nnz = d.moment_rownnz[gu];
        const long base = (long)wid * m.nJmom + d.moment_rowadr[gu];
        for (int p = tid(); p < nnz * nnz; p += BLK) {
          const int k1 = p / nnz, k2 = p - k1 * nnz;
          const int i = d.moment_colind[base + k1], j = d.moment_colind[base + k2];
          if (i < j) continue;
          const int adr = m.M_rowadr[i], rn = m.M_rownnz[i];
          int pos = -1;
          if (i == j) pos = adr + rn - 1;
          else
            for (int q2 = 0; q2 < rn - 1; q2++)
              if (m.M_colind[adr + q2] == j) pos = adr + q2;
          if (pos >= 0) LD2[pos] -= dt * vel * d.actuator_moment[base + k1] * d.actuator_moment[base + k2];
        }
        __syncthreads();
      }
    }
    if (implicitfast && m.ntendon && !(fl & DSBL_DAMPER)) {
      // derivative.py:267-320: tendon damping enters qDeriv as -damping J_i J_j on the ancestor pattern of M
      const float* tdamp = MR(tendon_damping);
      for (int t = 0; t < m.ntendon; t++) {
        if (tdamp[t] == 0.0f) continue;
        const int rn = m.ten_J_rownnz[t], ra = m.ten_J_rowadr[t];
        const float* J = d.ten_J + (long)wid * m.nJten + ra;
        for (int p = tid(); p < rn * rn; p += BLK) {
          const int k1 = p / rn, k2 = p - k1 * rn;
          if (k2 > k1) continue;
          const int pos = m_pos(m, m.ten_J_colind[ra + k1], m.ten_J_colind[ra + k2]);
          if (pos >= 0) LD2[pos] += dt * tdamp[t] * J[k1] * J[k2];
        }
        __syncthreads();
      }
    }
    factor_trees(m, LD2, LD2, nullptr, 0.0f);
    for (int i = tid(); i < nv; i += BLK) q[i] = d.efc_Ma[(long)wid * nv + i];
    __syncthreads();
    solve_trees(m, LD2, q);
    __syncthreads();
    adv = q;
  }
  for (int a = tid(); a < m.nu; a += BLK) {
    const int adr = m.actuator_actadr[a];
    for (int j = adr; adr >= 0 && j < adr + m.actuator_actnum[a]; j++) {
      const long g = (long)wid * m.na + j;
      d.act[g] = next_act(dt, m.actuator_dyntype[a], MR(actuator_dynprm)[10 * a], MR(actuator_actrange) + 2 * a, d.act[g], d.act_dot[g], 1.0f,
                          m.actuator_actlimited[a] != 0);
    }
  }
  for (int i = tid(); i < nv; i += BLK) qvel[i] += adv[i] * dt;
  __syncthreads();
  for (int j = tid(); j < m.njnt; j += BLK) {
    const int qa = m.jnt_qposadr[j], da = m.jnt_dofadr[j], jt = m.jnt_type[j];
    if (jt == JNT_FREE) {
      for (int i = 0; i < 3; i++) qpos[qa + i] += dt * qvel[da + i];
      float qn[4];
      quat_integrate(qn, qpos + qa + 3, qvel + da + 3, dt);
      for (int i = 0; i < 4; i++) qpos[qa + 3 + i] = qn[i];
    } else if (jt == JNT_BALL) {
      float qn[4];
      quat_integrate(qn, qpos + qa, qvel + da, dt);
      for (int i = 0; i < 4; i++) qpos[qa + i] = qn[i];
    } else {
      qpos[qa] += dt * qvel[da];
    }
  }
  for (int i = tid(); i < nv; i += BLK) d.qacc_warmstart[(long)wid * nv + i] = qacc[i];
  if (tid() == 0) d.time[wid] += dt;
}

}  // namespace sp

#ifdef MJW_PROFILE
extern "C" int mjw_prof_read_sparse(unsigned long long* out, int reset) {
  static unsigned long long c[sp::SPH_N * sp::SPROF_COPIES];
  hipError_t e = hipMemcpyFromSymbol(c, HIP_SYMBOL(sp::g_sprof), sizeof(c));
  for (int p = 0; p < sp::SPH_N; p++) {
    unsigned long long t = 0;
    for (int k = 0; k < sp::SPROF_COPIES; k++) t += c[p * sp::SPROF_COPIES + k];
    out[p] = t;
  }
  if (e == hipSuccess && reset) {
    for (auto& v : c) v = 0;
    e = hipMemcpyToSymbol(HIP_SYMBOL(sp::g_sprof), c, sizeof(c));
  }
  return (int)e;
}
#endif

// launcher used by the C entry points (mjw_step.hip) for models with m->is_sparse
int sparse_launch(int stages, const mjw_model_t* m, const mjw_data_t* d, hipStream_t s) {
  const int nw = d->nworld;
  if (nw <= 0) return 0;
  if (stages & ST_POOL) {
    // constraint rows (and transmission) again from the contact pool as a contactfilter left it
    hipLaunchKernelGGL(sp::forward_kernel<sp::SP_CON>, dim3(nw), dim3(sp::BLK), 0, s, *m, *d, (int)ST_POS);
    trace_launch(s, K_SP_CON);
    return (int)hipGetLastError();
  }
  const int fwd = stages & (ST_POS | ST_VEL | ST_ACT | ST_ACC);
  const bool ccd = (stages & ST_POS) && m->nxn_ccd > 0 && d->naconmax > 0 && !(m->opt_disableflags & (DSBL_CONSTRAINT | DSBL_CONTACT));
  if (fwd & ST_POS) {
    // frames, [the convex pre-pass,] collision, constraint rows
    hipLaunchKernelGGL(sp::forward_kernel<sp::SP_POS_A>, dim3(nw), dim3(sp::BLK), 0, s, *m, *d, fwd);
    trace_launch(s, K_SP_POS);
    if (ccd) {
      const size_t lds = ((size_t)ccd_layout(m->ccd_epa_iterations, m->nhfield > 0, m->nmaxpolygon, m->nmaxmeshdeg).total + 64) * 4;
      if (m->nhfield > 0) {
        hipLaunchKernelGGL(sp::ccd_hf_kernel, dim3(nw), dim3(64), lds, s, *m, *d);
        trace_launch(s, K_SP_CCD_HF);
      } else {
        hipLaunchKernelGGL(sp::ccd_kernel, dim3(nw), dim3(64), lds, s, *m, *d);
        trace_launch(s, K_SP_CCD);
      }
    }
    // collision items (upper bound of ncollide_items): one LDS byte each when they fit
    const long nitem = (long)m->nxn + (long)m->nflexvert * m->nplane + ((long)m->nflexelem + m->nflexshelldata / 3) * m->nflexcg;
    const size_t lds = nitem <= sp::SP_LDS_ITEMS_MAX ? (size_t)((nitem + 3) & ~3L) : 0;
    hipLaunchKernelGGL(sp::forward_kernel<sp::SP_COLL>, dim3(nw), dim3(sp::BLK), lds, s, *m, *d, fwd);
    trace_launch(s, K_SP_COLL);
    hipLaunchKernelGGL(sp::forward_kernel<sp::SP_CON>, dim3(nw), dim3(sp::BLK), 0, s, *m, *d, fwd);
    trace_launch(s, K_SP_CON);
  }
  if (fwd & (ST_VEL | ST_ACT | ST_ACC)) {
    hipLaunchKernelGGL(sp::forward_kernel<ST_VEL>, dim3(nw), dim3(sp::BLK), 0, s, *m, *d, fwd);
    trace_launch(s, K_SP_VEL);
  }
  if (stages & ST_SOLVE) {
    const size_t lds = (m->nv + 1) <= sp::SP_LDS_CNT_MAX ? (size_t)(m->nv + 1) * 4 : 0;
    hipLaunchKernelGGL(sp::solve_kernel<0>, dim3(nw), dim3(sp::BLK), lds, s, *m, *d);
    trace_launch(s, K_SP_INDEX);
    // CG iterations, the search direction in LDS.  MJW_SP_SOLVE_LDS=1 also keeps Jaref / jv of every
    // row in LDS (1024-thread worlds, when 2 * njmax floats fit): measured equal on aloha_cloth
    // (22.75 vs 22.80 ms per step) and 4 % slower on cloth, so the rows stay in HBM by default
    const size_t search_lds = m->nv <= sp::SP_LDS_SEARCH_MAX ? (size_t)m->nv * 4 : 0;
    const size_t row_lds = (size_t)2 * d->njmax * 4 + search_lds;
    static const bool lds_ok = [] {
      const char* e = getenv("MJW_SP_SOLVE_LDS");
      return e && e[0] == '1';
    }();
    if (m->opt_cone == CONE_ELLIPTIC) {
      hipLaunchKernelGGL(sp::solve_kernel<3>, dim3(nw), dim3(sp::BLK), search_lds, s, *m, *d);
      trace_launch(s, K_SP_SOLVE);
    } else if (lds_ok && d->njmax > 0 && row_lds <= 150 * 1024) {
      static std::once_flag once;
      std::call_once(once, [] {
        (void)hipFuncSetAttribute((const void*)sp::solve_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
      });
      hipLaunchKernelGGL(sp::solve_kernel<2>, dim3(nw), dim3(sp::SOLVE_LDS_THREADS), row_lds, s, *m, *d);
      trace_launch(s, K_SP_SOLVE_LDS);
    } else {
      hipLaunchKernelGGL(sp::solve_kernel<1>, dim3(nw), dim3(sp::BLK), search_lds, s, *m, *d);
      trace_launch(s, K_SP_SOLVE);
    }
  }
  if (stages & ST_EULER) {
    hipLaunchKernelGGL(sp::euler_kernel, dim3(nw), dim3(sp::BLK), 0, s, *m, *d);
    trace_launch(s, K_SP_EULER);
  }
  return (int)hipGetLastError();
}

}  // namespace mjw
