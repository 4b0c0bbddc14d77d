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
constexpr int CREC = 32;  // floats per staged contact record
constexpr int CMAX = 32;  // staged contacts per collision round

enum : int { ST_POS = 1, ST_VEL = 2, ST_ACT = 4, ST_ACC = 8, ST_SOLVE = 16, ST_EULER = 32, ST_NOFACTOR = 64 };
enum : int { JNT_FREE = 0, JNT_BALL = 1, JNT_SLIDE = 2, JNT_HINGE = 3 };
enum : int { GEOM_PLANE = 0, GEOM_SPHERE = 2, GEOM_CAPSULE = 3 };
enum : int {
  DSBL_CONSTRAINT = 1, DSBL_EQUALITY = 2, DSBL_FRICTIONLOSS = 4, DSBL_LIMIT = 8, DSBL_CONTACT = 16, DSBL_SPRING = 32,
  DSBL_DAMPER = 64, DSBL_GRAVITY = 128, DSBL_CLAMPCTRL = 256, DSBL_WARMSTART = 512, DSBL_ACTUATION = 2048,
  DSBL_REFSAFE = 4096, DSBL_EULERDAMP = 1 << 15
};
enum : int { ENBL_ENERGY = 2 };
enum : int { CNSTR_FRICTION_DOF = 1, CNSTR_LIMIT_JOINT = 3, CNSTR_CONTACT_FRICTIONLESS = 5, CNSTR_CONTACT_PYRAMIDAL = 6 };
enum : int { STATE_SATISFIED = 0, STATE_QUADRATIC = 1, STATE_LINEARNEG = 2, STATE_LINEARPOS = 3 };
enum : int { SOLVER_CG = 1, SOLVER_NEWTON = 2 };
enum : int { CAM_FIXED = 0, CAM_TRACK = 1, CAM_TRACKCOM = 2, CAM_TARGETBODY = 3, CAM_TARGETBODYCOM = 4 };
enum : int { FILTER_PLANE = 1, FILTER_SPHERE = 2, FILTER_AABB = 4, FILTER_OBB = 8 };

// batched model field base pointer for world w (types.py "*" semantics: worldid % nb)
__device__ __forceinline__ const float* mb(const float* p, int nb, int cnt, int w) {
  return nb <= 1 ? p : p + (long)(w % nb) * cnt;
}
#define MR(name) mb(m.name, m.name##_nb, m.name##_cnt, wid)


// dense (register-resident) factor / solve / euler kernel launcher, mjw_dense.hip
enum : int { DF_FACTOR = 1, DF_SOLVE = 2, DF_EULER = 4 };
int dense_launch(int flags, const mjw_model_t* m, const mjw_data_t* d, hipStream_t s);

}  // namespace mjw
