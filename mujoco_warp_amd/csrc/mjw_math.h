// Device math helpers (fp32) for the world-per-wavefront step.
// Formulas follow mujoco_warp/_src/math.py (cited per function); vectors are
// plain float arrays so the compiler keeps them in VGPRs.
#pragma once
#include <hip/hip_runtime.h>

#define MJW_MINVAL 1e-15f
#define MJW_MAXVAL 1e10f
#define MJW_MINIMP 0.0001f
#define MJW_MAXIMP 0.9999f
#define MJW_MINMU 1e-5f

namespace mjw {

__device__ __forceinline__ float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

__device__ __forceinline__ void cross3(float* r, const float* a, const float* b) {
  float t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// math.py:317-319
__device__ __forceinline__ float safe_div(float x, float y) { return x / (y != 0.0f ? y : MJW_MINVAL); }

// constraint.py:91-100 (_efc_row): the impedance shape of solimp's (mid, power) at imp_x, with the
// integer powers (solimp's default is 2) as products instead of powf, which costs ~100 VALU
// instructions per call and was a quarter of the forward kernel's code
__device__ __forceinline__ float imp_pow(float x, float p) {
  if (p == 1.0f) return x;
  if (p == 2.0f) return x * x;
  if (p == 3.0f) return x * x * x;
  return powf(x, p);
}
__device__ __forceinline__ float imp_shape(float imp_x, float mid, float power) {
  if (imp_x < mid) return (1.0f / imp_pow(mid, power - 1.0f)) * imp_pow(imp_x, power);
  return 1.0f - (1.0f / imp_pow(1.0f - mid, power - 1.0f)) * imp_pow(1.0f - imp_x, power);
}

// wp.normalize semantics: zero stays zero
__device__ __forceinline__ void normalize3(float* v) {
  float n = sqrtf(dot3(v, v));
  if (n > 0.0f) { v[0] /= n; v[1] /= n; v[2] /= n; } else { v[0] = v[1] = v[2] = 0.0f; }
}
__device__ __forceinline__ void normalize4(float* q) {
  float n = sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n > 0.0f) { q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n; } else { q[0] = q[1] = q[2] = q[3] = 0.0f; }
}

// math.py:23-30
__device__ __forceinline__ void mul_quat(float* r, const float* u, const float* v) {
  float t0 = u[0] * v[0] - u[1] * v[1] - u[2] * v[2] - u[3] * v[3];
  float t1 = u[0] * v[1] + u[1] * v[0] + u[2] * v[3] - u[3] * v[2];
  float t2 = u[0] * v[2] - u[1] * v[3] + u[2] * v[0] + u[3] * v[1];
  float t3 = u[0] * v[3] + u[1] * v[2] - u[2] * v[1] + u[3] * v[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}

// math.py:33-41: q * (0, axis)
__device__ __forceinline__ void quat_mul_axis(float* r, const float* q, const float* a) {
  float t0 = -q[1] * a[0] - q[2] * a[1] - q[3] * a[2];
  float t1 = q[0] * a[0] + q[2] * a[2] - q[3] * a[1];
  float t2 = q[0] * a[1] + q[3] * a[0] - q[1] * a[2];
  float t3 = q[0] * a[2] + q[1] * a[1] - q[2] * a[0];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
}

// math.py:44-49
__device__ __forceinline__ void rot_vec_quat(float* r, const float* vec, const float* q) {
  float s = q[0];
  float u[3] = {q[1], q[2], q[3]};
  float uv = dot3(u, vec), uu = dot3(u, u);
  float c[3];
  cross3(c, u, vec);
  float t0 = 2.0f * (uv * u[0]) + (s * s - uu) * vec[0] + 2.0f * s * c[0];
  float t1 = 2.0f * (uv * u[1]) + (s * s - uu) * vec[1] + 2.0f * s * c[1];
  float t2 = 2.0f * (uv * u[2]) + (s * s - uu) * vec[2] + 2.0f * s * c[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}

// math.py:52-56
__device__ __forceinline__ void axis_angle_to_quat(float* q, const float* axis, float angle) {
  float s = sinf(angle * 0.5f), c = cosf(angle * 0.5f);
  q[0] = c; q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}

// math.py:59-83 (row-major)
__device__ __forceinline__ void quat_to_mat(float* m, const float* q) {
  float q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  float q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3], q22 = q[2] * q[2];
  float q23 = q[2] * q[3], q33 = q[3] * q[3];
  m[0] = q00 + q11 - q22 - q33; m[1] = 2.0f * (q12 - q03); m[2] = 2.0f * (q13 + q02);
  m[3] = 2.0f * (q12 + q03); m[4] = q00 - q11 + q22 - q33; m[5] = 2.0f * (q23 - q01);
  m[6] = 2.0f * (q13 - q02); m[7] = 2.0f * (q23 + q01); m[8] = q00 - q11 - q22 + q33;
}

// math.py:120-130
__device__ __forceinline__ void inert_vec(float* r, const float* i, const float* v) {
  float t0 = i[0] * v[0] + i[3] * v[1] + i[4] * v[2] - i[8] * v[4] + i[7] * v[5];
  float t1 = i[3] * v[0] + i[1] * v[1] + i[5] * v[2] + i[8] * v[3] - i[6] * v[5];
  float t2 = i[4] * v[0] + i[5] * v[1] + i[2] * v[2] - i[7] * v[3] + i[6] * v[4];
  float t3 = i[8] * v[1] - i[7] * v[2] + i[9] * v[3];
  float t4 = i[6] * v[2] - i[8] * v[0] + i[9] * v[4];
  float t5 = i[7] * v[0] - i[6] * v[1] + i[9] * v[5];
  r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3; r[4] = t4; r[5] = t5;
}

// math.py:133-144
__device__ __forceinline__ void motion_cross(float* r, const float* u, const float* v) {
  float a[3], b[3], c[3];
  cross3(a, u, v);
  cross3(b, u + 3, v);
  cross3(c, u, v + 3);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
  r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}

// math.py:147-158
__device__ __forceinline__ void motion_cross_force(float* r, const float* v, const float* f) {
  float a[3], b[3], c[3];
  cross3(a, v, f);
  cross3(b, v + 3, f + 3);
  cross3(c, v, f + 3);
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
  r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}

// math.py:161-174
__device__ __forceinline__ void quat_to_vel(float* r, const float* q) {
  float axis[3] = {q[1], q[2], q[3]};
  float s = sqrtf(dot3(axis, axis));
  if (s == 0.0f) { r[0] = r[1] = r[2] = 0.0f; return; }
  float speed = 2.0f * atan2f(s, q[0]);
  if (speed > 3.14159265358979f) speed -= 2.0f * 3.14159265358979f;
  r[0] = axis[0] * speed / s; r[1] = axis[1] * speed / s; r[2] = axis[2] * speed / s;
}

// math.py:177-185
__device__ __forceinline__ void quat_sub(float* r, const float* qa, const float* qb) {
  float qneg[4] = {qb[0], -qb[1], -qb[2], -qb[3]}, qd[4];
  mul_quat(qd, qneg, qa);
  quat_to_vel(r, qd);
}

// math.py:188-199
__device__ __forceinline__ void quat_integrate(float* res, const float* qin, const float* vin, float dt) {
  float v[3] = {vin[0], vin[1], vin[2]};
  float n = sqrtf(dot3(v, v));
  normalize3(v);
  float qr[4], q[4] = {qin[0], qin[1], qin[2], qin[3]};
  axis_angle_to_quat(qr, v, dt * n);
  normalize4(q);
  mul_quat(res, q, qr);
  normalize4(res);
}

// math.py:202-213
__device__ __forceinline__ void orthogonals(float* b, float* c, const float* a) {
  bool usey = (-0.5f < a[1]) && (a[1] < 0.5f);
  b[0] = 0.0f; b[1] = usey ? 1.0f : 0.0f; b[2] = usey ? 0.0f : 1.0f;
  float d = dot3(a, b);
  b[0] -= a[0] * d; b[1] -= a[1] * d; b[2] -= a[2] * d;
  normalize3(b);
  if (sqrtf(dot3(a, a)) == 0.0f) b[0] = b[1] = b[2] = 0.0f;
  cross3(c, a, b);
}

// math.py:246-257, rows = normal, tangent1, tangent2
__device__ __forceinline__ void make_frame(float* f, const float* ain) {
  float a[3] = {ain[0], ain[1], ain[2]}, b[3], c[3];
  normalize3(a);
  orthogonals(b, c, a);
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2];
  f[3] = b[0]; f[4] = b[1]; f[5] = b[2];
  f[6] = c[0]; f[7] = c[1]; f[8] = c[2];
}

__device__ __forceinline__ void matvec3(float* r, const float* M, const float* v) {
  float t0 = M[0] * v[0] + M[1] * v[1] + M[2] * v[2];
  float t1 = M[3] * v[0] + M[4] * v[1] + M[5] * v[2];
  float t2 = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}

// util_misc.py:59-73
__device__ __forceinline__ float halton(int index, int base) {
  int n0 = index;
  float b = (float)base, f = 1.0f / b, hn = 0.0f;
  while (n0 > 0) {
    int n1 = n0 / base;
    int r = n0 - n1 * base;
    hn += f * (float)r;
    f /= b;
    n0 = n1;
  }
  return hn;
}

}  // namespace mjw
