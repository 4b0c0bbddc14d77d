// mjw_kat.hip -- device replay of the reference's collision known-answer tests (no reference
// counterpart on the step path; tests/test_gpu_golden.py drives it through mjw_kat).
//
//   which = 0: ccd() of one convex pair exactly as collision_gjk_test.py:34-265 `_geom_dist` calls it
//              (cutoff 1e30, gjk and epa iterations = opt.ccd_iterations, both geoms carrying `margin`)
//              followed, when requested, by box multi-contact -- the same mjw_ccd.h device code the
//              convex pre-pass kernels run, one wavefront per case in lockstep over an LDS workspace.
//   which = 1: the flex triangle narrowphase (mjw_flexcol.h) of collision_primitive_core_test.py.
//
// Record layouts (floats; ints stored as values) are documented with KAT_* below and mirrored in
// tests/test_gpu_golden.py.
#include <hip/hip_runtime.h>

#include "mjw_amd.h"
#include "mjw_ccd.h"
#include "mjw_flexcol.h"

namespace mjw {

// which = 0 record: type1 type2 pos1[3] mat1[9] size1[3] pos2[3] mat2[9] size2[3] margin tolerance
//                   iterations multiccd vertadr1 nvert1 vertadr2 nvert2   (40 floats, padded to 48)
// out: ncon dist x1[3] x2[3]  (8 floats; ncon -1 = multi-contact request not built)
constexpr int KAT_CCD_IN = 48, KAT_CCD_OUT = 8;
// which = 1 record: type pos[3] rot[9] size[3] t[9] tri_radius  (26 floats, padded to 32)
// out: n, then 2 x (dist pos[3] normal[3])  (15 floats, padded to 16)
constexpr int KAT_TRI_IN = 32, KAT_TRI_OUT = 16;

__global__ void __launch_bounds__(64) kat_ccd_kernel(const float* in, const float* mesh_vert, float* out, int n) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int c = blockIdx.x, lane = (int)threadIdx.x;
  if (c >= n) return;
  const float* r = in + (long)c * KAT_CCD_IN;
  const int it = (int)r[34];
  CcdWS w;
  w.W = smem;
  w.L = ccd_layout(it);  // the launch's LDS holds the layout of the batch's largest count (max_it)
  const int t1 = (int)r[0], t2 = (int)r[1];
  put_cgeom(w.W + w.L.geoms, r + 2, r + 5, r + 14, t1, (int)r[36], (int)r[37]);
  put_cgeom(w.W + w.L.geoms + CGEOM_WORDS, r + 17, r + 20, r + 29, t2, (int)r[38], (int)r[39]);
  __syncthreads();
  CGeom g1 = get_cgeom(w.W + w.L.geoms, mesh_vert), g2 = get_cgeom(w.W + w.L.geoms + CGEOM_WORDS, mesh_vert);
  g1.margin = g2.margin = r[32];
  float d, x1[3], x2[3];
  int idx;
  int ncon = ccd_raw(w, it, r[33], it, 1e30f, g1, g2, &d, x1, x2, &idx);
  const bool multi = r[35] != 0.0f;
  if (multi && (t1 == GEOM_MESH || t2 == GEOM_MESH)) ncon = -1;
  else if (multi && idx > -1) ncon = multicontact_box(w, idx, x1, x2, g1, g2);
  float* o = out + (long)c * KAT_CCD_OUT;
  if (lane == 0) {
    o[0] = (float)ncon;
    o[1] = d;
    for (int i = 0; i < 3; i++) { o[2 + i] = x1[i]; o[5 + i] = x2[i]; }
  }
}

__global__ void kat_tri_kernel(const float* in, float* out, int n) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const float* r = in + (long)c * KAT_TRI_IN;
  const float* t[3] = {r + 16, r + 19, r + 22};
  sp::Cand cand[2];
  const int nc = sp::geom_triangle(cand, (int)r[0], r + 1, r + 4, r + 13, t, r[25]);
  float* o = out + (long)c * KAT_TRI_OUT;
  o[0] = (float)nc;
  for (int k = 0; k < 2; k++) {
    o[1 + 7 * k] = k < nc ? cand[k].dist : MJW_MAXVAL;
    for (int i = 0; i < 3; i++) {
      o[2 + 7 * k + i] = k < nc ? cand[k].pos[i] : 0.0f;
      o[5 + 7 * k + i] = k < nc ? cand[k].nrm[i] : 0.0f;
    }
  }
}

}  // namespace mjw

extern "C" int mjw_kat(int which, const float* in, const float* aux, float* out, int n, void* stream) {
  if (n <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (which == 0) {
    // the workspace is sized for the largest iteration count of the batch (host-checked: <= 64)
    int max_it = (int)aux[0];
    if (max_it <= 0 || max_it > 64) return (int)hipErrorInvalidValue;
    const size_t lds = (size_t)mjw::ccd_layout(max_it).total * 4;
    hipLaunchKernelGGL(mjw::kat_ccd_kernel, dim3(n), dim3(64), lds, s, in, aux + 1, out, n);
  } else if (which == 1) {
    hipLaunchKernelGGL(mjw::kat_tri_kernel, dim3((n + 63) / 64), dim3(64), 0, s, in, out, n);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}
