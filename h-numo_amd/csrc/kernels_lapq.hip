// kernels_lapq.hip -- method_visc == 1: the LDG viscosity evaluated at the quadrature points.
//
//   interpolate_dpp                 mod_layer_terms.F90:25-55           lapq_dpp_kernel
//   btp_create_laplacian_v2         mod_laplacian_quad.F90:125-223      lapq_flux_kernel (mode 0)
//   bcl_create_laplacian_v2         mod_laplacian_quad.F90:252-355      lapq_flux_kernel (mode 1)
//     compute_gradient_uv_q         mod_barotropic_terms.F90:445-477      (inside lapq_flux_kernel)
//     compute_laplacian_quad        mod_laplacian_quad.F90:613-642      lapq_apply_kernel
//     create_rhs_laplacian_flux_quad mod_laplacian_quad.F90:644-722       (inside lapq_apply_kernel)
//
// Not a shipped configuration (SURVEY.md §8a "conditional branches", f1), so these are plain
// per-element kernels launched around the fused stage kernel (which then takes the Laplacian
// from lapq_apply_kernel instead of its own nodal LDG) and around mom_elem_kernel; the
// persistent sub-cycle is not used on this branch.  Arithmetic is the reference's, in its
// order: the dense psih/dpsidx/dpsidy entries are regenerated from the 1-D bases with the
// products of Tensor_product.F90 (as in the stage kernel), every ordered sum is accumulated
// by one thread in the reference's loop order, and a node's face contributions arrive in
// face-id order, quad point by quad point.
#include "engine_internal.h"

namespace hnumo {

// dpprime_visc_q[k][Iq] = sum_ip dpprime_visc(I,k) * psih(ip,Iq), ip = mm*NGL + n in order
template <int NGL, int NQ>
__global__ void lapq_dpp_kernel(DevMesh m, const double *dpv, double *dpq) {
  constexpr int P = NGL * NGL, Q = NQ * NQ;
  const size_t npq = m.npoin_q, n = (size_t)m.L * npq, s = (size_t)gridDim.x * blockDim.x;
  const double *psiq = m.basis;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += s) {
    const int k = (int)(t / npq);
    const size_t Iq = t % npq;
    const int e = (int)(Iq / Q), q = (int)(Iq % Q), iq = q % NQ, jq = q / NQ;
    const double *d = dpv + (size_t)k * m.npoin + (size_t)e * P;
    double acc = 0.0;
    for (int mm = 0; mm < NGL; mm++)
#pragma unroll
      for (int nn = 0; nn < NGL; nn++) {
        const double hi = psiq[nn * NQ + iq] * psiq[mm * NQ + jq];
        acc = acc + d[mm * NGL + nn] * hi;
      }
    dpq[t] = acc;
  }
}

// LDG fluxes at the quad points of element e0 + blockIdx.x:
//   mode 0 (barotropic stage): flux[e][4][Q]  = sum_k dpq_k * grad(U_k),
//                              U_k = qprime(2:3,k) + qb(3:4)/qb(1)            (:142-153)
//   mode 1 (baroclinic):       flux[k][e][4][Q] = dpq_k * grad(U_k),
//                              U_k = qprime(2:3,k) + uvb_ave_df               (:272-282)
// grad = (du/dx, du/dy, dv/dx, dv/dy) = compute_gradient_uv_q's grad_uv(1,1), (1,2), (2,1), (2,2)
template <int NGL, int NQ>
__global__ void __launch_bounds__(256) lapq_flux_kernel(DevMesh m, const double *qb, const double *qp,
                                                        const double *nacc, const double *dpq, double *flux,
                                                        int mode, int e0) {
  constexpr int P = NGL * NGL, Q = NQ * NQ;
  const int e = e0 + blockIdx.x, tid = threadIdx.x, L = m.L, E = m.nelem;
  const size_t npoin = m.npoin, npq = m.npoin_q;
  __shared__ double s_psiq[NGL * NQ], s_dpsiq[NGL * NQ], s_u[MAXL][2][P];
  for (int t = tid; t < NGL * NQ; t += blockDim.x) {
    s_psiq[t] = m.basis[t];
    s_dpsiq[t] = m.basis[NGL * NQ + t];
  }
  for (int t = tid; t < L * P; t += blockDim.x) {
    const int k = t / P, p = t % P;
    const size_t I = (size_t)e * P + p, Ik = ((size_t)k * npoin + I) * 3;
    if (mode == 0) {
      s_u[k][0][p] = qp[Ik + 1] + qb[I * 4 + 2] / qb[I * 4];
      s_u[k][1][p] = qp[Ik + 2] + qb[I * 4 + 3] / qb[I * 4];
    } else {
      s_u[k][0][p] = qp[Ik + 1] + nacc[NACC_I(NA_UB, e, p)];
      s_u[k][1][p] = qp[Ik + 2] + nacc[NACC_I(NA_VB, e, p)];
    }
  }
  __syncthreads();
  for (int q = tid; q < Q; q += blockDim.x) {
    const int iq = q % NQ, jq = q / NQ;
    const size_t Iq = (size_t)e * Q + q;
    const double ex = m.qstat[QS_EX * npq + Iq], ey = m.qstat[QS_EY * npq + Iq];
    const double nx = m.qstat[QS_NX * npq + Iq], ny = m.qstat[QS_NY * npq + Iq];
    double f[4] = {0.0, 0.0, 0.0, 0.0};
    for (int k = 0; k < L; k++) {
      double g[4] = {0.0, 0.0, 0.0, 0.0};
      for (int mm = 0; mm < NGL; mm++)
#pragma unroll
        for (int nn = 0; nn < NGL; nn++) {
          const double h_e = s_dpsiq[nn * NQ + iq] * s_psiq[mm * NQ + jq];
          const double h_n = s_psiq[nn * NQ + iq] * s_dpsiq[mm * NQ + jq];
          const double dhdx = h_e * ex + h_n * nx, dhdy = h_e * ey + h_n * ny;
          const double u = s_u[k][0][mm * NGL + nn], v = s_u[k][1][mm * NGL + nn];
          g[0] = g[0] + dhdx * u;
          g[1] = g[1] + dhdy * u;
          g[2] = g[2] + dhdx * v;
          g[3] = g[3] + dhdy * v;
        }
      const double d = dpq[(size_t)k * npq + Iq];
      if (mode == 0) {
#pragma unroll
        for (int c = 0; c < 4; c++) f[c] = f[c] + d * g[c];
      } else {
#pragma unroll
        for (int c = 0; c < 4; c++) flux[(((size_t)k * E + e) * 4 + c) * Q + q] = d * g[c];
      }
    }
    if (mode == 0)
#pragma unroll
      for (int c = 0; c < 4; c++) flux[((size_t)e * 4 + c) * Q + q] = f[c];
  }
}

// Laplacian of layer blockIdx.y's fluxes at the nodes of element blockIdx.x, without the
// visc*massinv factor (the consumers apply it as the reference does):
//   lap(c,I) = - sum_Iq wq*(dpsidx*F(2c) + dpsidy*F(2c+1))        compute_laplacian_quad
//              +/- sum_faces sum_iq (wq_f*psiq(n,iq))*flux_c        create_rhs_laplacian_flux_quad
// with the face values of :156-212 (neighbour quad point, or the wall reflection) and the
// central flux beta = 0.5.  fqL/fqR [F][NQ]: element-local quad point of face quad point iq
// on the face's left / right element (imapl_q / imapr_q).
// recv (processor-face halo): the neighbours' side-1 fluxes of the shared faces, [NS][nb][4][NQ]
// (lapq_pack_kernel on the other rank), the processor face's side 2 (create_nbhs_face_quad,
// create_rhs_dynamics_flux.F90:61-100); NULL on a single rank.
template <int NGL, int NQ>
__global__ void __launch_bounds__(64) lapq_apply_kernel(DevMesh m, const double *flux, double *lap, const int *fqL,
                                                        const int *fqR, const double *recv) {
  constexpr int P = NGL * NGL, Q = NQ * NQ, ERS = EREC_SIZE(NGL);
  const int e = blockIdx.x, k = blockIdx.y, tid = threadIdx.x, E = m.nelem;
  const size_t npoin = m.npoin, npq = m.npoin_q, FQ = (size_t)m.nface * NQ;
  const double *fk = flux + (size_t)k * E * 4 * Q;
  __shared__ double s_psiq[NGL * NQ], s_dpsiq[NGL * NQ], s_f[4][Q], s_m[5][Q];
  __shared__ int s_er[ERS];
  for (int t = tid; t < NGL * NQ; t += 64) {
    s_psiq[t] = m.basis[t];
    s_dpsiq[t] = m.basis[NGL * NQ + t];
  }
  for (int t = tid; t < 4 * Q; t += 64) s_f[t / Q][t % Q] = fk[(size_t)e * 4 * Q + t];
  for (int t = tid; t < 5 * Q; t += 64) {
    const int c = t / Q;
    s_m[c][t % Q] = m.qstat[(c < 4 ? QS_EX + c : QS_W) * npq + (size_t)e * Q + t % Q];
  }
  for (int t = tid; t < ERS; t += 64) s_er[t] = m.erec[(size_t)e * ERS + t];
  __syncthreads();
  const double beta = 0.5, alpha = 1.0 - beta;
  for (int t = tid; t < 2 * P; t += 64) {
    const int c = t / P, p = t % P, i = p % NGL, j = p / NGL;
    double acc = 0.0;
    for (int q = 0; q < Q; q++) {
      const int iq = q % NQ, jq = q / NQ;
      const double h_e = s_dpsiq[i * NQ + iq] * s_psiq[j * NQ + jq];
      const double h_n = s_psiq[i * NQ + iq] * s_dpsiq[j * NQ + jq];
      const double dhdx = h_e * s_m[0][q] + h_n * s_m[2][q], dhdy = h_e * s_m[1][q] + h_n * s_m[3][q];
      const double uv = dhdx * s_f[2 * c][q] + dhdy * s_f[2 * c + 1][q];
      acc = acc - s_m[4][q] * uv;
    }
#pragma unroll
    for (int kf = 0; kf < 2; kf++) {
      const int r = s_er[EREC_PF(NGL) + 2 * p + kf];
      if (r < 0) continue;
      const int lf = r / NGL, n = r % NGL;
      const int f = s_er[EREC_FACE + lf], side = s_er[EREC_SIDE + lf], er = s_er[EREC_BC + lf];
      const int nb = s_er[EREC_NBE + lf];
      for (int iq = 0; iq < NQ; iq++) {
        const size_t fq = (size_t)f * NQ + iq;
        const int qo = side == 0 ? fqL[fq] : fqR[fq];
        double own[4], oth[4];
#pragma unroll
        for (int v = 0; v < 4; v++) own[v] = s_f[v][qo];
        const double nx = m.fstat[FS_NX * FQ + fq], ny = m.fstat[FS_NY * FQ + fq], wq = m.fstat[FS_W * FQ + fq];
        if (er > 0) {
          const int qn = side == 0 ? fqR[fq] : fqL[fq];
#pragma unroll
          for (int v = 0; v < 4; v++) oth[v] = fk[((size_t)nb * 4 + v) * Q + qn];
        } else if (er == 0 && recv) {
          // processor face (the local element is its left side): shared slot (nb - E)*4 + nblf
          const size_t sl = (size_t)(nb - E) * 4 + s_er[EREC_NBLF + lf];
#pragma unroll
          for (int v = 0; v < 4; v++) oth[v] = recv[((sl * gridDim.y + k) * 4 + v) * NQ + iq];
        } else {
#pragma unroll
          for (int v = 0; v < 4; v++) oth[v] = own[v];
          if (er == -4) {
            double un = own[0] * nx + own[1] * ny;
            oth[0] = own[0] - 2.0 * un * nx;
            oth[1] = own[1] - 2.0 * un * ny;
            un = own[2] * nx + own[3] * ny;
            oth[2] = own[2] - 2.0 * un * nx;
            oth[3] = own[3] - 2.0 * un * ny;
          }
        }
        const double *l = side == 0 ? own : oth, *rr = side == 0 ? oth : own;
        const double mean0 = alpha * l[2 * c] + beta * rr[2 * c];
        const double mean1 = alpha * l[2 * c + 1] + beta * rr[2 * c + 1];
        const double fl = (mean0 - l[2 * c] * nx) + (mean1 - l[2 * c + 1] * ny);
        const double w = wq * s_psiq[n * NQ + iq];
        acc = side == 0 ? acc + w * fl : acc - w * fl;
      }
    }
    lap[((size_t)k * 2 + c) * npoin + (size_t)e * P + p] = acc;
  }
}

// Processor-face message of the LDG fluxes (pack_data_dg_quad, send_receive_bound.F90:215-270):
// buf[s][k][v][iq] = flux of layer block k, component v at the quad point of face sface[s]'s
// side 1 (its left, local element) that face quad point iq maps to (imapl_q)
__global__ void lapq_pack_kernel(double *buf, const double *flux, const int *sface, const int *fel, const int *fqL,
                                 int NS, int nb, int E, int NQ, int Q) {
  const size_t n = (size_t)NS * nb * 4 * NQ, st = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += st) {
    const int iq = (int)(t % NQ), v = (int)((t / NQ) % 4), k = (int)((t / (4 * (size_t)NQ)) % nb);
    const int s = (int)(t / (4 * (size_t)NQ * nb)), f = sface[s];
    buf[t] = flux[(((size_t)k * E + fel[f]) * 4 + v) * Q + fqL[(size_t)f * NQ + iq]];
  }
}

}  // namespace hnumo
