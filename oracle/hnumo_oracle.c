/*
 * hnumo_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's baroclinic/barotropic time step (ti_rk_bcl and
 * everything below it) used as the parity checker for the HIP engine and as the
 * "port" CPU baseline in bench.py.  It is never linked into, loaded by or called from
 * the product path (h-numo_amd/csrc); only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it.
 *
 * It follows the reference Fortran loop for loop and operation for operation, on the
 * same dense per-quad-point tables (psih, dpsidx, dpsidy, indexq, wjac and their nodal
 * twins, Tensor_product.F90:1-128), so that with -O2 -ffp-contract=off it reproduces
 * the reference's arithmetic bitwise.  Pinning: tests/test_oracle.py compares it against
 * the reference Fortran itself (oracle/_ref/ref_driver, built from /root/reference/src by
 * oracle/build_ref.sh; the -m ref tests) and against the committed golden vectors in
 * tests/golden/ (made by tests/golden/make_golden.py from the reference's own outputs).
 *
 * Each function cites the reference routine it restates.  Arrays use the reference's
 * Fortran layouts; the A*() macros index them 1-based exactly as the Fortran does.
 *
 * method_visc == 1 (quad-point LDG viscosity, mod_laplacian_quad.F90:125-223,252-355) is
 * restated below, and so is ad_mlswe > 0 (the implicit vertical shear stress,
 * mod_create_rhs_mlswe.F90:146-279, in momentum_mass / momentum): the reference reads two
 * never-assigned arrays there, tau_u(nlayers+1) (:246-247) and, in the corrector, uv
 * (mod_splitting.F90:158); both are taken as zero, as the reference build's -finit-real=zero
 * makes them, and the predictor is pinned bit for bit against the reference Fortran run with
 * oracle/zero_init_wrap.c (tests/test_oracle.py, fixtures *_predict).  Single rank only: the
 * multi-rank reference runs are the reference Fortran itself under mpiexec.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/hnumo_engine.h"

#define A2(a, i, j, n1) (a)[((size_t)(j)-1) * (size_t)(n1) + (size_t)(i)-1]
#define A3(a, i, j, k, n1, n2) \
  (a)[(((size_t)(k)-1) * (size_t)(n2) + (size_t)(j)-1) * (size_t)(n1) + (size_t)(i)-1]
#define A4(a, i, j, k, l, n1, n2, n3)                                                   \
  (a)[((((size_t)(l)-1) * (size_t)(n3) + (size_t)(k)-1) * (size_t)(n2) + (size_t)(j)-1) * \
          (size_t)(n1) +                                                                \
      (size_t)(i)-1]
#define A5(a, i, j, k, l, m, n1, n2, n3, n4)                                             \
  (a)[(((((size_t)(m)-1) * (size_t)(n4) + (size_t)(l)-1) * (size_t)(n3) + (size_t)(k)-1) * \
           (size_t)(n2) +                                                                \
       (size_t)(j)-1) *                                                                  \
          (size_t)(n1) +                                                                 \
      (size_t)(i)-1]

typedef struct oracle {
  hnumo_mesh_desc m;
  hnumo_static_desc s;
  hnumo_params p;
  int ngl, nq, npts, npoin, npoin_q, nface, nelem, L;
  char err[256];
  /* mod_variables (mod_variables.F90:26-47) */
  double *Q_uu_dp, *Q_uv_dp, *Q_vv_dp, *H_bcl;                      /* npoin_q     */
  double *Q_uu_dp_edge, *Q_uv_dp_edge, *Q_vv_dp_edge, *H_bcl_edge;  /* nq,nface    */
  double *ope_ave, *H_ave, *Qu_ave, *Qv_ave, *Quv_ave, *ope2_ave;   /* npoin_q     */
  double *btp_mass_flux_ave, *uvb_ave, *tau_bot_ave, *tau_wind_ave; /* 2,npoin_q   */
  double *ope2_ave_df;                                              /* npoin       */
  double *uvb_ave_df;                                               /* 2,npoin     */
  double *uvb_face_ave;                                             /* 2,2,nq,nface*/
  double *btp_mass_flux_face_ave, *ope_face_ave, *ope2_face_ave;    /* 2,nq,nface  */
  double *Qu_face_ave, *Qv_face_ave, *Quv_face_ave;                 /* 2,nq,nface  */
  double *H_face_ave, *one_plus_eta_edge_2_ave;                     /* nq,nface    */
  double *dpprime_visc;                                             /* npoin,L     */
  double *dpprime_visc_q;                                           /* npoin_q,L   */
  double *pbprime_visc;                                             /* npoin       */
  double *btp_dpp_graduv;                                           /* 4,npoin     */
  double *dpp_graduv;                                               /* 4,npoin,L   */
  double *graduv_dpp_face;                                          /* 5,2,ngl,nface,L */
  double *btp_graduv_dpp_face;                                      /* 5,2,ngl,nface   */
  double *graduvb_face_ave;                                         /* 4,2,ngl,nface   */
  double *graduvb_ave;                                              /* 4,npoin     */
  double *sum_layer_mass_flux;                                      /* 2,npoin_q   */
  double *sum_layer_mass_flux_face;                                 /* 2,nq,nface  */
} oracle;

static double *zalloc(size_t n) { return (double *)calloc(n ? n : 1, sizeof(double)); }

/* intma_dg (mod_grid.F90:230-239) for nglz = 1 */
static inline int INTMA(const oracle *o, int i, int j, int e) {
  return (e - 1) * o->npts + (j - 1) * o->ngl + i;
}

static int set_err(oracle *o, int code, const char *msg) {
  snprintf(o->err, sizeof o->err, "%s", msg);
  return code;
}

/* ------------------------------------------------------------------------------ */
/* btp_extract_df (mod_barotropic_terms.F90:25-97)                                 */
static void btp_extract_df(oracle *o, double *qbf, const double *qb) {
  const int ngl = o->ngl, nface = o->nface;
  memset(qbf, 0, sizeof(double) * 8 * ngl * nface);
  for (int f = 1; f <= nface; f++) {
    int el = A2(o->m.face, 7, f, 8), er = A2(o->m.face, 8, f, 8);
    for (int n = 1; n <= ngl; n++) {
      int I = INTMA(o, A3(o->m.imapl, 1, n, f, 3, ngl), A3(o->m.imapl, 2, n, f, 3, ngl), el);
      for (int v = 1; v <= 4; v++) A4(qbf, v, 1, n, f, 4, 2, ngl) = A2(qb, v, I, 4);
      if (er > 0) {
        int Ir = INTMA(o, A3(o->m.imapr, 1, n, f, 3, ngl), A3(o->m.imapr, 2, n, f, 3, ngl), er);
        for (int v = 1; v <= 4; v++) A4(qbf, v, 2, n, f, 4, 2, ngl) = A2(qb, v, Ir, 4);
      } else {
        for (int v = 1; v <= 4; v++) A4(qbf, v, 2, n, f, 4, 2, ngl) = A4(qbf, v, 1, n, f, 4, 2, ngl);
        if (er == -4) {
          double nx = A3(o->m.normal_vector, 1, n, f, 3, ngl);
          double ny = A3(o->m.normal_vector, 2, n, f, 3, ngl);
          double un = nx * A4(qbf, 3, 1, n, f, 4, 2, ngl) + ny * A4(qbf, 4, 1, n, f, 4, 2, ngl);
          A4(qbf, 3, 2, n, f, 4, 2, ngl) = A4(qbf, 3, 1, n, f, 4, 2, ngl) - 2.0 * un * nx;
          A4(qbf, 4, 2, n, f, 4, 2, ngl) = A4(qbf, 4, 1, n, f, 4, 2, ngl) - 2.0 * un * ny;
        } else if (er == -2) {
          A4(qbf, 3, 2, n, f, 4, 2, ngl) = -A4(qbf, 3, 1, n, f, 4, 2, ngl);
          A4(qbf, 4, 2, n, f, 4, 2, ngl) = -A4(qbf, 4, 1, n, f, 4, 2, ngl);
        }
      }
    }
  }
}

/* create_rhs_btp_volume_qdf (mod_rhs_btp.F90:102-209) */
static void btp_volume(oracle *o, double *rhs, const double *qb, const double *qp) {
  const int npts = o->npts, npoin = o->npoin, L = o->L;
  const hnumo_mesh_desc *m = &o->m;
  const hnumo_static_desc *s = &o->s;
  const double g = o->p.gravity, cd = o->p.cd_mlswe;
  memset(rhs, 0, sizeof(double) * 3 * npoin);
  double tb_u = 0.0, tb_v = 0.0;
  for (int Iq = 1; Iq <= o->npoin_q; Iq++) {
    double dp = 0, dpp = 0, udp = 0, vdp = 0, pp = 0, up = 0, vp = 0;
    for (int ip = 1; ip <= npts; ip++) {
      int I = A2(m->indexq, ip, Iq, npts);
      double hi = A2(m->psih, ip, Iq, npts);
      dp = dp + hi * A2(qb, 1, I, 4);
      dpp = dpp + hi * A2(qb, 2, I, 4);
      udp = udp + hi * A2(qb, 3, I, 4);
      vdp = vdp + hi * A2(qb, 4, I, 4);
      pp = pp + hi * A3(qp, 1, I, L, 3, npoin);
      up = up + hi * A3(qp, 2, I, L, 3, npoin);
      vp = vp + hi * A3(qp, 3, I, L, 3, npoin);
    }
    double wq = m->wjac[Iq - 1];
    double ub = udp / dp, vb = vdp / dp;
    if (o->p.botfr == 1) {
      double ubot = up + ub, vbot = vp + vb;
      double spd = (cd / g) * pp;
      tb_u = spd * ubot;
      tb_v = spd * vbot;
    } else if (o->p.botfr == 2) {
      double ubot = up + ub, vbot = vp + vb;
      double spd = (cd / s->alpha[L - 1]) * sqrt(ubot * ubot + vbot * vbot);
      tb_u = spd * ubot;
      tb_v = spd * vbot;
    }
    double cor = s->coriolis_quad[Iq - 1];
    double sc_x = cor * vdp + g * (A2(s->tau_wind, 1, Iq, 2) - tb_u) - g * dp * A2(s->grad_zbot_quad, 1, Iq, 2);
    double sc_y = -cor * udp + g * (A2(s->tau_wind, 2, Iq, 2) - tb_v) - g * dp * A2(s->grad_zbot_quad, 2, Iq, 2);
    double ope = 1.0 + dpp * s->one_over_pbprime[Iq - 1];
    double Hq = (ope * ope) * o->H_bcl[Iq - 1];
    double qu = ub * udp + ope * o->Q_uu_dp[Iq - 1];
    double quv = ub * vdp + ope * o->Q_uv_dp[Iq - 1];
    double qv = vb * vdp + ope * o->Q_vv_dp[Iq - 1];
    o->H_ave[Iq - 1] += Hq;
    o->Qu_ave[Iq - 1] += qu;
    o->Qv_ave[Iq - 1] += qv;
    o->Quv_ave[Iq - 1] += quv;
    A2(o->tau_bot_ave, 1, Iq, 2) += tb_u;
    A2(o->tau_bot_ave, 2, Iq, 2) += tb_v;
    o->ope_ave[Iq - 1] += ope;
    o->ope2_ave[Iq - 1] += ope * ope;
    A2(o->btp_mass_flux_ave, 1, Iq, 2) += udp;
    A2(o->btp_mass_flux_ave, 2, Iq, 2) += vdp;
    A2(o->uvb_ave, 1, Iq, 2) += ub;
    A2(o->uvb_ave, 2, Iq, 2) += vb;
    for (int ip = 1; ip <= npts; ip++) {
      int I = A2(m->indexq, ip, Iq, npts);
      double hi = A2(m->psih, ip, Iq, npts);
      double dhdx = A2(m->dpsidx, ip, Iq, npts);
      double dhdy = A2(m->dpsidy, ip, Iq, npts);
      A2(rhs, 1, I, 3) = A2(rhs, 1, I, 3) + wq * (dhdx * udp + dhdy * vdp);
      A2(rhs, 2, I, 3) = A2(rhs, 2, I, 3) + wq * (hi * sc_x + dhdx * (Hq + qu) + quv * dhdy);
      A2(rhs, 3, I, 3) = A2(rhs, 3, I, 3) + wq * (hi * sc_y + dhdx * quv + dhdy * (Hq + qv));
    }
  }
}

/* creat_btp_fluxes_qdf (mod_rhs_btp.F90:211-370) */
static void btp_fluxes(oracle *o, double *rhs, const double *qbf) {
  const int ngl = o->ngl, nq = o->nq, nface = o->nface;
  const hnumo_mesh_desc *m = &o->m;
  const hnumo_static_desc *s = &o->s;
  double qbl[4][32], qbr[4][32], pbl[32], pbr[32], ope_e[32], fex[32], fey[32];
  double ul[32], ur[32], vl[32], vr[32], quu[32], quv[32], qvu[32], qvv[32], Hf[32];
  for (int f = 1; f <= nface; f++) {
    int el = A2(m->face, 7, f, 8), er = A2(m->face, 8, f, 8);
    for (int iq = 0; iq < nq; iq++) {
      for (int v = 0; v < 4; v++) qbl[v][iq] = qbr[v][iq] = 0.0;
      pbl[iq] = pbr[iq] = 0.0;
    }
    for (int iq = 1; iq <= nq; iq++) {
      double nxl = A3(m->normal_vector_q, 1, iq, f, 3, nq);
      double nyl = A3(m->normal_vector_q, 2, iq, f, 3, nq);
      double nxr = -nxl, nyr = -nyl;
      for (int n = 1; n <= ngl; n++) {
        double hi = A2(m->psiq, n, iq, ngl);
        for (int v = 1; v <= 4; v++) {
          qbl[v - 1][iq - 1] = qbl[v - 1][iq - 1] + hi * A4(qbf, v, 1, n, f, 4, 2, ngl);
          qbr[v - 1][iq - 1] = qbr[v - 1][iq - 1] + hi * A4(qbf, v, 2, n, f, 4, 2, ngl);
        }
        pbl[iq - 1] = pbl[iq - 1] + hi * A3(s->pbprime_df_face, 1, n, f, 2, ngl);
        pbr[iq - 1] = pbr[iq - 1] + hi * A3(s->pbprime_df_face, 2, n, f, 2, ngl);
      }
      double pU_L = nxl * qbl[2][iq - 1] + nyl * qbl[3][iq - 1];
      double pU_R = nxr * qbr[2][iq - 1] + nyr * qbr[3][iq - 1];
      double pbpert_edge = A2(s->coeff_pbpert_L, iq, f, nq) * qbl[1][iq - 1] +
                           A2(s->coeff_pbpert_R, iq, f, nq) * qbr[1][iq - 1] +
                           A2(s->coeff_pbub_LR, iq, f, nq) * (pU_L + pU_R);
      ope_e[iq - 1] = 1.0 + pbpert_edge * A2(s->one_over_pbprime_edge, iq, f, nq);
      fex[iq - 1] = A2(s->coeff_mass_pbub_L, iq, f, nq) * qbl[2][iq - 1] +
                    A2(s->coeff_mass_pbub_R, iq, f, nq) * qbr[2][iq - 1] +
                    A2(s->coeff_mass_pbpert_LR, iq, f, nq) * (nxl * qbl[1][iq - 1] + nxr * qbr[1][iq - 1]);
      fey[iq - 1] = A2(s->coeff_mass_pbub_L, iq, f, nq) * qbl[3][iq - 1] +
                    A2(s->coeff_mass_pbub_R, iq, f, nq) * qbr[3][iq - 1] +
                    A2(s->coeff_mass_pbpert_LR, iq, f, nq) * (nyl * qbl[1][iq - 1] + nyr * qbr[1][iq - 1]);
    }
    for (int i = 0; i < nq; i++) {
      ul[i] = qbl[2][i] / qbl[0][i];
      ur[i] = qbr[2][i] / qbr[0][i];
      vl[i] = qbl[3][i] / qbl[0][i];
      vr[i] = qbr[3][i] / qbr[0][i];
    }
    for (int i = 0; i < nq; i++) {
      int iq = i + 1;
      quu[i] = 0.5 * (ul[i] * qbl[2][i] + ur[i] * qbr[2][i]) + ope_e[i] * A2(o->Q_uu_dp_edge, iq, f, nq);
      quv[i] = 0.5 * (vl[i] * qbl[2][i] + vr[i] * qbr[2][i]) + ope_e[i] * A2(o->Q_uv_dp_edge, iq, f, nq);
      qvu[i] = 0.5 * (ul[i] * qbl[3][i] + ur[i] * qbr[3][i]) + ope_e[i] * A2(o->Q_uv_dp_edge, iq, f, nq);
      qvv[i] = 0.5 * (vl[i] * qbl[3][i] + vr[i] * qbr[3][i]) + ope_e[i] * A2(o->Q_vv_dp_edge, iq, f, nq);
      Hf[i] = (ope_e[i] * ope_e[i]) * A2(o->H_bcl_edge, iq, f, nq);
    }
    for (int i = 0; i < nq; i++) {
      int iq = i + 1;
      A3(o->btp_mass_flux_face_ave, 1, iq, f, 2, nq) += fex[i];
      A3(o->btp_mass_flux_face_ave, 2, iq, f, 2, nq) += fey[i];
      A2(o->H_face_ave, iq, f, nq) += Hf[i];
      A3(o->Qu_face_ave, 1, iq, f, 2, nq) += quu[i];
      A3(o->Qu_face_ave, 2, iq, f, 2, nq) += quv[i];
      A3(o->Qv_face_ave, 1, iq, f, 2, nq) += qvu[i];
      A3(o->Qv_face_ave, 2, iq, f, 2, nq) += qvv[i];
      double opl = 1.0 + (qbl[1][i] / pbl[i]);
      double opr = 1.0 + (qbr[1][i] / pbr[i]);
      A3(o->ope_face_ave, 1, iq, f, 2, nq) += opl;
      A3(o->ope_face_ave, 2, iq, f, 2, nq) += opr;
      A3(o->ope2_face_ave, 1, iq, f, 2, nq) += opl * opl;
      A3(o->ope2_face_ave, 2, iq, f, 2, nq) += opr * opr;
      A2(o->one_plus_eta_edge_2_ave, iq, f, nq) += ope_e[i] * ope_e[i];
      A4(o->uvb_face_ave, 1, 1, iq, f, 2, 2, nq) += ul[i];
      A4(o->uvb_face_ave, 1, 2, iq, f, 2, 2, nq) += ur[i];
      A4(o->uvb_face_ave, 2, 1, iq, f, 2, 2, nq) += vl[i];
      A4(o->uvb_face_ave, 2, 2, iq, f, 2, 2, nq) += vr[i];
    }
    for (int iq = 1; iq <= nq; iq++) {
      double wq = A2(m->jac_faceq, iq, f, nq);
      double nxl = A3(m->normal_vector_q, 1, iq, f, 3, nq);
      double nyl = A3(m->normal_vector_q, 2, iq, f, 3, nq);
      double H_kx = nxl * Hf[iq - 1], H_ky = nyl * Hf[iq - 1];
      double lamb = A2(s->coeff_mass_pbpert_LR, iq, f, nq);
      double dispu = 0.5 * lamb * (qbr[2][iq - 1] - qbl[2][iq - 1]);
      double dispv = 0.5 * lamb * (qbr[3][iq - 1] - qbl[3][iq - 1]);
      double flux_x = nxl * quu[iq - 1] + nyl * quv[iq - 1] - dispu;
      double flux_y = nxl * qvu[iq - 1] + nyl * qvv[iq - 1] - dispv;
      double flux = nxl * fex[iq - 1] + nyl * fey[iq - 1];
      for (int n = 1; n <= ngl; n++) {
        double hi = A2(m->psiq, n, iq, ngl);
        int I = INTMA(o, A3(m->imapl, 1, n, f, 3, ngl), A3(m->imapl, 2, n, f, 3, ngl), el);
        A2(rhs, 1, I, 3) = A2(rhs, 1, I, 3) - wq * hi * flux;
        A2(rhs, 2, I, 3) = A2(rhs, 2, I, 3) - wq * hi * (H_kx + flux_x);
        A2(rhs, 3, I, 3) = A2(rhs, 3, I, 3) - wq * hi * (H_ky + flux_y);
        if (er > 0) {
          I = INTMA(o, A3(m->imapr, 1, n, f, 3, ngl), A3(m->imapr, 2, n, f, 3, ngl), er);
          A2(rhs, 1, I, 3) = A2(rhs, 1, I, 3) + wq * hi * flux;
          A2(rhs, 2, I, 3) = A2(rhs, 2, I, 3) + wq * hi * (H_kx + flux_x);
          A2(rhs, 3, I, 3) = A2(rhs, 3, I, 3) + wq * hi * (H_ky + flux_y);
        }
      }
    }
  }
  for (int I = 1; I <= o->npoin; I++) {
    double mi = m->massinv[I - 1];
    A2(rhs, 1, I, 3) = mi * A2(rhs, 1, I, 3);
    A2(rhs, 2, I, 3) = mi * A2(rhs, 2, I, 3);
    A2(rhs, 3, I, 3) = mi * A2(rhs, 3, I, 3);
  }
}

/* compute_gradient_uv (mod_barotropic_terms.F90:411-443); uv(ldu, npoin) with the two
 * components at rows off1, off2 (1-based) so that sections like qprime_df(2:3,:,k) work. */
static void compute_gradient_uv(oracle *o, double *grad, const double *uv, int ldu) {
  const int npts = o->npts;
  memset(grad, 0, sizeof(double) * 4 * o->npoin);
  for (int Iq = 1; Iq <= o->npoin; Iq++) {
    for (int ip = 1; ip <= npts; ip++) {
      int I = A2(o->m.index_df, ip, Iq, npts);
      double dhdx = A2(o->m.dpsidx_df, ip, Iq, npts);
      double dhdy = A2(o->m.dpsidy_df, ip, Iq, npts);
      double u = uv[(size_t)(I - 1) * ldu + 0], v = uv[(size_t)(I - 1) * ldu + 1];
      A2(grad, 1, Iq, 4) = A2(grad, 1, Iq, 4) + dhdx * u;
      A2(grad, 2, Iq, 4) = A2(grad, 2, Iq, 4) + dhdy * u;
      A2(grad, 3, Iq, 4) = A2(grad, 3, Iq, 4) + dhdx * v;
      A2(grad, 4, Iq, 4) = A2(grad, 4, Iq, 4) + dhdy * v;
    }
  }
}

/* LDG face flux (create_rhs_laplacian_flux mod_laplacian_quad.F90:427-519 and
 * bcl_create_rhs_laplacian_flux :521-611): flux_visc = c5 * gradq + c(ivar).         */
static void ldg_flux(oracle *o, double *rhs, const double *gradq_face, const double *coef_face) {
  const int ngl = o->ngl, nface = o->nface;
  const hnumo_mesh_desc *m = &o->m;
  const double beta = 0.5, alpha = 1.0 - beta;
  for (int f = 1; f <= nface; f++) {
    int iel = A2(m->face, 7, f, 8), ier = A2(m->face, 8, f, 8);
    for (int iq = 1; iq <= ngl; iq++) {
      double fv[4][2];
      for (int iv = 1; iv <= 4; iv++) {
        fv[iv - 1][0] = A4(coef_face, 5, 1, iq, f, 5, 2, ngl) * A4(gradq_face, iv, 1, iq, f, 4, 2, ngl) +
                        A4(coef_face, iv, 1, iq, f, 5, 2, ngl);
        fv[iv - 1][1] = A4(coef_face, 5, 2, iq, f, 5, 2, ngl) * A4(gradq_face, iv, 2, iq, f, 4, 2, ngl) +
                        A4(coef_face, iv, 2, iq, f, 5, 2, ngl);
      }
      double nx = A3(m->normal_vector, 1, iq, f, 3, ngl);
      double ny = A3(m->normal_vector, 2, iq, f, 3, ngl);
      double qul0 = fv[0][0], qul1 = fv[1][0], qvl0 = fv[2][0], qvl1 = fv[3][0];
      double qur0 = fv[0][1], qur1 = fv[1][1], qvr0 = fv[2][1], qvr1 = fv[3][1];
      double qum0 = alpha * qul0 + beta * qur0, qum1 = alpha * qul1 + beta * qur1;
      double qvm0 = alpha * qvl0 + beta * qvr0, qvm1 = alpha * qvl1 + beta * qvr1;
      double wq = A2(m->jac_face, iq, f, ngl);
      double flux_qu = (qum0 - qul0 * nx) + (qum1 - qul1 * ny);
      double flux_qv = (qvm0 - qvl0 * nx) + (qvm1 - qvl1 * ny);
      for (int i = 1; i <= ngl; i++) {
        double hi = A2(m->psi, i, iq, ngl);
        int ip = INTMA(o, A3(m->imapl, 1, i, f, 3, ngl), A3(m->imapl, 2, i, f, 3, ngl), iel);
        A2(rhs, 1, ip, 2) = A2(rhs, 1, ip, 2) + wq * hi * flux_qu;
        A2(rhs, 2, ip, 2) = A2(rhs, 2, ip, 2) + wq * hi * flux_qv;
        if (ier > 0) {
          ip = INTMA(o, A3(m->imapr, 1, i, f, 3, ngl), A3(m->imapr, 2, i, f, 3, ngl), ier);
          A2(rhs, 1, ip, 2) = A2(rhs, 1, ip, 2) - wq * hi * flux_qu;
          A2(rhs, 2, ip, 2) = A2(rhs, 2, ip, 2) - wq * hi * flux_qv;
        }
      }
    }
  }
}

/* Nodal LDG volume term (btp_compute_laplacian :357-390 / bcl_compute_laplacian :392-425):
 * qq = c(I) * grad(:,I) + d(:,I). */
static void ldg_volume(oracle *o, double *lap, const double *c, const double *grad, const double *d) {
  const int npts = o->npts;
  memset(lap, 0, sizeof(double) * 2 * o->npoin);
  for (int Iq = 1; Iq <= o->npoin; Iq++) {
    double wq = o->m.wjac_df[Iq - 1];
    double qq[4];
    for (int v = 1; v <= 4; v++) qq[v - 1] = c[Iq - 1] * A2(grad, v, Iq, 4) + A2(d, v, Iq, 4);
    for (int ip = 1; ip <= npts; ip++) {
      int I = A2(o->m.index_df, ip, Iq, npts);
      double dx = A2(o->m.dpsidx_df, ip, Iq, npts), dy = A2(o->m.dpsidy_df, ip, Iq, npts);
      A2(lap, 1, I, 2) = A2(lap, 1, I, 2) - wq * (dx * qq[0] + dy * qq[1]);
      A2(lap, 2, I, 2) = A2(lap, 2, I, 2) - wq * (dx * qq[2] + dy * qq[3]);
    }
  }
}

/* btp_create_laplacian (mod_laplacian_quad.F90:32-121) */
static void btp_create_laplacian(oracle *o, double *rhs_lap, const double *qb) {
  const int npoin = o->npoin, ngl = o->ngl, nface = o->nface;
  const hnumo_mesh_desc *m = &o->m;
  double *Uk = zalloc(2 * (size_t)npoin), *graduv = zalloc(4 * (size_t)npoin);
  double *gf = zalloc(4 * 2 * (size_t)ngl * nface);
  for (int I = 1; I <= npoin; I++) {
    A2(Uk, 1, I, 2) = A2(qb, 3, I, 4) / A2(qb, 1, I, 4);
    A2(Uk, 2, I, 2) = A2(qb, 4, I, 4) / A2(qb, 1, I, 4);
  }
  compute_gradient_uv(o, graduv, Uk, 2);
  for (size_t i = 0; i < 4 * (size_t)npoin; i++) o->graduvb_ave[i] = o->graduvb_ave[i] + graduv[i];
  for (int f = 1; f <= nface; f++) {
    int iel = A2(m->face, 7, f, 8), ier = A2(m->face, 8, f, 8);
    for (int iq = 1; iq <= ngl; iq++) {
      int Iq = INTMA(o, A3(m->imapl, 1, iq, f, 3, ngl), A3(m->imapl, 2, iq, f, 3, ngl), iel);
      for (int v = 1; v <= 4; v++) A4(gf, v, 1, iq, f, 4, 2, ngl) = A2(graduv, v, Iq, 4);
      if (ier > 0) {
        Iq = INTMA(o, A3(m->imapr, 1, iq, f, 3, ngl), A3(m->imapr, 2, iq, f, 3, ngl), ier);
        for (int v = 1; v <= 4; v++) A4(gf, v, 2, iq, f, 4, 2, ngl) = A2(graduv, v, Iq, 4);
      } else {
        for (int v = 1; v <= 4; v++) A4(gf, v, 2, iq, f, 4, 2, ngl) = A4(gf, v, 1, iq, f, 4, 2, ngl);
        if (ier == -4) {
          double nx = A3(m->normal_vector, 1, iq, f, 3, ngl), ny = A3(m->normal_vector, 2, iq, f, 3, ngl);
          double un = A4(gf, 1, 1, iq, f, 4, 2, ngl) * nx + A4(gf, 2, 1, iq, f, 4, 2, ngl) * ny;
          A4(gf, 1, 2, iq, f, 4, 2, ngl) = A4(gf, 1, 1, iq, f, 4, 2, ngl) - 2.0 * un * nx;
          A4(gf, 2, 2, iq, f, 4, 2, ngl) = A4(gf, 2, 1, iq, f, 4, 2, ngl) - 2.0 * un * ny;
          un = A4(gf, 3, 1, iq, f, 4, 2, ngl) * nx + A4(gf, 4, 1, iq, f, 4, 2, ngl) * ny;
          A4(gf, 3, 2, iq, f, 4, 2, ngl) = A4(gf, 3, 1, iq, f, 4, 2, ngl) - 2.0 * un * nx;
          A4(gf, 4, 2, iq, f, 4, 2, ngl) = A4(gf, 4, 1, iq, f, 4, 2, ngl) - 2.0 * un * ny;
        }
      }
    }
  }
  ldg_volume(o, rhs_lap, o->pbprime_visc, graduv, o->btp_dpp_graduv);
  for (size_t i = 0; i < 8 * (size_t)ngl * nface; i++) o->graduvb_face_ave[i] = o->graduvb_face_ave[i] + gf[i];
  ldg_flux(o, rhs_lap, gf, o->btp_graduv_dpp_face);
  for (int I = 1; I <= npoin; I++) {
    A2(rhs_lap, 1, I, 2) = o->p.visc_mlswe * m->massinv[I - 1] * A2(rhs_lap, 1, I, 2);
    A2(rhs_lap, 2, I, 2) = o->p.visc_mlswe * m->massinv[I - 1] * A2(rhs_lap, 2, I, 2);
  }
  free(Uk);
  free(graduv);
  free(gf);
}

/* ---------------------------------------------- method_visc == 1: quad-point LDG */

/* intma_dg_quad (mod_grid.F90:242-250) */
static inline int INTMA_Q(const oracle *o, int i, int j, int e) { return (e - 1) * o->nq * o->nq + (j - 1) * o->nq + i; }

/* interpolate_dpp (mod_layer_terms.F90:25-55): dprimeq(Iq,:) += dprime_df(I,:)*hi */
static void interpolate_dpp(oracle *o) {
  const int npts = o->npts, npoin = o->npoin, npq = o->npoin_q, L = o->L;
  memset(o->dpprime_visc_q, 0, sizeof(double) * (size_t)npq * L);
  for (int Iq = 1; Iq <= npq; Iq++)
    for (int ip = 1; ip <= npts; ip++) {
      int I = A2(o->m.indexq, ip, Iq, npts);
      double hi = A2(o->m.psih, ip, Iq, npts);
      for (int k = 1; k <= L; k++)
        A2(o->dpprime_visc_q, Iq, k, npq) = A2(o->dpprime_visc_q, Iq, k, npq) + A2(o->dpprime_visc, I, k, npoin) * hi;
    }
}

/* compute_gradient_uv_q (mod_barotropic_terms.F90:445-477): grad(2,2,npoin_q) of uv(2,npoin) */
static void gradient_uv_q(oracle *o, double *grad, const double *uv) {
  const int npts = o->npts;
  memset(grad, 0, sizeof(double) * 4 * (size_t)o->npoin_q);
  for (int Iq = 1; Iq <= o->npoin_q; Iq++)
    for (int ip = 1; ip <= npts; ip++) {
      int I = A2(o->m.indexq, ip, Iq, npts);
      double dhdx = A2(o->m.dpsidx, ip, Iq, npts), dhdy = A2(o->m.dpsidy, ip, Iq, npts);
      A3(grad, 1, 1, Iq, 2, 2) = A3(grad, 1, 1, Iq, 2, 2) + dhdx * A2(uv, 1, I, 2);
      A3(grad, 1, 2, Iq, 2, 2) = A3(grad, 1, 2, Iq, 2, 2) + dhdy * A2(uv, 1, I, 2);
      A3(grad, 2, 1, Iq, 2, 2) = A3(grad, 2, 1, Iq, 2, 2) + dhdx * A2(uv, 2, I, 2);
      A3(grad, 2, 2, Iq, 2, 2) = A3(grad, 2, 2, Iq, 2, 2) + dhdy * A2(uv, 2, I, 2);
    }
}

/* flux_uv_visc(4,npoin_q) -> face values flux_uv_visc_face(4,2,nq,nface) with the wall
 * reflection (mod_laplacian_quad.F90:156-212 / :296-344, one layer) */
static void lapq_face_values(oracle *o, double *ff, const double *fl) {
  const int nq = o->nq, nface = o->nface;
  const hnumo_mesh_desc *m = &o->m;
  for (int f = 1; f <= nface; f++) {
    int iel = A2(m->face, 7, f, 8), ier = A2(m->face, 8, f, 8);
    for (int iq = 1; iq <= nq; iq++) {
      int Iq = INTMA_Q(o, A3(m->imapl_q, 1, iq, f, 3, nq), A3(m->imapl_q, 2, iq, f, 3, nq), iel);
      for (int v = 1; v <= 4; v++) A4(ff, v, 1, iq, f, 4, 2, nq) = A2(fl, v, Iq, 4);
      if (ier > 0) {
        int Ir = INTMA_Q(o, A3(m->imapr_q, 1, iq, f, 3, nq), A3(m->imapr_q, 2, iq, f, 3, nq), ier);
        for (int v = 1; v <= 4; v++) A4(ff, v, 2, iq, f, 4, 2, nq) = A2(fl, v, Ir, 4);
      } else {
        for (int v = 1; v <= 4; v++) A4(ff, v, 2, iq, f, 4, 2, nq) = A4(ff, v, 1, iq, f, 4, 2, nq);
        if (ier == -4) {
          double nx = A3(m->normal_vector_q, 1, iq, f, 3, nq), ny = A3(m->normal_vector_q, 2, iq, f, 3, nq);
          double un = A2(fl, 1, Iq, 4) * nx + A2(fl, 2, Iq, 4) * ny;
          A4(ff, 1, 2, iq, f, 4, 2, nq) = A2(fl, 1, Iq, 4) - 2.0 * un * nx;
          A4(ff, 2, 2, iq, f, 4, 2, nq) = A2(fl, 2, Iq, 4) - 2.0 * un * ny;
          un = A2(fl, 3, Iq, 4) * nx + A2(fl, 4, Iq, 4) * ny;
          A4(ff, 3, 2, iq, f, 4, 2, nq) = A2(fl, 3, Iq, 4) - 2.0 * un * nx;
          A4(ff, 4, 2, iq, f, 4, 2, nq) = A2(fl, 4, Iq, 4) - 2.0 * un * ny;
        }
      }
    }
  }
}

/* compute_laplacian_quad (mod_laplacian_quad.F90:613-642) + create_rhs_laplacian_flux_quad
 * (:644-722) of one flux field, then visc*massinv (:217-218 / :349-350) into rhs_lap(2,npoin) */
static void lapq_apply(oracle *o, double *rhs_lap, const double *fl, const double *ff) {
  const int npts = o->npts, npoin = o->npoin, nq = o->nq, ngl = o->ngl, nface = o->nface;
  const hnumo_mesh_desc *m = &o->m;
  memset(rhs_lap, 0, sizeof(double) * 2 * (size_t)npoin);
  for (int Iq = 1; Iq <= o->npoin_q; Iq++) {
    double wq = m->wjac[Iq - 1];
    for (int ip = 1; ip <= npts; ip++) {
      int I = A2(m->indexq, ip, Iq, npts);
      double dhdx = A2(m->dpsidx, ip, Iq, npts), dhdy = A2(m->dpsidy, ip, Iq, npts);
      double u_visc = dhdx * A2(fl, 1, Iq, 4) + dhdy * A2(fl, 2, Iq, 4);
      double v_visc = dhdx * A2(fl, 3, Iq, 4) + dhdy * A2(fl, 4, Iq, 4);
      A2(rhs_lap, 1, I, 2) = A2(rhs_lap, 1, I, 2) - wq * u_visc;
      A2(rhs_lap, 2, I, 2) = A2(rhs_lap, 2, I, 2) - wq * v_visc;
    }
  }
  const double beta = 0.5, alpha = 1.0 - beta;
  for (int f = 1; f <= nface; f++) {
    int iel = A2(m->face, 7, f, 8), ier = A2(m->face, 8, f, 8);
    for (int iq = 1; iq <= nq; iq++) {
      double qul[2] = {A4(ff, 1, 1, iq, f, 4, 2, nq), A4(ff, 2, 1, iq, f, 4, 2, nq)};
      double qvl[2] = {A4(ff, 3, 1, iq, f, 4, 2, nq), A4(ff, 4, 1, iq, f, 4, 2, nq)};
      double qur[2] = {A4(ff, 1, 2, iq, f, 4, 2, nq), A4(ff, 2, 2, iq, f, 4, 2, nq)};
      double qvr[2] = {A4(ff, 3, 2, iq, f, 4, 2, nq), A4(ff, 4, 2, iq, f, 4, 2, nq)};
      double qu_mean[2], qv_mean[2];
      for (int c = 0; c < 2; c++) {
        qu_mean[c] = alpha * qul[c] + beta * qur[c];
        qv_mean[c] = alpha * qvl[c] + beta * qvr[c];
      }
      double wq = A2(m->jac_faceq, iq, f, nq);
      double nx = A3(m->normal_vector_q, 1, iq, f, 3, nq), ny = A3(m->normal_vector_q, 2, iq, f, 3, nq);
      double flux_qu = (qu_mean[0] - qul[0] * nx) + (qu_mean[1] - qul[1] * ny);
      double flux_qv = (qv_mean[0] - qvl[0] * nx) + (qv_mean[1] - qvl[1] * ny);
      for (int i = 1; i <= ngl; i++) {
        double hi = A2(m->psiq, i, iq, ngl);
        int ip = INTMA(o, A3(m->imapl, 1, i, f, 3, ngl), A3(m->imapl, 2, i, f, 3, ngl), iel);
        A2(rhs_lap, 1, ip, 2) = A2(rhs_lap, 1, ip, 2) + wq * hi * flux_qu;
        A2(rhs_lap, 2, ip, 2) = A2(rhs_lap, 2, ip, 2) + wq * hi * flux_qv;
        if (ier > 0) {
          ip = INTMA(o, A3(m->imapr, 1, i, f, 3, ngl), A3(m->imapr, 2, i, f, 3, ngl), ier);
          A2(rhs_lap, 1, ip, 2) = A2(rhs_lap, 1, ip, 2) - wq * hi * flux_qu;
          A2(rhs_lap, 2, ip, 2) = A2(rhs_lap, 2, ip, 2) - wq * hi * flux_qv;
        }
      }
    }
  }
  for (int I = 1; I <= npoin; I++) {
    A2(rhs_lap, 1, I, 2) = o->p.visc_mlswe * m->massinv[I - 1] * A2(rhs_lap, 1, I, 2);
    A2(rhs_lap, 2, I, 2) = o->p.visc_mlswe * m->massinv[I - 1] * A2(rhs_lap, 2, I, 2);
  }
}

/* btp_create_laplacian_v2 (mod_laplacian_quad.F90:125-223) */
static void btp_create_laplacian_v2(oracle *o, double *rhs_lap, const double *qp, const double *qb) {
  const int npoin = o->npoin, npq = o->npoin_q, L = o->L;
  double *Uk = zalloc(2 * (size_t)npoin), *grad = zalloc(4 * (size_t)npq), *fl = zalloc(4 * (size_t)npq);
  double *ff = zalloc(8 * (size_t)o->nq * o->nface);
  for (int k = 1; k <= L; k++) {
    for (int I = 1; I <= npoin; I++) {
      A2(Uk, 1, I, 2) = A3(qp, 2, I, k, 3, npoin) + A2(qb, 3, I, 4) / A2(qb, 1, I, 4);
      A2(Uk, 2, I, 2) = A3(qp, 3, I, k, 3, npoin) + A2(qb, 4, I, 4) / A2(qb, 1, I, 4);
    }
    gradient_uv_q(o, grad, Uk);
    for (int Iq = 1; Iq <= npq; Iq++) {
      double d = A2(o->dpprime_visc_q, Iq, k, npq);
      A2(fl, 1, Iq, 4) = A2(fl, 1, Iq, 4) + d * A3(grad, 1, 1, Iq, 2, 2);
      A2(fl, 2, Iq, 4) = A2(fl, 2, Iq, 4) + d * A3(grad, 1, 2, Iq, 2, 2);
      A2(fl, 3, Iq, 4) = A2(fl, 3, Iq, 4) + d * A3(grad, 2, 1, Iq, 2, 2);
      A2(fl, 4, Iq, 4) = A2(fl, 4, Iq, 4) + d * A3(grad, 2, 2, Iq, 2, 2);
    }
  }
  lapq_face_values(o, ff, fl);
  lapq_apply(o, rhs_lap, fl, ff);
  free(Uk);
  free(grad);
  free(fl);
  free(ff);
}

/* bcl_create_laplacian_v2 (mod_laplacian_quad.F90:252-355) into rhs_lap(2,npoin,nlayers) */
static void bcl_create_laplacian_v2(oracle *o, double *rhs_lap, const double *qp) {
  const int npoin = o->npoin, npq = o->npoin_q, L = o->L;
  double *Uk = zalloc(2 * (size_t)npoin), *grad = zalloc(4 * (size_t)npq), *fl = zalloc(4 * (size_t)npq);
  double *ff = zalloc(8 * (size_t)o->nq * o->nface);
  for (int k = 1; k <= L; k++) {
    for (int I = 1; I <= npoin; I++) {
      A2(Uk, 1, I, 2) = A3(qp, 2, I, k, 3, npoin) + A2(o->uvb_ave_df, 1, I, 2);
      A2(Uk, 2, I, 2) = A3(qp, 3, I, k, 3, npoin) + A2(o->uvb_ave_df, 2, I, 2);
    }
    gradient_uv_q(o, grad, Uk);
    for (int Iq = 1; Iq <= npq; Iq++) {
      double d = A2(o->dpprime_visc_q, Iq, k, npq);
      A2(fl, 1, Iq, 4) = d * A3(grad, 1, 1, Iq, 2, 2);
      A2(fl, 2, Iq, 4) = d * A3(grad, 1, 2, Iq, 2, 2);
      A2(fl, 3, Iq, 4) = d * A3(grad, 2, 1, Iq, 2, 2);
      A2(fl, 4, Iq, 4) = d * A3(grad, 2, 2, Iq, 2, 2);
    }
    /* (the reference builds every layer's face values before the laplacians; per layer the
     *  arithmetic is the same) */
    lapq_face_values(o, ff, fl);
    lapq_apply(o, rhs_lap + (size_t)(k - 1) * 2 * npoin, fl, ff);
  }
  free(Uk);
  free(grad);
  free(fl);
  free(ff);
}

/* create_rhs_btp (mod_rhs_btp.F90:28-59) */
static void create_rhs_btp(oracle *o, double *rhs, const double *qb, const double *qp) {
  const int npoin = o->npoin;
  double *qbf = zalloc(8 * (size_t)o->ngl * o->nface);
  double *rv = zalloc(2 * (size_t)npoin);
  btp_extract_df(o, qbf, qb);
  btp_volume(o, rhs, qb, qp);
  btp_fluxes(o, rhs, qbf);
  if (o->p.method_visc == 1)
    btp_create_laplacian_v2(o, rv, qp, qb);
  else
    btp_create_laplacian(o, rv, qb);
  for (int I = 1; I <= npoin; I++) {
    A2(rhs, 2, I, 3) = A2(rhs, 2, I, 3) + A2(rv, 1, I, 2);
    A2(rhs, 3, I, 3) = A2(rhs, 3, I, 3) + A2(rv, 2, I, 2);
  }
  free(qbf);
  free(rv);
}

/* btp_mom_boundary_df (mod_barotropic_terms.F90:165-217) on qb(3:4,:) */
static void btp_mom_boundary(oracle *o, double *qb) {
  const int ngl = o->ngl;
  const hnumo_mesh_desc *m = &o->m;
  for (int f = 1; f <= o->nface; f++) {
    int el = A2(m->face, 7, f, 8), er = A2(m->face, 8, f, 8);
    if (er == -4) {
      for (int n = 1; n <= ngl; n++) {
        int I = INTMA(o, A3(m->imapl, 1, n, f, 3, ngl), A3(m->imapl, 2, n, f, 3, ngl), el);
        double nx = A3(m->normal_vector, 1, n, f, 3, ngl), ny = A3(m->normal_vector, 2, n, f, 3, ngl);
        double unl = A2(qb, 3, I, 4) * nx + A2(qb, 4, I, 4) * ny;
        A2(qb, 3, I, 4) = A2(qb, 3, I, 4) - unl * nx;
        A2(qb, 4, I, 4) = A2(qb, 4, I, 4) - unl * ny;
      }
    } else if (er == -2) {
      for (int n = 1; n <= ngl; n++) {
        int I = INTMA(o, A3(m->imapl, 1, n, f, 3, ngl), A3(m->imapl, 2, n, f, 3, ngl), el);
        A2(qb, 3, I, 4) = 0.0;
        A2(qb, 4, I, 4) = 0.0;
      }
    }
  }
}

static void zero_btp_accumulators(oracle *o) {
  size_t nqf = (size_t)o->nq * o->nface, Nq = (size_t)o->npoin_q, N = (size_t)o->npoin;
  memset(o->one_plus_eta_edge_2_ave, 0, sizeof(double) * nqf);
  memset(o->uvb_ave, 0, sizeof(double) * 2 * Nq);
  memset(o->uvb_ave_df, 0, sizeof(double) * 2 * N);
  memset(o->ope_ave, 0, sizeof(double) * Nq);
  memset(o->btp_mass_flux_ave, 0, sizeof(double) * 2 * Nq);
  memset(o->H_ave, 0, sizeof(double) * Nq);
  memset(o->Qu_ave, 0, sizeof(double) * Nq);
  memset(o->Qv_ave, 0, sizeof(double) * Nq);
  memset(o->Quv_ave, 0, sizeof(double) * Nq);
  memset(o->ope2_ave_df, 0, sizeof(double) * N);
  memset(o->uvb_face_ave, 0, sizeof(double) * 4 * nqf);
  memset(o->ope_face_ave, 0, sizeof(double) * 2 * nqf);
  memset(o->ope2_face_ave, 0, sizeof(double) * 2 * nqf);
  memset(o->btp_mass_flux_face_ave, 0, sizeof(double) * 2 * nqf);
  memset(o->H_face_ave, 0, sizeof(double) * nqf);
  memset(o->Qu_face_ave, 0, sizeof(double) * 2 * nqf);
  memset(o->Qv_face_ave, 0, sizeof(double) * 2 * nqf);
  memset(o->Quv_face_ave, 0, sizeof(double) * 2 * nqf);
  memset(o->tau_wind_ave, 0, sizeof(double) * 2 * Nq);
  memset(o->tau_bot_ave, 0, sizeof(double) * 2 * Nq);
  memset(o->ope2_ave, 0, sizeof(double) * Nq);
  memset(o->graduvb_face_ave, 0, sizeof(double) * 8 * (size_t)o->ngl * o->nface);
  memset(o->graduvb_ave, 0, sizeof(double) * 4 * N);
}

static void scale(double *a, size_t n, double s) {
  for (size_t i = 0; i < n; i++) a[i] = s * a[i];
}

/* ti_barotropic_ssprk_mlswe (mod_rk_mlswe.F90:19-151) */
static void ti_barotropic_ssprk(oracle *o, double *qb, const double *qp) {
  const int npoin = o->npoin, K = o->p.kstages;
  const double *oop = o->s.one_over_pbprime_df, *pbp = o->s.pbprime_df;
  size_t n4 = 4 * (size_t)npoin;
  double *rhs = zalloc(3 * (size_t)npoin);
  double *qb0 = zalloc(n4), *qb1 = zalloc(n4), *qb2 = zalloc(n4);
  zero_btp_accumulators(o);
  for (int mstep = 1; mstep <= o->p.N_btp; mstep++) {
    memcpy(qb0, qb, sizeof(double) * n4);
    memcpy(qb1, qb, sizeof(double) * n4);
    for (int ik = 1; ik <= K; ik++) {
      double dtt = o->p.dt_btp * o->s.ssprk_beta[ik - 1];
      for (int I = 1; I <= npoin; I++) {
        double t = 1.0 + A2(qb1, 2, I, 4) * oop[I - 1];
        o->ope2_ave_df[I - 1] = o->ope2_ave_df[I - 1] + t * t;
      }
      for (int I = 1; I <= npoin; I++)
        A2(o->uvb_ave_df, 1, I, 2) = A2(o->uvb_ave_df, 1, I, 2) + A2(qb1, 3, I, 4) / A2(qb1, 1, I, 4);
      for (int I = 1; I <= npoin; I++)
        A2(o->uvb_ave_df, 2, I, 2) = A2(o->uvb_ave_df, 2, I, 2) + A2(qb1, 4, I, 4) / A2(qb1, 1, I, 4);
      create_rhs_btp(o, rhs, qb1, qp);
      double a1 = A2(o->s.ssprk_a, ik, 1, K), a2 = A2(o->s.ssprk_a, ik, 2, K), a3 = A2(o->s.ssprk_a, ik, 3, K);
      for (int v = 2; v <= 4; v++)
        for (int I = 1; I <= npoin; I++)
          A2(qb, v, I, 4) = a1 * A2(qb0, v, I, 4) + a2 * A2(qb1, v, I, 4) + a3 * A2(qb2, v, I, 4) +
                            dtt * A2(rhs, v - 1, I, 3);
      for (int I = 1; I <= npoin; I++) A2(qb, 1, I, 4) = A2(qb, 2, I, 4) + pbp[I - 1];
      btp_mom_boundary(o, qb);
      memcpy(qb1, qb, sizeof(double) * n4);
      if (K == 5 && ik == 2) memcpy(qb2, qb, sizeof(double) * n4);
    }
    for (size_t i = 0; i < 2 * (size_t)o->npoin_q; i++) o->tau_wind_ave[i] = o->tau_wind_ave[i] + o->s.tau_wind[i];
  }
  double N_inv = 1.0 / (double)(K * o->p.N_btp);
  size_t nqf = (size_t)o->nq * o->nface, Nq = (size_t)o->npoin_q, N = (size_t)npoin;
  scale(o->uvb_ave_df, 2 * N, N_inv);
  scale(o->graduvb_face_ave, 8 * (size_t)o->ngl * o->nface, N_inv);
  scale(o->graduvb_ave, 4 * N, N_inv);
  for (size_t i = 0; i < 2 * Nq; i++) o->tau_wind_ave[i] = o->tau_wind_ave[i] / (double)o->p.N_btp;
  scale(o->ope2_ave_df, N, N_inv);
  scale(o->ope2_ave, Nq, N_inv);
  scale(o->ope_ave, Nq, N_inv);
  scale(o->H_ave, Nq, N_inv);
  scale(o->Qu_ave, Nq, N_inv);
  scale(o->Qv_ave, Nq, N_inv);
  scale(o->Quv_ave, Nq, N_inv);
  scale(o->btp_mass_flux_ave, 2 * Nq, N_inv);
  scale(o->tau_bot_ave, 2 * Nq, N_inv);
  scale(o->ope_face_ave, 2 * nqf, N_inv);
  scale(o->ope2_face_ave, 2 * nqf, N_inv);
  scale(o->H_face_ave, nqf, N_inv);
  scale(o->Qu_face_ave, 2 * nqf, N_inv);
  scale(o->Qv_face_ave, 2 * nqf, N_inv);
  /* Quv_face_ave is never normalised in the reference (mod_rk_mlswe.F90:124-149) */
  scale(o->btp_mass_flux_face_ave, 2 * nqf, N_inv);
  scale(o->one_plus_eta_edge_2_ave, nqf, N_inv);
  scale(o->uvb_ave, 2 * Nq, N_inv);
  scale(o->uvb_face_ave, 4 * nqf, N_inv);
  free(rhs);
  free(qb0);
  free(qb1);
  free(qb2);
}

/* extract_qprime_df_face (mod_layer_terms.F90:354-415) */
static void extract_qprime_df_face(oracle *o, double *qf, const double *qp) {
  const int ngl = o->ngl, nface = o->nface, L = o->L, npoin = o->npoin;
  const hnumo_mesh_desc *m = &o->m;
  memset(qf, 0, sizeof(double) * 6 * (size_t)ngl * nface * L);
  for (int f = 1; f <= nface; f++) {
    int el = A2(m->face, 7, f, 8), er = A2(m->face, 8, f, 8);
    for (int n = 1; n <= ngl; n++) {
      int I = INTMA(o, A3(m->imapl, 1, n, f, 3, ngl), A3(m->imapl, 2, n, f, 3, ngl), el);
      for (int k = 1; k <= L; k++)
        for (int v = 1; v <= 3; v++) A5(qf, v, 1, n, f, k, 3, 2, ngl, nface) = A3(qp, v, I, k, 3, npoin);
      if (er > 0) {
        int Ir = INTMA(o, A3(m->imapr, 1, n, f, 3, ngl), A3(m->imapr, 2, n, f, 3, ngl), er);
        for (int k = 1; k <= L; k++)
          for (int v = 1; v <= 3; v++) A5(qf, v, 2, n, f, k, 3, 2, ngl, nface) = A3(qp, v, Ir, k, 3, npoin);
      } else {
        for (int k = 1; k <= L; k++)
          for (int v = 1; v <= 3; v++)
            A5(qf, v, 2, n, f, k, 3, 2, ngl, nface) = A5(qf, v, 1, n, f, k, 3, 2, ngl, nface);
        if (er == -4) {
          double nx = A3(m->normal_vector, 1, n, f, 3, ngl), ny = A3(m->normal_vector, 2, n, f, 3, ngl);
          for (int k = 1; k <= L; k++) {
            double un = A3(qp, 2, I, k, 3, npoin) * nx + A3(qp, 3, I, k, 3, npoin) * ny;
            A5(qf, 2, 2, n, f, k, 3, 2, ngl, nface) = A3(qp, 2, I, k, 3, npoin) - 2.0 * un * nx;
            A5(qf, 3, 2, n, f, k, 3, 2, ngl, nface) = A3(qp, 3, I, k, 3, npoin) - 2.0 * un * ny;
          }
        } else if (er == -2) {
          for (int k = 1; k <= L; k++) {
            A5(qf, 2, 2, n, f, k, 3, 2, ngl, nface) = -A5(qf, 2, 1, n, f, k, 3, 2, ngl, nface);
            A5(qf, 3, 2, n, f, k, 3, 2, ngl, nface) = -A5(qf, 3, 1, n, f, k, 3, 2, ngl, nface);
          }
        }
      }
    }
  }
}

/* btp_bcl_coeffs_qdf (mod_barotropic_terms.F90:219-409); dpprime_visc set by caller */
static void btp_bcl_coeffs(oracle *o, const double *qf, const double *qp) {
  const int npts = o->npts, npoin = o->npoin, L = o->L, ngl = o->ngl, nq = o->nq, nface = o->nface;
  const hnumo_mesh_desc *m = &o->m;
  const double *alpha = o->s.alpha;
  size_t Nq = (size_t)o->npoin_q, nqf = (size_t)nq * nface;
  memset(o->Q_uu_dp, 0, sizeof(double) * Nq);
  memset(o->Q_uv_dp, 0, sizeof(double) * Nq);
  memset(o->Q_vv_dp, 0, sizeof(double) * Nq);
  memset(o->H_bcl, 0, sizeof(double) * Nq);
  memset(o->Q_uu_dp_edge, 0, sizeof(double) * nqf);
  memset(o->Q_uv_dp_edge, 0, sizeof(double) * nqf);
  memset(o->Q_vv_dp_edge, 0, sizeof(double) * nqf);
  memset(o->H_bcl_edge, 0, sizeof(double) * nqf);
  memset(o->btp_dpp_graduv, 0, sizeof(double) * 4 * (size_t)npoin);
  memset(o->pbprime_visc, 0, sizeof(double) * (size_t)npoin);
  double pprime[64];
  for (int Iq = 1; Iq <= o->npoin_q; Iq++) {
    pprime[0] = 0.0;
    for (int k = 1; k <= L; k++) {
      double qq[3] = {0, 0, 0};
      for (int ip = 1; ip <= npts; ip++) {
        int I = A2(m->indexq, ip, Iq, npts);
        double hi = A2(m->psih, ip, Iq, npts);
        for (int v = 0; v < 3; v++) qq[v] = qq[v] + hi * A3(qp, v + 1, I, k, 3, npoin);
      }
      o->Q_uu_dp[Iq - 1] = o->Q_uu_dp[Iq - 1] + qq[1] * (qq[1] * qq[0]);
      o->Q_uv_dp[Iq - 1] = o->Q_uv_dp[Iq - 1] + qq[2] * (qq[1] * qq[0]);
      o->Q_vv_dp[Iq - 1] = o->Q_vv_dp[Iq - 1] + qq[2] * (qq[2] * qq[0]);
      pprime[k] = pprime[k - 1] + qq[0];
      o->H_bcl[Iq - 1] = o->H_bcl[Iq - 1] + 0.5 * alpha[k - 1] * (pprime[k] * pprime[k] - pprime[k - 1] * pprime[k - 1]);
    }
  }
  double *graduv = zalloc(4 * (size_t)npoin);
  for (int k = 1; k <= L; k++) {
    compute_gradient_uv(o, graduv, qp + (size_t)(k - 1) * 3 * npoin + 1, 3);
    for (int I = 1; I <= npoin; I++) {
      double d = A2(o->dpprime_visc, I, k, npoin);
      for (int v = 1; v <= 4; v++) A3(o->dpp_graduv, v, I, k, 4, npoin) = d * A2(graduv, v, I, 4);
    }
    for (int I = 1; I <= npoin; I++)
      for (int v = 1; v <= 4; v++)
        A2(o->btp_dpp_graduv, v, I, 4) = A2(o->btp_dpp_graduv, v, I, 4) + A3(o->dpp_graduv, v, I, k, 4, npoin);
    for (int I = 1; I <= npoin; I++) o->pbprime_visc[I - 1] = o->pbprime_visc[I - 1] + A2(o->dpprime_visc, I, k, npoin);
  }
  free(graduv);
  double pl[64], pr[64];
  for (int f = 1; f <= nface; f++) {
    int iel = A2(m->face, 7, f, 8), ier = A2(m->face, 8, f, 8);
    for (int iq = 1; iq <= nq; iq++) {
      pl[0] = 0.0;
      pr[0] = 0.0;
      for (int k = 1; k <= L; k++) {
        double ql[3] = {0, 0, 0}, qr[3] = {0, 0, 0};
        for (int n = 1; n <= ngl; n++) {
          double hi = A2(m->psiq, n, iq, ngl);
          for (int v = 0; v < 3; v++) {
            ql[v] = ql[v] + hi * A5(qf, v + 1, 1, n, f, k, 3, 2, ngl, nface);
            qr[v] = qr[v] + hi * A5(qf, v + 1, 2, n, f, k, 3, 2, ngl, nface);
          }
        }
        A2(o->Q_uu_dp_edge, iq, f, nq) += 0.5 * ((ql[1] * ql[1] * ql[0]) + (qr[1] * qr[1] * qr[0]));
        A2(o->Q_uv_dp_edge, iq, f, nq) += 0.5 * ((ql[2] * ql[1] * ql[0]) + (qr[2] * qr[1] * qr[0]));
        A2(o->Q_vv_dp_edge, iq, f, nq) += 0.5 * ((ql[2] * ql[2] * ql[0]) + (qr[2] * qr[2] * qr[0]));
        pl[k] = pl[k - 1] + ql[0];
        double left_dp = 0.5 * alpha[k - 1] * (pl[k] * pl[k] - pl[k - 1] * pl[k - 1]);
        pr[k] = pr[k - 1] + qr[0];
        double right_dp = 0.5 * alpha[k - 1] * (pr[k] * pr[k] - pr[k - 1] * pr[k - 1]);
        A2(o->H_bcl_edge, iq, f, nq) += 0.5 * (left_dp + right_dp);
      }
    }
    for (int iq = 1; iq <= ngl; iq++) {
      int Iq = INTMA(o, A3(m->imapl, 1, iq, f, 3, ngl), A3(m->imapl, 2, iq, f, 3, ngl), iel);
      for (int k = 1; k <= L; k++) {
        for (int v = 1; v <= 4; v++)
          A5(o->graduv_dpp_face, v, 1, iq, f, k, 5, 2, ngl, nface) = A3(o->dpp_graduv, v, Iq, k, 4, npoin);
        A5(o->graduv_dpp_face, 5, 1, iq, f, k, 5, 2, ngl, nface) = A2(o->dpprime_visc, Iq, k, npoin);
      }
      if (ier > 0) {
        int Ir = INTMA(o, A3(m->imapr, 1, iq, f, 3, ngl), A3(m->imapr, 2, iq, f, 3, ngl), ier);
        for (int k = 1; k <= L; k++) {
          for (int v = 1; v <= 4; v++)
            A5(o->graduv_dpp_face, v, 2, iq, f, k, 5, 2, ngl, nface) = A3(o->dpp_graduv, v, Ir, k, 4, npoin);
          A5(o->graduv_dpp_face, 5, 2, iq, f, k, 5, 2, ngl, nface) = A2(o->dpprime_visc, Ir, k, npoin);
        }
      } else {
        for (int k = 1; k <= L; k++)
          for (int v = 1; v <= 5; v++)
            A5(o->graduv_dpp_face, v, 2, iq, f, k, 5, 2, ngl, nface) =
                A5(o->graduv_dpp_face, v, 1, iq, f, k, 5, 2, ngl, nface);
        if (ier == -4) {
          double nx = A3(m->normal_vector, 1, iq, f, 3, ngl), ny = A3(m->normal_vector, 2, iq, f, 3, ngl);
          for (int k = 1; k <= L; k++) {
            double d1 = A3(o->dpp_graduv, 1, Iq, k, 4, npoin), d2 = A3(o->dpp_graduv, 2, Iq, k, 4, npoin);
            double d3 = A3(o->dpp_graduv, 3, Iq, k, 4, npoin), d4 = A3(o->dpp_graduv, 4, Iq, k, 4, npoin);
            double un = d1 * nx + d2 * ny;
            A5(o->graduv_dpp_face, 1, 2, iq, f, k, 5, 2, ngl, nface) = d1 - 2.0 * un * nx;
            A5(o->graduv_dpp_face, 2, 2, iq, f, k, 5, 2, ngl, nface) = d2 - 2.0 * un * ny;
            un = d3 * nx + d4 * ny;
            A5(o->graduv_dpp_face, 3, 2, iq, f, k, 5, 2, ngl, nface) = d3 - 2.0 * un * nx;
            A5(o->graduv_dpp_face, 4, 2, iq, f, k, 5, 2, ngl, nface) = d4 - 2.0 * un * ny;
          }
        }
      }
    }
  }
  memset(o->btp_graduv_dpp_face, 0, sizeof(double) * 10 * (size_t)ngl * nface);
  for (int f = 1; f <= nface; f++)
    for (int iq = 1; iq <= ngl; iq++)
      for (int k = 1; k <= L; k++)
        for (int s2 = 1; s2 <= 2; s2++)
          for (int v = 1; v <= 5; v++)
            A4(o->btp_graduv_dpp_face, v, s2, iq, f, 5, 2, ngl) =
                A4(o->btp_graduv_dpp_face, v, s2, iq, f, 5, 2, ngl) +
                A5(o->graduv_dpp_face, v, s2, iq, f, k, 5, 2, ngl, nface);
}

/* ---------------------------------------------------------- baroclinic layer terms */

/* create_layers_volume_mass (mod_create_rhs_mlswe.F90:822-877) */
static void layers_volume_mass(oracle *o, double *dp_advec, const double *qp) {
  const int npts = o->npts, npoin = o->npoin, L = o->L;
  const hnumo_mesh_desc *m = &o->m;
  memset(dp_advec, 0, sizeof(double) * (size_t)npoin * L);
  memset(o->sum_layer_mass_flux, 0, sizeof(double) * 2 * (size_t)o->npoin_q);
  for (int Iq = 1; Iq <= o->npoin_q; Iq++) {
    double qb0 = o->ope_ave[Iq - 1], qb1 = A2(o->uvb_ave, 1, Iq, 2), qb2 = A2(o->uvb_ave, 2, Iq, 2);
    double wq = m->wjac[Iq - 1];
    for (int k = 1; k <= L; k++) {
      double q[3] = {0, 0, 0};
      for (int ip = 1; ip <= npts; ip++) {
        int I = A2(m->indexq, ip, Iq, npts);
        double hi = A2(m->psih, ip, Iq, npts);
        for (int v = 0; v < 3; v++) q[v] = q[v] + hi * A3(qp, v + 1, I, k, 3, npoin);
      }
      double dp_temp = q[0] * qb0;
      double udp = (q[1] + qb1) * dp_temp;
      double vdp = (q[2] + qb2) * dp_temp;
      A2(o->sum_layer_mass_flux, 1, Iq, 2) += udp;
      A2(o->sum_layer_mass_flux, 2, Iq, 2) += vdp;
      for (int ip = 1; ip <= npts; ip++) {
        int I = A2(m->indexq, ip, Iq, npts);
        A2(dp_advec, I, k, npoin) =
            A2(dp_advec, I, k, npoin) + wq * (A2(m->dpsidx, ip, Iq, npts) * udp + A2(m->dpsidy, ip, Iq, npts) * vdp);
      }
    }
  }
}

/* create_layer_mass_flux (mod_create_rhs_mlswe.F90:922-1034) */
static void layer_mass_flux(oracle *o, double *dp_advec, const double *qf) {
  const int ngl = o->ngl, nq = o->nq, nface = o->nface, L = o->L, npoin = o->npoin;
  const hnumo_mesh_desc *m = &o->m;
  memset(o->sum_layer_mass_flux_face, 0, sizeof(double) * 2 * (size_t)nq * nface);
  double feu[32], fev[32];
  for (int f = 1; f <= nface; f++) {
    int el = A2(m->face, 7, f, 8), er = A2(m->face, 8, f, 8);
    for (int k = 1; k <= L; k++) {
      for (int iq = 1; iq <= nq; iq++) {
        double ql[3] = {0, 0, 0}, qr[3] = {0, 0, 0};
        for (int n = 1; n <= ngl; n++) {
          double hi = A2(m->psiq, n, iq, ngl);
          for (int v = 0; v < 3; v++) {
            ql[v] = ql[v] + hi * A5(qf, v + 1, 1, n, f, k, 3, 2, ngl, nface);
            qr[v] = qr[v] + hi * A5(qf, v + 1, 2, n, f, k, 3, 2, ngl, nface);
          }
        }
        double nxl = A3(m->normal_vector_q, 1, iq, f, 3, nq), nyl = A3(m->normal_vector_q, 2, iq, f, 3, nq);
        double qbl0 = A3(o->ope_face_ave, 1, iq, f, 2, nq), qbr0 = A3(o->ope_face_ave, 2, iq, f, 2, nq);
        double qbl1 = A4(o->uvb_face_ave, 1, 1, iq, f, 2, 2, nq), qbr1 = A4(o->uvb_face_ave, 1, 2, iq, f, 2, 2, nq);
        double qbl2 = A4(o->uvb_face_ave, 2, 1, iq, f, 2, 2, nq), qbr2 = A4(o->uvb_face_ave, 2, 2, iq, f, 2, 2, nq);
        double uu = 0.5 * ((ql[1] + qbl1) + (qr[1] + qbr1));
        double vv = 0.5 * ((ql[2] + qbl2) + (qr[2] + qbr2));
        double dpl = qbl0 * ql[0], dpr = qbr0 * qr[0];
        feu[iq - 1] = (uu * nxl > 0.0) ? uu * dpl : uu * dpr;
        fev[iq - 1] = (vv * nyl > 0.0) ? vv * dpl : vv * dpr;
      }
      for (int iq = 1; iq <= nq; iq++) {
        A3(o->sum_layer_mass_flux_face, 1, iq, f, 2, nq) += feu[iq - 1];
        A3(o->sum_layer_mass_flux_face, 2, iq, f, 2, nq) += fev[iq - 1];
      }
      for (int iq = 1; iq <= nq; iq++) {
        double wq = A2(m->jac_faceq, iq, f, nq);
        double nxl = A3(m->normal_vector_q, 1, iq, f, 3, nq), nyl = A3(m->normal_vector_q, 2, iq, f, 3, nq);
        double flux = nxl * feu[iq - 1] + nyl * fev[iq - 1];
        for (int n = 1; n <= ngl; n++) {
          double hi = A2(m->psiq, n, iq, ngl);
          int I = INTMA(o, A3(m->imapl, 1, n, f, 3, ngl), A3(m->imapl, 2, n, f, 3, ngl), el);
          A2(dp_advec, I, k, npoin) = A2(dp_advec, I, k, npoin) - wq * hi * flux;
          if (er > 0) {
            I = INTMA(o, A3(m->imapr, 1, n, f, 3, ngl), A3(m->imapr, 2, n, f, 3, ngl), er);
            A2(dp_advec, I, k, npoin) = A2(dp_advec, I, k, npoin) + wq * hi * flux;
          }
        }
      }
    }
  }
}

/* layer_mass_rhs (mod_create_rhs_mlswe.F90:53-78) */
static void layer_mass_rhs(oracle *o, double *dp_advec, const double *qp, const double *qf) {
  layers_volume_mass(o, dp_advec, qp);
  layer_mass_flux(o, dp_advec, qf);
  for (int k = 1; k <= o->L; k++)
    for (int I = 1; I <= o->npoin; I++)
      A2(dp_advec, I, k, o->npoin) = o->m.massinv[I - 1] * A2(dp_advec, I, k, o->npoin);
}

/* apply_consistency (mod_splitting.F90:324-366) with evaluate_consistency_face
 * (mod_layer_terms.F90:57-137), create_consistency_volume_mass / _mass_flux
 * (mod_create_rhs_mlswe.F90:879-920, 1036-1115). */
static void apply_consistency(oracle *o, double *q) {
  const int npoin = o->npoin, L = o->L, ngl = o->ngl, nq = o->nq, nface = o->nface, npts = o->npts;
  const hnumo_mesh_desc *m = &o->m;
  const hnumo_static_desc *s = &o->s;
  double *ope = zalloc(npoin), *dpp = zalloc((size_t)npoin * L), *adv = zalloc((size_t)npoin * L);
  double *mdm = zalloc(4 * (size_t)nq * nface * L);
  for (int I = 1; I <= npoin; I++) {
    double sm = 0.0;
    for (int k = 1; k <= L; k++) sm = sm + A3(q, 1, I, k, 3, npoin);
    ope[I - 1] = sm / s->pbprime_df[I - 1];
  }
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++) A2(dpp, I, k, npoin) = A3(q, 1, I, k, 3, npoin) / ope[I - 1];
  /* evaluate_consistency_face */
  for (int k = 1; k <= L; k++)
    for (int f = 1; f <= nface; f++) {
      int el = A2(m->face, 7, f, 8), er = A2(m->face, 8, f, 8);
      for (int iq = 1; iq <= nq; iq++) {
        double ql = 0.0, qr = 0.0;
        for (int n = 1; n <= ngl; n++) {
          double hi = A2(m->psiq, n, iq, ngl);
          int I = INTMA(o, A3(m->imapl, 1, n, f, 3, ngl), A3(m->imapl, 2, n, f, 3, ngl), el);
          ql = ql + hi * A2(dpp, I, k, npoin);
        }
        if (er > 0) {
          for (int n = 1; n <= ngl; n++) {
            double hi = A2(m->psiq, n, iq, ngl);
            int I = INTMA(o, A3(m->imapr, 1, n, f, 3, ngl), A3(m->imapr, 2, n, f, 3, ngl), er);
            qr = qr + hi * A2(dpp, I, k, npoin);
          }
        } else {
          qr = ql;
        }
        double wl = ql / A3(s->pbprime_face, 1, iq, f, 2, nq);
        double wr = qr / A3(s->pbprime_face, 2, iq, f, 2, nq);
        double d1 = A3(o->btp_mass_flux_face_ave, 1, iq, f, 2, nq) - A3(o->sum_layer_mass_flux_face, 1, iq, f, 2, nq);
        double d2 = A3(o->btp_mass_flux_face_ave, 2, iq, f, 2, nq) - A3(o->sum_layer_mass_flux_face, 2, iq, f, 2, nq);
        A5(mdm, 1, 1, iq, f, k, 2, 2, nq, nface) = wl * d1;
        A5(mdm, 2, 1, iq, f, k, 2, 2, nq, nface) = wl * d2;
        A5(mdm, 1, 2, iq, f, k, 2, 2, nq, nface) = wr * d1;
        A5(mdm, 2, 2, iq, f, k, 2, 2, nq, nface) = wr * d2;
      }
    }
  /* create_consistency_volume_mass */
  for (int k = 1; k <= L; k++)
    for (int Iq = 1; Iq <= o->npoin_q; Iq++) {
      double dp = 0.0;
      for (int ip = 1; ip <= npts; ip++) {
        int I = A2(m->indexq, ip, Iq, npts);
        dp = dp + A2(m->psih, ip, Iq, npts) * A2(dpp, I, k, npoin);
      }
      double weight = dp / s->pbprime[Iq - 1];
      double udp = weight * (A2(o->btp_mass_flux_ave, 1, Iq, 2) - A2(o->sum_layer_mass_flux, 1, Iq, 2));
      double vdp = weight * (A2(o->btp_mass_flux_ave, 2, Iq, 2) - A2(o->sum_layer_mass_flux, 2, Iq, 2));
      double wq = m->wjac[Iq - 1];
      for (int ip = 1; ip <= npts; ip++) {
        int I = A2(m->indexq, ip, Iq, npts);
        A2(adv, I, k, npoin) =
            A2(adv, I, k, npoin) + wq * (A2(m->dpsidx, ip, Iq, npts) * udp + A2(m->dpsidy, ip, Iq, npts) * vdp);
      }
    }
  /* create_consistency_mass_flux */
  double feu[32], fev[32];
  for (int k = 1; k <= L; k++)
    for (int f = 1; f <= nface; f++) {
      int el = A2(m->face, 7, f, 8), er = A2(m->face, 8, f, 8);
      for (int iq = 1; iq <= nq; iq++) {
        double nxl = A3(m->normal_vector_q, 1, iq, f, 3, nq), nyl = A3(m->normal_vector_q, 2, iq, f, 3, nq);
        feu[iq - 1] = (A5(mdm, 1, 1, iq, f, k, 2, 2, nq, nface) * nxl > 0.0) ? A5(mdm, 1, 1, iq, f, k, 2, 2, nq, nface)
                                                                            : A5(mdm, 1, 2, iq, f, k, 2, 2, nq, nface);
        fev[iq - 1] = (A5(mdm, 2, 1, iq, f, k, 2, 2, nq, nface) * nyl > 0.0) ? A5(mdm, 2, 1, iq, f, k, 2, 2, nq, nface)
                                                                            : A5(mdm, 2, 2, iq, f, k, 2, 2, nq, nface);
      }
      for (int iq = 1; iq <= nq; iq++) {
        double wq = A2(m->jac_faceq, iq, f, nq);
        double nxl = A3(m->normal_vector_q, 1, iq, f, 3, nq), nyl = A3(m->normal_vector_q, 2, iq, f, 3, nq);
        double flux = nxl * feu[iq - 1] + nyl * fev[iq - 1];
        for (int n = 1; n <= ngl; n++) {
          double hi = A2(m->psiq, n, iq, ngl);
          int I = INTMA(o, A3(m->imapl, 1, n, f, 3, ngl), A3(m->imapl, 2, n, f, 3, ngl), el);
          A2(adv, I, k, npoin) = A2(adv, I, k, npoin) - wq * hi * flux;
          if (er > 0) {
            I = INTMA(o, A3(m->imapr, 1, n, f, 3, ngl), A3(m->imapr, 2, n, f, 3, ngl), er);
            A2(adv, I, k, npoin) = A2(adv, I, k, npoin) + wq * hi * flux;
          }
        }
      }
    }
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++)
      A3(q, 1, I, k, 3, npoin) = A3(q, 1, I, k, 3, npoin) + o->p.dt * m->massinv[I - 1] * A2(adv, I, k, npoin);
  free(ope);
  free(dpp);
  free(adv);
  free(mdm);
}

/* bcl_create_laplacian (mod_laplacian_quad.F90:227-248) */
static void bcl_create_laplacian(oracle *o, double *rhs_lap) {
  const int npoin = o->npoin, L = o->L, ngl = o->ngl, nface = o->nface;
  double *tmp = zalloc(2 * (size_t)npoin);
  double *coef = zalloc(10 * (size_t)ngl * nface);
  memset(rhs_lap, 0, sizeof(double) * 2 * (size_t)npoin * L);
  for (int k = 1; k <= L; k++) {
    ldg_volume(o, tmp, o->dpprime_visc + (size_t)(k - 1) * npoin, o->graduvb_ave,
               o->dpp_graduv + (size_t)(k - 1) * 4 * npoin);
    memcpy(coef, o->graduv_dpp_face + (size_t)(k - 1) * 10 * ngl * nface, sizeof(double) * 10 * (size_t)ngl * nface);
    ldg_flux(o, tmp, o->graduvb_face_ave, coef);
    for (int I = 1; I <= npoin; I++) {
      A3(rhs_lap, 1, I, k, 2, npoin) = o->p.visc_mlswe * o->m.massinv[I - 1] * A2(tmp, 1, I, 2);
      A3(rhs_lap, 2, I, k, 2, npoin) = o->p.visc_mlswe * o->m.massinv[I - 1] * A2(tmp, 2, I, 2);
    }
  }
  free(tmp);
  free(coef);
}

/* create_rhs_dynamics_volume_layers (mod_create_rhs_mlswe.F90:281-456) */
static void dynamics_volume_layers(oracle *o, double *rhs_mom, const double *qp, const double *q) {
  const int npts = o->npts, npoin = o->npoin, L = o->L;
  const hnumo_mesh_desc *m = &o->m;
  const hnumo_static_desc *s = &o->s;
  const double g = o->p.gravity, eps1 = 1.0e-20;
  const double *alpha = s->alpha;
  memset(rhs_mom, 0, sizeof(double) * 2 * (size_t)npoin * L);
  double Pstress = (g / alpha[0]) * 50.0;
  double Pbstress = (g / alpha[L - 1]) * 10.0;
  double *z_elv = zalloc((size_t)npoin * (L + 1));
  for (int I = 1; I <= npoin; I++) A2(z_elv, I, L + 1, npoin) = s->zbot_df[I - 1];
  for (int k = L; k >= 1; k--)
    for (int I = 1; I <= npoin; I++)
      A2(z_elv, I, k, npoin) =
          A2(z_elv, I, k + 1, npoin) + (alpha[k - 1] / g) * (sqrt(o->ope2_ave_df[I - 1]) * A3(qp, 1, I, k, 3, npoin));
  double p_tmp[64], H_tmp[64], temp_uu[64], temp_vv[64], u_udp[64], v_vdp[64], u_vdp[2][64], pprime_temp[64];
  double gradz[2][64], qpv[3];
  for (int Iq = 1; Iq <= o->npoin_q; Iq++) {
    p_tmp[0] = 0.0;
    for (int k = 0; k < L; k++) temp_uu[k] = temp_vv[k] = 0.0;
    for (int k = 1; k <= L; k++) {
      qpv[0] = qpv[1] = qpv[2] = 0.0;
      for (int ip = 1; ip <= npts; ip++) {
        int I = A2(m->indexq, ip, Iq, npts);
        double hi = A2(m->psih, ip, Iq, npts);
        for (int v = 0; v < 3; v++) qpv[v] = qpv[v] + hi * A3(qp, v + 1, I, k, 3, npoin);
        temp_uu[k - 1] = temp_uu[k - 1] + hi * A3(q, 2, I, k, 3, npoin);
        temp_vv[k - 1] = temp_vv[k - 1] + hi * A3(q, 3, I, k, 3, npoin);
      }
      double qb0 = o->ope_ave[Iq - 1], qb1 = A2(o->uvb_ave, 1, Iq, 2), qb2 = A2(o->uvb_ave, 2, Iq, 2);
      p_tmp[k] = p_tmp[k - 1] + sqrt(o->ope2_ave[Iq - 1]) * qpv[0];
      H_tmp[k - 1] = 0.5 * alpha[k - 1] * (p_tmp[k] * p_tmp[k] - p_tmp[k - 1] * p_tmp[k - 1]);
      double dp = qpv[0] * qb0, u = qpv[1] + qb1, v = qpv[2] + qb2;
      u_udp[k - 1] = dp * u * u;
      v_vdp[k - 1] = dp * v * v;
      u_vdp[0][k - 1] = u * v * dp;
      u_vdp[1][k - 1] = v * u * dp;
      temp_uu[k - 1] = fabs(temp_uu[k - 1]) + eps1;
      temp_vv[k - 1] = fabs(temp_vv[k - 1]) + eps1;
    }
    for (int k = 0; k <= L; k++) gradz[0][k] = gradz[1][k] = 0.0;
    for (int ip = 1; ip <= npts; ip++) {
      int I = A2(m->indexq, ip, Iq, npts);
      double dx = A2(m->dpsidx, ip, Iq, npts), dy = A2(m->dpsidy, ip, Iq, npts);
      for (int k = 1; k <= L + 1; k++) {
        gradz[0][k - 1] = gradz[0][k - 1] + dx * A2(z_elv, I, k, npoin);
        gradz[1][k - 1] = gradz[1][k - 1] + dy * A2(z_elv, I, k, npoin);
      }
    }
    double su = 0, suv = 0, sv = 0, stu = 0, stv = 0;
    for (int k = 0; k < L; k++) su = su + u_udp[k];
    for (int k = 0; k < L; k++) suv = suv + u_vdp[0][k];
    for (int k = 0; k < L; k++) sv = sv + v_vdp[k];
    double uu_def = o->Qu_ave[Iq - 1] - su;
    double uv_def = o->Quv_ave[Iq - 1] - suv;
    double vv_def = o->Qv_ave[Iq - 1] - sv;
    for (int k = 0; k < L; k++) stu = stu + temp_uu[k];
    for (int k = 0; k < L; k++) stv = stv + temp_vv[k];
    double one_over_sumuq = 1.0 / stu, one_over_sumvq = 1.0 / stv;
    double wq = m->wjac[Iq - 1];
    for (int k = 0; k <= L; k++) pprime_temp[k] = 0.0;
    for (int k = 1; k <= L; k++) {
      /* QUIRK (mod_create_rhs_mlswe.F90:382): qp(k) is the last layer's (dp',u',v')
       * indexed by the layer number.  Reproduced as written (L <= 3). */
      pprime_temp[k] = pprime_temp[k - 1] + qpv[k - 1];
      double wgt = temp_uu[k - 1] * one_over_sumuq;
      u_udp[k - 1] = u_udp[k - 1] + wgt * uu_def;
      u_vdp[0][k - 1] = u_vdp[0][k - 1] + wgt * uv_def;
      wgt = temp_vv[k - 1] * one_over_sumvq;
      u_vdp[1][k - 1] = u_vdp[1][k - 1] + wgt * uv_def;
      v_vdp[k - 1] = v_vdp[k - 1] + wgt * vv_def;
      double Hq = H_tmp[k - 1];
      double weight = 1.0, acc = 0.0;
      for (int kk = 0; kk < L; kk++) acc = acc + H_tmp[kk];
      if (acc > 0.0) weight = o->H_ave[Iq - 1] / acc;
      Hq = Hq * weight;
      double var_uu = u_udp[k - 1], var_uv = u_vdp[0][k - 1], var_vu = u_vdp[1][k - 1], var_vv = v_vdp[k - 1];
      double temp1 = (fmin(pprime_temp[k], Pstress) - fmin(pprime_temp[k - 1], Pstress)) / Pstress;
      double twu = temp1 * A2(s->tau_wind, 1, Iq, 2), twv = temp1 * A2(s->tau_wind, 2, Iq, 2);
      double pb = s->pbprime[Iq - 1];
      double tempbot = fmin(Pbstress, pb - pprime_temp[k]) - fmin(Pbstress, pb - pprime_temp[k - 1]);
      tempbot = tempbot / Pbstress;
      double source_x = g * (twu - tempbot * A2(o->tau_bot_ave, 1, Iq, 2) + p_tmp[k - 1] * gradz[0][k - 1] -
                             p_tmp[k] * gradz[0][k]);
      double source_y = g * (twv - tempbot * A2(o->tau_bot_ave, 2, Iq, 2) + p_tmp[k - 1] * gradz[1][k - 1] -
                             p_tmp[k] * gradz[1][k]);
      for (int ip = 1; ip <= npts; ip++) {
        int I = A2(m->indexq, ip, Iq, npts);
        double hi = A2(m->psih, ip, Iq, npts);
        double dhdx = A2(m->dpsidx, ip, Iq, npts), dhdy = A2(m->dpsidy, ip, Iq, npts);
        A3(rhs_mom, 1, I, k, 2, npoin) =
            A3(rhs_mom, 1, I, k, 2, npoin) + wq * (hi * source_x + dhdx * (Hq + var_uu) + var_uv * dhdy);
        A3(rhs_mom, 2, I, k, 2, npoin) =
            A3(rhs_mom, 2, I, k, 2, npoin) + wq * (hi * source_y + var_vu * dhdx + dhdy * (Hq + var_vv));
      }
    }
  }
  free(z_elv);
}

/* Apply_layers_fluxes (mod_create_rhs_mlswe.F90:458-820) */
static void apply_layers_fluxes(oracle *o, double *rhs_mom, const double *qf) {
  const int ngl = o->ngl, nq = o->nq, nface = o->nface, L = o->L, npoin = o->npoin;
  const hnumo_mesh_desc *m = &o->m;
  const hnumo_static_desc *s = &o->s;
  const double g = o->p.gravity, eps1 = 1.0e-20;
  const double *alpha = s->alpha;
  double aog[64], goa[64];
  for (int k = 0; k < L; k++) {
    aog[k] = alpha[k] / g;
    goa[k] = g / alpha[k];
  }
  /* per-face work arrays, indexed [iq][k] */
  double ql[32][64][3], qr[32][64][3], udpl[32][64], udpr[32][64], vdpl[32][64], vdpr[32][64];
  double udpf[2][32][64], vdpf[2][32][64], Hface[2][32][64];
  double pf[2][65], zf[2][65], pep[65], pem[65], zep[65], zem[65], p2l[65], p2r[65];
  for (int f = 1; f <= nface; f++) {
    int el = A2(m->face, 7, f, 8), er = A2(m->face, 8, f, 8);
    for (int iq = 0; iq < nq; iq++)
      for (int k = 0; k < L; k++)
        for (int v = 0; v < 3; v++) ql[iq][k][v] = qr[iq][k][v] = 0.0;
    for (int iq = 1; iq <= nq; iq++) {
      double qbl0 = A3(o->ope_face_ave, 1, iq, f, 2, nq), qbr0 = A3(o->ope_face_ave, 2, iq, f, 2, nq);
      double qbl1 = A4(o->uvb_face_ave, 1, 1, iq, f, 2, 2, nq), qbr1 = A4(o->uvb_face_ave, 1, 2, iq, f, 2, 2, nq);
      double qbl2 = A4(o->uvb_face_ave, 2, 1, iq, f, 2, 2, nq), qbr2 = A4(o->uvb_face_ave, 2, 2, iq, f, 2, 2, nq);
      double nxl = A3(m->normal_vector_q, 1, iq, f, 3, nq), nyl = A3(m->normal_vector_q, 2, iq, f, 3, nq);
      int i = iq - 1;
      for (int k = 1; k <= L; k++) {
        int kk = k - 1;
        for (int n = 1; n <= ngl; n++) {
          double hi = A2(m->psiq, n, iq, ngl);
          for (int v = 0; v < 3; v++) {
            ql[i][kk][v] = ql[i][kk][v] + hi * A5(qf, v + 1, 1, n, f, k, 3, 2, ngl, nface);
            qr[i][kk][v] = qr[i][kk][v] + hi * A5(qf, v + 1, 2, n, f, k, 3, 2, ngl, nface);
          }
        }
        double dpl = qbl0 * ql[i][kk][0], dpr = qbr0 * qr[i][kk][0];
        double ul = ql[i][kk][1] + qbl1, ur = qr[i][kk][1] + qbr1;
        double vl = ql[i][kk][2] + qbl2, vr = qr[i][kk][2] + qbr2;
        double uu = 0.5 * (ul + ur), vv = 0.5 * (vl + vr);
        udpl[i][kk] = ul * dpl;
        udpr[i][kk] = ur * dpr;
        vdpl[i][kk] = vl * dpl;
        vdpr[i][kk] = vr * dpr;
        if (uu * nxl > 0.0) {
          udpf[0][i][kk] = uu * (ul * dpl);
          vdpf[0][i][kk] = uu * (vl * dpl);
        } else {
          udpf[0][i][kk] = uu * (ur * dpr);
          vdpf[0][i][kk] = uu * (vr * dpr);
        }
        if (vv * nyl > 0.0) {
          udpf[1][i][kk] = vv * (ul * dpl);
          vdpf[1][i][kk] = vv * (vl * dpl);
        } else {
          udpf[1][i][kk] = vv * (ur * dpr);
          vdpf[1][i][kk] = vv * (vr * dpr);
        }
      }
      double s1 = 0, s2 = 0, s3 = 0, s4 = 0;
      for (int k = 0; k < L; k++) s1 = s1 + udpf[0][i][k];
      for (int k = 0; k < L; k++) s2 = s2 + udpf[1][i][k];
      for (int k = 0; k < L; k++) s3 = s3 + vdpf[0][i][k];
      for (int k = 0; k < L; k++) s4 = s4 + vdpf[1][i][k];
      double uu_def = A3(o->Qu_face_ave, 1, iq, f, 2, nq) - s1;
      double uv_def = A3(o->Qu_face_ave, 2, iq, f, 2, nq) - s2;
      double vu_def = A3(o->Qv_face_ave, 1, iq, f, 2, nq) - s3;
      double vv_def = A3(o->Qv_face_ave, 2, iq, f, 2, nq) - s4;
      double sl = 0, sr = 0;
      for (int k = 0; k < L; k++) sl = sl + (fabs(udpl[i][k]) + eps1);
      for (int k = 0; k < L; k++) sr = sr + (fabs(udpr[i][k]) + eps1);
      double oosl = 1.0 / sl, oosr = 1.0 / sr;
      if (uu_def * nxl > 0.0) {
        for (int k = 0; k < L; k++) udpf[0][i][k] = udpf[0][i][k] + (fabs(udpl[i][k]) * oosl) * uu_def;
      } else {
        for (int k = 0; k < L; k++) udpf[0][i][k] = udpf[0][i][k] + (fabs(udpr[i][k]) * oosr) * uu_def;
      }
      if (uv_def * nyl > 0.0) {
        for (int k = 0; k < L; k++) udpf[1][i][k] = udpf[1][i][k] + (fabs(udpl[i][k]) * oosl) * uv_def;
      } else {
        for (int k = 0; k < L; k++) udpf[1][i][k] = udpf[1][i][k] + (fabs(udpr[i][k]) * oosr) * uv_def;
      }
      sl = 0;
      sr = 0;
      for (int k = 0; k < L; k++) sl = sl + (fabs(vdpl[i][k]) + eps1);
      for (int k = 0; k < L; k++) sr = sr + (fabs(vdpr[i][k]) + eps1);
      oosl = 1.0 / sl;
      oosr = 1.0 / sr;
      if (vu_def * nxl > 0.0) {
        for (int k = 0; k < L; k++) vdpf[0][i][k] = vdpf[0][i][k] + (fabs(vdpl[i][k]) * oosl) * vu_def;
      } else {
        for (int k = 0; k < L; k++) vdpf[0][i][k] = vdpf[0][i][k] + (fabs(vdpr[i][k]) * oosr) * vu_def;
      }
      if (vv_def * nyl > 0.0) {
        for (int k = 0; k < L; k++) vdpf[1][i][k] = vdpf[1][i][k] + (fabs(vdpl[i][k]) * oosl) * vv_def;
      } else {
        for (int k = 0; k < L; k++) vdpf[1][i][k] = vdpf[1][i][k] + (fabs(vdpr[i][k]) * oosr) * vv_def;
      }
      for (int k = 0; k <= L; k++) {
        zf[0][k] = zf[1][k] = pf[0][k] = pf[1][k] = 0.0;
        zep[k] = zem[k] = pep[k] = pem[k] = 0.0;
      }
      double ope_l = sqrt(A3(o->ope2_face_ave, 1, iq, f, 2, nq));
      double ope_r = sqrt(A3(o->ope2_face_ave, 2, iq, f, 2, nq));
      pf[0][0] = 0.0;
      pf[1][0] = 0.0;
      for (int k = 1; k <= L; k++) {
        pf[0][k] = pf[0][k - 1] + ope_l * ql[i][k - 1][0];
        pf[1][k] = pf[1][k - 1] + ope_r * qr[i][k - 1][0];
      }
      double ope_e = sqrt(A2(o->one_plus_eta_edge_2_ave, iq, f, nq));
      zf[0][L] = A3(s->zbot_face, 1, iq, f, 2, nq);
      zf[1][L] = A3(s->zbot_face, 2, iq, f, 2, nq);
      zep[L] = A3(s->zbot_face, 1, iq, f, 2, nq);
      zem[L] = A3(s->zbot_face, 2, iq, f, 2, nq);
      for (int k = L; k >= 1; k--) {
        zf[0][k - 1] = zf[0][k] + aog[k - 1] * (ope_l * ql[i][k - 1][0]);
        zf[1][k - 1] = zf[1][k] + aog[k - 1] * (ope_r * qr[i][k - 1][0]);
        zep[k - 1] = zep[k] + aog[k - 1] * (ope_e * ql[i][k - 1][0]);
        zem[k - 1] = zem[k] + aog[k - 1] * (ope_e * qr[i][k - 1][0]);
      }
      pep[1] = ope_e * ql[i][0][0];
      pem[1] = ope_e * qr[i][0][0];
      for (int k = 2; k <= L; k++) {
        pep[k] = pep[k - 1] + ope_e * ql[i][k - 1][0];
        pem[k] = pem[k - 1] + ope_e * qr[i][k - 1][0];
      }
      for (int k = 1; k <= L; k++) {
        double Hrp = 0.5 * alpha[k - 1] * (pep[k] * pep[k] - pep[k - 1] * pep[k - 1]);
        double Hrm = 0.0;
        for (int kt = 1; kt <= L; kt++) {
          double zt = fmin(zem[kt - 1], zep[k - 1]);
          double zb = fmax(zem[kt], zep[k]);
          double dz = zt - zb;
          if (dz > 0.0) {
            double pbot = pem[kt] - goa[kt - 1] * (zb - zem[kt]);
            double ptop = pem[kt] - goa[kt - 1] * (zt - zem[kt]);
            Hrm = Hrm + 0.5 * alpha[kt - 1] * (pbot * pbot - ptop * ptop);
          }
        }
        Hface[0][i][k - 1] = 0.5 * (Hrp + Hrm);
        Hrm = 0.5 * alpha[k - 1] * (pem[k] * pem[k] - pem[k - 1] * pem[k - 1]);
        Hrp = 0.0;
        for (int kt = 1; kt <= L; kt++) {
          double zt = fmin(zep[kt - 1], zem[k - 1]);
          double zb = fmax(zep[kt], zem[k]);
          double dz = zt - zb;
          if (dz > 0.0) {
            double pbot = pep[kt] - goa[kt - 1] * (zb - zep[kt]);
            double ptop = pep[kt] - goa[kt - 1] * (zt - zep[kt]);
            Hrp = Hrp + 0.5 * alpha[kt - 1] * (pbot * pbot - ptop * ptop);
          }
        }
        Hface[1][i][k - 1] = 0.5 * (Hrp + Hrm);
      }
      if (er == -4) {
        for (int k = 0; k <= L; k++) p2l[k] = p2r[k] = 0.0;
        for (int k = 1; k <= L; k++) {
          p2l[k] = pf[0][k];
          Hface[0][i][k - 1] = 0.5 * alpha[k - 1] * (p2l[k] * p2l[k] - p2l[k - 1] * p2l[k - 1]);
          p2r[k] = pf[1][k];
          Hface[1][i][k - 1] = 0.5 * alpha[k - 1] * (p2r[k] * p2r[k] - p2r[k - 1] * p2r[k - 1]);
        }
      }
      if (er != -4) {
        for (int k = 1; k <= L - 1; k++) {
          double pinc1 = goa[k - 1] * (zf[0][k] - zep[k]);
          double Hc1 = 0.5 * alpha[k - 1] * ((pf[0][k] + pinc1) * (pf[0][k] + pinc1) - pf[0][k] * pf[0][k]);
          Hface[0][i][k - 1] = Hface[0][i][k - 1] - Hc1;
          Hface[0][i][k] = Hface[0][i][k] + Hc1;
          double pinc2 = goa[k - 1] * (zf[1][k] - zem[k]);
          double Hc2 = 0.5 * alpha[k - 1] * ((pf[1][k] + pinc2) * (pf[1][k] + pinc2) - pf[1][k] * pf[1][k]);
          Hface[1][i][k - 1] = Hface[1][i][k - 1] - Hc2;
          Hface[1][i][k] = Hface[1][i][k] + Hc2;
        }
      }
      for (int sd = 0; sd < 2; sd++) {
        double weight = 1.0, acc = 0.0;
        for (int k = 0; k < L; k++) acc = acc + Hface[sd][i][k];
        if (acc > 0.0) weight = A2(o->H_face_ave, iq, f, nq) / acc;
        for (int k = 0; k < L; k++) Hface[sd][i][k] = Hface[sd][i][k] * weight;
      }
    }
    for (int k = 1; k <= L; k++) {
      for (int iq = 1; iq <= nq; iq++) {
        int i = iq - 1;
        double wq = A2(m->jac_faceq, iq, f, nq);
        double nxl = A3(m->normal_vector_q, 1, iq, f, 3, nq), nyl = A3(m->normal_vector_q, 2, iq, f, 3, nq);
        double hlx = nxl * Hface[0][i][k - 1], hrx = nxl * Hface[1][i][k - 1];
        double hly = nyl * Hface[0][i][k - 1], hry = nyl * Hface[1][i][k - 1];
        double flux_x = nxl * udpf[0][i][k - 1] + nyl * udpf[1][i][k - 1];
        double flux_y = nxl * vdpf[0][i][k - 1] + nyl * vdpf[1][i][k - 1];
        for (int n = 1; n <= ngl; n++) {
          double hi = A2(m->psiq, n, iq, ngl);
          int I = INTMA(o, A3(m->imapl, 1, n, f, 3, ngl), A3(m->imapl, 2, n, f, 3, ngl), el);
          A3(rhs_mom, 1, I, k, 2, npoin) = A3(rhs_mom, 1, I, k, 2, npoin) - wq * hi * (hlx + flux_x);
          A3(rhs_mom, 2, I, k, 2, npoin) = A3(rhs_mom, 2, I, k, 2, npoin) - wq * hi * (hly + flux_y);
          if (er > 0) {
            I = INTMA(o, A3(m->imapr, 1, n, f, 3, ngl), A3(m->imapr, 2, n, f, 3, ngl), er);
            A3(rhs_mom, 1, I, k, 2, npoin) = A3(rhs_mom, 1, I, k, 2, npoin) + wq * hi * (hrx + flux_x);
            A3(rhs_mom, 2, I, k, 2, npoin) = A3(rhs_mom, 2, I, k, 2, npoin) + wq * hi * (hry + flux_y);
          }
        }
      }
    }
  }
}

/* rhs_momentum (mod_splitting.F90:289-322) -> layer_momentum_rhs (mod_create_rhs_mlswe.F90:28-51) */
static void rhs_momentum(oracle *o, double *rhs_mom, const double *qp, const double *q, const double *qf) {
  const int npoin = o->npoin, L = o->L;
  double *visc = zalloc(2 * (size_t)npoin * L);
  if (o->p.method_visc == 1)
    bcl_create_laplacian_v2(o, visc, qp);
  else
    bcl_create_laplacian(o, visc);
  dynamics_volume_layers(o, rhs_mom, qp, q);
  apply_layers_fluxes(o, rhs_mom, qf);
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++) {
      A3(rhs_mom, 1, I, k, 2, npoin) = o->m.massinv[I - 1] * A3(rhs_mom, 1, I, k, 2, npoin) + A3(visc, 1, I, k, 2, npoin);
      A3(rhs_mom, 2, I, k, 2, npoin) = o->m.massinv[I - 1] * A3(rhs_mom, 2, I, k, 2, npoin) + A3(visc, 2, I, k, 2, npoin);
    }
  free(visc);
}

/* extract_velocity (mod_layer_terms.F90:272-320) */
static void extract_velocity(oracle *o, double *uv, const double *q, const double *qb) {
  const int npoin = o->npoin, L = o->L;
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++) {
      A3(uv, 1, I, k, 2, npoin) = A3(q, 2, I, k, 3, npoin) / A3(q, 1, I, k, 3, npoin);
      A3(uv, 2, I, k, 2, npoin) = A3(q, 3, I, k, 3, npoin) / A3(q, 1, I, k, 3, npoin);
    }
  for (int I = 1; I <= npoin; I++) {
    double ubar = 0.0, vbar = 0.0;
    for (int k = 1; k <= L; k++) {
      ubar = ubar + A3(uv, 1, I, k, 2, npoin) * A3(q, 1, I, k, 3, npoin);
      vbar = vbar + A3(uv, 2, I, k, 2, npoin) * A3(q, 1, I, k, 3, npoin);
    }
    if (A2(qb, 1, I, 4) > 0.0) {
      ubar = ubar / A2(qb, 1, I, 4);
      vbar = vbar / A2(qb, 1, I, 4);
      for (int k = 1; k <= L; k++) {
        A3(uv, 1, I, k, 2, npoin) = A3(uv, 1, I, k, 2, npoin) - ubar + A2(qb, 3, I, 4) / A2(qb, 1, I, 4);
        A3(uv, 2, I, k, 2, npoin) = A3(uv, 2, I, k, 2, npoin) - vbar + A2(qb, 4, I, 4) / A2(qb, 1, I, 4);
      }
    } else {
      for (int k = 1; k <= L; k++) A3(uv, 1, I, k, 2, npoin) = A3(uv, 2, I, k, 2, npoin) = 0.0;
    }
  }
}

/* evaluate_bcl (mod_layer_terms.F90:198-238) and evaluate_bcl_v1 (:240-270) */
static void evaluate_bcl(oracle *o, double *qf, double *q, double *qp, const double *qb, int v1) {
  const int npoin = o->npoin, L = o->L;
  double *uv = zalloc(2 * (size_t)npoin * L), *ope = zalloc(npoin);
  extract_velocity(o, uv, q, qb);
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++) {
      A3(q, 2, I, k, 3, npoin) = A3(uv, 1, I, k, 2, npoin) * A3(q, 1, I, k, 3, npoin);
      A3(q, 3, I, k, 3, npoin) = A3(uv, 2, I, k, 2, npoin) * A3(q, 1, I, k, 3, npoin);
      if (!v1) ope[I - 1] = ope[I - 1] + A3(q, 1, I, k, 3, npoin);
    }
  if (!v1)
    for (int I = 1; I <= npoin; I++) ope[I - 1] = ope[I - 1] / o->s.pbprime_df[I - 1];
  extract_velocity(o, uv, q, qb);
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++) {
      if (!v1) A3(qp, 1, I, k, 3, npoin) = A3(q, 1, I, k, 3, npoin) / ope[I - 1];
      A3(qp, 2, I, k, 3, npoin) = A3(uv, 1, I, k, 2, npoin) - A2(qb, 3, I, 4) / A2(qb, 1, I, 4);
      A3(qp, 3, I, k, 3, npoin) = A3(uv, 2, I, k, 2, npoin) - A2(qb, 4, I, 4) / A2(qb, 1, I, 4);
    }
  if (!v1) extract_qprime_df_face(o, qf, qp);
  free(uv);
  free(ope);
}

/* layer_mom_boundary_df (mod_layer_terms.F90:529-584) on q(2:3,:,:) */
static void layer_mom_boundary(oracle *o, double *q) {
  const int ngl = o->ngl, npoin = o->npoin, L = o->L;
  const hnumo_mesh_desc *m = &o->m;
  for (int f = 1; f <= o->nface; f++) {
    int el = A2(m->face, 7, f, 8), er = A2(m->face, 8, f, 8);
    if (er != -4 && er != -2) continue;
    for (int n = 1; n <= ngl; n++) {
      int I = INTMA(o, A3(m->imapl, 1, n, f, 3, ngl), A3(m->imapl, 2, n, f, 3, ngl), el);
      double nx = A3(m->normal_vector, 1, n, f, 3, ngl), ny = A3(m->normal_vector, 2, n, f, 3, ngl);
      for (int k = 1; k <= L; k++) {
        if (er == -4) {
          double u = A3(q, 2, I, k, 3, npoin), v = A3(q, 3, I, k, 3, npoin);
          double upnl = u * nx + v * ny;
          A3(q, 2, I, k, 3, npoin) = u - upnl * nx;
          A3(q, 3, I, k, 3, npoin) = v - upnl * ny;
        } else {
          A3(q, 2, I, k, 3, npoin) = 0.0;
          A3(q, 3, I, k, 3, npoin) = 0.0;
        }
      }
    }
  }
}

static int check_thickness(oracle *o, const double *q) {
  for (int k = 1; k <= o->L; k++)
    for (int I = 1; I <= o->npoin; I++)
      if (A3(q, 1, I, k, 3, o->npoin) < 0.0) return set_err(o, HNUMO_ERR_NEGATIVE_THICKNESS, "Negative mass in thickness at some points");
  return 0;
}

/* velocity_df (mod_layer_terms.F90:139-196): layer momenta made consistent with the
 * barotropic velocity, q(2:3) <- u_k dp_k (the arithmetic of extract_velocity) */
static void velocity_df(oracle *o, double *q, const double *qb) {
  const int npoin = o->npoin, L = o->L;
  double *uv = zalloc(2 * (size_t)npoin * L);
  extract_velocity(o, uv, q, qb);
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++) {
      A3(q, 2, I, k, 3, npoin) = A3(uv, 1, I, k, 2, npoin) * A3(q, 1, I, k, 3, npoin);
      A3(q, 3, I, k, 3, npoin) = A3(uv, 2, I, k, 2, npoin) * A3(q, 1, I, k, 3, npoin);
    }
  free(uv);
}

/* rhs_layer_shear_stress (mod_create_rhs_mlswe.F90:146-279): per quad point the implicit
 * vertical shear-stress system over the layers (tridiagonal; sub-diagonal -coeff,
 * super-diagonal -coeff1, as written), the interface stresses and their weak form.
 * tau(nlayers+1) is never assigned in the reference (:160,:246-251): zero, as under the
 * reference build's -finit-real=zero. */
static void rhs_layer_shear_stress(oracle *o, double *rs, const double *q) {
  const int npts = o->npts, npoin = o->npoin, L = o->L;
  const hnumo_mesh_desc *m = &o->m;
  const double g = o->p.gravity, ad = o->p.ad_mlswe, dt = o->p.dt, al1 = o->s.alpha[0];
  double dp[3], udp[3], vdp[3], a[3], b[3], c[3], r[2][3], uv[2][3], tu[4], tv[4];
  memset(rs, 0, sizeof(double) * 2 * (size_t)npoin * L);
  for (int Iq = 1; Iq <= o->npoin_q; Iq++) {
    for (int k = 0; k < L; k++) dp[k] = udp[k] = vdp[k] = 0.0;
    for (int ip = 1; ip <= npts; ip++) {
      int I = A2(m->indexq, ip, Iq, npts);
      double hi = A2(m->psih, ip, Iq, npts);
      for (int k = 0; k < L; k++) {
        dp[k] = dp[k] + hi * A3(q, 1, I, k + 1, 3, npoin);
        udp[k] = udp[k] + hi * A3(q, 2, I, k + 1, 3, npoin);
        vdp[k] = vdp[k] + hi * A3(q, 3, I, k + 1, 3, npoin);
      }
    }
    /* Fortran MAX as gfortran evaluates it: the second argument if larger or the first is NaN */
    double coeff = sqrt(0.5 * o->s.coriolis_quad[Iq - 1] * ad) / al1;
    const double c2 = ad / (al1 * o->p.max_shear_dz);
    if (c2 > coeff || isnan(coeff)) coeff = c2;
    const double coeff1 = g * dt * coeff;
    for (int k = 0; k < L; k++) {
      a[k] = -coeff;
      b[k] = dp[k] + 2.0 * coeff1;
      c[k] = -coeff1;
      r[0][k] = udp[k] / dp[k];
      r[1][k] = vdp[k] / dp[k];
    }
    b[0] = dp[0] + coeff1;
    b[L - 1] = dp[L - 1] + coeff1;
    a[0] = 0.0;
    c[L - 1] = 0.0;
    for (int k = 1; k < L; k++) {
      const double mult = a[k] / b[k - 1];
      b[k] = b[k] - mult * c[k - 1];
      r[0][k] = r[0][k] - mult * r[0][k - 1];
      r[1][k] = r[1][k] - mult * r[1][k - 1];
    }
    r[0][L - 1] = r[0][L - 1] / b[L - 1];
    r[1][L - 1] = r[1][L - 1] / b[L - 1];
    uv[0][L - 1] = r[0][L - 1];
    uv[1][L - 1] = r[1][L - 1];
    for (int k = L - 2; k >= 0; k--) {
      r[0][k] = (r[0][k] - c[k] * r[0][k + 1]) / b[k];
      r[1][k] = (r[1][k] - c[k] * r[1][k + 1]) / b[k];
      uv[0][k] = r[0][k];
      uv[1][k] = r[1][k];
    }
    tu[0] = tv[0] = 0.0;
    for (int k = 1; k < L; k++) {
      tu[k] = coeff * (uv[0][k - 1] - uv[0][k]);
      tv[k] = coeff * (uv[1][k - 1] - uv[1][k]);
    }
    tu[L] = tv[L] = 0.0;
    const double wq = m->wjac[Iq - 1];
    for (int k = 0; k < L; k++) {
      const double tuq = g * (tu[k] - tu[k + 1]), tvq = g * (tv[k] - tv[k + 1]);
      for (int ip = 1; ip <= npts; ip++) {
        int I = A2(m->indexq, ip, Iq, npts);
        double hi = A2(m->psih, ip, Iq, npts);
        A3(rs, 1, I, k + 1, 2, npoin) = A3(rs, 1, I, k + 1, 2, npoin) + wq * hi * tuq;
        A3(rs, 2, I, k + 1, 2, npoin) = A3(rs, 2, I, k + 1, 2, npoin) + wq * hi * tvq;
      }
    }
  }
}

/* momentum update (mod_splitting.F90:131-175 / :239-282): q_df_temp = q + dt*rhs_mom; with
 * ad_mlswe > 0 the implicit vertical shear stress (:140-164 / :248-271); then the implicit
 * Coriolis rotation and the wall fix.  corrector != 0: the momentum() call, whose
 * shear-stress input is its never-assigned `uv` (:119,:158) -- zeros, unless
 * shear_corrector selects q_df3 (include/hnumo_engine.h, hnumo_params). */
static void momentum_update(oracle *o, double *q, const double *rhs_mom, const double *qb, int corrector) {
  const int npoin = o->npoin, L = o->L;
  const double dt = o->p.dt;
  const double *f2 = o->s.fdt2_bcl, *a = o->s.a_bcl, *b = o->s.b_bcl;
  double *tmp = zalloc(2 * (size_t)npoin * L);
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++) {
      A3(tmp, 1, I, k, 2, npoin) = A3(q, 2, I, k, 3, npoin) + dt * A3(rhs_mom, 1, I, k, 2, npoin);
      A3(tmp, 2, I, k, 2, npoin) = A3(q, 3, I, k, 3, npoin) + dt * A3(rhs_mom, 2, I, k, 2, npoin);
    }
  if (o->p.ad_mlswe > 0.0) {
    double *q3 = zalloc(3 * (size_t)npoin * L), *rs = zalloc(2 * (size_t)npoin * L);
    for (int k = 1; k <= L; k++)
      for (int I = 1; I <= npoin; I++) {
        double tu = A3(tmp, 1, I, k, 2, npoin) + f2[I - 1] * A3(q, 3, I, k, 3, npoin);
        double tv = A3(tmp, 2, I, k, 2, npoin) - f2[I - 1] * A3(q, 2, I, k, 3, npoin);
        A3(q3, 1, I, k, 3, npoin) = A3(q, 1, I, k, 3, npoin);
        A3(q3, 2, I, k, 3, npoin) = a[I - 1] * tu + b[I - 1] * tv;
        A3(q3, 3, I, k, 3, npoin) = -b[I - 1] * tu + a[I - 1] * tv;
      }
    velocity_df(o, q3, qb);
    if (corrector && o->p.shear_corrector != HNUMO_SHEAR_CORRECTOR_PREDICTED)
      memset(q3, 0, sizeof(double) * 3 * (size_t)npoin * L);
    rhs_layer_shear_stress(o, rs, q3);
    for (int k = 1; k <= L; k++)
      for (int I = 1; I <= npoin; I++) {
        A3(tmp, 1, I, k, 2, npoin) = A3(tmp, 1, I, k, 2, npoin) + dt * (o->m.massinv[I - 1] * A3(rs, 1, I, k, 2, npoin));
        A3(tmp, 2, I, k, 2, npoin) = A3(tmp, 2, I, k, 2, npoin) + dt * (o->m.massinv[I - 1] * A3(rs, 2, I, k, 2, npoin));
      }
    free(q3);
    free(rs);
  }
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++) {
      double tu = A3(tmp, 1, I, k, 2, npoin) + f2[I - 1] * A3(q, 3, I, k, 3, npoin);
      double tv = A3(tmp, 2, I, k, 2, npoin) - f2[I - 1] * A3(q, 2, I, k, 3, npoin);
      A3(q, 2, I, k, 3, npoin) = a[I - 1] * tu + b[I - 1] * tv;
      A3(q, 3, I, k, 3, npoin) = -b[I - 1] * tu + a[I - 1] * tv;
    }
  free(tmp);
  layer_mom_boundary(o, q);
}

/* momentum_mass (mod_splitting.F90:182-287) */
static int momentum_mass(oracle *o, double *q, double *qf, double *qp, const double *qb) {
  const int npoin = o->npoin, L = o->L;
  double *adv = zalloc((size_t)npoin * L), *rhs_mom = zalloc(2 * (size_t)npoin * L);
  layer_mass_rhs(o, adv, qp, qf);
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++)
      A3(q, 1, I, k, 3, npoin) = A3(q, 1, I, k, 3, npoin) + o->p.dt * A2(adv, I, k, npoin);
  int rc = check_thickness(o, q);
  if (!rc) {
    apply_consistency(o, q);
    rhs_momentum(o, rhs_mom, qp, q, qf);
    momentum_update(o, q, rhs_mom, qb, 0);
    evaluate_bcl(o, qf, q, qp, qb, 0);
  }
  free(adv);
  free(rhs_mom);
  return rc;
}

/* thickness (mod_splitting.F90:25-91) */
static int thickness(oracle *o, double *qp, double *q, const double *qb, double *qf) {
  const int npoin = o->npoin, L = o->L, ngl = o->ngl, nface = o->nface;
  const hnumo_mesh_desc *m = &o->m;
  double *adv = zalloc((size_t)npoin * L), *ope = zalloc(npoin);
  layer_mass_rhs(o, adv, qp, qf);
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++)
      A3(q, 1, I, k, 3, npoin) = A3(q, 1, I, k, 3, npoin) + o->p.dt * A2(adv, I, k, npoin);
  int rc = check_thickness(o, q);
  if (!rc) {
    apply_consistency(o, q);
    for (int I = 1; I <= npoin; I++) {
      double sm = 0.0;
      for (int k = 1; k <= L; k++) sm = sm + A3(q, 1, I, k, 3, npoin);
      ope[I - 1] = sm / o->s.pbprime_df[I - 1];
    }
    for (int k = 1; k <= L; k++)
      for (int I = 1; I <= npoin; I++) A3(qp, 1, I, k, 3, npoin) = A3(q, 1, I, k, 3, npoin) / ope[I - 1];
    /* extract_dprime_df_face (mod_layer_terms.F90:417-465) into qprime_df_face(1,...) */
    for (int f = 1; f <= nface; f++) {
      int el = A2(m->face, 7, f, 8), er = A2(m->face, 8, f, 8);
      for (int n = 1; n <= ngl; n++) {
        int I = INTMA(o, A3(m->imapl, 1, n, f, 3, ngl), A3(m->imapl, 2, n, f, 3, ngl), el);
        for (int k = 1; k <= L; k++) A5(qf, 1, 1, n, f, k, 3, 2, ngl, nface) = A3(qp, 1, I, k, 3, npoin);
        if (er > 0) {
          int Ir = INTMA(o, A3(m->imapr, 1, n, f, 3, ngl), A3(m->imapr, 2, n, f, 3, ngl), er);
          for (int k = 1; k <= L; k++) A5(qf, 1, 2, n, f, k, 3, 2, ngl, nface) = A3(qp, 1, Ir, k, 3, npoin);
        } else {
          for (int k = 1; k <= L; k++) A5(qf, 1, 2, n, f, k, 3, 2, ngl, nface) = A5(qf, 1, 1, n, f, k, 3, 2, ngl, nface);
        }
      }
    }
  }
  free(adv);
  free(ope);
  return rc;
}

/* momentum (mod_splitting.F90:94-180) */
static void momentum(oracle *o, double *q, double *qp, const double *qb, const double *qf) {
  const int npoin = o->npoin, L = o->L;
  double *rhs_mom = zalloc(2 * (size_t)npoin * L);
  rhs_momentum(o, rhs_mom, qp, q, qf);
  momentum_update(o, q, rhs_mom, qb, 1);
  evaluate_bcl(o, NULL, q, qp, qb, 1);
  free(rhs_mom);
}

static void set_dpprime_visc(oracle *o, const double *qp) {
  for (int k = 1; k <= o->L; k++)
    for (int I = 1; I <= o->npoin; I++)
      A2(o->dpprime_visc, I, k, o->npoin) = A3(qp, 1, I, k, 3, o->npoin);
  if (o->p.method_visc == 1) interpolate_dpp(o);  /* ti_rk_bcl.F90:48,67 */
}

/* ============================================================== exported API */

int oracle_ti_rk_bcl(oracle *o, double *q_df, double *qb_df, double *qprime_df) {
  const int npoin = o->npoin, L = o->L;
  size_t nq3 = 3 * (size_t)npoin * L, nf = 6 * (size_t)o->ngl * o->nface * L;
  double *qf = zalloc(nf), *qf2 = zalloc(nf), *qbp = zalloc(4 * (size_t)npoin);
  double *qp2 = zalloc(nq3), *q2 = zalloc(nq3), *dpp2 = zalloc((size_t)npoin * L);
  int rc = 0;
  /* prediction (ti_rk_bcl.F90:43-57) */
  extract_qprime_df_face(o, qf, qprime_df);
  memcpy(qbp, qb_df, sizeof(double) * 4 * npoin);
  set_dpprime_visc(o, qprime_df);
  btp_bcl_coeffs(o, qf, qprime_df);
  ti_barotropic_ssprk(o, qbp, qprime_df);
  memcpy(q2, q_df, sizeof(double) * nq3);
  memcpy(qp2, qprime_df, sizeof(double) * nq3);
  memcpy(qf2, qf, sizeof(double) * nf);
  rc = momentum_mass(o, q2, qf2, qp2, qbp);
  if (rc) goto done;
  /* correction (ti_rk_bcl.F90:62-85) */
  for (size_t i = 0; i < nq3; i++) qp2[i] = 0.5 * (qp2[i] + qprime_df[i]);
  for (size_t i = 0; i < nf; i++) qf2[i] = 0.5 * (qf[i] + qf2[i]);
  set_dpprime_visc(o, qp2);
  btp_bcl_coeffs(o, qf2, qp2);
  ti_barotropic_ssprk(o, qb_df, qp2);
  rc = thickness(o, qp2, q_df, qb_df, qf2);
  if (rc) goto done;
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++) {
      A2(dpp2, I, k, npoin) = A3(qp2, 1, I, k, 3, npoin);
      A3(qp2, 1, I, k, 3, npoin) = 0.5 * (A3(qprime_df, 1, I, k, 3, npoin) + A2(dpp2, I, k, npoin));
    }
  for (size_t i = 0; i < nf; i += 3) qf2[i] = 0.5 * (qf[i] + qf2[i]);
  momentum(o, q_df, qp2, qb_df, qf2);
  for (int k = 1; k <= L; k++)
    for (int I = 1; I <= npoin; I++) {
      A3(qprime_df, 1, I, k, 3, npoin) = A2(dpp2, I, k, npoin);
      A3(qprime_df, 2, I, k, 3, npoin) = A3(qp2, 2, I, k, 3, npoin);
      A3(qprime_df, 3, I, k, 3, npoin) = A3(qp2, 3, I, k, 3, npoin);
    }
done:
  free(qf);
  free(qf2);
  free(qbp);
  free(qp2);
  free(q2);
  free(dpp2);
  return rc;
}

int oracle_btp_bcl_coeffs(oracle *o, const double *qprime_df) {
  double *qf = zalloc(6 * (size_t)o->ngl * o->nface * o->L);
  extract_qprime_df_face(o, qf, qprime_df);
  set_dpprime_visc(o, qprime_df);
  btp_bcl_coeffs(o, qf, qprime_df);
  free(qf);
  return 0;
}

int oracle_ti_barotropic_ssprk(oracle *o, double *qb_df, const double *qprime_df) {
  ti_barotropic_ssprk(o, qb_df, qprime_df);
  return 0;
}

int oracle_create_rhs_btp(oracle *o, double *rhs, const double *qb_df, const double *qprime_df) {
  create_rhs_btp(o, rhs, qb_df, qprime_df);
  return 0;
}

/* The prediction half of ti_rk_bcl (ti_rk_bcl.F90:43-57) in place: q_df, qb_df, qprime_df
 * become q_df2, qbp_df, qprime_df2 -- the parity hook for momentum_mass (and through it the
 * ad_mlswe > 0 shear stress), whose reference counterpart is oracle/ref_driver mode 4. */
int oracle_predict(oracle *o, double *q_df, double *qb_df, double *qprime_df) {
  double *qf = zalloc(6 * (size_t)o->ngl * o->nface * o->L);
  extract_qprime_df_face(o, qf, qprime_df);
  set_dpprime_visc(o, qprime_df);
  btp_bcl_coeffs(o, qf, qprime_df);
  ti_barotropic_ssprk(o, qb_df, qprime_df);
  int rc = momentum_mass(o, q_df, qf, qprime_df, qb_df);
  free(qf);
  return rc;
}

void oracle_zero_accumulators(oracle *o) { zero_btp_accumulators(o); }

const char *oracle_last_error(const oracle *o) { return o->err; }

#define FIELD(nm, ptr, cnt) \
  if (!strcmp(name, nm)) {  \
    p = (ptr);              \
    cnt_ = (cnt);           \
  }
int oracle_get_field(oracle *o, const char *name, double *out, int64_t n) {
  size_t Nq = (size_t)o->npoin_q, N = (size_t)o->npoin, nqf = (size_t)o->nq * o->nface;
  size_t ngf = (size_t)o->ngl * o->nface, L = (size_t)o->L;
  const double *p = NULL;
  size_t cnt_ = 0;
  FIELD("Q_uu_dp", o->Q_uu_dp, Nq) FIELD("Q_uv_dp", o->Q_uv_dp, Nq) FIELD("Q_vv_dp", o->Q_vv_dp, Nq)
  FIELD("H_bcl", o->H_bcl, Nq) FIELD("Q_uu_dp_edge", o->Q_uu_dp_edge, nqf)
  FIELD("Q_uv_dp_edge", o->Q_uv_dp_edge, nqf) FIELD("Q_vv_dp_edge", o->Q_vv_dp_edge, nqf)
  FIELD("H_bcl_edge", o->H_bcl_edge, nqf) FIELD("ope_ave", o->ope_ave, Nq) FIELD("H_ave", o->H_ave, Nq)
  FIELD("Qu_ave", o->Qu_ave, Nq) FIELD("Qv_ave", o->Qv_ave, Nq) FIELD("Quv_ave", o->Quv_ave, Nq)
  FIELD("ope2_ave", o->ope2_ave, Nq) FIELD("btp_mass_flux_ave", o->btp_mass_flux_ave, 2 * Nq)
  FIELD("uvb_ave", o->uvb_ave, 2 * Nq) FIELD("tau_bot_ave", o->tau_bot_ave, 2 * Nq)
  FIELD("tau_wind_ave", o->tau_wind_ave, 2 * Nq) FIELD("ope2_ave_df", o->ope2_ave_df, N)
  FIELD("uvb_ave_df", o->uvb_ave_df, 2 * N) FIELD("uvb_face_ave", o->uvb_face_ave, 4 * nqf)
  FIELD("btp_mass_flux_face_ave", o->btp_mass_flux_face_ave, 2 * nqf)
  FIELD("ope_face_ave", o->ope_face_ave, 2 * nqf) FIELD("ope2_face_ave", o->ope2_face_ave, 2 * nqf)
  FIELD("Qu_face_ave", o->Qu_face_ave, 2 * nqf) FIELD("Qv_face_ave", o->Qv_face_ave, 2 * nqf)
  FIELD("Quv_face_ave", o->Quv_face_ave, 2 * nqf) FIELD("H_face_ave", o->H_face_ave, nqf)
  FIELD("one_plus_eta_edge_2_ave", o->one_plus_eta_edge_2_ave, nqf)
  FIELD("dpprime_visc", o->dpprime_visc, N * L) FIELD("pbprime_visc", o->pbprime_visc, N)
  FIELD("btp_dpp_graduv", o->btp_dpp_graduv, 4 * N) FIELD("dpp_graduv", o->dpp_graduv, 4 * N * L)
  FIELD("graduv_dpp_face", o->graduv_dpp_face, 10 * ngf * L)
  FIELD("btp_graduv_dpp_face", o->btp_graduv_dpp_face, 10 * ngf)
  FIELD("graduvb_face_ave", o->graduvb_face_ave, 8 * ngf) FIELD("graduvb_ave", o->graduvb_ave, 4 * N)
  FIELD("sum_layer_mass_flux", o->sum_layer_mass_flux, 2 * Nq)
  FIELD("sum_layer_mass_flux_face", o->sum_layer_mass_flux_face, 2 * nqf)
  if (!p) return set_err(o, HNUMO_ERR_INVALID, "unknown field");
  if ((size_t)n != cnt_) return set_err(o, HNUMO_ERR_INVALID, "field size mismatch");
  memcpy(out, p, sizeof(double) * cnt_);
  return 0;
}

int oracle_create(const hnumo_mesh_desc *m, const hnumo_static_desc *s, const hnumo_params *p, oracle **out) {
  oracle *o = (oracle *)calloc(1, sizeof(oracle));
  *out = o;
  o->m = *m;
  o->s = *s;
  o->p = *p;
  o->ngl = m->ngl;
  o->nq = m->nq;
  o->npts = m->ngl * m->ngl;
  o->npoin = m->npoin;
  o->npoin_q = m->npoin_q;
  o->nface = m->nface;
  o->nelem = m->nelem;
  o->L = m->nlayers;
  if (p->method_visc == 1 && (!m->imapl_q || !m->imapr_q))
    return set_err(o, HNUMO_ERR_INVALID, "method_visc==1 needs imapl_q/imapr_q");
  if (o->L < 1 || o->L > 3) return set_err(o, HNUMO_ERR_INVALID, "nlayers must be 1..3 (qp(k) quirk)");
  if (o->nq > 32 || !m->psih || !m->index_df) return set_err(o, HNUMO_ERR_INVALID, "dense tables required");
  size_t Nq = (size_t)o->npoin_q, N = (size_t)o->npoin, nqf = (size_t)o->nq * o->nface;
  size_t ngf = (size_t)o->ngl * o->nface, L = (size_t)o->L;
  o->Q_uu_dp = zalloc(Nq); o->Q_uv_dp = zalloc(Nq); o->Q_vv_dp = zalloc(Nq); o->H_bcl = zalloc(Nq);
  o->Q_uu_dp_edge = zalloc(nqf); o->Q_uv_dp_edge = zalloc(nqf); o->Q_vv_dp_edge = zalloc(nqf);
  o->H_bcl_edge = zalloc(nqf);
  o->ope_ave = zalloc(Nq); o->H_ave = zalloc(Nq); o->Qu_ave = zalloc(Nq); o->Qv_ave = zalloc(Nq);
  o->Quv_ave = zalloc(Nq); o->ope2_ave = zalloc(Nq);
  o->btp_mass_flux_ave = zalloc(2 * Nq); o->uvb_ave = zalloc(2 * Nq); o->tau_bot_ave = zalloc(2 * Nq);
  o->tau_wind_ave = zalloc(2 * Nq);
  o->ope2_ave_df = zalloc(N); o->uvb_ave_df = zalloc(2 * N);
  o->uvb_face_ave = zalloc(4 * nqf);
  o->btp_mass_flux_face_ave = zalloc(2 * nqf); o->ope_face_ave = zalloc(2 * nqf);
  o->ope2_face_ave = zalloc(2 * nqf); o->Qu_face_ave = zalloc(2 * nqf); o->Qv_face_ave = zalloc(2 * nqf);
  o->Quv_face_ave = zalloc(2 * nqf); o->H_face_ave = zalloc(nqf); o->one_plus_eta_edge_2_ave = zalloc(nqf);
  o->dpprime_visc = zalloc(N * L); o->dpprime_visc_q = zalloc(Nq * L); o->pbprime_visc = zalloc(N); o->btp_dpp_graduv = zalloc(4 * N);
  o->dpp_graduv = zalloc(4 * N * L); o->graduv_dpp_face = zalloc(10 * ngf * L);
  o->btp_graduv_dpp_face = zalloc(10 * ngf); o->graduvb_face_ave = zalloc(8 * ngf);
  o->graduvb_ave = zalloc(4 * N); o->sum_layer_mass_flux = zalloc(2 * Nq);
  o->sum_layer_mass_flux_face = zalloc(2 * nqf);
  return 0;
}

void oracle_destroy(oracle *o) {
  if (!o) return;
  double **ptrs[] = {&o->Q_uu_dp, &o->Q_uv_dp, &o->Q_vv_dp, &o->H_bcl, &o->Q_uu_dp_edge, &o->Q_uv_dp_edge,
                     &o->Q_vv_dp_edge, &o->H_bcl_edge, &o->ope_ave, &o->H_ave, &o->Qu_ave, &o->Qv_ave,
                     &o->Quv_ave, &o->ope2_ave, &o->btp_mass_flux_ave, &o->uvb_ave, &o->tau_bot_ave,
                     &o->tau_wind_ave, &o->ope2_ave_df, &o->uvb_ave_df, &o->uvb_face_ave,
                     &o->btp_mass_flux_face_ave, &o->ope_face_ave, &o->ope2_face_ave, &o->Qu_face_ave,
                     &o->Qv_face_ave, &o->Quv_face_ave, &o->H_face_ave, &o->one_plus_eta_edge_2_ave,
                     &o->dpprime_visc, &o->dpprime_visc_q, &o->pbprime_visc, &o->btp_dpp_graduv, &o->dpp_graduv,
                     &o->graduv_dpp_face, &o->btp_graduv_dpp_face, &o->graduvb_face_ave, &o->graduvb_ave,
                     &o->sum_layer_mass_flux, &o->sum_layer_mass_flux_face};
  for (size_t i = 0; i < sizeof ptrs / sizeof ptrs[0]; i++) free(*ptrs[i]);
  free(o);
}
