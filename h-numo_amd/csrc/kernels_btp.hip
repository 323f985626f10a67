// kernels_btp.hip -- barotropic SSP-RK stage as one fused CDNA4 kernel per stage.
//
// One workgroup (BS threads) owns one element.  A stage (ti_barotropic_ssprk_mlswe body,
// mod_rk_mlswe.F90:87-114) is:
//   create_rhs_btp (mod_rhs_btp.F90:28-59)
//     = volume term  create_rhs_btp_volume_qdf (:102-209)
//     + face fluxes  creat_btp_fluxes_qdf       (:211-370), traces btp_extract_df
//                                               (mod_barotropic_terms.F90:25-97)
//     + LDG viscosity btp_create_laplacian (mod_laplacian_quad.F90:32-121)
//   then the Shu-Osher update and the wall fix btp_mom_boundary_df (:165-217).
//
// Arithmetic is the reference's, term by term and in the reference's summation order
// (the momentum RHS cancels to ~1e-8 relative, so any reordering shows up in the state):
// the dense psih/dpsidx tables are regenerated on the fly from the 1-D bases (same
// products), and every ordered sum is accumulated sequentially by one thread.
//
// The kernel is latency-bound at one workgroup per element, so it is organised to keep
// every dependent chain short and every SIMD busy:
//   A  all element-indexed loads (state, metrics, neighbour traces) in one round trip
//   B  quad-point physics | nodal grad(u_bar) | face fluxes       (concurrent task ranges)
//   D0..D_NCH  weak-form terms T(v,p,q) computed in parallel per chunk of quad rows into
//      LDS (double buffered) while the previous chunk is summed in quad order by one
//      thread per (v,p); LDG face fluxes, qq and the Laplacian sums ride along
//   E  update + wall fix, then the state and the face traces the neighbours need next
//      stage, written straight into the neighbours' trace slots (no gather next stage).
// With psi(i,k) the identity at LGL nodes (checked on the host), the nodal derivative
// sums keep only their 2*NGL-1 nonzero terms, in order (the zero terms add +-0).
#include "engine_internal.h"

namespace hnumo {

struct StageArgs {
  DevMesh m;
  const double *qb_in, *qb0, *qb2, *qprime;  // qb(4,npoin); qprime(3,npoin,L)
  const double *qcoef;                       // [QC_N][npoin_q]
  const double *ncoef;                       // [NC_N][npoin]
  const double *fcoef;                       // [FC_N][F*NQ]
  const double *fncoef;                      // [10][F*NGL]  btp_graduv_dpp_face(v,s) at v+5*s
  const double *trace_in;                    // [E][4][8][NGL] neighbour qb(4) + grad(4) face traces
  double *trace_out;
  double *qacc, *facc, *nacc, *gfacc;        // accumulators (see engine_internal.h)
  double *qb_out;                            // stage result, qb(4,npoin)
  double *rhs_out;                           // rhs(3,npoin) in rhs-only mode
  double a1, a2, a3, dtt;
  int rhs_only, write_trace, accumulate;
  unsigned long long *prof;                  // optional [E][12] phase timestamps (diagnostics)
};

#define STAGE_MARK(k) \
  if (a.prof && tid == 0) s_prof[k] = clock64();

template <int NGL, int NQ>
struct StageCfg {
  static constexpr int P = NGL * NGL, Q = NQ * NQ;
  static constexpr int BS = (Q <= 25) ? 128 : 256;
  static constexpr int TBYTES = (P <= 25) ? 36864 : 65536;  // LDS for the two term buffers
  static constexpr int RCMAX0 = TBYTES / (2 * 3 * P * NQ * 8);
  static constexpr int RCMAX = RCMAX0 < 1 ? 1 : RCMAX0;
  static constexpr int NCH = (NQ + RCMAX - 1) / RCMAX;      // chunks of quad rows
  static constexpr int RC = (NQ + NCH - 1) / NCH;           // rows per chunk
  static constexpr int QC = RC * NQ;                        // quad points per chunk
  static constexpr int MINW = (BS == 256) ? 3 : 4;          // waves/SIMD wanted
  // one LDS arena: term buffers T0 | T1; the quad statics (A->B) are staged over T0, the
  // old quad accumulators (A->B) and the face increments (B->D0) over T1, before either
  // term buffer is written
  static constexpr int TSZ = 3 * P * QC;
  static constexpr int NSTAT = 11;                          // 7 quad statics + 4 sub-cycle coefficients
  static constexpr int OFF_ADD = TSZ > NSTAT * Q ? TSZ : NSTAT * Q;
  static constexpr int NADD = QA_N * Q + FA_N * 4 * NQ;
  static constexpr int ARENA = (2 * TSZ > OFF_ADD + NADD) ? 2 * TSZ : OFF_ADD + NADD;
};

// The 2*NGL-1 nonzero source nodes of a nodal derivative at node (i,j), in the reference
// loop order (outer index jj / mm, inner ii / n): r < j -> (jj=r, ii=i); j <= r < j+NGL ->
// (jj=j, ii=r-j); r >= j+NGL -> (jj=r-NGL+1, ii=i).  Uniform trip count, no divergence.
template <int NGL>
__device__ __forceinline__ void nz_term(int r, int i, int j, int &jj, int &ii) {
  if (r < j) {
    jj = r;
    ii = i;
  } else if (r < j + NGL) {
    jj = j;
    ii = r - j;
  } else {
    jj = r - NGL + 1;
    ii = i;
  }
}

// grad of u_bar at node (i,j) along one metric pair: sum over source nodes (mm,n) of
// (HE_DF(n,mm,i,j)*ex + HN_DF(n,mm,i,j)*nx) * u(mm,n)  (mod_barotropic_terms.F90:427-441),
// nonzero terms only (mm==j or n==i), in the reference order.
template <int NGL>
__device__ __forceinline__ double nodal_grad(const double *s_dpsi, int i, int j, double ex, double nx,
                                             const double (*s_qb)[4], int comp) {
  double gsum = 0.0;
#pragma unroll
  for (int r = 0; r < 2 * NGL - 1; r++) {
    int mm, n;
    nz_term<NGL>(r, i, j, mm, n);
    const int s = mm * NGL + n;
    const double u = s_qb[s][comp] / s_qb[s][0];
    double d;
    if (mm == j)
      d = (n == i) ? s_dpsi[i * NGL + i] * ex + s_dpsi[j * NGL + j] * nx : s_dpsi[n * NGL + i] * ex;
    else
      d = s_dpsi[mm * NGL + j] * nx;
    gsum = gsum + d * u;
  }
  return gsum;
}

template <int NGL, int NQ>
__global__ void __launch_bounds__((StageCfg<NGL, NQ>::BS), (StageCfg<NGL, NQ>::MINW)) btp_stage_kernel(StageArgs a) {
  using C = StageCfg<NGL, NQ>;
  constexpr int P = C::P, Q = C::Q, BS = C::BS, NCH = C::NCH, RC = C::RC, QC = C::QC;
  const DevMesh &m = a.m;
  const int e = blockIdx.x, tid = threadIdx.x;
  const int npoin = m.npoin, npq = m.npoin_q, F = m.nface;
  const size_t FQ = (size_t)F * NQ, FN = (size_t)F * NGL;

  __shared__ double s_psiq[NGL * NQ], s_dpsiq[NGL * NQ], s_dpsi[NGL * NGL];
  __shared__ double s_qb[P][4];      // stage input state at the nodes
  __shared__ double s_qp[P][4];      // qprime of the bottom layer (dp, u, v)
  __shared__ double s_q0[P][4], s_q2[P][4];  // Shu-Osher operands qb0 / qb2 (components 1..3)
  __shared__ double s_nm[7][P];      // nodal e_x, e_y, n_x, n_y, w, massinv, pbprime
  __shared__ double s_grad[4][P], s_qq[4][P];
  __shared__ double s_qd[Q][12];     // per quad point: wq, ex, ey, nx, ny, udp, vdp, scx, scy, Hq+qu, quv, Hq+qv
  __shared__ double s_tr[4][8][NGL]; // neighbour traces per local face: qb(4), grad(4)
  __shared__ double s_fq[4][NQ][4];  // face: wq, flux, H_kx+flux_x, H_ky+flux_y
  __shared__ double s_fl[4][NGL][2]; // LDG face: signed wq*flux_qu, wq*flux_qv
  __shared__ double s_rhs[3][P], s_lap[2][P];
  __shared__ double s_qn[P][4];
  __shared__ double s_arena[C::ARENA];
  double (*s_stat)[Q] = reinterpret_cast<double (*)[Q]>(s_arena);                    // [11][Q]
  double (*s_qadd)[Q] = reinterpret_cast<double (*)[Q]>(s_arena + C::OFF_ADD);       // [12][Q] old qacc
  double (*s_fadd)[4 * NQ] = reinterpret_cast<double (*)[4 * NQ]>(s_arena + C::OFF_ADD + QA_N * Q);  // [16][4NQ]
  __shared__ int s_map[4][NGL], s_face[4], s_side[4], s_bc[4], s_nbe[4], s_nblf[4];
  __shared__ int s_pf[P][2];         // (lf*NGL+n) of the <=2 faces through node p, lf order; -1 none

  // ------------------------------------------------------------- A: loads
  __shared__ unsigned long long s_prof[12];
  if (a.prof && tid == 0) s_prof[10] = wall_clock64();
  STAGE_MARK(0);
  for (int t = tid; t < NGL * NQ; t += BS) {
    s_psiq[t] = m.basis[t];
    s_dpsiq[t] = m.basis[NGL * NQ + t];
  }
  for (int t = tid; t < NGL * NGL; t += BS) s_dpsi[t] = m.basis[2 * NGL * NQ + t];
  if (tid < 4) {
    s_face[tid] = m.efaces[e * 4 + tid];
    s_side[tid] = m.eside[e * 4 + tid];
    s_bc[tid] = m.ebc[e * 4 + tid];
    s_nbe[tid] = m.enbr_e[e * 4 + tid];
    s_nblf[tid] = m.enbr_lf[e * 4 + tid];
  }
  for (int t = tid; t < 4 * NGL; t += BS) s_map[t / NGL][t % NGL] = m.efmap[e * 4 * NGL + t];
  for (int t = tid; t < 4 * P; t += BS) s_qb[t / 4][t % 4] = a.qb_in[(size_t)e * 4 * P + t];
  if (m.botfr) {
    const double *qpL = a.qprime + (size_t)(m.L - 1) * 3 * npoin + (size_t)e * 3 * P;
    for (int t = tid; t < 3 * P; t += BS) s_qp[t / 3][t % 3] = qpL[t];
  }
  if (!a.rhs_only) {
    if (a.a1 != 0.0)
      for (int t = tid; t < 4 * P; t += BS) s_q0[t / 4][t % 4] = a.qb0[(size_t)e * 4 * P + t];
    if (a.a3 != 0.0)
      for (int t = tid; t < 4 * P; t += BS) s_q2[t / 4][t % 4] = a.qb2[(size_t)e * 4 * P + t];
  }
  for (int t = tid; t < 4 * Q; t += BS) {
    const int c = t / Q, q = t % Q;
    s_qd[q][1 + c] = m.qstat[(QS_EX + c) * (size_t)npq + (size_t)e * Q + q];
  }
  if (a.accumulate)
    for (int t = tid; t < QA_N * Q; t += BS) {
      const int c = t / Q, q = t % Q;
      s_qadd[c][q] = a.qacc[c * (size_t)npq + (size_t)e * Q + q];
    }
  for (int t = tid; t < C::NSTAT * Q; t += BS) {
    const int c = t / Q, q = t % Q;
    const size_t Iq = (size_t)e * Q + q;
    s_stat[c][q] = c < 7 ? m.qstat[(QS_W + c) * (size_t)npq + Iq] : a.qcoef[(c - 7) * (size_t)npq + Iq];
  }
  for (int t = tid; t < 7 * P; t += BS) {
    const int c = t / P, p = t % P;
    const int fld = c < 4 ? NS_EX + c : (c == 4 ? NS_W : (c == 5 ? NS_MINV : NS_PB));
    s_nm[c][p] = m.nstat[fld * (size_t)npoin + (size_t)e * P + p];
  }
  for (int t = tid; t < 4 * 8 * NGL; t += BS) (&s_tr[0][0][0])[t] = a.trace_in[(size_t)e * 32 * NGL + t];
  __syncthreads();
  STAGE_MARK(1);

  // ------------------------------------------------------------- B
  {
    constexpr int WQ = Q, WG = 4 * P, WF = 4 * NQ;
    for (int w = tid; w < WQ + WG + WF; w += BS) {
      asm volatile("" ::: "memory");
      if (w < WQ) {
        // ---- quad-point physics (mod_rhs_btp.F90:136-192)
        const int q = w, iq = q % NQ, jq = q / NQ;
        double pa[NGL], pb[NGL];
#pragma unroll
        for (int n = 0; n < NGL; n++) {
          pa[n] = s_psiq[n * NQ + iq];
          pb[n] = s_psiq[n * NQ + jq];
        }
        double dp = 0, dpp = 0, udp = 0, vdp = 0, pp = 0, up = 0, vp = 0;
#pragma unroll 1
        for (int mm = 0; mm < NGL; mm++)
#pragma unroll
          for (int n = 0; n < NGL; n++) {
            const int ip = mm * NGL + n;
            const double hi = pa[n] * pb[mm];  // PSIH(n,mm,iq,jq)
            dp = dp + hi * s_qb[ip][0];
            dpp = dpp + hi * s_qb[ip][1];
            udp = udp + hi * s_qb[ip][2];
            vdp = vdp + hi * s_qb[ip][3];
          }
        if (m.botfr) {
#pragma unroll
          for (int mm = 0; mm < NGL; mm++)
#pragma unroll
            for (int n = 0; n < NGL; n++) {
              const int ip = mm * NGL + n;
              const double hi = pa[n] * pb[mm];
              pp = pp + hi * s_qp[ip][0];
              up = up + hi * s_qp[ip][1];
              vp = vp + hi * s_qp[ip][2];
            }
        }
        const double wq = s_stat[QS_W][q], cor = s_stat[QS_COR][q];
        const double tw1 = s_stat[QS_TW1][q], tw2 = s_stat[QS_TW2][q];
        const double gz1 = s_stat[QS_GZ1][q], gz2 = s_stat[QS_GZ2][q], oop = s_stat[QS_OOP][q];
        const double chb = s_stat[7 + QC_HBCL][q], cuu = s_stat[7 + QC_QUU][q];
        const double cuv = s_stat[7 + QC_QUV][q], cvv = s_stat[7 + QC_QVV][q];
        const double ub = udp / dp, vb = vdp / dp;
        double tb_u = 0.0, tb_v = 0.0;
        if (m.botfr == 1) {
          const double ubot = up + ub, vbot = vp + vb;
          const double spd = (m.cd / m.gravity) * pp;
          tb_u = spd * ubot;
          tb_v = spd * vbot;
        } else if (m.botfr == 2) {
          const double ubot = up + ub, vbot = vp + vb;
          const double spd = (m.cd / m.alpha[m.L - 1]) * sqrt(ubot * ubot + vbot * vbot);
          tb_u = spd * ubot;
          tb_v = spd * vbot;
        }
        const double g = m.gravity;
        const double sc_x = cor * vdp + g * (tw1 - tb_u) - g * dp * gz1;
        const double sc_y = -cor * udp + g * (tw2 - tb_v) - g * dp * gz2;
        const double ope = 1.0 + dpp * oop;
        const double Hq = (ope * ope) * chb;
        const double qu = ub * udp + ope * cuu;
        const double quv = ub * vdp + ope * cuv;
        const double qv = vb * vdp + ope * cvv;
        if (a.accumulate) {  // time averages (old values staged in A)
          double add[QA_N];
          add[QA_H] = Hq; add[QA_QU] = qu; add[QA_QV] = qv; add[QA_QUV] = quv;
          add[QA_TBU] = tb_u; add[QA_TBV] = tb_v; add[QA_OPE] = ope; add[QA_OPE2] = ope * ope;
          add[QA_MFX] = udp; add[QA_MFY] = vdp; add[QA_UB] = ub; add[QA_VB] = vb;
          const size_t Iq = (size_t)e * Q + q;
#pragma unroll
          for (int k = 0; k < QA_N; k++) a.qacc[k * (size_t)npq + Iq] = s_qadd[k][q] + add[k];
        }
        s_qd[q][0] = wq;
        s_qd[q][5] = udp;
        s_qd[q][6] = vdp;
        s_qd[q][7] = sc_x;
        s_qd[q][8] = sc_y;
        s_qd[q][9] = Hq + qu;
        s_qd[q][10] = quv;
        s_qd[q][11] = Hq + qv;
      } else if (w < WQ + WG) {
        // ---- nodal grad(u_bar) (compute_gradient_uv) + stage-start nodal averages
        const int t = w - WQ, c = t / P, p = t % P, i = p % NGL, j = p / NGL;
        const double ex = s_nm[(c & 1) ? 1 : 0][p], nx = s_nm[(c & 1) ? 3 : 2][p];
        const size_t I = (size_t)e * P + p;
        // all global reads of the task first (one round trip), then the stores
        double g_old = 0.0, o_old = 0.0, u_old = 0.0, v_old = 0.0, oop = 0.0;
        if (a.accumulate) {
          g_old = a.nacc[(NA_G1 + c) * (size_t)npoin + I];
          if (c == 0) {
            o_old = a.nacc[NA_OPE2 * (size_t)npoin + I];
            u_old = a.nacc[NA_UB * (size_t)npoin + I];
            v_old = a.nacc[NA_VB * (size_t)npoin + I];
            oop = m.nstat[NS_OOP * (size_t)npoin + I];
          }
        }
        if (c == 0) {
          int k = 0, f0 = -1, f1 = -1;
          for (int r = 0; r < 4 * NGL; r++)
            if (s_map[r / NGL][r % NGL] == p) {
              if (k == 0) f0 = r; else f1 = r;
              k++;
            }
          s_pf[p][0] = f0;
          s_pf[p][1] = f1;
        }
        const double gsum = nodal_grad<NGL>(s_dpsi, i, j, ex, nx, s_qb, 2 + (c >> 1));
        s_grad[c][p] = gsum;
        if (a.accumulate) {
          a.nacc[(NA_G1 + c) * (size_t)npoin + I] = g_old + gsum;
          if (c == 0) {  // mod_rk_mlswe.F90:90-92
            const double q1 = s_qb[p][0], q2 = s_qb[p][1], q3 = s_qb[p][2], q4 = s_qb[p][3];
            const double t1 = 1.0 + q2 * oop;
            a.nacc[NA_OPE2 * (size_t)npoin + I] = o_old + t1 * t1;
            a.nacc[NA_UB * (size_t)npoin + I] = u_old + q3 / q1;
            a.nacc[NA_VB * (size_t)npoin + I] = v_old + q4 / q1;
          }
        }
      } else {
        // ---- creat_btp_fluxes_qdf at (face lf, quad iq) (mod_rhs_btp.F90:246-337)
        const int t = w - WQ - WG, lf = t / NQ, iq = t % NQ;
        const int f = s_face[lf], side = s_side[lf], er = s_bc[lf];
        const size_t fq = (size_t)f * NQ + iq;
        const double *FS = m.fstat;
        const double nxl = FS[FS_NX * FQ + fq], nyl = FS[FS_NY * FQ + fq], fw = FS[FS_W * FQ + fq];
        const double fcl = FS[FS_CL * FQ + fq], fcr = FS[FS_CR * FQ + fq], fclr = FS[FS_CLR * FQ + fq];
        const double cml = FS[FS_CML * FQ + fq], cmr = FS[FS_CMR * FQ + fq], cmlr = FS[FS_CMLR * FQ + fq];
        const double oope = FS[FS_OOPE * FQ + fq];
        const double *FC = a.fcoef;
        const double fquu = FC[FC_QUU * FQ + fq], fquv = FC[FC_QUV * FQ + fq], fqvv = FC[FC_QVV * FQ + fq];
        const double fhb = FC[FC_HBCL * FQ + fq];
        double pbn[2][NGL];
#pragma unroll
        for (int n = 0; n < NGL; n++) {
          pbn[0][n] = m.fnstat[FN_PBL * FN + (size_t)f * NGL + n];
          pbn[1][n] = m.fnstat[FN_PBR * FN + (size_t)f * NGL + n];
        }
        double ql[4] = {0, 0, 0, 0}, qr[4] = {0, 0, 0, 0}, pbl = 0.0, pbr = 0.0;
#pragma unroll
        for (int n = 0; n < NGL; n++) {
          const double hi = s_psiq[n * NQ + iq];
          const int p = s_map[lf][n];
          double own[4] = {s_qb[p][0], s_qb[p][1], s_qb[p][2], s_qb[p][3]};
          double oth[4];
          if (er > 0) {
#pragma unroll
            for (int c = 0; c < 4; c++) oth[c] = s_tr[lf][c][n];
          } else {
            // ghost state of btp_extract_df (mod_barotropic_terms.F90:75-91)
#pragma unroll
            for (int c = 0; c < 4; c++) oth[c] = own[c];
            if (er == -4) {
              const double nxn = m.fnstat[FN_NX * FN + (size_t)f * NGL + n];
              const double nyn = m.fnstat[FN_NY * FN + (size_t)f * NGL + n];
              const double un = nxn * own[2] + nyn * own[3];
              oth[2] = own[2] - 2.0 * un * nxn;
              oth[3] = own[3] - 2.0 * un * nyn;
            } else if (er == -2) {
              oth[2] = -own[2];
              oth[3] = -own[3];
            }
          }
#pragma unroll
          for (int c = 0; c < 4; c++) {
            const double l = side == 0 ? own[c] : oth[c], r = side == 0 ? oth[c] : own[c];
            ql[c] = ql[c] + hi * l;
            qr[c] = qr[c] + hi * r;
          }
          pbl = pbl + hi * pbn[0][n];
          pbr = pbr + hi * pbn[1][n];
        }
        const double nxr = -nxl, nyr = -nyl;
        const double pU_L = nxl * ql[2] + nyl * ql[3];
        const double pU_R = nxr * qr[2] + nyr * qr[3];
        const double pbpert_edge = fcl * ql[1] + fcr * qr[1] + fclr * (pU_L + pU_R);
        const double ope_e = 1.0 + pbpert_edge * oope;
        const double fex = cml * ql[2] + cmr * qr[2] + cmlr * (nxl * ql[1] + nxr * qr[1]);
        const double fey = cml * ql[3] + cmr * qr[3] + cmlr * (nyl * ql[1] + nyr * qr[1]);
        const double ul = ql[2] / ql[0], ur = qr[2] / qr[0], vl = ql[3] / ql[0], vr = qr[3] / qr[0];
        const double quu = 0.5 * (ul * ql[2] + ur * qr[2]) + ope_e * fquu;
        const double quv = 0.5 * (vl * ql[2] + vr * qr[2]) + ope_e * fquv;
        const double qvu = 0.5 * (ul * ql[3] + ur * qr[3]) + ope_e * fquv;
        const double qvv = 0.5 * (vl * ql[3] + vr * qr[3]) + ope_e * fqvv;
        const double Hf = (ope_e * ope_e) * fhb;
        {  // face time-average increments, added in D0 (face's left element only)
          const double opl = 1.0 + (ql[1] / pbl), opr = 1.0 + (qr[1] / pbr);
          double *ad = &s_fadd[0][t];
          constexpr int S = 4 * NQ;
          ad[FA_MFX * S] = fex; ad[FA_MFY * S] = fey; ad[FA_H * S] = Hf; ad[FA_QUU * S] = quu;
          ad[FA_QUV * S] = quv; ad[FA_QVU * S] = qvu; ad[FA_QVV * S] = qvv; ad[FA_OPEL * S] = opl;
          ad[FA_OPER * S] = opr; ad[FA_OPE2L * S] = opl * opl; ad[FA_OPE2R * S] = opr * opr;
          ad[FA_OPEE2 * S] = ope_e * ope_e; ad[FA_UL * S] = ul; ad[FA_UR * S] = ur; ad[FA_VL * S] = vl;
          ad[FA_VR * S] = vr;
        }
        const double H_kx = nxl * Hf, H_ky = nyl * Hf;
        const double lamb = cmlr;
        const double dispu = 0.5 * lamb * (qr[2] - ql[2]);
        const double dispv = 0.5 * lamb * (qr[3] - ql[3]);
        const double flux_x = nxl * quu + nyl * quv - dispu;
        const double flux_y = nxl * qvu + nyl * qvv - dispv;
        const double flux = nxl * fex + nyl * fey;
        s_fq[lf][iq][0] = fw;
        s_fq[lf][iq][1] = flux;
        s_fq[lf][iq][2] = H_kx + flux_x;
        s_fq[lf][iq][3] = H_ky + flux_y;
      }
    }
  }
  __syncthreads();
  STAGE_MARK(2);

  // ------------------------------------------------------------- D0 .. D_NCH
  // term task (q in chunk, i): T(v, p=(i,j), q) for j = 0..NGL-1
  // (create_rhs_btp_volume_qdf, mod_rhs_btp.F90:194-206: rhs(v,I) += wq*(...))
  auto term_task = [&](int k, int t) {
    const int buf = k & 1;
    const int qi = t / NGL, i = t % NGL;
    const int q = k * QC + qi, iq = q % NQ, jq = q / NQ;
    const double *d = s_qd[q];
    const double wq = d[0], ex = d[1], ey = d[2], nx = d[3], ny = d[4];
    const double udp = d[5], vdp = d[6], scx = d[7], scy = d[8], A = d[9], quv = d[10], B = d[11];
    const double pi = s_psiq[i * NQ + iq], dpi = s_dpsiq[i * NQ + iq];
#pragma unroll
    for (int j = 0; j < NGL; j++) {
      const double pj = s_psiq[j * NQ + jq], dpj = s_dpsiq[j * NQ + jq];
      const double hi = pi * pj, h_e = dpi * pj, h_n = pi * dpj;
      const double dhdx = h_e * ex + h_n * nx;
      const double dhdy = h_e * ey + h_n * ny;
      const int p = j * NGL + i;
      double *T = s_arena + buf * C::TSZ;
      T[p * QC + qi] = wq * (dhdx * udp + dhdy * vdp);
      T[(P + p) * QC + qi] = wq * (hi * scx + dhdx * A + quv * dhdy);
      T[(2 * P + p) * QC + qi] = wq * (hi * scy + dhdx * quv + dhdy * B);
    }
  };
  // sum task (v, p): rhs(v,p) += T over the chunk in quad order; faces after the last chunk
  auto sum_task = [&](int k, int t) {
    const int buf = k & 1, v = t / P, p = t % P;
    const int nq_k = (k == NCH - 1) ? Q - k * QC : QC;
    double acc = k == 0 ? 0.0 : s_rhs[v][p];
    const double *T = s_arena + buf * C::TSZ + t * QC;
    if (nq_k == QC) {
#pragma unroll
      for (int qi = 0; qi < QC; qi++) acc = acc + T[qi];
    } else {
      for (int qi = 0; qi < nq_k; qi++) acc = acc + T[qi];
    }
    if (k == NCH - 1) {
      // creat_btp_fluxes_qdf projection (mod_rhs_btp.F90:339-362): left -, right +
#pragma unroll
      for (int kf = 0; kf < 2; kf++) {
        const int r = s_pf[p][kf];
        if (r < 0) continue;
        const int lf = r / NGL, n = r % NGL;
        const bool left = s_side[lf] == 0;
#pragma unroll
        for (int iq = 0; iq < NQ; iq++) {
          const double c = s_fq[lf][iq][0] * s_psiq[n * NQ + iq] * s_fq[lf][iq][1 + v];
          acc = left ? acc - c : acc + c;
        }
      }
    }
    s_rhs[v][p] = acc;
  };

  // face time averages: the old values are loaded at the start of D0 and written back
  // (plus the increments staged in s_fadd) after D0's tasks, hiding the round trip
  constexpr int NFA = FA_N * 4 * NQ, RF = (NFA + BS - 1) / BS;
  double fa_old[RF];
  if (a.accumulate) {
#pragma unroll
    for (int r = 0; r < RF; r++) {
      const int t = tid + r * BS;
      if (t < NFA) {
        const int kk = t / (4 * NQ), rr = t % (4 * NQ), lf = rr / NQ, iq = rr % NQ;
        if (s_side[lf] == 0) fa_old[r] = a.facc[kk * FQ + (size_t)s_face[lf] * NQ + iq];
      }
    }
  }
  for (int k = 0; k <= NCH; k++) {
    asm volatile("" ::: "memory");  // keep LDS reads inside their phase (no hoisting)
    const int WT = (k < NCH) ? ((k == NCH - 1) ? (Q - k * QC) : QC) * NGL : 0;  // term tasks
    const int WS = (k >= 1) ? 3 * P : 0;                                          // sums of chunk k-1
    const int WL = (k == 0) ? 4 * NGL + P : 0;                                    // LDG faces + qq
    const int WP = (k == NCH) ? 2 * P : 0;                                        // Laplacian sums
    for (int w = tid; w < WT + WS + WL + WP; w += BS) {
      asm volatile("" ::: "memory");
      if (w < WT) {
        term_task(k, w);
      } else if (w < WT + WS) {
        sum_task(k - 1, w - WT);
      } else if (w < WT + WS + WL) {
        const int t = w - WT - WS;
        if (t < 4 * NGL) {
          // ---- create_rhs_laplacian_flux at (face lf, node n) (mod_laplacian_quad.F90:452-517)
          const int lf = t / NGL, n = t % NGL;
          const int f = s_face[lf], side = s_side[lf], er = s_bc[lf];
          const int p = s_map[lf][n];
          const size_t fn = (size_t)f * NGL + n;
          const double *B = a.fncoef;
          const double nxn = m.fnstat[FN_NX * FN + fn], nyn = m.fnstat[FN_NY * FN + fn];
          const double wq = m.fnstat[FN_W * FN + fn];
          const double b4 = B[4 * FN + fn], b9 = B[9 * FN + fn];
          double bl[4], br[4], gf_old[8];
#pragma unroll
          for (int iv = 0; iv < 4; iv++) {
            bl[iv] = B[(size_t)iv * FN + fn];
            br[iv] = B[(size_t)(5 + iv) * FN + fn];
          }
          const bool own_acc = a.accumulate && side == 0;
          if (own_acc)
#pragma unroll
            for (int c = 0; c < 8; c++) gf_old[c] = a.gfacc[(size_t)c * FN + fn];
          double own[4] = {s_grad[0][p], s_grad[1][p], s_grad[2][p], s_grad[3][p]};
          double oth[4];
          if (er > 0) {
#pragma unroll
            for (int c = 0; c < 4; c++) oth[c] = s_tr[lf][4 + c][n];
          } else {
#pragma unroll
            for (int c = 0; c < 4; c++) oth[c] = own[c];
            if (er == -4) {  // mod_laplacian_quad.F90:85-98
              double un = own[0] * nxn + own[1] * nyn;
              oth[0] = own[0] - 2.0 * un * nxn;
              oth[1] = own[1] - 2.0 * un * nyn;
              un = own[2] * nxn + own[3] * nyn;
              oth[2] = own[2] - 2.0 * un * nxn;
              oth[3] = own[3] - 2.0 * un * nyn;
            }
          }
          double gl[4], gr[4];
#pragma unroll
          for (int c = 0; c < 4; c++) {
            gl[c] = side == 0 ? own[c] : oth[c];
            gr[c] = side == 0 ? oth[c] : own[c];
          }
          if (own_acc) {
#pragma unroll
            for (int c = 0; c < 4; c++) {
              a.gfacc[(size_t)c * FN + fn] = gf_old[c] + gl[c];
              a.gfacc[(size_t)(4 + c) * FN + fn] = gf_old[4 + c] + gr[c];
            }
          }
          double fl[4], fr[4];
#pragma unroll
          for (int iv = 0; iv < 4; iv++) {
            fl[iv] = b4 * gl[iv] + bl[iv];
            fr[iv] = b9 * gr[iv] + br[iv];
          }
          const double beta = 0.5, alpha = 1.0 - beta;
          const double qum0 = alpha * fl[0] + beta * fr[0], qum1 = alpha * fl[1] + beta * fr[1];
          const double qvm0 = alpha * fl[2] + beta * fr[2], qvm1 = alpha * fl[3] + beta * fr[3];
          const double flux_qu = (qum0 - fl[0] * nxn) + (qum1 - fl[1] * nyn);
          const double flux_qv = (qvm0 - fl[2] * nxn) + (qvm1 - fl[3] * nyn);
          // psi(n,n) == 1: node n receives wq*1*flux
          const double c0 = wq * 1.0 * flux_qu, c1 = wq * 1.0 * flux_qv;
          s_fl[lf][n][0] = side == 0 ? c0 : -c0;
          s_fl[lf][n][1] = side == 0 ? c1 : -c1;
        } else {
          // ---- LDG volume fluxes qq (btp_compute_laplacian, mod_laplacian_quad.F90:374-380)
          const int p = t - 4 * NGL;
          const size_t I = (size_t)e * P + p;
          const double *NC = a.ncoef;
          const double pv = NC[NC_PV * (size_t)npoin + I];
          s_qq[0][p] = pv * s_grad[0][p] + NC[NC_D1 * (size_t)npoin + I];
          s_qq[1][p] = pv * s_grad[1][p] + NC[NC_D2 * (size_t)npoin + I];
          s_qq[2][p] = pv * s_grad[2][p] + NC[NC_D3 * (size_t)npoin + I];
          s_qq[3][p] = pv * s_grad[3][p] + NC[NC_D4 * (size_t)npoin + I];
        }
      } else {
        // ---- lap(c,p): volume over source nodes s=(ii,jj) (mod_laplacian_quad.F90:382-386),
        //      nonzero terms only (jj==j or ii==i), then faces (:489-513)
        const int t = w - WT - WS - WL, c = t / P, p = t % P, i = p % NGL, j = p / NGL;
        double acc = 0.0;
#pragma unroll
        for (int r = 0; r < 2 * NGL - 1; r++) {
          int jj, ii;
          nz_term<NGL>(r, i, j, jj, ii);
          const int s = jj * NGL + ii;
          double dx, dy;
          if (jj == j && ii == i) {
            const double he = s_dpsi[i * NGL + ii], hn = s_dpsi[j * NGL + jj];
            dx = he * s_nm[0][s] + hn * s_nm[2][s];
            dy = he * s_nm[1][s] + hn * s_nm[3][s];
          } else if (jj == j) {
            const double he = s_dpsi[i * NGL + ii];  // HE_DF(i,j,ii,jj); HN_DF = 0
            dx = he * s_nm[0][s];
            dy = he * s_nm[1][s];
          } else {
            const double hn = s_dpsi[j * NGL + jj];  // HN_DF(i,j,ii,jj); HE_DF = 0
            dx = hn * s_nm[2][s];
            dy = hn * s_nm[3][s];
          }
          acc = acc - s_nm[4][s] * (dx * s_qq[2 * c][s] + dy * s_qq[2 * c + 1][s]);
        }
#pragma unroll
        for (int kf = 0; kf < 2; kf++) {
          const int r = s_pf[p][kf];
          if (r >= 0) acc = acc + s_fl[r / NGL][r % NGL][c];
        }
        s_lap[c][p] = acc;
      }
    }
    if (k == 0 && a.accumulate) {
#pragma unroll
      for (int r = 0; r < RF; r++) {
        const int t = tid + r * BS;
        if (t < NFA) {
          const int kk = t / (4 * NQ), rr = t % (4 * NQ), lf = rr / NQ, iq = rr % NQ;
          if (s_side[lf] == 0) a.facc[kk * FQ + (size_t)s_face[lf] * NQ + iq] = fa_old[r] + s_fadd[kk][rr];
        }
      }
    }
    __syncthreads();
    if (k < 4) STAGE_MARK(6 + k);
  }
  STAGE_MARK(3);

  // ------------------------------------------------------------- E1: update + wall fix
  for (int p = tid; p < P; p += BS) {
    const size_t I = (size_t)e * P + p;
    const double mi = s_nm[5][p];
    double rh0 = mi * s_rhs[0][p], rh1 = mi * s_rhs[1][p], rh2 = mi * s_rhs[2][p];
    rh1 = rh1 + m.visc * mi * s_lap[0][p];
    rh2 = rh2 + m.visc * mi * s_lap[1][p];
    if (a.rhs_only) {
      a.rhs_out[I * 3 + 0] = rh0;
      a.rhs_out[I * 3 + 1] = rh1;
      a.rhs_out[I * 3 + 2] = rh2;
      continue;
    }
    // Shu-Osher combination (mod_rk_mlswe.F90:99-106)
    const double rh[3] = {rh0, rh1, rh2};
    double qn[4];
#pragma unroll
    for (int v = 1; v < 4; v++) {
      double x = 0.0;
      if (a.a1 != 0.0) x = a.a1 * s_q0[p][v];
      x = x + a.a2 * s_qb[p][v];
      if (a.a3 != 0.0) x = x + a.a3 * s_q2[p][v];
      qn[v] = x + a.dtt * rh[v - 1];
    }
    qn[0] = qn[1] + s_nm[6][p];
    // btp_mom_boundary_df (mod_barotropic_terms.F90:180-215), faces in face-id order
#pragma unroll
    for (int kf = 0; kf < 2; kf++) {
      const int r = s_pf[p][kf];
      if (r < 0) continue;
      const int lf = r / NGL, n = r % NGL, er = s_bc[lf];
      if (er != -4 && er != -2) continue;
      {
        if (er == -4) {
          const size_t fn = (size_t)s_face[lf] * NGL + n;
          const double nx = m.fnstat[FN_NX * FN + fn], ny = m.fnstat[FN_NY * FN + fn];
          const double unl = qn[2] * nx + qn[3] * ny;
          qn[2] = qn[2] - unl * nx;
          qn[3] = qn[3] - unl * ny;
        } else {
          qn[2] = 0.0;
          qn[3] = 0.0;
        }
      }
    }
#pragma unroll
    for (int v = 0; v < 4; v++) s_qn[p][v] = qn[v];
  }
  if (a.rhs_only) return;
  __syncthreads();
  STAGE_MARK(4);

  // ------------------------------------------------------------- E2: outputs
  for (int t = tid; t < 4 * P; t += BS) a.qb_out[(size_t)e * 4 * P + t] = s_qn[t / 4][t % 4];
  if (a.write_trace) {
    // traces of the new state on each interior face, into the neighbour's slot:
    // qb(4) and grad(u_bar)(4) at the face nodes
    for (int t = tid; t < 4 * 8 * NGL; t += BS) {
      const int lf = t / (8 * NGL), c = (t / NGL) % 8, n = t % NGL;
      if (s_bc[lf] <= 0) continue;
      const int p = s_map[lf][n];
      double val;
      if (c < 4) {
        val = s_qn[p][c];
      } else {
        const int cg = c - 4, i = p % NGL, j = p / NGL;
        const double ex = s_nm[(cg & 1) ? 1 : 0][p], nx = s_nm[(cg & 1) ? 3 : 2][p];
        val = nodal_grad<NGL>(s_dpsi, i, j, ex, nx, s_qn, 2 + (cg >> 1));
      }
      a.trace_out[(((size_t)s_nbe[lf] * 4 + s_nblf[lf]) * 8 + c) * NGL + n] = val;
    }
  }
  if (a.prof) {
    __syncthreads();
    STAGE_MARK(5);
    if (tid == 0) {
      s_prof[11] = wall_clock64();
      for (int k = 0; k < 12; k++) a.prof[(size_t)e * 12 + k] = s_prof[k];
    }
  }
}

// Face traces of a state for the first stage of a sub-cycle / a lone RHS: qb(4) and
// grad(u_bar)(4) at the face nodes, written into the neighbours' trace slots.
template <int NGL, int NQ>
__global__ void __launch_bounds__(64) grad_trace_kernel(DevMesh m, const double *qb, double *trace) {
  constexpr int P = NGL * NGL;
  const int e = blockIdx.x, tid = threadIdx.x;
  __shared__ double s_dpsi[NGL * NGL], s_qb[P][4], s_nm[4][P];
  __shared__ int s_map[4][NGL], s_bc[4], s_nbe[4], s_nblf[4];
  for (int t = tid; t < NGL * NGL; t += 64) s_dpsi[t] = m.basis[2 * NGL * NQ + t];
  for (int t = tid; t < 4 * NGL; t += 64) s_map[t / NGL][t % NGL] = m.efmap[e * 4 * NGL + t];
  if (tid < 4) {
    s_bc[tid] = m.ebc[e * 4 + tid];
    s_nbe[tid] = m.enbr_e[e * 4 + tid];
    s_nblf[tid] = m.enbr_lf[e * 4 + tid];
  }
  for (int t = tid; t < 4 * P; t += 64) s_qb[t / 4][t % 4] = qb[(size_t)e * 4 * P + t];
  for (int t = tid; t < 4 * P; t += 64) {
    const int c = t / P, p = t % P;
    s_nm[c][p] = m.nstat[(NS_EX + c) * (size_t)m.npoin + (size_t)e * P + p];
  }
  __syncthreads();
  for (int t = tid; t < 4 * 8 * NGL; t += 64) {
    const int lf = t / (8 * NGL), c = (t / NGL) % 8, n = t % NGL;
    if (s_bc[lf] <= 0) continue;
    const int p = s_map[lf][n];
    double val;
    if (c < 4) {
      val = s_qb[p][c];
    } else {
      const int cg = c - 4, i = p % NGL, j = p / NGL;
      const double ex = s_nm[(cg & 1) ? 1 : 0][p], nx = s_nm[(cg & 1) ? 3 : 2][p];
      val = nodal_grad<NGL>(s_dpsi, i, j, ex, nx, s_qb, 2 + (cg >> 1));
    }
    trace[(((size_t)s_nbe[lf] * 4 + s_nblf[lf]) * 8 + c) * NGL + n] = val;
  }
}

// Normalisation of the time averages after the sub-cycle (mod_rk_mlswe.F90:124-149).
// tau_wind_ave = (sum over N_btp of tau_wind) / N_btp, summed the same way as the reference.
__global__ void btp_finalize_kernel(double *qacc, double *facc, double *nacc, double *gfacc, double *tau_wind_ave,
                                    const double *tau_wind, int npq, int nfq, int npoin, int nfn, int N_btp,
                                    double N_inv) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = tid; i < (size_t)QA_N * npq; i += stride) qacc[i] = N_inv * qacc[i];
  for (size_t i = tid; i < (size_t)FA_N * nfq; i += stride) facc[i] = N_inv * facc[i];
  for (size_t i = tid; i < (size_t)NA_N * npoin; i += stride) nacc[i] = N_inv * nacc[i];
  for (size_t i = tid; i < (size_t)8 * nfn; i += stride) gfacc[i] = N_inv * gfacc[i];
  for (size_t i = tid; i < (size_t)2 * npq; i += stride) {
    double s = 0.0, t = tau_wind[i];
    for (int k = 0; k < N_btp; k++) s = s + t;
    tau_wind_ave[i] = s / (double)N_btp;
  }
}

#define HNUMO_INSTANTIATE_BTP(NGL, NQ)                                 \
  template __global__ void btp_stage_kernel<NGL, NQ>(StageArgs);        \
  template __global__ void grad_trace_kernel<NGL, NQ>(DevMesh, const double *, double *);

}  // namespace hnumo
