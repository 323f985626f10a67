// kernels_bcl.hip -- baroclinic (layer) kernels of the MI355X MLSWE engine.
//
// Pattern: face kernels (one 64-thread workgroup per face) evaluate numerical fluxes
// at face quad points from face traces and project them onto the face nodes
// (per-face contribution buffers, no atomics); element kernels (one workgroup per
// element, all layers) evaluate volume terms by sum factorisation, gather the four
// faces' contributions in face-id order and apply the nodal updates.
//
// Reference routines restated here (arithmetic per term as in the reference):
//   btp_bcl_coeffs_qdf            mod_barotropic_terms.F90:219-409
//   extract_qprime_df_face         mod_layer_terms.F90:354-415 (+ extract_dprime :417-465)
//   layer_mass_rhs                 mod_create_rhs_mlswe.F90:53-78, :822-877, :922-1034
//   apply_consistency              mod_splitting.F90:324-366, mod_layer_terms.F90:57-137,
//                                  mod_create_rhs_mlswe.F90:879-920, :1036-1115
//   bcl_create_laplacian           mod_laplacian_quad.F90:227-248, :392-425, :521-611
//   create_rhs_dynamics_volume_layers  mod_create_rhs_mlswe.F90:281-456
//   Apply_layers_fluxes            mod_create_rhs_mlswe.F90:458-820
//   momentum / momentum_mass update, implicit Coriolis, layer_mom_boundary_df,
//   evaluate_bcl / evaluate_bcl_v1 / extract_velocity
//                                  mod_splitting.F90:94-287, mod_layer_terms.F90:198-320, :529-584
#include "engine_internal.h"

namespace hnumo {

// Diagnostics (HNUMO_BCL_PROF builds only): per-block phase clocks of the element kernels,
// [kernel][block][8]: marks 0..5 clock64 at the phase boundaries of thread 0, 6/7 wall clock
// at its start / end (read by hnumo_bcl_prof; tools/bcl_profile.py)
#ifndef HNUMO_BCL_PROF
#define HNUMO_BCL_PROF HNUMO_DIAG
#endif
#if HNUMO_BCL_PROF
__device__ unsigned long long g_bcl_prof[4][8192][8];
#define BCL_MARK(kid, k) \
  if (threadIdx.x == 0 && blockIdx.x < 8192) g_bcl_prof[kid][blockIdx.x][k] = clock64();
#define BCL_WALL(kid, k) \
  if (threadIdx.x == 0 && blockIdx.x < 8192) g_bcl_prof[kid][blockIdx.x][k] = wall_clock64();
#else
#define BCL_MARK(kid, k)
#define BCL_WALL(kid, k)
#endif

#define QF(v, s, n, f, k) qf[((((size_t)(k) * F + (f)) * NGL + (n)) * 2 + (s)) * 3 + (v)]


__device__ __forceinline__ double dmin(double a, double b) { return a < b ? a : (b < a ? b : a); }
__device__ __forceinline__ double dmax(double a, double b) { return a > b ? a : (b > a ? b : a); }

template <int NGL, int NQ>
__device__ __forceinline__ void load_basis(const DevMesh &m, double *s_psiq, double *s_dpsiq, double *s_dpsi,
                                           double *s_psi, int tid, int bs) {
  for (int t = tid; t < NGL * NQ; t += bs) {
    s_psiq[t] = m.basis[t];
    s_dpsiq[t] = m.basis[NGL * NQ + t];
  }
  for (int t = tid; t < NGL * NGL; t += bs) {
    s_dpsi[t] = m.basis[2 * NGL * NQ + t];
    s_psi[t] = m.basis[2 * NGL * NQ + NGL * NGL + t];
  }
}

// Gathered staging (the element kernels' load phases): every gather's loads are issued before any
// of them is stored to LDS, so a kernel's inputs arrive in one memory round trip (a strided
// load-then-store loop waits for its own loads before the next loop's go out: mom_elem's sixteen
// such loops were sixteen round trips, ~14.5k clocks of its ~70k at dg25).  N: the most entries
// (MAXL layers), n >= 1: this call's; ld(t) returns entry t, st(t, v) stores it.  Within a wave the
// loads are unconditional (a lane past n loads entry n-1 again, unused): loads under a lane
// branch leave their registers to be merged at the join, which waits for them there.
template <class T, int N, int BS>
struct Gather {
  static constexpr int NI = (N + BS - 1) / BS;
  T v[NI];
  template <class LoadF>
  __device__ __forceinline__ void load(int tid, int n, LoadF &&ld) {
    const int w0 = __builtin_amdgcn_readfirstlane(tid & ~63);  // (the wave's first thread)
#pragma unroll
    for (int j = 0; j < NI; j++) {
      const int t = tid + j * BS;
      if (w0 + j * BS < n) v[j] = ld(t < n ? t : n - 1);  // (a wave past n issues nothing)
    }
  }
  template <class StoreF>
  __device__ __forceinline__ void store(int tid, int n, StoreF &&st) const {
#pragma unroll
    for (int j = 0; j < NI; j++) {
      const int t = tid + j * BS;
      if (t < n) st(t, v[j]);
    }
  }
  // st(t, j): entry t is v[j] (for stores that combine two gathers of the same layout)
  template <class StoreF>
  __device__ __forceinline__ void store_j(int tid, int n, StoreF &&st) const {
#pragma unroll
    for (int j = 0; j < NI; j++) {
      const int t = tid + j * BS;
      if (t < n) st(t, j);
    }
  }
};
// the basis tables (psiq, dpsiq, dpsi, psi: contiguous in m.basis) as one gather
template <int NGL, int NQ, int BS>
struct BasisGather {
  static constexpr int NB = 2 * NGL * NQ + 2 * NGL * NGL;
  Gather<double, NB, BS> g;
  __device__ __forceinline__ void load(const DevMesh &m, int tid) {
    g.load(tid, NB, [&](int t) { return m.basis[t]; });
  }
  __device__ __forceinline__ void store(double *s_psiq, double *s_dpsiq, double *s_dpsi, double *s_psi, int tid) const {
    g.store(tid, NB, [&](int t, double v) {
      constexpr int A = NGL * NQ, P = NGL * NGL;
      if (t < A)
        s_psiq[t] = v;
      else if (t < 2 * A)
        s_dpsiq[t - A] = v;
      else if (t < 2 * A + P)
        s_dpsi[t - 2 * A] = v;
      else
        s_psi[t - 2 * A - P] = v;
    });
  }
};

// Reference-order term definitions (Tensor_product.F90:71-114); see kernels_btp.hip.
#define PSIH(n, m, iq, jq) (s_psiq[(n)*NQ + (iq)] * s_psiq[(m)*NQ + (jq)])
#define HE(n, m, iq, jq) (s_dpsiq[(n)*NQ + (iq)] * s_psiq[(m)*NQ + (jq)])
#define HN(n, m, iq, jq) (s_psiq[(n)*NQ + (iq)] * s_dpsiq[(m)*NQ + (jq)])
#define HE_DF(n, m, i, j) (s_dpsi[(n)*NGL + (i)] * s_psi[(m)*NGL + (j)])
#define HN_DF(n, m, i, j) (s_psi[(n)*NGL + (i)] * s_dpsi[(m)*NGL + (j)])

// Workgroup barrier for LDS hand-offs only (no release fence: outstanding global stores of the
// wave are not drained, unlike __syncthreads())
// mom_elem phase 2: the interface-height gradient sums on their own threads first (see GZS there)
#ifndef HNUMO_MOM_GZS
#define HNUMO_MOM_GZS 1
#endif
// the element of this block (DevMesh::eperm)
__device__ __forceinline__ int blk_elem(const DevMesh &m) {
  return m.eperm ? __builtin_amdgcn_readfirstlane(m.eperm[blockIdx.x]) : (int)blockIdx.x;
}
#define BCL_LDS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// Term buffers of ordered_node_sums: chunks of RC quad rows (RC | NQ) for NT chains, two buffers
// when they fit the budget (doubles), else one
template <int NQ, int NT, int BUDGET>
struct QSumCfg {
  static constexpr int rc_pick(int nbuf) {
    for (int rc = NQ; rc >= 1; rc--)
      if (NQ % rc == 0 && nbuf * NT * ((rc * NQ) | 1) <= BUDGET) return rc;
    return 0;
  }
  static constexpr int NBUF = rc_pick(2) ? 2 : 1;
  static constexpr int RC = rc_pick(NBUF) ? rc_pick(NBUF) : 1;
  static constexpr int QC = RC * NQ, QCP = QC | 1, NCH = NQ / RC;
  static constexpr int SIZE = NBUF * NT * QCP;
};

// Reference-order quad-point sums of the chains (p, c) -- p < NP nodes, c < nc <= CPN sums per
// node -- chain p*CPN + c summed by thread p*CPN + c:
//   acc = sum over q = 0..Q-1, in order, of T(p, c, q).
// The terms of a chunk of RC quad rows are evaluated in parallel into LDS: task (p, quad point q of
// the chunk) writes all nc terms of node p at q, eval(p, q, dst, stride) -> dst[c*stride] = T(p, c, q),
// so the node's basis products and metric derivatives are formed once for its nc terms; the
// summing threads add the chunk in quad order (with two buffers, while the next chunk's terms are
// evaluated).  The same terms in the same order as one thread forming and adding each itself, so
// the same bits, but the dependent chain is one add per quad point instead of the whole term (the
// element kernels ran ~40k clocks per such sum with one wave per SIMD).  Every thread must call it.
template <int NQ, int NP, int CPN, int BS, class CFG, class EvalF>
__device__ __forceinline__ double ordered_node_sums(double *tb, int tid, int nc, EvalF &&eval) {
  constexpr int NT = NP * CPN, QC = CFG::QC, QCP = CFG::QCP, NCH = CFG::NCH, NBUF = CFG::NBUF, RC = CFG::RC;
  static_assert(NT <= BS, "one sum per thread");
  double acc = 0.0;
  const bool summer = tid < NT && tid % CPN < nc;
  auto ev = [&](int k) {
    double *T = tb + (NBUF == 2 ? (k & 1) * NT * QCP : 0);
    for (int t = tid; t < NP * QC; t += BS) {
      const int p = t / QC, qi = t - p * QC;
      eval(p, k * QC + qi, T + p * CPN * QCP + qi, QCP);
    }
  };
  auto add = [&](int k) {
    if (summer) {
      const double *T = tb + (NBUF == 2 ? (k & 1) * NT * QCP : 0) + tid * QCP;
#pragma unroll
      for (int r = 0; r < RC; r++) {
        double tv[NQ];
#pragma unroll
        for (int i = 0; i < NQ; i++) tv[i] = T[r * NQ + i];
        asm volatile("" ::: "memory");  // the row's loads before its adds
#pragma unroll
        for (int i = 0; i < NQ; i++) acc = acc + tv[i];
      }
    }
  };
  if constexpr (NBUF == 2) {
#pragma unroll 1
    for (int k = 0; k <= NCH; k++) {
      if (k < NCH) ev(k);
      if (k >= 1) add(k - 1);
      BCL_LDS_BARRIER();
    }
  } else {
#pragma unroll 1
    for (int k = 0; k < NCH; k++) {
      ev(k);
      BCL_LDS_BARRIER();
      add(k);
      BCL_LDS_BARRIER();
    }
  }
  return acc;
}

// The weak-form divergence terms w(q)*(dpsidx(p,q)*fx_k(q) + dpsidy(p,q)*fy_k(q)) of the layers
// k < L at node p, quad point q (mod_create_rhs_mlswe.F90:866-868 / :911-913), f[k][0..1][Q]
template <int NGL, int NQ>
__device__ __forceinline__ void weak_div_terms(const double *s_psiq, const double *s_dpsiq, const double (*qm)[NQ * NQ],
                                               const double (*f)[2][NQ * NQ], int L, int p, int q, double *dst,
                                               int stride) {
  const int i = p % NGL, j = p / NGL, iq = q % NQ, jq = q / NQ;
  const double h_e = s_dpsiq[i * NQ + iq] * s_psiq[j * NQ + jq], h_n = s_psiq[i * NQ + iq] * s_dpsiq[j * NQ + jq];
  const double dhdx = h_e * qm[0][q] + h_n * qm[2][q];
  const double dhdy = h_e * qm[1][q] + h_n * qm[3][q];
  const double w = qm[4][q];
#pragma unroll
  for (int k = 0; k < MAXL; k++) {
    if (k >= L) break;
    dst[k * stride] = w * (dhdx * f[k][0][q] + dhdy * f[k][1][q]);
  }
}

template <int NGL, int NQ>
struct Blk {
  static constexpr int P = NGL * NGL, Q = NQ * NQ, BS = ((Q + 63) / 64) * 64;
  // mass_elem / cons_elem: 256 threads at least (the quad-point sums, ordered_node_sums)
  static constexpr int BSW = BS < 256 ? 256 : BS;
  using QS = QSumCfg<NQ, P * MAXL, 34 * 1024 / 8>;
  // BIG (meshes of many rounds, HNUMO_BCL_BIG): one quad row per term chunk, double-buffered --
  // more barriers per element, but a third of the LDS, so more workgroups per CU
  template <bool BIG>
  using QSB = typename std::conditional<BIG, QSumCfg<NQ, P * MAXL, 2 * P * MAXL * (NQ | 1)>, QS>::type;
};

// sum over the element's nodes of PSIH(n,mm,iq,jq)*x(v, mm*NGL+n), mm outer, n inner (the
// reference's interpolation order), for NV components x[v*stride + node]; pa/pb = the thread's
// psiq(:,iq), psiq(:,jq)
template <int NGL, int NV>
__device__ __forceinline__ void interp_q(const double *pa, const double *pb, const double *x, int stride,
                                         double out[NV]) {
#pragma unroll
  for (int v = 0; v < NV; v++) out[v] = 0.0;
#pragma unroll 1
  for (int mm = 0; mm < NGL; mm++)
#pragma unroll
    for (int n = 0; n < NGL; n++) {
      const double hi = pa[n] * pb[mm];
#pragma unroll
      for (int v = 0; v < NV; v++) out[v] = out[v] + hi * x[v * stride + mm * NGL + n];
    }
}

// Face terms onto node p: acc -/+ (wq*hi)*flux(iq) in quad order (left: -, right: +), faces in
// the order of the element's local faces, from the element's own face data staged in LDS:
// s_fw[lf][NQ] (w of the face quad points) and s_fx[lf][NQ] (the flux).  node_faces finds the
// (at most two) face points lf*NGL + n at node p, ascending (-1: none), once per thread (a search
// loop per sum diverged into one masked pass per face point of the element) ...
template <int NGL>
__device__ __forceinline__ void node_faces(const int *s_map, int p, int &r0, int &r1) {
  int m_[4 * NGL];
#pragma unroll
  for (int x = 0; x < 4 * NGL; x++) m_[x] = s_map[x];
  r0 = r1 = -1;
#pragma unroll
  for (int x = 4 * NGL - 1; x >= 0; x--)
    if (m_[x] == p) {
      r1 = r0;
      r0 = x;
    }
}
// ... and face_terms_at adds their terms, each face's loads before its chain
template <int NGL, int NQ>
__device__ __forceinline__ double face_terms_at(const double *s_psiq, const int *s_side, const double *s_fw,
                                                const double *s_fx, int r0, int r1, double acc) {
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int r = h ? r1 : r0;
    if (r < 0) continue;
    const int lf = r / NGL, n = r - lf * NGL;
    const bool left = s_side[lf] == 0;
    double c[NQ];
#pragma unroll
    for (int iq = 0; iq < NQ; iq++) c[iq] = s_fw[lf * NQ + iq] * s_psiq[n * NQ + iq] * s_fx[lf * NQ + iq];
#pragma unroll
    for (int iq = 0; iq < NQ; iq++) acc = left ? acc - c[iq] : acc + c[iq];
  }
  return acc;
}

// Stage an element's face data into LDS with the element's other loads (the element kernels
// otherwise read it from global memory inside their ordered sums, one round trip per face):
// dst[c][lf][NQ] = src[c*cstride + face(lf)*NQ + iq] for c < nc (before the first barrier,
// after s_face is set -- it is read from global memory here).
template <int NQ>
__device__ __forceinline__ void stage_face_quads(double *dst, const double *src, size_t cstride, int nc,
                                                 const int *efaces_e, int tid, int bs) {
  for (int t = tid; t < nc * 4 * NQ; t += bs) {
    const int c = t / (4 * NQ), lf = (t / NQ) % 4, iq = t % NQ;
    dst[t] = src[c * cstride + (size_t)efaces_e[lf] * NQ + iq];
  }
}

// A face's qf block (v, side, n) of every layer into s_qf[k][6*NGL] (contiguous per layer)
template <int NGL>
__device__ __forceinline__ void stage_qf(double (*s_qf)[6 * NGL], const double *qf, int f, int F, int L, int tid,
                                         int bs) {
  for (int t = tid; t < L * 6 * NGL; t += bs) {
    const int k = t / (6 * NGL), r = t % (6 * NGL);
    s_qf[k][r] = qf[((size_t)k * F + f) * NGL * 6 + r];
  }
}
#define SQF(v, s, n, k) s_qf[k][((n)*2 + (s)) * 3 + (v)]

// ===================================================================== face traces
// extract_qprime_df_face: qf(3,2,ngl,nface,L) from nodal qprime(3,npoin,L), with wall ghosts.
// only_dp: extract_dprime_df_face into component 1 (no reflection).
template <int NGL>
__global__ void extract_face_kernel(DevMesh m, const double *qp, double *qf, int only_dp) {
  const int F = m.nface, L = m.L, npoin = m.npoin;
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (size_t)F * NGL) return;
  const int f = gid / NGL, n = gid % NGL;
  const int IL = m.fnodeL[gid], IR = m.fnodeR[gid], er = m.fer[f];
  for (int k = 0; k < L; k++) {
    const double *q = qp + (size_t)k * 3 * npoin;
    if (only_dp) {
      double l = q[(size_t)IL * 3];
      QF(0, 0, n, f, k) = l;
      QF(0, 1, n, f, k) = er > 0 ? q[(size_t)IR * 3] : l;
      continue;
    }
    double l0 = q[(size_t)IL * 3], l1 = q[(size_t)IL * 3 + 1], l2 = q[(size_t)IL * 3 + 2];
    QF(0, 0, n, f, k) = l0;
    QF(1, 0, n, f, k) = l1;
    QF(2, 0, n, f, k) = l2;
    if (er > 0) {
      QF(0, 1, n, f, k) = q[(size_t)IR * 3];
      QF(1, 1, n, f, k) = q[(size_t)IR * 3 + 1];
      QF(2, 1, n, f, k) = q[(size_t)IR * 3 + 2];
    } else {
      double r1 = l1, r2 = l2;
      if (er == -4) {
        double nx = m.fnstat[FN_NX * (size_t)F * NGL + gid], ny = m.fnstat[FN_NY * (size_t)F * NGL + gid];
        double un = l1 * nx + l2 * ny;
        r1 = l1 - 2.0 * un * nx;
        r2 = l2 - 2.0 * un * ny;
      } else if (er == -2) {
        r1 = -l1;
        r2 = -l2;
      }
      QF(0, 1, n, f, k) = l0;
      QF(1, 1, n, f, k) = r1;
      QF(2, 1, n, f, k) = r2;
    }
  }
}

// extract_qprime_df_face fused into the kernel that writes the nodal qprime (single rank, every
// face's elements in the launch): the thread of node p writes, for each face point r = lf*NGL + n
// at p (node_faces), its element's side of face lf and, on a physical boundary (er < 0), the
// ghost side -- the values extract_face_kernel would read back from qprime, the same arithmetic.
// v[k][c] = qprime(c, p, k) of the node; only_dp: component 0 alone (extract_dprime_df_face).
template <int NGL>
__device__ __forceinline__ void extract_node_faces(const DevMesh &m, double *qf, const int *s_face, const int *s_side,
                                                   const int *s_bc, int r0, int r1, const double (*v)[3], int only_dp) {
  const int F = m.nface, L = m.L;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int r = h ? r1 : r0;
    if (r < 0) continue;
    const int lf = r / NGL, n = r - lf * NGL, f = s_face[lf], s = s_side[lf], er = s_bc[lf];
    const size_t gid = (size_t)f * NGL + n;
    double nx = 0.0, ny = 0.0;
    if (!only_dp && er == -4) {
      nx = m.fnstat[FN_NX * (size_t)F * NGL + gid];
      ny = m.fnstat[FN_NY * (size_t)F * NGL + gid];
    }
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      const double l0 = v[k][0];
      QF(0, s, n, f, k) = l0;
      if (er <= 0) QF(0, 1, n, f, k) = l0;
      if (only_dp) continue;
      const double l1 = v[k][1], l2 = v[k][2];
      QF(1, s, n, f, k) = l1;
      QF(2, s, n, f, k) = l2;
      if (er <= 0) {
        double r1_ = l1, r2_ = l2;
        if (er == -4) {
          double un = l1 * nx + l2 * ny;
          r1_ = l1 - 2.0 * un * nx;
          r2_ = l2 - 2.0 * un * ny;
        } else if (er == -2) {
          r1_ = -l1;
          r2_ = -l2;
        }
        QF(1, 1, n, f, k) = r1_;
        QF(2, 1, n, f, k) = r2_;
      }
    }
  }
}

// btp_bcl_coeffs_qdf at face quad point iq (mod_barotropic_terms.F90:306-337) from the face's qf
// block s_qf [MAXL][6*NGL]: Q_*_dp_edge and H_bcl_edge, the average of the two sides -- one
// restatement for bcl_coeffs_face_kernel and bcl_coeffs_elem_kernel's fused faces
template <int NGL, int NQ>
__device__ __forceinline__ void bcl_face_quad(const DevMesh &m, const double (*s_qf)[6 * NGL], const double *s_psiq,
                                              int iq, double &quu, double &quv, double &qvv, double &hb) {
  const int L = m.L;
  double pl = 0, pr = 0;
  quu = 0;
  quv = 0;
  qvv = 0;
  hb = 0;
#pragma unroll
  for (int k = 0; k < MAXL; k++) {
    if (k >= L) break;
    double ql[3] = {0, 0, 0}, qr[3] = {0, 0, 0};
#pragma unroll
    for (int n = 0; n < NGL; n++) {
      double hi = s_psiq[n * NQ + iq];
      for (int v = 0; v < 3; v++) {
        ql[v] = ql[v] + hi * SQF(v, 0, n, k);
        qr[v] = qr[v] + hi * SQF(v, 1, n, k);
      }
    }
    quu = quu + 0.5 * ((ql[1] * ql[1] * ql[0]) + (qr[1] * qr[1] * qr[0]));
    quv = quv + 0.5 * ((ql[2] * ql[1] * ql[0]) + (qr[2] * qr[1] * qr[0]));
    qvv = qvv + 0.5 * ((ql[2] * ql[2] * ql[0]) + (qr[2] * qr[2] * qr[0]));
    double pl1 = pl + ql[0];
    double left_dp = 0.5 * m.alpha[k] * (pl1 * pl1 - pl * pl);
    double pr1 = pr + qr[0];
    double right_dp = 0.5 * m.alpha[k] * (pr1 * pr1 - pr * pr);
    hb = hb + 0.5 * (left_dp + right_dp);
    pl = pl1;
    pr = pr1;
  }
}

// the ghost side of graduv_dpp_face on a physical boundary (mod_barotropic_terms.F90:360-390):
// a copy, the two gradient pairs reflected at a free-slip wall (er == -4)
__device__ __forceinline__ void bcl_face_ghost(const double l[5], double r[5], int er, double nx, double ny) {
  for (int c = 0; c < 5; c++) r[c] = l[c];
  if (er == -4) {
    double un = l[0] * nx + l[1] * ny;
    r[0] = l[0] - 2.0 * un * nx;
    r[1] = l[1] - 2.0 * un * ny;
    un = l[2] * nx + l[3] * ny;
    r[2] = l[2] - 2.0 * un * nx;
    r[3] = l[3] - 2.0 * un * ny;
  }
}

// ======================================================= btp_bcl_coeffs_qdf: element
// Q_uu_dp, Q_uv_dp, Q_vv_dp, H_bcl at quad points (mod_barotropic_terms.F90:265-283);
// dpp_graduv, btp_dpp_graduv, pbprime_visc at nodes (:287-304).  dpprime_visc =
// qprime(1,:,:) is stored for the layer LDG (ti_rk_bcl.F90:47,66).
template <int NGL, int NQ>
__global__ void __launch_bounds__((Blk<NGL, NQ>::BSW))
    bcl_coeffs_elem_kernel(DevMesh m, double *qp, const double *qp_avg, double *qcoef, double *ncoef,
                           double *dpp_graduv, double *dpprime_visc, double *ecoef, const double *qf,
                           const double *qf_avg, double *qf_out, double *fcoef, double *fncoef, double *gdpp_face,
                           double *efcoef) {
  // qp_avg (the corrector): qprime_df2 = 0.5*(qprime_df2 + qprime_df) of the element's nodes first
  // (ti_rk_bcl.F90:64), written back
  // qf != NULL (single rank): the face part of btp_bcl_coeffs_qdf is formed here too, in place of
  // bcl_coeffs_face_kernel -- the element's four faces' quad-point coefficients into its own efcoef
  // slots (both elements of a face compute them, the same bits; the left one writes fcoef), and its
  // side's face-node dpp_graduv / dpprime_visc traces with their layer sums into gdpp_face, fncoef
  // and both elements' efcoef slots (a physical boundary: both sides, the ghost side reflected).
  // qf_avg (the corrector): the averaged qprime_face2 = 0.5*(qprime_face + qprime_face2) goes to
  // qf_out (not in place: the neighbour reads the face block too), each element writing its side
  constexpr int P = Blk<NGL, NQ>::P, Q = Blk<NGL, NQ>::Q, BS = Blk<NGL, NQ>::BSW;
  static_assert(BS >= 192 && 4 * NQ <= 64 && 4 * NGL <= 64, "face tasks on waves 1 and 2");
  const int e = blk_elem(m), tid = threadIdx.x, L = m.L, npoin = m.npoin, npq = m.npoin_q, F = m.nface;
  __shared__ double s_psiq[NGL * NQ], s_dpsiq[NGL * NQ], s_dpsi[NGL * NGL], s_psi[NGL * NGL];
  __shared__ double s_q[MAXL][3][P];
  __shared__ double s_nm[4][P];
  __shared__ double s_g[MAXL][4][P];
  __shared__ double s_qfF[4][MAXL][6 * NGL];  // (qf) the four faces' qf blocks (averaged)
  __shared__ int s_map[4 * NGL], s_face[4], s_side[4], s_bc[4];
  // every load of the phase first (Gather), then the LDS stores (and the averaged copies): the
  // element's face ids, sides and boundary codes (scalar loads) and the element-major inputs, then
  // the face-indexed qf blocks
  int fr[12];  // face ids, sides, boundary codes of the four faces
#pragma unroll
  for (int x = 0; x < 4; x++) {
    fr[x] = m.efaces[e * 4 + x];
    fr[4 + x] = m.eside[e * 4 + x];
    fr[8 + x] = m.ebc[e * 4 + x];
  }
  auto sel4 = [&](const int *a, int lf) { return lf == 0 ? a[0] : (lf == 1 ? a[1] : (lf == 2 ? a[2] : a[3])); };
  BasisGather<NGL, NQ, BS> g_bas;
  g_bas.load(m, tid);
  Gather<int, 4 * NGL, BS> g_map;
  if (qf) g_map.load(tid, 4 * NGL, [&](int t) { return m.efmap[e * 4 * NGL + t]; });
  auto qidx = [&](int t) { return (size_t)(t / (3 * P)) * 3 * npoin + (size_t)e * 3 * P + t % (3 * P); };
  Gather<double, MAXL * 3 * P, BS> g_q, g_qa;
  g_q.load(tid, L * 3 * P, [&](int t) { return qp[qidx(t)]; });
  if (qp_avg) g_qa.load(tid, L * 3 * P, [&](int t) { return qp_avg[qidx(t)]; });
  Gather<double, 4 * P, BS> g_nm;
  g_nm.load(tid, 4 * P, [&](int t) { return m.nstat[(NS_EX + t / P) * (size_t)npoin + (size_t)e * P + t % P]; });
  auto fidx = [&](int t, int &lf, int &rr) {
    lf = t / (L * 6 * NGL);
    const int r = t % (L * 6 * NGL), k = r / (6 * NGL);
    rr = r % (6 * NGL);
    return ((size_t)k * F + sel4(fr, lf)) * NGL * 6 + rr;
  };
  Gather<double, 4 * MAXL * 6 * NGL, BS> g_qf, g_qfa;
  if (qf) {
    int lf, rr;
    g_qf.load(tid, 4 * L * 6 * NGL, [&](int t) { return qf[fidx(t, lf, rr)]; });
    if (qf_avg) g_qfa.load(tid, 4 * L * 6 * NGL, [&](int t) { return qf_avg[fidx(t, lf, rr)]; });
  }
  // the stores
  g_bas.store(s_psiq, s_dpsiq, s_dpsi, s_psi, tid);
  if (qf) {
    if (tid < 4) {
      s_face[tid] = sel4(fr, tid);
      s_side[tid] = sel4(fr + 4, tid);
      s_bc[tid] = sel4(fr + 8, tid);
    }
    g_map.store(tid, 4 * NGL, [&](int t, int v) { s_map[t] = v; });
    g_qf.store_j(tid, 4 * L * 6 * NGL, [&](int t, int j) {
      int lf, rr;
      const size_t i = fidx(t, lf, rr);
      double v = g_qf.v[j];
      if (qf_avg) {
        v = 0.5 * (g_qfa.v[j] + v);
        if ((rr / 3) % 2 == sel4(fr + 4, lf) || sel4(fr + 8, lf) <= 0) qf_out[i] = v;
      }
      s_qfF[lf][(t % (L * 6 * NGL)) / (6 * NGL)][rr] = v;
    });
  }
  g_q.store_j(tid, L * 3 * P, [&](int t, int j) {
    const int k = t / (3 * P), r = t % (3 * P);
    double v = g_q.v[j];
    if (qp_avg) {
      v = 0.5 * (v + g_qa.v[j]);
      qp[qidx(t)] = v;
    }
    s_q[k][r % 3][r / 3] = v;
  });
  g_nm.store(tid, 4 * P, [&](int t, double v) { s_nm[t / P][t % P] = v; });
  __syncthreads();
  // GSPLIT: quad-point tasks on threads [0, Q), the nodal gradient tasks on the threads past them
  constexpr bool GSPLIT = BS - Q >= 128;
  constexpr int EFC = 4 * NQ + 10 * NGL;
  const size_t FQ = (size_t)F * NQ, FN = (size_t)F * NGL;
  // (qf) the faces' quad-point coefficients (bcl_coeffs_face_kernel's arithmetic), task t < 4*NQ
  auto face_quad = [&](int t) {
    const int lf = t / NQ, iq = t % NQ;
    double quu, quv, qvv, hb;
    bcl_face_quad<NGL, NQ>(m, s_qfF[lf], s_psiq, iq, quu, quv, qvv, hb);
    const double vals[4] = {quu, quv, qvv, hb};
    for (int c = 0; c < 4; c++) efcoef[(size_t)(e * 4 + lf) * EFC + c * NQ + iq] = vals[c];
    if (s_side[lf] == 0) {
      const size_t fq = (size_t)s_face[lf] * NQ + iq;
      for (int c = 0; c < 4; c++) fcoef[(FC_QUU + c) * FQ + fq] = vals[c];
    }
  };
  for (int q = tid; q < Q; q += BS) {
    const int iq = q % NQ, jq = q / NQ;
    double quu = 0.0, quv = 0.0, qvv = 0.0, hb = 0.0, pk = 0.0;
    double pa[NGL], pb[NGL];
#pragma unroll
    for (int n = 0; n < NGL; n++) {
      pa[n] = s_psiq[n * NQ + iq];
      pb[n] = s_psiq[n * NQ + jq];
    }
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      double qq[3];
      interp_q<NGL, 3>(pa, pb, &s_q[k][0][0], P, qq);
      quu = quu + qq[1] * (qq[1] * qq[0]);
      quv = quv + qq[2] * (qq[1] * qq[0]);
      qvv = qvv + qq[2] * (qq[2] * qq[0]);
      double pk1 = pk + qq[0];
      hb = hb + 0.5 * m.alpha[k] * (pk1 * pk1 - pk * pk);
      pk = pk1;
    }
    const size_t Iq = (size_t)e * Q + q;
    qcoef[QC_QUU * (size_t)npq + Iq] = quu;
    qcoef[QC_QUV * (size_t)npq + Iq] = quv;
    qcoef[QC_QVV * (size_t)npq + Iq] = qvv;
    qcoef[QC_HBCL * (size_t)npq + Iq] = hb;
    double *ec = ecoef + (size_t)e * eco_stride(Q, P);  // element-major copy for the stage kernel
    ec[QC_QUU * Q + q] = quu;
    ec[QC_QUV * Q + q] = quv;
    ec[QC_QVV * Q + q] = qvv;
    ec[QC_HBCL * Q + q] = hb;
  }
  // compute_gradient_uv of (u'_k, v'_k), reference order, one thread per (layer, comp, node)
  for (int t = GSPLIT ? tid - Q : tid; t >= 0 && t < L * 4 * P; t += GSPLIT ? BS - Q : BS) {
    const int k = t / (4 * P), c = (t / P) % 4, p = t % P, i = p % NGL, j = p / NGL;
    const double *u = s_q[k][1 + (c >> 1)];
    const double ex = s_nm[(c & 1) ? 1 : 0][p], nx = s_nm[(c & 1) ? 3 : 2][p];
    // the 2*NGL-1 nonzero terms (row mm == j, column n == i) of the reference's 25-term sum, in
    // its order: with psi the identity at the LGL nodes (checked at engine creation) HE_DF =
    // dpsi(n,i) on the row and HN_DF = dpsi(mm,j) on the column, zero elsewhere, and a dropped
    // zero term leaves the sum unchanged (as in the stage kernel's nodal_grad)
    double cA[2 * NGL - 1], cB[2 * NGL - 1], cU[2 * NGL - 1];
#pragma unroll
    for (int r = 0; r < 2 * NGL - 1; r++) {
      const int d = r - j;
      const bool row = (unsigned)d < (unsigned)NGL;
      const int mm = min(r, j) + max(d - NGL + 1, 0), n = row ? d : i;
      cA[r] = row ? s_dpsi[n * NGL + i] : 0.0;
      cB[r] = (row & (d != i)) ? 0.0 : s_dpsi[mm * NGL + j];
      cU[r] = u[mm * NGL + n];
    }
    double gsum = 0.0;
#pragma unroll
    for (int r = 0; r < 2 * NGL - 1; r++) gsum = gsum + (cA[r] * ex + cB[r] * nx) * cU[r];
    s_g[k][c][p] = gsum;
  }
  __syncthreads();
  for (int p = tid; p < P; p += BS) {
    const size_t I = (size_t)e * P + p;
    double sum[4] = {0, 0, 0, 0}, pv = 0.0;
    for (int k = 0; k < L; k++) {
      double d = s_q[k][0][p];
      dpprime_visc[(size_t)k * npoin + I] = d;
      for (int c = 0; c < 4; c++) {
        double dg = d * s_g[k][c][p];
        dpp_graduv[((size_t)k * 4 + c) * npoin + I] = dg;
        sum[c] = sum[c] + dg;
      }
      pv = pv + d;
    }
    ncoef[NC_PV * (size_t)npoin + I] = pv;
    for (int c = 0; c < 4; c++) ncoef[(NC_D1 + c) * (size_t)npoin + I] = sum[c];
    double *ec = ecoef + (size_t)e * eco_stride(Q, P) + 4 * Q;
    ec[NC_PV * P + p] = pv;
    for (int c = 0; c < 4; c++) ec[(NC_D1 + c) * P + p] = sum[c];
  }
  if (!qf) return;
  // (the face quad tasks here, not beside the quad-point tasks: there they took lanes from the
  // gradient tasks, 2 -> 3 rounds, 14.8 -> 16.2 us per launch at dg25L3)
  if (tid >= 64 && tid < 64 + 4 * NQ) {  // face quad points
    face_quad(tid - 64);
  } else if (tid >= 128 && tid < 128 + 4 * NGL) {  // face nodes: this element's side
    const int lf = (tid - 128) / NGL, n = (tid - 128) % NGL, p = s_map[lf * NGL + n];
    const int s = s_side[lf], er = s_bc[lf];
    const size_t fn = (size_t)s_face[lf] * NGL + n;
    double *eo = efcoef + (size_t)(e * 4 + lf) * EFC + 4 * NQ;
    if (er > 0) {
      double hs[5] = {0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        const double d = s_q[k][0][p];
        double h[5];
        for (int c = 0; c < 4; c++) h[c] = d * s_g[k][c][p];
        h[4] = d;
        for (int c = 0; c < 5; c++) {
          gdpp_face[((size_t)k * 10 + 5 * s + c) * FN + fn] = h[c];
          hs[c] = hs[c] + h[c];
        }
      }
      double *en = efcoef + (size_t)(m.enbr_e[e * 4 + lf] * 4 + m.enbr_lf[e * 4 + lf]) * EFC + 4 * NQ;
      for (int c = 0; c < 5; c++) {
        fncoef[(size_t)(5 * s + c) * FN + fn] = hs[c];
        eo[(5 * s + c) * NGL + n] = hs[c];
        en[(5 * s + c) * NGL + n] = hs[c];
      }
    } else {
      const double nx = m.fnstat[FN_NX * FN + fn], ny = m.fnstat[FN_NY * FN + fn];
      double bsum[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        const double d = s_q[k][0][p];
        double l[5], r[5];
        for (int c = 0; c < 4; c++) l[c] = d * s_g[k][c][p];
        l[4] = d;
        bcl_face_ghost(l, r, er, nx, ny);
        for (int c = 0; c < 5; c++) {
          gdpp_face[((size_t)k * 10 + c) * FN + fn] = l[c];
          gdpp_face[((size_t)k * 10 + 5 + c) * FN + fn] = r[c];
        }
        for (int c = 0; c < 5; c++) {
          bsum[c] = bsum[c] + l[c];
          bsum[5 + c] = bsum[5 + c] + r[c];
        }
      }
      for (int c = 0; c < 10; c++) {
        fncoef[(size_t)c * FN + fn] = bsum[c];
        eo[c * NGL + n] = bsum[c];
      }
    }
  }
}

// ========================================================= btp_bcl_coeffs_qdf: faces
// Q_*_dp_edge, H_bcl_edge at face quad points (mod_barotropic_terms.F90:306-337) and the
// face traces graduv_dpp_face + their layer sum btp_graduv_dpp_face (:339-407).
template <int NGL, int NQ>
__global__ void __launch_bounds__(64)
    bcl_coeffs_face_kernel(DevMesh m, double *qf, const double *qf_avg, const double *dpp_graduv,
                           const double *dpprime_visc, double *fcoef, double *fncoef, double *gdpp_face,
                           double *efcoef) {
  // qf_avg (the corrector): qprime_face2 = 0.5*(qprime_face + qprime_face2) of the face first
  // (ti_rk_bcl.F90:65), written back
  const int f = blockIdx.x, tid = threadIdx.x, F = m.nface, L = m.L, npoin = m.npoin;
  __shared__ double s_psiq[NGL * NQ];
  __shared__ double s_qf[MAXL][6 * NGL];
  __shared__ double s_lr[MAXL][2][5][NGL];  // dpp_graduv(4), dpprime_visc at the left | right face nodes
  const size_t FQ = (size_t)F * NQ, FN = (size_t)F * NGL;
  const int erf = m.fer[f];
  for (int t = tid; t < NGL * NQ; t += 64) s_psiq[t] = m.basis[t];
  for (int t = tid; t < L * 6 * NGL; t += 64) {
    const int k = t / (6 * NGL), r = t % (6 * NGL);
    const size_t i = ((size_t)k * F + f) * NGL * 6 + r;
    double v = qf[i];
    if (qf_avg) {
      v = 0.5 * (qf_avg[i] + v);
      qf[i] = v;
    }
    s_qf[k][r] = v;
  }
  for (int t = tid; t < L * 2 * 5 * NGL; t += 64) {
    const int k = t / (10 * NGL), sd = (t / (5 * NGL)) % 2, c = (t / NGL) % 5, n = t % NGL;
    if (sd == 1 && erf <= 0) continue;
    const int I = (sd ? m.fnodeR : m.fnodeL)[(size_t)f * NGL + n];
    s_lr[k][sd][c][n] = c < 4 ? dpp_graduv[((size_t)k * 4 + c) * npoin + I] : dpprime_visc[(size_t)k * npoin + I];
  }
  __syncthreads();
  if (tid < NQ) {
    const int iq = tid;
    double quu, quv, qvv, hb;
    bcl_face_quad<NGL, NQ>(m, s_qf, s_psiq, iq, quu, quv, qvv, hb);
    const size_t fq = (size_t)f * NQ + iq;
    fcoef[FC_QUU * FQ + fq] = quu;
    fcoef[FC_QUV * FQ + fq] = quv;
    fcoef[FC_QVV * FQ + fq] = qvv;
    fcoef[FC_HBCL * FQ + fq] = hb;
    // element-side copies [slot][4*NQ + 10*NGL] for both elements of the face
    constexpr int EFC = 4 * NQ + 10 * NGL;
    const int sl = m.fslotL[f], sr = m.fslotR[f];
    const double vals[4] = {quu, quv, qvv, hb};
    for (int c = 0; c < 4; c++) {
      efcoef[(size_t)sl * EFC + c * NQ + iq] = vals[c];
      if (sr >= 0) efcoef[(size_t)sr * EFC + c * NQ + iq] = vals[c];
    }
  } else if (tid >= 32 && tid < 32 + NGL) {
    const int n = tid - 32, er = erf;
    const size_t fn = (size_t)f * NGL + n;
    double nx = m.fnstat[FN_NX * FN + fn], ny = m.fnstat[FN_NY * FN + fn];
    double bsum[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      double l[5], r[5];
      for (int c = 0; c < 5; c++) l[c] = s_lr[k][0][c][n];
      if (er > 0) {
        for (int c = 0; c < 5; c++) r[c] = s_lr[k][1][c][n];
      } else {
        bcl_face_ghost(l, r, er, nx, ny);
      }
      for (int c = 0; c < 5; c++) {
        gdpp_face[((size_t)k * 10 + c) * FN + fn] = l[c];
        gdpp_face[((size_t)k * 10 + 5 + c) * FN + fn] = r[c];
      }
      for (int c = 0; c < 5; c++) {
        bsum[c] = bsum[c] + l[c];
        bsum[5 + c] = bsum[5 + c] + r[c];
      }
    }
    for (int c = 0; c < 10; c++) fncoef[(size_t)c * FN + fn] = bsum[c];
    constexpr int EFC = 4 * NQ + 10 * NGL;
    const int sl = m.fslotL[f], sr = m.fslotR[f];
    for (int c = 0; c < 10; c++) {
      efcoef[(size_t)sl * EFC + 4 * NQ + c * NGL + n] = bsum[c];
      if (sr >= 0) efcoef[(size_t)sr * EFC + 4 * NQ + c * NGL + n] = bsum[c];
    }
  }
}

// ====================================================== layer mass: face fluxes
// create_layer_mass_flux (mod_create_rhs_mlswe.F90:922-1034): upwind mass flux per face,
// layer and face quad point: fmass[k][f*NQ+iq] = nx*flux_edge_u + ny*flux_edge_v; the
// element kernels apply -/+ (wq*hi)*flux in the reference's order.
// create_layer_mass_flux at (face f, quad point iq) from the face's qf block staged as s_qf
// [MAXL][6*NGL] (stage_qf): fm[k] = nx*flux_edge_u + ny*flux_edge_v per layer and the layer sums
// (su, sv) -- one restatement for mass_flux_face_kernel and mass_elem_kernel's fused faces
// (its global inputs at (f, iq): the normal and the face averages, MFIn -- loaded ahead by the
// caller, mass_elem_kernel with its other loads)
struct MFIn {
  double nx, ny, qbl0, qbr0, qbl1, qbr1, qbl2, qbr2;
};
template <int NQ>
__device__ __forceinline__ MFIn mass_flux_in(const DevMesh &m, const double *facc, int f, int sa, int iq) {
  const size_t FQ = (size_t)m.nface * NQ, fq = (size_t)f * NQ + iq;
  MFIn x;
  x.nx = m.fstat[FS_NX * FQ + fq];
  x.ny = m.fstat[FS_NY * FQ + fq];
  x.qbl0 = facc[FACC_I(FA_OPEL, sa, iq)];
  x.qbr0 = facc[FACC_I(FA_OPER, sa, iq)];
  x.qbl1 = facc[FACC_I(FA_UL, sa, iq)];
  x.qbr1 = facc[FACC_I(FA_UR, sa, iq)];
  x.qbl2 = facc[FACC_I(FA_VL, sa, iq)];
  x.qbr2 = facc[FACC_I(FA_VR, sa, iq)];
  return x;
}
template <int NGL, int NQ>
__device__ __forceinline__ void mass_flux_at(const DevMesh &m, const double (*s_qf)[6 * NGL], const double *s_psiq,
                                              const MFIn &x, int iq, double fm[MAXL], double &su, double &sv) {
  const int L = m.L;
  const double nxl = x.nx, nyl = x.ny, qbl0 = x.qbl0, qbr0 = x.qbr0, qbl1 = x.qbl1, qbr1 = x.qbr1, qbl2 = x.qbl2,
               qbr2 = x.qbr2;
  su = 0.0;
  sv = 0.0;
#pragma unroll
  for (int k = 0; k < MAXL; k++) {
    if (k >= L) break;
    double ql[3] = {0, 0, 0}, qr[3] = {0, 0, 0};
#pragma unroll
    for (int n = 0; n < NGL; n++) {
      double hi = s_psiq[n * NQ + iq];
      for (int v = 0; v < 3; v++) {
        ql[v] = ql[v] + hi * SQF(v, 0, n, k);
        qr[v] = qr[v] + hi * SQF(v, 1, n, k);
      }
    }
    double uu = 0.5 * ((ql[1] + qbl1) + (qr[1] + qbr1));
    double vv = 0.5 * ((ql[2] + qbl2) + (qr[2] + qbr2));
    double dpl = qbl0 * ql[0], dpr = qbr0 * qr[0];
    double feu = (uu * nxl > 0.0) ? uu * dpl : uu * dpr;
    double fev = (vv * nyl > 0.0) ? vv * dpl : vv * dpr;
    su = su + feu;
    sv = sv + fev;
    fm[k] = nxl * feu + nyl * fev;
  }
}

template <int NGL, int NQ>
__global__ void __launch_bounds__(64)
    mass_flux_face_kernel(DevMesh m, const double *qf, const double *facc, double *fmass, double *slmf_face) {
  const int f = blockIdx.x, tid = threadIdx.x, F = m.nface, L = m.L;
  __shared__ double s_psiq[NGL * NQ];
  __shared__ double s_qf[MAXL][6 * NGL];
  for (int t = tid; t < NGL * NQ; t += 64) s_psiq[t] = m.basis[t];
  stage_qf<NGL>(s_qf, qf, f, F, L, tid, 64);
  __syncthreads();
  const size_t FQ = (size_t)F * NQ;
  if (tid < NQ) {
    const size_t fq = (size_t)f * NQ + tid;
    double fm[MAXL], su, sv;
    mass_flux_at<NGL, NQ>(m, s_qf, s_psiq, mass_flux_in<NQ>(m, facc, f, m.fslotA[f], tid), tid, fm, su, sv);
    for (int k = 0; k < L; k++) fmass[(size_t)k * FQ + fq] = fm[k];
    slmf_face[0 * FQ + fq] = su;
    slmf_face[1 * FQ + fq] = sv;
  }
}

// =============================================== consistency: face deficit fluxes
// evaluate_consistency_face (mod_layer_terms.F90:57-137) + the upwind selection of
// create_consistency_mass_flux (mod_create_rhs_mlswe.F90:1036-1115); dpp = dp'(npoin,L).
// Processor-face halo (cdef != NULL): the side-1 deficits (m11, m21) of every face are kept in
// cdef [L][side][2][F*NQ]; a processor face's side 2 is its neighbour's side 1, which only
// arrives with the exchange (bcl_create_communicator at mod_layer_terms.F90:135), so its flux
// is formed afterwards by cons_flux_proc_kernel.
// evaluate_consistency_face + the upwind selection at face quad point iq of one layer, from the
// face nodes' dp' of the left (dnl) and right (dnr) side: the side-1 deficits m11, m21 and the flux
// -- one restatement for cons_flux_face_kernel and cons_elem_kernel's fused faces
template <int NGL, int NQ>
__device__ __forceinline__ void cons_face_layer(const double *s_psiq, const double *dnl, const double *dnr, int er,
                                                int iq, double pbl, double pbr, double d1, double d2, double nxl,
                                                double nyl, double &m11, double &m21, double &flux) {
  double ql = 0.0, qr = 0.0;
#pragma unroll
  for (int n = 0; n < NGL; n++) ql = ql + s_psiq[n * NQ + iq] * dnl[n];
  if (er > 0) {
#pragma unroll
    for (int n = 0; n < NGL; n++) qr = qr + s_psiq[n * NQ + iq] * dnr[n];
  } else {
    qr = ql;
  }
  double wl = ql / pbl, wr = qr / pbr;
  m11 = wl * d1;
  m21 = wl * d2;
  double m12 = wr * d1, m22 = wr * d2;
  double feu = (m11 * nxl > 0.0) ? m11 : m12;
  double fev = (m21 * nyl > 0.0) ? m21 : m22;
  flux = nxl * feu + nyl * fev;
}

template <int NGL, int NQ>
__global__ void __launch_bounds__(64)
    cons_flux_face_kernel(DevMesh m, const double *dpp, const double *facc, const double *slmf_face, double *fcons,
                          double *cdef) {
  const int f = blockIdx.x, tid = threadIdx.x, F = m.nface, L = m.L, npoin = m.npoin;
  const int erf = m.fer[f];
  __shared__ double s_psiq[NGL * NQ];
  __shared__ double s_dn[MAXL][2][NGL];  // dp' at the left | right face nodes
  for (int t = tid; t < NGL * NQ; t += 64) s_psiq[t] = m.basis[t];
  for (int t = tid; t < L * 2 * NGL; t += 64) {
    const int k = t / (2 * NGL), sd = (t / NGL) % 2, n = t % NGL;
    if (sd == 1 && erf <= 0) continue;
    s_dn[k][sd][n] = dpp[(size_t)k * npoin + (sd ? m.fnodeR : m.fnodeL)[(size_t)f * NGL + n]];
  }
  __syncthreads();
  const size_t FQ = (size_t)F * NQ;
  if (tid < NQ) {
    const int iq = tid, er = erf;
    const size_t fq = (size_t)f * NQ + iq;
    double nxl = m.fstat[FS_NX * FQ + fq], nyl = m.fstat[FS_NY * FQ + fq];
    double d1 = facc[FACC_I(FA_MFX, m.fslotA[f], iq)] - slmf_face[0 * FQ + fq];
    double d2 = facc[FACC_I(FA_MFY, m.fslotA[f], iq)] - slmf_face[1 * FQ + fq];
    double pbl = m.fstat[FS_PBL * FQ + fq], pbr = m.fstat[FS_PBR * FQ + fq];
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      double m11, m21, fl;
      cons_face_layer<NGL, NQ>(s_psiq, s_dn[k][0], s_dn[k][1], er, iq, pbl, pbr, d1, d2, nxl, nyl, m11, m21, fl);
      if (cdef) {
        cdef[((size_t)k * 4 + 0) * FQ + fq] = m11;
        cdef[((size_t)k * 4 + 1) * FQ + fq] = m21;
        if (er == 0) continue;  // processor face: cons_flux_proc_kernel after the exchange
      }
      fcons[(size_t)k * FQ + fq] = fl;
    }
  }
}

// create_consistency_mass_flux (mod_create_rhs_mlswe.F90:1036-1115) on the processor faces,
// with side 2 = the neighbour's side-1 deficits received into cdef: one thread per
// (shared face, quad point).
template <int NQ>
__global__ void cons_flux_proc_kernel(DevMesh m, const double *cdef, const int *sface, int NS, double *fcons) {
  const int F = m.nface, L = m.L;
  const size_t FQ = (size_t)F * NQ;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= NS * NQ) return;
  const int f = sface[t / NQ], iq = t % NQ;
  const size_t fq = (size_t)f * NQ + iq;
  const double nxl = m.fstat[FS_NX * FQ + fq], nyl = m.fstat[FS_NY * FQ + fq];
  for (int k = 0; k < L; k++) {
    const double m11 = cdef[((size_t)k * 4 + 0) * FQ + fq], m21 = cdef[((size_t)k * 4 + 1) * FQ + fq];
    const double m12 = cdef[((size_t)k * 4 + 2) * FQ + fq], m22 = cdef[((size_t)k * 4 + 3) * FQ + fq];
    const double feu = (m11 * nxl > 0.0) ? m11 : m12;
    const double fev = (m21 * nyl > 0.0) ? m21 : m22;
    fcons[(size_t)k * FQ + fq] = nxl * feu + nyl * fev;
  }
}

// btp_graduv_dpp_face side 2 of the processor faces (mod_barotropic_terms.F90:395-407): the
// layer sum of the received graduv_dpp_face (:393), into fncoef and the element-side copies.
template <int NGL, int NQ>
__global__ void bcl_coeffs_proc_kernel(DevMesh m, const double *gdpp_face, const int *sface, int NS, double *fncoef,
                                       double *efcoef) {
  const int F = m.nface, L = m.L;
  const size_t FN = (size_t)F * NGL;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= NS * NGL) return;
  const int f = sface[t / NGL], n = t % NGL;
  const size_t fn = (size_t)f * NGL + n;
  double bsum[5] = {0, 0, 0, 0, 0};
  for (int k = 0; k < L; k++)
    for (int c = 0; c < 5; c++) bsum[c] = bsum[c] + gdpp_face[((size_t)k * 10 + 5 + c) * FN + fn];
  constexpr int EFC = 4 * NQ + 10 * NGL;
  const int sl = m.fslotL[f];
  for (int c = 0; c < 5; c++) {
    fncoef[(size_t)(5 + c) * FN + fn] = bsum[c];
    efcoef[(size_t)sl * EFC + 4 * NQ + (5 + c) * NGL + n] = bsum[c];
  }
}

// Pack / unpack of a face array for the processor-face exchange (send_receive_bound.F90:272-327
// pack_data_dg_*, create_rhs_dynamics_flux.F90:104-182 create_nbhs_face_*): for shared face s
// (face sface[s]), layer k, component c < nc, point n < nn, element
//   base[k*sk + c*sc + f*sf + n*sn]  (side 1)  ->  buf[((s*L + k)*nc + c)*nn + n]
// and back into base[s2 + ...] (side 2).  The message of neighbour j is the slice of its
// faces (contiguous in list order).
__global__ void face_pack_kernel(double *buf, const double *base, const int *sface, int NS, int L, int nc, int nn,
                                 size_t sk, size_t sc, size_t sf, size_t sn) {
  const size_t n = (size_t)NS * L * nc * nn, st = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += st) {
    const int p = (int)(t % nn), c = (int)((t / nn) % nc), k = (int)((t / ((size_t)nn * nc)) % L);
    const int s = (int)(t / ((size_t)nn * nc * L));
    buf[t] = base[k * sk + c * sc + (size_t)sface[s] * sf + p * sn];
  }
}
__global__ void face_unpack_kernel(double *base, const double *buf, const int *sface, int NS, int L, int nc, int nn,
                                   size_t sk, size_t sc, size_t sf, size_t sn, size_t s2) {
  const size_t n = (size_t)NS * L * nc * nn, st = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += st) {
    const int p = (int)(t % nn), c = (int)((t / nn) % nc), k = (int)((t / ((size_t)nn * nc)) % L);
    const int s = (int)(t / ((size_t)nn * nc * L));
    base[s2 + k * sk + c * sc + (size_t)sface[s] * sf + p * sn] = buf[t];
  }
}

// ==================================================== layer mass: element update
// create_layers_volume_mass (mod_create_rhs_mlswe.F90:822-877) + face terms + massinv
// (:74-76), q(1) += dt*dp_advec and the negativity check (mod_splitting.F90:69-78 /
// :224-232), then dp' = q(1)/(sum_k q(1)/pb') for the consistency step (:350-353).
template <int NGL, int NQ, bool BIG>
__global__ void __launch_bounds__((Blk<NGL, NQ>::BSW))
    mass_elem_kernel(DevMesh m, const double *qp, const double *qacc, const double *fmass, const double *q_in,
                     double *q, double *slmf, double *dpp, int *neg_flag, const double *qf, const double *facc,
                     double *slmf_face) {
  // qf != NULL (single rank): the layer mass fluxes of the element's four faces are formed here
  // (mass_flux_at, in place of mass_flux_face_kernel; each face by both its elements, the same
  // bits), the left element of a face writing its layer sums slmf_face for the consistency step
  constexpr int P = Blk<NGL, NQ>::P, Q = Blk<NGL, NQ>::Q, BS = Blk<NGL, NQ>::BSW;
  using QS = typename Blk<NGL, NQ>::template QSB<BIG>;
  static_assert(MAXL * P <= BS, "one quad-point sum per thread");
  BCL_MARK(0, 0) BCL_WALL(0, 6)
  const int e = blk_elem(m), tid = threadIdx.x, L = m.L, npoin = m.npoin, npq = m.npoin_q, F = m.nface;
  __shared__ double s_psiq[NGL * NQ], s_dpsiq[NGL * NQ], s_dpsi[NGL * NGL], s_psi[NGL * NGL];
  __shared__ double s_qm[5][Q];             // e_x, e_y, n_x, n_y, w
  __shared__ double s_f[MAXL][2][Q];        // udp, vdp per layer
  __shared__ double s_adv[MAXL][P];
  __shared__ double s_fw[4 * NQ], s_fx[MAXL][4 * NQ];  // face weights, layer mass fluxes of the 4 faces
  // phase 1's nodal layers and (qf) the four faces' qf blocks, then (phase 2, after the barrier
  // that ends phase 1) the quad-sum term buffers in the same words: at N=7 the element then fits
  // three workgroups per CU (all 625 of dg25 in one round)
  constexpr int U1 = MAXL * 3 * P + 4 * MAXL * 6 * NGL;
  __shared__ double s_un[U1 > QS::SIZE ? U1 : QS::SIZE];
  double(*s_q)[3][P] = reinterpret_cast<double(*)[3][P]>(s_un);
  double(*s_qfF)[MAXL][6 * NGL] = reinterpret_cast<double(*)[MAXL][6 * NGL]>(s_un + MAXL * 3 * P);
  double *s_tb = s_un;
  __shared__ int s_map[4 * NGL], s_face[4], s_side[4];
  // every load of the phase first (Gather), then the LDS stores: the face ids (scalar loads) and
  // the element-major inputs in one round, the face-indexed ones (qf blocks or fluxes, the face
  // tasks' averages) in a second
  const int fid0 = m.efaces[e * 4], fid1 = m.efaces[e * 4 + 1], fid2 = m.efaces[e * 4 + 2], fid3 = m.efaces[e * 4 + 3];
  auto fid = [&](int lf) { return lf == 0 ? fid0 : (lf == 1 ? fid1 : (lf == 2 ? fid2 : fid3)); };
  // the face task's accumulator slot first (round 2 waits for it, and vmcnt counts in order)
  constexpr int FT0 = ((Q + 63) / 64) * 64;
  // (this thread's face task w = FT0 + ft is w = tid or tid + BS: at most one, 4*NQ <= BS)
  static_assert(Q <= BS && 4 * NQ <= BS && FT0 + 4 * NQ <= 2 * BS, "at most one phase-1 task of each kind per thread");
  const int ft = (tid - FT0 + BS) % BS, ft_lf = ft < 4 * NQ ? ft / NQ : 0, ft_iq = ft < 4 * NQ ? ft % NQ : 0;
  const int ft_sa = qf ? m.fslotA[fid(ft_lf)] : 0;
  BasisGather<NGL, NQ, BS> g_bas;
  g_bas.load(m, tid);
  Gather<int, 4, BS> g_side;
  g_side.load(tid, 4, [&](int t) { return m.eside[e * 4 + t]; });
  Gather<double, 4 * NQ, BS> g_fw;  // (efstat's EF_W: fstat's FS_W of the element's faces)
  g_fw.load(tid, 4 * NQ, [&](int t) { return m.efstat[((size_t)e * 4 + t / NQ) * EFBLK(NGL, NQ) + EF_W * NQ + t % NQ]; });
  Gather<int, 4 * NGL, BS> g_map;
  g_map.load(tid, 4 * NGL, [&](int t) { return m.efmap[e * 4 * NGL + t]; });
  Gather<double, MAXL * 3 * P, BS> g_q;
  g_q.load(tid, L * 3 * P, [&](int t) { return qp[(size_t)(t / (3 * P)) * 3 * npoin + (size_t)e * 3 * P + t % (3 * P)]; });
  Gather<double, 5 * Q, BS> g_qm;
  g_qm.load(tid, 5 * Q, [&](int t) {
    const int c = t / Q;
    return m.qstat[(c < 4 ? QS_EX + c : QS_W) * (size_t)npq + (size_t)e * Q + t % Q];
  });
  // phase 1: the quad task's averages (quad point tid) and, with qf, the face task's inputs
  // (thread FT0 + lf*NQ + iq); phase 3: pb' of node tid
  double r_qb[3];
  {
    const int q = tid < Q ? tid : Q - 1;
    r_qb[0] = qacc[QACC_I(QA_OPE, e, q)];
    r_qb[1] = qacc[QACC_I(QA_UB, e, q)];
    r_qb[2] = qacc[QACC_I(QA_VB, e, q)];
  }
  const double r_pb = m.nstat[NS_PB * (size_t)npoin + (size_t)e * P + (tid < P ? tid : P - 1)];
  // (round 2) the face-indexed loads
  Gather<double, 4 * MAXL * 6 * NGL, BS> g_qfF;
  Gather<double, MAXL * 4 * NQ, BS> g_fx;
  MFIn r_mf;
  if (qf) {
    g_qfF.load(tid, 4 * L * 6 * NGL, [&](int t) {
      const int lf = t / (L * 6 * NGL), r = t % (L * 6 * NGL), k = r / (6 * NGL), rr = r % (6 * NGL);
      return qf[((size_t)k * F + fid(lf)) * NGL * 6 + rr];
    });
    r_mf = mass_flux_in<NQ>(m, facc, fid(ft_lf), ft_sa, ft_iq);
  } else {
    g_fx.load(tid, L * 4 * NQ, [&](int t) {
      const int c = t / (4 * NQ), lf = (t / NQ) % 4, iq = t % NQ;
      return fmass[c * (size_t)F * NQ + (size_t)fid(lf) * NQ + iq];
    });
  }
  // the stores
  g_bas.store(s_psiq, s_dpsiq, s_dpsi, s_psi, tid);
  if (tid < 4) s_face[tid] = fid(tid);
  g_side.store(tid, 4, [&](int t, int v) { s_side[t] = v; });
  g_fw.store(tid, 4 * NQ, [&](int t, double v) { s_fw[t] = v; });
  g_map.store(tid, 4 * NGL, [&](int t, int v) { s_map[t] = v; });
  g_q.store(tid, L * 3 * P, [&](int t, double v) {
    const int k = t / (3 * P), r = t % (3 * P);
    s_q[k][r % 3][r / 3] = v;
  });
  g_qm.store(tid, 5 * Q, [&](int t, double v) { s_qm[t / Q][t % Q] = v; });
  if (qf) {
    g_qfF.store(tid, 4 * L * 6 * NGL, [&](int t, double v) {
      const int lf = t / (L * 6 * NGL), r = t % (L * 6 * NGL), k = r / (6 * NGL), rr = r % (6 * NGL);
      s_qfF[lf][k][rr] = v;
    });
  } else {
    g_fx.store(tid, L * 4 * NQ, [&](int t, double v) { (&s_fx[0][0])[t] = v; });
  }
  __syncthreads();
  if (*m.runflag & RUN_ABORT) return;  // (a persistent sub-cycle of this run did no work: DevMesh)
  BCL_MARK(0, 1)
  // quad points [0, Q); with qf, the four faces' flux tasks from the next whole wave on
  for (int w = tid; w < (qf ? FT0 + 4 * NQ : Q); w += BS) {
    if (w >= Q) {
      if (w < FT0) continue;
      const int lf = (w - FT0) / NQ, iq = (w - FT0) % NQ, f = s_face[lf];
      double fm[MAXL], su, sv;
      mass_flux_at<NGL, NQ>(m, s_qfF[lf], s_psiq, r_mf, iq, fm, su, sv);
#pragma unroll
      for (int k = 0; k < MAXL; k++)
        if (k < L) s_fx[k][lf * NQ + iq] = fm[k];
      if (s_side[lf] == 0) {
        const size_t FQ = (size_t)F * NQ, fq = (size_t)f * NQ + iq;
        slmf_face[0 * FQ + fq] = su;
        slmf_face[1 * FQ + fq] = sv;
      }
      continue;
    }
    const int q = w;
    const int iq = q % NQ, jq = q / NQ;
    const size_t Iq = (size_t)e * Q + q;
    const double qb0 = r_qb[0], qb1 = r_qb[1], qb2 = r_qb[2];
    double pa[NGL], pb[NGL];
#pragma unroll
    for (int n = 0; n < NGL; n++) {
      pa[n] = s_psiq[n * NQ + iq];
      pb[n] = s_psiq[n * NQ + jq];
    }
    double su = 0.0, sv = 0.0;
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      double qq[3];
      interp_q<NGL, 3>(pa, pb, &s_q[k][0][0], P, qq);
      double dp_temp = qq[0] * qb0;
      double udp = (qq[1] + qb1) * dp_temp;
      double vdp = (qq[2] + qb2) * dp_temp;
      su = su + udp;
      sv = sv + vdp;
      s_f[k][0][q] = udp;
      s_f[k][1][q] = vdp;
    }
    slmf[0 * (size_t)npq + Iq] = su;
    slmf[1 * (size_t)npq + Iq] = sv;
  }
  __syncthreads();
  BCL_MARK(0, 2)
  {
    // thread t: node p, layer k -- the weak-form divergence (ordered_node_sums), then the faces
    const int t = tid, p = t / MAXL, k = t % MAXL;
    const bool mine = t < P * MAXL && k < L;
    const size_t I = (size_t)e * P + p;
    double r_mi = 0.0, r_q = 0.0;
    if (mine) {
      r_mi = m.nstat[NS_MINV * (size_t)npoin + I];
      r_q = q_in[((size_t)k * npoin + I) * 3];  // (q_in: the predictor reads q_df, writes q_df2)
    }
    double acc = ordered_node_sums<NQ, P, MAXL, BS, QS>(s_tb, tid, L, [&](int pp, int qd, double *dst, int st) {
      weak_div_terms<NGL, NQ>(s_psiq, s_dpsiq, s_qm, s_f, L, pp, qd, dst, st);
    });
    BCL_MARK(0, 3)
    if (mine) {
      int r0, r1;
      node_faces<NGL>(s_map, p, r0, r1);
      acc = face_terms_at<NGL, NQ>(s_psiq, s_side, s_fw, s_fx[k], r0, r1, acc);
      double adv = r_mi * acc;
      double v = r_q + m.dt * adv;
      if (v < 0.0) atomicOr(neg_flag, 1);
      q[((size_t)k * npoin + I) * 3] = v;
      s_adv[k][p] = v;
    }
  }
  __syncthreads();
  BCL_MARK(0, 4)
  for (int p = tid; p < P; p += BS) {
    const size_t I = (size_t)e * P + p;
    double sum = 0.0;
    for (int k = 0; k < L; k++) sum = sum + s_adv[k][p];
    double ope = sum / r_pb;  // (p == tid: P <= BS)
    for (int k = 0; k < L; k++) dpp[(size_t)k * npoin + I] = s_adv[k][p] / ope;
  }
  BCL_MARK(0, 5) BCL_WALL(0, 7)
}

// ============================================== consistency: element update
// create_consistency_volume_mass (mod_create_rhs_mlswe.F90:879-920) + face terms, then
// q(1) += dt*massinv*dp_advec (mod_splitting.F90:362-364).  finalize_dp (thickness): also
// qprime(1,:,k) = q(1,:,k)/(sum_k q(1)/pb') (mod_splitting.F90:84-87).
template <int NGL, int NQ, bool BIG>
__global__ void __launch_bounds__((Blk<NGL, NQ>::BSW))
    cons_elem_kernel(DevMesh m, const double *dpp, const double *qacc, const double *slmf, const double *fcons,
                     double *q, double *qp_out, int finalize_dp, double *qf, const double *facc,
                     const double *slmf_face) {
  // facc != NULL (single rank): the consistency fluxes of the element's four faces are formed here
  // (cons_face_layer, in place of cons_flux_face_kernel; each face by both its elements, the same bits)
  // qf (finalize_dp, single rank): extract_dprime_df_face of the new thickness fused into the
  // finalize (extract_node_faces), in place of the extract launch after this kernel
  constexpr int P = Blk<NGL, NQ>::P, Q = Blk<NGL, NQ>::Q, BS = Blk<NGL, NQ>::BSW;
  using QS = typename Blk<NGL, NQ>::template QSB<BIG>;
  static_assert(MAXL * P <= BS, "one quad-point sum per thread");
  BCL_MARK(1, 0) BCL_WALL(1, 6)
  const int e = blk_elem(m), tid = threadIdx.x, L = m.L, npoin = m.npoin, npq = m.npoin_q, F = m.nface;
  __shared__ double s_psiq[NGL * NQ], s_dpsiq[NGL * NQ], s_dpsi[NGL * NGL], s_psi[NGL * NGL];
  __shared__ double s_d[MAXL][P];
  __shared__ double s_qm[5][Q];
  __shared__ double s_f[MAXL][2][Q];
  __shared__ double s_new[MAXL][P];
  __shared__ double s_fw[4 * NQ], s_fx[MAXL][4 * NQ];  // face weights, consistency fluxes of the 4 faces
  __shared__ double s_tb[QS::SIZE];                    // quad-sum term buffers
  __shared__ double s_dnF[4][MAXL][2][NGL];            // (facc) dp' at the four faces' left | right nodes
  __shared__ int s_map[4 * NGL], s_face[4], s_side[4], s_bc[4];
  // every load of the phase first (Gather), then the LDS stores: the face ids (scalar loads), then
  // the face-indexed tables (node ids, accumulator slots) and the element-major inputs, then the
  // face-indexed data
  const int fid0 = m.efaces[e * 4], fid1 = m.efaces[e * 4 + 1], fid2 = m.efaces[e * 4 + 2], fid3 = m.efaces[e * 4 + 3];
  auto fid = [&](int lf) { return lf == 0 ? fid0 : (lf == 1 ? fid1 : (lf == 2 ? fid2 : fid3)); };
  constexpr int FT0 = ((Q + 63) / 64) * 64;
  // (this thread's face task w = FT0 + ft is w = tid or tid + BS: at most one, 4*NQ <= BS)
  static_assert(Q <= BS && 4 * NQ <= BS && FT0 + 4 * NQ <= 2 * BS, "at most one phase-1 task of each kind per thread");
  const int ft = (tid - FT0 + BS) % BS, ft_lf = ft < 4 * NQ ? ft / NQ : 0, ft_iq = ft < 4 * NQ ? ft % NQ : 0;
  const int ft_f = fid(ft_lf);
  const int ft_sa = facc ? m.fslotA[ft_f] : 0;
  // (facc) dp' at the four faces' left | right nodes, entry t = (lf, k, sd, n): the node ids
  // (fnodeL / fnodeR, -1 on a side without an element) first, the values after them
  constexpr int NDI = (4 * MAXL * 2 * NGL + BS - 1) / BS;
  const int nd = 4 * L * 2 * NGL;
  auto dnf_idx = [&](int t, int &lf, int &k, int &sd, int &n) {
    lf = t / (L * 2 * NGL);
    const int r = t % (L * 2 * NGL);
    k = r / (2 * NGL);
    sd = (r / NGL) % 2;
    n = r % NGL;
  };
  int dn_id[NDI];
  double dn_v[NDI];
  if (facc) {
#pragma unroll
    for (int j = 0; j < NDI; j++) {
      const int t = tid + j * BS;
      int lf, k, sd, n;
      dnf_idx(t < nd ? t : nd - 1, lf, k, sd, n);
      dn_id[j] = (sd ? m.fnodeR : m.fnodeL)[(size_t)fid(lf) * NGL + n];
    }
  }
  BasisGather<NGL, NQ, BS> g_bas;
  g_bas.load(m, tid);
  Gather<int, 4, BS> g_side, g_bc;
  g_side.load(tid, 4, [&](int t) { return m.eside[e * 4 + t]; });
  g_bc.load(tid, 4, [&](int t) { return m.ebc[e * 4 + t]; });
  Gather<double, 4 * NQ, BS> g_fw;  // (efstat's EF_W: fstat's FS_W of the element's faces)
  g_fw.load(tid, 4 * NQ, [&](int t) { return m.efstat[((size_t)e * 4 + t / NQ) * EFBLK(NGL, NQ) + EF_W * NQ + t % NQ]; });
  Gather<int, 4 * NGL, BS> g_map;
  g_map.load(tid, 4 * NGL, [&](int t) { return m.efmap[e * 4 * NGL + t]; });
  Gather<double, MAXL * P, BS> g_d;
  g_d.load(tid, L * P, [&](int t) { return dpp[(size_t)(t / P) * npoin + (size_t)e * P + t % P]; });
  Gather<double, 5 * Q, BS> g_qm;
  g_qm.load(tid, 5 * Q, [&](int t) {
    const int c = t / Q;
    return m.qstat[(c < 4 ? QS_EX + c : QS_W) * (size_t)npq + (size_t)e * Q + t % Q];
  });
  // phase 1: the quad task's inputs (quad point tid) and, with facc, the face task's; the
  // finalize: pb' of node tid
  double r_pbq, r_dx0, r_dx1, r_dy0, r_dy1;
  {
    const size_t Iq = (size_t)e * Q + (tid < Q ? tid : Q - 1);
    r_pbq = m.qstat[QS_PB * (size_t)npq + Iq];
    r_dx0 = qacc[QACC_I(QA_MFX, e, 0) + (Iq - (size_t)e * Q)];
    r_dx1 = slmf[0 * (size_t)npq + Iq];
    r_dy0 = qacc[QACC_I(QA_MFY, e, 0) + (Iq - (size_t)e * Q)];
    r_dy1 = slmf[1 * (size_t)npq + Iq];
  }
  const double r_pbn = m.nstat[NS_PB * (size_t)npoin + (size_t)e * P + (tid < P ? tid : P - 1)];
  double f_nx = 0.0, f_ny = 0.0, f_s1 = 0.0, f_s2 = 0.0, f_pbl = 0.0, f_pbr = 0.0, f_a1 = 0.0, f_a2 = 0.0;
  if (facc) {
    const size_t FQ = (size_t)F * NQ, fq = (size_t)ft_f * NQ + ft_iq;
    f_nx = m.fstat[FS_NX * FQ + fq];
    f_ny = m.fstat[FS_NY * FQ + fq];
    f_s1 = slmf_face[0 * FQ + fq];
    f_s2 = slmf_face[1 * FQ + fq];
    f_pbl = m.fstat[FS_PBL * FQ + fq];
    f_pbr = m.fstat[FS_PBR * FQ + fq];
    f_a1 = facc[FACC_I(FA_MFX, ft_sa, ft_iq)];
    f_a2 = facc[FACC_I(FA_MFY, ft_sa, ft_iq)];
  }
  // the face-indexed data: dp' at the faces' nodes, or the faces' fluxes
  Gather<double, MAXL * 4 * NQ, BS> g_fx;
  if (facc) {
#pragma unroll
    for (int j = 0; j < NDI; j++) {
      const int t = tid + j * BS;
      int lf, k, sd, n;
      dnf_idx(t < nd ? t : nd - 1, lf, k, sd, n);
      dn_v[j] = dpp[(size_t)k * npoin + (dn_id[j] >= 0 ? dn_id[j] : 0)];
    }
  } else {
    g_fx.load(tid, L * 4 * NQ, [&](int t) {
      const int c = t / (4 * NQ), lf = (t / NQ) % 4, iq = t % NQ;
      return fcons[c * (size_t)F * NQ + (size_t)fid(lf) * NQ + iq];
    });
  }
  // the stores
  g_bas.store(s_psiq, s_dpsiq, s_dpsi, s_psi, tid);
  if (tid < 4) s_face[tid] = fid(tid);
  g_side.store(tid, 4, [&](int t, int v) { s_side[t] = v; });
  g_bc.store(tid, 4, [&](int t, int v) { s_bc[t] = v; });
  g_fw.store(tid, 4 * NQ, [&](int t, double v) { s_fw[t] = v; });
  g_map.store(tid, 4 * NGL, [&](int t, int v) { s_map[t] = v; });
  g_d.store(tid, L * P, [&](int t, double v) { s_d[t / P][t % P] = v; });
  g_qm.store(tid, 5 * Q, [&](int t, double v) { s_qm[t / Q][t % Q] = v; });
  if (facc) {
#pragma unroll
    for (int j = 0; j < NDI; j++) {
      const int t = tid + j * BS;
      int lf, k, sd, n;
      dnf_idx(t, lf, k, sd, n);
      if (t < nd && dn_id[j] >= 0) s_dnF[lf][k][sd][n] = dn_v[j];  // (no right element: never read)
    }
  } else {
    g_fx.store(tid, L * 4 * NQ, [&](int t, double v) { (&s_fx[0][0])[t] = v; });
  }
  __syncthreads();
  if (*m.runflag & RUN_ABORT) return;  // (a persistent sub-cycle of this run did no work: DevMesh)
  BCL_MARK(1, 1)
  // quad points [0, Q); with facc, the four faces' flux tasks from the next whole wave on
  for (int w = tid; w < (facc ? FT0 + 4 * NQ : Q); w += BS) {
    if (w >= Q) {
      if (w < FT0) continue;
      const int lf = (w - FT0) / NQ, iq = (w - FT0) % NQ, er = s_bc[lf];  // (== ft_lf, ft_iq)
      const double nxl = f_nx, nyl = f_ny;
      const double d1 = f_a1 - f_s1;
      const double d2 = f_a2 - f_s2;
      const double pbl = f_pbl, pbr = f_pbr;
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        double m11, m21, fl;
        cons_face_layer<NGL, NQ>(s_psiq, s_dnF[lf][k][0], s_dnF[lf][k][1], er, iq, pbl, pbr, d1, d2, nxl, nyl, m11,
                                 m21, fl);
        s_fx[k][lf * NQ + iq] = fl;
      }
      continue;
    }
    const int q = w;
    const int iq = q % NQ, jq = q / NQ;
    double pb = r_pbq;
    double dx = r_dx0 - r_dx1;
    double dy = r_dy0 - r_dy1;
    double pa[NGL], pbq[NGL];
#pragma unroll
    for (int n = 0; n < NGL; n++) {
      pa[n] = s_psiq[n * NQ + iq];
      pbq[n] = s_psiq[n * NQ + jq];
    }
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      double dpv[1];
      interp_q<NGL, 1>(pa, pbq, &s_d[k][0], P, dpv);
      const double dp = dpv[0];
      double weight = dp / pb;
      s_f[k][0][q] = weight * dx;
      s_f[k][1][q] = weight * dy;
    }
  }
  __syncthreads();
  BCL_MARK(1, 3)
  {
    // thread t: node p, layer k -- the weak-form divergence (ordered_node_sums), then the faces
    const int t = tid, p = t / MAXL, k = t % MAXL;
    const bool mine = t < P * MAXL && k < L;
    const size_t I = (size_t)e * P + p;
    double r_mi = 0.0, r_q = 0.0;
    if (mine) {
      r_mi = m.nstat[NS_MINV * (size_t)npoin + I];
      r_q = q[((size_t)k * npoin + I) * 3];
    }
    double acc = ordered_node_sums<NQ, P, MAXL, BS, QS>(s_tb, tid, L, [&](int pp, int qd, double *dst, int st) {
      weak_div_terms<NGL, NQ>(s_psiq, s_dpsiq, s_qm, s_f, L, pp, qd, dst, st);
    });
    if (mine) {
      int r0, r1;
      node_faces<NGL>(s_map, p, r0, r1);
      acc = face_terms_at<NGL, NQ>(s_psiq, s_side, s_fw, s_fx[k], r0, r1, acc);
      double v = r_q + m.dt * r_mi * acc;
      q[((size_t)k * npoin + I) * 3] = v;
      s_new[k][p] = v;
    }
  }
  if (!finalize_dp) return;
  __syncthreads();
  BCL_MARK(1, 4)
  for (int p = tid; p < P; p += BS) {
    const size_t I = (size_t)e * P + p;
    double sum = 0.0;
    for (int k = 0; k < L; k++) sum = sum + s_new[k][p];
    double ope = sum / r_pbn;  // (p == tid: P <= BS)
    double v[MAXL][3];
    for (int k = 0; k < L; k++) {
      v[k][0] = s_new[k][p] / ope;
      qp_out[((size_t)k * npoin + I) * 3] = v[k][0];
    }
    if (qf) {
      int r0, r1;
      node_faces<NGL>(s_map, p, r0, r1);
      extract_node_faces<NGL>(m, qf, s_face, s_side, s_bc, r0, r1, v, 1);
    }
  }
  BCL_MARK(1, 5) BCL_WALL(1, 7)
}

// ========================================== layer momentum: face kernel
// Apply_layers_fluxes (mod_create_rhs_mlswe.F90:458-820) and the layer LDG flux
// bcl_create_rhs_laplacian_flux (mod_laplacian_quad.F90:521-611).  Outputs per face
// face quad point: (nx*H_face + flux_x, ny*H_face + flux_y) of the left / right side into the
// element-side slot (fslotL / fslotR) of that side, momL[slot][L][2][NQ] (MSLOT; the element
// kernel applies -/+ (wq*hi)*value in reference order and loads its four slots without first
// reading its face ids), and per face node wq*psi(n,n)*flux (LDG; + for left, - for right) into
// both sides' slots, lap[slot][L][2][NGL].  (momR is unused.)
template <int NGL, int NQ>
__global__ void __launch_bounds__(64)
    mom_flux_face_kernel(DevMesh m, const double *qf, const double *facc, const double *gdpp_face,
                         const double *gfacc, double *momL, double *momR, double *lap, const double *qf_avg0) {
  // qf_avg0 (the corrector): the face thickness traces enter as 0.5*(qf_avg0 + qf) (component 1,
  // ti_rk_bcl.F90:80), formed on load
  const int f = blockIdx.x, tid = threadIdx.x, F = m.nface, L = m.L;
  const size_t FQ = (size_t)F * NQ, FN = (size_t)F * NGL;
  BCL_MARK(3, 0) BCL_WALL(3, 6)
  const int slot = m.fslotA[f], slotL = m.fslotL[f], slotR = m.fslotR[f];
  // every input of the face in one round of independent loads (the face's qf block per layer,
  // its 16 averages, the LDG face averages and coefficients, the face statics), then the
  // arithmetic from LDS: one memory round trip instead of one per dependent step
  __shared__ double s_psiq[NGL * NQ], s_psi[NGL * NGL];
  __shared__ double s_qf[MAXL][NGL * 6];          // qf(v, side, n) of each layer
  __shared__ double s_fa[FA_N * NQ];              // face averages (FACC_I order)
  __shared__ double s_gf[8 * NGL];                // graduvb face averages, left | right
  __shared__ double s_gd[MAXL][10][NGL];          // graduv_dpp_face per layer
  __shared__ double s_fs[4][NQ];                  // nx, ny, zbot left, zbot right at the quad points
  __shared__ double s_fn[3][NGL];                 // nx, ny, w at the face nodes
  // (Gather: every load, then the stores)
  Gather<double, NGL * NQ, 64> g_psiq;
  g_psiq.load(tid, NGL * NQ, [&](int t) { return m.basis[t]; });
  Gather<double, NGL * NGL, 64> g_psi;
  g_psi.load(tid, NGL * NGL, [&](int t) { return m.basis[2 * NGL * NQ + NGL * NGL + t]; });
  auto qf_i = [&](int t) { return ((size_t)(t / (6 * NGL)) * F + f) * NGL * 6 + t % (6 * NGL); };
  Gather<double, MAXL * 6 * NGL, 64> g_qf, g_qfa;
  g_qf.load(tid, L * 6 * NGL, [&](int t) { return qf[qf_i(t)]; });
  if (qf_avg0) g_qfa.load(tid, L * 6 * NGL, [&](int t) { return qf_avg0[qf_i(t)]; });
  Gather<double, FA_N * NQ, 64> g_fa;
  g_fa.load(tid, FA_N * NQ, [&](int t) { return facc[FACC_I(0, slot, 0) + t]; });
  Gather<double, 8 * NGL, 64> g_gf;
  g_gf.load(tid, 8 * NGL, [&](int t) { return gfacc[GFACC_I(0, slot, 0) + t]; });
  Gather<double, MAXL * 10 * NGL, 64> g_gd;
  g_gd.load(tid, L * 10 * NGL, [&](int t) {
    const int k = t / (10 * NGL), c = (t / NGL) % 10, n = t % NGL;
    return gdpp_face[((size_t)k * 10 + c) * FN + (size_t)f * NGL + n];
  });
  Gather<double, 4 * NQ, 64> g_fs;
  g_fs.load(tid, 4 * NQ, [&](int t) {
    const int c = t / NQ, iq = t % NQ;
    const int fld = c == 0 ? FS_NX : (c == 1 ? FS_NY : (c == 2 ? FS_ZBL : FS_ZBR));
    return m.fstat[fld * FQ + (size_t)f * NQ + iq];
  });
  Gather<double, 3 * NGL, 64> g_fn;
  g_fn.load(tid, 3 * NGL, [&](int t) {
    const int c = t / NGL, n = t % NGL;
    const int fld = c == 0 ? FN_NX : (c == 1 ? FN_NY : FN_W);
    return m.fnstat[fld * FN + (size_t)f * NGL + n];
  });
  g_psiq.store(tid, NGL * NQ, [&](int t, double v) { s_psiq[t] = v; });
  g_psi.store(tid, NGL * NGL, [&](int t, double v) { s_psi[t] = v; });
  g_qf.store_j(tid, L * 6 * NGL, [&](int t, int j) {
    const int k = t / (6 * NGL), r = t % (6 * NGL);
    double v = g_qf.v[j];
    if (qf_avg0 && r % 3 == 0) v = 0.5 * (g_qfa.v[j] + v);
    s_qf[k][r] = v;
  });
  g_fa.store(tid, FA_N * NQ, [&](int t, double v) { s_fa[t] = v; });
  g_gf.store(tid, 8 * NGL, [&](int t, double v) { s_gf[t] = v; });
  g_gd.store(tid, L * 10 * NGL, [&](int t, double v) { (&s_gd[0][0][0])[t] = v; });
  g_fs.store(tid, 4 * NQ, [&](int t, double v) { s_fs[t / NQ][t % NQ] = v; });
  g_fn.store(tid, 3 * NGL, [&](int t, double v) { s_fn[t / NGL][t % NGL] = v; });
  __syncthreads();
  BCL_MARK(3, 1)
  const int er = m.fer[f];
  const double g = m.gravity, eps1 = 1.0e-20;
#define FA(k) s_fa[(k) * NQ + iq]
  // two lanes per face quad point, sd = 0 (left) and 1 (right): both form the shared upwind
  // fluxes, each only its own side's layer-overlap pressure H_r and output
  static_assert(2 * NQ <= 32, "quad lanes below the LDG lanes");
  if (tid < 2 * NQ) {
    const int sd = tid / NQ, iq = tid - sd * NQ;
    const double *alpha = m.alpha;
    double nxl = s_fs[0][iq], nyl = s_fs[1][iq];
    double qbl0 = FA(FA_OPEL), qbr0 = FA(FA_OPER);
    double qbl1 = FA(FA_UL), qbr1 = FA(FA_UR);
    double qbl2 = FA(FA_VL), qbr2 = FA(FA_VR);
    double ql[MAXL][3], qr[MAXL][3], udpl[MAXL], udpr[MAXL], vdpl[MAXL], vdpr[MAXL];
    double udpf[2][MAXL], vdpf[2][MAXL];
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      for (int v = 0; v < 3; v++) ql[k][v] = qr[k][v] = 0.0;
#pragma unroll
      for (int n = 0; n < NGL; n++) {
        double hi = s_psiq[n * NQ + iq];
        for (int v = 0; v < 3; v++) {
          ql[k][v] = ql[k][v] + hi * s_qf[k][(n * 2 + 0) * 3 + v];
          qr[k][v] = qr[k][v] + hi * s_qf[k][(n * 2 + 1) * 3 + v];
        }
      }
      double dpl = qbl0 * ql[k][0], dpr = qbr0 * qr[k][0];
      double ul = ql[k][1] + qbl1, ur = qr[k][1] + qbr1, vl = ql[k][2] + qbl2, vr = qr[k][2] + qbr2;
      double uu = 0.5 * (ul + ur), vv = 0.5 * (vl + vr);
      udpl[k] = ul * dpl;
      udpr[k] = ur * dpr;
      vdpl[k] = vl * dpl;
      vdpr[k] = vr * dpr;
      if (uu * nxl > 0.0) {
        udpf[0][k] = uu * (ul * dpl);
        vdpf[0][k] = uu * (vl * dpl);
      } else {
        udpf[0][k] = uu * (ur * dpr);
        vdpf[0][k] = uu * (vr * dpr);
      }
      if (vv * nyl > 0.0) {
        udpf[1][k] = vv * (ul * dpl);
        vdpf[1][k] = vv * (vl * dpl);
      } else {
        udpf[1][k] = vv * (ur * dpr);
        vdpf[1][k] = vv * (vr * dpr);
      }
    }
    double s1 = 0, s2 = 0, s3 = 0, s4 = 0;
#pragma unroll
    for (int k = 0; k < MAXL; k++)
      if (k < L) s1 = s1 + udpf[0][k];
#pragma unroll
    for (int k = 0; k < MAXL; k++)
      if (k < L) s2 = s2 + udpf[1][k];
#pragma unroll
    for (int k = 0; k < MAXL; k++)
      if (k < L) s3 = s3 + vdpf[0][k];
#pragma unroll
    for (int k = 0; k < MAXL; k++)
      if (k < L) s4 = s4 + vdpf[1][k];
    double uu_def = FA(FA_QUU) - s1, uv_def = FA(FA_QUV) - s2;
    double vu_def = FA(FA_QVU) - s3, vv_def = FA(FA_QVV) - s4;
    double sl = 0, sr = 0;
#pragma unroll
    for (int k = 0; k < MAXL; k++)
      if (k < L) sl = sl + (fabs(udpl[k]) + eps1);
#pragma unroll
    for (int k = 0; k < MAXL; k++)
      if (k < L) sr = sr + (fabs(udpr[k]) + eps1);
    double oosl = 1.0 / sl, oosr = 1.0 / sr;
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      udpf[0][k] = udpf[0][k] + ((uu_def * nxl > 0.0) ? fabs(udpl[k]) * oosl : fabs(udpr[k]) * oosr) * uu_def;
      udpf[1][k] = udpf[1][k] + ((uv_def * nyl > 0.0) ? fabs(udpl[k]) * oosl : fabs(udpr[k]) * oosr) * uv_def;
    }
    sl = 0;
    sr = 0;
#pragma unroll
    for (int k = 0; k < MAXL; k++)
      if (k < L) sl = sl + (fabs(vdpl[k]) + eps1);
#pragma unroll
    for (int k = 0; k < MAXL; k++)
      if (k < L) sr = sr + (fabs(vdpr[k]) + eps1);
    oosl = 1.0 / sl;
    oosr = 1.0 / sr;
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      vdpf[0][k] = vdpf[0][k] + ((vu_def * nxl > 0.0) ? fabs(vdpl[k]) * oosl : fabs(vdpr[k]) * oosr) * vu_def;
      vdpf[1][k] = vdpf[1][k] + ((vv_def * nyl > 0.0) ? fabs(vdpl[k]) * oosl : fabs(vdpr[k]) * oosr) * vv_def;
    }
    // H_r at the face (layer-overlap pressure, :627-707), side sd: the reference's left and right
    // formulas are mirror images -- own = this side's layer pressure, other = the overlap sum over
    // the other side's layers (zo, po) against this side's interfaces (zs); the left side adds
    // 0.5*(own + other), the right 0.5*(other + own): the same sum
    double pf[MAXL + 1], zf[MAXL + 1], pep[MAXL + 1], pem[MAXL + 1], zep[MAXL + 1], zem[MAXL + 1], Hf[MAXL];
#pragma unroll
    for (int k = 0; k <= MAXL; k++) zf[k] = pf[k] = zep[k] = zem[k] = pep[k] = pem[k] = 0.0;
    const double ope_s = sqrt(sd ? FA(FA_OPE2R) : FA(FA_OPE2L));
#pragma unroll
    for (int k = 1; k <= MAXL; k++) {
      if (k > L) break;
      pf[k] = pf[k - 1] + ope_s * (sd ? qr[k - 1][0] : ql[k - 1][0]);
    }
    const double ope_e = sqrt(FA(FA_OPEE2));
    const double zbl = s_fs[2][iq], zbr = s_fs[3][iq];
#pragma unroll
    for (int k = 1; k <= MAXL; k++)
      if (k == L) {
        zf[k] = sd ? zbr : zbl;
        zep[k] = zbl;
        zem[k] = zbr;
      }
#pragma unroll
    for (int k = MAXL; k >= 1; k--) {
      if (k > L) continue;
      double aog = alpha[k - 1] / g;
      zf[k - 1] = zf[k] + aog * (ope_s * (sd ? qr[k - 1][0] : ql[k - 1][0]));
      zep[k - 1] = zep[k] + aog * (ope_e * ql[k - 1][0]);
      zem[k - 1] = zem[k] + aog * (ope_e * qr[k - 1][0]);
    }
    pep[1] = ope_e * ql[0][0];
    pem[1] = ope_e * qr[0][0];
#pragma unroll
    for (int k = 2; k <= MAXL; k++) {
      if (k > L) break;
      pep[k] = pep[k - 1] + ope_e * ql[k - 1][0];
      pem[k] = pem[k - 1] + ope_e * qr[k - 1][0];
    }
    double zs[MAXL + 1], zo[MAXL + 1], ps[MAXL + 1], po[MAXL + 1];
#pragma unroll
    for (int k = 0; k <= MAXL; k++) {
      zs[k] = sd ? zem[k] : zep[k];
      zo[k] = sd ? zep[k] : zem[k];
      ps[k] = sd ? pem[k] : pep[k];
      po[k] = sd ? pep[k] : pem[k];
    }
#pragma unroll
    for (int k = 1; k <= MAXL; k++) {
      if (k > L) break;
      double own = 0.5 * alpha[k - 1] * (ps[k] * ps[k] - ps[k - 1] * ps[k - 1]);
      double other = 0.0;
#pragma unroll
      for (int kt = 1; kt <= MAXL; kt++) {
        if (kt > L) break;
        double goa = g / alpha[kt - 1];
        double zt = dmin(zo[kt - 1], zs[k - 1]), zb = dmax(zo[kt], zs[k]);
        if (zt - zb > 0.0) {
          double pbot = po[kt] - goa * (zb - zo[kt]);
          double ptop = po[kt] - goa * (zt - zo[kt]);
          other = other + 0.5 * alpha[kt - 1] * (pbot * pbot - ptop * ptop);
        }
      }
      Hf[k - 1] = 0.5 * (own + other);
    }
    if (er == -4) {
#pragma unroll
      for (int k = 1; k <= MAXL; k++) {
        if (k > L) break;
        Hf[k - 1] = 0.5 * alpha[k - 1] * (pf[k] * pf[k] - pf[k - 1] * pf[k - 1]);
      }
    } else {
#pragma unroll
      for (int k = 1; k <= MAXL - 1; k++) {
        if (k > L - 1) break;
        double goa = g / alpha[k - 1];
        double pinc = goa * (zf[k] - zs[k]);
        double Hc = 0.5 * alpha[k - 1] * ((pf[k] + pinc) * (pf[k] + pinc) - pf[k] * pf[k]);
        Hf[k - 1] = Hf[k - 1] - Hc;
        Hf[k] = Hf[k] + Hc;
      }
    }
    {
      double weight = 1.0, acc = 0.0;
#pragma unroll
      for (int k = 0; k < MAXL; k++)
        if (k < L) acc = acc + Hf[k];
      if (acc > 0.0) weight = FA(FA_H) / acc;
#pragma unroll
      for (int k = 0; k < MAXL; k++)
        if (k < L) Hf[k] = Hf[k] * weight;
    }
    const int so = sd ? slotR : slotL;
    if (so >= 0) {
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        double hx = nxl * Hf[k], hy = nyl * Hf[k];
        double flux_x = nxl * udpf[0][k] + nyl * udpf[1][k];
        double flux_y = nxl * vdpf[0][k] + nyl * vdpf[1][k];
        momL[MSLOT(so, k, 0, iq, NQ)] = hx + flux_x;
        momL[MSLOT(so, k, 1, iq, NQ)] = hy + flux_y;
      }
    }
    BCL_MARK(3, 2)
  } else if (tid >= 32 && tid < 32 + NGL) {
    // layer LDG flux at face node n for every layer
    const int n = tid - 32;
    double nx = s_fn[0][n], ny = s_fn[1][n], wq = s_fn[2][n];
    const double beta = 0.5, alpha = 1.0 - beta;
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      double fl[4], fr[4];
      for (int iv = 0; iv < 4; iv++) {
        fl[iv] = s_gd[k][4][n] * s_gf[iv * NGL + n] + s_gd[k][iv][n];
        fr[iv] = s_gd[k][9][n] * s_gf[(4 + iv) * NGL + n] + s_gd[k][5 + iv][n];
      }
      double qum0 = alpha * fl[0] + beta * fr[0], qum1 = alpha * fl[1] + beta * fr[1];
      double qvm0 = alpha * fl[2] + beta * fr[2], qvm1 = alpha * fl[3] + beta * fr[3];
      double flux_qu = (qum0 - fl[0] * nx) + (qum1 - fl[1] * ny);
      double flux_qv = (qvm0 - fl[2] * nx) + (qvm1 - fl[3] * ny);
      double h1 = s_psi[n * NGL + n];
      const double l0 = wq * h1 * flux_qu, l1 = wq * h1 * flux_qv;
      lap[MSLOT(slotL, k, 0, n, NGL)] = l0;
      lap[MSLOT(slotL, k, 1, n, NGL)] = l1;
      if (slotR >= 0) {
        lap[MSLOT(slotR, k, 0, n, NGL)] = l0;
        lap[MSLOT(slotR, k, 1, n, NGL)] = l1;
      }
    }
  }
  BCL_MARK(3, 5) BCL_WALL(3, 7)
#undef FA
}

// ===================================== layer momentum: element volume + update
// rhs_momentum (mod_splitting.F90:289-322): bcl_create_laplacian (mod_laplacian_quad.F90:
// 227-248, :392-425, :521-611) and layer_momentum_rhs = create_rhs_dynamics_volume_layers
// (mod_create_rhs_mlswe.F90:281-456) + Apply_layers_fluxes (:778-817), then the momentum
// update with implicit Coriolis (mod_splitting.F90:131-173 / :239-280), layer_mom_boundary_df
// (mod_layer_terms.F90:529-584) and evaluate_bcl (mode 0, :198-238) / evaluate_bcl_v1
// (mode 1, :240-270).
template <int NGL, int NQ>
struct MomCfg {
  static constexpr int P = NGL * NGL, Q = NQ * NQ;
  static constexpr int BS = 256;
  // waves per SIMD the registers are sized for: three workgroups per CU; N=7 (82 KB of LDS, GIV):
  // two, so at most 256 registers a lane in all
  static constexpr int MINW = NGL >= 8 ? 2 : 3;
};

template <int NGL, int NQ>
__global__ void __launch_bounds__(256, (MomCfg<NGL, NQ>::MINW))
    mom_elem_kernel(DevMesh m, const double *qp_in, const double *qacc, const double *nacc, const double *dpp_graduv,
                    const double *dpprime_visc, const double *momL, const double *momR, const double *lapf,
                    const double *qb, const double *q_in, double *q, double *qp_out, int mode, const double *lapx,
                    const double *dpp2, int *flag, const double *qp_avg0, double *qf) {
  // qf (single rank): extract_qprime_df_face of the new qprime fused into the tail
  // (extract_node_faces), in place of the extract launch after this kernel
  // qp_avg0 (the corrector, non-NULL: dpp2 is then not read): the layer thicknesses qprime(1)
  // enter as 0.5*(qp_avg0 + qp_in) (ti_rk_bcl.F90:78-79, formed on load) and the final qprime(1)
  // is qp_in's own (dpp2 of :78, read back from qp_in).  The engine passes qp_avg0 == qp_out (both
  // qprime_df): safe because every access is element-local -- each workgroup reads its own
  // element's nodes of qp_avg0 into LDS in the load phase and writes the same nodes of qp_out only
  // in its last phase; no workgroup touches another element's nodes of either.
  // q_in: the momenta entering the update (the predictor: q_df, its thicknesses already in q =
  // q_df2); mode 1 (the corrector) writes the step's final qprime straight into qp_out = qprime_df
  // (ti_rk_bcl.F90:81-84: thickness from dpp2 = the corrector's own, momenta from evaluate_bcl_v1)
  // and flags a non-finite barotropic state (bit 2) of its element
  constexpr int P = MomCfg<NGL, NQ>::P, Q = MomCfg<NGL, NQ>::Q, BS = MomCfg<NGL, NQ>::BS;
  const int e = blk_elem(m), tid = threadIdx.x, L = m.L, npoin = m.npoin, npq = m.npoin_q, F = m.nface;
  const double g = m.gravity, eps1 = 1.0e-20;
  BCL_MARK(2, 0) BCL_WALL(2, 6)
  __shared__ double s_psiq[NGL * NQ], s_dpsiq[NGL * NQ], s_dpsi[NGL * NGL], s_psi[NGL * NGL];
  __shared__ double s_qp[MAXL][3][P], s_qm2[MAXL][2][P], s_z[MAXL + 1][P];
  __shared__ double s_qm[5][Q];            // e_x, e_y, n_x, n_y, w at quad points
  __shared__ double s_nm[5][P];            // e_x, e_y, n_x, n_y, w at nodes
  // interpolated dp', u', v', u*dp, v*dp per layer (phases 1-2); then the weak forms' term buffers
  using QS = QSumCfg<NQ, P * 2 * MAXL, 2700>;
  constexpr bool QSUM = P * 2 * MAXL <= BS;  // one weak-form sum per thread (ordered_node_sums)
  // GIV (no term buffers, N=7): s_G in the words of s_iv.  Both are [row][Q], so the coupling task
  // of quad point qd, which reads every s_iv value of column qd before it writes s_G's (the QUIRK
  // row in registers), is the only one touching that column: 108 -> 82 KB, two workgroups per CU
  constexpr bool GIV = !QSUM;
  constexpr int IVTB0 = (QSUM && QS::SIZE > MAXL * 5 * Q) ? QS::SIZE : MAXL * 5 * Q;
  constexpr int IVTB = (GIV && MAXL * 6 * Q > IVTB0) ? MAXL * 6 * Q : IVTB0;
  __shared__ double s_ivtb[IVTB];
  double(*s_iv)[5][Q] = reinterpret_cast<double(*)[5][Q]>(s_ivtb);
  __shared__ double s_Gs[GIV ? 1 : MAXL * 6 * Q];
  double(*s_G)[6][Q] = reinterpret_cast<double(*)[6][Q]>(GIV ? s_ivtb : s_Gs);  // source_x, Hq+uu, uv, source_y, vu, Hq+vv
  __shared__ double s_qq[MAXL][4][P];      // LDG volume fluxes per layer
  __shared__ double s_r[MAXL][4][P];       // rhs_mom(2) and lap(2) per layer
  __shared__ double s_fw[4 * NQ];          // face quad weights of the 4 faces
  __shared__ double s_fm[MAXL][2][4 * NQ]; // momentum face terms of this element's side, per face
  __shared__ double s_fl[MAXL][2][4 * NGL];// layer LDG face fluxes at the face nodes
  __shared__ int s_map[4 * NGL], s_face[4], s_side[4], s_bc[4];
  // the nodal inputs of phase 4 (massinv, f2, A, B, qb(4), pbprime, the layer thicknesses of q
  // and, mode 1, of the final qprime), fetched with the other loads instead of in that phase
  enum { P4_MI = 0, P4_F2, P4_A, P4_B, P4_QB, P4_PB = P4_QB + 4, P4_H, P4_D = P4_H + MAXL, P4_N = P4_D + MAXL };
  __shared__ double s_p4[P4_N][P];

  // quad-point scalars for the layer-coupling task of quad point tid, in flight during
  // the loads and the interpolation
  double r_qa[10], r_qs[3];
  if (tid < Q) {
    const int kk[10] = {QA_OPE, QA_UB, QA_VB, QA_OPE2, QA_QU, QA_QUV, QA_QV, QA_H, QA_TBU, QA_TBV};
#pragma unroll
    for (int c = 0; c < 10; c++) r_qa[c] = qacc[QACC_I(kk[c], e, tid)];
    const size_t Iq = (size_t)e * Q + tid;
    r_qs[0] = m.qstat[QS_TW1 * (size_t)npq + Iq];
    r_qs[1] = m.qstat[QS_TW2 * (size_t)npq + Iq];
    r_qs[2] = m.qstat[QS_PB * (size_t)npq + Iq];
  }
  // every load of the phase first (Gather), then the LDS stores: one memory round trip.  The
  // sources are element-major (the element's face data -- Apply_layers_fluxes' lifts, the LDG face
  // fluxes -- in its own element-side slots), so no load waits for another.
  BasisGather<NGL, NQ, BS> g_bas;
  g_bas.load(m, tid);
  // element record: the face-node map, face ids, sides, boundary codes (one gather per array: a
  // source selected per lane would load its pointer from the kernel arguments first)
  Gather<int, 4 * NGL, BS> g_map;
  g_map.load(tid, 4 * NGL, [&](int t) { return m.efmap[e * 4 * NGL + t]; });
  Gather<int, 4, BS> g_face, g_side, g_bc;
  g_face.load(tid, 4, [&](int t) { return m.efaces[e * 4 + t]; });
  g_side.load(tid, 4, [&](int t) { return m.eside[e * 4 + t]; });
  g_bc.load(tid, 4, [&](int t) { return m.ebc[e * 4 + t]; });
  Gather<double, 4 * NQ, BS> g_fw;
  g_fw.load(tid, 4 * NQ, [&](int t) { return m.efstat[((size_t)e * 4 + t / NQ) * EFBLK(NGL, NQ) + EF_W * NQ + t % NQ]; });
  Gather<double, MAXL * 2 * 4 * NQ, BS> g_fm;
  g_fm.load(tid, L * 2 * 4 * NQ, [&](int t) {
    const int ko = t / (4 * NQ), lf = (t / NQ) % 4, iq = t % NQ;
    return momL[MSLOT(e * 4 + lf, ko >> 1, ko & 1, iq, NQ)];
  });
  Gather<double, MAXL * 2 * 4 * NGL, BS> g_fl;
  g_fl.load(tid, L * 2 * 4 * NGL, [&](int t) {
    const int ko = t / (4 * NGL), lf = (t / NGL) % 4, n = t % NGL;
    return lapf[MSLOT(e * 4 + lf, ko >> 1, ko & 1, n, NGL)];
  });
  // qprime (and, thickness: the corrector's qp_avg0 | momenta: q_in) of every layer
  Gather<double, MAXL * 3 * P, BS> g_qp, g_qx;
  auto qidx = [&](int t) { return (size_t)(t / (3 * P)) * 3 * npoin + (size_t)e * 3 * P + t % (3 * P); };
  g_qp.load(tid, L * 3 * P, [&](int t) { return qp_in[qidx(t)]; });
  g_qx.load(tid, L * 3 * P, [&](int t) {
    const int r = t % (3 * P);
    return ((r % 3 || !qp_avg0) ? q_in : qp_avg0)[qidx(t)];  // (r%3 == 0 without qp_avg0: unused)
  });
  Gather<double, 5 * Q, BS> g_qm;
  g_qm.load(tid, 5 * Q, [&](int t) {
    const int c = t / Q;
    return m.qstat[(c < 4 ? QS_EX + c : QS_W) * (size_t)npq + (size_t)e * Q + t % Q];
  });
  Gather<double, 5 * P, BS> g_nm;
  g_nm.load(tid, 5 * P, [&](int t) {
    const int c = t / P;
    return m.nstat[(c < 4 ? NS_EX + c : NS_W) * (size_t)npoin + (size_t)e * P + t % P];
  });
  Gather<double, P4_N * P, BS> g_p4;
  // (one address per entry, selected: no load under a branch; entries without a source read
  // massinv and are zeroed at the store)
  auto p4_src = [&](int c, int p) -> const double * {
    const size_t I = (size_t)e * P + p;
    const int ns = c == 0 ? NS_MINV : (c == 1 ? NS_F2 : (c == 2 ? NS_A : (c == 3 ? NS_B : NS_PB)));
    const int kh = c - P4_H, kd = c - P4_D;
    if (c < P4_QB || c == P4_PB) return m.nstat + ns * (size_t)npoin + I;
    if (c < P4_PB) return qb + I * 4 + (c - P4_QB);
    if (c < P4_D) return kh < L ? q + ((size_t)kh * npoin + I) * 3 : m.nstat + NS_MINV * (size_t)npoin + I;
    if (mode == 1 && kd < L) return qp_avg0 ? qp_in + ((size_t)kd * npoin + I) * 3 : dpp2 + (size_t)kd * npoin + I;
    return m.nstat + NS_MINV * (size_t)npoin + I;
  };
  auto p4_zero = [&](int c) { return (c >= P4_H && c < P4_D && c - P4_H >= L) || (c >= P4_D && !(mode == 1 && c - P4_D < L)); };
  g_p4.load(tid, P4_N * P, [&](int t) { return *p4_src(t / P, t % P); });
  // phase 1's node task of this thread (task w = L*Q + p: at most one per thread), its inputs
  int my_p = -1;
  static_assert(P <= BS, "one node task per thread");
#pragma unroll
  for (int jw = 0; jw < (MAXL * Q + P + BS - 1) / BS; jw++) {
    const int w = tid + jw * BS;
    if (w >= L * Q && w < L * Q + P) my_p = w - L * Q;
  }
  double r_z, r_so2, r_gs[4], r_dv[MAXL], r_dg[MAXL][4];
  {
    const size_t I = (size_t)e * P + (my_p >= 0 ? my_p : 0);  // (no node task: loaded, unused)
    r_z = m.nstat[NS_ZB * (size_t)npoin + I];
    r_so2 = nacc[NACC_I(NA_OPE2, e, 0) + (I - (size_t)e * P)];
#pragma unroll
    for (int c = 0; c < 4; c++) r_gs[c] = nacc[NACC_I((NA_G1 + c), e, 0) + (I - (size_t)e * P)];
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      const int kk = k < L ? k : L - 1;  // (layers past L: loaded, unused)
      r_dv[k] = dpprime_visc[(size_t)kk * npoin + I];
#pragma unroll
      for (int c = 0; c < 4; c++) r_dg[k][c] = dpp_graduv[((size_t)kk * 4 + c) * npoin + I];
    }
  }
  // the stores
  g_bas.store(s_psiq, s_dpsiq, s_dpsi, s_psi, tid);
  g_map.store(tid, 4 * NGL, [&](int t, int v) { s_map[t] = v; });
  g_face.store(tid, 4, [&](int t, int v) { s_face[t] = v; });
  g_side.store(tid, 4, [&](int t, int v) { s_side[t] = v; });
  g_bc.store(tid, 4, [&](int t, int v) { s_bc[t] = v; });
  g_fw.store(tid, 4 * NQ, [&](int t, double v) { s_fw[t] = v; });
  g_fm.store(tid, L * 2 * 4 * NQ, [&](int t, double v) { (&s_fm[0][0][0])[t] = v; });
  g_fl.store(tid, L * 2 * 4 * NGL, [&](int t, double v) { (&s_fl[0][0][0])[t] = v; });
  g_qp.store_j(tid, L * 3 * P, [&](int t, int j) {
    const int k = t / (3 * P), r = t % (3 * P);
    const double v = g_qp.v[j], x = g_qx.v[j];
    s_qp[k][r % 3][r / 3] = (qp_avg0 && r % 3 == 0) ? 0.5 * (x + v) : v;
    if (r % 3) s_qm2[k][r % 3 - 1][r / 3] = x;
  });
  g_qm.store(tid, 5 * Q, [&](int t, double v) { s_qm[t / Q][t % Q] = v; });
  g_nm.store(tid, 5 * P, [&](int t, double v) { s_nm[t / P][t % P] = v; });
  g_p4.store(tid, P4_N * P, [&](int t, double v) { s_p4[t / P][t % P] = p4_zero(t / P) ? 0.0 : v; });
  __syncthreads();
  if (*m.runflag & RUN_ABORT) return;  // (a persistent sub-cycle of this run did no work: DevMesh)
  // the corrector of a completed step (mode 1) counts it: the host's retry point after an abort
  if (mode == 1 && e == 0 && tid == 0 && m.steps_done) atomicAdd(m.steps_done, 1u);
  BCL_MARK(2, 1)

  // ---- 1: per (layer, quad point) interpolations of dp', u', v', u*dp, v*dp (reference
  //      order: PSIH(n,mm,iq,jq) over mm outer, n inner); per node the layer interfaces
  //      (mod_create_rhs_mlswe.F90:320-325) and the LDG volume fluxes
  //      qq = dpprime_visc*graduvb_ave + dpp_graduv (mod_laplacian_quad.F90:409-413)
  for (int w = tid; w < L * Q + P; w += BS) {
    if (w < L * Q) {
      const int k = w / Q, qd = w % Q, iq = qd % NQ, jq = qd / NQ;
      double pa[NGL], pb[NGL];
#pragma unroll
      for (int n = 0; n < NGL; n++) {
        pa[n] = s_psiq[n * NQ + iq];
        pb[n] = s_psiq[n * NQ + jq];
      }
      double v0 = 0.0, v1 = 0.0, v2 = 0.0, t0 = 0.0, t1 = 0.0;
#pragma unroll 1
      for (int mm = 0; mm < NGL; mm++)
#pragma unroll
        for (int n = 0; n < NGL; n++) {
          const int ip = mm * NGL + n;
          const double hi = pa[n] * pb[mm];
          v0 = v0 + hi * s_qp[k][0][ip];
          v1 = v1 + hi * s_qp[k][1][ip];
          v2 = v2 + hi * s_qp[k][2][ip];
          t0 = t0 + hi * s_qm2[k][0][ip];
          t1 = t1 + hi * s_qm2[k][1][ip];
        }
      s_iv[k][0][qd] = v0;
      s_iv[k][1][qd] = v1;
      s_iv[k][2][qd] = v2;
      s_iv[k][3][qd] = t0;
      s_iv[k][4][qd] = t1;
    } else {
      const int p = w - L * Q;  // (== my_p: its inputs were loaded with the others)
      double z = r_z;
      const double so = sqrt(r_so2);
      s_z[L][p] = z;
      for (int k = L - 1; k >= 0; k--) {
        z = z + (m.alpha[k] / g) * (so * s_qp[k][0][p]);
        s_z[k][p] = z;
      }
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
#pragma unroll
        for (int c = 0; c < 4; c++) s_qq[k][c][p] = r_dv[k] * r_gs[c] + r_dg[k][c];
      }
    }
  }
  __syncthreads();
  BCL_MARK(2, 2)

  // ---- 2: per quad point the layer coupling (mod_create_rhs_mlswe.F90:326-400);
  //      alongside, per (layer, component, node) the LDG Laplacian (mod_laplacian_quad.F90:
  //      392-425, nonzero terms only, then the face terms :521-611)
  const double Pstress = (g / m.alpha[0]) * 50.0;
  const double Pbstress = (g / m.alpha[L - 1]) * 10.0;
  // GZS: the interface-height gradients gz0[k] (x), gz1[k] (y) at the quad points (the coupling's
  // 25-term sums, :339-349) first, one thread per (quad point, direction), into s_gz (in the part
  // of s_ivtb past the interpolations, free until phase 3); the coupling then reads them
  constexpr bool GZS = HNUMO_MOM_GZS && 2 * Q <= BS && MAXL * 5 * Q + 2 * (MAXL + 1) * Q <= IVTB;
  double(*s_gz)[MAXL + 1][Q] = reinterpret_cast<double(*)[MAXL + 1][Q]>(s_ivtb + MAXL * 5 * Q);
  if constexpr (GZS) {
    if (tid < 2 * Q) {
      const int d = tid / Q, qd = tid - d * Q, iq = qd % NQ, jq = qd / NQ;
      double gz[MAXL + 1];
#pragma unroll
      for (int k = 0; k <= MAXL; k++) gz[k] = 0.0;
      double pa[NGL], da[NGL], pb[NGL], db[NGL];
#pragma unroll
      for (int n = 0; n < NGL; n++) {
        pa[n] = s_psiq[n * NQ + iq];
        da[n] = s_dpsiq[n * NQ + iq];
        pb[n] = s_psiq[n * NQ + jq];
        db[n] = s_dpsiq[n * NQ + jq];
      }
      const double ea = s_qm[d][qd], eb = s_qm[2 + d][qd];  // (e_x, n_x) | (e_y, n_y)
#pragma unroll 1
      for (int mm = 0; mm < NGL; mm++)
#pragma unroll
        for (int n = 0; n < NGL; n++) {
          const int ip = mm * NGL + n;
          const double h_e = da[n] * pb[mm], h_n = pa[n] * db[mm];
          const double dd = h_e * ea + h_n * eb;
#pragma unroll
          for (int k = 0; k <= MAXL; k++) {
            if (k > L) break;
            gz[k] = gz[k] + dd * s_z[k][ip];
          }
        }
#pragma unroll
      for (int k = 0; k <= MAXL; k++) s_gz[d][k][qd] = gz[k];
    }
    BCL_LDS_BARRIER();
  }
  for (int w = tid; w < Q + L * 2 * P; w += BS) {
    if (w < Q) {
      const int qd = w, iq = qd % NQ, jq = qd / NQ;
      const double qb0 = r_qa[0], qb1 = r_qa[1], qb2 = r_qa[2];
      const double so2 = sqrt(r_qa[3]);
      double tuu[MAXL], tvv[MAXL], p_tmp[MAXL + 1], H_tmp[MAXL], u_udp[MAXL], v_vdp[MAXL];
      double u_vdp0[MAXL], u_vdp1[MAXL], gz0[MAXL + 1], gz1[MAXL + 1], ppl[MAXL];
      p_tmp[0] = 0.0;
#pragma unroll
      for (int k = 0; k < MAXL; k++)
        if (k < L) ppl[k] = s_iv[L - 1][k][qd];  // (the QUIRK row below, read before s_G is written)
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        const double v0 = s_iv[k][0][qd], v1 = s_iv[k][1][qd], v2 = s_iv[k][2][qd];
        p_tmp[k + 1] = p_tmp[k] + so2 * v0;
        H_tmp[k] = 0.5 * m.alpha[k] * (p_tmp[k + 1] * p_tmp[k + 1] - p_tmp[k] * p_tmp[k]);
        const double dp = v0 * qb0, u = v1 + qb1, v = v2 + qb2;
        u_udp[k] = dp * u * u;
        v_vdp[k] = dp * v * v;
        u_vdp0[k] = u * v * dp;
        u_vdp1[k] = v * u * dp;
        tuu[k] = fabs(s_iv[k][3][qd]) + eps1;
        tvv[k] = fabs(s_iv[k][4][qd]) + eps1;
      }
#pragma unroll
      for (int k = 0; k <= MAXL; k++) gz0[k] = gz1[k] = 0.0;
      if constexpr (GZS) {
#pragma unroll
        for (int k = 0; k <= MAXL; k++)
          if (k <= L) {
            gz0[k] = s_gz[0][k][qd];
            gz1[k] = s_gz[1][k][qd];
          }
      } else {
      double pa[NGL], da[NGL], pb[NGL], db[NGL];
#pragma unroll
      for (int n = 0; n < NGL; n++) {
        pa[n] = s_psiq[n * NQ + iq];
        da[n] = s_dpsiq[n * NQ + iq];
        pb[n] = s_psiq[n * NQ + jq];
        db[n] = s_dpsiq[n * NQ + jq];
      }
      const double e0 = s_qm[0][qd], e1 = s_qm[1][qd], e2 = s_qm[2][qd], e3 = s_qm[3][qd];
#pragma unroll 1
      for (int mm = 0; mm < NGL; mm++)
#pragma unroll
        for (int n = 0; n < NGL; n++) {
          const int ip = mm * NGL + n;
          const double h_e = da[n] * pb[mm], h_n = pa[n] * db[mm];
          const double dx = h_e * e0 + h_n * e2;
          const double dy = h_e * e1 + h_n * e3;
#pragma unroll
          for (int k = 0; k <= MAXL; k++) {
            if (k > L) break;
            gz0[k] = gz0[k] + dx * s_z[k][ip];
            gz1[k] = gz1[k] + dy * s_z[k][ip];
          }
        }
      }
      double su = 0, suv = 0, sv = 0, stu = 0, stv = 0, sH = 0;
#pragma unroll
      for (int k = 0; k < MAXL; k++)
        if (k < L) su = su + u_udp[k];
#pragma unroll
      for (int k = 0; k < MAXL; k++)
        if (k < L) suv = suv + u_vdp0[k];
#pragma unroll
      for (int k = 0; k < MAXL; k++)
        if (k < L) sv = sv + v_vdp[k];
      const double uu_def = r_qa[4] - su;
      const double uv_def = r_qa[5] - suv;
      const double vv_def = r_qa[6] - sv;
#pragma unroll
      for (int k = 0; k < MAXL; k++)
        if (k < L) stu = stu + tuu[k];
#pragma unroll
      for (int k = 0; k < MAXL; k++)
        if (k < L) stv = stv + tvv[k];
#pragma unroll
      for (int k = 0; k < MAXL; k++)
        if (k < L) sH = sH + H_tmp[k];
      const double oosu = 1.0 / stu, oosv = 1.0 / stv;
      double weight = 1.0;
      if (sH > 0.0) weight = r_qa[7] / sH;
      const double tw1 = r_qs[0], tw2 = r_qs[1], tb1 = r_qa[8], tb2 = r_qa[9], pb_ = r_qs[2];
      double ppt0 = 0.0;
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        // QUIRK (mod_create_rhs_mlswe.F90:382): qp(k) = the LAST layer's (dp',u',v') indexed by k
        const double ppt1 = ppt0 + ppl[k];
        double wgt = tuu[k] * oosu;
        const double uu = u_udp[k] + wgt * uu_def;
        const double uv0 = u_vdp0[k] + wgt * uv_def;
        wgt = tvv[k] * oosv;
        const double uv1 = u_vdp1[k] + wgt * uv_def;
        const double vv = v_vdp[k] + wgt * vv_def;
        const double Hq = H_tmp[k] * weight;
        const double temp1 = (dmin(ppt1, Pstress) - dmin(ppt0, Pstress)) / Pstress;
        double tempbot = dmin(Pbstress, pb_ - ppt1) - dmin(Pbstress, pb_ - ppt0);
        tempbot = tempbot / Pbstress;
        const double sx = g * (temp1 * tw1 - tempbot * tb1 + p_tmp[k] * gz0[k] - p_tmp[k + 1] * gz0[k + 1]);
        const double sy = g * (temp1 * tw2 - tempbot * tb2 + p_tmp[k] * gz1[k] - p_tmp[k + 1] * gz1[k + 1]);
        s_G[k][0][qd] = sx;
        s_G[k][1][qd] = Hq + uu;
        s_G[k][2][qd] = uv0;
        s_G[k][3][qd] = sy;
        s_G[k][4][qd] = uv1;
        s_G[k][5][qd] = Hq + vv;
        ppt0 = ppt1;
      }
    } else {
      const int t = w - Q, k = t / (2 * P), c = (t / P) % 2, p = t % P, i = p % NGL, j = p / NGL;
      double acc = 0.0;
#pragma unroll
      for (int r = 0; r < 2 * NGL - 1; r++) {
        const bool mid = (r >= j) && (r < j + NGL);
        const int jj = mid ? j : (r < j ? r : r - NGL + 1);
        const int ii = mid ? r - j : i;
        const int sn = jj * NGL + ii;
        // HE_DF(i,j,ii,jj) = dpsi(i,ii) [jj==j], HN_DF(i,j,ii,jj) = dpsi(j,jj) [ii==i]
        const double he = s_dpsi[i * NGL + ii], hn = s_dpsi[j * NGL + jj];
        const double ex_ = he * s_nm[0][sn], ey_ = he * s_nm[1][sn];
        const double nx_ = hn * s_nm[2][sn], ny_ = hn * s_nm[3][sn];
        const bool both = mid && ii == i;
        const double dx = both ? ex_ + nx_ : (mid ? ex_ : nx_);
        const double dy = both ? ey_ + ny_ : (mid ? ey_ : ny_);
        acc = acc - s_nm[4][sn] * (dx * s_qq[k][2 * c][sn] + dy * s_qq[k][2 * c + 1][sn]);
      }
      int r0, r1;
      node_faces<NGL>(s_map, p, r0, r1);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int r = h ? r1 : r0;
        if (r < 0) continue;
        const double v = s_fl[k][c][r];
        acc = s_side[r / NGL] == 0 ? acc + v : acc - v;
      }
      s_r[k][2 + c][p] = acc;
    }
  }
  __syncthreads();
  BCL_MARK(2, 3)

  // ---- 3: weak forms, one thread per (layer, output, node), reference accumulation order
  //      (create_rhs_dynamics_volume_layers :401-456, then Apply_layers_fluxes :778-817)
  if constexpr (QSUM) {
    // thread t: node p, chain ko = (k, o) -- its terms evaluated in parallel per node and quad
    // point (ordered_node_sums), then the face lifts
    constexpr int CPN = 2 * MAXL;
    const int t = tid, p = t / CPN, ko = t % CPN, k = ko >> 1, o = ko & 1;
    double acc = ordered_node_sums<NQ, P, CPN, BS, QS>(s_ivtb, tid, 2 * L, [&](int pp, int qd, double *dst, int st) {
      const int i = pp % NGL, j = pp / NGL, iq = qd % NQ, jq = qd / NQ;
      const double pi = s_psiq[i * NQ + iq], dpi = s_dpsiq[i * NQ + iq];
      const double pj = s_psiq[j * NQ + jq], dpj = s_dpsiq[j * NQ + jq];
      const double hi = pi * pj, h_e = dpi * pj, h_n = pi * dpj;
      const double dhdx = h_e * s_qm[0][qd] + h_n * s_qm[2][qd];
      const double dhdy = h_e * s_qm[1][qd] + h_n * s_qm[3][qd];
      const double w = s_qm[4][qd];
#pragma unroll
      for (int kk = 0; kk < MAXL; kk++) {
        if (kk >= L) break;
#pragma unroll
        for (int oo = 0; oo < 2; oo++)
          dst[(2 * kk + oo) * st] =
              w * (hi * s_G[kk][3 * oo][qd] + dhdx * s_G[kk][3 * oo + 1][qd] + dhdy * s_G[kk][3 * oo + 2][qd]);
      }
    });
    if (t < P * CPN && ko < 2 * L) {
      int r0, r1;
      node_faces<NGL>(s_map, p, r0, r1);
      acc = face_terms_at<NGL, NQ>(s_psiq, s_side, s_fw, s_fm[k][o], r0, r1, acc);
      s_r[k][o][p] = acc;
    }
  } else
  for (int t = tid; t < L * 2 * P; t += BS) {
    const int k = t / (2 * P), o = (t / P) % 2, p = t % P, i = p % NGL, j = p / NGL;
    const double *G0 = s_G[k][3 * o], *G1 = s_G[k][3 * o + 1], *G2 = s_G[k][3 * o + 2];
    double acc = 0.0;
#pragma unroll 1
    for (int jq = 0; jq < NQ; jq++) {
      const double pj = s_psiq[j * NQ + jq], dpj = s_dpsiq[j * NQ + jq];
#pragma unroll
      for (int iq = 0; iq < NQ; iq++) {
        const int qd = jq * NQ + iq;
        const double pi = s_psiq[i * NQ + iq], dpi = s_dpsiq[i * NQ + iq];
        const double hi = pi * pj, h_e = dpi * pj, h_n = pi * dpj;
        const double dhdx = h_e * s_qm[0][qd] + h_n * s_qm[2][qd];
        const double dhdy = h_e * s_qm[1][qd] + h_n * s_qm[3][qd];
        // o = 0: w*(hi*G0 + dhdx*G1 + G2*dhdy); o = 1: w*(hi*G3 + G4*dhdx + dhdy*G5)
        const double term = s_qm[4][qd] * (hi * G0[qd] + dhdx * G1[qd] + dhdy * G2[qd]);
        acc = acc + term;
      }
    }
    int r0, r1;
    node_faces<NGL>(s_map, p, r0, r1);
    acc = face_terms_at<NGL, NQ>(s_psiq, s_side, s_fw, s_fm[k][o], r0, r1, acc);
    s_r[k][o][p] = acc;
  }
  __syncthreads();
  BCL_MARK(2, 4)

  // ---- 4: per node: rhs_mom and q_df_temp = q + dt*rhs_mom (mod_splitting.F90:134-137 /
  //      :242-245), kept in s_r[k][0..1].  With ad_mlswe > 0 also the shear-stress input
  //      q_df3 = the Coriolis-rotated q_df_temp (:141-150 / :249-257) made consistent with
  //      u_bar by velocity_df (mod_layer_terms.F90:139-196), into s_qq[k][0..2] (dead since
  //      phase 2); momentum() (mode 1) passes its never-assigned `uv` instead (mod_splitting.
  //      F90:119,158): zeros unless shear_corr selects q_df3 (hnumo_params.shear_corrector)
  const bool shear = m.ad > 0.0, shear_zero = mode == 1 && m.shear_corr != 1;
  for (int p = tid; p < P; p += BS) {
    const size_t I = (size_t)e * P + p;
    const double mi = s_p4[P4_MI][p];
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      // (method_visc == 1: the layer's Laplacian comes from lapq_apply_kernel, [L][2][npoin])
      const double l0 = lapx ? lapx[((size_t)k * 2) * npoin + I] : s_r[k][2][p];
      const double l1 = lapx ? lapx[((size_t)k * 2 + 1) * npoin + I] : s_r[k][3][p];
      const double v0 = m.visc * mi * l0, v1 = m.visc * mi * l1;
      const double rm0 = mi * s_r[k][0][p] + v0;
      const double rm1 = mi * s_r[k][1][p] + v1;
      s_r[k][0][p] = s_qm2[k][0][p] + m.dt * rm0;
      s_r[k][1][p] = s_qm2[k][1][p] + m.dt * rm1;
    }
    if (shear) {
      const double f2 = m.nstat[NS_F2 * (size_t)npoin + I], ab = m.nstat[NS_A * (size_t)npoin + I],
                   bb = m.nstat[NS_B * (size_t)npoin + I];
      const double b1 = qb[I * 4], b3 = qb[I * 4 + 2], b4 = qb[I * 4 + 3];
      double h[MAXL], uv[MAXL][2], ub = 0.0, vb = 0.0;
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        h[k] = q[((size_t)k * npoin + I) * 3];
        const double q2 = s_qm2[k][0][p], q3 = s_qm2[k][1][p];
        const double tu = s_r[k][0][p] + f2 * q3, tv = s_r[k][1][p] - f2 * q2;
        uv[k][0] = (ab * tu + bb * tv) / h[k];
        uv[k][1] = (-bb * tu + ab * tv) / h[k];
      }
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        ub = ub + uv[k][0] * h[k];
        vb = vb + uv[k][1] * h[k];
      }
      if (b1 > 0.0) {
        ub = ub / b1;
        vb = vb / b1;
#pragma unroll
        for (int k = 0; k < MAXL; k++) {
          if (k >= L) break;
          uv[k][0] = uv[k][0] - ub + b3 / b1;
          uv[k][1] = uv[k][1] - vb + b4 / b1;
        }
      } else {
#pragma unroll
        for (int k = 0; k < MAXL; k++) uv[k][0] = uv[k][1] = 0.0;
      }
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        s_qq[k][0][p] = shear_zero ? 0.0 : h[k];
        s_qq[k][1][p] = shear_zero ? 0.0 : uv[k][0] * h[k];
        s_qq[k][2][p] = shear_zero ? 0.0 : uv[k][1] * h[k];
      }
    }
  }
  if (shear) {
    __syncthreads();
    // ---- 4b: rhs_layer_shear_stress (mod_create_rhs_mlswe.F90:181-251), one thread per quad
    //      point: dp, u*dp, v*dp of every layer (reference order), the tridiagonal system over
    //      the layers (sub-diagonal -coeff, super-diagonal -coeff1, as written), the interface
    //      stresses; g*(tau_k - tau_{k+1}) into s_G[k][0..1] (dead since phase 3).
    //      tau(nlayers+1) is never assigned there (:160,:246-251): zero, as under the reference
    //      build's -finit-real=zero
    const double al1 = m.alpha[0];
    for (int qd = tid; qd < Q; qd += BS) {
      const int iq = qd % NQ, jq = qd / NQ;
      double pa[NGL], pb[NGL], dp[MAXL], udp[MAXL], vdp[MAXL];
#pragma unroll
      for (int n = 0; n < NGL; n++) {
        pa[n] = s_psiq[n * NQ + iq];
        pb[n] = s_psiq[n * NQ + jq];
      }
#pragma unroll
      for (int k = 0; k < MAXL; k++) dp[k] = udp[k] = vdp[k] = 0.0;
#pragma unroll 1
      for (int mm = 0; mm < NGL; mm++)
#pragma unroll
        for (int n = 0; n < NGL; n++) {
          const int ip = mm * NGL + n;
          const double hi = pa[n] * pb[mm];
#pragma unroll
          for (int k = 0; k < MAXL; k++) {
            if (k >= L) break;
            dp[k] = dp[k] + hi * s_qq[k][0][ip];
            udp[k] = udp[k] + hi * s_qq[k][1][ip];
            vdp[k] = vdp[k] + hi * s_qq[k][2][ip];
          }
        }
      // Fortran MAX as gfortran evaluates it: the second argument if larger or the first is NaN
      double coeff = sqrt(0.5 * m.qstat[QS_COR * (size_t)npq + (size_t)e * Q + qd] * m.ad) / al1;
      const double cz = m.ad / (al1 * m.max_shear_dz);
      if (cz > coeff || isnan(coeff)) coeff = cz;
      const double coeff1 = g * m.dt * coeff;
      double bd[MAXL], r0[MAXL], r1[MAXL], tu[MAXL + 1], tv[MAXL + 1];
#pragma unroll
      for (int k = 0; k <= MAXL; k++) tu[k] = tv[k] = 0.0;
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        bd[k] = (k == 0 || k == L - 1) ? dp[k] + coeff1 : dp[k] + 2.0 * coeff1;
        r0[k] = udp[k] / dp[k];
        r1[k] = vdp[k] / dp[k];
      }
#pragma unroll
      for (int k = 1; k < MAXL; k++) {
        if (k >= L) break;
        const double mult = -coeff / bd[k - 1];
        bd[k] = bd[k] - mult * (-coeff1);
        r0[k] = r0[k] - mult * r0[k - 1];
        r1[k] = r1[k] - mult * r1[k - 1];
      }
#pragma unroll
      for (int k = 0; k < MAXL; k++)
        if (k == L - 1) {
          r0[k] = r0[k] / bd[k];
          r1[k] = r1[k] / bd[k];
        }
#pragma unroll
      for (int k = MAXL - 2; k >= 0; k--) {
        if (k >= L - 1) continue;
        r0[k] = (r0[k] - (-coeff1) * r0[k + 1]) / bd[k];
        r1[k] = (r1[k] - (-coeff1) * r1[k + 1]) / bd[k];
      }
#pragma unroll
      for (int k = 1; k < MAXL; k++) {
        if (k >= L) break;
        tu[k] = coeff * (r0[k - 1] - r0[k]);
        tv[k] = coeff * (r1[k - 1] - r1[k]);
      }
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        s_G[k][0][qd] = g * (tu[k] - tu[k + 1]);
        s_G[k][1][qd] = g * (tv[k] - tv[k + 1]);
      }
    }
    __syncthreads();
    // ---- 4c: rhs_stress(c,p,k) = sum over the quad points in order of wq*hi*tau_q (:253-269);
    //      q_df_temp += dt*(massinv*rhs_stress) (mod_splitting.F90:160-163 / :267-270)
    for (int t = tid; t < L * 2 * P; t += BS) {
      const int k = t / (2 * P), c = (t / P) % 2, p = t % P, i = p % NGL, j = p / NGL;
      const double *T = s_G[k][c];
      double acc = 0.0;
#pragma unroll 1
      for (int jq = 0; jq < NQ; jq++) {
        const double pj = s_psiq[j * NQ + jq];
#pragma unroll
        for (int iq = 0; iq < NQ; iq++) {
          const int qd = jq * NQ + iq;
          acc = acc + s_qm[4][qd] * (s_psiq[i * NQ + iq] * pj) * T[qd];
        }
      }
      const double mi = m.nstat[NS_MINV * (size_t)npoin + (size_t)e * P + p];
      s_r[k][c][p] = s_r[k][c][p] + m.dt * (mi * acc);
    }
    __syncthreads();
  }

  // ---- 4d: implicit Coriolis (mod_splitting.F90:166-173 / :273-280), layer_mom_boundary_df
  //      on the element's wall faces in face order (mod_layer_terms.F90:529-584),
  //      evaluate_bcl / evaluate_bcl_v1 with extract_velocity (:198-320)
  for (int p = tid; p < P; p += BS) {
    const size_t I = (size_t)e * P + p;
    const double f2 = s_p4[P4_F2][p], ab = s_p4[P4_A][p], bb = s_p4[P4_B][p];
    const double b1 = s_p4[P4_QB][p], b3 = s_p4[P4_QB + 2][p], b4 = s_p4[P4_QB + 3][p];
    double nw[MAXL][3];
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      const double q2 = s_qm2[k][0][p], q3 = s_qm2[k][1][p];
      const double tu = s_r[k][0][p] + f2 * q3, tv = s_r[k][1][p] - f2 * q2;
      nw[k][1] = ab * tu + bb * tv;
      nw[k][2] = -bb * tu + ab * tv;
      nw[k][0] = s_p4[P4_H + k][p];
    }
    for (int lf = 0; lf < 4; lf++) {
      const int er = s_bc[lf];
      if (er != -4 && er != -2) continue;
      for (int n = 0; n < NGL; n++) {
        if (s_map[lf * NGL + n] != p) continue;
        const size_t fn = (size_t)s_face[lf] * NGL + n, FN = (size_t)F * NGL;
        const double nx = m.fnstat[FN_NX * FN + fn], ny = m.fnstat[FN_NY * FN + fn];
#pragma unroll
        for (int k = 0; k < MAXL; k++) {
          if (k >= L) break;
          if (er == -4) {
            const double u = nw[k][1], v = nw[k][2];
            const double up = u * nx + v * ny;
            nw[k][1] = u - up * nx;
            nw[k][2] = v - up * ny;
          } else {
            nw[k][1] = 0.0;
            nw[k][2] = 0.0;
          }
        }
      }
    }
    double uv[MAXL][2], h[MAXL];
#pragma unroll
    for (int pass = 0; pass < 2; pass++) {
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        h[k] = nw[k][0];
        uv[k][0] = nw[k][1] / h[k];
        uv[k][1] = nw[k][2] / h[k];
      }
      double ub = 0.0, vb = 0.0;
#pragma unroll
      for (int k = 0; k < MAXL; k++) {
        if (k >= L) break;
        ub = ub + uv[k][0] * h[k];
        vb = vb + uv[k][1] * h[k];
      }
      if (b1 > 0.0) {
        ub = ub / b1;
        vb = vb / b1;
#pragma unroll
        for (int k = 0; k < MAXL; k++) {
          if (k >= L) break;
          uv[k][0] = uv[k][0] - ub + b3 / b1;
          uv[k][1] = uv[k][1] - vb + b4 / b1;
        }
      } else {
#pragma unroll
        for (int k = 0; k < MAXL; k++) uv[k][0] = uv[k][1] = 0.0;
      }
      if (pass == 0) {
#pragma unroll
        for (int k = 0; k < MAXL; k++) {
          if (k >= L) break;
          nw[k][1] = uv[k][0] * h[k];
          nw[k][2] = uv[k][1] * h[k];
        }
      }
    }
    double ope = 0.0;
    if (mode == 0) {
#pragma unroll
      for (int k = 0; k < MAXL; k++)
        if (k < L) ope = ope + h[k];
      ope = ope / s_p4[P4_PB][p];
    }
    double ov[MAXL][3];
#pragma unroll
    for (int k = 0; k < MAXL; k++) {
      if (k >= L) break;
      double *qq = q + ((size_t)k * npoin + I) * 3;
      qq[1] = nw[k][1];
      qq[2] = nw[k][2];
      double *o = qp_out + ((size_t)k * npoin + I) * 3;
      ov[k][0] = mode == 0 ? h[k] / ope : s_p4[P4_D + k][p];
      ov[k][1] = uv[k][0] - b3 / b1;
      ov[k][2] = uv[k][1] - b4 / b1;
      o[0] = ov[k][0];
      o[1] = ov[k][1];
      o[2] = ov[k][2];
    }
    if (qf) {
      int r0, r1;
      node_faces<NGL>(s_map, p, r0, r1);
      extract_node_faces<NGL>(m, qf, s_face, s_side, s_bc, r0, r1, ov, 0);
    }
    if (mode == 1) {
      const double b2 = s_p4[P4_QB + 1][p];
      if (!(isfinite(b1) && isfinite(b2) && isfinite(b3) && isfinite(b4))) atomicOr(flag, 2);
    }
  }
  BCL_MARK(2, 5) BCL_WALL(2, 7)
}

#define HNUMO_INSTANTIATE_BCL(NGL, NQ)                                                                              \
  template __global__ void extract_face_kernel<NGL>(DevMesh, const double *, double *, int);                      \
  template __global__ void bcl_coeffs_elem_kernel<NGL, NQ>(DevMesh, double *, const double *, double *, double *,    \
                                                           double *, double *, double *, const double *,           \
                                                           const double *, double *, double *, double *, double *, \
                                                           double *);                                              \
  template __global__ void bcl_coeffs_face_kernel<NGL, NQ>(DevMesh, double *, const double *, const double *,        \
                                                           const double *, double *, double *, double *, double *);

}  // namespace hnumo
