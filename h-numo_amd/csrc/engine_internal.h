// engine_internal.h -- device-side data layout of the MI355X MLSWE engine.
//
// Layout in HBM (all fp64 unless noted; E elements, P = NGL^2 nodes, Q = NQ^2 quad points,
// F faces, L layers; node index I = e*P + j*NGL + i, quad index Iq = e*Q + jq*NQ + iq):
//
//   state            qb(4,npoin), q(3,npoin,L), qprime(3,npoin,L)   -- reference layouts
//   quad statics     SoA [field][npoin_q]  (coalesced: lane = quad point of one element)
//   quad accums      SoA [12][npoin_q]     (read-modify-written once per barotropic stage)
//   nodal statics    SoA [field][npoin]
//   face statics     [field][F*NQ] or [field][F*NGL]  (lane = face quad point / face node)
//   face accums      SoA [16][F*NQ]        (owned by the face's left element)
//   element->face    efaces[e][4], eside[e][4], ebc[e][4], efmap[e][4][NGL],
//                    enbr_node[e][4][NGL], enbr_e[e][4], enbr_lf[e][4]
//   face traces      trace[e][4][8][NGL]   (qb(4) and grad(u_bar)(4) of the neighbour at each
//                    face node, written by the neighbour's stage into this element's slot;
//                    processor-face halo: + [NS] send slots + [NS] receive slots, see DevMesh)
//
// Element-major copies for the barotropic stage kernel (one contiguous record per element,
// so a stage loads everything it needs with one round of async global->LDS copies):
//   erec   int  [E][ERS]              faces, side, bc, nbr elem, nbr local face, keeps-averages flag, face->node map,
//                                     node->(lf*NGL+n) of the <=2 faces through each node
//   qstatE      [E][QE_N][Q] (+1 pad)  W, e_x, e_y, n_x, n_y, coriolis, tau_wind(2), grad_zbot(2), 1/pb
//   nstatE      [E][NE_N][P]          e_x, e_y, n_x, n_y, w, 1/pbprime, massinv, pbprime
//   efstat      [E][4][FBLK]          face statics at face quad points (EF_*) and face nodes (EFN_*)
//   ecoef       [E][4Q + 5P] (even)    per-sub-cycle Q_uu/uv/vv_dp, H_bcl | pbprime_visc, btp_dpp_graduv
//   efcoef      [E][4][4NQ + 10NGL]   per-sub-cycle face Q_*_edge, H_bcl_edge | btp_graduv_dpp_face
//   accumulators (element-major)      qacc [E][QA_N][Q], nacc [E][NA_N][P],
//                                     facc [E][4][FA_N][NQ], gfacc [E][4][8][NGL]
//                                     (face slots e*4+lf of the face's left element, or of its
//                                     right element when the left one is a ghost: fslotA)
// HNUMO_DIAG=1 (HNUMO_EXTRA_FLAGS=-DHNUMO_DIAG=1 csrc/build.sh): the diagnostics build -- phase
// switches and phase clocks of the stage kernels (HNUMO_STAGE_DBG, HNUMO_STAGE_PROF), the two-stream
// schedule's timing switches (HNUMO_SCHED_DBG), the element kernels' phase clocks (HNUMO_BCL_PROF).
// Timing experiments only: most switches break the physics.  The product build reads none of them.
#ifndef HNUMO_DIAG
#define HNUMO_DIAG 0
#endif
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hnumo {

constexpr int MAXNGL = 8;
constexpr int MAXNQ = 15;
constexpr int MAXL = 3;

// quad accumulators (mod_variables): index into the [12][npoin_q] block
enum QAcc { QA_H = 0, QA_QU, QA_QV, QA_QUV, QA_TBU, QA_TBV, QA_OPE, QA_OPE2, QA_MFX, QA_MFY, QA_UB, QA_VB, QA_N };
// face accumulators: [16][F*NQ]
enum FAcc {
  FA_MFX = 0, FA_MFY, FA_H, FA_QUU, FA_QUV, FA_QVU, FA_QVV, FA_OPEL, FA_OPER, FA_OPE2L, FA_OPE2R, FA_OPEE2,
  FA_UL, FA_UR, FA_VL, FA_VR, FA_N
};
// nodal accumulators: [7][npoin] (ope2_ave_df, uvb_ave_df(2), graduvb_ave(4))
enum NAcc { NA_OPE2 = 0, NA_UB, NA_VB, NA_G1, NA_G2, NA_G3, NA_G4, NA_N };
// quad statics: [QS_N][npoin_q]
enum QStat { QS_W = 0, QS_COR, QS_TW1, QS_TW2, QS_GZ1, QS_GZ2, QS_OOP, QS_EX, QS_EY, QS_NX, QS_NY, QS_PB, QS_N };
// per-sub-cycle baroclinic coefficients at quad points: [4][npoin_q]
enum QCoef { QC_HBCL = 0, QC_QUU, QC_QUV, QC_QVV, QC_N };
// nodal statics: [NS_N][npoin]
enum NStat { NS_PB = 0, NS_OOP, NS_MINV, NS_W, NS_EX, NS_EY, NS_NX, NS_NY, NS_ZB, NS_F2, NS_A, NS_B, NS_N };
// per-sub-cycle nodal coefficients: pbprime_visc, btp_dpp_graduv(4): [5][npoin]
enum NCoef { NC_PV = 0, NC_D1, NC_D2, NC_D3, NC_D4, NC_N };
// face statics at face quad points: [FS_N][F*NQ]
enum FStat {
  FS_NX = 0, FS_NY, FS_W, FS_CL, FS_CR, FS_CLR, FS_CML, FS_CMR, FS_CMLR, FS_OOPE, FS_PBL, FS_PBR, FS_ZBL, FS_ZBR, FS_N
};
// per-sub-cycle face coefficients at face quad points: [4][F*NQ]
enum FCoef { FC_QUU = 0, FC_QUV, FC_QVV, FC_HBCL, FC_N };
// face statics at face nodes: [FN_N][F*NGL]
enum FNStat { FN_NX = 0, FN_NY, FN_W, FN_PBL, FN_PBR, FN_N };

// element-major quad statics order (qstatE): the first QE_KEEP rows live for the whole stage
enum QStatE { QE_W = 0, QE_EX, QE_EY, QE_NX, QE_NY, QE_COR, QE_TW1, QE_TW2, QE_GZ1, QE_GZ2, QE_OOP, QE_N };
constexpr int QE_KEEP = 5;
// Positions in the first QE_KEEP rows of an element's qstatE record (Q quad points): W, then the
// metric pairs interleaved per quad point -- (e_x, n_x), (e_y, n_y) adjacent, read together with
// one ds_read2 where a row layout put them 2Q apart -- the later rows field-major (c*Q + q)
__host__ __device__ constexpr int qe_pos(int c, int q, int Q) {
  return c == QE_W ? q
                   : c == QE_EX ? Q + 2 * q
                   : c == QE_NX ? Q + 2 * q + 1
                   : c == QE_EY ? 3 * Q + 2 * q
                   : c == QE_NY ? 3 * Q + 2 * q + 1 : c * Q + q;
}
// element-major nodal statics order (nstatE); the first NE_LDS rows are the ones the stage
// kernel's slim LDS arena (StageCfg::SLIM) stages -- its E1 reads massinv and pbprime into
// registers from global memory
enum NStatE { NE_EX = 0, NE_EY, NE_NX, NE_NY, NE_W, NE_OOP, NE_MINV, NE_PB, NE_N };
constexpr int NE_LDS = 6;
// element-side face statics block: FS fields at NQ face quad points, then FN fields at NGL nodes
// (EF_PBLQ/EF_PBRQ: pbprime_df_face interpolated to the face quad points, sum_n psiq(n,iq) *
//  pbprime_df_face(s,n,f) in the reference's order -- static, so computed once on the host)
enum EFStat { EF_NX = 0, EF_NY, EF_W, EF_CL, EF_CR, EF_CLR, EF_CML, EF_CMR, EF_CMLR, EF_OOPE, EF_PBLQ, EF_PBRQ, EF_N };
enum EFNStat { EFN_NX = 0, EFN_NY, EFN_W, EFN_PBL, EFN_PBR, EFN_N };
// per-element int record (erec) offsets
#define EREC_FACE 0
#define EREC_SIDE 4
#define EREC_BC 8
#define EREC_NBE 12
#define EREC_NBLF 16
#define EREC_ACC 20   /* 1: this element keeps the face time averages of local face lf */
#define EREC_MAP 24
#define EREC_PF(ngl) (24 + 4 * (ngl))
// (records padded to 16 bytes: the stage kernel copies them into LDS with 16-byte LDS-DMA)
#define EREC_SIZE(ngl) ((24 + 4 * (ngl) + 2 * (ngl) * (ngl) + 3) & ~3)
// per-element strides of the element-major double records, even (16-byte aligned records)
__host__ __device__ constexpr int qe_stride(int Q) { return (QE_N * Q + 1) & ~1; }
__host__ __device__ constexpr int eco_stride(int Q, int P) { return (4 * Q + 5 * P + 1) & ~1; }

// element-major accumulator indices
#define QACC_I(k, e, q) ((((size_t)(e)) * QA_N + (k)) * Q + (q))
#define NACC_I(k, e, p) ((((size_t)(e)) * NA_N + (k)) * P + (p))
#define FACC_I(k, slot, iq) ((((size_t)(slot)) * FA_N + (k)) * NQ + (iq))
#define GFACC_I(c, slot, n) ((((size_t)(slot)) * 8 + (c)) * NGL + (n))
// layer momentum face terms / LDG face fluxes per element-side slot: [slot][L][2][N] (N = NQ or
// NGL; needs L in scope)
#define MSLOT(slot, k, o, i, N) (((((size_t)(slot)) * L + (k)) * 2 + (o)) * (N) + (i))
// the efstat block of one element side (StageCfg::FBLK)
#define EFBLK(NGL, NQ) (EF_N * (NQ) + EFN_N * (NGL))

struct DevMesh {
  int nelem, npoin, npoin_q, nface, ngl, nq, L;
  const int *efaces, *eside, *ebc, *efmap, *enbr_node, *enbr_e, *enbr_lf;
  const int *fnodeL, *fnodeR;     // [F][NGL] global node of face node n, left/right (-1 if none)
  const int *fel, *fer;           // [F] face(7)-1, face(8) (raw: >0 element+1, <=0 code)
  const int *fslotL, *fslotR;     // [F] element-side slot e*4+lf of the face's left / right element (-1)
  const int *fslotA;              // [F] slot whose face accumulators hold the face's averages
  const int *erec;                // [E][EREC_SIZE]
  const double *qstatE, *nstatE, *efstat;
  const double *basis;            // psiq[NGL*NQ] dpsiq[NGL*NQ] dpsi[NGL*NGL]
  const double *basis_pd;         // the stage kernel's copy: (psiq, dpsiq)[NGL*NQ] interleaved, dpsi[NGL*NGL]
  const double *qstat;            // [QS_N][npoin_q]
  const double *nstat;            // [NS_N][npoin]
  const double *fstat;            // [FS_N][F*NQ]
  const double *fnstat;           // [FN_N][F*NGL]
  const double *alpha;            // [L]
  double gravity, cd, visc, dt, dt_btp;
  int botfr;
  double ad, max_shear_dz;        // ad_mlswe, max_shear_dz (implicit vertical shear stress)
  int shear_corr;                 // hnumo_params.shear_corrector
  // processor-face halo (NULL on a single rank / the ghost-element halo): per element and local
  // face, the trace-buffer slot its neighbour trace arrives in -- e*4+lf, or for a processor
  // face the receive slot 4E+NS+s of shared face s (the trace buffers are [4E + 2NS][8][NGL]:
  // element slots, then the send slots the stage writes processor-face traces into, then the
  // receive slots the transport fills)
  const int *etsrc;
  // the run's device flag word (engine neg_flag): a persistent sub-cycle that found its
  // workgroups not co-resident sets RUN_ABORT and did no work; the kernels that write the step's
  // final state (mass_elem, cons_elem, mom_elem) then leave it untouched, so the host can redo
  // the step on per-stage launches.  steps_done counts the steps whose corrector completed.
  const int *runflag;
  unsigned *steps_done;
  // [nelem] block -> element of the element kernels (the persistent sub-cycle's placement, engine.hip
  // d_eperm; single-rank engines only; NULL: block b runs element b)
  const int *eperm;
};

// device flag word bits (engine.hip flag_error): 1 negative thickness, 2 non-finite state,
// 8 a persistent trace wait timed out, 16 a persistent launch was not co-resident (no work done)
constexpr int RUN_ABORT = 16;

}  // namespace hnumo
