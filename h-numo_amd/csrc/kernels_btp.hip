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
// products), and every ordered sum is accumulated sequentially by one thread.  With
// psi(i,k) the identity at the LGL nodes (checked on the host) the nodal derivative sums
// keep only their 2*NGL-1 nonzero terms, in order (the dropped terms add +-0).
//
// At one workgroup per element the kernel is latency-bound, so it is built around few
// memory round trips and short dependent chains:
//   A   every input of the element -- state, statics, coefficients, neighbour traces, old
//       accumulator values -- is one contiguous record per element (engine_internal.h),
//       copied global->LDS with async global_load_lds (one round trip, no VGPRs);
//   B   quad-point physics | nodal grad(u_bar) | face fluxes | LDG face fluxes, as
//       concurrent task ranges, LDS only; accumulators are written back here;
//   D0..D_NCH  weak-form terms T(v,p,q) computed in parallel per chunk of quad rows into
//       double-buffered LDS (overlaying the dead B-only inputs) while the previous chunk
//       is summed in quad order by one thread per (v,p); qq and the Laplacian ride along;
//   E   update + wall fix, then the new state and the face traces the neighbours need
//       next stage, written straight into the neighbours' trace slots.
#include "engine_internal.h"

// Design constants (the alternatives each replaced were measured and removed):
// OTF_MIN_NGL: from this NGL on the reference-order volume integral runs without term buffers
//   ("on the fly", OTF): one thread per (component v, node p) computes its terms T(v,p,q) itself, in
//   quad order, as it sums them -- same terms, same order, same bits as the chunked term buffers,
//   without their [3P][Q] LDS staging (46 KB at N=7), so the persistent N=7 arena fits 3 per CU;
// OTF_UNROLL: unroll of the on-the-fly sums' inner quad loop;
// PRIO_*: wave priorities by role (stage_body, s_setprio).  On a CU holding three elements the
//   elements' waves compete for the SIMDs; the waves whose chains a phase waits for -- the volume
//   sums, the last D phase, E -- issue ahead of the ones with slack (the term tasks, which finish
//   behind the sums anyway): PRIO_S for the summing waves in D, PRIO_E for the last D phase and E,
//   0 for the term tasks, PRIO_B elsewhere.
constexpr int OTF_MIN_NGL = 8;
#define OTF_UNROLL 3
constexpr int PRIO_B = 1, PRIO_S = 2, PRIO_E = 3;
// Diagnostics (HNUMO_DIAG builds only, engine_internal.h; timing experiments, most break the
// physics): StageArgs::dbg phase switches -- 1 the face lifts of the volume sums, 2 the Laplacian,
// 4 the volume sums, 16 the persistent trace waits, 32 the time averages (engine), 64 the term
// tasks, 128 A2 interpolations, 256 B quad-point tasks, 512 B face tasks, 1024 B nodal tasks,
// 2048 E2 trace stores, 4096 the A copies of the records (tools/dbg_sweep.py, tools/pmc_ablate.sh)
// -- and StageArgs::prof, the per-element phase clocks (tools/stage_profile.py)
#define DBG(bit) (HNUMO_DIAG && (a.dbg & (bit)))
#define DBGX(bit) DBG(bit)
#define PROF (HNUMO_DIAG && a.prof)
#define SETPRIO_IF(cond, hi, lo)        \
  do {                                  \
    if (cond)                           \
      __builtin_amdgcn_s_setprio(hi);   \
    else                                \
      __builtin_amdgcn_s_setprio(lo);   \
  } while (0)
namespace hnumo {

// A trace value with the tag of the stage it is for: one 16-byte write-through store makes
// both visible together (MI355X_MICROARCH.md: untorn 16-B sc1 granules), so a consumer
// polls the data itself, with no separate flag.
struct alignas(16) TraceGranule {
  double v;
  unsigned long long tag;
};
__device__ __forceinline__ void st_granule(TraceGranule *p, double v, unsigned long long tag) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  u4 x;
  const unsigned long long vb = __builtin_bit_cast(unsigned long long, v);
  x[0] = (unsigned)vb;
  x[1] = (unsigned)(vb >> 32);
  x[2] = (unsigned)tag;
  x[3] = (unsigned)(tag >> 32);
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
}
typedef unsigned granule_u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void ld_granule(const TraceGranule *p, double &v, unsigned long long &tag) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  u4 x;
  asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(x) : "v"(p) : "memory");
  v = __builtin_bit_cast(double, ((unsigned long long)x[1] << 32) | x[0]);
  tag = ((unsigned long long)x[3] << 32) | x[2];
}
// a time-average slot of this element: the first stage of a sub-cycle stores 0 + x (the reference's
// sum starts at zero: the same bits as adding x to a zeroed slot), the later stages add -- so no
// zeroing pass runs before the sub-cycle (StageArgs::accumulate == 2)
__device__ __forceinline__ void acc_put(double *p, double x, bool first) {
  if (first)
    *p = 0.0 + x;
  else
    atomicAdd(p, x);
}
struct StageArgs {
  DevMesh m;
  const double *qb_in, *qb0, *qb2, *qprime;  // qb(4,npoin); qprime(3,npoin,L)
  const double *ecoef;                       // [E][4Q + 5P]
  const double *efcoef;                      // [E][4][4NQ + 10NGL]
  const double *trace_in;                    // [E][4][8][NGL] neighbour qb(4) + grad(4) face traces
  double *trace_out;
  double *qacc, *facc, *nacc, *gfacc;        // element-major accumulators (engine_internal.h)
  double *qb_out;                            // stage result, qb(4,npoin)
  double *rhs_out;                           // rhs(3,npoin) in rhs-only mode
  double a1, a2, a3, dtt;
  int rhs_only, write_trace, accumulate;
  unsigned long long *prof;                  // optional [E][32] phase clocks (diagnostics)
  int dbg;                                   // diagnostics: bits skip D-phase parts (timing only)
  // persistent sub-cycle only: tagged trace granules, stage position in the RK scheme
  TraceGranule *gtr_in, *gtr_out;            // [E][4][8][NGL] {value, tag}
  unsigned long long tag_in, tag_out;        // stage tags (the launch epoch << 20 is or-ed in)
  int first_of_step, save_q2;                // ik == 0 (state -> qb0), K == 5 && ik == 2 (state -> qb2)
  int *err;                                  // bit 8: a granule wait timed out
  // method_visc == 1: the viscous Laplacian (without visc*massinv) from lapq_apply_kernel,
  // [2][npoin]; the fused nodal LDG then only keeps its ope2/uvb averages (graduvb_ave and
  // graduvb_face_ave are not accumulated on that branch, mod_laplacian_quad.F90:125-223)
  const double *lapq;
  // processor-face halo: the elements of this launch (block b runs element elist[b]; NULL:
  // element b) -- the boundary / interior split of the two-stream schedule
  const int *elist;
  // processor-face halo: 1 when no element of this launch has a processor face (the interior list):
  // its four trace slots are then its own, contiguous, and copied as one block
  int tcontig;
  // bottom-layer qprime at the quad points (pp, up, vp; mod_rhs_btp.F90:146-152), constant over a
  // sub-cycle: [E][3][Q] scratch (NULL: interpolated by every stage).  qpq_mode 1: this stage
  // interpolates and stores them (a sub-cycle's first stage), 2: loads them (the later stages)
  double *qpq;
  int qpq_mode;
  // persistent sub-cycle, slim arena (StageCfg::SLIM): the element's Shu-Osher states qb0, qb2
  // ([E][2][P][4], components 1..3) -- kept by the E1 lane of each node
  double *qsv;
  double n_inv;                              // 1/(N_btp*kstages): the averages' normalisation
  // persistent sub-cycle, stage 0: publish the input state's face traces (qb and grad(u_bar))
  // as this stage's granules before polling the neighbours' (no grad_trace launch before it)
  int self_trace;
};

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

// the four face-slot ids of an element (processor-face halo), one scalar load issued and waited
// for before the copies (a vector load's wait, vmcnt(0), would hold up every copy issued before it)
__device__ __forceinline__ int4 slot_ids4(const int *p) {
  typedef unsigned u4v __attribute__((ext_vector_type(4)));
  u4v t;
  asm volatile("s_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "s"(p));
  return make_int4((int)t.x, (int)t.y, (int)t.z, (int)t.w);
}

// Block-cooperative async copy of ndw dwords, global -> LDS, both contiguous.  One
// global_load_lds_dword per lane; chunks of 64 dwords rotate over the waves.
// G16: a 16-byte aligned source and destination move in whole 16-byte pieces first
// (global_load_lds_dwordx4, 1 KiB per wave-instruction: a quarter of the instructions, and of
// their address processing, of the dword form), the rest dword by dword
template <int BS, bool G16 = false>
__device__ __forceinline__ void glds_copy(const void *g, void *l, int ndw, int tid, int &rot) {
  constexpr int NW = BS / 64;
  const int wave = tid >> 6, lane = tid & 63;
  int d0 = 0;
  if (G16 && (((uintptr_t)g | (uintptr_t)l) & 15) == 0) {
    const int n4 = ndw >> 2;
    const int nch = (n4 + 63) >> 6;
    int c = (wave - rot) % NW;
    if (c < 0) c += NW;
    for (; c < nch; c += NW) {
      const int i = (c << 6) + lane;
      if (i < n4)
        __builtin_amdgcn_global_load_lds((glb_void_t *)((const uint4 *)g + i), (lds_void_t *)((uint4 *)l + (c << 6)),
                                         16, 0, 0);
    }
    rot = (rot + nch) % NW;
    d0 = n4 << 2;
  }
  const int nch = (ndw - d0 + 63) >> 6;
  int c = (wave - rot) % NW;
  if (c < 0) c += NW;
  for (; c < nch; c += NW) {
    const int i = d0 + (c << 6) + lane;
    if (i < ndw)
      __builtin_amdgcn_global_load_lds((glb_void_t *)((const unsigned *)g + i),
                                       (lds_void_t *)((unsigned *)l + d0 + (c << 6)), 4, 0, 0);
  }
  rot = (rot + nch) % NW;
}

// NBK: workgroups per CU the LDS arena is sized for (0: 3 for 256-thread blocks, the persistent
// sub-cycle's need at 625 elements).  The per-stage kernel on large meshes (every CU busy for
// many rounds) is also built for NBK = 4, 5: a smaller arena (fewer quad rows per term chunk,
// more D phases) buys more resident elements per CU to hide latency with.
template <int NGL, int NQ, bool SF = false, int NBK = 0>
struct StageCfg {
  static constexpr int P = NGL * NGL, Q = NQ * NQ;
  static constexpr int BS = (Q <= 25) ? 128 : 256;
  static constexpr int MINW = NBK ? NBK * BS / 256 : ((BS == 256) ? 3 : 4);  // waves/SIMD wanted
  static constexpr int NBLK_CU = (MINW * 4 * 64) / BS;      // resident blocks per CU wanted
  static constexpr int BUDGET = (163840 / NBLK_CU - 512) / 8;  // LDS doubles per block
  static constexpr int ERS = EREC_SIZE(NGL), ERSD = (ERS + 1) / 2;
  static constexpr int FBLK = EF_N * NQ + EFN_N * NGL;      // efstat block per element side
  static constexpr int EFC = 4 * NQ + 10 * NGL;             // efcoef block per element side
  static constexpr int ECO = eco_stride(Q, P);              // ecoef record per element (4Q + 5P, even)
  static constexpr int NB = 2 * NGL * NQ + NGL * NGL;       // psiq, dpsiq, dpsi (+ a zero slot)
  static_assert(Q <= BS, "one quad-point task per thread");
  static constexpr bool OTF = !SF && NGL >= OTF_MIN_NGL;
  // SLIM, SLATE, OPAIR and QPM name four aspects of the one OTF arena (all on together with OTF):
  // SLIM (OTF): an arena small enough for 3 workgroups per CU, so the persistent sub-cycle holds
  // all 625 elements of dg25 at N=7 at once.  The last wave (EW), idle beside the on-the-fly
  // volume sums of waves 0..2, runs the LDG volume fluxes, LDG face fluxes and the Laplacian
  // there and then E1; what only E1 and qq read -- the Shu-Osher states qb0/qb2, massinv,
  // pbprime, the nodal coefficients, the Laplacian -- lives in that wave's registers (loaded
  // from global memory while waves 0..2 sum) instead of LDS; the new state overwrites the
  // stage input in place; the bottom-layer qprime (A2 only) overlays the nodal gradients.
  static constexpr bool SLIM = OTF;
  // SLATE (SLIM): the face fluxes also run on the last wave in D, so the neighbour traces are
  // needed (persistent: polled) only there, behind the element's own interpolation, quad-point
  // physics and most of its volume sums -- the neighbours' stage-to-stage skew hides behind them;
  // the volume sums' face lifts follow a barrier
  static constexpr bool SLATE = SLIM;
  // OPAIR (SLATE): a node's component-1 and -2 volume sums on one thread (see otf_sum12) in the
  // per-stage kernel (dg25N7L3: 65.0 -> 57.0 us per launch); the persistent sub-cycle instead sums
  // all three components of a node on one thread (otf_sum012, TRIPLE)
  static constexpr bool OPAIR = SLATE;
  static constexpr int EW = BS / 64 - 1;
  // LEAN (the per-stage kernel's arenas for large meshes, NBK != 0): less fixed LDS so that more
  // workgroups fit a CU or more quad rows fit a term chunk -- E1 on the last wave (the volume-sum
  // lanes of D) with the Shu-Osher states qb0 / qb2 in its registers (loaded from global memory
  // during D) instead of LDS; the right-hand side and the Laplacian in the term buffer that is dead
  // in the last D phase, the new state in the other one (dead after D), the face-quad traces of
  // FPRE in term buffer 0 (A2 -> B; D0 writes it first)
  static constexpr bool LEAN = NBK != 0 && !SF && !OTF;
  // G16: 16-byte LDS-DMA for the element's records (glds_copy).  Not in the slim N=7 arena: there
  // it measured slower (dg25N7L3 persistent 50.2 -> 53.0 us per stage, while dg25L3 persistent
  // 13.0 -> 12.7 and C4 1.322 -> 1.296 ms; profiles/r03h)
  static constexpr bool G16 = !SLIM;
  static_assert(!SLIM || (P <= 64 && 3 * P <= EW * 64), "SLIM: one node per lane of the last wave");
  // LDS arena (doubles).  Persistent (A..E); the wall normals of the face nodes are copied
  // out of the face statics (which live in the B region) for E1:
  // (the regions LDS-DMA writes start on 16 bytes: ev; not the slim arena, which keeps the dword
  // copies -- see G16)
  static constexpr int ev(int x) { return SLIM ? x : (x + 1) & ~1; }
  // QPM (SLIM): the quad-point values by quad point, s_qv [4][Q][2] = pairs of (w, the 7 integrand factors) --
  // A2's interpolations in slots 0..3 and the bottom layer's in 4..6 until B overwrites them -- so the
  // on-the-fly sums read a quad point's 8 values as four ds_read_b128 from one address; w moves out of
  // s_qk, which keeps the metric pairs alone (16-byte aligned)
  static constexpr bool QPM = SLIM;
  static constexpr int QKR = QPM ? 4 : QE_KEEP;  // s_qk rows
  static constexpr int al2(int x) { return (x + 1) & ~1; }
  static constexpr int O_BASIS = 0, O_EREC = ev(O_BASIS + NB + 1), O_QB = ev(O_EREC + ERSD), O_Q0 = O_QB + 4 * P,
                       O_Q2 = O_Q0 + ((SLIM || LEAN) ? 0 : 4 * P),
                       O_QK = QPM ? al2(O_Q2) : O_Q2 + ((SLIM || LEAN) ? 0 : 4 * P),
                       O_NS = ev(O_QK + QKR * Q),
                       O_NC = ev(O_NS + (SLIM ? NE_LDS : NE_N) * P), O_UV = O_NC + (SLIM ? 0 : 5 * P), O_WN = O_UV + 2 * P;
  // working arrays: quad-point values (exact: the 7 integrand factors; SF: the 8 weighted
  // integrands F1,F2,G0..G2,H0..H2), B outputs, then a region written only after B that the
  // SF variant also uses for the interpolation partials Y [NYV][NGL][NQ] (A2 -> B)
  static constexpr int NQV = (SF || QPM) ? 8 : 7, NYV = 7;
  // (SLIM: no Laplacian / new-state buffers; the face-quad traces of FPRE, A2 -> B, share the W
  // region with qq and rhs, D -> E)
  static constexpr int O_QV = QPM ? al2(O_WN + 8 * NGL) : O_WN + 8 * NGL, O_GR = ev(O_QV + NQV * Q), O_FQ = O_GR + 4 * P, O_FL = O_FQ + 16 * NQ,
                       O_W = O_FL + 8 * NGL, O_QQ = O_W, O_RHS = O_QQ + 4 * P, O_LAP = O_RHS + (LEAN ? 0 : 3 * P),
                       O_QN = O_LAP + ((SLIM || LEAN) ? 0 : 2 * P), O_Y = O_W,
                       W_END0 = O_QN + ((SLIM || LEAN) ? 0 : 4 * P),
                       QN_END_W = W_END0 - O_W,
                       W_END = W_END0,
                       O_BIN = ev((SF && O_Y + NYV * NGL * NQ > W_END) ? O_Y + NYV * NGL * NQ : W_END);
  // B inputs: the bottom-layer qprime, face statics, neighbour traces, face coefficients,
  // reloaded every stage (the persistent kernel: re-fetched behind E1) and overlaid by term
  // buffer 1 once B and the LDG fluxes (D0) are done.  (SLIM: the qprime of A2 in the
  // nodal-gradient slot, written only from B on)
  static constexpr int B_QP = 0, B_EF = ev(B_QP + (SLIM ? 0 : 3 * P)), B_TR = B_EF + 4 * FBLK, B_EC = B_TR + 32 * NGL,
                       B_SIZE = B_EC + 4 * EFC, O_B = O_BIN;
  // exact: term chunks of RC quad rows, two buffers of [3P][QCP] (odd pitch against bank
  // conflicts), as many rows as the LDS budget allows
  static constexpr int TAV = (BUDGET - O_B) / 2;
  static constexpr int rc_fit(int tav) {  // largest RC with 3P*((RC*NQ)|1) <= TAV (0 if none)
    int rc = NQ;
    while (rc > 0 && 3 * P * ((rc * NQ) | 1) > tav) rc--;
    return rc;
  }
  static constexpr int RC0 = rc_fit(TAV);
  static constexpr int RCM = RC0 < 1 ? 1 : (RC0 > NQ ? NQ : RC0);
  static constexpr int NCH = (NQ + RCM - 1) / RCM, RC = (NQ + NCH - 1) / NCH, QC = RC * NQ;
  static constexpr int QCP = QC | 1, TSZ = OTF ? 0 : 3 * P * QCP;
  static constexpr int TB0 = ev(TSZ > B_SIZE ? TSZ : B_SIZE), TB1 = 0;
  // SF: first-pass contraction partials U, W [3][2][NGL][NQ] (C1 runs the LDG face fluxes)
  static constexpr int UWSZ = 3 * 2 * NGL * NQ, B_UW = B_SIZE;
  static constexpr int ARENA = O_B + (SF ? B_UW + UWSZ : TB0 + TSZ);
  static constexpr int NGR = (32 * NGL + 63) / 64;  // granules per lane of the polling wave (SLATE)
  // B task ranges: quad points [0,Q) | face points [OF,OF+4NQ) (not SLATE) | nodal grad
  // [OG,OG+P) | LDG face nodes [OL,OL+4NGL) (SF: C1), on their own
  // waves when they fit
  static constexpr int RU = 64, OFa = ((Q + RU - 1) / RU) * RU,
                       OGa = SLATE ? OFa : ((OFa + 4 * NQ + RU - 1) / RU) * RU;
  static constexpr bool WIDE = OGa + P + (SF ? 4 * NGL : 0) <= BS;  // (exact: the LDG range runs in D0)
  static constexpr int OF = WIDE ? OFa : Q, OG = WIDE ? OGa : (SLATE ? Q : OF + 4 * NQ), OL = OG + P,
                       WEND = OL + 4 * NGL, BEND = OL;
  // FPRE (exact): A2 also interpolates each face's own-side traces and, on physical
  // boundaries, the ghost-side traces to the face quad points, into s_fi [8][4*NQ] (in the
  // W region, dead from A to D0), so B's face fluxes interpolate only the neighbour traces
  static constexpr bool FPRE = !SF && !SLATE && (LEAN || 4 * NQ * 8 <= QN_END_W);
  static constexpr int WTMAX = QC * NGL;  // term tasks of a full chunk
  // VSUM (exact, chunked D): a chunk's term tasks split in two node halves on threads
  // [0, 2*WTMAX) (the longest lane forms ceil(NGL/2) nodes' terms instead of NGL), and the 3P
  // ordered chains summed by threads [OVS, BS), one per (component, node) and the same in every
  // phase, the partial sum in a register (instead of 3 chains per thread through s_rhs); qq and
  // the LDG face fluxes (D0, no sums yet) after the terms
  static constexpr int OVS = BS - 3 * P;
  static constexpr bool VSUM = !SF && !OTF && 2 * WTMAX <= OVS &&
                               2 * WTMAX + P <= BS && OL >= 2 * WTMAX + P && OL + 4 * NGL <= BS;
  // NSPLIT: node groups of the term tasks (VSUM: two node halves), task t = (group t / WTMAX,
  // task t % WTMAX) on thread t.  (Measured, not kept: one group in the LEAN arenas, thirds, and the
  // summing chains packed onto fewer waves -- DESIGN.md §9.)
  static constexpr int NSPLIT = VSUM ? 2 : 1;
  // (LEAN: the rhs is written only in the last D phase, by the VSUM lanes)
  static_assert(!LEAN || (VSUM && TSZ >= 32 * NQ && TSZ >= 5 * P && 3 * P <= 64 * EW + 64), "LEAN layout");
  static constexpr int TB_LAST = (NCH & 1) ? TB1 : TB0, TB_PREV = (NCH & 1) ? TB0 : TB1;
  // REGACC (persistent sub-cycle): every accumulating task (quad point, face quad point, node,
  // LDG face node) has its own thread, the same in every stage, so the time averages can live in
  // that thread's registers for the whole launch and be written once, scaled, at the end
  static constexpr bool REGACC = WIDE && OL + 4 * NGL <= BS;
};

// Nodal derivatives at node (i,j) keep the reference's 2*NGL-1 nonzero terms (mm==j or
// n==i) in its order.  Each term's coefficient is written uniformly as A*e + B*n with
//   A = HE_DF coefficient = dpsi(n,i) on the row through the node (mm == j), else 0,
//   B = HN_DF coefficient = dpsi(mm,j) on the column (n == i), else 0,
// taken from the LDS table with a zero slot at index NGL*NGL: on the node itself both are
// present and A*e + B*n is the reference's full expression, elsewhere the missing half adds
// a signed zero (x + 0 == x), so the sums are the reference's without selects or branches.
// (Written with selects only: short-circuit conditions here compiled to exec-mask branches per
// term, ~25 VALU + 10 SALU per term.)
template <int NGL>
__device__ __forceinline__ void nz_coef(int r, int i, int j, int &mm, int &n, int &ia, int &ib) {
  const int d = r - j;
  const bool row = (unsigned)d < (unsigned)NGL;
  mm = min(r, j) + max(d - NGL + 1, 0);
  n = row ? d : i;
  ia = row ? d * NGL + i : NGL * NGL;
  ib = (row & (d != i)) ? NGL * NGL : mm * NGL + j;
}

// grad of u_bar at node (i,j) along one metric pair: sum over source nodes (mm,n) of
// (HE_DF(n,mm,i,j)*ex + HN_DF(n,mm,i,j)*nx) * u(mm,n)  (mod_barotropic_terms.F90:427-441);
// u = qb(comp)/qb(0).  s_dpsi needs the zero slot [NGL*NGL].
template <int NGL>
__device__ __forceinline__ double nodal_grad(const double *s_dpsi, int i, int j, double ex, double nx,
                                             const double *s_w) {
  constexpr int NT = 2 * NGL - 1;
  double A[NT], B[NT], W[NT];
#pragma unroll
  for (int r = 0; r < NT; r++) {
    int mm, n, ia, ib;
    nz_coef<NGL>(r, i, j, mm, n, ia, ib);
    A[r] = s_dpsi[ia];
    B[r] = s_dpsi[ib];
    W[r] = s_w[mm * NGL + n];
  }
  asm volatile("" ::: "memory");  // all loads in flight before the ordered sum
  double gsum = 0.0;
#pragma unroll
  for (int r = 0; r < NT; r++) gsum = gsum + (A[r] * ex + B[r] * nx) * W[r];
  return gsum;
}

// all four components grad(u_bar) = (du/dx, du/dy, dv/dx, dv/dy) at node (i,j): the same four
// ordered sums as nodal_grad, sharing the coefficient and source-node loads
template <int NGL>
__device__ __forceinline__ void nodal_grad4(const double *s_dpsi, int i, int j, double ex, double ey, double nx,
                                            double ny, const double *s_u, const double *s_v, double g[4]) {
  constexpr int NT = 2 * NGL - 1, GB = NT <= 9 ? NT : 5;  // terms per load batch (VGPRs at NGL = 8)
  g[0] = g[1] = g[2] = g[3] = 0.0;
#pragma unroll
  for (int r0 = 0; r0 < NT; r0 += GB) {
    double A[GB], B[GB], U[GB], V[GB];
#pragma unroll
    for (int r = r0; r < r0 + GB && r < NT; r++) {
      int mm, n, ia, ib;
      nz_coef<NGL>(r, i, j, mm, n, ia, ib);
      A[r - r0] = s_dpsi[ia];
      B[r - r0] = s_dpsi[ib];
      U[r - r0] = s_u[mm * NGL + n];
      V[r - r0] = s_v[mm * NGL + n];
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int r = r0; r < r0 + GB && r < NT; r++) {
      const double d0 = A[r - r0] * ex + B[r - r0] * nx, d1 = A[r - r0] * ey + B[r - r0] * ny;
      g[0] = g[0] + d0 * U[r - r0];
      g[1] = g[1] + d1 * U[r - r0];
      g[2] = g[2] + d0 * V[r - r0];
      g[3] = g[3] + d1 * V[r - r0];
    }
  }
}

// Task range [0,n) laid out from virtual slot o on: task t runs on thread (o+t) % BS, in
// the first pass iff o+t < BS (tasks of a first pass may use registers preloaded by role).
template <int BS, class F>
__device__ __forceinline__ void for_tasks(int tid, int o, int n, F &&f) {
  static_assert((BS & (BS - 1)) == 0, "BS must be a power of two");
  for (int t = (tid - o) & (BS - 1); t < n; t += BS) {
    asm volatile("" ::: "memory");
    f(t, o + t < BS);
  }
}

#define STAGE_MARK(k) \
  if (PROF && tid == 0) s_prof[k] = clock64();

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for
// its outstanding global stores (accumulators / outputs are read by later kernels only),
// unlike __syncthreads(), whose release fence drains every store of the wave first.
#define LDS_BARRIER() asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory")

// SF = false: the reference's summation order (bitwise parity, see the header);
// SF = true: sum-factorised interpolation and volume integral (tensor-product contractions,
// ~7x fewer flops, equal to the reference up to rounding -- hnumo_set_summation).
// PERSIST: the body inside btp_subcycle_kernel.  The element's statics stay in LDS from the
// first stage on; the data other workgroups (or this one, earlier in the launch) wrote --
// the state buffers and the neighbour traces -- move with sc1 (L2-coherent, write-through)
// register loads and stores (MI355X_MICROARCH.md, inter-workgroup visibility).
// ACCF: the stage's time-average mode fixed at compile time (per-stage launches of the LEAN arenas:
// 1 the first stage of a sub-cycle, which stores 0 + x; 2 the later ones, which add), instead of a
// branch on StageArgs::accumulate at every one of the ~35 accumulator sites; 0: read at run time.
// (C4 1264-1273 -> 1249-1255 us per stage, lake200 516 -> 508, same bits: profiles/r06/ab_accf.log.
// The scratch-loaded bottom-layer qprime of the later stages fixed the same way measured slower,
// 1252 -> 1261-1264 us, and is not kept.)
// FST: whether this is a sub-cycle's first stage fixed at compile time (1 first, 2 a later one; 0:
// the argument first_rt decides).
template <int NGL, int NQ, bool SF, bool PERSIST, class ARGS, int NB = 0, int ACCF = 0, int FST = 0>
__device__ __forceinline__ void stage_body(const ARGS &a, double *s_arena, unsigned long long *s_prof,
                                           bool first_rt, const int e, const int tid, unsigned long long ep = 0,
                                           double *pacc = nullptr) {
  const int accm = ACCF == 1 ? 2 : (ACCF == 2 ? 1 : a.accumulate);
  const bool first = FST == 0 ? first_rt : FST == 1;
  using C = StageCfg<NGL, NQ, SF, NB>;
  // persistent: the time averages accumulate in pacc (this thread's registers, see REGACC)
  constexpr bool REGACC = PERSIST && C::REGACC;
  constexpr int P = C::P, Q = C::Q, BS = C::BS, NCH = C::NCH, QC = C::QC, QCP = C::QCP;
  const auto &m = a.m;
  const int npoin = m.npoin;
  double *const S = s_arena;
  // basis: psiq [NGL][NQ], dpsiq [NGL][NQ] (PDI: interleaved [NGL][NQ][2]), dpsi [NGL][NGL] + a zero slot
  const double *s_psiq = S + C::O_BASIS, *s_dpsiq = s_psiq + NGL * NQ, *s_dpsi = s_dpsiq + NGL * NQ;
  // (interleaved, m.basis_pd: psiq(n, iq) and dpsiq(n, iq) adjacent, read together with one
  // ds_read_b128 where the pair is needed -- the volume terms)
  auto PSQ = [&](int x) -> double { return s_psiq[2 * x]; };
  auto DPSQ = [&](int x) -> double { return s_psiq[2 * x + 1]; };
  auto PDQ = [&](int x, double &pv, double &dv) {
    const double2 w = reinterpret_cast<const double2 *>(s_psiq)[x];
    pv = w.x;
    dv = w.y;
  };
  const int *s_er = reinterpret_cast<const int *>(S + C::O_EREC);
  const int *s_side = s_er + EREC_SIDE, *s_bc = s_er + EREC_BC;
  const int *s_nbe = s_er + EREC_NBE, *s_nblf = s_er + EREC_NBLF, *s_map = s_er + EREC_MAP, *s_pf = s_er + EREC_PF(NGL);
  const int *s_acc = s_er + EREC_ACC;
  double *s_qb = S + C::O_QB, *s_q0 = S + C::O_Q0, *s_q2 = S + C::O_Q2;  // [P][4]
  double *s_qk = S + C::O_QK;      // [QE_KEEP*Q]: W, (e_x, n_x), (e_y, n_y) pairs (qe_pos)
  double *s_ns = S + C::O_NS;      // [NE_N][P]
  double *s_nc = S + C::O_NC;      // [5][P] pbprime_visc, btp_dpp_graduv(4)
  double *s_u = S + C::O_UV, *s_v = s_u + P;  // u_bar = qb(3)/qb(1), v_bar = qb(4)/qb(1) at the nodes
  double *s_wn = S + C::O_WN;      // [4][2][NGL] face-node normals (wall fix)
  double *s_qv = S + C::O_QV;      // [NQV][Q] (see StageCfg)
  double *s_pq = s_qv + 4 * Q;     // [3][Q] bottom-layer pp, up, vp (exact, A2 -> B)
  // the quad-point values by role (StageCfg::QPM: quad-point-major): A2's interpolations c = 0..3
  // (dp, dpp, udp, vdp), the bottom layer's c = 0..2, B's outputs k = 0..6, the weight w, and the
  // metric pairs (QE_EX, QE_NX, QE_EY, QE_NY)
  constexpr bool QPM = C::QPM;
  // (QPM: slot sl of quad point q in pair-major order [4][Q][2] -- pair sl/2 of every quad point in one
  // row: a writer lane q stores a 16-byte pair 16 B past its neighbour's, conflict-free, where the
  // record-per-quad-point order [Q][8] put the 16 lanes of a ds_write_b64 group 64 B apart on two bank
  // pairs, 8-way (C3: ~1,100 conflict cycles an element-stage); the on-the-fly sums still read the
  // four pairs of a quad point with one address and four immediate offsets)
  auto QSL = [&](int sl, int q) -> double & { return s_qv[((sl >> 1) * Q + q) * 2 + (sl & 1)]; };
  auto QI = [&](int c, int q) -> double & { return QPM ? QSL(c, q) : s_qv[c * Q + q]; };
  auto QP = [&](int c, int q) -> double & { return QPM ? QSL(4 + c, q) : s_pq[c * Q + q]; };
  auto QO = [&](int k, int q) -> double & { return QPM ? QSL(1 + k, q) : s_qv[k * Q + q]; };
  auto QW = [&](int q) -> double { return QPM ? QSL(0, q) : s_qk[qe_pos(QE_W, q, Q)]; };
  auto QK = [&](int c, int q) -> double { return s_qk[qe_pos(c, q, Q) - (QPM ? Q : 0)]; };
  double *s_y = S + C::O_Y;        // SF: [NYV][NGL][NQ] interpolation partials
  double *s_grad = S + C::O_GR, *s_qq = S + C::O_QQ;  // [4][P]
  // [4][4*NQ]: wq, flux, H_kx+flux_x, H_ky+flux_y at (face lf, quad iq) = lf*NQ + iq, component-major
  // so the face tasks' lanes (consecutive lf*NQ + iq) write consecutive doubles
  double *s_fq = S + C::O_FQ;
  constexpr int FQS = 4 * NQ;
  double *s_fl = S + C::O_FL;      // [4][NGL][2]
  // [3][P], [2][P] (LEAN: in the term buffer that is dead in the last D phase)
  double *s_rhs = C::LEAN ? S + C::O_B + C::TB_LAST : S + C::O_RHS;
  double *s_lap = C::LEAN ? s_rhs + 3 * P : S + C::O_LAP;
  // [P][4] (SLIM: in place of the input; LEAN: the other term buffer, dead after D)
  double *s_qn = C::SLIM ? s_qb : (C::LEAN ? S + C::O_B + C::TB_PREV : S + C::O_QN);
  // FPRE: [8][4*NQ] face-quad traces, own side | ghost side (A2 -> B; LEAN: in term buffer 0)
  double *s_fi = C::LEAN ? S + C::O_B + C::TB0 : S + C::O_W;
  double *SI = S + C::O_BIN;       // B inputs
  double *SB = S + C::O_B;         // term buffers / partials
  double *s_qp = C::SLIM ? S + C::O_GR : SI + C::B_QP;  // [P][3] qprime of the bottom layer (A2)
  double *s_ef = SI + C::B_EF;     // [4][FBLK]
  double *s_tr = SI + C::B_TR;     // [4][8][NGL]
  double *s_ec = SI + C::B_EC;     // [4][EFC]

  // ------------------------------------------------------------- A: async loads
  if (PROF && tid == 0) s_prof[30] = wall_clock64();
  if (PROF && (tid & 63) == 0) {
    s_prof[16 + (tid >> 6)] = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_ID
    if (tid == 0) s_prof[20] = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // XCC_ID
  }
  STAGE_MARK(0);
  __builtin_amdgcn_s_setprio(PRIO_B);
  if (PROF && tid == 0) s_prof[22] = 0;
  const bool use_q0 = !a.rhs_only && a.a1 != 0.0, use_q2 = !a.rhs_only && a.a3 != 0.0;
  const int qpm = (SF || !m.botfr || !a.qpq) ? 0 : a.qpq_mode;  // see StageArgs::qpq
  if (!DBGX(4096)) {
    int rot = 0;
    const bool tsl = !PERSIST && m.etsrc && !a.tcontig;
    const int4 ts = tsl ? slot_ids4(m.etsrc + 4 * e) : make_int4(0, 0, 0, 0);
    if (!PERSIST || first) {
      glds_copy<BS, C::G16>(m.basis_pd, S + C::O_BASIS, 2 * C::NB, tid, rot);
      glds_copy<BS, C::G16>(m.erec + (size_t)e * C::ERS, S + C::O_EREC, C::ERS, tid, rot);
      glds_copy<BS, C::G16>(m.qstatE + (size_t)e * qe_stride(Q) + (QPM ? Q : 0), s_qk, 2 * C::QKR * Q, tid, rot);
      if constexpr (!C::SLIM) glds_copy<BS, C::G16>(a.ecoef + (size_t)e * C::ECO + 4 * Q, s_nc, 2 * 5 * P, tid, rot);
      glds_copy<BS, C::G16>(m.nstatE + (size_t)e * NE_N * P, s_ns, 2 * (C::SLIM ? NE_LDS : NE_N) * P, tid, rot);
    }
    if (!PERSIST) {
      glds_copy<BS, C::G16>(a.qb_in + (size_t)e * 4 * P, s_qb, 8 * P, tid, rot);
      if (!C::SLIM && !C::LEAN && use_q0) glds_copy<BS, C::G16>(a.qb0 + (size_t)e * 4 * P, s_q0, 8 * P, tid, rot);
      if (!C::SLIM && !C::LEAN && use_q2) glds_copy<BS, C::G16>(a.qb2 + (size_t)e * 4 * P, s_q2, 8 * P, tid, rot);
      if (tsl) {
        // processor-face halo: each face's neighbour trace from its own slot (the receive
        // slot of a processor face)
        glds_copy<BS, C::G16>(a.trace_in + (size_t)ts.x * 8 * NGL, s_tr + 0 * 8 * NGL, 2 * 8 * NGL, tid, rot);
        glds_copy<BS, C::G16>(a.trace_in + (size_t)ts.y * 8 * NGL, s_tr + 1 * 8 * NGL, 2 * 8 * NGL, tid, rot);
        glds_copy<BS, C::G16>(a.trace_in + (size_t)ts.z * 8 * NGL, s_tr + 2 * 8 * NGL, 2 * 8 * NGL, tid, rot);
        glds_copy<BS, C::G16>(a.trace_in + (size_t)ts.w * 8 * NGL, s_tr + 3 * 8 * NGL, 2 * 8 * NGL, tid, rot);
      } else {
        glds_copy<BS, C::G16>(a.trace_in + (size_t)e * 32 * NGL, s_tr, 2 * 32 * NGL, tid, rot);
      }
    }
    // qprime, the face statics and the face coefficients are constant over a sub-cycle
    // (persistent: the previous stage re-fetched them in E1, see there)
    if (!PERSIST || first) {
      if (m.botfr && qpm != 2)
        glds_copy<BS, C::G16>(a.qprime + (size_t)(m.L - 1) * 3 * npoin + (size_t)e * 3 * P, s_qp, 6 * P, tid, rot);
      glds_copy<BS, C::G16>(m.efstat + (size_t)e * 4 * C::FBLK, s_ef, 2 * 4 * C::FBLK, tid, rot);
      glds_copy<BS, C::G16>(a.efcoef + (size_t)e * 4 * C::EFC, s_ec, 2 * 4 * C::EFC, tid, rot);
    }
  }
  if constexpr (PERSIST) {
    // the element's state stays in LDS from stage to stage: the previous stage's result
    // (s_qn) becomes the input, and the Shu-Osher states qb0 / qb2 are kept copies of it.
    // Stage 0 reads the sub-cycle input written by the previous launch.
    if constexpr (C::SLIM) {  // (s_qn is s_qb; qb0 / qb2 are saved below)
      if (first)
        for (int t = tid; t < 4 * P; t += BS) s_qb[t] = a.qb_in[(size_t)e * 4 * P + t];
    } else {
      for (int t = tid; t < 4 * P; t += BS) {
        const double x = first ? a.qb_in[(size_t)e * 4 * P + t] : s_qn[t];
        s_qb[t] = x;
        if (a.first_of_step) s_q0[t] = x;
        if (a.save_q2) s_q2[t] = x;
      }
    }
  }
  // Register loads for this thread's quad-point task in B (quad point tid), issued before
  // the wait so they overlap the LDS copies and the interpolation: the remaining quad
  // statics (coriolis, tau_wind, grad_zbot, 1/pb) and the baroclinic coefficients.
  // (The time averages are never read here: every stage adds its values with a global
  // float64 atomic add, which rounds exactly as acc = acc + x and, one stage per launch,
  // keeps the reference's summation order.)
  constexpr int NST = QE_N - QE_KEEP, NPRE = NST + 7;
  double pre[NPRE];
  double r_wq = 0.0;  // (QPM: the quad task's weight, into s_qv slot 0 in B)
  auto load_pre = [&]() {
    if (tid < Q) {
      const double *qse = m.qstatE + (size_t)e * qe_stride(Q) + tid;
      if (QPM) r_wq = qse[0];  // (qe_pos(QE_W, q) = q)
#pragma unroll
      for (int k = 0; k < NST; k++) pre[k] = qse[(QE_KEEP + k) * Q];
      const double *eco = a.ecoef + (size_t)e * C::ECO + tid;
#pragma unroll
      for (int k = 0; k < 4; k++) pre[NST + k] = eco[k * Q];
      if (qpm == 2) {
        const double *qq = a.qpq + (size_t)e * 3 * Q + tid;
#pragma unroll
        for (int k = 0; k < 3; k++) pre[NST + 4 + k] = qq[k * Q];
      }
    }
  };
  if (!PERSIST || first) {
    load_pre();
    __syncthreads();  // the async LDS copies have landed
  } else {
    // persistent, later stages: the B inputs re-fetched in the previous stage's E1 must have
    // landed (this wave's copies; the barrier covers the
    // others').  The register loads go out after the wait, so it does not cover them.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    LDS_BARRIER();
    load_pre();
  }
  STAGE_MARK(21);
  if constexpr (C::SLIM && PERSIST) {
    // the Shu-Osher states, saved by the E1 lane of each node (which reads them back in D)
    if ((a.first_of_step || a.save_q2) && tid >= C::EW * 64 && tid - C::EW * 64 < P) {
      const int p = tid - C::EW * 64;
      double *d = a.qsv + (size_t)e * 8 * P + p * 4;
#pragma unroll
      for (int v = 1; v < 4; v++) {
        const double x = s_qb[p * 4 + v];
        if (a.first_of_step) d[v] = x;
        if (a.save_q2) d[4 * P + v] = x;
      }
    }
  }

  if (tid == 0) S[C::O_BASIS + C::NB] = 0.0;  // zero slot of the dpsi table (nz_coef)

  // ------------------------------------------------------------- A2
  // u_bar, v_bar of the stage-input state once per node (Uk of mod_laplacian_quad.F90:48-49);
  // the face-node wall normals; and the nodal -> quad interpolations of mod_rhs_btp.F90:
  // 141-152, split over threads by variable group: (dp, dpp) | (udp, vdp) | bottom-layer
  // (pp, up, vp).  exact: one thread per (group, quad point), the reference's ordered
  // 25-term sum with PSIH = psiq(n,iq)*psiq(mm,jq); SF: first pass of the factorised sum,
  // Y(var, mm, iq) = sum_n psiq(n, iq) X(var, n + mm*NGL), one thread per (group, mm, iq).
  // persistent: this thread's neighbour-trace granule is loaded now and checked after the
  // interpolation, so the hand-off latency hides behind it
  constexpr bool GR1 = 32 * NGL <= BS;  // at most one granule per thread
  granule_u4 gx = {0u, 0u, 0u, 0u};
  bool gwant = false;
  // issue this thread's granule load (GR1) now; poll_traces checks it and polls again while
  // it is older than this stage
  auto issue_granule = [&]() {
    if constexpr (PERSIST && GR1) {
      if (tid < 32 * NGL) {
        gwant = s_bc[tid / (8 * NGL)] > 0;  // interior face: a neighbour writes this slot
        if (gwant) {
          // a compiler-tracked sc1 (L1-bypassing, L2-served) 16-byte load: it may stay in
          // flight across phases, and the compiler waits for it where gx is first used
          const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
              (void *)(a.gtr_in + (size_t)e * 32 * NGL), 0, 32 * NGL * (int)sizeof(TraceGranule), 0x00020000);
          gx = __builtin_amdgcn_raw_buffer_load_b128(r, tid * (int)sizeof(TraceGranule), 0, 16 /* sc1 */);
        }
      }
    }
  };
  auto poll_traces = [&]() {
    if constexpr (PERSIST) {
      const unsigned long long want = (ep << 20) | a.tag_in;
      const unsigned long long c0 = PROF ? clock64() : 0;
      for (int t = tid; t < 32 * NGL; t += BS) {
        bool w_ = GR1 ? gwant : s_bc[t / (8 * NGL)] > 0;
        if (!w_) continue;
        const TraceGranule *g = a.gtr_in + (size_t)e * 32 * NGL + t;
        double v;
        unsigned long long tag;
        if (GR1) {
          v = __builtin_bit_cast(double, ((unsigned long long)gx[1] << 32) | gx[0]);
          tag = ((unsigned long long)gx[3] << 32) | gx[2];
        } else {
          ld_granule(g, v, tag);
        }
        unsigned spins = 0;
        while (tag != want && !DBG(16)) {
          __builtin_amdgcn_s_sleep(1);
          ld_granule(g, v, tag);
          if (++spins > (1u << 20)) {  // never expected: report instead of hanging the GPU
            atomicOr(a.err, 8);
            break;
          }
        }
        s_tr[t] = v;
      }
      if (PROF) atomicMax(&s_prof[22], clock64() - c0);  // longest trace wait of the stage
    }
  };
  // SLATE: the last wave loads every granule of the element (NGR per lane) and checks them in D
  // (poll_wave), before the face fluxes it runs there
  granule_u4 gxr[C::NGR];
  auto issue_granules_wave = [&]() {
    if constexpr (PERSIST && C::SLATE) {
      if (tid >= BS - 64) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(a.gtr_in + (size_t)e * 32 * NGL), 0, 32 * NGL * (int)sizeof(TraceGranule), 0x00020000);
#pragma unroll
        for (int k = 0; k < C::NGR; k++)  // (past the record: the buffer bound returns zeros)
          gxr[k] = __builtin_amdgcn_raw_buffer_load_b128(r, ((tid & 63) + 64 * k) * (int)sizeof(TraceGranule), 0, 16);
      }
    }
  };
  auto poll_wave = [&]() {
    if constexpr (PERSIST && C::SLATE) {
      const unsigned long long want = (ep << 20) | a.tag_in;
      const unsigned long long c0 = PROF ? clock64() : 0;
#pragma unroll
      for (int k = 0; k < C::NGR; k++) {
        const int t = (tid & 63) + 64 * k;
        if (t >= 32 * NGL || s_bc[t / (8 * NGL)] <= 0) continue;  // no neighbour writes this slot
        double v = __builtin_bit_cast(double, ((unsigned long long)gxr[k][1] << 32) | gxr[k][0]);
        unsigned long long tag = ((unsigned long long)gxr[k][3] << 32) | gxr[k][2];
        unsigned spins = 0;
        while (tag != want && !DBG(16)) {
          __builtin_amdgcn_s_sleep(1);
          ld_granule(a.gtr_in + (size_t)e * 32 * NGL + t, v, tag);
          if (++spins > (1u << 20)) {  // never expected: report instead of hanging the GPU
            atomicOr(a.err, 8);
            break;
          }
        }
        s_tr[t] = v;
      }
      if (PROF) atomicMax(&s_prof[22], clock64() - c0);
    }
  };
  if constexpr (!C::SLATE) issue_granule();
  {
    // persistent, after the first stage: the wall normals and u_bar, v_bar of this state are in
    // LDS already (E1 formed u_bar, v_bar of the new state); qpm == 2: pp, up, vp are loaded
    const bool full = !PERSIST || first;
    // I4 (more quad points than half the block): one task per quad point forms all four of
    // (dp, dpp, udp, vdp) -- one pass instead of two -- and the bottom layer's three another
    constexpr bool I4 = !SF && 2 * Q > BS;
    const int ng = (m.botfr && qpm != 2) ? 3 : 2;
    constexpr int TPG = SF ? NQ * NGL : Q;  // tasks per group
    const int nint = (I4 ? ng - 1 : ng) * TPG;
    const int T_WN = nint + (full ? 8 * NGL : 0), T_UV = T_WN + (full ? P : 0);
    constexpr int NFP = C::FPRE ? 8 * NQ : 0;  // face-quad pre-interpolation tasks (own | ghost side)
    for (int w = tid; w < T_UV + NFP; w += BS) {
      asm volatile("" ::: "memory");
      if (w < nint) {
        if (DBGX(128)) continue;
        const int g = w / TPG, r = w % TPG;
        if constexpr (SF) {
          const int mm = r / NQ, iq = r % NQ;
          double pa[NGL];
#pragma unroll
          for (int n = 0; n < NGL; n++) pa[n] = PSQ(n * NQ + iq);
          if (g < 2) {
            double x0 = 0.0, x1 = 0.0;
#pragma unroll
            for (int n = 0; n < NGL; n++) {
              const int ip = mm * NGL + n;
              x0 = x0 + pa[n] * s_qb[ip * 4 + 2 * g];
              x1 = x1 + pa[n] * s_qb[ip * 4 + 2 * g + 1];
            }
            s_y[((2 * g) * NGL + mm) * NQ + iq] = x0;
            s_y[((2 * g + 1) * NGL + mm) * NQ + iq] = x1;
          } else {
            double x0 = 0.0, x1 = 0.0, x2 = 0.0;
#pragma unroll
            for (int n = 0; n < NGL; n++) {
              const int ip = mm * NGL + n;
              x0 = x0 + pa[n] * s_qp[ip * 3 + 0];
              x1 = x1 + pa[n] * s_qp[ip * 3 + 1];
              x2 = x2 + pa[n] * s_qp[ip * 3 + 2];
            }
            s_y[(4 * NGL + mm) * NQ + iq] = x0;
            s_y[(5 * NGL + mm) * NQ + iq] = x1;
            s_y[(6 * NGL + mm) * NQ + iq] = x2;
          }
        } else if (I4 && g == 0) {
          const int q = r, iq = q % NQ, jq = q / NQ;
          double pa[NGL];
#pragma unroll
          for (int n = 0; n < NGL; n++) pa[n] = PSQ(n * NQ + iq);
          double x0 = 0.0, x1 = 0.0, x2 = 0.0, x3 = 0.0;
#pragma unroll 1
          for (int mm = 0; mm < NGL; mm++) {
            const double pbm = PSQ(mm * NQ + jq);
#pragma unroll
            for (int n = 0; n < NGL; n++) {
              const int ip = mm * NGL + n;
              const double hi = pa[n] * pbm;  // PSIH(n,mm,iq,jq)
              x0 = x0 + hi * s_qb[ip * 4 + 0];
              x1 = x1 + hi * s_qb[ip * 4 + 1];
              x2 = x2 + hi * s_qb[ip * 4 + 2];
              x3 = x3 + hi * s_qb[ip * 4 + 3];
            }
          }
          QI(0, q) = x0;
          QI(1, q) = x1;
          QI(2, q) = x2;
          QI(3, q) = x3;
        } else {
          const int q = r, iq = q % NQ, jq = q / NQ;
          double pa[NGL], pb[NGL];
#pragma unroll
          for (int n = 0; n < NGL; n++) {
            pa[n] = PSQ(n * NQ + iq);
            pb[n] = PSQ(n * NQ + jq);
          }
          if (!I4 && g < 2) {
            // broadcast LDS reads (every lane of the group reads the same node)
            double x0 = 0.0, x1 = 0.0;
#pragma unroll 1
            for (int mm = 0; mm < NGL; mm++)
#pragma unroll
              for (int n = 0; n < NGL; n++) {
                const int ip = mm * NGL + n;
                const double hi = pa[n] * pb[mm];  // PSIH(n,mm,iq,jq)
                x0 = x0 + hi * s_qb[ip * 4 + 2 * g];
                x1 = x1 + hi * s_qb[ip * 4 + 2 * g + 1];
              }
            QI(2 * g, q) = x0;
            QI(2 * g + 1, q) = x1;
          } else {
            double x0 = 0.0, x1 = 0.0, x2 = 0.0;
#pragma unroll 1
            for (int mm = 0; mm < NGL; mm++)
#pragma unroll
              for (int n = 0; n < NGL; n++) {
                const int ip = mm * NGL + n;
                const double hi = pa[n] * pb[mm];
                x0 = x0 + hi * s_qp[ip * 3 + 0];
                x1 = x1 + hi * s_qp[ip * 3 + 1];
                x2 = x2 + hi * s_qp[ip * 3 + 2];
              }
            QP(0, q) = x0;
            QP(1, q) = x1;
            QP(2, q) = x2;
          }
        }
      } else if (w < T_WN) {
        const int t = w - nint, lf = t / (2 * NGL), c = (t / NGL) & 1, n = t % NGL;
        s_wn[t] = s_ef[lf * C::FBLK + EF_N * NQ + (c ? EFN_NY : EFN_NX) * NGL + n];
      } else if (w < T_UV) {
        const int p = w - T_WN;
        s_u[p] = s_qb[p * 4 + 2] / s_qb[p * 4];
        s_v[p] = s_qb[p * 4 + 3] / s_qb[p * 4];
      } else if constexpr (C::FPRE) {
        // face lf, quad iq: own-side traces (part 0), or on a physical boundary the ghost state
        // of btp_extract_df (mod_barotropic_terms.F90:75-91) (part 1), interpolated in the
        // reference's node order (creat_btp_fluxes_qdf, mod_rhs_btp.F90:246-259)
        const int t = w - T_UV, part = t / (4 * NQ), lf = (t / NQ) & 3, iq = t % NQ;
        const int er = s_bc[lf];
        if (part == 0 || er < 0) {  // (er == 0: processor face, the neighbour trace is received)
          const double *efn = s_ef + lf * C::FBLK + EF_N * NQ;
          double x[4][NGL], hv[NGL];
#pragma unroll
          for (int n = 0; n < NGL; n++) {
            hv[n] = PSQ(n * NQ + iq);
            const int p = s_map[lf * NGL + n];
#pragma unroll
            for (int c = 0; c < 4; c++) x[c][n] = s_qb[p * 4 + c];
            if (part == 1) {
              if (er == -4) {
                const double nxn = efn[EFN_NX * NGL + n], nyn = efn[EFN_NY * NGL + n];
                const double un = nxn * x[2][n] + nyn * x[3][n];
                x[2][n] = x[2][n] - 2.0 * un * nxn;
                x[3][n] = x[3][n] - 2.0 * un * nyn;
              } else if (er == -2) {
                x[2][n] = -x[2][n];
                x[3][n] = -x[3][n];
              }
            }
          }
          double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int n = 0; n < NGL; n++)
#pragma unroll
            for (int c = 0; c < 4; c++) acc[c] = acc[c] + hv[n] * x[c][n];
#pragma unroll
          for (int c = 0; c < 4; c++) s_fi[(4 * part + c) * FQS + lf * NQ + iq] = acc[c];
        }
      }
    }
  }
  if constexpr (PERSIST) {
    if (first && a.self_trace) {
      // the input state's traces for the neighbours' stage 0 (what grad_trace_kernel writes for the
      // per-stage path): grad(u_bar) at every node (B takes it from s_grad), then the granules
      LDS_BARRIER();  // u_bar, v_bar (A2)
      if (tid < P) {
        const int p = tid, i = p % NGL, j = p / NGL;
        double g[4];
        nodal_grad4<NGL>(s_dpsi, i, j, s_ns[NE_EX * P + p], s_ns[NE_EY * P + p], s_ns[NE_NX * P + p],
                         s_ns[NE_NY * P + p], s_u, s_v, g);
#pragma unroll
        for (int c = 0; c < 4; c++) s_grad[c * P + p] = g[c];
      }
      LDS_BARRIER();
      for (int t = tid; t < 4 * 8 * NGL; t += BS) {
        const int lf = t / (8 * NGL), c = (t / NGL) % 8, n = t % NGL;
        if (s_bc[lf] < 0) continue;
        const int p = s_map[lf * NGL + n];
        const double val = c < 4 ? s_qb[p * 4 + c] : s_grad[(c - 4) * P + p];
        const size_t slot = (((size_t)s_nbe[lf] * 4 + s_nblf[lf]) * 8 + c) * NGL + n;
        st_granule(a.gtr_in + slot, val, (ep << 20) | a.tag_in);
      }
    }
  }
  if constexpr (!C::SLATE) poll_traces();  // (the granule was issued before the interpolation)
  LDS_BARRIER();
  STAGE_MARK(1);

  // ---- creat_btp_fluxes_qdf at (face lf, quad iq) (mod_rhs_btp.F90:246-337); t = lf*NQ + iq
  auto face_task = [&](int t) {
    const int lf = t / NQ, iq = t % NQ;
    const int side = s_side[lf], er = s_bc[lf];
    const bool keep = accm && s_acc[lf];
    const double *ef = s_ef + lf * C::FBLK, *efn = ef + EF_N * NQ;
    const double *ec = s_ec + lf * C::EFC;
    const double *tr = s_tr + lf * 8 * NGL;
    double ql[4] = {0, 0, 0, 0}, qr[4] = {0, 0, 0, 0};
    const double pbl = ef[EF_PBLQ * NQ + iq], pbr = ef[EF_PBRQ * NQ + iq];
    if constexpr (C::FPRE) {
      // own side and ghost side interpolated in A2; the neighbour side here
      const double *fi = s_fi + lf * NQ + iq;  // [8][4*NQ]
      double fo[4], fr[4];
#pragma unroll
      for (int c = 0; c < 4; c++) fo[c] = fi[c * FQS];
      if (er >= 0) {  // interior or processor face: the neighbour's trace
        double tv[4][NGL], hv[NGL];
#pragma unroll
        for (int n = 0; n < NGL; n++) {
          hv[n] = PSQ(n * NQ + iq);
#pragma unroll
          for (int c = 0; c < 4; c++) tv[c][n] = tr[c * NGL + n];
        }
        asm volatile("" ::: "memory");
#pragma unroll
        for (int c = 0; c < 4; c++) fr[c] = 0.0;
#pragma unroll
        for (int n = 0; n < NGL; n++)
#pragma unroll
          for (int c = 0; c < 4; c++) fr[c] = fr[c] + hv[n] * tv[c][n];
      } else {
#pragma unroll
        for (int c = 0; c < 4; c++) fr[c] = fi[(4 + c) * FQS];
      }
#pragma unroll
      for (int c = 0; c < 4; c++) {
        ql[c] = side == 0 ? fo[c] : fr[c];
        qr[c] = side == 0 ? fr[c] : fo[c];
      }
    } else {
#pragma unroll
    for (int n = 0; n < NGL; n++) {
      const double hi = PSQ(n * NQ + iq);
      const int p = s_map[lf * NGL + n];
      double own[4] = {s_qb[p * 4], s_qb[p * 4 + 1], s_qb[p * 4 + 2], s_qb[p * 4 + 3]};
      double oth[4];
      if (er >= 0) {
#pragma unroll
        for (int c = 0; c < 4; c++) oth[c] = tr[c * NGL + n];
      } else {
        // ghost state of btp_extract_df (mod_barotropic_terms.F90:75-91)
#pragma unroll
        for (int c = 0; c < 4; c++) oth[c] = own[c];
        if (er == -4) {
          const double nxn = efn[EFN_NX * NGL + n], nyn = efn[EFN_NY * NGL + n];
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
    }
    }
    const double nxl = ef[EF_NX * NQ + iq], nyl = ef[EF_NY * NQ + iq];
    const double nxr = -nxl, nyr = -nyl;
    const double pU_L = nxl * ql[2] + nyl * ql[3];
    const double pU_R = nxr * qr[2] + nyr * qr[3];
    const double pbpert_edge =
        ef[EF_CL * NQ + iq] * ql[1] + ef[EF_CR * NQ + iq] * qr[1] + ef[EF_CLR * NQ + iq] * (pU_L + pU_R);
    const double ope_e = 1.0 + pbpert_edge * ef[EF_OOPE * NQ + iq];
    const double cml = ef[EF_CML * NQ + iq], cmr = ef[EF_CMR * NQ + iq], cmlr = ef[EF_CMLR * NQ + iq];
    const double fex = cml * ql[2] + cmr * qr[2] + cmlr * (nxl * ql[1] + nxr * qr[1]);
    const double fey = cml * ql[3] + cmr * qr[3] + cmlr * (nyl * ql[1] + nyr * qr[1]);
    const double ul = ql[2] / ql[0], ur = qr[2] / qr[0], vl = ql[3] / ql[0], vr = qr[3] / qr[0];
    const double quu = 0.5 * (ul * ql[2] + ur * qr[2]) + ope_e * ec[FC_QUU * NQ + iq];
    const double quv = 0.5 * (vl * ql[2] + vr * qr[2]) + ope_e * ec[FC_QUV * NQ + iq];
    const double qvu = 0.5 * (ul * ql[3] + ur * qr[3]) + ope_e * ec[FC_QUV * NQ + iq];
    const double qvv = 0.5 * (vl * ql[3] + vr * qr[3]) + ope_e * ec[FC_QVV * NQ + iq];
    const double Hf = (ope_e * ope_e) * ec[FC_HBCL * NQ + iq];
    if (keep) {  // face time averages, kept by one element per face
      const double opl = 1.0 + (ql[1] / pbl), opr = 1.0 + (qr[1] / pbr);
      double add[FA_N];
      add[FA_MFX] = fex; add[FA_MFY] = fey; add[FA_H] = Hf; add[FA_QUU] = quu; add[FA_QUV] = quv;
      add[FA_QVU] = qvu; add[FA_QVV] = qvv; add[FA_OPEL] = opl; add[FA_OPER] = opr;
      add[FA_OPE2L] = opl * opl; add[FA_OPE2R] = opr * opr; add[FA_OPEE2] = ope_e * ope_e;
      add[FA_UL] = ul; add[FA_UR] = ur; add[FA_VL] = vl; add[FA_VR] = vr;
      if constexpr (REGACC) {
#pragma unroll
        for (int k = 0; k < FA_N; k++) pacc[k] = pacc[k] + add[k];
      } else {
#pragma unroll
        for (int k = 0; k < FA_N; k++) acc_put(&a.facc[FACC_I(k, e * 4 + lf, iq)], add[k], accm == 2);
      }
    }
    const double H_kx = nxl * Hf, H_ky = nyl * Hf;
    const double lamb = cmlr;
    const double dispu = 0.5 * lamb * (qr[2] - ql[2]);
    const double dispv = 0.5 * lamb * (qr[3] - ql[3]);
    const double flux_x = nxl * quu + nyl * quv - dispu;
    const double flux_y = nxl * qvu + nyl * qvv - dispv;
    const double flux = nxl * fex + nyl * fey;
    double *fq = s_fq + lf * NQ + iq;
    fq[0] = ef[EF_W * NQ + iq];
    fq[FQS] = flux;
    fq[2 * FQS] = H_kx + flux_x;
    fq[3 * FQS] = H_ky + flux_y;
  };

  // ------------------------------------------------------------- B
  for (int w = tid; w < C::BEND; w += BS) {
    asm volatile("" ::: "memory");
    if (w < Q) {
      if (DBGX(256)) continue;
      // ---- quad-point physics (mod_rhs_btp.F90:136-192)
      const int q = w, iq = q % NQ, jq = q / NQ;
      double dp = 0, dpp = 0, udp = 0, vdp = 0, pp = 0, up = 0, vp = 0;
      if constexpr (SF) {
        // second interpolation pass: sum_mm psiq(mm, jq) Y(var, mm, iq)
#pragma unroll
        for (int mm = 0; mm < NGL; mm++) {
          const double pb = PSQ(mm * NQ + jq);
          const double *y = s_y + mm * NQ + iq;
          dp = dp + pb * y[0 * NGL * NQ];
          dpp = dpp + pb * y[1 * NGL * NQ];
          udp = udp + pb * y[2 * NGL * NQ];
          vdp = vdp + pb * y[3 * NGL * NQ];
        }
        if (m.botfr) {
#pragma unroll
          for (int mm = 0; mm < NGL; mm++) {
            const double pb = PSQ(mm * NQ + jq);
            const double *y = s_y + mm * NQ + iq;
            pp = pp + pb * y[4 * NGL * NQ];
            up = up + pb * y[5 * NGL * NQ];
            vp = vp + pb * y[6 * NGL * NQ];
          }
        }
      } else {
        dp = QI(0, q);
        dpp = QI(1, q);
        udp = QI(2, q);
        vdp = QI(3, q);
        if (qpm == 2) {
          pp = pre[NST + 4];
          up = pre[NST + 5];
          vp = pre[NST + 6];
        } else if (m.botfr) {
          pp = QP(0, q);
          up = QP(1, q);
          vp = QP(2, q);
          if (qpm == 1) {
            double *qq = a.qpq + (size_t)e * 3 * Q + q;
            qq[0] = pp;
            qq[Q] = up;
            qq[2 * Q] = vp;
          }
        }
      }
      const double cor = pre[QE_COR - QE_KEEP];
      const double tw1 = pre[QE_TW1 - QE_KEEP], tw2 = pre[QE_TW2 - QE_KEEP];
      const double gz1 = pre[QE_GZ1 - QE_KEEP], gz2 = pre[QE_GZ2 - QE_KEEP];
      const double oop = pre[QE_OOP - QE_KEEP];
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
      const double Hq = (ope * ope) * pre[NST + QC_HBCL];
      const double qu = ub * udp + ope * pre[NST + QC_QUU];
      const double quv = ub * vdp + ope * pre[NST + QC_QUV];
      const double qv = vb * vdp + ope * pre[NST + QC_QVV];
      if (accm) {  // time averages (mod_rk_mlswe.F90:107-113)
        double add[QA_N];
        add[QA_H] = Hq; add[QA_QU] = qu; add[QA_QV] = qv; add[QA_QUV] = quv;
        add[QA_TBU] = tb_u; add[QA_TBV] = tb_v; add[QA_OPE] = ope; add[QA_OPE2] = ope * ope;
        add[QA_MFX] = udp; add[QA_MFY] = vdp; add[QA_UB] = ub; add[QA_VB] = vb;
        if constexpr (REGACC) {
#pragma unroll
          for (int k = 0; k < QA_N; k++) pacc[k] = pacc[k] + add[k];
        } else {
#pragma unroll
          for (int k = 0; k < QA_N; k++) acc_put(&a.qacc[QACC_I(k, e, q)], add[k], accm == 2);
        }
      }
      if constexpr (SF) {
        // weighted integrands of T(v) = wq*(hi*S_v + dhdx*X_v + dhdy*Y_v) split by basis
        // factor: psi*psi -> F_v = wq*S_v, dpsi*psi -> G_v = wq*(e_x X_v + e_y Y_v),
        // psi*dpsi -> H_v = wq*(n_x X_v + n_y Y_v)  (create_rhs_btp_volume_qdf, :194-206)
        const double wq = s_qk[qe_pos(QE_W, q, Q)], ex = s_qk[qe_pos(QE_EX, q, Q)], ey = s_qk[qe_pos(QE_EY, q, Q)];
        const double nx = s_qk[qe_pos(QE_NX, q, Q)], ny = s_qk[qe_pos(QE_NY, q, Q)];
        const double A = Hq + qu, B = Hq + qv;
        s_qv[0 * Q + q] = wq * sc_x;
        s_qv[1 * Q + q] = wq * sc_y;
        s_qv[2 * Q + q] = wq * (ex * udp + ey * vdp);
        s_qv[3 * Q + q] = wq * (ex * A + ey * quv);
        s_qv[4 * Q + q] = wq * (ex * quv + ey * B);
        s_qv[5 * Q + q] = wq * (nx * udp + ny * vdp);
        s_qv[6 * Q + q] = wq * (nx * A + ny * quv);
        s_qv[7 * Q + q] = wq * (nx * quv + ny * B);
      } else {
        if (QPM) QSL(0, q) = r_wq;
        QO(0, q) = udp;
        QO(1, q) = vdp;
        QO(2, q) = sc_x;
        QO(3, q) = Hq + qu;
        QO(4, q) = quv;
        QO(5, q) = sc_y;
        QO(6, q) = Hq + qv;
      }
    } else if (!C::SLATE && w >= C::OF && w < C::OF + 4 * NQ) {
      if (!DBGX(512)) face_task(w - C::OF);
    } else if (w >= C::OG && w < C::OL) {
      if (DBGX(1024)) continue;
      const int p = w - C::OG, i = p % NGL, j = p / NGL;
      double g[4];
      if (PERSIST && (!first || a.self_trace)) {  // formed by the previous stage's E2 (or A2) for this state
#pragma unroll
        for (int c = 0; c < 4; c++) g[c] = s_grad[c * P + p];
      } else {
        nodal_grad4<NGL>(s_dpsi, i, j, s_ns[NE_EX * P + p], s_ns[NE_EY * P + p], s_ns[NE_NX * P + p],
                         s_ns[NE_NY * P + p], s_u, s_v, g);
#pragma unroll
        for (int c = 0; c < 4; c++) s_grad[c * P + p] = g[c];
      }
      if (accm) {
        const double t1 = 1.0 + s_qb[p * 4 + 1] * s_ns[NE_OOP * P + p];
        if constexpr (REGACC) {  // (persistent: never the method_visc == 1 branch)
#pragma unroll
          for (int c = 0; c < 4; c++) pacc[NA_G1 + c] = pacc[NA_G1 + c] + g[c];
          pacc[NA_OPE2] = pacc[NA_OPE2] + t1 * t1;
          pacc[NA_UB] = pacc[NA_UB] + s_u[p];
          pacc[NA_VB] = pacc[NA_VB] + s_v[p];
        } else {
          if (!a.lapq)
#pragma unroll
            for (int c = 0; c < 4; c++) acc_put(&a.nacc[NACC_I(NA_G1 + c, e, p)], g[c], accm == 2);
          acc_put(&a.nacc[NACC_I(NA_OPE2, e, p)], t1 * t1, accm == 2);
          acc_put(&a.nacc[NACC_I(NA_UB, e, p)], s_u[p], accm == 2);
          acc_put(&a.nacc[NACC_I(NA_VB, e, p)], s_v[p], accm == 2);
        }
      }
    }
  }
  if (PROF && (tid & 63) == 0) s_prof[12 + (tid >> 6)] = clock64();
  LDS_BARRIER();
  STAGE_MARK(2);

  // ------------------------------------------------------------- D: volume integral + LDG
  // creat_btp_fluxes_qdf projection onto node p (mod_rhs_btp.F90:339-362): left -, right +
  auto face_proj = [&](int v, int p, double acc) {
#pragma unroll
    for (int kf = 0; kf < 2; kf++) {
      const int r = s_pf[2 * p + kf];
      if (r < 0) continue;
      const int lf = r / NGL, n = r % NGL;
      const double sg = s_side[lf] == 0 ? -1.0 : 1.0;  // acc - c == acc + (-c)
      const double *fq = s_fq + lf * NQ;
#pragma unroll
      for (int iq = 0; iq < NQ; iq++) acc = acc + sg * (fq[iq] * PSQ(n * NQ + iq) * fq[(1 + v) * FQS + iq]);
    }
    return acc;
  };
  // create_rhs_laplacian_flux at (face lf, node n) (mod_laplacian_quad.F90:452-517), with the
  // element's own grad(u_bar) from B
  auto ldg_task = [&](int t, bool first) {
    const int lf = t / NGL, n = t % NGL;
    const int side = s_side[lf], er = s_bc[lf];
    const bool keep = accm && s_acc[lf] && !a.lapq;
    const int p = s_map[lf * NGL + n];
    const double *efn = s_ef + lf * C::FBLK + EF_N * NQ;
    const double *B = s_ec + lf * C::EFC + 4 * NQ;  // btp_graduv_dpp_face(c) at [c][NGL]
    const double *tr = s_tr + lf * 8 * NGL;
    const double nxn = efn[EFN_NX * NGL + n], nyn = efn[EFN_NY * NGL + n], wq = efn[EFN_W * NGL + n];
    double own[4] = {s_grad[0 * P + p], s_grad[1 * P + p], s_grad[2 * P + p], s_grad[3 * P + p]};
    double oth[4];
    if (er >= 0) {  // interior or processor face (create_rhs_lap_postcommunicator_df)
#pragma unroll
      for (int c = 0; c < 4; c++) oth[c] = tr[(4 + c) * NGL + n];
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
    if (keep) {
#pragma unroll
      for (int c = 0; c < 4; c++) {
        if constexpr (REGACC) {
          pacc[c] = pacc[c] + gl[c];
          pacc[4 + c] = pacc[4 + c] + gr[c];
        } else {
          acc_put(&a.gfacc[GFACC_I(c, e * 4 + lf, n)], gl[c], accm == 2);
          acc_put(&a.gfacc[GFACC_I(4 + c, e * 4 + lf, n)], gr[c], accm == 2);
        }
      }
    }
    double fl[4], fr[4];
#pragma unroll
    for (int iv = 0; iv < 4; iv++) {
      fl[iv] = B[4 * NGL + n] * gl[iv] + B[iv * NGL + n];
      fr[iv] = B[9 * NGL + n] * gr[iv] + B[(5 + iv) * NGL + n];
    }
    const double beta = 0.5, alpha = 1.0 - beta;
    const double qum0 = alpha * fl[0] + beta * fr[0], qum1 = alpha * fl[1] + beta * fr[1];
    const double qvm0 = alpha * fl[2] + beta * fr[2], qvm1 = alpha * fl[3] + beta * fr[3];
    const double flux_qu = (qum0 - fl[0] * nxn) + (qum1 - fl[1] * nyn);
    const double flux_qv = (qvm0 - fl[2] * nxn) + (qvm1 - fl[3] * nyn);
    // psi(n,n) == 1: node n receives wq*1*flux
    const double c0 = wq * 1.0 * flux_qu, c1 = wq * 1.0 * flux_qv;
    s_fl[(lf * NGL + n) * 2 + 0] = side == 0 ? c0 : -c0;
    s_fl[(lf * NGL + n) * 2 + 1] = side == 0 ? c1 : -c1;
  };
  // LDG volume fluxes qq (btp_compute_laplacian, mod_laplacian_quad.F90:374-380)
  auto qq_task = [&](int p) {
    const double pv = s_nc[NC_PV * P + p];
#pragma unroll
    for (int c = 0; c < 4; c++) s_qq[c * P + p] = pv * s_grad[c * P + p] + s_nc[(NC_D1 + c) * P + p];
  };
  // lap(c,p): volume over source nodes s=(ii,jj) (mod_laplacian_quad.F90:382-386), nonzero
  // terms only (jj==j or ii==i), then faces (:489-513)
  auto lap_val = [&](int c, int p) {
    const int i = p % NGL, j = p / NGL;
    double acc = 0.0;
    const int qa = (2 * c) * P, qb_ = (2 * c + 1) * P;
    // batches of LB source nodes: loads first, then the ordered updates
    constexpr int NT = 2 * NGL - 1, LB = 3;
#pragma unroll
    for (int r0 = 0; r0 < NT; r0 += LB) {
      double L_[9][LB];
#pragma unroll
      for (int r = r0; r < r0 + LB && r < NT; r++) {
        const int d = r - j;
        const bool mid = (unsigned)d < (unsigned)NGL;
        const int jj = min(r, j) + max(d - NGL + 1, 0);
        const int ii = mid ? d : i;
        const int s = jj * NGL + ii;
        const int b = r - r0;
        // HE_DF(i,j,ii,jj) = dpsi(i,ii) on the row (jj==j), HN_DF(i,j,ii,jj) = dpsi(j,jj) on
        // the column (ii==i), the zero slot elsewhere (see nz_coef)
        L_[0][b] = s_dpsi[mid ? i * NGL + d : NGL * NGL];
        L_[1][b] = s_dpsi[(mid & (d != i)) ? NGL * NGL : j * NGL + jj];
        L_[2][b] = s_ns[NE_EX * P + s];
        L_[3][b] = s_ns[NE_EY * P + s];
        L_[4][b] = s_ns[NE_NX * P + s];
        L_[5][b] = s_ns[NE_NY * P + s];
        L_[6][b] = s_ns[NE_W * P + s];
        L_[7][b] = s_qq[qa + s];
        L_[8][b] = s_qq[qb_ + s];
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int r = r0; r < r0 + LB && r < NT; r++) {
        const int b = r - r0;
        const double he = L_[0][b], hn = L_[1][b];
        const double dx = he * L_[2][b] + hn * L_[4][b];
        const double dy = he * L_[3][b] + hn * L_[5][b];
        acc = acc - L_[6][b] * (dx * L_[7][b] + dy * L_[8][b]);
      }
    }
    const int r0 = s_pf[2 * p], r1 = s_pf[2 * p + 1];
    if (r0 >= 0) acc = acc + s_fl[r0 * 2 + c];
    if (r1 >= 0) acc = acc + s_fl[r1 * 2 + c];
    return acc;
  };
  auto lap_task = [&](int c, int p) { s_lap[c * P + p] = lap_val(c, p); };
  // SLIM: values the last wave loads for its qq and E1 lanes (see StageCfg::SLIM)
  double r_q0[3] = {0.0, 0.0, 0.0}, r_q2[3] = {0.0, 0.0, 0.0}, r_mi = 0.0, r_pb = 0.0, r_lap[2] = {0.0, 0.0};

  if constexpr (SF) {
    // C1: first contraction pass over iq, per (v, i, jq):
    //   U_v(i,jq) = sum_iq psiq(i,iq) F_v + dpsiq(i,iq) G_v,  W_v(i,jq) = sum_iq psiq(i,iq) H_v
    // (F_0 = 0), with the LDG volume fluxes qq alongside
    double *s_uw = SB + C::B_UW;  // [3][2][NGL][NQ]
    constexpr int NT1 = 3 * NGL * NQ;
    for_tasks<BS>(tid, C::OL, 4 * NGL, ldg_task);
    for (int w = tid; w < NT1 + P; w += BS) {
      asm volatile("" ::: "memory");
      if (w < NT1) {
        const int v = w / (NGL * NQ), r = w % (NGL * NQ), i = r / NQ, jq = r % NQ;
        const double *F = s_qv + (v > 0 ? v - 1 : 0) * Q + jq * NQ, *G = s_qv + (2 + v) * Q + jq * NQ;
        const double *H = s_qv + (5 + v) * Q + jq * NQ;
        double u = 0.0, wv = 0.0;
#pragma unroll
        for (int iq = 0; iq < NQ; iq++) {
          double pi, dpi;
          PDQ(i * NQ + iq, pi, dpi);
          if (v > 0) u = u + pi * F[iq];
          u = u + dpi * G[iq];
          wv = wv + pi * H[iq];
        }
        s_uw[((2 * v) * NGL + i) * NQ + jq] = u;
        s_uw[((2 * v + 1) * NGL + i) * NQ + jq] = wv;
      } else {
        qq_task(w - NT1);
      }
    }
    LDS_BARRIER();
    STAGE_MARK(6);
    // C2: second pass over jq per (v, p=(i,j)): rhs = sum_jq psiq(j,jq) U + dpsiq(j,jq) W,
    // then the face projections; the Laplacian alongside
    for (int w = tid; w < 3 * P + 2 * P; w += BS) {
      asm volatile("" ::: "memory");
      if (w < 3 * P) {
        const int v = w / P, p = w % P, i = p % NGL, j = p / NGL;
        const double *U = s_uw + ((2 * v) * NGL + i) * NQ, *W = s_uw + ((2 * v + 1) * NGL + i) * NQ;
        double acc = 0.0;
#pragma unroll
        for (int jq = 0; jq < NQ; jq++) acc = acc + (PSQ(j * NQ + jq) * U[jq] + DPSQ(j * NQ + jq) * W[jq]);
        s_rhs[v * P + p] = face_proj(v, p, acc);
      } else {
        const int t = w - 3 * P;
        lap_task(t / P, t % P);
      }
    }
    LDS_BARRIER();
    STAGE_MARK(7);
  } else if constexpr (C::OTF) {
    // D (OTF): rhs(v,p) = sum_q T(v,p,q) summed in quad order by one thread, each term computed
    // as it goes (create_rhs_btp_volume_qdf, mod_rhs_btp.F90:194-206):
    //   T(0) = wq*(dhdx*udp + dhdy*vdp), T(1) = wq*(hi*scx + dhdx*A + quv*dhdy),
    //   T(2) = wq*(hi*scy + dhdx*quv + dhdy*B)
    // Then the face projections; qq and the LDG face fluxes run beside; the Laplacian after the
    // barrier.  (quad-point values by role: QO(k, q), k = 0..6 = udp, vdp, scx, A, quv, scy, B; QW,
    // QK -- see QPM)
    // OPAIR: node p's component-0 sum on one thread (without the zero hi*s1 term: the
    // reference's own wq*(dhdx*udp + dhdy*vdp)), its component-1 and -2 sums together on
    // another, sharing hi, dhdx, dhdy -- 36 instead of 48 f64 operations per (p, q), the same
    // terms in the same order
    auto otf_sum0 = [&](int p) {
      const int i = p % NGL, j = p / NGL;
      const int bi = i * NQ, bj = j * NQ;
      double acc = 0.0;
#pragma unroll 1
      for (int jq = 0; jq < NQ; jq++) {
        double pj, dpj;
        PDQ(bj + jq, pj, dpj);
        const int q0 = jq * NQ;
#pragma unroll OTF_UNROLL
        for (int iq = 0; iq < NQ; iq++) {
          const int q = q0 + iq;
          double pi, dpi;
          PDQ(bi + iq, pi, dpi);
          const double h_e = dpi * pj, h_n = pi * dpj;
          const double dhdx = h_e * QK(QE_EX, q) + h_n * QK(QE_NX, q);
          const double dhdy = h_e * QK(QE_EY, q) + h_n * QK(QE_NY, q);
          acc = acc + QW(q) * (dhdx * QO(0, q) + QO(1, q) * dhdy);
        }
      }
      return acc;
    };
    auto otf_sum12 = [&](int p, double &acc1, double &acc2) {
      const int i = p % NGL, j = p / NGL;
      const int bi = i * NQ, bj = j * NQ;
      double a1 = 0.0, a2 = 0.0;
#pragma unroll 1
      for (int jq = 0; jq < NQ; jq++) {
        double pj, dpj;
        PDQ(bj + jq, pj, dpj);
        const int q0 = jq * NQ;
#pragma unroll OTF_UNROLL
        for (int iq = 0; iq < NQ; iq++) {
          const int q = q0 + iq;
          double pi, dpi;
          PDQ(bi + iq, pi, dpi);
          const double hi = pi * pj, h_e = dpi * pj, h_n = pi * dpj;
          const double dhdx = h_e * QK(QE_EX, q) + h_n * QK(QE_NX, q);
          const double dhdy = h_e * QK(QE_EY, q) + h_n * QK(QE_NY, q);
          const double w = QW(q), uv = QO(4, q);
          a1 = a1 + w * ((hi * QO(2, q) + dhdx * QO(3, q)) + uv * dhdy);
          a2 = a2 + w * ((hi * QO(5, q) + dhdx * uv) + QO(6, q) * dhdy);
        }
      }
      acc1 = a1;
      acc2 = a2;
    };
    // TRIPLE: the three sums of node p on one thread, sharing hi, dhdx, dhdy (otf_sum0's and
    // otf_sum12's terms, the same order)
    auto otf_sum012 = [&](int p, double &acc0, double &acc1, double &acc2) {
      const int i = p % NGL, j = p / NGL;
      const int bi = i * NQ, bj = j * NQ;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll 1
      for (int jq = 0; jq < NQ; jq++) {
        double pj, dpj;
        PDQ(bj + jq, pj, dpj);
        const int q0 = jq * NQ;
#pragma unroll OTF_UNROLL
        for (int iq = 0; iq < NQ; iq++) {
          const int q = q0 + iq;
          double pi, dpi;
          PDQ(bi + iq, pi, dpi);
          const double hi = pi * pj, h_e = dpi * pj, h_n = pi * dpj;
          const double dhdx = h_e * QK(QE_EX, q) + h_n * QK(QE_NX, q);
          const double dhdy = h_e * QK(QE_EY, q) + h_n * QK(QE_NY, q);
          const double w = QW(q), uv = QO(4, q);
          a0 = a0 + w * (dhdx * QO(0, q) + QO(1, q) * dhdy);
          a1 = a1 + w * ((hi * QO(2, q) + dhdx * QO(3, q)) + uv * dhdy);
          a2 = a2 + w * ((hi * QO(5, q) + dhdx * uv) + QO(6, q) * dhdy);
        }
      }
      acc0 = a0;
      acc1 = a1;
      acc2 = a2;
    };
    {
      // waves 0..EW-1: the volume sums; the last wave: its register loads, qq, the LDG face
      // fluxes and the Laplacian (it alone writes and reads qq and the face fluxes: a wave-local
      // LDS wait, no barrier)
      double acc_r = 0.0, acc_r2 = 0.0;  // this thread's volume sum(s), lifted after the barrier
      SETPRIO_IF(tid < C::EW * 64, PRIO_S, PRIO_B);  // the volume sums ahead
      if (tid < C::EW * 64) {
        if constexpr (PERSIST) {  // (TRIPLE: the three sums of a node on one thread)
          if (tid < P) {
            double a1_, a2_;
            otf_sum012(tid, acc_r, a1_, a2_);
            s_rhs[P + tid] = a1_;  // (lifted after the barrier by waves 1 and 2)
            s_rhs[2 * P + tid] = a2_;
          }
          if (PROF && tid == 0) s_prof[28] = clock64();
        } else {  // (OPAIR: component 0 on wave 0, components 1 and 2 together on wave 1)
          if (tid < P)
            acc_r = otf_sum0(tid);
          else if (tid >= 64 && tid < 64 + P)
            otf_sum12(tid - 64, acc_r, acc_r2);
          if (PROF && tid == 0) s_prof[28] = clock64();
        }
      } else {
        const int p = tid - C::EW * 64;
        // the E1 lane's values (see StageCfg::SLIM), loaded after the Laplacian
        auto load_e1 = [&]() {
          if (p < P) {
            const double *q0s = PERSIST ? a.qsv + (size_t)e * 8 * P : a.qb0 + (size_t)e * 4 * P;
            const double *q2s = PERSIST ? a.qsv + (size_t)e * 8 * P + 4 * P : a.qb2 + (size_t)e * 4 * P;
#pragma unroll
            for (int v = 0; v < 3; v++) {
              if (use_q0) r_q0[v] = q0s[p * 4 + 1 + v];
              if (use_q2) r_q2[v] = q2s[p * 4 + 1 + v];
            }
            r_mi = m.nstatE[((size_t)e * NE_N + NE_MINV) * P + p];
            r_pb = m.nstatE[((size_t)e * NE_N + NE_PB) * P + p];
          }
        };
        if (p < P) {
          const double *nco = a.ecoef + (size_t)e * C::ECO + 4 * Q + p;
          double nc[5];
#pragma unroll
          for (int k = 0; k < 5; k++) nc[k] = nco[k * P];
          // qq_task with its coefficients from registers
#pragma unroll
          for (int c = 0; c < 4; c++) s_qq[c * P + p] = nc[NC_PV] * s_grad[c * P + p] + nc[NC_D1 + c];
        }
        // the neighbour traces (persistent: checked now), then the face fluxes (SLATE)
        issue_granules_wave();
        poll_wave();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int t = p; t < 4 * NQ; t += 64) face_task(t);
        asm volatile("" ::: "memory");
        if (p < 4 * NGL) ldg_task(p, false);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (p < P && !DBG(2)) {
          r_lap[0] = lap_val(0, p);
          r_lap[1] = lap_val(1, p);
        }
        load_e1();
        if (PROF && p == 0) s_prof[23] = clock64();  // (the last wave's D work done)
      }
      {
        LDS_BARRIER();  // the face fluxes are in
        STAGE_MARK(6);
        if constexpr (PERSIST) {
          if (tid < P) {
            s_rhs[tid] = face_proj(0, tid, acc_r);
          } else if ((tid & 63) < P && tid < 3 * 64) {
            const int v = tid >> 6, p = tid & 63;
            s_rhs[v * P + p] = face_proj(v, p, s_rhs[v * P + p]);
          }
        } else {
          if (tid < P) {
            s_rhs[tid] = face_proj(0, tid, acc_r);
          } else if (tid >= 64 && tid < 64 + P) {
            s_rhs[P + tid - 64] = face_proj(1, tid - 64, acc_r);
            s_rhs[2 * P + tid - 64] = face_proj(2, tid - 64, acc_r2);
          }
        }
      }
      LDS_BARRIER();
      STAGE_MARK(7);
      SETPRIO_IF(tid >= C::EW * 64, PRIO_E, PRIO_B);  // E1 runs on the last wave
    }
  } else {
    // D0 .. D_NCH: weak-form terms T(v,p,q) of quad-row chunk k computed in parallel into
    // term buffer k&1 (create_rhs_btp_volume_qdf, mod_rhs_btp.F90:194-206: rhs(v,I) +=
    // wq*(...)) while chunk k-1 is summed in quad order by one thread per (v,p); qq rides in
    // D0, the Laplacian in the last phase.
    // term task (q in chunk k, i): T(v, p=(i,j), q) for j = 0..NGL-1
    auto tbuf = [&](int k) { return SB + ((k & 1) ? C::TB1 : C::TB0); };
    // (VSUM: task t >= WTMAX is the second node half of pair t - WTMAX: j from JH on; the halves
    // run the same code, the second's surplus iteration masked)
    constexpr bool VSUM = C::VSUM;
    constexpr int NSP = C::NSPLIT, JH = (NGL + NSP - 1) / NSP;
    // FULLCH (every chunk whole quad rows): a term lane's (i, qi) and its quad point's column iq and
    // row offset are the same in every phase, so they are formed once, before the phases, and the
    // per-phase LDS addresses are one per-lane base plus the phase's constant (immediate offsets)
    constexpr bool FULLCH = (Q % QC == 0) && (QC % NQ == 0) && C::WTMAX * NSP <= BS;  // (task t on thread t)
    int tl_i = 0, tl_qi = 0, tl_iq = 0, tl_jr = 0;
    if constexpr (FULLCH) {
      const int h = NSP == 2 ? (tid >= C::WTMAX ? 1 : 0) : (NSP > 1 ? tid / C::WTMAX : 0), tq = tid - h * C::WTMAX;
      tl_i = tq / QC;
      tl_qi = tq - tl_i * QC;
      tl_iq = (QC == NQ) ? tl_qi : tl_qi % NQ;
      tl_jr = (QC == NQ) ? 0 : tl_qi / NQ;
    }
    auto term_task = [&](int k, int t) {
      double *T = tbuf(k);
      const int h = NSP == 2 ? (t >= C::WTMAX ? 1 : 0) : (NSP > 1 ? t / C::WTMAX : 0), tq = t - h * C::WTMAX;
      // task tq = i*nq_k + qi: consecutive lanes write consecutive quad points of one node's row
      // of the term buffer (pitch QCP = QC | 1), so a wave's ds_write_b64 lanes hit distinct banks
      // (qi-major, the lanes were QCP doubles apart: 2-way conflicts)
      const int nq_k = (k == NCH - 1) ? Q - k * QC : QC;
      const int i = FULLCH ? tl_i : tq / nq_k, qi = FULLCH ? tl_qi : tq - i * nq_k;
      const int q = k * QC + qi;
      const int iq = FULLCH ? tl_iq : q % NQ, jq = FULLCH ? k * (QC / NQ) + tl_jr : q / NQ;
      const double wq = s_qk[qe_pos(QE_W, q, Q)], ex = s_qk[qe_pos(QE_EX, q, Q)], ey = s_qk[qe_pos(QE_EY, q, Q)];
      const double nx = s_qk[qe_pos(QE_NX, q, Q)], ny = s_qk[qe_pos(QE_NY, q, Q)];
      const double udp = s_qv[0 * Q + q], vdp = s_qv[1 * Q + q], scx = s_qv[2 * Q + q], A = s_qv[3 * Q + q];
      const double quv = s_qv[4 * Q + q], scy = s_qv[5 * Q + q], B = s_qv[6 * Q + q];
      double pi, dpi;
      PDQ(i * NQ + iq, pi, dpi);
#pragma unroll
      for (int jj = 0; jj < JH; jj++) {
        const int j = h * JH + jj;
        if (j >= NGL) break;
        double pj, dpj;
        PDQ(j * NQ + jq, pj, dpj);
        const double hi = pi * pj, h_e = dpi * pj, h_n = pi * dpj;
        const double dhdx = h_e * ex + h_n * nx;
        const double dhdy = h_e * ey + h_n * ny;
        const int p = j * NGL + i;
        T[p * QCP + qi] = wq * (dhdx * udp + dhdy * vdp);
        T[(P + p) * QCP + qi] = wq * (hi * scx + dhdx * A + quv * dhdy);
        T[(2 * P + p) * QCP + qi] = wq * (hi * scy + dhdx * quv + dhdy * B);
      }
    };
    // sum task (p): rhs(v,p) += T(v,p,q) over chunk k in quad order for v = 0..2 (three
    // independent ordered chains); the face projections after the last chunk
    auto sum_task = [&](int k, int p) {
      const int nq_k = (k == NCH - 1) ? Q - k * QC : QC;
      double acc[3];
#pragma unroll
      for (int v = 0; v < 3; v++) acc[v] = k == 0 ? 0.0 : s_rhs[v * P + p];
      const double *T = tbuf(k) + p * QCP;
      // blocks of SBK quad points: all loads of a block are issued before its adds (the
      // empty asm keeps the compiler from sinking them into the dependent chain)
      constexpr int SBK = 9;
#pragma unroll 1  // (unrolled, the blocks' values stay live together: +50 VGPRs)
      for (int q0 = 0; q0 < QC; q0 += SBK) {
        double tv[3][SBK];
#pragma unroll
        for (int qi = q0; qi < q0 + SBK && qi < QC; qi++)
#pragma unroll
          for (int v = 0; v < 3; v++) tv[v][qi - q0] = qi < nq_k ? T[v * P * QCP + qi] : 0.0;
        asm volatile("" ::: "memory");
#pragma unroll
        for (int qi = q0; qi < q0 + SBK && qi < QC; qi++)
          if (qi < nq_k) {
#pragma unroll
            for (int v = 0; v < 3; v++) acc[v] = acc[v] + tv[v][qi - q0];
          }
      }
      if (k == NCH - 1 && !DBG(1)) {
        // face projections of the three components, each in the reference order; a face's
        // NQ points are loaded as one batch, and acc - c is formed as acc + (-c) (exact) so
        // only the adds sit on the dependent chain
#pragma unroll
        for (int kf = 0; kf < 2; kf++) {
          asm volatile("" ::: "memory");
          const int r = s_pf[2 * p + kf];
          if (r < 0) continue;
          const int lf = r / NGL, n = r % NGL;
          const double sg = s_side[lf] == 0 ? -1.0 : 1.0;
          const double *fq = s_fq + lf * NQ;
          constexpr int FB = (NQ + 1) / 2;  // points per load batch
#pragma unroll
          for (int i0 = 0; i0 < NQ; i0 += FB) {
            double c[3][FB], fw[FB], ps[FB];
#pragma unroll
            for (int iq = i0; iq < i0 + FB && iq < NQ; iq++) {
              fw[iq - i0] = fq[iq];
              ps[iq - i0] = PSQ(n * NQ + iq);
#pragma unroll
              for (int v = 0; v < 3; v++) c[v][iq - i0] = fq[(1 + v) * FQS + iq];
            }
            asm volatile("" ::: "memory");
#pragma unroll
            for (int iq = i0; iq < i0 + FB && iq < NQ; iq++) {
              const double wp = fw[iq - i0] * ps[iq - i0];
#pragma unroll
              for (int v = 0; v < 3; v++) acc[v] = acc[v] + sg * (wp * c[v][iq - i0]);
            }
          }
        }
      }
#pragma unroll
      for (int v = 0; v < 3; v++) s_rhs[v * P + p] = acc[v];
    };
    // the last chunk, one thread per (v, p) (one chain each, a third of the face-lift chain of
    // sum_task): rhs(v,p) += T(v,p,q) over the chunk, then the face projections of component v,
    // the same adds in the same order as sum_task
    auto sum_last_v = [&](int v, int p) {
      constexpr int kc = NCH - 1, nq_k = Q - kc * QC;
      double acc = kc == 0 ? 0.0 : s_rhs[v * P + p];
      const double *T = tbuf(kc) + (v * P + p) * QCP;
      constexpr int SBK = 9;
#pragma unroll 1
      for (int q0 = 0; q0 < nq_k; q0 += SBK) {
        double tv[SBK];
#pragma unroll
        for (int qi = 0; qi < SBK; qi++) tv[qi] = q0 + qi < nq_k ? T[q0 + qi] : 0.0;
        asm volatile("" ::: "memory");
#pragma unroll
        for (int qi = 0; qi < SBK; qi++)
          if (q0 + qi < nq_k) acc = acc + tv[qi];
      }
      if (!DBG(1)) {
#pragma unroll
        for (int kf = 0; kf < 2; kf++) {
          asm volatile("" ::: "memory");
          const int r = s_pf[2 * p + kf];
          if (r < 0) continue;
          const int lf = r / NGL, n = r % NGL;
          const double sg = s_side[lf] == 0 ? -1.0 : 1.0;
          const double *fq = s_fq + lf * NQ;
          double c[NQ], fw[NQ], ps[NQ];
#pragma unroll
          for (int iq = 0; iq < NQ; iq++) {
            fw[iq] = fq[iq];
            ps[iq] = PSQ(n * NQ + iq);
            c[iq] = fq[(1 + v) * FQS + iq];
          }
          asm volatile("" ::: "memory");
#pragma unroll
          for (int iq = 0; iq < NQ; iq++) acc = acc + sg * ((fw[iq] * ps[iq]) * c[iq]);
        }
      }
      s_rhs[v * P + p] = acc;
    };
    // (the Laplacian from thread 0 in the last phase, these after it)
    constexpr int OSV = ((2 * P + 63) / 64) * 64;
    constexpr bool VSPLIT = OSV + 3 * P <= BS;
    // lanes: terms from 0, the sums on the last wave when they fit beside the terms, qq
    // after the terms (D0), the Laplacian from 0 in the last phase (no terms there); the face
    // fluxes ran in B, the LDG fluxes run in D0
    constexpr int WTMAX = C::WTMAX;
    constexpr int OSUM = (P <= 64 && WTMAX <= BS - 64) ? BS - 64 : WTMAX;
    // VSUM: thread OVS + (v*P + p) sums chain (v, p) of every chunk, the partial sum in vacc
    // (VPACK: chain tid - VCH_HI on the last wave, 64 + tid - VCH_LO on wave 1)
    const int vch = tid >= C::OVS ? tid - C::OVS : -1;
    double vacc = 0.0;
    auto vsum_chunk = [&](int k) {
      const int t = vch, v = t / P, p = t - v * P;
      const int nq_k = (k == NCH - 1) ? Q - k * QC : QC;
      const double *T = tbuf(k) + (v * P + p) * QCP;
      constexpr int SBK = 9;
#pragma unroll 1
      for (int q0 = 0; q0 < nq_k; q0 += SBK) {
        double tv[SBK];
#pragma unroll
        for (int qi = 0; qi < SBK; qi++) tv[qi] = q0 + qi < nq_k ? T[q0 + qi] : 0.0;
        asm volatile("" ::: "memory");
#pragma unroll
        for (int qi = 0; qi < SBK; qi++)
          if (q0 + qi < nq_k) vacc = vacc + tv[qi];
      }
      if (k == NCH - 1) {
        if (!DBG(1)) {  // the face projections of component v (sum_last_v's)
#pragma unroll
          for (int kf = 0; kf < 2; kf++) {
            asm volatile("" ::: "memory");
            const int r = s_pf[2 * p + kf];
            if (r < 0) continue;
            const int lf = r / NGL, n = r % NGL;
            const double sg = s_side[lf] == 0 ? -1.0 : 1.0;
            const double *fq = s_fq + lf * NQ;
            double c[NQ], fw[NQ], ps[NQ];
#pragma unroll
            for (int iq = 0; iq < NQ; iq++) {
              fw[iq] = fq[iq];
              ps[iq] = PSQ(n * NQ + iq);
              c[iq] = fq[(1 + v) * FQS + iq];
            }
            asm volatile("" ::: "memory");
#pragma unroll
            for (int iq = 0; iq < NQ; iq++) vacc = vacc + sg * ((fw[iq] * ps[iq]) * c[iq]);
          }
        }
        s_rhs[v * P + p] = vacc;
      }
    };
    if constexpr (C::LEAN) {
      // the E1 lanes' Shu-Osher states (qb0, qb2 components 1..3), in flight during D
      const int p = tid - C::EW * 64;
      if (p >= 0 && p < P) {
#pragma unroll
        for (int v = 0; v < 3; v++) {
          if (use_q0) r_q0[v] = a.qb0[((size_t)e * P + p) * 4 + 1 + v];
          if (use_q2) r_q2[v] = a.qb2[((size_t)e * P + p) * 4 + 1 + v];
        }
      }
    }
    // the term-task waves behind everything else, the summing waves ahead
    SETPRIO_IF(VSUM ? tid >= C::OVS - (C::OVS & 63) : (OSUM == BS - 64 && tid >= OSUM), PRIO_S, 0);
#pragma unroll
    for (int k = 0; k <= NCH; k++) {
      asm volatile("" ::: "memory");  // keep LDS reads inside their phase (no hoisting)
      if (k == NCH) __builtin_amdgcn_s_setprio(PRIO_E);
      const int WT = (k < NCH) ? ((k == NCH - 1) ? (Q - k * QC) : QC) * NGL : 0;  // term tasks
      if constexpr (VSUM) {
        // first node halves on [0, WT), second halves on [WTMAX, WTMAX + WT)
        if ((NSP == 2 ? (tid < WT || (tid >= WTMAX && tid < WTMAX + WT))
                      : (tid < NSP * WTMAX && tid - (tid / WTMAX) * WTMAX < WT)) && !DBG(64))
          term_task(k, tid);
        if (k >= 1 && vch >= 0 && !DBG(4)) vsum_chunk(k - 1);
      } else {
      for_tasks<BS>(tid, 0, WT, [&](int t, bool) { term_task(k, t); });
      if (k >= 1 && k < NCH) for_tasks<BS>(tid, OSUM, P, [&](int t, bool) { sum_task(k - 1, t); });
      if (k == NCH && !DBG(4)) {
        if constexpr (VSPLIT)
          for_tasks<BS>(tid, OSV, 3 * P, [&](int t, bool) { sum_last_v(t / P, t % P); });
        else
          for_tasks<BS>(tid, OSUM, P, [&](int t, bool) { sum_task(k - 1, t); });
      }
      }
      if (k == 0) for_tasks<BS>(tid, VSUM ? C::NSPLIT * WTMAX : WT, P, [&](int t, bool) { qq_task(t); });
      if (k == 0) for_tasks<BS>(tid, C::OL, 4 * NGL, ldg_task);
      if (k == NCH && !DBG(2)) for_tasks<BS>(tid, 0, 2 * P, [&](int t, bool) { lap_task(t / P, t % P); });
      LDS_BARRIER();
      if (k < (PERSIST ? 2 : 6)) STAGE_MARK(6 + k);  // (persistent: slots 8-11 accumulate the phases)
    }
  }
  STAGE_MARK(3);

  // persistent: the term buffers are dead now, so the next stage's
  // bottom-layer qprime, face statics and face coefficients (constant over the sub-cycle,
  // overlaid by term buffer 1 in D1..D2) are re-fetched here, behind E1/E2, instead of at
  // the start of the next stage (the traces' slot is not touched: A2 of the next stage
  // fills it)
  if constexpr (PERSIST) {
    if (a.write_trace) {  // a next stage follows
      int rot = 0;
      if (!C::SLIM && m.botfr && qpm == 0) glds_copy<BS, C::G16>(a.qprime + (size_t)(m.L - 1) * 3 * npoin + (size_t)e * 3 * P, s_qp, 6 * P, tid, rot);
      glds_copy<BS, C::G16>(m.efstat + (size_t)e * 4 * C::FBLK, s_ef, 2 * 4 * C::FBLK, tid, rot);
      glds_copy<BS, C::G16>(a.efcoef + (size_t)e * 4 * C::EFC, s_ec, 2 * 4 * C::EFC, tid, rot);
    }
  }

  // ------------------------------------------------------------- E1: update + wall fix
  // (SLIM: on the last wave, with its registers; otherwise wave 0)
  constexpr int EW0 = (C::SLIM || C::LEAN) ? C::EW * 64 : 0;
  static_assert(P <= 64, "E1 and the nodal gradients run on one wave");
  for (int p = tid - EW0; p >= 0 && p < P; p += BS) {
    const size_t I = (size_t)e * P + p;
    const double mi = C::SLIM ? r_mi : s_ns[NE_MINV * P + p];
    double rh0 = mi * s_rhs[0 * P + p], rh1 = mi * s_rhs[1 * P + p], rh2 = mi * s_rhs[2 * P + p];
    const double l0 = a.lapq ? a.lapq[I] : (C::SLIM ? r_lap[0] : s_lap[0 * P + p]);
    const double l1 = a.lapq ? a.lapq[(size_t)npoin + I] : (C::SLIM ? r_lap[1] : s_lap[1 * P + p]);
    rh1 = rh1 + m.visc * mi * l0;
    rh2 = rh2 + m.visc * mi * l1;
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
      if (a.a1 != 0.0) x = a.a1 * ((C::SLIM || C::LEAN) ? r_q0[v - 1] : s_q0[p * 4 + v]);
      x = x + a.a2 * s_qb[p * 4 + v];
      if (a.a3 != 0.0) x = x + a.a3 * ((C::SLIM || C::LEAN) ? r_q2[v - 1] : s_q2[p * 4 + v]);
      qn[v] = x + a.dtt * rh[v - 1];
    }
    qn[0] = qn[1] + (C::SLIM ? r_pb : s_ns[NE_PB * P + p]);
    // btp_mom_boundary_df (mod_barotropic_terms.F90:180-215), faces in face-id order
#pragma unroll
    for (int kf = 0; kf < 2; kf++) {
      const int r = s_pf[2 * p + kf];
      if (r < 0) continue;
      const int lf = r / NGL, n = r % NGL, er = s_bc[lf];
      if (er == -4) {
        const double nx = s_wn[(lf * 2 + 0) * NGL + n], ny = s_wn[(lf * 2 + 1) * NGL + n];
        const double unl = qn[2] * nx + qn[3] * ny;
        qn[2] = qn[2] - unl * nx;
        qn[3] = qn[3] - unl * ny;
      } else if (er == -2) {
        qn[2] = 0.0;
        qn[3] = 0.0;
      }
    }
#pragma unroll
    for (int v = 0; v < 4; v++) s_qn[p * 4 + v] = qn[v];
    s_u[p] = qn[2] / qn[0];  // u_bar, v_bar of the new state for its face traces
    s_v[p] = qn[3] / qn[0];
  }
  if (a.rhs_only) return;
  if (a.write_trace && EW0 == 0 && BS == 256) {
    // the new state's grad(u_bar) on four waves, one component each (nodal_grad: the same terms
    // and order as nodal_grad4's), after a barrier, instead of on the E1 wave alone
    LDS_BARRIER();  // u_bar, v_bar of every node
    if ((tid & 63) < P) {
      const int c = tid >> 6, p = tid & 63, i = p % NGL, j = p / NGL;
      const double ex = s_ns[((c & 1) ? NE_EY : NE_EX) * P + p], nx = s_ns[((c & 1) ? NE_NY : NE_NX) * P + p];
      s_grad[c * P + p] = nodal_grad<NGL>(s_dpsi, i, j, ex, nx, (c >> 1) ? s_v : s_u);
    }
  } else if (a.write_trace) {
    // grad(u_bar) of the new state at every node, once (the sums B's nodal task forms): the
    // traces below read it, and the persistent kernel's next stage takes it as its own.  The
    // nodes' u_bar, v_bar were written by this same wave (P <= 64).
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (tid >= EW0 && tid - EW0 < P) {
      const int p = tid - EW0, i = p % NGL, j = p / NGL;
      double g[4];
      nodal_grad4<NGL>(s_dpsi, i, j, s_ns[NE_EX * P + p], s_ns[NE_EY * P + p], s_ns[NE_NX * P + p],
                       s_ns[NE_NY * P + p], s_u, s_v, g);
#pragma unroll
      for (int c = 0; c < 4; c++) s_grad[c * P + p] = g[c];
    }
  }
  LDS_BARRIER();
  STAGE_MARK(4);

  // ------------------------------------------------------------- E2: outputs
  // (persistent: the state stays in LDS; only the sub-cycle's last stage writes it out)
  if (!PERSIST || !a.write_trace)
    for (int t = tid; t < 4 * P; t += BS) a.qb_out[(size_t)e * 4 * P + t] = s_qn[t];
  if (a.write_trace && !DBGX(2048)) {
    // traces of the new state on each interior face, into the neighbour's slot:
    // qb(4) and grad(u_bar)(4) at the face nodes
    for (int t = tid; t < 4 * 8 * NGL; t += BS) {
      asm volatile("" ::: "memory");
      const int lf = t / (8 * NGL), c = (t / NGL) % 8, n = t % NGL;
      if (s_bc[lf] < 0) continue;  // (processor faces: into the face's send slot)
      const int p = s_map[lf * NGL + n];
      const double val = c < 4 ? s_qn[p * 4 + c] : s_grad[(c - 4) * P + p];
      const size_t slot = (((size_t)s_nbe[lf] * 4 + s_nblf[lf]) * 8 + c) * NGL + n;
      if constexpr (PERSIST)
        st_granule(a.gtr_out + slot, val, (ep << 20) | a.tag_out);
      else
        a.trace_out[slot] = val;
    }
  }
  __builtin_amdgcn_s_setprio(PRIO_B);
  if constexpr (REGACC) {
    // the sub-cycle's last stage: each accumulating thread writes its time averages once, scaled
    // as btp_finalize_kernel scales the atomically summed ones (mod_rk_mlswe.F90:124-149); the
    // face slots of faces another element keeps get zeros, as the zeroed atomic buffers did
    if (!a.write_trace && accm) {
      const double ni = a.n_inv;
      if (tid < Q) {
#pragma unroll
        for (int k = 0; k < QA_N; k++) a.qacc[QACC_I(k, e, tid)] = ni * pacc[k];
      } else if (tid >= C::OF && tid < C::OF + 4 * NQ) {
        const int t = tid - C::OF, lf = t / NQ, iq = t % NQ;
#pragma unroll
        for (int k = 0; k < FA_N; k++) a.facc[FACC_I(k, e * 4 + lf, iq)] = ni * pacc[k];
      } else if (tid >= C::OG && tid < C::OL) {
        const int p = tid - C::OG;
#pragma unroll
        for (int k = 0; k < NA_N; k++) a.nacc[NACC_I(k, e, p)] = ni * pacc[k];
      } else if (tid >= C::OL && tid < C::OL + 4 * NGL) {
        const int t = tid - C::OL, lf = t / NGL, n = t % NGL;
#pragma unroll
        for (int c = 0; c < 8; c++) a.gfacc[GFACC_I(c, e * 4 + lf, n)] = ni * pacc[c];
      }
    }
  }
  if (PROF) {
    LDS_BARRIER();
    STAGE_MARK(5);
    if (tid == 0) {
      if (PERSIST) {  // sums over the stages: A incl. the trace waits | the rest | stages
        if (first) s_prof[24] = s_prof[25] = s_prof[26] = s_prof[27] = s_prof[8] = s_prof[9] = s_prof[10] = s_prof[11] = s_prof[29] = 0;
        // per-phase sums over the stages: A2 | B | D | E, and (SLATE) the volume sums of wave 0
        s_prof[8] += s_prof[1] - s_prof[21];
        s_prof[9] += s_prof[2] - s_prof[1];
        s_prof[10] += s_prof[3] - s_prof[2];
        s_prof[11] += s_prof[5] - s_prof[3];
        if (C::SLATE) s_prof[29] += s_prof[28] - s_prof[2];
        s_prof[27] += s_prof[22];
        s_prof[24] += s_prof[21] - s_prof[0];
        s_prof[25] += s_prof[5] - s_prof[21];
        s_prof[26] += 1;
      }
      s_prof[31] = wall_clock64();
      for (int k = 0; k < 32; k++) a.prof[(size_t)e * 32 + k] = s_prof[k];
    }
  }
}

template <int NGL, int NQ, bool SF, int NB = 0, int ACCF = 0>
__global__ void __launch_bounds__((StageCfg<NGL, NQ, SF, NB>::BS), (StageCfg<NGL, NQ, SF, NB>::MINW))
    btp_stage_kernel(StageArgs a) {
  __shared__ __attribute__((aligned(16))) double s_arena[StageCfg<NGL, NQ, SF, NB>::ARENA];
  __shared__ unsigned long long s_prof[HNUMO_DIAG ? 32 : 1];
  stage_body<NGL, NQ, SF, false, StageArgs, NB, ACCF>(a, s_arena, s_prof, true,
                                                      a.elist ? a.elist[blockIdx.x] : (int)blockIdx.x, threadIdx.x);
}

// The whole barotropic sub-cycle (N_btp x kstages stages, ti_barotropic_ssprk_mlswe
// mod_rk_mlswe.F90:60-122) as ONE launch, one persistent workgroup per element: every
// workgroup must be resident at once (the engine checks the occupancy before choosing this
// path).  An element's state never leaves LDS between stages; the only data crossing
// workgroups are the face traces, written as tagged 16-byte granules that the neighbour
// polls until the tag of its stage appears (two trace buffers alternate; a neighbour that
// produced my stage-s traces has finished reading the buffer stage s+1 overwrites).  The
// tags carry a per-launch epoch, so no buffer clearing is needed.  The per-stage arguments
// (buffer rotation, Shu-Osher coefficients) come from a table the host prepares
// (engine.hip, stage_table).
struct SubArgs {
  const StageArgs *stages;         // [NS]
  int NS;
  unsigned long long *epoch;       // tag base of this launch; the last workgroup to finish bumps it
  unsigned *done;                  // finished-workgroup counter (back to 0 after every launch)
  unsigned *arrive;                // residency rendezvous word (back to 0 after every launch)
  int *err;                        // the run's flag word: RUN_ABORT (see residency_rendezvous)
  // test hook (hnumo_debug_force_abort): the launch whose epoch equals *abort_epoch gives up as a
  // non-resident one does (NULL: never)
  const unsigned long long *abort_epoch;
  // workgroup -> element (NULL: the identity; HNUMO_PERSIST_PERM, engine.hip persist_perm)
  const int *eperm;
};

// Residency rendezvous of a persistent launch (one thread per workgroup).  The sub-cycle's
// workgroups wait on each other's traces, so they must all be resident at once; whatever the
// occupancy estimate said at engine creation (co-resident work of another process, a CU count
// or LDS allocation granule the estimate did not see), a launch whose workgroups are not all
// resident must end, not spin.  Every workgroup adds 1 to the arrival word and waits until the
// count reaches the grid size.  A workgroup that waited RDV_TICKS (constant 100 MHz clock) sets
// RDV_ABORT with a compare-and-swap -- only while the count is still short, so the outcome is
// one for the whole launch: the grid-th arrival precedes any abort (every workgroup proceeds)
// or an abort precedes it (every workgroup, including the ones dispatched later as the aborting
// ones leave, sees the bit and leaves without work).  An abort also sets RUN_ABORT in the run's
// flag word; the later launches of the same run see it and leave at once.  Returns true: go.
constexpr unsigned RDV_ABORT = 0x80000000u;
constexpr unsigned long long RDV_TICKS = 2000000ull;  // 20 ms; a full grid dispatches in ~0.05 ms
__device__ __forceinline__ bool residency_rendezvous(unsigned *arrive, int *err, unsigned grid) {
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & RUN_ABORT) return false;
  const unsigned old = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old & RDV_ABORT) return false;
  if (old + 1 == grid) return true;
  const unsigned long long t0 = wall_clock64();
  for (;;) {
    unsigned w = __hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w & RDV_ABORT) return false;
    if (w == grid) return true;
    if (wall_clock64() - t0 > RDV_TICKS &&
        __hip_atomic_compare_exchange_strong(arrive, &w, w | RDV_ABORT, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)) {
      __hip_atomic_fetch_or(err, RUN_ABORT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

template <int NGL, int NQ, bool SF>
__global__ void __launch_bounds__((StageCfg<NGL, NQ, SF>::BS), (StageCfg<NGL, NQ, SF>::MINW))
    btp_subcycle_kernel(SubArgs sa) {
  using C = StageCfg<NGL, NQ, SF>;
  __shared__ __attribute__((aligned(16))) double s_arena[C::ARENA];
  __shared__ unsigned long long s_prof[HNUMO_DIAG ? 32 : 1];
  const int e = sa.eperm ? __builtin_amdgcn_readfirstlane(sa.eperm[blockIdx.x]) : (int)blockIdx.x, tid = threadIdx.x;
  const unsigned long long ep = *sa.epoch;
  typedef const __attribute__((address_space(4))) StageArgs CStageArgs;
  CStageArgs *tab = (CStageArgs *)sa.stages;
  __shared__ int s_go;
  if (tid == 0) {
    if (sa.abort_epoch && *sa.abort_epoch == ep) {  // (test hook: every workgroup leaves without work)
      __hip_atomic_fetch_or(sa.arrive, RDV_ABORT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_or(sa.err, RUN_ABORT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_go = 0;
    } else {
      s_go = residency_rendezvous(sa.arrive, sa.err, gridDim.x);
    }
  }
  __syncthreads();
  const int NS = s_go ? sa.NS : 0;  // (not resident: no stage, straight to the exit count)
  double pacc[16];  // this thread's time averages (StageCfg::REGACC)
#pragma unroll
  for (int k = 0; k < 16; k++) pacc[k] = 0.0;
  // the first stage peeled off the stage loop, so that neither copy of the body branches on it (two
  // inlined bodies; C3 35.8 -> 34.8-35.4 us per stage, dg25L3 unchanged, same bits:
  // profiles/r06/ab_pfirst.log)
  if (NS > 0) {
    int tid_s = tid, e_s = e;
    asm volatile("" : "+v"(tid_s), "+s"(e_s));
    tid_s &= C::BS - 1;
    stage_body<NGL, NQ, SF, true, CStageArgs, 0, 0, 1>(tab[0], s_arena, s_prof, true, e_s, tid_s, ep, pacc);
  }
#pragma unroll 1
  for (int stage = 1; stage < NS; stage++) {
    __syncthreads();
    // opaque per stage: keeps the body's per-thread index math from being hoisted out of the
    // stage loop (it would stay live across every phase)
    int tid_s = tid, e_s = e;
    asm volatile("" : "+v"(tid_s), "+s"(e_s));
    tid_s &= C::BS - 1;  // restore the known range of the thread index
    stage_body<NGL, NQ, SF, true, CStageArgs, 0, 0, 2>(tab[stage], s_arena, s_prof, false, e_s, tid_s, ep, pacc);
  }
  // the next launch's tags: every workgroup read the epoch at its start, so the last one to
  // finish (agent-scope counter) moves it on and resets the counters (every workgroup has passed
  // the rendezvous before it counts itself out)
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add(sa.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(sa.epoch, ep + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sa.arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sa.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Face traces of a state for the first stage of a sub-cycle / a lone RHS: qb(4) and
// grad(u_bar)(4) at the face nodes, written into the neighbours' trace slots (or, with gtr,
// as tagged granules for the persistent sub-cycle).
template <int NGL, int NQ>
__global__ void __launch_bounds__(64) grad_trace_kernel(DevMesh m, const double *qb, double *trace, int e0,
                                                         TraceGranule *gtr, const unsigned long long *epoch) {
  constexpr int P = NGL * NGL, ERS = EREC_SIZE(NGL);
  const int e = e0 + blockIdx.x, tid = threadIdx.x;
  __shared__ double s_dpsi[NGL * NGL + 1], s_qb[P * 4], s_nm[4 * P], s_u[P], s_v[P];
  __shared__ int s_er[ERS];
  for (int t = tid; t < NGL * NGL; t += 64) s_dpsi[t] = m.basis[2 * NGL * NQ + t];
  if (tid == 0) s_dpsi[NGL * NGL] = 0.0;  // zero slot (nz_coef)
  for (int t = tid; t < ERS; t += 64) s_er[t] = m.erec[(size_t)e * ERS + t];
  for (int t = tid; t < 4 * P; t += 64) s_qb[t] = qb[(size_t)e * 4 * P + t];
  for (int t = tid; t < 4 * P; t += 64) s_nm[t] = m.nstatE[(size_t)e * NE_N * P + t];  // e_x, e_y, n_x, n_y
  __syncthreads();
  for (int p = tid; p < P; p += 64) {
    s_u[p] = s_qb[p * 4 + 2] / s_qb[p * 4];
    s_v[p] = s_qb[p * 4 + 3] / s_qb[p * 4];
  }
  __syncthreads();
  for (int t = tid; t < 4 * 8 * NGL; t += 64) {
    const int lf = t / (8 * NGL), c = (t / NGL) % 8, n = t % NGL;
    if (s_er[EREC_BC + lf] < 0) continue;  // (processor faces: into the face's send slot)
    const int p = s_er[EREC_MAP + lf * NGL + n];
    double val;
    if (c < 4) {
      val = s_qb[p * 4 + c];
    } else {
      const int cg = c - 4, i = p % NGL, j = p / NGL;
      const double ex = s_nm[((cg & 1) ? NE_EY : NE_EX) * P + p], nx = s_nm[((cg & 1) ? NE_NY : NE_NX) * P + p];
      val = nodal_grad<NGL>(s_dpsi, i, j, ex, nx, (cg >> 1) ? s_v : s_u);
    }
    const size_t slot = (((size_t)s_er[EREC_NBE + lf] * 4 + s_er[EREC_NBLF + lf]) * 8 + c) * NGL + n;
    if (gtr)  // persistent sub-cycle: tagged for its stage 0
      st_granule(gtr + slot, val, (*epoch << 20) | 1ull);
    else
      trace[slot] = val;
  }
}

// Normalisation of the time averages after the sub-cycle (mod_rk_mlswe.F90:124-149).
// tau_wind_ave = (sum over N_btp of tau_wind) / N_btp, summed the same way as the reference.
// It also copies the sub-cycle's result state into qb_state (one launch instead of two).
__global__ void btp_finalize_kernel(double *qacc, double *facc, double *nacc, double *gfacc, double *tau_wind_ave,
                                    const double *tau_wind, int npq, int nfq, int npoin, int nfn, int N_btp,
                                    double N_inv, double *qb_state, const double *qb_result, int scale_acc) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  if (qb_state != qb_result)
    for (size_t i = tid; i < (size_t)4 * npoin; i += stride) qb_state[i] = qb_result[i];
  if (scale_acc) {  // (0: the persistent kernel wrote them scaled, StageCfg::REGACC)
    for (size_t i = tid; i < (size_t)QA_N * npq; i += stride) qacc[i] = N_inv * qacc[i];
    for (size_t i = tid; i < (size_t)FA_N * nfq; i += stride) facc[i] = N_inv * facc[i];
    for (size_t i = tid; i < (size_t)NA_N * npoin; i += stride) nacc[i] = N_inv * nacc[i];
    for (size_t i = tid; i < (size_t)8 * nfn; i += stride) gfacc[i] = N_inv * gfacc[i];
  }
  for (size_t i = tid; i < (size_t)2 * npq; i += stride) {
    double s = 0.0, t = tau_wind[i];
    for (int k = 0; k < N_btp; k++) s = s + t;
    tau_wind_ave[i] = s / (double)N_btp;
  }
}

#define HNUMO_INSTANTIATE_BTP(NGL, NQ)                                 \
  template __global__ void btp_stage_kernel<NGL, NQ, false>(StageArgs); \
  template __global__ void btp_stage_kernel<NGL, NQ, true>(StageArgs);  \
  template __global__ void btp_subcycle_kernel<NGL, NQ, false>(SubArgs); \
  template __global__ void btp_subcycle_kernel<NGL, NQ, true>(SubArgs);  \
  template __global__ void grad_trace_kernel<NGL, NQ>(DevMesh, const double *, double *, int, TraceGranule *, \
                                                       const unsigned long long *);

}  // namespace hnumo
