// engine.hip -- host side of libhnumo_engine: the C ABI of include/hnumo_engine.h.
//
// The engine owns all device state and reproduces the call sequence of ti_rk_bcl
// (ti_rk_bcl.F90:9-87) with the kernels of kernels_btp.hip / kernels_bcl.hip.  A whole
// baroclinic step (2 barotropic sub-cycles = 2*N_btp*kstages fused stage kernels plus
// ~20 baroclinic kernels) is captured once into a hipGraph and replayed.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hnumo_engine.h"
#include "engine_internal.h"
#include "kernels_bcl.hip"
#include "kernels_btp.hip"
#include "kernels_lapq.hip"

using namespace hnumo;

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t err_ = (x);                                                                 \
    if (err_ != hipSuccess) {                                                              \
      eng->err = std::string("HIP error: ") + hipGetErrorString(err_) + " at " #x;         \
      return HNUMO_ERR_DEVICE;                                                             \
    }                                                                                      \
  } while (0)

struct LocalGroup;

// one neighbour rank of the ghost-layer halo (h-numo_amd/hnumo/partition.py)
struct Neighbour {
  int rank = -1, nsend = 0, nrecv = 0;
  int *d_send = nullptr, *d_recv = nullptr;  // 0-based local element ids
  double *sbuf = nullptr, *rbuf = nullptr;
};

struct hnumo_engine {
  int device = 0;
  // multi-rank: 0 single, 1 local group (one process, shared stream), 2 RCCL
  int comm_mode = 0, rank = 0, nranks = 1, nelem_owned = 0;
  std::vector<Neighbour> nbh;
  ncclComm_t comm = nullptr;
  LocalGroup *group = nullptr;
  bool own_stream = true;
  std::string err;
  std::string comm_err;  // first halo-transport failure (sticky until reported)
  // environment settings this engine read at create, honoured or ignored (hnumo_overrides)
  std::string overrides;
  hipStream_t stream = nullptr;
  DevMesh m{};
  hnumo_params p{};
  int nelem, npoin, npq, nface, ngl, nq, L, P, Q, K;
  size_t FQ, FN;
  std::vector<void *> allocs;
  // statics
  double *basis, *qstat, *nstat, *fstat, *fnstat, *alpha, *tau_wind;
  int *iconn;
  std::vector<double> ssprk_a, ssprk_beta;  // host copies (kstages x 3), (kstages)
  // state and step temporaries
  double *q, *qb, *qp, *q2, *qp2, *qbp, *qf, *qf2, *qfa, *dpp2;  // (qfa: fused faces, bcl_coeffs)
  double *qbuf[4], *gtrace[2];  // gtrace: [E][4][8][NGL] face traces (qb, grad u_bar) in the reader's slot
  // per-sub-cycle coefficients
  double *qcoef, *ncoef, *fcoef, *fncoef, *dpp_graduv, *dpprime_visc, *gdpp_face;
  double *ecoef, *efcoef;                   // element-major copies for the stage kernel
  double *qstatE, *nstatE, *efstat;         // element-major statics for the stage kernel
  std::vector<int> fslotA;                  // host copy: face -> slot holding its averages
  // accumulators
  double *qacc, *facc, *nacc, *gfacc, *tau_wind_ave;
  // baroclinic scratch
  double *slmf, *slmf_face, *dpp, *fmass, *fcons, *momL, *momR, *lapf, *rhs;
  int *neg_flag, *h_neg;
  // graph
  hipGraph_t graph = nullptr;
  hipGraphExec_t graph_exec = nullptr;
  bool resident = false, uploaded = false, alloc_failed = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // events recorded inside the captured step around the corrector sub-cycle's stage kernels
  hipEvent_t evk0 = nullptr, evk1 = nullptr;
  bool capturing = false, kernel_events = false, no_graph = false;
  int graph_env = -1;                        // HNUMO_GRAPH at create: 0 direct launches, 1 capture (RCCL too), -1 unset
  bool no_fuse = false;                      // HNUMO_FUSE=0: face kernels and extract launches (A/B)
  int sched_dbg = 0;                         // HNUMO_SCHED_DBG (timing experiments only, wrong results):
                                             // 1 the interior launch skips its wait for the boundary one
  int summation = HNUMO_SUM_REFERENCE;        // hnumo_set_summation
  unsigned long long *stage_prof = nullptr;  // HNUMO_STAGE_PROF=1: per-element phase clocks
  int stage_dbg = 0;                         // HNUMO_STAGE_DBG: diagnostic phase switches (timing only)
  int stage_nb = 0;                          // per-stage kernel arena sizing (StageCfg NB; HNUMO_STAGE_NB)
  bool bcl_big = false;                      // mass/cons element kernels' small-LDS variant (HNUMO_BCL_BIG)
  bool acc_zero = false;                     // HNUMO_ACC_ZERO=1: zero the time averages before a sub-cycle (A/B)
  // persistent sub-cycle (btp_subcycle_kernel): allowed per summation mode when every element's
  // workgroup fits on the device at once (and HNUMO_PERSISTENT != 0); used on single-rank engines
  bool persistent_ok[2] = {false, false};
  bool regacc[2] = {false, false};           // persistent kernel keeps the averages in registers
  TraceGranule *gtr[2] = {nullptr, nullptr};  // tagged face traces of the persistent sub-cycle
  unsigned long long *epoch = nullptr;        // tag epoch, bumped by every persistent sub-cycle launch
  unsigned *sub_done = nullptr;               // its finished-workgroup counter
  unsigned *sub_arrive = nullptr;             // its residency rendezvous word (residency_rendezvous)
  unsigned *steps_done = nullptr, *h_steps = nullptr;  // steps completed in a run (DevMesh::steps_done)
  // residency of the persistent launch: the occupancy estimate (workgroups per CU, per summation
  // mode), the CU count, and the outcome of the creation-time trial launch (1 resident, 0 not,
  // -1 not run).  HNUMO_PERSIST_LDS_PAD (bytes of dynamic LDS per workgroup) and
  // HNUMO_PERSIST_GUARD (0: no estimate, no trial; estimate; trial) exist to test the in-launch
  // fallback and each check alone.
  int occ_blocks[2] = {0, 0}, occ_ncu = 0, probe_ok[2] = {-1, -1};
  int persist_pad = 0;
  int persist_guard = 3;                      // bit 1: occupancy estimate, bit 2: trial launch
  int persist_aborts = 0;                     // runs that found a persistent launch not co-resident
  // after an abort the persistent path is suspended, not dropped (maybe_reprobe): per-stage runs
  // while persist_wait counts down, then a stage-less trial launch decides; the wait doubles with
  // every abort or failed re-probe (up to 1024 runs) and resets after a completed persistent run
  bool persist_suspended = false;
  int persist_wait = 0, persist_backoff = 1, persist_reprobes = 0, persist_recovered = 0;
  unsigned long long *dbg_abort_epoch = nullptr;  // hnumo_debug_force_abort: the launch epoch to abort
  StageArgs *d_stages[2] = {nullptr, nullptr};  // per-stage arguments: predictor (qp), corrector (qp2)
  // processor-face halo: the reference's own partition contract (face(8) = 0 faces listed per
  // neighbour rank in nbh_send_recv; p4est.c:1686-1712, mod_parallel).  NS shared-face slots in
  // list order; neighbour j owns slots [off, off+n).  Stage traces move between the trace
  // buffers' send / receive slots (no packing); the baroclinic face exchanges pack side 1 of
  // the listed faces and unpack the neighbour's into side 2.
  bool face_halo = false;
  int NS = 0;
  struct FNbr {
    int rank = -1, off = 0, n = 0;
  };
  std::vector<FNbr> fnb;
  int *d_sface = nullptr;                    // [NS] local face of each shared slot
  double *bx_sbuf = nullptr, *bx_rbuf = nullptr;  // [NS * per-face message] baroclinic exchanges
  size_t bx_per_max = 0;
  int *d_elB = nullptr, *d_elI = nullptr;    // elements with / without a processor face
  int nB = 0, nI = 0;
  double *cdef = nullptr;                    // consistency deficits [L][side][2][F*NQ]
  // hnumo_debug_frozen_halo (self-neighbour emulation only): each exchange site's first message,
  // kept and sent again by every later exchange of the site (halo_src); site = the trace buffer
  // for the stage traces, the position in the step's sequence of baroclinic exchanges for the rest
  // (one array may carry different quantities at different points of the step)
  bool emu_frozen = false;
  int xseq = 0;                              // baroclinic exchanges so far in this step (their site)
  struct Frozen {
    const void *key;
    size_t n;
    double *buf;
  };
  std::vector<Frozen> frozen;
  hipStream_t stream2 = nullptr;             // boundary elements + trace transport (two-stream schedule)
  hipEvent_t ev_fork = nullptr, ev_join = nullptr, ev_I = nullptr, ev_B[2] = {nullptr, nullptr};
  hipEvent_t ev_Is = nullptr, ev_Bs[2] = {nullptr, nullptr};  // kernel stop events of the same hand-offs
  // local exchange group, processor-face transport: device copies ordered by events
  hipEvent_t ev_tsent = nullptr, ev_bpacked = nullptr, ev_bdone = nullptr;
  // method_visc == 1 (quad-point LDG, kernels_lapq.hip)
  bool lapq_on = false;
  double *dpq = nullptr;      // dpprime_visc_q [L][npoin_q]
  double *lq_flux = nullptr;  // LDG fluxes at the quad points [L][E][4][Q] (barotropic: layer block 0)
  double *lapq = nullptr;     // Laplacians [L][2][npoin] (barotropic: [2][npoin])
  int *fqLR = nullptr;        // [2][F][NQ] element-local quad point of each face quad point, left | right
  // bottom-layer qprime at the quad points, interpolated once per sub-cycle (StageArgs::qpq;
  // botfr != 0; HNUMO_QPQ=0: every stage interpolates, for A/B timing)
  double *qpq = nullptr;      // [E][3][Q]
  double *qsv = nullptr;      // [E][2][P][4] Shu-Osher states of the slim persistent sub-cycle (StageArgs::qsv)
  int *d_eperm = nullptr;     // persistent sub-cycle: workgroup -> element (SubArgs::eperm), NULL = identity
  // hnumo_step_breakdown: events recorded on the engine stream after every launch of a direct
  // (uncaptured) step, each with the name of the kernel family it closes (kmark)
  struct KMarks {
    std::vector<hipEvent_t> ev;
    std::vector<const char *> name;
    size_t n = 0;
  } *km = nullptr;
};

// the per-kernel breakdown's mark after a launch on the engine stream (no-op outside
// hnumo_step_breakdown; never inside a capture)
static void kmark(hnumo_engine *e, const char *name) {
  if (!e->km) return;
  auto &k = *e->km;
  if (k.n == k.ev.size()) {
    hipEvent_t ev = nullptr;
    if (hipEventCreate(&ev) != hipSuccess) return;
    k.ev.push_back(ev);
    k.name.push_back(nullptr);
  }
  (void)hipEventRecord(k.ev[k.n], e->stream);
  k.name[k.n++] = name;
}

template <typename T>
static T *dalloc(hnumo_engine *eng, size_t n) {
  void *ptr = nullptr;
  if (hipMalloc(&ptr, (n ? n : 1) * sizeof(T)) != hipSuccess) {
    eng->alloc_failed = true;
    return nullptr;
  }
  (void)hipMemset(ptr, 0, (n ? n : 1) * sizeof(T));
  eng->allocs.push_back(ptr);
  return (T *)ptr;
}

// Environment settings read at engine creation.  Two kinds:
//  * public (documented in include/hnumo_engine.h): HNUMO_PERSISTENT=0, HNUMO_GRAPH=0|1 (same
//    bits, another launch schedule) and HNUMO_SUMMATION=reference|factored (any other value is an
//    error, not a silent switch);
//  * experiment knobs (A/B timing and the equivalence tests of old behaviour, tests/
//    test_placement_gpu.py): honoured ONLY when HNUMO_EXPERIMENTS=1 is set as well, ignored
//    otherwise.
// Every variable found is recorded in eng->overrides ("NAME=value" honoured, "NAME=value
// (ignored)" not), which hnumo_overrides returns and bench.py puts in its line, so a stray
// variable on a benchmark box can never change the measured path unseen.
static const char *env_knob(hnumo_engine *eng, const char *name, bool experiment = true) {
  const char *v = getenv(name);
  if (!v) return nullptr;
  const char *x = experiment ? getenv("HNUMO_EXPERIMENTS") : nullptr;
  const bool on = !experiment || (x && x[0] == '1' && x[1] == 0);
  if (!eng->overrides.empty()) eng->overrides += ';';
  eng->overrides += std::string(name) + "=" + v + (on ? "" : " (ignored: HNUMO_EXPERIMENTS!=1)");
  return on ? v : nullptr;
}

static void face_exchange_qf(hnumo_engine *e, double *qf, int nc);
static const double *face_exchange_lapq(hnumo_engine *e, const double *flux, int nb, int nq, int Q);
static void face_exchange_gdpp(hnumo_engine *e);
static void face_exchange_cdef(hnumo_engine *e);

// ------------------------------------------------------------------ kernel dispatch
// On a single rank every face's elements are in the element kernels' launches, so
// fused_extract(e): the face traces qf of qprime are written by the kernels that write qprime
// (mom_elem, cons_elem) instead of by extract launches after them (the face traces of a qprime
// uploaded by the host are extracted at the upload, upload_state);
// fused_faces(e): the layer mass and consistency fluxes of a face are formed by the element
// kernels of both its elements instead of by the face kernels before them (HNUMO_FUSE=0: off).
static bool fused_extract(const hnumo_engine *e) {
  return e->comm_mode == 0 && e->nranks == 1 && !e->face_halo && !e->no_fuse;
}
static bool fused_faces(const hnumo_engine *e) { return fused_extract(e); }

template <int NGL, int NQ>
struct Launch {
  static constexpr int BSE = ((NQ * NQ + 63) / 64) * 64;
  // one stage over the owned elements, or over the `n` elements of a.elist on stream `st`
  // (stop: an event the launch itself signals at completion -- the two-stream schedule's hand-offs
  // without separate record packets, hipExtLaunchKernelGGL)
  static void stage(hnumo_engine *e, const StageArgs &a, int n = -1, hipStream_t st = nullptr,
                    hipEvent_t stop = nullptr) {
    if (n < 0) n = e->nelem_owned;
    if (!st) st = e->stream;
    if (n == 0) {
      if (stop) (void)hipEventRecord(stop, st);
      return;
    }
    if constexpr (NGL == 5) {
      // the LEAN arenas of large meshes (StageCfg NBK workgroups per CU; HNUMO_STAGE_NB)
      if (e->summation == HNUMO_SUM_REFERENCE && (e->stage_nb == 4 || e->stage_nb == 5)) {
        if (e->stage_nb == 5)
          launch_nb<5>(n, st, stop, a);
        else
          launch_nb<4>(n, st, stop, a);
        return;
      }
    }
    if (e->summation == HNUMO_SUM_REFERENCE)
      hipLaunchKernelGGL((btp_stage_kernel<NGL, NQ, false>), dim3(n), dim3(StageCfg<NGL, NQ, false>::BS), 0, st, a);
    else
      hipLaunchKernelGGL((btp_stage_kernel<NGL, NQ, true>), dim3(n), dim3(StageCfg<NGL, NQ, true>::BS), 0, st, a);
    if (stop) (void)hipEventRecord(stop, st);
  }
  template <int NB>
  static void launch_nb(int n, hipStream_t st, hipEvent_t stop, const StageArgs &a) {
    // (the time-average mode as a template argument: stage_body ACCF)
    if (a.accumulate == 2)
      launch_nb_acc<NB, 1>(n, st, stop, a);
    else if (a.accumulate == 1)
      launch_nb_acc<NB, 2>(n, st, stop, a);
    else
      launch_nb_acc<NB, 0>(n, st, stop, a);
  }
  template <int NB, int ACCF>
  static void launch_nb_acc(int n, hipStream_t st, hipEvent_t stop, const StageArgs &a) {
    using K = StageCfg<NGL, NQ, false, NB>;
    if (stop)
      hipExtLaunchKernelGGL((btp_stage_kernel<NGL, NQ, false, NB, ACCF>), dim3(n), dim3(K::BS), 0, st, nullptr, stop, 0,
                            a);
    else
      hipLaunchKernelGGL((btp_stage_kernel<NGL, NQ, false, NB, ACCF>), dim3(n), dim3(K::BS), 0, st, a);
  }
  static void subcycle(hnumo_engine *e, const StageArgs *stages, int ns) {
    SubArgs sa{stages, ns, e->epoch, e->sub_done, e->sub_arrive, e->neg_flag, e->dbg_abort_epoch, e->d_eperm};
    if (e->summation == HNUMO_SUM_REFERENCE)
      hipLaunchKernelGGL((btp_subcycle_kernel<NGL, NQ, false>), dim3(e->nelem_owned),
                         dim3(StageCfg<NGL, NQ, false>::BS), e->persist_pad, e->stream, sa);
    else
      hipLaunchKernelGGL((btp_subcycle_kernel<NGL, NQ, true>), dim3(e->nelem_owned), dim3(StageCfg<NGL, NQ, true>::BS),
                         e->persist_pad, e->stream, sa);
  }
  // can every workgroup of the persistent sub-cycle kernel be resident at once?  The occupancy
  // estimate first; the launch itself then checks (residency_rendezvous) and the engine runs one
  // stage-less trial launch per summation mode at creation (probe)
  static void occupancy(hnumo_engine *e, int ncu) {
    int nb0 = 0, nb1 = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb0, btp_subcycle_kernel<NGL, NQ, false>,
                                                       StageCfg<NGL, NQ, false>::BS, e->persist_pad);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb1, btp_subcycle_kernel<NGL, NQ, true>,
                                                       StageCfg<NGL, NQ, true>::BS, e->persist_pad);
    (void)hipGetLastError();
    e->occ_blocks[0] = nb0;
    e->occ_blocks[1] = nb1;
    e->occ_ncu = ncu;
    const bool est = e->persist_guard & 1;
    e->persistent_ok[0] = !est || (long)nb0 * ncu >= e->nelem_owned;
    // the slim arena keeps the bottom-layer qprime only for the first stage: the later ones need
    // the per-sub-cycle quad-point scratch
    if (StageCfg<NGL, NQ, false>::SLIM && e->m.botfr && !e->qpq) e->persistent_ok[0] = false;
    e->persistent_ok[1] = !est || (long)nb1 * ncu >= e->nelem_owned;
    e->regacc[0] = StageCfg<NGL, NQ, false>::REGACC;
    e->regacc[1] = StageCfg<NGL, NQ, true>::REGACC;
  }
  // the trial launch: the persistent grid with no stages, i.e. the residency rendezvous alone
  static void probe(hnumo_engine *e, int sum) {
    SubArgs sa{e->d_stages[0], 0, e->epoch, e->sub_done, e->sub_arrive, e->neg_flag, nullptr, e->d_eperm};
    if (sum == HNUMO_SUM_REFERENCE)
      hipLaunchKernelGGL((btp_subcycle_kernel<NGL, NQ, false>), dim3(e->nelem_owned),
                         dim3(StageCfg<NGL, NQ, false>::BS), e->persist_pad, e->stream, sa);
    else
      hipLaunchKernelGGL((btp_subcycle_kernel<NGL, NQ, true>), dim3(e->nelem_owned), dim3(StageCfg<NGL, NQ, true>::BS),
                         e->persist_pad, e->stream, sa);
  }
  // face traces of elements [e0, e0+n) into their neighbours' slots
  static void grad_trace(hnumo_engine *e, const double *qb, double *gt, int e0, int n, TraceGranule *gtr = nullptr) {
    if (n > 0) {
      hipLaunchKernelGGL((grad_trace_kernel<NGL, NQ>), dim3(n), dim3(64), 0, e->stream, e->m, qb, gt, e0, gtr,
                         e->epoch);
      kmark(e, "grad_trace");
    }
  }
  // extract_qprime_df_face / extract_dprime_df_face + bcl_create_communicator (ti_rk_bcl.F90:43-44,
  // :62, :75-76): processor faces take the neighbour's side 1 as their side 2
  static void extract(hnumo_engine *e, const double *qp, double *qf, int only_dp) {
    size_t n = (size_t)e->nface * NGL;
    hipLaunchKernelGGL((extract_face_kernel<NGL>), dim3((n + 255) / 256), dim3(256), 0, e->stream, e->m, qp, qf,
                       only_dp);
    kmark(e, "extract_face");
    face_exchange_qf(e, qf, only_dp ? 1 : 3);
  }
  // (qp_avg, qf_avg: the corrector's averages qp = 0.5*(qp + qp_avg), qf = 0.5*(qf_avg + qf) formed
  // and written back by the two kernels, ti_rk_bcl.F90:64-65)
  // (single rank, fused_faces: the element kernel forms the face part as well; the corrector's
  // averaged face traces then go to qf_out = e->qfa, which the rest of the corrector reads)
  static void bcl_coeffs(hnumo_engine *e, double *qp, double *qf, const double *qp_avg = nullptr,
                         const double *qf_avg = nullptr, double *qf_out = nullptr) {
    const bool fz = fused_faces(e);
    hipLaunchKernelGGL((bcl_coeffs_elem_kernel<NGL, NQ>), dim3(e->nelem), dim3(Blk<NGL, NQ>::BSW), 0, e->stream, e->m, qp,
                       qp_avg, e->qcoef, e->ncoef, e->dpp_graduv, e->dpprime_visc, e->ecoef, fz ? qf : nullptr,
                       qf_avg, qf_out, e->fcoef, e->fncoef, e->gdpp_face, e->efcoef);
    kmark(e, "bcl_coeffs_elem");
    if (!fz)
      hipLaunchKernelGGL((bcl_coeffs_face_kernel<NGL, NQ>), dim3(e->nface), dim3(64), 0, e->stream, e->m, qf, qf_avg,
                         e->dpp_graduv, e->dpprime_visc, e->fcoef, e->fncoef, e->gdpp_face, e->efcoef);
    if (!fz) kmark(e, "bcl_coeffs_face");
    if (e->face_halo) {  // graduv_dpp_face halo (mod_barotropic_terms.F90:393) and its layer sums
      face_exchange_gdpp(e);
      if (e->NS)
        hipLaunchKernelGGL((bcl_coeffs_proc_kernel<NGL, NQ>), dim3((e->NS * NGL + 63) / 64), dim3(64), 0, e->stream, e->m,
                         e->gdpp_face, e->d_sface, e->NS, e->fncoef, e->efcoef);
    }
    if (e->lapq_on)  // interpolate_dpp right after dpprime_visc is set (ti_rk_bcl.F90:48,67)
      hipLaunchKernelGGL((lapq_dpp_kernel<NGL, NQ>), dim3(std::min<size_t>(((size_t)e->L * e->npq + 255) / 256, 4096)),
                         dim3(256), 0, e->stream, e->m, e->dpprime_visc, e->dpq);
    if (e->lapq_on) kmark(e, "lapq_dpp");
  }
  // method_visc == 1, one barotropic stage: btp_create_laplacian_v2's Laplacian of state qb
  static void lapq_btp(hnumo_engine *e, const double *qb, const double *qp) {
    hipLaunchKernelGGL((lapq_flux_kernel<NGL, NQ>), dim3(e->nelem), dim3(256), 0, e->stream, e->m, qb, qp, e->nacc,
                       e->dpq, e->lq_flux, 0, 0);
    // processor faces: the neighbour's side-1 fluxes (create_communicator_quad,
    // mod_laplacian_quad.F90:214)
    const double *recv = face_exchange_lapq(e, e->lq_flux, 1, NQ, NQ * NQ);
    hipLaunchKernelGGL((lapq_apply_kernel<NGL, NQ>), dim3(e->nelem_owned, 1), dim3(64), 0, e->stream, e->m, e->lq_flux,
                       e->lapq, e->fqLR, e->fqLR + e->FQ, recv);
  }
  // method_visc == 1, baroclinic: bcl_create_laplacian_v2's per-layer Laplacians of qprime
  static void lapq_bcl(hnumo_engine *e, const double *qp) {
    hipLaunchKernelGGL((lapq_flux_kernel<NGL, NQ>), dim3(e->nelem), dim3(256), 0, e->stream, e->m, nullptr, qp,
                       e->nacc, e->dpq, e->lq_flux, 1, 0);
    // (bcl_create_communicator of flux_uv_visc_face, mod_laplacian_quad.F90:342)
    const double *recv = face_exchange_lapq(e, e->lq_flux, e->L, NQ, NQ * NQ);
    hipLaunchKernelGGL((lapq_apply_kernel<NGL, NQ>), dim3(e->nelem_owned, e->L), dim3(64), 0, e->stream, e->m,
                       e->lq_flux, e->lapq, e->fqLR, e->fqLR + e->FQ, recv);
  }
  // layer mass update (owned elements); produces dp' (e->dpp) for the consistency step
  // (q_in: the layer thicknesses entering the update; q: where they are written)
  // (single rank: the element kernels form their faces' fluxes themselves, fused_faces)
  static void mass(hnumo_engine *e, const double *qp, const double *qf, const double *q_in, double *q) {
    const bool fz = fused_faces(e);
    if (!fz)
      hipLaunchKernelGGL((mass_flux_face_kernel<NGL, NQ>), dim3(e->nface), dim3(64), 0, e->stream, e->m, qf, e->facc,
                         e->fmass, e->slmf_face);
    if (!fz) kmark(e, "mass_flux_face");
    hipLaunchKernelGGL((e->bcl_big ? mass_elem_kernel<NGL, NQ, true> : mass_elem_kernel<NGL, NQ, false>),
                       dim3(e->nelem_owned), dim3(Blk<NGL, NQ>::BSW), 0, e->stream, e->m, qp, e->qacc, e->fmass, q_in, q,
                       e->slmf, e->dpp, e->neg_flag, fz ? qf : nullptr, e->facc, e->slmf_face);
    kmark(e, "mass_elem");
  }
  // (qf: the face traces of qp_out's thickness written by cons_elem itself -- fused extract)
  static void cons(hnumo_engine *e, double *q, double *qp_out, int finalize_dp, double *qf = nullptr) {
    const bool fz = fused_faces(e);
    if (!fz)
      hipLaunchKernelGGL((cons_flux_face_kernel<NGL, NQ>), dim3(e->nface), dim3(64), 0, e->stream, e->m, e->dpp,
                         e->facc, e->slmf_face, e->fcons, e->face_halo ? e->cdef : nullptr);
    if (!fz) kmark(e, "cons_flux_face");
    if (e->face_halo) {  // mass_deficit_mass_face halo (mod_layer_terms.F90:135)
      face_exchange_cdef(e);
      if (e->NS)
        hipLaunchKernelGGL((cons_flux_proc_kernel<NQ>), dim3((e->NS * NQ + 63) / 64), dim3(64), 0, e->stream, e->m,
                         e->cdef, e->d_sface, e->NS, e->fcons);
    }
    hipLaunchKernelGGL((e->bcl_big ? cons_elem_kernel<NGL, NQ, true> : cons_elem_kernel<NGL, NQ, false>),
                       dim3(e->nelem_owned), dim3(Blk<NGL, NQ>::BSW), 0, e->stream, e->m, e->dpp, e->qacc, e->slmf,
                       e->fcons, q, qp_out, finalize_dp, qf, fz ? e->facc : nullptr, e->slmf_face);
    kmark(e, "cons_elem");
  }
  // (q_in: the momenta entering the update; mode 1 writes the final qprime, see mom_elem_kernel)
  // (qp_avg0, qf_avg0: the corrector's thickness averages of ti_rk_bcl.F90:78-80, formed by the two
  // kernels on load instead of by a launch before them; the final qprime(1) is then qp_in's own)
  static void momentum(hnumo_engine *e, const double *qf, const double *qp_in, const double *qb, const double *q_in,
                       double *q, double *qp_out, int mode, const double *qp_avg0 = nullptr,
                       const double *qf_avg0 = nullptr, double *qf_out = nullptr) {
    if (e->lapq_on) lapq_bcl(e, qp_in);
    hipLaunchKernelGGL((mom_flux_face_kernel<NGL, NQ>), dim3(e->nface), dim3(64), 0, e->stream, e->m, qf, e->facc,
                       e->gdpp_face, e->gfacc, e->momL, e->momR, e->lapf, qf_avg0);
    kmark(e, "mom_flux_face");
    hipLaunchKernelGGL((mom_elem_kernel<NGL, NQ>), dim3(e->nelem_owned), dim3(MomCfg<NGL, NQ>::BS), 0, e->stream, e->m, qp_in, e->qacc,
                       e->nacc, e->dpp_graduv, e->dpprime_visc, e->momL, e->momR, e->lapf, qb, q_in, q, qp_out, mode,
                       e->lapq_on ? e->lapq : nullptr, e->dpp2, e->neg_flag, qp_avg0, qf_out);
    kmark(e, "mom_elem");
  }
};

#define DISPATCH(eng, CALL)                                                     \
  switch ((eng)->ngl) {                                                         \
    case 3: Launch<3, 5>::CALL; break;                                          \
    case 4: Launch<4, 7>::CALL; break;                                          \
    case 5: Launch<5, 9>::CALL; break;                                          \
    case 6: Launch<6, 11>::CALL; break;                                         \
    case 8: Launch<8, 15>::CALL; break;                                         \
    default: break;                                                             \
  }

static bool supported_ngl(int ngl) { return ngl == 3 || ngl == 4 || ngl == 5 || ngl == 6 || ngl == 8; }

// ------------------------------------------------------------------ step pieces
__global__ void copy_kernel(double *dst, const double *src, size_t n) {
  const size_t s = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += s) dst[i] = src[i];
}

// non-finite guard on the barotropic state (ABI return code 2); bit 2 of the flag word
__global__ void finite_check_kernel(const double *x, size_t n, int *flag) {
  const size_t s = (size_t)gridDim.x * blockDim.x;
  bool bad = false;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += s) bad |= !isfinite(x[i]);
  if (__any(bad) && (threadIdx.x % 64) == 0) atomicOr(flag, 2);
}

// dpp2 = qp2(1); qp2(1) = 0.5*(qp(1) + dpp2) (ti_rk_bcl.F90:78-79) with, in the same launch, the
// face average of component 1: qf2(1) = 0.5*(qf(1) + qf2(1)) at stride 3 (:80)
__global__ void dp_average_face_kernel(double *qp2, const double *qp, double *dpp2, size_t n, double *qf2,
                                       const double *qf, size_t nf) {
  const size_t s = (size_t)gridDim.x * blockDim.x, t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (size_t i = t0; i < n; i += s) {
    double d = qp2[i * 3];
    dpp2[i] = d;
    qp2[i * 3] = 0.5 * (qp[i * 3] + d);
  }
  for (size_t i = t0; i < nf; i += s) qf2[i * 3] = 0.5 * (qf[i * 3] + qf2[i * 3]);
}

// ------------------------------------------------------------------ ghost exchange
// Element block of a nodal array: for each of `nblk` blocks (layers) at `blk_stride`, the
// element's P*ncomp contiguous doubles (qb(4,npoin): ncomp 4, 1 block; qprime(3,npoin,L):
// ncomp 3, L blocks of stride 3*npoin; dp'(npoin,L): ncomp 1, L blocks of stride npoin).
__global__ void ghost_pack_kernel(double *buf, const double *base, const int *elems, int nel, int per, int nblk,
                                  size_t stride) {
  const size_t n = (size_t)nel * nblk * per, s = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += s) {
    const int i = (int)(t / ((size_t)nblk * per)), r = (int)(t % ((size_t)nblk * per)), b = r / per, k = r % per;
    buf[t] = base[b * stride + (size_t)elems[i] * per + k];
  }
}
__global__ void ghost_unpack_kernel(double *base, const double *buf, const int *elems, int nel, int per, int nblk,
                                    size_t stride) {
  const size_t n = (size_t)nel * nblk * per, s = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += s) {
    const int i = (int)(t / ((size_t)nblk * per)), r = (int)(t % ((size_t)nblk * per)), b = r / per, k = r % per;
    base[b * stride + (size_t)elems[i] * per + k] = buf[t];
  }
}

// engines of one process joined by hnumo_local_group: a host barrier per exchange keeps
// every engine's pack ahead of the copies and the copies ahead of the next pack (one stream)
// An engine that fails (or is destroyed) aborts the group: every waiting engine wakes up,
// stops exchanging and reports the abort (no thread is left waiting in a barrier).  The
// group and its shared stream (created by engine 0) live until the last engine is destroyed.
struct LocalGroup {
  std::vector<hnumo_engine *> eng;
  std::mutex mu;
  std::condition_variable cv;
  int count = 0, gen = 0, refs = 0;
  bool aborted = false;
  hipStream_t stream = nullptr;
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) return false;
    int g = gen;
    if (++count == (int)eng.size()) {
      count = 0;
      gen++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g || aborted; });
    }
    return !aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
};

// RCCL results are checked at every call; the first failure is kept (sticky) and turned into
// HNUMO_ERR_DEVICE by run_steps -- a failed exchange must not pass as a good step
static void nccl_check(hnumo_engine *e, ncclResult_t r, const char *what) {
  if (r != ncclSuccess && e->comm_err.empty()) e->comm_err = std::string(what) + ": " + ncclGetErrorString(r);
}

// refresh the ghost elements' block of `base` from their owners
static void exchange(hnumo_engine *e, double *base, int ncomp, int nblk, size_t stride) {
  if (e->comm_mode == 0 || e->face_halo) return;
  const int per = e->P * ncomp;
  for (auto &n : e->nbh)
    if (n.nsend) {
      size_t tot = (size_t)n.nsend * nblk * per;
      hipLaunchKernelGGL(ghost_pack_kernel, dim3((unsigned)std::min<size_t>((tot + 255) / 256, 1024)), dim3(256), 0,
                         e->stream, n.sbuf, base, n.d_send, n.nsend, per, nblk, stride);
    }
  if (e->comm_mode == 2) {
    nccl_check(e, ncclGroupStart(), "ncclGroupStart");
    for (auto &n : e->nbh) {
      if (n.nsend)
        nccl_check(e, ncclSend(n.sbuf, (size_t)n.nsend * nblk * per, ncclDouble, n.rank, e->comm, e->stream), "ncclSend");
      if (n.nrecv)
        nccl_check(e, ncclRecv(n.rbuf, (size_t)n.nrecv * nblk * per, ncclDouble, n.rank, e->comm, e->stream), "ncclRecv");
    }
    nccl_check(e, ncclGroupEnd(), "ncclGroupEnd");
  } else {
    LocalGroup *g = e->group;
    if (!g->barrier()) return;
    for (auto &n : e->nbh) {
      if (!n.nrecv) continue;
      hnumo_engine *peer = g->eng[n.rank];
      for (auto &pn : peer->nbh)
        if (pn.rank == e->rank &&
            hipMemcpyAsync(n.rbuf, pn.sbuf, sizeof(double) * (size_t)n.nrecv * nblk * per, hipMemcpyDeviceToDevice,
                           e->stream) != hipSuccess)
          e->comm_err = "local group: hipMemcpyAsync of a ghost block failed";
    }
    if (!g->barrier()) return;
  }
  for (auto &n : e->nbh)
    if (n.nrecv) {
      size_t tot = (size_t)n.nrecv * nblk * per;
      hipLaunchKernelGGL(ghost_unpack_kernel, dim3((unsigned)std::min<size_t>((tot + 255) / 256, 1024)), dim3(256), 0,
                         e->stream, base, n.rbuf, n.d_recv, n.nrecv, per, nblk, stride);
    }
}
static void exchange_qb(hnumo_engine *e, double *qb) { exchange(e, qb, 4, 1, 0); }
static void exchange_qp(hnumo_engine *e, double *qp) { exchange(e, qp, 3, e->L, 3 * (size_t)e->npoin); }
static void exchange_dpp(hnumo_engine *e) { exchange(e, e->dpp, 1, e->L, (size_t)e->npoin); }

// ------------------------------------------------------------------ processor-face exchanges
// The peer engine of a local group holding rank r.
static hnumo_engine *group_peer(hnumo_engine *e, int r) { return e->group->eng[r]; }
// the peer's entry for my list `mine`: the peer's one entry for my rank, or -- a self-neighbour
// engine, whose lists may all name itself -- the same list
static const hnumo_engine::FNbr *peer_entry(hnumo_engine *peer, int rank, const hnumo_engine::FNbr *mine) {
  if (peer->rank == rank) return mine;
  for (auto &n : peer->fnb)
    if (n.rank == rank) return &n;
  return nullptr;
}

// (a rank without shared faces still takes part in a local group's barriers)
static bool face_tx_skip(const hnumo_engine *e) { return !e->face_halo || (e->NS == 0 && e->comm_mode != 1); }

// The source of a halo message of `n` doubles at `live` (exchange site `key`, stream st): live, or
// with hnumo_debug_frozen_halo the copy of the site's first message.  The frozen halo is an
// emulation device (bench.py --emulate of an at-rest case): a self-neighbour rank
// otherwise receives its own processor faces' traces, a zero-jump (extrapolation) boundary whose
// faces lose the upwind dissipation -- stable for the double gyre at CFL ~0.03, not for the lake
// at CFL ~1, which runs away within two steps.  Frozen, each processor face keeps receiving the
// first message, at the initial condition the same values the real neighbour sends (a continuous
// state's traces are equal from both sides: the first RHS is bit-identical to the whole mesh's,
// tools/mirror_rhs.py) -- an at-rest neighbour for a lake at rest.  Same messages, sizes, sources
// in HBM and transport calls; only their content stops following the rank's own state.
static const double *halo_src(hnumo_engine *e, const void *key, const double *live, size_t n, hipStream_t st) {
  if (!e->emu_frozen || n == 0) return live;
  for (const auto &f : e->frozen)
    if (f.key == key && f.n == n) return f.buf;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (e->capturing || (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)) {
    e->comm_err = "frozen halo: an exchange site's first message inside a graph capture (use direct launches)";
    return live;
  }
  // (not dalloc: its zero fill is a null-stream memset, unordered with this non-blocking stream's copy)
  double *d = nullptr;
  if (hipMalloc(&d, n * sizeof(double)) != hipSuccess) d = nullptr;
  if (d) e->allocs.push_back(d);
  if (!d || hipMemcpyAsync(d, live, n * sizeof(double), hipMemcpyDeviceToDevice, st) != hipSuccess) {
    e->comm_err = "frozen halo: snapshot of a message failed";
    return live;
  }
  e->frozen.push_back({key, n, d});
  return d;
}

// before packing bx_sbuf: in a local group my previous message must have been read by every peer
static void face_tx_begin(hnumo_engine *e) {
  if (e->comm_mode == 1)
    for (auto &n : e->fnb) (void)hipStreamWaitEvent(e->stream, group_peer(e, n.rank)->ev_bdone, 0);
}

// the packed messages bx_sbuf (`per` doubles per shared face, slots in nbh_send_recv order) into
// the neighbours' bx_rbuf slots of the same faces, on the engine stream
static void face_tx(hnumo_engine *e, size_t per) {
  const double *src = halo_src(e, (const void *)(uintptr_t)(1 + e->xseq++), e->bx_sbuf, per * e->NS, e->stream);
  if (e->comm_mode == 2) {
    nccl_check(e, ncclGroupStart(), "ncclGroupStart");
    for (auto &n : e->fnb) {
      nccl_check(e, ncclSend(src + per * n.off, per * n.n, ncclDouble, n.rank, e->comm, e->stream), "ncclSend");
      nccl_check(e, ncclRecv(e->bx_rbuf + per * n.off, per * n.n, ncclDouble, n.rank, e->comm, e->stream), "ncclRecv");
    }
    nccl_check(e, ncclGroupEnd(), "ncclGroupEnd");
  } else {
    (void)hipEventRecord(e->ev_bpacked, e->stream);
    if (!e->group->barrier()) return;
    for (auto &n : e->fnb) {
      hnumo_engine *peer = group_peer(e, n.rank);
      const hnumo_engine::FNbr *pn = peer_entry(peer, e->rank, &n);
      if (!pn || pn->n != n.n) {
        e->comm_err = "local group: neighbour lists of two ranks disagree";
        continue;
      }
      (void)hipStreamWaitEvent(e->stream, peer->ev_bpacked, 0);
      if (hipMemcpyAsync(e->bx_rbuf + per * n.off, (peer == e ? src : peer->bx_sbuf) + per * pn->off, per * n.n * sizeof(double),
                         hipMemcpyDeviceToDevice, e->stream) != hipSuccess)
        e->comm_err = "local group: hipMemcpyAsync of a face message failed";
    }
    (void)hipEventRecord(e->ev_bdone, e->stream);
    (void)e->group->barrier();
  }
}

// Baroclinic face exchange on the engine stream (bcl_create_communicator,
// create_rhs_communicator.F90:384-438): side 1 of every shared face -> the neighbour's side 2.
// Face array element (side 1) of layer k, component c < nc, point p < nn of face f:
// base[k*sk + c*sc + f*sf + p*sn]; side 2 at + s2.
static void face_exchange(hnumo_engine *e, double *base, int nc, int nn, size_t sk, size_t sc, size_t sf, size_t sn,
                          size_t s2) {
  if (face_tx_skip(e)) return;
  const int L = e->L;
  const size_t per = (size_t)L * nc * nn, tot = per * e->NS;
  const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>((tot + 255) / 256, 1024));
  face_tx_begin(e);
  if (tot)
    hipLaunchKernelGGL(face_pack_kernel, dim3(blocks), dim3(256), 0, e->stream, e->bx_sbuf, base, e->d_sface, e->NS,
                       L, nc, nn, sk, sc, sf, sn);
  face_tx(e, per);
  if (e->group && e->group->aborted) return;
  if (tot)
    hipLaunchKernelGGL(face_unpack_kernel, dim3(blocks), dim3(256), 0, e->stream, base, e->bx_rbuf, e->d_sface,
                       e->NS, L, nc, nn, sk, sc, sf, sn, s2);
}

// method_visc == 1: the LDG fluxes at the quad points of every processor face's local side ->
// the neighbour (create_communicator_quad, create_rhs_communicator.F90:82-134, and
// bcl_create_communicator of flux_uv_visc_face; pack_data_dg_quad, send_receive_bound.F90:215-270:
// side 1 of each listed face, quad point by quad point).  Returns the receive buffer,
// [NS][nb][4][NQ] (nb layer blocks), or NULL without processor faces.
static const double *face_exchange_lapq(hnumo_engine *e, const double *flux, int nb, int nq, int Q) {
  if (face_tx_skip(e)) return nullptr;
  const size_t per = (size_t)nb * 4 * nq, tot = per * e->NS;
  face_tx_begin(e);
  if (tot)
    hipLaunchKernelGGL(lapq_pack_kernel, dim3((unsigned)std::min<size_t>((tot + 255) / 256, 1024)), dim3(256), 0,
                       e->stream, e->bx_sbuf, flux, e->d_sface, e->m.fel, e->fqLR, e->NS, nb, e->nelem, nq, Q);
  face_tx(e, per);
  if (e->group && e->group->aborted) return nullptr;  // (as face_exchange: no message arrived)
  return e->NS ? e->bx_rbuf : nullptr;
}

// qprime_df_face-like arrays qf(3,2,ngl,F,L) (QF macro): components [0,nc)
static void face_exchange_qf(hnumo_engine *e, double *qf, int nc) {
  const size_t F = e->nface, N = e->ngl;
  face_exchange(e, qf, nc, e->ngl, F * N * 6, 1, N * 6, 6, 3);
}
// graduv_dpp_face [L][10][F*NGL]: components 0..4 (side 1) -> 5..9 (side 2)
static void face_exchange_gdpp(hnumo_engine *e) {
  face_exchange(e, e->gdpp_face, 5, e->ngl, 10 * e->FN, e->FN, e->ngl, 1, 5 * e->FN);
}
// mass_deficit_mass_face [L][side][2][F*NQ]
static void face_exchange_cdef(hnumo_engine *e) {
  face_exchange(e, e->cdef, 2, e->nq, 4 * e->FQ, e->FQ, e->nq, 1, 2 * e->FQ);
}

// Stage-trace exchange (btp_create_pre/postcommunicator + create_rhs_lap_pre/postcommunicator_df,
// one message for both: qb(4) and grad(u_bar)(4) at the face nodes) on stream `st`: the send
// slots [4E, 4E+NS) of trace buffer `tb` go to the neighbours' receive slots [4E+NS, 4E+2NS).
static void trace_exchange(hnumo_engine *e, double *tb, hipStream_t st) {
  if (!e->face_halo || (e->NS == 0 && e->comm_mode != 1)) return;
  const size_t slot = 8 * (size_t)e->ngl, s0 = 4 * (size_t)e->nelem, r0 = s0 + e->NS;
  const double *src = halo_src(e, tb, tb + s0 * slot, slot * e->NS, st);  // = the send slots
  if (e->comm_mode == 2) {
    nccl_check(e, ncclGroupStart(), "ncclGroupStart");
    for (auto &n : e->fnb) {
      nccl_check(e, ncclSend(src + n.off * slot, slot * n.n, ncclDouble, n.rank, e->comm, st), "ncclSend");
      nccl_check(e, ncclRecv(tb + (r0 + n.off) * slot, slot * n.n, ncclDouble, n.rank, e->comm, st), "ncclRecv");
    }
    nccl_check(e, ncclGroupEnd(), "ncclGroupEnd");
    return;
  }
  // local group: every engine runs the same stage sequence, so the peer's buffer of the same
  // index holds the traces of the same stage
  const int bi = tb == e->gtrace[0] ? 0 : 1;
  (void)hipEventRecord(e->ev_tsent, st);
  if (!e->group->barrier()) return;
  for (auto &n : e->fnb) {
    hnumo_engine *peer = group_peer(e, n.rank);
    const hnumo_engine::FNbr *pn = peer_entry(peer, e->rank, &n);
    if (!pn || pn->n != n.n) {
      e->comm_err = "local group: neighbour lists of two ranks disagree";
      continue;
    }
    (void)hipStreamWaitEvent(st, peer->ev_tsent, 0);
    if (hipMemcpyAsync(tb + (r0 + n.off) * slot, (peer == e ? src + pn->off * slot : peer->gtrace[bi] + (4 * (size_t)peer->nelem + pn->off) * slot),
                       slot * n.n * sizeof(double), hipMemcpyDeviceToDevice, st) != hipSuccess)
      e->comm_err = "local group: hipMemcpyAsync of a trace message failed";
  }
  (void)e->group->barrier();
}


static void launch_copy(hnumo_engine *e, double *dst, const double *src, size_t n) {
  (void)hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToDevice, e->stream);
}

// Sub-cycle prologue (mod_rk_mlswe.F90:45-72): zero the time averages, copy the state into
// stage buffer 0 and bump the persistent kernel's epoch -- one launch instead of four memsets,
// a copy and a one-thread kernel (each a graph node of ~4 us at this size).
__global__ void subcycle_prologue_kernel(double *qacc, size_t nqa, double *facc, size_t nfa, double *nacc, size_t nna,
                                         double *gfacc, size_t nga, double *qbuf0, const double *qb, size_t nqb,
                                         unsigned long long *epoch) {
  const size_t s = (size_t)gridDim.x * blockDim.x, t0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (size_t i = t0; i < nqa; i += s) qacc[i] = 0.0;
  for (size_t i = t0; i < nfa; i += s) facc[i] = 0.0;
  for (size_t i = t0; i < nna; i += s) nacc[i] = 0.0;
  for (size_t i = t0; i < nga; i += s) gfacc[i] = 0.0;
  for (size_t i = t0; i < nqb; i += s) qbuf0[i] = qb[i];
  if (epoch && t0 == 0) *epoch = *epoch + 1;
}

// (zero_acc false: the persistent kernel writes every average itself, StageCfg::REGACC)
static void subcycle_prologue(hnumo_engine *e, const double *qb_state, unsigned long long *epoch, bool zero_acc) {
  const size_t z = zero_acc ? 1 : 0;
  const size_t nqa = z * QA_N * (size_t)e->npq, nfa = z * FA_N * 4 * (size_t)e->nelem * e->nq;
  const int blocks = (int)std::min<size_t>((std::max<size_t>(nqa, 4 * (size_t)e->npoin) + 255) / 256, 2048);
  hipLaunchKernelGGL(subcycle_prologue_kernel, dim3(blocks), dim3(256), 0, e->stream, e->qacc, nqa, e->facc, nfa,
                     e->nacc, z * NA_N * (size_t)e->npoin, e->gfacc, z * 8 * 4 * (size_t)e->nelem * e->ngl,
                     e->qbuf[0], qb_state, 4 * (size_t)e->npoin, epoch);
  kmark(e, "subcycle_prologue");
}

static void launch_bcl_coeffs(hnumo_engine *e, double *qp, double *qf) {
  if (!fused_extract(e)) DISPATCH(e, extract(e, qp, qf, 0));
  DISPATCH(e, bcl_coeffs(e, qp, qf));
}

// The stages of one sub-cycle: Shu-Osher coefficients and the rotation of the four state
// buffers (input, stage-0 state, stage-2 state of the 5-stage scheme, output) and of the two
// trace buffers.  Returns the buffer holding the result.
static int stage_table(hnumo_engine *e, const double *qp, std::vector<StageArgs> &out_args) {
  int cur = 0, gt = 0, qb0i = 0, qb2i = -1;
  const int K = e->K, NB = e->p.N_btp;
  out_args.clear();
  for (int mstep = 0; mstep < NB; mstep++) {
    qb0i = cur;
    qb2i = -1;
    for (int ik = 0; ik < K; ik++) {
      int out = 0;
      while (out == cur || out == qb0i || out == qb2i) out++;
      StageArgs a{};
      a.m = e->m;
      a.qb_in = e->qbuf[cur];
      a.qb0 = e->qbuf[qb0i];
      a.qb2 = qb2i >= 0 ? e->qbuf[qb2i] : e->qbuf[cur];
      a.qprime = qp;
      a.ecoef = e->ecoef;
      a.efcoef = e->efcoef;
      a.trace_in = e->gtrace[gt];
      a.trace_out = e->gtrace[1 - gt];
      a.qacc = e->qacc;
      a.facc = e->facc;
      a.nacc = e->nacc;
      a.gfacc = e->gfacc;
      a.qb_out = e->qbuf[out];
      a.rhs_out = nullptr;
      a.a1 = e->ssprk_a[ik + 0 * K];
      a.a2 = e->ssprk_a[ik + 1 * K];
      a.a3 = e->ssprk_a[ik + 2 * K];
      a.dtt = e->p.dt_btp * e->ssprk_beta[ik];
      a.rhs_only = 0;
      a.write_trace = !(mstep == NB - 1 && ik == K - 1);
      a.accumulate = !(e->stage_dbg & 32);  // dbg bit 32: no time averages (timing experiments)
      // the sub-cycle's first stage stores its time-average terms (acc_put), so the slots need no
      // zeroing before it -- except with the quad-point LDG (method_visc == 1), whose stages leave
      // the graduvb slots to lapq kernels
      if (out_args.empty() && a.accumulate && !e->lapq_on && !e->acc_zero) a.accumulate = 2;
      a.prof = e->stage_prof;
      a.dbg = e->stage_dbg;
      const int stage = (int)out_args.size();
      a.gtr_in = e->gtr[gt];
      a.gtr_out = e->gtr[1 - gt];
      a.tag_in = (unsigned long long)stage + 1;
      a.tag_out = (unsigned long long)stage + 2;
      a.first_of_step = ik == 0;
      a.save_q2 = K == 5 && ik == 2;
      a.err = e->neg_flag;
      a.lapq = e->lapq_on ? e->lapq : nullptr;
      a.qpq = e->qpq;
      a.qpq_mode = stage == 0 ? 1 : 2;
      a.qsv = e->qsv;
      a.n_inv = 1.0 / (double)(K * NB);
      out_args.push_back(a);
      gt = 1 - gt;
      cur = out;
      if (K == 5 && ik == 1) qb2i = out;
    }
  }
  return cur;
}

// (method_visc == 1 needs its Laplacian kernels between the stages: per-stage launches)
// (single rank only: its stage tables send every trace to an element slot)
static bool use_persistent(const hnumo_engine *e) {
  return e->comm_mode == 0 && e->nranks == 1 && !e->face_halo && !e->lapq_on && e->persistent_ok[e->summation] &&
         !e->persist_suspended;
}

// ti_barotropic_ssprk_mlswe (mod_rk_mlswe.F90:19-151) on device state qb_state
// ti_barotropic_ssprk_mlswe (mod_rk_mlswe.F90:19-151) from the step-start state e->qb (both
// sub-cycles of a step start from it, ti_rk_bcl.F90:50,71) into dst: e->qbp (predictor, qp =
// e->qp) or e->qb (corrector, qp = e->qp2).  The persistent kernel's stage tables read e->qb
// and write dst themselves; with the averages in registers (REGACC) nothing else runs around it.
static void launch_subcycle(hnumo_engine *e, double *dst, const double *qp, bool timed = false) {
  const int tab = (dst == e->qbp && qp == e->qp) ? 0 : ((dst == e->qb && qp == e->qp2) ? 1 : -1);
  const bool pers = use_persistent(e) && tab >= 0;
  // persistent with register averages: the kernel writes them, zeroed and scaled as below
  const bool racc = pers && e->regacc[e->summation] && !(e->stage_dbg & 32);
  // (the first stage stores the time averages unless method_visc == 1: no zeroing, StageArgs::accumulate)
  if (!racc) subcycle_prologue(e, e->qb, nullptr, e->lapq_on || e->acc_zero);
  if (!pers) exchange_qb(e, e->qbuf[0]);
  if (!pers) DISPATCH(e, grad_trace(e, e->qbuf[0], e->gtrace[0], 0, e->nelem));  // (persistent: its stage 0)
  const int K = e->K, NB = e->p.N_btp;
  int cur;
  if (pers) {
    if (timed && e->kernel_events) (void)hipEventRecord(e->evk0, e->stream);
    DISPATCH(e, subcycle(e, e->d_stages[tab], K * NB));
    kmark(e, "btp_subcycle");
    if (timed && e->kernel_events) (void)hipEventRecord(e->evk1, e->stream);
    if (racc) return;
    cur = -1;  // (the last stage wrote dst)
  } else if (e->face_halo && !e->lapq_on) {
    // Processor-face halo, two streams (the overlap of mod_rhs_btp.F90:40-46): elements with a
    // processor face ("boundary", B) run on stream2, which then ships their new face traces to
    // the neighbours; the interior elements (I) run on the engine stream meanwhile.  Stage s:
    //   B_s waits for I_{s-1} (its interior neighbours' traces); the transport of stage s-1
    //       precedes it on stream2;
    //   I_s waits for B_{s-1} only -- never for the transport, which overlaps I_s.
    trace_exchange(e, e->gtrace[0], e->stream);  // the sub-cycle input's traces (grad_trace above)
    std::vector<StageArgs> st;
    cur = stage_table(e, qp, st);
    if (timed && e->kernel_events) (void)hipEventRecord(e->evk0, e->stream);
    // (stop events: each launch signals its own completion, no record packet between the
    // interior launches; HNUMO_SCHED_DBG 2, diagnostics builds, restores the recorded events for A/B)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    (void)hipStreamIsCapturing(e->stream, &cap);
    const bool sev = !(e->sched_dbg & 2) && e->ev_Bs[0] && cap == hipStreamCaptureStatusNone;
    // ev_fork orders stream2 after the sub-cycle input's traces (grad_trace, trace_exchange above):
    // that is B_0's whole dependency, so B_0 waits for nothing else
    (void)hipEventRecord(e->ev_fork, e->stream);
    (void)hipStreamWaitEvent(e->stream2, e->ev_fork, 0);
    if (!sev) (void)hipEventRecord(e->ev_I, e->stream);
    for (size_t i = 0; i < st.size(); i++) {
      StageArgs a = st[i];
      if (i > 0 || !sev) (void)hipStreamWaitEvent(e->stream2, sev ? e->ev_Is : e->ev_I, 0);
      a.elist = e->d_elB;
      DISPATCH(e, stage(e, a, e->nB, e->stream2, sev ? e->ev_Bs[i & 1] : nullptr));
      if (!sev) (void)hipEventRecord(e->ev_B[i & 1], e->stream2);
      if (i > 0 && !(e->sched_dbg & 1))
        (void)hipStreamWaitEvent(e->stream, sev ? e->ev_Bs[(i - 1) & 1] : e->ev_B[(i - 1) & 1], 0);
      const StageArgs aB = a;
      a.elist = e->d_elI;
      a.tcontig = 1;  // (interior elements: trace slots 4e..4e+3, StageArgs::tcontig)
      DISPATCH(e, stage(e, a, e->nI, e->stream, sev ? e->ev_Is : nullptr));
      if (!sev) (void)hipEventRecord(e->ev_I, e->stream);
      // the transport of B_s's traces, enqueued after I_s (stream2 after B_s as before; the order of
      // the host calls only): RCCL's enqueue can hold the host until an earlier transport has
      // finished -- at the end of the interior launch it overlaps -- and I_s must be queued by then,
      // or every stage waits for the host to queue it (~10 us a stage on the C4/8 rank, r05q)
      if (aB.write_trace) trace_exchange(e, aB.trace_out, e->stream2);
    }
    (void)hipEventRecord(e->ev_join, e->stream2);
    (void)hipStreamWaitEvent(e->stream, e->ev_join, 0);
    if (timed && e->kernel_events) (void)hipEventRecord(e->evk1, e->stream);
  } else {
    // one stream: a single rank, the ghost-element halo, or the processor-face halo with the
    // quad-point LDG (method_visc == 1), whose per-stage Laplacian needs the neighbours' face
    // fluxes of the stage (create_communicator_quad) before any element's stage can run
    if (e->face_halo) trace_exchange(e, e->gtrace[0], e->stream);  // the sub-cycle input's traces
    std::vector<StageArgs> st;
    cur = stage_table(e, qp, st);
    if (timed && e->kernel_events) (void)hipEventRecord(e->evk0, e->stream);
    for (const StageArgs &a : st) {
      if (e->lapq_on) DISPATCH(e, lapq_btp(e, a.qb_in, a.qprime));
      DISPATCH(e, stage(e, a));
      kmark(e, "btp_stage");
      if (a.write_trace && e->face_halo) {
        trace_exchange(e, a.trace_out, e->stream);
      } else if (a.write_trace && e->comm_mode) {
        // ghosts take the owners' new state; their traces go into the owned elements' slots
        exchange_qb(e, a.qb_out);
        DISPATCH(e, grad_trace(e, a.qb_out, a.trace_out, e->nelem_owned, e->nelem - e->nelem_owned));
      }
    }
    if (timed && e->kernel_events) (void)hipEventRecord(e->evk1, e->stream);
  }
  int nblk = 1024;
  hipLaunchKernelGGL(btp_finalize_kernel, dim3(nblk), dim3(256), 0, e->stream, e->qacc, e->facc, e->nacc, e->gfacc,
                     e->tau_wind_ave, e->tau_wind, e->npq, 4 * e->nelem * e->nq, e->npoin, 4 * e->nelem * e->ngl, NB,
                     1.0 / (double)(K * NB), dst, cur >= 0 ? e->qbuf[cur] : dst, 1);
  kmark(e, "btp_finalize");
}

// the prediction half of ti_rk_bcl (ti_rk_bcl.F90:43-57) on device state (e->q, e->qb, e->qp):
// results in e->q2 (q_df2), e->qbp (qb after the sub-cycle), e->qp2 (qprime_df2)
static void launch_predict(hnumo_engine *e) {
  e->xseq = 0;  // (every step starts here: its baroclinic exchanges' sites, see halo_src)
  launch_bcl_coeffs(e, e->qp, e->qf);
  launch_subcycle(e, e->qbp, e->qp);
  // (q_df2 = q_df, qprime_df2 = qprime_df, qprime_face2 = qprime_face (ti_rk_bcl.F90:53-55) without
  // copies: the predictor's kernels read q_df, qprime_df and qprime_face and write q_df2 and
  // qprime_df2 in full -- thicknesses by momentum_mass' mass and consistency updates, momenta and
  // qprime by its momentum update -- before anything reads them)
  DISPATCH(e, mass(e, e->qp, e->qf, e->q, e->q2));
  exchange_dpp(e);
  DISPATCH(e, cons(e, e->q2, nullptr, 0));
  DISPATCH(e, momentum(e, e->qf, e->qp, e->qbp, e->q, e->q2, e->qp2, 0, nullptr, nullptr,
                       fused_extract(e) ? e->qf2 : nullptr));
  exchange_qp(e, e->qp2);
}

// the full ti_rk_bcl on device state (e->q, e->qb, e->qp)
static void launch_step(hnumo_engine *e) {
  const size_t n3 = 3 * (size_t)e->npoin * e->L, nf = 6 * e->FN * e->L, nl = (size_t)e->npoin * e->L;
  int blocks = (int)std::min<size_t>((nl + 255) / 256, 4096);
  const bool fx = fused_extract(e);
  launch_predict(e);
  if (!fx) DISPATCH(e, extract(e, e->qp2, e->qf2, 0));
  // correction (ti_rk_bcl.F90:62-85); qfc = the averaged qprime_face2 (fused faces: e->qfa)
  double *qfc = fused_faces(e) ? e->qfa : e->qf2;
  DISPATCH(e, bcl_coeffs(e, e->qp2, e->qf2, e->qp, e->qf, qfc == e->qf2 ? nullptr : qfc));
  launch_subcycle(e, e->qb, e->qp2, true);
  DISPATCH(e, mass(e, e->qp2, qfc, e->q, e->q));
  exchange_dpp(e);
  DISPATCH(e, cons(e, e->q, e->qp2, 1, fx ? qfc : nullptr));
  exchange_qp(e, e->qp2);
  if (!fx) DISPATCH(e, extract(e, e->qp2, qfc, 1));
  // (the corrector's momentum update writes the final qprime_df -- thickness dpp2, momenta of
  // evaluate_bcl_v1 -- and checks the barotropic state, ti_rk_bcl.F90:81-84; the thickness averages
  // of :78-80 are formed by its kernels on load, except with the quad-point LDG Laplacian, which
  // reads the averaged qprime before them)
  if (e->lapq_on) {
    hipLaunchKernelGGL(dp_average_face_kernel, dim3(blocks), dim3(256), 0, e->stream, e->qp2, e->qp, e->dpp2, nl,
                       qfc, e->qf, nf / 3);
    DISPATCH(e, momentum(e, qfc, e->qp2, e->qb, e->q, e->q, e->qp, 1, nullptr, nullptr, fx ? e->qf : nullptr));
  } else {
    DISPATCH(e, momentum(e, qfc, e->qp2, e->qb, e->q, e->q, e->qp, 1, e->qp, e->qf, fx ? e->qf : nullptr));
  }
  exchange_qp(e, e->qp);
  // ad_mlswe > 0 with the reference's corrector input leaves NaN layer momenta (hnumo_params)
  if (e->p.ad_mlswe > 0.0)
    hipLaunchKernelGGL(finite_check_kernel, dim3(256), dim3(256), 0, e->stream, e->q, n3, e->neg_flag);
}

// ------------------------------------------------------------------ C ABI
extern "C" {

int hnumo_abi_version(void) { return HNUMO_ABI_VERSION; }

int hnumo_overrides(const hnumo_engine *eng, char *out, int64_t len) {
  if (!eng || !out || len <= 0) return HNUMO_ERR_INVALID;
  const size_t n = std::min((size_t)len - 1, eng->overrides.size());
  std::memcpy(out, eng->overrides.data(), n);
  out[n] = 0;
  return eng->overrides.size() < (size_t)len ? HNUMO_OK : HNUMO_ERR_INVALID;
}

const char *hnumo_last_error(const hnumo_engine *eng) { return eng ? eng->err.c_str() : "null engine"; }

void hnumo_engine_destroy(hnumo_engine *eng) {
  if (!eng) return;
  (void)hipSetDevice(eng->device);
  if (eng->graph_exec) (void)hipGraphExecDestroy(eng->graph_exec);
  if (eng->graph) (void)hipGraphDestroy(eng->graph);
  for (void *ptr : eng->allocs) (void)hipFree(ptr);
  if (eng->h_neg) (void)hipHostFree(eng->h_neg);
  if (eng->h_steps) (void)hipHostFree(eng->h_steps);
  if (eng->stream && eng->own_stream) (void)hipStreamDestroy(eng->stream);
  if (LocalGroup *g = eng->group) {
    // the destroyed engine cannot take part in exchanges any more; the last one out frees
    // the group and the shared stream
    g->abort();
    bool last;
    {
      std::lock_guard<std::mutex> lk(g->mu);
      last = --g->refs == 0;
    }
    if (last) {
      if (g->stream) (void)hipStreamDestroy(g->stream);
      delete g;
    }
  }
  if (eng->comm) (void)ncclCommDestroy(eng->comm);
  if (eng->ev0) (void)hipEventDestroy(eng->ev0);
  if (eng->ev1) (void)hipEventDestroy(eng->ev1);
  if (eng->evk0) (void)hipEventDestroy(eng->evk0);
  if (eng->evk1) (void)hipEventDestroy(eng->evk1);
  for (hipEvent_t ev : {eng->ev_Is, eng->ev_Bs[0], eng->ev_Bs[1]})
    if (ev) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : {eng->ev_fork, eng->ev_join, eng->ev_I, eng->ev_B[0], eng->ev_B[1], eng->ev_tsent,
                        eng->ev_bpacked, eng->ev_bdone})
    if (ev) (void)hipEventDestroy(ev);
  if (eng->stream2) (void)hipStreamDestroy(eng->stream2);
  delete eng;
}

static int fail(hnumo_engine *eng, int code, const std::string &msg) {
  eng->err = msg;
  return code;
}

int hnumo_engine_create(const hnumo_mesh_desc *mesh, const hnumo_static_desc *st, const hnumo_params *par,
                        const hnumo_halo_desc *halo, int device, hnumo_engine **out) {
  hnumo_engine *eng = new hnumo_engine();
  *out = eng;
  eng->device = device;
  if (!mesh || !st || !par) return fail(eng, HNUMO_ERR_INVALID, "null descriptor");
  // multi-rank: the reference's processor-face lists (num_send_recv / nbh_send_recv), or the
  // ghost-element lists (num_ghost_send / num_ghost_recv) -- one of the two
  std::vector<int> sface;                 // processor-face halo: shared slot -> local face
  std::vector<int> face_slot(mesh->nface > 0 ? mesh->nface : 0, -1);
  // (nranks == 1 with processor-face lists: the self-neighbour test contract -- every listed face
  // is shared with this rank itself, so each receives its own side 1 as side 2 over the same
  // transport code as a real neighbour's; tests/test_rccl_self_gpu.py)
  if (halo && (halo->nranks > 1 || halo->num_nbh > 0)) {
    if (halo->rank < 0 || halo->rank >= halo->nranks) return fail(eng, HNUMO_ERR_INVALID, "bad rank");
    bool any_face = false, any_ghost = false;
    for (int k = 0; k < halo->num_nbh; k++) {
      if (halo->num_send_recv && halo->num_send_recv[k] > 0) any_face = true;
      if ((halo->num_ghost_send && halo->num_ghost_send[k] > 0) || (halo->num_ghost_recv && halo->num_ghost_recv[k] > 0))
        any_ghost = true;
    }
    if (any_face && any_ghost)
      return fail(eng, HNUMO_ERR_INVALID, "give either processor-face lists or ghost-element lists, not both");
    if (any_face) {
      eng->face_halo = true;
      if (halo->nelem_owned != 0 && halo->nelem_owned != mesh->nelem)
        return fail(eng, HNUMO_ERR_INVALID, "processor-face halo: every local element is owned (nelem_owned = nelem)");
      if (!halo->nbh_proc || !halo->num_send_recv || !halo->nbh_send_recv)
        return fail(eng, HNUMO_ERR_INVALID, "processor-face halo needs nbh_proc, num_send_recv, nbh_send_recv");
      size_t o = 0;
      for (int k = 0; k < halo->num_nbh; k++) {
        hnumo_engine::FNbr nb;
        nb.rank = halo->nbh_proc[k] - 1;  // mod_parallel nbh_proc is 1-based (p4est.c:1357)
        nb.off = (int)sface.size();
        nb.n = halo->num_send_recv[k];
        if (nb.rank < 0 || nb.rank >= halo->nranks || (nb.rank == halo->rank && halo->nranks > 1))
          return fail(eng, HNUMO_ERR_INVALID, "nbh_proc: bad neighbour rank (1-based ranks expected)");
        // mod_parallel lists each neighbour process once (p4est.c:1343-1360); the transports pair a
        // rank's message with the peer's one entry for it.  The one exception is the self-neighbour
        // contract (nranks == 1): a W-rank partition's rank emulated on one GPU may keep its real
        // per-neighbour lists, every one addressed to itself -- one ncclSend/ncclRecv pair per list
        // inside the group (RCCL matches same-peer operations in issue order), each list's message
        // at its own offset and size, as on the W-GPU run
        if (halo->nranks > 1)
          for (const auto &pn : eng->fnb)
            if (pn.rank == nb.rank) return fail(eng, HNUMO_ERR_INVALID, "nbh_proc: a neighbour rank is listed twice");
        if (nb.n < 0) return fail(eng, HNUMO_ERR_INVALID, "num_send_recv < 0");
        for (int i = 0; i < nb.n; i++) {
          const int f = halo->nbh_send_recv[o + i] - 1;
          if (f < 0 || f >= mesh->nface) return fail(eng, HNUMO_ERR_INVALID, "nbh_send_recv: face id out of range");
          if (mesh->face[8 * f + 7] != 0)
            return fail(eng, HNUMO_ERR_INVALID, "nbh_send_recv lists a face whose face(8) is not 0 (not a processor face)");
          if (face_slot[f] >= 0)
            return fail(eng, HNUMO_ERR_INVALID,
                        "a processor face is listed twice (non-conforming multiplicity > 1 is not supported)");
          face_slot[f] = (int)sface.size();
          sface.push_back(f);
        }
        o += nb.n;
        eng->fnb.push_back(nb);
      }
      eng->NS = (int)sface.size();
    } else {
      if (halo->nranks < 2) return fail(eng, HNUMO_ERR_INVALID, "ghost-element lists need nranks > 1");
      if (halo->nelem_owned < 1 || halo->nelem_owned > mesh->nelem)
        return fail(eng, HNUMO_ERR_INVALID, "nelem_owned must be in 1..nelem (owned elements first)");
    }
  }
  if (par->method_visc == 1) {
    if (!mesh->imapl_q || !mesh->imapr_q) return fail(eng, HNUMO_ERR_INVALID, "method_visc==1 needs imapl_q/imapr_q");
    if (halo && halo->nranks > 1 && !eng->face_halo)
      return fail(eng, HNUMO_ERR_INVALID,
                  "method_visc==1 (quad-point LDG) runs on one rank or on the processor-face halo, not on ghost elements");
  }
  if (par->shear_corrector != HNUMO_SHEAR_CORRECTOR_REFERENCE && par->shear_corrector != HNUMO_SHEAR_CORRECTOR_PREDICTED)
    return fail(eng, HNUMO_ERR_INVALID, "shear_corrector must be HNUMO_SHEAR_CORRECTOR_REFERENCE or _PREDICTED");
  if (mesh->nlayers < 1 || mesh->nlayers > MAXL)
    return fail(eng, HNUMO_ERR_INVALID, "nlayers must be 1..3 (qp(k) quirk, mod_create_rhs_mlswe.F90:382)");
  if (!supported_ngl(mesh->ngl) || mesh->nq != 2 * mesh->ngl - 1)
    return fail(eng, HNUMO_ERR_INVALID, "unsupported polynomial order (N in {2,3,4,5,7}, nq=2N+1)");
  if (par->kstages < 1 || par->kstages > 5 || par->N_btp < 1) return fail(eng, HNUMO_ERR_INVALID, "bad kstages/N_btp");
  HIPCHK(hipSetDevice(device));
  HIPCHK(hipStreamCreateWithFlags(&eng->stream, hipStreamNonBlocking));
  HIPCHK(hipEventCreate(&eng->ev0));
  HIPCHK(hipEventCreate(&eng->ev1));
  eng->p = *par;
  const int E = mesh->nelem, ngl = mesh->ngl, nq = mesh->nq, F = mesh->nface, L = mesh->nlayers;
  const int P = ngl * ngl, Q = nq * nq;
  if (mesh->npoin != E * P || mesh->npoin_q != E * Q) return fail(eng, HNUMO_ERR_INVALID, "npoin/npoin_q mismatch");
  eng->nelem = E; eng->npoin = E * P; eng->npq = E * Q; eng->nface = F; eng->ngl = ngl; eng->nq = nq;
  eng->L = L; eng->P = P; eng->Q = Q; eng->K = par->kstages;
  eng->nelem_owned = (halo && halo->nranks > 1 && !eng->face_halo) ? halo->nelem_owned : E;
  const int EO = eng->nelem_owned;
  eng->FQ = (size_t)F * nq; eng->FN = (size_t)F * ngl;
  const size_t npoin = eng->npoin, npq = eng->npq, FQ = eng->FQ, FN = eng->FN;

  // ---- element -> face connectivity from the reference face arrays
  std::vector<std::vector<std::pair<int, int>>> ef(E);
  for (int f = 0; f < F; f++) {
    int el = mesh->face[8 * f + 6] - 1, er = mesh->face[8 * f + 7];
    if (el < 0 || el >= E) return fail(eng, HNUMO_ERR_INVALID, "face(7) out of range");
    ef[el].push_back({f, 0});
    if (er > 0) {
      if (er > E) return fail(eng, HNUMO_ERR_INVALID, "face(8) out of range");
      ef[er - 1].push_back({f, 1});
    } else if (er == 0 && face_slot[f] < 0) {
      return fail(eng, HNUMO_ERR_INVALID,
                  "face(8) = 0 (processor face) but the face is not in the halo's nbh_send_recv lists");
    }
  }
  auto lnode = [&](const int32_t *imap, int f, int n) {
    int i = imap[3 * (n + ngl * f)] - 1, j = imap[3 * (n + ngl * f) + 1] - 1;
    return j * ngl + i;
  };
  std::vector<int> efaces(4 * E), eside(4 * E), ebc(4 * E), efmap(4 * E * ngl), enbr_node(4 * E * ngl, -1);
  std::vector<int> enbr_e(4 * E, -1), enbr_lf(4 * E, -1), fnodeL(FN), fnodeR(FN, -1), fel(F), fer(F);
  for (int e = 0; e < E; e++) {
    if (ef[e].size() != 4) return fail(eng, HNUMO_ERR_INVALID, "every element needs exactly 4 faces");
    std::sort(ef[e].begin(), ef[e].end());
  }
  for (int e = 0; e < E; e++)
    for (int lf = 0; lf < 4; lf++) {
      int f = ef[e][lf].first, s = ef[e][lf].second;
      int el = mesh->face[8 * f + 6] - 1, er = mesh->face[8 * f + 7];
      efaces[4 * e + lf] = f;
      eside[4 * e + lf] = s;
      ebc[4 * e + lf] = er;
      for (int n = 0; n < ngl; n++) efmap[(4 * e + lf) * ngl + n] = lnode(s == 0 ? mesh->imapl : mesh->imapr, f, n);
      if (er > 0) {
        int nb = s == 0 ? er - 1 : el;
        enbr_e[4 * e + lf] = nb;
        for (int k = 0; k < 4; k++)
          if (ef[nb][k].first == f) enbr_lf[4 * e + lf] = k;
        for (int n = 0; n < ngl; n++)
          enbr_node[(4 * e + lf) * ngl + n] = nb * P + lnode(s == 0 ? mesh->imapr : mesh->imapl, f, n);
      } else if (er == 0) {
        // processor face: the stage writes this face's traces into send slot 4E + s of the
        // trace buffer, i.e. "element" E + s/4, local face s%4
        const int sl = face_slot[f];
        enbr_e[4 * e + lf] = E + sl / 4;
        enbr_lf[4 * e + lf] = sl % 4;
      }
    }
  for (int f = 0; f < F; f++) {
    int el = mesh->face[8 * f + 6] - 1, er = mesh->face[8 * f + 7];
    fel[f] = el;
    fer[f] = er;
    for (int n = 0; n < ngl; n++) {
      fnodeL[(size_t)f * ngl + n] = el * P + lnode(mesh->imapl, f, n);
      if (er > 0) fnodeR[(size_t)f * ngl + n] = (er - 1) * P + lnode(mesh->imapr, f, n);
    }
  }
  // face -> element-side slots; per-element int records for the stage kernel
  std::vector<int> fslotL(F, -1), fslotR(F, -1), fslotA(F, -1);
  for (int e = 0; e < E; e++)
    for (int lf = 0; lf < 4; lf++) (eside[4 * e + lf] == 0 ? fslotL : fslotR)[efaces[4 * e + lf]] = 4 * e + lf;
  // face averages are kept by the left element, or by the right one when the left is a ghost
  for (int f = 0; f < F; f++) {
    const int el = fel[f], er = fer[f];
    fslotA[f] = (el >= EO && er > 0 && er - 1 < EO) ? fslotR[f] : fslotL[f];
  }
  const int ERS = EREC_SIZE(ngl);
  std::vector<int> erec((size_t)E * ERS, -1);
  for (int e = 0; e < E; e++) {
    int *r = &erec[(size_t)e * ERS];
    for (int lf = 0; lf < 4; lf++) {
      r[EREC_FACE + lf] = efaces[4 * e + lf];
      r[EREC_SIDE + lf] = eside[4 * e + lf];
      r[EREC_BC + lf] = ebc[4 * e + lf];
      r[EREC_NBE + lf] = enbr_e[4 * e + lf];
      r[EREC_NBLF + lf] = enbr_lf[4 * e + lf];
      r[EREC_ACC + lf] = fslotA[efaces[4 * e + lf]] == 4 * e + lf ? 1 : 0;
      for (int n = 0; n < ngl; n++) r[EREC_MAP + lf * ngl + n] = efmap[(4 * e + lf) * ngl + n];
      if (ebc[4 * e + lf] > 0) {
        // the stage kernel writes face traces into the neighbour's slot with the same face-node index
        const int nb = enbr_e[4 * e + lf], nlf = enbr_lf[4 * e + lf];
        for (int n = 0; n < ngl; n++)
          if (enbr_node[(4 * e + lf) * ngl + n] != nb * P + efmap[(4 * nb + nlf) * ngl + n])
            return fail(eng, HNUMO_ERR_INVALID, "face node orderings of neighbouring elements disagree");
      }
    }
    for (int lf = 0; lf < 4; lf++)
      for (int n = 0; n < ngl; n++) {
        int *pf = &r[EREC_PF(ngl) + 2 * efmap[(4 * e + lf) * ngl + n]];
        if (pf[0] < 0) pf[0] = lf * ngl + n; else if (pf[1] < 0) pf[1] = lf * ngl + n;
        else return fail(eng, HNUMO_ERR_INVALID, "a node lies on more than two faces of its element");
      }
  }
  eng->fslotA = fslotA;
  std::vector<int> conn;
  auto append = [&](const std::vector<int> &v) {
    size_t off = conn.size();
    conn.insert(conn.end(), v.begin(), v.end());
    return off;
  };
  size_t o_ef = append(efaces), o_es = append(eside), o_eb = append(ebc), o_em = append(efmap);
  size_t o_en = append(enbr_node), o_ee = append(enbr_e), o_el = append(enbr_lf), o_fl = append(fnodeL);
  size_t o_fr = append(fnodeR), o_fe = append(fel), o_fer = append(fer);
  size_t o_sl = append(fslotL), o_sr = append(fslotR), o_sa = append(fslotA), o_er = append(erec);
  eng->iconn = dalloc<int>(eng, conn.size());
  if (!eng->iconn) return fail(eng, HNUMO_ERR_DEVICE, "hipMalloc failed");
  HIPCHK(hipMemcpy(eng->iconn, conn.data(), conn.size() * sizeof(int), hipMemcpyHostToDevice));

  // ---- statics
  // (+ the stage kernel's interleaved copy, basis_pd: 16-byte aligned, the counts above are even)
  const size_t nb0 = 2 * (size_t)ngl * nq + 2 * (size_t)ngl * ngl;
  std::vector<double> hb(nb0 + 2 * ngl * nq + ngl * ngl);
  for (int n = 0; n < ngl; n++)
    for (int iq = 0; iq < nq; iq++) {
      hb[n * nq + iq] = mesh->psiq[n + ngl * iq];
      hb[ngl * nq + n * nq + iq] = mesh->dpsiq[n + ngl * iq];
    }
  for (int n = 0; n < ngl; n++)
    for (int k = 0; k < ngl; k++) {
      hb[2 * ngl * nq + n * ngl + k] = mesh->dpsi[n + ngl * k];
      hb[2 * ngl * nq + ngl * ngl + n * ngl + k] = mesh->psi[n + ngl * k];
    }
  for (int x = 0; x < ngl * nq; x++) {
    hb[nb0 + 2 * x] = hb[x];
    hb[nb0 + 2 * x + 1] = hb[ngl * nq + x];
  }
  for (int x = 0; x < ngl * ngl; x++) hb[nb0 + 2 * ngl * nq + x] = hb[2 * ngl * nq + x];
  // the stage kernels drop the zero terms of the nodal derivative sums: psi must be the
  // identity at the LGL nodes (it is, exactly, for the reference's nodal basis)
  for (int n = 0; n < ngl; n++)
    for (int k = 0; k < ngl; k++)
      if (mesh->psi[n + ngl * k] != (n == k ? 1.0 : 0.0))
        return fail(eng, HNUMO_ERR_INVALID, "nodal basis psi is not the identity at the LGL nodes");
  std::vector<double> qs(QS_N * npq), ns(NS_N * npoin), fs(FS_N * FQ), fns(FN_N * FN);
  for (size_t i = 0; i < npq; i++) {
    qs[QS_W * npq + i] = mesh->jacq[i];
    qs[QS_COR * npq + i] = st->coriolis_quad[i];
    qs[QS_TW1 * npq + i] = st->tau_wind[2 * i];
    qs[QS_TW2 * npq + i] = st->tau_wind[2 * i + 1];
    qs[QS_GZ1 * npq + i] = st->grad_zbot_quad[2 * i];
    qs[QS_GZ2 * npq + i] = st->grad_zbot_quad[2 * i + 1];
    qs[QS_OOP * npq + i] = st->one_over_pbprime[i];
    qs[QS_EX * npq + i] = mesh->ksiq_x[i];
    qs[QS_EY * npq + i] = mesh->ksiq_y[i];
    qs[QS_NX * npq + i] = mesh->etaq_x[i];
    qs[QS_NY * npq + i] = mesh->etaq_y[i];
    qs[QS_PB * npq + i] = st->pbprime[i];
  }
  for (size_t i = 0; i < npoin; i++) {
    ns[NS_PB * npoin + i] = st->pbprime_df[i];
    ns[NS_OOP * npoin + i] = st->one_over_pbprime_df[i];
    ns[NS_MINV * npoin + i] = mesh->massinv[i];
    ns[NS_W * npoin + i] = mesh->jac[i];
    ns[NS_EX * npoin + i] = mesh->ksi_x[i];
    ns[NS_EY * npoin + i] = mesh->ksi_y[i];
    ns[NS_NX * npoin + i] = mesh->eta_x[i];
    ns[NS_NY * npoin + i] = mesh->eta_y[i];
    ns[NS_ZB * npoin + i] = st->zbot_df[i];
    ns[NS_F2 * npoin + i] = st->fdt2_bcl[i];
    ns[NS_A * npoin + i] = st->a_bcl[i];
    ns[NS_B * npoin + i] = st->b_bcl[i];
  }
  for (size_t i = 0; i < FQ; i++) {
    fs[FS_NX * FQ + i] = mesh->normal_vector_q[3 * i];
    fs[FS_NY * FQ + i] = mesh->normal_vector_q[3 * i + 1];
    fs[FS_W * FQ + i] = mesh->jac_faceq[i];
    fs[FS_CL * FQ + i] = st->coeff_pbpert_L[i];
    fs[FS_CR * FQ + i] = st->coeff_pbpert_R[i];
    fs[FS_CLR * FQ + i] = st->coeff_pbub_LR[i];
    fs[FS_CML * FQ + i] = st->coeff_mass_pbub_L[i];
    fs[FS_CMR * FQ + i] = st->coeff_mass_pbub_R[i];
    fs[FS_CMLR * FQ + i] = st->coeff_mass_pbpert_LR[i];
    fs[FS_OOPE * FQ + i] = st->one_over_pbprime_edge[i];
    fs[FS_PBL * FQ + i] = st->pbprime_face[2 * i];
    fs[FS_PBR * FQ + i] = st->pbprime_face[2 * i + 1];
    fs[FS_ZBL * FQ + i] = st->zbot_face[2 * i];
    fs[FS_ZBR * FQ + i] = st->zbot_face[2 * i + 1];
  }
  for (size_t i = 0; i < FN; i++) {
    fns[FN_NX * FN + i] = mesh->normal_vector[3 * i];
    fns[FN_NY * FN + i] = mesh->normal_vector[3 * i + 1];
    fns[FN_W * FN + i] = mesh->jac_face[i];
    fns[FN_PBL * FN + i] = st->pbprime_df_face[2 * i];
    fns[FN_PBR * FN + i] = st->pbprime_df_face[2 * i + 1];
  }
  // element-major statics (engine_internal.h)
  const int Qe = nq * nq, FBLK = EF_N * nq + EFN_N * ngl;
  std::vector<double> qsE((size_t)E * qe_stride(Qe)), nsE((size_t)E * NE_N * P), efs((size_t)E * 4 * FBLK);
  {
    const int qmap[QE_N] = {QS_W, QS_EX, QS_EY, QS_NX, QS_NY, QS_COR, QS_TW1, QS_TW2, QS_GZ1, QS_GZ2, QS_OOP};
    const int nmap[NE_N] = {NS_EX, NS_EY, NS_NX, NS_NY, NS_W, NS_OOP, NS_MINV, NS_PB};
    const int fmap_[EF_PBLQ] = {FS_NX, FS_NY, FS_W, FS_CL, FS_CR, FS_CLR, FS_CML, FS_CMR, FS_CMLR, FS_OOPE};
    const int fnmap[EFN_N] = {FN_NX, FN_NY, FN_W, FN_PBL, FN_PBR};
    for (int e = 0; e < E; e++) {
      for (int c = 0; c < QE_N; c++)
        for (int q = 0; q < Qe; q++) qsE[(size_t)e * qe_stride(Qe) + qe_pos(c, q, Qe)] = qs[qmap[c] * npq + (size_t)e * Qe + q];
      for (int c = 0; c < NE_N; c++)
        for (int p = 0; p < P; p++) nsE[((size_t)e * NE_N + c) * P + p] = ns[nmap[c] * npoin + (size_t)e * P + p];
      for (int lf = 0; lf < 4; lf++) {
        const size_t f = efaces[4 * e + lf];
        double *b = &efs[((size_t)e * 4 + lf) * FBLK];
        for (int c = 0; c < EF_PBLQ; c++)
          for (int iq = 0; iq < nq; iq++) b[c * nq + iq] = fs[fmap_[c] * FQ + f * nq + iq];
        // creat_btp_fluxes_qdf's pbl/pbr (mod_rhs_btp.F90:255-258): same products, same order
        for (int iq = 0; iq < nq; iq++) {
          double pl = 0.0, pr = 0.0;
          for (int n = 0; n < ngl; n++) {
            pl = pl + hb[n * nq + iq] * fns[FN_PBL * FN + f * ngl + n];
            pr = pr + hb[n * nq + iq] * fns[FN_PBR * FN + f * ngl + n];
          }
          b[EF_PBLQ * nq + iq] = pl;
          b[EF_PBRQ * nq + iq] = pr;
        }
        for (int c = 0; c < EFN_N; c++)
          for (int n = 0; n < ngl; n++) b[EF_N * nq + c * ngl + n] = fns[fnmap[c] * FN + f * ngl + n];
      }
    }
  }
  eng->ssprk_a.assign(st->ssprk_a, st->ssprk_a + 3 * par->kstages);
  eng->ssprk_beta.assign(st->ssprk_beta, st->ssprk_beta + par->kstages);

  eng->basis = dalloc<double>(eng, hb.size());
  eng->qstat = dalloc<double>(eng, qs.size());
  eng->nstat = dalloc<double>(eng, ns.size());
  eng->fstat = dalloc<double>(eng, fs.size());
  eng->fnstat = dalloc<double>(eng, fns.size());
  eng->qstatE = dalloc<double>(eng, qsE.size());
  eng->nstatE = dalloc<double>(eng, nsE.size());
  eng->efstat = dalloc<double>(eng, efs.size());
  eng->ecoef = dalloc<double>(eng, (size_t)E * eco_stride(Qe, P));
  eng->efcoef = dalloc<double>(eng, (size_t)E * 4 * (4 * nq + 10 * ngl));
  eng->alpha = dalloc<double>(eng, L);
  eng->tau_wind = dalloc<double>(eng, 2 * npq);
  const size_t n3 = 3 * npoin * L;
  eng->q = dalloc<double>(eng, n3); eng->qp = dalloc<double>(eng, n3); eng->qb = dalloc<double>(eng, 4 * npoin);
  eng->q2 = dalloc<double>(eng, n3); eng->qp2 = dalloc<double>(eng, n3); eng->qbp = dalloc<double>(eng, 4 * npoin);
  eng->qf = dalloc<double>(eng, 6 * FN * L); eng->qf2 = dalloc<double>(eng, 6 * FN * L);
  eng->qfa = dalloc<double>(eng, 6 * FN * L);
  eng->dpp2 = dalloc<double>(eng, npoin * L);
  for (int i = 0; i < 4; i++) eng->qbuf[i] = dalloc<double>(eng, 4 * npoin);
  // trace buffers: element slots [4E], then (processor-face halo) NS send + NS receive slots
  for (int i = 0; i < 2; i++) eng->gtrace[i] = dalloc<double>(eng, (4 * (size_t)E + 2 * (size_t)eng->NS) * 8 * ngl);
  eng->qcoef = dalloc<double>(eng, QC_N * npq); eng->ncoef = dalloc<double>(eng, NC_N * npoin);
  eng->fcoef = dalloc<double>(eng, FC_N * FQ); eng->fncoef = dalloc<double>(eng, 10 * FN);
  eng->dpp_graduv = dalloc<double>(eng, 4 * npoin * L); eng->dpprime_visc = dalloc<double>(eng, npoin * L);
  eng->gdpp_face = dalloc<double>(eng, 10 * FN * L);
  eng->qacc = dalloc<double>(eng, QA_N * npq); eng->facc = dalloc<double>(eng, FA_N * 4 * (size_t)E * nq);
  eng->nacc = dalloc<double>(eng, NA_N * npoin); eng->gfacc = dalloc<double>(eng, 8 * 4 * (size_t)E * ngl);
  eng->tau_wind_ave = dalloc<double>(eng, 2 * npq);
  eng->slmf = dalloc<double>(eng, 2 * npq); eng->slmf_face = dalloc<double>(eng, 2 * FQ);
  eng->dpp = dalloc<double>(eng, npoin * L);
  eng->fmass = dalloc<double>(eng, FQ * L); eng->fcons = dalloc<double>(eng, FQ * L);
  eng->momL = dalloc<double>(eng, 4 * (size_t)E * 2 * nq * L);  // [slot][L][2][NQ] (MSLOT)
  eng->momR = nullptr;
  eng->lapf = dalloc<double>(eng, 4 * (size_t)E * 2 * ngl * L);  // [slot][L][2][NGL]
  if (par->method_visc == 1) {  // quad-point LDG (kernels_lapq.hip)
    eng->lapq_on = true;
    eng->dpq = dalloc<double>(eng, npq * L);
    eng->lq_flux = dalloc<double>(eng, 4 * npq * L);
    eng->lapq = dalloc<double>(eng, 2 * npoin * L);
    std::vector<int> fq(2 * FQ, -1);
    for (int s = 0; s < 2; s++) {
      const int32_t *imq = s == 0 ? mesh->imapl_q : mesh->imapr_q;
      for (int f = 0; f < F; f++)
        for (int iq = 0; iq < nq; iq++) {
          const int i = imq[3 * (iq + nq * f)] - 1, j = imq[3 * (iq + nq * f) + 1] - 1;
          if (s == 1 && mesh->face[8 * f + 7] <= 0) continue;
          if (i < 0 || i >= nq || j < 0 || j >= nq) return fail(eng, HNUMO_ERR_INVALID, "imapl_q/imapr_q out of range");
          fq[s * FQ + (size_t)f * nq + iq] = j * nq + i;
        }
    }
    eng->fqLR = dalloc<int>(eng, 2 * FQ);
    if (eng->fqLR) HIPCHK(hipMemcpy(eng->fqLR, fq.data(), fq.size() * sizeof(int), hipMemcpyHostToDevice));
  }
  eng->rhs = dalloc<double>(eng, 3 * npoin);
  eng->neg_flag = dalloc<int>(eng, 1);
  if (const char *ge = env_knob(eng, "HNUMO_GRAPH", false)) eng->graph_env = ge[0] == '0' ? 0 : ge[0] == '1' ? 1 : -1;
  if (const char *sm = env_knob(eng, "HNUMO_SUMMATION", false)) {
    if (!strcmp(sm, "reference"))
      eng->summation = HNUMO_SUM_REFERENCE;
    else if (!strcmp(sm, "factored"))
      eng->summation = HNUMO_SUM_FACTORED;
    else
      return fail(eng, HNUMO_ERR_INVALID, std::string("HNUMO_SUMMATION=") + sm + ": only 'reference' or 'factored'");
  }
  if (HNUMO_DIAG)  // (diagnostics builds only; see engine_internal.h)
    if (const char *sd = env_knob(eng, "HNUMO_STAGE_DBG")) eng->stage_dbg = atoi(sd);
  if (const char *fz = env_knob(eng, "HNUMO_FUSE")) eng->no_fuse = fz[0] == '0';
  // (bit 1 drops a required stream dependency -- wrong results, timing only: diagnostics builds)
  if (HNUMO_DIAG)
    if (const char *sd = env_knob(eng, "HNUMO_SCHED_DBG")) eng->sched_dbg = atoi(sd);
  // per-stage kernel arena: on meshes that take several residency rounds per stage, the arena
  // sized for 4 workgroups per CU (1-row term chunks) -- 1.566 -> 1.517 ms per stage at C4
  // (tools/ab_env.py, round 2); small meshes keep the 3-per-CU arena
  // large meshes: the LEAN 5-per-CU arena (C4: 1.331 ms per stage against 1.409 for the 4-per-CU
  // one with 2-row term chunks and 1.501 for round 2's, profiles/r03f)
  eng->stage_nb = eng->nelem_owned >= 2048 ? 5 : 0;
  if (const char *sn = env_knob(eng, "HNUMO_STAGE_NB")) eng->stage_nb = atoi(sn);
  eng->bcl_big = eng->nelem_owned >= 2048;
  if (const char *bb = env_knob(eng, "HNUMO_BCL_BIG")) eng->bcl_big = bb[0] == '1';
  if (const char *az = env_knob(eng, "HNUMO_ACC_ZERO")) eng->acc_zero = az[0] == '1';
  {
    const char *qv = env_knob(eng, "HNUMO_QPQ");
    if (par->botfr && !(qv && atoi(qv) == 0)) eng->qpq = dalloc<double>(eng, (size_t)E * 3 * eng->nq * eng->nq);
  }
  if (const char *sp = HNUMO_DIAG ? env_knob(eng, "HNUMO_STAGE_PROF") : nullptr)
    if (sp[0] == '1') eng->stage_prof = dalloc<unsigned long long>(eng, (size_t)eng->nelem * 32);
  if (eng->face_halo) {
    eng->rank = halo->rank;
    eng->nranks = halo->nranks;
    const int NS = eng->NS;
    // trace source slot of every element face; boundary / interior element lists
    std::vector<int> tsrc(4 * (size_t)E), elB, elI;
    for (int e = 0; e < E; e++) {
      bool bnd = false;
      for (int lf = 0; lf < 4; lf++) {
        const int f = efaces[4 * e + lf];
        const bool proc = ebc[4 * e + lf] == 0;
        tsrc[4 * e + lf] = proc ? 4 * E + NS + face_slot[f] : 4 * e + lf;
        bnd |= proc;
      }
      (bnd ? elB : elI).push_back(e);
    }
    eng->nB = (int)elB.size();
    eng->nI = (int)elI.size();
    int *d_tsrc = dalloc<int>(eng, tsrc.size());
    eng->d_sface = dalloc<int>(eng, NS);
    eng->d_elB = dalloc<int>(eng, elB.size());
    eng->d_elI = dalloc<int>(eng, elI.size());
    eng->cdef = dalloc<double>(eng, 4 * FQ * L);
    eng->bx_per_max = (size_t)L * std::max({5 * ngl, 2 * nq, eng->lapq_on ? 4 * nq : 0});
    eng->bx_sbuf = dalloc<double>(eng, eng->bx_per_max * NS);
    eng->bx_rbuf = dalloc<double>(eng, eng->bx_per_max * NS);
    if (eng->alloc_failed) return fail(eng, HNUMO_ERR_DEVICE, "hipMalloc failed (halo buffers)");
    HIPCHK(hipMemcpy(d_tsrc, tsrc.data(), tsrc.size() * sizeof(int), hipMemcpyHostToDevice));
    if (NS) HIPCHK(hipMemcpy(eng->d_sface, sface.data(), NS * sizeof(int), hipMemcpyHostToDevice));
    if (eng->nB) HIPCHK(hipMemcpy(eng->d_elB, elB.data(), elB.size() * sizeof(int), hipMemcpyHostToDevice));
    if (eng->nI) HIPCHK(hipMemcpy(eng->d_elI, elI.data(), elI.size() * sizeof(int), hipMemcpyHostToDevice));
    eng->m.etsrc = d_tsrc;
    // the boundary elements and their transport are the critical path of the stage chain:
    // their stream gets the highest priority, so their workgroups dispatch ahead of the
    // interior launch's
    int prio_lo = 0, prio_hi = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    HIPCHK(hipStreamCreateWithPriority(&eng->stream2, hipStreamNonBlocking, prio_hi));
    for (hipEvent_t *ev : {&eng->ev_fork, &eng->ev_join, &eng->ev_I, &eng->ev_B[0], &eng->ev_B[1], &eng->ev_tsent,
                           &eng->ev_bpacked, &eng->ev_bdone})
      HIPCHK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
    for (hipEvent_t *ev : {&eng->ev_Is, &eng->ev_Bs[0], &eng->ev_Bs[1]}) HIPCHK(hipEventCreate(ev));
    if (halo->comm_id) {  // RCCL point-to-point over xGMI
      ncclUniqueId id;
      static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
      std::memcpy(&id, halo->comm_id, sizeof(id));
      ncclResult_t nr = ncclCommInitRank(&eng->comm, halo->nranks, id, halo->rank);
      if (nr != ncclSuccess) return fail(eng, HNUMO_ERR_DEVICE, std::string("ncclCommInitRank: ") + ncclGetErrorString(nr));
      eng->comm_mode = 2;
    }
  } else if (halo && halo->nranks > 1) {
    eng->rank = halo->rank;
    eng->nranks = halo->nranks;
    size_t os = 0, orr = 0;
    const size_t per_max = (size_t)P * std::max(4, 3 * L);
    for (int k = 0; k < halo->num_nbh; k++) {
      Neighbour nb;
      nb.rank = halo->nbh_proc[k];
      nb.nsend = halo->num_ghost_send ? halo->num_ghost_send[k] : 0;
      nb.nrecv = halo->num_ghost_recv ? halo->num_ghost_recv[k] : 0;
      if (nb.rank < 0 || nb.rank >= halo->nranks || nb.rank == halo->rank)
        return fail(eng, HNUMO_ERR_INVALID, "bad neighbour rank");
      for (const auto &pn : eng->nbh)
        if (pn.rank == nb.rank) return fail(eng, HNUMO_ERR_INVALID, "a neighbour rank is listed twice");
      std::vector<int> snd(nb.nsend), rcv(nb.nrecv);
      for (int i = 0; i < nb.nsend; i++) {
        snd[i] = halo->ghost_send[os + i] - 1;
        if (snd[i] < 0 || snd[i] >= eng->nelem_owned) return fail(eng, HNUMO_ERR_INVALID, "ghost_send must list owned elements");
      }
      for (int i = 0; i < nb.nrecv; i++) {
        rcv[i] = halo->ghost_recv[orr + i] - 1;
        if (rcv[i] < eng->nelem_owned || rcv[i] >= E) return fail(eng, HNUMO_ERR_INVALID, "ghost_recv must list ghost elements");
      }
      os += nb.nsend;
      orr += nb.nrecv;
      nb.d_send = dalloc<int>(eng, nb.nsend);
      nb.d_recv = dalloc<int>(eng, nb.nrecv);
      nb.sbuf = dalloc<double>(eng, nb.nsend * per_max);
      nb.rbuf = dalloc<double>(eng, nb.nrecv * per_max);
      if (eng->alloc_failed) return fail(eng, HNUMO_ERR_DEVICE, "hipMalloc failed (halo buffers)");
      if (nb.nsend) HIPCHK(hipMemcpy(nb.d_send, snd.data(), nb.nsend * sizeof(int), hipMemcpyHostToDevice));
      if (nb.nrecv) HIPCHK(hipMemcpy(nb.d_recv, rcv.data(), nb.nrecv * sizeof(int), hipMemcpyHostToDevice));
      eng->nbh.push_back(nb);
    }
    if (halo->comm_id) {  // RCCL point-to-point over xGMI
      ncclUniqueId id;
      static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
      std::memcpy(&id, halo->comm_id, sizeof(id));
      ncclResult_t nr = ncclCommInitRank(&eng->comm, halo->nranks, id, halo->rank);
      if (nr != ncclSuccess) return fail(eng, HNUMO_ERR_DEVICE, std::string("ncclCommInitRank: ") + ncclGetErrorString(nr));
      eng->comm_mode = 2;
    }
  }
  if (eng->alloc_failed) return fail(eng, HNUMO_ERR_DEVICE, "hipMalloc failed (out of device memory?)");
  HIPCHK(hipHostMalloc((void **)&eng->h_neg, sizeof(int)));
  HIPCHK(hipMemcpy(eng->basis, hb.data(), hb.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->qstat, qs.data(), qs.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->nstat, ns.data(), ns.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->fstat, fs.data(), fs.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->fnstat, fns.data(), fns.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->qstatE, qsE.data(), qsE.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->nstatE, nsE.data(), nsE.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->efstat, efs.data(), efs.size() * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->alpha, st->alpha, L * 8, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(eng->tau_wind, st->tau_wind, 2 * npq * 8, hipMemcpyHostToDevice));

  DevMesh &m = eng->m;
  m.nelem = E; m.npoin = (int)npoin; m.npoin_q = (int)npq; m.nface = F; m.ngl = ngl; m.nq = nq; m.L = L;
  m.efaces = eng->iconn + o_ef; m.eside = eng->iconn + o_es; m.ebc = eng->iconn + o_eb; m.efmap = eng->iconn + o_em;
  m.enbr_node = eng->iconn + o_en; m.enbr_e = eng->iconn + o_ee; m.enbr_lf = eng->iconn + o_el;
  m.fnodeL = eng->iconn + o_fl; m.fnodeR = eng->iconn + o_fr; m.fel = eng->iconn + o_fe; m.fer = eng->iconn + o_fer;
  m.fslotL = eng->iconn + o_sl; m.fslotR = eng->iconn + o_sr; m.fslotA = eng->iconn + o_sa;
  m.erec = eng->iconn + o_er;
  m.qstatE = eng->qstatE; m.nstatE = eng->nstatE; m.efstat = eng->efstat;
  m.basis = eng->basis; m.basis_pd = eng->basis + nb0; m.qstat = eng->qstat; m.nstat = eng->nstat; m.fstat = eng->fstat; m.fnstat = eng->fnstat;
  m.alpha = eng->alpha;
  m.gravity = par->gravity; m.cd = par->cd_mlswe; m.visc = par->visc_mlswe; m.dt = par->dt; m.dt_btp = par->dt_btp;
  m.botfr = par->botfr;
  m.ad = par->ad_mlswe; m.max_shear_dz = par->max_shear_dz; m.shear_corr = par->shear_corrector;
  m.runflag = eng->neg_flag;
  eng->steps_done = dalloc<unsigned>(eng, 1);
  m.steps_done = eng->steps_done;
  HIPCHK(hipHostMalloc((void **)&eng->h_steps, sizeof(unsigned)));

  // persistent sub-cycle: stage tables for the two sub-cycles of a step and the residency check
  if (supported_ngl(ngl) && eng->K <= 8) {
    eng->epoch = dalloc<unsigned long long>(eng, 1);
    eng->qsv = dalloc<double>(eng, (size_t)E * 8 * ngl * ngl);
    eng->sub_done = dalloc<unsigned>(eng, 1);
    eng->sub_arrive = dalloc<unsigned>(eng, 1);
    eng->dbg_abort_epoch = dalloc<unsigned long long>(eng, 1);
    if (eng->dbg_abort_epoch) HIPCHK(hipMemset(eng->dbg_abort_epoch, 0xff, sizeof(unsigned long long)));  // never
    for (int b = 0; b < 2; b++) eng->gtr[b] = dalloc<TraceGranule>(eng, (size_t)E * 32 * ngl);
    const char *pe = env_knob(eng, "HNUMO_PERSISTENT", false);
    const bool persist_on = !(pe && pe[0] == '0');
    if (persist_on) {
      if (const char *pp = env_knob(eng, "HNUMO_PERSIST_LDS_PAD")) eng->persist_pad = std::max(0, atoi(pp));
      // HNUMO_PERSIST_GUARD: 0 none (the in-launch rendezvous alone), 'estimate', 'trial', 1 both
      if (const char *pg = env_knob(eng, "HNUMO_PERSIST_GUARD"))
        eng->persist_guard = pg[0] == '0' ? 0 : pg[0] == 'e' ? 1 : pg[0] == 't' ? 2 : 3;
      int ncu = 0;
      HIPCHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, eng->device));
      DISPATCH(eng, occupancy(eng, ncu));
      // (HNUMO_PERSIST_PERM=0: the identity) workgroup b runs on CU b % ncu (the dispatcher's round-robin; blocks b,
      // b + ncu, b + 2 ncu share a CU), so with E/ncu not whole some CUs hold one element more; the
      // elements with a physical-boundary face (more work: ghost states, wall fluxes) go to the CUs
      // holding fewer, the others fill the rest in order.  Same arithmetic per element, same bits
      // (dg25L3: 16 us less sub-cycle time per step in 3 interleaved pairs, profiles/r05x).
      const char *pm = env_knob(eng, "HNUMO_PERSIST_PERM");
      if (!(pm && pm[0] == '0') && ncu > 0 && E % ncu && eng->nranks == 1 && !eng->face_halo && eng->comm_mode == 0 &&
          eng->nelem_owned == E) {
        const int nheavy = E % ncu;  // CUs k < nheavy hold one block more
        // (measured, not kept: also grouping by XCD -- blocks b and b + 8 share one, so group b % 8
        // took the (b % 8)-th strip of consecutive element ids: 2268 against 2224 us of sub-cycle per
        // step, profiles/r05z)
        std::vector<int> bnd, inr, perm(E);
        for (int el = 0; el < E; el++) {
          bool b = false;
          for (int lf = 0; lf < 4; lf++) b = b || ebc[4 * el + lf] < 0;
          (b ? bnd : inr).push_back(el);
        }
        size_t ib = 0, ii = 0;
        // (measured, not kept: a CU's blocks on consecutive element ids -- neighbours sharing a CU --
        // 2357 against 2208 us of sub-cycle per step, profiles/r05ac)
        for (int b = 0; b < E; b++) {
          const bool light = (b % ncu) >= nheavy;
          perm[b] = (light && ib < bnd.size()) ? bnd[ib++] : (ii < inr.size() ? inr[ii++] : bnd[ib++]);
        }
        eng->d_eperm = dalloc<int>(eng, E);
        if (eng->d_eperm) HIPCHK(hipMemcpy(eng->d_eperm, perm.data(), E * sizeof(int), hipMemcpyHostToDevice));
        // the element kernels of the step (625 blocks at dg25 too: the same CUs hold one block more)
        const char *pg = env_knob(eng, "HNUMO_GLUE_PERM");
        if (!(pg && pg[0] == '0')) eng->m.eperm = eng->d_eperm;
      }
    }
    // the stage tables copy eng->m: built after the placement above, so every DevMesh copy (these,
    // the per-stage tables of stage_table at run time) carries the same eperm
    const double *qps[2] = {eng->qp, eng->qp2};
    for (int v = 0; v < 2; v++) {
      std::vector<StageArgs> st;
      (void)stage_table(eng, qps[v], st);
      st.front().qb_in = eng->qb;                        // the step-start state (launch_subcycle)
      st.front().self_trace = 1;                         // stage 0 publishes its input traces
      st.back().qb_out = v == 0 ? eng->qbp : eng->qb;    // predictor / corrector result
      eng->d_stages[v] = dalloc<StageArgs>(eng, st.size());
      if (eng->alloc_failed) return fail(eng, HNUMO_ERR_DEVICE, "hipMalloc failed (stage tables)");
      HIPCHK(hipMemcpy(eng->d_stages[v], st.data(), st.size() * sizeof(StageArgs), hipMemcpyHostToDevice));
    }
    if (persist_on) {
      // the trial launches: what the dispatcher does, not what the estimate says, decides
      for (int sm = 0; sm < 2 && (eng->persist_guard & 2); sm++) {
        if (!eng->persistent_ok[sm] || eng->comm_mode != 0 || eng->nranks != 1) continue;
        HIPCHK(hipMemsetAsync(eng->neg_flag, 0, sizeof(int), eng->stream));
        DISPATCH(eng, probe(eng, sm));
        HIPCHK(hipMemcpyAsync(eng->h_neg, eng->neg_flag, sizeof(int), hipMemcpyDeviceToHost, eng->stream));
        HIPCHK(hipStreamSynchronize(eng->stream));
        HIPCHK(hipGetLastError());
        eng->probe_ok[sm] = (*eng->h_neg & RUN_ABORT) ? 0 : 1;
        if (!eng->probe_ok[sm]) eng->persistent_ok[sm] = false;
        HIPCHK(hipMemsetAsync(eng->neg_flag, 0, sizeof(int), eng->stream));
      }
    }
  }
  // tau_wind_ave = (N_btp times tau_wind summed) / N_btp (mod_rk_mlswe.F90:148) is constant: formed
  // once here (btp_finalize_kernel also re-forms it after every per-stage sub-cycle)
  hipLaunchKernelGGL(btp_finalize_kernel, dim3(256), dim3(256), 0, eng->stream, eng->qacc, eng->facc, eng->nacc,
                     eng->gfacc, eng->tau_wind_ave, eng->tau_wind, (int)npq, 0, 0, 0, par->N_btp, 1.0, nullptr,
                     nullptr, 0);
  HIPCHK(hipDeviceSynchronize());
  return HNUMO_OK;
}

static int upload_state(hnumo_engine *eng, const double *q, const double *qb, const double *qp) {
  const size_t n3 = 3 * (size_t)eng->npoin * eng->L;
  if (q) HIPCHK(hipMemcpyAsync(eng->q, q, n3 * 8, hipMemcpyHostToDevice, eng->stream));
  if (qb) HIPCHK(hipMemcpyAsync(eng->qb, qb, 4 * (size_t)eng->npoin * 8, hipMemcpyHostToDevice, eng->stream));
  if (qp) HIPCHK(hipMemcpyAsync(eng->qp, qp, n3 * 8, hipMemcpyHostToDevice, eng->stream));
  if (qp && fused_extract(eng)) DISPATCH(eng, extract(eng, eng->qp, eng->qf, 0));
  return 0;
}

static int download_state(hnumo_engine *eng, double *q, double *qb, double *qp) {
  const size_t n3 = 3 * (size_t)eng->npoin * eng->L;
  if (q) HIPCHK(hipMemcpyAsync(q, eng->q, n3 * 8, hipMemcpyDeviceToHost, eng->stream));
  if (qb) HIPCHK(hipMemcpyAsync(qb, eng->qb, 4 * (size_t)eng->npoin * 8, hipMemcpyDeviceToHost, eng->stream));
  if (qp) HIPCHK(hipMemcpyAsync(qp, eng->qp, n3 * 8, hipMemcpyDeviceToHost, eng->stream));
  HIPCHK(hipStreamSynchronize(eng->stream));
  return 0;
}

// The whole step is captured once into a hipGraph (RCCL calls included) and replayed.  A
// local exchange group (host barriers between engines) and a failed capture run the
// same launch sequence directly.
static int ensure_graph(hnumo_engine *eng) {
  if (eng->graph_exec || eng->no_graph) return 0;
  // RCCL engines replay direct launches unless HNUMO_GRAPH=1: capturing RCCL point-to-point
  // into a graph cannot be exercised on a one-GPU box, and at the multi-GPU sizes (~1e4
  // elements per GPU, ~0.2 ms per stage) the host issues a stage's launches faster than the
  // GPU runs them
  if (eng->comm_mode == 1 || eng->graph_env == 0 || (eng->comm_mode == 2 && eng->graph_env != 1)) {
    eng->no_graph = true;
    return 0;
  }
  eng->kernel_events = false;
  HIPCHK(hipStreamBeginCapture(eng->stream, hipStreamCaptureModeThreadLocal));
  launch_step(eng);
  hipError_t err = hipStreamEndCapture(eng->stream, &eng->graph);
  if (err == hipSuccess) err = hipGraphInstantiate(&eng->graph_exec, eng->graph, nullptr, nullptr, 0);
  if (err != hipSuccess) {
    (void)hipGetLastError();
    if (eng->graph) (void)hipGraphDestroy(eng->graph);
    eng->graph = nullptr;
    eng->graph_exec = nullptr;
    eng->no_graph = true;
    // RCCL calls were recorded into the failed capture: this rank's point-to-point sequence
    // can no longer be trusted to match its peers', so report instead of falling back
    if (eng->comm_mode == 2)
      return fail(eng, HNUMO_ERR_DEVICE,
                  std::string("step graph capture with RCCL failed (") + hipGetErrorString(err) +
                      "); rerun with HNUMO_GRAPH=0 for direct launches");
  }
  if (!eng->comm_err.empty()) return fail(eng, HNUMO_ERR_DEVICE, eng->comm_err);
  return 0;
}

// error bits of the device flag word (neg_flag): 1 negative thickness, 2 non-finite
// state, 8 a persistent sub-cycle trace wait timed out, 16 (RUN_ABORT) a persistent launch found
// its workgroups not co-resident -- handled by the callers (persistent_abort), never an error
static int flag_error(hnumo_engine *eng, int flags) {
  if (flags & 1) return fail(eng, HNUMO_ERR_NEGATIVE_THICKNESS, "Negative mass in thickness at some points");
  if (flags & 2) return fail(eng, HNUMO_ERR_NONFINITE, "non-finite barotropic state");
  if (flags & 8) return fail(eng, HNUMO_ERR_DEVICE, "persistent sub-cycle: a trace granule wait timed out");
  return 0;
}

// the captured step holds the stage path and summation mode: capture again on the next step
static void drop_graph(hnumo_engine *eng) {
  if (eng->graph_exec) (void)hipGraphExecDestroy(eng->graph_exec);
  if (eng->graph) (void)hipGraphDestroy(eng->graph);
  eng->graph_exec = nullptr;
  eng->graph = nullptr;
  if (eng->comm_mode != 1) eng->no_graph = false;
}

// A persistent launch of the run was not co-resident (RUN_ABORT): it did no work, and neither
// did anything after it that writes the step state, so the state is that of the last completed
// step.  The engine suspends the persistent path (maybe_reprobe brings it back once a trial launch
// finds the grid resident again) and the caller repeats what is left on per-stage launches.
static void persistent_abort(hnumo_engine *eng) {
  eng->persist_suspended = true;
  eng->persist_aborts++;
  eng->persist_wait = eng->persist_backoff;
  eng->persist_backoff = std::min(2 * eng->persist_backoff, 1024);
  drop_graph(eng);
}

// Before a run: a suspended persistent path whose wait is over gets one stage-less trial launch
// (Launch::probe, the residency rendezvous alone); all workgroups resident -> persistent again.
// (A co-resident job that held CUs for a moment costs a few per-stage runs, not the engine's
// lifetime on per-stage launches; one that stays costs a 20 ms probe every 1024 runs at most.)
static int maybe_reprobe(hnumo_engine *eng) {
  if (!eng->persist_suspended || !eng->persistent_ok[eng->summation]) return 0;
  if (eng->persist_wait > 0) {
    eng->persist_wait--;
    return 0;
  }
  eng->persist_reprobes++;
  HIPCHK(hipMemsetAsync(eng->neg_flag, 0, sizeof(int), eng->stream));
  DISPATCH(eng, probe(eng, eng->summation));
  HIPCHK(hipMemcpyAsync(eng->h_neg, eng->neg_flag, sizeof(int), hipMemcpyDeviceToHost, eng->stream));
  HIPCHK(hipStreamSynchronize(eng->stream));
  HIPCHK(hipGetLastError());
  const bool resident = !(*eng->h_neg & RUN_ABORT);
  HIPCHK(hipMemsetAsync(eng->neg_flag, 0, sizeof(int), eng->stream));
  if (resident) {
    eng->persist_suspended = false;
    eng->persist_recovered++;
    drop_graph(eng);
  } else {
    eng->persist_wait = eng->persist_backoff;
    eng->persist_backoff = std::min(2 * eng->persist_backoff, 1024);
  }
  return 0;
}

static int transport_error(hnumo_engine *eng) {
  if (!eng->comm_err.empty()) {
    std::string m = eng->comm_err;
    eng->comm_err.clear();
    return fail(eng, HNUMO_ERR_DEVICE, "halo exchange failed: " + m);
  }
  if (eng->group && eng->group->aborted) return fail(eng, HNUMO_ERR_DEVICE, "local exchange group aborted by another engine");
  return 0;
}

static int launch_steps(hnumo_engine *eng, int nsteps) {
  int rc = ensure_graph(eng);
  if (rc) return rc;
  for (int s = 0; s < nsteps; s++) {
    if (eng->graph_exec)
      HIPCHK(hipGraphLaunch(eng->graph_exec, eng->stream));
    else
      launch_step(eng);
  }
  return 0;
}

// (retry: the per-stage repeat of a run whose persistent launch gave up -- it does not count as a
// run of the back-off wait that abort just set)
static int run_steps(hnumo_engine *eng, int nsteps, bool retry = false) {
  int rc = retry ? 0 : maybe_reprobe(eng);
  if (rc) return rc;
  const bool pers = use_persistent(eng);
  HIPCHK(hipMemsetAsync(eng->neg_flag, 0, sizeof(int), eng->stream));
  HIPCHK(hipMemsetAsync(eng->steps_done, 0, sizeof(unsigned), eng->stream));
  rc = launch_steps(eng, nsteps);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(eng->h_neg, eng->neg_flag, sizeof(int), hipMemcpyDeviceToHost, eng->stream));
  HIPCHK(hipMemcpyAsync(eng->h_steps, eng->steps_done, sizeof(unsigned), hipMemcpyDeviceToHost, eng->stream));
  HIPCHK(hipStreamSynchronize(eng->stream));
  HIPCHK(hipGetLastError());
  if ((rc = transport_error(eng))) return rc;
  if ((*eng->h_neg & RUN_ABORT) && !use_persistent(eng)) return fail(eng, HNUMO_ERR_DEVICE, "run aborted off the persistent path");
  if (*eng->h_neg & RUN_ABORT) {
    const int done = (int)*eng->h_steps;
    // an error of a step that completed before the abort is reported, not cleared by the retry
    if ((rc = flag_error(eng, *eng->h_neg & ~RUN_ABORT))) return rc;
    persistent_abort(eng);
    return done < nsteps ? run_steps(eng, nsteps - done, true) : 0;
  }
  if (pers) eng->persist_backoff = 1;  // a completed persistent run
  return flag_error(eng, *eng->h_neg);
}

// A multi-rank engine exchanges halos inside these calls: it needs its RCCL transport (a local
// group's engines run together, through hnumo_group_ti_rk_bcl only)
static int component_transport_check(hnumo_engine *eng) {
  if (eng->comm_mode == 1) return fail(eng, HNUMO_ERR_INVALID, "engine is in a local group: use hnumo_group_ti_rk_bcl");
  if ((eng->nranks > 1 || eng->face_halo) && eng->comm_mode == 0)
    return fail(eng, HNUMO_ERR_INVALID, "multi-rank engine without transport (comm_id or hnumo_local_group)");
  return 0;
}

int hnumo_ti_rk_bcl(hnumo_engine *eng, double *q_df, double *qb_df, double *qprime_df) {
  if (!eng) return HNUMO_ERR_INVALID;
  if (int rc = component_transport_check(eng)) return rc;
  HIPCHK(hipSetDevice(eng->device));
  if (!eng->resident || !eng->uploaded) {
    int rc = upload_state(eng, q_df, qb_df, qprime_df);
    if (rc) return rc;
    eng->uploaded = true;
  }
  int rc = run_steps(eng, 1);
  if (rc) return rc;
  if (!eng->resident) return download_state(eng, q_df, qb_df, qprime_df);
  return 0;
}

int hnumo_set_resident(hnumo_engine *eng, int on) {
  if (!eng) return HNUMO_ERR_INVALID;
  eng->resident = on != 0;
  eng->uploaded = false;
  return 0;
}

int hnumo_set_summation(hnumo_engine *eng, int mode) {
  if (!eng) return HNUMO_ERR_INVALID;
  if (mode != HNUMO_SUM_REFERENCE && mode != HNUMO_SUM_FACTORED)
    return fail(eng, HNUMO_ERR_INVALID, "hnumo_set_summation: mode must be HNUMO_SUM_REFERENCE or HNUMO_SUM_FACTORED");
  if (mode != eng->summation) {
    eng->summation = mode;
    drop_graph(eng);  // (the captured step holds the other kernel)
  }
  return 0;
}

int hnumo_get_summation(hnumo_engine *eng) { return eng ? eng->summation : -1; }

int hnumo_stage_path(hnumo_engine *eng) { return eng ? (use_persistent(eng) ? 1 : 0) : -1; }

extern "C++" template <int NGL, int NQ>
static int subcycle_lds_bytes(const hnumo_engine *e) {
  hipFuncAttributes fa{};
  if (e->summation == HNUMO_SUM_REFERENCE)
    (void)hipFuncGetAttributes(&fa, (const void *)btp_subcycle_kernel<NGL, NQ, false>);
  else
    (void)hipFuncGetAttributes(&fa, (const void *)btp_subcycle_kernel<NGL, NQ, true>);
  return (int)fa.sharedSizeBytes + e->persist_pad;
}

int hnumo_persistent_info(hnumo_engine *eng, int32_t *out) {
  if (!eng || !out) return HNUMO_ERR_INVALID;
  int lds = 0;
  switch (eng->ngl) {
    case 3: lds = subcycle_lds_bytes<3, 5>(eng); break;
    case 4: lds = subcycle_lds_bytes<4, 7>(eng); break;
    case 5: lds = subcycle_lds_bytes<5, 9>(eng); break;
    case 6: lds = subcycle_lds_bytes<6, 11>(eng); break;
    case 8: lds = subcycle_lds_bytes<8, 15>(eng); break;
    default: break;
  }
  (void)hipGetLastError();
  const int32_t v[8] = {use_persistent(eng) ? 1 : 0, eng->occ_blocks[0], eng->occ_blocks[1], eng->occ_ncu,
                        eng->probe_ok[0], eng->probe_ok[1], eng->persist_aborts, lds};
  std::memcpy(out, v, sizeof(v));
  return 0;
}

int hnumo_persistent_stats(hnumo_engine *eng, int32_t *out4) {
  if (!eng || !out4) return HNUMO_ERR_INVALID;
  const int32_t v[4] = {eng->persist_aborts, eng->persist_reprobes, eng->persist_recovered,
                        eng->persist_suspended ? eng->persist_wait : -1};
  std::memcpy(out4, v, sizeof(v));
  return 0;
}

int hnumo_debug_frozen_halo(hnumo_engine *eng, int on) {
  if (!eng) return HNUMO_ERR_INVALID;
  if (!eng->face_halo || eng->nranks != 1) {
    eng->err = "the frozen halo is for self-neighbour engines (one-rank processor-face halo) only";
    return HNUMO_ERR_INVALID;
  }
  eng->emu_frozen = on != 0;
  return HNUMO_OK;
}

int hnumo_debug_force_abort(hnumo_engine *eng, int k) {
  if (!eng || k < 0) return HNUMO_ERR_INVALID;
  if (!eng->dbg_abort_epoch) return fail(eng, HNUMO_ERR_INVALID, "engine has no persistent sub-cycle");
  HIPCHK(hipSetDevice(eng->device));
  HIPCHK(hipStreamSynchronize(eng->stream));
  unsigned long long ep = 0;
  HIPCHK(hipMemcpy(&ep, eng->epoch, sizeof(ep), hipMemcpyDeviceToHost));
  ep += (unsigned long long)k;
  HIPCHK(hipMemcpy(eng->dbg_abort_epoch, &ep, sizeof(ep), hipMemcpyHostToDevice));
  return 0;
}

#if HNUMO_BCL_PROF
// diagnostics build only (not part of the ABI): the element kernels' phase clocks, see g_bcl_prof
int hnumo_bcl_prof(unsigned long long *dst, int n) {
  const size_t bytes = std::min<size_t>((size_t)n, 4 * 8192 * 8) * sizeof(unsigned long long);
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_bcl_prof), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

int hnumo_sync(hnumo_engine *eng, double *q_df, double *qb_df, double *qprime_df) {
  if (!eng) return HNUMO_ERR_INVALID;
  HIPCHK(hipSetDevice(eng->device));
  return download_state(eng, q_df, qb_df, qprime_df);
}

int hnumo_btp_bcl_coeffs(hnumo_engine *eng, const double *qprime_df) {
  if (!eng) return HNUMO_ERR_INVALID;
  int rc = component_transport_check(eng);
  if (rc) return rc;
  HIPCHK(hipSetDevice(eng->device));
  rc = upload_state(eng, nullptr, nullptr, qprime_df);
  if (rc) return rc;
  launch_bcl_coeffs(eng, eng->qp, eng->qf);
  HIPCHK(hipStreamSynchronize(eng->stream));
  HIPCHK(hipGetLastError());
  return 0;
}

int hnumo_ti_barotropic_ssprk(hnumo_engine *eng, double *qb_df, const double *qprime_df) {
  if (!eng) return HNUMO_ERR_INVALID;
  int rc = component_transport_check(eng);
  if (rc) return rc;
  HIPCHK(hipSetDevice(eng->device));
  rc = upload_state(eng, nullptr, qb_df, qprime_df);
  if (rc) return rc;
  if ((rc = maybe_reprobe(eng))) return rc;
  for (;;) {
    HIPCHK(hipMemsetAsync(eng->neg_flag, 0, sizeof(int), eng->stream));
    launch_subcycle(eng, eng->qbp, eng->qp);
    HIPCHK(hipMemcpyAsync(eng->h_neg, eng->neg_flag, sizeof(int), hipMemcpyDeviceToHost, eng->stream));
    HIPCHK(hipStreamSynchronize(eng->stream));
    HIPCHK(hipGetLastError());
    if ((rc = transport_error(eng))) return rc;
    if (!(*eng->h_neg & RUN_ABORT) || !use_persistent(eng)) break;
    persistent_abort(eng);  // (the launch did no work: qb is still the input)
  }
  if (use_persistent(eng)) eng->persist_backoff = 1;  // a completed persistent run
  if ((rc = flag_error(eng, *eng->h_neg & ~RUN_ABORT))) return rc;
  launch_copy(eng, eng->qb, eng->qbp, 4 * (size_t)eng->npoin);
  return download_state(eng, nullptr, qb_df, nullptr);
}

int hnumo_predict(hnumo_engine *eng, double *q_df, double *qb_df, double *qprime_df) {
  if (!eng) return HNUMO_ERR_INVALID;
  int rc = component_transport_check(eng);
  if (rc) return rc;
  HIPCHK(hipSetDevice(eng->device));
  rc = upload_state(eng, q_df, qb_df, qprime_df);
  if (rc) return rc;
  if ((rc = maybe_reprobe(eng))) return rc;
  for (;;) {
    HIPCHK(hipMemsetAsync(eng->neg_flag, 0, sizeof(int), eng->stream));
    launch_predict(eng);
    HIPCHK(hipMemcpyAsync(eng->h_neg, eng->neg_flag, sizeof(int), hipMemcpyDeviceToHost, eng->stream));
    HIPCHK(hipStreamSynchronize(eng->stream));
    HIPCHK(hipGetLastError());
    if ((rc = transport_error(eng))) return rc;
    if (!(*eng->h_neg & RUN_ABORT) || !use_persistent(eng)) break;
    persistent_abort(eng);  // (the predictor writes only q_df2, qbp, qprime_df2: redo it)
  }
  if (use_persistent(eng)) eng->persist_backoff = 1;  // a completed persistent run
  if ((rc = flag_error(eng, *eng->h_neg & ~RUN_ABORT))) return rc;
  const size_t n3 = 3 * (size_t)eng->npoin * eng->L;
  HIPCHK(hipMemcpyAsync(q_df, eng->q2, n3 * 8, hipMemcpyDeviceToHost, eng->stream));
  HIPCHK(hipMemcpyAsync(qb_df, eng->qbp, 4 * (size_t)eng->npoin * 8, hipMemcpyDeviceToHost, eng->stream));
  HIPCHK(hipMemcpyAsync(qprime_df, eng->qp2, n3 * 8, hipMemcpyDeviceToHost, eng->stream));
  HIPCHK(hipStreamSynchronize(eng->stream));
  // the device state is now the caller's input: a resident engine uploads again on its next step
  eng->uploaded = false;
  return 0;
}

int hnumo_create_rhs_btp(hnumo_engine *eng, double *rhs, const double *qb_df, const double *qprime_df) {
  if (!eng) return HNUMO_ERR_INVALID;
  int rc = component_transport_check(eng);
  if (rc) return rc;
  HIPCHK(hipSetDevice(eng->device));
  rc = upload_state(eng, nullptr, qb_df, qprime_df);
  if (rc) return rc;
  subcycle_prologue(eng, eng->qb, nullptr, true);  // zeroed time averages (qbuf[0] is the rhs-only output slot)
  DISPATCH(eng, grad_trace(eng, eng->qb, eng->gtrace[0], 0, eng->nelem));
  trace_exchange(eng, eng->gtrace[0], eng->stream);
  StageArgs a{};
  a.m = eng->m;
  a.qb_in = eng->qb; a.qb0 = eng->qb; a.qb2 = eng->qb; a.qprime = eng->qp;
  a.ecoef = eng->ecoef; a.efcoef = eng->efcoef;
  a.trace_in = eng->gtrace[0]; a.trace_out = eng->gtrace[1];
  a.qacc = eng->qacc; a.facc = eng->facc; a.nacc = eng->nacc; a.gfacc = eng->gfacc;
  a.qb_out = eng->qbuf[0]; a.rhs_out = eng->rhs;
  a.rhs_only = 1; a.write_trace = 0; a.accumulate = 1;
  a.lapq = eng->lapq_on ? eng->lapq : nullptr;
  if (eng->lapq_on) DISPATCH(eng, lapq_btp(eng, eng->qb, eng->qp));
  DISPATCH(eng, stage(eng, a));
  HIPCHK(hipMemcpyAsync(rhs, eng->rhs, 3 * (size_t)eng->npoin * 8, hipMemcpyDeviceToHost, eng->stream));
  HIPCHK(hipStreamSynchronize(eng->stream));
  HIPCHK(hipGetLastError());
  return 0;
}

// ---- field copy-out in the reference layouts
int hnumo_get_field(hnumo_engine *eng, const char *name, double *out, int64_t n) {
  if (!eng || !name || !out) return HNUMO_ERR_INVALID;
  HIPCHK(hipSetDevice(eng->device));
  HIPCHK(hipStreamSynchronize(eng->stream));
  const size_t npq = eng->npq, npoin = eng->npoin, FQ = eng->FQ, FN = eng->FN, L = eng->L;
  const int nq = eng->nq, ngl = eng->ngl;
  auto fetch = [&](const double *src, size_t cnt, std::vector<double> &h) -> int {
    h.resize(cnt);
    HIPCHK(hipMemcpy(h.data(), src, cnt * 8, hipMemcpyDeviceToHost));
    return 0;
  };
  std::vector<double> h;
  std::string s(name);
  auto soa = [&](const double *base, size_t N, std::initializer_list<int> fields) -> int {
    // interleave SoA fields [field][N] into reference (ncomp, N)
    size_t nc = fields.size();
    if ((size_t)n != nc * N) return fail(eng, HNUMO_ERR_INVALID, "field size mismatch");
    size_t c = 0;
    for (int fld : fields) {
      int rc = fetch(base + (size_t)fld * N, N, h);
      if (rc) return rc;
      for (size_t i = 0; i < N; i++) out[i * nc + c] = h[i];
      c++;
    }
    return 0;
  };
  // element-major accumulators -> reference (ncomp, N) layouts
  const int E_ = eng->nelem, Q_ = nq * nq, P_ = ngl * ngl;
  auto qacc_f = [&](std::initializer_list<int> fields) -> int {
    size_t nc = fields.size();
    if ((size_t)n != nc * npq) return fail(eng, HNUMO_ERR_INVALID, "field size mismatch");
    int rc = fetch(eng->qacc, QA_N * npq, h);
    if (rc) return rc;
    size_t c = 0;
    for (int k : fields) {
      for (int e = 0; e < E_; e++)
        for (int q = 0; q < Q_; q++) out[((size_t)e * Q_ + q) * nc + c] = h[((size_t)e * QA_N + k) * Q_ + q];
      c++;
    }
    return 0;
  };
  auto nacc_f = [&](std::initializer_list<int> fields) -> int {
    size_t nc = fields.size();
    if ((size_t)n != nc * npoin) return fail(eng, HNUMO_ERR_INVALID, "field size mismatch");
    int rc = fetch(eng->nacc, NA_N * npoin, h);
    if (rc) return rc;
    size_t c = 0;
    for (int k : fields) {
      for (int e = 0; e < E_; e++)
        for (int p = 0; p < P_; p++) out[((size_t)e * P_ + p) * nc + c] = h[((size_t)e * NA_N + k) * P_ + p];
      c++;
    }
    return 0;
  };
  auto facc_f = [&](std::initializer_list<int> fields) -> int {
    size_t nc = fields.size();
    if ((size_t)n != nc * FQ) return fail(eng, HNUMO_ERR_INVALID, "field size mismatch");
    int rc = fetch(eng->facc, (size_t)FA_N * 4 * E_ * nq, h);
    if (rc) return rc;
    size_t c = 0;
    for (int k : fields) {
      for (size_t f = 0; f < (size_t)eng->nface; f++)
        for (int iq = 0; iq < nq; iq++)
          out[(f * nq + iq) * nc + c] = h[((size_t)eng->fslotA[f] * FA_N + k) * nq + iq];
      c++;
    }
    return 0;
  };
  struct QF1 { const char *nm; int fld; };
  static const QF1 qsingle[] = {{"ope_ave", QA_OPE}, {"H_ave", QA_H}, {"Qu_ave", QA_QU}, {"Qv_ave", QA_QV},
                                {"Quv_ave", QA_QUV}, {"ope2_ave", QA_OPE2}};
  for (auto &x : qsingle)
    if (s == x.nm) return qacc_f({x.fld});
  if (s == "btp_mass_flux_ave") return qacc_f({QA_MFX, QA_MFY});
  if (s == "uvb_ave") return qacc_f({QA_UB, QA_VB});
  if (s == "tau_bot_ave") return qacc_f({QA_TBU, QA_TBV});
  if (s == "tau_wind_ave") {  // kept in the reference layout (2,npoin_q)
    if ((size_t)n != 2 * npq) return fail(eng, HNUMO_ERR_INVALID, "field size mismatch");
    int rc = fetch(eng->tau_wind_ave, 2 * npq, h);
    if (rc) return rc;
    std::copy(h.begin(), h.end(), out);
    return 0;
  }
  if (s == "ope2_ave_df") return nacc_f({NA_OPE2});
  if (s == "uvb_ave_df") return nacc_f({NA_UB, NA_VB});
  if (s == "graduvb_ave") return nacc_f({NA_G1, NA_G2, NA_G3, NA_G4});
  if (s == "uvb_face_ave") return facc_f({FA_UL, FA_VL, FA_UR, FA_VR});
  if (s == "btp_mass_flux_face_ave") return facc_f({FA_MFX, FA_MFY});
  if (s == "ope_face_ave") return facc_f({FA_OPEL, FA_OPER});
  if (s == "ope2_face_ave") return facc_f({FA_OPE2L, FA_OPE2R});
  if (s == "Qu_face_ave") return facc_f({FA_QUU, FA_QUV});
  if (s == "Qv_face_ave") return facc_f({FA_QVU, FA_QVV});
  if (s == "H_face_ave") return facc_f({FA_H});
  if (s == "one_plus_eta_edge_2_ave") return facc_f({FA_OPEE2});
  if (s == "Quv_face_ave") {  // never accumulated by the reference (mod_rk_mlswe.F90:114-149)
    if ((size_t)n != 2 * FQ) return fail(eng, HNUMO_ERR_INVALID, "field size mismatch");
    std::fill(out, out + n, 0.0);
    return 0;
  }
  if (s == "graduvb_face_ave") {
    if ((size_t)n != 8 * FN) return fail(eng, HNUMO_ERR_INVALID, "field size mismatch");
    int rc = fetch(eng->gfacc, (size_t)8 * 4 * E_ * ngl, h);
    if (rc) return rc;
    for (size_t f = 0; f < (size_t)eng->nface; f++)
      for (int nn = 0; nn < ngl; nn++)
        for (int c = 0; c < 8; c++) out[(f * ngl + nn) * 8 + c] = h[((size_t)eng->fslotA[f] * 8 + c) * ngl + nn];
    return 0;
  }
  if (s == "Q_uu_dp") return soa(eng->qcoef, npq, {QC_QUU});
  if (s == "Q_uv_dp") return soa(eng->qcoef, npq, {QC_QUV});
  if (s == "Q_vv_dp") return soa(eng->qcoef, npq, {QC_QVV});
  if (s == "H_bcl") return soa(eng->qcoef, npq, {QC_HBCL});
  if (s == "Q_uu_dp_edge") return soa(eng->fcoef, FQ, {FC_QUU});
  if (s == "Q_uv_dp_edge") return soa(eng->fcoef, FQ, {FC_QUV});
  if (s == "Q_vv_dp_edge") return soa(eng->fcoef, FQ, {FC_QVV});
  if (s == "H_bcl_edge") return soa(eng->fcoef, FQ, {FC_HBCL});
  if (s == "btp_dpp_graduv") return soa(eng->ncoef, npoin, {NC_D1, NC_D2, NC_D3, NC_D4});
  if (s == "pbprime_visc") return soa(eng->ncoef, npoin, {NC_PV});
  if (s == "btp_graduv_dpp_face") return soa(eng->fncoef, FN, {0, 1, 2, 3, 4, 5, 6, 7, 8, 9});
  if (s == "sum_layer_mass_flux") return soa(eng->slmf, npq, {0, 1});
  if (s == "sum_layer_mass_flux_face") return soa(eng->slmf_face, FQ, {0, 1});
  if (s == "dpprime_visc") {
    if ((size_t)n != npoin * L) return fail(eng, HNUMO_ERR_INVALID, "field size mismatch");
    int rc = fetch(eng->dpprime_visc, npoin * L, h);
    if (rc) return rc;
    std::copy(h.begin(), h.end(), out);
    return 0;
  }
  (void)nq;
  (void)ngl;
  return fail(eng, HNUMO_ERR_INVALID, "unknown field " + s);
}

int hnumo_bench_steps(hnumo_engine *eng, int nsteps, double *ms_total, double *ms_kernel_avg,
                      int64_t *kernel_launches) {
  if (!eng) return HNUMO_ERR_INVALID;
  HIPCHK(hipSetDevice(eng->device));
  int rc = maybe_reprobe(eng);
  if (rc) return rc;
  if ((rc = ensure_graph(eng))) return rc;
  HIPCHK(hipMemsetAsync(eng->neg_flag, 0, sizeof(int), eng->stream));
  HIPCHK(hipEventRecord(eng->ev0, eng->stream));
  rc = launch_steps(eng, nsteps);
  if (rc) return rc;
  HIPCHK(hipEventRecord(eng->ev1, eng->stream));
  HIPCHK(hipMemcpyAsync(eng->h_neg, eng->neg_flag, sizeof(int), hipMemcpyDeviceToHost, eng->stream));
  HIPCHK(hipEventSynchronize(eng->ev1));
  HIPCHK(hipStreamSynchronize(eng->stream));
  HIPCHK(hipGetLastError());
  // a timed run whose state went bad (or whose persistent hand-offs timed out) is no result
  if ((rc = transport_error(eng))) return rc;
  if ((*eng->h_neg & RUN_ABORT) && use_persistent(eng)) {
    // (not co-resident: drop the persistent path and time the run again on per-stage launches)
    persistent_abort(eng);
    return hnumo_bench_steps(eng, nsteps, ms_total, ms_kernel_avg, kernel_launches);
  }
  if ((rc = flag_error(eng, *eng->h_neg))) return rc;
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, eng->ev0, eng->ev1));
  if (ms_total) *ms_total = ms;
  // average stage-kernel duration of the last replay's corrector sub-cycle (N_btp*K
  // back-to-back launches of btp_stage_kernel bracketed by in-graph event nodes)
  double kavg = -1.0;
  if (eng->kernel_events) {
    float mk = 0.f;
    if (hipEventElapsedTime(&mk, eng->evk0, eng->evk1) == hipSuccess) kavg = mk / (double)(eng->p.N_btp * eng->K);
  }
  if (ms_kernel_avg) *ms_kernel_avg = kavg;
  if (kernel_launches) *kernel_launches = (int64_t)nsteps * 2 * eng->p.N_btp * eng->K;
  return 0;
}

int hnumo_time_stage_kernel(hnumo_engine *eng, int nsubcycles, double *ms_kernel_avg) {
  if (!eng || nsubcycles < 1 || !ms_kernel_avg) return HNUMO_ERR_INVALID;
  HIPCHK(hipSetDevice(eng->device));
  if (!eng->evk0) {
    HIPCHK(hipEventCreate(&eng->evk0));
    HIPCHK(hipEventCreate(&eng->evk1));
  }
  (void)hipGetLastError();  // clear a sticky error left by an unsupported in-graph event record
  // the corrector sub-cycle of the current device state, on a scratch copy of qb
  const bool ke = eng->kernel_events;
  eng->kernel_events = true;
  HIPCHK(hipMemsetAsync(eng->neg_flag, 0, sizeof(int), eng->stream));
  double total = 0.0;
  for (int s = 0; s < nsubcycles; s++) {
    launch_subcycle(eng, eng->qbp, eng->qp, true);
    HIPCHK(hipEventSynchronize(eng->evk1));
    float mk = 0.f;
    HIPCHK(hipEventElapsedTime(&mk, eng->evk0, eng->evk1));
    total += mk;
  }
  eng->kernel_events = ke;
  HIPCHK(hipMemcpyAsync(eng->h_neg, eng->neg_flag, sizeof(int), hipMemcpyDeviceToHost, eng->stream));
  HIPCHK(hipStreamSynchronize(eng->stream));
  HIPCHK(hipGetLastError());
  if ((*eng->h_neg & RUN_ABORT) && use_persistent(eng)) {
    persistent_abort(eng);
    HIPCHK(hipMemsetAsync(eng->neg_flag, 0, sizeof(int), eng->stream));
    return hnumo_time_stage_kernel(eng, nsubcycles, ms_kernel_avg);
  }
  int rc = transport_error(eng);
  if (!rc) rc = flag_error(eng, *eng->h_neg & 8);
  if (rc) return rc;
  *ms_kernel_avg = total / ((double)nsubcycles * eng->p.N_btp * eng->K);
  return 0;
}

int hnumo_debug_stage_profile(hnumo_engine *eng, uint64_t *out, int64_t n) {
  if (!eng || !out) return HNUMO_ERR_INVALID;
  if (!eng->stage_prof)
    return fail(eng, HNUMO_ERR_INVALID, HNUMO_DIAG ? "engine created without HNUMO_STAGE_PROF=1"
                                                   : "phase clocks: diagnostics builds only (-DHNUMO_DIAG=1)");
  if (n < (int64_t)eng->nelem * 32) return fail(eng, HNUMO_ERR_INVALID, "buffer too small");
  HIPCHK(hipSetDevice(eng->device));
  HIPCHK(hipStreamSynchronize(eng->stream));
  HIPCHK(hipMemcpy(out, eng->stage_prof, (size_t)eng->nelem * 32 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return 0;
}

int hnumo_rccl_unique_id(unsigned char *out128) {
  if (!out128) return HNUMO_ERR_INVALID;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return HNUMO_ERR_DEVICE;
  std::memcpy(out128, &id, sizeof(id));
  return 0;
}

int hnumo_local_group(hnumo_engine **engines, int n) {
  if (!engines || n < 1) return HNUMO_ERR_INVALID;
  for (int i = 0; i < n; i++)
    if (!engines[i] || engines[i]->rank != i || engines[i]->nranks != n || engines[i]->comm_mode != 0 ||
        engines[i]->device != engines[0]->device)
      return HNUMO_ERR_INVALID;
  for (int i = 0; i < n; i++)
    if (engines[i]->face_halo != engines[0]->face_halo) return HNUMO_ERR_INVALID;
  LocalGroup *g = new LocalGroup();
  g->eng.assign(engines, engines + n);
  g->refs = n;
  // ghost-element halo: one shared stream orders every engine's packs, copies and unpacks;
  // processor-face halo: each engine keeps its streams, the copies are ordered by events
  const bool share = !engines[0]->face_halo;
  if (share) g->stream = engines[0]->stream;  // the group owns engine 0's stream from now on
  for (int i = 0; i < n; i++) {
    hnumo_engine *e = engines[i];
    (void)hipSetDevice(e->device);
    if (share) {
      if (i > 0 && e->own_stream && e->stream) (void)hipStreamDestroy(e->stream);
      e->stream = g->stream;
      e->own_stream = false;
    }
    e->group = g;
    e->comm_mode = 1;
  }
  return 0;
}

int hnumo_group_ti_rk_bcl(hnumo_engine **engines, int n, double **q_df, double **qb_df, double **qprime_df) {
  if (!engines || n < 1 || !engines[0]->group || (int)engines[0]->group->eng.size() != n) return HNUMO_ERR_INVALID;
  std::vector<int> rc(n, 0);
  std::vector<std::thread> th;
  for (int i = 0; i < n; i++)
    th.emplace_back([&, i] {
      hnumo_engine *eng = engines[i];
      (void)hipSetDevice(eng->device);
      if (!eng->resident || !eng->uploaded) {
        rc[i] = upload_state(eng, q_df[i], qb_df[i], qprime_df[i]);
        eng->uploaded = true;
      }
      int r = rc[i] ? rc[i] : run_steps(eng, 1);
      if (!rc[i]) rc[i] = r;
      if (!rc[i] && !eng->resident) rc[i] = download_state(eng, q_df[i], qb_df[i], qprime_df[i]);
      // a failing engine must not leave the others waiting in an exchange barrier
      if (rc[i]) eng->group->abort();
    });
  for (auto &t : th) t.join();
  for (int i = 0; i < n; i++)
    if (rc[i]) return rc[i];
  return 0;
}

// Per-kernel breakdown of a step: `nsteps` direct (uncaptured) steps of the resident device state
// with an event after every launch on the engine stream; the span between two marks is charged to
// the kernel family of the later one.  Single-stream engines (one rank) only.
// (retry: the per-stage repeat of the steps a persistent launch that gave up left undone, as in
// run_steps: it neither re-probes nor counts as a run of the back-off wait)
static int step_breakdown(hnumo_engine *eng, int nsteps, char *names, int64_t names_len, double *us_per_step,
                          int max_kernels, int *count, bool retry) {
  if (eng->comm_mode != 0 || eng->nranks != 1 || eng->face_halo)
    return fail(eng, HNUMO_ERR_INVALID, "step breakdown: single-rank engines only");
  if (!eng->resident || !eng->uploaded)
    return fail(eng, HNUMO_ERR_INVALID, "step breakdown: needs a resident, uploaded state (hnumo_set_resident)");
  HIPCHK(hipSetDevice(eng->device));
  int rc = retry ? 0 : maybe_reprobe(eng);
  if (rc) return rc;
  hnumo_engine::KMarks km;
  HIPCHK(hipMemsetAsync(eng->neg_flag, 0, sizeof(int), eng->stream));
  HIPCHK(hipMemsetAsync(eng->steps_done, 0, sizeof(unsigned), eng->stream));
  eng->km = &km;
  kmark(eng, "start");
  for (int s = 0; s < nsteps; s++) launch_step(eng);
  eng->km = nullptr;
  auto release = [&]() {
    for (hipEvent_t ev : km.ev) (void)hipEventDestroy(ev);
  };
  if (hipStreamSynchronize(eng->stream) != hipSuccess ||
      hipMemcpy(eng->h_neg, eng->neg_flag, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(eng->h_steps, eng->steps_done, sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess) {
    release();
    return fail(eng, HNUMO_ERR_DEVICE, "step breakdown: HIP error");
  }
  if ((*eng->h_neg & RUN_ABORT) && use_persistent(eng)) {
    // the steps completed before the abort stand (their errors are reported); the rest are redone
    // and timed on per-stage launches, so the state advances by exactly nsteps
    release();
    const int done = (int)*eng->h_steps;
    if ((rc = flag_error(eng, *eng->h_neg & ~RUN_ABORT))) return rc;
    persistent_abort(eng);
    return step_breakdown(eng, nsteps - done, names, names_len, us_per_step, max_kernels, count, true);
  }
  if ((rc = flag_error(eng, *eng->h_neg))) {
    release();
    return rc;
  }
  std::vector<std::string> nm;
  std::vector<double> ms;
  for (size_t i = 1; i < km.n; i++) {
    float dt = 0.f;
    if (hipEventElapsedTime(&dt, km.ev[i - 1], km.ev[i]) != hipSuccess) {
      release();
      return fail(eng, HNUMO_ERR_DEVICE, "step breakdown: event timing failed");
    }
    size_t j = 0;
    while (j < nm.size() && nm[j] != km.name[i]) j++;
    if (j == nm.size()) {
      nm.emplace_back(km.name[i]);
      ms.push_back(0.0);
    }
    ms[j] += dt;
  }
  release();
  std::string joined;
  const int nk = std::min<int>((int)nm.size(), max_kernels);
  for (int j = 0; j < nk; j++) {
    joined += (j ? "\n" : "") + nm[j];
    us_per_step[j] = 1e3 * ms[j] / nsteps;
  }
  if ((int64_t)joined.size() + 1 > names_len) return fail(eng, HNUMO_ERR_INVALID, "step breakdown: names buffer too small");
  std::memcpy(names, joined.c_str(), joined.size() + 1);
  *count = nk;
  return 0;
}

int hnumo_step_breakdown(hnumo_engine *eng, int nsteps, char *names, int64_t names_len, double *us_per_step,
                         int max_kernels, int *count) {
  if (!eng || nsteps < 1 || !names || names_len < 1 || !us_per_step || max_kernels < 1 || !count)
    return HNUMO_ERR_INVALID;
  return step_breakdown(eng, nsteps, names, names_len, us_per_step, max_kernels, count, false);
}

}  // extern "C"

// ------------------------------------------------------------------ stream-copy bandwidth
// The measured HBM denominator of the roofline: a grid-stride 16-byte copy,
// four independent loads in flight per thread before their stores; NT: non-temporal loads and
// stores (the streaming policy); and a one-pass form (stream_copy_pass_kernel).  hnumo_stream_copy_bw
// reports the fastest.
typedef unsigned copy_v4u __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ void __launch_bounds__(256) stream_copy_kernel(const copy_v4u *__restrict__ src, copy_v4u *__restrict__ dst,
                                                          size_t n) {
  const size_t s = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  auto ld = [&](size_t k) -> copy_v4u { return NT ? __builtin_nontemporal_load(src + k) : src[k]; };
  auto st = [&](size_t k, copy_v4u v) {
    if (NT)
      __builtin_nontemporal_store(v, dst + k);
    else
      dst[k] = v;
  };
  for (; i + 3 * s < n; i += 4 * s) {
    const copy_v4u a = ld(i), b = ld(i + s), c = ld(i + 2 * s), d = ld(i + 3 * s);
    st(i, a);
    st(i + s, b);
    st(i + 2 * s, c);
    st(i + 3 * s, d);
  }
  for (; i < n; i += s) st(i, ld(i));
}

// one pass: every block copies its own contiguous 16 KiB (4 x 256 lanes x 16 B), grid = n / 1024
__global__ void __launch_bounds__(256) stream_copy_pass_kernel(const copy_v4u *__restrict__ src,
                                                               copy_v4u *__restrict__ dst, size_t n) {
  const size_t b = (size_t)blockIdx.x * 1024 + threadIdx.x;
  if (b + 768 < n) {
    const copy_v4u x0 = __builtin_nontemporal_load(src + b), x1 = __builtin_nontemporal_load(src + b + 256),
                   x2 = __builtin_nontemporal_load(src + b + 512), x3 = __builtin_nontemporal_load(src + b + 768);
    __builtin_nontemporal_store(x0, dst + b);
    __builtin_nontemporal_store(x1, dst + b + 256);
    __builtin_nontemporal_store(x2, dst + b + 512);
    __builtin_nontemporal_store(x3, dst + b + 768);
  } else {
    for (size_t k = b; k < n && k < b + 1024 - threadIdx.x; k += 256) dst[k] = src[k];
  }
}

extern "C" int hnumo_stream_copy_bw(int device, int64_t bytes, int reps, double *gbs_out2) {
  if (bytes < (1 << 20) || reps < 1 || !gbs_out2) return HNUMO_ERR_INVALID;
  if (hipSetDevice(device) != hipSuccess) return HNUMO_ERR_DEVICE;
  const size_t n = (size_t)bytes / 16;
  void *a = nullptr, *b = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  hipStream_t st = nullptr;
  int rc = HNUMO_ERR_DEVICE;
  if (hipMalloc(&a, n * 16) == hipSuccess && hipMalloc(&b, n * 16) == hipSuccess && hipMemset(a, 0, n * 16) == hipSuccess &&
      hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess && hipEventCreate(&e0) == hipSuccess &&
      hipEventCreate(&e1) == hipSuccess) {
    int ncu = 256;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
    const unsigned grid = (unsigned)std::min<size_t>((size_t)ncu * 16, (n + 255) / 256);
    // per variant: one untimed launch, then `reps` launches back to back between two events (the
    // launch gaps amortised: the rate of a steady copy stream)
    double rate[3] = {0.0, 0.0, 0.0};
    bool ok = true;
    auto launch = [&](int v) {
      if (v == 2)
        hipLaunchKernelGGL(stream_copy_pass_kernel, dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, st,
                           (const copy_v4u *)a, (copy_v4u *)b, n);
      else if (v == 1)
        hipLaunchKernelGGL(stream_copy_kernel<true>, dim3(grid), dim3(256), 0, st, (const copy_v4u *)a, (copy_v4u *)b, n);
      else
        hipLaunchKernelGGL(stream_copy_kernel<false>, dim3(grid), dim3(256), 0, st, (const copy_v4u *)a, (copy_v4u *)b, n);
    };
    for (int v = 0; v < 3 && ok; v++) {
      launch(v);
      ok = hipEventRecord(e0, st) == hipSuccess;
      for (int r = 0; r < reps; r++) launch(v);
      ok = ok && hipEventRecord(e1, st) == hipSuccess && hipEventSynchronize(e1) == hipSuccess;
      float ms = 0.f;
      ok = ok && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms > 0.f;
      if (ok) rate[v] = 2.0 * (double)(n * 16) * reps / (ms * 1e-3) / 1e9;
    }
    if (ok && hipGetLastError() == hipSuccess) {
      const int w = (rate[1] > rate[0]) ? (rate[2] > rate[1] ? 2 : 1) : (rate[2] > rate[0] ? 2 : 0);
      gbs_out2[0] = rate[w];
      gbs_out2[1] = (double)w;
      rc = 0;
    }
  }
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  if (a) (void)hipFree(a);
  if (b) (void)hipFree(b);
  return rc;
}
