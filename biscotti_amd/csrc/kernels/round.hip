// Native round driver pieces: the secure aggregation a round queues behind the committee's selection,
// enqueued from C++ in ONE call instead of ~25 Python-level tensor / stream operations (each 5-20 us
// of the round's host thread, which is the round's critical path).
//
// bsc_round_secagg  -- the miners' sums and the leader's recovery (aggregateSecret + recoverSecret,
//                      DistSys/kyber.go:244-287,809-857) for the rows the selection kept:
//                        side: chunk-commitment sums of the kept rows (the audit's input)
//                        wit:  witness sums (no consumer on the protocol path; own low-priority stream)
//                        main: fused share sums + exact recovery + W update (k_recover_w), then the
//                              read-back of (status, W_new) into pinned memory, event `readback`
// bsc_round_audit   -- verifyCommitment on the aggregate (kyber.go:564-577): main waits for the side
//                      stream's sums, k_chunk_check, read-back of the verdicts, event `audit`
// bsc_round_wait    -- host wait for one of the two events
// bsc_round_partials / bsc_round_combine -- the same aggregation on several ranks, split around the one
//                      all_gather the caller issues between them (below)
//
// The launchers of the individual kernels (msm.hip, ml.hip) are called directly; every buffer is
// resident (allocated once by the engine), so the call allocates nothing.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>   // types only: the entry points are resolved at run time (bsc_rccl_load)
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <thread>

extern "C" int bsc_sum_rows2(const uint32_t* pts, int ncols_in, const int* rows, int nrows, const int* cols,
                             int ncols, const int* row_mask, uint32_t* out, void* stream);
extern "C" int bsc_recover_w(const long long* ys, int nrows, int nch, int T, const int* mask, const int* ycols,
                             const int* xs, int npts, const long long* A, const int* basis, int poly, int shift,
                             unsigned long long inv_lo, unsigned long long inv_hi, int d, const double* W,
                             double qscale, double* W_new, long long* coeffs, int* status, long long* agg_out,
                             void* stream);
extern "C" int bsc_recover_w_strided(const long long* ys, int nrows, long long rstride, int nch, int T, const int* mask,
                                     const int* ycols, const int* xs, int npts, const long long* A, const int* basis,
                                     int poly, int shift, unsigned long long inv_lo, unsigned long long inv_hi, int d,
                                     const double* W, double qscale, double* W_new, long long* coeffs, int* status,
                                     long long* agg_out, double* h_W, int* h_status, void* stream);
extern "C" int bsc_recover_w_clock(const long long* ys, int nrows, long long rstride, int nch, int T, const int* mask,
                                   const int* ycols, const int* xs, int npts, const long long* A, const int* basis,
                                   int poly, int shift, unsigned long long inv_lo, unsigned long long inv_hi, int d,
                                   const double* W, double qscale, double* W_new, long long* coeffs, int* status,
                                   long long* agg_out, double* h_W, int* h_status, long long* h_clock, void* stream);
extern "C" int bsc_segment_sum_h(const uint32_t* pts, int ngroups, int n, int stride, int off, uint32_t* out,
                                 uint32_t* hout, void* stream);
extern "C" int bsc_chunk_check_h(const long long* coeffs, int d, int poly, const uint32_t* tbl_pk, int B0, int NW,
                                 const uint32_t* csum, int nm, int nch, int* ok, int* h_ok, void* stream);
extern "C" int bsc_sum_rows_i64(const long long* ys, int R, long long C, const int* rows, int nsel, const int* mask,
                                long long* out, void* stream);
extern "C" int bsc_sum_rows_i64_tail(const long long* ys, int R, long long C, const int* mask, long long* out,
                                     long long tail, void* stream);
extern "C" int bsc_sum_cols_serial(const uint32_t* pts, int ncols_in, int nrows, const int* cols, int ncols,
                                   const int* row_mask, uint32_t* out, void* stream);
extern "C" int bsc_sum_rows2_pos(const uint32_t* pts, int ncols_in, const int* rows, int nrows, const int* cols,
                                 int ncols, const int* row_mask, uint32_t* out, void* stream);
extern "C" int bsc_shares_msm(const long long* coeffs, int d, const int* rows, int nrows, const uint32_t* tbl_pk,
                              const uint32_t* tbl_wb, int poly, int T, int B0, int NW, int commit_only,
                              const int* alive, const int* compact, int group_rows, uint32_t* out_pts,
                              long long* out_y, void* stream);
extern "C" int bsc_softmax_step_ones(const float* X, const int* y, const long long* off, const int* ntrain,
                                     const int* pid, const double* W, int D_IN, int D_OUT, int B, int P,
                                     unsigned long long seed, int iteration, float max_norm, double qscale, float* delta,
                                     long long* qdelta, float* loss, int lo, int* ones, int nones, void* stream);
extern "C" int bsc_shares_msm_ka(const long long* coeffs, int d, const int* rows_host, int nrows, const uint32_t* tbl_pk,
                                 const uint32_t* tbl_wb, int poly, int T, int B0, int NW, int commit_only,
                                 const int* alive, int group_rows, uint32_t* out_pts, long long* out_y, void* stream);
#define ROWARG_MAX 248   // msm.hip: rows passed in the MSM kernel's arguments
extern "C" int bsc_gram_stacked(const float* X, int U1, const float* X2, int U2, long long stride2, int D, int kchunk,
                                double* part, double* gram, unsigned int* count, const double* nn, void* stream);
extern "C" int bsc_segment_sum(const uint32_t* pts, int ngroups, int n, int stride, int off, uint32_t* out,
                               void* stream);
extern "C" int bsc_gram_stacked_range(const float* X, int U1, const float* X2, int U2, long long stride2, int D,
                                      int kchunk, int p0, int p1, double* part, double* gram, unsigned int* count,
                                      const double* nn, void* stream);
extern "C" int bsc_commit_rows(const long long* coeffs, int d, const int* rows, int nrows, const uint32_t* tbl_pk,
                               int B0, int NW, uint32_t* partial, uint32_t* out, void* stream);
extern "C" int bsc_chunk_check(const long long* coeffs, int d, int poly, const uint32_t* tbl_pk, int B0, int NW,
                               const uint32_t* csum, int nm, int nch, int* ok, void* stream);

extern "C" int bsc_set_alive(const int* accept, const int* src, int n, int* alive, void* stream);

namespace {
// resident state of the fused round calls (bsc_round_bind_* / bsc_round_add_*, registered once per run)
struct Layout {   // one miner layout: which share columns the contributing miners hold, its recovery weights
  const int *ccols, *wcols, *ycols, *xs, *basis;
  int nwc, npts, shift;
  const long long* A;
  unsigned long long inv_lo, inv_hi;
  long long* agg;   // [nch][npts] resident output
  uint32_t* ws;     // [nwc][24] resident witness sums
};
struct PreSlot {  // one slot of the pre-step's output ring
  float* delta;
  long long* qdelta;
  float* loss;
  uint32_t *ccom, *jac, *jac_host;
  double *part, *gram;
  hipEvent_t ev_step, ev_ccom, ev_commit, ev_gram;
};
struct TaskCfg {  // the softmax task's resident data and the pre-step's constants
  int bound = 0;
  hipStream_t gram;
  const float* X;
  const int *y, *ntrain, *pid, *rows_arange;
  const long long* off;
  int d_in, d_out, B, P, lo, kchunk;
  unsigned long long seed;
  float max_norm;
  double qs;
  const uint32_t* tbl_wb;
  const float* noise;       // resident noise table [N][100][d] (nullptr: no noise-aware Gram)
  int noise_n;
  const double* nn_tab;     // [100][N][N] Gram of each iteration's noise rows (nullptr: computed every round)
  unsigned int* counters;
};
struct RoundCtx {
  hipStream_t main, side, bg;
  hipStream_t wit;   // the miners' witness sums (no consumer in the round; default: bg)
  hipEvent_t ev_main, ev_side, ev_readback, ev_audit, ev_pre;
  // the audit's read-back is double-buffered (event + pinned row aud_k of h_ok): a round's audit can be read
  // after the next round's aggregation was queued (the speculative front, engine._spec_front_launch)
  hipEvent_t ev_audit1;
  int aud_k = 0;
  const uint32_t* tbl_pk;
  int d, poly, T, nch, b0, nw;
  double qscale;
  // fused-call state
  double* W_ring[8];
  int nW = 0, Wk = 0;
  const void* recent[2] = {nullptr, nullptr};
  long long* coeffs = nullptr;
  int *status = nullptr, *ok = nullptr, *h_status = nullptr, *h_ok = nullptr;
  uint32_t* cs = nullptr;
  double* h_W = nullptr;
  Layout layouts[256];
  int nlayouts = 0;
  PreSlot pre[8];
  int npre = 0, pre_k = 0;
  TaskCfg task;
  // the speculative MSM's output ring (bsc_round_set_spec_ring): per slot the rows' flags (cap entries), an
  // event on the background stream after the slot's last reader (the witness sums), whether the next
  // pre-step has set the flags already; spec_k = the slot of the last launch
  int* spec_alive[8];
  hipEvent_t spec_done[8];
  bool spec_used[8], spec_filled[8];
  int nspec = 0, spec_cap = 0, spec_k = -1;
  // several ranks (bsc_round_comm_init): the round's own RCCL communicator -- every collective of a round goes
  // through it, on ONE comm stream, in the order the round issues them (the same on every rank) -- or, emulating
  // rank 0 of a `cworld`-rank job on one GPU, local copies of rank 0's contribution into every slot
  ncclComm_t comm = nullptr;
  int cworld = 1, crank = 0, emulate = 0;
  long long timeout_ns = 0;   // bsc_round_wait gives up (and aborts the communicator) after this; 0: never
  hipStream_t cstream = nullptr;
  hipEvent_t ev_c0 = nullptr, ev_c1 = nullptr;
  // the multi-rank aggregation's resident buffers and the next Gram's inputs (bsc_round_bind_multi)
  struct Multi {
    int bound = 0;
    unsigned char *send = nullptr, *recv = nullptr;
    long long row_bytes = 0;
    long long* h_clock = nullptr;
    int maxlocal = 0, U1 = 0, p0 = 0, p1 = 0, chunk = 0;
    float *pad = nullptr, *X = nullptr;      // [maxlocal][d] send buffer (ranks with fewer peers), [world maxlocal][d]
    double* part = nullptr;                  // [nsplit][p1 - p0][256] split-K partials of this rank's tile pairs
    unsigned char* vg_recv[2] = {nullptr, nullptr};   // the verification gather's rows (alternating by iteration)
    long long vg_row_bytes = 0;
  } m;
};
#define RC_CHECK(x)                        \
  do {                                     \
    const int e_ = (int)(x);               \
    if (e_ != 0) return e_;                \
  } while (0)
// the speculative slot whose flags `mask` is (-1: not a speculative slot's)
static int spec_slot_of(const RoundCtx* c, const int* mask) {
  for (int i = 0; i < c->nspec; ++i)
    if (c->spec_alive[i] == mask) return i;
  return -1;
}
// after the witness sums over a speculative slot: the slot's last reader is queued (witness stream)
static int spec_mark_read(RoundCtx* c, const int* mask) {
  const int s = spec_slot_of(c, mask);
  if (s >= 0) {
    RC_CHECK(hipEventRecord(c->spec_done[s], c->wit));
    c->spec_used[s] = true;
  }
  return 0;
}
}  // namespace

extern "C" void* bsc_round_create(void* main, void* side, void* bg, const uint32_t* tbl_pk, int d, int poly, int T,
                                  int b0, int nw, double qscale) {
  RoundCtx* c = new RoundCtx();
  c->main = (hipStream_t)main;
  c->side = (hipStream_t)side;
  c->bg = (hipStream_t)bg;
  c->wit = c->bg;
  c->tbl_pk = tbl_pk;
  c->d = d;
  c->poly = poly;
  c->T = T;
  c->nch = (d + poly - 1) / poly;
  c->b0 = b0;
  c->nw = nw;
  c->qscale = qscale;
  hipEvent_t* evs[6] = {&c->ev_main, &c->ev_side, &c->ev_readback, &c->ev_audit, &c->ev_pre, &c->ev_audit1};
  for (hipEvent_t* e : evs)
    if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
      delete c;
      return nullptr;
    }
  return c;
}

// The witness sums' own stream: on the background stream they queued the pre-step's commitments -- which the
// round's block carries -- behind ~0.5 ms of low-priority sums (the block build then waited for them).
extern "C" int bsc_round_set_witness_stream(void* ctx, void* stream) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || stream == nullptr) return -1;
  c->wit = (hipStream_t)stream;
  return 0;
}

extern "C" int bsc_wave_prio_ml(int on);
extern "C" int bsc_wave_prio_msm(int on);
extern "C" int bsc_wave_prio_vrf(int on);
// the round kernels' wave priority classes (kernels/wave_prio.h) on or off, in every kernel file
extern "C" int bsc_wave_prio(int on) {
  RC_CHECK(bsc_wave_prio_ml(on));
  RC_CHECK(bsc_wave_prio_msm(on));
  return bsc_wave_prio_vrf(on);
}

namespace {
// The RCCL entry points of the library the process already runs (torch's, which owns the other communicators):
// resolved once by bsc_rccl_load, so one RCCL instance serves the process.
struct RcclApi {
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
};
RcclApi g_rccl;
}  // namespace

extern "C" void bsc_round_destroy(void* ctx) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr) return;
  if (c->comm != nullptr && g_rccl.comm_destroy != nullptr) g_rccl.comm_destroy(c->comm);
  if (c->ev_c0 != nullptr) (void)hipEventDestroy(c->ev_c0);
  if (c->ev_c1 != nullptr) (void)hipEventDestroy(c->ev_c1);
  hipEventDestroy(c->ev_main);
  hipEventDestroy(c->ev_side);
  hipEventDestroy(c->ev_readback);
  hipEventDestroy(c->ev_audit);
  hipEventDestroy(c->ev_audit1);
  hipEventDestroy(c->ev_pre);
  for (int i = 0; i < c->nspec; ++i) hipEventDestroy(c->spec_done[i]);
  delete c;
}

// pts [R][nch * (T + 1)][24] Jacobian shares + chunk commitments of the speculative rows, ys [R][nch][T]
// share values, mask [R] the selection's keep flags; ccols [nch] / wcols [nwc] the commitment and witness
// columns, ycols / xs [npts] the contributing miners' share columns and x-points; A / basis / shift /
// inv the exact recovery weights of this miner layout; W the current model.  Outputs (resident):
// W_new [d], coeffs [nch][poly], status [nch], agg [nch][npts], cs [nch][24], ws [nwc][24]; pinned host
// copies h_status [nch], h_W [d].  audit = 0: no commitment sums.
extern "C" int bsc_round_secagg(void* ctx, const uint32_t* pts, int R, const long long* ys, const int* mask,
                                const int* ccols, const int* wcols, int nwc, const int* ycols, const int* xs, int npts,
                                const long long* A, const int* basis, int shift, unsigned long long inv_lo,
                                unsigned long long inv_hi, const double* W, double* W_new, long long* coeffs,
                                int* status, long long* agg, uint32_t* cs, uint32_t* ws, int* h_status, double* h_W,
                                int audit) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || R <= 0) return -1;
  const int ncols_in = c->nch * (c->T + 1);
  RC_CHECK(hipEventRecord(c->ev_main, c->main));
  if (audit == 1) {   // audit == 2: the commitment sums were queued early (bsc_round_csum_early)
    RC_CHECK(hipStreamWaitEvent(c->side, c->ev_main, 0));
    RC_CHECK(bsc_sum_rows2(pts, ncols_in, nullptr, R, ccols, c->nch, mask, cs, c->side));
    RC_CHECK(hipEventRecord(c->ev_side, c->side));
  }
  RC_CHECK(hipStreamWaitEvent(c->wit, c->ev_main, 0));
  RC_CHECK(bsc_sum_cols_serial(pts, ncols_in, R, wcols, nwc, mask, ws, c->wit));
  RC_CHECK(spec_mark_read(c, mask));
  // the recovery writes (status, W_new) into the pinned read-back buffers itself: no copies behind it
  RC_CHECK(bsc_recover_w_strided(ys, R, (long long)c->nch * c->T, c->nch, c->T, mask, ycols, xs, npts, A, basis,
                                 c->poly, shift, inv_lo, inv_hi, c->d, W, c->qscale, W_new, coeffs, status, agg, h_W,
                                 h_status, c->main));
  RC_CHECK(hipEventRecord(c->ev_readback, c->main));
  return 0;
}

// h_ok: [2][nch] pinned; this audit's verdicts go to row aud_k (flipped per audit, bsc_round_audit_slot)
extern "C" int bsc_round_audit(void* ctx, const long long* coeffs, const uint32_t* cs, int* ok, int* h_ok) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr) return -1;
  c->aud_k ^= 1;
  RC_CHECK(hipStreamWaitEvent(c->main, c->ev_side, 0));
  RC_CHECK(bsc_chunk_check_h(coeffs, c->d, c->poly, c->tbl_pk, c->b0, c->nw, cs, 1, c->nch, ok,
                             h_ok + (size_t)c->aud_k * c->nch, c->main));
  RC_CHECK(hipEventRecord(c->aud_k ? c->ev_audit1 : c->ev_audit, c->main));
  return 0;
}

// the h_ok row (and bsc_round_wait's 2 + slot) of the audit queued last
extern "C" int bsc_round_audit_slot(void* ctx) {
  RoundCtx* c = (RoundCtx*)ctx;
  return c == nullptr ? -1 : c->aud_k;
}

// The audit's commitment sums taken early, from the pre-step's per-peer chunk commitments instead of the
// share MSM's commitment slots: as soon as the committee's selection has set the speculative rows' flags
// (queued on main before main waits for the MSM), the side stream sums ccom[rows[r]] over the rows r
// still alive -- the same rows the share sums use -- while the MSM is still running.  ccom: Jacobian
// [npeer][nch][24], produced on another stream (ev_ccom).  bsc_round_secagg(.., audit = 2) then skips
// its own commitment sums and bsc_round_audit waits for these.
// `stream`: where the sums run -- NOT the side stream, which is still busy with the share MSM (they would
// queue behind it); nullptr = the side stream.
extern "C" int bsc_round_csum_early(void* ctx, const uint32_t* ccom, void* ev_ccom, const int* rows, int R,
                                    const int* mask, uint32_t* cs, void* stream) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || R <= 0) return -1;
  hipStream_t st = stream != nullptr ? (hipStream_t)stream : c->side;
  RC_CHECK(hipEventRecord(c->ev_main, c->main));
  RC_CHECK(hipStreamWaitEvent(st, c->ev_main, 0));
  if (ev_ccom != nullptr) RC_CHECK(hipStreamWaitEvent(st, (hipEvent_t)ev_ccom, 0));
  RC_CHECK(bsc_sum_rows2_pos(ccom, c->nch, rows, R, nullptr, c->nch, mask, cs, st));
  RC_CHECK(hipEventRecord(c->ev_side, st));
  return 0;
}

// The speculative MSM's slot ring: nslots slots whose row flags are alive[k] (cap entries each).  Registered
// once; the pre-steps then set the next slot's flags to 1 inside the local step (which the MSM waits for).
extern "C" int bsc_round_set_spec_ring(void* ctx, int* const* alive, int nslots, int cap) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || nslots < 3 || nslots > 8 || cap <= 0) return -1;
  for (int i = 0; i < c->nspec; ++i) hipEventDestroy(c->spec_done[i]);
  c->nspec = 0;
  for (int i = 0; i < nslots; ++i) {
    c->spec_alive[i] = alive[i];
    RC_CHECK(hipEventCreateWithFlags(&c->spec_done[i], hipEventDisableTiming));
    c->spec_used[i] = c->spec_filled[i] = false;
    c->nspec = i + 1;
  }
  c->spec_cap = cap;
  c->spec_k = -1;
  return 0;
}

// The next round's speculative share MSM (head.py _spec_head_launch) into ring slot `slot` (which must be the
// next one): the side stream waits for the pre-step (ev_wait: its quantised updates) and for the slot's last
// reader, sets the slot's flags unless a pre-step did, and runs the MSM over rows_host (pinned, n rows) into
// pts / ys.  Up to ROWARG_MAX rows travel in the kernel's arguments, so nothing stands between the launch and
// the MSM (an upload's copy kernel waited 20-120 us for a CU slot behind the round's work); the device copy
// of the row list (rows_dev: the early audit sums read it) then goes up on `up` (high priority; event ev_up),
// which is also where those sums run.  More rows: the copy first, and the MSM reads rows_dev.
extern "C" int bsc_round_spec_msm2(void* ctx, int slot, void* ev_wait, const long long* coeffs, const int* rows_host,
                                   int n, const uint32_t* tbl_wb, int commit_only, int group_rows, uint32_t* pts,
                                   long long* ys, int* rows_dev, void* up, void* ev_up, void* ev_flags) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || n <= 0 || c->nspec == 0 || n > c->spec_cap || up == nullptr || ev_up == nullptr ||
      ev_flags == nullptr)
    return -1;
  if (slot != (c->spec_k + 1) % c->nspec) return -5;
  c->spec_k = slot;
  int* alive = c->spec_alive[slot];
  hipStream_t st = (hipStream_t)up;
  if (ev_wait != nullptr) RC_CHECK(hipStreamWaitEvent(c->side, (hipEvent_t)ev_wait, 0));
  if (c->spec_used[slot]) RC_CHECK(hipStreamWaitEvent(c->side, c->spec_done[slot], 0));
  if (!c->spec_filled[slot]) RC_CHECK(hipMemsetD32Async((hipDeviceptr_t)alive, 1, (size_t)n, c->side));
  c->spec_filled[slot] = false;
  // the flags are set from here on: the selection's writes to them (main) wait for this
  RC_CHECK(hipEventRecord((hipEvent_t)ev_flags, c->side));
  if (n <= ROWARG_MAX) {
    RC_CHECK(bsc_shares_msm_ka(coeffs, c->d, rows_host, n, c->tbl_pk, tbl_wb, c->poly, c->T, c->b0, c->nw, commit_only,
                               alive, group_rows, pts, ys, c->side));
    RC_CHECK(hipMemcpyAsync(rows_dev, rows_host, (size_t)n * sizeof(int), hipMemcpyHostToDevice, st));
    RC_CHECK(hipEventRecord((hipEvent_t)ev_up, st));
    return 0;
  }
  RC_CHECK(hipMemcpyAsync(rows_dev, rows_host, (size_t)n * sizeof(int), hipMemcpyHostToDevice, st));
  RC_CHECK(hipEventRecord((hipEvent_t)ev_up, st));
  RC_CHECK(hipStreamWaitEvent(c->side, (hipEvent_t)ev_up, 0));
  return bsc_shares_msm(coeffs, c->d, rows_dev, n, c->tbl_pk, tbl_wb, c->poly, c->T, c->b0, c->nw, commit_only, alive,
                        nullptr, group_rows, pts, ys, c->side);
}

// A block that reaches past the speculative MSM's rows (a speculative miss: its horizon was too short): the missing
// rows' shares go into the SAME ring slot behind its n rows, so one aggregation reads them all.  Behind everything
// queued on main so far (the aggregation that already read the slot) the side stream uploads the slot's flags
// (keep_host [n + m]: the host-decided block rows among the speculative ones, 1 for the new ones) and runs the MSM
// over rows_host [m] into rows n.. of pts / ys; the new rows' device list goes up on `up` (event ev_up).
extern "C" int bsc_round_spec_topup(void* ctx, int slot, const int* keep_host, int n, const int* rows_host, int m,
                                    const long long* coeffs, const uint32_t* tbl_wb, int commit_only, int group_rows,
                                    uint32_t* pts_n, long long* ys_n, int* rows_dev_n, void* up, void* ev_up) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || slot < 0 || slot >= c->nspec || n < 0 || m < 0 || n + m <= 0 || n + m > c->spec_cap ||
      up == nullptr || ev_up == nullptr)
    return -1;
  int* alive = c->spec_alive[slot];
  RC_CHECK(hipEventRecord(c->ev_main, c->main));
  RC_CHECK(hipStreamWaitEvent(c->side, c->ev_main, 0));
  RC_CHECK(hipMemcpyAsync(alive, keep_host, (size_t)(n + m) * sizeof(int), hipMemcpyHostToDevice, c->side));
  hipStream_t st = (hipStream_t)up;
  if (m > 0) {   // (m = 0: every block row was speculative -- only the flags change)
    RC_CHECK(bsc_shares_msm_ka(coeffs, c->d, rows_host, m, c->tbl_pk, tbl_wb, c->poly, c->T, c->b0, c->nw,
                               commit_only, alive + n, group_rows, pts_n, ys_n, c->side));
    RC_CHECK(hipMemcpyAsync(rows_dev_n, rows_host, (size_t)m * sizeof(int), hipMemcpyHostToDevice, st));
  }
  RC_CHECK(hipEventRecord((hipEvent_t)ev_up, st));
  return 0;   // (the aggregation that reads the slot again re-marks it read: spec_mark_read)
}

// The next round's pre-step (head.py _queue_pre_step) in one call, queued behind everything on main so far
// (the recovery of W):
//   gram stream: local SGD step of every local peer (delta, qdelta, loss), event ev_step; then, when
//                do_gram, the noise-aware Krum's phase-1 Gram of [delta; this iteration's noise rows],
//                event ev_gram
//   background:  behind the step, the per-chunk commitments of every row (ccom, event ev_ccom), their
//                per-row sums = the full commitments (jac), read back into pinned jac_host, event ev_commit
// Outputs are resident (the caller rotates them over slots); events are caller-owned and re-recorded.
static int prestep_impl(RoundCtx* c, hipStream_t gs, const float* X, const int* y, const long long* off,
                        const int* ntrain, const int* pid, const double* W, int d_in, int d_out, int B, int P,
                        unsigned long long seed, int iteration, float max_norm, double qscale, int lo, float* delta,
                        long long* qdelta, float* loss, const uint32_t* tbl_wb, const int* rows_arange, uint32_t* ccom,
                        uint32_t* jac, uint32_t* jac_host, int do_gram, const float* T_rows, int U2, long long stride2,
                        int kchunk, double* part, double* gram, unsigned int* counters, void* ev_step, void* ev_ccom,
                        void* ev_commit, void* ev_gram, int chunked, hipStream_t cst, int* ones, int nones,
                        hipEvent_t ones_wait, const double* nn) {
  if (c == nullptr || P <= 0 || d_in * d_out + d_out != c->d) return -1;
  RC_CHECK(hipEventRecord(c->ev_pre, c->main));
  RC_CHECK(hipStreamWaitEvent(gs, c->ev_pre, 0));
  if (ones_wait != nullptr) RC_CHECK(hipStreamWaitEvent(gs, ones_wait, 0));
  RC_CHECK(bsc_softmax_step_ones(X, y, off, ntrain, pid, W, d_in, d_out, B, P, seed, iteration, max_norm, qscale, delta,
                                 qdelta, loss, lo, ones, nones, gs));
  RC_CHECK(hipEventRecord((hipEvent_t)ev_step, gs));
  RC_CHECK(hipStreamWaitEvent(cst, (hipEvent_t)ev_step, 0));
  if (chunked) {
    RC_CHECK(bsc_shares_msm(qdelta, c->d, rows_arange, P, c->tbl_pk, tbl_wb, c->poly, c->T, c->b0, c->nw, 1, nullptr,
                            nullptr, 0, ccom, nullptr, cst));
    RC_CHECK(hipEventRecord((hipEvent_t)ev_ccom, cst));
    RC_CHECK(bsc_segment_sum_h(ccom, P, c->nch, 1, 0, jac, jac_host, cst));   // full commitments + host mirror
  } else {   // full commitments only (1024-coefficient slabs; ccom is the slab-partials scratch)
    RC_CHECK(bsc_commit_rows(qdelta, c->d, rows_arange, P, c->tbl_pk, c->b0, c->nw, ccom, jac, cst));
    RC_CHECK(hipMemcpyAsync(jac_host, jac, (size_t)P * 24 * sizeof(uint32_t), hipMemcpyDeviceToHost, cst));
  }
  RC_CHECK(hipEventRecord((hipEvent_t)ev_commit, cst));
  if (do_gram) {
    RC_CHECK(bsc_gram_stacked(delta, P, T_rows, U2, stride2, c->d, kchunk, part, gram, counters, nn, gs));
    RC_CHECK(hipEventRecord((hipEvent_t)ev_gram, gs));
  }
  return 0;
}

extern "C" int bsc_round_prestep(void* ctx, void* gram_stream, const float* X, const int* y, const long long* off,
                                 const int* ntrain, const int* pid, const double* W, int d_in, int d_out, int B, int P,
                                 unsigned long long seed, int iteration, float max_norm, double qscale, int lo,
                                 float* delta, long long* qdelta, float* loss, const uint32_t* tbl_wb,
                                 const int* rows_arange, uint32_t* ccom, uint32_t* jac, uint32_t* jac_host,
                                 int do_gram, const float* T_rows, int U2, long long stride2, int kchunk, double* part,
                                 double* gram, unsigned int* counters, void* ev_step, void* ev_ccom, void* ev_commit,
                                 void* ev_gram, int chunked, void* commit_stream) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr) return -1;
  // the commitments' stream (default: background; an A/B passes one masked to the CUs the MSM leaves)
  hipStream_t cst = commit_stream != nullptr ? (hipStream_t)commit_stream : c->bg;
  return prestep_impl(c, (hipStream_t)gram_stream, X, y, off, ntrain, pid, W, d_in, d_out, B, P, seed, iteration,
                      max_norm, qscale, lo, delta, qdelta, loss, tbl_wb, rows_arange, ccom, jac, jac_host, do_gram,
                      T_rows, U2, stride2, kchunk, part, gram, counters, ev_step, ev_ccom, ev_commit, ev_gram, chunked,
                      cst, nullptr, 0, nullptr, nullptr);
}

// ---------------------------------------------------------------------------------------------------------
// Several ranks (one per GPU).  The aggregation's ONE all_gather moves a packed row per rank,
//     [ cs: nch x 24 u32 | ys: nch x T int64 | clock: int64 | pad ]      (row_bytes: a multiple of 96)
// so the gathered buffer is at once a [world][row_bytes / 96][24] point array whose first nch columns are the
// ranks' chunk-commitment partial sums (bsc_sum_rows2 sums them) and a strided [world][nch][T] share-sum
// array (k_recover_w with a row stride sums and recovers).  No repacking on either side of the collective.
// (The native path, bsc_round_agg_multi, gathers the same send row in two pieces -- [ys | clock] for the recovery
// first, [cs] for the audit behind the early commitment sums -- into recv = [world][cs] + [world][ys | clock].)
//
// bsc_round_partials: this rank's partials of its kept rows, written straight into its send row -- the
//   miners' share-value sums (main), the chunk-commitment sums (side, or already queued on another stream by
//   bsc_round_csum_early into the same slot: audit = 2), the witness sums (background; per-rank, no
//   consumer on the protocol path), the rank's clock; main then waits for the commitment sums, so the
//   collective the caller issues next on main sees a complete row.  R = 0: no local rows (zero partials,
//   the point at infinity for the commitment sums).
// bsc_round_combine: on main, behind the collective: the commitment totals over the ranks (the audit's
//   input), the fused share totals + exact recovery + W update, and the read-back of (status, W_new, every
//   rank's clock) -- event `readback`.
extern "C" int bsc_round_row_bytes(int nch, int T) {
  const long long raw = 96ll * nch + 8ll * nch * T + 8;
  return (int)((raw + 95) / 96 * 96);
}

static int partials_impl(void* ctx, const uint32_t* pts, int R, const long long* ys, const int* mask, const int* ccols,
                         const int* wcols, int nwc, uint32_t* ws, unsigned char* send, long long clock, int audit,
                         int wait_cs, int defer_wit = 0);

extern "C" int bsc_round_partials(void* ctx, const uint32_t* pts, int R, const long long* ys, const int* mask,
                                  const int* ccols, const int* wcols, int nwc, uint32_t* ws, unsigned char* send,
                                  long long clock, int audit) {
  return partials_impl(ctx, pts, R, ys, mask, ccols, wcols, nwc, ws, send, clock, audit, 1);
}

// wait_cs = 0: main does not wait for the commitment partials (the native path gathers them separately);
// defer_wit = 1: no witness sums here (the caller queues them after the recovery: they have no consumer in the round)
static int partials_impl(void* ctx, const uint32_t* pts, int R, const long long* ys, const int* mask, const int* ccols,
                         const int* wcols, int nwc, uint32_t* ws, unsigned char* send, long long clock, int audit,
                         int wait_cs, int defer_wit) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || R < 0) return -1;
  const int nch = c->nch, T = c->T;
  uint32_t* cs_slot = (uint32_t*)send;
  long long* ys_slot = (long long*)(send + 96ll * nch);
  unsigned char* clk = send + 96ll * nch + 8ll * nch * T;
  RC_CHECK(hipEventRecord(c->ev_main, c->main));
  if (R > 0) {
    const int ncols_in = nch * (T + 1);
    if (audit == 1) {
      RC_CHECK(hipStreamWaitEvent(c->side, c->ev_main, 0));
      RC_CHECK(bsc_sum_rows2(pts, ncols_in, nullptr, R, ccols, nch, mask, cs_slot, c->side));
      RC_CHECK(hipEventRecord(c->ev_side, c->side));
    }
    if (nwc > 0 && ws != nullptr && !defer_wit) {
      RC_CHECK(hipStreamWaitEvent(c->wit, c->ev_main, 0));
      RC_CHECK(bsc_sum_cols_serial(pts, ncols_in, R, wcols, nwc, mask, ws, c->wit));
      RC_CHECK(spec_mark_read(c, mask));
    }
  } else if (audit != 0) {
    RC_CHECK(hipMemsetAsync(cs_slot, 0, 96ull * nch, c->main));
  }
  // the share-value sums (zeros without local rows) and the clock right behind them, in one launch
  if ((long long*)clk != ys_slot + (long long)nch * T) return -1;
  RC_CHECK(bsc_sum_rows_i64_tail(R > 0 ? ys : nullptr, R > 0 ? R : 0, (long long)nch * T, R > 0 ? mask : nullptr,
                                 ys_slot, clock, c->main));
  if (R > 0 && audit != 0 && wait_cs) RC_CHECK(hipStreamWaitEvent(c->main, c->ev_side, 0));
  return 0;
}

extern "C" int bsc_round_combine(void* ctx, const unsigned char* recv, int world, long long row_bytes,
                                 const int* ycols, const int* xs, int npts, const long long* A, const int* basis,
                                 int shift, unsigned long long inv_lo, unsigned long long inv_hi, const double* W,
                                 double* W_new, long long* coeffs, int* status, long long* agg, uint32_t* cs,
                                 int* h_status, double* h_W, long long* h_clock, int audit) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || world <= 0 || row_bytes % 96 != 0 || row_bytes < bsc_round_row_bytes(c->nch, c->T)) return -1;
  const int nch = c->nch, T = c->T;
  if (audit != 0) {
    RC_CHECK(bsc_sum_rows2((const uint32_t*)recv, (int)(row_bytes / 96), nullptr, world, nullptr, nch, nullptr, cs,
                           c->main));
    RC_CHECK(hipEventRecord(c->ev_side, c->main));   // bsc_round_audit waits for the sums through ev_side
  }
  // (every rank's clock is mirrored to h_clock by the recovery itself: no strided read-back copy behind it)
  RC_CHECK(bsc_recover_w_clock((const long long*)(recv + 96ll * nch), world, row_bytes / 8, nch, T, nullptr, ycols, xs,
                               npts, A, basis, c->poly, shift, inv_lo, inv_hi, c->d, W, c->qscale, W_new, coeffs, status,
                               agg, h_W, h_status, h_clock, c->main));
  RC_CHECK(hipEventRecord(c->ev_readback, c->main));
  return 0;
}

// ---------------------------------------------------------------------------------------------------------
// Fused round calls.  The host loop of a round is its critical path; each Python-level launch with its
// argument marshalling costs 5-60 us of it.  The buffers these calls use are registered once per run
// (model ring, outputs, miner layouts, pre-step slots, the task), so one call per phase takes a handful of
// arguments:
//   bsc_round_after_select   behind the committee's selection (one rank): the speculative rows' flags
//                            (k_set_alive), the early audit sums, the miners' sums + recovery + read-back,
//                            the next round's pre-step, the audit -- what NativeSecAgg.secagg + prestep +
//                            audit and four Python helpers did in ~130 us of host time
//   bsc_round_select_partials / bsc_round_after_gather   the same on several ranks, split around the
//                            aggregation's all_gather
extern "C" int bsc_round_bind_outputs(void* ctx, double* const* W_ring, int nW, long long* coeffs, int* status,
                                      uint32_t* cs, int* ok, int* h_status, double* h_W, int* h_ok) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || nW < 3 || nW > 8) return -1;
  for (int i = 0; i < nW; ++i) c->W_ring[i] = W_ring[i];
  c->nW = nW;
  c->coeffs = coeffs;
  c->status = status;
  c->cs = cs;
  c->ok = ok;
  c->h_status = h_status;
  c->h_W = h_W;
  c->h_ok = h_ok;
  return 0;
}

extern "C" int bsc_round_add_layout(void* ctx, const int* ccols, const int* wcols, int nwc, const int* ycols,
                                    const int* xs, int npts, const long long* A, const int* basis, int shift,
                                    unsigned long long inv_lo, unsigned long long inv_hi, long long* agg, uint32_t* ws) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || c->nlayouts >= 256) return -1;
  Layout& L = c->layouts[c->nlayouts];
  L.ccols = ccols;
  L.wcols = wcols;
  L.nwc = nwc;
  L.ycols = ycols;
  L.xs = xs;
  L.npts = npts;
  L.A = A;
  L.basis = basis;
  L.shift = shift;
  L.inv_lo = inv_lo;
  L.inv_hi = inv_hi;
  L.agg = agg;
  L.ws = ws;
  return c->nlayouts++;
}

extern "C" int bsc_round_bind_task(void* ctx, void* gram_stream, const float* X, const int* y, const long long* off,
                                   const int* ntrain, const int* pid, int d_in, int d_out, int B, int P,
                                   unsigned long long seed, float max_norm, double qs, int lo, const uint32_t* tbl_wb,
                                   const int* rows_arange, const float* noise, int noise_n, int kchunk,
                                   unsigned int* counters) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || P <= 0 || d_in * d_out + d_out != c->d) return -1;
  TaskCfg& t = c->task;
  t.gram = (hipStream_t)gram_stream;
  t.X = X;
  t.y = y;
  t.off = off;
  t.ntrain = ntrain;
  t.pid = pid;
  t.d_in = d_in;
  t.d_out = d_out;
  t.B = B;
  t.P = P;
  t.seed = seed;
  t.max_norm = max_norm;
  t.qs = qs;
  t.lo = lo;
  t.tbl_wb = tbl_wb;
  t.rows_arange = rows_arange;
  t.noise = noise;
  t.noise_n = noise_n;
  t.nn_tab = nullptr;
  t.kchunk = kchunk;
  t.counters = counters;
  t.bound = 1;
  return 0;
}

// The [100][N][N] Gram of each iteration's noise rows (built at setup, ml.py NoiseRows.gram_table): the pre-step's
// noise-aware Gram copies its noise x noise tiles from it instead of computing them (nullptr: compute).
extern "C" int bsc_round_set_nn_table(void* ctx, const double* nn) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || !c->task.bound) return -1;
  c->task.nn_tab = nn;
  return 0;
}

extern "C" int bsc_round_add_pre_slot(void* ctx, float* delta, long long* qdelta, float* loss, uint32_t* ccom,
                                      uint32_t* jac, uint32_t* jac_host, double* part, double* gram, void* ev_step,
                                      void* ev_ccom, void* ev_commit, void* ev_gram) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || c->npre >= 8) return -1;
  PreSlot& p = c->pre[c->npre];
  p.delta = delta;
  p.qdelta = qdelta;
  p.loss = loss;
  p.ccom = ccom;
  p.jac = jac;
  p.jac_host = jac_host;
  p.part = part;
  p.gram = gram;
  p.ev_step = (hipEvent_t)ev_step;
  p.ev_ccom = (hipEvent_t)ev_ccom;
  p.ev_commit = (hipEvent_t)ev_commit;
  p.ev_gram = (hipEvent_t)ev_gram;
  return c->npre++;
}

// the model ring slot for the next recovered model: never W (its input) and never one of the last two
// results (one may still feed a queued pre-step), so a dropped aggregate can never overwrite the live model
// (host-only, testable without a GPU) ring[*k + 1 ...]: the next entry that is neither W nor recent[0..1];
// advances *k and shifts it into recent.  -1 when none is free (a ring of >= 4 always has one).
extern "C" int bsc_ring_pick(const void* const* ring, int n, int* k, const void* W, const void** recent) {
  for (int step = 1; step <= n; ++step) {
    const int j = (*k + step) % n;
    const void* cand = ring[j];
    if (cand != W && cand != recent[0] && cand != recent[1]) {
      *k = j;
      recent[0] = recent[1];
      recent[1] = cand;
      return j;
    }
  }
  return -1;
}

extern "C" int bsc_round_pick_W(void* ctx, const double* W) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || c->nW < 3) return -1;
  return bsc_ring_pick((const void* const*)c->W_ring, c->nW, &c->Wk, W, (const void**)c->recent);
}

// the next round's pre-step into the next ring slot (noise-aware Gram when do_gram and a noise table is
// bound; its rows for iteration `it` are the table's rows it % 100); returns the slot
extern "C" int bsc_round_prestep_slot(void* ctx, const double* W, int it, int do_gram) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || !c->task.bound || c->npre < 3) return -1;
  c->pre_k = (c->pre_k + 1) % c->npre;
  const PreSlot& p = c->pre[c->pre_k];
  const TaskCfg& t = c->task;
  const bool g = do_gram && t.noise != nullptr;
  const float* rows = g ? t.noise + (size_t)(it % 100) * c->d : nullptr;
  // the next speculative slot's flags are set inside the step (after the slot's last reader)
  int* ones = nullptr;
  hipEvent_t ones_wait = nullptr;
  if (c->nspec > 0) {
    const int ns = (c->spec_k + 1) % c->nspec;
    ones = c->spec_alive[ns];
    ones_wait = c->spec_used[ns] ? c->spec_done[ns] : nullptr;
    c->spec_filled[ns] = true;
  }
  RC_CHECK(prestep_impl(c, t.gram, t.X, t.y, t.off, t.ntrain, t.pid, W, t.d_in, t.d_out, t.B, t.P, t.seed, it,
                        t.max_norm, t.qs, t.lo, p.delta, p.qdelta, p.loss, t.tbl_wb, t.rows_arange, p.ccom, p.jac,
                        p.jac_host, g ? 1 : 0, rows, g ? t.noise_n : 0, 100ll * c->d, t.kchunk, p.part, p.gram,
                        t.counters, p.ev_step, p.ev_ccom, p.ev_commit, p.ev_gram, 1, c->bg, ones, c->spec_cap,
                        ones_wait, g && t.nn_tab ? t.nn_tab + (size_t)(it % 100) * t.noise_n * t.noise_n : nullptr));
  return c->pre_k;
}

// the selection's flags for the speculative rows, then (early_slot >= 0) the audit's commitment sums from
// that pre-step slot's chunk commitments into `cs_out`, then main waits for the MSM (spec_ev)
static int select_head(RoundCtx* c, const int* node, const int* amap, int* alive, int nspec, const int* spec_rows,
                       void* spec_ev, int early_slot, void* upload, uint32_t* cs_out) {
  // node == nullptr: the selection kernel has set the flags itself (k_krum_vote with amap / alive)
  if (nspec > 0 && node != nullptr) RC_CHECK(bsc_set_alive(node, amap, nspec, alive, c->main));
  if (early_slot >= 0) {
    if (early_slot >= c->npre || nspec <= 0) return -1;
    const PreSlot& p = c->pre[early_slot];
    RC_CHECK(bsc_round_csum_early(c, p.ccom, p.ev_ccom, spec_rows, nspec, alive, cs_out, upload));
  }
  if (spec_ev != nullptr) RC_CHECK(hipStreamWaitEvent(c->main, (hipEvent_t)spec_ev, 0));
  return 0;
}

// One rank.  out[0] = model ring slot of the recovered model, out[1] = pre-step slot (-1: none queued).
// pre_it >= 0 queues the next round's pre-step (iteration pre_it) behind the recovery; audit_now = 0 leaves
// the audit to a later bsc_round_audit (the caller queues its own pre-step first).
extern "C" int bsc_round_after_select(void* ctx, const int* node, const int* amap, int* alive, int nspec,
                                      const int* spec_rows, void* spec_ev, const uint32_t* pts, const long long* ys,
                                      int early_slot, void* upload, int layout, const double* W, int audit,
                                      int pre_it, int do_gram, int audit_now, int* out) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || layout < 0 || layout >= c->nlayouts || nspec <= 0 || c->nW < 3) return -1;
  const Layout& L = c->layouts[layout];
  RC_CHECK(select_head(c, node, amap, alive, nspec, spec_rows, spec_ev, audit == 2 ? early_slot : -1, upload, c->cs));
  const int wk = bsc_round_pick_W(ctx, W);
  if (wk < 0) return -2;
  double* W_new = c->W_ring[wk];
  RC_CHECK(bsc_round_secagg(ctx, pts, nspec, ys, alive, L.ccols, L.wcols, L.nwc, L.ycols, L.xs, L.npts, L.A, L.basis,
                            L.shift, L.inv_lo, L.inv_hi, W, W_new, c->coeffs, c->status, L.agg, c->cs, L.ws,
                            c->h_status, c->h_W, audit));
  int ps = -1;
  if (pre_it >= 0) {
    ps = bsc_round_prestep_slot(ctx, W_new, pre_it, do_gram);
    if (ps < 0) return -3;
  }
  if (audit != 0 && audit_now) RC_CHECK(bsc_round_audit(ctx, c->coeffs, c->cs, c->ok, c->h_ok));
  out[0] = wk;
  out[1] = ps;
  return 0;
}

// Several ranks, before the aggregation's all_gather: flags, early audit sums and this rank's partials into
// the send row (nspec = 0: no local rows).
static int select_partials_impl(void* ctx, const int* node, const int* amap, int* alive, int nspec,
                                 const int* spec_rows, void* spec_ev, const uint32_t* pts, const long long* ys,
                                 int early_slot, void* upload, int layout, unsigned char* send, long long clock, int audit,
                                 int wait_cs, int defer_wit = 0) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || layout < 0 || layout >= c->nlayouts) return -1;
  const Layout& L = c->layouts[layout];
  RC_CHECK(select_head(c, node, amap, alive, nspec, spec_rows, nspec > 0 ? spec_ev : nullptr,
                       audit == 2 && nspec > 0 ? early_slot : -1, upload, (uint32_t*)send));
  return partials_impl(ctx, nspec > 0 ? pts : nullptr, nspec, nspec > 0 ? ys : nullptr, nspec > 0 ? alive : nullptr,
                       L.ccols, L.wcols, nspec > 0 ? L.nwc : 0, L.ws, send, clock, nspec > 0 ? audit : (audit ? 1 : 0),
                       wait_cs, defer_wit);
}

extern "C" int bsc_round_select_partials(void* ctx, const int* node, const int* amap, int* alive, int nspec,
                                         const int* spec_rows, void* spec_ev, const uint32_t* pts, const long long* ys,
                                         int early_slot, void* upload, int layout, unsigned char* send, long long clock,
                                         int audit) {
  return select_partials_impl(ctx, node, amap, alive, nspec, spec_rows, spec_ev, pts, ys, early_slot, upload, layout,
                              send, clock, audit, 1);
}

// Several ranks, behind the all_gather into recv: totals + recovery + read-back (clocks included), the next
// pre-step (no Gram: the caller gathers the deltas and splits the Gram across ranks), the audit.
extern "C" int bsc_round_after_gather(void* ctx, const unsigned char* recv, int world, long long row_bytes, int layout,
                                      const double* W, long long* h_clock, int audit, int pre_it, int audit_now,
                                      int* out) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || layout < 0 || layout >= c->nlayouts) return -1;
  const Layout& L = c->layouts[layout];
  const int wk = bsc_round_pick_W(ctx, W);
  if (wk < 0) return -2;
  RC_CHECK(bsc_round_combine(ctx, recv, world, row_bytes, L.ycols, L.xs, L.npts, L.A, L.basis, L.shift, L.inv_lo,
                             L.inv_hi, W, c->W_ring[wk], c->coeffs, c->status, L.agg, c->cs, c->h_status, c->h_W,
                             h_clock, audit));
  int ps = -1;
  if (pre_it >= 0) {
    ps = bsc_round_prestep_slot(ctx, c->W_ring[wk], pre_it, 0);
    if (ps < 0) return -3;
  }
  if (audit != 0 && audit_now) RC_CHECK(bsc_round_audit(ctx, c->coeffs, c->cs, c->ok, c->h_ok));
  out[0] = wk;
  out[1] = ps;
  return 0;
}

// Host wait for an event: spin for SPIN_NS (the round's waits are tens to a few hundred us, and a sleeping
// thread wakes late), then poll with short sleeps -- a long wait (ranks sharing a GPU, a collective behind a
// slow rank) does not burn a core the way hipEventSynchronize's busy wait does (docs/PERF.md, multi-rank CPU).
static long long g_spin_ns = 200000;   // bsc_set_host_spin_ns: the engine spins longer with one rank per process

extern "C" void bsc_set_host_spin_ns(long long ns) { g_spin_ns = ns < 0 ? 0 : ns; }

static int host_wait(hipEvent_t ev, long long timeout_ns = 0) {
  const long long SPIN_NS = g_spin_ns;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return (int)e;
    const long long ns =
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_ns > 0 && ns > timeout_ns) return -99;
    if (ns > SPIN_NS) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// which: 0 = the recovery read-back, 1 = the last audit's read-back, 2 / 3 = audit slot 0 / 1's.  With the round's own communicator, a wait longer
// than the collective timeout means a rank is gone (the reference's crashed peer): the communicator is aborted
// -- its kernels return -- and -99 goes back to the engine, which fails the job for the elastic restart
// (parallel/comm.py), as torch's watchdog does for its own collectives
extern "C" int bsc_round_wait(void* ctx, int which) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr) return -1;
  if (which == 1) which = 2 + c->aud_k;
  const hipEvent_t ev = which == 0 ? c->ev_readback : which == 2 ? c->ev_audit : c->ev_audit1;
  const int r = host_wait(ev, c->comm != nullptr ? c->timeout_ns : 0);
  if (r == -99 && c->comm != nullptr && g_rccl.comm_abort != nullptr) {
    g_rccl.comm_abort(c->comm);
    c->comm = nullptr;
  }
  return r;
}

// ---------------------------------------------------------------------------------------------------------
// The round's collectives, native (several ranks, one per GPU).  Each rank's round owns ONE RCCL communicator
// (bsc_round_comm_init: the unique id travels over the job's process group once) and issues every collective
// of its round on ONE comm stream, inside the fused calls that produce and consume the data:
//   bsc_round_agg_multi     behind the committee's selection: this rank's partial sums -> all_gather of the
//                           packed rows -> totals + exact recovery + read-back + the next pre-step -> all_gather
//                           of the pre-step's deltas -> this rank's tile pairs of the next noise-aware Gram,
//                           written into its slot of the next verification row
//   bsc_round_vg_exchange   the verification row: pack -> all_gather in place -> unpack (ops/gather.py)
// The order is the round's issue order, the same on every rank; RCCL pairs the ranks' operations op by op.  A
// rank emulating rank 0 of a larger job (bench.py --emulate-world) fills the other ranks' slots with its own
// contribution by device copies instead.  The library is the one torch already loaded (bsc_rccl_load).
extern "C" int bsc_rccl_load(const char* path) {
  if (g_rccl.all_gather != nullptr) return 0;
  void* h = nullptr;
  if (path != nullptr && path[0] != 0) {
    h = dlopen(path, RTLD_NOW | RTLD_NOLOAD);   // the copy the process runs already
    if (h == nullptr) h = dlopen(path, RTLD_NOW);
  }
  if (h == nullptr) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
  if (h == nullptr) return -1;
  g_rccl.get_unique_id = (decltype(g_rccl.get_unique_id))dlsym(h, "ncclGetUniqueId");
  g_rccl.comm_init_rank = (decltype(g_rccl.comm_init_rank))dlsym(h, "ncclCommInitRank");
  g_rccl.all_gather = (decltype(g_rccl.all_gather))dlsym(h, "ncclAllGather");
  g_rccl.comm_destroy = (decltype(g_rccl.comm_destroy))dlsym(h, "ncclCommDestroy");
  g_rccl.comm_abort = (decltype(g_rccl.comm_abort))dlsym(h, "ncclCommAbort");
  if (!g_rccl.get_unique_id || !g_rccl.comm_init_rank || !g_rccl.all_gather || !g_rccl.comm_destroy ||
      !g_rccl.comm_abort) {
    g_rccl.all_gather = nullptr;
    return -2;
  }
  g_rccl.h = h;
  return 0;
}

extern "C" int bsc_rccl_unique_id(unsigned char* out) {
  if (g_rccl.get_unique_id == nullptr) return -1;
  ncclUniqueId id;
  if (g_rccl.get_unique_id(&id) != ncclSuccess) return -2;
  memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

// world ranks, this one `rank`; uid: the NCCL_UNIQUE_ID_BYTES rank 0 drew (every rank passes the same);
// comm_stream: where the collectives run (nullptr: main); emulate: rank 0 alone (no communicator)
extern "C" int bsc_round_comm_init(void* ctx, const unsigned char* uid, int world, int rank, void* comm_stream,
                                   int emulate, double timeout_s) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || world < 2 || rank < 0 || rank >= world || c->comm != nullptr || (emulate && rank != 0)) return -1;
  if (c->ev_c0 == nullptr) {
    RC_CHECK(hipEventCreateWithFlags(&c->ev_c0, hipEventDisableTiming));
    RC_CHECK(hipEventCreateWithFlags(&c->ev_c1, hipEventDisableTiming));
  }
  c->cworld = world;
  c->crank = rank;
  c->emulate = emulate ? 1 : 0;
  c->cstream = comm_stream != nullptr ? (hipStream_t)comm_stream : c->main;
  c->timeout_ns = timeout_s > 0 ? (long long)(timeout_s * 1e9) : 0;
  if (!emulate) {
    if (g_rccl.comm_init_rank == nullptr || uid == nullptr) return -2;
    ncclUniqueId id;
    memcpy(id.internal, uid, NCCL_UNIQUE_ID_BYTES);
    const ncclResult_t r = g_rccl.comm_init_rank(&c->comm, world, id, rank);
    if (r != ncclSuccess) {
      c->comm = nullptr;
      return -100 - (int)r;
    }
  }
  return 0;
}

// the emulated all_gather: every one of `world` rows of dst [world][n] (32-bit words) gets src [n] -- ONE launch,
// as a real all_gather is one RCCL call (in place, src = dst's row 0, row 0 is rewritten with its own words)
__global__ void __launch_bounds__(256) k_replicate_rows(const uint32_t* src, uint32_t* dst, long long n, int world) {
  const long long total = n * world;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x)
    dst[i] = src[i % n];
}

// all_gather of `bytes` per rank from `send` into recv [world][bytes] (in place when send is this rank's slot of
// recv): the comm stream waits for the producer stream, the consumer stream for the collective
static int round_all_gather(RoundCtx* c, const void* send, void* recv, size_t bytes, hipStream_t prod,
                            hipStream_t cons) {
  unsigned char* r = (unsigned char*)recv;
  if (c->emulate) {   // rank 0 alone: every slot holds rank 0's contribution (same shapes, no transport)
    if (bytes % 4 != 0) return -31;
    const long long n = (long long)(bytes / 4), total = n * c->cworld;
    const int blocks = (int)std::min<long long>((total + 255) / 256, 1024);
    hipLaunchKernelGGL(k_replicate_rows, dim3(blocks), dim3(256), 0, prod, (const uint32_t*)send, (uint32_t*)r, n,
                       c->cworld);
    RC_CHECK(hipGetLastError());
    if (cons != prod) {
      RC_CHECK(hipEventRecord(c->ev_c1, prod));
      RC_CHECK(hipStreamWaitEvent(cons, c->ev_c1, 0));
    }
    return 0;
  }
  if (c->comm == nullptr) return -30;
  RC_CHECK(hipEventRecord(c->ev_c0, prod));
  RC_CHECK(hipStreamWaitEvent(c->cstream, c->ev_c0, 0));
  const ncclResult_t e = g_rccl.all_gather(send, recv, bytes, ncclUint8, c->comm, c->cstream);
  if (e != ncclSuccess) return -100 - (int)e;
  RC_CHECK(hipEventRecord(c->ev_c1, c->cstream));
  RC_CHECK(hipStreamWaitEvent(cons, c->ev_c1, 0));
  return 0;
}

// the resident buffers of the fused multi-rank calls: the aggregation's packed rows (send, recv [world][row_bytes],
// pinned h_clock [world]); the next Gram's inputs -- pad [maxlocal][d] (zeroed: a rank with fewer peers sends its
// rows then zeros), X [world maxlocal][d], part [nsplit][p1 - p0][256], this rank's tile pairs [p0, p1) of the
// U1 + N row Gram -- and the verification rows (two, alternating by iteration, vg_row_bytes each per rank) whose
// leading chunk x 256 doubles are each rank's Gram slot.  vg0 == nullptr: no packed verification row (the engine
// then gathers the Gram's deltas itself)
extern "C" int bsc_round_bind_multi(void* ctx, unsigned char* send, unsigned char* recv, long long row_bytes,
                                    long long* h_clock, int maxlocal, float* pad, float* X, double* part, int U1, int p0,
                                    int p1, unsigned char* vg0, unsigned char* vg1, long long vg_row_bytes) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || c->cworld < 2 || row_bytes < bsc_round_row_bytes(c->nch, c->T) || maxlocal <= 0) return -1;
  auto& m = c->m;
  m.send = send;
  m.recv = recv;
  m.row_bytes = row_bytes;
  m.h_clock = h_clock;
  m.maxlocal = maxlocal;
  m.pad = pad;
  m.X = X;
  m.part = part;
  m.U1 = U1;
  m.p0 = p0;
  m.p1 = p1;
  m.vg_recv[0] = vg0;
  m.vg_recv[1] = vg1;
  m.vg_row_bytes = vg_row_bytes;
  m.bound = 1;
  return 0;
}

// the next round's noise-aware Gram on several ranks, on the Gram stream behind pre-step slot `slot`: the deltas'
// all_gather (the rank's rows padded to maxlocal), then this rank's tile pairs into its verification-row slot of
// iteration `it`; event ev_gram of the slot
static int round_multi_gram(RoundCtx* c, int slot, int it) {
  const TaskCfg& t = c->task;
  const PreSlot& p = c->pre[slot];
  auto& m = c->m;
  if (t.noise == nullptr || m.vg_recv[0] == nullptr || m.X == nullptr) return -40;
  hipStream_t gs = t.gram;
  const size_t rowb = (size_t)c->d * sizeof(float);
  const float* src = p.delta;
  if (t.P != m.maxlocal) {
    RC_CHECK(hipMemcpyAsync(m.pad, p.delta, (size_t)t.P * rowb, hipMemcpyDeviceToDevice, gs));
    src = m.pad;
  }
  RC_CHECK(round_all_gather(c, src, m.X, (size_t)m.maxlocal * rowb, gs, gs));
  double* out = (double*)(m.vg_recv[it % 2] + (size_t)c->crank * m.vg_row_bytes);
  const int k = it % 100;   // the noisers' pre-sampled vectors of this iteration (client_obj.py:97-98)
  RC_CHECK(bsc_gram_stacked_range(m.X, m.U1, t.noise + (size_t)k * c->d, t.noise_n, 100ll * c->d, c->d, t.kchunk, m.p0,
                                  m.p1, m.part, out - (size_t)m.p0 * 256, t.counters,
                                  t.nn_tab != nullptr ? t.nn_tab + (size_t)k * t.noise_n * t.noise_n : nullptr, gs));
  RC_CHECK(hipEventRecord(p.ev_gram, gs));
  return 0;
}

// Several ranks, behind the committee's selection, in one call: this rank's partials, the aggregation's
// all_gather, totals + recovery + read-back + the next pre-step + the audit (bsc_round_after_gather), and with
// gram the next Gram (round_multi_gram).  out as bsc_round_after_select.
extern "C" int bsc_round_agg_multi(void* ctx, const int* node, const int* amap, int* alive, int nspec,
                                   const int* spec_rows, void* spec_ev, const uint32_t* pts, const long long* ys,
                                   int early_slot, void* upload, int layout, long long clock, const double* W,
                                   int audit, int pre_it, int audit_now, int gram, int* out) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || !c->m.bound || c->cworld < 2 || layout < 0 || layout >= c->nlayouts || upload == nullptr) return -1;
  const Layout& L = c->layouts[layout];
  const int nch = c->nch, T = c->T, world = c->cworld;
  // two gathers out of the one send row [cs | ys | clock]: the share sums + clocks (the recovery's input) first, on
  // main; the chunk-commitment partials (the audit's input) behind the early audit sums, on the upload stream -- so
  // the recovery never waits for the commitment sums.  recv = [world][cs] then [world][ys | clock].
  const size_t cs_bytes = 96ull * nch, ys_bytes = 8ull * nch * T + 8;
  if ((long long)(cs_bytes + ys_bytes) > c->m.row_bytes) return -1;
  unsigned char* recv_cs = c->m.recv;
  unsigned char* recv_ys = c->m.recv + (size_t)world * cs_bytes;
  // issue order = the critical path first: partials -> share-sum gather -> recovery; then what only the audit, the
  // witness sums and the next round read (the host issues ~5 us per launch: the recovery no longer queues behind them)
  RC_CHECK(select_partials_impl(ctx, node, amap, alive, nspec, spec_rows, spec_ev, pts, ys, early_slot, upload, layout,
                                c->m.send, clock, audit, 0, 1));
  RC_CHECK(hipEventRecord(c->ev_main, c->main));   // the partials (or, no local rows, the zeroed commitment slot)
  RC_CHECK(round_all_gather(c, c->m.send + cs_bytes, recv_ys, ys_bytes, c->main, c->main));
  const int wk = bsc_round_pick_W(ctx, W);
  if (wk < 0) return -2;
  RC_CHECK(bsc_recover_w_clock((const long long*)recv_ys, world, (long long)(ys_bytes / 8), nch, T, nullptr, L.ycols, L.xs,
                               L.npts, L.A, L.basis, c->poly, L.shift, L.inv_lo, L.inv_hi, c->d, W, c->qscale,
                               c->W_ring[wk], c->coeffs, c->status, L.agg, c->h_W, c->h_status, c->m.h_clock, c->main));
  RC_CHECK(hipEventRecord(c->ev_readback, c->main));
  if (audit != 0) {
    hipStream_t up = (hipStream_t)upload;
    RC_CHECK(hipStreamWaitEvent(up, c->ev_main, 0));
    if (nspec > 0) RC_CHECK(hipStreamWaitEvent(up, c->ev_side, 0));   // the commitment partials
    RC_CHECK(round_all_gather(c, c->m.send, recv_cs, cs_bytes, up, up));
    RC_CHECK(bsc_sum_rows2((const uint32_t*)recv_cs, nch, nullptr, world, nullptr, nch, nullptr, c->cs, up));
    RC_CHECK(hipEventRecord(c->ev_side, up));   // bsc_round_audit waits for the totals through ev_side
  }
  if (nspec > 0 && L.nwc > 0) {   // the witness sums (per rank; no consumer in the round)
    RC_CHECK(hipStreamWaitEvent(c->wit, c->ev_main, 0));
    RC_CHECK(bsc_sum_cols_serial(pts, nch * (T + 1), nspec, L.wcols, L.nwc, alive, L.ws, c->wit));
    RC_CHECK(spec_mark_read(c, alive));
  }
  int ps = -1;
  if (pre_it >= 0) {
    ps = bsc_round_prestep_slot(ctx, c->W_ring[wk], pre_it, 0);
    if (ps < 0) return -3;
  }
  if (audit != 0 && audit_now) RC_CHECK(bsc_round_audit(ctx, c->coeffs, c->cs, c->ok, c->h_ok));
  out[0] = wk;
  out[1] = ps;
  if (ps >= 0 && gram) RC_CHECK(round_multi_gram(c, ps, pre_it));
  return 0;
}

extern "C" int bsc_vg_pack(uint8_t* row, long long commit_off, long long nz_off, long long sc_off,
                           const uint32_t* commits, int maxlocal, int pw, const int* src_row, const int* nz,
                           const float* sc, int nnz, void* stream);
extern "C" int bsc_vg_unpack(const uint8_t* recv, long long row_bytes, int chunk, int npairs, long long commit_off,
                             long long nz_off, long long sc_off, int maxlocal, int pw, int nn, int world,
                             const int* wrow, int nw, double* gram, int* nz, float* sc, uint32_t* commits_host,
                             void* stream);

// The verification row of iteration `it` (ops/gather.py): pack this rank's row, all_gather in place, unpack, on
// `stream`; the Gram slot at the row's head was written by round_multi_gram (or the caller's Gram launch)
extern "C" int bsc_round_vg_exchange(void* ctx, int it, long long commit_off, long long nz_off, long long sc_off,
                                     const uint32_t* commits, int maxlocal, int pw, const int* src_row, const int* nz,
                                     const float* sc, int nnz, int chunk, int npairs, int nn, const int* wrow, int nw,
                                     double* gram, int* nz_out, float* sc_out, uint32_t* host, void* stream) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || !c->m.bound || c->m.vg_recv[0] == nullptr) return -1;
  hipStream_t st = (hipStream_t)stream;
  unsigned char* buf = c->m.vg_recv[it % 2];
  const size_t rb = (size_t)c->m.vg_row_bytes;
  unsigned char* row = buf + (size_t)c->crank * rb;
  RC_CHECK(bsc_vg_pack(row, commit_off, nz_off, sc_off, commits, maxlocal, pw, src_row, nz, sc, nnz, st));
  RC_CHECK(round_all_gather(c, row, buf, rb, st, st));
  return bsc_vg_unpack(buf, (long long)rb, chunk, npairs, commit_off, nz_off, sc_off, maxlocal, pw, nn, c->cworld, wrow,
                       nw, gram, nz_out, sc_out, host, st);
}
