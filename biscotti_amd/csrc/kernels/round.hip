// Native round driver pieces: the secure aggregation a round queues behind the committee's selection,
// enqueued from C++ in ONE call instead of ~25 Python-level tensor / stream operations (each 5-20 us
// of the round's host thread, which is the round's critical path).
//
// bsc_round_secagg  -- the miners' sums and the leader's recovery (aggregateSecret + recoverSecret,
//                      DistSys/kyber.go:244-287,809-857) for the rows the selection kept:
//                        side: chunk-commitment sums of the kept rows (the audit's input)
//                        bg:   witness sums (no consumer on the protocol path)
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
#include <hip/hip_runtime.h>
#include <stdint.h>

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
                                     long long* agg_out, void* stream);
extern "C" int bsc_sum_rows_i64(const long long* ys, int R, long long C, const int* rows, int nsel, const int* mask,
                                long long* out, void* stream);
extern "C" int bsc_sum_rows2_pos(const uint32_t* pts, int ncols_in, const int* rows, int nrows, const int* cols,
                                 int ncols, const int* row_mask, uint32_t* out, void* stream);
extern "C" int bsc_shares_msm(const long long* coeffs, int d, const int* rows, int nrows, const uint32_t* tbl_pk,
                              const uint32_t* tbl_wb, int poly, int T, int B0, int NW, int commit_only,
                              const int* alive, const int* compact, int group_rows, uint32_t* out_pts,
                              long long* out_y, void* stream);
extern "C" int bsc_softmax_step(const float* X, const int* y, const long long* off, const int* ntrain,
                                const int* pid, const double* W, int D_IN, int D_OUT, int B, int P, unsigned long long seed,
                                int iteration, float max_norm, double qscale, float* delta, long long* qdelta,
                                float* loss, int lo, void* stream);
extern "C" int bsc_gram_stacked(const float* X, int U1, const float* X2, int U2, long long stride2, int D, int kchunk,
                                double* part, double* gram, unsigned int* count, void* stream);
extern "C" int bsc_segment_sum(const uint32_t* pts, int ngroups, int n, int stride, int off, uint32_t* out,
                               void* stream);
extern "C" int bsc_commit_rows(const long long* coeffs, int d, const int* rows, int nrows, const uint32_t* tbl_pk,
                               int B0, int NW, uint32_t* partial, uint32_t* out, void* stream);
extern "C" int bsc_chunk_check(const long long* coeffs, int d, int poly, const uint32_t* tbl_pk, int B0, int NW,
                               const uint32_t* csum, int nm, int nch, int* ok, void* stream);

namespace {
struct RoundCtx {
  hipStream_t main, side, bg;
  hipEvent_t ev_main, ev_side, ev_readback, ev_audit, ev_pre;
  const uint32_t* tbl_pk;
  int d, poly, T, nch, b0, nw;
  double qscale;
};
#define RC_CHECK(x)                        \
  do {                                     \
    const int e_ = (int)(x);               \
    if (e_ != 0) return e_;                \
  } while (0)
}  // namespace

extern "C" void* bsc_round_create(void* main, void* side, void* bg, const uint32_t* tbl_pk, int d, int poly, int T,
                                  int b0, int nw, double qscale) {
  RoundCtx* c = new RoundCtx();
  c->main = (hipStream_t)main;
  c->side = (hipStream_t)side;
  c->bg = (hipStream_t)bg;
  c->tbl_pk = tbl_pk;
  c->d = d;
  c->poly = poly;
  c->T = T;
  c->nch = (d + poly - 1) / poly;
  c->b0 = b0;
  c->nw = nw;
  c->qscale = qscale;
  hipEvent_t* evs[5] = {&c->ev_main, &c->ev_side, &c->ev_readback, &c->ev_audit, &c->ev_pre};
  for (hipEvent_t* e : evs)
    if (hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
      delete c;
      return nullptr;
    }
  return c;
}

extern "C" void bsc_round_destroy(void* ctx) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr) return;
  hipEventDestroy(c->ev_main);
  hipEventDestroy(c->ev_side);
  hipEventDestroy(c->ev_readback);
  hipEventDestroy(c->ev_audit);
  hipEventDestroy(c->ev_pre);
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
  RC_CHECK(hipStreamWaitEvent(c->bg, c->ev_main, 0));
  RC_CHECK(bsc_sum_rows2(pts, ncols_in, nullptr, R, wcols, nwc, mask, ws, c->bg));
  RC_CHECK(bsc_recover_w(ys, R, c->nch, c->T, mask, ycols, xs, npts, A, basis, c->poly, shift, inv_lo, inv_hi, c->d, W,
                         c->qscale, W_new, coeffs, status, agg, c->main));
  RC_CHECK(hipMemcpyAsync(h_status, status, (size_t)c->nch * sizeof(int), hipMemcpyDeviceToHost, c->main));
  RC_CHECK(hipMemcpyAsync(h_W, W_new, (size_t)c->d * sizeof(double), hipMemcpyDeviceToHost, c->main));
  RC_CHECK(hipEventRecord(c->ev_readback, c->main));
  return 0;
}

extern "C" int bsc_round_audit(void* ctx, const long long* coeffs, const uint32_t* cs, int* ok, int* h_ok) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr) return -1;
  RC_CHECK(hipStreamWaitEvent(c->main, c->ev_side, 0));
  RC_CHECK(bsc_chunk_check(coeffs, c->d, c->poly, c->tbl_pk, c->b0, c->nw, cs, 1, c->nch, ok, c->main));
  RC_CHECK(hipMemcpyAsync(h_ok, ok, (size_t)c->nch * sizeof(int), hipMemcpyDeviceToHost, c->main));
  RC_CHECK(hipEventRecord(c->ev_audit, c->main));
  return 0;
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

// The next round's speculative share MSM (head.py _spec_head_launch) in one call: the side stream waits for
// the pre-step (ev_wait: its quantised updates), uploads the row list and the all-ones alive flags from
// pinned staging (host [2n] int32: rows, then ones) into rows_dev [2n], and runs the MSM over them into
// resident pts / ys.  The caller rotates staging / device buffers over enough slots that a slot is
// rewritten only after its MSM and every consumer of its outputs are done.
// The upload goes through `up` (a high-priority stream on every CU, event ev_up): on the CU-masked, low-
// priority side stream the copy kernel waited ~150 us for a free slot behind the pre-step's MSM.
extern "C" int bsc_round_spec_msm(void* ctx, void* ev_wait, const long long* coeffs, const int* rows_host,
                                  int* rows_dev, int n, const uint32_t* tbl_wb, int commit_only, int group_rows,
                                  uint32_t* pts, long long* ys, void* up, void* ev_up) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || n <= 0) return -1;
  if (ev_wait != nullptr) RC_CHECK(hipStreamWaitEvent(c->side, (hipEvent_t)ev_wait, 0));
  if (up != nullptr && ev_up != nullptr) {
    RC_CHECK(hipMemcpyAsync(rows_dev, rows_host, 2 * (size_t)n * sizeof(int), hipMemcpyHostToDevice, (hipStream_t)up));
    RC_CHECK(hipEventRecord((hipEvent_t)ev_up, (hipStream_t)up));
    RC_CHECK(hipStreamWaitEvent(c->side, (hipEvent_t)ev_up, 0));
  } else {
    RC_CHECK(hipMemcpyAsync(rows_dev, rows_host, 2 * (size_t)n * sizeof(int), hipMemcpyHostToDevice, c->side));
  }
  RC_CHECK(bsc_shares_msm(coeffs, c->d, rows_dev, n, c->tbl_pk, tbl_wb, c->poly, c->T, c->b0, c->nw, commit_only,
                          rows_dev + n, nullptr, group_rows, pts, ys, c->side));
  return 0;
}

// The next round's pre-step (head.py _queue_pre_step) in one call, queued behind everything on main so far
// (the recovery of W):
//   gram stream: local SGD step of every local peer (delta, qdelta, loss), event ev_step; then, when
//                do_gram, the noise-aware Krum's phase-1 Gram of [delta; this iteration's noise rows],
//                event ev_gram
//   background:  behind the step, the per-chunk commitments of every row (ccom, event ev_ccom), their
//                per-row sums = the full commitments (jac), read back into pinned jac_host, event ev_commit
// Outputs are resident (the caller rotates them over slots); events are caller-owned and re-recorded.
extern "C" int bsc_round_prestep(void* ctx, void* gram_stream, const float* X, const int* y, const long long* off,
                                 const int* ntrain, const int* pid, const double* W, int d_in, int d_out, int B, int P,
                                 unsigned long long seed, int iteration, float max_norm, double qscale, int lo,
                                 float* delta, long long* qdelta, float* loss, const uint32_t* tbl_wb,
                                 const int* rows_arange, uint32_t* ccom, uint32_t* jac, uint32_t* jac_host,
                                 int do_gram, const float* T_rows, int U2, long long stride2, int kchunk, double* part,
                                 double* gram, unsigned int* counters, void* ev_step, void* ev_ccom, void* ev_commit,
                                 void* ev_gram, int chunked, void* commit_stream) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr || P <= 0 || d_in * d_out + d_out != c->d) return -1;
  hipStream_t gs = (hipStream_t)gram_stream;
  // the commitments' stream (default: background; an A/B passes one masked to the CUs the MSM leaves)
  hipStream_t cst = commit_stream != nullptr ? (hipStream_t)commit_stream : c->bg;
  RC_CHECK(hipEventRecord(c->ev_pre, c->main));
  RC_CHECK(hipStreamWaitEvent(gs, c->ev_pre, 0));
  RC_CHECK(bsc_softmax_step(X, y, off, ntrain, pid, W, d_in, d_out, B, P, seed, iteration, max_norm, qscale, delta,
                            qdelta, loss, lo, gs));
  RC_CHECK(hipEventRecord((hipEvent_t)ev_step, gs));
  RC_CHECK(hipStreamWaitEvent(cst, (hipEvent_t)ev_step, 0));
  if (chunked) {
    RC_CHECK(bsc_shares_msm(qdelta, c->d, rows_arange, P, c->tbl_pk, tbl_wb, c->poly, c->T, c->b0, c->nw, 1, nullptr,
                            nullptr, 0, ccom, nullptr, cst));
    RC_CHECK(hipEventRecord((hipEvent_t)ev_ccom, cst));
    RC_CHECK(bsc_segment_sum(ccom, P, c->nch, 1, 0, jac, cst));
  } else {   // full commitments only (1024-coefficient slabs; ccom is the slab-partials scratch)
    RC_CHECK(bsc_commit_rows(qdelta, c->d, rows_arange, P, c->tbl_pk, c->b0, c->nw, ccom, jac, cst));
  }
  RC_CHECK(hipMemcpyAsync(jac_host, jac, (size_t)P * 24 * sizeof(uint32_t), hipMemcpyDeviceToHost, cst));
  RC_CHECK(hipEventRecord((hipEvent_t)ev_commit, cst));
  if (do_gram) {
    RC_CHECK(bsc_gram_stacked(delta, P, T_rows, U2, stride2, c->d, kchunk, part, gram, counters, gs));
    RC_CHECK(hipEventRecord((hipEvent_t)ev_gram, gs));
  }
  return 0;
}

// ---------------------------------------------------------------------------------------------------------
// Several ranks (one per GPU).  The aggregation's ONE all_gather moves a packed row per rank,
//     [ cs: nch x 24 u32 | ys: nch x T int64 | clock: int64 | pad ]      (row_bytes: a multiple of 96)
// so the gathered buffer is at once a [world][row_bytes / 96][24] point array whose first nch columns are the
// ranks' chunk-commitment partial sums (bsc_sum_rows2 sums them) and a strided [world][nch][T] share-sum
// array (k_recover_w with a row stride sums and recovers).  No repacking on either side of the collective.
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

extern "C" int bsc_round_partials(void* ctx, const uint32_t* pts, int R, const long long* ys, const int* mask,
                                  const int* ccols, const int* wcols, int nwc, uint32_t* ws, unsigned char* send,
                                  long long clock, int audit) {
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
    if (nwc > 0 && ws != nullptr) {
      RC_CHECK(hipStreamWaitEvent(c->bg, c->ev_main, 0));
      RC_CHECK(bsc_sum_rows2(pts, ncols_in, nullptr, R, wcols, nwc, mask, ws, c->bg));
    }
    RC_CHECK(bsc_sum_rows_i64(ys, R, (long long)nch * T, nullptr, R, mask, ys_slot, c->main));
  } else {
    RC_CHECK(hipMemsetAsync(ys_slot, 0, 8ull * nch * T, c->main));
    if (audit != 0) RC_CHECK(hipMemsetAsync(cs_slot, 0, 96ull * nch, c->main));
  }
  const unsigned long long u = (unsigned long long)clock;
  RC_CHECK(hipMemsetD32Async((hipDeviceptr_t)clk, (int)(u & 0xffffffffull), 1, c->main));
  RC_CHECK(hipMemsetD32Async((hipDeviceptr_t)(clk + 4), (int)(u >> 32), 1, c->main));
  if (R > 0 && audit != 0) RC_CHECK(hipStreamWaitEvent(c->main, c->ev_side, 0));
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
  RC_CHECK(bsc_recover_w_strided((const long long*)(recv + 96ll * nch), world, row_bytes / 8, nch, T, nullptr, ycols,
                                 xs, npts, A, basis, c->poly, shift, inv_lo, inv_hi, c->d, W, c->qscale, W_new, coeffs,
                                 status, agg, c->main));
  RC_CHECK(hipMemcpyAsync(h_status, status, (size_t)nch * sizeof(int), hipMemcpyDeviceToHost, c->main));
  RC_CHECK(hipMemcpyAsync(h_W, W_new, (size_t)c->d * sizeof(double), hipMemcpyDeviceToHost, c->main));
  RC_CHECK(hipMemcpy2DAsync(h_clock, sizeof(long long), recv + 96ll * nch + 8ll * nch * T, (size_t)row_bytes,
                            sizeof(long long), (size_t)world, hipMemcpyDeviceToHost, c->main));
  RC_CHECK(hipEventRecord(c->ev_readback, c->main));
  return 0;
}

// Host wait for an event: spin for SPIN_NS (the round's waits are tens to a few hundred us, and a sleeping
// thread wakes late), then poll with short sleeps -- a long wait (ranks sharing a GPU, a collective behind a
// slow rank) does not burn a core the way hipEventSynchronize's busy wait does (docs/PERF.md, multi-rank CPU).
static int host_wait(hipEvent_t ev) {
  constexpr long long SPIN_NS = 200000;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return (int)e;
    const long long ns =
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    if (ns > SPIN_NS) std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

// which: 0 = the recovery read-back, 1 = the audit read-back
extern "C" int bsc_round_wait(void* ctx, int which) {
  RoundCtx* c = (RoundCtx*)ctx;
  if (c == nullptr) return -1;
  return host_wait(which == 0 ? c->ev_readback : c->ev_audit);
}
