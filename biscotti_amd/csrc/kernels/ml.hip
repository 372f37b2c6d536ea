// Learning-side kernels of a Biscotti round (gfx950):
//   K1  batched softmax-regression local step: minibatch draw, (x-0.5)/0.5 transform, logits
//       (f32 MFMA), softmax + CE, backward dW (f32 MFMA) / db, clip_grad_norm(100), negate,
//       fixed-point quantisation -- one workgroup per virtual peer
//       (ML/Pytorch/client.py:38-65, client_obj.py:73-77, DistSys/kyber.go:698-710)
//   K3  batched logistic-regression step with DP noise at source (ML/code/logistic_model.py:92-140)
//   K4  counter-based Gaussian DP noise, averaged over each worker's noisers, added to the delta
//       (client_obj.py:42-67,97-98; DistSys/main.go:1592-1660,1530-1537)
//   K5  Multi-Krum: f64-MFMA Gram (split-K) + distances/scores/selection in LDS
//       (client_obj.py:114-143)
//   K2  test error / 1->7 attack rate (client.py:146-172)
//   K12 exact secret recovery (128-bit Newton) + dequantisation + W update (kyber.go:809-857,
//       honest.go:398-411,442-502)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define BSC_PRIO_FLAG bsc_prio_on_ml
#include "wave_prio.h"
BSC_PRIO_SETTER(bsc_wave_prio_ml)

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- Philox4x32-10
struct u4 {
  uint32_t x, y, z, w;
};
__device__ __forceinline__ u4 philox(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    u4 n;
    n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
    n.y = (uint32_t)p1;
    n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
    n.w = (uint32_t)p0;
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
__device__ __forceinline__ float u01(uint32_t v) { return ((float)(v >> 8) + 0.5f) * (1.0f / 16777216.0f); }
__device__ __forceinline__ float gauss(uint32_t a, uint32_t b) {
  const float r = sqrtf(-2.0f * logf(u01(a)));
  return r * cosf(6.28318530717958647692f * u01(b));
}

__device__ __forceinline__ long long quantize(float v, double scale) {
  // Go: int64(float64(delta) * 10^precision) -- truncation toward zero
  return (long long)((double)v * scale);
}

}  // namespace

// =====================================================================================
// K1: softmax regression local step.  Any D_IN (K-tiled through LDS), D_OUT <= 16, B <= 16.
// X: [Ntot, D_IN] fp32 (standardised pixels), y: [Ntot] int32.  Peer p trains on rows
// [off[p], off[p] + ntrain[p]).  W: [D_OUT*D_IN + D_OUT] fp64 global model (W row-major, b).
// Outputs: delta fp32 [P, nparam], qdelta int64 [P, nparam], loss fp32 [P].
// =====================================================================================
constexpr int SM_MAXK = 1024;
constexpr int SM_THREADS = 256;

extern "C" __global__ void __launch_bounds__(SM_THREADS) k_softmax_step(
    const float* X, const int* y, const long long* off, const int* ntrain, const int* pid, const double* W, int D_IN,
    int D_OUT, int B, int P, unsigned long long seed, int iteration, float max_norm, double qscale, float* delta,
    long long* qdelta, float* loss, int lo, int* ones, int nones) {
  // the next round's speculative share MSM waits for this step (and the Gram behind it on the same stream):
  // a short latency chain at the front of the round
  BSC_SET_PRIO(BSC_PRIO_CRITICAL);
  // ones (optional): the next speculative MSM's row flags, set to 1 here (the MSM waits for this step anyway)
  // instead of by an upload or a kernel of their own in front of the MSM
  if (ones != nullptr && blockIdx.x == 0)
    for (int i = threadIdx.x; i < nones; i += blockDim.x) ones[i] = 1;
  __shared__ float xs[16 * SM_MAXK];  // minibatch rows, transformed; rows >= B are zero
  __shared__ float red[4][16][16];    // per-wave partial logits
  __shared__ float G[16][16];         // (softmax - onehot) / B
  __shared__ int bidx[16];
  __shared__ float nrm[SM_THREADS / 64];
  __shared__ float scale_sh;
  const int p = blockIdx.x;
  if (p >= P) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nparam = D_OUT * D_IN + D_OUT;
  // lo >= 0: off / ntrain are indexed by local peer (pid - lo), resident for every local peer, so a
  // round uploads only the peer ids; lo < 0: per-row arrays
  const int li = lo >= 0 ? pid[p] - lo : p;
  const long long offp = off[li];
  const int n = ntrain[li];
  // 1. draw B distinct minibatch indices (DataLoader(shuffle=True) takes the first batch)
  if (tid == 0) {
    int cnt = 0;
    uint32_t ctr = 0;
    while (cnt < B && cnt < n) {
      u4 r = philox(u4{(uint32_t)pid[p], (uint32_t)iteration, ctr++, 0x5EEDu}, (uint32_t)seed, (uint32_t)(seed >> 32));
      const uint32_t cand[4] = {r.x, r.y, r.z, r.w};
      for (int q = 0; q < 4 && cnt < B && cnt < n; ++q) {
        const int c = (int)(cand[q] % (uint32_t)n);
        bool dup = false;
        for (int t = 0; t < cnt; ++t) dup |= bidx[t] == c;
        if (!dup) bidx[cnt++] = c;
      }
    }
    for (int t = cnt; t < 16; ++t) bidx[t] = -1;
  }
  __syncthreads();
  const int Bq = min(B, n);
  // 2-3. logits via f32 MFMA 16x16x4: A[s][k] = xs, B[k][c] = W[c][k].  The minibatch rows are staged
  // through LDS in K tiles of SM_MAXK (one tile for MNIST's 784 features, nine for LFW's 8742);
  // within a tile the 4 waves split K, each accumulating its share across tiles in registers.
  const int ktiles = (D_IN + SM_MAXK - 1) / SM_MAXK;
  auto stage = [&](int kt) {  // (x - 0.5) / 0.5 (torchvision Normalize(0.5, 0.5)); zero padding
    const int k0 = kt * SM_MAXK, kw = min(SM_MAXK, D_IN - k0);
    for (int i = tid; i < 16 * kw; i += SM_THREADS) {
      const int s = i / kw, k = i % kw;
      float v = 0.f;
      if (s < Bq) v = (X[(offp + bidx[s]) * (long long)D_IN + k0 + k] - 0.5f) * 2.0f;
      xs[s * SM_MAXK + k] = v;
    }
  };
  {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int i = lane & 15, kk = lane >> 4;
    for (int kt = 0; kt < ktiles; ++kt) {
      const int k0 = kt * SM_MAXK, kw = min(SM_MAXK, D_IN - k0);
      if (kt > 0) __syncthreads();  // the previous tile has been consumed
      stage(kt);
      __syncthreads();
      const int ksteps = (kw + 3) / 4;
      const int per = (ksteps + 3) / 4;
      for (int st = wid * per; st < min(ksteps, (wid + 1) * per); ++st) {
        const int k = st * 4 + kk;
        const float av = (k < kw) ? xs[i * SM_MAXK + k] : 0.f;
        const float bv = (k < kw && i < D_OUT) ? (float)W[i * D_IN + k0 + k] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wid][(lane >> 4) * 4 + r][lane & 15] = acc[r];
  }
  __syncthreads();
  // 4. softmax + cross-entropy on rows s < Bq (one thread per row)
  if (tid < 16) {
    const int s = tid;
    if (s < Bq) {
      float lg[16];
      float mx = -INFINITY;
      for (int c = 0; c < D_OUT; ++c) {
        lg[c] = red[0][s][c] + red[1][s][c] + red[2][s][c] + red[3][s][c] + (float)W[D_OUT * D_IN + c];
        mx = fmaxf(mx, lg[c]);
      }
      float se = 0.f;
      for (int c = 0; c < D_OUT; ++c) se += expf(lg[c] - mx);
      const int lab = y[offp + bidx[s]];
      for (int c = 0; c < D_OUT; ++c) G[s][c] = (expf(lg[c] - mx) / se - (c == lab ? 1.f : 0.f)) / (float)Bq;
      for (int c = D_OUT; c < 16; ++c) G[s][c] = 0.f;
      red[0][s][0] = (mx + logf(se)) - lg[lab];  // per-row CE (red no longer needed)
    } else {
      for (int c = 0; c < 16; ++c) G[s][c] = 0.f;
    }
  }
  __syncthreads();
  if (tid == 0) {
    float l = 0.f;
    for (int s = 0; s < Bq; ++s) l += red[0][s][0];
    loss[p] = l / (float)max(Bq, 1);
  }
  // 5. dW[c][k] = sum_s G[s][c] xs[s][k] via f32 MFMA (M = classes, N = k tiles, K = samples); with
  // several K tiles the rows are staged again (the last tile is still resident: it goes first)
  float* dst = delta + (size_t)p * nparam;
  float sq = 0.f;
  for (int q = 0; q < ktiles; ++q) {
    const int kt = (ktiles - 1 + q) % ktiles;
    const int k0 = kt * SM_MAXK, kw = min(SM_MAXK, D_IN - k0);
    if (q > 0) {
      __syncthreads();
      stage(kt);
      __syncthreads();
    }
    const int ntiles = (kw + 15) / 16;
    const int col = lane & 15, kk = lane >> 4;
    for (int t = wid; t < ntiles; t += 4) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int s = ks * 4 + kk;
        const float av = G[s][col];  // A[c = col][s]
        const int k = t * 16 + col;
        const float bv = (k < kw) ? xs[s * SM_MAXK + k] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
      }
      const int k = t * 16 + col;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = (lane >> 4) * 4 + r;
        if (c < D_OUT && k < kw) {
          dst[c * D_IN + k0 + k] = acc[r];
          sq += acc[r] * acc[r];
        }
      }
    }
  }
  if (tid < D_OUT) {
    float db = 0.f;
    for (int s = 0; s < 16; ++s) db += G[s][tid];
    dst[D_OUT * D_IN + tid] = db;
    sq += db * db;
  }
  // 6. clip_grad_norm(max_norm): total L2 norm over W and b
  for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
  if (lane == 0) nrm[wid] = sq;
  __syncthreads();
  if (tid == 0) {
    const float tot = sqrtf(nrm[0] + nrm[1] + nrm[2] + nrm[3]);
    const float coef = max_norm / (tot + 1e-6f);
    scale_sh = coef < 1.f ? coef : 1.f;
  }
  __syncthreads();
  // 7. delta = -grad (client_obj.privateFun), quantised like updateFloatToInt
  const float sc = -scale_sh;
  long long* qd = qdelta + (size_t)p * nparam;
  for (int i = tid; i < nparam; i += SM_THREADS) {
    const float v = dst[i] * sc;
    dst[i] = v;
    qd[i] = quantize(v, qscale);
  }
}

// =====================================================================================
// K3: logistic regression step (creditcard path).  One wave per peer.
// X: [Ntot, D] fp64 with bias column, y: [Ntot] (+1/-1); peer p samples B rows of
// [off[p], off[p]+n[p]).  delta = -alpha * g + noise_at_source;  g = X^T(-y/(1+e^{yXw}))/B + lam*w
// noise = (-alpha/B) * sigma*sqrt(B) * N(0,1)  (getNoise: samples are sums over the batch axis)
// =====================================================================================
extern "C" __global__ void __launch_bounds__(64) k_logreg_step(
    const double* X, const double* y, const long long* off, const int* nrows, const int* pid, const double* W, int D,
    int B, int P, unsigned long long seed, const int* calls, double alpha, double lammy, const double* sigma, double qscale,
    float* delta, long long* qdelta) {
  const int p = blockIdx.x;
  if (p >= P) return;
  const int lane = threadIdx.x;
  __shared__ int bidx[64];
  __shared__ double res[64];
  const int n = nrows[p];
  if (lane == 0) {
    int cnt = 0;
    uint32_t ctr = 0;
    while (cnt < B && cnt < n) {
      u4 r = philox(u4{(uint32_t)pid[p], (uint32_t)calls[p], ctr++, 0x106u}, (uint32_t)seed, (uint32_t)(seed >> 32));
      const uint32_t cand[4] = {r.x, r.y, r.z, r.w};
      for (int q = 0; q < 4 && cnt < B && cnt < n; ++q) {
        const int c = (int)(cand[q] % (uint32_t)n);
        bool dup = false;
        for (int t = 0; t < cnt; ++t) dup |= bidx[t] == c;
        if (!dup) bidx[cnt++] = c;
      }
    }
  }
  __syncthreads();
  const int Bq = min(B, n);
  if (lane < Bq) {
    const double* xr = X + (off[p] + bidx[lane]) * (long long)D;
    double z = 0.0;
    for (int k = 0; k < D; ++k) z += xr[k] * W[k];
    const double yy = y[off[p] + bidx[lane]];
    // -y / exp(logaddexp(0, y*z)) == -y / (1 + exp(y*z))
    const double t = yy * z;
    const double lae = t > 0 ? t + log1p(exp(-t)) : log1p(exp(t));
    res[lane] = -yy / exp(lae);
  }
  __syncthreads();
  for (int k = lane; k < D; k += 64) {
    double g = 0.0;
    for (int s = 0; s < Bq; ++s) g += X[(off[p] + bidx[s]) * (long long)D + k] * res[s];
    g = g / (double)B + lammy * W[k];
    double v = -alpha * g;
    if (sigma[p] > 0.0) {
      u4 r = philox(u4{(uint32_t)k, (uint32_t)(calls[p] % 100), (uint32_t)pid[p], 0xD9u}, (uint32_t)(seed >> 7),
                    (uint32_t)(seed >> 39));
      v += (-alpha / (double)B) * sigma[p] * sqrt((double)B) * (double)gauss(r.x, r.y);
    }
    delta[(size_t)p * D + k] = (float)v;
    qdelta[(size_t)p * D + k] = (long long)(v * qscale);
  }
}

// =====================================================================================
// K4: DP noise.  noised[p][i] = delta[p][i] + (1/nn) sum_j scale[j] * N(0,1; key=(seed,noiser_j),
// ctr=(i, it%100)).  A noiser's vector depends only on (noiser, iteration % 100), like the
// reference's pre-sampled samples[it % 100] (client_obj.py:61-63,97-98).
// scale[j] = -sigma_j / sqrt(B)  (sigma_j = 0 for colluding noisers that pre-sampled with eps = 0)
// =====================================================================================
extern "C" __global__ void k_dp_noise(const float* delta, int P, int D, const int* noisers, int nn,
                                      const float* noiser_scale, unsigned long long seed, int iter_mod,
                                      float* noised) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (long long)P * D) return;
  const int p = (int)(g / D), i = (int)(g % D);
  float acc = 0.f;
  for (int j = 0; j < nn; ++j) {
    const int nid = noisers[p * nn + j];
    u4 r = philox(u4{(uint32_t)i, (uint32_t)iter_mod, (uint32_t)nid, 0xA11CEu}, (uint32_t)seed, (uint32_t)(seed >> 32));
    acc += noiser_scale[p * nn + j] * gauss(r.x, r.y);
  }
  noised[g] = delta[g] + (nn > 0 ? acc / (float)nn : 0.f);
}

// K4, resident form.  The reference pre-samples each peer's 100 noise vectors at init
// (samples[it % 100], client_obj.py:61-63); here the whole federation's table [N][100][D]
// (314 MB for MNIST, 100 peers) is built once in HBM with the same Philox counters, and the
// per-round kernel becomes a gather + average (memory-bound) instead of ~2 Philox + Box-Muller
// evaluations per element on the critical path.  Values and float operations are those of
// k_dp_noise, so both forms give identical bits.
extern "C" __global__ void k_noise_table(int nnoisers, int D, unsigned long long seed, float* tbl) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (long long)nnoisers * 100 * D) return;
  const int i = (int)(g % D);
  const long long nm = g / D;
  const int m = (int)(nm % 100), nid = (int)(nm / 100);
  u4 r = philox(u4{(uint32_t)i, (uint32_t)m, (uint32_t)nid, 0xA11CEu}, (uint32_t)seed, (uint32_t)(seed >> 32));
  tbl[g] = gauss(r.x, r.y);
}

// rows (optional): output row p is worker rows[p] -- the verifiers' inbox gathered in arrival order
// straight out of the noise kernel (no separate index_select pass over [n, D])
extern "C" __global__ void k_dp_noise_tbl(const float* delta, int P, int D, const int* noisers, int nn,
                                          const float* noiser_scale, const float* tbl, int iter_mod,
                                          const int* rows, float* noised) {
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (long long)P * D) return;
  const int p = (int)(g / D), i = (int)(g % D);
  const int src = rows ? rows[p] : p;
  float acc = 0.f;
  for (int j = 0; j < nn; ++j) {
    const int nid = noisers[src * nn + j];
    acc += noiser_scale[src * nn + j] * tbl[((size_t)nid * 100 + iter_mod) * D + i];
  }
  noised[g] = delta[(size_t)src * D + i] + (nn > 0 ? acc / (float)nn : 0.f);
}

// =====================================================================================
// K5a: Gram partials G_part[split][i][j] = sum_{k in split} X[i][k] X[j][k] in f64 via
// v_mfma_f64_16x16x4f64.  Grid (tiles_i, tiles_j, splits), one wave per block.
// f64 16x16x4 layout: A[i=l&15][k=l>>4], B[k=l>>4][j=l&15]; D: col=l&15, row=(l>>4)+4*r.
// =====================================================================================
extern "C" __global__ void __launch_bounds__(64) k_gram_f64(const float* X, int n, int D, int ksplit,
                                                           double* part) {
  const int ti = blockIdx.x, tj = blockIdx.y, sp = blockIdx.z;
  const int lane = threadIdx.x;
  const int i = ti * 16 + (lane & 15), j = tj * 16 + (lane & 15), kk = lane >> 4;
  const int k0 = sp * ksplit, k1 = min(D, k0 + ksplit);
  const float* xa = X + (size_t)min(i, n - 1) * D;
  const float* xb = X + (size_t)min(j, n - 1) * D;
  const bool va = i < n, vb = j < n;
  // loads issued 8 k-steps ahead of the MFMAs, two accumulators (one wave per block, so the
  // memory latency is otherwise fully exposed at every step)
  f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
  int k = k0;
  for (; k + 32 <= k1; k += 32) {
    float a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a[u] = xa[k + 4 * u + kk];
      b[u] = xb[k + 4 * u + kk];
    }
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(va ? (double)a[u] : 0.0, vb ? (double)b[u] : 0.0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(va ? (double)a[u + 1] : 0.0, vb ? (double)b[u + 1] : 0.0, acc1,
                                                  0, 0, 0);
    }
  }
  for (; k < k1; k += 4) {
    const int kx = k + kk;
    const double a = (va && kx < k1) ? (double)xa[kx] : 0.0;
    const double b = (vb && kx < k1) ? (double)xb[kx] : 0.0;
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
  }
  const f64x4 acc = acc0 + acc1;
  const int npad = gridDim.x * 16;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = ti * 16 + (lane >> 4) + 4 * r, col = tj * 16 + (lane & 15);
    part[((size_t)sp * npad + row) * npad + col] = acc[r];
  }
}

// K5b: Krum scores, one wave per row i (n blocks): reduce the split-K Gram partials of row i and of
// the diagonal, D_ij = G_ii + G_jj - 2 G_ij, then score_i = sum of D_ij whose rank in row i lies in
// [1, groupsize-2] -- the sum of the groupsize-2 nearest neighbours after the zero self-distance
// (sort(D_i)[1:groupsize-1], client_obj.py:114-143).  Ranks by parallel counting, ties broken by
// column index; the kept distances are summed in column order (bit-reproducible).  n <= 128.
extern "C" __global__ void __launch_bounds__(64) k_krum_scores(const double* part, int nsplit, int n, int npad,
                                                              int groupsize, double* dist, double* scores) {
  __shared__ double row[128];
  __shared__ double kept[128];
  const int i = blockIdx.x, lane = threadIdx.x;
  double gii = 0.0;
#pragma unroll 8
  for (int s = 0; s < nsplit; ++s) gii += part[((size_t)s * npad + i) * npad + i];
  for (int j = lane; j < n; j += 64) {
    double gij = 0.0, gjj = 0.0;
#pragma unroll 8
    for (int s = 0; s < nsplit; ++s) {
      gij += part[((size_t)s * npad + i) * npad + j];
      gjj += part[((size_t)s * npad + j) * npad + j];
    }
    const double d = gii + gjj - 2.0 * gij;
    row[j] = d;
    dist[(size_t)i * n + j] = d;
  }
  __syncthreads();
  for (int j = lane; j < n; j += 64) {
    const double v = row[j];
    int rank = 0;
    for (int k = 0; k < n; ++k) {
      const double u = row[k];
      rank += (u < v) || (u == v && k < j);
    }
    kept[j] = (rank >= 1 && rank < groupsize - 1) ? v : 0.0;
  }
  __syncthreads();
  if (lane == 0) {
    double a = 0.0;
    for (int j = 0; j < n; ++j) a += kept[j];
    scores[i] = a;
  }
}

// K5c: Multi-Krum selection: accept the n_accept lowest scores (index tiebreak).  One block.
extern "C" __global__ void __launch_bounds__(128) k_krum_accept(const double* scores, int n, int n_accept,
                                                               int* accept) {
  __shared__ double sc[128];
  const int t = threadIdx.x;
  if (t < n) sc[t] = scores[t];
  __syncthreads();
  if (t < n) {
    int rank = 0;
    for (int j = 0; j < n; ++j) rank += (sc[j] < sc[t]) || (sc[j] == sc[t] && j < t);
    accept[t] = rank < n_accept ? 1 : 0;
  }
}

// =====================================================================================
// K5 committee form: every verifier runs Multi-Krum on ITS OWN inbox (krum.go:284-322 runs in each
// verifier process over the first KRUM_UPDATETHRESH updates that process received), and an update
// is approved with >= floor(nv/2) signatures (main.go:1686); the leader then builds its block from
// the first NUM_SAMPLES/2 approved arrivals (main.go:360).  All inboxes are subsets of one row set
// X [U, D] (the submitted workers' noised deltas), so the Gram matrix is computed ONCE over X and
// each verifier's distances are gathered out of it:
//   KC1 k_gram_pairs     upper-triangular 16x16 tile pairs x K splits, f64 MFMA, 4 waves per block
//                        split K further and reduce through LDS -> part[split][pair][16][16]
//   KC2 k_krum_rows      one block per (inbox row, verifier): D_ij from the (deterministically
//                        reduced) Gram, rank-select of the groupsize-2 nearest neighbours, score
//   KC3 k_krum_vote      one block: per-verifier selection of the n_accept lowest scores, signature
//                        count per worker row, approval (>= need), leader cap by arrival rank
// Limits: U <= 1024 rows, inbox n <= 256 on this path; larger committees take the *_big kernels below.
// =====================================================================================
namespace {
__device__ __forceinline__ int pair_index(int ti, int tj, int T) {
  // row-major enumeration of the upper triangle ti <= tj of a T x T tile grid
  return ti * T - (ti * (ti - 1)) / 2 + (tj - ti);
}
// Gram entry G[a][b] out of the reduced upper-triangular tiles
__device__ __forceinline__ double gram_at(const double* gram, int T, int a, int b) {
  int ta = a >> 4, tb = b >> 4, ra = a & 15, rb = b & 15;
  if (ta > tb) {
    const int t = ta; ta = tb; tb = t;
    const int r = ra; ra = rb; rb = r;
  }
  return gram[(size_t)pair_index(ta, tb, T) * 256 + ra * 16 + rb];
}
}  // namespace

// rows [0, U1) of the Gram's operand come from X (row stride D), rows [U1, U) from X2 (row stride
// stride2): the committee Krum's noise-aware form stacks the workers' deltas over the noisers'
// pre-sampled vectors of this iteration (a strided view of the resident noise table)
extern "C" __global__ void __launch_bounds__(256) k_gram_pairs(const float* X, int U, int D, int kchunk, int T,
                                                              double* part, double* gram, unsigned int* count,
                                                              const float* X2, int U1, long long stride2, int pair0,
                                                              const double* nn, int tn0) {
  // high: at priority 1 the pre-step's commitment MSM squeezed it to ~220 us, and its resident workgroups kept
  // the speculative share MSM from being dispatched until it ended (docs/PERF.md round 5); its work is ~10 us
  BSC_SET_PRIO(BSC_PRIO_CRITICAL);
  __shared__ double red[4][256];
  // this launch covers the tile pairs [pair0, pair0 + gridDim.x) (several ranks split one Gram); part and
  // the arrival counters are indexed by the launch-local pair index, gram by the global one
  const int lp = blockIdx.x, pair = pair0 + lp, sp = blockIdx.y;
  const int npairs = gridDim.x;
  // decode the pair index (T <= 64: a short scan)
  int ti = 0, rem = pair;
  while (rem >= T - ti) {
    rem -= T - ti;
    ++ti;
  }
  const int tj = ti + rem;
  if (nn != nullptr && ti >= tn0) {
    // both tiles hold noise rows only (rows >= U1): the noisers' pre-sampled vectors repeat with the iteration
    // modulo 100 (client_obj.py:61-63,97-98), so this block of the Gram was computed at setup, by this kernel
    // (bit-identical entries), into the dense [U2, U2] table nn of this iteration: copy, no split-K
    if (sp == 0) {
      const int U2 = U - U1, e = threadIdx.x;
      const int a = ti * 16 + (e >> 4) - U1, b = tj * 16 + (e & 15) - U1;
      gram[(size_t)pair * 256 + e] = (a < U2 && b < U2) ? nn[(size_t)a * U2 + b] : 0.0;
    }
    return;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int i = ti * 16 + (lane & 15), j = tj * 16 + (lane & 15), kk = lane >> 4;
  const bool va = i < U, vb = j < U;
  const int ia = va ? i : 0, jb = vb ? j : 0;
  const float* xa = ia < U1 ? X + (size_t)ia * D : X2 + (size_t)(ia - U1) * stride2;
  const float* xb = jb < U1 ? X + (size_t)jb * D : X2 + (size_t)(jb - U1) * stride2;
  // this block's K range, split into 4 wave ranges that are multiples of 4
  const int k0b = sp * kchunk, k1b = min(D, k0b + kchunk);
  const int per = (((k1b - k0b) + 15) / 16) * 4;
  int k = k0b + wid * per;
  const int kend = min(k1b, k + per);
  f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
  // 32 k per step: lane (r, kk) reads k + 16h + 4kk .. +3 of its row as ONE 16-byte load per half h
  // (4 vector loads per step instead of 16 dword loads); MFMA step (h, c) then sums the elements
  // k + 16h + 4kk + c over kk -- the same k set for A and B, only the summation order differs
  typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
  for (; k + 32 <= kend; k += 32) {
    const f32x4u a0 = *(const f32x4u*)(xa + k + 4 * kk), a1 = *(const f32x4u*)(xa + k + 16 + 4 * kk);
    const f32x4u b0 = *(const f32x4u*)(xb + k + 4 * kk), b1 = *(const f32x4u*)(xb + k + 16 + 4 * kk);
#pragma unroll
    for (int c = 0; c < 4; c += 2) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(va ? (double)a0[c] : 0.0, vb ? (double)b0[c] : 0.0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(va ? (double)a0[c + 1] : 0.0, vb ? (double)b0[c + 1] : 0.0, acc1,
                                                  0, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < 4; c += 2) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(va ? (double)a1[c] : 0.0, vb ? (double)b1[c] : 0.0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(va ? (double)a1[c + 1] : 0.0, vb ? (double)b1[c + 1] : 0.0, acc1,
                                                  0, 0, 0);
    }
  }
  for (; k < kend; k += 4) {
    const int kx = k + kk;
    const double a = (va && kx < kend) ? (double)xa[kx] : 0.0;
    const double b = (vb && kx < kend) ? (double)xb[kx] : 0.0;
    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
  }
  const f64x4 acc = acc0 + acc1;
  // D layout: lane l holds D[row (l>>4) + 4r][col l&15]
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wid][((lane >> 4) + 4 * r) * 16 + (lane & 15)] = acc[r];
  __syncthreads();
  const int e = threadIdx.x;  // 256 threads = the 16x16 tile
  part[((size_t)sp * npairs + lp) * 256 + e] = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]);
  // the split-K partials are summed by k_gram_reduce (the next launch on the stream).  An in-kernel
  // last-block reduction needed an agent-scope release / acquire per block: on gfx950 that is an L2
  // write-back + invalidate (buffer_wbl2 / buffer_inv sc1) in each of the ~1450 blocks -- ~100 us for ~10 us of
  // MFMA work, and every kernel beside it (the share MSMs' table lookups) lost its L2 lines too
}

// KC1b: tile pair p's reduced Gram tile = sum of its split-K partials in split order (bit-reproducible, the
// same order as before); the noise-only tile pairs were copied from the table by k_gram_pairs (split 0)
extern "C" __global__ void __launch_bounds__(256) k_gram_reduce(const double* part, double* gram, int npairs,
                                                               int nsplit, int pair0, int T, int tn0, int has_nn) {
  BSC_SET_PRIO(BSC_PRIO_CRITICAL);
  const int lp = blockIdx.x, pair = pair0 + lp, e = threadIdx.x;
  if (has_nn) {
    int ti = 0, rem = pair;
    while (rem >= T - ti) {
      rem -= T - ti;
      ++ti;
    }
    if (ti >= tn0) return;   // noise x noise: already in place
  }
  double g = 0.0;
  for (int q = 0; q < nsplit; ++q) g += part[((size_t)q * npairs + lp) * 256 + e];
  gram[(size_t)pair * 256 + e] = g;
}

extern "C" __global__ void __launch_bounds__(256) k_krum_rows(const double* gram, int T, const int* inbox, int n,
                                                             int groupsize, double* scores) {
  __shared__ double row[256];
  __shared__ double kept[256];
  __shared__ double gdiag_a;
  const int i = blockIdx.x, v = blockIdx.y, t = threadIdx.x;
  const int* box = inbox + (size_t)v * n;
  const int a = box[i];
  if (t == 0) gdiag_a = gram_at(gram, T, a, a);
  __syncthreads();
  if (t < n) {
    const int b = box[t];
    const double gab = gram_at(gram, T, a, b);
    const double gbb = gram_at(gram, T, b, b);
    row[t] = gdiag_a + gbb - 2.0 * gab;
  }
  __syncthreads();
  if (t < n) {
    const double val = row[t];
    int rank = 0;
    for (int k2 = 0; k2 < n; ++k2) {
      const double u = row[k2];
      rank += (u < val) || (u == val && k2 < t);
    }
    kept[t] = (rank >= 1 && rank < groupsize - 1) ? val : 0.0;
  }
  __syncthreads();
  if (t == 0) {
    double s = 0.0;
    for (int j = 0; j < n; ++j) s += kept[j];
    scores[(size_t)v * n + i] = s;
  }
}

// KC2, noise-aware form: the candidate rows are x_a = delta_a + (1/nn) sum_s sc[a][s] t_{nz[a][s]}
// (the noisers' pre-sampled vectors, main.go:1592-1660), and the Gram was taken over the stacked
// [deltas; noise vectors] rows, so <x_a, x_b> expands into (1 + nn)^2 Gram entries -- the
// d-dimensional work (the Gram) runs before the noisers are known (they come from the workers' VRF
// outputs on the host); only this O(n^2 nn^2) assembly waits for them.
namespace {
// the noisers' ids and weights: device arrays, or (NoiseArg) the kernel's argument block -- the round's tables
// are ~1.6 KB at 100 peers, so they ride in the launch instead of an upload copy the selection queues behind
#define NOISE_ARG_MAX 400
struct NoiseArg {
  int nz[NOISE_ARG_MAX];
  float sc[NOISE_ARG_MAX];
};
struct NoisePtr {
  const int* z;
  const float* s;
  __device__ __forceinline__ int nz(int i) const { return z[i]; }
  __device__ __forceinline__ float sc(int i) const { return s[i]; }
};
struct NoiseByVal {
  const NoiseArg* a;
  __device__ __forceinline__ int nz(int i) const { return a->nz[i]; }
  __device__ __forceinline__ float sc(int i) const { return a->sc[i]; }
};

template <class N>
__device__ __forceinline__ double xx_dot(const double* gram, int T, int U1, N q, int nn, int a, int b) {
  double v = gram_at(gram, T, a, b);
  const double inv = 1.0 / (double)nn;
  for (int t = 0; t < nn; ++t) {
    v += inv * (double)q.sc(b * nn + t) * gram_at(gram, T, a, U1 + q.nz(b * nn + t));
    v += inv * (double)q.sc(a * nn + t) * gram_at(gram, T, U1 + q.nz(a * nn + t), b);
  }
  for (int s2 = 0; s2 < nn; ++s2)
    for (int t = 0; t < nn; ++t)
      v += inv * inv * (double)q.sc(a * nn + s2) * (double)q.sc(b * nn + t) *
           gram_at(gram, T, U1 + q.nz(a * nn + s2), U1 + q.nz(b * nn + t));
  return v;
}
// wrapper kept for k_krum_rows_big (device arrays)
__device__ __forceinline__ double xx_dot(const double* gram, int T, int U1, const int* nz, const float* sc, int nn,
                                         int a, int b) {
  return xx_dot(gram, T, U1, NoisePtr{nz, sc}, nn, a, b);
}

template <class N>
__device__ __forceinline__ void krum_rows_noise_body(const double* gram, int T, int U1, N q, int nn, const int* inbox,
                                                     int n, int groupsize, double* scores) {
  __shared__ double row[256];
  BSC_SET_PRIO(BSC_PRIO_CRITICAL);
  __shared__ double kept[256];
  __shared__ double xaa;
  const int i = blockIdx.x, v = blockIdx.y, t = threadIdx.x;
  const int* box = inbox + (size_t)v * n;
  const int a = box[i];
  if (t == 0) xaa = xx_dot(gram, T, U1, q, nn, a, a);
  __syncthreads();
  if (t < n) {
    const int b = box[t];
    row[t] = xaa + xx_dot(gram, T, U1, q, nn, b, b) - 2.0 * xx_dot(gram, T, U1, q, nn, a, b);
  }
  __syncthreads();
  if (t < n) {
    const double val = row[t];
    int rank = 0;
    for (int k2 = 0; k2 < n; ++k2) {
      const double u = row[k2];
      rank += (u < val) || (u == val && k2 < t);
    }
    kept[t] = (rank >= 1 && rank < groupsize - 1) ? val : 0.0;
  }
  __syncthreads();
  if (t == 0) {
    double s = 0.0;
    for (int j = 0; j < n; ++j) s += kept[j];
    scores[(size_t)v * n + i] = s;
  }
}
}  // namespace

extern "C" __global__ void __launch_bounds__(256) k_krum_rows_noise(const double* gram, int T, int U1,
                                                                   const int* nz, const float* sc, int nn,
                                                                   const int* inbox, int n, int groupsize,
                                                                   double* scores) {
  krum_rows_noise_body(gram, T, U1, NoisePtr{nz, sc}, nn, inbox, n, groupsize, scores);
}

extern "C" __global__ void __launch_bounds__(256) k_krum_rows_noise_ka(const double* gram, int T, int U1, NoiseArg q,
                                                                      int nn, const int* inbox, int n, int groupsize,
                                                                      double* scores) {
  krum_rows_noise_body(gram, T, U1, NoiseByVal{&q}, nn, inbox, n, groupsize, scores);
}

// h_acc / h_node (nullable): the same verdicts written straight into pinned host memory (the host reads them
// after the kernel's event: no read-back copy); amap / alive / nspec (nullable): the speculative share MSM's
// row flags set from the block mask (k_set_alive fused: alive[i] = node[amap[i]], 0 where amap[i] < 0)
extern "C" __global__ void __launch_bounds__(1024) k_krum_vote(const double* scores, const int* inbox, int V, int n,
                                                              int n_accept, int U, int need, const int* lead_rank,
                                                              int cap, int* acc, int* node, int* h_acc, int* h_node,
                                                              const int* amap, int nspec, int* alive) {
  BSC_SET_PRIO(BSC_PRIO_CRITICAL);
  __shared__ int sigs[1024];
  __shared__ int appr[1024];
  __shared__ int lr[1024];
  __shared__ int kept[1024];
  __shared__ double sv[4][256];
  const int t = threadIdx.x;
  for (int w = t; w < U; w += 1024) {
    sigs[w] = 0;
    lr[w] = lead_rank[w];
  }
  // per-verifier Multi-Krum selection: the n_accept lowest scores (index tie-break); four verifiers
  // at a time, their scores staged in LDS
  for (int v0 = 0; v0 < V; v0 += 4) {
    const int nv = min(4, V - v0);
    __syncthreads();
    for (int e = t; e < nv * n; e += 1024) sv[e / n][e % n] = scores[(size_t)(v0 + e / n) * n + e % n];
    __syncthreads();
    for (int e = t; e < nv * n; e += 1024) {
      const int vv = e / n, i = e % n;
      const double s = sv[vv][i];
      int rank = 0;
      for (int j = 0; j < n; ++j) rank += (sv[vv][j] < s) || (sv[vv][j] == s && j < i);
      const int ok = rank < n_accept ? 1 : 0;
      const size_t ge = (size_t)(v0 + vv) * n + i;
      acc[ge] = ok;
      if (h_acc != nullptr) h_acc[ge] = ok;
      if (ok) atomicAdd(&sigs[inbox[ge]], 1);
    }
  }
  __syncthreads();
  // approval: >= need signatures among the submitted workers (lead_rank >= 0)
  for (int w = t; w < U; w += 1024) appr[w] = (lr[w] >= 0 && sigs[w] >= need) ? 1 : 0;
  __syncthreads();
  // the leader's block: the first `cap` approved rows in leader arrival order (cap <= 0: all)
  for (int w = t; w < U; w += 1024) {
    int keep = appr[w];
    if (keep && cap > 0) {
      int before = 0;
      const int r = lr[w];
      for (int x = 0; x < U; ++x) before += appr[x] && lr[x] < r;
      keep = before < cap;
    }
    node[w] = keep;
    kept[w] = keep;
    if (h_node != nullptr) h_node[w] = keep;
  }
  if (alive != nullptr) {
    __syncthreads();
    for (int i = t; i < nspec; i += 1024) {
      const int j = amap[i];
      __hip_atomic_store(alive + i, (j >= 0 && j < U && kept[j]) ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (h_acc != nullptr || h_node != nullptr) __threadfence_system();
}

// ---- large committees (an inbox of more than 256 updates, or more than 1024 candidate rows): the
// reference's Krum has no size limit (client_obj.py:114-143).  A row's distances are sorted in LDS
// (bitonic) and its score is the sum of the sorted values at positions 1 .. groupsize-2 -- the same
// multiset as k_krum_rows' rank select (ties cannot change it); the vote counts signatures in a global
// workspace and the leader cap runs one thread per candidate row.  Limits: U <= 8192, n <= 4096.
namespace {
__device__ void bitonic_sort_lds(double* a, int npow2) {
  for (int k = 2; k <= npow2; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < npow2; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const bool up = (i & k) == 0;
          const double x = a[i], y = a[ixj];
          if ((x > y) == up) {
            a[i] = y;
            a[ixj] = x;
          }
        }
      }
      __syncthreads();
    }
}
}  // namespace

template <bool NOISE>
__global__ void __launch_bounds__(1024) k_krum_rows_big(const double* gram, int T, int U1, const int* nz,
                                                        const float* sc, int nn, const int* inbox, int n, int npow2,
                                                        int groupsize, double* scores) {
  extern __shared__ double row[];   // [npow2]
  __shared__ double xaa;
  const int i = blockIdx.x, v = blockIdx.y;
  const int* box = inbox + (size_t)v * n;
  const int a = box[i];
  if (threadIdx.x == 0) xaa = NOISE ? xx_dot(gram, T, U1, nz, sc, nn, a, a) : gram_at(gram, T, a, a);
  __syncthreads();
  for (int t = threadIdx.x; t < npow2; t += blockDim.x) {
    double val = __builtin_huge_val();
    if (t < n) {
      const int b = box[t];
      val = NOISE ? xaa + xx_dot(gram, T, U1, nz, sc, nn, b, b) - 2.0 * xx_dot(gram, T, U1, nz, sc, nn, a, b)
                  : xaa + gram_at(gram, T, b, b) - 2.0 * gram_at(gram, T, a, b);
    }
    row[t] = val;
  }
  __syncthreads();
  bitonic_sort_lds(row, npow2);
  if (threadIdx.x == 0) {
    double s = 0.0;
    const int hi = min(groupsize - 1, n);
    for (int j = 1; j < hi; ++j) s += row[j];
    scores[(size_t)v * n + i] = s;
  }
}

// per-verifier selection (one block per verifier): the n_accept lowest scores, index tie-break; the
// signatures each candidate row collects go to `sigs` (zeroed by the launcher)
extern "C" __global__ void __launch_bounds__(1024) k_krum_select_big(const double* scores, const int* inbox, int n,
                                                                    int n_accept, int* acc, int* sigs) {
  extern __shared__ double sv[];   // [n]
  const int v = blockIdx.x;
  for (int e = threadIdx.x; e < n; e += blockDim.x) sv[e] = scores[(size_t)v * n + e];
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double s = sv[i];
    int rank = 0;
    for (int j = 0; j < n; ++j) rank += (sv[j] < s) || (sv[j] == s && j < i);
    const int ok = rank < n_accept ? 1 : 0;
    acc[(size_t)v * n + i] = ok;
    if (ok) atomicAdd(&sigs[inbox[(size_t)v * n + i]], 1);
  }
}

// approval (>= need signatures, submitted) and the leader's cap: the first `cap` approved rows in
// leader arrival order (cap <= 0: all); one thread per candidate row
extern "C" __global__ void __launch_bounds__(256) k_krum_cap_big(const int* sigs, const int* lead_rank, int U,
                                                                int need, int cap, int* node) {
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= U) return;
  const int lr = lead_rank[w];
  int keep = (lr >= 0 && sigs[w] >= need) ? 1 : 0;
  if (keep && cap > 0) {
    int before = 0;
    for (int x = 0; x < U; ++x) before += (lead_rank[x] >= 0 && sigs[x] >= need && lead_rank[x] < lr) ? 1 : 0;
    keep = before < cap;
  }
  node[w] = keep;
}

extern "C" int bsc_set_alive(const int* accept, const int* src, int n, int* alive, void* stream);
namespace {
int krum_vote_any(hipStream_t s, const double* scores, const int* inbox, int V, int n, int n_accept, int U, int need,
                  const int* lead_rank, int cap, int* acc, int* node, int* ws, int* h_out = nullptr,
                  const int* amap = nullptr, int nspec = 0, int* alive = nullptr) {
  if (U <= 1024 && n <= 256) {
    hipLaunchKernelGGL(k_krum_vote, dim3(1), dim3(1024), 0, s, scores, inbox, V, n, n_accept, U, need, lead_rank,
                       cap, acc, node, h_out, h_out != nullptr ? h_out + (size_t)V * n : nullptr, amap, nspec, alive);
  } else {
    if (ws == nullptr) return -1;
    hipMemsetAsync(ws, 0, (size_t)U * sizeof(int), s);
    hipLaunchKernelGGL(k_krum_select_big, dim3(V), dim3(1024), (size_t)n * sizeof(double), s, scores, inbox, n,
                       n_accept, acc, ws);
    hipLaunchKernelGGL(k_krum_cap_big, dim3((U + 255) / 256), dim3(256), 0, s, (const int*)ws, lead_rank, U, need, cap,
                       node);
    // large committees: the read-back copy and the flag update stay separate launches
    if (h_out != nullptr && hipMemcpyAsync(h_out, acc, ((size_t)V * n + U) * sizeof(int), hipMemcpyDeviceToHost, s) !=
                                hipSuccess)
      return -1;
    if (alive != nullptr && nspec > 0 && bsc_set_alive(node, amap, nspec, alive, s) != 0) return -1;
  }
  return 0;
}
int pow2_at_least(int n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}
}  // namespace

// =====================================================================================
// LSH sieve (ML/code/logistic_aggregator.py:7-29, the third poisoning defence next to Krum and RONI):
// every update's weight is 1 / #(its near neighbours within squared distance thr among the
// (centred) updates), so a cluster of sybil updates shares the weight of one.  The reference asks a
// FALCONN index (random-projection LSH) for the neighbours; here:
//   LS1 k_lsh_codes    L tables x K sign bits of <x_i - mu, r> per row (one block per row)
//   LS2 k_lsh_count    neighbour count of each listed row: candidates share a bucket in some table
//                      (L = 0: every pair, the exact query), confirmed on the f64 Gram (KC1 tiles;
//                      centring cancels in differences)
//   LS3 k_weighted_rows  out = sum_i w_i x_i in fp64
// =====================================================================================
extern "C" __global__ void __launch_bounds__(256) k_lsh_codes(const float* X, const float* mu, int n, int D,
                                                             const float* planes, int L, int K,
                                                             unsigned int* codes) {
  __shared__ float red[4][64];
  const int i = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int P = L * K;   // <= 64 planes
  float acc[64];
#pragma unroll
  for (int q = 0; q < 64; ++q) acc[q] = 0.f;
  for (int k = t; k < D; k += 256) {
    const float v = X[(size_t)i * D + k] - mu[k];
#pragma unroll
    for (int q = 0; q < 64; ++q)
      if (q < P) acc[q] += v * planes[(size_t)q * D + k];
  }
#pragma unroll
  for (int q = 0; q < 64; ++q) {
    float v = acc[q];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[wid][q] = v;
  }
  __syncthreads();
  if (t < L) {
    unsigned int c = 0;
    for (int b = 0; b < K; ++b) {
      const int q = t * K + b;
      const float v = (red[0][q] + red[1][q]) + (red[2][q] + red[3][q]);
      c |= (v > 0.f ? 1u : 0u) << b;
    }
    codes[(size_t)i * L + t] = c;
  }
}

extern "C" __global__ void __launch_bounds__(256) k_lsh_count(const double* gram, int T, const unsigned int* codes,
                                                             int L, const int* rows, int m, double thr, int* counts) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= m) return;
  const int i = rows[a];
  const double gii = gram_at(gram, T, i, i);
  int c = 0;
  for (int b = 0; b < m; ++b) {
    const int j = rows[b];
    bool cand = L == 0 || j == i;
    for (int tb = 0; tb < L && !cand; ++tb) cand = codes[(size_t)i * L + tb] == codes[(size_t)j * L + tb];
    if (!cand) continue;
    const double d2 = gii + gram_at(gram, T, j, j) - 2.0 * gram_at(gram, T, i, j);
    c += (j == i || d2 < thr) ? 1 : 0;
  }
  counts[a] = c;
}

extern "C" __global__ void k_weighted_rows(const float* X, int n, int D, const double* w, double* out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= D) return;
  double acc = 0.0;
  for (int i = 0; i < n; ++i) acc += w[i] * (double)X[(size_t)i * D + k];
  out[k] = acc;
}

extern "C" int bsc_lsh_codes(const float* X, const float* mu, int n, int D, const float* planes, int L, int K,
                             unsigned int* codes, void* stream) {
  if (n <= 0 || L <= 0) return 0;
  if (L * K > 64 || K > 32 || K <= 0) return -1;
  hipLaunchKernelGGL(k_lsh_codes, dim3(n), dim3(256), 0, (hipStream_t)stream, X, mu, n, D, planes, L, K, codes);
  return (int)hipGetLastError();
}
extern "C" int bsc_lsh_count(const double* gram, int U, const unsigned int* codes, int L, const int* rows, int m,
                             double thr, int* counts, void* stream) {
  if (m <= 0) return 0;
  const int T = (U + 15) / 16;
  hipLaunchKernelGGL(k_lsh_count, dim3((m + 255) / 256), dim3(256), 0, (hipStream_t)stream, gram, T, codes, L, rows, m,
                     thr, counts);
  return (int)hipGetLastError();
}
extern "C" int bsc_weighted_rows(const float* X, int n, int D, const double* w, double* out, void* stream) {
  if (D <= 0) return 0;
  hipLaunchKernelGGL(k_weighted_rows, dim3((D + 255) / 256), dim3(256), 0, (hipStream_t)stream, X, n, D, w, out);
  return (int)hipGetLastError();
}

// =====================================================================================
// K2: classification error of a softmax model over up to two row sets in ONE launch (test rows
// [0, split), attack rows [split, N)): err[row >= split] += #(argmax != label).
// One wave per 16-row tile: logits = X_tile[16 x D_IN] . W^T on v_mfma_f32_16x16x4f32 (lane l
// holds A[row l&15][k l>>4] with the (x-0.5)/0.5 transform fused and B[k][class l&15]; two
// accumulators hide the 40-cycle dependent latency, loads are issued 8 k-steps ahead), then the
// argmax across the 16 class lanes by xor-shuffles (first maximum, like np.argmax) and one atomic
// per (wave, set).  Replaces a wave-per-row kernel that re-staged W into 64 KB of LDS per block.
// =====================================================================================
extern "C" __global__ void __launch_bounds__(256) k_eval_error(const float* X, const int* y, int N, int D_IN,
                                                              int D_OUT, const double* W, int transform, int split,
                                                              unsigned int* err) {
  // one block per 16-row tile; its 4 waves split K and reduce the logits through LDS
  __shared__ float red[4][4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int row0 = blockIdx.x * 16;
  const int i = lane & 15, kk = lane >> 4;
  const float* xr = X + (size_t)min(row0 + i, N - 1) * D_IN;
  const bool cval = i < D_OUT;
  const double* wr = W + (size_t)(cval ? i : 0) * D_IN;
  const float tsub = transform ? 0.5f : 0.f, tmul = transform ? 2.f : 1.f;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const int kq = ((D_IN + 15) / 16) * 4;  // this wave's K range: multiple of 4
  int k0 = wid * kq;
  const int kend = min(D_IN, k0 + kq);
  for (; k0 + 32 <= kend; k0 += 32) {
    float a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + 4 * u + kk;
      a[u] = xr[k];
      b[u] = cval ? (float)wr[k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32((a[u] - tsub) * tmul, b[u], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32((a[u + 1] - tsub) * tmul, b[u + 1], acc1, 0, 0, 0);
    }
  }
  for (; k0 < kend; k0 += 4) {
    const int k = k0 + kk;
    const float a = k < kend ? (xr[k] - tsub) * tmul : 0.f;
    const float b = (k < kend && cval) ? (float)wr[k] : 0.f;
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc0, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wid][r][lane] = acc0[r] + acc1[r];
  __syncthreads();
  if (wid != 0) return;
  const float bias = cval ? (float)W[(size_t)D_OUT * D_IN + i] : 0.f;
  unsigned int cnt0 = 0, cnt1 = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    // D layout of 16x16x4 f32: lane l holds D[row (l>>4)*4 + r][class l&15]
    const float logit = (red[0][r][lane] + red[1][r][lane]) + (red[2][r][lane] + red[3][r][lane]);
    float bv = cval ? logit + bias : -__builtin_huge_valf();
    int bc = i;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 16);
      const int oc = __shfl_xor(bc, o, 16);
      if (ov > bv || (ov == bv && oc < bc)) {
        bv = ov;
        bc = oc;
      }
    }
    const int row = row0 + kk * 4 + r;
    if (i == 0 && row < N && bc != y[row]) {
      if (row < split) ++cnt0;
      else ++cnt1;
    }
  }
  if (i == 0) {
    if (cnt0) atomicAdd(err, cnt0);
    if (cnt1) atomicAdd(err + 1, cnt1);
  }
}

// The same on a cached, pre-transformed test set: Xt[tile][g][64] holds (x - 0.5) / 0.5 of row
// tile*16 + (l & 15), feature 4g + (l >> 4) for lane l -- exactly the A operand of one
// v_mfma_f32_16x16x4f32 step -- built once per task (the test rows never change).  Each MFMA step is one
// coalesced 256-byte load: the row-strided gathers and the per-element transform of k_eval_error are gone.
extern "C" __global__ void __launch_bounds__(256) k_eval_error_t(const float* Xt, const int* y, int N, int KG, int D_IN,
                                                                int D_OUT, const double* W, int split,
                                                                unsigned int* err, unsigned int* err_host) {
  BSC_SET_PRIO(BSC_PRIO_AHEAD);
  // 4 waves per tile split the K loop (latency: the evaluation is read one round later and must be done by
  // then under the share MSM's load), then reduce the logits through LDS
  __shared__ float red[4][4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, tile = blockIdx.x;
  const int i = lane & 15, kk = lane >> 4;
  const bool cval = i < D_OUT;
  const double* wr = W + (size_t)(cval ? i : 0) * D_IN;
  const float* xp = Xt + (size_t)tile * KG * 64 + lane;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const int gq = (KG + 3) / 4;
  int g = wid * gq;
  const int gend = min(KG, g + gq);
  for (; g + 8 <= gend; g += 8) {
    float a[8], b[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a[u] = xp[(size_t)(g + u) * 64];
      const int k = 4 * (g + u) + kk;
      b[u] = (cval && k < D_IN) ? (float)wr[k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; u += 2) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b[u], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u + 1], b[u + 1], acc1, 0, 0, 0);
    }
  }
  for (; g < gend; ++g) {
    const int k = 4 * g + kk;
    const float b = (cval && k < D_IN) ? (float)wr[k] : 0.f;
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(xp[(size_t)g * 64], b, acc0, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wid][r][lane] = acc0[r] + acc1[r];
  __syncthreads();
  if (wid != 0) return;
  const float bias = cval ? (float)W[(size_t)D_OUT * D_IN + i] : 0.f;
  unsigned int cnt0 = 0, cnt1 = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float logit = (red[0][r][lane] + red[1][r][lane]) + (red[2][r][lane] + red[3][r][lane]);
    float bv = cval ? logit + bias : -__builtin_huge_valf();
    int bc = i;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 16);
      const int oc = __shfl_xor(bc, o, 16);
      if (ov > bv || (ov == bv && oc < bc)) {
        bv = ov;
        bc = oc;
      }
    }
    const int row = tile * 16 + kk * 4 + r;
    if (i == 0 && row < N && bc != y[row]) {
      if (row < split) ++cnt0;
      else ++cnt1;
    }
  }
  if (i == 0) {
    if (cnt0) atomicAdd(err, cnt0);
    if (cnt1) atomicAdd(err + 1, cnt1);
  }
  // err_host (bsc_eval_error_t_rb): k_eval_finish, the next launch, hands the counts to the host and re-zeroes
  // them.  (A last-tile hand-off inside this kernel needed an agent-scope fence per wave -- on gfx950 an L2
  // write-back + invalidate, ~625 of them beside the share MSMs.)
  (void)err_host;
}

// the evaluation's two counts into pinned host memory, counters re-zeroed for the next launch: one wave, behind
// k_eval_error_t on its stream (no fill and no copy blit: each waited ~20-40 us for a CU slot behind the MSMs)
extern "C" __global__ void __launch_bounds__(64) k_eval_finish(unsigned int* err, unsigned int* err_host) {
  if (threadIdx.x == 0) {
    err_host[0] = err[0];
    err_host[1] = err[1];
    err[0] = 0u;
    err[1] = 0u;
    err[2] = 0u;
  }
}

// =====================================================================================
// K12: exact recovery of the aggregated chunk polynomials from miner shares.
// ys: int64 [nchunks][npts], xs: int [npts] distinct; deg+1 <= npts.  Newton divided differences
// in 128-bit on the deg+1 nodes of smallest |x|, verified against every share.  Writes the
// dequantised aggregate into W_new = W + coeff / 10^prec  (fp64, the reference's mat.Dense.Add).
// status[k] = 1 exact, 0 inconsistent shares (caller falls back to least squares).
// =====================================================================================
namespace {
__device__ __forceinline__ bool div_small(__int128 a, long long d, __int128* q) {
  // exact division of a signed 128-bit value by a small non-zero divisor (|d| < 2^31)
  const bool neg = (a < 0) != (d < 0);
  unsigned __int128 m = a < 0 ? (unsigned __int128)(-a) : (unsigned __int128)a;
  const unsigned long long dd = d < 0 ? (unsigned long long)(-d) : (unsigned long long)d;
  const unsigned long long hi = (unsigned long long)(m >> 64), lo = (unsigned long long)m;
  const unsigned long long qh = hi / dd;
  unsigned long long r = hi % dd;
  unsigned long long t = (r << 32) | (lo >> 32);
  const unsigned long long q1 = t / dd;
  r = t % dd;
  t = (r << 32) | (lo & 0xFFFFFFFFull);
  const unsigned long long q0 = t / dd;
  r = t % dd;
  if (r != 0) return false;
  unsigned __int128 qq = ((unsigned __int128)qh << 64) | ((unsigned __int128)q1 << 32) | q0;
  *q = neg ? -(__int128)qq : (__int128)qq;
  return true;
}
}  // namespace

extern "C" __global__ void k_recover(const long long* ys, int nchunks, int npts, const int* xs, int poly, int d,
                                     const double* W, double qscale, double* W_new, long long* coeffs,
                                     int* status) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nchunks) return;
  const int n = poly;  // degree poly-1
  // node choice: smallest |x| first (stable)
  int order[32];
  for (int i = 0; i < npts; ++i) order[i] = i;
  for (int a = 1; a < npts; ++a) {
    const int v = order[a];
    const int av = xs[v] < 0 ? -xs[v] : xs[v];
    int b = a - 1;
    while (b >= 0) {
      const int ob = xs[order[b]] < 0 ? -xs[order[b]] : xs[order[b]];
      if (ob > av || (ob == av && xs[order[b]] > xs[v])) {
        order[b + 1] = order[b];
        --b;
      } else {
        break;
      }
    }
    order[b + 1] = v;
  }
  __int128 nx[16], dd[16], c[16];
  bool ok = npts >= n;
  for (int i = 0; i < n && ok; ++i) {
    nx[i] = xs[order[i]];
    dd[i] = ys[(size_t)k * npts + order[i]];
  }
  for (int lvl = 1; lvl < n && ok; ++lvl)
    for (int i = n - 1; i >= lvl && ok; --i) {
      __int128 q;
      ok = div_small(dd[i] - dd[i - 1], (long long)(nx[i] - nx[i - lvl]), &q);
      dd[i] = q;
    }
  if (ok) {
    for (int i = 0; i < n; ++i) c[i] = 0;
    c[0] = dd[n - 1];
    int cur = 0;
    for (int kk = n - 2; kk >= 0; --kk) {
      for (int j = cur + 1; j >= 1; --j) c[j] = c[j - 1] - nx[kk] * c[j];
      c[0] = -nx[kk] * c[0] + dd[kk];
      ++cur;
    }
    for (int pt = 0; pt < npts && ok; ++pt) {
      __int128 acc = 0;
      for (int j = n - 1; j >= 0; --j) acc = acc * xs[pt] + c[j];
      ok = acc == (__int128)ys[(size_t)k * npts + pt];
    }
  }
  status[k] = ok ? 1 : 0;
  const int prev = k * poly;
  for (int j = 0; j < n; ++j) {
    const long long v = ok ? (long long)c[j] : 0;
    coeffs[(size_t)k * n + j] = v;
    const int idx = prev + j;
    if (idx < d) W_new[idx] = W[idx] + (double)v / qscale;
  }
}

// =====================================================================================
// K12, fused form: share-value sums + exact recovery with precomputed integer weights.
// For a fixed x-point layout (the contributing miners' parts) the inverse Vandermonde on the `poly`
// basis nodes is A / Dn with integer A (host-computed exactly, |A| < 2^40, Dn = 2^s * Dodd), so
// c_j = (sum_i A[j][i] y_{basis_i}) / Dn -- an int128 mat-vec and one exact division, done as a
// shift plus a multiplication by Dodd^-1 mod 2^128 (no 128-bit divisions).  Every share is then
// re-checked by Horner in int128 (status 0 -> the host's least squares, like the old kernel).
// The miners' sums are fused in: agg[k][p] = sum over rows r with mask[r] of ys[r][k][ycols[p]]
// (nrows = 1 and mask = null when ys already holds totals).  One block: 8 chunks.
// =====================================================================================
namespace {
constexpr int RW_CPB = 8;     // chunks per block
constexpr int RW_MAXP = 32;   // points per chunk
constexpr int RW_MAXC = 16;   // coefficients per chunk
}  // namespace

extern "C" __global__ void __launch_bounds__(256) k_recover_w(
    const long long* ys, int nrows, long long rstride, int nch, int T, const int* mask, const int* ycols, const int* xs, int npts,
    const long long* A, const int* basis, int poly, int shift, unsigned long long inv_lo, unsigned long long inv_hi,
    int d, const double* W, double qscale, double* W_new, long long* coeffs, int* status, long long* agg_out,
    double* h_W, int* h_status, long long* h_clock) {
  BSC_SET_PRIO(BSC_PRIO_CRITICAL);
  // several ranks (h_clock): each rank's row carries its clock right after its share sums -- block 0 mirrors
  // them to the host with the model (no strided read-back copy behind the kernel)
  if (h_clock != nullptr && blockIdx.x == 0 && threadIdx.x < nrows)
    h_clock[threadIdx.x] = ys[(size_t)threadIdx.x * rstride + (size_t)nch * T];
  __shared__ long long agg[RW_CPB][RW_MAXP];
  __shared__ __int128 cf[RW_CPB][RW_MAXC];
  __shared__ int ok[RW_CPB];
  const int t = threadIdx.x;
  const int k0 = blockIdx.x * RW_CPB;
  if (t < RW_CPB) ok[t] = 1;
  // 1. the miners' share sums for this block's chunks
  for (int e = t; e < RW_CPB * npts; e += 256) {
    const int c = e / npts, p = e % npts, k = k0 + c;
    if (k >= nch) continue;
    long long s = 0;
    const int col = ycols[p];
    for (int r = 0; r < nrows; ++r)
      if (mask == nullptr || mask[r]) s += ys[(size_t)r * rstride + (size_t)k * T + col];
    agg[c][p] = s;
    agg_out[(size_t)k * npts + p] = s;
  }
  __syncthreads();
  // 2. coefficients: int128 mat-vec, exact division by Dn = 2^shift * Dodd
  const unsigned __int128 inv = ((unsigned __int128)inv_hi << 64) | inv_lo;
  for (int e = t; e < RW_CPB * poly; e += 256) {
    const int c = e / poly, j = e % poly;
    if (k0 + c >= nch) continue;
    __int128 n = 0;
    for (int i = 0; i < poly; ++i) n += (__int128)A[j * poly + i] * (__int128)agg[c][basis[i]];
    bool exact = (shift == 0) || ((n & ((((__int128)1) << shift) - 1)) == 0);
    const __int128 q = (__int128)((unsigned __int128)(n >> shift) * inv);
    // a true coefficient is tiny next to 2^100; an inexact division lands anywhere in 2^128
    const __int128 lim = ((__int128)1) << 100;
    exact = exact && q < lim && q > -lim;
    cf[c][j] = q;
    if (!exact) atomicAnd(&ok[c], 0);
  }
  __syncthreads();
  // 3. every share must lie on the recovered polynomial (Horner, int128)
  for (int e = t; e < RW_CPB * npts; e += 256) {
    const int c = e / npts, p = e % npts;
    if (k0 + c >= nch) continue;
    __int128 acc = 0;
    const __int128 x = xs[p];
    for (int j = poly - 1; j >= 0; --j) acc = acc * x + cf[c][j];
    if (acc != (__int128)agg[c][p]) atomicAnd(&ok[c], 0);
  }
  __syncthreads();
  // 4. outputs: coefficients, dequantised model update
  for (int e = t; e < RW_CPB * poly; e += 256) {
    const int c = e / poly, j = e % poly, k = k0 + c;
    if (k >= nch) continue;
    const bool good = ok[c] != 0;
    const long long v = good ? (long long)cf[c][j] : 0;
    coeffs[(size_t)k * poly + j] = v;
    if (j == 0) {
      status[k] = good ? 1 : 0;
      if (h_status != nullptr) h_status[k] = good ? 1 : 0;
    }
    const int idx = k * poly + j;
    if (idx < d) {
      const double w = W[idx] + (double)v / qscale;
      W_new[idx] = w;
      if (h_W != nullptr) h_W[idx] = w;   // pinned host mirror: the host reads it after the kernel's event
    }
  }
  // (no system-scope fence: the host reads the mirrors only after the kernel's completion event, whose
  // end-of-kernel release makes them visible; a fence per block was an L2 write-back per block on the chain)
}

// =====================================================================================
// Plain aggregation (non-secure-agg / FedSys): W_new = W + sum_r delta64[rows[r]] in fp64,
// in row order (mat.Dense.Add sequence).
// =====================================================================================
extern "C" __global__ void k_add_rows(const float* delta, int D, const int* rows, int nrows, const double* W,
                                      double* W_new) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= D) return;
  double acc = W[i];
  for (int r = 0; r < nrows; ++r) acc += (double)delta[(size_t)rows[r] * D + i];
  W_new[i] = acc;
}

// ---------------------------------------------------------------- C ABI launchers
static inline int nblk(long long n, int bs) { return (int)((n + bs - 1) / bs); }

// =====================================================================================
// K11 (several ranks): a rank's partial share-value sums of its kept rows, exact in int64:
// out[c] = sum over selected rows r of ys[r][c], c < C (C = nchunks * TOTAL_SHARES).  Rows come from an
// index list, a device-side selection mask (the committee's block mask) or all rows.  One thread per
// column; consecutive threads read consecutive columns of a row (coalesced), rows in order (exact and
// order-independent anyway: integer adds).  The sums go straight into the aggregation's all_gather.
// =====================================================================================
extern "C" __global__ void __launch_bounds__(256) k_sum_rows_i64(const long long* __restrict__ ys, int R, long long C,
                                                                const int* __restrict__ rows, int nsel,
                                                                const int* __restrict__ mask,
                                                                long long* __restrict__ out) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  long long s = 0;
  for (int i = 0; i < nsel; ++i) {
    const int r = rows != nullptr ? rows[i] : i;
    if (r < 0 || r >= R) continue;
    if (mask != nullptr && !mask[r]) continue;
    s += ys[(size_t)r * C + c];
  }
  out[c] = s;
}

extern "C" int bsc_sum_rows_i64(const long long* ys, int R, long long C, const int* rows, int nsel, const int* mask,
                                long long* out, void* stream) {
  if (C <= 0) return 0;
  if (rows == nullptr) nsel = R;
  hipLaunchKernelGGL(k_sum_rows_i64, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, (hipStream_t)stream, ys, R, C,
                     rows, nsel, mask, out);
  return (int)hipGetLastError();
}

// the same sums with one more int64 after them: out[C] = tail (the multi-rank send row's clock, kernels/round.hip)
// -- written by the sums' own launch instead of two memset launches behind it on the critical path; R = 0: zeros
extern "C" __global__ void __launch_bounds__(256) k_sum_rows_i64_tail(const long long* __restrict__ ys, int R,
                                                                     long long C, const int* __restrict__ mask,
                                                                     long long* __restrict__ out, long long tail) {
  const long long c = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c > C) return;
  if (c == C) {
    out[C] = tail;
    return;
  }
  long long s = 0;
  for (int r = 0; r < R; ++r)
    if (mask == nullptr || mask[r]) s += ys[(size_t)r * C + c];
  out[c] = s;
}

extern "C" int bsc_sum_rows_i64_tail(const long long* ys, int R, long long C, const int* mask, long long* out,
                                     long long tail, void* stream) {
  if (C < 0 || R < 0 || (R > 0 && ys == nullptr)) return -1;
  hipLaunchKernelGGL(k_sum_rows_i64_tail, dim3((unsigned)((C + 1 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     ys, R, C, mask, out, tail);
  return (int)hipGetLastError();
}

extern "C" int bsc_softmax_step_ones(const float* X, const int* y, const long long* off, const int* ntrain,
                                     const int* pid, const double* W, int D_IN, int D_OUT, int B, int P,
                                     unsigned long long seed, int iteration, float max_norm, double qscale, float* delta,
                                     long long* qdelta, float* loss, int lo, int* ones, int nones, void* stream) {
  if (D_IN <= 0 || D_OUT > 16 || B > 16) return -1;
  if (P <= 0) return 0;
  hipLaunchKernelGGL(k_softmax_step, dim3(P), dim3(SM_THREADS), 0, (hipStream_t)stream, X, y, off, ntrain, pid, W, D_IN,
                     D_OUT, B, P, seed, iteration, max_norm, qscale, delta, qdelta, loss, lo, ones, nones);
  return (int)hipGetLastError();
}

extern "C" int bsc_softmax_step(const float* X, const int* y, const long long* off, const int* ntrain,
                                const int* pid, const double* W, int D_IN, int D_OUT, int B, int P, unsigned long long seed,
                                int iteration, float max_norm, double qscale, float* delta, long long* qdelta,
                                float* loss, int lo, void* stream) {
  return bsc_softmax_step_ones(X, y, off, ntrain, pid, W, D_IN, D_OUT, B, P, seed, iteration, max_norm, qscale, delta,
                               qdelta, loss, lo, nullptr, 0, stream);
}

extern "C" int bsc_logreg_step(const double* X, const double* y, const long long* off, const int* nrows,
                               const int* pid, const double* W, int D, int B, int P, unsigned long long seed, const int* calls,
                               double alpha, double lammy, const double* sigma, double qscale, float* delta,
                               long long* qdelta, void* stream) {
  if (B > 64) return -1;
  if (P <= 0) return 0;
  hipLaunchKernelGGL(k_logreg_step, dim3(P), dim3(64), 0, (hipStream_t)stream, X, y, off, nrows, pid, W, D, B, P, seed,
                     calls, alpha, lammy, sigma, qscale, delta, qdelta);
  return (int)hipGetLastError();
}

extern "C" int bsc_dp_noise(const float* delta, int P, int D, const int* noisers, int nn, const float* scale,
                            unsigned long long seed, int iter_mod, float* noised, void* stream) {
  const long long n = (long long)P * D;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_dp_noise, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, delta, P, D, noisers, nn,
                     scale, seed, iter_mod, noised);
  return (int)hipGetLastError();
}

extern "C" int bsc_krum(const float* X, int n, int D, int ksplit, double* part, double* dist, double* scores,
                        int* accept, int groupsize, int n_accept, void* stream) {
  if (n <= 0) return 0;
  if (n > 128) return -1;
  const int tiles = (n + 15) / 16;
  const int nsplit = (D + ksplit - 1) / ksplit;
  hipLaunchKernelGGL(k_gram_f64, dim3(tiles, tiles, nsplit), dim3(64), 0, (hipStream_t)stream, X, n, D, ksplit,
                     part);
  hipLaunchKernelGGL(k_krum_scores, dim3(n), dim3(64), 0, (hipStream_t)stream, part, nsplit, n, tiles * 16,
                     groupsize, dist, scores);
  hipLaunchKernelGGL(k_krum_accept, dim3(1), dim3(128), 0, (hipStream_t)stream, scores, n, n_accept, accept);
  return (int)hipGetLastError();
}

// Committee Multi-Krum: X [U, D] fp32; inbox [V, n] rows of X; lead_rank [U] (-1: not submitted).
// part: [nsplit, npairs, 256] f64 scratch (npairs = T(T+1)/2, T = ceil(U/16), nsplit = ceil(D/kchunk));
// scores [V, n] f64; acc [V, n] int32; node [U] int32.
// Limits: U <= 8192 candidate rows, inbox n <= 4096, V <= 64 verifiers; ws: int32 [U] workspace
// (used when n > 256 or U > 1024).
extern "C" int bsc_krum_committee(const float* X, int U, int D, int kchunk, const int* inbox, int V, int n,
                                  int groupsize, int n_accept, int need, const int* lead_rank, int cap, double* part,
                                  double* gram, unsigned int* count, double* scores, int* acc, int* node, int* ws,
                                  void* stream) {
  if (U <= 0 || V <= 0 || n <= 0) return 0;
  if (U > 8192 || n > 4096 || V > 64 || n > U || kchunk <= 0) return -1;
  const int T = (U + 15) / 16;
  const int npairs = T * (T + 1) / 2;
  const int nsplit = (D + kchunk - 1) / kchunk;
  hipStream_t s = (hipStream_t)stream;
  // count: npairs zeroed counters (re-armed by the kernel itself)
  hipLaunchKernelGGL(k_gram_pairs, dim3(npairs, nsplit), dim3(256), 0, s, X, U, D, kchunk, T, part, gram, count,
                     (const float*)nullptr, U, 0ll, 0, (const double*)nullptr, 0);
  hipLaunchKernelGGL(k_gram_reduce, dim3(npairs), dim3(256), 0, s, part, gram, npairs, nsplit, 0, T, 0, 0);
  if (n <= 256) {
    hipLaunchKernelGGL(k_krum_rows, dim3(n, V), dim3(256), 0, s, gram, T, inbox, n, groupsize, scores);
  } else {
    const int np2 = pow2_at_least(n);
    hipLaunchKernelGGL(k_krum_rows_big<false>, dim3(n, V), dim3(1024), (size_t)np2 * sizeof(double), s, gram, T, U,
                       (const int*)nullptr, (const float*)nullptr, 0, inbox, n, np2, groupsize, scores);
  }
  if (krum_vote_any(s, scores, inbox, V, n, n_accept, U, need, lead_rank, cap, acc, node, ws) != 0) return -1;
  return (int)hipGetLastError();
}
// Tile pairs [p0, p1) of the stacked Gram only (p1 <= 0: all of them): several ranks split one Gram's tiles
// and exchange the reduced tiles (engine: the verification all_gather).  part: [nsplit, p1 - p0, 256].
// nn (nullable): this iteration's dense [U2, U2] Gram of the noise rows (setup, bsc_gram_noise_table); the tile
// pairs of noise rows only are copied from it instead of computed.
extern "C" int bsc_gram_stacked_range(const float* X, int U1, const float* X2, int U2, long long stride2, int D,
                                      int kchunk, int p0, int p1, double* part, double* gram, unsigned int* count,
                                      const double* nn, void* stream) {
  const int U = U1 + U2;
  if (U <= 0) return 0;
  if (U > 8192 || kchunk <= 0) return -1;
  const int T = (U + 15) / 16;
  const int npairs = T * (T + 1) / 2;
  if (p1 <= 0 || p1 > npairs) p1 = npairs;
  if (p0 < 0 || p0 > p1) return -1;
  if (p0 == p1) return 0;
  const int nsplit = (D + kchunk - 1) / kchunk;
  hipLaunchKernelGGL(k_gram_pairs, dim3(p1 - p0, nsplit), dim3(256), 0, (hipStream_t)stream, X, U, D, kchunk, T, part,
                     gram, count, X2, U1, stride2, p0, nn, (U1 + 15) / 16);
  hipLaunchKernelGGL(k_gram_reduce, dim3(p1 - p0), dim3(256), 0, (hipStream_t)stream, part, gram, p1 - p0, nsplit, p0,
                     T, (U1 + 15) / 16, nn != nullptr ? 1 : 0);
  return (int)hipGetLastError();
}
extern "C" int bsc_gram_stacked(const float* X, int U1, const float* X2, int U2, long long stride2, int D, int kchunk,
                                double* part, double* gram, unsigned int* count, const double* nn, void* stream) {
  return bsc_gram_stacked_range(X, U1, X2, U2, stride2, D, kchunk, 0, 0, part, gram, count, nn, stream);
}
// h_out (nullable): [V * n + U1] pinned host mirror of (acc, node), written by the vote itself (acc and node
// must be contiguous there too); amap / nspec / alive (nullable): the speculative MSM's row flags set in the
// same kernel
extern "C" int bsc_krum_committee_noise2(const double* gram, int U1, int U, const int* nz, const float* sc, int nn,
                                         const int* inbox, int V, int n, int groupsize, int n_accept, int need,
                                         const int* lead_rank, int cap, double* scores, int* acc, int* node, int* ws,
                                         int* h_out, const int* amap, int nspec, int* alive, void* stream) {
  if (U1 <= 0 || V <= 0 || n <= 0) return 0;
  if (U > 8192 || U1 > 8192 || n > 4096 || V > 64 || n > U1 || nn <= 0 || nn > 16) return -1;
  const int T = (U + 15) / 16;
  hipStream_t s = (hipStream_t)stream;
  if (n <= 256) {
    hipLaunchKernelGGL(k_krum_rows_noise, dim3(n, V), dim3(256), 0, s, gram, T, U1, nz, sc, nn, inbox, n, groupsize,
                       scores);
  } else {
    const int np2 = pow2_at_least(n);
    hipLaunchKernelGGL(k_krum_rows_big<true>, dim3(n, V), dim3(1024), (size_t)np2 * sizeof(double), s, gram, T, U1,
                       nz, sc, nn, inbox, n, np2, groupsize, scores);
  }
  if (krum_vote_any(s, scores, inbox, V, n, n_accept, U1, need, lead_rank, cap, acc, node, ws, h_out, amap, nspec,
                    alive) != 0)
    return -1;
  return (int)hipGetLastError();
}
// the same with the noisers' ids / weights read from HOST memory (nz_host / sc_host [U1][nn]) into the rows
// kernel's argument block (U1 * nn <= NOISE_ARG_MAX, n <= 256; else -2: the caller uploads and uses the above)
extern "C" int bsc_krum_committee_noise_ka(const double* gram, int U1, int U, const int* nz_host, const float* sc_host,
                                           int nn, const int* inbox, int V, int n, int groupsize, int n_accept,
                                           int need, const int* lead_rank, int cap, double* scores, int* acc, int* node,
                                           int* ws, int* h_out, const int* amap, int nspec, int* alive, void* stream) {
  if (U1 <= 0 || V <= 0 || n <= 0) return 0;
  if (U > 8192 || U1 > 8192 || n > 4096 || V > 64 || n > U1 || nn <= 0 || nn > 16) return -1;
  if ((long long)U1 * nn > NOISE_ARG_MAX || n > 256) return -2;
  NoiseArg q;
  for (int i = 0; i < U1 * nn; ++i) {
    q.nz[i] = nz_host[i];
    q.sc[i] = sc_host[i];
  }
  const int T = (U + 15) / 16;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_krum_rows_noise_ka, dim3(n, V), dim3(256), 0, s, gram, T, U1, q, nn, inbox, n, groupsize,
                     scores);
  if (krum_vote_any(s, scores, inbox, V, n, n_accept, U1, need, lead_rank, cap, acc, node, ws, h_out, amap, nspec,
                    alive) != 0)
    return -1;
  return (int)hipGetLastError();
}
extern "C" int bsc_krum_committee_noise(const double* gram, int U1, int U, const int* nz, const float* sc, int nn,
                                        const int* inbox, int V, int n, int groupsize, int n_accept, int need,
                                        const int* lead_rank, int cap, double* scores, int* acc, int* node, int* ws,
                                        void* stream) {
  if (U1 <= 0 || V <= 0 || n <= 0) return 0;
  if (U > 8192 || U1 > 8192 || n > 4096 || V > 64 || n > U1 || nn <= 0 || nn > 16) return -1;
  const int T = (U + 15) / 16;
  hipStream_t s = (hipStream_t)stream;
  if (n <= 256) {
    hipLaunchKernelGGL(k_krum_rows_noise, dim3(n, V), dim3(256), 0, s, gram, T, U1, nz, sc, nn, inbox, n, groupsize,
                       scores);
  } else {
    const int np2 = pow2_at_least(n);
    hipLaunchKernelGGL(k_krum_rows_big<true>, dim3(n, V), dim3(1024), (size_t)np2 * sizeof(double), s, gram, T, U1,
                       nz, sc, nn, inbox, n, np2, groupsize, scores);
  }
  if (krum_vote_any(s, scores, inbox, V, n, n_accept, U1, need, lead_rank, cap, acc, node, ws) != 0) return -1;
  return (int)hipGetLastError();
}
extern "C" int bsc_eval_error(const float* X, const int* y, int N, int D_IN, int D_OUT, const double* W,
                              int transform, int split, unsigned int* err, void* stream) {
  if (D_OUT > 16 || D_IN <= 0) return -1;
  if (N <= 0) return 0;
  const int tiles = (N + 15) / 16;
  hipLaunchKernelGGL(k_eval_error, dim3(tiles), dim3(256), 0, (hipStream_t)stream, X, y, N, D_IN, D_OUT, W,
                     transform, split, err);
  return (int)hipGetLastError();
}

// the evaluation with its accumulator reset and its read-back into pinned memory in one call (the engine
// queues it every round; three Python-level stream operations cost more host time than the kernel)
extern "C" int bsc_eval_error_rb(const float* X, const int* y, int N, int D_IN, int D_OUT, const double* W,
                                 int transform, int split, unsigned int* err, unsigned int* err_host, void* stream) {
  if (hipMemsetAsync(err, 0, 2 * sizeof(unsigned int), (hipStream_t)stream) != hipSuccess) return -1;
  const int rc = bsc_eval_error(X, y, N, D_IN, D_OUT, W, transform, split, err, stream);
  if (rc != 0) return rc;
  return (int)hipMemcpyAsync(err_host, err, 2 * sizeof(unsigned int), hipMemcpyDeviceToHost, (hipStream_t)stream);
}

extern "C" int bsc_eval_error_t_rb(const float* Xt, const int* y, int N, int KG, int D_IN, int D_OUT, const double* W,
                                   int split, unsigned int* err, unsigned int* err_host, void* stream) {
  if (D_OUT > 16 || D_IN <= 0 || KG * 4 < D_IN) return -1;
  if (N <= 0) {
    if (hipMemsetAsync(err, 0, 3 * sizeof(unsigned int), (hipStream_t)stream) != hipSuccess) return -1;
    return (int)hipMemcpyAsync(err_host, err, 2 * sizeof(unsigned int), hipMemcpyDeviceToHost, (hipStream_t)stream);
  }
  // err: 3 zeroed counters; k_eval_finish writes err_host and re-zeroes them
  hipLaunchKernelGGL(k_eval_error_t, dim3((N + 15) / 16), dim3(256), 0, (hipStream_t)stream, Xt, y, N, KG, D_IN, D_OUT,
                     W, split, err, err_host);
  hipLaunchKernelGGL(k_eval_finish, dim3(1), dim3(64), 0, (hipStream_t)stream, err, err_host);
  return (int)hipGetLastError();
}

extern "C" int bsc_noise_table(int nnoisers, int D, unsigned long long seed, float* tbl, void* stream) {
  const long long n = (long long)nnoisers * 100 * D;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_noise_table, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, nnoisers, D, seed, tbl);
  return (int)hipGetLastError();
}

extern "C" int bsc_dp_noise_tbl(const float* delta, int P, int D, const int* noisers, int nn, const float* scale,
                                const float* tbl, int iter_mod, const int* rows, float* noised, void* stream) {
  const long long n = (long long)P * D;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_dp_noise_tbl, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, delta, P, D, noisers,
                     nn, scale, tbl, iter_mod, rows, noised);
  return (int)hipGetLastError();
}

extern "C" int bsc_recover(const long long* ys, int nchunks, int npts, const int* xs, int poly, int d,
                           const double* W, double qscale, double* W_new, long long* coeffs, int* status,
                           void* stream) {
  if (nchunks <= 0) return 0;
  if (npts > 32 || poly > 16) return -1;
  hipLaunchKernelGGL(k_recover, dim3(nblk(nchunks, 64)), dim3(64), 0, (hipStream_t)stream, ys, nchunks, npts, xs,
                     poly, d, W, qscale, W_new, coeffs, status);
  return (int)hipGetLastError();
}

// rstride: int64 elements between consecutive rows of ys (nch * T for a dense [nrows][nch][T] tensor; the
// packed row length when ys are the ranks' partials inside an all_gather buffer, round.hip)
// h_W / h_status (nullable): pinned host mirrors of W_new / status written by the kernel (no read-back copies)
// h_clock (nullable, several ranks): every row's int64 right after its nch x T sums, mirrored to pinned memory
extern "C" int bsc_recover_w_clock(const long long* ys, int nrows, long long rstride, int nch, int T, const int* mask,
                                   const int* ycols, const int* xs, int npts, const long long* A, const int* basis,
                                   int poly, int shift, unsigned long long inv_lo, unsigned long long inv_hi, int d,
                                   const double* W, double qscale, double* W_new, long long* coeffs, int* status,
                                   long long* agg_out, double* h_W, int* h_status, long long* h_clock, void* stream) {
  if (nch <= 0) return 0;
  if (npts > RW_MAXP || poly > RW_MAXC || poly > npts || shift < 0 || shift > 100 || nrows <= 0) return -1;
  if (rstride < (long long)nch * T || (h_clock != nullptr && (nrows > 256 || rstride < (long long)nch * T + 1)))
    return -1;
  hipLaunchKernelGGL(k_recover_w, dim3(nblk(nch, RW_CPB)), dim3(256), 0, (hipStream_t)stream, ys, nrows, rstride, nch,
                     T, mask, ycols, xs, npts, A, basis, poly, shift, inv_lo, inv_hi, d, W, qscale, W_new, coeffs,
                     status, agg_out, h_W, h_status, h_clock);
  return (int)hipGetLastError();
}

extern "C" int bsc_recover_w_strided(const long long* ys, int nrows, long long rstride, int nch, int T, const int* mask,
                                     const int* ycols, const int* xs, int npts, const long long* A, const int* basis,
                                     int poly, int shift, unsigned long long inv_lo, unsigned long long inv_hi, int d,
                                     const double* W, double qscale, double* W_new, long long* coeffs, int* status,
                                     long long* agg_out, double* h_W, int* h_status, void* stream) {
  return bsc_recover_w_clock(ys, nrows, rstride, nch, T, mask, ycols, xs, npts, A, basis, poly, shift, inv_lo, inv_hi, d,
                             W, qscale, W_new, coeffs, status, agg_out, h_W, h_status, nullptr, stream);
}

extern "C" int bsc_recover_w(const long long* ys, int nrows, int nch, int T, const int* mask, const int* ycols,
                             const int* xs, int npts, const long long* A, const int* basis, int poly, int shift,
                             unsigned long long inv_lo, unsigned long long inv_hi, int d, const double* W, double qscale,
                             double* W_new, long long* coeffs, int* status, long long* agg_out, void* stream) {
  return bsc_recover_w_strided(ys, nrows, (long long)nch * T, nch, T, mask, ycols, xs, npts, A, basis, poly, shift,
                               inv_lo, inv_hi, d, W, qscale, W_new, coeffs, status, agg_out, nullptr, nullptr, stream);
}

extern "C" int bsc_add_rows(const float* delta, int D, const int* rows, int nrows, const double* W, double* W_new,
                            void* stream) {
  if (D <= 0) return 0;
  hipLaunchKernelGGL(k_add_rows, dim3(nblk(D, 256)), dim3(256), 0, (hipStream_t)stream, delta, D, rows, nrows, W,
                     W_new);
  return (int)hipGetLastError();
}
